"""One-shot all-reduce workspace of one tensor-parallel rank (csrc/kernels/allreduce.hip).

Each rank allocates its slab buffer (partial sums of the row-parallel projections, the LM-head vocab
shard) and its barrier flags in device memory, exports both as hipIpc handles, and opens every
peer's handles, so the decode step's collectives are plain kernels reading peers' HBM over xGMI:
no host round trip, no RCCL launch, and the whole TP decode step is capturable into one hipGraph.
Handles travel over the (gloo) control group once, at model load.

RCCL keeps the large messages (prefill chunks above `slab_rows` rows): one-shot reads
world x n bytes per rank, which only wins while latency dominates.
"""
from __future__ import annotations

import ctypes
import os

import numpy as np
import torch.distributed as dist

from ..ops import native

DEFAULT_TIMEOUT_S = float(os.environ.get("OMX_AR_TIMEOUT_S", "20"))


class TPCollectiveError(RuntimeError):
    """A peer missed a one-shot all-reduce barrier: the TP group is out of step and every later
    collective on this rank is skipped on device (allreduce.hip), so the process must end -- the
    server treats this like a HIP fault (server/app.py `is_device_fault`) and exits non-zero."""


class CustomAllReduce:
    def __init__(self, group, rank: int, world: int, slab_floats: int, timeout_s: float = DEFAULT_TIMEOUT_S):
        C = self.C = native()
        if world > C.AR_MAX_RANKS:
            raise ValueError(f"custom all-reduce supports up to {C.AR_MAX_RANKS} ranks, got {world}")
        slab_floats = (slab_floats + 3) // 4 * 4
        loc = self._local = C.ar_alloc(slab_floats)
        handles = [None] * world
        dist.all_gather_object(handles, (loc["data_handle"], loc["flags_handle"]), group=group)
        data, flags, self._opened = [], [], []
        for r, (hd, hf) in enumerate(handles):
            if r == rank:
                data.append(loc["data"])
                flags.append(loc["flags"])
                continue
            pd, pf = C.ar_open(hd), C.ar_open(hf)
            self._opened += [pd, pf]
            data.append(pd)
            flags.append(pf)
        self.group = group
        self.rank, self.world, self.slab_floats = rank, world, slab_floats
        # host-mapped mirror of the error word: the watchdog thread polls it with a plain memory read
        # (a hipMemcpy from another thread would queue behind -- or disturb the capture of -- the
        # decode graph)
        self._err_h, err_d = C.host_alloc_mapped(64)
        self._err_view = np.ctypeslib.as_array((ctypes.c_int32 * 1).from_address(self._err_h))
        self.params = dict(data=data, flags=flags, epoch=loc["epoch"], err=loc["err"], err_host=err_d, rank=rank,
                           world=world, slab_floats=slab_floats,
                           timeout_ticks=int(timeout_s * C.wall_clock_khz() * 1000))
        dist.barrier(group=group)  # every rank mapped every peer before any kernel signals

    def slab_ptr(self, slab: int) -> int:
        return self._local["data"] + 4 * slab * self.slab_floats

    def error(self) -> int:
        """0, or 1 + the peer whose barrier flag never arrived (a dead / wedged rank). A plain read of
        the host-mapped mirror: safe from any thread, never waits on the GPU."""
        if self._local is None:
            return 0
        return int(self._err_view[0])

    def check(self) -> None:
        e = self.error()
        if e:
            raise TPCollectiveError(f"tensor-parallel rank {self.rank}: peer {e - 1} missed an all-reduce barrier")

    def all_reduce_add(self, slab: int, y_ptr: int, n: int, stream: int) -> None:
        self.C.ar_allreduce_add(self.params, slab, y_ptr, n, stream)

    def all_reduce_add_emit(self, slab: int, y_ptr: int, E: int, B: int, img_ptr: int, nw_ptr: int, stat_ptr: int,
                            stream: int) -> None:
        """y[:B*E] += sum of the ranks' slabs, then each new row is written as the int8 activation image
        of y * nw (+ per-16 sums of squares) for the next GEMV (executor forward_tp, int8 chain)."""
        self.C.ar_allreduce_add_emit(self.params, slab, y_ptr, E, B, img_ptr, nw_ptr, stat_ptr, stream)

    def all_gather(self, slab: int, out_ptr: int, rows: int, n_local: int, ld_out: int, stream: int) -> None:
        self.C.ar_allgather(self.params, slab, out_ptr, rows, n_local, ld_out, stream)

    def close(self) -> None:
        if self._local is None:
            return
        try:
            dist.barrier(group=self.group)  # no peer still reads our slabs
        except Exception:  # noqa: BLE001 - peers may be gone at teardown
            pass
        for p in self._opened:
            self.C.ar_close(p)
        for k in ("data", "flags", "epoch"):
            self.C.ar_free(self._local[k])
        self._opened, self._local = [], None
        self._err_view = None
        self.C.host_free_mapped(self._err_h)
        self._err_h = 0
