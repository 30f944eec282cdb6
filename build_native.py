"""In-tree build of the native core `ollama_operator_amd/_C*.so` for gfx950.

hipcc compiles every `csrc/**/*.hip` (device code) and `csrc/**/*.cpp` (host code: loader,
executor, pybind11 bindings) in parallel, incrementally, then links one shared object against the
HIP runtime that torch ships (same SONAME, so one runtime instance per process). No torch headers
are used, which keeps a full rebuild to well under a minute on 8 cores.

    python build_native.py [--clean] [--jobs N]
"""
from __future__ import annotations

import argparse
import concurrent.futures as cf
import glob
import os
import subprocess
import sys
import sysconfig

ROOT = os.path.dirname(os.path.abspath(__file__))
CSRC = os.path.join(ROOT, "csrc")
CPU_SRC = os.path.join(CSRC, "cpu")
BUILD = os.path.join(ROOT, "build", "native")
ARCH = os.environ.get("OMX_ARCH", "gfx950")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")


def _ext_suffix() -> str:
    return sysconfig.get_config_var("EXT_SUFFIX") or ".so"


def target_path() -> str:
    return os.path.join(ROOT, "ollama_operator_amd", "_C" + _ext_suffix())


def _torch_lib() -> str | None:
    try:
        import importlib.util
        spec = importlib.util.find_spec("torch")
        if spec and spec.origin:
            d = os.path.join(os.path.dirname(spec.origin), "lib")
            if os.path.exists(os.path.join(d, "libamdhip64.so")):
                return d
    except Exception:
        pass
    return None


def _headers() -> list[str]:
    return glob.glob(os.path.join(CSRC, "**", "*.h"), recursive=True)


def _needs(obj: str, src: str, hdr_mtime: float) -> bool:
    if not os.path.exists(obj):
        return True
    m = os.path.getmtime(obj)
    return m < os.path.getmtime(src) or m < hdr_mtime


DEBUG_BUILD = os.path.join(ROOT, "build", "debug")
DEBUG_FLAGS = ["-O1", "-g", "-DOMX_DEBUG_KERNELS"]


def build(jobs: int | None = None, clean: bool = False, verbose: bool = False, debug: bool = False,
          sources: list[str] | None = None) -> str:
    """debug: the in-kernel bounds assertions (OMX_KASSERT) and -O1 -g, objects in build/debug and the
    module in build/debug/ollama_operator_amd (put that directory first on sys.path to load it).
    sources: compile only these csrc-relative translation units (no link), e.g. for a build check."""
    import pybind11
    build_dir = DEBUG_BUILD if debug else BUILD
    os.makedirs(build_dir, exist_ok=True)
    if clean:
        for f in glob.glob(os.path.join(build_dir, "*.o")):
            os.remove(f)
    srcs = sorted(s for s in glob.glob(os.path.join(CSRC, "**", "*.hip"), recursive=True) +
                  glob.glob(os.path.join(CSRC, "**", "*.cpp"), recursive=True)
                  if not s.startswith(CPU_SRC + os.sep))  # the CPU backend is its own module (build_cpu)
    hdr_mtime = max((os.path.getmtime(h) for h in _headers()), default=0.0)
    py_inc = sysconfig.get_paths()["include"]
    if sources is not None:
        srcs = [os.path.join(CSRC, x) for x in sources]
    opt = DEBUG_FLAGS if debug else ["-O3"]
    common = [*opt, "-std=c++17", "-fPIC", f"--offload-arch={ARCH}", "-I", CSRC,
              "-I", pybind11.get_include(), "-I", py_inc, "-Wno-unused-result"]
    jobs_list = []
    objs = []
    for s in srcs:
        rel = os.path.relpath(s, CSRC).replace(os.sep, "_")
        obj = os.path.join(build_dir, rel + ".o")
        objs.append(obj)
        if _needs(obj, s, hdr_mtime):
            if s.endswith(".hip"):
                cmd = [HIPCC, *common, "-c", s, "-o", obj]
            else:  # host-only translation unit
                cmd = [HIPCC, *common, "-x", "c++", "-D__HIP_PLATFORM_AMD__", "-I/opt/rocm/include", "-c", s, "-o", obj,
                       "-fvisibility=hidden"]
            jobs_list.append((s, cmd))
    jobs = jobs or min(8, os.cpu_count() or 4)

    def run(item):
        s, cmd = item
        r = subprocess.run(cmd, capture_output=True, text=True)
        return s, r.returncode, r.stdout + r.stderr, " ".join(cmd)

    failed = []
    if jobs_list:
        with cf.ThreadPoolExecutor(max_workers=jobs) as ex:
            for s, rc, out, cmd in ex.map(run, jobs_list):
                if rc != 0:
                    failed.append((s, out, cmd))
                elif verbose:
                    print("compiled", os.path.relpath(s, ROOT))
    if failed:
        for s, out, cmd in failed:
            sys.stderr.write(f"--- {s}\n{cmd}\n{out}\n")
        raise RuntimeError(f"native build failed ({len(failed)} translation units)")
    if sources is not None:
        return build_dir
    out = target_path()
    if debug:
        os.makedirs(os.path.join(build_dir, "ollama_operator_amd"), exist_ok=True)
        out = os.path.join(build_dir, "ollama_operator_amd", os.path.basename(out))
    if not os.path.exists(out) or jobs_list or any(os.path.getmtime(o) > os.path.getmtime(out) for o in objs):
        # linked beside the target, then renamed: a reader of the tree (a test, a tree snapshot) never
        # sees a half-written library
        tmp = out + ".tmp"
        link = [HIPCC, "-shared", f"--offload-arch={ARCH}", "-o", tmp, *objs, "-lpthread"]
        tl = _torch_lib()
        if tl:
            link += [f"-L{tl}", f"-Wl,-rpath,{tl}"]
        # hipBLASLt for the large-M prefill GEMM (csrc/runtime/blas.cpp): torch's copy when present
        # (one instance per process), else the ROCm one
        link += ["-lhipblaslt"] + ([] if tl and os.path.exists(os.path.join(tl, "libhipblaslt.so")) else ["-L/opt/rocm/lib"])
        r = subprocess.run(link, capture_output=True, text=True)
        if r.returncode != 0:
            raise RuntimeError("link failed:\n" + " ".join(link) + "\n" + r.stdout + r.stderr)
        os.replace(tmp, out)
    return out


def cpu_target_path() -> str:
    return os.path.join(ROOT, "ollama_operator_amd", "_cpu" + _ext_suffix())


def build_cpu(verbose: bool = False) -> str:
    """`ollama_operator_amd/_cpu*.so`: the CPU serving backend (csrc/cpu), host compiler only (no HIP
    runtime dependency, so it loads on a CPU-only node). AVX2 + FMA + F16C baseline, OpenMP threads."""
    import pybind11
    srcs = sorted(glob.glob(os.path.join(CPU_SRC, "*.cpp")))
    hdrs = glob.glob(os.path.join(CPU_SRC, "*.h"))
    out = cpu_target_path()
    newest = max(os.path.getmtime(f) for f in srcs + hdrs)
    if os.path.exists(out) and os.path.getmtime(out) >= newest:
        return out
    cxx = os.environ.get("CXX", "g++")
    cmd = [cxx, "-O3", "-std=c++17", "-fPIC", "-shared", "-fopenmp", "-mavx2", "-mfma", "-mf16c",
           "-fvisibility=hidden", "-I", CPU_SRC, "-I", pybind11.get_include(), "-I", sysconfig.get_paths()["include"],
           *srcs, "-o", out]
    r = subprocess.run(cmd, capture_output=True, text=True)
    if r.returncode != 0:
        raise RuntimeError("CPU backend build failed:\n" + " ".join(cmd) + "\n" + r.stdout + r.stderr)
    if verbose:
        print("built", os.path.relpath(out, ROOT))
    return out


if __name__ == "__main__":
    ap = argparse.ArgumentParser()
    ap.add_argument("--clean", action="store_true")
    ap.add_argument("--jobs", type=int, default=None)
    ap.add_argument("--cpu-only", action="store_true", help="build only the CPU backend module")
    ap.add_argument("--debug", action="store_true",
                    help="kernels with in-kernel bounds assertions (OMX_KASSERT), -O1 -g, into build/debug")
    a = ap.parse_args()
    if not a.debug:
        print(build_cpu(verbose=True))
    if not a.cpu_only:
        print(build(a.jobs, a.clean, verbose=True, debug=a.debug))
