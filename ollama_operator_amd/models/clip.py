"""LLaVA vision side: the CLIP ViT image encoder + multimodal projector of an Ollama `projector` layer
(a GGUF with general.architecture = "clip", llama.cpp's mmproj layout), producing one LLM-width
embedding row per image patch. The rows enter the language model's sequence as external embedding
rows (negative token ids, engine/runner.py `set_ext`), so prefill, KV prefix reuse, continuous
batching and tensor parallelism work for image prompts unchanged.

The reference lists LLaVA among the models its images serve (/root/reference/README.md:57, via
ollama/ollama); the projector media type is `application/vnd.ollama.image.projector`
(server/store.py MT_PROJECTOR).

Design: the encoder runs once per image (576 patches for LLaVA-1.5 at 336 px), so it is a plain
PyTorch module on the runner's device -- fp16 GEMMs on hipBLASLt and fused SDPA attention on the
GPU -- not a hand-written kernel path; the language model's prefill/decode loop is where the time
goes. Image preprocessing follows LLaVA-1.5 ("pad" aspect): pad to a square with the mean colour,
resize to image_size, normalise by image_mean / image_std. A LLaVA-1.6 projector (metadata
clip.vision.image_grid_pinpoints + mm_patch_merge_type, tensor model.image_newline) takes the
any-resolution path instead (`preprocess_anyres` / `ClipEncoder.encode`): the grid resolution that
keeps the most image detail is picked from the pinpoints, the image is fitted into it and cut into
image_size tiles, every tile and a downsized whole-image view go through the tower, and the tile
features are stitched back into one patch grid, unpadded to the image's aspect and closed per row
with the image_newline embedding ("spatial_unpad"; "flat" concatenates the views).

Tensor names / metadata (llama.cpp clip GGUF): v.patch_embd.weight [E,3,p,p], v.class_embd [E],
v.position_embd.weight [n_pos,E], v.pre_ln.{weight,bias}, v.blk.{i}.{attn_q,attn_k,attn_v,attn_out,
ffn_up,ffn_down}.{weight,bias}, v.blk.{i}.{ln1,ln2}.{weight,bias}, optional v.post_ln, projector
mm.0 / mm.2 (Linear-GELU-Linear, projector_type "mlp"); clip.vision.{image_size, patch_size,
embedding_length, feature_length, block_count, attention.head_count, attention.layer_norm_epsilon,
image_mean, image_std}, clip.use_gelu (false: quick-GELU as OpenAI CLIP). Parity unpinned: no real
mmproj file exists in this environment; tests pin the module to an independent fp32 numpy oracle.
"""
from __future__ import annotations

import hashlib
import io
import math
import os
from dataclasses import dataclass

import numpy as np
import torch
import torch.nn.functional as F

from ..gguf import read_gguf

MAX_PATCHES_PER_IMAGE = 4096


class VisionError(ValueError):
    pass


@dataclass
class ClipConfig:
    image_size: int
    patch_size: int
    E: int
    F: int
    n_layer: int
    n_head: int
    eps: float
    mean: tuple[float, float, float]
    std: tuple[float, float, float]
    use_gelu: bool
    projector: str
    out_dim: int
    grid_pinpoints: tuple[tuple[int, int], ...] = ()  # LLaVA-1.6 any-resolution grids (w, h); () = 1.5
    merge: str = "flat"

    @property
    def n_patches(self) -> int:
        return (self.image_size // self.patch_size) ** 2

    @property
    def max_rows(self) -> int:
        """Most embedding rows one image can produce (ids / external-row capacity)."""
        if not self.grid_pinpoints:
            return self.n_patches
        g, S = self.image_size // self.patch_size, self.image_size
        nl = 1 if self.merge == "spatial_unpad" else 0
        return self.n_patches + max((H // S) * g * ((W // S) * g + nl) for W, H in self.grid_pinpoints)


def clip_config(md: dict, tensors: dict) -> ClipConfig:
    if str(md.get("general.architecture", "")) != "clip":
        raise VisionError("projector is not a CLIP GGUF (general.architecture != clip)")
    g = lambda k, d=None: md.get("clip.vision." + k, d)  # noqa: E731
    proj = str(md.get("clip.projector_type", "mlp"))
    if proj != "mlp":
        raise VisionError(f"unsupported projector type {proj!r} (supported: mlp)")
    out_dim = tensors["mm.2.weight"].torch_shape[0]
    S = int(g("image_size", 336))
    pins = [int(v) for v in g("image_grid_pinpoints", ())]
    if len(pins) % 2:
        raise VisionError("clip.vision.image_grid_pinpoints must hold (width, height) pairs")
    grid = tuple((pins[i], pins[i + 1]) for i in range(0, len(pins), 2))
    if any(W <= 0 or H <= 0 or W % S or H % S for W, H in grid):
        raise VisionError(f"grid pinpoints {grid} are not positive multiples of image_size {S}")
    merge = str(g("mm_patch_merge_type", "flat"))
    if merge not in ("flat", "spatial_unpad"):
        raise VisionError(f"unsupported mm_patch_merge_type {merge!r} (supported: flat, spatial_unpad)")
    if grid and merge == "spatial_unpad" and "model.image_newline" not in tensors:
        raise VisionError("spatial_unpad merge needs the model.image_newline tensor")
    c = ClipConfig(image_size=int(g("image_size", 336)), patch_size=int(g("patch_size", 14)),
                      E=int(g("embedding_length")), F=int(g("feature_length")), n_layer=int(g("block_count")),
                      n_head=int(g("attention.head_count")), eps=float(g("attention.layer_norm_epsilon", 1e-5)),
                      mean=tuple(float(v) for v in g("image_mean", (0.48145466, 0.4578275, 0.40821073))),
                      std=tuple(float(v) for v in g("image_std", (0.26862954, 0.26130258, 0.27577711))),
                      use_gelu=bool(md.get("clip.use_gelu", False)), projector=proj, out_dim=int(out_dim),
                      grid_pinpoints=grid, merge=merge)
    if c.max_rows > MAX_PATCHES_PER_IMAGE:
        raise VisionError(f"grid pinpoints give up to {c.max_rows} rows per image (> {MAX_PATCHES_PER_IMAGE})")
    return c


# decoded-size limits: a tiny file can declare a huge (or extremely thin) canvas; nothing larger than
# this is ever decoded or padded (PIL's decompression-bomb check counts pixels only, so a 1 x 200000
# image passes it and its square padding would be a 200000 x 200000 canvas)
MAX_IMAGE_SIDE = 16384
MAX_IMAGE_PIXELS = 1 << 26


def _decode(image: bytes | np.ndarray):
    """Encoded image bytes (PNG/JPEG/...) or an HxWx3 uint8 array -> RGB PIL image, size-checked
    from the header before any pixel is decoded."""
    from PIL import Image
    if isinstance(image, (bytes, bytearray)):
        try:
            im = Image.open(io.BytesIO(image))
        except Exception as e:  # noqa: BLE001 -- any decoder error is a bad request
            raise VisionError(f"cannot decode image: {e}") from None
        w, h = im.size  # from the header: checked before any pixel is decoded
        if w <= 0 or h <= 0 or max(w, h) > MAX_IMAGE_SIDE or w * h > MAX_IMAGE_PIXELS:
            raise VisionError(f"image {w}x{h} exceeds the limits ({MAX_IMAGE_SIDE} px a side, "
                              f"{MAX_IMAGE_PIXELS} pixels)")
        try:
            im.load()
        except Exception as e:  # noqa: BLE001
            raise VisionError(f"cannot decode image: {e}") from None
    else:
        a = np.asarray(image, dtype=np.uint8)
        if a.ndim != 3 or max(a.shape[:2]) > MAX_IMAGE_SIDE or a.shape[0] * a.shape[1] > MAX_IMAGE_PIXELS:
            raise VisionError(f"image array of shape {a.shape} exceeds the limits")
        im = Image.fromarray(a)
    return im.convert("RGB")


def _cap(im, cap: int):
    """Downscale (aspect kept) so the longer side is at most `cap`: later resizes go below it anyway."""
    from PIL import Image
    w, h = im.size
    if max(w, h) > cap:
        f = cap / max(w, h)
        im = im.resize((max(1, round(w * f)), max(1, round(h * f))), Image.BICUBIC)
    return im


def _normalise(im, cfg: ClipConfig) -> np.ndarray:
    a = np.asarray(im, dtype=np.float32) / 255.0
    a = (a - np.asarray(cfg.mean, np.float32)) / np.asarray(cfg.std, np.float32)
    return np.ascontiguousarray(a.transpose(2, 0, 1))


def preprocess(image: bytes | np.ndarray, cfg: ClipConfig) -> np.ndarray:
    """Encoded image bytes (PNG/JPEG/...) or an HxWx3 uint8 array -> float32 [3, S, S] normalised.
    LLaVA-1.5 "pad" aspect: pad to a square with the mean colour, resize to image_size. Images larger
    than a few times image_size are first downscaled (aspect kept), so the padded canvas stays small."""
    from PIL import Image
    im = _cap(_decode(image), 4 * cfg.image_size)
    w, h = im.size
    side = max(w, h)
    bg = tuple(int(round(255 * m)) for m in cfg.mean)
    sq = Image.new("RGB", (side, side), bg)
    sq.paste(im, ((side - w) // 2, (side - h) // 2))
    return _normalise(sq.resize((cfg.image_size, cfg.image_size), Image.BICUBIC), cfg)


def select_best_resolution(size: tuple[int, int], grid: tuple[tuple[int, int], ...]) -> tuple[int, int]:
    """The grid (w, h) that keeps the most of the image's pixels when it is fitted in (aspect kept),
    ties broken by the least canvas left empty (LLaVA-NeXT any-resolution selection)."""
    w, h = size
    best, key = grid[0], None
    for W, H in grid:
        f = min(W / w, H / h)
        kept = min(int(w * f) * int(h * f), w * h)
        k = (kept, -(W * H - kept))
        if key is None or k > key:
            best, key = (W, H), k
    return best


def preprocess_anyres(image: bytes | np.ndarray, cfg: ClipConfig):
    """LLaVA-1.6 views of one image -> (float32 [1 + tiles, 3, S, S], original (w, h), grid (W, H)).
    View 0 is the whole image resized to S x S; then the image fitted (aspect kept, centred on black)
    into the best grid resolution and cut into S x S tiles, row-major."""
    from PIL import Image
    S = cfg.image_size
    im = _decode(image)
    w, h = im.size
    W, H = select_best_resolution((w, h), cfg.grid_pinpoints)
    im = _cap(im, 2 * max(W, H))
    fw, fh = W / w, H / h
    nw, nh = (W, min(math.ceil(h * fw), H)) if fw < fh else (min(math.ceil(w * fh), W), H)
    canvas = Image.new("RGB", (W, H), (0, 0, 0))
    canvas.paste(im.resize((nw, nh), Image.BICUBIC), ((W - nw) // 2, (H - nh) // 2))
    views = [_normalise(im.resize((S, S), Image.BICUBIC), cfg)]
    for r in range(H // S):
        for c in range(W // S):
            views.append(_normalise(canvas.crop((c * S, r * S, (c + 1) * S, (r + 1) * S)), cfg))
    return np.stack(views), (w, h), (W, H)


def unpad_grid(t: torch.Tensor, size: tuple[int, int]) -> torch.Tensor:
    """[rows, cols, D] patch grid of the fitted canvas -> the rows / columns that cover the image
    (the black bands added to reach the grid's aspect are dropped)."""
    w, h = size
    rows, cols = t.shape[:2]
    if w / h > cols / rows:  # image wider than the grid: bands above and below
        pad = (rows - int(round(h * (cols / w), 7))) // 2
        return t[pad:rows - pad]
    pad = (cols - int(round(w * (rows / h), 7))) // 2
    return t[:, pad:cols - pad]


class _NativeTower:
    """The CLIP tower on the engine's own kernels (GPU): every projection is the stream-order MFMA GEMM
    (csrc/kernels/gemm_dq.hip) on fp16 weight rows (QT_F16, K zero-padded to 256) with the LayerNorm
    fused into its activation prologue and bias / quick-GELU / erf-GELU / residual add in its epilogue;
    QKV goes through the same RoPE-less QKV epilogue as the LLM and scatters K/V into a private paged
    cache that the MFMA flash-attention kernel (attention.hip) reads with every key visible to every
    query (q_len = n: bidirectional). Only the patch im2col, the class/position add and the stand-alone
    pre/post LayerNorms stay torch element-wise ops."""

    QT_F16 = 1
    EPI_STORE, EPI_ADD, EPI_QKV, EPI_GELU_ERF, EPI_QGELU = 0, 1, 4, 6, 7
    NORM_LAYER = 2

    def __init__(self, enc: "ClipEncoder"):
        from ..ops import native
        self.C = native()
        self.enc = enc
        c = enc.cfg
        dev = enc.device
        h16 = dict(device=dev, dtype=torch.float16)
        f32 = dict(device=dev, dtype=torch.float32)

        def mat(w: torch.Tensor):  # [N][K] -> fp16 rows padded to whole 256-blocks (QMat tuple, tensor)
            N, K = w.shape
            Kp = (K + 255) // 256 * 256
            t = torch.zeros(N, Kp, **h16)
            t[:, :K] = w.to(torch.float16)
            return (t.data_ptr(), 0, 0, 0, N, K, self.QT_F16), t

        self.keep = []

        def M(w):
            tup, t = mat(w)
            self.keep.append(t)
            return tup

        f = lambda v: v.to(**f32).contiguous()  # noqa: E731
        E, n = c.E, c.n_patches + 1
        self.patch = M(enc.patch_w.reshape(E, -1))
        self.patch_b = f(enc.patch_b) if enc.patch_b is not None else None
        self.layers = []
        for b in enc.blocks:
            self.layers.append(dict(
                qkv=M(torch.cat([b["attn_q.weight"], b["attn_k.weight"], b["attn_v.weight"]], 0)),
                bqkv=f(torch.cat([b["attn_q.bias"], b["attn_k.bias"], b["attn_v.bias"]], 0)),
                o=M(b["attn_out.weight"]), bo=f(b["attn_out.bias"]),
                up=M(b["ffn_up.weight"]), bup=f(b["ffn_up.bias"]),
                down=M(b["ffn_down.weight"]), bdown=f(b["ffn_down.bias"]),
                ln1=(f(b["ln1.weight"]), f(b["ln1.bias"])), ln2=(f(b["ln2.weight"]), f(b["ln2.bias"]))))
        (w0, b0), (w2, b2) = enc.mm
        self.mm0, self.mb0 = M(w0), f(b0)
        self.mm2, self.mb2 = M(w2), f(b2)
        self.F = enc.blocks[0]["ffn_up.weight"].shape[0] if enc.blocks else E
        self.P = w0.shape[0]
        # workspaces: fp16 activations (largest K), split-K slabs, the attention cache and step inputs
        kmax = max((w.shape[1] + 255) // 256 * 256 for w in [enc.patch_w.reshape(E, -1), w0, w2] +
                   [b["ffn_down.weight"] for b in enc.blocks] + [b["attn_q.weight"] for b in enc.blocks])
        self.xws = torch.empty(n * kmax, **h16)
        self.gws = torch.empty(8 << 20, **f32)
        self.H, self.D = c.n_head, E // c.n_head
        self.bs = 16
        nblk = (n + self.bs - 1) // self.bs
        self.kc = torch.zeros(nblk, self.H, self.bs, self.D, **h16)
        self.vc = torch.zeros_like(self.kc)
        i32 = dict(device=dev, dtype=torch.int32)
        self.pos = torch.arange(n, **i32)
        self.qlen = torch.full((n,), n, **i32)  # every key visible to every query: bidirectional
        self.bt = torch.arange(nblk, **i32)[None].contiguous()
        self.nblk = nblk
        self.q = torch.empty(n, E, **f32)
        self.a = torch.empty(n, E, **f32)
        self.h = torch.empty(n, max(self.F, self.P), **f32)
        self.dummy = torch.zeros(max(1, self.D), **f32)

    def _gemm(self, w, B, x, ldx, y, ldy, epi, bias=None, norm=None, extra=None):
        d = dict(extra or {})
        d.update(xws=self.xws.data_ptr(), xws_elems=self.xws.numel(), gws=self.gws.data_ptr(),
                 gws_elems=self.gws.numel())
        nw, nb = norm if norm is not None else (None, None)
        p = lambda t: t.data_ptr() if t is not None else 0  # noqa: E731
        self.C.gemv(w, B, x.data_ptr(), ldx, self.NORM_LAYER if norm is not None else 0, p(nw), p(nb),
                    self.enc.cfg.eps, epi, y.data_ptr(), ldy, p(bias), 0, d, torch.cuda.current_stream().cuda_stream)

    @torch.no_grad()
    def encode(self, px: torch.Tensor) -> torch.Tensor:
        enc, c = self.enc, self.enc.cfg
        E, ps, n, H, D = c.E, c.patch_size, c.n_patches + 1, self.H, self.D
        # patch embedding as a GEMM: im2col rows in the conv weight's (channel, y, x) order
        x = torch.as_tensor(px).to(enc.device, torch.float32)
        cols = x.unfold(1, ps, ps).unfold(2, ps, ps)  # [3, g, g, ps, ps]
        cols = cols.permute(1, 2, 0, 3, 4).reshape(c.n_patches, -1).contiguous()
        emb = torch.empty(c.n_patches, E, device=enc.device)
        self._gemm(self.patch, c.n_patches, cols, cols.shape[1], emb, E, self.EPI_STORE, self.patch_b)
        xs = torch.cat([enc.cls.float()[None], emb], 0) + enc.pos.float()
        if enc.pre_ln[0] is not None:
            xs = F.layer_norm(xs, (E,), enc.pre_ln[0].float(), enc.pre_ln[1].float(), c.eps)
        xs = xs.contiguous()
        qkv = dict(pos=self.pos.data_ptr(), slot=self.pos.data_ptr(), kc=self.kc.data_ptr(), vc=self.vc.data_ptr(),
                   inv_freq=self.dummy.data_ptr(), Eq=E, Ekv=E, D=D, n_rot=0, n_kv=H, bs=self.bs)
        st = torch.cuda.current_stream().cuda_stream
        for L in self.layers:
            self._gemm(L["qkv"], n, xs, E, self.q, E, self.EPI_QKV, L["bqkv"], L["ln1"], qkv)
            self.C.attention(self.q.data_ptr(), E, self.kc.data_ptr(), self.vc.data_ptr(), self.bt.data_ptr(),
                             self.nblk, 0, self.qlen.data_ptr(), n, H, H, D, self.bs, 1.0 / math.sqrt(D), 0,
                             self.a.data_ptr(), E, 0, 1, 0, st, 1, D)
            self._gemm(L["o"], n, self.a, E, xs, E, self.EPI_ADD, L["bo"])
            act = self.EPI_GELU_ERF if c.use_gelu else self.EPI_QGELU
            self._gemm(L["up"], n, xs, E, self.h, self.h.shape[1], act, L["bup"], L["ln2"])
            self._gemm(L["down"], n, self.h, self.h.shape[1], xs, E, self.EPI_ADD, L["bdown"])
        if enc.post_ln[0] is not None:
            xs = F.layer_norm(xs, (E,), enc.post_ln[0].float(), enc.post_ln[1].float(), c.eps)
        xs = xs[1:].contiguous()  # LLaVA drops the class token
        m = n - 1
        self._gemm(self.mm0, m, xs, E, self.h, self.h.shape[1], self.EPI_GELU_ERF, self.mb0)
        out = torch.empty(m, self.mm2[4], device=enc.device)
        self._gemm(self.mm2, m, self.h, self.h.shape[1], out, out.shape[1], self.EPI_STORE, self.mb2)
        return out


class ClipEncoder:
    """CLIP ViT + LLaVA MLP projector on `device`: on a GPU the engine's own kernels (`_NativeTower`:
    MFMA GEMMs + flash attention; OMX_CLIP_NATIVE=0 keeps the fp16 torch path), on a CPU fp32 torch."""

    def __init__(self, path: str, device: str | torch.device = "cpu"):
        self.device = torch.device(device)
        self.dtype = torch.float16 if self.device.type == "cuda" else torch.float32
        g = read_gguf(path)
        try:
            self.cfg = clip_config(g.metadata, g.tensors)
            t = lambda n: torch.from_numpy(np.array(g.array(n), np.float32)).to(self.device, self.dtype)  # noqa: E731
            opt = lambda n: t(n) if n in g.tensors else None  # noqa: E731
            self.patch_w = t("v.patch_embd.weight")
            self.patch_b = opt("v.patch_embd.bias")
            self.cls = t("v.class_embd").reshape(-1)
            self.pos = t("v.position_embd.weight")
            self.pre_ln = (opt("v.pre_ln.weight"), opt("v.pre_ln.bias"))
            self.post_ln = (opt("v.post_ln.weight"), opt("v.post_ln.bias"))
            self.blocks = []
            for i in range(self.cfg.n_layer):
                b = f"v.blk.{i}."
                self.blocks.append({k: t(b + k) for k in (
                    "attn_q.weight", "attn_q.bias", "attn_k.weight", "attn_k.bias", "attn_v.weight", "attn_v.bias",
                    "attn_out.weight", "attn_out.bias", "ln1.weight", "ln1.bias", "ln2.weight", "ln2.bias",
                    "ffn_up.weight", "ffn_up.bias", "ffn_down.weight", "ffn_down.bias")})
            self.mm = [(t("mm.0.weight"), t("mm.0.bias")), (t("mm.2.weight"), t("mm.2.bias"))]
            nl = opt("model.image_newline")
            self.newline = nl.float().reshape(-1) if nl is not None else None
        finally:
            g.close()
        if self.pos.shape[0] != self.cfg.n_patches + 1:
            raise VisionError(f"position table has {self.pos.shape[0]} rows, expected {self.cfg.n_patches + 1}")
        # the native tower needs >= 128 patch rows (the MFMA GEMM's row minimum) and a flash-attention
        # head dim; smaller / odd towers (test fixtures) keep the fp16 torch path
        self.native = None
        c = self.cfg
        if (self.device.type == "cuda" and os.environ.get("OMX_CLIP_NATIVE", "1") != "0" and c.n_patches >= 128
                and c.E % c.n_head == 0 and c.E // c.n_head in (64, 80, 96, 128)):
            self.native = _NativeTower(self)

    @property
    def out_dim(self) -> int:
        return self.cfg.out_dim

    def _act(self, x: torch.Tensor) -> torch.Tensor:
        if self.cfg.use_gelu:
            return F.gelu(x)
        return x * torch.sigmoid(1.702 * x)  # quick-GELU (OpenAI CLIP)

    @torch.no_grad()
    def encode_pixels(self, px: np.ndarray | torch.Tensor) -> torch.Tensor:
        """[3, S, S] normalised pixels -> [n_patches, out_dim] fp32 LLM embedding rows."""
        if self.native is not None:
            return self.native.encode(px)
        return self.encode_pixels_torch(px)

    @torch.no_grad()
    def encode_pixels_torch(self, px: np.ndarray | torch.Tensor) -> torch.Tensor:
        c = self.cfg
        x = torch.as_tensor(px).to(self.device, self.dtype)[None]
        x = F.conv2d(x, self.patch_w, self.patch_b, stride=c.patch_size)  # [1, E, g, g]
        x = x.flatten(2).transpose(1, 2)[0]  # [n_patches, E], row-major patch order
        x = torch.cat([self.cls[None], x], 0) + self.pos
        if self.pre_ln[0] is not None:
            x = F.layer_norm(x, (c.E,), self.pre_ln[0], self.pre_ln[1], c.eps)
        H, D = c.n_head, c.E // c.n_head
        n = x.shape[0]
        for b in self.blocks:
            h = F.layer_norm(x, (c.E,), b["ln1.weight"], b["ln1.bias"], c.eps)
            q = F.linear(h, b["attn_q.weight"], b["attn_q.bias"]).view(n, H, D).transpose(0, 1)
            k = F.linear(h, b["attn_k.weight"], b["attn_k.bias"]).view(n, H, D).transpose(0, 1)
            v = F.linear(h, b["attn_v.weight"], b["attn_v.bias"]).view(n, H, D).transpose(0, 1)
            a = F.scaled_dot_product_attention(q[None], k[None], v[None])[0]  # bidirectional
            x = x + F.linear(a.transpose(0, 1).reshape(n, c.E), b["attn_out.weight"], b["attn_out.bias"])
            h = F.layer_norm(x, (c.E,), b["ln2.weight"], b["ln2.bias"], c.eps)
            h = self._act(F.linear(h, b["ffn_up.weight"], b["ffn_up.bias"]))
            x = x + F.linear(h, b["ffn_down.weight"], b["ffn_down.bias"])
        if self.post_ln[0] is not None:
            x = F.layer_norm(x, (c.E,), self.post_ln[0], self.post_ln[1], c.eps)
        x = x[1:]  # LLaVA drops the class token
        (w0, b0), (w2, b2) = self.mm
        x = F.linear(F.gelu(F.linear(x, w0, b0)), w2, b2)
        return x.float()

    def encode(self, image: bytes | np.ndarray) -> torch.Tensor:
        """One image -> [rows, out_dim] fp32 embedding rows (n_patches for LLaVA-1.5; base view + the
        stitched tile grid for a LLaVA-1.6 any-resolution projector)."""
        if not self.cfg.grid_pinpoints:
            return self.encode_pixels(preprocess(image, self.cfg))
        views, size, (W, H) = preprocess_anyres(image, self.cfg)
        feats = [self.encode_pixels(v) for v in views]
        if self.cfg.merge == "flat":
            return torch.cat(feats)
        S, g = self.cfg.image_size, self.cfg.image_size // self.cfg.patch_size
        gh, gw, D = H // S, W // S, feats[0].shape[1]
        grid = torch.stack(feats[1:]).view(gh, gw, g, g, D).permute(0, 2, 1, 3, 4).reshape(gh * g, gw * g, D)
        grid = unpad_grid(grid, size)
        nl = self.newline.to(grid.device).view(1, 1, D).expand(grid.shape[0], 1, D)
        return torch.cat([feats[0], torch.cat([grid, nl], 1).reshape(-1, D)])


ID_BUCKETS = 500_000  # id ranges of MAX_PATCHES_PER_IMAGE: |id| < 2^31


class ImageIds:
    """Negative token ids for images' patch rows, keyed by the FULL content digest.

    The same image gets the same ids (a KV prefix holding it is reused across requests); two different
    images never share ids: the digest picks a starting bucket and a bucket owned by another digest is
    probed past (linear probing), so a collision of the truncated hash can never make one image's
    prompt reuse another image's embedding rows or KV. A bucket is never handed to a second digest
    during the registry's lifetime (one loaded model), because idle sequences may still hold KV under
    its ids. Only ids issued here are valid in client-supplied `context` (`issued`)."""

    def __init__(self, n_buckets: int = ID_BUCKETS):
        self.n_buckets = n_buckets
        self._bucket: dict[bytes, tuple[int, int]] = {}  # digest -> (bucket, rows)
        self._owner: dict[int, bytes] = {}                # bucket -> digest
        self._mu = __import__("threading").Lock()

    def ids_for(self, image: bytes, n: int) -> list[int]:
        if n > MAX_PATCHES_PER_IMAGE:
            raise VisionError(f"{n} patches per image exceeds {MAX_PATCHES_PER_IMAGE}")
        dg = hashlib.sha256(bytes(image)).digest()
        with self._mu:
            hit = self._bucket.get(dg)
            if hit is None:
                if len(self._owner) >= self.n_buckets:
                    raise VisionError("image id space of this model load is exhausted; reload the model")
                b = int.from_bytes(dg[:8], "little") % self.n_buckets
                while b in self._owner:
                    b = (b + 1) % self.n_buckets
                self._owner[b] = dg
                hit = self._bucket[dg] = (b, n)
        b, n0 = hit
        if n0 != n:
            raise VisionError(f"image encoded to {n} rows, registered with {n0}")
        base = 1 + b * MAX_PATCHES_PER_IMAGE
        return [-(base + j) for j in range(n)]

    def issued(self, tok: int) -> bool:
        """True for a negative id this registry handed out (a patch row of a registered image)."""
        if tok >= 0:
            return False
        b, j = divmod(-tok - 1, MAX_PATCHES_PER_IMAGE)
        with self._mu:
            dg = self._owner.get(b)
            return dg is not None and j < self._bucket[dg][1]


# ---------------------------------------------------------------------------------------------------
# fp32 numpy oracle (tests) and random-init projector files
def reference_encode(path: str, px: np.ndarray) -> np.ndarray:
    """Independent float64 numpy forward of the same GGUF (test oracle for ClipEncoder)."""
    g = read_gguf(path)
    try:
        c = clip_config(g.metadata, g.tensors)
        a = lambda n: np.asarray(g.array(n), np.float64)  # noqa: E731
        p = c.patch_size
        gsz = c.image_size // p
        w = a("v.patch_embd.weight").reshape(c.E, -1)  # [E, 3*p*p]
        patches = px.astype(np.float64).reshape(3, gsz, p, gsz, p).transpose(1, 3, 0, 2, 4).reshape(gsz * gsz, -1)
        x = patches @ w.T
        if "v.patch_embd.bias" in g.tensors:
            x = x + a("v.patch_embd.bias")
        x = np.concatenate([a("v.class_embd").reshape(1, -1), x], 0) + a("v.position_embd.weight")

        def ln(x, wn, bn):
            mu = x.mean(-1, keepdims=True)
            var = ((x - mu) ** 2).mean(-1, keepdims=True)
            return (x - mu) / np.sqrt(var + c.eps) * a(wn) + a(bn)

        if "v.pre_ln.weight" in g.tensors:
            x = ln(x, "v.pre_ln.weight", "v.pre_ln.bias")
        H, D = c.n_head, c.E // c.n_head
        n = x.shape[0]
        lin = lambda h, name: h @ a(name + ".weight").T + a(name + ".bias")  # noqa: E731
        for i in range(c.n_layer):
            b = f"v.blk.{i}."
            h = ln(x, b + "ln1.weight", b + "ln1.bias")
            q = lin(h, b + "attn_q").reshape(n, H, D).transpose(1, 0, 2)
            k = lin(h, b + "attn_k").reshape(n, H, D).transpose(1, 0, 2)
            v = lin(h, b + "attn_v").reshape(n, H, D).transpose(1, 0, 2)
            s = q @ k.transpose(0, 2, 1) / math.sqrt(D)
            s = np.exp(s - s.max(-1, keepdims=True))
            s /= s.sum(-1, keepdims=True)
            o = (s @ v).transpose(1, 0, 2).reshape(n, c.E)
            x = x + lin(o, b + "attn_out")
            h = lin(ln(x, b + "ln2.weight", b + "ln2.bias"), b + "ffn_up")
            h = 0.5 * h * (1 + np.vectorize(math.erf)(h / math.sqrt(2))) if c.use_gelu else h / (1 + np.exp(-1.702 * h))
            x = x + lin(h, b + "ffn_down")
        if "v.post_ln.weight" in g.tensors:
            x = ln(x, "v.post_ln.weight", "v.post_ln.bias")
        x = x[1:]
        h = lin(x, "mm.0")
        h = 0.5 * h * (1 + np.vectorize(math.erf)(h / math.sqrt(2)))
        return lin(h, "mm.2")
    finally:
        g.close()


def write_random_clip_gguf(path: str, out_dim: int, image_size: int = 336, patch_size: int = 14, E: int = 1024,
                           F_: int = 4096, n_layer: int = 23, n_head: int = 16, seed: int = 0,
                           use_gelu: bool = False, grid_pinpoints=None, merge: str = "spatial_unpad") -> None:
    """Random-init LLaVA-1.5-shaped projector file (F16 matrices, F32 norms/biases), as llama.cpp's
    llava surgery writes it. Defaults: CLIP ViT-L/14-336 with 23 of 24 blocks, 4096-wide MLP projector.
    grid_pinpoints [(w, h), ...] makes it LLaVA-1.6-shaped (any-resolution metadata + image_newline)."""
    from ..gguf.constants import GGMLType
    from ..gguf.writer import GGUFWriter
    rng = np.random.default_rng(seed)
    w = GGUFWriter(path)
    md = {"general.architecture": "clip", "general.name": "random-clip", "clip.has_text_encoder": False,
          "clip.has_vision_encoder": True, "clip.has_llava_projector": True, "clip.projector_type": "mlp",
          "clip.use_gelu": bool(use_gelu), "clip.vision.image_size": image_size, "clip.vision.patch_size": patch_size,
          "clip.vision.embedding_length": E, "clip.vision.feature_length": F_, "clip.vision.projection_dim": 768,
          "clip.vision.block_count": n_layer, "clip.vision.attention.head_count": n_head,
          "clip.vision.attention.layer_norm_epsilon": 1e-5,
          "clip.vision.image_mean": [0.48145466, 0.4578275, 0.40821073],
          "clip.vision.image_std": [0.26862954, 0.26130258, 0.27577711]}
    if grid_pinpoints:
        md["clip.vision.image_grid_pinpoints"] = [int(v) for wh in grid_pinpoints for v in wh]
        md["clip.vision.mm_patch_merge_type"] = merge
    for k, v in md.items():
        w.add(k, v)
    n_pos = (image_size // patch_size) ** 2 + 1

    def add(name, torch_shape, std, f16=True, base=0.0):
        data = (base + std * rng.standard_normal(int(np.prod(torch_shape)))).astype(np.float32)
        gt = GGMLType.F16 if f16 else GGMLType.F32
        w.add_tensor(name, tuple(reversed(torch_shape)), gt, data.astype(np.float16) if f16 else data)

    add("v.patch_embd.weight", (E, 3, patch_size, patch_size), 0.02)
    add("v.class_embd", (E,), 0.02, f16=False)
    add("v.position_embd.weight", (n_pos, E), 0.02)
    add("v.pre_ln.weight", (E,), 0.05, f16=False, base=1.0)
    add("v.pre_ln.bias", (E,), 0.02, f16=False)
    for i in range(n_layer):
        b = f"v.blk.{i}."
        for m in ("attn_q", "attn_k", "attn_v", "attn_out"):
            add(b + m + ".weight", (E, E), 1.0 / math.sqrt(E))
            add(b + m + ".bias", (E,), 0.02, f16=False)
        add(b + "ffn_up.weight", (F_, E), 1.0 / math.sqrt(E))
        add(b + "ffn_up.bias", (F_,), 0.02, f16=False)
        add(b + "ffn_down.weight", (E, F_), 1.0 / math.sqrt(F_))
        add(b + "ffn_down.bias", (E,), 0.02, f16=False)
        for ln in ("ln1", "ln2"):
            add(b + ln + ".weight", (E,), 0.05, f16=False, base=1.0)
            add(b + ln + ".bias", (E,), 0.02, f16=False)
    add("mm.0.weight", (out_dim, E), 1.0 / math.sqrt(E))
    add("mm.0.bias", (out_dim,), 0.02, f16=False)
    add("mm.2.weight", (out_dim, out_dim), 1.0 / math.sqrt(out_dim))
    add("mm.2.bias", (out_dim,), 0.02, f16=False)
    if grid_pinpoints and merge == "spatial_unpad":
        add("model.image_newline", (out_dim,), 0.5, f16=False)
    w.write()
