"""Debug helper: decode which V element the MFMA prefill attention's transposed LDS reads deliver
(K = 0 -> uniform attention; V[t][d] = 128 t + d, exact in fp16)."""
import math
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from ollama_operator_amd.ops import native  # noqa: E402

C = native()
S = torch.cuda.current_stream().cuda_stream
D, Hkv, G, bs, NQ = 64, 1, 1, 16, 16
H = Hkv * G
mb = NQ // bs
kc = torch.zeros(mb, Hkv, bs, D, device="cuda").half()
vc = torch.zeros(mb, Hkv, bs, D, device="cuda").half()
t = torch.arange(NQ, device="cuda")
d = torch.arange(D, device="cuda")
vc[t // bs, 0, t % bs, :] = (128 * t[:, None] + d[None, :]).half()
bt = torch.arange(mb, device="cuda", dtype=torch.int32).view(1, mb)
q = torch.randn(NQ, H * D, device="cuda")
qlen = torch.arange(1, NQ + 1, device="cuda", dtype=torch.int32)
qseq = torch.zeros(NQ, device="cuda", dtype=torch.int32)
out = torch.zeros(NQ, H * D, device="cuda")
C.attention(q.data_ptr(), H * D, kc.data_ptr(), vc.data_ptr(), bt.data_ptr(), mb, qseq.data_ptr(), qlen.data_ptr(), NQ,
            H, Hkv, D, bs, 1 / math.sqrt(D), 0, out.data_ptr(), H * D, 0, 1, 0, S, prefill=1)
torch.cuda.synchronize()
o0 = out[0].round().int().tolist()
print("query 0 (key 0 only): d -> (t_src, d_src)")
print([(v // 128, v % 128) for v in o0[:20]])
# query 1: mean of keys 0,1 -> key1 value = 2*out1 - out0
o1 = (2 * out[1] - out[0]).round().int().tolist()
print("key 1 slot:", [(v // 128, v % 128) for v in o1[:20]])
o2 = (3 * out[2] - 2 * out[1]).round().int().tolist()
print("key 2 slot:", [(v // 128, v % 128) for v in o2[:20]])
o3 = (4 * out[3] - 3 * out[2]).round().int().tolist()
print("key 3 slot:", [(v // 128, v % 128) for v in o3[:20]])
o4 = (5 * out[4] - 4 * out[3]).round().int().tolist()
print("key 4 slot:", [(v // 128, v % 128) for v in o4[:20]])
