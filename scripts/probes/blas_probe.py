"""Probe: library fp16 GEMM throughput on the prefill shapes (Y[M][N] = X[M][K] . W[N][K]^T)."""
import torch
import time

shapes = [(2048, 22016, 4096), (2048, 12288, 4096), (2048, 4096, 11008), (2048, 4096, 4096), (512, 22016, 4096),
          (2048, 32000, 4096)]
for M, N, K in shapes:
    x = torch.randn(M, K, device="cuda", dtype=torch.float16)
    w = torch.randn(N, K, device="cuda", dtype=torch.float16)
    for name, fn in [("f16out", lambda: torch.mm(x, w.t())),
                     ("f32out", lambda: torch.mm(x, w.t(), out_dtype=torch.float32))]:
        try:
            fn()
        except Exception as e:  # noqa: BLE001
            print(name, "unsupported:", str(e)[:100])
            continue
        torch.cuda.synchronize()
        n = 20
        t0 = time.perf_counter()
        for _ in range(n):
            fn()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / n
        print(f"M={M} N={N} K={K} {name}: {dt * 1e6:8.1f} us  {2 * M * N * K / dt / 1e12:7.1f} TFLOP/s", flush=True)
