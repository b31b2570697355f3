"""Measurement tool: hipBLASLt bf16 throughput on a large square GEMM (the achievable MFMA rate on this box) and on
the roofline conv's im2col GEMM shape (M=131072, N=128, K=1152). Not part of the product."""
import torch


def timeit(fn, n=20):
    fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(n):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / n * 1e-3


for (M, N, K) in [(8192, 8192, 8192), (16384, 16384, 8192), (131072, 128, 1152), (131072, 256, 1152),
                  (65536, 1152, 384), (65536, 384, 1536)]:
    a = torch.randn(M, K, device="cuda").bfloat16()
    b = torch.randn(K, N, device="cuda").bfloat16()
    t = timeit(lambda: a @ b)
    print(f"M={M} N={N} K={K}: {t * 1e6:9.1f} us  {2.0 * M * N * K / t / 1e12:7.1f} TF/s", flush=True)
