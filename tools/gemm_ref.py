#!/usr/bin/env python3
"""Library reference point for the conv roofline discussion: hipBLASLt bf16
GEMM (torch.matmul) TFLOP/s on the implicit-GEMM shape of the dominant conv
(M pixels x K=1152 x N=128) and on square shapes, same HIP-event protocol."""
import torch
dev = torch.device("cuda", 0)
def bench(M, K, N, it=10):
    a = torch.randn(M, K, device=dev, dtype=torch.bfloat16)
    b = torch.randn(K, N, device=dev, dtype=torch.bfloat16)
    for _ in range(3):
        c = a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        c = a @ b
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / it
    print(f"M={M:9d} K={K:5d} N={N:5d}  {ms:8.3f} ms  {2*M*K*N/ms/1e9:7.1f} TF", flush=True)
for M, K, N in [(1 << 21, 1152, 128), (1 << 22, 1152, 128), (1 << 21, 1152, 256), (1 << 21, 576, 64),
                (8192, 8192, 8192), (4096, 4096, 4096)]:
    bench(M, K, N)
