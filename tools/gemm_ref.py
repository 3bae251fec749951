"""Library GEMM reference (torch.mm -> hipBLASLt) at the implicit-GEMM shapes of the res conv:
what a plain GEMM of the same M x N x K reaches on this box, as a calibration for the conv
kernels' TFLOP/s (they also do the im2col staging the GEMM does not)."""
import json
import torch

def bench(m, n, k, iters=20):
    a = torch.randn(m, k, device="cuda", dtype=torch.bfloat16)
    b = torch.randn(k, n, device="cuda", dtype=torch.bfloat16)
    for _ in range(3):
        torch.mm(a, b)
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.mm(a, b)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    return {"m": m, "n": n, "k": k, "us": round(us, 1), "tflops": round(2 * m * n * k / us / 1e6, 1)}

for shape in [(131072, 256, 2304), (256, 131072, 2304), (2304, 256, 131072), (8192, 8192, 8192)]:
    print(json.dumps(bench(*shape)))
