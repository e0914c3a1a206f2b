"""Calibration of the headline kernel against the vendor library: the 60
batched GEMMs of one F(4x8) Winograd residual conv at 2,048 boards
(M = 4,096 tile rows, N = 512, K = 512 per point) and a square 8192^3 GEMM in
fp32 through torch (rocBLAS / hipBLASLt, TF32 off), HIP-event timed -- the
yardstick for wino_gemm_kernel<512,4,2,1,2,32,60> (bench.py roofline)."""
import torch


def rate(b, m, n, k, iters=10):
    torch.backends.cuda.matmul.allow_tf32 = False
    x = torch.randn(b, m, k, device="cuda")
    w = torch.randn(b, k, n, device="cuda")
    for _ in range(3):
        torch.bmm(x, w)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        torch.bmm(x, w)
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    tf = 2.0 * b * m * n * k / (us * 1e-6) / 1e12
    print(f"torch.bmm fp32 {b} x M={m} N={n} K={k}: {us:8.1f} us  {tf:6.1f} TFLOP/s  {tf / 157.3:.3f} of 157.3",
          flush=True)


if __name__ == "__main__":
    rate(60, 4096, 512, 512)
    rate(1, 8192, 8192, 8192)
    rate(60, 4096, 512, 512)
