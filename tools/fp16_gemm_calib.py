"""Calibration of the fp16 MFMA rate this box sustains under power limits:
hipBLASLt (torch.matmul, fp16 in / fp32 accumulate) on the training conv's
implicit-GEMM shape (M = 4,096 boards x 64 squares, N = 512, K = 9 x 512) and
on a square 8192^3 GEMM, HIP-event timed -- the yardstick for the hand-written
conv3x3_f16_kernel (tools/train_conv_bench.py), which also needs no im2col."""
import torch


def rate(m, n, k, iters=20):
    a = torch.randn(m, k, device="cuda", dtype=torch.float16)
    b = torch.randn(k, n, device="cuda", dtype=torch.float16)
    for _ in range(3):
        a @ b
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(iters):
        a @ b
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) / iters * 1e3
    tf = 2.0 * m * n * k / (us * 1e-6) / 1e12
    print(f"hipBLASLt fp16 M={m} N={n} K={k}: {us:8.1f} us  {tf:7.1f} TFLOP/s  {tf / 2500:.3f} of 2.5 PF", flush=True)


if __name__ == "__main__":
    rate(4096 * 64, 512, 9 * 512)
    rate(8192, 8192, 8192)
    rate(4096 * 64, 512, 9 * 512)
