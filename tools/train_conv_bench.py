"""Microbenchmark of the HIP training convolutions (csrc/kv_train.hip) at one
shape: forward (= data-gradient kernel), weight gradient; HIP-event time per
launch and TFLOP/s against the dense fp16 MFMA peak (2.5 PFLOP/s).

    python tools/train_conv_bench.py [boards] [ci] [co] [iters]
"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd import train_ops as TO  # noqa: E402

PEAK = 2500.0


def timeit(fn, iters):
    fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(iters):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / iters * 1e3  # us


def main():
    n, ci, co, iters = (int(x) for x in (sys.argv[1:] + ["4096", "512", "512", "20"][len(sys.argv) - 1:])[:4])
    g = torch.Generator(device="cuda").manual_seed(1)
    x = torch.randn(n, 64, ci, device="cuda", generator=g).half()
    dy = torch.randn(n, 64, co, device="cuda", generator=g).half()
    w = torch.randn(co, ci, 3, 3, device="cuda", generator=g) * 0.02
    wf, _ = TO.conv_weight_images(w, ci, False)
    flop = 2.0 * n * 64 * co * ci * 9
    t_f = timeit(lambda: TO.conv3x3_f16(x, wf, None), iters)
    t_w = timeit(lambda: TO.conv3x3_wgrad_f16(dy, x, ci), iters)
    for name, t in (("forward", t_f), ("wgrad", t_w)):
        tf = flop / (t * 1e-6) / 1e12
        print(f"{name:8s} n={n} ci={ci} co={co}: {t:8.1f} us  {tf:7.1f} TFLOP/s  {tf / PEAK:.3f} of fp16 MFMA peak",
              flush=True)


if __name__ == "__main__":
    main()
