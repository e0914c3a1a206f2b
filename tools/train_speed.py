"""Update-step throughput of the training forward + backward (train.py's per-batch
work) under different convolution formulations, on one GPU.

    python tools/train_speed.py [B ...]
"""
import os
import sys
import time

import numpy as np
import torch
import torch.nn.functional as F

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
from knightvision_amd.model import ChessNet  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402
from knightvision_amd import train as T  # noqa: E402


def conv_gemm(x, w, b):
    """3x3 conv, padding 1, as im2col + one GEMM (hipBLASLt under autocast)."""
    B, C, H, W = x.shape
    cols = F.unfold(x, 3, padding=1)  # [B, C*9, 64]
    y = torch.matmul(w.view(w.shape[0], -1), cols)  # [B, Cout, 64]
    return (y + b.view(1, -1, 1)).view(B, -1, H, W)


def run(mode, B, iters=5):
    m = ChessNet().cuda()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()})
    m.train()
    if mode == "channels_last":
        m = m.to(memory_format=torch.channels_last)
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    scaler = T.make_scaler("cuda")
    x = torch.randint(0, 2, (B, 12, 8, 8), device="cuda").float()
    if mode == "channels_last":
        x = x.to(memory_format=torch.channels_last)
    mv = torch.randint(0, 4096, (B,), device="cuda")
    oc = torch.rand(B, device="cuda") * 2 - 1
    b = T.Batch(x, mv, oc)
    orig = F.conv2d
    if mode == "gemm":
        def patched(inp, weight, bias=None, stride=1, padding=0, dilation=1, groups=1):
            if weight.shape[-1] == 3:
                return conv_gemm(inp, weight, bias)
            return orig(inp, weight, bias, stride, padding, dilation, groups)
        torch.nn.modules.conv.F.conv2d = patched
    try:
        for it in range(iters + 2):
            if it == 2:
                torch.cuda.synchronize()
                t0 = time.perf_counter()
            loss = T.batch_loss(m, b)[0]
            scaler.scale(loss).backward()
            scaler.step(opt)
            scaler.update()
            opt.zero_grad()
        torch.cuda.synchronize()
        dt = (time.perf_counter() - t0) / iters
    finally:
        torch.nn.modules.conv.F.conv2d = orig
    flop = 3 * 3175744512 * B
    print(f"{mode:14s} B={B:5d} {dt * 1e3:8.1f} ms/step {B / dt:9.0f} samples/s {flop / dt / 1e12:6.1f} TFLOP/s",
          flush=True)


if __name__ == "__main__":
    for B in [int(a) for a in (sys.argv[1:] or ["1024", "4096"])]:
        for mode in ["miopen", "channels_last", "gemm"]:
            run(mode, B)
