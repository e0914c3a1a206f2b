"""Update-step throughput of the training forward + backward + Adam step
(train.py's per-batch work, autocast fp16) on one GPU: "hip" = the tower on the
HIP training kernels (train_ops, the default), "miopen" = whole-batch MIOpen
convolutions, "chunked" = MIOpen convolutions split into 1024-image chunks
(model.conv_chunked). KV_TRAIN_MODES picks the modes (default hip,chunked). (A channels-last im2col-GEMM formulation of the convolutions was also
measured: 14.4 K samples/s at 1024, 15.6 K at 4096 -- not kept.)

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


def run(mode, B, iters=5):
    m = ChessNet().cuda()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()})
    m.train()
    opt = torch.optim.Adam(m.parameters(), lr=1e-4)
    scaler = T.make_scaler("cuda")
    x = torch.randint(0, 2, (B, 12, 8, 8), device="cuda").float()
    mv = torch.randint(0, 4096, (B,), device="cuda")
    oc = torch.rand(B, device="cuda") * 2 - 1
    b = T.Batch(x, mv, oc)
    import knightvision_amd.model as KM
    KM.CONV_CHUNK = 0 if mode in ("miopen", "channels_last") else 1024
    KM.TRAIN_BACKEND = "hip" if mode == "hip" else "miopen"
    if mode.startswith("channels_last"):
        m = m.to(memory_format=torch.channels_last)
        b = T.Batch(x.contiguous(memory_format=torch.channels_last), mv, oc)
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
        KM.CONV_CHUNK = 1024
        KM.TRAIN_BACKEND = "hip"
    flop = 3 * 3175744512 * B
    print(f"{mode:14s} B={B:5d} {dt * 1e3:8.1f} ms/step {B / dt:9.0f} samples/s {flop / dt / 1e12:6.1f} TFLOP/s",
          flush=True)


if __name__ == "__main__":
    for B in [int(a) for a in (sys.argv[1:] or ["1024", "4096"])]:
        for mode in os.environ.get("KV_TRAIN_MODES", "hip,chunked").split(","):
            run(mode, B)
