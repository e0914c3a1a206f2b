"""Quick ChessNet forward timing on one GPU (HIP events)."""
import sys
import time

import os
import numpy as np
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
import torch

from knightvision_amd.model import ChessNet
from knightvision_amd.weights import synthetic_state_dict

FLOP = 3175744512
prec = os.environ.get("KV_PREC", "fp32")
algo = os.environ.get("KV_ALGO", "auto")
m = ChessNet(precision=prec, algo=algo)
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "bn").items()})
m.eval()
net = m.kv_net(0)
for B in [int(a) for a in (sys.argv[1:] or ["256", "1024", "2048"])]:
    codes = torch.randint(0, 13, (B, 64), dtype=torch.int8, device="cuda")
    for _ in range(3):
        net.forward_boards(codes)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 10
    e0.record()
    for _ in range(n):
        net.forward_boards(codes)
    e1.record()
    torch.cuda.synchronize()
    ms = e0.elapsed_time(e1) / n
    print(f"{prec}/{algo} B={B} forward {ms:.3f} ms  {B/ms*1e3:.0f} boards/s  {B*FLOP/ms/1e9:.1f} TFLOP/s", flush=True)
