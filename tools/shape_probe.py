"""MIOpen cost of a new training batch size: one update step per listed size (the
first call of a size pays the convolution solution selection)."""
import os, sys, time
import numpy as np, torch
sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")
from knightvision_amd.model import ChessNet
from knightvision_amd.weights import synthetic_state_dict
from knightvision_amd import train as T
m = ChessNet().cuda(); m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()}); m.train()
opt = torch.optim.Adam(m.parameters(), lr=1e-4); scaler = T.make_scaler("cuda")
def step(B):
    x = torch.randint(0, 2, (B, 12, 8, 8), device="cuda").float()
    b = T.Batch(x, torch.randint(0, 4096, (B,), device="cuda"), torch.rand(B, device="cuda"))
    torch.cuda.synchronize(); t0 = time.perf_counter()
    loss = T.batch_loss(m, b)[0]; scaler.scale(loss).backward(); scaler.step(opt); scaler.update(); opt.zero_grad()
    torch.cuda.synchronize(); return time.perf_counter() - t0
for B in [1024, 1024, 1416, 1416, 1417, 1417, 2000, 2000, 4096, 4096]:
    print(B, round(step(B) * 1e3, 1), "ms", flush=True)
