"""Plies/s of the sequential drop-in path: self_play(model, n, device) with a
model instance (one process-wide stream, one slot, the lazy schedule), as the
reference's callers invoke it (scripts/self_play.py:258-291)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd import self_play as SP  # noqa: E402
from knightvision_amd.model import ChessNet  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 4
m = ChessNet()
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()})
m.eval()
dev = torch.device("cuda", 0)
SP.self_play(m, 1, dev, max_moves=40)  # warm-up (engine creation, first launches)
t0 = time.perf_counter()
data = SP.self_play(m, n, dev)
dt = time.perf_counter() - t0
print(f"sequential self_play: {n} games, {len(data)} plies in {dt:.2f} s = {len(data) / dt:.0f} plies/s", flush=True)
