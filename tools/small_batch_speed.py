"""Forward time of the <= 16-board (split-K) class at batch 1, 2, 8 and 16
(HIP events): the GUI / sequential self-play network path."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd.model import ChessNet  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402

m = ChessNet()
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "bn").items()})
m.eval()
net = m.kv_net(0)
out = []
for B in (1, 2, 8, 16):
    codes = torch.randint(0, 13, (B, 64), dtype=torch.int8, device="cuda")
    for _ in range(10):
        net.forward_boards(codes)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(100):
        net.forward_boards(codes)
    e1.record()
    torch.cuda.synchronize()
    out.append(f"B={B} {e0.elapsed_time(e1) * 10:.1f}us")
print(os.environ.get("KV_LIB_PATH", "default"), " ".join(out), flush=True)
