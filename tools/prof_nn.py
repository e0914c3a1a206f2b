"""Five ChessNet forwards at batch 256 (the bench's per-sim batch) for PMC passes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd.model import ChessNet  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402

B = int(sys.argv[1]) if len(sys.argv) > 1 else 256
m = ChessNet(precision=os.environ.get("KV_PREC", "fp32"))
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()})
m.eval()
net = m.kv_net(0)
codes = torch.randint(0, 13, (B, 64), dtype=torch.int8, device="cuda")
for _ in range(5):
    net.forward_boards(codes)
torch.cuda.synchronize()
print("done", B)
