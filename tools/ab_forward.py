"""A/B helper: forward timing (HIP events) of the library at KV_LIB_PATH on
seeded boards, and the outputs saved for a bit-for-bit comparison of builds.

    KV_LIB_PATH=knightvision_amd/libkv_b.so python tools/ab_forward.py TAG 2048 256
    (KV_PREC=f64w: the fp64 Winograd domain; KV_ALGO=winograd88 etc.: an fp32 conv algorithm)
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd.model import ChessNet  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402

tag = sys.argv[1]
m = ChessNet(precision=os.environ.get("KV_PREC", "fp32"), algo=os.environ.get("KV_ALGO", "auto"))
m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "bn").items()})
m.eval()
net = m.kv_net(0)
OUT = os.environ.get("AB_DIR", "gpurun_out")  # the saved outputs: 2048-board logits are 32 MB each
os.makedirs(OUT, exist_ok=True)
for B in [int(a) for a in sys.argv[2:]]:
    g = torch.Generator().manual_seed(B)
    codes = torch.randint(0, 13, (B, 64), dtype=torch.int8, generator=g).cuda()
    for _ in range(3):
        p, v = net.forward_boards(codes)
    torch.cuda.synchronize()
    np.save(f"{OUT}/ab_{tag}_{B}_p.npy", p.cpu().numpy())
    np.save(f"{OUT}/ab_{tag}_{B}_v.npy", v.cpu().numpy())
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    best = []
    for rep in range(3):
        e0.record()
        for _ in range(10):
            net.forward_boards(codes)
        e1.record()
        torch.cuda.synchronize()
        best.append(e0.elapsed_time(e1) / 10)
    print(f"{tag} B={B} forward ms {' '.join(f'{x:.3f}' for x in best)}", flush=True)
