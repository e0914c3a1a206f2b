"""F(8x8) vs F(4x8) on one GPU: forward time (alternating, HIP events) at
256 / 1,024 / 2,048 boards and max |dlogit| / |dvalue| against the float64
restatement on the peaked and bn weights (KV_PROBE_BOARDS random boards, 64).

    python tools/wino88_probe.py
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd.ai import codes_to_planes  # noqa: E402
from knightvision_amd.model import ChessNet  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402
from oracle import torch_ref  # noqa: E402


def net(variant, algo):
    m = ChessNet(algo=algo)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, variant).items()})
    return m.eval()


def main():
    rng = np.random.default_rng(5)
    nb = int(os.environ.get("KV_PROBE_BOARDS", "64"))
    codes = rng.integers(0, 13, size=(nb, 64)) * (rng.random((nb, 64)) < 0.4)
    planes = codes_to_planes(codes)
    for variant in ("peaked", "bn"):
        sd64 = {k: torch.from_numpy(np.asarray(v, dtype=np.float64)) for k, v in synthetic_state_dict(42, variant).items()}
        rp, rv = torch_ref.forward(sd64, torch.from_numpy(planes.astype(np.float64)))
        for algo in ("winograd48", "winograd88"):
            p, v = net(variant, algo)(torch.from_numpy(planes).cuda())
            dp = np.abs(p.cpu().numpy().astype(np.float64) - rp.numpy()).max()
            dv = np.abs(v.cpu().numpy().astype(np.float64) - rv.numpy()).max()
            print(f"{variant} {algo}: max |dlogit| {dp:.3e} max |dvalue| {dv:.3e}", flush=True)
    nets = {a: net("bn", a).kv_net(0) for a in ("winograd48", "winograd88")}
    for B in (256, 1024, 2048):
        codes = torch.randint(0, 13, (B, 64), dtype=torch.int8, device="cuda")
        res = {a: [] for a in nets}
        for rep in range(3):
            for a, n in nets.items():
                for _ in range(3):
                    n.forward_boards(codes)
                torch.cuda.synchronize()
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                e0.record()
                for _ in range(10):
                    n.forward_boards(codes)
                e1.record()
                torch.cuda.synchronize()
                res[a].append(e0.elapsed_time(e1) / 10)
        print(f"B={B}: " + "  ".join(f"{a} {min(t):.3f} ms ({' '.join(f'{x:.3f}' for x in t)})"
                                     for a, t in res.items()), flush=True)


if __name__ == "__main__":
    main()
