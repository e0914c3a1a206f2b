"""Point-set search for an fp32 Winograd F(8x8,3x3) (planning tool only).

Proxy for the tower's logit error: one 512 -> 512 convolution
(res_blocks.0.conv1 of the peaked synthetic weights) on the tower's own
activations at that layer (float64 stem + conv2 of golden positions), computed
through fp32 transforms and an fp32 K-order GEMM accumulation (two products per
step, as tools/wino_emulate.py), error = max |dy| / rms(y) against the float64
convolution. Every candidate: 0, infinity and four symmetric pairs +-a drawn
from a small set of simple rationals (the same set on both axes). The current
F(4x8) (rows F(4,3) on 0, +-1, +-2; columns F(8,3) on 0, +-1/2, +-1, +-2,
+-3/4) is the yardstick.

    python tools/wino_points_search.py [n_boards]
"""
import itertools
import os
import sys
from fractions import Fraction as Fr

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd.ai import codes_to_planes  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402
from tools.wino_emulate import P4, P8, toom_cook  # noqa: E402

F32 = np.float32
CANDS = [Fr(1, 4), Fr(1, 3), Fr(1, 2), Fr(2, 3), Fr(3, 4), Fr(1), Fr(4, 3), Fr(3, 2), Fr(2), Fr(5, 2), Fr(3)]


def activations(n):
    sd = {k: torch.from_numpy(np.asarray(v, dtype=np.float64)) for k, v in synthetic_state_dict(42, "peaked").items()}
    g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "movegen.npz"))
    codes = np.ascontiguousarray(g["states"][::700][:n, :64]).astype(np.int8)
    x = torch.from_numpy(codes_to_planes(codes).astype(np.float64))
    F = torch.nn.functional
    for c, b in (("conv1", "bn1"), ("conv2", "bn2")):
        x = F.relu(F.batch_norm(F.conv2d(x, sd[c + ".weight"], sd[c + ".bias"], padding=1), sd[b + ".running_mean"],
                                sd[b + ".running_var"], sd[b + ".weight"], sd[b + ".bias"], False, 0.0, 1e-5))
    x = x.to(torch.float32).to(torch.float64)  # the tower carries fp32 activations
    w = sd["res_blocks.0.conv1.weight"]
    y = F.conv2d(x, w, padding=1)
    return x.numpy().transpose(0, 2, 3, 1), w.numpy(), y.numpy().transpose(0, 2, 3, 1)


def conv(x, w, tiles):
    (mr, ATr, Gr, BTr), (mc, ATc, Gc, BTc) = tiles
    B, _, _, Cin = x.shape
    nr, nc = mr + 2, mc + 2
    U = np.einsum("ak,oikl,bl->abio", Gr, w, Gc).astype(F32).reshape(nr * nc, Cin, -1)
    xp = np.zeros((B, 18, 18, Cin), F32)
    xp[:, 1:9, 1:9] = x.astype(F32)
    out = np.zeros((B, 8, 8, U.shape[2]), F32)
    BTr32, BTc32, ATr32, ATc32 = (t.astype(F32) for t in (BTr, BTc, ATr, ATc))
    for ty in range(0, 8, mr):
        for tx in range(0, 8, mc):
            d = xp[:, ty:ty + nr, tx:tx + nc]
            V = np.einsum("ai,bicq->bacq", BTr32, d).astype(F32)
            V = np.einsum("bj,xajq->xabq", BTc32, V).astype(F32).reshape(B, nr * nc, Cin)
            acc = np.zeros((B, nr * nc, U.shape[2]), F32)
            for k in range(0, Cin, 2):
                p0 = (V[:, :, k, None] * U[None, :, k, :]).astype(F32)
                p1 = (V[:, :, k + 1, None] * U[None, :, k + 1, :]).astype(F32)
                acc = ((acc + p0).astype(F32) + p1).astype(F32)
            M = acc.reshape(B, nr, nc, -1)
            Y = np.einsum("ia,bacq->bicq", ATr32, M).astype(F32)
            Y = np.einsum("jc,bicq->bijq", ATc32, Y).astype(F32)
            out[:, ty:ty + mr, tx:tx + mc] = Y[:, :min(mr, 8 - ty), :min(mc, 8 - tx)]
    return out


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 2
    x, w, y = activations(n)
    rms = float(np.sqrt((y ** 2).mean()))

    def err(tiles):
        return float(np.abs(conv(x, w, tiles).astype(np.float64) - y).max()) / rms

    t4, t8 = toom_cook(P4, 4), toom_cook(P8, 8)
    print(f"F(4x8) current: {err(((4,) + t4, (8,) + t8)):.3e}", flush=True)
    print(f"F(8x8) current points: {err(((8,) + t8, (8,) + t8)):.3e}", flush=True)
    res = []
    for pairs in itertools.combinations(CANDS, 4):
        P = [Fr(0)] + [s * a for a in pairs for s in (1, -1)]
        t = toom_cook(P, 8)
        e = err(((8,) + t, (8,) + t))
        res.append((e, pairs))
        print(f"{e:.3e} " + " ".join(str(a) for a in pairs), flush=True)
    res.sort()
    print("best:")
    for e, pairs in res[:10]:
        print(f"  {e:.3e} " + " ".join(str(a) for a in pairs))


if __name__ == "__main__":
    main()
