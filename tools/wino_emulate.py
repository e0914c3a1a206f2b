"""Host emulation of the fp32 Winograd tower's rounding (ChessNet, ai/model.py):
F(4x8) (the GPU default above 16 boards) against F(8x8) (one 10x10 tile per
board: 100 points instead of 120, 17 % fewer GEMM FLOPs and transform bytes),
with the GEMM's K = 512 accumulation emulated in fp32 in K order (two products
per step, as v_mfma_f32_32x32x2_f32 chains them) or split into S partial
accumulators summed at the end (S = 2, 4: the cost would be S x the
accumulator registers). Logit / value error against the float64 forward of
the same weights (oracle/torch_ref.forward), on the peaked weight set.

    python tools/wino_emulate.py [n_boards]

Planning tool only: nothing in the product depends on it.
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
from oracle import torch_ref  # noqa: E402

F32 = np.float32


def toom_cook(P, m, r=3):
    """A^T [m][n], G [n][r], B^T [n][n] as float64 arrays for points P + infinity."""
    f = lambda T: np.array([[float(x) for x in row] for row in T])  # noqa: E731
    return tuple(f(T) for T in toom_cook_exact(P, m, r))


def toom_cook_exact(P, m, r=3):
    """A^T [m][n], G [n][r], B^T [n][n] (exact rationals) for points P + infinity, n = m + r - 1."""
    n = m + r - 1
    assert len(P) == n - 1
    AT = [[Fr(0)] * n for _ in range(m)]
    G = [[Fr(0)] * r for _ in range(n)]
    for j, a in enumerate(P):
        den = Fr(1)
        for l, b in enumerate(P):
            if l != j:
                den *= a - b
        for i in range(m):
            AT[i][j] = a ** i
        for k in range(r):
            G[j][k] = a ** k / den
    AT[m - 1][n - 1] = Fr(1)
    G[n - 1][r - 1] = Fr(1)
    unknowns = n * n
    rows, rhs = [], []
    for i in range(m):
        for k in range(r):
            for l in range(n):
                row = [Fr(0)] * unknowns
                for j in range(n):
                    row[j * n + l] = AT[i][j] * G[j][k]
                rows.append(row)
                rhs.append(Fr(1) if l == i + k else Fr(0))
    A = [rw[:] + [b] for rw, b in zip(rows, rhs)]
    piv, rr = [], 0
    for c in range(unknowns):
        p = next((q for q in range(rr, len(A)) if A[q][c] != 0), None)
        if p is None:
            continue
        A[rr], A[p] = A[p], A[rr]
        inv = 1 / A[rr][c]
        A[rr] = [x * inv for x in A[rr]]
        for q in range(len(A)):
            if q != rr and A[q][c] != 0:
                f = A[q][c]
                A[q] = [x - f * y for x, y in zip(A[q], A[rr])]
        piv.append(c)
        rr += 1
    sol = [Fr(0)] * unknowns
    for q, c in enumerate(piv):
        sol[c] = A[q][-1]
    BT = [[sol[j * n + l] for l in range(n)] for j in range(n)]
    for i, k, l in itertools.product(range(m), range(r), range(n)):
        assert sum(AT[i][j] * G[j][k] * BT[j][l] for j in range(n)) == (1 if l == i + k else 0)
    return AT, G, BT


P4 = [Fr(0), Fr(1), Fr(-1), Fr(2), Fr(-2)]
P8 = [Fr(0), Fr(1), Fr(-1), Fr(1, 2), Fr(-1, 2), Fr(2), Fr(-2), Fr(3, 4), Fr(-3, 4)]


def conv_wino(x, w, tiles, split):
    """x [B,8,8,Cin] fp32 (NHWC), w [Cout,Cin,3,3] fp64 -> fp32 [B,8,8,Cout] 3x3 correlation, pad 1, through
    Winograd tiles (mr, mc) with fp32 transforms and the GEMM accumulated in fp32 in K order (split partials)."""
    (mr, ATr, Gr, BTr), (mc, ATc, Gc, BTc) = tiles
    B, _, _, Cin = x.shape
    Cout = w.shape[0]
    nr, nc = mr + 2, mc + 2
    # U = G g G^T in fp64, rounded once
    U = np.einsum("ak,oikl,bl->abio", Gr, w, Gc).astype(F32)  # [nr][nc][Cin][Cout]
    xp = np.zeros((B, 8 + 2 + 8, 8 + 2 + 8, Cin), F32)
    xp[:, 1:9, 1:9] = x
    out = np.zeros((B, 8, 8, Cout), F32)
    BTr32, BTc32, ATr32, ATc32 = (t.astype(F32) for t in (BTr, BTc, ATr, ATc))
    for ty in range(0, 8, mr):
        for tx in range(0, 8, mc):
            d = xp[:, ty:ty + nr, tx:tx + nc]  # [B, nr, nc, Cin]
            V = np.einsum("ai,bicq->bacq", BTr32, d).astype(F32)
            V = np.einsum("bj,xajq->xabq", BTc32, V).astype(F32)  # [B, nr, nc, Cin]
            M = np.zeros((B, nr, nc, Cout), F32)
            Vf = V.reshape(B, nr * nc, Cin)
            Uf = U.reshape(nr * nc, Cin, Cout)
            parts = []
            for s in range(split):
                acc = np.zeros((B, nr * nc, Cout), F32)
                k0, k1 = s * Cin // split, (s + 1) * Cin // split
                for k in range(k0, k1, 2):
                    p0 = (Vf[:, :, k, None] * Uf[None, :, k, :]).astype(F32)
                    p1 = (Vf[:, :, k + 1, None] * Uf[None, :, k + 1, :]).astype(F32)
                    acc = ((acc + p0).astype(F32) + p1).astype(F32)
                parts.append(acc)
            tot = parts[0]
            for p in parts[1:]:
                tot = (tot + p).astype(F32)
            M = tot.reshape(B, nr, nc, Cout)
            Y = np.einsum("ia,bacq->bicq", ATr32, M).astype(F32)
            Y = np.einsum("jc,bicq->bijq", ATc32, Y).astype(F32)  # [B, mr, mc, Cout]
            hy, hx = min(mr, 8 - ty), min(mc, 8 - tx)
            out[:, ty:ty + hy, tx:tx + hx] = Y[:, :hy, :hx]
    return out


def forward(sd, planes, tiles, split):
    """ChessNet eval forward: conv1 in fp64 (the GPU runs it direct), the 11 convs with Cin 256/512 through
    conv_wino, heads in fp64 (tiny); BN folded as the GPU folds it."""
    t = {k: np.asarray(v, dtype=np.float64) for k, v in sd.items()}

    def fold(conv, bn):
        sc = t[bn + ".weight"] / np.sqrt(t[bn + ".running_var"] + 1e-5)
        return sc, t[bn + ".bias"] + (t[conv + ".bias"] - t[bn + ".running_mean"]) * sc

    x = torch.nn.functional.conv2d(torch.from_numpy(planes.astype(np.float64)), torch.from_numpy(t["conv1.weight"]),
                                   torch.from_numpy(t["conv1.bias"]), padding=1).numpy()
    sc, sh = fold("conv1", "bn1")
    x = np.maximum((x - t["conv1.bias"][None, :, None, None]) * sc[None, :, None, None] + sh[None, :, None, None], 0)
    x = x.transpose(0, 2, 3, 1).astype(F32)

    def cbr(x, conv, bn, res=None):
        y = conv_wino(x, t[conv + ".weight"], tiles, split)
        sc, sh = fold(conv, bn)
        y = (y * sc.astype(F32) + sh.astype(F32)).astype(F32)
        if res is not None:
            y = (y + res).astype(F32)
        return np.maximum(y, 0).astype(F32)

    x = cbr(x, "conv2", "bn2")
    for r in range(5):
        h = cbr(x, f"res_blocks.{r}.conv1", f"res_blocks.{r}.bn1")
        x = cbr(h, f"res_blocks.{r}.conv2", f"res_blocks.{r}.bn2", res=x)
    xt = torch.from_numpy(x.transpose(0, 3, 1, 2).astype(np.float64))
    sdt = {k: torch.from_numpy(v) for k, v in t.items()}
    # heads in fp64 from the emulated tower output
    return torch_ref.heads(sdt, xt) if hasattr(torch_ref, "heads") else _heads(sdt, xt)


def _heads(p, x):
    F = torch.nn.functional

    def cbr(x, conv, bn):
        y = F.conv2d(x, p[conv + ".weight"], p[conv + ".bias"])
        y = F.batch_norm(y, p[bn + ".running_mean"], p[bn + ".running_var"], p[bn + ".weight"], p[bn + ".bias"],
                         False, 0.0, 1e-5)
        return F.relu(y)
    pol = F.linear(torch.flatten(cbr(x, "policy_conv", "policy_bn"), 1), p["policy_fc.weight"], p["policy_fc.bias"])
    v = torch.flatten(cbr(x, "value_conv", "value_bn"), 1)
    v = torch.tanh(F.linear(F.relu(F.linear(v, p["value_fc1.weight"], p["value_fc1.bias"])), p["value_fc2.weight"],
                            p["value_fc2.bias"]))
    return pol.numpy(), v.numpy().reshape(-1)


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 6
    sd = synthetic_state_dict(42, "peaked")
    g = np.load(os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "tests", "golden",
                             "movegen.npz"))
    codes = np.ascontiguousarray(g["states"][::700][:n, :64]).astype(np.int8)
    planes = codes_to_planes(codes)
    sd64 = {k: np.asarray(v, dtype=np.float64) for k, v in sd.items()}
    p64, v64 = torch_ref.forward({k: torch.from_numpy(v) for k, v in sd64.items()},
                                 torch.from_numpy(planes.astype(np.float64)))
    p64, v64 = p64.numpy(), v64.numpy().reshape(-1)
    AT4, G4, BT4 = toom_cook(P4, 4)
    AT8, G8, BT8 = toom_cook(P8, 8)
    f4x8 = ((4, AT4, G4, BT4), (8, AT8, G8, BT8))
    f8x8 = ((8, AT8, G8, BT8), (8, AT8, G8, BT8))
    for name, tiles in (("F(4x8)", f4x8), ("F(8x8)", f8x8)):
        for split in (1, 2, 4):
            p, v = forward(sd, planes, tiles, split)
            print(f"{name} split {split}: max |dlogit| {np.abs(p - p64).max():.3e}  max |dvalue| "
                  f"{np.abs(v - v64).max():.3e}", flush=True)


if __name__ == "__main__":
    main()
