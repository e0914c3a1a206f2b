"""Host emulation (planning only; nothing in the product depends on it): the
F(8x8) Winograd GEMMs computed from int8 slices with exact integer accumulation
(Ozaki-style splitting), transforms and M in fp64, activations fp32 between
layers, against the float64 forward of the same weights.

Each V row (point xi, board; K = input channels) and each U row (xi, output
channel) is scaled by a power of two to |a| < 1 and split into s signed int8
digits d_i = round(r * 2^(7(i+1))) clamped to [-127, 127], remainder r carried
(|d_i| <= 64 unless a clamp carried). The product keeps the digit pairs
with i + j <= s - 1 (s(s+1)/2 int8 GEMMs, exact in int32 over K = 512), summed
per level and scaled back in fp64.

Mode prefix "f32" (e.g. f32row:4): the fp32 Winograd domain (U, V, M and
the transforms rounded to fp32, as the fp32 F(8x8) tower) with only the GEMM
from digits. Exponent modes for V: 'row' = exact max over the row's K channels; 'groupN'
= one exponent per N-channel group; 'bound' = per board, from max |y| of the
board's activations times the point's transform gain sum|B^T|.

    python tools/wino_ozaki_emulate.py stress 4
"""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from fractions import Fraction as Fr  # noqa: E402

from wino_emulate import _heads, toom_cook  # noqa: E402

from knightvision_amd.ai import codes_to_planes  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402
from oracle import torch_ref  # noqa: E402

F32 = np.float32
P88 = [Fr(0), Fr(2, 5), Fr(-2, 5), Fr(4, 5), Fr(-4, 5), Fr(5, 4), Fr(-5, 4), Fr(2), Fr(-2)]
AT, G, BT = toom_cook(P88, 8)


HEADROOM = 0  # 1: scale rows to |a| < 1/2 (no digit can exceed 64: no clamp needed)


def split(a, e, s):
    """a [..., K] fp64, e [..., 1] exponents with |a| * 2^-e < 1 -> s int digit arrays (as fp64)."""
    r = a * np.exp2(-e - HEADROOM)
    out = []
    for i in range(s):
        d = np.rint(r * 2.0 ** (7 * (i + 1)))
        d = np.clip(d, -127, 127)  # every digit int8 (a clamped digit carries into the next)
        out.append(d)
        r = r - d * 2.0 ** (-7 * (i + 1))
    return out


def split8(a, e, s):
    """radix-256 digits: N = rint(a 2^(31 - e)) (|a| 2^-e < 0.9921875 by the exponent rule), split into s signed
    bytes by the sign-extended low byte of what remains (d_{s-1} first), so N = sum_i d_i 2^(8 (s - 1 - i)) with
    every d_i in [-128, 127]; bits below 2^(e - 8 s + 1) are rounded away (s = 4: 31-bit block fixed point)."""
    N = np.rint(a * np.exp2(8 * s - 1 - e)).astype(np.int64)
    out = []
    for i in range(s):
        d = ((N + 128) & 255) - 128
        out.append(d.astype(np.float64))
        N = (N - d) >> 8
    assert np.abs(N).max() == 0 if N.size else True
    return out[::-1]


def exps8(a):
    m = np.abs(a).max(axis=-1, keepdims=True)
    m = np.maximum(m, 1e-300)
    fr, ex = np.frexp(m)  # m = fr 2^ex, fr in [0.5, 1)
    return ex + (fr >= 0.9921875)


def ozaki_gemm8(V, U, s, pairs):
    ev, eu = exps8(V), exps8(U)
    dv, du = split8(V, ev, s), split8(U, eu, s)
    M = np.zeros((V.shape[0], V.shape[1], U.shape[1]))
    for i in range(s):
        for j in range(s):
            if (i, j) in pairs:
                M += np.einsum("bxk,xok->bxo", dv[i], du[j]) * 2.0 ** (-8 * (i + j))
    return M * np.exp2(ev - 7) * np.exp2(eu[..., 0] - 7)[None]  # a = 2^(e - 7) sum_i d_i 2^(-8 i)


def exps(a, mode, gain=None, ymax=None):
    if mode == "row":
        m = np.abs(a).max(axis=-1, keepdims=True)
    elif mode == "bound":
        m = np.broadcast_to(gain[None, :, None] * ymax[:, None, None], a.shape[:-1] + (1,))
    m = np.maximum(m, 1e-300)
    return np.floor(np.log2(m)) + 1  # 2^(e-1) <= m < 2^e


def ozaki_gemm(V, U, s, mode, gain, ymax):
    """V [B,100,K], U [100,Cout,K] -> M [B,100,Cout]"""
    if mode == "f64":
        return np.einsum("bxk,xok->bxo", V, U)
    if mode.startswith("r8"):  # r8:4 the 10 pairs i + j <= 3 of radix-256 digits; r8p:4 also (1,3),(2,2),(3,1)
        pairs = {(i, j) for i in range(s) for j in range(s) if i + j <= s - 1}
        if mode == "r8p":
            pairs |= {(i, j) for i in range(s) for j in range(s) if i + j == s and 0 < i < s}
        return ozaki_gemm8(V, U, s, pairs)
    if mode.startswith("group"):
        B, X, K = V.shape
        gs = int(mode[5:])
        M = np.zeros((B, X, U.shape[1]))
        for g in range(K // gs):
            sl = slice(gs * g, gs * (g + 1))
            M += ozaki_gemm(V[..., sl], U[..., sl], s, "row", gain, ymax)
        return M
    # "rowNN" variants of 5 digits: row12 drops the interior top-level pairs (1,3), (2,2), (3,1); row11v keeps only
    # (4,0) (V's 5th digit) of them, row11u only (0,4) (U's)
    drop = {"row12": {(1, 3), (2, 2), (3, 1)}, "row11v": {(0, 4), (1, 3), (2, 2), (3, 1)},
            "row11u": {(4, 0), (1, 3), (2, 2), (3, 1)}}.get(mode, set())
    if mode in ("row12", "row11v", "row11u"):
        mode = "row"
    ev = exps(V, mode, gain, ymax)
    eu = exps(U, "row")
    dv, du = split(V, ev, s), split(U, eu, s)
    M = np.zeros((V.shape[0], V.shape[1], U.shape[1]))
    for lev in range(s):
        acc = np.zeros_like(M)
        for i in range(lev + 1):
            if (i, lev - i) in drop:
                continue
            acc += np.einsum("bxk,xok->bxo", dv[i], du[lev - i])  # exact: |acc| < 2^53
        M += acc * 2.0 ** (-7 * (lev + 2))
    return M * np.exp2(ev + HEADROOM) * np.exp2(eu[..., 0] + HEADROOM)[None]


def conv(x, w, s, mode):
    B, _, _, Cin = x.shape
    f32 = mode.startswith("f32")  # the fp32 Winograd domain: U, V, M and both transforms fp32
    if f32:
        mode = mode[3:] or "row"
    U = np.einsum("ak,oikl,bl->abio", G, w, G).reshape(100, Cin, -1).transpose(0, 2, 1)  # [100][Cout][Cin]
    xp = np.zeros((B, 10, 10, Cin))
    xp[:, 1:9, 1:9] = x
    if f32:
        U = U.astype(F32).astype(np.float64)
        V = np.einsum("ai,bicq->bacq", BT.astype(F32), xp.astype(F32)).astype(F32)
        V = np.einsum("bj,xajq->xabq", BT.astype(F32), V).astype(F32).reshape(B, 100, Cin).astype(np.float64)
    else:
        V = np.einsum("ai,bicq->bacq", BT, xp)
        V = np.einsum("bj,xajq->xabq", BT, V).reshape(B, 100, Cin)
    gain = np.outer(np.abs(BT).sum(1), np.abs(BT).sum(1)).reshape(100)
    ymax = np.abs(x).reshape(B, -1).max(1)
    M = ozaki_gemm(V, U, s, mode, gain, ymax).reshape(B, 10, 10, -1)
    if f32:
        M = M.astype(F32)
        Y = np.einsum("ia,bacq->bicq", AT.astype(F32), M).astype(F32)
        return np.einsum("jc,bicq->bijq", AT.astype(F32), Y).astype(F32).astype(np.float64)
    Y = np.einsum("ia,bacq->bicq", AT, M)
    return np.einsum("jc,bicq->bijq", AT, Y)


def fwd(sd, planes, s, mode):
    t = {k: np.asarray(v, dtype=np.float64) for k, v in sd.items()}

    def fold(c, b):
        sc = t[b + ".weight"] / np.sqrt(t[b + ".running_var"] + 1e-5)
        return sc, t[b + ".bias"] + (t[c + ".bias"] - t[b + ".running_mean"]) * sc

    x = torch.nn.functional.conv2d(torch.from_numpy(planes.astype(np.float64)), torch.from_numpy(t["conv1.weight"]),
                                   torch.from_numpy(t["conv1.bias"]), padding=1).numpy()
    sc, sh = fold("conv1", "bn1")
    x = np.maximum((x - t["conv1.bias"][None, :, None, None]) * sc[None, :, None, None] + sh[None, :, None, None], 0)
    x = x.transpose(0, 2, 3, 1).astype(F32)

    def cbr(x, c, b, res=None):
        y = conv(x.astype(np.float64), t[c + ".weight"], s, mode)
        sc, sh = fold(c, b)
        y = y * sc + sh
        if res is not None:
            y = y + res
        return np.maximum(y, 0).astype(F32)

    x = cbr(x, "conv2", "bn2")
    for r in range(5):
        h = cbr(x, f"res_blocks.{r}.conv1", f"res_blocks.{r}.bn1")
        x = cbr(h, f"res_blocks.{r}.conv2", f"res_blocks.{r}.bn2", res=x)
    sdt = {k: torch.from_numpy(v) for k, v in t.items()}
    return _heads(sdt, torch.from_numpy(x.transpose(0, 3, 1, 2).astype(np.float64)))


if __name__ == "__main__":
    variant = sys.argv[1]
    nb = int(sys.argv[2])
    if os.environ.get("HEADROOM"):
        HEADROOM = int(os.environ["HEADROOM"])
    cases = sys.argv[3:] or ["f64:0", "row:3", "row:4", "row:5", "row:6", "group128:5", "bound:5", "bound:6"]
    sd = synthetic_state_dict(42, variant)
    rng = np.random.default_rng(5)
    codes = rng.integers(0, 13, size=(nb, 64)) * (rng.random((nb, 64)) < 0.4)
    planes = codes_to_planes(codes)
    p64, v64 = torch_ref.forward({k: torch.from_numpy(np.asarray(v, dtype=np.float64)) for k, v in sd.items()},
                                 torch.from_numpy(planes.astype(np.float64)))
    p64, v64 = p64.numpy(), v64.numpy().reshape(-1)
    print(f"# python tools/wino_ozaki_emulate.py {variant} {nb}  (max over boards vs float64; budget 4e-5 / 4e-6)")
    for c in cases:
        mode, s = c.split(":")
        p, v = fwd(sd, planes, int(s), mode)
        print(f"{variant} {mode:9s} s={s} ({int(s) * (int(s) + 1) // 2:2d} int8 GEMMs)  dlogit {np.abs(p - p64).max():.3e}"
              f"  dvalue {np.abs(v - v64).max():.3e}", flush=True)
