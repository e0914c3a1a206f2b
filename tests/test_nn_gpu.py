"""HIP ChessNet forward vs the reference's own outputs (golden nn.npz) and vs
the torch fp32 restatement at several batch sizes. Tolerance: |logit| abs
error <= 1e-4 (north_star), value abs error <= 1e-5."""
import os

import numpy as np
import pytest
import torch

from knightvision_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
TOL_P, TOL_V = 1e-4, 1e-5


# (precision, conv algorithm): fp32 direct / fp32 Winograd F(8x8,3x3) on fp32 MFMA / fp32 auto (the calibrated
# choice every product caller runs) / F(8x8) with the fp64 Winograd domain on fp64 MFMA / the same domain with the
# GEMMs on int8 digits; ("fp32", "winograd88i8") the fp32 F(8x8) tower with its GEMMs on 4 int8 digits,
# ("fp32", "winograd88i8v") the same with fp64 input transforms, ("fp32", "winograd88i8r3") on 3 radix-256 digits.
# (The F(4x8) towers in fp32 and on the f16x3 split were retired in round 6.)
MODES = [("fp32", "direct"), ("fp32", "winograd88"), ("fp32", "winograd88i8"), ("fp32", "winograd88i8v"),
         ("fp32", "winograd88i8r3"), ("fp32", "auto"), ("f64w", "auto"), ("i8x5", "auto"), ("i8r4", "auto")]
# the explicit fp32 Winograd towers are outside the tolerance at trained magnitudes ("stress": 1.2e-3 to
# 3.6e-3); AUTO measures that at load time and runs the fp64 Winograd domain instead (test_nn_accuracy_gpu.py)
UNGUARDED = {("fp32", "winograd88"), ("fp32", "winograd88i8"), ("fp32", "winograd88i8v"),
             ("fp32", "winograd88i8r3")}
# the 24-bit tower (3 radix-256 digits) is also outside at the peaked set's logit magnitudes (|logit| up to 8.2:
# 1.03e-4, a relative 1.3e-5); AUTO measures that too and takes it only where it holds the budget (random-init
# weights: 2.4e-6 on the calibration boards)
UNGUARDED_PEAKED = {("fp32", "winograd88i8r3")}


def _net(variant, precision="fp32", algo="auto"):
    from knightvision_amd.model import ChessNet
    m = ChessNet(precision=precision, algo=algo)
    sd = synthetic_state_dict(42, variant)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.eval()


@pytest.mark.parametrize("precision,algo", MODES)
@pytest.mark.parametrize("variant", ["init", "bn", "peaked", "stress"])
def test_forward_matches_reference_golden(golden_dir, variant, precision, algo):
    if variant == "stress" and (precision, algo) in UNGUARDED:
        pytest.skip("explicit fp32 Winograd towers: outside the tolerance at trained magnitudes by design")
    if variant == "peaked" and (precision, algo) in UNGUARDED_PEAKED:
        pytest.skip("explicit 24-bit tower: outside the tolerance at peaked-logit magnitudes; AUTO guards it")
    g = np.load(os.path.join(golden_dir, "nn.npz"))
    m = _net(variant, precision, algo)
    p, v = m(torch.from_numpy(g["planes"]).cuda())
    torch.cuda.synchronize()
    dp = np.abs(p.cpu().numpy() - g[f"policy_{variant}"]).max()
    dv = np.abs(v.cpu().numpy() - g[f"value_{variant}"]).max()
    print(precision, algo, variant, "max |dpolicy|", dp, "max |dvalue|", dv)
    assert dp <= TOL_P and dv <= TOL_V


@pytest.mark.parametrize("precision,algo", MODES)
@pytest.mark.parametrize("B", [1, 2, 3, 31, 64, 257])
def test_forward_batch_sizes_vs_torch(B, precision, algo):
    from oracle import torch_ref
    rng = np.random.default_rng(B)
    codes = rng.integers(0, 13, size=(B, 64)) * (rng.random((B, 64)) < 0.4)
    from knightvision_amd.ai import codes_to_planes
    planes = codes_to_planes(codes)
    sd = synthetic_state_dict(42, "bn")
    m = _net("bn", precision, algo)
    p, v = m(torch.from_numpy(planes).cuda())
    rp, rv = torch_ref.forward(sd, planes)
    dp = np.abs(p.cpu().numpy() - rp.numpy()).max()
    dv = np.abs(v.cpu().numpy() - rv.numpy()).max()
    assert dp <= TOL_P and dv <= TOL_V, (dp, dv)
    # boards path (int8 codes, on-device encode) is the same computation
    pb, vb = m.kv_net(0).forward_boards(torch.from_numpy(codes.astype(np.int8)).cuda())
    assert np.abs(pb.cpu().numpy() - p.cpu().numpy()).max() == 0.0
    assert np.abs(vb.cpu().numpy() - v.cpu().numpy()).max() == 0.0


@pytest.mark.parametrize("precision", ["fp32", "f64w", "i8x5"])
def test_batch_invariance(precision):
    """A board's outputs do not depend on the batch it is evaluated in, within a
    batch-size class (<= 16 boards: split-K direct kernels; > 16: whole-K
    kernels, Winograd for fp32); across the two classes only the rounding
    differs (fp32 summation order / Winograd transforms)."""
    from knightvision_amd.ai import codes_to_planes
    rng = np.random.default_rng(7)
    codes = rng.integers(0, 13, size=(40, 64)) * (rng.random((40, 64)) < 0.4)
    planes = torch.from_numpy(codes_to_planes(codes)).cuda()
    m = _net("peaked", precision)
    p_all, v_all = m(planes)  # 40 boards: whole-K class
    p_20, v_20 = m(planes[20:])
    assert torch.equal(p_20, p_all[20:]) and torch.equal(v_20, v_all[20:])
    if precision in ("fp32", "f64w", "i8x5"):  # 300 boards run the 128-row GEMM tiles, 40 the 64-row ones
        codes_l = rng.integers(0, 13, size=(300, 64)) * (rng.random((300, 64)) < 0.4)
        codes_l[:40] = codes
        p_l, v_l = m(torch.from_numpy(codes_to_planes(codes_l)).cuda())
        assert torch.equal(p_l[:40], p_all) and torch.equal(v_l[:40], v_all)
    p_16, v_16 = m(planes[:16])  # split-K class
    for i in (0, 5, 15):
        p1, v1 = m(planes[i:i + 1])
        assert torch.equal(p1[0], p_16[i]) and torch.equal(v1[0], v_16[i])
    assert float((p_16 - p_all[:16]).abs().max()) < 1e-4


def test_forward_over_the_slice_limit():
    """a forward of more boards than one pass holds (16,384: the int8 kernels' 32-bit offsets) runs as
    equal slices (for_slices) -- 16,768 boards as 2 x 8,384 -- and every board's outputs are the bits it gets in a
    small batch of the same size class (batch invariance), at both ends of the range."""
    rng = np.random.default_rng(11)
    B = 16768
    codes = (rng.integers(0, 13, size=(B, 64)) * (rng.random((B, 64)) < 0.4)).astype(np.int8)
    net = _net("init").kv_net(0)  # random-init weights: the headline's path
    assert net.calibration()["path_large"] == "winograd88_i8f32r3"
    cd = torch.from_numpy(codes).cuda()
    p_all, v_all = net.forward_boards(cd)
    for lo, hi in ((0, 300), (8300, 8500), (B - 300, B)):
        p, v = net.forward_boards(cd[lo:hi])
        assert torch.equal(p, p_all[lo:hi]) and torch.equal(v, v_all[lo:hi]), (lo, hi)


@pytest.mark.parametrize("precision", ["fp32", "f64w", "i8x5", "i8r4", "fp32-i8", "fp32-r3"])
def test_wino88_batch_invariance(precision):
    """F(8x8) (one row per board): a board's outputs are the same bits at 20
    boards (padded to 32: 32-row GEMM tiles, k-tiles of 32), 80 / 96 (padded to
    96: 32-row tiles, k-tiles of 16), 40 / 300 (padded to 64 / 320: 64x128
    tiles) and 512 boards (128x128 tiles for points 0-95, 64x128 for 96-99).
    f64w (the fp64 Winograd domain, every batch size): 32 / 64 / 128-row tiles,
    the same k-steps. i8x5: 32 / 64-row tiles of an exact integer GEMM."""
    from knightvision_amd.ai import codes_to_planes
    rng = np.random.default_rng(88)
    codes = rng.integers(0, 13, size=(512, 64)) * (rng.random((512, 64)) < 0.4)
    planes = torch.from_numpy(codes_to_planes(codes)).cuda()
    m = (_net("peaked", "fp32", "winograd88") if precision == "fp32" else
         _net("peaked", "fp32", "winograd88i8") if precision == "fp32-i8" else
         _net("peaked", "fp32", "winograd88i8r3") if precision == "fp32-r3" else _net("peaked", precision, "auto"))
    p_l, v_l = m(planes)
    for lo, hi in ((0, 40), (20, 40), (0, 300), (0, 96), (16, 96)) + (((0, 1), (5, 8)) if precision != "fp32" else ()):
        p, v = m(planes[lo:hi])
        assert torch.equal(p, p_l[lo:hi]) and torch.equal(v, v_l[lo:hi]), (lo, hi)


@pytest.mark.parametrize("precision,tol", [("i8x5", 1e-5), ("i8r4", 4e-5)])
@pytest.mark.parametrize("variant", ["peaked", "stress"])
def test_i8_digits_track_fp64_domain(variant, precision, tol):
    """The int8-digit GEMMs (KV_PREC_I8X5: per-row 35-bit block fixed point, 15 of 25 digit pairs, exact
    int32 levels) are within ~2^-36 of the fp64 products, so the tower lands on the fp64-MFMA tower's outputs to
    within the truncation (~2^-35 of each row's magnitude) and the fp32 rounding
    of the activations between layers it can flip: logits within 1e-5 (a few
    fp32 ulps of the peaked set's logits, which reach ~30) of KV_PREC_F64W's at
    1 / 31 / 300 boards (measured: 2.4e-6 at one board, peaked). KV_PREC_I8R4 (31-bit block fixed point, 13
    of 16 radix-256 pairs) within the calibration's 4e-5."""
    from knightvision_amd.ai import codes_to_planes
    rng = np.random.default_rng(55)
    codes = rng.integers(0, 13, size=(300, 64)) * (rng.random((300, 64)) < 0.4)
    planes = torch.from_numpy(codes_to_planes(codes)).cuda()
    mi, md = _net(variant, precision), _net(variant, "f64w")
    for n in (1, 31, 300):
        pi, vi = mi(planes[:n])
        pd, vd = md(planes[:n])
        dp, dv = float((pi - pd).abs().max()), float((vi - vd).abs().max())
        print(variant, n, precision, "vs f64w: max |dlogit|", dp, "|dvalue|", dv)
        assert dp < tol and dv < tol / 10, (n, dp, dv)


@pytest.mark.parametrize("B", [17, 300, 2048])
def test_legal_logits_equal_full_rows(B):
    """kv_net_forward_boards_legal (the MCTS leaves' policy: listed moves only,
    one fmaf chain per move) equals the full policy_fc rows bit for bit."""
    from knightvision_amd.engine import packed_from
    from knightvision_amd.model import KVNet
    net = KVNet(0, packed_from(synthetic_state_dict(42, "peaked")))
    g = torch.Generator().manual_seed(B)
    codes = (torch.randint(0, 13, (B, 64), generator=g) * (torch.rand(B, 64, generator=g) < 0.4)).to(torch.int8)
    moves = torch.randint(0, 4096, (B, 320), generator=g, dtype=torch.int32).to(torch.int16)
    n = torch.randint(0, 321, (B,), generator=g, dtype=torch.int32)
    n[0], n[-1] = 0, 320
    pol, val = net.forward_boards(codes.cuda())
    leg, lval = net.forward_boards_legal(codes.cuda(), moves.cuda(), n.cuda())
    pol, leg = pol.cpu().numpy(), leg.cpu().numpy()
    mv = moves.numpy().astype(np.int64) & 0xFFFF
    idx = (mv & 63) * 64 + ((mv >> 6) & 63)
    for b in range(B):
        k = int(n[b])
        assert np.array_equal(leg[b, :k].view(np.int32), pol[b, idx[b, :k]].view(np.int32)), b
        assert np.all(leg[b, k:] == 0)
    assert torch.equal(val.cpu(), lval.cpu())
    net.close()
