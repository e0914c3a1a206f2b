"""Accuracy of every fp32 conv path of the HIP ChessNet against a float64
forward (oracle/torch_ref.py in float64, the reference's ChessNet math,
ai/model.py:51-77), beside the reference's own fp32 CPU forward's error, on
256 seeded random boards, for the weight sets of weights.py -- "stress" is the
one at trained-network magnitudes (BN calibrated on data, logits of std 4).

north_star's bar: logits within 1e-4 of the reference (fp32), values within
1e-5. The AUTO path (what every product caller runs) must hold it against the
reference's fp32 forward; each explicit algorithm's error is printed."""
import numpy as np
import pytest
import torch

from knightvision_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu
TOL_P, TOL_V = 1e-4, 1e-5
N_BOARDS = 256


def _planes(n, seed=5):
    from knightvision_amd.ai import codes_to_planes
    rng = np.random.default_rng(seed)
    codes = rng.integers(0, 13, size=(n, 64)) * (rng.random((n, 64)) < 0.4)
    return codes_to_planes(codes)


def _net(sd, algo):
    from knightvision_amd.model import ChessNet
    m = ChessNet(precision=algo) if algo in ("f64w", "i8x5", "i8r4") else ChessNet(algo=algo)
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    return m.eval()


def _f64(sd, planes):
    from oracle import torch_ref
    sd64 = {k: torch.from_numpy(np.asarray(v, dtype=np.float64)) for k, v in sd.items()}
    p, v = torch_ref.forward(sd64, torch.from_numpy(planes.astype(np.float64)))
    return p.numpy(), v.numpy()


def accuracy_table(sd, planes, algos=("direct", "winograd88", "winograd88i8r3", "winograd88i8",
                                      "winograd88i8v", "i8r4", "i8x5", "f64w", "auto")):
    """{name: (max |dlogit|, max |dvalue|) vs float64} for the reference's fp32
    forward ("ref32") and each HIP algorithm, plus each algorithm against ref32."""
    from oracle import torch_ref
    p64, v64 = _f64(sd, planes)
    r32, rv32 = (t.numpy() for t in torch_ref.forward(sd, planes))
    out = {"ref32": (np.abs(r32 - p64).max(), np.abs(rv32 - v64).max(), 0.0, 0.0)}
    calib = None
    for a in algos:
        m = _net(sd, a)
        p, v = m(torch.from_numpy(planes).cuda())
        p, v = p.cpu().numpy(), v.cpu().numpy()
        out[a] = (np.abs(p - p64).max(), np.abs(v - v64).max(), np.abs(p - r32).max(), np.abs(v - rv32).max())
        if a == "auto":
            calib = m.kv_net(0).calibration()
            # the small-batch class (<= 16 boards) of the AUTO path too
            ps, vs = (t.cpu().numpy() for t in m(torch.from_numpy(planes[:16]).cuda()))
            out["auto<=16"] = (np.abs(ps - p64[:16]).max(), np.abs(vs - v64[:16]).max(),
                               np.abs(ps - r32[:16]).max(), np.abs(vs - rv32[:16]).max())
    return out, float(np.abs(p64).max()), calib


def _report(name, tab, pmax, nb, calib=None):
    print(f"\n{name}: max |logit| {pmax:.2f}, {nb} boards")
    if calib is not None:
        print(f"  AUTO calibration: > 16 boards {calib['path_large']}, <= 16 {calib['path_small']}; candidates "
              f"(max |dlogit|, |dvalue| vs fp64 on {calib['n_boards']} boards) "
              f"{ {k: (round(v, 9), round(calib['err_value'][k], 9)) for k, v in calib['err_logit'].items()} }, "
              f"direct <= 16: ({calib['err_small_logit']:.2e}, {calib['err_small_value']:.2e}); {calib['ms']:.0f} ms")
    for k, (dp, dv, dpr, dvr) in tab.items():
        print(f"  {k:10s} vs f64: dlogit {dp:.3e} dvalue {dv:.3e} | vs ref32: dlogit {dpr:.3e} dvalue {dvr:.3e}",
              flush=True)


@pytest.mark.parametrize("variant", ["bn", "peaked", "stress"])
def test_auto_within_tolerance_of_reference(variant):
    sd = synthetic_state_dict(42, variant)
    planes = _planes(N_BOARDS)
    tab, pmax, calib = accuracy_table(sd, planes)
    _report(variant, tab, pmax, N_BOARDS, calib)
    for k in ("auto", "auto<=16", "f64w", "i8x5", "i8r4"):
        _, _, dpr, dvr = tab[k]
        assert dpr <= TOL_P and dvr <= TOL_V, (k, dpr, dvr)
    if variant in ("bn",):  # random-init magnitudes: the fp32 F(8x8) tower on int8 digits passes and is chosen
        # (on 3 radix-256 digits where they hold the budget, else on 4 radix-128 ones)
        assert calib["path_large"] in ("winograd88_i8f32r3", "winograd88_i8f32") and calib["path_small"] == "direct"
    if variant == "stress":  # trained magnitudes: no fp32 Winograd tower passes; the fp64 domain on digits does
        assert calib["path_large"] == "winograd88_i8r"


def _bn_summary(sd):
    from knightvision_amd.weights import N_RES
    names = ["bn1", "bn2"] + [f"res_blocks.{i}.bn{j}" for i in range(N_RES) for j in (1, 2)]
    r = [np.abs(sd[n + ".running_mean"]) / np.sqrt(sd[n + ".running_var"] + 1e-5) for n in names]
    s = [sd[n + ".weight"] / np.sqrt(sd[n + ".running_var"] + 1e-5) for n in names]
    return float(np.median(np.concatenate(r))), float(np.median(np.abs(np.concatenate(s))))


def test_trained_weights_table():
    """Weights trained by the learn loop (knightvision_amd.learn.reinforcement_loop
    from the "init" set; scripts/learn.py:152-209) -- what the reference's
    self-play actually runs (a checkpoint, scripts/self_play.py:71-77).
    KV_TRAINED_ITERS / KV_TRAINED_GAMES / KV_TRAINED_MAX_MOVES size the run
    (default 2 x 64 games x 40 plies); the AUTO path must hold the tolerance."""
    import os
    from knightvision_amd.learn import reinforcement_loop
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import state_dict_to_numpy
    iters = int(os.environ.get("KV_TRAINED_ITERS", "2"))
    games = int(os.environ.get("KV_TRAINED_GAMES", "64"))
    mm = int(os.environ.get("KV_TRAINED_MAX_MOVES", "40"))
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()})
    stats = reinforcement_loop(m, iters, games, "cuda:0", max_moves=mm, log=print)
    sd = state_dict_to_numpy(m.state_dict())
    mu_sigma, scale = _bn_summary(sd)
    print(f"\ntrained: {iters} iterations x {games} games x <= {mm} plies, {stats[-1].get('records')} records, "
          f"last val_loss {stats[-1].get('val_loss')}; tower BN median |mu|/sigma {mu_sigma:.2f}, "
          f"median |scale| {scale:.2f}")
    nb = int(os.environ.get("KV_TRAINED_BOARDS", str(N_BOARDS)))
    tab, pmax, calib = accuracy_table(sd, _planes(nb))
    _report(f"trained-{iters}x{games}", tab, pmax, nb, calib)
    for k in ("auto", "auto<=16", "f64w", "i8x5", "i8r4"):
        _, _, dpr, dvr = tab[k]
        assert dpr <= TOL_P and dvr <= TOL_V, (k, dpr, dvr)


@pytest.mark.parametrize("variant", ["init", "peaked", "stress"])
def test_calibration_choice_is_consistent(variant):
    """kv_net_calibration: each candidate run was measured, the chosen path is the
    first in F(8x8) fp32 on 3 radix-256 int8 digits -> on 4 radix-128 ones -> the same with fp64 input transforms
    -> F(8x8) fp64 domain on int8
    digits -> F(8x8) fp64 order within the budget (the fp32-MFMA towers F(8x8) / F(4x8) left the chain in round 5: never within the budget
    where the int8-digit fp32 tower is not), and the engine reports the same choice for the same weights."""
    from knightvision_amd.engine import SelfPlayEngine
    sd = synthetic_state_dict(42, variant)
    c = _net(sd, "auto").kv_net(0).calibration()
    assert c["calibrated"] and c["n_boards"] == 64
    order = ["winograd88_i8f32r3", "winograd88_i8f32", "winograd88_i8f32v", "winograd88_i8r", "winograd88_f64"]
    ok = {k: c["err_logit"][k] <= c["tol_logit"] and c["err_value"][k] <= c["tol_value"] for k in c["err_logit"]}
    first = next(k for k in order if k == "winograd88_f64" or ok.get(k))
    assert c["path_large"] == first, c
    assert sorted(c["err_logit"]) == sorted(order[:order.index(first) + 1])  # each candidate up to the choice
    assert c["err_logit"].get("winograd88_f64", 0.0) < 1e-5 and c["err_logit"].get("winograd88_i8", 0.0) < 1e-5
    small_ok = c["err_small_logit"] <= c["tol_logit"] and c["err_small_value"] <= c["tol_value"]
    assert c["path_small"] == ("direct" if small_ok else "winograd88_f64")
    with SelfPlayEngine(sd, slots=4, n_games=4, max_moves=2) as eng:
        e = eng.calibration()
    assert (e["path_large"], e["path_small"]) == (c["path_large"], c["path_small"])
    assert e["err_logit"] == c["err_logit"]
