"""CPU-side checks of the boundary: the C-ABI library loads and exports every
symbol include/kv.h declares (no device calls), the packed-weight layout of
the Python packer equals the library's, and the reference API surface
(ai/ai.py encoders, self_play constants / errors) behaves like the reference."""
import ctypes as C
import json
import os
import re

import numpy as np
import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def declared_symbols():
    hdr = open(os.path.join(REPO, "include", "kv.h")).read()
    hdr = re.sub(r"/\*.*?\*/", "", hdr, flags=re.S)
    return sorted(set(re.findall(r"\b(kv_[a-z_]+)\s*\(", hdr)))


def test_library_exports_every_declared_symbol():
    from knightvision_amd import _lib
    L = C.CDLL(_lib.LIB_PATH)
    missing = [s for s in declared_symbols() if not hasattr(L, s)]
    assert not missing, missing
    assert set(declared_symbols()) <= set(_lib.EXPORTED)


def test_packed_layout_matches_library():
    from knightvision_amd import _lib
    from knightvision_amd.weights import pack_weights, synthetic_state_dict
    blob, layout = pack_weights(synthetic_state_dict(42, "bn"))
    L = C.CDLL(_lib.LIB_PATH)
    L.kv_net_packed_size.restype = C.c_size_t
    assert blob.size == L.kv_net_packed_size()
    # conv weights are [Cout][9][CinPad] with BN folded into scale/shift
    off, n = layout["L2.w"]
    assert n == 512 * 9 * 512


def test_bn_folding_matches_reference_formula():
    from knightvision_amd.weights import _fold, synthetic_state_dict
    sd = synthetic_state_dict(42, "bn")
    w, scale, shift = _fold(sd, "conv2", "bn2")
    x = np.random.default_rng(0).standard_normal(512)
    conv = x  # per-channel pre-BN activations
    ref = ((conv + sd["conv2.bias"] - sd["bn2.running_mean"]) / np.sqrt(sd["bn2.running_var"] + 1e-5)
           * sd["bn2.weight"] + sd["bn2.bias"])
    np.testing.assert_allclose(conv * scale + shift, ref, rtol=1e-5, atol=1e-5)


def test_encoders_match_golden(golden_dir):
    from knightvision_amd.ai import encode_board, encode_move, decode_move_index, board_to_codes, codes_to_planes
    g = np.load(os.path.join(golden_dir, "nn.npz"))
    mg = np.load(os.path.join(golden_dir, "movegen.npz"))
    idx = np.linspace(0, len(mg["states"]) - 1, 12).astype(int)
    names = ["--", "wK", "wQ", "wR", "wB", "wN", "wp", "bK", "bQ", "bR", "bB", "bN", "bp"]
    for k, i in enumerate(idx):
        board = [[names[int(mg["states"][i][r * 8 + c])] for c in range(8)] for r in range(8)]
        assert np.array_equal(encode_board(board), g["planes"][k])
        assert np.array_equal(codes_to_planes(board_to_codes(board))[0], g["planes"][k])
    for sr, sc, er, ec in [(6, 4, 4, 4), (0, 0, 7, 7), (7, 6, 5, 5)]:
        i = encode_move(sr, sc, er, ec)
        assert 0 <= i < 4096 and decode_move_index(i) == (sr, sc, er, ec)


def test_self_play_api_surface():
    import knightvision_amd.self_play as sp
    assert sp.EPSILON == 0.25 and sp.ALPHA == 0.3 and sp.SEED == 42 and sp.BATCH_SIZE == 16
    with pytest.raises(ValueError):
        sp.self_play(None, 1, None)
    with pytest.raises(FileNotFoundError):
        sp._init_worker("/nonexistent/ckpt.pth", "cpu", 42)
    assert sp.piece_value("q") == 9 and sp.piece_value("wK") == 0
    for name in ("self_play", "generate_self_play_data", "_run_single_game", "_init_worker", "piece_value"):
        assert callable(getattr(sp, name))


def test_chessnet_state_dict_keys_match_reference_layout():
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import state_dict_spec
    sd = ChessNet().state_dict()
    spec = state_dict_spec()
    assert list(sd.keys()) == [n for n, _ in spec]
    for n, shape in spec:
        assert tuple(sd[n].shape) == tuple(shape), n


def _cfg(**kw):
    from knightvision_amd import _lib
    base = dict(device=0, slots=4, n_games=4, game_id_base=0, game_id_stride=1, seed=42, seed_mode=0, max_moves=0,
                batch=16, eps=0.25, alpha=0.3, sims=0, c_puct=1.5, eval_mode=0, record_cap=1 << 16, recycle=1,
                precision=0, algo=0, tree_edge_cap=0, keep_root_visits=0)
    base.update(kw)
    return _lib.Config(**base)


@pytest.mark.parametrize("kw, msg", [
    (dict(slots=0), "slots must be > 0"),
    (dict(n_games=-1), "slots must be > 0"),
    (dict(alpha=0.0), "DIR_NOISE_ALPHA"),
    (dict(alpha=1.5), "DIR_NOISE_ALPHA"),
    (dict(alpha=1.0), "DIR_NOISE_ALPHA"),          # shape 1: numpy's exponential branch, not restated
    (dict(alpha=1e-310), "DIR_NOISE_ALPHA"),       # subnormal: 1/alpha overflows
    (dict(alpha=float("nan")), "DIR_NOISE_ALPHA"),
    (dict(batch=0), "SELFPLAY_BATCH_SIZE"),
    (dict(seed_mode=7), "bad seed_mode"),
    (dict(seed_mode=1, slots=2), "sequential seeding"),
    (dict(sims=-1), "out of range"),
    (dict(sims=65001), "out of range"),
    (dict(sims=64, tree_edge_cap=100), "tree_edge_cap"),
    (dict(sims=64, seed_mode=1, slots=1), "per-game seeding"),
    (dict(sims=64, eval_mode=1), "eval_mode 1 not available"),
    (dict(eval_mode=5), "eval_mode 5 not available"),
])
def test_kv_create_rejects_bad_configs(kw, msg):
    """kv_create validates its kv_config before touching the device (include/kv.h conventions: KV_EINVAL
    and the reason in kv_last_error()), so these run without a GPU."""
    from knightvision_amd import _lib
    L = _lib.lib()
    h = C.c_void_p()
    cfg = _cfg(**kw)
    assert L.kv_create(C.byref(cfg), C.byref(h)) == -1  # KV_EINVAL
    assert msg in L.kv_last_error().decode()
    assert not h.value


def test_null_engine_arguments_are_einval():
    """Every engine entry point refuses a NULL engine / output pointer with KV_EINVAL (no device call)."""
    from knightvision_amd import _lib
    L = _lib.lib()
    n = C.c_size_t()
    assert L.kv_create(None, None) == -1 and "NULL" in L.kv_last_error().decode()
    assert L.kv_load_weights(None, None, 0) == -1
    assert L.kv_run(None, -1, -1) == -1 and "no weights" in L.kv_last_error().decode()
    assert L.kv_set_max_moves(None, 10) == -1
    assert L.kv_records(None, None, 0, C.byref(n)) == -1
    assert L.kv_records_device(None, None, 0, C.byref(n), None) == -1
    assert L.kv_games(None, None, 0, C.byref(n)) == -1
    assert L.kv_stats_get(None, None) == -1
    assert L.kv_root_visits(None, None, 0, C.byref(n)) == -1
    assert L.kv_root_visits_device(None, None, 0, C.byref(n), None) == -1
    assert L.kv_reset_records(None) == -1
    assert L.kv_sync(None) == -1
