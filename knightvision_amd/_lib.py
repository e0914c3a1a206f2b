"""ctypes binding of libkv.so (include/kv.h). The product has no CPU fallback:
if the HIP library is missing or fails to load, every entry point raises."""
from __future__ import annotations

import ctypes as C
import os

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("KV_LIB_PATH") or os.path.join(HERE, "libkv.so")  # override: A/B of two builds

_lib = None


class KVError(RuntimeError):
    pass


class Config(C.Structure):
    _fields_ = [("device", C.c_int), ("slots", C.c_int), ("n_games", C.c_int64), ("game_id_base", C.c_int64),
                ("game_id_stride", C.c_int64), ("seed", C.c_uint64), ("seed_mode", C.c_int),
                ("max_moves", C.c_int), ("batch", C.c_int), ("eps", C.c_double), ("alpha", C.c_double),
                ("sims", C.c_int), ("c_puct", C.c_float), ("eval_mode", C.c_int), ("record_cap", C.c_int64),
                ("recycle", C.c_int), ("precision", C.c_int), ("algo", C.c_int), ("tree_edge_cap", C.c_int),
                ("keep_root_visits", C.c_int)]


class Record(C.Structure):
    _fields_ = [("game_id", C.c_int64), ("ply", C.c_int32), ("move", C.c_uint16), ("pad", C.c_uint16),
                ("board", C.c_int8 * 64)]


class Game(C.Structure):
    _fields_ = [("game_id", C.c_int64), ("plies", C.c_int32), ("outcome", C.c_int32), ("reward", C.c_float),
                ("reason", C.c_int32), ("n_evals", C.c_int32), ("pad", C.c_int32)]


class Stats(C.Structure):
    _fields_ = [("steps", C.c_int64), ("plies", C.c_int64), ("games_done", C.c_int64), ("nn_rows", C.c_int64),
                ("sims", C.c_int64), ("records", C.c_int64), ("res_conv_ms", C.c_double),
                ("res_conv_launches", C.c_int64), ("step_ms", C.c_double), ("dom_flop", C.c_double),
                ("dom_algo", C.c_int64), ("tree_overflows", C.c_int64), ("nn_rows_lazy", C.c_int64),
                ("dom_path", C.c_int64), ("dom_split", C.c_int64), ("dom_kernel", C.c_char * 96)]


NPATH = 10  # KV_NPATH
PATHS = {0: "direct", 1: "winograd48 (retired)", 2: "winograd88", 3: "winograd88_f64", 4: "winograd48_f16x3 (retired)",
         5: "winograd88_i8", 6: "winograd88_i8f32", 7: "winograd88_i8f32v",
         8: "winograd88_i8r", 9: "winograd88_i8f32r3"}  # KV_PATH_*


class Calib(C.Structure):
    _fields_ = [("calibrated", C.c_int), ("path_large", C.c_int), ("path_small", C.c_int), ("n_boards", C.c_int),
                ("tol_logit", C.c_double), ("tol_value", C.c_double), ("err_logit", C.c_double * NPATH),
                ("err_value", C.c_double * NPATH), ("err_small_logit", C.c_double),
                ("err_small_value", C.c_double), ("ms", C.c_double)]


def calib_dict(c: "Calib") -> dict:
    """kv_calib as a plain dict (path names, candidate errors; -1 = candidate not run)."""
    return {"calibrated": bool(c.calibrated), "path_large": PATHS[c.path_large], "path_small": PATHS[c.path_small],
            "n_boards": c.n_boards, "tol_logit": c.tol_logit, "tol_value": c.tol_value,
            "err_logit": {PATHS[p]: c.err_logit[p] for p in range(NPATH) if c.err_logit[p] >= 0},
            "err_value": {PATHS[p]: c.err_value[p] for p in range(NPATH) if c.err_value[p] >= 0},
            "err_small_logit": c.err_small_logit, "err_small_value": c.err_small_value, "ms": c.ms}


class PgnRecord(C.Structure):
    _fields_ = [("fen", C.c_char * 100), ("san", C.c_char * 12), ("outcome", C.c_int32), ("game", C.c_int32)]


PGN_OUTCOME_NONE = -128
MAXM = 320  # KV_MAXM, move-list capacity per position

assert C.sizeof(Record) == 80 and C.sizeof(Game) == 32 and C.sizeof(PgnRecord) == 120


def _declare(L):
    vp, i, i64, sz = C.c_void_p, C.c_int, C.c_int64, C.c_size_t
    P = C.POINTER
    sig = {
        "kv_last_error": ([], C.c_char_p),
        "kv_version": ([], i),
        "kv_net_packed_size": ([], sz),
        "kv_net_create": ([i, P(vp)], i),
        "kv_net_load": ([vp, P(C.c_float), sz], i),
        "kv_net_forward": ([vp, vp, i, vp, vp, vp], i),
        "kv_net_forward_boards": ([vp, vp, i, vp, vp, vp], i),
        "kv_net_forward_boards_legal": ([vp, vp, i, vp, vp, i, vp, vp, vp], i),
        "kv_net_set_timing": ([vp, i], i),
        "kv_net_last_timing": ([vp, P(C.c_float), P(i)], i),
        "kv_net_destroy": ([vp], None),
        "kv_net_set_precision": ([vp, i], i),
        "kv_net_set_algo": ([vp, i], i),
        "kv_net_calibration": ([vp, P(Calib)], i),
        "kv_engine_calibration": ([vp, P(Calib)], i),
        "kv_create": ([P(Config), P(vp)], i),
        "kv_load_weights": ([vp, P(C.c_float), sz], i),
        "kv_run": ([vp, i64, i64], i),
        "kv_set_max_moves": ([vp, i], i),
        "kv_records": ([vp, P(Record), sz, P(sz)], i),
        "kv_games": ([vp, P(Game), sz, P(sz)], i),
        "kv_stats_get": ([vp, P(Stats)], i),
        "kv_root_visits": ([vp, P(C.c_int32), sz, P(sz)], i),
        "kv_root_visits_device": ([vp, vp, sz, P(sz), vp], i),
        "kv_records_device": ([vp, vp, sz, P(sz), vp], i),
        "kv_sync": ([vp], i),
        "kv_reset_records": ([vp], i),
        "kv_destroy": ([vp], None),
        "kv_dev_valid_moves": ([i, P(C.c_int8), i, P(C.c_uint16), i, P(i), P(C.c_int8), P(C.c_uint8)], i),
        "kv_dev_make_move": ([i, P(C.c_int8), P(i), i], i),
        "kv_dev_attacks": ([i, P(C.c_int8), i, P(C.c_uint64)], i),
        "kv_dev_dirichlet": ([i, P(C.c_uint64), i, C.c_double, i, i, P(C.c_double), P(i64), P(C.c_double)], i),
        "kv_dev_py_random": ([i, P(C.c_uint64), i, i, P(C.c_double)], i),
        "kv_host_libm": ([i, P(C.c_double), P(C.c_double), i, P(C.c_double)], i),
        "kv_dev_wino88i": ([i, P(C.c_double), i, P(C.c_double), i, i, i, P(C.c_double), P(C.c_int8), P(i)], i),
        "kv_dev_i8gemm_bench": ([i, i, i, i, i, P(C.c_float), P(C.c_float)], i),
        "kv_dev_gemm_clock": ([i, i, i, C.c_double, P(C.c_double)], i),
        "kv_dev_out_phases": ([i, i, i, i, P(C.c_uint64), P(C.c_float)], i),
        "kv_dev_wino88i32_out": ([i, P(C.c_float), i, P(C.c_float), P(C.c_float), P(C.c_float), i, P(C.c_float),
                                  P(C.c_int8), P(i)], i),
        "kv_dev_wino88r_out": ([i, P(C.c_double), i, P(C.c_float), P(C.c_float), P(C.c_float), i, P(C.c_float),
                                P(C.c_int8), P(i)], i),
        "kv_pgn_extract": ([C.c_char_p, sz, P(PgnRecord), sz, P(sz), P(sz), P(i64)], i),
        "kv_fen_codes": ([C.c_char_p, sz, i, P(C.c_int8)], i),
        "kv_san_move_index": ([C.c_char_p, sz, C.c_char_p, sz, i, P(C.c_int32)], i),
        "kv_chess_perft": ([C.c_char_p, i, P(C.c_uint64)], i),
        "kv_chess_san": ([C.c_char_p, C.c_char_p, C.c_char_p, sz, C.c_char_p, sz], i),
        "kv_chess_fen": ([C.c_char_p, C.c_char_p, sz], i),
        "kv_tr_conv3x3_f16": ([vp, i, i, vp, vp, i, vp, vp], i),
        "kv_tr_conv3x3_add_f16": ([vp, i, i, vp, vp, i, vp, vp, vp], i),
        "kv_tr_conv_weights_f16": ([vp, i, i, i, vp, vp, vp], i),
        "kv_tr_wgrad_workspace": ([i, i, i, P(i)], sz),
        "kv_tr_conv3x3_wgrad_f16": ([vp, vp, i, i, i, i, vp, vp, sz, vp], i),
        "kv_tr_bn_workspace": ([i, i], sz),
        "kv_tr_bn_stats_f16": ([vp, i, i, C.c_float, vp, vp, vp, vp, sz, vp], i),
        "kv_tr_bn_apply_f16": ([vp, i, i, vp, vp, vp, vp, vp, i, vp, vp], i),
        "kv_tr_bn_backward_f16": ([vp, vp, vp, i, i, i, vp, vp, vp, vp, vp, vp, vp, vp, vp, sz, vp], i),
        "kv_tr_channel_sum_f16": ([vp, i, i, vp, vp, sz, vp], i),
        "kv_tr_planes_to_nhwc": ([vp, i, i, vp, vp], i),
        "kv_tr_head1x1_f16": ([vp, i, vp, vp, vp, vp], i),
        "kv_tr_head1x1_workspace": ([i], sz),
        "kv_tr_head1x1_backward_f16": ([vp, vp, i, vp, vp, vp, vp, vp, sz, vp], i),
    }
    for name, (args, res) in sig.items():
        if not hasattr(L, name):
            continue
        f = getattr(L, name)
        f.argtypes = args
        f.restype = res
    return L


EXPORTED = ["kv_last_error", "kv_version", "kv_net_packed_size", "kv_net_create", "kv_net_load", "kv_net_forward",
            "kv_net_forward_boards", "kv_net_forward_boards_legal", "kv_net_set_timing", "kv_net_last_timing", "kv_net_destroy", "kv_net_set_precision", "kv_net_set_algo",
            "kv_net_calibration", "kv_engine_calibration",
            "kv_create",
            "kv_load_weights", "kv_run", "kv_set_max_moves", "kv_records", "kv_games", "kv_stats_get", "kv_root_visits", "kv_root_visits_device", "kv_records_device", "kv_sync", "kv_reset_records", "kv_destroy",
            "kv_dev_valid_moves", "kv_dev_make_move", "kv_dev_attacks", "kv_dev_dirichlet", "kv_dev_py_random", "kv_host_libm",
            "kv_dev_wino88i", "kv_dev_wino88i32_out", "kv_dev_wino88r_out", "kv_dev_i8gemm_bench",
            "kv_dev_gemm_clock", "kv_dev_out_phases",
            "kv_pgn_extract", "kv_fen_codes", "kv_san_move_index", "kv_chess_perft", "kv_chess_san", "kv_chess_fen",
            "kv_tr_conv3x3_f16", "kv_tr_conv3x3_add_f16", "kv_tr_conv_weights_f16", "kv_tr_wgrad_workspace", "kv_tr_conv3x3_wgrad_f16",
            "kv_tr_bn_workspace", "kv_tr_bn_stats_f16", "kv_tr_bn_apply_f16", "kv_tr_bn_backward_f16",
            "kv_tr_channel_sum_f16", "kv_tr_planes_to_nhwc", "kv_tr_head1x1_f16", "kv_tr_head1x1_workspace",
            "kv_tr_head1x1_backward_f16"]


def lib():
    """Load libkv.so (build it first if this is a source tree with hipcc)."""
    global _lib
    if _lib is None:
        import torch  # noqa: F401  -- load torch's HIP runtime first so both share one
        if not os.path.exists(LIB_PATH):
            raise KVError(f"{LIB_PATH} is missing: run `python -c 'import __graft_entry__ as g; g.build()'` "
                          "(the HIP library is required; there is no CPU fallback)")
        _lib = _declare(C.CDLL(LIB_PATH))
    return _lib


def check(rc: int, what: str = ""):
    if rc != 0:
        msg = lib().kv_last_error().decode(errors="replace")
        raise KVError(f"{what} failed ({rc}): {msg}")
