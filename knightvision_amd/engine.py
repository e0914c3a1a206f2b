"""Python owner of one kv_engine (include/kv.h): the batched self-play engine
on one GPU. self_play.py builds the reference's API on top of this class."""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .weights import pack_weights, state_dict_to_numpy

SEED_PER_GAME, SEED_SEQUENTIAL = 0, 1
EVAL_FAITHFUL, EVAL_LAZY, EVAL_HASH = 0, 1, 2

RECORD_DTYPE = np.dtype([("game_id", "<i8"), ("ply", "<i4"), ("move", "<u2"), ("pad", "<u2"),
                         ("board", "i1", (64,))])
GAME_DTYPE = np.dtype([("game_id", "<i8"), ("plies", "<i4"), ("outcome", "<i4"), ("reward", "<f4"),
                       ("reason", "<i4"), ("n_evals", "<i4"), ("pad", "<i4")])
assert RECORD_DTYPE.itemsize == C.sizeof(_lib.Record) and GAME_DTYPE.itemsize == C.sizeof(_lib.Game)

REASONS = {0: "max_moves", 1: "Resignation", 2: "Checkmate", 3: "Stalemate", 4: "Draw", 5: "Material"}


def packed_from(weights) -> np.ndarray:
    """ChessNet module / state_dict / checkpoint dict / packed array -> packed fp32 blob."""
    if isinstance(weights, np.ndarray) and weights.ndim == 1:
        return np.ascontiguousarray(weights, dtype=np.float32)
    if hasattr(weights, "state_dict") and callable(weights.state_dict):
        m = weights.module if hasattr(weights, "module") else weights  # nn.DataParallel
        weights = m.state_dict()
    return pack_weights(state_dict_to_numpy(weights))[0]


from .model import ALGOS, PRECISIONS  # noqa: E402


class SelfPlayEngine:
    def __init__(self, weights, *, slots=256, n_games=256, seed=42, seed_mode=SEED_PER_GAME, max_moves=None,
                 batch=16, eps=0.25, alpha=0.3, sims=0, c_puct=1.5, eval_mode=EVAL_FAITHFUL, record_cap=None,
                 recycle=True, device=0, game_id_base=0, game_id_stride=1, precision="fp32",
                 algo="auto", tree_edge_cap=0, keep_root_visits=False):
        L = _lib.lib()
        if record_cap is None:
            # one record per committed ply: a capped game holds at most max_moves; an uncapped one
            # (the reference default) is given 1,024 plies (its random-init games run 116-660). A
            # run that still fills the buffer fails with KV_EOVERFLOW ("record buffer full").
            per_game = int(max_moves) if max_moves else 1024
            record_cap = max(1 << 16, min(1 << (22 if keep_root_visits else 27), int(n_games) * per_game))
        cfg = _lib.Config(device=device, slots=slots, n_games=n_games, game_id_base=game_id_base,
                          game_id_stride=game_id_stride, seed=seed, seed_mode=seed_mode,
                          max_moves=max_moves if max_moves else 0, batch=batch, eps=eps, alpha=alpha, sims=sims,
                          c_puct=c_puct, eval_mode=eval_mode, record_cap=record_cap, recycle=1 if recycle else 0,
                          precision=PRECISIONS[precision], algo=ALGOS[algo],
                          tree_edge_cap=int(tree_edge_cap), keep_root_visits=1 if keep_root_visits else 0)
        h = C.c_void_p()
        _lib.check(L.kv_create(C.byref(cfg), C.byref(h)), "kv_create")
        self.h = h
        self.cfg = cfg
        packed = packed_from(weights)
        _lib.check(L.kv_load_weights(self.h, packed.ctypes.data_as(C.POINTER(C.c_float)), packed.size),
                   "kv_load_weights")

    def run(self, max_steps: int = -1, stop_after_games: int = -1):
        _lib.check(_lib.lib().kv_run(self.h, int(max_steps), int(stop_after_games)), "kv_run")

    def set_max_moves(self, max_moves):
        _lib.check(_lib.lib().kv_set_max_moves(self.h, max_moves if max_moves else 0), "kv_set_max_moves")

    def reset_records(self):
        _lib.check(_lib.lib().kv_reset_records(self.h), "kv_reset_records")

    def sync(self):
        _lib.check(_lib.lib().kv_sync(self.h), "kv_sync")

    def records(self) -> np.ndarray:
        """All records so far, ordered by (game_id, ply)."""
        L = _lib.lib()
        n = C.c_size_t()
        _lib.check(L.kv_records(self.h, None, 0, C.byref(n)), "kv_records")
        out = np.zeros(n.value, dtype=RECORD_DTYPE)
        if n.value:
            _lib.check(L.kv_records(self.h, out.ctypes.data_as(C.POINTER(_lib.Record)), n.value, C.byref(n)),
                       "kv_records")
        return out

    def records_device(self):
        """The records as a uint8 CUDA tensor [n, 80] on the engine's GPU, in allocation order
        (kv_records_device: no host round trip; sort after gathering)."""
        import torch
        L = _lib.lib()
        n = C.c_size_t()
        _lib.check(L.kv_records_device(self.h, None, 0, C.byref(n), None), "kv_records_device")
        dev = torch.device("cuda", self.cfg.device)
        out = torch.empty((n.value, RECORD_DTYPE.itemsize), dtype=torch.uint8, device=dev)
        if n.value:
            st = torch.cuda.current_stream(dev).cuda_stream
            _lib.check(L.kv_records_device(self.h, C.c_void_p(out.data_ptr()), n.value, C.byref(n), C.c_void_p(st)),
                       "kv_records_device")
        return out

    def root_visits_device(self):
        """The MCTS root visit counts (pi) as a uint8 CUDA tensor [n, MAXM * 2] (uint16 counts, 0xffff padded),
        row k belonging to row k of records_device() (needs keep_root_visits=True)."""
        import torch
        L = _lib.lib()
        n = C.c_size_t()
        _lib.check(L.kv_root_visits_device(self.h, None, 0, C.byref(n), None), "kv_root_visits_device")
        dev = torch.device("cuda", self.cfg.device)
        out = torch.empty((n.value, _lib.MAXM * 2), dtype=torch.uint8, device=dev)
        if n.value:
            st = torch.cuda.current_stream(dev).cuda_stream
            _lib.check(L.kv_root_visits_device(self.h, C.c_void_p(out.data_ptr()), n.value, C.byref(n),
                                               C.c_void_p(st)), "kv_root_visits_device")
        return out

    def root_visits(self) -> np.ndarray:
        """MCTS root visit counts [records, MAXM] (-1 padded), rows in records() order
        (needs keep_root_visits=True)."""
        L = _lib.lib()
        n = C.c_size_t()
        _lib.check(L.kv_root_visits(self.h, None, 0, C.byref(n)), "kv_root_visits")
        out = np.zeros((n.value, _lib.MAXM), dtype=np.int32)
        if n.value:
            _lib.check(L.kv_root_visits(self.h, out.ctypes.data_as(C.POINTER(C.c_int32)), n.value, C.byref(n)),
                       "kv_root_visits")
        return out

    def games(self) -> np.ndarray:
        L = _lib.lib()
        n = C.c_size_t()
        _lib.check(L.kv_games(self.h, None, 0, C.byref(n)), "kv_games")
        out = np.zeros(n.value, dtype=GAME_DTYPE)
        if n.value:
            _lib.check(L.kv_games(self.h, out.ctypes.data_as(C.POINTER(_lib.Game)), n.value, C.byref(n)),
                       "kv_games")
        return out

    def calibration(self) -> dict:
        """The network's conv paths and load-time calibration (kv_engine_calibration)."""
        c = _lib.Calib()
        _lib.check(_lib.lib().kv_engine_calibration(self.h, C.byref(c)), "kv_engine_calibration")
        return _lib.calib_dict(c)

    def stats(self) -> dict:
        st = _lib.Stats()
        _lib.check(_lib.lib().kv_stats_get(self.h, C.byref(st)), "kv_stats_get")
        out = {k: getattr(st, k) for k, _ in _lib.Stats._fields_}
        out["dom_kernel"] = out["dom_kernel"].decode()
        return out

    def close(self):
        if getattr(self, "h", None):
            _lib.lib().kv_destroy(self.h)
            self.h = None

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


def records_by_game(recs: np.ndarray, games: np.ndarray):
    """-> {game_id: (moves uint16[plies], boards int8[plies,64], reward)}."""
    out = {}
    if len(recs) == 0:
        return out
    ids = recs["game_id"]
    cuts = np.flatnonzero(np.diff(ids)) + 1
    starts = np.concatenate([[0], cuts])
    ends = np.concatenate([cuts, [len(recs)]])
    reward = {int(g["game_id"]): float(g["reward"]) for g in games}
    for s, e in zip(starts, ends):
        gid = int(ids[s])
        out[gid] = (recs["move"][s:e].copy(), recs["board"][s:e].copy(), reward.get(gid))
    return out
