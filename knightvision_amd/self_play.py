"""Drop-in for scripts/self_play.py: same names, signatures, module constants,
environment variables, return types and error behaviour; the games are played
by the HIP engine (libkv.so) on the GPU.

Semantics (scripts/self_play.py):
  * self_play(model, num_games, device, max_moves=None, model_path=None) :258-291
      - model instance, or model_path with SELFPLAY_SEQ=1 / SELFPLAY_WORKERS<=1:
        games in order on one numpy + one CPython stream seeded SEED (at import,
        or by _init_worker for a checkpoint), the evaluated row carried across
        games exactly as _run_single_game._last_outputs is -- the same moves as
        the reference at the same seed.
      - model_path with several workers (the reference's fork Pool :273-282,
        whose workers are all reseeded SEED and so replay identical games,
        SURVEY.md 0.7): the games run concurrently on the GPU, game g seeded
        SEED+g in both streams -- the per-game-seeded form of that path.
  * generate_self_play_data :300-311 -- decisive-record filter (>= 10 records).
  * _run_single_game(game_idx, sleep_time, max_moves=80) :111-255 -> (idx, records)
  * records: [(np.ndarray (12,8,8) float32, move_index int, reward float)]
"""
from __future__ import annotations

import logging
import os
from typing import Any, List, Tuple

import numpy as np
import torch

from .ai import codes_to_planes
from .engine import EVAL_FAITHFUL, EVAL_LAZY, SEED_PER_GAME, SEED_SEQUENTIAL, REASONS, SelfPlayEngine, packed_from, records_by_game

EPSILON = float(os.getenv("DIR_NOISE_EPS", "0.25"))
# DIR_NOISE_ALPHA (scripts/self_play.py:13): any normal double in (0, 1) -- numpy's legacy gamma branch for
# shape < 1, which the device restates bit for bit down to subnormal and zero draws (glibc pow's underflow
# special case, csrc/kv_libm.h); shape >= 1 (a different numpy branch) is rejected by kv_create (KV_EINVAL),
# and a ply whose 4096 draws are all 0 fails the run as the reference's random.choices raises ValueError
ALPHA = float(os.getenv("DIR_NOISE_ALPHA", "0.3"))
SEED = int(os.getenv("SEED", "42"))
BATCH_SIZE = int(os.getenv("SELFPLAY_BATCH_SIZE", "16"))
logging.basicConfig(level=getattr(logging, os.getenv("LOG_LEVEL", "INFO").upper(), logging.INFO))
logger = logging.getLogger(__name__)

device = torch.device("cuda" if torch.cuda.is_available() else "cpu")
_shared_model = None


class _Stream:
    """The process-wide sequential state the reference keeps in the `random`
    and `np.random` globals plus _run_single_game._last_outputs: one
    sequential-seed engine whose device streams persist across calls."""

    def __init__(self, seed: int):
        self.seed = seed
        self.engine = None
        self.weights_key = None
        self.games_done = 0

    def reseed(self, seed: int):
        self.close()
        self.seed = seed

    def close(self):
        if self.engine is not None:
            self.engine.close()
        self.engine = None
        self.weights_key = None
        self.games_done = 0

    def ensure(self, model, dev_index: int):
        key = (id(model), dev_index, tuple(t._version for t in _model_state(model).values()))
        if self.engine is None:
            self.engine = SelfPlayEngine(packed_from(model), slots=1, n_games=1 << 40, seed=self.seed,
                                         seed_mode=SEED_SEQUENTIAL, batch=BATCH_SIZE, eps=EPSILON, alpha=ALPHA,
                                         eval_mode=EVAL_LAZY, record_cap=1 << 20, recycle=True, device=dev_index)
        elif key != self.weights_key:
            # new weights, same streams (the reference keeps its RNG state too)
            from . import _lib
            import ctypes as C
            p = packed_from(model)
            _lib.check(_lib.lib().kv_load_weights(self.engine.h, p.ctypes.data_as(C.POINTER(C.c_float)), p.size),
                       "kv_load_weights")
        self.weights_key = key
        return self.engine


def _model_state(model):
    m = model.module if hasattr(model, "module") else model
    return m.state_dict()


_stream = _Stream(SEED)


def _device_index(dev) -> int:
    if not torch.cuda.is_available():
        raise RuntimeError("knightvision_amd self-play runs on the GPU (HIP); no CUDA/ROCm device is visible")
    if isinstance(dev, torch.device) and dev.type == "cuda" and dev.index is not None:
        return dev.index
    return torch.cuda.current_device()


def _init_worker(model_path, device_str, seed):
    """Load a checkpoint (dict with 'model_state_dict' or a raw state_dict) and
    reseed the streams (self_play.py:52-85)."""
    global _shared_model, device
    from .model import ChessNet
    device = torch.device(device_str)
    if not os.path.exists(model_path):
        raise FileNotFoundError(f"❌ Specified model checkpoint not found: {model_path}")
    m = ChessNet()
    checkpoint = torch.load(model_path, map_location="cpu", weights_only=True)
    if "model_state_dict" in checkpoint:
        m.load_state_dict(checkpoint["model_state_dict"])
    else:
        m.load_state_dict(checkpoint)
    m.eval()
    _shared_model = m
    _stream.reseed(seed)


def _to_records(recs, games):
    out = []
    by = records_by_game(recs, games)
    for gid in sorted(by):
        moves, boards, reward = by[gid]
        planes = codes_to_planes(boards)
        out.append([(planes[i], int(moves[i]), float(reward)) for i in range(len(moves))])
    return out


def _run_single_game(game_idx, sleep_time, max_moves=80):
    """Play the next game of the process-wide sequential stream."""
    model = _shared_model
    if model is None:
        raise ValueError("no model: call self_play(...) or _init_worker(...) first")
    logger.info("🕹️ Starting game %s", game_idx + 1)
    eng = _stream.ensure(model, _device_index(device))
    eng.set_max_moves(max_moves)
    eng.reset_records()
    target = _stream.games_done + 1
    eng.run(-1, target)
    _stream.games_done = target
    games = eng.games()
    g = games[-1]
    recs = eng.records()
    recs = recs[recs["game_id"] == g["game_id"]]
    if len(recs) != int(g["plies"]):
        raise RuntimeError(f"engine returned {len(recs)} records for a {int(g['plies'])}-ply game")
    planes = codes_to_planes(recs["board"])
    reward = float(g["reward"])
    logger.info("✅ Game %s complete. Moves played: %s | Outcome: %s (%s)", game_idx + 1, int(g["plies"]),
                int(g["outcome"]), REASONS.get(int(g["reason"]), "?"))
    return game_idx, [(planes[i], int(recs["move"][i]), reward) for i in range(len(recs))]


def self_play(model, num_games, device, max_moves=None, model_path=None):
    global _shared_model
    if model is None and model_path is None:
        raise ValueError("Either a model instance or model_path must be provided.")
    logger.info("Starting self-play with %s games...", num_games)
    data = []
    SEQUENTIAL = os.getenv("SELFPLAY_SEQ", "0") == "1"
    WORKERS = int(os.getenv("SELFPLAY_WORKERS", str(min(num_games, os.cpu_count() or 1))))
    if model_path is not None:
        _init_worker(model_path, device.type, SEED)
        if SEQUENTIAL or WORKERS <= 1:
            results = [_run_single_game(idx, 0.0, max_moves) for idx in range(num_games)]
        else:
            results = list(enumerate(play_batched(_shared_model, num_games, max_moves=max_moves)))
    else:
        _shared_model = model
        results = [_run_single_game(idx, 0.0, max_moves) for idx in range(num_games)]
    for idx, game_data in results:
        data.extend(game_data)
    logger.info("✅ Completed all self-play games: %s/%s", num_games, num_games)
    return data


def batched_eval_mode() -> int:
    """Network schedule of the many-slot paths (play_batched, learn.selfplay_shard): KV_SELFPLAY_EVAL=faithful
    (default: every board evaluated, as the reference does) or lazy (only the rows the schedule consumes, one
    compact batch per ply-step: identical games, ~1/16 of the network work)."""
    mode = os.getenv("KV_SELFPLAY_EVAL", "faithful")
    if mode not in ("faithful", "lazy"):
        raise ValueError(f"KV_SELFPLAY_EVAL must be 'faithful' or 'lazy', got {mode!r}")
    return EVAL_LAZY if mode == "lazy" else EVAL_FAITHFUL


def play_batched(model, num_games, max_moves=None, slots=None, seed=None, device_index=None):
    """num_games concurrent-slot games on one GPU, game g seeded SEED+g."""
    slots = slots or min(int(os.getenv("KV_SELFPLAY_SLOTS", "256")), max(1, num_games))
    with SelfPlayEngine(packed_from(model), slots=slots, n_games=num_games, seed=SEED if seed is None else seed,
                        seed_mode=SEED_PER_GAME, max_moves=max_moves, batch=BATCH_SIZE, eps=EPSILON, alpha=ALPHA,
                        eval_mode=batched_eval_mode(),
                        device=_device_index(device) if device_index is None else device_index) as eng:
        eng.run()
        return _to_records(eng.records(), eng.games())


def piece_value(piece):
    values = {"P": 1, "N": 3, "B": 3, "R": 5, "Q": 9, "K": 0}
    return values.get(piece.upper(), 0)


def generate_self_play_data(model, num_games: int, device: torch.device, max_moves: int = None
                            ) -> List[Tuple[Any, int, float]]:
    data = self_play(model, num_games, device, max_moves)
    decisive_data = [record for record in data if record[2] == 1.0 or record[2] == -1.0]
    MIN_DECISIVE_GAMES = 10
    if len(decisive_data) < MIN_DECISIVE_GAMES:
        print(f"⚠️ Only {len(decisive_data)} decisive games generated; consider generating more or adjusting parameters.")
    else:
        print(f"✅ Using {len(decisive_data)} decisive self-play games for training.")
        data = decisive_data
    return data
