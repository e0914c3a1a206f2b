"""Edge cases of the engine boundary on the GPU: empty and ragged runs (no
games, more slots than games), the smallest game caps against the oracle's
_run_single_game (self_play.py:111-255), and the loud failures of
include/kv.h (record buffer full, caller buffers too small, pi without
keep_root_visits) -- never a silent truncation."""
import ctypes as C

import numpy as np
import pytest

from knightvision_amd import _lib
from knightvision_amd.engine import SelfPlayEngine, records_by_game
from knightvision_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def sd():
    return synthetic_state_dict(42, "init")


def test_no_games_is_an_empty_run(sd):
    with SelfPlayEngine(sd, slots=4, n_games=0, seed=42, max_moves=8) as eng:
        eng.run()
        assert len(eng.records()) == 0 and len(eng.games()) == 0
        st = eng.stats()
        assert st["plies"] == 0 and st["games_done"] == 0


def test_more_slots_than_games_plays_the_same_games(sd):
    """Idle slots change nothing: 3 games on 8 slots equal the same 3 games on 3 slots."""
    out = []
    for slots in (3, 8):
        with SelfPlayEngine(sd, slots=slots, n_games=3, seed=42, max_moves=20) as eng:
            eng.run()
            out.append((eng.records(), eng.games()))
    (r3, g3), (r8, g8) = out
    assert len(g3) == len(g8) == 3
    assert np.array_equal(r3, r8) and np.array_equal(g3, g8)


@pytest.mark.parametrize("max_moves", [1, 2, 17])
def test_short_caps_equal_the_oracle(sd, max_moves):
    """max_moves 1 / 2 (the buffer never reaches 16 rows: every row comes from the first-ply
    evaluation and the end-of-game flush) and 17 (one full batch of 16 plus one) against the
    oracle's restatement of _run_single_game."""
    from oracle import oracle as O
    from oracle import torch_ref
    n = 3
    with SelfPlayEngine(sd, slots=n, n_games=n, seed=42, max_moves=max_moves, batch=16) as eng:
        eng.run()
        by = records_by_game(eng.records(), eng.games())
    ev = torch_ref.make_eval_fn(sd)
    for g in range(n):
        ref = O.play_game(ev, O.MT(42 + g, "numpy"), O.MT(42 + g, "python"), O.Last(), max_moves=max_moves,
                          batch=16, softmax_fn=torch_ref.torch_softmax)
        moves, _, reward = by[g]
        assert len(moves) == len(ref["moves"]) <= max_moves
        assert np.array_equal(moves, ref["moves"]), f"game {g}"
        assert abs(reward - ref["reward"]) < 1e-6


def test_record_buffer_full_is_an_error(sd):
    with SelfPlayEngine(sd, slots=4, n_games=4, seed=42, max_moves=40, record_cap=20) as eng:
        with pytest.raises(_lib.KVError, match="record buffer full"):
            eng.run()


def test_caller_buffers_are_checked(sd):
    L = _lib.lib()
    with SelfPlayEngine(sd, slots=2, n_games=2, seed=42, max_moves=6) as eng:
        eng.run()
        n = C.c_size_t()
        one = (_lib.Record * 1)()
        assert L.kv_records(eng.h, one, 1, C.byref(n)) == -1
        assert "buffer holds 1" in L.kv_last_error().decode()
        games = (_lib.Game * 1)()
        assert L.kv_games(eng.h, games, 1, C.byref(n)) == -1
        pi = (C.c_int32 * 16)()
        assert L.kv_root_visits(eng.h, pi, 16, C.byref(n)) == -1
        assert "keep_root_visits" in L.kv_last_error().decode()
        assert len(eng.records()) == 12  # the engine is intact after the refused calls


def test_default_record_cap_holds_capped_games(sd):
    """The default buffer holds every ply of max_moves-capped games (at least n_games x max_moves
    records), so a capped run never reports "record buffer full"."""
    with SelfPlayEngine(sd, slots=64, n_games=64, seed=7, max_moves=64) as eng:
        assert eng.cfg.record_cap >= 64 * 64
        eng.run()
        recs, games = eng.records(), eng.games()
    assert len(games) == 64 and len(recs) == int(games["plies"].sum())
