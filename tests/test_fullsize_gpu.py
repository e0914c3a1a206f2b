"""Parity at BASELINE.json's full sizes through size-independent properties
(the oracle cannot play 2,048 searched games in seconds):

  * slot-count invariance: with per-game seeds a game's trajectory depends only
    on its seed and on the network rows of its own boards, and the Winograd
    towers (F(8x8), the fp32 default, F(4x8) and F(4x4)) are batch-invariant bit for
    bit (tests/test_nn_gpu.py), so the first
    16 games of a 256- or 2,048-slot run must equal a 16-slot run move for move;
  * every recorded game replays legally on the oracle rules from the start
    position, record boards equal the replayed boards, and the recorded end
    reason agrees with the final position (mate / stalemate / draw);
  * work accounting: completed backups = slots x plies x sims.
Configs: C3 (2,048 games x 800 sims, one move), C2 (256 x 400, three moves),
C2-ref (256 games, reference move selection, complete games)."""
import numpy as np
import pytest

from knightvision_amd.engine import SelfPlayEngine, records_by_game
from knightvision_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

SD = synthetic_state_dict(42, "init")


def _run(slots, n_games, sims, max_moves, steps=-1, algo="winograd88"):
    with SelfPlayEngine(SD, slots=slots, n_games=n_games, seed=42, max_moves=max_moves, batch=16, sims=sims,
                        algo=algo) as eng:
        eng.run(steps)
        return eng.records(), eng.games(), eng.stats()


def _replay(moves, boards, game):
    """Replay one game on the oracle rules; returns the final state."""
    from oracle import oracle as O
    st = O.initial_state()
    for p, mv in enumerate(moves):
        lst, after = O.valid_moves(st)
        assert np.array_equal(boards[p], st[:64]) or np.array_equal(boards[p], after[:64]), f"ply {p}: board"
        idx = [k for k in range(len(lst)) if int(lst[k, 0]) * 64 + int(lst[k, 1]) == int(mv)]
        assert idx, f"ply {p}: move {mv} is not legal"
        st = O.make_valid_move(after, idx[0])
    return st


def _check_end(st, game):
    from oracle import oracle as O
    lst, _ = O.valid_moves(st)
    reason = int(game["reason"])
    if reason == 2:    # Checkmate
        assert len(lst) == 0 and O.in_check(st)
    elif reason == 3:  # Stalemate
        assert len(lst) == 0 and not O.in_check(st)
    elif reason == 4:  # isDraw: kings only
        assert O.is_draw(st)
    assert float(game["reward"]) == pytest.approx({1: 1.0, 0: 0.2, -1: -1.0}[int(game["outcome"])])


def _same_first_games(big, small, n):
    bb = records_by_game(big[0], big[1])
    sb = records_by_game(small[0], small[1])
    for g in range(n):
        assert np.array_equal(bb[g][0], sb[g][0]), f"game {g} differs between slot counts"
        assert np.array_equal(bb[g][1], sb[g][1])


def test_c3_2048x800_one_move():
    big = _run(2048, 2048, 800, 1)
    st = big[2]
    assert st["sims"] == 2048 * 800 and st["plies"] == 2048 and len(big[1]) == 2048
    small = _run(16, 16, 800, 1)
    _same_first_games(big, small, 16)
    by = records_by_game(big[0], big[1])
    assert len(by) == 2048
    for g in range(0, 2048, 97):
        _replay(by[g][0], by[g][1], None)


@pytest.mark.parametrize("algo", ["winograd88i8r3", "winograd88"])
def test_c2_256x400_three_moves(algo):
    big = _run(256, 256, 400, 3, algo=algo)
    assert big[2]["sims"] == 256 * 3 * 400 and len(big[1]) == 256
    small = _run(16, 16, 400, 3, algo=algo)
    _same_first_games(big, small, 16)
    by = records_by_game(big[0], big[1])
    for g in range(256):
        _replay(by[g][0], by[g][1], None)


def test_c2_ref_256_complete_games():
    big = _run(256, 256, 0, None)
    games = big[1]
    assert len(games) == 256 and big[2]["plies"] == int(games["plies"].sum())
    small = _run(16, 16, 0, None)
    _same_first_games(big, small, 16)
    by = records_by_game(big[0], games)
    gi = {int(g["game_id"]): g for g in games}
    for gid in range(256):
        st = _replay(by[gid][0], by[gid][1], gi[gid])
        _check_end(st, gi[gid])
