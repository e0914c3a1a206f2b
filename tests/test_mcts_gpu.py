"""PUCT search on the GPU (kv_mcts.hip) vs its CPU restatement
(oracle kvo_mcts_play_game), through the C ABI.

* Hash test evaluator (uniform logits, dyadic values): every PUCT score is
  bit-reproducible on both sides, so the games must be identical move for move.
* The real ChessNet: the oracle's evaluator returns the HIP network's own rows
  for each leaf, evaluated in the > 16-board class that the engine's batch is
  in (the Winograd tower is batch-invariant bit for bit inside it,
  tests/test_nn_gpu.py). Priors use det_expf and the device's summation order
  on both sides, so root visit-count vectors and chosen moves must be
  identical; a divergence is counted as a tie and printed (expected 0).
  Anchor: the move choice this replaces, scripts/self_play.py:150-167.
* Tree pools: a forced-small edge pool raises KV_EOVERFLOW (and the oracle's
  TreeOverflow at the same configuration); the default pool never overflows."""
import numpy as np
import pytest
import torch

from knightvision_amd import _lib
from knightvision_amd.engine import EVAL_HASH, SelfPlayEngine, records_by_game, packed_from
from knightvision_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

CLASS_ROWS = 17  # smallest batch of the Winograd (> 16 boards) class


@pytest.mark.parametrize("sims,max_moves,n", [(16, 60, 6), (64, 40, 4), (200, 24, 2)])
def test_mcts_hash_games_identical_to_oracle(sims, max_moves, n):
    from oracle import oracle as O
    with SelfPlayEngine(synthetic_state_dict(42, "init"), slots=n, n_games=n, seed=42, max_moves=max_moves,
                        sims=sims, c_puct=1.5, eval_mode=EVAL_HASH) as eng:
        eng.run()
        by = records_by_game(eng.records(), eng.games())
        st = eng.stats()
    assert st["sims"] > 0
    for g in range(n):
        r = O.mcts_play_game(sims, O.MT(42 + g, "numpy"), O.MT(42 + g, "python"), None, max_moves=max_moves,
                             c_puct=1.5)
        moves, _, reward = by[g]
        assert np.array_equal(moves, r["moves"]), f"game {g}: first diff at {np.flatnonzero(moves[:len(r['moves'])] != r['moves'][:len(moves)])[:1]}"
        assert reward == pytest.approx(r["reward"])


def _hip_eval(sd, class_rows=CLASS_ROWS):
    """Oracle evaluator: the HIP network's row for one board, computed in a
    batch of class_rows copies (the engine's batch class: 17 = the > 16-board
    Winograd class, 1 = the <= 16-board direct class of a one-slot engine)."""
    from knightvision_amd.model import KVNet
    net = KVNet(0, packed_from(sd))

    def ev(planes):
        planes = np.asarray(planes, dtype=np.float32).reshape(-1, 12, 64)
        n = planes.shape[0]
        codes = np.zeros((n, 64), dtype=np.int8)
        b, c, sq = np.nonzero(planes)
        codes[b, sq] = c + 1
        rows = torch.from_numpy(np.repeat(codes, class_rows, axis=0)).cuda()
        pol, val = net.forward_boards(rows)
        torch.cuda.synchronize()
        return pol.cpu().numpy()[::class_rows], val.cpu().numpy().reshape(-1)[::class_rows]

    return ev, net


def _compare_network_games(variant, slots, n_check, sims, max_moves, steps=-1):
    from oracle import oracle as O
    sd = synthetic_state_dict(42, variant)
    assert slots >= CLASS_ROWS
    with SelfPlayEngine(sd, slots=slots, n_games=slots, seed=42, max_moves=max_moves, sims=sims, c_puct=1.5,
                        keep_root_visits=True) as eng:
        eng.run(steps)
        recs = eng.records()
        visits = eng.root_visits()
        st = eng.stats()
    assert st["tree_overflows"] == 0
    ev, net = _hip_eval(sd)
    ties = compared = 0
    for g in range(n_check):
        sel = recs["game_id"] == g
        moves, vis = recs["move"][sel], visits[sel]
        r = O.mcts_play_game(sims, O.MT(42 + g, "numpy"), O.MT(42 + g, "python"), ev,
                             max_moves=max_moves if steps < 0 else len(moves), c_puct=1.5)
        n = len(moves)
        assert len(r["moves"]) >= n
        for p in range(n):
            compared += 1
            if not (np.array_equal(vis[p], r["visits"][p]) and moves[p] == r["moves"][p]):
                ties += 1
                print(f"{variant} game {g} ply {p}: GPU visits {vis[p][vis[p] >= 0]} oracle "
                      f"{r['visits'][p][r['visits'][p] >= 0]}")
                break  # the games part here
    net.close()
    print(f"MCTS network parity ({variant}, {slots} slots x {sims} sims): {compared} root visit vectors "
          f"compared, ties/divergences: {ties}")
    assert ties == 0


@pytest.mark.parametrize("variant", ["init", "peaked"])
def test_mcts_network_visits_identical_to_oracle_c1(variant):
    """C1-sized search (64 sims/move) with the real network, 8 games x 6 plies."""
    _compare_network_games(variant, slots=20, n_check=8, sims=64, max_moves=6)


@pytest.mark.parametrize("variant", ["init", "peaked"])
def test_mcts_network_c1_single_game(variant):
    """BASELINE config C1 itself: ONE game, 64 sims/move (a one-slot engine, so every leaf batch is one board
    in the <= 16-board direct class), 10 moves, root visit vectors identical to the oracle's PUCT."""
    from oracle import oracle as O
    sd = synthetic_state_dict(42, variant)
    with SelfPlayEngine(sd, slots=1, n_games=1, seed=42, max_moves=10, sims=64, c_puct=1.5,
                        keep_root_visits=True) as eng:
        eng.run()
        recs, visits = eng.records(), eng.root_visits()
    ev, net = _hip_eval(sd, class_rows=1)
    r = O.mcts_play_game(64, O.MT(42, "numpy"), O.MT(42, "python"), ev, max_moves=10, c_puct=1.5)
    net.close()
    assert np.array_equal(recs["move"], r["moves"])
    for p in range(len(r["moves"])):
        assert np.array_equal(visits[p], r["visits"][p]), p
    print(f"C1 ({variant}): {len(r['moves'])} root visit vectors identical")


def test_mcts_network_visits_identical_to_oracle_c2_first_move():
    """C2 (256 slots x 400 sims): the first move of the first 16 games."""
    _compare_network_games("init", slots=256, n_check=16, sims=400, max_moves=None, steps=1)


def test_mcts_network_visits_identical_to_oracle_c2_peaked_three_moves():
    """C2 with the peaked weight set (priors the search follows, not near-uniform
    ones): the first three moves of the first 8 games."""
    _compare_network_games("peaked", slots=256, n_check=8, sims=400, max_moves=None, steps=3)


@pytest.mark.parametrize("variant", ["init", "peaked"])
def test_mcts_network_visits_identical_to_oracle_c3_first_move(variant):
    """C3, the headline config (2,048 slots x 800 sims): the first move of the first 8 games."""
    _compare_network_games(variant, slots=2048, n_check=8, sims=800, max_moves=None, steps=1)


@pytest.mark.parametrize("variant", ["init", "peaked", "stress"])
def test_mcts_network_visits_identical_to_oracle_c3_three_moves(variant):
    """C3, the headline config (2,048 slots x 800 sims): the first three moves of the first 8 games -- trees
    that start from positions the search itself chose. "stress" (trained-network magnitudes): the AUTO path
    there is the fp64 Winograd domain on int8 digits, and the peaked priors give the trees their own shapes."""
    _compare_network_games(variant, slots=2048, n_check=8, sims=800, max_moves=None, steps=3)


def test_mcts_network_games_run():
    """The real network path: games complete, sims are counted per backup."""
    with SelfPlayEngine(synthetic_state_dict(42, "init"), slots=8, n_games=8, seed=42, max_moves=6,
                        sims=32) as eng:
        eng.run()
        games = eng.games()
        st = eng.stats()
    assert len(games) == 8 and (games["plies"] == 6).all()
    assert st["sims"] == 8 * 6 * 32
    assert st["nn_rows"] >= 8 * 6
    assert st["tree_overflows"] == 0


def test_mcts_tree_overflow_is_an_error():
    """An edge pool smaller than the search needs fails loudly on both sides."""
    from oracle import oracle as O
    cap = _lib.MAXM + 40
    with SelfPlayEngine(synthetic_state_dict(42, "init"), slots=4, n_games=4, seed=42, max_moves=4, sims=64,
                        eval_mode=EVAL_HASH, tree_edge_cap=cap) as eng:
        with pytest.raises(_lib.KVError, match="tree pool full"):
            eng.run()
        assert eng.stats()["tree_overflows"] > 0
    with pytest.raises(O.TreeOverflow):
        O.mcts_play_game(64, O.MT(42, "numpy"), O.MT(42, "python"), None, max_moves=4, edge_cap=cap)
    with pytest.raises(_lib.KVError, match="tree_edge_cap"):
        SelfPlayEngine(synthetic_state_dict(42, "init"), slots=1, n_games=1, sims=8, tree_edge_cap=100)


def test_mcts_compact_tail_batches_identical_to_oracle():
    """Games that end at different plies (mates / draws before max_moves) leave fewer active slots than
    slots; their leaf batches then carry the active slots only (k_compact_active, padded to the > 16-board
    class). Full games of the first 4 slots -- the tails included -- equal the oracle's PUCT restatement
    root vector for root vector."""
    slots, sims, mm = 17, 16, 120  # 17: once a game ends the batch is padded (16 active + 1)
    from oracle import oracle as O
    sd = synthetic_state_dict(42, "peaked")
    with SelfPlayEngine(sd, slots=slots, n_games=slots, seed=42, max_moves=mm, sims=sims, c_puct=1.5,
                        keep_root_visits=True) as eng:
        eng.run()
        recs, visits, games = eng.records(), eng.root_visits(), eng.games()
    ends = np.sort(games["plies"])
    print("game lengths:", ends.tolist())
    assert ends[0] < ends[-1], "every game ended on the same ply: no compact tail was exercised"
    ev, net = _hip_eval(sd)
    compared = 0
    for g in range(4):
        sel = recs["game_id"] == g
        r = O.mcts_play_game(sims, O.MT(42 + g, "numpy"), O.MT(42 + g, "python"), ev, max_moves=mm, c_puct=1.5)
        assert np.array_equal(recs["move"][sel], r["moves"]), f"game {g}: moves differ"
        for p in range(len(r["moves"])):
            assert np.array_equal(visits[sel][p], r["visits"][p]), (g, p)
            compared += 1
    net.close()
    print(f"compact-tail MCTS parity: {compared} root vectors identical")


def test_mcts_recycled_slots_then_compact_tail_identical_to_oracle():
    """Slot recycling (more games than slots) followed by the compact tail once the game queue is empty:
    games 0..19 on 17 slots, each equal to the oracle's game of the same id move for move."""
    from oracle import oracle as O
    slots, n, sims, mm = 17, 20, 16, 40
    sd = synthetic_state_dict(42, "peaked")
    with SelfPlayEngine(sd, slots=slots, n_games=n, seed=42, max_moves=mm, sims=sims, c_puct=1.5) as eng:
        eng.run()
        by = records_by_game(eng.records(), eng.games())
    assert len(by) == n
    ev, net = _hip_eval(sd)
    for g in range(n):
        r = O.mcts_play_game(sims, O.MT(42 + g, "numpy"), O.MT(42 + g, "python"), ev, max_moves=mm, c_puct=1.5)
        moves, _, reward = by[g]
        assert np.array_equal(moves, r["moves"]), f"game {g}"
        assert reward == pytest.approx(r["reward"])
    net.close()
