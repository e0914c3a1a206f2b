"""PUCT search on the GPU (kv_mcts.hip) vs its CPU restatement
(oracle kvo_mcts_play_game). With the hash test evaluator (uniform logits,
dyadic values) every PUCT score is bit-reproducible on both sides, so the
games -- which depend on every visit count through random.choices -- must be
identical move for move."""
import numpy as np
import pytest

from knightvision_amd.engine import EVAL_HASH, SelfPlayEngine, records_by_game
from knightvision_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu


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
