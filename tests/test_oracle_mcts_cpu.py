"""The oracle's PUCT restatement played as a lock-step batch (kvo_mcts_play_batch:
the leaves of every game's simulation evaluated as one network batch, the
device's batch shape -- used by bench.py's batched CPU baseline) equals the
single-game restatement game by game (CPU; test infrastructure)."""
import numpy as np
import pytest

from oracle import oracle as O


def _single(sims, seed, ev, max_moves):
    return O.mcts_play_game(sims, O.MT(seed, "numpy"), O.MT(seed, "python"), ev, max_moves=max_moves)


@pytest.mark.parametrize("sims,max_moves", [(16, 6), (48, 3)])
def test_batch_equals_single_games_hash_evaluator(sims, max_moves):
    seeds = [42, 43, 44, 45, 46]
    batch = O.mcts_play_batch(sims, seeds, None, max_moves=max_moves, keep_visits=True)
    for s, b in zip(seeds, batch):
        g = _single(sims, s, None, max_moves)
        assert np.array_equal(g["moves"], b["moves"]) and np.array_equal(g["visits"], b["visits"])
        assert (g["plies"], g["outcome"], g["reason"], g["n_evals"]) == (b["plies"], b["outcome"], b["reason"],
                                                                          b["n_evals"])


def test_batch_equals_single_games_network():
    """With the torch ChessNet restatement: the batched evaluation gives each leaf the row it gets alone
    (compared on the chosen moves and root visit vectors; logits may differ in the last bit between a
    batched and a batch-1 CPU forward, so the games are short and the priors the hash-free network's)."""
    from knightvision_amd.weights import synthetic_state_dict
    from oracle import torch_ref
    ev = torch_ref.make_eval_fn(synthetic_state_dict(42, "peaked"))
    calls = []

    def counting(x):
        calls.append(len(x))
        return ev(x)
    seeds = [42, 43, 44]
    batch = O.mcts_play_batch(8, seeds, counting, max_moves=2, keep_visits=True)
    assert max(calls) == 3  # the leaves of the three games went out together
    for s, b in zip(seeds, batch):
        g = _single(8, s, ev, 2)
        assert np.array_equal(g["moves"], b["moves"]) and np.array_equal(g["visits"], b["visits"])
