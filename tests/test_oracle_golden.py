"""Pin the CPU oracle (oracle/kv_oracle.c, oracle/torch_ref.py) to the golden
fixtures generated from the reference itself (tests/golden/make_golden.py) and
to the live numpy / CPython RNGs it restates."""
import json
import os
import random

import numpy as np
import pytest
import torch

from oracle import oracle as O
from oracle import torch_ref
from knightvision_amd.weights import synthetic_state_dict


@pytest.fixture(scope="module")
def movegen(golden_dir):
    return np.load(os.path.join(golden_dir, "movegen.npz"))


def test_movegen_matches_reference(movegen):
    states, post, offs, moves, chk = (movegen[k] for k in ("states", "post_states", "offsets", "moves", "in_check"))
    bad = []
    for i in range(len(states)):
        got, st_after = O.valid_moves(states[i])
        want = moves[offs[i]:offs[i + 1]]
        if got.shape != want.shape or not np.array_equal(got, want) or not np.array_equal(st_after, post[i]):
            bad.append(i)
            continue
        if O.in_check(st_after) != bool(chk[i]):
            bad.append(i)
    assert not bad, f"{len(bad)} positions differ, first {bad[:5]}"


def test_unittest_scenarios(golden_dir):
    cases = json.load(open(os.path.join(golden_dir, "unittests.json")))
    for c in cases:
        if "seq" in c:
            for step in c["seq"]:
                got, _ = O.valid_moves(np.array(step["state"], dtype=np.int8))
                assert got.tolist() == step["moves"], c["name"]
        elif "after" in c:
            st = np.array(c["state"], dtype=np.int8)
            got, _ = O.valid_moves(st)
            idx = [i for i, m in enumerate(got.tolist()) if m == c["move"]][0]
            assert O.make_valid_move(st, idx).tolist() == c["after"]
        else:
            got, _ = O.valid_moves(np.array(c["state"], dtype=np.int8))
            assert got.tolist() == c["moves"], c["name"]


@pytest.mark.parametrize("seed", [0, 42, 43, 2**31 + 5])
def test_numpy_stream(seed):
    rs = np.random.RandomState(seed)
    mt = O.MT(seed, "numpy")
    ref = rs.randint(0, 2**32, size=700, dtype=np.uint64)  # not the legacy u32 path; use random_sample
    rs = np.random.RandomState(seed)
    want = rs.random_sample(700)
    got = np.array([mt.random() for _ in range(700)])
    assert np.array_equal(got, want)
    del ref


@pytest.mark.parametrize("seed", [42, 43, 44, 45, 7])
def test_dirichlet_bitexact_and_aligned(seed):
    rs = np.random.RandomState(seed)
    mt = O.MT(seed, "numpy")
    for _ in range(3):
        want = rs.dirichlet([0.3] * 4096)
        got, att = mt.dirichlet(0.3, 4096)
        assert np.array_equal(got, want)
        assert att >= 4096
    assert mt.random() == rs.random_sample()


@pytest.mark.parametrize("seed", [42, 43, 0, 123456789012])
def test_python_stream(seed):
    r = random.Random(seed)
    mt = O.MT(seed, "python")
    assert [mt.random() for _ in range(1000)] == [r.random() for _ in range(1000)]
    for n in (1, 2, 3, 7, 23, 64, 218):
        w = np.random.RandomState(n).random_sample(n)
        w = (w / w.sum()).tolist()
        assert mt.choices_index(w) == r.choices(range(n), weights=w, k=1)[0]
        assert mt.randbelow(n) == r.choice(range(n))


@pytest.fixture(scope="module")
def nn(golden_dir):
    return np.load(os.path.join(golden_dir, "nn.npz"))


@pytest.mark.parametrize("variant", ["init", "bn", "peaked"])
def test_torch_ref_matches_reference_net(nn, variant):
    sd = synthetic_state_dict(42, variant)
    p, v = torch_ref.forward(sd, nn["planes"])
    np.testing.assert_allclose(p.numpy(), nn[f"policy_{variant}"], rtol=0, atol=1e-6)
    np.testing.assert_allclose(v.numpy(), nn[f"value_{variant}"], rtol=0, atol=1e-6)


def test_encode_board_matches_golden_planes(nn, movegen):
    st = movegen["states"]
    idx = np.linspace(0, len(st) - 1, 12).astype(int)
    for k, i in enumerate(idx):
        assert np.array_equal(O.encode_board(st[i]), nn["planes"][k])


def _games(golden_dir, group):
    g = np.load(os.path.join(golden_dir, "games.npz"))
    n = g[f"{group}.n"]
    offs = np.concatenate([[0], np.cumsum(n)])
    ns = g[f"{group}.n_sizes"]
    soffs = np.concatenate([[0], np.cumsum(ns)])
    out = []
    for i in range(len(n)):
        out.append(dict(seed=int(g[f"{group}.seed"][i]), moves=g[f"{group}.moves"][offs[i]:offs[i + 1]],
                        reward=float(g[f"{group}.reward"][i]), sizes=g[f"{group}.sizes"][soffs[i]:soffs[i + 1]],
                        margins=g[f"{group}.margins"][offs[i]:offs[i + 1]]))
    return out


GROUPS = {"pg_init_mm80": ("init", 80, 16, False, 8), "pg_peaked_mm80": ("peaked", 80, 16, False, 6),
          "pg_init_b1_mm60": ("init", 60, 1, False, 3), "pg_init_full": ("init", None, 16, False, 2),
          "seq_init_full": ("init", None, 16, True, 2)}


@pytest.mark.parametrize("group", list(GROUPS))
def test_oracle_games_match_reference(golden_dir, group):
    variant, mm, batch, seq, ngames = GROUPS[group]
    games = _games(golden_dir, group)[:ngames]
    ev = torch_ref.make_eval_fn(synthetic_state_dict(42, variant))
    last = O.Last()
    if seq:
        npm, pym = O.MT(games[0]["seed"], "numpy"), O.MT(games[0]["seed"], "python")
    for g in games:
        if not seq:
            npm, pym, last = O.MT(g["seed"], "numpy"), O.MT(g["seed"], "python"), O.Last()
        r = O.play_game(ev, npm, pym, last, max_moves=mm, batch=batch, softmax_fn=torch_ref.torch_softmax)
        assert np.array_equal(r["moves"], g["moves"]), (group, g["seed"])
        assert r["reward"] == pytest.approx(g["reward"])
        assert r["eval_sizes"].tolist() == g["sizes"].tolist()
