"""Shard equivalence of the multi-GPU self-play path. The
reference's Pool "parallelism" plays the same seeded game in every worker
(scripts/self_play.py:273-282); the build shards global game ids instead --
rank r plays ids r, r+W, r+2W, ... with per-game seeds SEED + id -- so the
shard rule is the correctness argument: the union of the W shards must be
exactly the games of one unsharded engine over the same ids.

Both halves run on the 1-GPU box: two engines with game_id_base 0/1 and
game_id_stride 2 in one process, and two ranks (gloo, sharing cuda:0) that
gather their device-resident records to rank 0 through
knightvision_amd.distributed.gather_experience."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from knightvision_amd.engine import SelfPlayEngine
from knightvision_amd.weights import synthetic_state_dict

pytestmark = pytest.mark.gpu

SD = synthetic_state_dict(42, "init")
N_GAMES = 40  # 20 per shard: both engines batch > 16 boards (the same network class)


def _play(base, stride, n, sims, max_moves, device_records=False, pi=False):
    with SelfPlayEngine(SD, slots=n, n_games=n, seed=42, max_moves=max_moves, sims=sims, game_id_base=base,
                        game_id_stride=stride, keep_root_visits=pi) as eng:
        eng.run()
        recs = eng.records_device() if device_records else eng.records()
        if pi:
            return recs, eng.games(), (eng.root_visits_device() if device_records else eng.root_visits())
        return recs, eng.games()


def _sorted(recs, games):
    recs = recs[np.lexsort((recs["ply"], recs["game_id"]))]
    return recs, games[np.argsort(games["game_id"], kind="stable")]


@pytest.mark.parametrize("sims,max_moves", [(0, 40), (16, 4)])
def test_two_shards_equal_one_engine(sims, max_moves):
    whole_r, whole_g = _play(0, 1, N_GAMES, sims, max_moves)
    parts = [_play(r, 2, N_GAMES // 2, sims, max_moves) for r in range(2)]
    for r, (recs, games) in enumerate(parts):
        assert set(np.unique(recs["game_id"]).tolist()) == set(range(r, N_GAMES, 2))
    u_r, u_g = _sorted(np.concatenate([p[0] for p in parts]), np.concatenate([p[1] for p in parts]))
    assert len(u_r) == len(whole_r) and len(u_g) == len(whole_g) == N_GAMES
    assert np.array_equal(u_r, whole_r), "sharded records differ from the unsharded run"
    assert np.array_equal(u_g, whole_g), "sharded game results differ from the unsharded run"


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank(rank, world, port, q, sims=0, max_moves=30):
    import torch.distributed as dist
    from knightvision_amd.distributed import gather_experience
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)  # RCCL refuses two ranks on one GPU
    if sims:
        recs, games, pi = _play(rank, world, N_GAMES // world, sims, max_moves, device_records=True, pi=True)
        all_r, all_g, all_p = gather_experience(recs, games, dst=0, pi=pi)
    else:
        recs, games = _play(rank, world, N_GAMES // world, 0, max_moves, device_records=True)
        all_r, all_g = gather_experience(recs, games, dst=0)
        all_p = None
    if rank == 0:
        q.put((all_r.tobytes(), all_g.tobytes(), None if all_p is None else all_p.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def test_gather_of_engine_shards_to_root():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    rb, gb, _ = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole_r, whole_g = _play(0, 1, N_GAMES, 0, 30)
    from knightvision_amd.engine import GAME_DTYPE, RECORD_DTYPE
    got_r = np.frombuffer(rb, dtype=RECORD_DTYPE)
    got_g = np.frombuffer(gb, dtype=GAME_DTYPE)
    assert np.array_equal(got_r, whole_r) and np.array_equal(got_g, whole_g)


def test_gather_of_mcts_shards_with_pi_to_root():
    """BASELINE config C4's gather of (s, pi, z): MCTS shards gather their records and root visit counts
    (pi) to rank 0 straight from HBM; both equal the unsharded run's, row for row."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank, args=(r, 2, port, q, 16, 4)) for r in range(2)]
    for p in procs:
        p.start()
    rb, gb, pb = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    whole_r, whole_g, whole_p = _play(0, 1, N_GAMES, 16, 4, pi=True)
    from knightvision_amd import _lib
    from knightvision_amd.engine import GAME_DTYPE, RECORD_DTYPE
    got_r = np.frombuffer(rb, dtype=RECORD_DTYPE)
    got_g = np.frombuffer(gb, dtype=GAME_DTYPE)
    got_p = np.frombuffer(pb, dtype=np.uint16).reshape(-1, _lib.MAXM)
    assert np.array_equal(got_r, whole_r) and np.array_equal(got_g, whole_g)
    want_p = np.where(whole_p < 0, 0xffff, whole_p).astype(np.uint16)
    assert np.array_equal(got_p, want_p)
    assert (got_p[:, 0] != 0xffff).all() and (np.where(got_p == 0xffff, 0, got_p).sum(axis=1) == 16).all()
