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


def _rccl_world1(port, q):
    """One rank on RCCL ('nccl' backend = RCCL on ROCm) with the collectives forced: the all_gather of the
    per-rank counts and the gather / all_gather of device-resident records and pi run through RCCL on
    device tensors -- the code path of the driver's 8-GPU run, on the one GPU this box has."""
    import torch
    import torch.distributed as dist
    from knightvision_amd.distributed import comm_device, gather_experience
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    assert dist.get_backend() == "nccl" and comm_device().type == "cuda"
    with SelfPlayEngine(SD, slots=20, n_games=20, seed=42, max_moves=4, sims=16, keep_root_visits=True) as eng:
        eng.run()
        host_r, host_g, host_p = eng.records(), eng.games(), eng.root_visits()
        dev_r, dev_p = eng.records_device(), eng.root_visits_device()
        assert dev_r.is_cuda and dev_p.is_cuda
        out = []
        for dst in (0, None):
            r, g, p = gather_experience(dev_r, host_g, dst=dst, pi=dev_p, force_collective=True)
            out.append((r.tobytes(), g.tobytes(), p.tobytes()))
    want_p = np.where(host_p < 0, 0xffff, host_p).astype(np.uint16)
    q.put((out, host_r.tobytes(), host_g.tobytes(), want_p.tobytes()))
    dist.barrier()
    dist.destroy_process_group()


def test_rccl_gather_path_world1():
    """VERDICT r2 #3a: the experience gather over RCCL on device tensors (the all_gather of counts and the
    gather / all_gather of packed records and legal-move pi), forced through the collectives at world
    size 1, equals the engine's own host-side records and visit counts."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_rccl_world1, args=(_free_port(), q))
    p.start()
    out, hr, hg, hp = q.get(timeout=300)
    p.join(timeout=120)
    assert p.exitcode == 0
    for rb, gb, pb in out:
        assert rb == hr and gb == hg and pb == hp


def test_bench_json_line_contract():
    """bench.py's one JSON line (the driver's contract) on a tiny MCTS config, run as the driver runs it (a
    child process): every required key, value = completed backups / timed seconds, roofline + cpu_baseline
    objects present."""
    import json
    import subprocess
    import sys
    repo = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = dict(os.environ, KV_CPU_WORKERS="2")
    out = subprocess.run([sys.executable, os.path.join(repo, "bench.py"), "--slots", "32", "--sims", "8",
                          "--steps", "2", "--warmup", "1", "--alt-precision=", "--ref-block", "0",
                          "--cpu-seconds", "2"], capture_output=True, text=True, timeout=240, env=env, cwd=repo)
    assert out.returncode == 0, out.stderr[-2000:]
    lines = [l for l in out.stdout.splitlines() if l.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 2 and d["warmup"] == 1 and d["unit"] == "sims/s"
    assert d["value"] > 0 and abs(d["value"] * d["ms_per_step"] * 1e-3 * 2 - 32 * 8 * 2) < 1e-6 * 32 * 8 * 2
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in d["roofline"], k
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in d["cpu_baseline"], k
    c = d["calibration"]  # the conv paths the run used, chosen by the load-time calibration (random-init: the
    # fp32 F(8x8) tower on 3 radix-256 int8 digits)
    assert c["calibrated"] and c["path_large"] == "winograd88_i8f32r3" and c["path_small"] == "direct"
    assert d["conv_path"] == "winograd88_i8f32r3" and d["roofline"]["peak"] == 5000.0  # int8 operations vs the peak
    # the name the library reported for the launch it made: R3's 64-k-stage GEMM (KV_I8R3_K64=0: the 32-k one)
    assert d["roofline"]["kernel"].startswith(("wino88i32_gemm_r3k64_kernel<512,", "wino88i32_gemm_lagt_kernel<512,"))
    assert d["roofline"]["sclk_mhz"] is None or 500 < d["roofline"]["sclk_mhz"] < 2600
    assert d["trained_weights_path"]["value"] > 0


def _ddp_world1(port, q):
    """One RCCL rank with DistributedDataParallel forced on (train.wrap_ddp(force=True)) and the rank-agreed
    NaN skip's all_reduce forced through RCCL (train_one_epoch(force_collective=True)): one epoch of the HIP
    update step equals the unwrapped one bit for bit -- the learn loop's 8-GPU code path
    (scripts/train.py:604-606 nn.DataParallel -> DDP over RCCL) on the one GPU this box has."""
    import torch
    import torch.distributed as dist
    from knightvision_amd import train as T
    from knightvision_amd.model import ChessNet
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    torch.cuda.set_device(0)
    dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
    sd = synthetic_state_dict(42, "bn")
    g = torch.Generator().manual_seed(3)
    codes = (torch.randint(1, 13, (64, 64), generator=g) * (torch.rand(64, 64, generator=g) < 0.4)).to(torch.int8)
    moves = torch.randint(0, 4096, (64,), generator=g)
    rew = torch.randint(0, 3, (64,), generator=g).float() - 1.0
    codes, moves, rew = codes.cuda(), moves.cuda(), rew.cuda()
    batches = [T.Batch(T.codes_to_planes_t(codes[i:i + 16]), moves[i:i + 16], rew[i:i + 16]) for i in range(0, 64, 16)]
    res = {}
    for mode in ("plain", "ddp"):
        m = ChessNet()
        m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
        m.cuda().train()
        model = T.wrap_ddp(m, "cuda:0", force=(mode == "ddp"))
        assert isinstance(model, torch.nn.parallel.DistributedDataParallel) == (mode == "ddp")
        opt = torch.optim.Adam(m.parameters(), lr=1e-3)
        st = T.train_one_epoch(model, batches, opt, T.make_scaler("cuda"), accumulate_steps=2,
                               force_collective=(mode == "ddp"))
        torch.cuda.synchronize()
        res[mode] = ([p.detach().cpu().clone() for p in m.parameters()],
                     [b.detach().cpu().clone() for b in m.buffers()], st)
    diff = max(float((a.double() - b.double()).abs().max()) for a, b in zip(res["plain"][0], res["ddp"][0]))
    same_p = all(torch.equal(a, b) for a, b in zip(res["plain"][0], res["ddp"][0]))
    same_b = all(torch.equal(a, b) for a, b in zip(res["plain"][1], res["ddp"][1]))
    moved = max(float((a.double() - torch.from_numpy(np.asarray(sd[k], dtype=np.float64))).abs().max())
                for (k, _), a in zip(ChessNet().named_parameters(), res["ddp"][0]))
    ok = T._finite_on_all_ranks(torch.tensor(1.5, device="cuda"), force=True)
    bad = T._finite_on_all_ranks(torch.tensor(float("nan"), device="cuda"), force=True)
    inf = T._finite_on_all_ranks(torch.tensor(float("inf"), device="cuda"), force=True)
    q.put(dict(same_p=same_p, same_b=same_b, diff=diff, moved=moved, ok=ok, bad=bad, inf=inf,
               st_plain=res["plain"][2], st_ddp=res["ddp"][2], backend=dist.get_backend()))
    dist.barrier()
    dist.destroy_process_group()


def test_ddp_and_nan_skip_over_rccl_world1():
    """DDP over RCCL and the NaN skip's all_reduce on device tensors, executed (world 1, forced)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    p = ctx.Process(target=_ddp_world1, args=(_free_port(), q))
    p.start()
    r = q.get(timeout=300)
    p.join(timeout=120)
    print(r)
    assert p.exitcode == 0 and r["backend"] == "nccl"
    assert r["ok"] is True and r["bad"] is False and r["inf"] is False
    assert r["st_ddp"]["optimizer_steps"] == r["st_plain"]["optimizer_steps"] == 2
    assert r["st_ddp"]["loss"] == r["st_plain"]["loss"]
    assert r["moved"] > 0  # the epoch changed the weights
    assert r["same_p"] and r["same_b"], f"DDP update differs from the unwrapped one by up to {r['diff']}"
