"""The reinforcement loop of scripts/learn.py (reinforcement_loop :152-209) on
one process per GPU (BASELINE configs[4]):

    for each iteration:
        train on the data so far       (train_model -> train.py update step, DDP over RCCL)
        self-play with the new weights (generate_self_play_data -> libkv.so engine, games sharded by rank)
        dataset.extend(new records)    (decisive-record filter of generate_self_play_data :304-310)

Every rank keeps a shard of the experience on its GPU (int8 board codes, move
index, reward: 74 B per record instead of a 3 KB plane tensor, expanded per
batch on the device) and trains on it; DistributedDataParallel averages the
gradients with bucketed RCCL all-reduces overlapped with the backward pass.
The one data exchange is the end-of-iteration all-gather of the new records
(distributed.gather_rows, dst=None), filtered as one dataset (the reference's
global decisive filter) and re-sharded round-robin.
The global batch is the reference's: nn.DataParallel splits one batch of
BATCH_SIZE over the GPUs (utils/model_utils.py:26-28), so each of the W ranks
trains on batch_size // W rows per micro-batch with the same accumulation
count -- W x (batch_size // W) rows per micro-batch, one optimizer step per
accumulate_steps micro-batches, as on one process. Self-play game g of iteration i has the global id
i * games_per_iter + g and the seeds SEED + id (per-game seeding).

Not reproduced (out of the self-play path): the PGN dataset and
its 90/10 split, the Stockfish evaluation, checkpoints, Telegram and
TensorBoard logging.
"""
from __future__ import annotations

import time

import torch

from . import train as T
from .distributed import gather_rows
from .engine import SelfPlayEngine, packed_from
from .self_play import ALPHA, BATCH_SIZE as SELFPLAY_BATCH, EPSILON, SEED


def _dist():
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized():
        return dist, dist.get_rank(), dist.get_world_size()
    return None, 0, 1


def selfplay_shard(model, n_games: int, iteration: int, device, *, sims=0, max_moves=None, slots=256,
                   precision="fp32"):
    """This rank's share of one iteration's games, played by the HIP engine with
    the model's current weights. Returns (records, games) numpy arrays."""
    dist, rank, world = _dist()
    dev = torch.device(device)
    ids = list(range(rank, n_games, world))
    if not ids:
        return None, None
    base = iteration * n_games + rank
    from .self_play import batched_eval_mode
    with SelfPlayEngine(packed_from(model), slots=min(slots, len(ids)), n_games=len(ids), seed=SEED,
                        max_moves=max_moves, batch=SELFPLAY_BATCH, eps=EPSILON, alpha=ALPHA, sims=sims,
                        game_id_base=base, game_id_stride=world, device=dev.index or 0,
                        precision=precision, eval_mode=batched_eval_mode() if sims == 0 else 0) as eng:
        eng.run()
        return eng.records(), eng.games()


def _max_over_ranks(n: int, dev) -> int:
    dist, _, world = _dist()
    if dist is None or world == 1:
        return n
    t = torch.tensor([n], dtype=torch.int64, device=dev if dist.get_backend() == "nccl" else "cpu")
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return int(t.item())


def rank_batch_size(batch_size: int, world: int) -> int:
    """Per-rank micro-batch that keeps the reference's global batch (DataParallel
    scatters one batch of `batch_size` rows over the devices)."""
    return max(1, batch_size // world)


def decisive_filter(codes, moves, rewards):
    """generate_self_play_data (self_play.py:304-310): keep only records whose
    reward is +-1 when there are at least 10 of them."""
    dec = rewards.abs() == 1.0
    if int(dec.sum()) >= 10:
        return codes[dec], moves[dec], rewards[dec]
    return codes, moves, rewards


def extend_dataset(data, recs, games, dev):
    """dataset.extend(generate_self_play_data(...)) for one iteration: the ranks'
    new records are all-gathered (the one end-of-iteration exchange), filtered
    as one dataset, and re-sharded round-robin so every rank trains on an
    equal share."""
    _, rank, world = _dist()
    if recs is not None and len(recs):
        local = T.records_to_tensors(recs, games, dev)
    else:
        local = (torch.zeros((0, 64), dtype=torch.int8, device=dev), torch.zeros(0, dtype=torch.int64, device=dev),
                 torch.zeros(0, dtype=torch.float32, device=dev))
    union = decisive_filter(*(gather_rows(x, dst=None).to(dev) for x in local))
    mine = tuple(x[rank::world] for x in union)
    return mine if data is None else tuple(torch.cat([a, b]) for a, b in zip(data, mine))


def reinforcement_loop(model, iterations: int, games_per_iter: int, device, *, epochs: int = 1,
                       batch_size: int = T.BATCH_SIZE, lr: float = T.LR, accumulate_steps: int = T.ACCUM_STEPS,
                       sims: int = 0, max_moves=None, slots: int = 256, seed: int = 0, log=print):
    """Run the loop; returns per-iteration statistics. `model` is a
    knightvision_amd.model.ChessNet (same parameters as ai/model.py) on `device`."""
    _, rank, world = _dist()
    dev = torch.device(device)
    model.to(dev)
    optimizer = torch.optim.Adam(model.parameters(), lr=lr)
    scaler = T.make_scaler(dev)
    ddp = T.wrap_ddp(model, dev)
    gen = torch.Generator().manual_seed(seed + rank)
    data = None  # (codes, moves, rewards) on the device: this rank's dataset
    stats = []
    for it in range(iterations):
        st = {"iteration": it + 1}
        n_local = int(data[0].shape[0]) if data is not None else 0
        n_max = _max_over_ranks(n_local, dev)
        n_min = -_max_over_ranks(-n_local, dev)
        if n_min > 0:  # every rank holds data (fewer records than ranks: no update this iteration)
            t0 = time.perf_counter()
            per_rank = rank_batch_size(batch_size, world)
            for _ in range(epochs):
                ep = T.train_one_epoch(ddp, T.batches(*data, per_rank, True, gen, total=n_max), optimizer, scaler,
                                       accumulate_steps=accumulate_steps)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            st.update(train_s=time.perf_counter() - t0, train_loss=ep["loss"], train_samples=ep["samples"],
                      optimizer_steps=ep["optimizer_steps"])
        model.eval()
        t0 = time.perf_counter()
        recs, games = selfplay_shard(model, games_per_iter, it, dev, sims=sims, max_moves=max_moves, slots=slots)
        st["selfplay_s"] = time.perf_counter() - t0
        model.train()
        data = extend_dataset(data, recs, games, dev)
        st.update(records=int(data[0].shape[0]) if data is not None else 0,
                  games=int(len(games)) if games is not None else 0)
        if rank == 0 and log:
            log(f"iteration {it + 1}/{iterations}: {st}")
        stats.append(st)
    return stats
