"""The reinforcement loop of scripts/learn.py (reinforcement_loop :152-209) on
one process per GPU (BASELINE configs[4]):

    for each iteration:
        train_with_validation on a 90/10 random split of the data so far (train.py:293-420: epochs of
            the update step, DDP over RCCL, validation loss, ReduceLROnPlateau, early stopping)
        self-play with the new weights (generate_self_play_data -> libkv.so engine, games sharded by rank)
        dataset.extend(new records)    (decisive-record filter of generate_self_play_data :304-310)

The dataset is optionally seeded with the reference's JSONL training data
(ChessPGNDataset, learn.py:162). Every rank holds the whole dataset on its GPU
(int8 board codes, move index, reward: 76 B per sample instead of a 3 KB plane
tensor, expanded per batch on the device), draws the same split and trains on
its round-robin shard of the train subset; DistributedDataParallel averages
the gradients with bucketed RCCL all-reduces overlapped with the backward
pass. The one data exchange is the end-of-iteration all-gather of the new
records (distributed.gather_rows, dst=None), filtered as one dataset (the
reference's global decisive filter).
The global batch is the reference's: nn.DataParallel splits one batch of
BATCH_SIZE over the GPUs (utils/model_utils.py:26-28), so each of the W ranks
trains on batch_size // W rows per micro-batch with the same accumulation
count -- W x (batch_size // W) rows per micro-batch, one optimizer step per
accumulate_steps micro-batches, as on one process. Self-play game g of iteration i has the global id
i * games_per_iter + g and the seeds SEED + id (per-game seeding).

Not reproduced (out of the self-play path): the Stockfish
evaluation, checkpoints, Telegram and TensorBoard logging.
"""
from __future__ import annotations

import math
import os
import time

import torch

from . import train as T
from .distributed import gather_rows
from .engine import SelfPlayEngine, packed_from
from .self_play import ALPHA, BATCH_SIZE as SELFPLAY_BATCH, EPSILON, SEED

# learn.py's configuration (:105-112) and train.py's scheduler constants (:21, :463-464)
TRAIN_EPOCHS = int(os.getenv("TRAIN_EPOCHS", "2"))
LEARN_BATCH_SIZE = int(os.getenv("BATCH_SIZE", "2048"))
LEARN_LR = float(os.getenv("LR", "1e-3"))
PATIENCE = int(os.getenv("PATIENCE", "5"))
LR_GAMMA = float(os.getenv("LR_GAMMA", "0.1"))
LR_STEP_SIZE = int(os.getenv("LR_STEP_SIZE", "10"))  # train.py:463
COSINE_T0 = int(os.getenv("COSINE_T0", "10"))        # train.py:295
VAL_FRAC = 0.1


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
        selfplay_shard.last_calibration = eng.calibration()  # the conv paths these weights ran on
        selfplay_shard.last_stats = eng.stats()
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
    """dataset.extend(generate_self_play_data(...)) for one iteration
    (learn.py:194-199): the ranks' new records are all-gathered (the one
    end-of-iteration exchange) and filtered as one dataset (the reference's
    global decisive filter); every rank appends the same union, so every rank
    holds the whole dataset (64 + 12 B per sample) and the 90/10 split below is
    the same on all of them."""
    if recs is not None and len(recs):
        local = T.records_to_tensors(recs, games, dev)
    else:
        local = (torch.zeros((0, 64), dtype=torch.int8, device=dev), torch.zeros(0, dtype=torch.int64, device=dev),
                 torch.zeros(0, dtype=torch.float32, device=dev))
    union = decisive_filter(*(gather_rows(x, dst=None).to(dev) for x in local))
    return union if data is None else tuple(torch.cat([a, b]) for a, b in zip(data, union))


def split_train_val(n: int, gen: torch.Generator):
    """random_split(dataset, [int(0.9 n), n - int(0.9 n)]) (learn.py:162-165, :196-199): index tensors of the
    train and validation subsets (the generator is seeded alike on every rank)."""
    perm = torch.randperm(n, generator=gen)
    n_train = int((1.0 - VAL_FRAC) * n)
    return perm[:n_train], perm[n_train:]


def evaluate_sharded(model, data, idx, batch_size: int, dev) -> float:
    """train.evaluate (train.py:109-124) over a validation subset split round-robin over the ranks:
    sum of per-sample (CE + MSE) and the sample count all-reduced, then their ratio."""
    dist, rank, world = _dist()
    mine = idx[rank::world].to(dev)
    tot = torch.zeros(2, dtype=torch.float64, device=dev)
    if mine.numel():
        batches = list(T.batches(*(x[mine] for x in data), batch_size, False))
        n = sum(b.boards.shape[0] for b in batches)
        tot[0] = T.evaluate(model, batches) * n
        tot[1] = n
    if dist is not None and world > 1:
        t = tot.to(dev if dist.get_backend() == "nccl" else "cpu")
        dist.all_reduce(t)
        tot = t
    return float(tot[0] / tot[1]) if float(tot[1]) > 0 else math.inf


def train_with_validation(ddp, model, optimizer, data, epochs: int, batch_size: int, accumulate_steps: int,
                          gen: torch.Generator, split_gen: torch.Generator, dev) -> dict:
    """train.py train_with_validation (:293-420) as the learn loop calls it (TRAIN_EPOCHS = 2 <
    NUM_PGN_EPOCHS, so no self-play inside it). Per call, as the reference: a fresh GradScaler and the
    three LR schedulers in its order -- CosineAnnealingWarmRestarts(T_0=COSINE_T0, T_mult=1) (:293-297;
    constructing it resets the LR to the optimizer's initial LR, so the cosine schedule restarts every
    iteration), ReduceLROnPlateau(mode='min', factor=LR_GAMMA, patience=PATIENCE) (:298-304) and
    StepLR(LR_STEP_SIZE, LR_GAMMA) (:306-307). Per epoch one pass of _train_one_epoch over the train
    split, evaluate() on the validation split and the plateau step on its loss (_run_validation
    :198-218), early stopping after PATIENCE epochs without improvement (before the other two
    schedulers step), then cos.step(epoch + 1) and step.step() (:421-423). Checkpoints, TensorBoard
    and Telegram are not reproduced."""
    import warnings
    dist, rank, world = _dist()
    tr, va = split_train_val(int(data[0].shape[0]), split_gen)
    mine = tr[rank::world].to(dev)
    n_max = _max_over_ranks(int(mine.numel()), dev)
    scaler = T.make_scaler(dev)
    cos, plateau, step = make_lr_schedulers(optimizer)
    best, no_improve, ep, val_loss, done = math.inf, 0, None, math.inf, 0
    shard = tuple(x[mine] for x in data)
    lrs = []
    for epoch in range(epochs):
        ep = T.train_one_epoch(ddp, T.batches(*shard, rank_batch_size(batch_size, world), True, gen, total=n_max),
                               optimizer, scaler, accumulate_steps=accumulate_steps)
        val_loss = evaluate_sharded(model, data, va, batch_size, dev)
        plateau.step(val_loss)
        done += 1
        if val_loss < best:
            best, no_improve = val_loss, 0
        else:
            no_improve += 1
            if no_improve >= PATIENCE:
                break
        with warnings.catch_warnings():  # the reference passes the epoch to step() (deprecated form)
            warnings.simplefilter("ignore")
            cos.step(epoch + 1)
        step.step()
        lrs.append(optimizer.param_groups[0]["lr"])
    return {"ep": ep, "val_loss": val_loss, "epochs_run": done, "train_split": int(tr.numel()),
            "val_split": int(va.numel()), "lr": optimizer.param_groups[0]["lr"], "lr_per_epoch": lrs}


def make_lr_schedulers(optimizer):
    """The three schedulers train_with_validation builds per call (train.py:293-307), in its order."""
    cos = torch.optim.lr_scheduler.CosineAnnealingWarmRestarts(optimizer, T_0=COSINE_T0, T_mult=1)
    plateau = torch.optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=LR_GAMMA, patience=PATIENCE)
    step = torch.optim.lr_scheduler.StepLR(optimizer, step_size=LR_STEP_SIZE, gamma=LR_GAMMA)
    return cos, plateau, step


def reinforcement_loop(model, iterations: int, games_per_iter: int, device, *, epochs: int = TRAIN_EPOCHS,
                       batch_size: int = LEARN_BATCH_SIZE, lr: float = LEARN_LR,
                       accumulate_steps: int = T.ACCUM_STEPS, sims: int = 0, max_moves=None, slots: int = 256,
                       seed: int = 0, games_path: str | None = None, max_samples: int = 10000, log=print):
    """Run the loop (learn.py reinforcement_loop :152-209); returns per-iteration statistics.
    `model` is a knightvision_amd.model.ChessNet (same parameters as ai/model.py) on `device`.
    `games_path`: the reference's JSONL dataset (ChessPGNDataset, :162) the self-play records extend --
    each sample keeps its own source's plane order and move indexing, as in the reference; None:
    self-play records only (iteration 1 then has nothing to train on)."""
    _, rank, world = _dist()
    dev = torch.device(device)
    model.to(dev)
    optimizer = torch.optim.Adam(model.parameters(), lr=lr)
    ddp = T.wrap_ddp(model, dev)
    gen = torch.Generator().manual_seed(seed + rank)      # batch order (DataLoader shuffle), per rank
    split_gen = torch.Generator().manual_seed(seed)       # random_split: the same on every rank
    data = None  # (codes, moves, rewards) on the device: the whole dataset, on every rank
    if games_path is not None:
        data = T.ChessPGNDataset(games_path, max_samples=max_samples).materialize(dev)
    stats = []
    for it in range(iterations):
        st = {"iteration": it + 1}
        n = int(data[0].shape[0]) if data is not None else 0
        if n >= 2 * world:  # every rank holds train data (fewer samples: no update this iteration)
            t0 = time.perf_counter()
            tv = train_with_validation(ddp, model, optimizer, data, epochs, batch_size, accumulate_steps, gen,
                                       split_gen, dev)
            if dev.type == "cuda":
                torch.cuda.synchronize(dev)
            ep = tv["ep"]
            st.update(train_s=time.perf_counter() - t0, train_loss=ep["loss"], train_samples=ep["samples"],
                      optimizer_steps=ep["optimizer_steps"], val_loss=tv["val_loss"], epochs_run=tv["epochs_run"],
                      train_split=tv["train_split"], val_split=tv["val_split"], lr=tv["lr"])
        model.eval()
        t0 = time.perf_counter()
        recs, games = selfplay_shard(model, games_per_iter, it, dev, sims=sims, max_moves=max_moves, slots=slots)
        st["selfplay_s"] = time.perf_counter() - t0
        cal = getattr(selfplay_shard, "last_calibration", None)
        if cal is not None:  # fp32 AUTO: the self-play network's conv path for this iteration's weights
            st["nn_path"] = cal["path_large"]
            if cal.get("calibrated"):  # the load-time calibration (inside selfplay_s) and its candidates' errors
                st["calib_ms"] = cal["ms"]
                st["calib_err"] = {k: (cal["err_logit"][k], cal["err_value"][k]) for k in cal["err_logit"]}
        es = getattr(selfplay_shard, "last_stats", None)
        if es is not None:  # this rank's engine: plies and MCTS simulations (the throughput a path flip moves)
            st.update(plies=int(es["plies"]), sims=int(es["sims"]))
        model.train()
        data = extend_dataset(data, recs, games, dev)
        st.update(records=int(data[0].shape[0]) if data is not None else 0,
                  games=int(len(games)) if games is not None else 0)
        if rank == 0 and log:
            log(f"iteration {it + 1}/{iterations}: {st}")
        stats.append(st)
    return stats
