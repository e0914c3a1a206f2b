"""Multi-GPU self-play: one process per GPU, games sharded by global id
(rank r plays ids r, r+W, r+2W, ... -- per-game seeds make the shards
independent, so there is no collective in the inner loop), and one gather of
the packed experience records to rank 0 at the end of an iteration.

The gather moves packed 80-byte records (kv_record: game id, ply, move index,
64 board codes) -- 38x smaller than the (12,8,8) float32 planes the trainer
expands them into. With the "nccl" backend (RCCL over xGMI on ROCm) the
buffers are GPU tensors; with "gloo" (CPU tests) they are host tensors.
"""
from __future__ import annotations

import numpy as np
import torch
import torch.distributed as dist

from .engine import GAME_DTYPE, RECORD_DTYPE


def rank_world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def _gather_bytes(buf: np.ndarray, device) -> list:
    """all-gather variable-length uint8 arrays (counts first, then padded)."""
    rank, world = rank_world()
    if world == 1:
        return [buf]
    n = torch.tensor([buf.size], dtype=torch.int64, device=device)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    mx = max(max(counts), 1)
    t = torch.zeros(mx, dtype=torch.uint8, device=device)
    if buf.size:
        t[:buf.size] = torch.from_numpy(buf).to(device)
    outs = [torch.zeros(mx, dtype=torch.uint8, device=device) for _ in range(world)]
    dist.all_gather(outs, t)
    return [o[:c].cpu().numpy() for o, c in zip(outs, counts)]


def gather_experience(records: np.ndarray, games: np.ndarray, device=None):
    """-> (records, games) of every rank, ordered by (game_id, ply), on every
    rank (all-gather: the data-parallel trainer of the next iteration reads it
    on every rank)."""
    if device is None:
        backend = dist.get_backend() if dist.is_initialized() else "gloo"
        device = torch.device("cuda", torch.cuda.current_device()) if backend == "nccl" else torch.device("cpu")
    r = _gather_bytes(np.ascontiguousarray(records).view(np.uint8).reshape(-1), device)
    g = _gather_bytes(np.ascontiguousarray(games).view(np.uint8).reshape(-1), device)
    recs = np.concatenate([x.view(RECORD_DTYPE) for x in r]) if r else np.zeros(0, RECORD_DTYPE)
    gms = np.concatenate([x.view(GAME_DTYPE) for x in g]) if g else np.zeros(0, GAME_DTYPE)
    recs = recs[np.lexsort((recs["ply"], recs["game_id"]))]
    gms = gms[np.argsort(gms["game_id"], kind="stable")]
    return recs, gms


def shard_ids(n_games: int, rank: int, world: int):
    """global game ids of this rank's shard: base=rank, stride=world."""
    return rank, world, len(range(rank, n_games, world))
