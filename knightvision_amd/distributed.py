"""Multi-GPU self-play: one process per GPU, games sharded by global id
(rank r plays ids r, r+W, r+2W, ... -- per-game seeds make the shards
independent, so there is no collective in the inner loop), and one gather of
the packed experience records at the end of an iteration.

The gather moves packed 80-byte records (kv_record: game id, ply, move index,
64 board codes) -- 38x smaller than the (12,8,8) float32 planes the trainer
expands them into -- and, for MCTS, each record's root visit counts (pi,
uint16 per legal move) straight from HBM: the engine copies its record buffer
device-to-device (kv_records_device) and RCCL (the "nccl" backend on ROCm,
over xGMI) moves it; "gloo" (CPU tests) moves host tensors.

One implementation, `gather_rows`, serves both consumers:
  * dst=0: gather to the root (the data-generation path: one trainer process,
    as the reference's generate_self_play_data returns the list to its caller,
    scripts/learn.py:186-191) -- N-1 shards cross xGMI once;
  * dst=None: all-gather (the data-parallel learn loop, knightvision_amd/
    learn.py, where every rank trains on its slice of the filtered union).
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


def comm_device(t: torch.Tensor | None = None) -> torch.device:
    """Where collectives run: the current GPU under RCCL, the host under gloo."""
    if dist.is_initialized() and dist.get_backend() == "nccl":
        return t.device if (t is not None and t.is_cuda) else torch.device("cuda", torch.cuda.current_device())
    return torch.device("cpu")


def gather_rows(t: torch.Tensor, dst: int | None = 0, force_collective: bool = False):
    """Concatenation over ranks (rank order) of a tensor whose first dimension
    differs per rank: per-rank row counts are all-gathered (int64), then the
    rows padded to the largest count are gathered to `dst` (None: to every
    rank). Returns the concatenation on `dst` / every rank, None elsewhere.
    A world of one returns `t` itself unless force_collective (tests: the
    collectives then run on a one-rank group, e.g. RCCL on one GPU)."""
    rank, world = rank_world()
    if world == 1 and not (force_collective and dist.is_initialized()):
        return t
    dev = comm_device(t)
    src = t.to(dev)
    n = torch.tensor([src.shape[0]], dtype=torch.int64, device=dev)
    counts = [torch.zeros_like(n) for _ in range(world)]
    dist.all_gather(counts, n)
    counts = [int(c.item()) for c in counts]
    mx = max(max(counts), 1)
    pad = torch.zeros((mx,) + tuple(src.shape[1:]), dtype=src.dtype, device=dev)
    pad[:src.shape[0]] = src
    if dst is None:
        parts = [torch.empty_like(pad) for _ in range(world)]
        dist.all_gather(parts, pad)
    else:
        parts = [torch.empty_like(pad) for _ in range(world)] if rank == dst else None
        dist.gather(pad, parts, dst=dst)
        if rank != dst:
            return None
    return torch.cat([p[:k] for p, k in zip(parts, counts)])


def record_order(rows: torch.Tensor) -> torch.Tensor:
    """uint8 [n, 80] kv_record rows -> the permutation ordering them by (game_id, ply) (two stable sorts)."""
    gid = rows[:, 0:8].contiguous().view(torch.int64).reshape(-1)
    ply = rows[:, 8:12].contiguous().view(torch.int32).reshape(-1)
    o1 = torch.sort(ply, stable=True).indices
    o2 = torch.sort(gid[o1], stable=True).indices
    return o1[o2]


def sort_records(rows: torch.Tensor) -> torch.Tensor:
    """uint8 [n, 80] kv_record rows -> ordered by (game_id, ply) (on the rows' device)."""
    if rows.shape[0] == 0:
        return rows
    return rows[record_order(rows)]


def _as_rows(x, dtype) -> torch.Tensor:
    if isinstance(x, torch.Tensor):
        return x.reshape(-1, dtype.itemsize)
    return torch.from_numpy(np.ascontiguousarray(x).view(np.uint8).reshape(-1, dtype.itemsize))


def pack_pi(pi_rows: torch.Tensor):
    """Root visit counts as they cross xGMI: uint8 [n, 2 * MAXM] rows (uint16 per
    move slot, 0xffff past the position's move list -- kv_root_visits_device)
    -> (counts int16 [n], packed int16 [sum counts]): each row's legal-move
    prefix only, rows concatenated in order. 2 B per legal move + 2 B per record
    instead of 640 B per record (MAXM 320, ~23 legal moves on average).
    The valid entries of a row are a prefix (kv_root_visits_device pads past
    the move list) and never 0xffff themselves (visit counts <= KV_MAX_SIMS =
    65000)."""
    if pi_rows.shape[0] == 0:
        z = torch.zeros(0, dtype=torch.int16, device=pi_rows.device)
        return z, z.clone()
    v = pi_rows.contiguous().view(torch.int16)  # 2-D rows of bytes -> int16 per move slot
    valid = v != -1
    counts = valid.sum(1, dtype=torch.int32)
    return counts.to(torch.int16), v[valid]


def unpack_pi(counts: torch.Tensor, packed: torch.Tensor, maxm: int) -> torch.Tensor:
    """pack_pi's inverse: int16 [n, maxm] rows, -1 (0xffff) past each row's count."""
    n = int(counts.shape[0])
    out = torch.full((n, maxm), -1, dtype=torch.int16, device=packed.device)
    if n == 0 or packed.numel() == 0:
        return out
    c = counts.to(device=packed.device, dtype=torch.int64)
    row = torch.repeat_interleave(torch.arange(n, device=packed.device), c)
    start = torch.cumsum(c, 0) - c
    col = torch.arange(packed.numel(), device=packed.device) - start[row]
    out[row, col] = packed
    return out


def gather_experience(records, games, dst: int | None = 0, pi=None, force_collective: bool = False):
    """End-of-iteration gather of every rank's (records, games), ordered by
    (game_id, ply) / game_id. `records` is a numpy RECORD_DTYPE array or the
    engine's device tensor (SelfPlayEngine.records_device(), uint8 [n, 80]);
    `games` a GAME_DTYPE array. MCTS runs also pass `pi`, the root visit counts
    row for row with `records` (SelfPlayEngine.root_visits_device(), uint8
    [n, 2 * MAXM]): the (s, pi, z) triple of BASELINE config C4 (s = board,
    z = the game's reward) then crosses xGMI in the same gather, as each
    record's legal-move prefix (pack_pi: 2 B per legal move + a 2-B count) and
    is re-padded on the receiver. Returns numpy arrays on `dst` (every rank
    when dst is None) and Nones elsewhere: (records, games), or (records,
    games, pi uint16 [n, MAXM]) when pi is given."""
    fc = force_collective
    r = gather_rows(_as_rows(records, RECORD_DTYPE), dst, fc)
    g = gather_rows(_as_rows(games, GAME_DTYPE), dst, fc)
    p = None
    if pi is not None:
        maxm = pi.shape[-1] // 2
        counts, packed = pack_pi(pi)
        # int16 travels as byte pairs (gloo has no int16 collectives; RCCL moves the same bytes)
        c_all = gather_rows(counts.view(torch.uint8).reshape(-1, 2), dst, fc)
        k_all = gather_rows(packed.view(torch.uint8).reshape(-1, 2), dst, fc)
        if c_all is not None:
            p = unpack_pi(c_all.contiguous().view(torch.int16).reshape(-1),
                          k_all.contiguous().view(torch.int16).reshape(-1), maxm)
    if r is None:
        return (None, None) if pi is None else (None, None, None)
    order = record_order(r) if r.shape[0] else None
    r = (r[order] if order is not None else r).cpu().numpy()
    gms = g.cpu().numpy().reshape(-1).view(GAME_DTYPE) if g.numel() else np.zeros(0, GAME_DTYPE)
    recs = np.ascontiguousarray(r).reshape(-1).view(RECORD_DTYPE) if r.size else np.zeros(0, RECORD_DTYPE)
    gms = gms[np.argsort(gms["game_id"], kind="stable")]
    if pi is None:
        return recs, gms
    p = (p[order] if order is not None else p).cpu().numpy()
    return recs, gms, np.ascontiguousarray(p).view(np.uint16).reshape(p.shape[0], -1)


def pi_wire_bytes(pi) -> int:
    """Bytes the compact (s, pi, z) gather moves for these root visit rows (pack_pi)."""
    counts, packed = pack_pi(pi)
    return 2 * int(counts.numel()) + 2 * int(packed.numel())


def shard_ids(n_games: int, rank: int, world: int):
    """global game ids of this rank's shard: base=rank, stride=world."""
    return rank, world, len(range(rank, n_games, world))
