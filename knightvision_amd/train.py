"""Policy/value update step of the learn loop on MI355X:
the per-batch math of scripts/train.py _train_one_epoch (:126-196) and
evaluate (:109-124), data-parallel over RCCL with DistributedDataParallel (one
process per GPU; the reference wraps nn.DataParallel, ai/model_utils.py:26-28).

Per batch, as the reference:
  * forward under torch.cuda.amp.autocast (:161-162), losses in fp32:
    loss_policy = cross_entropy(policy, move) (:169), loss_value =
    mse(value.squeeze(), outcome) (:171), entropy of softmax(policy) (:173-175),
    loss = loss_policy + loss_value - ENTROPY_COEF * entropy (:176);
  * NaN / Inf loss -> batch skipped (:178-180);
  * loss / accumulate_steps, GradScaler backward (:183-184); every
    accumulate_steps batches or at the last one: unscale, clip_grad_norm 1.0,
    scaler.step, scaler.update, zero_grad (:187-192).
Defaults follow the reference's environment variables: BATCH_SIZE 4096,
ACCUM_STEPS 2, LR 5e-4 (train.py:17-20), ENTROPY_COEF 0.01 (:461).

Data bridge: the engine's records (int8 board codes,
encode_move index, per-game reward) are expanded to the (12,8,8) planes of
encode_board (ai/ai.py:17-30) on the device; self-play keeps the reference's
plane order (K,Q,R,B,N,p) and move indexing (row 0 = rank 8), which differ from
the PGN dataset's (train.py:542-545, :553-558) exactly as in the reference.
"""
from __future__ import annotations

import json
import math
import os
from dataclasses import dataclass

# MIOpen's default find mode benchmarks every new convolution shape for tens of
# seconds (measured 15-47 s per shape on MI355X); the update step sees a new
# last-batch shape every iteration, so use the fast heuristic selection unless
# the caller chose otherwise. Must be set before the first convolution runs.
os.environ.setdefault("MIOPEN_FIND_MODE", "FAST")

import numpy as np
import torch
import torch.nn.functional as F

BATCH_SIZE = int(os.getenv("BATCH_SIZE", "4096"))
ACCUM_STEPS = int(os.getenv("ACCUM_STEPS", "2"))
LR = float(os.getenv("LR", "5e-4"))
ENTROPY_COEF = float(os.getenv("ENTROPY_COEF", "0.01"))
CLIP_NORM = 1.0


def codes_to_planes_t(codes: torch.Tensor) -> torch.Tensor:
    """int8 board codes [N,64] (0 empty, 1..12 = wK..bp) -> fp32 planes [N,12,8,8]
    in encode_board's channel order (ai/ai.py:7-10, :17-30), on codes' device."""
    c = codes.long()
    planes = F.one_hot(c, 13)[..., 1:]  # [N,64,12]
    return planes.permute(0, 2, 1).reshape(-1, 12, 8, 8).to(torch.float32).contiguous()


@dataclass
class Batch:
    boards: torch.Tensor    # [B,12,8,8] fp32
    moves: torch.Tensor     # [B] int64
    outcomes: torch.Tensor  # [B] fp32


def records_to_tensors(records: np.ndarray, games: np.ndarray, device) -> tuple:
    """Engine records + finished-game table -> (codes int8 [N,64], moves int64 [N],
    rewards fp32 [N]) on `device`; every record of a game carries that game's
    reward (self_play.py:245-253)."""
    reward_of = {int(g["game_id"]): float(g["reward"]) for g in games}
    keep = np.array([int(r) in reward_of for r in records["game_id"]], dtype=bool)
    rec = records[keep]
    codes = torch.from_numpy(np.ascontiguousarray(rec["board"]).astype(np.int8)).to(device)
    moves = torch.from_numpy(rec["move"].astype(np.int64)).to(device)
    rew = torch.tensor([reward_of[int(g)] for g in rec["game_id"]], dtype=torch.float32, device=device)
    return codes, moves, rew


def batches(codes, moves, rewards, batch_size: int, shuffle: bool, generator: torch.Generator | None = None,
            total: int | None = None):
    """DataLoader(batch_size, shuffle) over the tensors (train.py:238-249). With
    `total` > len (data-parallel ranks holding unequal shards) the epoch order
    wraps around to `total` samples, so every rank runs the same number of
    equal batches (DistributedSampler's padding)."""
    n = codes.shape[0]
    order = torch.randperm(n, generator=generator) if shuffle else torch.arange(n)
    if total is not None and total > n:
        order = order.repeat((total + n - 1) // n)[:total]
    order = order.to(codes.device)
    for i in range(0, order.numel(), batch_size):
        ix = order[i:i + batch_size]
        yield Batch(codes_to_planes_t(codes[ix]), moves[ix], rewards[ix])


# MIOpen selects convolution solutions per input shape (≈0.85 s for each new
# batch size on MI355X, measured: tools/shape_probe.py), and the learn loop's
# last batch has a new size every iteration. On the GPU the batch is padded to a
# multiple of ROW_BUCKET rows; the padding rows are excluded from every
# BatchNorm statistic (model.batch_norm_rows) and from the loss, so the update
# is the unpadded batch's. 0 disables.
ROW_BUCKET = int(os.getenv("KV_TRAIN_ROW_BUCKET", "256"))


def _pad_rows(model, x, bucket):
    m = model.module if hasattr(model, "module") else model
    n = x.shape[0]
    if bucket <= 0 or not getattr(m, "supports_row_padding", False) or n % bucket == 0:
        return x, None
    pad = (n + bucket - 1) // bucket * bucket - n
    return torch.cat([x, x.new_zeros((pad,) + tuple(x.shape[1:]))]), n


def batch_loss(model, b: Batch, entropy_coef: float = ENTROPY_COEF, amp: bool = True, bucket: int | None = None):
    """The reference's per-batch loss (train.py:161-176): returns
    (loss, loss_policy, loss_value, entropy, policy_logits)."""
    dev_type = b.boards.device.type
    if bucket is None:
        bucket = ROW_BUCKET if dev_type == "cuda" else 0
    x, n_real = _pad_rows(model, b.boards, bucket)
    with torch.autocast(device_type=dev_type, enabled=amp and dev_type == "cuda"):
        pol, val = model(x, n_real) if n_real is not None else model(x)
    if n_real is not None:
        pol, val = pol[:n_real], val[:n_real]
    loss_policy = F.cross_entropy(pol.float(), b.moves)
    loss_value = F.mse_loss(val.squeeze().float(), b.outcomes)
    logp = F.log_softmax(pol.float(), dim=1)
    entropy = -(F.softmax(pol.float(), dim=1) * logp).sum(dim=1).mean()
    loss = loss_policy + loss_value - entropy_coef * entropy
    return loss, loss_policy, loss_value, entropy, pol


def _finite_on_all_ranks(loss: torch.Tensor, force: bool = False) -> bool:
    """isfinite(loss), agreed over the ranks of an initialised process group
    (MIN all-reduce of the flag: one rank's NaN skips the batch everywhere).
    force: run the all-reduce even at world size 1 (tests of the RCCL path)."""
    ok = torch.isfinite(loss.detach()).all()
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or force):
        dev = loss.device if dist.get_backend() == "nccl" else torch.device("cpu")
        flag = ok.to(device=dev, dtype=torch.int32).reshape(1)
        dist.all_reduce(flag, op=dist.ReduceOp.MIN)
        return bool(flag.item())
    return bool(ok)


def make_scaler(device) -> torch.amp.GradScaler:
    return torch.amp.GradScaler("cuda", enabled=torch.device(device).type == "cuda")


def train_one_epoch(model, data, optimizer, scaler, accumulate_steps: int = ACCUM_STEPS,
                    entropy_coef: float = ENTROPY_COEF, amp: bool = True, force_collective: bool = False) -> dict:
    """_train_one_epoch (train.py:126-196) over an iterable of Batch. `model` may be
    a DistributedDataParallel wrapper: gradients are averaged over the ranks by
    RCCL all-reduce during backward (bucketed, overlapped with the backward).
    force_collective: the rank-agreed NaN skip all-reduces even at world size 1."""
    data = list(data)
    n = len(data)
    model.train()
    optimizer.zero_grad()
    total, skipped, correct, seen, steps = 0.0, 0, 0, 0, 0
    for i, b in enumerate(data):
        loss, lp, lv, ent, pol = batch_loss(model, b, entropy_coef, amp)
        if not _finite_on_all_ranks(loss, force_collective):
            # the reference skips a non-finite batch (train.py:178-180); under DDP every
            # rank skips together, or the gradient all-reduces of backward would pair up
            # different batches across ranks (or hang)
            skipped += 1
            continue
        scaler.scale(loss / accumulate_steps).backward()
        if (i + 1) % accumulate_steps == 0 or i == n - 1:
            scaler.unscale_(optimizer)
            torch.nn.utils.clip_grad_norm_(model.parameters(), max_norm=CLIP_NORM)
            scaler.step(optimizer)
            scaler.update()
            optimizer.zero_grad()
            steps += 1
        total += float(loss.detach())
        correct += int((pol.detach().argmax(1) == b.moves).sum())
        seen += b.moves.numel()
    return {"loss": total, "batches": n, "skipped": skipped, "optimizer_steps": steps,
            "accuracy": correct / max(seen, 1), "samples": seen}


@torch.no_grad()
def evaluate(model, data) -> float:
    """evaluate (train.py:109-124): mean of (CE + MSE) over samples, eval-mode
    forward (the HIP tower for knightvision_amd.ChessNet)."""
    model = model.module if hasattr(model, "module") else model  # DDP wrapper: evaluate the local replica
    was = model.training
    model.eval()
    tot, cnt = 0.0, 0
    for b in data:
        pol, val = model(b.boards)
        lp = F.cross_entropy(pol.float(), b.moves)
        lv = F.mse_loss(val.squeeze().float(), b.outcomes)
        tot += float(lp + lv) * b.boards.shape[0]
        cnt += b.boards.shape[0]
    model.train(was)
    return tot / cnt if cnt else math.inf


def wrap_ddp(model, device, force: bool = False):
    """DistributedDataParallel over the default process group (RCCL on GPUs, gloo on
    CPU) when one is initialised with more than one rank (or with one, when
    `force`: the RCCL path exercised on a 1-GPU box); else the model itself."""
    import torch.distributed as dist
    if dist.is_available() and dist.is_initialized() and (dist.get_world_size() > 1 or force):
        dev = torch.device(device)
        ids = [dev.index if dev.index is not None else 0] if dev.type == "cuda" else None
        return torch.nn.parallel.DistributedDataParallel(model, device_ids=ids, bucket_cap_mb=64)
    return model


class ChessPGNDataset(torch.utils.data.Dataset):
    """The trainer's JSONL dataset (scripts/train.py:497-561), chess work native
    (kv_fen_codes / kv_san_move_index, csrc/kv_chess.cpp). As the reference:
      * indexes the byte offsets of the first max_samples lines; a sample is read
        and decoded on access; extend() appends ready samples after them;
      * board = fen_to_tensor(fen): numpy fp32 [12,8,8], planes P N B R Q K
        p n b r q k, row 0 = rank 8 (:531-545);
      * move = move_encoder(san, fen), default board.parse_san -> from*64+to in
        python-chess squares (:553-558) -- not the self-play encode_move indexing;
      * outcome from record.get("result", "1/2-1/2") (:525-532): the parser writes
        "outcome", not "result", so file samples read 0.0 -- kept as is.
    `materialize(device)` decodes every file sample at once (codes, move
    indices and outcomes as device tensors) for batched training."""

    def __init__(self, path, move_encoder=None, max_samples=10000):
        self.file_path = path
        self.move_encoder = move_encoder or self.default_move_encoder
        self.max_samples = max_samples
        self.additional_data = []
        self.line_offsets = []
        with open(self.file_path, "rb") as f:
            offset = 0
            for i, line in enumerate(f):
                if i >= self.max_samples:
                    break
                self.line_offsets.append(offset)
                offset += len(line)

    def __len__(self):
        return len(self.line_offsets) + len(self.additional_data)

    @staticmethod
    def _outcome(record):
        result = record.get("result", "1/2-1/2")
        return 1.0 if result == "1-0" else (-1.0 if result == "0-1" else 0.0)

    def __getitem__(self, idx):
        if idx >= len(self.line_offsets):
            return self.additional_data[idx - len(self.line_offsets)]
        with open(self.file_path, "rb") as f:
            f.seek(self.line_offsets[idx])
            record = json.loads(f.readline().decode().strip())
        fen = record["fen"]
        return self.fen_to_tensor(fen), self.move_encoder(record["move"], fen), self._outcome(record)

    def fen_to_tensor(self, fen):
        from .data_utils import _chess
        from .data_utils.dataset import codes_to_tensor
        return codes_to_tensor(_chess.fen_codes([fen])[0]).numpy()

    def default_move_encoder(self, move_san, fen):
        from .data_utils import _chess
        return int(_chess.san_move_index([fen], [move_san])[0])

    def extend(self, new_records):
        self.additional_data.extend(new_records)

    def materialize(self, device):
        """(codes int8 [N,64], moves int64 [N], outcomes fp32 [N]) of the file samples
        on `device` (default move encoder only)."""
        from .data_utils import _chess
        if getattr(self.move_encoder, "__func__", None) is not ChessPGNDataset.default_move_encoder:
            raise ValueError("materialize() decodes moves with the default encoder only")
        fens, sans, outs = [], [], []
        with open(self.file_path, "rb") as f:
            for i, line in enumerate(f):
                if i >= len(self.line_offsets):
                    break
                rec = json.loads(line.decode().strip())
                fens.append(rec["fen"])
                sans.append(rec["move"])
                outs.append(self._outcome(rec))
        codes = torch.from_numpy(_chess.fen_codes(fens)).to(device)
        moves = torch.from_numpy(_chess.san_move_index(fens, sans).astype(np.int64)).to(device)
        return codes, moves, torch.tensor(outs, dtype=torch.float32, device=device)
