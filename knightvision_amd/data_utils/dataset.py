"""JSONL dataset of (FEN, SAN, outcome) records: the reference's
data_utils/dataset.py ChessDataset and create_dataloaders (:29-120), with
fen_to_tensor's board scan done natively (kv_fen_codes, csrc/kv_chess.cpp).

Same semantics as the reference:
  * records in file order, at most max_games lines; a relative path is taken
    under BASE_DIR;
  * move_to_idx / idx_to_move: SAN strings numbered in first-seen order
    (shared with a caller-supplied move_to_idx);
  * sample = (board tensor fp32 [12,8,8], move index, outcome) with planes
    P N B R Q K p n b r q k and row 0 = rank 8 (fen_to_tensor, :59-68), outcome
    = record.get("outcome", 0.0) unchanged (None stays None);
  * extend(games) appends dict records (:76-91).
Storage is 64 int8 board codes per sample instead of a 3 KB tensor;
`board_planes(device)` expands all samples at once on a device (one one-hot
launch on the GPU) for a training loop that batches on the device.
"""
from __future__ import annotations

import json
import logging
import os

import numpy as np
import torch
from torch.utils.data import DataLoader, Dataset

from . import _chess

logger = logging.getLogger(__name__)

BASE_DIR = os.path.abspath(os.path.join(os.path.dirname(__file__), "..", ".."))

PIECE_TO_IDX = {
    "P": 0, "N": 1, "B": 2, "R": 3, "Q": 4, "K": 5,
    "p": 6, "n": 7, "b": 8, "r": 9, "q": 10, "k": 11,
}


def codes_to_tensor(codes: np.ndarray) -> torch.Tensor:
    """int8 [64] or [N,64] codes (1..12 = plane + 1) -> fp32 [12,8,8] / [N,12,8,8]."""
    c = torch.from_numpy(np.ascontiguousarray(codes)).long()
    single = c.dim() == 1
    c = c.view(-1, 64)
    planes = torch.nn.functional.one_hot(c, 13)[..., 1:].permute(0, 2, 1).reshape(-1, 12, 8, 8).float()
    return planes[0] if single else planes


class ChessDataset(Dataset):
    def __init__(self, jsonl_path, move_to_idx=None, max_games=None):
        self.move_to_idx = move_to_idx or {}
        self.idx_to_move = {}
        self._codes = []  # int8 [k,64] blocks
        self._moves = []
        self._outcomes = []
        jsonl_path = os.path.join(BASE_DIR, jsonl_path) if not os.path.isabs(jsonl_path) else jsonl_path
        try:
            fens = []
            with open(jsonl_path, "r") as f:
                for i, line in enumerate(f):
                    if max_games and i >= max_games:
                        break
                    game = json.loads(line)
                    fen, move = game["fen"], game["move"]
                    outcome = game.get("outcome", 0.0)
                    self._add_move(move)
                    fens.append(fen)
                    self._moves.append(self.move_to_idx[move])
                    self._outcomes.append(outcome)
            self._codes.append(_chess.fen_codes(fens))
            logger.info("[DATASET] Loaded %s samples from %s", len(self), jsonl_path)
            logger.info("[DATASET] Unique moves encoded: %s", len(self.move_to_idx))
        except (IOError, json.JSONDecodeError) as e:
            logger.error("[ERROR] Failed to load dataset from %s: %s", jsonl_path, e)
            raise

    def _add_move(self, move):
        if move not in self.move_to_idx:
            idx = len(self.move_to_idx)
            self.move_to_idx[move] = idx
            self.idx_to_move[idx] = move

    @property
    def codes(self) -> np.ndarray:
        if len(self._codes) != 1:
            self._codes = [np.concatenate(self._codes) if self._codes else np.zeros((0, 64), np.int8)]
        return self._codes[0]

    def fen_to_tensor(self, fen):
        return codes_to_tensor(_chess.fen_codes([fen])[0])

    def __len__(self):
        return len(self._moves)

    def __getitem__(self, idx):
        if idx < 0:
            idx += len(self)
        if not 0 <= idx < len(self):
            raise IndexError(idx)
        return codes_to_tensor(self.codes[idx]), self._moves[idx], self._outcomes[idx]

    def extend(self, games):
        """Append dict records {'fen', 'move', 'outcome'} (dataset.py:76-91)."""
        fens = []
        for game in games:
            move = game["move"]
            self._add_move(move)
            fens.append(game["fen"])
            self._moves.append(self.move_to_idx[move])
            self._outcomes.append(game.get("outcome", 0.0))
        if fens:
            self._codes.append(_chess.fen_codes(fens))

    def board_planes(self, device) -> torch.Tensor:
        """All samples' planes [N,12,8,8] fp32, expanded on `device`."""
        from ..train import codes_to_planes_t
        return codes_to_planes_t(torch.from_numpy(self.codes).to(device))


def create_dataloaders(jsonl_path, batch_size=64, val_split=0.1, max_games=None, num_workers=os.cpu_count(),
                       pin_memory=torch.cuda.is_available(), seed: int = 42):
    """random_split with a seeded generator, then train / val DataLoaders
    (dataset.py:94-118)."""
    dataset = ChessDataset(jsonl_path, max_games=max_games)
    val_size = int(len(dataset) * val_split)
    train_size = len(dataset) - val_size
    generator = torch.Generator().manual_seed(seed)
    train_ds, val_ds = torch.utils.data.random_split(dataset, [train_size, val_size], generator=generator)
    train_loader = DataLoader(train_ds, batch_size=batch_size, shuffle=True, num_workers=num_workers,
                              pin_memory=pin_memory)
    val_loader = DataLoader(val_ds, batch_size=batch_size, num_workers=num_workers, pin_memory=pin_memory)
    return train_loader, val_loader, dataset.move_to_idx
