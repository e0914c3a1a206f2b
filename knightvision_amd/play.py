"""Inference-only move choice for the GUI / evaluation callers (SURVEY.md 8f
rank 3): play_vs_model.get_ai_move (scripts/play_vs_model.py:34-49) and the
masked argmax of stockfish_play.py:64-84, on the HIP network (batch 1, the
split-K small-batch class) and the device rules.
"""
from __future__ import annotations

import numpy as np
import torch

from .ai import encode_board, encode_move


def get_ai_move(gs, model):
    """Greedy move of play_vs_model.get_ai_move: softmax of the policy row,
    the legal entries in list order, normalised; the first maximum wins, the
    first move when every legal probability is 0."""
    valid = gs.getValidMoves()
    x = torch.tensor(np.asarray([encode_board(gs.board)], dtype=np.float32))
    with torch.no_grad():
        logits, _ = model(x)
    policy = torch.softmax(logits.squeeze(), dim=0).cpu().numpy()
    legal = [policy[encode_move(m.startRow, m.startCol, m.endRow, m.endCol)] for m in valid]
    total = sum(legal)
    if total == 0:
        return valid[0]
    norm = [w / total for w in legal]
    return valid[norm.index(max(norm))]


def masked_argmax_move(logits: torch.Tensor, legal_indices) -> int:
    """stockfish_play.py:64-84: argmax of the logits restricted to the legal
    move indices (encode_move), -1 when there are none."""
    if len(legal_indices) == 0:
        return -1
    row = logits.reshape(-1)
    mask = torch.full_like(row, float("-inf"))
    idx = torch.as_tensor(list(legal_indices), device=row.device, dtype=torch.long)
    mask[idx] = 0.0
    return int(torch.argmax(row + mask).item())
