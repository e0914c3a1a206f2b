"""Board / move encoders: drop-in for ai/ai.py (same names and semantics).

encode_board (ai/ai.py:17-41): 12 one-hot planes, channel order wK wQ wR wB wN
wp bK bQ bR bB bN bp, [c, row, col] with row 0 = rank 8. The list/ndarray input
path is the one the self-play path uses; a python-chess Board is accepted too
when python-chess is installed. encode_move / decode_move_index (ai/ai.py:43-57):
index = (sr*8+sc)*64 + (er*8+ec).
"""
from __future__ import annotations

import numpy as np

PIECE_TO_INDEX = {
    "wK": 0, "wQ": 1, "wR": 2, "wB": 3, "wN": 4, "wp": 5,
    "bK": 6, "bQ": 7, "bR": 8, "bB": 9, "bN": 10, "bp": 11,
}
INDEX_TO_PIECE = {v: k for k, v in PIECE_TO_INDEX.items()}
PIECE_CODES = ["--"] + [INDEX_TO_PIECE[i] for i in range(12)]  # code = index + 1, 0 = empty


def board_to_codes(board) -> np.ndarray:
    """8x8 list of piece strings -> int8[64] codes (0 empty, 1..12 = PIECE_TO_INDEX + 1)."""
    out = np.zeros(64, dtype=np.int8)
    for r in range(8):
        row = board[r]
        for c in range(8):
            idx = PIECE_TO_INDEX.get(row[c])
            if idx is not None:
                out[r * 8 + c] = idx + 1
    return out


def codes_to_planes(codes) -> np.ndarray:
    codes = np.asarray(codes, dtype=np.int64).reshape(-1, 64)
    planes = np.zeros((codes.shape[0], 12, 64), dtype=np.float32)
    b, s = np.nonzero(codes)
    planes[b, codes[b, s] - 1, s] = 1.0
    return planes.reshape(-1, 12, 8, 8)


def encode_board(board) -> np.ndarray:
    if isinstance(board, (list, np.ndarray)):
        arr = np.array(board)
        encoded = np.zeros((12, 8, 8), dtype=np.float32)
        for row, col in zip(*np.nonzero(arr)):
            idx = PIECE_TO_INDEX.get(arr[row, col])
            if idx is not None:
                encoded[idx, row, col] = 1.0
        return encoded
    # python-chess Board (ai/ai.py:33-39); square -> (7 - sq//8, sq%8)
    encoded = np.zeros((12, 8, 8), dtype=np.float32)
    for square, piece in board.piece_map().items():
        color = "w" if piece.color else "b"
        letter = "p" if piece.piece_type == 1 else piece.symbol().upper()
        encoded[PIECE_TO_INDEX[color + letter], 7 - square // 8, square % 8] = 1.0
    return encoded


def decode_move_index(index):
    start, end = index // 64, index % 64
    return (start // 8, start % 8, end // 8, end % 8)


def encode_move(start_row, start_col, end_row, end_col):
    return (start_row * 8 + start_col) * 64 + (end_row * 8 + end_col)


__all__ = ["encode_board", "decode_move_index", "encode_move"]
