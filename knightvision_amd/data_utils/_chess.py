"""ctypes helpers over libkv.so's full-rules chess (include/kv.h, data
pipeline section). Host code only; squares are python-chess's (a1 = 0)."""
from __future__ import annotations

import ctypes as C

import numpy as np

from .. import _lib

PGN_RECORD_DTYPE = np.dtype([("fen", "S100"), ("san", "S12"), ("outcome", "<i4"), ("game", "<i4")])
assert PGN_RECORD_DTYPE.itemsize == C.sizeof(_lib.PgnRecord)


def pgn_records(text: bytes, cap: int = 1 << 18):
    """Yield numpy record arrays (fen, san, outcome, game) for every mainline move
    of every game in `text` (whole games per chunk; `game` counts from 0 over
    the whole text). Outcome KV_PGN_OUTCOME_NONE (-128) = the reference's None."""
    L = _lib.lib()
    buf = np.zeros(cap, dtype=PGN_RECORD_DTYPE)
    pos, game_base = 0, 0
    n = C.c_size_t()
    used = C.c_size_t()
    games = C.c_int64()
    while pos < len(text):
        chunk = text[pos:]
        rc = L.kv_pgn_extract(chunk, len(chunk), buf.ctypes.data_as(C.POINTER(_lib.PgnRecord)), cap, C.byref(n),
                              C.byref(used), C.byref(games))
        if rc == -4:  # KV_EOVERFLOW: one game longer than the buffer
            cap = max(2 * cap, int(n.value) + 1)
            buf = np.zeros(cap, dtype=PGN_RECORD_DTYPE)
            continue
        _lib.check(rc, "kv_pgn_extract")
        if n.value:
            out = buf[:n.value].copy()
            out["game"] += game_base
            yield out
        game_base += int(games.value)
        if used.value == 0:
            break
        pos += int(used.value)


def _fixed(strings, width):
    a = np.zeros(len(strings), dtype=f"S{width}")
    for i, s in enumerate(strings):
        b = s.encode() if isinstance(s, str) else bytes(s)
        if len(b) >= width:
            raise ValueError(f"string longer than {width - 1} bytes: {b[:40]!r}")
        a[i] = b
    return a


def fen_codes(fens) -> np.ndarray:
    """FEN strings -> int8 [N,64] codes (1..12 = P N B R Q K p n b r q k, row 0 = rank 8)."""
    fa = fens if isinstance(fens, np.ndarray) and fens.dtype.kind == "S" else _fixed(list(fens), 100)
    out = np.zeros((len(fa), 64), dtype=np.int8)
    if len(fa):
        _lib.check(_lib.lib().kv_fen_codes(fa.tobytes(), fa.dtype.itemsize, len(fa),
                                           out.ctypes.data_as(C.POINTER(C.c_int8))), "kv_fen_codes")
    return out


def san_move_index(fens, sans) -> np.ndarray:
    """board.parse_san(san) -> from_square*64 + to_square, per (fen, san) pair."""
    fa = _fixed(list(fens), 100)
    sa = _fixed(list(sans), 16)
    out = np.zeros(len(fa), dtype=np.int32)
    if len(fa):
        _lib.check(_lib.lib().kv_san_move_index(fa.tobytes(), 100, sa.tobytes(), 16, len(fa),
                                                out.ctypes.data_as(C.POINTER(C.c_int32))), "kv_san_move_index")
    return out


def perft(fen: str, depth: int) -> int:
    n = C.c_uint64()
    _lib.check(_lib.lib().kv_chess_perft(fen.encode(), depth, C.byref(n)), "kv_chess_perft")
    return int(n.value)


def san_push(fen: str, san: str) -> tuple[str, str]:
    """(board.san(board.parse_san(san)), board.fen() after the push)."""
    so = C.create_string_buffer(16)
    fo = C.create_string_buffer(100)
    _lib.check(_lib.lib().kv_chess_san(fen.encode(), san.encode(), so, 16, fo, 100), "kv_chess_san")
    return so.value.decode(), fo.value.decode()


def normalize_fen(fen: str) -> str:
    """chess.Board(fen).fen()."""
    fo = C.create_string_buffer(100)
    _lib.check(_lib.lib().kv_chess_fen(fen.encode(), fo, 100), "kv_chess_fen")
    return fo.value.decode()
