"""Drop-in for core/chessEngine.py's public surface: GameState,
Move and CastleRights with the reference's attribute names and methods
(getValidMoves, inCheck, squareUnderAttack, makeMove, undoMove, isDraw,
getFEN, loadFEN, checkForEndConditions), for the GUI / evaluation callers
(play_vs_model.py, chessMain.py).

The rules run in libkv.so: getValidMoves is the device generator the
self-play engine uses (kv_dev_valid_moves -> wave_valid_moves, every quirk of
chessEngine.py:277-630, including the board write of the stale-king probe),
inCheck / squareUnderAttack the device attack set (kv_dev_attacks). There is
no host rules engine: without the HIP library these raise. The move log and
its bookkeeping (makeMove :127-197, undoMove :199-274, getFEN :654-680,
loadFEN :84-122, isDraw :21-33) are host-side list edits, reproduced with the
reference's quirks: the en-passant log is pushed twice per move and popped
twice per undo, halfMoveClock resets only on captures (its pawn test compares
'P'), the repetition counters are never decremented, loadFEN writes pawns as
'wP'/'bP' and leaves the king locations alone.

Not reproduced: a loadFEN board's 'wP'/'bP' pawns are generated as pawns by
the device (the reference's own pawn logic skips some 'P' cases: pawn checks,
promotion, en passant); positions reached by play use 'wp'/'bp' throughout.
"""
from __future__ import annotations

import ctypes as C
import logging
from typing import List

import numpy as np

from . import _lib

logger = logging.getLogger(__name__)

_CODE = {"--": 0, "wK": 1, "wQ": 2, "wR": 3, "wB": 4, "wN": 5, "wp": 6, "wP": 6,
         "bK": 7, "bQ": 8, "bR": 9, "bB": 10, "bN": 11, "bp": 12, "bP": 12}
_NAME = ["--", "wK", "wQ", "wR", "wB", "wN", "wp", "bK", "bQ", "bR", "bB", "bN", "bp"]
_MF_EP, _MF_CASTLE = 1, 2
DEVICE = 0  # GPU the rules run on


class CastleRights:
    def __init__(self, wks, wqs, bks, bqs):
        self.wks = wks
        self.wqs = wqs
        self.bks = bks
        self.bqs = bqs


class Move:
    """chessEngine.py:686-735: squares are (row, col), row 0 = rank 8."""
    ranksToRows = {"1": 7, "2": 6, "3": 5, "4": 4, "5": 3, "6": 2, "7": 1, "8": 0}
    rowsToRanks = {v: k for k, v in ranksToRows.items()}
    filesToCols = {"a": 0, "b": 1, "c": 2, "d": 3, "e": 4, "f": 5, "g": 6, "h": 7}
    colsToFiles = {v: k for k, v in filesToCols.items()}

    def __init__(self, startSq, endSq, board, isCastleMove=False, isEnPassantMove=False):
        self.startRow, self.startCol = startSq
        self.endRow, self.endCol = endSq
        self.pieceMoved = board[self.startRow][self.startCol]
        self.pieceCaptured = board[self.endRow][self.endCol]
        self.isEnPassantMove = isEnPassantMove
        self.enPassantPossible = ()
        if isEnPassantMove:
            self.pieceCaptured = "bp" if self.pieceMoved == "wp" else "wp"
        self.isPawnPromotion = self.pieceMoved[1] == "p" and (
            (self.pieceMoved[0] == "w" and self.endRow == 0) or (self.pieceMoved[0] == "b" and self.endRow == 7))
        self.moveID = self.startRow * 1000 + self.startCol * 100 + self.endRow * 10 + self.endCol
        self.promotionChoice = "Q"
        self.isCastleMove = isCastleMove

    def __eq__(self, other):
        if not isinstance(other, Move):
            return False
        return (self.startRow, self.startCol, self.endRow, self.endCol, self.pieceMoved, self.isEnPassantMove) == \
            (other.startRow, other.startCol, other.endRow, other.endCol, other.pieceMoved, other.isEnPassantMove)

    __hash__ = None

    def getChessNotation(self):
        return self.getRankFile(self.startRow, self.startCol) + self.getRankFile(self.endRow, self.endCol)

    def getRankFile(self, r, c):
        return self.colsToFiles[c] + self.rowsToRanks[r]

    def __repr__(self):
        return f"Move({self.getChessNotation()})"


def _initial_board():
    back = ["R", "N", "B", "Q", "K", "B", "N", "R"]
    return [["b" + p for p in back], ["bp"] * 8] + [["--"] * 8 for _ in range(4)] + \
        [["wp"] * 8, ["w" + p for p in back]]


class GameState:
    def __init__(self):
        self.board = _initial_board()
        self.whiteToMove = True
        self.moveLog = []
        self.whiteKingLocation = (7, 4)
        self.blackKingLocation = (0, 4)
        self.insideSquareUnderAttack = False
        self.checkMate = False
        self.staleMate = False
        self.wKingMoved = False
        self.bKingMoved = False
        self.wRookKingsideMoved = False
        self.wRookQueensideMoved = False
        self.bRookKingsideMoved = False
        self.bRookQueensideMoved = False
        self.enPassantPossible = ()
        self.enPassantPossibleLog = []
        self.moveLogHistory = []
        self.boardHistory = {}
        self.halfMoveClock = 0
        self.boardStateCounter = {}
        self.draw50 = False
        self.drawRepetition = False
        self.positionCounts = {}

    # ------------------------------------------------------------ device --
    def _state(self) -> np.ndarray:
        """The 80-byte state the device rules read (include/kv.h)."""
        v = np.zeros(80, dtype=np.int8)
        v[:64] = [_CODE[sq] for row in self.board for sq in row]
        v[64] = 1 if self.whiteToMove else 0
        v[65:69] = (*self.whiteKingLocation, *self.blackKingLocation)
        v[69:75] = (self.wKingMoved, self.bKingMoved, self.wRookKingsideMoved, self.wRookQueensideMoved,
                     self.bRookKingsideMoved, self.bRookQueensideMoved)
        v[75:77] = self.enPassantPossible if self.enPassantPossible else (-1, -1)
        return v

    def _device_moves(self):
        L = _lib.lib()
        st = self._state()
        cap = 320
        mv = np.zeros(cap, dtype=np.uint16)
        nm = np.zeros(1, dtype=np.int32)
        after = np.zeros(80, dtype=np.int8)
        chk = np.zeros(1, dtype=np.uint8)
        p = lambda a, t: a.ctypes.data_as(C.POINTER(t))
        _lib.check(L.kv_dev_valid_moves(DEVICE, p(st, C.c_int8), 1, p(mv, C.c_uint16), cap, p(nm, C.c_int),
                                        p(after, C.c_int8), p(chk, C.c_uint8)), "kv_dev_valid_moves")
        if nm[0] < 0:
            raise _lib.KVError("move list overflow")
        return mv[:nm[0]], after, bool(chk[0])

    def _attacked(self) -> int:
        L = _lib.lib()
        st = self._state()
        out = np.zeros(1, dtype=np.uint64)
        _lib.check(L.kv_dev_attacks(DEVICE, st.ctypes.data_as(C.POINTER(C.c_int8)), 1,
                                    out.ctypes.data_as(C.POINTER(C.c_uint64))), "kv_dev_attacks")
        return int(out[0])

    # -------------------------------------------------------------- rules --
    def getValidMoves(self) -> List[Move]:
        """chessEngine.py:277-321 on the device; the board write the reference's
        king probe can leave (stale king location) is applied to self.board."""
        words, after, in_check = self._device_moves()
        for s in range(64):  # only the probe's king write can differ
            name = _NAME[after[s]]
            if _CODE[self.board[s // 8][s % 8]] != after[s]:
                self.board[s // 8][s % 8] = name
        moves = []
        for w in words:
            w = int(w)
            fr, to, fl = w & 63, (w >> 6) & 63, w >> 12
            moves.append(Move((fr // 8, fr % 8), (to // 8, to % 8), self.board,
                              isCastleMove=bool(fl & _MF_CASTLE), isEnPassantMove=bool(fl & _MF_EP)))
        self.checkMate, self.staleMate, self.draw50, self.drawRepetition = \
            self._end_conditions(moves, in_check)
        return moves

    def squareUnderAttack(self, r, c):
        return bool((self._attacked() >> (r * 8 + c)) & 1)

    def inCheck(self):
        r, c = self.whiteKingLocation if self.whiteToMove else self.blackKingLocation
        return self.squareUnderAttack(r, c)

    def _end_conditions(self, moves, in_check):
        if len(moves) == 0:
            return (True, False, False, False) if in_check else (False, True, False, False)
        if self.halfMoveClock >= 100:
            return False, False, True, False
        if self.positionCounts.get(self.getFEN(), 0) >= 3:
            return False, False, False, True
        return False, False, False, False

    def checkForEndConditions(self, moves):
        """chessEngine.py:632-652: (checkmate, stalemate, draw50, drawRepetition)."""
        return self._end_conditions(moves, self.inCheck() if len(moves) == 0 else False)

    def isDraw(self):
        """GameState.isDraw (:21-33): the 50-move branch needs a logged move with
        pieceMoved == pieceCaptured == '--' (never true), then kings only."""
        if self.moveLog and self.moveLog[-1].pieceMoved == self.moveLog[-1].pieceCaptured == "--":
            if len(self.moveLog) >= 100:
                return True
        return {sq for row in self.board for sq in row if sq != "--"} <= {"wK", "bK"}

    # ---------------------------------------------------------- move log --
    def _rook_flag(self, piece, r, c):
        if piece == "wR" and r == 7:
            return {0: "wRookQueensideMoved", 7: "wRookKingsideMoved"}.get(c)
        if piece == "bR" and r == 0:
            return {0: "bRookQueensideMoved", 7: "bRookKingsideMoved"}.get(c)
        return None

    def makeMove(self, move):
        """chessEngine.py:127-197 (bookkeeping quirks included)."""
        b = self.board
        self.enPassantPossibleLog.append(self.enPassantPossible)
        if not hasattr(self, "halfMoveClockLog"):
            self.halfMoveClockLog = []
        self.halfMoveClockLog.append(self.halfMoveClock)
        b[move.startRow][move.startCol] = "--"
        b[move.endRow][move.endCol] = move.pieceMoved
        if move.pieceMoved in ("wK", "bK"):
            setattr(self, move.pieceMoved[0] + "KingMoved", True)
        else:
            f = self._rook_flag(move.pieceMoved, move.startRow, move.startCol)
            if f:
                setattr(self, f, True)
        if move.isEnPassantMove:
            b[move.startRow][move.endCol] = "--"
        if getattr(move, "isCastleMove", False):
            row, ec = move.endRow, move.endCol
            if ec - move.startCol == 2:
                b[row][ec - 1], b[row][ec + 1] = b[row][ec + 1], "--"
            else:
                b[row][ec + 1], b[row][ec - 2] = b[row][ec - 2], "--"
        self.enPassantPossibleLog.append(self.enPassantPossible)  # pushed a second time (:167)
        if move.pieceMoved[1] == "p" and abs(move.startRow - move.endRow) == 2:
            self.enPassantPossible = ((move.startRow + move.endRow) // 2, move.startCol)
        else:
            self.enPassantPossible = ()
        self.moveLog.append(move)
        if move.pieceCaptured != "--" or move.pieceMoved[1] == "P":
            self.halfMoveClock = 0
        else:
            self.halfMoveClock += 1
        key = self.getBoardStateKey()
        self.boardStateCounter[key] = self.boardStateCounter.get(key, 0) + 1
        self.whiteToMove = not self.whiteToMove
        if move.pieceMoved == "wK":
            self.whiteKingLocation = (move.endRow, move.endCol)
        elif move.pieceMoved == "bK":
            self.blackKingLocation = (move.endRow, move.endCol)
        if move.isPawnPromotion:
            b[move.endRow][move.endCol] = move.pieceMoved[0] + move.promotionChoice
        fen = self.getFEN()
        self.positionCounts[fen] = self.positionCounts.get(fen, 0) + 1

    def undoMove(self):
        """chessEngine.py:199-274 (two en-passant pops, counters untouched)."""
        if not self.moveLog:
            return
        b = self.board
        self.enPassantPossible = self.enPassantPossibleLog.pop() if self.enPassantPossibleLog else ()
        if getattr(self, "halfMoveClockLog", None):
            self.halfMoveClock = self.halfMoveClockLog.pop()
        move = self.moveLog.pop()
        b[move.startRow][move.startCol] = move.pieceMoved
        b[move.endRow][move.endCol] = move.pieceCaptured
        if move.isEnPassantMove:
            b[move.endRow][move.endCol] = "--"
            b[move.startRow][move.startCol] = move.pieceMoved
            cap_row = move.endRow + 1 if move.pieceMoved[0] == "w" else move.endRow - 1
            b[cap_row][move.endCol] = move.pieceCaptured
        if move.pieceMoved in ("wK", "bK"):
            setattr(self, move.pieceMoved[0] + "KingMoved", False)
        else:
            f = self._rook_flag(move.pieceMoved, move.startRow, move.startCol)
            if f:
                setattr(self, f, False)
        if getattr(move, "isCastleMove", False):
            row, ec = move.endRow, move.endCol
            if ec - move.startCol == 2:
                b[row][ec + 1], b[row][ec - 1] = b[row][ec - 1], "--"
            else:
                b[row][ec - 2], b[row][ec + 1] = b[row][ec + 1], "--"
        self.whiteToMove = not self.whiteToMove
        if move.pieceMoved == "wK":
            self.whiteKingLocation = (move.startRow, move.startCol)
        elif move.pieceMoved == "bK":
            self.blackKingLocation = (move.startRow, move.startCol)
        if move.isPawnPromotion:
            b[move.startRow][move.startCol] = move.pieceMoved
            b[move.endRow][move.endCol] = move.pieceCaptured
        if move.isEnPassantMove:
            b[move.endRow][move.endCol] = "--"
            b[move.startRow][move.endCol] = move.pieceCaptured
        self.enPassantPossible = self.enPassantPossibleLog.pop() if self.enPassantPossibleLog else ()

    # --------------------------------------------------------------- FEN --
    def getFEN(self):
        """chessEngine.py:654-680: placement + side to move only."""
        rows = []
        for row in self.board:
            out, gap = "", 0
            for sq in row:
                if sq == "--":
                    gap += 1
                    continue
                if gap:
                    out += str(gap)
                    gap = 0
                out += sq[1].upper() if sq[0] == "w" else sq[1].lower()
            rows.append(out + (str(gap) if gap else ""))
        return "/".join(rows) + (" w" if self.whiteToMove else " b")

    def loadFEN(self, fen):
        """chessEngine.py:84-122: placement, side, castling into castleRights (which
        move generation ignores), en-passant square; king locations untouched."""
        placement, turn, castling, ep = fen.split()[:4]
        for r, text in enumerate(placement.split("/")):
            row = []
            for ch in text:
                if ch.isdigit():
                    row.extend(["--"] * int(ch))
                else:
                    row.append(("w" if ch.isupper() else "b") + ch.upper())
            self.board[r] = row
        self.whiteToMove = turn == "w"
        if not hasattr(self, "castleRights"):
            self.castleRights = CastleRights(False, False, False, False)
        self.castleRights.wks, self.castleRights.bks = "K" in castling, "k" in castling
        self.castleRights.wqs, self.castleRights.bqs = "Q" in castling, "q" in castling
        self.enPassantPossible = (8 - int(ep[1]), ord(ep[0]) - ord("a")) if ep != "-" else ()
        self.moveLog = []
        self.enPassantPossibleLog = []

    def getBoardStateKey(self):
        return str(self.board) + str(self.whiteToMove)
