"""knightvision_amd.chess_engine (the core/chessEngine.py drop-in: device move
generation + host move log) replayed against the reference GameState's own
trajectories (tests/golden/gamestate.json.gz, made by
make_gamestate_golden.py): after every getValidMoves / makeMove / undoMove the
board, side, king locations, castle flags, en-passant square and log,
halfMoveClock, FEN, isDraw, checkMate / staleMate, inCheck and the ordered
move list (with pieceMoved / pieceCaptured / flags) must equal the reference's.
Plus play.get_ai_move on the HIP network against the same choice computed
from the torch fp32 restatement."""
import gzip
import json
import os

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def _snap(gs, moves):
    return {
        "board": [sq for row in gs.board for sq in row],
        "wtm": gs.whiteToMove,
        "wk": list(gs.whiteKingLocation), "bk": list(gs.blackKingLocation),
        "flags": [gs.wKingMoved, gs.bKingMoved, gs.wRookKingsideMoved, gs.wRookQueensideMoved,
                  gs.bRookKingsideMoved, gs.bRookQueensideMoved],
        "ep": list(gs.enPassantPossible), "eplog": len(gs.enPassantPossibleLog),
        "hmc": gs.halfMoveClock, "fen": gs.getFEN(), "draw": gs.isDraw(),
        "mate": gs.checkMate, "stale": gs.staleMate, "check": gs.inCheck(),
        "moves": [[m.getChessNotation(), m.pieceMoved, m.pieceCaptured, bool(m.isEnPassantMove),
                   bool(m.isCastleMove), bool(m.isPawnPromotion)] for m in moves],
    }


def _golden(golden_dir):
    with gzip.open(os.path.join(golden_dir, "gamestate.json.gz"), "rt") as f:
        return json.load(f)


def test_gamestate_trajectories_match_reference(golden_dir):
    from knightvision_amd.chess_engine import GameState
    g = _golden(golden_dir)
    steps = 0
    for t, traj in enumerate(g["trajectories"]):
        gs = GameState()
        for k, want in enumerate(traj):
            moves = gs.getValidMoves()
            got = _snap(gs, moves)
            for key in want:
                if key == "action":
                    continue
                assert got[key] == want[key], (t, k, key, got[key], want[key])
            a = want["action"]
            if a is None:
                break
            if a < 0:
                gs.undoMove()
            else:
                gs.makeMove(moves[a])
            steps += 1
    assert steps > 600


def test_loadfen_fields_match_reference(golden_dir):
    from knightvision_amd.chess_engine import GameState
    for case in _golden(golden_dir)["fens"]:
        gs = GameState()
        gs.loadFEN(case["fen"])
        moves = gs.getValidMoves()
        got, want = _snap(gs, moves), case["after"]
        for key in ("board", "wtm", "wk", "bk", "ep", "eplog", "fen"):
            assert got[key] == want[key], (case["fen"], key)
        if not any(sq[1] == "P" for sq in want["board"] if sq != "--"):
            # loadFEN writes 'wP'/'bP'; the device treats them as pawns throughout (documented), so the
            # move lists are compared on pawn-free positions only
            assert got["moves"] == want["moves"]


def test_get_ai_move_matches_torch_choice():
    from knightvision_amd.ai import encode_board, encode_move
    from knightvision_amd.chess_engine import GameState
    from knightvision_amd.model import ChessNet
    from knightvision_amd.play import get_ai_move
    from knightvision_amd.weights import synthetic_state_dict
    from oracle import torch_ref
    sd = synthetic_state_dict(42, "peaked")
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m.eval()
    gs = GameState()
    for ply in range(12):
        mv = get_ai_move(gs, m)
        valid = gs.getValidMoves()
        logits, _ = torch_ref.forward(sd, np.asarray([encode_board(gs.board)], dtype=np.float32))
        pol = torch.softmax(logits.squeeze(), dim=0).numpy()
        legal = np.array([pol[encode_move(x.startRow, x.startCol, x.endRow, x.endCol)] for x in valid])
        order = np.argsort(-legal, kind="stable")
        # same choice unless the top two are within the logit tolerance's effect on probabilities
        if legal[order[0]] - legal[order[1]] > 1e-6:
            assert mv == valid[order[0]], ply
        gs.makeMove(mv)
