"""Generate tests/golden/gamestate.json.gz by driving the REFERENCE GameState
(core/chessEngine.py) through seeded trajectories of getValidMoves / makeMove /
undoMove, plus loadFEN positions, and recording what the reference reports
after every action (board strings, side, king locations, castle flags,
en-passant square and log length, halfMoveClock, FEN, isDraw, checkMate,
staleMate, inCheck, and the ordered valid-move list). Data only: the fixture
holds the actions taken and the reference's observable state.

    python tests/golden/make_gamestate_golden.py [/root/reference]

Same import recipe as make_golden.py.
"""
import gzip
import json
import os
import random
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
from make_golden import import_reference  # noqa: E402

FENS = [
    "r3k2r/pppq1ppp/2npbn2/4p3/2B1P3/2NP1N2/PPPQ1PPP/R3K2R w KQkq - 0 1",
    "8/8/8/3k4/8/8/3K4/8 w - - 0 1",
    "4k3/8/8/2pP4/8/8/8/4K3 w - c6 0 1",
]


def snap(gs, moves):
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


def trajectory(ce, seed, steps):
    rng = random.Random(seed)
    gs = ce.GameState()
    out = []
    for _ in range(steps):
        moves = gs.getValidMoves()
        rec = snap(gs, moves)
        if gs.moveLog and rng.random() < 0.15:
            action = -1  # undo
            gs.undoMove()
        elif moves:
            action = rng.randrange(len(moves))
            gs.makeMove(moves[action])
        else:
            rec["action"] = None
            out.append(rec)
            break
        rec["action"] = action
        out.append(rec)
    return out


def main():
    ref = sys.argv[1] if len(sys.argv) > 1 else "/root/reference"
    _, ce, _, _ = import_reference(ref)
    data = {"trajectories": [trajectory(ce, 1000 + k, 90) for k in range(8)], "fens": []}
    for fen in FENS:
        gs = ce.GameState()
        gs.loadFEN(fen)
        moves = gs.getValidMoves()
        data["fens"].append({"fen": fen, "after": snap(gs, moves)})
    with gzip.open(os.path.join(HERE, "gamestate.json.gz"), "wt") as f:
        json.dump(data, f, separators=(",", ":"))
    print("trajectories", [len(t) for t in data["trajectories"]])


if __name__ == "__main__":
    main()
