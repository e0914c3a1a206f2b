"""Full-rules chess of the data pipeline (csrc/kv_chess.cpp, python-chess 1.999
semantics): host code in libkv.so, no GPU.

python-chess is not installed here, so nothing can be compared against it
directly: legality is pinned by the published perft node counts of the six
standard test positions (chessprogramming.org "Perft Results"), and SAN / FEN /
PGN behaviour by hand-checked positions and well-known games whose final FENs
are textbook (fool's mate, scholar's mate). Everything else is "parity
unpinned" against python-chess itself."""
import json

import numpy as np
import pytest

from knightvision_amd.data_utils import _chess

START = "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1"

PERFT = [
    (START, [20, 400, 8902, 197281]),
    ("r3k2r/p1ppqpb1/bn2pnp1/3PN3/1p2P3/2N2Q1p/PPPBBPPP/R3K2R w KQkq - 0 1", [48, 2039, 97862]),
    ("8/2p5/3p4/KP5r/1R3p1k/8/4P1P1/8 w - - 0 1", [14, 191, 2812, 43238]),
    ("r3k2r/Pppp1ppp/1b3nbN/nP6/BBP1P3/q4N2/Pp1P2PP/R2Q1RK1 w kq - 0 1", [6, 264, 9467]),
    ("rnbq1k1r/pp1Pbppp/2p5/8/2B5/8/PPP1NnPP/RNBQK2R w KQ - 1 8", [44, 1486, 62379]),
    ("r4rk1/1pp1qppp/p1np1n2/2b1p1B1/2B1P1b1/P1NP1N2/1PP1QPPP/R4RK1 w - - 0 10", [46, 2079, 89890]),
]


@pytest.mark.parametrize("fen,counts", PERFT)
def test_perft(fen, counts):
    assert [_chess.perft(fen, d + 1) for d in range(len(counts))] == counts


def test_fen_normalisation():
    # en-passant square printed only when a legal capture exists (python-chess fen(en_passant="legal"))
    assert _chess.normalize_fen("rnbqkbnr/pppppppp/8/8/4P3/8/PPPP1PPP/RNBQKBNR b KQkq e3 0 1") == \
        "rnbqkbnr/pppppppp/8/8/4P3/8/PPPP1PPP/RNBQKBNR b KQkq - 0 1"
    fen = "rnbqkbnr/ppp1p1pp/8/3pPp2/8/8/PPPP1PPP/RNBQKBNR w KQkq f6 0 3"
    assert _chess.normalize_fen(fen) == fen
    # castling rights cleaned to rooks on their corners
    assert _chess.normalize_fen("r3k2r/8/8/8/8/8/8/R3K3 w KQkq - 0 1") == "r3k2r/8/8/8/8/8/8/R3K3 w Qkq - 0 1"
    # missing fields take python-chess's defaults
    assert _chess.normalize_fen("8/8/8/8/8/8/8/K6k") == "8/8/8/8/8/8/8/K6k w - - 0 1"


def test_san_and_push():
    assert _chess.san_push(START, "e4") == ("e4", "rnbqkbnr/pppppppp/8/8/4P3/8/PPPP1PPP/RNBQKBNR b KQkq - 0 1")
    assert _chess.san_push(START, "Ng1-f3")[0] == "Nf3"       # over-specified input, canonical output
    assert _chess.san_push(START, "g1f3")[0] == "Nf3"         # fully specified from-square
    # en passant: SAN with the from-file and "x", captured pawn removed
    san, after = _chess.san_push("rnbqkbnr/ppp1p1pp/8/3pPp2/8/8/PPPP1PPP/RNBQKBNR w KQkq f6 0 3", "exf6")
    assert san == "exf6" and after == "rnbqkbnr/ppp1p1pp/5P2/3p4/8/8/PPPP1PPP/RNBQKBNR b KQkq - 0 3"
    # disambiguation: file when the files differ, rank when the file is shared, both when needed
    two_files = "4k3/8/8/8/8/8/8/1N2KN2 w - - 0 1"
    assert _chess.san_push(two_files, "Nbd2")[0] == "Nbd2"
    assert _chess.san_push(two_files, "Nfd2")[0] == "Nfd2"
    with pytest.raises(Exception, match="ambiguous"):
        _chess.san_push(two_files, "Nd2")
    one_file = "4k3/8/8/8/8/1N6/8/1N2K3 w - - 0 1"
    assert _chess.san_push(one_file, "Nb1d2")[0] == "N1d2"
    assert _chess.san_push(one_file, "N3d2")[0] == "N3d2"
    three = "4k3/8/8/8/8/1N6/8/1N2KN2 w - - 0 1"
    assert _chess.san_push(three, "Nb1d2")[0] == "Nb1d2"
    # promotion spellings, check and mate suffixes
    promo = "8/4P3/8/8/8/8/k7/4K3 w - - 0 1"
    assert _chess.san_push(promo, "e8=Q")[0] == "e8=Q"
    assert _chess.san_push(promo, "e8Q")[0] == "e8=Q"
    assert _chess.san_push(promo, "e8=N")[0] == "e8=N"
    with pytest.raises(Exception, match="missing promotion"):
        _chess.san_push(promo, "e7e8")
    assert _chess.san_push("4k3/8/8/8/8/8/8/R3K3 w Q - 0 1", "Ra8")[0] == "Ra8+"
    assert _chess.san_push("4k3/8/8/8/8/8/8/R3K3 w Q - 0 1", "O-O-O")[0] == "O-O-O"
    assert _chess.san_push("4k3/8/8/8/8/8/8/R3K3 w Q - 0 1", "0-0-0")[0] == "O-O-O"
    assert _chess.san_push("4k3/8/8/8/8/8/8/4K2R w K - 0 1", "e1h1")[0] == "O-O"  # king-takes-rook spelling
    fool = ["f3", "e5", "g4", "Qh4"]
    fen = START
    for s in fool:
        out, fen = _chess.san_push(fen, s)
    assert out == "Qh4#" and fen == "rnb1kbnr/pppp1ppp/8/4p3/6Pq/5P2/PPPPP2P/RNBQKBNR w KQkq - 1 3"
    with pytest.raises(Exception, match="illegal"):
        _chess.san_push(START, "e5")
    with pytest.raises(Exception, match="invalid"):
        _chess.san_push(START, "Zz9")
    with pytest.raises(Exception, match="illegal"):
        _chess.san_push(START, "O-O")


PGN = """[Event "Scholar"]
[Site "?"]
[Result "1-0"]

1. e4 e5 2. Qh5 {attacking f7} Nc6 (2... g6 3. Qf3) 3. Bc4 $1 Nf6?? 4. Qxf7# 1-0

[Event "Fool"]
[Result "*"]

1.f3 e5 2.g4 ; a comment to the end of the line
Qh4# 0-1

[Event "Illegal"]
[Result "1/2-1/2"]

1. d4 d5 2. Ke3 Nf6 1/2-1/2

[Event "FromFen"]
[FEN "4k3/8/8/8/8/8/8/R3K3 w Q - 0 1"]
[SetUp "1"]

1. O-O-O+ Kf7 { multi
line comment } 2. Rd7+ *

"""


def _records(text):
    out = []
    for arr in _chess.pgn_records(text.encode()):
        for r in arr:
            out.append((r["fen"].decode(), r["san"].decode(), int(r["outcome"]), int(r["game"])))
    return out


def test_pgn_records():
    recs = _records(PGN)
    games = [[r for r in recs if r[3] == g] for g in range(4)]
    assert [r[1] for r in games[0]] == ["e4", "e5", "Qh5", "Nc6", "Bc4", "Nf6", "Qxf7#"]
    assert all(r[2] == 1 for r in games[0])
    assert games[0][-1][0] == "r1bqkb1r/pppp1ppp/2n2n2/4p2Q/2B1P3/8/PPPP1PPP/RNB1K1NR w KQkq - 4 4"
    _, after = _chess.san_push(games[0][-1][0], "Qxf7")
    assert after == "r1bqkb1r/pppp1Qpp/2n2n2/4p3/2B1P3/8/PPPP1PPP/RNB1K1NR b KQkq - 0 4"
    # a "*" Result header takes the movetext result
    assert [r[1] for r in games[1]] == ["f3", "e5", "g4", "Qh4#"] and all(r[2] == -1 for r in games[1])
    # the first illegal mainline move ends the game's records (chess.pgn error handling)
    assert [r[1] for r in games[2]] == ["d4", "d5"] and all(r[2] == 0 for r in games[2])
    # FEN tag start position; outcome None ("*")
    assert [r[1] for r in games[3]] == ["O-O-O", "Kf7", "Rd7+"]  # the "+" in the movetext was wrong: dropped
    assert games[3][0][0] == "4k3/8/8/8/8/8/8/R3K3 w Q - 0 1"
    assert all(r[2] == -128 for r in games[3])


def test_pgn_chunked_cap():
    # a tiny record buffer forces several native calls over whole games
    text = PGN * 3
    recs = []
    for arr in _chess.pgn_records(text.encode(), cap=8):
        recs += [(r["san"].decode(), int(r["game"])) for r in arr]
    assert len(recs) == 3 * len(_records(PGN))
    assert max(g for _, g in recs) == 11


def test_parser_module(tmp_path, monkeypatch):
    from knightvision_amd.data_utils import parser_pgn
    monkeypatch.setattr(parser_pgn, "ZST_LOG", str(tmp_path / "zst.log"))
    monkeypatch.setattr(parser_pgn, "PARSED_LOG", str(tmp_path / "parsed.log"))
    pgn_dir = tmp_path / "pgn"
    pgn_dir.mkdir()
    (pgn_dir / "a.pgn").write_text(PGN)
    recs = list(parser_pgn.extract_data_from_pgn(str(pgn_dir / "a.pgn")))
    assert recs[0] == {"fen": "rnbqkbnr/pppppppp/8/8/8/8/PPPPPPPP/RNBQKBNR w KQkq - 0 1", "move": "e4", "outcome": 1}
    assert recs[-1]["outcome"] is None
    out = tmp_path / "games.jsonl"
    parser_pgn.parse_all_games(str(pgn_dir), str(out))
    lines = out.read_text().splitlines()
    assert lines[0] == json.dumps(recs[0]) and len(lines) == len(recs)
    parser_pgn.parse_all_games(str(pgn_dir), str(out))  # already in PARSED_LOG: nothing appended
    assert len(out.read_text().splitlines()) == len(recs)
    with pytest.raises(ImportError):
        next(parser_pgn.extract_data_from_pgn_zst(str(tmp_path / "x.pgn.zst")))


def _planes_by_hand(fen):
    order = "PNBRQKpnbrqk"
    t = np.zeros((12, 8, 8), np.float32)
    for r, row in enumerate(fen.split()[0].split("/")):
        c = 0
        for ch in row:
            if ch.isdigit():
                c += int(ch)
            else:
                t[order.index(ch), r, c] = 1.0
                c += 1
    return t


def test_datasets(tmp_path, monkeypatch):
    from knightvision_amd.data_utils import parser_pgn
    monkeypatch.setattr(parser_pgn, "ZST_LOG", str(tmp_path / "zst.log"))
    from knightvision_amd.data_utils.dataset import ChessDataset
    from knightvision_amd.train import ChessPGNDataset
    (tmp_path / "a.pgn").write_text(PGN)
    recs = list(parser_pgn.extract_data_from_pgn(str(tmp_path / "a.pgn")))
    path = tmp_path / "games.jsonl"
    path.write_text("".join(json.dumps(r) + "\n" for r in recs))
    ds = ChessDataset(str(path))
    assert len(ds) == len(recs)
    vocab = list(dict.fromkeys(r["move"] for r in recs))
    assert list(ds.move_to_idx) == vocab
    for i, r in enumerate(recs):
        board, mi, oc = ds[i]
        assert np.array_equal(board.numpy(), _planes_by_hand(r["fen"]))
        assert ds.idx_to_move[mi] == r["move"] and oc == r["outcome"]
    ds.extend([{"fen": START, "move": "Nf3"}])
    assert ds[len(recs)][2] == 0.0 and len(ds) == len(recs) + 1
    assert np.array_equal(ds.board_planes("cpu")[0].numpy(), _planes_by_hand(recs[0]["fen"]))
    # the trainer's dataset: python-chess square indexing and the "result"-key outcome quirk
    pds = ChessPGNDataset(str(path), max_samples=5)
    assert len(pds) == 5
    board, mi, oc = pds[0]
    assert isinstance(board, np.ndarray) and np.array_equal(board, _planes_by_hand(START))
    assert mi == 12 * 64 + 28 and oc == 0.0  # e2e4 in python-chess squares
    codes, moves, outs = pds.materialize("cpu")
    assert [int(m) for m in moves] == [pds[i][1] for i in range(5)]
    assert codes.shape == (5, 64) and float(outs.abs().sum()) == 0.0
    pds.extend([("b", 1, 1.0)])
    assert pds[5] == ("b", 1, 1.0)


def test_san_edge_cases():
    """More python-chess parse_san / san / push semantics (hand-checked positions; python-chess itself is not
    installed here, so these are pinned by the rules, not by the library)."""
    # capture-promotion giving check: the SAN carries "x", "=Q" and "+"; halfmove clock reset
    san, after = _chess.san_push("3r2k1/4P3/8/8/8/8/8/4K3 w - - 0 1", "exd8=Q")
    assert san == "exd8=Q+" and after == "3Q2k1/8/8/8/8/8/8/4K3 b - - 0 1"
    # castling through an attacked square is illegal
    with pytest.raises(Exception, match="illegal"):
        _chess.san_push("4k3/8/8/8/8/8/5r2/4K2R w K - 0 1", "O-O")
    # an en-passant capture that exposes the own king along the rank is illegal
    with pytest.raises(Exception, match="illegal"):
        _chess.san_push("8/8/8/KPp4r/8/8/8/7k w - c6 0 1", "bxc6")
    # long-algebraic pawn capture spelling, canonical SAN out; en-passant square cleared after the push
    san, after = _chess.san_push("rnbqkbnr/ppp1pppp/8/3p4/4P3/8/PPPP1PPP/RNBQKBNR w KQkq - 0 2", "e4xd5")
    assert san == "exd5" and after == "rnbqkbnr/ppp1pppp/8/3P4/8/8/PPPP1PPP/RNBQKBNR b KQkq - 0 2"
    # a king move drops both castling rights of its side; a rook capture on a corner drops the opponent's right
    san, after = _chess.san_push("r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1", "Rxa8+")
    assert san == "Rxa8+" and after == "R3k2r/8/8/8/8/8/8/4K2R b Kk - 0 1"
    san, after = _chess.san_push("r3k2r/8/8/8/8/8/8/R3K2R w KQkq - 0 1", "Kd1")
    assert san == "Kd1" and after == "r3k2r/8/8/8/8/8/8/R2K3R b kq - 1 1"
