"""The reference's data pipeline around self-play:
PGN -> JSONL ingestion (data_utils/parser_pgn.py) and the JSONL datasets
(data_utils/dataset.py ChessDataset; scripts/train.py ChessPGNDataset lives in
knightvision_amd.train). The chess rules they need (python-chess 1.999 in the
reference, absent here) are restated natively in libkv.so (csrc/kv_chess.cpp)."""
from .dataset import ChessDataset, create_dataloaders  # noqa: F401
from .parser_pgn import extract_data_from_pgn, parse_all_games  # noqa: F401
