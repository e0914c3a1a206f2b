"""knightvision_amd -- MI355X-native self-play engine for the KnightVision
self-play data-generation path (scripts/self_play.py, ai/ai.py, ai/model.py,
core/chessEngine.py of TheRealShamsaba/KnightVision)."""
from .ai import PIECE_TO_INDEX, INDEX_TO_PIECE, decode_move_index, encode_board, encode_move  # noqa: F401

__all__ = ["encode_board", "encode_move", "decode_move_index", "PIECE_TO_INDEX", "INDEX_TO_PIECE", "ChessNet"]


def __getattr__(name):
    if name == "ChessNet":
        from .model import ChessNet
        return ChessNet
    raise AttributeError(name)
