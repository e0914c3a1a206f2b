"""PGN -> JSONL ingestion: the reference's data_utils/parser_pgn.py with its
chess work (chess.pgn.read_game, board.fen(), board.san(move), board.push)
done natively by libkv.so (csrc/kv_chess.cpp, python-chess 1.999 semantics).

Same names, record format and file conventions as the reference:
  * extract_data_from_pgn(pgn_path)           parser_pgn.py:81-118
  * extract_data_from_pgn_zst(path, move_limit, skip_moves)   :120-175
  * parse_all_games(pgn_dir, output_path)     :177-196
  * get_parsed_files / mark_file_parsed (PARSED_LOG), get_last_parsed_count /
    set_last_parsed_count (ZST_LOG)           :15-31, :63-70
Records are dicts {"fen": <board.fen() before the move>, "move": <SAN>,
"outcome": 1 | -1 | 0 | None} in file order; JSONL lines are json.dumps of
them, as the reference writes.

Not restated: the Telegram notifications (send_telegram_message /
notify_bot, :33-61) -- network side effects outside the data path -- and the
per-move progress-file rewrite inside extract_data_from_pgn (:105); the
progress count is written once per call instead (same final content).
The .zst reader needs the `zstandard` module (requirements.txt:6), which this
image lacks: it raises ImportError, as the reference's import would.
"""
from __future__ import annotations

import io
import json
import logging
import os

from . import _chess
from .._lib import PGN_OUTCOME_NONE

logger = logging.getLogger(__name__)

BASE_DIR = os.getenv("KV_DATA_DIR", os.path.join(os.getcwd(), "data"))
ZST_LOG = os.path.join(BASE_DIR, "parsed_zst_progress.log")
PARSED_LOG = os.path.join(BASE_DIR, "parsed_files.log")

# chunk size for streaming large PGN files (whole games per native call)
CHUNK_BYTES = 32 << 20


def get_last_parsed_count():
    if os.path.exists(ZST_LOG):
        with open(ZST_LOG, "r") as f:
            content = f.read().strip()
            if not content:
                logger.warning("ZST_LOG is empty. Starting from 0.")
                return 0
            try:
                return int(content)
            except ValueError:
                logger.warning("ZST_LOG has invalid content. Starting from 0.")
                return 0
    return 0


def set_last_parsed_count(count):
    os.makedirs(os.path.dirname(ZST_LOG) or ".", exist_ok=True)
    with open(ZST_LOG, "w") as f:
        f.write(str(count))


def get_parsed_files():
    if os.path.exists(PARSED_LOG):
        with open(PARSED_LOG, "r") as f:
            return set(line.strip() for line in f)
    return set()


def mark_file_parsed(filename):
    os.makedirs(os.path.dirname(PARSED_LOG) or ".", exist_ok=True)
    with open(PARSED_LOG, "a") as f:
        f.write(filename + "\n")


def _game_chunks(handle):
    """Text chunks of `handle` that end on a game boundary (a blank line followed
    by a tag line), so every game reaches the native parser whole."""
    carry = ""
    while True:
        block = handle.read(CHUNK_BYTES)
        if not block:
            if carry:
                yield carry
            return
        carry += block
        cut = _boundary(carry)
        if cut < 0:
            continue
        yield carry[:cut]
        carry = carry[cut:]


def _boundary(text: str) -> int:
    """Offset of the last game start in `text`: a tag line after a blank line
    whose preceding non-blank line is movetext (not a tag: read_game allows one
    blank line inside a tag section). -1 if none."""
    end = len(text)
    while True:
        k = text.rfind("\n\n[", 0, end)
        if k < 0:
            return -1
        prev = text.rfind("\n", 0, k)
        if not text[prev + 1:k].startswith("["):
            return k + 2
        end = k


def _records(handle):
    """(fen, san, outcome) tuples of every mainline move, in file order."""
    for text in _game_chunks(handle):
        for arr in _chess.pgn_records(text.encode("utf-8")):
            fens = arr["fen"]
            sans = arr["san"]
            outs = arr["outcome"]
            for i in range(len(arr)):
                oc = int(outs[i])
                yield fens[i].decode(), sans[i].decode(), (None if oc == PGN_OUTCOME_NONE else oc)


def extract_data_from_pgn(pgn_path):
    """Yield {"fen", "move", "outcome"} for every mainline move of every game in
    the PGN file (parser_pgn.py:81-118)."""
    count = 0
    try:
        with open(pgn_path, "r", encoding="utf-8", errors="ignore") as pgn_file:
            for fen, san, outcome in _records(pgn_file):
                yield {"fen": fen, "move": san, "outcome": outcome}
                count += 1
                if count % 100000 == 0:
                    logger.info("Parsed %s moves so far...", f"{count:,}")
    except OSError as e:
        logger.error("Failed to parse %s: %s", pgn_path, e)
    if count:
        set_last_parsed_count(count)


def extract_data_from_pgn_zst(zst_path, move_limit=None, skip_moves=0):
    """The .zst variant (parser_pgn.py:120-175): skips the first `skip_moves`
    moves of the stream, stops after `move_limit` records."""
    import zstandard as zstd  # requirements.txt:6; absent in this image -> ImportError, as in the reference
    count = 0
    skipped = 0
    dctx = zstd.ZstdDecompressor()
    with open(zst_path, "rb") as compressed:
        with dctx.stream_reader(compressed) as reader:
            text_stream = io.TextIOWrapper(reader, encoding="utf-8", errors="ignore")
            for fen, san, outcome in _records(text_stream):
                if skipped < skip_moves:
                    skipped += 1
                    continue
                yield {"fen": fen, "move": san, "outcome": outcome}
                count += 1
                if move_limit and count >= move_limit:
                    set_last_parsed_count(skip_moves + count)
                    return
    set_last_parsed_count(skip_moves + count)


def parse_all_games(pgn_dir=os.path.join(BASE_DIR, "data", "pgn"),
                    output_path=os.path.join(BASE_DIR, "data", "games.jsonl")):
    """Append the records of every not-yet-parsed *.pgn in pgn_dir to output_path
    (JSONL), marking each file in PARSED_LOG (parser_pgn.py:177-196)."""
    if not os.path.exists(pgn_dir):
        logger.error("PGN directory not found: %s", pgn_dir)
        return
    os.makedirs(os.path.dirname(output_path) or ".", exist_ok=True)
    parsed_files = get_parsed_files()
    with open(output_path, "a", encoding="utf-8") as out_file:
        for filename in os.listdir(pgn_dir):
            if filename.endswith(".pgn") and filename not in parsed_files:
                logger.info("Parsing %s...", filename)
                count = 0
                for record in extract_data_from_pgn(os.path.join(pgn_dir, filename)):
                    out_file.write(json.dumps(record) + "\n")
                    count += 1
                mark_file_parsed(filename)
                logger.info("Finished parsing %s (%d moves)", filename, count)
