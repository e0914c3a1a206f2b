"""Batch-1 latency of the inference-only move choice:
the HIP network at batch 1 (device time, HIP events, and host wall time of
ChessNet.__call__ including the H2D / D2H copies) and play.get_ai_move end to
end (device getValidMoves + encode + forward + host softmax / argmax) on a
fixed set of positions. The reference's CPU forward at B = 1 is 7.6 ms
(SURVEY.md 8d perf table, ai/model.py:51 on 8 Xeon threads)."""
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from knightvision_amd.ai import encode_board  # noqa: E402
from knightvision_amd.chess_engine import GameState  # noqa: E402
from knightvision_amd.model import ChessNet  # noqa: E402
from knightvision_amd.play import get_ai_move  # noqa: E402
from knightvision_amd.weights import synthetic_state_dict  # noqa: E402


def main():
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "bn").items()})
    m.eval()
    gs = GameState()
    x = torch.tensor(np.asarray([encode_board(gs.board)], dtype=np.float32))
    net = m.kv_net(0)
    codes = torch.randint(0, 13, (1, 64), dtype=torch.int8, device="cuda")
    for _ in range(20):
        net.forward_boards(codes)
        m(x)
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    n = 200
    e0.record()
    for _ in range(n):
        net.forward_boards(codes)
    e1.record()
    torch.cuda.synchronize()
    dev_us = e0.elapsed_time(e1) / n * 1e3
    t0 = time.perf_counter()
    for _ in range(n):
        with torch.no_grad():
            p, v = m(x)
        p.cpu()
    call_us = (time.perf_counter() - t0) / n * 1e6
    # get_ai_move over the first plies of a greedy game (the GUI loop)
    lat = []
    for _ in range(40):
        t0 = time.perf_counter()
        mv = get_ai_move(gs, m)
        lat.append(time.perf_counter() - t0)
        gs.makeMove(mv)
    lat = np.array(lat[5:]) * 1e3
    print(f"HIP forward B=1 (device, HIP events): {dev_us:.1f} us")
    print(f"ChessNet(x) B=1 host wall incl. copies: {call_us:.1f} us")
    print(f"get_ai_move end to end: median {np.median(lat):.3f} ms, p90 {np.percentile(lat, 90):.3f} ms "
          f"over {len(lat)} plies (reference CPU forward alone at B=1: 7.6 ms)", flush=True)


if __name__ == "__main__":
    main()
