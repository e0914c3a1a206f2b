"""Length of complete MCTS self-play games at the C3 settings (800 sims/move,
uncapped, per-game seeds 42 + id, random-init weights seed 42), played to
the end on fewer slots. Games are per-game seeded and the > 16-board network
class is batch-invariant, so game g here is move for move game g of the C3
bench run (tests/test_fullsize_gpu.py checks that a small run equals the first
games of a big one). The C3 bench times 20 moves of games that started
together, so its own games/hour is a transient count; this gives the game
lengths the steady-state figure needs.

    python tools/mcts_game_length.py [--games 384] [--first 0] [--seconds 1000] [--out profiles/r03_mcts_game_length_c3.json]
    python tools/mcts_game_length.py --merge a.json b.json --out merged.json   (disjoint game-id ranges)

Prints a progress line per 20 plies and one JSON line (also written to --out):
per-game plies, end reasons, the mean with its standard error and 95 %
interval, games still running at the time limit (censored; none when the run
completes). bench.py reads the newest such file for its steady-state MCTS
games/hour. Once games start to end, the engine's leaf batches carry only the
active slots (k_compact_active), so the tail of long games is cheap.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=384)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--seconds", type=float, default=1000.0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--first", type=int, default=0, help="first game id (seeds 42 + id): a later batch of the same run")
    ap.add_argument("--merge", nargs="+", default=None, help="merge runs over disjoint game-id ranges")
    a = ap.parse_args()
    if a.merge:
        return merge(a.merge, a.out)
    import torch  # noqa: F401
    from knightvision_amd.engine import REASONS, SelfPlayEngine
    from knightvision_amd.weights import synthetic_state_dict
    t0 = time.perf_counter()
    with SelfPlayEngine(synthetic_state_dict(42, "init"), slots=a.games, n_games=a.games, seed=42, max_moves=None,
                        sims=a.sims, recycle=False, record_cap=a.games * 2048, game_id_base=a.first,
                        game_id_stride=1) as eng:
        ply = 0
        while time.perf_counter() - t0 < a.seconds:
            eng.run(max_steps=20)
            ply += 20
            st = eng.stats()
            print(f"ply {ply}: {st['games_done']}/{a.games} games done, {time.perf_counter() - t0:.0f} s",
                  file=sys.stderr, flush=True)
            if st["games_done"] >= a.games:
                break
        games = eng.games()
        st = eng.stats()
        cal = eng.calibration()
    plies = np.sort(games["plies"]).tolist()
    reasons = {REASONS.get(int(r), "?"): int((games["reason"] == r).sum()) for r in np.unique(games["reason"])}
    n = len(plies)
    res = summary(plies, reasons, a.sims, a.games, n, ply)
    res.update({"first_game_id": a.first, "wall_s": time.perf_counter() - t0, "total_sims": int(st["sims"]),
                "conv_path": cal["path_large"], "conv_path_small": cal["path_small"], "dom_kernel": st["dom_kernel"]})
    line = json.dumps(res)
    print(line, flush=True)
    if a.out:
        with open(a.out, "w") as f:
            f.write(line + "\n")


def summary(plies, reasons, sims, games, n, ply):
    plies = sorted(plies)
    mean = float(np.mean(plies)) if plies else None
    sd = float(np.std(plies, ddof=1)) if n > 1 else None
    se = sd / np.sqrt(n) if sd is not None else None
    return {"what": "complete MCTS games at the C3 settings (game ids 0..n-1 of the C3 run: 800 sims/move, "
                   "uncapped, per-game seeds 42+id, random-init weights seed 42, c_puct 1.5) on the conv path the "
                   "AUTO calibration chose (conv_path): the games the headline plays",
           "sims": sims, "games": games, "finished": n, "still_running": games - n,
           "plies_played_by_running_games": ply if n < games else None,
           "mean_plies_finished": mean, "median_plies_finished": float(np.median(plies)) if plies else None,
           "sd_plies": sd, "se_mean_plies": se, "se_frac": (se / mean) if se else None,
           "ci95_mean_plies": [mean - 1.96 * se, mean + 1.96 * se] if se else None,
           "plies": plies, "reasons": reasons}


def merge(files, out):
    runs = [json.loads(open(f).read().splitlines()[-1]) for f in files]
    ids = sorted((r.get("first_game_id", 0), r["games"]) for r in runs)
    assert all(ids[i][0] + ids[i][1] == ids[i + 1][0] for i in range(len(ids) - 1)) and ids[0][0] == 0, ids
    assert len({r["conv_path"] for r in runs}) == 1 and all(r["sims"] == runs[0]["sims"] for r in runs)
    plies = [p for r in runs for p in r["plies"]]
    reasons = {}
    for r in runs:
        for k, v in r["reasons"].items():
            reasons[k] = reasons.get(k, 0) + v
    games = sum(r["games"] for r in runs)
    res = summary(plies, reasons, runs[0]["sims"], games, len(plies), None)
    res.update({"merged_from": [os.path.basename(f) for f in files], "conv_path": runs[0]["conv_path"],
                "conv_path_small": runs[0]["conv_path_small"], "dom_kernel": runs[0]["dom_kernel"],
                "wall_s": sum(r["wall_s"] for r in runs), "total_sims": sum(r["total_sims"] for r in runs)})
    line = json.dumps(res)
    print(line)
    if out:
        with open(out, "w") as f:
            f.write(line + "\n")


if __name__ == "__main__":
    main()
