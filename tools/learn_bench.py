"""Learn-loop throughput (BASELINE configs[4]): self-play
on the HIP engine, then the update step with DDP over RCCL, per iteration.

    python tools/learn_bench.py [--iterations 3] [--games 256] [--max-moves 80] [--sims 0]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 tools/learn_bench.py ...

Prints one JSON line from rank 0: self-play plies/s and training samples/s over
all ranks for the last iteration, with the per-phase times (max over ranks).
Synthetic random-init weights (seed 42), per-game seeds 42 + global id.
"""
import argparse
import json
import os
import sys
import time

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--iterations", type=int, default=3)
    ap.add_argument("--games", type=int, default=256, help="games per iteration over all ranks")
    ap.add_argument("--max-moves", type=int, default=80)
    ap.add_argument("--sims", type=int, default=0)
    ap.add_argument("--batch-size", type=int, default=4096)
    ap.add_argument("--epochs", type=int, default=1)
    a = ap.parse_args()
    rank, world = int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    local = local % max(torch.cuda.device_count(), 1)  # ranks > GPUs (a gloo rehearsal) share the devices
    torch.cuda.set_device(local)
    import torch.distributed as dist
    if world > 1:
        backend = os.environ.get("KV_LEARN_BACKEND", "nccl")  # gloo: a rehearsal with ranks sharing one GPU
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
    from knightvision_amd.learn import reinforcement_loop
    from knightvision_amd.model import ChessNet
    from knightvision_amd.weights import synthetic_state_dict
    m = ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in synthetic_state_dict(42, "init").items()})
    t0 = time.perf_counter()
    stats = reinforcement_loop(m, a.iterations, a.games, f"cuda:{local}", epochs=a.epochs, batch_size=a.batch_size,
                               max_moves=a.max_moves, sims=a.sims, log=None)
    wall = time.perf_counter() - t0
    last = stats[-1]
    vals = torch.tensor([last.get("selfplay_s", 0.0), last.get("train_s", 0.0)], dtype=torch.float64, device="cuda")
    cnt = torch.tensor([float(last.get("train_samples", 0))], dtype=torch.float64, device="cuda")
    if world > 1:
        dist.all_reduce(vals, op=dist.ReduceOp.MAX)
        dist.all_reduce(cnt)
    sp_s, tr_s = vals.tolist()
    if rank == 0:
        print(json.dumps({"metric": "learn loop: self-play + DDP update per iteration", "n_ranks": world,
                          "backend": dist.get_backend() if world > 1 else None,
                          "iterations": a.iterations, "games_per_iteration": a.games, "max_moves": a.max_moves,
                          "sims": a.sims, "selfplay_s": sp_s, "train_s": tr_s,
                          "train_samples_per_s": cnt.item() / tr_s if tr_s else None,
                          "val_loss": last.get("val_loss"), "records": last["records"], "wall_s": wall,
                          "nn_path_per_iteration": [st.get("nn_path") for st in stats],
                          # rank 0's self-play per iteration (sims/s with --sims > 0, else plies/s): the spread a
                          # change of conv path between iterations would show
                          "selfplay_rate_per_iteration": [
                              round((st.get("sims") or st.get("plies", 0)) / st["selfplay_s"], 1) for st in stats],
                          "selfplay_s_per_iteration": [round(st["selfplay_s"], 3) for st in stats],
                          "sims_per_iteration": [st.get("sims") for st in stats],
                          "plies_per_iteration": [st.get("plies") for st in stats],
                          "calib_ms_per_iteration": [round(st["calib_ms"]) if "calib_ms" in st else None
                                                     for st in stats],
                          "calib_err_per_iteration": [st.get("calib_err") for st in stats],
                          "data": "synthetic"}), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
