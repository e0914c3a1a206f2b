"""CPU calibration: time the REFERENCE self-play loop and this
repo's CPU restatement (the bench's `cpu_baseline` "port") on the same work in
THIS container, so the port's number on the GPU box can be read as a
reference-equivalent rate: ref_box ~= port_box * (ref_here / port_here).

Runs only where /root/reference exists (never on the GPU box). Work: N games
from the start position, max_moves=64, batch-16 reference eval schedule,
synthetic random-init weights (seed 42), torch-CPU fp32 on all cores.
Reference: scripts/self_play.py `self_play(model, N, cpu, 64)` (model-instance
path = sequential, :283-287). Port: oracle.play_game per game with the same
schedule (test infrastructure, as in bench.py's cpu_baseline).

    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_cpu.py [N] [THREADS] > profiles/r01_cpu_calibration.json

THREADS (default: torch's default, all cores) sets the torch threads of both
sides; 1 matches bench.py's cpu_baseline pool (one thread per worker process):
    PYTHONDONTWRITEBYTECODE=1 python tools/calibrate_cpu.py 12 1 > profiles/r03_cpu_calibration_1thread.json
"""
from __future__ import annotations

import json
import os
import platform
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
REPO = os.path.dirname(HERE)
sys.path.insert(0, REPO)
sys.path.insert(0, os.path.join(REPO, "tests", "golden"))


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return platform.processor()


def main():
    n = int(sys.argv[1]) if len(sys.argv) > 1 else 12
    if len(sys.argv) > 2:
        torch.set_num_threads(int(sys.argv[2]))
    from make_golden import import_reference
    from knightvision_amd.weights import synthetic_state_dict
    from oracle import oracle as O
    from oracle import torch_ref
    sd = synthetic_state_dict(42, "init")
    sp, _, ref_model, _ = import_reference("/root/reference")
    m = ref_model.ChessNet()
    m.load_state_dict({k: torch.from_numpy(np.asarray(v)) for k, v in sd.items()})
    m.eval()
    # reference: one sequential run of n games (its own module-level streams, seeded SEED=42 at import)
    t0 = time.perf_counter()
    data = sp.self_play(m, n, torch.device("cpu"), max_moves=64)
    t_ref = time.perf_counter() - t0
    ref_plies = len(data)
    # port: the oracle restatement, n games, per-game seeds
    ev = torch_ref.make_eval_fn(sd)
    t0 = time.perf_counter()
    port_plies = 0
    for g in range(n):
        r = O.play_game(ev, O.MT(42 + g, "numpy"), O.MT(42 + g, "python"), O.Last(), max_moves=64, batch=16,
                        softmax_fn=torch_ref.torch_softmax)
        port_plies += r["plies"]
    t_port = time.perf_counter() - t0
    ref_rate, port_rate = ref_plies / t_ref, port_plies / t_port
    print(json.dumps({
        "what": "reference scripts/self_play.py vs the oracle CPU restatement (bench cpu_baseline 'port'), same work, "
                "this container",
        "games": n, "max_moves": 64, "batch": 16, "weights": "synthetic init seed 42",
        "cpu": cpu_model(), "cores": os.cpu_count(), "torch_threads": torch.get_num_threads(),
        "reference": {"plies": ref_plies, "seconds": t_ref, "plies_per_s": ref_rate},
        "port": {"plies": port_plies, "seconds": t_port, "plies_per_s": port_rate},
        "ref_over_port": ref_rate / port_rate,
        "use": "reference-equivalent CPU rate on another host ~= port rate there x ref_over_port",
    }, indent=1))


if __name__ == "__main__":
    main()
