"""Benchmark of the self-play data-generation path on MI355X.

    python bench.py [--gpus N] [--steps K] [--warmup W] [--mode mcts|ref] ...

Workload (BASELINE.json configs[2], C3 -- the largest single-GPU config):
2,048 concurrent games per GPU, 800 PUCT simulations per move, fp32 ChessNet
(the reference's precision), batch-2048 network evaluation, random-init
synthetic weights (seed 42, knightvision_amd.weights), games from the initial
position with per-game seeds 42 + global game id, slots recycled.

One step = one move of every slot: the full search (800 sim-steps, each one
2,048-board network batch + the tree kernels) and the committed move. The
timed region covers plies W+1 .. W+K of games started at the initial position;
no MCTS game finishes inside it at the default K, so MCTS games/hour is
reported only when games actually completed (else null), and the measured
games/hour comes from the C3-ref block: the reference's own move selection
(sims = 0, one network row per ply, softmax + Dirichlet + random.choices) on
the same 2,048 slots, long enough for thousands of games to complete.

N > 1: `bench.py --gpus N` starts N ranks itself (torch.distributed.run as a
child process, before any GPU call), or runs under an external
torch.distributed.run; one process per GPU, games sharded by global id (weak
scaling, no collective in the loop); the timed region is bracketed by barrier
+ synchronize and the max over ranks is used. After the timed region the
ranks gather their device-resident experience records to rank 0 over RCCL
(gather_ms, not part of `value`).
"""
from __future__ import annotations

import argparse
import json
import os
import socket
import subprocess
import sys
import time

import numpy as np
import torch

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)

FLOP_PER_EVAL = 3175744512            # SURVEY.md 8d, ChessNet forward per position
FLOP_RES_CONV_PER_BOARD = 301989888   # one 3x3 512->512 conv on 8x8 (2*64*512*4608)
FLOP_WINO48_GEMM_PER_BOARD = 62914560  # its Winograd F(4x8,3x3) GEMMs: 2 * 2 tiles * 60 * 512 * 512
FLOP_WINO88_GEMM_PER_BOARD = 52428800  # the fp32 default, F(8x8,3x3) GEMMs: 2 * 1 tile * 100 * 512 * 512
FP32_MFMA_PEAK_TFLOPS = 157.3         # MI355X_MICROARCH.md, f32-input MFMA (dense)
FP64_MFMA_PEAK_TFLOPS = 78.6          # AMD's MI355X FP64 matrix spec figure (the guides give no f64 row; not
                                      # measured here)
PATH_NAMES = {0: "direct", 1: "winograd48 (retired)", 2: "winograd88", 3: "winograd88_f64",
              4: "winograd48_f16x3 (retired)",
              5: "winograd88_i8", 6: "winograd88_i8f32", 7: "winograd88_i8f32v",
              8: "winograd88_i8r", 9: "winograd88_i8f32r3"}  # KV_PATH_*
BF16_MFMA_PEAK_TFLOPS = 2500.0        # dense bf16 MFMA
I8_MFMA_PEAK_TOPS = 5000.0            # dense int8 MFMA: 2x the bf16 rate (cdna_hip_programming.md, MFMA rate per dtype);
                                      # v_mfma_i32_32x32x32_i8 back to back measured 4.1 POPS at the clock the chip
                                      # holds under it (profiles/r04_mfma_rate.log)
I8_MFMA_MEASURED_TOPS = 4098.0
I8_DIGIT_PRODUCTS = {5: 15, 6: 10, 7: 10, 8: 13, 9: 6}    # int8 GEMMs per Winograd GEMM: digit pairs i + j < 5 (KV_PREC_I8X5, fp64
                                      # domain) / < 4 (KV_ALGO_WINOGRAD88_I8, fp32 domain)


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=None)
    ap.add_argument("--warmup", type=int, default=None)
    ap.add_argument("--mode", choices=["mcts", "ref"], default=os.environ.get("KV_BENCH_MODE", "mcts"))
    ap.add_argument("--slots", type=int, default=2048)
    ap.add_argument("--sims", type=int, default=800)
    ap.add_argument("--precision", choices=["fp32", "f64w", "i8x5", "i8r4"], default="fp32")
    ap.add_argument("--algo", choices=["auto", "direct", "winograd88", "winograd88i8", "winograd88i8v",
                                       "winograd88i8r3"],
                    default="auto",
                    help="conv algorithm of the fp32 tower (auto: the library's calibrated choice per weight load -- "
                         "Winograd F(8x8,3x3) fp32 for the random-init weights)")
    ap.add_argument("--compare-direct", type=int, default=0,
                    help="also measure the fp32 direct implicit-GEMM tower ('fp32_direct'; ~40 s per step at C3)")
    ap.add_argument("--weights", choices=["init", "stress"], default="init",
                    help="synthetic weights of the headline run: init (random init, the reference's untrained "
                         "network) or stress (trained-network magnitudes, weights.stress_state_dict)")
    ap.add_argument("--trained-steps", type=int, default=2,
                    help="also time this many moves on the stress weights (trained-network magnitudes: AUTO "
                         "chooses the fp64 Winograd domain on int8 digits there, and the priors are peaked, so the "
                         "trees take their own shapes), reported under 'trained_weights_path'; 0 to skip")
    ap.add_argument("--f64w-steps", type=int, default=0,
                    help="also time this many moves with the fp64 Winograd domain on fp64 MFMA (KV_PREC_F64W), "
                         "reported under 'f64w_path'")
    ap.add_argument("--alt-precision", default="",
                    help="also measure this network precision (reported under 'alt_precision'; '' to skip)")
    ap.add_argument("--alt-algo", default="winograd88",
                    help="fp32 only: also time this conv algorithm for --alt-steps moves beside the headline's own "
                         "(the fp32 MFMA F(8x8) tower beside the int8-digit one AUTO chooses); '' to skip")
    ap.add_argument("--alt-steps", type=int, default=2)
    ap.add_argument("--alt-warmup", type=int, default=1)
    ap.add_argument("--ref-block", type=int, default=1,
                    help="mcts mode: also run the reference's own move selection (sims=0) on the same slots long "
                         "enough for games to complete, reported under 'ref_selection' with measured games/hour")
    ap.add_argument("--ref-steps", type=int, default=1200)
    ap.add_argument("--ref-warmup", type=int, default=600)
    ap.add_argument("--eval", choices=["faithful", "lazy", "hash"], default="faithful",
                    help="reference-selection network schedule: faithful (every board evaluated, as the reference "
                         "does) or lazy (only the rows the schedule consumes, identical games); hash: PROFILING "
                         "ONLY -- the MCTS test evaluator (uniform priors, hashed values) instead of the network, "
                         "3 launches per sim-step, so a tree-kernel counter run of a whole 800-sim move stays under "
                         "rocprofv3's dispatch limit (tools/runs/r03_tree.sh); its line is not a measurement")
    ap.add_argument("--tree-edge-cap", type=int, default=0,
                    help="MCTS edge pool per slot (0: KV_MAXM x (sims+1), which cannot overflow; an overflow "
                         "fails the run). Profiling runs under rocprofv3 --pmc use a smaller pool")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--clock-seconds", type=float, default=2.0,
                    help="after the timed region: the headline GEMM back to back for this long, then one stamped "
                         "launch of it -- the in-kernel clock the chip held (roofline.sclk_mhz); 0 to skip")
    ap.add_argument("--cpu-seconds", type=float, default=60.0,
                    help="duration of the MCTS CPU-baseline legs: 2/3 leaf-batched, 1/3 one leaf per call (the "
                         "reference-selection leg runs <= 10 s)")
    ap.add_argument("--cpu-leaf-batch", type=int, default=16,
                    help="games in lock-step per CPU-baseline process (their leaves as one torch batch)")
    return ap.parse_args()


def _mcts_game_length(sims: int, conv_path: str = None):
    """The newest committed game-length run at these search settings (tools/mcts_game_length.py: complete
    MCTS games at C3's settings, game ids 0..n-1 of the C3 run played to the end), preferring one played on
    `conv_path` (the conv path the run's AUTO chose: those are the games it plays), or (None, None)."""
    d = os.path.join(HERE, "profiles")
    found = []
    for f in sorted((x for x in os.listdir(d) if "mcts_game_length" in x and x.endswith(".json")), reverse=True):
        try:
            gl = json.loads(open(os.path.join(d, f)).read().splitlines()[-1])
        except (OSError, ValueError, IndexError):
            continue
        if gl.get("sims") == sims and gl.get("still_running") == 0 and gl.get("finished", 0) >= 2:
            found.append((gl, f))
    for gl, f in found:
        if conv_path is not None and gl.get("conv_path") == conv_path:
            return gl, f
    return found[0] if found else (None, None)


def _free_port() -> int:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def launch_ranks(n: int) -> int:
    """`bench.py --gpus N` without an external launcher: run N ranks under
    torch.distributed.run as a child process (nothing here has touched the GPU;
    rank 0 prints the JSON line) and return its exit code."""
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={_free_port()}", os.path.abspath(__file__), *sys.argv[1:]]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0")
    return subprocess.call(cmd, env=env)


def process_group_info(rank: int, world: int, local: int, backend: str) -> dict:
    """What the N-rank run actually was: the process group's size and backend and, per rank, its host and GPU
    (PCI domain / bus / device of the device it bound). Under nccl (RCCL) two ranks on one GPU are an error:
    the scaling line must come from N distinct GPUs."""
    import torch.distributed as dist
    props = torch.cuda.get_device_properties(local)
    pci = [int(getattr(props, k, -1)) for k in ("pci_domain_id", "pci_bus_id", "pci_device_id")]
    me = {"rank": rank, "host": socket.gethostname(), "local_device": local, "pci": pci, "name": props.name}
    ranks = [None] * world
    dist.all_gather_object(ranks, me)
    if backend == "nccl":
        seen = {}
        for r in ranks:
            key = (r["host"], tuple(r["pci"])) if -1 not in r["pci"] else (r["host"], "device", r["local_device"])
            if key in seen:
                raise SystemExit(f"bench.py: ranks {seen[key]} and {r['rank']} share one GPU {key} under nccl")
            seen[key] = r["rank"]
    return {"world_size": dist.get_world_size(), "backend": dist.get_backend(), "ranks": ranks}


def host_cpu() -> dict:
    try:
        aff = len(os.sched_getaffinity(0))
    except AttributeError:
        aff = os.cpu_count()
    return {"cpu": cpu_model(), "nproc": os.cpu_count(), "affinity_cpus": aff,
            "torch_threads": torch.get_num_threads()}


def _cpu_worker(wid: int, workers: int, sims: int, seconds: float, threads: int, barrier, q, batch: int = 1):
    """One CPU-baseline worker process: `threads` torch threads, games with seeds 42 + wid + k * workers,
    complete units (MCTS: one move of `sims` simulations; reference selection: one game of <= 64 plies)
    counted until `seconds` have passed after the common start barrier. MCTS with batch > 1: `batch` games
    in lock-step (oracle.mcts_play_batch), each simulation's leaves evaluated as one torch batch -- the
    GPU's batch shape; the unit is a leaf evaluation (= a completed simulation) finished before the deadline
    (the move in flight at the deadline finishes without the network and is not counted)."""
    import torch as _t
    _t.set_num_threads(threads)
    from oracle import oracle as O
    from oracle import torch_ref
    from knightvision_amd.weights import synthetic_state_dict
    ev = torch_ref.make_eval_fn(synthetic_state_dict(42, "init"))
    ev(np.zeros((max(batch, 1), 12, 8, 8), dtype=np.float32))  # first-call setup outside the timed loop
    barrier.wait(timeout=600)
    t0 = time.perf_counter()
    deadline = t0 + seconds
    units = games = 0
    seed = 42 + wid
    if sims > 0 and batch > 1:
        leaves = [0]
        roots = [True]

        def ev_b(x):
            if time.perf_counter() > deadline:
                return np.zeros((len(x), 4096), dtype=np.float32), np.zeros(len(x), dtype=np.float32)
            out = ev(x)
            if roots[0]:
                roots[0] = False  # the move's root evaluations are not simulations
            else:
                leaves[0] += len(x)
            return out
        while time.perf_counter() < deadline:
            roots[0] = True
            O.mcts_play_batch(sims, [seed + k * workers for k in range(batch)], ev_b, max_moves=1)
            games += batch
            seed += batch * workers
        q.put((wid, leaves[0], games, seconds))
        return
    while time.perf_counter() - t0 < seconds:
        if sims > 0:
            r = O.mcts_play_game(sims, O.MT(seed, "numpy"), O.MT(seed, "python"), ev, max_moves=1)
            units += r["plies"] * sims
        else:
            r = O.play_game(ev, O.MT(seed, "numpy"), O.MT(seed, "python"), O.Last(), max_moves=64, batch=16,
                            softmax_fn=torch_ref.torch_softmax)
            units += r["plies"]
        games += 1
        seed += workers
    q.put((wid, units, games, time.perf_counter() - t0))


def cpu_baseline(seconds: float, sims: int, batch: int = 1):
    """The oracle restatement (C rules + RNG + the reference's eval schedule /
    the build's PUCT restatement) with the reference's network run by torch on
    the host CPU (test infrastructure; never the measured product). MCTS: the
    same sims/move as the GPU; batch 1: one leaf per network call; batch G:
    each worker plays G games in lock-step and evaluates their leaves as one
    torch batch (the GPU's batch shape; 16 is the fastest per thread here:
    47.5 boards/s against 26.8 at batch 1 and 39.9 at 64).

    A pool of worker processes, one torch thread each (the reference's
    network calls are batch-1 / batch-16: processes scale where threads do
    not), as many as this job's CPU share: KV_CPU_WORKERS, else the box's
    OMP_NUM_THREADS (16 per GPU job on the GPU pool; the host's other CPUs
    serve the other GPUs' jobs), capped by the affinity mask. Reports the pool
    rate (`value`), the mean per-process rate, and a linear extrapolation to
    every CPU of the affinity mask (an upper bound, not measured)."""
    import multiprocessing as mp
    host = host_cpu()
    host.pop("torch_threads")  # the parent's; every worker runs one thread
    share = int(os.environ.get("KV_CPU_WORKERS", os.environ.get("OMP_NUM_THREADS", "16")))
    workers = max(1, min(share, host["affinity_cpus"] or 1))
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    barrier = ctx.Barrier(workers)
    procs = [ctx.Process(target=_cpu_worker, args=(w, workers, sims, seconds, 1, barrier, q, batch))
             for w in range(workers)]
    for p in procs:
        p.start()
    import queue
    res, deadline = [], time.perf_counter() + seconds + 900
    while len(res) < workers:  # fail loudly (not after a long block) if a worker dies
        try:
            res.append(q.get(timeout=5))
        except queue.Empty:
            dead = [p.exitcode for p in procs if p.exitcode not in (None, 0)]
            if dead or time.perf_counter() > deadline:
                for p in procs:
                    if p.is_alive():
                        p.terminate()
                raise RuntimeError(f"cpu_baseline: worker exit codes {dead or 'timeout'}")
    for p in procs:
        p.join(timeout=60)
    units = sum(r[1] for r in res)
    games = sum(r[2] for r in res)
    dt = max(r[3] for r in res)
    per_proc = [r[1] / r[3] for r in res]
    unit = "sims/s" if sims > 0 else "plies/s"
    what = (f"{games} games x 1 move x {sims} sims (per-game seeds 42+), oracle PUCT restatement + torch-CPU "
            "ChessNet fp32, " + (f"{batch} games in lock-step per process, their leaves as one torch batch; "
                                 "unit = leaf evaluations finished before the deadline" if batch > 1 else
                                 "one leaf per network call") if sims > 0 else
            f"{games} games x <=64 plies (per-game seeds 42+), oracle rules/RNG + torch-CPU ChessNet fp32, "
            "batch-16 reference schedule")
    return dict(value=units / dt, unit=unit, cores=workers, kind="port", **host, workers=workers, leaf_batch=batch,
                threads_per_worker=1, per_process_value=float(np.mean(per_proc)),
                whole_host_extrapolated=units / dt * (host["affinity_cpus"] or workers) / workers,
                whole_host_note="pool rate x affinity_cpus / workers: linear extrapolation to every CPU the "
                                "process may run on (an upper bound; not measured -- the GPU pool gives one GPU job "
                                f"a {share}-CPU share)",
                sample=f"{what}; {workers} processes x 1 torch thread, {dt:.1f}s")


def cpu_model() -> str:
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def gemm_label(path: int, kernel: str):
    """(kernel name, description) of the dominant Winograd GEMM launch: `kernel` is the name the library
    reports for the launch it made (kv_stats.dom_kernel, set by the launcher in knightvision_amd/csrc/kv_nn.hip
    that chose it), so a form switch (KV_I8F32_TPW=1, another CU count) relabels the line by itself; the
    description is looked up from the name's kernel family."""
    name = kernel or "?"
    fam = name.split("<")[0]
    targs = name[len(fam) + 1:-1].split(",") if "<" in name else []
    if fam == "wino_gemm_kernel" and name.endswith(",100>") or "+" in name:
        first, _, second = name.partition("+")
        if second:
            return first, (f" + {second} (residual-tower Winograd F(8x8,3x3) GEMM layer: the first points as "
                           "128x128 tiles, the rest as 64x128 tiles in a second launch, both inside the timed events)")
        return name, " (residual-tower Winograd F(8x8,3x3) GEMMs, 100 points)"
    if fam == "wino88i32_gemm_r3k64_kernel":
        tpw = int(targs[1])
        return name, (
            " (residual-tower Winograd F(8x8,3x3) GEMMs of the fp32 tower from 3 radix-256 int8 digits per value: the "
            "6 pairs i + j <= 2, v_mfma_i32_32x32x32_i8 chains, exact int32 accumulation, one rounding to fp32, "
            "128x128 tiles, " + (f"{tpw} per workgroup with the copy ring across them, " if tpw > 1 else "") +
            "64-k stages of 96-byte row copies (24 MFMAs per wave per barrier), chunk 1's last B digits per wave "
            "under the next stage's first LDS reads)")
    if fam == "wino88i32_gemm_lagt_kernel" and len(targs) > 2 and targs[2] == "3":
        tpw = int(targs[1])
        return name, (
            " (residual-tower Winograd F(8x8,3x3) GEMMs of the fp32 tower from 3 radix-256 int8 digits per value: the "
            "6 pairs i + j <= 2, v_mfma_i32_32x32x32_i8 chains, exact int32 accumulation, one rounding to fp32, "
            "128x128 tiles, " + (f"{tpw} per workgroup with the copy ring across them, " if tpw > 1 else "") +
            "each stage's last B digits per wave under the next stage's first LDS reads)")
    if fam in ("wino88i32_gemm_lagt_kernel", "wino88i32_gemm_lag_kernel"):
        tpw = int(targs[1]) if fam == "wino88i32_gemm_lagt_kernel" else 1
        return name, (
            " (residual-tower Winograd F(8x8,3x3) GEMMs of the fp32 tower from 4 int8 digits per value: 10 "
            "v_mfma_i32_32x32x32_i8 chains per point, exact int32 accumulation, one rounding to fp32, 128x128 "
            "tiles, " + (f"{tpw} per workgroup with the copy ring across them, " if tpw > 1 else "") +
            "each stage's last 6 MFMAs per wave under the next stage's first LDS reads)")
    if fam == "wino88i_gemm_lag5_kernel" and targs[-1] == "true":
        return name, (
            " (residual-tower Winograd F(8x8,3x3) GEMMs in the fp64 domain from 4 radix-256 int8 digits per value in "
            "row lines: the 13 pairs i + j <= 4, v_mfma_i32_32x32x32_i8 chains with exact int32 accumulation, "
            "128x128 tiles, each stage's last B digit under the next stage's first LDS reads; the operands' digits "
            "come from the previous output kernel, wino88i64r_out_kernel)")
    if fam in ("wino88i_gemm_lag5_kernel", "wino88i_gemm_kernel"):
        return name, (
            " (residual-tower Winograd F(8x8,3x3) GEMMs from int8 digits per value, v_mfma_i32_32x32x32_i8 chains, "
            "exact int32 accumulation, 128x128 tiles)")
    if fam == "wino88i32_gemm_kernel":
        return name, " (residual-tower Winograd F(8x8,3x3) GEMMs of the fp32 tower from 4 int8 digits, A/B form)"
    if fam == "wino88d_gemm_kernel":
        return name, " (residual-tower Winograd F(8x8,3x3) GEMMs in fp64, 100 points, v_mfma_f64_16x16x4_f64)"
    if fam == "wino_gemm_h3_kernel":
        return name, " (residual-tower Winograd F(4x8,3x3) GEMMs, f16x3 split; retired)"
    if fam == "wino_gemm_kernel":
        return name, " (residual-tower Winograd F(4x8,3x3) GEMMs, 60 points)"
    if fam == "conv3x3_kernel":
        return name, " (residual-tower 3x3 conv, implicit GEMM)"
    return name, ""


def baseline_config_tag(mcts: bool, G: int, sims: int, world: int) -> str:
    """Which BASELINE.json config the run is: C3 (2,048 games x 800 sims on one GPU), C4 (the same per GPU on 8
    GPUs, RCCL gather), C2 (256 x 400 on one GPU); other shapes name none."""
    if mcts and G == 2048 and sims == 800:
        return " (BASELINE configs[2], C3)" if world == 1 else (
            " (BASELINE configs[3], C4)" if world == 8 else f" (BASELINE configs[3]'s per-GPU shape, C4 at {world} GPUs)")
    if mcts and G == 256 and sims == 400 and world == 1:
        return " (BASELINE configs[1], C2)"
    return ""


def dom_units(path: int, dom_flop: float, G: int):
    """(algorithmic FLOP per board of the dominant launch, boards per launch, rows per Winograd point) for the
    conv path the library ran: every F(8x8) path (2, 3, 5-8) has 100 points of [rows x 512] x [512 x 512],
    F(4x8) (1, 4) 60 points at 2 rows per board, the direct conv 10 launches' worth per board."""
    f88 = path in (2, 3, 5, 6, 7, 8, 9)
    per_board = (FLOP_WINO88_GEMM_PER_BOARD if f88 else FLOP_WINO48_GEMM_PER_BOARD if path in (1, 4)
                 else FLOP_RES_CONV_PER_BOARD)
    bpl = min(G, int(round(dom_flop / per_board))) if dom_flop else G
    rows = int(round(dom_flop / (2 * 512 * 512 * (100 if f88 else 60)))) if (path and dom_flop) else bpl
    return per_board, bpl, rows


def _pmc_traffic(kname: str, bpl: int):
    """HBM bytes per launch of the dominant kernel at this batch from the newest
    committed PMC summary (tools/pmc_summary.py), or None."""
    for f in sorted((x for x in os.listdir(os.path.join(HERE, "profiles")) if "pmc" in x and x.endswith(".json")),
                    reverse=True):
        try:
            pj = json.load(open(os.path.join(HERE, "profiles", f)))
        except (OSError, ValueError):
            continue
        if (isinstance(pj, dict) and pj.get("batch") == bpl and
                pj.get("kernel", "").replace(" ", "") == kname and "hbm_bytes_per_launch" in pj):
            return pj["hbm_bytes_per_launch"], f
    return None, None


def gemm_clock(device: int, rows: int, seconds: float, digits: int = 4):
    """The clock this GPU holds under the headline GEMM (kv_dev_gemm_clock: the product's fp32-tower GEMM back to
    back for `seconds` on seeded digits, then one launch of its stamped build; MI355X_MICROARCH.md DVFS item 6),
    so a box-to-box spread of the line can be attributed."""
    import ctypes as C
    from knightvision_amd import _lib
    out = (C.c_double * 4)()
    _lib.check(_lib.lib().kv_dev_gemm_clock(device, rows, digits, seconds, out), "kv_dev_gemm_clock")
    return {"sclk_mhz": out[0], "gemm_us_back_to_back": out[1], "launches": int(out[2]),
            "tiles_per_workgroup": int(out[3]), "digits": digits,
            "method": f"median over workgroups of s_memtime delta / s_memrealtime delta x 100 MHz in a stamped build "
                      f"of the headline GEMM, launched right after {int(out[2])} back-to-back launches "
                      f"({seconds:.1f} s) on seeded random digits at {rows} boards; after the timed region"}


def _tree_pmc(G: int):
    """Tree-kernel HBM summary (tools/tree_hbm.py) for this slot count, newest round first."""
    for f in sorted((x for x in os.listdir(os.path.join(HERE, "profiles")) if x.endswith(".json") and "pmc_tree" in x),
                    reverse=True):
        tj = json.load(open(os.path.join(HERE, "profiles", f)))
        if tj.get("slots") == G and "per_sim" in tj:
            return tj, f
    return None, None


def main():
    args = parse()
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return launch_ranks(args.gpus)
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    if world != args.gpus:
        print(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world}", file=sys.stderr)
        return 2
    # one rank per GPU; more ranks than GPUs (a rehearsal of the sharded path on a 1-GPU box, with
    # KV_BENCH_BACKEND=gloo since RCCL refuses two ranks on one device) share the devices round-robin
    local = int(os.environ.get("LOCAL_RANK", "0")) % max(torch.cuda.device_count(), 1)
    torch.cuda.set_device(local)
    import torch.distributed as dist
    backend = None
    if world > 1:
        backend = os.environ.get("KV_BENCH_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(backend)
        if dist.get_world_size() != args.gpus:
            raise SystemExit(f"process group has {dist.get_world_size()} ranks, --gpus {args.gpus}")
    pg_info = process_group_info(rank, world, local, backend) if world > 1 else None
    from knightvision_amd.engine import EVAL_FAITHFUL, EVAL_HASH, EVAL_LAZY, SelfPlayEngine
    from knightvision_amd.weights import synthetic_state_dict
    from knightvision_amd.distributed import gather_experience

    mcts = args.mode == "mcts"
    sims = args.sims if mcts else 0
    steps = args.steps if args.steps is not None else (2 if mcts else 600)
    warmup = args.warmup if args.warmup is not None else (1 if mcts else 300)
    G = args.slots
    dev = torch.device("cuda", local)

    def run_chunks(eng, n, chunk, what, t0=None):
        # kv_run in chunks so a long region prints progress (stderr, rank 0); each kv_run already
        # synchronises with the device at its end, so the chunking adds no device idle time
        done = 0
        while done < n:
            k = min(chunk, n - done)
            eng.run(k)
            done += k
            if rank == 0 and (done == n or done % max(chunk, 1) == 0):
                el = f" {time.perf_counter() - t0:.1f}s" if t0 is not None else ""
                print(f"bench: {what} {done}/{n}{el}", file=sys.stderr, flush=True)

    def measure(precision, algo="auto", sims=sims, steps=steps, warmup=warmup, keep=False, tag="main",
                eval_mode="faithful", weights="init"):
        eng = SelfPlayEngine(synthetic_state_dict(42, weights), slots=G, n_games=1 << 40, seed=42, max_moves=None,
                             batch=16, sims=sims, game_id_base=rank, game_id_stride=world,
                             eval_mode=(EVAL_LAZY if (eval_mode == "lazy" and sims == 0) else
                                        EVAL_HASH if (eval_mode == "hash" and sims > 0) else EVAL_FAITHFUL),
                             record_cap=max(1 << 16, G * (steps + warmup + 8)), device=local, precision=precision,
                             algo=algo, tree_edge_cap=args.tree_edge_cap if sims > 0 else 0,
                             keep_root_visits=keep and sims > 0)
        chunk = 1 if sims > 0 else 100  # one progress line per move (MCTS: ~10 s at C3) or per 100 ply-steps
        run_chunks(eng, warmup, chunk, f"{tag} warmup")
        s0 = eng.stats()
        eng.reset_records()
        if world > 1:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        run_chunks(eng, steps, chunk, f"{tag} timed", t0)
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        dt = time.perf_counter() - t0
        s1 = eng.stats()
        t = torch.tensor([dt], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
        dt = float(t.item())
        d = {k: s1[k] - s0[k] for k in ("plies", "games_done", "nn_rows", "sims", "res_conv_ms", "res_conv_launches",
                                        "nn_rows_lazy")}
        tot = torch.tensor([d["plies"], d["games_done"], d["nn_rows"], d["sims"]], dtype=torch.float64, device=dev)
        if world > 1:
            dist.all_reduce(tot)
        plies, games_done, nn_rows, sims_done = (float(x) for x in tot.tolist())
        out = dict(dt=dt, plies=plies, games_done=games_done, nn_rows=nn_rows, sims=sims_done,
                   nn_rows_evaluated=float(d["nn_rows_lazy"]) if eval_mode == "lazy" else nn_rows,
                   conv_ms=d["res_conv_ms"] / max(d["res_conv_launches"], 1), dom_flop=s1["dom_flop"],
                   dom_algo=s1["dom_algo"], dom_path=s1["dom_path"], dom_split=s1["dom_split"],
                   dom_kernel=s1["dom_kernel"],
                   tree_overflows=s1["tree_overflows"], steps=steps, warmup=warmup)
        if tag in ("main", "trained"):
            out["calibration"] = eng.calibration()
        if keep:  # the timed region's experience, left in HBM for the gather (MCTS: with pi)
            out["recs_dev"], out["gms"] = eng.records_device(), eng.games()
            out["pi_dev"] = eng.root_visits_device() if sims > 0 else None
        eng.close()
        return out

    m = measure(args.precision, args.algo, keep=True, eval_mode=args.eval, weights=args.weights)
    calib_ranks = None
    if world > 1:  # every rank must run the same conv path (the calibration is per process)
        calib_ranks = [None] * world
        dist.all_gather_object(calib_ranks, {"rank": rank, "path_large": m["calibration"]["path_large"],
                                             "path_small": m["calibration"]["path_small"],
                                             "err_logit": m["calibration"]["err_logit"],
                                             "err_value": m["calibration"]["err_value"]})
        paths = {(c["path_large"], c["path_small"]) for c in calib_ranks}
        if len(paths) != 1:
            raise SystemExit(f"bench.py: ranks chose different conv paths {calib_ranks}")
    dt, plies, games_done, nn_rows, sims_done, conv_ms = (m[k] for k in ("dt", "plies", "games_done", "nn_rows",
                                                                          "sims", "conv_ms"))

    # end-of-iteration experience gather to rank 0 (RCCL over xGMI from HBM), outside `value`
    torch.cuda.synchronize()
    if world > 1:
        dist.barrier()
    tg = time.perf_counter()
    pi_dev = m.pop("pi_dev")
    if pi_dev is not None:  # (s, pi, z): records + root visit counts (BASELINE config C4)
        recs_all, gms_all, pi_all = gather_experience(m.pop("recs_dev"), m["gms"], dst=0, pi=pi_dev)
    else:
        recs_all, gms_all = gather_experience(m.pop("recs_dev"), m["gms"], dst=0)
        pi_all = None
    gather_ms = (time.perf_counter() - tg) * 1e3 if world > 1 else None
    n_records = int(len(recs_all)) if recs_all is not None else 0
    # wire bytes: 80-B records + pi as legal-move prefixes (2 B per legal move + a 2-B count per record,
    # distributed.pack_pi); the padded uint16 [n, MAXM] form would be 640 B per record
    pi_wire = (2 * int(pi_all.shape[0]) + 2 * int((pi_all != 0xffff).sum())) if pi_all is not None else 0
    gathered_bytes = n_records * 80 + pi_wire

    alt = None
    if args.alt_precision and args.alt_precision != args.precision:
        alt = measure(args.alt_precision, steps=args.alt_steps, warmup=args.alt_warmup, tag="alt " + args.alt_precision)
    alt_algo = None
    if args.alt_algo and args.precision == "fp32" and PATH_NAMES.get(m["dom_path"]) != {
            "winograd88": "winograd88", "direct": "direct",
            "winograd88i8": "winograd88_i8f32"}.get(args.alt_algo):
        alt_algo = measure("fp32", args.alt_algo, steps=args.alt_steps, warmup=args.alt_warmup,
                           tag="alt " + args.alt_algo)
    refsel = reflazy = None
    if mcts and args.ref_block:
        # C3-ref: the reference's move selection (one network row per ply, sampled move) on the same slots;
        # the warm-up ply-steps fill the slots with games at every stage, the timed ones complete games at
        # the steady-state rate
        refsel = measure(args.precision, sims=0, steps=args.ref_steps, warmup=args.ref_warmup, tag="ref-selection")
        # the same games with the network only on the rows the schedule consumes (KV_EVAL_LAZY): a side
        # figure, never the measured games/hour -- the reference evaluates every board
        reflazy = measure(args.precision, sims=0, steps=args.ref_steps, warmup=args.ref_warmup,
                          tag="ref-selection lazy", eval_mode="lazy")
    direct = None
    if args.compare_direct and args.precision == "fp32" and m["dom_path"] != 0:
        direct = measure("fp32", "direct", steps=1, warmup=1, tag="direct")
    trained = None
    if args.trained_steps > 0 and args.precision == "fp32" and args.weights != "stress":
        trained = measure("fp32", "auto", steps=args.trained_steps, warmup=args.alt_warmup, tag="trained",
                          weights="stress")
    f64w = None
    if args.f64w_steps > 0 and args.precision == "fp32" and m["dom_path"] != 3:
        f64w = measure("f64w", steps=args.f64w_steps, warmup=args.alt_warmup, tag="f64w")

    # roofline of the dominant kernel, timed with HIP events on the engine stream: one residual-tower
    # Winograd GEMM layer per forward (fp32 F(8x8) by default; [boards x 512] x [512 x 512] per point) or, for
    # the direct algorithm, the residual convs
    path = m["dom_path"]  # KV_PATH_* (include/kv.h): 0 direct, 2 F(8x8) fp32, 3 F(8x8) fp64, 5-9 int8-digit towers
    per_board, bpl, rows = dom_units(path, m["dom_flop"], G)
    flop_alg = per_board * bpl
    achieved = flop_alg / (conv_ms * 1e-3) / 1e12 if conv_ms > 0 else None
    kname, kdesc = gemm_label(path, m["dom_kernel"])
    peak = FP64_MFMA_PEAK_TFLOPS if path == 3 else FP32_MFMA_PEAK_TFLOPS
    if path in I8_DIGIT_PRODUCTS:  # int8 operations of the digit products against the int8 peak
        achieved = achieved * I8_DIGIT_PRODUCTS[path] if achieved else None
        flop_alg *= I8_DIGIT_PRODUCTS[path]
        peak = I8_MFMA_PEAK_TOPS
    traffic, traffic_src = _pmc_traffic(kname, bpl)
    # (rows: the launch's padded rows per point, a multiple of the GEMM's 128-row tile)
    clock = (gemm_clock(local, rows, args.clock_seconds, 3 if path == 9 else 4)
             if (path in (6, 7, 9) and args.clock_seconds > 0) else None)
    clock_ranks = None
    if world > 1 and clock is not None:
        clock_ranks = [None] * world
        dist.all_gather_object(clock_ranks, {"rank": rank, "sclk_mhz": clock["sclk_mhz"]})

    # HBM side of the search (north_star: tree kernels as a fraction of the HBM roofline), from the
    # rocprofv3 PMC + kernel-trace summary committed for this slot count (tools/tree_hbm.py)
    tree_hbm = None
    tj, tf = _tree_pmc(G)
    if mcts and tj is not None:
        tree_hbm = {"kernels": tj["per_sim"].get("note", "k_mcts_select + k_mcts_backup"),
                    "bytes_per_sim": tj["per_sim"]["bytes_per_sim"], "achieved_GBps": tj["per_sim"]["GBps"],
                    "peak_GBps": tj["peak_GBps"], "frac": tj["per_sim"]["frac"],
                    "source": "profiles/" + tf,
                    "note": "latency-bound: one wave per game (select descent + leaf getValidMoves, backup)"}

    # complete-game length at these search settings (per-game seeds: the same distribution at any slot count)
    gl, gl_file = _mcts_game_length(sims, PATH_NAMES.get(path)) if mcts else (None, None)
    steady = bool(gl) and warmup >= 2 * gl["mean_plies_finished"]  # slots have cycled through whole games
    if rank == 0:
        if mcts:
            metric, unit, value = "MCTS simulations/sec + self-play games/hour", "sims/s", sims_done / dt
        else:
            metric, unit, value = "self-play plies/sec + games/hour (reference move selection, sims=0)", \
                "plies/s", plies / dt
        mean_len = float(gms_all["plies"].mean()) if gms_all is not None and len(gms_all) else None
        gph = games_done / dt * 3600.0 if games_done > 0 else None
        wl = (f"{G} concurrent games/GPU, {sims} sims/move, batch-{G} NN eval, fp32" +
              (" [hash test evaluator instead of the network: PROFILING ONLY, not a measurement]"
               if args.eval == "hash" else "") if mcts else
              f"{G} concurrent games/GPU, reference move selection (sims=0), batch-{G} NN eval, fp32")
        out = {
            "metric": metric, "value": value, "unit": unit, "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": dt * 1e3 / steps, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": args.precision,
            "data": (f"synthetic ({'random-init' if args.weights == 'init' else 'trained-magnitude (stress)'} weights "
                     "seed 42, self-play from the start position, per-game seeds)"),
            "config": {"workload": wl + baseline_config_tag(mcts, G, sims, world),
                       "slots_per_gpu": G, "sims_per_move": sims, "nn_batch": G, "parallelism": f"games sharded x{world}",
                       "step": "one move of every slot (the whole search + the committed move)" if mcts else
                               "one ply of every slot"},
            "plies_per_s": plies / dt, "games_per_hour": gph,
            "games_per_hour_note": (
                (f"{int(games_done)} games ended inside the timed region / its duration, slots recycled; the "
                 f"warm-up ({warmup} moves) is >= 2 mean game lengths, so the slots hold games at every stage: a "
                 "steady-state rate" if (mcts and steady) else
                 f"{int(games_done)} games ended inside the timed region / its duration -- a transient count, not "
                 f"a steady-state rate: every slot started at ply 0, the region covers plies {warmup + 1}-"
                 f"{warmup + steps}, so only early endings are in it; see games_per_hour_steady_derived and "
                 "ref_selection" if mcts else
                 "games completed inside the timed region / its duration (slots recycled)") if gph is not None else
                f"no game completed inside the {steps} timed moves (plies {warmup + 1}-{warmup + steps} of games "
                f"from the start position); measured games/hour: ref_selection"),
            "games_per_hour_steady_derived": (plies / dt * 3600.0 / gl["mean_plies_finished"]
                                              if gl is not None else None),
            "games_per_hour_steady_ci95": ([plies / dt * 3600.0 / gl["ci95_mean_plies"][1],
                                            plies / dt * 3600.0 / gl["ci95_mean_plies"][0]]
                                           if gl is not None and gl.get("ci95_mean_plies") else None),
            "games_per_hour_steady_note": (
                f"this run's measured plies/s x 3600 / the mean length of complete games at these settings, "
                f"{gl['mean_plies_finished']:.1f} plies (game ids 0-{gl['games'] - 1} played to the end on "
                f"{gl.get('conv_path', 'winograd88 (round 3)')}: "
                f"{gl['reasons']}; median {gl['median_plies_finished']:.0f}, range {gl['plies'][0]}-"
                f"{gl['plies'][-1]}, standard error {100 * gl['se_frac']:.1f} %; the 95 % interval of the mean "
                f"gives games_per_hour_steady_ci95) -- profiles/{gl_file}, tools/mcts_game_length.py"
                if gl is not None else None),
            "games_completed": games_done, "nn_evals_per_s": nn_rows / dt,
            "nn_tflops": nn_rows * FLOP_PER_EVAL / dt / 1e12, "gather_ms": gather_ms,
            "gather": ((f"{'RCCL' if backend == 'nccl' else backend} gather to rank 0 of the timed region's "
                        "device-resident (s, pi, z): 80-B records + the root visit counts of each record's "
                        "legal moves (uint16 each, plus a 2-B count)"
                        if mcts else f"{'RCCL' if backend == 'nccl' else backend} gather to rank 0 of the timed "
                        "region's device-resident records") if world > 1 else "none at N=1 (no collective)"),
            "records_gathered": n_records, "gathered_bytes": gathered_bytes,
            "gathered_bytes_per_record": (gathered_bytes / n_records) if n_records else None,
            "mean_plies_per_game": mean_len,
            "tree_overflows": m["tree_overflows"],
            "roofline": {"bound": "mfma",
                         "kernel": kname + kdesc + (
                             "; GEMM only: the operands' int8 digits come from the previous output kernel "
                             "(wino88i32_out_kernel, which writes them instead of fp32 V; conv2's from a slice "
                             "kernel)" if path == 6 else
                             "; GEMM only: the operands' int8 digits come from the previous output kernel "
                             "(wino88i32v_out_kernel: the fp64 input transform of the fp32 activation, cut to 4 digits; "
                             "conv2's from a slice kernel)" if path == 7 else
                             "; GEMM only: the operands' 3 radix-256 int8 digits come from the previous output kernel "
                             "(wino88i32_out_kernel<., ., 512, true>; conv2's from a slice kernel)" if path == 9 else ""),
                         "measured_peak_note": (f"v_mfma_i32_32x32x32_i8 back to back: {I8_MFMA_MEASURED_TOPS:.0f} "
                                                "TOPS at the clock held (profiles/r04_mfma_rate.log)"
                                                if path in I8_DIGIT_PRODUCTS else None),
                         "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "operations": ("int8 multiply-adds of the digit products (2 operations each) against the "
                                        "dense int8 MFMA peak" if path in I8_DIGIT_PRODUCTS else
                                        "fp64 MFMA FLOP" if path == 3 else "fp32 MFMA FLOP"),
                         "frac": (achieved / peak) if achieved else None,
                         "traffic": traffic, "traffic_source": ("profiles/" + traffic_src) if traffic_src else None,
                         "avg_launch_ms": conv_ms, "boards_per_launch": bpl,
                         "flop_per_launch": flop_alg, "mfma_flop_per_launch_incl_padding": m["dom_flop"],
                         "sclk_mhz": clock["sclk_mhz"] if clock else None, "clock": clock,
                         "clock_ranks": clock_ranks,
                         "direct_conv_equiv_tflops": (FLOP_RES_CONV_PER_BOARD * bpl / (conv_ms * 1e-3) / 1e12
                                                      if conv_ms > 0 else None)},
        }
        if tree_hbm is not None:
            out["tree_hbm"] = tree_hbm
        if direct is not None:
            d_ach = (FLOP_RES_CONV_PER_BOARD * G / (direct["conv_ms"] * 1e-3) / 1e12) if direct["conv_ms"] > 0 else None
            out["fp32_direct"] = {
                "note": "same fp32 network with the direct implicit-GEMM convs (exact fp32 products, 9 taps)",
                "value": (direct["sims"] if mcts else direct["plies"]) / direct["dt"], "unit": unit,
                "ms_per_step": direct["dt"] * 1e3 / direct["steps"],
                "res_conv_avg_launch_ms": direct["conv_ms"], "res_conv_tflops": d_ach,
                "res_conv_frac": (d_ach / FP32_MFMA_PEAK_TFLOPS) if d_ach else None}
        out["calibration"] = dict(m["calibration"], note=(
            "the network's conv paths for these weights: fp32 + AUTO measures its candidates at load time against an "
            "fp64 forward on 64 seeded boards and keeps the fastest within max |dlogit| 4e-5 / |dvalue| 4e-6 "
            "(F(8x8) fp32 with int8-digit GEMMs, the same with fp64 input transforms, the fp64 Winograd domain on 4 radix-256 then 5 radix-128 int8 digits, else on fp64 MFMA); "
            "errors are max |x - fp64|"))
        out["conv_path"] = PATH_NAMES.get(path)
        out["conv_arithmetic"] = {
            6: "fp32 network (fp32 activations, fp32 Winograd transforms, U, V and M); each Winograd GEMM on int8 "
               "digits: per-row 28-bit block fixed point (4 int8 digits per value under its row's exponent), the 10 "
               "digit pairs i + j <= 3 of 16 as v_mfma_i32_32x32x32_i8 chains, exact int32 levels, exact combine, one "
               "rounding to fp32 -- closer to the fp64 result than fp32 MFMA accumulation (calibration errors above; "
               "per-element bound vs the fp64 product tested; fp32_winograd88 is the fp32 MFMA tower)",
            2: "fp32 network, Winograd GEMMs on v_mfma_f32_32x32x2_f32",
            1: "fp32 network, Winograd F(4x8) GEMMs on v_mfma_f32_32x32x2_f32",
            5: "fp32 activations, fp64 Winograd domain, GEMMs on 5 int8 digits per value (per-row 35-bit block fixed "
               "point, 15 of 25 digit pairs, exact int32 levels, exact fp64 combine)",
            8: "fp32 activations, fp64 Winograd domain, GEMMs on 4 radix-256 int8 digits per value (per-row 31-bit "
               "block fixed point, 13 of 16 digit pairs, exact int32 levels, fp64 combine)",
            7: "fp32 network with fp64 input transforms (V cut to 4 int8 digits from fp64); GEMMs as path 6",
            9: "fp32 network (fp32 activations, fp32 Winograd transforms, U, V and M); each Winograd GEMM on 3 "
               "radix-256 int8 digits per value: per-row 24-bit block fixed point (N = rint(a 2^(23-e)) as balanced "
               "bytes), the 6 digit pairs i + j <= 2 of 9 as v_mfma_i32_32x32x32_i8 chains, exact int32 levels, "
               "exact combine, one rounding to fp32 (calibration errors above)",
            3: "fp32 activations, fp64 Winograd domain on v_mfma_f64",
            0: "fp32 direct implicit-GEMM convs"}.get(path)
        if pg_info is not None:
            out["process_group"] = pg_info
        if calib_ranks is not None:
            out["calibration_ranks"] = calib_ranks
        if trained is not None:
            tp = trained["dom_path"]
            t_ach = (FLOP_WINO88_GEMM_PER_BOARD * bpl / (trained["conv_ms"] * 1e-3) / 1e12) \
                if trained["conv_ms"] > 0 else None
            out["trained_weights_path"] = {
                "note": "the same workload on the stress weights (weights.stress_state_dict: trained-network "
                        "magnitudes, BN statistics of the data, logits of std 4 -- what a checkpoint looks like, "
                        "scripts/self_play.py:71-77) under fp32 + AUTO: no fp32 Winograd tower holds the 1e-4 "
                        "logit tolerance there, so the calibration picks the fp64 Winograd domain with int8-digit "
                        "GEMMs (4 radix-256 digits when they hold the budget, else 5 radix-128 ones); the peaked "
                        "priors give the trees their own shapes",
                "weights": "stress", "conv_path": PATH_NAMES.get(tp),
                "calibration": {k: trained["calibration"][k] for k in ("path_large", "path_small", "err_logit",
                                                                      "err_value", "ms")},
                "value": (trained["sims"] if mcts else trained["plies"]) / trained["dt"], "unit": unit,
                "steps": trained["steps"], "warmup": trained["warmup"],
                "ms_per_step": trained["dt"] * 1e3 / trained["steps"],
                "dominant_kernel": trained["dom_kernel"], "res_gemm_avg_launch_ms": trained["conv_ms"],
                "res_gemm_fp64_equiv_tflops": t_ach if tp == 5 else None,
                "res_gemm_i8_tops": (t_ach * I8_DIGIT_PRODUCTS[tp]) if (t_ach and tp in I8_DIGIT_PRODUCTS) else None,
                "peak_i8_tops": I8_MFMA_PEAK_TOPS,
                "res_gemm_frac_i8": (t_ach * I8_DIGIT_PRODUCTS[tp] / I8_MFMA_PEAK_TOPS)
                if (t_ach and tp in I8_DIGIT_PRODUCTS) else None,
                "res_gemm_over_fp64_mfma_peak": (t_ach / FP64_MFMA_PEAK_TFLOPS) if (t_ach and tp == 5) else None}
        if f64w is not None:
            f_ach = (FLOP_WINO88_GEMM_PER_BOARD * bpl / (f64w["conv_ms"] * 1e-3) / 1e12) if f64w["conv_ms"] > 0 \
                else None
            out["f64w_path"] = {
                "note": "the fp64 Winograd domain on v_mfma_f64 (KV_PREC_F64W)",
                "value": (f64w["sims"] if mcts else f64w["plies"]) / f64w["dt"], "unit": unit,
                "steps": f64w["steps"], "warmup": f64w["warmup"], "ms_per_step": f64w["dt"] * 1e3 / f64w["steps"],
                "dominant_kernel": f64w["dom_kernel"], "res_gemm_avg_launch_ms": f64w["conv_ms"],
                "res_gemm_tflops": f_ach, "peak": FP64_MFMA_PEAK_TFLOPS,
                "res_gemm_frac_fp64": (f_ach / FP64_MFMA_PEAK_TFLOPS) if f_ach else None}
        if alt_algo is not None:
            aa = alt_algo
            per = {1: FLOP_WINO48_GEMM_PER_BOARD, 2: FLOP_WINO88_GEMM_PER_BOARD}.get(aa["dom_path"],
                                                                                    FLOP_RES_CONV_PER_BOARD)
            aa_ach = (per * bpl / (aa["conv_ms"] * 1e-3) / 1e12) if aa["conv_ms"] > 0 else None
            out["fp32_" + args.alt_algo] = {
                "note": ("the same fp32 F(8x8) tower with its GEMMs on v_mfma_f32_32x32x2_f32 (fp32 products, "
                         "fp32 accumulation after every product; KV_ALGO_WINOGRAD88)" if aa["dom_path"] == 2
                         else f"the same fp32 network with algo {args.alt_algo}"),
                "value": (aa["sims"] if mcts else aa["plies"]) / aa["dt"], "unit": unit,
                "steps": aa["steps"], "warmup": aa["warmup"], "ms_per_step": aa["dt"] * 1e3 / aa["steps"],
                "res_gemm_avg_launch_ms": aa["conv_ms"], "res_gemm_tflops": aa_ach,
                "res_gemm_frac": (aa_ach / FP32_MFMA_PEAK_TFLOPS) if aa_ach else None}
        if alt is not None:
            # dominant launch of the alternate run (Winograd GEMM or direct residual conv), fp32-equivalent FLOPs
            a_ach = (alt["dom_flop"] / (alt["conv_ms"] * 1e-3) / 1e12) if alt["conv_ms"] > 0 else None
            a_prod = None  # bf16-class MFMA products per fp32 product (none of the remaining precisions)
            notes = {
                "f64w": "the fp64 Winograd domain on v_mfma_f64 (KV_PREC_F64W)",
                "i8r4": "the fp64 Winograd domain on 4 radix-256 int8 digits (KV_PREC_I8R4)",
                "i8x5": "the fp64 Winograd domain on 5 radix-128 int8 digits (KV_PREC_I8X5)"}
            out["alt_precision"] = {
                "precision": args.alt_precision, "note": notes.get(args.alt_precision, ""),
                "value": (alt["sims"] if mcts else alt["plies"]) / alt["dt"], "unit": unit,
                "steps": alt["steps"], "warmup": alt["warmup"],
                "ms_per_step": alt["dt"] * 1e3 / alt["steps"], "plies_per_s": alt["plies"] / alt["dt"],
                "nn_tflops_fp32_equiv": alt["nn_rows"] * FLOP_PER_EVAL / alt["dt"] / 1e12,
                "dominant_kernel": alt["dom_kernel"],
                "dominant_avg_launch_ms": alt["conv_ms"], "dominant_tflops_fp32_equiv": a_ach,
                "dominant_bf16_mfma_frac": (a_ach * a_prod / BF16_MFMA_PEAK_TFLOPS) if (a_ach and a_prod) else None}
        if refsel is not None:
            out["ref_selection"] = {
                "note": f"C{'3' if G == 2048 else '2' if G == 256 else ''}-ref: the reference's own move selection "
                        "(sims=0: one network row per ply, softmax + Dirichlet + random.choices) on the same "
                        f"{G} slots, uncapped games, slots recycled; games/hour counts games completed inside the "
                        "timed region",
                "slots": G, "plies_per_s": refsel["plies"] / refsel["dt"],
                "games_per_hour": refsel["games_done"] / refsel["dt"] * 3600.0,
                "games_completed": refsel["games_done"], "timed_s": refsel["dt"], "steps": refsel["steps"],
                "warmup": refsel["warmup"],
                "reference_cpu": {"plies_per_s": 250.0, "games_per_hour": 2424.0,
                                  "source": "BASELINE.md: reference self_play.py (SELFPLAY_SEQ=1) on 8 Xeon cores"}}
            if reflazy is not None:
                out["ref_selection"]["lazy_eval_side_figure"] = {
                    "note": "NOT the measured games/hour: the same games (identical records, "
                            "tests/test_engine_gpu.py::test_compact_lazy_eval_matches_faithful) with the network run "
                            "only on the rows the reference's schedule reads -- self_play.py evaluates a 16-board "
                            "buffer and uses its last row (:129-150); here those rows alone form one compact batch "
                            "per ply-step (KV_EVAL_LAZY)",
                    "plies_per_s": reflazy["plies"] / reflazy["dt"],
                    "games_per_hour": reflazy["games_done"] / reflazy["dt"] * 3600.0,
                    "games_completed": reflazy["games_done"], "timed_s": reflazy["dt"],
                    "network_rows": reflazy["nn_rows_evaluated"], "faithful_network_rows": reflazy["nn_rows"]}
            # reference / port on identical work at one torch thread per process, as the pool runs
            cal = os.path.join(HERE, "profiles", "r03_cpu_calibration_1thread.json")
            if not args.no_cpu_baseline and world == 1:
                # the reference's selection restated on this box's host cores, and the reference-equivalent rate
                # through the container calibration (reference / port on identical work, tools/calibrate_cpu.py)
                port = cpu_baseline(min(args.cpu_seconds, 10.0), 0)
                out["ref_selection"]["cpu_port_box"] = port
                if os.path.exists(cal):
                    r = json.load(open(cal))["ref_over_port"]
                    eq = port["value"] * r
                    out["ref_selection"]["reference_equiv_box"] = {
                        "plies_per_s": eq, "ref_over_port": r, "source": os.path.relpath(cal, HERE),
                        "gpu_over_reference_equiv": (refsel["plies"] / refsel["dt"]) / eq}
        if not args.no_cpu_baseline and world == 1:  # the CPU leg is timed at N=1 only
            if mcts:
                # two CPU restatements of the same search: leaves batched per process (the GPU's batch shape) and
                # one leaf per network call; `cpu_baseline` is the faster, the other is reported beside it
                b16 = cpu_baseline(args.cpu_seconds * 2 / 3, sims, batch=args.cpu_leaf_batch)
                b1 = cpu_baseline(args.cpu_seconds / 3, sims, batch=1)
                fast, slow = (b16, b1) if b16["value"] >= b1["value"] else (b1, b16)
                out["cpu_baseline"] = dict(fast, other_leg=slow, gpu_over_cpu=value / fast["value"])
            else:
                out["cpu_baseline"] = cpu_baseline(args.cpu_seconds, sims)
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()
    return 0


if __name__ == "__main__":
    sys.exit(main())
