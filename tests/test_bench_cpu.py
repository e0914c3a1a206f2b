"""bench.py's contract pieces that need no GPU: the committed measurement
summaries it reads (steady-state game length, tree-kernel HBM bytes, GEMM PMC
traffic) and the pooled CPU baseline (oracle restatement, test
infrastructure)."""
import json
import os

import pytest

import bench


def test_game_length_summary_is_complete_and_tight():
    gl, f = bench._mcts_game_length(800)
    assert gl is not None and f.startswith("r03_")
    assert gl["still_running"] == 0 and gl["finished"] == gl["games"] >= 256
    assert gl["se_frac"] <= 0.05  # SE <= 5 %
    lo, hi = gl["ci95_mean_plies"]
    assert lo < gl["mean_plies_finished"] < hi
    assert sum(gl["reasons"].values()) == gl["finished"] and len(gl["plies"]) == gl["finished"]


def test_tree_summary_is_at_c3_sims():
    """The tree-kernel HBM figure the bench line carries is measured at C3 itself (800 sims, round 4); it
    agrees with round 3's derived estimate (300-sim network run x the hash evaluator's growth)."""
    tj, f = bench._tree_pmc(2048)
    assert f.startswith("r04_") and tj["measured_directly"]
    assert tj["sims_per_move"] == 800 and tj["per_sim"]["bytes_per_sim"] > 0
    old = json.load(open(os.path.join(os.path.dirname(bench.__file__), "profiles", "r03_pmc_tree_c3_2048.json")))
    assert abs(old["per_sim"]["bytes_per_sim"] / tj["per_sim"]["bytes_per_sim"] - 1) < 0.02


def test_gemm_traffic_summary_present():
    t, f = bench._pmc_traffic("wino_gemm_kernel<512,4,2,1,2,32,60>", 2048)
    assert t is not None and t > 1.0e9
    # the default fp32 tower's GEMM (F(8x8)) at C3's 2,048 boards: 0.94 GB algorithmic per launch
    t, f = bench._pmc_traffic("wino_gemm_kernel<512,4,2,1,2,32,100>", 2048)
    assert t is not None and 0.94e9 <= t < 1.2e9
    # the int8-digit GEMMs (fp32 tower: 4 digits, fp32 M; fp64 domain: 5 digits, fp64 M)
    t, f = bench._pmc_traffic("wino88i_gemm_kernel<512,4,true,float,true>", 2048)
    assert t is not None and 0.94e9 <= t < 1.2e9
    t, f = bench._pmc_traffic("wino88i_gemm_kernel<512,5,true,double>", 2048)
    assert t is not None and 1.49e9 <= t < 1.8e9


@pytest.mark.parametrize("path,rows,split,name", [
    (2, 2048, 100, "wino_gemm_kernel<512,4,2,1,2,32,100>"), (2, 256, 64, "wino_gemm_kernel<512,4,2,1,2,32,100>"),
    (2, 320, 100, "wino_gemm_kernel<512,2,2,1,2,16,100>"), (2, 32, 100, "wino_gemm_kernel<512,1,2,1,2,32,100>"),
    (2, 96, 100, "wino_gemm_kernel<512,1,2,1,2,16,100>"), (3, 2048, 0, "wino88d_gemm_kernel<512,2,4,4,2>"),
    (3, 64, 0, "wino88d_gemm_kernel<512,1,4,4,2>"), (3, 32, 0, "wino88d_gemm_kernel<512,1,4,2,2>"),
    (1, 4096, 0, "wino_gemm_kernel<512,4,2,1,2,32,60>"), (0, 2048, 0, "conv3x3_kernel<512,32>"),
    (5, 2048, 0, "wino88i_gemm_lag5_kernel<512,3,5,7,false>"), (8, 2048, 0, "wino88i_gemm_lag5_kernel<512,3,4,8,true>"),
    (6, 2048, 0, "wino88i32_gemm_lagt_kernel<512,5>"),
    (6, 256, 0, "wino88i32_gemm_lagt_kernel<512,4>"), (6, 128, 0, "wino88i32_gemm_lag_kernel<512,false>"),
    (6, 1024, 0, "wino88i32_gemm_lag_kernel<512,false>")])
def test_gemm_label(path, rows, split, name):
    """bench.py names the dominant GEMM launch as kv_nn.hip picks it (rows per point; the F(8x8) point split
    is the one the library reports in kv_stats.dom_split, not re-derived)."""
    got, desc = bench.gemm_label(path, rows, split)
    assert got == name
    assert (f"points 0-{split - 1}" in desc) == (path == 2 and split < 100)


@pytest.mark.parametrize("sims,batch", [(0, 1), (8, 1), (8, 4)])
def test_cpu_baseline_pool(monkeypatch, sims, batch):
    monkeypatch.setenv("KV_CPU_WORKERS", "2")
    r = bench.cpu_baseline(2.0, sims, batch=batch)
    assert r["kind"] == "port" and r["workers"] == 2 and r["cores"] == 2 and r["threads_per_worker"] == 1
    assert r["leaf_batch"] == batch
    assert r["value"] > 0 and r["unit"] == ("sims/s" if sims else "plies/s")
    assert r["whole_host_extrapolated"] >= r["value"]
    json.dumps(r)
