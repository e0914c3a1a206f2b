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
    tj, f = bench._tree_pmc(2048)
    assert tj["sims_per_move"] == 800 and tj["per_sim"]["bytes_per_sim"] > 0
    m = tj["measured"]
    assert m["hash_evaluator_800_sims"]["launches"] == 799
    est = m["network_300_sims"]["bytes_per_sim"] * m["growth_300_to_800"]
    assert abs(est - tj["per_sim"]["bytes_per_sim"]) < 1e-6 * est


def test_gemm_traffic_summary_present():
    t, f = bench._pmc_traffic("wino_gemm_kernel<512,4,2,1,2,32,60>", 2048)
    assert t is not None and t > 1.0e9
    # the default fp32 tower's GEMM (F(8x8)) at C3's 2,048 boards: 0.94 GB algorithmic per launch
    t, f = bench._pmc_traffic("wino_gemm_kernel<512,4,2,1,2,32,100>", 2048)
    assert t is not None and 0.94e9 <= t < 1.2e9


@pytest.mark.parametrize("rows,cus,xa", [(2048, 256, 100), (1024, 256, 96), (512, 256, 96), (256, 256, 64),
                                         (384, 256, 100), (128, 256, 100), (64, 256, 100), (2048, 304, 95)])
def test_w88_split_rule(monkeypatch, rows, cus, xa):
    """bench.py's label of the F(8x8) GEMM layer mirrors kv_nn.hip wino88_split_points: the points whose
    128x128 tiles fill whole rounds of 2 workgroups per CU, unless the last round of the one-launch grid is
    empty or puts exactly one tile on every CU (then one launch)."""
    monkeypatch.delenv("KV_W88_SPLIT", raising=False)
    got = bench._w88_split_points(rows, cus)
    assert got == xa
    if got < 100:
        assert (got * (rows // 128) * 4) % (2 * cus) == 0


@pytest.mark.parametrize("sims", [0, 8])
def test_cpu_baseline_pool(monkeypatch, sims):
    monkeypatch.setenv("KV_CPU_WORKERS", "2")
    r = bench.cpu_baseline(2.0, sims)
    assert r["kind"] == "port" and r["workers"] == 2 and r["cores"] == 2 and r["threads_per_worker"] == 1
    assert r["value"] > 0 and r["unit"] == ("sims/s" if sims else "plies/s")
    assert r["whole_host_extrapolated"] >= r["value"]
    json.dumps(r)
