"""bench.py's contract pieces that need no GPU: the committed measurement
summaries it reads (steady-state game length, tree-kernel HBM bytes, GEMM PMC
traffic) and the pooled CPU baseline (oracle restatement, test
infrastructure)."""
import json
import os

import pytest

import bench


def test_game_length_summary_is_complete_and_tight():
    """re-measured on the path the headline's AUTO chooses (round 6: R3), >= 256 games."""
    gl, f = bench._mcts_game_length(800, "winograd88_i8f32r3")
    assert gl is not None and f.startswith("r06_") and gl["conv_path"] == "winograd88_i8f32r3"
    assert gl["still_running"] == 0 and gl["finished"] == gl["games"] >= 256
    assert bench._mcts_game_length(800)[1] == f  # the newest run is the default too
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


@pytest.mark.parametrize("path,kernel,tpw", [
    (2, "wino_gemm_kernel<512,4,2,1,2,32,100>", 0),
    (2, "wino_gemm_kernel<512,4,2,1,2,32,100>+wino_gemm_kernel<512,2,2,1,2,16,100>", 0),
    (3, "wino88d_gemm_kernel<512,2,4,4,2>", 0), (1, "wino_gemm_kernel<512,4,2,1,2,32,60>", 0),
    (0, "conv3x3_kernel<512,32>", 0), (5, "wino88i_gemm_lag5_kernel<512,3,5,7,false>", 0),
    (8, "wino88i_gemm_lag5_kernel<512,3,4,8,true>", 0), (6, "wino88i32_gemm_lagt_kernel<512,5>", 5),
    (6, "wino88i32_gemm_lagt_kernel<512,4>", 4), (7, "wino88i32_gemm_lagt_kernel<512,5>", 5),
    (9, "wino88i32_gemm_r3k64_kernel<512,5>", 5), (9, "wino88i32_gemm_r3k64_kernel<512,4>", 4),
    (9, "wino88i32_gemm_lagt_kernel<512,5,3>", 5),
    # KV_I8F32_TPW=1 (or a CU count where multi-tile workgroups do not pay): the library reports the
    # single-tile kernel, and the line follows it
    (6, "wino88i32_gemm_lag_kernel<512,false>", 1)])
def test_gemm_label_is_the_librarys(path, kernel, tpw):
    """bench.py labels the dominant GEMM with the name the library reports for the launch it made
    (kv_stats.dom_kernel), not a rule re-derived in Python; the description follows the name."""
    got, desc = bench.gemm_label(path, kernel)
    assert got == kernel.partition("+")[0]
    assert ("second launch" in desc) == ("+" in kernel)
    if tpw:
        assert (f"{tpw} per workgroup" in desc) == (tpw > 1)


def test_roofline_units_of_every_f88_path():
    """the F(8x8) int8-digit paths 7 (fp64 input transforms) and 8 (radix-256 fp64 domain) are
    costed as F(8x8) GEMMs (100 points x 512 x 512 per board), not as the direct conv or F(4x8)."""
    G = 2048
    for path in (2, 3, 5, 6, 7, 8, 9):
        flop = 2.0 * 100 * G * 512 * 512
        per_board, bpl, rows = bench.dom_units(path, flop, G)
        assert per_board == bench.FLOP_WINO88_GEMM_PER_BOARD and bpl == G and rows == G, path
    assert bench.dom_units(1, 2.0 * 60 * 2 * G * 512 * 512, G) == (bench.FLOP_WINO48_GEMM_PER_BOARD, G, 2 * G)
    assert bench.dom_units(0, 0.0, G)[0] == bench.FLOP_RES_CONV_PER_BOARD


def test_pmc_traffic_follows_the_reported_kernel():
    """The PMC traffic is looked up by the reported kernel's name: the 5-tile kernel's summary exists at C3,
    and a single-tile report does not pick it up."""
    t5, f5 = bench._pmc_traffic("wino88i32_gemm_lagt_kernel<512,5>", 2048)
    assert t5 is not None and 0.94e9 <= t5 < 1.3e9
    t1, f1 = bench._pmc_traffic("wino88i32_gemm_lag_kernel<512,false>", 2048)
    assert f1 != f5
    # the headline's kernel since round 6 (R3, 64-k stages): its own summary, 3-digit V read + fp32 M written
    tk, fk = bench._pmc_traffic("wino88i32_gemm_r3k64_kernel<512,5>", 2048)
    assert tk is not None and fk.startswith("r06_") and 0.81e9 <= tk < 1.2e9


@pytest.mark.parametrize("G,sims,world,tag", [(2048, 800, 1, "configs[2], C3"), (2048, 800, 8, "configs[3], C4"),
                                              (256, 400, 1, "configs[1], C2"), (512, 800, 1, "")])
def test_workload_names_the_baseline_config(G, sims, world, tag):
    got = bench.baseline_config_tag(True, G, sims, world)
    assert (tag in got) if tag else got == ""


@pytest.mark.parametrize("sims,batch", [(0, 1), (8, 1), (8, 4)])
def test_cpu_baseline_pool(monkeypatch, sims, batch):
    monkeypatch.setenv("KV_CPU_WORKERS", "2")
    r = bench.cpu_baseline(2.0, sims, batch=batch)
    assert r["kind"] == "port" and r["workers"] == 2 and r["cores"] == 2 and r["threads_per_worker"] == 1
    assert r["leaf_batch"] == batch
    assert r["value"] > 0 and r["unit"] == ("sims/s" if sims else "plies/s")
    assert r["whole_host_extrapolated"] >= r["value"]
    json.dumps(r)
