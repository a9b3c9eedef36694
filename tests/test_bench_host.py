"""bench.py's host logic on the CPU: the algorithmic FLOP counts, the workloads against
BASELINE.json's configs, the roofline record (traffic per launch x passes for the CEM line), the committed PMC
traffic file the bench quotes, and the CPU-baseline record's thread choice (the oracle at a tiny K).  The GPU
lines themselves run in the driver's bench and in tests/test_gpu_*.py."""
import json
import time
import os

import numpy as np
import pytest

import bench

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_flop_per_cand_step_matches_survey():
    # 2*[(S+A)h + (L-1)h^2 + hS]: 2x500 546,000; 2x256 154,624; 3x1024 4,288,512
    assert bench.flop_per_cand_step(500, 2) == 546000
    assert bench.flop_per_cand_step(256, 2) == 154624
    assert bench.flop_per_cand_step(1024, 3) == 4288512


def test_workloads_are_baseline_configs():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))["configs"]
    assert "K=1000, H=15" in base[0] and "K=4096, H=20" in base[1] and "K=65536, H=20" in base[2]
    assert "K=262144, H=20" in base[3] and "8" in base[3]
    W = bench.WORKLOADS
    assert (W["cfg1"]["K"], W["cfg1"]["H"]) == (1000, 15)
    assert (W["cfg2"]["K"], W["cfg2"]["H"]) == (4096, 20)
    assert (W["cfg3"]["K"], W["cfg3"]["H"]) == (65536, 20)
    assert W["cfg4_shard"]["K"] * 8 == 262144 and W["cfg4_shard"]["H"] == 20
    for name in ("cfg1", "cfg2", "cfg3", "cfg4_shard"):
        assert (W[name]["hidden"], W[name]["L"], W[name]["act"]) == (500, 2, "tanh"), name
    c5 = W["cfg5"]
    assert (c5["K"], c5["H"], c5["hidden"], c5["L"], c5["act"]) == (65536, 50, 1024, 3, "tanh")
    assert c5["cem"]["iterations"] == 4


def test_roofline_line_counts_every_cem_pass():
    fpcs = bench.flop_per_cand_step(1024, 3)
    one = bench.roofline_line(65536, 50, fpcs, 37.5, "split", iters=1, traffic_key="cfg5:split:device")
    four = bench.roofline_line(65536, 50, fpcs, 150.0, "split", iters=4, traffic_key="cfg5:split:device")
    assert four["flop_per_launch"] == 4 * one["flop_per_launch"]
    assert four["achieved"] == pytest.approx(one["achieved"])        # 4x the work in 4x the time
    assert four["frac"] == pytest.approx(four["achieved"] / bench.SPLIT_PEAK_TFLOPS)
    if one["traffic"] is not None:
        assert four["traffic"] == pytest.approx(4 * one["traffic"])
        assert "x 4 passes" in four["traffic_source"]
    f16 = bench.roofline_line(65536, 20, bench.flop_per_cand_step(500, 2), 0.78, "f16")
    assert f16["peak"] == bench.F16_MFMA_PEAK_TFLOPS and "traffic" not in f16


def test_committed_traffic_file_covers_the_bench_lines():
    path = os.path.join(REPO, "profiles", bench.TRAFFIC_FILE)
    tr = json.load(open(path))
    for key in ("cfg3:split:device", "cfg3:f16:device", "cfg2:split:device", "ns_shard:split:device",
                "cfg4_shard:split:device", "cfg5:split:device"):
        assert key in tr, key
        rec = tr[key]
        # every XCD misses the packed weights into its own L2: measured bytes >= the algorithmic ones
        assert rec["hbm_bytes_per_launch"] >= rec["algorithmic_bytes_per_launch"] > 0, key
        assert rec["dispatches"] >= 1 and "rollout" in rec["kernel"]
    assert bench.pmc_traffic("cfg3:split:device") == tr["cfg3:split:device"]["hbm_bytes_per_launch"]
    assert bench.pmc_traffic("no-such-line") is None


def test_cpu_baseline_record_and_thread_choice():
    wl = dict(K=64, H=2, hidden=32, L=2, act="tanh")
    prob = bench.synthetic_problem(wl)
    from oracle import mpc_oracle as orc
    w = orc.MLPWeights(prob["kernels"], prob["biases"], "tanh", None, None)
    rec = bench.cpu_baseline(w, prob["norm"], prob["state"], wl["H"], 0.2, wl["K"], "2x32 tanh")
    assert rec["kind"] == "port" and rec["unit"] == "candidate-steps/s"
    assert rec["value"] == max(rec["value_pool"], rec["value_1thread"])
    assert rec["cores"] == (rec["pool_threads"] if rec["value_pool"] >= rec["value_1thread"] else 1)
    assert rec["K_sampled_pool"] == 64 and 64 <= rec["K_sampled_1thread"] <= 64
    assert rec["host_cpus"] == os.cpu_count()
    assert "OpenBLAS" in rec["sample"] and "1 thread" in rec["sample"]
    assert np.isfinite(rec["value"]) and rec["value"] > 0


def test_launch_plan_follows_gpus_and_world_size():
    # the driver's N=1 form and the self-launch form (no WORLD_SIZE)
    assert bench.launch_plan(1, {}) == "single"
    assert bench.launch_plan(8, {}) == "spawn"
    assert bench.launch_plan(2, {"WORLD_SIZE": ""}) == "spawn"
    # torch.distributed.run started us: WORLD_SIZE must equal --gpus
    assert bench.launch_plan(8, {"WORLD_SIZE": "8"}) == "ranks"
    assert bench.launch_plan(1, {"WORLD_SIZE": "1"}) == "ranks"
    with pytest.raises(SystemExit, match="WORLD_SIZE=4 but --gpus 8"):
        bench.launch_plan(8, {"WORLD_SIZE": "4"})
    with pytest.raises(SystemExit):
        bench.launch_plan(0, {})


def test_spawn_command_is_a_child_torchrun_on_loopback():
    cmd = bench.spawn_command(4, ["--gpus", "4", "--steps", "3"], 29123)
    assert cmd[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--master-addr=127.0.0.1" in cmd and "--master-port=29123" in cmd
    assert cmd[-4:] == ["--gpus", "4", "--steps", "3"] and cmd[-5].endswith("bench.py")


@pytest.mark.parametrize("n", [1, 2, 3, 4, 8])
def test_workload_shard_strong_splits_the_global_k(n):
    """north_star: K = 65,536 GLOBAL over N ranks, contiguous, covering [0, K) once (distributed.shard_range);
    configs[3]: 262,144 -> 32,768 per GPU at N = 8."""
    from bc_mpc_amd.distributed import shard_range
    for K in (65536, 262144, 1000):
        parts = [bench.workload_shard(K, r, n, "strong") for r in range(n)]
        assert parts[0][0] == 0 and parts[-1][1] == K
        assert all(p[1] == q[0] for p, q in zip(parts, parts[1:]))
        assert all(p[2] == K for p in parts)
        assert [p[:2] for p in parts] == [shard_range(K, r, n) for r in range(n)]
    assert bench.workload_shard(65536, 7, 8, "strong") == (57344, 65536, 65536)
    assert bench.workload_shard(262144, 3, 8, "strong")[1] - bench.workload_shard(262144, 3, 8, "strong")[0] == 32768


def test_workload_shard_weak_keeps_k_per_rank():
    assert bench.workload_shard(65536, 0, 8, "weak") == (0, 65536, 524288)
    assert bench.workload_shard(65536, 5, 8, "weak") == (5 * 65536, 6 * 65536, 524288)


def test_summary_key_is_compact_and_covers_every_line():
    out = {"value": 6.9e8, "p50_ms": 1.88, "ms_per_step": 1.9, "roofline": {"frac": 0.4591234},
           "cfg2": {"value": 3.3e8, "p50_ms": 0.25, "roofline": {"frac": 0.25}},
           "ns_shard": {"value": 5e8, "p50_ms": 0.33, "roofline": {"frac": 0.3}},
           "scale": {"cfg4": {"value": 1e9, "ms_per_step": 5.0, "roofline": {"frac": 0.4}}, "cfg3_weak": "= the headline"},
           "small_k": {"ppo_defaults": {"p50_ms": 0.047, "roofline": {"frac": 0.01}}}}
    s = bench.summary_of(out)
    assert s["headline"] == {"value": 6.9e8, "p50_ms": 1.88, "ms_per_step": 1.9, "frac": 0.4591}
    assert s["small_k.ppo_defaults"]["p50_ms"] == 0.047
    assert s["scale.cfg4"]["frac"] == 0.4 and s["scale.cfg3_weak"] is None
    assert list(s)[0] == "headline" and "ns_shard" in s and "cfg2" in s


def test_ns_shard_is_the_north_star_per_gpu_shard():
    base = json.load(open(os.path.join(REPO, "BASELINE.json")))
    assert "K=65536" in base["north_star"] and "8" in base["north_star"]
    ns = bench.WORKLOADS["ns_shard"]
    assert ns["K"] * 8 == 65536 and ns["H"] == 20 and (ns["hidden"], ns["L"], ns["act"]) == (500, 2, "tanh")


def test_prewarm_runs_the_step_for_its_budget_with_fresh_seeds():
    seen = []

    def step(i):
        seen.append(i)
        time.sleep(0.002)
    rec = bench.prewarm(step, budget_s=0.02)
    assert rec["calls"] == len(seen) and 8 <= len(seen) <= 15 and rec["seconds"] >= 0.018
    assert len(set(seen)) == len(seen) and min(seen) >= 1 << 40          # never a timed step's seed
    seen.clear()
    assert bench.prewarm(step, fixed_calls=7)["calls"] == 7 == len(seen)
