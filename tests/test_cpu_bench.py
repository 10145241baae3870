"""bench.py's host-side contract pieces, on the CPU: the fraction guard, the config naming, the L2 weight-stream
arithmetic and the committed measurement records the bench line quotes (every fraction in them a fraction of a
true peak, every record keyed the way bench.py looks it up)."""
import json
import os
import sys

import pytest

ROOT = os.path.join(os.path.dirname(os.path.abspath(__file__)), "..")
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "muzero-breakout_amd"))
import bench  # noqa: E402


def test_check_fracs_fails_on_any_fraction_above_one():
    ok = {"roofline": {"frac": 0.96, "executed_frac": 0.68, "l2_weight_stream": {"frac": 0.59},
                       "kernel_timed": {"frac": 0.41}}, "parity_path": {"roofline": {"frac": 0.93}}}
    bench.check_fracs(ok)
    for bad in ({"roofline": {"frac": 1.0001}}, {"parity_path": {"roofline": {"frac": 1.59}}},
                {"roofline": {"l2_weight_stream": {"frac": 1.058}}}, {"roofline": {"executed_frac": 1.2}}):
        with pytest.raises(SystemExit):
            bench.check_fracs(bad)
    bench.check_fracs({"roofline": {"fraction_note": 3.0, "frac": None}})  # only numeric *frac keys are checked


def test_cfg_name_maps_the_baseline_configs():
    assert bench.cfg_name(4096, 50).startswith("north_star")
    assert bench.cfg_name(1024, 50) == "config 2"
    assert bench.cfg_name(4096, 200, "fp16") == "config 5"
    assert bench.cfg_name(4096, 200, "bf16").startswith("config 5 geometry")
    assert bench.cfg_name(512, 50) == "custom"


def test_l2_weight_stream_arithmetic():
    r = bench.l2_weight_stream(0.0147)  # a 14.7 us tower conv
    assert r["bytes_per_cu_per_conv"] == 256 * 9 * 256 * 2
    assert abs(r["achieved_per_cu_GBps"] - 1179648 / 14.7e-6 / 1e9) < 1e-6
    assert abs(r["peak_per_cu_GBps"] - bench.L2_PEAK_TBPS * 1e3 / 256) < 1e-9
    assert abs(r["frac"] - r["achieved_per_cu_GBps"] / r["peak_per_cu_GBps"]) < 1e-12
    assert bench.l2_weight_stream(None) is None


def test_env_bytes_and_committed_env_kernel_times():
    assert bench.env_bytes(84, 84) == 7104 and bench.env_bytes(16, 20) == 368
    recs = json.load(open(os.path.join(ROOT, "profiles", "env_kernel_time.json")))
    assert {(r["H"], r["W"], r["hist"]) for r in recs} >= {(84, 84, 4), (16, 20, 32)}
    for r in recs:
        assert r["kernel"].startswith("env_step_compact_kernel") and r["calls"] > 0
        assert 0 < r["min_ns"] <= r["avg_ns"]
        gbps = r["envs"] * bench.env_bytes(r["H"], r["W"]) / (r["avg_ns"] * 1e-9) / 1e9
        assert gbps / 8000.0 <= 1.0
        assert os.path.exists(os.path.join(ROOT, r["source"]))


def test_committed_tower_records_are_keyed_as_bench_reads_them():
    traffic = json.load(open(os.path.join(ROOT, "profiles", "tower_hbm_traffic.json")))["records"]
    for rec in traffic:
        assert isinstance(rec["envs"], int) and rec["kernel_name"] in bench.EXECUTED_FRACTION
        assert rec["bytes_per_launch"] >= rec["algorithmic_bytes"] > 0
    counters = json.load(open(os.path.join(ROOT, "profiles", "tower_sq_counters.json")))["records"]
    keys = [(r.get("envs"), r.get("kernel_name"), r.get("sims", 50), r.get("dyn_dtype")) for r in counters]
    assert len(keys) == len(set(keys))  # one record per (batch, instance, sims, dynamics precision)
    for r in counters:
        for k, v in r.items():
            if (k == "frac" or k.endswith("_frac") or k.endswith("_busy")) and isinstance(v, float):
                assert 0.0 <= v <= 1.0, (k, v)
    headline = [r for r in counters if (r.get("envs"), r.get("kernel_name")) == (4096, "towerp_kernel<0>")
                and r.get("sims", 50) == 50]
    assert headline, "the north_star line's counters"


def test_conv_counter_record_for_config3():
    """The non-fused path's PMC record (config 3's halo conv at the 21x21 latent): found by bench.conv_counters for
    the config 3 batch and latent size only; traffic at least the algorithmic bytes, fractions within [0, 1]."""
    rec = bench.conv_counters(4096, 21, 21, "conv_halo_kernel")
    assert rec is not None and rec["kernel_name"].startswith("conv_halo_kernel<256, 1, 2, 1, 256, false>")
    assert rec["bytes_per_launch"] >= rec["algorithmic_bytes"] > 0
    for k in ("mfma_busy", "wait_inst", "lds_bank_conflict_frac"):
        assert 0.0 <= rec[k] <= 1.0
    assert os.path.isdir(os.path.join(ROOT, rec["source"]))
    assert bench.conv_counters(1024, 21, 21, "conv_halo_kernel") is None
    assert bench.conv_counters(4096, 4, 5, "conv_halo_kernel") is None


def test_learner_kernel_breakdown_record():
    rec = bench.learner_kernels(512, "bf16")
    assert rec is not None and rec["kernels"][0]["kernel"].startswith("conv_lat_kernel")
    shares = [k["share_of_kernel_time"] for k in rec["kernels"]]
    assert shares == sorted(shares, reverse=True) and sum(shares) <= 1.0
    assert bench.learner_kernels(512, "f32") is None and bench.learner_kernels(256, "bf16") is None
    bench.check_fracs({"roofline": {"top_kernels": rec}})


def test_self_launcher_argv_runs_n_ranks_of_this_bench():
    argv = bench.launcher_argv(8, ["--gpus", "8", "--steps", "5"], 29511)
    assert argv[1:3] == ["-m", "torch.distributed.run"]
    assert "--nproc-per-node=8" in argv and "--nnodes=1" in argv and "--master-addr=127.0.0.1" in argv
    assert "--master-port=29511" in argv
    i = argv.index(os.path.abspath(bench.__file__))
    assert argv[i + 1:] == ["--gpus", "8", "--steps", "5"]


def test_world_size_mismatch_is_refused():
    assert bench.world_from_env(1, {}) == (1, 0, 0)
    assert bench.world_from_env(4, {"WORLD_SIZE": "4", "RANK": "2", "LOCAL_RANK": "2"}) == (4, 2, 2)
    for gpus, ws in ((8, "4"), (1, "2"), (2, "1")):
        with pytest.raises(SystemExit):
            bench.world_from_env(gpus, {"WORLD_SIZE": ws, "RANK": "0", "LOCAL_RANK": "0"})


def test_self_launched_ranks_report_ranks_seen(tmp_path):
    """`bench.py --gpus 2` with no torchrun environment starts two ranks itself; a gloo rehearsal of the launcher
    path (the bench's --workload selfcheck: process group only, no GPU) prints ranks_seen 2 from rank 0 only."""
    import subprocess
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    env["MZBA_DIST_REHEARSAL"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--workload", "selfcheck"],
                       capture_output=True, text=True, env=env, timeout=240)
    assert r.returncode == 0, r.stderr[-2000:]
    lines = [json.loads(x) for x in r.stdout.splitlines() if x.startswith("{")]
    assert len(lines) == 1
    assert lines[0]["n_gpus"] == 2 and lines[0]["ranks_seen"] == 2 and lines[0]["backend"] == "gloo"


def test_fp16_clock_record():
    """Config 5's fp16 note: the committed probe record has both element types and the ratios bench.py quotes."""
    r = bench.fp16_clock_note()
    assert r is not None and 0 < r["fp16_over_bf16_clock"] <= 1.0 and 0 < r["fp16_over_bf16_rate"] <= 1.0
    assert os.path.exists(os.path.join(ROOT, "profiles", "r06", "r6l", "mfma_clock_dtype.jsonl"))
