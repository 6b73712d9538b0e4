"""The committed headline bench lines (profiles/r03_final_bench_line*.json, measured on an MI355X)
carry every field of the bench contract with consistent values: metric / unit from
BASELINE.json, value = iterations / timed seconds, roofline.frac = achieved / peak, the CPU
baseline object at N = 1, and the kernel-sum figures of BASELINE's metric."""
import json
import os

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LINES = ["r03_final_bench_line.json", "r03_final_bench_line_driver_form.json"]


def _load(name):
    with open(os.path.join(ROOT, "profiles", name)) as f:
        return json.load(f)


@pytest.mark.parametrize("name", LINES)
def test_headline_line_contract(name):
    d = _load(name)
    base = json.load(open(os.path.join(ROOT, "BASELINE.json")))
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["metric"] == base["metric"]
    assert d["n_gpus"] == 1 and d["higher_is_better"] is True and d["vs_baseline"] is None
    assert d["dtype"] == "f32" and d["data"] == "synthetic"
    assert "100000" in d["config"]["workload"]
    # one PSR iteration per step at N = 1
    assert d["value"] == pytest.approx(1000.0 / d["ms_per_step"], rel=2e-3)
    r = d["roofline"]
    for k in ("bound", "achieved", "peak", "unit", "frac", "traffic"):
        assert k in r, k
    assert r["bound"] in ("hbm", "mfma", "valu") and r["unit"] in ("GB/s", "TFLOP/s")
    assert r["frac"] == pytest.approx(r["achieved"] / r["peak"], rel=2e-3)
    assert 0.0 < r["frac"] <= 1.0
    # achieved = algorithmic flops per launch / average launch time
    assert r["achieved"] == pytest.approx(
        r["pairs_per_launch"] * r["flops_per_pair"] / (r["avg_launch_ms"] * 1e-3) / 1e12, rel=5e-3)
    c = d["cpu_baseline"]
    for k in ("value", "unit", "cores", "kind", "sample"):
        assert k in c, k
    assert c["kind"] in ("reference", "port") and c["cores"] >= 1 and c["value"] > 0
    ks = d["kernel_sum_100k"]
    assert ks["M"] == 100000 and ks["ms"] > 0
    assert ks["Tpair_per_s"] == pytest.approx(1e10 / (ks["ms"] * 1e-3) / 1e12, rel=2e-3)


def test_strong_scaling_atlas_line():
    d = _load("r03_final_bench_line_c4_fixed.json")
    assert d["scaling"] == "strong" and "32 frames" in d["config"]["workload"]
    assert d["value"] == pytest.approx(1000.0 / d["ms_per_step"], rel=2e-3)


# --- bench.py --gpus N: how the ranks are started (VERDICT r03 "Next round" 1) ---

def _bench():
    import importlib
    import sys
    sys.path.insert(0, ROOT)
    return importlib.import_module("bench")


def test_launch_plan_single_gpu_runs_in_process():
    b = _bench()
    assert b.launch_plan([], {}) == ("run", 1)
    assert b.launch_plan(["--gpus", "1", "--steps", "2"], {}) == ("run", 1)


def test_launch_plan_spawns_torchrun_child_with_args_passed_through():
    import sys
    b = _bench()
    argv = ["--gpus", "4", "--steps", "7", "--warmup", "2", "--workload", "atlas_c4_fixed"]
    kind, cmd = b.launch_plan(argv, {"MASTER_PORT": "29533"})
    assert kind == "spawn"
    assert cmd[:3] == [sys.executable, "-m", "torch.distributed.run"]
    assert "--nproc-per-node=4" in cmd and "--nnodes=1" in cmd
    assert "--master-addr=127.0.0.1" in cmd and "--master-port=29533" in cmd
    i = cmd.index(os.path.join(ROOT, "bench.py"))
    assert cmd[i + 1:] == argv       # every argument reaches the ranks unchanged
    # without MASTER_PORT a free local port is picked
    kind, cmd = b.launch_plan(["--gpus", "2"], {})
    port = [c for c in cmd if c.startswith("--master-port=")][0].split("=")[1]
    assert kind == "spawn" and 0 < int(port) < 65536


def test_launch_plan_rank_under_torchrun_and_world_mismatch():
    b = _bench()
    assert b.launch_plan(["--gpus", "8"], {"WORLD_SIZE": "8", "RANK": "3"}) == ("run", 8)
    with pytest.raises(SystemExit):
        b.launch_plan(["--gpus", "4"], {"WORLD_SIZE": "2"})
    with pytest.raises(SystemExit):
        b.launch_plan(["--gpus", "0"], {})
    # a torchrun launch without --gpus is a mismatch too (the line would claim 1 GPU)
    with pytest.raises(SystemExit):
        b.launch_plan([], {"WORLD_SIZE": "2"})


def test_two_set_2d_workload_is_declared():
    b = _bench()
    wl = b.WORKLOADS["two_set_100k_2d"]
    assert wl["kind"] == "two_set" and wl["D"] == 2 and wl["N"] == 100000


def test_flops_per_pair_dimension_scaling():
    """2D workloads price the pair operators at D = 2 (SURVEY Appendix A term counts)."""
    from difficp_amd import _lib
    assert _lib.flops_per_pair("ode_self_bwd", 3) == _lib.FLOPS_PER_PAIR["ode_self_bwd"]
    assert _lib.flops_per_pair("ode_self_fwd", 2) == pytest.approx(22.0)    # 11 D
    assert _lib.flops_per_pair("gauss_red", 2) == pytest.approx(10.0)       # 5 D
    assert _lib.flops_per_pair("ode_self_bwd", 2) == pytest.approx(70 * 64 / 95)
    assert _lib.flops_per_pair("no_such_kernel", 2) is None
