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
    assert r["bound"] in ("hbm", "mfma") and r["unit"] in ("GB/s", "TFLOP/s")
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
