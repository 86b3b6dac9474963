"""The driver's bench.py contract on the GPU: one JSON line on stdout with the
keys the driver and the judge read (metric, value, unit, n_gpus, steps,
warmup, ms_per_step, higher_is_better, scaling, vs_baseline, dtype, data,
config.workload, roofline{bound, achieved, peak, unit, frac, traffic},
cpu_baseline{value, unit, cores, kind, sample}), at a small size so the suite
stays short; the full-size line is what the driver runs."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


@pytest.mark.gpu
def test_bench_json_line(gpu):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--packets", str(1 << 20), "--steps", "3", "--warmup", "1",
           "--no-node", "--no-e2e", "--extra", "", "--cpu-budget", "0.5"]
    p = subprocess.run(cmd, cwd=ROOT, capture_output=True, text=True, timeout=240)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, p.stdout[-2000:]
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better", "scaling",
              "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["steps"] == 3 and d["warmup"] == 1 and d["higher_is_better"] is True
    assert d["scaling"] == "weak" and d["value"] > 0 and d["ms_per_step"] > 0
    assert d["config"]["workload"] and d["config"]["packets_per_gpu"] == 1 << 20
    r = d["roofline"]
    assert r["bound"] == "hbm" and r["unit"] == "GB/s" and 0 < r["frac"] < 1
    assert abs(r["frac"] - r["achieved"] / r["peak"]) < 1e-3
    # the same-box access-shape probe (cndp_amd/csrc/roofline_probe.hip)
    assert r["probe_ms"] > 0 and abs(r["kernel_over_probe"] - r["kernel_ms"] / r["probe_ms"]) < 2e-3
    cb = d["cpu_baseline"]
    assert cb["value"] > 0 and cb["cores"] >= 1 and cb["kind"] in ("port", "reference") and cb["sample"]
    assert d["config"]["bins_total"] == 3 * (1 << 20)  # the timed steps: every packet binned once a step
