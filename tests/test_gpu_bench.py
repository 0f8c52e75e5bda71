"""GPU: bench.py's N-rank path as the driver runs it (`python bench.py --gpus N`, no launcher).

On a one-GPU box DWPA_BENCH_ONE_DEVICE=1 puts every rank on device 0: this rehearses the spawn, the gloo control
plane and the max-over-ranks timing, not scaling.  Both the weak-scaling bench line (C2 shape, small dictionary)
and the C4 strong-scaling leg must report n_gpus == 2 and verified hits.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _bench(*argv, timeout=240):
    env = {k: v for k, v in os.environ.items()
           if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK", "MASTER_ADDR", "MASTER_PORT", "LOCAL_WORLD_SIZE")}
    env["DWPA_BENCH_ONE_DEVICE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), *argv], capture_output=True, text=True,
                       env=env, timeout=timeout, cwd=ROOT)
    assert r.returncode == 0, r.stderr[-3000:]
    lines = [ln for ln in r.stdout.splitlines() if ln.strip()]
    assert len(lines) == 1 and lines[0].startswith("{"), r.stdout  # the JSON line only
    return json.loads(lines[0])


def test_bench_gpus2_weak_one_device():
    out = _bench("--gpus", "2", "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--dict-words", "4000000",
                 "--batch", "1048576")
    assert out["n_gpus"] == 2 and out["hits_verified"] is True and out["scaling"] == "weak"
    assert out["value"] > 0


def test_bench_gpus2_c4_strong_one_device():
    out = _bench("--gpus", "2", "--workload", "c4", "--scaling", "strong", "--steps", "1", "--warmup", "0",
                 "--no-cpu-baseline", "--t1-s", "20.0")
    assert out["n_gpus"] == 2 and out["hits_verified"] is True and out["scaling"] == "strong"
    assert [s[:2] for s in out["shards"]] == [[0, 50_000_000], [50_000_000, 100_000_000]]
    assert out["speedup"] and out["t_exhaust_s"] > 0
