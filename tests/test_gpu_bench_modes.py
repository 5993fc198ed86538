"""bench.py's C3 step in single-stream mode (PGP_BENCH_ONE_STREAM=1, what the
shared-device rehearsals set): detect is issued between the tuning forward and
its targets / backward on the same stream, so it must use its own forward
context (it overwrote the trainer's workspace and the backward
raised).  One short run as a child process."""
import json
import os
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
pytestmark = pytest.mark.gpu


@pytest.mark.timeout(240)
@pytest.mark.parametrize("one_stream", ["1", "0"])
def test_tune_bench_single_and_two_streams(one_stream):
    env = dict(os.environ, PGP_BENCH_ONE_STREAM=one_stream)
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "tune", "--hosts", "16",
                        "--steps", "3", "--warmup", "1", "--no-cpu-baseline"], cwd=ROOT, env=env,
                       capture_output=True, text=True, timeout=220)
    assert p.returncode == 0, p.stderr[-3000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    res = json.loads(lines[0])
    assert res["value"] > 0 and res["n_gpus"] == 1


@pytest.mark.timeout(240)
def test_fleet_stream_line():
    """bench.py --config fleet --stream: the PCIe-inclusive rate is the line's
    value (the whole share streamed from pinned host memory), the kernel-only
    rate beside it; both measured, the streamed one no faster than the
    resident one (it does the same launches plus the copies)."""
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--config", "fleet", "--stream", "--batch",
                        "65536", "--steps", "5", "--warmup", "1", "--no-cpu-baseline"], cwd=ROOT,
                       capture_output=True, text=True, timeout=220)
    assert p.returncode == 0, p.stderr[-3000:]
    res = json.loads([ln for ln in p.stdout.splitlines() if ln.startswith("{")][-1])
    s, k = res["streamed"], res["kernel_only"]
    assert res["value"] == s["value"] > 0 and k["value"] > 0
    assert s["value"] <= 1.05 * k["value"]
    assert s["chunks"] * s["chunk_windows"] >= 64 * 1_000_000 and s["h2d_gbs"] > 0
    assert "streamed" in res["config"]["timing"]
