"""bench.py's N-rank launcher (CPU, gloo): `python bench.py --gpus N` with no
torchrun environment starts N ranks itself as a child torch.distributed.run,
every rank joins one all-reduce of ones (`ranks_seen`), and a world size that
differs from --gpus fails loudly.  The GPU configs use the same _dist_setup."""
import json
import os
import subprocess
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, extra_env=None, timeout=180):
    env = dict(os.environ, PGP_DEVICE="cpu", PGP_DIST_BACKEND="gloo", MASTER_ADDR="127.0.0.1")
    env.pop("WORLD_SIZE", None)
    env.update(extra_env or {})
    return subprocess.run([sys.executable, os.path.join(ROOT, "bench.py")] + args, cwd=ROOT, env=env,
                          capture_output=True, text=True, timeout=timeout)


def _json_line(out):
    lines = [ln for ln in out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1, out
    return json.loads(lines[0])


def test_gpus2_starts_two_ranks():
    p = _run(["--config", "ranks", "--gpus", "2"])
    assert p.returncode == 0, p.stderr[-2000:]
    res = _json_line(p.stdout)
    assert res["n_gpus"] == 2 and res["ranks_seen"] == 2


def test_gpus1_single_process():
    p = _run(["--config", "ranks"])
    assert p.returncode == 0, p.stderr[-2000:]
    res = _json_line(p.stdout)
    assert res["n_gpus"] == 1 and res["ranks_seen"] == 1


def test_world_size_mismatch_fails():
    p = _run(["--config", "ranks", "--gpus", "3"], {"WORLD_SIZE": "2", "RANK": "0"})
    assert p.returncode != 0
    assert "world size 2 != --gpus 3" in p.stderr
