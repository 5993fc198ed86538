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


def _c3dp_rank(rank, world, port, q):
    import torch
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    sys.path.insert(0, ROOT)
    import bench
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        buf = torch.ones(4096)
        calls = []

        def make_step(H, E, rk, dev):   # the exchange pattern of a step, on CPU tensors
            def run():
                dist.all_reduce(buf)
                calls.append(1)

            def exchange_ms():
                import time
                t0 = time.perf_counter()
                dist.all_reduce(buf)
                return (time.perf_counter() - t0) * 1e3
            return run, exchange_ms
        rec = bench.c3_dp_record(world, rank, torch.device("cpu"), steps=4, warmup=1, make_step=make_step)
        q.put((rank, rec, len(calls)))
    finally:
        dist.destroy_process_group()


def test_c2_line_carries_c3_dp_at_world_gt_1():
    """At world > 1 the default (c2) line gets the data-parallel C3 sub-record
    (the tuning all-reduce north_star names; c2 itself has no data-path
    collective); at world 1 it does not.  The record's timing / exchange /
    backend logic runs over two gloo ranks with a stand-in step."""
    import multiprocessing as mp
    sys.path.insert(0, ROOT)
    import bench
    assert bench.c2_subrecords(1) == () and bench.c2_subrecords(2) == ("c3_dp",)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = 32500 + os.getpid() % 1000
    procs = [ctx.Process(target=_c3dp_rank, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = [q.get(timeout=120) for _ in range(2)]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for rank, rec, ncalls in got:
        assert ncalls == 1 + 4                      # warmup + timed steps, on every rank
        assert rec["backend"] == "gloo" and rec["n_gpus"] == 2 and rec["steps"] == 4
        assert rec["ms_per_step"] > 0 and rec["all_reduce_ms"] > 0 and rec["windows_per_s"] > 0
    # the timing is the max over ranks: both ranks report the same numbers
    assert got[0][1]["ms_per_step"] == got[1][1]["ms_per_step"]


def test_subrecord_deadline_emits_the_line_and_ends_the_process():
    """bench.with_deadline: a sub-record that never returns (a collective that
    never completes) ends the process after its deadline, on_timeout first
    (rank 0 emits the headline there), exit status 0."""
    code = ("import sys, time; sys.path.insert(0, %r); import bench\n"
            "bench.with_deadline(lambda: time.sleep(60), 1, lambda: print('{\"emitted\": true}'))\n"
            "print('not reached')\n") % ROOT
    p = subprocess.run([sys.executable, "-c", code], cwd=ROOT, capture_output=True, text=True, timeout=120,
                       env=dict(os.environ, PGP_DEVICE="cpu"))
    assert p.returncode == 0, p.stderr[-2000:]
    assert json.loads(p.stdout.strip().splitlines()[-1]) == {"emitted": True}
    assert "not reached" not in p.stdout


def test_subrecord_deadline_returns_the_value_in_time():
    sys.path.insert(0, ROOT)
    import bench
    assert bench.with_deadline(lambda: 7, 30, lambda: None) == 7
