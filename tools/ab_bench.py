"""Interleaved A/B of bench.py lines on one box: each variant is a set of
environment variables; rounds run every variant once in turn, so drift of the
box hits all variants alike.  Prints per variant the ms_per_step of each round
and the median.

  python3 tools/ab_bench.py --rounds 3 --args "--config tune --hosts 16 --steps 50 --warmup 5 --no-cpu-baseline" \
      base= eager=PGP_BENCH_GRAPH=0 prev=PGP_LIB=preganplus_amd/_lib/var/libpreganplus_prev.so

The library reads no tuning switches from the environment (round 5 removed
them, _native.REMOVED_ENV): a variant is another build (PGP_LIB) or a
bench.py switch (ARGS=--flag in a variant appends that switch to --args).
"""
import argparse
import json
import os
import statistics
import subprocess
import sys


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--rounds", type=int, default=3)
    ap.add_argument("--args", default="")
    ap.add_argument("--timeout", type=int, default=120)
    ap.add_argument("variants", nargs="+", help="name=VAR=value,VAR2=value (empty after name= for the base)")
    a = ap.parse_args()
    variants = []
    for v in a.variants:
        name, _, spec = v.partition("=")
        env = {}
        for kv in filter(None, spec.split(",")):
            k, _, val = kv.partition("=")
            env[k] = val
        variants.append((name, env))
    res = {n: [] for n, _ in variants}
    extra = {n: [] for n, _ in variants}
    for r in range(a.rounds):
        for name, env in variants:
            env = dict(env)
            extra_args = env.pop("ARGS", "").split()
            e = dict(os.environ, **env)
            out = subprocess.run([sys.executable, "bench.py"] + a.args.split() + extra_args, env=e, capture_output=True, text=True,
                                 timeout=a.timeout)
            if out.returncode != 0:
                print(out.stderr[-2000:], flush=True)
                raise SystemExit(f"variant {name} failed: rc {out.returncode}")
            line = [ln for ln in out.stdout.splitlines() if ln.startswith("{")][-1]
            d = json.loads(line)
            res[name].append(d["ms_per_step"])
            extra[name].append({k: d[k] for k in ("eager_ms_per_step", "stage_ms", "kernel_ms", "train_gan_alone") if k in d})
            print(f"round {r} {name:10s} {d['ms_per_step']:.4f} ms", flush=True)
    for name, _ in variants:
        print(f"{name:10s} median {statistics.median(res[name]):.4f} ms  rounds {[round(x, 4) for x in res[name]]}")
    print(json.dumps({"ms_per_step": res, "extra": extra}))


if __name__ == "__main__":
    main()
