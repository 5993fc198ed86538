"""GOBI A/B against another build of the library: the same 1,024 inits (the
bench's: the reference's scheduling dataset rows, tests/golden/gobi_h16.npz)
through the in-tree library and through PGP_LIB=<other>, in two child
processes; results, iteration counts and fitness compared bitwise, and each
build's kernel time (HIP events, median of 20 launches).
usage: python tools/dbg/gobi_ab.py <other.so>"""
import json
import os
import subprocess
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def child(out):
    import torch
    sys.path.insert(0, ROOT)
    from preganplus_amd.gobi import GOBIOptimizer
    z = np.load(os.path.join(ROOT, "tests", "golden", "gobi_h16.npz"))
    E = 1024
    inits = torch.tensor(np.concatenate([z["inits"]] * (-(-E // z["inits"].shape[0])))[:E], device="cuda")
    g = GOBIOptimizer(device="cuda")
    o = (torch.empty_like(inits), torch.empty(E, dtype=torch.int32, device="cuda"),
         torch.empty(E, dtype=torch.float32, device="cuda"))
    for _ in range(3):
        g.optimize(inits, out=o)
    ts = []
    for _ in range(20):
        a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        a.record()
        g.optimize(inits, out=o)
        b.record()
        torch.cuda.synchronize()
        ts.append(a.elapsed_time(b))
    np.savez(out, result=o[0].cpu().numpy(), its=o[1].cpu().numpy(), fit=o[2].cpu().numpy(), ms=np.median(ts))


def main():
    if len(sys.argv) == 3 and sys.argv[1] == "--child":
        return child(sys.argv[2])
    other = sys.argv[1]
    os.makedirs(os.path.join(ROOT, "gpurun_out"), exist_ok=True)
    pa, pb = (os.path.join(ROOT, "gpurun_out", f"gobi_ab_{t}.npz") for t in ("new", "old"))
    subprocess.check_call([sys.executable, __file__, "--child", pa])
    subprocess.check_call([sys.executable, __file__, "--child", pb], env=dict(os.environ, PGP_LIB=other))
    a, b = np.load(pa), np.load(pb)
    rep = {"new_ms": float(a["ms"]), "old_ms": float(b["ms"]),
           "mean_iterations_new": float(a["its"].mean()), "mean_iterations_old": float(b["its"].mean()),
           "result_identical": bool(np.array_equal(a["result"], b["result"])),
           "iterations_identical": bool(np.array_equal(a["its"], b["its"])),
           "fitness_identical": bool(np.array_equal(a["fit"].view(np.int32), b["fit"].view(np.int32)))}
    print(json.dumps(rep))


if __name__ == "__main__":
    main()
