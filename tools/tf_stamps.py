"""Phase attribution of the fused tuning-encoder kernels (pgp_tunef.hip) from
a profiling build (make variant NAME=st VFLAGS=-DPGP_TF_STAMPS; run with
PGP_LIB=preganplus_amd/_lib/var/libpreganplus_st.so): one tuning forward +
backward at H, B after warm-up; prints, per kernel and phase, the mean and max
over waves of the shader-clock cycles spent between consecutive marks."""
import ctypes
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

PHASES = {
    "fwd l0": ["prologue", "load", "te gemm", "qk gemm (+x0 store)", "probs + v gemm + P.v", "o gemm+res", "ln1",
               "f1 gemm+relu (+x-hat store)", "f2 gemm+res (+prefetch)", "ln2+store", "tail"],
    "fwd l1": None,
    "bwd ffn": ["prologue", "load", "f1 gemm", "f2 gemm", "ln2+ln2 bwd", "dW2 contraction", "dW2 lds add",
                "dF gemm+mask", "dW1 contraction", "dW1 lds add", "dy1 gemm", "ln1 bwd+store", "tail", "epilogue"],
    "bwd att": ["prologue", "load x", "qkv gemm", "attention fwd", "load dR1", "dWo contraction", "dO gemm",
                "attention bwd", "dqkv store", "dX gemm+store", "tail", "epilogue"],
}


def main(H=50, B=1030):
    import torch
    from preganplus_amd import _native
    from preganplus_amd import train as TR
    from preganplus_amd import weights as W
    L = _native.lib()
    L.pgp_debug_tf_stamps.argtypes = [ctypes.c_void_p]
    L.pgp_debug_tf_stamps.restype = ctypes.c_int
    w = W.synth_weights(H, seed=0)
    tr = TR.Trainer(H, w, max_batch=B)
    rng = np.random.Generator(np.random.PCG64(3))
    x = torch.tensor(rng.uniform(0, 0.8, size=(B, 3, 3 * H)).astype(np.float32), device=tr.device)
    y = (rng.uniform(size=(B, H)) < 0.2).astype(np.int32)
    mult = rng.uniform(0.5, 2.0, size=(B, H)).astype(np.float32)
    tgt = rng.uniform(size=(B, H, 2)).astype(np.float32)
    for _ in range(3):
        tr.tune_forward(x)
        tr.tune_backward(B, y, mult, tgt)
    torch.cuda.synchronize()
    assert L.pgp_debug_tf_stamps(None) == 0
    tr.tune_forward(x)
    tr.tune_backward(B, y, mult, tgt)
    torch.cuda.synchronize()
    buf = np.zeros((4, 2048, 16), dtype=np.uint64)
    assert L.pgp_debug_tf_stamps(buf.ctypes.data) == 0
    names = list(PHASES)
    for k, name in enumerate(names):
        ph = PHASES[name] or PHASES["fwd l0"]
        a = buf[k].astype(np.float64)
        tot = a.sum(1)
        print(f"== {name}: wave total cycles mean {tot.mean():.0f} max {tot.max():.0f}")
        for i, pn in enumerate(ph):
            print(f"   {i:2d} {pn:22s} mean {a[:, i].mean():9.0f}  max {a[:, i].max():9.0f}  "
                  f"share {a[:, i].sum() / max(tot.sum(), 1):6.1%}")


if __name__ == "__main__":
    main(*(int(v) for v in sys.argv[1:]))
