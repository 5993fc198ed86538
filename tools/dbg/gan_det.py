"""Determinism probe of the C3 step (debug): eager vs eager and eager vs graph, per section."""
import sys
import numpy as np
import torch
sys.path.insert(0, ".")
from tests.test_gpu_c3step import _online

H = int(sys.argv[1]) if len(sys.argv) > 1 else 50
main = torch.cuda.Stream()
with torch.cuda.stream(main):
    res = []
    for mode in ("eager", "eager", "graph"):
        tr, st = _online(H, 6)
        if mode == "eager":
            for _ in range(3):
                st.run()
        else:
            st.run()
            st.capture()
            for _ in range(2):
                st.run()
        torch.cuda.synchronize()
        res.append((tr, st))
for k in (1, 2):
    tr0, tr1 = res[0][0], res[k][0]
    for sec in ("transformer", "gen", "disc"):
        a = tr0.P[tr0.sec_off[sec]:tr0.sec_end[sec]].cpu().numpy()
        b = tr1.P[tr1.sec_off[sec]:tr1.sec_end[sec]].cpu().numpy()
        print(("eager" if k == 1 else "graph"), sec, "mismatch", int((a != b).sum()), "of", a.size)
    print(" target equal", bool((res[0][1].target == res[k][1].target).all()))
