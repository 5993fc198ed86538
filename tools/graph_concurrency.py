"""Does a replayed HIP graph run independent branches concurrently on this
ROCm?  Two streams each spin for `cycles` (torch.cuda._sleep, one small
kernel), captured as a fork / join; the replay time is compared with one
branch alone and with the same work eager on two streams.  ~1x: concurrent
branches, ~2x: serialised."""
import time

import torch


def timed(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / reps * 1e3


def main():
    cyc = 2_000_000
    main_s = torch.cuda.current_stream()
    side = torch.cuda.Stream()

    def one():
        torch.cuda._sleep(cyc)

    def two():
        side.wait_stream(main_s)
        torch.cuda._sleep(cyc)
        with torch.cuda.stream(side):
            torch.cuda._sleep(cyc)
        main_s.wait_stream(side)

    print(f"eager one branch   {timed(one):.3f} ms")
    print(f"eager two branches {timed(two):.3f} ms")
    torch.cuda.synchronize()
    g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g1):
            torch.cuda._sleep(cyc)
        with torch.cuda.graph(g2):
            cur = torch.cuda.current_stream()
            side.wait_stream(cur)
            torch.cuda._sleep(cyc)
            with torch.cuda.stream(side):
                torch.cuda._sleep(cyc)
            cur.wait_stream(side)
    print(f"graph one branch   {timed(g1.replay):.3f} ms")
    print(f"graph two branches {timed(g2.replay):.3f} ms")
    # launch cost: 60 tiny kernels eager vs one replay
    x = torch.zeros(16, device="cuda")

    def many():
        for _ in range(60):
            x.add_(1.0)

    g3 = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(g3):
            many()
    print(f"60 tiny kernels eager {timed(many, 50):.3f} ms, graph {timed(g3.replay, 50):.3f} ms")


if __name__ == "__main__":
    main()
