"""Benchmark of the PreGAN+ decision path (BASELINE.json config 2).

One step = detect + diagnose + generate over one batch of synthetic windows
already resident in HBM: K1 GAT aggregation -> K2 encoder -> K2b decoders +
classify -> K3 Gen+Disc+decision tensors -> K5 per-container moves
(libpreganplus.so).  Multi-GPU: one process per GPU
(torchrun, or `--gpus N` starting N ranks itself); every rank processes its own batch of independent windows (weak
scaling, no data-path collective); timing is max over ranks.

Prints ONE JSON line (rank 0).  The roofline object is for the dominant kernel
(K2, fp32 MFMA-bound); its kernel time is measured live with HIP events on the
stream the kernels run on.  cpu_baseline times the numpy oracle (a CPU port of
the reference math) on a bounded sample, rank 0 at N=1 only.
"""
import argparse
import ctypes
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from preganplus_amd import _native  # noqa: E402
from preganplus_amd import roofline as R  # noqa: E402

R_ROOF = R
from preganplus_amd import weights as W  # noqa: E402
from preganplus_amd.model import DecisionModel, embedding, migrations  # noqa: E402


def log(*a):
    print(*a, file=sys.stderr, flush=True)


def synth_inputs(B, H, device, seed):
    """load U(0,0.6), 2% spikes U(0.9,1.3); one-hot schedule."""
    g = torch.Generator(device=device).manual_seed(seed)
    x = torch.rand((B, 3, 3 * H), generator=g, device=device) * 0.6
    spike = torch.rand((B, 3, 3 * H), generator=g, device=device) < 0.02
    x = torch.where(spike, 0.9 + 0.4 * torch.rand((B, 3, 3 * H), generator=g, device=device), x)
    idx = torch.randint(0, H, (B, H), generator=g, device=device)
    s = torch.zeros((B, H, H), device=device)
    s.scatter_(2, idx.unsqueeze(-1), 1.0)
    return x.contiguous(), s.contiguous()


def cpu_baseline(weights, x, s, per_window_n=256, batch_n=1024):
    """the CPU restatement timed on this box's host cores, on the
    GPU run's own first windows (same C2 inputs, spikes included), in two modes
    (reference-faithful per-window fp64; batched fp32 torch-CPU), median of 5."""
    from oracle import cpu_baseline as CB  # CPU baseline leg only
    n = max(per_window_n, batch_n)
    return CB.measure(weights, x[:n].cpu().numpy(), s[:n].cpu().numpy(), per_window_n, batch_n)


def load_traffic(H, B, kernel="encoder", targs=None):
    """HBM bytes per launch of one kernel from the committed rocprofv3 --pmc
    FETCH_SIZE / WRITE_SIZE passes (profiles/pmc_<kernel>_h<H>.json, corrected
    per MI355X_MICROARCH.md §HBM, tools/pmc_traffic.py), or None when absent,
    taken at another batch, or taken with a different build of that kernel
    (the file's isa_sha256 against the loaded library's instructions: a
    stale counter pass is never reported as this build's traffic)."""
    d = traffic_record(H, B, kernel, targs=targs)
    return None if d is None else d.get("hbm_bytes_per_launch")


def traffic_record(H, B, kernel, path=None, targs=None):
    """targs: the template arguments the file must have been taken with (a
    kernel with several forms, e.g. encoder_kernel<50, split>)."""
    p = path or os.path.join(ROOT, "profiles", f"pmc_{kernel}_h{H}.json")
    if not os.path.exists(p):
        return None
    try:
        d = json.load(open(p))
        if int(d.get("batch", -1)) != B:
            return None
        if targs is not None and d.get("template_args") != list(targs):
            return None
        if d.get("isa_sha256") is None or d["isa_sha256"] != loaded_isa_hash(kernel + "_kernel", H,
                                                                             d.get("template_args")):
            return None
        return d
    except Exception:
        return None


def loaded_isa_hash(name, H, targs=None):
    """sha256 of kernel `name`<H> (or `name`<targs...>) in the library this
    process loads (PGP_LIB or the in-tree build), tools/isa_count.kernel_isa_hash;
    None without llvm-objdump."""
    try:
        sys.path.insert(0, os.path.join(ROOT, "tools"))
        import isa_count
        return isa_count.kernel_isa_hash(name, H, lib=_native.LIB_PATH, targs=targs)
    except Exception:
        return None


def launch_ranks(n, argv=None):
    """`python bench.py --gpus N` without a torchrun environment: start N ranks,
    one process per GPU, as a CHILD `torch.distributed.run` (the driver's own
    launch form; 127.0.0.1 rendezvous on a free port) and return its exit
    code.  Called before anything touches the GPU (no re-exec of this process:
    the parent only waits)."""
    import socket
    import subprocess
    argv = sys.argv[1:] if argv is None else list(argv)
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={n}",
           "--master-addr=127.0.0.1", f"--master-port={port}", os.path.abspath(__file__)] + argv
    log(f"launching {n} ranks: {' '.join(cmd[1:])}")
    return subprocess.call(cmd, env=dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY="0"))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1, help="ranks (one process per GPU); without a torchrun "
                                                          "environment, N > 1 starts N ranks itself")
    ap.add_argument("--steps", type=int, default=300)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--hosts", type=int, default=50)
    ap.add_argument("--batch", type=int, default=65536, help="windows per GPU per step")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-budget", type=float, default=12.0)
    ap.add_argument("--no-gan", action="store_true", help="tune config: Transformer tuning step only")
    ap.add_argument("--fp32-encoder", action="store_true", help="c2: K2's feed-forward on the fp32 MFMA instead of "
                                                                 "the split-bf16 form (A/B)")
    ap.add_argument("--fp32-decoder", action="store_true", help="c2: K2b on the fp32 MFMA instead of the "
                                                                 "split-bf16 form (A/B)")
    ap.add_argument("--fp32-gan", action="store_true", help="c2: K3 on the fp32 MFMA instead of the split-bf16 "
                                                             "form (A/B)")
    ap.add_argument("--stream", action="store_true", help="fleet config: the streamed (PCIe-inclusive) rate as "
                                                          "the line's value, kernel-only beside it")
    ap.add_argument("--config", choices=["c2", "fleet", "tune", "fpe", "gobi", "sim", "loop", "plugin", "ranks"],
                    default="c2",
                    help="c2: BASELINE config 2 (default, the headline line); fleet: config 5 "
                         "(1024-host fleet = 64 cells of 16 hosts, shipped weights); tune: config 3 "
                         "(tuning step fwd+bwd+AdamW, data-parallel with an RCCL all-reduce); fpe: config 4 "
                         "(PreGAN FPE_16 encoder + K=3 classifier + PreGAN's Gen/Disc, shipped weights); "
                         "gobi: SURVEY 8f row f3, the schedule producer (GOBI's opt() over the "
                         "energy_latency_16 surrogate, a batch of independent environments); ranks: the "
                         "launcher / rendezvous check alone (one all-reduce of ones)")
    args = ap.parse_args()
    if args.gpus < 1:
        ap.error("--gpus must be >= 1")
    if args.gpus > 1 and "WORLD_SIZE" not in os.environ:
        sys.exit(launch_ranks(args.gpus))
    global _GPUS_REQUESTED
    _GPUS_REQUESTED = args.gpus
    if args.config == "ranks":
        return bench_ranks(args)
    if args.config == "fleet":
        return bench_fleet(args)
    if args.config == "tune":
        return bench_tune(args)
    if args.config == "fpe":
        return bench_fpe(args)
    if args.config == "gobi":
        return bench_gobi(args)
    if args.config == "sim":
        return bench_sim(args)
    if args.config == "loop":
        return bench_loop(args)
    if args.config == "plugin":
        return bench_plugin(args)

    world, rank, device = _dist_setup()
    H, B = args.hosts, args.batch

    weights = W.synth_weights(H, seed=0)
    model = DecisionModel(H, weights, device=device)
    model.reserve(B)
    x, s = synth_inputs(B, H, device, 1234 + rank)
    g = torch.Generator(device=device).manual_seed(4242 + rank)
    cur = torch.randint(-1, H, (B, H), generator=g, device=device, dtype=torch.int32)  # -1: unplaced
    out = model.alloc_outputs(B)
    mv_out = (torch.empty((B, H), dtype=torch.int32, device=device),
              torch.empty((B, H), dtype=torch.int32, device=device))
    torch.cuda.synchronize()

    NK = 5  # K1 gat, K2 encoder, K2b decoder, K3 gan, K5 container moves

    def step(evs=None):
        if evs is None:
            model.forward(x, s, out=out, stage=-1)
            migrations(out["keep"], out["final_target"], cur, out=mv_out)
            return
        for k in range(4):
            evs[k].record()
            model.forward(x, s, out=out, stage=k)
        evs[4].record()
        migrations(out["keep"], out["final_target"], cur, out=mv_out)
        evs[NK].record()

    if args.fp32_encoder:
        model.encoder_split(False)
    if args.fp32_decoder:
        model.decoder_split(False)
    if args.fp32_gan:
        model.gan_split(False)
    split = R.decoder_split(H) and not args.fp32_decoder
    esplit = R.encoder_split(H) and not args.fp32_encoder
    gsplit = R.gan_split(H) and not args.fp32_gan
    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    # the timed loop: events at its ends only (barrier + sync on both sides)
    elapsed = _timed(world, device, step, args.steps)
    # per-stage HIP events in a separate pass right after (same inputs, same
    # process): kernel times and the roofline's launch duration
    n_prof = min(args.steps, 40)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(NK + 1)] for _ in range(n_prof)]
    for i in range(n_prof):
        step(evs[i])
    torch.cuda.synchronize()
    k_ms = np.array([[e[k].elapsed_time(e[k + 1]) for k in range(NK)] for e in evs])  # [steps, NK]
    k_mean = k_ms.mean(axis=0)

    if rank == 0:
        ms = elapsed / args.steps * 1e3
        hw = B * world * H * args.steps / elapsed
        k2_s = k_mean[1] * 1e-3
        # executed work: the MFMAs K2 issues (ISA count); the reference formulation's
        # flops are reported beside it (the layer-0 folds issue 0.67x of them)
        alg = R.encoder_flops_per_window(H)
        if esplit:
            # fp32 and bf16 MFMAs in one kernel: achieved = its MFMA work in
            # fp32-MFMA-equivalent flops (the bf16 flops weighted by the peaks'
            # ratio, 1/16), so achieved / the fp32 peak is the matrix pipe's
            # busy fraction the ISA-counted work implies
            ef, eb = R.encoder_split_executed_flops_per_window(H)
            exe = ef + eb * R.PEAK_FP32_TFLOPS / R.PEAK_BF16_TFLOPS
        else:
            exe = R.encoder_executed_flops_per_window(H)
        achieved = (exe if exe is not None else alg) * B / k2_s / 1e12
        traffic = load_traffic(H, B, targs=[H, esplit])
        kn = {"gat_agg": "gat_agg", "encoder": "encoder", "decoder": "decoder_split" if split else "decoder",
              "gan": "gan_split" if gsplit else "gan"}
        ktargs = {"encoder": [H, esplit], "gan": [H, 16 if B >= 65536 else 4] if gsplit else None}
        k_traffic = {k: load_traffic(H, B, v, targs=ktargs.get(k)) for k, v in kn.items()}
        path_bytes = R.path_bytes_per_window(H) * B
        res = {
            "metric": "host-windows/sec (detect+diagnose+generate)",
            "value": hw,
            "unit": "host-windows/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": ms,
            "higher_is_better": True,
            "scaling": "weak",
            "vs_baseline": None,
            "dtype": "fp32",
            "data": "synthetic (SURVEY §8d C2 distribution; seeded random-init weights of the H=50 architecture)",
            "config": {"workload": f"C2: PreGAN+ batched inference, {H} hosts x W=3 x 3 resources, "
                                   f"{B} windows per GPU, fp32",
                       "hosts": H, "windows_per_gpu": B, "parallelism": f"dp{world} (independent windows)"},
            "kernel_ms": {"gat_agg": k_mean[0], "encoder": k_mean[1], "decoder": k_mean[2], "gan": k_mean[3],
                          "moves": k_mean[4]},
            "kernel_tflops": {
                "encoder": achieved,
                "decoder": R.decoder_flops_per_window(H) * B / (k_mean[2] * 1e-3) / 1e12,
                "gan": R.gan_flops_per_window(H) * B / (k_mean[3] * 1e-3) / 1e12},
            "kernel_timing": f"per-stage HIP events over {n_prof} steps after the timed loop",
            "decoder_form": ({"form": "split-bf16: each fp32 operand split exactly into 3 bf16 parts, 6 "
                                      "v_mfma_f32_16x16x32_bf16 per fp32 product (terms below 2^-26 dropped), fp32 "
                                      "accumulation; K2b's fp32-equivalent rate above may exceed the fp32 peak",
                              "executed_bf16_tflops": R.decoder_split_flops_per_window(H) * B / (k_mean[2] * 1e-3)
                              / 1e12, "bf16_dense_peak_tflops": R.PEAK_BF16_TFLOPS,
                              "frac_of_bf16_peak": R.decoder_split_flops_per_window(H) * B / (k_mean[2] * 1e-3)
                              / 1e12 / R.PEAK_BF16_TFLOPS}
                             if split else {"form": "fp32 MFMA (v_mfma_f32_16x16x4_f32)"}),
            "encoder_form": ({"form": "feed-forward (both layers' linear1 / linear2) split-bf16, 6 "
                                      "v_mfma_f32_16x16x32_bf16 per fp32 product; attention projections fp32 MFMA",
                              "executed_fp32_tflops": ef * B / k2_s / 1e12,
                              "executed_bf16_tflops": eb * B / k2_s / 1e12}
                             if esplit else {"form": "fp32 MFMA (v_mfma_f32_16x16x4_f32)"}),
            "gan_form": ("split-bf16 (6 v_mfma_f32_16x16x32_bf16 per fp32 product; schedule blocks exact in "
                         "bf16, e.g. one-hot, in 3)" if gsplit else "fp32 MFMA (v_mfma_f32_16x16x4_f32)"),
            "roofline": {"kernel": "encoder_kernel (K2)", "bound": "mfma", "achieved": achieved,
                         "peak": R.PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": achieved / R.PEAK_FP32_TFLOPS,
                         "basis": ("executed MFMA flops per launch (ISA count, tools/isa_count.py) / HIP-event "
                                   "kernel time" + ("; the split feed-forward's bf16 flops counted at 1/16 (fp32 / "
                                                    "bf16 dense peak): fp32-MFMA-equivalent work" if esplit else "")),
                         "executed_flops_per_window": exe,
                         "algorithmic_flops_per_window": alg,
                         "algorithmic_rate": alg * B / k2_s / 1e12,
                         "traffic": traffic,
                         "traffic_ratio": (None if traffic is None else
                                           traffic / (R.encoder_io_bytes_per_window(H) * B)),
                         "io_bytes_per_window": R.encoder_io_bytes_per_window(H)},
            "path_roofline": {
                "flops_per_window": R.total_flops_per_window(H),
                # the reference formulation's flops over the step time: NOT a roofline rate (the
                # kernels execute fewer flops than this, DESIGN §3 folds; it may exceed the peak)
                "algorithmic_rate_tflops": R.total_flops_per_window(H) * B * world * args.steps / elapsed / 1e12,
                "hbm_algorithmic_gbs": path_bytes * world * args.steps / elapsed / 1e9,
                "hbm_frac": path_bytes * world * args.steps / elapsed / 1e9 / R.PEAK_HBM_GBS,
                "traffic_per_step": (None if None in k_traffic.values() else sum(k_traffic.values())),
                "traffic_ratio": (None if None in k_traffic.values() else sum(k_traffic.values()) / path_bytes),
                "traffic_by_kernel": k_traffic,
            },
        }
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline ...")
            res["cpu_baseline"] = cpu_baseline(weights, x, s)
        else:
            res["cpu_baseline"] = None
    # sub-records (every rank takes part; rank 0 reports them in the line)
    # The headline never waits on a sub-record: an exception in one is recorded
    # in its place, and a sub-record still running after SUBRECORD_DEADLINE_S
    # (a collective that never completes) ends every rank, rank 0 emitting the
    # line first with the timeout recorded.
    sub = {}
    if "c3_dp" in c2_subrecords(world):
        del out, mv_out, model

        def on_timeout():
            if rank == 0:
                res["c3_dp"] = {"error": f"did not complete within {SUBRECORD_DEADLINE_S} s"}
                emit(res)
        try:
            sub["c3_dp"] = with_deadline(lambda: c3_dp_record(world, rank, device), SUBRECORD_DEADLINE_S, on_timeout)
        except Exception as e:  # noqa: BLE001 - recorded, the headline stands
            sub["c3_dp"] = {"error": f"{type(e).__name__}: {e}"[:400]}
    if rank == 0:
        res.update(sub)
        emit(res)
    if world > 1:
        with_deadline(torch.distributed.destroy_process_group, SUBRECORD_DEADLINE_S, lambda: None)


_RANKS_SEEN = 1
_GPUS_REQUESTED = 1


def _dist_setup():
    """One process per GPU (torchrun env, or the ranks launch_ranks started).
    The world size must equal --gpus (fail loudly otherwise), and every rank
    takes part in one all-reduce of ones whose sum is reported as
    `ranks_seen`.  Rehearsal knobs for a 1-GPU box: PGP_DIST_BACKEND=gloo and
    PGP_DEVICE=0 put every rank on that GPU (RCCL refuses two ranks on one
    device); PGP_DEVICE=cpu runs the rendezvous check (--config ranks) with no
    GPU at all.  The driver's runs use neither."""
    global _RANKS_SEEN
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    if world != _GPUS_REQUESTED:
        raise SystemExit(f"bench.py: world size {world} != --gpus {_GPUS_REQUESTED}")
    dev_env = os.environ.get("PGP_DEVICE", os.environ.get("LOCAL_RANK", "0"))
    if world > 1 and "PGP_DEVICE" in os.environ:
        # a rehearsal with every rank on ONE device: one stream per rank (the
        # GAN / tuning overlap and the library's side stream multiply the
        # processes' hardware queues on that device and time-slice them; the
        # driver's runs, one GPU per rank, keep the GAN / tuning overlap)
        os.environ["PGP_BENCH_ONE_STREAM"] = "1"

    if dev_env == "cpu":
        device = torch.device("cpu")
    else:
        device = torch.device("cuda", int(dev_env))
        torch.cuda.set_device(device)
    if world > 1:
        import torch.distributed as dist
        backend = os.environ.get("PGP_DIST_BACKEND", "nccl")
        if backend == "nccl":
            dist.init_process_group("nccl", device_id=device)
        else:
            dist.init_process_group(backend)
        ones = torch.ones(1, dtype=torch.float32, device=device)
        dist.all_reduce(ones)
        _RANKS_SEEN = int(round(float(ones.item())))
        if _RANKS_SEEN != world:
            raise SystemExit(f"bench.py: all-reduce of ones saw {_RANKS_SEEN} ranks, world size {world}")
    return world, rank, device


_HOST_ISSUE_S = None


GAN_RESERVED_CUS = 8   # CUs the fused tuning launches leave to the GAN step beside them (pgp_tune_reserve_cus).
# The online loop (H = 16 cells, GOBI beside) measured better with none
# (1.616 -> 1.599 ms, profiles/r04/reserve_ab/); C3 keeps 8 (H = 16: 0.290 -> 0.273 ms)
LOOP_RESERVED_CUS = 0


def _reserve_cus(main, side, count=None):
    """With the GAN step on a second stream beside the tuning step, the fused
    tuning launches leave GAN_RESERVED_CUS CUs to it: they hold whole CUs and
    deal their units statically, so a CU taken by a GAN workgroup would hold
    back the whole launch (and the GAN workgroups would wait for CUs the fused
    launches hold).  Returns the count set."""
    n = (GAN_RESERVED_CUS if count is None else count) if side is not main else 0
    L = _native.lib()
    L.pgp_tune_reserve_cus.argtypes = [ctypes.c_int]
    L.pgp_tune_reserve_cus.restype = ctypes.c_int
    _native.check(L.pgp_tune_reserve_cus(n), "pgp_tune_reserve_cus")
    return n


def _share_side_stream(world, main, side):
    """At world size > 1: make the second stream the tuning backward's side
    stream too (see bench_tune); in one-stream mode (side is main) the library
    then keeps everything on the main stream.  Returns whether a second stream
    is shared."""
    if world == 1:
        return False
    L = _native.lib()
    L.pgp_tune_set_side_stream.argtypes = [ctypes.c_void_p]
    L.pgp_tune_set_side_stream.restype = ctypes.c_int
    _native.check(L.pgp_tune_set_side_stream(ctypes.c_void_p(side.cuda_stream)), "pgp_tune_set_side_stream")
    return side is not main


def _backend_label():
    """The collective backend the ranks actually use (RCCL is torch's "nccl"
    backend on ROCm; gloo in CPU / shared-device rehearsals)."""
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()):
        return "none"
    b = dist.get_backend()
    return "RCCL" if b == "nccl" else b


SUBRECORD_DEADLINE_S = 180


def with_deadline(fn, seconds, on_timeout):
    """fn() on this thread; if it has not returned after `seconds`, a watchdog
    thread calls on_timeout() and ends the process (os._exit(0): stdout
    flushed first; exiting, not replacing the program)."""
    import threading
    done = threading.Event()

    def watch():
        if not done.wait(seconds):
            on_timeout()
            sys.stdout.flush()
            os._exit(0)
    threading.Thread(target=watch, daemon=True).start()
    try:
        return fn()
    finally:
        done.set()


def emit(res):
    """Rank 0's one JSON line, with the rendezvous count (and, for the timed
    loop, the host's own time to issue the steps: a line whose host_issue_ms
    approaches ms_per_step is bound by the launches, not the device)."""
    res["ranks_seen"] = _RANKS_SEEN
    if _HOST_ISSUE_S is not None and res.get("steps"):
        res["host_issue_ms_per_step"] = _HOST_ISSUE_S / res["steps"] * 1e3
    print(json.dumps(res), flush=True)


def bench_ranks(args):
    """The launcher / rendezvous alone: N ranks, one all-reduce of ones."""
    world, rank, device = _dist_setup()
    if rank == 0:
        emit({"metric": "ranks", "value": world, "unit": "ranks", "n_gpus": world, "device": str(device),
              "backend": os.environ.get("PGP_DIST_BACKEND", "nccl") if world > 1 else None})
    if world > 1:
        torch.distributed.destroy_process_group()


def _timed(world, device, fn, steps):
    sync = torch.cuda.synchronize if device.type == "cuda" else (lambda: None)
    if world > 1:
        torch.distributed.barrier()
    sync()
    t0 = time.perf_counter()
    for _ in range(steps):
        fn()
    global _HOST_ISSUE_S
    _HOST_ISSUE_S = time.perf_counter() - t0   # host time to issue the K steps (no sync inside)
    sync()
    if world > 1:
        torch.distributed.barrier()
    el = torch.tensor([time.perf_counter() - t0], dtype=torch.float64, device=device)
    if world > 1:
        torch.distributed.all_reduce(el, op=torch.distributed.ReduceOp.MAX)
    return float(el.item())


def bench_fleet(args):
    """BASELINE config 5: a 1024-host fleet as 64 independent 16-host cells
    (SURVEY §8d), 1M windows per cell = 64M cell-windows sharded over the GPUs.
    One step = one launch sequence over a chunk of cell-windows resident in HBM;
    the per-GPU share is covered in ceil(share / chunk) steps.  The roofline is
    the dominant kernel's (K2 encoder_kernel<16>, executed MFMA flops over its
    HIP-event time, recorded around each stage on the kernels' stream)."""
    world, rank, device = _dist_setup()
    w, _ = W.load_npz(os.path.join(ROOT, "preganplus_amd/data/simulator_16.npz"))
    H, B = 16, args.batch if args.batch != 65536 else 262144
    model = DecisionModel(H, w, device=device)
    model.reserve(B)
    x, s = synth_inputs(B, H, device, 77 + rank)
    out = model.alloc_outputs(B)
    total = 64 * 1_000_000
    share = total // world
    steps = -(-share // B) if args.steps <= 0 else args.steps
    NK = 4   # K1 gat, K2 encoder, K2b decoder, K3 gan
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(NK + 1)] for _ in range(steps)]
    it = iter(evs)

    def step():
        e = next(it)
        for k in range(NK):
            e[k].record()
            model.forward(x, s, out=out, stage=k)
        e[NK].record()

    for _ in range(args.warmup):
        model.forward(x, s, out=out)
    el = _timed(world, device, step, steps)
    k_mean = np.array([[e[k].elapsed_time(e[k + 1]) for k in range(NK)] for e in evs]).mean(axis=0)
    streamed = _fleet_streamed(model, B, share, world, device, rank)
    if rank == 0:
        cw = B * steps * world
        names = ("gat_agg", "encoder", "decoder", "gan")
        dom = int(np.argmax(k_mean))
        exe = R.encoder_executed_flops_per_window(H)
        ach = exe * B / (k_mean[1] * 1e-3) / 1e12
        k_traffic = {k: load_traffic(H, B, k) for k in names}
        path_bytes = R.path_bytes_per_window(H) * B
        res = {
            "metric": "host-windows/sec (detect+diagnose+generate), fleet", "value": cw * H / el,
            "unit": "host-windows/s", "n_gpus": world, "steps": steps, "warmup": args.warmup,
            "ms_per_step": el / steps * 1e3, "higher_is_better": True, "scaling": "strong" if args.steps <= 0 else "weak",
            "vs_baseline": None, "dtype": "fp32", "data": "synthetic (C2 distribution), shipped H=16 weights",
            "config": {"workload": "C5: 1024-host fleet = 64 x 16-host cells, cell-windows sharded over GPUs",
                       "timing": "kernel-only: one resident chunk of cell-windows re-run per step "
                                 "(inputs in HBM, no host->device streaming)",
                       "hosts_per_cell": H, "cells": 64, "cell_windows_per_step_per_gpu": B,
                       "cell_windows_total": cw, "parallelism": f"dp{world}"},
            "kernel_ms": {n: float(k_mean[k]) for k, n in enumerate(names)},
            "roofline": {"kernel": "encoder_kernel<16> (K2)" + ("" if dom == 1 else
                                                                 f" (the longest stage is {names[dom]})"),
                         "bound": "mfma", "achieved": ach, "peak": R.PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                         "frac": ach / R.PEAK_FP32_TFLOPS,
                         "basis": "executed MFMA flops per launch (ISA count, tools/isa_count.py) / HIP-event kernel "
                                  "time on the kernels' stream",
                         "executed_flops_per_window": exe,
                         "traffic": k_traffic["encoder"],
                         "traffic_ratio": (None if k_traffic["encoder"] is None else
                                           k_traffic["encoder"] / (R.encoder_io_bytes_per_window(H) * B))},
            "path_roofline": {
                "hbm_algorithmic_gbs": path_bytes / (k_mean.sum() * 1e-3) / 1e9,
                "traffic_per_step": (None if None in k_traffic.values() else sum(k_traffic.values())),
                "traffic_ratio": (None if None in k_traffic.values() else sum(k_traffic.values()) / path_bytes),
                "traffic_by_kernel": k_traffic,
                "kernel_tflops": {"encoder": ach,
                                  "decoder": R.decoder_flops_per_window(H) * B / (k_mean[2] * 1e-3) / 1e12,
                                  "gan": R.gan_flops_per_window(H) * B / (k_mean[3] * 1e-3) / 1e12}},
            "streamed": streamed,
        }
        if args.stream:
            # the PCIe-inclusive figure as the line's value (--stream): the whole
            # share streamed from pinned host memory once, decisions copied back
            res["kernel_only"] = {"value": res["value"], "ms_per_step": res["ms_per_step"], "steps": steps}
            res["value"] = streamed["value"]
            res["ms_per_step"] = streamed["ms_per_chunk"]
            res["steps"] = streamed["chunks"]
            res["scaling"] = "strong"
            res["config"]["timing"] = ("streamed: every chunk of this rank's share copied in from pinned host memory "
                                       "(copy stream), K1-K3 on the compute stream, decisions copied out; "
                                       "double-buffered")
            res["config"]["cell_windows_total"] = streamed["cell_windows_total"]
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline ...")
            res["cpu_baseline"] = cpu_baseline(w, x, s, per_window_n=256, batch_n=4096)
        emit(res)
    if world > 1:
        torch.distributed.destroy_process_group()


def _fleet_streamed(model, B, share, world, device, rank, n_src=4):
    """C5 streamed (preganplus_amd/fleet.py): this rank's whole share of the
    64M cell-windows, in chunks of B, copied in from pinned host memory (n_src
    distinct pinned chunks cycled: windows fp32 + one byte of placement per
    container), one-hot rows expanded on the device, K1-K3, the decision
    arrays copied out to pinned host memory; double-buffered over three
    streams.  Timed once over the share, barrier + sync on both sides, max over
    ranks."""
    from preganplus_amd.fleet import FleetStreamer, pinned_chunk
    H = model.H
    srcs = []
    for k in range(n_src):
        xk, sk = synth_inputs(B, H, device, 1000 + 31 * rank + k)
        srcs.append(pinned_chunk(xk, sk.argmax(dim=-1)))
        del xk, sk
    fs = FleetStreamer(model, B)
    dest = fs.host_outputs(2)
    n = -(-share // B)
    fs.run(srcs, 2, dest)   # warm-up
    torch.cuda.synchronize()
    el = _timed(world, device, lambda: fs.run(srcs, n, dest), 1)
    in_b = B * (4 * 3 * 3 * H + H)
    out_b = sum(v.numel() * v.element_size() for v in dest[0].values())
    return {"value": n * B * world * H / el, "unit": "host-windows/s", "chunks": n, "chunk_windows": B,
            "cell_windows_total": n * B * world, "seconds": el, "ms_per_chunk": el / n * 1e3,
            "h2d_bytes_per_chunk": in_b, "d2h_bytes_per_chunk": out_b,
            "h2d_gbs": in_b * n / el / 1e9, "d2h_gbs": out_b * n / el / 1e9,
            "outputs": list(dest[0].keys()),
            "note": "PCIe-inclusive: inputs start in pinned host memory (4 distinct chunks cycled), decisions end "
                    "there; copy-in, kernels and copy-out of neighbouring chunks overlap (fleet.py)"}


def synth_series(E, H, seed, R=10):
    """Raw stats.time_series rows per environment (Stats.py:46-48 layout: per
    host cpu, ram, disk) with per-column scales and 3% contention spikes, and
    the training series' column max used to normalise them (utils.py:94-95)."""
    rng = np.random.Generator(np.random.PCG64(seed))
    scale = rng.uniform(20, 100, size=3 * H)
    x = rng.uniform(0.05, 0.6, size=(E, R, 3 * H)) * scale
    spike = rng.uniform(size=x.shape) < 0.03
    x = np.where(spike, rng.uniform(0.8, 1.0, size=x.shape) * scale, x)
    train_max = scale * rng.uniform(0.9, 1.0, size=3 * H)
    return x, train_max


def _build_c3_step(H, E, R, world, rank, device):
    """The C3 step of one rank (TR.OnlineTrainStep, native): seeded
    H-architecture weights, synthetic series / one-hot schedules /
    environment records of E environments, the step's two streams (the GAN
    step on a second stream beside the tuning step: no shared data,
    PreGANPlus.py:133-134) and, at world > 1, the two process groups."""
    import types
    from preganplus_amd import simulate as SIM
    from preganplus_amd import train as TR
    B = E * R
    w = W.synth_weights(H, seed=0)
    tr = TR.Trainer(H, w, device=device, max_batch=B + E)   # the tuning windows + run_encoder's, one forward
    st = TR.TuneState(w["prototypes"])
    series_h, tmax_h = synth_series(E, H, 5 + rank, R)
    g = torch.Generator(device=device).manual_seed(17 + rank)
    s = torch.zeros((E, H, H), device=device)
    s.scatter_(2, torch.randint(0, H, (E, H, 1), generator=g, device=device), 1.0)
    envs = SIM.synth_envs(E, H, seed=5 + rank)
    sim = SIM.Simulation(H, device=device)
    main = torch.cuda.Stream(device)
    torch.cuda.set_stream(main)
    side = main if os.environ.get("PGP_BENCH_ONE_STREAM") == "1" else torch.cuda.Stream(device)
    # world > 1, one GPU per rank: main + this second stream + the two
    # communicators' streams are the 4 hardware queues a process gets
    # (GPU_MAX_HW_QUEUES), so the tuning backward's side work (decoder and
    # in_proj weight gradients) runs on this same second stream instead of a
    # fifth (pgp_tune_set_side_stream); the GAN step is issued ahead of that
    # side work (pgp_online_step issues it right after the forward)
    _share_side_stream(world, main, side)
    reserved = _reserve_cus(main, side)
    step = TR.OnlineTrainStep(tr, st, sim, series_h, tmax_h, s, envs, R=R, side=side, groups=TR.dp_groups())
    if step.native and os.environ.get("PGP_BENCH_SERIAL_ISSUE") == "1":
        step.issue_worker(False)   # A/B: one host thread issues both streams
    return types.SimpleNamespace(tr=tr, w=w, series=series_h, tmax=tmax_h, s=s, sim=sim, step=step, main=main,
                                 side=side, reserved=reserved)


def _sim_envs(E, H, seed):
    from preganplus_amd import simulate as SIM
    return SIM.synth_envs(E, H, seed=seed)


def c2_subrecords(world):
    """Sub-records the default (c2) line carries besides its headline value:
    at world > 1 the data-parallel C3 step over the ranks' collective backend
    (the one exchange step north_star names: the tuning gradient all-reduce),
    so the driver's multi-GPU run of the default config measures it too."""
    return ("c3_dp",) if world > 1 else ()


def c3_dp_record(world, rank, device, steps=20, warmup=3, hosts=50, envs_per_gpu=103, make_step=None):
    """The C3 data-parallel step (H = 50, 103 environments x 10 windows per
    rank: OnlineTrainStep over the ranks' groups) timed like every line
    (barrier + synchronize around `steps` steps, max over ranks), with the
    main stream's exchange span (the tuning gradient + state all-reduces) from
    the library's HIP events.  ``make_step(hosts, envs, rank, device)`` ->
    (run, exchange_ms) replaces the real step (the CPU test's gloo stand-in).
    Returns the sub-record (every rank; rank 0 emits it)."""
    global _HOST_ISSUE_S
    R = 10
    if make_step is None:
        def make_step(H, E, rk, dev):
            c3 = _build_c3_step(H, E, R, world, rk, dev)

            def exchange_ms(n=5):
                c3.step.timing(True)
                v = []
                for _ in range(n):
                    c3.step.run()
                    v.append(c3.step.stage_ms()["exchange"])
                c3.step.timing(False)
                return float(np.mean(v))
            return c3.step.run, exchange_ms
    run, exchange_ms = make_step(hosts, envs_per_gpu, rank, device)
    saved = _HOST_ISSUE_S
    for _ in range(warmup):
        run()
    el = _timed(world, device, run, steps)
    _HOST_ISSUE_S = saved
    ar = exchange_ms()
    ar_t = torch.tensor([ar], dtype=torch.float64, device=device)
    if world > 1:
        torch.distributed.all_reduce(ar_t, op=torch.distributed.ReduceOp.MAX)
    B = envs_per_gpu * R
    return {"workload": f"C3: semi-supervised tuning step, {hosts} hosts, {envs_per_gpu} environments x {R} windows "
                        f"per GPU, data parallel", "n_gpus": world, "steps": steps, "warmup": warmup,
            "ms_per_step": el / steps * 1e3, "windows_per_s": B * world * steps / el,
            "all_reduce_ms": float(ar_t.item()), "backend": _backend_label(),
            "all_reduce_note": "main stream span of the tuning gradient + state-increment all-reduces (the GAN "
                               "step's two all-reduces run on its own group and stream beside the backward)"}


def bench_tune(args):
    """BASELINE config 3: the semi-supervised training of run_model
    (PreGANPlus.py:115-136, everything but the decision) for a batch of
    environments per GPU, data-parallel over the GPUs.  One step, all on the
    device, in the reference's order:
      1. tune_model's on-the-fly dataset (utils.py:40-47): each environment's
         last 10 rows -> 10 windows + 98th-percentile labels and classes
         (pgp_tune_dataset), and run_encoder's window of the same rows
      2. detect (PreGANPlus.py:107-131): encoder forward of that window (the
         last E rows of the tuning forward's batch: same step-start weights) ->
         masked prototype embedding
      3. train_gan (PreGANPlus.py:60-81): Gen + Disc forward, the label from
         two runSimulation scores on the device (pgp_simulate),
         Disc BCE step, Gen BCE step; each section's gradients all-reduced
      4. tune_model (train.py:42-57 in the DP form): forward over
         the 10E windows, custom_loss / triplet_loss bookkeeping against the
         step-start state (pgp_tune_targets_dp), backward, one RCCL gradient
         all-reduce + one all-reduce of the state increments, state update and
         AdamW from device tables (DPTuner)
    No fixed labels, CE weights or targets, and no host round trip: each step
    is ONE C-ABI call (TR.OnlineTrainStep -> pgp_online_step, which issues
    every launch of both streams from C++; the collectives call back into
    torch.distributed)."""
    from preganplus_amd import train as TR
    world, rank, device = _dist_setup()
    H = args.hosts
    E = args.batch if args.batch != 65536 else 103     # 103 environments x 10 windows ~ SURVEY's 1,024
    R = 10                                             # LATEST_WINDOW_SIZE (constants.py:16)
    B = E * R
    c3 = _build_c3_step(H, E, R, world, rank, device)
    tr, w, series_h, tmax_h, s, sim, step = c3.tr, c3.w, c3.series, c3.tmax, c3.s, c3.sim, c3.step
    main, side, reserved = c3.main, c3.side, c3.reserved
    # detect shares the tuning forward (the last E rows) and its masked embedding is
    # formed inside train_gan's first launch, so it has no span of its own
    names = ("dataset", "train_gan", "tune_model")
    subs = TR.DPTuner.SUBSTAGES
    for _ in range(args.warmup):
        step.run()
    el = _timed(world, device, step.run, args.steps)
    # stage spans: more steps with the library's HIP events on (dataset on
    # the main stream; the embedding and train_gan on the GAN stream;
    # tune_model = the main stream from the forward to AdamW, with its
    # sub-stages); the GAN stream overlaps the targets and the backward
    n_ev = max(3, min(args.steps, 20))
    step.timing(True)
    spans = []
    for _ in range(n_ev):
        step.run()
        spans.append(step.stage_ms())
    step.timing(False)
    mean = lambda k: float(np.mean([d[k] for d in spans]))
    stage = np.array([mean("dataset"), mean("train_gan"), mean("tune_model")])
    sub = np.array([mean(k) for k in ("forward", "targets", "backward", "exchange", "apply_adamw")])
    eager_ms = mean("main")
    # roofline of the dominant kernels: the six fused encoder launches of the
    # tuning forward + backward, timed live with HIP events recorded on their
    # stream inside the library (pgp_tune_timing) over extra eager steps after
    # the timed region; achieved = their executed MFMA flops (ISA-counted per
    # unit, roofline.TUNE_MFMA_PER_UNIT / TUNE_BF16_PER_UNIT) / the mean launch duration
    RL = R_ROOF  # (R is the window count here)
    L = _native.lib()
    L.pgp_tune_timing.argtypes = [ctypes.c_int]
    L.pgp_tune_fused_ms.argtypes = [ctypes.c_void_p]
    _native.check(L.pgp_tune_timing(1), "pgp_tune_timing")
    fused = []
    ms6 = (ctypes.c_float * 6)()
    for _ in range(max(3, min(args.steps, 10))):
        step.run()
        _native.check(L.pgp_tune_fused_ms(ms6), "pgp_tune_fused_ms")
        fused.append(list(ms6))
    _native.check(L.pgp_tune_timing(0), "pgp_tune_timing")
    fused_ms = np.array(fused).mean(0)
    # each training stage ALONE on the device (the timed step runs them
    # concurrently, the GAN step on the CUs the fused tuning launches leave it):
    # train_gan for the E environments, and the tuning step without the GAN
    n_alone = max(5, min(args.steps, 20))
    torch.cuda.synchronize()
    a0, a1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a0.record(main)
    for _ in range(n_alone):
        step.gan_step()
    a1.record(main)
    torch.cuda.synchronize()
    gan_alone = a0.elapsed_time(a1) / n_alone
    flops = RL.tune_fused_flops(H, B, B + E)
    roof = None
    if flops is not None:
        rates = [f / (t * 1e-3) / 1e12 for f, t in zip(flops, fused_ms)]
        k = int(np.argmax(fused_ms))
        roof = {"kernel": f"tf_*_kernel<{H}> ({RL.TUNE_FUSED_LAUNCHES[k]}, the longest fused launch)",
                "bound": "mfma", "achieved": rates[k], "peak": RL.PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
                "frac": rates[k] / RL.PEAK_FP32_TFLOPS, "traffic": None,
                "basis": "executed MFMA flops of the batch's units (ISA count per unit; the split-bf16 GEMMs' "
                         "v_mfma_f32_16x16x32_bf16 counted at 1/16, the fp32 / bf16 dense-peak ratio: "
                         "fp32-MFMA-equivalent work) / mean launch duration (HIP events on the launch stream)",
                "fused_launches": {n: {"ms": float(t), "tflops": float(r), "frac": float(r / RL.PEAK_FP32_TFLOPS)}
                                   for n, t, r in zip(RL.TUNE_FUSED_LAUNCHES, fused_ms, rates)},
                "fused_total": {"ms": float(fused_ms.sum()),
                                "frac": float(sum(flops) / (fused_ms.sum() * 1e-3) / 1e12 / RL.PEAK_FP32_TFLOPS)}}
        # HBM bytes per launch of the dominant launch's kernel (both layers'
        # launches averaged) from the committed, ISA-stamped counter pass
        kname = {0: "tf_fwd", 1: "tf_fwd", 2: "tf_bwd_ffn", 3: "tf_bwd_att", 4: "tf_bwd_ffn", 5: "tf_bwd_att"}[k]
        roof["traffic"] = load_traffic(H, B, kname)
        roof["traffic_kernel"] = kname + "_kernel (mean over its two layer launches per step)"
        try:   # the CUs each launch holds (it takes the fewest that keep its longest wave)
            cus = torch.cuda.get_device_properties(device).multi_processor_count
            grids = RL.tune_fused_grids(H, B, B + E, cus, reserved)
            for (n, d), g in zip(roof["fused_launches"].items(), grids):
                d["cus"] = int(g)
                d["frac_of_its_cus"] = float(d["frac"] * cus / g)
            roof["cus"] = int(grids[k])
            roof["frac_of_its_cus"] = float(roof["frac"] * cus / grids[k])
            roof["cus_note"] = (f"each fused launch holds one CU per workgroup; the rest ({cus} CUs in all) run "
                                "the GAN step and the side weight gradients beside it")
        except Exception as exc:   # reporting only: never lose the line
            roof["cus_note"] = f"CU count unavailable: {exc}"
    if rank == 0:
        res = {
            "metric": "tuning windows/sec (semi-supervised step: dataset + detect + train_gan + DP tune_model)",
            "value": B * world * args.steps / el,
            "unit": "windows/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32 (fp64 bookkeeping and simulation scores)",
            "data": "synthetic per-environment time series (labels from their 98th percentiles), schedules and "
                    "environment records; GAN labels simulated; seeded H-architecture weights",
            "config": {"workload": f"C3: semi-supervised tuning step, {H} hosts, {E} environments x {R} windows "
                                   f"= {B} tuning windows per GPU", "hosts": H, "environments_per_gpu": E,
                       "windows_per_gpu": B, "parallelism": f"dp{world}" + (f" + {_backend_label()} all-reduce "
                                                                           "(grads, state; GAN on its own group)"
                                                                           if world > 1 else "")},
            "timed": "one pgp_online_step C-ABI call per step (every launch issued from C++)",
            "timed_with_events_ms_per_step": eager_ms,
            "stage_ms": {n: float(stage[k]) for k, n in enumerate(names)},
            "stage_note": ("steps with the library's HIP events; detect = run_encoder's windows as the last E rows "
                           "of the tuning forward (same step-start weights); their masked embedding is formed "
                           "inside train_gan's first launch (Gen forward) on the second stream"),
            "streams": "train_gan (detect's embedding inside) on a second stream, concurrent with tune_model's backward "
                       "(no shared data)" if side is not main else "one stream",
            "reserved_cus": reserved,
            "tune_model_ms": {n: float(sub[k]) for k, n in enumerate(subs)},
            "grad_all_reduce_ms": float(sub[subs.index("all_reduce")]),
            "train_gan_alone": {"ms": gan_alone, "environments": E,
                                "achieved_tflops": RL.gan_step_flops_per_env(H) * E / (gan_alone * 1e-3) / 1e12,
                                "note": "the step's GAN part by itself on the whole device (pgp_online_gan_step, "
                                        "HIP events); in the timed step it runs beside the tuning step on its stream"},
            "roofline": roof,
            # the two training stages as a whole, on the reference formulation's
            # flops (algorithmic, not executed) over the stage's HIP-event span;
            # train_gan runs on the second stream beside tune_model, so its span
            # includes the time its launches wait for CUs the tuning kernels hold
            "stage_roofline": {
                n: {"ms": float(ms), "achieved": fl / (ms * 1e-3) / 1e12, "peak": RL.PEAK_FP32_TFLOPS,
                    "unit": "TFLOP/s", "frac": fl / (ms * 1e-3) / 1e12 / RL.PEAK_FP32_TFLOPS, "flops": fl,
                    "basis": basis}
                for n, ms, fl, basis in (
                    ("tune_model", stage[2], RL.tune_step_flops_per_window(H) * (B + E / 3),
                     f"{RL.tune_step_flops_per_window(H) / 1e6:.2f} MFLOP per tuning window (3 x the Transformer "
                     f"forward: input and weight gradients) x {B} windows + 1/3 of it (the forward) x {E} detect "
                     f"windows"),
                    ("train_gan", stage[1], RL.gan_step_flops_per_env(H) * E,
                     f"{RL.gan_step_flops_per_env(H) / 1e6:.2f} MFLOP per environment (Gen + Disc forward, Disc "
                     f"step, Gen step through the updated Disc) x {E} environments"))},
        }
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline ...")
            res["cpu_baseline"] = tune_cpu_baseline(w, series_h, tmax_h, s.cpu().numpy(), _sim_envs(4, H, 5), H)
        emit(res)
    if world > 1:
        torch.distributed.destroy_process_group()


def tune_cpu_baseline(w, series, tmax, sched, envs, H, per_repeat=8, repeats=5):
    """The same per-environment work through the CPU restatements, as the
    reference runs it (CPU baseline leg only): run_encoder window -> detect ->
    train_gan with runSimulation labels (bit-identical restatement) ->
    backprop over the 10 windows, batch-1 sequential (train.py:42-57), fp64
    torch-CPU on the host's CPU share; median of 5 repeats."""
    from oracle import cpu_baseline as CB
    from oracle import pregan_oracle as O
    from oracle import pregan_train_oracle as TO
    from oracle import sim_oracle as SO
    threads = CB.host_threads()
    torch.set_num_threads(threads)
    P = TO.PluginOracle(w, {}, np.ones((1, 3 * H)), lrs=(1e-4, 3e-5 if H > 16 else 5e-5, 3e-5 if H > 16 else 5e-5))
    rates = []
    n = 0
    for rep in range(repeats + 1):
        t0 = time.perf_counter()
        for _ in range(per_repeat):
            i = n % series.shape[0]
            td = O.normalize_test_time_data(series[i], tmax[None])
            win = O.inference_window(series[i], tmax[None])
            with torch.no_grad():
                logits, protos = TO.decode_t(P.tw, TO.encode_t(P.tw, torch.tensor(win[None])))
            anom = logits[0, :, 1] > logits[0, :, 0]
            emb = torch.where(anom[:, None], protos[0], torch.zeros_like(protos[0]))
            s = torch.tensor(sched[i], dtype=torch.float64)
            TO.train_gan(P.gw, P.dw, P.gopt, P.dopt, emb, s, lambda sch: SO.score(envs[n % len(envs)], sch, H)[1])
            wins = O.convert_to_windows(td)
            an, cl = O.form_test_dataset(td)
            TO.backprop(P.tw, P.topt, P.st, wins, np.repeat(sched[i][None], 10, 0), an, cl)
            n += 1
        if rep:
            rates.append(per_repeat * 10 / (time.perf_counter() - t0))
    return {"value": float(np.median(rates)), "unit": "windows/s", "cores": threads, "kind": "port", **CB.thread_report(),
            "sample": f"{per_repeat} environments x 10 tuning windows per repeat, median of {repeats}: detect, "
                      f"train_gan (runSimulation restatement), sequential batch-1 backprop; fp64 torch-CPU "
                      f"(the reference's algorithm, H={H})",
            "repeats": rates, "cpu_model": CB.cpu_model()}


def fpe_cpu_baseline(weights, budget_s=12.0, max_threads=16, H=16):
    """numpy fp64 FPE oracle on the host cores, bounded sample (C4)."""
    from threadpoolctl import threadpool_limits
    from oracle import cpu_baseline as CB  # CPU baseline leg only
    from oracle import pregan_oracle as O  # CPU baseline leg only
    threads = min(max_threads, CB.host_threads())
    rng = np.random.Generator(np.random.PCG64(98))
    nb = 256 if H <= 16 else 64
    x = rng.uniform(0, 0.6, size=(nb, 3, 3 * H))
    h0 = rng.standard_normal((nb, 3))
    s = np.zeros((nb, H, H))
    s[np.arange(nb)[:, None], np.arange(H)[None, :], rng.integers(0, H, size=(nb, H))] = 1.0
    done = 0
    with threadpool_limits(limits=threads):
        O.forward_fpe(weights, x[:8], h0[:8], s[:8])
        t0 = time.perf_counter()
        while time.perf_counter() - t0 < budget_s:
            O.forward_fpe(weights, x, h0, s)
            done += nb
    dt = time.perf_counter() - t0
    return {"value": done * H / dt, "unit": "host-windows/s", "cores": threads, "kind": "port", **CB.thread_report(),
            "sample": f"{done} windows (H={H}, batches of {nb}), numpy fp64 FPE oracle, {dt:.1f}s"}


def bench_fpe(args):
    """BASELINE config 4: PreGAN's FPE path (K4 + K3), 64k synthetic windows per
    GPU (C2 distribution), GRU h0 ~ N(0,1) as an input.  --hosts 50 (the
    default, C4's "50 hosts"): the reference's FPE_16 code at n_hosts=50 with
    seeded weights (tests/golden/make_golden_fpe50.py pins it; the reference's
    FPE_50 itself raises); --hosts 16: the shipped checkpoints/ FPE_16."""
    from preganplus_amd.model import FPEDecisionModel
    world, rank, device = _dist_setup()
    H, B = args.hosts, args.batch
    if H == 16:
        w, _ = W.load_npz(os.path.join(ROOT, "preganplus_amd", "data", "pregan_simulator_16.npz"))
        wdesc = "shipped checkpoints/ FPE_16, Gen_16, Disc_16 weights"
    else:
        w = W.synth_fpe_weights(H, seed=0)
        wdesc = (f"seeded weights (synth_fpe_weights({H}, 0)); the reference FPE_16 code at n_hosts={H} "
                 f"with Gen_{H}/Disc_{H} (an extrapolation of FPE_16: the reference FPE_50 raises)")
    model = FPEDecisionModel(H, w, device=device)
    model.reserve(B)
    x, s = synth_inputs(B, H, device, 4321 + rank)
    g = torch.Generator(device=device).manual_seed(77 + rank)
    h0 = torch.randn((B, 3), generator=g, device=device).contiguous()
    out = model.alloc_outputs(B)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(3)] for _ in range(args.steps)]
    it = iter(range(args.steps))

    def step(timed=False):
        if not timed:
            model.forward(x, h0, s, out=out)
            return
        e = evs[next(it)]
        e[0].record()
        model.forward(x, h0, s, out=out, stage=0)
        e[1].record()
        model.forward(x, h0, s, out=out, stage=1)
        e[2].record()

    for _ in range(args.warmup):
        step()
    torch.cuda.synchronize()
    elapsed = _timed(world, device, lambda: step(True), args.steps)
    k = np.array([[e[0].elapsed_time(e[1]), e[1].elapsed_time(e[2])] for e in evs]).mean(axis=0)
    if rank == 0:
        fpe_bytes = R.fpe_bytes_per_window(H) * B
        gan_fl = R.gan_flops_per_window(H) * B
        dom_fpe = k[0] >= k[1]
        if dom_fpe:
            # K4 is one window per lane on the VALU (too little work per window for MFMA
            # operand shuffles): its roofline is the fp32 vector peak (= the f32 MFMA rate);
            # its HBM rate is reported beside it
            # K4's algebra removes most of the reference formulation's flops (rank-3 GAT node
            # mean, factorised edge softmax), so it is priced on what it executes
            ach = R.fpe_executed_flops_per_window(H) * B / (k[0] * 1e-3) / 1e12
            roof = {"kernel": "fpe_kernel (K4)", "bound": "valu", "achieved": ach, "peak": R.PEAK_FP32_TFLOPS,
                    "unit": "TFLOP/s", "frac": ach / R.PEAK_FP32_TFLOPS, "traffic": None,
                    "basis": "executed (roofline.fpe_executed_flops_per_window)",
                    "flops_per_window": R.fpe_executed_flops_per_window(H),
                    "reference_formulation_flops_per_window": R.fpe_flops_per_window(H),
                    "hbm_gbs": fpe_bytes / (k[0] * 1e-3) / 1e9,
                    "hbm_frac": fpe_bytes / (k[0] * 1e-3) / 1e9 / R.PEAK_HBM_GBS}
        elif R.gan_split(H):
            # K3 on split-bf16 MFMAs (pgp_gansplit.hip): priced on the bf16 flops it executes
            # (one-hot schedules: their blocks take 3 products) against the dense bf16 peak
            exe = R.gan_split_flops_per_window(H, onehot=True)
            ach = exe * B / (k[1] * 1e-3) / 1e12
            roof = {"kernel": f"gan_split_kernel<{H}> (K3, split-bf16)", "bound": "mfma", "achieved": ach,
                    "peak": R.PEAK_BF16_TFLOPS, "unit": "TFLOP/s", "frac": ach / R.PEAK_BF16_TFLOPS,
                    "traffic": None, "basis": "executed v_mfma_f32_16x16x32_bf16 flops (roofline."
                                              "gan_split_flops_per_window) / HIP-event launch time",
                    "flops_per_window": exe,
                    "fp32_equivalent_tflops": gan_fl / (k[1] * 1e-3) / 1e12}
        else:
            ach = gan_fl / (k[1] * 1e-3) / 1e12
            roof = {"kernel": "gan_kernel (K3)", "bound": "mfma", "achieved": ach, "peak": R.PEAK_FP32_TFLOPS,
                    "unit": "TFLOP/s", "frac": ach / R.PEAK_FP32_TFLOPS, "traffic": None,
                    "flops_per_window": R.gan_flops_per_window(H)}
        res = {
            "metric": "host-windows/sec (detect+diagnose+generate)",
            "value": B * world * H * args.steps / elapsed, "unit": "host-windows/s",
            "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": elapsed / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "data": f"synthetic windows (SURVEY §8d C2 distribution at H={H}), h0 ~ N(0,1); {wdesc}",
            "config": {"workload": f"C4: PreGAN FPE encoder (H={H}) + K=3 classifier + GAN, {B} windows per GPU, "
                                   f"fp32",
                       "hosts": H, "windows_per_gpu": B, "parallelism": f"dp{world} (independent windows)"},
            "kernel_ms": {"fpe": k[0], "gan": k[1]},
            "kernel_rates": {"fpe_gbs": fpe_bytes / (k[0] * 1e-3) / 1e9,
                             "fpe_gflops": R.fpe_flops_per_window(H) * B / (k[0] * 1e-3) / 1e9,
                             "gan_tflops": gan_fl / (k[1] * 1e-3) / 1e12},
            "roofline": roof,
        }
        if world == 1 and not args.no_cpu_baseline:
            log("timing CPU baseline ...")
            res["cpu_baseline"] = fpe_cpu_baseline(w, args.cpu_budget, H=H)
        else:
            res["cpu_baseline"] = None
        emit(res)
    if world > 1:
        torch.distributed.destroy_process_group()


def gobi_flops(its, E):
    """Algorithmic flops of one pgp_gobi_optimize launch: per environment and
    iteration the surrogate's forward + input gradient, 2 x (288x128 + 128x128
    + 128x64 + 64x2) MACs, for the mean iterations + 2 (the first forward and
    the final scoring pass)."""
    macs_it = 2 * (288 * 128 + 128 * 128 + 128 * 64 + 64 * 2)
    return 2 * macs_it * (its + 2) * E


def gobi_roofline(its, E, k_ms):
    """GOBI's roofline field: the fp32 VALU peak (the kernel's dot products
    are VALU FMAs, not MFMAs; the same 157.3 TF); achieved = algorithmic flops
    per launch / the launch's HIP-event time.  The iterations of one
    environment are a dependent chain (each step's input is the last step's
    output), so the kernel is latency-bound and far below the peak by
    construction; the line shows how far."""
    ach = gobi_flops(its, E) / (k_ms * 1e-3) / 1e12
    return {"kernel": "gobi_kernel", "bound": "latency (dependent VALU chain; priced on the fp32 VALU peak)",
            "achieved": ach, "peak": R.PEAK_FP32_TFLOPS, "unit": "TFLOP/s",
            "frac": ach / R.PEAK_FP32_TFLOPS, "kernel_ms": k_ms,
            "basis": "algorithmic flops (forward + input gradient per iteration, mean iterations + 2) / HIP-event "
                     "time of the launch on its stream; latency-bound dependent iteration chain",
            "traffic": None}


def bench_gobi(args):
    """GOBI (scheduler/GOBI.py:19-42, BaGTI/src/opt.py:17-33)
    over a batch of independent 16-host environments per GPU (the fleet's
    cells), one pgp_gobi_optimize launch per step, inits drawn from the
    reference's own scheduling dataset rows (tests/golden/gobi_h16.npz)."""
    from preganplus_amd.gobi import GOBIOptimizer
    world, rank, device = _dist_setup()
    E = args.batch if args.batch != 65536 else 1024
    z = np.load(os.path.join(ROOT, "tests", "golden", "gobi_h16.npz"))
    reps = -(-E // z["inits"].shape[0])
    inits = torch.tensor(np.concatenate([z["inits"]] * reps)[:E], device=device)
    g = GOBIOptimizer(device=device)
    out = (torch.empty_like(inits), torch.empty(E, dtype=torch.int32, device=device),
           torch.empty(E, dtype=torch.float32, device=device))
    for _ in range(args.warmup):
        g.optimize(inits, out=out)
    evs = [[torch.cuda.Event(enable_timing=True) for _ in range(2)] for _ in range(args.steps)]
    it = iter(evs)

    def step():
        e = next(it)
        e[0].record()
        g.optimize(inits, out=out)
        e[1].record()

    el = _timed(world, device, step, args.steps)
    its = out[1].float().mean().item()
    k_ms = float(np.mean([e[0].elapsed_time(e[1]) for e in evs]))
    if rank == 0:
        res = {
            "metric": "GOBI schedules/sec (opt() over energy_latency_16)", "value": E * world * args.steps / el,
            "unit": "schedules/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": el / args.steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32",
            "data": "inits = the reference's scheduling dataset rows + synthetic (tests/golden/gobi_h16.npz)",
            "config": {"workload": f"f3: GOBI, {E} independent 16-host environments per GPU", "hosts": 16,
                       "environments_per_gpu": E, "mean_iterations": its, "parallelism": f"dp{world}"},
            "algorithmic_rate_tflops": gobi_flops(its, E) / (el / args.steps) / 1e12,
            "roofline": gobi_roofline(its, E, k_ms),
        }
        if world == 1 and not args.no_cpu_baseline:
            from oracle import gobi_oracle as GO  # CPU baseline leg only
            sd, _ = GO.load(os.path.join(ROOT, "preganplus_amd", "data", "gobi_energy_latency_16.npz"))
            torch.set_num_threads(1)
            t0, n = time.perf_counter(), 0
            while time.perf_counter() - t0 < args.cpu_budget:
                GO.opt(sd, z["inits"][n % z["inits"].shape[0]])
                n += 1
            dt = time.perf_counter() - t0
            res["cpu_baseline"] = {"value": n / dt, "unit": "schedules/s", "cores": 1, "kind": "port", "threads_note": "sequential per-environment restatement (the reference's one-call-at-a-time loop over small tensors, below torch's intra-op parallel grain): 1 thread",
                                   "sample": f"{n} opt() runs of the torch-CPU restatement (bit-identical to the "
                                             f"reference's), 1 thread, {dt:.1f}s"}
        emit(res)
    if world > 1:
        torch.distributed.destroy_process_group()


def bench_sim(args):
    """the GAN label's two Stats.runSimulation calls
    (PreGANPlus.py:65, Stats.py:154-177) for a batch of environments per GPU,
    one pgp_simulate launch per step (generator-like and original schedule per
    environment, synthetic records of simulate.synth_envs)."""
    from preganplus_amd import simulate as SIM
    world, rank, device = _dist_setup()
    H = args.hosts
    E = args.batch if args.batch != 65536 else 4096
    rng = np.random.Generator(np.random.PCG64(9 + rank))
    envs_h = SIM.synth_envs(E, H, seed=3 + rank)
    new_h = rng.uniform(size=(E, H, H)).astype(np.float32)
    orig_h = np.zeros((E, H, H), np.float32)
    orig_h[np.arange(E)[:, None], np.arange(H)[None, :], rng.integers(0, H, (E, H))] = 1.0
    envs, new, orig = (torch.tensor(a, device=device) for a in (envs_h, new_h, orig_h))
    sim = SIM.Simulation(H, device=device)
    out = torch.empty((E, 4), dtype=torch.float64, device=device)
    target = torch.empty((E, 2), dtype=torch.float32, device=device)

    def step():
        sim.score(envs, new, orig, out=out, target=target)

    for _ in range(args.warmup):
        step()
    el = _timed(world, device, step, args.steps)
    if rank == 0:
        t = el / args.steps
        byt = E * (8 * SIM.env_len(H) + 2 * 4 * H * H + 8 * 4 + 4 * 2)  # record + 2 schedules in; out + target
        res = {
            "metric": "GAN-label simulations/sec (2 x runSimulation per environment)", "value": E * world / t,
            "unit": "environments/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
            "ms_per_step": t * 1e3, "higher_is_better": True, "scaling": "weak", "vs_baseline": None,
            "dtype": "fp64 (scores), fp32 (schedules)",
            "data": "synthetic environment records (simulate.synth_envs), random generator-like and one-hot schedules",
            "config": {"workload": f"f4: runSimulation label, {E} environments x {H} hosts per GPU", "hosts": H,
                       "environments_per_gpu": E, "parallelism": f"dp{world}"},
            "roofline": {"kernel": "simulate_kernel", "bound": "hbm", "achieved": byt / t / 1e9,
                         "peak": R.PEAK_HBM_GBS, "unit": "GB/s", "frac": byt / t / 1e9 / R.PEAK_HBM_GBS,
                         "traffic": None, "bytes_per_environment": byt / E},
        }
        if world == 1 and not args.no_cpu_baseline:
            from oracle import sim_oracle as SO  # CPU baseline leg only
            t0, n = time.perf_counter(), 0
            while time.perf_counter() - t0 < args.cpu_budget:
                i = n % E
                SO.simulate_batch(envs_h[i:i + 1], new_h[i:i + 1], orig_h[i:i + 1], H)
                n += 1
            dt = time.perf_counter() - t0
            res["cpu_baseline"] = {"value": n / dt, "unit": "environments/s", "cores": 1, "kind": "port", "threads_note": "sequential per-environment restatement (the reference's one-call-at-a-time loop over small tensors, below torch's intra-op parallel grain): 1 thread",
                                   "sample": f"{n} environments through the Python restatement (bit-identical to "
                                             f"the reference's runSimulation), 1 thread, {dt:.1f}s"}
        emit(res)
    if world > 1:
        torch.distributed.destroy_process_group()


def bench_loop(args):
    """One online interval of PreGAN+ for a fleet of independent 16-host cells,
    every stage on the device (f3 -> path -> f4 -> a11/a12):
      GOBI schedules (pgp_gobi_optimize)  -> result_cache [E,16,16]
      K1/K2/K2b encode + detect/classify  (run_model up to the embedding)
      GAN step, labels simulated           (train_gan, pgp_simulate)
      tuning step                          (tune_model's DP form with its device bookkeeping,
                                            DPTuner; synthetic labels / classes, as C3)
      inference weight sync                (pgp_repack_master on the device: master +
                                            the tuning state's prototypes -> packed layouts)
      K3 + K5 with the updated GAN         (recover_decision)
    in the reference's order (PreGANPlus.py:115-136).  All cells train as one
    data-parallel batch (sum of their losses).  Shipped H=16 weights (PreGAN+
    and the GOBI surrogate); GOBI inits from the reference's scheduling dataset;
    synthetic windows and environment records."""
    from preganplus_amd import simulate as SIM
    from preganplus_amd import train as TR
    from preganplus_amd.gobi import GOBIOptimizer
    world, rank, device = _dist_setup()
    H = 16
    E = args.batch if args.batch != 65536 else 1024
    w, extra = W.load_npz(os.path.join(ROOT, "preganplus_amd/data/simulator_16.npz"))
    model = DecisionModel(H, w, device=device)
    model.reserve(E)
    tr = TR.Trainer(H, w, device=device, max_batch=E)
    gobi = GOBIOptimizer(device=device)
    sim = SIM.Simulation(H, device=device)
    z = np.load(os.path.join(ROOT, "tests", "golden", "gobi_h16.npz"))
    reps = -(-E // z["inits"].shape[0])
    inits_h = np.concatenate([z["inits"]] * reps)[:E]
    inits = torch.tensor(inits_h, device=device)
    cur_h = inits_h[:, :, 2:].argmax(-1).astype(np.int32)
    cur_host = torch.tensor(cur_h, device=device)
    envs_h = SIM.synth_envs(E, H, seed=13 + rank)
    envs_h[:, 2:2 + H] = cur_h  # the records' placement = GOBI's current allocation
    envs = torch.tensor(envs_h, device=device)
    x, _ = synth_inputs(E, H, device, 31 + rank)
    g = torch.Generator(device=device).manual_seed(19 + rank)
    y = (torch.rand((E, H), generator=g, device=device) < 0.1).to(torch.int32)
    cls = torch.randint(0, 3, (E, H), generator=g, device=device, dtype=torch.int32)
    tune_group, gan_group = TR.dp_groups()
    tun = TR.DPTuner(tr, TR.TuneState(np.asarray(model.prototypes, dtype=np.float64)), E, group=tune_group)
    K = model.K
    gout = (torch.empty_like(inits), torch.empty(E, dtype=torch.int32, device=device),
            torch.empty(E, dtype=torch.float32, device=device))
    out = model.alloc_outputs(E)
    sim_out = torch.empty((E, 4), dtype=torch.float64, device=device)
    gan_target = torch.empty((E, 2), dtype=torch.float32, device=device)
    sched = torch.empty((E, H, H), device=device)
    emb_buf = torch.empty((E, H, 2), dtype=torch.float32, device=device)
    names = ("gobi", "encode_classify", "gan_step", "tune_step", "weight_sync", "gan_decide_moves")
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(len(names) + 1)]
    acc = np.zeros(len(names))
    main = torch.cuda.current_stream(device)
    side = main if os.environ.get("PGP_BENCH_ONE_STREAM") == "1" else torch.cuda.Stream(device)
    shared_side = _share_side_stream(world, main, side)   # see bench_tune
    _reserve_cus(main, side, LOOP_RESERVED_CUS)

    emb_ready = torch.cuda.Event()

    def interval(timed=False):
        if timed:
            ev[0].record()
        if shared_side:
            # world > 1 sharing the second stream with the tuning backward's
            # side work: GOBI first on the main stream (its 0.8 ms would hold
            # that side work back)
            res, _, _ = gobi.optimize(inits, out=gout)
            sched.copy_(res[:, :, 2:])
            if timed:
                ev[1].record()
        else:
            # GOBI on the second stream: only the GAN step and K3 read its
            # schedule, so the encoder stages and the tuning step run beside it
            # on the main stream, on the CUs its finished workgroups leave
            # (its time is its slowest workgroup's iteration chain)
            side.wait_stream(main)
            with torch.cuda.stream(side):
                res, _, _ = gobi.optimize(inits, out=gout)
                sched.copy_(res[:, :, 2:])
                if timed:
                    ev[1].record(side)
        for st in (0, 1, 2):
            model.forward(x, sched, out=out, stage=st)
        emb = embedding(out["logits"], out["protos"], out=emb_buf)   # PreGANPlus.py:129
        if timed:
            ev[2].record()
        # the GAN step on the second stream beside the tuning step (no shared
        # data, see bench_tune), after GOBI and the embedding; the repack
        # reads both sections of the master
        emb_ready.record(main)
        side.wait_event(emb_ready)

        def gan_step():
            with torch.cuda.stream(side):
                TR.train_gan_batched(tr, sim, envs, emb, sched, out=sim_out, target=gan_target, all_reduce=True,
                                     group=gan_group)
                if timed:
                    ev[3].record(side)
        if shared_side:              # ahead of the tuning backward's side work on the shared stream
            gan_step()
        tun.step(x, y, cls)          # issued first at N = 1 (see bench_tune)
        if timed:
            ev[4].record(main)
        # the weight sync in two parts (pgp_repack_master_sections): the
        # PreGAN+ part as soon as the tuning step has updated its section,
        # beside the GAN step; after it only the GAN part
        model.repack_master(tr.P, tun.state[:2 * K], sections=1)
        if not shared_side:
            gan_step()
        main.wait_stream(side)
        model.repack_master(tr.P, tun.state[:2 * K], sections=2)
        if timed:
            ev[5].record()
        model.forward(x, sched, out=out, stage=3)
        migrations(out["keep"], out["final_target"], cur_host)
        if timed:
            ev[6].record()

    for _ in range(args.warmup):
        interval()
    steps = args.steps

    # stage spans: gobi ev0 -> ev1 (second stream at N = 1), encode_classify
    # ev0 -> ev2 (beside GOBI), gan_step from the later of GOBI's end and the
    # embedding to ev3, tune_step ev2 -> ev4, weight_sync ev4 -> ev5 (with the
    # wait for the GAN step), gan_decide_moves ev5 -> ev6
    def timed_interval():
        interval(True)
        torch.cuda.synchronize()
        t = [ev[0].elapsed_time(e) for e in ev]   # ms from the interval's start
        spans = (t[1], t[2], t[3] - max(t[1], t[2]), t[4] - t[2], t[5] - t[4], t[6] - t[5])
        for k in range(len(names)):
            acc[k] += spans[k]

    el = _timed(world, device, timed_interval, steps)
    if rank == 0:
        res = {
            "metric": "fleet cell-intervals/sec (GOBI + decision + GAN/tuning steps + decisions)",
            "value": E * world * steps / el, "unit": "cell-intervals/s", "n_gpus": world, "steps": steps,
            "warmup": args.warmup, "ms_per_step": el / steps * 1e3, "higher_is_better": True, "scaling": "weak",
            "vs_baseline": None, "dtype": "fp32 (fp64 simulation scores)",
            "data": "GOBI inits from the reference's scheduling dataset; synthetic windows, environment records "
                    "and tuning labels; shipped H=16 weights",
            "config": {"workload": f"online interval, {E} independent 16-host cells per GPU", "hosts": H,
                       "cells_per_gpu": E, "parallelism": f"dp{world}"},
            "stage_ms": {n: float(acc[k] / steps) for k, n in enumerate(names)},
            "streams": "GOBI on a second stream beside the encoder stages and the tuning step (only the GAN "
                       "step and K3 read its schedule); the GAN step on that stream after GOBI and the "
                       "embedding, concurrent with the tuning step (no shared data)"}
        # the longest stage is GOBI (a latency-bound iteration chain): its roofline
        res["roofline"] = gobi_roofline(float(gout[1].float().mean().item()), E, float(acc[0] / steps))
        res["roofline"]["basis"] += "; the loop's gobi stage time (events around the launch and the schedule copy)"
        if world == 1 and not args.no_cpu_baseline:
            res["cpu_baseline"] = loop_cpu_baseline(w, extra, inits_h, x.cpu().numpy(), envs_h,
                                                    y.cpu().numpy(), args.cpu_budget)
        emit(res)
    if world > 1:
        torch.distributed.destroy_process_group()


def loop_cpu_baseline(w, extra, inits, wins, envs, y, budget_s):
    """The same per-cell interval on the host from the pinned restatements
    (CPU baseline leg only): GOBI opt() (bit-identical to the reference's),
    encode + classify (torch fp64), train_gan with runSimulation labels
    (bit-identical restatement), one tuning step on the cell's window
    (train.py backprop), recover_decision's Gen/Disc forward.  1 thread."""
    from oracle import gobi_oracle as GO
    from oracle import pregan_train_oracle as TO
    from oracle import sim_oracle as SO
    sd, _ = GO.load(os.path.join(ROOT, "preganplus_amd", "data", "gobi_energy_latency_16.npz"))
    P = TO.PluginOracle(w, extra, np.ones((1, 48)))
    torch.set_num_threads(1)
    H = 16
    t0, n = time.perf_counter(), 0
    while time.perf_counter() - t0 < budget_s:
        i = n % len(inits)
        res, _, _ = GO.opt(sd, inits[i])
        s = torch.tensor(np.asarray(res)[:, 2:], dtype=torch.float64)
        with torch.no_grad():
            logits, protos = TO.decode_t(P.tw, TO.encode_t(P.tw, torch.tensor(wins[i:i + 1], dtype=torch.float64)))
        anom = logits[0, :, 1] > logits[0, :, 0]
        emb = torch.where(anom[:, None], protos[0], torch.zeros_like(protos[0]))
        TO.train_gan(P.gw, P.dw, P.gopt, P.dopt, emb, s, lambda sch: SO.score(envs[i], sch, H)[1])
        TO.backprop(P.tw, P.topt, P.st, wins[i:i + 1].astype(np.float64), s.numpy()[None], y[i:i + 1],
                    np.zeros_like(y[i:i + 1]))
        with torch.no_grad():
            ns = TO.gen_t(P.gw, emb[None], s[None])
            TO.disc_t(P.dw, s[None], ns)
        n += 1
    dt = time.perf_counter() - t0
    return {"value": n / dt, "unit": "cell-intervals/s", "cores": 1, "kind": "port", "threads_note": "sequential per-environment restatement (the reference's one-call-at-a-time loop over small tensors, below torch's intra-op parallel grain): 1 thread",
            "sample": f"{n} cell-intervals through the CPU restatements (GOBI opt, encode/classify, train_gan with "
                      f"runSimulation labels, one tuning window, Gen/Disc), 1 thread, {dt:.1f}s"}


class _Obj:
    pass


class _Container:
    def __init__(self, cid, hid):
        self.id, self._h = cid, hid

    def getHostID(self):
        return self._h


class _NpzDict(dict):
    """A decompressed npz fixture (``files`` like np.lib.npyio.NpzFile)."""

    @property
    def files(self):
        return list(self.keys())


def _plugin_env(z, step, train_time):
    """A COSCO-shaped environment for one interval of the plugin fixture
    (tests/golden/plugin_h16.npz): placement, GOBI schedule, time series, and
    runSimulation returning that interval's recorded scores."""
    env = _Obj()
    env.hostlist = list(range(16))
    placement = z[f"s{step}/placement"]
    cl = [_Container(c, int(placement[c])) for c in range(16)]
    cl[int(z["container_none"]) if "container_none" in z.files else 3] = None
    env.containerlist = cl
    env.scheduler = _Obj()
    env.scheduler.result_cache = z[f"s{step}/sched"]
    env.stats = _Obj()
    tt = int(z["T0"]) + step
    env.stats.time_series = train_time[:tt + 1]
    env.stats.schedule_series = z["schedule_series"][:tt + 1]
    sc = [tuple(x) for x in z[f"s{step}/scores"]]
    env.stats.runSimulation = lambda sched: sc.pop(0)
    return env


def bench_plugin(args):
    """BASELINE config 1: one PreGANPlusRecovery.run_model call (PreGANPlus.py:115-136)
    as COSCO makes it each interval, H=16 shipped weights: encoder, detect,
    train_gan, tune_model (10 sequential windows), recover_decision.  The
    environment replays the reference-recorded intervals of
    tests/golden/plugin_h16.npz (runSimulation returns the recorded scores).
    The Gen / Disc checkpoints are rewritten every call (save_gan, on a writer
    thread); plotting is off.  The CPU baseline is
    the torch-fp64 restatement of the same call (oracle/pregan_train_oracle.py
    PluginOracle, pinned to the reference's own outputs)."""
    from preganplus_amd.recovery import PreGANPlusRecovery
    world, rank, device = _dist_setup()
    w, extra = W.load_npz(os.path.join(ROOT, "preganplus_amd/data/simulator_16.npz"))
    zf = np.load(os.path.join(ROOT, "tests", "golden", "plugin_h16.npz"))
    z = _NpzDict({k: zf[k] for k in zf.files})      # decompressed once: the env is the caller's, not timed
    tr_time = extra["train_time_data"]
    import tempfile
    ckdir = tempfile.mkdtemp(prefix="pgp_save_gan_")
    # save_gan on, as in the reference (Gen / Disc checkpoints rewritten every call, PreGANPlus.py:76-81)
    rec = PreGANPlusRecovery(16, "", training=True, weights=w, extra=extra, device=device, save_folder=ckdir)

    def prepare(k):
        step = k % 4
        rec.setEnvironment(_plugin_env(z, step, tr_time))
        return [tuple(x) for x in z[f"s{step}/decision_in"]]

    def call(k):
        return rec.run_model(None, prepare(k))

    for k in range(args.warmup):
        call(k)
    lat = []
    for k in range(args.steps):
        dec = prepare(k)                       # COSCO's side of the interval (env, decision list)
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        rec.run_model(None, dec)
        torch.cuda.synchronize()
        lat.append(time.perf_counter() - t0)
    # per-stage wall time (a separate pass: each stage bracketed by synchronize)
    stages = {}

    def timed(name, fn):
        def wrapper(*a, **k):
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            r = fn(*a, **k)
            torch.cuda.synchronize()
            stages.setdefault(name, []).append(time.perf_counter() - t0)
            return r
        return wrapper

    # (this pass serialises the stages; run_model overlaps the tuning graph,
    # launched by _tune_launch, with train_gan's host simulator call)
    staged = ("train_gan", "_tune_launch", "_tune_finish", "sync_inference_weights", "recover_decision")
    for name in staged:
        setattr(rec, name, timed(name.lstrip("_"), getattr(rec, name)))
    rec._detect = timed("detect_forward", rec._detect)
    import preganplus_amd.train as TRm
    bp, ds = TRm.backprop, TRm.on_the_fly_dataset
    TRm.backprop, TRm.on_the_fly_dataset = timed("tune_backprop", bp), timed("tune_dataset", ds)
    try:
        for k in range(min(args.steps, 20)):
            call(k)
    finally:
        TRm.backprop, TRm.on_the_fly_dataset = bp, ds
        for name in staged:
            delattr(rec, name)
        del rec._detect
    stage_ms = {k: float(np.median(v) * 1e3) for k, v in stages.items()}
    # batch-1 inference latency (the encoder + classify + GAN gate of one window)
    model = rec.infer
    x1 = torch.tensor(rec.input_window()[None], dtype=torch.float32, device=device)
    s1 = torch.tensor(np.asarray(z["s0/sched"])[None], dtype=torch.float32, device=device)
    out = model.alloc_outputs(1)
    for _ in range(5):
        model.forward(x1, s1, out=out)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(50):
        model.forward(x1, s1, out=out)
    torch.cuda.synchronize()
    fwd_ms = (time.perf_counter() - t0) / 50 * 1e3
    ms = float(np.median(lat) * 1e3)
    rec.flush_checkpoints()
    if rank == 0:
        res = {"metric": "plugin run_model calls/sec (H=16, train_gan + tune_model + decision)", "value": 1e3 / ms,
               "unit": "calls/s", "n_gpus": 1, "steps": args.steps, "warmup": args.warmup, "ms_per_step": ms,
               "higher_is_better": True, "scaling": "replicas only", "vs_baseline": None, "dtype": "fp32",
               "data": "reference-recorded intervals (tests/golden/plugin_h16.npz), shipped H=16 weights",
               "config": {"workload": "C1: PreGANPlusRecovery.run_model, one COSCO interval, 16 hosts",
                          "hosts": 16, "tuning_windows": 10},
               "latency_ms": {"run_model_median": ms, "run_model_p90": float(np.percentile(lat, 90) * 1e3),
                              "forward_batch1": fwd_ms},
               "stages_ms": stage_ms,
               "save_gan": {"on": rec.save_gan, "files": sorted(os.listdir(ckdir))}}
        if not args.no_cpu_baseline:
            from oracle import pregan_train_oracle as TO  # CPU baseline leg only
            torch.set_num_threads(1)
            po = TO.PluginOracle(w, extra, tr_time)
            t0, n = time.perf_counter(), 0
            while time.perf_counter() - t0 < args.cpu_budget:
                step = n % 4
                po.run_model(_plugin_env(z, step, tr_time), [tuple(x) for x in z[f"s{step}/decision_in"]])
                n += 1
            dt = time.perf_counter() - t0
            res["cpu_baseline"] = {"value": n / dt, "unit": "calls/s", "cores": 1, "kind": "port", "threads_note": "sequential per-environment restatement (the reference's one-call-at-a-time loop over small tensors, below torch's intra-op parallel grain): 1 thread",
                                   "sample": f"{n} run_model calls of the torch-fp64 plugin restatement "
                                             f"(pinned to the reference's outputs), 1 thread, {dt:.1f}s"}
        emit(res)


if __name__ == "__main__":
    main()
