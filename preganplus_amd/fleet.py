"""Streaming a fleet's cell-windows through the decision path (BASELINE config
C5, SURVEY.md §8(d): 1024 hosts = 64 independent 16-host cells, 1M windows per
cell, sharded over the GPUs).

A fleet's share does not sit in HBM when the interval starts: the windows
(run_encoder's normalised rows, PreGANPlus.py:107-112) and GOBI's placements
(result_cache, one-hot rows, scheduler/BaGTI/src/opt.py:9-15) arrive from host
memory.  ``FleetStreamer`` moves chunks of cell-windows through three streams:

  copy-in   pinned host -> HBM: the windows (fp32, 36H B per window) and one
            byte per container of placement (H B per window), into one of two
            device slots
  compute   pgp_schedule_onehot (the dense [C,H] rows K3 reads) ->
            pgp_forward (K1 GAT, K2 encoder, K2b decoders + classify, K3 GAN
            + decisions) into the slot's outputs
  copy-out  the slot's decision arrays -> pinned host (class per host, any,
            keep, final target per container; optionally every output)

Slot k of chunk i is reused by chunk i + 2: the copy-in waits for the compute
that read it, the compute waits for the copy-out that drained its outputs.
So PCIe in, the kernels and PCIe out of neighbouring chunks overlap, and the
rate is that of the slowest of the three.
"""
from __future__ import annotations

import ctypes

import torch

from . import _native

DECISION_KEYS = ("cls", "any", "keep", "final_target")
ALL_KEYS = ("logits", "protos", "cls", "any", "probs", "keep", "final_target", "gen_target")


def pinned_chunk(x: torch.Tensor, idx: torch.Tensor):
    """Host-side source chunk (pinned, so copy-in is an async DMA)."""
    return x.cpu().pin_memory(), idx.to(torch.uint8).cpu().pin_memory()


def schedule_onehot(idx: torch.Tensor, out: torch.Tensor, n_hosts: int, stream=None):
    """[B,C] uint8 placements (>= n_hosts: no host) -> [B,C,H] fp32 one-hot on
    the device (pgp_schedule_onehot)."""
    B = idx.shape[0]
    if idx.dtype != torch.uint8 or tuple(idx.shape) != (B, n_hosts) or tuple(out.shape) != (B, n_hosts, n_hosts) \
            or out.dtype != torch.float32 or not idx.is_cuda or not out.is_cuda:
        raise ValueError("schedule_onehot: uint8 [B,H] device placements -> float32 [B,H,H] device")
    st = stream if stream is not None else torch.cuda.current_stream(idx.device)
    _native.check(_native.lib().pgp_schedule_onehot(n_hosts, B, idx.data_ptr(), out.data_ptr(),
                                                    ctypes.c_void_p(st.cuda_stream)), "pgp_schedule_onehot")
    return out


class FleetStreamer:
    """Double-buffered host -> HBM -> host pipeline of one rank over a
    ``DecisionModel`` (see the module docstring).  ``chunk`` cell-windows per
    launch sequence; ``keys``: the outputs copied back."""

    def __init__(self, model, chunk: int, keys=DECISION_KEYS):
        self.m, self.chunk, self.keys = model, int(chunk), tuple(keys)
        H, dev = model.H, model.device
        self.H, self.dev = H, dev
        model.reserve(self.chunk)
        self.x = [torch.empty((self.chunk, 3, 3 * H), dtype=torch.float32, device=dev) for _ in range(2)]
        self.idx = [torch.empty((self.chunk, H), dtype=torch.uint8, device=dev) for _ in range(2)]
        self.sched = torch.empty((self.chunk, H, H), dtype=torch.float32, device=dev)
        self.out = [model.alloc_outputs(self.chunk) for _ in range(2)]
        self.s_in, self.s_cmp, self.s_out = (torch.cuda.Stream(dev) for _ in range(3))
        ev = lambda: [torch.cuda.Event() for _ in range(2)]
        self.in_done, self.cmp_done, self.out_done = ev(), ev(), ev()
        self.used = [False, False]

    def host_outputs(self, n_chunks: int):
        """Pinned host destinations for n_chunks chunks' outputs."""
        specs = {k: (v.shape[1:], v.dtype) for k, v in self.out[0].items() if k in self.keys}
        return [{k: torch.empty((self.chunk,) + tuple(s), dtype=d, pin_memory=True) for k, (s, d) in specs.items()}
                for _ in range(n_chunks)]

    def run(self, sources, n_chunks: int, dest=None):
        """Stream n_chunks chunks, chunk i from sources[i % len(sources)]
        ((x, idx) pinned pairs of ``chunk`` windows); outputs of chunk i go to
        dest[i % len(dest)] (pinned dicts, ``host_outputs``).  Returns after
        issuing; the caller synchronises (``torch.cuda.synchronize``)."""
        cur = torch.cuda.current_stream(self.dev)
        for s in (self.s_in, self.s_cmp, self.s_out):
            s.wait_stream(cur)   # inputs the caller prepared on its stream
        for i in range(n_chunks):
            k = i % 2
            xs, ids = sources[i % len(sources)]
            if xs.shape[0] != self.chunk or ids.shape[0] != self.chunk:
                raise ValueError("every source chunk holds `chunk` windows")
            if self.used[k]:
                self.s_in.wait_event(self.cmp_done[k])
            with torch.cuda.stream(self.s_in):
                self.x[k].copy_(xs, non_blocking=True)
                self.idx[k].copy_(ids, non_blocking=True)
                self.in_done[k].record(self.s_in)
            self.s_cmp.wait_event(self.in_done[k])
            if self.used[k]:
                self.s_cmp.wait_event(self.out_done[k])
            schedule_onehot(self.idx[k], self.sched, self.H, stream=self.s_cmp)
            self.m.forward(self.x[k], self.sched, out=self.out[k], stream=self.s_cmp)
            self.cmp_done[k].record(self.s_cmp)
            self.s_out.wait_event(self.cmp_done[k])
            if dest is not None:
                d = dest[i % len(dest)]
                with torch.cuda.stream(self.s_out):
                    for key in self.keys:
                        d[key].copy_(self.out[k][key], non_blocking=True)
            self.out_done[k].record(self.s_out)
            self.used[k] = True
        for s in (self.s_in, self.s_cmp, self.s_out):
            cur.wait_stream(s)
