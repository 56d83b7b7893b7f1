"""Data parallelism over independent meshes: one process per GPU, every rank runs
the full forward/backward on its own meshes, then ONE gradient all-reduce (RCCL over xGMI on
the MI355X node; gloo in CPU tests) and a replicated optimizer step.

Loss normalisation matches a single-process MSELoss over the union batch (utils.py:191):
each rank back-propagates sum((pred - y)^2) / N_global, where N_global = all-reduced count of
target elements, so the summed gradients equal the union-batch gradient exactly even when
ranks hold different node counts.
"""
from __future__ import annotations

import os

import torch
import torch.distributed as dist


def init_from_env(backend=None, force=None):
    """Initialise torch.distributed from torchrun's env (RANK/WORLD_SIZE/MASTER_*).

    Backend: `backend`, else $AEROGNN_DIST_BACKEND, else "nccl" (= RCCL on ROCm) when a GPU is
    present and "gloo" otherwise. gloo with device tensors stages through host memory
    (rehearsing N ranks on one GPU; never the production path). A single process stays
    undistributed unless `force` (or $AEROGNN_DIST_FORCE=1): then a world of one runs the whole
    collective path (bucketed async all-reduce, wait, unpack) on a real communicator."""
    if force is None:
        force = os.environ.get("AEROGNN_DIST_FORCE", "0") == "1"
    if not dist.is_available() or (int(os.environ.get("WORLD_SIZE", "1")) <= 1 and not force):
        return 0, 1
    if not dist.is_initialized():
        if backend is None:
            backend = os.environ.get("AEROGNN_DIST_BACKEND") or ("nccl" if torch.cuda.is_available() else "gloo")
        dist.init_process_group(backend=backend)
    return dist.get_rank(), dist.get_world_size()


def _host_staged() -> bool:
    return dist.get_backend() == "gloo"


def all_reduce_(t, async_op=False):
    """SUM all-reduce in place; device tensors go through host memory under gloo."""
    if t.is_cuda and _host_staged():
        h = t.cpu()
        dist.all_reduce(h)
        t.copy_(h)
        return None
    return dist.all_reduce(t, async_op=async_op)


def world():
    if dist.is_available() and dist.is_initialized():
        return dist.get_rank(), dist.get_world_size()
    return 0, 1


def active() -> bool:
    """A process group exists (also a forced world of one): collectives run."""
    return dist.is_available() and dist.is_initialized()


def global_count(n_local: int, device) -> float:
    t = torch.tensor([float(n_local)], dtype=torch.float64, device=device)
    if active():
        all_reduce_(t)
    return float(t.item())


def mse_sum_loss(pred, y, n_global: float):
    """sum of squared errors / global element count (== MSELoss on the union batch), computed
    in at least fp32 (bf16 predictions are promoted; fp64 stays fp64)."""
    dt = torch.promote_types(pred.dtype, torch.float32)
    return ((pred.to(dt) - y.to(dt)) ** 2).sum() / n_global


class GradAllReduce:
    """Bucketed gradient all-reduce (SUM) of a module's parameters, overlapped with the backward.

    Gradients are packed into a few contiguous buckets in the parameters' own dtype (fp32 master
    weights: ~4 buckets of <= 4 MB for the 2.9M-parameter model, each one RCCL ring all-reduce,
    link-bound on point-to-point xGMI) and unpacked in place. A bucket never mixes dtypes.
    Buckets are formed in REVERSE registration order, the order the backward produces them
    (decoder, up path, ..., encoders).

    `arm()` before the last (or only) micro-batch's backward: each bucket is then packed and its
    all-reduce launched (async, on the collective stream) from a post-accumulate-grad hook the
    moment its last gradient lands, so the transfer overlaps the rest of the backward. Calling
    the object afterwards launches any bucket that never fired, waits for all of them and
    unpacks. Without `arm()` everything happens in the call, after the backward.
    """

    def __init__(self, params, bucket_bytes=4 << 20):
        self.params = [p for p in params if p.requires_grad]
        self.buckets = []
        cur, size = [], 0
        for p in reversed(self.params):
            if cur and cur[-1].dtype != p.dtype:
                self.buckets.append(cur)
                cur, size = [], 0
            cur.append(p)
            size += p.numel() * p.element_size()
            if size >= bucket_bytes:
                self.buckets.append(cur)
                cur, size = [], 0
        if cur:
            self.buckets.append(cur)
        self._flat = None
        self._armed = False
        self._works = {}
        self._pending = None
        self._hooks = []
        self.launched_in_hooks = 0  # buckets the last armed backward launched from its hooks
        # optional: a list that __call__ appends (start, end) HIP-event pairs to, bracketing the
        # all-reduce work left after the backward (the exposed part: remaining launches, waits, unpack)
        self.exposed_events = None
        if active():
            where = {}
            for bi, b in enumerate(self.buckets):
                for p in b:
                    where[id(p)] = bi
            for p in self.params:
                if hasattr(p, "register_post_accumulate_grad_hook"):
                    self._hooks.append(p.register_post_accumulate_grad_hook(self._hook(where[id(p)])))

    def _ensure_flat(self):
        if self._flat is None:
            dev = self.params[0].device
            self._flat = [torch.empty(sum(p.numel() for p in b), dtype=b[0].dtype, device=dev)
                          for b in self.buckets]

    def arm(self):
        if not active():
            return
        self._armed = True
        self._works = {}
        self.launched_in_hooks = 0
        self._pending = [len(b) for b in self.buckets]
        self._next = 0

    def _hook(self, bi):
        def fire(_p):
            if not self._armed:
                return
            self._pending[bi] -= 1
            # RCCL matches collectives across ranks by call order: launch buckets strictly in
            # index order (as DDP's reducer does), each as soon as it and all before it are ready
            while self._next < len(self.buckets) and self._pending[self._next] == 0:
                self._launch(self._next)
                self._next += 1
                self.launched_in_hooks += 1
        return fire

    def _launch(self, bi):
        self._ensure_flat()
        flat = self._flat[bi]
        o = 0
        for p in self.buckets[bi]:
            n = p.numel()
            if p.grad is not None:
                flat[o:o + n].copy_(p.grad.reshape(-1))
            else:
                flat[o:o + n].zero_()
            o += n
        self._works[bi] = all_reduce_(flat, async_op=True)

    def __call__(self):
        # step boundary: a fused-backward fault word read during this backward raises here, on the
        # faulting rank, before it waits for its buckets (aerognn/core.py fault_checkpoint)
        from . import core
        core.fault_checkpoint()
        if not active():
            return
        ev = None
        if self.exposed_events is not None:
            ev = (torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True))
            ev[0].record()
        for bi in range(len(self.buckets)):  # the rest, in index order
            if bi not in self._works:
                self._launch(bi)
        self._armed = False
        for bi, (b, flat) in enumerate(zip(self.buckets, self._flat)):
            w = self._works.get(bi)
            if w is not None:
                w.wait()
            o = 0
            for p in b:
                n = p.numel()
                if p.grad is None:
                    p.grad = torch.zeros_like(p)
                p.grad.copy_(flat[o:o + n].view_as(p.grad))
                o += n
        self._works = {}
        if ev is not None:
            ev[1].record()
            self.exposed_events.append(ev)
