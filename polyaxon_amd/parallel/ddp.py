"""Data parallelism over RCCL for flat-parameter models (PyTorchJob-equivalent training inside a trial).

The reference provides no collectives; its PyTorch experiments get MASTER_ADDR/RANK/
WORLD_SIZE and call NCCL themselves.  This module is what a polyflow DP trial uses on MI355X:

* gradients already live in ONE flat fp32 buffer (ops/flat.py); it is cut into contiguous buckets of
  ``bucket_mb`` (default 64 MB: large enough that each RCCL ring/tree step saturates the 7 xGMI links
  of an MI355X, small enough that the first bucket is ready early in the backward);
* a post-accumulate-grad hook on every parameter counts down its bucket; the moment a bucket is complete
  its ``all_reduce(AVG)`` is launched asynchronously (``async_op=True``: RCCL runs on its own stream),
  so communication overlaps the rest of the backward; ``finish()`` waits for the tail;
* segments are bucketed in reverse registration order so the buckets fill in backward order;
* lp mode (FlatParams ``lp_dtype=bf16``, the language models): the weight gradients are bf16, so the
  all-reduce moves half the bytes; buckets never straddle the bf16 / fp32-tail boundary.  Direct-gradient
  ops (ops/lm.py, ops/rmsnorm.py: GEMM-written weights, bias / norm sums written into the slots) return None and
  are still counted by autograd's post-accumulate hook, which runs once per parameter per backward after every
  Function feeding it; each segment counts its bucket down once per step.  (Optimizer-state sharding / ZeRO-1 is
  not implemented: an 8B model's fp32 master + moments are 96 GB, which one 288 GB MI355X holds unsharded.)
* optimizer in the backward (``optimizer=``, a FusedAdamW): the moment a bucket's gradient is complete (and, with
  DP, its all-reduce is done) the AdamW update of that bucket runs on a side stream, overlapped with the rest of
  the backward instead of one HBM-bound pass over every parameter after it (~41 ms of a 227 ms Llama-3 8B step on
  one MI355X; measured: the overlap mostly moves that time into the backward's memory-bound kernels, so the LM
  trainer leaves it off by default, PLX_OPT_IN_BACKWARD=1).  Each parameter's backward uses are issued before its
  bucket counts down (its AccumulateGrad hook runs after every Function that reads the weight), and ``finish()``
  makes the main stream wait for the optimizer stream before the next forward reads the updated bf16 weights.
  Same per-element update as the monolithic step.
Backend ``"nccl"`` is RCCL on ROCm; ``"gloo"`` works for CPU tests.
"""
from __future__ import annotations

import datetime
import os
from typing import List, Optional

import torch
import torch.distributed as dist

from polyaxon_amd.ops.flat import FlatParams


def init_from_env(backend: Optional[str] = None, device: Optional[torch.device] = None) -> dict:
    """Initialise torch.distributed from the polyflow / torchrun env contract (RANK, WORLD_SIZE,
    MASTER_ADDR, MASTER_PORT, LOCAL_RANK). Returns {rank, world, local_rank, device}."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if backend is None:
        backend = "nccl" if torch.cuda.is_available() else "gloo"
    if device is None:
        device = torch.device("cuda", local) if backend == "nccl" else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if backend == "nccl" else {}
        # collective watchdog: polyflow sets PLX_COLLECTIVE_TIMEOUT_S (+ TORCH_NCCL_ASYNC_ERROR_HANDLING) for
        # multi-rank trials so a dead peer fails this rank instead of hanging it (polyflow/env.py)
        timeout = float(os.environ.get("PLX_COLLECTIVE_TIMEOUT_S", "0") or 0)
        if timeout > 0:
            kw["timeout"] = datetime.timedelta(seconds=timeout)
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return {"rank": rank, "world": world, "local_rank": local, "device": device, "backend": backend}


class MetricReducer:
    """Cross-rank mean of a DP trial's scalar metrics (the loss the tracking client logs, the final result).

    SURVEY.md §2.3 names the metric all-reduce as a framework-owned collective: on the GPU it runs on the C++ RCCL
    communicator (csrc/rccl_comm.cpp, one ``ncclAllReduce(avg)`` of a few floats on the current HIP stream, no
    ProcessGroup layer and no host sync); on the CPU (gloo tests) through torch.distributed.  World 1: identity."""

    def __init__(self, device: torch.device, process_group=None, force_comm: bool = False):
        """``force_comm``: build the RCCL communicator even at world 1 (a single-GPU test of the real path)."""
        self.device = device
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.comm = None
        if (self.world > 1 or force_comm) and device.type == "cuda" and dist.is_initialized():
            from polyaxon_amd.parallel.rccl import RcclComm

            self.comm = RcclComm.from_torch_distributed(process_group)

    def mean(self, t: torch.Tensor) -> torch.Tensor:
        """Mean over ranks of a small float tensor (returned new; the input is untouched)."""
        out = t.detach().float().reshape(-1).clone()
        if self.comm is not None:
            return self.comm.all_reduce(out, op="avg")
        if self.world == 1:
            return out
        dist.all_reduce(out, op=dist.ReduceOp.SUM, group=self.pg)
        return out.div_(self.world)

    def close(self) -> None:
        if self.comm is not None:
            self.comm.close()
            self.comm = None


class FlatDDP:
    def __init__(self, flat: FlatParams, process_group=None, bucket_mb: float = 64.0, overlap: bool = True,
                 force_collectives: bool = False, optimizer=None):
        """``force_collectives``: launch every bucket's all-reduce even at world 1 (hooks on), so a single-GPU
        test executes the real RCCL path and can count the launches (``launched``).  ``optimizer``: a FusedAdamW
        whose update then runs per bucket inside the backward (``step_range_``); its ``step_()`` only closes the
        step."""
        self.flat = flat
        self.opt = optimizer
        if optimizer is not None:
            optimizer.in_backward = True
            if flat.params.is_cuda:  # A/B knob: block cap of the in-backward update (csrc/train_kernels.hip)
                from polyaxon_amd.ops import _native

                _native.lib("plx_train").plx_set_adamw_grid_cap(int(os.environ.get("PLX_OPT_BWD_GRID", "2048")))
        self._side = torch.cuda.Stream(device=flat.device) if (optimizer is not None and flat.params.is_cuda) else None
        self.stepped = 0
        if flat.lp_params is None:
            # fp32 (ResNet) mode keeps autograd's accumulation: its native ops' direct writes are not ordered
            # against the all-reduce streams.  lp-mode direct writes are counted by the same post-accumulate hooks.
            flat.enable_direct_grads(False)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.force = bool(force_collectives) and dist.is_initialized()
        self.overlap = (overlap and (self.world > 1 or self.force)) or optimizer is not None
        self.launched = 0
        self.avg_supported = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
        bucket_elems = max(1, int(bucket_mb * 2 ** 20 / 4))
        segs = list(reversed(flat.segments))
        self.buckets: List[tuple] = []          # (lo, hi) element ranges of the flat buffer
        self.seg_bucket = {}
        cur: List = []
        size = 0
        for seg in segs:
            if cur and flat.lp_grads is not None and cur[-1].decay != seg.decay:
                self._close(cur)  # a bucket never spans the fp32 tail and the bf16 gradients
                cur, size = [], 0
            cur.append(seg)
            size += seg.numel
            if size >= bucket_elems:
                self._close(cur)
                cur, size = [], 0
        if cur:
            self._close(cur)
        self._pending = [0] * len(self.buckets)
        self._handles: List = []
        self._hooks = []
        self._ready: List[bool] = [False] * len(flat.segments)
        if self.overlap:
            # autograd runs a parameter's AccumulateGrad node -- and so this hook -- once per backward, after every
            # Function that feeds it, including direct-gradient ops (ops/lm.py, ops/rmsnorm.py) that wrote the
            # flat slot themselves and returned None: the hook is the readiness signal for both kinds
            for i, seg in enumerate(flat.segments):
                p = flat.parameter(seg.name)
                self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(self.seg_bucket[seg.name], i)))
        self.reset()

    def _close(self, segs) -> None:
        lo = min(s.offset for s in segs)
        hi = max(s.offset + ((s.numel + 3) & ~3) for s in segs)
        b = len(self.buckets)
        self.buckets.append((lo, hi, len(segs)))
        for s in segs:
            self.seg_bucket[s.name] = b

    def reset(self) -> None:
        self._pending = [n for _, _, n in self.buckets]
        self._ready = [False] * len(self.flat.segments)
        self._handles = []

    def _make_hook(self, b: int, seg: int):
        def hook(_p):
            if self._ready[seg]:  # a segment counts its bucket down once per step
                return
            self._ready[seg] = True
            self._pending[b] -= 1
            if self._pending[b] == 0:
                self._launch(b)
        return hook

    def _launch(self, b: int) -> None:
        lo, hi, _ = self.buckets[b]
        view = self.flat.grad_view(lo, hi)
        h, div = None, None
        if self.world > 1 or self.force:
            self.launched += 1
            if self.avg_supported:
                h = dist.all_reduce(view, op=dist.ReduceOp.AVG, group=self.pg, async_op=True)
            else:
                h = dist.all_reduce(view, op=dist.ReduceOp.SUM, group=self.pg, async_op=True)
                div = view
        if self.opt is None:
            self._handles.append((h, div))
            return
        # the bucket's update: after its (reduced) gradient, on the optimizer stream
        self.stepped += 1
        if self._side is None:  # CPU: synchronous
            if h is not None:
                h.wait()
            if div is not None:
                div.div_(self.world)
            self.opt.step_range_(lo, hi)
            return
        self._side.wait_stream(torch.cuda.current_stream(self.flat.device))
        with torch.cuda.stream(self._side):
            if h is not None:
                h.wait()  # the optimizer stream waits for RCCL's stream (host does not block)
            if div is not None:
                div.div_(self.world)
            self.opt.step_range_(lo, hi, self._side.cuda_stream)

    def finish(self) -> None:
        """Call after backward(): launches any bucket not fired by hooks, waits, averages (and, with an optimizer
        in the backward, has the main stream wait for every bucket's update)."""
        if self.world == 1 and not self.force and self.opt is None:
            return
        if not self.overlap:
            for b in range(len(self.buckets)):
                self._launch(b)
        else:
            for b, left in enumerate(self._pending):
                if left > 0:  # parameters without grads this step (unused): reduce / update anyway
                    self._launch(b)
        for h, view in self._handles:
            if h is not None:
                h.wait()
            if view is not None:
                view.div_(self.world)
        if self._side is not None:
            torch.cuda.current_stream(self.flat.device).wait_stream(self._side)
        self.reset()

    def broadcast_params(self, src: int = 0) -> None:
        """Make every rank start from rank ``src``'s weights (one collective over the flat buffer)."""
        if self.world > 1 or self.force:
            dist.broadcast(self.flat.params, src=src, group=self.pg)
            self.flat.sync_lp()

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
