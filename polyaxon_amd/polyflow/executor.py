"""Resident (warm) trial executor: one per GPU, runs trial after trial without leaving the process.

The reference runs every trial — including every Hyperband promotion, which it models as a *new*
experiment (``experiment.resume/restart``, polyaxon/hpsearch/iteration_managers/hyperband.py:94-113) —
as a fresh Kubernetes pod: image check, pod create, container start, framework import, CUDA context,
cuDNN autotune, and a 1–30 s chain of Celery hops around it (BASELINE.md "reference design constants").
On a single MI355X node the expensive, trial-invariant parts are all reusable, so polyflow keeps them
resident:

* the model, its flat fp32 weights/grads and optimizer state are allocated once (``FlatParams``);
* the full training step (forward, backward, fused optimizer, metric record) is captured once as a
  hipGraph and replayed for every step of every trial;
* everything trial-specific is device data rewritten by kernels: weights (``plx_init_flat``),
  optimizer state (``plx_zero_flat``), hyper-parameters (one 32-byte H2D copy), step counter;
* the step loss goes to a device ring (``plx_record_metric``); a trial's result is reduced on the device
  into the HPO metric tensor (``plx_commit_metric``), so no host sync happens inside a trial;
* Hyperband *resume* snapshots live in HBM (288 GB per GPU holds hundreds of ResNet-50 trial states), so
  a promotion is a device-to-device copy instead of a checkpoint file round trip.

The same class runs on CPU (no graph, reference kernels) for the unit tests.
"""
from __future__ import annotations

import time
from dataclasses import dataclass
from typing import Callable, Dict, Optional, Tuple

import torch
import torch.nn as nn

from polyaxon_amd.ops import _native, side_stream
from polyaxon_amd.ops.flat import FlatParams
from polyaxon_amd.ops.optim import FusedAdamW, FusedSGD
from polyaxon_amd.ops.wcache import ConvWeightCache


def _stream_ptr(dev: torch.device) -> int:
    return torch.cuda.current_stream(dev).cuda_stream


@dataclass
class TrialState:
    params: torch.Tensor
    opt: Dict[str, torch.Tensor]
    buffers: torch.Tensor
    step: torch.Tensor


class ResidentTrialExecutor:
    def __init__(self, model: nn.Module, batch: Tuple[torch.Tensor, torch.Tensor], device,
                 loss_fn: Optional[Callable] = None, optimizer: str = "sgd", use_graph: bool = True,
                 amp_dtype: Optional[torch.dtype] = torch.bfloat16, channels_last: bool = True,
                 ring_size: int = 4096, init_spec: Optional[Callable] = None,
                 lp_dtype: Optional[torch.dtype] = None):
        """``lp_dtype`` (the language models, GPU): the model computes from bf16 weights with bf16 gradients and the
        optimizer keeps the fp32 master (ops/flat.py lp mode); every re-init / restore refreshes the bf16 copy."""
        self.device = torch.device(device)
        self.is_cuda = self.device.type == "cuda"
        if channels_last:
            model = model.to(memory_format=torch.channels_last)
        self.model = model
        self.flat = FlatParams(model, self.device, channels_last=channels_last,
                               lp_dtype=lp_dtype if self.is_cuda else None)
        self.flat.enable_direct_grads(True)  # native ops accumulate weight grads straight into flat.grads
        self._flatten_buffers()
        self.step = torch.zeros(1, dtype=torch.int32, device=self.device)
        if optimizer == "sgd":
            self.opt = FusedSGD(self.flat, step_counter=self.step)
        elif optimizer == "adamw":
            self.opt = FusedAdamW(self.flat, step_counter=self.step)
        else:
            raise ValueError(f"unknown optimizer {optimizer!r}")
        # default: cross entropy of the fp32-cast logits; on the GPU in one fused HIP kernel each way (ops/lm.py
        # class_xent: no fp32 logits copy, log-softmax or NLL kernels between the head GEMM and its backward, where the
        # host launching them was the bottleneck of the forward -> backward hand-off; +0.1-0.2 %, r5_class_xent_ab.jsonl)
        # labels guaranteed inside [0, classes): the executor's own synthetic source with no more classes than the
        # head has outputs -- the fused kernels then skip F.cross_entropy's valid-row count
        fc = getattr(model, "fc", None)
        self._labels_in_range = (hasattr(batch, "next") and isinstance(getattr(batch, "classes", None), int)
                                 and isinstance(fc, nn.Linear) and batch.classes <= fc.out_features)
        if loss_fn is None:
            from polyaxon_amd.ops.lm import class_xent

            in_range = self._labels_in_range
            loss_fn = lambda out, y: class_xent(out, y, in_range=in_range)  # noqa: E731
        self.loss_fn = loss_fn
        # ``batch`` is either a fixed (x, y) pair or a data source with in-place ``next()`` (ops/synth.py) that the
        # step refills before every forward: a fresh device-generated batch per step, inside the captured graph
        self.data = batch if hasattr(batch, "next") else None
        if self.data is not None:
            self.x, self.y = self.data.x, self.data.y
        else:
            self.x, self.y = batch[0].to(self.device), batch[1].to(self.device)
        self.amp_dtype = amp_dtype if self.is_cuda else None
        self.ring_size = ring_size
        self.ring = torch.zeros(ring_size, dtype=torch.float32, device=self.device)
        spec = init_spec() if init_spec is not None else (model.init_spec() if hasattr(model, "init_spec") else None)
        self._init_spec = spec
        self._init_tables = self.flat.init_tables(spec) if (spec is not None and self.is_cuda) else None
        self.use_graph = use_graph and self.is_cuda
        # Eager device path: batch k+1 is generated on the side stream while step k's backward ends (the side
        # stream idles once its last weight gradient is done, beside the main stream's stem chain and optimizer),
        # into the other of two batch buffers; step k+1's forward waits on an event instead of running the
        # generator.  A graph-captured step keeps the generator inside the graph.  (Queueing batch k+1 at the start of
        # step k instead, beside the forward, measured no better; removed in round 6.)
        self._prefetch = (self.is_cuda and not self.use_graph and self.data is not None
                          and hasattr(self.data, "next_into") and side_stream.enabled())
        self._bufs = None          # [(x, y), (x, y)] when prefetching
        self._cur = 0              # buffer the next step consumes
        self._ready = None         # event after the generator wrote self._bufs[self._cur], or None
        self.graph: Optional[torch.cuda.CUDAGraph] = None
        self.graph_rejected = False
        self.graph_check_error: Optional[float] = None
        self.snapshots: Dict[object, TrialState] = {}
        # bf16 operands of every native conv from one launch per step (ops/wcache.py)
        self.wcache = None
        if self.is_cuda:
            cache = ConvWeightCache(model, self.flat.params)
            self.wcache = cache if len(cache) else None
        self.model.train()

    def enable_dp(self, bucket_mb="auto", process_group=None) -> None:
        """Data parallel over ``process_group`` (default: the default group; a resident DP gang, polyflow/resident.py):
        bucketed, backward-overlapped gradient all-reduce (parallel/ddp.py FlatDDP) before every optimizer step; the
        DP step runs eagerly."""
        from polyaxon_amd.parallel.ddp import FlatDDP

        self.ddp = FlatDDP(self.flat, process_group=process_group, bucket_mb=bucket_mb)
        self.use_graph = False
        self._prefetch = False

    ddp = None

    # ------------------------------------------------------------------ buffers (BN running stats)
    def _flatten_buffers(self) -> None:
        bufs = [(n, b) for n, b in self.model.named_buffers() if b.dtype == torch.float32]
        total = sum(b.numel() for _, b in bufs)
        self.buffers = torch.zeros(max(total, 1), dtype=torch.float32, device=self.device)
        self._buffer_init = torch.zeros_like(self.buffers)
        off = 0
        for name, b in bufs:
            view = self.buffers[off: off + b.numel()].view_as(b)
            view.copy_(b)
            self._buffer_init[off: off + b.numel()].copy_(b.reshape(-1))
            mod = self.model
            parts = name.split(".")
            for p in parts[:-1]:
                mod = getattr(mod, p)
            mod._buffers[parts[-1]] = view
            off += b.numel()

    # ------------------------------------------------------------------ the step
    def _train_step(self) -> None:
        prefetch = self._prefetch and not torch.cuda.is_current_stream_capturing()
        if prefetch:
            main = torch.cuda.current_stream(self.device)
            if self._bufs is None:
                self._bufs = [(self.data.x, self.data.y), (torch.empty_like(self.data.x), torch.empty_like(self.data.y))]
            if self._ready is None:
                self.data.next_into(*self._bufs[self._cur], main)
            else:
                main.wait_event(self._ready)
            self.x, self.y = self._bufs[self._cur]
            # every earlier step's use of the other buffer is complete in main-stream order from here
            step_start = torch.cuda.Event()
            step_start.record(main)
        elif self.data is not None:
            self.data.next()
        if self.wcache is not None:
            self.wcache.activate()
        try:
            if self.amp_dtype is not None:
                with torch.autocast("cuda", dtype=self.amp_dtype):
                    out = self.model(self.x)
                    loss = self.loss_fn(out, self.y)
                loss.backward()
            else:
                out = self.model(self.x)
                loss = self.loss_fn(out, self.y)
                loss.backward()
        finally:
            if self.wcache is not None:
                self.wcache.deactivate()
        side_stream.join(self.device)  # weight-gradient GEMMs overlapped on the side stream (ops/side_stream.py)
        if self.ddp is not None:
            self.ddp.finish()  # the gang's averaged gradients
        if prefetch:
            # queued after the join: the main stream does not wait for it before the optimizer
            self._queue_next_batch(step_start)
        self.opt.step_()
        self._record(loss.detach())

    def _queue_next_batch(self, step_start) -> None:
        """Generate the next batch into the other buffer on the side stream, after ``step_start`` (the main-stream
        point from which every earlier step's use of that buffer is complete); the next step waits on ``_ready``."""
        side = side_stream.stream_for(self.device)
        side.wait_event(step_start)
        nxt = self._cur ^ 1
        self.data.next_into(*self._bufs[nxt], side)
        self._ready = torch.cuda.Event()
        self._ready.record(side)
        self._cur = nxt

    def _record(self, loss: torch.Tensor) -> None:
        if self.is_cuda:
            loss = loss.float().contiguous()
            rc = _native.lib("plx_train").plx_record_metric(loss.data_ptr(), 0, self.ring.data_ptr(),
                                                             self.step.data_ptr(), self.ring_size,
                                                             _stream_ptr(self.device))
            _native.check(rc, "plx_record_metric")
            self._last_loss = loss  # keep alive for the graph's lifetime
        else:
            s = int(self.step.item())
            self.ring[s % self.ring_size] = float(loss)
            self.step += 1

    def capture(self, warmup: int = 3, verify: bool = True, tol: float = 0.05) -> bool:
        """Warm up (MIOpen find, allocator) and capture the training step as a hipGraph.

        With ``verify`` the graph is checked before it is trusted: one eager step and one replay run from the
        same saved state and their parameter updates must agree to ``tol`` (relative, and finite).  A library
        kernel that is not capture-safe (e.g. one relying on an uncaptured memset) shows up here as a diverging
        update, and the executor stays eager instead of training on garbage.  Returns whether the graph is used.
        """
        if not self.use_graph:
            return False
        s = torch.cuda.Stream(self.device)
        s.wait_stream(torch.cuda.current_stream(self.device))
        with torch.cuda.stream(s):
            for _ in range(warmup):
                self._train_step()
        torch.cuda.current_stream(self.device).wait_stream(s)
        torch.cuda.synchronize(self.device)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self._train_step()
        torch.cuda.synchronize(self.device)
        self.graph = g
        if verify and not self._verify_graph(tol):
            self.graph = None
            self.graph_rejected = True
        return self.graph is not None

    def _verify_graph(self, tol: float) -> bool:
        key = "__graph_check__"
        self.snapshot(key)
        p0 = self.flat.params.detach().clone()
        # a device data stream (ops/synth.py) advances its counter every step: both runs must see the same batch
        counter = getattr(self.data, "counter", None)
        c0 = counter.clone() if counter is not None else None
        self.graph, g = None, self.graph
        self.run(1)  # eager
        d_eager = self.flat.params.detach() - p0
        self.restore(key)
        if counter is not None:
            counter.copy_(c0)
        self.graph = g
        self.run(1)  # replay
        d_graph = self.flat.params.detach() - p0
        self.restore(key)
        self.drop(key)
        torch.cuda.synchronize(self.device)
        err = float((d_eager - d_graph).norm() / (d_eager.norm() + 1e-12))
        self.graph_check_error = err
        return bool(torch.isfinite(d_graph).all()) and err < tol

    # ------------------------------------------------------------------ trial lifecycle
    def reset(self, seed: int) -> None:
        """Fresh random weights + zero optimizer state + step 0 (a new trial, reference RESTART)."""
        with torch.no_grad():
            if self.is_cuda and self._init_tables is not None:
                t = self._init_tables
                rc = _native.lib("plx_train").plx_init_flat(
                    self.flat.params.data_ptr(), t["chunk_lo"].data_ptr(), t["chunk_hi"].data_ptr(),
                    t["chunk_seg"].data_ptr(), int(t["chunk_lo"].numel()), t["seg_kind"].data_ptr(),
                    t["seg_scale"].data_ptr(), int(seed) & 0xFFFFFFFFFFFFFFFF, _stream_ptr(self.device))
                _native.check(rc, "plx_init_flat")
            elif self._init_spec is not None:
                self.flat.init_reference(self._init_spec, seed)
            self.opt.reset_state()
            self._zero_grads()
            self.flat.sync_lp()
            self.buffers.copy_(self._buffer_init)
            self.step.zero_()

    def _zero_grads(self) -> None:
        self.flat.grads.zero_()
        if self.flat.lp_grads is not None:
            self.flat.lp_grads.zero_()
        self.flat.grads_consumed()

    def set_hparams(self, **hp) -> None:
        self.opt.set_hparams(**{k: v for k, v in hp.items() if k in self.opt.HP})

    def run(self, n_steps: int) -> None:
        for _ in range(n_steps):
            if self.graph is not None:
                self.graph.replay()
            else:
                self._train_step()

    def commit(self, out: torch.Tensor, slot: int, window: int = 10) -> None:
        """out[slot] = mean loss over the last ``window`` steps, computed on the device."""
        if self.is_cuda:
            rc = _native.lib("plx_train").plx_commit_metric(self.ring.data_ptr(), self.step.data_ptr(),
                                                             self.ring_size, window, out.data_ptr(), slot,
                                                             _stream_ptr(self.device))
            _native.check(rc, "plx_commit_metric")
        else:
            s = int(self.step.item())
            w = min(window, s)
            if w == 0:
                out.view(-1)[slot] = float("nan")
            else:
                idx = [(s - 1 - j) % self.ring_size for j in range(w)]
                out.view(-1)[slot] = self.ring[idx].mean()

    def losses(self) -> torch.Tensor:
        s = int(self.step.item())
        n = min(s, self.ring_size)
        idx = [(s - n + j) % self.ring_size for j in range(n)]
        return self.ring[idx].cpu()

    # ------------------------------------------------------------------ HBM-resident snapshots
    def snapshot(self, key) -> None:
        st = self.snapshots.get(key)
        bufs = self.opt.state_buffers()
        if st is None:
            st = TrialState(torch.empty_like(self.flat.params), {k: torch.empty_like(v) for k, v in bufs.items()},
                            torch.empty_like(self.buffers), torch.empty_like(self.step))
            self.snapshots[key] = st
        st.params.copy_(self.flat.params, non_blocking=True)
        for k, v in bufs.items():
            st.opt[k].copy_(v, non_blocking=True)
        st.buffers.copy_(self.buffers, non_blocking=True)
        st.step.copy_(self.step, non_blocking=True)

    def restore(self, key) -> None:
        st = self.snapshots[key]
        self.flat.params.copy_(st.params, non_blocking=True)
        for k, v in self.opt.state_buffers().items():
            v.copy_(st.opt[k], non_blocking=True)
        self.buffers.copy_(st.buffers, non_blocking=True)
        self.step.copy_(st.step, non_blocking=True)
        self._zero_grads()
        self.flat.sync_lp()

    def drop(self, key) -> None:
        self.snapshots.pop(key, None)

    def snapshot_bytes(self) -> int:
        n = self.flat.params.numel() * (1 + len(self.opt.state_buffers())) + self.buffers.numel()
        return 4 * n
