"""Data parallelism over RCCL for flat-parameter models (PyTorchJob-equivalent training inside a trial).

The reference provides no collectives; its PyTorch experiments get MASTER_ADDR/RANK/
WORLD_SIZE and call NCCL themselves.  This module is what a polyflow DP trial uses on MI355X:

* gradients already live in ONE flat fp32 buffer (ops/flat.py); it is cut into contiguous buckets of
  ``bucket_mb`` (default ``"auto"``: the xGMI cost model of parallel/comm_plan.py -- the smallest bucket whose ring
  all-reduce runs at >= 90 % of the W - 1 links' bandwidth, capped so >= 4 buckets overlap the backward);
* a post-accumulate-grad hook on every parameter counts down its bucket; the moment a bucket is complete
  its ``all_reduce(AVG)`` is launched asynchronously (``async_op=True``: RCCL runs on its own stream),
  so communication overlaps the rest of the backward; ``finish()`` waits for the tail;
* segments are bucketed in reverse registration order so the buckets fill in backward order;
* lp mode (FlatParams ``lp_dtype=bf16``, the language models): the weight gradients are bf16, so the
  all-reduce moves half the bytes; buckets never straddle the bf16 / fp32-tail boundary.  Direct-gradient
  ops (ops/lm.py, ops/rmsnorm.py: GEMM-written weights, bias / norm sums written into the slots) return None and
  are still counted by autograd's post-accumulate hook, which runs once per parameter per backward after every
  Function feeding it; each segment counts its bucket down once per step.
* optimizer in the backward (``optimizer=``, a FusedAdamW): the moment a bucket's gradient is complete (and, with
  DP, its all-reduce is done) the AdamW update of that bucket runs on a side stream, overlapped with the rest of
  the backward instead of one HBM-bound pass over every parameter after it (~41 ms of a 227 ms Llama-3 8B step on
  one MI355X; measured: the overlap mostly moves that time into the backward's memory-bound kernels, so the LM
  trainer leaves it off by default, PLX_OPT_IN_BACKWARD=1).  Each parameter's backward uses are issued before its
  bucket counts down (its AccumulateGrad hook runs after every Function that reads the weight), and ``finish()``
  makes the main stream wait for the optimizer stream before the next forward reads the updated bf16 weights.
  Same per-element update as the monolithic step.
* ZeRO-1 (``shard_optimizer=True``, with ``optimizer``): each bucket's gradient is reduce-scattered instead of
  all-reduced -- rank r receives the averaged gradient of the r-th W-th of the bucket (in place, in its own slice of
  the flat gradient buffer) --, AdamW updates only that slice (its moments live in a packed 1/W-size state), and the
  updated weights are all-gathered back (the bf16 model copy in lp mode, the fp32 parameters otherwise) before the
  next forward.  Reduce-scatter + all-gather move the bytes of one all-reduce; the update pass and the AdamW moments
  shrink W-fold (Llama-3 8B at DP 8: 64 GB of moments -> 8 GB per rank, ~42 ms of update -> ~5 ms).  The last
  ``numel % 4W`` elements of a bucket are all-reduced and updated identically on every rank.  In lp mode the fp32
  master of the slices other ranks own goes stale (only the bf16 copy is gathered): ``gather_master()`` refreshes it
  for a checkpoint.
Backend ``"nccl"`` is RCCL on ROCm; ``"gloo"`` works for CPU tests.
"""
from __future__ import annotations

import datetime
import os
from contextlib import nullcontext as _nullcontext
from typing import List, Optional

import torch
import torch.distributed as dist

from polyaxon_amd.ops import side_stream
from polyaxon_amd.ops.flat import FlatParams


def init_from_env(backend: Optional[str] = None, device: Optional[torch.device] = None) -> dict:
    """Initialise torch.distributed from the polyflow / torchrun env contract (RANK, WORLD_SIZE,
    MASTER_ADDR, MASTER_PORT, LOCAL_RANK). Returns {rank, world, local_rank, device}.  The default backend is gloo:
    the process group is the rendezvous (it ships the RCCL unique id and the host-side control traffic); a DP trial's
    device collectives run on ONE framework communicator (parallel/comm.py), not on ProcessGroupNCCL's."""
    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    explicit = backend is not None
    if backend is None:  # the rendezvous: device collectives go through parallel/comm.py's communicator
        backend = "gloo"
    if device is None:
        # the GPU only when the caller asks for it (nccl, or no backend named on a GPU host): an explicit gloo backend
        # keeps the CPU, so CPU data-parallel runs on a GPU host never initialise HIP
        cuda = backend == "nccl" or (not explicit and torch.cuda.is_available())
        device = torch.device("cuda", local) if cuda else torch.device("cpu")
    if device.type == "cuda":
        torch.cuda.set_device(device)
    if world > 1 and not dist.is_initialized():
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        kw = {"device_id": device} if backend == "nccl" else {}
        # the rendezvous' own deadline: polyflow sets PLX_COLLECTIVE_TIMEOUT_S for multi-rank trials
        # (polyflow/env.py), so a dead peer fails this rank's gloo control traffic instead of hanging it; the device
        # collectives' deadline is the framework communicator's watchdog (csrc/rccl_comm.cpp), same variable
        timeout = float(os.environ.get("PLX_COLLECTIVE_TIMEOUT_S", "0") or 0)
        if timeout > 0:
            kw["timeout"] = datetime.timedelta(seconds=timeout)
        dist.init_process_group(backend, rank=rank, world_size=world, **kw)
    return {"rank": rank, "world": world, "local_rank": local, "device": device, "backend": backend}


class MetricReducer:
    """Cross-rank mean of a DP trial's scalar metrics (the loss the tracking client logs, the final result).

    SURVEY.md §2.3 names the metric all-reduce as a framework-owned collective: it runs on the process's shared
    communicator (parallel/comm.py: RCCL on the GPU -- one ``ncclAllReduce(avg)`` of a few floats on the current HIP
    stream, no host sync --, the gloo shim on the CPU), the same one FlatDDP uses.  World 1: identity."""

    def __init__(self, device: torch.device, process_group=None, force_comm: bool = False):
        """``force_comm``: take the communicator even at world 1 (a single-GPU test of the real path)."""
        self.device = device
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.comm = None
        if (self.world > 1 or force_comm) and dist.is_initialized():
            from polyaxon_amd.parallel import comm as _comm

            self.comm = _comm.acquire(process_group, device)

    def mean(self, t: torch.Tensor) -> torch.Tensor:
        """Mean over ranks of a small float tensor (returned new; the input is untouched)."""
        out = t.detach().float().reshape(-1).clone()
        if self.comm is None:
            return out
        if self.comm.native_avg:
            return self.comm.all_reduce(out, op="avg")
        return self.comm.all_reduce(out, op="sum").div_(self.world)

    def close(self) -> None:
        if self.comm is not None:
            from polyaxon_amd.parallel import comm as _comm

            _comm.release(self.comm)
            self.comm = None


class _StreamWork:
    """A collective issued on our own stream: ``wait()`` orders the CURRENT stream after it (the host never blocks),
    as ProcessGroupNCCL's ``Work.wait()`` does."""

    def __init__(self, stream: "torch.cuda.Stream"):
        self.event = torch.cuda.Event()
        self.event.record(stream)

    def wait(self) -> None:
        torch.cuda.current_stream().wait_event(self.event)


class FlatDDP:
    def __init__(self, flat: FlatParams, process_group=None, bucket_mb="auto", overlap: bool = True,
                 force_collectives: bool = False, optimizer=None, shard_optimizer: bool = False):
        """``bucket_mb``: bucket size in MB of fp32-sized elements, or ``"auto"``: planned from the gradient bytes
        and the world size by the xGMI cost model (parallel/comm_plan.py; ``self.plan`` keeps its numbers).
        ``force_collectives``: launch every bucket's all-reduce even at world 1 (hooks on), so a single-GPU
        test executes the real RCCL path and can count the launches (``launched``).  ``optimizer``: a FusedAdamW
        whose update then runs per bucket inside the backward (``step_range_``); its ``step_()`` only closes the
        step.  ``shard_optimizer``: ZeRO-1 over the optimizer's state (see the module docstring)."""
        if shard_optimizer and optimizer is None:
            raise ValueError("shard_optimizer needs the optimizer that runs inside the backward")
        self.flat = flat
        self.opt = optimizer
        if optimizer is not None:
            optimizer.in_backward = True
        self._side = torch.cuda.Stream(device=flat.device) if (optimizer is not None and flat.params.is_cuda) else None
        self.stepped = 0
        if flat.lp_params is None:
            # fp32 (ResNet) mode keeps autograd's accumulation: its native ops' direct writes are not ordered
            # against the all-reduce streams.  lp-mode direct writes are counted by the same post-accumulate hooks.
            flat.enable_direct_grads(False)
        self.pg = process_group
        self.world = dist.get_world_size(process_group) if dist.is_initialized() else 1
        self.rank = dist.get_rank(process_group) if dist.is_initialized() else 0
        self.force = bool(force_collectives) and dist.is_initialized()
        self.coll = self.world > 1 or self.force            # collectives run (world > 1, or forced at world 1)
        self.nccl = dist.is_initialized() and dist.get_backend(process_group) == "nccl"
        pg_mode = os.environ.get("PLX_DDP_COMM", "comm") == "pg"
        if pg_mode and self.coll and flat.params.is_cuda and not self.nccl:
            # the torch.distributed A/B path on the GPU needs ProcessGroupNCCL: the trial's process group is the gloo
            # rendezvous, so build an nccl group over the same ranks (collective: every rank constructs FlatDDP here)
            ranks = dist.get_process_group_ranks(process_group) if process_group is not None else None
            self.pg = process_group = dist.new_group(ranks=ranks, backend="nccl")
            self.nccl = True
        self.overlap = (overlap and self.coll) or optimizer is not None
        self.launched = 0
        # Every collective of the trial -- bucket all-reduces, ZeRO-1's reduce-scatter / all-gather, the parameter
        # broadcast -- runs on the process's ONE framework communicator (parallel/comm.py: RCCL on the GPU, the gloo
        # shim on the CPU, so the CPU tests execute this same path).  GPU bucket all-reduces run on a stream of their
        # own, event-ordered after the bucket's gradient: through ProcessGroupNCCL's work objects the GPT-2 step lost
        # 35 % at world 1 to a host / dispatch stall, this way 3.4 % (profiles/r4_gpt2_world1_collectives.md).
        # PLX_DDP_COMM=pg: torch.distributed's own collectives (ProcessGroupNCCL on the GPU, built above; gloo on the
        # CPU) -- the reference path the CPU tests compare the communicator branch with (A/B).
        self._comm = self._comm_stream = None
        if self.coll and not pg_mode:
            from polyaxon_amd.parallel import comm as _comm

            self._comm = _comm.acquire(process_group, flat.device)
            if not self._comm.synchronous and not shard_optimizer:
                self._comm_stream = torch.cuda.Stream(device=flat.device)
        # an average in the collective (RCCL's AVG: a pre-multiplied sum) where the backend has one, else SUM + our
        # own 1/W scale (the gloo shim)
        if self._comm is not None:
            self.avg_supported = bool(self._comm.native_avg)
        else:
            self.avg_supported = self.nccl
        self.plan = None
        if bucket_mb is None or bucket_mb == "auto":
            from polyaxon_amd.parallel.comm_plan import plan as _plan

            elem = 2 if flat.lp_grads is not None else 4  # bytes per gradient element on the wire (bf16 / fp32)
            model = None
            if self.world > 1 and self._comm is not None and not os.environ.get("PLX_COMM_TABLE"):
                # the node's own link, timed on this trial's communicator (same fit on every rank)
                from polyaxon_amd.parallel.comm_plan import calibrate

                model = calibrate(self._comm, self.world, flat.device)
            self.plan = _plan(flat.numel * elem, self.world, model=model)
            bucket_elems = max(1, self.plan["bucket_bytes"] // elem)
        else:
            bucket_elems = max(1, int(float(bucket_mb) * 2 ** 20 / 4))
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
        self.zero = bool(shard_optimizer)
        self.shards: List[tuple] = []           # ZeRO-1, per bucket: (slice length s, reduce-scattered length, state offset)
        if self.zero:
            self.shards, state = self.plan_shards(self.buckets, self.world)
            optimizer.shard_state(state)
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

    @staticmethod
    def plan_shards(buckets, world: int):
        """ZeRO-1 layout: per bucket (slice length s, reduce-scattered length W s, offset of the rank's packed
        state), and the packed state's total length: s + the bucket's sub-4W remainder per bucket."""
        shards, off = [], 0
        for lo, hi, _ in buckets:
            main = ((hi - lo) // (4 * world)) * 4 * world
            shards.append((main // world, main, off))
            off += main // world + (hi - lo - main)
        return shards, off

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

    def _wait_grads(self, stream) -> None:
        """``stream`` waits for the bucket's gradients: the main stream's, and the weight gradients that ops queued on
        the side stream (ops/side_stream.py) before their parameters' hooks fired"""
        stream.wait_stream(torch.cuda.current_stream(self.flat.device))
        side_stream.fence(stream, self.flat.device)

    def _launch(self, b: int) -> None:
        if self.zero:
            self._launch_sharded(b)
            return
        lo, hi, _ = self.buckets[b]
        view = self.flat.grad_view(lo, hi)
        h, div = None, None
        if self._comm is not None:
            self.launched += 1
            op = "avg" if self.avg_supported else "sum"
            if self._comm.synchronous:
                side_stream.join(self.flat.device)  # the bucket's side-stream weight gradients (ops/side_stream.py)
                self._comm.all_reduce(view.data, op=op)
                div = None if self.avg_supported else view
            else:
                self._wait_grads(self._comm_stream)
                with torch.cuda.stream(self._comm_stream):
                    self._comm.all_reduce(view.data, op=op)
                    if not self.avg_supported:
                        view.data.div_(self.world)  # on the collective's stream, before anyone waits on it
                h = _StreamWork(self._comm_stream)
        elif self.coll:
            self.launched += 1
            side_stream.join(self.flat.device)  # the PG collective orders after the current stream only
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
        self._wait_grads(self._side)
        with torch.cuda.stream(self._side):
            if h is not None:
                h.wait()  # the optimizer stream waits for RCCL's stream (host does not block)
            if div is not None:
                div.div_(self.world)
            self.opt.step_range_(lo, hi, self._side.cuda_stream)

    def _launch_sharded(self, b: int) -> None:
        """ZeRO-1 bucket: reduce-scatter (+ all-reduce of the sub-4W remainder) -> AdamW on this rank's slice ->
        all-gather of the updated weights.  GPU: the collectives run on RCCL's streams and the update on the optimizer
        stream, each waiting for the previous one on the device (the host never blocks); CPU: synchronous."""
        f, opt = self.flat, self.opt
        lo, hi, _ = self.buckets[b]
        s, main, so = self.shards[b]
        r, w = self.rank, self.world
        own_lo, own_hi, rem_lo = lo + r * s, lo + (r + 1) * s, lo + main
        coll = self.world > 1 or self.force
        lp = f.lp_params is not None and hi <= f.n_decay
        gv = lambda a, z: f.grad_view(a, z).data  # noqa: E731  (no autograd version bumps inside the backward)
        op = dist.ReduceOp.AVG if self.avg_supported else dist.ReduceOp.SUM
        self.stepped += 1
        cuda = self._side is not None
        if cuda:
            self._wait_grads(self._side)
        ctx = torch.cuda.stream(self._side) if cuda else _nullcontext()
        c = self._comm
        with ctx:
            if coll:
                self.launched += 1
                cop = "avg" if self.avg_supported else "sum"
                if main:
                    out, inp = gv(own_lo, own_hi), gv(lo, rem_lo)
                    if c is not None:  # in place: the output is this rank's slice of the input (NCCL's in-place form)
                        c.reduce_scatter_into(out, inp, op=cop)
                    elif self.nccl:
                        dist.reduce_scatter_tensor(out, inp, op=op, group=self.pg, async_op=True).wait()
                    else:
                        tmp = torch.empty_like(out)
                        dist.reduce_scatter_tensor(tmp, inp, op=op, group=self.pg)
                        out.copy_(tmp)
                    if not self.avg_supported:
                        out.div_(w)
                if rem_lo < hi:
                    rv = gv(rem_lo, hi)
                    if c is not None:
                        c.all_reduce(rv, op=cop)
                    elif cuda:
                        dist.all_reduce(rv, op=op, group=self.pg, async_op=True).wait()
                    else:
                        dist.all_reduce(rv, op=op, group=self.pg)
                    if not self.avg_supported:
                        rv.div_(w)
            st = self._side.cuda_stream if cuda else None
            if main:
                opt.step_range_(own_lo, own_hi, st, state_off=so)
                # the other ranks' slices of the gradient are not read here: zero them for the next accumulation
                if own_lo > lo:
                    gv(lo, own_lo).zero_()
                if rem_lo > own_hi:
                    gv(own_hi, rem_lo).zero_()
            if rem_lo < hi:
                opt.step_range_(rem_lo, hi, st, state_off=so + s)
            if coll and main:
                buf = f.lp_params.data if lp else f.params.data
                full, mine = buf[lo:rem_lo], buf[own_lo:own_hi]
                if c is not None:  # GPU: on the optimizer stream, after the update (finish() joins that stream)
                    c.all_gather_into(full, mine)
                elif self.nccl:  # in place: this rank's slice already sits at its place in the output
                    self._handles.append((dist.all_gather_into_tensor(full, mine, group=self.pg, async_op=True), None))
                else:
                    dist.all_gather_into_tensor(full, mine.clone(), group=self.pg)

    def gather_master(self) -> None:
        """ZeRO-1 in lp mode: refresh the fp32 master of the slices other ranks own (all-gather per bucket), e.g.
        before a checkpoint; the bf16 model weights are always current."""
        if not self.zero or not self.coll:
            return
        f = self.flat
        for (lo, hi, _), (s, main, _) in zip(self.buckets, self.shards):
            if main and f.lp_params is not None and hi <= f.n_decay:
                own = f.params.data[lo + self.rank * s: lo + (self.rank + 1) * s]
                if self._comm is not None:
                    self._comm.all_gather_into(f.params.data[lo:lo + main], own)
                else:
                    dist.all_gather_into_tensor(f.params.data[lo:lo + main], own if self.nccl else own.clone(),
                                                group=self.pg)

    def finish(self) -> None:
        """Call after backward(): launches any bucket not fired by hooks, waits, averages (and, with an optimizer
        in the backward, has the main stream wait for every bucket's update)."""
        if not self.coll and self.opt is None:
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
        if not self.coll:
            return
        if self._comm is not None:
            self._comm.broadcast(self.flat.params.data, root=src)
        else:
            dist.broadcast(self.flat.params, src=src, group=self.pg)
        self.flat.sync_lp()

    def close(self) -> None:
        """Drop this FlatDDP's hold on the process's framework communicator (the last holder closes it)."""
        if self._comm is not None:
            from polyaxon_amd.parallel import comm as _comm

            if self._comm_stream is not None:
                self._comm_stream.synchronize()
            _comm.release(self._comm)
            self._comm = None

    def remove_hooks(self) -> None:
        for h in self._hooks:
            h.remove()
        self._hooks = []
        if self.opt is not None:  # the optimizer steps on its own again (it silently skipped updates)
            self.opt.in_backward = False
