"""One framework communicator per process and group: RCCL on the GPU, a gloo shim with the same interface on the CPU.

A data-parallel trial used to hold three RCCL communicators (ProcessGroupNCCL's, FlatDDP's bucket communicator and
the metric reducer's), each with its own streams; on a 4-queue box their streams pushed the weight-gradient side
stream onto the compute stream's hardware queue (profiles/r4_rccl_slowdown.md).  Now the process group is only the
rendezvous -- gloo, which exchanges the RCCL unique id and carries the host-side control traffic -- and every device
collective of a trial (FlatDDP's bucket all-reduces, ZeRO-1's reduce-scatter / all-gather, the parameter broadcast,
the metric mean, the bench's per-rank gather) goes through :func:`acquire`'s shared communicator:

    comm = acquire(group, device)     # RcclComm (csrc/rccl_comm.cpp) for a cuda device, GlooComm for the CPU
    comm.all_reduce(t, op="avg")      # in place, on the current HIP stream (GPU) / synchronously (CPU)
    release(comm)                     # the last holder closes it

:class:`GlooComm` exists so the CPU tests (gloo, world 2 / 4) run the SAME FlatDDP code path the GPU ranks run:
FlatDDP and the metric reducer no longer branch on the backend, only on ``comm.synchronous``.  Reference: the
reference spawns one pod per rank and leaves the collectives to the user's framework
(/root/reference/polyaxon/scheduler/spawners/pytorch_spawner.py:12-25, experiment_scheduler.py:225-271).
"""
from __future__ import annotations

import threading
from typing import Dict, Optional, Tuple

import torch
import torch.distributed as dist

_OPS = {"sum": dist.ReduceOp.SUM, "max": dist.ReduceOp.MAX, "min": dist.ReduceOp.MIN, "prod": dist.ReduceOp.PRODUCT}


def group_rank0(group=None) -> int:
    """Global rank of the group's rank 0 (the source of a broadcast over a subgroup)."""
    if group is None or group is dist.group.WORLD:
        return 0
    return dist.get_global_rank(group, 0)


class GlooComm:
    """The RcclComm interface over a torch.distributed gloo group, on CPU tensors.  Every call completes before it
    returns (``synchronous``).  ``avg`` is a sum followed by a division by the world size, which is what the GPU
    path's RCCL average computes up to rounding (the CPU tests compare CPU runs with CPU runs)."""

    synchronous = True
    native_avg = False

    def __init__(self, group=None):
        self.group = group
        self.nranks = dist.get_world_size(group)
        self.rank = dist.get_rank(group)
        self.h = True

    def _op(self, op: str):
        if op == "avg":
            return dist.ReduceOp.SUM
        return _OPS[op]

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        dist.all_reduce(t, op=self._op(op), group=self.group)
        if op == "avg":
            t.div_(self.nranks)
        return t

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """``out`` (numel n) = this rank's n-slice of the reduction of ``inp`` (numel n * W); ``out`` may alias that
        slice of ``inp`` (the in-place form)."""
        tmp = torch.empty_like(out)
        dist.reduce_scatter_tensor(tmp, inp, op=self._op(op), group=self.group)
        out.copy_(tmp)
        if op == "avg":
            out.div_(self.nranks)
        return out

    def all_gather_into(self, full: torch.Tensor, mine: torch.Tensor) -> torch.Tensor:
        """``full`` (numel n * W) = every rank's ``mine`` (numel n) in rank order; ``mine`` may alias this rank's slice
        of ``full``."""
        dist.all_gather_into_tensor(full, mine.clone(), group=self.group)
        return full

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.nranks, *t.shape), dtype=t.dtype, device=t.device)
        self.all_gather_into(out.view(-1), t.reshape(-1))
        return out

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        src = root if self.group is None else dist.get_global_rank(self.group, root)
        dist.broadcast(t, src=src, group=self.group)
        return t

    def close(self) -> None:
        self.h = None


_lock = threading.Lock()
_comms: Dict[Tuple, list] = {}   # key -> [comm, holders]


def _key(group, device: torch.device) -> Tuple:
    return (id(group) if group is not None else None, device.type, device.index)


def acquire(group=None, device: Optional[torch.device] = None):
    """The process's communicator for ``group`` on ``device`` (created on first use: collective over the group, so
    every rank of it must call this at the same program point).  cuda: the RCCL communicator, its unique id shipped
    over ``group`` (gloo, the rendezvous); cpu: :class:`GlooComm`."""
    device = torch.device(device) if device is not None else torch.device("cpu")
    if device.type == "cuda" and device.index is None:
        device = torch.device("cuda", torch.cuda.current_device())
    k = _key(group, device)
    with _lock:
        e = _comms.get(k)
        if e is not None:
            e[1] += 1
            return e[0]
    if device.type == "cuda":
        from polyaxon_amd.parallel.rccl import RcclComm

        comm = RcclComm.from_torch_distributed(group, device=device)
    else:
        comm = GlooComm(group)
    with _lock:
        e = _comms.get(k)
        if e is not None:  # another thread of this process won the race (not a collective-safe pattern; be exact)
            comm.close()
            e[1] += 1
            return e[0]
        _comms[k] = [comm, 1]
    return comm


def release(comm) -> None:
    """Drop one holder; the last one closes the communicator."""
    if comm is None:
        return
    with _lock:
        for k, e in list(_comms.items()):
            if e[0] is comm:
                e[1] -= 1
                if e[1] > 0:
                    return
                del _comms[k]
                break
    comm.close()


def live() -> int:
    """Number of shared communicators this process holds (tests: one per DP trial)."""
    with _lock:
        return len(_comms)
