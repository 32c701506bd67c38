"""Python face of the framework RCCL communicator (csrc/rccl_comm.cpp) + an xGMI bandwidth probe.

    comm = RcclComm.from_torch_distributed()          # id shipped over the process group (the gloo rendezvous)
    comm.all_reduce(t)                                  # in place, on the current HIP stream
    python -m torch.distributed.run --nproc-per-node 8 -m polyaxon_amd.parallel.rccl   # busbw table

The bandwidth table is the rccl-tests ``all_reduce_perf`` equivalent that SURVEY.md §6 names as the
hardware ceiling for the Llama-3 8B DP=8 config (xGMI: 7 links × ~153 GB/s per MI355X).
"""
from __future__ import annotations

import ctypes
import json
import os
from typing import List

import torch

from polyaxon_amd.ops import _native

DTYPES = {torch.float32: 0, torch.bfloat16: 1, torch.float16: 2, torch.float64: 3, torch.int32: 4}
OPS = {"sum": 0, "prod": 1, "max": 2, "min": 3, "avg": 4}


class RcclError(RuntimeError):
    pass


TIMEOUT = 1000  # plx_rccl status: the watchdog aborted the communicator on its deadline (csrc/rccl_comm.cpp)


def _env_seconds(name: str, default: float) -> float:
    try:
        return float(os.environ.get(name, "") or default)
    except ValueError:
        return default


class RcclComm:
    """One RCCL communicator, created non-blocking and watched (csrc/rccl_comm.cpp).

    ``init_timeout_s``: every rank must join within it, else RcclError (default PLX_RCCL_INIT_TIMEOUT_S, else
    PLX_COLLECTIVE_TIMEOUT_S, else 600 s).  ``timeout_s``: a collective not complete that long after it was enqueued
    makes the process's watchdog thread abort the communicator -- RCCL's kernels in flight exit, and every later call
    raises RcclError, so the rank fails and polyflow tears its gang down (default PLX_COLLECTIVE_TIMEOUT_S, which
    polyflow sets for multi-rank trials, polyflow/env.py; 0 = no deadline, asynchronous RCCL errors still abort).
    Reference behaviour: the reference stops every job of an experiment when one fails
    (/root/reference/polyaxon/signals/experiments.py:252-281)."""

    synchronous = False  # collectives are enqueued on the current HIP stream
    native_avg = True  # RCCL's AVG (a pre-multiplied sum) rather than SUM + the caller's 1/W scale

    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int, timeout_s: float = None,
                 init_timeout_s: float = None):
        self.lib = _native.lib("plx_rccl")
        coll = _env_seconds("PLX_COLLECTIVE_TIMEOUT_S", 0.0) if timeout_s is None else float(timeout_s)
        if init_timeout_s is None:
            init_timeout_s = _env_seconds("PLX_RCCL_INIT_TIMEOUT_S", coll if coll > 0 else 600.0)
        err = ctypes.c_int(0)
        self.h = self.lib.plx_rccl_init(unique_id, nranks, rank, device, int(init_timeout_s * 1000), int(coll * 1000),
                                        ctypes.byref(err))
        if not self.h:
            raise RcclError(f"RCCL communicator init (rank {rank} of {nranks}) failed: "
                            f"{self.lib.plx_rccl_error(err.value).decode()}")
        self.nranks, self.rank, self.device = nranks, rank, device
        self.timeout_s = coll

    @staticmethod
    def new_unique_id() -> bytes:
        lib = _native.lib("plx_rccl")
        buf = ctypes.create_string_buffer(128)
        rc = lib.plx_rccl_unique_id(buf)
        if rc != 0:
            raise RcclError(f"ncclGetUniqueId failed: {rc}")
        return buf.raw

    @classmethod
    def from_torch_distributed(cls, group=None, device=None) -> "RcclComm":
        """Rank 0 of ``group`` creates the unique id and ships it over the group (gloo or nccl: any backend that
        carries Python objects); ``device`` defaults to the current one."""
        import torch.distributed as dist

        from polyaxon_amd.parallel.comm import group_rank0

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj: List = [cls.new_unique_id() if rank == 0 else None]
        # src is a GLOBAL rank: the group's rank 0 (a subgroup without global rank 0 hung or errored with src=0)
        dist.broadcast_object_list(obj, src=group_rank0(group), group=group)
        idx = torch.device(device).index if device is not None else None
        return cls(obj[0], world, rank, torch.cuda.current_device() if idx is None else idx)

    def _check(self, rc: int, what: str) -> None:
        if not self.h:
            raise RcclError(f"{what}: communicator is closed")
        if rc != 0:
            raise RcclError(f"{what}: {self.lib.plx_rccl_error(rc).decode()}")

    def status(self) -> int:
        """0 while healthy, else the error code that aborted the communicator (:data:`TIMEOUT`: the watchdog)."""
        return int(self.lib.plx_rccl_status(self.h)) if self.h else 0

    def check(self) -> None:
        """Raise RcclError if the watchdog (or an asynchronous RCCL error) aborted the communicator."""
        self._check(self.status(), "communicator")

    def pending(self) -> int:
        """Collectives enqueued and not yet seen complete by the watchdog."""
        return int(self.lib.plx_rccl_pending(self.h)) if self.h else 0

    def set_timeout(self, seconds: float) -> None:
        self._check(self.lib.plx_rccl_set_timeout(self.h, int(seconds * 1000)), "set_timeout")
        self.timeout_s = float(seconds)

    def abort(self) -> None:
        """Abort now (in-flight RCCL kernels exit; later calls raise)."""
        if self.h:
            self.lib.plx_rccl_abort(self.h)

    @staticmethod
    def _stream() -> int:
        return torch.cuda.current_stream().cuda_stream

    def all_reduce(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        self._check(self.lib.plx_rccl_all_reduce(self.h, t.data_ptr(), t.data_ptr(), t.numel(), DTYPES[t.dtype],
                                                 OPS[op], self._stream()), "all_reduce")
        return t

    def all_gather(self, t: torch.Tensor) -> torch.Tensor:
        out = torch.empty((self.nranks, *t.shape), dtype=t.dtype, device=t.device)
        self._check(self.lib.plx_rccl_all_gather(self.h, t.data_ptr(), out.data_ptr(), t.numel(), DTYPES[t.dtype],
                                                 self._stream()), "all_gather")
        return out

    def reduce_scatter(self, t: torch.Tensor, op: str = "sum") -> torch.Tensor:
        if t.numel() % self.nranks:
            raise ValueError("reduce_scatter needs numel divisible by the world size")
        out = torch.empty(t.numel() // self.nranks, dtype=t.dtype, device=t.device)
        self._check(self.lib.plx_rccl_reduce_scatter(self.h, t.data_ptr(), out.data_ptr(), out.numel(),
                                                     DTYPES[t.dtype], OPS[op], self._stream()), "reduce_scatter")
        return out

    def reduce_scatter_into(self, out: torch.Tensor, inp: torch.Tensor, op: str = "sum") -> torch.Tensor:
        """``out`` (numel n) = this rank's n-slice of the reduction of ``inp`` (numel n * W); in place when ``out`` is
        that slice of ``inp`` (NCCL's in-place form)."""
        if inp.numel() != out.numel() * self.nranks:
            raise ValueError("reduce_scatter_into: input numel must be W x output numel")
        self._check(self.lib.plx_rccl_reduce_scatter(self.h, inp.data_ptr(), out.data_ptr(), out.numel(),
                                                     DTYPES[out.dtype], OPS[op], self._stream()), "reduce_scatter")
        return out

    def all_gather_into(self, full: torch.Tensor, mine: torch.Tensor) -> torch.Tensor:
        """``full`` (numel n * W) = every rank's ``mine`` (numel n) in rank order; in place when ``mine`` is this rank's
        slice of ``full``."""
        if full.numel() != mine.numel() * self.nranks:
            raise ValueError("all_gather_into: output numel must be W x input numel")
        self._check(self.lib.plx_rccl_all_gather(self.h, mine.data_ptr(), full.data_ptr(), mine.numel(),
                                                 DTYPES[mine.dtype], self._stream()), "all_gather")
        return full

    def broadcast(self, t: torch.Tensor, root: int = 0) -> torch.Tensor:
        self._check(self.lib.plx_rccl_broadcast(self.h, t.data_ptr(), t.data_ptr(), t.numel(), DTYPES[t.dtype], root,
                                                self._stream()), "broadcast")
        return t

    def bus_bandwidth(self, nbytes: int, iters: int = 20):
        buf = torch.ones(nbytes // 4, dtype=torch.float32, device=f"cuda:{self.device}")
        alg, bus = ctypes.c_double(0), ctypes.c_double(0)
        self._check(self.lib.plx_rccl_bus_bw(self.h, buf.data_ptr(), buf.numel() * 4, iters, self._stream(),
                                             ctypes.byref(alg), ctypes.byref(bus)), "bus_bw")
        return alg.value, bus.value

    def close(self) -> None:
        if self.h:
            self.lib.plx_rccl_destroy(self.h)
            self.h = None


def main() -> None:
    import torch.distributed as dist

    from polyaxon_amd.parallel.ddp import init_from_env

    info = init_from_env("gloo", device=torch.device("cuda", int(os.environ.get("LOCAL_RANK", "0"))))
    comm = RcclComm.from_torch_distributed(device=info["device"])
    x = torch.full((1024,), float(info["rank"] + 1), device=info["device"])
    comm.all_reduce(x)
    torch.cuda.synchronize()
    expect = info["world"] * (info["world"] + 1) / 2
    assert float(x[0]) == expect, (float(x[0]), expect)
    rows = []
    for mb in (1, 8, 64, 256, 1024):
        alg, bus = comm.bus_bandwidth(mb * 2 ** 20)
        rows.append({"bytes": mb * 2 ** 20, "algbw_GBps": round(alg, 1), "busbw_GBps": round(bus, 1)})
    if info["rank"] == 0:
        print(json.dumps({"world": info["world"], "all_reduce": rows}))
    comm.close()
    dist.destroy_process_group()


if __name__ == "__main__":
    main()
