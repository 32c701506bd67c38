"""Python face of the framework RCCL communicator (csrc/rccl_comm.cpp) + an xGMI bandwidth probe.

    comm = RcclComm.from_torch_distributed()          # id shipped over the existing process group
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


class RcclComm:
    def __init__(self, unique_id: bytes, nranks: int, rank: int, device: int):
        self.lib = _native.lib("plx_rccl")
        err = ctypes.c_int(0)
        self.h = self.lib.plx_rccl_init(unique_id, nranks, rank, device, ctypes.byref(err))
        if not self.h:
            raise RcclError(f"ncclCommInitRank failed: {err.value}")
        self.nranks, self.rank, self.device = nranks, rank, device

    @staticmethod
    def new_unique_id() -> bytes:
        lib = _native.lib("plx_rccl")
        buf = ctypes.create_string_buffer(128)
        rc = lib.plx_rccl_unique_id(buf)
        if rc != 0:
            raise RcclError(f"ncclGetUniqueId failed: {rc}")
        return buf.raw

    @classmethod
    def from_torch_distributed(cls, group=None) -> "RcclComm":
        import torch.distributed as dist

        rank, world = dist.get_rank(group), dist.get_world_size(group)
        obj: List = [cls.new_unique_id() if rank == 0 else None]
        dist.broadcast_object_list(obj, src=0, group=group)
        return cls(obj[0], world, rank, torch.cuda.current_device())

    def _check(self, rc: int, what: str) -> None:
        if not self.h:
            raise RcclError(f"{what}: communicator is closed")
        if rc != 0:
            raise RcclError(f"{what}: {self.lib.plx_rccl_error(rc).decode()}")

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

    info = init_from_env("nccl")
    comm = RcclComm.from_torch_distributed()
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
