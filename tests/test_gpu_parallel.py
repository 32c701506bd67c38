"""Multi-GPU readiness proven on one MI355X: the framework RCCL communicator (csrc/rccl_comm.cpp) at nranks = 1
and FlatDDP on the nccl (RCCL) backend at world 1, in a child process (RCCL/process-group state stays out of the
pytest process)."""
import json
import os
import socket
import subprocess
import sys
import textwrap

import pytest

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(code: str, timeout: int = 180) -> dict:
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    # prepend (never overwrite) PYTHONPATH: the driver's native-load hook rides on it and must see the child's .so
    pp = os.environ.get("PYTHONPATH")
    env = dict(os.environ, MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK="0", WORLD_SIZE="1", LOCAL_RANK="0",
               PYTHONPATH=ROOT + (os.pathsep + pp if pp else ""))
    out = subprocess.run([sys.executable, "-c", textwrap.dedent(code)], capture_output=True, text=True,
                         timeout=timeout, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-4000:]
    return json.loads([l for l in out.stdout.splitlines() if l.startswith("{")][-1])


def test_rccl_comm_single_rank_collectives():
    res = _run("""
        import json, torch
        from polyaxon_amd.parallel.rccl import RcclComm
        from polyaxon_amd.ops import _native
        torch.cuda.set_device(0)
        comm = RcclComm(RcclComm.new_unique_id(), 1, 0, 0)
        x = torch.arange(1024, dtype=torch.float32, device="cuda")
        comm.all_reduce(x)
        g = comm.all_gather(torch.full((8,), 3.0, device="cuda"))
        rs = comm.reduce_scatter(torch.ones(16, device="cuda"))
        b = comm.broadcast(torch.full((4,), 7.0, dtype=torch.bfloat16, device="cuda"))
        mx = comm.all_reduce(torch.tensor([5.0], device="cuda"), op="max")
        torch.cuda.synchronize()
        alg, bus = comm.bus_bandwidth(64 << 20, iters=5)
        raw = comm.h
        comm.close()
        import ctypes
        from polyaxon_amd.parallel.rccl import RcclError
        try:  # the Python face refuses a closed communicator
            comm.bus_bandwidth(1 << 20, iters=1)
            closed_raises = False
        except RcclError:
            closed_raises = True
        # the C++ probe itself refuses the destroyed handle (live-communicator registry), reporting no bandwidth
        buf = torch.ones(1 << 18, device="cuda")
        a2, b2 = ctypes.c_double(-1), ctypes.c_double(-1)
        rc_dead = comm.lib.plx_rccl_bus_bw(raw, buf.data_ptr(), buf.numel() * 4, 1,
                                           torch.cuda.current_stream().cuda_stream, ctypes.byref(a2), ctypes.byref(b2))
        print(json.dumps({"closed_raises": closed_raises, "rc_dead": rc_dead, "alg_dead": a2.value,
                          "ar_dead": comm.lib.plx_rccl_all_reduce(raw, buf.data_ptr(), buf.data_ptr(), 4, 0, 0,
                                                                  torch.cuda.current_stream().cuda_stream),
                          "sum_ok": bool(torch.equal(x, torch.arange(1024, dtype=torch.float32, device="cuda"))),
                          "gather": g.shape[0], "gather_ok": bool((g == 3).all()), "rs": rs.numel(),
                          "rs_ok": bool((rs == 1).all()), "bcast_ok": bool((b.float() == 7).all()),
                          "max": float(mx[0]), "algbw": alg, "busbw": bus,
                          "loaded": "plx_rccl" in _native._loaded}))
    """)
    assert res["sum_ok"] and res["gather"] == 1 and res["gather_ok"] and res["rs"] == 16 and res["rs_ok"]
    assert res["bcast_ok"] and res["max"] == 5.0 and res["loaded"]
    assert res["algbw"] > 0
    assert res["closed_raises"] and res["rc_dead"] != 0 and res["alg_dead"] == 0.0 and res["ar_dead"] != 0


def test_flat_ddp_on_rccl_backend_world1():
    """force_collectives: every bucket's RCCL all-reduce (AVG) really runs through the post-accumulate hooks at
    world 1, and the averaged gradient equals the single-process one; the metric reducer's RCCL communicator
    (csrc/rccl_comm.cpp) averages a loss in the same process."""
    res = _run("""
        import json, torch
        import torch.distributed as dist
        from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
        from polyaxon_amd.ops.flat import FlatParams
        from polyaxon_amd.ops import _native
        from polyaxon_amd.parallel.ddp import FlatDDP, MetricReducer, init_from_env
        import os
        os.environ["WORLD_SIZE"] = "1"
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        info = init_from_env("nccl")
        torch.manual_seed(0)
        m = Transformer(tiny_llama()).cuda()
        flat = FlatParams(m, info["device"], channels_last=False)
        ddp = FlatDDP(flat, bucket_mb=0.01, force_collectives=True)
        ddp.broadcast_params()
        tok = torch.randint(0, 256, (4, 16), device="cuda")
        loss = lm_loss(m(tok), tok)
        loss.backward()
        ddp.finish()
        red = MetricReducer(info["device"], force_comm=True)
        lm = red.mean(loss)
        torch.cuda.synchronize()
        g = flat.grads.clone()
        # the same step without DDP
        torch.manual_seed(0)
        m2 = Transformer(tiny_llama()).cuda()
        f2 = FlatParams(m2, info["device"], channels_last=False)
        lm_loss(m2(tok), tok).backward()
        print(json.dumps({"backend": dist.get_backend(), "buckets": len(ddp.buckets), "launched": ddp.launched,
                          "err": float((g - f2.grads).abs().max()), "norm": float(g.norm()),
                          "loss": float(loss), "loss_mean": float(lm[0]), "rccl": red.comm is not None,
                          "loaded": "plx_rccl" in _native._loaded}))
        red.close()
        dist.destroy_process_group()
    """)
    assert res["backend"] == "nccl" and res["buckets"] > 1 and res["launched"] == res["buckets"]
    assert res["norm"] > 0 and res["err"] < 1e-5
    assert res["rccl"] and res["loaded"] and abs(res["loss_mean"] - res["loss"]) < 1e-6


def test_flat_ddp_bucket_all_reduce_on_the_framework_communicator():
    """PLX_DDP_COMM=rccl: the bucket all-reduces run on csrc/rccl_comm.cpp's communicator on their own stream
    (event-ordered) instead of ProcessGroupNCCL; at world 1 the averaged gradient equals the single-process one."""
    res = _run("""
        import json, os, torch
        os.environ["PLX_DDP_COMM"] = "rccl"
        os.environ["WORLD_SIZE"] = "1"
        import torch.distributed as dist
        from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
        from polyaxon_amd.ops.flat import FlatParams
        from polyaxon_amd.ops import _native
        from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        info = init_from_env("nccl")
        torch.manual_seed(0)
        m = Transformer(tiny_llama()).cuda()
        flat = FlatParams(m, info["device"], channels_last=False)
        ddp = FlatDDP(flat, bucket_mb=0.01, force_collectives=True)
        tok = torch.randint(0, 256, (4, 16), device="cuda")
        lm_loss(m(tok), tok).backward()
        ddp.finish()
        torch.cuda.synchronize()
        g = flat.grads.clone()
        torch.manual_seed(0)
        m2 = Transformer(tiny_llama()).cuda()
        f2 = FlatParams(m2, info["device"], channels_last=False)
        lm_loss(m2(tok), tok).backward()
        print(json.dumps({"own_comm": ddp._comm is not None, "buckets": len(ddp.buckets), "launched": ddp.launched,
                          "err": float((g - f2.grads).abs().max()), "norm": float(g.norm()),
                          "loaded": "plx_rccl" in _native._loaded}))
        ddp.close()
        dist.destroy_process_group()
    """)
    assert res["own_comm"] and res["loaded"] and res["buckets"] > 1 and res["launched"] == res["buckets"]
    assert res["norm"] > 0 and res["err"] < 1e-5


def test_zero1_on_rccl_backend_world1_matches_unsharded():
    """ZeRO-1 at world 1 with force_collectives on the nccl (RCCL) backend: every bucket runs the in-place
    reduce-scatter, the AdamW update of its slice on the optimizer stream and the in-place all-gather of the bf16
    weights, and three steps of the tiny Llama in lp mode (bf16 weights, direct GEMM gradients) follow the unsharded
    in-backward trajectory bitwise."""
    res = _run("""
        import json, torch
        import torch.distributed as dist
        from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
        from polyaxon_amd.ops.flat import FlatParams
        from polyaxon_amd.ops.optim import FusedAdamW
        from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env
        import os
        os.environ["WORLD_SIZE"] = "1"
        dist.init_process_group("nccl", rank=0, world_size=1, device_id=torch.device("cuda", 0))
        info = init_from_env("nccl")
        out = {}
        for zero in (False, True):
            torch.manual_seed(0)
            m = Transformer(tiny_llama()).cuda()
            flat = FlatParams(m, info["device"], channels_last=False, lp_dtype=torch.bfloat16)
            flat.enable_direct_grads(True)
            opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1)
            ddp = FlatDDP(flat, bucket_mb=0.01, force_collectives=True, optimizer=opt, shard_optimizer=zero)
            gen = torch.Generator(device="cuda").manual_seed(5)
            losses = []
            for _ in range(3):
                tok = torch.randint(0, 256, (4, 16), device="cuda", generator=gen)
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = lm_loss(m(tok), tok)
                loss.backward()
                ddp.finish()
                opt.step_()
                opt.step += 1
                losses.append(float(loss))
            ddp.gather_master()
            torch.cuda.synchronize()
            out[zero] = (losses, flat.params.clone(), flat.lp_params.clone(), ddp.launched, len(ddp.buckets),
                         opt.exp_avg.numel(), flat.numel)
            ddp.remove_hooks()
        a, b = out[False], out[True]
        print(json.dumps({"losses_equal": a[0] == b[0], "master_equal": bool(torch.equal(a[1], b[1])),
                          "lp_equal": bool(torch.equal(a[2], b[2])), "launched": b[3], "buckets": b[4],
                          "state": b[5], "numel": b[6], "losses": b[0]}))
        dist.destroy_process_group()
    """)
    assert res["losses_equal"] and res["master_equal"] and res["lp_equal"], res
    assert res["buckets"] > 1 and res["launched"] == 3 * res["buckets"]
    assert res["state"] == res["numel"]  # world 1: the slice is the whole bucket


def test_rccl_init_with_a_peer_that_never_joins_fails_within_the_deadline():
    """SURVEY.md §5.3 watchdog: a 2-rank communicator whose peer never calls init raises RcclError after the init
    deadline (non-blocking ncclCommInitRankConfig polled, then ncclCommAbort) instead of blocking the rank forever."""
    res = _run("""
        import json, time, torch
        from polyaxon_amd.parallel.rccl import RcclComm, RcclError
        torch.cuda.set_device(0)
        uid = RcclComm.new_unique_id()
        t0 = time.monotonic()
        out = {"raised": False}
        try:
            RcclComm(uid, 2, 0, 0, timeout_s=5, init_timeout_s=4)
        except RcclError as e:
            out = {"raised": True, "msg": str(e)}
        out["elapsed"] = time.monotonic() - t0
        print(json.dumps(out))
    """, timeout=120)
    assert res["raised"] and "timed out" in res["msg"], res
    assert 3.5 <= res["elapsed"] < 40, res


def test_rccl_watchdog_aborts_a_collective_that_does_not_complete():
    """The progress half of the watchdog: an all-reduce queued behind a 3 s kernel is still incomplete after the
    communicator's 1 s deadline, so the watchdog aborts the communicator; the stream still drains and the NEXT call
    raises RcclError.  With no deadline hit, completed collectives are retired (pending drains to 0)."""
    res = _run("""
        import json, time, torch
        from polyaxon_amd.parallel.rccl import RcclComm, RcclError, TIMEOUT
        torch.cuda.set_device(0)
        comm = RcclComm(RcclComm.new_unique_id(), 1, 0, 0, timeout_s=30)
        x = torch.ones(1024, device="cuda")
        for _ in range(8):
            comm.all_reduce(x)
        torch.cuda.synchronize()
        t0 = time.monotonic()
        while comm.pending() and time.monotonic() - t0 < 5:
            time.sleep(0.02)
        out = {"drained": comm.pending(), "ok_status": comm.status(), "x": float(x[0])}
        comm.set_timeout(1.0)
        # ~3 s of GPU spin ahead of the collective (clock cycles at ~100 MHz for s_memrealtime-based sleep is not
        # portable: calibrate by timing a short sleep first)
        torch.cuda._sleep(1000000)
        torch.cuda.synchronize()
        t = time.monotonic()
        torch.cuda._sleep(1000000)
        torch.cuda.synchronize()
        per = max(time.monotonic() - t, 1e-4) / 1000000
        torch.cuda._sleep(int(3.0 / per))
        comm.all_reduce(x)
        torch.cuda.synchronize()
        out["spin_s"] = time.monotonic() - t
        out["status"] = comm.status()
        try:
            comm.all_reduce(x)
            out["raised"] = False
        except RcclError as e:
            out["raised"], out["msg"] = True, str(e)
        out["timeout_code"] = TIMEOUT
        print(json.dumps(out))
    """, timeout=120)
    assert res["drained"] == 0 and res["ok_status"] == 0 and res["x"] == 1.0, res
    assert res["spin_s"] > 1.5, res
    assert res["status"] == res["timeout_code"] and res["raised"] and "timed out" in res["msg"], res
