"""One framework communicator per DP trial (parallel/comm.py): the gloo shim with RcclComm's interface runs the same
FlatDDP / MetricReducer code path the GPU ranks run, on CPU ranks (gloo, world 2 / 4)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _run(target, world, *args, timeout=300):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=target, args=(r, world, port, q) + args) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=timeout) for _ in procs), key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs), [p.exitcode for p in procs]
    return res


def _train(world, zero, lp, pg: bool):
    """3 AdamW steps of the tiny Llama under FlatDDP (buckets / ZeRO-1) + the metric mean; returns the trajectory and
    how many framework communicators the process held while training."""
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel import comm
    from polyaxon_amd.parallel.ddp import FlatDDP, MetricReducer

    rank = int(os.environ["RANK"])
    os.environ["PLX_DDP_COMM"] = "pg" if pg else "comm"
    torch.manual_seed(0)
    model = Transformer(tiny_llama())
    flat = FlatParams(model, "cpu", channels_last=False, lp_dtype=lp)
    opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1)
    in_bwd = zero or lp is not None
    ddp = FlatDDP(flat, bucket_mb=0.01, optimizer=opt if in_bwd else None, shard_optimizer=zero)
    red = MetricReducer(torch.device("cpu"))
    live = comm.live()
    # rank 1 starts from other weights: the broadcast must overwrite them
    if rank:
        with torch.no_grad():
            flat.params.add_(1.0)
        flat.sync_lp()
    ddp.broadcast_params()
    gen = torch.Generator().manual_seed(100 + rank)
    losses, means = [], []
    for _ in range(3):
        tok = torch.randint(0, 256, (4, 16), generator=gen)
        loss = lm_loss(model(tok), torch.randint(0, 256, (4, 16), generator=gen))
        loss.backward()
        ddp.finish()
        opt.step_()
        opt.step += 1
        losses.append(float(loss))
        means.append(float(red.mean(loss.detach())[0]))
    ddp.gather_master()
    params = flat.params.detach().clone()
    uses_comm = ddp._comm is not None
    launched = ddp.launched
    ddp.remove_hooks()
    ddp.close()
    red.close()
    return {"losses": losses, "means": means, "params": params, "live": live, "after": comm.live(),
            "uses_comm": uses_comm, "launched": launched, "buckets": len(ddp.buckets)}


def _parity_worker(rank, world, port, q, zero, lp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.parallel.ddp import init_from_env

    torch.set_num_threads(2)
    init_from_env("gloo")
    a = _train(world, zero, lp, pg=False)
    b = _train(world, zero, lp, pg=True)
    gathered = [torch.zeros_like(a["params"]) for _ in range(world)]
    dist.all_gather(gathered, a["params"])
    q.put({"rank": rank, "comm": a["uses_comm"], "pg": not b["uses_comm"], "live": a["live"], "after": a["after"],
           "losses_equal": a["losses"] == b["losses"], "params_equal": bool(torch.equal(a["params"], b["params"])),
           "means_equal": a["means"] == b["means"], "mean0": a["means"][0],
           "loss0": a["losses"][0], "ranks_equal": all(torch.equal(gathered[0], x) for x in gathered),
           "launched": a["launched"], "buckets": a["buckets"]})
    dist.destroy_process_group()


@pytest.mark.parametrize("world,zero,lp", [(2, False, None), (2, True, None), (2, True, torch.bfloat16),
                                           (4, True, None), (4, False, torch.bfloat16)])
def test_framework_comm_path_matches_process_group_path(world, zero, lp):
    """FlatDDP's default path -- every bucket all-reduce, ZeRO-1 reduce-scatter / all-gather, the parameter broadcast
    and the metric mean on ONE framework communicator (the gloo shim here, RCCL on the GPU) -- follows the
    PLX_DDP_COMM=pg (torch.distributed) trajectory bitwise, with the ranks identical and exactly one communicator
    alive per process while training (none after close)."""
    res = _run(_parity_worker, world, zero, lp)
    for r in res:
        assert r["comm"] and r["pg"], r
        assert r["live"] == 1 and r["after"] == 0, r
        assert r["losses_equal"] and r["params_equal"] and r["means_equal"] and r["ranks_equal"], r
        assert r["launched"] == 3 * r["buckets"], r
    mean = sum(r["loss0"] for r in res) / world
    assert all(abs(r["mean0"] - mean) < 1e-5 for r in res)
    assert len({r["loss0"] for r in res}) > 1  # the ranks saw different data


def _subgroup_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    import torch.distributed as dist

    from polyaxon_amd.parallel import comm

    dist.init_process_group("gloo", rank=rank, world_size=world)
    sub = dist.new_group([1, 2])  # a subgroup without global rank 0
    out = {"rank": rank}
    if rank in (1, 2):
        c = comm.acquire(sub, torch.device("cpu"))
        t = torch.full((3,), float(rank))
        c.broadcast(t, root=0)  # group rank 0 = global rank 1
        out["bcast"] = t.tolist()
        out["src"] = comm.group_rank0(sub)
        x = torch.full((4,), float(rank))
        c.all_reduce(x, op="avg")
        out["avg"] = x.tolist()
        full = torch.zeros(4)
        c.all_gather_into(full, torch.full((2,), float(rank)))
        out["gather"] = full.tolist()
        comm.release(c)
    out["live"] = comm.live()
    q.put(out)
    dist.destroy_process_group()


def test_group_collectives_use_the_groups_own_rank0():
    """Collectives over a subgroup that does not contain global rank 0 (the RCCL unique-id broadcast's source is the
    group's rank 0 as a GLOBAL rank: src=0 hung or errored there)."""
    res = _run(_subgroup_worker, 3)
    for r in res[1:]:
        assert r["src"] == 1 and r["bcast"] == [1.0] * 3, r
        assert r["avg"] == [1.5] * 4 and r["gather"] == [1.0, 1.0, 2.0, 2.0], r
    assert all(r["live"] == 0 for r in res)


def _calib_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.models.transformer import Transformer, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env

    torch.set_num_threads(2)
    init_from_env("gloo")
    flat = FlatParams(Transformer(tiny_llama()), "cpu", channels_last=False)
    ddp = FlatDDP(flat, bucket_mb="auto")
    q.put({"rank": rank, "plan": ddp.plan, "buckets": ddp.buckets})
    ddp.remove_hooks()
    ddp.close()
    dist.destroy_process_group()


def test_auto_buckets_are_planned_from_a_measured_link_and_agree_across_ranks():
    """bucket_mb="auto" at world > 1 times all-reduces on the trial's communicator (comm_plan.calibrate) and plans
    with that fit; the times are averaged over the ranks first, so every rank cuts the same buckets."""
    res = _run(_calib_worker, 2)
    a, b = res[0], res[1]
    assert a["plan"]["source"] == "measured", a["plan"]
    assert a["plan"] == b["plan"] and a["buckets"] == b["buckets"]
    assert a["plan"]["busbw_GBps"] > 0 and a["plan"]["bucket_bytes"] >= 4 * 2 ** 20


def _missing_peer_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank), PLX_COLLECTIVE_TIMEOUT_S="3")
    import time

    import torch.distributed as dist

    from polyaxon_amd.parallel import comm
    from polyaxon_amd.parallel.ddp import init_from_env

    init_from_env("gloo")
    c = comm.acquire(None, torch.device("cpu"))
    out = {"rank": rank}
    if rank == 0:  # rank 1 never joins the collective: rank 0 must fail within the deadline, not hang
        t0 = time.monotonic()
        try:
            c.all_reduce(torch.ones(4), op="sum")
            out["raised"] = False
        except RuntimeError as e:  # gloo's timeout surfaces as a RuntimeError (DistBackendError)
            out["raised"], out["msg"] = True, str(e)[:200]
        out["elapsed"] = time.monotonic() - t0
    else:
        time.sleep(8)
    q.put(out)
    q.close()
    q.join_thread()  # flush the result before skipping the broken group's teardown
    os._exit(0)


def test_gloo_shim_collective_with_a_missing_peer_fails_within_the_timeout():
    """The CPU twin of the RCCL watchdog (csrc/rccl_comm.cpp): a DP rank whose peer stops issuing collectives gets an
    error after PLX_COLLECTIVE_TIMEOUT_S (the rendezvous group's deadline, parallel/ddp.init_from_env) instead of
    blocking forever; polyflow then tears the gang down."""
    res = _run(_missing_peer_worker, 2, timeout=60)
    r0 = res[0]
    assert r0["raised"], r0
    assert 2.0 <= r0["elapsed"] < 8.0, r0


def test_init_from_env_keeps_an_explicit_gloo_backend_on_the_cpu(monkeypatch):
    """an explicit gloo backend means the CPU even on a GPU host (no HIP initialisation, no device ordinal
    taken from LOCAL_RANK); only nccl or an unnamed backend on a GPU host selects cuda:LOCAL_RANK."""
    from polyaxon_amd.parallel import ddp

    monkeypatch.setenv("WORLD_SIZE", "1")
    monkeypatch.setenv("LOCAL_RANK", "5")
    monkeypatch.setattr(torch.cuda, "is_available", lambda: True)
    set_to = []
    monkeypatch.setattr(torch.cuda, "set_device", lambda d: set_to.append(d))
    assert ddp.init_from_env("gloo")["device"].type == "cpu"
    assert set_to == []
    assert ddp.init_from_env()["device"] == torch.device("cuda", 5)
    assert ddp.init_from_env("nccl")["device"] == torch.device("cuda", 5)
