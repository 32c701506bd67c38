"""FlatDDP's default GPU path at world 2: the bucket all-reduces, ZeRO-1's reduce-scatter / all-gather, the parameter
broadcast and the metric mean on the framework's RCCL communicator (parallel/comm.py) against ProcessGroupNCCL
(PLX_DDP_COMM=pg over an nccl group).  Needs two GPUs (one rank per device; RCCL refuses two ranks on one device), so
it skips on a 1-GPU box; the same comparison runs on CPU ranks through the gloo shim in tests/test_comm.py."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp

pytestmark = pytest.mark.gpu


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _train(rank, zero, pg_group):
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel.ddp import FlatDDP, MetricReducer

    dev = torch.device("cuda", rank)
    os.environ["PLX_DDP_COMM"] = "pg" if pg_group is not None else "comm"
    torch.manual_seed(0)
    model = Transformer(tiny_llama()).to(dev)
    flat = FlatParams(model, dev, channels_last=False, lp_dtype=torch.bfloat16)
    flat.enable_direct_grads(True)  # as trainers.train_lm: weight-gradient GEMMs write the flat bf16 grads
    opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1)
    ddp = FlatDDP(flat, process_group=pg_group, bucket_mb=0.01, optimizer=opt, shard_optimizer=zero)
    red = MetricReducer(dev, process_group=pg_group)
    if rank:
        with torch.no_grad():
            flat.params.add_(1.0)
        flat.sync_lp()
    ddp.broadcast_params()
    gen = torch.Generator(device=dev).manual_seed(100 + rank)
    losses, means = [], []
    for _ in range(3):
        tok = torch.randint(0, 256, (4, 16), generator=gen, device=dev)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            loss = lm_loss(model(tok), torch.randint(0, 256, (4, 16), generator=gen, device=dev))
        loss.backward()
        ddp.finish()
        opt.step_()
        opt.step += 1
        losses.append(float(loss))
        means.append(float(red.mean(loss.detach())[0]))
    ddp.gather_master()
    torch.cuda.synchronize()
    out = {"losses": losses, "means": means, "params": flat.params.detach().cpu().clone(),
           "comm": ddp._comm is not None}
    ddp.remove_hooks()
    ddp.close()
    red.close()
    return out


def _worker(rank, world, port, q, zero):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.parallel.ddp import init_from_env

    try:
        init_from_env()  # gloo rendezvous, as every DP trial
        nccl = dist.new_group(backend="nccl")
        a = _train(rank, zero, None)
        b = _train(rank, zero, nccl)
        rel = float((a["params"] - b["params"]).abs().max() / b["params"].abs().max())
        q.put({"rank": rank, "comm": a["comm"], "pg": not b["comm"], "rel": rel,
               "loss_diff": max(abs(x - y) for x, y in zip(a["losses"], b["losses"])),
               "mean_diff": max(abs(x - y) for x, y in zip(a["means"], b["means"]))})
        dist.destroy_process_group()
    except Exception as e:  # report instead of hanging the parent on the queue
        q.put({"rank": rank, "error": repr(e)})


@pytest.mark.skipif(not torch.cuda.is_available() or torch.cuda.device_count() < 2, reason="needs 2 GPUs")
@pytest.mark.parametrize("zero", [False, True])
def test_framework_rccl_path_matches_process_group_nccl(zero):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, zero)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted((q.get(timeout=240) for _ in procs), key=lambda r: r["rank"])
    for p in procs:
        p.join(timeout=60)
    for r in res:
        assert "error" not in r, r
        assert r["comm"] and r["pg"], r
        # same library, same ring: equal up to the reduction order RCCL picks per communicator
        assert r["rel"] < 1e-5 and r["loss_diff"] < 1e-4 and r["mean_diff"] < 1e-4, r
