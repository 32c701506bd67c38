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


def _reducer_worker(rank, world, port, q):
    import os

    import torch
    import torch.distributed as dist

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.parallel.ddp import FlatDDP, MetricReducer, init_from_env

    init_from_env("gloo")
    torch.manual_seed(0)
    model = Transformer(tiny_llama())
    flat = FlatParams(model, "cpu", channels_last=False)
    ddp = FlatDDP(flat, bucket_mb=0.01, force_collectives=True)
    red = MetricReducer(torch.device("cpu"))
    torch.manual_seed(7 + rank)
    tokens = torch.randint(0, 256, (2, 16))
    loss = lm_loss(model(tokens), tokens)
    loss.backward()
    ddp.finish()
    m = red.mean(loss)
    q.put((rank, float(loss), float(m[0]), ddp.launched, len(ddp.buckets)))
    dist.destroy_process_group()


def test_metric_reducer_and_bucket_launches_gloo_world2():
    """The DP trial's metric all-reduce (MetricReducer: the RCCL communicator on the GPU, torch.distributed here)
    returns the cross-rank mean on every rank, and every gradient bucket's all-reduce is launched exactly once."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_reducer_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    mean = (res[0][1] + res[1][1]) / 2
    assert res[0][1] != res[1][1]
    assert all(abs(r[2] - mean) < 1e-5 for r in res)
    assert all(r[3] == r[4] > 1 for r in res)


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


def _avg_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env

    init_from_env("gloo")
    torch.manual_seed(0)
    model = Transformer(tiny_llama())
    flat = FlatParams(model, "cpu", channels_last=False)
    ddp = FlatDDP(flat, bucket_mb=0.01)
    ddp.broadcast_params()
    tokens = torch.randint(0, 256, (4, 16), generator=torch.Generator().manual_seed(100 + rank))
    lm_loss(model(tokens), tokens).backward()
    ddp.finish()
    q.put((rank, flat.grads.numpy().copy()))  # by value: a shared-memory tensor dies with its exiting producer
    dist.destroy_process_group()


def test_ddp_matches_single_process_average():
    """FlatDDP over gloo (world 2, each rank its own batch) yields on every rank exactly the gradient of the MEAN
    of the two ranks' losses computed in one process -- the DP correctness contract."""
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams

    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_avg_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    got = dict(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    torch.manual_seed(0)
    m = Transformer(tiny_llama())
    flat = FlatParams(m, "cpu", channels_last=False)
    toks = [torch.randint(0, 256, (4, 16), generator=torch.Generator().manual_seed(100 + r)) for r in range(2)]
    (sum(lm_loss(m(t), t) for t in toks) / 2).backward()
    ref = flat.grads.clone()
    assert float(ref.norm()) > 0
    for r in (0, 1):
        torch.testing.assert_close(torch.from_numpy(got[r]), ref, rtol=1e-4, atol=1e-6)


def _lp_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env

    init_from_env("gloo")
    torch.manual_seed(0)
    model = Transformer(tiny_llama())
    flat = FlatParams(model, "cpu", channels_last=False, lp_dtype=torch.bfloat16)
    flat.enable_direct_grads(True)  # weight grads written by the GEMM; buckets counted by post-accumulate hooks
    ddp = FlatDDP(flat, bucket_mb=0.01)
    torch.manual_seed(100 + rank)
    tokens = torch.randint(0, 256, (4, 16))
    ddp.broadcast_params()
    lm_loss(model(tokens), tokens).backward()
    ddp.finish()
    g = torch.cat([flat.lp_grads.float(), flat.grads])
    gathered = [torch.zeros_like(g) for _ in range(world)]
    dist.all_gather(gathered, g)
    # no bucket straddles the bf16 / fp32 boundary
    ok_buckets = all(hi <= flat.n_decay or lo >= flat.n_decay for lo, hi, _ in ddp.buckets)
    q.put((rank, ok_buckets, all(torch.equal(gathered[0], x) for x in gathered), float(g.norm())))
    dist.destroy_process_group()


def test_flat_ddp_lp_mode_gloo_world2():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_lp_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in procs)
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(r[1] and r[2] for r in res) and res[0][3] > 0


def test_lp_mode_matches_fp32_training():
    """bf16 model weights + fp32 master (lp mode) track the all-fp32 flat path within bf16 tolerance."""
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW

    tokens = torch.randint(0, 256, (4, 16), generator=torch.Generator().manual_seed(3))
    out = {}
    for lp in (None, torch.bfloat16):
        torch.manual_seed(0)
        model = Transformer(tiny_llama())
        flat = FlatParams(model, "cpu", channels_last=False, lp_dtype=lp)
        if lp is not None:
            assert model.embed.weight.dtype == torch.bfloat16 and model.norm.weight.dtype == torch.float32
            assert flat.grads.numel() == flat.numel - flat.n_decay
        opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1)
        losses = []
        for _ in range(3):
            loss = lm_loss(model(tokens), tokens)
            loss.backward()
            opt.step_()
            opt.step += 1
            losses.append(float(loss))
        if lp is not None:
            assert float(flat.lp_grads.abs().max()) == 0.0  # zeroed by the step
            assert torch.equal(flat.lp_params, flat.params[: flat.n_decay].to(torch.bfloat16))
        out[lp] = (losses, flat.params.clone())
    (l32, p32), (l16, p16) = out[None], out[torch.bfloat16]
    assert abs(l32[0] - l16[0]) < 0.05 and l16[-1] < l16[0]
    assert (p32 - p16).abs().max() < 0.05


def test_direct_grad_linear_matches_autograd():
    """lp mode: the direct-gradient GEMM path (ops/lm.linear) leaves exactly autograd's gradients in the flat
    buffer, also across two backward passes (accumulation) and an optimizer step (overwrite again)."""
    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams

    tokens = torch.randint(0, 256, (2, 16), generator=torch.Generator().manual_seed(5))
    grads = {}
    for direct in (False, True):
        torch.manual_seed(0)
        model = Transformer(tiny_llama())
        flat = FlatParams(model, "cpu", channels_last=False, lp_dtype=torch.bfloat16)
        flat.enable_direct_grads(direct)
        for _ in range(2):
            lm_loss(model(tokens), tokens).backward()
        grads[direct] = (flat.lp_grads.float().clone(), flat.grads.clone())
        if direct:
            assert len(flat._written) > 0
            flat.zero_grads()
            lm_loss(model(tokens), tokens).backward()
            torch.testing.assert_close(flat.lp_grads.float() * 2, grads[True][0], rtol=0.02, atol=2e-3)
    torch.testing.assert_close(grads[True][0], grads[False][0], rtol=0.02, atol=2e-3)
    torch.testing.assert_close(grads[True][1], grads[False][1], rtol=1e-3, atol=1e-5)


def _train_steps(lp, in_backward, steps=3, bucket_mb=0.01, arch="llama", direct=False):
    from polyaxon_amd.models.transformer import Transformer, gpt2_125m, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel.ddp import FlatDDP

    torch.manual_seed(0)
    cfg = tiny_llama() if arch == "llama" else gpt2_125m(vocab_size=256, n_layers=2, d_model=64, n_heads=2,
                                                            d_ff=256, max_seq_len=32)
    model = Transformer(cfg)
    flat = FlatParams(model, "cpu", channels_last=False, lp_dtype=lp)
    flat.enable_direct_grads(direct)
    opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1)
    ddp = FlatDDP(flat, bucket_mb=bucket_mb, optimizer=opt if in_backward else None)
    gen = torch.Generator().manual_seed(5)
    losses = []
    for _ in range(steps):
        tokens = torch.randint(0, 256, (4, 16), generator=gen)
        with torch.autocast("cpu", dtype=torch.bfloat16, enabled=lp is not None and arch != "llama"):
            loss = lm_loss(model(tokens), tokens)
        loss.backward()
        ddp.finish()
        opt.step_()
        opt.step += 1
        losses.append(float(loss))
    return losses, flat, ddp


@pytest.mark.parametrize("lp", [None, torch.bfloat16])
def test_optimizer_in_backward_matches_monolithic_step(lp):
    """FlatDDP(optimizer=...): AdamW runs per gradient bucket as each bucket completes in the backward; the
    trajectory (losses, fp32 master, bf16 model copy, moments) is bitwise the monolithic step's, every bucket is
    updated exactly once per step, and the gradients are left zeroed."""
    la, fa, _ = _train_steps(lp, False)
    lb, fb, ddp = _train_steps(lp, True)
    assert la == lb
    assert torch.equal(fa.params, fb.params)
    if lp is not None:
        assert torch.equal(fa.lp_params, fb.lp_params)
        assert float(fb.lp_grads.abs().max()) == 0.0
    assert float(fb.grads.abs().max()) == 0.0
    assert len(ddp.buckets) > 3 and ddp.stepped == 3 * len(ddp.buckets)


@pytest.mark.parametrize("arch", ["llama", "gpt2"])
def test_optimizer_in_backward_direct_grads_shared_buckets(arch):
    """Direct gradients (GEMM-written weights, bias sums written into their flat slots) with several parameters per
    bucket: each parameter counts its bucket down exactly once per backward -- autograd's post-accumulate hook also
    fires for a parameter whose Function returned None -- so no bucket is updated before all of its gradients are
    in, and the trajectory is bitwise the monolithic step's."""
    la, fa, _ = _train_steps(torch.bfloat16, False, bucket_mb=0.25, arch=arch, direct=True)
    lb, fb, ddp = _train_steps(torch.bfloat16, True, bucket_mb=0.25, arch=arch, direct=True)
    assert any(n > 2 for _, _, n in ddp.buckets)
    assert la == lb
    assert torch.equal(fa.params, fb.params) and torch.equal(fa.lp_params, fb.lp_params)
    assert ddp.stepped == 3 * len(ddp.buckets)


def _opt_in_bwd_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env

    init_from_env("gloo")
    out = {}
    for in_bwd in (False, True):
        torch.manual_seed(0)
        model = Transformer(tiny_llama())
        flat = FlatParams(model, "cpu", channels_last=False)
        opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1)
        ddp = FlatDDP(flat, bucket_mb=0.01, optimizer=opt if in_bwd else None)
        ddp.broadcast_params()
        gen = torch.Generator().manual_seed(100 + rank)  # different data per rank
        for _ in range(2):
            loss = lm_loss(model(torch.randint(0, 256, (4, 16), generator=gen)), torch.randint(0, 256, (4, 16),
                                                                                                generator=gen))
            loss.backward()
            ddp.finish()
            opt.step_()
            opt.step += 1
        p = flat.params.clone()
        gathered = [torch.zeros_like(p) for _ in range(world)]
        dist.all_gather(gathered, p)
        out[in_bwd] = (p, all(torch.equal(gathered[0], x) for x in gathered))
        ddp.remove_hooks()
    q.put((rank, out[True][1], out[False][1], bool(torch.allclose(out[True][0], out[False][0], rtol=0, atol=1e-6))))
    dist.destroy_process_group()


def test_optimizer_in_backward_gloo_world2():
    """DP world 2: each bucket's update waits for its all-reduce; the ranks stay identical and match the
    all-reduce-then-step path."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_opt_in_bwd_worker, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    res = [q.get(timeout=180) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    assert all(r[1] and r[2] and r[3] for r in res), res


def _zero_worker(rank, world, port, q, lp):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_RANK=str(rank))
    import torch.distributed as dist

    from polyaxon_amd.models.transformer import Transformer, lm_loss, tiny_llama
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.ops.optim import FusedAdamW
    from polyaxon_amd.parallel.ddp import FlatDDP, init_from_env

    torch.set_num_threads(2)  # W ranks share the CPU with the rest of the suite
    init_from_env("gloo")
    out = {}
    for zero in (False, True):
        torch.manual_seed(0)
        model = Transformer(tiny_llama())
        flat = FlatParams(model, "cpu", channels_last=False, lp_dtype=lp)
        opt = FusedAdamW(flat, lr=1e-2, weight_decay=0.1)
        ddp = FlatDDP(flat, bucket_mb=0.01, optimizer=opt, shard_optimizer=zero)
        ddp.broadcast_params()
        gen = torch.Generator().manual_seed(100 + rank)  # different data per rank
        losses = []
        for _ in range(3):
            tok = torch.randint(0, 256, (4, 16), generator=gen)
            loss = lm_loss(model(tok), torch.randint(0, 256, (4, 16), generator=gen))
            loss.backward()
            ddp.finish()
            opt.step_()
            opt.step += 1
            losses.append(float(loss))
        lp_copy = flat.lp_params.clone() if lp is not None else None
        ddp.gather_master()
        grads_zero = float(flat.grads.abs().max()) == 0.0 and (lp is None or float(flat.lp_grads.abs().max()) == 0.0)
        out[zero] = (losses, flat.params.clone(), lp_copy, opt.exp_avg.numel(), flat.numel, grads_zero,
                     ddp.launched, len(ddp.buckets))
        ddp.remove_hooks()
    (la, pa, lpa, na, numel, za, _, _), (lb, pb, lpb, nb, _, zb, launched, nbuck) = out[False], out[True]
    res = {"rank": rank, "losses_equal": la == lb, "master_equal": bool(torch.equal(pa, pb)),
           "lp_equal": lpa is None or bool(torch.equal(lpa, lpb)), "state_full": na, "state_sharded": nb,
           "numel": numel, "grads_zero": za and zb, "launched": launched, "buckets": nbuck,
           "max_diff": float((pa - pb).abs().max())}
    gathered = [torch.zeros_like(pb) for _ in range(world)]
    dist.all_gather(gathered, pb)
    res["ranks_equal"] = all(torch.equal(gathered[0], x) for x in gathered)
    q.put(res)
    dist.destroy_process_group()


@pytest.mark.parametrize("world,lp", [(2, None), (2, torch.bfloat16), (4, None), (4, torch.bfloat16)])
def test_zero1_sharded_adamw_matches_unsharded(world, lp):
    """ZeRO-1 (FlatDDP(shard_optimizer=True)): reduce-scatter -> AdamW on this rank's 1/W of each bucket ->
    all-gather of the updated weights follows the unsharded (all-reduce, every rank updates everything) trajectory
    bitwise -- losses, fp32 master (after gather_master), bf16 model copy -- with the ranks identical, the gradients
    left zeroed, and the AdamW moments W times smaller (up to the all-reduced sub-4W remainders)."""
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_zero_worker, args=(r, world, port, q, lp)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=300) for _ in procs]
    for p in procs:
        p.join(timeout=60)
    assert all(p.exitcode == 0 for p in procs)
    for r in res:
        assert r["losses_equal"] and r["master_equal"] and r["lp_equal"] and r["ranks_equal"], r
        assert r["grads_zero"] and r["launched"] == 3 * r["buckets"], r
        assert r["state_full"] == r["numel"]
        # each bucket keeps at most 4W - 1 replicated remainder elements beside its 1/W slice
        assert r["state_sharded"] <= r["numel"] / world + (4 * world) * r["buckets"], r
        assert r["state_sharded"] < 0.75 * r["numel"], r


def test_zero1_llama3_8b_state_shrinks_by_world_size():
    """The Llama-3 8B flat layout (built on the meta device: no memory) under ZeRO-1 with 64 MB buckets: every
    rank's packed AdamW state is numel / W exactly at W = 2, 4, 8 (the buckets divide evenly), i.e. the 64 GB of fp32
    moments become 8 GB per rank at DP 8; a shard never straddles a bucket."""
    from polyaxon_amd.models.transformer import Transformer, llama3_8b
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.parallel.ddp import FlatDDP

    with torch.device("meta"):
        model = Transformer(llama3_8b())
    flat = FlatParams(model, torch.device("meta"), channels_last=False, lp_dtype=torch.bfloat16)
    ddp = FlatDDP(flat, bucket_mb=64)
    assert flat.numel > 8.0e9
    for w in (2, 4, 8):
        shards, state = FlatDDP.plan_shards(ddp.buckets, w)
        assert state <= flat.numel / w + 4 * w * len(ddp.buckets)
        assert 2 * state * 4 / 2 ** 30 <= 64 / w * 1.001 * (flat.numel * 8 / 2 ** 30) / 64  # moments bytes / W
        for (lo, hi, _), (s, main, off) in zip(ddp.buckets, shards):
            assert main == s * w and main <= hi - lo and s % 4 == 0
