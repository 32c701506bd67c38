"""Fused NHWC bf16 BatchNorm(+add)(+ReLU) HIP kernels vs an fp32 PyTorch reference of the same op."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


def _ref(x, w, b, rm, rv, res, relu, momentum=0.1, eps=1e-5):
    y = F.batch_norm(x.float(), rm, rv, w, b, True, momentum, eps)
    if res is not None:
        y = y + res.float()
    return F.relu(y) if relu else y


@pytest.mark.parametrize("shape", [(4, 64, 14, 14), (2, 256, 7, 9), (3, 2048, 3, 3), (2, 4096, 2, 2),
                                   (2, 128, 1, 1), (8, 64, 56, 56)])
@pytest.mark.parametrize("relu,residual", [(True, False), (True, True), (False, False)])
def test_bn_act_forward_backward(cuda, shape, relu, residual):
    from polyaxon_amd.ops.bn_fused import bn_act, supported

    torch.manual_seed(0)
    n, c, h, w = shape
    x = (torch.randn(shape, device=cuda) * 2 + 0.5).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    assert supported(x)
    res = (torch.randn(shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
           if residual else None)
    wgt = (torch.rand(c, device=cuda) + 0.5).requires_grad_()
    bias = (torch.randn(c, device=cuda) * 0.1).requires_grad_()
    rm, rv = torch.zeros(c, device=cuda), torch.ones(c, device=cuda)
    rm_ref, rv_ref = rm.clone(), rv.clone()

    xa = x.clone().requires_grad_()
    ra = res.clone().requires_grad_() if residual else None
    y = bn_act(xa, wgt, bias, rm, rv, True, 0.1, 1e-5, ra, relu)
    xr = x.float().clone().requires_grad_()
    rr = res.float().clone().requires_grad_() if residual else None
    wr = wgt.detach().clone().requires_grad_()
    br = bias.detach().clone().requires_grad_()
    yr = _ref(xr, wr, br, rm_ref, rv_ref, rr, relu)

    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=3e-2)
    torch.testing.assert_close(rm, rm_ref, rtol=1e-3, atol=1e-3)
    torch.testing.assert_close(rv, rv_ref, rtol=1e-3, atol=1e-3)

    g = torch.randn(shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y.backward(g)
    yr.backward(g.float())
    scale = max(1.0, float(xr.grad.abs().max()))
    torch.testing.assert_close(xa.grad.float(), xr.grad, rtol=3e-2, atol=3e-2 * scale)
    m = n * h * w
    torch.testing.assert_close(wgt.grad, wr.grad, rtol=2e-2, atol=2e-2 * m ** 0.5)
    torch.testing.assert_close(bias.grad, br.grad, rtol=2e-2, atol=2e-2 * m ** 0.5)
    if residual:
        torch.testing.assert_close(ra.grad.float(), rr.grad, rtol=2e-2, atol=2e-2)


def test_bn_act_eval_matches_reference(cuda):
    from polyaxon_amd.ops.bn_fused import bn_act

    x = torch.randn(2, 64, 5, 5, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    w, b = torch.rand(64, device=cuda) + 0.5, torch.randn(64, device=cuda)
    rm, rv = torch.randn(64, device=cuda), torch.rand(64, device=cuda) + 0.5
    y = bn_act(x, w, b, rm, rv, False, 0.1, 1e-5, None, True)
    yr = F.relu(F.batch_norm(x.float(), rm, rv, w, b, False, 0.1, 1e-5))
    torch.testing.assert_close(y.float(), yr, rtol=2e-2, atol=2e-2)


def test_resnet_fused_matches_unfused_loss(cuda):
    """Fused bf16 path vs unfused bf16 path, both judged against an fp32 run of the same network."""
    from polyaxon_amd.models.resnet import resnet18ish

    torch.manual_seed(0)
    x32 = torch.randn(8, 3, 32, 32, device=cuda).contiguous(memory_format=torch.channels_last)
    x = x32.to(torch.bfloat16)
    y = torch.randint(0, 10, (8,), device=cuda)
    res = {}
    for name, fused, amp in (("fused", True, True), ("unfused", False, True), ("fp32", False, False)):
        torch.manual_seed(1)
        m = resnet18ish(fused=fused).to(cuda).to(memory_format=torch.channels_last)
        with torch.autocast("cuda", dtype=torch.bfloat16, enabled=amp):
            out = m(x if amp else x32)
        loss = F.cross_entropy(out.float(), y)
        loss.backward()
        res[name] = (float(loss.detach()), m.stem.weight.grad.flatten().float().clone())
    assert abs(res["fused"][0] - res["fp32"][0]) < 3e-2
    cos = {k: float(F.cosine_similarity(res[k][1], res["fp32"][1], dim=0)) for k in ("fused", "unfused")}
    assert cos["fused"] > 0.9, cos
    assert cos["fused"] >= cos["unfused"] - 0.01, cos


def test_reduce_finalize_one_launch_matches_two(cuda):
    """The one-launch reduce + finalize (ticket counters, last-arriver finalize) gives bit-identical statistics and
    backward coefficients to the two-launch path, over many row splits (S = 16) and repeated calls (the counters
    return to zero)."""
    from polyaxon_amd.ops import _native

    lib = _native.lib("plx_bn")
    torch.manual_seed(7)
    m, c, nblk = 128 * 1000, 256, 1000
    f32 = dict(dtype=torch.float32, device=cuda)
    x = torch.randn(m, c, device=cuda).to(torch.bfloat16)
    part = torch.rand(2 * nblk * c, **f32) * 4.0
    l2 = torch.empty(int(lib.plx_bn_l2_workspace(nblk, c)), **f32)
    cnt = torch.zeros(64, dtype=torch.int32, device=cuda)
    w, b = torch.rand(c, **f32) + 0.5, torch.randn(c, **f32)
    st = torch.cuda.current_stream().cuda_stream

    def fwd(counters):
        stats, rm, rv = torch.empty(4 * c, **f32), torch.zeros(c, **f32), torch.ones(c, **f32)
        rc = lib.plx_bn_forward_from_partials(x.data_ptr(), None, None, m, c, w.data_ptr(), b.data_ptr(), 1e-5, 0.1,
                                              rm.data_ptr(), rv.data_ptr(), stats.data_ptr(), stats[c:].data_ptr(),
                                              stats[2 * c:].data_ptr(), part.data_ptr(), nblk, l2.data_ptr(), None, 0,
                                              None, counters, st)
        assert rc == 0
        return torch.cat([stats, rm, rv])

    mean, inv = torch.randn(c, **f32), torch.rand(c, **f32) + 0.5

    def bwd(counters):
        dg, db, coef = torch.zeros(c, **f32), torch.zeros(c, **f32), torch.empty(3 * c, **f32)
        dx = torch.empty_like(x)
        rc = lib.plx_bn_backward_from_partials(x.data_ptr(), None, x.data_ptr(), dx.data_ptr(), None, m, c,
                                               w.data_ptr(), mean.data_ptr(), inv.data_ptr(), dg.data_ptr(),
                                               db.data_ptr(), coef.data_ptr(), part.data_ptr(), nblk, l2.data_ptr(),
                                               0, 1, None, counters, st)
        assert rc == 0
        return torch.cat([dg, db, coef])

    ref_f, ref_b = fwd(None), bwd(None)
    for _ in range(3):
        assert torch.equal(fwd(cnt.data_ptr()), ref_f)
        assert torch.equal(bwd(cnt.data_ptr()), ref_b)
    torch.cuda.synchronize()
    assert int(cnt.abs().sum()) == 0
    # and against the fp64 host sums
    p = part.view(2, nblk, c).double().sum(1)
    mean = p[0] / m
    torch.testing.assert_close(ref_f[:c].double(), mean, rtol=1e-5, atol=1e-6)


def test_fence_free_handoff_stress(cuda):
    """csrc/handoff.h's hardware assumption under load: 200 back-to-back one-launch reduce + finalize calls
    over fresh partials, each grid (C/64 x S = 8 x 64 blocks of 1024 threads) larger than one workgroup per CU, while a
    second stream keeps every CU busy with a streaming copy (uneven load, consumers L1-warm from the previous call):
    every result bitwise equals the two-launch path (whose hand-off is a kernel boundary)."""
    from polyaxon_amd.ops import _native

    lib = _native.lib("plx_bn")
    torch.manual_seed(11)
    m, c, nblk = 128 * 4096, 512, 4096
    f32 = dict(dtype=torch.float32, device=cuda)
    x = torch.randn(m, c, device=cuda).to(torch.bfloat16)
    l2 = torch.empty(int(lib.plx_bn_l2_workspace(nblk, c)), **f32)
    cnt = torch.zeros(64, dtype=torch.int32, device=cuda)
    w, b = torch.rand(c, **f32) + 0.5, torch.randn(c, **f32)
    side = torch.cuda.Stream()
    big = torch.empty(64 << 20, **f32)
    bigo = torch.empty_like(big)
    parts = [torch.rand(2 * nblk * c, **f32) * 4.0 for _ in range(4)]

    def fwd(part, counters):
        stats, rm, rv = torch.empty(4 * c, **f32), torch.zeros(c, **f32), torch.ones(c, **f32)
        rc = lib.plx_bn_forward_from_partials(x.data_ptr(), None, None, m, c, w.data_ptr(), b.data_ptr(), 1e-5, 0.1,
                                              rm.data_ptr(), rv.data_ptr(), stats.data_ptr(), stats[c:].data_ptr(),
                                              stats[2 * c:].data_ptr(), part.data_ptr(), nblk, l2.data_ptr(), None, 0,
                                              None, counters, torch.cuda.current_stream().cuda_stream)
        assert rc == 0
        return torch.cat([stats, rm, rv])

    refs = [fwd(p, None) for p in parts]
    got = []
    for i in range(200):
        if i % 10 == 0:
            with torch.cuda.stream(side):  # every CU streaming beside the hand-offs
                bigo.copy_(big)
        got.append(fwd(parts[i % 4], cnt.data_ptr()))
    torch.cuda.synchronize()
    bad = [i for i, g in enumerate(got) if not torch.equal(g, refs[i % 4])]
    assert not bad, f"{len(bad)} of 200 calls differ from the two-launch path (first: {bad[:5]})"
    assert int(cnt.abs().sum()) == 0


@pytest.mark.parametrize("shape", [(4, 64, 112, 112), (3, 64, 15, 17), (2, 128, 9, 8), (2, 8, 6, 5)])
def test_stem_bn_relu_pool_matches_unfused(cuda, shape):
    """ops.stem: BN + ReLU + max-pool in one forward pass and two backward passes (csrc/bn_kernels.hip) gives the
    unfused ops' pooled output (bit-exact: same bf16 values pooled, same ties), the same running stats and the same
    dx / dgamma / dbeta, and both match an fp32 PyTorch reference of the composition."""
    from polyaxon_amd.ops.norm import BatchNormAct
    from polyaxon_amd.ops.pool import MaxPool3s2
    from polyaxon_amd.ops.stem import stem_bn_relu_pool, supported

    torch.manual_seed(0)
    n, c, h, w = shape
    x = (torch.randn(shape, device=cuda) * 2 + 0.3).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    oh, ow = (h - 1) // 2 + 1, (w - 1) // 2 + 1
    g = torch.randn(n, c, oh, ow, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    outs = []
    for fused in (True, False):
        bn = BatchNormAct(c, act=True).to(cuda)
        with torch.no_grad():
            bn.weight.copy_(torch.linspace(0.5, 1.5, c))
            bn.bias.copy_(torch.linspace(-0.2, 0.2, c))
        pool = MaxPool3s2()
        xa = x.clone().requires_grad_()
        if fused:
            assert supported(xa, bn, pool)
            y = stem_bn_relu_pool(xa, bn, pool)
        else:
            y = pool(bn(xa))
        y.backward(g)
        outs.append((y.detach().float(), xa.grad.float(), bn.weight.grad.clone(), bn.bias.grad.clone(),
                     bn.running_mean.clone(), bn.running_var.clone(), g))
    (yf, dxf, dgf, dbf, rmf, rvf, gf), (yu, dxu, dgu, dbu, rmu, rvu, _) = outs
    assert torch.equal(yf, yu)
    torch.testing.assert_close(rmf, rmu)
    torch.testing.assert_close(rvf, rvu)
    scale = float(dxu.abs().max())
    torch.testing.assert_close(dxf, dxu, rtol=2e-2, atol=2e-2 * scale)
    torch.testing.assert_close(dgf, dgu, rtol=1e-3, atol=1e-3 * float(dgu.abs().max()))
    torch.testing.assert_close(dbf, dbu, rtol=1e-3, atol=1e-3 * float(dbu.abs().max()))
    # fp32 reference of the composition
    xr = x.float().clone().requires_grad_()
    wr = torch.linspace(0.5, 1.5, c, device=cuda).requires_grad_()
    br = torch.linspace(-0.2, 0.2, c, device=cuda).requires_grad_()
    yr = F.max_pool2d(F.relu(F.batch_norm(xr, None, None, wr, br, True, 0.1, 1e-5)), 3, 2, 1)
    yr.backward(gf.float())
    torch.testing.assert_close(yf, yr, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(dgf, wr.grad, rtol=5e-2, atol=5e-2 * float(wr.grad.abs().max()))
    torch.testing.assert_close(dbf, br.grad, rtol=5e-2, atol=5e-2 * float(br.grad.abs().max()))
