"""Numerics of the hand-written HIP kernels vs plain PyTorch fp32 references (run on a real MI355X)."""
import math

import numpy as np
import pytest
import torch

from polyaxon_amd.ops import _native

pytestmark = pytest.mark.gpu


def _stream():
    return torch.cuda.current_stream().cuda_stream


def test_sgd_flat_matches_reference(cuda):
    lib = _native.lib("plx_train")
    n, n_decay = 4096 * 37 + 4, 4096 * 20
    for first in (0, 5):
        for nesterov in (0.0, 1.0):
            p = torch.randn(n, device=cuda)
            g = torch.randn(n, device=cuda)
            m = torch.randn(n, device=cuda)
            hp = torch.tensor([0.1, 0.9, 1e-3, nesterov, 0.1, 0, 0, 0], device=cuda)
            step = torch.tensor([first], dtype=torch.int32, device=cuda)
            pr, gr, mr = p.clone(), g.clone(), m.clone()
            gr[:n_decay] += 1e-3 * pr[:n_decay]
            mr = gr.clone() if first == 0 else 0.9 * mr + 0.9 * gr
            d = gr + 0.9 * mr if nesterov else mr
            pr = pr - 0.1 * d
            _native.check(lib.plx_sgd_flat(p.data_ptr(), g.data_ptr(), m.data_ptr(), n, n_decay, hp.data_ptr(),
                                           step.data_ptr(), _stream()), "sgd")
            torch.cuda.synchronize()
            torch.testing.assert_close(p, pr, rtol=1e-5, atol=1e-6)
            torch.testing.assert_close(m, mr, rtol=1e-5, atol=1e-6)
            assert float(g.abs().max()) == 0.0


def test_adamw_flat_matches_torch(cuda):
    lib = _native.lib("plx_train")
    n, n_decay = 8192, 4096
    p = torch.randn(n, device=cuda)
    ref = p.clone().requires_grad_(False)
    m = torch.zeros(n, device=cuda)
    v = torch.zeros(n, device=cuda)
    hp = torch.tensor([1e-3, 0.9, 0.999, 1e-8, 0.01, 0, 0, 0], device=cuda)
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    pa = torch.nn.Parameter(ref[:n_decay].clone())
    pb = torch.nn.Parameter(ref[n_decay:].clone())
    opt = torch.optim.AdamW([{"params": [pa], "weight_decay": 0.01}, {"params": [pb], "weight_decay": 0.0}],
                            lr=1e-3, betas=(0.9, 0.999), eps=1e-8)
    for it in range(3):
        grad = torch.randn(n, device=cuda)
        g = grad.clone()
        _native.check(lib.plx_adamw_flat(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), n, n_decay,
                                         hp.data_ptr(), step.data_ptr(), _stream()), "adamw")
        step += 1
        pa.grad, pb.grad = grad[:n_decay].clone(), grad[n_decay:].clone()
        opt.step()
    torch.cuda.synchronize()
    torch.testing.assert_close(p, torch.cat([pa.detach(), pb.detach()]), rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n", [4096 * 9 + 4, 4096 * 9 + 8])
def test_adamw_mixed_matches_torch(cuda, n):
    """bf16 grads + fp32 master: same update as torch AdamW fed the (bf16-exact) grads; the bf16 model copy is
    the round-to-nearest-even of the master; the bf16 grads are zeroed.  n % 8 == 4 takes the 4-wide kernel, n % 8
    == 0 the 8-wide non-temporal one."""
    lib = _native.lib("plx_train")
    p = torch.randn(n, device=cuda)
    m = torch.zeros(n, device=cuda)
    v = torch.zeros(n, device=cuda)
    plp = torch.empty(n, dtype=torch.bfloat16, device=cuda)
    hp = torch.tensor([1e-3, 0.9, 0.95, 1e-8, 0.1, 0, 0, 0], device=cuda)
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    pa = torch.nn.Parameter(p.clone())
    opt = torch.optim.AdamW([pa], lr=1e-3, betas=(0.9, 0.95), eps=1e-8, weight_decay=0.1)
    for it in range(3):
        g = torch.randn(n, device=cuda).to(torch.bfloat16)
        pa.grad = g.float()
        _native.check(lib.plx_adamw_mixed(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), plp.data_ptr(), n,
                                          1, hp.data_ptr(), step.data_ptr(), _stream()), "adamw_mixed")
        step += 1
        opt.step()
        torch.cuda.synchronize()
        assert float(g.float().abs().max()) == 0.0
    torch.testing.assert_close(p, pa.detach(), rtol=1e-5, atol=1e-6)
    assert torch.equal(plp, p.to(torch.bfloat16))
    q = torch.empty_like(plp)
    _native.check(lib.plx_cast_lp(p.data_ptr(), q.data_ptr(), n, _stream()), "cast_lp")
    torch.cuda.synchronize()
    assert torch.equal(q, p.to(torch.bfloat16))


def test_init_flat_statistics(cuda):
    from polyaxon_amd.ops.flat import FlatParams
    from polyaxon_amd.models.resnet import resnet50

    model = resnet50()
    flat = FlatParams(model.to(memory_format=torch.channels_last), cuda)
    spec = model.init_spec()
    t = flat.init_tables(spec)
    flat.params.fill_(123.0)
    lib = _native.lib("plx_train")
    _native.check(lib.plx_init_flat(flat.params.data_ptr(), t["chunk_lo"].data_ptr(), t["chunk_hi"].data_ptr(),
                                    t["chunk_seg"].data_ptr(), int(t["chunk_lo"].numel()), t["seg_kind"].data_ptr(),
                                    t["seg_scale"].data_ptr(), 42, _stream()), "init")
    torch.cuda.synchronize()
    for p, kind, scale in spec:
        v = p.detach().float()
        if kind == "const":
            assert torch.all(v == scale)
        elif kind == "normal" and v.numel() > 10000:
            assert abs(float(v.mean())) < 0.05 * scale
            assert abs(float(v.std()) / scale - 1) < 0.03
        elif kind == "uniform":
            assert float(v.abs().max()) <= scale * (1 + 1e-6)
    # different seed -> different weights; same seed -> identical
    a = flat.params.clone()
    _native.check(lib.plx_init_flat(flat.params.data_ptr(), t["chunk_lo"].data_ptr(), t["chunk_hi"].data_ptr(),
                                    t["chunk_seg"].data_ptr(), int(t["chunk_lo"].numel()), t["seg_kind"].data_ptr(),
                                    t["seg_scale"].data_ptr(), 42, _stream()), "init")
    torch.cuda.synchronize()
    assert torch.equal(a, flat.params)


def test_record_and_commit_metric(cuda):
    lib = _native.lib("plx_train")
    ring = torch.zeros(16, device=cuda)
    step = torch.zeros(1, dtype=torch.int32, device=cuda)
    vals = [float(i) for i in range(20)]
    for v in vals:
        loss = torch.tensor(v, device=cuda)
        _native.check(lib.plx_record_metric(loss.data_ptr(), 0, ring.data_ptr(), step.data_ptr(), 16, _stream()), "r")
    out = torch.full((4,), math.nan, device=cuda)
    _native.check(lib.plx_commit_metric(ring.data_ptr(), step.data_ptr(), 16, 5, out.data_ptr(), 2, _stream()), "c")
    torch.cuda.synchronize()
    assert int(step) == 20
    assert float(out[2]) == pytest.approx(np.mean(vals[-5:]))
    assert math.isnan(float(out[0]))


def test_topk_brackets_matches_numpy(cuda):
    from polyaxon_amd.polytune.kernels import topk_order, topk_order_reference

    rng = np.random.default_rng(0)
    for B, C in ((1, 1), (3, 7), (64, 81), (5, 1000), (2, 2048)):
        m = rng.standard_normal((B, C)).astype(np.float32)
        m[rng.random((B, C)) < 0.1] = np.nan
        m[:, ::5] = np.round(m[:, ::5])  # ties
        counts = rng.integers(0, C + 1, size=B).astype(np.int32)
        for maximize in (False, True):
            got = topk_order(torch.from_numpy(m).to(cuda), torch.from_numpy(counts).to(cuda), maximize).cpu().numpy()
            exp = topk_order_reference(m, counts, maximize)
            np.testing.assert_array_equal(got, exp)


def test_select_top_matches_python_sorted(cuda):
    from polyaxon_amd.polytune.kernels import select_top

    metrics = [(10 + i, v) for i, v in enumerate([0.5, 0.1, 0.9, 0.1, 0.3, 0.7])]
    for maximize in (False, True):
        exp = [m[0] for m in sorted(metrics, key=lambda x: x[1], reverse=maximize)[:3]]
        if maximize:
            assert select_top(metrics, 3, True) == exp
        else:
            assert select_top(metrics, 3, False) == exp


def test_early_stop_any(cuda):
    from polyaxon_amd.polytune.kernels import early_stop_any

    m = torch.tensor([[0.5, 0.2], [0.95, float("nan")], [0.1, 0.05]], device=cuda)
    rules = [(0, 0.9, True), (1, 0.01, False), (1, 0.1, False), (0, 0.99, True)]
    assert early_stop_any(m, rules) == [True, False, True, False]
    assert early_stop_any(m.cpu(), rules) == [True, False, True, False]


def test_executor_graph_matches_eager(cuda):
    from polyaxon_amd.models.resnet import resnet18ish
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    torch.manual_seed(0)
    x = torch.randn(8, 3, 32, 32).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,))
    losses = []
    for use_graph in (False, True):
        ex = ResidentTrialExecutor(resnet18ish(), (x, y), cuda, use_graph=use_graph)
        ex.capture(warmup=2)
        ex.reset(seed=7)
        ex.set_hparams(lr=0.05, momentum=0.9, weight_decay=1e-4)
        ex.run(6)
        torch.cuda.synchronize()
        losses.append(ex.losses())
    torch.testing.assert_close(losses[0], losses[1], rtol=2e-2, atol=2e-2)


def test_executor_snapshot_restore_is_exact(cuda):
    from polyaxon_amd.models.resnet import resnet18ish
    from polyaxon_amd.polyflow.executor import ResidentTrialExecutor

    x = torch.randn(8, 3, 32, 32).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    y = torch.randint(0, 10, (8,))
    ex = ResidentTrialExecutor(resnet18ish(), (x, y), cuda)
    ex.capture(warmup=1)
    ex.reset(seed=3)
    ex.set_hparams(lr=0.01, momentum=0.9, weight_decay=0.0)
    ex.run(3)
    ex.snapshot("a")
    ex.run(3)
    p1 = ex.flat.params.clone()
    l1 = ex.losses()[-3:]
    ex.reset(seed=99)
    ex.run(2)
    ex.restore("a")
    ex.run(3)
    torch.cuda.synchronize()
    torch.testing.assert_close(ex.flat.params, p1, rtol=1e-4, atol=1e-5)
    torch.testing.assert_close(ex.losses()[-3:], l1, rtol=1e-3, atol=1e-3)


@pytest.mark.parametrize("shape", [(2, 64, 112, 112), (3, 16, 9, 7), (1, 8, 2, 2)])
def test_maxpool3s2_matches_torch(cuda, shape):
    from polyaxon_amd.ops.pool import _MaxPool3s2

    torch.manual_seed(0)
    x = torch.randn(shape, device=cuda).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
    x[0, 0, 0, :2] = 3.0  # a tie inside one window: both implementations keep the first maximum
    xa = x.clone().requires_grad_()
    y = _MaxPool3s2.apply(xa)
    xr = x.clone().requires_grad_()
    yr = torch.nn.functional.max_pool2d(xr, 3, 2, 1)
    assert torch.equal(y, yr)
    g = torch.randn_like(yr)
    y.backward(g)
    yr.backward(g)
    torch.testing.assert_close(xa.grad.float(), xr.grad.float(), rtol=1e-2, atol=1e-2)


def test_adamw_mixed_wide_matches_narrow(cuda):
    """The 8-wide non-temporal AdamW kernel (plx_set_adamw_wide 1) is bitwise the 4-wide one: both run adamw_elem,
    whose rounding steps are explicit (per-bucket launches mixing the two must equal one monolithic launch)."""
    lib = _native.lib("plx_train")
    n = 8192 * 5
    torch.manual_seed(4)
    p0, m0, v0 = torch.randn(n, device=cuda), torch.randn(n, device=cuda) * 0.1, torch.rand(n, device=cuda) * 0.01
    g0 = torch.randn(n, device=cuda).to(torch.bfloat16)
    hp = torch.tensor([1e-3, 0.9, 0.95, 1e-8, 0.1, 0, 0, 0], device=cuda)
    step = torch.full((1,), 7, dtype=torch.int32, device=cuda)
    res = {}
    try:
        for wide in (0, 1, 2):
            lib.plx_set_adamw_wide(wide)
            p, m, v, g = p0.clone(), m0.clone(), v0.clone(), g0.clone()
            plp = torch.empty(n, dtype=torch.bfloat16, device=cuda)
            _native.check(lib.plx_adamw_mixed(p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr(), plp.data_ptr(),
                                              n, 1, hp.data_ptr(), step.data_ptr(), _stream()), "adamw_mixed")
            torch.cuda.synchronize()
            res[wide] = (p, m, v, plp, g)
    finally:
        lib.plx_set_adamw_wide(0)  # the library default
    for wide in (1, 2):
        for a, b in zip(res[0], res[wide]):
            assert torch.equal(a, b)
        assert float(res[wide][4].float().abs().max()) == 0.0
