"""The 256x256 MFMA GEMM of the LM linears (csrc/gemm256.hip via ops/gemm.py) vs fp32 PyTorch references."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def cuda():
    if not torch.cuda.is_available():
        pytest.skip("needs a GPU")
    return torch.device("cuda", 0)


def _rand(shape, device, seed):
    g = torch.Generator(device=device).manual_seed(seed)
    return torch.randn(shape, device=device, generator=g).to(torch.bfloat16)


def _check(out, ref, K):
    # bf16 output of a K-long fp32 accumulation of bf16 products: relative error ~2^-8 on the output
    err = (out.float() - ref).abs().max().item()
    scale = ref.abs().max().item()
    assert err <= 1.5e-2 * scale + 1e-3, (err, scale, K)


@pytest.mark.parametrize("a_kmajor,b_kmajor", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 320), (768, 512, 1024)])
def test_gemm256_layouts_match_fp32(cuda, a_kmajor, b_kmajor, M, N, K):
    from polyaxon_amd.ops import gemm

    a = _rand((M, K) if a_kmajor else (K, M), cuda, 1)
    b = _rand((N, K) if b_kmajor else (K, N), cuda, 2)
    out = gemm.gemm(a, b, M, N, K, a_kmajor, b_kmajor)
    af = a.float() if a_kmajor else a.float().t()
    bf = b.float() if b_kmajor else b.float().t()
    torch.cuda.synchronize()
    _check(out, af @ bf.t(), K)


@pytest.mark.parametrize("accumulate", [False, True])
@pytest.mark.parametrize("M,N,K", [(256, 256, 8192), (512, 256, 4096), (256, 512, 2048 + 64)])
def test_gemm256_split_k_and_accumulate(cuda, accumulate, M, N, K):
    """Small tile grids with long K (the weight gradient) run split-K over fp32 slabs; accumulate adds into C."""
    from polyaxon_amd.ops import _native, gemm

    splits = _native.size("plx_gemm", "plx_gemm256_splits", M, N, K)
    if K >= 4096:
        assert splits > 1
    a = _rand((K, M), cuda, 3)
    b = _rand((K, N), cuda, 4)
    c0 = _rand((M, N), cuda, 5)
    out = c0.clone()
    gemm.gemm(a, b, M, N, K, False, False, out=out, accumulate=accumulate, alpha=0.5)
    ref = 0.5 * (a.float().t() @ b.float())
    if accumulate:
        ref = ref + c0.float()
    torch.cuda.synchronize()
    _check(out, ref, K)


@pytest.mark.parametrize("M,N,K", [(512, 768, 768), (256, 256, 8192)])
def test_gemm256_bias_epilogue(cuda, M, N, K):
    """The fp32 bias added by the epilogue (plx_gemm256_bias): one-pass tiles and the split-K reduce, a bf16 bias
    (cast to fp32 on the host side) included."""
    from polyaxon_amd.ops import gemm

    a = _rand((M, K), cuda, 6)
    b = _rand((N, K), cuda, 7)
    for bias in (torch.randn(N, device=cuda), torch.randn(N, device=cuda).to(torch.bfloat16)):
        out = gemm.gemm(a, b, M, N, K, True, True, bias=bias)
        ref = a.float() @ b.float().t() + bias.float()
        torch.cuda.synchronize()
        _check(out, ref, K)


@pytest.fixture(params=[5], ids=["barrier_per_two_phases"])
def four_waves(cuda, request):
    from polyaxon_amd.ops import _native

    lib = _native.lib("plx_gemm")
    prev = lib.plx_gemm256_set_waves(request.param)
    yield
    lib.plx_gemm256_set_waves(prev)


@pytest.mark.parametrize("a_kmajor,b_kmajor", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [(256, 256, 64), (512, 768, 320), (768, 512, 1024), (256, 512, 8192)])
def test_gemm256_four_wave_kernel_matches_fp32(cuda, four_waves, a_kmajor, b_kmajor, M, N, K):
    """The 4-wave kernel (AGPR accumulators through inline-asm MFMAs): every layout, 1 / odd / many K-tiles, and the
    split-K slabs (256 x 512 x 8192), plain and accumulating with alpha."""
    from polyaxon_amd.ops import gemm

    a = _rand((M, K) if a_kmajor else (K, M), cuda, 11)
    b = _rand((N, K) if b_kmajor else (K, N), cuda, 12)
    af = a.float() if a_kmajor else a.float().t()
    bf = b.float() if b_kmajor else b.float().t()
    out = gemm.gemm(a, b, M, N, K, a_kmajor, b_kmajor)
    torch.cuda.synchronize()
    _check(out, af @ bf.t(), K)
    c0 = _rand((M, N), cuda, 13)
    acc = c0.clone()
    gemm.gemm(a, b, M, N, K, a_kmajor, b_kmajor, out=acc, accumulate=True, alpha=0.5)
    torch.cuda.synchronize()
    _check(acc, 0.5 * (af @ bf.t()) + c0.float(), K)


def test_gemm256_four_wave_epilogues_and_repeat(cuda, four_waves):
    """Bias + GELU epilogue on the 4-wave kernel, and 20 back-to-back launches bitwise equal (a DMA / read race
    shows up as run-to-run differences)."""
    from polyaxon_amd.ops import gemm

    M, N, K = 512, 768, 2048
    a, b = _rand((M, K), cuda, 14), _rand((N, K), cuda, 15)
    bias = torch.randn(N, device=cuda)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    g = torch.empty_like(h)
    gemm.gemm(a, b, M, N, K, True, True, out=h, bias=bias, gelu_out=g)
    ref = a.float() @ b.float().t() + bias
    torch.cuda.synchronize()
    _check(h, ref, K)
    _check(g, F.gelu(h.float(), approximate="tanh"), K)
    first = gemm.gemm(a, b, M, N, K, True, True)
    for _ in range(20):
        again = gemm.gemm(a, b, M, N, K, True, True)
        assert torch.equal(first, again)


def test_gemm256_strided_output(cuda):
    """out may be a column block of a wider matrix (ldc > N)."""
    from polyaxon_amd.ops import gemm

    M, N, K = 256, 256, 512
    a, b = _rand((M, K), cuda, 6), _rand((N, K), cuda, 7)
    wide = torch.zeros(M, 3 * N, dtype=torch.bfloat16, device=cuda)
    gemm.gemm(a, b, M, N, K, True, True, out=wide[:, N:2 * N])
    torch.cuda.synchronize()
    _check(wide[:, N:2 * N], a.float() @ b.float().t(), K)
    assert wide[:, :N].abs().max().item() == 0 and wide[:, 2 * N:].abs().max().item() == 0


@pytest.mark.parametrize("bias", [False, True])
def test_lm_linear_on_mfma_matches_fp32(cuda, bias, monkeypatch):
    """ops.lm.linear: forward, dx and dW (and db) of the MFMA path vs fp32 autograd."""
    from polyaxon_amd.ops import _native, lm

    monkeypatch.setenv("PLX_LM_GEMM", "1")

    B, S, fin, fout = 2, 256, 768, 1280
    x = _rand((B, S, fin), cuda, 8).requires_grad_()
    w = (_rand((fout, fin), cuda, 9).float() * 0.05).to(torch.bfloat16).requires_grad_()
    b = (_rand((fout,), cuda, 10).float() * 0.1).to(torch.bfloat16).requires_grad_() if bias else None
    y = lm.linear(x, w, b)
    assert y.grad_fn is not None and "Mfma" in type(y.grad_fn).__name__
    dy = _rand((B, S, fout), cuda, 11)
    y.backward(dy)
    xr = x.detach().float().requires_grad_()
    wr = w.detach().float().requires_grad_()
    br = b.detach().float().requires_grad_() if bias else None
    yr = F.linear(xr, wr, br)
    yr.backward(dy.float())
    torch.cuda.synchronize()
    _check(y, yr.detach(), fin)
    _check(x.grad, xr.grad, fout)
    _check(w.grad, wr.grad, B * S)
    if bias:
        torch.testing.assert_close(b.grad.float(), br.grad, rtol=2e-2, atol=2e-1)
    assert _native.lib_path("plx_gemm").exists()


@pytest.mark.parametrize("mode", ["1", "0"])
def test_lm_linear_direct_grad_slot_accumulates(cuda, mode, monkeypatch):
    """A flat-parameter weight used twice: the first wgrad writes the bf16 slot, the second accumulates in place
    (on the MFMA kernel's epilogue, and on the hipBLASLt addmm path)."""
    from polyaxon_amd.ops import lm

    monkeypatch.setenv("PLX_LM_GEMM", mode)

    class _Flat:
        def __init__(self):
            self.written = set()

        def mark_written(self, g):
            k = g.data_ptr()
            seen = k in self.written
            self.written.add(k)
            return seen

    T, fin, fout = 512, 512, 768
    w = (_rand((fout, fin), cuda, 12).float() * 0.05).to(torch.bfloat16).requires_grad_()
    w.grad = torch.full_like(w, 7.0)  # stale content: the first write must overwrite it
    w._plx_flat, w._plx_direct_grad = _Flat(), True
    x1, x2 = _rand((T, fin), cuda, 13).requires_grad_(), _rand((T, fin), cuda, 14).requires_grad_()
    y = lm.linear(x1, w) + lm.linear(x2, w)
    dy = _rand((T, fout), cuda, 15)
    slot = w.grad
    y.backward(dy)
    ref = dy.float().t() @ (x1.detach().float() + x2.detach().float())
    torch.cuda.synchronize()
    assert w.grad.data_ptr() == slot.data_ptr()
    _check(w.grad, ref, 2 * T)


def test_transformer_step_uses_mfma_linears(cuda, monkeypatch):
    """A GPT-2-shaped block in lp-bf16 takes the MFMA path for every projection (no hipBLASLt fallback)."""
    from polyaxon_amd.models.transformer import Block, gpt2_125m

    monkeypatch.setenv("PLX_LM_GEMM", "1")

    cfg = gpt2_125m(n_layers=1)
    blk = Block(cfg).to(cuda).to(torch.bfloat16)
    x = _rand((1, 256, cfg.d_model), cuda, 16).requires_grad_()
    y = blk(x)
    names = set()
    stack = [y.grad_fn]
    while stack:
        fn = stack.pop()
        if fn is None:
            continue
        names.add(type(fn).__name__)
        stack.extend(f for f, _ in fn.next_functions)
    assert any("Mfma" in n for n in names), names
    assert not any(n.startswith("AddmmBackward") or n.startswith("MmBackward") for n in names), names
    y.float().square().mean().backward()
    assert torch.isfinite(x.grad.float()).all()


def test_auto_dispatch_runs_both_paths_and_matches(cuda, monkeypatch):
    """``auto``: a table / split-K shape runs the kernel, a large forward shape hipBLASLt; both match fp32."""
    from polyaxon_amd.ops import gemm

    monkeypatch.setenv("PLX_LM_GEMM", "auto")
    gemm._seen.clear()
    T, fin, fout = 4096, 768, 2304  # outside the table: the forward goes to hipBLASLt
    x, w = _rand((T, fin), cuda, 17), _rand((fout, fin), cuda, 18)
    dy = _rand((T, fout), cuda, 19)
    y = gemm.forward(x, w)
    dw = gemm.wgrad(dy, x)
    dec = gemm.decisions()
    assert dec[f"{T}x{fout}x{fin}:KK"]["native"] is False
    assert dec[f"{fout}x{fin}x{T}:MN"]["native"] is True  # split-K weight gradient
    torch.cuda.synchronize()
    _check(y, x.float() @ w.float().t(), fin)
    _check(dw, dy.float().t() @ x.float(), T)
    gemm._seen.clear()


def test_autocast_fp32_input_takes_mfma_path(cuda, monkeypatch):
    """Under bf16 autocast a LayerNorm output arrives in fp32: lm.linear casts it like autocast's F.linear would and
    keeps the projection on the MFMA kernel (GPT-2's qkv / up linears)."""
    from polyaxon_amd.ops import lm

    monkeypatch.setenv("PLX_LM_GEMM", "1")
    x = torch.randn(256, 768, device=cuda, requires_grad=True)
    w = (_rand((2304, 768), cuda, 19).float() * 0.05).to(torch.bfloat16).requires_grad_()
    with torch.autocast("cuda", dtype=torch.bfloat16):
        y = lm.linear(x, w)
    assert y.dtype == torch.bfloat16 and "Mfma" in type(y.grad_fn).__name__
    y.float().sum().backward()
    torch.cuda.synchronize()
    _check(y, x.detach().to(torch.bfloat16).float() @ w.detach().float().t(), 768)
    assert x.grad is not None and x.grad.dtype == torch.float32


@pytest.mark.parametrize("M,N,K", [(512, 3072, 768), (256, 256, 8192)])
def test_gemm256_gelu_epilogue(cuda, M, N, K):
    """gelu_out (plx_gemm256_ex): the epilogue's second store is gelu_tanh of the bf16 output it stored, against
    F.gelu(approximate='tanh') of that output -- one-pass tiles and the split-K reduce."""
    import torch.nn.functional as F

    from polyaxon_amd.ops import gemm

    a = _rand((M, K), cuda, 8)
    b = _rand((N, K), cuda, 9)
    bias = torch.randn(N, device=cuda)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    g = torch.empty_like(h)
    gemm.gemm(a, b, M, N, K, True, True, out=h, bias=bias, gelu_out=g)
    _check(h, a.float() @ b.float().t() + bias, K)
    ref = F.gelu(h.float(), approximate="tanh")
    torch.testing.assert_close(g.float(), ref, rtol=1e-2, atol=1e-2)


@pytest.fixture(params=[1, 0], ids=["split_all", "cost_rule"])
def stream_k(cuda, request):
    """schedule 9 with every partial wave split along K (the split / last-arriver paths on small shapes), and with
    the planner's cost rule (mostly the chained data-parallel loop)"""
    from polyaxon_amd.ops import gemm

    lib = gemm._native.lib("plx_gemm")
    prev, prev_force = gemm.FORCE_SCHEDULE, lib.plx_gemm256_set_sk_force(request.param)
    gemm.FORCE_SCHEDULE = gemm.SK
    yield gemm
    gemm.FORCE_SCHEDULE = prev
    lib.plx_gemm256_set_sk_force(prev_force)


@pytest.mark.parametrize("a_kmajor,b_kmajor", [(True, True), (True, False), (False, True), (False, False)])
@pytest.mark.parametrize("M,N,K", [
    (512, 768, 1408),   # 6 tiles < the CU count: 22 K-tiles in pieces of 4, 2-K-tile pieces across tile boundaries
    (512, 768, 1344),   # 21 K-tiles (odd): the 8-wave kernel runs instead
    (256, 256, 8192),   # one tile over 32 workgroups
    (512, 512, 64),     # one K-tile: the 8-wave kernel
    (4352, 4096, 768),  # 272 tiles = one data-parallel wave + 16 stream-K tiles
    (1536, 4096, 4096),  # 96 tiles, 64 K-tiles: split by the cost rule too
    (8192, 8192, 512),   # 1024 tiles = 4 chained data-parallel tiles per workgroup
])
def test_gemm256_stream_k_matches_fp32(stream_k, cuda, a_kmajor, b_kmajor, M, N, K):
    """Schedule 9 (gemm256_sk_kernel): tile counts that do not divide the persistent grid, pieces that cross tile
    boundaries, every operand layout, against fp32 torch."""
    gemm = stream_k
    g, skt, ipb = gemm.sk_plan(M, N, K)
    assert g >= 1 and 0 <= skt <= (M // 256) * (N // 256) and ipb >= 1
    a = _rand((M, K) if a_kmajor else (K, M), cuda, 21)
    b = _rand((N, K) if b_kmajor else (K, N), cuda, 22)
    out = gemm.gemm(a, b, M, N, K, a_kmajor, b_kmajor)
    af = a.float() if a_kmajor else a.float().t()
    bf = b.float() if b_kmajor else b.float().t()
    torch.cuda.synchronize()
    _check(out, af @ bf.t(), K)


@pytest.mark.parametrize("M,N,K", [(512, 3072, 768), (4352, 4096, 768), (256, 512, 4096)])
def test_gemm256_stream_k_epilogues_deterministic(stream_k, cuda, M, N, K):
    """Bias + GELU on the persistent kernel (data-parallel tiles and last-arriver tiles), alpha, a strided output, and
    30 back-to-back launches bitwise equal: the split tiles' partials are summed in workgroup order whichever
    workgroup arrives last, and the tickets are left zeroed for the next launch."""
    gemm = stream_k
    a, b = _rand((M, K), cuda, 23), _rand((N, K), cuda, 24)
    bias = torch.randn(N, device=cuda)
    h = torch.empty(M, N, dtype=torch.bfloat16, device=cuda)
    g = torch.empty_like(h)
    gemm.gemm(a, b, M, N, K, True, True, out=h, bias=bias, gelu_out=g)
    ref = a.float() @ b.float().t()
    torch.cuda.synchronize()
    _check(h, ref + bias, K)
    torch.testing.assert_close(g.float(), F.gelu(h.float(), approximate="tanh"), rtol=1e-2, atol=1e-2)
    wide = torch.zeros(M, N + 256, dtype=torch.bfloat16, device=cuda)
    gemm.gemm(a, b, M, N, K, True, True, out=wide[:, 256:], alpha=0.5)
    torch.cuda.synchronize()
    _check(wide[:, 256:], 0.5 * ref, K)
    assert wide[:, :256].abs().max().item() == 0
    first = gemm.gemm(a, b, M, N, K, True, True)
    for _ in range(30):
        assert torch.equal(first, gemm.gemm(a, b, M, N, K, True, True))
    tickets = gemm._native.counters(cuda, f"plx_gemm256_sk:{gemm._native.current_stream()}", 1024)
    torch.cuda.synchronize()
    assert int(tickets.abs().sum().item()) == 0


def test_gemm256_stream_k_accumulate_falls_back(stream_k, cuda):
    """accumulate=True under schedule 9 runs the 8-wave kernel's read-modify-write epilogue (same numbers)."""
    gemm = stream_k
    M, N, K = 512, 512, 1024
    a, b = _rand((M, K), cuda, 25), _rand((N, K), cuda, 26)
    c0 = _rand((M, N), cuda, 27)
    out = c0.clone()
    gemm.gemm(a, b, M, N, K, True, True, out=out, accumulate=True)
    torch.cuda.synchronize()
    _check(out, a.float() @ b.float().t() + c0.float(), K)


def test_gemm256_stream_k_in_graph(stream_k, cuda):
    """Captured into a hipGraph and replayed: the tickets the kernel resets make every replay start from zero."""
    gemm = stream_k
    M, N, K = 512, 768, 1408
    a, b = _rand((M, K), cuda, 28), _rand((N, K), cuda, 29)
    out = gemm.gemm(a, b, M, N, K, True, True)  # warm: workspace + tickets allocated outside the capture
    ref = out.clone()
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.stream(s):
        with torch.cuda.graph(graph, stream=s):
            gemm.gemm(a, b, M, N, K, True, True, out=out)
    torch.cuda.current_stream().wait_stream(s)
    for _ in range(5):
        out.zero_()
        graph.replay()
        torch.cuda.synchronize()
        assert torch.equal(out, ref)


def _gelu_grad_ref(h):
    """d/dh gelu_tanh(h) in fp32 (torch's own formula, through autograd)"""
    hh = h.float().detach().requires_grad_()
    F.gelu(hh, approximate="tanh").sum().backward()
    return hh.grad


def test_gemm256_stream_k_gelu_backward_epilogue(stream_k, cuda):
    """gelu_h: the data gradient's epilogue stores bf16(dy . W) * gelu_tanh'(h) -- against the fp32 chain, and against
    the separate pass it replaces (the stored bf16 data gradient, then plx_gelu_bwd_colsum's dh) to one bf16 rounding
    step: the same formula, but the two kernels' instruction sequences may differ in the last fp32 bit before the
    bf16 rounding."""
    gemm = stream_k
    from polyaxon_amd.ops import lm

    T, d, d_ff = 512, 768, 3072
    dy = _rand((T, d), cuda, 31)
    w = (_rand((d, d_ff), cuda, 32).float() * 0.05).to(torch.bfloat16)  # W_down [out = d][in = d_ff]
    h = _rand((T, d_ff), cuda, 33)
    dh = gemm.gemm(dy, w, T, d_ff, d, True, False, gelu_h=h)
    da = gemm.gemm(dy, w, T, d_ff, d, True, False)  # the unfused data gradient
    torch.cuda.synchronize()
    ref = (dy.float() @ w.float()) * _gelu_grad_ref(h)
    _check(dh, ref, d)
    b = torch.zeros(d_ff, device=cuda, requires_grad=True)
    dh2, _ = lm.bias_grad(da, b, gelu_h=h)  # the separate pass
    torch.cuda.synchronize()
    diff = (dh.float() - dh2.float()).abs()
    assert bool((diff <= dh2.float().abs() * 2.0 ** -7 + 1e-30).all()), diff.max().item()
    assert (diff > 0).float().mean().item() < 0.01
    with pytest.raises(ValueError):
        gemm.gemm(dy, w, T, d_ff, d, True, False, gelu_h=h, bias=torch.zeros(d_ff, device=cuda))


@pytest.mark.parametrize("T", [512, 16384])
def test_gelu_mlp_fused_backward_matches_fp32(cuda, monkeypatch, T):
    """ops.lm.gelu_mlp (GPT-2's MLP as one op, the GELU backward in the down-projection's data-gradient epilogue):
    output, dx, both weight and bias gradients against fp32 autograd of linear -> gelu_tanh -> linear.  T = 16384 is
    GPT-2's bs 16 x 1024 (the table routes its down-projection data gradient to the stream-K schedule); T = 512
    forces that schedule through PLX_LM_GEMM=1 and PLX_GEMM_WAVES=9."""
    from polyaxon_amd.ops import lm

    monkeypatch.setenv("PLX_LM_GEMM", "auto")
    if T != 16384:  # every GEMM on the kernel, the stream-K schedule outside the table
        monkeypatch.setenv("PLX_LM_GEMM", "1")
        monkeypatch.setenv("PLX_GEMM_WAVES", "9")
    d, d_ff = 768, 3072
    x = _rand((T, d), cuda, 34).requires_grad_()
    wu = (_rand((d_ff, d), cuda, 35).float() * 0.03).to(torch.bfloat16).requires_grad_()
    bu = (_rand((d_ff,), cuda, 36).float() * 0.1).to(torch.bfloat16).requires_grad_()
    wd = (_rand((d, d_ff), cuda, 37).float() * 0.03).to(torch.bfloat16).requires_grad_()
    bd = (_rand((d,), cuda, 38).float() * 0.1).to(torch.bfloat16).requires_grad_()
    y = lm.gelu_mlp(x, wu, bu, wd, bd)
    assert "GeluMlpMfma" in type(y.grad_fn).__name__
    dy = _rand((T, d), cuda, 39)
    y.backward(dy)
    ref = [t.detach().float().requires_grad_() for t in (x, wu, bu, wd, bd)]
    yr = F.linear(F.gelu(F.linear(ref[0], ref[1], ref[2]), approximate="tanh"), ref[3], ref[4])
    yr.backward(dy.float())
    torch.cuda.synchronize()
    _check(y, yr.detach(), d_ff)
    _check(x.grad, ref[0].grad, d_ff)
    _check(wu.grad, ref[1].grad, T)
    _check(wd.grad, ref[3].grad, T)
    # bias gradients: column sums of T bf16-rounded gradient rows, so the error grows like sqrt(T): relative to scale
    _check(bu.grad, ref[2].grad, T)
    _check(bd.grad, ref[4].grad, T)
