"""Host-side contract of the LM GEMM path (ops/gemm.py, ops/lm.py): shape gating, fallbacks, argument checks.
The kernel's numerics are in tests/test_gpu_gemm.py."""
import pytest
import torch
import torch.nn.functional as F

from polyaxon_amd.ops import gemm, lm


def test_supported_shapes():
    assert gemm.supported(4096, 6144, 4096)
    assert gemm.supported(256, 256, 64)
    assert not gemm.supported(4096, 50257, 768)  # GPT-2 vocab: not a multiple of 256
    assert not gemm.supported(4096, 768, 96)     # K not a multiple of 64
    assert not gemm.supported(0, 256, 64)


def test_linear_supported_needs_cuda_bf16_and_tiles():
    x = torch.zeros(2, 128, 768, dtype=torch.bfloat16)
    w = torch.zeros(2304, 768, dtype=torch.bfloat16)
    assert not gemm.linear_supported(x, w)  # CPU tensors never take the kernel


def test_linear_on_cpu_is_f_linear():
    torch.manual_seed(0)
    x = torch.randn(3, 5, 16, requires_grad=True)
    w = torch.randn(8, 16, requires_grad=True)
    b = torch.randn(8, requires_grad=True)
    y = lm.linear(x, w, b)
    torch.testing.assert_close(y, F.linear(x, w, b))
    y.sum().backward()
    assert x.grad is not None and w.grad is not None and b.grad is not None


def test_gemm_rejects_bad_shapes_before_launch():
    a = torch.zeros(256, 64, dtype=torch.bfloat16)
    b = torch.zeros(256, 64, dtype=torch.bfloat16)
    with pytest.raises(ValueError):
        gemm.gemm(a, b, 256, 256, 96, True, True)
    with pytest.raises(ValueError):
        gemm.gemm(a.float(), b, 256, 256, 64, True, True)
    with pytest.raises(ValueError):
        gemm.gemm(a, b, 256, 256, 64, True, True, accumulate=True)


def test_knob_modes(monkeypatch):
    monkeypatch.setenv("PLX_LM_GEMM", "0")
    assert not gemm.enabled() and gemm.mode() == "0"
    monkeypatch.setenv("PLX_LM_GEMM", "1")
    assert gemm.enabled() and gemm.mode() == "1"
    monkeypatch.delenv("PLX_LM_GEMM")
    assert gemm.mode() == "auto" and gemm.enabled()
    monkeypatch.setenv("PLX_LM_GEMM", "bogus")
    assert gemm.mode() == "auto"


def test_torch_path_layouts_match_reference():
    """The hipBLASLt side of the dispatch (here on CPU) computes the same layouts as the kernel contract."""
    torch.manual_seed(0)
    M, N, K = 8, 6, 4
    a_k, b_k = torch.randn(M, K), torch.randn(N, K)
    ref = a_k @ b_k.t()
    for ak in (True, False):
        for bk in (True, False):
            a = a_k.contiguous() if ak else a_k.t().contiguous()
            b = b_k.contiguous() if bk else b_k.t().contiguous()
            torch.testing.assert_close(gemm._torch_gemm(a, b, M, N, K, ak, bk), ref)
            out = torch.ones(M, N)
            gemm._torch_gemm(a, b, M, N, K, ak, bk, out=out, accumulate=True)
            torch.testing.assert_close(out, ref + 1)


def test_auto_dispatch_is_a_pure_function_of_the_shape(monkeypatch):
    """``auto``: the measured table's shapes on the kernel with their schedule, any other split-K shape on the kernel
    (schedule 0 = library default), the rest on hipBLASLt (-1).  No timing, no CUDA call: reproducible across runs
    and identical on every DP rank."""
    monkeypatch.setenv("PLX_LM_GEMM", "auto")
    assert set(gemm.SCHEDULE.values()) <= {4, 5, 6, 7, 8, 9}
    assert gemm.schedule(2304, 768, 16384, False, False) == 5      # GPT-2 qkv wgrad (split-K)
    assert gemm.schedule(50432, 768, 16384, False, False) == 5     # GPT-2 tied head wgrad
    assert gemm.schedule(16384, 768, 3072, True, True) == 9        # GPT-2 down fwd: stream-K
    assert gemm.schedule(16384, 768, 50432, True, False) == 5      # GPT-2 head dgrad: 4-wave
    assert gemm.schedule(16384, 768, 2304, True, False) == 9       # GPT-2 qkv dgrad (192 tiles): stream-K
    # the whole GPT-2 125M step (bs 16 x 1024) is on the kernel
    for fin, fout in ((768, 2304), (768, 768), (768, 3072), (3072, 768), (768, 50432)):
        assert gemm.schedule(16384, fout, fin, True, True) >= 0
        assert gemm.schedule(16384, fin, fout, True, False) >= 0
        assert gemm.schedule(fout, fin, 16384, False, False) >= 0
    assert gemm.schedule(4096, 3072, 768, True, True) == -1        # the same linear at another token count
    assert gemm.schedule(4096, 28672, 4096, True, True) == -1      # Llama up fwd: hipBLASLt
    assert gemm.schedule(28672, 4096, 4096, False, False) == 5     # Llama up wgrad
    assert gemm.splits(256, 256, 8192) > 1 and gemm.schedule(256, 256, 8192, False, False) == 0
    assert gemm.splits(4096, 4096, 512) == 1 and gemm.schedule(4096, 4096, 512, True, True) == -1
    for (M, N, K, ak, bk) in gemm.SCHEDULE:
        assert gemm.supported(M, N, K)
    gemm._seen.clear()
    assert gemm._use_native(2304, 768, 16384, False, False) and not gemm._use_native(4096, 3072, 768, True, True)
    d = gemm.decisions()
    assert d["2304x768x16384:MN"] == {"native": True, "schedule": 5} and d["4096x3072x768:KK"]["native"] is False
    gemm._seen.clear()


def test_stream_k_plan_and_routing(monkeypatch):
    """Schedule 9's host side on the CPU (the planner and the routing; no launch): the partial wave is split along K
    only for long reductions whose split saves >= 16 K-tiles per workgroup, pieces are even for an even K-tile count,
    odd / short K and accumulating calls fall back to the 8-wave kernel, PLX_GEMM_WAVES=9 selects it."""
    lib = gemm._native.lib("plx_gemm")
    prev = lib.plx_gemm256_set_sk_force(0)
    try:
        g, skt, ipb = gemm.sk_plan(4096, 6144, 4096)     # Llama QKV forward: 384 tiles, 64 K-tiles
        assert skt == 384 % g and ipb % 2 == 0 and 4 <= ipb <= 64 - 16
        g, skt, ipb = gemm.sk_plan(16384, 50432, 768)    # GPT-2 head: K too short to split
        assert skt == 0 and ipb == 1
        g, skt, ipb = gemm.sk_plan(4096, 4096, 4096)     # a full wave on a 256-CU chip: nothing to split
        assert (skt == 0) == (256 % g == 0)
        lib.plx_gemm256_set_sk_force(1)                  # tests split every partial wave
        g, skt, ipb = gemm.sk_plan(512, 768, 1408)
        assert skt == 6 and ipb >= 4 and ipb % 2 == 0
    finally:
        lib.plx_gemm256_set_sk_force(prev)
    # the workspace is sized for any plan of the shape (memoised sizes stay valid when the force knob changes)
    assert gemm._native.size("plx_gemm", "plx_gemm256_sk_ws", 512, 768, 1408) > 0
    # shape checks happen before any device call: odd / short K is refused, ops/gemm.py runs schedule 8 instead
    assert lib.plx_gemm256_sk(None, None, None, None, None, 512, 768, 1344, 1344, 1344, 768, 1, 1, 1.0, None, None,
                              None, None) == -1
    # the fused GELU backward is refused with a bias (before any device call)
    assert lib.plx_gemm256_sk(None, None, None, None, None, 512, 768, 1408, 1408, 1408, 768, 1, 0, 1.0, 16, None, 16,
                              None) == -1
    assert not gemm.gelu_bwd_supported(512, 3072, 96)
    assert not gemm.sk_supported(512, 768, 1344) and not gemm.sk_supported(512, 512, 128)
    assert gemm.sk_supported(512, 768, 1408) and gemm.sk_supported(16384, 50432, 768)
    monkeypatch.setattr(gemm, "FORCE_SCHEDULE", 0)
    monkeypatch.delenv("PLX_GEMM_WAVES", raising=False)
    # outside the table (4096 tokens): the layout defaults, or the PLX_GEMM_WAVES override
    assert gemm._schedule_of(4096, 3072, 768, True, True) == gemm.SK       # forward layout default
    assert gemm._schedule_of(4096, 768, 3072, True, False) == 5            # data gradient
    monkeypatch.setenv("PLX_GEMM_WAVES", "9")
    assert gemm._schedule_of(4096, 768, 3072, True, False) == gemm.SK
    monkeypatch.setenv("PLX_GEMM_WAVES", "8")
    assert gemm._schedule_of(4096, 3072, 768, True, True) == 0             # the library's global knob
    assert gemm._schedule_of(16384, 3072, 768, True, True) == gemm.SK      # the table wins over the override
