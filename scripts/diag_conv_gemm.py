"""Time the ResNet-50 1x1 convolutions: MIOpen (F.conv2d fwd+bwd) vs the plx MFMA GEMM op, per pass.

Interleaved rounds in one process (guide §5.4 rule 24); random bf16 data; CUDA events."""
import sys

import torch
import torch.nn.functional as F

from polyaxon_amd.ops.conv1x1 import conv1x1, gemm_nt, gemm_tn, weight_prep

dev = torch.device("cuda", 0)
SHAPES = [(256, 64, 56, 56, 256), (256, 256, 56, 56, 64), (256, 64, 56, 56, 64), (256, 512, 28, 28, 128),
          (256, 128, 28, 28, 512), (256, 1024, 14, 14, 256), (256, 256, 14, 14, 1024), (256, 2048, 7, 7, 512),
          (256, 512, 7, 7, 2048)]


def timeit(fn, it=10):
    fn()
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    s.record()
    for _ in range(it):
        fn()
    e.record()
    torch.cuda.synchronize()
    return s.elapsed_time(e) / it


def main():
    tot = {"miopen": 0.0, "plx": 0.0}
    for n, cin, h, w, cout in SHAPES:
        x = torch.randn(n, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt32 = torch.randn(cout, cin, 1, 1, device=dev) * 0.05
        g = torch.randn(n, cout, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        xm = x.clone().requires_grad_()
        wm = wt32.to(torch.bfloat16).contiguous(memory_format=torch.channels_last).requires_grad_()
        xp = x.clone().requires_grad_()
        wp = wt32.clone().requires_grad_()

        def miopen():
            xm.grad = None
            wm.grad = None
            F.conv2d(xm, wm).backward(g)

        def plx():
            xp.grad = None
            wp.grad = None
            conv1x1(xp, wp).backward(g)

        m = n * h * w
        xr = x.permute(0, 2, 3, 1).reshape(m, cin)
        gr = g.permute(0, 2, 3, 1).reshape(m, cout)
        wb, wtt = weight_prep(wt32)
        parts = {"fwd": lambda: gemm_nt(xr, wb), "dgrad": lambda: gemm_nt(gr, wtt), "wgrad": lambda: gemm_tn(gr, xr)}
        res = {"miopen": [], "plx": []}
        for _ in range(3):
            res["miopen"].append(timeit(miopen))
            res["plx"].append(timeit(plx))
        a, b = min(res["miopen"]), min(res["plx"])
        tot["miopen"] += a
        tot["plx"] += b
        pt = {k: timeit(f) for k, f in parts.items()}
        fl = 3 * 2 * m * cin * cout
        byts = 2 * (2 * m * cin + 3 * m * cout)  # fwd: x r, y w; dgrad: dy r, dx w; wgrad: dy r, x r (+y rewritten)
        # correctness spot check vs MIOpen result
        torch.testing.assert_close(xp.grad.float(), xm.grad.float(), rtol=5e-2, atol=1.0)
        print(f"{(n, cin, h, w, cout)}  miopen {a:.3f} ms  plx {b:.3f} ms  ({b / a:.2f}x)  "
              f"plx {fl / b / 1e9:.0f} TF  parts " + " ".join(f"{k}={v:.3f}" for k, v in pt.items())
              + f"  roofline~{byts / 6.3e9:.3f} ms", flush=True)
    print(f"total miopen {tot['miopen']:.3f} ms  plx {tot['plx']:.3f} ms")
    conv3()


def conv3():
    """3x3 stride-1 convs of ResNet-50: MIOpen vs the implicit-GEMM kernels (kernel time per pass)."""
    from polyaxon_amd.ops import _native
    from polyaxon_amd.ops.conv1x1 import _num_cus, _stream, _zero_page
    from polyaxon_amd.ops.conv import weight_prep_k

    lib = _native.lib("plx_conv")
    for n, c, h, w in [(256, 64, 56, 56), (256, 128, 28, 28), (256, 256, 14, 14), (256, 512, 7, 7)]:
        x = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(c, c, 3, 3, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        g = torch.randn(n, c, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        xm = x.clone().requires_grad_()
        wm = wt.to(torch.bfloat16).requires_grad_()

        def miopen():
            xm.grad = None
            wm.grad = None
            F.conv2d(xm, wm, padding=1).backward(g)

        wf, wd = weight_prep_k(wt)
        y = torch.empty_like(x)
        dx = torch.empty_like(x)
        z = _zero_page(dev).data_ptr()
        cus = _num_cus(dev)
        ws = torch.empty(int(lib.plx_conv_wgrad_workspace(n, h, w, c, c, 3, 1, cus)), device=dev)
        dw = torch.empty(c, 9, c, device=dev)
        parts = {
            "fwd": lambda: lib.plx_conv_fwd(x.data_ptr(), wf.data_ptr(), y.data_ptr(), n, h, w, c, c, 3, 1, z, None,
                                            _stream()),
            "dgrad": lambda: lib.plx_conv_dgrad(g.data_ptr(), wd.data_ptr(), dx.data_ptr(), n, h, w, c, c, 3, 1, z,
                                                _stream()),
            "wgrad": lambda: lib.plx_conv_wgrad(g.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(), n, h, w,
                                                c, c, 3, 1, z, cus, 0, _stream()),
        }
        a = min(timeit(miopen) for _ in range(3))
        pt = {k: min(timeit(f) for _ in range(2)) for k, f in parts.items()}
        fl = 2 * n * h * w * c * c * 9
        print(f"3x3 {(n, c, h, w)}  miopen fwd+bwd {a:.3f} ms  plx " +
              " ".join(f"{k}={v:.3f}({fl / v / 1e9:.0f}TF)" for k, v in pt.items()) + f"  sum {sum(pt.values()):.3f}",
              flush=True)


def strided():
    """Strided convs of ResNet-50 (3x3 s2 in conv2 of each stage's first block, 1x1 s2 downsample):
    MIOpen fwd+bwd vs the implicit-GEMM passes."""
    from polyaxon_amd.ops import _native
    from polyaxon_amd.ops.conv import weight_prep_k
    from polyaxon_amd.ops.conv1x1 import _num_cus, _stream, _zero_page

    lib = _native.lib("plx_conv")
    for n, cin, h, w, cout, k in [(256, 128, 56, 56, 128, 3), (256, 256, 28, 28, 256, 3), (256, 512, 14, 14, 512, 3),
                                  (256, 256, 56, 56, 512, 1), (256, 512, 28, 28, 1024, 1),
                                  (256, 1024, 14, 14, 2048, 1)]:
        ho, wo = (h + 2 * (k // 2) - k) // 2 + 1, (w + 2 * (k // 2) - k) // 2 + 1
        x = torch.randn(n, cin, h, w, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        wt = (torch.randn(cout, cin, k, k, device=dev) * 0.05).contiguous(memory_format=torch.channels_last)
        g = torch.randn(n, cout, ho, wo, device=dev).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        xm = x.clone().requires_grad_()
        wm = wt.to(torch.bfloat16).requires_grad_()

        def miopen():
            xm.grad = None
            wm.grad = None
            F.conv2d(xm, wm, stride=2, padding=k // 2).backward(g)

        wf, wd = weight_prep_k(wt)
        y = torch.empty(n, cout, ho, wo, device=dev, dtype=torch.bfloat16)
        dx = torch.zeros_like(x)
        z = _zero_page(dev).data_ptr()
        cus = _num_cus(dev)
        ws = torch.empty(int(lib.plx_conv_wgrad_workspace(n, h, w, cin, cout, k, 2, cus)), device=dev)
        dw = torch.empty(cout, k * k, cin, device=dev)
        parts = {
            "fwd": lambda: lib.plx_conv_fwd(x.data_ptr(), wf.data_ptr(), y.data_ptr(), n, h, w, cin, cout, k, 2, z,
                                            None, _stream()),
            "dgrad": lambda: lib.plx_conv_dgrad(g.data_ptr(), wd.data_ptr(), dx.data_ptr(), n, h, w, cin, cout, k, 2,
                                                z, _stream()),
            "wgrad": lambda: lib.plx_conv_wgrad(g.data_ptr(), x.data_ptr(), dw.data_ptr(), ws.data_ptr(), n, h, w,
                                                cin, cout, k, 2, z, cus, 0, _stream()),
        }
        a = min(timeit(miopen) for _ in range(3))
        pt = {kk: min(timeit(f) for _ in range(2)) for kk, f in parts.items()}
        print(f"s2 k{k} {(n, cin, h, w, cout)}  miopen fwd+bwd {a:.3f} ms  plx " +
              " ".join(f"{kk}={v:.3f}" for kk, v in pt.items()) + f"  sum {sum(pt.values()):.3f}", flush=True)


if __name__ == "__main__":
    if "--strided" in sys.argv:
        strided()
    else:
        main()
