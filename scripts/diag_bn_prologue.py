"""Price the BatchNorm-apply prologue fusion on the ResNet-50 1x1 consumers of bn2 (each bottleneck's conv3).

Today: bn2's apply pass writes relu(bn2(x)) (read + write of [M, C]) and conv3 reads it.  Fused: conv3's NT GEMM
applies scale / bias / ReLU to its A fragments (csrc/conv_gemm.hip MODE 4, plx_gemm_nt_prologue) and the apply pass
disappears.  Per layer this prints the GEMM time with and without the prologue (both with the fused BN3 statistics
epilogue) and the apply pass it would remove; plus a numerics check of the prologue against the materialised path.
(Forward only: the backward would also need the activation recomputed in the weight-gradient GEMM and the ReLU
mask recomputed in the BN backward -- priced separately if the forward pays.)"""
import json
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))

import torch

from polyaxon_amd.ops import _native


def timed(fn, reps=20):
    for _ in range(3):
        fn()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(reps):
        fn()
    e1.record()
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps * 1e3  # us


def main():
    dev = torch.device("cuda", 0)
    conv, bn = _native.lib("plx_conv"), _native.lib("plx_bn")
    st = torch.cuda.current_stream().cuda_stream
    zero = torch.zeros(1 << 16, dtype=torch.bfloat16, device=dev)
    out = []
    for name, M, C in (("layer1", 256 * 56 * 56, 64), ("layer2", 256 * 28 * 28, 128), ("layer3", 256 * 14 * 14, 256),
                       ("layer4", 256 * 7 * 7, 512)):
        N = 4 * C
        g = torch.Generator(device=dev).manual_seed(C)
        x = torch.randn(M, C, device=dev, generator=g).to(torch.bfloat16)
        w = (torch.randn(N, C, device=dev, generator=g) * C ** -0.5).to(torch.bfloat16)
        scale = torch.rand(C, device=dev, generator=g) + 0.5
        bias = torch.randn(C, device=dev, generator=g) * 0.5
        sb = torch.cat([scale, bias]).contiguous()
        y = torch.empty_like(x)
        c_plain = torch.empty(M, N, dtype=torch.bfloat16, device=dev)
        c_pro = torch.empty_like(c_plain)
        rows = conv.plx_gemm_nt_rows_per_block(N)
        stats = torch.empty(2 * ((M + rows - 1) // rows) * N, dtype=torch.float32, device=dev)

        def apply():
            _native.check(bn.plx_bn_apply(x.data_ptr(), None, y.data_ptr(), M, C, sb.data_ptr(), 1, st), "apply")

        def plain():
            rc = conv.plx_gemm_nt(y.data_ptr(), w.data_ptr(), c_plain.data_ptr(), M, N, C, C, C, N, zero.data_ptr(),
                                  stats.data_ptr(), None, 0, None, None, st)
            assert rc == 0, rc

        def pro():
            rc = conv.plx_gemm_nt_prologue(x.data_ptr(), w.data_ptr(), c_pro.data_ptr(), M, N, C, C, C, N,
                                           zero.data_ptr(), scale.data_ptr(), bias.data_ptr(), stats.data_ptr(), st)
            assert rc == 0, rc

        apply()
        plain()
        pro()
        torch.cuda.synchronize()
        err = float((c_pro.float() - c_plain.float()).abs().max() / c_plain.float().abs().max())
        t_apply, t_plain, t_pro = timed(apply), timed(plain), timed(pro)
        r = {"layer": name, "M": M, "K": C, "N": N, "apply_us": round(t_apply, 1), "gemm_us": round(t_plain, 1),
             "gemm_prologue_us": round(t_pro, 1), "fused_saves_us": round(t_apply + t_plain - t_pro, 1),
             "rel_err_vs_materialised": round(err, 4)}
        out.append(r)
        print(json.dumps(r), flush=True)
    blocks = {"layer1": 3, "layer2": 4, "layer3": 6, "layer4": 3}
    print(json.dumps({"forward_saving_us_per_step": round(sum(r["fused_saves_us"] * blocks[r["layer"]] for r in out),
                                                          1)}))


if __name__ == "__main__":
    main()
