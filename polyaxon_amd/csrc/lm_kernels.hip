// Fused elementwise/layout kernels of the decoder-only language models (Llama-3 8B, GPT-2) on MI355X.
//
//   plx_qkv_rope_fwd   qkv[T][(H+2KV)*D] (the fused QKV GEMM's output, T = B*S rows)
//                        -> q[B][H][S][D], k[B][KV][S][D] rotated by RoPE, v[B][KV][S][D]
//                      one pass instead of split / view / transpose / 2x(cat, 4 mul, add, sub) / contiguous:
//                      the rotation is fused into the head-major relayout attention wants.
//   plx_qkv_rope_bwd   dq, dk, dv -> dqkv[T][(H+2KV)*D] (inverse rotation + the transpose back)
//   plx_swiglu_fwd     h[T][2F] (gate | up halves of the fused gate/up GEMM) -> a[T][F] = silu(g) * u
//   plx_swiglu_bwd     da, h -> dh[T][2F]: dg = da*u*silu'(g), du = da*silu(g)
//   plx_xent_fwd       next-token cross entropy from bf16 logits [B][S][V]: per row (b, s < S-1) the log-sum-exp
//                      (online max / sum over 16-byte chunks, one workgroup per row) and loss = lse - x[target]
//   plx_xent_bwd       dlogits[B][S][V] (bf16) = (softmax - onehot(target)) * dloss / rows, zero rows at s = S-1
//   plx_xent_cls_*     the same pair for classification logits [N][V] and labels [N] (the ResNet head)
//                      -- replaces slice copy + fp32 cast + log_softmax + NLL and their backward chain (~5.5 ms of
//                      a 37 ms GPT-2 125M step: vocab 50257 x 16k tokens through fp32 twice)
//   plx_colsum         bias gradients: out[N] = sum over rows of a bf16 [T][N] matrix, fp32 accumulation, one launch
//                      (64-column tiles x row splits, fp32 partials, last-arriving split reduces them in a fixed
//                      order: deterministic).  The generic column reduction it replaces ran ~26 us per GPT-2 bias at
//                      16k tokens, several times the 25-100 MB read.
//   plx_gelu_bwd_colsum GPT-2 MLP: dh = dA * gelu_tanh'(h) and the up-projection's bias gradient (column sums of
//                      dh) in one pass -- replaces the activation-backward kernel plus a separate read of dh.
//
// Llama RoPE convention (rotate the two halves of each head): for j < D/2
//   y[j] = x[j] c_j - x[j+D/2] s_j,  y[j+D/2] = x[j] s_j + x[j+D/2] c_j,  c_j = cos(pos * theta^(-2j/D)).
// cos / sin come from an fp32 [S][D/2] table.  `rot_heads` = number of leading heads that rotate (H + KV for
// RoPE models, 0 for GPT-2's learned positions: the kernel is then the pure relayout).
//
// Memory-bound: every lane moves 16-byte vectors (8 bf16) and computes in fp32; a lane owns one 8-wide chunk of
// the first half of a head row and the matching chunk of the second half, so the pair it rotates is in
// registers.  Grid-strided, 256-thread blocks, capped at 8192 blocks (>> 256 CUs x 8 waves).
#include <hip/hip_runtime.h>

#include "handoff.h"
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kBlock = 256;

struct alignas(16) bf16x8 {
  uint16_t v[8];
};

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // hardware RNE conversion, NaN stays NaN
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

inline int grid_for(int64_t items) {
  int64_t g = (items + kBlock - 1) / kBlock;
  if (g > 8192) g = 8192;
  if (g < 1) g = 1;
  return (int)g;
}

// work item i -> (row t, head h, chunk c of the first half); head-major destination row (b, h, s)
__global__ __launch_bounds__(kBlock) void qkv_rope_fwd_kernel(const bf16x8* __restrict__ qkv,
                                                              const float* __restrict__ cosv,
                                                              const float* __restrict__ sinv,
                                                              bf16x8* __restrict__ q, bf16x8* __restrict__ k,
                                                              bf16x8* __restrict__ v, int64_t T, int S, int H,
                                                              int KV, int D, int rot_heads) {
  const int NH = H + 2 * KV, half8 = D / 16, row8 = D / 8;
  const int64_t items = T * NH * half8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += stride) {
    const int c = (int)(i % half8);
    const int64_t th = i / half8;
    const int h = (int)(th % NH);
    const int64_t t = th / NH;
    const int s = (int)(t % S);
    const int64_t b = t / S;
    const bf16x8* src = qkv + (t * NH + h) * row8;
    bf16x8 x1 = src[c], x2 = src[c + half8];
    if (h < rot_heads) {
      const float* cs = cosv + (int64_t)s * (D / 2) + c * 8;
      const float* sn = sinv + (int64_t)s * (D / 2) + c * 8;
      bf16x8 y1, y2;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = bf2f(x1.v[e]), bb = bf2f(x2.v[e]), co = cs[e], si = sn[e];
        y1.v[e] = f2bf(a * co - bb * si);
        y2.v[e] = f2bf(a * si + bb * co);
      }
      x1 = y1;
      x2 = y2;
    }
    bf16x8* dst;
    if (h < H) {
      dst = q + ((b * H + h) * S + s) * row8;
    } else if (h < H + KV) {
      dst = k + ((b * KV + (h - H)) * S + s) * row8;
    } else {
      dst = v + ((b * KV + (h - H - KV)) * S + s) * row8;
    }
    dst[c] = x1;
    dst[c + half8] = x2;
  }
}

__global__ __launch_bounds__(kBlock) void qkv_rope_bwd_kernel(const bf16x8* __restrict__ dq,
                                                              const bf16x8* __restrict__ dk,
                                                              const bf16x8* __restrict__ dv,
                                                              const float* __restrict__ cosv,
                                                              const float* __restrict__ sinv,
                                                              bf16x8* __restrict__ dqkv, int64_t T, int S, int H,
                                                              int KV, int D, int rot_heads) {
  const int NH = H + 2 * KV, half8 = D / 16, row8 = D / 8;
  const int64_t items = T * NH * half8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += stride) {
    const int c = (int)(i % half8);
    const int64_t th = i / half8;
    const int h = (int)(th % NH);
    const int64_t t = th / NH;
    const int s = (int)(t % S);
    const int64_t b = t / S;
    const bf16x8* src;
    if (h < H) {
      src = dq + ((b * H + h) * S + s) * row8;
    } else if (h < H + KV) {
      src = dk + ((b * KV + (h - H)) * S + s) * row8;
    } else {
      src = dv + ((b * KV + (h - H - KV)) * S + s) * row8;
    }
    bf16x8 g1 = src[c], g2 = src[c + half8];
    if (h < rot_heads) {  // transpose of the rotation: [c s; -s c]
      const float* cs = cosv + (int64_t)s * (D / 2) + c * 8;
      const float* sn = sinv + (int64_t)s * (D / 2) + c * 8;
      bf16x8 y1, y2;
#pragma unroll
      for (int e = 0; e < 8; ++e) {
        const float a = bf2f(g1.v[e]), bb = bf2f(g2.v[e]), co = cs[e], si = sn[e];
        y1.v[e] = f2bf(a * co + bb * si);
        y2.v[e] = f2bf(bb * co - a * si);
      }
      g1 = y1;
      g2 = y2;
    }
    bf16x8* dst = dqkv + (t * NH + h) * row8;
    dst[c] = g1;
    dst[c + half8] = g2;
  }
}

__device__ __forceinline__ float sigmoidf(float x) { return 1.f / (1.f + __expf(-x)); }

__global__ __launch_bounds__(kBlock) void swiglu_fwd_kernel(const bf16x8* __restrict__ h, bf16x8* __restrict__ a,
                                                            int64_t T, int F8) {
  const int64_t items = T * F8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += stride) {
    const int64_t t = i / F8;
    const int c = (int)(i - t * F8);
    const bf16x8 g = h[t * 2 * F8 + c], u = h[t * 2 * F8 + F8 + c];
    bf16x8 o;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gf = bf2f(g.v[e]);
      o.v[e] = f2bf(gf * sigmoidf(gf) * bf2f(u.v[e]));
    }
    a[i] = o;
  }
}

__global__ __launch_bounds__(kBlock) void swiglu_bwd_kernel(const bf16x8* __restrict__ da,
                                                            const bf16x8* __restrict__ h,
                                                            bf16x8* __restrict__ dh, int64_t T, int F8) {
  const int64_t items = T * F8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < items; i += stride) {
    const int64_t t = i / F8;
    const int c = (int)(i - t * F8);
    const bf16x8 g = h[t * 2 * F8 + c], u = h[t * 2 * F8 + F8 + c], d = da[i];
    bf16x8 dg, du;
#pragma unroll
    for (int e = 0; e < 8; ++e) {
      const float gf = bf2f(g.v[e]), uf = bf2f(u.v[e]), df = bf2f(d.v[e]);
      const float sg = sigmoidf(gf), si = gf * sg;
      du.v[e] = f2bf(df * si);
      dg.v[e] = f2bf(df * uf * sg * (1.f + gf * (1.f - sg)));
    }
    dh[t * 2 * F8 + c] = dg;
    dh[t * 2 * F8 + F8 + c] = du;
  }
}


// ------------------------------------------------------------------------------------------- cross entropy
// Rows of V bf16 at an element stride of V: with V odd a row starts anywhere inside a 16-byte chunk, so a row is
// walked as the aligned chunks that cover it (head = misalignment in elements) and elements outside [0, V) are
// masked; the backward stores whole chunks inside the row and single elements in the two edge chunks (a chunk
// shared with the neighbouring row is never written as a whole).
constexpr float kNegInf = -__builtin_huge_valf();

__device__ __forceinline__ void lse_combine(float& m, float& s, float m2, float s2) {
  const float mn = fmaxf(m, m2);
  if (mn == kNegInf) return;
  s = s * __expf(m - mn) + s2 * __expf(m2 - mn);
  m = mn;
}

// CLS: classification rows instead of next-token positions -- logits [N][V], target labels[r] of row r (the
// ResNet head's cross entropy, ops/lm.py class_xent); S is unused then
template <bool CLS = false>
__global__ __launch_bounds__(kBlock) void xent_fwd_kernel(const uint16_t* __restrict__ logits,
                                                          const int64_t* __restrict__ tokens, float* __restrict__ lse,
                                                          float* __restrict__ loss, int S, int V) {
  const int r = blockIdx.x;                      // loss row: (b, s), s < S - 1
  const int b = CLS ? r : r / (S - 1), s = CLS ? 0 : r - b * (S - 1);
  const int64_t lrow = CLS ? (int64_t)r : (int64_t)b * S + s;
  const uint16_t* row = logits + lrow * V;
  const uintptr_t p0 = (uintptr_t)row;
  const bf16x8* base = (const bf16x8*)(p0 & ~(uintptr_t)15);
  const int head = (int)((p0 & 15) >> 1);
  const int nch = (head + V + 7) >> 3;
  float m = kNegInf, sum = 0.f;
  // 4 chunks (64 bytes) per lane in flight per trip: one load per trip left the row walk latency-bound (~3.9 TB/s)
  for (int c0 = threadIdx.x; c0 < nch; c0 += 4 * kBlock) {
    bf16x8 v[4];
#pragma unroll
    for (int u = 0; u < 4; ++u) {
      const int c = c0 + u * kBlock;
      v[u] = c < nch ? base[c] : bf16x8{};
    }
    float x[4][8], cm = kNegInf;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = (c0 + u * kBlock) * 8 + j - head;
        x[u][j] = (e >= 0 && e < V) ? bf2f(v[u].v[j]) : kNegInf;
        cm = fmaxf(cm, x[u][j]);
      }
    if (cm == kNegInf) continue;
    float cs = 0.f;
#pragma unroll
    for (int u = 0; u < 4; ++u)
#pragma unroll
      for (int j = 0; j < 8; ++j) cs += __expf(x[u][j] - cm);
    lse_combine(m, sum, cm, cs);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) lse_combine(m, sum, __shfl_xor(m, off), __shfl_xor(sum, off));
  __shared__ float sm[kBlock / 64], ss[kBlock / 64];
  const int wave = threadIdx.x >> 6;
  if ((threadIdx.x & 63) == 0) {
    sm[wave] = m;
    ss[wave] = sum;
  }
  __syncthreads();
  if (threadIdx.x == 0) {
    for (int w = 1; w < kBlock / 64; ++w) lse_combine(m, sum, sm[w], ss[w]);
    const float l = m + __logf(sum);
    const int64_t t = CLS ? tokens[r] : tokens[lrow + 1];
    lse[r] = l;
    // a label outside [0, V) (ignore_index -100, or a bad label) contributes nothing and is never read
    loss[r] = (t >= 0 && t < V) ? l - bf2f(row[t]) : 0.f;
  }
}

// scale: device scalar dloss (the mean's incoming gradient); inv_rows = 1 / (B * (S - 1))
template <bool CLS = false>
__global__ __launch_bounds__(kBlock) void xent_bwd_kernel(const uint16_t* __restrict__ logits,
                                                          const int64_t* __restrict__ tokens,
                                                          const float* __restrict__ lse, const float* __restrict__ dloss,
                                                          uint16_t* __restrict__ grad, int S, int V, float inv_rows) {
  const int lrow = blockIdx.x;                   // every logits row (b, s), s < S
  const int b = CLS ? lrow : lrow / S, s = CLS ? 0 : lrow - b * S;
  uint16_t* grow = grad + (int64_t)lrow * V;
  const uintptr_t q0 = (uintptr_t)grow;
  bf16x8* gbase = (bf16x8*)(q0 & ~(uintptr_t)15);
  const int head = (int)((q0 & 15) >> 1);       // logits and grad share the layout (same offsets)
  const int nch = (head + V + 7) >> 3;
  const int64_t tl = CLS ? tokens[lrow] : (s < S - 1 ? tokens[(int64_t)lrow + 1] : 0);
  if ((!CLS && s == S - 1) || tl < 0 || tl >= V) {  // predicts nothing (last position, ignored label): zero gradient
    for (int c = threadIdx.x; c < nch; c += kBlock) {
      if (c * 8 - head >= 0 && c * 8 - head + 8 <= V) {
        gbase[c] = bf16x8{};
      } else {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
          const int e = c * 8 + j - head;
          if (e >= 0 && e < V) grow[e] = 0;
        }
      }
    }
    return;
  }
  const int r = CLS ? lrow : b * (S - 1) + s;
  const float l = lse[r], g = dloss[0] * inv_rows;
  const int64_t t = tl;
  const bf16x8* base = (const bf16x8*)((uintptr_t)(logits + (int64_t)lrow * V) & ~(uintptr_t)15);
  for (int c = threadIdx.x; c < nch; c += kBlock) {
    const bf16x8 v = base[c];
    bf16x8 o;
#pragma unroll
    for (int j = 0; j < 8; ++j) {
      const int e = c * 8 + j - head;
      const float p = __expf(bf2f(v.v[j]) - l);
      o.v[j] = f2bf((p - (e == t ? 1.f : 0.f)) * g);
    }
    if (c * 8 - head >= 0 && c * 8 - head + 8 <= V) {
      gbase[c] = o;
    } else {
#pragma unroll
      for (int j = 0; j < 8; ++j) {
        const int e = c * 8 + j - head;
        if (e >= 0 && e < V) grow[e] = o.v[j];
      }
    }
  }
}

// ------------------------------------------------------------------------------------------------- column sums
// Block = 8 lanes x 8 columns (one 128-byte row segment per 8 lanes) x 32 row groups; grid (ceil(N/64), R) with R
// row splits of rpb rows.  Each split writes its 64 fp32 column partials (agent-scope atomic stores), drains and
// takes a ticket on the column tile's counter; the last one sums the R partial rows in split order.  Counters start zeroed and the last arriver resets its own; launches sharing the counters are
// stream-ordered.
constexpr int kCsGroups = 32;

// GELU (tanh approximation, GPT-2) derivative: d/dh [0.5 h (1 + tanh(u))], u = sqrt(2/pi) (h + 0.044715 h^3)
__device__ __forceinline__ float gelu_tanh_grad(float h) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  // tanh(u) = 1 - 2 / (1 + e^{2u}) on v_exp_f32 and v_rcp_f32 (saturates to +-1 at the extremes): libm tanhf made
  // this pass VALU-bound at ~3 TB/s
  const float e = __expf(2.f * k0 * fmaf(k1 * h * h, h, h));
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
  return fmaf(0.5f, 1.f + t, 0.5f * h * (1.f - t * t) * k0 * fmaf(3.f * k1, h * h, 1.f));
}

// GELU = true: x is dA (the gradient of gelu(h)) and the kernel also writes dh = dA * gelu'(h) (bf16, rounded
// before it is summed, so the bias gradient is the column sum of exactly the dh the GEMMs read) -- the activation
// backward and the up-projection's bias gradient in one pass over dA and h.
template <bool GELU>
__global__ __launch_bounds__(kBlock) void colsum_kernel(const bf16x8* __restrict__ x, int64_t T, int N, int rpb,
                                                        float* part, unsigned* cnt, void* out, int mode,
                                                        const bf16x8* __restrict__ h, bf16x8* __restrict__ dh) {
  const int N8 = N >> 3;
  const int cl = threadIdx.x & 7, rg = threadIdx.x >> 3;
  const int ch = blockIdx.x * 8 + cl;
  const int R = gridDim.y, s = blockIdx.y;
  const int64_t r0 = (int64_t)s * rpb;
  const int64_t r1 = r0 + rpb < T ? r0 + rpb : T;
  float acc[8];
#pragma unroll
  for (int j = 0; j < 8; ++j) acc[j] = 0.f;
  if (ch < N8) {
    for (int64_t r = r0 + rg; r < r1; r += 4 * kCsGroups) {  // 4 row segments in flight per lane
      bf16x8 v[4], hv[4];
#pragma unroll
      for (int u = 0; u < 4; ++u) {
        const int64_t rr = r + u * kCsGroups;
        v[u] = rr < r1 ? x[rr * N8 + ch] : bf16x8{};
        if (GELU) hv[u] = rr < r1 ? h[rr * N8 + ch] : bf16x8{};
      }
      if (GELU) {
#pragma unroll
        for (int u = 0; u < 4; ++u) {
#pragma unroll
          for (int j = 0; j < 8; ++j) v[u].v[j] = f2bf(bf2f(v[u].v[j]) * gelu_tanh_grad(bf2f(hv[u].v[j])));
          const int64_t rr = r + u * kCsGroups;
          if (rr < r1) dh[rr * N8 + ch] = v[u];
        }
      }
#pragma unroll
      for (int u = 0; u < 4; ++u)
#pragma unroll
        for (int j = 0; j < 8; ++j) acc[j] += bf2f(v[u].v[j]);
    }
  }
  __shared__ float sh[kCsGroups][65];
  __shared__ float sf[4][64];
  __shared__ int s_last;
#pragma unroll
  for (int j = 0; j < 8; ++j) sh[rg][cl * 8 + j] = acc[j];
  __syncthreads();
  if (threadIdx.x < 64) {
    const int col = blockIdx.x * 64 + threadIdx.x;
    float t = 0.f;
#pragma unroll 8
    for (int g = 0; g < kCsGroups; ++g) t += sh[g][threadIdx.x];
    if (col < N) __hip_atomic_store(part + (int64_t)s * N + col, t, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  // Hand-off without agent-scope fences: on gfx950 a release fence is an L2 write-back (buffer_wbl2) and an acquire
  // an L2 invalidate, per workgroup -- with ~1000 workgroups (and, in the GELU form, 100 MB of dirty dh in the L2s)
  // that dominated the kernel.  The partials are agent-scope atomic stores instead (coherent across the XCDs'
  // L2s), drained (vmcnt(0)) before the ticket, and the last arriver reads them with agent-scope atomic loads.
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  if (threadIdx.x == 0) {
    plx_handoff_release();  // no-op unless built with PLX_HANDOFF_FENCES (csrc/handoff.h: the hardware assumption)
    const unsigned old = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned)(R - 1);
    if (last) plx_handoff_acquire();
    if (last) __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int col = blockIdx.x * 64 + lc;
  float a = 0.f;
  if (col < N) {
    for (int b = g; b < R; b += 32) {  // 8 partial rows in flight per lane
      float y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        y[u] = b + 4 * u < R ? __hip_atomic_load(part + (int64_t)(b + 4 * u) * N + col, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) a += y[u];
    }
  }
  sf[g][lc] = a;
  __syncthreads();
  if (g == 0 && col < N) {
    const float v = ((sf[0][lc] + sf[1][lc]) + sf[2][lc]) + sf[3][lc];
    if (mode == 2)
      ((float*)out)[col] += v;
    else if (mode == 1)
      ((float*)out)[col] = v;
    else
      ((uint16_t*)out)[col] = f2bf(v);
  }
}
}  // namespace

PLX_API int plx_qkv_rope_fwd(const void* qkv, const float* cosv, const float* sinv, void* q, void* k, void* v,
                             int64_t T, int S, int H, int KV, int D, int rot_heads, hipStream_t stream) {
  if (T <= 0 || S <= 0 || T % S || D % 16 || rot_heads < 0 || rot_heads > H + KV) return 1;
  const int64_t items = T * (H + 2 * KV) * (D / 16);
  hipLaunchKernelGGL(qkv_rope_fwd_kernel, dim3(grid_for(items)), dim3(kBlock), 0, stream, (const bf16x8*)qkv, cosv,
                     sinv, (bf16x8*)q, (bf16x8*)k, (bf16x8*)v, T, S, H, KV, D, rot_heads);
  return (int)hipGetLastError();
}

PLX_API int plx_qkv_rope_bwd(const void* dq, const void* dk, const void* dv, const float* cosv, const float* sinv,
                             void* dqkv, int64_t T, int S, int H, int KV, int D, int rot_heads, hipStream_t stream) {
  if (T <= 0 || S <= 0 || T % S || D % 16 || rot_heads < 0 || rot_heads > H + KV) return 1;
  const int64_t items = T * (H + 2 * KV) * (D / 16);
  hipLaunchKernelGGL(qkv_rope_bwd_kernel, dim3(grid_for(items)), dim3(kBlock), 0, stream, (const bf16x8*)dq,
                     (const bf16x8*)dk, (const bf16x8*)dv, cosv, sinv, (bf16x8*)dqkv, T, S, H, KV, D, rot_heads);
  return (int)hipGetLastError();
}

PLX_API int plx_swiglu_fwd(const void* h, void* a, int64_t T, int F, hipStream_t stream) {
  if (T <= 0 || F % 8) return 1;
  hipLaunchKernelGGL(swiglu_fwd_kernel, dim3(grid_for(T * (F / 8))), dim3(kBlock), 0, stream, (const bf16x8*)h,
                     (bf16x8*)a, T, F / 8);
  return (int)hipGetLastError();
}

PLX_API int plx_swiglu_bwd(const void* da, const void* h, void* dh, int64_t T, int F, hipStream_t stream) {
  if (T <= 0 || F % 8) return 1;
  hipLaunchKernelGGL(swiglu_bwd_kernel, dim3(grid_for(T * (F / 8))), dim3(kBlock), 0, stream, (const bf16x8*)da,
                     (const bf16x8*)h, (bf16x8*)dh, T, F / 8);
  return (int)hipGetLastError();
}

// logits bf16 [B][S][V] contiguous, tokens int64 [B][S]; lse / loss fp32 [B * (S - 1)]
PLX_API int plx_xent_fwd(const void* logits, const int64_t* tokens, float* lse, float* loss, int B, int S, int V,
                         hipStream_t stream) {
  if (B <= 0 || S < 2 || V <= 0) return 1;
  hipLaunchKernelGGL(xent_fwd_kernel<false>, dim3(B * (S - 1)), dim3(kBlock), 0, stream, (const uint16_t*)logits, tokens,
                     lse, loss, S, V);
  return (int)hipGetLastError();
}

// classification cross entropy: logits bf16 [N][V] contiguous, labels int64 [N]; lse / loss fp32 [N]
PLX_API int plx_xent_cls_fwd(const void* logits, const int64_t* labels, float* lse, float* loss, int N, int V,
                             hipStream_t stream) {
  if (N <= 0 || V <= 0) return 1;
  hipLaunchKernelGGL(xent_fwd_kernel<true>, dim3(N), dim3(kBlock), 0, stream, (const uint16_t*)logits, labels, lse, loss,
                     1, V);
  return (int)hipGetLastError();
}

// grad bf16 [N][V] = (softmax - onehot(label)) * dloss * scale (scale <= 0: 1 / N, the mean over all rows); rows whose
// label is outside [0, V) get a zero gradient; dloss: device scalar gradient of the loss
PLX_API int plx_xent_cls_bwd(const void* logits, const int64_t* labels, const float* lse, const float* dloss,
                             void* grad, int N, int V, float scale, hipStream_t stream) {
  if (N <= 0 || V <= 0) return 1;
  hipLaunchKernelGGL(xent_bwd_kernel<true>, dim3(N), dim3(kBlock), 0, stream, (const uint16_t*)logits, labels, lse,
                     dloss, (uint16_t*)grad, 1, V, scale > 0.f ? scale : 1.f / (float)N);
  return (int)hipGetLastError();
}

// grad bf16 [B][S][V] (same layout as logits); dloss: device scalar gradient of the mean loss
PLX_API int plx_xent_bwd(const void* logits, const int64_t* tokens, const float* lse, const float* dloss, void* grad,
                         int B, int S, int V, hipStream_t stream) {
  if (B <= 0 || S < 2 || V <= 0) return 1;
  hipLaunchKernelGGL(xent_bwd_kernel<false>, dim3(B * S), dim3(kBlock), 0, stream, (const uint16_t*)logits, tokens,
                     lse, dloss, (uint16_t*)grad, S, V, 1.f / (float)(B * (S - 1)));
  return (int)hipGetLastError();
}

// partial rows a launch of plx_colsum writes (size its fp32 workspace [rows][N])
PLX_API int plx_colsum_splits(int64_t T, int N) {
  if (T <= 0 || N <= 0) return 0;
  const int tiles = (N + 63) / 64;
  int64_t R = (1024 + tiles - 1) / tiles;                 // ~1024 workgroups over the 256 CUs
  const int64_t rmax = (T + 4 * kCsGroups - 1) / (4 * kCsGroups);  // >= 4 rows per lane
  if (R > rmax) R = rmax;
  if (R < 1) R = 1;
  const int64_t rpb = (T + R - 1) / R;
  return (int)((T + rpb - 1) / rpb);
}

// out[N] = column sums (mode 0: bf16 store, 1: fp32 store, 2: fp32 accumulate into out) of x bf16 [T][N] (N % 8 == 0, 16-byte aligned rows);
// part: fp32 [plx_colsum_splits(T, N)][N]; cnt: >= ceil(N/64) zeroed counters
PLX_API int plx_colsum(const void* x, int64_t T, int N, float* part, unsigned* cnt, void* out, int mode,
                       hipStream_t stream) {
  if (T <= 0 || N <= 0 || N % 8 || ((uintptr_t)x & 15) || mode < 0 || mode > 2) return 1;
  const int R0 = plx_colsum_splits(T, N);
  const int rpb = (int)((T + R0 - 1) / R0);
  const int R = (int)((T + rpb - 1) / rpb);
  hipLaunchKernelGGL(colsum_kernel<false>, dim3((N + 63) / 64, R), dim3(kBlock), 0, stream, (const bf16x8*)x, T, N, rpb,
                     part, cnt, out, mode, nullptr, nullptr);
  return (int)hipGetLastError();
}

// dh = dA * gelu_tanh'(h) (bf16 [T][N], written) and out = column sums of dh (modes as plx_colsum); same workspace
PLX_API int plx_gelu_bwd_colsum(const void* da, const void* h, void* dh, int64_t T, int N, float* part, unsigned* cnt,
                                void* out, int mode, hipStream_t stream) {
  if (T <= 0 || N <= 0 || N % 8 || (((uintptr_t)da | (uintptr_t)h | (uintptr_t)dh) & 15) || mode < 0 || mode > 2)
    return 1;
  const int R0 = plx_colsum_splits(T, N);
  const int rpb = (int)((T + R0 - 1) / R0);
  const int R = (int)((T + rpb - 1) / rpb);
  hipLaunchKernelGGL(colsum_kernel<true>, dim3((N + 63) / 64, R), dim3(kBlock), 0, stream, (const bf16x8*)da, T, N, rpb,
                     part, cnt, out, mode, (const bf16x8*)h, (bf16x8*)dh);
  return (int)hipGetLastError();
}
