// Fused RMSNorm and LayerNorm forward/backward for bf16 activations (Llama-3 8B / GPT-2 configs) on MI355X.
//
// LayerNorm (GPT-2): y = (x - mean) * rstd * w + b; dx = rstd * (g - mean(g) - xhat * mean(g * xhat)), g = w * dy;
// dw = sum dy * xhat, db = sum dy.  bf16 in / out with fp32 statistics: under autocast PyTorch's layer_norm runs in
// fp32, i.e. a bf16 -> fp32 copy in, an fp32 -> bf16 copy out for the next GEMM, and the same again backward.
//
//   y  = x * rstd * w,            rstd = 1 / sqrt(mean(x^2) + eps)        (rstd saved per row, fp32)
//   dx = rstd * (w*dy - xhat * mean(w*dy*xhat)),  xhat = x * rstd
//   dw = sum_rows dy * xhat      (per-block partials in registers -> [gridDim.x, d] fp32, summed on host side)
//
// One 256-thread workgroup per row (grid-strided over rows); each lane moves 16-byte vectors (8 x bf16),
// wave64 shuffle + LDS reductions, fp32 math.  d % 8 == 0 and d <= 8192 (column partials of dw live in
// registers: d / 8 / 256 vectors per lane).
#include <hip/hip_runtime.h>

#include "handoff.h"
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kBlock = 256;
constexpr int kMaxVecPerLane = 4;  // d <= 256 * 8 * 4 = 8192

struct alignas(16) bf16x8 {
  uint16_t v[8];
};

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {  // hardware RNE conversion, NaN stays NaN
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ float block_sum(float v, float* sh) {
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  const int w = threadIdx.x >> 6;
  __syncthreads();
  if ((threadIdx.x & 63) == 0) sh[w] = v;
  __syncthreads();
  float t = 0.f;
#pragma unroll
  for (int i = 0; i < kBlock / 64; ++i) t += sh[i];
  return t;
}

// ADD: the residual add feeding the norm is fused in -- s = bf16(x + res) is written (the next residual) and
// normalised; the second pass re-reads the s chunk this same thread wrote.
template <bool ADD = false>
__global__ __launch_bounds__(kBlock) void rms_fwd_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                         bf16x8* __restrict__ y, float* __restrict__ rstd_out,
                                                         int64_t rows, int dv, float eps,
                                                         const bf16x8* __restrict__ res = nullptr,
                                                         bf16x8* __restrict__ s_out = nullptr) {
  __shared__ float sh[kBlock / 64];
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const bf16x8* xr = ADD ? s_out + r * dv : x + r * dv;  // pass 2 reads the sum
    float ss = 0.f;
    for (int i = threadIdx.x; i < dv; i += kBlock) {
      bf16x8 v = x[r * dv + i];
      if (ADD) {
        const bf16x8 rv = res[r * dv + i];
#pragma unroll
        for (int k = 0; k < 8; ++k) v.v[k] = f2bf(bf2f(v.v[k]) + bf2f(rv.v[k]));
        s_out[r * dv + i] = v;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float f = bf2f(v.v[k]);
        ss = fmaf(f, f, ss);
      }
    }
    const float tot = block_sum(ss, sh);
    const float rstd = rsqrtf(tot / (float)(dv * 8) + eps);
    if (threadIdx.x == 0 && rstd_out) rstd_out[r] = rstd;
    for (int i = threadIdx.x; i < dv; i += kBlock) {
      const bf16x8 v = xr[i];
      bf16x8 o;
#pragma unroll
      for (int k = 0; k < 8; ++k) o.v[k] = f2bf(bf2f(v.v[k]) * rstd * w[i * 8 + k]);
      y[r * dv + i] = o;
    }
  }
}

// ADD: dx = RMSNorm backward + dres (the residual path's gradient), fp32 sum rounded once
template <bool ADD = false>
__global__ __launch_bounds__(kBlock) void rms_bwd_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                         const bf16x8* __restrict__ dy, const float* __restrict__ rstd_in,
                                                         bf16x8* __restrict__ dx, float* __restrict__ dw_part,
                                                         int64_t rows, int dv,
                                                         const bf16x8* __restrict__ dres = nullptr) {
  __shared__ float sh[kBlock / 64];
  float dwacc[kMaxVecPerLane][8];
#pragma unroll
  for (int j = 0; j < kMaxVecPerLane; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) dwacc[j][k] = 0.f;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float rstd = rstd_in[r];
    float dot = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxVecPerLane; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < dv) {
        const bf16x8 xv = x[r * dv + i], gv = dy[r * dv + i];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = bf2f(xv.v[k]) * rstd, g = bf2f(gv.v[k]);
          dot = fmaf(g * w[i * 8 + k], xh, dot);
          dwacc[j][k] = fmaf(g, xh, dwacc[j][k]);
        }
      }
    }
    const float mean_dot = block_sum(dot, sh) / (float)(dv * 8);
#pragma unroll
    for (int j = 0; j < kMaxVecPerLane; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < dv) {
        const bf16x8 xv = x[r * dv + i], gv = dy[r * dv + i];
        bf16x8 dr = {};
        if (ADD) dr = dres[r * dv + i];
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = bf2f(xv.v[k]) * rstd;
          const float g = rstd * (bf2f(gv.v[k]) * w[i * 8 + k] - xh * mean_dot);
          o.v[k] = f2bf(ADD ? g + bf2f(dr.v[k]) : g);
        }
        dx[r * dv + i] = o;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kMaxVecPerLane; ++j) {
    const int i = threadIdx.x + j * kBlock;
    if (i < dv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) dw_part[(int64_t)blockIdx.x * dv * 8 + i * 8 + k] = dwacc[j][k];
    }
  }
}


// ------------------------------------------------------------------------------------------------ LayerNorm
__global__ __launch_bounds__(kBlock) void ln_fwd_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                        const float* __restrict__ bias, bf16x8* __restrict__ y,
                                                        float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                        int64_t rows, int dv, float eps) {
  __shared__ float sh[kBlock / 64];
  const float inv_d = 1.f / (float)(dv * 8);
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const bf16x8* xr = x + r * dv;
    float xs[kMaxVecPerLane][8];
    float s1 = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxVecPerLane; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < dv) {
        const bf16x8 v = xr[i];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          xs[j][k] = bf2f(v.v[k]);
          s1 += xs[j][k];
        }
      }
    }
    const float mean = block_sum(s1, sh) * inv_d;
    float s2 = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxVecPerLane; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < dv) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float c = xs[j][k] - mean;
          s2 = fmaf(c, c, s2);
        }
      }
    }
    const float rstd = rsqrtf(block_sum(s2, sh) * inv_d + eps);
    if (threadIdx.x == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
#pragma unroll
    for (int j = 0; j < kMaxVecPerLane; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < dv) {
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = f2bf(fmaf((xs[j][k] - mean) * rstd, w[i * 8 + k], bias[i * 8 + k]));
        y[r * dv + i] = o;
      }
    }
  }
}

__global__ __launch_bounds__(kBlock) void ln_bwd_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                        const bf16x8* __restrict__ dy, const float* __restrict__ mean_in,
                                                        const float* __restrict__ rstd_in, bf16x8* __restrict__ dx,
                                                        float* __restrict__ dw_part, float* __restrict__ db_part,
                                                        int64_t rows, int dv) {
  __shared__ float sh[kBlock / 64];
  const float inv_d = 1.f / (float)(dv * 8);
  float dwacc[kMaxVecPerLane][8], dbacc[kMaxVecPerLane][8];
#pragma unroll
  for (int j = 0; j < kMaxVecPerLane; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) dwacc[j][k] = dbacc[j][k] = 0.f;
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const float mean = mean_in[r], rstd = rstd_in[r];
    float xh[kMaxVecPerLane][8], gw[kMaxVecPerLane][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < kMaxVecPerLane; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < dv) {
        const bf16x8 xv = x[r * dv + i], gv = dy[r * dv + i];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = bf2f(gv.v[k]);
          xh[j][k] = (bf2f(xv.v[k]) - mean) * rstd;
          gw[j][k] = g * w[i * 8 + k];
          sg += gw[j][k];
          sgx = fmaf(gw[j][k], xh[j][k], sgx);
          dwacc[j][k] = fmaf(g, xh[j][k], dwacc[j][k]);
          dbacc[j][k] += g;
        }
      }
    }
    const float mg = block_sum(sg, sh) * inv_d;
    const float mgx = block_sum(sgx, sh) * inv_d;
#pragma unroll
    for (int j = 0; j < kMaxVecPerLane; ++j) {
      const int i = threadIdx.x + j * kBlock;
      if (i < dv) {
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = f2bf(rstd * (gw[j][k] - mg - xh[j][k] * mgx));
        dx[r * dv + i] = o;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < kMaxVecPerLane; ++j) {
    const int i = threadIdx.x + j * kBlock;
    if (i < dv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        dw_part[(int64_t)blockIdx.x * dv * 8 + i * 8 + k] = dwacc[j][k];
        db_part[(int64_t)blockIdx.x * dv * 8 + i * 8 + k] = dbacc[j][k];
      }
    }
  }
}

// Narrow rows (GPT-2: d = 768 -> 96 vectors) leave most of a 256-thread workgroup idle and pay two LDS barriers per
// row: there one WAVE owns a row (VPL 16-byte vectors per lane, d <= 64 * 8 * VPL), statistics are wave shuffles
// only, and the 4 waves of a workgroup walk independent rows.  Backward column partials stay in registers per wave
// and are combined through LDS once per workgroup at the end.
__device__ __forceinline__ float wave_sum(float v) {
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) v += __shfl_xor(v, off, 64);
  return v;
}

// ADD: the residual add feeding the norm is fused in: s = bf16(x + res) is written (the next residual) and
// normalised -- one pass instead of an add kernel (3 row streams) followed by the norm (2).
template <int VPL, bool ADD = false>
__global__ __launch_bounds__(kBlock) void ln_fwd_wave_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                             const float* __restrict__ bias, bf16x8* __restrict__ y,
                                                             float* __restrict__ mean_out, float* __restrict__ rstd_out,
                                                             int64_t rows, int dv, float eps,
                                                             const bf16x8* __restrict__ res = nullptr,
                                                             bf16x8* __restrict__ s_out = nullptr) {
  const int lane = threadIdx.x & 63;
  const float inv_d = 1.f / (float)(dv * 8);
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t r = (int64_t)blockIdx.x * (kBlock / 64) + (threadIdx.x >> 6); r < rows; r += nw) {
    const bf16x8* xr = x + r * dv;
    float xs[VPL][8];
    float s1 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int i = lane + j * 64;
      bf16x8 v = i < dv ? xr[i] : bf16x8{};
      if (ADD && i < dv) {
        const bf16x8 rv = res[r * dv + i];
#pragma unroll
        for (int k = 0; k < 8; ++k) v.v[k] = f2bf(bf2f(v.v[k]) + bf2f(rv.v[k]));
        s_out[r * dv + i] = v;
      }
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        xs[j][k] = bf2f(v.v[k]);
        s1 += xs[j][k];
      }
    }
    const float mean = wave_sum(s1) * inv_d;
    float s2 = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      if (lane + j * 64 < dv) {
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float c = xs[j][k] - mean;
          s2 = fmaf(c, c, s2);
        }
      }
    }
    const float rstd = rsqrtf(wave_sum(s2) * inv_d + eps);
    if (lane == 0) {
      mean_out[r] = mean;
      rstd_out[r] = rstd;
    }
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int i = lane + j * 64;
      if (i < dv) {
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) o.v[k] = f2bf(fmaf((xs[j][k] - mean) * rstd, w[i * 8 + k], bias[i * 8 + k]));
        y[r * dv + i] = o;
      }
    }
  }
}

// ADD: dx = LN backward + dres (the gradient arriving through the residual path), summed in fp32 and rounded once:
// the backward of the fused add + norm (both of its inputs get this same gradient)
template <int VPL, bool ADD = false>
__global__ __launch_bounds__(kBlock) void ln_bwd_wave_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                             const bf16x8* __restrict__ dy,
                                                             const float* __restrict__ mean_in,
                                                             const float* __restrict__ rstd_in, bf16x8* __restrict__ dx,
                                                             float* __restrict__ dw_part, float* __restrict__ db_part,
                                                             int64_t rows, int dv,
                                                             const bf16x8* __restrict__ dres = nullptr) {
  __shared__ float shw[kBlock / 64][VPL * 64 * 8];
  __shared__ float shb[kBlock / 64][VPL * 64 * 8];
  const int lane = threadIdx.x & 63, wv = threadIdx.x >> 6;
  const float inv_d = 1.f / (float)(dv * 8);
  float dwacc[VPL][8], dbacc[VPL][8];
#pragma unroll
  for (int j = 0; j < VPL; ++j)
#pragma unroll
    for (int k = 0; k < 8; ++k) dwacc[j][k] = dbacc[j][k] = 0.f;
  const int64_t nw = (int64_t)gridDim.x * (kBlock / 64);
  for (int64_t r = (int64_t)blockIdx.x * (kBlock / 64) + wv; r < rows; r += nw) {
    const float mean = mean_in[r], rstd = rstd_in[r];
    float xh[VPL][8], gw[VPL][8];
    float sg = 0.f, sgx = 0.f;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int i = lane + j * 64;
      if (i < dv) {
        const bf16x8 xv = x[r * dv + i], gv = dy[r * dv + i];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float g = bf2f(gv.v[k]);
          xh[j][k] = (bf2f(xv.v[k]) - mean) * rstd;
          gw[j][k] = g * w[i * 8 + k];
          sg += gw[j][k];
          sgx = fmaf(gw[j][k], xh[j][k], sgx);
          dwacc[j][k] = fmaf(g, xh[j][k], dwacc[j][k]);
          dbacc[j][k] += g;
        }
      }
    }
    const float mg = wave_sum(sg) * inv_d;
    const float mgx = wave_sum(sgx) * inv_d;
#pragma unroll
    for (int j = 0; j < VPL; ++j) {
      const int i = lane + j * 64;
      if (i < dv) {
        bf16x8 o;
        if (ADD) {
          const bf16x8 dr = dres[r * dv + i];
#pragma unroll
          for (int k = 0; k < 8; ++k) o.v[k] = f2bf(fmaf(rstd, gw[j][k] - mg - xh[j][k] * mgx, bf2f(dr.v[k])));
        } else {
#pragma unroll
          for (int k = 0; k < 8; ++k) o.v[k] = f2bf(rstd * (gw[j][k] - mg - xh[j][k] * mgx));
        }
        dx[r * dv + i] = o;
      }
    }
  }
#pragma unroll
  for (int j = 0; j < VPL; ++j) {
    const int i = lane + j * 64;
    if (i < dv) {
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        shw[wv][i * 8 + k] = dwacc[j][k];
        shb[wv][i * 8 + k] = dbacc[j][k];
      }
    }
  }
  __syncthreads();
  const int d = dv * 8;
  for (int c = threadIdx.x; c < d; c += kBlock) {  // the 4 waves' columns in wave order
    dw_part[(int64_t)blockIdx.x * d + c] = ((shw[0][c] + shw[1][c]) + shw[2][c]) + shw[3][c];
    db_part[(int64_t)blockIdx.x * d + c] = ((shb[0][c] + shb[1][c]) + shb[2][c]) + shb[3][c];
  }
}

// ----------------------------------------------------------------------------- partial rows -> parameter gradient
// The backward kernels leave fp32 [nb][d] partial rows of dw (and db); this sums up to two such matrices column-wise
// into their outputs in ONE launch: grid (ceil(d/64), R row splits of 64, nz matrices), block = 64 columns x 4 row
// groups (a wave reads 256 contiguous bytes per row), level-2 rows published as agent-scope atomic stores (coherent
// across the XCDs' L2s; no release fence = no per-workgroup L2 write-back), drained before a relaxed ticket, read by
// the last split (which resets its counter) with agent-scope atomic loads and summed in split order: deterministic.  out = sum (store) or out += sum (accumulate: the parameter's flat gradient
// slot, instead of autograd's separate `grad += g` pass).  Replaces a strided torch reduction (~19 us at nb = 1024,
// d = 768) plus one accumulate kernel per parameter.
constexpr int kPsRows = 64;

__global__ __launch_bounds__(kBlock) void partial_colsum_kernel(const float* __restrict__ p0, const float* __restrict__ p1,
                                                                int rows, int d, float* l2, unsigned* cnt, float* o0,
                                                                float* o1, int acc0, int acc1) {
  const int z = blockIdx.z;
  const float* p = z ? p1 : p0;
  const int lc = threadIdx.x & 63, g = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  const int R = gridDim.y, s = blockIdx.y;
  const int r0 = s * kPsRows;
  const int r1 = r0 + kPsRows < rows ? r0 + kPsRows : rows;
  float a = 0.f;
  if (c < d) {
    float x[kPsRows / 4];
#pragma unroll
    for (int u = 0; u < kPsRows / 4; ++u) {
      const int r = r0 + g + 4 * u;
      x[u] = r < r1 ? p[(int64_t)r * d + c] : 0.f;
    }
#pragma unroll
    for (int u = 0; u < kPsRows / 4; ++u) a += x[u];
  }
  __shared__ float sh[4][64];
  __shared__ int s_last;
  sh[g][lc] = a;
  __syncthreads();
  float* l2z = l2 + (int64_t)z * R * d;
  if (g == 0 && c < d)  // agent-scope atomic store: coherent across the XCDs' L2s without a release fence
    __hip_atomic_store(l2z + (int64_t)s * d + c, ((sh[0][lc] + sh[1][lc]) + sh[2][lc]) + sh[3][lc], __ATOMIC_RELAXED,
                       __HIP_MEMORY_SCOPE_AGENT);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  unsigned* ctr = cnt + (int64_t)z * gridDim.x + blockIdx.x;
  if (threadIdx.x == 0) {
    plx_handoff_release();  // no-op unless built with PLX_HANDOFF_FENCES (csrc/handoff.h: the hardware assumption)
    const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned)(R - 1);
    if (last) plx_handoff_acquire();
    if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  if (!s_last) return;
  float b = 0.f;
  if (c < d) {
    for (int r = g; r < R; r += 32) {  // 8 level-2 rows in flight per lane
      float y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u)
        y[u] = r + 4 * u < R ? __hip_atomic_load(l2z + (int64_t)(r + 4 * u) * d + c, __ATOMIC_RELAXED,
                                                 __HIP_MEMORY_SCOPE_AGENT)
                             : 0.f;
#pragma unroll
      for (int u = 0; u < 8; ++u) b += y[u];
    }
  }
  __syncthreads();
  sh[g][lc] = b;
  __syncthreads();
  if (g == 0 && c < d) {
    const float v = ((sh[0][lc] + sh[1][lc]) + sh[2][lc]) + sh[3][lc];
    float* o = z ? o1 : o0;
    o[c] = (z ? acc1 : acc0) ? o[c] + v : v;
  }
}
}  // namespace

PLX_API int plx_rms_forward(const void* x, const float* w, void* y, float* rstd, int64_t rows, int d, float eps,
                            hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  int64_t g = rows < 4096 ? rows : 4096;
  hipLaunchKernelGGL(rms_fwd_kernel<false>, dim3((int)g), dim3(kBlock), 0, stream, (const bf16x8*)x, w, (bf16x8*)y, rstd,
                     rows, d / 8, eps, (const bf16x8*)nullptr, (bf16x8*)nullptr);
  return (int)hipGetLastError();
}

// grid size the host must allocate dw partials for: [plx_rms_bwd_blocks(rows), d]
PLX_API int plx_rms_bwd_blocks(int64_t rows) { return (int)(rows < 1024 ? rows : 1024); }

PLX_API int plx_rms_backward(const void* x, const float* w, const void* dy, const float* rstd, void* dx,
                             float* dw_part, int64_t rows, int d, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  hipLaunchKernelGGL(rms_bwd_kernel<false>, dim3(plx_rms_bwd_blocks(rows)), dim3(kBlock), 0, stream, (const bf16x8*)x, w,
                     (const bf16x8*)dy, rstd, (bf16x8*)dx, dw_part, rows, d / 8, (const bf16x8*)nullptr);
  return (int)hipGetLastError();
}

// LayerNorm: mean / rstd fp32 [rows] saved for the backward

// wave-per-row path: 16-byte vectors per lane (1 or 2: d <= 1024), 0 = workgroup-per-row kernels
static inline int ln_vpl(int d) { return d <= 512 ? 1 : d <= 1024 ? 2 : 0; }

PLX_API int plx_ln_forward(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                           int64_t rows, int d, float eps, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  const int vpl = ln_vpl(d);
  if (vpl) {
    int64_t g = (rows + 3) / 4;
    if (g > 8192) g = 8192;
    hipLaunchKernelGGL(vpl == 1 ? ln_fwd_wave_kernel<1> : ln_fwd_wave_kernel<2>, dim3((int)g), dim3(kBlock), 0, stream,
                       (const bf16x8*)x, w, b, (bf16x8*)y, mean, rstd, rows, d / 8, eps, (const bf16x8*)nullptr,
                       (bf16x8*)nullptr);
    return (int)hipGetLastError();
  }
  int64_t g = rows < 4096 ? rows : 4096;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((int)g), dim3(kBlock), 0, stream, (const bf16x8*)x, w, b, (bf16x8*)y, mean,
                     rstd, rows, d / 8, eps);
  return (int)hipGetLastError();
}

// partial rows plx_ln_backward writes: [plx_ln_bwd_blocks(rows, d), d] for dw and for db
PLX_API int plx_ln_bwd_blocks(int64_t rows, int d) {
  if (ln_vpl(d)) {
    const int64_t g = (rows + 3) / 4;
    return (int)(g < 1024 ? g : 1024);
  }
  return plx_rms_bwd_blocks(rows);
}

// dw / db partials [plx_ln_bwd_blocks(rows, d), d] each, summed by plx_partial_colsum
PLX_API int plx_ln_backward(const void* x, const float* w, const void* dy, const float* mean, const float* rstd,
                            void* dx, float* dw_part, float* db_part, int64_t rows, int d, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  const int vpl = ln_vpl(d);
  if (vpl) {
    hipLaunchKernelGGL(vpl == 1 ? ln_bwd_wave_kernel<1> : ln_bwd_wave_kernel<2>, dim3(plx_ln_bwd_blocks(rows, d)),
                       dim3(kBlock), 0, stream, (const bf16x8*)x, w, (const bf16x8*)dy, mean, rstd, (bf16x8*)dx,
                       dw_part, db_part, rows, d / 8, (const bf16x8*)nullptr);
    return (int)hipGetLastError();
  }
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(plx_ln_bwd_blocks(rows, d)), dim3(kBlock), 0, stream, (const bf16x8*)x, w,
                     (const bf16x8*)dy, mean, rstd, (bf16x8*)dx, dw_part, db_part, rows, d / 8);
  return (int)hipGetLastError();
}

// level-2 workspace floats for plx_partial_colsum: nz * ceil(rows / 64) * d
PLX_API int64_t plx_partial_colsum_workspace(int rows, int d, int nz) {
  return (int64_t)nz * ((rows + kPsRows - 1) / kPsRows) * d;
}

// o_z[c] (+)= sum_r p_z[r][c] for z < nz (1 or 2); cnt: >= nz * ceil(d/64) zeroed counters (stream-ordered reuse)
PLX_API int plx_partial_colsum(const float* p0, const float* p1, int rows, int d, int nz, float* l2, unsigned* cnt,
                               float* o0, float* o1, int acc0, int acc1, hipStream_t stream) {
  if (rows <= 0 || d <= 0 || nz < 1 || nz > 2) return 1;
  const int R = (rows + kPsRows - 1) / kPsRows;
  hipLaunchKernelGGL(partial_colsum_kernel, dim3((d + 63) / 64, R, nz), dim3(kBlock), 0, stream, p0, p1, rows, d, l2,
                     cnt, o0, o1, acc0, acc1);
  return (int)hipGetLastError();
}

// fused residual add + LayerNorm: s = bf16(x + res) (written), y = LN(s).  Wave path only (d <= 1024): returns 2
// (nothing launched) otherwise, and the caller adds and normalises separately.
PLX_API int plx_add_ln_forward(const void* x, const void* res, const float* w, const float* b, void* s, void* y,
                               float* mean, float* rstd, int64_t rows, int d, float eps, hipStream_t stream) {
  if (d % 8 || rows <= 0) return 1;
  const int vpl = ln_vpl(d);
  if (!vpl) return 2;
  int64_t g = (rows + 3) / 4;
  if (g > 8192) g = 8192;
  auto k = vpl == 1 ? ln_fwd_wave_kernel<1, true> : ln_fwd_wave_kernel<2, true>;
  hipLaunchKernelGGL(k, dim3((int)g), dim3(kBlock), 0, stream, (const bf16x8*)x, w, b, (bf16x8*)y, mean, rstd, rows, d / 8, eps, (const bf16x8*)res,
                     (bf16x8*)s);
  return (int)hipGetLastError();
}

// its backward: dx = LN backward(s, dy) + dres (the gradient of both x and res); partials as plx_ln_backward
PLX_API int plx_add_ln_backward(const void* s, const float* w, const void* dy, const float* mean, const float* rstd,
                                const void* dres, void* dx, float* dw_part, float* db_part, int64_t rows, int d,
                                hipStream_t stream) {
  if (d % 8 || rows <= 0) return 1;
  const int vpl = ln_vpl(d);
  if (!vpl) return 2;
  auto k = vpl == 1 ? ln_bwd_wave_kernel<1, true> : ln_bwd_wave_kernel<2, true>;
  hipLaunchKernelGGL(k, dim3(plx_ln_bwd_blocks(rows, d)), dim3(kBlock), 0, stream, (const bf16x8*)s, w, (const bf16x8*)dy,
                     mean, rstd, (bf16x8*)dx, dw_part, db_part, rows, d / 8, (const bf16x8*)dres);
  return (int)hipGetLastError();
}

// fused residual add + RMSNorm (Llama): s = bf16(x + res) (written), y = RMSNorm(s); backward dx = RMSNorm backward
// (s, dy) + dres for both inputs, dw partials as plx_rms_backward
PLX_API int plx_add_rms_forward(const void* x, const void* res, const float* w, void* s, void* y, float* rstd,
                                int64_t rows, int d, float eps, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  int64_t g = rows < 4096 ? rows : 4096;
  hipLaunchKernelGGL(rms_fwd_kernel<true>, dim3((int)g), dim3(kBlock), 0, stream, (const bf16x8*)x, w, (bf16x8*)y, rstd,
                     rows, d / 8, eps, (const bf16x8*)res, (bf16x8*)s);
  return (int)hipGetLastError();
}

PLX_API int plx_add_rms_backward(const void* s, const float* w, const void* dy, const float* rstd, const void* dres,
                                 void* dx, float* dw_part, int64_t rows, int d, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  hipLaunchKernelGGL(rms_bwd_kernel<true>, dim3(plx_rms_bwd_blocks(rows)), dim3(kBlock), 0, stream, (const bf16x8*)s, w,
                     (const bf16x8*)dy, rstd, (bf16x8*)dx, dw_part, rows, d / 8, (const bf16x8*)dres);
  return (int)hipGetLastError();
}
