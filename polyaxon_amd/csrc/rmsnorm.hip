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

__global__ __launch_bounds__(kBlock) void rms_fwd_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                         bf16x8* __restrict__ y, float* __restrict__ rstd_out,
                                                         int64_t rows, int dv, float eps) {
  __shared__ float sh[kBlock / 64];
  for (int64_t r = blockIdx.x; r < rows; r += gridDim.x) {
    const bf16x8* xr = x + r * dv;
    float ss = 0.f;
    for (int i = threadIdx.x; i < dv; i += kBlock) {
      const bf16x8 v = xr[i];
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

__global__ __launch_bounds__(kBlock) void rms_bwd_kernel(const bf16x8* __restrict__ x, const float* __restrict__ w,
                                                         const bf16x8* __restrict__ dy, const float* __restrict__ rstd_in,
                                                         bf16x8* __restrict__ dx, float* __restrict__ dw_part,
                                                         int64_t rows, int dv) {
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
        bf16x8 o;
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float xh = bf2f(xv.v[k]) * rstd;
          o.v[k] = f2bf(rstd * (bf2f(gv.v[k]) * w[i * 8 + k] - xh * mean_dot));
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
}  // namespace

PLX_API int plx_rms_forward(const void* x, const float* w, void* y, float* rstd, int64_t rows, int d, float eps,
                            hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  int64_t g = rows < 4096 ? rows : 4096;
  hipLaunchKernelGGL(rms_fwd_kernel, dim3((int)g), dim3(kBlock), 0, stream, (const bf16x8*)x, w, (bf16x8*)y, rstd, rows,
                     d / 8, eps);
  return (int)hipGetLastError();
}

// grid size the host must allocate dw partials for: [plx_rms_bwd_blocks(rows), d]
PLX_API int plx_rms_bwd_blocks(int64_t rows) { return (int)(rows < 1024 ? rows : 1024); }

PLX_API int plx_rms_backward(const void* x, const float* w, const void* dy, const float* rstd, void* dx,
                             float* dw_part, int64_t rows, int d, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  hipLaunchKernelGGL(rms_bwd_kernel, dim3(plx_rms_bwd_blocks(rows)), dim3(kBlock), 0, stream, (const bf16x8*)x, w,
                     (const bf16x8*)dy, rstd, (bf16x8*)dx, dw_part, rows, d / 8);
  return (int)hipGetLastError();
}

// LayerNorm: mean / rstd fp32 [rows] saved for the backward
PLX_API int plx_ln_forward(const void* x, const float* w, const float* b, void* y, float* mean, float* rstd,
                           int64_t rows, int d, float eps, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  int64_t g = rows < 4096 ? rows : 4096;
  hipLaunchKernelGGL(ln_fwd_kernel, dim3((int)g), dim3(kBlock), 0, stream, (const bf16x8*)x, w, b, (bf16x8*)y, mean,
                     rstd, rows, d / 8, eps);
  return (int)hipGetLastError();
}

// dw / db partials [plx_rms_bwd_blocks(rows), d] each, summed by the host side
PLX_API int plx_ln_backward(const void* x, const float* w, const void* dy, const float* mean, const float* rstd,
                            void* dx, float* dw_part, float* db_part, int64_t rows, int d, hipStream_t stream) {
  if (d % 8 || d > kBlock * 8 * kMaxVecPerLane || rows <= 0) return 1;
  hipLaunchKernelGGL(ln_bwd_kernel, dim3(plx_rms_bwd_blocks(rows)), dim3(kBlock), 0, stream, (const bf16x8*)x, w,
                     (const bf16x8*)dy, mean, rstd, (bf16x8*)dx, dw_part, db_part, rows, d / 8);
  return (int)hipGetLastError();
}
