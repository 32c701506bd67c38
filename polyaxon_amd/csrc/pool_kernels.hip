// 3x3 / stride-2 / pad-1 max pooling (the ResNet stem pool) on NHWC bf16, forward + backward.
//
// PyTorch's NHWC max-pool forward writes an int64 argmax per output element (8 B against a 2 B value) and
// its backward scatters through it after zero-filling dx.  Here the forward stores the window position
// (0..8) as one byte per element and the backward GATHERS: each thread owns 8 channels of one input pixel,
// visits the <= 2x2 output windows that contain it and sums dy where that window's argmax is this pixel.
// No zero-fill, no atomics, every dx element written exactly once.  Ties keep the first maximum in (kh, kw)
// scan order and NaN wins, as in PyTorch.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

struct alignas(16) bf16x8 { uint16_t v[8]; };
struct alignas(8) u8x8 { uint8_t v[8]; };

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }
__device__ __forceinline__ uint16_t f2bf(float f) {
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
}

// one thread = 8 channels of one output pixel
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16x8* __restrict__ x, bf16x8* __restrict__ y,
                                                          u8x8* __restrict__ idx, int N, int H, int W, int G, int OH,
                                                          int OW) {
  const int64_t total = (int64_t)N * OH * OW * G;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(t % G);
    int64_t p = t / G;
    const int ow = (int)(p % OW);
    p /= OW;
    const int oh = (int)(p % OH);
    const int n = (int)(p / OH);
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = -INFINITY;
      arg[k] = 255;
    }
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * 2 - 1 + kh;
      if (ih < 0 || ih >= H) continue;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = ow * 2 - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        const bf16x8 v = x[(((int64_t)n * H + ih) * W + iw) * G + g];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          const float f = bf2f(v.v[k]);
          if (f > best[k] || (f != f && best[k] == best[k]) || arg[k] == 255) {
            best[k] = f;
            arg[k] = (uint8_t)(kh * 3 + kw);
          }
        }
      }
    }
    bf16x8 o;
    u8x8 a;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o.v[k] = f2bf(best[k]);
      a.v[k] = arg[k];
    }
    y[t] = o;
    idx[t] = a;
  }
}

// one thread = 8 channels of one input pixel
__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16x8* __restrict__ dy, const u8x8* __restrict__ idx,
                                                          bf16x8* __restrict__ dx, int N, int H, int W, int G, int OH,
                                                          int OW) {
  const int64_t total = (int64_t)N * H * W * G;
  for (int64_t t = blockIdx.x * (int64_t)blockDim.x + threadIdx.x; t < total; t += (int64_t)gridDim.x * blockDim.x) {
    const int g = (int)(t % G);
    int64_t p = t / G;
    const int iw = (int)(p % W);
    p /= W;
    const int ih = (int)(p % H);
    const int n = (int)(p / H);
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) acc[k] = 0.f;
    // ih = 2*oh - 1 + kh  =>  oh = (ih + 1 - kh) / 2 for kh in 0..2 with (ih + 1 - kh) even
    const int oh_hi = (ih + 1) >> 1, oh_lo = ih >= 1 ? (ih) >> 1 : 0;
    const int ow_hi = (iw + 1) >> 1, ow_lo = iw >= 1 ? (iw) >> 1 : 0;
    for (int oh = oh_lo; oh <= oh_hi && oh < OH; ++oh) {
      const int kh = ih + 1 - 2 * oh;
      if (kh < 0 || kh > 2) continue;
      for (int ow = ow_lo; ow <= ow_hi && ow < OW; ++ow) {
        const int kw = iw + 1 - 2 * ow;
        if (kw < 0 || kw > 2) continue;
        const int64_t o = (((int64_t)n * OH + oh) * OW + ow) * G + g;
        const u8x8 a = idx[o];
        const uint8_t me = (uint8_t)(kh * 3 + kw);
        bool any = false;
#pragma unroll
        for (int k = 0; k < 8; ++k) any |= a.v[k] == me;
        if (!any) continue;
        const bf16x8 d = dy[o];
#pragma unroll
        for (int k = 0; k < 8; ++k)
          if (a.v[k] == me) acc[k] += bf2f(d.v[k]);
      }
    }
    bf16x8 out;
#pragma unroll
    for (int k = 0; k < 8; ++k) out.v[k] = f2bf(acc[k]);
    dx[t] = out;
  }
}

inline int grid_for(int64_t total) {
  int64_t g = (total + 255) / 256;
  if (g > 8192) g = 8192;
  return (int)(g < 1 ? 1 : g);
}

}  // namespace

PLX_API int plx_maxpool3s2_forward(const void* x, void* y, void* idx, int N, int H, int W, int C, hipStream_t s) {
  if (C % 8 || N <= 0 || H <= 0 || W <= 0) return 1;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1, G = C / 8;
  hipLaunchKernelGGL(maxpool_fwd_kernel, dim3(grid_for((int64_t)N * OH * OW * G)), dim3(256), 0, s,
                     (const bf16x8*)x, (bf16x8*)y, (u8x8*)idx, N, H, W, G, OH, OW);
  return (int)hipGetLastError();
}

PLX_API int plx_maxpool3s2_backward(const void* dy, const void* idx, void* dx, int N, int H, int W, int C,
                                    hipStream_t s) {
  if (C % 8 || N <= 0 || H <= 0 || W <= 0) return 1;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1, G = C / 8;
  hipLaunchKernelGGL(maxpool_bwd_kernel, dim3(grid_for((int64_t)N * H * W * G)), dim3(256), 0, s,
                     (const bf16x8*)dy, (const u8x8*)idx, (bf16x8*)dx, N, H, W, G, OH, OW);
  return (int)hipGetLastError();
}
