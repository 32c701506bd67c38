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
__device__ __forceinline__ uint16_t f2bf(float f) {  // hardware RNE conversion, NaN stays NaN
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

// Grid: x = 8-channel groups of one image row (256 per block), y = image rows (n, h) with a stride loop.  All
// index math is 32-bit and the row split is per block (scalar): the first version decoded a flat int64 element
// index with three 64-bit div/mods per thread, which made the stem-pool backward ALU-bound (380 us against a
// ~100 us HBM floor on 256x112x112x64).

// one thread = 8 channels of one output pixel
__global__ __launch_bounds__(256) void maxpool_fwd_kernel(const bf16x8* __restrict__ x, bf16x8* __restrict__ y,
                                                          u8x8* __restrict__ idx, int N, int H, int W, int G, int OH,
                                                          int OW) {
  const unsigned j = blockIdx.x * 256u + threadIdx.x;
  if (j >= (unsigned)(OW * G)) return;
  const unsigned g = j % (unsigned)G, ow = j / (unsigned)G;
  for (int row = blockIdx.y; row < N * OH; row += gridDim.y) {
    const int n = row / OH, oh = row - n * OH;
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
      const bf16x8* xr = x + ((size_t)(n * H + ih) * W) * G + g;
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = (int)ow * 2 - 1 + kw;
        if (iw < 0 || iw >= W) continue;
        const bf16x8 v = xr[(size_t)iw * G];
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
    const size_t t = (size_t)row * OW * G + j;
    y[t] = o;
    idx[t] = a;
  }
}

// one thread = 8 channels of one input pixel.  Input row ih is covered by output rows oh = (ih+1-kh)/2 for the
// kh in 0..2 of matching parity: ih even -> (ih/2, kh=1); ih odd -> ((ih+1)/2, kh=0) and ((ih-1)/2, kh=2).
__device__ __forceinline__ int pool_cover(int i, int O, int* o, int* k) {
  int n = 0;
  if (i & 1) {
    if ((i + 1) >> 1 < O) { o[n] = (i + 1) >> 1; k[n++] = 0; }
    o[n] = (i - 1) >> 1; k[n++] = 2;
  } else if ((i >> 1) < O) {
    o[n] = i >> 1; k[n++] = 1;
  }
  return n;
}

__global__ __launch_bounds__(256) void maxpool_bwd_kernel(const bf16x8* __restrict__ dy, const u8x8* __restrict__ idx,
                                                          bf16x8* __restrict__ dx, int N, int H, int W, int G, int OH,
                                                          int OW) {
  const unsigned j = blockIdx.x * 256u + threadIdx.x;
  if (j >= (unsigned)(W * G)) return;
  const unsigned g = j % (unsigned)G;
  const int iw = (int)(j / (unsigned)G);
  int ows[2], kws[2];
  const int nw = pool_cover(iw, OW, ows, kws);
  for (int row = blockIdx.y; row < N * H; row += gridDim.y) {
    const int n = row / H, ih = row - n * H;
    int ohs[2], khs[2];
    const int nh = pool_cover(ih, OH, ohs, khs);
    // all (<= 4) covering windows' argmax bytes and dy vectors are loaded up front as independent loads (a
    // missing window re-reads a valid one and is masked out): the load -> test -> dependent-load chain per
    // window left the kernel latency-bound at ~1.4 TB/s
    size_t off[4];
    bool valid[4];
    uint8_t me[4];
#pragma unroll
    for (int a = 0; a < 2; ++a)
#pragma unroll
      for (int b = 0; b < 2; ++b) {
        const int q = a * 2 + b;
        valid[q] = a < nh && b < nw;
        const int oh = ohs[a < nh ? a : 0], ow = ows[b < nw ? b : 0];
        off[q] = ((size_t)(n * OH + oh) * OW + ow) * G + g;
        me[q] = (uint8_t)(khs[a < nh ? a : 0] * 3 + kws[b < nw ? b : 0]);
      }
    u8x8 am[4];
    bf16x8 d[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      am[q] = idx[off[q]];
      d[q] = dy[off[q]];
    }
    float acc[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      float v = 0.f;
#pragma unroll
      for (int q = 0; q < 4; ++q)
        if (valid[q] && am[q].v[k] == me[q]) v += bf2f(d[q].v[k]);
      acc[k] = v;
    }
    bf16x8 out;
#pragma unroll
    for (int k = 0; k < 8; ++k) out.v[k] = f2bf(acc[k]);
    dx[(size_t)row * W * G + j] = out;
  }
}

inline dim3 grid_for(int row_elems, int rows) {
  return dim3((row_elems + 255) / 256, rows < 65535 ? rows : 65535);
}

// Global average pool over H x W of NHWC bf16 x [N][HW][C] (the ResNet head): one thread = 8 channels of one image,
// fp32 sums over the HW pixels (each a coalesced 16-byte row read across the threads), the mean rounded to bf16.
__global__ __launch_bounds__(256) void gap_fwd_kernel(const bf16x8* __restrict__ x, bf16x8* __restrict__ y, int N, int HW,
                                                      int G, float inv) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // (n, g)
  if (i >= N * G) return;
  const int n = i / G, g = i - n * G;
  const bf16x8* p = x + (size_t)n * HW * G + g;
  float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
  for (int k = 0; k < HW; ++k) {
    const bf16x8 v = p[(size_t)k * G];
#pragma unroll
    for (int j = 0; j < 8; ++j) acc[j] += bf2f(v.v[j]);
  }
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.v[j] = f2bf(acc[j] * inv);
  y[i] = o;
}

// its backward: dx[n][k][c] = dy[n][c] / HW for every pixel k, one 16-byte store per thread and pixel
__global__ __launch_bounds__(256) void gap_bwd_kernel(const bf16x8* __restrict__ dy, bf16x8* __restrict__ dx, int N, int HW,
                                                      int G, float inv) {
  const int i = blockIdx.x * 256 + threadIdx.x;  // (n, g)
  if (i >= N * G) return;
  const int n = i / G, g = i - n * G;
  const bf16x8 v = dy[i];
  bf16x8 o;
#pragma unroll
  for (int j = 0; j < 8; ++j) o.v[j] = f2bf(bf2f(v.v[j]) * inv);
  bf16x8* q = dx + (size_t)n * HW * G + g;
  for (int k = 0; k < HW; ++k) q[(size_t)k * G] = o;
}

}  // namespace

// y[N][C] = mean over the HW pixels of x[N][HW][C] (NHWC bf16, C % 8 == 0, 16-byte aligned)
PLX_API int plx_gap_forward(const void* x, void* y, int N, int HW, int C, hipStream_t s) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % 8) return 1;
  const int G = C / 8;
  hipLaunchKernelGGL(gap_fwd_kernel, dim3((N * G + 255) / 256), dim3(256), 0, s, (const bf16x8*)x, (bf16x8*)y, N, HW, G,
                     1.f / (float)HW);
  return (int)hipGetLastError();
}

// dx[N][HW][C] = dy[N][C] / HW broadcast over the pixels (bf16)
PLX_API int plx_gap_backward(const void* dy, void* dx, int N, int HW, int C, hipStream_t s) {
  if (N <= 0 || HW <= 0 || C <= 0 || C % 8) return 1;
  const int G = C / 8;
  hipLaunchKernelGGL(gap_bwd_kernel, dim3((N * G + 255) / 256), dim3(256), 0, s, (const bf16x8*)dy, (bf16x8*)dx, N, HW, G,
                     1.f / (float)HW);
  return (int)hipGetLastError();
}

PLX_API int plx_maxpool3s2_forward(const void* x, void* y, void* idx, int N, int H, int W, int C, hipStream_t s) {
  if (C % 8 || N <= 0 || H <= 0 || W <= 0) return 1;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1, G = C / 8;
  hipLaunchKernelGGL(maxpool_fwd_kernel, grid_for(OW * G, N * OH), dim3(256), 0, s,
                     (const bf16x8*)x, (bf16x8*)y, (u8x8*)idx, N, H, W, G, OH, OW);
  return (int)hipGetLastError();
}

PLX_API int plx_maxpool3s2_backward(const void* dy, const void* idx, void* dx, int N, int H, int W, int C,
                                    hipStream_t s) {
  if (C % 8 || N <= 0 || H <= 0 || W <= 0) return 1;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1, G = C / 8;
  hipLaunchKernelGGL(maxpool_bwd_kernel, grid_for(W * G, N * H), dim3(256), 0, s,
                     (const bf16x8*)dy, (const u8x8*)idx, (bf16x8*)dx, N, H, W, G, OH, OW);
  return (int)hipGetLastError();
}
