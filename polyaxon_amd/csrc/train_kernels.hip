// Trial-executor kernels for the resident (warm) trial runtime on MI355X (gfx950).
//
// The reference (Polyaxon 0.2.8) never touches the training step: each trial is a pod running user
// code (polyaxon/scheduler/spawners/experiment_spawner.py:108-179).  The MI355X-native executor keeps
// one warm process per GPU and replays a captured hipGraph for every trial, so everything that differs
// between trials (hyper-parameters, weights, optimizer state, step counter) must live in device memory
// and be (re)written by kernels, never by re-capturing.  This file provides those kernels:
//
//   plx_sgd_flat      fused SGD(momentum, nesterov, decoupled-from-BN weight decay) over ONE flat fp32
//                     parameter/grad/momentum buffer; reads hyper-parameters from device memory and zeroes
//                     the gradient in the same pass (no separate zero_grad memset).
//   plx_adamw_flat    fused AdamW over flat buffers, bias correction from a device step counter.
//   plx_init_flat     re-initialises every parameter segment in one launch (Philox4x32-10 normal /
//                     uniform / constant) so a new trial starts from fresh random weights in-place.
//   plx_record_metric appends the step loss to a device ring and advances the device step counter.
//   plx_commit_metric reduces the last `window` ring entries into a slot of the HPO metric tensor.
//
// All memory-bound kernels use 16-byte (float4) accesses and a grid capped at 2048 blocks with a
// grid-stride loop (cdna_hip_programming.md Guideline 11/13).
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kBlock = 256;

inline int grid_for(int64_t n_vec, int cap = 2048) {
  int64_t g = (n_vec + kBlock - 1) / kBlock;
  if (g > cap) g = cap;
  if (g < 1) g = 1;
  return (int)g;
}

// Block cap of the AdamW launches (plx_set_adamw_grid_cap; measured for the update inside the
// backward, parallel/ddp.py FlatDDP(optimizer=...)).  That update is HBM-bound like the backward's elementwise
// kernels: with the full grid those ran 2-40x slower beside it; capped at 32 / 64 / 128 / 256 blocks the update
// outlasted the backward (Llama-3 8B 13.4k / 16.1k / 17.5k / 17.8k vs 17.8k tokens/s without it, same box).
int g_adamw_grid_cap = 2048;

// ---------------------------------------------------------------- SGD
// hp layout (fp32, device): [0] lr, [1] momentum, [2] weight_decay, [3] nesterov (0/1), [4] dampening
// Elements [0, n_decay) receive weight decay (conv / linear weights), [n_decay, n) do not (BN, bias).
__global__ __launch_bounds__(kBlock) void sgd_flat_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                          float4* __restrict__ m, int64_t n_vec,
                                                          int64_t n_decay_vec, const float* __restrict__ hp,
                                                          const int* __restrict__ first_step) {
  const float lr = hp[0], mom = hp[1], wd = hp[2], damp = hp[4];
  const bool nesterov = hp[3] != 0.f;
  // First step after (re)initialisation: momentum buffer := grad (torch.optim.SGD semantics).
  const bool first = first_step != nullptr && *first_step == 0;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
    float4 pv = p[i], gv = g[i], mv = m[i];
    const float w = i < n_decay_vec ? wd : 0.f;
    float gg[4] = {gv.x + w * pv.x, gv.y + w * pv.y, gv.z + w * pv.z, gv.w + w * pv.w};
    float mm[4] = {mv.x, mv.y, mv.z, mv.w};
    float pp[4] = {pv.x, pv.y, pv.z, pv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mm[k] = first ? gg[k] : mom * mm[k] + (1.f - damp) * gg[k];
      const float d = nesterov ? gg[k] + mom * mm[k] : mm[k];
      pp[k] -= lr * d;
    }
    p[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
    m[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// ---------------------------------------------------------------- AdamW
// hp layout: [0] lr, [1] beta1, [2] beta2, [3] eps, [4] weight_decay. step = *step_ptr + 1.
__global__ __launch_bounds__(kBlock) void adamw_flat_kernel(float4* __restrict__ p, float4* __restrict__ g,
                                                            float4* __restrict__ m, float4* __restrict__ v,
                                                            int64_t n_vec, int64_t n_decay_vec,
                                                            const float* __restrict__ hp,
                                                            const int* __restrict__ step_ptr) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4];
  const float t = (float)(*step_ptr + 1);
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  const float step_size = lr / bc1, inv_sqrt_bc2 = rsqrtf(bc2);
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
    float4 pv = p[i], gv = g[i], mv = m[i], vv = v[i];
    const float decay = i < n_decay_vec ? (1.f - lr * wd) : 1.f;
    float pp[4] = {pv.x, pv.y, pv.z, pv.w}, gg[4] = {gv.x, gv.y, gv.z, gv.w};
    float mm[4] = {mv.x, mv.y, mv.z, mv.w}, vq[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      mm[k] = b1 * mm[k] + (1.f - b1) * gg[k];
      vq[k] = b2 * vq[k] + (1.f - b2) * gg[k] * gg[k];
      const float denom = sqrtf(vq[k]) * inv_sqrt_bc2 + eps;
      pp[k] = pp[k] * decay - step_size * mm[k] / denom;
    }
    p[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
    m[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    v[i] = make_float4(vq[0], vq[1], vq[2], vq[3]);
    g[i] = make_float4(0.f, 0.f, 0.f, 0.f);
  }
}

// Mixed-precision AdamW for the language models (ops/flat.py lp mode): the model computes with bf16 weights
// (views into `plp`) and produces bf16 gradients (`g`, zeroed here after use); the fp32 master copy `p` and the
// moments stay fp32.  One pass: read p, g, m, v (14 B/elem), write p, m, v, plp and g (16 B/elem) -- no
// separate fp32->bf16 weight cast per forward and no bf16->fp32 gradient cast per backward.
// `decay` applies weight decay to the whole range (callers pass the decay segment only).
typedef unsigned short u16x4 __attribute__((ext_vector_type(4)));

__device__ __forceinline__ float bf16_to_f(unsigned short h) { return __uint_as_float((uint32_t)h << 16); }

__device__ __forceinline__ unsigned short f_to_bf16(float f) {  // hardware RNE conversion (v_cvt_pk_bf16_f32)
  return __builtin_bit_cast(unsigned short, (__bf16)f);
}

// One mixed-precision AdamW element, with every rounding step explicit (no contraction left to the compiler), so the
// 4-wide and 8-wide kernels -- and per-bucket launches that mix them -- give bitwise the same update
__device__ __forceinline__ float adamw_elem(float p, float& m, float& v, float g, float b1, float b2, float eps,
                                            float step_size, float inv_sqrt_bc2, float decay) {
#pragma clang fp contract(off)
  m = fmaf(b1, m, (1.f - b1) * g);
  v = fmaf(b2, v, ((1.f - b2) * g) * g);
  const float denom = fmaf(sqrtf(v), inv_sqrt_bc2, eps);
  return fmaf(p, decay, -((step_size * m) / denom));
}

__global__ __launch_bounds__(kBlock) void adamw_mixed_kernel(float4* __restrict__ p, u16x4* __restrict__ g,
                                                             float4* __restrict__ m, float4* __restrict__ v,
                                                             u16x4* __restrict__ plp, int64_t n_vec, int decay_on,
                                                             const float* __restrict__ hp,
                                                             const int* __restrict__ step_ptr) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4];
  const float t = (float)(*step_ptr + 1);
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  const float step_size = lr / bc1, inv_sqrt_bc2 = rsqrtf(bc2);
  const float decay = decay_on ? (1.f - lr * wd) : 1.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
    const float4 pv = p[i], mv = m[i], vv = v[i];
    const u16x4 gv = g[i];
    float pp[4] = {pv.x, pv.y, pv.z, pv.w}, mm[4] = {mv.x, mv.y, mv.z, mv.w}, vq[4] = {vv.x, vv.y, vv.z, vv.w};
    u16x4 lo;
#pragma unroll
    for (int k = 0; k < 4; ++k) {
      pp[k] = adamw_elem(pp[k], mm[k], vq[k], bf16_to_f(gv[k]), b1, b2, eps, step_size, inv_sqrt_bc2, decay);
      lo[k] = f_to_bf16(pp[k]);
    }
    p[i] = make_float4(pp[0], pp[1], pp[2], pp[3]);
    m[i] = make_float4(mm[0], mm[1], mm[2], mm[3]);
    v[i] = make_float4(vq[0], vq[1], vq[2], vq[3]);
    plp[i] = lo;
    g[i] = u16x4{0, 0, 0, 0};
  }
}

// Same update, 8 elements per thread: the bf16 gradient / model-copy accesses become 16-B vectors (4 x 16 B + 2 x
// 16 B per lane instead of 3 x 16 B + 3 x 8 B per 4 elements) and every stream is non-temporal -- each of the ~30 B
// per parameter is touched once per step, far past the caches.  Used when n % 8 == 0 and every pointer is 16-B
// aligned (plx_set_adamw_wide A/B knob).
typedef float f32x4v __attribute__((ext_vector_type(4)));
typedef unsigned short u16x8v __attribute__((ext_vector_type(8)));

template <bool NT>
__global__ __launch_bounds__(kBlock) void adamw_mixed8_kernel(f32x4v* __restrict__ p, u16x8v* __restrict__ g,
                                                              f32x4v* __restrict__ m, f32x4v* __restrict__ v,
                                                              u16x8v* __restrict__ plp, int64_t n8, int decay_on,
                                                              const float* __restrict__ hp,
                                                              const int* __restrict__ step_ptr) {
  const float lr = hp[0], b1 = hp[1], b2 = hp[2], eps = hp[3], wd = hp[4];
  const float t = (float)(*step_ptr + 1);
  const float bc1 = 1.f - __powf(b1, t), bc2 = 1.f - __powf(b2, t);
  const float step_size = lr / bc1, inv_sqrt_bc2 = rsqrtf(bc2);
  const float decay = decay_on ? (1.f - lr * wd) : 1.f;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n8; i += stride) {
    f32x4v pv[2], mv[2], vv[2];
#pragma unroll
    for (int h = 0; h < 2; ++h) {
      pv[h] = NT ? __builtin_nontemporal_load(p + 2 * i + h) : p[2 * i + h];
      mv[h] = NT ? __builtin_nontemporal_load(m + 2 * i + h) : m[2 * i + h];
      vv[h] = NT ? __builtin_nontemporal_load(v + 2 * i + h) : v[2 * i + h];
    }
    const u16x8v gv = NT ? __builtin_nontemporal_load(g + i) : g[i];
    u16x8v lo;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const int h = k >> 2, e = k & 3;
      float mk = mv[h][e], vk = vv[h][e];
      const float pk = adamw_elem(pv[h][e], mk, vk, bf16_to_f(gv[k]), b1, b2, eps, step_size, inv_sqrt_bc2, decay);
      mv[h][e] = mk;
      vv[h][e] = vk;
      pv[h][e] = pk;
      lo[k] = f_to_bf16(pk);
    }
    if constexpr (NT) {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        __builtin_nontemporal_store(pv[h], p + 2 * i + h);
        __builtin_nontemporal_store(mv[h], m + 2 * i + h);
        __builtin_nontemporal_store(vv[h], v + 2 * i + h);
      }
      __builtin_nontemporal_store(lo, plp + i);
      __builtin_nontemporal_store(u16x8v{0, 0, 0, 0, 0, 0, 0, 0}, g + i);
    } else {
#pragma unroll
      for (int h = 0; h < 2; ++h) {
        p[2 * i + h] = pv[h];
        m[2 * i + h] = mv[h];
        v[2 * i + h] = vv[h];
      }
      plp[i] = lo;
      g[i] = u16x8v{0, 0, 0, 0, 0, 0, 0, 0};
    }
  }
}

int g_adamw_wide = 0;

// fp32 master -> bf16 model copy (after re-initialisation, checkpoint load or a parameter broadcast)
__global__ __launch_bounds__(kBlock) void cast_lp_kernel(const float4* __restrict__ p, u16x4* __restrict__ plp,
                                                         int64_t n_vec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride) {
    const float4 pv = p[i];
    plp[i] = u16x4{f_to_bf16(pv.x), f_to_bf16(pv.y), f_to_bf16(pv.z), f_to_bf16(pv.w)};
  }
}

// ---------------------------------------------------------------- Philox4x32-10
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox(U4 c, uint32_t k0, uint32_t k1) {
#pragma unroll
  for (int r = 0; r < 10; ++r) {
    const uint32_t lo0 = 0xD2511F53u * c.x, hi0 = __umulhi(0xD2511F53u, c.x);
    const uint32_t lo1 = 0xCD9E8D57u * c.z, hi1 = __umulhi(0xCD9E8D57u, c.z);
    c = U4{hi1 ^ c.y ^ k0, lo1, hi0 ^ c.w ^ k1, lo0};
    k0 += 0x9E3779B9u;
    k1 += 0xBB67AE85u;
  }
  return c;
}

__device__ __forceinline__ float u01(uint32_t x) {  // (0, 1]
  return ((float)(x >> 8) + 1.0f) * (1.0f / 16777216.0f);
}

// Segment table (device): per chunk -> (segment start, chunk begin, chunk end); per segment kind/scale.
// kind 0: normal(0, scale); 1: constant(scale); 2: uniform(-scale, scale).
__global__ __launch_bounds__(kBlock) void init_flat_kernel(float* __restrict__ p, const int64_t* __restrict__ chunk_lo,
                                                           const int64_t* __restrict__ chunk_hi,
                                                           const int* __restrict__ chunk_seg,
                                                           const int* __restrict__ seg_kind,
                                                           const float* __restrict__ seg_scale, uint64_t seed) {
  const int c = blockIdx.x;
  const int64_t lo = chunk_lo[c], hi = chunk_hi[c];
  const int s = chunk_seg[c];
  const int kind = seg_kind[s];
  const float scale = seg_scale[s];
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  for (int64_t base = lo + 4 * (int64_t)threadIdx.x; base < hi; base += 4 * (int64_t)blockDim.x) {
    float vals[4];
    if (kind == 1) {
      vals[0] = vals[1] = vals[2] = vals[3] = scale;
    } else {
      const uint64_t ctr = (uint64_t)base >> 2;
      U4 r = philox(U4{(uint32_t)ctr, (uint32_t)(ctr >> 32), 0x5eedu, 0u}, k0, k1);
      if (kind == 0) {
        const float r1 = sqrtf(-2.f * __logf(u01(r.x))), r2 = sqrtf(-2.f * __logf(u01(r.z)));
        float sn, cs, sn2, cs2;
        __sincosf(6.2831853f * u01(r.y), &sn, &cs);
        __sincosf(6.2831853f * u01(r.w), &sn2, &cs2);
        vals[0] = scale * r1 * cs;
        vals[1] = scale * r1 * sn;
        vals[2] = scale * r2 * cs2;
        vals[3] = scale * r2 * sn2;
      } else {
        vals[0] = scale * (2.f * u01(r.x) - 1.f);
        vals[1] = scale * (2.f * u01(r.y) - 1.f);
        vals[2] = scale * (2.f * u01(r.z) - 1.f);
        vals[3] = scale * (2.f * u01(r.w) - 1.f);
      }
    }
#pragma unroll
    for (int k = 0; k < 4; ++k)
      if (base + k < hi) p[base + k] = vals[k];
  }
}

// ---------------------------------------------------------------- synthetic learnable ImageNet-shape batches
// A fresh batch per training step, generated on the device (no host->device copy, no fixed batch to memorise):
//   y[b]          = Philox(seed; b, step) mod n_cls
//   x[b,h,w,c]    = signal * proto[y[b]][h*G/H][w*G/W][c] + N(0, 1)        (NHWC / channels_last, bf16)
// so the label is a function of a coarse G x G x 3 class pattern buried in unit noise: learnable, never repeated.
// `counter` (device int) is the data-stream position; it is read here and advanced by counter_add_kernel, so the
// pair is graph-capturable.  Each thread writes 8 consecutive bf16 (16-B store); H*W*3 % 8 == 0 is required so
// an 8-element chunk never straddles two images (the host entry point checks it).
typedef unsigned short u16x8 __attribute__((ext_vector_type(8)));

// The pattern cell of a pixel, gh = h * G / H and gw = w * G / W, comes from a per-block LDS table built once
// (H + W shorts) instead of two runtime integer divisions per element: the 8 elements of a chunk span <= 4 pixels of
// one or two rows, so the chunk walks (h, w) incrementally.  (The first version divided per element -- 24 runtime
// divisions per 16-B store -- and ran 152 us per bs-256 224^2 batch, compute-bound, beside the backward's tail.)
__global__ __launch_bounds__(kBlock) void synth_images_kernel(u16x8* __restrict__ x, int64_t* __restrict__ y, int B,
                                                              int H, int W, const float* __restrict__ proto,
                                                              int n_cls, int G, float signal, uint64_t seed,
                                                              const int* __restrict__ counter) {
  extern __shared__ short gtab[];  // [H] row cells, then [W] column cells
  for (int i = threadIdx.x; i < H + W; i += blockDim.x)
    gtab[i] = (short)(i < H ? i * G / H : (i - H) * G / W);
  __syncthreads();
  const short* gy = gtab;
  const short* gx = gtab + H;
  const uint32_t k0 = (uint32_t)seed, k1 = (uint32_t)(seed >> 32);
  const uint32_t step = (uint32_t)(*counter);
  const int64_t per_img = (int64_t)H * W * 3;
  const int64_t n8 = (int64_t)B * per_img / 8;
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t t = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; t < n8; t += stride) {
    const int64_t i0 = t * 8;
    const int b = (int)(i0 / per_img);
    const U4 lr = philox(U4{(uint32_t)b, step, 0x1abe1u, 0u}, k0, k1);
    const int label = (int)(lr.x % (uint32_t)n_cls);
    const int64_t rem = i0 - (int64_t)b * per_img;
    if (rem == 0) y[b] = label;
    const U4 r0 = philox(U4{(uint32_t)t, (uint32_t)(t >> 32), step, 0xda7a0u}, k0, k1);
    const U4 r1 = philox(U4{(uint32_t)t, (uint32_t)(t >> 32), step, 0xda7a1u}, k0, k1);
    const uint32_t ur[8] = {r0.x, r0.y, r0.z, r0.w, r1.x, r1.y, r1.z, r1.w};
    float nz[8];
#pragma unroll
    for (int k = 0; k < 4; ++k) {  // Box-Muller: 2 normals per pair of uniforms
      const float rad = sqrtf(-2.f * __logf(u01(ur[2 * k])));
      float sn, cs;
      __sincosf(6.2831853f * u01(ur[2 * k + 1]), &sn, &cs);
      nz[2 * k] = rad * cs;
      nz[2 * k + 1] = rad * sn;
    }
    const float* pl = proto + (int64_t)label * G * G * 3;
    const int pix = (int)(rem / 3);
    int c = (int)(rem - (int64_t)pix * 3);
    int h = pix / W, w = pix - h * W;
    int row = gy[h] * G;
    u16x8 out;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      out[k] = f_to_bf16(signal * pl[(row + gx[w]) * 3 + c] + nz[k]);
      if (++c == 3) {
        c = 0;
        if (++w == W) {
          w = 0;
          ++h;
          if (h < H) row = gy[h] * G;  // h == H only after the image's last element
        }
      }
    }
    x[t] = out;
  }
}

__global__ void counter_add_kernel(int* __restrict__ c, int v) {
  if (threadIdx.x == 0 && blockIdx.x == 0) *c += v;
}

__global__ void zero_kernel(float4* __restrict__ x, int64_t n_vec) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  for (int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n_vec; i += stride)
    x[i] = make_float4(0.f, 0.f, 0.f, 0.f);
}

// ---------------------------------------------------------------- metric ring
// loss: one scalar (fp32 or bf16 bits selected by is_bf16). ring[step % ring_size] = loss; ++step.
__global__ void record_metric_kernel(const void* __restrict__ loss, int is_bf16, float* __restrict__ ring,
                                     int* __restrict__ step, int ring_size) {
  if (threadIdx.x == 0 && blockIdx.x == 0) {
    float v;
    if (is_bf16) {
      const uint16_t b = *reinterpret_cast<const uint16_t*>(loss);
      v = __uint_as_float(((uint32_t)b) << 16);
    } else {
      v = *reinterpret_cast<const float*>(loss);
    }
    const int s = *step;
    ring[s % ring_size] = v;
    *step = s + 1;
  }
}

// out[slot] = mean of the last `window` ring entries ending at step-1 (NaN if no steps ran).
__global__ void commit_metric_kernel(const float* __restrict__ ring, const int* __restrict__ step, int ring_size,
                                     int window, float* __restrict__ out, int slot) {
  __shared__ float part[64];
  const int s = *step;
  const int w = window < s ? window : s;
  float acc = 0.f;
  for (int j = threadIdx.x; j < w; j += blockDim.x) acc += ring[(s - 1 - j) % ring_size];
  for (int off = 32; off > 0; off >>= 1) acc += __shfl_down(acc, off, 64);
  if ((threadIdx.x & 63) == 0) part[threadIdx.x >> 6] = acc;
  __syncthreads();
  if (threadIdx.x == 0) {
    float t = 0.f;
    for (int k = 0; k < (int)(blockDim.x >> 6); ++k) t += part[k];
    out[slot] = w > 0 ? t / (float)w : __builtin_nanf("");
  }
}

}  // namespace

PLX_API int plx_sgd_flat(float* p, float* g, float* m, int64_t n, int64_t n_decay, const float* hp,
                         const int* first_step, hipStream_t stream) {
  if ((n & 3) || (n_decay & 3)) return 1;  // caller pads flat buffers to a multiple of 4 floats
  const int64_t nv = n >> 2;
  hipLaunchKernelGGL(sgd_flat_kernel, dim3(grid_for(nv)), dim3(kBlock), 0, stream, (float4*)p, (float4*)g,
                     (float4*)m, nv, n_decay >> 2, hp, first_step);
  return (int)hipGetLastError();
}

PLX_API int plx_adamw_flat(float* p, float* g, float* m, float* v, int64_t n, int64_t n_decay, const float* hp,
                           const int* step, hipStream_t stream) {
  if ((n & 3) || (n_decay & 3)) return 1;
  const int64_t nv = n >> 2;
  hipLaunchKernelGGL(adamw_flat_kernel, dim3(grid_for(nv, g_adamw_grid_cap)), dim3(kBlock), 0, stream, (float4*)p, (float4*)g,
                     (float4*)m, (float4*)v, nv, n_decay >> 2, hp, step);
  return (int)hipGetLastError();
}

// A/B knob: 8-wide mixed-precision AdamW with non-temporal streams (1), with plain loads / stores (2), or the
// 4-wide kernel (0, default)
PLX_API void plx_set_adamw_wide(int on) { g_adamw_wide = on < 0 ? 0 : (on > 2 ? 2 : on); }

PLX_API void plx_set_adamw_grid_cap(int blocks) { g_adamw_grid_cap = blocks < 1 ? 1 : (blocks > 2048 ? 2048 : blocks); }

PLX_API int plx_adamw_mixed(float* p, void* g, float* m, float* v, void* plp, int64_t n, int decay_on,
                            const float* hp, const int* step, hipStream_t stream) {
  if (n & 3) return 1;
  const bool aligned = ((uintptr_t)p | (uintptr_t)g | (uintptr_t)m | (uintptr_t)v | (uintptr_t)plp) % 16 == 0;
  if (g_adamw_wide && (n & 7) == 0 && aligned) {
    const int64_t n8 = n >> 3;
    hipLaunchKernelGGL(g_adamw_wide == 2 ? adamw_mixed8_kernel<false> : adamw_mixed8_kernel<true>, dim3(grid_for(n8, g_adamw_grid_cap)), dim3(kBlock), 0, stream,
                       (f32x4v*)p, (u16x8v*)g, (f32x4v*)m, (f32x4v*)v, (u16x8v*)plp, n8, decay_on, hp, step);
    return (int)hipGetLastError();
  }
  const int64_t nv = n >> 2;
  hipLaunchKernelGGL(adamw_mixed_kernel, dim3(grid_for(nv, g_adamw_grid_cap)), dim3(kBlock), 0, stream, (float4*)p, (u16x4*)g,
                     (float4*)m, (float4*)v, (u16x4*)plp, nv, decay_on, hp, step);
  return (int)hipGetLastError();
}

PLX_API int plx_cast_lp(const float* p, void* plp, int64_t n, hipStream_t stream) {
  if (n & 3) return 1;
  hipLaunchKernelGGL(cast_lp_kernel, dim3(grid_for(n >> 2)), dim3(kBlock), 0, stream, (const float4*)p,
                     (u16x4*)plp, n >> 2);
  return (int)hipGetLastError();
}

PLX_API int plx_init_flat(float* p, const int64_t* chunk_lo, const int64_t* chunk_hi, const int* chunk_seg,
                          int n_chunks, const int* seg_kind, const float* seg_scale, uint64_t seed,
                          hipStream_t stream) {
  if (n_chunks <= 0) return 0;
  hipLaunchKernelGGL(init_flat_kernel, dim3(n_chunks), dim3(kBlock), 0, stream, p, chunk_lo, chunk_hi, chunk_seg,
                     seg_kind, seg_scale, seed);
  return (int)hipGetLastError();
}

PLX_API int plx_synth_images(void* x, int64_t* y, int B, int H, int W, const float* proto, int n_cls, int G,
                             float signal, uint64_t seed, int* counter, hipStream_t stream) {
  const int64_t per_img = (int64_t)H * W * 3;
  if (B <= 0 || per_img % 8 || n_cls <= 0 || G <= 0 || G > H || G > W) return 1;
  const int64_t n8 = (int64_t)B * per_img / 8;
  if ((int64_t)(H + W) * 2 > 32768) return 1;  // the cell table lives in LDS
  hipLaunchKernelGGL(synth_images_kernel, dim3(grid_for(n8, 8192)), dim3(kBlock), (H + W) * sizeof(short), stream,
                     (u16x8*)x, y, B, H, W, proto, n_cls, G, signal, seed, (const int*)counter);
  hipLaunchKernelGGL(counter_add_kernel, dim3(1), dim3(64), 0, stream, counter, 1);
  return (int)hipGetLastError();
}

PLX_API int plx_zero_flat(float* x, int64_t n, hipStream_t stream) {
  if (n & 3) return 1;
  hipLaunchKernelGGL(zero_kernel, dim3(grid_for(n >> 2)), dim3(kBlock), 0, stream, (float4*)x, n >> 2);
  return (int)hipGetLastError();
}

PLX_API int plx_record_metric(const void* loss, int is_bf16, float* ring, int* step, int ring_size,
                              hipStream_t stream) {
  hipLaunchKernelGGL(record_metric_kernel, dim3(1), dim3(64), 0, stream, loss, is_bf16, ring, step, ring_size);
  return (int)hipGetLastError();
}

PLX_API int plx_commit_metric(const float* ring, const int* step, int ring_size, int window, float* out, int slot,
                              hipStream_t stream) {
  hipLaunchKernelGGL(commit_metric_kernel, dim3(1), dim3(256), 0, stream, ring, step, ring_size, window, out, slot);
  return (int)hipGetLastError();
}
