// Fused BatchNorm(+residual add)(+ReLU) for NHWC bf16 activations on MI355X (gfx950).
//
// A ResNet-50 training step runs 53 BatchNorms, 49 of them followed by ReLU and 16 by a residual add
// first.  Unfused, that is stats + normalise + add + relu in the forward and relu-backward + BN-backward
// (+ the add's gradient copy) in the backward: 7-9 full passes over each activation, all HBM-bound.
// These kernels do it in 2 passes forward (stats, apply) and 2 backward (reduce, dx), 16-byte vectors
// (8 x bf16) per lane, fp32 math, fp32 per-channel partials.
//
// Layout: x viewed as [M, C] row-major, M = N*H*W (channels_last), C % 8 == 0 and C/8 a power of two.
// Thread t of a 256-thread block owns channel group cg = t % Gb (8 channels, Gb = min(C/8, 256)) and row
// lane t / Gb, so its per-channel state (shift, scale, bias, mean, invstd) stays in registers while it
// walks rows; one wave reads 64 x 16 B = 1 KiB contiguous per instruction.
//
//   plx_bn_fwd_stats     per-block shifted sum / sum-of-squares partials  [nblk, C] (+ level-2 reduce)
//   plx_bn_fwd_finalize  mean, invstd, fused scale/bias, running-stat update (unbiased var)
//   plx_bn_fwd_apply     y = act(x*scale + bias [+ res])
//   plx_bn_bwd_reduce    partial sums of dz and dz*xhat   (dz = dy * [y > 0] when act)
//   plx_bn_bwd_finalize  dgamma, dbeta and the dx coefficients  dx = A*dz + B*x + D
//   plx_bn_bwd_dx        dx (and d_residual = dz) in one pass, optionally with the reduction partials of the
//                        BatchNorm that produced the residual (ResBn: a downsampling branch's BN skips its reduce)
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

__device__ __forceinline__ uint16_t f2bf(float f) {  // round-to-nearest-even, NaN stays NaN
  // a plain cast: hipcc emits v_cvt_pk_bf16_f32 (MI355X_MICROARCH.md, correctness table) -- one instruction where the
  // integer form was ~6, which showed in the VALU-heavy passes (fused stem forward 342 -> 284 us)
  return __builtin_bit_cast(uint16_t, (__bf16)f);
}

__device__ __forceinline__ void load8(const bf16x8* p, float* f) {
  const bf16x8 v = *p;
#pragma unroll
  for (int k = 0; k < 8; ++k) f[k] = bf2f(v.v[k]);
}

__device__ __forceinline__ void store8(bf16x8* p, const float* f) {
  bf16x8 v;
#pragma unroll
  for (int k = 0; k < 8; ++k) v.v[k] = f2bf(f[k]);
  *p = v;
}

// ------------------------------------------------------------------------------- forward stats
__global__ __launch_bounds__(kBlock) void bn_stats_kernel(const bf16x8* __restrict__ x, int64_t M, int G, int Gb,
                                                          int64_t rows_per_block, float* __restrict__ psum,
                                                          float* __restrict__ psq) {
  __shared__ float s_sum[kBlock * 8];
  __shared__ float s_sq[kBlock * 8];
  const int tid = threadIdx.x;
  const int cg_local = tid % Gb, rlane = tid / Gb, R = kBlock / Gb;
  const int cg = blockIdx.y * Gb + cg_local;
  const int C = G * 8;
  float shift[8], s[8], q[8];
  load8(x + cg, shift);  // row 0 as the shift: var = E[(x-k)^2] - E[x-k]^2 stays well conditioned
#pragma unroll
  for (int k = 0; k < 8; ++k) s[k] = q[k] = 0.f;
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
#pragma unroll 4
  for (int64_t r = r0 + rlane; r < r1; r += R) {
    float v[8];
    load8(x + r * G + cg, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const float d = v[k] - shift[k];
      s[k] += d;
      q[k] = fmaf(d, d, q[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s_sum[tid * 8 + k] = s[k];
    s_sq[tid * 8 + k] = q[k];
  }
  __syncthreads();
  if (rlane == 0) {
    for (int j = 1; j < R; ++j) {
      const int o = (j * Gb + cg_local) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        s[k] += s_sum[o + k];
        q[k] += s_sq[o + k];
      }
    }
    float* ps = psum + (int64_t)blockIdx.x * C + cg * 8;
    float* pq = psq + (int64_t)blockIdx.x * C + cg * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ps[k] = s[k];
      pq[k] = q[k];
    }
  }
}

// Level-2 reduction of the per-block partials: [2][nblk][C] -> [2][S][C], S = ceil(nblk / 64).
// Block = 64 channels x 4 row lanes (one wave reads 64 consecutive channels = 256 B per row), grid
// (ceil(C/64), S, 2): parallel over channels AND partial rows, so neither a large C (layer4) nor a
// large nblk (stem) leaves the reduction on a handful of CUs.
constexpr int kRowsPerSplit = 64;

// Per thread: the U = kRowsPerSplit / G rows lane, lane + G, ... of split s, all loads issued at once, summed in
// row order; the G group sums are then combined in group order.  bn_partial_reduce_kernel<NT> and the one-launch
// reduce_l2_last<NT> share this arithmetic, so both paths give bit-identical level-2 rows.
template <int NT>
__device__ __forceinline__ float l1_rows(const float* __restrict__ src, int b0, int b1, int C, int c, int lane) {
  constexpr int G = NT / 64, U = kRowsPerSplit / G;
  float x[U];
#pragma unroll
  for (int u = 0; u < U; ++u) {
    const int b = b0 + lane + u * G;
    x[u] = b < b1 ? src[(int64_t)b * C + c] : 0.f;
  }
  float a = 0.f;
#pragma unroll
  for (int u = 0; u < U; ++u) a += x[u];
  return a;
}

template <int NT>
__global__ __launch_bounds__(NT) void bn_partial_reduce_kernel(const float* __restrict__ part, int nblk, int C,
                                                               float* __restrict__ out, int S) {
  constexpr int G = NT / 64;
  __shared__ float sh[NT];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane = threadIdx.x >> 6;
  const int s = blockIdx.y, which = blockIdx.z;
  const int b0 = s * kRowsPerSplit;
  const int b1 = b0 + kRowsPerSplit < nblk ? b0 + kRowsPerSplit : nblk;
  sh[threadIdx.x] = c < C ? l1_rows<NT>(part + (int64_t)which * nblk * C, b0, b1, C, c, lane) : 0.f;
  __syncthreads();
  if (lane == 0 && c < C) {
    float r = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) r += sh[threadIdx.x + 64 * g];
    out[((int64_t)which * S + s) * C + c] = r;
  }
}

// Level-2 -> per-channel totals for the finalize kernels: block = 64 channels x 4 split lanes-groups, each group
// sums every 4th of the S partial rows (independent loads, fp64 accumulation), then the 4 group sums are combined
// through LDS in a fixed order (deterministic).  One thread per channel walking all S rows serially was 19 us per
// backward BatchNorm on the 56x56 layers (S ~ 100 dependent-latency iterations on a single 256-thread block).
// ATOMIC: the rows were published inside this launch by other workgroups (agent-scope atomic stores): read them with
// agent-scope atomic loads (coherent across the XCDs' L2s without an acquire fence / L2 invalidate)
template <int NT = 256, bool ATOMIC = false>
__device__ __forceinline__ bool fin_sum2(const float* __restrict__ pa, const float* __restrict__ pb, int nblk, int C,
                                         double& A, double& B) {
  constexpr int G = NT / 64;  // split lane-groups
  __shared__ double sh[2][G][64];
  const int lc = threadIdx.x & 63, sp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  double a0 = 0.0, b0 = 0.0;
  if (c < C) {
    // 8 rows (16 predicated loads) in flight per trip: this runs in the last-arriving block, on the critical path of
    // every BatchNorm; with 16 groups (1024 threads) S <= 128 level-2 rows is ONE dependent L2 round trip
    for (int b = sp; b < nblk; b += 8 * G) {
      float x[8], y[8];
#pragma unroll
      for (int u = 0; u < 8; ++u) {
        const int r = b + u * G;
        if (ATOMIC) {
          x[u] = r < nblk ? __hip_atomic_load(pa + (int64_t)r * C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
          y[u] = r < nblk ? __hip_atomic_load(pb + (int64_t)r * C + c, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) : 0.f;
        } else {
          x[u] = r < nblk ? pa[(int64_t)r * C + c] : 0.f;
          y[u] = r < nblk ? pb[(int64_t)r * C + c] : 0.f;
        }
      }
#pragma unroll
      for (int u = 0; u < 8; ++u) { a0 += x[u]; b0 += y[u]; }
    }
  }
  sh[0][sp][lc] = a0;
  sh[1][sp][lc] = b0;
  __syncthreads();
  if (sp != 0 || c >= C) return false;
  double sa = 0.0, sb = 0.0;
#pragma unroll
  for (int g = 0; g < G; ++g) { sa += sh[0][g][lc]; sb += sh[1][g][lc]; }  // fixed order: deterministic
  A = sa;
  B = sb;
  return true;
}

struct FwdFin {
  const uint16_t* x_row0;  // shift of the stats pass (nullptr: producer-fused, unshifted sums)
  int C;
  int64_t M;
  const float* gamma;
  const float* beta;
  float eps, momentum;
  float* running_mean;
  float* running_var;
  float* save_mean;
  float* save_invstd;
  float* scale;
  float* bias;
};

struct BwdFin {
  int C;
  int64_t M;
  const float* gamma;
  const float* mean;
  const float* invstd;
  float* dgamma;
  float* dbeta;
  float* coef;
  int accumulate;
};

template <int NT, bool ATOMIC = false>
__device__ __forceinline__ void fwd_finalize(const float* psum, const float* psq, int nblk, const FwdFin& f) {
  double S, Q;  // level-2 partials per channel, summed in fp64
  if (!fin_sum2<NT, ATOMIC>(psum, psq, nblk, f.C, S, Q)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const double m = S / (double)f.M;
  double var = Q / (double)f.M - m * m;
  if (var < 0.0) var = 0.0;
  const float mean = (f.x_row0 != nullptr ? bf2f(f.x_row0[c]) : 0.f) + (float)m;
  const float invstd = rsqrtf((float)var + f.eps);
  const float g = f.gamma[c];
  f.save_mean[c] = mean;
  f.save_invstd[c] = invstd;
  f.scale[c] = g * invstd;
  f.bias[c] = f.beta[c] - mean * g * invstd;
  if (f.running_mean != nullptr) {
    const float unbiased = f.M > 1 ? (float)(var * (double)f.M / (double)(f.M - 1)) : (float)var;
    f.running_mean[c] = (1.f - f.momentum) * f.running_mean[c] + f.momentum * mean;
    f.running_var[c] = (1.f - f.momentum) * f.running_var[c] + f.momentum * unbiased;
  }
}

template <int NT, bool ATOMIC = false>
__device__ __forceinline__ void bwd_finalize(const float* pdz, const float* pdzx, int nblk, const BwdFin& f) {
  double A, B;
  if (!fin_sum2<NT, ATOMIC>(pdz, pdzx, nblk, f.C, A, B)) return;
  const int C = f.C;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const float db = (float)A, dg = (float)B;
  // accumulate: dgamma / dbeta are the parameters' own (flat) gradient slots, summed into like autograd would
  f.dbeta[c] = f.accumulate ? f.dbeta[c] + db : db;
  f.dgamma[c] = f.accumulate ? f.dgamma[c] + dg : dg;
  const float is = f.invstd[c], k1 = f.gamma[c] * is;
  const float k2 = db / (float)f.M, k3 = dg / (float)f.M;
  // dx = k1 * (dz - k2 - xhat*k3),  xhat = (x - mean) * is   =>  dx = A*dz + B*x + D
  f.coef[c] = k1;                                    // A
  f.coef[C + c] = -k1 * k3 * is;                     // B
  f.coef[2 * C + c] = -k1 * k2 + k1 * k3 * is * f.mean[c];  // D
}

// Level-1 -> level-2 reduce and the finalize in ONE launch: grid (ceil(C/64), S), every block reduces its 64 partial
// rows of both sums for 64 channels (same order as bn_partial_reduce_kernel), publishes them, and takes a ticket on
// its channel group's counter; the block drawing S-1 runs the finalize over the S level-2 rows.  The hand-off is
// the split-K last-arriver recipe (cdna_hip_programming.md §5, in-launch split-K reduction): plain stores, every
// wave drained, agent-scope release by one lane before a relaxed agent-scope ticket add, agent-scope acquire by the
// last arriver before the workgroup reads.  Counters start at zero (allocated zeroed) and the last arriver resets
// its own; launches that share a counter array are stream-ordered.  Saves a launch boundary and the separate
// finalize pass's own ramp per BatchNorm direction (106 per ResNet-50 step).
template <int NT>
__device__ __forceinline__ bool reduce_l2_last(const float* __restrict__ part, int nblk, int C, float* l2, int S,
                                               unsigned* cnt) {
  constexpr int G = NT / 64;
  __shared__ float sh[2][NT];
  __shared__ int s_last;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const int b0 = s * kRowsPerSplit;
  int b1 = b0 + kRowsPerSplit;
  if (b1 > nblk) b1 = nblk;
  float a0 = 0.f, a1 = 0.f;
  if (c < C) {
    a0 = l1_rows<NT>(part, b0, b1, C, c, lane);
    a1 = l1_rows<NT>(part + (int64_t)nblk * C, b0, b1, C, c, lane);
  }
  sh[0][threadIdx.x] = a0;
  sh[1][threadIdx.x] = a1;
  __syncthreads();
  if (lane == 0 && c < C) {
    const int t = threadIdx.x;
    float r0 = 0.f, r1 = 0.f;
#pragma unroll
    for (int g = 0; g < G; ++g) { r0 += sh[0][t + 64 * g]; r1 += sh[1][t + 64 * g]; }
    // agent-scope atomic stores: coherent across the XCDs' L2s, so no release fence (an L2 write-back per
    // workgroup on gfx950) and, on the reading side, no acquire fence (an L2 invalidate): atomic loads instead
    __hip_atomic_store(l2 + (int64_t)s * C + c, r0, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    __hip_atomic_store(l2 + ((int64_t)S + s) * C + c, r1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    plx_handoff_release();  // no-op unless built with PLX_HANDOFF_FENCES (csrc/handoff.h: the hardware assumption)
    const unsigned old = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned)(S - 1);
    if (last) plx_handoff_acquire();
    if (last) __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

// 1024 threads: 16 row groups make both the level-1 rows (4 per thread) and the S level-2 rows (<= 8 per thread
// up to S = 128) a single L2 round trip each; with 256 threads they were 2 and up to 4 dependent trips
constexpr int kFinNT = 1024;
// (round 6 removed the 256-thread finalize variant: -0.5 %, profiles/r5_knob_recheck_ab.jsonl)
template <int NT>
__global__ __launch_bounds__(NT) void bn_fwd_reduce_finalize_kernel(const float* __restrict__ part, int nblk, float* l2,
                                                                    int S, unsigned* cnt, FwdFin f) {
  if (!reduce_l2_last<NT>(part, nblk, f.C, l2, S, cnt)) return;
  fwd_finalize<NT, true>(l2, l2 + (int64_t)S * f.C, S, f);
}

template <int NT>
__global__ __launch_bounds__(NT) void bn_bwd_reduce_finalize_kernel(const float* __restrict__ part, int nblk, float* l2,
                                                                    int S, unsigned* cnt, BwdFin f) {
  if (!reduce_l2_last<NT>(part, nblk, f.C, l2, S, cnt)) return;
  bwd_finalize<NT, true>(l2, l2 + (int64_t)S * f.C, S, f);
}

template <int NT>
__global__ __launch_bounds__(NT) void bn_fwd_finalize_kernel(const float* __restrict__ psum, const float* __restrict__ psq, int nblk,
                                       const uint16_t* __restrict__ x_row0, int C, int64_t M,
                                       const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                                       float momentum, float* __restrict__ running_mean,
                                       float* __restrict__ running_var, float* __restrict__ save_mean,
                                       float* __restrict__ save_invstd, float* __restrict__ scale,
                                       float* __restrict__ bias) {
  double S, Q;  // level-2 partials per channel, summed in fp64
  if (!fin_sum2<NT>(psum, psq, nblk, C, S, Q)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const double m = S / (double)M;
  double var = Q / (double)M - m * m;
  if (var < 0.0) var = 0.0;
  const float mean = (x_row0 != nullptr ? bf2f(x_row0[c]) : 0.f) + (float)m;  // no shift: producer-fused stats
  const float invstd = rsqrtf((float)var + eps);
  const float g = gamma[c];
  save_mean[c] = mean;
  save_invstd[c] = invstd;
  scale[c] = g * invstd;
  bias[c] = beta[c] - mean * g * invstd;
  if (running_mean != nullptr) {
    const float unbiased = M > 1 ? (float)(var * (double)M / (double)(M - 1)) : (float)var;
    running_mean[c] = (1.f - momentum) * running_mean[c] + momentum * mean;
    running_var[c] = (1.f - momentum) * running_var[c] + momentum * unbiased;
  }
}

// ------------------------------------------------------------------------------- forward apply
// RES / RELU are compile-time: with a runtime residual test hipcc waited for x's load before issuing the residual's
// (one extra HBM round trip per trip), and a per-element `rsb ? rsb[c] : 1` in the prologue became eight
// load-then-wait branches (cdna_hip_programming.md §5 item 4(c)) -- ~20 us of latency per block that dominated the
// 14x14 / 7x7 layers (35 us for a 53 MB apply, profiles/r2_resnet50_roofline.md).
template <bool RES, bool RELU>
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const bf16x8* __restrict__ x, const bf16x8* __restrict__ res,
                                                          bf16x8* __restrict__ y, const float* __restrict__ scale,
                                                          const float* __restrict__ bias, int64_t n_vec, int G,
                                                          uint8_t* __restrict__ mask, const float* __restrict__ rsb) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;  // multiple of G (G | 256 or G % 256 == 0 handled by host)
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_vec) return;
  const int cg = (int)(i % G);
  float a[8], b[8], ra[8], rb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = scale[cg * 8 + k];
    b[k] = bias[cg * 8 + k];
    ra[k] = 1.f;
    rb[k] = 0.f;
  }
  // rsb: the residual is the raw input of a BatchNorm (no activation) whose apply pass is deferred to here:
  // res' = res * rsb[c] + rsb[C + c]  (a ResNet downsampling branch feeds only this add)
  if (RES && rsb != nullptr) {
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      ra[k] = rsb[cg * 8 + k];
      rb[k] = rsb[G * 8 + cg * 8 + k];
    }
  }
  for (; i < n_vec; i += stride) {
    const bf16x8 xv = x[i];
    bf16x8 rv;
    if constexpr (RES) rv = res[i];
    float v[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaf(bf2f(xv.v[k]), a[k], b[k]);
    if constexpr (RES) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += fmaf(bf2f(rv.v[k]), ra[k], rb[k]);
    }
    if constexpr (RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
    }
    store8(y + i, v);
    if (RELU && mask != nullptr) {
      // ReLU mask, 1 bit per element (bit k of byte i = channel 8*cg+k of vector i): the backward reads this
      // 1/16-size tensor instead of y (a positive float stays positive after bf16 rounding, so bit == y > 0).
      uint32_t bits = 0;
#pragma unroll
      for (int k = 0; k < 8; ++k) bits |= (uint32_t)(v[k] > 0.f) << k;
      mask[i] = (uint8_t)bits;
    }
  }
}

// ------------------------------------------------------------------------------- backward reduce
template <bool RELU>  // compile-time, so the mask load issues with the x / dy loads (see bn_apply_kernel)
__global__ __launch_bounds__(kBlock) void bn_bwd_reduce_kernel(const bf16x8* __restrict__ x, const uint8_t* __restrict__ mask,
                                                               const bf16x8* __restrict__ dy, int64_t M, int G, int Gb,
                                                               int64_t rows_per_block, const float* __restrict__ mean,
                                                               const float* __restrict__ invstd, int relu,
                                                               float* __restrict__ pdz, float* __restrict__ pdzx) {
  __shared__ float s_a[kBlock * 8];
  __shared__ float s_b[kBlock * 8];
  const int tid = threadIdx.x;
  const int cg_local = tid % Gb, rlane = tid / Gb, R = kBlock / Gb;
  const int cg = blockIdx.y * Gb + cg_local;
  const int C = G * 8;
  float mu[8], is[8], sa[8], sb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    mu[k] = mean[cg * 8 + k];
    is[k] = invstd[cg * 8 + k];
    sa[k] = sb[k] = 0.f;
  }
  const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
  int64_t r1 = r0 + rows_per_block;
  if (r1 > M) r1 = M;
#pragma unroll 4
  for (int64_t r = r0 + rlane; r < r1; r += R) {
    const int64_t off = r * G + cg;
    float xv[8], g[8];
    uint32_t mb = 0xffu;
    if constexpr (RELU) mb = mask[off];
    load8(x + off, xv);
    load8(dy + off, g);
    if constexpr (RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = (mb >> k) & 1u ? g[k] : 0.f;
    }
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      sa[k] += g[k];
      sb[k] = fmaf(g[k], (xv[k] - mu[k]) * is[k], sb[k]);
    }
  }
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    s_a[tid * 8 + k] = sa[k];
    s_b[tid * 8 + k] = sb[k];
  }
  __syncthreads();
  if (rlane == 0) {
    for (int j = 1; j < R; ++j) {
      const int o = (j * Gb + cg_local) * 8;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        sa[k] += s_a[o + k];
        sb[k] += s_b[o + k];
      }
    }
    float* pa = pdz + (int64_t)blockIdx.x * C + cg * 8;
    float* pb = pdzx + (int64_t)blockIdx.x * C + cg * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pa[k] = sa[k];
      pb[k] = sb[k];
    }
  }
}

template <int NT>
__global__ __launch_bounds__(NT) void bn_bwd_finalize_kernel(const float* __restrict__ pdz, const float* __restrict__ pdzx, int nblk, int C,
                                       int64_t M, const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float* __restrict__ coef, int accumulate) {
  double A, B;
  if (!fin_sum2<NT>(pdz, pdzx, nblk, C, A, B)) return;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const float db = (float)A, dg = (float)B;
  // accumulate: dgamma / dbeta are the parameters' own (flat) gradient slots, summed into like autograd would
  dbeta[c] = accumulate ? dbeta[c] + db : db;
  dgamma[c] = accumulate ? dgamma[c] + dg : dg;
  const float is = invstd[c], k1 = gamma[c] * is;
  const float k2 = db / (float)M, k3 = dg / (float)M;
  // dx = k1 * (dz - k2 - xhat*k3),  xhat = (x - mean) * is   =>  dx = A*dz + B*x + D
  coef[c] = k1;                                  // A
  coef[C + c] = -k1 * k3 * is;                   // B
  coef[2 * C + c] = -k1 * k2 + k1 * k3 * is * mean[c];  // D
}

// The BatchNorm that produced this one's residual input (a ResNet downsampling branch), when d_residual is that
// BatchNorm's complete gradient: the dx pass also reduces its per-block partials  sum dz2  and
// sum dz2 * (x2 - mean2) * invstd2  (dz2 = d_residual, masked by its own ReLU if it had one) into
// part[2][gridDim.x][C], so that BatchNorm's backward skips its reduce pass (plx_bn_backward_from_partials).
struct ResBn {
  const bf16x8* x;
  const uint8_t* mask;   // nullptr: no ReLU
  const float* mean;
  const float* invstd;
  float* part;           // nullptr: disabled
};

// RP: also reduce the residual BatchNorm's partials (ResBn).  A separate instantiation: its extra state
// (90 VGPRs) would cut the plain pass from 8 to 5 waves per SIMD, and this memory-bound pass needs them.
// RMASK (RP only): the residual BatchNorm had a ReLU (rb.mask set) -- compile-time, no per-trip pointer test
template <bool RP, bool RELU, bool RMASK = false>
__global__ __launch_bounds__(kBlock) void bn_bwd_dx_kernel(const bf16x8* __restrict__ x, const uint8_t* __restrict__ mask,
                                                           const bf16x8* __restrict__ dy, bf16x8* __restrict__ dx,
                                                           bf16x8* __restrict__ dres, const float* __restrict__ coef,
                                                           int64_t n_vec, int G, int relu, ResBn rb) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (!RP && i >= n_vec) return;
  const int cg = (int)(i % G);  // fixed over the grid stride (grid * 256 % G == 0)
  const int C = G * 8;
  constexpr bool rp = RP;
  float A[8], B[8], D[8], mu2[8], is2[8], ra[8], rc[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    A[k] = coef[cg * 8 + k];
    B[k] = coef[C + cg * 8 + k];
    D[k] = coef[2 * C + cg * 8 + k];
    ra[k] = rc[k] = 0.f;
    mu2[k] = rp ? rb.mean[cg * 8 + k] : 0.f;
    is2[k] = rp ? rb.invstd[cg * 8 + k] : 0.f;
  }
  for (; i < n_vec; i += stride) {
    float xv[8], g[8];
    uint32_t mb = 0xffu;
    if constexpr (RELU) mb = mask[i];  // issued with the x / dy loads (RELU is compile-time)
    load8(x + i, xv);
    load8(dy + i, g);
    if constexpr (RELU) {
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = (mb >> k) & 1u ? g[k] : 0.f;
    }
    if (dres != nullptr) store8(dres + i, g);
    if constexpr (rp) {
      float x2[8];
      load8(rb.x + i, x2);
      const uint32_t m2 = RMASK ? rb.mask[i] : 0xffu;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float g2 = (m2 >> k) & 1u ? g[k] : 0.f;
        ra[k] += g2;
        rc[k] = fmaf(g2, (x2[k] - mu2[k]) * is2[k], rc[k]);
      }
    }
    float o[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) o[k] = fmaf(A[k], g[k], fmaf(B[k], xv[k], D[k]));
    store8(dx + i, o);
  }
  if constexpr (rp) {
  // threads tid, tid + G, ... of this block share channel group cg: sum them through LDS (G <= 256)
  __shared__ float red[kBlock * 16];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    red[threadIdx.x * 16 + k] = ra[k];
    red[threadIdx.x * 16 + 8 + k] = rc[k];
  }
  __syncthreads();
  if ((int)threadIdx.x < G) {
    for (int j = 1; j < kBlock / G; ++j) {
      const float* o = red + (j * G + threadIdx.x) * 16;
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        ra[k] += o[k];
        rc[k] += o[8 + k];
      }
    }
    float* pa = rb.part + (int64_t)blockIdx.x * C + cg * 8;
    float* pc = rb.part + ((int64_t)gridDim.x + blockIdx.x) * C + cg * 8;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      pa[k] = ra[k];
      pc[k] = rc[k];
    }
  }
  }
}

struct Plan {
  int G, Gb, gy, nblk, S;
  int64_t rows_per_block;
};

inline bool plan_for(int64_t M, int C, Plan* p) {
  if (C <= 0 || (C & 7)) return false;
  const int G = C / 8;
  if (G & (G - 1)) return false;  // power of two channel groups
  p->G = G;
  p->Gb = G < kBlock ? G : kBlock;
  p->gy = G / p->Gb;
  const int R = kBlock / p->Gb;
  const int64_t cap = (2048 + p->gy - 1) / p->gy;
  int64_t want = (M + 16 * R - 1) / (16 * R);  // every thread streams >= 16 rows
  if (want > cap) want = cap;
  if (want < 1) want = 1;
  int64_t rpb = (M + want - 1) / want;
  rpb = (rpb + R - 1) / R * R;
  p->rows_per_block = rpb;
  p->nblk = (int)((M + rpb - 1) / rpb);
  p->S = (p->nblk + kRowsPerSplit - 1) / kRowsPerSplit;
  return true;
}

// grid-stride must keep each thread on one channel group: grid*256 % G == 0
inline int apply_grid(int64_t n_vec, int G) {
  int64_t g = (n_vec + kBlock - 1) / kBlock;
  if (g > 4096) g = 4096;
  if (g < 1) g = 1;
  const int64_t mult = G > kBlock ? G / kBlock : 1;
  g = (g + mult - 1) / mult * mult;
  return (int)g;
}

inline void launch_dx(hipStream_t stream, int64_t n_vec, int G, const void* x, const uint8_t* mask, const void* dy,
                      void* dx, void* dres, const float* coef, int relu, const ResBn& rb) {
  const dim3 grid(apply_grid(n_vec, G));
  auto k = rb.part == nullptr ? (relu ? bn_bwd_dx_kernel<false, true> : bn_bwd_dx_kernel<false, false>)
           : rb.mask != nullptr ? (relu ? bn_bwd_dx_kernel<true, true, true> : bn_bwd_dx_kernel<true, false, true>)
                                : (relu ? bn_bwd_dx_kernel<true, true> : bn_bwd_dx_kernel<true, false>);
  hipLaunchKernelGGL(k, grid, dim3(kBlock), 0, stream, (const bf16x8*)x, mask, (const bf16x8*)dy, (bf16x8*)dx,
                     (bf16x8*)dres, coef, n_vec, G, relu, rb);
}

inline void launch_apply(hipStream_t stream, int64_t n_vec, int G, const void* x, const void* res, void* y,
                         const float* scale, const float* bias, int relu, uint8_t* mask, const float* rsb) {
  auto k = res != nullptr ? (relu ? bn_apply_kernel<true, true> : bn_apply_kernel<true, false>)
                          : (relu ? bn_apply_kernel<false, true> : bn_apply_kernel<false, false>);
  hipLaunchKernelGGL(k, dim3(apply_grid(n_vec, G)), dim3(kBlock), 0, stream, (const bf16x8*)x, (const bf16x8*)res,
                     (bf16x8*)y, scale, bias, n_vec, G, mask, rsb);
}

// level-1 partials [2][nblk][C] -> finalize: one fused launch with a counter array (>= ceil(C/64) zeroed words),
// else the reduce and finalize kernels back to back
inline void reduce_finalize_fwd(hipStream_t stream, const float* part, int nblk, float* l2, unsigned* cnt,
                                const FwdFin& f) {
  const int C = f.C, S = (nblk + kRowsPerSplit - 1) / kRowsPerSplit;
  if (cnt != nullptr) {
    hipLaunchKernelGGL(bn_fwd_reduce_finalize_kernel<kFinNT>, dim3((C + 63) / 64, S), dim3(kFinNT), 0, stream, part, nblk, l2, S,
                       cnt, f);
    return;
  }
  hipLaunchKernelGGL(bn_partial_reduce_kernel<kFinNT>,
                     dim3((C + 63) / 64, S, 2), dim3(kFinNT), 0, stream, part, nblk, C, l2, S);
  hipLaunchKernelGGL(bn_fwd_finalize_kernel<kFinNT>, dim3((C + 63) / 64),
                     dim3(kFinNT), 0, stream, l2, l2 + (int64_t)S * C, S,
                     f.x_row0, C, f.M, f.gamma, f.beta, f.eps, f.momentum, f.running_mean, f.running_var, f.save_mean,
                     f.save_invstd, f.scale, f.bias);
}

inline void reduce_finalize_bwd(hipStream_t stream, const float* part, int nblk, float* l2, unsigned* cnt,
                                const BwdFin& f) {
  const int C = f.C, S = (nblk + kRowsPerSplit - 1) / kRowsPerSplit;
  if (cnt != nullptr) {
    hipLaunchKernelGGL(bn_bwd_reduce_finalize_kernel<kFinNT>, dim3((C + 63) / 64, S), dim3(kFinNT), 0, stream, part, nblk, l2, S,
                       cnt, f);
    return;
  }
  hipLaunchKernelGGL(bn_partial_reduce_kernel<kFinNT>,
                     dim3((C + 63) / 64, S, 2), dim3(kFinNT), 0, stream, part, nblk, C, l2, S);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel<kFinNT>, dim3((C + 63) / 64),
                     dim3(kFinNT), 0, stream, l2, l2 + (int64_t)S * C, S, C,
                     f.M, f.gamma, f.mean, f.invstd, f.dgamma, f.dbeta, f.coef, f.accumulate);
}

// ------------------------------------------------------------------------------- ResNet stem: BN + ReLU + max-pool
// The stem's BatchNorm(+ReLU) output only feeds the 3x3/s2/p1 max-pool.  Forward: p = maxpool(bf16(relu(x*scale +
// bias))) in one pass over x with the window position (0..8) of each max (first max in (kh, kw) order, the rule of
// csrc/pool_kernels.hip), so the BatchNorm output (4x the pooled size) and its ReLU mask are never written or re-read.
// Backward: every input pixel gathers dy from the <= 2x2 windows whose argmax it is (maxpool_bwd_kernel's gather, the
// sum rounded to bf16 as that kernel stores it), masks it by the recomputed ReLU test (x*scale + bias > 0, the apply
// pass's test bit for bit) and either reduces the BatchNorm partials (pass 1) or writes dx = A*dz + B*x + D (pass 2):
// 2 passes over x instead of pool-bwd write + BN reduce + BN dx (3 reads and 2 writes of the 112x112 tensor).
struct alignas(8) u8x8 {
  uint8_t v[8];
};

__global__ __launch_bounds__(256) void stem_apply_pool_kernel(const bf16x8* __restrict__ x,
                                                              const float* __restrict__ sb, bf16x8* __restrict__ y,
                                                              u8x8* __restrict__ idx, int N, int H, int W, int G,
                                                              int OH, int OW) {
  const unsigned j = blockIdx.x * 256u + threadIdx.x;
  if (j >= (unsigned)(OW * G)) return;
  const unsigned g = j % (unsigned)G, ow = j / (unsigned)G;
  const int C = G * 8;
  float a[8], b[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = sb[g * 8 + k];
    b[k] = sb[C + g * 8 + k];
  }
  for (int row = blockIdx.y; row < N * OH; row += gridDim.y) {
    const int n = row / OH, oh = row - n * OH;
    float best[8];
    uint8_t arg[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      best[k] = -INFINITY;
      arg[k] = 255;
    }
    // all 9 window loads first, from clamped (always valid) addresses; out-of-image taps are skipped in the max
    // (a branch around each load made hipcc wait for every load before issuing the next)
    uint4 q[9];
    bool ok[9];
#pragma unroll
    for (int kh = 0; kh < 3; ++kh) {
      const int ih = oh * 2 - 1 + kh;
      const int ihc = ih < 0 ? 0 : (ih >= H ? H - 1 : ih);
#pragma unroll
      for (int kw = 0; kw < 3; ++kw) {
        const int iw = (int)ow * 2 - 1 + kw;
        const int iwc = iw < 0 ? 0 : (iw >= W ? W - 1 : iw);
        ok[kh * 3 + kw] = ih >= 0 && ih < H && iw >= 0 && iw < W;
        q[kh * 3 + kw] = *(const uint4*)(x + ((size_t)(n * H + ihc) * W + iwc) * G + g);
      }
    }
#pragma unroll
    for (int t9 = 0; t9 < 9; ++t9) {
      const uint32_t qw[4] = {q[t9].x, q[t9].y, q[t9].z, q[t9].w};
#pragma unroll
      for (int k = 0; k < 8; ++k) {
        const float xk = __uint_as_float((k & 1) ? (qw[k >> 1] & 0xffff0000u) : (qw[k >> 1] << 16));
        const float f = (float)(__bf16)fmaxf(fmaf(xk, a[k], b[k]), 0.f);  // the apply pass's bf16 value (RNE)
        if (ok[t9] && (f > best[k] || arg[k] == 255)) {
          best[k] = f;
          arg[k] = (uint8_t)t9;
        }
      }
    }
    bf16x8 o;
    u8x8 m;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      o.v[k] = f2bf(best[k]);
      m.v[k] = arg[k];
    }
    const size_t t = (size_t)row * OW * G + j;
    y[t] = o;
    idx[t] = m;
  }
}

// input row / column i of a 3x3/s2/p1 pool is covered by output o = (i + 1 - k) / 2 for the taps k of matching parity
__device__ __forceinline__ int stem_cover(int i, int O, int* o, int* k) {
  int n = 0;
  if (i & 1) {
    if ((i + 1) >> 1 < O) { o[n] = (i + 1) >> 1; k[n++] = 0; }
    o[n] = (i - 1) >> 1; k[n++] = 2;
  } else if ((i >> 1) < O) {
    o[n] = i >> 1; k[n++] = 1;
  }
  return n;
}

// One thread = 8 channels of a 2x2 quad of input pixels (2a + di, 2b + dj): row 2a is covered only by output row a
// (tap kh = 1), row 2a + 1 by rows a (kh = 2) and a + 1 (kh = 0), likewise for columns, so the quad's gradient comes
// from the 4 windows (a + p, b + q) -- one window load per input pixel instead of every pixel gathering all 4 windows
// (a first per-pixel version ran 1.6x the unfused pool-bwd + BN-bwd time).  Grid (ceil(QW*G / 256), rows_y) over quad
// rows (n, a); block (bx, by) walks quad rows by, by + rows_y, ...  DX = false: per-block partials
// part[2][gridDim.x * gridDim.y][C] of sum dz and sum dz * xhat; DX = true: dx from coef = [A | B | D].
template <bool DX>
__global__ __launch_bounds__(256) void stem_pool_bn_bwd_kernel(const bf16x8* __restrict__ dy, const u8x8* __restrict__ idx,
                                                               const bf16x8* __restrict__ x, const float* __restrict__ sb,
                                                               const float* __restrict__ mean,
                                                               const float* __restrict__ invstd,
                                                               const float* __restrict__ coef, bf16x8* __restrict__ dx,
                                                               float* __restrict__ part, int N, int H, int W, int G,
                                                               int OH, int OW) {
  const int QH = (H + 1) / 2, QW = (W + 1) / 2;
  const unsigned j0 = blockIdx.x * 256u + threadIdx.x;
  const bool active = j0 < (unsigned)(QW * G);
  const unsigned j = active ? j0 : 0u;
  const unsigned g = j % (unsigned)G;                     // == threadIdx.x % G (256 % G == 0)
  const int qb = (int)(j / (unsigned)G);
  const int C = G * 8;
  float a[8], b[8], c1[8], c2[8], c3[8], s1[8], s2[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = sb[g * 8 + k];
    b[k] = sb[C + g * 8 + k];
    if constexpr (DX) {
      c1[k] = coef[g * 8 + k];
      c2[k] = coef[C + g * 8 + k];
      c3[k] = coef[2 * C + g * 8 + k];
    } else {
      c1[k] = mean[g * 8 + k];
      c2[k] = invstd[g * 8 + k];
      c3[k] = 0.f;
    }
    s1[k] = s2[k] = 0.f;
  }
  for (int row = blockIdx.y; active && row < N * QH; row += gridDim.y) {
    const int n = row / QH, qa = row - n * QH;
    // windows (qa + p, qb + q) and the quad's pixels: whole-vector loads from clamped addresses, all issued before
    // any use; validity is applied per element
    uint2 am[4];
    uint4 d[4], xq[4];
    bool wv[4], pv[4];
#pragma unroll
    for (int p = 0; p < 2; ++p)
#pragma unroll
      for (int q = 0; q < 2; ++q) {
        const int w4 = p * 2 + q, oh = qa + p, ow = qb + q;
        wv[w4] = oh < OH && ow < OW;
        const size_t off = ((size_t)(n * OH + (oh < OH ? oh : OH - 1)) * OW + (ow < OW ? ow : OW - 1)) * G + g;
        am[w4] = *(const uint2*)(idx + off);
        d[w4] = *(const uint4*)(dy + off);
        if (!wv[w4]) am[w4] = make_uint2(0xffffffffu, 0xffffffffu);  // no tap code (0..8) matches 0xff
        const int ih = 2 * qa + p, iw = 2 * qb + q;         // quad pixel (di, dj) = (p, q)
        pv[w4] = ih < H && iw < W;
        xq[w4] = *(const uint4*)(x + ((size_t)(n * H + (ih < H ? ih : H - 1)) * W + (iw < W ? iw : W - 1)) * G + g);
      }
#pragma unroll
    for (int di = 0; di < 2; ++di)
#pragma unroll
      for (int dj = 0; dj < 2; ++dj) {
        const int e = di * 2 + dj;
        const uint32_t xw[4] = {xq[e].x, xq[e].y, xq[e].z, xq[e].w};
        float o[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) {
          float acc = 0.f;
#pragma unroll
          for (int p = 0; p < 2; ++p)
#pragma unroll
            for (int q = 0; q < 2; ++q) {
              const int kh = di + 1 - 2 * p, kw = dj + 1 - 2 * q;   // this pixel's tap in window (p, q)
              if (kh < 0 || kw < 0) continue;                      // compile-time
              const int w4 = p * 2 + q;
              const uint32_t ab = (k < 4 ? am[w4].x : am[w4].y) >> (8 * (k & 3)) & 0xffu;
              const uint32_t dw = (k >> 1) == 0 ? d[w4].x : (k >> 1) == 1 ? d[w4].y : (k >> 1) == 2 ? d[w4].z : d[w4].w;
              const float dv = __uint_as_float((k & 1) ? (dw & 0xffff0000u) : (dw << 16));
              acc += ab == (uint32_t)(kh * 3 + kw) ? dv : 0.f;   // invalid windows' bytes were set to 0xff
            }
          const float xf = __uint_as_float((k & 1) ? (xw[k >> 1] & 0xffff0000u) : (xw[k >> 1] << 16));
          // rounded to bf16 as the unfused pool backward stores it (a plain cast: one v_cvt_pk_bf16_f32, RNE)
          const float dz = (pv[e] && fmaf(xf, a[k], b[k]) > 0.f) ? (float)(__bf16)acc : 0.f;
          if constexpr (DX) {
            o[k] = fmaf(c1[k], dz, fmaf(c2[k], xf, c3[k]));
          } else {
            s1[k] += dz;
            s2[k] = fmaf(dz, (xf - c1[k]) * c2[k], s2[k]);
          }
        }
        if constexpr (DX) {
          if (pv[e]) store8(dx + ((size_t)(n * H + 2 * qa + di) * W + 2 * qb + dj) * G + g, o);
        }
      }
  }
  if constexpr (!DX) {
    // the 256 / G threads of this block that share channel group g: fixed-order sum through LDS
    __shared__ float red[256 * 17];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      red[threadIdx.x * 17 + k] = s1[k];
      red[threadIdx.x * 17 + 8 + k] = s2[k];
    }
    __syncthreads();
    const int nb = gridDim.x * gridDim.y, blk = blockIdx.y * gridDim.x + blockIdx.x;
    for (int e = threadIdx.x; e < G * 16; e += 256) {     // e = (value v, group gg)
      const int gg = e % G, v = e / G;
      float sum = 0.f;
      for (int r = gg; r < 256; r += G) sum += red[r * 17 + v];
      const int c = gg * 8 + (v & 7);
      part[((int64_t)(v < 8 ? 0 : nb) + blk) * C + c] = sum;
    }
  }
}

// over quad rows: pass 1 (partials) a few per block (rows_y <= g_stem_bwd_cap bounds the level-1 partials: 4096 rows
// ~4 MB at the stem's shape), pass 2 (dx) one per block.
constexpr int g_stem_bwd_cap = 4096;

inline dim3 stem_bwd_grid(int N, int H, int W, int G, bool dx) {
  const int rows = N * ((H + 1) / 2), cap = dx ? 65535 : g_stem_bwd_cap;
  return dim3((((W + 1) / 2) * G + 255) / 256, rows < cap ? rows : cap);
}

}  // namespace

// fp32 workspace the host must pass as `partials`: level-1 [2][nblk][C] + level-2 [2][S][C].
PLX_API int64_t plx_bn_workspace(int64_t M, int C) {
  Plan p;
  if (!plan_for(M, C, &p)) return -1;
  return 2 * (int64_t)(p.nblk + p.S) * C;
}

PLX_API int plx_bn_forward(const void* x, const void* res, void* y, int64_t M, int C, const float* gamma,
                           const float* beta, float eps, float momentum, float* running_mean, float* running_var,
                           float* save_mean, float* save_invstd, float* scale_bias /* [2C] */,
                           float* partials /* plx_bn_workspace floats */, uint8_t* mask /* M*C/8 bytes or null */,
                           int relu, const float* res_sb /* nullable [2C], see bn_apply_kernel */,
                           unsigned* counters /* nullable: >= ceil(C/64) zeroed words, one launch for
                                                 reduce + finalize */,
                           hipStream_t stream) {
  Plan p;
  if (!plan_for(M, C, &p) || M < 1) return 1;
  float* psum = partials;
  float* psq = partials + (int64_t)p.nblk * C;
  hipLaunchKernelGGL(bn_stats_kernel, dim3(p.nblk, p.gy), dim3(kBlock), 0, stream, (const bf16x8*)x, M, p.G, p.Gb,
                     p.rows_per_block, psum, psq);
  float* l2 = partials + 2 * (int64_t)p.nblk * C;
  reduce_finalize_fwd(stream, partials, p.nblk, l2, counters,
                      FwdFin{(const uint16_t*)x, C, M, gamma, beta, eps, momentum, running_mean, running_var,
                             save_mean, save_invstd, scale_bias, scale_bias + C});
  const int64_t n_vec = M * p.G;
  if (y != nullptr)  // y == nullptr: statistics and scale/bias only (the apply is deferred to the consumer)
    launch_apply(stream, n_vec, p.G, x, res, y, scale_bias, scale_bias + C, relu, relu ? mask : nullptr, res_sb);
  return (int)hipGetLastError();
}

// Level-2 workspace for externally produced level-1 partials ([2][nblk][C], e.g. from the 1x1-conv GEMM
// epilogue, csrc/conv_gemm.hip): 2 * ceil(nblk / 64) * C floats.
PLX_API int64_t plx_bn_l2_workspace(int nblk, int C) {
  return 2 * (int64_t)((nblk + kRowsPerSplit - 1) / kRowsPerSplit) * C;
}

// Forward with the per-channel sums already produced by the op that wrote x (unshifted sums over nblk row
// blocks): skips the stats pass over x.  l2 holds plx_bn_l2_workspace(nblk, C) floats.
PLX_API int plx_bn_forward_from_partials(const void* x, const void* res, void* y, int64_t M, int C,
                                         const float* gamma, const float* beta, float eps, float momentum,
                                         float* running_mean, float* running_var, float* save_mean,
                                         float* save_invstd, float* scale_bias, const float* partials, int nblk,
                                         float* l2, uint8_t* mask, int relu, const float* res_sb,
                                         unsigned* counters, hipStream_t stream) {
  Plan p;
  if (!plan_for(M, C, &p) || M < 1 || nblk < 1) return 1;
  reduce_finalize_fwd(stream, partials, nblk, l2, counters,
                      FwdFin{nullptr, C, M, gamma, beta, eps, momentum, running_mean, running_var, save_mean,
                             save_invstd, scale_bias, scale_bias + C});
  const int64_t n_vec = M * p.G;
  if (y != nullptr)
    launch_apply(stream, n_vec, p.G, x, res, y, scale_bias, scale_bias + C, relu, relu ? mask : nullptr, res_sb);
  return (int)hipGetLastError();
}

PLX_API int plx_bn_apply(const void* x, const void* res, void* y, int64_t M, int C, const float* scale_bias, int relu,
                         hipStream_t stream) {
  Plan p;
  if (!plan_for(M, C, &p)) return 1;
  const int64_t n_vec = M * p.G;
  launch_apply(stream, n_vec, p.G, x, res, y, scale_bias, scale_bias + C, relu, nullptr, nullptr);
  return (int)hipGetLastError();
}

// mask: the ReLU bit mask written by the forward (required when relu); accumulate: dgamma/dbeta += (else =)
// Row blocks of the dx pass = the nblk of the residual-BatchNorm partials it writes (ResBn, plx_bn_backward*).
PLX_API int plx_bn_dx_blocks(int64_t M, int C) {
  Plan p;
  if (!plan_for(M, C, &p)) return -1;
  return apply_grid(M * p.G, p.G);
}

PLX_API int plx_bn_backward(const void* x, const uint8_t* mask, const void* dy, void* dx, void* dres, int64_t M, int C,
                            const float* gamma, const float* save_mean, const float* save_invstd, float* dgamma,
                            float* dbeta, float* coef /* [3C] */, float* partials /* plx_bn_workspace floats */, int relu,
                            int accumulate, const ResBn* resbn /* nullable, needs dres */, unsigned* counters,
                            hipStream_t stream) {
  Plan p;
  if (!plan_for(M, C, &p) || M < 1 || (relu && mask == nullptr)) return 1;
  if (resbn != nullptr && (dres == nullptr || resbn->part == nullptr)) return 1;
  const ResBn rb = resbn != nullptr ? *resbn : ResBn{};
  float* pa = partials;
  float* pb = partials + (int64_t)p.nblk * C;
  hipLaunchKernelGGL(relu ? bn_bwd_reduce_kernel<true> : bn_bwd_reduce_kernel<false>, dim3(p.nblk, p.gy), dim3(kBlock), 0, stream, (const bf16x8*)x,
                     mask, (const bf16x8*)dy, M, p.G, p.Gb, p.rows_per_block, save_mean, save_invstd,
                     relu, pa, pb);
  float* l2 = partials + 2 * (int64_t)p.nblk * C;
  reduce_finalize_bwd(stream, partials, p.nblk, l2, counters,
                      BwdFin{C, M, gamma, save_mean, save_invstd, dgamma, dbeta, coef, accumulate});
  const int64_t n_vec = M * p.G;
  launch_dx(stream, n_vec, p.G, x, mask, dy, dx, dres, coef, relu, rb);
  return (int)hipGetLastError();
}

// Backward whose per-block partials ([2][nblk][C]: sum dz, sum dz*xhat) were produced by the op that wrote dy
// (the data-gradient GEMM epilogue, csrc/conv_gemm.hip BnBwd): skips the reduce pass over x and dy.  l2 holds
// plx_bn_l2_workspace(nblk, C) floats.
PLX_API int plx_bn_backward_from_partials(const void* x, const uint8_t* mask, const void* dy, void* dx, void* dres,
                                          int64_t M, int C, const float* gamma, const float* save_mean,
                                          const float* save_invstd, float* dgamma, float* dbeta, float* coef,
                                          const float* partials, int nblk, float* l2, int relu, int accumulate,
                                          const ResBn* resbn, unsigned* counters, hipStream_t stream) {
  Plan p;
  if (!plan_for(M, C, &p) || M < 1 || nblk < 1 || (relu && mask == nullptr)) return 1;
  if (resbn != nullptr && (dres == nullptr || resbn->part == nullptr)) return 1;
  const ResBn rb = resbn != nullptr ? *resbn : ResBn{};
  reduce_finalize_bwd(stream, partials, nblk, l2, counters,
                      BwdFin{C, M, gamma, save_mean, save_invstd, dgamma, dbeta, coef, accumulate});
  const int64_t n_vec = M * p.G;
  launch_dx(stream, n_vec, p.G, x, mask, dy, dx, dres, coef, relu, rb);
  return (int)hipGetLastError();
}

// ---- ResNet stem BatchNorm + ReLU + 3x3/s2/p1 max-pool (see stem_apply_pool_kernel)
// Forward: statistics (workspace `partials`: plx_bn_workspace(N*H*W, C) floats) -> mean / invstd / scale|bias ->
// y [N][OH][OW][C] bf16 and idx [N*OH*OW*C] window positions.
// ext_part / ext_nblk (nullable / 0): level-1 channel-stat partials [2][ext_nblk][C] from the producing convolution's
// epilogue (plx_stem_conv_fwd); `partials` then only needs the level-2 rows (plx_bn_l2_workspace(ext_nblk, C))
PLX_API int plx_stem_bn_pool_forward(const void* x, void* y, void* idx, int N, int H, int W, int C, const float* gamma,
                                     const float* beta, float eps, float momentum, float* running_mean,
                                     float* running_var, float* save_mean, float* save_invstd, float* scale_bias,
                                     float* partials, const float* ext_part, int ext_nblk, unsigned* counters,
                                     hipStream_t stream) {
  const int G = C / 8;
  if (N <= 0 || H <= 0 || W <= 0 || C % 8 || G > 256 || 256 % G) return 1;
  const int rc = ext_part != nullptr
                     ? plx_bn_forward_from_partials(x, nullptr, nullptr, (int64_t)N * H * W, C, gamma, beta, eps,
                                                    momentum, running_mean, running_var, save_mean, save_invstd,
                                                    scale_bias, ext_part, ext_nblk, partials, nullptr, 1, nullptr,
                                                    counters, stream)
                     : plx_bn_forward(x, nullptr, nullptr, (int64_t)N * H * W, C, gamma, beta, eps, momentum,
                                      running_mean, running_var, save_mean, save_invstd, scale_bias, partials, nullptr,
                                      1, nullptr, counters, stream);
  if (rc) return rc;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const int rows = N * OH;
  hipLaunchKernelGGL(stem_apply_pool_kernel, dim3((OW * G + 255) / 256, rows < 65535 ? rows : 65535), dim3(256), 0,
                     stream, (const bf16x8*)x, scale_bias, (bf16x8*)y, (u8x8*)idx, N, H, W, G, OH, OW);
  return (int)hipGetLastError();
}

// A/B knob: quad rows of the stem backward's partials pass (1 .. 65535; set before sizing the workspace)

// floats of workspace plx_stem_bn_pool_backward needs: level-1 [2][nblk][C] + level-2 [2][S][C]
PLX_API int64_t plx_stem_bn_pool_bwd_workspace(int N, int H, int W, int C) {
  const dim3 g = stem_bwd_grid(N, H, W, C / 8, false);
  const int64_t nblk = (int64_t)g.x * g.y;
  return 2 * (nblk + (nblk + kRowsPerSplit - 1) / kRowsPerSplit) * C;
}

// dy: gradient of the pooled output; dx: gradient of the BatchNorm input x.  dgamma / dbeta (+)= with accumulate.
PLX_API int plx_stem_bn_pool_backward(const void* dy, const void* idx, const void* x, void* dx, int N, int H, int W,
                                      int C, const float* gamma, const float* save_mean, const float* save_invstd,
                                      const float* scale_bias, float* dgamma, float* dbeta, float* coef,
                                      float* workspace, int accumulate, unsigned* counters, hipStream_t stream) {
  const int G = C / 8;
  if (N <= 0 || H <= 0 || W <= 0 || C % 8 || G > 256 || 256 % G) return 1;
  const int OH = (H - 1) / 2 + 1, OW = (W - 1) / 2 + 1;
  const dim3 grid = stem_bwd_grid(N, H, W, G, false), grid_dx = stem_bwd_grid(N, H, W, G, true);
  const int nblk = grid.x * grid.y;
  hipLaunchKernelGGL(stem_pool_bn_bwd_kernel<false>, grid, dim3(256), 0, stream, (const bf16x8*)dy, (const u8x8*)idx,
                     (const bf16x8*)x, scale_bias, save_mean, save_invstd, (const float*)nullptr, (bf16x8*)nullptr,
                     workspace, N, H, W, G, OH, OW);
  reduce_finalize_bwd(stream, workspace, nblk, workspace + 2 * (int64_t)nblk * C, counters,
                      BwdFin{C, (int64_t)N * H * W, gamma, save_mean, save_invstd, dgamma, dbeta, coef, accumulate});
  hipLaunchKernelGGL(stem_pool_bn_bwd_kernel<true>, grid_dx, dim3(256), 0, stream, (const bf16x8*)dy, (const u8x8*)idx,
                     (const bf16x8*)x, scale_bias, save_mean, save_invstd, coef, (bf16x8*)dx, (float*)nullptr, N, H,
                     W, G, OH, OW);
  return (int)hipGetLastError();
}
