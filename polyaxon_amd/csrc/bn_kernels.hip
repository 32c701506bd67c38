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
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kBlock = 256;

struct alignas(16) bf16x8 {
  uint16_t v[8];
};

__device__ __forceinline__ float bf2f(uint16_t b) { return __uint_as_float(((uint32_t)b) << 16); }

__device__ __forceinline__ uint16_t f2bf(float f) {  // round-to-nearest-even
  uint32_t u = __float_as_uint(f);
  if ((u & 0x7fffffffu) > 0x7f800000u) return (uint16_t)((u >> 16) | 0x40);  // NaN stays NaN
  u += 0x7fffu + ((u >> 16) & 1u);
  return (uint16_t)(u >> 16);
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

__global__ __launch_bounds__(256) void bn_partial_reduce_kernel(const float* __restrict__ part, int nblk, int C,
                                                                float* __restrict__ out, int S) {
  __shared__ float sh[256];
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane = threadIdx.x >> 6;
  const int s = blockIdx.y, which = blockIdx.z;
  const float* src = part + (int64_t)which * nblk * C;
  const int b0 = s * kRowsPerSplit;
  int b1 = b0 + kRowsPerSplit;
  if (b1 > nblk) b1 = nblk;
  float acc = 0.f;
  if (c < C) {
#pragma unroll 4
    for (int b = b0 + lane; b < b1; b += 4) acc += src[(int64_t)b * C + c];
  }
  sh[threadIdx.x] = acc;
  __syncthreads();
  if (lane == 0 && c < C) {
    const int t = threadIdx.x;
    out[((int64_t)which * S + s) * C + c] = sh[t] + sh[t + 64] + sh[t + 128] + sh[t + 192];
  }
}

// Level-2 -> per-channel totals for the finalize kernels: block = 64 channels x 4 split lanes-groups, each group
// sums every 4th of the S partial rows (independent loads, fp64 accumulation), then the 4 group sums are combined
// through LDS in a fixed order (deterministic).  One thread per channel walking all S rows serially was 19 us per
// backward BatchNorm on the 56x56 layers (S ~ 100 dependent-latency iterations on a single 256-thread block).
constexpr int kFinSplit = 4;
__device__ __forceinline__ bool fin_sum2(const float* __restrict__ pa, const float* __restrict__ pb, int nblk, int C,
                                         double& A, double& B) {
  __shared__ double sh[2][kFinSplit][64];
  const int lc = threadIdx.x & 63, sp = threadIdx.x >> 6;
  const int c = blockIdx.x * 64 + lc;
  double a0 = 0.0, b0 = 0.0, a1 = 0.0, b1 = 0.0;
  if (c < C) {
    int b = sp;
    for (; b + kFinSplit < nblk; b += 2 * kFinSplit) {
      const float x0 = pa[(int64_t)b * C + c], y0 = pb[(int64_t)b * C + c];
      const float x1 = pa[(int64_t)(b + kFinSplit) * C + c], y1 = pb[(int64_t)(b + kFinSplit) * C + c];
      a0 += x0; b0 += y0; a1 += x1; b1 += y1;
    }
    if (b < nblk) { a0 += pa[(int64_t)b * C + c]; b0 += pb[(int64_t)b * C + c]; }
  }
  sh[0][sp][lc] = a0 + a1;
  sh[1][sp][lc] = b0 + b1;
  __syncthreads();
  if (sp != 0 || c >= C) return false;
  A = ((sh[0][0][lc] + sh[0][1][lc]) + sh[0][2][lc]) + sh[0][3][lc];
  B = ((sh[1][0][lc] + sh[1][1][lc]) + sh[1][2][lc]) + sh[1][3][lc];
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

__device__ __forceinline__ void fwd_finalize(const float* psum, const float* psq, int nblk, const FwdFin& f) {
  double S, Q;  // level-2 partials per channel, summed in fp64
  if (!fin_sum2(psum, psq, nblk, f.C, S, Q)) return;
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

__device__ __forceinline__ void bwd_finalize(const float* pdz, const float* pdzx, int nblk, const BwdFin& f) {
  double A, B;
  if (!fin_sum2(pdz, pdzx, nblk, f.C, A, B)) return;
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
__device__ __forceinline__ bool reduce_l2_last(const float* __restrict__ part, int nblk, int C, float* l2, int S,
                                               unsigned* cnt) {
  __shared__ float sh[2][256];
  __shared__ int s_last;
  const int c = blockIdx.x * 64 + (threadIdx.x & 63);
  const int lane = threadIdx.x >> 6;
  const int s = blockIdx.y;
  const int b0 = s * kRowsPerSplit;
  int b1 = b0 + kRowsPerSplit;
  if (b1 > nblk) b1 = nblk;
  float a0 = 0.f, a1 = 0.f;
  if (c < C) {
    const float* p0 = part;
    const float* p1 = part + (int64_t)nblk * C;
#pragma unroll 4
    for (int b = b0 + lane; b < b1; b += 4) {
      a0 += p0[(int64_t)b * C + c];
      a1 += p1[(int64_t)b * C + c];
    }
  }
  sh[0][threadIdx.x] = a0;
  sh[1][threadIdx.x] = a1;
  __syncthreads();
  if (lane == 0 && c < C) {
    const int t = threadIdx.x;
    l2[(int64_t)s * C + c] = sh[0][t] + sh[0][t + 64] + sh[0][t + 128] + sh[0][t + 192];
    l2[((int64_t)S + s) * C + c] = sh[1][t] + sh[1][t + 64] + sh[1][t + 128] + sh[1][t + 192];
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // every storing wave drains
  __syncthreads();
  if (threadIdx.x == 0) {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    const unsigned old = __hip_atomic_fetch_add(cnt + blockIdx.x, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    const int last = old == (unsigned)(S - 1);
    if (last) {
      __hip_atomic_store(cnt + blockIdx.x, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
      __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "agent");
      asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    }
    s_last = last;
  }
  __syncthreads();
  return s_last != 0;
}

__global__ __launch_bounds__(256) void bn_fwd_reduce_finalize_kernel(const float* __restrict__ part, int nblk,
                                                                     float* l2, int S, unsigned* cnt, FwdFin f) {
  if (!reduce_l2_last(part, nblk, f.C, l2, S, cnt)) return;
  fwd_finalize(l2, l2 + (int64_t)S * f.C, S, f);
}

__global__ __launch_bounds__(256) void bn_bwd_reduce_finalize_kernel(const float* __restrict__ part, int nblk,
                                                                     float* l2, int S, unsigned* cnt, BwdFin f) {
  if (!reduce_l2_last(part, nblk, f.C, l2, S, cnt)) return;
  bwd_finalize(l2, l2 + (int64_t)S * f.C, S, f);
}

__global__ __launch_bounds__(256) void bn_fwd_finalize_kernel(const float* __restrict__ psum, const float* __restrict__ psq, int nblk,
                                       const uint16_t* __restrict__ x_row0, int C, int64_t M,
                                       const float* __restrict__ gamma, const float* __restrict__ beta, float eps,
                                       float momentum, float* __restrict__ running_mean,
                                       float* __restrict__ running_var, float* __restrict__ save_mean,
                                       float* __restrict__ save_invstd, float* __restrict__ scale,
                                       float* __restrict__ bias) {
  double S, Q;  // level-2 partials per channel, summed in fp64
  if (!fin_sum2(psum, psq, nblk, C, S, Q)) return;
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
__global__ __launch_bounds__(kBlock) void bn_apply_kernel(const bf16x8* __restrict__ x, const bf16x8* __restrict__ res,
                                                          bf16x8* __restrict__ y, const float* __restrict__ scale,
                                                          const float* __restrict__ bias, int64_t n_vec, int G,
                                                          int relu, uint8_t* __restrict__ mask,
                                                          const float* __restrict__ rsb) {
  const int64_t stride = (int64_t)gridDim.x * blockDim.x;  // multiple of G (G | 256 or G % 256 == 0 handled by host)
  int64_t i = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;
  if (i >= n_vec) return;
  const int cg = (int)(i % G);
  float a[8], b[8], ra[8], rb[8];
#pragma unroll
  for (int k = 0; k < 8; ++k) {
    a[k] = scale[cg * 8 + k];
    b[k] = bias[cg * 8 + k];
    // rsb: the residual is the raw input of a BatchNorm (no activation) whose apply pass is deferred to here:
    // res' = res * rsb[c] + rsb[C + c]  (a ResNet downsampling branch feeds only this add)
    ra[k] = rsb != nullptr ? rsb[cg * 8 + k] : 1.f;
    rb[k] = rsb != nullptr ? rsb[G * 8 + cg * 8 + k] : 0.f;
  }
  for (; i < n_vec; i += stride) {
    float v[8];
    load8(x + i, v);
#pragma unroll
    for (int k = 0; k < 8; ++k) v[k] = fmaf(v[k], a[k], b[k]);
    if (res != nullptr) {
      float r[8];
      load8(res + i, r);
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] += fmaf(r[k], ra[k], rb[k]);
    }
    if (relu) {
#pragma unroll
      for (int k = 0; k < 8; ++k) v[k] = fmaxf(v[k], 0.f);
    }
    store8(y + i, v);
    if (mask != nullptr) {
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
    load8(x + off, xv);
    load8(dy + off, g);
    if (relu) {
      const uint32_t mb = mask[off];
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

__global__ __launch_bounds__(256) void bn_bwd_finalize_kernel(const float* __restrict__ pdz, const float* __restrict__ pdzx, int nblk, int C,
                                       int64_t M, const float* __restrict__ gamma, const float* __restrict__ mean,
                                       const float* __restrict__ invstd, float* __restrict__ dgamma,
                                       float* __restrict__ dbeta, float* __restrict__ coef, int accumulate) {
  double A, B;
  if (!fin_sum2(pdz, pdzx, nblk, C, A, B)) return;
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
template <bool RP>
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
    load8(x + i, xv);
    load8(dy + i, g);
    if (relu) {
      const uint32_t mb = mask[i];
#pragma unroll
      for (int k = 0; k < 8; ++k) g[k] = (mb >> k) & 1u ? g[k] : 0.f;
    }
    if (dres != nullptr) store8(dres + i, g);
    if constexpr (rp) {
      float x2[8];
      load8(rb.x + i, x2);
      const uint32_t m2 = rb.mask != nullptr ? rb.mask[i] : 0xffu;
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
  if (rb.part != nullptr)
    hipLaunchKernelGGL(bn_bwd_dx_kernel<true>, grid, dim3(kBlock), 0, stream, (const bf16x8*)x, mask,
                       (const bf16x8*)dy, (bf16x8*)dx, (bf16x8*)dres, coef, n_vec, G, relu, rb);
  else
    hipLaunchKernelGGL(bn_bwd_dx_kernel<false>, grid, dim3(kBlock), 0, stream, (const bf16x8*)x, mask,
                       (const bf16x8*)dy, (bf16x8*)dx, (bf16x8*)dres, coef, n_vec, G, relu, rb);
}

// level-1 partials [2][nblk][C] -> finalize: one fused launch with a counter array (>= ceil(C/64) zeroed words),
// else the reduce and finalize kernels back to back
inline void reduce_finalize_fwd(hipStream_t stream, const float* part, int nblk, float* l2, unsigned* cnt,
                                const FwdFin& f) {
  const int C = f.C, S = (nblk + kRowsPerSplit - 1) / kRowsPerSplit;
  if (cnt != nullptr) {
    hipLaunchKernelGGL(bn_fwd_reduce_finalize_kernel, dim3((C + 63) / 64, S), dim3(256), 0, stream, part, nblk, l2, S,
                       cnt, f);
    return;
  }
  hipLaunchKernelGGL(bn_partial_reduce_kernel, dim3((C + 63) / 64, S, 2), dim3(256), 0, stream, part, nblk, C, l2, S);
  hipLaunchKernelGGL(bn_fwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, stream, l2, l2 + (int64_t)S * C, S,
                     f.x_row0, C, f.M, f.gamma, f.beta, f.eps, f.momentum, f.running_mean, f.running_var, f.save_mean,
                     f.save_invstd, f.scale, f.bias);
}

inline void reduce_finalize_bwd(hipStream_t stream, const float* part, int nblk, float* l2, unsigned* cnt,
                                const BwdFin& f) {
  const int C = f.C, S = (nblk + kRowsPerSplit - 1) / kRowsPerSplit;
  if (cnt != nullptr) {
    hipLaunchKernelGGL(bn_bwd_reduce_finalize_kernel, dim3((C + 63) / 64, S), dim3(256), 0, stream, part, nblk, l2, S,
                       cnt, f);
    return;
  }
  hipLaunchKernelGGL(bn_partial_reduce_kernel, dim3((C + 63) / 64, S, 2), dim3(256), 0, stream, part, nblk, C, l2, S);
  hipLaunchKernelGGL(bn_bwd_finalize_kernel, dim3((C + 63) / 64), dim3(256), 0, stream, l2, l2 + (int64_t)S * C, S, C,
                     f.M, f.gamma, f.mean, f.invstd, f.dgamma, f.dbeta, f.coef, f.accumulate);
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
    hipLaunchKernelGGL(bn_apply_kernel, dim3(apply_grid(n_vec, p.G)), dim3(kBlock), 0, stream, (const bf16x8*)x,
                       (const bf16x8*)res, (bf16x8*)y, scale_bias, scale_bias + C, n_vec, p.G, relu,
                       relu ? mask : nullptr, res_sb);
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
    hipLaunchKernelGGL(bn_apply_kernel, dim3(apply_grid(n_vec, p.G)), dim3(kBlock), 0, stream, (const bf16x8*)x,
                       (const bf16x8*)res, (bf16x8*)y, scale_bias, scale_bias + C, n_vec, p.G, relu,
                       relu ? mask : nullptr, res_sb);
  return (int)hipGetLastError();
}

PLX_API int plx_bn_apply(const void* x, const void* res, void* y, int64_t M, int C, const float* scale_bias, int relu,
                         hipStream_t stream) {
  Plan p;
  if (!plan_for(M, C, &p)) return 1;
  const int64_t n_vec = M * p.G;
  hipLaunchKernelGGL(bn_apply_kernel, dim3(apply_grid(n_vec, p.G)), dim3(kBlock), 0, stream, (const bf16x8*)x,
                     (const bf16x8*)res, (bf16x8*)y, scale_bias, scale_bias + C, n_vec, p.G, relu, nullptr, nullptr);
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
  hipLaunchKernelGGL(bn_bwd_reduce_kernel, dim3(p.nblk, p.gy), dim3(kBlock), 0, stream, (const bf16x8*)x,
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
