// polytune bracket kernels for MI355X (gfx950).
//
// Reference behaviour being replaced:
//   * Hyperband rung reduction: `sorted(experiments_metrics, key=metric, reverse=maximize)[:n_keep]`
//     (polyaxon/hpsearch/iteration_managers/hyperband.py:52-77), executed once per rung in Python on
//     rows pulled out of Postgres JSON (polyaxon/db/models/experiment_groups.py:223-246).
//   * Early-stopping check: "does any experiment have last_metric[m] >=/<= value"
//     (polyaxon/db/models/experiment_groups.py:211-221).
//
// MI355X design: the metric of every (bracket, config) slot lives in ONE device tensor [B, C] that the
// trial executors write into directly (train_kernels.hip: plx_commit_metric), so a rung decision is a
// single launch over all brackets, not a DB round trip.
//
//   plx_topk_brackets   one workgroup per bracket; the bracket's (key, index) pairs are bitonic-sorted in
//                       LDS (C <= 2048 -> 16 KiB per workgroup) and the full order is written back;
//                       invalid / NaN entries sort last, ties keep the lower index first (stable, like
//                       Python's sorted()).
//   plx_early_stop_any  one wave64 per rule, ballot-OR over experiments, flag per rule.
//   plx_philox_sample   random-search suggestions (reference search_managers/utils.py:41-64):
//                       one thread per (suggestion, parameter) draws from a counter-based Philox4x32-10 stream,
//                       so suggestion r of a seeded search is the same whatever n or the device; the numpy twin
//                       in polytune/sampler.py reproduces it bit for bit on the host.
#include <hip/hip_runtime.h>
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int kSortBlock = 256;
constexpr int kMaxSort = 2048;

// Total order on (key, idx): NaN/invalid keys are +inf-like and go last; ties broken by index.
__device__ __forceinline__ bool less_pair(float ka, int ia, float kb, int ib) {
  const bool na = ka != ka, nb = kb != kb;
  if (na != nb) return nb;  // non-NaN < NaN
  if (!na && ka != kb) return ka < kb;
  return ia < ib;
}

__global__ __launch_bounds__(kSortBlock) void topk_brackets_kernel(const float* __restrict__ metrics,
                                                                   const int* __restrict__ counts, int C,
                                                                   int ld, int maximize, int* __restrict__ order,
                                                                   int P) {
  __shared__ float skey[kMaxSort];
  __shared__ int sidx[kMaxSort];
  const int b = blockIdx.x;
  const int cnt = counts[b];
  const float* row = metrics + (int64_t)b * ld;
  for (int i = threadIdx.x; i < P; i += blockDim.x) {
    float k = __builtin_nanf("");
    if (i < cnt && i < C) {
      const float v = row[i];
      k = maximize ? -v : v;
    }
    skey[i] = k;
    sidx[i] = i;
  }
  __syncthreads();
  for (int k = 2; k <= P; k <<= 1) {
    for (int j = k >> 1; j > 0; j >>= 1) {
      for (int i = threadIdx.x; i < P; i += blockDim.x) {
        const int l = i ^ j;
        if (l > i) {
          const bool asc = (i & k) == 0;
          const float ki = skey[i], kl = skey[l];
          const int ii = sidx[i], il = sidx[l];
          const bool swap = asc ? less_pair(kl, il, ki, ii) : less_pair(ki, ii, kl, il);
          if (swap) {
            skey[i] = kl;
            skey[l] = ki;
            sidx[i] = il;
            sidx[l] = ii;
          }
        }
      }
      __syncthreads();
    }
  }
  int* out = order + (int64_t)b * ld;
  for (int i = threadIdx.x; i < C; i += blockDim.x) out[i] = i < cnt ? sidx[i] : -1;
}

// metrics: [E, M] row-major (NaN = metric not reported). rules r: metric column, threshold, maximize.
// flags[r] = 1 if any experiment satisfies rule r (>= for maximize, <= for minimize).
__global__ void early_stop_any_kernel(const float* __restrict__ metrics, int E, int M,
                                      const int* __restrict__ rule_col, const float* __restrict__ rule_val,
                                      const int* __restrict__ rule_max, int* __restrict__ flags) {
  const int r = blockIdx.x;
  const int col = rule_col[r];
  const float thr = rule_val[r];
  const int mx = rule_max[r];
  int hit = 0;
  for (int e = threadIdx.x; e < E; e += blockDim.x) {
    const float v = metrics[(int64_t)e * M + col];
    hit |= (v == v) && (mx ? v >= thr : v <= thr);
  }
  const unsigned long long any = __ballot(hit);
  __shared__ int sh;
  if (threadIdx.x == 0) sh = 0;
  __syncthreads();
  if ((threadIdx.x & 63) == 0 && any) atomicOr(&sh, 1);
  __syncthreads();
  if (threadIdx.x == 0) flags[r] = sh;
}

// ---------------------------------------------------------------- Philox sampler
struct U4 {
  uint32_t x, y, z, w;
};

__device__ __forceinline__ U4 philox10(U4 c, uint32_t k0, uint32_t k1) {
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

// 53-bit uniform in [0, 1) from two words
__device__ __forceinline__ double u53(uint32_t a, uint32_t b) {
  return (double)(((uint64_t)(a >> 5) << 26) | (uint64_t)(b >> 6)) * (1.0 / 9007199254740992.0);
}

// One hyper-parameter: kind 0 uniform(a, b), 1 normal(a, b) (log: exp of the draw; q > 0: round(x / q) * q),
// 2 discrete index in [0, count), 3 categorical with probabilities (index into the cumulative table at cdf).
struct ParamDesc {
  int kind, log, count, cdf;
  double a, b, q;
};

__global__ __launch_bounds__(256) void philox_sample_kernel(const ParamDesc* __restrict__ desc,
                                                            const double* __restrict__ cdf, int P, int64_t n,
                                                            int64_t row0, uint32_t k0, uint32_t k1,
                                                            double* __restrict__ out) {
  // no FMA contraction: the host twin (numpy) rounds every multiply and add separately, so the affine maps
  // here must too for the two streams to agree bit for bit
#pragma clang fp contract(off)
  const int64_t e = (int64_t)blockIdx.x * 256 + threadIdx.x;
  if (e >= n * P) return;
  const int64_t r = e / P;
  const int p = (int)(e - r * P);
  const int64_t row = row0 + r;
  const U4 w = philox10(U4{(uint32_t)row, (uint32_t)(row >> 32), (uint32_t)p, 0x5a3e1e5u}, k0, k1);
  const ParamDesc d = desc[p];
  const double u = u53(w.x, w.y);
  double v;
  if (d.kind == 0) {
    v = d.a + (d.b - d.a) * u;
  } else if (d.kind == 1) {
    const double u1 = 1.0 - u;  // (0, 1]
    const double u2 = u53(w.z, w.w);
    v = d.a + d.b * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
  } else if (d.kind == 2) {
    const int i = (int)(u * d.count);
    v = (double)(i < d.count ? i : d.count - 1);
  } else {
    int i = 0;
    while (i < d.count - 1 && cdf[d.cdf + i] <= u) ++i;
    v = (double)i;
  }
  if (d.kind <= 1) {
    if (d.log) v = exp(v);
    if (d.q > 0.0) v = rint(v / d.q) * d.q;
  }
  out[e] = v;
}

}  // namespace

PLX_API int plx_topk_brackets(const float* metrics, const int* counts, int n_brackets, int C, int ld, int maximize,
                              int* order, hipStream_t stream) {
  if (C > kMaxSort || C <= 0 || n_brackets <= 0 || ld < C) return 1;
  int P = 1;
  while (P < C) P <<= 1;
  hipLaunchKernelGGL(topk_brackets_kernel, dim3(n_brackets), dim3(kSortBlock), 0, stream, metrics, counts, C, ld,
                     maximize, order, P);
  return (int)hipGetLastError();
}

PLX_API int plx_early_stop_any(const float* metrics, int E, int M, const int* rule_col, const float* rule_val,
                               const int* rule_max, int n_rules, int* flags, hipStream_t stream) {
  if (n_rules <= 0) return 0;
  hipLaunchKernelGGL(early_stop_any_kernel, dim3(n_rules), dim3(256), 0, stream, metrics, E, M, rule_col, rule_val,
                     rule_max, flags);
  return (int)hipGetLastError();
}

// out[n][P] (fp64, device) = rows row0 .. row0 + n - 1 of the seeded suggestion stream; desc: ParamDesc[P] and
// cdf: the concatenated cumulative probability tables, both device memory.
PLX_API int plx_philox_sample(const void* desc, const double* cdf, int P, long long n, long long row0,
                              unsigned long long seed, double* out, hipStream_t stream) {
  if (P <= 0 || n <= 0 || row0 < 0) return 1;
  const int64_t total = (int64_t)n * P;
  hipLaunchKernelGGL(philox_sample_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream,
                     (const ParamDesc*)desc, cdf, P, (int64_t)n, (int64_t)row0, (uint32_t)seed, (uint32_t)(seed >> 32),
                     out);
  return (int)hipGetLastError();
}

PLX_API int plx_philox_desc_size() { return (int)sizeof(ParamDesc); }
