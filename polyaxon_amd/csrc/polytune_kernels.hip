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
