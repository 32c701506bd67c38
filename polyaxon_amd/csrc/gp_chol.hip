// Blocked fp64 Cholesky for polytune's GP on MI355X (gfx950): batched over length scales, n up to a few
// thousand, with "augmented rows" that turn the same sweep into the triangular solves the GP needs.
//
// Reference hot spot: sklearn GaussianProcessRegressor.fit -> cholesky + cho_solve, called once per L-BFGS-B
// step of the length-scale fit (polyaxon/hpsearch/search_managers/bayesian_optimization/acquisition_function.py
// :17-29 builds the regressor).  At n_obs = 1000 those O(n^3) factorisations dominate a
// suggestion, so the whole LML search runs here: one batch entry per candidate length scale.
//
// Layout: matrix b starts at A + b * bstride, row-major with leading dimension ld.  Rows [0, n) hold the SPD
// matrix (lower triangle read, L written in place; the upper triangle is never touched).  Rows [n, rows) are
// appended right-hand sides r: the sweep leaves x = r L^-T in them, i.e. x^T = L^-1 r^T.  Appending y gives
// z = L^-1 y (so y^T K^-1 y = |z|^2 and the LML needs no extra solve); appending the identity gives L^-T.
//
// Right-looking, panel width PB = 32, two launches per panel:
//   gp_chol_panel_kernel   tall-panel factorisation by one wave, one row per lane held in registers: lanes
//                          0-31 factor the 32x32 diagonal block (redundantly in every workgroup -- it saves a
//                          launch) while lanes 32-63 solve 32 rows below against it (x = a L11^-T) in the same
//                          32-step loop; column k travels by v_readlane (no LDS, no barrier).  Workgroup 0
//                          writes L11 back and records the first bad pivot.
//   gp_chol_update_kernel  trailing update A[i][j] -= sum_k P[i][k] P[j][k] over the lower-trailing square and
//                          every appended row: 64x64 output tiles, 256 threads x 4x4 fp64 accumulators, both
//                          panel slices staged in LDS (row stride 33 doubles: conflict-free column reads).
// Every panel workgroup reads the diagonal block A11 from a per-matrix scratch copy (D[b], PB x PB), never from
// A itself: workgroup 0 overwrites A11 with L11 inside the same launch, and workgroups are not ordered, so a
// workgroup reading A11 from A could see L11 and solve its rows against the wrong block.  The copy is made by
// gp_chol_diag_copy_kernel for the first panel and by the update tile that produces the next A11 afterwards.
//   gp_lml_kernel          per batch entry: -0.5 |z|^2 - sum log L_jj - n/2 log 2 pi, -inf when not SPD
//                          (sklearn semantics: a failed factorisation scores -inf, no jitter retry).
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

constexpr int PB = 32;   // panel width
constexpr int UT = 64;   // update tile
constexpr int PT = 64;   // panel workgroup = one wave: PB diagonal-block rows + PT - PB rows below

__device__ __forceinline__ double readlane_f64(double v, int lane) {
  const uint64_t u = __builtin_bit_cast(uint64_t, v);
  const uint32_t lo = __builtin_amdgcn_readlane((uint32_t)u, lane);
  const uint32_t hi = __builtin_amdgcn_readlane((uint32_t)(u >> 32), lane);
  return __builtin_bit_cast(double, ((uint64_t)hi << 32) | lo);
}

// Tall-panel factorisation of columns [c, c + w) by ONE wave per workgroup: lane t < PB owns row c + t of the
// diagonal block (every workgroup factors it redundantly, which saves a launch), lane t >= PB owns row
// c + w + blockIdx.x * PB + t - PB below it; each lane keeps its 32-column row slice in registers.  Step k
// (unrolled, so k and j are compile-time lane indices): the pivot a_kk and then column k of L come from lane k / j
// by v_readlane -- no LDS and no barrier on the critical path; 1/sqrt(a_kk) is v_rsq_f64 + two Newton steps.
// Every lane scales its own a_k and applies a_j -= l_k l_jk (j > k).  So the factorisation of L11 and the
// solve of the rows below (x = a L11^-T) are the same 32-step register loop.
__global__ __launch_bounds__(PT) void gp_chol_panel_kernel(double* __restrict__ A, int n, int rows, int ld,
                                                           int64_t bstride, int c, int* __restrict__ status,
                                                           const double* __restrict__ D) {
  double* M = A + (int64_t)blockIdx.y * bstride;
  const int w = min(PB, n - c);
  const int tid = threadIdx.x;
  const bool diag = tid < PB;
  const int r = diag ? c + tid : c + w + blockIdx.x * (PT - PB) + (tid - PB);
  const bool live = diag ? tid < w : r < rows;
  double a[PB];
  // diagonal-block rows come from the scratch copy (row stride PB), the rows below from A (each owned by this lane)
  const double* src = diag ? D + (int64_t)blockIdx.y * PB * PB + (live ? tid : 0) * PB
                           : M + (int64_t)(live ? r : c) * ld + c;
#pragma unroll
  for (int j = 0; j < PB; ++j) a[j] = (live && j < w && (!diag || j <= tid)) ? src[j] : (diag && j == tid ? 1.0 : 0.0);
  int bad = 0;
#pragma unroll
  for (int k = 0; k < PB; ++k) {
    const double p = readlane_f64(a[k], k);
    const bool ok = p > 0.0;
    if (!ok && k < w && !bad) bad = c + k + 1;
    const double q = ok ? p : 1.0;
    double inv = __builtin_amdgcn_rsq(q);
    inv = inv * fma(-0.5 * q * inv, inv, 1.5);
    inv = inv * fma(-0.5 * q * inv, inv, 1.5);
    const double lk = (diag && tid == k) ? q * inv : a[k] * inv;
    a[k] = lk;
    const bool upd = !diag || tid > k;
#pragma unroll
    for (int j = k + 1; j < PB; ++j) {
      const double ljk = readlane_f64(lk, j);
      if (upd) a[j] = fma(-lk, ljk, a[j]);
    }
    __builtin_amdgcn_sched_barrier(0);  // keep the readlanes of later steps from being hoisted into SGPR spills
  }
  if (live && (!diag || blockIdx.x == 0)) {
    double* dst = M + (int64_t)r * ld + c;
#pragma unroll
    for (int j = 0; j < PB; ++j)
      if (j < w && (!diag || j <= tid)) dst[j] = a[j];
  }
  if (blockIdx.x == 0 && tid == 0 && bad && status[blockIdx.y] == 0) status[blockIdx.y] = bad;
}

__global__ __launch_bounds__(256) void gp_chol_update_kernel(double* __restrict__ A, int n, int rows, int ld,
                                                             int64_t bstride, int c, int w, double* __restrict__ D) {
  const int c0 = c + w;
  const int i0 = c0 + blockIdx.y * UT, j0 = c0 + blockIdx.x * UT;
  if (i0 < n && j0 > i0 + UT - 1) return;  // tile strictly above the diagonal of the square part
  __shared__ double Pi[UT][PB + 1];
  __shared__ double Pj[UT][PB + 1];
  double* M = A + (int64_t)blockIdx.z * bstride;
  const int tid = threadIdx.x;
  for (int e = tid; e < UT * PB; e += 256) {
    const int r = e / PB, k = e % PB;
    const bool kin = k < w;
    Pi[r][k] = (kin && i0 + r < rows) ? M[(int64_t)(i0 + r) * ld + c + k] : 0.0;
    Pj[r][k] = (kin && j0 + r < n) ? M[(int64_t)(j0 + r) * ld + c + k] : 0.0;
  }
  __syncthreads();
  const int tx = tid & 15, ty = tid >> 4;
  double acc[4][4] = {};
  for (int k = 0; k < w; ++k) {
    double a[4], b[4];
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      a[q] = Pi[ty + 16 * q][k];
      b[q] = Pj[tx + 16 * q][k];
    }
#pragma unroll
    for (int q = 0; q < 4; ++q)
#pragma unroll
      for (int s = 0; s < 4; ++s) acc[q][s] = fma(a[q], b[s], acc[q][s]);
  }
#pragma unroll
  for (int q = 0; q < 4; ++q) {
    const int i = i0 + ty + 16 * q;
    if (i >= rows) continue;
#pragma unroll
    for (int s = 0; s < 4; ++s) {
      const int j = j0 + tx + 16 * s;
      if (j < n && (i >= n || j <= i)) {
        const double v = M[(int64_t)i * ld + j] - acc[q][s];
        M[(int64_t)i * ld + j] = v;
        // the next panel's diagonal block (rows / columns [c0, c0 + PB)): its scratch copy for the panel kernel
        if (i < n && i < c0 + PB && j < c0 + PB) D[(int64_t)blockIdx.z * PB * PB + (i - c0) * PB + (j - c0)] = v;
      }
    }
  }
}

// First panel's diagonal block -> scratch (lower triangle incl. the diagonal; the rest is never read)
__global__ __launch_bounds__(256) void gp_chol_diag_copy_kernel(const double* __restrict__ A, int n, int ld,
                                                                int64_t bstride, double* __restrict__ D) {
  const double* M = A + (int64_t)blockIdx.x * bstride;
  const int w = min(PB, n);
  for (int e = threadIdx.x; e < PB * PB; e += 256) {
    const int i = e / PB, j = e % PB;
    if (i < w && j <= i) D[(int64_t)blockIdx.x * PB * PB + e] = M[(int64_t)i * ld + j];
  }
}

__global__ __launch_bounds__(256) void gp_lml_kernel(const double* __restrict__ A, int n, int ld, int64_t bstride,
                                                     const int* __restrict__ status, double* __restrict__ out) {
  const double* M = A + (int64_t)blockIdx.x * bstride;
  __shared__ double red[2][256];
  double sl = 0.0, sz = 0.0;
  for (int j = threadIdx.x; j < n; j += 256) {
    sl += log(M[(int64_t)j * ld + j]);
    const double z = M[(int64_t)n * ld + j];
    sz = fma(z, z, sz);
  }
  red[0][threadIdx.x] = sl;
  red[1][threadIdx.x] = sz;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      red[0][threadIdx.x] += red[0][threadIdx.x + s];
      red[1][threadIdx.x] += red[1][threadIdx.x + s];
    }
    __syncthreads();
  }
  if (threadIdx.x == 0) {
    const double v = -0.5 * red[1][0] - red[0][0] - 0.5 * n * 1.8378770664093453;
    out[blockIdx.x] = (status[blockIdx.x] == 0 && isfinite(v)) ? v : -INFINITY;
  }
}

// Posterior epilogue over candidate rows V (m x n fp32, row c = (L^-1 k_c)^T from one GEMM with L^-T):
// mean = v . z, var = kxx - |v|^2, then UCB / EI / POI.  One wave per candidate, lanes stride the row.
__global__ __launch_bounds__(256) void gp_acq_rows_kernel(const float* __restrict__ V, int m, int n,
                                                          const float* __restrict__ z, float kxx, int acq, float kappa,
                                                          float xi, float y_max, float* __restrict__ out,
                                                          float* __restrict__ out_mean, float* __restrict__ out_std) {
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int c = blockIdx.x * 4 + wave;
  if (c >= m) return;
  const float* v = V + (int64_t)c * n;
  float q = 0.0f, mu = 0.0f;
  for (int j = lane; j < n; j += 64) {
    const float t = v[j];
    q = fmaf(t, t, q);
    mu = fmaf(t, z[j], mu);
  }
#pragma unroll
  for (int off = 32; off > 0; off >>= 1) {
    q += __shfl_xor(q, off, 64);
    mu += __shfl_xor(mu, off, 64);
  }
  if (lane != 0) return;
  const float sd = sqrtf(fmaxf(kxx - q, 0.0f));
  float a;
  if (acq == 0) {
    a = mu + kappa * sd;
  } else {
    const float imp = mu - y_max - xi;
    const float zz = sd > 0.0f ? imp / sd : 0.0f;
    const float cdf = 0.5f * erfcf(-zz * 0.7071067811865475f);
    if (acq == 2) {
      a = sd > 0.0f ? cdf : (imp > 0.0f ? 1.0f : 0.0f);
    } else {
      const float pdf = 0.3989422804014327f * __expf(-0.5f * zz * zz);
      a = sd > 0.0f ? imp * cdf + sd * pdf : fmaxf(imp, 0.0f);
    }
  }
  out[c] = a;
  if (out_mean) out_mean[c] = mu;
  if (out_std) out_std[c] = sd;
}

}  // namespace

// In-place blocked Cholesky of nb matrices (see the layout above). status: int[nb], zeroed by the caller;
// status[b] = 1-based column of the first non-positive pivot.  scratch: device fp64 [nb][PB][PB] (contents ignored).
PLX_API int plx_gp_chol_aug_f64(double* A, int n, int rows, int ld, long long bstride, int nb, int* status,
                                double* scratch, hipStream_t stream) {
  if (n <= 0 || rows < n || ld < n || nb <= 0 || scratch == nullptr) return 1;
  hipLaunchKernelGGL(gp_chol_diag_copy_kernel, dim3(nb), dim3(256), 0, stream, A, n, ld, (int64_t)bstride, scratch);
  for (int c = 0; c < n; c += PB) {
    const int w = n - c < PB ? n - c : PB;
    const int below = rows - c - w;
    const int gx = below > 0 ? (below + PT - PB - 1) / (PT - PB) : 1;
    hipLaunchKernelGGL(gp_chol_panel_kernel, dim3(gx, nb), dim3(PT), 0, stream, A, n, rows, ld, (int64_t)bstride,
                       c, status, (const double*)scratch);
    const int c0 = c + w;
    if (c0 < n) {
      dim3 grid((n - c0 + UT - 1) / UT, (rows - c0 + UT - 1) / UT, nb);
      hipLaunchKernelGGL(gp_chol_update_kernel, grid, dim3(256), 0, stream, A, n, rows, ld, (int64_t)bstride, c, w,
                         scratch);
    }
  }
  return (int)hipGetLastError();
}

PLX_API int plx_gp_chol_scratch_doubles() { return PB * PB; }

// LML per batch entry of a factor produced by plx_gp_chol_aug_f64 with y appended as row n.
PLX_API int plx_gp_lml_f64(const double* A, int n, int ld, long long bstride, int nb, const int* status, double* out,
                           hipStream_t stream) {
  if (n <= 0 || nb <= 0) return 1;
  hipLaunchKernelGGL(gp_lml_kernel, dim3(nb), dim3(256), 0, stream, A, n, ld, (int64_t)bstride, status, out);
  return (int)hipGetLastError();
}

PLX_API int plx_gp_acq_rows(const float* V, int m, int n, const float* z, float kxx, int acq, float kappa, float xi,
                            float y_max, float* out, float* out_mean, float* out_std, hipStream_t stream) {
  if (m <= 0 || n <= 0) return 1;
  hipLaunchKernelGGL(gp_acq_rows_kernel, dim3((m + 3) / 4), dim3(256), 0, stream, V, m, n, z, kxx, acq, kappa, xi,
                     y_max, out, out_mean, out_std);
  return (int)hipGetLastError();
}
