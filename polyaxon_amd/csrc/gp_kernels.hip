// Gaussian-process kernels for polytune's Bayesian optimisation on MI355X (gfx950).
//
// Reference hot spots: sklearn GaussianProcessRegressor.fit / predict(return_std) and the
// UCB/EI/POI acquisition evaluated over random warm-up candidates and L-BFGS-B restarts
// (polyaxon/hpsearch/search_managers/bayesian_optimization/acquisition_function.py:31-115).
//
//   plx_gp_kmat         K[i,j] = k(A_i, B_j). Pairwise squared distances from the GEMM identity
//                       |a|^2 + |b|^2 - 2 a.b with the exact-fp32 MFMA v_mfma_f32_32x32x2_f32 (64x64 block
//                       tile = 2x2 waves of 32x32, A/B tiles staged in LDS), Matern / RBF fused in the
//                       epilogue.  Matern with a non half-integer nu (the reference's nu = 1.9) is evaluated
//                       on the device through K_nu(z) = int_0^inf exp(-z cosh t) cosh(nu t) dt with the
//                       trapezoidal rule (spectrally accurate for this doubly-exponentially decaying
//                       integrand), so no Bessel library is needed.  That quadrature runs once per nu to fill
//                       a (value, derivative) table (plx_gp_matern_table); every Gram / cross-kernel entry is
//                       then a cubic Hermite lookup (16384 nodes over s in [0, 50]); the fp64 Gram takes the exact power
//                       series below s = 2 (matern_series_f64).
//   plx_gp_chol         in-place Cholesky of the n x n Gram matrix (n <= 128) inside ONE workgroup, fp64 in
//                       LDS (128 KiB), right-looking, with the diagonal jitter retry done by the caller.
//   plx_gp_predict_acq  per candidate: k* (n kernel evals), mean = k*.alpha, v = L^-1 k* by forward
//                       substitution held in registers (N templated: 16/32/64/128, fully unrolled), var,
//                       then the UCB / EI / POI epilogue (erfc-based Phi) and a per-block argmax.
//                       X, L and alpha are staged once per workgroup in LDS and read as broadcasts.
#include <hip/hip_runtime.h>
#include <math.h>
#include <stdint.h>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

typedef float f32x16 __attribute__((ext_vector_type(16)));

enum KernelKind { kRBF = 0, kMatern05 = 1, kMatern15 = 2, kMatern25 = 3, kMaternNu = 4, kSqDist = 5 };

__device__ __forceinline__ float bessel_k_nu(float z, float nu) {
  // K_nu(z) = int_0^inf exp(-z cosh t) cosh(nu t) dt, trapezoid on [0, T], T where the integrand < 1e-9
  const float tmax = acoshf(fmaxf(1.0f, 25.0f / fmaxf(z, 1e-6f))) + 2.0f;
  const int n = 96;
  const float h = tmax / n;
  float s = 0.5f * __expf(-z);  // t = 0 term (cosh 0 = 1)
  for (int i = 1; i <= n; ++i) {
    const float t = i * h;
    const float et = __expf(t), ei = 1.0f / et;
    const float ch = 0.5f * (et + ei);
    const float w = (i == n) ? 0.5f : 1.0f;
    s += w * __expf(-z * ch) * coshf(nu * t);
  }
  return s * h;
}

// Matern with a general nu, tabulated once per nu by gp_matern_table_kernel: node i at r_i = i h holds
// (f(r_i), h f'(r_i)); a lookup is one cubic Hermite step instead of a 96/160-node quadrature.  The first
// interval of nu < 1 (f'(0) unbounded) and tab == nullptr fall back to the quadrature.
struct MaternTab {
  const double* t64;
  const float* t32;
  double inv_h;
  int n;
};

template <typename T>
__device__ __forceinline__ T hermite(T t, T f0, T d0, T f1, T d1) {
  const T t2 = t * t, t3 = t2 * t;
  return (2 * t3 - 3 * t2 + 1) * f0 + (t3 - 2 * t2 + t) * d0 + (3 * t2 - 2 * t3) * f1 + (t3 - t2) * d1;
}

__device__ __forceinline__ float kernel_from_sq(float sq, int kind, float inv_ls2, float nu, float matern_c,
                                                const MaternTab& tab) {
  sq = fmaxf(sq, 0.0f);
  if (kind == kSqDist) return sq;
  const float r2 = sq * inv_ls2;
  if (kind == kRBF) return __expf(-0.5f * r2);
  const float r = sqrtf(r2);
  if (kind == kMatern05) return __expf(-r);
  if (kind == kMatern15) {
    const float a = 1.7320508075688772f * r;
    return (1.0f + a) * __expf(-a);
  }
  if (kind == kMatern25) {
    const float a = 2.23606797749979f * r;
    return (1.0f + a + a * a * (1.0f / 3.0f)) * __expf(-a);
  }
  if (tab.t32) {
    const float u = r * (float)tab.inv_h;
    const int i = (int)u;
    if (i >= tab.n - 1) return 0.0f;
    if (i > 0 || nu >= 1.0f) {
      const float2 a = reinterpret_cast<const float2*>(tab.t32)[i];
      const float2 b = reinterpret_cast<const float2*>(tab.t32)[i + 1];
      return hermite(u - (float)i, a.x, a.y, b.x, b.y);
    }
  }
  // general nu: c * s^nu * K_nu(s), s = sqrt(2 nu) r, c = 2^(1-nu)/Gamma(nu); k(0) = 1
  const float s = sqrtf(2.0f * nu) * r;
  if (s < 1e-6f) return 1.0f;
  return matern_c * __powf(s, nu) * bessel_k_nu(s, nu);
}

// ------------------------------------------------------------------------------------------ kmat
constexpr int KB = 64;      // block tile (rows of A, rows of B)
constexpr int KMAX_D = 64;  // feature dim staged in LDS (padded to even)

__global__ __launch_bounds__(256) void gp_kmat_kernel(const float* __restrict__ A, const float* __restrict__ B, int n,
                                                      int m, int d, float* __restrict__ K, int ldk, int kind,
                                                      float inv_ls2, float nu, float matern_c, int add_diag,
                                                      float diag, MaternTab tab) {
  __shared__ float sA[KB][KMAX_D + 1];
  __shared__ float sB[KB][KMAX_D + 1];
  __shared__ float nA[KB], nB[KB];
  const int row0 = blockIdx.y * KB, col0 = blockIdx.x * KB;
  const int dpad = (d + 1) & ~1;
  for (int e = threadIdx.x; e < KB * dpad; e += 256) {
    const int r = e / dpad, k = e % dpad;
    const int ga = row0 + r, gb = col0 + r;
    sA[r][k] = (ga < n && k < d) ? A[(int64_t)ga * d + k] : 0.0f;
    sB[r][k] = (gb < m && k < d) ? B[(int64_t)gb * d + k] : 0.0f;
  }
  __syncthreads();
  if (threadIdx.x < KB) {
    float sa = 0.f, sb = 0.f;
    for (int k = 0; k < dpad; ++k) {
      sa = fmaf(sA[threadIdx.x][k], sA[threadIdx.x][k], sa);
      sb = fmaf(sB[threadIdx.x][k], sB[threadIdx.x][k], sb);
    }
    nA[threadIdx.x] = sa;
    nB[threadIdx.x] = sb;
  }
  __syncthreads();
  const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
  const int wr = (wave >> 1) * 32, wc = (wave & 1) * 32;
  f32x16 acc = {0};
  // v_mfma_f32_32x32x2_f32: lane l holds A[i = l&31][k = l>>5] and B[k = l>>5][j = l&31]; here B = Bmat^T
  for (int k = 0; k < dpad; k += 2) {
    const float a = sA[wr + (lane & 31)][k + (lane >> 5)];
    const float b = sB[wc + (lane & 31)][k + (lane >> 5)];
    acc = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc, 0, 0, 0);
  }
#pragma unroll
  for (int r = 0; r < 16; ++r) {
    const int i = wr + (r & 3) + 8 * (r >> 2) + 4 * (lane >> 5);
    const int j = wc + (lane & 31);
    const int gi = row0 + i, gj = col0 + j;
    if (gi < n && gj < m) {
      const float sq = nA[i] + nB[j] - 2.0f * acc[r];
      float v = kernel_from_sq(sq, kind, inv_ls2, nu, matern_c, tab);
      if (add_diag && gi == gj) v += diag;
      K[(int64_t)gi * ldk + gj] = v;
    }
  }
}

// ------------------------------------------------------------------------------------------ batched fp64 Gram
// Length-scale fit (log marginal likelihood over a batch of scales): K[b][i][j] = k(|X_i - X_j| / ls_b) + diag
// in fp64 end to end.  The fp32 MFMA Gram above is exact enough for the posterior, but a long length scale
// makes K nearly singular (entries 1 - O(r^2)) and fp32 rounding turns it indefinite, so the LML search would
// wrongly reject the scales the fp64 objective prefers.  One thread per (i, j <= i) pair: the distance is
// summed once in fp64 from direct differences and every scale of the batch is written (mirrored to (j, i)).
__device__ __forceinline__ double bessel_k_nu_f64(double z, double nu) {
  const double tmax = acosh(fmax(1.0, 40.0 / fmax(z, 1e-12))) + 2.5;
  const int n = 160;
  const double h = tmax / n;
  double s = 0.5 * exp(-z);
  for (int i = 1; i <= n; ++i) {
    const double t = i * h;
    const double et = exp(t), ei = 1.0 / et;
    const double w = (i == n) ? 0.5 : 1.0;
    s += w * exp(-z * 0.5 * (et + ei)) * 0.5 * (exp(nu * t) + exp(-nu * t));
  }
  return s * h;
}

// Small-s Matern-nu from the power series of K_nu (nu not an integer):
//   s^nu K_nu(s) = pi 2^nu / (2 sin(nu pi)) * sum_k [ (s/2)^2k / (k! G(k-nu+1)) - (s/2)^(2k+2nu) / (k! G(k+nu+1)) ]
// whose k = 0 term times c = 2^(1-nu)/G(nu) is exactly 1 (reflection formula), so f = 1 + (small terms) with no
// cancellation: the 1 - k(r) differences that set a long-length-scale Gram's small eigenvalues keep full fp64
// precision (a lookup table's interpolation error would swamp them).
__device__ __forceinline__ bool s_small(double r, double nu) {
  return sqrt(2.0 * nu) * r < 2.0 && fabs(nu - rint(nu)) > 1e-3;
}

__device__ __forceinline__ double matern_series_f64(double s, double nu, double matern_c) {
  const double pref = matern_c * 3.141592653589793 * exp2(nu) / (2.0 * sin(nu * 3.141592653589793));
  const double x = 0.25 * s * s;
  double a = pref / tgamma(1.0 - nu);            // == 1 up to rounding: the k = 0 term, added exactly below
  double b = pref * pow(0.5 * s, 2.0 * nu) / tgamma(1.0 + nu);
  double sum = -b;
#pragma unroll
  for (int k = 1; k <= 20; ++k) {
    a *= x / (k * (k - nu));
    b *= x / (k * (k + nu));
    sum += a - b;
  }
  return 1.0 + sum;
}

__device__ __forceinline__ double kernel_from_sq_f64(double r2, int kind, double nu, double matern_c,
                                                     const MaternTab& tab) {
  if (kind == kRBF) return exp(-0.5 * r2);
  const double r = sqrt(r2);
  if (kind == kMatern05) return exp(-r);
  if (kind == kMatern15) {
    const double a = 1.7320508075688772 * r;
    return (1.0 + a) * exp(-a);
  }
  if (kind == kMatern25) {
    const double a = 2.23606797749979 * r;
    return (1.0 + a + a * a / 3.0) * exp(-a);
  }
  if (s_small(r, nu)) return matern_series_f64(sqrt(2.0 * nu) * r, nu, matern_c);
  if (tab.t64) {
    const double u = r * tab.inv_h;
    const int i = u < (double)tab.n ? (int)u : tab.n;
    if (i >= tab.n - 1) return 0.0;
    if (i > 0 || nu >= 1.0) {
      const double2 a = reinterpret_cast<const double2*>(tab.t64)[i];
      const double2 b = reinterpret_cast<const double2*>(tab.t64)[i + 1];
      return hermite(u - (double)i, a.x, a.y, b.x, b.y);
    }
  }
  const double s = sqrt(2.0 * nu) * r;
  if (s < 1e-12) return 1.0;
  if (s > 700.0) return 0.0;
  return matern_c * pow(s, nu) * bessel_k_nu_f64(s, nu);
}

__global__ __launch_bounds__(256) void gp_kmat_batch_f64_kernel(const double* __restrict__ X, int n, int d,
                                                                const double* __restrict__ inv_ls2, int nb,
                                                                double* __restrict__ K, int ld, int64_t bstride,
                                                                int kind, double nu, double matern_c, double diag,
                                                                MaternTab tab) {
  const int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x;   // packed lower-triangle index
  const int64_t total = (int64_t)n * (n + 1) / 2;
  if (p >= total) return;
  int i = (int)((sqrt(8.0 * (double)p + 1.0) - 1.0) * 0.5);
  while ((int64_t)i * (i + 1) / 2 > p) --i;
  while ((int64_t)(i + 1) * (i + 2) / 2 <= p) ++i;
  const int j = (int)(p - (int64_t)i * (i + 1) / 2);
  double sq = 0.0;
  for (int k = 0; k < d; ++k) {
    const double t = X[(int64_t)i * d + k] - X[(int64_t)j * d + k];
    sq = fma(t, t, sq);
  }
  for (int b = 0; b < nb; ++b) {
    double v = kernel_from_sq_f64(sq * inv_ls2[b], kind, nu, matern_c, tab);
    if (i == j) v += diag;
    double* Kb = K + (int64_t)b * bstride;
    Kb[(int64_t)i * ld + j] = v;
    Kb[(int64_t)j * ld + i] = v;
  }
}

// ------------------------------------------------------------------------------------------ cholesky
constexpr int CHOL_MAX = 128;

// In-place lower Cholesky of K (n x n, row-major fp32 in HBM, fp64 in LDS). status[0] = 0 ok, else the
// 1-based column where the pivot was not positive (caller adds jitter and retries).
__global__ __launch_bounds__(1024) void gp_chol_kernel(float* __restrict__ K, int n, int ldk, int* __restrict__ status) {
  __shared__ double S[CHOL_MAX * CHOL_MAX];
  __shared__ int bad;
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) S[e] = (double)K[(int64_t)(e / n) * ldk + (e % n)];
  if (threadIdx.x == 0) bad = 0;
  __syncthreads();
  for (int j = 0; j < n; ++j) {
    if (threadIdx.x == 0) {
      const double p = S[j * n + j];
      if (!(p > 0.0) && bad == 0) bad = j + 1;
      S[j * n + j] = p > 0.0 ? sqrt(p) : 1.0;
    }
    __syncthreads();
    const double piv = S[j * n + j];
    for (int i = j + 1 + threadIdx.x; i < n; i += blockDim.x) S[i * n + j] /= piv;
    __syncthreads();
    // trailing update of the lower triangle: S[i][k] -= S[i][j] * S[k][j], j < k <= i
    const int rem = n - j - 1;
    for (int e = threadIdx.x; e < rem * rem; e += blockDim.x) {
      const int i = j + 1 + e / rem, k = j + 1 + e % rem;
      if (k <= i) S[i * n + k] -= S[i * n + j] * S[k * n + j];
    }
    __syncthreads();
  }
  for (int e = threadIdx.x; e < n * n; e += blockDim.x) {
    const int i = e / n, k = e % n;
    K[(int64_t)i * ldk + k] = k <= i ? (float)S[e] : 0.0f;
  }
  if (threadIdx.x == 0) status[0] = bad;
}

// ------------------------------------------------------------------------------------------ predict + acq
enum Acq { kUCB = 0, kEI = 1, kPOI = 2, kMeanStd = 3 };

// Posterior of one candidate against n <= N training points staged in LDS (X row-major n x d, L lower n x N
// padded with the identity, alpha): k* (n kernel evals), mean = k*.alpha, v = L^-1 k* by forward substitution
// held in registers, sd = sqrt(kxx - |v|^2).  Every lane reads the same L entry: LDS broadcasts.
template <int N>
__device__ __forceinline__ void posterior_point(const float* xc, int n, int d, const float* sX, const float* sL,
                                                const float* sAlpha, int kind, float inv_ls2, float nu,
                                                float matern_c, float kxx, const MaternTab& tab, float& mean,
                                                float& sd) {
  float v[N];
  mean = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    float sq = 0.0f;
#pragma unroll
    for (int k = 0; k < 16; ++k) {
      if (k < d) {
        const float t = xc[k] - sX[i * d + k];
        sq = fmaf(t, t, sq);
      }
    }
    v[i] = i < n ? kernel_from_sq(sq, kind, inv_ls2, nu, matern_c, tab) : 0.0f;
    mean = fmaf(v[i], sAlpha[i], mean);
  }
  float q = 0.0f;
#pragma unroll
  for (int i = 0; i < N; ++i) {
    float s = v[i];
#pragma unroll
    for (int j = 0; j < i; ++j) s = fmaf(-sL[i * N + j], v[j], s);
    v[i] = s / sL[i * N + i];
    q = fmaf(v[i], v[i], q);
  }
  sd = sqrtf(fmaxf(kxx - q, 0.0f));
}

__device__ __forceinline__ float acq_value(float mean, float sd, int acq, float kappa, float xi, float y_max) {
  if (acq == kUCB) return mean + kappa * sd;
  const float imp = mean - y_max - xi;
  const float z = sd > 0.0f ? imp / sd : 0.0f;
  const float cdf = 0.5f * erfcf(-z * 0.7071067811865475f);
  if (acq == kPOI) return sd > 0.0f ? cdf : (imp > 0.0f ? 1.0f : 0.0f);
  const float pdf = 0.3989422804014327f * __expf(-0.5f * z * z);
  return sd > 0.0f ? imp * cdf + sd * pdf : fmaxf(imp, 0.0f);
}

template <int N>
__device__ __forceinline__ void stage_gp(const float* X, int n, int d, const float* L, int ldl, const float* alpha,
                                         float* sX, float* sL, float* sAlpha, int tid, int nthreads) {
  for (int e = tid; e < N * d; e += nthreads) sX[e] = (e / d) < n ? X[e] : 0.0f;
  for (int e = tid; e < N * N; e += nthreads) {
    const int i = e / N, j = e % N;
    sL[e] = (i < n && j < n) ? L[(int64_t)i * ldl + j] : (i == j ? 1.0f : 0.0f);
  }
  for (int e = tid; e < N; e += nthreads) sAlpha[e] = e < n ? alpha[e] : 0.0f;
}

template <int N>
__global__ __launch_bounds__(256) void gp_predict_acq_kernel(const float* __restrict__ Xc, int m, const float* __restrict__ X,
                                                             int n, int d, const float* __restrict__ L, int ldl,
                                                             const float* __restrict__ alpha, int kind, float inv_ls2,
                                                             float nu, float matern_c, float kxx, int acq, float kappa,
                                                             float xi, float y_max, float* __restrict__ out_acq,
                                                             float* __restrict__ out_mean, float* __restrict__ out_std,
                                                             float* __restrict__ blk_best, int* __restrict__ blk_idx,
                                                             MaternTab tab) {
  __shared__ float sX[N * 16];
  __shared__ float sL[N * N];
  __shared__ float sAlpha[N];
  __shared__ float redv[256];
  __shared__ int redi[256];
  stage_gp<N>(X, n, d, L, ldl, alpha, sX, sL, sAlpha, threadIdx.x, 256);
  __syncthreads();
  const int c = blockIdx.x * 256 + threadIdx.x;
  float best = -INFINITY;
  int best_i = -1;
  if (c < m) {
    float xc[16];
#pragma unroll
    for (int k = 0; k < 16; ++k) xc[k] = k < d ? Xc[(int64_t)c * d + k] : 0.0f;
    float mean, sd;
    posterior_point<N>(xc, n, d, sX, sL, sAlpha, kind, inv_ls2, nu, matern_c, kxx, tab, mean, sd);
    const float a = acq_value(mean, sd, acq, kappa, xi, y_max);
    if (out_acq) out_acq[c] = a;
    if (out_mean) out_mean[c] = mean;
    if (out_std) out_std[c] = sd;
    best = a;
    best_i = c;
  }
  redv[threadIdx.x] = best;
  redi[threadIdx.x] = best_i;
  __syncthreads();
  for (int s = 128; s > 0; s >>= 1) {
    if (threadIdx.x < s) {
      const float o = redv[threadIdx.x + s];
      const int oi = redi[threadIdx.x + s];
      if (o > redv[threadIdx.x] || (o == redv[threadIdx.x] && oi >= 0 && (redi[threadIdx.x] < 0 || oi < redi[threadIdx.x]))) {
        redv[threadIdx.x] = o;
        redi[threadIdx.x] = oi;
      }
    }
    __syncthreads();
  }
  if (threadIdx.x == 0 && blk_best) {
    blk_best[blockIdx.x] = redv[0];
    blk_idx[blockIdx.x] = redi[0];
  }
}

// Multi-start finite-difference ascent on the acquisition (the reference's L-BFGS-B restarts, all seeds at
// once): one wave per seed runs every step inside the kernel.  Per step lanes 0..2d-1 evaluate the clamped
// probes x +- h e_j, lane 0 forms the normalised gradient step, evaluates the candidate and accepts it
// (step x1.2) or rejects it (step x0.5).  Replaces ~30 small launches per step of the torch version.
template <int N>
__global__ __launch_bounds__(64) void gp_ascent_kernel(float* __restrict__ xs, float* __restrict__ fx,
                                                       const float* __restrict__ lo, const float* __restrict__ hi,
                                                       const float* __restrict__ X, int n, int d,
                                                       const float* __restrict__ L, const float* __restrict__ alpha,
                                                       int kind, float inv_ls2, float nu, float matern_c, float kxx,
                                                       int acq, float kappa, float xi, float y_max, int steps,
                                                       MaternTab tab) {
  __shared__ float sX[N * 16];
  __shared__ float sL[N * N];
  __shared__ float sAlpha[N];
  __shared__ float x[16], stp[16], wd[16], lo_s[16], hi_s[16], fp[32];
  __shared__ float fcur;
  const int lane = threadIdx.x, seed = blockIdx.x;
  stage_gp<N>(X, n, d, L, n, alpha, sX, sL, sAlpha, lane, 64);
  if (lane < 16) {
    const float l = lane < d ? lo[lane] : 0.0f, h = lane < d ? hi[lane] : 0.0f;
    lo_s[lane] = l;
    hi_s[lane] = h;
    wd[lane] = fmaxf(h - l, 1e-12f);
    stp[lane] = 0.05f * fmaxf(h - l, 1e-12f);
    x[lane] = lane < d ? xs[(int64_t)seed * d + lane] : 0.0f;
  }
  __syncthreads();
  float p[16];
  float mean, sd;
  if (lane == 0) {
#pragma unroll
    for (int k = 0; k < 16; ++k) p[k] = x[k];
    posterior_point<N>(p, n, d, sX, sL, sAlpha, kind, inv_ls2, nu, matern_c, kxx, tab, mean, sd);
    fcur = acq_value(mean, sd, acq, kappa, xi, y_max);
  }
  __syncthreads();
  for (int it = 0; it < steps; ++it) {
    if (lane < 2 * d) {
      const int j = lane < d ? lane : lane - d;
      const float sgn = lane < d ? 1.0f : -1.0f;
#pragma unroll
      for (int k = 0; k < 16; ++k) p[k] = x[k];
#pragma unroll
      for (int k = 0; k < 16; ++k)
        if (k == j) p[k] = fminf(fmaxf(x[k] + sgn * 1e-4f * wd[k], lo_s[k]), hi_s[k]);
      posterior_point<N>(p, n, d, sX, sL, sAlpha, kind, inv_ls2, nu, matern_c, kxx, tab, mean, sd);
      fp[lane] = acq_value(mean, sd, acq, kappa, xi, y_max);
    }
    __syncthreads();
    if (lane == 0) {
      float g[16];
      float gn = 0.0f;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        g[k] = k < d ? (fp[k] - fp[d + k]) / (2e-4f * wd[k]) : 0.0f;
        gn = fmaf(g[k] / wd[k], g[k] / wd[k], gn);
      }
      gn = fmaxf(sqrtf(gn), 1e-30f);
#pragma unroll
      for (int k = 0; k < 16; ++k) p[k] = k < d ? fminf(fmaxf(x[k] + stp[k] * g[k] / gn, lo_s[k]), hi_s[k]) : 0.0f;
      posterior_point<N>(p, n, d, sX, sL, sAlpha, kind, inv_ls2, nu, matern_c, kxx, tab, mean, sd);
      const float fc = acq_value(mean, sd, acq, kappa, xi, y_max);
      const bool better = fc > fcur;
      if (better) fcur = fc;
#pragma unroll
      for (int k = 0; k < 16; ++k) {
        if (better) x[k] = p[k];
        stp[k] *= better ? 1.2f : 0.5f;
      }
    }
    __syncthreads();
  }
  if (lane < d) xs[(int64_t)seed * d + lane] = x[lane];
  if (lane == 0) fx[seed] = fcur;
}

// Node i of the Matern-nu table: r = i h, s = sqrt(2 nu) r, f = c s^nu K_nu(s) and, from
// d/ds [s^nu K_nu(s)] = -s^nu K_{nu-1}(s) (K_{nu-1} = K_{1-nu}), h f'(r) = -h c sqrt(2 nu) s^nu K_{nu-1}(s).
__global__ __launch_bounds__(256) void gp_matern_table_kernel(double nu, double matern_c, double h, int n,
                                                              double* __restrict__ t64, float* __restrict__ t32) {
  const int i = blockIdx.x * 256 + threadIdx.x;
  if (i >= n) return;
  const double sn = sqrt(2.0 * nu);
  const double s = sn * h * i;
  double f = 1.0, d = 0.0;
  if (s > 1e-12) {
    const double p = matern_c * pow(s, nu);
    f = p * bessel_k_nu_f64(s, nu);
    d = -h * sn * p * bessel_k_nu_f64(s, fabs(nu - 1.0));
  }
  t64[2 * i] = f;
  t64[2 * i + 1] = d;
  t32[2 * i] = (float)f;
  t32[2 * i + 1] = (float)d;
}

}  // namespace

// Matern-nu lookup table (n nodes over [0, rmax]): t64 = double[2n], t32 = float[2n].
PLX_API int plx_gp_matern_table(double nu, double matern_c, double rmax, int n, double* t64, float* t32,
                                hipStream_t stream) {
  if (n < 2 || !(rmax > 0.0) || !(nu > 0.0)) return 1;
  hipLaunchKernelGGL(gp_matern_table_kernel, dim3((n + 255) / 256), dim3(256), 0, stream, nu, matern_c,
                     rmax / (n - 1), n, t64, t32);
  return (int)hipGetLastError();
}

static MaternTab make_tab(const double* t64, const float* t32, double rmax, int ntab) {
  MaternTab t{t64, t32, ntab > 1 ? (ntab - 1) / rmax : 0.0, ntab};
  if (ntab < 2) t.t64 = nullptr, t.t32 = nullptr;
  return t;
}

PLX_API int plx_gp_kmat(const float* A, const float* B, int n, int m, int d, float* K, int ldk, int kind,
                        float length_scale, float nu, float matern_c, int add_diag, float diag, const double* t64,
                        const float* t32, double rmax, int ntab, hipStream_t stream) {
  if (d > KMAX_D || n <= 0 || m <= 0 || d <= 0) return 1;
  const float inv_ls2 = 1.0f / (length_scale * length_scale);
  dim3 grid((m + KB - 1) / KB, (n + KB - 1) / KB);
  hipLaunchKernelGGL(gp_kmat_kernel, grid, dim3(256), 0, stream, A, B, n, m, d, K, ldk, kind, inv_ls2, nu, matern_c,
                     add_diag, diag, make_tab(t64, t32, rmax, ntab));
  return (int)hipGetLastError();
}

// K: fp64, entry b at K + b * bstride, row-major with leading dimension ld (>= n; rows past n are left for
// plx_gp_chol_aug_f64's appended right-hand sides); inv_ls2: device fp64 [nb] (1 / length_scale^2 per entry)
PLX_API int plx_gp_kmat_batch_f64(const double* X, int n, int d, const double* inv_ls2, int nb, double* K, int ld,
                                  long long bstride, int kind, double nu, double matern_c, double diag,
                                  const double* t64, const float* t32, double rmax, int ntab, hipStream_t stream) {
  if (n <= 0 || d <= 0 || nb <= 0 || ld < n || bstride < (long long)n * ld) return 1;
  const int64_t total = (int64_t)n * (n + 1) / 2;
  hipLaunchKernelGGL(gp_kmat_batch_f64_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, stream, X, n, d,
                     inv_ls2, nb, K, ld, (int64_t)bstride, kind, nu, matern_c, diag,
                     make_tab(t64, t32, rmax, ntab));
  return (int)hipGetLastError();
}

PLX_API int plx_gp_chol(float* K, int n, int ldk, int* status, hipStream_t stream) {
  if (n <= 0 || n > CHOL_MAX) return 1;
  hipLaunchKernelGGL(gp_chol_kernel, dim3(1), dim3(1024), 0, stream, K, n, ldk, status);
  return (int)hipGetLastError();
}

PLX_API int plx_gp_predict_acq(const float* Xc, int m, const float* X, int n, int d, const float* L, int ldl,
                               const float* alpha, int kind, float length_scale, float nu, float matern_c, float kxx,
                               int acq, float kappa, float xi, float y_max, float* out_acq, float* out_mean,
                               float* out_std, float* blk_best, int* blk_idx, const double* t64, const float* t32,
                               double rmax, int ntab, hipStream_t stream) {
  if (d > 16 || n <= 0 || m <= 0) return 1;
  const float inv_ls2 = 1.0f / (length_scale * length_scale);
  dim3 grid((m + 255) / 256);
#define PLX_LAUNCH(NN)                                                                                              \
  hipLaunchKernelGGL(gp_predict_acq_kernel<NN>, grid, dim3(256), 0, stream, Xc, m, X, n, d, L, ldl, alpha, kind,    \
                     inv_ls2, nu, matern_c, kxx, acq, kappa, xi, y_max, out_acq, out_mean, out_std, blk_best, blk_idx,  \
                     make_tab(t64, t32, rmax, ntab))
  if (n <= 16)
    PLX_LAUNCH(16);
  else if (n <= 32)
    PLX_LAUNCH(32);
  else if (n <= 64)
    PLX_LAUNCH(64);
  else
    return 2;  // larger training sets take the kmat + TRSM path on the host side
#undef PLX_LAUNCH
  return (int)hipGetLastError();
}

// In-place ascent of k seeds (xs: k x d fp32) under the fused posterior (n <= 64, d <= 16); fx[k] receives the
// final acquisition values.  lo / hi: device fp32 [d] bounds.
PLX_API int plx_gp_ascent(float* xs, float* fx, int k, const float* lo, const float* hi, const float* X, int n, int d,
                          const float* L, const float* alpha, int kind, float length_scale, float nu, float matern_c,
                          float kxx, int acq, float kappa, float xi, float y_max, int steps, const double* t64,
                          const float* t32, double rmax, int ntab, hipStream_t stream) {
  if (d > 16 || n <= 0 || k <= 0 || steps < 0) return 1;
  const float inv_ls2 = 1.0f / (length_scale * length_scale);
  const MaternTab tab = make_tab(t64, t32, rmax, ntab);
#define PLX_LAUNCH(NN)                                                                                              \
  hipLaunchKernelGGL(gp_ascent_kernel<NN>, dim3(k), dim3(64), 0, stream, xs, fx, lo, hi, X, n, d, L, alpha, kind,   \
                     inv_ls2, nu, matern_c, kxx, acq, kappa, xi, y_max, steps, tab)
  if (n <= 16)
    PLX_LAUNCH(16);
  else if (n <= 32)
    PLX_LAUNCH(32);
  else if (n <= 64)
    PLX_LAUNCH(64);
  else
    return 2;
#undef PLX_LAUNCH
  return (int)hipGetLastError();
}
