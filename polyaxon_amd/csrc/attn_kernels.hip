// Flash attention for MI355X (gfx950): causal / full, GQA, bf16 in/out, fp32 accumulation, head_dim 64 or 128.
//
// Replaces scaled_dot_product_attention (AOTriton on ROCm) on the language-model path (models/transformer.py).
// Three kernels, all 4 waves (256 threads) per workgroup, all on v_mfma_f32_32x32x16_bf16:
//
//   attn_fwd_kernel      128 queries / workgroup (32 per wave).  Scores are computed TRANSPOSED, S^T = K.Q^T,
//                        so each lane owns one query column: the online-softmax row max / row sum are lane-local
//                        plus one cross-half shuffle, and the probability tile P^T in the accumulator registers is
//                        directly the B operand of O^T += V^T . P^T (cdna_hip_programming.md §3 "accumulator tile
//                        as the next MFMA's operand") -- P never touches LDS.  V^T fragments come from
//                        ds_read_b64_tr_b16 transposed reads of the row-major V tile (T10).
//   attn_bwd_dq_kernel   same orientation: S^T, dP^T = V.dO^T, dS^T = P^T*(dP^T - delta), dQ^T += K^T . dS^T.
//   attn_bwd_dkdv_kernel 128 keys / workgroup (32 per wave), sweeping every query head of its GQA group and every
//                        query tile: S = Q.K^T, dP = dO.V^T (query rows in registers: the log-sum-exp and delta of
//                        each row are per-register constants, no reductions), dV += P^T.dO and dK += dS^T.Q with
//                        P / dS as the A operand straight from the accumulators, so dK/dV are complete in one
//                        workgroup (no atomics, no cross-workgroup sums).
//
// Tiles are staged global -> LDS with 16-byte global_load_lds into lane-linear images; one XOR swizzle per image
// (swz<D>) keeps both the ds_read_b128 row reads (the 4 non-contiguous 16-lane groups of gfx950, MI355X_MICROARCH
// §LDS) and the 4-row transposed reads conflict-free; the swizzle goes on the per-lane SOURCE address (rule 21).
// Rows past the sequence end read a zero page; their scores are masked to -inf.  Softmax runs in the log2 domain
// (c = softmax_scale * log2 e); the forward writes lse2 = m + log2(l) per query for the backward.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include <algorithm>

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

constexpr int NT = 256;
constexpr float NEG_INF = -__builtin_huge_valf();

struct Strides {
  long long b, h, s;  // element strides of batch, head, sequence (head_dim is contiguous)
};

struct AttnArgs {
  const __bf16 *q, *k, *v, *o, *dout;
  __bf16 *out, *dq, *dk, *dv;
  float *lse2, *delta;  // [B][H][S]
  Strides sq, sk, sv, so, sdo, sdq, sdk, sdv;
  int B, H, Hkv, S, Skv, causal;
  float c;      // softmax_scale * log2(e)
  float scale;  // softmax_scale
  const __bf16* zero;  // >= 16 zero bytes
};

template <int D>
__device__ __forceinline__ int swz(int row) {
  if constexpr (D == 128) return ((row & 3) << 2) | ((row >> 2) & 3);
  else return (((row >> 1) & 1) << 2) | ((row >> 2) & 3);
}

// Stage R rows x D of a row-major tile (row stride ld elements, rows >= nvalid -> zero page) into a lane-linear
// LDS image: wave instruction i writes bytes [1024 i, 1024 i + 1024) = rows of 2D bytes, physical 16-B chunk
// p of row r holds logical chunk p ^ swz(r).
template <int D, int R, int NW = 4>
__device__ __forceinline__ void stage_tile(char* img, const __bf16* g, long long ld, int nvalid,
                                           const __bf16* zero, int wave, int lane) {
  constexpr int ROWB = 2 * D;
  constexpr int INSTR = R * ROWB / 1024;
  static_assert(INSTR % NW == 0, "tile must split evenly over the waves");
#pragma unroll
  for (int i = 0; i < INSTR / NW; ++i) {
    const int off = (i * NW + wave) * 1024 + lane * 16;
    const int row = off / ROWB, pc = (off % ROWB) >> 4;
    const int lc = pc ^ swz<D>(row);
    const __bf16* src = row < nvalid ? g + (long long)row * ld + lc * 8 : zero;
    __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(img + (i * NW + wave) * 1024), 16, 0, 0);
  }
}

// 8 consecutive head-dim elements (logical chunk) of one row: ds_read_b128
template <int D>
__device__ __forceinline__ bf16x8 row_frag(const char* img, int row, int chunk) {
  return *(const bf16x8*)(img + row * (2 * D) + ((chunk ^ swz<D>(row)) << 4));
}

template <int D>
__device__ __forceinline__ s16x4 tr4(const char* img, int row, int col) {
  const int chunk = col >> 3, half = (col >> 2) & 1;
  return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
      (__attribute__((address_space(3))) s16x4*)(img + row * (2 * D) + ((chunk ^ swz<D>(row)) << 4) + half * 8));
}

// A (or B) fragment of the transpose of an image, in the k order of an accumulator tile used as the other operand:
// lane l, element j = img[r0 + 8(j>>2) + 4h + (j&3)][c0 + (l & 31)]   (h = l >> 5)
template <int D>
__device__ __forceinline__ bf16x8 tr_frag(const char* img, int r0, int c0, int lane) {
  const int h = lane >> 5, g1 = (lane >> 4) & 1, i = lane & 15;
  const int row = r0 + 4 * h + (i >> 2);
  const int col = c0 + 16 * g1 + 4 * (i & 3);
  const s16x4 a = tr4<D>(img, row, col), b = tr4<D>(img, row + 8, col);
  typedef short s16x8 __attribute__((ext_vector_type(8)));
  const s16x8 r = {a[0], a[1], a[2], a[3], b[0], b[1], b[2], b[3]};
  return __builtin_bit_cast(bf16x8, r);
}

// registers 8s .. 8s+7 of an accumulator tile as a bf16 MFMA operand (k-step s of the tile's row index)
__device__ __forceinline__ bf16x8 acc_frag(const f32x16& x, int s) {
  bf16x8 r;
#pragma unroll
  for (int j = 0; j < 8; ++j) r[j] = (__bf16)x[8 * s + j];
  return r;
}

__device__ __forceinline__ f32x16 mfma(const bf16x8& a, const bf16x8& b, const f32x16& c) {
  return __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, c, 0, 0, 0);
}

__device__ __forceinline__ f32x16 zero16() {
  f32x16 z;
#pragma unroll
  for (int i = 0; i < 16; ++i) z[i] = 0.f;
  return z;
}

// row of a 32x32 accumulator register r held by lane half h (column = lane & 31)
__device__ __forceinline__ int acc_row(int r, int h) { return (r & 3) + 8 * (r >> 2) + 4 * h; }

__device__ __forceinline__ uint2 pack4(float a, float b, float c, float d) {
  auto bits = [](float f) -> uint32_t {  // hardware RNE conversion (v_cvt_pk_bf16_f32)
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)f);
  };
  return make_uint2(bits(a) | (bits(b) << 16), bits(c) | (bits(d) << 16));
}

// Store a transposed accumulator set X^T[d][query] (rows = head dim, column = this lane's query) as the query's
// output row: registers 4g..4g+3 of tile dt are d = 32 dt + 8 g + 4 h + 0..3.
template <int D>
__device__ __forceinline__ void store_row(__bf16* row, const f32x16 (&acc)[D / 32], float mul, int h) {
#pragma unroll
  for (int dt = 0; dt < D / 32; ++dt)
#pragma unroll
    for (int g = 0; g < 4; ++g) {
      const int d = 32 * dt + 8 * g + 4 * h;
      *(uint2*)(row + d) = pack4(acc[dt][4 * g] * mul, acc[dt][4 * g + 1] * mul, acc[dt][4 * g + 2] * mul,
                                 acc[dt][4 * g + 3] * mul);
    }
}

struct QBlock {
  int b, hq, hk, q0;
};

// Query block of this workgroup (QB rows).  Heaviest-first over the WHOLE grid: block id i covers q-block index
// nqb - 1 - i / (B*H) of head i % (B*H), so under the causal mask the longest key ranges of every head are
// dispatched first and the short ones fill the tail (a per-head order still put heavy blocks of late heads last).
template <int QB>
__device__ __forceinline__ QBlock q_block(const AttnArgs& a) {
  const int nqb = (a.S + QB - 1) / QB;
  const int bhn = a.B * a.H;
  const int bid = blockIdx.x;
  QBlock r;
  r.q0 = (nqb - 1 - bid / bhn) * QB;
  const int bh = bid % bhn;
  r.b = bh / a.H;
  r.hq = bh % a.H;
  r.hk = r.hq / (a.H / a.Hkv);
  return r;
}

// raw v_exp_f32 (2^x): the libm exp2f adds a denormal range fix-up (compare, two selects, ldexp) per call; softmax
// arguments are <= RESCALE_TH and anything below 2^-126 may flush to zero
__device__ __forceinline__ float fast_exp2(float x) { return __builtin_amdgcn_exp2f(x); }

// Deferred rescale (lazy max): the running max m of a query row only moves when a tile's max exceeds it by more than
// RESCALE_TH (log2 units), so O and l are rescaled on a few tiles instead of every tile; probabilities stay
// <= 2^RESCALE_TH (fp32 sums and bf16 P are exact enough there), and o / l always see the same reference max.
constexpr float RESCALE_TH = 8.f;

// ------------------------------------------------------------------------------------------------ forward
// NW waves x 32 queries per workgroup: one K/V tile in LDS feeds NW * 32 queries (8 waves halve the per-CU LDS-DMA
// fill of the 4-wave form, which at the MFMA-bound rate needed ~77 GB/s per CU, above what LDS-DMA sustains).
template <int D, int NW>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void attn_fwd_kernel(AttnArgs a) {
  constexpr int QB = 32 * NW, TB = 64 * 2 * D, STAGE = 2 * TB, ND = D / 32, NS = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, ql = lane & 31;
  const QBlock blk = q_block<QB>(a);
  const int q0w = blk.q0 + 32 * wave, qi = q0w + ql;
  const __bf16* Q = a.q + blk.b * a.sq.b + blk.hq * a.sq.h;
  const __bf16* K = a.k + blk.b * a.sk.b + blk.hk * a.sk.h;
  const __bf16* V = a.v + blk.b * a.sv.b + blk.hk * a.sv.h;

  const int kv_end = a.causal ? min(a.Skv, blk.q0 + QB) : a.Skv;
  const int nt = (kv_end + 63) / 64;
  stage_tile<D, 64, NW>(smem, K, a.sk.s, a.Skv, a.zero, wave, lane);
  stage_tile<D, 64, NW>(smem + TB, V, a.sv.s, a.Skv, a.zero, wave, lane);
  bf16x8 qf[NS];
  {
    const __bf16* qr = Q + (long long)min(qi, a.S - 1) * a.sq.s + 8 * h;
#pragma unroll
    for (int s = 0; s < NS; ++s) qf[s] = *(const bf16x8*)(qr + 16 * s);
  }
  f32x16 o[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) o[dt] = zero16();
  float m_run = NEG_INF, l_run = 0.f;
  const float c = a.c;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int j = 0; j < nt; ++j) {
    const int kv0 = j * 64;
    if (j + 1 < nt) {
      char* nb = smem + ((j + 1) & 1) * STAGE;
      stage_tile<D, 64, NW>(nb, K + (long long)(kv0 + 64) * a.sk.s, a.sk.s, a.Skv - kv0 - 64, a.zero, wave, lane);
      stage_tile<D, 64, NW>(nb + TB, V + (long long)(kv0 + 64) * a.sv.s, a.sv.s, a.Skv - kv0 - 64, a.zero, wave, lane);
    }
    const char* Ks = smem + (j & 1) * STAGE;
    const char* Vs = Ks + TB;
    if (!(a.causal && kv0 > q0w + 31)) {  // wave-uniform: tile entirely in this wave's causal future
      f32x16 st[2] = {zero16(), zero16()};
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        st[0] = mfma(row_frag<D>(Ks, ql, 2 * s + h), qf[s], st[0]);
        st[1] = mfma(row_frag<D>(Ks, 32 + ql, 2 * s + h), qf[s], st[1]);
      }
      if ((a.causal && kv0 + 63 > q0w) || kv0 + 64 > a.Skv) {  // diagonal / ragged tile: mask (raw scores)
#pragma unroll
        for (int t = 0; t < 2; ++t)
#pragma unroll
          for (int r = 0; r < 16; ++r) {
            const int key = kv0 + 32 * t + acc_row(r, h);
            if ((a.causal && key > qi) || key >= a.Skv) st[t][r] = NEG_INF;
          }
      }
      float mx = NEG_INF;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) mx = fmaxf(mx, st[t][r]);
      mx = fmaxf(mx, __shfl_xor(mx, 32)) * c;  // c > 0: max of the scaled scores
      const bool grow = mx > m_run + RESCALE_TH;
      if (__builtin_amdgcn_ballot_w64(grow)) {   // wave-uniform branch; lanes that do not grow keep alpha = 1
        const float m_new = grow ? mx : m_run;
        const float alpha = m_run == NEG_INF ? 0.f : fast_exp2(m_run - m_new);
        l_run *= alpha;
#pragma unroll
        for (int dt = 0; dt < ND; ++dt)
#pragma unroll
          for (int r = 0; r < 16; ++r) o[dt][r] *= alpha;
        m_run = m_new;
      }
      const float msub = m_run == NEG_INF ? 0.f : m_run;  // a fully masked row so far: p = 2^-inf = 0
      float sum = 0.f;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          const float p = fast_exp2(fmaf(st[t][r], c, -msub));
          st[t][r] = p;
          sum += p;
        }
      l_run += sum + __shfl_xor(sum, 32);
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 pb = acc_frag(st[t], s);
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) o[dt] = mfma(tr_frag<D>(Vs, 32 * t + 16 * s, 32 * dt, lane), pb, o[dt]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (qi < a.S) {
    const float inv = l_run > 0.f ? 1.f / l_run : 0.f;
    store_row<D>(a.out + blk.b * a.so.b + blk.hq * a.so.h + (long long)qi * a.so.s, o, inv, h);
    if (h == 0) a.lse2[((long long)blk.b * a.H + blk.hq) * a.S + qi] = m_run + log2f(l_run);
  }
}

// ---------------------------------------------------------------------------------------- backward: delta
// delta[b][h][q] = sum_d dO . O   (16 lanes per row, 8 elements each)
template <int D>
__global__ __launch_bounds__(NT) void attn_bwd_delta_kernel(AttnArgs a) {
  constexpr int LPR = D / 8;  // lanes per row
  const long long rows = (long long)a.B * a.H * a.S;
  const long long row = ((long long)blockIdx.x * NT + threadIdx.x) / LPR;
  const int part = threadIdx.x % LPR;
  float acc = 0.f;
  if (row < rows) {
    const int q = (int)(row % a.S);
    const long long bh = row / a.S;
    const int b = (int)(bh / a.H), hh = (int)(bh % a.H);
    const bf16x8 o = *(const bf16x8*)(a.o + b * a.so.b + hh * a.so.h + (long long)q * a.so.s + part * 8);
    const bf16x8 g = *(const bf16x8*)(a.dout + b * a.sdo.b + hh * a.sdo.h + (long long)q * a.sdo.s + part * 8);
#pragma unroll
    for (int j = 0; j < 8; ++j) acc += (float)o[j] * (float)g[j];
  }
#pragma unroll
  for (int off = LPR / 2; off > 0; off >>= 1) acc += __shfl_xor(acc, off);
  if (row < rows && part == 0) a.delta[row] = acc;
}

// ------------------------------------------------------------------------------------------- backward: dQ
// NW waves x 32 queries per workgroup: the K / V tile in LDS serves NW * 32 query rows (see the forward)
template <int D, int NW>
__global__ __launch_bounds__(64 * NW, NW == 4 ? 2 : 1) void attn_bwd_dq_kernel(AttnArgs a) {
  constexpr int QB = 32 * NW, TB = 64 * 2 * D, STAGE = 2 * TB, ND = D / 32, NS = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, ql = lane & 31;
  const QBlock blk = q_block<QB>(a);
  const int q0w = blk.q0 + 32 * wave, qi = q0w + ql, qc = min(qi, a.S - 1);
  const __bf16* K = a.k + blk.b * a.sk.b + blk.hk * a.sk.h;
  const __bf16* V = a.v + blk.b * a.sv.b + blk.hk * a.sv.h;
  const int kv_end = a.causal ? min(a.Skv, blk.q0 + QB) : a.Skv;
  const int nt = (kv_end + 63) / 64;
  stage_tile<D, 64, NW>(smem, K, a.sk.s, a.Skv, a.zero, wave, lane);
  stage_tile<D, 64, NW>(smem + TB, V, a.sv.s, a.Skv, a.zero, wave, lane);
  bf16x8 qf[NS], gf[NS];
  {
    const __bf16* qr = a.q + blk.b * a.sq.b + blk.hq * a.sq.h + (long long)qc * a.sq.s + 8 * h;
    const __bf16* gr = a.dout + blk.b * a.sdo.b + blk.hq * a.sdo.h + (long long)qc * a.sdo.s + 8 * h;
#pragma unroll
    for (int s = 0; s < NS; ++s) {
      qf[s] = *(const bf16x8*)(qr + 16 * s);
      gf[s] = *(const bf16x8*)(gr + 16 * s);
    }
  }
  const long long srow = ((long long)blk.b * a.H + blk.hq) * a.S + qc;
  const float lse2 = a.lse2[srow], dlt = a.delta[srow], c = a.c;
  f32x16 dq[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) dq[dt] = zero16();
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int j = 0; j < nt; ++j) {
    const int kv0 = j * 64;
    if (j + 1 < nt) {
      char* nb = smem + ((j + 1) & 1) * STAGE;
      stage_tile<D, 64, NW>(nb, K + (long long)(kv0 + 64) * a.sk.s, a.sk.s, a.Skv - kv0 - 64, a.zero, wave, lane);
      stage_tile<D, 64, NW>(nb + TB, V + (long long)(kv0 + 64) * a.sv.s, a.sv.s, a.Skv - kv0 - 64, a.zero, wave, lane);
    }
    const char* Ks = smem + (j & 1) * STAGE;
    const char* Vs = Ks + TB;
    if (!(a.causal && kv0 > q0w + 31)) {
      f32x16 st[2] = {zero16(), zero16()}, dp[2] = {zero16(), zero16()};
#pragma unroll
      for (int s = 0; s < NS; ++s)
#pragma unroll
        for (int t = 0; t < 2; ++t) {
          st[t] = mfma(row_frag<D>(Ks, 32 * t + ql, 2 * s + h), qf[s], st[t]);
          dp[t] = mfma(row_frag<D>(Vs, 32 * t + ql, 2 * s + h), gf[s], dp[t]);
        }
      const bool mask = (a.causal && kv0 + 63 > q0w) || kv0 + 64 > a.Skv || qi >= a.S;
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int r = 0; r < 16; ++r) {
          float p = fast_exp2(fmaf(st[t][r], c, -lse2));
          if (mask) {
            const int key = kv0 + 32 * t + acc_row(r, h);
            if ((a.causal && key > qi) || key >= a.Skv || qi >= a.S) p = 0.f;
          }
          st[t][r] = p * (dp[t][r] - dlt);  // dS^T (softmax_scale applied at the end)
        }
#pragma unroll
      for (int t = 0; t < 2; ++t)
#pragma unroll
        for (int s = 0; s < 2; ++s) {
          const bf16x8 db = acc_frag(st[t], s);
#pragma unroll
          for (int dt = 0; dt < ND; ++dt) dq[dt] = mfma(tr_frag<D>(Ks, 32 * t + 16 * s, 32 * dt, lane), db, dq[dt]);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (qi < a.S) store_row<D>(a.dq + blk.b * a.sdq.b + blk.hq * a.sdq.h + (long long)qi * a.sdq.s, dq, a.scale, h);
}

// ---------------------------------------------------------------------------------------- backward: dK, dV
// One workgroup = 128 keys (32 per wave) x ONE query head: grid = B x H x key blocks, key block 0 (the longest
// causal query range) first, so the 4-8x causal spread of work per key block is balanced by the dispatcher over
// ~4 workgroups per CU instead of serialising a whole GQA group in one workgroup.  With GQA (G query heads per
// KV head) each workgroup writes its head's fp32 partial dK/dV to a workspace that attn_bwd_reduce_kernel sums
// over the G heads (plain stores, no atomics, deterministic); without GQA it writes bf16 dK/dV directly.
// Query tiles of 64 rows (two 32-row MFMA sub-tiles per stage, one barrier per 64 rows).
// LDS: K image [128][D] | V image [128][D] | 2 x { Q tile [64][D] | dO tile [64][D] | lse2[64] | delta[64] }
template <int D>
__global__ __launch_bounds__(NT, 1) void attn_bwd_dkdv_kernel(AttnArgs a, float* __restrict__ ws) {
  constexpr int KB = 128 * 2 * D, QTB = 64 * 2 * D, QSTAGE = 2 * QTB + 512, ND = D / 32, NS = D / 16;
  extern __shared__ __attribute__((aligned(16))) char smem[];
  char* Kimg = smem;
  char* Vimg = smem + KB;
  char* qbase = smem + 2 * KB;
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, kl = lane & 31;
  const int nkb = (a.Skv + 127) / 128;
  const int bid = blockIdx.x;
  const int kb = bid % nkb, bh = bid / nkb;
  const int b = bh / a.H, hq = bh % a.H, G = a.H / a.Hkv, hk = hq / G;
  const int k0 = kb * 128, kw0 = k0 + 32 * wave;
  const __bf16* K = a.k + b * a.sk.b + hk * a.sk.h + (long long)k0 * a.sk.s;
  const __bf16* V = a.v + b * a.sv.b + hk * a.sv.h + (long long)k0 * a.sv.s;
  const __bf16* Qh = a.q + b * a.sq.b + hq * a.sq.h;
  const __bf16* Gh = a.dout + b * a.sdo.b + hq * a.sdo.h;
  const long long srow0 = ((long long)b * a.H + hq) * a.S;
  stage_tile<D, 128>(Kimg, K, a.sk.s, a.Skv - k0, a.zero, wave, lane);
  stage_tile<D, 128>(Vimg, V, a.sv.s, a.Skv - k0, a.zero, wave, lane);

  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    dk[dt] = zero16();
    dv[dt] = zero16();
  }
  const int qt0 = a.causal ? k0 / 64 : 0;
  const int total = (a.S + 63) / 64 - qt0;
  auto stage_q = [&](int buf, int it) {
    const int q0 = (qt0 + it) * 64;
    char* base = qbase + buf * QSTAGE;
    stage_tile<D, 64>(base, Qh + (long long)q0 * a.sq.s, a.sq.s, a.S - q0, a.zero, wave, lane);
    stage_tile<D, 64>(base + QTB, Gh + (long long)q0 * a.sdo.s, a.sdo.s, a.S - q0, a.zero, wave, lane);
    if (wave < 2) {  // lse2[64] | delta[64]: one 4-byte LDS-DMA per lane (rows past S: clamp, masked later)
      const long long srow = srow0 + min(q0 + lane, a.S - 1);
      const float* src = wave == 0 ? a.lse2 + srow : a.delta + srow;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(base + 2 * QTB + 256 * wave), 4, 0, 0);
    }
  };
  if (total > 0) stage_q(0, 0);
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  const int key = kw0 + kl;
  // this wave's 32 keys are fixed for the whole sweep: their K / V row fragments live in registers (the one-wave-per-
  // SIMD budget has the room), which takes 2 of the 4 ds_read_b128 streams out of every S / dP step
  bf16x8 kf[NS], vf[NS];
#pragma unroll
  for (int s = 0; s < NS; ++s) {
    kf[s] = row_frag<D>(Kimg, 32 * wave + kl, 2 * s + h);
    vf[s] = row_frag<D>(Vimg, 32 * wave + kl, 2 * s + h);
  }
  for (int it = 0; it < total; ++it) {
    if (it + 1 < total) stage_q((it + 1) & 1, it + 1);
    const char* Qs = qbase + (it & 1) * QSTAGE;
    const char* Gs = Qs + QTB;
    const float* st_lse = (const float*)(Qs + 2 * QTB);
    const float* st_dlt = st_lse + 64;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int q0 = (qt0 + it) * 64 + 32 * sub;
      if (a.causal && q0 + 31 < kw0) continue;  // wave-uniform: every query precedes this wave's keys
      f32x16 s_acc = zero16(), dp = zero16();
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        s_acc = mfma(row_frag<D>(Qs, 32 * sub + kl, 2 * s + h), kf[s], s_acc);  // S[q][key]
        dp = mfma(row_frag<D>(Gs, 32 * sub + kl, 2 * s + h), vf[s], dp);         // dP[q][key]
      }
      const bool mask = (a.causal && kw0 + 31 > q0) || q0 + 32 > a.S || kw0 + 32 > a.Skv;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *(const float4*)(st_lse + 32 * sub + 8 * g + 4 * h);
        const float4 d4 = *(const float4*)(st_dlt + 32 * sub + 8 * g + 4 * h);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          float p = fast_exp2(fmaf(s_acc[r], a.c, -lv[e]));
          if (mask) {
            const int q = q0 + 8 * g + 4 * h + e;
            if ((a.causal && key > q) || q >= a.S || key >= a.Skv) p = 0.f;
          }
          s_acc[r] = p;
          dp[r] = p * (dp[r] - dv4[e]);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pa = acc_frag(s_acc, s), da = acc_frag(dp, s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          dv[dt] = mfma(pa, tr_frag<D>(Gs, 32 * sub + 16 * s, 32 * dt, lane), dv[dt]);
          dk[dt] = mfma(da, tr_frag<D>(Qs, 32 * sub + 16 * s, 32 * dt, lane), dk[dt]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (G > 1) {
    // fp32 partials of this query head: ws[{dk, dv}][b][hq][key][d]; rows = keys (registers), column = d (lane)
    const long long plane = (long long)a.B * a.H * a.Skv * D;
    float* wk = ws + (((long long)b * a.H + hq) * a.Skv) * D;
    float* wv = wk + plane;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = kw0 + acc_row(r, h);
        if (kr < a.Skv) {
          wk[(long long)kr * D + 32 * dt + kl] = dk[dt][r] * a.scale;
          wv[(long long)kr * D + 32 * dt + kl] = dv[dt][r];
        }
      }
    return;
  }
  // no GQA: stage [128][D] bf16 through the K / V image regions, then write whole rows with 16-B stores
  __bf16* dks = (__bf16*)Kimg;
  __bf16* dvs = (__bf16*)Vimg;
#pragma unroll
  for (int dt = 0; dt < ND; ++dt)
#pragma unroll
    for (int r = 0; r < 16; ++r) {
      const int row = 32 * wave + acc_row(r, h), col = 32 * dt + kl;
      dks[row * D + col] = (__bf16)(dk[dt][r] * a.scale);
      dvs[row * D + col] = (__bf16)dv[dt][r];
    }
  __syncthreads();
  constexpr int CH = D / 8;  // 16-B chunks per row
  for (int i = threadIdx.x; i < 128 * CH; i += NT) {
    const int row = i / CH, ch = i % CH;
    if (k0 + row >= a.Skv) continue;
    *(uint4*)(a.dk + b * a.sdk.b + hk * a.sdk.h + (long long)(k0 + row) * a.sdk.s + ch * 8) =
        *(const uint4*)(dks + row * D + ch * 8);
    *(uint4*)(a.dv + b * a.sdv.b + hk * a.sdv.h + (long long)(k0 + row) * a.sdv.s + ch * 8) =
        *(const uint4*)(dvs + row * D + ch * 8);
  }
}

// 8-wave form: one workgroup = 256 keys (32 per wave) x one query head, so every Q / dO tile staged into LDS feeds
// 8 waves (half the LDS-DMA fill per FLOP of the 128-key form) at two waves per SIMD.  A wave's K / V row fragments
// come straight from global memory into registers (they are fixed for the whole sweep), so LDS holds only the
// double-buffered { Q tile [64][D] | dO tile [64][D] | lse2[64] | delta[64] } stages; the bf16 dK / dV rows (no GQA)
// are staged through that region one tensor at a time.
template <int D>
__global__ __launch_bounds__(512, 1) void attn_bwd_dkdv8_kernel(AttnArgs a, float* __restrict__ ws) {
  constexpr int NW = 8, KBLK = 32 * NW, QTB = 64 * 2 * D, QSTAGE = 2 * QTB + 512, ND = D / 32, NS = D / 16;
  extern __shared__ __attribute__((aligned(16))) char lds[];
  char* Vimg = lds;                                    // [256][D] V rows of this key block
  char* smem = lds + KBLK * 2 * D;                     // 2 Q / dO stages
  const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6, h = lane >> 5, kl = lane & 31;
  const int nkb = (a.Skv + KBLK - 1) / KBLK;
  const int bhn = a.B * a.H;
  const int bid = blockIdx.x;
  const int kb = bid / bhn, bh = bid % bhn;            // key block 0 (the longest causal query range) first
  const int b = bh / a.H, hq = bh % a.H, G = a.H / a.Hkv, hk = hq / G;
  const int k0 = kb * KBLK, kw0 = k0 + 32 * wave;
  (void)nkb;
  const __bf16* Qh = a.q + b * a.sq.b + hq * a.sq.h;
  const __bf16* Gh = a.dout + b * a.sdo.b + hq * a.sdo.h;
  const long long srow0 = ((long long)b * a.H + hq) * a.S;
  const int qt0 = a.causal ? k0 / 64 : 0;
  const int total = (a.S + 63) / 64 - qt0;
  auto stage_q = [&](int buf, int it) {
    const int q0 = (qt0 + it) * 64;
    char* base = smem + buf * QSTAGE;
    stage_tile<D, 64, NW>(base, Qh + (long long)q0 * a.sq.s, a.sq.s, a.S - q0, a.zero, wave, lane);
    stage_tile<D, 64, NW>(base + QTB, Gh + (long long)q0 * a.sdo.s, a.sdo.s, a.S - q0, a.zero, wave, lane);
    if (wave < 2) {  // lse2[64] | delta[64]: one 4-byte LDS-DMA per lane (rows past S: clamp, masked later)
      const long long srow = srow0 + min(q0 + lane, a.S - 1);
      const float* src = wave == 0 ? a.lse2 + srow : a.delta + srow;
      __builtin_amdgcn_global_load_lds((gbl_void*)src, (lds_void*)(base + 2 * QTB + 256 * wave), 4, 0, 0);
    }
  };
  stage_tile<D, KBLK, NW>(Vimg, a.v + b * a.sv.b + hk * a.sv.h + (long long)k0 * a.sv.s, a.sv.s, a.Skv - k0, a.zero,
                          wave, lane);
  if (total > 0) stage_q(0, 0);
  const int key = kw0 + kl;
  bf16x8 kf[NS];
  {
    const int kr = min(key, a.Skv - 1);  // rows past Skv: any valid row, their scores are masked
    const __bf16* kp = a.k + b * a.sk.b + hk * a.sk.h + (long long)kr * a.sk.s + 8 * h;
#pragma unroll
    for (int s = 0; s < NS; ++s) kf[s] = *(const bf16x8*)(kp + 16 * s);
  }
  f32x16 dk[ND], dv[ND];
#pragma unroll
  for (int dt = 0; dt < ND; ++dt) {
    dk[dt] = zero16();
    dv[dt] = zero16();
  }
  const float c = a.c;
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  __syncthreads();
  for (int it = 0; it < total; ++it) {
    if (it + 1 < total) stage_q((it + 1) & 1, it + 1);
    const char* Qs = smem + (it & 1) * QSTAGE;
    const char* Gs = Qs + QTB;
    const float* st_lse = (const float*)(Qs + 2 * QTB);
    const float* st_dlt = st_lse + 64;
#pragma unroll
    for (int sub = 0; sub < 2; ++sub) {
      const int q0 = (qt0 + it) * 64 + 32 * sub;
      if (a.causal && q0 + 31 < kw0) continue;  // wave-uniform: every query precedes this wave's keys
      f32x16 s_acc = zero16(), dp = zero16();
#pragma unroll
      for (int s = 0; s < NS; ++s) {
        s_acc = mfma(row_frag<D>(Qs, 32 * sub + kl, 2 * s + h), kf[s], s_acc);  // S[q][key]
        dp = mfma(row_frag<D>(Gs, 32 * sub + kl, 2 * s + h), row_frag<D>(Vimg, 32 * wave + kl, 2 * s + h), dp);
      }
      const bool mask = (a.causal && kw0 + 31 > q0) || q0 + 32 > a.S || kw0 + 32 > a.Skv;
#pragma unroll
      for (int g = 0; g < 4; ++g) {
        const float4 l4 = *(const float4*)(st_lse + 32 * sub + 8 * g + 4 * h);
        const float4 d4 = *(const float4*)(st_dlt + 32 * sub + 8 * g + 4 * h);
        const float lv[4] = {l4.x, l4.y, l4.z, l4.w}, dv4[4] = {d4.x, d4.y, d4.z, d4.w};
#pragma unroll
        for (int e = 0; e < 4; ++e) {
          const int r = 4 * g + e;
          float p = fast_exp2(fmaf(s_acc[r], c, -lv[e]));
          if (mask) {
            const int q = q0 + 8 * g + 4 * h + e;
            if ((a.causal && key > q) || q >= a.S || key >= a.Skv) p = 0.f;
          }
          s_acc[r] = p;
          dp[r] = p * (dp[r] - dv4[e]);
        }
      }
#pragma unroll
      for (int s = 0; s < 2; ++s) {
        const bf16x8 pa = acc_frag(s_acc, s), da = acc_frag(dp, s);
#pragma unroll
        for (int dt = 0; dt < ND; ++dt) {
          dv[dt] = mfma(pa, tr_frag<D>(Gs, 32 * sub + 16 * s, 32 * dt, lane), dv[dt]);
          dk[dt] = mfma(da, tr_frag<D>(Qs, 32 * sub + 16 * s, 32 * dt, lane), dk[dt]);
        }
      }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
  }
  if (G > 1) {
    // fp32 partials of this query head: ws[{dk, dv}][b][hq][key][d]; rows = keys (registers), column = d (lane)
    const long long plane = (long long)a.B * a.H * a.Skv * D;
    float* wk = ws + (((long long)b * a.H + hq) * a.Skv) * D;
    float* wv = wk + plane;
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int kr = kw0 + acc_row(r, h);
        if (kr < a.Skv) {
          wk[(long long)kr * D + 32 * dt + kl] = dk[dt][r] * a.scale;
          wv[(long long)kr * D + 32 * dt + kl] = dv[dt][r];
        }
      }
    return;
  }
  // no GQA: stage [256][D] bf16 through the (now idle) Q/dO stage region, dK then dV, and write whole rows
  __bf16* st = (__bf16*)smem;
  constexpr int CH = D / 8;  // 16-B chunks per row
#pragma unroll
  for (int which = 0; which < 2; ++which) {
#pragma unroll
    for (int dt = 0; dt < ND; ++dt)
#pragma unroll
      for (int r = 0; r < 16; ++r) {
        const int row = 32 * wave + acc_row(r, h), col = 32 * dt + kl;
        st[row * D + col] = which == 0 ? (__bf16)(dk[dt][r] * a.scale) : (__bf16)dv[dt][r];
      }
    __syncthreads();
    __bf16* dst = which == 0 ? a.dk + b * a.sdk.b + hk * a.sdk.h : a.dv + b * a.sdv.b + hk * a.sdv.h;
    const long long ld = which == 0 ? a.sdk.s : a.sdv.s;
    for (int i = threadIdx.x; i < KBLK * CH; i += 64 * NW) {
      const int row = i / CH, ch = i % CH;
      if (k0 + row < a.Skv) *(uint4*)(dst + (long long)(k0 + row) * ld + ch * 8) = *(const uint4*)(st + row * D + ch * 8);
    }
    __syncthreads();
  }
}

// dK/dV[b][hk][key][:] = sum over the G query heads of the group of the fp32 partials -> bf16 (8 elements per thread)
template <int D>
__global__ __launch_bounds__(NT) void attn_bwd_reduce_kernel(AttnArgs a, const float* __restrict__ ws) {
  const int G = a.H / a.Hkv;
  const long long n8 = (long long)a.B * a.Hkv * a.Skv * (D / 8);
  const long long plane = (long long)a.B * a.H * a.Skv * D;
  for (long long i = (long long)blockIdx.x * NT + threadIdx.x; i < n8; i += (long long)gridDim.x * NT) {
    const int c8 = (int)(i % (D / 8));
    const long long row = i / (D / 8);
    const int key = (int)(row % a.Skv);
    const long long bh = row / a.Skv;
    const int b = (int)(bh / a.Hkv), hk = (int)(bh % a.Hkv);
#pragma unroll
    for (int which = 0; which < 2; ++which) {
      float acc[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
      for (int g = 0; g < G; ++g) {
        const float* src = ws + which * plane + (((long long)b * a.H + hk * G + g) * a.Skv + key) * D + c8 * 8;
        const float4 x = *(const float4*)src, y = *(const float4*)(src + 4);
        acc[0] += x.x; acc[1] += x.y; acc[2] += x.z; acc[3] += x.w;
        acc[4] += y.x; acc[5] += y.y; acc[6] += y.z; acc[7] += y.w;
      }
      const uint2 lo = pack4(acc[0], acc[1], acc[2], acc[3]), hi = pack4(acc[4], acc[5], acc[6], acc[7]);
      __bf16* dst = which == 0 ? a.dk + b * a.sdk.b + hk * a.sdk.h + (long long)key * a.sdk.s
                               : a.dv + b * a.sdv.b + hk * a.sdv.h + (long long)key * a.sdv.s;
      *(uint4*)(dst + c8 * 8) = make_uint4(lo.x, lo.y, hi.x, hi.y);
    }
  }
}

template <typename Kern>
int prepare(Kern k, int bytes) {
  return hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0 : 3;
}

bool args_ok(const AttnArgs& a, int D) {
  if (a.B <= 0 || a.H <= 0 || a.Hkv <= 0 || a.S <= 0 || a.Skv <= 0 || a.H % a.Hkv) return false;
  if (D != 64 && D != 128) return false;
  // 16-B aligned rows (vector loads / LDS-DMA of 8 bf16 per lane)
  const long long strides[] = {a.sq.s, a.sk.s, a.sv.s, a.sq.h, a.sk.h, a.sv.h, a.sq.b, a.sk.b, a.sv.b};
  for (long long s : strides)
    if (s % 8) return false;
  return true;
}

}  // namespace

// forward waves per workgroup (A/B knob plx_attn_set_fwd_waves: 4 or 8)
int g_fwd_waves = 8;

template <int D, int NW>
int launch_fwd(const AttnArgs& a, hipStream_t stream) {
  constexpr int LDS = 4 * 64 * 2 * D;  // 2 stages x {K, V} x 64 rows
  static int once = prepare(attn_fwd_kernel<D, NW>, LDS);
  if (once) return once;
  const int grid = ((a.S + 32 * NW - 1) / (32 * NW)) * a.H * a.B;
  hipLaunchKernelGGL((attn_fwd_kernel<D, NW>), dim3(grid), dim3(64 * NW), LDS, stream, a);
  return (int)hipGetLastError();
}

PLX_API void plx_attn_set_fwd_waves(int nw) { g_fwd_waves = nw == 4 ? 4 : 8; }
PLX_API void plx_attn_set_dq_waves(int nw);

PLX_API int plx_attn_fwd(const AttnArgs* args, int D, hipStream_t stream) {
  const AttnArgs& a = *args;
  if (!args_ok(a, D)) return 1;
  if (a.so.s % 4 || a.so.h % 4 || a.so.b % 4) return 1;
  if (D == 128) return g_fwd_waves == 4 ? launch_fwd<128, 4>(a, stream) : launch_fwd<128, 8>(a, stream);
  return g_fwd_waves == 4 ? launch_fwd<64, 4>(a, stream) : launch_fwd<64, 8>(a, stream);
}

PLX_API long long plx_attn_bwd_workspace(int B, int H, int Hkv, int Skv, int D) {
  // fp32 partial dK and dV per query head when the heads are grouped (GQA); none otherwise
  return H == Hkv ? 0 : 2LL * B * H * Skv * D * (long long)sizeof(float);
}

// dQ / dK-dV waves per workgroup (A/B knobs plx_attn_set_dq_waves / plx_attn_set_dkdv_waves: 4 or 8)
int g_dq_waves = 8, g_dkdv_waves = 8;

template <int D>
int launch_bwd(const AttnArgs& a, float* ws, hipStream_t stream) {
  constexpr int QLDS = 4 * 64 * 2 * D, KLDS = 2 * 128 * 2 * D + 2 * (2 * 64 * 2 * D + 512);
  constexpr int KLDS8 = 256 * 2 * D + 2 * (2 * 64 * 2 * D + 512);
  static_assert(KLDS8 - 256 * 2 * D >= 256 * D * 2, "the dK / dV output staging must fit the stage region");
  static int once = prepare(attn_bwd_dq_kernel<D, 4>, QLDS) | prepare(attn_bwd_dq_kernel<D, 8>, QLDS) |
                    prepare(attn_bwd_dkdv_kernel<D>, KLDS) | prepare(attn_bwd_dkdv8_kernel<D>, KLDS8);
  if (once) return once;
  const long long rows = (long long)a.B * a.H * a.S;
  const int qb = 32 * g_dq_waves;
  const int qgrid = ((a.S + qb - 1) / qb) * a.H * a.B;
  const int kgrid = ((a.Skv + 127) / 128) * a.H * a.B;
  hipLaunchKernelGGL(attn_bwd_delta_kernel<D>, dim3((unsigned)((rows * (D / 8) + NT - 1) / NT)), dim3(NT), 0, stream,
                     a);
  if (g_dq_waves == 4) hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 4>), dim3(qgrid), dim3(256), QLDS, stream, a);
  else hipLaunchKernelGGL((attn_bwd_dq_kernel<D, 8>), dim3(qgrid), dim3(512), QLDS, stream, a);
  if (g_dkdv_waves == 8)
    hipLaunchKernelGGL(attn_bwd_dkdv8_kernel<D>, dim3(((a.Skv + 255) / 256) * a.H * a.B), dim3(512), KLDS8, stream, a,
                       ws);
  else hipLaunchKernelGGL(attn_bwd_dkdv_kernel<D>, dim3(kgrid), dim3(NT), KLDS, stream, a, ws);
  if (a.H != a.Hkv) {
    const long long n8 = (long long)a.B * a.Hkv * a.Skv * (D / 8);
    const int grid = (int)std::min<long long>((n8 + NT - 1) / NT, 2048);
    hipLaunchKernelGGL(attn_bwd_reduce_kernel<D>, dim3(grid), dim3(NT), 0, stream, a, (const float*)ws);
  }
  return (int)hipGetLastError();
}

PLX_API void plx_attn_set_dq_waves(int nw) { g_dq_waves = nw == 4 ? 4 : 8; }
PLX_API void plx_attn_set_dkdv_waves(int nw) { g_dkdv_waves = nw == 4 ? 4 : 8; }

PLX_API int plx_attn_bwd(const AttnArgs* args, int D, float* ws, hipStream_t stream) {
  const AttnArgs& a = *args;
  if (!args_ok(a, D)) return 1;
  const long long strides[] = {a.so.s, a.sdo.s, a.sdq.s, a.sdk.s, a.sdv.s, a.so.h, a.sdo.h, a.sdq.h, a.sdk.h, a.sdv.h};
  for (long long s : strides)
    if (s % 8) return 1;
  if (a.H != a.Hkv && ws == nullptr) return 2;
  return D == 128 ? launch_bwd<128>(a, ws, stream) : launch_bwd<64>(a, ws, stream);
}

PLX_API int plx_attn_args_size() { return (int)sizeof(AttnArgs); }
