// Large-tile bf16 GEMMs for the language-model linears on MI355X (gfx950).
//
//   C[M][N] = alpha * sum_k A(m, k) B(n, k)   (+ C when accumulating), C bf16 row-major (ldc)
//
// with each operand either K-MAJOR (X[r][k], k contiguous) or MN-MAJOR (X[k][r], r contiguous).  A transformer linear
// y = x W^T (W stored [out][in], as nn.Linear) needs all three combinations (ops/gemm.py):
//   forward  y[T][out]  = x[T][in] . W[out][in]^T    A K-major, B K-major   ("NT")
//   dgrad    dx[T][in]  = dy[T][out] . W[out][in]    A K-major, B MN-major  ("NN")
//   wgrad    dW[out][in] = dy[T][out]^T . x[T][in]   A MN-major, B MN-major ("TN"), K = tokens
//
// The kernel is the 256 x 256 x 64 tile of cdna_hip_programming.md §5 ("the 256^2 8-phase template"), written for
// this repository:
//   * 512 threads = 8 waves as 2 (M) x 4 (N); each wave owns a 128 x 64 block of C as 8 x 4 tiles of
//     v_mfma_f32_16x16x32_bf16 (128 accumulator registers).  The MFMA A operand is B's rows (n), its B operand A's
//     rows (m), so each lane's accumulator holds 4 consecutive n of one m: the epilogue stores 8 contiguous bytes.
//   * LDS: 2 buffers x (A 256 x 64 + B 256 x 64) bf16 = 128 KiB, one block per CU.  A buffer is staged as four 16 KiB
//     "quarters" by global_load_lds (buffer-resource LDS-DMA, 16 B per lane, lane-linear 1 KiB pieces, XOR swizzle
//     applied to the per-lane SOURCE chunk and to the read: rule 21).  A-mi0 / A-mi1 hold rows 0-63 / 64-127 of each
//     wave row's 128, B-ni0 / B-ni1 columns 0-31 / 32-63 of each wave column's 64.  A K-major quarter is 128 rows of
//     128 B read with ds_read_b128; an MN-major quarter is 64 k-rows of 256 B read with ds_read_b64_tr_b16 (T10, the
//     hardware transpose), two reads per fragment.
//   * A K-tile runs as 4 phases, one C quadrant (4 x 2 MFMA tiles x K 64 = 16 MFMAs per wave) each, in the order
//     (mi, ni) = (0,0) (0,1) (1,1) (1,0).  Phase p reads B-ni0, B-ni1, A-mi1, and in phase 3 the NEXT tile's A-mi0
//     (B-ni0 stays in registers for phase 3), so every wave reads 8 / 4 / 4 / 8 KiB per phase instead of 12 / 4 / 8 / 0.
//     Each phase: ds_read its fragments -> issue one quarter DMA -> counted vmcnt -> lgkmcnt(0) -> raw s_barrier ->
//     16 MFMAs at s_setprio 1 -> raw s_barrier.
//   * DMA ring: a slot is restaged one phase after its last read, for the tile two ahead, so six quarters (12 DMAs)
//     stay in flight and vmcnt never drains in the loop (see `ring` below for the sequence numbering).  A quarter
//     is rewritten only after the barrier that follows the lgkmcnt retiring its last read (WAR) and read only one
//     phase after the wait that retired it (RAW).  Never __syncthreads() here: its fence would drain vmcnt.
//   * Ping-pong (T5): the waves of row 1 run one barrier behind row 0, so on every SIMD one wave's MFMAs overlap
//     the other wave's LDS reads (measured +5-10 % on the K-major shapes over the lock-step schedule).
//   * blockIdx is remapped so consecutive tiles share an XCD (T1), and blockIdx.y splits K when the tile grid alone
//     cannot fill the 256 CUs (weight gradients of narrow layers: out x in tiles, K = tokens): the splits write fp32
//     slabs that gemm256_reduce sums (and adds to C).
// Requirements (host-checked): M, N multiples of 256, K of 64, 16-B aligned rows, offsets below 2 GiB per tile origin.
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "handoff.h"

#define PLX_API extern "C" __attribute__((visibility("default")))

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef unsigned u32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;

constexpr int BM = 256, BN = 256, BK = 64, NTH = 512;
constexpr int QUARTER = 16384;             // 128 rows x 128 B (K-major) or 64 k-rows x 256 B (MN-major)
constexpr int BUF = 4 * QUARTER;           // one K-tile: [A-mi0 | A-mi1 | B-ni0 | B-ni1]
constexpr int LDS_BYTES = 2 * BUF;

// K-major quarter rows (128 B): physical 16-B chunk = logical ^ kswz(row) (conflict-free ds_read_b128)
__device__ __forceinline__ int kswz(int row) { return (row >> 1) & 7; }
// MN-major quarter k-rows (256 B): physical chunk = logical ^ tswz(row): the 8 k-rows one 32-lane half of a
// ds_read_b64_tr_b16 touches land on 8 disjoint 32-B bank windows
__device__ __forceinline__ int tswz(int row) { return 2 * ((row & 3) | (((row >> 3) & 1) << 2)); }

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
  const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
  const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
  return base + (bid >> 3);
}

// Tile of logical id (consecutive ids share an XCD, xcd_remap): ids walk `group` M-tiles of one N-column, then the
// next column -- the ~32 blocks an XCD holds at once cover a group x (32 / group) patch, so each A slab is read by
// 32 / group of them and each B slab by `group` from that XCD's L2.  group 1 (row-major: every concurrent block a
// different B tile) left the Llama MLP-up forward at a 51 % L2 hit rate against hipBLASLt's 79 %
// (profiles/r4_lm_gemm.md).
__device__ __forceinline__ void tile_of(int id, int ntm, int ntn, int group, int& tm, int& tn) {
  const int per = group * ntn;
  const int first = (id / per) * group;
  const int gs = min(ntm - first, group);
  const int r = id - (id / per) * per;
  tm = first + r % gs;
  tn = r / gs;
}

__device__ __forceinline__ __amdgpu_buffer_rsrc_t rsrc(const void* base) {
  return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, 0x7ffffff0, 0x00020000);
}

__device__ __forceinline__ void glds(__amdgpu_buffer_rsrc_t r, uint32_t off, void* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)l, 16, off, 0, 0, 0);
}

__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
  return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)b) << 16);
}

// tile row/column of quarter position c (0..127) of quarter `sub`: A quarters split each wave row's 128 rows into
// 64 + 64, B quarters each wave column's 64 columns into 32 + 32
template <bool IS_A>
__device__ __forceinline__ int tile_idx(int sub, int c) {
  return IS_A ? (c >> 6) * 128 + sub * 64 + (c & 63) : (c >> 5) * 64 + sub * 32 + (c & 31);
}

// byte offset (relative to the operand's tile origin at the block's first k) that this lane's DMA of piece `piece`
// of quarter `sub` fetches at K-tile 0; K-tile kt adds kt * (K-tile stride)
template <bool IS_A, bool KMAJ>
__device__ __forceinline__ uint32_t src_off(int sub, int piece, int lane, int ld) {
  if (KMAJ) {
    const int row = piece * 8 + (lane >> 3);
    const int chunk = (lane & 7) ^ kswz(row);
    return (uint32_t)((tile_idx<IS_A>(sub, row) * ld + chunk * 8) * 2);
  } else {
    const int kr = piece * 4 + (lane >> 4);
    const int chunk = (lane & 15) ^ tswz(kr);
    return (uint32_t)((kr * ld + tile_idx<IS_A>(sub, chunk * 8)) * 2);
  }
}

// src_off(sub, wave + 8 pc, lane) = v(lane, wave) + s(sub, pc, wave): the lane-dependent part (K-major: row
// lane >> 3 and the swizzled chunk, whose swizzle depends on the piece only through wave & 1; MN-major: k-row
// lane >> 4 and the chunk, through (wave >> 1) & 1) is the same for every quarter and piece of a wave, the rest is
// uniform.  v = the offset of (sub 0, piece wave); s = each piece's difference, taken at lane 0.
template <bool IS_A, bool KMAJ>
__device__ __forceinline__ void src_split(int wave, int lane, int ld, uint32_t& v, uint32_t (&s0)[2],
                                          uint32_t (&s1)[2]) {
  v = src_off<IS_A, KMAJ>(0, wave, lane, ld);
  const uint32_t base = src_off<IS_A, KMAJ>(0, wave, 0, ld);
#pragma unroll
  for (int pc = 0; pc < 2; ++pc) {
    s0[pc] = src_off<IS_A, KMAJ>(0, wave + 8 * pc, 0, ld) - base;
    s1[pc] = src_off<IS_A, KMAJ>(1, wave + 8 * pc, 0, ld) - base;
  }
}

__device__ __forceinline__ void glds2(__amdgpu_buffer_rsrc_t r, uint32_t voff, uint32_t soff, void* l) {
  __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)l, 16, voff, soff, 0, 0);
}

// Fragment addresses.  An MFMA fragment holds row r = c0 + (lane & 15) of a quarter image (c0 = 16-aligned quarter
// position), k = 32 s + 8 (lane >> 4) + j.  The per-lane byte offset is computed once; the rest of the address is a
// compile-time constant, so every ds_read in the loop is "base VGPR + immediate" (computing the XOR-swizzled
// address per read made the compiler hoist ~50 loop-invariant addresses into VGPRs and spill).
//   K-major: kswz(c0 + fr) = kswz(fr), so the offset depends on (lane, s) only; tile t adds t * 16 rows * 128 B.
//   MN-major: tswz(kr) is unchanged by kr + 32 s and kr + 4, so (lane, t) fixes the offset; step s adds 32 k-rows
//   (8192 B) and the second half of the fragment 4 k-rows (1024 B).
template <bool KMAJ>
__device__ __forceinline__ int frag_off(int c0, int ts, int lane) {
  const int fr = lane & 15, fq = lane >> 4;
  if (KMAJ) {  // ts = s
    return (c0 + fr) * 128 + (((ts * 4 + fq) ^ kswz(fr)) << 4);
  } else {     // ts = t; T10: lane 4q+p of a 16-lane group addresses k-row q, columns c + 4p .. 4p+3
    const int col = c0 + ts * 16 + 4 * (lane & 3);
    const int kr = 8 * fq + (fr >> 2);
    return kr * 256 + (((col >> 3) ^ tswz(kr)) << 4) + ((col >> 2) & 1) * 8;
  }
}

__device__ __forceinline__ bf16x8 ld_frag_k(const char* p) { return *(const bf16x8*)p; }

__device__ __forceinline__ bf16x8 ld_frag_t(const char* p) {
  const s16x4 lo = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)p);
  const s16x4 hi = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) s16x4*)(p + 1024));
  return __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
}

struct FragA {
  bf16x8 v[4][2];
};
struct FragB {
  bf16x8 v[2][2];
};

template <int V>
struct IC {
  static constexpr int value = V;
};
template <bool V>
struct IB {
  static constexpr bool value = V;
};

struct Gemm256Args {
  const __bf16* A;
  const __bf16* B;
  void* C;            // bf16 [M][ldc], or fp32 slabs [splits][M][N] when K is split
  int M, N, K, lda, ldb, ldc;
  int kt_per_split;   // K-tiles per blockIdx.y
  float alpha;
  const float* bias;  // fp32 [N] added after alpha in the bf16 epilogue (the Linear bias), or null
  void* C2;           // bf16 [M][ldc]: gelu_tanh of the stored (bf16-rounded) C, or null (GPT-2's up-projection)
  int group;          // M-tiles per tile group (tile_of)
  const __bf16* gelu_h;  // bf16 [M][ldc] or null: the epilogue stores bf16(C) * gelu_tanh'(gelu_h) instead of C (the
                         // GELU backward of an MLP fused into the down-projection's data gradient); no bias / C2
};

// GELU, tanh approximation, of the bf16-rounded value (what a separate activation pass reading C would compute);
// tanh(u) = 1 - 2 / (1 + e^{2u}) on v_exp_f32 / v_rcp_f32
__device__ __forceinline__ float gelu_tanh(float h) {
  const float u = 0.7978845608028654f * fmaf(0.044715f * h * h, h, h);
  return 0.5f * h * (2.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * u)));
}

__device__ __forceinline__ float bf16_round(float f) { return (float)(__bf16)f; }

// d/dh gelu_tanh(h): the formula of csrc/lm_kernels.hip gelu_tanh_grad (bit-identical results), so the fused GELU
// backward equals the separate pass over the stored data gradient
__device__ __forceinline__ float gelu_tanh_grad(float h) {
  const float k0 = 0.7978845608028654f, k1 = 0.044715f;
  const float e = __expf(2.f * k0 * fmaf(k1 * h * h, h, h));
  const float t = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + e);
  return fmaf(0.5f, 1.f + t, 0.5f * h * (1.f - t * t) * k0 * fmaf(3.f * k1, h * h, 1.f));
}

// Epilogue store layout.  An MFMA tile's lane holds 4 consecutive columns of one row, so storing tiles one by one
// writes 8 bytes per lane and 32 contiguous bytes per row: the memory side then sees 32-byte partial-line writes
// (PMC on the GPT-2 head forward: 1.85x hipBLASLt's TCC_EA0_WRREQ for the same output; profiles/r5_lm_gemm.md).
// pair_permute regroups two column-adjacent tiles a (columns 0-15) and b (16-31) with two cross-lane swaps per
// register (gfx950 v_permlane32_swap / v_permlane16_swap, VALU, no LDS): afterwards lane quarter q = lane >> 4 holds
// columns 8q..8q+3 in a and 8q+4..8q+7 in b, so each lane stores 16 contiguous bytes and a row gets 64.
//   permlane32_swap(a, b): a's quarters 2, 3 <-> b's quarters 0, 1  ->  a = [a0 a1 b0 b1], b = [a2 a3 b2 b3]
//   permlane16_swap(a, b): a's quarters 1, 3 <-> b's quarters 0, 2  ->  a = [a0 a2 b0 b2], b = [a1 a3 b1 b3]
// (xk = quarter k of x: columns 4k..4k+3 of its tile), i.e. quarter q holds columns 8q..8q+7 of the 32.
__device__ __forceinline__ void pair_permute(f32x4& a, f32x4& b) {
#pragma unroll
  for (int j = 0; j < 4; ++j) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a[j]), __float_as_uint(b[j]), false, false);
    const auto t = __builtin_amdgcn_permlane16_swap(r[0], r[1], false, false);
    a[j] = __uint_as_float(t[0]);
    b[j] = __uint_as_float(t[1]);
  }
}

// the bias of a lane's 8 columns n8..n8+7 (zeros without one), loaded once per column pair outside the row loop: in
// the row loop the loads were re-issued for every row (no restrict on the bias / C pointers) and each waited on
// its own round trip, +22 us on the GPT-2 QKV forward and +317 us on the head (r5_lm_gemm_epilogue_ab.jsonl)
__device__ __forceinline__ void load_bias8(const Gemm256Args& p, int n8, f32x4& ba, f32x4& bb) {
  if (p.bias != nullptr) {  // uniform branch; 32-byte aligned (bias 16-byte aligned, n8 % 8 == 0)
    ba = *(const f32x4*)(p.bias + n8);
    bb = *(const f32x4*)(p.bias + n8 + 4);
  } else {
    ba = f32x4{0.f, 0.f, 0.f, 0.f};
    bb = ba;
  }
}

// bf16 epilogue of one permuted tile pair at row m, columns n8..n8+7 (n8 % 8 == 0: 16-byte aligned stores);
// ba / bb: load_bias8 of n8 (ignored when accumulating)
// GB: the kernel supports the fused GELU backward (p.gelu_h; the persistent kernel only, so the other kernels'
// epilogues do not carry its registers)
template <bool ACC, bool GB = false>
__device__ __forceinline__ void store_pair(const Gemm256Args& p, f32x4 a, f32x4 b, int m, int n8, const f32x4& ba,
                                           const f32x4& bb) {
  __bf16* dst = (__bf16*)p.C + (size_t)m * p.ldc + n8;
  if (ACC) {
    const uint4 o = *(const uint4*)dst;
    a[0] = p.alpha * a[0] + __uint_as_float(o.x << 16);
    a[1] = p.alpha * a[1] + __uint_as_float(o.x & 0xffff0000u);
    a[2] = p.alpha * a[2] + __uint_as_float(o.y << 16);
    a[3] = p.alpha * a[3] + __uint_as_float(o.y & 0xffff0000u);
    b[0] = p.alpha * b[0] + __uint_as_float(o.z << 16);
    b[1] = p.alpha * b[1] + __uint_as_float(o.z & 0xffff0000u);
    b[2] = p.alpha * b[2] + __uint_as_float(o.w << 16);
    b[3] = p.alpha * b[3] + __uint_as_float(o.w & 0xffff0000u);
  } else {
    a = a * p.alpha + ba;
    b = b * p.alpha + bb;
    if (GB && p.gelu_h != nullptr) {  // uniform branch: dh = bf16(dA) * gelu'(h), dA rounded as a stored C would be
      const uint4 hv = *(const uint4*)(p.gelu_h + (size_t)m * p.ldc + n8);
      a[0] = bf16_round(a[0]) * gelu_tanh_grad(__uint_as_float(hv.x << 16));
      a[1] = bf16_round(a[1]) * gelu_tanh_grad(__uint_as_float(hv.x & 0xffff0000u));
      a[2] = bf16_round(a[2]) * gelu_tanh_grad(__uint_as_float(hv.y << 16));
      a[3] = bf16_round(a[3]) * gelu_tanh_grad(__uint_as_float(hv.y & 0xffff0000u));
      b[0] = bf16_round(b[0]) * gelu_tanh_grad(__uint_as_float(hv.z << 16));
      b[1] = bf16_round(b[1]) * gelu_tanh_grad(__uint_as_float(hv.z & 0xffff0000u));
      b[2] = bf16_round(b[2]) * gelu_tanh_grad(__uint_as_float(hv.w << 16));
      b[3] = bf16_round(b[3]) * gelu_tanh_grad(__uint_as_float(hv.w & 0xffff0000u));
    }
  }
  uint4 packed;
  packed.x = pack_bf16x2(a[0], a[1]);
  packed.y = pack_bf16x2(a[2], a[3]);
  packed.z = pack_bf16x2(b[0], b[1]);
  packed.w = pack_bf16x2(b[2], b[3]);
  *(uint4*)dst = packed;
  if (!ACC && p.C2 != nullptr) {  // uniform branch
    uint4 g;
    g.x = pack_bf16x2(gelu_tanh(bf16_round(a[0])), gelu_tanh(bf16_round(a[1])));
    g.y = pack_bf16x2(gelu_tanh(bf16_round(a[2])), gelu_tanh(bf16_round(a[3])));
    g.z = pack_bf16x2(gelu_tanh(bf16_round(b[0])), gelu_tanh(bf16_round(b[1])));
    g.w = pack_bf16x2(gelu_tanh(bf16_round(b[2])), gelu_tanh(bf16_round(b[3])));
    *(uint4*)((__bf16*)p.C2 + (size_t)m * p.ldc + n8) = g;
  }
}

// One output tile's K loop, K-tiles [kt0, kt0 + nk), accumulated into acc (callers zero it): the 256 x 256 x 64
// ping-pong schedule described in the file header.  Leaves every LDS read of the tile done (all waves past the same
// barriers) and, standalone, every DMA retired, so the caller may restage the LDS right away.
//
// Chained (the persistent kernel; nk even, the next piece >= 2 K-tiles): the tile's first two K-tiles were issued
// before it (gemm256_prologue, or the previous tile's chained ring), followed by `extra` more vector-memory ops (the
// previous tile's epilogue stores, 0 / 16 / 32): the waits of the first six phases count them in, so those stores
// drain behind the fill instead of before it (vmcnt retires loads and stores in issue order).  The ring does not
// drain at the end of the tile but goes on with `chain`'s K-tiles 0 and 1 (and wave 0 its bias), into the same
// slots: the next tile starts with its first two K-tiles landed.  nk even keeps the slot parity: the next piece's
// K-tile j lands where this tile's K-tile nk + j would have.
struct Chain {
  int m0, n0, kt0;
  float* bias_lds;
};

template <bool AK, bool BKM>
__device__ __forceinline__ void gemm256_prologue(const Gemm256Args& p, int m0, int n0, int kt0, int nk, char* smem,
                                                 int wave, int lane, float* bias_lds = nullptr);

// CHAINED = false: standalone (issues its own fill, drains at the end).  CHAINED = true (the persistent kernel): the
// fill was issued by the previous tile's chained ring (or the caller's prologue), the first K-tile pair is peeled
// (only its waits count the previous tile's stores: with that runtime check in every phase the GPT-2 head forward
// took 1.38 ms instead of 1.27), and the chain is a compile-time branch of the ring (a runtime chain check in every
// phase, with the chained operands' buffer resources live across the K loop, had 2.6x the branches and ran 13 %
// slower on Llama's 4096^3 projection).
template <bool AK, bool BKM, bool CHAINED = false>
__device__ __forceinline__ void gemm256_tile(const Gemm256Args& p, int m0, int n0, int kt0, int nk, f32x4 (&acc)[4][8],
                                             char* smem, int wave, int lane, int wm, int wn, int extra = 0,
                                             const Chain& chain = Chain{0, 0, 0, nullptr}) {
  const size_t k0 = (size_t)kt0 * BK;

  // buffer resources anchored at this block's tile origin (offsets stay 32-bit for any matrix size)
  const __bf16* abase = AK ? p.A + (size_t)m0 * p.lda + k0 : p.A + k0 * p.lda + m0;
  const __bf16* bbase = BKM ? p.B + (size_t)n0 * p.ldb + k0 : p.B + k0 * p.ldb + n0;
  const __amdgpu_buffer_rsrc_t ra = rsrc(abase), rb = rsrc(bbase);
  const uint32_t astep = AK ? BK * 2 : (uint32_t)(BK * p.lda * 2);
  const uint32_t bstep = BKM ? BK * 2 : (uint32_t)(BK * p.ldb * 2);

  // Source offsets of the two pieces (wave, wave + 8) of each quarter, in issue order 0 = A-mi0, 1 = B-ni0,
  // 2 = B-ni1, 3 = A-mi1, split as one per-lane VGPR per operand + a wave-uniform SGPR part (src_split): 2 VGPRs
  // instead of 8 next to the 128 accumulators.
  uint32_t va, vb, sof[4][2];
  src_split<true, AK>(wave, lane, p.lda, va, sof[0], sof[3]);
  src_split<false, BKM>(wave, lane, p.ldb, vb, sof[1], sof[2]);
  auto issue_from = [&](__amdgpu_buffer_rsrc_t ra_, __amdgpu_buffer_rsrc_t rb_, int buf, int kt, int q) {
    // LDS placement: A-mi0 at 0, A-mi1 at QUARTER, B-ni0 at 2 QUARTER, B-ni1 at 3 QUARTER
    const int qoff = q == 0 ? 0 : q == 3 ? QUARTER : q == 1 ? 2 * QUARTER : 3 * QUARTER;
    char* dst = smem + buf * BUF + qoff;
    const bool isa = q == 0 || q == 3;
    const uint32_t koff = (uint32_t)kt * (isa ? astep : bstep);
    const __amdgpu_buffer_rsrc_t r = isa ? ra_ : rb_;
    glds2(r, isa ? va : vb, sof[q][0] + koff, dst + wave * 1024);
    glds2(r, isa ? va : vb, sof[q][1] + koff, dst + (wave + 8) * 1024);
  };
  auto issue = [&](int buf, int kt, int q) { issue_from(ra, rb, buf, kt, q); };
  // the chained next piece's operands (same strides)
  // (built where used: the chain's origin goes through an opaque move so its buffer resources are not hoisted out of
  // the K loop, where 8 more live SGPRs pushed SGPRs into VGPR lanes)
  auto chain_issue = [&](int buf, int j, int q) {
    int cm = chain.m0, cn = chain.n0, ck = chain.kt0;
    asm volatile("" : "+s"(cm), "+s"(cn), "+s"(ck));
    const size_t nk0 = (size_t)ck * BK;
    issue_from(rsrc(AK ? p.A + (size_t)cm * p.lda + nk0 : p.A + nk0 * p.lda + cm),
               rsrc(BKM ? p.B + (size_t)cn * p.ldb + nk0 : p.B + nk0 * p.ldb + cn), buf, j, q);
  };


  // per-lane fragment offsets inside a quarter image (K-major: [s]; MN-major: [t])
  int aoff[4], boff[2];
#pragma unroll
  for (int i = 0; i < 4; ++i) aoff[i] = frag_off<AK>(wm * 64, AK ? (i & 1) : i, lane);
#pragma unroll
  for (int i = 0; i < 2; ++i) boff[i] = frag_off<BKM>(wn * 32, i, lane);
  // Fragments are returned by value and live only inside one K-tile (declaring them outside the loop made them
  // loop-carried: phis over the issue / no-issue paths kept dead copies alive and the kernel spilled).
  // img = smem + compile-time constant, so each read is base VGPR + immediate offset.
  auto read_a = [&](const char* img) {  // MFMA B operand = A rows (m): [m tile of the quadrant][k step]
    FragA f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        f.v[t][s] = AK ? ld_frag_k(img + aoff[s] + t * 2048) : ld_frag_t(img + aoff[t] + s * 8192);
    return f;
  };
  auto read_b = [&](const char* img) {  // MFMA A operand = B rows (n): [n tile of the quadrant][k step]
    FragB f;
#pragma unroll
    for (int t = 0; t < 2; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s)
        f.v[t][s] = BKM ? ld_frag_k(img + boff[s] + t * 2048) : ld_frag_t(img + boff[t] + s * 8192);
    return f;
  };
  // One phase's synchronisation + MFMAs.  This wave's ds_reads retire (lgkmcnt(0)) BEFORE the first barrier, so
  // a slot read in phase p may be restaged by any wave from phase p + 1 on (WAR), and a DMA retired by the issuing
  // waves' vmcnt before phase p's first barrier may be read from phase p + 1 on (RAW).
  auto mfma_phase = [&](const FragA& fa, const FragB& fb, int mi, int ni) {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_setprio(1);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 2; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b)
          acc[ni * 2 + a][mi * 4 + b] =
              __builtin_amdgcn_mfma_f32_16x16x32_bf16(fb.v[a][s], fa.v[b][s], acc[ni * 2 + a][mi * 4 + b], 0, 0, 0);
    __builtin_amdgcn_s_setprio(0);
    __builtin_amdgcn_sched_barrier(0);
    __builtin_amdgcn_s_barrier();
  };
  // DMA ring.  Quarters are numbered in issue order, seq = 4 u + o for K-tile u and o = 0 A-mi0, 1 B-ni0, 2 B-ni1,
  // 3 A-mi1; there are S = 4 nk of them.  Tile t reads B-ni0 in phase 0, B-ni1 in phase 1, A-mi1 in phase 2 and
  // the NEXT tile's A-mi0 in phase 3 (its own A-mi0 came in the previous tile's phase 3), 8 / 4 / 4 / 8 KiB-reads
  // per wave.  Each slot of buffer t & 1 is free one phase after its last read, so global phase g = 4 t + p
  // restages quarter o = p of tile t + 2, seq g + 8 (the prologue issues 0..7), and every phase retires up to
  // seq g + 2, the quarter first read in phase g + 1: six quarters = 12 DMAs stay in flight in the steady state.
  const int S = 4 * nk;
  auto wait_vm = [&](int n) {  // n = DMAs allowed in flight (even), wave-uniform
    if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    else if (n >= 10) asm volatile("s_waitcnt vmcnt(10)" ::: "memory");
    else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
    else if (n >= 6) asm volatile("s_waitcnt vmcnt(6)" ::: "memory");
    else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
    else if (n >= 2) asm volatile("s_waitcnt vmcnt(2)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
  };
  // steady-state wait for seq g + 2: 12 DMAs younger -- plus, in the persistent modes' first K-tile pair, the
  // previous tile's stores while they are younger than it (phases 0 .. 5: seq 2 .. 7 were issued before the stores)
  auto wait12 = [&](auto first, int g) {
    if constexpr (decltype(first)::value) {
      if (g < 6 && extra >= 32) asm volatile("s_waitcnt vmcnt(44)" ::: "memory");
      else if (g < 6 && extra >= 16) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
      else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    } else {
      asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
    }
  };
  // Issue seq g + 8 (tile kt + 2, kind P, into this tile's buffer CB) and wait for seq g + 2.  Past this tile's last
  // K-tile, the chained kernel issues the next piece's K-tile kt + 2 - nk instead (wave 0 also stages that piece's bias) and
  // the other modes drain the ring.
  auto ring = [&](auto cb, auto ph, auto first, int kt) {
    constexpr int CB = decltype(cb)::value, P = decltype(ph)::value;
    const int g = 4 * kt + P;
    if (g + 8 < S) {
      issue(CB, kt + 2, P);
      wait12(first, g);
    } else if constexpr (CHAINED) {
      if (P == 0 && kt == nk - 2 && wave == 0 && p.bias != nullptr && chain.bias_lds != nullptr)
        glds(rsrc(p.bias + chain.n0), lane * 16, chain.bias_lds);
      chain_issue(CB, kt + 2 - nk, P);
      wait12(first, g);
    } else {
      wait_vm(2 * ((S - 1) - (g + 2)));
    }
  };
  auto tile = [&](auto cb, auto first, int kt, FragA& a0) {
    constexpr int CB = decltype(cb)::value;
    const char* qa1 = smem + CB * BUF + QUARTER;
    const char* qb0 = smem + CB * BUF + 2 * QUARTER;
    const char* qb1 = smem + CB * BUF + 3 * QUARTER;
    const char* qa0_next = smem + (1 - CB) * BUF;
    // phase 0: quadrant (0,0); reads B-ni0
    const FragB b0 = read_b(qb0);
    ring(cb, IC<0>{}, first, kt);
    mfma_phase(a0, b0, 0, 0);
    // phase 1: quadrant (0,1); reads B-ni1
    const FragB b1 = read_b(qb1);
    ring(cb, IC<1>{}, first, kt);
    mfma_phase(a0, b1, 0, 1);
    // phase 2: quadrant (1,1); reads A-mi1
    const FragA a1 = read_a(qa1);
    ring(cb, IC<2>{}, first, kt);
    mfma_phase(a1, b1, 1, 1);
    // phase 3: quadrant (1,0) from registers; reads the next tile's A-mi0
    if (kt + 1 < nk) a0 = read_a(qa0_next);
    ring(cb, IC<3>{}, first, kt);
    mfma_phase(a1, b0, 1, 0);
  };

  // prologue: seq 0 .. min(7, S - 1) (tiles 0 and 1); retire seq 0, 1 and read tile 0's A-mi0
  if constexpr (!CHAINED) {
#pragma unroll
    for (int q = 0; q < 4; ++q) issue(0, 0, q);
    if (nk > 1) {
#pragma unroll
      for (int q = 0; q < 4; ++q) issue(1, 1, q);
    }
  }
  if (nk > 1) {
    if (extra >= 32) asm volatile("s_waitcnt vmcnt(44)" ::: "memory");
    else if (extra >= 16) asm volatile("s_waitcnt vmcnt(28)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  } else {
    if (extra >= 32) asm volatile("s_waitcnt vmcnt(36)" ::: "memory");
    else if (extra >= 16) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
    else asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  }
  __builtin_amdgcn_s_barrier();
  FragA a0 = read_a(smem);
  // Ping-pong (T5): the waves of row wm = 1 (one per SIMD) run one barrier behind those of row 0, so on every SIMD
  // one wave's MFMAs (priority 1) overlap the other wave's ds_reads and DMA issue.
  if (wm == 1) __builtin_amdgcn_s_barrier();

  int kt = 0;
  if constexpr (CHAINED) {  // peeled first pair: the only phases whose waits count the previous tile's stores
    tile(IC<0>{}, IB<true>{}, 0, a0);
    if (1 < nk) tile(IC<1>{}, IB<true>{}, 1, a0);
    kt = 2;
  }
  for (; kt < nk; kt += 2) {
    tile(IC<0>{}, IB<false>{}, kt, a0);
    if (kt + 1 < nk) tile(IC<1>{}, IB<false>{}, kt + 1, a0);
  }
  if (wm == 0) __builtin_amdgcn_s_barrier();  // every wave executes the same number of barriers

}

// bf16 epilogue of one tile (bias / GELU / accumulate per the args): column-adjacent tile pairs regrouped to 16-byte
// stores (pair_permute)
// (bias: load_bias16 of the tile, or zeros when accumulating); 16 stores per lane, 32 with the GELU output
template <bool ACC, bool GB = false>
__device__ __forceinline__ void gemm256_store(const Gemm256Args& p, f32x4 (&acc)[4][8], int m0, int n0, int lane, int wm,
                                              int wn, const f32x4 (&bias)[2][2]) {
  const int fr = lane & 15, fq = lane >> 4;
#pragma unroll
  for (int np = 0; np < 2; ++np) {
    const int n8 = n0 + wn * 64 + np * 32 + 8 * fq;
#pragma unroll
    for (int mt = 0; mt < 8; ++mt) {
      f32x4 a = acc[2 * np][mt], b = acc[2 * np + 1][mt];
      pair_permute(a, b);
      store_pair<ACC, GB>(p, a, b, m0 + wm * 128 + mt * 16 + fr, n8, bias[np][0], bias[np][1]);
    }
  }
}

// the bias of this lane's 16 columns of the tile at n0 (gemm256_store's column pairs)
__device__ __forceinline__ void load_bias16(const Gemm256Args& p, int n0, int lane, int wn, f32x4 (&bias)[2][2]) {
#pragma unroll
  for (int np = 0; np < 2; ++np) load_bias8(p, n0 + wn * 64 + np * 32 + 8 * (lane >> 4), bias[np][0], bias[np][1]);
}

// bias_lds: when the GEMM has a bias, wave 0 also stages the tile's 256 bias values there (one 1 KiB DMA, older than
// every ring DMA, so the ring's first wait retires it)
// load_bias16 from the tile's bias staged in LDS by gemm256_prologue (zeros without a bias)
__device__ __forceinline__ void lds_bias16(const Gemm256Args& p, const float* bias_lds, int lane, int wn,
                                           f32x4 (&bias)[2][2]) {
#pragma unroll
  for (int np = 0; np < 2; ++np) {
    if (p.bias != nullptr) {
      const float* b = bias_lds + wn * 64 + np * 32 + 8 * (lane >> 4);
      bias[np][0] = *(const f32x4*)b;
      bias[np][1] = *(const f32x4*)(b + 4);
    } else {
      bias[np][0] = f32x4{0.f, 0.f, 0.f, 0.f};
      bias[np][1] = bias[np][0];
    }
  }
}

template <bool AK, bool BKM>
__device__ __forceinline__ void gemm256_prologue(const Gemm256Args& p, int m0, int n0, int kt0, int nk, char* smem,
                                                 int wave, int lane, float* bias_lds) {
  if (bias_lds != nullptr && p.bias != nullptr && wave == 0) glds(rsrc(p.bias + n0), lane * 16, bias_lds);
  const size_t k0 = (size_t)kt0 * BK;
  const __bf16* abase = AK ? p.A + (size_t)m0 * p.lda + k0 : p.A + k0 * p.lda + m0;
  const __bf16* bbase = BKM ? p.B + (size_t)n0 * p.ldb + k0 : p.B + k0 * p.ldb + n0;
  const __amdgpu_buffer_rsrc_t ra = rsrc(abase), rb = rsrc(bbase);
  const uint32_t astep = AK ? BK * 2 : (uint32_t)(BK * p.lda * 2);
  const uint32_t bstep = BKM ? BK * 2 : (uint32_t)(BK * p.ldb * 2);
  // the same quarter order and placement as gemm256_tile's `issue`
#pragma unroll
  for (int kt = 0; kt < 2; ++kt) {
    if (kt == 1 && nk < 2) break;
#pragma unroll
    for (int q = 0; q < 4; ++q) {
      const int qoff = q == 0 ? 0 : q == 3 ? QUARTER : q == 1 ? 2 * QUARTER : 3 * QUARTER;
      char* dst = smem + kt * BUF + qoff;
      const bool isa = q == 0 || q == 3;
      const int sub = q == 0 || q == 1 ? 0 : 1;
      const uint32_t koff = (uint32_t)kt * (isa ? astep : bstep);
#pragma unroll
      for (int pc = 0; pc < 2; ++pc) {
        const uint32_t off = isa ? src_off<true, AK>(sub, wave + 8 * pc, lane, p.lda)
                                 : src_off<false, BKM>(sub, wave + 8 * pc, lane, p.ldb);
        glds(isa ? ra : rb, off + koff, dst + (wave + 8 * pc) * 1024);
      }
    }
  }
}

// ACC: C += alpha * AB (bf16 read-modify-write); SLAB: write fp32 partials (split K)
template <bool AK, bool BKM, bool ACC, bool SLAB>
__global__ void __launch_bounds__(NTH, 1) gemm256_kernel(Gemm256Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int ntn = p.N / BN, ntm = p.M / BM;
  int tm, tn;
  tile_of(xcd_remap(blockIdx.x, ntm * ntn), ntm, ntn, p.group, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = blockIdx.y * p.kt_per_split;
  const int nk = min(p.kt_per_split, p.K / BK - kt0);

  f32x4 acc[4][8];  // [n tile: 4 x 16 = the wave's 64 columns][m tile: 8 x 16 = its 128 rows]
#pragma unroll
  for (int a = 0; a < 4; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
  gemm256_tile<AK, BKM>(p, m0, n0, kt0, nk, acc, smem, wave, lane, wm, wn);

  // epilogue: acc[nt][mt] is a 16 x 16 tile D[n][m]: m = lane & 15, n = 4 (lane >> 4) + j, j = 0..3
  const int fr = lane & 15, fq = lane >> 4;
  if (SLAB) {
#pragma unroll
    for (int nt = 0; nt < 4; ++nt)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int m = m0 + wm * 128 + mt * 16 + fr;
        const int n = n0 + wn * 64 + nt * 16 + 4 * fq;
        *(f32x4*)((float*)p.C + ((size_t)blockIdx.y * p.M + m) * p.N + n) = acc[nt][mt];
      }
  } else {
    f32x4 bias[2][2];
    load_bias16(p, n0, lane, wn, bias);
    gemm256_store<ACC>(p, acc, m0, n0, lane, wm, wn, bias);
  }
}

// ---------------------------------------------------------------------------------------------------------------
// Persistent stream-K variant of the 8-wave kernel (schedule 9).  One workgroup per CU (G = the CU count) walks
//   1. its contiguous share (ipb iterations) of the "stream-K" iteration space -- the first sk_tiles tiles x their
//      K-tiles, flattened tile-major -- so the partial wave of tiles that would leave CUs idle (T % G of them, or all
//      of them when T < G) is split along K over every CU, then
//   2. the remaining (T - sk_tiles, a multiple of G) tiles data-parallel, tile sk_tiles + blk, + G, ...
// A tile split over several workgroups is finished by the last of them to arrive (the hand-off of csrc/handoff.h:
// sc1 fp32 partials per workgroup slot, one relaxed agent-scope ticket per tile, reset by the last arriver, so
// back-to-back and graph-replayed launches reuse the zeroed tickets): nobody waits on anybody, so a workgroup that
// is not yet resident (another kernel holding CUs) can never stall the others.  A workgroup's partial pieces are its
// first (a tile's tail, slot 0) and its last SK piece (a tile's head, slot 1), so 2 G slots of 256 x 256 fp32.
// The DMA ring never drains between items: a tile's last two K-tiles issue the next item's first two (gemm256_tile
// CHAINED), the finished tile's stores follow, and the next tile's first waits count them in (`extra`): the 128 KiB
// store of one tile drains under the next tile's first loads and the workgroups' tile ends drift apart instead of
// all 256 CUs paying the ring fill and a 32 MB store burst at once (the per-tile fixed cost of
// profiles/r5_lm_gemm.md; profiles/r6_lm_gemm.md).
struct SkArgs {
  float* part;        // fp32 [2 G][65536]: per-workgroup partial slots (lane-linear f32x4 layout)
  unsigned* tickets;  // [G], zero between launches
  int sk_tiles;       // tiles in the stream-K phase (ids 0 .. sk_tiles - 1)
  int ipb;            // stream-K iterations (K-tiles) per workgroup
};

__device__ __forceinline__ __amdgpu_buffer_rsrc_t slot_rsrc(float* part, int slot) {
  return rsrc(part + (size_t)slot * 65536);
}

template <bool AK, bool BKM>
__global__ void __launch_bounds__(NTH, 1) gemm256_sk_kernel(Gemm256Args p, SkArgs s) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  __shared__ __attribute__((aligned(16))) float s_bias[2][BN];  // per-tile bias, double-buffered across tiles
  __shared__ int s_last;
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 2, wn = wave & 3;
  const int G = gridDim.x, blk = xcd_remap(blockIdx.x, G);
  const int ntn = p.N / BN, ntm = p.M / BM, T = ntm * ntn, nk = p.K / BK;
  const int sk_total = s.sk_tiles * nk;
  int it = min(sk_total, blk * s.ipb);
  const int it_end = min(sk_total, it + s.ipb);
  int dp = s.sk_tiles + blk;

  int tile = 0, kb = 0, ke = 0;
  auto next = [&]() -> bool {
    if (it < it_end) {
      tile = it / nk;
      kb = it - tile * nk;
      ke = min(nk, kb + (it_end - it));
      it += ke - kb;
      return true;
    }
    if (dp < T) {
      tile = dp;
      kb = 0;
      ke = nk;
      dp += G;
      return true;
    }
    return false;
  };
  auto origin = [&](int t, int& m0, int& n0) {
    int tm, tn;
    tile_of(t, ntm, ntn, p.group, tm, tn);
    m0 = tm * BM;
    n0 = tn * BN;
  };
  if (!next()) return;
  int ctile = tile, ckb = kb, cke = ke, cm0, cn0;  // the current item; tile / kb / ke: the one after it
  origin(ctile, cm0, cn0);
  gemm256_prologue<AK, BKM>(p, cm0, cn0, ckb, cke - ckb, smem, wave, lane, s_bias[0]);
  // The host launches this kernel for an even K-tile count >= 4 only, so every piece is even and >= 2 (ipb is even
  // then): every tile's ring chains into the next item, the last one into a dummy re-read of itself that is drained
  // before the exit.
  int extra = 0;
  for (int slot = 0;; slot ^= 1) {
    const bool more = next();
    int m0 = cm0, n0 = cn0;
    if (more) origin(tile, m0, n0);
    const Chain ch{m0, n0, more ? kb : ckb, more ? s_bias[slot ^ 1] : nullptr};
    // The lane index is laundered once per tile so that the K loop's per-lane LDS / DMA offsets are recomputed per
    // tile instead of hoisted out of the tile loop: hoisted, they stayed live through the epilogue next to the 128
    // accumulator VGPRs and the kernel spilled (136 VGPRs).
    int ln;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln) : "v"(lane));
    f32x4 acc[4][8];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
      for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    gemm256_tile<AK, BKM, true>(p, cm0, cn0, ckb, cke - ckb, acc, smem, wave, ln, wm, wn, extra, ch);
    // every LDS read of this tile done; the next item's first two K-tiles (and its bias) are in flight
    bool store = ckb == 0 && cke == nk;
    if (!store) {
      // pieces of tile ctile: workgroups bf .. bl (the iteration space is split at multiples of ipb); the one that
      // arrives last adds the others' partials and stores the tile.  A piece that already sees every other piece's
      // ticket is last without writing its own partial.
      const int bf = (ctile * nk) / s.ipb, bl = (ctile * nk + nk - 1) / s.ipb;
      const int np = bl - bf + 1;
      if (tid == 0)
        s_last = __hip_atomic_load(s.tickets + bf, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT) == (unsigned)(np - 1);
      __syncthreads();
      int last = s_last;
      if (!last) {
        const __amdgpu_buffer_rsrc_t r = slot_rsrc(s.part, 2 * blk + (ckb == 0 ? 1 : 0));
#pragma unroll
        for (int i = 0; i < 32; ++i)
          __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i >> 3][i & 7]), r, tid * 16,
                                                 i * NTH * 16, 16 /* sc1 */);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
          plx_handoff_release();
          const unsigned old = __hip_atomic_fetch_add(s.tickets + bf, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
          s_last = old == (unsigned)(np - 1);
          if (s_last) plx_handoff_acquire();
        }
        __syncthreads();
        last = s_last;
      }
      if (last) {
        // Sum the pieces in workgroup order bf .. bl whoever arrived last (this piece from registers, the others
        // from their slots), so the result is bitwise independent of the arrival order.  8 f32x4 at a time: all 32
        // loads in flight next to the 128 accumulators spilled.
#pragma unroll
        for (int g = 0; g < 4; ++g) {
          f32x4 t[8];
#pragma unroll
          for (int u = 0; u < 8; ++u) t[u] = f32x4{0.f, 0.f, 0.f, 0.f};
          for (int b = bf; b <= bl; ++b) {
            if (b == blk) {
#pragma unroll
              for (int u = 0; u < 8; ++u) t[u] += acc[g][u];
            } else {
              const __amdgpu_buffer_rsrc_t r = slot_rsrc(s.part, 2 * b + (b == bf ? 1 : 0));
              f32x4 v[8];
#pragma unroll
              for (int u = 0; u < 8; ++u)
                v[u] = __builtin_bit_cast(
                    f32x4, __builtin_amdgcn_raw_buffer_load_b128(r, tid * 16, (g * 8 + u) * NTH * 16, 16 /* sc1 */));
#pragma unroll
              for (int u = 0; u < 8; ++u) t[u] += v[u];
            }
          }
#pragma unroll
          for (int u = 0; u < 8; ++u) acc[g][u] = t[u];
          __builtin_amdgcn_sched_barrier(0);
        }
        if (tid == 0) __hip_atomic_store(s.tickets + bf, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        store = true;
      }
    }
    // The stores go out after the next item's fill and take their bias from LDS, so nothing in the epilogue waits on
    // vmcnt behind the fill.  ln2: a fresh laundered lane (the epilogue's offsets are not kept live across the K loop).
    int ln2;
    asm volatile("v_mov_b32 %0, %1" : "=v"(ln2) : "v"(lane));
    if (store) {
      f32x4 bias[2][2];
      lds_bias16(p, s_bias[slot], ln2, wn, bias);
      gemm256_store<false, true>(p, acc, cm0, cn0, ln2, wm, wn, bias);
    }
    extra = store ? (p.C2 != nullptr ? 32 : 16) : 0;
    if (!more) break;
    ctile = tile;
    ckb = kb;
    cke = ke;
    cm0 = m0;
    cn0 = n0;
  }
  asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the dummy fill lands before the workgroup's LDS is released
}


// ---------------------------------------------------------------------------------------------------------------
// 4-wave variant: the same 256 x 256 x 64 tile, LDS layout and DMA engine, but 4 waves as 2 (M) x 2 (N), each
// owning a 128 x 128 block of C as 8 x 8 MFMA tiles.  That is a third fewer LDS fragment bytes per MFMA than the
// 8-wave kernel (each wave reads 2 x 128 x 64 bf16 per K-tile for 128 MFMAs instead of 192 x 64 for 64) and one
// wave per SIMD, so the overlap comes from software pipelining inside the wave instead of ping-pong:
//   * accumulators: 256 fp32 per lane, which only fits as AGPRs.  With __builtin_amdgcn_mfma_* hipcc keeps part of
//     them in VGPRs and shuttles them through v_accvgpr_read/write around the MFMAs (r3_negative_results.md); the
//     MFMAs are therefore issued as inline asm with the accumulator bound to an AGPR tuple ("+a"), which pins the
//     whole accumulator block in AGPRs.  The compiler does not know these are MFMAs, so the two hazards it would
//     otherwise cover are handled here: the zero-initialised AGPRs are first read many instructions later (DMA
//     issue, waits, barriers) and the epilogue's AGPR reads follow an explicit s_nop run (mfma_drain).
//   * phases: a K-tile is four 64 x 64 quadrants of the wave's block, 32 MFMAs each, in the order (0,0) (0,1)
//     (1,0) (1,1).  Quarters are numbered seq = 4 t + o in READ order (o: 0 A-lo, 1 B-lo, 2 B-hi, 3 A-hi) and
//     global phase g (= 4 t + p) issues the ds_reads of seq g + 2 (the fragments phase g + 1 needs) before its own
//     MFMAs, so an LDS read always has a full phase of MFMAs to land.  Fragment sets: A-lo, A-hi and two B sets
//     that swap roles every K-tile (B-lo of tile t + 1 is read into the set B-hi of tile t just released).
//   * DMA ring: one barrier per TWO phases.  Seq q's slot is free once its reads retired (lgkmcnt(0) at the end of
//     an odd phase + barrier), so phase g restages seq g + 8; the end of each odd phase g waits (counted vmcnt) for
//     seq g + 4, the last quarter the next two phases read.
//   (Round 5 removed the one-barrier-per-phase and the MFMA-interleaved read/DMA variants of this schedule, measured
//   slower on every LM shape: profiles/r4_lm_gemm.md, r4_lm_gemm_variants_vs_hipblaslt.jsonl.)
// ---------------------------------------------------------------------------------------------------------------
constexpr int NTH4 = 256;

__device__ __forceinline__ void mfma_agpr(f32x4& acc, const bf16x8& a, const bf16x8& b) {
  asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(acc) : "v"(a), "v"(b));
}

// XDL write -> VALU / memory read of the result needs up to 18 wait states; the compiler cannot see the asm MFMAs
__device__ __forceinline__ void mfma_drain() { asm volatile("s_nop 7\n\ts_nop 7\n\ts_nop 7" ::: "memory"); }

__device__ __forceinline__ void wait_vm4(int n) {  // n = DMAs allowed in flight (multiple of 4), wave-uniform
  if (n >= 24) asm volatile("s_waitcnt vmcnt(24)" ::: "memory");
  else if (n >= 20) asm volatile("s_waitcnt vmcnt(20)" ::: "memory");
  else if (n >= 16) asm volatile("s_waitcnt vmcnt(16)" ::: "memory");
  else if (n >= 12) asm volatile("s_waitcnt vmcnt(12)" ::: "memory");
  else if (n >= 8) asm volatile("s_waitcnt vmcnt(8)" ::: "memory");
  else if (n >= 4) asm volatile("s_waitcnt vmcnt(4)" ::: "memory");
  else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

template <bool AK, bool BKM, bool ACC, bool SLAB>
__global__ void __launch_bounds__(NTH4, 1) gemm256w4_kernel(Gemm256Args p) {
  extern __shared__ __attribute__((aligned(16))) char smem[];
  const int tid = threadIdx.x, lane = tid & 63;
  const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);
  const int wm = wave >> 1, wn = wave & 1;
  const int ntn = p.N / BN, ntm = p.M / BM;
  int tm, tn;
  tile_of(xcd_remap(blockIdx.x, ntm * ntn), ntm, ntn, p.group, tm, tn);
  const int m0 = tm * BM, n0 = tn * BN;
  const int kt0 = blockIdx.y * p.kt_per_split;
  const int nk = min(p.kt_per_split, p.K / BK - kt0);
  const size_t k0 = (size_t)kt0 * BK;

  const __bf16* abase = AK ? p.A + (size_t)m0 * p.lda + k0 : p.A + k0 * p.lda + m0;
  const __bf16* bbase = BKM ? p.B + (size_t)n0 * p.ldb + k0 : p.B + k0 * p.ldb + n0;
  const __amdgpu_buffer_rsrc_t ra = rsrc(abase), rb = rsrc(bbase);
  const uint32_t astep = AK ? BK * 2 : (uint32_t)(BK * p.lda * 2);
  const uint32_t bstep = BKM ? BK * 2 : (uint32_t)(BK * p.ldb * 2);

  // Quarter images: A-lo / A-hi hold rows 0-63 / 64-127 of each wave row's 128, B-lo / B-hi columns 0-63 / 64-127
  // of each wave column's 128 (tile_idx<true> for both operands).  LDS slot of kind o: buffer * BUF + o * QUARTER.
  // Per-lane source offsets of this wave's 4 pieces (wave + 4 pc) of each kind.
  uint32_t src[4][4];
#pragma unroll
  for (int pc = 0; pc < 4; ++pc) {
    src[0][pc] = src_off<true, AK>(0, wave + 4 * pc, lane, p.lda);
    src[1][pc] = src_off<true, BKM>(0, wave + 4 * pc, lane, p.ldb);
    src[2][pc] = src_off<true, BKM>(1, wave + 4 * pc, lane, p.ldb);
    src[3][pc] = src_off<true, AK>(1, wave + 4 * pc, lane, p.lda);
  }
  const int S = 4 * nk;
  // DMA of quarter seq q = 4 t + o (o compile-time after unrolling)
  auto issue = [&](auto ko, int q) {
    constexpr int O = decltype(ko)::value;
    constexpr bool ISA = O == 0 || O == 3;
    const int t = q >> 2;
    char* dst = smem + (t & 1) * BUF + O * QUARTER;
    const uint32_t koff = (uint32_t)t * (ISA ? astep : bstep);
    const __amdgpu_buffer_rsrc_t r = ISA ? ra : rb;
#pragma unroll
    for (int pc = 0; pc < 4; ++pc) glds(r, src[O][pc] + koff, dst + (wave + 4 * pc) * 1024);
  };

  f32x4 acc[8][8];  // [n tile: 8 x 16 = the wave's 128 columns][m tile: 8 x 16 = its 128 rows]
#pragma unroll
  for (int a = 0; a < 8; ++a)
#pragma unroll
    for (int b = 0; b < 8; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

  int aoff[4], boff[4];
#pragma unroll
  for (int i = 0; i < 4; ++i) {
    aoff[i] = frag_off<AK>(wm * 64, AK ? (i & 1) : i, lane);
    boff[i] = frag_off<BKM>(wn * 64, BKM ? (i & 1) : i, lane);
  }
  // one quarter's fragments for this wave: 4 tiles of 16 (rows of A or columns of B) x 2 k-steps
  auto read_q = [&](const char* img, const int (&off)[4], auto kmaj) {
    constexpr bool KM = decltype(kmaj)::value;
    FragA f;
#pragma unroll
    for (int t = 0; t < 4; ++t)
#pragma unroll
      for (int s = 0; s < 2; ++s) f.v[t][s] = KM ? ld_frag_k(img + off[s] + t * 2048) : ld_frag_t(img + off[t] + s * 8192);
    return f;
  };
  auto read_seq = [&](auto ko, int q) {
    constexpr int O = decltype(ko)::value;
    const char* img = smem + ((q >> 2) & 1) * BUF + O * QUARTER;
    if constexpr (O == 0 || O == 3) return read_q(img, aoff, IC<AK>{});
    else return read_q(img, boff, IC<BKM>{});
  };

  // prologue: seq 0 .. min(8, S) - 1 (tiles 0 and 1), read seq 0 (A-lo) and 1 (B-lo) of tile 0
  auto pro = [&](auto qc) {
    constexpr int Q = decltype(qc)::value;
    if (Q < S) issue(IC<(Q & 3)>{}, Q);
  };
  pro(IC<0>{}), pro(IC<1>{}), pro(IC<2>{}), pro(IC<3>{}), pro(IC<4>{}), pro(IC<5>{}), pro(IC<6>{}), pro(IC<7>{});
  wait_vm4(4 * (min(8, S) - 2));
  __builtin_amdgcn_s_barrier();
  FragA a_lo = read_seq(IC<0>{}, 0);
  FragA b_lo = read_seq(IC<1>{}, 1);
  FragA a_hi, b_hi;
  asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
  __builtin_amdgcn_s_barrier();
  wait_vm4(4 * (min(8, S) - 1 - 3));  // phases 0 and 1 read seq 2 and 3 after the next barrier
  __builtin_amdgcn_s_barrier();

  // One phase g = 4 kt + P: ds_reads of seq g + 2 into `nxt`, DMA of seq g + 8, the quadrant's 32 MFMAs, then
  // (odd phases) lgkmcnt(0) + vmcnt for seq g + 4 + barrier.
  auto phase = [&](auto ph, int kt, const FragA& fa, const FragA& fb, FragA& nxt, auto mi_, auto ni_) {
    constexpr int P = decltype(ph)::value, MI = decltype(mi_)::value, NI = decltype(ni_)::value;
    const int g = 4 * kt + P;
    constexpr int AHEAD = 8, RO = (P + 2) & 3, DO = (P + AHEAD) & 3;
    nxt = read_seq(IC<RO>{}, g + 2);  // past the last tile: stale LDS into a dead set, harmless
    if (g + AHEAD < S) issue(IC<DO>{}, g + AHEAD);
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int s = 0; s < 2; ++s)
#pragma unroll
      for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) mfma_agpr(acc[NI * 4 + a][MI * 4 + b], fb.v[a][s], fa.v[b][s]);
    __builtin_amdgcn_sched_barrier(0);
    if constexpr (P & 1) {  // seqs g + 3 and g + 4 are read in the next two phases
      asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
      wait_vm4(4 * (min(g + 8, S - 1) - (g + 4)));
      __builtin_amdgcn_s_barrier();
    }
  };
  // tile kt: quadrants (0,0) (0,1) (1,0) (1,1), so the last phase uses (A-hi, B-hi) and the sets the next tile's
  // first phase needs (A-lo, B-lo) are free for phases 2 and 3 to refill: every set keeps its role
  auto tile = [&](int kt) {
    phase(IC<0>{}, kt, a_lo, b_lo, b_hi, IC<0>{}, IC<0>{});  // reads B-hi(kt)
    phase(IC<1>{}, kt, a_lo, b_hi, a_hi, IC<0>{}, IC<1>{});  // reads A-hi(kt)
    phase(IC<2>{}, kt, a_hi, b_lo, a_lo, IC<1>{}, IC<0>{});  // reads A-lo(kt + 1)
    phase(IC<3>{}, kt, a_hi, b_hi, b_lo, IC<1>{}, IC<1>{});  // reads B-lo(kt + 1)
  };
#pragma unroll 1
  for (int kt = 0; kt < nk; ++kt) tile(kt);
  mfma_drain();

  const int fr = lane & 15, fq = lane >> 4;
  if (SLAB) {
#pragma unroll
    for (int nt = 0; nt < 8; ++nt)
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        const int m = m0 + wm * 128 + (mt >> 2) * 64 + (mt & 3) * 16 + fr;
        const int n = n0 + wn * 128 + (nt >> 2) * 64 + (nt & 3) * 16 + 4 * fq;
        *(f32x4*)((float*)p.C + ((size_t)blockIdx.y * p.M + m) * p.N + n) = acc[nt][mt];
      }
  } else {
#pragma unroll
    for (int np = 0; np < 4; ++np) {  // column-adjacent tile pairs (2 np, 2 np + 1): same 64-column half
      const int n8 = n0 + wn * 128 + (np >> 1) * 64 + (np & 1) * 32 + 8 * fq;
      f32x4 ba, bb;
      load_bias8(p, n8, ba, bb);
#pragma unroll
      for (int mt = 0; mt < 8; ++mt) {
        f32x4 a = acc[2 * np][mt], b = acc[2 * np + 1][mt];
        pair_permute(a, b);
        store_pair<ACC>(p, a, b, m0 + wm * 128 + (mt >> 2) * 64 + (mt & 3) * 16 + fr, n8, ba, bb);
      }
    }
  }
}

// C (bf16, ldc) = alpha * sum over splits of the fp32 slabs (+ C when accumulating); 8 elements per thread
template <bool ACC>
__global__ void __launch_bounds__(256) gemm256_reduce(const float* __restrict__ ws, __bf16* __restrict__ C, int M,
                                                      int N, int ldc, int splits, float alpha,
                                                      const float* __restrict__ bias, __bf16* __restrict__ C2) {
  const size_t i8 = (size_t)blockIdx.x * 256 + threadIdx.x;
  if (i8 >= (size_t)M * N / 8) return;
  const size_t e = i8 * 8;
  const int m = (int)(e / N), n = (int)(e % N);
  f32x4 s0 = {0.f, 0.f, 0.f, 0.f}, s1 = s0;
  const size_t slab = (size_t)M * N;
  for (int k = 0; k < splits; ++k) {
    const f32x4* src = (const f32x4*)(ws + k * slab + e);
    s0 += src[0];
    s1 += src[1];
  }
  s0 *= alpha;
  s1 *= alpha;
  if (bias != nullptr) {
    s0 += *(const f32x4*)(bias + n);
    s1 += *(const f32x4*)(bias + n + 4);
  }
  __bf16* dst = C + (size_t)m * ldc + n;
  if (ACC) {
    const uint4 o = *(const uint4*)dst;
    s0[0] += __uint_as_float(o.x << 16);
    s0[1] += __uint_as_float(o.x & 0xffff0000u);
    s0[2] += __uint_as_float(o.y << 16);
    s0[3] += __uint_as_float(o.y & 0xffff0000u);
    s1[0] += __uint_as_float(o.z << 16);
    s1[1] += __uint_as_float(o.z & 0xffff0000u);
    s1[2] += __uint_as_float(o.w << 16);
    s1[3] += __uint_as_float(o.w & 0xffff0000u);
  }
  uint4 packed;
  packed.x = pack_bf16x2(s0[0], s0[1]);
  packed.y = pack_bf16x2(s0[2], s0[3]);
  packed.z = pack_bf16x2(s1[0], s1[1]);
  packed.w = pack_bf16x2(s1[2], s1[3]);
  *(uint4*)dst = packed;
  if (!ACC && C2 != nullptr) {
    uint4 g;
    g.x = pack_bf16x2(gelu_tanh(bf16_round(s0[0])), gelu_tanh(bf16_round(s0[1])));
    g.y = pack_bf16x2(gelu_tanh(bf16_round(s0[2])), gelu_tanh(bf16_round(s0[3])));
    g.z = pack_bf16x2(gelu_tanh(bf16_round(s1[0])), gelu_tanh(bf16_round(s1[1])));
    g.w = pack_bf16x2(gelu_tanh(bf16_round(s1[2])), gelu_tanh(bf16_round(s1[3])));
    *(uint4*)(C2 + (size_t)m * ldc + n) = g;
  }
}

int g_waves = 8;  // 8: the ping-pong kernel, 4: gemm256w4_kernel (plx_gemm256_set_waves 8 / 5)

// variant: 8 = the ping-pong kernel, 5 = the 4-wave kernel, 0 = the global knob
template <bool AK, bool BKM, bool ACC, bool SLAB>
int launch(const Gemm256Args& a, int splits, hipStream_t st, int variant) {
  const dim3 grid((a.M / BM) * (a.N / BN), splits);
  const bool four = variant == 5 || (variant != 8 && g_waves == 4);
  if (four) {
    auto k = gemm256w4_kernel<AK, BKM, ACC, SLAB>;
    static const int attr =
        hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess ? 0
                                                                                                                 : -4;
    if (attr) return attr;
    hipLaunchKernelGGL(k, grid, dim3(NTH4), LDS_BYTES, st, a);
    return 0;
  }
  auto k = gemm256_kernel<AK, BKM, ACC, SLAB>;
  static const int attr =
      hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess ? 0 : -4;
  if (attr) return attr;
  hipLaunchKernelGGL(k, grid, dim3(NTH), LDS_BYTES, st, a);
  return 0;
}

template <bool AK, bool BKM>
int dispatch(const Gemm256Args& a, int splits, int accumulate, hipStream_t st, int variant) {
  if (splits > 1) return launch<AK, BKM, false, true>(a, splits, st, variant);
  return accumulate ? launch<AK, BKM, true, false>(a, 1, st, variant) : launch<AK, BKM, false, false>(a, 1, st, variant);
}

int g_group = 4;  // M-tiles per tile group (tile_of; plx_gemm256_set_group, 1 = row-major order)
int g_split_target = 256;  // blocks the split-K planner aims for (one per CU: splitting a grid that already
                           // fills the chip measured slower); plx_gemm256_set_split_target

// K-tiles per split: the most blocks (tiles x splits) up to g_split_target, every split >= 8 K-tiles and even.
// Any split count, not only powers of two: GPT-2's 36-tile MLP weight gradients took 4 splits = 144 blocks (56 % of
// the CUs) under the power-of-two rule and take 7 = 252 now; the 9-tile projection 16 -> 26 splits.
int plan_kt_per_split(int M, int N, int K) {
  const int tiles = (M / BM) * (N / BN), nk = K / BK;
  int best = nk, best_blocks = tiles;
  for (int s = 2; 2 * tiles <= g_split_target && s <= nk / 8; ++s) {
    int kps = (nk + s - 1) / s;
    kps += kps & 1;
    if (kps < 8) break;
    const int blocks = tiles * ((nk + kps - 1) / kps);
    if (blocks > g_split_target) break;
    if (blocks > best_blocks) best = kps, best_blocks = blocks;
  }
  return best;
}

// Stream-K plan for G persistent workgroups.  The partial wave of tiles (T % G; all of them when T < G) is split along
// K only when that pays: a split tile costs its pieces' fp32 partials (256 KiB each, written and read back: all
// workgroups at once, so HBM-bound -- the GPT-2 768-wide projections, 192 tiles of 12 K-tiles split in two, ran
// 0.041 ms against 0.027 unsplit, r6_lm_gemm_sk.jsonl), so only long reductions (>= 32 K-tiles) whose split saves
// >= 16 K-tiles per workgroup are split, e.g. Llama-3's 384-tile QKV forward.  Pieces are >= 4 K-tiles and, for an
// even K-tile count, even (the chained ring needs even pieces).
int g_sk_force = 0;  // 1: split every partial wave (tests: the split paths on small shapes); plx_gemm256_set_sk_force

void sk_plan(int M, int N, int K, int G, int& sk_tiles, int& ipb) {
  const int T = (M / BM) * (N / BN), nk = K / BK;
  const int rem = T % G;
  ipb = rem ? max((rem * nk + G - 1) / G, min(nk, 4)) : 1;
  if (nk % 2 == 0) ipb += ipb & 1;
  sk_tiles = rem && (g_sk_force || (nk >= 32 && nk - ipb >= 16)) ? rem : 0;
  if (!sk_tiles) ipb = 1;
}

int cu_count() {
  static int cus[64] = {0};
  int dev = 0;
  if (hipGetDevice(&dev) != hipSuccess || dev < 0 || dev >= 64) return 256;
  if (cus[dev] == 0) {
    int n = 0;
    cus[dev] = hipDeviceGetAttribute(&n, hipDeviceAttributeMultiprocessorCount, dev) == hipSuccess && n > 0 ? n : 256;
  }
  return cus[dev];
}

template <bool AK, bool BKM>
int launch_sk(const Gemm256Args& a, const SkArgs& sk, int G, hipStream_t st) {
  auto k = gemm256_sk_kernel<AK, BKM>;
  static const int attr =
      hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, LDS_BYTES) == hipSuccess ? 0 : -4;
  if (attr) return attr;
  hipLaunchKernelGGL(k, dim3(G), dim3(NTH), LDS_BYTES, st, a, sk);
  return 0;
}

}  // namespace

// fp32 workspace floats plx_gemm256_sk needs for this shape on the current device (0: no tile is split)
// (sized for any plan of the shape, so a memoised answer stays valid when plx_gemm256_set_sk_force changes)
PLX_API long long plx_gemm256_sk_ws(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return -1;
  const int G = cu_count();
  return (M / BM) * (N / BN) % G ? 2LL * G * 65536 : 0;
}

// test knob: 1 splits every partial wave of tiles along K (the split / last-arriver paths on small shapes), 0 the
// cost rule of sk_plan; returns the previous value
PLX_API int plx_gemm256_set_sk_force(int force) {
  const int prev = g_sk_force;
  g_sk_force = force ? 1 : 0;
  return prev;
}

// workgroups / stream-K tiles / iterations per workgroup of the plan (tests and the bench report it)
PLX_API int plx_gemm256_sk_plan(int M, int N, int K, int* sk_tiles, int* ipb) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return -1;
  const int G = cu_count();
  sk_plan(M, N, K, G, *sk_tiles, *ipb);
  return G;
}

// C[M][N] = alpha * A . B (+ bias) (gelu_out as plx_gemm256_exv) on the persistent stream-K kernel: one workgroup per
// CU.  K must be an even multiple of 64, >= 256 (-1 otherwise: ops/gemm.py runs the 8-wave kernel then).  ws: plx_gemm256_sk_ws floats (may be null when that is 0); tickets: >= CU-count zeroed uint32 that the kernel
// leaves zeroed (one array per device, launches on one stream at a time).  No accumulate.
// gelu_h: bf16 [M][ldc] (16-byte aligned) or null: C = bf16(alpha A.B) * gelu_tanh'(gelu_h), the GELU backward
// fused into the data gradient (not with bias / gelu_out)
PLX_API int plx_gemm256_sk(const void* A, const void* B, void* C, void* ws, void* tickets, int M, int N, int K, int lda,
                           int ldb, int ldc, int a_kmajor, int b_kmajor, float alpha, const float* bias,
                           void* gelu_out, const void* gelu_h, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return -1;
  if ((K / BK) % 2 || K / BK < 4) return -1;  // the chained ring needs an even K-tile count >= 4
  if (bias != nullptr && (uintptr_t)bias % 16) return -1;
  if (gelu_out != nullptr && (uintptr_t)gelu_out % 16) return -1;
  if (gelu_h != nullptr && ((uintptr_t)gelu_h % 16 || bias != nullptr || gelu_out != nullptr)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 8 || (uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return -1;
  const long long aspan = a_kmajor ? (long long)BM * lda * 2 : (long long)K * lda * 2;
  const long long bspan = b_kmajor ? (long long)BN * ldb * 2 : (long long)K * ldb * 2;
  if (aspan >= 0x7ffffff0LL || bspan >= 0x7ffffff0LL) return -2;
  int G = cu_count();
  SkArgs sk{(float*)ws, (unsigned*)tickets, 0, 1};
  sk_plan(M, N, K, G, sk.sk_tiles, sk.ipb);
  if (!sk.sk_tiles) G = min(G, (M / BM) * (N / BN));  // data-parallel only: no idle workgroups
  if (sk.sk_tiles && (!ws || !tickets)) return -5;
  Gemm256Args a{(const __bf16*)A, (const __bf16*)B, C, M, N, K, lda, ldb, ldc, 0, alpha, bias, gelu_out,
                g_group > 0 ? g_group : 1, (const __bf16*)gelu_h};
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if (a_kmajor && b_kmajor) rc = launch_sk<true, true>(a, sk, G, st);
  else if (a_kmajor) rc = launch_sk<true, false>(a, sk, G, st);
  else if (b_kmajor) rc = launch_sk<false, true>(a, sk, G, st);
  else rc = launch_sk<false, false>(a, sk, G, st);
  if (rc) return rc;
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Split-K plan: number of K splits (blockIdx.y) the kernel uses for this shape (1 = no workspace needed);
// the fp32 workspace must hold splits * M * N floats
PLX_API int plx_gemm256_splits(int M, int N, int K) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return 0;
  const int kps = plan_kt_per_split(M, N, K);
  return (K / BK + kps - 1) / kps;
}

// A/B knob: blocks the split-K planner aims for (0 disables splitting)
PLX_API void plx_gemm256_set_split_target(int blocks) { g_split_target = blocks; }

// A/B knob: M-tiles per tile group of the block order (1 = row-major); returns the previous value
PLX_API int plx_gemm256_set_group(int group) {
  const int prev = g_group;
  if (group >= 1 && group <= 64) g_group = group;
  return prev;
}

// A/B knob: 8 (the 8-wave ping-pong kernel) or 5 (the 4-wave AGPR-accumulator kernel, one barrier per two phases)
// for calls without a per-call variant; returns the previous value
PLX_API int plx_gemm256_set_waves(int waves) {
  const int prev = g_waves == 4 ? 5 : 8;
  if (waves == 8) g_waves = 8;
  if (waves == 5) g_waves = 4;
  return prev;
}

// C[M][N] (bf16, ldc) = alpha * A . B (+ bias[n]) (+ C when accumulate), layouts per a_kmajor / b_kmajor (see the
// file header).  bias: fp32 [N], 16-byte aligned, or null (not combined with accumulate).
// ws: fp32 workspace of plx_gemm256_splits(M, N, K) * M * N floats when that is > 1 (may be null otherwise).
// Returns 0, or < 0 on a shape / layout the kernel does not take (nothing launched).
// gelu_out: bf16 [M][ldc] (same layout as C, 16-byte aligned) receiving gelu_tanh(C), or null (not with accumulate).
// variant: the kernel schedule for this call (8 or 5: see plx_gemm256_set_waves; 0 = the global knob)
PLX_API int plx_gemm256_exv(const void* A, const void* B, void* C, void* ws, int M, int N, int K, int lda, int ldb,
                            int ldc, int a_kmajor, int b_kmajor, float alpha, int accumulate, const float* bias,
                            void* gelu_out, int variant, void* stream) {
  if (M <= 0 || N <= 0 || K <= 0 || M % BM || N % BN || K % BK) return -1;
  if (bias != nullptr && (accumulate || (uintptr_t)bias % 16)) return -1;
  if (gelu_out != nullptr && (accumulate || (uintptr_t)gelu_out % 16)) return -1;
  if (lda % 8 || ldb % 8 || ldc % 8 || (uintptr_t)A % 16 || (uintptr_t)B % 16 || (uintptr_t)C % 16) return -1;
  // largest relative byte offset a block's buffer resource sees
  const long long aspan = a_kmajor ? (long long)BM * lda * 2 : (long long)K * lda * 2;
  const long long bspan = b_kmajor ? (long long)BN * ldb * 2 : (long long)K * ldb * 2;
  if (aspan >= 0x7ffffff0LL || bspan >= 0x7ffffff0LL) return -2;
  const int kps = plan_kt_per_split(M, N, K);
  const int splits = (K / BK + kps - 1) / kps;
  if (splits > 1 && !ws) return -5;
  Gemm256Args a{(const __bf16*)A, (const __bf16*)B, splits > 1 ? ws : C, M, N, K, lda, ldb, ldc, kps, alpha, bias,
                splits > 1 ? nullptr : gelu_out, g_group > 0 ? g_group : 1};
  hipStream_t st = (hipStream_t)stream;
  int rc;
  if (a_kmajor && b_kmajor) rc = dispatch<true, true>(a, splits, accumulate, st, variant);
  else if (a_kmajor) rc = dispatch<true, false>(a, splits, accumulate, st, variant);
  else if (b_kmajor) rc = dispatch<false, true>(a, splits, accumulate, st, variant);
  else rc = dispatch<false, false>(a, splits, accumulate, st, variant);
  if (rc) return rc;
  if (splits > 1) {
    const size_t total8 = (size_t)M * N / 8;
    const dim3 grid((unsigned)((total8 + 255) / 256));
    if (accumulate)
      hipLaunchKernelGGL(gemm256_reduce<true>, grid, dim3(256), 0, st, (const float*)ws, (__bf16*)C, M, N, ldc, splits,
                         alpha, (const float*)nullptr, (__bf16*)nullptr);
    else
      hipLaunchKernelGGL(gemm256_reduce<false>, grid, dim3(256), 0, st, (const float*)ws, (__bf16*)C, M, N, ldc,
                         splits, alpha, bias, (__bf16*)gelu_out);
  }
  return hipGetLastError() == hipSuccess ? 0 : -3;
}

PLX_API int plx_gemm256_ex(const void* A, const void* B, void* C, void* ws, int M, int N, int K, int lda, int ldb,
                           int ldc, int a_kmajor, int b_kmajor, float alpha, int accumulate, const float* bias,
                           void* gelu_out, void* stream) {
  return plx_gemm256_exv(A, B, C, ws, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor, alpha, accumulate, bias, gelu_out, 0,
                         stream);
}

PLX_API int plx_gemm256_bias(const void* A, const void* B, void* C, void* ws, int M, int N, int K, int lda, int ldb,
                             int ldc, int a_kmajor, int b_kmajor, float alpha, int accumulate, const float* bias,
                             void* stream) {
  return plx_gemm256_ex(A, B, C, ws, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor, alpha, accumulate, bias, nullptr,
                        stream);
}

PLX_API int plx_gemm256(const void* A, const void* B, void* C, void* ws, int M, int N, int K, int lda, int ldb, int ldc,
                        int a_kmajor, int b_kmajor, float alpha, int accumulate, void* stream) {
  return plx_gemm256_ex(A, B, C, ws, M, N, K, lda, ldb, ldc, a_kmajor, b_kmajor, alpha, accumulate, nullptr, nullptr,
                        stream);
}

// the kernel's tile edge: M and N must be multiples of it, K of 64
PLX_API int plx_gemm256_tile() { return BM; }
