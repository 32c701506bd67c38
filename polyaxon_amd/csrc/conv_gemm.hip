// MFMA GEMMs for stride-1 1x1 convolutions on NHWC bf16 activations (ResNet-50 bottleneck conv1/conv3).
//
// On NHWC the three convolution passes are plain GEMMs over M = N*H*W pixel rows:
//   forward      y[M][Cout]  = x[M][Cin]   . W[Cout][Cin]^T       -> plx_gemm_nt   (A = x,  B = W)
//   data grad    dx[M][Cin]  = dy[M][Cout] . Wt[Cin][Cout]^T      -> plx_gemm_nt   (A = dy, B = W^T)
//   weight grad  dW[Cout][Cin] = sum_m dy[m][Cout]^T x[m][Cin]    -> plx_gemm_tn   (split over m, fp32 out)
// plx_gemm_nt needs both operands K-contiguous (row-major [rows][K]); plx_gemm_tn reads both operands
// row-major over the reduction index m and feeds the MFMA through ds_read_b64_tr_b16 transposed LDS reads.
//
// Kernel structure (cdna_hip_programming.md §5): 256 threads = 4 waves, each wave owns a WT1 x WT2 output
// sub-tile computed with v_mfma_f32_16x16x32_bf16; tiles are staged global -> LDS with 16-byte
// global_load_lds (LDS image lane-linear, bank swizzle applied on the per-lane SOURCE address and on the
// read, rule 21), double-buffered over BK = 64; blockIdx is remapped so blocks sharing an operand panel
// run on one XCD (T1, bijective form).  The NT GEMM stages through buffer-resource LDS-DMA: rows past the end
// of M and the taps of a convolution that fall outside the image get an out-of-range offset and read zeros, so
// partial tiles and padding need no branches around the DMA; the TN GEMM reads a zero page instead.
#include <hip/hip_runtime.h>

#include <stdint.h>

namespace {

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef short s16x4 __attribute__((ext_vector_type(4)));
typedef float f32x4 __attribute__((ext_vector_type(4)));
typedef __attribute__((address_space(3))) void lds_void;
typedef __attribute__((address_space(1))) const void gbl_void;

constexpr int BK = 64;          // reduction depth per LDS stage (bf16 elements)

// Implicit-GEMM geometry of a convolution on NHWC rows (1x1 or 3x3, stride 1 or 2).
// GEMM rows are pixels of a row grid (Hr x Wr per image): row m = (n*Hr + r)*Wr + c.  The reduction index is
// k = t*C + ch over `ntaps` taps; for tap t the operand row is the source pixel (r*S + offh[t], c*S + offw[t])
// of an H x W image (out-of-image -> the zero page, i.e. the zero padding), and the B operand column is
// btap[t]*C + ch (B holds all 9 (or 1) taps).  Forward / weight-gradient use S = stride, off = tap - pad;
// the stride-1 data gradient flips the taps (off = pad - tap); the stride-2 data gradient is split into the
// four (ih, iw) parity classes of the input, each a stride-1 gather over the taps of matching parity, whose
// output rows are scattered back to input pixels (2r + ph, 2c + pw) of an Hc x Wc grid (OS = 2).
struct ConvGeom {
    int H, W;        // gathered (source) image
    int Hr, Wr;      // row grid
    int C, S, ntaps;
    int Hc, Wc, OS, oph, opw;  // output-row scatter (OS == 0: row m is output row m)
    signed char offh[9], offw[9], btap[9];
    // per-tap byte offsets for the NT GEMM's staging (filled by finish_geom): A row shift (offh*W + offw)*C*2
    // and B column start btap*C*2 -- dword arrays so a uniform tap index reads them with scalar loads
    int tap_a[9], tap_b[9];
    // x / Wr and q / Hr as __umulhi(x, m): m = floor(2^32 / d) + 1 is exact while x * d < 2^32, which holds for
    // pixel indices (< 2^24) and row-grid sides (<= 255); m = 0 marks d == 1
    uint32_t mWr, mHr;
    // the taps factored into <= 3 distinct row offsets hv x <= 3 column offsets wv; pat[i * 3 + j] = bit set of
    // the taps at (hv[i], wv[j]): a row's in-image tap mask is 6 compares and 9 selects (NT GEMM staging)
    int nh, nw, hv[3], wv[3];
    uint32_t pat[9];
    // reduction order of the NT GEMM's stages: 0 tap-major (k = t * C + ch, tap outer), 1 tap-inner (all taps of a
    // 64-channel chunk back to back: the shifted A rows of consecutive stages overlap and are re-read from L1)
    int tap_inner;
};

// v[t] for a wave-uniform runtime t < 9 as a select chain: indexing the by-value ConvGeom's arrays with a runtime
// index made hipcc copy the struct to scratch and reload from it per stage (a VMEM load whose wait, vmcnt(0), also
// drained every LDS-DMA in flight)
__device__ __forceinline__ int pick9(const int (&v)[9], int t) {
    int r = v[0];
#pragma unroll
    for (int i = 1; i < 9; ++i) r = t == i ? v[i] : r;
    return r;
}

inline uint32_t div_magic(int d) { return d <= 1 ? 0u : (uint32_t)((1ull << 32) / (unsigned)d + 1); }

inline ConvGeom finish_geom(ConvGeom g) {
    g.nh = g.nw = 0;
    for (int i = 0; i < 9; ++i) g.pat[i] = 0;
    for (int t = 0; t < 9; ++t) {
        g.tap_a[t] = t < g.ntaps ? (g.offh[t] * g.W + g.offw[t]) * g.C * 2 : 0;
        g.tap_b[t] = t < g.ntaps ? g.btap[t] * g.C * 2 : 0;
        if (t >= g.ntaps) continue;
        int i = 0, j = 0;
        while (i < g.nh && g.hv[i] != g.offh[t]) ++i;
        if (i == g.nh) g.hv[g.nh++] = g.offh[t];
        while (j < g.nw && g.wv[j] != g.offw[t]) ++j;
        if (j == g.nw) g.wv[g.nw++] = g.offw[t];
        g.pat[i * 3 + j] |= 1u << t;
    }
    g.mWr = div_magic(g.Wr);
    g.mHr = div_magic(g.Hr);
    return g;
}

// BatchNorm-backward channel reduction fused into a data-gradient GEMM's epilogue.  The GEMM's output C is
// dy of a BatchNorm(+ReLU) whose input x (same [rows][ldc] layout as C) and 1-bit ReLU mask the forward kept;
// the epilogue adds per-block partials of  sum dz  and  sum dz * (x - mean) * invstd  (dz = dy * mask) to
// part[blk_off + tm][n] and part[part_ld + blk_off + tm][n], so the BatchNorm backward skips its reduce pass
// (one full read of dy) -- the same hand-off the forward does with its channel stats.
struct BnBwd {
    const __bf16* x;
    const uint8_t* mask;   // nullptr: no ReLU
    const float* mean;
    const float* invstd;
    float* part;           // nullptr: disabled
    int part_ld, blk_off;
    // skip_w > 0 (dense GEMM rows = pixels of [n][skip_h][skip_w] images): rows of even-even pixels add nothing --
    // a strided 1x1 data gradient adds to exactly those pixels afterwards and reduces their final values itself
    // (ResNet downsampling block: conv1's dgrad here, the downsample conv's in the rows from blk_off on)
    int skip_h, skip_w;
};

__device__ __forceinline__ void row_coords(int m, int Hr, int Wr, int& n, int& r, int& c) {
    const int q = m / Wr;
    c = m - q * Wr;
    n = q / Hr;
    r = q - n * Hr;
}

// row_coords with the host-computed magic divisors (ConvGeom::mWr / mHr): 2 multiply-highs instead of 2 divisions
__device__ __forceinline__ void row_coords(int m, const ConvGeom& g, int& n, int& r, int& c) {
    const int q = g.mWr ? (int)__umulhi((uint32_t)m, g.mWr) : m;
    c = m - q * g.Wr;
    n = g.mHr ? (int)__umulhi((uint32_t)q, g.mHr) : q;
    r = q - n * g.Hr;
}

__device__ __forceinline__ size_t out_row(const ConvGeom& g, int m) {
    if (g.OS == 0) return (size_t)m;
    int n, r, c;
    row_coords(m, g.Hr, g.Wr, n, r, c);
    return ((size_t)n * g.Hc + r * g.OS + g.oph) * g.Wc + c * g.OS + g.opw;
}
constexpr int NTHREADS = 256;   // 4 waves

// vmcnt(n) with a run-time n in [0, 4 * step] in multiples of `step` (the counter is an instruction immediate)
template <int STEP>
__device__ __forceinline__ void wait_vm_stages(int stages) {
    if (stages >= 4 && 4 * STEP <= 63) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(4 * STEP < 63 ? 4 * STEP : 63) : "memory");
    else if (stages >= 3) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(3 * STEP) : "memory");
    else if (stages == 2) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(2 * STEP) : "memory");
    else if (stages == 1) asm volatile("s_waitcnt vmcnt(%0)" ::"n"(STEP) : "memory");
    else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
}

__device__ __forceinline__ int xcd_remap(int bid, int nwg) {
    // consecutive logical ids on one XCD (blocks are dealt round-robin over the 8 XCDs); bijective for any nwg
    const int xcd = bid & 7, q = nwg >> 3, r = nwg & 7;
    const int base = xcd < r ? xcd * (q + 1) : r * (q + 1) + (xcd - r) * q;
    return base + (bid >> 3);
}

__device__ __forceinline__ void glds16(const void* g, void* l) {
    __builtin_amdgcn_global_load_lds((gbl_void*)g, (lds_void*)l, 16, 0, 0);
}

// LDS-DMA through a buffer resource: base and range live in SGPRs, each lane supplies a 32-bit byte offset, and an
// offset at or past the range (OOB) returns zeros -- the zero padding of a convolution costs one select, no
// zero page and no 64-bit address math.  Operands here are < 2 GiB, so the range is 2^31 bytes.
constexpr uint32_t OOB = 0x80000000u;

__device__ __forceinline__ __amdgpu_buffer_rsrc_t buf_rsrc(const void* base) {
    return __builtin_amdgcn_make_buffer_rsrc(const_cast<void*>(base), 0, (int)OOB, 0x00020000);
}

__device__ __forceinline__ void blds16(__amdgpu_buffer_rsrc_t r, uint32_t off, void* l) {
    __builtin_amdgcn_raw_ptr_buffer_load_lds(r, (lds_void*)l, 16, off, 0, 0, 0);
}

// round to nearest even with the hardware conversion (v_cvt_pk_bf16_f32: one instruction per pair, NaN-preserving)
__device__ __forceinline__ uint32_t pack_bf16x2(float a, float b) {
    return (uint32_t)__builtin_bit_cast(uint16_t, (__bf16)a) | ((uint32_t)__builtin_bit_cast(uint16_t, (__bf16)b) << 16);
}

// ------------------------------------------------------------------------------------------- NT GEMM
// C[M][N] (bf16, ldc) = A[M][K] (lda) . B[N][K]^T (ldb).  N % BN == 0, K % 64 == 0 (host-checked).
// LDS row = 64 bf16 = 128 B = 8 chunks of 16 B; physical chunk = logical ^ ((row >> 1) & 7), which puts the
// 16 rows of a fragment read on 16 distinct bank slots.
__device__ __forceinline__ int nt_swz(int row) { return (row >> 1) & 7; }

// NBUF = 2: double-buffered K stages (2 blocks per CU); NBUF = 1: one stage buffer (stage, wait, compute, barrier)
// and 4 blocks per CU, whose interleaving hides the staging instead (MINB = blocks per CU the registers allow)
// BWD: the data-gradient epilogue (D add, ReLU-masked D, BatchNorm-backward partials); !BWD: the forward one (channel
// stats).  Compile-time so each kernel only holds the epilogue registers it uses.
// MODE: 0 dense rows, 1 implicit-GEMM convolution (ConvGeom gather), 2 the ResNet stem (see plx_stem_conv_fwd).
// (Round 6 removed the halo mode (3: input rows staged once per channel chunk for all 9 taps; 0.99-1.17x the gather
// mode's time, profiles/r3_negative_results.md) and the BatchNorm-apply prologue prototype (4: -159 us per step,
// profiles/r5_bn_fusion_bound.md).  Round 5 removed the 8-wave 3-stage ring variant (NBUF 3) and the 4-5 stage software pipeline (NBUF 4-5): both
// measured slower in the training step than these lock-step kernels, profiles/r4_conv3x3_scratch_fix_ring_ab.jsonl,
// r4_conv3x3_swp_ab.jsonl, r4_bench_swp4_conv.json.)
template <int BM, int BN, int WGM, int WGN, int MODE, int MINB = 2, int NBUF = 2, bool BWD = false, int NTH = NTHREADS>
__global__ void __launch_bounds__(NTH, MINB)
gemm_nt_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B, __bf16* __restrict__ C,
               int M, int N, int K, int lda, int ldb, int ldc, const __bf16* __restrict__ zero,
               float* __restrict__ stats, ConvGeom geo, const __bf16* __restrict__ D, int ldd, BnBwd bnr,
               const uint8_t* __restrict__ dmask) {
    constexpr bool CONV = MODE == 1, STEM = MODE == 2;
    static_assert(MODE >= 0 && MODE <= 2, "dense, gather or stem");
    constexpr int NW = NTH / 64;                           // waves
    static_assert(WGM * WGN == NW, "one wave per wave tile");
    static_assert(NTH == 256 && NBUF >= 1 && NBUF <= 2, "4-wave kernels, one or two K stages");
    constexpr int WTM = BM / WGM, WTN = BN / WGN;          // wave tile
    constexpr int RM = WTM / 16, RN = WTN / 16;            // 16x16 MFMA repeats
    constexpr int A_BYTES = BM * BK * 2, B_BYTES = BN * BK * 2, STAGE = A_BYTES + B_BYTES;
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: LDS-DMA destinations (M0) stay scalar
    const int ntn = N / BN, ntm = (M + BM - 1) / BM;
    const int id = xcd_remap(blockIdx.x, ntm * ntn);
    const int tn = id % ntn, tm = id / ntn;
    const int m0 = tm * BM, n0 = tn * BN;
    const int wm = wave / WGN, wn = wave % WGN;

    // Staging addresses, fixed over the whole k loop: each A row this thread stages gets its element offset
    // (with the lane's swizzled 16-B chunk folded in) and, in conv mode, a bit per tap saying whether that tap's
    // source pixel is inside the image (else the zero page is read: the zero padding).  A stage then costs one
    // bit test, one add and a select per row -- the per-stage bounds checks and 64-bit address math were ~20
    // VALU per row and, beside 32 MFMAs per wave and stage, set the loop's pace.
    constexpr int AI = BM / (8 * NW), BI = BN / (8 * NW);  // LDS-DMA instructions per wave per stage (A, B)
    int a_off[AI];                                          // byte offsets
    uint32_t a_ok[AI];
#pragma unroll
    for (int i = 0; i < AI; ++i) {
        const int row = (i * NW + wave) * 8 + (lane >> 3);
        const int lc = (lane & 7) ^ nt_swz(row);
        const int gm = m0 + row;
        if constexpr (CONV) {
            int n, r, c;
            row_coords(gm, geo, n, r, c);
            const int ih0 = r * geo.S, iw0 = c * geo.S;
            a_off[i] = (((n * geo.H + ih0) * geo.W + iw0) * lda + lc * 8) * 2;
            uint32_t ok = 0;
#pragma unroll
            for (int hi = 0; hi < 3; ++hi) {
                const bool vh = hi < geo.nh && (unsigned)(ih0 + geo.hv[hi]) < (unsigned)geo.H;
#pragma unroll
                for (int wj = 0; wj < 3; ++wj) {
                    const bool vw = wj < geo.nw && (unsigned)(iw0 + geo.wv[wj]) < (unsigned)geo.W;
                    ok |= (vh && vw) ? geo.pat[hi * 3 + wj] : 0u;
                }
            }
            a_ok[i] = gm < M ? ok : 0u;
        } else if constexpr (STEM) {
            // row = output pixel (n, r, c); A row chunk t (16 B) = super-pixel (2r - 3 + t / 4, c - 2 + t % 4) of the
            // packed input (2 pixels x 4 channels); stage s stages chunk t = 8 s + lc, bit s says it is in the image
            int n, r, c;
            row_coords(gm, geo, n, r, c);
            const int ih0 = 2 * r - 3, sc0 = c - 2;
            a_off[i] = ((n * geo.H + ih0) * geo.W + sc0) * 16;
            uint32_t ok = 0;
#pragma unroll
            for (int st = 0; st < 4; ++st) {
                const int t = st * 8 + lc;
                ok |= (t < 28 && (unsigned)(ih0 + (t >> 2)) < (unsigned)geo.H && (unsigned)(sc0 + (t & 3)) < (unsigned)geo.W)
                          ? 1u << st : 0u;
            }
            a_ok[i] = gm < M ? ok : 0u;
        } else {
            a_off[i] = (gm * lda + lc * 8) * 2;
            a_ok[i] = gm < M ? 1u : 0u;
        }
    }
    int b_off[BI];
#pragma unroll
    for (int i = 0; i < BI; ++i) {
        const int row = (i * NW + wave) * 8 + (lane >> 3);
        b_off[i] = ((n0 + row) * ldb + ((lane & 7) ^ nt_swz(row)) * 8) * 2;
    }
    const __amdgpu_buffer_rsrc_t ra = buf_rsrc(A), rb = buf_rsrc(B);

    // staging: each wave instruction moves 1024 B = 8 rows x 8 chunks.  (t, c0): tap and channel offset of
    // reduction index k0 = t * C + c0 (conv mode; t = 0, c0 = k0 otherwise)
    auto stage_a = [&](int buf, int k0, int t, int c0) {
        char* base = smem + buf * STAGE;
        int a_add = k0 * 2, bit = 0;
        if constexpr (CONV) {                               // lda == C in conv mode
            a_add = pick9(geo.tap_a, t) + c0 * 2;
            bit = t;
        }
        if constexpr (STEM) bit = k0 / BK;
#pragma unroll
        for (int i = 0; i < AI; ++i) {                      // A: BM rows / 8 rows per instr / NW waves
            if constexpr (STEM) {                           // this lane's chunk = tap t of the 7 x 4 super-pixel window
                const int t = bit * 8 + ((lane & 7) ^ nt_swz((i * NW + wave) * 8 + (lane >> 3)));
                a_add = ((t >> 2) * geo.W + (t & 3)) * 16;
            }
            const uint32_t off = (a_ok[i] >> bit) & 1u ? (uint32_t)(a_off[i] + a_add) : OOB;
            blds16(ra, off, base + (i * NW + wave) * 1024);
        }
    };
    auto stage_b = [&](int buf, int k0, int t, int c0) {
        char* base = smem + buf * STAGE;
        const int bk0 = CONV ? pick9(geo.tap_b, t) + c0 * 2 : k0 * 2;
#pragma unroll
        for (int i = 0; i < BI; ++i) blds16(rb, (uint32_t)(b_off[i] + bk0), base + A_BYTES + (i * NW + wave) * 1024);
    };
    auto stage = [&](int buf, int k0, int t, int c0) {
        stage_a(buf, k0, t, c0);
        stage_b(buf, k0, t, c0);
    };

    f32x4 acc[RN][RM];
#pragma unroll
    for (int a = 0; a < RN; ++a)
#pragma unroll
        for (int b = 0; b < RM; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int fr = lane & 15, fq = lane >> 4;
    const int nk = K / BK;
    const int cdim = CONV ? geo.C : K;                      // channels per tap
    int st = 0, sc = 0;                                     // (tap, channel offset) of the next stage
    const bool tap_inner = CONV && geo.tap_inner;           // uniform
    auto advance = [&]() {                                  // selects, no branches (see the ring loop's advance)
        const bool wt = st + 1 == geo.ntaps, wc = sc + BK == cdim;
        const int st_i = wt ? 0 : st + 1, sc_i = wt ? sc + BK : sc;
        const int st_m = wc ? st + 1 : st, sc_m = wc ? 0 : sc + BK;
        st = tap_inner ? st_i : st_m;
        sc = tap_inner ? sc_i : sc_m;
    };
    stage(0, 0, 0, 0);
    advance();
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    for (int kt = 0; kt < nk; ++kt) {
        const int cur = NBUF == 2 ? kt & 1 : 0;
        if (NBUF == 1 && kt > 0) {                          // restage the single buffer (the loop's tail barrier
            stage(0, kt * BK, st, sc);                      // retired its readers)
            advance();
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
        if (NBUF == 2 && kt + 1 < nk) {
            stage(cur ^ 1, (kt + 1) * BK, st, sc);
            advance();
        }
        const char* As = smem + cur * STAGE;
        const char* Bs = As + A_BYTES;
#pragma unroll
        for (int kk = 0; kk < 2; ++kk) {                    // two 32-deep MFMA steps per stage
            bf16x8 fa[RN], fb[RM];
#pragma unroll
            for (int rn = 0; rn < RN; ++rn) {               // MFMA A operand = B rows (output channel n)
                const int row = wn * WTN + rn * 16 + fr;
                const int pc = (kk * 4 + fq) ^ nt_swz(row);
                fa[rn] = *(const bf16x8*)(Bs + row * 128 + pc * 16);
            }
#pragma unroll
            for (int rm = 0; rm < RM; ++rm) {               // MFMA B operand = A rows (pixel m)
                const int row = wm * WTM + rm * 16 + fr;
                const int pc = (kk * 4 + fq) ^ nt_swz(row);
                fb[rm] = *(const bf16x8*)(As + row * 128 + pc * 16);
            }
#pragma unroll
            for (int rn = 0; rn < RN; ++rn)
#pragma unroll
                for (int rm = 0; rm < RM; ++rm)
                    acc[rn][rm] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[rn], fb[rm], acc[rn][rm], 0, 0, 0);
        }
        if (NBUF == 2) asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
    }
    // Epilogue through LDS (the k-loop's last barrier freed it): D[n][m] has column m = fr and rows
    // n = 4*fq + r in each lane, i.e. 4 consecutive channels of one pixel.  Stage the bf16 tile as [m][n] rows
    // padded by 16 B, then store whole output rows with 16 B per lane (a wave instruction writes contiguous
    // row segments instead of 32-B pieces of 16 different rows).  Thread tid owns chunk column tid % CHUNKS of
    // rows tid / CHUNKS + it * RSTEP; the epilogue's global operands (D, and x / mask of the fused BatchNorm
    // backward) are loaded for all of its rows BEFORE the tile is staged, so their latency hides behind the LDS
    // pass (rows past M are clamped to a valid row and discarded: no per-row branch around a load).
    constexpr int CROW = BN * 2 + 16;
    constexpr int CHUNKS = BN / 8;                          // 16-B chunks per output row
    static_assert(NTH % CHUNKS == 0, "a thread keeps one chunk column over the store loop");
    constexpr int RSTEP = NTH / CHUNKS, ITERS = BM / RSTEP;
    const int rows = min(BM, M - m0);
    const int cc = tid % CHUNKS, r0 = tid / CHUNKS;
    const int ch0 = n0 + cc * 8;                            // this thread's 8 channels
    const bool bnr_on = BWD && bnr.part != nullptr;
    const bool stats_on = !BWD && stats != nullptr;
    const bool d_on = BWD && D != nullptr;
    int orow[ITERS];                                        // output pixel rows (< 2^31)
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        const int gm = min(m0 + r0 + it * RSTEP, M - 1);
        if constexpr (CONV) orow[it] = (int)out_row(geo, gm);
        else orow[it] = gm;
    }
    auto tile_to_lds = [&]() {
#pragma unroll
        for (int rm = 0; rm < RM; ++rm) {
            const int ml = wm * WTM + rm * 16 + fr;
#pragma unroll
            for (int rn = 0; rn < RN; ++rn) {
                const int nl = wn * WTN + rn * 16 + fq * 4;
                const f32x4 v = acc[rn][rm];
                uint2 packed;
                packed.x = pack_bf16x2(v[0], v[1]);
                packed.y = pack_bf16x2(v[2], v[3]);
                *(uint2*)(smem + ml * CROW + nl * 2) = packed;
            }
        }
    };
    // LATE: the single-buffer data-gradient kernel parks the accumulators in LDS BEFORE it issues the epilogue
    // loads, so they do not hold 64 VGPRs through the loads' latency (other resident blocks hide it instead)
    constexpr bool LATE = BWD && NBUF == 1;
    if constexpr (LATE) tile_to_lds();
    uint4 dpre[ITERS], xpre[ITERS];
    uint32_t mpre[ITERS], dmpre[ITERS];
    if (d_on) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) dpre[it] = *(const uint4*)(D + (size_t)orow[it] * ldd + ch0);
        // dmask: D is a ReLU's incoming gradient and this bit mask (1 bit per element, ldd == N) its forward
        // mask -- the residual gradient dz = D * mask is formed here instead of being written out by the ReLU's
        // backward and read back
        if (dmask != nullptr) {
#pragma unroll
            for (int it = 0; it < ITERS; ++it) dmpre[it] = dmask[((size_t)orow[it] * ldd + ch0) >> 3];
        }
    }
    float sa[8], sb[8], mu[8], is[8];
    float s1[8], s2[8];                                     // channel stats of this thread's rows (stats_on)
#pragma unroll
    for (int k = 0; k < 8; ++k) s1[k] = s2[k] = 0.f;
    if (bnr_on) {
#pragma unroll
        for (int it = 0; it < ITERS; ++it) xpre[it] = *(const uint4*)(bnr.x + (size_t)orow[it] * ldc + ch0);
        if (bnr.mask != nullptr) {
#pragma unroll
            for (int it = 0; it < ITERS; ++it) mpre[it] = bnr.mask[((size_t)orow[it] * ldc + ch0) >> 3];
        } else {
#pragma unroll
            for (int it = 0; it < ITERS; ++it) mpre[it] = 0xffu;
        }
        if (bnr.skip_w > 0) {
#pragma unroll
            for (int it = 0; it < ITERS; ++it) {
                const int gm = m0 + r0 + it * RSTEP, q = gm / bnr.skip_w;
                if (((gm - q * bnr.skip_w) | (q % bnr.skip_h)) % 2 == 0) mpre[it] = 0u;
            }
        }
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            sa[k] = sb[k] = 0.f;
            mu[k] = bnr.mean[ch0 + k];
            is[k] = bnr.invstd[ch0 + k];
        }
    }
    if constexpr (!LATE) tile_to_lds();
    __syncthreads();
#pragma unroll
    for (int it = 0; it < ITERS; ++it) {
        const int r = r0 + it * RSTEP;
        if (r >= rows) break;
        uint4 v = *(const uint4*)(smem + r * CROW + cc * 16);
        if (stats_on) {
            // sums / sums of squares of the bf16-rounded product (before any D), from the 8 channels in hand
            const uint32_t* pv = (const uint32_t*)&v;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float lo = __uint_as_float(pv[j] << 16), hi = __uint_as_float(pv[j] & 0xffff0000u);
                s1[2 * j] += lo;
                s1[2 * j + 1] += hi;
                s2[2 * j] = fmaf(lo, lo, s2[2 * j]);
                s2[2 * j + 1] = fmaf(hi, hi, s2[2 * j + 1]);
            }
        }
        if (d_on) {
            // C = A.B^T + D (a second gradient into the same tensor, e.g. the residual branch's): added in fp32
            // and rounded once, instead of a separate bf16 add pass over both tensors.  D is indexed like C, so
            // D == C (in place) is allowed.
            uint32_t* pv = (uint32_t*)&v;
            const uint32_t* pd = (const uint32_t*)&dpre[it];
            const uint32_t db = dmask != nullptr ? dmpre[it] : 0xffu;
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float d0 = (db >> (2 * j)) & 1u ? __uint_as_float(pd[j] << 16) : 0.f;
                const float d1 = (db >> (2 * j + 1)) & 1u ? __uint_as_float(pd[j] & 0xffff0000u) : 0.f;
                const float lo = __uint_as_float(pv[j] << 16) + d0;
                const float hi = __uint_as_float(pv[j] & 0xffff0000u) + d1;
                pv[j] = pack_bf16x2(lo, hi);
            }
        }
        *(uint4*)(C + (size_t)orow[it] * ldc + ch0) = v;
        if (bnr_on) {
            const uint32_t mb = mpre[it];
            const uint32_t* pv = (const uint32_t*)&v;
            const uint32_t* px = (const uint32_t*)&xpre[it];
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                const float g0 = (mb >> (2 * j)) & 1u ? __uint_as_float(pv[j] << 16) : 0.f;
                const float g1 = (mb >> (2 * j + 1)) & 1u ? __uint_as_float(pv[j] & 0xffff0000u) : 0.f;
                const float x0 = __uint_as_float(px[j] << 16), x1 = __uint_as_float(px[j] & 0xffff0000u);
                sa[2 * j] += g0;
                sa[2 * j + 1] += g1;
                sb[2 * j] = fmaf(g0, (x0 - mu[2 * j]) * is[2 * j], sb[2 * j]);
                sb[2 * j + 1] = fmaf(g1, (x1 - mu[2 * j + 1]) * is[2 * j + 1], sb[2 * j + 1]);
            }
        }
    }
    // Per-channel partials of this block's rows: the RSTEP threads sharing a chunk column each hold 16 values
    // (8 channels x 2 sums).  They go through LDS over the staged tile (rows of 17 floats: conflict-free both
    // ways) and every thread then sums ONE (chunk column, value) pair over the RSTEP rows -- 16 loads per thread
    // instead of 16 threads each walking 15 x 16 dependent loads while the rest of the block waits.
    auto reduce_store = [&](const float* va, const float* vb, float* dst_a, float* dst_b) {
        float* red = (float*)smem;                          // [NTH][17], over the staged tile: its reads
        __syncthreads();                                    // (the store loop) must be done
#pragma unroll
        for (int k = 0; k < 8; ++k) {
            red[tid * 17 + k] = va[k];
            red[tid * 17 + 8 + k] = vb[k];
        }
        __syncthreads();
        if (tid < CHUNKS * 16) {
            const int c = tid % CHUNKS, v = tid / CHUNKS;
            float sum = 0.f;
#pragma unroll 4
            for (int j = 0; j < RSTEP; ++j) sum += red[(j * CHUNKS + c) * 17 + v];
            if (v < 8) dst_a[c * 8 + v] = sum;
            else dst_b[c * 8 + v - 8] = sum;
        }
        __syncthreads();                                    // red is reused by the next reduction
    };
    // Partial rows are in units of SROWS pixel rows (plx_gemm_nt_rows_per_block(N): 128 for N % 128 == 0, else 256)
    // whatever the tile height, so the host sizes them without knowing the tile; a taller block writes its partial
    // into its first row and zeros into the others.
    constexpr int SROWS = BN % 128 == 0 ? 128 : 256, SPB = BM / SROWS;
    static_assert(SPB >= 1 && BM % SROWS == 0, "block height must be a multiple of the stats row height");
    const int srow = m0 / SROWS, nsr = (M + SROWS - 1) / SROWS;
    auto zero_rows = [&](float* base_a, float* base_b, int ld) {  // rows srow+1 .. srow+SPB-1 (those < nsr)
        if constexpr (SPB > 1) {
            for (int i = tid; i < (SPB - 1) * BN; i += NTH) {
                const int r = srow + 1 + i / BN, c = i % BN;
                if (r < nsr) {
                    base_a[(size_t)(r - srow) * ld + c] = 0.f;
                    base_b[(size_t)(r - srow) * ld + c] = 0.f;
                }
            }
        }
    };
    if (bnr_on) {
        float* pa = bnr.part + (size_t)(bnr.blk_off + srow) * ldc + n0;
        float* pb = bnr.part + (size_t)(bnr.part_ld + bnr.blk_off + srow) * ldc + n0;
        reduce_store(sa, sb, pa, pb);
        zero_rows(pa, pb, ldc);
    }
    // per-channel partial sum / sum of squares -> stats[0][srow][n], stats[1][srow][n] (the BatchNorm that consumes
    // this conv skips its stats pass)
    if (stats_on) {
        float* pa = stats + (size_t)srow * N + n0;
        float* pb = stats + (size_t)(nsr + srow) * N + n0;
        reduce_store(s1, s2, pa, pb);
        zero_rows(pa, pb, N);
    }
}

// ------------------------------------------------------------------------------------------- TN GEMM
// W[slice][N1][N2] (fp32 slab per m-slice, ld = N2) = sum_{m in slice} A[m][N1] (lda) * B[m][N2] (ldb).
// The slabs are summed by slab_partial_kernel / slab_final_kernel (the guide's slab reducer).  The first version accumulated with
// per-element fp32 atomics instead; on the 7x7 layers (16 slices into one 4 MB output) its weight gradient ran
// at half the forward GEMM's rate.
// LDS images are [BK rows = m][BNx cols] in natural row order; MFMA fragments come from ds_read_b64_tr_b16
// (T10): lane 4q+p of a 16-lane group addresses row kb+q, columns c0+4p..4p+3 and receives column (lane&15)
// of those 4 rows.  Physical 16-B chunk = logical ^ tr_swz(row) makes both 32-lane halves conflict-free.
template <int ROWB>
__device__ __forceinline__ int tr_swz(int row) {
    if constexpr (ROWB >= 256) return 2 * ((row & 3) | (((row >> 3) & 1) << 2));
    else return 2 * (((row >> 1) & 1) | (((row >> 3) & 1) << 1));
}

template <int ROWB>
__device__ __forceinline__ s16x4 tr_read(const char* img, int row, int col /* element */) {
    const int lc = col >> 3, half = (col >> 2) & 1;
    const int pc = lc ^ tr_swz<ROWB>(row);
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (__attribute__((address_space(3))) s16x4*)(img + row * ROWB + pc * 16 + half * 8));
}

// 32-bit LDS address of a pointer into the dynamic LDS (for inline-asm ds instructions)
__device__ __forceinline__ uint32_t lds_addr(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) char*)p;
}

// ds_read_b64_tr_b16 the compiler cannot see (no waitcnt inserted for it; the caller waits lgkmcnt itself)
__device__ __forceinline__ s16x4 ds_tr(uint32_t addr) {
    s16x4 r;
    asm volatile("ds_read_b64_tr_b16 %0, %1" : "=v"(r) : "v"(addr) : "memory");
    return r;
}

// GATHER: 0 dense rows, 1 the pixel shifted by (dh, dw) (3x3 weight gradient), 2 the stem's packed super-pixel
// window: chunk k / 8 of row (n, r, c) is super-pixel (2r - 3 + t / 4, c - 2 + t % 4), t = k / 8 (plx_stem_conv_fwd)
template <int ROWB, int GATHER = 0, int BKR = BK>
__device__ __forceinline__ void stage_rows(char* img, __amdgpu_buffer_rsrc_t rsrc, int ld, int r0, int rend, int c0,
                                           int wave, int lane, const ConvGeom* geo = nullptr, int dh = 0, int dw = 0) {
    // BKR rows x ROWB bytes, lane-linear image; 1024 B per wave instruction, through buffer-resource LDS-DMA (rows
    // past rend and gathered pixels outside the image get an out-of-range offset: zeros).  GATHER: row gr is the
    // pixel shifted by (dh, dw), for the weight gradient of a 3x3 convolution.
    constexpr int INSTR = BKR * ROWB / 1024;
    static_assert(INSTR % 4 == 0, "a stage splits evenly over the 4 waves");
#pragma unroll
    for (int i = 0; i < INSTR / 4; ++i) {
        const int off = (i * 4 + wave) * 1024 + lane * 16;
        const int row = off / ROWB, pc = (off % ROWB) >> 4;
        const int lc = pc ^ tr_swz<ROWB>(row);
        const int gr = r0 + row;
        uint32_t boff;
        if constexpr (GATHER == 2) {
            int n, r, c;
            row_coords(gr, *geo, n, r, c);
            const int t = (c0 >> 3) + lc, ih = 2 * r - 3 + (t >> 2), sc = c - 2 + (t & 3);
            const bool ok = gr < rend && t < 28 && (unsigned)ih < (unsigned)geo->H && (unsigned)sc < (unsigned)geo->W;
            boff = ok ? (uint32_t)(((n * geo->H + ih) * geo->W + sc) * 16) : OOB;
        } else if constexpr (GATHER == 1) {
            int n, r, c;
            row_coords(gr, *geo, n, r, c);
            const int ih = r * geo->S + dh, iw = c * geo->S + dw;
            const bool ok = gr < rend && (unsigned)ih < (unsigned)geo->H && (unsigned)iw < (unsigned)geo->W;
            boff = ok ? (uint32_t)(((((n * geo->H + ih) * geo->W + iw) * ld) + c0 + lc * 8) * 2) : OOB;
        } else {
            boff = gr < rend ? (uint32_t)((gr * ld + c0 + lc * 8) * 2) : OOB;
        }
        blds16(rsrc, boff, img + (i * 4 + wave) * 1024);
    }
}


// CONV: 0 dense, 1 3x3 gather (tap per N2 tile), 2 the stem's super-pixel window (plx_stem_conv_wgrad)
// NST: K-stages in the LDS ring.  2 = double buffering (stage k+1 in flight while k computes, vmcnt(0) + barrier
// per stage); 3-4 = a ring with NST-1 stages in flight behind a counted vmcnt.  A stage is 32 KB for a 128x128 tile
// and takes longer to land by LDS-DMA (~1.5 us incl. latency) than its 32 MFMAs per wave take to run (~0.2 us),
// so with one block per CU (the side-stream plan) the double-buffered loop mostly waited on its own fills.
// BKT: reduction rows per stage (64, or 32: half-size stages, so a 4-deep ring fits the double buffer's 64 KB)
template <int BN1, int BN2, int WG1, int WG2, int CONV, int NST = 2, int BKT = BK>
__global__ void __launch_bounds__(NTHREADS, NST * BKT <= 2 * BK ? 2 : 1)
gemm_tn_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B, float* __restrict__ W,
               int M, int N1, int N2, int lda, int ldb, int kchunk, const __bf16* __restrict__ zero,
               ConvGeom geo) {
    constexpr int WT1 = BN1 / WG1, WT2 = BN2 / WG2, R1 = WT1 / 16, R2 = WT2 / 16;
    constexpr int ROWA = BN1 * 2, ROWB_ = BN2 * 2;
    constexpr int A_BYTES = BKT * ROWA, STAGE = BKT * (ROWA + ROWB_);
    constexpr int PER_STAGE = (BKT * ROWA / 1024 + BKT * ROWB_ / 1024) / 4;  // LDS-DMA instructions per wave per stage
    static_assert(BKT == 64 || BKT == 32, "32- or 64-row stages");
    static_assert(NST >= 2 && NST <= 4, "2-4 stages");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // uniform: LDS-DMA destinations (M0) stay scalar
    const int nt1 = N1 / BN1, nt2 = N2 / BN2, ntiles = nt1 * nt2;
    const int nslices = (M + kchunk - 1) / kchunk;
    const int id = xcd_remap(blockIdx.x, ntiles * nslices);
    const int tile = id % ntiles, slice = id / ntiles;
    const int t1 = tile / nt2, t2 = tile % nt2;
    const int n10 = t1 * BN1, n20 = t2 * BN2;
    const int kbeg = slice * kchunk, kend = min(M, kbeg + kchunk);
    const int w1 = wave / WG2, w2 = wave % WG2;

    f32x4 acc[R1][R2];
#pragma unroll
    for (int a = 0; a < R1; ++a)
#pragma unroll
        for (int b = 0; b < R2; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int nk = (kend - kbeg + BKT - 1) / BKT;
    // conv mode: N2 = 9*C and a BN2 tile lies inside one tap (C % BN2 == 0, host-checked)
    int bc0 = n20, dh = 0, dw = 0;
    if constexpr (CONV == 1) {
        const int t = n20 / geo.C;
        bc0 = n20 - t * geo.C;
        dh = geo.offh[t];
        dw = geo.offw[t];
    }
    const __amdgpu_buffer_rsrc_t ra = buf_rsrc(A), rb = buf_rsrc(B);
    auto stage = [&](int buf, int k0) {
        char* base = smem + buf * STAGE;
        stage_rows<ROWA, 0, BKT>(base, ra, lda, k0, kend, n10, wave, lane);
        stage_rows<ROWB_, CONV, BKT>(base + A_BYTES, rb, ldb, k0, kend, bc0, wave, lane, &geo, dh, dw);
    };
    const int gi = lane & 15, g = lane >> 4, q = gi >> 2, p = gi & 3;
    if constexpr (NST == 2) {
        if (nk > 0) {
            stage(0, kbeg);
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    } else {
        for (int st = 0; st < NST - 1 && st < nk; ++st) stage(st, kbeg + st * BKT);
    }
    for (int kt = 0; kt < nk; ++kt) {
        int cur;
        if constexpr (NST == 2) {
            cur = kt & 1;
            if (kt + 1 < nk) stage(cur ^ 1, kbeg + (kt + 1) * BKT);
        } else {
            // stages kt+1 .. min(kt+NST-2, nk-1) may stay in flight; stage kt must have landed for every wave, and
            // every wave is done with stage kt-1's buffer, which the fill of stage kt+NST-1 reuses
            const int later = min(NST - 2, nk - 1 - kt);
            wait_vm_stages<PER_STAGE>(later);
            __syncthreads();
            if (kt + NST - 1 < nk) stage((kt + NST - 1) % NST, kbeg + (kt + NST - 1) * BKT);
            cur = kt % NST;
        }
        const char* As = smem + cur * STAGE;
        const char* Bs = As + A_BYTES;
#pragma unroll
        for (int kk = 0; kk < BKT / 32; ++kk) {
            const int kb = kk * 32 + 8 * g + q;             // this lane's address row for the first tr read
            bf16x8 fa[R1], fb[R2];
#pragma unroll
            for (int r = 0; r < R1; ++r) {
                const int c = w1 * WT1 + r * 16 + 4 * p;
                const s16x4 lo = tr_read<ROWA>(As, kb, c), hi = tr_read<ROWA>(As, kb + 4, c);
                fa[r] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int r = 0; r < R2; ++r) {
                const int c = w2 * WT2 + r * 16 + 4 * p;
                const s16x4 lo = tr_read<ROWB_>(Bs, kb, c), hi = tr_read<ROWB_>(Bs, kb + 4, c);
                fb[r] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(lo, hi, 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int a = 0; a < R1; ++a)
#pragma unroll
                for (int b = 0; b < R2; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
        }
        if constexpr (NST == 2) {
            asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
            __syncthreads();
        }
    }
    // D[n1][n2]: lane holds column n2 = lane&15, rows n1 = 4*(lane>>4) + r
    float* slab = W + (size_t)slice * N1 * N2;
#pragma unroll
    for (int a = 0; a < R1; ++a)
#pragma unroll
        for (int b = 0; b < R2; ++b) {
            const int c2 = n20 + w2 * WT2 + b * 16 + gi;
            const int r1 = n10 + w1 * WT1 + a * 16 + 4 * g;
#pragma unroll
            for (int r = 0; r < 4; ++r) slab[(size_t)(r1 + r) * N2 + c2] = acc[a][b][r];
        }
}

// Slab reduction, deterministic and graph-capturable (no memset, no atomics):
//   slab_partial_kernel  P[g][i] = sum of slabs [g*per_group, (g+1)*per_group)   (only when many slabs)
//   slab_final_kernel    C[i][j] (ldc) (+)= sum_s S[s][i][j]
// one float4 per thread; blockIdx.y = group in the partial pass.
__global__ void slab_partial_kernel(const float* __restrict__ W, float* __restrict__ P, long plane, int slices,
                                    int per_group) {
    const long total4 = plane / 4;
    const int s0 = blockIdx.y * per_group, s1 = min(slices, s0 + per_group);
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s = s0; s < s1; ++s) {
            const float4 v = ((const float4*)(W + s * plane))[i];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        ((float4*)(P + blockIdx.y * plane))[i] = acc;
    }
}

__global__ void slab_final_kernel(const float* __restrict__ S, float* __restrict__ C, int N1, int N2, int ldc,
                                  int nslabs, int accumulate) {
    const long total4 = (long)N1 * N2 / 4;
    const long plane = (long)N1 * N2;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total4; i += (long)gridDim.x * blockDim.x) {
        float4 acc = make_float4(0.f, 0.f, 0.f, 0.f);
        for (int s = 0; s < nslabs; ++s) {
            const float4 v = ((const float4*)(S + s * plane))[i];
            acc.x += v.x; acc.y += v.y; acc.z += v.z; acc.w += v.w;
        }
        const long e = i * 4;
        const int r = (int)(e / N2), c = (int)(e % N2);
        float* dst = C + (size_t)r * ldc + c;
        if (accumulate) {
            const float4 o = *(const float4*)dst;
            acc.x += o.x; acc.y += o.y; acc.z += o.z; acc.w += o.w;
        }
        *(float4*)dst = acc;
    }
}

// ------------------------------------------------------------------------------------------- TN GEMM, v2
// W[slice][N1][N2] (fp32 slab per m-slice) = sum_{m in slice} A[m][N1] * Bg[m][N2] with the same gathers as v1 (CONV 0
// dense, 1 the pixel shifted by the column's tap, 2 the stem's super-pixel window), summed by the same slab reducer.
//
// Why v1 is slow: one 4-wave block per CU (the slab budget keeps the grid near one block per CU) with ONE 32 KB stage
// in flight; an L2 -> LDS fill of that size takes ~1.5 us under load against ~0.2 us of MFMAs, so v1 ran at
// ~360 TFLOP/s on the 3x3 layers.  The per-CU LDS-DMA path needs ~100 KB in flight to run at its rate.
//
// v2: one block of NW = KS * NA * NB waves per CU.  Wave (g, w1, w2) owns the 64 x 64 output sub-tile (w1, w2) of a
// (64 NA) x (64 NB) tile, and of the K-stages it computes every KS-th, starting at g: the K range is split across the
// block's KS wave groups, whose accumulators are summed through LDS once at the end (several waves per SIMD without
// multiplying the slab bytes).  Operands are staged as 64-column sub-images [BKT rows][128 B] (NA of A, NB of B per
// stage; the ds_read_b64_tr_b16 swizzle of v1's 64-wide images) by buffer-resource LDS-DMA.  Each group owns RING / KS
// slots of the LDS ring and stages its own stages into them (its waves issue the DMAs), RING / KS - 1 of them in flight
// behind a counted vmcnt while it computes one.  Ping-pong (cdna_hip_programming.md T5): the second half of the waves
// (the SIMD partners of the first half; KS even, so every group lies in one half) runs one barrier behind, and an
// iteration has two barriers, [wait; barrier; MFMAs; barrier; refill DMAs], so on every SIMD one wave's MFMAs overlap
// its partner's DMA issue, gather address math and wait.  A group refills a slot right after the barrier that follows
// its own last read of it.  A 64-column sub-image lies inside one tap of a 3x3 gather (C % 64 == 0), so tiles may span
// taps: the gathered B tile of a C = 64 layer is 3 taps wide.
//
// ATOMIC: instead of a slab per slice (summed by the slab reducer's two extra launches), each block adds its tile into
// the fp32 output C (ldc) with no-return float atomics, which execute at the memory side (MI355X_MICROARCH.md, Global
// float atomics: ~1.3 TB/s of added bytes chip-wide, full rate for 256 contiguous bytes per wave instruction).  The
// finished tile goes through LDS (XOR-swizzled, conflict-free both ways) so every atomic instruction covers one 64-float
// row, and all NW waves of the block issue them.  The caller zeroes C first unless it accumulates.
template <int NA, int NB, int KS, int CONV, int BKT, int RING, bool ATOMIC = false>
__global__ void __launch_bounds__(64 * KS * NA * NB, 1)
wgrad_kernel(const __bf16* __restrict__ A, const __bf16* __restrict__ B, float* __restrict__ W, int M, int N1, int N2,
             int lda, int ldb, int kchunk, ConvGeom geo, int ldc) {
    constexpr int GW = NA * NB;                      // waves per group
    constexpr int NW = KS * GW;
    constexpr int R2 = RING / KS;                    // slots per group
    constexpr int SUB = BKT * 128;                   // one 64-column sub-image
    constexpr int STAGE = (NA + NB) * SUB;
    constexpr int PPS = SUB / 1024;                  // 1 KB DMA pieces per sub-image (8 rows each)
    static_assert(BKT == 32 || BKT == 64, "32- or 64-row stages");
    static_assert(KS % 2 == 0, "ping-pong pairs the two halves of the wave groups");
    static_assert(RING % KS == 0 && R2 >= 2, "every group owns >= 2 ring slots");
    static_assert(RING * STAGE <= 160 * 1024, "LDS ring exceeds the CU's LDS");
    static_assert((KS - 1) * GW * 16384 <= RING * STAGE, "the wave-group reduction reuses the ring");
    extern __shared__ __attribute__((aligned(16))) char smem[];

    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    constexpr int BN1 = 64 * NA, BN2 = 64 * NB;
    const int nt1 = N1 / BN1, nt2 = N2 / BN2, ntiles = nt1 * nt2;
    const int nslices = (M + kchunk - 1) / kchunk;
    const int id = xcd_remap(blockIdx.x, ntiles * nslices);   // consecutive ids (one slice's tiles) share an XCD
    const int tile = id % ntiles, slice = id / ntiles;
    const int n10 = (tile / nt2) * BN1, n20 = (tile % nt2) * BN2;
    const int kbeg = slice * kchunk, kend = min(M, kbeg + kchunk);
    const int nk = kend > kbeg ? (kend - kbeg + BKT - 1) / BKT : 0;
    const int grp = wave / GW, wg = wave % GW, w1 = wg / NB, w2 = wg % NB;
    const int nu = nk > grp ? (nk - grp + KS - 1) / KS : 0;   // this group's stages: s = grp + KS u, u < nu
    const int nit = (nk + KS - 1) / KS;                        // iterations (the same for every wave: barriers)
    const bool lag = wave >= NW / 2;

    // this wave's share of its group's DMA pieces of every stage, A and B separately (a run-time choice between the
    // two buffer resources put both in scratch): A piece pa = wg + i * GW < PA, B piece pb = wg + i * GW < PB; LDS
    // destination (A: pa, B: PA + pb) * 1024 in the stage's slot; row (pa % PPS) * 8 + lane / 8 of sub-image pa / PPS,
    // logical 16-B chunk (lane % 8) ^ swizzle(row)
    constexpr int PA = NA * PPS, PB = NB * PPS;
    constexpr int IA = (PA + GW - 1) / GW, IB = (PB + GW - 1) / GW;
    int cnta = 0, cntb = 0, arow[IA], acol[IA], brow[IB], bcol[IB], bdh[IB], bdw[IB];
#pragma unroll
    for (int i = 0; i < IA; ++i) {
        const int pa = wg + i * GW, row = (pa % PPS) * 8 + (lane >> 3);
        cnta += pa < PA ? 1 : 0;
        arow[i] = row;
        acol[i] = n10 + (pa / PPS) * 64 + (((lane & 7) ^ tr_swz<128>(row)) * 8);
    }
#pragma unroll
    for (int i = 0; i < IB; ++i) {
        const int pb = wg + i * GW, row = (pb % PPS) * 8 + (lane >> 3);
        const int col = n20 + (pb / PPS) * 64, lc8 = ((lane & 7) ^ tr_swz<128>(row)) * 8;
        cntb += pb < PB ? 1 : 0;
        brow[i] = row;
        bdh[i] = bdw[i] = 0;
        bcol[i] = col + lc8;
        if constexpr (CONV == 1) {                          // a 64-column chunk lies inside one tap: (tap, channel)
            const int t = col / geo.C;
            bdh[i] = geo.offh[t];
            bdw[i] = geo.offw[t];
            bcol[i] = col - t * geo.C + lc8;
        }
    }
    cnta = __builtin_amdgcn_readfirstlane(cnta);
    cntb = __builtin_amdgcn_readfirstlane(cntb);
    const int cnt = cnta + cntb;                            // DMAs per wave per stage
    const __amdgpu_buffer_rsrc_t ra = buf_rsrc(A), rb = buf_rsrc(B);
    // the gather's geometry as scalars
    const int gH = geo.H, gW = geo.W, gS = geo.S, gWr = geo.Wr, gHr = geo.Hr;
    const uint32_t gmWr = geo.mWr, gmHr = geo.mHr;
    auto coords = [=](int m, int& n, int& r, int& c) {
        const int qq = gmWr ? (int)__umulhi((uint32_t)m, gmWr) : m;
        c = m - qq * gWr;
        n = gmHr ? (int)__umulhi((uint32_t)qq, gmHr) : qq;
        r = qq - n * gHr;
    };
    char* const gslots = smem + grp * R2 * STAGE;           // this group's slots

    // stage u of this group (s = grp + KS u) into slot u % R2
    auto issue = [&](int u) {
        char* base = gslots + (u % R2) * STAGE;
        const int k0 = kbeg + (grp + KS * u) * BKT;
#pragma unroll
        for (int i = 0; i < IA; ++i) {
            if (i < cnta) {                                 // wave-uniform
                const int gr = k0 + arow[i];
                blds16(ra, gr < kend ? (uint32_t)((gr * lda + acol[i]) * 2) : OOB, base + (wg + i * GW) * 1024);
            }
        }
#pragma unroll
        for (int i = 0; i < IB; ++i) {
            if (i < cntb) {
                const int gr = k0 + brow[i];
                uint32_t off;
                if constexpr (CONV == 1) {
                    int n, r, c;
                    coords(gr, n, r, c);
                    const int ih = r * gS + bdh[i], iw = c * gS + bdw[i];
                    const bool ok = gr < kend && (unsigned)ih < (unsigned)gH && (unsigned)iw < (unsigned)gW;
                    off = ok ? (uint32_t)((((n * gH + ih) * gW + iw) * ldb + bcol[i]) * 2) : OOB;
                } else if constexpr (CONV == 2) {               // the stem's super-pixel window, chunk t = column / 8
                    int n, r, c;
                    coords(gr, n, r, c);
                    const int t = bcol[i] >> 3, ih = 2 * r - 3 + (t >> 2), sc = c - 2 + (t & 3);
                    const bool ok = gr < kend && t < 28 && (unsigned)ih < (unsigned)gH && (unsigned)sc < (unsigned)gW;
                    off = ok ? (uint32_t)(((n * gH + ih) * gW + sc) * 16) : OOB;
                } else {
                    off = gr < kend ? (uint32_t)((gr * ldb + bcol[i]) * 2) : OOB;
                }
                blds16(rb, off, base + (PA + wg + i * GW) * 1024);
            }
        }
    };
    // s_waitcnt vmcnt(n) for a wave-uniform run-time n (the counter is an instruction immediate)
    auto vm_wait = [&](int n) {
        switch (n < 0 ? 0 : n) {
#define PLX_VMW(k) case k: asm volatile("s_waitcnt vmcnt(" #k ")" ::: "memory"); break;
            PLX_VMW(1) PLX_VMW(2) PLX_VMW(3) PLX_VMW(4) PLX_VMW(5) PLX_VMW(6) PLX_VMW(7) PLX_VMW(8)
            PLX_VMW(9) PLX_VMW(10) PLX_VMW(11) PLX_VMW(12) PLX_VMW(13) PLX_VMW(14) PLX_VMW(15) PLX_VMW(16)
            PLX_VMW(17) PLX_VMW(18) PLX_VMW(19) PLX_VMW(20) PLX_VMW(21) PLX_VMW(22) PLX_VMW(23) PLX_VMW(24)
            PLX_VMW(25) PLX_VMW(26) PLX_VMW(27) PLX_VMW(28) PLX_VMW(29) PLX_VMW(30) PLX_VMW(31) PLX_VMW(32)
#undef PLX_VMW
            default:
                if (n > 32) asm volatile("s_waitcnt vmcnt(32)" ::: "memory");
                else asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        }
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) acc[a][b] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int gi = lane & 15, g4 = lane >> 4, q = gi >> 2, pp = gi & 3;
    // byte offsets (within a stage slot) of this lane's ds_read_b64_tr_b16 for fragment r of its A / B sub-image:
    // T10 addressing, k-row 8 (lane / 16) + (lane % 16) / 4, columns r * 16 + 4 (lane % 4) (BKT = 32: one k-step);
    // the second half of a fragment is 4 k-rows down, +512 B (the swizzle does not change over those rows)
    static_assert(BKT == 32, "the asm fragment path reads one 32-deep k-step per stage");
    uint32_t aoffr[4], boffr[4];
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        const int kb = 8 * g4 + q, col = r * 16 + 4 * pp;
        const int off = kb * 128 + (((col >> 3) ^ tr_swz<128>(kb)) << 4) + ((col >> 2) & 1) * 8;
        aoffr[r] = (uint32_t)(w1 * SUB + off);
        boffr[r] = (uint32_t)((NA + w2) * SUB + off);
    }

    for (int u = 0; u < R2 && u < nu; ++u) issue(u);
    if (lag) __builtin_amdgcn_s_barrier();                  // ping-pong: this half runs one barrier behind
    for (int it = 0; it < nit; ++it) {
        // stages [0, it] of the group must have landed; [0, min(nu, R2 + it)) were issued
        vm_wait(cnt * (min(nu, R2 + it) - min(nu, it + 1)));
        __builtin_amdgcn_s_barrier();                       // every wave of the group waited for its DMAs
        if (it < nu) {                                      // wave-uniform
            // fragment reads as inline asm: with the builtin, hipcc could not tell this slot from the ones the ring's
            // DMAs are filling and put s_waitcnt vmcnt(0) in front of the reads -- every stage in flight drained per
            // phase.  The asm wait below carries the fragments, so no MFMA can be scheduled above it.
            const uint32_t sa = lds_addr(gslots + (it % R2) * STAGE);
            s16x4 alo[4], ahi[4], blo[4], bhi[4];
            __builtin_amdgcn_s_setprio(1);
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                alo[r] = ds_tr(sa + aoffr[r]);
                ahi[r] = ds_tr(sa + aoffr[r] + 512);
                blo[r] = ds_tr(sa + boffr[r]);
                bhi[r] = ds_tr(sa + boffr[r] + 512);
            }
            asm volatile("s_waitcnt lgkmcnt(0)"
                         : "+v"(alo[0]), "+v"(alo[1]), "+v"(alo[2]), "+v"(alo[3]), "+v"(ahi[0]), "+v"(ahi[1]),
                           "+v"(ahi[2]), "+v"(ahi[3]), "+v"(blo[0]), "+v"(blo[1]), "+v"(blo[2]), "+v"(blo[3]),
                           "+v"(bhi[0]), "+v"(bhi[1]), "+v"(bhi[2]), "+v"(bhi[3]));
            bf16x8 fa[4], fb[4];
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                fa[r] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(alo[r], ahi[r], 0, 1, 2, 3, 4, 5, 6, 7));
                fb[r] = __builtin_bit_cast(bf16x8, __builtin_shufflevector(blo[r], bhi[r], 0, 1, 2, 3, 4, 5, 6, 7));
            }
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
                    acc[a][b] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[a], fb[b], acc[a][b], 0, 0, 0);
            __builtin_amdgcn_s_setprio(0);
        }
        asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");  // this wave's reads of the slot are done
        __builtin_amdgcn_s_barrier();                       // ... and every wave's of the group
        if (it + R2 < nu) issue(it + R2);                   // refill the slot just read
    }
    if (!lag) __builtin_amdgcn_s_barrier();                 // every wave executes the same number of barriers
    asm volatile("s_waitcnt vmcnt(0) lgkmcnt(0)" ::: "memory");
    __syncthreads();
    // groups 1..KS-1 hand their sums to group 0 through LDS (lane-contiguous, no conflicts), summed in group order
    float* red = (float*)smem;
    if (grp > 0) {
        float* dst = red + ((grp - 1) * GW + wg) * 4096 + lane;
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 4; ++b)
#pragma unroll
                for (int r = 0; r < 4; ++r) dst[((a * 4 + b) * 4 + r) * 64] = acc[a][b][r];
    }
    __syncthreads();
    if (!ATOMIC && grp > 0) return;
    if (grp == 0) {
#pragma unroll 1
        for (int g = 1; g < KS; ++g) {
            const float* src = red + ((g - 1) * GW + wg) * 4096 + lane;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) acc[a][b][r] += src[((a * 4 + b) * 4 + r) * 64];
        }
    }
    if constexpr (ATOMIC) {
        // group 0's sub-tiles -> LDS [wg][row][col ^ swz(row)], then every wave adds whole 64-float rows into C
        __syncthreads();  // every group-0 wave is done reading the hand-off area it now overwrites
        if (grp == 0) {
            float* t = red + wg * 4096;
#pragma unroll
            for (int a = 0; a < 4; ++a)
#pragma unroll
                for (int b = 0; b < 4; ++b)
#pragma unroll
                    for (int r = 0; r < 4; ++r) {
                        const int row = a * 16 + 4 * g4 + r, col = b * 16 + gi;
                        t[row * 64 + (col ^ (((row >> 2) & 3) << 4))] = acc[a][b][r];
                    }
        }
        __syncthreads();
#pragma unroll 4
        for (int j = wave; j < GW * 64; j += NW) {
            const int tw = j >> 6, row = j & 63;
            const float v = red[tw * 4096 + row * 64 + (lane ^ (((row >> 2) & 3) << 4))];
            float* dst = W + (size_t)(n10 + (tw / NB) * 64 + row) * ldc + n20 + (tw % NB) * 64 + lane;
            __hip_atomic_fetch_add(dst, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        }
        return;
    }
    // D[n1][n2]: lane holds column n2 = lane & 15, rows n1 = 4 (lane >> 4) + r
    float* slab = W + (size_t)slice * N1 * N2;
#pragma unroll
    for (int a = 0; a < 4; ++a)
#pragma unroll
        for (int b = 0; b < 4; ++b) {
            const int c2 = n20 + w2 * 64 + b * 16 + gi;
            const int r1 = n10 + w1 * 64 + a * 16 + 4 * g4;
#pragma unroll
            for (int r = 0; r < 4; ++r) slab[(size_t)(r1 + r) * N2 + c2] = acc[a][b][r];
        }
}

// fp32 W[Cout][Cin] -> bf16 W[Cout][Cin] and bf16 W^T[Cin][Cout] (both used by the 1x1 conv passes)
__global__ void weight_prep_kernel(const float* __restrict__ w, __bf16* __restrict__ wb, __bf16* __restrict__ wt,
                                   int cout, int cin) {
    __shared__ float tile[32][33];
    const int c0 = blockIdx.x * 32, o0 = blockIdx.y * 32;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;   // 256 threads: 32 x 8
    for (int j = ty; j < 32; j += 8) {
        const int o = o0 + j, c = c0 + tx;
        float v = (o < cout && c < cin) ? w[(size_t)o * cin + c] : 0.f;
        tile[j][tx] = v;
        if (o < cout && c < cin) wb[(size_t)o * cin + c] = (__bf16)v;
    }
    __syncthreads();
    for (int j = ty; j < 32; j += 8) {
        const int c = c0 + j, o = o0 + tx;
        if (o < cout && c < cin) wt[(size_t)c * cout + o] = (__bf16)tile[tx][j];
    }
}

template <typename KernelT>
int set_lds(KernelT k, int bytes) {
    return hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, bytes) == hipSuccess ? 0
                                                                                                                 : -2;
}

// NBUF = 1: one K-stage buffer, LDS = max(stage, epilogue staging), 3-4 blocks per CU (the skinny GEMMs)
template <int BM, int BN, int WGM, int WGN, int CONV = 0, int NBUF = 2>
int launch_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
              const void* zero, float* stats, hipStream_t s, ConvGeom geo = {}, const void* D = nullptr,
              int ldd = 0, BnBwd bnr = {}, const uint8_t* dmask = nullptr) {
    constexpr int NTH = NTHREADS;
    constexpr int TILE = BM * (BN * 2 + 16), RED = NTH * 17 * 4;
    constexpr int EPI = TILE > RED ? TILE : RED;            // the reduction reuses the tile's LDS
    constexpr int KLOOP = NBUF * (BM + BN) * BK * 2;
    constexpr int LDS = KLOOP > EPI ? KLOOP : EPI;
    static_assert(NBUF >= 1 && NBUF <= 2, "one or two K stages");
    static_assert(NBUF == 1 || EPI <= KLOOP, "epilogue staging must fit the k-loop LDS");
    static_assert(LDS <= 160 * 1024, "LDS");
    constexpr int PER_CU = (160 * 1024) / LDS;
    // blocks per CU the registers are asked to allow (128 VGPRs at 4): the double-buffered data-gradient kernel
    // keeps its accumulators live through the epilogue prefetch (~178 VGPRs), the single-buffer one parks them in
    // LDS first (LATE in gemm_nt_kernel)
    constexpr int CAP = CONV != 0 && BN == 64 ? 3 : 4;     // the 256x64 conv staging spills 7-8 VGPRs at 4
    constexpr int MIN_F = NBUF == 1 ? (PER_CU < CAP ? PER_CU : CAP) : 2, MIN_B = MIN_F;
    auto kf = gemm_nt_kernel<BM, BN, WGM, WGN, CONV, MIN_F, NBUF, false, NTH>;
    auto kb = gemm_nt_kernel<BM, BN, WGM, WGN, CONV, MIN_B, NBUF, true, NTH>;
    static int attr = set_lds(kf, LDS) | set_lds(kb, LDS);
    if (attr) return attr;
    const bool bwd = D != nullptr || bnr.part != nullptr;
    if (bwd && stats != nullptr) return -1;
    auto k = bwd ? kb : kf;
    const int nwg = ((M + BM - 1) / BM) * (N / BN);
    hipLaunchKernelGGL(k, dim3(nwg), dim3(NTH), LDS, s, (const __bf16*)A, (const __bf16*)B, (__bf16*)C, M, N,
                       K, lda, ldb, ldc, (const __bf16*)zero, stats, geo, (const __bf16*)D, ldd, bnr, dmask);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// Single-buffer NT GEMM (NBUF = 1) or double-buffered.  The single-buffer kernels run 4 blocks per CU (3 for the
// 256x64 conv tile), which hides the staging better than double buffering at 2 blocks -- when the grid has the
// blocks to fill them (>= 3 per CU), or when K == BK leaves nothing to double-buffer.  Measured on the ResNet-50
// shapes (scripts/ab_modes.sh, profiles/r2_nt_single_buffer_ab.md): single-buffered when the grid has >= 3 blocks per
// CU, or for plain GEMMs with K == BK.

inline bool nt_single(bool conv, int K, int nwg) { return nwg >= 768 || (!conv && K == BK); }

// m-slicing of the weight-gradient GEMM
struct TnPlan { int kchunk, slices, groups, per_group, blocks, bn1, bn2; };

inline void tn_tile(int N1, int N2, int& bn1, int& bn2) {
    bn1 = N1 % 128 == 0 ? 128 : 64;
    bn2 = N2 % 128 == 0 ? 128 : 64;
}

// v1 slicing: target resident blocks per CU, cap on the fp32 slab bytes.  (v1 serves the stem's weight gradient, alone
// at the end of the backward with 4 blocks per CU, and the v1 variant of the tests.)  Swept in isolation (scripts/diag_wgrad_plan.py) 3 / 32 MB was best; in the training step the weight gradients run on
// the side stream beside the data-gradient chain, and there fewer slices (less slab traffic competing with the main
// stream) win, except for the 56x56 layers whose gradients finish the backward: 0 = by size (tn_plan), 16 MB.  Same-box
// bench, 2 interleaved rounds (blocks per CU / slab MB): 3/32 11.61k, 11.70k; 1/16 11.71k, 11.75k; by size 11.85k, 11.87k trials/h.
// Slab cap under the by-size plan: 8 MB 10.62k / 10.60k (too few slices), 16 MB 11.92k / 11.93k, 32 MB 11.91k / 11.91k
constexpr int g_tn_blocks_per_cu = 0;
constexpr int g_tn_bpc_big = 3, g_tn_bpc_mid = 1;  // by-size plan: 56x56 layers, 28x28 layers
constexpr long g_tn_slab_bytes = 16l << 20;

// bpc > 0 overrides the blocks-per-CU target (the stem's weight gradient runs alone at the end of the backward)
inline TnPlan tn_plan(int M, int N1, int N2, int num_cus, int bpc = 0) {
    int bn1, bn2;
    tn_tile(N1, N2, bn1, bn2);
    const int ntiles = (N1 / bn1) * (N2 / bn2);
    const long plane = (long)N1 * N2;
    // ~4 blocks per CU (one 4-wave block per CU leaves each SIMD a single wave: latency-bound), >= 4
    // k-stages per block, slabs <= 32 MB (they are re-read by the reducer, mostly from the infinity cache)
    // g_tn_blocks_per_cu == 0: by size -- the 56x56 layers (M >= 400k rows) are the last weight gradients of the
    // backward, with little main-stream work left to hide them behind, so they get 3 blocks per CU; the rest 1
    const int bpc_eff = bpc > 0 ? bpc
                                : (g_tn_blocks_per_cu > 0 ? g_tn_blocks_per_cu
                                                          : (M >= 400000 ? g_tn_bpc_big : M >= 150000 ? g_tn_bpc_mid : 1));
    int slices = (bpc_eff * (num_cus > 0 ? num_cus : 256)) / ntiles;
    const int by_depth = M / (4 * BK);
    const int by_bytes = (int)(g_tn_slab_bytes / (plane * 4));
    if (slices > by_depth) slices = by_depth;
    if (slices > by_bytes) slices = by_bytes;
    if (slices < 1) slices = 1;
    int kchunk = (M + slices - 1) / slices;
    kchunk = ((kchunk + BK - 1) / BK) * BK;
    slices = (M + kchunk - 1) / kchunk;
    // reducer: ~1024 blocks; many slabs are first summed in groups of >= 8 so a small plane still spreads out
    const long total4 = plane / 4;
    int blocks = (int)((total4 + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    int groups = 1024 / blocks;
    if (groups > slices / 8) groups = slices / 8;
    if (groups < 1) groups = 1;
    const int per_group = (slices + groups - 1) / groups;
    groups = (slices + per_group - 1) / per_group;
    return {kchunk, slices, groups, per_group, blocks, bn1, bn2};
}

template <int BN1, int BN2, int WG1, int WG2, int CONV, int NST, int BKT = BK>
int launch_tn_st(const void* A, const void* B, float* W, int M, int N1, int N2, int lda, int ldb, const TnPlan& plan,
                 const void* zero, hipStream_t s, const ConvGeom& geo) {
    constexpr int LDS = NST * BKT * (BN1 + BN2) * 2;
    static_assert(LDS <= 160 * 1024, "LDS ring exceeds the CU's LDS");
    auto k = gemm_tn_kernel<BN1, BN2, WG1, WG2, CONV, NST, BKT>;
    static int attr = set_lds(k, LDS);
    if (attr) return attr;
    const int ntiles = (N1 / BN1) * (N2 / BN2);
    hipLaunchKernelGGL(k, dim3(ntiles * plan.slices), dim3(NTHREADS), LDS, s, (const __bf16*)A, (const __bf16*)B, W,
                       M, N1, N2, lda, ldb, plan.kchunk, (const __bf16*)zero, geo);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---- v2 weight-gradient plan (wgrad_kernel): one block per CU, tile by the output shape, slices by a cost model
// In the training step (weight gradients on the side stream beside the data-gradient chain) v2 with a 64 KB ring and
// 3/4 of the CUs' worth of blocks measured +0.7 % trials/h over v1 (4 runs each on 2 boxes); with a 128 KB ring or
// one block on every CU it was 2-4 % slower, although faster in isolation (profiles/r5_wgrad_v2.md)
int g_tn_v2 = 1;        // 1: wgrad_kernel (v2), 0: gemm_tn_kernel (v1), 2: v2 for the gathered convolutions only
                        // (test hook plx_set_tn_v2)
int g_tn2_lds_kb = 64;  // LDS ring budget of a v2 block: 128 KB (one block per CU) or 64 KB (two per CU, or room for the
                        // main stream's blocks beside it); configurations whose groups would get < 2 slots keep 128

struct V2Cfg { int na, nb, ks; };

// 64-column sub-images per operand and wave groups: always 8 waves except the C = 64 3x3 (3 x 2 = 6)
inline V2Cfg v2_cfg(int N1, int N2) {
    if (N1 % 128 == 0 && N2 % 128 == 0) return {2, 2, 2};
    if (N1 % 128 != 0) {  // N1 an odd multiple of 64 (64: ResNet layer 1)
        if (N1 == 64 && N2 % 256 == 0) return {1, 4, 2};
        if (N1 == 64 && N2 % 192 == 0) return {1, 3, 2};
        if (N1 == 64 && N2 % 128 == 0) return {1, 2, 4};
        return {1, 1, 8};
    }
    return N1 % 256 == 0 ? V2Cfg{4, 1, 2} : V2Cfg{2, 1, 4};  // N2 an odd multiple of 64
}

// slab reducer sizing (shared by both plans): ~1024 blocks; many slabs are first summed in groups of >= 8
inline void plan_reducer(TnPlan& p, long plane) {
    const long total4 = plane / 4;
    int blocks = (int)((total4 + 255) / 256);
    if (blocks > 2048) blocks = 2048;
    int groups = 1024 / blocks;
    if (groups > p.slices / 8) groups = p.slices / 8;
    if (groups < 1) groups = 1;
    const int per_group = (p.slices + groups - 1) / groups;
    p.groups = (p.slices + per_group - 1) / per_group;
    p.per_group = per_group;
    p.blocks = blocks;
}

// Slices: the grid runs one block per CU, so slices s put ceil(tiles * s / CUs) blocks on the busiest CU.  Modelled
// time = compute (FLOP / chip rate, stretched by that quantisation) + a per-block fixed cost (ring fill + epilogue)
// per round of blocks + the slab bytes (s + 1 planes: written, read back by the reducer) when s > 1.  Rates are
// round numbers from the v2 isolated runs (profiles/r5_wgrad_v2.md).
constexpr double kTnCuFlops = 3.2e12, kTnBlockUs = 2.5;
// slab bandwidth the plan prices: 4.5 TB/s, the isolated rate of the slab write + reduce passes (with the in-kernel
// atomic reduction the same plan is kept: the added bytes cost about what the slab round trip did)
constexpr double g_tn2_slab_bw = 4.5e12;

// ring slots of a v2 block within an LDS budget (a multiple of KS, <= 16); 0 when a group would get < 2 slots
constexpr int tn2_ring(int na, int nb, int ks, int lds_kb) {
    const int stage = (na + nb) * 32 * 128, r0 = (lds_kb * 1024) / stage, r1 = r0 > 16 ? 16 : r0, r = r1 - r1 % ks;
    return r / ks >= 2 && (ks - 1) * na * nb * 16384 <= r * stage ? r : 0;
}

inline int tn2_ring_kb(const V2Cfg& c) {
    return g_tn2_lds_kb <= 64 && tn2_ring(c.na, c.nb, c.ks, 64) ? 64 : 128;
}

// blocks the v2 plan aims for: 1 or 2 per CU, or (> 2) a total block count; 0 (default): 3/4 of the CUs, which leaves
// a quarter of the CUs whole to the main stream's kernels (in-step sweep over 128-256 blocks: 192 best, 176 / 208 /
// 224 / 256 at or below v1)
constexpr int g_tn2_bpc = 0;

// the stem's weight gradient (CONV 2), which runs alone on the main stream at the very end of the backward: 0 v1
// (gemm_tn_kernel, 4 blocks per CU), 1 v2 planned for 2 blocks on every CU, 2 v2 with the side stream's block target
// (test hook plx_set_tn2_stem)
int g_tn2_stem = 0;

// v2 for the 6-wave configuration (N1 = 64, N2 a multiple of 192: the C = 64 3x3 weight gradients); test hook
// plx_set_tn2_c64
int g_tn2_c64 = 1;
constexpr int kStemV2Bpc = 2;

// v2 weight gradients reduce their K slices in the kernel with float atomics into the output (wgrad_kernel ATOMIC) --
// 1, default -- or through fp32 slabs and the slab reducer's launches (0; deterministic summation order).  A/B knob
// plx_set_tn_atomic (PLX_WGRAD_ATOMIC)
int g_tn_atomic = 1;

// full_bpc > 0: plan for that many blocks on EVERY CU (the stem's weight gradient, alone on the GPU at the end of the
// backward), whatever the block target
inline TnPlan tn2_plan(int M, int N1, int N2, int num_cus, const V2Cfg& c, int full_bpc = 0) {
    const int bn1 = 64 * c.na, bn2 = 64 * c.nb;
    const int ntiles = (N1 / bn1) * (N2 / bn2);
    const int ncu = num_cus > 0 ? num_cus : 256;
    const int cus = full_bpc > 0     ? ncu * full_bpc
                    : g_tn2_bpc > 2  ? g_tn2_bpc
                    : g_tn2_bpc > 0  ? ncu * g_tn2_bpc
                                     : (ncu * 3) / 4;
    const int step = 32 * c.ks;                       // rows per iteration
    const long plane = (long)N1 * N2;
    const double flops = 2.0 * M * plane;
    int by_depth = M / (4 * step);                    // >= 4 iterations per block
    if (by_depth < 1) by_depth = 1;
    if (by_depth > 1024) by_depth = 1024;
    int best = 1;
    double best_t = 1e30;
    for (int s = 1; s <= by_depth; ++s) {
        const long blocks = (long)ntiles * s;
        const long rounds = (blocks + cus - 1) / cus;
        const double t = flops / (kTnCuFlops * cus) * ((double)rounds * cus / blocks) + rounds * kTnBlockUs * 1e-6 +
                         (s > 1 ? (double)(s + 1) * plane * 4 / g_tn2_slab_bw : 0.0);
        if (t < best_t * 0.995) best_t = t, best = s;
    }
    int kchunk = (M + best - 1) / best;
    kchunk = ((kchunk + step - 1) / step) * step;
    TnPlan p{kchunk, (M + kchunk - 1) / kchunk, 1, 1, 0, bn1, bn2};
    plan_reducer(p, plane);
    return p;
}

template <int NA, int NB, int KS, int CONV, int LDSK, bool ATOMIC>
int launch_tn2_k(const void* A, const void* B, float* W, int M, int N1, int N2, int lda, int ldb, const TnPlan& plan,
                 hipStream_t s, const ConvGeom& geo, int ldc) {
    constexpr int BKT = 32, STAGE = (NA + NB) * BKT * 128;
    constexpr int RING = tn2_ring(NA, NB, KS, LDSK);
    static_assert(RING > 0, "ring budget too small for this configuration");
    constexpr int LDS = RING * STAGE;
    static_assert(!ATOMIC || NA * NB * 16384 <= LDS, "the atomic epilogue's tile image exceeds the ring");
    auto k = wgrad_kernel<NA, NB, KS, CONV, BKT, RING, ATOMIC>;
    static int attr = set_lds(k, LDS);
    if (attr) return attr;
    const int ntiles = (N1 / (64 * NA)) * (N2 / (64 * NB));
    hipLaunchKernelGGL(k, dim3(ntiles * plan.slices), dim3(64 * NA * NB * KS), LDS, s, (const __bf16*)A,
                       (const __bf16*)B, W, M, N1, N2, lda, ldb, plan.kchunk, geo, ldc);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

template <int NA, int NB, int KS, int CONV, bool ATOMIC>
int launch_tn2(const void* A, const void* B, float* W, int M, int N1, int N2, int lda, int ldb, const TnPlan& plan,
               hipStream_t s, const ConvGeom& geo, int ldc) {
    if constexpr (tn2_ring(NA, NB, KS, 64) > 0) {
        if (tn2_ring_kb(V2Cfg{NA, NB, KS}) <= 64)
            return launch_tn2_k<NA, NB, KS, CONV, 64, ATOMIC>(A, B, W, M, N1, N2, lda, ldb, plan, s, geo, ldc);
    }
    return launch_tn2_k<NA, NB, KS, CONV, 128, ATOMIC>(A, B, W, M, N1, N2, lda, ldb, plan, s, geo, ldc);
}

// atomic: add into W = C (ldc) in the kernel (wgrad_kernel ATOMIC) instead of writing slabs (ld N2)
template <int CONV>
int dispatch_tn2(const V2Cfg& c, const void* A, const void* B, float* W, int M, int N1, int N2, int lda, int ldb,
                 const TnPlan& plan, hipStream_t s, const ConvGeom& geo, bool atomic = false, int ldc = 0) {
    if constexpr (CONV == 2) {  // the stem: 64 x 256
        if (c.na == 1 && c.nb == 4 && c.ks == 2)
            return atomic ? launch_tn2<1, 4, 2, 2, true>(A, B, W, M, N1, N2, lda, ldb, plan, s, geo, ldc)
                          : launch_tn2<1, 4, 2, 2, false>(A, B, W, M, N1, N2, lda, ldb, plan, s, geo, ldc);
        return -1;
    } else {
#define PLX_TN2(a, b, k) \
    if (c.na == a && c.nb == b && c.ks == k) \
        return atomic ? launch_tn2<a, b, k, CONV, true>(A, B, W, M, N1, N2, lda, ldb, plan, s, geo, ldc) \
                      : launch_tn2<a, b, k, CONV, false>(A, B, W, M, N1, N2, lda, ldb, plan, s, geo, ldc);
        PLX_TN2(2, 2, 2) PLX_TN2(1, 4, 2) PLX_TN2(1, 3, 2) PLX_TN2(1, 2, 4) PLX_TN2(1, 1, 8) PLX_TN2(4, 1, 2)
        PLX_TN2(2, 1, 4)
#undef PLX_TN2
        return -1;
    }
}

template <int BN1, int BN2, int WG1, int WG2, int CONV = 0>
int launch_tn(const void* A, const void* B, float* W, int M, int N1, int N2, int lda, int ldb, const TnPlan& plan,
              const void* zero, hipStream_t s, ConvGeom geo = {}) {
    // double buffering (deeper rings measured slower in the step: a 96-128 KB ring leaves no LDS on its CU for the
    // data-gradient chain's blocks, profiles/r3_negative_results.md)
    return launch_tn_st<BN1, BN2, WG1, WG2, CONV, 2>(A, B, W, M, N1, N2, lda, ldb, plan, zero, s, geo);
}

}  // namespace

extern "C" {

// tile selection: wide-N problems use 128x128, N == 64 uses 256x64 (pixels x channels)
int plx_gemm_nt_rows_per_block(int N) { return N % 128 == 0 ? 128 : 256; }

// stats (nullable): fp32 [2][ceil(M / rows_per_block)][N] per-block channel sums / sums of squares of C
// D (nullable, bf16 [M][N], ldd): added to the product (C = A.B^T + D); not reflected in stats
// bnr (nullable host struct): fused BatchNorm-backward partials of C (see BnBwd; needs ldc == N)
// dmask (nullable, needs D and ldd == N): D is added where its bit is set (D * ReLU mask, 1 bit per element)
int plx_gemm_nt(const void* A, const void* B, void* C, int M, int N, int K, int lda, int ldb, int ldc,
                const void* zero, float* stats, const void* D, int ldd, const uint8_t* dmask, const BnBwd* bnr,
                void* stream) {
    if (M <= 0 || N % 64 || K % BK || lda % 8 || ldb % 8 || ldc % 8 || (D != nullptr && ldd % 8)) return -1;
    if (dmask != nullptr && (D == nullptr || ldd != N)) return -1;
    if (bnr != nullptr && (ldc != N || bnr->part == nullptr)) return -1;
    const BnBwd b = bnr != nullptr ? *bnr : BnBwd{};
    hipStream_t s = (hipStream_t)stream;
    if (N % 128 == 0) {
        const bool one = nt_single(false, K, ((M + 127) / 128) * (N / 128));
        return one ? launch_nt<128, 128, 2, 2, false, 1>(A, B, C, M, N, K, lda, ldb, ldc, zero, stats, s, {}, D, ldd, b,
                                                         dmask)
                   : launch_nt<128, 128, 2, 2>(A, B, C, M, N, K, lda, ldb, ldc, zero, stats, s, {}, D, ldd, b, dmask);
    }
    const bool one = nt_single(false, K, ((M + 255) / 256) * (N / 64));
    return one ? launch_nt<256, 64, 4, 1, false, 1>(A, B, C, M, N, K, lda, ldb, ldc, zero, stats, s, {}, D, ldd, b, dmask)
               : launch_nt<256, 64, 4, 1>(A, B, C, M, N, K, lda, ldb, ldc, zero, stats, s, {}, D, ldd, b, dmask);
}

// diagnostics: K slices (fp32 slabs) the weight-gradient plan of this problem uses (v2: wgrad_kernel's plan)
int plx_tn_plan_slices(int M, int N1, int N2, int num_cus, int v2) {
    if (M <= 0 || N1 % 64 || N2 % 64) return -1;
    return v2 ? tn2_plan(M, N1, N2, num_cus, v2_cfg(N1, N2)).slices : tn_plan(M, N1, N2, num_cus).slices;
}

// Kernel selection hooks of the weight-gradient tests (tests/test_gpu_conv.py runs every variant against fp32; no
// environment knob sets them): the C = 64 3x3 6-wave v2 configuration, the in-kernel atomic reduction (else slabs),
// the stem's kernel (0 v1, 1 v2 on every CU, 2 v2 with the side-stream block target), v2 (1) or v1 (0) with v2's LDS
// ring budget (64 or 128 KB, <= 0 keeps it; workspace queries size for every plan)
void plx_set_tn2_c64(int on) { g_tn2_c64 = on ? 1 : 0; }

void plx_set_tn_atomic(int on) { g_tn_atomic = on ? 1 : 0; }

void plx_set_tn2_stem(int mode) { g_tn2_stem = mode < 0 ? 0 : (mode > 2 ? 2 : mode); }

void plx_set_tn_v2(int on, int lds_kb) {
    g_tn_v2 = on < 0 ? 0 : (on > 2 ? 2 : on);
    if (lds_kb > 0) g_tn2_lds_kb = lds_kb <= 64 ? 64 : 128;
}

// floats of slab workspace plx_gemm_tn needs for this problem
long plx_gemm_tn_workspace(int M, int N1, int N2, int num_cus) {
    if (M <= 0 || N1 % 64 || N2 % 64) return -1;
    const TnPlan a = tn_plan(M, N1, N2, num_cus);
    long n = a.slices + (a.groups > 1 ? a.groups : 0);
    for (int kb = 64; kb <= 128; kb += 64) {  // both v2 ring budgets, whatever the knob
        const int keep = g_tn2_lds_kb;
        g_tn2_lds_kb = kb;
        const TnPlan c = tn2_plan(M, N1, N2, num_cus, v2_cfg(N1, N2));
        g_tn2_lds_kb = keep;
        const long nc = c.slices + (c.groups > 1 ? c.groups : 0);
        if (nc > n) n = nc;
    }
    return n * N1 * N2;
}

}  // extern "C"

namespace {
template <int CONV>
int run_tn(const void* A, const void* B, float* C, float* ws, int M, int N1, int N2, int lda, int ldb, int ldc,
           const void* zero, int num_cus, int accumulate, hipStream_t s, ConvGeom geo, int bpc = 0) {
    // 2: v2 for the gathered (KxK / strided) ones; the stem (CONV 2) by its own knob g_tn2_stem
    const V2Cfg cfg = v2_cfg(N1, N2);
    // the 6-wave configuration (the C = 64 3x3 layers: N2 = 9 x 64) is slower than v1 in isolation (144 vs 127 us)
    // and holds the side stream 1.5 ms/step in the step (3 calls at ~500 us), yet the step is faster with it
    // (12.38-12.41k vs 12.35k trials/h, r5_wgrad_c64_ab.jsonl): g_tn2_c64 = 0 moves it back to v1 (A/B)
    const bool six = cfg.na == 1 && cfg.nb == 3;
    const bool v2 = CONV == 2 ? g_tn2_stem > 0
                              : (g_tn_v2 == 1 || (g_tn_v2 == 2 && CONV != 0)) && (!six || g_tn2_c64);
    const TnPlan plan = v2 ? tn2_plan(M, N1, N2, num_cus, cfg, CONV == 2 && g_tn2_stem == 1 ? kStemV2Bpc : 0)
                           : tn_plan(M, N1, N2, num_cus, bpc);
    int rc;
    if (v2 && g_tn_atomic) {  // in-kernel reduction: float atomics into C, no slabs, no reducer launches
        if (!accumulate && hipMemset2DAsync(C, (size_t)ldc * 4, 0, (size_t)N2 * 4, N1, s) != hipSuccess) return -3;
        return dispatch_tn2<CONV>(cfg, A, B, C, M, N1, N2, lda, ldb, plan, s, geo, true, ldc);
    }
    if (v2)
        rc = dispatch_tn2<CONV>(cfg, A, B, ws, M, N1, N2, lda, ldb, plan, s, geo);
    else if (N1 % 128 == 0 && N2 % 128 == 0)
        rc = launch_tn<128, 128, 2, 2, CONV>(A, B, ws, M, N1, N2, lda, ldb, plan, zero, s, geo);
    else if (N1 % 128 == 0)
        rc = launch_tn<128, 64, 4, 1, CONV>(A, B, ws, M, N1, N2, lda, ldb, plan, zero, s, geo);
    else if (N2 % 128 == 0)
        rc = launch_tn<64, 128, 1, 4, CONV>(A, B, ws, M, N1, N2, lda, ldb, plan, zero, s, geo);
    else
        rc = launch_tn<64, 64, 2, 2, CONV>(A, B, ws, M, N1, N2, lda, ldb, plan, zero, s, geo);
    if (rc) return rc;
    const long plane = (long)N1 * N2;
    const float* slabs = ws;
    int nslabs = plan.slices;
    if (plan.groups > 1) {
        float* part = ws + (long)plan.slices * plane;
        hipLaunchKernelGGL(slab_partial_kernel, dim3(plan.blocks, plan.groups), dim3(256), 0, s, ws, part, plane,
                           plan.slices, plan.per_group);
        slabs = part;
        nslabs = plan.groups;
    }
    hipLaunchKernelGGL(slab_final_kernel, dim3(plan.blocks), dim3(256), 0, s, slabs, C, N1, N2, ldc, nslabs, accumulate);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// fp32 weight [Cout][Cin][K][K] (any strides) -> bf16 Wf[Cout][tap][Cin] (forward B operand) and
// Wd[Cin][tap][Cout] (data-gradient B operand; tap flips / parity classes live in the gather, not in the copy)
__global__ void weight_prepk_kernel(const float* __restrict__ w, long s_co, long s_ci, long s_kh, long s_kw,
                                    __bf16* __restrict__ wf, __bf16* __restrict__ wd, int cout, int cin, int K) {
    const int taps = K * K;
    const long total = (long)cout * cin * taps;
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < total; i += (long)gridDim.x * blockDim.x) {
        const int ci = (int)(i % cin);
        const long r = i / cin;
        const int tap = (int)(r % taps), co = (int)(r / taps);
        const __bf16 v = (__bf16)w[co * s_co + ci * s_ci + (tap / K) * s_kh + (tap % K) * s_kw];
        wf[i] = v;                                            // [co][tap][ci]
        wd[((long)ci * taps + tap) * cout + co] = v;          // [ci][tap][co]
    }
}

// One launch for every convolution weight of a model (plx_weight_prep_all): segment s reads the fp32 weight
// [cout][taps][cin] at base + src (the flat buffer's channels_last order) and writes bf16 Wf (same order) at
// wf + dst_f and bf16 Wd [cin][taps][cout] at wd + dst_d.  Block b handles one 32 x 32 (cout x cin) tile of one
// tap of the segment whose tile0 <= b < next tile0; the transpose goes through LDS so both stores coalesce.
struct WSeg {
    long src, dst_f, dst_d;
    int cout, cin, taps, tile0;
};

__global__ void __launch_bounds__(256) weight_prep_all_kernel(const float* __restrict__ base, __bf16* __restrict__ wf,
                                                              __bf16* __restrict__ wd, const WSeg* __restrict__ segs,
                                                              int nseg) {
    __shared__ float tile[32][33];
    int lo = 0, hi = nseg - 1;                              // last segment with tile0 <= blockIdx.x (uniform)
    while (lo < hi) {
        const int mid = (lo + hi + 1) >> 1;
        if (segs[mid].tile0 <= (int)blockIdx.x) lo = mid;
        else hi = mid - 1;
    }
    const WSeg s = segs[lo];
    int t = blockIdx.x - s.tile0;
    const int nci = (s.cin + 31) >> 5, nco = (s.cout + 31) >> 5;
    const int ci0 = (t % nci) * 32;
    t /= nci;
    const int co0 = (t % nco) * 32, tap = t / nco;
    const int tx = threadIdx.x & 31, ty = threadIdx.x >> 5;  // 32 x 8
    for (int j = ty; j < 32; j += 8) {
        const int co = co0 + j, ci = ci0 + tx;
        float v = 0.f;
        if (co < s.cout && ci < s.cin) {
            const long e = ((long)co * s.taps + tap) * s.cin + ci;
            v = base[s.src + e];
            wf[s.dst_f + e] = (__bf16)v;
        }
        tile[j][tx] = v;
    }
    __syncthreads();
    for (int j = ty; j < 32; j += 8) {
        const int ci = ci0 + j, co = co0 + tx;
        if (co < s.cout && ci < s.cin) wd[s.dst_d + ((long)ci * s.taps + tap) * s.cout + co] = (__bf16)tile[tx][j];
    }
}
}  // namespace

extern "C" {

// C[N1][N2] (ldc, fp32) = (accumulate ? C : 0) + A^T B over M rows; ws holds plx_gemm_tn_workspace floats
int plx_gemm_tn(const void* A, const void* B, float* C, float* ws, int M, int N1, int N2, int lda, int ldb, int ldc,
                const void* zero, int num_cus, int accumulate, void* stream) {
    if (M <= 0 || N1 % 64 || N2 % 64 || lda % 8 || ldb % 8 || ldc % 4) return -1;
    return run_tn<false>(A, B, C, ws, M, N1, N2, lda, ldb, ldc, zero, num_cus, accumulate, (hipStream_t)stream, {});
}

// ---- KxK (K = 1 or 3, pad = K/2) convolutions with stride 1 or 2 on NHWC bf16 (Cin, Cout multiples of 64)
}  // extern "C"

namespace {
inline int out_dim(int H, int K, int S) { return (H + 2 * (K / 2) - K) / S + 1; }

// forward / weight-gradient gather: rows = output pixels, tap t -> source (r*S + kh - p, c*S + kw - p)
inline ConvGeom fwd_geom(int H, int W, int C, int K, int S) {
    ConvGeom g{};
    g.H = H; g.W = W; g.Hr = out_dim(H, K, S); g.Wr = out_dim(W, K, S);
    g.C = C; g.S = S; g.ntaps = K * K; g.OS = 0;
    for (int t = 0; t < K * K; ++t) {
        g.offh[t] = (signed char)(t / K - K / 2);
        g.offw[t] = (signed char)(t % K - K / 2);
        g.btap[t] = (signed char)t;
    }
    return finish_geom(g);
}

template <int BM_, int BN_, int WGM_, int WGN_, int NBUF_>
int nt_conv(const void* A, const void* B, void* C, int M, int N, const ConvGeom& g, int ldb, int ldc,
            const void* zero, float* stats, hipStream_t s, const void* D, const BnBwd& bnr) {
    return launch_nt<BM_, BN_, WGM_, WGN_, true, NBUF_>(A, B, C, M, N, g.ntaps * g.C, g.C, ldb, ldc, zero, stats, s, g, D,
                                                 D != nullptr ? ldc : 0, bnr);
}

inline int nt_rows_per_block(int N) { return N % 128 == 0 ? 128 : 256; }

int nt_conv_any(const void* A, const void* B, void* C, int M, int N, const ConvGeom& g_in, int ldb, int ldc,
                const void* zero, float* stats, hipStream_t s, const void* D = nullptr, const BnBwd& bnr = {}) {
    ConvGeom g = g_in;
    g.tap_inner = 1;  // tap-inner reduction order (ConvGeom::tap_inner; tap-major measured slower)
    const int K = g.ntaps * g.C;
    if (N % 128 == 0)
        return nt_single(true, K, ((M + 127) / 128) * (N / 128))
                   ? nt_conv<128, 128, 2, 2, 1>(A, B, C, M, N, g, ldb, ldc, zero, stats, s, D, bnr)
                   : nt_conv<128, 128, 2, 2, 2>(A, B, C, M, N, g, ldb, ldc, zero, stats, s, D, bnr);
    return nt_single(true, K, ((M + 255) / 256) * (N / 64))
               ? nt_conv<256, 64, 4, 1, 1>(A, B, C, M, N, g, ldb, ldc, zero, stats, s, D, bnr)
               : nt_conv<256, 64, 4, 1, 2>(A, B, C, M, N, g, ldb, ldc, zero, stats, s, D, bnr);
}

// the GEMMs of a data gradient: (row grid geometry, ntaps) per launch; S == 2 gives one per parity class
template <typename F>
int for_each_dgrad_gemm(int Nb, int H, int W, int Cin, int Cout, int K, int S, F&& f) {
    const int Ho = out_dim(H, K, S), Wo = out_dim(W, K, S), p = K / 2;
    if (S == 1) {  // flipped taps over the same grid
        ConvGeom g = fwd_geom(Ho, Wo, Cout, K, 1);
        g.Hr = H; g.Wr = W;
        for (int t = 0; t < K * K; ++t) {
            g.offh[t] = (signed char)(p - t / K);
            g.offw[t] = (signed char)(p - t % K);
        }
        return f(finish_geom(g), Nb * H * W);
    }
    // stride 2: input pixel (ih, iw) = (2a + ph, 2b + pw) receives dy at ho = (ih + p - kh) / 2 for the taps kh
    // with (ih + p - kh) even; one GEMM per parity class, rows scattered back into dx.
    for (int ph = 0; ph < 2; ++ph)
        for (int pw = 0; pw < 2; ++pw) {
            ConvGeom g{};
            g.H = Ho; g.W = Wo; g.C = Cout; g.S = 1;
            g.Hr = (H - ph + 1) / 2; g.Wr = (W - pw + 1) / 2;
            g.Hc = H; g.Wc = W; g.OS = 2; g.oph = ph; g.opw = pw;
            int nt = 0;
            for (int kh = 0; kh < K; ++kh) {
                if ((ph + p - kh) & 1) continue;
                for (int kw = 0; kw < K; ++kw) {
                    if ((pw + p - kw) & 1) continue;
                    g.offh[nt] = (signed char)((ph + p - kh) / 2);  // ho = a + offh
                    g.offw[nt] = (signed char)((pw + p - kw) / 2);
                    g.btap[nt] = (signed char)(kh * K + kw);
                    ++nt;
                }
            }
            g.ntaps = nt;
            if (nt == 0 || g.Hr <= 0 || g.Wr <= 0) continue;
            const int rc = f(finish_geom(g), Nb * g.Hr * g.Wr);
            if (rc) return rc;
        }
    return 0;
}
}  // namespace

extern "C" {

// y[Nb*Ho*Wo][Cout] = conv(x[Nb*H*W][Cin], Wf[Cout][K*K][Cin]); stats as in plx_gemm_nt
int plx_conv_fwd(const void* x, const void* wf, void* y, int Nb, int H, int W, int Cin, int Cout, int K, int S,
                 const void* zero, float* stats, void* stream) {
    if (Nb <= 0 || Cin % 64 || Cout % 64 || (K != 1 && K != 3) || (S != 1 && S != 2)) return -1;
    const ConvGeom g = fwd_geom(H, W, Cin, K, S);
    return nt_conv_any(x, wf, y, Nb * g.Hr * g.Wr, Cout, g, K * K * Cin, Cout, zero, stats, (hipStream_t)stream);
}

// dx[Nb*H*W][Cin] = conv^T(dy[Nb*Ho*Wo][Cout], Wd[Cin][K*K][Cout]) (+ D, bf16 [Nb*H*W][Cin], may alias dx).
// For S == 2 and K == 1 only the even-even pixels are written: the caller passes a zeroed dx, or D == dx (the
// other rows then keep D).  bnr (nullable): fused BatchNorm-backward partials of dx, one block row per GEMM
// block over all launches (plx_conv_dgrad_blocks of them); only valid when every pixel is written (not S2/K1).
int plx_conv_dgrad(const void* dy, const void* wd, void* dx, int Nb, int H, int W, int Cin, int Cout, int K, int S,
                   const void* zero, const void* D, const BnBwd* bnr, void* stream) {
    if (Nb <= 0 || Cin % 64 || Cout % 64 || (K != 1 && K != 3) || (S != 1 && S != 2)) return -1;
    // a strided 1x1 writes the even-even pixels only: its partials can only continue a buffer whose other rows
    // (blk_off before it) cover the rest (BnBwd::skip_w)
    if (bnr != nullptr && (S == 2 && K == 1) && bnr->blk_off == 0) return -1;
    hipStream_t st = (hipStream_t)stream;
    BnBwd b = bnr != nullptr ? *bnr : BnBwd{};
    const int rpb = nt_rows_per_block(Cin);
    return for_each_dgrad_gemm(Nb, H, W, Cin, Cout, K, S, [&](const ConvGeom& g, int M) {
        const int rc = nt_conv_any(dy, wd, dx, M, Cin, g, K * K * Cout, Cin, zero, nullptr, st, D, b);
        b.blk_off += (M + rpb - 1) / rpb;
        return rc;
    });
}

// number of BatchNorm-partial block rows plx_conv_dgrad writes (part_ld for its bnr)
int plx_conv_dgrad_blocks(int Nb, int H, int W, int Cin, int Cout, int K, int S) {
    int total = 0;
    const int rpb = nt_rows_per_block(Cin);
    const int rc = for_each_dgrad_gemm(Nb, H, W, Cin, Cout, K, S, [&](const ConvGeom&, int M) {
        total += (M + rpb - 1) / rpb;
        return 0;
    });
    return rc ? rc : total;
}

long plx_conv_wgrad_workspace(int Nb, int H, int W, int Cin, int Cout, int K, int S, int num_cus) {
    return plx_gemm_tn_workspace(Nb * out_dim(H, K, S) * out_dim(W, K, S), Cout, K * K * Cin, num_cus);
}

// dW[co][tap][ci] (fp32, (+)=) = sum over output pixels m of dy[m][co] * x[gather_tap(m)][ci]
int plx_conv_wgrad(const void* dy, const void* x, float* dw, float* ws, int Nb, int H, int W, int Cin, int Cout, int K,
                   int S, const void* zero, int num_cus, int accumulate, void* stream) {
    if (Nb <= 0 || Cin % 64 || Cout % 64 || (K != 1 && K != 3) || (S != 1 && S != 2)) return -1;
    const ConvGeom g = fwd_geom(H, W, Cin, K, S);
    const int M = Nb * g.Hr * g.Wr;
    return run_tn<true>(dy, x, dw, ws, M, Cout, K * K * Cin, Cout, Cin, K * K * Cin, zero, num_cus, accumulate,
                        (hipStream_t)stream, g);
}

int plx_weight_prepk(const float* w, long s_co, long s_ci, long s_kh, long s_kw, void* wf, void* wd, int cout, int cin,
                     int K, void* stream) {
    const long total = (long)cout * cin * K * K;
    int blocks = (int)((total + 255) / 256);
    if (blocks > 4096) blocks = 4096;
    hipLaunchKernelGGL(weight_prepk_kernel, dim3(blocks), dim3(256), 0, (hipStream_t)stream, w, s_co, s_ci, s_kh, s_kw,
                       (__bf16*)wf, (__bf16*)wd, cout, cin, K);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// segs: device array of nseg WSeg records (40 bytes each: int64 src, dst_f, dst_d; int32 cout, cin, taps, tile0),
// sorted by tile0, tile0[0] == 0; total_tiles = sum over segments of taps * ceil(cout/32) * ceil(cin/32)
int plx_weight_prep_all(const float* base, void* wf, void* wd, const void* segs, int nseg, int total_tiles,
                        void* stream) {
    static_assert(sizeof(WSeg) == 40, "WSeg layout is shared with ops/wcache.py");
    if (nseg <= 0 || total_tiles <= 0) return -1;
    hipLaunchKernelGGL(weight_prep_all_kernel, dim3(total_tiles), dim3(256), 0, (hipStream_t)stream, base,
                       (__bf16*)wf, (__bf16*)wd, (const WSeg*)segs, nseg);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// ---- ResNet stem: 7x7 / stride 2 / pad 3 convolution, 3 -> 64 channels, as an MFMA GEMM with K = 256.
// The input is packed once per step into "super-pixels" of 2 horizontally adjacent pixels x 4 channels (3 + a zero)
// = 16 B, so one LDS-DMA chunk is one super-pixel and a 7 x 4 window of them (7 rows x 8 columns, the first column a
// zero-weight tap) covers an output pixel's 7 x 7 receptive field: 28 chunks = 224 reduction values, padded to 256.
// The epilogue writes the BatchNorm channel stats (as the other convolutions do), so the stem BatchNorm needs no
// statistics pass over the 112 x 112 x 64 output.
__global__ void stem_pack_input_kernel(const uint32_t* __restrict__ x, uint4* __restrict__ xp, long n_sp) {
    for (long i = blockIdx.x * (long)blockDim.x + threadIdx.x; i < n_sp; i += (long)gridDim.x * blockDim.x) {
        const uint32_t d0 = x[3 * i], d1 = x[3 * i + 1], d2 = x[3 * i + 2];  // 2 pixels x 3 bf16, 4-byte aligned
        xp[i] = make_uint4(d0, d1 & 0xffffu, (d1 >> 16) | (d2 << 16), d2 >> 16);
    }
}

// wp[co][t * 8 + px * 4 + ch] = w[co][ch][t / 4][2 (t % 4) - 1 + px]   (0 outside the 7x7x3 kernel and for t >= 28)
__global__ void stem_pack_weight_kernel(const float* __restrict__ w, long s_co, long s_ci, long s_kh, long s_kw,
                                        __bf16* __restrict__ wp, int cout) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= cout * 256) return;
    const int co = e >> 8, k = e & 255, t = k >> 3, px = (k >> 2) & 1, ch = k & 3;
    const int kh = t >> 2, kw = 2 * (t & 3) - 1 + px;
    const bool ok = t < 28 && ch < 3 && kw >= 0 && kw < 7;
    wp[e] = (__bf16)(ok ? w[co * s_co + ch * s_ci + kh * s_kh + kw * s_kw] : 0.f);
}

// dw[co][ci][kh][kw] (+)= packed[co][(kh * 4 + j) * 8 + px * 4 + ci] with kw = 2j - 1 + px
__global__ void stem_unpack_wgrad_kernel(const float* __restrict__ packed, float* __restrict__ dw, long s_co, long s_ci,
                                         long s_kh, long s_kw, int accumulate) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    if (e >= 64 * 147) return;
    const int co = e / 147, r = e % 147, ci = r / 49, kh = (r % 49) / 7, kw = r % 7;
    const int j = (kw + 1) >> 1, px = (kw + 1) & 1;
    const float v = packed[co * 256 + (kh * 4 + j) * 8 + px * 4 + ci];
    float* d = dw + co * s_co + ci * s_ci + kh * s_kh + kw * s_kw;
    *d = accumulate ? *d + v : v;
}

int plx_weight_prep(const float* w, void* wb, void* wt, int cout, int cin, void* stream) {
    dim3 grid((cin + 31) / 32, (cout + 31) / 32);
    hipLaunchKernelGGL(weight_prep_kernel, grid, dim3(256), 0, (hipStream_t)stream, w, (__bf16*)wb, (__bf16*)wt, cout,
                       cin);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

}  // extern "C"

extern "C" {

// x: NHWC bf16 [N][H][W][3] (H, W even) -> xp [N][H][W/2][8] bf16 super-pixels
int plx_stem_pack_input(const void* x, void* xp, int N, int H, int W, void* stream) {
    if (N <= 0 || H <= 0 || W <= 0 || (W & 1)) return -1;
    const long n_sp = (long)N * H * (W / 2);
    long blocks = (n_sp + 255) / 256;
    if (blocks > 8192) blocks = 8192;
    hipLaunchKernelGGL(stem_pack_input_kernel, dim3((int)blocks), dim3(256), 0, (hipStream_t)stream, (const uint32_t*)x,
                       (uint4*)xp, n_sp);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// fp32 weight [cout][3][7][7] (any strides) -> bf16 wp [cout][256]
int plx_stem_pack_weight(const float* w, long s_co, long s_ci, long s_kh, long s_kw, void* wp, int cout, void* stream) {
    hipLaunchKernelGGL(stem_pack_weight_kernel, dim3((cout * 256 + 255) / 256), dim3(256), 0, (hipStream_t)stream, w,
                       s_co, s_ci, s_kh, s_kw, (__bf16*)wp, cout);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

constexpr int kStemWgradBpc = 4;  // blocks per CU for the stem's weight gradient (alone on the GPU at the end)

// slab planes (slices + reducer groups) of the stem's weight gradient under either plan
static long stem_slabs(int M, int num_cus) {
    const TnPlan p = tn_plan(M, 64, 256, num_cus, kStemWgradBpc);
    const TnPlan q = tn2_plan(M, 64, 256, num_cus, v2_cfg(64, 256));
    const TnPlan r = tn2_plan(M, 64, 256, num_cus, v2_cfg(64, 256), kStemV2Bpc);
    const long a = p.slices + (p.groups > 1 ? p.groups : 0), b = q.slices + (q.groups > 1 ? q.groups : 0);
    const long c = r.slices + (r.groups > 1 ? r.groups : 0);
    return a > b ? (a > c ? a : c) : (b > c ? b : c);
}

// floats of workspace plx_stem_conv_wgrad needs: the slab reduction's (as plx_gemm_tn_workspace) + dW packed [64][256]
long plx_stem_conv_wgrad_workspace(int N, int H, int W, int num_cus) {
    const int M = N * ((H - 1) / 2 + 1) * ((W - 1) / 2 + 1);
    return stem_slabs(M, num_cus) * 64 * 256 + 64 * 256;
}

// dw (fp32 [64][3][7][7], strides s_*; (+)= with accumulate) = the stem's weight gradient from dy (NHWC bf16
// [N][Ho][Wo][64]) and the packed input xp: a TN GEMM over the output pixels gathering the super-pixel window
// (stage_rows GATHER 2), then unpacked from the [64][28 x 8] chunk layout
int plx_stem_conv_wgrad(const void* dy, const void* xp, float* dw, long s_co, long s_ci, long s_kh, long s_kw,
                        float* ws, int N, int H, int W, const void* zero, int num_cus, int accumulate, void* stream) {
    if (N <= 0 || H <= 0 || W <= 0 || (W & 1)) return -1;
    ConvGeom g{};
    g.H = H;
    g.W = W / 2;
    g.Hr = (H - 1) / 2 + 1;
    g.Wr = (W - 1) / 2 + 1;
    g.mWr = div_magic(g.Wr);
    g.mHr = div_magic(g.Hr);
    const int M = N * g.Hr * g.Wr;
    float* packed = ws + stem_slabs(M, num_cus) * 64 * 256;
    hipStream_t s = (hipStream_t)stream;
    const int rc = run_tn<2>(dy, xp, packed, ws, M, 64, 256, 64, 8, 256, zero, num_cus, 0, s, g, kStemWgradBpc);
    if (rc) return rc;
    hipLaunchKernelGGL(stem_unpack_wgrad_kernel, dim3((64 * 147 + 255) / 256), dim3(256), 0, s, packed, dw, s_co, s_ci,
                       s_kh, s_kw, accumulate);
    return hipGetLastError() == hipSuccess ? 0 : -3;
}

// rows of plx_stem_conv_fwd's channel-stat partials: stats is fp32 [2][ceil(M / 256)][64], M = N * Ho * Wo
int plx_stem_conv_rows_per_block() { return 256; }

// y[N*Ho*Wo][64] (NHWC bf16) = conv7x7/s2/p3(x) from the packed input xp (plx_stem_pack_input) and weights wp
// (plx_stem_pack_weight); stats (nullable) as plx_gemm_nt's
int plx_stem_conv_fwd(const void* xp, const void* wp, void* y, int N, int H, int W, const void* zero, float* stats,
                      void* stream) {
    if (N <= 0 || H <= 0 || W <= 0 || (W & 1)) return -1;
    ConvGeom g{};
    g.H = H;
    g.W = W / 2;                                    // super-pixel columns
    g.Hr = (H - 1) / 2 + 1;                         // (H + 2*3 - 7) / 2 + 1
    g.Wr = (W - 1) / 2 + 1;
    g.mWr = div_magic(g.Wr);
    g.mHr = div_magic(g.Hr);
    const int M = N * g.Hr * g.Wr;
    return nt_single(true, 256, (M + 255) / 256)
               ? launch_nt<256, 64, 4, 1, 2, 1>(xp, wp, y, M, 64, 256, 8, 256, 64, zero, stats, (hipStream_t)stream, g)
               : launch_nt<256, 64, 4, 1, 2, 2>(xp, wp, y, M, 64, 256, 8, 256, 64, zero, stats, (hipStream_t)stream, g);
}

}  // extern "C"
