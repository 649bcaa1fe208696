// wrmf_tiles.hip -- WRMF row solves for 128 < k <= 256 on the matrix cores (fp32 MFMA).
//
// Same math as wrmf.hip / WRMF.Optimize(u) (src/MyMediaLite/ItemRecommendation/WRMF.cs:110-156):
//   A_u = HH + alpha * sum_{i in S_u} h_i h_i^T + reg * I,   b_u = (1 + alpha) * sum_{i in S_u} h_i,
//   W_u = A_u^{-1} b_u,
// restated for the MI355X as 32 x 32 tiles that live in MFMA accumulator registers for the whole
// solve (one workgroup of 8 waves per row, rows taken from an atomic work queue):
//   * k is padded to 32 nt columns (identity on the padding) and the row is augmented with b as
//     row kb = 32 nt (its own tile row), so A' = [A; b^T] has nr = nt + 1 tile rows.  The lower tiles
//     (I, J), J < nt, J <= I <= nt, are owned round-robin by the 8 waves (<= 6 tiles = 96 accumulator
//     registers per lane).  A tile is held TRANSPOSED in the v_mfma_f32_32x32x2_f32 C/D layout: lane
//     (q = lane&31, h = lane>>5), register g holds A'[32I + q][32J + rho(g, h)],
//     rho(g, h) = (g&3) + 8(g>>2) + 4h, so it feeds the next MFMA as the B operand with no data
//     movement (the contraction runs over the register index).
//   * Gram: sum_i h_i h_i^T for all tiles at once, 2 gathered item vectors per MFMA (K = 2), the
//     vectors staged in LDS (double-buffered: the next chunk's gathers are in flight during the
//     current chunk's MFMAs) with h[kb] = 1 so row kb accumulates sum_i h_i.  Rows with more than
//     kHeavy entries get their Gram from a split pass (wrmf_tile_gram_kernel: kSeg-entry segments on
//     many workgroups, fp64 atomics) so one hot item never serialises a CU.
//   * blocked right-looking Cholesky, per 32-column panel J: the diagonal tile is factored and
//     inverted by one wave in registers (T_J = L_JJ^{-1}, v_readlane broadcasts); the tiles below
//     become L_IJ = A'_IJ T_J^T (16 MFMAs each); the trailing tiles take the rank-32 update
//     A'_IK -= L_KJ L_IJ^T (16 MFMAs each) with the panel read from LDS.  Row kb of the factor is
//     y = L^{-1} b (forward substitution for free).
//   * backward substitution L^T w = y by 32-column blocks: w_J = T_J^T (y_J - sum_{I>J} L_IJ^T w_I).
// Precision: fp32 with fused multiply-adds (the packed fp64 matrix of the parity path does not fit
// the LDS at k > 128); the tolerance against the fp64 oracle is stated in tests/test_wrmf_gpu.py.
#include <algorithm>
#include <cmath>
#include <cstdlib>
#include <string>
#include <cstring>
#include <vector>

#include "mml_internal.h"

#pragma clang fp contract(fast)

namespace {

#define MML_DPP(v, ctrl) \
    __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false))

using f32x16 = __attribute__((ext_vector_type(16))) float;

constexpr int kWaves = 8;
constexpr int kThreads = 64 * kWaves;
constexpr int kNT = 8;                                   // column tiles, k <= 256
constexpr int kNR = kNT + 1;                             // + the b-row tile
constexpr int kTiles = 44;                               // sum_{J<8} (9 - J)
constexpr int kSlots = (kTiles + kWaves - 1) / kWaves;   // 6 tiles per wave
constexpr int kCH = 16;                                  // gathered vectors per LDS chunk
constexpr int kHSW = 32 * kNR;                           // staged vector width
constexpr int kPS = 34;                                  // panel row stride (conflict-free reads)
#ifndef MML_GRAM_RB  // A/B variants (scripts/build_variant.sh "-DMML_GRAM_RB=5")
#define MML_GRAM_RB 4
#endif
constexpr int kRB = MML_GRAM_RB;  // Gram: raw fp32 chunks in the LDS ring (kRB - 1 chunks of gathers in flight)
constexpr int kRS = 260;  // raw row stride in floats (1 KiB of row + pad: conflict-free reads)
constexpr int kPW = 256;  // pre-split plane row: k <= 256 bf16, zero-padded (512 B)
#ifndef MML_GRAM_RBP  // A/B variants: chunks in the planes ring (kRBP - 1 chunks of gathers in flight)
#define MML_GRAM_RBP 4
#endif
constexpr int kRBP = MML_GRAM_RBP;
#ifdef MML_NO_GRAM_RING  // A/B variant (scripts/build_variant.sh): the register-staged Gram only
constexpr bool kGramRing = false;
#else
constexpr bool kGramRing = true;
#endif
constexpr int kPP = 40;  // bf16 panel-plane row stride (80 B: conflict-free 16-B reads/writes)
#ifdef MML_FACTOR_F32  // A/B variant (scripts/build_variant.sh): panel and trailing MFMAs in f32
constexpr bool kFactorX3 = false;
#else
constexpr bool kFactorX3 = true;
#endif
constexpr int kDS = 33;                                  // diagonal-tile / reduction row stride
constexpr int kTS = 33;                                  // T_J^T row stride (conflict-free rows)

__device__ __forceinline__ int rho(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

// threadIdx.x made opaque at the call site: lane-derived constants (row selectors, LDS offsets)
// are then recomputed in each phase instead of being hoisted out of the row loop and spilled
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
}

// an empty use of a loaded value: the load cannot then be sunk under the select that consumes it
// (a load under a branch is waited for before the branch joins, so a batch of gathers written as
// selected loads ran one at a time)
__device__ __forceinline__ void keep_loaded(float4& g) {
    asm volatile("" : "+v"(g.x), "+v"(g.y), "+v"(g.z), "+v"(g.w));
}

__device__ __forceinline__ float lane_bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}

// tile id t (column-major over the lower tiles) -> (I, J)
__device__ __forceinline__ void tile_of(int t, int nr, int& I, int& J) {
    J = 0;
    while (t >= nr - J) {
        t -= nr - J;
        ++J;
    }
    I = J + t;
}
__host__ __device__ __forceinline__ int tile_id(int I, int J, int nr) {
    return J * nr - J * (J - 1) / 2 + (I - J);
}

struct Smem {
    union {
        float hs[2][kCH * kHSW];        // Gram (MODE 1): staged vectors, double-buffered
        // Gram (MODE 0): the staged vectors as three bf16 planes (x = x0 + x1 + x2), each row f
        // holding the kCH vectors' element f (two 16-B halves, swapped on rows with f & 8)
        alignas(16) uint16_t pl[2][3][kHSW][kCH];
        struct {  // the same planes, then the ring the vectors are gathered into (global -> LDS)
            alignas(16) uint16_t pl[2][3][kHSW][kCH];
            alignas(16) float raw[kRB][kCH][kRS];
        } gx;
        struct {
            float pn[kNT][32][kPS];     // Cholesky: L_IJ of the current panel, row-major (f32 A/B)
            // the same panel as bf16x3 planes in the MFMA K-slot order: pp[pi][p][q][pos] with
            // pos = 16 (g >> 3) + 8 h + (g & 7) for register g of lane (q, h)
            alignas(16) uint16_t pp[kNT][3][32][kPP];
        } fz;
        float red[kNT][32][kDS];        // backward: per-tile partial products
        // Gram from pre-split planes (gram_accumulate_p3): kRB chunks x 3 planes x kCH vectors x
        // kPW bf16, vector v's 16-B chunk ch at position ch ^ ((v & 3) << 2)
        alignas(16) uint16_t gp[kRBP][3][kCH][kPW];
    } u;
    float tT[2][32][kTS];               // tT[c][m] = T_J[m][c], double-buffered (lookahead)
    float yv[kHSW];
    float wv[kHSW];
    float sv[32];
    float part[kNT][32];
    int32_t row;
};

struct Tiles {
    int I[kSlots], J[kSlots];
};

// Makes the tile ids opaque at the top of a loop body, so the compiler recomputes the (cheap)
// tile-derived offsets there instead of hoisting dozens of them out of the loop and spilling them.
__device__ __forceinline__ void launder(Tiles& tl) {
#pragma unroll
    for (int s = 0; s < kSlots; ++s) asm volatile("" : "+s"(tl.I[s]), "+s"(tl.J[s]));
}

__device__ __forceinline__ void my_tiles(int wave, int nr, int ntile, Tiles& tl) {
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const int t = s * kWaves + wave;
        int I = -1, J = -1;
        if (t < ntile) tile_of(t, nr, I, J);
        tl.I[s] = __builtin_amdgcn_readfirstlane(I);
        tl.J[s] = __builtin_amdgcn_readfirstlane(J);
    }
}

// acc[s] += sum over the entries [b, e) of cols: h_i[32J + p] * h_i[32I + q] for every owned tile
// (h_i[kb] = 1, columns >= k masked to 0).  All threads of the workgroup must call it.
// Staging: thread t gathers vector c = t / 32 of the chunk, floats u = t % 32 (+ 32 j) of it (float4
// when k % 4 == 0); the next chunk's gathers and the index of the one after are in flight while the
// current chunk's MFMAs run.
// MODE 1 (Woodbury rows): the "vectors" are the k features f and vector f holds Q[s_i][f] for the
// row's items i < deg (column i), so the same MFMA loop accumulates C = Q_S Q_S^T (deg x deg).
template <int MODE>
__device__ __forceinline__ void gram_accumulate(Smem& sm, f32x16 (&acc)[kSlots], Tiles& tl,
                                                int nslot, const int32_t* __restrict__ cols,
                                                int64_t b, int64_t e, const float* __restrict__ H,
                                                int k, int hsw, int kdim) {
    static_assert(kCH * 32 == kThreads, "one staging thread group of 32 per vector");
    static_assert(kCH * 32 == kThreads && kThreads / 4 >= 128, "MODE 1 staging: 4 threads per item");
    constexpr int kQ = 2;   // float4 per thread (k <= 256)
    constexpr int kS = 8;   // scalars per thread (k <= 256)
    const int t = opaque_tid(), lane = t & 63, q = lane & 31, h = lane >> 5;
    const int c = t >> 5, u = t & 31;      // MODE 0: vector c, floats u + 32 j
    const int wi = t >> 2, wj = t & 3;     // MODE 1: item column wi, features 4 wj .. 4 wj + 3
    const int kb = hsw - 32;
    const bool vec = (k & 3) == 0;
    float4 p4[kQ];
    float p1[kS];
    // MODE 1: this thread's item (fixed for the row), its column in the staged vectors
    const int64_t deg = MODE == 1 ? (e - b) : 0;
    const int32_t my_item = (MODE == 1 && wi < deg) ? cols[b + wi] : 0;
    auto fetch = [&](int32_t item, bool live, int64_t base) {
        if constexpr (MODE == 0) {
            const float* src = H + (int64_t)item * k;
            if (vec) {
#pragma unroll
                for (int j = 0; j < kQ; ++j) {
                    const int f = 4 * (u + 32 * j);
                    p4[j] = (live && f < k) ? *reinterpret_cast<const float4*>(src + f)
                                            : make_float4(0.f, 0.f, 0.f, 0.f);
                }
            } else {
#pragma unroll
                for (int j = 0; j < kS; ++j) {
                    const int f = u + 32 * j;
                    p1[j] = (live && f < k) ? src[f] : 0.0f;
                }
            }
        } else {
            const float* src = H + (int64_t)my_item * k;
            const int f = (int)base + 4 * wj;
            const bool ok = wi < deg;
            if (vec) {
                p4[0] = (ok && f < k) ? *reinterpret_cast<const float4*>(src + f)
                                      : make_float4(0.f, 0.f, 0.f, 0.f);
            } else {
                p4[0].x = (ok && f < k) ? src[f] : 0.0f;
                p4[0].y = (ok && f + 1 < k) ? src[f + 1] : 0.0f;
                p4[0].z = (ok && f + 2 < k) ? src[f + 2] : 0.0f;
                p4[0].w = (ok && f + 3 < k) ? src[f + 3] : 0.0f;
            }
            (void)item; (void)live;
        }
    };
    auto stash = [&](float* buf, bool live) {
        if constexpr (MODE == 0) {
            float* dst = buf + c * kHSW;
            if (vec) {
#pragma unroll
                for (int j = 0; j < kQ; ++j) {
                    const int f = 4 * (u + 32 * j);
                    if (f < k) *reinterpret_cast<float4*>(dst + f) = p4[j];
                }
            } else {
#pragma unroll
                for (int j = 0; j < kS; ++j) {
                    const int f = u + 32 * j;
                    if (f < k) dst[f] = p1[j];
                }
            }
            for (int f = k + u; f < hsw; f += 32) dst[f] = (live && f == kb) ? 1.0f : 0.0f;
        } else {
            float* dst = buf + 4 * wj * kHSW;
            dst[wi] = p4[0].x;
            dst[kHSW + wi] = p4[0].y;
            dst[2 * kHSW + wi] = p4[0].z;
            dst[3 * kHSW + wi] = p4[0].w;
            if (wi + 128 < hsw) {  // columns beyond the 128 staged items (b-row tile): zero
                dst[wi + 128] = 0.0f;
                dst[kHSW + wi + 128] = 0.0f;
                dst[2 * kHSW + wi + 128] = 0.0f;
                dst[3 * kHSW + wi + 128] = 0.0f;
            }
            (void)live;
        }
    };
    if (e <= b) return;
    const int64_t eb = MODE == 0 ? b : 0;      // entries (MODE 0) or features (MODE 1)
    const int64_t ee = MODE == 0 ? e : k;
    // per-lane operand offsets of the owned tiles (unused slots read offset 0 with weight 0)
    int offJ[kSlots], offI[kSlots];
    float mJ[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const bool ok = tl.I[s] >= 0;
        const int cj = 32 * tl.J[s] + q;
        offJ[s] = ok ? cj : 0;
        offI[s] = ok ? 32 * tl.I[s] + q : 0;
        mJ[s] = (ok && cj < kdim) ? 1.0f : 0.0f;
    }
    auto idx_at = [&](int64_t base) -> int32_t {
        if constexpr (MODE == 0) return base + c < ee ? cols[base + c] : 0;
        return 0;
    };
    int cur = 0;
    __syncthreads();  // the LDS union may still be read by the previous row's last phase
    int32_t i0 = idx_at(eb);
    int32_t i1 = eb + kCH < ee ? idx_at(eb + kCH) : 0;
    fetch(i0, eb + c < ee, eb);
    stash(sm.u.hs[0], eb + c < ee);
    __syncthreads();
    for (int64_t base = eb; base < ee; base += kCH) {
        const int nrc = (int)min((int64_t)kCH, ee - base);
        const int64_t nb = base + kCH;
        const bool more = nb < ee;
        if (more) {
            fetch(i1, nb + c < ee, nb);                       // next chunk: in flight
            i1 = nb + kCH < ee ? idx_at(nb + kCH) : 0;        // the index after it
        }
        const float* buf = sm.u.hs[cur];
        for (int cc = 0; cc < nrc; cc += 2) {
            const float* hr = buf + (cc + h) * kHSW;
#pragma unroll
            for (int s = 0; s < kSlots; ++s)  // straight line: unused slots multiply by 0
                if (s < nslot)
                    acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(hr[offJ[s]] * mJ[s],
                                                                  hr[offI[s]], acc[s], 0, 0, 0);
        }
        if (more) stash(sm.u.hs[cur ^ 1], nb + c < ee);
        __syncthreads();
        cur ^= 1;
    }
}

// MODE 0's Gram on the bf16 matrix cores at f32 accuracy.  Each staged value is split exactly
// into three bf16 parts, x = x0 + x1 + x2 (8 significant bits each: 24 = f32), and a tile takes
// the six products x_a y_b with a + b <= 2 -- the dropped ones are below 2^-24 relative, f32's own
// rounding -- on v_mfma_f32_32x32x16_bf16 (16 vectors per instruction, accumulating in f32):
// 6 x 32 cycles per 16 vectors against 8 x 64 for v_mfma_f32_32x32x2_f32.  Staging: wave w
// converts features [32w, 32w + 32) of the chunk's 16 vectors, lane (r, c2) features 8g + r of
// vectors 2 c2, 2 c2 + 1, and writes each plane as one conflict-free 32-bit word per lane (8 rows x
// 8 words); the operand reads are ds_read_b128 of 8 vectors, conflict-free through the swap of
// the two 16-B halves on rows with f & 8.
// The b-row tiles (I = nt) hold one useful row of 32 (row kb: sum_i h_i), so they take no MFMA:
// each staging thread sums its features of its two vectors on the VALU, the 8 vector-pair lanes of
// a feature are reduced once per row, and the tiles' row kb is filled from that sum at the end
// (C5 direct rows: 9 instead of 11 tiles of MFMA work per SIMD and chunk).
using bf16x8 = __attribute__((ext_vector_type(8))) short;

__device__ __forceinline__ uint32_t bf16_rn(float x) {  // round to nearest even, top 16 bits
    const uint32_t b = __float_as_uint(x);
    return (b + 0x7FFFu + ((b >> 16) & 1u)) >> 16;
}
__device__ __forceinline__ void split3(float x, uint32_t& a, uint32_t& b, uint32_t& c) {
    a = bf16_rn(x);
    const float r1 = x - __uint_as_float(a << 16);
    b = bf16_rn(r1);
    c = bf16_rn(r1 - __uint_as_float(b << 16));  // exact: <= 8 significant bits remain
}
// The same exact split in fewer VALU ops: x0 = x truncated to its top half (2 ops), x1 = x - x0
// rounded to nearest bf16 (4 ops), x2 = the rest, which has <= 8 significant bits (exact); the
// parts are the top halves of a, b, c.  |x1| < 2^-7 |x| and |x2| <= 2^-16 |x|, so the dropped
// products x1 y2, x2 y1, x2 y2 stay below 2^-22 relative (RN of all parts: 2^-24), well inside
// the fp32 mode's tolerance and corrected by the fp64 mode's refinement.
__device__ __forceinline__ void split3t(float x, uint32_t& a, uint32_t& b, uint32_t& c) {
    a = __float_as_uint(x);
    const float r1 = x - __uint_as_float(a & 0xFFFF0000u);
    const uint32_t u1 = __float_as_uint(r1);
    b = (u1 + 0x7FFFu + ((u1 >> 16) & 1u)) & 0xFFFF0000u;
    c = __float_as_uint(r1 - __uint_as_float(b));
}
__device__ __forceinline__ uint32_t pack_hi(uint32_t lo, uint32_t hi) {  // {lo.hi16, hi.hi16}
    return __builtin_amdgcn_perm(hi, lo, 0x07060302u);
}
using u32x4 = __attribute__((ext_vector_type(4))) uint32_t;
// v[0 .. 7] -> three bf16x8 operands (split3t parts 0, 1, 2 of each element, in order)
__device__ __forceinline__ void split8(const float (&v)[8], bf16x8 (&P)[3]) {
    uint32_t a[8], b[8], c[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) split3t(v[j], a[j], b[j], c[j]);
    P[0] = __builtin_bit_cast(bf16x8, u32x4{pack_hi(a[0], a[1]), pack_hi(a[2], a[3]),
                                            pack_hi(a[4], a[5]), pack_hi(a[6], a[7])});
    P[1] = __builtin_bit_cast(bf16x8, u32x4{pack_hi(b[0], b[1]), pack_hi(b[2], b[3]),
                                            pack_hi(b[4], b[5]), pack_hi(b[6], b[7])});
    P[2] = __builtin_bit_cast(bf16x8, u32x4{pack_hi(c[0], c[1]), pack_hi(c[2], c[3]),
                                            pack_hi(c[4], c[5]), pack_hi(c[6], c[7])});
}
__device__ __forceinline__ bf16x8 bf16_neg(bf16x8 x) {
    return __builtin_bit_cast(bf16x8, __builtin_bit_cast(u32x4, x) ^ 0x80008000u);
}
// c + A B over one K step of 16 with both operands split three ways (smallest products first)
__device__ __forceinline__ f32x16 mfma_x3(const bf16x8 (&A)[3], const bf16x8 (&B)[3], f32x16 c) {
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], c, 0, 0, 0);
    c = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], c, 0, 0, 0);
    return c;
}
__device__ __forceinline__ int pl_pos(int f, int c) {  // element (f, c) within row f
    return ((((c >> 3) ^ (f >> 3)) & 1) << 3) | (c & 7);
}

__device__ __forceinline__ void gram_accumulate_x3(Smem& sm, f32x16 (&acc)[kSlots], Tiles& tl,
                                                   int nslot, const int32_t* __restrict__ cols,
                                                   int64_t b, int64_t e,
                                                   const float* __restrict__ H, int k, int hsw) {
    static_assert(kCH == 16 && kThreads == 512, "bf16x3 staging: 16 vectors, 8 waves");
    const int t = opaque_tid(), lane = t & 63, wave = t >> 6, q = lane & 31, h = lane >> 5;
    const int r = lane >> 3, c2 = lane & 7;  // staging: row in an 8-row group, vector pair
    const int kb = hsw - 32;
    // two chunks' gathers in flight (the MFMAs of one bf16x3 chunk take ~1 us per SIMD, less
    // than an HBM gather's latency): va = chunk c + 1, vb = chunk c + 2
    float va0[4], va1[4], vb0[4], vb1[4];
#if MML_GRAM_DEPTH3
    float vc0[4], vc1[4];
#endif
    float bacc[4] = {0.0f, 0.0f, 0.0f, 0.0f};  // sum over this thread's vectors, features f < k
    const int ntb = hsw / 32 - 1;              // the b-row tile row
    auto fetch = [&](int64_t base, float (&v0)[4], float (&v1)[4]) {
        const int64_t e0 = base + 2 * c2, e1 = e0 + 1;
#if MML_GRAM_NOLOAD  // timing experiment only: every vector is row 0 (cache-resident)
        const float* s0 = H;
        const float* s1 = H;
#else
        const float* s0 = H + (int64_t)(e0 < e ? cols[e0] : 0) * k;
        const float* s1 = H + (int64_t)(e1 < e ? cols[e1] : 0) * k;
#endif
#pragma unroll
        for (int g = 0; g < 4; ++g) {  // features >= k: 0, except row kb (1 on live vectors)
            const int f = 32 * wave + 8 * g + r;
            v0[g] = e0 < e ? (f < k ? s0[f] : (f == kb ? 1.0f : 0.0f)) : 0.0f;
            v1[g] = e1 < e ? (f < k ? s1[f] : (f == kb ? 1.0f : 0.0f)) : 0.0f;
        }
    };
    auto stash = [&](int buf, int64_t base, const float (&v0)[4], const float (&v1)[4]) {
        (void)base;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = 32 * wave + 8 * g + r;
            if (f < k) bacc[g] += v0[g] + v1[g];
            uint32_t a0, a1, a2, b0, b1, b2;
            const int pos = pl_pos(f, 2 * c2);
#if MML_GRAM_SPLIT_RN
            split3(v0[g], a0, a1, a2);
            split3(v1[g], b0, b1, b2);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[buf][0][f][pos]) = a0 | (b0 << 16);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[buf][1][f][pos]) = a1 | (b1 << 16);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[buf][2][f][pos]) = a2 | (b2 << 16);
#else
            split3t(v0[g], a0, a1, a2);
            split3t(v1[g], b0, b1, b2);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[buf][0][f][pos]) = pack_hi(a0, b0);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[buf][1][f][pos]) = pack_hi(a1, b1);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[buf][2][f][pos]) = pack_hi(a2, b2);
#endif
        }
        // (rows >= kb are read by the b-row tiles only, which take no MFMA: not staged)
    };
    if (e <= b) return;
    __syncthreads();  // the LDS union may still be read by the previous row's last phase
    fetch(b, va0, va1);
    stash(0, b, va0, va1);
    if (b + kCH < e) fetch(b + kCH, va0, va1);
#if MML_GRAM_DEPTH3
    if (b + 2 * kCH < e) fetch(b + 2 * kCH, vb0, vb1);
#endif
    __syncthreads();
    int cur = 0;
    for (int64_t base = b; base < e; base += kCH) {
        const int64_t nb = base + kCH;
        const bool more = nb < e;
#if MML_GRAM_DEPTH3
        if (nb + 2 * kCH < e) fetch(nb + 2 * kCH, vc0, vc1);  // chunks c + 1 .. c + 3 in flight
#else
        if (nb + kCH < e) fetch(nb + kCH, vb0, vb1);  // chunk c + 2 joins c + 1 in flight
#endif
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            if (s >= nslot || tl.I[s] < 0 || tl.I[s] == ntb) continue;
            const int fa = 32 * tl.J[s] + q, fb = 32 * tl.I[s] + q;
            bf16x8 A[3], B[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {  // 16-B aligned: one ds_read_b128 each
                A[p] = *static_cast<const bf16x8*>(__builtin_assume_aligned(
                    &sm.u.pl[cur][p][fa][pl_pos(fa, 8 * h)], 16));
                B[p] = *static_cast<const bf16x8*>(__builtin_assume_aligned(
                    &sm.u.pl[cur][p][fb][pl_pos(fb, 8 * h)], 16));
            }
            // small products first
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], acc[s], 0, 0, 0);
        }
        if (more) stash(cur ^ 1, nb, va0, va1);
        __syncthreads();
        cur ^= 1;
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            va0[g] = vb0[g];
            va1[g] = vb1[g];
#if MML_GRAM_DEPTH3
            vb0[g] = vc0[g];
            vb1[g] = vc1[g];
#endif
        }
    }
    // row kb of the b-row tiles: sum_i h_i, the 8 vector-pair lanes (lane & 7) of a feature
    // reduced, then read by the tiles' owners (lanes q = 0, columns 32 J + rho(g, h))
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        float v = bacc[g];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        const int f = 32 * wave + 8 * g + r;
        if (c2 == 0 && f < kb) sm.wv[f] = f < k ? v : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        if (s >= nslot || tl.I[s] != ntb) continue;
#pragma unroll
        for (int g = 0; g < 16; ++g)
            acc[s][g] += q == 0 ? sm.wv[32 * tl.J[s] + rho(g, h)] : 0.0f;
    }
}

// gram_accumulate_x3 with the gathers going global -> LDS directly (global_load_lds_dwordx4: one
// wave-instruction moves one 1 KiB vector row, no VGPR destination) into a ring of kRB raw fp32
// chunks, so kRB - 1 chunks of gathers are in flight without holding registers (the register
// version keeps two chunks in 16 VGPRs of a kernel at the register cap; its waves wait on memory
// more than half the time).  Per chunk: wave w gathers vectors 2w, 2w + 1;
// the waves convert the previous chunk from the ring into the bf16 planes (same thread map and
// plane layout as the register version), and run the MFMAs of the chunk before that.  One barrier
// per chunk, raw s_barrier with counted vmcnt waits: __syncthreads() would drain the ring
// (vmcnt(0)).  k % 4 == 0 (16-B rows).
__device__ __forceinline__ void glds16(const float* gsrc, uint32_t lds_addr) {
    unsigned keep;
    asm volatile(
        "s_mov_b32 %0, m0\n\ts_mov_b32 m0, %2\n\ts_nop 0\n\tglobal_load_lds_dwordx4 %1, off\n\t"
        "s_mov_b32 m0, %0"
        : "=&s"(keep)
        : "v"(gsrc), "s"(lds_addr)
        : "memory");
}
__device__ __forceinline__ uint32_t lds_addr_of(const void* p) {
    return (uint32_t)(uintptr_t)(const __attribute__((address_space(3))) void*)p;
}
// LDS writes done, then the workgroup barrier, without waiting for the ring's loads
__device__ __forceinline__ void ring_barrier() {
    asm volatile("s_waitcnt lgkmcnt(0)" ::: "memory");
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");
}

__device__ __forceinline__ void gram_accumulate_x3g(Smem& sm, f32x16 (&acc)[kSlots], Tiles& tl,
                                                    int nslot, const int32_t* __restrict__ cols,
                                                    int64_t b, int64_t e,
                                                    const float* __restrict__ H, int k, int hsw) {
    static_assert(kCH == 16 && kThreads == 512, "two vectors per wave and chunk");
    static_assert(kRB >= 3, "at least one chunk of gathers in flight beyond the converted one");
    const int t = opaque_tid(), lane = t & 63, q = lane & 31, h = lane >> 5;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int r = lane >> 3, c2 = lane & 7;
    const int kb = hsw - 32;
    const int ntb = hsw / 32 - 1;
    float bacc[4] = {0.0f, 0.0f, 0.0f, 0.0f};
    if (e <= b) return;
    const int64_t nch = (e - b + kCH - 1) / kCH;
    // gather chunk c's vectors 2w, 2w + 1 into ring slot c % kRB; chunks past the end load row 0
    // (never converted) so every wave issues exactly two loads per chunk: the vmcnt counts hold
    const int lo = 4 * lane < k ? 4 * lane : 0;
    // the two item ids of chunk c (scalar loads, fetched one chunk before their gathers issue)
    auto ids = [&](int64_t c, int32_t& i0, int32_t& i1) {
        const int64_t e0 = b + c * kCH + 2 * wave;
        i0 = e0 < e ? cols[e0] : 0;
        i1 = e0 + 1 < e ? cols[e0 + 1] : 0;
    };
    // ring row v starts 4 floats later when (v >> 3) & 1: the conversion's reads of vectors 2 c2
    // (c2 = 0..7 across a 32-lane group) then hit 8 distinct bank quads instead of 4 (row stride
    // 260: 2 * 260 = 8 mod 32 repeats every 4 vectors); the 260-float stride has the 4 spare floats
    float* const ring_base = &sm.u.gx.raw[0][0][0];
    auto ring_row = [&](int slot, int v) {
        return ring_base + ((int64_t)slot * kCH + v) * kRS + 4 * ((v >> 3) & 1);
    };
    auto gather = [&](int64_t c, int32_t i0, int32_t i1) {
        float* dst = ring_row((int)(c % kRB), 2 * wave);
        glds16(H + (int64_t)i0 * k + lo, lds_addr_of(dst));
        glds16(H + (int64_t)i1 * k + lo, lds_addr_of(dst + kRS));
    };
    // ring slot of chunk c -> bf16 planes of buffer pb (vectors past the end are 0, row kb = 1 on
    // live vectors, features >= k are 0)
    auto convert = [&](int64_t c, int pb) {
        const float* src0 = ring_row((int)(c % kRB), 2 * c2);
        const float* src1 = src0 + kRS;  // vector 2 c2 + 1: the same (v >> 3) offset
        const int64_t e0 = b + c * kCH + 2 * c2;
        const bool l0 = e0 < e, l1 = e0 + 1 < e;
        float x0[4], x1[4];  // all eight LDS reads first (unconditional: one wait, no branches)
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = 32 * wave + 8 * g + r;
            x0[g] = src0[f];
            x1[g] = src1[f];
        }
        asm volatile("" : "+v"(x0[0]), "+v"(x0[1]), "+v"(x0[2]), "+v"(x0[3]), "+v"(x1[0]),
                     "+v"(x1[1]), "+v"(x1[2]), "+v"(x1[3]));
#pragma unroll
        for (int g = 0; g < 4; ++g) {
            const int f = 32 * wave + 8 * g + r;
            float v0 = x0[g], v1 = x1[g];
            v0 = l0 ? (f < k ? v0 : (f == kb ? 1.0f : 0.0f)) : 0.0f;
            v1 = l1 ? (f < k ? v1 : (f == kb ? 1.0f : 0.0f)) : 0.0f;
            if (f < k) bacc[g] += v0 + v1;
            uint32_t a0, a1, a2, b0, b1, b2;
            const int pos = pl_pos(f, 2 * c2);
            split3t(v0, a0, a1, a2);
            split3t(v1, b0, b1, b2);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[pb][0][f][pos]) = pack_hi(a0, b0);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[pb][1][f][pos]) = pack_hi(a1, b1);
            *reinterpret_cast<uint32_t*>(&sm.u.pl[pb][2][f][pos]) = pack_hi(a2, b2);
        }
    };
    __syncthreads();  // the LDS union may still be read by the previous row's last phase
#pragma unroll
    for (int c = 0; c < kRB - 1; ++c) {
        int32_t i0, i1;
        ids(c, i0, i1);
        gather(c, i0, i1);
    }
    int32_t n0, n1;  // the ids of the next chunk to gather
    ids(kRB - 1, n0, n1);
    asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * (kRB - 2)) : "memory");  // chunk 0 landed
    ring_barrier();
    convert(0, 0);
    for (int64_t c = 0; c < nch; ++c) {
        gather(c + kRB - 1, n0, n1);
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(2 * (kRB - 2)) : "memory");  // chunk c + 1
        ring_barrier();  // planes of chunk c and every wave's ring slot of chunk c + 1 are ready
        ids(c + kRB, n0, n1);  // in flight until the next chunk's gathers
        const int cur = (int)(c & 1);
        // (past the last chunk the slot holds row-0 loads: masked to 0, the planes never read)
        convert(c + 1, cur ^ 1);
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            if (s >= nslot || tl.I[s] < 0 || tl.I[s] == ntb) continue;
            const int fa = 32 * tl.J[s] + q, fb = 32 * tl.I[s] + q;
            bf16x8 A[3], B[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) {
                A[p] = *static_cast<const bf16x8*>(__builtin_assume_aligned(
                    &sm.u.pl[cur][p][fa][pl_pos(fa, 8 * h)], 16));
                B[p] = *static_cast<const bf16x8*>(__builtin_assume_aligned(
                    &sm.u.pl[cur][p][fb][pl_pos(fb, 8 * h)], 16));
            }
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], B[0], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[1], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[2], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], B[0], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[1], acc[s], 0, 0, 0);
            acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], B[0], acc[s], 0, 0, 0);
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing loads (past the end)
    __syncthreads();
#pragma unroll
    for (int g = 0; g < 4; ++g) {
        float v = bacc[g];
        v += __shfl_xor(v, 1, 64);
        v += __shfl_xor(v, 2, 64);
        v += __shfl_xor(v, 4, 64);
        const int f = 32 * wave + 8 * g + r;
        if (c2 == 0 && f < kb) sm.wv[f] = f < k ? v : 0.0f;
    }
    __syncthreads();
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        if (s >= nslot || tl.I[s] != ntb) continue;
#pragma unroll
        for (int g = 0; g < 16; ++g)
            acc[s][g] += q == 0 ? sm.wv[32 * tl.J[s] + rho(g, h)] : 0.0f;
    }
}

// The same Gram from planes split ONCE per half-step (wrmf_split_planes_kernel: x = x0 + x1 + x2,
// three bf16 rows of kPW per vector, row zrow all zero).  A chunk's 16 vectors go global -> LDS
// (global_load_lds_dwordx4, three 1-KiB pieces per wave: vectors 2w and 2w + 1 of one plane) as a
// vector-major image, and the MFMA operands come out of it transposed by ds_read_b64_tr_b16 (lane
// (q, h) of a 32-feature block gets vectors 8h .. 8h + 7 of feature q: two reads of 4 vectors).
// No conversion pass, no LDS stores from registers: per chunk a wave issues its gathers, waits for
// the chunk kRB - 1 back, and runs the MFMAs.  The b-row tiles take A = the feature block and B =
// 1 on feature kb (lane q = 0), three MFMAs (one per plane) instead of the VALU sums.
// Swizzle: in the image, vector v's 16-B chunk ch sits at position ch ^ ((v & 3) << 2); the gather
// lanes fetch the permuted source chunks (the DMA writes lane-linearly), and a transposed read's
// four vectors v = 4m .. 4m + 3 then take four distinct 64-B bank groups (conflict-free).
using v4s = __attribute__((ext_vector_type(4))) short;
__device__ __forceinline__ v4s lds_tr16(const uint16_t* p) {
    using lp = __attribute__((address_space(3))) v4s*;
    return __builtin_amdgcn_ds_read_tr16_b64_v4i16(
        (lp)(__attribute__((address_space(3))) void*)(p));
}
__device__ __forceinline__ void gram_accumulate_p3(Smem& sm, f32x16 (&acc)[kSlots], Tiles& tl,
                                                   int nslot, const int32_t* __restrict__ cols,
                                                   int64_t b, int64_t e,
                                                   const uint16_t* __restrict__ P, int64_t ps,
                                                   int32_t zrow, int hsw) {
    static_assert(kCH == 16 && kThreads == 512, "two vectors per wave and chunk");
    static_assert(kRBP >= 3, "at least one chunk of gathers in flight beyond the current one");
    const int t = opaque_tid(), lane = t & 63, q = lane & 31;
    const int wave = __builtin_amdgcn_readfirstlane(t >> 6);
    const int ntb = hsw / 32 - 1;
    if (e <= b) return;
    const int64_t nch = (e - b + kCH - 1) / kCH;
    const int vh = lane >> 5, v = 2 * wave + vh;
    const int gpos = (lane & 31) ^ ((v & 3) << 2);  // the logical chunk this lane's DMA fetches
    auto ids = [&](int64_t c, int32_t& i0, int32_t& i1) {
        const int64_t e0 = b + c * kCH + 2 * wave;
        i0 = e0 < e ? cols[e0] : zrow;
        i1 = e0 + 1 < e ? cols[e0 + 1] : zrow;
    };
    auto gather = [&](int64_t c, int32_t i0, int32_t i1) {
        const int slot = (int)(c % kRBP);
        const uint16_t* src = P + (int64_t)(vh ? i1 : i0) * kPW + 8 * gpos;
#pragma unroll
        for (int p = 0; p < 3; ++p)
            glds16(reinterpret_cast<const float*>(src + p * ps),
                   lds_addr_of(&sm.u.gp[slot][p][2 * wave][0]));
    };
    // transposed operand reads: lane 4 qq + pp of 16-lane group g4 addresses vector
    // 8 (g4 >> 1) + 4 s + qq, features 32 X + 16 (g4 & 1) + 4 pp .. + 3
    const int g4 = lane >> 4, qq = (lane >> 2) & 3, pp = lane & 3;
    const int rowv = 8 * (g4 >> 1) + qq;
    auto opnd = [&](int slot, int p, int X) -> bf16x8 {
        const int ch = 4 * X + 2 * (g4 & 1) + (pp >> 1);
        const uint16_t* a0 = &sm.u.gp[slot][p][rowv][8 * (ch ^ (qq << 2)) + 4 * (pp & 1)];
        const v4s lo = lds_tr16(a0), hi = lds_tr16(a0 + 4 * kPW);
        return bf16x8{lo.x, lo.y, lo.z, lo.w, hi.x, hi.y, hi.z, hi.w};
    };
    const uint32_t one2 = q == 0 ? 0x3F803F80u : 0u;  // two bf16 1.0 on feature kb
    __syncthreads();  // the LDS union may still be read by the previous row's last phase
#pragma unroll
    for (int c = 0; c < kRBP - 1; ++c) {
        int32_t i0, i1;
        ids(c, i0, i1);
        gather(c, i0, i1);
    }
    int32_t n0, n1;  // the ids of the next chunk to gather
    ids(kRBP - 1, n0, n1);
    for (int64_t c = 0; c < nch; ++c) {
        asm volatile("s_waitcnt vmcnt(%0)" ::"i"(3 * (kRBP - 2)) : "memory");  // chunk c landed
        ring_barrier();  // chunk c visible; every wave is done with the slot of chunk c - 1
        gather(c + kRBP - 1, n0, n1);  // into that slot (chunks past the end: the zero row)
        ids(c + kRBP, n0, n1);
        const int slot = (int)(c % kRBP);
        // (every slot with the same six MFMAs and no branch -- b-row tiles against (1, 0, 0), an
        // empty slot on tile (0, 0) -- removes the accumulator copies the branches cause, but the
        // 20 % more MFMAs cost more than the copies: split Gram 90 -> 98 ms, profiles/r4m_*)
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            if (s >= nslot || tl.I[s] < 0) continue;
            bf16x8 A[3];
#pragma unroll
            for (int p = 0; p < 3; ++p) A[p] = opnd(slot, p, tl.J[s]);
            if (tl.I[s] == ntb) {  // row kb: sum_i h_i = the B operand 1 on feature kb
                const bf16x8 ones = __builtin_bit_cast(bf16x8, u32x4{one2, one2, one2, one2});
                acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[2], ones, acc[s], 0, 0, 0);
                acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[1], ones, acc[s], 0, 0, 0);
                acc[s] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[0], ones, acc[s], 0, 0, 0);
            } else {
                bf16x8 B[3];
#pragma unroll
                for (int p = 0; p < 3; ++p) B[p] = opnd(slot, p, tl.I[s]);
                acc[s] = mfma_x3(A, B, acc[s]);
            }
        }
    }
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");  // the ring's trailing loads (past the end)
    __syncthreads();
}

// x = x0 + x1 + x2 (split3t) of every H row, as three bf16 planes of kPW per row (features >= k
// and row n: 0): P[p * (n + 1) * kPW + r * kPW + f]
__global__ __launch_bounds__(256) void wrmf_split_planes_kernel(const float* __restrict__ H,
                                                                int64_t n, int32_t k,
                                                                uint16_t* __restrict__ P) {
    const int64_t ps = (n + 1) * kPW;
    for (int64_t x = (int64_t)blockIdx.x * 256 + threadIdx.x; x < ps;
         x += (int64_t)gridDim.x * 256) {
        const int64_t r = x / kPW;
        const int f = (int)(x - r * kPW);
        const float h = (r < n && f < k) ? H[r * k + f] : 0.0f;
        uint32_t a, b, c;
        split3t(h, a, b, c);
        P[x] = (uint16_t)(a >> 16);
        P[ps + x] = (uint16_t)(b >> 16);
        P[2 * ps + x] = (uint16_t)(c >> 16);
    }
}

// Split Gram of the heavy rows: one workgroup per (row, segment of <= kSeg entries), fp64 atomics
// into gram[(li * kTiles + tile) * 1024 + g * 64 + lane].
struct Seg {
    int32_t li, pad;
    int64_t b, e;
};

template <bool PL>  // PL: the Gram from pre-split planes (P), else from the fp32 rows of H
__global__ __launch_bounds__(kThreads, 2) void wrmf_tile_gram_kernel(
    const Seg* __restrict__ segs, int32_t nseg, int32_t li0, const int32_t* __restrict__ cols,
    const float* __restrict__ H, int32_t k, double* __restrict__ gram,
    const uint16_t* __restrict__ P, int64_t ps, int32_t zrow) {
    __shared__ Smem sm;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int nt = (k + 31) >> 5, nr = nt + 1;
    const int ntile = nt * nr - nt * (nt - 1) / 2;
    Tiles tl;
    my_tiles(wave, nr, ntile, tl);
    for (int sgi = blockIdx.x; sgi < nseg; sgi += gridDim.x) {
        const Seg sg = segs[sgi];
        f32x16 acc[kSlots];
#pragma unroll
        for (int s = 0; s < kSlots; ++s)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[s][g] = 0.0f;
        if constexpr (PL)
            gram_accumulate_p3(sm, acc, tl, kSlots, cols, sg.b, sg.e, P, ps, zrow, 32 * nr);
        else if (kGramRing && (k & 3) == 0)
            gram_accumulate_x3g(sm, acc, tl, kSlots, cols, sg.b, sg.e, H, k, 32 * nr);
        else
            gram_accumulate_x3(sm, acc, tl, kSlots, cols, sg.b, sg.e, H, k, 32 * nr);
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            if (tl.I[s] < 0) continue;
            double* dst =
                gram + ((int64_t)(sg.li - li0) * kTiles + s * kWaves + wave) * 1024 + lane;
#pragma unroll
            for (int g = 0; g < 16; ++g) unsafeAtomicAdd(dst + g * 64, (double)acc[s][g]);
        }
    }
}

// HHt[tile][g][lane] = (HH + reg I)[32I + q][32J + rho(g, h)] inside the k x k block, 1 on the
// diagonal of the padding, else 0.
__global__ __launch_bounds__(256) void wrmf_tile_hh_kernel(const double* __restrict__ HH, int32_t k,
                                                           double reg, float* __restrict__ HHt) {
    const int nt = (k + 31) >> 5, nr = nt + 1;
    const int ntile = nt * nr - nt * (nt - 1) / 2;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < ntile * 1024;
         e += gridDim.x * blockDim.x) {
        const int tile = e >> 10, g = (e >> 6) & 15, lane = e & 63;
        int I, J;
        tile_of(tile, nr, I, J);
        const int r = 32 * I + (lane & 31), c = 32 * J + rho(g, lane >> 5);
        double v = (r == c && r < 32 * nt) ? 1.0 : 0.0;  // identity on the padding
        if (r < k && c < k) v = HH[(int64_t)r * k + c] + (r == c ? reg : 0.0);
        HHt[e] = (float)v;
    }
}

// lanes 0-31 <-> 32-63: each lane gets its partner half's x (v_permlane32_swap)
__device__ __forceinline__ float half_swap(float x, int h) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x), false,
                                                    false);
    return __uint_as_float(h ? r[0] : r[1]);
}

// One wave: T = L^{-1} of the SPD diagonal tile a (held in the C/D layout: lane (q, h), register g
// = element (rho(g, h), q), symmetric), written as tT[c][m] = T[m][c].  Right-looking Cholesky by
// column PAIRS on the matrix core: per pair (c, c + 1) the two pivots and L's two columns come
// from v_readlane broadcasts, then ONE v_mfma_f32_32x32x2_f32 applies the rank-2 update
// A -= l_c l_c^T + l_{c+1} l_{c+1}^T to the whole tile (the operand of lane (q, h) is
// l_{c+h}[q] for both A and B).  T is built alongside from R = I by the same elimination: rows c,
// c + 1 of R are scaled and combined on the VALU (they live in registers gc, gc + 1 of one half),
// then one MFMA applies R[m] -= L[m][c] R[c] + L[m][c+1] R[c+1] to the rows below.  16 dependent
// steps of ~1 MFMA latency each, instead of 32 x 31 serial readlane updates and a row-by-row
// substitution for T (~12 k cycles per tile).
__device__ __forceinline__ void diag_factor_mfma(f32x16 a, float (*tT)[kTS]) {
    const int lane = opaque_tid() & 63, q = lane & 31, h = lane >> 5;
    f32x16 r;
#pragma unroll
    for (int g = 0; g < 16; ++g) r[g] = rho(g, h) == q ? 1.0f : 0.0f;
#pragma unroll
    for (int c = 0; c < 32; c += 2) {
        const int hc = (c >> 2) & 1, gc = (c & 3) + 4 * (c >> 3);  // rho(gc, hc) = c
        // columns c, c + 1 of the updated tile in every lane (row q)
        const float s0 = half_swap(a[gc], h), s1 = half_swap(a[gc + 1], h);
        const float a0 = h == hc ? a[gc] : s0;
        const float piv0 = lane_bcast(a0, c);
        const float rs0 = __builtin_amdgcn_rsqf(piv0);
        const float l0 = q < c ? 0.0f : (q == c ? piv0 * rs0 : a0 * rs0);
        const float l10 = lane_bcast(l0, c + 1);
        const float a1 = (h == hc ? a[gc + 1] : s1) - l0 * l10;
        const float piv1 = lane_bcast(a1, c + 1);
        const float rs1 = __builtin_amdgcn_rsqf(piv1);
        const float l1 = q <= c ? 0.0f : (q == c + 1 ? piv1 * rs1 : a1 * rs1);
        // rows c, c + 1 of R: R[c] /= L[c][c]; R[c+1] = (R[c+1] - L[c+1][c] R[c]) / L[c+1][c+1]
        const float r0 = r[gc] * rs0;
        const float r1 = (r[gc + 1] - l10 * r0) * rs1;
        r[gc] = h == hc ? r0 : r[gc];
        r[gc + 1] = h == hc ? r1 : r[gc + 1];
        if (c + 2 < 32) {
            const float op = h ? l1 : l0;
            a = __builtin_amdgcn_mfma_f32_32x32x2f32(-op, op, a, 0, 0, 0);
            const float t0 = half_swap(r[gc], h), t1 = half_swap(r[gc + 1], h);
            const float opb = hc == 0 ? (h == 0 ? r[gc] : t1) : (h == 0 ? t0 : r[gc + 1]);
            const float opa = q > c + 1 ? op : 0.0f;
            r = __builtin_amdgcn_mfma_f32_32x32x2f32(-opa, opb, r, 0, 0, 0);
        }
    }
#pragma unroll
    for (int g = 0; g < 16; ++g) tT[q][rho(g, h)] = r[g];
}

// The owner of diagonal tile `slot` factors it (T_J = L_JJ^{-1} to tT); no LDS parking: the
// factorisation needs ~40 registers beside the accumulators.
__device__ __forceinline__ void factor_tile(Smem& sm, f32x16 (&acc)[kSlots], int slot,
                                            float (*tT)[kTS]) {
    (void)sm;
    f32x16 a;
#pragma unroll
    for (int g = 0; g < 16; ++g) a[g] = 0.0f;
#pragma unroll
    for (int s = 0; s < kSlots; ++s)
        if (s == slot) a = acc[s];
    diag_factor_mfma(a, tT);
}

// trailing update of tile (I, K) by panel tiles pk = K - J - 1, pi = I - J - 1:
// a -= L_IJ L_KJ^T, from the bf16x3 planes (A = -L_KJ rows, B = L_IJ rows; 12 MFMAs of 32 cycles
// against 16 of 64 for v_mfma_f32_32x32x2_f32)
__device__ __forceinline__ f32x16 panel_update_x3(Smem& sm, f32x16 a, int pk, int pi, int q,
                                                  int h) {
#pragma unroll
    for (int s2 = 0; s2 < 2; ++s2) {
        bf16x8 A[3], B[3];
#pragma unroll
        for (int p = 0; p < 3; ++p) {
            A[p] = bf16_neg(*reinterpret_cast<const bf16x8*>(&sm.u.fz.pp[pk][p][q][16 * s2 + 8 * h]));
            B[p] = *reinterpret_cast<const bf16x8*>(&sm.u.fz.pp[pi][p][q][16 * s2 + 8 * h]);
        }
        a = mfma_x3(A, B, a);
    }
    return a;
}

// L^T w = y by 32-column blocks, w_J = T_J^T (y_J - sum_{I>J} L_IJ^T w_I): the factor in the
// owners' accumulators (L_IJ below the diagonal, T_J = L_JJ^{-1} on it), y in sm.yv, w to sm.wv.
__device__ __forceinline__ void back_substitute(Smem& sm, f32x16 (&acc)[kSlots], Tiles& tl,
                                                int nt) {
    const int t = opaque_tid(), lane = t & 63, q = lane & 31, h = lane >> 5;
    for (int J = nt - 1; J >= 0; --J) {
        launder(tl);
        __syncthreads();
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            if (tl.J[s] != J) continue;
            if (tl.I[s] == J) {
#pragma unroll
                for (int g = 0; g < 16; ++g) sm.tT[0][2 * g + h][q] = acc[s][g];
            } else if (tl.I[s] < nt) {
                const float wr = sm.wv[32 * tl.I[s] + q];
                const int pi = tl.I[s] - J - 1;
#pragma unroll
                for (int g = 0; g < 16; ++g) sm.u.red[pi][rho(g, h)][q] = acc[s][g] * wr;
            }
        }
        __syncthreads();
        const int nparts = nt - 1 - J;
        if (t < 32 * nparts) {
            const int pi = t >> 5, c = t & 31;
            float sacc = 0.0f;
#pragma unroll
            for (int x = 0; x < 32; ++x) sacc += sm.u.red[pi][c][x];
            sm.part[pi][c] = sacc;
        }
        __syncthreads();
        if (t < 32) {
            float sacc = sm.yv[32 * J + t];
            for (int pi = 0; pi < nparts; ++pi) sacc -= sm.part[pi][t];
            sm.sv[t] = sacc;
        }
        __syncthreads();
        if (t < 32) {
            float w = 0.0f;
#pragma unroll
            for (int c = 0; c < 32; ++c) w += (c >= t) ? sm.tT[0][t][c] * sm.sv[c] : 0.0f;
            sm.wv[32 * J + t] = w;
        }
    }
}

// MODE 0: the direct row solve (W_u = A_u^{-1} b_u), kdim = k.
// MODE 1: the Woodbury row solve for rows with deg <= kWood (WRMF.cs:110-156 restated):
//   A_u = B + alpha H_S^T H_S with B = HH + reg I = L L^T shared by all rows, Q = H L^{-T}:
//   W_u = ((1 + alpha) / alpha) L^{-T} Q_S^T C^{-1} 1,  C = I / alpha + Q_S Q_S^T  (deg x deg).
//   The kernel solves C v = 1 on the same tile machinery (kdim = 32 * ceil(deg_max / 32)) and
//   writes t = Q_S^T v to Tout[list index]; W rows = c t L^{-1} follow as one batched GEMM.
template <int MODE, bool PL = false>  // PL (MODE 0): the Gram from pre-split planes
__global__ __launch_bounds__(kThreads, 2) void wrmf_tile_solve_kernel(
    const int32_t* __restrict__ rows, int32_t n_list, int32_t* __restrict__ counter,
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols, float* __restrict__ W,
    const float* __restrict__ H, const float* __restrict__ HHt, const double* __restrict__ gram,
    int32_t k, int32_t kdim, float alpha, float* __restrict__ Tout, int32_t dbg,
    const float* __restrict__ rhs, float* __restrict__ F, const uint16_t* __restrict__ P = nullptr,
    int64_t ps = 0, int32_t zrow = 0) {
    __shared__ Smem sm;
#ifndef MML_EXPERIMENTS
    // the phase masks are switches of the experiments build: a constant here folds their branches
    // (each one around an MFMA chain made the compiler copy the accumulators behind it)
    dbg = 0;
#endif
    const bool gram_x3 = !(dbg & 32);  // MML_WRMF_DEBUG & 32: the f32 MFMA Gram (A/B)
    const int wave = threadIdx.x >> 6;
    const int nt = (kdim + 31) >> 5, nr = nt + 1;
    const int ntile = nt * nr - nt * (nt - 1) / 2;
    const int nslot = (ntile + kWaves - 1) / kWaves;
    const int hsw = 32 * nr;
    Tiles tl;
    my_tiles(wave, nr, ntile, tl);
    for (;;) {
        const int t = opaque_tid(), lane = t & 63, q = lane & 31, h = lane >> 5;
        __syncthreads();
        if (t == 0) sm.row = atomicAdd(counter, 1);
        __syncthreads();
        const int li = sm.row;
        if (li >= n_list) break;
        // (also keeps the row-invariant HHt loads inside the row loop)
        launder(tl);
        const int32_t row = rows[li];
        const int64_t rb = off[row], re = off[row + 1];
        if (re == rb) {  // no entries: A^{-1} 0 = 0 (WRMF.cs:126-155)
            if (MODE == 0)
                for (int f = t; f < k; f += kThreads) W[(int64_t)row * k + f] = 0.0f;
            else
                for (int f = t; f < k; f += kThreads) Tout[(int64_t)li * k + f] = 0.0f;
            continue;
        }
        f32x16 acc[kSlots];
#pragma unroll
        for (int s = 0; s < kSlots; ++s)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[s][g] = 0.0f;
        // ---- 1. Gram (+ b in row kb)
        if (MODE == 0 && gram) {
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] < 0) continue;
                const double* src = gram + ((int64_t)li * kTiles + s * kWaves + wave) * 1024 + lane;
#pragma unroll
                for (int g = 0; g < 16; ++g) acc[s][g] = (float)src[g * 64];
            }
        } else if (!(dbg & 8)) {
            if constexpr (MODE == 0) {
                if constexpr (PL)
                    gram_accumulate_p3(sm, acc, tl, nslot, cols, rb, re, P, ps, zrow, hsw);
                else if (gram_x3 && kGramRing && (k & 3) == 0)
                    gram_accumulate_x3g(sm, acc, tl, nslot, cols, rb, re, H, k, hsw);
                else if (gram_x3)
                    gram_accumulate_x3(sm, acc, tl, nslot, cols, rb, re, H, k, hsw);
                else gram_accumulate<0>(sm, acc, tl, nslot, cols, rb, re, H, k, hsw, kdim);
            } else {
                gram_accumulate<MODE>(sm, acc, tl, nslot, cols, rb, re, H, k, hsw, kdim);
            }
        }
        // ---- 2. A' = HHt + alpha * S above row kb (HHt = HH + reg I, identity on the padding;
        //         S is 0 on the padding), (1 + alpha) * S on the b-row tile
        if constexpr (MODE == 0) {
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] < 0) continue;
                if (tl.I[s] < nt) {
                    const float* hh = HHt + tile_id(tl.I[s], tl.J[s], nr) * 1024 + lane;
#pragma unroll
                    for (int g = 0; g < 16; ++g) acc[s][g] = hh[g * 64] + alpha * acc[s][g];
                } else if (rhs) {  // a refinement pass: the residual row replaces b
#pragma unroll
                    for (int g = 0; g < 16; ++g) {
                        const int cc = 32 * tl.J[s] + rho(g, h);
                        acc[s][g] = (q == 0 && cc < k) ? rhs[(int64_t)row * k + cc] : 0.0f;
                    }
                } else {
#pragma unroll
                    for (int g = 0; g < 16; ++g) acc[s][g] *= 1.0f + alpha;
                }
            }
        } else {
            // C' = [I / alpha + Q_S Q_S^T (identity on the padding); b row = 1 on the deg columns]
            const int deg = (int)(re - rb);
            const float ainv = 1.0f / alpha;
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] < 0) continue;
                const int r = 32 * tl.I[s] + q;
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int cc = 32 * tl.J[s] + rho(g, h);
                    float v = acc[s][g];
                    if (tl.I[s] < nt) {
                        if (r == cc) v += cc < deg ? ainv : 1.0f;
                    } else {
                        v = (q == 0 && cc < deg) ? 1.0f : 0.0f;
                    }
                    acc[s][g] = v;
                }
            }
        }
        // ---- 3. blocked Cholesky by 32-column panels, with a one-panel lookahead: the owner of
        //         the next diagonal tile updates and factors it first, while the other waves are
        //         still applying the current panel to the rest of the trailing matrix
        if (wave == 0 && !(dbg & 1)) factor_tile(sm, acc, 0, sm.tT[0]);  // tile (0, 0): slot 0
        __syncthreads();
        for (int J = 0; J < nt; ++J) {
            launder(tl);
            const int td = tile_id(J, J, nr), tdn = tile_id(J + 1, J + 1, nr);
            float (*tT)[kTS] = sm.tT[J & 1];
            // (c) L_IJ = A'_IJ T_J^T for the tiles below; the panel goes to LDS; the diagonal
            //     owner keeps T_J in the (now free) accumulators of tile (J, J) for step 4
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.J[s] != J) continue;
                if (tl.I[s] == J) {
#pragma unroll
                    for (int g = 0; g < 16; ++g) acc[s][g] = tT[2 * g + h][q];
                    continue;
                }
                f32x16 nv;
#pragma unroll
                for (int g = 0; g < 16; ++g) nv[g] = 0.0f;
                const int pi = tl.I[s] - J - 1;
                if constexpr (kFactorX3) {
                    // bf16x3 on v_mfma_f32_32x32x16_bf16: K slot (h, j) of step s2 is column
                    // rho(8 s2 + j, h), so B is registers 8 s2 .. 8 s2 + 7 of the tile as they sit
                    // (12 instead of 16 x 64 MFMA cycles per tile)
                    if (!(dbg & 2))
#pragma unroll
                        for (int s2 = 0; s2 < 2; ++s2) {
                            float av[8], bv[8];
#pragma unroll
                            for (int j = 0; j < 8; ++j) {
                                av[j] = tT[rho(8 * s2 + j, h)][q];
                                bv[j] = acc[s][8 * s2 + j];
                            }
                            bf16x8 A[3], B[3];
                            split8(av, A);
                            split8(bv, B);
                            nv = mfma_x3(A, B, nv);
                        }
                    // the panel's planes for the trailing updates, in the same K-slot order
#pragma unroll
                    for (int s2 = 0; s2 < 2; ++s2) {
                        float v[8];
#pragma unroll
                        for (int j = 0; j < 8; ++j) v[j] = nv[8 * s2 + j];
                        bf16x8 P[3];
                        split8(v, P);
#pragma unroll
                        for (int p = 0; p < 3; ++p)
                            *reinterpret_cast<bf16x8*>(&sm.u.fz.pp[pi][p][q][16 * s2 + 8 * h]) = P[p];
                    }
                } else {
                    if (!(dbg & 2))
#pragma unroll
                        for (int st = 0; st < 16; ++st)
                            nv = __builtin_amdgcn_mfma_f32_32x32x2f32(tT[rho(st, h)][q], acc[s][st],
                                                                      nv, 0, 0, 0);
#pragma unroll
                    for (int g = 0; g < 16; ++g) sm.u.fz.pn[pi][q][rho(g, h)] = nv[g];
                }
                acc[s] = nv;
                if (tl.I[s] == nt && q == 0)  // row kb: y_J
#pragma unroll
                    for (int g = 0; g < 16; ++g) sm.yv[32 * J + rho(g, h)] = nv[g];
            }
            (void)td;
            __syncthreads();
            // (d) trailing update A'_IK -= L_KJ L_IJ^T, K > J; tile (J+1, J+1) first, then factored
            if (J + 1 < nt && (tdn % kWaves) == wave) {
                const int own = tdn / kWaves;
#pragma unroll
                for (int s = 0; s < kSlots; ++s) {
                    if (s != own || (dbg & 2)) continue;
                    if constexpr (kFactorX3) {
                        acc[s] = panel_update_x3(sm, acc[s], 0, 0, q, h);
                    } else {
                        const float* lr = sm.u.fz.pn[0][q];
#pragma unroll
                        for (int st = 0; st < 16; ++st)
                            acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                                -lr[2 * st + h], lr[2 * st + h], acc[s], 0, 0, 0);
                    }
                }
                if (!(dbg & 1)) factor_tile(sm, acc, own, sm.tT[(J + 1) & 1]);
            }
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] < 0 || tl.J[s] <= J || (dbg & 2)) continue;
                if (s * kWaves + wave == tdn) continue;
                if constexpr (kFactorX3) {
                    acc[s] = panel_update_x3(sm, acc[s], tl.J[s] - J - 1, tl.I[s] - J - 1, q, h);
                } else {
                    const float* lk = sm.u.fz.pn[tl.J[s] - J - 1][q];
                    const float* lr = sm.u.fz.pn[tl.I[s] - J - 1][q];
#pragma unroll
                    for (int st = 0; st < 16; ++st)
                        acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(-lk[2 * st + h],
                                                                      lr[2 * st + h], acc[s], 0, 0, 0);
                }
            }
            __syncthreads();
        }
        // the factor, kept for the refinement passes (wrmf_tile_resolve_kernel)
        if (MODE == 0 && F)
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] < 0 || tl.I[s] >= nt) continue;
                float* dst = F + ((int64_t)li * kTiles + s * kWaves + wave) * 1024 + lane;
#pragma unroll
                for (int g = 0; g < 16; ++g) dst[g * 64] = acc[s][g];
            }
        // ---- 4. backward substitution L^T w = y (padding entries come out 0).  With the factor
        //         kept (fp64 mode) it is deferred to wrmf_tile_resolve_wave_kernel (backward_only):
        //         y goes to the W row, and one wave per row streams the kept tiles, without the
        //         8-wave workgroup's barrier per block row (31 -> ~11 ms per C5 iteration)
        const bool defer = MODE == 0 && F != nullptr;
        if (!defer && !(dbg & 4)) back_substitute(sm, acc, tl, nt);
        __syncthreads();
        if constexpr (MODE == 0) {
            const float* src = defer ? sm.yv : sm.wv;
            for (int f = t; f < k; f += kThreads) W[(int64_t)row * k + f] = src[f];
        } else {
            // t = Q_S^T v (the item ids staged in LDS first)
            const int deg = (int)(re - rb);
            int32_t* ids = reinterpret_cast<int32_t*>(sm.u.red);
            for (int x = t; x < deg; x += kThreads) ids[x] = cols[rb + x];
            __syncthreads();
            for (int f = t; f < k; f += kThreads) {
                float a0 = 0.0f, a1 = 0.0f;
                int x = 0;
                for (; x + 1 < deg; x += 2) {
                    a0 += sm.wv[x] * H[(int64_t)ids[x] * k + f];
                    a1 += sm.wv[x + 1] * H[(int64_t)ids[x + 1] * k + f];
                }
                if (x < deg) a0 += sm.wv[x] * H[(int64_t)ids[x] * k + f];
                Tout[(int64_t)li * k + f] = a0 + a1;
            }
        }
    }
}

// A refinement pass on a direct row whose factor wrmf_tile_solve_kernel<0> kept in F: forward
// substitution L y = r by 32-row blocks, y_J = T_J (r_J - sum_{K<J} L_JK y_K), then the same
// backward substitution; W row <- L^{-T} y.  No Gram, no factorisation.
__global__ __launch_bounds__(kThreads, 2) void wrmf_tile_resolve_kernel(
    const int32_t* __restrict__ rows, int32_t n_list, int32_t* __restrict__ counter,
    const int64_t* __restrict__ off, const float* __restrict__ F, const float* __restrict__ rhs,
    int32_t k, float* __restrict__ W) {
    __shared__ Smem sm;
    const int wave = threadIdx.x >> 6;
    const int nt = (k + 31) >> 5, nr = nt + 1;
    const int ntile = nt * nr - nt * (nt - 1) / 2;
    Tiles tl;
    my_tiles(wave, nr, ntile, tl);
    for (;;) {
        const int t = opaque_tid(), lane = t & 63, q = lane & 31, h = lane >> 5;
        __syncthreads();
        if (t == 0) sm.row = atomicAdd(counter, 1);
        __syncthreads();
        const int li = sm.row;
        if (li >= n_list) break;
        launder(tl);
        const int32_t row = rows[li];
        if (off[row + 1] == off[row]) {  // no entries: the main solve kept no factor; d = 0
            for (int f = t; f < k; f += kThreads) W[(int64_t)row * k + f] = 0.0f;
            continue;
        }
        f32x16 acc[kSlots];
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            const bool own = tl.I[s] >= 0 && tl.I[s] < nt;
            const float* src = F + ((int64_t)li * kTiles + s * kWaves + wave) * 1024 + lane;
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[s][g] = own ? src[g * 64] : 0.0f;
        }
        for (int J = 0; J < nt; ++J) {
            launder(tl);
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] != J || tl.J[s] > J) continue;
                if (tl.J[s] == J) {  // T_J, for the 32 threads below
#pragma unroll
                    for (int g = 0; g < 16; ++g) sm.tT[0][2 * g + h][q] = acc[s][g];
                    continue;
                }
                // row q of L_JK y_K: this lane's 16 columns, then the other half's
                float a = 0.0f;
#pragma unroll
                for (int g = 0; g < 16; ++g) a += acc[s][g] * sm.yv[32 * tl.J[s] + rho(g, h)];
                a += __shfl_xor(a, 32, 64);
                if (h == 0) sm.part[tl.J[s]][q] = a;
            }
            __syncthreads();
            if (t < 32) {
                const int f = 32 * J + t;
                float sacc = f < k ? rhs[(int64_t)row * k + f] : 0.0f;
                for (int K = 0; K < J; ++K) sacc -= sm.part[K][t];
                sm.sv[t] = sacc;
            }
            __syncthreads();
            if (t < 32) {  // y_J = T_J s, T_J lower: tT[c][m] = T_J[m][c]
                float y = 0.0f;
#pragma unroll
                for (int c = 0; c < 32; ++c) y += (c <= t) ? sm.tT[0][c][t] * sm.sv[c] : 0.0f;
                sm.yv[32 * J + t] = y;
            }
            __syncthreads();
        }
        back_substitute(sm, acc, tl, nt);
        __syncthreads();
        for (int f = t; f < k; f += kThreads) W[(int64_t)row * k + f] = sm.wv[f];
    }
}

// The same refinement pass with one wave per row and no workgroup barrier: the wave streams the
// row's kept tiles from memory (each lower tile once per substitution) instead of holding them in
// 8 waves' registers, so ~100 VGPRs and many rows per CU keep the tile loads in flight; the
// workgroup version waits on 56 barriers per row, with one row per CU.
//   forward  y_J = T_J (r_J - sum_{K<J} L_JK y_K):  lane (q, h) sums its 16 columns rho(g, h) of
//            row q against y from LDS, the halves meet by a lane-32 swap;
//   backward w_J = T_J^T (y_J - sum_{I>J} L_IJ^T w_I):  lane (q, h) scales its 16 columns by w_I[q]
//            (its own row), and the column sums over q go through a transposed LDS tile.
// Tile (I, J) of row li is F[(li * kTiles + tile_id(I, J, nr)) * 1024 + g * 64 + lane]: lane (q, h)
// register g holds L[32 I + q][32 J + rho(g, h)] below the diagonal and T_J[q][2 g + h] on it.
constexpr int kRvWaves = 4;
constexpr int kRvS = 36;  // transposed-tile row stride (16-B aligned rows)
struct alignas(16) RvSmem {
    float ys[kHSW];          // y, then read by the backward pass
    float ws[kHSW];          // w
    float sv[32];
    float red[32 * kRvS];    // red[c * kRvS + q]: column sums over q
};
__device__ __forceinline__ void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}
// backward_only: rhs holds y = L^{-1} b already (the main solve's forward result, deferred here
// from wrmf_tile_solve_kernel), and may alias W: the wave reads its row into LDS before writing.
// (five waves per SIMD, <= 96 VGPRs: a wave per SIMD fits beside the tile solve's two when the
// item half's pipeline runs a range's correction under the next range's solve)
__global__ __launch_bounds__(64 * kRvWaves, 5) void wrmf_tile_resolve_wave_kernel(
    const int32_t* __restrict__ rows, int32_t n_list, const int64_t* __restrict__ off,
    const float* __restrict__ F, const float* rhs, int32_t k, float* W, int32_t backward_only) {
    __shared__ RvSmem smem[kRvWaves];
    const int wv = threadIdx.x >> 6, lane = threadIdx.x & 63, q = lane & 31, h = lane >> 5;
    RvSmem& sm = smem[wv];
    const int nt = (k + 31) >> 5, nr = nt + 1;
    const int64_t nwave = (int64_t)gridDim.x * kRvWaves;
    for (int64_t li = (int64_t)blockIdx.x * kRvWaves + wv; li < n_list; li += nwave) {
        const int32_t row = rows[li];
        float* wr = W + (int64_t)row * k;
        if (off[row + 1] == off[row]) {  // no entries: the main solve kept no factor; d = 0
            for (int f = lane; f < k; f += 64) wr[f] = 0.0f;
            continue;
        }
        const float* Fr = F + (int64_t)li * kTiles * 1024 + lane;
        const float* rr = rhs + (int64_t)row * k;
        float tv[16];
        auto load_tile = [&](int I, int J) {
            const float* src = Fr + (int64_t)tile_id(I, J, nr) * 1024;
#pragma unroll
            for (int g = 0; g < 16; ++g) tv[g] = src[g * 64];
        };
        if (backward_only) {
            for (int f = lane; f < 32 * nt; f += 64) sm.ys[f] = f < k ? rr[f] : 0.0f;
            wave_sync();
        }
        // ---- forward substitution
        for (int J = 0; J < (backward_only ? 0 : nt); ++J) {
            float a = 0.0f;
            for (int K = 0; K < J; ++K) {
                load_tile(J, K);
#pragma unroll
                for (int m = 0; m < 4; ++m) {
                    const float4 y4 = *reinterpret_cast<const float4*>(&sm.ys[32 * K + 8 * m + 4 * h]);
                    a += tv[4 * m] * y4.x + tv[4 * m + 1] * y4.y + tv[4 * m + 2] * y4.z +
                         tv[4 * m + 3] * y4.w;
                }
            }
            a += __shfl_xor(a, 32, 64);
            const int f = 32 * J + q;
            const float s = (f < k ? rr[f] : 0.0f) - a;
            if (h == 0) sm.sv[q] = s;
            load_tile(J, J);
            wave_sync();
            float y = 0.0f;
#pragma unroll
            for (int g = 0; g < 16; ++g) y += tv[g] * sm.sv[2 * g + h];
            y += __shfl_xor(y, 32, 64);
            if (h == 0) sm.ys[f] = y;
            wave_sync();
        }
        // ---- backward substitution
        for (int J = nt - 1; J >= 0; --J) {
            float p[16];
#pragma unroll
            for (int g = 0; g < 16; ++g) p[g] = 0.0f;
            for (int I = J + 1; I < nt; ++I) {
                load_tile(I, J);
                const float wq = sm.ws[32 * I + q];
#pragma unroll
                for (int g = 0; g < 16; ++g) p[g] += tv[g] * wq;
            }
#pragma unroll
            for (int g = 0; g < 16; ++g) sm.red[rho(g, h) * kRvS + q] = p[g];
            load_tile(J, J);
            wave_sync();
            float v = sm.ys[32 * J + q];
#pragma unroll
            for (int x = 0; x < 32; x += 4) {
                const float4 r4 = *reinterpret_cast<const float4*>(&sm.red[q * kRvS + x]);
                v -= (r4.x + r4.y) + (r4.z + r4.w);
            }
            wave_sync();
            // w_J[c] = sum_m T_J[m][c] v[m]: lane (q, h) holds T_J[q][2 g + h], v[q] is its own
#pragma unroll
            for (int g = 0; g < 16; ++g) sm.red[(2 * g + h) * kRvS + q] = tv[g] * v;
            wave_sync();
            float w = 0.0f;
#pragma unroll
            for (int x = 0; x < 32; x += 4) {
                const float4 r4 = *reinterpret_cast<const float4*>(&sm.red[q * kRvS + x]);
                w += (r4.x + r4.y) + (r4.z + r4.w);
            }
            if (h == 0) sm.ws[32 * J + q] = w;
            wave_sync();
        }
        for (int f = lane; f < k; f += 64) wr[f] = sm.ws[f];
        wave_sync();  // the next row's forward pass rewrites ys / ws
    }
}

// ---------------------------------------------------------------------------------------------
// Woodbury rows, several per workgroup.  A row with deg <= 32 NT entries has only
// NT (NT + 1) - NT (NT - 1) / 2 tiles (<= 14), so the 8 waves split into R groups of WPG waves and
// each group solves its own row: the groups run the same phases in lockstep (shared barriers), so
// their serial diagonal factorisations run side by side on different waves.  Same math as
// wrmf_tile_solve_kernel<1>; every group owns a private LDS slice.
template <int NT>
struct WoodCfg {
    static constexpr int R = (NT >= 3) ? 2 : 4;             // rows per workgroup (registers)
    static constexpr int WPG = kWaves / R;                  // waves per row
    static constexpr int TG = 64 * WPG;                     // threads per row
    static constexpr int NR = NT + 1;
    static constexpr int NTILE = NT * NR - NT * (NT - 1) / 2;
    static constexpr int SLOTS = (NTILE + WPG - 1) / WPG;
    static constexpr int ITEMS = 32 * NT;                   // item columns (deg <= ITEMS)
    static constexpr int HSW = 32 * NR;                     // staged width (+ the b-row tile)
    static constexpr int F4 = (ITEMS * 4 + TG - 1) / TG;    // float4 staged per thread and chunk
};

template <int NT>
struct WoodSmem {
    using C = WoodCfg<NT>;
    union {
        float hs[2][kCH][C::HSW];
        float pn[NT][32][kPS];
        float red[NT][32][kDS];
    } u;
    float tT[2][32][kTS];
    float yv[C::HSW];
    float wv[C::HSW];
    float sv[32];
    float part[NT][32];
    float yr[C::ITEMS];  // a refinement pass: the b row y = Q_S s
    int32_t ids[C::ITEMS];
};

// __launch_bounds__' second argument is the minimum waves per SIMD: 4 caps the kernel at 128
// registers, so two 8-wave workgroups (4 rows) share a CU.  With (kThreads, 2) the compiler took
// 142 VGPRs at NT = 4 and only one workgroup fit (C5 PMC: MFMA busy 25 %, waves parked 58 % of
// their cycles on memory / barrier waits).
template <int NT>
__global__ __launch_bounds__(kThreads, 4) void wrmf_wood_kernel(
    const int32_t* __restrict__ rows, int32_t n_list, int32_t* __restrict__ counter,
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols,
    const float* __restrict__ Q, int32_t k, float alpha, float* __restrict__ Tout,
    const float* __restrict__ S) {
    using C = WoodCfg<NT>;
    extern __shared__ __attribute__((aligned(16))) char wood_smem[];
    __shared__ int32_t base_row;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int grp = wave / C::WPG, wig = wave % C::WPG;
    WoodSmem<NT>& sm = reinterpret_cast<WoodSmem<NT>*>(wood_smem)[grp];
    int TI[C::SLOTS], TJ[C::SLOTS];
#pragma unroll
    for (int s = 0; s < C::SLOTS; ++s) {
        const int t = s * C::WPG + wig;
        int I = -1, J = -1;
        if (t < C::NTILE) tile_of(t, C::NR, I, J);
        TI[s] = __builtin_amdgcn_readfirstlane(I);
        TJ[s] = __builtin_amdgcn_readfirstlane(J);
    }
    const float ainv = 1.0f / alpha;
    const bool vec = (k & 3) == 0;
    for (;;) {
        const int tid = opaque_tid(), lane = tid & 63, q = lane & 31, h = lane >> 5;
        const int tg = tid - grp * C::TG;
        __syncthreads();
        if (tid == 0) base_row = atomicAdd(counter, C::R);
        __syncthreads();
        const int b0 = base_row;
        if (b0 >= n_list) break;
        const int li = b0 + grp;
        const bool live = li < n_list;
        const int32_t row = live ? rows[li] : 0;
        const int64_t rb = live ? off[row] : 0;
        const int deg = live ? (int)(off[row + 1] - rb) : 0;
        for (int x = tg; x < C::ITEMS; x += C::TG) sm.ids[x] = x < deg ? cols[rb + x] : 0;
        f32x16 acc[C::SLOTS];
#pragma unroll
        for (int s = 0; s < C::SLOTS; ++s)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[s][g] = 0.0f;
        // ---- C = Q_S Q_S^T: the k features are the vectors, 16 per LDS chunk, double-buffered
        float4 p4[C::F4];
        auto fetch = [&](int f0) {
#pragma unroll
            for (int j = 0; j < C::F4; ++j) {
                const int x = tg + j * C::TG;
                const int wi = x >> 2, f = f0 + 4 * (x & 3);
                float4 v = make_float4(0.f, 0.f, 0.f, 0.f);
                if (x < C::ITEMS * 4 && wi < deg) {
                    const float* src = Q + (int64_t)sm.ids[wi] * k + f;
                    if (vec) {
                        if (f < k) v = *reinterpret_cast<const float4*>(src);
                    } else {
                        v.x = f < k ? src[0] : 0.f;
                        v.y = f + 1 < k ? src[1] : 0.f;
                        v.z = f + 2 < k ? src[2] : 0.f;
                        v.w = f + 3 < k ? src[3] : 0.f;
                    }
                }
                p4[j] = v;
            }
        };
        auto stash = [&](int buf) {
#pragma unroll
            for (int j = 0; j < C::F4; ++j) {
                const int x = tg + j * C::TG;
                if (x < C::ITEMS * 4) {
                    const int wi = x >> 2, r4 = 4 * (x & 3);
                    sm.u.hs[buf][r4][wi] = p4[j].x;
                    sm.u.hs[buf][r4 + 1][wi] = p4[j].y;
                    sm.u.hs[buf][r4 + 2][wi] = p4[j].z;
                    sm.u.hs[buf][r4 + 3][wi] = p4[j].w;
                }
            }
        };
        __syncthreads();  // ids visible; the LDS union is free
        for (int x = tg; x < 2 * kCH * 32; x += C::TG)  // the b-row tile's columns stay 0
            sm.u.hs[x / (kCH * 32)][(x / 32) % kCH][C::ITEMS + (x & 31)] = 0.0f;
        fetch(0);
        stash(0);
        __syncthreads();
        int cur = 0;
        for (int f0 = 0; f0 < k; f0 += kCH) {
            const bool more = f0 + kCH < k;
            if (more) fetch(f0 + kCH);
#pragma unroll
            for (int cc = 0; cc < kCH; cc += 2) {
                const float* hr = sm.u.hs[cur][cc + h];
#pragma unroll
                for (int s = 0; s < C::SLOTS; ++s) {
                    // the b-row tiles (I = NT) are set below, not accumulated: no MFMAs for them
                    // (TI is wave-uniform, so this is a scalar branch)
                    if (TI[s] < 0 || TI[s] >= NT) continue;
                    acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(hr[32 * TJ[s] + q],
                                                                  hr[32 * TI[s] + q], acc[s], 0, 0,
                                                                  0);
                }
            }
            if (more) stash(cur ^ 1);
            __syncthreads();
            cur ^= 1;
        }
        // a refinement pass solves A d = r: with s = L^{-1} r (S, one row per list entry) the
        // b row is y = Q_S s and the output t = s - Q_S^T w (then d = L^{-T} t, scale 1)
        if (S) {
            for (int x = tg; x < C::ITEMS; x += C::TG) {
                float a = 0.0f;
                if (x < deg)
                    for (int f = 0; f < k; ++f)
                        a += Q[(int64_t)sm.ids[x] * k + f] * S[(int64_t)li * k + f];
                sm.yr[x] = a;
            }
            __syncthreads();
        }
        // ---- C' = [I / alpha + C (identity on the padding); b row = 1 (or y) on the deg columns]
#pragma unroll
        for (int s = 0; s < C::SLOTS; ++s) {
            if (TI[s] < 0) continue;
            const int r = 32 * TI[s] + q;
#pragma unroll
            for (int g = 0; g < 16; ++g) {
                const int cc = 32 * TJ[s] + rho(g, h);
                float v = acc[s][g];
                if (TI[s] < NT) {
                    if (r == cc) v += cc < deg ? ainv : 1.0f;
                } else {
                    v = (q == 0 && cc < deg) ? (S ? sm.yr[cc] : 1.0f) : 0.0f;
                }
                acc[s][g] = v;
            }
        }
        // ---- blocked Cholesky with a one-panel lookahead (as wrmf_tile_solve_kernel)
        auto factor_owned = [&](int tile, float (*tT)[kTS]) {
            f32x16 a;
#pragma unroll
            for (int g = 0; g < 16; ++g) a[g] = 0.0f;
#pragma unroll
            for (int s = 0; s < C::SLOTS; ++s)
                if (s * C::WPG + wig == tile) a = acc[s];
            diag_factor_mfma(a, tT);
        };
        if (wig == 0) factor_owned(0, sm.tT[0]);
        __syncthreads();
#pragma unroll
        for (int J = 0; J < NT; ++J) {
            const int tdn = tile_id(J + 1, J + 1, C::NR);
            float (*tT)[kTS] = sm.tT[J & 1];
#pragma unroll
            for (int s = 0; s < C::SLOTS; ++s) {
                if (TJ[s] != J) continue;
                if (TI[s] == J) {
#pragma unroll
                    for (int g = 0; g < 16; ++g) acc[s][g] = tT[2 * g + h][q];
                    continue;
                }
                f32x16 nv;
#pragma unroll
                for (int g = 0; g < 16; ++g) nv[g] = 0.0f;
#pragma unroll
                for (int st = 0; st < 16; ++st)
                    nv = __builtin_amdgcn_mfma_f32_32x32x2f32(tT[rho(st, h)][q], acc[s][st], nv, 0,
                                                              0, 0);
                acc[s] = nv;
                const int pi = TI[s] - J - 1;
#pragma unroll
                for (int g = 0; g < 16; ++g) sm.u.pn[pi][q][rho(g, h)] = nv[g];
                if (TI[s] == NT && q == 0)
#pragma unroll
                    for (int g = 0; g < 16; ++g) sm.yv[32 * J + rho(g, h)] = nv[g];
            }
            __syncthreads();
            if (J + 1 < NT) {
                const bool own_next = (tdn % C::WPG) == wig;
#pragma unroll
                for (int s = 0; s < C::SLOTS; ++s) {
                    if (TI[s] < 0 || TJ[s] <= J) continue;
                    const bool next = s * C::WPG + wig == tdn;
                    if (own_next != next && next) continue;
                    const float* lk = sm.u.pn[TJ[s] - J - 1][q];
                    const float* lr = sm.u.pn[TI[s] - J - 1][q];
#pragma unroll
                    for (int st = 0; st < 16; ++st)
                        acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(-lk[2 * st + h],
                                                                      lr[2 * st + h], acc[s], 0, 0,
                                                                      0);
                    if (next) factor_owned(tdn, sm.tT[(J + 1) & 1]);
                }
            }
            __syncthreads();
        }
        // ---- backward substitution L^T v = y
#pragma unroll
        for (int J = NT - 1; J >= 0; --J) {
#pragma unroll
            for (int s = 0; s < C::SLOTS; ++s) {
                if (TJ[s] != J) continue;
                if (TI[s] == J) {
#pragma unroll
                    for (int g = 0; g < 16; ++g) sm.tT[0][2 * g + h][q] = acc[s][g];
                } else if (TI[s] < NT) {
                    const float wr = sm.wv[32 * TI[s] + q];
                    const int pi = TI[s] - J - 1;
#pragma unroll
                    for (int g = 0; g < 16; ++g) sm.u.red[pi][rho(g, h)][q] = acc[s][g] * wr;
                }
            }
            __syncthreads();
            const int nparts = NT - 1 - J;
            if (tg < 32 * nparts) {
                const int pi = tg >> 5, c = tg & 31;
                float sacc = 0.0f;
#pragma unroll
                for (int x = 0; x < 32; ++x) sacc += sm.u.red[pi][c][x];
                sm.part[pi][c] = sacc;
            }
            __syncthreads();
            if (tg < 32) {
                float sacc = sm.yv[32 * J + tg];
                for (int pi = 0; pi < nparts; ++pi) sacc -= sm.part[pi][tg];
                sm.sv[tg] = sacc;
            }
            __syncthreads();
            if (tg < 32) {
                float w = 0.0f;
#pragma unroll
                for (int c = 0; c < 32; ++c) w += (c >= tg) ? sm.tT[0][tg][c] * sm.sv[c] : 0.0f;
                sm.wv[32 * J + tg] = w;
            }
            __syncthreads();
        }
        // ---- t = Q_S^T v
        if (live)
            for (int f = tg; f < k; f += C::TG) {
                float a0 = 0.0f, a1 = 0.0f;
                int x = 0;
                for (; x + 1 < deg; x += 2) {
                    a0 += sm.wv[x] * Q[(int64_t)sm.ids[x] * k + f];
                    a1 += sm.wv[x + 1] * Q[(int64_t)sm.ids[x + 1] * k + f];
                }
                if (x < deg) a0 += sm.wv[x] * Q[(int64_t)sm.ids[x] * k + f];
                Tout[(int64_t)li * k + f] = S ? S[(int64_t)li * k + f] - (a0 + a1) : a0 + a1;
            }
    }
}

template <int NT>
void launch_wood(hipStream_t st, const int32_t* rows, int32_t n, int32_t* counter,
                 const int64_t* off, const int32_t* cols, const float* Q, int32_t k, float alpha,
                 float* Tout, const float* S) {
    using C = WoodCfg<NT>;
    constexpr size_t lds = sizeof(WoodSmem<NT>) * C::R;
    static const bool attr = [] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wrmf_wood_kernel<NT>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        return true;
    }();
    (void)attr;
    MML_HIP(hipMemsetAsync(counter, 0, sizeof(int32_t), st));
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + C::R - 1) / C::R, 512));
    wrmf_wood_kernel<NT><<<grid, kThreads, lds, st>>>(rows, n, counter, off, cols, Q, k, alpha,
                                                      Tout, S);
}

// ---------------------------------------------------------------------------------------------
// Woodbury rows by conjugate gradients.  C = I/alpha + Q_S Q_S^T has its spectrum in
// [1/alpha, 1/alpha + 1]: Q_S Q_S^T = H_S B^{-1} H_S^T and H_S^T H_S <= HH <= B = HH + reg I, so
// cond(C) <= 1 + alpha and CG gains a factor (sqrt(1+alpha) - 1) / (sqrt(1+alpha) + 1) per step
// (0.17 at alpha = 1) whatever the row.  One 4-wave workgroup per row: thread f keeps column f of
// Q_S (deg <= NJ values) in registers for the whole solve, so each step is two register
// mat-vecs -- u = Q_S^T p (p broadcast from LDS) and z = Q_S u, whose sum over the 256 features
// is a transposing butterfly (each xor stage halves the values a lane carries, ~NJ shuffles per
// step instead of 6 NJ) plus a 4-wave LDS sum.  Output as wrmf_wood_kernel: t = Q_S^T v for
// C v = 1, or t = s - Q_S^T w for C w = Q_S s when S (a refinement pass) is given.
// Cross-lane steps without the LDS (ds_bpermute): lane i pairs with i ^ 32 through
// v_permlane32_swap, with i ^ 16 through v_permlane16_swap (gfx950), and within a 16-lane row with
// 15 - i (row_mirror), 7 - i within 8 (row_half_mirror), i ^ 2 and i ^ 1 (quad_perm) through DPP.
// Partners always differ in the stage's bit (5, 4, 3, 2, 1, 0) and agree above it, so the stages
// form a butterfly: after all six every lane has combined all 64.
__device__ __forceinline__ float fbits(uint32_t u) { return __uint_as_float(u); }
template <int STAGE>  // 0..5 = bit 5 .. bit 0
__device__ __forceinline__ float partner_of(float v) {
    if constexpr (STAGE == 2) return MML_DPP(v, 0x140);   // row_mirror
    if constexpr (STAGE == 3) return MML_DPP(v, 0x141);   // row_half_mirror
    if constexpr (STAGE == 4) return MML_DPP(v, 0x4E);    // quad_perm [2,3,0,1]
    if constexpr (STAGE == 5) return MML_DPP(v, 0xB1);    // quad_perm [1,0,3,2]
    return v;
}
// keep + partner's send, lane bit b = 5 - STAGE: lo lanes (bit clear) keep index x and hi lanes
// x + H; the permlane swaps do the exchange and the selection in one instruction per pair
template <int STAGE>
__device__ __forceinline__ float tstage(float a, float b, int lane) {  // a = v[x], b = v[x + H]
    if constexpr (STAGE == 0) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(a), __float_as_uint(b),
                                                        false, false);
        return fbits(r[0]) + fbits(r[1]);
    } else if constexpr (STAGE == 1) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(a), __float_as_uint(b),
                                                        false, false);
        return fbits(r[0]) + fbits(r[1]);
    } else {
        const bool lo = (lane & (32 >> STAGE)) == 0;
        return (lo ? a : b) + partner_of<STAGE>(lo ? b : a);
    }
}
// two independent tstage's on packed pairs (a.x with b.x, a.y with b.y): the swaps stay per
// register, the products and the sums after them become v_pk_mul_f32 / v_pk_add_f32
using f32x2 = __attribute__((ext_vector_type(2))) float;
template <int STAGE>
__device__ __forceinline__ f32x2 tstage2(f32x2 a, f32x2 b, int lane) {
    if constexpr (STAGE == 0 || STAGE == 1) {
        const auto r0 = STAGE == 0 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(a.x),
                                                                       __float_as_uint(b.x), false,
                                                                       false)
                                   : __builtin_amdgcn_permlane16_swap(__float_as_uint(a.x),
                                                                       __float_as_uint(b.x), false,
                                                                       false);
        const auto r1 = STAGE == 0 ? __builtin_amdgcn_permlane32_swap(__float_as_uint(a.y),
                                                                       __float_as_uint(b.y), false,
                                                                       false)
                                   : __builtin_amdgcn_permlane16_swap(__float_as_uint(a.y),
                                                                       __float_as_uint(b.y), false,
                                                                       false);
        return f32x2{fbits(r0[0]), fbits(r1[0])} + f32x2{fbits(r0[1]), fbits(r1[1])};
    } else {
        return f32x2{tstage<STAGE>(a.x, b.x, lane), tstage<STAGE>(a.y, b.y, lane)};
    }
}
template <int STAGE>
__device__ __forceinline__ float pstage(float x) {  // x + the partner's x
    if constexpr (STAGE == 0) {
        const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(x), __float_as_uint(x),
                                                        false, false);
        return fbits(r[0]) + fbits(r[1]);
    } else if constexpr (STAGE == 1) {
        const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(x), __float_as_uint(x),
                                                        false, false);
        return fbits(r[0]) + fbits(r[1]);
    } else {
        return x + partner_of<STAGE>(x);
    }
}

// v[0 .. SIZE) per lane -> sums over the 64 lanes, SIZE / 64 values per lane (lane l holds
// indices (SIZE / 64) l + x), or one value for SIZE < 64 (index l / (64 / SIZE))
template <int N, int SIZE, int STAGE>
struct XorReduce {
    __device__ static __forceinline__ void run(float (&v)[N], int lane) {
        if constexpr (STAGE < 6) {
            if constexpr (SIZE > 1) {
                constexpr int H = SIZE / 2;
#pragma unroll
                for (int x = 0; x < H; ++x) v[x] = tstage<STAGE>(v[x], v[x + H], lane);
                XorReduce<N, H, STAGE + 1>::run(v, lane);
            } else {
                v[0] = pstage<STAGE>(v[0]);
                XorReduce<N, 1, STAGE + 1>::run(v, lane);
            }
        }
    }
};

// (x, y) summed over the workgroup, in one pass (sdot: 2 x WAVES floats).  One barrier: the
// caller alternates two sdot buffers, and every earlier read of this buffer (two calls back) is
// ordered by the barriers between the calls.
template <int WAVES>
__device__ __forceinline__ float2 block_sum2(float x, float y, float* sdot) {
    x = pstage<0>(x); y = pstage<0>(y);
    x = pstage<1>(x); y = pstage<1>(y);
    x = pstage<2>(x); y = pstage<2>(y);
    x = pstage<3>(x); y = pstage<3>(y);
    x = pstage<4>(x); y = pstage<4>(y);
    x = pstage<5>(x); y = pstage<5>(y);
    if ((threadIdx.x & 63) == 0) {
        sdot[threadIdx.x >> 6] = x;
        sdot[WAVES + (threadIdx.x >> 6)] = y;
    }
    __syncthreads();
    float2 r = make_float2(0.0f, 0.0f);
#pragma unroll
    for (int w = 0; w < WAVES; ++w) {
        r.x += sdot[w];
        r.y += sdot[WAVES + w];
    }
    return r;
}

// NJ = 32 / 64: 4 waves, thread f holds q[0 .. NJ) of feature f.  NJ = 128: 8 waves, the items
// split in two halves of 64 (waves 0-3 / 4-7), so a thread holds 64 values (128 would spill);
// bounds of 4 waves per SIMD keep two such workgroups per CU (128 VGPRs), since the solve is
// barrier-latency bound.  NJ = 96 (rows of 65 .. 96 items): 12 waves, three parts of 32 items
// (32 values per thread, six waves per SIMD keep two workgroups per CU), instead of 128 slots
// of which up to half sit idle.  The CG is Chronopoulos-Gear's single-reduction form: one mat-vec
// w = C r and one fused reduction of (r.r, w.r) per step.
// (PARTS = 4 at NJ = 128: 16 waves of 32 items each, the experiments build's A/B)
template <int NJ>
constexpr int wood_parts() {
    return NJ == 96 ? 3 : NJ > 64 ? 2 : 1;
}
template <int NJ, int PARTS = wood_parts<NJ>()>
__global__ __launch_bounds__(256 * PARTS, PARTS == 3 ? 6 : PARTS >= 2 ? 4 : 2) void
wrmf_wood_cg_kernel(
    const int32_t* __restrict__ rows, int32_t n_list, const int64_t* __restrict__ off,
    const int32_t* __restrict__ cols, const float* __restrict__ Q, int32_t k, float alpha,
    const float* __restrict__ S, float* __restrict__ Tout, int32_t max_it, float tol2,
    float skip2, float abs2, int32_t cheb_m, float cheb_theta, float cheb_delta,
    float cheb_acosh, const int32_t* __restrict__ spos) {
    static_assert(NJ == 32 || NJ == 64 || NJ == 96 || NJ == 128, "NJ: 32, 64, 96 or 128");
    static_assert(NJ % PARTS == 0 && NJ / PARTS <= 64, "parts of <= 64 items");
    constexpr int HALVES = PARTS;
    constexpr int WAVES = 4 * HALVES;
    constexpr int NL = NJ / HALVES;             // items per thread (<= 64)
    constexpr int E = NL / 8;                   // partial sums after the fused first stages
    constexpr int NV = NL >= 64 ? NL / 64 : 1;  // butterfly outputs per lane
    constexpr int LPJ = NL >= 64 ? 1 : 64 / NL; // lanes holding one output (NL < 64)
    __shared__ int32_t sid[NJ];
    __shared__ float sp[NJ];
    __shared__ float su[HALVES][256];
    __shared__ float red[WAVES][NL];
    __shared__ float sdot[2][2 * WAVES];  // alternated per CG step (block_sum2)
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int f = t & 255, half = t >> 8, hw = wave & 3;  // feature, item half, wave in half
    const float ainv = 1.0f / alpha;
    const bool fon = f < k;
    for (int li = blockIdx.x; li < n_list; li += gridDim.x) {
        const int32_t row = rows[li];
        const int64_t rb = off[row];
        const int deg = (int)(off[row + 1] - rb);
        __syncthreads();  // the previous row is done with the LDS
        float sf = 0.0f;
        if (S) {
            // refinement, d = L^-T (s - Q_S^T w) with C w = Q_S s: |d|_2 <= |L^-1|_2 |s|_2 (the
            // middle factor I - Q_S^T C^-1 Q_S has norm <= 1), so a row whose bound is below the
            // absolute target keeps d = 0 without gathering Q_S
            const int64_t sl = spos ? spos[li] : li;  // s of list entry spos[li] (the screen)
            sf = fon && half == 0 ? S[sl * k + f] : 0.0f;
            const float2 ss = block_sum2<WAVES>(sf * sf, 0.0f, sdot[1]);
            if (ss.x <= skip2) {
                if (fon && half == 0) Tout[(int64_t)li * k + f] = 0.0f;
                continue;
            }
            if (half != 0) sf = fon ? S[sl * k + f] : 0.0f;
        }
        if (t < NJ) sid[t] = t < deg ? cols[rb + t] : 0;
        __syncthreads();
        float q[NL];
#pragma unroll
        for (int j = 0; j < NL; ++j) {
            const int jj = half * NL + j;
            q[j] = (fon && jj < deg) ? Q[(int64_t)sid[jj] * k + f] : 0.0f;
        }
        // z_j (thread j < NJ) = sum_f Q_S[j][f] uf; the first three butterfly stages (xor 32,
        // 16, 8) are fused per group of 8 products, so only NL / 8 partial sums sit next to q
        static_assert(E % 2 == 0, "packed pairs of partial sums");
        auto qs_times = [&](float uf) -> float {
            float v[E];
            const f32x2 u2 = {uf, uf};
#pragma unroll
            for (int x = 0; x < E; x += 2) {  // partial sums x and x + 1 as packed pairs
                f32x2 s1[4], s2[2];
#pragma unroll
                for (int c = 0; c < 4; ++c)
                    s1[c] = tstage2<0>(f32x2{q[x + c * E], q[x + 1 + c * E]} * u2,
                                       f32x2{q[x + (c + 4) * E], q[x + 1 + (c + 4) * E]} * u2,
                                       lane);
#pragma unroll
                for (int c = 0; c < 2; ++c) s2[c] = tstage2<1>(s1[c], s1[c + 2], lane);
                const f32x2 r = tstage2<2>(s2[0], s2[1], lane);
                v[x] = r.x;
                v[x + 1] = r.y;
            }
            XorReduce<E, E, 3>::run(v, lane);
            if constexpr (NL >= 64) {
#pragma unroll
                for (int x = 0; x < NV; ++x) red[wave][NV * lane + x] = v[x];
            } else {
                if (lane % LPJ == 0) red[wave][lane / LPJ] = v[0];
            }
            __syncthreads();
            float z = 0.0f;
            if (t < NJ) {
                const int h = t / NL, jl = t % NL;
#pragma unroll
                for (int w = 0; w < 4; ++w) z += red[4 * h + w][jl];
            }
            return z;
        };
        auto qt_times = [&]() -> float {  // u_f = sum_j Q_S[j][f] sp[j] (all threads: feature f)
            // two packed accumulators (v_pk_fma_f32): partial sums over j = 0, 1 mod 4 and 2, 3
            static_assert(NL % 4 == 0, "packed accumulators");
            f32x2 a0 = {0.0f, 0.0f}, a1 = {0.0f, 0.0f};
#pragma unroll
            for (int j = 0; j < NL; j += 4) {
                const float* pj = sp + half * NL + j;
                a0 = __builtin_elementwise_fma(f32x2{q[j], q[j + 1]}, f32x2{pj[0], pj[1]}, a0);
                a1 = __builtin_elementwise_fma(f32x2{q[j + 2], q[j + 3]}, f32x2{pj[2], pj[3]}, a1);
            }
            float u = (a0.x + a0.y) + (a1.x + a1.y);
            if constexpr (HALVES == 1) return u;
            su[half][f] = u;
            __syncthreads();
            float sum = su[0][f];
#pragma unroll
            for (int x = 1; x < HALVES; ++x) sum += su[x][f];
            return sum;
        };
        float y;
        if (S) {
            y = qs_times(sf);
        } else {
            y = t < deg ? 1.0f : 0.0f;
        }
        float w = 0.0f, r = t < deg ? y : 0.0f, p = 0.0f, sv = 0.0f;
        float g_prev = 1.0f, a_prev = 1.0f, stop = 0.0f;
        if (cheb_m > 0) {
            // Chebyshev iteration on a spectrum bound [1/alpha, 1/alpha + b] (centre theta,
            // half-width delta): no inner products, so no block reduction and no barrier beyond
            // the mat-vec's own; m updates take m - 1 mat-vecs.  b = min(1, tr): Q_S Q_S^T <=
            // Q^T Q <= I bounds it by 1 (the host's cheb_m, theta, delta), and its largest
            // eigenvalue is at most its trace tr = sum_{j in S} |q_j|^2, which for a row of a
            // few hundred entries out of hundreds of thousands is far below 1 (q_j's squared norm
            // is item j's leverage, summing to k over all rows): the same relative error bound
            // 2 / T_m(theta / delta) then takes m = acosh(2 / tol) / acosh(1 + 2 / (alpha b)) + 1
            // updates instead of the worst case's (C5 users: ~4 instead of 10)
            float qq = 0.0f;
#pragma unroll
            for (int j = 0; j < NL; ++j) qq += q[j] * q[j];
            const float tr = block_sum2<WAVES>(qq, 0.0f, sdot[1]).x;
            int m = cheb_m;
            float theta = cheb_theta, delta = cheb_delta;
            if (cheb_acosh > 0.0f && tr < 1.0f) {
                const float b = fmaxf(tr, 1e-20f);
                m = min(cheb_m, (int)ceilf(cheb_acosh / acoshf(1.0f + 2.0f / (alpha * b))) + 1);
                theta = ainv + 0.5f * b;
                delta = 0.5f * b;
            }
            const float s1 = theta / delta;
            float dv = r / theta, rho_p = 1.0f / s1;
            for (int it = 0; it < m; ++it) {
                w += dv;
                if (it + 1 == m) break;
                // the step's coefficients (scalars of the row alone) before the barrier, so their
                // division's latency hides behind it; the same float operations as after it
                const float rho = 1.0f / (2.0f * s1 - rho_p);
                const float c1 = rho * rho_p, c2 = 2.0f * rho / delta;
                if (t < NJ) sp[t] = dv;
                __syncthreads();
                const float uf = qt_times();
                r -= (t < deg ? dv * ainv : 0.0f) + qs_times(uf);  // r -= C d
                dv = c1 * dv + c2 * r;
                rho_p = rho;
            }
        }
        for (int it = 0; it <= (cheb_m > 0 ? -1 : max_it); ++it) {
            if (t < NJ) sp[t] = r;
            __syncthreads();
            const float uf = qt_times();
            const float cr = (t < deg ? r * ainv : 0.0f) + qs_times(uf);  // C r
            const float2 gd = block_sum2<WAVES>(t < NJ ? r * r : 0.0f, t < NJ ? cr * r : 0.0f,
                                                sdot[it & 1]);
            // relative target, or (refinement) the absolute one: d's error from w's is at most
            // |L^-1|_2 |C^-1|_2 |res| <= |L^-1|_2 alpha |res|
            if (it == 0) stop = fmaxf(tol2 * gd.x, abs2);
            if (gd.x <= stop || it == max_it) break;
            const float b = it == 0 ? 0.0f : gd.x / g_prev;
            const float a = it == 0 ? gd.x / gd.y : gd.x / (gd.y - b * gd.x / a_prev);
            p = r + b * p;
            sv = cr + b * sv;  // C p
            w += a * p;
            r -= a * sv;
            g_prev = gd.x;
            a_prev = a;
        }
        __syncthreads();
        if (t < NJ) sp[t] = t < deg ? w : 0.0f;
        __syncthreads();
        const float tf = qt_times();
        if (fon && half == 0) Tout[(int64_t)li * k + f] = S ? sf - tf : tf;
        (void)hw;
    }
}

// Woodbury rows of 65 .. 128 items on a 16 x 4 register block per thread.  Wave w owns items
// 16 w .. 16 w + 15 of the row and lane l features 4 l .. 4 l + 3 (one float4 of each item's Q
// row, so a gather is one 1 KiB row per wave-instruction).  Both mat-vecs of a step are register
// FMAs over the block:
//   z = Q_S u: 16 partial sums per lane, then a transposing butterfly inside the wave (16 values
//     over 64 lanes: item j0 + l / 4 ends in lanes 4 j .. 4 j + 3), no LDS;
//   u = Q_S^T p: p_j from v_readlane of its lane, 4 partial sums per lane, then the waves'
//     partials summed through the LDS in wave order (the step's only barrier).
// wrmf_wood_cg_kernel<128> spends three barriers and a 64-value butterfly per step, and its
// z sums cross four waves through the LDS.  Same parameters, same arithmetic (Chebyshev main
// solve, CG refinement), same output t.
template <int WAVES, bool VEC>  // VEC: k % 4 == 0 (a feature quad is one 16-B load)
__global__ __launch_bounds__(64 * WAVES, 4) void wrmf_wood_w16_kernel(
    const int32_t* __restrict__ rows, int32_t n_list, const int64_t* __restrict__ off,
    const int32_t* __restrict__ cols, const float* __restrict__ Q, int32_t k, float alpha,
    const float* __restrict__ S, float* __restrict__ Tout, int32_t max_it, float tol2,
    float skip2, float abs2, int32_t cheb_m, float cheb_theta, float cheb_delta,
    float cheb_acosh, const int32_t* __restrict__ spos) {
    static_assert(WAVES >= 1 && WAVES <= 8, "16 items per wave, <= 128 items");
    __shared__ float4 pu[2][WAVES][64];   // the waves' partial u, alternated per mat-vec
    __shared__ float sdot[2][2 * WAVES];  // block_sum2, alternated per CG step
    const int lane = threadIdx.x & 63;
    const int wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const int f0 = 4 * lane;
    constexpr bool vec = VEC;
    const float ainv = 1.0f / alpha;
    int par = 0;
    const int j0 = 16 * wave;
    // a row's item ids: rows[li] -> off[row] -> cols is a chain of three dependent loads ahead of
    // the Q gathers, so the next row's are fetched while this row computes (after its gathers are
    // issued).  The cols load is clamped into the row, no branch around it: the lanes past the
    // wave's items hold a valid id, whose gathered row is zeroed (j >= nloc)
    auto ids_of = [&](int l, int32_t& r, int64_t& b, int& d) -> int {
        r = rows[l];
        b = off[r];
        d = (int)(off[r + 1] - b);
        return cols[d > 0 ? b + min(j0 + lane, d - 1) : 0];
    };
    int32_t row = 0, row_n = 0;
    int64_t rb = 0, rb_n = 0;
    int deg = 0, deg_n = 0, idv = 0, idv_n = 0;
    if ((int)blockIdx.x < n_list) idv = ids_of(blockIdx.x, row, rb, deg);
    for (int li = blockIdx.x; li < n_list;
         li += gridDim.x, row = row_n, rb = rb_n, deg = deg_n, idv = idv_n) {
        const int ln = min(li + (int)gridDim.x, n_list - 1);  // (the last row: fetched again)
        const int nloc = __builtin_amdgcn_readfirstlane(max(0, min(16, deg - j0)));
        const bool live = j0 + (lane >> 2) < deg;  // the item this lane carries the state of
        __syncthreads();  // the previous row is done with the LDS
        float sf[4] = {0.0f, 0.0f, 0.0f, 0.0f};
        if (S) {
            // refinement: |d|_2 <= |L^-1|_2 |s|_2 (wrmf_wood_cg_kernel), a wave holds all of s
            const int64_t sl = spos ? spos[li] : li;  // s of list entry spos[li] (the screen)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                sf[c] = f0 + c < k ? S[sl * k + f0 + c] : 0.0f;
            float ss = (sf[0] * sf[0] + sf[1] * sf[1]) + (sf[2] * sf[2] + sf[3] * sf[3]);
            ss = pstage<0>(ss);
            ss = pstage<1>(ss);
            ss = pstage<2>(ss);
            ss = pstage<3>(ss);
            ss = pstage<4>(ss);
            ss = pstage<5>(ss);
            if (ss <= skip2) {  // the same sum in every wave: a workgroup-uniform branch
                if (wave == 0)
#pragma unroll
                    for (int c = 0; c < 4; ++c)
                        if (f0 + c < k) Tout[(int64_t)li * k + f0 + c] = 0.0f;
                idv_n = ids_of(ln, row_n, rb_n, deg_n);
                continue;
            }
        }
        // qp[c][jp] = (Q_S[2 jp][f0 + c], Q_S[2 jp + 1][f0 + c]): item pairs as packed operands
        f32x2 qp[4][8];
        if constexpr (vec) {
            // all 16 row loads in flight at once: no branch around a load (a load under a branch
            // is waited for before the join, which serialised the 16 gathers); the slots past the
            // wave's items re-read a valid row (ids_of) and are zeroed after the loads
            float4 g[16];
            const int fo = f0 < k ? f0 : 0;
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int id = __builtin_amdgcn_readlane(idv, j);
                g[j] = *reinterpret_cast<const float4*>(Q + (int64_t)id * k + fo);
            }
            // the next row's ids after all 16 gathers (the wait counter is in order: a gather
            // issued after them would make the first use of these wait for the ids too)
            __builtin_amdgcn_sched_barrier(0);
            idv_n = ids_of(ln, row_n, rb_n, deg_n);
            keep_loaded(g[0]);  // (the compiler sank slot 0's load under its select)
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const bool ok = j < nloc && f0 < k;
                qp[0][j >> 1][j & 1] = ok ? g[j].x : 0.0f;
                qp[1][j >> 1][j & 1] = ok ? g[j].y : 0.0f;
                qp[2][j >> 1][j & 1] = ok ? g[j].z : 0.0f;
                qp[3][j >> 1][j & 1] = ok ? g[j].w : 0.0f;
            }
        } else {
#pragma unroll
            for (int j = 0; j < 16; ++j) {
                const int id = __builtin_amdgcn_readlane(idv, j);
                const float* src = Q + (int64_t)id * k + f0;
                float4 v = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                if (j < nloc) {
                    v.x = f0 < k ? src[0] : 0.0f;
                    v.y = f0 + 1 < k ? src[1] : 0.0f;
                    v.z = f0 + 2 < k ? src[2] : 0.0f;
                    v.w = f0 + 3 < k ? src[3] : 0.0f;
                }
                qp[0][j >> 1][j & 1] = v.x;
                qp[1][j >> 1][j & 1] = v.y;
                qp[2][j >> 1][j & 1] = v.z;
                qp[3][j >> 1][j & 1] = v.w;
            }
            idv_n = ids_of(ln, row_n, rb_n, deg_n);
        }
        // z_j = sum_f Q_S[j][f] u_f for this wave's items: the lane's value for item j0 + l / 4
        auto z_of = [&](const float (&u)[4]) -> float {
            if (nloc == 0) return 0.0f;
            float v[16];
#pragma unroll
            for (int jp = 0; jp < 8; ++jp) {
                f32x2 a = qp[0][jp] * f32x2{u[0], u[0]};
#pragma unroll
                for (int c = 1; c < 4; ++c)
                    a = __builtin_elementwise_fma(qp[c][jp], f32x2{u[c], u[c]}, a);
                v[2 * jp] = a.x;
                v[2 * jp + 1] = a.y;
            }
            XorReduce<16, 16, 0>::run(v, lane);
            return v[0];
        };
        // u_f = sum_j Q_S[j][f] p_j (p_j = the state value of item j's lanes), every wave gets all
        // four of its features, summed over the waves in order
        auto u_of = [&](float pl, float (&u)[4]) {
            float a[4] = {0.0f, 0.0f, 0.0f, 0.0f};
            if (nloc > 0) {
                f32x2 pp[8];
#pragma unroll
                for (int jp = 0; jp < 8; ++jp)
                    pp[jp] = f32x2{lane_bcast(pl, 8 * jp), lane_bcast(pl, 8 * jp + 4)};
#pragma unroll
                for (int c = 0; c < 4; ++c) {
                    f32x2 acc = qp[c][0] * pp[0];
#pragma unroll
                    for (int jp = 1; jp < 8; ++jp) acc = __builtin_elementwise_fma(qp[c][jp], pp[jp], acc);
                    a[c] = acc.x + acc.y;
                }
            }
            pu[par][wave][lane] = make_float4(a[0], a[1], a[2], a[3]);
            __syncthreads();
            float4 s = pu[par][0][lane];
#pragma unroll
            for (int w = 1; w < WAVES; ++w) {
                const float4 x = pu[par][w][lane];
                s.x += x.x;
                s.y += x.y;
                s.z += x.z;
                s.w += x.w;
            }
            par ^= 1;
            u[0] = s.x;
            u[1] = s.y;
            u[2] = s.z;
            u[3] = s.w;
        };
        const float y = S ? z_of(sf) : (live ? 1.0f : 0.0f);
        float w = 0.0f, r = live ? y : 0.0f, p = 0.0f, sv = 0.0f;
        float g_prev = 1.0f, a_prev = 1.0f, stop = 0.0f;
        float u[4];
        if (cheb_m > 0) {
            // Chebyshev iteration on [1/alpha, 1/alpha + b], b = min(1, trace) (wrmf_wood_cg_kernel)
            f32x2 q2 = {0.0f, 0.0f};
#pragma unroll
            for (int c = 0; c < 4; ++c)
#pragma unroll
                for (int jp = 0; jp < 8; ++jp) q2 = __builtin_elementwise_fma(qp[c][jp], qp[c][jp], q2);
            const float tr = block_sum2<WAVES>(q2.x + q2.y, 0.0f, sdot[1]).x;
            int m = cheb_m;
            float theta = cheb_theta, delta = cheb_delta;
            if (cheb_acosh > 0.0f && tr < 1.0f) {
                const float b = fmaxf(tr, 1e-20f);
                m = min(cheb_m, (int)ceilf(cheb_acosh / acoshf(1.0f + 2.0f / (alpha * b))) + 1);
                theta = ainv + 0.5f * b;
                delta = 0.5f * b;
            }
            const float s1 = theta / delta;
            float dv = r / theta, rho_p = 1.0f / s1;
            for (int it = 0; it < m; ++it) {
                w += dv;
                if (it + 1 == m) break;
                // the step's coefficients before u_of's barrier (as in wrmf_wood_cg_kernel)
                const float rho = 1.0f / (2.0f * s1 - rho_p);
                const float c1 = rho * rho_p, c2 = 2.0f * rho / delta;
                u_of(dv, u);
                r -= (live ? dv * ainv : 0.0f) + z_of(u);  // r -= C d
                dv = c1 * dv + c2 * r;
                rho_p = rho;
            }
        }
        // CG (Chronopoulos-Gear, one fused reduction per step): each item counted by one lane
        const bool own = (lane & 3) == 0;
        for (int it = 0; it <= (cheb_m > 0 ? -1 : max_it); ++it) {
            u_of(r, u);
            const float cr = (live ? r * ainv : 0.0f) + z_of(u);  // C r
            const float2 gd = block_sum2<WAVES>(own ? r * r : 0.0f, own ? cr * r : 0.0f,
                                                sdot[it & 1]);
            if (it == 0) stop = fmaxf(tol2 * gd.x, abs2);
            if (gd.x <= stop || it == max_it) break;
            const float b = it == 0 ? 0.0f : gd.x / g_prev;
            const float a = it == 0 ? gd.x / gd.y : gd.x / (gd.y - b * gd.x / a_prev);
            p = r + b * p;
            sv = cr + b * sv;  // C p
            w += a * p;
            r -= a * sv;
            g_prev = gd.x;
            a_prev = a;
        }
        u_of(live ? w : 0.0f, u);  // t = Q_S^T w
        if (wave == 0)
#pragma unroll
            for (int c = 0; c < 4; ++c)
                if (f0 + c < k) Tout[(int64_t)li * k + f0 + c] = S ? sf[c] - u[c] : u[c];
    }
}

// MML_WRMF_WOOD16 (experiments builds): 0 = rows of 97 .. 128 items on wrmf_wood_cg_kernel<128>,
// 1 = 97 .. 128 only, 2 (default) = rows of 65 .. 96 items on wrmf_wood_w16_kernel<8> too, 3 = those
// on wrmf_wood_w16_kernel<6>.  With its gathers issued together (round 5) the w16 kernel takes the
// 65 .. 96-item rows in less time than wrmf_wood_cg_kernel<96, 3>: C5 127.0 + 36.2 -> 156.8 ms per
// iteration for both buckets (profiles/r5j/); in round 4 it was 45 ms against 36 for that bucket
int wood_w16_mode() {
    static const int v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOOD16");
        return e ? std::atoi(e) : 2;
    }();
    return v;
}
bool wood_w16() { return wood_w16_mode() > 0; }

// the item half's pipeline: the direct rows' first-pass residual of a row range runs on a second
// stream under the next range's main solve (wrmf_tile_plan, wrmf_tile_solve).  MML_WRMF_PIPE=n
// (experiments builds): n row ranges, 1 = off; MML_WRMF_PIPE_GRID: the residual kernel's grid
// while it shares the CUs with the solve.  12 by default (round 6, C5 per iteration on one box,
// two runs each: 4 ranges 685.2 / 690.0 ms, 8 677.5 / 680.6, 12 676.6 / 679.3, 16 676.8 / 676.2,
// profiles/r6/pipe_sweep/): the last range's residual, which runs alone, is shorter
int32_t pipe_batches() {
    static const int32_t v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_PIPE");
        return e ? std::max(1, std::min(16, std::atoi(e))) : 12;
    }();
    return v;
}
// grid caps of the row kernels, for A/B in experiments builds (the release build: the defaults)
int64_t exp_grid(const char* name, int64_t def) {
    const char* e = MML_EXPERIMENT_ENV(name);
    return e ? std::max<int64_t>(64, std::atoll(e)) : def;
}
int64_t rv_grid() {
    static const int64_t v = exp_grid("MML_WRMF_RV_GRID", 256 * 16);
    return v;
}
int pipe_grid() {
    static const int v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_PIPE_GRID");
        return e ? std::max(64, std::atoi(e)) : 8192;
    }();
    return v;
}

// MML_WRMF_WOOD=chol keeps the Cholesky Woodbury kernel (A/B measurements); the default solves
// the Woodbury rows by CG
bool wood_cg() {
    static const bool v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOOD");
        return !(e && std::string(e) == "chol");
    }();
    return v;
}

// the refinement's absolute target for a Woodbury row's correction d (2-norm, so also per entry
// relative to 1 + |x|): under one float ulp at |x| = 1 and a quarter of the fp64 mode's 2e-7.
// C5 (A/B, experiments build): refinement CG 118 ms per iteration at 1e-8, 90 at 3e-8, 12 at 1e-7
// (most rows' bound |L^-1| |s| then falls under the target before Q_S is gathered)
constexpr double kWoodAbs = 5e-8;

int debug_mask();
// rows of 65 .. 96 items on the 96-slot kernel (MML_WRMF_WOOD96=0 in experiments builds: 128)
bool wood96() {
    static const bool v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOOD96");
        return !(e && std::string(e) == "0");
    }();
    return v;
}
// MML_WRMF_WOOD128=4 (experiments builds): rows of 65 .. 128 items on 4 parts of 32 (16 waves)
int wood128_parts() {
    static const int v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOOD128");
        return e ? std::atoi(e) : 2;
    }();
    return v;
}
// the refinement's absolute target for a Woodbury row's correction (A/B in experiments builds)
double wood_abs() {
    static const double v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOOD_ABS");
        return e ? std::atof(e) : kWoodAbs;
    }();
    return v;
}
// a refinement row with |s|_2^2 <= this keeps d = 0 (|d|_2 <= |L^-1|_2 |s|_2)
float wood_skip2(double lnorm) {
    const double sk = lnorm > 0.0 ? wood_abs() / lnorm : 0.0;
    return (float)(sk * sk);
}

// The refinement's screen ahead of the Woodbury kernels.  A list entry whose |s|_2^2 (in fp64 here)
// is below the kernels' skip bound by a 1e-4 margin is one they would skip: its correction row D is
// zeroed here (what the row GEMM makes of t = 0).  The kernels' own fp32 sums are within ~1e-6 of
// the fp64 one.  The other entries go to a compact list (row, list position; in any order, rows are
// independent), and the kernels decide those, as without the screen.  C5's users: all skip.
__global__ __launch_bounds__(256) void wrmf_wood_screen_kernel(
    const int32_t* __restrict__ rows, int32_t n, const float* __restrict__ S, int32_t k,
    double lim, float* __restrict__ D, int32_t* __restrict__ crow, int32_t* __restrict__ cpos,
    int32_t* __restrict__ count) {
    const int lane = threadIdx.x & 63;
    const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
    for (int64_t li = w0; li < n; li += nw) {
        double ss = 0.0;
        for (int f = lane; f < k; f += 64) {
            const double v = S[li * k + f];
            ss += v * v;
        }
        for (int o = 32; o > 0; o >>= 1) ss += __shfl_xor(ss, o);
        ss = __shfl(ss, 0);  // lane 0's sum for every lane: one decision per wave
        const int32_t r = rows[li];
        if (ss <= lim) {
            for (int f = lane; f < k; f += 64) D[(int64_t)r * k + f] = 0.0f;
        } else if (lane == 0) {
            const int32_t c = atomicAdd(count, 1);
            crow[c] = r;
            cpos[c] = (int32_t)li;
        }
    }
}

// lnorm: |L^{-1}|_2 (refinement only); refined: fp64 refinement passes follow this main solve
// spos (refinement after wrmf_wood_screen_kernel): list entry li's s is S row spos[li]
void launch_wood_cg(hipStream_t st, int g, const int32_t* rows, int32_t n, const int64_t* off,
                    const int32_t* cols, const float* Q, int32_t k, float alpha, float* Tout,
                    const float* S, double lnorm = 0.0, bool refined = false,
                    const int32_t* spos = nullptr) {
    // 32 workgroups per CU, 16 times the w16 kernel's resident two: a workgroup's rows are a
    // shorter run, so the two resident ones drift out of step (one gathers while the other runs
    // its steps) and the launch ends on shorter tails.  C5 per iteration on one box, two runs each
    // (profiles/r6/wood_grid/): grid 512 674.9 / 677.9 ms, 1,024 (round 5) 669.7 / 671.7, 2,048
    // 665.8 / 665.2, 8,192 659.8 / 661.5, up to 1 M the same.  MML_WRMF_WOOD_GRID (experiments
    // builds): A/B
    static const int64_t grid_cap = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOOD_GRID");
        return e ? std::max<int64_t>(256, std::atoll(e)) : (int64_t)256 * 32;
    }();
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(n, grid_cap));
    // main solve: relative residual 1e-6 (fp32 CG stagnates not far below: a tighter target
    // just runs to max_it on trained factors), 1e-5 when the fp64 refinement follows and corrects
    // the rest (C5: the users' largest correction stays 0 / 0 / 1e-8 with 1e-6 / 1e-5 / 1e-4 and
    // the iteration takes 723.3 / 712.7 / 707.9 ms, profiles/r5al/).  A refinement correction d:
    // 3e-3.  The pass's
    // contraction on Woodbury rows is set by fp32 rounding in the CG as much as by this target
    // (1e-4 measured 0.027 .. 0.06 on the tests' sets, no better than 3e-3), so the error left is
    // bounded by further passes instead (kRefineStopWood), and C5, whose Woodbury corrections are
    // ~1e-8, keeps the cheaper target.  max_it = the steps the cond(C) <= 1 + alpha bound needs, + 4
    static const double refine_tol = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_REFINE_TOL");
        return e ? std::atof(e) : 3e-3;
    }();
    static const double main_tol = [] {  // MML_WRMF_MAIN_TOL (experiments builds): A/B
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_MAIN_TOL");
        return e ? std::atof(e) : 1e-5;
    }();
    const double tol = S ? refine_tol : refined ? main_tol : 1e-6;
    const double rho = (std::sqrt(1.0 + alpha) - 1.0) / (std::sqrt(1.0 + alpha) + 1.0);
    // MML_WRMF_DEBUG & 64 (timing only): no CG step, the gathers and the t = Q_S^T w pass alone
    const int max_it = (debug_mask() & 64) ? 0
                       : std::min(200, (int)std::ceil(std::log(tol) / std::log(rho)) + 4);
    const float tol2 = (float)(tol * tol);
    const double sk = S && lnorm > 0.0 ? wood_abs() / lnorm : 0.0, ab = sk / alpha;
    const float skip2 = S ? wood_skip2(lnorm) : -1.0f, abs2 = (float)(ab * ab);
    // the main solve by Chebyshev iteration: error <= 2 / T_m(theta / delta) relative, so
    // m = acosh(2 / tol) / acosh(theta / delta) updates, + 1 for fp32 (alpha = 1: 9 updates and 8
    // mat-vecs, against 13 mat-vecs and 13 block reductions for the CG at its step cap);
    // MML_WRMF_WOOD_MAIN=cg (experiments builds) keeps the CG
    static const bool main_cg = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOOD_MAIN");
        return e && std::string(e) == "cg";
    }();
    const double theta = 1.0 / alpha + 0.5, delta = 0.5;
    const int cheb_m = (S || main_cg || (debug_mask() & 64))
                           ? 0
                           : (int)std::ceil(std::acosh(2.0 / tol) / std::acosh(theta / delta)) + 1;
    // the per-row bound's numerator (the kernel takes the smaller of the two counts)
    static const bool row_bound = [] {  // MML_WRMF_CHEB_TRACE=0 (experiments builds): worst case only
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_CHEB_TRACE");
        return !(e && std::string(e) == "0");
    }();
    const float cheb_acosh = row_bound ? (float)std::acosh(2.0 / tol) : -1.0f;
    if (g == 2 && wood_w16_mode() == 3)
        ((k & 3) == 0 ? &wrmf_wood_w16_kernel<6, true> : &wrmf_wood_w16_kernel<6, false>)<<<
            grid, 64 * 6, 0, st>>>(rows, n, off, cols, Q, k, alpha, S, Tout, max_it, tol2, skip2,
                                   abs2, cheb_m, (float)theta, (float)delta, cheb_acosh, spos);
    else if ((g == 3 && wood_w16()) || (g == 2 && wood_w16_mode() == 2))
        ((k & 3) == 0 ? &wrmf_wood_w16_kernel<8, true> : &wrmf_wood_w16_kernel<8, false>)<<<
            grid, 64 * 8, 0, st>>>(rows, n, off, cols, Q, k, alpha, S, Tout, max_it, tol2, skip2,
                                   abs2, cheb_m, (float)theta, (float)delta, cheb_acosh, spos);
    else if (g == 0)
        wrmf_wood_cg_kernel<32><<<grid, 256, 0, st>>>(rows, n, off, cols, Q, k, alpha, S, Tout,
                                                      max_it, tol2, skip2, abs2, cheb_m,
                                                      (float)theta, (float)delta, cheb_acosh, spos);
    else if (g == 1)
        wrmf_wood_cg_kernel<64><<<grid, 256, 0, st>>>(rows, n, off, cols, Q, k, alpha, S, Tout,
                                                      max_it, tol2, skip2, abs2, cheb_m,
                                                      (float)theta, (float)delta, cheb_acosh, spos);
    else if (wood128_parts() == 4)
        wrmf_wood_cg_kernel<128, 4><<<grid, 1024, 0, st>>>(
            rows, n, off, cols, Q, k, alpha, S, Tout, max_it, tol2, skip2, abs2, cheb_m,
            (float)theta, (float)delta, cheb_acosh, spos);
    else if (g == 2 && wood96())
        wrmf_wood_cg_kernel<96><<<grid, 768, 0, st>>>(rows, n, off, cols, Q, k, alpha, S, Tout,
                                                      max_it, tol2, skip2, abs2, cheb_m,
                                                      (float)theta, (float)delta, cheb_acosh, spos);
    else
        wrmf_wood_cg_kernel<128><<<grid, 512, 0, st>>>(rows, n, off, cols, Q, k, alpha, S, Tout,
                                                       max_it, tol2, skip2, abs2, cheb_m,
                                                       (float)theta, (float)delta, cheb_acosh, spos);
}

// Y[yrow(r)] = scale * X[xrow(r)] * M for n rows (X, Y row-major [.. x k], M [k x k] row-major,
// k <= 256; xrows / yrows null = identity).  32 rows per workgroup staged in LDS, 4 waves x 2
// output tiles of 32 x 32 on v_mfma_f32_32x32x2_f32; M streams from L2.
constexpr int kGS = 257;  // LDS row stride of the staged rows
__global__ __launch_bounds__(256) void wrmf_rows_matmul_kernel(
    const float* __restrict__ X, const int32_t* __restrict__ xrows, int64_t n,
    const float* __restrict__ M, int32_t k, float scale, float* __restrict__ Y,
    const int32_t* __restrict__ yrows) {
    __shared__ float xs[32 * kGS];
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, q = lane & 31, h = lane >> 5;
    const int nct = (k + 31) >> 5;
    for (int64_t blk = blockIdx.x; blk * 32 < n; blk += gridDim.x) {
        const int64_t r0 = blk * 32;
        __syncthreads();
        for (int x = t; x < 32 * k; x += 256) {
            const int i = x / k, f = x - i * k;
            float v = 0.0f;
            if (r0 + i < n) {
                const int64_t src = xrows ? xrows[r0 + i] : r0 + i;
                v = X[src * k + f];
            }
            xs[i * kGS + f] = v;
        }
        __syncthreads();
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            const int J = wave * 2 + jt;
            if (J >= nct) continue;
            f32x16 d;
#pragma unroll
            for (int g = 0; g < 16; ++g) d[g] = 0.0f;
            const int col = 32 * J + q;
            for (int f0 = 0; f0 < k; f0 += 2) {
                const int f = f0 + h;
                const float a = f < k ? xs[q * kGS + f] : 0.0f;
                const float bv = (f < k && col < k) ? M[(int64_t)f * k + col] : 0.0f;
                d = __builtin_amdgcn_mfma_f32_32x32x2f32(a, bv, d, 0, 0, 0);
            }
            if (col < k)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int i = rho(g, h);
                    if (r0 + i < n) {
                        const int64_t dst = yrows ? yrows[r0 + i] : r0 + i;
                        Y[dst * k + col] = scale * d[g];
                    }
                }
        }
    }
}

// The same row GEMM on the bf16 matrix cores at f32 accuracy (the Gram's 3-way split, six
// products per K step, split3t): 2.7x fewer MFMA cycles than v_mfma_f32_32x32x2_f32.  M comes as
// its bf16 planes, transposed and K-padded (wrmf_split_mt_kernel, once per half-step), so a lane's
// B operand (8 consecutive k of one column) is one 16-B load from L2; X's rows are split into
// three bf16 planes in LDS (padded rows: the A reads are conflict-free per 16 lanes).
__global__ __launch_bounds__(256) void wrmf_split_mt_kernel(const float* __restrict__ M, int32_t k,
                                                            int32_t kpad,
                                                            uint16_t* __restrict__ MT) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)k * kpad;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int c = (int)(e / kpad), kk = (int)(e - (int64_t)c * kpad);
        const float v = kk < k ? M[(int64_t)kk * k + c] : 0.0f;
        uint32_t a, b, d;
        split3t(v, a, b, d);
        MT[((int64_t)0 * k + c) * kpad + kk] = (uint16_t)(a >> 16);
        MT[((int64_t)1 * k + c) * kpad + kk] = (uint16_t)(b >> 16);
        MT[((int64_t)2 * k + c) * kpad + kk] = (uint16_t)(d >> 16);
    }
}
// 64 rows per workgroup, so each 16-B B load from L2 feeds two row tiles (B is re-read once per 64
// rows instead of per 32: the kernel waits on those loads, 80 % of its wave cycles at 32 rows);
// wave w takes column tiles 2w and 2w + 1 for both row tiles (4 accumulators).  X is staged in K
// halves of kRH columns (3 planes x 64 rows x (kRH + 8) bf16 = 52 KB of LDS: 3 workgroups per CU).
constexpr int kRH = 128, kRHS = kRH + 8;
// three waves per SIMD: 163 VGPRs and no AGPRs (130 + 64 AGPRs at the default bounds: two waves),
// three workgroups per CU in 3 x 52 KB of LDS: 20.9 -> 19.1 ms per C5 iteration (profiles/r4t_*)
#ifndef MML_MATMUL_WAVES
#define MML_MATMUL_WAVES 3
#endif
__global__ __launch_bounds__(256, MML_MATMUL_WAVES) void wrmf_rows_matmul_x3_kernel(
    const float* __restrict__ X, const int32_t* __restrict__ xrows, int64_t n,
    const uint16_t* __restrict__ MT, int32_t k, int32_t kpad, float scale, float* __restrict__ Y,
    const int32_t* __restrict__ yrows) {
    __shared__ __attribute__((aligned(16))) uint16_t xs[3][64 * kRHS];
    __shared__ int64_t srow[2][64];  // the block's source / destination rows (-1: past n)
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6, q = lane & 31, h = lane >> 5;
    const int nct = (k + 31) >> 5;
    const bool vec = (k & 3) == 0;
    const int64_t pstride = (int64_t)k * kpad;
    for (int64_t blk = blockIdx.x; blk * 64 < n; blk += gridDim.x) {
        const int64_t r0 = blk * 64;
        __syncthreads();
        if (t < 128) {  // the row ids once per block: staging and stores read them from LDS
            const int i = t & 63;
            const int32_t* ids = t < 64 ? xrows : yrows;
            srow[t >> 6][i] = r0 + i < n ? (ids ? (int64_t)ids[r0 + i] : r0 + i) : -1;
        }
        f32x16 d[2][2];
#pragma unroll
        for (int rt = 0; rt < 2; ++rt)
#pragma unroll
            for (int jt = 0; jt < 2; ++jt)
#pragma unroll
                for (int g = 0; g < 16; ++g) d[rt][jt][g] = 0.0f;
        for (int k0 = 0; k0 < kpad; k0 += kRH) {
            const int kw = min(kRH, kpad - k0);  // a multiple of 16
            __syncthreads();  // the previous half's reads (and the row ids' writes) are done
            auto put = [&](int i, int fl, const float (&v)[4]) {
                uint32_t a[4], b[4], c[4];
#pragma unroll
                for (int j = 0; j < 4; ++j) split3t(v[j], a[j], b[j], c[j]);
                *reinterpret_cast<uint2*>(&xs[0][i * kRHS + fl]) =
                    make_uint2(pack_hi(a[0], a[1]), pack_hi(a[2], a[3]));
                *reinterpret_cast<uint2*>(&xs[1][i * kRHS + fl]) =
                    make_uint2(pack_hi(b[0], b[1]), pack_hi(b[2], b[3]));
                *reinterpret_cast<uint2*>(&xs[2][i * kRHS + fl]) =
                    make_uint2(pack_hi(c[0], c[1]), pack_hi(c[2], c[3]));
            };
            if (vec) {
                // the half's kRH / 16 row gathers per thread issued together (clamped addresses,
                // zeroed after): under a branch each was waited for before the next went out
                constexpr int kG = kRH / 16;
                float4 g[kG];
#pragma unroll
                for (int it = 0; it < kG; ++it) {  // 4 consecutive k of one row
                    const int x = 4 * t + 1024 * it, i = min(x / kw, 63), f = k0 + x - i * kw;
                    const int64_t sr = srow[0][i];
                    g[it] = *reinterpret_cast<const float4*>(X + (sr >= 0 ? sr : 0) * k +
                                                             (f + 3 < k ? f : 0));
                }
#pragma unroll
                for (int it = 0; it < kG; ++it) {
                    const int x = 4 * t + 1024 * it;
                    keep_loaded(g[it]);
                    if (x < 64 * kw) {
                        const int i = x / kw, fl = x - i * kw;
                        const bool ok = srow[0][i] >= 0 && k0 + fl + 3 < k;
                        const float v[4] = {ok ? g[it].x : 0.0f, ok ? g[it].y : 0.0f,
                                            ok ? g[it].z : 0.0f, ok ? g[it].w : 0.0f};
                        put(i, fl, v);
                    }
                }
            } else {
                for (int x = 4 * t; x < 64 * kw; x += 4 * 256) {  // 4 consecutive k of one row
                    const int i = x / kw, fl = x - i * kw, f = k0 + fl;
                    float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                    const int64_t sr = srow[0][i];
                    if (sr >= 0) {
                        const float* src = X + sr * k;
#pragma unroll
                        for (int j = 0; j < 4; ++j) v[j] = f + j < k ? src[f + j] : 0.0f;
                    }
                    put(i, fl, v);
                }
            }
            __syncthreads();
            for (int kc = 0; kc < kw; kc += 16) {
                bf16x8 B[2][3], A[2][3];
#pragma unroll
                for (int jt = 0; jt < 2; ++jt) {
                    const int col = 32 * (wave * 2 + jt) + q;
                    const uint16_t* m0 = MT + (int64_t)(col < k ? col : 0) * kpad + k0 + kc + 8 * h;
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        B[jt][p] = *reinterpret_cast<const bf16x8*>(m0 + p * pstride);
                }
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int p = 0; p < 3; ++p)
                        A[rt][p] = *reinterpret_cast<const bf16x8*>(
                            &xs[p][(32 * rt + q) * kRHS + kc + 8 * h]);
#pragma unroll
                for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                    for (int jt = 0; jt < 2; ++jt) {
                        if (wave * 2 + jt >= nct) continue;
                        f32x16 e = d[rt][jt];
                        e = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][2], B[jt][0], e, 0, 0, 0);
                        e = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][1], B[jt][1], e, 0, 0, 0);
                        e = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][0], B[jt][2], e, 0, 0, 0);
                        e = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][1], B[jt][0], e, 0, 0, 0);
                        e = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][0], B[jt][1], e, 0, 0, 0);
                        e = __builtin_amdgcn_mfma_f32_32x32x16_bf16(A[rt][0], B[jt][0], e, 0, 0, 0);
                        d[rt][jt] = e;
                    }
            }
        }
#pragma unroll
        for (int jt = 0; jt < 2; ++jt) {
            const int col = 32 * (wave * 2 + jt) + q;
            if (col >= k) continue;
#pragma unroll
            for (int rt = 0; rt < 2; ++rt)
#pragma unroll
                for (int g = 0; g < 16; ++g) {
                    const int64_t dst = srow[1][32 * rt + rho(g, h)];
                    if (dst >= 0) Y[dst * k + col] = scale * d[rt][jt][g];
                }
        }
    }
}

// Y = scale X M through the bf16x3 kernel (MX: M's planes from wrmf_split_mt_kernel), or the f32
// MFMA kernel with MML_WRMF_GEMM=f32 (A/B)
bool gemm_f32() {
    static const bool v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_GEMM");
        return e && std::string(e) == "f32";
    }();
    return v;
}
void rows_matmul(hipStream_t st, const float* X, const int32_t* xrows, int64_t n, const float* M,
                 const uint16_t* MX, int32_t k, float scale, float* Y, const int32_t* yrows) {
    const int grid = (int)std::min<int64_t>((n + 31) / 32, 8192);
    const int grid64 = (int)std::min<int64_t>((n + 63) / 64, 8192);
    if (gemm_f32())
        wrmf_rows_matmul_kernel<<<grid, 256, 0, st>>>(X, xrows, n, M, k, scale, Y, yrows);
    else
        wrmf_rows_matmul_x3_kernel<<<grid64, 256, 0, st>>>(X, xrows, n, MX, k, (k + 15) & ~15,
                                                           scale, Y, yrows);
}

// MML_WRMF_DEBUG: phase-skip mask for timing experiments only (results are wrong when set):
// 1 diagonal factorisation, 2 panel MFMAs, 4 backward substitution, 8 Gram, 64 no CG steps
int debug_mask() {
    static const int v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_DEBUG");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}

// ---- fp64 iterative refinement: r = b - A x = sum_{i in S} ((1 + alpha) - alpha h_i.x) h_i
//      - (HH + reg I) x, the first term per entry segment (one wave per entry, lane l holds
//      features 4l .. 4l + 3: h_i.x by a wave reduction, then the scaled h_i accumulated), the
//      second by one dgemm over all rows (R is initialised to it).  float * float products are
//      exact in double, so A is the reference's matrix up to its own float rounding of products.
struct RSeg {
    int32_t row;   // local row (row - r0)
    int32_t slot;  // -1: the row's only segment (adds into R); else its partial's slot
    int64_t b, e;
};
struct RMulti {
    int32_t row, slot0, nslot, pad;
};
constexpr int kRSeg = 2048;  // entries per residual segment

// doubles across lanes, both 32-bit halves moved by the same instruction
__device__ __forceinline__ uint32_t lo32(double v) { return (uint32_t)(uint64_t)__double_as_longlong(v); }
__device__ __forceinline__ uint32_t hi32(double v) {
    return (uint32_t)((uint64_t)__double_as_longlong(v) >> 32);
}
__device__ __forceinline__ double f64_of(uint32_t lo, uint32_t hi) {
    return __longlong_as_double((long long)(((uint64_t)hi << 32) | lo));
}
template <int CTRL>
__device__ __forceinline__ double dpp_f64(double v) {
    return f64_of((uint32_t)__builtin_amdgcn_update_dpp(0, (int)lo32(v), CTRL, 0xF, 0xF, false),
                  (uint32_t)__builtin_amdgcn_update_dpp(0, (int)hi32(v), CTRL, 0xF, 0xF, false));
}
__device__ __forceinline__ double readlane_f64(double v, int l) {
    return f64_of((uint32_t)__builtin_amdgcn_readlane((int)lo32(v), l),
                  (uint32_t)__builtin_amdgcn_readlane((int)hi32(v), l));
}
// The butterfly of the CG kernel's tstage / pstage on doubles: stage s pairs lanes differing in bit
// 5 - s (permlane32 / permlane16 swaps, then row_mirror, row_half_mirror, quad_perm xor 2 / xor 1)
template <int STAGE>
__device__ __forceinline__ double partner_f64(double v) {
    if constexpr (STAGE == 2) return dpp_f64<0x140>(v);
    if constexpr (STAGE == 3) return dpp_f64<0x141>(v);
    if constexpr (STAGE == 4) return dpp_f64<0x4E>(v);
    return dpp_f64<0xB1>(v);
}
template <int STAGE>  // a = v[x], b = v[x + H]: lanes with the stage's bit clear keep x, set x + H
__device__ __forceinline__ double tstage_f64(double a, double b, int lane) {
    if constexpr (STAGE <= 1) {
        const auto rl = STAGE == 0 ? __builtin_amdgcn_permlane32_swap(lo32(a), lo32(b), false, false)
                                   : __builtin_amdgcn_permlane16_swap(lo32(a), lo32(b), false, false);
        const auto rh = STAGE == 0 ? __builtin_amdgcn_permlane32_swap(hi32(a), hi32(b), false, false)
                                   : __builtin_amdgcn_permlane16_swap(hi32(a), hi32(b), false, false);
        return f64_of(rl[0], rh[0]) + f64_of(rl[1], rh[1]);
    } else {
        const bool lo = (lane & (32 >> STAGE)) == 0;
        return (lo ? a : b) + partner_f64<STAGE>(lo ? b : a);
    }
}
template <int STAGE>
__device__ __forceinline__ double pstage_f64(double x) {
    return x + partner_f64<STAGE>(x);
}

// One wave per entry segment, lane l holding features 4 l .. 4 l + 3 (h_i's 1 KB row is one
// coalesced float4 load per lane).  The segment's column ids are read 64 at a time (one load), and
// kResE entries per step are in flight together: their rows are loaded, h_i.x is summed by a
// transposing butterfly (kResE values per lane -> one, 3 swaps + 3 DPP stages, no LDS), and each
// entry's sum is read back from lane 8 u.  No barrier and no LDS: a wave's only dependent latencies
// are its segment's ids and its rows, so thousands of waves keep the gathers in flight.  The order
// of every sum is fixed (deterministic).
constexpr int kResE = 8;
// X: fp64 rows, or (first pass) the fp32 W rows, widened on load.  VEC: k % 4 == 0 (a feature quad
// is one 16-B load).  Five waves per SIMD (<= 96 VGPRs): a wave per SIMD then fits beside the tile
// solve's two (2 x 208 registers) when a batch's residual runs under the next batch's solve.
template <typename XT, bool VEC>
__global__ __launch_bounds__(256, 5) void wrmf_resid_seg_kernel(
    const RSeg* __restrict__ segs, int64_t nseg, const int32_t* __restrict__ cols,
    const float* __restrict__ H, int32_t k, const XT* __restrict__ X, double alpha,
    double* __restrict__ R, double* __restrict__ partial) {
    static_assert(kResE == 8, "the butterfly below reduces 8 entries");
    const int lane = threadIdx.x & 63, f0 = 4 * lane;
    const int64_t wave0 =
        (int64_t)blockIdx.x * 4 + __builtin_amdgcn_readfirstlane((int)(threadIdx.x >> 6));
    const int64_t nwave = (int64_t)gridDim.x * 4;
    constexpr bool vec = VEC;
    for (int64_t s = wave0; s < nseg; s += nwave) {
        const RSeg sg = segs[s];
        const XT* xr = X + (int64_t)sg.row * k;
        XT x[4];  // kept in X's own type (widened at each use: exact), 4 registers fewer for fp32
        double acc[4];
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            x[j] = f0 + j < k ? xr[f0 + j] : XT(0);
            acc[j] = 0.0;
        }
        for (int64_t e0 = sg.b; e0 < sg.e; e0 += 64) {
            const int n = (int)min((int64_t)64, sg.e - e0);
            const int32_t my = lane < n ? cols[e0 + lane] : 0;
            for (int x0 = 0; x0 < n; x0 += kResE) {
                float4 g[kResE];  // the entries' h_i features f0 .. f0 + 3 (0 past the segment)
                if constexpr (vec) {
                    // the kResE row loads issued together, none under a branch (entries past the
                    // segment read row my = 0 and are zeroed in place after): a load under a
                    // branch was waited for before the next one was issued
                    const int fo = f0 < k ? f0 : 0;
#pragma unroll
                    for (int u = 0; u < kResE; ++u)
                        g[u] = *reinterpret_cast<const float4*>(
                            H + (int64_t)__builtin_amdgcn_readlane(my, x0 + u) * k + fo);
#pragma unroll
                    for (int u = 0; u < kResE; ++u) {
                        keep_loaded(g[u]);
                        if (!(x0 + u < n && f0 < k)) g[u] = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
                    }
                } else {
#pragma unroll
                    for (int u = 0; u < kResE; ++u) {
                        float v[4] = {0.0f, 0.0f, 0.0f, 0.0f};
                        if (x0 + u < n) {  // wave-uniform; entries past the segment have h = 0
                            const float* hr =
                                H + (int64_t)__builtin_amdgcn_readlane(my, x0 + u) * k;
#pragma unroll
                            for (int j = 0; j < 4; ++j) v[j] = f0 + j < k ? hr[f0 + j] : 0.0f;
                        }
                        g[u] = make_float4(v[0], v[1], v[2], v[3]);
                    }
                }
                double t[kResE];
#pragma unroll
                for (int u = 0; u < kResE; ++u)
                    t[u] = (double)g[u].x * (double)x[0] + (double)g[u].y * (double)x[1] +
                           (double)g[u].z * (double)x[2] + (double)g[u].w * (double)x[3];
                double a4[4], a2[2];
#pragma unroll
                for (int u = 0; u < 4; ++u) a4[u] = tstage_f64<0>(t[u], t[u + 4], lane);
#pragma unroll
                for (int u = 0; u < 2; ++u) a2[u] = tstage_f64<1>(a4[u], a4[u + 2], lane);
                double a1 = tstage_f64<2>(a2[0], a2[1], lane);  // entry lane / 8
                a1 = pstage_f64<3>(a1);
                a1 = pstage_f64<4>(a1);
                a1 = pstage_f64<5>(a1);
#pragma unroll
                for (int u = 0; u < kResE; ++u) {
                    const double c = (1.0 + alpha) - alpha * readlane_f64(a1, 8 * u);
                    acc[0] += c * (double)g[u].x;
                    acc[1] += c * (double)g[u].y;
                    acc[2] += c * (double)g[u].z;
                    acc[3] += c * (double)g[u].w;
                }
            }
        }
#pragma unroll
        for (int j = 0; j < 4; ++j) {
            const int f = f0 + j;
            if (f < k) {
                if (sg.slot < 0)
                    R[(int64_t)sg.row * k + f] += acc[j];
                else
                    partial[(int64_t)sg.slot * k + f] = acc[j];
            }
        }
    }
}

// rows with several segments: R += their partials, in segment order (deterministic)
__global__ __launch_bounds__(256) void wrmf_resid_multi_kernel(const RMulti* __restrict__ m,
                                                               int64_t n, int32_t k,
                                                               const double* __restrict__ partial,
                                                               double* __restrict__ R) {
    for (int64_t x = blockIdx.x; x < n; x += gridDim.x) {
        const RMulti r = m[x];
        for (int f = threadIdx.x; f < k; f += blockDim.x) {
            double v = 0.0;
            for (int s = 0; s < r.nslot; ++s) v += partial[(int64_t)(r.slot0 + s) * k + f];
            R[(int64_t)r.row * k + f] += v;
        }
    }
}

// rows [r0, r0 + n): op 0 X = (double) W, 1 Rf = (float) R, 2 X += D, 3 W = (float) X
// The refinement residual's dense part on the fp64 matrix cores: R = -X (HH + reg I) for the rows
// of X ([n x k] fp64, row-major; HH symmetric, so X HH = (HH x_r^T)^T per row).  A workgroup takes
// 64 rows and all k <= 256 columns: 4 waves x 16 rows, 16 column tiles of v_mfma_f64_16x16x4_f64
// each (64 f64 accumulators per lane); K runs in chunks of 16 staged through LDS, HH's chunk
// (16 x 256) shared by the 4 waves, double-buffered so the next chunk's loads fly during the
// current chunk's 64 MFMAs per wave.  (Replaces the rocBLAS dgemm: the training path links no
// vendor BLAS.)
using f64x4 = __attribute__((ext_vector_type(4))) double;
#ifndef MML_XHH_K  // the K chunk of wrmf_xhh_kernel: LDS 42 KB at 8 (83 KB at 16: one workgroup per CU)
#define MML_XHH_K 8
#endif
constexpr int kXB = 64, kXK = MML_XHH_K, kXN = 256, kXNP = kXN + 2, kXKP = kXK + 1;
constexpr int kXV = kXK / 4;  // X values per thread and chunk
// two waves per SIMD: the accumulators move from AGPRs to VGPRs (192 registers, no spills) and two
// workgroups share a CU.  With one (K chunk 16) the kernel held 358 registers and ran one wave per
// SIMD: 23.8 -> 16.7 ms per C5 iteration (profiles/r4r_c5_*_kernel_stats.csv)
#ifndef MML_XHH_WAVES
#define MML_XHH_WAVES 2
#endif
template <typename XT>  // X: fp64 rows, or (first pass) the fp32 W rows, widened on load
__global__ __launch_bounds__(256, MML_XHH_WAVES) void wrmf_xhh_kernel(const XT* __restrict__ X,
                                                       const double* __restrict__ HH, int64_t n,
                                                       int32_t k, double reg,
                                                       double* __restrict__ R, int add) {
    __shared__ double sb[2][kXK][kXNP];
    __shared__ double sa[2][kXB][kXKP];
    const int t = threadIdx.x, wave = t >> 6, lane = t & 63, i = lane & 15, kk = lane >> 4;
    const int nk = (k + kXK - 1) / kXK;
    for (int64_t r0 = (int64_t)blockIdx.x * kXB; r0 < n; r0 += (int64_t)gridDim.x * kXB) {
        f64x4 acc[16];
#pragma unroll
        for (int jt = 0; jt < 16; ++jt) acc[jt] = f64x4{0.0, 0.0, 0.0, 0.0};
        // staging of chunk c into buffer bb: HH rows c*16 .. +16 (all columns), X rows r0 .. r0+64
        // columns c*16 .. +16; zero past k and past n
        // the chunk's loads go out unconditionally (clamped in-range addresses; the values past k
        // or n are zeroed when stored to LDS): a select around a load became a branch, and each
        // load was waited for before the next was issued, so the prefetch of chunk c + 1 did not
        // fly under chunk c's MFMAs
        double hv[kXK], xv[kXV];
        auto load = [&](int c) {
            const int tc = t < k ? t : k - 1;
#pragma unroll
            for (int x = 0; x < kXK; ++x) {  // kXK x 256 HH values: thread t -> row x, column t
                const int f = min(c * kXK + x, k - 1);
                hv[x] = HH[(int64_t)f * k + tc];
            }
            const int64_t row = min(r0 + (t >> 2), n - 1);
#pragma unroll
            for (int x = 0; x < kXV; ++x) {  // 64 x kXK X values: row t / 4, col kXV (t % 4) + x
                const int f = min(c * kXK + kXV * (t & 3) + x, k - 1);
                xv[x] = X[row * k + f];
            }
        };
        auto store = [&](int bb, int c) {
#pragma unroll
            for (int x = 0; x < kXK; ++x) sb[bb][x][t] = (c * kXK + x < k && t < k) ? hv[x] : 0.0;
            const bool rin = r0 + (t >> 2) < n;
#pragma unroll
            for (int x = 0; x < kXV; ++x)
                sa[bb][t >> 2][kXV * (t & 3) + x] =
                    (rin && c * kXK + kXV * (t & 3) + x < k) ? xv[x] : 0.0;
        };
        load(0);
        __syncthreads();  // the previous row block's last chunk has been read
        store(0, 0);
        __syncthreads();
        for (int c = 0; c < nk; ++c) {
            const int bb = c & 1;
            if (c + 1 < nk) load(c + 1);  // in flight during this chunk's MFMAs
#pragma unroll
            for (int s = 0; s < kXK / 4; ++s) {
                const double a = sa[bb][16 * wave + i][4 * s + kk];
#pragma unroll
                for (int jt = 0; jt < 16; ++jt)
                    acc[jt] = __builtin_amdgcn_mfma_f64_16x16x4f64(a, sb[bb][4 * s + kk][16 * jt + i],
                                                                   acc[jt], 0, 0, 0);
            }
            if (c + 1 < nk) store(bb ^ 1, c + 1);
            __syncthreads();
        }
        // D layout: column 16 jt + (lane & 15), row 4 v + (lane >> 4) of the wave's 16 rows
        // X's values for two column tiles loaded together (clamped addresses, no branch), then the
        // in-range stores
#pragma unroll
        for (int j2 = 0; j2 < 16; j2 += 2) {
            double xe[2][4];
#pragma unroll
            for (int u = 0; u < 2; ++u)
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int64_t row = min(r0 + 16 * wave + 4 * v + kk, n - 1);
                    xe[u][v] = X[row * k + min(16 * (j2 + u) + i, k - 1)];
                }
#pragma unroll
            for (int u = 0; u < 2; ++u) {
                const int col = 16 * (j2 + u) + i;
#pragma unroll
                for (int v = 0; v < 4; ++v) {
                    const int64_t row = r0 + 16 * wave + 4 * v + kk;
                    if (col < k && row < n) {
                        const double t = -acc[j2 + u][v] - reg * xe[u][v];
                        R[row * k + col] = add ? R[row * k + col] + t : t;
                    }
                }
            }
        }
    }
}

// op 0: X = W; 1: Rf = R; 2: X += D and W = (float) X, and dmax[t] = max |D| / (1 + |X|) over the
// rows of type t (0 direct, 1 Woodbury: 1 <= deg <= kWood when wood): the size of the correction
// relative to the solution, i.e. the error the pass removed; 3: W = X; 4: op 2 on the first pass,
// whose x is W itself (X = (double) W + D: no op 0 before it, no op 3 after the last pass)
__global__ __launch_bounds__(256) void wrmf_refine_rows_kernel(int op, int64_t r0, int64_t n,
                                                               int32_t k, float* __restrict__ W,
                                                               double* __restrict__ X,
                                                               const double* __restrict__ R,
                                                               float* __restrict__ Rf,
                                                               const float* __restrict__ D,
                                                               const int64_t* __restrict__ off,
                                                               int wood,
                                                               unsigned* __restrict__ dmax) {
    // one row per block step, the features across the threads: the row (and, for op 2, its type)
    // is known per step instead of a 64-bit division per element
    float m[2] = {0.0f, 0.0f};
    for (int64_t lr = blockIdx.x; lr < n; lr += gridDim.x) {
        const int64_t row = r0 + lr;
        const int64_t le = lr * k, ge = row * k;
        int t = 0;
        if (op == 2 || op == 4) {
            const int64_t deg = off[row + 1] - off[row];
            t = wood && deg >= 1 && deg <= 128 ? 1 : 0;
        }
        for (int f = threadIdx.x; f < k; f += blockDim.x) {
            switch (op) {
                case 0: X[le + f] = (double)W[ge + f]; break;
                case 1: Rf[ge + f] = (float)R[le + f]; break;
                case 2:
                case 4: {
                    const double x = (op == 4 ? (double)W[ge + f] : X[le + f]) + (double)D[ge + f];
                    X[le + f] = x;
                    W[ge + f] = (float)x;
                    const float c = (float)(fabs((double)D[ge + f]) / (1.0 + fabs(x)));
                    m[t] = fmaxf(m[t], c);
                    break;
                }
                default: W[ge + f] = (float)X[le + f]; break;
            }
        }
    }
    if (op == 2 || op == 4)  // non-negative floats order like their bit patterns
        for (int t = 0; t < 2; ++t) {
            float v = m[t];
            for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
            if ((threadIdx.x & 63) == 0 && v > 0.0f) atomicMax(dmax + t, __float_as_uint(v));
        }
}

// The same ops with one wave per row and four features per lane (k % 4 == 0): 16-B loads and
// stores, the row's type read once per wave, four rows per workgroup.  The per-element arithmetic
// is the scalar kernel's, so the results are the same bit for bit.  (The scalar kernel, a row per
// workgroup and a float per thread, ran C5's users' op 4 at 25 GB in 6.7 ms.)
__global__ __launch_bounds__(256) void wrmf_refine_rows_vec_kernel(int op, int64_t r0, int64_t n,
                                                                   int32_t k, float* __restrict__ W,
                                                                   double* __restrict__ X,
                                                                   const double* __restrict__ R,
                                                                   float* __restrict__ Rf,
                                                                   const float* __restrict__ D,
                                                                   const int64_t* __restrict__ off,
                                                                   int wood,
                                                                   unsigned* __restrict__ dmax) {
    const int lane = threadIdx.x & 63, f0 = 4 * lane;
    const bool on = f0 < k;
    float m0 = 0.0f, m1 = 0.0f;
    const int64_t w0 = (int64_t)blockIdx.x * 4 + (threadIdx.x >> 6), nw = (int64_t)gridDim.x * 4;
    for (int64_t lr = w0; lr < n; lr += nw) {
        const int64_t row = r0 + lr, le = lr * k + f0, ge = row * k + f0;
        bool t = false;
        if (op == 2 || op == 4) {
            const int64_t deg = off[row + 1] - off[row];
            t = wood && deg >= 1 && deg <= 128;
        }
        if (!on) continue;
        if (op == 0) {
            const float4 w = *reinterpret_cast<const float4*>(W + ge);
            *reinterpret_cast<double2*>(X + le) = make_double2((double)w.x, (double)w.y);
            *reinterpret_cast<double2*>(X + le + 2) = make_double2((double)w.z, (double)w.w);
        } else if (op == 1) {
            const double2 a = *reinterpret_cast<const double2*>(R + le);
            const double2 b = *reinterpret_cast<const double2*>(R + le + 2);
            *reinterpret_cast<float4*>(Rf + ge) =
                make_float4((float)a.x, (float)a.y, (float)b.x, (float)b.y);
        } else if (op == 2 || op == 4) {
            const float4 d4 = *reinterpret_cast<const float4*>(D + ge);
            double b[4];
            if (op == 4) {
                const float4 w = *reinterpret_cast<const float4*>(W + ge);
                b[0] = w.x; b[1] = w.y; b[2] = w.z; b[3] = w.w;
            } else {
                const double2 a = *reinterpret_cast<const double2*>(X + le);
                const double2 c = *reinterpret_cast<const double2*>(X + le + 2);
                b[0] = a.x; b[1] = a.y; b[2] = c.x; b[3] = c.y;
            }
            const float d[4] = {d4.x, d4.y, d4.z, d4.w};
            double x[4];
            float mc = 0.0f;
#pragma unroll
            for (int c = 0; c < 4; ++c) {
                x[c] = b[c] + (double)d[c];
                mc = fmaxf(mc, (float)(fabs((double)d[c]) / (1.0 + fabs(x[c]))));
            }
            *reinterpret_cast<double2*>(X + le) = make_double2(x[0], x[1]);
            *reinterpret_cast<double2*>(X + le + 2) = make_double2(x[2], x[3]);
            *reinterpret_cast<float4*>(W + ge) =
                make_float4((float)x[0], (float)x[1], (float)x[2], (float)x[3]);
            if (t) m1 = fmaxf(m1, mc);
            else m0 = fmaxf(m0, mc);
        } else {
            const double2 a = *reinterpret_cast<const double2*>(X + le);
            const double2 c = *reinterpret_cast<const double2*>(X + le + 2);
            *reinterpret_cast<float4*>(W + ge) =
                make_float4((float)a.x, (float)a.y, (float)c.x, (float)c.y);
        }
    }
    if (op == 2 || op == 4)  // non-negative floats order like their bit patterns
        for (int t = 0; t < 2; ++t) {
            float v = t ? m1 : m0;
            for (int o = 32; o > 0; o >>= 1) v = fmaxf(v, __shfl_xor(v, o));
            if (lane == 0 && v > 0.0f) atomicMax(dmax + t, __float_as_uint(v));
        }
}

// rows [r0, r0 + n) of a refinement op: the vector kernel when k % 4 == 0
void refine_rows(hipStream_t s, int op, int64_t r0, int64_t n, int32_t k, float* W, double* X,
                 const double* R, float* Rf, const float* D, const int64_t* off, int wood,
                 unsigned* dmax) {
    if (n <= 0) return;
    if ((k & 3) == 0 && k <= 256) {
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 3) / 4, 16384));
        wrmf_refine_rows_vec_kernel<<<grid, 256, 0, s>>>(op, r0, n, k, W, X, R, Rf, D, off, wood,
                                                         dmax);
    } else {
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(n, 16384));
        wrmf_refine_rows_kernel<<<grid, 256, 0, s>>>(op, r0, n, k, W, X, R, Rf, D, off, wood,
                                                     dmax);
    }
}

constexpr int kHeavy = 8192;   // rows with more entries take the split Gram
constexpr int kWood = 128;     // rows with at most this many entries take the Woodbury solve
constexpr int kSeg = 8192;     // entries per split-Gram segment
constexpr int64_t kGramBatchBytes = (int64_t)1 << 30;

}  // namespace

namespace mml {

void wrmf_tile_plan(const std::vector<int64_t>& deg, hipStream_t st, WrmfTilePlan& p, int64_t r0,
                    int64_t r1, bool woodbury, int32_t pipe) {
    const int32_t n = (int32_t)deg.size();
    p.woodbury = woodbury;
    // light rows by degree, descending (longest first: the work queue then ends on short rows)
    std::vector<int32_t> light, heavy;
    std::vector<int64_t> begin(n + 1, 0);
    for (int32_t r = 0; r < n; ++r) begin[r + 1] = begin[r] + deg[r];
    std::vector<int64_t> bucket(kHeavy + 2, 0);
    std::vector<int32_t> wood[4];
    auto is_wood = [&](int32_t r) { return woodbury && deg[r] >= 1 && deg[r] <= kWood; };
    for (int32_t r = (int32_t)r0; r < (int32_t)r1; ++r)
        if (is_wood(r)) wood[(deg[r] - 1) / 32].push_back(r);
        else if (deg[r] <= kHeavy) ++bucket[kHeavy - deg[r]];
        else heavy.push_back(r);
    int64_t acc = 0;
    for (auto& b : bucket) {
        const int64_t c = b;
        b = acc;
        acc += c;
    }
    light.resize(acc);
    for (int32_t r = (int32_t)r0; r < (int32_t)r1; ++r)
        if (!is_wood(r) && deg[r] <= kHeavy) light[bucket[kHeavy - deg[r]]++] = r;
    // the pipeline's row ranges (wrmf_tile_solve): only without Woodbury rows, whose solve comes
    // after the light rows' and whose W every range's residual would need
    size_t n_wood_rows = 0;
    for (auto& w : wood) n_wood_rows += w.size();
    // the default: pipe_batches() ranges, fewer where the half has fewer than 4,096 light rows per
    // range (and none below 4 such ranges, as before round 6's 12)
    int32_t want = pipe > 0 ? std::min(16, pipe) : pipe_batches();
    if (pipe <= 0 && want > 4) {
        const int64_t fit = (int64_t)light.size() / 4096;
        want = fit >= 4 ? (int32_t)std::min<int64_t>(want, fit) : want;
    }
    p.nbatch = 1;
    p.b_row.assign({0, r1 - r0});
    if (want > 1 && n_wood_rows == 0 && (int64_t)light.size() >= (int64_t)want * 4096) {
        // ranges of equal light work (Gram entries + a factorisation's worth per row), the light
        // list range-major and degree-descending within a range (each range's work queue still
        // ends on short rows)
        int64_t total = 0;
        for (int32_t r : light) total += deg[r] + 256;
        std::vector<int32_t> cut(want + 1, (int32_t)r1);
        cut[0] = (int32_t)r0;
        int64_t run = 0;
        int b = 1;
        std::vector<char> is_light(r1 - r0, 0);
        for (int32_t r : light) is_light[r - r0] = 1;
        for (int32_t r = (int32_t)r0; r < (int32_t)r1 && b < want; ++r) {
            if (is_light[r - r0]) run += deg[r] + 256;
            if (run * want >= total * b) cut[b++] = r + 1;
        }
        std::vector<int32_t> by(light.size());
        p.b_light.assign(want + 1, 0);
        p.b_row.assign(want + 1, 0);
        size_t at = 0;
        for (int x = 0; x < want; ++x) {
            p.b_row[x] = cut[x] - r0;
            p.b_light[x] = (int32_t)at;
            for (int32_t r : light)  // light is degree-descending: the range's rows in that order
                if (r >= cut[x] && r < cut[x + 1]) by[at++] = r;
        }
        p.b_row[want] = r1 - r0;
        p.b_light[want] = (int32_t)at;
        light.swap(by);
        p.nbatch = want;
    }
    if (p.nbatch == 1) p.b_light.assign({0, (int32_t)light.size()});
    for (int g = 0; g < 4; ++g) {
        p.n_wood[g] = (int32_t)wood[g].size();
        p.wood[g].alloc(std::max<size_t>(1, wood[g].size()));
        if (!wood[g].empty())
            MML_HIP(hipMemcpyAsync(p.wood[g].get(), wood[g].data(),
                                   sizeof(int32_t) * wood[g].size(), hipMemcpyHostToDevice, st));
    }
    std::sort(heavy.begin(), heavy.end(), [&](int32_t a, int32_t b) { return deg[a] > deg[b]; });
    std::vector<Seg> segs;
    p.seg_first.assign(heavy.size() + 1, 0);
    for (size_t x = 0; x < heavy.size(); ++x) {
        p.seg_first[x] = (int64_t)segs.size();
        const int64_t b = begin[heavy[x]], e = begin[heavy[x] + 1];
        for (int64_t s = b; s < e; s += kSeg)
            segs.push_back(Seg{(int32_t)x, 0, s, std::min(e, s + kSeg)});
    }
    p.seg_first[heavy.size()] = (int64_t)segs.size();
    p.n_light = (int32_t)light.size();
    p.light.alloc(std::max<size_t>(1, light.size()));
    if (!light.empty())
        MML_HIP(hipMemcpyAsync(p.light.get(), light.data(), sizeof(int32_t) * light.size(),
                               hipMemcpyHostToDevice, st));
    p.heavy = heavy;
    p.heavy_dev.alloc(std::max<size_t>(1, heavy.size()));
    if (!heavy.empty())
        MML_HIP(hipMemcpyAsync(p.heavy_dev.get(), heavy.data(), sizeof(int32_t) * heavy.size(),
                               hipMemcpyHostToDevice, st));
    p.segs.alloc(std::max<size_t>(1, segs.size() * sizeof(Seg)));
    if (!segs.empty())
        MML_HIP(hipMemcpyAsync(p.segs.get(), segs.data(), segs.size() * sizeof(Seg),
                               hipMemcpyHostToDevice, st));
    p.counter.alloc(1);
    // the refinement residual's entry segments over rows [r0, r1)
    std::vector<RSeg> rs;
    std::vector<RMulti> rm;
    int32_t slots = 0;
    p.b_seg.assign(p.nbatch + 1, 0);
    p.b_multi.assign(p.nbatch + 1, 0);
    int nb = 0;
    for (int64_t r = r0; r < r1; ++r) {
        while (nb < p.nbatch && r - r0 >= p.b_row[nb]) {  // the range starting at this row
            p.b_seg[nb] = (int64_t)rs.size();
            p.b_multi[nb] = (int64_t)rm.size();
            ++nb;
        }
        const int64_t b = begin[r], e = begin[r + 1];
        if (e == b) continue;
        const int32_t lr = (int32_t)(r - r0);
        if (e - b <= kRSeg) {
            rs.push_back(RSeg{lr, -1, b, e});
            continue;
        }
        const int32_t s0 = slots;
        for (int64_t x = b; x < e; x += kRSeg) rs.push_back(RSeg{lr, slots++, x, std::min(e, x + kRSeg)});
        rm.push_back(RMulti{lr, s0, slots - s0, 0});
    }
    for (; nb <= p.nbatch; ++nb) {
        p.b_seg[nb] = (int64_t)rs.size();
        p.b_multi[nb] = (int64_t)rm.size();
    }
    p.r0 = r0;
    p.r1 = r1;
    p.n_rsegs = (int64_t)rs.size();
    p.n_rmulti = (int64_t)rm.size();
    p.n_rslots = slots;
    p.rsegs.alloc(std::max<size_t>(1, rs.size() * sizeof(RSeg)));
    if (!rs.empty())
        MML_HIP(hipMemcpyAsync(p.rsegs.get(), rs.data(), rs.size() * sizeof(RSeg),
                               hipMemcpyHostToDevice, st));
    p.rmulti.alloc(std::max<size_t>(1, rm.size() * sizeof(RMulti)));
    if (!rm.empty())
        MML_HIP(hipMemcpyAsync(p.rmulti.get(), rm.data(), rm.size() * sizeof(RMulti),
                               hipMemcpyHostToDevice, st));
    MML_HIP(hipStreamSynchronize(st));
}

hipStream_t wrmf_plan_side(WrmfTilePlan& p, hipStream_t st) {
    int dev_cur = -1, dev_st = -1;
    MML_HIP(hipGetDevice(&dev_cur));
    MML_HIP(hipStreamGetDevice(st, &dev_st));
    if (dev_cur != dev_st) return nullptr;
    if (!p.side) MML_HIP(hipStreamCreateWithFlags(&p.side, hipStreamNonBlocking));
    return p.side;
}

WrmfTilePlan::~WrmfTilePlan() {
    if (hh_start) (void)hipEventDestroy(hh_start);
    if (hh_done) (void)hipEventDestroy(hh_done);
    for (hipEvent_t e : ev) (void)hipEventDestroy(e);
    if (side) (void)hipStreamDestroy(side);
}

// the first refinement pass's residual over local rows [lr0, lr1) of a plan (its entry segments
// [sg0, sg1) and multi-segment rows [m0, m1), which the plan keeps in row order): R = -X (HH + reg I)
// with x = the fp32 W rows widened on load, + sum_i c_i h_i, then Rf = (float) R.
// part 1: the dense term (it sets R), then the data term added, then Rf.  The pipeline splits it:
// part 4 (the handle's stream, right after the range's solve): the dense term added to R = 0;
// part 2 (the side stream): the data term added, then Rf.  0 + t = t, so R is part 1's bit for bit
// (a -0 dense term becomes +0: the same correction and W).
static void first_residual(hipStream_t s, WrmfTilePlan& p, float* W, const float* H,
                           const int32_t* cols, const double* HH, int32_t k, double alpha,
                           double reg, int64_t lr0, int64_t lr1, int64_t sg0, int64_t sg1,
                           int64_t m0, int64_t m1, int grid_cap, int& launches, int part = 1) {
    const int64_t n = lr1 - lr0;
    if (n <= 0) return;
    const float* w0 = W + (p.r0 + lr0) * (int64_t)k;
    double* r = p.ws->r64.get() + lr0 * (int64_t)k;
    auto dense = [&](int add) {
        static const int64_t xg = exp_grid("MML_WRMF_XHH_GRID", 2048);
        const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((n + kXB - 1) / kXB, xg));
        wrmf_xhh_kernel<float><<<gx, 256, 0, s>>>(w0, HH, n, k, reg, r, add);
        ++launches;
    };
    if (part == 1) dense(0);
    if (part == 1 && p.after_dense) {
        p.after_dense(s);
        p.after_dense = nullptr;
    }
    if (part == 4) {
        dense(1);
        MML_HIP(hipGetLastError());
        return;
    }
    {
        if (sg1 > sg0) {
            const int gs = (int)std::min<int64_t>((sg1 - sg0 + 3) / 4, grid_cap);  // 4 waves
            const RSeg* sg = reinterpret_cast<const RSeg*>(p.rsegs.get()) + sg0;
            // segment rows are local to r0: X is W from row r0 on, R the whole half's r64
            (((k & 3) == 0) ? &wrmf_resid_seg_kernel<float, true>
                            : &wrmf_resid_seg_kernel<float, false>)<<<gs, 256, 0, s>>>(
                sg, sg1 - sg0, cols, H, k, W + p.r0 * (int64_t)k, alpha, p.ws->r64.get(),
                p.ws->rpartial.get());
            ++launches;
        }
        if (m1 > m0) {
            wrmf_resid_multi_kernel<<<(int)std::min<int64_t>(m1 - m0, 8192), 256, 0, s>>>(
                reinterpret_cast<const RMulti*>(p.rmulti.get()) + m0, m1 - m0, k,
                p.ws->rpartial.get(), p.ws->r64.get());
            ++launches;
        }
    }
    refine_rows(s, 1, p.r0 + lr0, n, k, W, nullptr, r, p.ws->rf.get(), nullptr, nullptr, 0,
                nullptr);
    ++launches;
    MML_HIP(hipGetLastError());
}

// a further pass runs while the last correction was larger than these (relative to 1 + |x|), per
// row type.  The error left after a pass is the correction times the pass's contraction.  Direct
// rows solve the correction on the kept fp32 factor: contraction 3e-6 .. 2e-5 measured (C5's
// largest item correction 1.1e-4 was followed by 3e-10), so 3e-4 leaves <= ~6e-9.  Woodbury rows
// solve it by the fp32 CG at launch_wood_cg's refinement tolerance: contraction up to 0.06 measured on the tests'
// ill-conditioned small sets (a 3.4e-5 correction left 9.4e-7), so 2e-6 leaves <= ~1.2e-7.  C5
// (users Woodbury, corrections ~1e-8; items direct, ~1e-4) stops after one pass.
constexpr float kRefineStopDirect = 3e-4f;
constexpr float kRefineStopWood = 2e-6f;

int32_t wrmf_tile_refine(hipStream_t st, WrmfTilePlan& p, float* W, const float* H,
                         int64_t h_rows, const int64_t* off, const int32_t* cols, const double* HH,
                         int32_t k, double alpha, double reg, int32_t passes, int& launches,
                         float* corrections, const mml_ctx* sync) {
    const int64_t n = p.r1 - p.r0, n_w = (int64_t)(p.r1);  // W rows addressed up to r1
    // row shards over several ranks take each "another pass?" decision together (the max over
    // the ranks of the last correction), so the sharded model is the one-rank model bit for bit
    const bool rccl = sync && sync->comm && sync->nranks > 1;
    const bool peers = sync && sync->peers && sync->peers->n > 1;
    if (passes <= 0 || (n <= 0 && !rccl && !peers)) return 0;
    if (!p.ws->dmax.get()) p.ws->dmax.alloc(2);
    auto largest = [&](float d[2]) {  // this pass's corrections, combined over the ranks
        unsigned bits[2] = {0, 0};
        if (rccl)
            MML_RCCL(ncclAllReduce(p.ws->dmax.get(), p.ws->dmax.get(), 2, ncclUint32, ncclMax,
                                   sync->comm, st));
        MML_HIP(hipMemcpyAsync(bits, p.ws->dmax.get(), sizeof(bits), hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        if (peers) sync->peers->max_u32(sync, bits, 2);
        std::memcpy(d, bits, sizeof(bits));
    };
    auto stop = [](const float d[2]) {
        return !(d[0] > kRefineStopDirect) && !(d[1] > kRefineStopWood);
    };
    if (n <= 0) {  // a rank without rows still joins every decision
        for (int32_t pass = 0; pass + 1 < passes; ++pass) {
            MML_HIP(hipMemsetAsync(p.ws->dmax.get(), 0, 2 * sizeof(unsigned), st));
            float d[2];
            largest(d);
            if (stop(d)) break;
        }
        return 0;
    }
    p.ws->x64.reserve((size_t)n * k);
    p.ws->r64.reserve((size_t)n * k);
    p.ws->rf.reserve((size_t)n_w * k);
    p.ws->df.reserve((size_t)n_w * k);
    p.ws->rpartial.reserve(std::max<int64_t>(1, p.n_rslots) * (size_t)k);
    auto rows = [&](int op) {
        refine_rows(st, op, p.r0, n, k, W, p.ws->x64.get(), p.ws->r64.get(), p.ws->rf.get(),
                    p.ws->df.get(), off, p.woodbury ? 1 : 0, p.ws->dmax.get());
        ++launches;
    };
    // the first pass reads x as the fp32 W rows (widened on load, exactly) instead of a widened
    // copy, and every pass's x += d also writes W = (float) x: no X = W pass before the first
    // residual, no W = X pass after the last (C5: ~7 ms per iteration of row traffic)
    int32_t done = 0;
    p.screen_left = 0;
    for (int32_t pass = 0; pass < passes; ++pass) {
        // R = -X (HH + reg I) on the fp64 matrix cores, then + sum_i c_i h_i per row, R -> Rf
        if (pass == 0 && p.residual_ready) {
            // computed range by range under the main solve (wrmf_tile_solve's pipeline)
        } else if (pass == 0) {
            static const int rg = (int)exp_grid("MML_WRMF_RESID_GRID", 8192);
            first_residual(st, p, W, H, cols, HH, k, alpha, reg, 0, n, 0, p.n_rsegs, 0,
                           p.n_rmulti, rg, launches);
        } else {
            const int gx = (int)std::max<int64_t>(1, std::min<int64_t>((n + kXB - 1) / kXB, 2048));
            wrmf_xhh_kernel<double><<<gx, 256, 0, st>>>(p.ws->x64.get(), HH, n, k, reg,
                                                        p.ws->r64.get(), 0);
            ++launches;
            if (p.n_rsegs > 0) {
                const int gs = (int)std::min<int64_t>((p.n_rsegs + 3) / 4, 8192);  // 4 waves
                const RSeg* sg = reinterpret_cast<const RSeg*>(p.rsegs.get());
                (((k & 3) == 0) ? &wrmf_resid_seg_kernel<double, true>
                                : &wrmf_resid_seg_kernel<double, false>)<<<gs, 256, 0, st>>>(
                    sg, p.n_rsegs, cols, H, k, p.ws->x64.get(), alpha, p.ws->r64.get(),
                    p.ws->rpartial.get());
            }
            if (p.n_rmulti > 0)
                wrmf_resid_multi_kernel<<<(int)std::min<int64_t>(p.n_rmulti, 8192), 256, 0, st>>>(
                    reinterpret_cast<const RMulti*>(p.rmulti.get()), p.n_rmulti, k,
                    p.ws->rpartial.get(), p.ws->r64.get());
            MML_HIP(hipGetLastError());
            rows(1);
        }
        p.residual_ready = false;
        // D = A^{-1} R on the fp32 solver (rows outside [r0, r1) are not read)
        wrmf_tile_solve(st, p, p.ws->df.get(), H, h_rows, off, cols, HH, k, alpha, reg, launches,
                        p.ws->rf.get());
        MML_HIP(hipMemsetAsync(p.ws->dmax.get(), 0, 2 * sizeof(unsigned), st));
        if (p.pre_update_wait) {
            MML_HIP(hipStreamWaitEvent(st, p.pre_update_wait, 0));
            p.pre_update_wait = nullptr;
        }
        rows(pass == 0 ? 4 : 2);
        launches += 3;
        ++done;
        if (pass + 1 < passes) {  // another pass only while the correction was large
            float d[2];
            largest(d);
            if (corrections && pass < 4) corrections[pass] = std::max(d[0], d[1]);
            if (stop(d)) break;
        }
    }
    MML_HIP(hipGetLastError());
    return done;
}

// L^{-1} (lower) of B = HH + reg I by Cholesky in fp64 on the host (k <= 256: ~10 M flops)
// a . b over n doubles with four independent partial sums (the host step sits between two
// half-step kernels with the GPU idle: the serial-add chain was most of its ~4 ms at k = 256)
static inline double dot4(const double* a, const double* b, int n) {
    double s0 = 0.0, s1 = 0.0, s2 = 0.0, s3 = 0.0;
    int m = 0;
    for (; m + 4 <= n; m += 4) {
        s0 += a[m] * b[m];
        s1 += a[m + 1] * b[m + 1];
        s2 += a[m + 2] * b[m + 2];
        s3 += a[m + 3] * b[m + 3];
    }
    for (; m < n; ++m) s0 += a[m] * b[m];
    return (s0 + s1) + (s2 + s3);
}

static void chol_inverse(const std::vector<double>& HH, int k, double reg, std::vector<double>& Li) {
    std::vector<double> L(HH);
    for (int i = 0; i < k; ++i) L[(size_t)i * k + i] += reg;
    for (int j = 0; j < k; ++j) {
        const double* Lj = &L[(size_t)j * k];
        double d = L[(size_t)j * k + j] - dot4(Lj, Lj, j);
        MML_REQUIRE(d > 0.0, "HH + reg I is not positive definite");
        d = std::sqrt(d);
        L[(size_t)j * k + j] = d;
        for (int i = j + 1; i < k; ++i) {
            const double* Lr = &L[(size_t)i * k];
            L[(size_t)i * k + j] = (L[(size_t)i * k + j] - dot4(Lr, Lj, j)) / d;
        }
    }
    // L^{-1} row by row: row i = (e_i - sum_{m < i} L[i][m] row m) / L[i][i], contiguous axpys
    Li.assign((size_t)k * k, 0.0);
    for (int i = 0; i < k; ++i) {
        double* ri = &Li[(size_t)i * k];
        ri[i] = 1.0;
        for (int m = 0; m < i; ++m) {
            const double c = L[(size_t)i * k + m];
            const double* rm = &Li[(size_t)m * k];
            for (int x = 0; x <= m; ++x) ri[x] -= c * rm[x];
        }
        const double inv = 1.0 / L[(size_t)i * k + i];
        for (int x = 0; x <= i; ++x) ri[x] *= inv;
    }
}

// |Li|_2 of a lower-triangular k x k matrix: sqrt of the largest eigenvalue of Li^T Li by power
// iteration (60 steps from a fixed start), times 1.25.  Power iteration approaches the eigenvalue
// from below; the margin covers what 60 steps leave when the top eigenvalues are close.
static double spectral_norm_lower(const std::vector<double>& Li, int k) {
    std::vector<double> v(k), u(k);
    for (int i = 0; i < k; ++i) v[i] = 1.0 + 0.001 * (i % 7);
    double lam = 0.0;
    for (int it = 0; it < 60; ++it) {
        double nv = 0.0;
        for (double x : v) nv += x * x;
        nv = std::sqrt(nv);
        for (double& x : v) x /= nv;
        for (int i = 0; i < k; ++i) u[i] = dot4(&Li[(size_t)i * k], v.data(), i + 1);  // u = Li v
        double uu = 0.0;
        for (double x : u) uu += x * x;
        lam = uu;  // v^T Li^T Li v, |v| = 1
        std::fill(v.begin(), v.end(), 0.0);  // v = Li^T u
        for (int i = 0; i < k; ++i)
            for (int j = 0; j <= i; ++j) v[j] += Li[(size_t)i * k + j] * u[i];
    }
    return 1.25 * std::sqrt(lam);
}

// MML_WRMF_PLANES=0 (experiments builds): the direct rows' Gram gathers fp32 rows and splits them
// in the kernel (gram_accumulate_x3g) instead of reading planes split once per half-step
bool use_planes() {
    static const bool v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_PLANES");
        return !(e && std::string(e) == "0");
    }();
    return v;
}

void wrmf_tile_solve(hipStream_t st, WrmfTilePlan& p, float* W, const float* H, int64_t h_rows,
                     const int64_t* off, const int32_t* cols, const double* HH, int32_t k,
                     double alpha, double reg, int& launches, const float* rhs) {
    MML_REQUIRE(k > 128 && k <= 256, "tile solver covers 128 < k <= 256");
    const int nt = (k + 31) >> 5, nr = nt + 1;
    const int ntile = nt * nr - nt * (nt - 1) / 2;
    // the HH tiles (HHt); when HH is still being computed on the side stream (half_step), after
    // the first split Gram batch, which does not read them
    auto hh_tiles = [&]() {
        if (p.hh_pending) {
            MML_HIP(hipStreamWaitEvent(st, p.hh_done, 0));
            p.hh_pending = false;
        }
        p.hht.alloc((size_t)kTiles * 1024);
        wrmf_tile_hh_kernel<<<(ntile * 1024 + 255) / 256, 256, 0, st>>>(HH, k, reg, p.hht.get());
        ++launches;
    };
    if (!rhs && !p.hh_pending) hh_tiles();  // a refinement pass reuses the half-step's tables
    const int grid_cap = 256 * 2;  // 256 CUs; a second resident workgroup where registers allow
    const int64_t nh = (int64_t)p.heavy.size();
    const size_t tile_floats = (size_t)kTiles * 1024;
    if (rhs && p.keep_factor) {  // refinement: the kept factors, no Gram, no factorisation
        // one wave per row (default) or the 8-wave workgroup per row (MML_WRMF_RESOLVE=wg, A/B)
        static const bool wg = [] {
            const char* e = MML_EXPERIMENT_ENV("MML_WRMF_RESOLVE");
            return e && std::string(e) == "wg";
        }();
        auto resolve = [&](const int32_t* list, int64_t n, const float* Fl) {
            if (n <= 0) return;
            if (wg) {
                MML_HIP(hipMemsetAsync(p.counter.get(), 0, sizeof(int32_t), st));
                wrmf_tile_resolve_kernel<<<(int)std::min<int64_t>(n, grid_cap), kThreads, 0, st>>>(
                    list, (int32_t)n, p.counter.get(), off, Fl, rhs, k, W);
            } else {
                const int64_t blocks = std::min<int64_t>((n + kRvWaves - 1) / kRvWaves, rv_grid());
                wrmf_tile_resolve_wave_kernel<<<(int)blocks, 64 * kRvWaves, 0, st>>>(
                    list, (int32_t)n, off, Fl, rhs, k, W, 0);
            }
            ++launches;
        };
        resolve(p.heavy_dev.get(), nh, p.ws->factor.get() + (size_t)p.n_light * tile_floats);
        if (p.light_corr_ready && W == p.ws->df.get() && rhs == p.ws->rf.get())
            p.light_corr_ready = false;  // the pipeline already solved them (wrmf_tile_solve)
        else
            resolve(p.light.get(), p.n_light, p.ws->factor.get());
        MML_HIP(hipGetLastError());
    } else {
        // the factors of the direct rows, kept when refinement passes follow (fp64 mode)
        float* F = nullptr;
        if (p.keep_factor && !rhs) {
            // 176 KB per direct row at k = 256: keep them only if they fit the free HBM with a
            // margin (the workspace's current block counts as free: it is reallocated here)
            const size_t need = std::max<size_t>(1, (size_t)(p.n_light + nh) * tile_floats);
            size_t free_b = 0, total_b = 0;
            MML_HIP(hipMemGetInfo(&free_b, &total_b));
            const size_t have = free_b + p.ws->factor.count * sizeof(float);
            if (need <= p.ws->factor.count) {
                F = p.ws->factor.get();  // the shared workspace already holds enough
            } else if (need * sizeof(float) + total_b / 16 > have) {
                p.keep_factor = false;
                p.ws->factor.reset();
            } else {
                p.ws->factor.alloc(need);
                F = p.ws->factor.get();
            }
        }
        // the Gram vectors as bf16 planes, split once per half-step (the refinement's refactoring
        // passes reuse them), if they fit the free HBM with a margin; else the fp32 gathers
        const uint16_t* P = nullptr;
        const int64_t ps = (h_rows + 1) * kPW;
        if (nh + p.n_light > 0 && use_planes()) {
            if (!rhs) {
                p.ws->planes_of = nullptr;
                const size_t need = (size_t)3 * ps;
                size_t free_b = 0, total_b = 0;
                MML_HIP(hipMemGetInfo(&free_b, &total_b));
                const size_t have = free_b + p.ws->planes.count * sizeof(uint16_t);
                if (need <= p.ws->planes.count || need * sizeof(uint16_t) + total_b / 16 <= have) {
                    if (need > p.ws->planes.count) p.ws->planes.alloc(need);
                    const int blocks = (int)std::min<int64_t>((ps + 255) / 256, 256 * 64);
                    wrmf_split_planes_kernel<<<blocks, 256, 0, st>>>(H, h_rows, k,
                                                                     p.ws->planes.get());
                    MML_HIP(hipGetLastError());
                    ++launches;
                    p.ws->planes_of = H;
                }
            }
            if (p.ws->planes_of == H) P = p.ws->planes.get();
        }
        // heavy rows: batches whose fp64 Grams fit the workspace
        const int64_t per_row = (int64_t)kTiles * 1024 * sizeof(double);
        const int64_t batch_rows = std::max<int64_t>(1, kGramBatchBytes / per_row);
        for (int64_t h0 = 0; h0 < nh; h0 += batch_rows) {
            const int64_t h1 = std::min(nh, h0 + batch_rows);
            const int64_t s0 = p.seg_first[h0], s1 = p.seg_first[h1];
            p.gram.alloc((size_t)std::min(nh, batch_rows) * kTiles * 1024);
            MML_HIP(hipMemsetAsync(p.gram.get(), 0, (size_t)(h1 - h0) * per_row, st));
            static const int64_t gram_grid = [] {  // MML_WRMF_GRAM_GRID (experiments): A/B
                const char* e = MML_EXPERIMENT_ENV("MML_WRMF_GRAM_GRID");
                return e ? std::max<int64_t>(256, std::atoll(e)) : (int64_t)256 * 2;
            }();
            const int gg = (int)std::min<int64_t>(s1 - s0, gram_grid);
            auto gk = P ? &wrmf_tile_gram_kernel<true> : &wrmf_tile_gram_kernel<false>;
            gk<<<gg, kThreads, 0, st>>>(
                reinterpret_cast<const Seg*>(p.segs.get()) + s0, (int32_t)(s1 - s0), (int32_t)h0,
                cols, H, k, p.gram.get(), P, ps, (int32_t)h_rows);
            if (!rhs && p.hh_pending) hh_tiles();
            MML_HIP(hipMemsetAsync(p.counter.get(), 0, sizeof(int32_t), st));
            const int gs = (int)std::min<int64_t>(h1 - h0, grid_cap);
            wrmf_tile_solve_kernel<0><<<gs, kThreads, 0, st>>>(
                p.heavy_dev.get() + h0, (int32_t)(h1 - h0), p.counter.get(), off, cols, W, H,
                p.hht.get(), p.gram.get(), k, k, (float)alpha, nullptr, debug_mask(), rhs,
                F ? F + (size_t)(p.n_light + h0) * tile_floats : nullptr);
            MML_HIP(hipGetLastError());
            launches += 2;
        }
        if (!rhs && p.hh_pending) hh_tiles();  // no hot rows: HH before the light rows
        auto sk = P ? &wrmf_tile_solve_kernel<0, true> : &wrmf_tile_solve_kernel<0, false>;
        auto solve_light = [&](int64_t l0, int64_t l1) {  // light-list slice [l0, l1)
            if (l1 <= l0) return;
            MML_HIP(hipMemsetAsync(p.counter.get(), 0, sizeof(int32_t), st));
            const int gs = (int)std::min<int64_t>(l1 - l0, grid_cap);
            sk<<<gs, kThreads, 0, st>>>(
                p.light.get() + l0, (int32_t)(l1 - l0), p.counter.get(), off, cols, W, H,
                p.hht.get(), nullptr, k, k, (float)alpha, nullptr, debug_mask(), rhs,
                F ? F + (size_t)l0 * tile_floats : nullptr, P, ps, (int32_t)h_rows);
            MML_HIP(hipGetLastError());
            ++launches;
        };
        // the deferred backward substitutions: W rows hold y, the kept tiles L
        auto back = [&](const int32_t* list, int64_t n, const float* Fl) {
            if (n <= 0) return;
            const int64_t blocks = std::min<int64_t>((n + kRvWaves - 1) / kRvWaves, rv_grid());
            wrmf_tile_resolve_wave_kernel<<<(int)blocks, 64 * kRvWaves, 0, st>>>(
                list, (int32_t)n, off, Fl, W, k, W, 1);
            ++launches;
        };
        // the pipeline (fp64 mode, no Woodbury rows): range b's first-pass residual on the side
        // stream under range b + 1's solve; the side stream must belong to this stream's device
        bool pipe = F && p.nbatch > 1 && p.n_wood[0] + p.n_wood[1] + p.n_wood[2] + p.n_wood[3] == 0;
        if (pipe) {
            int dev_cur = -1, dev_st = -1;
            MML_HIP(hipGetDevice(&dev_cur));
            MML_HIP(hipStreamGetDevice(st, &dev_st));
            pipe = dev_cur == dev_st;
        }
        if (pipe) {
            // (the side stream at the least or greatest priority, or the handle's stream at the
            // greatest, measured the same: 741.8 / 744.0 / 742.2 ms against 741.3 / 743.9,
            // profiles/r5u/)
            if (!p.side) MML_HIP(hipStreamCreateWithFlags(&p.side, hipStreamNonBlocking));
            while ((int)p.ev.size() < p.nbatch + 1) {
                hipEvent_t e;
                MML_HIP(hipEventCreateWithFlags(&e, hipEventDisableTiming));
                p.ev.push_back(e);
            }
            const int64_t n = p.r1 - p.r0;
            p.ws->r64.reserve((size_t)n * k);  // the sizes wrmf_tile_refine reserves
            p.ws->rf.reserve((size_t)p.r1 * k);
            p.ws->rpartial.reserve(std::max<int64_t>(1, p.n_rslots) * (size_t)k);
            p.ws->df.reserve((size_t)p.r1 * k);
            MML_HIP(hipMemsetAsync(p.ws->r64.get(), 0, sizeof(double) * (size_t)n * k, st));
            back(p.heavy_dev.get(), nh, F + (size_t)p.n_light * tile_floats);
            for (int b = 0; b < p.nbatch; ++b) {
                const int64_t l0 = p.b_light[b], l1 = p.b_light[b + 1];
                solve_light(l0, l1);
                back(p.light.get() + l0, l1 - l0, F + (size_t)l0 * tile_floats);
                // the dense term on this stream (the fp64 MFMA kernel takes whole SIMDs), between
                // the ranges' solves
                first_residual(st, p, W, H, cols, HH, k, alpha, reg, p.b_row[b], p.b_row[b + 1],
                               0, 0, 0, 0, 8192, launches, 4);
                MML_HIP(hipEventRecord(p.ev[b], st));
                MML_HIP(hipStreamWaitEvent(p.side, p.ev[b], 0));
                // the data term, Rf, and the range's light rows' corrections on their kept
                // factors, beside range b + 1's solve
                first_residual(p.side, p, W, H, cols, HH, k, alpha, reg, p.b_row[b],
                               p.b_row[b + 1], p.b_seg[b], p.b_seg[b + 1], p.b_multi[b],
                               p.b_multi[b + 1], pipe_grid(), launches, 2);
                if (l1 > l0) {
                    const int64_t blocks =
                        std::min<int64_t>((l1 - l0 + kRvWaves - 1) / kRvWaves, rv_grid());
                    wrmf_tile_resolve_wave_kernel<<<(int)blocks, 64 * kRvWaves, 0, p.side>>>(
                        p.light.get() + l0, (int32_t)(l1 - l0), off, F + (size_t)l0 * tile_floats,
                        p.ws->rf.get(), k, p.ws->df.get(), 0);
                    ++launches;
                }
            }
            MML_HIP(hipEventRecord(p.ev[p.nbatch], p.side));
            MML_HIP(hipStreamWaitEvent(st, p.ev[p.nbatch], 0));
            p.residual_ready = true;
            p.light_corr_ready = true;
        } else {
            solve_light(0, p.n_light);
            if (F) {
                back(p.heavy_dev.get(), nh, F + (size_t)p.n_light * tile_floats);
                back(p.light.get(), p.n_light, F);
            }
        }
        MML_HIP(hipGetLastError());
    }
    int64_t nw = 0, nw_max = 0;
    for (int g = 0; g < 4; ++g) {
        nw += p.n_wood[g];
        nw_max = std::max<int64_t>(nw_max, p.n_wood[g]);
    }
    if (nw == 0) return;
    if (rhs) {  // d = L^{-T} (s - Q_S^T w), s = L^{-1} r, C w = Q_S s
        p.sbuf.alloc((size_t)nw_max * k);
        for (int g = 0; g < 4; ++g) {
            if (!p.n_wood[g]) continue;
            rows_matmul(st, rhs, p.wood[g].get(), p.n_wood[g], p.linvt.get(), p.linvt_x3.get(), k,
                        1.0f, p.sbuf.get(), nullptr);
            if (wood_cg()) {
                // the rows whose correction is 0 by the bound are settled here; the kernels and
                // the row GEMM run on the rest (none for C5's users)
                p.crow.reserve(nw_max);
                p.cpos.reserve(nw_max);
                p.ccount.reserve(1);
                MML_HIP(hipMemsetAsync(p.ccount.get(), 0, sizeof(int32_t), st));
                const double lim = (double)wood_skip2(p.linv_norm) * (1.0 - 1e-4);
                const int sg = (int)std::min<int64_t>((p.n_wood[g] + 3) / 4, 4096);
                wrmf_wood_screen_kernel<<<sg, 256, 0, st>>>(p.wood[g].get(), p.n_wood[g],
                                                            p.sbuf.get(), k, lim, W, p.crow.get(),
                                                            p.cpos.get(), p.ccount.get());
                int32_t m = 0;
                MML_HIP(hipMemcpyAsync(&m, p.ccount.get(), sizeof(int32_t), hipMemcpyDeviceToHost,
                                       st));
                MML_HIP(hipStreamSynchronize(st));
                p.screen_left += m;
                if (m > 0) {
                    launch_wood_cg(st, g, p.crow.get(), m, off, cols, p.qbuf.get(), k,
                                   (float)alpha, p.tbuf.get(), p.sbuf.get(), p.linv_norm, false,
                                   p.cpos.get());
                    rows_matmul(st, p.tbuf.get(), nullptr, m, p.linv.get(), p.linv_x3.get(), k,
                                1.0f, W, p.crow.get());
                }
                MML_HIP(hipGetLastError());
                launches += 4;
                continue;
            } else {
                p.screen_left += p.n_wood[g];  // no screen: the rows' corrections are unknown
                auto* L = g == 0 ? &launch_wood<1> : g == 1 ? &launch_wood<2>
                          : g == 2 ? &launch_wood<3> : &launch_wood<4>;
                L(st, p.wood[g].get(), p.n_wood[g], p.counter.get(), off, cols, p.qbuf.get(), k,
                  (float)alpha, p.tbuf.get(), p.sbuf.get());
            }
            rows_matmul(st, p.tbuf.get(), nullptr, p.n_wood[g], p.linv.get(), p.linv_x3.get(), k,
                        1.0f, W, p.wood[g].get());
            MML_HIP(hipGetLastError());
            launches += 3;
        }
        return;
    }
    // Woodbury rows: B = HH + reg I = L L^T (host fp64), Q = H L^{-T}, per-row C v = 1 and
    // t = Q_S^T v on the tiles, then W rows = ((1 + alpha) / alpha) t L^{-1}
    std::vector<double> hh((size_t)k * k), li;
    MML_HIP(hipMemcpyAsync(hh.data(), HH, sizeof(double) * hh.size(), hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    chol_inverse(hh, k, reg, li);
    p.linv_norm = spectral_norm_lower(li, k);
    std::vector<float> lf((size_t)k * k), ltf((size_t)k * k);
    for (int i = 0; i < k; ++i)
        for (int j = 0; j < k; ++j) {
            lf[(size_t)i * k + j] = (float)li[(size_t)i * k + j];
            ltf[(size_t)j * k + i] = (float)li[(size_t)i * k + j];
        }
    p.linv.alloc(lf.size());
    p.linvt.alloc(ltf.size());
    MML_HIP(hipMemcpyAsync(p.linv.get(), lf.data(), sizeof(float) * lf.size(),
                           hipMemcpyHostToDevice, st));
    MML_HIP(hipMemcpyAsync(p.linvt.get(), ltf.data(), sizeof(float) * ltf.size(),
                           hipMemcpyHostToDevice, st));
    const int kpad = (k + 15) & ~15;
    p.linv_x3.alloc((size_t)3 * k * kpad);
    p.linvt_x3.alloc((size_t)3 * k * kpad);
    const int gsp = (int)std::min<int64_t>(((int64_t)k * kpad + 255) / 256, 1024);
    wrmf_split_mt_kernel<<<gsp, 256, 0, st>>>(p.linv.get(), k, kpad, p.linv_x3.get());
    wrmf_split_mt_kernel<<<gsp, 256, 0, st>>>(p.linvt.get(), k, kpad, p.linvt_x3.get());
    launches += 2;
    p.qbuf.alloc((size_t)h_rows * k);
    rows_matmul(st, H, nullptr, h_rows, p.linvt.get(), p.linvt_x3.get(), k, 1.0f, p.qbuf.get(),
                nullptr);
    p.tbuf.alloc((size_t)nw_max * k);
    const float cw = (float)((1.0 + alpha) / alpha);
    launches += 1;
    for (int g = 0; g < 4; ++g) {
        if (!p.n_wood[g]) continue;
        if (debug_mask() & 16) {  // the one-row-per-workgroup MODE 1 kernel (A/B)
            MML_HIP(hipMemsetAsync(p.counter.get(), 0, sizeof(int32_t), st));
            const int gs = (int)std::min<int64_t>(p.n_wood[g], grid_cap);
            wrmf_tile_solve_kernel<1><<<gs, kThreads, 0, st>>>(
                p.wood[g].get(), p.n_wood[g], p.counter.get(), off, cols, W, p.qbuf.get(),
                nullptr, nullptr, k, 32 * (g + 1), (float)alpha, p.tbuf.get(), debug_mask(),
                nullptr, nullptr);
        } else if (wood_cg()) {
            launch_wood_cg(st, g, p.wood[g].get(), p.n_wood[g], off, cols, p.qbuf.get(), k,
                           (float)alpha, p.tbuf.get(), nullptr, 0.0, p.refined);
        } else {
            auto* L = g == 0 ? &launch_wood<1> : g == 1 ? &launch_wood<2>
                      : g == 2 ? &launch_wood<3> : &launch_wood<4>;
            L(st, p.wood[g].get(), p.n_wood[g], p.counter.get(), off, cols, p.qbuf.get(), k,
              (float)alpha, p.tbuf.get(), nullptr);
        }
        rows_matmul(st, p.tbuf.get(), nullptr, p.n_wood[g], p.linv.get(), p.linv_x3.get(), k, cw,
                    W, p.wood[g].get());
        MML_HIP(hipGetLastError());
        launches += 2;
    }
}

}  // namespace mml
