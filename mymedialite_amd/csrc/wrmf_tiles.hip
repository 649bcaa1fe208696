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
#include <cstdlib>
#include <vector>

#include "mml_internal.h"

#pragma clang fp contract(fast)

namespace {

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
constexpr int kDS = 33;                                  // diagonal-tile / reduction row stride
constexpr int kTS = 40;                                  // T_J^T row stride
constexpr int kDG = 36;                                  // diagonal-tile row stride

__device__ __forceinline__ int rho(int g, int h) { return (g & 3) + 8 * (g >> 2) + 4 * h; }

// threadIdx.x made opaque at the call site: lane-derived constants (row selectors, LDS offsets)
// are then recomputed in each phase instead of being hoisted out of the row loop and spilled
__device__ __forceinline__ int opaque_tid() {
    int t = threadIdx.x;
    asm volatile("" : "+v"(t));
    return t;
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
        float hs[2][kCH * kHSW];        // Gram: staged item vectors, double-buffered
        float pn[kNT][32][kPS];         // Cholesky: L_IJ of the current panel, row-major
        float red[kNT][32][kDS];        // backward: per-tile partial products
    } u;
    float dg[32][kDG];                  // diagonal tile (rows 16-B aligned)
    float tT[2][32][kTS];               // tT[c][m] = T_J[m][c], double-buffered (lookahead)
    float yv[kHSW];
    float wv[kHSW];
    float sv[32];
    float part[kNT][32];
    float park[kSlots][4][64][4];       // one wave's accumulators during a diagonal factorisation
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
__device__ __forceinline__ void gram_accumulate(Smem& sm, f32x16 (&acc)[kSlots], Tiles& tl,
                                                const int32_t* __restrict__ cols, int64_t b,
                                                int64_t e, const float* __restrict__ H, int k,
                                                int hsw) {
    static_assert(kCH * 32 == kThreads, "one staging thread group of 32 per vector");
    constexpr int kQ = 2;   // float4 per thread (k <= 256)
    constexpr int kS = 8;   // scalars per thread (k <= 256)
    const int t = opaque_tid(), lane = t & 63, q = lane & 31, h = lane >> 5;
    const int c = t >> 5, u = t & 31;
    const int kb = hsw - 32;
    const bool vec = (k & 3) == 0;
    float4 p4[kQ];
    float p1[kS];
    auto fetch = [&](int32_t item, bool live) {
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
    };
    auto stash = [&](float* buf, bool live) {
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
    };
    if (e <= b) return;
    // per-lane operand offsets of the owned tiles (unused slots read offset 0 with weight 0)
    int offJ[kSlots], offI[kSlots];
    float mJ[kSlots];
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        const bool ok = tl.I[s] >= 0;
        const int cj = 32 * tl.J[s] + q;
        offJ[s] = ok ? cj : 0;
        offI[s] = ok ? 32 * tl.I[s] + q : 0;
        mJ[s] = (ok && cj < k) ? 1.0f : 0.0f;
    }
    auto idx_at = [&](int64_t base) -> int32_t {
        return base + c < e ? cols[base + c] : 0;
    };
    int cur = 0;
    __syncthreads();  // the LDS union may still be read by the previous row's last phase
    int32_t i0 = idx_at(b);
    int32_t i1 = b + kCH < e ? idx_at(b + kCH) : 0;
    fetch(i0, b + c < e);
    stash(sm.u.hs[0], b + c < e);
    __syncthreads();
    for (int64_t base = b; base < e; base += kCH) {
        const int nrc = (int)min((int64_t)kCH, e - base);
        const int64_t nb = base + kCH;
        const bool more = nb < e;
        if (more) {
            fetch(i1, nb + c < e);                            // next chunk: in flight
            i1 = nb + kCH < e ? idx_at(nb + kCH) : 0;         // the index after it
        }
        const float* buf = sm.u.hs[cur];
        for (int cc = 0; cc < nrc; cc += 2) {
            const float* hr = buf + (cc + h) * kHSW;
#pragma unroll
            for (int s = 0; s < kSlots; ++s)  // straight line: unused slots multiply by 0
                acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(hr[offJ[s]] * mJ[s], hr[offI[s]],
                                                              acc[s], 0, 0, 0);
        }
        if (more) stash(sm.u.hs[cur ^ 1], nb + c < e);
        __syncthreads();
        cur ^= 1;
    }
}

// Split Gram of the heavy rows: one workgroup per (row, segment of <= kSeg entries), fp64 atomics
// into gram[(li * kTiles + tile) * 1024 + g * 64 + lane].
struct Seg {
    int32_t li, pad;
    int64_t b, e;
};

__global__ __launch_bounds__(kThreads, 2) void wrmf_tile_gram_kernel(
    const Seg* __restrict__ segs, int32_t nseg, int32_t li0, const int32_t* __restrict__ cols,
    const float* __restrict__ H, int32_t k, double* __restrict__ gram) {
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
        gram_accumulate(sm, acc, tl, cols, sg.b, sg.e, H, k, 32 * nr);
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

// One wave: T = L^{-1} for the diagonal tile the caller wrote to sm.dg (row-major):
// L = chol(tile) with row q of the tile in lane q (v_readlane broadcasts of the pivot column), then
// column q of T in lane q from the rows of L broadcast out of LDS.  Writes tT[c][m] = T[m][c].
__device__ __forceinline__ void diag_factor(Smem& sm, float (*tT)[kTS]) {
    const int lane = opaque_tid() & 63, q = lane & 31, h = lane >> 5;
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float x[32];
#pragma unroll
    for (int c = 0; c < 32; c += 4) {
        const float4 v = *reinterpret_cast<const float4*>(&sm.dg[q][c]);
        x[c] = v.x; x[c + 1] = v.y; x[c + 2] = v.z; x[c + 3] = v.w;
    }
#pragma unroll
    for (int c = 0; c < 32; ++c) {
        const float piv = lane_bcast(x[c], c);
        const float inv = __builtin_amdgcn_rsqf(piv);
        x[c] = (q == c) ? piv * inv : x[c] * inv;
#pragma unroll
        for (int c2 = c + 1; c2 < 32; ++c2) x[c2] -= x[c] * lane_bcast(x[c], c2);
    }
    __builtin_amdgcn_wave_barrier();
    if (h == 0)
#pragma unroll
        for (int c = 0; c < 32; c += 4)
            *reinterpret_cast<float4*>(&sm.dg[q][c]) = make_float4(x[c], x[c + 1], x[c + 2], x[c + 3]);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    float tc[32];
#pragma unroll
    for (int m = 0; m < 32; ++m) {
        float sacc = (m == q) ? 1.0f : 0.0f;
#pragma unroll
        for (int j4 = 0; j4 < m; j4 += 4) {
            const float4 l = *reinterpret_cast<const float4*>(&sm.dg[m][j4]);
            sacc -= l.x * tc[j4];
            if (j4 + 1 < m) sacc -= l.y * tc[j4 + 1];
            if (j4 + 2 < m) sacc -= l.z * tc[j4 + 2];
            if (j4 + 3 < m) sacc -= l.w * tc[j4 + 3];
        }
        tc[m] = sacc * __builtin_amdgcn_rcpf(sm.dg[m][m]);
    }
    if (h == 0)
#pragma unroll
        for (int m = 0; m < 32; ++m) tT[q][m] = tc[m];
}

// The calling wave parks its accumulators in LDS around diag_factor, so the factorisation's
// registers do not have to coexist with the tiles (which would spill).
__device__ __forceinline__ void factor_tile(Smem& sm, f32x16 (&acc)[kSlots], int slot,
                                            float (*tT)[kTS]) {
    const int lane = opaque_tid() & 63, q = lane & 31, h = lane >> 5;
#pragma unroll
    for (int s = 0; s < kSlots; ++s) {
        if (s == slot)
#pragma unroll
            for (int g = 0; g < 16; ++g) sm.dg[q][rho(g, h)] = acc[s][g];
#pragma unroll
        for (int g = 0; g < 16; g += 4)
            *reinterpret_cast<float4*>(&sm.park[s][g / 4][lane][0]) =
                make_float4(acc[s][g], acc[s][g + 1], acc[s][g + 2], acc[s][g + 3]);
    }
    diag_factor(sm, tT);
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
#pragma unroll
    for (int s = 0; s < kSlots; ++s)
#pragma unroll
        for (int g = 0; g < 16; g += 4) {
            const float4 v = *reinterpret_cast<const float4*>(&sm.park[s][g / 4][lane][0]);
            acc[s][g] = v.x; acc[s][g + 1] = v.y; acc[s][g + 2] = v.z; acc[s][g + 3] = v.w;
        }
}

__global__ __launch_bounds__(kThreads, 2) void wrmf_tile_solve_kernel(
    const int32_t* __restrict__ rows, int32_t n_list, int32_t* __restrict__ counter,
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols, float* __restrict__ W,
    const float* __restrict__ H, const float* __restrict__ HHt, const double* __restrict__ gram,
    int32_t k, float alpha, int32_t dbg) {
    __shared__ Smem sm;
    const int wave = threadIdx.x >> 6;
    const int nt = (k + 31) >> 5, nr = nt + 1;
    const int ntile = nt * nr - nt * (nt - 1) / 2;
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
            for (int f = t; f < k; f += kThreads) W[(int64_t)row * k + f] = 0.0f;
            continue;
        }
        f32x16 acc[kSlots];
#pragma unroll
        for (int s = 0; s < kSlots; ++s)
#pragma unroll
            for (int g = 0; g < 16; ++g) acc[s][g] = 0.0f;
        // ---- 1. Gram (+ b in row kb)
        if (gram) {
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] < 0) continue;
                const double* src = gram + ((int64_t)li * kTiles + s * kWaves + wave) * 1024 + lane;
#pragma unroll
                for (int g = 0; g < 16; ++g) acc[s][g] = (float)src[g * 64];
            }
        } else if (!(dbg & 8)) {
            gram_accumulate(sm, acc, tl, cols, rb, re, H, k, hsw);
        }
        // ---- 2. A' = HHt + alpha * S above row kb (HHt = HH + reg I, identity on the padding;
        //         S is 0 on the padding), (1 + alpha) * S on the b-row tile
#pragma unroll
        for (int s = 0; s < kSlots; ++s) {
            if (tl.I[s] < 0) continue;
            if (tl.I[s] < nt) {
                const float* hh = HHt + tile_id(tl.I[s], tl.J[s], nr) * 1024 + lane;
#pragma unroll
                for (int g = 0; g < 16; ++g) acc[s][g] = hh[g * 64] + alpha * acc[s][g];
            } else {
#pragma unroll
                for (int g = 0; g < 16; ++g) acc[s][g] *= 1.0f + alpha;
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
                if (!(dbg & 2))
#pragma unroll
                    for (int st = 0; st < 16; ++st)
                        nv = __builtin_amdgcn_mfma_f32_32x32x2f32(tT[rho(st, h)][q], acc[s][st], nv,
                                                                  0, 0, 0);
                acc[s] = nv;
                const int pi = tl.I[s] - J - 1;
#pragma unroll
                for (int g = 0; g < 16; ++g) sm.u.pn[pi][q][rho(g, h)] = nv[g];
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
                    if (s != own) continue;
                    const float* lr = sm.u.pn[0][q];
                    if (!(dbg & 2))
#pragma unroll
                        for (int st = 0; st < 16; ++st)
                            acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(
                                -lr[2 * st + h], lr[2 * st + h], acc[s], 0, 0, 0);
                }
                if (!(dbg & 1)) factor_tile(sm, acc, own, sm.tT[(J + 1) & 1]);
            }
#pragma unroll
            for (int s = 0; s < kSlots; ++s) {
                if (tl.I[s] < 0 || tl.J[s] <= J || (dbg & 2)) continue;
                if (s * kWaves + wave == tdn) continue;
                const float* lk = sm.u.pn[tl.J[s] - J - 1][q];
                const float* lr = sm.u.pn[tl.I[s] - J - 1][q];
#pragma unroll
                for (int st = 0; st < 16; ++st)
                    acc[s] = __builtin_amdgcn_mfma_f32_32x32x2f32(-lk[2 * st + h], lr[2 * st + h],
                                                                  acc[s], 0, 0, 0);
            }
            __syncthreads();
        }
        // ---- 4. backward substitution L^T w = y (padding entries come out 0)
        for (int J = nt - 1; J >= 0; --J) {
            if (dbg & 4) break;
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
        __syncthreads();
        for (int f = t; f < k; f += kThreads) W[(int64_t)row * k + f] = sm.wv[f];
    }
}

// MML_WRMF_DEBUG: phase-skip mask for timing experiments only (results are wrong when set):
// 1 diagonal factorisation, 2 panel MFMAs, 4 backward substitution, 8 Gram
int debug_mask() {
    static const int v = [] {
        const char* e = std::getenv("MML_WRMF_DEBUG");
        return e ? std::atoi(e) : 0;
    }();
    return v;
}

constexpr int kHeavy = 8192;   // rows with more entries take the split Gram
constexpr int kSeg = 8192;     // entries per split-Gram segment
constexpr int64_t kGramBatchBytes = (int64_t)1 << 30;

}  // namespace

namespace mml {

void wrmf_tile_plan(const std::vector<int64_t>& deg, hipStream_t st, WrmfTilePlan& p, int64_t r0,
                    int64_t r1) {
    const int32_t n = (int32_t)deg.size();
    // light rows by degree, descending (longest first: the work queue then ends on short rows)
    std::vector<int32_t> light, heavy;
    std::vector<int64_t> begin(n + 1, 0);
    for (int32_t r = 0; r < n; ++r) begin[r + 1] = begin[r] + deg[r];
    std::vector<int64_t> bucket(kHeavy + 2, 0);
    for (int32_t r = (int32_t)r0; r < (int32_t)r1; ++r)
        if (deg[r] <= kHeavy) ++bucket[kHeavy - deg[r]];
        else heavy.push_back(r);
    int64_t acc = 0;
    for (auto& b : bucket) {
        const int64_t c = b;
        b = acc;
        acc += c;
    }
    light.resize(acc);
    for (int32_t r = (int32_t)r0; r < (int32_t)r1; ++r)
        if (deg[r] <= kHeavy) light[bucket[kHeavy - deg[r]]++] = r;
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
    MML_HIP(hipStreamSynchronize(st));
}

void wrmf_tile_solve(hipStream_t st, WrmfTilePlan& p, float* W, const float* H, const int64_t* off,
                     const int32_t* cols, const double* HH, int32_t k, double alpha, double reg,
                     int& launches) {
    MML_REQUIRE(k > 128 && k <= 256, "tile solver covers 128 < k <= 256");
    const int nt = (k + 31) >> 5, nr = nt + 1;
    const int ntile = nt * nr - nt * (nt - 1) / 2;
    p.hht.alloc((size_t)kTiles * 1024);
    wrmf_tile_hh_kernel<<<(ntile * 1024 + 255) / 256, 256, 0, st>>>(HH, k, reg, p.hht.get());
    ++launches;
    const int grid_cap = 256 * 2;  // 256 CUs; a second resident workgroup where registers allow
    // heavy rows: batches whose fp64 Grams fit the workspace
    const int64_t per_row = (int64_t)kTiles * 1024 * sizeof(double);
    const int64_t batch_rows = std::max<int64_t>(1, kGramBatchBytes / per_row);
    const int64_t nh = (int64_t)p.heavy.size();
    for (int64_t h0 = 0; h0 < nh; h0 += batch_rows) {
        const int64_t h1 = std::min(nh, h0 + batch_rows);
        const int64_t s0 = p.seg_first[h0], s1 = p.seg_first[h1];
        p.gram.alloc((size_t)std::min(nh, batch_rows) * kTiles * 1024);
        MML_HIP(hipMemsetAsync(p.gram.get(), 0, (size_t)(h1 - h0) * per_row, st));
        const int gg = (int)std::min<int64_t>(s1 - s0, grid_cap);
        wrmf_tile_gram_kernel<<<gg, kThreads, 0, st>>>(reinterpret_cast<const Seg*>(p.segs.get()) + s0,
                                                  (int32_t)(s1 - s0), (int32_t)h0, cols, H, k,
                                                  p.gram.get());
        MML_HIP(hipMemsetAsync(p.counter.get(), 0, sizeof(int32_t), st));
        const int gs = (int)std::min<int64_t>(h1 - h0, grid_cap);
        wrmf_tile_solve_kernel<<<gs, kThreads, 0, st>>>(p.heavy_dev.get() + h0, (int32_t)(h1 - h0),
                                                   p.counter.get(), off, cols, W, H, p.hht.get(),
                                                   p.gram.get(), k, (float)alpha, debug_mask());
        MML_HIP(hipGetLastError());
        launches += 2;
    }
    if (p.n_light > 0) {
        MML_HIP(hipMemsetAsync(p.counter.get(), 0, sizeof(int32_t), st));
        const int gs = (int)std::min<int64_t>(p.n_light, grid_cap);
        wrmf_tile_solve_kernel<<<gs, kThreads, 0, st>>>(p.light.get(), p.n_light, p.counter.get(), off,
                                                   cols, W, H, p.hht.get(), nullptr, k,
                                                   (float)alpha, debug_mask());
        MML_HIP(hipGetLastError());
        ++launches;
    }
}

}  // namespace mml
