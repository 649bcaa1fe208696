// wrmf.hip -- WRMF (implicit ALS) on MI355X (gfx950), fp64 "parity" precision.
//
// Replaces WRMF.Iterate / Optimize / ComputeSquareMatrix
// (src/MyMediaLite/ItemRecommendation/WRMF.cs:68-156):
//   half-step W <- H:  HH = H^T H (k x k, float products, double sums)         [wrmf_gram_*]
//                      for every row u of W (one workgroup per row):
//                        A = HH + alpha * sum_{i in S_u} h_i h_i^T + reg * I   (double)
//                        b = (1 + alpha) * sum_{i in S_u} h_i
//                        W_u = (float) A^{-1} b                                 [wrmf_solve_kernel]
// The reference inverts A with MathNet's LU (partial pivoting) and multiplies; A is symmetric
// positive definite, so the device factors it by Cholesky in LDS and solves two triangular systems:
// same solution up to double rounding (~1e-15 relative), identical after the cast to float except
// in the last float ulp.
//
// HBM layout: U [n_users x k], V [n_items x k] fp32 row-major (exactly Matrix<float>), the data as
// two CSRs (user -> items, item -> users; sorted, de-duplicated = the SparseBooleanMatrix sets).
// k <= 64: A in LDS as a full double matrix (32 KiB), column Cholesky (exact parity path).
// 64 < k <= 128: block-packed lower triangle in double; 128 < k <= 256 (C5): the same in float
// (140 KiB of LDS) -- see wrmf_solve_blocked_kernel.
#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "mml_internal.h"

namespace {

constexpr int kMaxK = 64;
constexpr int kChunk = 32;  // item rows staged in LDS per pass

// Partial H^T H over a slice of rows, tiled: workgroup (tile, slice) computes one 64 x 64 tile
// (ti <= tj) of HH over rows [slice * rows_per_slice, ...), each thread a 4 x 4 patch in double;
// the tile's two 64-column strips of H are staged through LDS kChunk rows at a time.  Products are
// float, sums double, like WRMF.ComputeSquareMatrix (WRMF.cs:94-108).
__global__ __launch_bounds__(256) void wrmf_gram_partial_kernel(const float* __restrict__ H,
                                                                int64_t rows, int32_t k,
                                                                int64_t rows_per_slice,
                                                                double* __restrict__ partial) {
    __shared__ float sa[kChunk][64];
    __shared__ float sb[kChunk][64];
    const int t = threadIdx.x;
    const int nt = (k + 63) / 64;
    int tile = blockIdx.x, ti = 0;
    while (tile >= nt - ti) {  // enumerate (ti, tj) with ti <= tj
        tile -= nt - ti;
        ++ti;
    }
    const int tj = ti + tile;
    const int slice = blockIdx.y;
    const int pr = (t / 16) * 4, pc = (t % 16) * 4;  // this thread's 4 x 4 patch in the tile
    double acc[4][4] = {};
    const int64_t r0 = (int64_t)slice * rows_per_slice;
    const int64_t r1 = min(rows, r0 + rows_per_slice);
    for (int64_t base = r0; base < r1; base += kChunk) {
        const int nr = (int)min((int64_t)kChunk, r1 - base);
        __syncthreads();
        for (int e = t; e < kChunk * 64; e += 256) {
            const int c = e / 64, f = e % 64;
            const int fa = ti * 64 + f, fb = tj * 64 + f;
            sa[c][f] = (c < nr && fa < k) ? H[(base + c) * k + fa] : 0.0f;
            sb[c][f] = (c < nr && fb < k) ? H[(base + c) * k + fb] : 0.0f;
        }
        __syncthreads();
        for (int c = 0; c < nr; ++c) {
#pragma unroll
            for (int x = 0; x < 4; ++x)
#pragma unroll
                for (int y = 0; y < 4; ++y) acc[x][y] += (double)(sa[c][pr + x] * sb[c][pc + y]);
        }
    }
    const int64_t kk = (int64_t)k * k;
    for (int x = 0; x < 4; ++x)
        for (int y = 0; y < 4; ++y) {
            const int f1 = ti * 64 + pr + x, f2 = tj * 64 + pc + y;
            if (f1 < k && f2 < k) partial[(int64_t)slice * kk + (int64_t)f1 * k + f2] = acc[x][y];
        }
}

// HH = sum of the partials in block order (deterministic), mirrored from the upper triangle.
__global__ __launch_bounds__(256) void wrmf_gram_reduce_kernel(const double* __restrict__ partial,
                                                               int32_t nparts, int32_t k,
                                                               double* __restrict__ HH) {
    const int e = blockIdx.x * blockDim.x + threadIdx.x;
    const int kk = k * k;
    if (e >= kk) return;
    const int f1 = e / k, f2 = e % k;
    const int src = (f1 / 64) <= (f2 / 64) ? e : f2 * k + f1;
    double s = 0.0;
    for (int p = 0; p < nparts; ++p) s += partial[(int64_t)p * kk + src];
    HH[e] = s;
}

// One workgroup per row of W.
__global__ __launch_bounds__(256) void wrmf_solve_kernel(
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols, int64_t n_data_rows,
    int64_t row_begin, int64_t row_end, float* __restrict__ W, const float* __restrict__ H,
    const double* __restrict__ HH, int32_t k, double alpha, double reg) {
    __shared__ double A[kMaxK][kMaxK + 1];
    __shared__ double bv[kMaxK];
    __shared__ float hs[kChunk][kMaxK];
    __shared__ int32_t idx[kChunk];
    const int t = threadIdx.x;
    const int kk = k * k;
    for (int64_t row = row_begin + blockIdx.x; row < row_end; row += gridDim.x) {
        const int64_t b = row < n_data_rows ? off[row] : 0;
        const int64_t e = row < n_data_rows ? off[row + 1] : 0;
        double acc[kMaxK * kMaxK / 256];
        for (int x = 0; x < kMaxK * kMaxK / 256; ++x) acc[x] = 0.0;
        double hsum = 0.0;
        for (int64_t base = b; base < e; base += kChunk) {
            const int nr = (int)min((int64_t)kChunk, e - base);
            __syncthreads();
            if (t < nr) idx[t] = cols[base + t];
            __syncthreads();
            for (int x = t; x < nr * k; x += 256)
                hs[x / k][x % k] = H[(int64_t)idx[x / k] * k + x % k];
            __syncthreads();
            for (int x = 0; x < kMaxK * kMaxK / 256; ++x) {
                const int en = t + 256 * x;
                if (en >= kk) break;
                const int f1 = en / k, f2 = en % k;
                if (f1 > f2) continue;
                double a = acc[x];
                for (int c = 0; c < nr; ++c) a += (double)(hs[c][f1] * hs[c][f2]);
                acc[x] = a;
            }
            if (t < k)
                for (int c = 0; c < nr; ++c) hsum += (double)hs[c][t];
        }
        __syncthreads();
        // A = HH + alpha * S (+ reg on the diagonal), symmetric (WRMF.cs:137-146)
        for (int x = 0; x < kMaxK * kMaxK / 256; ++x) {
            const int en = t + 256 * x;
            if (en >= kk) break;
            const int f1 = en / k, f2 = en % k;
            if (f1 > f2) continue;
            double d = HH[f1 * k + f2] + acc[x] * alpha;
            if (f1 == f2) d += reg;
            A[f1][f2] = d;
            A[f2][f1] = d;
        }
        if (t < k) bv[t] = hsum * (1.0 + alpha);
        __syncthreads();
        // Cholesky, right-looking, lower triangle in place
        for (int j = 0; j < k; ++j) {
            if (t == 0) A[j][j] = sqrt(A[j][j]);
            __syncthreads();
            const double djj = A[j][j];
            for (int i = j + 1 + t; i < k; i += 256) A[i][j] /= djj;
            __syncthreads();
            const int m = k - j - 1;  // trailing size
            for (int x = t; x < m * m; x += 256) {
                const int i = j + 1 + x / m, l = j + 1 + x % m;
                if (l <= i) A[i][l] -= A[i][j] * A[l][j];
            }
            __syncthreads();
        }
        // forward L y = b, then backward L^T w = y (column-oriented, in place in bv)
        for (int j = 0; j < k; ++j) {
            if (t == 0) bv[j] /= A[j][j];
            __syncthreads();
            for (int i = j + 1 + t; i < k; i += 256) bv[i] -= A[i][j] * bv[j];
            __syncthreads();
        }
        for (int j = k - 1; j >= 0; --j) {
            if (t == 0) bv[j] /= A[j][j];
            __syncthreads();
            for (int i = t; i < j; i += 256) bv[i] -= A[j][i] * bv[j];
            __syncthreads();
        }
        if (t < k) W[row * k + t] = (float)bv[t];
        __syncthreads();
    }
}

// ---------------------------------------------------------------------------------------------
// k in (64, 256]: one workgroup (4 waves) per row; A lives in LDS as a BLOCK-PACKED lower triangle
// of 8 x 8 blocks (block (bi, bj), bj <= bi, stored contiguously: element (i, j) at
// BP(i/8, j/8) + 8*(i%8) + j%8), so every phase moves whole 32-B (float) / 64-B (double) block rows
// with 16-B LDS accesses.  T = double for k <= 128 (78 KiB), float for k <= 256 (140 KiB; the
// reference's doubles do not fit the 160 KiB LDS at k = 256).  b is appended as row k, so the
// forward substitution L y = b happens inside the factorisation (y = row k of L).  Per row:
//   1. Gram S = sum_i h_i h_i^T into A's blocks (acc in registers per block, chunks of the row's
//      item vectors staged in LDS), b = sum_i h_i;
//   2. A = HHp + alpha * S (HHp = HH + reg I, block-packed once per half-step), row k = (1+alpha) b;
//   3. blocked right-looking Cholesky: wave 0 factors block column p in registers (pivot rows
//      p*8+c live in lane c: broadcast by v_readlane), then all waves apply the rank-8 update to the
//      trailing blocks;
//   4. blocked backward substitution L^T w = y, one 8-block at a time.
template <typename T>
__device__ __forceinline__ void lds_load8(const T* p, T (&v)[8]) {
    if constexpr (sizeof(T) == 4) {
        const float4 a = reinterpret_cast<const float4*>(p)[0];
        const float4 b = reinterpret_cast<const float4*>(p)[1];
        v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
        v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
    } else {
#pragma unroll
        for (int x = 0; x < 4; ++x) {
            const double2 a = reinterpret_cast<const double2*>(p)[x];
            v[2 * x] = a.x;
            v[2 * x + 1] = a.y;
        }
    }
}
__device__ __forceinline__ float bcast(float v, int lane) {
    return __int_as_float(__builtin_amdgcn_readlane(__float_as_int(v), lane));
}
__device__ __forceinline__ double bcast(double v, int lane) {
    const unsigned long long u = (unsigned long long)__double_as_longlong(v);
    const unsigned lo = __builtin_amdgcn_readlane((int)(unsigned)u, lane);
    const unsigned hi = __builtin_amdgcn_readlane((int)(unsigned)(u >> 32), lane);
    return __longlong_as_double((long long)(((unsigned long long)hi << 32) | lo));
}

// Block rows are stored bank-rotated: the 16-B chunks of a block (16 for float, 32 for double)
// are rotated by the block's linear index, so 16 lanes that touch the same row of 16 different
// blocks (Gram, trailing update) hit 16 different LDS bank groups instead of one (a 16-way
// conflict for ds_read_b128 with 256-B blocks: MI355X_MICROARCH.md, LDS).
template <typename T>
__device__ __forceinline__ int chunk_addr(int q, int chunk) {
    constexpr int NCH = 64 * (int)sizeof(T) / 16;  // 16-B chunks per block
    constexpr int PER = 16 / (int)sizeof(T);       // T per chunk
    return q * 64 + ((chunk + q) & (NCH - 1)) * PER;
}
template <typename T>
__device__ __forceinline__ void row_load8(const T* A, int q, int x, T (&v)[8]) {
    constexpr int CPR = 8 * (int)sizeof(T) / 16;  // chunks per 8-element row
    constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
    for (int c = 0; c < CPR; ++c) {
        const T* p = A + chunk_addr<T>(q, x * CPR + c);
        if constexpr (sizeof(T) == 4) {
            const float4 a = *reinterpret_cast<const float4*>(p);
            v[c * PER] = a.x; v[c * PER + 1] = a.y; v[c * PER + 2] = a.z; v[c * PER + 3] = a.w;
        } else {
            const double2 a = *reinterpret_cast<const double2*>(p);
            v[c * PER] = a.x; v[c * PER + 1] = a.y;
        }
    }
}
template <typename T>
__device__ __forceinline__ void row_store8(T* A, int q, int x, const T (&v)[8]) {
    constexpr int CPR = 8 * (int)sizeof(T) / 16;
    constexpr int PER = 16 / (int)sizeof(T);
#pragma unroll
    for (int c = 0; c < CPR; ++c) {
        T* p = A + chunk_addr<T>(q, x * CPR + c);
        if constexpr (sizeof(T) == 4)
            *reinterpret_cast<float4*>(p) =
                make_float4(v[c * PER], v[c * PER + 1], v[c * PER + 2], v[c * PER + 3]);
        else
            *reinterpret_cast<double2*>(p) = make_double2(v[c * PER], v[c * PER + 1]);
    }
}
// element (x, y) of block q
template <typename T>
__device__ __forceinline__ int elem(int q, int x, int y) {
    constexpr int PER = 16 / (int)sizeof(T);
    return chunk_addr<T>(q, (x * 8 + y) / PER) + (x * 8 + y) % PER;
}
__device__ __forceinline__ int bidx(int bi, int bj) { return bi * (bi + 1) / 2 + bj; }

template <int KMAX>
struct BlockedGeom {
    static constexpr int NB1 = (KMAX + 8) / 8;  // block rows for rows 0..KMAX (b row included)
    static constexpr int NBLK = NB1 * (NB1 + 1) / 2;
    static constexpr int CH = 16;
    static constexpr int RPL = (KMAX + 1 + 63) / 64;  // panel rows per lane
};

__device__ __forceinline__ void decode_lower(int q, int& bi, int& bj) {
    bi = (int)((sqrtf(8.0f * (float)q + 1.0f) - 1.0f) * 0.5f);
    while (bi * (bi + 1) / 2 > q) --bi;
    while ((bi + 1) * (bi + 2) / 2 <= q) ++bi;
    bj = q - bi * (bi + 1) / 2;
}

// HHp = HH + reg * I in the block-packed layout (zero outside the k x k lower triangle)
template <typename T, int KMAX>
__global__ __launch_bounds__(256) void wrmf_pack_hh_kernel(const double* __restrict__ HH, int32_t k,
                                                           double reg, T* __restrict__ HHp) {
    using G = BlockedGeom<KMAX>;
    for (int e = blockIdx.x * blockDim.x + threadIdx.x; e < G::NBLK * 64;
         e += gridDim.x * blockDim.x) {
        int bi, bj;
        const int q = e / 64, x = (e % 64) / 8, y = e % 8;
        decode_lower(q, bi, bj);
        const int i = bi * 8 + x, j = bj * 8 + y;
        double v = 0.0;
        if (i < k && j < k && j <= i) v = HH[i * k + j] + (i == j ? reg : 0.0);
        HHp[elem<T>(q, x, y)] = (T)v;
    }
}

template <typename T, int KMAX>
__global__ __launch_bounds__(256, 1) void wrmf_solve_blocked_kernel(
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols, int64_t n_data_rows,
    int64_t row_begin, int64_t row_end, float* __restrict__ W, const float* __restrict__ H,
    const T* __restrict__ HHp,
    int32_t k, double alpha) {
    using G = BlockedGeom<KMAX>;
    constexpr int CH = G::CH, RPL = G::RPL;
    constexpr int A_BYTES = G::NBLK * 64 * (int)sizeof(T);
    extern __shared__ __attribute__((aligned(16))) char smem[];
    T* A = reinterpret_cast<T*>(smem);
    float* hs = reinterpret_cast<float*>(smem + A_BYTES);  // [CH][KMAX]
    T* wv = reinterpret_cast<T*>(hs + CH * KMAX);          // [KMAX]
    int32_t* idx = reinterpret_cast<int32_t*>(wv + KMAX);  // [CH]
    const int t = threadIdx.x, lane = t & 63, wave = t >> 6;
    const int nb = (k + 7) / 8;        // block rows/cols of A proper
    const int nbr = k / 8 + 1;         // block rows incl. the b row (row k)
    const int ngram = nb * (nb + 1) / 2;
    constexpr int V4 = 16 / (int)sizeof(T);  // T per 16-B granule
    auto E = [](int i, int j) { return elem<T>(bidx(i >> 3, j >> 3), i & 7, j & 7); };
    for (int64_t row = row_begin + blockIdx.x; row < row_end; row += gridDim.x) {
        const int64_t rb = row < n_data_rows ? off[row] : 0;
        const int64_t re = row < n_data_rows ? off[row + 1] : 0;
        __syncthreads();
        for (int g = t; g < G::NBLK * 64 / V4; g += 256)
            reinterpret_cast<float4*>(A)[g] = make_float4(0.f, 0.f, 0.f, 0.f);
        T hsum = (T)0;
        // ---- 1. Gram
        for (int64_t base = rb; base < re; base += CH) {
            const int nr = (int)min((int64_t)CH, re - base);
            __syncthreads();
            if (t < nr) idx[t] = cols[base + t];
            __syncthreads();
            for (int e = t; e < CH * KMAX; e += 256) {
                const int c = e / KMAX, f = e % KMAX;
                hs[e] = (c < nr && f < k) ? H[(int64_t)idx[c] * k + f] : 0.0f;
            }
            __syncthreads();
            for (int q = t; q < ngram; q += 256) {
                int bi, bj;
                decode_lower(q, bi, bj);
                T acc[8][8];
#pragma unroll
                for (int x = 0; x < 8; ++x) row_load8(A, q, x, acc[x]);
                for (int c = 0; c < nr; ++c) {
                    float xa[8], ya[8];
                    lds_load8(hs + c * KMAX + bi * 8, xa);
                    lds_load8(hs + c * KMAX + bj * 8, ya);
#pragma unroll
                    for (int x = 0; x < 8; ++x)
#pragma unroll
                        for (int y = 0; y < 8; ++y) acc[x][y] += (T)(xa[x] * ya[y]);
                }
#pragma unroll
                for (int x = 0; x < 8; ++x) row_store8(A, q, x, acc[x]);
            }
            if (t < k)
                for (int c = 0; c < nr; ++c) hsum += (T)hs[c * KMAX + t];
        }
        __syncthreads();
        // ---- 2. A = HHp + alpha * S; row k = (1 + alpha) * b
        for (int e = t; e < G::NBLK * 64; e += 256) A[e] = HHp[e] + (T)alpha * A[e];
        __syncthreads();
        if (t < k) A[E(k, t)] = hsum * (T)(1.0 + alpha);
        __syncthreads();
        // ---- 3. blocked Cholesky (columns 0..k-1, rows 0..k)
        for (int p = 0; p < nb; ++p) {
            const int j0 = p * 8, pw = min(8, k - j0);
            if (wave == 0) {
                T pv[RPL][8];
#pragma unroll
                for (int m = 0; m < RPL; ++m) {
                    const int r = j0 + lane + 64 * m;
                    if (r <= k) row_load8(A, bidx(r >> 3, p), r & 7, pv[m]);
                    else
#pragma unroll
                        for (int c = 0; c < 8; ++c) pv[m][c] = (T)0;
                }
#pragma unroll
                for (int c = 0; c < 8; ++c) {
                    if (c >= pw) break;
                    const int j = j0 + c;  // pivot row j lives in lane c, slot 0
                    const T djj = sqrt(bcast(pv[0][c], c));
                    const T inv = (T)1 / djj;
#pragma unroll
                    for (int m = 0; m < RPL; ++m) {
                        const int r = j0 + lane + 64 * m;
                        if (r == j) pv[m][c] = djj;
                        else if (r > j && r <= k) pv[m][c] *= inv;
                    }
#pragma unroll
                    for (int l = c + 1; l < 8; ++l) {
                        if (l >= pw) break;
                        const T ljl = bcast(pv[0][c], l);  // L[j0 + l][j]
#pragma unroll
                        for (int m = 0; m < RPL; ++m) {
                            const int r = j0 + lane + 64 * m;
                            if (r >= j0 + l && r <= k) pv[m][l] -= pv[m][c] * ljl;
                        }
                    }
                }
#pragma unroll
                for (int m = 0; m < RPL; ++m) {
                    const int r = j0 + lane + 64 * m;
                    if (r <= k) row_store8(A, bidx(r >> 3, p), r & 7, pv[m]);
                }
            }
            __syncthreads();
            // trailing blocks (bi, bj): p < bj <= bi, bi < nbr (rows <= k), bj < nb (cols < k)
            const int tn = nbr - (p + 1);           // block rows in the trailing part
            const int tcols = nb - (p + 1);         // block cols in the trailing part
            const int ntr = tn * (tn + 1) / 2;
            if (tcols > 0)
                for (int q = t; q < ntr; q += 256) {
                    int di, dj;
                    decode_lower(q, di, dj);
                    if (dj >= tcols) continue;
                    const int bi = p + 1 + di, bj = p + 1 + dj;
                    const int qi = bidx(bi, p), qj = bidx(bj, p), qa = bidx(bi, bj);
                    T li[8][8], lj[8][8];
#pragma unroll
                    for (int x = 0; x < 8; ++x) {
                        row_load8(A, qi, x, li[x]);
                        row_load8(A, qj, x, lj[x]);
                    }
#pragma unroll
                    for (int x = 0; x < 8; ++x) {
                        T a[8];
                        row_load8(A, qa, x, a);
#pragma unroll
                        for (int y = 0; y < 8; ++y) {
                            T sacc = a[y];
#pragma unroll
                            for (int c = 0; c < 8; ++c) sacc -= li[x][c] * lj[y][c];
                            a[y] = sacc;
                        }
                        row_store8(A, qa, x, a);
                    }
                }
            __syncthreads();
        }
        // ---- 4. backward substitution L^T w = y
        if (t < k) wv[t] = A[E(k, t)];
        __syncthreads();
        for (int p = nb - 1; p >= 0; --p) {
            const int j0 = p * 8, pw = min(8, k - j0);
            if (wave == 0) {
                T L[8][8], w[8];
#pragma unroll
                for (int x = 0; x < 8; ++x) row_load8(A, bidx(p, p), x, L[x]);
#pragma unroll
                for (int x = 0; x < 8; ++x) w[x] = x < pw ? wv[j0 + x] : (T)0;
#pragma unroll
                for (int j = 7; j >= 0; --j) {
                    if (j < pw) {
                        T v = w[j];
#pragma unroll
                        for (int i = j + 1; i < 8; ++i)
                            if (i < pw) v -= L[i][j] * w[i];
                        w[j] = v / L[j][j];
                    }
                }
                if (lane < pw) {
                    T out = w[0];
#pragma unroll
                    for (int x = 1; x < 8; ++x)
                        if (lane == x) out = w[x];
                    wv[j0 + lane] = out;
                }
            }
            __syncthreads();
            for (int i = t; i < j0; i += 256) {
                T v = wv[i];
                const int qb = bidx(p, i >> 3);
                for (int j = 0; j < pw; ++j) v -= A[elem<T>(qb, j, i & 7)] * wv[j0 + j];
                wv[i] = v;
            }
            __syncthreads();
        }
        if (t < k) W[row * k + t] = (float)wv[t];
    }
}

template <typename T, int KMAX>
constexpr size_t blocked_lds_bytes() {
    return (size_t)BlockedGeom<KMAX>::NBLK * 64 * sizeof(T) +
           (size_t)BlockedGeom<KMAX>::CH * KMAX * sizeof(float) + (size_t)KMAX * sizeof(T) +
           (size_t)BlockedGeom<KMAX>::CH * sizeof(int32_t);
}

__global__ __launch_bounds__(256) void wrmf_predict_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, int64_t n,
    int32_t n_users, int32_t n_items, const float* __restrict__ U, const float* __restrict__ V,
    int32_t k, float* __restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = users[x], i = items[x];
        if (u < 0 || u >= n_users || i < 0 || i >= n_items) {
            out[x] = -3.402823466e+38f;  // MF.Predict: float.MinValue (MF.cs:151-157)
            continue;
        }
        float dot = 0.0f;
        for (int f = 0; f < k; ++f) dot += U[(int64_t)u * k + f] * V[(int64_t)i * k + f];
        out[x] = dot;
    }
}

// host: CSR of distinct (row, col) pairs, each row sorted
void build_csr(const int32_t* rows, const int32_t* cols, int64_t n, int32_t n_rows,
               std::vector<int64_t>& off, std::vector<int32_t>& out) {
    off.assign(n_rows + 1, 0);
    for (int64_t x = 0; x < n; ++x) ++off[rows[x] + 1];
    for (int32_t r = 0; r < n_rows; ++r) off[r + 1] += off[r];
    std::vector<int32_t> tmp(n);
    std::vector<int64_t> fill(off.begin(), off.end() - 1);
    for (int64_t x = 0; x < n; ++x) tmp[fill[rows[x]]++] = cols[x];
    out.clear();
    out.reserve(n);
    std::vector<int64_t> doff(n_rows + 1, 0);
    for (int32_t r = 0; r < n_rows; ++r) {
        auto b = tmp.begin() + off[r], e = tmp.begin() + off[r + 1];
        std::sort(b, e);
        auto last = std::unique(b, e);
        out.insert(out.end(), b, last);
        doff[r + 1] = (int64_t)out.size();
    }
    off.swap(doff);
}

}  // namespace

struct mml_wrmf {
    mml_ctx* ctx = nullptr;
    mml_wrmf_params p{};
    int32_t n_users = 0, n_items = 0, k = 0;
    mml::DeviceArray<float> U, V, q_out;
    mml::DeviceArray<int64_t> uoff, ioff;
    mml::DeviceArray<int32_t> ucols, icols, q_u, q_i;
    mml::DeviceArray<double> HH, partial;
    bool has_data = false, has_model = false;
    float last_ms = 0.0f;
    float last_gather_ms = 0.0f;             // the last iterate's two all-gathers (device time)
    hipEvent_t ev_g[4] = {nullptr, nullptr, nullptr, nullptr};
    int32_t last_launches = 0;
    int32_t last_refine = 0;  // the most refinement passes a half-step of the last iterate ran
    float last_corr[8] = {};  // per half-step (users, items) and pass: the max relative correction
    int32_t nparts = 1;
    int64_t nnz = 0;
    // the item half's pipeline (mml_wrmf_set_pipeline): 0 = the default row ranges, 1 = off (the
    // residual after the whole solve, HH on the handle's stream), n = n ranges
    int32_t pipe_req = 0;
    mml::DeviceArray<uint8_t> hhp;  // HH + reg I, block-packed (k > 64 path)
    // the items' HH = U^T U computed from the users' solve while the users' refinement runs
    // (half_step); valid when that refinement left U as it was (every Woodbury row screened)
    mml::DeviceArray<double> HHspec;
    hipEvent_t spec_go = nullptr, spec_done = nullptr;
    bool spec_valid = false;
    mml::WrmfTilePlan uplan, iplan;  // k > 128: matrix-core row solves (wrmf_tiles.hip)
    // row shards (one process per GPU): rank r solves rows [ub[r], ub[r+1]) of U and
    // [ib[r], ib[r+1]) of V; the halves are exchanged by an all-gather (grouped broadcasts)
    std::vector<int64_t> udeg, ideg, ub, ib;
    int32_t shard_nranks = 0, shard_rank = -1;
    // multi-device context: one single-device handle per GPU, each holding the whole data set
    // and solving its row shards (rank d of the context's communicator); after every half-step
    // the shards are all-gathered, so every device ends an iteration with the full model
    std::vector<mml_wrmf*> shards;
};

namespace {

// MML_WRMF_SOLVER=blocked keeps the LDS-packed fp32 solver for k > 128 (A/B measurements)
bool use_blocked_solver() {
    static const bool v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_SOLVER");
        return e && std::string(e) == "blocked";
    }();
    return v;
}

// MML_WRMF_WOODBURY=0 solves every row directly (A/B measurements of the Woodbury rows)
bool no_woodbury() {
    static const bool v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_WOODBURY");
        return e && std::string(e) == "0";
    }();
    return v;
}

// MML_WRMF_SPEC_HH=0 (experiments builds): the items' HH after the users' refinement (A/B)
bool spec_hh() {
    static const bool v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_SPEC_HH");
        return !(e && std::string(e) == "0");
    }();
    return v;
}

template <typename T, int KMAX>
void run_blocked(mml_wrmf* h, float* W, int64_t r0, int64_t r1, const float* H, const int64_t* off,
                 const int32_t* cols, int64_t n_data_rows) {
    hipStream_t st = h->ctx->stream;
    static const bool attr = [] {
        (void)hipFuncSetAttribute(reinterpret_cast<const void*>(&wrmf_solve_blocked_kernel<T, KMAX>),
                                  hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)blocked_lds_bytes<T, KMAX>());
        return true;
    }();
    (void)attr;
    constexpr int nblk = BlockedGeom<KMAX>::NBLK;
    h->hhp.alloc((size_t)nblk * 64 * sizeof(T));
    T* hhp = reinterpret_cast<T*>(h->hhp.get());
    wrmf_pack_hh_kernel<T, KMAX><<<(nblk * 64 + 255) / 256, 256, 0, st>>>(
        h->HH.get(), h->k, h->p.regularization, hhp);
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(r1 - r0, 256 * 4));
    wrmf_solve_blocked_kernel<T, KMAX><<<grid, 256, blocked_lds_bytes<T, KMAX>(), st>>>(
        off, cols, n_data_rows, r0, r1, W, H, hhp, h->k, h->p.alpha);
}

// W rows [r0, r1) <- H (all h_rows rows); off/cols: the CSR of W's rows
// (plan: the k > 128 row plan of W's rows; null = the handle's plan of U or V)
void half_step(mml_wrmf* h, float* W, int64_t r0, int64_t r1, const float* H, int64_t h_rows,
               const int64_t* off, const int32_t* cols, int64_t n_data_rows, int& launches,
               mml::WrmfTilePlan* plan_in = nullptr) {
    hipStream_t st = h->ctx->stream;
    const int k = h->k;
    const int nt = (k + 63) / 64;
    const int tiles = nt * (nt + 1) / 2;
    const int nparts = h->nparts;
    const int64_t rps = (h_rows + nparts - 1) / nparts;
    const bool tiles_path = k > 128 && !use_blocked_solver();
    // HH = H^T H on the plan's second stream while the hot rows' split Gram runs (it needs H
    // only), when the half has hot rows and no Woodbury rows (those read HH on the host first)
    hipStream_t hs = st;
    mml::WrmfTilePlan* dplan = nullptr;
    // the users' half-step already computed this HH from U, which its refinement left unchanged
    const bool spec = h->spec_valid && H == h->U.get() && h_rows == h->n_users;
    h->spec_valid = false;
    static const bool hh_side = [] {  // MML_WRMF_HH_SIDE=0 (experiments builds): HH on st (A/B)
        const char* e = MML_EXPERIMENT_ENV("MML_WRMF_HH_SIDE");
        return !(e && std::string(e) == "0");
    }();
    if (tiles_path && r1 > r0 && hh_side && h->pipe_req != 1 && !spec) {
        mml::WrmfTilePlan& pl = plan_in ? *plan_in : W == h->U.get() ? h->uplan : h->iplan;
        if (!pl.heavy.empty() && pl.n_wood[0] + pl.n_wood[1] + pl.n_wood[2] + pl.n_wood[3] == 0) {
            hipStream_t side = mml::wrmf_plan_side(pl, st);
            if (side) {
                if (!pl.hh_start) MML_HIP(hipEventCreateWithFlags(&pl.hh_start, hipEventDisableTiming));
                if (!pl.hh_done) MML_HIP(hipEventCreateWithFlags(&pl.hh_done, hipEventDisableTiming));
                MML_HIP(hipEventRecord(pl.hh_start, st));  // H is final on st
                MML_HIP(hipStreamWaitEvent(side, pl.hh_start, 0));
                hs = side;
                dplan = &pl;
            }
        }
    }
    if (spec) {
        MML_HIP(hipStreamWaitEvent(st, h->spec_done, 0));
        h->HH.swap(h->HHspec);  // the same kernels over the same rows: the same HH
    } else {
        wrmf_gram_partial_kernel<<<dim3(tiles, nparts), 256, 0, hs>>>(H, h_rows, k, rps,
                                                                     h->partial.get());
        wrmf_gram_reduce_kernel<<<(k * k + 255) / 256, 256, 0, hs>>>(h->partial.get(), nparts, k,
                                                                      h->HH.get());
        launches += 2;
    }
    if (dplan) {
        MML_HIP(hipEventRecord(dplan->hh_done, hs));
        dplan->hh_pending = true;
    }
    if (r1 <= r0) {
        // a rank without rows in this half still joins the ranks' refinement decisions
        if (tiles_path && !plan_in) {
            mml::WrmfTilePlan& plan = W == h->U.get() ? h->uplan : h->iplan;
            mml::wrmf_tile_refine(st, plan, W, H, h_rows, off, cols, h->HH.get(), k, h->p.alpha,
                                  h->p.regularization, h->p.refine_passes, launches, nullptr,
                                  h->ctx);
        }
        return;
    }
    if (k <= kMaxK) {
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(r1 - r0, 256 * 16));
        wrmf_solve_kernel<<<grid, 256, 0, st>>>(off, cols, n_data_rows, r0, r1, W, H, h->HH.get(),
                                                k, h->p.alpha, h->p.regularization);
    } else if (k <= 128) {
        run_blocked<double, 128>(h, W, r0, r1, H, off, cols, n_data_rows);
    } else if (use_blocked_solver()) {
        run_blocked<float, 256>(h, W, r0, r1, H, off, cols, n_data_rows);
    } else {
        mml::WrmfTilePlan& plan = plan_in ? *plan_in : W == h->U.get() ? h->uplan : h->iplan;
        plan.keep_factor = h->p.refine_passes > 0;
        plan.refined = h->p.refine_passes > 0;
        mml::wrmf_tile_solve(st, plan, W, H, h_rows, off, cols, h->HH.get(), k, h->p.alpha,
                             h->p.regularization, launches);
        // the items' HH = U^T U from the solved U on the second stream while the refinement
        // runs: one rank, all of U solved here, every row a Woodbury row (the refinement then
        // leaves U as it is when the screen settles every row: x += 0, and a -0 that becomes +0
        // does not change a sum that starts from +0)
        const bool spec_users = !plan_in && W == h->U.get() && plan.refined && r0 == 0 &&
                                r1 == h->n_users && h->shard_nranks == 1 && plan.n_light == 0 &&
                                plan.heavy.empty() && spec_hh();
        hipStream_t sside = spec_users ? mml::wrmf_plan_side(plan, st) : nullptr;
        // the hooks capture this call's locals: cleared on every way out of it, a throw included,
        // so no later refinement calls a stale one
        struct HookReset {
            mml::WrmfTilePlan& p;
            ~HookReset() {
                p.after_dense = nullptr;
                p.pre_update_wait = nullptr;
            }
        } hook_reset{plan};
        if (sside) {
            if (!h->spec_go) {
                MML_HIP(hipEventCreateWithFlags(&h->spec_go, hipEventDisableTiming));
                MML_HIP(hipEventCreateWithFlags(&h->spec_done, hipEventDisableTiming));
            }
            h->HHspec.reserve((size_t)k * k);
            const int64_t rps_u = (h->n_users + nparts - 1) / nparts;  // as the items' half-step
            // issued by the refinement after its dense term: beside the data term's gathers
            // (beside the dense term's fp64 MFMAs it slowed them 15 -> 32 ms, profiles/r5ax/)
            plan.after_dense = [h, sside, W, k, rps_u, tiles, nparts, &launches](hipStream_t s) {
                MML_HIP(hipEventRecord(h->spec_go, s));
                MML_HIP(hipStreamWaitEvent(sside, h->spec_go, 0));
                wrmf_gram_partial_kernel<<<dim3(tiles, nparts), 256, 0, sside>>>(
                    W, h->n_users, k, rps_u, h->partial.get());
                wrmf_gram_reduce_kernel<<<(k * k + 255) / 256, 256, 0, sside>>>(
                    h->partial.get(), nparts, k, h->HHspec.get());
                MML_HIP(hipEventRecord(h->spec_done, sside));
                launches += 2;
            };
            plan.pre_update_wait = h->spec_done;
        }
        const int32_t done = mml::wrmf_tile_refine(
            st, plan, W, H, h_rows, off, cols, h->HH.get(), k, h->p.alpha, h->p.regularization,
            h->p.refine_passes, launches, h->last_corr + (W == h->U.get() ? 0 : 4),
            plan_in ? nullptr : h->ctx);
        h->last_refine = std::max(h->last_refine, done);
        if (sside) {
            plan.pre_update_wait = nullptr;  // (no pass ran: nothing waited)
            MML_REQUIRE(!plan.after_dense, "the speculative HH was not issued");
            h->spec_valid = done == 1 && plan.screen_left == 0;
            if (!h->spec_valid)  // U changed: the items' half-step computes its own HH
                MML_HIP(hipStreamWaitEvent(st, h->spec_done, 0));
        }
    }
    MML_HIP(hipGetLastError());
    launches += 1;
}

// all-gather of the row shards of W [rows x k] in place: one broadcast per rank, grouped (a
// repeated-device context: peer copies between the ranks' threads, peer.hip)
void allgather_rows(mml_wrmf* h, float* W, const std::vector<int64_t>& b) {
    mml_ctx* c = h->ctx;
    if (!c->comm) {
        MML_REQUIRE(c->peers, "row shards without a communicator or peer group");
        c->peers->allgather_rows(c, W, b, h->k);
        return;
    }
    MML_RCCL(ncclGroupStart());
    for (int r = 0; r < c->nranks; ++r) {
        const size_t cnt = (size_t)(b[r + 1] - b[r]) * h->k;
        if (!cnt) continue;
        float* p = W + (size_t)b[r] * h->k;
        MML_RCCL(ncclBroadcast(p, p, cnt, ncclFloat, r, c->comm, c->stream));
    }
    MML_RCCL(ncclGroupEnd());
}

// (re)derive the shards for the context's communicator and the row plans of this rank
void ensure_shards(mml_wrmf* h) {
    const mml_ctx* c = h->ctx;
    const int32_t nr = c->comm ? c->nranks : c->peers ? c->peers->n : 1;
    const int32_t rk = c->comm ? c->rank : c->peers ? c->peer_rank : 0;
    if (nr == h->shard_nranks && rk == h->shard_rank) return;
    h->ub = mml::balanced_rows(h->udeg, h->k, nr);
    h->ib = mml::balanced_rows(h->ideg, h->k, nr);
    if (h->k > 128) {
        // the half-steps run one after another on one stream: one refinement workspace for both
        h->iplan.ws = &h->uplan.own;
        const bool wood = h->p.alpha > 0.0 && !no_woodbury();
        mml::wrmf_tile_plan(h->udeg, h->ctx->stream, h->uplan, h->ub[rk], h->ub[rk + 1], wood,
                            h->pipe_req);
        mml::wrmf_tile_plan(h->ideg, h->ctx->stream, h->iplan, h->ib[rk], h->ib[rk + 1], wood,
                            h->pipe_req);
    }
    h->shard_nranks = nr;
    h->shard_rank = rk;
}

// the row degrees of both CSRs (host): shard bounds and the k > 128 row plans derive from them
void set_degrees(mml_wrmf* h, std::vector<int64_t> udeg, std::vector<int64_t> ideg) {
    h->udeg = std::move(udeg);
    h->ideg = std::move(ideg);
    h->shard_nranks = 0;
    h->shard_rank = -1;
}

}  // namespace

using mml::guard;

extern "C" mml_status mml_wrmf_create(mml_ctx* ctx, const mml_wrmf_params* params,
                                      int32_t n_users, int32_t n_items, mml_wrmf** out) {
    return guard([&] {
        MML_REQUIRE(ctx && params && out, "null argument");
        MML_REQUIRE(n_users >= 1 && n_items >= 1, "need >= 1 user and item");
        MML_REQUIRE(params->num_factors >= 1 && params->num_factors <= 256,
                    "num_factors must be in [1, 256]");
        if (ctx->multi()) {
            auto* h = new mml_wrmf();
            h->ctx = ctx;
            h->p = *params;
            h->n_users = n_users;
            h->n_items = n_items;
            h->k = params->num_factors;
            h->shards.assign(ctx->sub.size(), nullptr);
            for (size_t d = 0; d < ctx->sub.size(); ++d) {
                const mml_status st =
                    mml_wrmf_create(ctx->sub[d], params, n_users, n_items, &h->shards[d]);
                if (st != MML_OK) {
                    const std::string m = mml_last_error();
                    mml_wrmf_destroy(h);
                    mml::fail(st, m);
                }
            }
            *out = h;
            return;
        }
        ctx->activate();
        auto* h = new mml_wrmf();
        try {
            h->ctx = ctx;
            h->p = *params;
            h->n_users = n_users;
            h->n_items = n_items;
            h->k = params->num_factors;
            h->U.alloc((size_t)n_users * h->k);
            h->V.alloc((size_t)n_items * h->k);
            h->HH.alloc((size_t)h->k * h->k);
            // Gram partial slices: <= 1024 and <= 32M doubles of workspace
            h->nparts = (int)std::max<int64_t>(
                1, std::min<int64_t>(1024, ((int64_t)32 << 20) / ((int64_t)h->k * h->k)));
            h->partial.alloc((size_t)h->nparts * h->k * h->k);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

extern "C" mml_status mml_wrmf_destroy(mml_wrmf* h) {
    return guard([&] {
        if (!h) return;
        if (!h->ctx) {  // a create that failed before binding the context
            delete h;
            return;
        }
        if (h->ctx && h->ctx->multi()) {
            for (mml_wrmf* s : h->shards)
                if (s) mml_wrmf_destroy(s);
            delete h;
            return;
        }
        (void)hipSetDevice(h->ctx->device);
        (void)hipStreamSynchronize(h->ctx->stream);
        for (hipEvent_t e : h->ev_g)
            if (e) (void)hipEventDestroy(e);
        if (h->spec_go) (void)hipEventDestroy(h->spec_go);
        if (h->spec_done) (void)hipEventDestroy(h->spec_done);
        delete h;
    });
}

extern "C" mml_status mml_wrmf_set_data(mml_wrmf* h, const int32_t* users, const int32_t* items,
                                        int64_t n) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {
            mml::on_devices(h->ctx, [&](int32_t d) { return mml_wrmf_set_data(h->shards[d], users, items, n); });
            h->has_data = true;
            return;
        }
        MML_REQUIRE(n >= 0 && (n == 0 || (users && items)), "bad event arrays");
        for (int64_t x = 0; x < n; ++x)
            MML_REQUIRE(users[x] >= 0 && users[x] < h->n_users && items[x] >= 0 &&
                            items[x] < h->n_items,
                        "event user/item id out of range");
        std::vector<int64_t> uoff, ioff;
        std::vector<int32_t> ucols, icols;
        build_csr(users, items, n, h->n_users, uoff, ucols);
        build_csr(items, users, n, h->n_items, ioff, icols);
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->uoff.alloc(uoff.size());
        h->ioff.alloc(ioff.size());
        h->ucols.alloc(std::max<size_t>(1, ucols.size()));
        h->icols.alloc(std::max<size_t>(1, icols.size()));
        MML_HIP(hipMemcpyAsync(h->uoff.get(), uoff.data(), sizeof(int64_t) * uoff.size(),
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(h->ioff.get(), ioff.data(), sizeof(int64_t) * ioff.size(),
                               hipMemcpyHostToDevice, st));
        if (!ucols.empty())
            MML_HIP(hipMemcpyAsync(h->ucols.get(), ucols.data(), sizeof(int32_t) * ucols.size(),
                                   hipMemcpyHostToDevice, st));
        if (!icols.empty())
            MML_HIP(hipMemcpyAsync(h->icols.get(), icols.data(), sizeof(int32_t) * icols.size(),
                                   hipMemcpyHostToDevice, st));
        MML_HIP(hipStreamSynchronize(st));
        std::vector<int64_t> udeg(h->n_users), ideg(h->n_items);
        for (int32_t r = 0; r < h->n_users; ++r) udeg[r] = uoff[r + 1] - uoff[r];
        for (int32_t r = 0; r < h->n_items; ++r) ideg[r] = ioff[r + 1] - ioff[r];
        set_degrees(h, std::move(udeg), std::move(ideg));
        h->has_data = true;
    });
}

extern "C" mml_status mml_wrmf_set_data_device(mml_wrmf* h, const int32_t* users,
                                               const int32_t* items, int64_t n) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        MML_REQUIRE(!h->ctx->multi(), "a multi-device context takes host arrays (set_data)");
        MML_REQUIRE(n >= 0 && (n == 0 || (users && items)), "bad event arrays");
        h->ctx->activate();
        // the arrays may come from any stream of the caller's (e.g. torch's): wait for the device
        MML_HIP(hipDeviceSynchronize());
        hipStream_t st = h->ctx->stream;
        h->has_data = false;
        mml::DeviceCsr ucsr, icsr;
        mml::build_csr_device(users, items, n, h->n_users, h->n_items, st, ucsr);
        mml::build_csr_device(items, users, n, h->n_items, h->n_users, st, icsr);
        h->uoff.swap(ucsr.off);
        h->ucols.swap(ucsr.cols);
        h->ioff.swap(icsr.off);
        h->icols.swap(icsr.cols);
        h->nnz = ucsr.nnz;
        set_degrees(h, std::vector<int64_t>(ucsr.deg_host.begin(), ucsr.deg_host.end()),
                    std::vector<int64_t>(icsr.deg_host.begin(), icsr.deg_host.end()));
        h->has_data = true;
    });
}

namespace {
__device__ __forceinline__ uint64_t wrmf_mix(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}
__global__ __launch_bounds__(256) void wrmf_init_normal_kernel(float* __restrict__ M, int64_t n,
                                                               uint64_t seed, double mean,
                                                               double stddev) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t x = wrmf_mix(seed ^ (uint64_t)e * 0x9E3779B97F4A7C15ull);
        const double u1 = ((x >> 11) + 1.0) * (1.0 / 9007199254740993.0);
        const double u2 = (double)(wrmf_mix(x) >> 11) * (1.0 / 9007199254740992.0);
        M[e] = (float)(mean + stddev * sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
    }
}
}  // namespace

extern "C" mml_status mml_wrmf_init_model(mml_wrmf* h, uint64_t seed, double mean,
                                          double stddev) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {
            mml::on_devices(h->ctx, [&](int32_t d) { return mml_wrmf_init_model(h->shards[d], seed, mean, stddev); });
            h->has_model = true;
            return;
        }
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        wrmf_init_normal_kernel<<<8192, 256, 0, st>>>(h->U.get(), (int64_t)h->n_users * h->k, seed,
                                                      mean, stddev);
        wrmf_init_normal_kernel<<<8192, 256, 0, st>>>(h->V.get(), (int64_t)h->n_items * h->k,
                                                      seed ^ 0x5DEECE66Dull, mean, stddev);
        MML_HIP(hipGetLastError());
        MML_HIP(hipStreamSynchronize(st));
        h->has_model = true;
    });
}

extern "C" mml_status mml_wrmf_set_model(mml_wrmf* h, const float* U, const float* V) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx && U && V, "null argument");
        if (h->ctx->multi()) {
            mml::on_devices(h->ctx, [&](int32_t d) { return mml_wrmf_set_model(h->shards[d], U, V); });
            h->has_model = true;
            return;
        }
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        MML_HIP(hipMemcpyAsync(h->U.get(), U, sizeof(float) * h->n_users * h->k,
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(h->V.get(), V, sizeof(float) * h->n_items * h->k,
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipStreamSynchronize(st));
        h->has_model = true;
    });
}

extern "C" mml_status mml_wrmf_get_model(mml_wrmf* h, float* U, float* V) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) return (void)mml::on_devices(h->ctx, [&](int32_t d) {
            return d == 0 ? mml_wrmf_get_model(h->shards[0], U, V) : (mml_status)MML_OK;
        });
        MML_REQUIRE(h->has_model, "no model");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        if (U)
            MML_HIP(hipMemcpyAsync(U, h->U.get(), sizeof(float) * h->n_users * h->k,
                                   hipMemcpyDeviceToHost, st));
        if (V)
            MML_HIP(hipMemcpyAsync(V, h->V.get(), sizeof(float) * h->n_items * h->k,
                                   hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_wrmf_iterate(mml_wrmf* h) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {  // every device solves its row shards; all-gathers inside
            std::vector<float> ms(h->shards.size(), 0.0f);
            // a repeated device: the shards are the ranks of a peer group (one thread each)
            mml::PeerGroup* g = h->shards[0]->ctx->peers.get();
            if (g) g->reset();
            mml::on_devices(h->ctx, [&](int32_t d) {
                const mml_status st = mml_wrmf_iterate(h->shards[d]);
                if (st != MML_OK && g) g->abort();  // the other ranks leave their barriers
                ms[d] = h->shards[d]->last_ms;
                return st;
            });
            h->last_ms = *std::max_element(ms.begin(), ms.end());
            h->last_launches = h->shards[0]->last_launches;
            h->last_refine = 0;
            for (mml_wrmf* s : h->shards) h->last_refine = std::max(h->last_refine, s->last_refine);
            return;
        }
        MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede iterate");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        int launches = 0;
        h->last_refine = 0;
        h->spec_valid = false;
        std::fill(h->last_corr, h->last_corr + 8, 0.0f);
        MML_HIP(hipEventRecord(h->ctx->ev_begin, st));
        ensure_shards(h);
        const int rk = h->shard_rank;
        // WRMF.Iterate (:68-73): users from items, then items from the updated users; with
        // several ranks each solves its row shard and the shards are all-gathered in between
        const bool gather = h->shard_nranks > 1;
        if (gather && !h->ev_g[0])
            for (hipEvent_t& e : h->ev_g) MML_HIP(hipEventCreate(&e));
        half_step(h, h->U.get(), h->ub[rk], h->ub[rk + 1], h->V.get(), h->n_items, h->uoff.get(),
                  h->ucols.get(), h->n_users, launches);
        if (gather) {
            MML_HIP(hipEventRecord(h->ev_g[0], st));
            allgather_rows(h, h->U.get(), h->ub);
            MML_HIP(hipEventRecord(h->ev_g[1], st));
        }
        half_step(h, h->V.get(), h->ib[rk], h->ib[rk + 1], h->U.get(), h->n_users, h->ioff.get(),
                  h->icols.get(), h->n_items, launches);
        if (gather) {
            MML_HIP(hipEventRecord(h->ev_g[2], st));
            allgather_rows(h, h->V.get(), h->ib);
            MML_HIP(hipEventRecord(h->ev_g[3], st));
        }
        MML_HIP(hipEventRecord(h->ctx->ev_end, st));
        MML_HIP(hipEventSynchronize(h->ctx->ev_end));
        MML_HIP(hipEventElapsedTime(&h->last_ms, h->ctx->ev_begin, h->ctx->ev_end));
        h->last_gather_ms = 0.0f;
        if (gather) {
            float a = 0.0f, b = 0.0f;
            MML_HIP(hipEventElapsedTime(&a, h->ev_g[0], h->ev_g[1]));
            MML_HIP(hipEventElapsedTime(&b, h->ev_g[2], h->ev_g[3]));
            h->last_gather_ms = a + b;
        }
        h->last_launches = launches;
    });
}

namespace {
__global__ __launch_bounds__(256) void wrmf_rows_scatter_kernel(const float* __restrict__ src,
                                                                const int32_t* __restrict__ rows,
                                                                int32_t n, int32_t k,
                                                                float* __restrict__ W) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < (int64_t)n * k;
         e += (int64_t)gridDim.x * blockDim.x)
        W[(int64_t)rows[e / k] * k + e % k] = src[e];
}
}  // namespace

extern "C" mml_status mml_wrmf_retrain(mml_wrmf* h, int32_t side, int32_t n_rows,
                                       const int32_t* rows, const int64_t* rated_off,
                                       const int32_t* rated_ids) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        MML_REQUIRE(!h->ctx->multi(), "RetrainUser / RetrainItem run on a single-device handle");
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(side == 0 || side == 1, "side: 0 (users) or 1 (items)");
        MML_REQUIRE(n_rows >= 0, "negative sizes");
        if (n_rows == 0) return;
        MML_REQUIRE(rows && rated_off, "null arguments");
        const int32_t n_own = side == 0 ? h->n_users : h->n_items;
        const int32_t n_oth = side == 0 ? h->n_items : h->n_users;
        std::vector<int32_t> sorted(rows, rows + n_rows);
        std::sort(sorted.begin(), sorted.end());
        for (int32_t x = 0; x < n_rows; ++x) {
            MML_REQUIRE(sorted[x] >= 0 && sorted[x] < n_own, "retrained row id beyond the model");
            MML_REQUIRE(x == 0 || sorted[x] != sorted[x - 1], "a row is listed twice");
        }
        MML_REQUIRE(rated_off[0] == 0, "rated_off[0] must be 0");
        std::vector<int64_t> deg(n_rows);
        for (int32_t x = 0; x < n_rows; ++x) {
            MML_REQUIRE(rated_off[x + 1] >= rated_off[x], "rated_off must be non-decreasing");
            deg[x] = rated_off[x + 1] - rated_off[x];
        }
        const int64_t nr = rated_off[n_rows];
        MML_REQUIRE(nr == 0 || rated_ids, "null rated ids");
        for (int64_t x = 0; x < nr; ++x)
            MML_REQUIRE(rated_ids[x] >= 0 && rated_ids[x] < n_oth, "rated id beyond the model");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        // the listed rows as a CSR of their own: one half-step over it solves them with the
        // iterate's kernels (HH recomputed from the fixed side, as RetrainUser's
        // ComputeSquareMatrix), then the solved rows go to their places
        mml::DeviceArray<int64_t> doff;
        mml::DeviceArray<int32_t> dids, drows;
        mml::DeviceArray<float> wsub;
        doff.alloc(n_rows + 1);
        dids.alloc(std::max<int64_t>(1, nr));
        drows.alloc(n_rows);
        wsub.alloc((size_t)n_rows * h->k);
        MML_HIP(hipMemcpyAsync(doff.get(), rated_off, sizeof(int64_t) * (n_rows + 1),
                               hipMemcpyHostToDevice, st));
        if (nr > 0)
            MML_HIP(hipMemcpyAsync(dids.get(), rated_ids, sizeof(int32_t) * nr,
                                   hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(drows.get(), rows, sizeof(int32_t) * n_rows, hipMemcpyHostToDevice,
                               st));
        float* W = side == 0 ? h->U.get() : h->V.get();
        const float* H = side == 0 ? h->V.get() : h->U.get();
        const int64_t h_rows = side == 0 ? h->n_items : h->n_users;
        mml::WrmfTilePlan plan;
        if (h->k > 128)
            mml::wrmf_tile_plan(deg, st, plan, 0, n_rows, h->p.alpha > 0.0 && !no_woodbury(),
                                h->pipe_req);
        int launches = 0;
        h->last_refine = 0;
        std::fill(h->last_corr, h->last_corr + 8, 0.0f);
        half_step(h, wsub.get(), 0, n_rows, H, h_rows, doff.get(), dids.get(), n_rows, launches,
                  &plan);
        wrmf_rows_scatter_kernel<<<(int)std::min<int64_t>(4096, ((int64_t)n_rows * h->k + 255) / 256),
                                   256, 0, st>>>(wsub.get(), drows.get(), n_rows, h->k, W);
        MML_HIP(hipGetLastError());
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_wrmf_last_allgather_ms(mml_wrmf* h, float* out) {
    return guard([&] {
        MML_REQUIRE(h && out, "null argument");
        *out = h->last_gather_ms;
        for (mml_wrmf* s : h->shards) *out = std::max(*out, s->last_gather_ms);
    });
}

extern "C" mml_status mml_wrmf_set_pipeline(mml_wrmf* h, int32_t ranges) {
    return guard([&] {
        MML_REQUIRE(h, "null argument");
        MML_REQUIRE(ranges >= 0 && ranges <= 16, "pipeline ranges: 0 (default), 1 (off) .. 16");
        h->pipe_req = ranges;
        h->shard_nranks = 0;  // the row plans are rebuilt at the next iterate
        h->shard_rank = -1;
        for (mml_wrmf* s : h->shards) {
            s->pipe_req = ranges;
            s->shard_nranks = 0;
            s->shard_rank = -1;
        }
    });
}

extern "C" mml_status mml_wrmf_last_timing(mml_wrmf* h, float* out) {
    return guard([&] {
        MML_REQUIRE(h && out, "null argument");
        out[0] = h->last_ms;
        out[1] = (float)h->last_launches;
    });
}

extern "C" mml_status mml_wrmf_last_refine_passes(mml_wrmf* h, int32_t* out,
                                                  float* corrections) {
    return guard([&] {
        MML_REQUIRE(h && out, "null argument");
        *out = h->last_refine;
        if (corrections) std::copy(h->last_corr, h->last_corr + 8, corrections);
    });
}

extern "C" mml_status mml_wrmf_predict(mml_wrmf* h, const int32_t* users, const int32_t* items,
                                       int64_t n, float* out) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) return (void)mml::on_devices(h->ctx, [&](int32_t d) {
            return d == 0 ? mml_wrmf_predict(h->shards[0], users, items, n, out)
                          : (mml_status)MML_OK;
        });
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(n >= 0 && (n == 0 || (users && items && out)), "bad arguments");
        if (n == 0) return;
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->q_u.alloc(n);
        h->q_i.alloc(n);
        h->q_out.alloc(n);
        MML_HIP(hipMemcpyAsync(h->q_u.get(), users, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                               st));
        MML_HIP(hipMemcpyAsync(h->q_i.get(), items, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                               st));
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
        wrmf_predict_kernel<<<grid, 256, 0, st>>>(h->q_u.get(), h->q_i.get(), n, h->n_users,
                                                  h->n_items, h->U.get(), h->V.get(), h->k,
                                                  h->q_out.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemcpyAsync(out, h->q_out.get(), sizeof(float) * n, hipMemcpyDeviceToHost,
                               st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_wrmf_auc(mml_wrmf* h, const int32_t* candidates, int32_t n_candidates,
                                   const int32_t* users, int32_t n_users, const int64_t* test_off,
                                   const int32_t* test_items, double* out_auc) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) return (void)mml::on_devices(h->ctx, [&](int32_t d) {
            return d == 0 ? mml_wrmf_auc(h->shards[0], candidates, n_candidates, users, n_users,
                                         test_off, test_items, out_auc)
                          : (mml_status)MML_OK;
        });
        MML_REQUIRE(h->has_model && h->has_data, "model and training data required");
        h->ctx->activate();
        mml::item_auc(h->ctx->stream, h->U.get(), h->k, h->n_users, h->V.get(), h->k, h->n_items,
                      nullptr, h->k, h->uoff.get(), h->ucols.get(), h->n_users, candidates,
                      n_candidates, users, n_users, test_off, test_items, out_auc);
    });
}
