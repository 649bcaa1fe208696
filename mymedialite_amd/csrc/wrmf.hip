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
// This round covers k <= 64 (A in LDS as double: 32 KiB); k = 256 (C5) needs the register-tiled
// MFMA path described in DESIGN.md.
#include <algorithm>
#include <vector>

#include "mml_internal.h"

namespace {

constexpr int kMaxK = 64;
constexpr int kChunk = 32;  // item rows staged in LDS per pass

// Partial H^T H over a slice of rows: each thread owns entries e = t, t + 256, ... of the k x k
// matrix (only f1 <= f2 are used later), rows are staged through LDS kChunk at a time.
__global__ __launch_bounds__(256) void wrmf_gram_partial_kernel(const float* __restrict__ H,
                                                                int64_t rows, int32_t k,
                                                                int64_t rows_per_block,
                                                                double* __restrict__ partial) {
    __shared__ float hs[kChunk][kMaxK];
    const int t = threadIdx.x;
    const int kk = k * k;
    double acc[kMaxK * kMaxK / 256];
    for (int x = 0; x < kMaxK * kMaxK / 256; ++x) acc[x] = 0.0;
    const int64_t r0 = (int64_t)blockIdx.x * rows_per_block;
    const int64_t r1 = min(rows, r0 + rows_per_block);
    for (int64_t base = r0; base < r1; base += kChunk) {
        const int nr = (int)min((int64_t)kChunk, r1 - base);
        __syncthreads();
        for (int e = t; e < nr * k; e += 256) hs[e / k][e % k] = H[(base + e / k) * k + e % k];
        __syncthreads();
        for (int x = 0; x < kMaxK * kMaxK / 256; ++x) {
            const int e = t + 256 * x;
            if (e >= kk) break;
            const int f1 = e / k, f2 = e % k;
            double a = acc[x];
            for (int c = 0; c < nr; ++c) a += (double)(hs[c][f1] * hs[c][f2]);
            acc[x] = a;
        }
    }
    for (int x = 0; x < kMaxK * kMaxK / 256; ++x) {
        const int e = t + 256 * x;
        if (e < kk) partial[(int64_t)blockIdx.x * kk + e] = acc[x];
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
    const int src = f1 <= f2 ? e : f2 * k + f1;
    double s = 0.0;
    for (int p = 0; p < nparts; ++p) s += partial[(int64_t)p * kk + src];
    HH[e] = s;
}

// One workgroup per row of W.
__global__ __launch_bounds__(256) void wrmf_solve_kernel(
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols, int64_t n_data_rows,
    int64_t n_rows, float* __restrict__ W, const float* __restrict__ H,
    const double* __restrict__ HH, int32_t k, double alpha, double reg) {
    __shared__ double A[kMaxK][kMaxK + 1];
    __shared__ double bv[kMaxK];
    __shared__ float hs[kChunk][kMaxK];
    __shared__ int32_t idx[kChunk];
    const int t = threadIdx.x;
    const int kk = k * k;
    for (int64_t row = blockIdx.x; row < n_rows; row += gridDim.x) {
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
    int32_t last_launches = 0;
};

namespace {

void half_step(mml_wrmf* h, float* W, int64_t w_rows, const float* H, int64_t h_rows,
               const int64_t* off, const int32_t* cols, int64_t n_data_rows, int& launches) {
    hipStream_t st = h->ctx->stream;
    const int k = h->k;
    const int nparts = (int)std::max<int64_t>(1, std::min<int64_t>(1024, (h_rows + 255) / 256));
    const int64_t rpb = (h_rows + nparts - 1) / nparts;
    wrmf_gram_partial_kernel<<<nparts, 256, 0, st>>>(H, h_rows, k, rpb, h->partial.get());
    wrmf_gram_reduce_kernel<<<(k * k + 255) / 256, 256, 0, st>>>(h->partial.get(), nparts, k,
                                                                  h->HH.get());
    const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(w_rows, 256 * 16));
    wrmf_solve_kernel<<<grid, 256, 0, st>>>(off, cols, n_data_rows, w_rows, W, H, h->HH.get(), k,
                                            h->p.alpha, h->p.regularization);
    MML_HIP(hipGetLastError());
    launches += 3;
}

}  // namespace

using mml::guard;

extern "C" mml_status mml_wrmf_create(mml_ctx* ctx, const mml_wrmf_params* params,
                                      int32_t n_users, int32_t n_items, mml_wrmf** out) {
    return guard([&] {
        MML_REQUIRE(ctx && params && out, "null argument");
        MML_REQUIRE(n_users >= 1 && n_items >= 1, "need >= 1 user and item");
        MML_REQUIRE(params->num_factors >= 1 && params->num_factors <= kMaxK,
                    "num_factors must be in [1, 64] on this build");
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
            h->partial.alloc((size_t)1024 * h->k * h->k);
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
        (void)hipSetDevice(h->ctx->device);
        (void)hipStreamSynchronize(h->ctx->stream);
        delete h;
    });
}

extern "C" mml_status mml_wrmf_set_data(mml_wrmf* h, const int32_t* users, const int32_t* items,
                                        int64_t n) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
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
        h->has_data = true;
    });
}

extern "C" mml_status mml_wrmf_set_model(mml_wrmf* h, const float* U, const float* V) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx && U && V, "null argument");
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
        MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede iterate");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        int launches = 0;
        MML_HIP(hipEventRecord(h->ctx->ev_begin, st));
        // WRMF.Iterate (:68-73): users from items, then items from the updated users
        half_step(h, h->U.get(), h->n_users, h->V.get(), h->n_items, h->uoff.get(),
                  h->ucols.get(), h->n_users, launches);
        half_step(h, h->V.get(), h->n_items, h->U.get(), h->n_users, h->ioff.get(),
                  h->icols.get(), h->n_items, launches);
        MML_HIP(hipEventRecord(h->ctx->ev_end, st));
        MML_HIP(hipEventSynchronize(h->ctx->ev_end));
        MML_HIP(hipEventElapsedTime(&h->last_ms, h->ctx->ev_begin, h->ctx->ev_end));
        h->last_launches = launches;
    });
}

extern "C" mml_status mml_wrmf_last_timing(mml_wrmf* h, float* out) {
    return guard([&] {
        MML_REQUIRE(h && out, "null argument");
        out[0] = h->last_ms;
        out[1] = (float)h->last_launches;
    });
}

extern "C" mml_status mml_wrmf_predict(mml_wrmf* h, const int32_t* users, const int32_t* items,
                                       int64_t n, float* out) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
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
