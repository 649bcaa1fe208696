// auc.hip -- item-ranking AUC on the GPU for the MF scorers (BPRMF, WRMF).
//
// Replaces Eval.Items.Evaluate restricted to AUC (src/MyMediaLite/Eval/Items.cs:126-209) with
// Recommender.Recommend(n = -1) (src/MyMediaLite/Recommender.cs:52-103) and AUC.Compute
// (src/MyMediaLite/Eval/Measures/AUC.cs:42-68).  For a test user u the reference scores every
// candidate that is not one of u's training items, sorts descending (stable: ties keep candidate
// order) and counts, for every non-relevant item, the relevant items ranked above it.  Equivalently,
// for every relevant item r in the list: below(r) = #{non-relevant listed c ranked after r}, where
// c is after r iff s_c < s_r, or s_c == s_r and pos_c > pos_r.  No sort is needed:
//   1. prep (one thread per user): R' = relevant items in the list with exact scores (float, left to
//      right like RowScalarProduct), and sub[r] = #{ignored candidates or other relevant items that
//      rank after r} -- the few items the full scan must not count;
//   2. scan: workgroup (64 users, slice of candidates) scores all 64 x 128 pairs of an LDS tile
//      with the same exact float arithmetic (4 x 8 register patch per thread), compares against the
//      users' relevant scores and adds the counts (LDS, then one global atomic per pair per slice);
//   3. host: AUC from (below_all - sub, |R'|, list size, dropped) exactly as AUC.Compute.
// The scan is O(users x candidates x k) flops, the dominant term; candidate rows stream through
// LDS once per 64 users.
#include <algorithm>
#include <cmath>
#include <vector>

#include "mml_internal.h"

namespace {

constexpr int kUB = 64;    // users per workgroup
constexpr int kIT = 128;   // candidates per LDS tile
constexpr int kMaxR = 64;  // relevant items per user per pass

__device__ __forceinline__ float exact_score(const float* __restrict__ U, const float* __restrict__ V,
                                             const float* __restrict__ bias, int32_t u, int32_t i,
                                             int32_t k, int32_t ldu, int32_t ldv) {
    const float* a = U + (int64_t)u * ldu;
    const float* c = V + (int64_t)i * ldv;
    float dot = 0.0f;
    for (int f = 0; f < k; ++f) dot += a[f] * c[f];
    return bias ? bias[i] + dot : dot;
}

__device__ __forceinline__ bool beats(float sr, int32_t pr, float sc, int32_t pc) {
    return sc < sr || (sc == sr && pc > pr);  // c ranked after r
}

// binary search of item in a sorted CSR row [b, e)
__device__ __forceinline__ bool in_row(const int32_t* __restrict__ cols, int64_t b, int64_t e,
                                       int32_t item) {
    int64_t lo = b, hi = e;
    while (lo < hi) {
        const int64_t m = (lo + hi) >> 1;
        if (cols[m] < item) lo = m + 1;
        else hi = m;
    }
    return lo < e && cols[lo] == item;
}

// prep: one thread per eval user.  Writes rel_pos/rel_score (pass slots), n_rel_total, sub counts.
__global__ __launch_bounds__(64) void auc_prep_kernel(
    const int32_t* __restrict__ users, int32_t n_eval, const int64_t* __restrict__ te_off,
    const int32_t* __restrict__ te_items, const int64_t* __restrict__ tr_off,
    const int32_t* __restrict__ tr_cols, int32_t n_tr_rows, const int32_t* __restrict__ cand_pos,
    int32_t n_pos_items, const int32_t* __restrict__ candidates, const float* __restrict__ U,
    const float* __restrict__ V, const float* __restrict__ bias, int32_t k, int32_t ldu,
    int32_t ldv, int32_t n_users_model, int32_t n_items_model, int32_t pass,
    int32_t* __restrict__ rel_pos, float* __restrict__ rel_score, int32_t* __restrict__ stats,
    int32_t* __restrict__ sub) {
    const int x = blockIdx.x * blockDim.x + threadIdx.x;
    if (x >= n_eval) return;
    const int32_t u = users[x];
    const bool u_in = u >= 0 && u < n_users_model;
    const int64_t tb = (u >= 0 && u < n_tr_rows) ? tr_off[u] : 0;
    const int64_t tr_end = (u >= 0 && u < n_tr_rows) ? tr_off[u + 1] : 0;
    int n_correct = 0, n_rel = 0, n_ignored = 0;
    // relevant = test items in candidates; in the list = in model and not a training item
    for (int64_t a = te_off[x]; a < te_off[x + 1]; ++a) {
        const int32_t it = te_items[a];
        if (it < 0 || it >= n_pos_items || cand_pos[it] < 0) continue;
        ++n_correct;
        if (!u_in || it >= n_items_model || in_row(tr_cols, tb, tr_end, it)) continue;
        if (n_rel >= pass * kMaxR && n_rel < (pass + 1) * kMaxR) {
            const int slot = n_rel - pass * kMaxR;
            rel_pos[x * kMaxR + slot] = cand_pos[it];
            rel_score[x * kMaxR + slot] = exact_score(U, V, bias, u, it, k, ldu, ldv);
        }
        ++n_rel;
    }
    for (int64_t a = tb; a < tr_end; ++a) {
        const int32_t it = tr_cols[a];
        if (it >= 0 && it < n_pos_items && cand_pos[it] >= 0) ++n_ignored;
    }
    stats[x * 4 + 0] = n_correct;
    stats[x * 4 + 1] = n_rel;
    stats[x * 4 + 2] = n_ignored;
    // sub[r]: ignored candidates and other relevant items that rank after r (in-model only)
    const int lo = pass * kMaxR, hi = min(n_rel, (pass + 1) * kMaxR);
    for (int r = lo; r < hi; ++r) {
        const int slot = r - lo;
        const float sr = rel_score[x * kMaxR + slot];
        const int32_t pr = rel_pos[x * kMaxR + slot];
        int cnt = 0;
        if (u_in)
            for (int64_t a = tb; a < tr_end; ++a) {
                const int32_t it = tr_cols[a];
                if (it < 0 || it >= n_pos_items || cand_pos[it] < 0 || it >= n_items_model) continue;
                if (beats(sr, pr, exact_score(U, V, bias, u, it, k, ldu, ldv), cand_pos[it])) ++cnt;
            }
        // other relevant items (all passes): recompute their scores
        for (int64_t a = te_off[x]; a < te_off[x + 1]; ++a) {
            const int32_t it = te_items[a];
            if (it < 0 || it >= n_pos_items || cand_pos[it] < 0) continue;
            if (!u_in || it >= n_items_model || in_row(tr_cols, tb, tr_end, it)) continue;
            if (cand_pos[it] == pr) continue;
            if (beats(sr, pr, exact_score(U, V, bias, u, it, k, ldu, ldv), cand_pos[it])) ++cnt;
        }
        sub[x * kMaxR + slot] = cnt;
    }
}

// scan: grid (ceil(n_eval / 64), slices); tile of 128 candidates x 64 users, the factor dimension
// staged 64 at a time (LDS independent of k); thread patch 4 users x 8 candidates (users
// 4*(t/16).., candidates 8*(t%16)..).  dot accumulates f = 0..k-1 in order: RowScalarProduct.
constexpr int kKC = 64;
__global__ __launch_bounds__(256) void auc_scan_kernel(
    const int32_t* __restrict__ users, int32_t n_eval, const int32_t* __restrict__ candidates,
    int32_t n_cand, int64_t per_slice, const float* __restrict__ U, const float* __restrict__ V,
    const float* __restrict__ bias, int32_t k, int32_t ldu, int32_t ldv, int32_t n_users_model,
    int32_t n_items_model, const int32_t* __restrict__ rel_pos, const float* __restrict__ rel_score,
    const int32_t* __restrict__ stats, int32_t pass, unsigned long long* __restrict__ below) {
    __shared__ float su[kUB][kKC + 1];
    __shared__ float sv[kIT][kKC + 1];
    __shared__ float sb[kIT];
    __shared__ int32_t spos[kIT];
    __shared__ float rs[kUB * kMaxR];
    __shared__ int32_t rp[kUB * kMaxR];
    __shared__ int32_t cnt[kUB * kMaxR];
    __shared__ int32_t nr[kUB];
    __shared__ int32_t urow[kUB];
    const int t = threadIdx.x;
    const int ub = blockIdx.x * kUB;
    for (int e = t; e < kUB * kMaxR; e += 256) {
        const int x = e / kMaxR;
        rs[e] = ub + x < n_eval ? rel_score[(int64_t)(ub + x) * kMaxR + e % kMaxR] : 0.0f;
        rp[e] = ub + x < n_eval ? rel_pos[(int64_t)(ub + x) * kMaxR + e % kMaxR] : 0;
        cnt[e] = 0;
    }
    for (int x = t; x < kUB; x += 256) {
        const int ux = ub + x;
        int n = 0, ur = -1;
        if (ux < n_eval) {
            const int32_t u = users[ux];
            if (u >= 0 && u < n_users_model) {
                n = min(kMaxR, max(0, stats[ux * 4 + 1] - pass * kMaxR));
                ur = u;
            }
        }
        nr[x] = n;
        urow[x] = ur;
    }
    const int64_t c0 = (int64_t)blockIdx.y * per_slice;
    const int64_t c1 = min((int64_t)n_cand, c0 + per_slice);
    const int pu = (t / 16) * 4, pc = (t % 16) * 8;
    for (int64_t base = c0; base < c1; base += kIT) {
        __syncthreads();
        for (int c = t; c < kIT; c += 256) {
            const int64_t ci = base + c;
            const int32_t it = ci < c1 ? candidates[ci] : -1;
            const bool ok = it >= 0 && it < n_items_model;
            sb[c] = (ok && bias) ? bias[it] : 0.0f;
            spos[c] = ok ? (int32_t)ci : -1;
        }
        float dot[4][8];
#pragma unroll
        for (int a = 0; a < 4; ++a)
#pragma unroll
            for (int b = 0; b < 8; ++b) dot[a][b] = 0.0f;
        for (int f0 = 0; f0 < k; f0 += kKC) {
            const int kc = min(kKC, k - f0);
            __syncthreads();
            for (int e = t; e < kUB * kKC; e += 256) {
                const int x = e / kKC, f = e % kKC;
                su[x][f] = (urow[x] >= 0 && f < kc) ? U[(int64_t)urow[x] * ldu + f0 + f] : 0.0f;
            }
            for (int e = t; e < kIT * kKC; e += 256) {
                const int c = e / kKC, f = e % kKC;
                const int64_t ci = base + c;
                const int32_t it = ci < c1 ? candidates[ci] : -1;
                sv[c][f] = (it >= 0 && it < n_items_model && f < kc)
                               ? V[(int64_t)it * ldv + f0 + f] : 0.0f;
            }
            __syncthreads();
            for (int f = 0; f < kc; ++f) {
                float ua[4], vb[8];
#pragma unroll
                for (int a = 0; a < 4; ++a) ua[a] = su[pu + a][f];
#pragma unroll
                for (int b = 0; b < 8; ++b) vb[b] = sv[pc + b][f];
#pragma unroll
                for (int a = 0; a < 4; ++a)
#pragma unroll
                    for (int b = 0; b < 8; ++b) dot[a][b] += ua[a] * vb[b];
            }
        }
#pragma unroll
        for (int a = 0; a < 4; ++a) {
            const int x = pu + a;
            const int n = nr[x];
            for (int r = 0; r < n; ++r) {
                const float sr = rs[x * kMaxR + r];
                const int32_t prr = rp[x * kMaxR + r];
                int c = 0;
#pragma unroll
                for (int b = 0; b < 8; ++b) {
                    const int32_t pcand = spos[pc + b];
                    const float s = bias ? sb[pc + b] + dot[a][b] : dot[a][b];
                    c += (pcand >= 0 && beats(sr, prr, s, pcand)) ? 1 : 0;
                }
                if (c) atomicAdd(&cnt[x * kMaxR + r], c);
            }
        }
    }
    __syncthreads();
    for (int e = t; e < kUB * kMaxR; e += 256) {
        const int x = e / kMaxR;
        if (ub + x < n_eval && (e % kMaxR) < nr[x] && cnt[e])
            atomicAdd(&below[(int64_t)(ub + x) * kMaxR + e % kMaxR], (unsigned long long)cnt[e]);
    }
}

__global__ void scatter_pos_kernel(const int32_t* __restrict__ candidates, int32_t n,
                                   int32_t* __restrict__ cand_pos) {
    for (int x = blockIdx.x * blockDim.x + threadIdx.x; x < n; x += gridDim.x * blockDim.x)
        cand_pos[candidates[x]] = x;
}

}  // namespace

namespace mml {

// Shared by mml_bpr_auc / mml_wrmf_auc.  U, V (leading dims ldu, ldv), bias (nullable) and the
// training CSR are device pointers of the handle; everything else is host input.
void item_auc(hipStream_t st, const float* U, int32_t ldu, int32_t n_users_model, const float* V,
              int32_t ldv, int32_t n_items_model, const float* bias, int32_t k,
              const int64_t* tr_off, const int32_t* tr_cols, int32_t n_tr_rows,
              const int32_t* candidates, int32_t n_cand, const int32_t* users, int32_t n_eval,
              const int64_t* test_off, const int32_t* test_items, double* out_auc) {
    MML_REQUIRE(n_cand >= 1 && candidates && n_eval >= 1 && users && test_off && test_items &&
                    out_auc,
                "bad AUC arguments");
    MML_REQUIRE(k >= 1 && k <= 256, "k out of range for the AUC scan");
    int32_t max_id = 0;
    {
        std::vector<char> seen;
        for (int32_t x = 0; x < n_cand; ++x) {
            MML_REQUIRE(candidates[x] >= 0, "negative candidate id");
            max_id = std::max(max_id, candidates[x]);
        }
        seen.assign((size_t)max_id + 1, 0);
        for (int32_t x = 0; x < n_cand; ++x) {
            MML_REQUIRE(!seen[candidates[x]], "duplicate candidate id");
            seen[candidates[x]] = 1;
        }
    }
    const int32_t n_pos = max_id + 1;
    const int64_t n_test = test_off[n_eval];
    MML_REQUIRE(test_off[0] == 0 && n_test >= 0, "bad test offsets");
    int32_t out_of_model = 0;
    for (int32_t x = 0; x < n_cand; ++x) out_of_model += candidates[x] >= n_items_model;
    DeviceArray<int32_t> dcand, dpos, dusers, dte, drelpos, dstats, dsub;
    DeviceArray<int64_t> dteoff;
    DeviceArray<float> drelscore;
    DeviceArray<unsigned long long> dbelow;
    dcand.alloc(n_cand);
    dpos.alloc(n_pos);
    dusers.alloc(n_eval);
    dteoff.alloc(n_eval + 1);
    dte.alloc(std::max<int64_t>(1, n_test));
    drelpos.alloc((size_t)n_eval * kMaxR);
    drelscore.alloc((size_t)n_eval * kMaxR);
    dstats.alloc((size_t)n_eval * 4);
    dsub.alloc((size_t)n_eval * kMaxR);
    dbelow.alloc((size_t)n_eval * kMaxR);
    MML_HIP(hipMemcpyAsync(dcand.get(), candidates, sizeof(int32_t) * n_cand, hipMemcpyHostToDevice, st));
    MML_HIP(hipMemsetAsync(dpos.get(), 0xff, sizeof(int32_t) * n_pos, st));
    MML_HIP(hipMemcpyAsync(dusers.get(), users, sizeof(int32_t) * n_eval, hipMemcpyHostToDevice, st));
    MML_HIP(hipMemcpyAsync(dteoff.get(), test_off, sizeof(int64_t) * (n_eval + 1),
                           hipMemcpyHostToDevice, st));
    if (n_test)
        MML_HIP(hipMemcpyAsync(dte.get(), test_items, sizeof(int32_t) * n_test,
                               hipMemcpyHostToDevice, st));
    scatter_pos_kernel<<<std::min(8192, (n_cand + 255) / 256), 256, 0, st>>>(dcand.get(), n_cand,
                                                                             dpos.get());
    MML_HIP(hipGetLastError());
    std::vector<int32_t> stats((size_t)n_eval * 4), sub((size_t)n_eval * kMaxR);
    std::vector<unsigned long long> below((size_t)n_eval * kMaxR);
    std::vector<double> correct_pairs(n_eval, 0.0);
    const int64_t slices = std::max<int64_t>(1, std::min<int64_t>(64, n_cand / 8192));
    const int64_t per_slice = ((n_cand + slices - 1) / slices + kIT - 1) / kIT * kIT;
    for (int pass = 0;; ++pass) {
        auc_prep_kernel<<<(n_eval + 63) / 64, 64, 0, st>>>(
            dusers.get(), n_eval, dteoff.get(), dte.get(), tr_off, tr_cols, n_tr_rows, dpos.get(),
            n_pos, dcand.get(), U, V, bias, k, ldu, ldv, n_users_model, n_items_model, pass,
            drelpos.get(), drelscore.get(), dstats.get(), dsub.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemsetAsync(dbelow.get(), 0, sizeof(unsigned long long) * n_eval * kMaxR, st));
        auc_scan_kernel<<<dim3((n_eval + kUB - 1) / kUB, (unsigned)slices), 256, 0, st>>>(
            dusers.get(), n_eval, dcand.get(), n_cand, per_slice, U, V, bias, k, ldu, ldv,
            n_users_model, n_items_model, drelpos.get(), drelscore.get(), dstats.get(), pass,
            dbelow.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemcpyAsync(stats.data(), dstats.get(), sizeof(int32_t) * stats.size(),
                               hipMemcpyDeviceToHost, st));
        MML_HIP(hipMemcpyAsync(sub.data(), dsub.get(), sizeof(int32_t) * sub.size(),
                               hipMemcpyDeviceToHost, st));
        MML_HIP(hipMemcpyAsync(below.data(), dbelow.get(), sizeof(unsigned long long) * below.size(),
                               hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        int32_t max_rel = 0;
        for (int32_t x = 0; x < n_eval; ++x) {
            const int n_rel = stats[x * 4 + 1];
            max_rel = std::max(max_rel, n_rel);
            const int lo = pass * kMaxR, hi = std::min(n_rel, (pass + 1) * kMaxR);
            for (int r = lo; r < hi; ++r)
                correct_pairs[x] += (double)(below[(size_t)x * kMaxR + (r - lo)] -
                                             (unsigned long long)sub[(size_t)x * kMaxR + (r - lo)]);
        }
        if ((pass + 1) * kMaxR >= max_rel) break;
    }
    // AUC.Compute per user (AUC.cs:42-68) with the list = candidates minus the user's training items
    for (int32_t x = 0; x < n_eval; ++x) {
        const int n_correct = stats[x * 4 + 0], n_rel = stats[x * 4 + 1];
        const int n_ignored = stats[x * 4 + 2];
        const int32_t u = users[x];
        const int64_t n_user_cand = (int64_t)n_cand - n_ignored;
        // Items.Evaluate skips users with no relevant candidate, or only relevant ones (:152-162)
        if (n_correct == 0 || n_correct == n_user_cand) {
            out_auc[x] = std::nan("");
            continue;
        }
        const bool u_in = u >= 0 && u < n_users_model;
        const int64_t listed = u_in ? (n_user_cand - out_of_model) : 0;  // Predict > MinValue
        const int64_t dropped = n_user_cand - listed;
        const int64_t eval_items = listed + dropped;
        const int64_t pairs = (eval_items - n_rel) * (int64_t)n_rel;
        if (pairs == 0) {
            out_auc[x] = 0.5;
            continue;
        }
        const int64_t missing = n_correct - n_rel;
        const double cp = correct_pairs[x] + (double)n_rel * (double)(dropped - missing);
        out_auc[x] = cp / (double)pairs;
    }
}

}  // namespace mml
