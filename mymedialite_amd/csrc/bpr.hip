// bpr.hip -- BPRMF pairwise SGD on MI355X (gfx950).
//
// Replaces BPRMF.Iterate() with its default sampler IterateWithoutReplacementUniformUser
// (src/MyMediaLite/ItemRecommendation/BPRMF.cs:160-226), the triple samplers SampleUser /
// SampleItemPair / SampleOtherItem (:275-321), UpdateFactors (:330-374) and Predict (:425-431).
//
// HBM layout (per mml_bpr handle):
//   U [n_users x ld], V [n_items x ld]  fp32 row-major, ld = 4 * LPR (zero padded)
//   bias [n_items]                      item biases
//   off [n_users + 1] (int64), cols     user -> positive items, CSR, each row sorted and
//                                       de-duplicated (the SparseBooleanMatrix sets)
//   eligible [n_eligible]               users with 0 < |S_u| < n_items (SampleUser's acceptance set)
//   ev_u, ev_i                          the events in visit order (UNIFORM_PAIR sampler only)
//
// Sampling is counter-based (splitmix64 of seed, sample index, draw index): sample s of an epoch is
// a pure function of (seed, s), independent of which wave draws it.  The reference draws from one
// sequential System.Random stream (variable draws per sample, HashSet insertion order for
// ElementAt), which cannot be parallelised bit-exactly; the distribution is the same:
//   u ~ Uniform(eligible)      == SampleUser's rejection loop
//   i ~ Uniform(S_u)           == user_items.ElementAt(random.Next(|S_u|))
//   j ~ Uniform(I \ S_u)       == SampleItemPair / SampleOtherItem's rejection loop
// Parity is therefore statistical (AUC, tests/test_bpr_gpu.py).
//
// The WithReplacement = true samplers (:183-211, :231-243; MML_BPR_SAMPLER_*_REPLACEMENT):
//   PAIR_REPLACEMENT  (u, i) = the event at a uniform index, j as above
//   USER_REPLACEMENT  u as above; i = the next item of the user's current round: the reference
//                     removes each drawn item from an epoch-local copy of S_u and refills the copy
//                     once it is empty, so a user's k-th sample of the epoch takes position k mod
//                     |S_u| of round floor(k / |S_u|), each round a fresh keyed permutation of S_u.
//                     k (the sample's rank among its user's samples, in sample order) comes from a
//                     stable radix sort of (u << 32 | s).
//
// Update (Hogwild!, LPR lanes per triple, one float4 per lane of U_u, V_i, V_j): the reference's
// float/double arithmetic -- x_uij = (b_i - b_j) + sum_f (double)(w_f * (h_if - h_jf)), double
// sigmoid, double deltas, float stores -- with the f-sum as per-lane partials + xor butterfly.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset on the host
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdlib>
#include <string>
#include <vector>

#include "mml_device.h"
#include "mml_internal.h"

namespace {

struct BprScalars {
    float lr, reg_u, reg_i, reg_j, bias_reg;
    int32_t update_j;
};

// UpdateFactors after x_uij: BPRMF.UpdateFactors (BPRMF.cs:330-374) or, SOFT,
// SoftMarginRankingMF.UpdateFactors (SoftMarginRankingMF.cs:66-113), whose update expressions are
// float arithmetic (float operands, the int literal 1) widened to double for the learn-rate step
// and which skips the triple when x_uij > 0.
template <bool SOFT>
struct TripleStep {
    double e = 0.0, lr;
    bool skip = false;
    __device__ __forceinline__ TripleStep(const BprScalars& s, double x_uij) : lr(s.lr) {
        if constexpr (SOFT) skip = x_uij > 0;
        else e = 1.0 / (1.0 + exp(x_uij));
    }
    __device__ __forceinline__ float bias_i(const BprScalars& s, float bi) const {
        if constexpr (SOFT) return bi + (float)(lr * (double)(1.0f - s.bias_reg * bi));
        else return bi + (float)(lr * (e - (double)(s.bias_reg * bi)));
    }
    __device__ __forceinline__ float bias_j(const BprScalars& s, float bj) const {
        if constexpr (SOFT) return bj + (float)(lr * (double)(-1.0f - s.bias_reg * bj));
        else return bj + (float)(lr * (-e - (double)(s.bias_reg * bj)));
    }
    __device__ __forceinline__ float u(const BprScalars& s, float wf, float hif, float hjf) const {
        if constexpr (SOFT) return (float)((double)wf + lr * (double)(hif - hjf - s.reg_u * wf));
        else return (float)((double)wf + lr * ((double)(hif - hjf) * e - (double)(s.reg_u * wf)));
    }
    __device__ __forceinline__ float i(const BprScalars& s, float wf, float hif) const {
        if constexpr (SOFT) return (float)((double)hif + lr * (double)(wf - s.reg_i * hif));
        else return (float)((double)hif + lr * ((double)wf * e - (double)(s.reg_i * hif)));
    }
    __device__ __forceinline__ float j(const BprScalars& s, float wf, float hjf) const {
        if constexpr (SOFT) return (float)((double)hjf + lr * (double)(-wf - s.reg_j * hjf));
        else return (float)((double)hjf + lr * ((double)(-wf) * e - (double)(s.reg_j * hjf)));
    }
};

__device__ __forceinline__ uint64_t splitmix64(uint64_t x) {
    x += 0x9E3779B97F4A7C15ull;
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return x ^ (x >> 31);
}

// uniform integer in [0, n) from draw d of sample s (Lemire multiply-shift on 32 high bits)
__device__ __forceinline__ uint32_t draw(uint64_t seed, uint64_t s, uint32_t d, uint32_t n) {
    const uint64_t x = splitmix64(seed ^ (s * 0xD1B54A32D192ED03ull + d));
    return (uint32_t)(((x >> 32) * (uint64_t)n) >> 32);
}

// A keyed bijection of [0, n): three rounds of xor / odd multiply / xorshift on the next power of
// two, cycle-walked back into [0, n) (the walk from x < n stays on x's cycle, < 2 steps expected).
__device__ __forceinline__ uint32_t keyed_perm(uint32_t x, uint32_t n, uint64_t key) {
    if (n <= 1) return 0;
    const int b = 32 - __clz(n - 1);
    const uint32_t mask = b >= 32 ? 0xffffffffu : ((1u << b) - 1u);
    const int sh = b > 1 ? b / 2 : 1;
    const uint64_t k1 = splitmix64(key), k2 = splitmix64(k1), k3 = splitmix64(k2);
    auto rounds = [&](uint32_t v) {
        v = ((v ^ (uint32_t)k1) * ((uint32_t)(k1 >> 32) | 1u)) & mask;
        v ^= v >> sh;
        v = ((v ^ (uint32_t)k2) * ((uint32_t)(k2 >> 32) | 1u)) & mask;
        v ^= v >> sh;
        v = ((v ^ (uint32_t)k3) * ((uint32_t)(k3 >> 32) | 1u)) & mask;
        v ^= v >> sh;
        return v;
    };
    uint32_t y = rounds(x);
    while (y >= n) y = rounds(y);
    return y;
}

// is item j in the sorted row [b, e)?  The LPR lanes of a group test a window of LPR entries per
// round (one coalesced load), switching to a group-uniform binary search for long rows.
template <int LPR>
__device__ __forceinline__ bool row_contains(const int32_t* __restrict__ cols, int64_t b,
                                             int64_t e, int32_t j, int q) {
    if (e - b <= 4 * LPR) {
        bool hit = false;
        for (int64_t x = b + q; x < e; x += LPR) hit |= (cols[x] == j);
        // OR over the group's lanes
#pragma unroll
        for (int off = LPR / 2; off >= 1; off >>= 1) hit |= (bool)__shfl_xor((int)hit, off);
        return hit;
    }
    int64_t lo = b, hi = e;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cols[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    return lo < e && cols[lo] == j;
}

template <int LPR, bool PAIR>
__global__ __launch_bounds__(256) void bpr_hogwild_kernel(
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols,
    const int32_t* __restrict__ eligible, int32_t n_eligible, const int32_t* __restrict__ ev_u,
    const int32_t* __restrict__ ev_i, int64_t n_samples, int64_t chunk, int32_t n_items,
    uint64_t seed, float* U, float* V, float* bias, int32_t ld4, BprScalars s) {
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const int64_t wave = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const int64_t begin = wave * chunk;
    const int64_t end = min(begin + chunk, n_samples);
    const int sub = lane / LPR, q = lane % LPR;
    float4* U4 = reinterpret_cast<float4*>(U);
    float4* V4 = reinterpret_cast<float4*>(V);
    for (int64_t base = begin; base < end; base += RPW) {
        const int64_t smp = base + sub;
        if (smp >= end) continue;
        int32_t u, i;
        if constexpr (PAIR) {
            u = ev_u[smp];
            i = ev_i[smp];
        } else {
            u = eligible[draw(seed, smp, 0, (uint32_t)n_eligible)];
            const int64_t b = off[u];
            const uint32_t deg = (uint32_t)(off[u + 1] - b);
            i = cols[b + draw(seed, smp, 1, deg)];
        }
        const int64_t ou = (int64_t)u * ld4 + q, oi = (int64_t)i * ld4 + q;
        const float4 w = U4[ou];
        const float4 hi = V4[oi];
        const int64_t rb = off[u], re = off[u + 1];
        int32_t j;
        for (uint32_t d = 2;; ++d) {
            j = (int32_t)draw(seed, smp, d, (uint32_t)n_items);
            if (!row_contains<LPR>(cols, rb, re, j, q)) break;
        }
        const int64_t oj = (int64_t)j * ld4 + q;
        const float4 hj = V4[oj];
        double part = (double)(w.x * (hi.x - hj.x));
        part += (double)(w.y * (hi.y - hj.y));
        part += (double)(w.z * (hi.z - hj.z));
        part += (double)(w.w * (hi.w - hj.w));
#pragma unroll
        for (int o = LPR / 2; o >= 1; o >>= 1) part += __shfl_xor(part, o);
        const float bi = bias[i], bj = bias[j];
        const double x_uij = (double)(bi - bj) + part;
        const double e = 1.0 / (1.0 + exp(x_uij));
        if (q == 0) {
            bias[i] = bi + (float)((double)s.lr * (e - (double)(s.bias_reg * bi)));
            if (s.update_j) bias[j] = bj + (float)((double)s.lr * (-e - (double)(s.bias_reg * bj)));
        }
        const double lr = s.lr;
        auto upd_u = [&](float wf, float hif, float hjf) {
            return (float)((double)wf + lr * ((double)(hif - hjf) * e - (double)(s.reg_u * wf)));
        };
        auto upd_i = [&](float wf, float hif) {
            return (float)((double)hif + lr * ((double)wf * e - (double)(s.reg_i * hif)));
        };
        auto upd_j = [&](float wf, float hjf) {
            return (float)((double)hjf + lr * ((double)(-wf) * e - (double)(s.reg_j * hjf)));
        };
        U4[ou] = make_float4(upd_u(w.x, hi.x, hj.x), upd_u(w.y, hi.y, hj.y),
                             upd_u(w.z, hi.z, hj.z), upd_u(w.w, hi.w, hj.w));
        V4[oi] = make_float4(upd_i(w.x, hi.x), upd_i(w.y, hi.y), upd_i(w.z, hi.z),
                             upd_i(w.w, hi.w));
        if (s.update_j)
            V4[oj] = make_float4(upd_j(w.x, hj.x), upd_j(w.y, hj.y), upd_j(w.z, hj.z),
                                 upd_j(w.w, hj.w));
    }
}

// Two-phase epoch (default): bpr_sample_kernel draws every triple of the epoch -- the same
// counter-based draws as the fused kernel, one thread per sample, so the dependent chain
// eligible -> off -> cols -> rejection search of one sample overlaps with thousands of others --
// and bpr_update_kernel then streams the triples like the BiasedMF Hogwild kernel (one row-load
// latency per step instead of the whole sampling chain).  Same triples, same visit order.
// Is j in the sorted row cols[rb, re)?  Rows of up to kScanMax entries are scanned flat: aligned
// int4 loads that do not depend on each other (one memory round trip instead of the log2(deg)
// dependent probes of a binary search; the CSR carries 16 entries of padding for the overrun),
// entries outside [rb, re) masked.  Longer rows fall back to the binary search.
constexpr int64_t kScanMax = 128;
__device__ __forceinline__ bool row_has(const int32_t* __restrict__ cols, int64_t rb, int64_t re,
                                        int32_t j) {
    if (re - rb <= kScanMax) {
        const int64_t a = rb & ~(int64_t)3;
        const int4* p = reinterpret_cast<const int4*>(cols + a);
        const int n4 = (int)((re - a + 3) >> 2);
        bool hit = false;
#pragma unroll 8
        for (int t = 0; t < n4; ++t) {
            const int4 v = p[t];
            const int64_t x = a + 4 * t;
            hit |= (v.x == j) & (x >= rb) & (x < re);
            hit |= (v.y == j) & (x + 1 >= rb) & (x + 1 < re);
            hit |= (v.z == j) & (x + 2 >= rb) & (x + 2 < re);
            hit |= (v.w == j) & (x + 3 < re);
        }
        return hit;
    }
    int64_t lo = rb, hi = re;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if (cols[mid] < j) lo = mid + 1;
        else hi = mid;
    }
    return lo < re && cols[lo] == j;
}

// Per-user record of the sampler: one aligned 64-B line per user holding the row start (words
// 0-1), |S_u| (word 2) and a 416-bit Bloom filter of S_u (words 3-15, three bits per item).  A
// sample reads this line instead of off[u], off[u + 1] and a separate filter line; the rejection
// test of j reads the filter and scans the row only when all three bits are set.  No false
// negatives, so the accepted j are exactly those of the plain test; for uniform j the scan then
// runs with probability ~(1 - e^{-3 deg / 416})^3 (2.8 % at deg 50).  The sampler is bound by the
// lines it moves (~10^9 samples/s), so the record takes one line per sample off the off[] gather.
constexpr int kRecWords = 16;
constexpr int kBloomBits = 416;
struct UserRec {
    int64_t rb, re;
};
__device__ __forceinline__ void bloom_bits(int32_t j, uint32_t& b0, uint32_t& b1, uint32_t& b2) {
    const uint64_t x = (uint64_t)(uint32_t)j * 0x9E3779B97F4A7C15ull;
    b0 = 96u + (uint32_t)((((x >> 48) & 0xFFFFu) * kBloomBits) >> 16);  // bit 96 = word 3
    b1 = 96u + (uint32_t)((((x >> 32) & 0xFFFFu) * kBloomBits) >> 16);
    b2 = 96u + (uint32_t)((((x >> 16) & 0xFFFFu) * kBloomBits) >> 16);
}
__device__ __forceinline__ bool bloom_maybe(const uint32_t* __restrict__ rec, int32_t j) {
    uint32_t b0, b1, b2;
    bloom_bits(j, b0, b1, b2);
    return ((rec[b0 >> 5] >> (b0 & 31)) & (rec[b1 >> 5] >> (b1 & 31)) & (rec[b2 >> 5] >> (b2 & 31)) &
            1u) != 0;
}
__device__ __forceinline__ UserRec user_rec(const uint32_t* __restrict__ rec) {
    const uint4 h = *reinterpret_cast<const uint4*>(rec);  // words 0-3: one load from the line
    const int64_t rb = (int64_t)(((uint64_t)h.y << 32) | h.x);
    return {rb, rb + (int64_t)h.z};
}
// 16 lanes per user, lane w owns word w of the user's record
__global__ __launch_bounds__(256) void bpr_user_rec_kernel(const int64_t* __restrict__ off,
                                                           const int32_t* __restrict__ cols,
                                                           int32_t n_users,
                                                           uint32_t* __restrict__ recs) {
    const int w = threadIdx.x & (kRecWords - 1);
    for (int64_t u = ((int64_t)blockIdx.x * blockDim.x + threadIdx.x) / kRecWords; u < n_users;
         u += (int64_t)gridDim.x * blockDim.x / kRecWords) {
        const int64_t rb = off[u], re = off[u + 1];
        uint32_t word = 0;
        if (w == 0) word = (uint32_t)(uint64_t)rb;
        else if (w == 1) word = (uint32_t)((uint64_t)rb >> 32);
        else if (w == 2) word = (uint32_t)(re - rb);
        else
            for (int64_t e = rb; e < re; ++e) {
                uint32_t b0, b1, b2;
                bloom_bits(cols[e], b0, b1, b2);
                if ((int)(b0 >> 5) == w) word |= 1u << (b0 & 31);
                if ((int)(b1 >> 5) == w) word |= 1u << (b1 & 31);
                if ((int)(b2 >> 5) == w) word |= 1u << (b2 & 31);
            }
        recs[u * kRecWords + w] = word;
    }
}

// SAMPLER: MML_BPR_SAMPLER_*.  eligible == nullptr: every user is eligible (u = the draw itself,
// no gather).  WEIGHTED (WeightedBPRMF.SampleTriple): (u, i) = event draw 0, j = the item of event
// draw d until j is not in S_u -- capped at kMaxWeightedDraws, after which the sample is flagged
// (*fail) instead of looping for ever on a user whose items carry all the event mass.
constexpr uint32_t kMaxWeightedDraws = 1u << 16;
// MML_BPR_SCHEDULE_AUTO applies epochs below this many samples in order (one wavefront)
constexpr int64_t kAutoOrderedBelow = 16 * 16384;
// The default sampler's triple of sample smp (IterateWithoutReplacementUniformUser: SampleUser,
// SampleItemPair, BPRMF.cs:290-310): u uniform over the eligible users, i uniform over S_u, j
// uniform over the items outside S_u (Bloom filter, then the row)
// User phases (bpr_phases): sample smp of phase p = the p with ptri[p] <= smp < ptri[p + 1] draws u
// uniformly over the phase's eligible users ph_users[ph_uoff[p] .. ph_uoff[p + 1]), and every
// phase holds triples in proportion to its users, so each user is still drawn with probability
// 1 / n_eligible per triple (SampleUser, BPRMF.cs:300-310); the triples come out phase-major.
struct BprPhases {
    const int32_t* users = nullptr;  // eligible users ordered by phase (stable)
    const int32_t* uoff = nullptr;   // [P + 1]
    const int64_t* tri = nullptr;    // [P + 1]
    int32_t n = 1;
};
__device__ __forceinline__ void draw_uniform_user(const int32_t* __restrict__ cols,
                                                  const int32_t* __restrict__ eligible,
                                                  int32_t n_eligible, int32_t n_items,
                                                  uint64_t seed, const uint32_t* __restrict__ recs,
                                                  int64_t smp, int32_t& u, int32_t& i,
                                                  int32_t& j, const BprPhases& ph, int& p) {
    if (ph.n > 1) {
        // p is carried over a thread's ascending samples: it only moves forward
        while (p + 1 < ph.n && smp >= ph.tri[p + 1]) ++p;
        const int32_t b = ph.uoff[p];
        u = ph.users[b + (int32_t)draw(seed, smp, 0, (uint32_t)(ph.uoff[p + 1] - b))];
    } else {
        const uint32_t du = draw(seed, smp, 0, (uint32_t)n_eligible);
        u = eligible ? eligible[du] : (int32_t)du;
    }
    const uint32_t* rec = recs + (int64_t)u * kRecWords;
    const UserRec ur = user_rec(rec);
    i = cols[ur.rb + draw(seed, smp, 1, (uint32_t)(ur.re - ur.rb))];
    for (uint32_t d = 2;; ++d) {
        j = (int32_t)draw(seed, smp, d, (uint32_t)n_items);
        if (!(bloom_maybe(rec, j) && row_has(cols, ur.rb, ur.re, j))) break;
    }
}

template <int SAMPLER>
__global__ __launch_bounds__(256) void bpr_sample_kernel(
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols,
    const int32_t* __restrict__ eligible, int32_t n_eligible, const int32_t* __restrict__ ev_u,
    const int32_t* __restrict__ ev_i, int64_t n_samples, int32_t n_items, uint64_t seed,
    int32_t* __restrict__ tu, int32_t* __restrict__ ti, int32_t* __restrict__ tj,
    int32_t* __restrict__ fail, uint64_t* __restrict__ user_keys,
    const uint32_t* __restrict__ recs, const uint8_t* __restrict__ gtab,
    uint8_t* __restrict__ tg, BprPhases ph) {
    int ph_p = 0;
    for (int64_t smp = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; smp < n_samples;
         smp += (int64_t)gridDim.x * blockDim.x) {
        int32_t u, i = 0, j = 0;
        if constexpr (SAMPLER == MML_BPR_SAMPLER_UNIFORM_USER) {
            draw_uniform_user(cols, eligible, n_eligible, n_items, seed, recs, smp, u, i, j, ph,
                              ph_p);
            tu[smp] = u;
            ti[smp] = i;
            tj[smp] = j;
            if (tg) tg[smp] = gtab[i];  // the XCD partition's key, while i is at hand
            continue;
        }
        if constexpr (SAMPLER == MML_BPR_SAMPLER_UNIFORM_PAIR) {
            u = ev_u[smp];
            i = ev_i[smp];
        } else if constexpr (SAMPLER == MML_BPR_SAMPLER_WEIGHTED ||
                             SAMPLER == MML_BPR_SAMPLER_PAIR_REPLACEMENT) {
            const uint32_t e = draw(seed, smp, 0, (uint32_t)n_samples);
            u = ev_u[e];
            i = ev_i[e];
        } else {
            const uint32_t du = draw(seed, smp, 0, (uint32_t)n_eligible);
            u = eligible ? eligible[du] : (int32_t)du;
        }
        const uint32_t* rec = recs + (int64_t)u * kRecWords;
        const UserRec ur = user_rec(rec);
        const int64_t rb = ur.rb, re = ur.re;
        auto in_row = [&](int32_t c) { return bloom_maybe(rec, c) && row_has(cols, rb, re, c); };
        // USER_REPLACEMENT: i is resolved after the epoch's samples are ranked per user
        if constexpr (SAMPLER == MML_BPR_SAMPLER_USER_REPLACEMENT)
            user_keys[smp] = ((uint64_t)(uint32_t)u << 32) | (uint32_t)smp;
        if constexpr (SAMPLER == MML_BPR_SAMPLER_WEIGHTED) {
            uint32_t d = 1;
            for (; d <= kMaxWeightedDraws; ++d) {
                j = ev_i[draw(seed, smp, d, (uint32_t)n_samples)];
                if (!in_row(j)) break;
            }
            if (d > kMaxWeightedDraws) {
                atomicOr(fail, 1);
                j = i;
            }
        } else {
            for (uint32_t d = 2;; ++d) {
                j = (int32_t)draw(seed, smp, d, (uint32_t)n_items);
                if (!in_row(j)) break;
            }
        }
        tu[smp] = u;
        if constexpr (SAMPLER != MML_BPR_SAMPLER_USER_REPLACEMENT) {
            ti[smp] = i;
            if (tg) tg[smp] = gtab[i];
        }
        tj[smp] = j;
    }
}

// USER_REPLACEMENT, after a stable sort of the keys (u << 32 | s) by u: head[u] = the position
// of user u's first sample, so sample s's rank among its user's samples is its position - head[u]
__global__ __launch_bounds__(256) void bpr_user_heads_kernel(const uint64_t* __restrict__ sorted,
                                                             int64_t n, int64_t* __restrict__ head) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
         p += (int64_t)gridDim.x * blockDim.x) {
        const uint32_t u = (uint32_t)(sorted[p] >> 32);
        if (p == 0 || (uint32_t)(sorted[p - 1] >> 32) != u) head[u] = p;
    }
}

// i of every USER_REPLACEMENT sample: rank r -> round r / deg, position r mod deg of that round's
// keyed permutation of S_u (IterateWithReplacementUniformUser, BPRMF.cs:190-203: draw from the
// remaining items, forget the drawn one, refill the user's copy when it is empty)
__global__ __launch_bounds__(256) void bpr_resolve_user_replacement_kernel(
    const uint64_t* __restrict__ sorted, int64_t n, const int64_t* __restrict__ head,
    const int64_t* __restrict__ off, const int32_t* __restrict__ cols, uint64_t seed,
    int32_t* __restrict__ ti) {
    for (int64_t p = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; p < n;
         p += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t key = sorted[p];
        const uint32_t u = (uint32_t)(key >> 32), s = (uint32_t)key;
        const uint32_t r = (uint32_t)(p - head[u]);
        const int64_t b = off[u];
        const uint32_t deg = (uint32_t)(off[u + 1] - b);
        const uint32_t round = r / deg, pos = r - round * deg;
        const uint64_t rk = splitmix64(seed ^ ((uint64_t)u * 0x9E3779B97F4A7C15ull) ^
                                       ((uint64_t)round << 40) ^ 0x2545F4914F6CDD1Dull);
        ti[s] = cols[b + keyed_perm(pos, deg, rk)];
    }
}

// the triple of lane base + lane / LPR: v_readlane per group while a step holds <= 4 groups
template <int LPR>
__device__ __forceinline__ int32_t bpr_group_fetch(int32_t v, int base, int lane) {
    constexpr int RPW = 64 / LPR;
    if constexpr (RPW <= 4) {
        const int sub = lane / LPR;
        int out = __builtin_amdgcn_readlane(v, base);
        if constexpr (RPW >= 2) out = sub == 1 ? __builtin_amdgcn_readlane(v, base + 1) : out;
        if constexpr (RPW >= 4) {
            out = sub == 2 ? __builtin_amdgcn_readlane(v, base + 2) : out;
            out = sub == 3 ? __builtin_amdgcn_readlane(v, base + 3) : out;
        }
        return out;
    } else {
        return __shfl(v, base + lane / LPR);
    }
}

// Access flags of the update kernel's item rows and biases (AM, a bit mask)
constexpr int kBprLdL2 = 1;   // V_i, V_j, b_i, b_j loaded sc1: L2-served, past the CU's stale L1
constexpr int kBprJThru = 2;  // V_j / b_j stored sc1: write-through, dropped from this XCD's L2
constexpr int kBprIThru = 4;  // V_i / b_i stored sc1 as well: every item row lives memory-side
constexpr int kBprUThru = 16;  // U_u loaded sc1 and stored sc1 (write-through): no stale user
                               // rows in any XCD's L2 (U < 4 GiB only: buffer addressing)
constexpr int kBprReplay = 32;  // (mml_bpr_replay_traffic) the same loads, every value stored
                                // back unchanged with the same flags: the traffic, no arithmetic
constexpr int kBprFlush = 8;  // one wave per XCD writes its L2's dirty lines back after every 64
                              // triples it applies (agent release fence = buffer_wbl2): the owner's
                              // hot rows reach memory, where the other XCDs read them as j, within
                              // one batch instead of at the end of the launch

// Triples split into ng group spans by the XCD group of i (mml_device.h group_wave); ng = 1: one span
template <int LPR, bool SOFT, int AM>
__global__ __launch_bounds__(256) void bpr_update_kernel(
    const int32_t* __restrict__ tu, const int32_t* __restrict__ ti, const int32_t* __restrict__ tj,
    const int64_t* __restrict__ goff, int32_t ng,
    int32_t waves_per_group, float* U, float* V, float* bias, int32_t ld4, uint32_t v_bytes,
    uint32_t b_bytes, uint32_t u_bytes, int32_t flushers, BprScalars s) {
    constexpr int RPW = 64 / LPR;
    const int lane = threadIdx.x & 63;
    const mml::GroupWave gw = mml::group_wave(goff, ng, waves_per_group,
                                              __builtin_amdgcn_readfirstlane(threadIdx.x >> 6),
                                              blockDim.x >> 6);
    const int64_t begin = gw.begin, end = gw.end;
    const int sub = lane / LPR, q = lane % LPR;
    float4* U4 = reinterpret_cast<float4*>(U);
    float4* V4 = reinterpret_cast<float4*>(V);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t vrs = mml::buffer_rsrc(V, v_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t brs = mml::buffer_rsrc(bias, b_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t urs = mml::buffer_rsrc(U, u_bytes);
    // the flushing waves: wave 0 of `flushers` evenly spaced blocks of each XCD's group
    [[maybe_unused]] const bool flusher =
        (AM & kBprFlush) != 0 && (threadIdx.x >> 6) == 0 &&
        (blockIdx.x >> 3) % max(1u, (gridDim.x >> 3) / (uint32_t)flushers) == 0;
    for (int64_t base = begin; base < end; base += 64) {
        if constexpr ((AM & kBprFlush) != 0)
            if (flusher) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        const int64_t x = base + lane;
        const bool in = x < end;
        const int32_t my_u = in ? tu[x] : 0, my_i = in ? ti[x] : 0, my_j = in ? tj[x] : 0;
        // consume the loads here, not at the top of the step loop (where the in-order counter
        // would also wait for the previous step's stores)
        asm volatile("" ::"v"(my_u), "v"(my_i), "v"(my_j));
        const int cnt = (int)min((int64_t)64, end - base);
        for (int step = 0; step < cnt; step += RPW) {
            const int32_t u = bpr_group_fetch<LPR>(my_u, step, lane);
            const int32_t i = bpr_group_fetch<LPR>(my_i, step, lane);
            const int32_t j = bpr_group_fetch<LPR>(my_j, step, lane);
            if (step + sub >= cnt) continue;
            const int64_t ou = (int64_t)u * ld4 + q, oi = (int64_t)i * ld4 + q,
                          oj = (int64_t)j * ld4 + q;
            float4 w;
            if constexpr ((AM & kBprUThru) != 0) w = mml::load4_l2(urs, (uint32_t)ou * 16u);
            else w = U4[ou];
            float4 hi, hj;
            float bi, bj;
            if constexpr (!(AM & kBprLdL2)) {
                hi = V4[oi];
                hj = V4[oj];
                bi = bias[i];
                bj = bias[j];
            } else {
                hi = mml::load4_l2(vrs, (uint32_t)oi * 16u);
                hj = mml::load4_l2(vrs, (uint32_t)oj * 16u);
                bi = mml::load1_l2(brs, (uint32_t)i * 4u);
                bj = mml::load1_l2(brs, (uint32_t)j * 4u);
            }
            if constexpr ((AM & kBprReplay) != 0) {
                asm volatile("" : "+v"(w.x), "+v"(w.y), "+v"(w.z), "+v"(w.w));
                asm volatile("" : "+v"(hi.x), "+v"(hi.y), "+v"(hi.z), "+v"(hi.w));
                asm volatile("" : "+v"(hj.x), "+v"(hj.y), "+v"(hj.z), "+v"(hj.w));
                asm volatile("" : "+v"(bi), "+v"(bj));
                using u4 = __attribute__((ext_vector_type(4))) uint32_t;
                if (q == 0) {
                    if constexpr ((AM & kBprIThru) != 0)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, bi), brs,
                                                              (uint32_t)i * 4u, 0, 16);
                    else
                        bias[i] = bi;
                    if (s.update_j) {
                        if constexpr ((AM & kBprJThru) != 0)
                            __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, bj),
                                                                  brs, (uint32_t)j * 4u, 0, 16);
                        else
                            bias[j] = bj;
                    }
                }
                if constexpr ((AM & kBprUThru) != 0)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, w), urs,
                                                           (uint32_t)ou * 16u, 0, 16);
                else
                    U4[ou] = w;
                if constexpr ((AM & kBprIThru) != 0)
                    __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, hi), vrs,
                                                           (uint32_t)oi * 16u, 0, 16);
                else
                    V4[oi] = hi;
                if (s.update_j) {
                    if constexpr ((AM & kBprJThru) != 0)
                        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u4, hj), vrs,
                                                               (uint32_t)oj * 16u, 0, 16);
                    else
                        V4[oj] = hj;
                }
                continue;
            }
            double part = (double)(w.x * (hi.x - hj.x));
            part += (double)(w.y * (hi.y - hj.y));
            part += (double)(w.z * (hi.z - hj.z));
            part += (double)(w.w * (hi.w - hj.w));
#pragma unroll
            for (int o = LPR / 2; o >= 1; o >>= 1) part += __shfl_xor(part, o);
            // every lane of the group holds the bit-identical sum: `skip` is group-uniform
            const TripleStep<SOFT> t(s, (double)(bi - bj) + part);
            if (t.skip) continue;
            if (q == 0) {  // i == j: the reference re-reads item_bias[j] after writing [i]
                const float nbi = t.bias_i(s, bi);
                if constexpr ((AM & kBprIThru) != 0)
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, nbi), brs,
                                                          (uint32_t)i * 4u, 0, 16);
                else
                    bias[i] = nbi;
                if (s.update_j) {
                    const float nbj = t.bias_j(s, i == j ? nbi : bj);
                    if constexpr ((AM & kBprJThru) != 0)
                        __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, nbj),
                                                              brs, (uint32_t)j * 4u, 0, 16);
                    else
                        bias[j] = nbj;
                }
            }
            const float4 nw = make_float4(t.u(s, w.x, hi.x, hj.x), t.u(s, w.y, hi.y, hj.y),
                                          t.u(s, w.z, hi.z, hj.z), t.u(s, w.w, hi.w, hj.w));
            if constexpr ((AM & kBprUThru) != 0)
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, nw), urs,
                    (uint32_t)ou * 16u, 0, 16);
            else
                U4[ou] = nw;
            const float4 ni = make_float4(t.i(s, w.x, hi.x), t.i(s, w.y, hi.y),
                                          t.i(s, w.z, hi.z), t.i(s, w.w, hi.w));
            if constexpr ((AM & kBprIThru) != 0)
                __builtin_amdgcn_raw_buffer_store_b128(
                    __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, ni), vrs,
                    (uint32_t)oi * 16u, 0, 16);
            else
                V4[oi] = ni;
            if (s.update_j) {
                const float4 nj = make_float4(t.j(s, w.x, hj.x), t.j(s, w.y, hj.y),
                                              t.j(s, w.z, hj.z), t.j(s, w.w, hj.w));
                if constexpr ((AM & kBprJThru) != 0)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, nj), vrs,
                        (uint32_t)oj * 16u, 0, 16);
                else
                    V4[oj] = nj;
            }
        }
    }
}

// mml_bpr_apply_triples: UpdateFactors for a given triple list strictly in order -- one
// wavefront, lane f owns factors f, f + 64, ... (KM per lane); x_uij summed left to right in
// double through v_readlane exactly as RowScalarProductWithRowDifference
// (DataType/MatrixExtensions.cs:276-298), so the result is bit-faithful to the managed loop.
template <bool SOFT, int KM, bool XCD1 = false>
// With W = blockDim.x / 64 > 1 waves, wave w applies the contiguous part [w n / W, (w+1) n / W) in
// order: W streams in flight at once (the small-epoch Hogwild form, one CU, see mml_bpr_iterate).
// XCD1: the streams of all blocks b with b % 8 == 0, i.e. of the CUs of ONE XCD (probed by
// mml::xcd_groups), whose single L2 then holds every row: loads are L2-served (sc1, past the
// CUs' non-coherent L1s), so no update is lost to a stale replica; the other blocks exit.
__global__ __launch_bounds__(256) void bpr_apply_ordered_kernel(
    const int32_t* __restrict__ tu, const int32_t* __restrict__ ti, const int32_t* __restrict__ tj,
    int64_t n, float* U, float* V, float* bias, int32_t k, int32_t ld, BprScalars s,
    uint32_t u_bytes = 0, uint32_t v_bytes = 0, uint32_t b_bytes = 0,
    const uint8_t* __restrict__ flags = nullptr) {
    const int lane = threadIdx.x & 63;
    int64_t W = blockDim.x >> 6, w = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    if constexpr (XCD1) {
        if (blockIdx.x % 8 != 0) return;
        w += (int64_t)(blockIdx.x / 8) * W;
        W *= (int64_t)((gridDim.x + 7) / 8);
    }
    const auto ru = mml::buffer_rsrc(U, u_bytes), rv = mml::buffer_rsrc(V, v_bytes),
               rb = mml::buffer_rsrc(bias, b_bytes);
    auto ld1 = [&](__amdgpu_buffer_rsrc_t r, const float* base, const float* p) -> float {
        if constexpr (XCD1) return mml::load1_l2(r, (uint32_t)((p - base) * 4));
        return *p;
    };
    const int64_t x0 = n * w / W, x1 = n * (w + 1) / W;
    for (int64_t x = x0; x < x1; ++x) {
        const int32_t u = tu[x], i = ti[x], j = tj[x];
        float* Wu = U + (int64_t)u * ld;
        float* Hi = V + (int64_t)i * ld;
        float* Hj = V + (int64_t)j * ld;
        float w[KM], hi[KM], hj[KM], prod[KM];
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            w[m] = f < k ? ld1(ru, U, Wu + f) : 0.0f;
            hi[m] = f < k ? ld1(rv, V, Hi + f) : 0.0f;
            hj[m] = f < k ? ld1(rv, V, Hj + f) : 0.0f;
            prod[m] = w[m] * (hi[m] - hj[m]);
        }
        double dot = 0.0;
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int lim = min(64, k - 64 * m);
            const int bits = __float_as_int(prod[m]);
            for (int l = 0; l < lim; ++l)
                dot += (double)__int_as_float(__builtin_amdgcn_readlane(bits, l));
        }
        const float bi = ld1(rb, bias, bias + i), bj = ld1(rb, bias, bias + j);
        const TripleStep<SOFT> t(s, (double)(bi - bj) + dot);
        if (t.skip) continue;
        // UpdateFactors' update_u / update_i / update_j (BPRMF.cs:330-374): per triple when
        // flags are given (bits 0, 1, 2: RetrainUser / RetrainItem, :391-422), else u, i and
        // UpdateJ as in Iterate
        const int fl = flags ? (int)flags[x] : (3 | (s.update_j ? 4 : 0));
        const bool up_u = (fl & 1) != 0, up_i = (fl & 2) != 0, up_j = (fl & 4) != 0;
        if (lane == 0) {  // i == j: the reference re-reads item_bias[j] after writing [i]
            const float nbi = up_i ? t.bias_i(s, bi) : bi;
            if (up_i) bias[i] = nbi;
            if (up_j) bias[j] = t.bias_j(s, i == j ? nbi : bj);
        }
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            if (f < k) {
                if (up_u) Wu[f] = t.u(s, w[m], hi[m], hj[m]);
                if (up_i) Hi[f] = t.i(s, w[m], hi[m]);
                if (up_j) Hj[f] = t.j(s, w[m], hj[m]);
            }
        }
    }
}

// BPRMF.Predict (:425-431): item_bias[i] + RowScalarProduct (float, left to right);
// float.MinValue for ids beyond the model.  MF.Predict (WRMF) passes bias = nullptr.
__global__ __launch_bounds__(256) void mf_predict_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, int64_t n,
    int32_t n_users, int32_t n_items, const float* __restrict__ U, const float* __restrict__ V,
    const float* __restrict__ bias, int32_t k, int32_t ld, float* __restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = users[x], i = items[x];
        if (u < 0 || u >= n_users || i < 0 || i >= n_items) {
            out[x] = -3.402823466e+38f;
            continue;
        }
        const float* a = U + (int64_t)u * ld;
        const float* c = V + (int64_t)i * ld;
        float dot = 0.0f;
        for (int f = 0; f < k; ++f) dot += a[f] * c[f];
        out[x] = bias ? bias[i] + dot : dot;
    }
}

inline int grid_for(int64_t n, int block = 256, int cap = 8192) {
    const int64_t g = (n + block - 1) / block;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

inline int lanes_per_row(int k) {
    const int vec = (k + 3) / 4;
    int lpr = 1;
    while (lpr < vec) lpr <<= 1;
    return lpr;
}

// one epoch's triples: as sampled (u, i, j and the group byte of i), partitioned by that group
// (xu, xi, xj) and the partition's 9 group offsets
struct BprTriples {
    mml::DeviceArray<int32_t> u, i, j, xu, xi, xj;
    mml::DeviceArray<uint8_t> g;
    mml::DeviceArray<int64_t> goff;
    bool partitioned = false;  // (experiments: MML_BPR_PF_MODE) xu / xi / xj hold a partition
};

}  // namespace

struct mml_bpr {
    mml_ctx* ctx = nullptr;
    std::string last_kernel;  // the last epoch's update kernel, as rocprof names it
    mml_bpr_params p{};
    int32_t n_users = 0, n_items = 0, k = 0, ld = 0, lpr = 0;
    mml::DeviceArray<float> U, V, bias, ev_out;
    mml::DeviceArray<int64_t> off;
    mml::DeviceArray<int32_t> cols, eligible, ev_u, ev_i, q_u, q_i;
    // the epoch's triples (two-phase epoch) in two sets, so that the next epoch's can be drawn
    // beside this epoch's update (mml_bpr_set_next_seed); cur = the last epoch's set
    BprTriples tb[2];
    int32_t cur = 0;
    // the draw ahead: its stream and events, the seed it was asked for, the set that holds it
    hipStream_t side = nullptr;
    hipEvent_t ev_pf_go = nullptr, ev_pf_done = nullptr, ev_upd = nullptr;
    bool next_seed_set = false, pf_ready = false, last_prefetched = false;
    uint64_t next_seed = 0, pf_seed = 0;
    int64_t pf_n = -1;
    int32_t pf_buf = 0;
    mml::DeviceArray<int32_t> fail;                 // WEIGHTED sampler: a sample ran out of draws
    mml::DeviceArray<uint32_t> recs;                // per-user sampler records (row, |S_u|, Bloom)
    mml::DeviceArray<uint64_t> rank_keys, rank_sorted;  // USER_REPLACEMENT: (u << 32 | s)
    mml::DeviceArray<int64_t> rank_head;                // USER_REPLACEMENT: first position per user
    mml::DeviceArray<uint8_t> rank_tmp;                 // its radix-sort scratch
    // Hogwild on XCD-owned item groups (xcd.hip): the epoch's triples partitioned by the group of
    // i (stable, into the set's xu / xi / xj); span1 = {0, n} for the one-span launch
    mml::XcdSplit xs;
    mml::DeviceArray<int64_t> span1;
    bool has_groups = false;
    // multi-device context: one single-device handle per GPU over a user range ub[d] .. ub[d + 1]
    std::vector<mml_bpr*> shards;
    std::vector<int32_t> ub;
    // a repeated-device context: the item average by peer copies (mml::peer_average)
    mml::DeviceArray<float> avg_stage;
    hipEvent_t ev_ar0 = nullptr, ev_ar1 = nullptr;
    bool has_ar = false;  // ev_ar0 / ev_ar1 bracket the last item average
    // the last Hogwild update launch, for mml_bpr_replay_traffic (its triples stay in tb[cur]
    // until the next epoch)
    struct {
        bool valid = false, soft = false;
        int am = 0, wpb = 4;
        int32_t ng = 1;
        const int64_t* goff = nullptr;
        const int32_t *tu = nullptr, *ti = nullptr, *tj = nullptr;
        int64_t blocks = 0;
        BprScalars s{};
        int32_t phases = 1;
        const int64_t* poff = nullptr;  // phases > 1: 8 span offsets per phase
    } last_launch;
    int64_t n_events = 0, nnz = 0;
    int64_t hog_waves = 0;  // mml_bpr_set_hogwild_waves (0: by the epoch size)
    // user phases of the default sampler's epoch (bpr_phases): the eligible users ordered by
    // phase, per-phase user and triple offsets, the partitioned triples' span offsets
    std::vector<int32_t> elig_host;
    int32_t n_phases = 1, phases_req = 0, last_phases = 1;
    int64_t phases_for_n = -1;
    std::vector<int64_t> ptri_host;
    mml::DeviceArray<int32_t> ph_users, ph_uoff;
    mml::DeviceArray<int64_t> ph_tri, poff, ph_zero;  // ph_zero: 8 zero offsets
    int32_t n_eligible = 0;
    bool has_data = false, has_model = false, has_order = false, has_triples = false;
    float last_ms = 0.0f, last_update_ms = 0.0f;
};

namespace {

void upload_padded(mml_bpr* h, float* dst, const float* src, int64_t rows) {
    if (rows == 0) return;
    MML_HIP(hipMemsetAsync(dst, 0, sizeof(float) * rows * h->ld, h->ctx->stream));
    MML_HIP(hipMemcpy2DAsync(dst, sizeof(float) * h->ld, src, sizeof(float) * h->k,
                             sizeof(float) * h->k, rows, hipMemcpyHostToDevice, h->ctx->stream));
}

void download_padded(mml_bpr* h, float* dst, const float* src, int64_t rows) {
    if (rows == 0) return;
    MML_HIP(hipMemcpy2DAsync(dst, sizeof(float) * h->k, src, sizeof(float) * h->ld,
                             sizeof(float) * h->k, rows, hipMemcpyDeviceToHost, h->ctx->stream));
}

}  // namespace

using mml::guard;

// ------------------------------------------------------------------ multi-device handles
// The one-process form of user-sharded BPRMF (the reference's parallel form is
// MultiCoreBPRMF, MultiCoreBPRMF.cs:49-63): events split into contiguous user ranges of equal
// event count, each device samples and updates its range (negatives over all items), and after
// every epoch one RCCL all-reduce of V || b averages the item side.
namespace {

void bpr_single_device_only(const mml_bpr* h) {
    if (h->ctx->multi())
        mml::fail(MML_ERR_STATE, "not available on a multi-device context (user-sharded "
                                 "Hogwild training, Predict and AUC only)");
}

std::vector<std::vector<int64_t>> bpr_route(const mml_bpr* h, const int32_t* users, int64_t n) {
    std::vector<std::vector<int64_t>> r(h->shards.size());
    for (int64_t x = 0; x < n; ++x) {
        const int32_t u = users[x];
        r[u >= 0 && u < h->n_users ? mml::owner_of(h->ub, u) : 0].push_back(x);
    }
    return r;
}

}  // namespace

extern "C" mml_status mml_bpr_create(mml_ctx* ctx, const mml_bpr_params* params, int32_t n_users,
                                     int32_t n_items, mml_bpr** out) {
    return guard([&] {
        MML_REQUIRE(ctx && params && out, "null argument");
        MML_REQUIRE(n_users >= 1 && n_items >= 2, "need >= 1 user and >= 2 items");
        MML_REQUIRE(params->num_factors >= 1 && params->num_factors <= 256,
                    "num_factors must be in [1, 256]");
        MML_REQUIRE(params->sampler >= MML_BPR_SAMPLER_UNIFORM_USER &&
                        params->sampler <= MML_BPR_SAMPLER_PAIR_REPLACEMENT,
                    "unknown sampler");
        MML_REQUIRE(params->model == MML_BPR_MODEL_BPR ||
                        params->model == MML_BPR_MODEL_SOFT_MARGIN,
                    "unknown model family");
        MML_REQUIRE(params->schedule >= MML_BPR_SCHEDULE_AUTO &&
                        params->schedule <= MML_BPR_SCHEDULE_ORDERED,
                    "unknown schedule");
        if (ctx->multi()) {
            // WeightedBPRMF draws j by item popularity (WeightedBPRMF.cs:55-67); a shard holds
            // only its users' events, so its popularity would be shard-local, not the reference's
            MML_REQUIRE(params->sampler != MML_BPR_SAMPLER_WEIGHTED,
                        "the WEIGHTED sampler (global item popularity) is single-device only");
            auto* h = new mml_bpr();
            h->ctx = ctx;
            h->p = *params;
            h->n_users = n_users;
            h->n_items = n_items;
            h->k = params->num_factors;
            h->shards.assign(ctx->sub.size(), nullptr);
            h->ub.assign(ctx->sub.size() + 1, n_users);
            h->ub[0] = 0;
            for (size_t d = 0; d < ctx->sub.size(); ++d) {
                const mml_status st =
                    mml_bpr_create(ctx->sub[d], params, n_users, n_items, &h->shards[d]);
                if (st != MML_OK) {
                    const std::string m = mml_last_error();
                    mml_bpr_destroy(h);
                    mml::fail(st, m);
                }
            }
            *out = h;
            return;
        }
        ctx->activate();
        auto* h = new mml_bpr();
        try {
            h->ctx = ctx;
            h->p = *params;
            h->n_users = n_users;
            h->n_items = n_items;
            h->k = params->num_factors;
            h->lpr = lanes_per_row(h->k);
            h->ld = 4 * h->lpr;
            h->U.alloc((size_t)n_users * h->ld);
            h->V.alloc((size_t)n_items * h->ld);
            h->bias.alloc(n_items);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

extern "C" mml_status mml_bpr_destroy(mml_bpr* h) {
    return guard([&] {
        if (!h) return;
        if (!h->ctx) {  // a create that failed before binding the context
            delete h;
            return;
        }
        if (h->ctx && h->ctx->multi()) {
            for (mml_bpr* s : h->shards)
                if (s) mml_bpr_destroy(s);
            if (h->ev_ar0) {
                (void)hipSetDevice(h->ctx->device);
                (void)hipEventDestroy(h->ev_ar0);
                (void)hipEventDestroy(h->ev_ar1);
            }
            delete h;
            return;
        }
        (void)hipSetDevice(h->ctx->device);
        (void)hipStreamSynchronize(h->ctx->stream);
        if (h->ev_ar0) {
            (void)hipEventDestroy(h->ev_ar0);
            (void)hipEventDestroy(h->ev_ar1);
        }
        if (h->side) {
            (void)hipStreamSynchronize(h->side);
            (void)hipStreamDestroy(h->side);
            (void)hipEventDestroy(h->ev_pf_go);
            (void)hipEventDestroy(h->ev_pf_done);
            (void)hipEventDestroy(h->ev_upd);
        }
        delete h;
    });
}

namespace {

__global__ __launch_bounds__(256) void bpr_gather_events_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items,
    const int32_t* __restrict__ order, int64_t n, int32_t* __restrict__ eu,
    int32_t* __restrict__ ei) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = order ? order[x] : x;
        eu[x] = users[o];
        ei[x] = items[o];
    }
}

// Common device path: CSR of the sets on the device, eligible users, events in visit order.
void bpr_ingest(mml_bpr* h, const int32_t* users, const int32_t* items, int64_t n,
                const int32_t* order) {
    hipStream_t st = h->ctx->stream;
    mml::DeviceCsr csr;
    mml::build_csr_device(users, items, n, h->n_users, h->n_items, st, csr);
    std::vector<int32_t> elig;
    for (int32_t u = 0; u < h->n_users; ++u) {
        const int32_t d = csr.deg_host[u];
        if (d > 0 && d < h->n_items) elig.push_back(u);  // SampleUser's acceptance set
    }
    MML_REQUIRE(!elig.empty(), "no user has 0 < |items| < n_items");
    h->off.swap(csr.off);
    h->cols.swap(csr.cols);
    h->nnz = csr.nnz;
    h->recs.alloc((size_t)h->n_users * kRecWords);
    bpr_user_rec_kernel<<<grid_for((int64_t)h->n_users * kRecWords), 256, 0, st>>>(
        h->off.get(), h->cols.get(), h->n_users, h->recs.get());
    MML_HIP(hipGetLastError());
    h->n_events = n;
    h->n_eligible = (int32_t)elig.size();
    h->n_phases = 1;
    h->phases_for_n = -1;
    h->eligible.alloc(elig.size());
    MML_HIP(hipMemcpyAsync(h->eligible.get(), elig.data(), sizeof(int32_t) * elig.size(),
                           hipMemcpyHostToDevice, st));
    MML_HIP(hipStreamSynchronize(st));
    h->elig_host.swap(elig);
    MML_REQUIRE(h->p.sampler != MML_BPR_SAMPLER_USER_REPLACEMENT || n <= (int64_t)UINT32_MAX,
                "USER_REPLACEMENT ranks samples with 32-bit indices: at most 2^32 - 1 events");
    h->has_triples = false;
    h->pf_ready = false;  // triples drawn ahead belong to the old data
    h->has_groups = false;
    h->span1.alloc(2);
    const int64_t span[2] = {0, n};
    MML_HIP(hipMemcpyAsync(h->span1.get(), span, sizeof(span), hipMemcpyHostToDevice, st));
    // PAIR: visit order; WEIGHTED / PAIR_REPLACEMENT: any order (events drawn by index)
    if (h->p.sampler != MML_BPR_SAMPLER_UNIFORM_USER &&
        h->p.sampler != MML_BPR_SAMPLER_USER_REPLACEMENT) {
        h->ev_u.alloc(n);
        h->ev_i.alloc(n);
        bpr_gather_events_kernel<<<grid_for(n), 256, 0, st>>>(users, items, order, n,
                                                              h->ev_u.get(), h->ev_i.get());
        MML_HIP(hipGetLastError());
    }
    MML_HIP(hipStreamSynchronize(st));
    h->has_data = true;
}

__global__ __launch_bounds__(256) void bpr_check_ids_kernel(const int32_t* __restrict__ users,
                                                            const int32_t* __restrict__ items,
                                                            const int32_t* __restrict__ order,
                                                            int64_t n, int32_t n_users,
                                                            int32_t n_items,
                                                            int32_t* __restrict__ bad) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        if (users[x] < 0 || users[x] >= n_users || items[x] < 0 || items[x] >= n_items)
            atomicOr(bad, 1);
        if (order && (order[x] < 0 || order[x] >= n)) atomicOr(bad, 2);
    }
}

// mml_bpr_set_data_device on a multi-device context: the arrays live on the first device.  The
// per-user counts, the user ranges of equal event count and a stable partition of the
// (visit-ordered) events by owner run there; each shard then ingests its contiguous part (a peer
// copy when its device differs) -- equal to mml_bpr_set_data with the same arrays on the host.
void bpr_multi_set_data_device(mml_bpr* h, const int32_t* users, const int32_t* items, int64_t n,
                               const int32_t* order) {
    const int32_t nd = (int32_t)h->shards.size();
    MML_REQUIRE(nd <= 8, "mml_bpr_set_data_device on a multi-device context shards over at most "
                         "8 devices (use mml_bpr_set_data)");
    mml_bpr* s0 = h->shards[0];
    s0->ctx->activate();
    hipStream_t st = s0->ctx->stream;
    {
        mml::DeviceArray<int32_t> bad;
        bad.alloc(1);
        MML_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int32_t), st));
        bpr_check_ids_kernel<<<grid_for(n), 256, 0, st>>>(users, items, order, n, h->n_users,
                                                          h->n_items, bad.get());
        MML_HIP(hipGetLastError());
        int32_t flag = 0;
        MML_HIP(hipMemcpyAsync(&flag, bad.get(), sizeof(int32_t), hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        MML_REQUIRE(!(flag & 1), "event user/item id out of range");
        MML_REQUIRE(!(flag & 2), "order index out of range");
    }
    h->has_data = false;
    h->ub = mml::balanced_user_bounds_counts(mml::device_id_counts(st, users, n, h->n_users), n,
                                             nd);
    mml::DeviceArray<int32_t> ou, oi, pu, pi;
    const int32_t *su = users, *si = items;
    if (order) {  // the visit order first (UNIFORM_PAIR's Feedback.RandomIndex)
        ou.alloc(n);
        oi.alloc(n);
        bpr_gather_events_kernel<<<grid_for(n), 256, 0, st>>>(users, items, order, n, ou.get(),
                                                              oi.get());
        MML_HIP(hipGetLastError());
        su = ou.get();
        si = oi.get();
    }
    std::vector<int64_t> goff(nd + 1, 0);
    goff[nd] = n;
    if (nd > 1) {
        std::vector<uint8_t> table(h->n_users);
        for (int32_t d = 0; d < nd; ++d)
            for (int32_t u = h->ub[d]; u < h->ub[d + 1]; ++u) table[u] = (uint8_t)d;
        mml::XcdSplit xs;
        xs.set_table(st, table);
        pu.alloc(n);
        pi.alloc(n);
        const int32_t* in[2] = {su, si};
        int32_t* out[2] = {pu.get(), pi.get()};
        xs.partition(st, su, n, 2, in, out);
        int64_t g[9];
        MML_HIP(hipMemcpyAsync(g, xs.goff.get(), sizeof(g), hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        for (int32_t d = 0; d < nd; ++d) goff[d] = g[d];
        ou.reset();
        oi.reset();
        su = pu.get();
        si = pi.get();
    }
    MML_HIP(hipStreamSynchronize(st));
    for (int32_t d = 0; d < nd; ++d)
        MML_REQUIRE(goff[d + 1] > goff[d], "a device's user range holds no event");
    for (int32_t d = 0; d < nd; ++d) {
        mml_bpr* s = h->shards[d];
        const int64_t o = goff[d], m = goff[d + 1] - goff[d];
        const int32_t *du = su + o, *di = si + o;
        mml::DeviceArray<int32_t> tu, ti;  // the shard's part on its own device
        if (s->ctx->device != s0->ctx->device) {
            s->ctx->activate();
            tu.alloc(m);
            ti.alloc(m);
            hipStream_t ss = s->ctx->stream;
            MML_HIP(hipMemcpyPeerAsync(tu.get(), s->ctx->device, du, s0->ctx->device,
                                       sizeof(int32_t) * m, ss));
            MML_HIP(hipMemcpyPeerAsync(ti.get(), s->ctx->device, di, s0->ctx->device,
                                       sizeof(int32_t) * m, ss));
            MML_HIP(hipStreamSynchronize(ss));
            du = tu.get();
            di = ti.get();
        }
        s->ctx->activate();
        s->has_data = false;
        bpr_ingest(s, du, di, m, nullptr);
    }
    s0->ctx->activate();
    h->n_events = n;
    h->has_data = true;
}

}  // namespace

extern "C" mml_status mml_bpr_set_data(mml_bpr* h, const int32_t* users, const int32_t* items,
                                       int64_t n, const int32_t* order) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        MML_REQUIRE(n >= 1 && users && items, "need >= 1 event");
        if (h->ctx->multi()) {
            if (order)
                for (int64_t x = 0; x < n; ++x)
                    MML_REQUIRE(order[x] >= 0 && order[x] < n, "order index out of range");
            for (int64_t x = 0; x < n; ++x)
                MML_REQUIRE(users[x] >= 0 && users[x] < h->n_users, "user id out of range");
            const int32_t nd = (int32_t)h->shards.size();
            h->ub = mml::balanced_user_bounds(users, n, h->n_users, nd);
            std::vector<std::vector<int32_t>> su(nd), si(nd);
            for (int64_t x = 0; x < n; ++x) {  // visit order (UNIFORM_PAIR), split by user owner
                const int64_t o = order ? order[x] : x;
                const int32_t d = mml::owner_of(h->ub, users[o]);
                su[d].push_back(users[o]);
                si[d].push_back(items[o]);
            }
            for (int32_t d = 0; d < nd; ++d)
                MML_REQUIRE(!su[d].empty(), "a device's user range holds no event");
            mml::on_devices(h->ctx, [&](int32_t d) {
                return mml_bpr_set_data(h->shards[d], su[d].data(), si[d].data(),
                                        (int64_t)su[d].size(), nullptr);
            });
            h->n_events = n;
            h->has_data = true;
            return;
        }
        if (order)
            for (int64_t x = 0; x < n; ++x)
                MML_REQUIRE(order[x] >= 0 && order[x] < n, "order index out of range");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->has_data = false;
        mml::DeviceArray<int32_t> du, di, dord;
        du.alloc(n);
        di.alloc(n);
        MML_HIP(hipMemcpyAsync(du.get(), users, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(di.get(), items, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
        if (order) {
            dord.alloc(n);
            MML_HIP(hipMemcpyAsync(dord.get(), order, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                                   st));
        }
        bpr_ingest(h, du.get(), di.get(), n, order ? dord.get() : nullptr);
    });
}

extern "C" mml_status mml_bpr_set_data_device(mml_bpr* h, const int32_t* users,
                                              const int32_t* items, int64_t n,
                                              const int32_t* order) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        MML_REQUIRE(n >= 1 && users && items, "need >= 1 event");
        // the arrays may come from any stream of the caller's (e.g. torch's): wait for the device
        h->ctx->activate();
        MML_HIP(hipDeviceSynchronize());
        MML_REQUIRE(!order || (h->p.sampler != MML_BPR_SAMPLER_UNIFORM_USER &&
                               h->p.sampler != MML_BPR_SAMPLER_USER_REPLACEMENT),
                    "a device order is not used by the user-sampling samplers");
        if (h->ctx->multi()) return bpr_multi_set_data_device(h, users, items, n, order);
        h->ctx->activate();
        h->has_data = false;
        bpr_ingest(h, users, items, n, order);
    });
}

extern "C" mml_status mml_bpr_set_model(mml_bpr* h, const float* U, const float* V,
                                        const float* item_bias) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {
            mml::on_devices(h->ctx, [&](int32_t d) {
                return mml_bpr_set_model(h->shards[d], U, V, item_bias);
            });
            h->has_model = true;
            return;
        }
        MML_REQUIRE(U && V && item_bias, "null model arrays");
        h->ctx->activate();
        upload_padded(h, h->U.get(), U, h->n_users);
        upload_padded(h, h->V.get(), V, h->n_items);
        MML_HIP(hipMemcpyAsync(h->bias.get(), item_bias, sizeof(float) * h->n_items,
                               hipMemcpyHostToDevice, h->ctx->stream));
        MML_HIP(hipStreamSynchronize(h->ctx->stream));
        h->has_model = true;
    });
}

namespace {

// N(mean, stddev) fill of a [rows x ld] matrix (first k columns, padding zero) from a counter-based
// generator: element e -> splitmix64(seed ^ e) -> Box-Muller.  Used for models too large for the
// host RNG chain (C3: 1.41e9 normals); statistically, not bitwise, equal to InitNormal.
__global__ __launch_bounds__(256) void init_normal_kernel(float* __restrict__ M, int64_t rows,
                                                          int32_t k, int32_t ld, uint64_t seed,
                                                          double mean, double stddev) {
    const int64_t total = rows * ld;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int32_t c = (int32_t)(e % ld);
        if (c >= k) {
            M[e] = 0.0f;
            continue;
        }
        const uint64_t x = splitmix64(seed ^ (uint64_t)e * 0x9E3779B97F4A7C15ull);
        const double u1 = ((x >> 11) + 1.0) * (1.0 / 9007199254740993.0);  // (0, 1]
        const double u2 = (double)(splitmix64(x) >> 11) * (1.0 / 9007199254740992.0);
        const double z = sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2);
        M[e] = (float)(mean + stddev * z);
    }
}

}  // namespace

extern "C" mml_status mml_bpr_init_model(mml_bpr* h, uint64_t seed, double mean, double stddev) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {  // same seed on every device: one initial model
            mml::on_devices(h->ctx, [&](int32_t d) {
                return mml_bpr_init_model(h->shards[d], seed, mean, stddev);
            });
            h->has_model = true;
            return;
        }
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        init_normal_kernel<<<8192, 256, 0, st>>>(h->U.get(), h->n_users, h->k, h->ld, seed, mean,
                                                 stddev);
        init_normal_kernel<<<8192, 256, 0, st>>>(h->V.get(), h->n_items, h->k, h->ld,
                                                 seed ^ 0x5DEECE66Dull, mean, stddev);
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemsetAsync(h->bias.get(), 0, sizeof(float) * h->n_items, st));
        MML_HIP(hipStreamSynchronize(st));
        h->has_model = true;
    });
}

extern "C" mml_status mml_bpr_get_model(mml_bpr* h, float* U, float* V, float* item_bias) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {
            MML_REQUIRE(h->has_model, "no model");
            mml::on_devices(h->ctx, [&](int32_t d) {
                return mml::guard([&] {
                    mml_bpr* s = h->shards[d];
                    s->ctx->activate();
                    const int64_t lo = h->ub[d], rows = h->ub[d + 1] - h->ub[d];
                    if (U && rows > 0)
                        download_padded(s, U + lo * h->k, s->U.get() + lo * s->ld, rows);
                    if (d == 0) {
                        if (V) download_padded(s, V, s->V.get(), h->n_items);
                        if (item_bias)
                            MML_HIP(hipMemcpyAsync(item_bias, s->bias.get(),
                                                   sizeof(float) * h->n_items,
                                                   hipMemcpyDeviceToHost, s->ctx->stream));
                    }
                    MML_HIP(hipStreamSynchronize(s->ctx->stream));
                });
            });
            return;
        }
        MML_REQUIRE(h->has_model, "no model");
        h->ctx->activate();
        if (U) download_padded(h, U, h->U.get(), h->n_users);
        if (V) download_padded(h, V, h->V.get(), h->n_items);
        if (item_bias)
            MML_HIP(hipMemcpyAsync(item_bias, h->bias.get(), sizeof(float) * h->n_items,
                                   hipMemcpyDeviceToHost, h->ctx->stream));
        MML_HIP(hipStreamSynchronize(h->ctx->stream));
    });
}

namespace {

// one wavefront applies n triples in order (bpr_apply_ordered_kernel), k <= 256
void launch_apply_ordered(mml_bpr* h, const int32_t* tu, const int32_t* ti, const int32_t* tj,
                          int64_t n, const BprScalars& s, hipStream_t st, int waves = 1,
                          int xcd1_blocks = 0, const uint8_t* flags = nullptr) {
    const int km = (h->k + 63) / 64;
    const bool soft = h->p.model == MML_BPR_MODEL_SOFT_MARGIN;
    const uint32_t ub = (uint32_t)((uint64_t)h->n_users * h->ld * 4);
    const uint32_t vb = (uint32_t)((uint64_t)h->n_items * h->ld * 4);
    const uint32_t bb = (uint32_t)((uint64_t)h->n_items * 4);
#define MML_APPLY(SOFT, KM)                                                                     \
    if (xcd1_blocks > 0)                                                                        \
        bpr_apply_ordered_kernel<SOFT, KM, true><<<8 * xcd1_blocks, 64 * waves, 0, st>>>(      \
            tu, ti, tj, n, h->U.get(), h->V.get(), h->bias.get(), h->k, h->ld, s, ub, vb, bb); \
    else                                                                                        \
        bpr_apply_ordered_kernel<SOFT, KM><<<1, 64 * waves, 0, st>>>(                           \
            tu, ti, tj, n, h->U.get(), h->V.get(), h->bias.get(), h->k, h->ld, s, 0, 0, 0, flags)
#define MML_APPLY_K(SOFT)                   \
    switch (km) {                           \
        case 1: MML_APPLY(SOFT, 1); break;  \
        case 2: MML_APPLY(SOFT, 2); break;  \
        case 3: MML_APPLY(SOFT, 3); break;  \
        default: MML_APPLY(SOFT, 4); break; \
    }
    if (soft) {
        MML_APPLY_K(true);
    } else {
        MML_APPLY_K(false);
    }
#undef MML_APPLY_K
#undef MML_APPLY
    MML_HIP(hipGetLastError());
}

// WeightedBPRMF Hogwild: streams on one XCD (MML_BPR_WSTREAMS overrides; 0 = the Hogwild update
// kernel over the whole chip); needs the probed block -> XCD mapping and rows < 4 GiB (the
// buffer resources of the L2-served loads)
int weighted_streams(mml_bpr* h) {
    static const int env = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_BPR_WSTREAMS");
        return e ? std::max(0, std::min(128, std::atoi(e))) / 4 * 4 : -1;
    }();
    const int v = env >= 0 ? env : 128;
    const bool fits = (uint64_t)h->n_users * h->ld * 4 < (1ull << 32) &&
                      (uint64_t)h->n_items * h->ld * 4 < (1ull << 32);
    return v > 0 && fits && mml::xcd_groups(h->ctx) == 8 ? v : 0;
}

BprScalars scalars_of(const mml_bpr* h) {
    BprScalars s;
    s.lr = h->p.learn_rate;
    s.reg_u = h->p.reg_u;
    s.reg_i = h->p.reg_i;
    s.reg_j = h->p.reg_j;
    s.bias_reg = h->p.bias_reg;
    s.update_j = h->p.update_j;
    return s;
}

// How the Hogwild update kernel splits and accesses the item side (MML_BPR_XCD = 0 .. 4):
//   0  one span over all XCDs, plain accesses (the round-1 kernel)
//   1  XCD-owned groups of i, item loads sc1, plain stores
//   2  the same, V_j / b_j stored write-through (sc1)
//   3  the same, V_i / b_i stored write-through too
//   4  one span, item loads sc1 and all item stores write-through (no owner: coherent item side)
//   5  mode 2 + one wave per XCD flushing its L2 after every batch of 64 triples (kBprFlush)
//   6  mode 5 + user rows written through (kBprUThru; mode 5 where U >= 4 GiB)
// Measured on the C3 replica (100k x 10k, tests/test_bpr_c3_replica_gpu.py): mode 1
// collapses (AUC 0.60 vs 0.78: a foreign XCD's plain j store leaves a dirty, stale copy of a hot
// row whose write-back reverts the owner's updates); modes 0 / 2 land +0.010 / +0.008 above the
// sequential AUC (foreign XCDs read hot j rows as of the owner's last write-back).
struct BprXcdMode {
    bool partition;
    int am;
};
BprXcdMode bpr_xcd_mode(int sampler) {
    static const int env = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_BPR_XCD");
        return e ? std::atoi(e) : -1;
    }();
    // WeightedBPRMF draws j by popularity: most j rows are hot rows of another XCD's group, so
    // the groups do not apply (mid replica: mode 2 +0.114 AUC, mode 0 -0.004)
    const int m = env >= 0 ? env : (sampler == MML_BPR_SAMPLER_WEIGHTED ? 0 : 6);
    switch (m) {
        case 1: return {true, kBprLdL2};
        case 2: return {true, kBprLdL2 | kBprJThru};
        case 3: return {true, kBprLdL2 | kBprJThru | kBprIThru};
        case 4: return {false, kBprLdL2 | kBprJThru | kBprIThru};
        case 5: return {true, kBprLdL2 | kBprJThru | kBprFlush};
        case 6: return {true, kBprLdL2 | kBprJThru | kBprFlush | kBprUThru};
        default: return {false, 0};
    }
}

// the phase of a user (the BiasedMF epoch's hash, bmf.hip user_phase): a random 1/P of the users
inline int32_t bpr_user_phase(int32_t u, int32_t P) {
    uint64_t x = (uint64_t)(uint32_t)u ^ 0x6A09E667F3BCC909ull;
    x += 0x9E3779B97F4A7C15ull;  // splitmix64's finaliser (mml_device.h mix64)
    x = (x ^ (x >> 30)) * 0xBF58476D1CE4E5B9ull;
    x = (x ^ (x >> 27)) * 0x94D049BB133111EBull;
    return (int32_t)((x ^ (x >> 31)) % (uint64_t)P);
}

// User phases of the default sampler's Hogwild epoch: off by default.  Measured at C3 (one box,
// profiles/r5e/c3_p*): update kernel 300.2 / 300.3 ms in one phase, 304.0 in 32, 310.3 in 51, 313.3
// in 64; sampler + partition 31.4 -> 35.6-36.9 ms.  Unlike BiasedMF's U, a phase's U rows do not
// stay in the Infinity Cache here: between two triples of a user the phase streams ~100 MB of
// uniform V_j rows (512 MB of V) through it.  mml_bpr_set_hogwild_phases turns them on.
// Phases for the sampler alone (triples drawn phase by phase, then partitioned and updated as one
// epoch) were measured too: sampler 32.7 -> 35.5 ms at 16 / 51 / 64 phases, the update unchanged
// (profiles/r5g/), so they were not kept.
int32_t bpr_phases(const mml_bpr* h) {
    static const int32_t env = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_BPR_PHASES");
        return e ? std::max(0, std::min(64, std::atoi(e))) : -1;
    }();
    int32_t P = 1;
    if (env >= 0) P = std::max(1, env);
    else if (h->phases_req > 0) P = h->phases_req;
    return std::max(1, std::min(P, h->n_eligible));
}

// the phase-ordered eligible users and the per-phase triple counts of an n-triple epoch
void ensure_bpr_phases(mml_bpr* h, int32_t P, int64_t n) {
    if (h->n_phases == P && h->phases_for_n == n) return;
    hipStream_t st = h->ctx->stream;
    h->n_phases = P;
    h->phases_for_n = n;
    if (P <= 1) return;
    std::vector<int32_t> cnt(P + 1, 0);
    std::vector<int32_t> ph(h->elig_host.size());
    for (size_t x = 0; x < ph.size(); ++x) {
        ph[x] = bpr_user_phase(h->elig_host[x], P);
        ++cnt[ph[x] + 1];
    }
    for (int32_t p = 0; p < P; ++p) cnt[p + 1] += cnt[p];
    std::vector<int32_t> users(ph.size()), at(cnt.begin(), cnt.end() - 1);
    for (size_t x = 0; x < ph.size(); ++x) users[at[ph[x]]++] = h->elig_host[x];
    // triples per phase in proportion to its users (cumulative rounding): each user is drawn with
    // probability 1 / n_eligible per triple, as SampleUser draws it
    std::vector<int64_t> tri(P + 1, 0);
    for (int32_t p = 1; p <= P; ++p)
        tri[p] = (int64_t)((long double)n * cnt[p] / (long double)h->n_eligible + 0.5L);
    tri[P] = n;
    h->ph_users.alloc(users.size());
    h->ph_uoff.alloc(P + 1);
    h->ph_tri.alloc(P + 1);
    h->poff.alloc((size_t)8 * P + 1);
    h->ph_zero.alloc(8);
    MML_HIP(hipMemsetAsync(h->ph_zero.get(), 0, sizeof(int64_t) * 8, st));
    MML_HIP(hipMemcpyAsync(h->ph_users.get(), users.data(), sizeof(int32_t) * users.size(),
                           hipMemcpyHostToDevice, st));
    MML_HIP(hipMemcpyAsync(h->ph_uoff.get(), cnt.data(), sizeof(int32_t) * (P + 1),
                           hipMemcpyHostToDevice, st));
    MML_HIP(hipMemcpyAsync(h->ph_tri.get(), tri.data(), sizeof(int64_t) * (P + 1),
                           hipMemcpyHostToDevice, st));
    MML_HIP(hipMemcpyAsync(h->poff.get() + (size_t)8 * P, &tri[P], sizeof(int64_t),
                           hipMemcpyHostToDevice, st));
    MML_HIP(hipStreamSynchronize(st));
    h->ptri_host.swap(tri);
}

// a phase's partition offsets (relative to its first triple) into the epoch's span offsets
__global__ void phase_span_kernel(const int64_t* __restrict__ goff, int64_t base,
                                  int64_t* __restrict__ out) {
    if (threadIdx.x < 8) out[threadIdx.x] = base + goff[threadIdx.x];
}

template <int LPR, bool SOFT>
void launch_update_lpr(mml_bpr* h, int am, int32_t ng, const int64_t* goff,
                       const int32_t* tu, const int32_t* ti, const int32_t* tj, int64_t blocks,
                       int wpb, const BprScalars& s,
                       hipStream_t st) {
    const int32_t wpg = (int32_t)(blocks / ng * wpb);
    const uint32_t vb = (uint32_t)std::min<uint64_t>((uint64_t)h->n_items * h->ld * 4, 0xFFFFFFFFull);
    const uint32_t bb = (uint32_t)((uint64_t)h->n_items * 4);
    const uint64_t u_all = (uint64_t)h->n_users * h->ld * 4;
    const uint32_t ub = (uint32_t)std::min<uint64_t>(u_all, 0xFFFFFFFFull);
    if (u_all >= (1ull << 32)) am &= ~kBprUThru;
#define MML_UPD(AM)                                                                           \
    bpr_update_kernel<LPR, SOFT, AM><<<(int)blocks, 64 * wpb, 0, st>>>(                      \
        tu, ti, tj, goff, ng, wpg, h->U.get(), h->V.get(), h->bias.get(), h->ld / 4, vb, \
        bb, ub, mml::flushers_per_xcd(4), s);                                                  \
    h->last_kernel = "bpr_update_kernel<" + std::to_string(LPR) + (SOFT ? ", true, " : ", false, ") + \
                     std::to_string((int)(AM)) + ">"
    switch (am) {
        case kBprLdL2: MML_UPD(kBprLdL2); break;
        case kBprLdL2 | kBprJThru: MML_UPD(kBprLdL2 | kBprJThru); break;
        case kBprLdL2 | kBprJThru | kBprIThru: MML_UPD(kBprLdL2 | kBprJThru | kBprIThru); break;
        case kBprLdL2 | kBprJThru | kBprFlush: MML_UPD(kBprLdL2 | kBprJThru | kBprFlush); break;
        case kBprLdL2 | kBprJThru | kBprFlush | kBprUThru:
            MML_UPD(kBprLdL2 | kBprJThru | kBprFlush | kBprUThru);
            break;
        default: MML_UPD(0); break;
    }
#undef MML_UPD
}

// the release access modes with the replay bit (mml_bpr_replay_traffic)
template <int LPR>
void launch_replay_lpr(mml_bpr* h, int am, int32_t ng, const int64_t* goff, const int32_t* tu,
                       const int32_t* ti, const int32_t* tj, int64_t blocks, int wpb,
                       const BprScalars& s, hipStream_t st) {
    const int32_t wpg = (int32_t)(blocks / ng * wpb);
    const uint32_t vb = (uint32_t)std::min<uint64_t>((uint64_t)h->n_items * h->ld * 4, 0xFFFFFFFFull);
    const uint32_t bb = (uint32_t)((uint64_t)h->n_items * 4);
    const uint64_t u_all = (uint64_t)h->n_users * h->ld * 4;
    const uint32_t ub = (uint32_t)std::min<uint64_t>(u_all, 0xFFFFFFFFull);
#define MML_REP(AM)                                                                           \
    bpr_update_kernel<LPR, false, (AM) | kBprReplay><<<(int)blocks, 64 * wpb, 0, st>>>(       \
        tu, ti, tj, goff, ng, wpg, h->U.get(), h->V.get(), h->bias.get(), h->ld / 4, vb, bb, ub, \
        mml::flushers_per_xcd(4), s)
    switch (am) {
        case kBprLdL2 | kBprJThru | kBprFlush: MML_REP(kBprLdL2 | kBprJThru | kBprFlush); break;
        case kBprLdL2 | kBprJThru | kBprFlush | kBprUThru:
            MML_REP(kBprLdL2 | kBprJThru | kBprFlush | kBprUThru);
            break;
        case 0: MML_REP(0); break;
        default: mml::fail(MML_ERR_STATE, "the traffic replay covers the release access modes");
    }
#undef MML_REP
}

void launch_update(mml_bpr* h, bool soft, int am, int32_t ng, const int64_t* goff,
                   const int32_t* tu, const int32_t* ti, const int32_t* tj, int64_t blocks,
                   int wpb, const BprScalars& s,
                   hipStream_t st) {
#define MML_UPL(LPR)                                                                           \
    if (soft)                                                                                  \
        launch_update_lpr<LPR, true>(h, am, ng, goff, tu, ti, tj, blocks, wpb, s, st);   \
    else                                                                                       \
        launch_update_lpr<LPR, false>(h, am, ng, goff, tu, ti, tj, blocks, wpb, s, st)
    switch (h->lpr) {
        case 1: MML_UPL(1); break;
        case 2: MML_UPL(2); break;
        case 4: MML_UPL(4); break;
        case 8: MML_UPL(8); break;
        case 16: MML_UPL(16); break;
        case 32: MML_UPL(32); break;
        default: MML_UPL(64); break;
    }
#undef MML_UPL
    MML_HIP(hipGetLastError());
}

}  // namespace

extern "C" mml_status mml_bpr_iterate(mml_bpr* h, uint64_t seed) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {  // every device's epoch (its own sample stream), then the average
            MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede iterate");
            const size_t nd = h->shards.size();
            std::vector<float> ms(nd, 0.0f), ums(nd, 0.0f);
            // phase 1: every shard's epoch; phase 2 (only when all succeeded, so no rank waits in
            // a collective another one skipped): the item average
            auto epoch = [&](int32_t d) {
                const mml_status st =
                    mml_bpr_iterate(h->shards[d], seed + 0x9E3779B97F4A7C15ull * d);
                ms[d] = h->shards[d]->last_ms;
                ums[d] = h->shards[d]->last_update_ms;
                return st;
            };
            if (h->ctx->repeated) {
                // shards of one GPU: one after another, each with the whole device (as it would
                // have a GPU of its own), then the average by peer copies, summed in shard order
                for (int32_t d = 0; d < (int32_t)nd; ++d) {
                    const mml_status st = epoch(d);
                    if (st != MML_OK)
                        mml::fail(st, "shard " + std::to_string(d) + ": " + mml_last_error());
                }
                mml_bpr* s0 = h->shards[0];
                s0->ctx->activate();
                if (!h->ev_ar0) {
                    MML_HIP(hipEventCreate(&h->ev_ar0));
                    MML_HIP(hipEventCreate(&h->ev_ar1));
                }
                std::vector<mml_ctx*> ctxs;
                std::vector<std::vector<float*>> arr;
                for (mml_bpr* s : h->shards) {
                    ctxs.push_back(s->ctx);
                    arr.push_back({s->V.get(), s->bias.get()});
                }
                mml::peer_average(ctxs, arr, {(int64_t)h->n_items * s0->ld, (int64_t)h->n_items},
                                  h->avg_stage, h->ev_ar0, h->ev_ar1);
                MML_HIP(hipEventSynchronize(h->ev_ar1));
                h->has_ar = true;
            } else {
                mml::on_devices(h->ctx, epoch);
                mml::on_devices(h->ctx,
                                [&](int32_t d) { return mml_bpr_allreduce_items(h->shards[d]); });
            }
            h->last_ms = *std::max_element(ms.begin(), ms.end());
            h->last_update_ms = *std::max_element(ums.begin(), ums.end());
            return;
        }
        MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede iterate");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        BprScalars s;
        s.lr = h->p.learn_rate;
        s.reg_u = h->p.reg_u;
        s.reg_i = h->p.reg_i;
        s.reg_j = h->p.reg_j;
        s.bias_reg = h->p.bias_reg;
        s.update_j = h->p.update_j;
        const int64_t n = h->n_events;  // Feedback.Count samples per epoch (:218)
        // >= 65,536 triples per wave: C3 (500 M) still runs 7,629 waves, and a 1.9 M-event epoch
        // runs 32 instead of 128 -- on the C3 replica the Hogwild AUC offset grows with the
        // triples in flight (+0.0037 at 32 waves, +0.0050 at 128, k = 128; profiles/r2_xcd/r2i_*)
        static const int64_t min_chunk = [] {
            const char* e = MML_EXPERIMENT_ENV("MML_HOGWILD_MIN_CHUNK");
            return e ? std::max<int64_t>(1, std::atoll(e)) : (int64_t)65536;
        }();
        int64_t waves = std::min<int64_t>(256 * 32, std::max<int64_t>(1, n / min_chunk));
        // an override keeps the partitioned multi-workgroup launch: at least 32 waves (8 groups x 4)
        if (h->hog_waves > 0 && waves >= 16)
            waves = std::min<int64_t>(256 * 32, std::max<int64_t>(32, h->hog_waves));
        // fewer than 16 waves' worth of samples run as ONE workgroup: one CU, one L2, where 2+
        // workgroups on different XCDs would each cache the hot item rows and overwrite each
        // other's updates on write-back (bmf.hip launch_hogwild)
        static const int64_t small_waves = [] {
            const char* e = MML_EXPERIMENT_ENV("MML_BPR_SMALL_WAVES");
            return e ? std::max<int64_t>(1, std::min<int64_t>(4, std::atoll(e))) : (int64_t)4;
        }();
        if (waves < 16) waves = small_waves;
        // larger epochs: a multiple of 8 blocks, so each XCD group gets the same number of blocks
        const int64_t blocks = waves < 16 ? 1 : (waves + 31) / 32 * 8;
        if (blocks > 1) waves = blocks * 4;
        const int64_t chunk = (n + waves - 1) / waves;
        const bool pair = h->p.sampler == MML_BPR_SAMPLER_UNIFORM_PAIR;
        const bool soft = h->p.model == MML_BPR_MODEL_SOFT_MARGIN;
        const bool weighted = h->p.sampler == MML_BPR_SAMPLER_WEIGHTED;
        const bool user_repl = h->p.sampler == MML_BPR_SAMPLER_USER_REPLACEMENT;
        static const bool fused_env = [] {
            const char* e = MML_EXPERIMENT_ENV("MML_BPR_FUSED");
            return e && std::atoi(e) > 0;
        }();
        // ORDERED (or AUTO on a small epoch): the sampled triples are applied in sample order by
        // one wavefront -- the reference's sequential loop on the device's triples
        const bool ordered = h->p.schedule == MML_BPR_SCHEDULE_ORDERED ||
                             (h->p.schedule == MML_BPR_SCHEDULE_AUTO && n < kAutoOrderedBelow);
        // the fused single-kernel epoch exists for the BPRMF update with the uniform samplers
        const bool fused = fused_env && !soft && !ordered &&
                           (pair || h->p.sampler == MML_BPR_SAMPLER_UNIFORM_USER);
        // XCD-owned item groups: the triples partitioned by the group of i (part of the sampling
        // phase), so that every access to V_i comes from the XCD that owns i
        const BprXcdMode xm = bpr_xcd_mode(h->p.sampler);
        const bool v_fits = (uint64_t)h->n_items * h->ld * sizeof(float) < (1ull << 32);
        const bool part = !ordered && !fused && n > 0 && waves >= 16 && xm.partition && v_fits &&
                          mml::xcd_groups(h->ctx) == 8;
        if (part && !h->has_groups) {
            h->xs.set_groups(st, mml::device_id_counts(st, h->cols.get(), h->nnz, h->n_items), 8);
            h->has_groups = true;
        }
        // the sampler writes each triple's group byte and the partition reads it instead of
        // looking the group up: sampler + partition 35.9 -> 32.7 ms per C3 epoch, same AUC
        // (profiles/r4r_c3_*.log; MML_BPR_GROUP_BYTES=0 in experiments builds: table lookups)
        // (the resolve kernel of USER_REPLACEMENT draws i later: that sampler keeps the lookups)
        static const bool group_bytes = [] {
            const char* e = MML_EXPERIMENT_ENV("MML_BPR_GROUP_BYTES");
            return !(e && std::string(e) == "0");
        }();
        const bool part_g = part && !user_repl && group_bytes;
        // user phases: the default sampler draws the epoch phase by phase, one update launch each
        const int32_t P =
            part_g && h->p.sampler == MML_BPR_SAMPLER_UNIFORM_USER ? bpr_phases(h) : 1;
        ensure_bpr_phases(h, P, n);
        BprPhases ph;
        if (P > 1) {
            ph.users = h->ph_users.get();
            ph.uoff = h->ph_uoff.get();
            ph.tri = h->ph_tri.get();
            ph.n = P;
        }
        h->last_phases = P;
        // the partitioned Hogwild epoch can draw the next epoch's triples beside its update
        // (mml_bpr_set_next_seed): the triples depend on the seed and the data, not on the model.
        // Not with phases (their span offsets are shared), WEIGHTED (a host check) or
        // USER_REPLACEMENT (a sort on shared scratch).
        const bool pf_path = part && P == 1 && !weighted && !user_repl && blocks > 1;
        const bool pre = pf_path && h->pf_ready && h->pf_seed == seed && h->pf_n == n;
        if (pre) h->cur = h->pf_buf;  // this epoch's triples were drawn ahead
        h->pf_ready = false;
        BprTriples& T = h->tb[h->cur];
        auto ensure = [&](BprTriples& X) {
            if (!fused && n > 0 && (int64_t)X.u.count < n) {
                X.u.alloc(n);
                X.i.alloc(n);
                X.j.alloc(n);
            }
            if (part_g && (int64_t)X.g.count < n) X.g.alloc(n);
            if (part && (int64_t)X.xu.count < n) {
                X.xu.alloc(n);
                X.xi.alloc(n);
                X.xj.alloc(n);
            }
            if (!X.goff.get()) X.goff.alloc(9);
        };
        ensure(T);
        // USER_REPLACEMENT: rank keys, their sorted copy, per-user heads and the sort's scratch
        int rank_end_bit = 0;
        size_t rank_tmp_bytes = 0;
        if (user_repl && n > 0) {
            if ((int64_t)h->rank_keys.count < n) {
                h->rank_keys.alloc(n);
                h->rank_sorted.alloc(n);
            }
            h->rank_head.alloc(h->n_users);
            int ub = 0;
            while (ub < 32 && ((uint32_t)(h->n_users - 1) >> ub) != 0) ++ub;
            rank_end_bit = 32 + std::max(ub, 1);
            MML_HIP(rocprim::radix_sort_keys(nullptr, rank_tmp_bytes, h->rank_keys.get(),
                                             h->rank_sorted.get(), n, 32, rank_end_bit, st));
            if (h->rank_tmp.count < rank_tmp_bytes) h->rank_tmp.alloc(rank_tmp_bytes);
        }
        const int sgrid = (int)std::min<int64_t>(256 * 64, (n + 255) / 256);
        // the sampler into set X with seed sd on stream s
        auto sample = [&](BprTriples& X, uint64_t sd, hipStream_t s, int grid) {
            if (weighted) {
                h->fail.alloc(1);
                MML_HIP(hipMemsetAsync(h->fail.get(), 0, sizeof(int32_t), s));
            }
#define MML_SMP(KIND, ELIG)                                                                     \
    bpr_sample_kernel<KIND><<<grid, 256, 0, s>>>(                                              \
        h->off.get(), h->cols.get(), ELIG, h->n_eligible, h->ev_u.get(), h->ev_i.get(), n,    \
        h->n_items, sd, X.u.get(), X.i.get(), X.j.get(), h->fail.get(), h->rank_keys.get(),    \
        h->recs.get(), part_g ? h->xs.group.get() : nullptr, part_g ? X.g.get() : nullptr, ph)
            int32_t* elig = h->n_eligible == h->n_users ? nullptr : h->eligible.get();
            switch (h->p.sampler) {
                case MML_BPR_SAMPLER_UNIFORM_PAIR:
                    MML_SMP(MML_BPR_SAMPLER_UNIFORM_PAIR, h->eligible.get());
                    break;
                case MML_BPR_SAMPLER_WEIGHTED: MML_SMP(MML_BPR_SAMPLER_WEIGHTED, nullptr); break;
                case MML_BPR_SAMPLER_USER_REPLACEMENT:
                    MML_SMP(MML_BPR_SAMPLER_USER_REPLACEMENT, elig);
                    break;
                case MML_BPR_SAMPLER_PAIR_REPLACEMENT:
                    MML_SMP(MML_BPR_SAMPLER_PAIR_REPLACEMENT, nullptr);
                    break;
                default: MML_SMP(MML_BPR_SAMPLER_UNIFORM_USER, elig); break;
            }
#undef MML_SMP
            MML_HIP(hipGetLastError());
            if (user_repl) {
                MML_HIP(rocprim::radix_sort_keys(h->rank_tmp.get(), rank_tmp_bytes,
                                                 h->rank_keys.get(), h->rank_sorted.get(), n, 32,
                                                 rank_end_bit, s));
                bpr_user_heads_kernel<<<sgrid, 256, 0, s>>>(h->rank_sorted.get(), n,
                                                            h->rank_head.get());
                bpr_resolve_user_replacement_kernel<<<sgrid, 256, 0, s>>>(
                    h->rank_sorted.get(), n, h->rank_head.get(), h->off.get(), h->cols.get(), sd,
                    X.i.get());
                MML_HIP(hipGetLastError());
            }
            if (weighted) {
                int32_t bad = 0;
                MML_HIP(hipMemcpyAsync(&bad, h->fail.get(), sizeof(int32_t),
                                       hipMemcpyDeviceToHost, s));
                MML_HIP(hipStreamSynchronize(s));
                if (bad)
                    mml::fail(MML_ERR_STATE,
                              "WeightedBPRMF: a user's items hold (nearly) all the event mass; no "
                              "negative item found in 65536 draws (the reference loops for ever)");
            }
        };
        // the stable partition of set X's triples by the group of i (XcdSplit) on stream s
        auto partition = [&](BprTriples& X, hipStream_t s) {
            const int32_t* in[3] = {X.u.get(), X.i.get(), X.j.get()};
            int32_t* out[3] = {X.xu.get(), X.xi.get(), X.xj.get()};
            if (P > 1) {  // each phase partitioned on its own: spans phase-major, group-minor
                for (int32_t p = 0; p < P; ++p) {
                    const int64_t b = h->ptri_host[p], m = h->ptri_host[p + 1] - b;
                    if (m == 0) {  // an empty phase: its 8 spans are empty at b
                        phase_span_kernel<<<1, 64, 0, s>>>(h->ph_zero.get(), b,
                                                            h->poff.get() + (size_t)8 * p);
                        continue;
                    }
                    const int32_t* inp[3] = {in[0] + b, in[1] + b, in[2] + b};
                    int32_t* outp[3] = {out[0] + b, out[1] + b, out[2] + b};
                    h->xs.partition_groups(s, X.g.get() + b, m, 3, inp, outp);
                    phase_span_kernel<<<1, 64, 0, s>>>(h->xs.goff.get(), b,
                                                        h->poff.get() + (size_t)8 * p);
                }
                MML_HIP(hipGetLastError());
            } else if (part_g) {
                h->xs.partition_groups(s, X.g.get(), n, 3, in, out, X.goff.get());
            } else {
                h->xs.partition(s, X.i.get(), n, 3, in, out, X.goff.get());
            }
            X.partitioned = true;
        };
        MML_HIP(hipEventRecord(h->ctx->ev_begin, st));
        if (!fused && n > 0 && !pre) sample(T, seed, st, sgrid);
        int32_t ng = 1;
        const int64_t* goff = h->span1.get();
        const int32_t *tu = T.u.get(), *ti = T.i.get(), *tj = T.j.get();
        // the access flags need the buffer resource (V < 4 GiB) and, for the owner modes, the
        // groups; a one-workgroup epoch keeps plain accesses (one CU, one L2)
        const int am = v_fits && waves >= 16 && (part || !xm.partition) ? xm.am : 0;
        if (part) {
            if (!pre) partition(T, st);
            ng = 8;
            goff = P > 1 ? h->poff.get() : T.goff.get();
            tu = T.xu.get();
            ti = T.xi.get();
            tj = T.xj.get();
        }
        MML_HIP(hipEventRecord(h->ctx->ev_mid, st));
        if (ordered && n > 0)
            launch_apply_ordered(h, T.u.get(), T.i.get(), T.j.get(), n, s, st);
        if (!ordered && !fused && n > 0 && blocks == 1) {
            // a small epoch (< 16 waves' worth): Hogwild with one stream per wave of ONE CU, each
            // applied in order (the lanes own factors, the exact arithmetic): 4 triples in flight
            // instead of 4 x 64 / LPR.  Measured on a 4,000-user WeightedBPRMF replica, whose
            // popularity-drawn j puts the hottest items into most concurrent triples: 1 wave of 16
            // triples per step -0.032 AUC vs the sequential oracle, 4 waves -0.038
            launch_apply_ordered(h, tu, ti, tj, n, s, st, (int)waves);
        } else if (!ordered && !fused && n > 0 && weighted && weighted_streams(h) > 0) {
            // WeightedBPRMF: popularity-drawn j puts the hottest rows into most triples in flight,
            // so it runs in-order streams on the CUs of one XCD (one L2, L2-served loads): fewer
            // triples in flight and no stale per-XCD replicas
            launch_apply_ordered(h, tu, ti, tj, n, s, st, 4, weighted_streams(h) / 4);
        } else if (!ordered && !fused && n > 0) {
            for (int32_t p = 0; p < P; ++p)
                launch_update(h, soft, am, ng, goff + (size_t)8 * p, tu, ti, tj, blocks, 4, s, st);
            int am_run = am;  // launch_update_lpr drops the user write-through past 4 GiB of U
            if ((uint64_t)h->n_users * h->ld * 4 >= (1ull << 32)) am_run &= ~kBprUThru;
            h->last_launch = {true, soft, am_run, 4, ng, goff, tu, ti, tj, blocks, s, P, goff};
        } else if (fused) {
#define MML_BPR(LPR)                                                                            \
    if (pair)                                                                                   \
        bpr_hogwild_kernel<LPR, true><<<(int)blocks, 256, 0, st>>>(                           \
            h->off.get(), h->cols.get(), h->eligible.get(), h->n_eligible, h->ev_u.get(),       \
            h->ev_i.get(), n, chunk, h->n_items, seed, h->U.get(), h->V.get(), h->bias.get(),   \
            h->ld / 4, s);                                                                      \
    else                                                                                        \
        bpr_hogwild_kernel<LPR, false><<<(int)blocks, 256, 0, st>>>(                          \
            h->off.get(), h->cols.get(), h->eligible.get(), h->n_eligible, h->ev_u.get(),       \
            h->ev_i.get(), n, chunk, h->n_items, seed, h->U.get(), h->V.get(), h->bias.get(),   \
            h->ld / 4, s)
            switch (h->lpr) {
                case 1: MML_BPR(1); break;
                case 2: MML_BPR(2); break;
                case 4: MML_BPR(4); break;
                case 8: MML_BPR(8); break;
                case 16: MML_BPR(16); break;
                case 32: MML_BPR(32); break;
                default: MML_BPR(64); break;
            }
#undef MML_BPR
        }
        MML_HIP(hipGetLastError());
        // the next epoch's triples into the other set on the second stream, beside the update;
        // the epoch ends when both are done, so its time holds one epoch's sampling either way
        const bool pf = pf_path && h->next_seed_set && n > 0;
        if (pf) {
            BprTriples& X = h->tb[h->cur ^ 1];
            ensure(X);
            if (!h->side) {
                MML_HIP(hipStreamCreateWithFlags(&h->side, hipStreamNonBlocking));
                MML_HIP(hipEventCreateWithFlags(&h->ev_pf_go, hipEventDisableTiming));
                MML_HIP(hipEventCreateWithFlags(&h->ev_pf_done, hipEventDisableTiming));
                MML_HIP(hipEventCreate(&h->ev_upd));
            }
            MML_HIP(hipEventRecord(h->ev_upd, st));
            // after this epoch's partition (ev_mid: the partition's scratch is shared)
            MML_HIP(hipStreamWaitEvent(h->side, h->ctx->ev_mid, 0));
            // (a thinner sampler disturbs the update no less: grids of 256 / 1,024 / 4,096 / 16,384
            // workgroups gave epochs of 333.3 / 327.4 / 323.3 / 324.6 ms, profiles/r5aj/)
#ifdef MML_EXPERIMENTS
            // MML_BPR_PF_MODE (timing A/B only, the triples go stale): 1 = the next epoch's sampler
            // without its partition, 2 = neither, once the set holds a partition
            static const int pf_mode = [] {
                const char* e = MML_EXPERIMENT_ENV("MML_BPR_PF_MODE");
                return e ? std::atoi(e) : 0;
            }();
            if (pf_mode == 0 || !X.partitioned) {
                sample(X, h->next_seed, h->side, sgrid);
                partition(X, h->side);
            } else if (pf_mode == 1) {
                sample(X, h->next_seed, h->side, sgrid);
            }
#else
            sample(X, h->next_seed, h->side, sgrid);
            partition(X, h->side);
#endif
            MML_HIP(hipEventRecord(h->ev_pf_done, h->side));
            MML_HIP(hipStreamWaitEvent(st, h->ev_pf_done, 0));
            h->pf_ready = true;
            h->pf_seed = h->next_seed;
            h->pf_n = n;
            h->pf_buf = h->cur ^ 1;
        }
        h->next_seed_set = false;
        h->last_prefetched = pre;
        MML_HIP(hipEventRecord(h->ctx->ev_end, st));
        MML_HIP(hipEventSynchronize(h->ctx->ev_end));
        MML_HIP(hipEventElapsedTime(&h->last_ms, h->ctx->ev_begin, h->ctx->ev_end));
        MML_HIP(hipEventElapsedTime(&h->last_update_ms, h->ctx->ev_mid,
                                    pf ? h->ev_upd : h->ctx->ev_end));
        h->has_triples = !fused && n > 0;
    });
}

extern "C" mml_status mml_bpr_set_next_seed(mml_bpr* h, uint64_t seed) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {  // each device's seed as mml_bpr_iterate derives it
            for (size_t d = 0; d < h->shards.size(); ++d) {
                const mml_status st =
                    mml_bpr_set_next_seed(h->shards[d], seed + 0x9E3779B97F4A7C15ull * d);
                if (st != MML_OK) mml::fail(st, mml_last_error());
            }
            return;
        }
        h->next_seed = seed;
        h->next_seed_set = true;
    });
}

extern "C" mml_status mml_bpr_last_triples(mml_bpr* h, int32_t* users, int32_t* items,
                                           int32_t* other_items, int64_t n) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {  // the shards' triples one after another, in shard order
            MML_REQUIRE(n == h->n_events && users && items && other_items,
                        "n must equal the epoch's sample count (Feedback.Count)");
            int64_t o = 0;
            for (mml_bpr* s : h->shards) {
                const mml_status st = mml_bpr_last_triples(s, users + o, items + o,
                                                           other_items + o, s->n_events);
                if (st != MML_OK) mml::fail(st, mml_last_error());
                o += s->n_events;
            }
            return;
        }
        MML_REQUIRE(h->has_triples, "no sampled epoch to report (run mml_bpr_iterate first; the "
                                    "fused experiment epoch keeps no triples)");
        MML_REQUIRE(n == h->n_events && users && items && other_items,
                    "n must equal the epoch's sample count (Feedback.Count)");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        const BprTriples& T = h->tb[h->cur];
        MML_HIP(hipMemcpyAsync(users, T.u.get(), sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
        MML_HIP(hipMemcpyAsync(items, T.i.get(), sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
        MML_HIP(hipMemcpyAsync(other_items, T.j.get(), sizeof(int32_t) * n, hipMemcpyDeviceToHost,
                               st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bpr_apply_triples(mml_bpr* h, const int32_t* users,
                                             const int32_t* items, const int32_t* other_items,
                                             int64_t n) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        bpr_single_device_only(h);
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(n >= 0 && (n == 0 || (users && items && other_items)), "bad arguments");
        for (int64_t x = 0; x < n; ++x)
            MML_REQUIRE(users[x] >= 0 && users[x] < h->n_users && items[x] >= 0 &&
                            items[x] < h->n_items && other_items[x] >= 0 &&
                            other_items[x] < h->n_items,
                        "triple id out of range");
        if (n == 0) return;
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        mml::DeviceArray<int32_t> du, di, dj;
        du.alloc(n);
        di.alloc(n);
        dj.alloc(n);
        MML_HIP(hipMemcpyAsync(du.get(), users, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(di.get(), items, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(dj.get(), other_items, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                               st));
        launch_apply_ordered(h, du.get(), di.get(), dj.get(), n, scalars_of(h), st);
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bpr_apply_triples_flags(mml_bpr* h, const int32_t* users,
                                                   const int32_t* items,
                                                   const int32_t* other_items,
                                                   const uint8_t* flags, int64_t n) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        bpr_single_device_only(h);
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(n >= 0 && (n == 0 || (users && items && other_items && flags)),
                    "bad arguments");
        for (int64_t x = 0; x < n; ++x)
            MML_REQUIRE(users[x] >= 0 && users[x] < h->n_users && items[x] >= 0 &&
                            items[x] < h->n_items && other_items[x] >= 0 &&
                            other_items[x] < h->n_items && flags[x] < 8,
                        "triple id or flag out of range");
        if (n == 0) return;
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        mml::DeviceArray<int32_t> du, di, dj;
        mml::DeviceArray<uint8_t> df;
        du.alloc(n);
        di.alloc(n);
        dj.alloc(n);
        df.alloc(n);
        MML_HIP(hipMemcpyAsync(du.get(), users, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(di.get(), items, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(dj.get(), other_items, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                               st));
        MML_HIP(hipMemcpyAsync(df.get(), flags, n, hipMemcpyHostToDevice, st));
        launch_apply_ordered(h, du.get(), di.get(), dj.get(), n, scalars_of(h), st, 1, 0,
                             df.get());
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bpr_set_rows(mml_bpr* h, int32_t side, int32_t n_rows,
                                       const int32_t* rows, const float* values) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        bpr_single_device_only(h);
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(side == 0 || side == 1, "side: 0 (users) or 1 (items)");
        MML_REQUIRE(n_rows >= 0 && (n_rows == 0 || (rows && values)), "bad arguments");
        const int32_t n_own = side == 0 ? h->n_users : h->n_items;
        for (int32_t x = 0; x < n_rows; ++x)
            MML_REQUIRE(rows[x] >= 0 && rows[x] < n_own, "row id beyond the model");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        float* M = side == 0 ? h->U.get() : h->V.get();
        for (int32_t x = 0; x < n_rows; ++x)  // in list order: a row listed twice takes the last
            MML_HIP(hipMemcpyAsync(M + (int64_t)rows[x] * h->ld, values + (int64_t)x * h->k,
                                   sizeof(float) * h->k, hipMemcpyHostToDevice, st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bpr_set_hogwild_phases(mml_bpr* h, int32_t phases) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        MML_REQUIRE(phases >= 0 && phases <= 64, "phases must be in [0, 64]");
        h->phases_req = phases;
        for (mml_bpr* s : h->shards) s->phases_req = phases;
    });
}

extern "C" mml_status mml_bpr_last_phases(mml_bpr* h, int32_t* out) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx && out, "null argument");
        *out = h->shards.empty() ? h->last_phases : h->shards[0]->last_phases;
    });
}

extern "C" mml_status mml_bpr_set_hogwild_waves(mml_bpr* h, int64_t waves) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        MML_REQUIRE(waves >= 0 && waves <= 256 * 32, "waves must be in [0, 8192]");
        h->hog_waves = waves;
        for (mml_bpr* s : h->shards) s->hog_waves = waves;
    });
}

extern "C" mml_status mml_bpr_last_kernel(mml_bpr* h, char* buf, int32_t cap) {
    return guard([&] {
        MML_REQUIRE(h && buf && cap > 0, "null argument");
        const std::string& k = h->shards.empty() ? h->last_kernel : h->shards[0]->last_kernel;
        const size_t n = std::min<size_t>(k.size(), (size_t)cap - 1);
        std::copy(k.begin(), k.begin() + n, buf);
        buf[n] = 0;
    });
}

extern "C" mml_status mml_bpr_last_timing(mml_bpr* h, float* out) {
    return guard([&] {
        MML_REQUIRE(h && out, "null argument");
        out[0] = h->last_ms;
        out[1] = h->last_update_ms;
    });
}

extern "C" mml_status mml_bpr_predict(mml_bpr* h, const int32_t* users, const int32_t* items,
                                      int64_t n, float* out) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {
            MML_REQUIRE(h->has_model, "no model");
            MML_REQUIRE(n >= 0 && (n == 0 || (users && items && out)), "bad arguments");
            const auto r = bpr_route(h, users, n);
            mml::on_devices(h->ctx, [&](int32_t d) {
                const auto& ix = r[d];
                if (ix.empty()) return (mml_status)MML_OK;
                std::vector<int32_t> u(ix.size()), i(ix.size());
                std::vector<float> o(ix.size());
                for (size_t x = 0; x < ix.size(); ++x) {
                    u[x] = users[ix[x]];
                    i[x] = items[ix[x]];
                }
                const mml_status st = mml_bpr_predict(h->shards[d], u.data(), i.data(),
                                                      (int64_t)ix.size(), o.data());
                for (size_t x = 0; st == MML_OK && x < ix.size(); ++x) out[ix[x]] = o[x];
                return st;
            });
            return;
        }
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(n >= 0 && (n == 0 || (users && items && out)), "bad arguments");
        if (n == 0) return;
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->q_u.alloc(n);
        h->q_i.alloc(n);
        h->ev_out.alloc(n);
        MML_HIP(hipMemcpyAsync(h->q_u.get(), users, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                               st));
        MML_HIP(hipMemcpyAsync(h->q_i.get(), items, sizeof(int32_t) * n, hipMemcpyHostToDevice,
                               st));
        mf_predict_kernel<<<grid_for(n), 256, 0, st>>>(h->q_u.get(), h->q_i.get(), n, h->n_users,
                                                       h->n_items, h->U.get(), h->V.get(),
                                                       h->bias.get(), h->k, h->ld,
                                                       h->ev_out.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemcpyAsync(out, h->ev_out.get(), sizeof(float) * n, hipMemcpyDeviceToHost,
                               st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bpr_allreduce_items(mml_bpr* h) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        bpr_single_device_only(h);
        mml_ctx* c = h->ctx;
        if (c->nranks <= 1 && !c->comm) return;  // no communicator: nothing to average
        MML_REQUIRE(c->comm, "context has no communicator (mml_ctx_comm_init)");
        c->activate();
        hipStream_t st = c->stream;
        // model averaging inside the collective (ncclAvg), stream-ordered: the next epoch's
        // kernels and every download run on this stream after it
        const size_t nv = (size_t)h->n_items * h->ld;
        if (!h->ev_ar0) {
            MML_HIP(hipEventCreate(&h->ev_ar0));
            MML_HIP(hipEventCreate(&h->ev_ar1));
        }
        MML_HIP(hipEventRecord(h->ev_ar0, st));
        MML_RCCL(ncclGroupStart());
        MML_RCCL(ncclAllReduce(h->V.get(), h->V.get(), nv, ncclFloat, ncclAvg, c->comm, st));
        MML_RCCL(ncclAllReduce(h->bias.get(), h->bias.get(), (size_t)h->n_items, ncclFloat,
                               ncclAvg, c->comm, st));
        MML_RCCL(ncclGroupEnd());
        MML_HIP(hipEventRecord(h->ev_ar1, st));
        h->has_ar = true;
    });
}

extern "C" mml_status mml_bpr_replay_traffic(mml_bpr* h, float* out_ms) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx && out_ms, "null argument");
        bpr_single_device_only(h);
        const auto& L = h->last_launch;
        MML_REQUIRE(L.valid && !L.soft && h->has_triples,
                    "the traffic replay repeats the last BPRMF Hogwild update launch: run a "
                    "HOGWILD epoch first");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        MML_HIP(hipEventRecord(h->ctx->ev_begin, st));
        for (int32_t p = 0; p < L.phases; ++p) {
            const int64_t* go = L.goff + (size_t)8 * p;
#define MML_RPL(LPR) \
    launch_replay_lpr<LPR>(h, L.am, L.ng, go, L.tu, L.ti, L.tj, L.blocks, L.wpb, L.s, st)
            switch (h->lpr) {
                case 1: MML_RPL(1); break;
                case 2: MML_RPL(2); break;
                case 4: MML_RPL(4); break;
                case 8: MML_RPL(8); break;
                case 16: MML_RPL(16); break;
                case 32: MML_RPL(32); break;
                default: MML_RPL(64); break;
            }
#undef MML_RPL
        }
        MML_HIP(hipGetLastError());
        MML_HIP(hipEventRecord(h->ctx->ev_end, st));
        MML_HIP(hipEventSynchronize(h->ctx->ev_end));
        MML_HIP(hipEventElapsedTime(out_ms, h->ctx->ev_begin, h->ctx->ev_end));
    });
}

extern "C" mml_status mml_bpr_last_allreduce_ms(mml_bpr* h, float* out) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx && out, "null argument");
        *out = 0.0f;
        auto one = [](mml_bpr* x, mml_ctx* c) {
            if (!x->has_ar) return 0.0f;
            c->activate();
            float ms = 0.0f;
            MML_HIP(hipEventSynchronize(x->ev_ar1));
            MML_HIP(hipEventElapsedTime(&ms, x->ev_ar0, x->ev_ar1));
            return ms;
        };
        if (h->ctx->multi()) {
            if (h->has_ar) {  // the peer average, on shard 0's device
                *out = one(h, h->shards[0]->ctx);
                return;
            }
            for (mml_bpr* s : h->shards) *out = std::max(*out, one(s, s->ctx));
            return;
        }
        *out = one(h, h->ctx);
    });
}

extern "C" mml_status mml_bpr_auc(mml_bpr* h, const int32_t* candidates, int32_t n_candidates,
                                  const int32_t* users, int32_t n_users, const int64_t* test_off,
                                  const int32_t* test_items, double* out_auc) {
    return guard([&] {
        MML_REQUIRE(h && h->ctx, "null handle");
        if (h->ctx->multi()) {  // each eval user on the device that holds its training items
            MML_REQUIRE(h->has_model && h->has_data, "model and training data required");
            MML_REQUIRE(n_users >= 0 && (n_users == 0 || (users && test_off && out_auc)),
                        "bad arguments");
            const auto r = bpr_route(h, users, n_users);
            mml::on_devices(h->ctx, [&](int32_t d) {
                const auto& ix = r[d];
                if (ix.empty()) return (mml_status)MML_OK;
                std::vector<int32_t> u(ix.size()), items;
                std::vector<int64_t> off(ix.size() + 1, 0);
                for (size_t x = 0; x < ix.size(); ++x) {
                    u[x] = users[ix[x]];
                    for (int64_t t = test_off[ix[x]]; t < test_off[ix[x] + 1]; ++t)
                        items.push_back(test_items[t]);
                    off[x + 1] = (int64_t)items.size();
                }
                std::vector<double> a(ix.size());
                const mml_status st = mml_bpr_auc(h->shards[d], candidates, n_candidates,
                                                  u.data(), (int32_t)ix.size(), off.data(),
                                                  items.empty() ? nullptr : items.data(),
                                                  a.data());
                for (size_t x = 0; st == MML_OK && x < ix.size(); ++x) out_auc[ix[x]] = a[x];
                return st;
            });
            return;
        }
        MML_REQUIRE(h->has_model && h->has_data, "model and training data required");
        h->ctx->activate();
        mml::item_auc(h->ctx->stream, h->U.get(), h->ld, h->n_users, h->V.get(), h->ld, h->n_items,
                      h->bias.get(), h->k, h->off.get(), h->cols.get(), h->n_users, candidates,
                      n_candidates, users, n_users, test_off, test_items, out_auc);
    });
}
