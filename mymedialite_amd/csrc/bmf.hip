// bmf.hip -- BiasedMatrixFactorization SGD on MI355X (gfx950).
//
// Replaces BiasedMatrixFactorization.Iterate(IList<int>,bool,bool)
// (src/MyMediaLite/RatingPrediction/BiasedMatrixFactorization.cs:264-310), its Predict (:313-325)
// and Eval.Ratings.Evaluate (src/MyMediaLite/Eval/Ratings.cs:96-139).
//
// HBM layout (per mml_bmf handle):
//   U [n_users x ld], V [n_items x ld]   fp32 row-major, ld = 4 * LPR (zero-padded columns), so a
//                                        factor row is LPR float4s = one coalesced 16-B-per-lane read
//   bu [n_users], bi [n_items]           fp32 biases
//   raw_{u,i,r}                          the training ratings as given (StaticRatings SoA)
//   s{u,i,r}                             the same ratings permuted into the epoch visit order
//                                        (DataSet.RandomIndex, fixed across epochs like the
//                                        reference, Data/DataSet.cs:100-110): the epoch reads it as
//                                        three perfectly coalesced streams
// Arithmetic follows the reference exactly: float dot / score / biases, double
// sigmoid, error and factor deltas, float increments; built with -ffp-contract=off.
//
// Schedules:
//   ORDERED  one wavefront walks the stream in order: lanes own factors, the dot product is summed
//            left to right through v_readlane, so the trajectory matches the CPU oracle bit for bit
//            (up to libm-vs-ocml exp rounding) -- the MaxThreads = 1 reference.
//   DSGD     the reference's MaxThreads = G schedule (:205-215): per sub-epoch one launch of G
//            wavefronts, wavefront j walks block (j, (s + j) mod G) in order; blocks of one sub-epoch
//            share no user and no item, so the result is deterministic and equals the reference's.
//   HOGWILD  lock-free: every wavefront owns a contiguous chunk of the permuted stream; LPR lanes
//            per rating (float4 each), 64/LPR ratings per wave step, dot product by xor-shuffle
//            reduction, plain (racy) stores of the updated rows -- Hogwild! semantics.
//   HOGWILD_COHERENT  the same with sc1 (agent-coherent) row and bias accesses, see load4 below.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset on the host
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <chrono>
#include <cstdlib>
#include <string>
#include <vector>

#include "mml_device.h"
#include "mml_internal.h"

namespace {

struct BmfScalars {
    float gb;         // global_bias
    float min_rating; // min_rating
    float range;      // rating_range_size
    float lr;         // current_learnrate
    float blr;        // BiasLearnRate * current_learnrate (float product, as in :286)
    float bias_reg;   // BiasReg
    float reg_u;      // RegU
    float reg_i;      // RegI
};

// compute_gradient_common (SetupLoss, :247-261)
template <int LOSS>
__device__ __forceinline__ float gradient_common(double sig, double err, float range) {
    if constexpr (LOSS == MML_LOSS_MAE) {
        const double sg = err > 0.0 ? 1.0 : (err < 0.0 ? -1.0 : 0.0);
        return (float)(sg * sig * (1.0 - sig) * (double)range);
    } else if constexpr (LOSS == MML_LOSS_LOGISTIC) {
        return (float)err;
    } else {
        return (float)(err * sig * (1.0 - sig) * (double)range);
    }
}

// Per-rating scalar part shared by all schedules: score, sigmoid, error, gradient, reg weights,
// new biases.  `dot` is the float row scalar product.
template <int LOSS>
struct RatingStep {
    float g, reg_u, reg_i, new_bu, new_bi;
    __device__ __forceinline__ RatingStep(const BmfScalars& s, float dot, float bu_u, float bi_i,
                                          float r, const int32_t* cnt_u, const int32_t* cnt_i,
                                          int32_t u, int32_t i) {
        const float score = ((s.gb + bu_u) + bi_i) + dot;
        const double sig = 1.0 / (1.0 + exp(-(double)score));
        const double prediction = (double)s.min_rating + sig * (double)s.range;
        const double err = (double)r - prediction;
        g = gradient_common<LOSS>(sig, err, s.range);
        reg_u = s.reg_u;
        reg_i = s.reg_i;
        if (cnt_u) {  // FrequencyRegularization (:281-282)
            reg_u = (float)((double)s.reg_u / sqrt((double)cnt_u[u]));
            reg_i = (float)((double)s.reg_i / sqrt((double)cnt_i[i]));
        }
        new_bu = bu_u + s.blr * (g - (s.bias_reg * reg_u) * bu_u);
        new_bi = bi_i + s.blr * (g - (s.bias_reg * reg_i) * bi_i);
    }
    // Matrix.Inc(u, f, lr * delta) (:291-308; DataType/MatrixExtensions.cs:76-79)
    __device__ __forceinline__ float new_u(const BmfScalars& s, float u_f, float i_f) const {
        const double delta = (double)g * (double)i_f - (double)reg_u * (double)u_f;
        return u_f + (float)((double)s.lr * delta);
    }
    __device__ __forceinline__ float inc_i(const BmfScalars& s, float u_f, float i_f) const {
        const double delta = (double)g * (double)u_f - (double)reg_i * (double)i_f;
        return (float)((double)s.lr * delta);
    }
    __device__ __forceinline__ float new_i(const BmfScalars& s, float u_f, float i_f) const {
        return i_f + inc_i(s, u_f, i_f);
    }
};

// MatrixFactorization (the plain model, MatrixFactorization.cs:166-196) runs on the same kernels
// as template value kPlainMF in the LOSS slot: no biases; err = r - (global_bias + dot) in float;
// delta = err * i_f - Regularization * u_f in float, widened to double; Inc adds
// (float)(current_learnrate * delta).
constexpr int kPlainMF = 8;
// The Hogwild kernel's memory traffic without its arithmetic (mml_bmf_replay_traffic): the same
// launch, stream, rows, biases and access flags, every loaded value stored back unchanged -- the
// access pattern's own ceiling on the GPU it runs on, measured beside the epoch (bench.py)
constexpr int kReplayTraffic = 9;

template <>
struct RatingStep<kPlainMF> {
    float err, reg_u, reg_i, new_bu, new_bi;
    __device__ __forceinline__ RatingStep(const BmfScalars& s, float dot, float, float, float r,
                                          const int32_t*, const int32_t*, int32_t, int32_t) {
        err = r - (s.gb + dot);
        reg_u = s.reg_u;
        reg_i = s.reg_i;
        new_bu = new_bi = 0.0f;
    }
    __device__ __forceinline__ float new_u(const BmfScalars& s, float u_f, float i_f) const {
        const double delta = (double)(err * i_f - reg_u * u_f);
        return u_f + (float)((double)s.lr * delta);
    }
    __device__ __forceinline__ float new_i(const BmfScalars& s, float u_f, float i_f) const {
        const double delta = (double)(err * u_f - reg_i * i_f);
        return i_f + (float)((double)s.lr * delta);
    }
};

// ORDERED / DSGD: workgroup = one wavefront; wavefront j walks block (j, (subepoch+j) mod G).
// A DSGD ring shard holds the block rows row0 .. row0 + gridDim.x - 1 only (block_off local to
// them).  KM = factors per lane (k <= 64 * KM).
template <int LOSS, int KM>
__global__ __launch_bounds__(64) void bmf_sgd_ordered_kernel(
    const int32_t* __restrict__ su, const int32_t* __restrict__ si, const float* __restrict__ sr,
    const int64_t* __restrict__ block_off, int32_t G, int32_t subepoch, int32_t row0, float* U,
    float* V, float* bu, float* bi, int32_t k, int32_t ld, BmfScalars s,
    const int32_t* __restrict__ cnt_u, const int32_t* __restrict__ cnt_i) {
    const int lane = threadIdx.x;
    const int j = row0 + blockIdx.x;
    const int64_t b = (int64_t)blockIdx.x * G + (subepoch + j) % G;
    const int64_t begin = block_off[b], end = block_off[b + 1];
    for (int64_t x = begin; x < end; ++x) {
        const int32_t u = su[x], i = si[x];
        const float r = sr[x];
        float* Uu = U + (int64_t)u * ld;
        float* Vi = V + (int64_t)i * ld;
        float pu[KM], qi[KM], prod[KM];
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            pu[m] = f < k ? Uu[f] : 0.0f;
            qi[m] = f < k ? Vi[f] : 0.0f;
            prod[m] = pu[m] * qi[m];
        }
        // RowScalarProduct: float accumulation, left to right (MatrixExtensions.cs:224-241)
        float dot = 0.0f;
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int lim = min(64, k - 64 * m);
            const int bits = __float_as_int(prod[m]);
            for (int l = 0; l < lim; ++l) dot += __int_as_float(__builtin_amdgcn_readlane(bits, l));
        }
        constexpr bool biased = LOSS != kPlainMF;
        const float bu_u = biased ? bu[u] : 0.0f, bi_i = biased ? bi[i] : 0.0f;
        const RatingStep<LOSS> st(s, dot, bu_u, bi_i, r, cnt_u, cnt_i, u, i);
        if (biased && lane == 0) {
            bu[u] = st.new_bu;
            bi[i] = st.new_bi;
        }
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            if (f < k) {
                Uu[f] = st.new_u(s, pu[m], qi[m]);
                Vi[f] = st.new_i(s, pu[m], qi[m]);
            }
        }
    }
}


// Row / bias access forms.  COH = false: plain loads/stores (cached in the CU's L1 and the XCD's
// L2).  COH = true: agent-scope relaxed atomics = global_load/store ... sc1, which bypass the
// non-coherent per-CU L1 and keep the eight per-XCD L2s from holding private dirty copies of a
// row (MI355X_MICROARCH.md, inter-workgroup visibility).  Plain Hogwild on MI355X therefore runs
// ~8 cache-level replicas of the hot Zipf items whose write-backs overwrite each other; COH makes
// every update land in one coherent copy, at the price of hot-row traffic at the memory side.
template <bool COH>
__device__ __forceinline__ float4 load4(const float4* p) {
    if constexpr (COH) {
        const unsigned long long* q = reinterpret_cast<const unsigned long long*>(p);
        const unsigned long long a = __hip_atomic_load(q, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const unsigned long long b =
            __hip_atomic_load(q + 1, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        return make_float4(__uint_as_float((unsigned)a), __uint_as_float((unsigned)(a >> 32)),
                           __uint_as_float((unsigned)b), __uint_as_float((unsigned)(b >> 32)));
    } else {
        return *p;
    }
}
template <bool COH>
__device__ __forceinline__ void store4(float4* p, float4 v) {
    if constexpr (COH) {
        unsigned long long* q = reinterpret_cast<unsigned long long*>(p);
        const unsigned long long a = (unsigned long long)__float_as_uint(v.x) |
                                     ((unsigned long long)__float_as_uint(v.y) << 32);
        const unsigned long long b = (unsigned long long)__float_as_uint(v.z) |
                                     ((unsigned long long)__float_as_uint(v.w) << 32);
        __hip_atomic_store(q, a, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        __hip_atomic_store(q + 1, b, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    } else {
        *p = v;
    }
}
template <bool COH>
__device__ __forceinline__ float load1(const float* p) {
    if constexpr (COH) return __hip_atomic_load(p, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else return *p;
}
template <bool COH>
__device__ __forceinline__ void store1(float* p, float v) {
    if constexpr (COH) __hip_atomic_store(p, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    else *p = v;
}

// Sum over an aligned group of LPR lanes, every lane of the group getting the bit-identical total
// (each pairwise add is x_self + x_partner, commutative).  Within a 16-lane row the partner comes
// through DPP (quad_perm xor 1 / xor 2, half-row mirror, row mirror): a VALU operand modifier with
// no LDS round trip, unlike __shfl_xor (ds_bpermute), which is kept only across rows.
#define MML_DPP_F32(v, ctrl) \
    __int_as_float(__builtin_amdgcn_update_dpp(0, __float_as_int(v), ctrl, 0xF, 0xF, false))
template <int LPR>
__device__ __forceinline__ float group_sum(float x) {
    if constexpr (LPR >= 2) x += MML_DPP_F32(x, 0xB1);   // quad_perm [1,0,3,2]
    if constexpr (LPR >= 4) x += MML_DPP_F32(x, 0x4E);   // quad_perm [2,3,0,1]
    if constexpr (LPR >= 8) x += MML_DPP_F32(x, 0x141);  // row_half_mirror
    if constexpr (LPR >= 16) x += MML_DPP_F32(x, 0x140); // row_mirror
    if constexpr (LPR >= 32) x += __shfl_xor(x, 16);
    if constexpr (LPR >= 64) x += __shfl_xor(x, 32);
    return x;
}

// value of lane base + (lane / LPR) for a wave-uniform base: v_readlane per group (scalar lane
// index, no LDS) while a step holds at most 4 groups, ds_bpermute beyond
template <int LPR, typename T>
__device__ __forceinline__ T group_fetch(T v, int base, int lane) {
    constexpr int RPW = 64 / LPR;
    if constexpr (RPW <= 4) {
        const int sub = lane / LPR;
        const int bits = __builtin_bit_cast(int, v);
        int out = __builtin_amdgcn_readlane(bits, base);
        if constexpr (RPW >= 2) out = sub == 1 ? __builtin_amdgcn_readlane(bits, base + 1) : out;
        if constexpr (RPW >= 4) {
            out = sub == 2 ? __builtin_amdgcn_readlane(bits, base + 2) : out;
            out = sub == 3 ? __builtin_amdgcn_readlane(bits, base + 3) : out;
        }
        return __builtin_bit_cast(T, out);
    } else {
        return __shfl(v, base + lane / LPR);
    }
}

// HOGWILD: LPR lanes per rating, VPL float4s of U_u and of V_i per lane (float4 q + LPR v of the
// row, so each load instruction reads 16 LPR contiguous bytes of every row in the step), plain
// racy stores of the new rows and biases (Hogwild!).  A float-atomic variant for item rows (no lost
// updates) was measured 7.5x slower on C2 (memory-side atomics serialise on hot Zipf items) for no
// RMSE gain at that scale, so it is not kept.  VPL > 1 puts more ratings in one wave
// step (64 / LPR): more rows in flight per wave and the per-rating scalar part (sigmoid, fp64
// gradient) shared by fewer lanes.
// Access flags of the Hogwild kernel's rows and biases (AM, a bit mask)
constexpr int kAccPlain = 0;     // plain loads / stores
constexpr int kAccCoherent = 1;  // every row / bias access agent-coherent (sc1), HOGWILD_COHERENT
constexpr int kAccItemL2 = 2;    // XCD-owned item groups: item rows / biases loaded sc1 (L2-served,
                                 // past the CU's stale L1), stored plain (kept in the owning L2)
constexpr int kAccUserThru = 4;  // user rows / biases loaded sc1 and stored sc1 (write-through,
                                 // dropped from this XCD's L2): a user's next rating, on any XCD,
                                 // reads the row from memory instead of a stale L2 copy
constexpr int kAccFlush = 8;     // one wave per XCD writes its L2's dirty lines back after every
                                 // 64 ratings it applies (agent release fence = buffer_wbl2)
constexpr int kAccUBiasPlain = 16;  // (experiments) with kAccUserThru: the user bias loaded and
                                    // stored plain, only the user rows written through

// The stream is split into ng group spans goff[g] .. goff[g + 1] (mml_device.h group_wave): ng = 8
// for XCD-owned item groups (block b serves group b % 8, one XCD per group), ng = 1 for one span.
// waves_per_group waves divide a span into contiguous chunks.
template <int LOSS, int LPR, int VPL, int AM>
__global__ __launch_bounds__(256) void bmf_sgd_hogwild_kernel(
    const int32_t* __restrict__ su, const int32_t* __restrict__ si, const float* __restrict__ sr,
    const int64_t* __restrict__ goff, int32_t ng, int32_t waves_per_group, float* U, float* V,
    float* bu, float* bi, int32_t ld4, uint32_t v_bytes, uint32_t bi_bytes, uint32_t u_bytes,
    uint32_t bu_bytes, int32_t flushers, BmfScalars s, const int32_t* __restrict__ cnt_u,
    const int32_t* __restrict__ cnt_i) {
    constexpr int RPW = 64 / LPR;  // ratings per wave step
    constexpr bool COH = AM == kAccCoherent;
    constexpr bool IL2 = (AM & kAccItemL2) != 0, UTH = (AM & kAccUserThru) != 0;
    constexpr bool BTH = UTH && (AM & kAccUBiasPlain) == 0;  // user bias written through
    const int lane = threadIdx.x & 63;
    // wave-uniform (SGPR) bounds: the loops' branches stay scalar
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    const mml::GroupWave gw = mml::group_wave(goff, ng, waves_per_group, wib, blockDim.x >> 6);
    const int64_t begin = gw.begin, end = gw.end;
    const int sub = lane / LPR, q = lane % LPR;
    float4* U4 = reinterpret_cast<float4*>(U);
    float4* V4 = reinterpret_cast<float4*>(V);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t vrs = mml::buffer_rsrc(V, v_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t brs = mml::buffer_rsrc(bi, bi_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t urs = mml::buffer_rsrc(U, u_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t burs = mml::buffer_rsrc(bu, bu_bytes);
    // the flushing waves: wave 0 of `flushers` evenly spaced blocks of each XCD's group
    [[maybe_unused]] const bool flusher =
        (AM & kAccFlush) != 0 && (threadIdx.x >> 6) == 0 &&
        (blockIdx.x >> 3) % max(1u, (gridDim.x >> 3) / (uint32_t)flushers) == 0;
    constexpr bool biased = LOSS != kPlainMF;
    // the rows and biases of one rating (this lane's float4s)
    auto fetch = [&](int32_t u, int32_t i, float4 (&pu)[VPL], float4 (&qi)[VPL], float& bu_u,
                     float& bi_i) {
        const int64_t ou = (int64_t)u * ld4 + q, oi = (int64_t)i * ld4 + q;
#pragma unroll
        for (int v = 0; v < VPL; ++v) {
            if constexpr (UTH)
                pu[v] = mml::load4_l2(urs, (uint32_t)(ou + LPR * v) * 16u);
            else
                pu[v] = load4<COH>(U4 + ou + LPR * v);
            if constexpr (IL2)
                qi[v] = mml::load4_l2(vrs, (uint32_t)(oi + LPR * v) * 16u);
            else
                qi[v] = load4<COH>(V4 + oi + LPR * v);
        }
        bu_u = 0.0f;
        bi_i = 0.0f;
        if constexpr (biased) {
            if constexpr (BTH) bu_u = mml::load1_l2(burs, (uint32_t)u * 4u);
            else bu_u = load1<COH>(bu + u);
            if constexpr (IL2) bi_i = mml::load1_l2(brs, (uint32_t)i * 4u);
            else bi_i = load1<COH>(bi + i);
        }
    };
    // the SGD step of one rating from its fetched rows, and the racy stores
    auto apply = [&](int32_t u, int32_t i, float r, const float4 (&pu)[VPL],
                     const float4 (&qi)[VPL], float bu_u, float bi_i) {
        const int64_t ou = (int64_t)u * ld4 + q, oi = (int64_t)i * ld4 + q;
        if constexpr (LOSS == kReplayTraffic) {
            // the loaded values, opaque to the compiler, stored with the epoch's access flags
            float4 a[VPL], c[VPL];
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                a[v] = pu[v];
                c[v] = qi[v];
                asm volatile("" : "+v"(a[v].x), "+v"(a[v].y), "+v"(a[v].z), "+v"(a[v].w));
                asm volatile("" : "+v"(c[v].x), "+v"(c[v].y), "+v"(c[v].z), "+v"(c[v].w));
            }
            asm volatile("" : "+v"(bu_u), "+v"(bi_i) : "v"(r));
            if (q == 0) {
                if constexpr (BTH)
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, bu_u), burs,
                                                          (uint32_t)u * 4u, 0, 16);
                else
                    store1<COH>(bu + u, bu_u);
                store1<COH>(bi + i, bi_i);
            }
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                if constexpr (UTH)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, a[v]),
                        urs, (uint32_t)(ou + LPR * v) * 16u, 0, 16);
                else
                    store4<COH>(U4 + ou + LPR * v, a[v]);
                store4<COH>(V4 + oi + LPR * v, c[v]);
            }
        } else {
            float part = 0.0f;
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                part += pu[v].x * qi[v].x;
                part += pu[v].y * qi[v].y;
                part += pu[v].z * qi[v].z;
                part += pu[v].w * qi[v].w;
            }
            part = group_sum<LPR>(part);
            const RatingStep<LOSS> st(s, part, bu_u, bi_i, r, cnt_u, cnt_i, u, i);
            if (biased && q == 0) {
                if constexpr (BTH)
                    __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, st.new_bu),
                                                          burs, (uint32_t)u * 4u, 0, 16);
                else
                    store1<COH>(bu + u, st.new_bu);
                store1<COH>(bi + i, st.new_bi);
            }
#pragma unroll
            for (int v = 0; v < VPL; ++v) {
                const float4 a = pu[v], c = qi[v];
                const float4 nu = make_float4(st.new_u(s, a.x, c.x), st.new_u(s, a.y, c.y),
                                              st.new_u(s, a.z, c.z), st.new_u(s, a.w, c.w));
                if constexpr (UTH)
                    __builtin_amdgcn_raw_buffer_store_b128(
                        __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, nu), urs,
                        (uint32_t)(ou + LPR * v) * 16u, 0, 16);
                else
                    store4<COH>(U4 + ou + LPR * v, nu);
                store4<COH>(V4 + oi + LPR * v,
                            make_float4(st.new_i(s, a.x, c.x), st.new_i(s, a.y, c.y),
                                        st.new_i(s, a.z, c.z), st.new_i(s, a.w, c.w)));
            }
        }
    };
    for (int64_t base = begin; base < end; base += 64) {
        if constexpr ((AM & kAccFlush) != 0)
            if (flusher) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
        // 64 ratings of the stream: three coalesced 256-B loads, then broadcast per group
        const int64_t idx = base + lane;
        const bool in = idx < end;
        const int32_t my_u = in ? su[idx] : 0;
        const int32_t my_i = in ? si[idx] : 0;
        const float my_r = in ? sr[idx] : 0.0f;
        // consume the three loads here: otherwise the wait for them lands at the top of the
        // step loop, where the in-order counter makes it a wait for the previous step's stores
        asm volatile("" ::"v"(my_u), "v"(my_i), "v"(my_r));
        const int cnt = (int)min((int64_t)64, end - base);
        // (requesting step t + 1's rows before step t's stores was measured 4 % slower on C2)
#if defined(MML_HOGWILD_PF) && MML_HOGWILD_PF
        // (experiments: the same again with the user phases, step t + 1's rows before step t's
        // update)
        {
            float4 pu[VPL], qi[VPL];
            float bu_u = 0.0f, bi_i = 0.0f;
            int32_t u = group_fetch<LPR>(my_u, 0, lane), i = group_fetch<LPR>(my_i, 0, lane);
            float r = group_fetch<LPR>(my_r, 0, lane);
            if (sub < cnt) fetch(u, i, pu, qi, bu_u, bi_i);
            for (int step = 0; step < cnt; step += RPW) {
                const int src = step + sub, nstep = step + RPW;
                float4 pn[VPL], qn[VPL];
                float bun = 0.0f, bin = 0.0f;
                int32_t un = 0, in_ = 0;
                float rn = 0.0f;
                if (nstep < cnt) {
                    un = group_fetch<LPR>(my_u, nstep, lane);
                    in_ = group_fetch<LPR>(my_i, nstep, lane);
                    rn = group_fetch<LPR>(my_r, nstep, lane);
                    if (nstep + sub < cnt) fetch(un, in_, pn, qn, bun, bin);
                }
                if (src < cnt) apply(u, i, r, pu, qi, bu_u, bi_i);
                u = un;
                i = in_;
                r = rn;
                bu_u = bun;
                bi_i = bin;
#pragma unroll
                for (int v = 0; v < VPL; ++v) {
                    pu[v] = pn[v];
                    qi[v] = qn[v];
                }
            }
        }
        continue;
#endif
        for (int step = 0; step < cnt; step += RPW) {
            const int src = step + sub;
            // lanes past cnt read lane min(src, 63): a real (loaded or zeroed) entry, unused
            const int32_t u = group_fetch<LPR>(my_u, step, lane);
            const int32_t i = group_fetch<LPR>(my_i, step, lane);
            const float r = group_fetch<LPR>(my_r, step, lane);
            if (src < cnt) {
                float4 pu[VPL], qi[VPL];
                float bu_u, bi_i;
                fetch(u, i, pu, qi, bu_u, bi_i);
                apply(u, i, r, pu, qi, bu_u, bi_i);
            }
        }
    }
}

// HOGWILD in user runs (mml_bmf_set_hogwild_runs, ABI 14).  Each XCD group's span is sorted by
// user (ensure_runs: stable, so a user's ratings keep their visit order), so a user's ratings of
// one group form a run.  Every lane group (LPR lanes, one rating at a time) walks its own
// contiguous slice of the wave's chunk, both slice ends moved to run starts, so a run belongs to
// one lane group: U_u and b_u are loaded once at the run's start (write-through mode, past any
// stale L2 copy), updated in registers rating after rating -- the reference's sequential
// arithmetic within the run -- and written through once at its end.  The item rows and biases
// keep the XCD-owned L2-served accesses and the racy Hogwild stores.  Where the phase schedule
// moves every rating's U row through the L2 twice (read, dirty write-back), a run moves it once
// each way.  A user's runs of the 8 groups must never be in flight at once (one write-back would
// drop the other's updates), so the epoch runs as 8 launches over DSGD-like strata: users in 8
// blocks of equal rating count, launch s gives group g the ratings of user block (g + s) mod 8
// (ensure_runs), so no two XCDs ever hold rows of one user block.
//
// A lane group's slice of a stratum's span: [b, e) of its wave's chunk, both ends moved to run
// starts (the same move for the slices on both sides of a bound, so every run has exactly one
// owner), walked in order.
struct RunSlice {
    int64_t b, e;
    __device__ __forceinline__ int64_t at(int64_t t) const { return b + t; }
};
template <int RPW>
__device__ __forceinline__ RunSlice run_slice(const int32_t* __restrict__ su, int64_t g0,
                                              int64_t g1, const mml::GroupWave& gw, int sub) {
    const int64_t per = (gw.end - gw.begin + RPW - 1) / RPW;
    auto run_start = [&](int64_t x) {
        while (x > g0 && x < g1 && su[x] == su[x - 1]) ++x;
        return x;
    };
    return RunSlice{run_start(min(gw.begin + sub * per, gw.end)),
                    run_start(min(gw.begin + (sub + 1) * per, gw.end))};
}

#ifndef MML_RUNS_PF  // (experiments: A/B) the next step's item row requested a step ahead
#define MML_RUNS_PF 0
#endif
#ifndef MML_RUNS_WPE  // (experiments: A/B) the runs kernel's waves-per-SIMD bound
#define MML_RUNS_WPE 1
#endif
template <int LOSS, int LPR, int AM>
__global__ __launch_bounds__(256, MML_RUNS_WPE) void bmf_sgd_runs_kernel(
    const int32_t* __restrict__ su, const int32_t* __restrict__ si, const float* __restrict__ sr,
    const int64_t* __restrict__ spans, int32_t waves_per_group, float* U, float* V,
    float* bu, float* bi, int32_t ld4, uint32_t v_bytes, uint32_t bi_bytes, uint32_t u_bytes,
    uint32_t bu_bytes, int32_t flushers, BmfScalars s, const int32_t* __restrict__ cnt_u,
    const int32_t* __restrict__ cnt_i) {
    static_assert(LPR >= 1 && LPR <= 64, "lanes per rating");
    constexpr int RPW = 64 / LPR;  // lane groups (runs in flight) per wave
    constexpr bool IL2 = (AM & kAccItemL2) != 0, UTH = (AM & kAccUserThru) != 0;
    constexpr bool biased = LOSS != kPlainMF;
    const int lane = threadIdx.x & 63;
    const int wib = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);
    // this launch's stratum of group grp: [spans[2 grp], spans[2 grp + 1]) (ensure_runs), cut
    // into the group's waves as mml::group_wave cuts a span
    const int grp = (int)(blockIdx.x % 8u);
    const int64_t g0 = spans[2 * grp], g1 = spans[2 * grp + 1];
    mml::GroupWave gw;
    {
        const int64_t w = (int64_t)(blockIdx.x / 8u) * (blockDim.x >> 6) + wib;
        const int64_t chunk = (g1 - g0 + waves_per_group - 1) / waves_per_group;
        gw.begin = min(g0 + w * chunk, g1);
        gw.end = min(gw.begin + chunk, g1);
    }
    const int sub = lane / LPR, q = lane % LPR;
    float4* U4 = reinterpret_cast<float4*>(U);
    float4* V4 = reinterpret_cast<float4*>(V);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t vrs = mml::buffer_rsrc(V, v_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t brs = mml::buffer_rsrc(bi, bi_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t urs = mml::buffer_rsrc(U, u_bytes);
    [[maybe_unused]] const __amdgpu_buffer_rsrc_t burs = mml::buffer_rsrc(bu, bu_bytes);
    [[maybe_unused]] const bool flusher =
        (AM & kAccFlush) != 0 && (threadIdx.x >> 6) == 0 &&
        (blockIdx.x >> 3) % max(1u, (gridDim.x >> 3) / (uint32_t)flushers) == 0;
    const RunSlice sl = run_slice<RPW>(su, g0, g1, gw, sub);
    const int64_t b = sl.b, e = sl.e, len = e - b;
    // the wave's trip count: the longest slice (wave-uniform)
    int64_t steps = len;
#pragma unroll
    for (int o = LPR; o < 64; o <<= 1) steps = max(steps, (int64_t)__shfl_xor((long long)steps, o));
    steps = __builtin_amdgcn_readfirstlane((int)steps);
    int32_t cur = -1;
    float4 pu = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float bu_u = 0.0f;
    const int64_t ou0 = q;  // this lane's float4 of a row
    auto put_user = [&]() {  // the run's U_u and b_u, written through
        const int64_t ou = (int64_t)cur * ld4 + ou0;
        if constexpr (UTH)
            __builtin_amdgcn_raw_buffer_store_b128(
                __builtin_bit_cast(__attribute__((ext_vector_type(4))) uint32_t, pu), urs,
                (uint32_t)ou * 16u, 0, 16);
        else
            store4<false>(U4 + ou, pu);
        if (biased && q == 0) {
            if constexpr (UTH)
                __builtin_amdgcn_raw_buffer_store_b32(__builtin_bit_cast(uint32_t, bu_u), burs,
                                                      (uint32_t)cur * 4u, 0, 16);
            else
                bu[cur] = bu_u;
        }
    };
    int32_t my_u = 0, my_i = 0;
    float my_r = 0.0f;
#if MML_RUNS_PF
    float4 qn = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    float bn = 0.0f;
    bool have = false;
#endif
    for (int64_t t = 0; t < steps; ++t) {
        if ((t % LPR) == 0) {
            if constexpr ((AM & kAccFlush) != 0)
                if (flusher) __builtin_amdgcn_fence(__ATOMIC_RELEASE, "agent");
            // the next LPR entries of every slice, one per lane of its group, in walk order
            const bool in = t + q < len;
            const int64_t x = sl.at(t + q);
            my_u = in ? su[x] : -1;
            my_i = in ? si[x] : 0;
            my_r = in ? sr[x] : 0.0f;
        }
        const int src = sub * LPR + (int)(t % LPR);
        const int32_t u = __shfl(my_u, src);
        const int32_t i = __shfl(my_i, src);
        const float r = __shfl(my_r, src);
        if (u < 0) continue;  // this slice is done (lane-group divergent)
        if (u != cur) {  // a run starts: the previous one's row goes out, this one's comes in
            if (cur >= 0) put_user();
            cur = u;
            const int64_t ou = (int64_t)u * ld4 + ou0;
            if constexpr (UTH) pu = mml::load4_l2(urs, (uint32_t)ou * 16u);
            else pu = U4[ou];
            if constexpr (biased) {
                if constexpr (UTH) bu_u = mml::load1_l2(burs, (uint32_t)u * 4u);
                else bu_u = bu[u];
            }
        }
        const int64_t oi = (int64_t)i * ld4 + ou0;
        float4 qi;
        float bi_i = 0.0f;
        auto load_item = [&](int32_t it, float4& q4, float& b1) {
            const int64_t o = (int64_t)it * ld4 + ou0;
            if constexpr (IL2) q4 = mml::load4_l2(vrs, (uint32_t)o * 16u);
            else q4 = V4[o];
            if constexpr (biased) {
                if constexpr (IL2) b1 = mml::load1_l2(brs, (uint32_t)it * 4u);
                else b1 = bi[it];
            }
        };
#if MML_RUNS_PF
        // the row of this step came with the previous one (same staged block); the next step's is
        // requested now, ahead of this step's arithmetic and stores
        if (have) {
            qi = qn;
            bi_i = bn;
        } else {
            load_item(i, qi, bi_i);
        }
        have = false;
        int32_t inx = -1;
        if ((int)((t + 1) % LPR) != 0 && t + 1 < len) {
            inx = __shfl(my_i, src + 1);
            load_item(inx, qn, bn);
            have = true;
        }
#else
        load_item(i, qi, bi_i);
#endif
        if constexpr (LOSS == kReplayTraffic) {
            asm volatile("" : "+v"(qi.x), "+v"(qi.y), "+v"(qi.z), "+v"(qi.w), "+v"(bi_i) : "v"(r));
            if (q == 0) bi[i] = bi_i;
            V4[oi] = qi;
        } else {
            float part = ((pu.x * qi.x + pu.y * qi.y) + pu.z * qi.z) + pu.w * qi.w;
            part = group_sum<LPR>(part);
            const RatingStep<LOSS> st(s, part, bu_u, bi_i, r, cnt_u, cnt_i, u, i);
            if (biased) {
                bu_u = st.new_bu;
                if (q == 0) bi[i] = st.new_bi;
            }
            const float4 nv = make_float4(st.new_i(s, pu.x, qi.x), st.new_i(s, pu.y, qi.y),
                                          st.new_i(s, pu.z, qi.z), st.new_i(s, pu.w, qi.w));
            V4[oi] = nv;
            pu = make_float4(st.new_u(s, pu.x, qi.x), st.new_u(s, pu.y, qi.y),
                             st.new_u(s, pu.z, qi.z), st.new_u(s, pu.w, qi.w));
#if MML_RUNS_PF
            if (inx == i) {  // the same item next (a repeated rating): this step's new row
                qn = nv;
                if (biased) bn = st.new_bi;
            }
#endif
        }
    }
    if (cur >= 0) put_user();
}

// BiasedMatrixFactorization.Predict(int,int) (:313-325): double score, float dot in order.
// plain: MatrixFactorization.Predict(int,int) (MatrixFactorization.cs:251-258 + :205-217):
// global_bias for ids beyond the model, else global_bias + dot clipped to [min, max].
__device__ __forceinline__ float bmf_predict1(int32_t u, int32_t i, int32_t n_users,
                                              int32_t n_items, const float* U, const float* V,
                                              const float* bu, const float* bi, int32_t k,
                                              int32_t ld, float gb, float min_rating,
                                              float max_rating, int kind) {
    const bool plain = kind == 1;
    const bool ku = u >= 0 && u < n_users, ki = i >= 0 && i < n_items;
    float dot = 0.0f;
    if (ku && ki) {
        const float* a = U + (int64_t)u * ld;
        const float* c = V + (int64_t)i * ld;
        for (int f = 0; f < k; ++f) dot += a[f] * c[f];
    }
    if (plain) {
        if (!(ku && ki)) return gb;
        float r = gb + dot;
        r = r > max_rating ? max_rating : r;
        return r < min_rating ? min_rating : r;
    }
    double score = (double)gb;
    if (ku) score += (double)bu[u];
    if (ki) score += (double)bi[i];
    if (ku && ki) score += (double)dot;
    if (kind == 2) {  // SVDPlusPlus.Predict (SVDPlusPlus.cs:106-126): no sigmoid, clamped
        if (score > (double)max_rating) return max_rating;
        if (score < (double)min_rating) return min_rating;
        return (float)score;
    }
    const float range = max_rating - min_rating;
    return (float)((double)min_rating + (1.0 / (1.0 + exp(-score))) * (double)range);
}

__global__ __launch_bounds__(256) void bmf_predict_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items, int64_t n,
    int32_t n_users, int32_t n_items, const float* __restrict__ U, const float* __restrict__ V,
    const float* __restrict__ bu, const float* __restrict__ bi, int32_t k, int32_t ld, float gb,
    float min_rating, float max_rating, int32_t plain, float* __restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = bmf_predict1(users[x], items[x], n_users, n_items, U, V, bu, bi, k, ld, gb,
                              min_rating, max_rating, plain);
}

// Eval.Ratings.Evaluate (:96-139): float error, float square, double sums; per-block partials.
__global__ __launch_bounds__(256) void bmf_eval_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items,
    const float* __restrict__ values, int64_t n, int32_t n_users, int32_t n_items,
    const float* __restrict__ U, const float* __restrict__ V, const float* __restrict__ bu,
    const float* __restrict__ bi, int32_t k, int32_t ld, float gb, float min_rating,
    float max_rating, int32_t plain, double* __restrict__ partials) {
    double se = 0.0, ae = 0.0;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const float p = bmf_predict1(users[x], items[x], n_users, n_items, U, V, bu, bi, k, ld,
                                     gb, min_rating, max_rating, plain);
        const float e = p - values[x];
        se += (double)(e * e);
        ae += (double)fabsf(e);
    }
    __shared__ double s_se[256], s_ae[256];
    s_se[threadIdx.x] = se;
    s_ae[threadIdx.x] = ae;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) {
            s_se[threadIdx.x] += s_se[threadIdx.x + w];
            s_ae[threadIdx.x] += s_ae[threadIdx.x + w];
        }
        __syncthreads();
    }
    if (threadIdx.x == 0) {
        partials[2 * blockIdx.x] = s_se[0];
        partials[2 * blockIdx.x + 1] = s_ae[0];
    }
}

// ComputeLoss (:496-514): RMSE.ComputeSquaredErrorSum / MAE.ComputeAbsoluteErrorSum /
// LogisticLoss.ComputeSum over the training ratings, double sums, per-block partials.
__global__ __launch_bounds__(256) void bmf_loss_kernel(
    const int32_t* __restrict__ users, const int32_t* __restrict__ items,
    const float* __restrict__ values, int64_t n, int32_t n_users, int32_t n_items,
    const float* __restrict__ U, const float* __restrict__ V, const float* __restrict__ bu,
    const float* __restrict__ bi, int32_t k, int32_t ld, float gb, float min_rating,
    float max_rating, int32_t loss_kind, double* __restrict__ partials) {
    const float range = max_rating - min_rating;
    double acc = 0.0;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const float p = bmf_predict1(users[x], items[x], n_users, n_items, U, V, bu, bi, k, ld,
                                     gb, min_rating, max_rating, false);
        if (loss_kind == MML_LOSS_RMSE) {
            const double d = (double)(p - values[x]);  // float difference, Math.Pow in double
            acc += d * d;
        } else if (loss_kind == MML_LOSS_MAE) {
            acc += fabs((double)(p - values[x]));
        } else {
            double pr = ((double)p - (double)min_rating) / (double)range;
            pr = pr < 0.0 ? 0.0 : (pr > 1.0 ? 1.0 : pr);
            const double act = (double)((values[x] - min_rating) / range);  // float arithmetic
            acc -= act * log(pr);
            acc -= (1 - act) * log(1 - pr);
        }
    }
    __shared__ double sh[256];
    sh[threadIdx.x] = acc;
    __syncthreads();
    for (int w = 128; w > 0; w >>= 1) {
        if ((int)threadIdx.x < w) sh[threadIdx.x] += sh[threadIdx.x + w];
        __syncthreads();
    }
    if (threadIdx.x == 0) partials[blockIdx.x] = sh[0];
}

// ComputeObjective's complexity term (:518-550) over the user rows then the item rows:
// Math.Pow(EuclideanNorm(row), 2) in double; weights count * reg (float, C# int * float) or
// reg / sqrt(count) with FrequencyRegularization.  One wavefront per row, per-block partials.
__global__ __launch_bounds__(256) void bmf_complexity_kernel(
    const float* __restrict__ U, const float* __restrict__ V, const float* __restrict__ bu,
    const float* __restrict__ bi, const int32_t* __restrict__ cnt_u,
    const int32_t* __restrict__ cnt_i, int32_t n_users, int32_t n_items, int32_t k, int32_t ld,
    float reg_u, float reg_i, float bias_reg, int32_t freq, double* __restrict__ partials) {
    const int lane = threadIdx.x & 63, wave = threadIdx.x >> 6;
    double acc = 0.0;
    const int64_t rows = (int64_t)n_users + n_items;
    for (int64_t r = (int64_t)blockIdx.x * 4 + wave; r < rows; r += (int64_t)gridDim.x * 4) {
        const bool user = r < n_users;
        const int64_t row = user ? r : r - n_users;
        const float* M = (user ? U : V) + row * ld;
        double sq = 0.0;
        for (int f = lane; f < k; f += 64) sq += (double)M[f] * (double)M[f];
        for (int o = 32; o > 0; o >>= 1) sq += __shfl_xor(sq, o);
        if (lane == 0) {
            const double norm2 = pow(sqrt(sq), 2.0);
            const int32_t c = user ? cnt_u[row] : cnt_i[row];
            const float reg = user ? reg_u : reg_i;
            const double b = (double)(user ? bu[row] : bi[row]);
            if (freq) {
                if (c > 0) {
                    const double w = (double)reg / sqrt((double)c);
                    acc += w * norm2;
                    acc += w * (double)bias_reg * (b * b);
                }
            } else {
                const float w = (float)c * reg, wb = (float)c * reg * bias_reg;
                acc += (double)w * norm2;
                acc += (double)wb * (b * b);
            }
        }
    }
    __shared__ double sh[4];
    if (lane == 0) sh[wave] = acc;
    __syncthreads();
    if (threadIdx.x == 0) partials[blockIdx.x] = (sh[0] + sh[1]) + (sh[2] + sh[3]);
}

// ---------------------------------------------------------------- fold-in (IFoldInRatingPredictor)
struct FoldScalars {
    float gb, min_rating, range, lr, blr, bias_reg, reg_u, decay;
    int32_t freq;
};

// BiasedMatrixFactorization.FoldIn (:447-492) / MatrixFactorization.FoldIn (MatrixFactorization.cs:
// 326-351, LOSS = kPlainMF) for fold-in user blockIdx.x: one wavefront, lane f owns factors
// f, f + 64, ...; the item-row dot is summed left to right via v_readlane (RowScalarProduct,
// DataType/MatrixExtensions.cs:183-196); the bias step and factor deltas are the reference's float
// expressions.  out: (bias, factors) rows of k + 1 (biased) or factor rows of k (plain).
template <int LOSS, int KM>
__global__ __launch_bounds__(64) void bmf_fold_in_kernel(
    const int64_t* __restrict__ off, const int32_t* __restrict__ items,
    const float* __restrict__ values, int32_t num_iter, const float* __restrict__ V,
    const float* __restrict__ bi, int32_t k, int32_t ld, FoldScalars s,
    const float* __restrict__ init, float* __restrict__ out) {
    constexpr bool plain = LOSS == kPlainMF;
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int64_t begin = off[b], end = off[b + 1];
    float fac[KM];
#pragma unroll
    for (int m = 0; m < KM; ++m) {
        const int f = lane + 64 * m;
        fac[m] = f < k ? init[b * k + f] : 0.0f;
    }
    const float reg_weight =
        (!plain && s.freq) ? (float)((double)s.reg_u / sqrt((double)(end - begin))) : s.reg_u;
    float ub = 0.0f;
    double lr = (double)s.lr;
    for (int32_t it = 0; it < num_iter; ++it) {
        for (int64_t x = begin; x < end; ++x) {
            const int32_t i = items[x];
            const float* Vi = V + (int64_t)i * ld;
            float vi[KM];
            float dot = 0.0f;
#pragma unroll
            for (int m = 0; m < KM; ++m) {
                const int f = lane + 64 * m;
                vi[m] = f < k ? Vi[f] : 0.0f;
                const int bits = __float_as_int(vi[m] * fac[m]);
                const int lim = min(64, k - 64 * m);
                for (int l = 0; l < lim; ++l)
                    dot += __int_as_float(__builtin_amdgcn_readlane(bits, l));
            }
            if constexpr (plain) {
                const float err = values[x] - (s.gb + dot);
#pragma unroll
                for (int m = 0; m < KM; ++m)
                    fac[m] += (float)(lr * (double)(err * vi[m] - s.reg_u * fac[m]));
            } else {
                const double score = (double)(((s.gb + ub) + bi[i]) + dot);
                const double sig = 1.0 / (1.0 + exp(-score));
                const double err =
                    (double)values[x] - ((double)s.min_rating + sig * (double)s.range);
                const float g = gradient_common<LOSS>(sig, err, s.range);
                ub += s.blr * (g - s.bias_reg * reg_weight * ub);
#pragma unroll
                for (int m = 0; m < KM; ++m)
                    fac[m] += (float)(lr * (double)(g * vi[m] - reg_weight * fac[m]));
            }
        }
        if constexpr (plain) lr *= (double)s.decay;
    }
    const int64_t w = plain ? k : k + 1;
    float* o = out + b * w + (plain ? 0 : 1);
    if (!plain && lane == 0) out[b * w] = ub;
#pragma unroll
    for (int m = 0; m < KM; ++m) {
        const int f = lane + 64 * m;
        if (f < k) o[f] = fac[m];
    }
}

// RetrainUser / RetrainItem (MatrixFactorization.cs:142-160, BiasedMatrixFactorization.cs:419-431)
// for row rows[blockIdx.x] of side SIDE (0: a user row of U, 1: an item row of V): bias <- 0, the
// factors <- init (RowInitNormal's draws), then num_iter x Iterate(ByUser[u] / ByItem[i],
// update_user = SIDE == 0, update_item = SIDE == 1) (:264-310 / MatrixFactorization.cs:166-196)
// over the row's ratings in index order, with the other side fixed.  Rows of one side are therefore
// independent: one wavefront per row, lane f owning factors f, f + 64, ...; the arithmetic is the
// ORDERED kernel's (RowScalarProduct left to right via v_readlane, RatingStep's float/double mix).
// Frequency regularisation reads count_by_user[u] (count_by_item[i]) = the row's own list length.
// lrs[blockIdx.x * num_iter + it] = current_learnrate of that Iterate call.
template <int LOSS, int KM, int SIDE>
__global__ __launch_bounds__(64) void bmf_retrain_kernel(
    const int32_t* __restrict__ rows, const int64_t* __restrict__ off,
    const int32_t* __restrict__ other, const float* __restrict__ values,
    const float* __restrict__ init, const float* __restrict__ lrs, int32_t num_iter, float* U,
    float* V, float* bu, float* bi, int32_t k, int32_t ld, BmfScalars s, float bias_learn_rate,
    int32_t freq) {
    constexpr bool plain = LOSS == kPlainMF;
    const int lane = threadIdx.x;
    const int64_t b = blockIdx.x;
    const int32_t row = rows[b];
    const int64_t begin = off[b], end = off[b + 1];
    float* own = (SIDE == 0 ? U : V) + (int64_t)row * ld;
    const float* oth = SIDE == 0 ? V : U;
    const float* obias = SIDE == 0 ? bi : bu;
    float fac[KM];
#pragma unroll
    for (int m = 0; m < KM; ++m) {
        const int f = lane + 64 * m;
        fac[m] = f < k ? init[b * k + f] : 0.0f;
    }
    const float reg0 = SIDE == 0 ? s.reg_u : s.reg_i;
    // FrequencyRegularization (:281-282) with the whole data set's count of this row
    const float reg = (!plain && freq) ? (float)((double)reg0 / sqrt((double)(end - begin))) : reg0;
    float ob = 0.0f;  // the row's own bias, reset by RetrainUser / RetrainItem
    for (int32_t it = 0; it < num_iter; ++it) {
        const float lr = lrs[b * num_iter + it];
        const float blr = bias_learn_rate * lr;
        for (int64_t x = begin; x < end; ++x) {
            const int32_t o = other[x];
            const float* Ro = oth + (int64_t)o * ld;
            float ro[KM];
            float dot = 0.0f;
#pragma unroll
            for (int m = 0; m < KM; ++m) {
                const int f = lane + 64 * m;
                ro[m] = f < k ? Ro[f] : 0.0f;
                // RowScalarProduct(user_factors, u, item_factors, i): U_u[f] * V_i[f]
                const int bits = __float_as_int(SIDE == 0 ? fac[m] * ro[m] : ro[m] * fac[m]);
                const int lim = min(64, k - 64 * m);
                for (int l = 0; l < lim; ++l)
                    dot += __int_as_float(__builtin_amdgcn_readlane(bits, l));
            }
            if constexpr (plain) {
                const float err = values[x] - (s.gb + dot);
#pragma unroll
                for (int m = 0; m < KM; ++m)
                    fac[m] += (float)((double)lr * (double)(err * ro[m] - reg * fac[m]));
            } else {
                const float bu_u = SIDE == 0 ? ob : obias[o], bi_i = SIDE == 0 ? obias[o] : ob;
                const double score = (double)(((s.gb + bu_u) + bi_i) + dot);
                const double sig = 1.0 / (1.0 + exp(-score));
                const double err =
                    (double)values[x] - ((double)s.min_rating + sig * (double)s.range);
                const float g = gradient_common<LOSS>(sig, err, s.range);
                ob = ob + blr * (g - (s.bias_reg * reg) * ob);
#pragma unroll
                for (int m = 0; m < KM; ++m) {
                    const double delta = (double)g * (double)ro[m] - (double)reg * (double)fac[m];
                    fac[m] += (float)((double)lr * delta);
                }
            }
        }
    }
    if (!plain && lane == 0) (SIDE == 0 ? bu : bi)[row] = ob;
#pragma unroll
    for (int m = 0; m < KM; ++m) {
        const int f = lane + 64 * m;
        if (f < k) own[f] = fac[m];
    }
}

// Predict(float[] user_vector, int item_id) for (vector, item) pairs: BiasedMatrixFactorization
// (:327-335) or, plain, MatrixFactorization's bound form (MatrixFactorization.cs:222-241).
__global__ __launch_bounds__(256) void bmf_predict_vectors_kernel(
    const float* __restrict__ vec, const int32_t* __restrict__ vidx,
    const int32_t* __restrict__ items, int64_t n, int32_t n_items, const float* __restrict__ V,
    const float* __restrict__ bi, int32_t k, int32_t ld, float gb, float min_rating,
    float max_rating, int32_t plain, float* __restrict__ out) {
    const int64_t w = plain ? k : k + 1;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const float* uv = vec + (int64_t)vidx[x] * w;
        const int32_t i = items[x];
        if (plain) {
            float dot = 0.0f;
            for (int f = 0; f < k; ++f) dot += V[(int64_t)i * ld + f] * uv[f];
            float r = gb + dot;
            r = r > max_rating ? max_rating : r;
            out[x] = r < min_rating ? min_rating : r;
            continue;
        }
        double score = (double)(gb + uv[0]);
        if (i < n_items) {
            float dot = 0.0f;
            for (int f = 0; f < k; ++f) dot += V[(int64_t)i * ld + f] * uv[1 + f];
            score += (double)(bi[i] + dot);
        }
        const float range = max_rating - min_rating;
        out[x] = (float)((double)min_rating + 1.0 / (1.0 + exp(-score)) * (double)range);
    }
}

// ---------------------------------------------------------------- SocialMF (IterateBatch)
// SocialMF.IterateBatch (SocialMF.cs:77-194) restated as a deterministic device batch step: every
// gradient element accumulates in the reference's order (ratings in visit order per user / item,
// then L2, then the social terms), so the step is bit-faithful up to libm-vs-ocml exp rounding.

// I.1 (:89-102): per rating of the stream, the loss gradient g[x] (float score, float
// prediction, error = prediction - rating)
template <int LOSS>
__global__ __launch_bounds__(256) void smf_error_kernel(
    const int32_t* __restrict__ su, const int32_t* __restrict__ si, const float* __restrict__ sr,
    int64_t n, const float* __restrict__ U, const float* __restrict__ V,
    const float* __restrict__ bu, const float* __restrict__ bi, int32_t k, int32_t ld, float gb,
    float min_rating, float range, float* __restrict__ g) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = su[x], i = si[x];
        float score = (gb + bu[u]) + bi[i];
        const float* a = U + (int64_t)u * ld;
        const float* c = V + (int64_t)i * ld;
        float dot = 0.0f;
        for (int f = 0; f < k; ++f) dot += a[f] * c[f];
        score += dot;
        const double sig = 1.0 / (1.0 + exp(-(double)score));
        const float prediction = (float)((double)min_rating + sig * (double)range);
        g[x] = gradient_common<LOSS>(sig, (double)(prediction - sr[x]), range);
    }
}

__device__ __forceinline__ int64_t smf_row_len(const int64_t* off, int32_t n_rows, int32_t r) {
    return r < n_rows ? off[r + 1] - off[r] : 0;
}

// User gradient, one wavefront per user, lane f owns factors f, f + 64, ... (KM per lane):
// I.1 over the user's ratings in visit order (pos CSR), I.2 (:119-126), I.3 (:133-177).
template <int KM>
__global__ __launch_bounds__(64) void smf_user_grad_kernel(
    const int64_t* __restrict__ pos_off, const int32_t* __restrict__ pos,
    const int32_t* __restrict__ si, const float* __restrict__ g, const float* __restrict__ U,
    const float* __restrict__ V, const float* __restrict__ bu, int32_t k, int32_t ld,
    float reg_u, float bias_reg, float soc, const int64_t* __restrict__ conn_off,
    const int32_t* __restrict__ conn_cols, int32_t n_conn, const int64_t* __restrict__ rev_off,
    const int32_t* __restrict__ rev_cols, int32_t n_rev, float* __restrict__ Ug,
    float* __restrict__ bug) {
    const int lane = threadIdx.x;
    const int32_t u = blockIdx.x;
    float acc[KM], tmp[KM];
    float bacc = 0.0f;
#pragma unroll
    for (int m = 0; m < KM; ++m) acc[m] = 0.0f;
    auto row = [&](const float* M, int32_t r, int m) {
        const int f = lane + 64 * m;
        return f < k ? M[(int64_t)r * ld + f] : 0.0f;
    };
    for (int64_t p = pos_off[u]; p < pos_off[u + 1]; ++p) {
        const int32_t x = pos[p];
        const float gx = g[x];
        const int32_t i = si[x];
        bacc += gx;
#pragma unroll
        for (int m = 0; m < KM; ++m) acc[m] += gx * row(V, i, m);
    }
    bacc += bu[u] * reg_u * bias_reg;
#pragma unroll
    for (int m = 0; m < KM; ++m) acc[m] += row(U, u, m) * reg_u;
    if (soc != 0.0f) {
        const int64_t num = smf_row_len(conn_off, n_conn, u);
        float bsum = 0.0f;
#pragma unroll
        for (int m = 0; m < KM; ++m) tmp[m] = 0.0f;
        for (int64_t x = 0; x < num; ++x) {
            const int32_t v = conn_cols[conn_off[u] + x];
            bsum += bu[v];
#pragma unroll
            for (int m = 0; m < KM; ++m) tmp[m] += row(U, v, m);
        }
        if (num != 0) {
            bacc += soc * (bu[u] - bsum / (float)num);
#pragma unroll
            for (int m = 0; m < KM; ++m) acc[m] += soc * (row(U, u, m) - tmp[m] / (float)num);
        }
        const int64_t nrev = smf_row_len(rev_off, n_rev, u);
        for (int64_t y = 0; y < nrev; ++y) {
            const int32_t v = rev_cols[rev_off[u] + y];
            const int64_t cv = smf_row_len(conn_off, n_conn, v);
            const float trust = 1.0f / (float)cv;
            const float neg = -soc * trust;
            float bd = 0.0f;
#pragma unroll
            for (int m = 0; m < KM; ++m) tmp[m] = 0.0f;
            for (int64_t x = 0; x < cv; ++x) {
                const int32_t w = conn_cols[conn_off[v] + x];
                bd -= bu[w];
#pragma unroll
                for (int m = 0; m < KM; ++m) tmp[m] -= row(U, w, m);
            }
            bd *= trust;
            bd += bu[v];
            bacc += neg * bd;
#pragma unroll
            for (int m = 0; m < KM; ++m) {
                tmp[m] *= trust;
                tmp[m] += row(U, v, m);
                acc[m] += neg * tmp[m];
            }
        }
    }
#pragma unroll
    for (int m = 0; m < KM; ++m) {
        const int f = lane + 64 * m;
        if (f < k) Ug[(int64_t)u * ld + f] = acc[m];
    }
    if (lane == 0) bug[u] = bacc;
}

// Item gradient, one wavefront per item: I.1 in visit order, then I.2 (:121-130)
template <int KM>
__global__ __launch_bounds__(64) void smf_item_grad_kernel(
    const int64_t* __restrict__ pos_off, const int32_t* __restrict__ pos,
    const int32_t* __restrict__ su, const float* __restrict__ g, const float* __restrict__ U,
    const float* __restrict__ V, const float* __restrict__ bi, int32_t k, int32_t ld,
    float reg_i, float bias_reg, float* __restrict__ Vg, float* __restrict__ big) {
    const int lane = threadIdx.x;
    const int32_t i = blockIdx.x;
    float acc[KM];
    float bacc = 0.0f;
#pragma unroll
    for (int m = 0; m < KM; ++m) acc[m] = 0.0f;
    for (int64_t p = pos_off[i]; p < pos_off[i + 1]; ++p) {
        const int32_t x = pos[p];
        const float gx = g[x];
        const int32_t u = su[x];
        bacc += gx;
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            acc[m] += gx * (f < k ? U[(int64_t)u * ld + f] : 0.0f);
        }
    }
    bacc += bi[i] * reg_i * bias_reg;
#pragma unroll
    for (int m = 0; m < KM; ++m) {
        const int f = lane + 64 * m;
        if (f < k) Vg[(int64_t)i * ld + f] = acc[m] + V[(int64_t)i * ld + f] * reg_i;
    }
    if (lane == 0) big[i] = bacc;
}

// II (:180-193): M += G * (-LearnRate) (Multiply then Inc), b -= g * LearnRate * BiasLearnRate
__global__ __launch_bounds__(256) void smf_apply_kernel(float* __restrict__ M,
                                                        const float* __restrict__ G, int64_t n,
                                                        float* __restrict__ b,
                                                        const float* __restrict__ gb, int64_t nb,
                                                        float lr, float blr) {
    const float neg = -lr;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n;
         e += (int64_t)gridDim.x * blockDim.x)
        M[e] += G[e] * neg;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < nb;
         e += (int64_t)gridDim.x * blockDim.x)
        b[e] -= gb[e] * lr * blr;
}

__global__ __launch_bounds__(256) void smf_iota_kernel(int32_t* __restrict__ a, int64_t n) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        a[x] = (int32_t)x;
}

__global__ __launch_bounds__(256) void smf_widen_kernel(const int32_t* __restrict__ c, int32_t n,
                                                        int64_t* __restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = c[x];
}

// stream[x] = raw[order[x]] for the three SoA columns
__global__ __launch_bounds__(256) void gather_stream_kernel(
    const int32_t* __restrict__ ru, const int32_t* __restrict__ ri, const float* __restrict__ rr,
    const int32_t* __restrict__ order, int64_t n, int32_t* __restrict__ su,
    int32_t* __restrict__ si, float* __restrict__ sr) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int64_t o = order ? order[x] : x;
        su[x] = ru[o];
        si[x] = ri[o];
        sr[x] = rr[o];
    }
}

// id range check + per-user / per-item counts (DataSet.CountByUser/CountByItem, :134-150)
__global__ __launch_bounds__(256) void count_kernel(const int32_t* __restrict__ users,
                                                    const int32_t* __restrict__ items, int64_t n,
                                                    int32_t n_users, int32_t n_items,
                                                    int32_t* cnt_u, int32_t* cnt_i,
                                                    int32_t* bad) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t u = users[x], i = items[x];
        if (u < 0 || u >= n_users || i < 0 || i >= n_items) {
            atomicOr(bad, 1);
            continue;
        }
        atomicAdd(cnt_u + u, 1);
        atomicAdd(cnt_i + i, 1);
    }
}

// order must be a permutation-subset of [0, n): range check
__global__ __launch_bounds__(256) void check_order_kernel(const int32_t* __restrict__ order,
                                                          int64_t n_order, int64_t n,
                                                          int32_t* bad) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n_order;
         x += (int64_t)gridDim.x * blockDim.x)
        if (order[x] < 0 || order[x] >= n) atomicOr(bad, 1);
}

// packed[x] = M[ids[x]] (rows of ld floats) and packed_b[x] = b[ids[x]] (b may be null)
__global__ __launch_bounds__(256) void rows_gather_kernel(const float* __restrict__ M,
                                                          const float* __restrict__ b,
                                                          const int32_t* __restrict__ ids,
                                                          int64_t n, int32_t ld,
                                                          float* __restrict__ packed,
                                                          float* __restrict__ packed_b) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * ld;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = e / ld;
        const int32_t f = (int32_t)(e - x * ld), r = ids[x];
        packed[e] = M[(int64_t)r * ld + f];
        if (f == 0 && b) packed_b[x] = b[r];
    }
}

// the inverse: M[ids[x]] = packed[x], b[ids[x]] = packed_b[x]
__global__ __launch_bounds__(256) void rows_scatter_kernel(const float* __restrict__ packed,
                                                           const float* __restrict__ packed_b,
                                                           const int32_t* __restrict__ ids,
                                                           int64_t n, int32_t ld,
                                                           float* __restrict__ M,
                                                           float* __restrict__ b) {
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < n * ld;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t x = e / ld;
        const int32_t f = (int32_t)(e - x * ld), r = ids[x];
        M[(int64_t)r * ld + f] = packed[e];
        if (f == 0) b[r] = packed_b[x];
    }
}

inline int grid_for(int64_t n, int block = 256, int cap = 8192) {
    const int64_t g = (n + block - 1) / block;
    return (int)std::max<int64_t>(1, std::min<int64_t>(g, cap));
}

inline int lanes_per_rating(int k) {
    const int vec = (k + 3) / 4;
    int lpr = 1;
    while (lpr < vec) lpr <<= 1;
    return lpr;
}

}  // namespace

// ---------------------------------------------------------------------------------------------
// The asymmetric factor models (ITransductiveRatingPredictor).  Two implicit-feedback slots:
//   slot 0: per user the items rated (training + AdditionalFeedback, ItemsRatedByUser) over y
//           [n_items x k]: the user vector = y summed over the user's items / sqrt(count)
//   slot 1: per item the users who rated it (UsersWhoRated) over x [n_users x k]: the item vector
//           = x summed over the item's users / sqrt(count)
// MODE kAsymItem (SigmoidItemAsymmetricFactorModel.cs:91-147): slot 0; trains V_i and y.
// MODE kAsymUser (SigmoidUserAsymmetricFactorModel.cs:91-144): slot 1; trains U_u and x.
// MODE kAsymCombined (SigmoidCombinedAsymmetricFactorModel.cs:108-182): both; trains x and y.
// MODE kSvdpp (SVDPlusPlus.cs:157-212, a MatrixFactorization: no sigmoid, err drives the steps)
// and kSigmoidSvdpp (SigmoidSVDPlusPlus.cs:111-173): slot 0 plus the free user offset p
// [n_users x k]: user vector = y sum / sqrt(count) + p_u (double, cast to float); trains p_u,
// V_i and y.
// One wavefront per rating at a time, lane f owns factors f, f + 64, ... (KM per lane), so every
// per-factor sum and update runs in the reference's order.  ORDERED = one wavefront over the
// whole stream (bit-faithful); HOGWILD = many wavefronts on chunks of it.
constexpr int kAsymItem = 0, kAsymUser = 1, kAsymCombined = 2, kSvdpp = 3, kSigmoidSvdpp = 4;

struct AsymSlot {
    float* X;                         // the implicit factors (y or x)
    const int64_t* __restrict__ off;  // the lists (CSR)
    const int32_t* __restrict__ ids;
    const float* __restrict__ reg;    // y_reg / x_reg
};

// the represented vector of row `key`: SumOfRows (DataType/MatrixExtensions.cs:125-135: float,
// list order), / sqrt(count) in double, cast to float (e.g. :104-107, PrecomputeUserFactors)
// The list is read 64 ids at a time (one coalesced load, then v_readlane per id) and its rows
// kAsymBatch at a time, so kAsymBatch row loads are in flight before the in-order adds.
constexpr int kAsymBatch = 8;

// adds rows [b, e) of the list onto vec, in list order
template <int KM>
__device__ __forceinline__ void asym_sum_add(const AsymSlot& sl, int32_t k, int32_t ld, int64_t b,
                                             int64_t e, int lane, float (&vec)[KM]) {
    for (int64_t base = b; base < e; base += 64) {
        const int cnt = (int)min((int64_t)64, e - base);
        const int32_t my_id = lane < cnt ? sl.ids[base + lane] : 0;
        for (int t = 0; t < cnt; t += kAsymBatch) {
            float v[kAsymBatch][KM];
#pragma unroll
            for (int q = 0; q < kAsymBatch; ++q) {
                const int32_t j = __builtin_amdgcn_readlane(my_id, min(t + q, cnt - 1));
                const float* row = sl.X + (int64_t)j * ld;
#pragma unroll
                for (int m = 0; m < KM; ++m) {
                    const int f = lane + 64 * m;
                    v[q][m] = (t + q < cnt && f < k) ? row[f] : 0.0f;
                }
            }
#pragma unroll
            for (int q = 0; q < kAsymBatch; ++q)
                if (t + q < cnt)
#pragma unroll
                    for (int m = 0; m < KM; ++m) vec[m] += v[q][m];  // list order
        }
    }
}

template <int KM>
__device__ __forceinline__ void asym_sum(const AsymSlot& sl, int32_t k, int32_t ld, int64_t b,
                                         int64_t e, int lane, float (&vec)[KM]) {
#pragma unroll
    for (int m = 0; m < KM; ++m) vec[m] = 0.0f;
    asym_sum_add<KM>(sl, k, ld, b, e, lane, vec);
}

template <int KM>
__device__ __forceinline__ double asym_vector(const AsymSlot& sl, int32_t k, int32_t ld,
                                              int32_t key, int lane, float (&vec)[KM]) {
    const int64_t b = sl.off[key], e = sl.off[key + 1];
    asym_sum<KM>(sl, k, ld, b, e, lane, vec);
    const double norm = sqrt((double)(e - b));
#pragma unroll
    for (int m = 0; m < KM; ++m) vec[m] = (float)((double)vec[m] / norm);
    return norm;
}

// x.Inc / y.Inc over the list of `key`: X[t, f] += (float)(lr * (common_f - reg[t] * X[t, f]))
template <int KM>
__device__ __forceinline__ void asym_list_step_range(const AsymSlot& sl, int32_t k, int32_t ld,
                                                     int64_t b, int64_t e, int lane, float lr,
                                                     const double (&common)[KM]) {
    for (int64_t base = b; base < e; base += 64) {
        const int cnt = (int)min((int64_t)64, e - base);
        const int32_t my_id = lane < cnt ? sl.ids[base + lane] : 0;
        for (int t = 0; t < cnt; t += kAsymBatch) {
            float y[kAsymBatch][KM], rg[kAsymBatch];
            int32_t j[kAsymBatch];
#pragma unroll
            for (int q = 0; q < kAsymBatch; ++q) {
                j[q] = __builtin_amdgcn_readlane(my_id, min(t + q, cnt - 1));
                rg[q] = sl.reg[j[q]];
                const float* row = sl.X + (int64_t)j[q] * ld;
#pragma unroll
                for (int m = 0; m < KM; ++m) {
                    const int f = lane + 64 * m;
                    y[q][m] = (t + q < cnt && f < k) ? row[f] : 0.0f;
                }
            }
            // the ids of a list are distinct, so the rows of a batch never alias
#pragma unroll
            for (int q = 0; q < kAsymBatch; ++q) {
                if (t + q >= cnt) continue;
                float* row = sl.X + (int64_t)j[q] * ld;
#pragma unroll
                for (int m = 0; m < KM; ++m) {
                    const int f = lane + 64 * m;
                    if (f < k)
                        row[f] = y[q][m] +
                                 (float)((double)lr * (common[m] - (double)(rg[q] * y[q][m])));
                }
            }
        }
    }
}

template <int KM>
__device__ __forceinline__ void asym_list_step(const AsymSlot& sl, int32_t k, int32_t ld,
                                               int32_t key, int lane, float lr,
                                               const double (&common)[KM]) {
    asym_list_step_range<KM>(sl, k, ld, sl.off[key], sl.off[key + 1], lane, lr, common);
}

// k <= 64: the first C rows of a rating's list stay in registers (one float per lane and row)
// from the sum to the step.  Between the two passes a rating writes only its trained row, p and
// the biases, never a row of its own list, so the step's y is exactly the value the sum read
// (ORDERED stays bit-faithful) and the step issues no loads for those rows.  All C row loads are
// issued before the in-order adds.  Rows past C are read and re-read as before.
template <int C>
struct AsymRowCache {
    float row[C];
    int32_t id;    // lane l: the list's l-th id (l < cnt)
    float reg;     // lane l: reg[id]
    int cnt;       // rows held (wave-uniform)
    int64_t b, e;  // the list
};

template <int C>
__device__ __forceinline__ void asym_sum_cached(const AsymSlot& sl, int32_t k, int32_t ld,
                                                int64_t b, int64_t e, int lane, float& acc,
                                                AsymRowCache<C>& rc) {
    static_assert(C % kAsymBatch == 0 && C <= 64, "cache rows");
    const int cnt = (int)min((int64_t)C, e - b);
    rc.cnt = cnt;
    rc.b = b;
    rc.e = e;
    rc.id = lane < cnt ? sl.ids[b + lane] : 0;
    rc.reg = lane < cnt ? sl.reg[rc.id] : 0.0f;
    const bool act = lane < k;
#pragma unroll
    for (int t = 0; t < C; t += kAsymBatch)
        if (t < cnt)
#pragma unroll
            for (int q = 0; q < kAsymBatch; ++q) {
                const int32_t j = __builtin_amdgcn_readlane(rc.id, min(t + q, cnt - 1));
                rc.row[t + q] = (t + q < cnt && act) ? sl.X[(int64_t)j * ld + lane] : 0.0f;
            }
    float vec[1] = {0.0f};
#pragma unroll
    for (int t = 0; t < C; t += kAsymBatch)
        if (t < cnt)
#pragma unroll
            for (int q = 0; q < kAsymBatch; ++q)
                if (t + q < cnt) vec[0] += rc.row[t + q];  // list order
    asym_sum_add<1>(sl, k, ld, b + cnt, e, lane, vec);
    acc = vec[0];
}

template <int C>
__device__ __forceinline__ void asym_list_step_cached(const AsymSlot& sl, int32_t k, int32_t ld,
                                                      int lane, float lr,
                                                      const double (&common)[1],
                                                      const AsymRowCache<C>& rc) {
    const int cnt = rc.cnt;
    const bool act = lane < k;
#pragma unroll
    for (int t = 0; t < C; t += kAsymBatch)
        if (t < cnt)
#pragma unroll
            for (int q = 0; q < kAsymBatch; ++q)
                if (t + q < cnt) {
                    const int32_t j = __builtin_amdgcn_readlane(rc.id, t + q);
                    const float rg =
                        __int_as_float(__builtin_amdgcn_readlane(__float_as_int(rc.reg), t + q));
                    const float y = rc.row[t + q];
                    if (act)
                        sl.X[(int64_t)j * ld + lane] =
                            y + (float)((double)lr * (common[0] - (double)(rg * y)));
                }
    asym_list_step_range<1>(sl, k, ld, rc.b + cnt, rc.e, lane, lr, common);
}

template <int LOSS, int KM, int MODE, int CACHE>
__global__ __launch_bounds__(256) void asym_sgd_kernel(
    const int32_t* __restrict__ su, const int32_t* __restrict__ si, const float* __restrict__ sr,
    int64_t n, int64_t chunk, AsymSlot s0, AsymSlot s1, float* U, float* V, float* bu, float* bi,
    int32_t k, int32_t ld, BmfScalars s, const int32_t* __restrict__ cnt_u,
    const int32_t* __restrict__ cnt_i, float* P) {
    constexpr bool svdpp = MODE == kSvdpp || MODE == kSigmoidSvdpp;
    constexpr bool kCached = CACHE > 0 && KM == 1 && MODE != kAsymUser;  // slot 0's rows
    // one wavefront per chunk; a workgroup is 1 wave (large sets) or 4 waves on one CU (small sets)
    const int lane = threadIdx.x & 63;
    const int64_t wave = (int64_t)blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6);
    const int64_t begin = wave * chunk;
    const int64_t end = min(begin + chunk, n);
    for (int64_t x = begin; x < end; ++x) {
        const int32_t u = su[x], i = si[x];
        const float r = sr[x];
        // a = the user side, c = the item side of the score
        float a[KM], c[KM], prod[KM];
        double norm_u = 1.0, norm_i = 1.0;
        float* trained = nullptr;  // kAsymItem: V_i, kAsymUser: U_u
        float pu[KM];  // svdpp: p_u
        AsymRowCache<kCached ? CACHE : kAsymBatch> rc;  // kCached: the list's first rows
        (void)rc;
        if constexpr (svdpp) {
            // p_plus_y_sum_vector[f] = (float)(y_sum[f] / norm + p[u, f]) (SVDPlusPlus.cs:166-170)
            float* Pu = P + (int64_t)u * ld;
            const int64_t b = s0.off[u], e = s0.off[u + 1];
            if constexpr (kCached) asym_sum_cached<CACHE>(s0, k, ld, b, e, lane, a[0], rc);
            else asym_sum<KM>(s0, k, ld, b, e, lane, a);
            norm_u = sqrt((double)(e - b));
#pragma unroll
            for (int m = 0; m < KM; ++m) {
                const int f = lane + 64 * m;
                pu[m] = f < k ? Pu[f] : 0.0f;
                a[m] = (float)((double)a[m] / norm_u + (double)pu[m]);
            }
        } else if constexpr (kCached) {  // asym_vector through the row cache
            const int64_t b = s0.off[u], e = s0.off[u + 1];
            asym_sum_cached<CACHE>(s0, k, ld, b, e, lane, a[0], rc);
            norm_u = sqrt((double)(e - b));
            a[0] = (float)((double)a[0] / norm_u);
        } else if constexpr (MODE != kAsymUser) {
            norm_u = asym_vector<KM>(s0, k, ld, u, lane, a);
        }
        if constexpr (MODE != kAsymItem && !svdpp) norm_i = asym_vector<KM>(s1, k, ld, i, lane, c);
        if constexpr (MODE == kAsymItem || svdpp) trained = V + (int64_t)i * ld;
        if constexpr (MODE == kAsymUser) trained = U + (int64_t)u * ld;
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            if constexpr (MODE == kAsymItem || svdpp) c[m] = f < k ? trained[f] : 0.0f;
            if constexpr (MODE == kAsymUser) a[m] = f < k ? trained[f] : 0.0f;
            prod[m] = a[m] * c[m];
        }
        // kAsymItem / kAsymUser: RowScalarProduct(row, IList<float>) (MatrixExtensions.cs:183-196),
        // float accumulation; kAsymCombined: VectorExtensions.ScalarProduct (VectorExtensions.cs:
        // 30-38), double accumulation of the float products, cast to float
        float dot = 0.0f;
        double dotd = 0.0;
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int lim = min(64, k - 64 * m);
            const int bits = __float_as_int(prod[m]);
            for (int l = 0; l < lim; ++l) {
                const float p = __int_as_float(__builtin_amdgcn_readlane(bits, l));
                if constexpr (MODE == kAsymCombined) dotd += (double)p;
                else dot += p;
            }
        }
        if constexpr (MODE == kAsymCombined) dot = (float)dotd;
        const float bu_u = bu[u], bi_i = bi[i];
        // score = global_bias + user_bias + item_bias in float, then + dot in double
        const double score = (double)((s.gb + bu_u) + bi_i) + (double)dot;
        double err;
        float g;
        if constexpr (MODE == kSvdpp) {  // prediction = score, no sigmoid; biases step on (float)err
            err = (double)r - score;
            g = (float)err;
        } else {
            const double sig = 1.0 / (1.0 + exp(-score));
            err = (double)r - ((double)s.min_rating + sig * (double)s.range);
            g = gradient_common<LOSS>(sig, err, s.range);
        }
        float reg_u = s.reg_u, reg_i = s.reg_i;
        if (cnt_u) {  // FrequencyRegularization
            reg_u = (float)((double)s.reg_u / sqrt((double)cnt_u[u]));
            reg_i = (float)((double)s.reg_i / sqrt((double)cnt_i[i]));
        }
        if (lane == 0) {
            bu[u] = bu_u + s.blr * (g - (s.bias_reg * reg_u) * bu_u);
            bi[i] = bi_i + s.blr * (g - (s.bias_reg * reg_i) * bi_i);
        }
        double cu[KM], ci[KM];  // common updates of the slot-0 and the slot-1 lists
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            if constexpr (MODE == kAsymItem) {  // :127-143: V_i step, y's common from old i_f
                const float i_f = c[m];
                const double delta = (double)(g * a[m] - reg_i * i_f);  // float expression
                if (f < k) trained[f] = i_f + (float)((double)s.lr * delta);
                cu[m] = ((double)g / norm_u) * (double)i_f;
            } else if constexpr (MODE == kSvdpp) {  // SVDPlusPlus.cs:186-209: double err drives
                const float i_f = c[m];
                const double delta_u = err * (double)i_f - (double)(reg_u * pu[m]);
                const double delta_i = err * (double)a[m] - (double)(reg_i * i_f);
                if (f < k) {
                    P[(int64_t)u * ld + f] = pu[m] + (float)((double)s.lr * delta_u);
                    trained[f] = i_f + (float)((double)s.lr * delta_i);
                }
                cu[m] = (err / norm_u) * (double)i_f;
            } else if constexpr (MODE == kSigmoidSvdpp) {  // SigmoidSVDPlusPlus.cs:152-170
                const float i_f = c[m];
                const double delta_u = (double)(g * i_f - reg_u * pu[m]);  // float expressions
                const double delta_i = (double)(g * a[m] - reg_i * i_f);
                if (f < k) {
                    P[(int64_t)u * ld + f] = pu[m] + (float)((double)s.lr * delta_u);
                    trained[f] = i_f + (float)((double)s.lr * delta_i);
                }
                cu[m] = ((double)g / norm_u) * (double)i_f;
            } else if constexpr (MODE == kAsymUser) {  // :127-142: U_u step, x's from old u_f
                const float u_f = a[m];
                const double delta = (double)(g * c[m] - reg_u * u_f);
                if (f < k) trained[f] = u_f + (float)((double)s.lr * delta);
                ci[m] = ((double)g / norm_i) * (double)u_f;
            } else {  // :151-180: x from the user vector, y from the item vector
                ci[m] = ((double)g / norm_i) * (double)a[m];
                cu[m] = ((double)g / norm_u) * (double)c[m];
            }
        }
        if constexpr (MODE == kAsymUser || MODE == kAsymCombined)
            asym_list_step<KM>(s1, k, ld, i, lane, s.lr, ci);
        if constexpr (kCached) asym_list_step_cached<CACHE>(s0, k, ld, lane, s.lr, cu, rc);
        else if constexpr (MODE != kAsymUser) asym_list_step<KM>(s0, k, ld, u, lane, s.lr, cu);
    }
}

// PrecomputeUserFactors / PrecomputeItemFactors: row r of `out` = the represented vector of r;
// rows with an empty list get zeros (the reference assigns a fresh zero matrix)
// P != nullptr (SVD++ PrecomputeFactors, SVDPlusPlus.cs:230-246): + p_r before the cast
template <int KM>
__global__ __launch_bounds__(64) void asym_precompute_kernel(AsymSlot sl, int32_t k, int32_t ld,
                                                             int32_t n_rows,
                                                             const float* __restrict__ P,
                                                             float* __restrict__ out) {
    const int lane = threadIdx.x;
    for (int32_t r = blockIdx.x; r < n_rows; r += gridDim.x) {
        float vec[KM];
        if (sl.off[r + 1] > sl.off[r] && P) {
            const int64_t b = sl.off[r], e = sl.off[r + 1];
            asym_sum<KM>(sl, k, ld, b, e, lane, vec);
            const double norm = sqrt((double)(e - b));
#pragma unroll
            for (int m = 0; m < KM; ++m) {
                const int f = lane + 64 * m;
                vec[m] = (float)((double)vec[m] / norm + (double)(f < k ? P[(int64_t)r * ld + f] : 0.0f));
            }
        } else if (sl.off[r + 1] > sl.off[r]) {
            asym_vector<KM>(sl, k, ld, r, lane, vec);
        } else {
#pragma unroll
            for (int m = 0; m < KM; ++m) vec[m] = 0.0f;
        }
#pragma unroll
        for (int m = 0; m < KM; ++m) {
            const int f = lane + 64 * m;
            if (f < k) out[(int64_t)r * ld + f] = vec[m];
        }
    }
}

struct mml_bmf {
    mml_ctx* ctx = nullptr;
    std::string last_kernel;  // the dominant kernel of the last epoch, as rocprof names it
    mml_bmf_params p{};
    int32_t n_users = 0, n_items = 0, k = 0, ld = 0, lpr = 0;
    mml::DeviceArray<float> U, V, bu, bi;
    mml::DeviceArray<int32_t> raw_u, raw_i, su, si, cnt_u, cnt_i, scratch_i32;
    mml::DeviceArray<float> raw_r, sr;
    mml::DeviceArray<int64_t> block_off, whole_off;
    mml::DeviceArray<int32_t> ev_u, ev_i;
    mml::DeviceArray<float> ev_r, ev_out;
    mml::DeviceArray<double> ev_partials;
    int64_t n = 0;
    int32_t G = 0;
    bool has_data = false, has_model = false;
    float gb = 0.0f, min_rating = 0.0f, max_rating = 0.0f;
    float last_ms = 0.0f;
    int32_t last_launches = 0;
    // SocialMF: the relation and its transpose, the stream positions per user / item in visit
    // order, the per-rating gradient and the batch gradients
    mml::DeviceArray<int64_t> conn_off, rev_off, upos_off, ipos_off;
    mml::DeviceArray<int32_t> conn_cols, rev_cols, upos, ipos;
    mml::DeviceArray<float> gerr, Ug, Vg, bug, big;
    int32_t n_conn = 0, n_rev = 0;
    bool has_positions = false;
    // the asymmetric models' implicit-feedback slots (0: lists per user over y, 1: per item over x)
    mml::DeviceArray<int64_t> asym_off[2];
    mml::DeviceArray<int32_t> asym_ids[2];
    mml::DeviceArray<float> asym_x[2], asym_reg[2];
    bool has_slot[2] = {false, false};
    mml::DeviceArray<float> P;  // SVD++: the free user offsets p [n_users x ld]
    bool has_p = false;
    // HOGWILD on XCD-owned item groups (xcd.hip): the stream partitioned by item group, visit
    // order kept within a group; built on the first Hogwild epoch after set_data
    mml::XcdSplit xs;
    mml::DeviceArray<int32_t> xu, xi, xr;  // xr holds the float ratings' bits
    bool has_xstream = false;
    // user phases of the XCD stream (hogwild_phases): phase-major, XCD-group-minor spans, so that
    // one launch per phase touches 1/P of U; poff = the P * 8 + 1 span offsets (device)
    int32_t n_phases = 1;
    int32_t phases_req = 0;       // mml_bmf_set_hogwild_phases (0: by the active users' bytes)
    int64_t active_users = -1;    // users with a rating in this handle (ensure_xstream)
    mml::DeviceArray<int64_t> poff;
    // user runs (mml_bmf_set_hogwild_runs): every XCD group's span of the group-major stream
    // sorted by user (ensure_runs); the spans are xs.goff's
    int32_t runs_req = -1;  // -1: on unless mml_bmf_set_hogwild_phases chose a phase count
    bool has_runs = false, last_runs = false;  // last_runs: the last Hogwild epoch ran in runs
    int64_t n_runs = 0;                        // runs of the runs stream (ensure_runs)
    // the strata: launch s gives group g user block (g + s) % 8; rspan[16 s + 2 g, + 1] = its
    // [begin, end) in the runs stream (device, and run_spans on the host)
    mml::DeviceArray<int64_t> rspan;
    std::vector<int64_t> run_spans;
    mml::DeviceArray<int32_t> rxu, rxi, rxr;
    // multi-device context: one single-device handle per GPU over a user range ub[d] .. ub[d + 1]
    // (U, b_u trained there; V, b_i replicated and averaged after every epoch)
    std::vector<mml_bmf*> shards;
    std::vector<int32_t> ub;
    std::vector<int32_t> cnt_u_host, cnt_i_host;  // the whole data set's counts
    // a rank of the DSGD ring (DSGD schedule on a context with a communicator or a peer group):
    // it owns the block rows [row0, row0 + m) (m = G / ranks) and with them its user groups; item
    // groups travel to the rank whose window needs them.  Every rank keeps the group of every
    // user / item (-1: no rating), per item group the rank holding its newest rows (-1: every
    // rank, as after set_model), the items of every group in group order (gi_off on the host)
    // and the staging rows of the moves.
    std::vector<int32_t> ugroup, igroup, hold;
    std::vector<int64_t> gi_off;
    bool ring_synced = true;  // every rank holds the newest copy of every row
    int32_t row0 = 0;
    mml::DeviceArray<int32_t> gi_ids;
    mml::DeviceArray<float> stage_v, stage_b;
    // the item average after an epoch: RCCL (ncclAvg) on a communicator, else (a device listed
    // more than once) the other shards' V || b_i staged on shard 0's device, averaged there and
    // copied back; events around it time it (mml_bmf_last_allreduce_ms)
    mml::DeviceArray<float> avg_stage;
    hipEvent_t ev_ar0 = nullptr, ev_ar1 = nullptr;
    bool has_ar = false;
};

namespace {

void check_handle(mml_bmf* h) { MML_REQUIRE(h && h->ctx, "null handle"); }

// "name<a, b, ...>": a kernel template's name as rocprofv3 prints it (integer arguments)
std::string kernel_label(const char* name, std::initializer_list<int> args) {
    std::string s = std::string(name) + "<";
    bool first = true;
    for (int a : args) {
        s += (first ? "" : ", ") + std::to_string(a);
        first = false;
    }
    return s + ">";
}

// bmf_predict1's kind: 0 BiasedMatrixFactorization (sigmoid), 1 MatrixFactorization (plain,
// clipped), 2 SVDPlusPlus (biases, clipped)
int32_t predict_kind(const mml_bmf* h) {
    return h->p.model == MML_MF_PLAIN ? 1 : h->p.model == MML_MF_SVDPP ? 2 : 0;
}

// upload / download a [rows x k] host matrix into a [rows x ld] zero-padded device matrix
void upload_padded(mml_bmf* h, float* dst, const float* src, int64_t rows) {
    if (rows == 0) return;
    MML_HIP(hipMemsetAsync(dst, 0, sizeof(float) * rows * h->ld, h->ctx->stream));
    MML_HIP(hipMemcpy2DAsync(dst, sizeof(float) * h->ld, src, sizeof(float) * h->k,
                             sizeof(float) * h->k, rows, hipMemcpyHostToDevice, h->ctx->stream));
}

void download_padded(mml_bmf* h, float* dst, const float* src, int64_t rows) {
    if (rows == 0) return;
    MML_HIP(hipMemcpy2DAsync(dst, sizeof(float) * h->k, src, sizeof(float) * h->ld,
                             sizeof(float) * h->k, rows, hipMemcpyDeviceToHost, h->ctx->stream));
}

void finish_data(mml_bmf* h, const int32_t* order_dev) {
    hipStream_t st = h->ctx->stream;
    const int64_t n = h->n;
    h->su.alloc(n);
    h->si.alloc(n);
    h->sr.alloc(n);
    h->cnt_u.alloc(h->n_users);
    h->cnt_i.alloc(h->n_items);
    h->scratch_i32.alloc(1);
    MML_HIP(hipMemsetAsync(h->cnt_u.get(), 0, sizeof(int32_t) * h->n_users, st));
    MML_HIP(hipMemsetAsync(h->cnt_i.get(), 0, sizeof(int32_t) * h->n_items, st));
    MML_HIP(hipMemsetAsync(h->scratch_i32.get(), 0, sizeof(int32_t), st));
    if (n > 0) {
        count_kernel<<<grid_for(n), 256, 0, st>>>(h->raw_u.get(), h->raw_i.get(), n, h->n_users,
                                                   h->n_items, h->cnt_u.get(), h->cnt_i.get(),
                                                   h->scratch_i32.get());
        MML_HIP(hipGetLastError());
        if (order_dev) {
            check_order_kernel<<<grid_for(n), 256, 0, st>>>(order_dev, n, n,
                                                             h->scratch_i32.get());
            MML_HIP(hipGetLastError());
        }
    }
    int32_t bad = 0;
    MML_HIP(hipMemcpyAsync(&bad, h->scratch_i32.get(), sizeof(int32_t), hipMemcpyDeviceToHost,
                           st));
    MML_HIP(hipStreamSynchronize(st));
    if (bad) {
        h->has_data = false;
        mml::fail(MML_ERR_ARG, "rating user/item id or order index out of range");
    }
    if (n > 0) {
        gather_stream_kernel<<<grid_for(n), 256, 0, st>>>(h->raw_u.get(), h->raw_i.get(),
                                                          h->raw_r.get(), order_dev, n,
                                                          h->su.get(), h->si.get(), h->sr.get());
        MML_HIP(hipGetLastError());
    }
    h->whole_off.alloc(2);
    const int64_t off[2] = {0, n};
    MML_HIP(hipMemcpyAsync(h->whole_off.get(), off, sizeof(off), hipMemcpyHostToDevice, st));
    MML_HIP(hipStreamSynchronize(st));
    h->G = 0;
    h->has_positions = false;
    h->has_xstream = false;
    h->n_phases = 1;
    h->has_runs = false;
    h->has_data = true;
}

// stream positions grouped by key (users or items) in visit order: stable radix sort of
// (key, position) pairs, offsets from the per-key counts
void build_positions(mml_bmf* h, const int32_t* keys, const int32_t* cnt, int32_t n_keys,
                     mml::DeviceArray<int64_t>& off, mml::DeviceArray<int32_t>& pos) {
    hipStream_t st = h->ctx->stream;
    const int64_t n = h->n;
    off.alloc((size_t)n_keys + 1);
    pos.alloc(std::max<int64_t>(1, n));
    MML_HIP(hipMemsetAsync(off.get(), 0, sizeof(int64_t) * (n_keys + 1), st));
    if (n == 0 || n_keys == 0) return;
    mml::DeviceArray<int32_t> iota, ksorted;
    mml::DeviceArray<int64_t> wide;
    iota.alloc(n);
    ksorted.alloc(n);
    wide.alloc(n_keys);
    smf_iota_kernel<<<grid_for(n), 256, 0, st>>>(iota.get(), n);
    smf_widen_kernel<<<grid_for(n_keys), 256, 0, st>>>(cnt, n_keys, wide.get());
    MML_HIP(hipGetLastError());
    int end_bit = 1;
    while (end_bit < 31 && (1 << end_bit) < n_keys) ++end_bit;
    size_t b1 = 0, b2 = 0;
    MML_HIP(rocprim::radix_sort_pairs(nullptr, b1, keys, ksorted.get(), iota.get(),
                                               pos.get(), (int)n, 0, end_bit, st));
    MML_HIP(rocprim::inclusive_scan(nullptr, b2, wide.get(), off.get() + 1, n_keys,
            rocprim::plus<int64_t>(), st));
    mml::DeviceArray<uint8_t> tmp;
    tmp.alloc(std::max(b1, b2));
    MML_HIP(rocprim::radix_sort_pairs(tmp.get(), b1, keys, ksorted.get(), iota.get(),
                                               pos.get(), (int)n, 0, end_bit, st));
    MML_HIP(rocprim::inclusive_scan(tmp.get(), b2, wide.get(), off.get() + 1, n_keys,
            rocprim::plus<int64_t>(), st));
    MML_HIP(hipStreamSynchronize(st));
}

template <int LOSS, int KM>
void social_epoch_km(mml_bmf* h, const BmfScalars& s) {
    hipStream_t st = h->ctx->stream;
    const int64_t n = h->n;
    if (n > 0) {
        smf_error_kernel<LOSS><<<grid_for(n), 256, 0, st>>>(
            h->su.get(), h->si.get(), h->sr.get(), n, h->U.get(), h->V.get(), h->bu.get(),
            h->bi.get(), h->k, h->ld, s.gb, s.min_rating, s.range, h->gerr.get());
        MML_HIP(hipGetLastError());
    }
    if (h->n_users > 0)
        smf_user_grad_kernel<KM><<<h->n_users, 64, 0, st>>>(
            h->upos_off.get(), h->upos.get(), h->si.get(), h->gerr.get(), h->U.get(), h->V.get(),
            h->bu.get(), h->k, h->ld, s.reg_u, s.bias_reg, h->p.social_regularization,
            h->conn_off.get(), h->conn_cols.get(), h->n_conn, h->rev_off.get(),
            h->rev_cols.get(), h->n_rev, h->Ug.get(), h->bug.get());
    if (h->n_items > 0)
        smf_item_grad_kernel<KM><<<h->n_items, 64, 0, st>>>(
            h->ipos_off.get(), h->ipos.get(), h->su.get(), h->gerr.get(), h->U.get(), h->V.get(),
            h->bi.get(), h->k, h->ld, s.reg_i, s.bias_reg, h->Vg.get(), h->big.get());
    MML_HIP(hipGetLastError());
    const float blr = h->p.bias_learn_rate;
    smf_apply_kernel<<<grid_for((int64_t)h->n_users * h->ld), 256, 0, st>>>(
        h->U.get(), h->Ug.get(), (int64_t)h->n_users * h->ld, h->bu.get(), h->bug.get(),
        h->n_users, s.lr, blr);
    smf_apply_kernel<<<grid_for((int64_t)h->n_items * h->ld), 256, 0, st>>>(
        h->V.get(), h->Vg.get(), (int64_t)h->n_items * h->ld, h->bi.get(), h->big.get(),
        h->n_items, s.lr, blr);
    MML_HIP(hipGetLastError());
}

// SocialMF.Iterate(IList<int>,bool,bool) -> IterateBatch (SocialMF.cs:72-194), one batch step
template <int LOSS>
void social_epoch(mml_bmf* h, const BmfScalars& s) {
    if (!h->has_positions) {
        build_positions(h, h->su.get(), h->cnt_u.get(), h->n_users, h->upos_off, h->upos);
        build_positions(h, h->si.get(), h->cnt_i.get(), h->n_items, h->ipos_off, h->ipos);
        h->gerr.alloc(std::max<int64_t>(1, h->n));
        h->Ug.alloc(std::max<size_t>(1, (size_t)h->n_users * h->ld));
        h->Vg.alloc(std::max<size_t>(1, (size_t)h->n_items * h->ld));
        h->bug.alloc(std::max<int32_t>(1, h->n_users));
        h->big.alloc(std::max<int32_t>(1, h->n_items));
        h->has_positions = true;
    }
    switch ((h->k + 63) / 64) {
        case 1: social_epoch_km<LOSS, 1>(h, s); break;
        case 2: social_epoch_km<LOSS, 2>(h, s); break;
        case 3: social_epoch_km<LOSS, 3>(h, s); break;
        default: social_epoch_km<LOSS, 4>(h, s); break;
    }
    h->last_launches = 5;
}

template <int LOSS>
void launch_ordered(mml_bmf* h, const int64_t* off, int32_t G, int32_t sub, int grid,
                    const BmfScalars& s, const int32_t* cu, const int32_t* ci, int32_t row0 = 0) {
    const int km = (h->k + 63) / 64;
    hipStream_t st = h->ctx->stream;
#define MML_ORD(KM)                                                                            \
    bmf_sgd_ordered_kernel<LOSS, KM><<<grid, 64, 0, st>>>(                                     \
        h->su.get(), h->si.get(), h->sr.get(), off, G, sub, row0, h->U.get(), h->V.get(),       \
        h->bu.get(), h->bi.get(), h->k, h->ld, s, cu, ci)
    switch (km) {
        case 1: MML_ORD(1); break;
        case 2: MML_ORD(2); break;
        case 3: MML_ORD(3); break;
        default: MML_ORD(4); break;
    }
#undef MML_ORD
    MML_HIP(hipGetLastError());
    h->last_kernel = kernel_label("bmf_sgd_ordered_kernel", {LOSS, km < 4 ? km : 4});
}

// The XCD-partitioned copy of the visit-order stream (built once per data set): items dealt into 8
// groups of equal rating count (cnt_i), ratings stably partitioned by their item's group.
void ensure_xstream(mml_bmf* h) {
    if (h->has_xstream) return;
    hipStream_t st = h->ctx->stream;
    std::vector<int32_t> ci(h->n_items);
    if (h->n_items > 0)
        MML_HIP(hipMemcpyAsync(ci.data(), h->cnt_i.get(), sizeof(int32_t) * h->n_items,
                               hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    std::vector<int32_t> cu(h->n_users);
    if (h->n_users > 0)
        MML_HIP(hipMemcpyAsync(cu.data(), h->cnt_u.get(), sizeof(int32_t) * h->n_users,
                               hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    h->active_users = std::count_if(cu.begin(), cu.end(), [](int32_t c) { return c > 0; });
    h->xs.set_groups(st, std::vector<int64_t>(ci.begin(), ci.end()), 8);
    h->xu.alloc(h->n);
    h->xi.alloc(h->n);
    h->xr.alloc(h->n);
    const int32_t* in[3] = {h->su.get(), h->si.get(), reinterpret_cast<const int32_t*>(h->sr.get())};
    int32_t* out[3] = {h->xu.get(), h->xi.get(), h->xr.get()};
    h->xs.partition(st, h->si.get(), h->n, 3, in, out);
    MML_HIP(hipStreamSynchronize(st));
    h->has_xstream = true;
}

// the phase of a user: a fixed hash, so every phase is a random 1/P of the users whatever the id
// order of the data set
__device__ __forceinline__ int32_t user_phase(int32_t u, int32_t P) {
    return (int32_t)(mml::mix64((uint64_t)(uint32_t)u ^ 0x6A09E667F3BCC909ull) % (uint64_t)P);
}

// key of stream position x of the XCD stream: phase of its user * 8 + its XCD group
__global__ __launch_bounds__(256) void phase_keys_kernel(const int32_t* __restrict__ xu,
                                                         const int64_t* __restrict__ goff,
                                                         int64_t n, int32_t P,
                                                         uint16_t* __restrict__ key,
                                                         int32_t* __restrict__ idx) {
    int64_t g_off[9];
#pragma unroll
    for (int g = 0; g < 9; ++g) g_off[g] = goff[g];
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        int g = 0;
#pragma unroll
        for (int c = 1; c < 8; ++c) g += x >= g_off[c];
        key[x] = (uint16_t)(user_phase(xu[x], P) * 8 + g);
        idx[x] = (int32_t)x;
    }
}

__global__ __launch_bounds__(256) void gather3_kernel(const int32_t* __restrict__ idx, int64_t n,
                                                      const int32_t* __restrict__ a,
                                                      const int32_t* __restrict__ b,
                                                      const int32_t* __restrict__ c,
                                                      int32_t* __restrict__ oa,
                                                      int32_t* __restrict__ ob,
                                                      int32_t* __restrict__ oc) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t y = idx[x];
        oa[x] = a[y];
        ob[x] = b[y];
        oc[x] = c[y];
    }
}

// span offsets of the sorted keys: off[k] = first position with key >= k, k = 0 .. nk
__global__ __launch_bounds__(256) void key_offsets_kernel(const uint16_t* __restrict__ key,
                                                          int64_t n, int32_t nk,
                                                          int64_t* __restrict__ off) {
    const int32_t k = blockIdx.x * blockDim.x + threadIdx.x;
    if (k > nk) return;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int32_t)key[mid] < k) lo = mid + 1;
        else hi = mid;
    }
    off[k] = lo;
}

// MML_HOGWILD_PHASES (experiments): user phases of the Hogwild epoch.  P > 1 splits every XCD
// group's stream into P phases by a hash of the user (stable: the visit order is kept within a
// phase) and runs one launch per phase, so a launch touches 1/P of U -- a phase's rows then stay
// in the 256 MB Infinity Cache between a user's ratings instead of coming from HBM each time.
static int32_t hogwild_phases_env() {
    static const int32_t m = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_HOGWILD_PHASES");
        return e ? std::max(0, std::min(32, std::atoi(e))) : -1;
    }();
    return m;
}
// Default: one phase per 96 MiB of the active users' rows, at most 32.  Measured on one MI355X
// (profiles/r5c_*): C4 (10 M users, 2.56 GB of U) 218.7 ms per epoch in one phase, 196.3 in 8,
// 180.3 in 16, 178.8 in 32 (replay ceilings 215.6 / 186.7 / 175.7 / 174.7 ms); C2 (256 MB of U)
// 22.3 ms in one phase, 20.0 in 2, 20.1 in 4; the test RMSE after 8 (C4) and 12 (C2) epochs
// unchanged within the run-to-run spread (C4 0.63100 / 0.63092 / 0.63113 / 0.63103).
// A phase also gathers each user's ratings of an epoch into 1/P of it, so at the end of an epoch
// the users of the early phases were last updated further back while the items kept moving: a
// lag that is visible while the items still move a lot per epoch (800 k users x 16 M ratings,
// RMSE after epochs 1-4 in 3 phases +0.3e-4 ... +1.9e-4 and in 8 phases +3.4e-4 ... +4.6e-4 over
// one phase, run to run spread ~1e-4; tests/test_phases_gpu.py) and gone near convergence (C4
// after 8 epochs: 0.63100 in one phase, 0.63092 / 0.63113 / 0.63103 in 16 / 8 / 32).
int32_t hogwild_phases(const mml_bmf* h) {
    const int32_t e = hogwild_phases_env();
    if (e >= 0) return std::max(1, e);
    if (h->phases_req > 0) return h->phases_req;
    const uint64_t bytes = (uint64_t)std::max<int64_t>(0, h->active_users) * h->ld * sizeof(float);
    const uint64_t per = 96ull << 20;
    return (int32_t)std::max<uint64_t>(1, std::min<uint64_t>(32, (bytes + per - 1) / per));
}

// the XCD stream reordered phase-major (built once per data set and phase count).  The phase keys
// take each position's XCD group from xs.goff, i.e. from the group-major order: a stream already
// sorted for another phase count is rebuilt group-major first (P <= 1 stops there).
void ensure_phases(mml_bmf* h, int32_t P) {
    if (h->n_phases == P) return;
    hipStream_t st = h->ctx->stream;
    const int64_t n = h->n;
    if (h->n_phases > 1 || P <= 1) {
        h->has_xstream = false;
        h->n_phases = 1;
        ensure_xstream(h);
        if (P <= 1) return;
    }
    const int nk = P * 8;
    int end_bit = 1;
    while ((1 << end_bit) < nk) ++end_bit;
    mml::DeviceArray<uint16_t> key, key_s;
    mml::DeviceArray<int32_t> idx, idx_s;
    key.alloc(n);
    key_s.alloc(n);
    idx.alloc(n);
    idx_s.alloc(n);
    phase_keys_kernel<<<grid_for(n), 256, 0, st>>>(h->xu.get(), h->xs.goff.get(), n, P, key.get(),
                                                   idx.get());
    MML_HIP(hipGetLastError());
    size_t tmp_bytes = 0;
    MML_HIP(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key.get(), key_s.get(),
                                               idx.get(), idx_s.get(), n, 0, end_bit, st));
    mml::DeviceArray<uint8_t> tmp;
    tmp.alloc(std::max<size_t>(1, tmp_bytes));
    MML_HIP(rocprim::radix_sort_pairs(tmp.get(), tmp_bytes, key.get(), key_s.get(),
                                               idx.get(), idx_s.get(), n, 0, end_bit, st));
    mml::DeviceArray<int32_t> ou, oi, orr;
    ou.alloc(n);
    oi.alloc(n);
    orr.alloc(n);
    gather3_kernel<<<grid_for(n), 256, 0, st>>>(idx_s.get(), n, h->xu.get(), h->xi.get(),
                                                h->xr.get(), ou.get(), oi.get(), orr.get());
    h->poff.alloc(nk + 1);
    key_offsets_kernel<<<(nk + 1 + 255) / 256, 256, 0, st>>>(key_s.get(), n, nk, h->poff.get());
    MML_HIP(hipGetLastError());
    MML_HIP(hipStreamSynchronize(st));
    h->xu.swap(ou);
    h->xi.swap(oi);
    h->xr.swap(orr);
    h->n_phases = P;
}

// key of position x of the group-major stream for the user runs: group * n_users + the user
__global__ __launch_bounds__(256) void run_keys_kernel(const int32_t* __restrict__ xu,
                                                       const int64_t* __restrict__ goff, int64_t n,
                                                       int32_t n_users, uint32_t* __restrict__ key,
                                                       int32_t* __restrict__ idx) {
    int64_t g_off[9];
#pragma unroll
    for (int g = 0; g < 9; ++g) g_off[g] = goff[g];
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        int g = 0;
#pragma unroll
        for (int c = 1; c < 8; ++c) g += x >= g_off[c];
        key[x] = (uint32_t)((int64_t)g * n_users + xu[x]);
        idx[x] = (int32_t)x;
    }
}

// runs of the runs stream: positions that start a group span or follow another user's rating
__global__ __launch_bounds__(256) void count_runs_kernel(const int32_t* __restrict__ su,
                                                         const int64_t* __restrict__ goff,
                                                         int64_t n,
                                                         unsigned long long* __restrict__ out) {
    int64_t g_off[9];
#pragma unroll
    for (int g = 0; g < 9; ++g) g_off[g] = goff[g];
    unsigned long long c = 0;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        bool start = x == 0 || su[x] != su[x - 1];
#pragma unroll
        for (int g = 1; g < 8; ++g) start = start || x == g_off[g];
        c += start ? 1 : 0;
    }
    for (int o = 32; o > 0; o >>= 1) c += __shfl_xor(c, o);
    if ((threadIdx.x & 63) == 0 && c) atomicAdd(out, c);
}

// first position of the sorted keys >= thr[t], t = 0 .. nt
__global__ __launch_bounds__(256) void key_thresholds_kernel(const uint32_t* __restrict__ key,
                                                             int64_t n,
                                                             const int64_t* __restrict__ thr,
                                                             int32_t nt,
                                                             int64_t* __restrict__ off) {
    const int32_t t = blockIdx.x * blockDim.x + threadIdx.x;
    if (t >= nt) return;
    int64_t lo = 0, hi = n;
    while (lo < hi) {
        const int64_t mid = (lo + hi) >> 1;
        if ((int64_t)key[mid] < thr[t]) lo = mid + 1;
        else hi = mid;
    }
    off[t] = lo;
}

// the user-runs stream (built once per data set): the group-major XCD stream, each group's span
// stably sorted by user, and its 8 x 8 strata (user blocks of equal rating count x XCD groups)
void ensure_runs(mml_bmf* h) {
    if (h->has_runs) return;
    if (h->n_phases != 1) ensure_phases(h, 1);
    ensure_xstream(h);
    MML_REQUIRE((int64_t)h->n_users * 8 < (1ll << 31), "user runs: at most 2^28 users");
    hipStream_t st = h->ctx->stream;
    const int64_t n = h->n;
    int end_bit = 1;
    while ((1ll << end_bit) < (int64_t)h->n_users * 8) ++end_bit;
    mml::DeviceArray<uint32_t> key, key_s;
    mml::DeviceArray<int32_t> idx, idx_s;
    key.alloc(n);
    key_s.alloc(n);
    idx.alloc(n);
    idx_s.alloc(n);
    run_keys_kernel<<<grid_for(n), 256, 0, st>>>(h->xu.get(), h->xs.goff.get(), n, h->n_users,
                                                 key.get(), idx.get());
    MML_HIP(hipGetLastError());
    size_t tmp_bytes = 0;
    MML_HIP(rocprim::radix_sort_pairs(nullptr, tmp_bytes, key.get(), key_s.get(), idx.get(),
                                      idx_s.get(), n, 0, end_bit, st));
    mml::DeviceArray<uint8_t> tmp;
    tmp.alloc(std::max<size_t>(1, tmp_bytes));
    MML_HIP(rocprim::radix_sort_pairs(tmp.get(), tmp_bytes, key.get(), key_s.get(), idx.get(),
                                      idx_s.get(), n, 0, end_bit, st));
    // user blocks of equal rating count: ub[b] = the first user of block b
    std::vector<int32_t> cu(h->n_users);
    if (h->n_users > 0)
        MML_HIP(hipMemcpyAsync(cu.data(), h->cnt_u.get(), sizeof(int32_t) * h->n_users,
                               hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    std::vector<int64_t> ub(9, h->n_users);
    ub[0] = 0;
    {
        int64_t run = 0;
        int b = 1;
        for (int32_t u = 0; u < h->n_users && b < 8; ++u) {
            run += cu[u];
            while (b < 8 && run * 8 >= n * b) ub[b++] = u + 1;
        }
    }
    std::vector<int64_t> thr(8 * 9);
    for (int g = 0; g < 8; ++g)
        for (int b = 0; b <= 8; ++b) thr[9 * g + b] = (int64_t)g * h->n_users + ub[b];
    mml::DeviceArray<int64_t> thr_d, off_d;
    thr_d.alloc(thr.size());
    off_d.alloc(thr.size());
    MML_HIP(hipMemcpyAsync(thr_d.get(), thr.data(), sizeof(int64_t) * thr.size(),
                           hipMemcpyHostToDevice, st));
    key_thresholds_kernel<<<1, 128, 0, st>>>(key_s.get(), n, thr_d.get(), (int32_t)thr.size(),
                                             off_d.get());
    MML_HIP(hipGetLastError());
    std::vector<int64_t> off(thr.size());
    MML_HIP(hipMemcpyAsync(off.data(), off_d.get(), sizeof(int64_t) * off.size(),
                           hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    h->run_spans.assign(8 * 16, 0);
    for (int sx = 0; sx < 8; ++sx)
        for (int g = 0; g < 8; ++g) {
            const int b = (g + sx) % 8;
            h->run_spans[16 * sx + 2 * g] = off[9 * g + b];
            h->run_spans[16 * sx + 2 * g + 1] = off[9 * g + b + 1];
        }
    h->rspan.alloc(h->run_spans.size());
    MML_HIP(hipMemcpyAsync(h->rspan.get(), h->run_spans.data(),
                           sizeof(int64_t) * h->run_spans.size(), hipMemcpyHostToDevice, st));
    key.reset();
    key_s.reset();
    idx.reset();
    tmp.reset();
    h->rxu.alloc(n);
    h->rxi.alloc(n);
    h->rxr.alloc(n);
    gather3_kernel<<<grid_for(n), 256, 0, st>>>(idx_s.get(), n, h->xu.get(), h->xi.get(),
                                                h->xr.get(), h->rxu.get(), h->rxi.get(),
                                                h->rxr.get());
    MML_HIP(hipGetLastError());
    mml::DeviceArray<unsigned long long> cnt;
    cnt.alloc(1);
    MML_HIP(hipMemsetAsync(cnt.get(), 0, sizeof(unsigned long long), st));
    count_runs_kernel<<<grid_for(n), 256, 0, st>>>(h->rxu.get(), h->xs.goff.get(), n, cnt.get());
    MML_HIP(hipGetLastError());
    unsigned long long runs = 0;
    MML_HIP(hipMemcpyAsync(&runs, cnt.get(), sizeof(runs), hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    h->n_runs = n > 0 ? (int64_t)runs : 0;
    h->has_runs = true;
}

// MML_HOGWILD_XCD: 4 (default) = XCD-owned item groups with L2-served item loads, user rows written
// through and flushing waves; 1 = the groups with L2-served item loads only, 2 = the groups
// with plain loads, 3 = 1 + user rows written through, 4 = 3 + flushing waves (mml::flushers_per_xcd),
// 5 = 1 + the flushing waves, 0 = one span over all XCDs (the round-1 kernel)
static int hogwild_xcd_mode() {
    static const int m = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_HOGWILD_XCD");
        return e ? std::atoi(e) : 4;
    }();
    return m;
}

template <int LOSS>
void launch_hogwild(mml_bmf* h, const BmfScalars& s, const int32_t* cu, const int32_t* ci) {
    hipStream_t st = h->ctx->stream;
    const int64_t n = h->n;
    // waves: up to 256 CUs x 32 (all resident at once), each walking >= min_chunk ratings of the
    // stream in order.  Fewer than 16 waves' worth of work runs as ONE workgroup: a single CU keeps
    // every row in one L1/L2 and bounds the updates in flight (C1: 4 waves on one CU RMSE +0.007 vs
    // sequential, 19 waves on 5 CUs +0.12).  Larger sets run on XCD-owned item groups (xcd.hip):
    // group g's ratings on the blocks b % 8 == g of one XCD, so a hot item's row lives in one L2
    // instead of 8 replicas whose write-backs overwrite each other's updates.
    static const int64_t min_chunk = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_HOGWILD_MIN_CHUNK");
        return e ? std::max<int64_t>(1, std::atoll(e)) : (int64_t)12000;
    }();
    int64_t waves = std::min<int64_t>(256 * 32, std::max<int64_t>(1, n / min_chunk));
    const bool coh = h->p.schedule == MML_SCHEDULE_HOGWILD_COHERENT;
    const int xmode = hogwild_xcd_mode();
    const uint64_t v_bytes = (uint64_t)h->n_items * h->ld * sizeof(float);
    int32_t ng = 1;
    const int64_t* goff = h->whole_off.get();
    const int32_t *su = h->su.get(), *si = h->si.get();
    const float* sr = h->sr.get();
    int am = coh ? kAccCoherent : kAccPlain;
    bool runs = false;
    if (waves < 16) {
        waves = 4;
    } else if (!coh && xmode > 0 && v_bytes < (1ull << 32) && mml::xcd_groups(h->ctx) == 8) {
        ensure_xstream(h);
        ng = 8;
        goff = h->xs.goff.get();
        su = h->xu.get();
        si = h->xi.get();
        sr = reinterpret_cast<const float*>(h->xr.get());
        const bool u_fits = (uint64_t)h->n_users * h->ld * sizeof(float) < (1ull << 32);
        switch (xmode) {
            case 2: am = kAccPlain; break;
            case 3: am = u_fits ? kAccItemL2 | kAccUserThru : kAccItemL2; break;
            case 4: am = u_fits ? kAccItemL2 | kAccUserThru | kAccFlush : kAccItemL2 | kAccFlush;
                break;
            case 5: am = kAccItemL2 | kAccFlush; break;
#ifdef MML_EXPERIMENTS
            case 6:  // 4 with the user bias plain (A/B of its write-through cost)
                am = u_fits ? kAccItemL2 | kAccUserThru | kAccFlush | kAccUBiasPlain
                            : kAccItemL2 | kAccFlush;
                break;
#endif
            default: am = kAccItemL2; break;
        }
        // the default (runs_req -1) from 16 M ratings: on the small skewed sets of the edge-case
        // and shard tests (300 k ratings over 300-800 items, a wave's slices a few runs long) the
        // runs measured up to 2x the phase kernel's Hogwild offset, so those keep the phases
        constexpr int64_t kRunsMinRatings = 16000000;
        const bool want_runs =
            h->runs_req > 0 || (h->runs_req < 0 && h->phases_req == 0 && hogwild_phases_env() < 0 &&
                                n >= kRunsMinRatings);
        if (want_runs && (am & kAccUserThru) != 0) {
            // user runs: one launch over the group-major stream sorted by user within a group
            ensure_runs(h);
            runs = true;
            su = h->rxu.get();
            si = h->rxi.get();
            sr = reinterpret_cast<const float*>(h->rxr.get());
        } else {
            // user phases: one launch per phase over the phase-major stream
            const int32_t P = hogwild_phases(h);
            if (P != h->n_phases) ensure_phases(h, P);
            su = h->xu.get();
            si = h->xi.get();
            sr = reinterpret_cast<const float*>(h->xr.get());
        }
    }
    const int32_t phases = ng == 8 && !runs ? h->n_phases : 1;
    if (LOSS != kReplayTraffic) h->last_runs = runs;
    int64_t blocks = (waves + 3) / 4;
    blocks = (blocks + ng - 1) / ng * ng;
    const int32_t wpg = (int32_t)(blocks / ng * 4);
    const int ld4 = h->ld / 4;
    const uint32_t vb = (uint32_t)std::min<uint64_t>(v_bytes, 0xFFFFFFFFull);
    const uint32_t bb = (uint32_t)((uint64_t)h->n_items * sizeof(float));
    const uint32_t ub = (uint32_t)std::min<uint64_t>((uint64_t)h->n_users * h->ld * sizeof(float),
                                                     0xFFFFFFFFull);
    const uint32_t bub = (uint32_t)((uint64_t)h->n_users * sizeof(float));
#define MML_HOG1(LPR, VPL, AM)                                                                  \
    bmf_sgd_hogwild_kernel<LOSS, LPR, VPL, AM><<<(int)blocks, 256, 0, st>>>(                  \
        su, si, sr, go, ng, wpg, h->U.get(), h->V.get(), h->bu.get(), h->bi.get(), ld4, vb, bb,   \
        ub, bub, mml::flushers_per_xcd(1), s, cu, ci);                                         \
    h->last_kernel = kernel_label("bmf_sgd_hogwild_kernel", {LOSS, LPR, VPL, (int)(AM)})
#ifdef MML_EXPERIMENTS
#define MML_HOG_EXP(LPR, VPL)                                                      \
    case kAccItemL2 | kAccUserThru | kAccFlush | kAccUBiasPlain:                   \
        MML_HOG1(LPR, VPL, kAccItemL2 | kAccUserThru | kAccFlush | kAccUBiasPlain); \
        break;
#else
#define MML_HOG_EXP(LPR, VPL)
#endif
#define MML_HOGV(LPR, VPL)                                                       \
    switch (am) {                                                                \
        case kAccCoherent: MML_HOG1(LPR, VPL, kAccCoherent); break;              \
        case kAccItemL2: MML_HOG1(LPR, VPL, kAccItemL2); break;                  \
        case kAccItemL2 | kAccUserThru:                                          \
            MML_HOG1(LPR, VPL, kAccItemL2 | kAccUserThru); break;                \
        case kAccItemL2 | kAccUserThru | kAccFlush:                              \
            MML_HOG1(LPR, VPL, kAccItemL2 | kAccUserThru | kAccFlush); break;    \
        case kAccItemL2 | kAccFlush: MML_HOG1(LPR, VPL, kAccItemL2 | kAccFlush); break; \
        MML_HOG_EXP(LPR, VPL)                                                    \
        default: MML_HOG1(LPR, VPL, kAccPlain); break;                           \
    }
#define MML_RUN1(LPR, AM)                                                                        \
    for (int sx = 0; sx < 8; ++sx)                                                                \
        bmf_sgd_runs_kernel<LOSS, LPR, AM><<<(int)blocks, 256, 0, st>>>(                          \
            su, si, sr, h->rspan.get() + 16 * sx, wpg, h->U.get(), h->V.get(), h->bu.get(),      \
            h->bi.get(), ld4, vb, bb, ub, bub, mml::flushers_per_xcd(1), s, cu, ci);              \
    h->last_kernel = kernel_label("bmf_sgd_runs_kernel", {LOSS, LPR, (int)(AM)})
// (no flushing waves: a group's item rows are read by its own XCD only, and the runs write U_u
// through; with them C4 was 112.3 / 113.2 against 107.0 / 107.3 ms per epoch, profiles/r6/runs/)
#define MML_RUNV(LPR) MML_RUN1(LPR, kAccItemL2 | kAccUserThru)
    if (runs) {
        switch (h->lpr) {
            case 1: MML_RUNV(1); break;
            case 2: MML_RUNV(2); break;
            case 4: MML_RUNV(4); break;
            case 8: MML_RUNV(8); break;
            case 16: MML_RUNV(16); break;
            case 32: MML_RUNV(32); break;
            default: MML_RUNV(64); break;
        }
        MML_HIP(hipGetLastError());
        return;
    }
#undef MML_RUNV
#undef MML_RUN1
    // one float4 of U_u and of V_i per lane (VPL 2 measured equal, VPL 4 10 % slower on C2)
    for (int32_t ph = 0; ph < phases; ++ph) {
        const int64_t* go = phases > 1 ? h->poff.get() + 8 * ph : goff;
        switch (h->lpr) {
            case 1: MML_HOGV(1, 1); break;
            case 2: MML_HOGV(2, 1); break;
            case 4: MML_HOGV(4, 1); break;
            case 8: MML_HOGV(8, 1); break;
            case 16: MML_HOGV(16, 1); break;
            case 32: MML_HOGV(32, 1); break;
            default: MML_HOGV(64, 1); break;
        }
    }
#undef MML_HOGV
#undef MML_HOG_EXP
#undef MML_HOG1
    MML_HIP(hipGetLastError());
}

bool is_asym(const mml_bmf* h) {
    return h->p.model >= MML_MF_ITEM_ASYM && h->p.model <= MML_MF_SIGMOID_SVDPP;
}
int asym_mode(const mml_bmf* h) {
    switch (h->p.model) {
        case MML_MF_ITEM_ASYM: return kAsymItem;
        case MML_MF_USER_ASYM: return kAsymUser;
        case MML_MF_SVDPP: return kSvdpp;
        case MML_MF_SIGMOID_SVDPP: return kSigmoidSvdpp;
        default: return kAsymCombined;
    }
}
bool is_svdpp(const mml_bmf* h) {
    return h->p.model == MML_MF_SVDPP || h->p.model == MML_MF_SIGMOID_SVDPP;
}
AsymSlot asym_slot(mml_bmf* h, int side) {
    return AsymSlot{h->asym_x[side].get(), h->asym_off[side].get(), h->asym_ids[side].get(),
                    h->asym_reg[side].get()};
}
// the sides a model reads: slot 0 for all but the user model, slot 1 for the user / combined ones
bool uses_side(const mml_bmf* h, int side) {
    const int mode = asym_mode(h);
    return side == 0 ? mode != kAsymUser : (mode == kAsymUser || mode == kAsymCombined);
}
bool asym_ready(const mml_bmf* h) {
    return (!uses_side(h, 0) || h->has_slot[0]) && (!uses_side(h, 1) || h->has_slot[1]) &&
           (!is_svdpp(h) || h->has_p);
}

// U <- PrecomputeUserFactors (slot 0) and / or V <- PrecomputeItemFactors (slot 1): what Predict
// and the evaluators read
void asym_precompute(mml_bmf* h) {
    const int km = (h->k + 63) / 64;
    const int mode = asym_mode(h);
    hipStream_t st = h->ctx->stream;
    (void)mode;
    for (int side = 0; side < 2; ++side) {
        if (!uses_side(h, side)) continue;
        const int32_t rows = side == 0 ? h->n_users : h->n_items;
        if (rows == 0) continue;
        const int grid = std::max(1, std::min(rows, 65536));
        float* out = side == 0 ? h->U.get() : h->V.get();
        const AsymSlot sl = asym_slot(h, side);
        const float* pp = side == 0 && is_svdpp(h) ? h->P.get() : nullptr;
#define MML_PRE(KM) \
    asym_precompute_kernel<KM><<<grid, 64, 0, st>>>(sl, h->k, h->ld, rows, pp, out)
        switch (km) {
            case 1: MML_PRE(1); break;
            case 2: MML_PRE(2); break;
            case 3: MML_PRE(3); break;
            default: MML_PRE(4); break;
        }
#undef MML_PRE
        MML_HIP(hipGetLastError());
    }
}

// MML_ASYM_CACHE: rows of a list kept in registers from the sum to the step at k <= 64 (0 / 32 /
// 64, default 64); read per epoch so a test can switch it
static int asym_cache_rows() {
    const char* e = MML_EXPERIMENT_ENV("MML_ASYM_CACHE");
    return e ? std::atoi(e) : 64;
}

template <int LOSS>
void asym_epoch(mml_bmf* h, const BmfScalars& s) {
    const int32_t* cu = h->p.frequency_regularization ? h->cnt_u.get() : nullptr;
    const int32_t* ci = h->p.frequency_regularization ? h->cnt_i.get() : nullptr;
    const int64_t n = h->n;
    hipStream_t st = h->ctx->stream;
    if (n > 0) {
        // ORDERED: one wavefront, the whole stream in order.  HOGWILD: a wavefront per >= 1,024
        // ratings (a rating reads and writes whole lists of implicit rows), at most 256 CUs x 32
        static const int64_t cap = [] {
            const char* e = MML_EXPERIMENT_ENV("MML_ASYM_WAVES");
            return e ? std::max<int64_t>(1, std::atoll(e)) : (int64_t)256 * 32;
        }();
        int64_t waves = 1;
        if (h->p.schedule != MML_SCHEDULE_ORDERED)
            waves = std::min<int64_t>(cap, std::max<int64_t>(1, n / 1024));
        // launch_hogwild's small-set rule: a set of fewer than 64 waves' worth of work (65,536
        // ratings) runs as ONE workgroup of 4 waves, so every row stays in one CU's L1 and one
        // XCD's L2 (spread over XCDs, their private write-back L2s replicate the hot rows and lose
        // updates: sigmoid SVD++ on 20 k ratings measured +0.12..0.15 RMSE with 19 one-wave
        // workgroups)
        int wg = 64;
        if (waves > 1 && waves < 64) {
            waves = 4;
            wg = 256;
        }
        const int64_t chunk = (n + waves - 1) / waves;
        const int64_t blocks = waves / (wg / 64);
        const int km = (h->k + 63) / 64;
        const AsymSlot s0 = asym_slot(h, 0), s1 = asym_slot(h, 1);
        const int cache_rows = asym_cache_rows();
#define MML_ASYM_KM1(MODE)                                        \
    do {                                                          \
        if (cache_rows >= 64) MML_ASYM(1, MODE, 64);              \
        else if (cache_rows >= 32) MML_ASYM(1, MODE, 32);         \
        else MML_ASYM(1, MODE, 0);                                \
    } while (0)
#define MML_ASYM(KM, MODE, C)                                                                     \
    asym_sgd_kernel<LOSS, KM, MODE, C><<<(int)blocks, wg, 0, st>>>(                                \
        h->su.get(), h->si.get(), h->sr.get(), n, chunk, s0, s1, h->U.get(), h->V.get(),       \
        h->bu.get(), h->bi.get(), h->k, h->ld, s, cu, ci, h->P.get())
#define MML_ASYM_K(MODE)                    \
    switch (km) {                           \
        case 1: MML_ASYM_KM1(MODE); break;   \
        case 2: MML_ASYM(2, MODE, 0); break;   \
        case 3: MML_ASYM(3, MODE, 0); break;   \
        default: MML_ASYM(4, MODE, 0); break;  \
    }
        switch (asym_mode(h)) {
            case kAsymItem: MML_ASYM_K(kAsymItem); break;
            case kAsymUser: MML_ASYM_K(kAsymUser); break;
            case kSvdpp: MML_ASYM_K(kSvdpp); break;
            case kSigmoidSvdpp: MML_ASYM_K(kSigmoidSvdpp); break;
            default: MML_ASYM_K(kAsymCombined); break;
        }
#undef MML_ASYM_K
#undef MML_ASYM_KM1
#undef MML_ASYM
        MML_HIP(hipGetLastError());
    }
    asym_precompute(h);
    h->last_launches = 1;
}

template <int LOSS>
void run_epoch(mml_bmf* h, const BmfScalars& s, const int32_t* seq) {
    const int32_t* cu = h->p.frequency_regularization ? h->cnt_u.get() : nullptr;
    const int32_t* ci = h->p.frequency_regularization ? h->cnt_i.get() : nullptr;
    int launches = 0;
    if (h->n == 0) {
        h->last_launches = 0;
        return;
    }
    switch (h->p.schedule) {
        case MML_SCHEDULE_ORDERED:
            launch_ordered<LOSS>(h, h->whole_off.get(), 1, 0, 1, s, cu, ci);
            launches = 1;
            break;
        case MML_SCHEDULE_DSGD:
            for (int32_t x = 0; x < h->G; ++x) {
                launch_ordered<LOSS>(h, h->block_off.get(), h->G, seq[x], h->G, s, cu, ci);
                ++launches;
            }
            break;
        default:
            launch_hogwild<LOSS>(h, s, cu, ci);
            launches = 1;
            break;
    }
    h->last_launches = launches;
}

}  // namespace

using mml::guard;

// ------------------------------------------------------------------ multi-device handles
// A handle on a multi-device context (mml_ctx_create_multi) is the one-process form of SURVEY
// 8(e)'s user shards: the ratings are split into contiguous user ranges of equal rating count
// (visit order kept within a shard), one single-device handle per GPU trains its range with the
// Hogwild schedule, and after every epoch one RCCL all-reduce of V || b_i over the devices
// (ncclCommInitAll communicator, one host thread per device) averages the item side.
namespace {

void single_device_only(const mml_bmf* h) {
    if (h->ctx->multi())
        mml::fail(MML_ERR_STATE, "not available on a multi-device context (user-sharded Hogwild "
                                 "training, Predict and Evaluate only)");
}

void multi_create(mml_ctx* ctx, const mml_bmf_params* params, int32_t n_users, int32_t n_items,
                  mml_bmf* h) {
    MML_REQUIRE(params->model == MML_MF_BIASED || params->model == MML_MF_PLAIN,
                "a multi-device context trains MML_MF_BIASED / MML_MF_PLAIN");
    MML_REQUIRE(params->schedule >= MML_SCHEDULE_ORDERED &&
                    params->schedule <= MML_SCHEDULE_HOGWILD_COHERENT,
                "unknown schedule");
    h->ctx = ctx;
    h->p = *params;
    h->n_users = n_users;
    h->n_items = n_items;
    h->k = params->num_factors;
    h->shards.assign(ctx->sub.size(), nullptr);
    for (size_t d = 0; d < ctx->sub.size(); ++d) {
        const mml_status st = mml_bmf_create(ctx->sub[d], params, n_users, n_items, &h->shards[d]);
        if (st != MML_OK) mml::fail(st, mml_last_error());
    }
    h->ub.assign(ctx->sub.size() + 1, n_users);
    h->ub[0] = 0;
}

bool multi_dsgd(const mml_bmf* h) { return h->p.schedule == MML_SCHEDULE_DSGD; }
bool ring_mode(const mml_bmf* h);
// entry points that read or average the model outside the ring's collectives: a DSGD ring rank
// holds stale copies of the rows other ranks trained since the last sync, so they are refused
void no_ring(const mml_bmf* h, const char* what) {
    if (ring_mode(h))
        mml::fail(MML_ERR_STATE, std::string(what) + " is not available on a DSGD ring rank (the "
                                 "ring's collectives are get_model, predict, evaluate, objective)");
}
template <class F>
void ring_all(mml_bmf* h, F&& f);

// a shard's frequency-regularisation / InitModel counts are the whole data set's
mml_status upload_counts(mml_bmf* s, const std::vector<int32_t>& cu,
                         const std::vector<int32_t>& ci) {
    return mml::guard([&] {
        s->ctx->activate();
        hipStream_t st = s->ctx->stream;
        if (!cu.empty())
            MML_HIP(hipMemcpyAsync(s->cnt_u.get(), cu.data(), sizeof(int32_t) * cu.size(),
                                   hipMemcpyHostToDevice, st));
        if (!ci.empty())
            MML_HIP(hipMemcpyAsync(s->cnt_i.get(), ci.data(), sizeof(int32_t) * ci.size(),
                                   hipMemcpyHostToDevice, st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

void multi_set_data(mml_bmf* h, const int32_t* users, const int32_t* items, const float* values,
                    int64_t n, const int32_t* order) {
    const int32_t nd = (int32_t)h->shards.size();
    for (int64_t x = 0; x < n; ++x) {
        MML_REQUIRE(users[x] >= 0 && users[x] < h->n_users && items[x] >= 0 &&
                        items[x] < h->n_items,
                    "rating user/item id or order index out of range");
        if (order) MML_REQUIRE(order[x] >= 0 && order[x] < n, "order index out of range");
    }
    h->cnt_u_host.assign(h->n_users, 0);
    h->cnt_i_host.assign(h->n_items, 0);
    for (int64_t x = 0; x < n; ++x) {
        ++h->cnt_u_host[users[x]];
        ++h->cnt_i_host[items[x]];
    }
    if (multi_dsgd(h)) {  // the ring's ranks each keep the whole set (set_blocks picks rows)
        ring_all(h, [&](int32_t d) {
            return mml_bmf_set_data(h->shards[d], users, items, values, n, order);
        });
        h->G = 0;
        h->n = n;
        h->has_data = true;
        return;
    }
    h->ub = mml::balanced_user_bounds(users, n, h->n_users, nd);
    std::vector<std::vector<int32_t>> su(nd), si(nd);
    std::vector<std::vector<float>> sr(nd);
    for (int64_t x = 0; x < n; ++x) {  // visit order, split by the owner of the user
        const int64_t o = order ? order[x] : x;
        const int32_t d = mml::owner_of(h->ub, users[o]);
        su[d].push_back(users[o]);
        si[d].push_back(items[o]);
        sr[d].push_back(values[o]);
    }
    mml::on_devices(h->ctx, [&](int32_t d) {
        mml_status st = mml_bmf_set_data(h->shards[d], su[d].data(), si[d].data(), sr[d].data(),
                                         (int64_t)su[d].size(), nullptr);
        if (st == MML_OK) st = upload_counts(h->shards[d], h->cnt_u_host, h->cnt_i_host);
        return st;
    });
    h->n = n;
    h->has_data = true;
}

// per-device index lists of (user-routed) queries: unknown users go to device 0
std::vector<std::vector<int64_t>> route_users(const mml_bmf* h, const int32_t* users, int64_t n) {
    std::vector<std::vector<int64_t>> r(h->shards.size());
    for (int64_t x = 0; x < n; ++x) {
        const int32_t u = users[x];
        r[u >= 0 && u < h->n_users ? mml::owner_of(h->ub, u) : 0].push_back(x);
    }
    return r;
}

void multi_predict(mml_bmf* h, const int32_t* users, const int32_t* items, int64_t n,
                   float* out) {
    const auto r = route_users(h, users, n);
    mml::on_devices(h->ctx, [&](int32_t d) {
        const auto& ix = r[d];
        if (ix.empty()) return (mml_status)MML_OK;
        std::vector<int32_t> u(ix.size()), i(ix.size());
        std::vector<float> o(ix.size());
        for (size_t x = 0; x < ix.size(); ++x) {
            u[x] = users[ix[x]];
            i[x] = items[ix[x]];
        }
        const mml_status st = mml_bmf_predict(h->shards[d], u.data(), i.data(),
                                              (int64_t)ix.size(), o.data());
        for (size_t x = 0; st == MML_OK && x < ix.size(); ++x) out[ix[x]] = o[x];
        return st;
    });
}

void multi_evaluate(mml_bmf* h, const int32_t* users, const int32_t* items, const float* values,
                    int64_t n, float* out) {
    const auto r = route_users(h, users, n);
    const size_t nd = h->shards.size();
    std::vector<double> sse(nd, 0.0), sae(nd, 0.0);
    mml::on_devices(h->ctx, [&](int32_t d) {
        const auto& ix = r[d];
        if (ix.empty()) return (mml_status)MML_OK;
        std::vector<int32_t> u(ix.size()), i(ix.size());
        std::vector<float> v(ix.size());
        for (size_t x = 0; x < ix.size(); ++x) {
            u[x] = users[ix[x]];
            i[x] = items[ix[x]];
            v[x] = values[ix[x]];
        }
        float o[2] = {0.0f, 0.0f};
        const mml_status st = mml_bmf_evaluate(h->shards[d], u.data(), i.data(), v.data(),
                                               (int64_t)ix.size(), o);
        sse[d] = (double)o[0] * o[0] * (double)ix.size();
        sae[d] = (double)o[1] * (double)ix.size();
        return st;
    });
    double a = 0.0, b = 0.0;
    for (size_t d = 0; d < nd; ++d) {
        a += sse[d];
        b += sae[d];
    }
    out[0] = n > 0 ? (float)std::sqrt(a / (double)n) : 0.0f;
    out[1] = n > 0 ? (float)(b / (double)n) : 0.0f;
}

void multi_get_model(mml_bmf* h, float* U, float* V, float* bu, float* bi) {
    mml::on_devices(h->ctx, [&](int32_t d) {
        return mml::guard([&] {
            mml_bmf* s = h->shards[d];
            s->ctx->activate();
            const int64_t lo = h->ub[d], rows = h->ub[d + 1] - h->ub[d];
            if (U && rows > 0) download_padded(s, U + lo * h->k, s->U.get() + lo * s->ld, rows);
            if (bu && rows > 0)
                MML_HIP(hipMemcpyAsync(bu + lo, s->bu.get() + lo, sizeof(float) * rows,
                                       hipMemcpyDeviceToHost, s->ctx->stream));
            if (d == 0) {
                if (V) download_padded(s, V, s->V.get(), h->n_items);
                if (bi && h->n_items)
                    MML_HIP(hipMemcpyAsync(bi, s->bi.get(), sizeof(float) * h->n_items,
                                           hipMemcpyDeviceToHost, s->ctx->stream));
            }
            MML_HIP(hipStreamSynchronize(s->ctx->stream));
        });
    });
}

// mml_bmf_set_data_device on a multi-device context: the arrays live on the context's first
// device.  The counts, the user ranges of equal rating count and a stable partition of the
// (visit-ordered) stream by owner run there; each shard then takes its contiguous part (a peer
// copy when its device differs).  Equal to mml_bmf_set_data with the same arrays on the host.
void multi_set_data_device(mml_bmf* h, const int32_t* users, const int32_t* items,
                           const float* values, int64_t n, const int32_t* order) {
    MML_REQUIRE(!multi_dsgd(h), "the DSGD ring takes host arrays (mml_bmf_set_data, then "
                                "mml_bmf_set_blocks)");
    const int32_t nd = (int32_t)h->shards.size();
    mml_bmf* s0 = h->shards[0];
    s0->ctx->activate();
    hipStream_t st = s0->ctx->stream;
    mml::DeviceArray<int32_t> cu, ci, bad;
    cu.alloc(std::max<int32_t>(1, h->n_users));
    ci.alloc(std::max<int32_t>(1, h->n_items));
    bad.alloc(1);
    MML_HIP(hipMemsetAsync(cu.get(), 0, sizeof(int32_t) * cu.count, st));
    MML_HIP(hipMemsetAsync(ci.get(), 0, sizeof(int32_t) * ci.count, st));
    MML_HIP(hipMemsetAsync(bad.get(), 0, sizeof(int32_t), st));
    if (n > 0) {
        count_kernel<<<grid_for(n), 256, 0, st>>>(users, items, n, h->n_users, h->n_items,
                                                   cu.get(), ci.get(), bad.get());
        if (order) check_order_kernel<<<grid_for(n), 256, 0, st>>>(order, n, n, bad.get());
        MML_HIP(hipGetLastError());
    }
    int32_t flag = 0;
    h->cnt_u_host.assign(h->n_users, 0);
    h->cnt_i_host.assign(h->n_items, 0);
    MML_HIP(hipMemcpyAsync(&flag, bad.get(), sizeof(int32_t), hipMemcpyDeviceToHost, st));
    if (h->n_users)
        MML_HIP(hipMemcpyAsync(h->cnt_u_host.data(), cu.get(), sizeof(int32_t) * h->n_users,
                               hipMemcpyDeviceToHost, st));
    if (h->n_items)
        MML_HIP(hipMemcpyAsync(h->cnt_i_host.data(), ci.get(), sizeof(int32_t) * h->n_items,
                               hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    MML_REQUIRE(!flag, "rating user/item id or order index out of range");
    h->has_data = false;
    h->ub = mml::balanced_user_bounds_counts(
        std::vector<int64_t>(h->cnt_u_host.begin(), h->cnt_u_host.end()), n, nd);
    // the stream in visit order, partitioned stably by the owner of its user
    mml::DeviceArray<int32_t> ou, oi, orr, pu, pi, pr;
    const int32_t *su = users, *si = items;
    const int32_t* sr = reinterpret_cast<const int32_t*>(values);
    std::vector<int64_t> goff(nd + 1, 0);
    goff[nd] = n;
    if (n > 0 && order) {
        ou.alloc(n);
        oi.alloc(n);
        orr.alloc(n);
        gather_stream_kernel<<<grid_for(n), 256, 0, st>>>(users, items, values, order, n,
                                                          ou.get(), oi.get(),
                                                          reinterpret_cast<float*>(orr.get()));
        MML_HIP(hipGetLastError());
        su = ou.get();
        si = oi.get();
        sr = orr.get();
    }
    if (n > 0 && nd > 1) {
        MML_REQUIRE(nd <= 8, "mml_bmf_set_data_device on a multi-device context shards over at "
                             "most 8 devices (use mml_bmf_set_data)");
        std::vector<uint8_t> table(h->n_users);
        for (int32_t d = 0; d < nd; ++d)
            for (int32_t u = h->ub[d]; u < h->ub[d + 1]; ++u) table[u] = (uint8_t)d;
        mml::XcdSplit xs;
        xs.set_table(st, table);
        pu.alloc(n);
        pi.alloc(n);
        pr.alloc(n);
        const int32_t* in[3] = {su, si, sr};
        int32_t* out[3] = {pu.get(), pi.get(), pr.get()};
        xs.partition(st, su, n, 3, in, out);
        int64_t g[9];
        MML_HIP(hipMemcpyAsync(g, xs.goff.get(), sizeof(g), hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        for (int32_t d = 0; d < nd; ++d) goff[d] = g[d];
        ou.reset();
        oi.reset();
        orr.reset();
        su = pu.get();
        si = pi.get();
        sr = pr.get();
    }
    MML_HIP(hipStreamSynchronize(st));
    for (int32_t d = 0; d < nd; ++d) {
        mml_bmf* s = h->shards[d];
        const int64_t o = goff[d], m = goff[d + 1] - goff[d];
        const int32_t* du = m ? su + o : nullptr;
        const int32_t* di = m ? si + o : nullptr;
        const float* dr = m ? reinterpret_cast<const float*>(sr) + o : nullptr;
        mml::DeviceArray<int32_t> tu, ti, tr;  // the shard's part on its own device
        if (m > 0 && s->ctx->device != s0->ctx->device) {
            s->ctx->activate();
            tu.alloc(m);
            ti.alloc(m);
            tr.alloc(m);
            hipStream_t ss = s->ctx->stream;
            MML_HIP(hipMemcpyPeerAsync(tu.get(), s->ctx->device, du, s0->ctx->device,
                                       sizeof(int32_t) * m, ss));
            MML_HIP(hipMemcpyPeerAsync(ti.get(), s->ctx->device, di, s0->ctx->device,
                                       sizeof(int32_t) * m, ss));
            MML_HIP(hipMemcpyPeerAsync(tr.get(), s->ctx->device, dr, s0->ctx->device,
                                       sizeof(float) * m, ss));
            MML_HIP(hipStreamSynchronize(ss));
            du = tu.get();
            di = ti.get();
            dr = reinterpret_cast<const float*>(tr.get());
        }
        mml_status r = mml_bmf_set_data_device(s, du, di, dr, m, nullptr);
        if (r == MML_OK) r = upload_counts(s, h->cnt_u_host, h->cnt_i_host);
        if (r != MML_OK)
            mml::fail(r, "device " + std::to_string(s->ctx->device) + ": " + mml_last_error());
    }
    h->n = n;
    h->has_data = true;
}

// The item average of the user shards without a communicator (a device listed more than once):
// the other shards' V || b_i are staged on shard 0's device (peer copies; device-local when the
// device repeats), averaged there in shard order (average_rows_kernel) and copied back.  Every
// shard's stream waits for the copies before its next call.  Equal bit for bit to the in-process
// emulation (tests/test_dist.py): sum over the shards left to right, then / N.
void multi_average_peer(mml_bmf* h) {
    mml_bmf* s0 = h->shards[0];
    s0->ctx->activate();
    if (!h->ev_ar0) {
        MML_HIP(hipEventCreate(&h->ev_ar0));
        MML_HIP(hipEventCreate(&h->ev_ar1));
    }
    std::vector<mml_ctx*> ctxs;
    std::vector<std::vector<float*>> arr;
    for (mml_bmf* s : h->shards) {
        ctxs.push_back(s->ctx);
        arr.push_back({s->V.get(), s->bi.get()});
    }
    mml::peer_average(ctxs, arr, {(int64_t)h->n_items * s0->ld, (int64_t)h->n_items},
                      h->avg_stage, h->ev_ar0, h->ev_ar1);
    h->has_ar = true;
}

// One epoch of the user shards, then the item average.  Phase 1 runs every shard's epoch (one
// after another when the devices repeat -- each shard then has the whole GPU, as it would have a
// GPU of its own -- else one host thread per device); phase 2 averages V || b_i and runs only
// after every shard succeeded, so no rank ever waits in a collective another one skipped.
void multi_epoch(mml_bmf* h, float learn_rate) {
    const int32_t nd = (int32_t)h->shards.size();
    std::vector<float> ms(nd, 0.0f);
    auto epoch = [&](int32_t d) {
        const mml_status st = mml_bmf_iterate(h->shards[d], learn_rate, nullptr);
        if (st == MML_OK) ms[d] = h->shards[d]->last_ms;
        return st;
    };
    if (h->ctx->repeated) {
        for (int32_t d = 0; d < nd; ++d) {
            const mml_status st = epoch(d);
            if (st != MML_OK) mml::fail(st, "shard " + std::to_string(d) + ": " + mml_last_error());
        }
    } else {
        mml::on_devices(h->ctx, epoch);
    }
    if (h->ctx->repeated || !h->shards[0]->ctx->comm) {
        multi_average_peer(h);
    } else {
        mml::on_devices(h->ctx, [&](int32_t d) { return mml_bmf_allreduce_items(h->shards[d]); });
        h->has_ar = false;
    }
    h->last_ms = *std::max_element(ms.begin(), ms.end());
    h->last_launches = h->shards[0]->last_launches;
}

// ---- DSGD ring (the reference's MaxThreads = G schedule, BiasedMatrixFactorization.cs:205-215,
// over several devices), one RANK per device.  Blocks of one sub-epoch share no user or item, so
// rank r runs the block rows it owns, [r m, (r + 1) m) with m = G / ranks, exactly as the
// single-device DSGD launch would, and the only exchange is an item group moving to the rank whose
// window (the m item groups its rows visit) needs it next: packed on the holder, sent, scattered
// on the new holder.  The result is the single-device DSGD result, bit for bit.
//
// Every rank keeps the whole rating set (set_data), derives the groups from the blocks
// (set_blocks) and tracks which rank holds the newest rows of each item group (hold[], the same on
// every rank).  Transport: RCCL ncclSend / ncclRecv and ncclBroadcast on a communicator (one
// process per GPU, mml_ctx_comm_init; or mml_ctx_create_multi over distinct devices, one host
// thread per rank), or peer copies between host barriers on a context that lists a device more
// than once (mml::PeerGroup).  get_model / predict / evaluate on a rank first bring every rank to
// the newest model (ring_sync, a collective: every rank calls them).

struct RingRank {
    int32_t r, n;
};
RingRank ring_rank(const mml_ctx* c) {
    if (c->comm && c->nranks > 1) return {c->rank, c->nranks};
    if (c->peers && c->peers->n > 1) return {c->peer_rank, c->peers->n};
    return {0, 1};
}
// a single-device handle that is one rank of the ring
bool ring_mode(const mml_bmf* h) {
    return !h->ctx->multi() && h->p.schedule == MML_SCHEDULE_DSGD && h->p.model <= MML_MF_PLAIN &&
           ring_rank(h->ctx).n > 1;
}

struct RingMove {
    int32_t from, to;
    int64_t r0, r1;  // rows of the group-ordered item list
};

// the group moves before sub-epoch sq (group c is visited by block row (c - sq) mod G), merged
// into runs of consecutive groups with the same endpoints; updates hold[] -- the same on every rank
std::vector<RingMove> ring_moves(mml_bmf* h, int32_t sq, int32_t m) {
    const int32_t G = h->G;
    std::vector<RingMove> mv;
    for (int32_t c = 0; c < G; ++c) {
        const int32_t to = ((c - sq) % G + G) % G / m, from = h->hold[c];
        h->hold[c] = to;
        if (from < 0 || from == to || h->gi_off[c + 1] == h->gi_off[c]) continue;
        if (!mv.empty() && mv.back().from == from && mv.back().to == to &&
            mv.back().r1 == h->gi_off[c])
            mv.back().r1 = h->gi_off[c + 1];
        else
            mv.push_back({from, to, h->gi_off[c], h->gi_off[c + 1]});
    }
    return mv;
}

// this rank's part of the moves: its packed runs to their new holders, the runs it receives into
// its staging rows (same offsets as on the sender)
void ring_exchange(mml_bmf* h, const std::vector<RingMove>& mv, int32_t r) {
    mml_ctx* c = h->ctx;
    hipStream_t st = c->stream;
    const int64_t ld = h->ld;
    if (c->comm) {
        MML_RCCL(ncclGroupStart());
        for (const RingMove& v : mv) {
            const int64_t n = v.r1 - v.r0;
            if (v.from == r) {
                MML_RCCL(ncclSend(h->stage_v.get() + v.r0 * ld, (size_t)(n * ld), ncclFloat, v.to,
                                  c->comm, st));
                MML_RCCL(ncclSend(h->stage_b.get() + v.r0, (size_t)n, ncclFloat, v.to, c->comm,
                                  st));
            } else if (v.to == r) {
                MML_RCCL(ncclRecv(h->stage_v.get() + v.r0 * ld, (size_t)(n * ld), ncclFloat,
                                  v.from, c->comm, st));
                MML_RCCL(ncclRecv(h->stage_b.get() + v.r0, (size_t)n, ncclFloat, v.from, c->comm,
                                  st));
            }
        }
        MML_RCCL(ncclGroupEnd());
        return;
    }
    mml::PeerGroup* g = c->peers.get();
    MML_HIP(hipStreamSynchronize(st));  // this rank's packs are complete
    g->publish(c, 0, h->stage_v.get());
    g->publish(c, 1, h->stage_b.get());
    g->barrier();
    for (const RingMove& v : mv) {
        if (v.to != r) continue;
        const int64_t n = v.r1 - v.r0;
        MML_HIP(hipMemcpyPeerAsync(h->stage_v.get() + v.r0 * ld, c->device,
                                   static_cast<float*>(g->peer(v.from, 0)) + v.r0 * ld,
                                   g->devices[v.from], sizeof(float) * n * ld, st));
        MML_HIP(hipMemcpyPeerAsync(h->stage_b.get() + v.r0, c->device,
                                   static_cast<float*>(g->peer(v.from, 1)) + v.r0,
                                   g->devices[v.from], sizeof(float) * n, st));
    }
    MML_HIP(hipStreamSynchronize(st));
    g->barrier();  // the senders' staging rows are read before anyone packs again
}

// count floats of rank q's buffer broadcast to every rank (RCCL broadcast or peer copies)
void ring_bcast(mml_bmf* h, float* buf, int64_t count, int32_t q) {
    mml_ctx* c = h->ctx;
    hipStream_t st = c->stream;
    if (c->comm) {
        if (count > 0)
            MML_RCCL(ncclBroadcast(buf, buf, (size_t)count, ncclFloat, q, c->comm, st));
        return;
    }
    mml::PeerGroup* g = c->peers.get();
    MML_HIP(hipStreamSynchronize(st));
    g->publish(c, 0, buf);
    g->barrier();
    if (c->peer_rank != q && count > 0)
        MML_HIP(hipMemcpyPeerAsync(buf, c->device, g->peer(q, 0), g->devices[q],
                                   sizeof(float) * count, st));
    MML_HIP(hipStreamSynchronize(st));
    g->barrier();
}

// every rank gets the newest copy of every row: rank q broadcasts the user rows of its block rows
// and the item groups it holds, the others scatter them; then no group has a holder (hold = -1)
void ring_sync(mml_bmf* h) {
    if (h->ring_synced || h->G == 0) {
        h->ring_synced = true;
        return;
    }
    const RingRank rr = ring_rank(h->ctx);
    const int32_t m = h->G / rr.n;
    h->ctx->activate();
    hipStream_t st = h->ctx->stream;
    std::vector<std::vector<int32_t>> uid(rr.n), iid(rr.n);
    for (int32_t u = 0; u < h->n_users; ++u)
        if (h->ugroup[u] >= 0) uid[h->ugroup[u] / m].push_back(u);
    for (int32_t i = 0; i < h->n_items; ++i) {
        const int32_t g = h->igroup[i];
        if (g >= 0 && h->hold[g] >= 0) iid[h->hold[g]].push_back(i);
    }
    mml::DeviceArray<int32_t> ids;
    mml::DeviceArray<float> buf;
    for (int32_t q = 0; q < rr.n; ++q) {
        const int64_t nu = (int64_t)uid[q].size(), ni = (int64_t)iid[q].size();
        const int64_t count = (nu + ni) * (h->ld + 1);
        ids.reserve(std::max<int64_t>(1, nu + ni));
        buf.reserve(std::max<int64_t>(1, count));
        if (nu)
            MML_HIP(hipMemcpyAsync(ids.get(), uid[q].data(), sizeof(int32_t) * nu,
                                   hipMemcpyHostToDevice, st));
        if (ni)
            MML_HIP(hipMemcpyAsync(ids.get() + nu, iid[q].data(), sizeof(int32_t) * ni,
                                   hipMemcpyHostToDevice, st));
        float* bu_ = buf.get() + nu * h->ld;          // [U rows][b_u][V rows][b_i]
        float* v_ = bu_ + nu;
        float* bi_ = v_ + ni * h->ld;
        if (q == rr.r) {
            if (nu)
                rows_gather_kernel<<<grid_for(nu * h->ld), 256, 0, st>>>(
                    h->U.get(), h->bu.get(), ids.get(), nu, h->ld, buf.get(), bu_);
            if (ni)
                rows_gather_kernel<<<grid_for(ni * h->ld), 256, 0, st>>>(
                    h->V.get(), h->bi.get(), ids.get() + nu, ni, h->ld, v_, bi_);
            MML_HIP(hipGetLastError());
        }
        ring_bcast(h, buf.get(), count, q);
        if (q != rr.r) {
            if (nu)
                rows_scatter_kernel<<<grid_for(nu * h->ld), 256, 0, st>>>(
                    buf.get(), bu_, ids.get(), nu, h->ld, h->U.get(), h->bu.get());
            if (ni)
                rows_scatter_kernel<<<grid_for(ni * h->ld), 256, 0, st>>>(
                    v_, bi_, ids.get() + nu, ni, h->ld, h->V.get(), h->bi.get());
            MML_HIP(hipGetLastError());
        }
        MML_HIP(hipStreamSynchronize(st));  // ids / buf are reused by the next rank's round
    }
    std::fill(h->hold.begin(), h->hold.end(), -1);
    h->ring_synced = true;
}

// the user group and item group of every rating of the blocks: block b = j G + c
__global__ __launch_bounds__(256) void ring_groups_kernel(const int64_t* __restrict__ off,
                                                          int64_t nb, int32_t G,
                                                          const int32_t* __restrict__ idx,
                                                          int64_t total,
                                                          const int32_t* __restrict__ users,
                                                          const int32_t* __restrict__ items,
                                                          int32_t* __restrict__ ug,
                                                          int32_t* __restrict__ ig, int32_t check,
                                                          int32_t* __restrict__ bad) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < total;
         x += (int64_t)gridDim.x * blockDim.x) {
        int64_t lo = 0, hi = nb;  // the block of position x: off[b] <= x < off[b + 1]
        while (hi - lo > 1) {
            const int64_t mid = (lo + hi) >> 1;
            if (off[mid] <= x) lo = mid;
            else hi = mid;
        }
        const int32_t j = (int32_t)(lo / G), c = (int32_t)(lo % G);
        const int32_t u = users[idx[x]], i = items[idx[x]];
        if (!check) {
            ug[u] = j;
            ig[i] = c;
        } else if (ug[u] != j || ig[i] != c) {
            atomicOr(bad, 1);
        }
    }
}

// set_blocks on a rank: the groups (checked to be a user-group x item-group partition), the item
// list in group order, and this rank's block rows as its stream (block_off local to them)
void ring_set_blocks(mml_bmf* h, int32_t G, const int64_t* offsets, const int32_t* indices) {
    const RingRank rr = ring_rank(h->ctx);
    MML_REQUIRE(G % rr.n == 0, "the DSGD ring needs num_groups (MaxThreads) to be a multiple of "
                               "the device count");
    const int64_t nb = (int64_t)G * G;
    MML_REQUIRE(offsets[0] == 0, "offsets[0] must be 0");
    for (int64_t b = 0; b < nb; ++b)
        MML_REQUIRE(offsets[b + 1] >= offsets[b], "offsets must be non-decreasing");
    const int64_t total = offsets[nb];
    MML_REQUIRE(total <= h->n && (total == 0 || indices), "block indices exceed ratings");
    if (h->has_model && h->G > 0) ring_sync(h);  // the holders refer to the old groups
    h->ctx->activate();
    hipStream_t st = h->ctx->stream;
    mml::DeviceArray<int64_t> doff;
    mml::DeviceArray<int32_t> ord, ug, ig;
    doff.alloc(nb + 1);
    ord.alloc(std::max<int64_t>(1, total));
    ug.alloc(std::max<int32_t>(1, h->n_users));
    ig.alloc(std::max<int32_t>(1, h->n_items));
    MML_HIP(hipMemcpyAsync(doff.get(), offsets, sizeof(int64_t) * (nb + 1), hipMemcpyHostToDevice,
                           st));
    if (total > 0)
        MML_HIP(hipMemcpyAsync(ord.get(), indices, sizeof(int32_t) * total, hipMemcpyHostToDevice,
                               st));
    MML_HIP(hipMemsetAsync(ug.get(), 0xff, sizeof(int32_t) * ug.count, st));
    MML_HIP(hipMemsetAsync(ig.get(), 0xff, sizeof(int32_t) * ig.count, st));
    MML_HIP(hipMemsetAsync(h->scratch_i32.get(), 0, sizeof(int32_t), st));
    int32_t bad = 0;
    if (total > 0) {
        check_order_kernel<<<grid_for(total), 256, 0, st>>>(ord.get(), total, h->n,
                                                            h->scratch_i32.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemcpyAsync(&bad, h->scratch_i32.get(), sizeof(int32_t), hipMemcpyDeviceToHost,
                               st));
        MML_HIP(hipStreamSynchronize(st));
        MML_REQUIRE(!bad, "block index out of range");
        for (int32_t check = 0; check < 2; ++check)
            ring_groups_kernel<<<grid_for(total), 256, 0, st>>>(
                doff.get(), nb, G, ord.get(), total, h->raw_u.get(), h->raw_i.get(), ug.get(),
                ig.get(), check, h->scratch_i32.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemcpyAsync(&bad, h->scratch_i32.get(), sizeof(int32_t), hipMemcpyDeviceToHost,
                               st));
    }
    std::vector<int32_t> ugh(h->n_users), igh(h->n_items);
    if (h->n_users)
        MML_HIP(hipMemcpyAsync(ugh.data(), ug.get(), sizeof(int32_t) * h->n_users,
                               hipMemcpyDeviceToHost, st));
    if (h->n_items)
        MML_HIP(hipMemcpyAsync(igh.data(), ig.get(), sizeof(int32_t) * h->n_items,
                               hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    MML_REQUIRE(!bad, "blocks are not a user-group x item-group partition");
    std::vector<int64_t> gi_off(G + 1, 0);
    for (int32_t i = 0; i < h->n_items; ++i)
        if (igh[i] >= 0) ++gi_off[igh[i] + 1];
    for (int32_t c = 0; c < G; ++c) gi_off[c + 1] += gi_off[c];
    std::vector<int32_t> gi_ids(std::max<int64_t>(1, gi_off[G]));
    {
        std::vector<int64_t> at(gi_off.begin(), gi_off.end() - 1);
        for (int32_t i = 0; i < h->n_items; ++i)
            if (igh[i] >= 0) gi_ids[at[igh[i]]++] = i;
    }
    // this rank's block rows [r m, (r + 1) m): one contiguous run of the blocks' indices
    const int32_t m = G / rr.n;
    const int64_t b0 = (int64_t)rr.r * m * G, b1 = b0 + (int64_t)m * G;
    const int64_t x0 = offsets[b0], x1 = offsets[b1];
    if (x1 > x0) {
        gather_stream_kernel<<<grid_for(x1 - x0), 256, 0, st>>>(
            h->raw_u.get(), h->raw_i.get(), h->raw_r.get(), ord.get() + x0, x1 - x0, h->su.get(),
            h->si.get(), h->sr.get());
        MML_HIP(hipGetLastError());
    }
    std::vector<int64_t> loff((size_t)m * G + 1);
    for (int64_t lb = 0; lb <= (int64_t)m * G; ++lb) loff[lb] = offsets[b0 + lb] - x0;
    h->block_off.alloc(loff.size());
    MML_HIP(hipMemcpyAsync(h->block_off.get(), loff.data(), sizeof(int64_t) * loff.size(),
                           hipMemcpyHostToDevice, st));
    h->gi_ids.alloc(gi_ids.size());
    MML_HIP(hipMemcpyAsync(h->gi_ids.get(), gi_ids.data(), sizeof(int32_t) * gi_ids.size(),
                           hipMemcpyHostToDevice, st));
    h->stage_v.alloc(gi_ids.size() * (size_t)h->ld);
    h->stage_b.alloc(gi_ids.size());
    MML_HIP(hipStreamSynchronize(st));
    h->ugroup.swap(ugh);
    h->igroup.swap(igh);
    h->gi_off.swap(gi_off);
    h->hold.assign(G, -1);
    h->ring_synced = true;
    h->row0 = rr.r * m;
    h->G = G;
}

template <int LOSS>
void ring_epoch(mml_bmf* h, float learn_rate, const int32_t* seq) {
    const RingRank rr = ring_rank(h->ctx);
    const int32_t G = h->G, m = G / rr.n;
    BmfScalars sc;
    sc.gb = h->gb;
    sc.min_rating = h->min_rating;
    sc.range = h->max_rating - h->min_rating;
    sc.lr = learn_rate;
    sc.blr = h->p.bias_learn_rate * learn_rate;
    sc.bias_reg = h->p.bias_reg;
    sc.reg_u = h->p.reg_u;
    sc.reg_i = h->p.reg_i;
    h->ctx->activate();
    hipStream_t st = h->ctx->stream;
    const bool fr = h->p.frequency_regularization != 0;
    MML_HIP(hipEventRecord(h->ctx->ev_begin, st));
    for (int32_t x = 0; x < G; ++x) {
        const std::vector<RingMove> mv = ring_moves(h, seq[x], m);
        for (const RingMove& v : mv) {  // pack what leaves this rank (after its last SGD launch)
            if (v.from != rr.r) continue;
            const int64_t n = v.r1 - v.r0;
            rows_gather_kernel<<<grid_for(n * h->ld), 256, 0, st>>>(
                h->V.get(), h->bi.get(), h->gi_ids.get() + v.r0, n, h->ld,
                h->stage_v.get() + v.r0 * h->ld, h->stage_b.get() + v.r0);
        }
        MML_HIP(hipGetLastError());
        if (!mv.empty()) ring_exchange(h, mv, rr.r);
        for (const RingMove& v : mv) {  // scatter what arrived
            if (v.to != rr.r) continue;
            const int64_t n = v.r1 - v.r0;
            rows_scatter_kernel<<<grid_for(n * h->ld), 256, 0, st>>>(
                h->stage_v.get() + v.r0 * h->ld, h->stage_b.get() + v.r0,
                h->gi_ids.get() + v.r0, n, h->ld, h->V.get(), h->bi.get());
        }
        MML_HIP(hipGetLastError());
        launch_ordered<LOSS>(h, h->block_off.get(), G, seq[x], m, sc,
                             fr ? h->cnt_u.get() : nullptr, fr ? h->cnt_i.get() : nullptr,
                             h->row0);
    }
    MML_HIP(hipEventRecord(h->ctx->ev_end, st));
    MML_HIP(hipEventSynchronize(h->ctx->ev_end));
    MML_HIP(hipEventElapsedTime(&h->last_ms, h->ctx->ev_begin, h->ctx->ev_end));
    h->last_launches = G;
    h->ring_synced = false;
}

// the ranks of a multi-device context, one host thread each (a repeated device: its peer group is
// reset first and released by a failing rank, so no rank waits at a barrier for ever)
template <class F>
void ring_all(mml_bmf* h, F&& f) {
    mml::PeerGroup* g = h->shards[0]->ctx->peers.get();
    if (g) g->reset();
    mml::on_devices(h->ctx, [&](int32_t d) {
        const mml_status st = f(d);
        if (st != MML_OK && g) g->abort();
        return st;
    });
}

// every shard (rank) of a multi-device DSGD handle brought to the newest model
void multi_ring_sync(mml_bmf* h) {
    ring_all(h, [&](int32_t d) {
        return mml::guard([&] { ring_sync(h->shards[d]); });
    });
}

}  // namespace

extern "C" mml_status mml_bmf_create(mml_ctx* ctx, const mml_bmf_params* params, int32_t n_users,
                                     int32_t n_items, mml_bmf** out) {
    return guard([&] {
        MML_REQUIRE(ctx && params && out, "null argument");
        MML_REQUIRE(n_users >= 0 && n_items >= 0, "negative sizes");
        MML_REQUIRE(params->num_factors >= 1 && params->num_factors <= 256,
                    "num_factors must be in [1, 256]");
        MML_REQUIRE(params->loss >= MML_LOSS_RMSE && params->loss <= MML_LOSS_LOGISTIC,
                    "unknown loss");
        MML_REQUIRE(params->model >= MML_MF_BIASED && params->model <= MML_MF_SIGMOID_SVDPP,
                    "unknown model family");
        MML_REQUIRE(params->schedule >= MML_SCHEDULE_ORDERED &&
                        params->schedule <= MML_SCHEDULE_HOGWILD_COHERENT,
                    "unknown schedule");
        if (ctx->multi()) {
            auto* h = new mml_bmf();
            try {
                multi_create(ctx, params, n_users, n_items, h);
            } catch (...) {
                mml_bmf_destroy(h);
                throw;
            }
            *out = h;
            return;
        }
        ctx->activate();
        auto* h = new mml_bmf();
        try {
            h->ctx = ctx;
            h->p = *params;
            h->n_users = n_users;
            h->n_items = n_items;
            h->k = params->num_factors;
            h->lpr = lanes_per_rating(h->k);
            h->ld = 4 * h->lpr;
            h->U.alloc((size_t)n_users * h->ld);
            h->V.alloc((size_t)n_items * h->ld);
            h->bu.alloc(n_users);
            h->bi.alloc(n_items);
        } catch (...) {
            delete h;
            throw;
        }
        *out = h;
    });
}

extern "C" mml_status mml_bmf_destroy(mml_bmf* h) {
    return guard([&] {
        if (!h) return;
        if (!h->ctx) {  // a create that failed before binding the context
            delete h;
            return;
        }
        if (!h->shards.empty() || (h->ctx && h->ctx->multi())) {
            if (h->ev_ar0 && !h->shards.empty() && h->shards[0]) {
                (void)hipSetDevice(h->shards[0]->ctx->device);
                (void)hipStreamSynchronize(h->shards[0]->ctx->stream);
                (void)hipEventDestroy(h->ev_ar0);
                (void)hipEventDestroy(h->ev_ar1);
            }
            for (mml_bmf* s : h->shards)
                if (s) mml_bmf_destroy(s);
            delete h;
            return;
        }
        (void)hipSetDevice(h->ctx->device);
        (void)hipStreamSynchronize(h->ctx->stream);
        if (h->ev_ar0) (void)hipEventDestroy(h->ev_ar0);
        if (h->ev_ar1) (void)hipEventDestroy(h->ev_ar1);
        delete h;
    });
}

extern "C" mml_status mml_bmf_set_data(mml_bmf* h, const int32_t* users, const int32_t* items,
                                       const float* values, int64_t n, const int32_t* order) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(n >= 0 && n <= INT32_MAX, "rating count out of range");
        MML_REQUIRE(n == 0 || (users && items && values), "null rating arrays");
        if (h->ctx->multi()) return multi_set_data(h, users, items, values, n, order);
        // a ring rank: every rank gets the newest model before the groups are forgotten
        if (ring_mode(h) && h->has_model) ring_sync(h);
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->has_data = false;
        h->n = n;
        h->raw_u.alloc(n);
        h->raw_i.alloc(n);
        h->raw_r.alloc(n);
        mml::DeviceArray<int32_t> ord;
        if (n > 0) {
            MML_HIP(hipMemcpyAsync(h->raw_u.get(), users, sizeof(int32_t) * n,
                                   hipMemcpyHostToDevice, st));
            MML_HIP(hipMemcpyAsync(h->raw_i.get(), items, sizeof(int32_t) * n,
                                   hipMemcpyHostToDevice, st));
            MML_HIP(hipMemcpyAsync(h->raw_r.get(), values, sizeof(float) * n,
                                   hipMemcpyHostToDevice, st));
            if (order) {
                ord.alloc(n);
                MML_HIP(hipMemcpyAsync(ord.get(), order, sizeof(int32_t) * n,
                                       hipMemcpyHostToDevice, st));
            }
        }
        finish_data(h, order ? ord.get() : nullptr);
    });
}

extern "C" mml_status mml_bmf_set_data_device(mml_bmf* h, const int32_t* users,
                                              const int32_t* items, const float* values,
                                              int64_t n, const int32_t* order) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(n >= 0 && n <= INT32_MAX, "rating count out of range");
        MML_REQUIRE(n == 0 || (users && items && values), "null rating arrays");
        // the arrays may come from any stream of the caller's (e.g. torch's): wait for the device
        h->ctx->activate();
        MML_HIP(hipDeviceSynchronize());
        if (h->ctx->multi()) return multi_set_data_device(h, users, items, values, n, order);
        // a ring rank: every rank gets the newest model before the groups are forgotten (as
        // mml_bmf_set_data)
        if (ring_mode(h) && h->has_model) ring_sync(h);
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->has_data = false;
        h->n = n;
        h->raw_u.alloc(n);
        h->raw_i.alloc(n);
        h->raw_r.alloc(n);
        if (n > 0) {
            MML_HIP(hipMemcpyAsync(h->raw_u.get(), users, sizeof(int32_t) * n,
                                   hipMemcpyDeviceToDevice, st));
            MML_HIP(hipMemcpyAsync(h->raw_i.get(), items, sizeof(int32_t) * n,
                                   hipMemcpyDeviceToDevice, st));
            MML_HIP(hipMemcpyAsync(h->raw_r.get(), values, sizeof(float) * n,
                                   hipMemcpyDeviceToDevice, st));
        }
        finish_data(h, order);
    });
}

extern "C" mml_status mml_bmf_set_blocks(mml_bmf* h, int32_t num_groups, const int64_t* offsets,
                                         const int32_t* indices) {
    return guard([&] {
        check_handle(h);
        if (h->ctx->multi()) {
            MML_REQUIRE(num_groups >= 1 && offsets, "bad block arguments");
            MML_REQUIRE(multi_dsgd(h), "set_blocks on a multi-device context needs the DSGD "
                                       "schedule");
            MML_REQUIRE(h->has_data, "set_data must precede set_blocks");
            ring_all(h, [&](int32_t d) {
                return mml_bmf_set_blocks(h->shards[d], num_groups, offsets, indices);
            });
            h->G = num_groups;
            return;
        }
        MML_REQUIRE(h->has_data, "set_data must precede set_blocks");
        MML_REQUIRE(num_groups >= 1 && offsets, "bad block arguments");
        if (ring_mode(h)) return ring_set_blocks(h, num_groups, offsets, indices);
        const int64_t nb = (int64_t)num_groups * num_groups;
        MML_REQUIRE(offsets[0] == 0, "offsets[0] must be 0");
        for (int64_t b = 0; b < nb; ++b)
            MML_REQUIRE(offsets[b + 1] >= offsets[b], "offsets must be non-decreasing");
        const int64_t total = offsets[nb];
        MML_REQUIRE(total <= h->n && (total == 0 || indices), "block indices exceed ratings");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        mml::DeviceArray<int32_t> ord;
        ord.alloc(total);
        if (total > 0)
            MML_HIP(hipMemcpyAsync(ord.get(), indices, sizeof(int32_t) * total,
                                   hipMemcpyHostToDevice, st));
        MML_HIP(hipMemsetAsync(h->scratch_i32.get(), 0, sizeof(int32_t), st));
        if (total > 0) {
            check_order_kernel<<<grid_for(total), 256, 0, st>>>(ord.get(), total, h->n,
                                                                h->scratch_i32.get());
            MML_HIP(hipGetLastError());
        }
        int32_t bad = 0;
        MML_HIP(hipMemcpyAsync(&bad, h->scratch_i32.get(), sizeof(int32_t), hipMemcpyDeviceToHost,
                               st));
        MML_HIP(hipStreamSynchronize(st));
        MML_REQUIRE(!bad, "block index out of range");
        if (total > 0) {
            gather_stream_kernel<<<grid_for(total), 256, 0, st>>>(
                h->raw_u.get(), h->raw_i.get(), h->raw_r.get(), ord.get(), total, h->su.get(),
                h->si.get(), h->sr.get());
            MML_HIP(hipGetLastError());
        }
        h->block_off.alloc(nb + 1);
        MML_HIP(hipMemcpyAsync(h->block_off.get(), offsets, sizeof(int64_t) * (nb + 1),
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipStreamSynchronize(st));
        h->G = num_groups;
    });
}

extern "C" mml_status mml_bmf_set_model(mml_bmf* h, const float* U, const float* V,
                                        const float* bu, const float* bi, float global_bias,
                                        float min_rating, float max_rating) {
    return guard([&] {
        check_handle(h);
        if (h->ctx->multi()) {
            mml::on_devices(h->ctx, [&](int32_t d) {
                return mml_bmf_set_model(h->shards[d], U, V, bu, bi, global_bias, min_rating,
                                         max_rating);
            });
            h->has_model = true;
            return;
        }
        MML_REQUIRE((h->n_users == 0 || (U && bu)) && (h->n_items == 0 || (V && bi)),
                    "null model arrays");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        upload_padded(h, h->U.get(), U, h->n_users);
        upload_padded(h, h->V.get(), V, h->n_items);
        if (h->n_users)
            MML_HIP(hipMemcpyAsync(h->bu.get(), bu, sizeof(float) * h->n_users,
                                   hipMemcpyHostToDevice, st));
        if (h->n_items)
            MML_HIP(hipMemcpyAsync(h->bi.get(), bi, sizeof(float) * h->n_items,
                                   hipMemcpyHostToDevice, st));
        MML_HIP(hipStreamSynchronize(st));
        h->gb = global_bias;
        h->min_rating = min_rating;
        h->max_rating = max_rating;
        h->has_model = true;
        std::fill(h->hold.begin(), h->hold.end(), -1);  // a ring rank: every rank has every row
        h->ring_synced = true;
    });
}

namespace {
// InitModel on the device: N(mean, stddev) in the first k columns of each row (padding 0), rows
// with no training rating zero (MatrixFactorization.cs:108-113)
__global__ __launch_bounds__(256) void bmf_init_normal_kernel(float* __restrict__ M, int64_t rows,
                                                              int32_t k, int32_t ld, uint64_t seed,
                                                              double mean, double stddev,
                                                              const int32_t* __restrict__ cnt) {
    const int64_t total = rows * ld;
    for (int64_t e = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; e < total;
         e += (int64_t)gridDim.x * blockDim.x) {
        const int64_t r = e / ld;
        const int32_t c = (int32_t)(e - r * ld);
        M[e] = c < k && cnt[r] > 0
                   ? (float)(mean + stddev * mml::counter_normal(seed, (uint64_t)(r * k + c)))
                   : 0.0f;
    }
}
}  // namespace

extern "C" mml_status mml_bmf_init_model(mml_bmf* h, uint64_t seed, double mean, double stddev,
                                         float global_bias, float min_rating, float max_rating) {
    return guard([&] {
        check_handle(h);
        if (h->ctx->multi()) {  // same seed on every device: one item side, users by range
            MML_REQUIRE(h->has_data, "set_data must precede init_model");
            MML_REQUIRE(!multi_dsgd(h) || h->G > 0, "set_blocks must precede init_model");
            mml::on_devices(h->ctx, [&](int32_t d) {
                return mml_bmf_init_model(h->shards[d], seed, mean, stddev, global_bias,
                                          min_rating, max_rating);
            });
            h->has_model = true;
            return;
        }
        MML_REQUIRE(h->has_data, "set_data must precede init_model (rows without ratings stay 0)");
        MML_REQUIRE(h->p.model <= MML_MF_PLAIN, "device init covers MML_MF_BIASED / MML_MF_PLAIN");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        if (h->n_users > 0)
            bmf_init_normal_kernel<<<8192, 256, 0, st>>>(h->U.get(), h->n_users, h->k, h->ld, seed,
                                                         mean, stddev, h->cnt_u.get());
        if (h->n_items > 0)
            bmf_init_normal_kernel<<<8192, 256, 0, st>>>(h->V.get(), h->n_items, h->k, h->ld,
                                                         seed ^ 0x5DEECE66Dull, mean, stddev,
                                                         h->cnt_i.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemsetAsync(h->bu.get(), 0, sizeof(float) * h->n_users, st));
        MML_HIP(hipMemsetAsync(h->bi.get(), 0, sizeof(float) * h->n_items, st));
        MML_HIP(hipStreamSynchronize(st));
        h->gb = global_bias;
        h->min_rating = min_rating;
        h->max_rating = max_rating;
        h->has_model = true;
        std::fill(h->hold.begin(), h->hold.end(), -1);
        h->ring_synced = true;
    });
}

extern "C" mml_status mml_bmf_get_model(mml_bmf* h, float* U, float* V, float* bu, float* bi) {
    return guard([&] {
        check_handle(h);
        if (h->ctx->multi()) {
            MML_REQUIRE(h->has_model, "no model");
            if (multi_dsgd(h)) {  // every rank synced (a collective), rank 0 downloads
                ring_all(h, [&](int32_t d) {
                    return d == 0 ? mml_bmf_get_model(h->shards[0], U, V, bu, bi)
                                  : mml_bmf_get_model(h->shards[d], nullptr, nullptr, nullptr,
                                                      nullptr);
                });
                return;
            }
            return multi_get_model(h, U, V, bu, bi);
        }
        MML_REQUIRE(h->has_model, "no model (set_model first)");
        if (ring_mode(h)) ring_sync(h);
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        if (U) download_padded(h, U, h->U.get(), h->n_users);
        if (V) download_padded(h, V, h->V.get(), h->n_items);
        if (bu && h->n_users)
            MML_HIP(hipMemcpyAsync(bu, h->bu.get(), sizeof(float) * h->n_users,
                                   hipMemcpyDeviceToHost, st));
        if (bi && h->n_items)
            MML_HIP(hipMemcpyAsync(bi, h->bi.get(), sizeof(float) * h->n_items,
                                   hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bmf_iterate(mml_bmf* h, float learn_rate,
                                      const int32_t* subepoch_sequence) {
    return guard([&] {
        check_handle(h);
        if (h->ctx->multi() && multi_dsgd(h)) {  // the ranks' epochs, one host thread each
            MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede iterate");
            MML_REQUIRE(h->G > 0, "DSGD schedule needs set_blocks");
            std::vector<float> ms(h->shards.size(), 0.0f);
            ring_all(h, [&](int32_t d) {
                const mml_status st = mml_bmf_iterate(h->shards[d], learn_rate, subepoch_sequence);
                ms[d] = h->shards[d]->last_ms;
                return st;
            });
            h->last_ms = *std::max_element(ms.begin(), ms.end());
            h->last_launches = h->shards[0]->last_launches * (int32_t)h->shards.size();
            return;
        }
        if (h->ctx->multi()) {  // every shard's epoch, then the item average
            MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede iterate");
            multi_epoch(h, learn_rate);
            return;
        }
        MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede iterate");
        h->last_kernel.clear();  // set again by the launch that runs (Hogwild / ordered / DSGD)
        const bool asym = is_asym(h);
        if (asym) {
            MML_REQUIRE(asym_ready(h), "set_implicit_feedback (each side the model uses) must "
                                       "precede iterate");
            MML_REQUIRE(h->p.schedule == MML_SCHEDULE_ORDERED ||
                            h->p.schedule == MML_SCHEDULE_HOGWILD,
                        "the asymmetric models run the ORDERED or HOGWILD schedule");
        }
        if (h->p.schedule == MML_SCHEDULE_DSGD && h->p.model != MML_MF_SOCIAL && !asym) {
            MML_REQUIRE(h->G > 0, "DSGD schedule needs set_blocks");
            MML_REQUIRE(subepoch_sequence, "DSGD schedule needs a sub-epoch sequence");
            for (int32_t x = 0; x < h->G; ++x)
                MML_REQUIRE(subepoch_sequence[x] >= 0 && subepoch_sequence[x] < h->G,
                            "sub-epoch index out of range");
        }
        if (ring_mode(h)) {  // one rank of the DSGD ring
            if (h->n == 0) return;
            switch (h->p.model == MML_MF_PLAIN ? kPlainMF : h->p.loss) {
                case kPlainMF: ring_epoch<kPlainMF>(h, learn_rate, subepoch_sequence); break;
                case MML_LOSS_MAE: ring_epoch<MML_LOSS_MAE>(h, learn_rate, subepoch_sequence); break;
                case MML_LOSS_LOGISTIC:
                    ring_epoch<MML_LOSS_LOGISTIC>(h, learn_rate, subepoch_sequence);
                    break;
                default: ring_epoch<MML_LOSS_RMSE>(h, learn_rate, subepoch_sequence); break;
            }
            return;
        }
        h->ctx->activate();
        BmfScalars s;
        s.gb = h->gb;
        s.min_rating = h->min_rating;
        s.range = h->max_rating - h->min_rating;
        s.lr = learn_rate;
        s.blr = h->p.bias_learn_rate * learn_rate;
        s.bias_reg = h->p.bias_reg;
        s.reg_u = h->p.reg_u;
        s.reg_i = h->p.reg_i;
        hipStream_t st = h->ctx->stream;
        MML_HIP(hipEventRecord(h->ctx->ev_begin, st));
        if (asym) {
            switch (h->p.loss) {
                case MML_LOSS_MAE: asym_epoch<MML_LOSS_MAE>(h, s); break;
                case MML_LOSS_LOGISTIC: asym_epoch<MML_LOSS_LOGISTIC>(h, s); break;
                default: asym_epoch<MML_LOSS_RMSE>(h, s); break;
            }
        } else if (h->p.model == MML_MF_SOCIAL) {
            switch (h->p.loss) {
                case MML_LOSS_MAE: social_epoch<MML_LOSS_MAE>(h, s); break;
                case MML_LOSS_LOGISTIC: social_epoch<MML_LOSS_LOGISTIC>(h, s); break;
                default: social_epoch<MML_LOSS_RMSE>(h, s); break;
            }
        } else switch (h->p.model == MML_MF_PLAIN ? kPlainMF : h->p.loss) {
            case kPlainMF: run_epoch<kPlainMF>(h, s, subepoch_sequence); break;
            case MML_LOSS_MAE: run_epoch<MML_LOSS_MAE>(h, s, subepoch_sequence); break;
            case MML_LOSS_LOGISTIC: run_epoch<MML_LOSS_LOGISTIC>(h, s, subepoch_sequence); break;
            default: run_epoch<MML_LOSS_RMSE>(h, s, subepoch_sequence); break;
        }
        MML_HIP(hipEventRecord(h->ctx->ev_end, st));
        MML_HIP(hipEventSynchronize(h->ctx->ev_end));
        MML_HIP(hipEventElapsedTime(&h->last_ms, h->ctx->ev_begin, h->ctx->ev_end));
    });
}

extern "C" mml_status mml_bmf_last_kernel(mml_bmf* h, char* buf, int32_t cap) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(buf && cap > 0, "null buffer");
        const std::string& k = h->shards.empty() ? h->last_kernel : h->shards[0]->last_kernel;
        const size_t n = std::min<size_t>(k.size(), (size_t)cap - 1);
        std::copy(k.begin(), k.begin() + n, buf);
        buf[n] = 0;
    });
}

extern "C" mml_status mml_bmf_set_hogwild_phases(mml_bmf* h, int32_t phases) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(phases >= 0 && phases <= 32, "phases must be in [0, 32]");
        h->phases_req = phases;
        for (mml_bmf* s : h->shards) s->phases_req = phases;
    });
}

extern "C" mml_status mml_bmf_set_hogwild_runs(mml_bmf* h, int32_t on) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(on >= -1 && on <= 1, "on must be -1 (default), 0 or 1");
        h->runs_req = on;
        for (mml_bmf* s : h->shards) s->runs_req = on;
    });
}

extern "C" mml_status mml_bmf_last_runs(mml_bmf* h, int64_t* out) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(out, "out is null");
        const mml_bmf* s = h->shards.empty() ? h : h->shards[0];
        *out = s->last_runs ? s->n_runs : 0;
    });
}

extern "C" mml_status mml_bmf_last_phases(mml_bmf* h, int32_t* out) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(out, "out is null");
        *out = h->shards.empty() ? h->n_phases : h->shards[0]->n_phases;
    });
}

extern "C" mml_status mml_bmf_hogwild_stream(mml_bmf* h, int32_t* users, int32_t* items,
                                             float* values, int64_t n, int64_t* span_offsets,
                                             int32_t cap_offsets, int32_t* n_spans) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(users && items && values && span_offsets && n_spans, "null output");
        MML_REQUIRE(h->has_data && n == h->n, "n must equal the handle's rating count");
        MML_REQUIRE(h->has_xstream,
                    "no XCD-grouped stream: run a HOGWILD epoch on an 8-XCD device first");
        const bool runs = h->last_runs && h->has_runs;  // the user-runs strata (8 launches)
        const int32_t spans = runs ? 64 : h->n_phases * 8;
        MML_REQUIRE(cap_offsets >= spans + 1, "span_offsets holds fewer than phases * 8 + 1");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        if (runs) {
            // launch-major, group-minor: the strata in the order the 8 launches walk them
            int64_t at = 0;
            for (int x = 0; x < 64; ++x) {
                const int64_t b = h->run_spans[2 * x], e = h->run_spans[2 * x + 1];
                span_offsets[x] = at;
                if (e > b) {
                    MML_HIP(hipMemcpyAsync(users + at, h->rxu.get() + b, sizeof(int32_t) * (e - b),
                                           hipMemcpyDeviceToHost, st));
                    MML_HIP(hipMemcpyAsync(items + at, h->rxi.get() + b, sizeof(int32_t) * (e - b),
                                           hipMemcpyDeviceToHost, st));
                    MML_HIP(hipMemcpyAsync(values + at, h->rxr.get() + b, sizeof(float) * (e - b),
                                           hipMemcpyDeviceToHost, st));
                }
                at += e - b;
            }
            span_offsets[64] = at;
            MML_HIP(hipStreamSynchronize(st));
            MML_REQUIRE(at == n, "the strata do not cover the stream");
            *n_spans = spans;
            return;
        }
        if (n > 0) {
            MML_HIP(hipMemcpyAsync(users, h->xu.get(), sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
            MML_HIP(hipMemcpyAsync(items, h->xi.get(), sizeof(int32_t) * n, hipMemcpyDeviceToHost, st));
            MML_HIP(hipMemcpyAsync(values, h->xr.get(), sizeof(float) * n, hipMemcpyDeviceToHost, st));
        }
        const int64_t* off = h->n_phases > 1 ? h->poff.get() : h->xs.goff.get();
        MML_HIP(hipMemcpyAsync(span_offsets, off, sizeof(int64_t) * (spans + 1),
                               hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        *n_spans = spans;
    });
}

extern "C" mml_status mml_bmf_replay_traffic(mml_bmf* h, float* out_ms) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(out_ms, "out is null");
        MML_REQUIRE(h->has_data && h->has_model, "set_data and set_model must precede the replay");
        MML_REQUIRE(h->p.model <= MML_MF_PLAIN && !is_asym(h) &&
                        (h->p.schedule == MML_SCHEDULE_HOGWILD ||
                         h->p.schedule == MML_SCHEDULE_HOGWILD_COHERENT),
                    "the traffic replay covers the BiasedMF / MF Hogwild epoch");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        BmfScalars sc{};
        const std::string label = h->last_kernel;
        MML_HIP(hipEventRecord(h->ctx->ev_begin, st));
        if (h->n > 0) launch_hogwild<kReplayTraffic>(h, sc, nullptr, nullptr);
        MML_HIP(hipEventRecord(h->ctx->ev_end, st));
        MML_HIP(hipEventSynchronize(h->ctx->ev_end));
        MML_HIP(hipEventElapsedTime(out_ms, h->ctx->ev_begin, h->ctx->ev_end));
        h->last_kernel = label;
    });
}

extern "C" mml_status mml_bmf_last_timing(mml_bmf* h, float* out) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(out, "out is null");
        out[0] = h->last_ms;
        out[1] = (float)h->last_launches;
    });
}

namespace {
void upload_pairs(mml_bmf* h, const int32_t* users, const int32_t* items, int64_t n) {
    hipStream_t st = h->ctx->stream;
    h->ev_u.alloc(n);
    h->ev_i.alloc(n);
    MML_HIP(hipMemcpyAsync(h->ev_u.get(), users, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
    MML_HIP(hipMemcpyAsync(h->ev_i.get(), items, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
}
}  // namespace

extern "C" mml_status mml_bmf_predict(mml_bmf* h, const int32_t* users, const int32_t* items,
                                      int64_t n, float* out) {
    return guard([&] {
        check_handle(h);
        if (h->ctx->multi()) {
            MML_REQUIRE(n >= 0 && (n == 0 || (users && items && out)), "null arrays");
            MML_REQUIRE(h->has_model, "no model");
            if (multi_dsgd(h)) {
                multi_ring_sync(h);
                const mml_status st = mml_bmf_predict(h->shards[0], users, items, n, out);
                if (st != MML_OK) mml::fail(st, mml_last_error());
                return;
            }
            return multi_predict(h, users, items, n, out);
        }
        MML_REQUIRE(h->has_model, "no model");
        // a collective on a ring rank: every rank syncs before the per-rank argument checks, so a
        // rank with an empty or bad slice cannot leave the others waiting in the broadcasts
        if (ring_mode(h)) ring_sync(h);
        MML_REQUIRE(n >= 0 && (n == 0 || (users && items && out)), "bad arguments");
        if (n == 0) return;
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        upload_pairs(h, users, items, n);
        h->ev_out.alloc(n);
        bmf_predict_kernel<<<grid_for(n), 256, 0, st>>>(
            h->ev_u.get(), h->ev_i.get(), n, h->n_users, h->n_items, h->U.get(), h->V.get(),
            h->bu.get(), h->bi.get(), h->k, h->ld, h->gb, h->min_rating, h->max_rating,
            predict_kind(h), h->ev_out.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemcpyAsync(out, h->ev_out.get(), sizeof(float) * n, hipMemcpyDeviceToHost,
                               st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bmf_evaluate(mml_bmf* h, const int32_t* users, const int32_t* items,
                                       const float* values, int64_t n, float* out) {
    return guard([&] {
        check_handle(h);
        if (h->ctx->multi()) {
            MML_REQUIRE(n >= 0 && (n == 0 || (users && items && values)) && out, "null arrays");
            MML_REQUIRE(h->has_model, "no model");
            if (multi_dsgd(h)) {
                multi_ring_sync(h);
                const mml_status st = mml_bmf_evaluate(h->shards[0], users, items, values, n, out);
                if (st != MML_OK) mml::fail(st, mml_last_error());
                return;
            }
            return multi_evaluate(h, users, items, values, n, out);
        }
        MML_REQUIRE(h->has_model, "no model");
        if (ring_mode(h)) ring_sync(h);  // a collective: every rank syncs before its own checks
        MML_REQUIRE(n > 0 && users && items && values && out, "bad arguments");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        upload_pairs(h, users, items, n);
        h->ev_r.alloc(n);
        MML_HIP(hipMemcpyAsync(h->ev_r.get(), values, sizeof(float) * n, hipMemcpyHostToDevice,
                               st));
        const int grid = grid_for(n, 256, 1024);
        h->ev_partials.alloc(2 * grid);
        bmf_eval_kernel<<<grid, 256, 0, st>>>(h->ev_u.get(), h->ev_i.get(), h->ev_r.get(), n,
                                              h->n_users, h->n_items, h->U.get(), h->V.get(),
                                              h->bu.get(), h->bi.get(), h->k, h->ld, h->gb,
                                              h->min_rating, h->max_rating,
                                              predict_kind(h),
                                              h->ev_partials.get());
        MML_HIP(hipGetLastError());
        std::vector<double> part(2 * grid);
        MML_HIP(hipMemcpyAsync(part.data(), h->ev_partials.get(), sizeof(double) * 2 * grid,
                               hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        double se = 0.0, ae = 0.0;
        for (int b = 0; b < grid; ++b) {
            se += part[2 * b];
            ae += part[2 * b + 1];
        }
        out[0] = (float)std::sqrt(se / (double)n);
        out[1] = (float)(ae / (double)n);
    });
}

extern "C" mml_status mml_bmf_objective(mml_bmf* h, double* out) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(h->has_model && h->has_data && out, "model, data and out required");
        MML_REQUIRE(h->p.model == MML_MF_BIASED,
                    "ComputeObjective is defined for BiasedMatrixFactorization only");
        // a ring rank (a collective): the newest model on every rank, and the loss over all n
        // ratings in set_data order -- su holds only this rank's block rows
        const bool ring = ring_mode(h);
        if (ring) ring_sync(h);
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        const int g1 = grid_for(h->n, 256, 1024);
        const int g2 = grid_for((int64_t)h->n_users + h->n_items, 4, 1024);
        h->ev_partials.alloc(g1 + g2);
        bmf_loss_kernel<<<g1, 256, 0, st>>>(ring ? h->raw_u.get() : h->su.get(),
                                            ring ? h->raw_i.get() : h->si.get(),
                                            ring ? h->raw_r.get() : h->sr.get(), h->n,
                                            h->n_users, h->n_items, h->U.get(), h->V.get(),
                                            h->bu.get(), h->bi.get(), h->k, h->ld, h->gb,
                                            h->min_rating, h->max_rating, h->p.loss,
                                            h->ev_partials.get());
        bmf_complexity_kernel<<<g2, 256, 0, st>>>(
            h->U.get(), h->V.get(), h->bu.get(), h->bi.get(), h->cnt_u.get(), h->cnt_i.get(),
            h->n_users, h->n_items, h->k, h->ld, h->p.reg_u, h->p.reg_i, h->p.bias_reg,
            h->p.frequency_regularization, h->ev_partials.get() + g1);
        MML_HIP(hipGetLastError());
        std::vector<double> part(g1 + g2);
        MML_HIP(hipMemcpyAsync(part.data(), h->ev_partials.get(), sizeof(double) * part.size(),
                               hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        double loss = 0.0, cx = 0.0;
        for (int b = 0; b < g1; ++b) loss += part[b];
        for (int b = 0; b < g2; ++b) cx += part[g1 + b];
        out[0] = loss;
        out[1] = cx;
    });
}

extern "C" mml_status mml_bmf_allreduce_items(mml_bmf* h) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        no_ring(h, "allreduce_items");
        MML_REQUIRE(h->has_model, "no model");
        mml_ctx* c = h->ctx;
        if (c->nranks <= 1 && !c->comm) return;  // no communicator: nothing to average
        MML_REQUIRE(c->comm, "context has no communicator (mml_ctx_comm_init)");
        MML_REQUIRE(!is_asym(h), "the asymmetric models' implicit factors are not averaged across ranks");
        c->activate();
        hipStream_t st = c->stream;
        if (!h->ev_ar0) {
            MML_HIP(hipEventCreate(&h->ev_ar0));
            MML_HIP(hipEventCreate(&h->ev_ar1));
        }
        // model averaging inside the collective (ncclAvg); stream-ordered, no host wait: the next
        // epoch's kernel and every download run on this stream after it
        const size_t nv = (size_t)h->n_items * h->ld;
        MML_HIP(hipEventRecord(h->ev_ar0, st));
        MML_RCCL(ncclGroupStart());
        MML_RCCL(ncclAllReduce(h->V.get(), h->V.get(), nv, ncclFloat, ncclAvg, c->comm, st));
        MML_RCCL(ncclAllReduce(h->bi.get(), h->bi.get(), (size_t)h->n_items, ncclFloat, ncclAvg,
                               c->comm, st));
        MML_RCCL(ncclGroupEnd());
        MML_HIP(hipEventRecord(h->ev_ar1, st));
        h->has_ar = true;
    });
}

extern "C" mml_status mml_bmf_last_allreduce_ms(mml_bmf* h, float* out) {
    return guard([&] {
        check_handle(h);
        MML_REQUIRE(out, "out is null");
        *out = 0.0f;
        auto one = [](mml_bmf* x) {
            if (!x->has_ar) return 0.0f;
            x->ctx->activate();
            float ms = 0.0f;
            MML_HIP(hipEventSynchronize(x->ev_ar1));
            MML_HIP(hipEventElapsedTime(&ms, x->ev_ar0, x->ev_ar1));
            return ms;
        };
        if (h->ctx->multi()) {
            if (h->has_ar) {  // the peer average, on shard 0's device
                mml_bmf* s0 = h->shards[0];
                s0->ctx->activate();
                MML_HIP(hipEventSynchronize(h->ev_ar1));
                MML_HIP(hipEventElapsedTime(out, h->ev_ar0, h->ev_ar1));
                return;
            }
            for (mml_bmf* s : h->shards) *out = std::max(*out, one(s));
            return;
        }
        *out = one(h);
    });
}

namespace {
template <int LOSS>
void launch_fold_in(mml_bmf* h, int32_t n_fold, const int64_t* off, const int32_t* items,
                    const float* values, int32_t num_iter, const FoldScalars& fs,
                    const float* init, float* out) {
    hipStream_t st = h->ctx->stream;
    const int km = (h->k + 63) / 64;
#define MML_FOLD(KM)                                                                            \
    bmf_fold_in_kernel<LOSS, KM><<<n_fold, 64, 0, st>>>(off, items, values, num_iter, h->V.get(), \
                                                        h->bi.get(), h->k, h->ld, fs, init, out)
    switch (km) {
        case 1: MML_FOLD(1); break;
        case 2: MML_FOLD(2); break;
        case 3: MML_FOLD(3); break;
        default: MML_FOLD(4); break;
    }
#undef MML_FOLD
    MML_HIP(hipGetLastError());
}
}  // namespace

extern "C" mml_status mml_bmf_fold_in(mml_bmf* h, int32_t n_fold, const int64_t* rated_off,
                                      const int32_t* rated_items, const float* rated_values,
                                      const float* init_factors, int32_t num_iter,
                                      float learn_rate, float decay, float* out_vectors) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        no_ring(h, "fold_in");
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(!is_asym(h), "the asymmetric models have their own FoldIn (not on the GPU path)");
        MML_REQUIRE(n_fold >= 0 && num_iter >= 0, "negative sizes");
        if (n_fold == 0) return;
        MML_REQUIRE(rated_off && init_factors && out_vectors, "null arguments");
        MML_REQUIRE(rated_off[0] == 0, "rated_off[0] must be 0");
        for (int32_t x = 0; x < n_fold; ++x)
            MML_REQUIRE(rated_off[x + 1] >= rated_off[x], "rated_off must be non-decreasing");
        const int64_t nr = rated_off[n_fold];
        MML_REQUIRE(nr == 0 || (rated_items && rated_values), "null rated arrays");
        for (int64_t x = 0; x < nr; ++x)
            MML_REQUIRE(rated_items[x] >= 0 && rated_items[x] < h->n_items,
                        "fold-in item id beyond the model");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        const bool plain = h->p.model == MML_MF_PLAIN;
        const int64_t w = plain ? h->k : h->k + 1;
        mml::DeviceArray<int64_t> doff;
        mml::DeviceArray<int32_t> ditems;
        mml::DeviceArray<float> dvals, dinit, dout;
        doff.alloc(n_fold + 1);
        ditems.alloc(std::max<int64_t>(1, nr));
        dvals.alloc(std::max<int64_t>(1, nr));
        dinit.alloc((size_t)n_fold * h->k);
        dout.alloc((size_t)n_fold * w);
        MML_HIP(hipMemcpyAsync(doff.get(), rated_off, sizeof(int64_t) * (n_fold + 1),
                               hipMemcpyHostToDevice, st));
        if (nr > 0) {
            MML_HIP(hipMemcpyAsync(ditems.get(), rated_items, sizeof(int32_t) * nr,
                                   hipMemcpyHostToDevice, st));
            MML_HIP(hipMemcpyAsync(dvals.get(), rated_values, sizeof(float) * nr,
                                   hipMemcpyHostToDevice, st));
        }
        MML_HIP(hipMemcpyAsync(dinit.get(), init_factors, sizeof(float) * n_fold * h->k,
                               hipMemcpyHostToDevice, st));
        FoldScalars fs;
        fs.gb = h->gb;
        fs.min_rating = h->min_rating;
        fs.range = h->max_rating - h->min_rating;
        fs.lr = learn_rate;
        fs.blr = h->p.bias_learn_rate * learn_rate;
        fs.bias_reg = h->p.bias_reg;
        fs.reg_u = h->p.reg_u;
        fs.decay = decay;
        fs.freq = h->p.frequency_regularization;
#define MML_FOLD_ARGS h, n_fold, doff.get(), ditems.get(), dvals.get(), num_iter, fs, dinit.get(), \
                      dout.get()
        switch (plain ? kPlainMF : h->p.loss) {
            case kPlainMF: launch_fold_in<kPlainMF>(MML_FOLD_ARGS); break;
            case MML_LOSS_MAE: launch_fold_in<MML_LOSS_MAE>(MML_FOLD_ARGS); break;
            case MML_LOSS_LOGISTIC: launch_fold_in<MML_LOSS_LOGISTIC>(MML_FOLD_ARGS); break;
            default: launch_fold_in<MML_LOSS_RMSE>(MML_FOLD_ARGS); break;
        }
#undef MML_FOLD_ARGS
        MML_HIP(hipMemcpyAsync(out_vectors, dout.get(), sizeof(float) * n_fold * w,
                               hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

namespace {
template <int LOSS, int SIDE>
void launch_retrain(mml_bmf* h, int32_t n, const int32_t* rows, const int64_t* off,
                    const int32_t* other, const float* values, const float* init, const float* lrs,
                    int32_t num_iter, const BmfScalars& s) {
    hipStream_t st = h->ctx->stream;
#define MML_RT(KM)                                                                              \
    bmf_retrain_kernel<LOSS, KM, SIDE><<<n, 64, 0, st>>>(                                       \
        rows, off, other, values, init, lrs, num_iter, h->U.get(), h->V.get(), h->bu.get(),     \
        h->bi.get(), h->k, h->ld, s, h->p.bias_learn_rate, h->p.frequency_regularization)
    switch ((h->k + 63) / 64) {
        case 1: MML_RT(1); break;
        case 2: MML_RT(2); break;
        case 3: MML_RT(3); break;
        default: MML_RT(4); break;
    }
#undef MML_RT
    MML_HIP(hipGetLastError());
}

template <int LOSS>
void launch_retrain_side(mml_bmf* h, int32_t side, int32_t n, const int32_t* rows,
                         const int64_t* off, const int32_t* other, const float* values,
                         const float* init, const float* lrs, int32_t num_iter,
                         const BmfScalars& s) {
    if (side == 0) launch_retrain<LOSS, 0>(h, n, rows, off, other, values, init, lrs, num_iter, s);
    else launch_retrain<LOSS, 1>(h, n, rows, off, other, values, init, lrs, num_iter, s);
}
}  // namespace

extern "C" mml_status mml_bmf_retrain(mml_bmf* h, int32_t side, int32_t n_rows,
                                      const int32_t* rows, const int64_t* rated_off,
                                      const int32_t* rated_ids, const float* rated_values,
                                      const float* init_factors, int32_t num_iter,
                                      const float* learn_rates) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        no_ring(h, "retrain");
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(h->p.model == MML_MF_BIASED || h->p.model == MML_MF_PLAIN,
                    "RetrainUser / RetrainItem on the GPU: BiasedMatrixFactorization and "
                    "MatrixFactorization");
        MML_REQUIRE(side == 0 || side == 1, "side: 0 (users) or 1 (items)");
        MML_REQUIRE(n_rows >= 0 && num_iter >= 0, "negative sizes");
        if (n_rows == 0) return;
        MML_REQUIRE(rows && rated_off && init_factors && (num_iter == 0 || learn_rates),
                    "null arguments");
        const int32_t n_own = side == 0 ? h->n_users : h->n_items;
        const int32_t n_oth = side == 0 ? h->n_items : h->n_users;
        // rows of one side train independently (the other side is fixed), so they run at once;
        // a row listed twice would race with itself: its last retraining alone decides the result
        std::vector<int32_t> sorted(rows, rows + n_rows);
        std::sort(sorted.begin(), sorted.end());
        for (int32_t x = 0; x < n_rows; ++x) {
            MML_REQUIRE(sorted[x] >= 0 && sorted[x] < n_own, "retrained row id beyond the model");
            MML_REQUIRE(x == 0 || sorted[x] != sorted[x - 1], "a row is listed twice");
        }
        MML_REQUIRE(rated_off[0] == 0, "rated_off[0] must be 0");
        for (int32_t x = 0; x < n_rows; ++x)
            MML_REQUIRE(rated_off[x + 1] >= rated_off[x], "rated_off must be non-decreasing");
        const int64_t nr = rated_off[n_rows];
        MML_REQUIRE(nr == 0 || (rated_ids && rated_values), "null rated arrays");
        for (int64_t x = 0; x < nr; ++x)
            MML_REQUIRE(rated_ids[x] >= 0 && rated_ids[x] < n_oth, "rated id beyond the model");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        mml::DeviceArray<int64_t> doff;
        mml::DeviceArray<int32_t> drows, dids;
        mml::DeviceArray<float> dvals, dinit, dlrs;
        doff.alloc(n_rows + 1);
        drows.alloc(n_rows);
        dids.alloc(std::max<int64_t>(1, nr));
        dvals.alloc(std::max<int64_t>(1, nr));
        dinit.alloc((size_t)n_rows * h->k);
        dlrs.alloc(std::max<int64_t>(1, (int64_t)n_rows * num_iter));
        MML_HIP(hipMemcpyAsync(doff.get(), rated_off, sizeof(int64_t) * (n_rows + 1),
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(drows.get(), rows, sizeof(int32_t) * n_rows, hipMemcpyHostToDevice,
                               st));
        if (nr > 0) {
            MML_HIP(hipMemcpyAsync(dids.get(), rated_ids, sizeof(int32_t) * nr,
                                   hipMemcpyHostToDevice, st));
            MML_HIP(hipMemcpyAsync(dvals.get(), rated_values, sizeof(float) * nr,
                                   hipMemcpyHostToDevice, st));
        }
        MML_HIP(hipMemcpyAsync(dinit.get(), init_factors, sizeof(float) * n_rows * h->k,
                               hipMemcpyHostToDevice, st));
        if (num_iter > 0)
            MML_HIP(hipMemcpyAsync(dlrs.get(), learn_rates,
                                   sizeof(float) * (int64_t)n_rows * num_iter,
                                   hipMemcpyHostToDevice, st));
        BmfScalars s;
        s.gb = h->gb;
        s.min_rating = h->min_rating;
        s.range = h->max_rating - h->min_rating;
        s.lr = 0.0f;   // per Iterate call: learn_rates
        s.blr = 0.0f;
        s.bias_reg = h->p.bias_reg;
        s.reg_u = h->p.reg_u;
        s.reg_i = h->p.reg_i;
#define MML_RT_ARGS h, side, n_rows, drows.get(), doff.get(), dids.get(), dvals.get(), dinit.get(), \
                    dlrs.get(), num_iter, s
        switch (h->p.model == MML_MF_PLAIN ? kPlainMF : h->p.loss) {
            case kPlainMF: launch_retrain_side<kPlainMF>(MML_RT_ARGS); break;
            case MML_LOSS_MAE: launch_retrain_side<MML_LOSS_MAE>(MML_RT_ARGS); break;
            case MML_LOSS_LOGISTIC: launch_retrain_side<MML_LOSS_LOGISTIC>(MML_RT_ARGS); break;
            default: launch_retrain_side<MML_LOSS_RMSE>(MML_RT_ARGS); break;
        }
#undef MML_RT_ARGS
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bmf_predict_vectors(mml_bmf* h, int32_t n_vectors, const float* vectors,
                                              const int32_t* vector_index, const int32_t* items,
                                              int64_t n, float* out) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        no_ring(h, "predict_vectors");
        MML_REQUIRE(h->has_model, "no model");
        MML_REQUIRE(!is_asym(h), "the asymmetric models have their own FoldIn (not on the GPU path)");
        MML_REQUIRE(n_vectors >= 0 && n >= 0, "negative sizes");
        if (n == 0) return;
        MML_REQUIRE(vectors && vector_index && items && out, "null arguments");
        const bool plain = h->p.model == MML_MF_PLAIN;
        for (int64_t x = 0; x < n; ++x) {
            MML_REQUIRE(vector_index[x] >= 0 && vector_index[x] < n_vectors,
                        "vector index out of range");
            MML_REQUIRE(items[x] >= 0 && (!plain || items[x] < h->n_items),
                        "item id beyond the model");
        }
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        const int64_t w = plain ? h->k : h->k + 1;
        mml::DeviceArray<float> dvec, dout;
        mml::DeviceArray<int32_t> dvi, dit;
        dvec.alloc((size_t)std::max<int64_t>(1, (int64_t)n_vectors * w));
        dvi.alloc(n);
        dit.alloc(n);
        dout.alloc(n);
        if (n_vectors > 0)
            MML_HIP(hipMemcpyAsync(dvec.get(), vectors, sizeof(float) * n_vectors * w,
                                   hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(dvi.get(), vector_index, sizeof(int32_t) * n,
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(dit.get(), items, sizeof(int32_t) * n, hipMemcpyHostToDevice, st));
        bmf_predict_vectors_kernel<<<grid_for(n), 256, 0, st>>>(
            dvec.get(), dvi.get(), dit.get(), n, h->n_items, h->V.get(), h->bi.get(), h->k, h->ld,
            h->gb, h->min_rating, h->max_rating, (int32_t)plain, dout.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemcpyAsync(out, dout.get(), sizeof(float) * n, hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bmf_set_user_relation(mml_bmf* h, int32_t n_rows, const int64_t* offsets,
                                                const int32_t* cols) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(h->p.model == MML_MF_SOCIAL, "the user relation belongs to SocialMF handles");
        MML_REQUIRE(n_rows >= 0 && n_rows <= h->n_users, "relation rows beyond the users");
        MML_REQUIRE(n_rows == 0 || offsets, "null offsets");
        const int64_t nnz = n_rows ? offsets[n_rows] : 0;
        MML_REQUIRE(n_rows == 0 || offsets[0] == 0, "offsets[0] must be 0");
        for (int32_t r = 0; r < n_rows; ++r)
            MML_REQUIRE(offsets[r + 1] >= offsets[r], "offsets must be non-decreasing");
        MML_REQUIRE(nnz == 0 || cols, "null cols");
        int32_t n_rev = 0;
        for (int64_t x = 0; x < nnz; ++x) {
            MML_REQUIRE(cols[x] >= 0 && cols[x] < h->n_users, "relation id beyond the users");
            n_rev = std::max(n_rev, cols[x] + 1);
        }
        // Transpose() (SparseBooleanMatrix.cs:200-207): rows filled by ascending source row
        std::vector<int64_t> roff((size_t)n_rev + 1, 0);
        for (int64_t x = 0; x < nnz; ++x) ++roff[(size_t)cols[x] + 1];
        for (int32_t r = 0; r < n_rev; ++r) roff[r + 1] += roff[r];
        std::vector<int32_t> rcols((size_t)std::max<int64_t>(1, nnz));
        std::vector<int64_t> fill(roff.begin(), roff.end() - 1);
        for (int32_t r = 0; r < n_rows; ++r)
            for (int64_t x = offsets[r]; x < offsets[r + 1]; ++x) rcols[fill[cols[x]]++] = r;
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->conn_off.alloc((size_t)n_rows + 1);
        h->conn_cols.alloc((size_t)std::max<int64_t>(1, nnz));
        h->rev_off.alloc((size_t)n_rev + 1);
        h->rev_cols.alloc((size_t)std::max<int64_t>(1, nnz));
        if (n_rows)
            MML_HIP(hipMemcpyAsync(h->conn_off.get(), offsets, sizeof(int64_t) * (n_rows + 1),
                                   hipMemcpyHostToDevice, st));
        if (nnz) {
            MML_HIP(hipMemcpyAsync(h->conn_cols.get(), cols, sizeof(int32_t) * nnz,
                                   hipMemcpyHostToDevice, st));
            MML_HIP(hipMemcpyAsync(h->rev_cols.get(), rcols.data(), sizeof(int32_t) * nnz,
                                   hipMemcpyHostToDevice, st));
        }
        MML_HIP(hipMemcpyAsync(h->rev_off.get(), roff.data(), sizeof(int64_t) * (n_rev + 1),
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipStreamSynchronize(st));
        h->n_conn = n_rows;
        h->n_rev = n_rev;
    });
}

extern "C" mml_status mml_bmf_set_implicit_feedback(mml_bmf* h, int32_t side, int32_t n_rows,
                                                    const int64_t* offsets, const int32_t* ids,
                                                    const float* factors, const float* reg) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(is_asym(h), "implicit feedback belongs to the asymmetric models' handles");
        MML_REQUIRE(side == 0 || side == 1, "side must be 0 (lists per user) or 1 (per item)");
        MML_REQUIRE(uses_side(h, side), "this model does not use that side");
        // side 0: a list of items per user, factors y [n_items x k]; side 1: a list of users per
        // item, factors x [n_users x k]
        const int32_t n_list = side == 0 ? h->n_users : h->n_items;
        const int32_t n_x = side == 0 ? h->n_items : h->n_users;
        MML_REQUIRE(n_rows == n_list, "one list per user (side 0) / per item (side 1)");
        MML_REQUIRE(offsets && factors && reg, "null argument");
        MML_REQUIRE(offsets[0] == 0, "offsets[0] must be 0");
        for (int32_t r = 0; r < n_rows; ++r)
            MML_REQUIRE(offsets[r + 1] >= offsets[r], "offsets must not decrease");
        const int64_t nnz = offsets[n_rows];
        MML_REQUIRE(nnz == 0 || ids, "null ids");
        for (int64_t x = 0; x < nnz; ++x)
            MML_REQUIRE(ids[x] >= 0 && ids[x] < n_x, "list id out of range");
        h->ctx->activate();
        hipStream_t st = h->ctx->stream;
        h->has_slot[side] = false;
        h->asym_off[side].alloc((size_t)n_rows + 1);
        h->asym_ids[side].alloc((size_t)std::max<int64_t>(1, nnz));
        h->asym_x[side].alloc((size_t)std::max<int64_t>(1, (int64_t)n_x * h->ld));
        h->asym_reg[side].alloc((size_t)std::max(1, n_x));
        MML_HIP(hipMemcpyAsync(h->asym_off[side].get(), offsets, sizeof(int64_t) * (n_rows + 1),
                               hipMemcpyHostToDevice, st));
        if (nnz)
            MML_HIP(hipMemcpyAsync(h->asym_ids[side].get(), ids, sizeof(int32_t) * nnz,
                                   hipMemcpyHostToDevice, st));
        upload_padded(h, h->asym_x[side].get(), factors, n_x);
        if (n_x)
            MML_HIP(hipMemcpyAsync(h->asym_reg[side].get(), reg, sizeof(float) * n_x,
                                   hipMemcpyHostToDevice, st));
        h->has_slot[side] = true;
        if (asym_ready(h)) asym_precompute(h);
        MML_HIP(hipStreamSynchronize(st));
    });
}

extern "C" mml_status mml_bmf_get_implicit_factors(mml_bmf* h, int32_t side, float* factors) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(side == 0 || side == 1, "side must be 0 or 1");
        MML_REQUIRE(h->has_slot[side], "no implicit factors on that side");
        MML_REQUIRE(factors, "null argument");
        h->ctx->activate();
        download_padded(h, factors, h->asym_x[side].get(), side == 0 ? h->n_items : h->n_users);
        MML_HIP(hipStreamSynchronize(h->ctx->stream));
    });
}

extern "C" mml_status mml_bmf_set_user_offsets(mml_bmf* h, const float* p) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(is_svdpp(h), "user offsets belong to SVD++ handles");
        MML_REQUIRE(p, "null argument");
        h->ctx->activate();
        h->P.alloc((size_t)std::max<int64_t>(1, (int64_t)h->n_users * h->ld));
        upload_padded(h, h->P.get(), p, h->n_users);
        h->has_p = true;
        if (asym_ready(h)) asym_precompute(h);
        MML_HIP(hipStreamSynchronize(h->ctx->stream));
    });
}

extern "C" mml_status mml_bmf_get_user_offsets(mml_bmf* h, float* p) {
    return guard([&] {
        check_handle(h);
        single_device_only(h);
        MML_REQUIRE(h->has_p, "no user offsets (set_user_offsets first)");
        MML_REQUIRE(p, "null argument");
        h->ctx->activate();
        download_padded(h, p, h->P.get(), h->n_users);
        MML_HIP(hipStreamSynchronize(h->ctx->stream));
    });
}
