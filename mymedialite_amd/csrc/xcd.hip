// xcd.hip -- XCD-owned item groups for the Hogwild kernels (BiasedMF SGD, BPR update).
//
// Why: each of the MI355X's 8 XCDs has its own write-back L2, and the L2s are not coherent with
// each other.  Plain Hogwild spread over all XCDs keeps up to 8 dirty replicas of a hot Zipf item
// row, and their write-backs overwrite each other's updates ("Hogwild and per-XCD
// caches": +1e-2 RMSE on a C2-shaped 4 M set, +0.0095 AUC on the C3 replica, -0.04 AUC for
// WeightedBPRMF).  Making the hot rows coherent sends every access to the memory side (2.8-15x
// slower).  Instead the items are dealt into 8 groups of equal rating mass, the stream is
// partitioned by the group of its item (stable: each group keeps the visit order), and the
// launch maps group g to blocks b with b % 8 == g -- blocks that share one XCD (dispatch deals
// blocks round-robin over the XCDs; mml::xcd_groups probes that on the device before relying on
// it).  Every access to an item row then comes from one XCD, whose single L2 holds the row.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset on the host
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdlib>
#include <numeric>
#include <vector>

#include "mml_internal.h"

namespace {

// lane 0 of every block writes the XCC (XCD) id its block runs on
__global__ __launch_bounds__(256) void xcd_probe_kernel(int32_t* __restrict__ out) {
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_XCC_ID)" : "=s"(id));
    // keep the block resident a little, so the whole grid is placed while others still run
    for (int x = 0; x < 64; ++x) __builtin_amdgcn_s_sleep(2);
    if (threadIdx.x == 0) out[blockIdx.x] = (int32_t)(id & 0xF);
}

// Both passes walk a block's segment in steps of kSub tiles of 256: every load of a step (keys,
// payloads, then the groups) is issued before the first tile is ranked, so a thread has kSub
// dependent load chains in flight instead of one (round 3: one tile per step, 2.5 + 7.3 ms per
// 500 M-entry partition at C3).
constexpr int kSub = 4;

// the group of entry x: group[key[x]], or (DIRECT) the byte gkey[x] the producer wrote
template <bool DIRECT>
__device__ __forceinline__ int32_t entry_key(const int32_t* __restrict__ key,
                                             const uint8_t* __restrict__ gkey, int64_t x) {
    if constexpr (DIRECT) return (int32_t)gkey[x];
    return key[x];
}
template <bool DIRECT>
__device__ __forceinline__ int entry_group(int32_t kx, const uint8_t* __restrict__ group) {
    if constexpr (DIRECT) return kx;
    return (int)group[kx];
}

// per (group, block) counts of one contiguous segment per block; groups by ballot, 8 per wave step
template <bool DIRECT>
__global__ __launch_bounds__(256) void xcd_count_kernel(const int32_t* __restrict__ key,
                                                        const uint8_t* __restrict__ gkey, int64_t n,
                                                        int64_t seg,
                                                        const uint8_t* __restrict__ group,
                                                        int64_t* __restrict__ cnt, int32_t nblk) {
    __shared__ int64_t c[4][8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t mine[8] = {0, 0, 0, 0, 0, 0, 0, 0};
    const int64_t b0 = (int64_t)blockIdx.x * seg, b1 = min(n, b0 + seg);
    for (int64_t t = b0; t < b1; t += 256 * kSub) {
        int32_t kx[kSub];
        int g[kSub];
#pragma unroll
        for (int u = 0; u < kSub; ++u) {
            const int64_t x = t + 256 * u + threadIdx.x;
            kx[u] = x < b1 ? entry_key<DIRECT>(key, gkey, x) : -1;
        }
#pragma unroll
        for (int u = 0; u < kSub; ++u) g[u] = kx[u] >= 0 ? entry_group<DIRECT>(kx[u], group) : -1;
#pragma unroll
        for (int u = 0; u < kSub; ++u)
#pragma unroll
            for (int gg = 0; gg < 8; ++gg) mine[gg] += __popcll(__ballot(g[u] == gg));
    }
    if (lane == 0)
        for (int gg = 0; gg < 8; ++gg) c[w][gg] = mine[gg];
    __syncthreads();
    if (threadIdx.x < 8)
        cnt[(int64_t)threadIdx.x * nblk + blockIdx.x] =
            c[0][threadIdx.x] + c[1][threadIdx.x] + c[2][threadIdx.x] + c[3][threadIdx.x];
}

struct Pay3 {
    const int32_t* in[3];
    int32_t* out[3];
};

// stable scatter: block b walks its segment in order; an entry of group g goes to base[g][b] +
// (entries of group g before it in the segment).  Every thread keeps the 8 group runs; per tile the
// waves' group counts go through the LDS (alternating buffers: one barrier per tile).
template <bool DIRECT>
__global__ __launch_bounds__(256) void xcd_scatter_kernel(const int32_t* __restrict__ key,
                                                          const uint8_t* __restrict__ gkey,
                                                          int64_t n, int64_t seg,
                                                          const uint8_t* __restrict__ group,
                                                          const int64_t* __restrict__ base,
                                                          int32_t nblk, int32_t npay, Pay3 p) {
    __shared__ int32_t wc[2][4][8];
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    int64_t run[8];
#pragma unroll
    for (int gg = 0; gg < 8; ++gg) run[gg] = base[(int64_t)gg * nblk + blockIdx.x];
    const int64_t b0 = (int64_t)blockIdx.x * seg, b1 = min(n, b0 + seg);
    const uint64_t below = (1ull << lane) - 1ull;
    int buf = 0;
    for (int64_t t = b0; t < b1; t += 256 * kSub) {
        int32_t kx[kSub], pv[3][kSub];
        int g[kSub];
#pragma unroll
        for (int u = 0; u < kSub; ++u) {
            const int64_t x = t + 256 * u + threadIdx.x;
            const bool in = x < b1;
            kx[u] = in ? entry_key<DIRECT>(key, gkey, x) : -1;
#pragma unroll
            for (int c = 0; c < 3; ++c) pv[c][u] = in && c < npay ? p.in[c][x] : 0;
        }
#pragma unroll
        for (int u = 0; u < kSub; ++u) g[u] = kx[u] >= 0 ? entry_group<DIRECT>(kx[u], group) : -1;
#pragma unroll
        for (int u = 0; u < kSub; ++u) {
            int rank = 0;
#pragma unroll
            for (int gg = 0; gg < 8; ++gg) {
                const uint64_t m = __ballot(g[u] == gg);
                if (lane == 0) wc[buf][w][gg] = __popcll(m);
                if (g[u] == gg) rank = __popcll(m & below);
            }
            __syncthreads();
            int32_t cw[4][8];
#pragma unroll
            for (int ww = 0; ww < 4; ++ww)
#pragma unroll
                for (int gg = 0; gg < 8; ++gg) cw[ww][gg] = wc[buf][ww][gg];
            if (g[u] >= 0) {
                int64_t dst = rank;
#pragma unroll
                for (int gg = 0; gg < 8; ++gg) {
                    if (gg != g[u]) continue;
                    dst += run[gg];
#pragma unroll
                    for (int ww = 0; ww < 4; ++ww) dst += ww < w ? cw[ww][gg] : 0;
                }
#pragma unroll
                for (int c = 0; c < 3; ++c)
                    if (c < npay) p.out[c][dst] = pv[c][u];
            }
#pragma unroll
            for (int gg = 0; gg < 8; ++gg)
                run[gg] += cw[0][gg] + cw[1][gg] + cw[2][gg] + cw[3][gg];
            buf ^= 1;
        }
    }
}

// goff[g] = start of group g (the scanned base of block 0), goff[ng] = n
__global__ void xcd_offsets_kernel(const int64_t* __restrict__ base, int32_t nblk, int64_t n,
                                   int64_t* __restrict__ goff) {
    const int g = threadIdx.x;
    if (g < 8) goff[g] = base[(int64_t)g * nblk];
    if (g == 8) goff[8] = n;
}

__global__ __launch_bounds__(256) void xcd_histogram_kernel(const int32_t* __restrict__ ids,
                                                            int64_t n, int32_t n_ids,
                                                            int32_t* __restrict__ cnt) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t v = ids[x];
        if (v >= 0 && v < n_ids) atomicAdd(cnt + v, 1);
    }
}

}  // namespace

namespace mml {

int32_t flushers_per_xcd(int32_t dflt) {
    static const int32_t v = [] {
        const char* e = MML_EXPERIMENT_ENV("MML_FLUSHERS");
        return e ? std::max(1, std::atoi(e)) : 0;
    }();
    return v > 0 ? v : dflt;
}

int32_t xcd_groups(mml_ctx* ctx) {
    if (ctx->xcd_groups > 0) return ctx->xcd_groups;
    const char* e = MML_EXPERIMENT_ENV("MML_XCD_GROUPS");
    if (e && std::atoi(e) <= 1) return ctx->xcd_groups = 1;
    constexpr int kBlocks = 2048;  // the Hogwild launches' grid size
    DeviceArray<int32_t> ids;
    ids.alloc(kBlocks);
    xcd_probe_kernel<<<kBlocks, 256, 0, ctx->stream>>>(ids.get());
    MML_HIP(hipGetLastError());
    std::vector<int32_t> h(kBlocks);
    MML_HIP(hipMemcpyAsync(h.data(), ids.get(), sizeof(int32_t) * kBlocks,
                           hipMemcpyDeviceToHost, ctx->stream));
    MML_HIP(hipStreamSynchronize(ctx->stream));
    bool ok = true;
    std::vector<bool> seen(16, false);
    for (int b = 0; b < 8; ++b) {
        ok &= !seen[h[b]];
        seen[h[b]] = true;
    }
    for (int b = 8; b < kBlocks && ok; ++b) ok = h[b] == h[b % 8];
    ctx->xcd_groups = ok ? 8 : 1;
    return ctx->xcd_groups;
}

std::vector<uint8_t> balanced_item_groups(const std::vector<int64_t>& weight, int32_t ng) {
    std::vector<uint8_t> g(weight.size(), 0);
    if (ng <= 1) return g;
    std::vector<int32_t> order(weight.size());
    std::iota(order.begin(), order.end(), 0);
    // heaviest first, ties by id: deterministic longest-processing-time deal
    std::stable_sort(order.begin(), order.end(),
                     [&](int32_t a, int32_t b) { return weight[a] > weight[b]; });
    std::vector<int64_t> load(ng, 0);
    for (int32_t i : order) {
        int best = 0;
        for (int x = 1; x < ng; ++x)
            if (load[x] < load[best]) best = x;
        g[i] = (uint8_t)best;
        load[best] += weight[i];
    }
    return g;
}

void XcdSplit::set_groups(hipStream_t st, const std::vector<int64_t>& weight, int32_t groups) {
    ng = groups;
    n_items = (int32_t)weight.size();
    const std::vector<uint8_t> g = balanced_item_groups(weight, groups);
    group.alloc(std::max<size_t>(1, g.size()));
    if (!g.empty())
        MML_HIP(hipMemcpyAsync(group.get(), g.data(), g.size(), hipMemcpyHostToDevice, st));
    goff.alloc(9);
    MML_HIP(hipStreamSynchronize(st));
}

void XcdSplit::set_table(hipStream_t st, const std::vector<uint8_t>& table) {
    ng = 8;
    n_items = (int32_t)table.size();
    group.alloc(std::max<size_t>(1, table.size()));
    if (!table.empty())
        MML_HIP(hipMemcpyAsync(group.get(), table.data(), table.size(), hipMemcpyHostToDevice, st));
    goff.alloc(9);
    MML_HIP(hipStreamSynchronize(st));
}

namespace {
template <bool DIRECT>
void partition_impl(XcdSplit& xs, hipStream_t st, const int32_t* key, const uint8_t* gkey,
                    int64_t n, int32_t npay, const int32_t* const* in, int32_t* const* out,
                    int64_t* goff_out) {
    MML_REQUIRE(xs.ng == 8 && npay >= 1 && npay <= 3, "XcdSplit::partition: bad setup");
    const int32_t nblk = (int32_t)std::max<int64_t>(1, std::min<int64_t>(2048, (n + 4095) / 4096));
    const int64_t seg = (n + nblk - 1) / nblk;
    xs.cnt.alloc((size_t)8 * nblk);
    xs.base.alloc((size_t)8 * nblk);
    size_t tb = 0;
    MML_HIP(rocprim::exclusive_scan(nullptr, tb, xs.cnt.get(), xs.base.get(), (int64_t)0,
                                    8 * nblk, rocprim::plus<int64_t>(), st));
    if (xs.tmp.count < tb) xs.tmp.alloc(tb);
    xcd_count_kernel<DIRECT><<<nblk, 256, 0, st>>>(key, gkey, n, seg, xs.group.get(), xs.cnt.get(),
                                                   nblk);
    MML_HIP(hipGetLastError());
    MML_HIP(rocprim::exclusive_scan(xs.tmp.get(), tb, xs.cnt.get(), xs.base.get(), (int64_t)0,
                                    8 * nblk, rocprim::plus<int64_t>(), st));
    Pay3 p{};
    for (int c = 0; c < npay; ++c) {
        p.in[c] = in[c];
        p.out[c] = out[c];
    }
    xcd_scatter_kernel<DIRECT><<<nblk, 256, 0, st>>>(key, gkey, n, seg, xs.group.get(),
                                                     xs.base.get(), nblk, npay, p);
    xcd_offsets_kernel<<<1, 64, 0, st>>>(xs.base.get(), nblk, n,
                                         goff_out ? goff_out : xs.goff.get());
    MML_HIP(hipGetLastError());
}
}  // namespace

void XcdSplit::partition(hipStream_t st, const int32_t* key, int64_t n, int32_t npay,
                         const int32_t* const* in, int32_t* const* out, int64_t* goff_out) {
    partition_impl<false>(*this, st, key, nullptr, n, npay, in, out, goff_out);
}

void XcdSplit::partition_groups(hipStream_t st, const uint8_t* gkey, int64_t n, int32_t npay,
                                const int32_t* const* in, int32_t* const* out,
                                int64_t* goff_out) {
    partition_impl<true>(*this, st, nullptr, gkey, n, npay, in, out, goff_out);
}

std::vector<int64_t> device_id_counts(hipStream_t st, const int32_t* ids, int64_t n,
                                      int32_t n_ids) {
    DeviceArray<int32_t> c;
    c.alloc(std::max<int32_t>(1, n_ids));
    MML_HIP(hipMemsetAsync(c.get(), 0, sizeof(int32_t) * std::max<int32_t>(1, n_ids), st));
    if (n > 0) {
        const int grid = (int)std::max<int64_t>(1, std::min<int64_t>(8192, (n + 255) / 256));
        xcd_histogram_kernel<<<grid, 256, 0, st>>>(ids, n, n_ids, c.get());
        MML_HIP(hipGetLastError());
    }
    std::vector<int32_t> h(std::max<int32_t>(1, n_ids));
    MML_HIP(hipMemcpyAsync(h.data(), c.get(), sizeof(int32_t) * h.size(), hipMemcpyDeviceToHost,
                           st));
    MML_HIP(hipStreamSynchronize(st));
    return std::vector<int64_t>(h.begin(), h.begin() + n_ids);
}

}  // namespace mml

using mml::guard;

extern "C" mml_status mml_ctx_xcd_groups(mml_ctx* ctx, int32_t* out) {
    return guard([&] {
        MML_REQUIRE(ctx && out, "null argument");
        ctx->activate();
        *out = mml::xcd_groups(ctx);
    });
}
