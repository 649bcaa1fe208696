// peer.hip -- collectives without a communicator, for a multi-device context that lists a device
// more than once (several shards on one GPU; mml_ctx_create_multi).  Two shapes:
//
//  * peer_average: the user shards' item average of BiasedMF and BPRMF (the
//    reference's parallel forms are BiasedMatrixFactorization.cs:205-215 and MultiCoreBPRMF.cs:
//    49-63).  The shards run one after another on one host thread; their arrays are staged on
//    shard 0's device by peer copies, summed there in shard order and divided by N (the
//    in-process emulation's arithmetic, tests/test_dist.py), and copied back.
//  * PeerGroup: one host thread per shard (mml::on_devices), each driving its own stream, meeting
//    at host barriers -- the shape of RCCL ranks.  WRMF's row shards all-gather through it
//    (each rank copies the other ranks' rows into its own matrix) and agree on the refinement's
//    stopping decision (the max over ranks of the last correction, as ncclMax would give); the
//    BiasedMF DSGD ring's ranks send item groups through it (bmf.hip ring_exchange / ring_bcast,
//    the peer-copy twins of ncclSend / ncclRecv and ncclBroadcast).
#include <condition_variable>
#include <mutex>

#include "mml_internal.h"

namespace {

// dst <- (dst + stage[0 .. parts - 2], left to right) / parts: the float sum in shard order, then
// one correctly rounded division
__global__ __launch_bounds__(256) void average_rows_kernel(float* __restrict__ dst,
                                                           const float* __restrict__ stage,
                                                           int64_t n, int64_t stride,
                                                           int32_t parts) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        float s = dst[x];
        for (int32_t p = 0; p + 1 < parts; ++p) s += stage[(int64_t)p * stride + x];
        dst[x] = s / (float)parts;
    }
}

inline int avg_grid(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

}  // namespace

namespace mml {

void peer_average(const std::vector<mml_ctx*>& ctxs, const std::vector<std::vector<float*>>& arr,
                  const std::vector<int64_t>& count, DeviceArray<float>& stage, hipEvent_t ev0,
                  hipEvent_t ev1) {
    const int32_t nd = (int32_t)ctxs.size();
    const size_t na = count.size();
    int64_t slot = 0;
    for (int64_t c : count) slot += c;
    mml_ctx* c0 = ctxs[0];
    c0->activate();
    hipStream_t st = c0->stream;
    // (the shards' epochs have returned: mml_*_iterate is synchronous)
    MML_HIP(hipEventRecord(ev0, st));
    if (nd > 1 && slot > 0) {
        stage.reserve((size_t)(nd - 1) * slot);
        for (int32_t d = 1; d < nd; ++d) {
            float* dst = stage.get() + (int64_t)(d - 1) * slot;
            for (size_t a = 0; a < na; ++a) {
                if (count[a] > 0)
                    MML_HIP(hipMemcpyPeerAsync(dst, c0->device, arr[d][a], ctxs[d]->device,
                                               sizeof(float) * count[a], st));
                dst += count[a];
            }
        }
        int64_t o = 0;
        for (size_t a = 0; a < na; ++a) {
            if (count[a] > 0)
                average_rows_kernel<<<avg_grid(count[a]), 256, 0, st>>>(arr[0][a],
                                                                        stage.get() + o, count[a],
                                                                        slot, nd);
            o += count[a];
        }
        MML_HIP(hipGetLastError());
        for (int32_t d = 1; d < nd; ++d)
            for (size_t a = 0; a < na; ++a)
                if (count[a] > 0)
                    MML_HIP(hipMemcpyPeerAsync(arr[d][a], ctxs[d]->device, arr[0][a], c0->device,
                                               sizeof(float) * count[a], st));
    }
    MML_HIP(hipEventRecord(ev1, st));
    for (int32_t d = 1; d < nd; ++d) {
        ctxs[d]->activate();
        MML_HIP(hipStreamWaitEvent(ctxs[d]->stream, ev1, 0));
    }
    c0->activate();
}

struct PeerGroup::Impl {
    std::mutex m;
    std::condition_variable cv;
    int32_t arrived = 0;
    uint64_t generation = 0;
    bool aborted = false;
};

PeerGroup::PeerGroup(int32_t n_) : n(n_), impl(new Impl), ptr((size_t)n_ * 4, nullptr), u32((size_t)n_ * 4, 0) {}
PeerGroup::~PeerGroup() { delete impl; }

void PeerGroup::barrier() {
    std::unique_lock<std::mutex> lk(impl->m);
    if (impl->aborted) fail(MML_ERR_STATE, "another shard of the context failed");
    const uint64_t gen = impl->generation;
    if (++impl->arrived == n) {
        impl->arrived = 0;
        ++impl->generation;
        impl->cv.notify_all();
        return;
    }
    impl->cv.wait(lk, [&] { return impl->generation != gen || impl->aborted; });
    if (impl->generation == gen) fail(MML_ERR_STATE, "another shard of the context failed");
}

void PeerGroup::abort() {
    std::lock_guard<std::mutex> lk(impl->m);
    impl->aborted = true;
    impl->cv.notify_all();
}

void PeerGroup::reset() {
    std::lock_guard<std::mutex> lk(impl->m);
    impl->aborted = false;
    impl->arrived = 0;
}

void PeerGroup::publish(const mml_ctx* ctx, int32_t slot, void* p) {
    ptr[(size_t)ctx->peer_rank * 4 + slot] = p;
}

void PeerGroup::allgather_rows(const mml_ctx* ctx, float* W, const std::vector<int64_t>& bounds,
                               int32_t k) {
    const int32_t r = ctx->peer_rank;
    MML_HIP(hipStreamSynchronize(ctx->stream));  // this rank's rows are final
    publish(ctx, 0, W);
    barrier();
    for (int32_t q = 0; q < n; ++q) {
        const int64_t rows = bounds[q + 1] - bounds[q];
        if (q == r || rows <= 0) continue;
        const size_t o = (size_t)bounds[q] * k;
        MML_HIP(hipMemcpyPeerAsync(W + o, ctx->device, static_cast<float*>(peer(q, 0)) + o,
                                   devices[q], sizeof(float) * rows * k, ctx->stream));
    }
    MML_HIP(hipStreamSynchronize(ctx->stream));
    barrier();  // nobody writes its matrix again before every rank has read it
}

void PeerGroup::max_u32(const mml_ctx* ctx, uint32_t* v, int32_t m) {
    const int32_t r = ctx->peer_rank;
    for (int32_t x = 0; x < m; ++x) u32[(size_t)r * 4 + x] = v[x];
    barrier();
    for (int32_t x = 0; x < m; ++x)
        for (int32_t q = 0; q < n; ++q) v[x] = std::max(v[x], u32[(size_t)q * 4 + x]);
    barrier();  // the slots are reused by the next call
}

}  // namespace mml
