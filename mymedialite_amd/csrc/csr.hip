// csr.hip -- building the positive-feedback sets on the device (data ingest for BPRMF / WRMF).
//
// PosOnlyFeedback.UserMatrix / ItemMatrix (src/MyMediaLite/Data/PosOnlyFeedback.cs:35-83) are
// HashSet rows; on the device they are CSR rows, sorted and de-duplicated:
//   key = row << 32 | col  ->  radix sort (hipCUB)  ->  unique  ->  per-row counts  ->  scan.
// 500M events (C3) take a few hundred ms instead of a host sort of minutes.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset on the host
#include <rocprim/rocprim.hpp>

#include <vector>

#include "mml_internal.h"

namespace {

__global__ __launch_bounds__(256) void pack_keys_kernel(const int32_t* __restrict__ rows,
                                                        const int32_t* __restrict__ cols,
                                                        int64_t n, int32_t n_rows, int32_t n_cols,
                                                        uint64_t* __restrict__ keys,
                                                        int32_t* __restrict__ bad) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const int32_t r = rows[x], c = cols[x];
        if (r < 0 || r >= n_rows || c < 0 || c >= n_cols) {
            atomicOr(bad, 1);
            keys[x] = 0;
            continue;
        }
        keys[x] = ((uint64_t)(uint32_t)r << 32) | (uint32_t)c;
    }
}

__global__ __launch_bounds__(256) void unpack_keys_kernel(const uint64_t* __restrict__ keys,
                                                          const int64_t* __restrict__ n_ptr,
                                                          int32_t* __restrict__ cols,
                                                          int32_t* __restrict__ deg) {
    const int64_t n = *n_ptr;
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        const uint64_t k = keys[x];
        cols[x] = (int32_t)(uint32_t)(k & 0xffffffffu);
        atomicAdd(deg + (int32_t)(k >> 32), 1);
    }
}

__global__ __launch_bounds__(256) void widen_kernel(const int32_t* __restrict__ deg, int32_t n,
                                                    int64_t* __restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[x] = deg[x];
}

inline int grid_for(int64_t n) {
    return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 8192));
}

int bits_for(uint32_t v) {
    int b = 0;
    while (b < 32 && (v >> b) != 0) ++b;
    return b;
}

}  // namespace

namespace mml {

void build_csr_device(const int32_t* rows, const int32_t* cols, int64_t n, int32_t n_rows,
                      int32_t n_cols, hipStream_t st, DeviceCsr& out) {
    MML_REQUIRE(n >= 0 && n_rows >= 1 && n_cols >= 1, "bad CSR sizes");
    out.off.alloc((size_t)n_rows + 1);
    out.deg_host.assign(n_rows, 0);
    if (n == 0) {
        MML_HIP(hipMemsetAsync(out.off.get(), 0, sizeof(int64_t) * (n_rows + 1), st));
        out.cols.alloc(16);
        out.nnz = 0;
        MML_HIP(hipStreamSynchronize(st));
        return;
    }
    DeviceArray<uint64_t> keys, sorted;
    DeviceArray<int32_t> flag, deg;
    DeviceArray<int64_t> nsel, deg64;
    keys.alloc(n);
    sorted.alloc(n);
    flag.alloc(1);
    nsel.alloc(1);
    MML_HIP(hipMemsetAsync(flag.get(), 0, sizeof(int32_t), st));
    pack_keys_kernel<<<grid_for(n), 256, 0, st>>>(rows, cols, n, n_rows, n_cols, keys.get(),
                                                  flag.get());
    MML_HIP(hipGetLastError());
    int32_t bad = 0;
    MML_HIP(hipMemcpyAsync(&bad, flag.get(), sizeof(int32_t), hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    MML_REQUIRE(!bad, "event user/item id out of range");
    const int end_bit = 32 + bits_for((uint32_t)(n_rows - 1));
    size_t tmp_bytes = 0;
    MML_HIP(rocprim::radix_sort_keys(nullptr, tmp_bytes, keys.get(), sorted.get(), n, 0,
                                              end_bit, st));
    size_t tmp2 = 0;
    MML_HIP(rocprim::unique(nullptr, tmp2, sorted.get(), keys.get(), nsel.get(), n,
            rocprim::equal_to<uint64_t>(), st));
    DeviceArray<uint8_t> tmp;
    tmp.alloc(std::max(tmp_bytes, tmp2));
    MML_HIP(rocprim::radix_sort_keys(tmp.get(), tmp_bytes, keys.get(), sorted.get(), n, 0,
                                              end_bit, st));
    MML_HIP(rocprim::unique(tmp.get(), tmp2, sorted.get(), keys.get(), nsel.get(), n,
            rocprim::equal_to<uint64_t>(), st));
    int64_t nnz = 0;
    MML_HIP(hipMemcpyAsync(&nnz, nsel.get(), sizeof(int64_t), hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    // 16 entries of padding: the BPR sampler scans rows with aligned int4 loads that may run up to
    // 15 entries past the last row (masked, never used)
    out.cols.alloc(nnz + 16);
    MML_HIP(hipMemsetAsync(out.cols.get() + nnz, 0xff, sizeof(int32_t) * 16, st));
    deg.alloc(n_rows);
    MML_HIP(hipMemsetAsync(deg.get(), 0, sizeof(int32_t) * n_rows, st));
    unpack_keys_kernel<<<grid_for(nnz), 256, 0, st>>>(keys.get(), nsel.get(), out.cols.get(),
                                                      deg.get());
    MML_HIP(hipGetLastError());
    deg64.alloc(n_rows);
    widen_kernel<<<grid_for(n_rows), 256, 0, st>>>(deg.get(), n_rows, deg64.get());
    MML_HIP(hipGetLastError());
    MML_HIP(hipMemsetAsync(out.off.get(), 0, sizeof(int64_t), st));
    size_t tmp3 = 0;
    MML_HIP(rocprim::inclusive_scan(nullptr, tmp3, deg64.get(), out.off.get() + 1, n_rows,
            rocprim::plus<int64_t>(), st));
    tmp.alloc(std::max(tmp.count, tmp3));
    MML_HIP(rocprim::inclusive_scan(tmp.get(), tmp3, deg64.get(), out.off.get() + 1, n_rows,
            rocprim::plus<int64_t>(), st));
    MML_HIP(hipMemcpyAsync(out.deg_host.data(), deg.get(), sizeof(int32_t) * n_rows,
                           hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    out.nnz = nnz;
}

}  // namespace mml
