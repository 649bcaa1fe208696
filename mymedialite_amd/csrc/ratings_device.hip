// ratings_device.hip -- IO/StaticRatingData.Read (src/MyMediaLite/IO/StaticRatingData.cs:36-117)
// with the parse on the device: the file's bytes go to HBM once and the lines are tokenised there,
// so a C4-sized file (1 B lines, ~16 GB of text) lands as SoA arrays in HBM without the host parse
// (66 M lines/s on 16 host threads).  Same results as the host reader
// (ratings_file.cpp), which stays the definition:
//   * lines as ReadLine splits them ("\n", a lone "\r", "\r\n"; a UTF-8 BOM dropped), the first one
//     skipped with MML_READ_IGNORE_FIRST_LINE, empty lines counted in n_lines but not stored;
//   * tokens split on every '\t', ' ', ',' (empty tokens kept, String.Split);
//   * IdentityMapping ids: the host's int.Parse restatement ('+' stripped, then [-]digits, no
//     overflow); Mapping ids (Data/Mapping.cs:75-85, first-appearance order after the caller's
//     seeds): resolved on the device when every token and seed is a canonical decimal ("0" or
//     [1-9][0-9]{0,17}, so the string and its value identify each other);
//   * ratings: float.Parse, correctly rounded: decimals with <= 19 significant digits whose
//     mantissa fits 2^24 and |exponent| <= 10 are exact by one IEEE multiply or divide (both
//     operands exact); anything else takes the host reader.
// Whatever the device path does not cover (ItemData, the binary cache, non-canonical Mapping ids,
// other rating spellings, any malformed line -- for the reference's exact error text) runs the host
// reader and uploads its arrays: the result is the same either way, and device_parsed says which
// path ran.
#include <cstring>  // rocprim/iterator/texture_cache_iterator.hpp uses memset on the host
#include <rocprim/rocprim.hpp>

#include <algorithm>
#include <cstdint>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include <fcntl.h>
#include <sys/stat.h>
#include <unistd.h>

#include "mml_internal.h"

namespace {

constexpr int64_t kSeg = 4096;   // bytes per thread: the lines that START in it are its lines
constexpr int64_t kPad = 64;     // zero bytes after the text (loads past the end read zeros)
enum : uint32_t { kErrFormat = 1, kErrKey = 2, kErrFloat = 4 };

__device__ __forceinline__ bool d_sep(uint8_t c) { return c == '\t' || c == ' ' || c == ','; }
__device__ __forceinline__ bool d_term(uint8_t c) { return c == '\n' || c == '\r'; }
// a line starts at p (bom <= p < n): after "\n", after a "\r" not followed by "\n", or at the BOM end
__device__ __forceinline__ bool d_start(const uint8_t* B, int64_t p, int64_t bom) {
    if (p == bom) return true;
    const uint8_t a = B[p - 1];
    return a == '\n' || (a == '\r' && B[p] != '\n');
}

// pass 1: per segment, the lines starting in it and the non-empty ones among them
__global__ __launch_bounds__(256) void rf_count_kernel(const uint8_t* __restrict__ B, int64_t n,
                                                       int64_t bom, int skip_first, int64_t nseg,
                                                       int64_t* __restrict__ lines,
                                                       int64_t* __restrict__ rows) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg;
         s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t lo = max(s * kSeg, bom), hi = min((s + 1) * kSeg, n);
        int64_t nl = 0, nr = 0;
        if (lo < hi) {
            const int64_t a0 = lo & ~(int64_t)15;
            uint8_t prev = a0 > 0 ? B[a0 - 1] : 0;
            for (int64_t p0 = a0; p0 < hi; p0 += 16) {
                const uint4 w = *reinterpret_cast<const uint4*>(B + p0);
                const uint32_t word[4] = {w.x, w.y, w.z, w.w};
#pragma unroll
                for (int b = 0; b < 16; ++b) {
                    const uint8_t c = (uint8_t)(word[b >> 2] >> (8 * (b & 3)));
                    const int64_t p = p0 + b;
                    if (p >= lo && p < hi) {
                        const bool st = p == bom || prev == '\n' || (prev == '\r' && c != '\n');
                        if (st && !(skip_first && p == bom)) {
                            ++nl;
                            nr += !d_term(c);
                        }
                    }
                    prev = c;
                }
            }
        }
        lines[s] = nl;
        rows[s] = nr;
    }
}

// int.Parse as the host reader restates it: one '+' stripped, then [-]digits, no overflow
__device__ __forceinline__ bool d_parse_int(const uint8_t* p, int64_t len, int32_t& out) {
    int64_t x = 0;
    if (x < len && p[x] == '+') ++x;
    bool neg = false;
    if (x < len && p[x] == '-') {
        neg = true;
        ++x;
    }
    if (x >= len) return false;
    int64_t v = 0;
    for (; x < len; ++x) {
        const uint8_t c = p[x];
        if (c < '0' || c > '9') return false;
        v = v * 10 + (c - '0');
        if (v > 2147483648ll) return false;
    }
    if (!neg && v > 2147483647ll) return false;
    out = (int32_t)(neg ? -v : v);
    return true;
}

// a canonical decimal id ("0" or [1-9][0-9]{0,17}): its value identifies the string
__device__ __forceinline__ bool d_parse_key(const uint8_t* p, int64_t len, int64_t& out) {
    if (len < 1 || len > 18) return false;
    if (p[0] == '0') {
        out = 0;
        return len == 1;
    }
    int64_t v = 0;
    for (int64_t x = 0; x < len; ++x) {
        const uint8_t c = p[x];
        if (c < '0' || c > '9') return false;
        v = v * 10 + (c - '0');
    }
    out = v;
    return true;
}

// float.Parse on the fast path: [+][-]digits[.digits][(e|E)[+-]digits] with the significant
// digits' value M <= 2^24 and the decimal exponent E in [-10, 10]: float(M) and 10^|E| are exact,
// so one multiply or divide rounds correctly.  false: not this shape (the host reader decides)
__device__ __forceinline__ bool d_parse_float(const uint8_t* p, int64_t len, float& out) {
    int64_t x = 0;
    if (x < len && p[x] == '+') ++x;
    bool neg = false;
    if (x < len && p[x] == '-') {
        neg = true;
        ++x;
    }
    uint64_t m = 0;
    int sig = 0, digits = 0, e10 = 0;
    for (; x < len && p[x] >= '0' && p[x] <= '9'; ++x, ++digits) {
        if (m == 0 && p[x] == '0') continue;
        if (++sig > 19) return false;
        m = m * 10 + (p[x] - '0');
    }
    if (x < len && p[x] == '.') {
        for (++x; x < len && p[x] >= '0' && p[x] <= '9'; ++x, ++digits) {
            --e10;
            if (m == 0 && p[x] == '0') continue;
            if (++sig > 19) return false;
            m = m * 10 + (p[x] - '0');
        }
    }
    if (digits == 0) return false;
    if (x < len && (p[x] == 'e' || p[x] == 'E')) {
        ++x;
        bool eneg = false;
        if (x < len && (p[x] == '+' || p[x] == '-')) eneg = p[x++] == '-';
        if (x >= len) return false;
        int ev = 0;
        for (; x < len; ++x) {
            if (p[x] < '0' || p[x] > '9') return false;
            ev = ev * 10 + (p[x] - '0');
            if (ev > 1000) return false;
        }
        e10 += eneg ? -ev : ev;
    }
    if (x != len) return false;
    if (m == 0) {
        out = neg ? -0.0f : 0.0f;
        return true;
    }
    if (m > (1u << 24) || e10 < -10 || e10 > 10) return false;
    float pw = 1.0f;
    for (int t = 0; t < (e10 < 0 ? -e10 : e10); ++t) pw *= 10.0f;  // exact up to 1e10
    const float v = e10 < 0 ? (float)m / pw : (float)m * pw;
    out = neg ? -v : v;
    return true;
}

// pass 2: each segment's lines tokenised into the outputs from its row offset on
__global__ __launch_bounds__(256) void rf_parse_kernel(
    const uint8_t* __restrict__ B, int64_t n, int64_t bom, int skip_first, int64_t nseg,
    const int64_t* __restrict__ at, int want, int user_identity, int item_identity,
    int32_t* __restrict__ users, int32_t* __restrict__ items, float* __restrict__ values,
    int64_t* __restrict__ ukeys, int64_t* __restrict__ ikeys, uint32_t* __restrict__ err) {
    for (int64_t s = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; s < nseg;
         s += (int64_t)gridDim.x * blockDim.x) {
        const int64_t lo = max(s * kSeg, bom), hi = min((s + 1) * kSeg, n);
        int64_t o = at[s];
        uint32_t e = 0;
        int64_t p = lo;
        while (p < hi && !d_start(B, p, bom)) ++p;  // the first line starting in the segment
        while (p < hi) {
            // the line [p, q) up to its terminator; the next line starts after "\n", "\r\n" or
            // a lone "\r"
            int64_t q = p, sep[3] = {-1, -1, -1};
            int ns = 0;
            while (q < n && !d_term(B[q])) {
                if (d_sep(B[q])) {
                    if (ns < 3) sep[ns] = q;
                    ++ns;
                }
                ++q;
            }
            const int64_t next = (q < n && B[q] == '\r' && B[q + 1] == '\n') ? q + 2 : q + 1;
            const bool skip = (skip_first && p == bom) || q == p;  // skipped / empty line
            const int64_t p_line = p;
            p = next;
            if (skip) continue;
            if (ns < want - 1) {
                e |= kErrFormat;
                break;
            }
            // tokens: [p, sep0), [sep0 + 1, sep1 or q), [sep1 + 1, sep2 or q)
            const int64_t t0 = p_line, l0 = sep[0] - p_line;
            const int64_t t1 = sep[0] + 1, l1 = (ns >= 2 ? sep[1] : q) - t1;
            if (user_identity) {
                if (!d_parse_int(B + t0, l0, users[o])) e |= kErrFormat;
            } else if (!d_parse_key(B + t0, l0, ukeys[o])) {
                e |= kErrKey;
            }
            if (item_identity) {
                if (!d_parse_int(B + t1, l1, items[o])) e |= kErrFormat;
            } else if (!d_parse_key(B + t1, l1, ikeys[o])) {
                e |= kErrKey;
            }
            if (want == 3) {
                const int64_t t2 = sep[1] + 1, l2 = (ns >= 3 ? sep[2] : q) - t2;
                if (!d_parse_float(B + t2, l2, values[o])) e |= kErrFloat;
            } else {
                values[o] = 0.0f;
            }
            if (e) break;
            ++o;
        }
        if (e) atomicOr(err, e);
    }
}

// ---- Mapping on the device: first-appearance order of canonical decimal keys
__global__ void rf_iota_kernel(int32_t* __restrict__ v, int64_t n) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        v[x] = (int32_t)x;
}
// heads of the sorted keys: flag 1 where a new key starts
__global__ void rf_heads_kernel(const int64_t* __restrict__ ks, int64_t n, int32_t* __restrict__ f) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        f[x] = x == 0 || ks[x] != ks[x - 1];
}
// per distinct key d (head at sorted position x, dix = inclusive scan - 1): its key, its first
// row (the stable sort keeps rows ascending within a key), and its seed id or -1
__global__ void rf_distinct_kernel(const int64_t* __restrict__ ks, const int32_t* __restrict__ rs,
                                   const int32_t* __restrict__ dix, int64_t n,
                                   const int64_t* __restrict__ seed_keys,
                                   const int32_t* __restrict__ seed_ids, int32_t n_seed,
                                   int64_t* __restrict__ dkey, int32_t* __restrict__ dfirst,
                                   int32_t* __restrict__ did) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x) {
        if (x != 0 && ks[x] == ks[x - 1]) continue;
        const int32_t d = dix[x] - 1;
        const int64_t key = ks[x];
        dkey[d] = key;
        int32_t lo = 0, hi = n_seed;
        while (lo < hi) {
            const int32_t mid = (lo + hi) >> 1;
            if (seed_keys[mid] < key) lo = mid + 1;
            else hi = mid;
        }
        const bool seeded = lo < n_seed && seed_keys[lo] == key;
        did[d] = seeded ? seed_ids[lo] : -1;
        dfirst[d] = seeded ? INT32_MAX : rs[x];  // seeded keys sort after every new one
    }
}
// new keys in first-appearance order (sorted by first row): id = n_seed + rank
__global__ void rf_new_ids_kernel(const int32_t* __restrict__ sorted_d, int32_t n_new,
                                  int32_t n_seed, int32_t* __restrict__ did) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n_new;
         x += (int64_t)gridDim.x * blockDim.x)
        did[sorted_d[x]] = n_seed + (int32_t)x;
}
__global__ void rf_scatter_ids_kernel(const int32_t* __restrict__ rs,
                                      const int32_t* __restrict__ dix, const int32_t* __restrict__ did,
                                      int64_t n, int32_t* __restrict__ out) {
    for (int64_t x = (int64_t)blockIdx.x * blockDim.x + threadIdx.x; x < n;
         x += (int64_t)gridDim.x * blockDim.x)
        out[rs[x]] = did[dix[x] - 1];
}

int grid_of(int64_t n) { return (int)std::max<int64_t>(1, std::min<int64_t>((n + 255) / 256, 16384)); }

bool canonical_seed(const char* s, int64_t& key) {
    const size_t len = std::strlen(s);
    if (len < 1 || len > 18) return false;
    if (s[0] == '0') {
        key = 0;
        return len == 1;
    }
    int64_t v = 0;
    for (size_t x = 0; x < len; ++x) {
        if (s[x] < '0' || s[x] > '9') return false;
        v = v * 10 + (s[x] - '0');
    }
    key = v;
    return true;
}

// Mapping.ToInternalID over a device key column (rows in file order) -> ids in `out`, the new
// external ids (in internal-id order) to `fresh`
void map_keys_device(hipStream_t st, const int64_t* keys, int64_t N, const std::vector<int64_t>& seed,
                     int32_t* out, std::vector<std::string>& fresh) {
    fresh.clear();
    if (N == 0) return;
    MML_REQUIRE(N < INT32_MAX, "device Mapping: at most 2^31 - 1 rows");
    // seeds sorted by key, with their ids
    std::vector<std::pair<int64_t, int32_t>> sv(seed.size());
    for (size_t x = 0; x < seed.size(); ++x) sv[x] = {seed[x], (int32_t)x};
    std::sort(sv.begin(), sv.end());
    std::vector<int64_t> sk(sv.size());
    std::vector<int32_t> si(sv.size());
    for (size_t x = 0; x < sv.size(); ++x) {
        sk[x] = sv[x].first;
        si[x] = sv[x].second;
    }
    mml::DeviceArray<int64_t> dsk, ks;
    mml::DeviceArray<int32_t> dsi, rows, rs, flag, dix;
    dsk.alloc(std::max<size_t>(1, sk.size()));
    dsi.alloc(std::max<size_t>(1, si.size()));
    if (!sk.empty()) {
        MML_HIP(hipMemcpyAsync(dsk.get(), sk.data(), sizeof(int64_t) * sk.size(),
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(dsi.get(), si.data(), sizeof(int32_t) * si.size(),
                               hipMemcpyHostToDevice, st));
    }
    rows.alloc(N);
    rf_iota_kernel<<<grid_of(N), 256, 0, st>>>(rows.get(), N);
    ks.alloc(N);
    rs.alloc(N);
    // canonical keys are < 10^18 < 2^60
    size_t tmp_b = 0;
    MML_HIP(rocprim::radix_sort_pairs(nullptr, tmp_b, keys, ks.get(), rows.get(), rs.get(),
                                               N, 0, 60, st));
    mml::DeviceArray<uint8_t> tmp;
    tmp.alloc(tmp_b);
    MML_HIP(rocprim::radix_sort_pairs(tmp.get(), tmp_b, keys, ks.get(), rows.get(), rs.get(),
                                               N, 0, 60, st));
    rows.reset();
    flag.alloc(N);
    dix.alloc(N);
    rf_heads_kernel<<<grid_of(N), 256, 0, st>>>(ks.get(), N, flag.get());
    size_t scan_b = 0;
    MML_HIP(rocprim::inclusive_scan(nullptr, scan_b, flag.get(), dix.get(), N,
            rocprim::plus<int32_t>(), st));
    tmp.reserve(scan_b);
    MML_HIP(rocprim::inclusive_scan(tmp.get(), scan_b, flag.get(), dix.get(), N,
            rocprim::plus<int32_t>(), st));
    int32_t D = 0;
    MML_HIP(hipMemcpyAsync(&D, dix.get() + N - 1, sizeof(int32_t), hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    flag.reset();
    mml::DeviceArray<int64_t> dkey;
    mml::DeviceArray<int32_t> dfirst, did, order, dfirst_s, order_s;
    dkey.alloc(D);
    dfirst.alloc(D);
    did.alloc(D);
    rf_distinct_kernel<<<grid_of(N), 256, 0, st>>>(ks.get(), rs.get(), dix.get(), N, dsk.get(),
                                                   dsi.get(), (int32_t)sk.size(), dkey.get(),
                                                   dfirst.get(), did.get());
    // new keys by first row
    order.alloc(D);
    rf_iota_kernel<<<grid_of(D), 256, 0, st>>>(order.get(), D);
    dfirst_s.alloc(D);
    order_s.alloc(D);
    size_t sort2_b = 0;
    MML_HIP(rocprim::radix_sort_pairs(nullptr, sort2_b, dfirst.get(), dfirst_s.get(),
                                               order.get(), order_s.get(), D, 0, 32, st));
    tmp.reserve(sort2_b);
    MML_HIP(rocprim::radix_sort_pairs(tmp.get(), sort2_b, dfirst.get(), dfirst_s.get(),
                                               order.get(), order_s.get(), D, 0, 32, st));
    std::vector<int32_t> first_s(D);
    MML_HIP(hipMemcpyAsync(first_s.data(), dfirst_s.get(), sizeof(int32_t) * D,
                           hipMemcpyDeviceToHost, st));
    MML_HIP(hipStreamSynchronize(st));
    const int32_t n_new = (int32_t)(std::lower_bound(first_s.begin(), first_s.end(), INT32_MAX) -
                                    first_s.begin());
    if (n_new > 0)
        rf_new_ids_kernel<<<grid_of(n_new), 256, 0, st>>>(order_s.get(), n_new, (int32_t)sk.size(),
                                                          did.get());
    rf_scatter_ids_kernel<<<grid_of(N), 256, 0, st>>>(rs.get(), dix.get(), did.get(), N, out);
    MML_HIP(hipGetLastError());
    // the new external ids, in internal-id order
    std::vector<int32_t> dord(n_new);
    std::vector<int64_t> allkeys(D);
    if (n_new > 0)
        MML_HIP(hipMemcpyAsync(dord.data(), order_s.get(), sizeof(int32_t) * n_new,
                               hipMemcpyDeviceToHost, st));
    MML_HIP(hipMemcpyAsync(allkeys.data(), dkey.get(), sizeof(int64_t) * D, hipMemcpyDeviceToHost,
                           st));
    MML_HIP(hipStreamSynchronize(st));
    fresh.reserve(n_new);
    for (int32_t x = 0; x < n_new; ++x) fresh.push_back(std::to_string(allkeys[dord[x]]));
}

// The file straight into a device buffer (kPad zero bytes after it): kRingSlots host threads each
// own one pinned kChunk slot and one stream, and loop pread(chunk) -> async copy -> next chunk, so
// the reads of one slot overlap the copies of the others and no file-sized host buffer is ever
// allocated (first-touching 16 GB of fresh pages costs seconds on its own).  Returns false if the
// file cannot be read (the host reader then reports it).
constexpr size_t kChunk = (size_t)64 << 20;
constexpr int kRingSlots = 8;
bool upload_file(const char* path, int64_t& n, mml::DeviceArray<uint8_t>& B, uint8_t* head,
                 hipStream_t st) {
    const int fd = ::open(path, O_RDONLY);
    if (fd < 0) return false;
    struct stat st_ {};
    if (::fstat(fd, &st_) != 0) {
        ::close(fd);
        return false;
    }
    n = (int64_t)st_.st_size;
    B.alloc((size_t)n + kPad);
    MML_HIP(hipMemsetAsync(B.get() + n, 0, kPad, st));
    const int64_t chunks = (n + (int64_t)kChunk - 1) / (int64_t)kChunk;
    uint8_t* ring = nullptr;
    MML_HIP(hipHostMalloc(reinterpret_cast<void**>(&ring), kChunk * kRingSlots, hipHostMallocDefault));
    std::vector<int> ok(kRingSlots, 1);
    std::vector<std::thread> th;
    for (int t = 0; t < kRingSlots; ++t)
        th.emplace_back([&, t] {
            hipStream_t cs = nullptr;
            if (hipStreamCreateWithFlags(&cs, hipStreamNonBlocking) != hipSuccess) {
                ok[t] = 0;
                return;
            }
            uint8_t* slot = ring + (size_t)t * kChunk;
            for (int64_t c = t; c < chunks && ok[t]; c += kRingSlots) {
                if (hipStreamSynchronize(cs) != hipSuccess) ok[t] = 0;  // the slot's last copy
                const int64_t a0 = c * (int64_t)kChunk;
                const int64_t len = std::min<int64_t>((int64_t)kChunk, n - a0);
                for (int64_t got = 0; got < len && ok[t];) {
                    const ssize_t r = ::pread(fd, slot + got, (size_t)(len - got), (off_t)(a0 + got));
                    if (r <= 0) ok[t] = 0;
                    else got += r;
                }
                if (c == 0 && ok[t]) std::memcpy(head, slot, (size_t)std::min<int64_t>(len, 3));
                if (ok[t] && hipMemcpyAsync(B.get() + a0, slot, (size_t)len, hipMemcpyHostToDevice,
                                            cs) != hipSuccess)
                    ok[t] = 0;
            }
            if (hipStreamSynchronize(cs) != hipSuccess) ok[t] = 0;
            (void)hipStreamDestroy(cs);
        });
    for (auto& x : th) x.join();
    ::close(fd);
    (void)hipHostFree(ring);
    for (int t = 0; t < kRingSlots; ++t)
        if (!ok[t]) return false;
    return true;
}

// the host reader's result uploaded to the context (the fallback path)
void upload(mml_rating_file* f, hipStream_t st) {
    const int64_t N = f->n_ratings;
    f->d_users.alloc(std::max<int64_t>(1, N));
    f->d_items.alloc(std::max<int64_t>(1, N));
    f->d_values.alloc(std::max<int64_t>(1, N));
    if (N > 0) {
        MML_HIP(hipMemcpyAsync(f->d_users.get(), f->users.get(), sizeof(int32_t) * N,
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(f->d_items.get(), f->items.get(), sizeof(int32_t) * N,
                               hipMemcpyHostToDevice, st));
        MML_HIP(hipMemcpyAsync(f->d_values.get(), f->values.get(), sizeof(float) * N,
                               hipMemcpyHostToDevice, st));
    }
    MML_HIP(hipStreamSynchronize(st));
}

}  // namespace

using mml::guard;

extern "C" mml_status mml_rating_file_read_device(mml_ctx* ctx, const char* path, int32_t flags,
                                                  int32_t n_threads, const char* const* user_seed,
                                                  int32_t n_user_seed, const char* const* item_seed,
                                                  int32_t n_item_seed, mml_rating_file** out) {
    return guard([&] {
        MML_REQUIRE(ctx && path && out, "null argument");
        MML_REQUIRE(!ctx->multi(), "a single-device context");
        MML_REQUIRE(n_user_seed >= 0 && n_item_seed >= 0, "bad seed counts");
        ctx->activate();
        hipStream_t st = ctx->stream;
        const int T = std::max(1, std::min<int>(n_threads > 0 ? n_threads : 8, 64));
        const bool user_identity = flags & MML_READ_USER_IDENTITY;
        const bool item_identity = flags & MML_READ_ITEM_IDENTITY;
        auto host_path = [&]() {
            mml_rating_file* hf = nullptr;
            const mml_status s = mml_rating_file_read(path, flags, n_threads, user_seed,
                                                      n_user_seed, item_seed, n_item_seed, &hf);
            if (s != MML_OK) mml::fail(s, mml_last_error());
            std::unique_ptr<mml_rating_file> f(hf);
            f->ctx = ctx;
            upload(f.get(), st);
            *out = f.release();
        };
        // seeds of Mapping columns as canonical keys (else the host path)
        std::vector<int64_t> useed, iseed;
        bool seeds_ok = true;
        for (int32_t x = 0; x < n_user_seed && !user_identity && seeds_ok; ++x) {
            int64_t k = 0;
            seeds_ok = canonical_seed(user_seed[x], k);
            useed.push_back(k);
        }
        for (int32_t x = 0; x < n_item_seed && !item_identity && seeds_ok; ++x) {
            int64_t k = 0;
            seeds_ok = canonical_seed(item_seed[x], k);
            iseed.push_back(k);
        }
        if ((flags & (MML_READ_ITEM_DATA | MML_READ_BINARY_CACHE)) || !seeds_ok) return host_path();
        int64_t n = 0;
        uint8_t head[3] = {0, 0, 0};
        mml::DeviceArray<uint8_t> B;
        if (!upload_file(path, n, B, head, st)) return host_path();
        if (n >= INT32_MAX * (int64_t)kSeg) return host_path();
        const int64_t bom = n >= 3 && std::memcmp(head, "\xEF\xBB\xBF", 3) == 0 ? 3 : 0;
        const int skip_first = (flags & MML_READ_IGNORE_FIRST_LINE) ? 1 : 0;
        const int want = (flags & MML_READ_WITHOUT_RATINGS) ? 2 : 3;
        const int64_t nseg = std::max<int64_t>(1, (n + kSeg - 1) / kSeg);
        mml::DeviceArray<int64_t> lines, rows, at;
        lines.alloc(nseg);
        rows.alloc(nseg);
        at.alloc(nseg + 1);
        rf_count_kernel<<<grid_of(nseg), 256, 0, st>>>(B.get(), n, bom, skip_first, nseg,
                                                       lines.get(), rows.get());
        MML_HIP(hipGetLastError());
        MML_HIP(hipMemsetAsync(at.get(), 0, sizeof(int64_t), st));
        size_t tb = 0;
        MML_HIP(rocprim::inclusive_scan(nullptr, tb, rows.get(), at.get() + 1, nseg,
                rocprim::plus<int64_t>(), st));
        mml::DeviceArray<uint8_t> tmp;
        tmp.alloc(tb);
        MML_HIP(rocprim::inclusive_scan(tmp.get(), tb, rows.get(), at.get() + 1, nseg,
                rocprim::plus<int64_t>(), st));
        mml::DeviceArray<int64_t> nl_sum;
        nl_sum.alloc(1);
        size_t rb = 0;
        MML_HIP(rocprim::reduce(nullptr, rb, lines.get(), nl_sum.get(), (int64_t)0, nseg,
                rocprim::plus<int64_t>(), st));
        tmp.reserve(rb);
        MML_HIP(rocprim::reduce(tmp.get(), rb, lines.get(), nl_sum.get(), (int64_t)0, nseg,
                rocprim::plus<int64_t>(), st));
        int64_t counts[2] = {0, 0};
        MML_HIP(hipMemcpyAsync(&counts[0], nl_sum.get(), sizeof(int64_t), hipMemcpyDeviceToHost, st));
        MML_HIP(hipMemcpyAsync(&counts[1], at.get() + nseg, sizeof(int64_t), hipMemcpyDeviceToHost,
                               st));
        MML_HIP(hipStreamSynchronize(st));
        const int64_t N = counts[1];
        std::unique_ptr<mml_rating_file> f(new mml_rating_file());
        f->threads = T;
        f->ctx = ctx;
        f->n_lines = counts[0];
        f->n_ratings = N;
        f->d_users.alloc(std::max<int64_t>(1, N));
        f->d_items.alloc(std::max<int64_t>(1, N));
        f->d_values.alloc(std::max<int64_t>(1, N));
        mml::DeviceArray<int64_t> ukeys, ikeys;
        if (!user_identity) ukeys.alloc(std::max<int64_t>(1, N));
        if (!item_identity) ikeys.alloc(std::max<int64_t>(1, N));
        mml::DeviceArray<uint32_t> err;
        err.alloc(1);
        MML_HIP(hipMemsetAsync(err.get(), 0, sizeof(uint32_t), st));
        rf_parse_kernel<<<grid_of(nseg), 256, 0, st>>>(
            B.get(), n, bom, skip_first, nseg, at.get(), want, user_identity, item_identity,
            f->d_users.get(), f->d_items.get(), f->d_values.get(), ukeys.get(), ikeys.get(),
            err.get());
        MML_HIP(hipGetLastError());
        uint32_t e = 0;
        MML_HIP(hipMemcpyAsync(&e, err.get(), sizeof(uint32_t), hipMemcpyDeviceToHost, st));
        MML_HIP(hipStreamSynchronize(st));
        B.reset();
        if (e != 0) return host_path();  // the host reader gives the reference's error or result
        if (!user_identity) map_keys_device(st, ukeys.get(), N, useed, f->d_users.get(), f->new_users);
        if (!item_identity) map_keys_device(st, ikeys.get(), N, iseed, f->d_items.get(), f->new_items);
        MML_HIP(hipStreamSynchronize(st));
        f->device_parsed = 1;
        *out = f.release();
    });
}

extern "C" mml_status mml_rating_file_device_arrays(mml_rating_file* f, const int32_t** users,
                                                    const int32_t** items, const float** values,
                                                    int32_t* device_parsed) {
    return guard([&] {
        MML_REQUIRE(f && users && items && values && device_parsed, "null argument");
        MML_REQUIRE(f->ctx, "a host-only rating file (mml_rating_file_read)");
        *users = f->d_users.get();
        *items = f->d_items.get();
        *values = f->d_values.get();
        *device_parsed = f->device_parsed;
    });
}
