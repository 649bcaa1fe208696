// mml_core.cpp -- library-level entry points: errors, devices, contexts, RCCL communicators,
// and the host-side MyMediaLite.Random / Utils.Shuffle / MultiCore equivalents that a non-.NET
// host needs to drive the path with the reference's RNG semantics.
#include <algorithm>
#include <cmath>
#include <cstring>
#include <numeric>
#include <vector>

#include "mml_internal.h"

namespace mml {
static thread_local std::string g_last_error;
void set_error(const std::string& msg) { g_last_error = msg; }
}  // namespace mml

using mml::guard;

extern "C" int mml_abi_version(void) { return MML_ABI_VERSION; }

extern "C" const char* mml_last_error(void) { return mml::g_last_error.c_str(); }

extern "C" mml_status mml_device_count(int32_t* out) {
    return guard([&] {
        MML_REQUIRE(out, "out is null");
        int n = 0;
        hipError_t e = hipGetDeviceCount(&n);
        if (e != hipSuccess) n = 0;
        *out = n;
    });
}

extern "C" mml_status mml_ctx_create(int32_t device_id, mml_ctx** out) {
    return guard([&] {
        MML_REQUIRE(out, "out is null");
        int n = 0;
        if (hipGetDeviceCount(&n) != hipSuccess || n == 0)
            mml::fail(MML_ERR_NODEV, "no HIP device visible");
        MML_REQUIRE(device_id >= 0 && device_id < n, "device_id out of range");
        hipDeviceProp_t prop;
        MML_HIP(hipGetDeviceProperties(&prop, device_id));
        if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
            mml::fail(MML_ERR_NODEV, std::string("libmml_hip is built for gfx950, device is ") +
                                         prop.gcnArchName);
        auto* ctx = new mml_ctx();
        ctx->device = device_id;
        try {
            ctx->activate();
            MML_HIP(hipStreamCreateWithFlags(&ctx->stream, hipStreamNonBlocking));
            MML_HIP(hipEventCreate(&ctx->ev_begin));
            MML_HIP(hipEventCreate(&ctx->ev_end));
            MML_HIP(hipEventCreate(&ctx->ev_mid));
        } catch (...) {
            delete ctx;
            throw;
        }
        *out = ctx;
    });
}

extern "C" mml_status mml_ctx_create_multi(const int32_t* device_ids, int32_t n_devices,
                                           mml_ctx** out) {
    return guard([&] {
        MML_REQUIRE(out && device_ids && n_devices >= 1, "need >= 1 device id");
        bool repeated = false;
        for (int32_t a = 0; a < n_devices; ++a)
            for (int32_t b = a + 1; b < n_devices; ++b) repeated |= device_ids[a] == device_ids[b];
        auto* ctx = new mml_ctx();
        ctx->repeated = repeated;
        try {
            for (int32_t d = 0; d < n_devices; ++d) {
                mml_ctx* s = nullptr;
                const mml_status st = mml_ctx_create(device_ids[d], &s);
                if (st != MML_OK) mml::fail(st, mml_last_error());
                ctx->sub.push_back(s);
            }
            // one communicator over the devices, driven from this process (no unique-id exchange);
            // a repeated device: host barriers between the shards' threads instead (peer.hip)
            if (repeated) {
                auto g = std::make_shared<mml::PeerGroup>(n_devices);
                g->devices.assign(device_ids, device_ids + n_devices);
                for (int32_t d = 0; d < n_devices; ++d) {
                    ctx->sub[d]->peers = g;
                    ctx->sub[d]->peer_rank = d;
                }
            } else {
                std::vector<ncclComm_t> comms(n_devices);
                MML_RCCL(ncclCommInitAll(comms.data(), n_devices, device_ids));
                for (int32_t d = 0; d < n_devices; ++d) {
                    ctx->sub[d]->comm = comms[d];
                    ctx->sub[d]->nranks = n_devices;
                    ctx->sub[d]->rank = d;
                }
            }
            ctx->device = ctx->sub[0]->device;
            ctx->stream = ctx->sub[0]->stream;
            ctx->nranks = n_devices;
        } catch (...) {
            for (mml_ctx* s : ctx->sub) mml_ctx_destroy(s);
            delete ctx;
            throw;
        }
        *out = ctx;
    });
}

extern "C" mml_status mml_ctx_destroy(mml_ctx* ctx) {
    return guard([&] {
        if (!ctx) return;
        if (ctx->multi()) {
            for (mml_ctx* s : ctx->sub) mml_ctx_destroy(s);
            delete ctx;
            return;
        }
        (void)hipSetDevice(ctx->device);
        if (ctx->comm) (void)ncclCommDestroy(ctx->comm);
        if (ctx->ev_begin) (void)hipEventDestroy(ctx->ev_begin);
        if (ctx->ev_end) (void)hipEventDestroy(ctx->ev_end);
        if (ctx->ev_mid) (void)hipEventDestroy(ctx->ev_mid);
        if (ctx->stream) (void)hipStreamDestroy(ctx->stream);
        delete ctx;
    });
}

namespace mml {
std::vector<int32_t> balanced_user_bounds_counts(const std::vector<int64_t>& count, int64_t n,
                                                 int32_t parts) {
    const int32_t n_users = (int32_t)count.size();
    std::vector<int64_t> c((size_t)n_users + 1, 0);
    for (int32_t u = 0; u < n_users; ++u) c[u + 1] = c[u] + count[u];  // c[u] = ratings of users < u
    std::vector<int32_t> b(parts + 1, n_users);
    b[0] = 0;
    for (int32_t r = 1; r < parts; ++r) {
        // first user boundary whose prefix reaches r/parts of the ratings
        const double target = (double)n * r / parts;
        b[r] = (int32_t)(std::lower_bound(c.begin(), c.end(), (int64_t)std::ceil(target)) -
                         c.begin());
        b[r] = std::min(std::max(b[r], b[r - 1]), n_users);
    }
    return b;
}

std::vector<int32_t> balanced_user_bounds(const int32_t* users, int64_t n, int32_t n_users,
                                          int32_t parts) {
    std::vector<int64_t> c((size_t)n_users, 0);
    for (int64_t x = 0; x < n; ++x) c[(size_t)users[x]]++;
    return balanced_user_bounds_counts(c, n, parts);
}
}  // namespace mml

extern "C" mml_status mml_comm_unique_id(uint8_t out_id[128]) {
    return guard([&] {
        MML_REQUIRE(out_id, "out_id is null");
        static_assert(sizeof(ncclUniqueId) == 128, "ncclUniqueId size");
        ncclUniqueId id;
        MML_RCCL(ncclGetUniqueId(&id));
        std::memcpy(out_id, &id, 128);
    });
}

extern "C" mml_status mml_ctx_comm_init(mml_ctx* ctx, const uint8_t id[128], int32_t nranks,
                                        int32_t rank) {
    return guard([&] {
        MML_REQUIRE(ctx && id, "null argument");
        MML_REQUIRE(nranks >= 1 && rank >= 0 && rank < nranks, "bad rank/nranks");
        ctx->activate();
        if (ctx->comm) {
            (void)ncclCommDestroy(ctx->comm);
            ctx->comm = nullptr;
        }
        ncclUniqueId uid;
        std::memcpy(&uid, id, 128);
        MML_RCCL(ncclCommInitRank(&ctx->comm, nranks, uid, rank));
        ctx->nranks = nranks;
        ctx->rank = rank;
    });
}

// --------------------------------------------------------------------------------------------
// System.Random(int) -- Knuth subtractive generator of the .NET reference source, as used through
// MyMediaLite.Random (src/MyMediaLite/Random.cs:23-64).
struct mml_random {
    int32_t seeds[56];
    int32_t inext = 0, inextp = 21;

    explicit mml_random(int32_t seed) {
        constexpr int32_t kBig = 2147483647, kSeed = 161803398;
        const int32_t sub = seed == INT32_MIN ? INT32_MAX : std::abs(seed);
        int32_t mj = kSeed - sub, mk = 1;
        seeds[55] = mj;
        for (int i = 1; i < 55; ++i) {
            const int ii = (21 * i) % 55;
            seeds[ii] = mk;
            mk = mj - mk;
            if (mk < 0) mk += kBig;
            mj = seeds[ii];
        }
        for (int pass = 0; pass < 4; ++pass)
            for (int i = 1; i < 56; ++i) {
                seeds[i] -= seeds[1 + (i + 30) % 55];
                if (seeds[i] < 0) seeds[i] += kBig;
            }
        seeds[0] = 0;
    }
    int32_t sample_int() {
        constexpr int32_t kBig = 2147483647;
        if (++inext >= 56) inext = 1;
        if (++inextp >= 56) inextp = 1;
        int32_t v = seeds[inext] - seeds[inextp];
        if (v == kBig) --v;
        if (v < 0) v += kBig;
        seeds[inext] = v;
        return v;
    }
    double next_double() { return sample_int() * (1.0 / 2147483647.0); }
    int32_t next(int32_t max_value) { return static_cast<int32_t>(next_double() * max_value); }
    // MathNet.Numerics 3.15 Normal.SampleUnchecked: polar transform, first variate returned.
    double normal(double mean, double stddev) {
        for (;;) {
            const double v1 = 2.0 * next_double() - 1.0;
            const double v2 = 2.0 * next_double() - 1.0;
            const double r = v1 * v1 + v2 * v2;
            if (r >= 1.0 || r == 0.0) continue;
            return mean + stddev * (v1 * std::sqrt(-2.0 * std::log(r) / r));
        }
    }
    void shuffle(int32_t* a, int64_t n) {
        for (int64_t i = n - 1; i >= 0; --i) {
            const int32_t j = next(static_cast<int32_t>(i + 1));
            std::swap(a[i], a[j]);
        }
    }
};

extern "C" mml_status mml_random_create(int32_t seed, mml_random** out) {
    return guard([&] {
        MML_REQUIRE(out, "out is null");
        *out = new mml_random(seed);
    });
}

extern "C" mml_status mml_random_destroy(mml_random* r) {
    return guard([&] { delete r; });
}

extern "C" mml_status mml_random_next(mml_random* r, int32_t max_value, int32_t* out) {
    return guard([&] {
        MML_REQUIRE(r && out, "null argument");
        MML_REQUIRE(max_value >= 0, "max_value must be >= 0");
        *out = r->next(max_value);
    });
}

extern "C" mml_status mml_random_next_double(mml_random* r, double* out) {
    return guard([&] {
        MML_REQUIRE(r && out, "null argument");
        *out = r->next_double();
    });
}

extern "C" mml_status mml_random_fill_normal(mml_random* r, double mean, double stddev,
                                             float* out, int64_t n) {
    return guard([&] {
        MML_REQUIRE(r && (out || n == 0) && n >= 0, "bad argument");
        for (int64_t i = 0; i < n; ++i) out[i] = static_cast<float>(r->normal(mean, stddev));
    });
}

extern "C" mml_status mml_random_shuffle_i32(mml_random* r, int32_t* a, int64_t n) {
    return guard([&] {
        MML_REQUIRE(r && (a || n == 0) && n >= 0 && n <= INT32_MAX, "bad argument");
        r->shuffle(a, n);
    });
}

extern "C" mml_status mml_partition_users_and_items(mml_random* r, const int32_t* users,
                                                    const int32_t* items, int64_t n,
                                                    int32_t max_user_id, int32_t max_item_id,
                                                    int32_t num_groups, int64_t* offsets,
                                                    int32_t* indices, int32_t* out_groups) {
    return guard([&] {
        MML_REQUIRE(r && offsets && out_groups && (n == 0 || (users && items && indices)),
                    "null argument");
        MML_REQUIRE(num_groups >= 1 && max_user_id >= 0 && max_item_id >= 0, "bad sizes");
        int32_t G = std::min(num_groups, max_user_id + 1);
        G = std::min(G, max_item_id + 1);
        std::vector<int32_t> up(max_user_id + 1), ip(max_item_id + 1);
        std::iota(up.begin(), up.end(), 0);
        std::iota(ip.begin(), ip.end(), 0);
        r->shuffle(up.data(), static_cast<int64_t>(up.size()));
        r->shuffle(ip.data(), static_cast<int64_t>(ip.size()));
        const int64_t nb = static_cast<int64_t>(G) * G;
        std::vector<int64_t> cnt(nb + 1, 0);
        std::vector<int32_t> blk(n);
        for (int64_t x = 0; x < n; ++x) {
            MML_REQUIRE(users[x] >= 0 && users[x] <= max_user_id && items[x] >= 0 &&
                            items[x] <= max_item_id,
                        "rating id out of range");
            blk[x] = static_cast<int32_t>((up[users[x]] % G) * G + ip[items[x]] % G);
            ++cnt[blk[x] + 1];
        }
        for (int64_t b = 0; b < nb; ++b) cnt[b + 1] += cnt[b];
        std::vector<int64_t> fill(cnt.begin(), cnt.end() - 1);
        for (int64_t x = 0; x < n; ++x) indices[fill[blk[x]]++] = static_cast<int32_t>(x);
        for (int64_t b = 0; b < nb; ++b) r->shuffle(indices + cnt[b], cnt[b + 1] - cnt[b]);
        std::memcpy(offsets, cnt.data(), sizeof(int64_t) * (nb + 1));
        *out_groups = G;
    });
}

namespace mml {
std::vector<int64_t> balanced_rows(const std::vector<int64_t>& deg, int32_t k, int32_t parts) {
    const int64_t n = (int64_t)deg.size();
    std::vector<int64_t> b(parts + 1, n);
    b[0] = 0;
    double total = 0.0;
    for (int64_t r = 0; r < n; ++r) total += (double)deg[r] + 0.5 * k;
    double acc = 0.0;
    int part = 1;
    for (int64_t r = 0; r < n && part < parts; ++r) {
        acc += (double)deg[r] + 0.5 * k;
        while (part < parts && acc >= total * part / parts) b[part++] = r + 1;
    }
    for (int p = 1; p <= parts; ++p) b[p] = std::max(b[p], b[p - 1]);
    return b;
}
}  // namespace mml

extern "C" mml_status mml_balanced_rows(const int64_t* deg, int64_t n, int32_t k, int32_t parts,
                                        int64_t* bounds) {
    return guard([&] {
        MML_REQUIRE(bounds && parts >= 1 && n >= 0 && (deg || n == 0), "bad argument");
        const auto b = mml::balanced_rows(std::vector<int64_t>(deg, deg + n), k, parts);
        std::memcpy(bounds, b.data(), sizeof(int64_t) * (parts + 1));
    });
}
