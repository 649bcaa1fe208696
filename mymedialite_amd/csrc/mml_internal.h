// mml_internal.h -- shared plumbing of libmml_hip.so: status/exception bridge, device buffers,
// the context (one GPU, one HIP stream, optional RCCL communicator).
#pragma once

#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <algorithm>
#include <cstdint>
#include <cstdlib>
#include <exception>
#include <memory>
#include <new>
#include <string>
#include <thread>
#include <utility>
#include <vector>

#include "mml.h"

struct mml_ctx;

// Experiment switches (environment variables that select A/B variants of a kernel: MML_HOGWILD_XCD,
// MML_WRMF_DEBUG, ...) exist only in a library built with -DMML_EXPERIMENTS
// (scripts/build_variant.sh).  The release library never reads the environment: the macro drops
// the variable's name, so a stray setting on a user's machine cannot select a slower or a
// deliberately wrong path.
#ifdef MML_EXPERIMENTS
#define MML_EXPERIMENT_ENV(name) std::getenv(name)
#else
#define MML_EXPERIMENT_ENV(name) ((const char*)nullptr)
#endif

namespace mml {

struct Error : std::exception {
    mml_status code;
    std::string msg;
    Error(mml_status c, std::string m) : code(c), msg(std::move(m)) {}
    const char* what() const noexcept override { return msg.c_str(); }
};

void set_error(const std::string& msg);

// Runs f(); converts any exception into a status + thread-local message (never aborts the host).
template <class F>
mml_status guard(F&& f) {
    try {
        f();
        return MML_OK;
    } catch (const Error& e) {
        set_error(e.msg);
        return e.code;
    } catch (const std::bad_alloc&) {
        set_error("host allocation failed");
        return MML_ERR_OOM;
    } catch (const std::exception& e) {
        set_error(e.what());
        return MML_ERR_STATE;
    }
}

[[noreturn]] inline void fail(mml_status code, const std::string& msg) { throw Error(code, msg); }

inline void hip_check(hipError_t e, const char* what) {
    if (e == hipSuccess) return;
    (void)hipGetLastError();  // clear sticky launch error state where possible
    fail(e == hipErrorOutOfMemory ? MML_ERR_OOM : MML_ERR_HIP,
         std::string(what) + ": " + hipGetErrorString(e));
}
#define MML_HIP(call) ::mml::hip_check((call), #call)

inline void rccl_check(ncclResult_t r, const char* what) {
    if (r == ncclSuccess) return;
    fail(MML_ERR_RCCL, std::string(what) + ": " + ncclGetErrorString(r));
}
#define MML_RCCL(call) ::mml::rccl_check((call), #call)

#define MML_REQUIRE(cond, msg) \
    do {                       \
        if (!(cond)) ::mml::fail(MML_ERR_ARG, (msg)); \
    } while (0)

// Owning device allocation (HBM of the context's device).
template <class T>
struct DeviceArray {
    T* ptr = nullptr;
    size_t count = 0;
    DeviceArray() = default;
    DeviceArray(const DeviceArray&) = delete;
    DeviceArray& operator=(const DeviceArray&) = delete;
    ~DeviceArray() { reset(); }
    void reset() {
        if (ptr) (void)hipFree(ptr);
        ptr = nullptr;
        count = 0;
    }
    void alloc(size_t n) {
        if (n == count && ptr) return;
        reset();
        if (n == 0) return;
        MML_HIP(hipMalloc(reinterpret_cast<void**>(&ptr), n * sizeof(T)));
        count = n;
    }
    // at least n elements, keeping a larger block (buffers shared by passes of different sizes:
    // no free / malloc round trip per use)
    void reserve(size_t n) {
        if (n <= count && ptr) return;
        alloc(n);
    }
    T* get() const { return ptr; }
    void swap(DeviceArray& o) noexcept {
        std::swap(ptr, o.ptr);
        std::swap(count, o.count);
    }
};

// CSR of the distinct (row, col) pairs of an event list, rows sorted by col (csr.hip).
struct DeviceCsr {
    DeviceArray<int64_t> off;   // [n_rows + 1]
    DeviceArray<int32_t> cols;  // [nnz]
    int64_t nnz = 0;
    std::vector<int32_t> deg_host;  // distinct entries per row (host copy)
};
void build_csr_device(const int32_t* rows_device, const int32_t* cols_device, int64_t n,
                      int32_t n_rows, int32_t n_cols, hipStream_t st, DeviceCsr& out);

// Eval.Items AUC for an MF scorer (auc.hip): per-user AUC, NaN for users Items.Evaluate skips.
void item_auc(hipStream_t st, const float* U, int32_t ldu, int32_t n_users_model, const float* V,
              int32_t ldv, int32_t n_items_model, const float* bias, int32_t k,
              const int64_t* tr_off, const int32_t* tr_cols, int32_t n_tr_rows,
              const int32_t* candidates, int32_t n_cand, const int32_t* users, int32_t n_eval,
              const int64_t* test_off, const int32_t* test_items, double* out_auc);

// contiguous row shards with balanced work (weight deg + k/2), bounds[parts + 1] (mml_core.cpp)
std::vector<int64_t> balanced_rows(const std::vector<int64_t>& deg, int32_t k, int32_t parts);

// WRMF row solves on the matrix cores for 128 < k <= 256 (wrmf_tiles.hip): a per-CSR plan of
// light rows (degree-descending work list) and heavy rows (split Gram segments).
struct WrmfTilePlan {
    DeviceArray<int32_t> light, heavy_dev, counter;
    int32_t n_light = 0;
    std::vector<int32_t> heavy;
    std::vector<int64_t> seg_first;  // per heavy row: first segment (+ sentinel)
    DeviceArray<uint8_t> segs;
    DeviceArray<float> hht;
    DeviceArray<double> gram;
    // Woodbury rows (1 <= deg <= 128), by 32-column group of their degree
    DeviceArray<int32_t> wood[4];
    int32_t n_wood[4] = {0, 0, 0, 0};
    DeviceArray<float> linv, linvt, qbuf, tbuf;  // L^{-1}, L^{-T} of HH + reg I; Q = H L^{-T}; t rows
    DeviceArray<uint16_t> linv_x3, linvt_x3;    // their bf16 planes, transposed (row GEMMs)
    DeviceArray<float> sbuf;                      // refinement: s = L^{-1} r per Woodbury row
    DeviceArray<int32_t> crow, cpos, ccount;      // refinement: the rows the screen left, count
    int64_t screen_left = 0;  // refinement: Woodbury rows any pass left to the kernels (or unknown)
    // refinement: the handle's stream waits on this before the pass's x += d row update (the
    // speculative HH of the next half-step is still reading W; consumed by the first pass)
    hipEvent_t pre_update_wait = nullptr;
    // refinement: issued right after the first pass's dense term (the speculative HH, so that it
    // runs beside the memory-bound data term rather than the dense term's fp64 MFMAs)
    std::function<void(hipStream_t)> after_dense;
    double linv_norm = 0.0;                       // |L^{-1}|_2 (estimate, 1.25 margin)
    bool woodbury = false;                        // rows with 1 <= deg <= 128 take Woodbury
    // fp64 iterative refinement (wrmf_tile_refine): the residual's entry segments (rows with
    // several segments reduce their partials in order), x and r in fp64 for rows [r0, r1), the
    // residual / correction rows in fp32 (W-shaped)
    int64_t r0 = 0, r1 = 0;
    DeviceArray<uint8_t> rsegs, rmulti;
    int64_t n_rsegs = 0, n_rmulti = 0, n_rslots = 0;
    // fp64 mode: the direct rows keep their factor tiles (L_IJ, T_J = L_JJ^{-1}; light rows, then
    // heavy ones) so a refinement pass is two triangular solves (wrmf_tile_resolve_kernel).  Set
    // per half-step: false when the tiles do not fit the free HBM (the refinement then
    // refactors each row instead).
    bool keep_factor = false;
    bool refined = false;  // fp64 refinement passes follow the half-step's solve (wood main target)
    // the item half's pipeline (fp64 mode, no Woodbury rows in the plan): the light rows in nbatch
    // contiguous row ranges (the light list range-major, degree-descending within a range), so the
    // first refinement pass's residual of range b (X (HH + reg I), the data term, R -> Rf) runs on
    // `side` while the main solve of range b + 1 runs on the handle's stream
    int32_t nbatch = 1;
    std::vector<int32_t> b_light;                // nbatch + 1 light-list offsets
    std::vector<int64_t> b_row, b_seg, b_multi;  // nbatch + 1 local-row / rseg / rmulti offsets
    hipStream_t side = nullptr;
    std::vector<hipEvent_t> ev;
    bool residual_ready = false;  // pass 0's R and Rf were computed inside wrmf_tile_solve
    bool light_corr_ready = false;  // and the light rows' pass-0 corrections (df) too
    // HH = H^T H computed on `side` (half_step) while the hot rows' split Gram runs: the solve
    // waits on hh_done before the HH tiles (nullptr: HH is already on the stream)
    hipEvent_t hh_start = nullptr, hh_done = nullptr;
    bool hh_pending = false;
    // the refinement's buffers (factor tiles, x and r in fp64, residual / correction rows): only
    // needed inside one half-step, so both plans of a handle point at ONE workspace (ws)
    struct Refine {
        DeviceArray<double> rpartial, x64, r64;
        DeviceArray<float> rf, df, factor;
        // the direct rows' Gram vectors split once per half-step into three bf16 planes
        // (wrmf_split_planes_kernel), of the H planes_of points at (h_rows + 1 rows)
        DeviceArray<uint16_t> planes;
        const float* planes_of = nullptr;
        // the last pass's largest relative correction (float bits): [0] direct rows, [1] Woodbury
        DeviceArray<unsigned> dmax;
    };
    Refine own;
    Refine* ws = &own;
    WrmfTilePlan() = default;
    WrmfTilePlan(const WrmfTilePlan&) = delete;
    WrmfTilePlan& operator=(const WrmfTilePlan&) = delete;
    ~WrmfTilePlan();
};
// pipe: the item half's pipeline ranges (0: the library's default, 1: off)
void wrmf_tile_plan(const std::vector<int64_t>& deg, hipStream_t st, WrmfTilePlan& p, int64_t r0,
                    int64_t r1, bool woodbury, int32_t pipe = 0);  // rows [r0, r1) of this rank
// the plan's second stream (created on first use), or nullptr when `st` is not on the current
// device (a multi-device context's rank: no second stream)
hipStream_t wrmf_plan_side(WrmfTilePlan& p, hipStream_t st);
// rhs == nullptr: W rows <- A^{-1} b (fp32).  rhs (W-shaped, fp32): W rows <- A^{-1} rhs rows,
// reusing the tables the preceding plain call of the same half-step built.
void wrmf_tile_solve(hipStream_t st, WrmfTilePlan& p, float* W, const float* H, int64_t h_rows,
                     const int64_t* off, const int32_t* cols, const double* HH, int32_t k,
                     double alpha, double reg, int& launches, const float* rhs = nullptr);
// after wrmf_tile_solve: up to `passes` rounds of x += A^{-1}(b - A x) with the residual in fp64
// (exact float products, double sums) and the correction from the fp32 solver, so W rows [r0, r1)
// reach the accuracy of the reference's fp64 solve (WRMF.cs:137-154); a further round runs only
// while the last correction exceeded 1e-4 relative.  Returns the rounds run.
// sync (nullable): the context whose ranks (communicator or peer group) each solve a row shard;
// the decision to run another pass is then taken on the max over the ranks, so every rank runs the
// same passes (a rank without rows still calls, to join the decisions).
int32_t wrmf_tile_refine(hipStream_t st, WrmfTilePlan& p, float* W, const float* H,
                         int64_t h_rows, const int64_t* off, const int32_t* cols, const double* HH,
                         int32_t k, double alpha, double reg, int32_t passes, int& launches,
                         float* corrections = nullptr,  // [4]: each pass's max correction
                         const mml_ctx* sync = nullptr);

// XCD-owned item groups (xcd.hip): items dealt into 8 groups of equal weight, a stream partitioned
// (stable) by the group of its item; group g's span goff[g] .. goff[g + 1] is served by blocks
// b % 8 == g, which share one XCD and therefore one L2.
struct XcdSplit {
    int32_t ng = 1, n_items = 0;
    DeviceArray<uint8_t> group;  // [n_items]
    DeviceArray<int64_t> goff;   // [9], device
    DeviceArray<int64_t> cnt, base;
    DeviceArray<uint8_t> tmp;
    void set_groups(hipStream_t st, const std::vector<int64_t>& weight, int32_t groups);
    // an explicit group per key (< 8), e.g. the device that owns a user (multi-device set_data)
    void set_table(hipStream_t st, const std::vector<uint8_t>& table);
    // out[c][...] = in[c][...] reordered by group(key[x]), stable; the 9 group offsets written on
    // the device into goff_out (nullptr: goff)
    void partition(hipStream_t st, const int32_t* key, int64_t n, int32_t npay,
                   const int32_t* const* in, int32_t* const* out, int64_t* goff_out = nullptr);
    // the same with each entry's group given as a byte (gkey[x] = group[key[x]], e.g. written by
    // the BPR sampler beside its triple): no table lookups in the count and scatter passes
    void partition_groups(hipStream_t st, const uint8_t* gkey, int64_t n, int32_t npay,
                          const int32_t* const* in, int32_t* const* out,
                          int64_t* goff_out = nullptr);
};
std::vector<uint8_t> balanced_item_groups(const std::vector<int64_t>& weight, int32_t ng);
// occurrences of each id in [0, n_ids) of a device id array, on the host
std::vector<int64_t> device_id_counts(hipStream_t st, const int32_t* ids, int64_t n,
                                      int32_t n_ids);

}  // namespace mml

struct mml_ctx;
namespace mml {
// Collectives of a context that lists a device more than once (peer.hip).  peer_average: arrays
// arr[d][a] of shard d (on ctxs[d]), count[a] floats each, replaced on every shard by their
// average over the shards (sum in shard order, then / N), staged on shard 0's device; ev0 / ev1
// bracket it on shard 0's stream and every other shard's stream waits on ev1.
void peer_average(const std::vector<mml_ctx*>& ctxs, const std::vector<std::vector<float*>>& arr,
                  const std::vector<int64_t>& count, DeviceArray<float>& stage, hipEvent_t ev0,
                  hipEvent_t ev1);
// The ranks of such a context when each runs on a host thread of its own (mml::on_devices): host
// barriers in place of a communicator.
struct PeerGroup {
    int32_t n;
    std::vector<int32_t> devices;  // device of each rank
    explicit PeerGroup(int32_t n);
    ~PeerGroup();
    PeerGroup(const PeerGroup&) = delete;
    PeerGroup& operator=(const PeerGroup&) = delete;
    // throws when a rank aborted (its call failed): the others then leave instead of waiting
    void barrier();
    void abort();  // by a failing rank
    void reset();  // before the ranks start a call (no rank inside the group)
    // every rank's rows [bounds[r], bounds[r + 1]) of W [rows x k] copied into every other rank's
    // W (W = the same matrix of each rank's handle); called by all ranks
    void allgather_rows(const mml_ctx* ctx, float* W, const std::vector<int64_t>& bounds,
                        int32_t k);
    // v[0 .. m) <- max over the ranks (m <= 4); called by all ranks
    void max_u32(const mml_ctx* ctx, uint32_t* v, int32_t m);
    // pointer slot (0 .. 3) of this rank, read by the others after the next barrier
    void publish(const mml_ctx* ctx, int32_t slot, void* p);
    void* peer(int32_t rank, int32_t slot) const { return ptr[(size_t)rank * 4 + slot]; }

  private:
    struct Impl;
    Impl* impl;
    std::vector<void*> ptr;
    std::vector<uint32_t> u32;
};

// Hogwild flushing waves per XCD: wave 0 of that many evenly spaced blocks of an XCD group writes
// the L2's dirty lines back after each batch of 64 updates (MML_FLUSHERS overrides the kernel's
// default: BiasedMF 1, BPR 4 -- measured in DESIGN.md)
int32_t flushers_per_xcd(int32_t dflt);
// 8 when blocks b and b + 8 run on one XCD for every b of a 2,048-block grid (probed once per
// context on the device; MML_XCD_GROUPS=1 forces 1), else 1
int32_t xcd_groups(mml_ctx* ctx);
}  // namespace mml

struct mml_ctx {
    // multi-device context (mml_ctx_create_multi): one single-device sub-context per GPU, each
    // holding rank d of one ncclCommInitAll communicator; the fields below are sub[0]'s copies
    std::vector<mml_ctx*> sub;
    bool multi() const { return !sub.empty(); }
    // a device id listed more than once (several shards on one GPU): no communicator is built;
    // the handles move data with peer copies instead (BiasedMF's DSGD ring; the BiasedMF / BPRMF
    // user shards' item averaging, mml::peer_average; WRMF's row all-gather through `peers`)
    bool repeated = false;
    // a repeated context's ranks (owned by the parent, shared by its sub-contexts): sub-context d
    // is rank peer_rank = d of `peers`
    std::shared_ptr<mml::PeerGroup> peers;
    int32_t peer_rank = 0;
    int32_t device = 0;
    hipStream_t stream = nullptr;
    ncclComm_t comm = nullptr;
    int32_t nranks = 1;
    int32_t rank = 0;
    int32_t xcd_groups = 0;  // mml::xcd_groups, 0 = not probed yet
    hipEvent_t ev_begin = nullptr, ev_end = nullptr, ev_mid = nullptr;
    void activate() const { MML_HIP(hipSetDevice(device)); }
};

// A parsed rating file (ratings_file.cpp; ratings_device.hip parses on the device): host arrays,
// or (device_parsed / uploaded) arrays in `ctx`'s HBM with the host copies made on demand
struct mml_rating_file {
    int64_t n_lines = 0;    // StaticRatings size (lines after the skipped first one)
    int64_t n_ratings = 0;  // non-empty lines
    std::unique_ptr<int32_t[]> users, items;
    std::unique_ptr<float[]> values;
    std::vector<std::string> new_users, new_items;  // ids the mapping did not hold, in order
    int32_t threads = 8;                            // the reader's thread count (copies, cache)
    mml_ctx* ctx = nullptr;                         // set: the arrays live in this context's HBM
    mml::DeviceArray<int32_t> d_users, d_items;
    mml::DeviceArray<float> d_values;
    int32_t device_parsed = 0;  // 1: parsed on the device; 0: host parse (then uploaded if ctx)
};

namespace mml {
// Runs f(d) -> mml_status for every device d of a multi-device context, each on a host thread of
// its own (rank d drives its device and its communicator rank, so collectives inside f meet),
// and turns the first failure into an exception carrying that thread's message.
template <class F>
void on_devices(const mml_ctx* ctx, F&& f) {
    const size_t n = ctx->sub.size();
    std::vector<mml_status> st(n, MML_OK);
    std::vector<std::string> msg(n);
    std::vector<std::thread> th;
    th.reserve(n);
    for (size_t d = 0; d < n; ++d)
        th.emplace_back([&, d] {
            st[d] = f((int32_t)d);
            if (st[d] != MML_OK) msg[d] = mml_last_error();
        });
    for (auto& t : th) t.join();
    for (size_t d = 0; d < n; ++d)
        if (st[d] != MML_OK)
            fail(st[d], "device " + std::to_string(ctx->sub[d]->device) + ": " + msg[d]);
}

// contiguous user ranges [b[d], b[d + 1]) with balanced rating counts (the multi-device shards;
// distributed.balanced_user_shards's rule)
std::vector<int32_t> balanced_user_bounds(const int32_t* users, int64_t n, int32_t n_users,
                                          int32_t parts);
// the same from per-user rating counts (n = their sum)
std::vector<int32_t> balanced_user_bounds_counts(const std::vector<int64_t>& count, int64_t n,
                                                 int32_t parts);
inline int32_t owner_of(const std::vector<int32_t>& b, int32_t u) {
    int32_t d = (int32_t)(std::upper_bound(b.begin(), b.end(), u) - b.begin()) - 1;
    return d < 0 ? 0 : (d >= (int32_t)b.size() - 1 ? (int32_t)b.size() - 2 : d);
}
}  // namespace mml
