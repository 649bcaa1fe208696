// tests/rccl_standin/standin.cpp -- TEST INFRASTRUCTURE ONLY: a checking stand-in for the RCCL
// calls libmml_hip.so makes, so that the library's communicator branches (`if (c->comm)`) run with
// several ranks on ONE GPU.  tests/rccl_standin/Makefile links the library's
// own objects against this file instead of librccl (libmml_hip_standin.so); the product library is
// never linked to it.
//
// Every rank is a host thread of one process with its own mml_ctx (device 0 repeated).  The
// stand-in executes each call for real (the caller's stream drained, then the data copied on that
// stream and the stream drained again, so a call is complete when it returns) and CHECKS the call
// pattern a real communicator would only expose as a hang or a wrong result:
//   * collectives (ncclAllReduce, ncclBroadcast): every rank of the communicator issues the same
//     sequence, with equal op, datatype, count, reduction and root -- checked at each call;
//   * point-to-point (ncclSend / ncclRecv): the m-th send from a to b pairs with the m-th recv on b
//     from a, with equal datatype and count; a send nobody receives is reported at the end;
//   * calls between ncclGroupStart / ncclGroupEnd run at ncclGroupEnd, as RCCL runs them.
// ncclAvg sums in rank order then divides once (float), the arithmetic of the peer-copy average
// (peer.hip average_rows_kernel), so a communicator run can be compared bit for bit with the
// repeated-device run.  A wait longer than MML_STANDIN_TIMEOUT seconds (default 60) fails the
// call instead of hanging (the ranks' sequences differ).  mml_standin_report() returns the counts
// and every error as JSON.
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <chrono>
#include <condition_variable>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <deque>
#include <map>
#include <memory>
#include <mutex>
#include <string>
#include <vector>

namespace {

size_t type_size(ncclDataType_t t) {
    switch (t) {
        case ncclInt8: case ncclUint8: return 1;
        case ncclFloat16: case ncclBfloat16: return 2;
        case ncclInt32: case ncclUint32: case ncclFloat32: return 4;
        default: return 8;
    }
}

struct Op {
    enum Kind { kAllReduce, kBroadcast, kSend, kRecv } kind;
    const void* send = nullptr;
    void* recv = nullptr;
    size_t count = 0;
    ncclDataType_t dtype = ncclFloat;
    ncclRedOp_t redop = ncclSum;
    int peer = 0;  // root of a broadcast, peer of a send / recv
    hipStream_t stream = nullptr;
    struct ncclComm* comm = nullptr;
};

const char* kind_name(int k) {
    static const char* n[] = {"allreduce", "broadcast", "send", "recv"};
    return n[k];
}

struct Msg {  // a posted send, consumed by the matching recv
    const void* buf;
    size_t count;
    ncclDataType_t dtype;
    bool consumed = false;
};

double timeout_s() {
    const char* e = std::getenv("MML_STANDIN_TIMEOUT");
    return e ? std::atof(e) : 60.0;
}

struct Stats {
    std::mutex m;
    long groups = 0, allreduce = 0, broadcast = 0, send = 0, recv = 0, comms = 0, worlds = 0;
    long bytes = 0;
    std::vector<std::string> errors;
    std::map<std::string, long> by_op;  // "allreduce avg float n=..." -> calls
    void error(const std::string& e) {
        std::lock_guard<std::mutex> lk(m);
        if (errors.size() < 64) errors.push_back(e);
    }
};
Stats g_stats;

struct World {
    int n;
    std::mutex m;
    std::condition_variable cv;
    // collectives: a generation barrier and the posted op of every rank
    int arrived = 0;
    uint64_t gen = 0;
    bool broken = false;
    std::vector<Op> slot;
    std::vector<long> coll_seq;
    // point-to-point mailboxes, (from, to) -> posted sends in order
    std::map<std::pair<int, int>, std::deque<std::shared_ptr<Msg>>> mail;
    explicit World(int n_) : n(n_), slot(n_), coll_seq(n_, 0) {}

    // false on timeout or when another rank broke the world
    bool barrier(int rank, const char* what) {
        std::unique_lock<std::mutex> lk(m);
        if (broken) return false;
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
            return true;
        }
        const bool ok = cv.wait_for(lk, std::chrono::duration<double>(timeout_s()),
                                    [&] { return gen != g || broken; });
        if (!ok || gen == g) {
            if (!broken)
                g_stats.error("rank " + std::to_string(rank) + " waited " +
                              std::to_string(timeout_s()) + " s at a " + what +
                              ": the ranks' call sequences differ");
            broken = true;
            cv.notify_all();
            return false;
        }
        return true;
    }
};

struct Registry {
    std::mutex m;
    std::map<std::string, std::shared_ptr<World>> by_id;
    uint64_t next_id = 1;
};
Registry g_reg;

}  // namespace

struct ncclComm {
    std::shared_ptr<World> world;
    int rank = 0, device = 0;
};

namespace {

thread_local int t_depth = 0;
thread_local std::vector<Op> t_pending;

template <class T>
void reduce_into(T* acc, const T* x, size_t n, ncclRedOp_t op) {
    for (size_t i = 0; i < n; ++i) {
        switch (op) {
            case ncclSum: case ncclAvg: acc[i] = acc[i] + x[i]; break;
            case ncclProd: acc[i] = acc[i] * x[i]; break;
            case ncclMax: acc[i] = acc[i] < x[i] ? x[i] : acc[i]; break;
            default: acc[i] = x[i] < acc[i] ? x[i] : acc[i]; break;
        }
    }
}

template <class T>
void finish_avg(T* acc, size_t n, int ranks) {
    for (size_t i = 0; i < n; ++i) acc[i] = acc[i] / (T)ranks;
}

bool hip_ok(hipError_t e, const std::string& what) {
    if (e == hipSuccess) return true;
    g_stats.error(what + ": " + hipGetErrorString(e));
    return false;
}

// a copy complete on return: on the caller's stream, then that stream drained (a plain hipMemcpy
// of device to device memory may return before the copy lands, and the null stream does not
// order against the library's non-blocking streams)
hipError_t copy_sync(void* dst, const void* src, size_t bytes, hipStream_t st) {
    hipError_t e = hipMemcpyAsync(dst, src, bytes, hipMemcpyDefault, st);
    if (e != hipSuccess) return e;
    return hipStreamSynchronize(st);
}

std::string describe(const Op& o) {
    return std::string(kind_name(o.kind)) + " dtype=" + std::to_string((int)o.dtype) +
           " count=" + std::to_string(o.count) +
           (o.kind == Op::kAllReduce ? " redop=" + std::to_string((int)o.redop) : "") +
           (o.kind != Op::kAllReduce ? " peer/root=" + std::to_string(o.peer) : "");
}

// one collective on rank c->rank: post, check every rank posted the same call, read, write
ncclResult_t run_collective(const Op& o) {
    ncclComm* c = o.comm;
    World& w = *c->world;
    const int r = c->rank;
    const size_t bytes = o.count * type_size(o.dtype);
    {
        std::lock_guard<std::mutex> lk(w.m);
        w.slot[r] = o;
    }
    const long seq = w.coll_seq[r]++;
    if (!w.barrier(r, "collective")) return ncclInvalidUsage;
    for (int q = 0; q < w.n; ++q) {
        const Op& x = w.slot[q];
        if (x.kind != o.kind || x.dtype != o.dtype || x.count != o.count ||
            (o.kind == Op::kAllReduce && x.redop != o.redop) ||
            (o.kind == Op::kBroadcast && x.peer != o.peer)) {
            if (r == 0)
                g_stats.error("collective #" + std::to_string(seq) + ": rank 0 issued " +
                              describe(o) + ", rank " + std::to_string(q) + " issued " +
                              describe(x));
            w.barrier(r, "collective (mismatch)");
            return ncclInvalidUsage;
        }
    }
    std::vector<char> acc(bytes);
    bool ok = true;
    if (bytes > 0) {
        if (o.kind == Op::kBroadcast) {
            ok = hip_ok(copy_sync(acc.data(), w.slot[o.peer].send, bytes, o.stream),
                        "broadcast read");
        } else {
            std::vector<char> x(bytes);
            ok = hip_ok(copy_sync(acc.data(), w.slot[0].send, bytes, o.stream),
                        "allreduce read");
            for (int q = 1; q < w.n && ok; ++q) {
                ok = hip_ok(copy_sync(x.data(), w.slot[q].send, bytes, o.stream),
                            "allreduce read");
                switch (o.dtype) {
                    case ncclFloat32:
                        reduce_into((float*)acc.data(), (const float*)x.data(), o.count, o.redop);
                        break;
                    case ncclFloat64:
                        reduce_into((double*)acc.data(), (const double*)x.data(), o.count,
                                    o.redop);
                        break;
                    case ncclUint32:
                        reduce_into((uint32_t*)acc.data(), (const uint32_t*)x.data(), o.count,
                                    o.redop);
                        break;
                    case ncclInt32:
                        reduce_into((int32_t*)acc.data(), (const int32_t*)x.data(), o.count,
                                    o.redop);
                        break;
                    default: ok = false; g_stats.error("allreduce: datatype not covered");
                }
            }
            if (ok && o.redop == ncclAvg) {
                if (o.dtype == ncclFloat32) finish_avg((float*)acc.data(), o.count, w.n);
                else if (o.dtype == ncclFloat64) finish_avg((double*)acc.data(), o.count, w.n);
                else { ok = false; g_stats.error("ncclAvg on an integer datatype"); }
            }
        }
    }
    // every rank has read every input before any rank overwrites its own buffer (in place)
    if (!w.barrier(r, "collective (read phase)")) return ncclInvalidUsage;
    if (ok && bytes > 0)
        ok = hip_ok(copy_sync(o.recv, acc.data(), bytes, o.stream), "collective write");
    {
        std::lock_guard<std::mutex> lk(g_stats.m);
        (o.kind == Op::kAllReduce ? g_stats.allreduce : g_stats.broadcast)++;
        g_stats.bytes += (long)bytes;
        g_stats.by_op[std::string(kind_name(o.kind)) + " redop=" + std::to_string((int)o.redop) +
                      " dtype=" + std::to_string((int)o.dtype)]++;
    }
    return ok ? ncclSuccess : ncclSystemError;
}

ncclResult_t run_group(std::vector<Op>& ops) {
    if (ops.empty()) return ncclSuccess;
    ncclComm* c = ops[0].comm;
    for (const Op& o : ops)
        if (o.comm != c) {
            g_stats.error("one group spans communicators on one thread (not covered)");
            return ncclInvalidUsage;
        }
    World& w = *c->world;
    const int r = c->rank;
    {
        std::lock_guard<std::mutex> lk(g_stats.m);
        ++g_stats.groups;
    }
    // the inputs are complete: the caller's streams drained (RCCL would order on the stream)
    for (const Op& o : ops)
        if (!hip_ok(hipStreamSynchronize(o.stream), "stream sync")) return ncclSystemError;
    // point-to-point: post every send, take every recv, then wait until the sends are consumed
    std::vector<std::shared_ptr<Msg>> mine;
    {
        std::lock_guard<std::mutex> lk(w.m);
        for (const Op& o : ops)
            if (o.kind == Op::kSend) {
                auto m = std::make_shared<Msg>();
                m->buf = o.send;
                m->count = o.count;
                m->dtype = o.dtype;
                w.mail[{r, o.peer}].push_back(m);
                mine.push_back(m);
            }
        w.cv.notify_all();
    }
    ncclResult_t res = ncclSuccess;
    for (const Op& o : ops) {
        if (o.kind != Op::kRecv) continue;
        std::shared_ptr<Msg> m;
        {
            std::unique_lock<std::mutex> lk(w.m);
            auto& q = w.mail[{o.peer, r}];
            const bool got = w.cv.wait_for(lk, std::chrono::duration<double>(timeout_s()),
                                           [&] { return !q.empty() || w.broken; });
            if (!got || w.broken) {
                g_stats.error("rank " + std::to_string(r) + ": recv from " +
                              std::to_string(o.peer) + " (count " + std::to_string(o.count) +
                              ") has no matching send");
                w.broken = true;
                w.cv.notify_all();
                return ncclInvalidUsage;
            }
            m = q.front();
            q.pop_front();
        }
        if (m->count != o.count || m->dtype != o.dtype) {
            g_stats.error("rank " + std::to_string(r) + ": recv from " + std::to_string(o.peer) +
                          " expects " + std::to_string(o.count) + " elements of type " +
                          std::to_string((int)o.dtype) + ", the matching send has " +
                          std::to_string(m->count) + " of type " + std::to_string((int)m->dtype));
            res = ncclInvalidUsage;
        } else if (o.count > 0 &&
                   !hip_ok(copy_sync(o.recv, m->buf, o.count * type_size(o.dtype), o.stream),
                           "recv copy")) {
            res = ncclSystemError;
        }
        std::lock_guard<std::mutex> lk(w.m);
        m->consumed = true;
        w.cv.notify_all();
        std::lock_guard<std::mutex> ls(g_stats.m);
        ++g_stats.recv;
        g_stats.bytes += (long)(o.count * type_size(o.dtype));
    }
    {
        std::unique_lock<std::mutex> lk(w.m);
        for (auto& m : mine) {
            const bool done = w.cv.wait_for(lk, std::chrono::duration<double>(timeout_s()),
                                            [&] { return m->consumed || w.broken; });
            if (!done || !m->consumed) {
                g_stats.error("rank " + std::to_string(r) + ": a send of " +
                              std::to_string(m->count) + " elements was never received");
                w.broken = true;
                w.cv.notify_all();
                return ncclInvalidUsage;
            }
        }
        std::lock_guard<std::mutex> ls(g_stats.m);
        g_stats.send += (long)mine.size();
    }
    for (const Op& o : ops)
        if (o.kind == Op::kAllReduce || o.kind == Op::kBroadcast) {
            const ncclResult_t x = run_collective(o);
            if (x != ncclSuccess) return x;
        }
    return res;
}

ncclResult_t submit(const Op& o) {
    if (!o.comm) return ncclInvalidArgument;
    if (o.comm->world->broken) return ncclInvalidUsage;
    if (t_depth > 0) {
        t_pending.push_back(o);
        return ncclSuccess;
    }
    std::vector<Op> one{o};
    return run_group(one);
}

std::string json_escape(const std::string& s) {
    std::string o;
    for (char ch : s) {
        if (ch == '"' || ch == '\\') o += '\\';
        o += ch;
    }
    return o;
}

}  // namespace

extern "C" {

ncclResult_t ncclGetUniqueId(ncclUniqueId* id) {
    if (!id) return ncclInvalidArgument;
    std::memset(id, 0, sizeof(*id));
    std::lock_guard<std::mutex> lk(g_reg.m);
    std::snprintf(id->internal, sizeof(id->internal), "mml-rccl-standin-%llu",
                  (unsigned long long)g_reg.next_id++);
    return ncclSuccess;
}

ncclResult_t ncclCommInitRank(ncclComm_t* comm, int nranks, ncclUniqueId id, int rank) {
    if (!comm || nranks < 1 || rank < 0 || rank >= nranks) return ncclInvalidArgument;
    std::shared_ptr<World> w;
    {
        std::lock_guard<std::mutex> lk(g_reg.m);
        const std::string key(id.internal, strnlen(id.internal, sizeof(id.internal)));
        auto& slot = g_reg.by_id[key];
        if (!slot) {
            slot = std::make_shared<World>(nranks);
            std::lock_guard<std::mutex> ls(g_stats.m);
            ++g_stats.worlds;
        }
        w = slot;
    }
    if (w->n != nranks) {
        g_stats.error("ncclCommInitRank: nranks differ between ranks");
        return ncclInvalidUsage;
    }
    auto* c = new ncclComm();
    c->world = w;
    c->rank = rank;
    (void)hipGetDevice(&c->device);
    if (!w->barrier(rank, "ncclCommInitRank")) {
        delete c;
        return ncclInvalidUsage;
    }
    {
        std::lock_guard<std::mutex> ls(g_stats.m);
        ++g_stats.comms;
    }
    *comm = c;
    return ncclSuccess;
}

ncclResult_t ncclCommInitAll(ncclComm_t* comms, int ndev, const int* devlist) {
    if (!comms || ndev < 1) return ncclInvalidArgument;
    auto w = std::make_shared<World>(ndev);
    for (int d = 0; d < ndev; ++d) {
        auto* c = new ncclComm();
        c->world = w;
        c->rank = d;
        c->device = devlist ? devlist[d] : d;
        comms[d] = c;
    }
    std::lock_guard<std::mutex> ls(g_stats.m);
    ++g_stats.worlds;
    g_stats.comms += ndev;
    return ncclSuccess;
}

ncclResult_t ncclCommDestroy(ncclComm_t comm) {
    delete comm;
    return ncclSuccess;
}

const char* ncclGetErrorString(ncclResult_t r) {
    switch (r) {
        case ncclSuccess: return "no error (stand-in)";
        case ncclInvalidUsage: return "invalid usage (stand-in: see mml_standin_report)";
        case ncclInvalidArgument: return "invalid argument (stand-in)";
        default: return "system error (stand-in)";
    }
}

ncclResult_t ncclGroupStart() {
    ++t_depth;
    return ncclSuccess;
}

ncclResult_t ncclGroupEnd() {
    if (t_depth <= 0) return ncclInvalidUsage;
    if (--t_depth > 0) return ncclSuccess;
    std::vector<Op> ops;
    ops.swap(t_pending);
    return run_group(ops);
}

ncclResult_t ncclAllReduce(const void* sendbuff, void* recvbuff, size_t count,
                           ncclDataType_t datatype, ncclRedOp_t op, ncclComm_t comm,
                           hipStream_t stream) {
    Op o;
    o.kind = Op::kAllReduce;
    o.send = sendbuff;
    o.recv = recvbuff;
    o.count = count;
    o.dtype = datatype;
    o.redop = op;
    o.stream = stream;
    o.comm = comm;
    return submit(o);
}

ncclResult_t ncclBroadcast(const void* sendbuff, void* recvbuff, size_t count,
                           ncclDataType_t datatype, int root, ncclComm_t comm,
                           hipStream_t stream) {
    Op o;
    o.kind = Op::kBroadcast;
    o.send = sendbuff;
    o.recv = recvbuff;
    o.count = count;
    o.dtype = datatype;
    o.peer = root;
    o.stream = stream;
    o.comm = comm;
    return submit(o);
}

ncclResult_t ncclSend(const void* sendbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t comm, hipStream_t stream) {
    Op o;
    o.kind = Op::kSend;
    o.send = sendbuff;
    o.count = count;
    o.dtype = datatype;
    o.peer = peer;
    o.stream = stream;
    o.comm = comm;
    return submit(o);
}

ncclResult_t ncclRecv(void* recvbuff, size_t count, ncclDataType_t datatype, int peer,
                      ncclComm_t comm, hipStream_t stream) {
    Op o;
    o.kind = Op::kRecv;
    o.recv = recvbuff;
    o.count = count;
    o.dtype = datatype;
    o.peer = peer;
    o.stream = stream;
    o.comm = comm;
    return submit(o);
}

// {"worlds":..,"comms":..,"groups":..,"allreduce":..,"broadcast":..,"send":..,"recv":..,
//  "bytes":..,"unmatched_sends":..,"by_op":{..},"errors":[..]}
int mml_standin_report(char* buf, int cap) {
    long unmatched = 0;
    {
        std::lock_guard<std::mutex> lk(g_reg.m);
        for (auto& kv : g_reg.by_id) {
            std::lock_guard<std::mutex> lw(kv.second->m);
            for (auto& q : kv.second->mail) unmatched += (long)q.second.size();
        }
    }
    std::lock_guard<std::mutex> lk(g_stats.m);
    std::string s = "{\"worlds\":" + std::to_string(g_stats.worlds) +
                    ",\"comms\":" + std::to_string(g_stats.comms) +
                    ",\"groups\":" + std::to_string(g_stats.groups) +
                    ",\"allreduce\":" + std::to_string(g_stats.allreduce) +
                    ",\"broadcast\":" + std::to_string(g_stats.broadcast) +
                    ",\"send\":" + std::to_string(g_stats.send) +
                    ",\"recv\":" + std::to_string(g_stats.recv) +
                    ",\"bytes\":" + std::to_string(g_stats.bytes) +
                    ",\"unmatched_sends\":" + std::to_string(unmatched) + ",\"by_op\":{";
    bool first = true;
    for (auto& kv : g_stats.by_op) {
        s += (first ? "\"" : ",\"") + json_escape(kv.first) + "\":" + std::to_string(kv.second);
        first = false;
    }
    s += "},\"errors\":[";
    for (size_t i = 0; i < g_stats.errors.size(); ++i)
        s += (i ? ",\"" : "\"") + json_escape(g_stats.errors[i]) + "\"";
    s += "]}";
    if (buf && cap > 0) {
        const size_t n = std::min<size_t>(s.size(), (size_t)cap - 1);
        std::memcpy(buf, s.data(), n);
        buf[n] = 0;
    }
    return (int)s.size();
}

void mml_standin_reset(void) {
    std::lock_guard<std::mutex> lk(g_stats.m);
    g_stats.groups = g_stats.allreduce = g_stats.broadcast = g_stats.send = g_stats.recv = 0;
    g_stats.bytes = 0;
    g_stats.by_op.clear();
    g_stats.errors.clear();
}

}  // extern "C"
