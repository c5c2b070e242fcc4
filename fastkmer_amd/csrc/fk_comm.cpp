// fk_comm.cpp -- transports of the bin exchange (see fk_comm.h).
#include "fk_comm.h"

#include <dlfcn.h>
#include <rccl/rccl.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <sched.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <condition_variable>
#include <memory>
#include <mutex>
#include <vector>

namespace fk {

namespace {

std::string hip_msg(const char *what, hipError_t e) {
    (void)hipGetLastError();
    return std::string(what) + ": " + hipGetErrorString(e);
}

// dst[i] = src[i]: the small collectives' staging copies between pinned (mapped) host memory and the
// device, as kernels on the collective's stream -- a small hipMemcpyAsync may be carried out by the
// host once the stream has drained, which would block the host outside the bounded wait
__global__ void k_comm_copy_u64(uint64_t *__restrict__ dst, const uint64_t *__restrict__ src, size_t n) {
    const size_t i = (size_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) dst[i] = src[i];
}

hipError_t comm_copy(uint64_t *dst, const uint64_t *src, size_t n, hipStream_t s) {
    if (!n) return hipSuccess;
    k_comm_copy_u64<<<(unsigned)((n + 255) / 256), 256, 0, s>>>(dst, src, n);
    return hipGetLastError();
}

#define COMM_HIP(expr)                                \
    do {                                              \
        hipError_t e_ = (expr);                       \
        if (e_ != hipSuccess) {                       \
            err = hip_msg(#expr, e_);                 \
            return -1;                                \
        }                                             \
    } while (0)

// ---------------------------------------------------------------------------
// RCCL, resolved at run time
// ---------------------------------------------------------------------------

struct RcclApi {
    void *handle = nullptr;
    std::string path;
    ncclResult_t (*GetUniqueId)(ncclUniqueId *) = nullptr;
    ncclResult_t (*CommInitRank)(ncclComm_t *, int, ncclUniqueId, int) = nullptr;
    ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
    ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;
    ncclResult_t (*CommSplit)(ncclComm_t, int, int, ncclComm_t *, ncclConfig_t *) = nullptr;
    ncclResult_t (*GroupStart)() = nullptr;
    ncclResult_t (*GroupEnd)() = nullptr;
    ncclResult_t (*Send)(const void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*Recv)(void *, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
    ncclResult_t (*AllReduce)(const void *, void *, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t,
                              hipStream_t) = nullptr;
    const char *(*GetErrorString)(ncclResult_t) = nullptr;
    ncclResult_t (*GetAsyncError)(ncclComm_t, ncclResult_t *) = nullptr;  // optional
};

std::mutex g_rccl_mu;
RcclApi g_rccl;
bool g_rccl_tried = false;
std::string g_rccl_err;

// The RCCL already mapped into the process first (torch's, bound to the same
// HIP runtime as this library), then the system one.
const RcclApi *rccl(std::string &err) {
    std::lock_guard<std::mutex> lk(g_rccl_mu);
    if (!g_rccl_tried) {
        g_rccl_tried = true;
        std::vector<std::pair<const char *, int>> tries;
        const char *env = getenv("FASTKMER_RCCL_LIB");
        if (env && env[0]) tries.push_back({env, RTLD_NOW | RTLD_LOCAL});
        tries.push_back({"librccl.so.1", RTLD_NOW | RTLD_NOLOAD});
        tries.push_back({"librccl.so", RTLD_NOW | RTLD_NOLOAD});
        tries.push_back({"librccl.so.1", RTLD_NOW | RTLD_LOCAL});
        tries.push_back({"/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_LOCAL});
        for (auto &t : tries) {
            void *h = dlopen(t.first, t.second);
            if (!h) continue;
            RcclApi a;
            a.handle = h;
            a.path = t.first;
#define SYM(field, name) a.field = reinterpret_cast<decltype(a.field)>(dlsym(h, name))
            SYM(GetUniqueId, "ncclGetUniqueId");
            SYM(CommInitRank, "ncclCommInitRank");
            SYM(CommDestroy, "ncclCommDestroy");
            SYM(CommAbort, "ncclCommAbort");
            SYM(CommSplit, "ncclCommSplit");
            SYM(GroupStart, "ncclGroupStart");
            SYM(GroupEnd, "ncclGroupEnd");
            SYM(Send, "ncclSend");
            SYM(Recv, "ncclRecv");
            SYM(AllReduce, "ncclAllReduce");
            SYM(GetErrorString, "ncclGetErrorString");
            SYM(GetAsyncError, "ncclCommGetAsyncError");
#undef SYM
            if (a.GetUniqueId && a.CommInitRank && a.CommDestroy && a.GroupStart && a.GroupEnd && a.Send && a.Recv &&
                a.AllReduce && a.GetErrorString) {
                Dl_info info;
                if (dladdr(reinterpret_cast<void *>(a.GetUniqueId), &info) && info.dli_fname) a.path = info.dli_fname;
                g_rccl = a;
                break;
            }
            g_rccl_err = std::string(t.first) + " lacks the RCCL entry points";
        }
        if (!g_rccl.handle && g_rccl_err.empty()) g_rccl_err = "librccl.so.1 could not be loaded";
    }
    if (!g_rccl.handle) {
        err = g_rccl_err;
        return nullptr;
    }
    return &g_rccl;
}

// Two communicators of the same ranks: the records' all-to-all-v on the caller's (comm) stream, and
// the small host-array collectives (per-step counts, all-reduces) on a communicator split off it
// (ncclCommSplit) with a stream and staging buffer of their own -- so a step's count exchange does
// not queue behind the previous step's records still moving on the comm stream (RCCL orders the
// operations of one communicator across streams).  Every rank issues both kinds in the same order.
// Without ncclCommSplit, or with FASTKMER_COMM_SPLIT=0, both run on the one communicator and the
// caller's stream.
//
// Failure semantics: a Spark job fails when one of its tasks fails (SBKC:1031-1043); here a rank
// that dies mid-exchange must not leave its peers blocked.  Every host wait on RCCL work goes
// through wait(): it polls the stream and ncclCommGetAsyncError, and after timeout_s_ (or on an
// asynchronous error) aborts both communicators -- RCCL kernels waiting for the dead peer then
// exit -- and fails; later calls fail at once.
class RcclComm : public Comm {
   public:
    RcclComm(const RcclApi *api, ncclComm_t comm, int n, int rank, double timeout_s)
        : api_(api), comm_(comm), timeout_s_(timeout_s) {
        n_ = n;
        rank_ = rank;
    }
    ~RcclComm() override {
        if (cstream_) (void)hipStreamSynchronize(cstream_);
        if (stage_) (void)hipFree(stage_);
        if (hstage_) (void)hipHostFree(hstage_);
        for (auto &r : retired_) (void)hipFree(r.first), (void)hipHostFree(r.second);
        if (cstream_) (void)hipStreamDestroy(cstream_);
        if (ccomm_) (void)api_->CommDestroy(ccomm_);
        if (comm_) (void)api_->CommDestroy(comm_);
    }
    const char *kind() const override { return "rccl"; }
    hipStream_t counts_stream() const override { return cstream_; }

    // collective over the ranks (every rank calls it once, right after joining)
    int init_counts(bool split, std::string &err) {
        if (!api_->CommSplit || !split) return 0;
        ncclComm_t c2 = nullptr;
        if (nccl(api_->CommSplit(comm_, 0, rank_, &c2, nullptr), err)) return -1;
        ccomm_ = c2;
        COMM_HIP(hipStreamCreateWithFlags(&cstream_, hipStreamNonBlocking));
        return 0;
    }

    int alltoall_u64(const uint64_t *in, uint64_t *out, size_t n, hipStream_t s, std::string &err) override {
        if (dead(err)) return -1;
        ncclComm_t cm = ccomm_ ? ccomm_ : comm_;
        if (cstream_) s = cstream_;
        const size_t bytes = (size_t)n_ * n * 8;
        if (stage(2 * bytes, s, err)) return -1;
        uint64_t *din = static_cast<uint64_t *>(stage_), *dout = din + (size_t)n_ * n;
        uint64_t *hin = static_cast<uint64_t *>(hstage_), *hout = hin + (size_t)n_ * n;
        uint64_t *hin_d = static_cast<uint64_t *>(hstage_dev_), *hout_d = hin_d + (size_t)n_ * n;
        memcpy(hin, in, bytes);  // mapped pinned memory, copied by kernels: nothing below blocks the host
        COMM_HIP(comm_copy(din, hin_d, (size_t)n_ * n, s));
        if (nccl(api_->GroupStart(), err)) return -1;
        for (int p = 0; p < n_; ++p) {
            if (nccl(api_->Send(din + (size_t)p * n, n, ncclUint64, p, cm, s), err)) return end_group(err);
            if (nccl(api_->Recv(dout + (size_t)p * n, n, ncclUint64, p, cm, s), err)) return end_group(err);
        }
        if (nccl(api_->GroupEnd(), err)) return -1;
        COMM_HIP(comm_copy(hout_d, dout, (size_t)n_ * n, s));
        if (wait(s, err)) return -1;
        memcpy(out, hout, bytes);
        return 0;
    }

    int allreduce_sum_u64(uint64_t *v, size_t n, hipStream_t s, std::string &err) override {
        if (dead(err)) return -1;
        if (!n) return 0;
        ncclComm_t cm = ccomm_ ? ccomm_ : comm_;
        if (cstream_) s = cstream_;
        if (stage(n * 8, s, err)) return -1;
        memcpy(hstage_, v, n * 8);
        COMM_HIP(comm_copy(static_cast<uint64_t *>(stage_), static_cast<const uint64_t *>(hstage_dev_), n, s));
        if (nccl(api_->AllReduce(stage_, stage_, n, ncclUint64, ncclSum, cm, s), err)) return -1;
        COMM_HIP(comm_copy(static_cast<uint64_t *>(hstage_dev_), static_cast<const uint64_t *>(stage_), n, s));
        if (wait(s, err)) return -1;
        memcpy(v, hstage_, n * 8);
        return 0;
    }

    int alltoallv(const uint8_t *send, const uint64_t *soff, const uint64_t *sbytes, uint8_t *recv,
                  const uint64_t *roff, const uint64_t *rbytes, hipStream_t s, std::string &err) override {
        if (dead(err)) return -1;
        if (nccl(api_->GroupStart(), err)) return -1;
        for (int p = 0; p < n_; ++p) {
            // a pair with nothing to move posts nothing on either side (both know the size)
            if (sbytes[p] && nccl(api_->Send(send + soff[p], sbytes[p], ncclUint8, p, comm_, s), err))
                return end_group(err);
            if (rbytes[p] && nccl(api_->Recv(recv + roff[p], rbytes[p], ncclUint8, p, comm_, s), err))
                return end_group(err);
        }
        return nccl(api_->GroupEnd(), err);
    }

    // Bounded host waits (see the class comment).  The first ~2 ms spin on the query (the per-step
    // waits are short), then the poll sleeps 50 us between queries.
    int wait(hipStream_t s, std::string &err) override {
        return poll([s] { return hipStreamQuery(s); }, "hipStreamQuery", err);
    }
    int wait_event(hipEvent_t ev, std::string &err) override {
        return poll([ev] { return hipEventQuery(ev); }, "hipEventQuery", err);
    }

    void abort() override {
        aborted_ = true;
        if (ccomm_ && api_->CommAbort) {
            (void)api_->CommAbort(ccomm_);
            ccomm_ = nullptr;
        }
        if (comm_ && api_->CommAbort) {
            (void)api_->CommAbort(comm_);
            comm_ = nullptr;
        }
    }
    bool split_counts() const { return ccomm_ != nullptr; }

   private:
    int nccl(ncclResult_t r, std::string &err) {
        if (r == ncclSuccess) return 0;
        err = std::string("RCCL: ") + api_->GetErrorString(r);
        return -1;
    }
    int end_group(std::string &err) {
        std::string ignore;
        (void)nccl(api_->GroupEnd(), ignore);
        (void)err;
        return -1;
    }
    bool dead(std::string &err) const {
        if (!aborted_) return false;
        err = "RCCL: the communicator was aborted by an earlier failure of this job";
        return true;
    }
    // an asynchronous error on either communicator (a peer's failure seen by RCCL's proxy)
    bool async_error(std::string &err) {
        if (!api_->GetAsyncError) return false;
        for (ncclComm_t cm : {comm_, ccomm_}) {
            if (!cm) continue;
            ncclResult_t ar = ncclSuccess;
            if (api_->GetAsyncError(cm, &ar) != ncclSuccess) continue;
            if (ar != ncclSuccess && ar != ncclInProgress) {
                err = std::string("RCCL asynchronous error: ") + api_->GetErrorString(ar);
                return true;
            }
        }
        return false;
    }
    template <typename Q>
    int poll(Q query, const char *what, std::string &err) {
        using clk = std::chrono::steady_clock;
        const auto t0 = clk::now();
        for (uint64_t it = 0;; ++it) {
            const hipError_t q = query();
            if (q == hipSuccess) return 0;
            if (q != hipErrorNotReady) {
                err = hip_msg(what, q);
                abort();
                return -1;
            }
            if ((it & 63) != 63) {
                sched_yield();
                continue;
            }
            if (async_error(err)) {
                abort();
                return -1;
            }
            const double el = std::chrono::duration<double>(clk::now() - t0).count();
            if (timeout_s_ > 0 && el > timeout_s_) {
                char msg[192];
                snprintf(msg, sizeof msg,
                         "RCCL: timed out after %.0f s waiting for rank %d's collective work "
                         "(FASTKMER_COMM_TIMEOUT_S); communicator aborted",
                         timeout_s_, rank_);
                err = msg;
                abort();
                return -1;
            }
            if (el > 0.002) usleep(50);
        }
    }
    // the device and mapped pinned host staging buffers of the small collectives (a pageable or small
    // hipMemcpyAsync can wait for the stream on the host, outside the bounded wait); the stream that
    // last used them has drained (every collective ends in a wait on it), so they can be replaced
    //    A grown buffer's predecessors are kept until the communicator is destroyed: hipFree
    //    synchronizes the device, which blocks for good behind a collective that never completes.
    int stage(size_t bytes, hipStream_t s, std::string &err) {
        (void)s;
        if (stage_bytes_ >= bytes) return 0;
        bytes = std::max<size_t>(bytes, std::max<size_t>(2 * stage_bytes_, 1u << 20));
        if (stage_) retired_.push_back({stage_, hstage_});
        stage_ = hstage_ = hstage_dev_ = nullptr;
        stage_bytes_ = 0;
        COMM_HIP(hipMalloc(&stage_, bytes));
        COMM_HIP(hipHostMalloc(&hstage_, bytes, hipHostMallocMapped | hipHostMallocCoherent));
        COMM_HIP(hipHostGetDevicePointer(&hstage_dev_, hstage_, 0));
        stage_bytes_ = bytes;
        return 0;
    }
    const RcclApi *api_;
    ncclComm_t comm_;
    ncclComm_t ccomm_ = nullptr;    // the counts' communicator (split off comm_)
    hipStream_t cstream_ = nullptr; // ... and its stream
    void *stage_ = nullptr, *hstage_ = nullptr, *hstage_dev_ = nullptr;
    std::vector<std::pair<void *, void *>> retired_;  // (device, host) staging buffers outgrown
    size_t stage_bytes_ = 0;
    double timeout_s_;
    bool aborted_ = false;
};

// ---------------------------------------------------------------------------
// in-process group
// ---------------------------------------------------------------------------

struct LocalGroup {
    explicit LocalGroup(int n) : n(n), device(n, 0) {
        for (auto &v : slot) v.resize(n);
        for (int p = 0; p < 2; ++p) ready[p].assign(n, nullptr), done[p].assign(n, nullptr);
    }
    // The ranks' events belong to the group, not to a rank: a peer may still wait on a rank's
    // `done` event after that rank has left the job's last collective and been destroyed (its
    // LocalComm gone), so they live until the last rank of the group is gone.
    ~LocalGroup() {
        int prev = -1;
        (void)hipGetDevice(&prev);
        for (int r = 0; r < n; ++r) {
            (void)hipSetDevice(device[r]);
            for (int p = 0; p < 2; ++p) {
                if (ready[p][r]) (void)hipEventDestroy(ready[p][r]);
                if (done[p][r]) (void)hipEventDestroy(done[p][r]);
            }
        }
        if (prev >= 0) (void)hipSetDevice(prev);
    }
    struct Slot {
        const uint64_t *in = nullptr;
        const uint8_t *send = nullptr;
        const uint64_t *soff = nullptr, *sbytes = nullptr;
    };
    int n;
    std::vector<int> device;                       // rank -> HIP device
    std::vector<hipEvent_t> ready[2], done[2];     // per collective parity, per rank
    std::mutex mu;
    std::condition_variable cv;
    uint64_t gen = 0;
    int arrived = 0;
    bool failed = false;
    std::vector<Slot> slot[2];  // by collective parity: a slot is rewritten two collectives later

    int barrier(std::string &err) {
        std::unique_lock<std::mutex> lk(mu);
        if (failed) {
            err = "a rank of the in-process group failed";
            return -1;
        }
        const uint64_t g = gen;
        if (++arrived == n) {
            arrived = 0;
            ++gen;
            cv.notify_all();
        } else {
            cv.wait(lk, [&] { return gen != g || failed; });
        }
        // a barrier every rank reached completed, whatever a rank did after leaving it (a rank
        // destroyed right after the job's last barrier fails the group only for later collectives)
        if (gen == g) {
            err = "a rank of the in-process group failed";
            return -1;
        }
        return 0;
    }
    void fail() {
        std::lock_guard<std::mutex> lk(mu);
        failed = true;
        cv.notify_all();
    }
};

class LocalComm : public Comm {
   public:
    LocalComm(std::shared_ptr<LocalGroup> g, int rank, int device) : g_(std::move(g)), dev_(device) {
        n_ = g_->n;
        rank_ = rank;
    }
    ~LocalComm() override {
        // a rank that leaves fails the group: peers blocked in (or entering) a collective return
        // an error instead of waiting for it.  Its events stay with the group (see LocalGroup).
        g_->fail();
    }
    int init(std::string &err) {
        g_->device[rank_] = dev_;
        for (int p = 0; p < 2; ++p) {
            COMM_HIP(hipEventCreateWithFlags(&g_->ready[p][rank_], hipEventDisableTiming));
            COMM_HIP(hipEventCreateWithFlags(&g_->done[p][rank_], hipEventDisableTiming));
        }
        return 0;
    }
    const char *kind() const override { return "local"; }

    int alltoall_u64(const uint64_t *in, uint64_t *out, size_t n, hipStream_t, std::string &err) override {
        auto &sl = g_->slot[next()];
        sl[rank_].in = in;
        if (g_->barrier(err)) return -1;
        for (int s = 0; s < n_; ++s) memcpy(out + (size_t)s * n, sl[s].in + (size_t)rank_ * n, n * 8);
        return g_->barrier(err);  // the peers' `in` arrays stay valid until everyone has read them
    }

    int allreduce_sum_u64(uint64_t *v, size_t n, hipStream_t, std::string &err) override {
        std::vector<uint64_t> mine(v, v + n);
        auto &sl = g_->slot[next()];
        sl[rank_].in = mine.data();
        if (g_->barrier(err)) return -1;
        for (size_t i = 0; i < n; ++i) {
            uint64_t t = 0;
            for (int s = 0; s < n_; ++s) t += sl[s].in[i];
            v[i] = t;
        }
        return g_->barrier(err);
    }

    int alltoallv(const uint8_t *send, const uint64_t *soff, const uint64_t *sbytes, uint8_t *recv,
                  const uint64_t *roff, const uint64_t *rbytes, hipStream_t s, std::string &err) override {
        const int p = next();
        auto &sl = g_->slot[p];
        hipEvent_t *ready = g_->ready[p].data(), *done = g_->done[p].data();
        COMM_HIP(hipEventRecord(ready[rank_], s));
        sl[rank_].send = send;
        sl[rank_].soff = soff;
        sl[rank_].sbytes = sbytes;
        if (g_->barrier(err)) return -1;
        int rc = 0;
        for (int r = 0; r < n_ && !rc; ++r) {
            const uint64_t nb = sl[r].sbytes[rank_];
            if (nb != rbytes[r]) {
                err = "in-process exchange: rank " + std::to_string(r) + " sends " + std::to_string(nb) +
                      " bytes, rank " + std::to_string(rank_) + " expects " + std::to_string(rbytes[r]);
                rc = -1;
                break;
            }
            if (!nb) continue;
            hipError_t e = hipStreamWaitEvent(s, ready[r], 0);
            if (e == hipSuccess)
                e = g_->device[r] == dev_
                        ? hipMemcpyAsync(recv + roff[r], sl[r].send + sl[r].soff[rank_], nb, hipMemcpyDeviceToDevice, s)
                        : hipMemcpyPeerAsync(recv + roff[r], dev_, sl[r].send + sl[r].soff[rank_], g_->device[r], nb,
                                             s);
            if (e != hipSuccess) {
                err = hip_msg("in-process exchange copy", e);
                rc = -1;
            }
        }
        if (rc) {
            g_->fail();
            return -1;
        }
        COMM_HIP(hipEventRecord(done[rank_], s));
        if (g_->barrier(err)) return -1;
        // this rank's send buffer stays untouched until every peer has copied out of it (the
        // context's teardown synchronizes this stream before it frees the send buffer)
        for (int r = 0; r < n_; ++r)
            if (r != rank_ && sbytes[r]) COMM_HIP(hipStreamWaitEvent(s, done[r], 0));
        return 0;
    }

    void abort() override { g_->fail(); }

   private:
    int next() { return (int)(seq_++ & 1u); }
    std::shared_ptr<LocalGroup> g_;
    int dev_;
    uint64_t seq_ = 0;
};

}  // namespace

int comm_unique_id(uint8_t id[COMM_ID_BYTES], std::string &err) {
    const RcclApi *a = rccl(err);
    if (!a) return -1;
    ncclUniqueId u;
    const ncclResult_t r = a->GetUniqueId(&u);
    if (r != ncclSuccess) {
        err = std::string("ncclGetUniqueId: ") + a->GetErrorString(r);
        return -1;
    }
    memcpy(id, u.internal, COMM_ID_BYTES);
    return 0;
}

Comm *comm_create_rccl(const uint8_t id[COMM_ID_BYTES], int n, int rank, int device, std::string &err) {
    const RcclApi *a = rccl(err);
    if (!a) return nullptr;
    ncclUniqueId u;
    memcpy(u.internal, id, COMM_ID_BYTES);
    ncclComm_t comm = nullptr;
    const ncclResult_t r = a->CommInitRank(&comm, n, u, rank);  // blocks until every rank has joined
    if (r != ncclSuccess) {
        err = std::string("ncclCommInitRank: ") + a->GetErrorString(r);
        return nullptr;
    }
    (void)device;
    double timeout = 120.0;
    if (const char *e = getenv("FASTKMER_COMM_TIMEOUT_S"); e && e[0]) timeout = atof(e);
    const char *sp = getenv("FASTKMER_COMM_SPLIT");
    const bool split = !(sp && sp[0] == '0');
    auto *rc = new RcclComm(a, comm, n, rank, timeout);
    if (rc->init_counts(split, err)) {
        delete rc;
        return nullptr;
    }
    return rc;
}

int comm_create_local(int n, const int *devices, Comm **out, std::string &err) {
    auto g = std::make_shared<LocalGroup>(n);
    int prev = -1;
    (void)hipGetDevice(&prev);
    int rc = 0;
    for (int r = 0; r < n; ++r) out[r] = nullptr;
    for (int r = 0; r < n && !rc; ++r) {
        if (hipSetDevice(devices[r]) != hipSuccess) {
            err = "cannot select device " + std::to_string(devices[r]);
            rc = -1;
            break;
        }
        auto *c = new LocalComm(g, r, devices[r]);
        rc = c->init(err);
        out[r] = c;
    }
    if (prev >= 0) (void)hipSetDevice(prev);
    if (rc)
        for (int r = 0; r < n; ++r) {
            delete out[r];
            out[r] = nullptr;
        }
    return rc;
}

const char *comm_rccl_path() {
    std::string ignore;
    const RcclApi *a = rccl(ignore);
    return a ? a->path.c_str() : "";
}

}  // namespace fk
