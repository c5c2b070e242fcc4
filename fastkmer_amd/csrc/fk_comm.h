// fk_comm.h -- rank-to-rank transports of the bin exchange.
//
// The reference moves super-k-mers to the executor that owns their bin with
// Spark's shuffle (reduceByKey, SparkBinKmerCounter.scala:1034-1042).  Here a
// context owns one GPU and the shuffle is a device all-to-all-v of packed
// records plus a small all-to-all of per-part counts.  Two transports:
//   * RCCL over xGMI (one process or thread per GPU; the communicator is
//     joined with a 128-byte unique id the caller distributes, as Spark's
//     driver distributes the job), librccl loaded at run time so the library
//     binds to the RCCL already mapped into the process (torch's, in Python)
//     or to /opt/rocm's (the CLI, a JVM executor);
//   * an in-process group (one host thread per context: tests, or executors
//     sharing one JVM): device-to-device copies between the contexts' buffers,
//     rendezvous on a shared barrier.
#pragma once

#include <hip/hip_runtime.h>
#include <stddef.h>
#include <stdint.h>

#include <string>

namespace fk {

constexpr int COMM_ID_BYTES = 128;  // NCCL_UNIQUE_ID_BYTES

class Comm {
   public:
    virtual ~Comm() = default;
    int size() const { return n_; }
    int rank() const { return rank_; }
    virtual const char *kind() const = 0;
    // Blocking all-to-all of `n` u64 per peer between host arrays:
    // out[s * n + i] = in[rank * n + i] of rank s.  `s` is the caller's stream.
    virtual int alltoall_u64(const uint64_t *in, uint64_t *out, size_t n, hipStream_t s, std::string &err) = 0;
    // Blocking sum over the ranks of a host u64 array, in place.
    virtual int allreduce_sum_u64(uint64_t *v, size_t n, hipStream_t s, std::string &err) = 0;
    // Device all-to-all-v, posted on stream `s` and asynchronous to the host:
    // sbytes[d] bytes at send + soff[d] go to rank d, rbytes[r] bytes from rank r
    // land at recv + roff[r].  The send bytes must be ready on `s`; the received
    // bytes are ready once `s` reaches the end of the call's work.
    virtual int alltoallv(const uint8_t *send, const uint64_t *soff, const uint64_t *sbytes, uint8_t *recv,
                          const uint64_t *roff, const uint64_t *rbytes, hipStream_t s, std::string &err) = 0;
    // Marks the group failed so that peers blocked in a collective return an
    // error instead of waiting (in-process groups; RCCL aborts the communicator).
    virtual void abort() {}
    // Host wait for everything queued on `s` (which may hold this transport's
    // work).  RCCL: bounded -- polls the stream and the communicators'
    // asynchronous error; after the timeout (FASTKMER_COMM_TIMEOUT_S) or on an
    // RCCL error it aborts the communicators and returns -1 with `err` set.
    virtual int wait(hipStream_t s, std::string &err) {
        const hipError_t e = hipStreamSynchronize(s);
        if (e == hipSuccess) return 0;
        (void)hipGetLastError();
        err = std::string("hipStreamSynchronize: ") + hipGetErrorString(e);
        return -1;
    }
    // The same for one event.
    virtual int wait_event(hipEvent_t ev, std::string &err) {
        const hipError_t e = hipEventSynchronize(ev);
        if (e == hipSuccess) return 0;
        (void)hipGetLastError();
        err = std::string("hipEventSynchronize: ") + hipGetErrorString(e);
        return -1;
    }
    // The stream the small host-array collectives run on when it is not the
    // caller's (RCCL with a split counts communicator), else null.
    virtual hipStream_t counts_stream() const { return nullptr; }

   protected:
    int n_ = 1, rank_ = 0;
};

// A fresh RCCL unique id (ncclGetUniqueId): created on one rank, handed to all.
int comm_unique_id(uint8_t id[COMM_ID_BYTES], std::string &err);
// Joins the RCCL communicator of `n` ranks as `rank` on HIP device `device`.
// Environment: FASTKMER_COMM_TIMEOUT_S (bounded waits, default 120 s; 0 = unbounded),
// FASTKMER_COMM_SPLIT=0 (the counts on the records' communicator and stream).
Comm *comm_create_rccl(const uint8_t id[COMM_ID_BYTES], int n, int rank, int device, std::string &err);
// n ranks in this process (devices[r] = rank r's HIP device): out[r] = rank r's Comm.
int comm_create_local(int n, const int *devices, Comm **out, std::string &err);
// The RCCL library the transport would use ("" when none loads).
const char *comm_rccl_path();

}  // namespace fk
