// raftmc — the exchange steps of the native sharded BFS (orig_backend.hip shard_run_native) behind
// one interface, so the same level loop runs over RCCL between GPUs (one process per GPU, the
// production path) or over an in-process loopback between W ranks that share one GPU (tests: every
// W > 1 branch of the loop, the self-segment offsets and the all-reduce, on a one-GPU box).
//
// exchange(): grouped point-to-point — rank `me` sends sbytes[r] bytes from src[r] to every r != me
// and receives rbytes[r] bytes from r into dst[r].  allreduce(): in place, element-wise sum of
// n_sum int64 at d_sum and max of n_max int64 at d_max over all ranks.  Both are enqueued on /
// ordered with the caller's stream; neither touches the caller's self segment.
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <atomic>
#include <chrono>
#include <climits>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "rccl_api.h"

namespace rmc {

struct ShardTransport {
  virtual ~ShardTransport() {}
  virtual int exchange(int me, int W, const char* const* src, const uint64_t* sbytes, char* const* dst,
                       const uint64_t* rbytes, hipStream_t s, std::string& err) = 0;
  virtual int allreduce(int64_t* d_sum, int n_sum, int64_t* d_max, int n_max, hipStream_t s, std::string& err) = 0;
  virtual bool allreduce_at_world1() const { return false; }   // run allreduce() with one rank too
};

// Abort coordination of the in-process multi-GPU run (mc_api.cpp run_multi): the ranks' RcclTransports
// share one RcclAbort.  The communicators are non-blocking (rccl_api.h rccl_init_all): no RCCL call
// blocks its thread, a rank waits for its exchanges by polling (RcclTransport::complete) and sees
// `aborted` between two polls.  Every RCCL call of a rank is bracketed by its `busy` flag, raised BEFORE
// the `aborted` flag is read (both sequentially consistent), so the aborting thread either sees the
// rank inside a call (which returns at once) and waits for it to leave, or the rank sees `aborted` and
// returns an error without touching its communicator.  Only then is the communicator aborted
// (ncclCommAbort frees it and stops its pending kernels): no rank uses a freed communicator.  (With
// an RCCL without non-blocking communicators the calls block; a rank still inside one after the grace
// period is aborted anyway, as that call cannot return otherwise.)
struct RcclAbort {
  explicit RcclAbort(int w) : busy(w) { for (auto& b : busy) b.store(false); }
  std::vector<std::atomic<bool>> busy;   // [rank] inside an RCCL call
  std::atomic<bool> aborted{false};
  std::atomic<int> first{-1};            // the rank that failed first in its own right
  std::mutex mu;
  bool done = false;                     // communicators aborted (under mu)
  // called by a failing rank; returns after every communicator is aborted
  void abort_all(int rank, std::vector<ncclComm_t>& comms) {
    int expect = -1;
    first.compare_exchange_strong(expect, rank);
    aborted.store(true);
    std::lock_guard<std::mutex> lk(mu);
    if (done) return;
    done = true;
    const int grace_ms = rccl().nonblocking() ? 60000 : 5000;   // non-blocking: calls return at once
    for (size_t r = 0; r < comms.size(); ++r) {
      for (int spin = 0; busy[r].load() && spin < grace_ms; ++spin) std::this_thread::sleep_for(std::chrono::milliseconds(1));
      if (comms[r]) (void)rccl().CommAbort(comms[r]);
      comms[r] = nullptr;                // freed by the abort: never destroyed again
    }
  }
};

// RCCL over xGMI: grouped ncclSend/ncclRecv straight between the kernels' buffers.  Each call
// returns once its transfers are done: the group is polled out of ncclInProgress (non-blocking
// communicator), an event recorded behind it on the stream is polled to completion, and between polls
// the communicator's asynchronous error (a peer's failure) and the in-process abort flag are checked
// -- so a rank never waits in a stream synchronisation on a transfer a failed peer will not serve.
struct RcclTransport : ShardTransport {
  ncclComm_t comm;
  RcclAbort* ab;   // the in-process run's abort coordination (nullptr: one rank per process)
  int rank;
  hipEvent_t done_ev = nullptr;
  explicit RcclTransport(ncclComm_t c, RcclAbort* a = nullptr, int r = 0) : comm(c), ab(a), rank(r) {}
  ~RcclTransport() override { if (done_ev) (void)hipEventDestroy(done_ev); }
  // raise busy, then check aborted (see RcclAbort); false = aborted, the call must not run
  bool enter(std::string& err) {
    if (!ab) return true;
    ab->busy[rank].store(true);
    if (ab->aborted.load()) { ab->busy[rank].store(false); err = "RCCL: another rank left the loop (communicators aborted)"; return false; }
    return true;
  }
  void leave() { if (ab) ab->busy[rank].store(false); }
  bool stopped() const { return ab && ab->aborted.load(); }
  // the group just ended: wait for it to be enqueued and then to finish on the stream
  int complete(hipStream_t s, const char* what, std::string& err) {
    RcclApi& R = rccl();
    if (!R.nonblocking()) return 0;   // blocking communicator: the caller's stream synchronisation waits
    for (;;) {   // out of ncclInProgress: the group's work is on the stream
      if (!enter(err)) return -5;
      ncclResult_t st = ncclSuccess;
      const ncclResult_t r = R.CommGetAsyncError(comm, &st);
      leave();
      if (r != ncclSuccess || (st != ncclSuccess && st != ncclInProgress)) {
        err = std::string(what) + ": " + R.GetErrorString(r != ncclSuccess ? r : st);
        return -5;
      }
      if (st == ncclSuccess) break;
      std::this_thread::yield();
    }
    if (!done_ev && hipEventCreateWithFlags(&done_ev, hipEventDisableTiming) != hipSuccess) { err = std::string(what) + ": hipEventCreate"; return -5; }
    if (hipEventRecord(done_ev, s) != hipSuccess) { err = std::string(what) + ": hipEventRecord"; return -5; }
    for (unsigned spin = 0;; ++spin) {
      const hipError_t q = hipEventQuery(done_ev);
      if (q == hipSuccess) return 0;
      if (q != hipErrorNotReady) { err = std::string(what) + ": " + hipGetErrorString(q); return -5; }
      if (stopped()) { err = std::string(what) + ": another rank left the loop (communicators aborted)"; return -5; }
      if ((spin & 1023) == 1023) {   // now and then: has a peer failed?
        if (!enter(err)) return -5;
        ncclResult_t st = ncclSuccess;
        const ncclResult_t r = R.CommGetAsyncError(comm, &st);
        leave();
        if (r != ncclSuccess || (st != ncclSuccess && st != ncclInProgress)) {
          err = std::string(what) + ": " + R.GetErrorString(r != ncclSuccess ? r : st);
          return -5;
        }
      }
      std::this_thread::yield();
    }
  }
  int exchange(int me, int W, const char* const* src, const uint64_t* sbytes, char* const* dst, const uint64_t* rbytes,
               hipStream_t s, std::string& err) override {
    RcclApi& R = rccl();
    if (W <= 1) return 0;
    if (!enter(err)) return -5;
    ncclResult_t r = R.GroupStart();
    for (int p = 0; p < W && r == ncclSuccess; ++p) {
      if (p == me) continue;
      if (sbytes[p]) r = R.Send(src[p], sbytes[p], ncclUint8, p, comm, s);
      if (r == ncclSuccess && rbytes[p]) r = R.Recv(dst[p], rbytes[p], ncclUint8, p, comm, s);
    }
    ncclResult_t r2 = R.GroupEnd();
    leave();
    if (r2 == ncclInProgress) r2 = ncclSuccess;   // non-blocking: complete() waits
    if (r != ncclSuccess || r2 != ncclSuccess) { err = std::string("RCCL exchange: ") + R.GetErrorString(r != ncclSuccess ? r : r2); return -5; }
    return complete(s, "RCCL exchange", err);
  }
  // also at world 1 (a one-rank all-reduce): the mc_shard_run_rccl path runs its communicator, the
  // non-blocking group and the completion polling at every level on a one-GPU machine too
  bool allreduce_at_world1() const override { return true; }
  int allreduce(int64_t* d_sum, int n_sum, int64_t* d_max, int n_max, hipStream_t s, std::string& err) override {
    RcclApi& R = rccl();
    if (!enter(err)) return -5;
    ncclResult_t r = R.GroupStart();
    if (r == ncclSuccess) r = R.AllReduce(d_sum, d_sum, n_sum, ncclInt64, ncclSum, comm, s);
    if (r == ncclSuccess) r = R.AllReduce(d_max, d_max, n_max, ncclInt64, ncclMax, comm, s);
    ncclResult_t r2 = R.GroupEnd();
    leave();
    if (r2 == ncclInProgress) r2 = ncclSuccess;
    if (r != ncclSuccess || r2 != ncclSuccess) { err = std::string("RCCL all-reduce: ") + R.GetErrorString(r != ncclSuccess ? r : r2); return -5; }
    return complete(s, "RCCL all-reduce", err);
  }
};

// In-process loopback between W ranks (one host thread each, all on one GPU): every exchange is a
// rendezvous — each rank publishes its send segments and a stream-ordered event, then pulls the
// segments addressed to it with device-to-device copies on its own stream, and waits for them
// before the next rendezvous (so no sender overwrites a segment that is still being read).
struct LoopbackWorld {
  int W;
  std::mutex mu;
  std::condition_variable cv;
  int arrived = 0;
  unsigned long long generation = 0;
  std::vector<std::vector<const char*>> src;        // [rank][peer]
  std::vector<std::vector<uint64_t>> sbytes;        // [rank][peer]
  std::vector<hipEvent_t> ready;                    // [rank]
  std::vector<std::vector<int64_t>> sum, mx;        // all-reduce staging [rank]
  std::atomic<bool> failed{false};   // a transfer failed on some rank
  bool aborted = false;              // a rank left the loop early: every rendezvous returns false
  explicit LoopbackWorld(int w) : W(w), src(w, std::vector<const char*>(w)), sbytes(w, std::vector<uint64_t>(w)), ready(w, nullptr),
                                  sum(w), mx(w) {}
  ~LoopbackWorld() {
    for (hipEvent_t e : ready)
      if (e) (void)hipEventDestroy(e);
  }
  bool barrier() {   // false once aborted
    std::unique_lock<std::mutex> lk(mu);
    if (aborted) return false;
    const unsigned long long g = generation;
    if (++arrived == W) { arrived = 0; ++generation; cv.notify_all(); return true; }
    cv.wait(lk, [&] { return generation != g || aborted; });
    return !aborted;
  }
  void abort() {
    std::lock_guard<std::mutex> lk(mu);
    aborted = true;
    cv.notify_all();
  }
};

struct LoopbackTransport : ShardTransport {
  LoopbackWorld& w;
  int me;
  LoopbackTransport(LoopbackWorld& world, int rank) : w(world), me(rank) {
    if (!w.ready[me]) (void)hipEventCreateWithFlags(&w.ready[me], hipEventDisableTiming);
  }
  int exchange(int me_, int W, const char* const* src, const uint64_t* sbytes, char* const* dst, const uint64_t* rbytes,
               hipStream_t s, std::string& err) override {
    (void)me_;
    for (int p = 0; p < W; ++p) { w.src[me][p] = src[p]; w.sbytes[me][p] = p == me ? 0 : sbytes[p]; }
    if (hipEventRecord(w.ready[me], s) != hipSuccess) { err = "loopback: hipEventRecord"; return -5; }
    if (!w.barrier()) { err = "loopback: another rank left the loop"; return -5; }
    for (int p = 0; p < W; ++p) {
      if (p == me) continue;
      if (w.sbytes[p][me] != rbytes[p]) { err = "loopback: send/receive sizes disagree"; w.failed = true; }
      if (!rbytes[p] || w.failed) continue;
      if (hipStreamWaitEvent(s, w.ready[p], 0) != hipSuccess ||
          hipMemcpyAsync(dst[p], w.src[p][me], rbytes[p], hipMemcpyDeviceToDevice, s) != hipSuccess) {
        err = "loopback: device copy failed"; w.failed = true;
      }
    }
    if (hipStreamSynchronize(s) != hipSuccess) { err = "loopback: stream synchronize"; w.failed = true; }
    if (!w.barrier()) { err = "loopback: another rank left the loop"; return -5; }
    return w.failed ? -5 : 0;
  }
  int allreduce(int64_t* d_sum, int n_sum, int64_t* d_max, int n_max, hipStream_t s, std::string& err) override {
    w.sum[me].assign(n_sum, 0); w.mx[me].assign(n_max, 0);
    if (hipMemcpyAsync(w.sum[me].data(), d_sum, n_sum * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(w.mx[me].data(), d_max, n_max * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) { err = "loopback: all-reduce staging"; w.failed = true; }
    if (!w.barrier()) { err = "loopback: another rank left the loop"; return -5; }
    std::vector<int64_t> a(n_sum, 0), b(n_max, INT64_MIN);
    for (int p = 0; p < w.W; ++p) {
      for (int k = 0; k < n_sum; ++k) a[k] += w.sum[p][k];
      for (int k = 0; k < n_max; ++k) b[k] = std::max(b[k], w.mx[p][k]);
    }
    if (!w.barrier()) { err = "loopback: another rank left the loop"; return -5; }   // all staging read
    if (hipMemcpyAsync(d_sum, a.data(), n_sum * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipMemcpyAsync(d_max, b.data(), n_max * 8, hipMemcpyHostToDevice, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess) { err = "loopback: all-reduce result"; w.failed = true; }
    return w.failed ? -5 : 0;
  }
};

}  // namespace rmc
