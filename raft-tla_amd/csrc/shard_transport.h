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
#include <climits>
#include <condition_variable>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rccl_api.h"

namespace rmc {

struct ShardTransport {
  virtual ~ShardTransport() {}
  virtual int exchange(int me, int W, const char* const* src, const uint64_t* sbytes, char* const* dst,
                       const uint64_t* rbytes, hipStream_t s, std::string& err) = 0;
  virtual int allreduce(int64_t* d_sum, int n_sum, int64_t* d_max, int n_max, hipStream_t s, std::string& err) = 0;
};

// RCCL over xGMI: grouped ncclSend/ncclRecv straight between the kernels' buffers
struct RcclTransport : ShardTransport {
  ncclComm_t comm;
  explicit RcclTransport(ncclComm_t c) : comm(c) {}
  int exchange(int me, int W, const char* const* src, const uint64_t* sbytes, char* const* dst, const uint64_t* rbytes,
               hipStream_t s, std::string& err) override {
    RcclApi& R = rccl();
    if (W <= 1) return 0;
    ncclResult_t r = R.GroupStart();
    for (int p = 0; p < W && r == ncclSuccess; ++p) {
      if (p == me) continue;
      if (sbytes[p]) r = R.Send(src[p], sbytes[p], ncclUint8, p, comm, s);
      if (r == ncclSuccess && rbytes[p]) r = R.Recv(dst[p], rbytes[p], ncclUint8, p, comm, s);
    }
    const ncclResult_t r2 = R.GroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) { err = std::string("RCCL exchange: ") + R.GetErrorString(r != ncclSuccess ? r : r2); return -5; }
    return 0;
  }
  int allreduce(int64_t* d_sum, int n_sum, int64_t* d_max, int n_max, hipStream_t s, std::string& err) override {
    RcclApi& R = rccl();
    ncclResult_t r = R.GroupStart();
    if (r == ncclSuccess) r = R.AllReduce(d_sum, d_sum, n_sum, ncclInt64, ncclSum, comm, s);
    if (r == ncclSuccess) r = R.AllReduce(d_max, d_max, n_max, ncclInt64, ncclMax, comm, s);
    const ncclResult_t r2 = R.GroupEnd();
    if (r != ncclSuccess || r2 != ncclSuccess) { err = std::string("RCCL all-reduce: ") + R.GetErrorString(r != ncclSuccess ? r : r2); return -5; }
    return 0;
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
