// raftmc — the native level loop of the FIFO-ranked sharded BFS (tlc_membership: VIEW vars, so the
// kept representative of a view class is TLC's single-worker first-found one).
//
// The loop that raft-tla_amd/shard.py fifo_sharded_bfs runs over torch.distributed, in C++ over a
// ShardTransport (RCCL between GPUs, or the in-process loopback), driving the Backend's rank-local
// shard_* steps.  Per level:
//   all-gather of the frontier sizes -> shard_layout (global parent ranks = concatenation)
//   per chunk: shard_generate -> counts all-to-all -> ROUTE payload all-to-all -> shard_dedup
//   shard_select -> counts all-to-all -> REPLY payload all-to-all -> shard_materialize
//   shard_level_stats -> all-gather of the new-state counts + all-reduce of the statistics
//   (sum; max of the flags and of the (2^62 - first event) word); on an event, the all-reduced
//   per-rank share of TLC's stop-point counters (shard_event_stats)
//   shard_level_commit; the rebalancing STATES all-to-all -> shard_store
// Counts and statistics travel through small device buffers on the loop's own stream; payloads go
// straight between the kernels' buffers (the self segment by a device copy).
#pragma once
#include <hip/hip_runtime.h>

#include <algorithm>
#include <string>
#include <vector>

#include "../../include/raftmc.h"
#include "backend.h"
#include "shard_transport.h"

namespace rmc {

struct FifoShardLoop {
  Backend& be;
  ShardTransport& T;
  int me, W;
  hipStream_t s = nullptr;
  int64_t* d_small = nullptr;    // [0,8) counts sent, [8,16) counts received, [16, 16+W) gather, then sum / max stats
  int64_t* h_small = nullptr;    // pinned mirror
  char* d_send = nullptr; char* d_recv = nullptr;
  uint64_t send_cap = 0, recv_cap = 0;
  static constexpr int NST = MC_SHARD_NSTAT;
  static constexpr int SMALL = 32 + 2 * MC_SHARD_NSTAT;

  FifoShardLoop(Backend& b, ShardTransport& t, int rank, int world) : be(b), T(t), me(rank), W(world) {}
  ~FifoShardLoop() {
    if (s) (void)hipStreamSynchronize(s);
    if (d_send) (void)hipFree(d_send);
    if (d_recv) (void)hipFree(d_recv);
    if (d_small) (void)hipFree(d_small);
    if (h_small) (void)hipHostFree(h_small);
    if (s) (void)hipStreamDestroy(s);
  }

#define FSL_HIP(x)                                                     \
  do {                                                                 \
    if ((x) != hipSuccess) { err = std::string("HIP: ") + #x; return MC_E_NO_DEVICE; } \
  } while (0)

  int grow(char*& p, uint64_t& cap, uint64_t need, std::string& err) {
    if (need <= cap && p) return 0;
    FSL_HIP(hipStreamSynchronize(s));
    if (p) FSL_HIP(hipFree(p));
    p = nullptr;
    cap = std::max<uint64_t>(need + need / 4, 1 << 20);
    FSL_HIP(hipMalloc(&p, cap));
    return 0;
  }
  // all-to-all of one int64 per peer: recv[r] = what rank r sends to me
  int counts(const int64_t* send, int64_t* recv, std::string& err) {
    for (int r = 0; r < W; ++r) h_small[r] = send[r];
    FSL_HIP(hipMemcpyAsync(d_small, h_small, 8 * (uint64_t)W, hipMemcpyHostToDevice, s));
    if (W > 1) {
      const char* src[8]; char* dst[8]; uint64_t n8[8];
      for (int r = 0; r < W; ++r) { src[r] = (const char*)(d_small + r); dst[r] = (char*)(d_small + 8 + r); n8[r] = 8; }
      if (T.exchange(me, W, src, n8, dst, n8, s, err)) return MC_E_NO_DEVICE;
    }
    FSL_HIP(hipMemcpyAsync(h_small + 8, d_small + 8, 8 * (uint64_t)W, hipMemcpyDeviceToHost, s));
    FSL_HIP(hipStreamSynchronize(s));
    for (int r = 0; r < W; ++r) recv[r] = r == me ? send[me] : h_small[8 + r];
    return 0;
  }
  // in-place all-reduce of n int64 at h (sum over ranks, or max where is_max[k])
  int allreduce(int64_t* h, int n, const bool* is_max, std::string& err) {
    int64_t* d_sum = d_small + 32;
    int64_t* d_max = d_sum + NST;
    std::vector<int64_t> mx(n, INT64_MIN);
    int nmax = 0;
    for (int k = 0; k < n; ++k) {
      h_small[32 + k] = is_max && is_max[k] ? 0 : h[k];
      if (is_max && is_max[k]) mx[k] = h[k], ++nmax;
    }
    for (int k = 0; k < n; ++k) h_small[32 + NST + k] = mx[k];
    FSL_HIP(hipMemcpyAsync(d_sum, h_small + 32, 2 * NST * 8, hipMemcpyHostToDevice, s));
    if ((W > 1 || T.allreduce_at_world1()) && T.allreduce(d_sum, n, d_max, nmax ? n : 1, s, err)) return MC_E_NO_DEVICE;
    FSL_HIP(hipMemcpyAsync(h_small + 32, d_sum, 2 * NST * 8, hipMemcpyDeviceToHost, s));
    FSL_HIP(hipStreamSynchronize(s));
    for (int k = 0; k < n; ++k) h[k] = is_max && is_max[k] ? h_small[32 + NST + k] : h_small[32 + k];
    return 0;
  }
  int allgather(int64_t x, int64_t* out, std::string& err) {
    for (int r = 0; r < W; ++r) out[r] = r == me ? x : 0;
    return allreduce(out, W, nullptr, err);
  }
  // the payload of record kind `what`: sc[r] records to rank r (shard_fill packs them at the send
  // offsets), rc[r] records from rank r land in d_recv in source-rank order
  int payload(int what, const int64_t* sc, const int64_t* rc, std::string& err) {
    const int rb = be.shard_record_bytes(what);
    if (rb <= 0) { err = "shard_record_bytes"; return MC_E_INVALID; }
    int64_t soff[8], roff[8];
    int64_t ts = 0, tr = 0;
    for (int r = 0; r < W; ++r) { soff[r] = ts; ts += sc[r]; roff[r] = tr; tr += rc[r]; }
    if (sc[me] != rc[me]) { err = "sharded exchange: self segment size mismatch"; return MC_E_STATE; }
    if (int e = grow(d_send, send_cap, (uint64_t)ts * rb, err)) return e;
    if (int e = grow(d_recv, recv_cap, (uint64_t)tr * rb, err)) return e;
    if (int e = be.shard_fill(what, d_send, soff, err)) return e;
    const char* src[8]; char* dst[8]; uint64_t sb[8], rbs[8];
    for (int r = 0; r < W; ++r) {
      src[r] = d_send + (uint64_t)soff[r] * rb; sb[r] = (uint64_t)sc[r] * rb;
      dst[r] = d_recv + (uint64_t)roff[r] * rb; rbs[r] = (uint64_t)rc[r] * rb;
    }
    if (sb[me]) FSL_HIP(hipMemcpyAsync(dst[me], src[me], sb[me], hipMemcpyDeviceToDevice, s));
    if (W > 1 && T.exchange(me, W, src, sb, dst, rbs, s, err)) return MC_E_NO_DEVICE;
    FSL_HIP(hipStreamSynchronize(s));
    return 0;
  }

  static int64_t overlap(int64_t a0, int64_t a1, int64_t b0, int64_t b1) {
    return std::max<int64_t>(0, std::min(a1, b1) - std::max(a0, b0));
  }

  int run(std::string& err) {
    FSL_HIP(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    FSL_HIP(hipMalloc(&d_small, SMALL * 8));
    FSL_HIP(hipHostMalloc((void**)&h_small, SMALL * 8, hipHostMallocDefault));
    bool flag_max[NST] = {false};
    for (int k = 3; k < 6; ++k) flag_max[k] = true;   // error flags, first event, deadlock (shard.py FLAG_SLICE)
    int64_t sc[8] = {0}, rc[8] = {0}, gat[8] = {0}, dummy[8] = {0};
    for (;;) {
      int64_t front = 0, chunk = 0;
      if (int e = be.shard_frontier(&front, &chunk)) { err = "shard_frontier"; return e; }
      if (int e = allgather(front, gat, err)) return e;
      if (int e = be.shard_layout(gat, err)) return e;
      int64_t nchunks = 0;
      for (int r = 0; r < W; ++r) if (chunk) nchunks = std::max<int64_t>(nchunks, (gat[r] + chunk - 1) / chunk);
      for (int64_t q = 0; q < nchunks; ++q) {
        const int64_t begin = q * chunk, count = std::max<int64_t>(0, std::min<int64_t>(chunk, front - begin));
        if (int e = be.shard_generate(std::min(begin, front), count, sc, err)) return e;
        if (int e = counts(sc, rc, err)) return e;
        if (int e = payload(MC_SHARD_ROUTE, sc, rc, err)) return e;
        if (int e = be.shard_dedup(d_recv, rc, dummy, err)) return e;
      }
      if (int e = be.shard_select(sc, err)) return e;      // winners generated by rank r go back to r
      if (int e = counts(sc, rc, err)) return e;
      if (int e = payload(MC_SHARD_REPLY, sc, rc, err)) return e;
      if (int e = be.shard_materialize(d_recv, rc, err)) return e;
      int64_t st[NST];
      if (int e = be.shard_level_stats(st, err)) return e;
      int64_t news[8];
      if (int e = allgather(st[0], news, err)) return e;
      const int64_t my_flags = st[3];
      if (int e = allreduce(st, NST, flag_max, err)) return e;
      if (st[3]) {   // some rank raised an error: the bitwise OR of every rank's flags, not the max
        int64_t fl[8];
        if (int e = allgather(my_flags, fl, err)) return e;
        st[3] = 0;
        for (int r = 0; r < W; ++r) st[3] |= fl[r];
      }
      if (st[4]) {   // the level's first event in key order stops the search
        int64_t ev[NST];
        if (int e = be.shard_event_stats(st, ev, err)) return e;
        if (int e = allreduce(ev, NST, nullptr, err)) return e;
        st[30] = ev[30]; st[31] = ev[31]; st[32] = ev[32];
        for (int k = 8; k < 30; ++k) st[k] = ev[k];        // per-action generated at the stop point
        for (int k = 40; k < 62; ++k) st[k] = ev[k];       // per-action distinct
      }
      int done = 0;
      if (int e = be.shard_level_commit(st, &done, err)) return e;
      if (done) break;
      // rebalance: rank k gets the slice [k*D/W, (k+1)*D/W) of the level's key-ordered runs
      int64_t total = 0, off[8];
      for (int r = 0; r < W; ++r) { off[r] = total; total += news[r]; }
      for (int k = 0; k < W; ++k) {
        const int64_t t0 = k * total / W, t1 = (k + 1) * total / W;
        sc[k] = overlap(off[me], off[me] + news[me], t0, t1);
      }
      const int64_t m0 = me * total / W, m1 = (me + 1) * total / W;
      int64_t nrecv = 0;
      for (int g = 0; g < W; ++g) { rc[g] = overlap(off[g], off[g] + news[g], m0, m1); nrecv += rc[g]; }
      if (int e = payload(MC_SHARD_STATES, sc, rc, err)) return e;
      if (int e = be.shard_store(d_recv, nrecv, err)) return e;
    }
    return 0;
  }
#undef FSL_HIP
};

}  // namespace rmc
