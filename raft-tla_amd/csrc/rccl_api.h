// raftmc: the RCCL entry points the native sharded level loop uses, resolved at run time.
//
// libraftmc does not link RCCL: single-GPU runs and the CLI never need it.  The first
// mc_rccl_unique_id / mc_shard_run_rccl call dlopen()s "librccl.so.1"; inside a
// torch.distributed job that is the copy torch already loaded (same soname), so the
// process holds one RCCL.  Types come from the ROCm header; only symbols are deferred.
#pragma once
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <rccl/rccl.h>

#include <string>
#include <thread>
#include <vector>

namespace rmc {

struct RcclApi {
  ncclResult_t (*GetUniqueId)(ncclUniqueId*) = nullptr;
  ncclResult_t (*CommInitRank)(ncclComm_t*, int, ncclUniqueId, int) = nullptr;
  ncclResult_t (*CommInitAll)(ncclComm_t*, int, const int*) = nullptr;   // one process, one rank per device
  ncclResult_t (*CommDestroy)(ncclComm_t) = nullptr;
  ncclResult_t (*CommAbort)(ncclComm_t) = nullptr;     // releases peers blocked in this comm's kernels
  ncclResult_t (*GroupStart)() = nullptr;
  ncclResult_t (*GroupEnd)() = nullptr;
  ncclResult_t (*Send)(const void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*Recv)(void*, size_t, ncclDataType_t, int, ncclComm_t, hipStream_t) = nullptr;
  ncclResult_t (*AllReduce)(const void*, void*, size_t, ncclDataType_t, ncclRedOp_t, ncclComm_t, hipStream_t) = nullptr;
  const char* (*GetErrorString)(ncclResult_t) = nullptr;
  // non-blocking communicators (ncclConfig_t.blocking = 0, rccl.h:93): every call returns at once,
  // ncclCommGetAsyncError (rccl.h:362) reports ncclInProgress until the work is enqueued and a peer's
  // failure afterwards; optional symbols (nullptr: the blocking calls above are used)
  ncclResult_t (*CommInitRankConfig)(ncclComm_t*, int, ncclUniqueId, int, ncclConfig_t*) = nullptr;
  ncclResult_t (*CommGetAsyncError)(ncclComm_t, ncclResult_t*) = nullptr;
  bool ok = false;
  bool nonblocking() const { return CommInitRankConfig && CommGetAsyncError; }

  // 0 on success; err names what is missing
  int load(std::string& err) {
    if (ok) return 0;
    void* h = dlopen("librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) h = dlopen("/opt/rocm/lib/librccl.so.1", RTLD_NOW | RTLD_GLOBAL);
    if (!h) { err = std::string("cannot load RCCL (librccl.so.1): ") + dlerror(); return -1; }
#define RMC_SYM(f, name)                                                       \
  f = reinterpret_cast<decltype(f)>(dlsym(h, name));                           \
  if (!f) { err = std::string("RCCL symbol missing: ") + name; return -1; }
    RMC_SYM(GetUniqueId, "ncclGetUniqueId");
    RMC_SYM(CommInitRank, "ncclCommInitRank");
    RMC_SYM(CommInitAll, "ncclCommInitAll");
    RMC_SYM(CommDestroy, "ncclCommDestroy");
    RMC_SYM(CommAbort, "ncclCommAbort");
    RMC_SYM(GroupStart, "ncclGroupStart");
    RMC_SYM(GroupEnd, "ncclGroupEnd");
    RMC_SYM(Send, "ncclSend");
    RMC_SYM(Recv, "ncclRecv");
    RMC_SYM(AllReduce, "ncclAllReduce");
    RMC_SYM(GetErrorString, "ncclGetErrorString");
#undef RMC_SYM
    CommInitRankConfig = reinterpret_cast<decltype(CommInitRankConfig)>(dlsym(h, "ncclCommInitRankConfig"));
    CommGetAsyncError = reinterpret_cast<decltype(CommGetAsyncError)>(dlsym(h, "ncclCommGetAsyncError"));
    ok = true;
    return 0;
  }
};

inline RcclApi& rccl() {
  static RcclApi api;
  return api;
}

// Wait until a non-blocking communicator has left ncclInProgress (its init, or the group just ended
// on it, is enqueued); `stop` is polled between the checks (true: give up, the caller's peers are
// gone).  0, or -1 with err set (the communicator's asynchronous error, or stopped).
template <class Stop>
inline int rccl_settle(ncclComm_t comm, Stop&& stop, std::string& err) {
  RcclApi& R = rccl();
  if (!R.nonblocking()) return 0;
  for (;;) {
    ncclResult_t st = ncclSuccess;
    const ncclResult_t r = R.CommGetAsyncError(comm, &st);
    if (r != ncclSuccess) { err = std::string("ncclCommGetAsyncError: ") + R.GetErrorString(r); return -1; }
    if (st == ncclSuccess) return 0;
    if (st != ncclInProgress) { err = std::string("RCCL: ") + R.GetErrorString(st); return -1; }
    if (stop()) { err = "RCCL: another rank left the loop (communicators aborted)"; return -1; }
    std::this_thread::yield();
  }
}

// A communicator for rank `rank` of `nranks` on the current device: non-blocking when the library has
// ncclCommInitRankConfig (so no later call blocks the calling thread: a failed peer never leaves a
// rank stuck inside RCCL, shard_transport.h), settled before it is returned
inline int rccl_init_rank(ncclComm_t* comm, int nranks, const ncclUniqueId& id, int rank, std::string& err) {
  RcclApi& R = rccl();
  *comm = nullptr;
  ncclResult_t r;
  if (R.nonblocking()) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    r = R.CommInitRankConfig(comm, nranks, id, rank, &cfg);
    if (r == ncclInProgress) r = ncclSuccess;
  } else {
    r = R.CommInitRank(comm, nranks, id, rank);
  }
  if (r != ncclSuccess) { err = std::string("ncclCommInitRank: ") + R.GetErrorString(r); *comm = nullptr; return -1; }
  if (rccl_settle(*comm, [] { return false; }, err)) { (void)R.CommAbort(*comm); *comm = nullptr; return -1; }
  return 0;
}

// One communicator per device of this process (mc_opts.n_gpus): non-blocking ones through one group of
// ncclCommInitRankConfig calls when available, else ncclCommInitAll (blocking)
inline int rccl_init_all(std::vector<ncclComm_t>& comms, const std::vector<int>& dev, std::string& err) {
  RcclApi& R = rccl();
  const int W = (int)dev.size();
  comms.assign(W, nullptr);
  if (!R.nonblocking()) {
    const ncclResult_t r = R.CommInitAll(comms.data(), W, dev.data());
    if (r != ncclSuccess) { err = std::string("ncclCommInitAll: ") + R.GetErrorString(r); comms.clear(); return -1; }
    return 0;
  }
  ncclUniqueId id;
  ncclResult_t r = R.GetUniqueId(&id);
  if (r != ncclSuccess) { err = std::string("ncclGetUniqueId: ") + R.GetErrorString(r); comms.clear(); return -1; }
  int cur = 0;
  (void)hipGetDevice(&cur);
  r = R.GroupStart();
  for (int k = 0; k < W && (r == ncclSuccess || r == ncclInProgress); ++k) {
    ncclConfig_t cfg = NCCL_CONFIG_INITIALIZER;
    cfg.blocking = 0;
    if (hipSetDevice(dev[k]) != hipSuccess) { r = ncclInvalidArgument; break; }
    r = R.CommInitRankConfig(&comms[k], W, id, k, &cfg);
  }
  const ncclResult_t r2 = R.GroupEnd();
  (void)hipSetDevice(cur);
  bool bad = (r != ncclSuccess && r != ncclInProgress) || (r2 != ncclSuccess && r2 != ncclInProgress);
  for (int k = 0; k < W && !bad; ++k) bad = !comms[k] || rccl_settle(comms[k], [] { return false; }, err) != 0;
  if (bad) {
    if (err.empty()) err = std::string("ncclCommInitRankConfig: ") + R.GetErrorString(r != ncclSuccess && r != ncclInProgress ? r : r2);
    for (ncclComm_t& c : comms) if (c) (void)R.CommAbort(c);
    comms.clear();
    return -1;
  }
  return 0;
}

}  // namespace rmc
