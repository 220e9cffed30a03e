// raftmc: the RCCL entry points the native sharded level loop uses, resolved at run time.
//
// libraftmc does not link RCCL: single-GPU runs and the CLI never need it.  The first
// mc_rccl_unique_id / mc_shard_run_rccl call dlopen()s "librccl.so.1"; inside a
// torch.distributed job that is the copy torch already loaded (same soname), so the
// process holds one RCCL.  Types come from the ROCm header; only symbols are deferred.
#pragma once
#include <dlfcn.h>
#include <rccl/rccl.h>

#include <string>

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
  bool ok = false;

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
    ok = true;
    return 0;
  }
};

inline RcclApi& rccl() {
  static RcclApi api;
  return api;
}

}  // namespace rmc
