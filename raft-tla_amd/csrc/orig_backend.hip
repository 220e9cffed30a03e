// raftmc — gfx950 BFS backend for thirdparty/raft_original.tla.
//
// One BFS level = one launch of orig_expand: one lane per frontier state, a
// wave-uniform loop over the Next relation's action instances (so every lane
// of a wave runs the same action code on a different state), and for every
// successor: constraint filter -> canonical pack -> FP64 -> lock-free
// open-addressing insert (atomicCAS on u64 slots) -> invariant check on
// !seen states -> wave-aggregated slot allocation (ballot + one atomic per
// wave per instance) and a 16-B-vector store of the new state and its
// parent pointer.  All distinct states stay resident in HBM (the trace is
// read back by chasing parent pointers; no host replay).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <functional>
#include <map>
#include <sstream>

#include "../../include/raftmc.h"
#include "backend.h"
#include "orig_spec.h"
#include "orig_text.h"

namespace rmc {

enum { K_NEW = 0, K_GEN_IN = 1, K_ERR = 2, K_VIOL = 3, K_ERRGID = 4, K_DEADLOCK = 5, K_ACT = 8, K_NCTR = K_ACT + 2 * OA_NACT };
enum { OE_CAP_STORE = 0x100, OE_TABLE_FULL = 0x200 };

struct ExpandArgs {
  u32* states;                 // [cap][NWP] packed states, all levels
  u64* meta;                   // [cap] parent_gid << 24 | action << 16 | instance
  u64 level_begin, level_count, next_base, cap;
  u64* table;                  // seen-set, 0 = empty
  u64 table_mask;
  u64 seed;
  OrigRuntime rt;
  u32 inv_oom;
  unsigned long long* ctr;     // K_* counters
  void* viol;                  // ViolRec<S>
};

template <class S>
struct ViolRec {
  u64 parent;
  u32 act, inst, bad, inmodel;
  typename S::Work w;
};

__device__ __forceinline__ bool seen_insert(u64* table, u64 mask, u64 fp, u32& err) {
  u64 slot = fp & mask;
  for (int probe = 0; probe < (1 << 20); ++probe) {
    const u64 cur = table[slot];                   // insert-only table: a non-zero read is final
    if (cur == fp) return false;
    if (cur == 0) {
      const unsigned long long old = atomicCAS((unsigned long long*)&table[slot], 0ull, (unsigned long long)fp);
      if (old == 0ull) return true;
      if (old == (unsigned long long)fp) return false;
    }
    slot = (slot + 1) & mask;
  }
  err |= OE_TABLE_FULL;
  return false;
}

template <class S, int BS>
__global__ void __launch_bounds__(BS) orig_expand(ExpandArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  __shared__ unsigned int lds_cnt[2 * OA_NACT + 1];
  for (int t = threadIdx.x; t < 2 * OA_NACT + 1; t += BS) lds_cnt[t] = 0;
  __syncthreads();

  const u64 tid = (u64)blockIdx.x * BS + threadIdx.x;
  const bool active = tid < a.level_count;
  const u64 gid = a.level_begin + tid;
  W s;
  u64 al[S::AW];
  u32 err = 0;
  if (active) {
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(a.states + gid * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    S::unpack(w, s);
    S::all_logs_next(s, al);
  } else {
    S::init(s);
#pragma unroll
    for (int q = 0; q < S::AW; ++q) al[q] = 0;
  }
  u32 nsucc = 0;
  const int lane = __lane_id();
  for (int k = 0; k < S::NI; ++k) {
    W t;
    const int act = active ? S::apply(s, k, t, err) : -1;
    const bool ok = act >= 0;
    bool isnew = false;
    u32 w[NWP];
#pragma unroll
    for (int q = 0; q < NWP; ++q) w[q] = 0;
    if (ok) {
#pragma unroll
      for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
      ++nsucc;
      atomicAdd(&lds_cnt[act], 1u);
      const bool inm = S::in_model(t, a.rt);
      if (inm) {
        atomicAdd(&lds_cnt[2 * OA_NACT], 1u);
        u32 pw[NW];
        S::pack(t, pw);
#pragma unroll
        for (int q = 0; q < NW; ++q) w[q] = pw[q];
        const u64 fp = fp64(pw, a.seed);
        isnew = seen_insert(a.table, a.table_mask, fp, err);
        if (isnew) atomicAdd(&lds_cnt[OA_NACT + act], 1u);
      }
      if (isnew || (!inm && a.inv_oom)) {
        const u32 bad = S::violated(t, a.rt.invariants);
        if (bad && atomicCAS(&a.ctr[K_VIOL], 0ull, 1ull) == 0ull) {
          ViolRec<S>* v = reinterpret_cast<ViolRec<S>*>(a.viol);
          v->parent = gid; v->act = (u32)act; v->inst = (u32)k; v->bad = bad; v->inmodel = inm; v->w = t;
        }
      }
    }
    const u64 m = __ballot(isnew);
    if (m) {
      const int leader = __ffsll((unsigned long long)m) - 1;
      unsigned long long base = 0;
      if (lane == leader) base = atomicAdd(&a.ctr[K_NEW], (unsigned long long)__popcll(m));
      base = __shfl(base, leader);
      if (isnew) {
        const u64 dst = a.next_base + base + (u64)__popcll(m & ((1ull << lane) - 1ull));
        if (dst < a.cap) {
          uint4* o = reinterpret_cast<uint4*>(a.states + dst * NWP);
#pragma unroll
          for (int q = 0; q < NWP / 4; ++q) o[q] = make_uint4(w[4 * q], w[4 * q + 1], w[4 * q + 2], w[4 * q + 3]);
          a.meta[dst] = (gid << 24) | ((u64)act << 16) | (u64)k;
        } else {
          err |= OE_CAP_STORE;
        }
      }
    }
  }
  if (active && nsucc == 0) atomicCAS(&a.ctr[K_DEADLOCK], 0ull, (unsigned long long)(gid + 1));
  if (err) {
    atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
    atomicCAS(&a.ctr[K_ERRGID], 0ull, (unsigned long long)(gid + 1));
  }
  __syncthreads();
  for (int t = threadIdx.x; t < 2 * OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + t], (unsigned long long)lds_cnt[t]);
  if (threadIdx.x == 0 && lds_cnt[2 * OA_NACT]) atomicAdd(&a.ctr[K_GEN_IN], (unsigned long long)lds_cnt[2 * OA_NACT]);
}

#define HIPCHK(x)                                                                             \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); return MC_E_NO_DEVICE; } \
  } while (0)

template <class S>
class OrigGpu : public Backend {
 public:
  using W = typename S::Work;
  static constexpr int NWP = (S::NW + 3) & ~3;
  explicit OrigGpu(const OrigModel& m) : m_(m) {}
  ~OrigGpu() override { release(); }

  std::string family() const override { return "raft_original"; }

  std::string describe_json() const override {
    std::ostringstream o;
    o << "{\"spec\": \"raft_original\", \"N\": " << S::N << ", \"NV\": " << S::NV << ", \"MaxTerm\": " << S::MT
      << ", \"MaxLogLen\": " << S::ML << ", \"MaxMsgDomain\": " << S::MK << ", \"MinMsgCount\": " << m_.rt.min_count
      << ", \"MaxMsgCount\": " << m_.rt.max_count << ", \"state_bits\": " << S::PBITS << ", \"state_words\": " << S::NW
      << ", \"state_bytes_stored\": " << NWP * 4 << ", \"instances\": " << S::NI << ", \"log_universe\": " << S::U
      << ", \"constraints\": [";
    for (size_t k = 0; k < m_.constraint_names.size(); ++k) o << (k ? ", " : "") << "\"" << m_.constraint_names[k] << "\"";
    o << "], \"invariants\": [";
    for (size_t k = 0; k < m_.inv_names.size(); ++k) o << (k ? ", " : "") << "\"" << m_.inv_names[k] << "\"";
    o << "], \"actions\": [";
    for (int k = 0; k < OA_NACT; ++k) o << (k ? ", " : "") << "\"" << kOrigActNames[k] << "\"";
    o << "]}";
    return o.str();
  }

  int run(const RunOpts& o, RunResult& r, std::string& err) override {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= o.device) { err = "no HIP device available (raftmc has no CPU fallback)"; return MC_E_NO_DEVICE; }
    HIPCHK(hipSetDevice(o.device));
    // ---- sizing; buffers are allocated on the first run and reused (a re-run
    // of the same handle re-zeroes the seen-set and overwrites the store)
    if (!d_table_ || o.device != dev_ || o.fp_table_bytes != req_table_ || o.state_store_bytes != req_store_) {
      release();
      size_t freeb = 0, totalb = 0;
      HIPCHK(hipMemGetInfo(&freeb, &totalb));
      uint64_t tb = o.fp_table_bytes ? o.fp_table_bytes : std::min<uint64_t>(8ull << 30, freeb / 4);
      uint64_t slots = 1; while (slots * 2 * 8 <= tb) slots *= 2;
      if (slots < 1024) slots = 1024;
      uint64_t sb = o.state_store_bytes ? o.state_store_bytes : std::min<uint64_t>(32ull << 30, freeb / 2);
      cap_ = sb / (NWP * 4 + 8);
      if (cap_ < 16) cap_ = 16;
      table_mask_ = slots - 1;
      HIPCHK(hipMalloc(&d_table_, slots * 8));
      HIPCHK(hipMalloc(&d_states_, cap_ * NWP * 4));
      HIPCHK(hipMalloc(&d_meta_, cap_ * 8));
      HIPCHK(hipMalloc(&d_ctr_, K_NCTR * 8));
      HIPCHK(hipMalloc(&d_viol_, sizeof(ViolRec<S>)));
      HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
      HIPCHK(hipEventCreate(&ev0_)); HIPCHK(hipEventCreate(&ev1_));
      dev_ = o.device; req_table_ = o.fp_table_bytes; req_store_ = o.state_store_bytes;
    }
    auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipMemsetAsync(d_table_, 0, (table_mask_ + 1) * 8, stream_));
    HIPCHK(hipStreamSynchronize(stream_));

    r = RunResult();
    r.seed = o.seed ? o.seed : 0x5EED5EED2024ull;
    r.state_bytes = NWP * 4;
    for (int k = 0; k < OA_NACT; ++k) r.action_names.push_back(kOrigActNames[k]);
    r.act_generated.assign(OA_NACT, 0); r.act_distinct.assign(OA_NACT, 0);

    // ---- Init (raft_original.tla:139-159): one state, generated and distinct
    W s0; S::init(s0);
    u32 w0[S::NW]; S::pack(s0, w0);
    u32 wp[NWP] = {0}; for (int q = 0; q < S::NW; ++q) wp[q] = w0[q];
    const u64 fp0 = fp64(w0, r.seed);
    HIPCHK(hipMemcpy(d_table_ + (fp0 & table_mask_), &fp0, 8, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_states_, wp, NWP * 4, hipMemcpyHostToDevice));
    const u64 nometa = ~0ull;
    HIPCHK(hipMemcpy(d_meta_, &nometa, 8, hipMemcpyHostToDevice));
    r.generated = 1; r.distinct = 1; total_ = 1;
    r.levels.push_back({1, 1, 0.0});
    r.depth = 1;
    if (!S::in_model(s0, m_.rt)) { err = "the initial state violates a state constraint"; r.verdict = MC_VERDICT_OK; r.distinct = 0; return 0; }
    if (u32 bad = S::violated(s0, m_.rt.invariants)) {
      r.verdict = MC_VERDICT_INVARIANT_VIOLATION; r.violated = first_violated(bad);
      r.trace.push_back({"<Initial predicate>", state_text(s0, true)});
      finish(r, t0); return 0;
    }

    u64 level_begin = 0, level_count = 1;
    while (level_count > 0) {
      if (o.max_depth && r.depth >= o.max_depth) { r.left_on_queue = (int64_t)level_count; r.verdict = MC_VERDICT_DEPTH_LIMIT; break; }
      HIPCHK(hipMemsetAsync(d_ctr_, 0, K_NCTR * 8, stream_));
      ExpandArgs a;
      a.states = d_states_; a.meta = d_meta_;
      a.level_begin = level_begin; a.level_count = level_count; a.next_base = level_begin + level_count; a.cap = cap_;
      a.table = d_table_; a.table_mask = table_mask_; a.seed = r.seed; a.rt = m_.rt;
      a.inv_oom = o.inv_out_of_model ? 1u : 0u; a.ctr = (unsigned long long*)d_ctr_; a.viol = d_viol_;
      const unsigned grid = (unsigned)((level_count + 255) / 256);
      HIPCHK(hipEventRecord(ev0_, stream_));
      hipLaunchKernelGGL((orig_expand<S, 256>), dim3(grid), dim3(256), 0, stream_, a);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(ev1_, stream_));
      u64 c[K_NCTR];
      HIPCHK(hipMemcpyAsync(c, d_ctr_, sizeof c, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
      float ms = 0; HIPCHK(hipEventElapsedTime(&ms, ev0_, ev1_));
      int64_t gen = 0;
      for (int k = 0; k < OA_NACT; ++k) { r.act_generated[k] += (int64_t)c[K_ACT + k]; r.act_distinct[k] += (int64_t)c[K_ACT + OA_NACT + k]; gen += (int64_t)c[K_ACT + k]; }
      r.generated += gen;
      r.generated_in_model += (int64_t)c[K_GEN_IN];
      r.seconds_kernels += ms / 1000.0;
      r.n_launches += 1;
      const u64 nnew = c[K_NEW];
      r.algo_bytes += (double)level_count * NWP * 4 + (double)c[K_GEN_IN] * 8 + (double)nnew * (16 + NWP * 4);
      if (c[K_ERR]) {
        const u64 e = c[K_ERR];
        r.verdict = (e & (OE_CAP_STORE | OE_TABLE_FULL | OE_CAP_ELECTIONS | OE_CAP_COUNT)) ? MC_VERDICT_CAPACITY_OVERFLOW : MC_VERDICT_EVAL_ERROR;
        std::ostringstream os;
        os << "error flags 0x" << std::hex << e << std::dec << " while expanding state " << (c[K_ERRGID] - 1) << ":";
        if (e & OE_EVAL_LOG_INDEX) os << " log[i][prevLogIndex] applied outside its domain (raft_original.tla:207-210);";
        if (e & OE_CAP_ELECTIONS) os << " elections set exceeds the compiled capacity;";
        if (e & OE_CAP_COUNT) os << " message count / bag capacity exceeded;";
        if (e & OE_CAP_STORE) os << " state store full (raise state_store_bytes);";
        if (e & OE_TABLE_FULL) os << " fingerprint table full (raise fp_table_bytes);";
        r.error = os.str();
        r.distinct = (int64_t)(total_ + std::min<u64>(nnew, cap_ - total_));
        break;
      }
      total_ += nnew;
      r.distinct = (int64_t)total_;
      r.levels.back().generated = gen;
      r.levels.back().kernel_ms = ms;
      if (nnew > 0) { r.levels.push_back({(int64_t)nnew, 0, 0.0}); r.depth += 1; }
      if (c[K_VIOL]) {
        ViolRec<S> v;
        HIPCHK(hipMemcpy(&v, d_viol_, sizeof v, hipMemcpyDeviceToHost));
        r.verdict = MC_VERDICT_INVARIANT_VIOLATION;
        r.violated = first_violated(v.bad);
        build_trace(v.parent, kOrigActNames[v.act], v.w, r, err);
        r.left_on_queue = (int64_t)nnew;
        break;
      }
      if (o.check_deadlock && c[K_DEADLOCK]) {
        r.verdict = MC_VERDICT_DEADLOCK;
        build_trace(c[K_DEADLOCK] - 1, nullptr, s0, r, err);
        r.left_on_queue = (int64_t)nnew;
        break;
      }
      level_begin += level_count;
      level_count = nnew;
    }
    finish(r, t0);
    return 0;
  }

  int dump_states(const std::string& path, std::string& err) override {
    if (!d_states_) { err = "mc_dump_states before mc_run"; return MC_E_STATE; }
    std::vector<u32> h(total_ * NWP);
    HIPCHK(hipMemcpy(h.data(), d_states_, h.size() * 4, hipMemcpyDeviceToHost));
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) { err = "cannot write " + path; return MC_E_IO; }
    for (u64 g = 0; g < total_; ++g) {
      u32 w[NWP];
      for (int q = 0; q < NWP; ++q) w[q] = h[g * NWP + q];
      W s; S::unpack(w, s);
      std::fprintf(f, "%s\n", state_text(s, false).c_str());
    }
    std::fclose(f);
    return 0;
  }

 private:
  OrigModel m_;
  u64* d_table_ = nullptr; u32* d_states_ = nullptr; u64* d_meta_ = nullptr; u64* d_ctr_ = nullptr; void* d_viol_ = nullptr;
  hipStream_t stream_ = nullptr; hipEvent_t ev0_ = nullptr, ev1_ = nullptr;
  u64 table_mask_ = 0, cap_ = 0, total_ = 0;
  int dev_ = -1; uint64_t req_table_ = 0, req_store_ = 0;

  void release() {
    if (d_table_) (void)hipFree(d_table_);
    if (d_states_) (void)hipFree(d_states_);
    if (d_meta_) (void)hipFree(d_meta_);
    if (d_ctr_) (void)hipFree(d_ctr_);
    if (d_viol_) (void)hipFree(d_viol_);
    if (ev0_) (void)hipEventDestroy(ev0_);
    if (ev1_) (void)hipEventDestroy(ev1_);
    if (stream_) (void)hipStreamDestroy(stream_);
    d_table_ = nullptr; d_states_ = nullptr; d_meta_ = nullptr; d_ctr_ = nullptr; d_viol_ = nullptr;
    ev0_ = ev1_ = nullptr; stream_ = nullptr;
  }

  std::string first_violated(u32 bad) const {
    for (auto& n : m_.inv_names) {
      const u32 bit = n == "ElectionSafety" ? OI_ElectionSafety : n == "LogMatching" ? OI_LogMatching : OI_NoLeader;
      if (bad & bit) return n;
    }
    return "?";
  }

  void finish(RunResult& r, std::chrono::steady_clock::time_point t0) {
    const double M = (double)r.distinct, Ng = (double)r.generated;
    r.collision_optimistic = M * (Ng - M) / 18446744073709551616.0;
    r.seconds_total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }

  // parent-pointer chase on the host (<= depth device reads of one state each)
  void build_trace(u64 parent, const char* last_act, const W& last, RunResult& r, std::string& err) {
    std::vector<std::pair<std::string, std::string>> tr;
    if (last_act) tr.push_back({last_act, state_text(last, true)});
    u64 g = parent;
    while (true) {
      u32 w[NWP]; u64 meta = 0;
      if (hipMemcpy(w, d_states_ + g * NWP, NWP * 4, hipMemcpyDeviceToHost) != hipSuccess ||
          hipMemcpy(&meta, d_meta_ + g, 8, hipMemcpyDeviceToHost) != hipSuccess) { err = "trace readback failed"; break; }
      W s; S::unpack(w, s);
      if (meta == ~0ull) { tr.push_back({"<Initial predicate>", state_text(s, true)}); break; }
      tr.push_back({kOrigActNames[(meta >> 16) & 0xff], state_text(s, true)});
      g = meta >> 24;
    }
    std::reverse(tr.begin(), tr.end());
    r.trace = tr;
  }

  std::string state_text(const W& s, bool multiline) const { return orig_state_text<S>(m_, s, multiline); }
};

// ------------------------------------------------------------------ shapes compiled into this build
// (N, NV, MaxTerm, MaxLogLen, MaxMsgDomain)
#ifdef RMC_QUICK_BUILD
#define RMC_ORIG_SHAPES(X) X(3, 2, 3, 2, 5)
#else
#define RMC_ORIG_SHAPES(X) \
  X(3, 1, 2, 1, 2) /* C1 */ \
  X(3, 2, 3, 2, 5) /* C2 */ \
  X(3, 2, 3, 2, 6)          \
  X(3, 2, 3, 2, 4)          \
  X(3, 2, 3, 2, 3)          \
  X(3, 2, 3, 2, 2)          \
  X(1, 2, 3, 2, 3)          \
  X(2, 1, 2, 1, 5)          \
  X(2, 1, 2, 1, 6)          \
  X(2, 1, 3, 2, 5)          \
  X(2, 2, 3, 2, 6)
#endif

static Backend* orig_factory(const OrigModel& m) {
#define X(n, nv, mt, ml, mk) \
  if (m.N == n && m.NV == nv && m.MT == mt && m.ML == ml && m.MK == mk) return new OrigGpu<Orig<n, nv, mt, ml, mk>>(m);
  RMC_ORIG_SHAPES(X)
#undef X
  return nullptr;
}

static std::string compiled_shapes() {
  std::string o;
#define X(n, nv, mt, ml, mk) o += std::string(o.empty() ? "" : ", ") + "(" #n "," #nv "," #mt "," #ml "," #mk ")";
  RMC_ORIG_SHAPES(X)
#undef X
  return o;
}

Backend* make_orig_backend(const CfgFile& cfg) {
  OrigModel m = resolve_orig_model(cfg);
  Backend* b = orig_factory(m);
  if (!b) {
    std::ostringstream os;
    os << "raft_original shape (N=" << m.N << ", NV=" << m.NV << ", MaxTerm=" << m.MT << ", MaxLogLen=" << m.ML
       << ", MaxMsgDomain=" << m.MK << ") is not compiled into this build; compiled shapes (N,NV,MaxTerm,MaxLogLen,MaxMsgDomain): "
       << compiled_shapes();
    throw CfgError(MC_E_UNSUPPORTED, os.str());
  }
  return b;
}

}  // namespace rmc
