// raftmc — gfx950 BFS backend for thirdparty/raft_original.tla.
//
// One BFS level is processed in frontier chunks; each chunk runs three
// kernels on one stream:
//
//  1. orig_generate  (compute): one lane per frontier state, a wave-uniform
//     loop over the Next relation's action instances (every lane of a wave
//     runs the same action code on a different state).  Each enabled
//     successor is constraint-filtered, canonically packed and fingerprinted
//     (FP64); the fingerprint goes to an instance-major slot array
//     cand[k][state] (0 = no in-model successor), so the stores of a wave are
//     contiguous and no atomic is needed.  Out-of-model successors get their
//     invariant check here (TLC semantics, [ext] switch).
//  2. orig_dedup     (HBM random access): each thread takes 16 slots, issues
//     their 16 independent seen-set loads together, then the atomicCAS
//     inserts of the empty ones together (lock-free open addressing over u64
//     fingerprints, linear probing); the new slots of a 4096-slot tile are
//     compacted with one global atomic per tile into (parent, instance)
//     records.
//  3. orig_materialize: one lane per new state re-derives it from
//     (parent, instance), stores the packed state + parent pointer into the
//     HBM-resident state store and checks the invariants.
//
// All distinct states stay resident in HBM; counterexamples are read back by
// chasing parent pointers (no host replay).
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

enum {
  K_NEW = 0, K_GEN_IN = 1, K_ERR = 2, K_VIOL = 3, K_ERRGID = 4, K_DEADLOCK = 5, K_CHUNK_NEW = 6,
  K_ACT = 8, K_NCTR = K_ACT + 2 * OA_NACT
};
enum { OE_CAP_STORE = 0x100, OE_TABLE_FULL = 0x200 };
constexpr int DEDUP_PER = 16;      // slots per dedup thread (independent probes in flight)
constexpr int BS = 256;            // workgroup size of every kernel (4 waves)

template <class S>
struct ViolRec {
  u64 parent;
  u32 act, inst, bad, inmodel;
  typename S::Work w;
};

struct GenArgs {
  const u32* states;           // [cap][NWP]
  u64 chunk_begin, chunk_count;
  u64* cand;                   // [NI][chunk_count] fingerprints, 0 = none
  u64 seed;
  OrigRuntime rt;
  u32 inv_oom;
  unsigned long long* ctr;
  void* viol;
};

template <class S>
__global__ void __launch_bounds__(BS) orig_generate(GenArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  __shared__ unsigned int lds_cnt[OA_NACT + 1];
  for (int t = threadIdx.x; t < OA_NACT + 1; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 tid = (u64)blockIdx.x * BS + threadIdx.x;
  const bool active = tid < a.chunk_count;
  const u64 gid = a.chunk_begin + tid;
  W s;
  u64 al[S::AW];
  u32 err = 0, nsucc = 0;
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
  for (int k = 0; k < S::NI; ++k) {
    W t;
    const int act = active ? S::apply(s, k, t, err) : -1;
    u64 fp = 0;
    if (act >= 0) {
#pragma unroll
      for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
      ++nsucc;
      atomicAdd(&lds_cnt[act], 1u);
      if (S::in_model(t, a.rt)) {
        atomicAdd(&lds_cnt[OA_NACT], 1u);
        u32 pw[NW];
        S::pack(t, pw);
        fp = fp64(pw, a.seed);
      } else if (a.inv_oom) {
        const u32 bad = S::violated(t, a.rt.invariants);
        if (bad && atomicCAS(&a.ctr[K_VIOL], 0ull, 1ull) == 0ull) {
          ViolRec<S>* v = reinterpret_cast<ViolRec<S>*>(a.viol);
          v->parent = gid; v->act = (u32)act; v->inst = (u32)k; v->bad = bad; v->inmodel = 0; v->w = t;
        }
      }
    }
    if (active) a.cand[(u64)k * a.chunk_count + tid] = fp;
  }
  if (active && nsucc == 0) atomicCAS(&a.ctr[K_DEADLOCK], 0ull, (unsigned long long)(gid + 1));
  if (err) {
    atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
    atomicCAS(&a.ctr[K_ERRGID], 0ull, (unsigned long long)(gid + 1));
  }
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + t], (unsigned long long)lds_cnt[t]);
  if (threadIdx.x == 0 && lds_cnt[OA_NACT]) atomicAdd(&a.ctr[K_GEN_IN], (unsigned long long)lds_cnt[OA_NACT]);
}

struct DedupArgs {
  const u64* cand;
  u64 nslots, chunk_begin, chunk_count;
  u64* table;
  u64 table_mask;
  u64* newrec;                 // (parent gid << 8 | instance), compacted
  unsigned long long* ctr;
};

__global__ void __launch_bounds__(BS) orig_dedup(DedupArgs a) {
  __shared__ unsigned int wave_tot[BS / 64];
  __shared__ unsigned long long base_sh;
  const u64 tile = (u64)blockIdx.x * (BS * DEDUP_PER);
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  u64 fp[DEDUP_PER], cur[DEDUP_PER];
  // 1. slot loads (coalesced), then all seen-set loads back to back
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j) {
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    fp[j] = idx < a.nslots ? a.cand[idx] : 0ull;
  }
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j) cur[j] = fp[j] ? a.table[fp[j] & a.table_mask] : ~0ull;
  // 2. CAS the empty home slots together
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j)
    if (fp[j] && cur[j] == 0ull)
      cur[j] = (u64)atomicCAS((unsigned long long*)&a.table[fp[j] & a.table_mask], 0ull, (unsigned long long)fp[j]);
  // 3. resolve; a home slot owned by another fingerprint continues linear probing
  u32 isnew = 0, err = 0;
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j) {
    if (!fp[j]) continue;
    if (cur[j] == 0ull) { isnew |= 1u << j; continue; }       // our CAS won on an empty home slot
    if (cur[j] == fp[j]) continue;                            // seen (or lost the CAS race to an equal fp)
    u64 slot = (fp[j] + 1) & a.table_mask;
    for (int probe = 0;; ++probe) {
      if (probe >= (1 << 20)) { err |= OE_TABLE_FULL; break; }
      const u64 c = a.table[slot];
      if (c == fp[j]) break;
      if (c == 0ull) {
        const u64 old = (u64)atomicCAS((unsigned long long*)&a.table[slot], 0ull, (unsigned long long)fp[j]);
        if (old == 0ull) { isnew |= 1u << j; break; }
        if (old == fp[j]) break;
      }
      slot = (slot + 1) & a.table_mask;
    }
  }
  // 4. tile compaction: wave prefix sums, one global atomic per tile
  const unsigned int mine = (unsigned int)__popc(isnew);
  unsigned int incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) { const unsigned int v = __shfl_up(incl, d); if (lane >= d) incl += v; }
  if (lane == 63) wave_tot[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int tot = 0;
    for (int w = 0; w < BS / 64; ++w) { const unsigned int x = wave_tot[w]; wave_tot[w] = tot; tot += x; }
    base_sh = tot ? atomicAdd(&a.ctr[K_CHUNK_NEW], (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  u64 pos = base_sh + wave_tot[wave] + (incl - mine);
  for (int j = 0; j < DEDUP_PER; ++j) {
    if (!((isnew >> j) & 1u)) continue;
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    const u64 k = idx / a.chunk_count, st = idx - k * a.chunk_count;
    a.newrec[pos++] = ((a.chunk_begin + st) << 8) | k;
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
}

struct MatArgs {
  u32* states;
  u64* meta;
  const u64* newrec;
  u64 n_new, dst_base, cap;
  OrigRuntime rt;
  unsigned long long* ctr;
  void* viol;
};

template <class S>
__global__ void __launch_bounds__(BS) orig_materialize(MatArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  __shared__ unsigned int lds_cnt[OA_NACT];
  for (int t = threadIdx.x; t < OA_NACT; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  u32 err = 0;
  if (i < a.n_new) {
    const u64 rec = a.newrec[i], gid = rec >> 8;
    const int k = (int)(rec & 0xff);
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(a.states + gid * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    W s, t;
    u64 al[S::AW];
    S::unpack(w, s);
    S::all_logs_next(s, al);
    const int act = S::apply(s, k, t, err);
#pragma unroll
    for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
    u32 pw[NW];
    S::pack(t, pw);
    const u64 dst = a.dst_base + i;
    if (act >= 0 && dst < a.cap) {
      uint4* o = reinterpret_cast<uint4*>(a.states + dst * NWP);
#pragma unroll
      for (int q = 0; q < NWP / 4; ++q)
        o[q] = make_uint4(pw[4 * q], 4 * q + 1 < NW ? pw[4 * q + 1] : 0u, 4 * q + 2 < NW ? pw[4 * q + 2] : 0u, 4 * q + 3 < NW ? pw[4 * q + 3] : 0u);
      a.meta[dst] = (gid << 24) | ((u64)act << 16) | (u64)k;
      atomicAdd(&lds_cnt[act], 1u);
      const u32 bad = S::violated(t, a.rt.invariants);
      if (bad && atomicCAS(&a.ctr[K_VIOL], 0ull, 1ull) == 0ull) {
        ViolRec<S>* v = reinterpret_cast<ViolRec<S>*>(a.viol);
        v->parent = gid; v->act = (u32)act; v->inst = (u32)k; v->bad = bad; v->inmodel = 1; v->w = t;
      }
    } else {
      err |= dst >= a.cap ? (u32)OE_CAP_STORE : (u32)OE_EVAL_LOG_INDEX;
    }
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + OA_NACT + t], (unsigned long long)lds_cnt[t]);
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
      uint64_t sb = o.state_store_bytes ? o.state_store_bytes : std::min<uint64_t>(32ull << 30, freeb / 3);
      cap_ = sb / (NWP * 4 + 8);
      if (cap_ < 16) cap_ = 16;
      // frontier chunk: the slot array holds chunk_states * NI fingerprints,
      // the record array as many (worst case: every slot new); ~1/8 of the store
      chunk_states_ = std::max<u64>(4096, std::min<u64>(cap_, (sb / 8) / (16 * (u64)S::NI)));
      table_mask_ = slots - 1;
      HIPCHK(hipMalloc(&d_table_, slots * 8));
      HIPCHK(hipMalloc(&d_states_, cap_ * NWP * 4));
      HIPCHK(hipMalloc(&d_meta_, cap_ * 8));
      HIPCHK(hipMalloc(&d_cand_, chunk_states_ * S::NI * 8));
      HIPCHK(hipMalloc(&d_newrec_, chunk_states_ * S::NI * 8));
      HIPCHK(hipMalloc(&d_ctr_, K_NCTR * 8));
      HIPCHK(hipMalloc(&d_viol_, sizeof(ViolRec<S>)));
      HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
      for (auto& e : ev_) HIPCHK(hipEventCreate(&e));
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
    r.kernels = {{"orig_generate", 0, 0, 0}, {"orig_dedup", 0, 0, 0}, {"orig_materialize", 0, 0, 0}};

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

    const u64 S_B = NWP * 4;
    u64 level_begin = 0, level_count = 1;
    while (level_count > 0) {
      if (o.max_depth && r.depth >= o.max_depth) { r.left_on_queue = (int64_t)level_count; r.verdict = MC_VERDICT_DEPTH_LIMIT; break; }
      HIPCHK(hipMemsetAsync(d_ctr_, 0, K_NCTR * 8, stream_));
      u64 next_write = level_begin + level_count;
      double level_ms = 0;
      for (u64 cb = level_begin; cb < level_begin + level_count; cb += chunk_states_) {
        const u64 cnt = std::min<u64>(chunk_states_, level_begin + level_count - cb);
        const u64 nslots = cnt * (u64)S::NI;
        HIPCHK(hipMemsetAsync(d_ctr_ + K_CHUNK_NEW, 0, 8, stream_));
        GenArgs g;
        g.states = d_states_; g.chunk_begin = cb; g.chunk_count = cnt; g.cand = d_cand_; g.seed = r.seed; g.rt = m_.rt;
        g.inv_oom = o.inv_out_of_model ? 1u : 0u; g.ctr = (unsigned long long*)d_ctr_; g.viol = d_viol_;
        DedupArgs d;
        d.cand = d_cand_; d.nslots = nslots; d.chunk_begin = cb; d.chunk_count = cnt; d.table = d_table_;
        d.table_mask = table_mask_; d.newrec = d_newrec_; d.ctr = (unsigned long long*)d_ctr_;
        HIPCHK(hipEventRecord(ev_[0], stream_));
        hipLaunchKernelGGL((orig_generate<S>), dim3((unsigned)((cnt + BS - 1) / BS)), dim3(BS), 0, stream_, g);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev_[1], stream_));
        hipLaunchKernelGGL(orig_dedup, dim3((unsigned)((nslots + BS * DEDUP_PER - 1) / (BS * DEDUP_PER))), dim3(BS), 0, stream_, d);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev_[2], stream_));
        u64 nnew = 0;
        HIPCHK(hipMemcpyAsync(&nnew, d_ctr_ + K_CHUNK_NEW, 8, hipMemcpyDeviceToHost, stream_));
        HIPCHK(hipStreamSynchronize(stream_));
        float ms_g = 0, ms_d = 0, ms_m = 0;
        HIPCHK(hipEventElapsedTime(&ms_g, ev_[0], ev_[1]));
        HIPCHK(hipEventElapsedTime(&ms_d, ev_[1], ev_[2]));
        if (nnew) {
          MatArgs m;
          m.states = d_states_; m.meta = d_meta_; m.newrec = d_newrec_; m.n_new = nnew; m.dst_base = next_write; m.cap = cap_;
          m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_; m.viol = d_viol_;
          HIPCHK(hipEventRecord(ev_[3], stream_));
          hipLaunchKernelGGL((orig_materialize<S>), dim3((unsigned)((nnew + BS - 1) / BS)), dim3(BS), 0, stream_, m);
          HIPCHK(hipGetLastError());
          HIPCHK(hipEventRecord(ev_[4], stream_));
          HIPCHK(hipEventSynchronize(ev_[4]));
          HIPCHK(hipEventElapsedTime(&ms_m, ev_[3], ev_[4]));
          r.kernels[2].ms += ms_m; r.kernels[2].launches += 1;
          r.kernels[2].algo_bytes += (double)nnew * (8 + S_B + S_B + 8);
        }
        next_write += nnew;
        level_ms += ms_g + ms_d + ms_m;
        r.kernels[0].ms += ms_g; r.kernels[0].launches += 1;
        r.kernels[0].algo_bytes += (double)cnt * S_B + (double)nslots * 8;
        r.kernels[1].ms += ms_d; r.kernels[1].launches += 1;
        r.kernels[1].algo_bytes += (double)nslots * 8 + (double)nnew * 16;   // + G_in*8 probe bytes added per level below
        if (next_write > cap_) break;
      }
      u64 c[K_NCTR];
      HIPCHK(hipMemcpyAsync(c, d_ctr_, sizeof c, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
      int64_t gen = 0;
      for (int k = 0; k < OA_NACT; ++k) { r.act_generated[k] += (int64_t)c[K_ACT + k]; r.act_distinct[k] += (int64_t)c[K_ACT + OA_NACT + k]; gen += (int64_t)c[K_ACT + k]; }
      r.generated += gen;
      r.generated_in_model += (int64_t)c[K_GEN_IN];
      r.kernels[1].algo_bytes += (double)c[K_GEN_IN] * 8;
      r.seconds_kernels += level_ms / 1000.0;
      r.n_launches += 1;
      const u64 nnew = next_write - (level_begin + level_count);
      r.algo_bytes += (double)level_count * S_B + (double)c[K_GEN_IN] * 8 + (double)nnew * (16 + S_B);
      if (next_write > cap_) c[K_ERR] |= OE_CAP_STORE;
      if (c[K_ERR]) {
        const u64 e = c[K_ERR];
        r.verdict = (e & (OE_CAP_STORE | OE_TABLE_FULL | OE_CAP_ELECTIONS | OE_CAP_COUNT)) ? MC_VERDICT_CAPACITY_OVERFLOW : MC_VERDICT_EVAL_ERROR;
        std::ostringstream os;
        os << "error flags 0x" << std::hex << e << std::dec << " while expanding state " << (c[K_ERRGID] ? (int64_t)c[K_ERRGID] - 1 : -1) << ":";
        if (e & OE_EVAL_LOG_INDEX) os << " log[i][prevLogIndex] applied outside its domain (raft_original.tla:207-210);";
        if (e & OE_CAP_ELECTIONS) os << " elections set exceeds the compiled capacity;";
        if (e & OE_CAP_COUNT) os << " message count / bag capacity exceeded;";
        if (e & OE_CAP_STORE) os << " state store full (raise state_store_bytes);";
        if (e & OE_TABLE_FULL) os << " fingerprint table full (raise fp_table_bytes);";
        r.error = os.str();
        total_ = std::min<u64>(next_write, cap_);
        r.distinct = (int64_t)total_;
        break;
      }
      total_ += nnew;
      r.distinct = (int64_t)total_;
      r.levels.back().generated = gen;
      r.levels.back().kernel_ms = level_ms;
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
  u64* d_cand_ = nullptr; u64* d_newrec_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_[5] = {nullptr, nullptr, nullptr, nullptr, nullptr};
  u64 table_mask_ = 0, cap_ = 0, total_ = 0, chunk_states_ = 0;
  int dev_ = -1; uint64_t req_table_ = 0, req_store_ = 0;

  void release() {
    for (void* p : {(void*)d_table_, (void*)d_states_, (void*)d_meta_, (void*)d_ctr_, d_viol_, (void*)d_cand_, (void*)d_newrec_})
      if (p) (void)hipFree(p);
    for (auto& e : ev_) { if (e) (void)hipEventDestroy(e); e = nullptr; }
    if (stream_) (void)hipStreamDestroy(stream_);
    d_table_ = nullptr; d_states_ = nullptr; d_meta_ = nullptr; d_ctr_ = nullptr; d_viol_ = nullptr;
    d_cand_ = nullptr; d_newrec_ = nullptr; stream_ = nullptr;
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
