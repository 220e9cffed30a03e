// raftmc — gfx950 BFS backend for thirdparty/raft_original.tla.
//
// One BFS level is processed in frontier chunks; each chunk runs three
// kernels on one stream:
//
//  1. orig_generate  (compute): one lane per frontier state, a wave-uniform
//     loop over the Next relation's action instances (every lane of a wave
//     runs the same action code on a different state); constraint filter,
//     TLC generated counts, out-of-model invariants (TLC semantics, [ext]
//     switch), canonical pack and FP64 of each in-model successor into the
//     slot array cand[block][instance][lane] (0 = none): coalesced, no atomics.
//  2. orig_dedup_blk (HBM random access): workgroup b takes generate
//     workgroup b's 256 parents, one per thread: coalesced slot loads, a
//     workgroup-local LDS fingerprint set drops the successors the 256
//     parents produce more than once (diamonds of commuting actions), the
//     rest probe the seen-set 16 at a time (lock-free open addressing over u64
//     fingerprints, linear probing, CAS insert); new states are numbered in
//     (parent, instance) order with one global atomic per workgroup, so the
//     next level is parent-major and its diamonds land in one workgroup again.
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
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <sstream>

#include "../../include/raftmc.h"
#include "backend.h"
#include "fp_gap.h"
#include "orig_spec.h"
#include "orig_text.h"
#include "rccl_api.h"

namespace rmc {

enum {
  K_NEW = 0, K_GEN_IN = 1, K_ERR = 2, K_VIOL = 3, K_ERRGID = 4, K_DEADLOCK = 5, K_CHUNK_NEW = 6, K_LEVEL_NEW = 7,
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

// One lane per frontier state, a wave-uniform loop over the action instances; successor,
// constraints, TLC generated counts, out-of-model invariants, canonical pack and FP64 in one
// pass; fingerprint slots written coalesced.  (A split expand + full-lane fingerprint
// pipeline measured 51.4 vs 49.4 ms/run on C2: apply, not the pack + hash, dominates this
// spec, so the split does not pay here.  Unrolling the ~50-instance loop is refused by the
// compiler at this body size.)
// PM (single-GPU pipeline): slots laid out per workgroup, cand[(block * NI + instance) * BS +
// lane] (coalesced stores), consumed by orig_dedup_blk one parent per thread, so the next level
// comes out parent-major (siblings adjacent) and the dedup workgroup can drop the successors its
// 256 parents produce more than once before they cost a seen-set probe.
//
// Workgroup-local fingerprint set (LDS): answers only "certainly produced here before"; when
// its probe window is full the successor goes to the global seen-set as usual.  A lane's
// "produced before" answer is only ever about an fp it reads back equal, so races (plain loads
// and stores, no atomics) can cost a probe but never lose a state.
constexpr int LDS_FP_SLOTS = 4096;   // 32 KB per workgroup
RMC_HD bool lds_first(unsigned long long* set, u64 fp) {
  // plain LDS loads and stores, no atomics: a race between two lanes can only make the set
  // forget an entry or let a duplicate through to the seen-set, never drop a new state
  u32 h = (u32)(fp >> 20) & (LDS_FP_SLOTS - 1);
#pragma unroll 1
  for (int p = 0; p < 8; ++p) {
    const unsigned long long cur = set[h];
    if (cur == fp) return false;            // produced here before
    if (cur == 0ull) { set[h] = fp; return true; }
    h = (h + 1) & (LDS_FP_SLOTS - 1);
  }
  return true;                              // window full: let the seen-set decide
}

template <class S, bool PM>
// 3 waves per SIMD (<= 168 VGPRs) measured fastest for C2's expand (19.9 vs 22.3 ms without the
// hint, 26.6 ms at the 2 waves the incremental fingerprint would otherwise get); larger states
// (C5: 24 words) would spill at 3 and get no hint.
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(S::NW <= 16 ? 3 : 1))) orig_generate(GenArgs a) {
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
  u32 err = 0, nsucc = 0, nin = 0;
  // the parent's packed words with allLogs' (every successor carries allLogs \cup {log[i]},
  // raft_original.tla:464) and their fingerprint terms: successors re-hash changed words only
  // (C5-sized states keep the plain hash: the base terms would cost them occupancy, measured
  // 45 vs 38 ms of expand time for C5 to depth 12)
  constexpr bool INC = NW <= 16;
  u32 bw[INC ? NW : 1];
  FpBase<INC ? NW : 2> fb;
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
  if constexpr (INC) {
    W b = s;
#pragma unroll
    for (int q = 0; q < S::AW; ++q) b.allLogs[q] = al[q];
    S::pack(b, bw);
    fb.init(bw, a.seed);
  }
#pragma unroll 1
  for (int k = 0; k < S::NI; ++k) {
    u64 fp = 0;
    if (active) {
      W t;
      const int act = S::apply(s, k, t, err);
      if (act >= 0) {
#pragma unroll
        for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
        ++nsucc;
        atomicAdd(&lds_cnt[act], 1u);
        if (S::in_model(t, a.rt)) {
          ++nin;
          u32 pw[NW];
          S::pack(t, pw);
          if constexpr (INC) fp = fb.fp(pw, bw, a.seed);
          else fp = fp64(pw, a.seed);
        } else if (a.inv_oom) {
          const u32 bad = S::violated(t, a.rt.invariants);
          if (bad && atomicCAS(&a.ctr[K_VIOL], 0ull, 1ull) == 0ull) {
            ViolRec<S>* v = reinterpret_cast<ViolRec<S>*>(a.viol);
            v->parent = gid; v->act = (u32)act; v->inst = (u32)k; v->bad = bad; v->inmodel = 0; v->w = t;
          }
        }
      }
      a.cand[PM ? ((u64)blockIdx.x * S::NI + (u64)k) * BS + threadIdx.x : (u64)k * a.chunk_count + tid] = fp;
    }
  }
  if (active && nsucc == 0) atomicCAS(&a.ctr[K_DEADLOCK], 0ull, (unsigned long long)(gid + 1));
  if (err) {
    atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
    atomicCAS(&a.ctr[K_ERRGID], 0ull, (unsigned long long)(gid + 1));
  }
  if (nin) atomicAdd(&lds_cnt[OA_NACT], nin);
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + t], (unsigned long long)lds_cnt[t]);
  if (threadIdx.x == 0 && lds_cnt[OA_NACT]) atomicAdd(&a.ctr[K_GEN_IN], (unsigned long long)lds_cnt[OA_NACT]);
}


struct DedupArgs {
  const u64* cand;
  u64 nslots, chunk_begin, chunk_count, ni;   // ni: instances per state (parent-major slot layout)
  u64* table;
  u64 table_mask;
  u64* newrec;                 // (parent gid << 8 | instance), compacted
  unsigned long long* ctr;
};

// Seen-set insertion for the PM layout: workgroup b takes generate-workgroup b's slots, one
// parent per thread; its NI slot loads are coalesced across the wave, its probes go out in
// groups of 16, and its new states are numbered in (parent, instance) order by a workgroup scan
// and one global atomic, so the next level is parent-major.
template <int NI>
__global__ void __launch_bounds__(BS) orig_dedup_blk(DedupArgs a) {
  static_assert(NI <= 128, "new-state bits are two u64 per parent");
  __shared__ unsigned int wave_tot[BS / 64];
  __shared__ unsigned long long base_sh;
  __shared__ unsigned long long lds_fp[LDS_FP_SLOTS];
  for (int t = threadIdx.x; t < LDS_FP_SLOTS; t += BS) lds_fp[t] = 0ull;
  __syncthreads();
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  const u64 st = (u64)blockIdx.x * BS + threadIdx.x;
  const u64* row = a.cand + (u64)blockIdx.x * NI * BS + threadIdx.x;
  u64 isnew = 0, isnew_hi = 0;   // instances 0..63 / 64..127 (the latter only for NI > 64, e.g. N = 5)
  auto mark = [&](int k) { if (NI <= 64 || k < 64) isnew |= 1ull << (k & 63); else isnew_hi |= 1ull << (k & 63); };
  u32 err = 0;
  constexpr int G = 16;
#pragma unroll 1
  for (int k0 = 0; k0 < NI; k0 += G) {
    u64 fp[G], cur[G];
#pragma unroll
    for (int j = 0; j < G; ++j) fp[j] = (st < a.chunk_count && k0 + j < NI) ? row[(u64)(k0 + j) * BS] : 0ull;
#pragma unroll
    for (int j = 0; j < G; ++j)   // diamonds of commuting actions: ~half of C2's successors within 256 parents
      if (fp[j] && !lds_first(lds_fp, fp[j])) fp[j] = 0;
#pragma unroll
    for (int j = 0; j < G; ++j) cur[j] = fp[j] ? a.table[fp[j] & a.table_mask] : ~0ull;
#pragma unroll
    for (int j = 0; j < G; ++j)
      if (fp[j] && cur[j] == 0ull)
        cur[j] = (u64)atomicCAS((unsigned long long*)&a.table[fp[j] & a.table_mask], 0ull, (unsigned long long)fp[j]);
#pragma unroll
    for (int j = 0; j < G; ++j) {
      if (!fp[j]) continue;
      if (cur[j] == 0ull) { mark(k0 + j); continue; }
      if (cur[j] == fp[j]) continue;
      u64 slot = (fp[j] + 1) & a.table_mask;
      for (int probe = 0;; ++probe) {
        if (probe >= (1 << 20)) { err |= OE_TABLE_FULL; break; }
        const u64 c = a.table[slot];
        if (c == fp[j]) break;
        if (c == 0ull) {
          const u64 old = (u64)atomicCAS((unsigned long long*)&a.table[slot], 0ull, (unsigned long long)fp[j]);
          if (old == 0ull) { mark(k0 + j); break; }
          if (old == fp[j]) break;
        }
        slot = (slot + 1) & a.table_mask;
      }
    }
  }
  const unsigned int mine = (unsigned int)(__popcll(isnew) + __popcll(isnew_hi));
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
  while (isnew) {
    const int k = __ffsll((unsigned long long)isnew) - 1;
    isnew &= isnew - 1;
    a.newrec[pos++] = ((a.chunk_begin + st) << 8) | (u64)k;
  }
  while (isnew_hi) {
    const int k = 64 + __ffsll((unsigned long long)isnew_hi) - 1;
    isnew_hi &= isnew_hi - 1;
    a.newrec[pos++] = ((a.chunk_begin + st) << 8) | (u64)k;
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
}

struct MatArgs {
  u32* states;
  u64* meta;
  const u64* newrec;
  u64 dst_base, cap;           // new state i of the chunk goes to dst_base + ctr[K_LEVEL_NEW] + i
  u64 base;                    // global id of device slot 0 (completed levels spilled to the host)
  OrigRuntime rt;
  unsigned long long* ctr;     // ctr[K_CHUNK_NEW] = the chunk's new states (set by orig_dedup_blk)
  void* viol;
};

// Grid-stride over the chunk's new states, whose number stays on the device: the host does
// not wait for the dedup kernel to size this launch (one host synchronisation per level).
template <class S>
__global__ void __launch_bounds__(BS) orig_materialize(MatArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  __shared__ unsigned int lds_cnt[OA_NACT];
  for (int t = threadIdx.x; t < OA_NACT; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 n_new = a.ctr[K_CHUNK_NEW];
  const u64 base = a.dst_base + a.ctr[K_LEVEL_NEW];
  u32 err = 0;
  for (u64 i = (u64)blockIdx.x * BS + threadIdx.x; i < n_new; i += (u64)gridDim.x * BS) {
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
    const u64 dst = base + i;
    if (act >= 0 && dst < a.cap) {
      uint4* o = reinterpret_cast<uint4*>(a.states + dst * NWP);
#pragma unroll
      for (int q = 0; q < NWP / 4; ++q)
        o[q] = make_uint4(pw[4 * q], 4 * q + 1 < NW ? pw[4 * q + 1] : 0u, 4 * q + 2 < NW ? pw[4 * q + 2] : 0u, 4 * q + 3 < NW ? pw[4 * q + 3] : 0u);
      a.meta[dst] = ((gid + a.base) << 24) | ((u64)act << 16) | (u64)k;
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

// after a chunk's materialize: the level's running count of new states
// after a chunk's materialize: fold its new-state count into the level's and re-arm the chunk
// counter for the next chunk (the level's first chunk starts from the per-level counter reset)
__global__ void orig_advance(unsigned long long* ctr) {
  if (threadIdx.x == 0) {
    ctr[K_LEVEL_NEW] += ctr[K_CHUNK_NEW];
    ctr[K_CHUNK_NEW] = 0;
  }
}

// ------------------------------------------------------------------ sharded (multi-GPU) kernels
// owner of a fingerprint: high half mod world (the seen-set index uses the low bits)
__device__ __host__ __forceinline__ u32 fp_owner(u64 fp, u32 world) { return (u32)((fp >> 32) % world); }

struct RouteArgs {
  const u64* cand;
  u64 nslots;
  u64* route;                  // [world][route_cap][2] (fp, slot)
  u64 route_cap;
  u32 world;
  unsigned long long* rcnt;    // [world]
};

// Sharded route over the PM slot layout: workgroup b takes generate-workgroup b's 256
// parents, drops the successors they produce more than once (the LDS set of orig_dedup_blk),
// and buckets the rest by owner, 16 instances at a time: LDS histogram, one global atomic per
// (workgroup, group, owner).  Records are (fp, state << 8 | instance).
template <int NI>
__global__ void __launch_bounds__(BS) orig_route_blk(RouteArgs a) {
  static_assert(NI <= 255, "instance in 8 bits");
  __shared__ unsigned long long lds_fp[LDS_FP_SLOTS];
  __shared__ unsigned int hist[8];
  __shared__ unsigned long long base[8];
  for (int t = threadIdx.x; t < LDS_FP_SLOTS; t += BS) lds_fp[t] = 0ull;
  const u64 st = (u64)blockIdx.x * BS + threadIdx.x;
  const u64* row = a.cand + (u64)blockIdx.x * NI * BS + threadIdx.x;
  constexpr int G = 16;
#pragma unroll 1
  for (int k0 = 0; k0 < NI; k0 += G) {
    if (threadIdx.x < 8) hist[threadIdx.x] = 0;
    __syncthreads();   // also orders the set's clearing before its first use
    u64 fp[G];
    unsigned int off[G];
    int own[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      fp[j] = (st < a.nslots / NI && k0 + j < NI) ? row[(u64)(k0 + j) * BS] : 0ull;
      if (fp[j] && !lds_first(lds_fp, fp[j])) fp[j] = 0;
      own[j] = fp[j] ? (int)fp_owner(fp[j], a.world) : -1;
      off[j] = own[j] >= 0 ? atomicAdd(&hist[own[j]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < a.world) base[threadIdx.x] = hist[threadIdx.x] ? atomicAdd(&a.rcnt[threadIdx.x], (unsigned long long)hist[threadIdx.x]) : 0ull;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < G; ++j) {
      if (own[j] < 0) continue;
      // one 16-B store per record
      *reinterpret_cast<ulonglong2*>(a.route + ((u64)own[j] * a.route_cap + base[own[j]] + off[j]) * 2) =
          make_ulonglong2((unsigned long long)fp[j], (unsigned long long)((st << 8) | (u64)(k0 + j)));
    }
    __syncthreads();   // hist / base reused by the next group
  }
}

struct DedupShArgs {
  const u64* recv;             // (fp, slot) records of one source rank
  u64 n;
  u64* table;
  u64 table_mask;
  u64* reply;                  // compacted slots of the new ones
  unsigned long long* counter; // per-source reply count
  unsigned long long* ctr;
};

__global__ void __launch_bounds__(BS) orig_dedup_sh(DedupShArgs a) {
  __shared__ unsigned int wave_tot[BS / 64];
  __shared__ unsigned long long base_sh;
  const u64 tile = (u64)blockIdx.x * (BS * DEDUP_PER);
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  u64 fp[DEDUP_PER], cur[DEDUP_PER];
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j) {
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    fp[j] = idx < a.n ? a.recv[2 * idx] : 0ull;
  }
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j) cur[j] = fp[j] ? a.table[fp[j] & a.table_mask] : ~0ull;
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j)
    if (fp[j] && cur[j] == 0ull)
      cur[j] = (u64)atomicCAS((unsigned long long*)&a.table[fp[j] & a.table_mask], 0ull, (unsigned long long)fp[j]);
  u32 isnew = 0, err = 0;
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j) {
    if (!fp[j]) continue;
    if (cur[j] == 0ull) { isnew |= 1u << j; continue; }
    if (cur[j] == fp[j]) continue;
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
  const unsigned int mine = (unsigned int)__popc(isnew);
  unsigned int incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) { const unsigned int v = __shfl_up(incl, d); if (lane >= d) incl += v; }
  if (lane == 63) wave_tot[wave] = incl;
  __syncthreads();
  if (threadIdx.x == 0) {
    unsigned int tot = 0;
    for (int w = 0; w < BS / 64; ++w) { const unsigned int x = wave_tot[w]; wave_tot[w] = tot; tot += x; }
    base_sh = tot ? atomicAdd(a.counter, (unsigned long long)tot) : 0ull;
  }
  __syncthreads();
  u64 pos = base_sh + wave_tot[wave] + (incl - mine);
  for (int j = 0; j < DEDUP_PER; ++j) {
    if (!((isnew >> j) & 1u)) continue;
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    a.reply[pos++] = a.recv[2 * idx + 1];
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
}

struct MatShArgs {
  const u32* states;
  const u64* acks;             // slots acknowledged as new by one owner
  u64 n, chunk_begin, chunk_count;
  u32* out;                    // [n][NWP + 4] state records for that owner
  u64 rank_bits;               // rank << 37
  u64 seed;
  OrigRuntime rt;
  unsigned long long* ctr;
  void* viol;
};

template <class S>
__global__ void __launch_bounds__(BS) orig_materialize_sh(MatShArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3, RW = NWP + 4;
  __shared__ unsigned int lds_cnt[OA_NACT];
  for (int t = threadIdx.x; t < OA_NACT; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  u32 err = 0;
  if (i < a.n) {
    const u64 slot = a.acks[i];   // state in chunk << 8 | instance (orig_route_blk)
    const u64 k = slot & 255ull, gid = a.chunk_begin + (slot >> 8);
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(a.states + gid * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    W s, t;
    u64 al[S::AW];
    S::unpack(w, s);
    S::all_logs_next(s, al);
    const int act = S::apply(s, (int)k, t, err);
#pragma unroll
    for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
    u32 pw[NW];
    S::pack(t, pw);
    const u64 fp = fp64(pw, a.seed);
    const u64 meta = ((a.rank_bits | gid) << 24) | ((u64)(act < 0 ? 0 : act) << 16) | k;
    u32* o = a.out + i * RW;
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q)
      reinterpret_cast<uint4*>(o)[q] = make_uint4(pw[4 * q], 4 * q + 1 < NW ? pw[4 * q + 1] : 0u, 4 * q + 2 < NW ? pw[4 * q + 2] : 0u, 4 * q + 3 < NW ? pw[4 * q + 3] : 0u);
    reinterpret_cast<uint4*>(o)[NWP / 4] = make_uint4((u32)meta, (u32)(meta >> 32), (u32)fp, (u32)(fp >> 32));
    if (act >= 0) {
      atomicAdd(&lds_cnt[act], 1u);
      const u32 bad = S::violated(t, a.rt.invariants);
      if (bad && atomicCAS(&a.ctr[K_VIOL], 0ull, 1ull) == 0ull) {
        ViolRec<S>* v = reinterpret_cast<ViolRec<S>*>(a.viol);
        v->parent = gid; v->act = (u32)act; v->inst = (u32)k; v->bad = bad; v->inmodel = 1; v->w = t;
      }
    } else {
      err |= OE_EVAL_LOG_INDEX;
    }
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + OA_NACT + t], (unsigned long long)lds_cnt[t]);
}

struct StoreArgs {
  const u32* in;               // [n][NWP + 4]
  u64 n, dst, cap;
  u32* states;
  u64* meta;
  unsigned long long* ctr;
};

template <int NWP>
__global__ void __launch_bounds__(BS) orig_store(StoreArgs a) {
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i >= a.n) return;
  const u64 dst = a.dst + i;
  if (dst >= a.cap) { atomicOr(&a.ctr[K_ERR], (unsigned long long)OE_CAP_STORE); return; }
  const uint4* src = reinterpret_cast<const uint4*>(a.in + i * (NWP + 4));
  uint4* o = reinterpret_cast<uint4*>(a.states + dst * NWP);
#pragma unroll
  for (int q = 0; q < NWP / 4; ++q) o[q] = src[q];
  const uint4 m = src[NWP / 4];
  a.meta[dst] = (u64)m.x | ((u64)m.y << 32);
}

// Recovery from a checkpoint: re-insert the fingerprints of every stored state into the
// zeroed seen-set (the checkpoint holds states, not the table; FP64 is a function of the
// packed words, so the rebuilt set is the saved one).
template <class S>
__global__ void __launch_bounds__(BS) orig_reinsert(const u32* states, u64 n, u64* table, u64 mask, u64 seed,
                                                    unsigned long long* ctr) {
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  u32 w[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) w[q] = states[i * NWP + q];
  const u64 fp = fp64(w, seed);
  u64 slot = fp & mask;
  for (int probe = 0; probe < (1 << 20); ++probe) {
    const u64 c = table[slot];
    if (c == fp) return;
    if (c == 0ull) {
      const u64 old = (u64)atomicCAS((unsigned long long*)&table[slot], 0ull, (unsigned long long)fp);
      if (old == 0ull || old == fp) return;
    }
    slot = (slot + 1) & mask;
  }
  atomicOr(&ctr[K_ERR], (unsigned long long)OE_TABLE_FULL);
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

  int observed_collision(double& v, std::string& err) override {
    if (!d_table_ || alloc_world_ != 0) { err = "after a single-GPU mc_run only"; return MC_E_STATE; }
    return fpgap::observed(d_table_, table_mask_ + 1, 1, stream_, v, err);
  }

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

  // Buffers are allocated on the first run and reused (a re-run of the same
  // handle re-zeroes the seen-set and overwrites the store).
  int ensure_alloc(const RunOpts& o, int world, std::string& err) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= o.device) { err = "no HIP device available (raftmc has no CPU fallback)"; return MC_E_NO_DEVICE; }
    HIPCHK(hipSetDevice(o.device));
    if (d_table_ && o.device == dev_ && o.fp_table_bytes == req_table_ && o.state_store_bytes == req_store_ && world == alloc_world_) return 0;
    release();
    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    uint64_t tb = o.fp_table_bytes ? o.fp_table_bytes : std::min<uint64_t>(8ull << 30, freeb / 4);
    uint64_t slots = 1; while (slots * 2 * 8 <= tb) slots *= 2;
    if (slots < 1024) slots = 1024;
    uint64_t sb = o.state_store_bytes ? o.state_store_bytes : std::min<uint64_t>(32ull << 30, freeb / 3);
    cap_ = sb / (NWP * 4 + 8);
    if (cap_ < 16) cap_ = 16;
    // frontier chunk: the slot array holds chunk_states * NI fingerprints and
    // the record array as many (worst case: every slot new): ~1/8 of the store;
    // sharded mode also needs world route regions of 16-B records per slot
    chunk_states_ = std::max<u64>(4096, std::min<u64>(cap_, (sb / 8) / (16 * (u64)S::NI)));
    if (world > 1) chunk_states_ = std::max<u64>(4096, chunk_states_ / (u64)world);
    chunk_states_ = (chunk_states_ / BS) * BS;   // whole workgroups: the PM slot layout is [block][instance][lane]
    table_mask_ = slots - 1;
    HIPCHK(hipMalloc(&d_table_, slots * 8));
    HIPCHK(hipMalloc(&d_states_, cap_ * NWP * 4));
    HIPCHK(hipMalloc(&d_meta_, cap_ * 8));
    HIPCHK(hipMalloc(&d_cand_, chunk_states_ * S::NI * 8));
    HIPCHK(hipMalloc(&d_newrec_, chunk_states_ * S::NI * 8));
    HIPCHK(hipMalloc(&d_ctr_, K_NCTR * 8));
    HIPCHK(hipMalloc(&d_viol_, sizeof(ViolRec<S>)));
    if (world >= 1) {   // sharded mode
      HIPCHK(hipMalloc(&d_route_, (u64)world * chunk_states_ * S::NI * 16));
      HIPCHK(hipMalloc(&d_rcnt_, 2 * 8 * 8));
    }
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (auto& e : ev_) HIPCHK(hipEventCreate(&e));
    dev_ = o.device; req_table_ = o.fp_table_bytes; req_store_ = o.state_store_bytes; alloc_world_ = world;
    return 0;
  }

  // event pairs (generate, dedup, materialize) of chunk q of the current level: lvl_ev_[6q .. 6q+6)
  int lvl_events(int q) {
    while ((int)lvl_ev_.size() < 6 * (q + 1)) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return MC_E_NO_DEVICE;
      lvl_ev_.push_back(e);
    }
    return 0;
  }

  int run_generate(GenArgs& g, u64 cnt, float& ms_g, std::string& err, bool pm = false) {
    const unsigned nblk = (unsigned)((cnt + BS - 1) / BS);
    HIPCHK(hipEventRecord(ev_[5], stream_));
    if (pm) hipLaunchKernelGGL((orig_generate<S, true>), dim3(nblk), dim3(BS), 0, stream_, g);
    else hipLaunchKernelGGL((orig_generate<S, false>), dim3(nblk), dim3(BS), 0, stream_, g);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev_[6], stream_));
    HIPCHK(hipEventSynchronize(ev_[6]));
    ms_g = time_ms(5, 6);
    return 0;
  }

  int run(const RunOpts& o, RunResult& r, std::string& err) override {
    if (int rc = ensure_alloc(o, 0, err)) return rc;   // world 0 = single-GPU pipeline
    auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipMemsetAsync(d_table_, 0, (table_mask_ + 1) * 8, stream_));
    HIPCHK(hipStreamSynchronize(stream_));

    r = RunResult();
    r.seed = o.seed ? o.seed : 0x5EED5EED2024ull;
    r.state_bytes = NWP * 4;
    for (int k = 0; k < OA_NACT; ++k) r.action_names.push_back(kOrigActNames[k]);
    r.act_generated.assign(OA_NACT, 0); r.act_distinct.assign(OA_NACT, 0);
    r.kernels = {{"orig_generate", 0, 0, 0}, {"orig_dedup_blk", 0, 0, 0}, {"orig_materialize", 0, 0, 0}};
    base_ = 0; host_states_.clear(); host_meta_.clear();

    W s0; S::init(s0);
    const u64 S_B = NWP * 4;
    u64 level_begin = 0, level_count = 1;
    if (!o.recover_path.empty()) {   // TLC -recover: continue the BFS saved by a checkpoint
      if (int rc = load_checkpoint(o.recover_path, r, level_begin, level_count, err)) return rc;
    } else {
    // ---- Init (raft_original.tla:139-159): one state, generated and distinct
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
    }

    while (level_count > 0) {
      if (o.max_depth && r.depth >= o.max_depth) { r.left_on_queue = (int64_t)level_count; r.verdict = MC_VERDICT_DEPTH_LIMIT; break; }
      // the device keeps what the search still reads (the frontier) and writes (the next
      // level); when the next level, predicted from the last growth ratio with a 1.5x margin,
      // might not fit behind what is stored, the completed levels move to host memory
      if (level_begin > base_) {
        const double prev = r.levels.size() >= 2 ? (double)r.levels[r.levels.size() - 2].states : 1.0;
        const double pred = (double)level_count * std::max(1.0, (double)level_count / std::max(prev, 1.0)) * 1.5;
        if ((double)(total_ - base_) + pred > (double)cap_)
          if (int rc = spill(level_begin, level_count, err)) return rc;
      }
      HIPCHK(hipMemsetAsync(d_ctr_, 0, K_NCTR * 8, stream_));
      const u64 level_end = level_begin + level_count;
      // every chunk's kernels are queued without waiting: the dedup kernel numbers the new
      // states on the device and the materialize kernel reads that count (grid-stride), so the
      // host synchronises once per level, for the counters
      int nch = 0;
      for (u64 cb = level_begin; cb < level_end; cb += chunk_states_, ++nch) {
        const u64 cnt = std::min<u64>(chunk_states_, level_end - cb);
        const u64 nslots = cnt * (u64)S::NI;
        const unsigned nblk = (unsigned)((cnt + BS - 1) / BS);
        if (int rc = lvl_events(nch)) { err = "hipEventCreate failed"; return rc; }
        hipEvent_t* e = &lvl_ev_[6 * nch];
        GenArgs g;
        // kernels index the device store (global id - base_); parent pointers are global
        g.states = d_states_; g.chunk_begin = cb - base_; g.chunk_count = cnt; g.cand = d_cand_; g.seed = r.seed; g.rt = m_.rt;
        g.inv_oom = o.inv_out_of_model ? 1u : 0u; g.ctr = (unsigned long long*)d_ctr_; g.viol = d_viol_;
        HIPCHK(hipEventRecord(e[0], stream_));
        hipLaunchKernelGGL((orig_generate<S, true>), dim3(nblk), dim3(BS), 0, stream_, g);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e[1], stream_));
        DedupArgs d;
        d.cand = d_cand_; d.nslots = nslots; d.chunk_begin = cb - base_; d.chunk_count = cnt; d.table = d_table_;
        d.table_mask = table_mask_; d.newrec = d_newrec_; d.ctr = (unsigned long long*)d_ctr_; d.ni = S::NI;
        HIPCHK(hipEventRecord(e[2], stream_));
        hipLaunchKernelGGL((orig_dedup_blk<S::NI>), dim3(nblk), dim3(BS), 0, stream_, d);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e[3], stream_));
        MatArgs m;
        m.states = d_states_; m.meta = d_meta_; m.newrec = d_newrec_; m.dst_base = level_end - base_; m.cap = cap_;
        m.base = base_; m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_; m.viol = d_viol_;
        const unsigned mblk = (unsigned)std::min<u64>(4096, (nslots + BS - 1) / BS);
        HIPCHK(hipEventRecord(e[4], stream_));
        hipLaunchKernelGGL((orig_materialize<S>), dim3(mblk), dim3(BS), 0, stream_, m);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e[5], stream_));
        hipLaunchKernelGGL(orig_advance, dim3(1), dim3(64), 0, stream_, (unsigned long long*)d_ctr_);
        HIPCHK(hipGetLastError());
        r.kernels[0].launches += 1; r.kernels[1].launches += 1; r.kernels[2].launches += 1;
        r.kernels[0].algo_bytes += (double)cnt * S_B + (double)nslots * 8;
        r.kernels[1].algo_bytes += (double)nslots * 8;   // + G_in*8 probe bytes and D*16 per level below
      }
      u64 c[K_NCTR];
      HIPCHK(hipMemcpyAsync(c, d_ctr_, sizeof c, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
      double level_ms = 0;
      for (int q = 0; q < nch; ++q)
        for (int k = 0; k < 3; ++k) {
          float ms = 0;
          (void)hipEventElapsedTime(&ms, lvl_ev_[6 * q + 2 * k], lvl_ev_[6 * q + 2 * k + 1]);
          r.kernels[k].ms += ms; level_ms += ms;
        }
      const u64 next_write = level_end + c[K_LEVEL_NEW];
      r.kernels[1].algo_bytes += (double)c[K_LEVEL_NEW] * 16;
      r.kernels[2].algo_bytes += (double)c[K_LEVEL_NEW] * (8 + S_B + S_B + 8);
      int64_t gen = 0;
      for (int k = 0; k < OA_NACT; ++k) { r.act_generated[k] += (int64_t)c[K_ACT + k]; r.act_distinct[k] += (int64_t)c[K_ACT + OA_NACT + k]; gen += (int64_t)c[K_ACT + k]; }
      r.generated += gen;
      r.generated_in_model += (int64_t)c[K_GEN_IN];
      r.kernels[1].algo_bytes += (double)c[K_GEN_IN] * 8;
      r.seconds_kernels += level_ms / 1000.0;
      r.n_launches += 1;
      const u64 nnew = next_write - (level_begin + level_count);
      r.algo_bytes += (double)level_count * S_B + (double)c[K_GEN_IN] * 8 + (double)nnew * (16 + S_B);
      if (next_write - base_ > cap_) c[K_ERR] |= OE_CAP_STORE;
      if (c[K_ERR]) {
        const u64 e = c[K_ERR];
        r.verdict = (e & (OE_CAP_STORE | OE_TABLE_FULL | OE_CAP_ELECTIONS | OE_CAP_COUNT)) ? MC_VERDICT_CAPACITY_OVERFLOW : MC_VERDICT_EVAL_ERROR;
        std::ostringstream os;
        os << "error flags 0x" << std::hex << e << std::dec << " while expanding state " << (c[K_ERRGID] ? (int64_t)(c[K_ERRGID] - 1 + base_) : -1) << ":";
        if (e & OE_EVAL_LOG_INDEX) os << " log[i][prevLogIndex] applied outside its domain (raft_original.tla:207-210);";
        if (e & OE_CAP_ELECTIONS) os << " elections set exceeds the compiled capacity;";
        if (e & OE_CAP_COUNT) os << " message count / bag capacity exceeded;";
        if (e & OE_CAP_STORE) os << " state store full (raise state_store_bytes);";
        if (e & OE_TABLE_FULL) os << " fingerprint table full (raise fp_table_bytes);";
        r.error = os.str();
        total_ = std::min<u64>(next_write, base_ + cap_);
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
        build_trace(v.parent + base_, kOrigActNames[v.act], v.w, r, err);
        r.left_on_queue = (int64_t)nnew;
        break;
      }
      if (o.check_deadlock && c[K_DEADLOCK]) {
        r.verdict = MC_VERDICT_DEADLOCK;
        build_trace(c[K_DEADLOCK] - 1 + base_, nullptr, s0, r, err);
        r.left_on_queue = (int64_t)nnew;
        break;
      }
      level_begin += level_count;
      level_count = nnew;
      if (o.checkpoint_every > 0 && !o.checkpoint_path.empty() && r.depth % o.checkpoint_every == 0 && level_count > 0)
        if (int rc = save_checkpoint(o.checkpoint_path, r, level_begin, level_count, err)) return rc;
    }
    finish(r, t0);
    return 0;
  }

  // ---------------------------------------------------------------- checkpoint / recover
  // File: magic, the model's describe_json (a checkpoint only resumes the same model), the BFS
  // position (level_begin/count, stored states) and TLC's counters, then the stored states and
  // parent pointers [0, total).  The seen-set is rebuilt from the states on recovery.
  struct CkptHead {
    char magic[8];
    u64 nwp, total, level_begin, level_count, seed;
    int64_t generated, distinct, depth, generated_in_model, n_act, n_levels, desc_len;
  };
  int save_checkpoint(const std::string& path, const RunResult& r, u64 level_begin, u64 level_count, std::string& err) {
    const std::string desc = describe_json();
    CkptHead h;
    std::memcpy(h.magic, "RAFTMCK1", 8);
    h.nwp = NWP; h.total = total_; h.level_begin = level_begin; h.level_count = level_count; h.seed = r.seed;
    h.generated = r.generated; h.distinct = r.distinct; h.depth = r.depth; h.generated_in_model = r.generated_in_model;
    h.n_act = OA_NACT; h.n_levels = (int64_t)r.levels.size(); h.desc_len = (int64_t)desc.size();
    std::vector<u32> st(total_ * NWP);
    std::vector<u64> me(total_);
    std::memcpy(st.data(), host_states_.data(), base_ * NWP * 4);
    std::memcpy(me.data(), host_meta_.data(), base_ * 8);
    HIPCHK(hipMemcpy(st.data() + base_ * NWP, d_states_, (total_ - base_) * NWP * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(me.data() + base_, d_meta_, (total_ - base_) * 8, hipMemcpyDeviceToHost));
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) { err = "cannot write checkpoint " + tmp; return MC_E_IO; }
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(desc.data(), 1, desc.size(), f) == desc.size() &&
              std::fwrite(r.act_generated.data(), 8, OA_NACT, f) == (size_t)OA_NACT &&
              std::fwrite(r.act_distinct.data(), 8, OA_NACT, f) == (size_t)OA_NACT;
    for (const auto& lv : r.levels) ok = ok && std::fwrite(&lv.states, 8, 1, f) == 1 && std::fwrite(&lv.generated, 8, 1, f) == 1;
    ok = ok && std::fwrite(st.data(), 4, st.size(), f) == st.size() && std::fwrite(me.data(), 8, me.size(), f) == me.size();
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) { err = "writing checkpoint " + path + " failed"; return MC_E_IO; }
    return 0;
  }
  int load_checkpoint(const std::string& path, RunResult& r, u64& level_begin, u64& level_count, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { err = "cannot read checkpoint " + path; return MC_E_IO; }
    CkptHead h;
    const std::string desc = describe_json();
    std::string fdesc;
    bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, "RAFTMCK1", 8) == 0 && h.nwp == (u64)NWP &&
              h.n_act == OA_NACT && h.desc_len >= 0 && h.desc_len < (1 << 20) && h.n_levels > 0 && h.n_levels < (1 << 20);
    if (ok) { fdesc.resize((size_t)h.desc_len); ok = std::fread(&fdesc[0], 1, fdesc.size(), f) == fdesc.size(); }
    if (!ok || fdesc != desc) { std::fclose(f); err = "checkpoint " + path + " is not a checkpoint of this model"; return MC_E_INVALID; }
    // completed levels that do not fit the device store stay in host memory (spilled)
    const u64 lb = h.total > cap_ ? h.level_begin : 0;
    if (h.total - lb > cap_ || h.level_begin > h.total) { std::fclose(f); err = "checkpoint frontier exceeds the state store (raise state_store_bytes)"; return MC_E_OOM; }
    ok = std::fread(r.act_generated.data(), 8, OA_NACT, f) == (size_t)OA_NACT &&
         std::fread(r.act_distinct.data(), 8, OA_NACT, f) == (size_t)OA_NACT;
    r.levels.clear();
    for (int64_t k = 0; ok && k < h.n_levels; ++k) {
      LevelStat lv;
      ok = std::fread(&lv.states, 8, 1, f) == 1 && std::fread(&lv.generated, 8, 1, f) == 1;
      r.levels.push_back(lv);
    }
    std::vector<u32> st(h.total * NWP);
    std::vector<u64> me(h.total);
    ok = ok && std::fread(st.data(), 4, st.size(), f) == st.size() && std::fread(me.data(), 8, me.size(), f) == me.size();
    std::fclose(f);
    if (!ok) { err = "checkpoint " + path + " is truncated"; return MC_E_IO; }
    HIPCHK(hipMemsetAsync(d_ctr_, 0, K_NCTR * 8, stream_));
    // the host part's fingerprints go in through the (idle) candidate buffer, chunk by chunk
    const u64 stage = std::max<u64>(1, chunk_states_ * S::NI * 8 / (NWP * 4));
    for (u64 b = 0; b < lb; b += stage) {
      const u64 n = std::min<u64>(stage, lb - b);
      HIPCHK(hipMemcpy(d_cand_, st.data() + b * NWP, n * NWP * 4, hipMemcpyHostToDevice));
      hipLaunchKernelGGL((orig_reinsert<S>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_,
                         (const u32*)d_cand_, n, d_table_, table_mask_, (u64)h.seed, (unsigned long long*)d_ctr_);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(stream_));
    }
    HIPCHK(hipMemcpy(d_states_, st.data() + lb * NWP, (h.total - lb) * NWP * 4, hipMemcpyHostToDevice));
    HIPCHK(hipMemcpy(d_meta_, me.data() + lb, (h.total - lb) * 8, hipMemcpyHostToDevice));
    if (h.total > lb) {
      hipLaunchKernelGGL((orig_reinsert<S>), dim3((unsigned)((h.total - lb + BS - 1) / BS)), dim3(BS), 0, stream_,
                         (const u32*)d_states_, (u64)(h.total - lb), d_table_, table_mask_, (u64)h.seed, (unsigned long long*)d_ctr_);
      HIPCHK(hipGetLastError());
    }
    host_states_.assign(st.begin(), st.begin() + lb * NWP);
    host_meta_.assign(me.begin(), me.begin() + lb);
    base_ = lb;
    u64 e = 0;
    HIPCHK(hipMemcpyAsync(&e, d_ctr_ + K_ERR, 8, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (e) { err = "fingerprint table too small for the checkpoint (raise fp_table_bytes)"; return MC_E_OOM; }
    r.seed = h.seed; r.generated = h.generated; r.distinct = h.distinct; r.depth = h.depth;
    r.generated_in_model = h.generated_in_model;
    total_ = h.total; level_begin = h.level_begin; level_count = h.level_count;
    return 0;
  }

  int dump_states(const std::string& path, std::string& err) override {
    if (!d_states_) { err = "mc_dump_states before mc_run"; return MC_E_STATE; }
    std::vector<u32> h(total_ * NWP);
    std::memcpy(h.data(), host_states_.data(), base_ * NWP * 4);
    HIPCHK(hipMemcpy(h.data() + base_ * NWP, d_states_, (total_ - base_) * NWP * 4, hipMemcpyDeviceToHost));
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

  // ================================================================ sharded mode
  int shard_open(const RunOpts& o, int rank, int world, std::string& err) override {
    if (world < 1 || world > 8 || rank < 0 || rank >= world) { err = "sharded mode supports 1..8 ranks"; return MC_E_INVALID; }
    if (int rc = ensure_alloc(o, world, err)) return rc;
    rank_ = rank; world_ = world; sopts_ = o;
    HIPCHK(hipMemsetAsync(d_table_, 0, (table_mask_ + 1) * 8, stream_));
    HIPCHK(hipMemsetAsync(d_ctr_, 0, K_NCTR * 8, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    sres_ = RunResult();
    sres_.seed = o.seed ? o.seed : 0x5EED5EED2024ull;
    sres_.state_bytes = NWP * 4;
    for (int k = 0; k < OA_NACT; ++k) sres_.action_names.push_back(kOrigActNames[k]);
    sres_.act_generated.assign(OA_NACT, 0); sres_.act_distinct.assign(OA_NACT, 0);
    sres_.kernels = {{"orig_generate", 0, 0, 0}, {"orig_route_blk", 0, 0, 0}, {"orig_dedup_sh", 0, 0, 0},
                     {"orig_materialize_sh", 0, 0, 0}, {"orig_store", 0, 0, 0}};
    st0_ = std::chrono::steady_clock::now();
    // Init: one state, stored and inserted by the owner of its fingerprint
    W s0; S::init(s0);
    u32 w0[S::NW]; S::pack(s0, w0);
    const u64 fp0 = fp64(w0, sres_.seed);
    total_ = 0; sh_level_begin_ = 0; sh_level_count_ = 0; sh_new_ = 0;
    base_ = 0; host_states_.clear(); host_meta_.clear();
    if ((int)fp_owner(fp0, (u32)world) == rank) {
      u32 wp[NWP] = {0}; for (int q = 0; q < S::NW; ++q) wp[q] = w0[q];
      HIPCHK(hipMemcpy(d_table_ + (fp0 & table_mask_), &fp0, 8, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(d_states_, wp, NWP * 4, hipMemcpyHostToDevice));
      const u64 nometa = ~0ull;
      HIPCHK(hipMemcpy(d_meta_, &nometa, 8, hipMemcpyHostToDevice));
      total_ = 1; sh_level_count_ = 1;
    }
    sres_.generated = 1; sres_.distinct = 1; sres_.depth = 1;
    sres_.levels.push_back({1, 0, 0.0});
    if (!S::in_model(s0, m_.rt)) { err = "the initial state violates a state constraint"; return MC_E_UNSUPPORTED; }
    if (S::violated(s0, m_.rt.invariants)) { err = "the initial state violates an invariant"; return MC_E_UNSUPPORTED; }
    sh_next_write_ = total_;
    return 0;
  }
  int shard_record_bytes(int what) const override {
    return what == MC_SHARD_ROUTE ? 16 : what == MC_SHARD_REPLY ? 8 : what == MC_SHARD_STATES ? (NWP + 4) * 4 : -1;
  }
  int shard_frontier(int64_t* states, int64_t* chunk) const override {
    if (states) *states = (int64_t)sh_level_count_;
    if (chunk) *chunk = (int64_t)chunk_states_;
    return 0;
  }
  float time_ms(int a, int b) { float ms = 0; (void)hipEventElapsedTime(&ms, ev_[a], ev_[b]); return ms; }

  int shard_generate(int64_t begin, int64_t count, int64_t* counts, std::string& err) override {
    if (begin < 0 || count < 0 || (u64)count > chunk_states_ || (u64)(begin + count) > sh_level_count_) { err = "shard_generate: chunk outside the frontier"; return MC_E_INVALID; }
    sh_chunk_begin_ = sh_level_begin_ + (u64)begin; sh_chunk_count_ = (u64)count;
    HIPCHK(hipMemsetAsync(d_rcnt_, 0, 8 * 8, stream_));
    if (count > 0) {
      const u64 nslots = (u64)count * S::NI;
      GenArgs g;
      g.states = d_states_; g.chunk_begin = sh_chunk_begin_; g.chunk_count = (u64)count; g.cand = d_cand_; g.seed = sres_.seed;
      g.rt = m_.rt; g.inv_oom = sopts_.inv_out_of_model ? 1u : 0u; g.ctr = (unsigned long long*)d_ctr_; g.viol = d_viol_;
      RouteArgs ra;
      ra.cand = d_cand_; ra.nslots = nslots; ra.route = d_route_; ra.route_cap = chunk_states_ * S::NI; ra.world = (u32)world_;
      ra.rcnt = (unsigned long long*)d_rcnt_;
      float ms_x = 0;
      if (int rc = run_generate(g, (u64)count, ms_x, err, true)) return rc;
      auto& ke = sres_.kernels[0]; ke.ms += ms_x; ke.launches++; ke.algo_bytes += (double)count * NWP * 4 + (double)nslots * 8;
      HIPCHK(hipEventRecord(ev_[1], stream_));
      hipLaunchKernelGGL((orig_route_blk<S::NI>), dim3((unsigned)((count + BS - 1) / BS)), dim3(BS), 0, stream_, ra);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(ev_[2], stream_));
    }
    u64 c[8] = {0};
    HIPCHK(hipMemcpyAsync(c, d_rcnt_, 8 * 8, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (count > 0) {
      const u64 nslots = (u64)count * S::NI;
      u64 valid = 0; for (int r = 0; r < world_; ++r) valid += c[r];
      auto& kr = sres_.kernels[1]; kr.ms += time_ms(1, 2); kr.launches++; kr.algo_bytes += (double)nslots * 8 + (double)valid * 16;
    }
    for (int r = 0; r < world_; ++r) { counts[r] = (int64_t)c[r]; fill_counts_route_[r] = c[r]; }
    return 0;
  }

  int shard_fill(int what, void* dst, const int64_t* offsets, std::string& err) override {
    const int rb = shard_record_bytes(what);
    if (rb < 0) { err = "shard_fill: bad record kind"; return MC_E_INVALID; }
    for (int r = 0; r < world_; ++r) {
      u64 n = 0;
      const char* src = nullptr;
      if (what == MC_SHARD_ROUTE) { n = fill_counts_route_[r]; src = (const char*)(d_route_ + (u64)r * chunk_states_ * S::NI * 2); }
      else if (what == MC_SHARD_REPLY) { n = fill_counts_reply_[r]; src = (const char*)(d_newrec_ + seg_off_[r]); }
      else { n = fill_counts_states_[r]; src = (const char*)(d_stout_ + seg_off_ack_[r] * (NWP + 4)); }
      if (n && !dst) { err = "shard_fill: null destination for a non-empty segment"; return MC_E_INVALID; }
      if (n) HIPCHK(hipMemcpyAsync((char*)dst + (u64)offsets[r] * rb, src, n * rb, hipMemcpyDeviceToDevice, stream_));
    }
    HIPCHK(hipStreamSynchronize(stream_));
    return 0;
  }

  int shard_dedup(const void* recv, const int64_t* counts, int64_t* reply_counts, std::string& err) override {
    u64 off = 0;
    HIPCHK(hipMemsetAsync(d_rcnt_ + 8, 0, 8 * 8, stream_));
    HIPCHK(hipEventRecord(ev_[0], stream_));
    u64 total = 0;
    for (int r = 0; r < world_; ++r) {
      seg_off_[r] = off;
      const u64 n = (u64)counts[r];
      if (off + n > chunk_states_ * S::NI) { err = "shard_dedup: received more records than one chunk holds"; return MC_E_INVALID; }
      if (n) {
        DedupShArgs d;
        d.recv = (const u64*)recv + 2 * off; d.n = n; d.table = d_table_; d.table_mask = table_mask_;
        d.reply = d_newrec_ + off; d.counter = (unsigned long long*)(d_rcnt_ + 8 + r); d.ctr = (unsigned long long*)d_ctr_;
        hipLaunchKernelGGL(orig_dedup_sh, dim3((unsigned)((n + BS * DEDUP_PER - 1) / (BS * DEDUP_PER))), dim3(BS), 0, stream_, d);
        HIPCHK(hipGetLastError());
      }
      off += n; total += n;
    }
    HIPCHK(hipEventRecord(ev_[1], stream_));
    u64 c[8] = {0};
    HIPCHK(hipMemcpyAsync(c, d_rcnt_ + 8, 8 * 8, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    u64 nnew = 0;
    for (int r = 0; r < world_; ++r) { reply_counts[r] = (int64_t)c[r]; fill_counts_reply_[r] = c[r]; nnew += c[r]; }
    auto& kd = sres_.kernels[2]; kd.ms += time_ms(0, 1); kd.launches++; kd.algo_bytes += (double)total * 24 + (double)nnew * 16;
    return 0;
  }

  int shard_materialize(const void* acks, const int64_t* counts, std::string& err) override {
    u64 total = 0;
    for (int r = 0; r < world_; ++r) { seg_off_ack_[r] = total; total += (u64)counts[r]; fill_counts_states_[r] = (u64)counts[r]; }
    if (total > stout_cap_) {
      if (d_stout_) (void)hipFree(d_stout_);
      stout_cap_ = std::max<u64>(total, 1 << 16);
      HIPCHK(hipMalloc(&d_stout_, stout_cap_ * (NWP + 4) * 4));
    }
    HIPCHK(hipEventRecord(ev_[0], stream_));
    for (int r = 0; r < world_; ++r) {
      const u64 n = (u64)counts[r];
      if (!n) continue;
      MatShArgs m;
      m.states = d_states_; m.acks = (const u64*)acks + seg_off_ack_[r]; m.n = n; m.chunk_begin = sh_chunk_begin_;
      m.chunk_count = sh_chunk_count_; m.out = d_stout_ + seg_off_ack_[r] * (NWP + 4); m.rank_bits = (u64)rank_ << 37;
      m.seed = sres_.seed; m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_; m.viol = d_viol_;
      hipLaunchKernelGGL((orig_materialize_sh<S>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_, m);
      HIPCHK(hipGetLastError());
    }
    HIPCHK(hipEventRecord(ev_[1], stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    auto& km = sres_.kernels[3]; km.ms += time_ms(0, 1); km.launches++; km.algo_bytes += (double)total * (8 + NWP * 4 + (NWP + 4) * 4);
    return 0;
  }

  int shard_store(const void* states, int64_t n, std::string& err) override {
    if (n <= 0) return 0;
    StoreArgs a;
    a.in = (const u32*)states; a.n = (u64)n; a.dst = sh_next_write_; a.cap = cap_; a.states = d_states_; a.meta = d_meta_;
    a.ctr = (unsigned long long*)d_ctr_;
    HIPCHK(hipEventRecord(ev_[0], stream_));
    hipLaunchKernelGGL((orig_store<NWP>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_, a);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev_[1], stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    auto& ks = sres_.kernels[4]; ks.ms += time_ms(0, 1); ks.launches++; ks.algo_bytes += (double)n * ((NWP + 4) * 4 + NWP * 4 + 8);
    sh_next_write_ += (u64)n; sh_new_ += (u64)n;
    return 0;
  }

  int shard_level_stats(int64_t* st, std::string& err) override {
    u64 c[K_NCTR];
    HIPCHK(hipMemcpy(c, d_ctr_, sizeof c, hipMemcpyDeviceToHost));
    std::memset(st, 0, MC_SHARD_NSTAT * sizeof(int64_t));
    st[0] = (int64_t)sh_new_;
    int64_t gen = 0;
    for (int k = 0; k < OA_NACT; ++k) { st[8 + k] = (int64_t)c[K_ACT + k]; st[40 + k] = (int64_t)c[K_ACT + OA_NACT + k]; gen += (int64_t)c[K_ACT + k]; }
    st[1] = gen; st[2] = (int64_t)c[K_GEN_IN];
    st[3] = (int64_t)(c[K_ERR] | (sh_next_write_ > cap_ ? (u64)OE_CAP_STORE : 0ull));
    st[4] = (int64_t)c[K_VIOL]; st[5] = (int64_t)c[K_DEADLOCK]; st[6] = (int64_t)sh_level_count_;
    return 0;
  }

  int shard_level_commit(const int64_t* g, int* done, std::string& err) override {
    sres_.generated += g[1];
    sres_.generated_in_model += g[2];
    for (int k = 0; k < OA_NACT; ++k) { sres_.act_generated[k] += g[8 + k]; sres_.act_distinct[k] += g[40 + k]; }
    sres_.levels.back().generated = g[1];
    *done = 0;
    if (g[3]) {
      sres_.verdict = (g[3] & (OE_CAP_STORE | OE_TABLE_FULL | OE_CAP_ELECTIONS | OE_CAP_COUNT)) ? MC_VERDICT_CAPACITY_OVERFLOW : MC_VERDICT_EVAL_ERROR;
      std::ostringstream os; os << "error flags 0x" << std::hex << g[3] << " raised on some rank"; sres_.error = os.str();
      *done = 1;
    }
    sres_.distinct += g[0];
    if (g[0] > 0) { sres_.levels.push_back({g[0], 0, 0.0}); sres_.depth += 1; }
    if (!*done && g[4]) { sres_.verdict = MC_VERDICT_INVARIANT_VIOLATION; *done = 1; sres_.left_on_queue = g[0]; }
    if (!*done && sopts_.check_deadlock && g[5]) { sres_.verdict = MC_VERDICT_DEADLOCK; *done = 1; sres_.left_on_queue = g[0]; }
    if (!*done && g[0] == 0) *done = 1;
    if (!*done && sopts_.max_depth && sres_.depth >= sopts_.max_depth) { sres_.verdict = MC_VERDICT_DEPTH_LIMIT; sres_.left_on_queue = g[0]; *done = 1; }
    // advance the local level
    sh_level_begin_ += sh_level_count_;
    sh_level_count_ = sh_new_;
    total_ = sh_next_write_;
    sh_new_ = 0;
    HIPCHK(hipMemset(d_ctr_, 0, K_NCTR * 8));
    sres_.n_launches += 1;
    if (*done) {
      if (sres_.verdict == MC_VERDICT_INVARIANT_VIOLATION) {
        ViolRec<S> v; (void)hipMemcpy(&v, d_viol_, sizeof v, hipMemcpyDeviceToHost);
        sviol_parent_ = ((u64)rank_ << 37) | v.parent; sviol_act_ = kOrigActNames[v.act]; sviol_text_ = state_text(v.w, true);
        sviol_bad_ = v.bad;
        sres_.violated = first_violated(v.bad);
      }
      double secs = 0; for (auto& k : sres_.kernels) secs += k.ms / 1000.0;
      sres_.seconds_kernels = secs;
      finish(sres_, st0_);
    }
    return 0;
  }

  int shard_read_state(uint64_t gid, std::string& text, uint64_t* meta, std::string& err) const override {
    const u64 local = gid & ((1ull << 37) - 1);
    if (local >= total_) { err = "shard_read_state: state id outside this rank's store"; return MC_E_INVALID; }
    u32 w[NWP]; u64 m = 0;
    if (hipMemcpy(w, d_states_ + local * NWP, NWP * 4, hipMemcpyDeviceToHost) != hipSuccess ||
        hipMemcpy(&m, d_meta_ + local, 8, hipMemcpyDeviceToHost) != hipSuccess) { err = "readback failed"; return MC_E_NO_DEVICE; }
    W s; S::unpack(w, s);
    text = state_text(s, true);
    if (meta) *meta = m;
    return 0;
  }
  int shard_violation(uint64_t* parent, std::string& action, std::string& text) const override {
    if (parent) *parent = sviol_parent_;
    action = sviol_act_; text = sviol_text_;
    return sviol_act_.empty() ? MC_E_STATE : 0;
  }
  const RunResult* shard_result() const override { return &sres_; }

  // ---------------------------------------------------------------- native level loop over RCCL
  // The whole sharded BFS of raft-tla_amd/shard.py (sharded_bfs) in C++ on one HIP stream:
  // per chunk generate+route -> counts exchange -> ROUTE payload -> dedup -> counts exchange ->
  // REPLY payload -> materialize -> STATES payload -> store, with grouped ncclSend/ncclRecv
  // straight from the kernels' buffers (no staging copies) and two host synchronisations per
  // chunk (the counts) plus one per level (the all-reduce of the level statistics).
  int shard_run_native(void* comm_v, std::string& err) override {
    RcclApi& R = rccl();
    if (!R.ok) { err = "RCCL not loaded"; return MC_E_STATE; }
    ncclComm_t comm = (ncclComm_t)comm_v;
#define NCCLCHK(x)                                                                                   \
  do {                                                                                               \
    ncclResult_t r_ = (x);                                                                           \
    if (r_ != ncclSuccess) { err = std::string(#x) + ": " + R.GetErrorString(r_); return MC_E_NO_DEVICE; } \
  } while (0)
    const int W = world_, me = rank_;
    const u64 SBW = (u64)(NWP + 4) * 4;          // STATES record bytes
    if (!d_nat_) HIPCHK(hipMalloc(&d_nat_, (32 + 2 * MC_SHARD_NSTAT) * 8));
    if (!h_nat_) HIPCHK(hipHostMalloc(&h_nat_, (32 + 2 * MC_SHARD_NSTAT) * 8));
    u64* d_xs = d_nat_;        // [0,8) counts I send  (copied from d_rcnt_)
    u64* d_xr = d_nat_ + 8;    // [8,16) counts I receive
    int64_t* d_sum = (int64_t*)(d_nat_ + 32);
    int64_t* d_max = d_sum + MC_SHARD_NSTAT;
    u64* h_xs = h_nat_; u64* h_xr = h_nat_ + 8;
    int64_t* h_sum = (int64_t*)(h_nat_ + 32);
    int64_t* h_max = h_sum + MC_SHARD_NSTAT;
    // grow-only device buffer
    auto grow = [&](void*& p, u64& cap, u64 need) -> int {
      if (need <= cap) return 0;
      if (p) { HIPCHK(hipStreamSynchronize(stream_)); HIPCHK(hipFree(p)); p = nullptr; }
      cap = std::max<u64>(need + need / 4, 1 << 20);
      HIPCHK(hipMalloc(&p, cap));
      return 0;
    };
    // counts exchange: send[r] from d_send (device), received into d_xr; both land on the host
    auto xcounts = [&](const u64* d_send) -> int {
      HIPCHK(hipMemcpyAsync(d_xs, d_send, 8 * (u64)W, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(d_xr + me, d_send + me, 8, hipMemcpyDeviceToDevice, stream_));
      if (W > 1) {
        NCCLCHK(R.GroupStart());
        for (int r = 0; r < W; ++r) {
          if (r == me) continue;
          NCCLCHK(R.Send(d_xs + r, 1, ncclUint64, r, comm, stream_));
          NCCLCHK(R.Recv(d_xr + r, 1, ncclUint64, r, comm, stream_));
        }
        NCCLCHK(R.GroupEnd());
      }
      HIPCHK(hipMemcpyAsync(h_xs, d_xs, 16 * 8, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
      return 0;
    };
    // payload exchange: segment r of the send side (bytes) goes to rank r, the receive side is
    // packed in source-rank order; the self segment is not copied (its consumer reads it in
    // place), so dst + roff[me] stays unused
    auto xpay = [&](const char* const* src, const u64* sbytes, char* dst, const u64* rbytes) -> int {
      u64 roff[8]; u64 acc = 0;
      for (int r = 0; r < W; ++r) { roff[r] = acc; acc += rbytes[r]; }
      if (sbytes[me] != rbytes[me]) { err = "sharded exchange: self segment size mismatch"; return MC_E_STATE; }
      if (W > 1) {
        NCCLCHK(R.GroupStart());
        for (int r = 0; r < W; ++r) {
          if (r == me) continue;
          if (sbytes[r]) NCCLCHK(R.Send(src[r], sbytes[r], ncclUint8, r, comm, stream_));
          if (rbytes[r]) NCCLCHK(R.Recv(dst + roff[r], rbytes[r], ncclUint8, r, comm, stream_));
        }
        NCCLCHK(R.GroupEnd());
      }
      return 0;
    };
    // HIP-event timing, read back at the level's synchronisation points
    std::vector<std::pair<int, int>> pending;   // (kernel index, event pair index)
    auto ev_pair = [&](int k) -> int {
      const int i = (int)pending.size();
      while ((int)nat_ev_.size() < 2 * (i + 1)) { hipEvent_t e; if (hipEventCreate(&e) != hipSuccess) return -1; nat_ev_.push_back(e); }
      pending.push_back({k, i});
      return i;
    };
    auto harvest = [&]() {
      for (auto& pr : pending) {
        float ms = 0;
        (void)hipEventElapsedTime(&ms, nat_ev_[2 * pr.second], nat_ev_[2 * pr.second + 1]);
        sres_.kernels[pr.first].ms += ms;
      }
      pending.clear();
    };
#define NAT_TIMED(k, launch)                                                   \
  do {                                                                         \
    const int ep_ = ev_pair(k);                                                \
    if (ep_ < 0) { err = "hipEventCreate failed"; return MC_E_NO_DEVICE; }     \
    HIPCHK(hipEventRecord(nat_ev_[2 * ep_], stream_));                         \
    launch;                                                                    \
    HIPCHK(hipGetLastError());                                                 \
    HIPCHK(hipEventRecord(nat_ev_[2 * ep_ + 1], stream_));                     \
    sres_.kernels[k].launches++;                                               \
  } while (0)
    auto allreduce_level = [&](int64_t* g, int64_t next_chunks, int64_t& chunks_out) -> int {
      // g: local stats in, global stats out; MAX slots: [3,6) flags, [6] chunk rounds of the next level
      for (int k = 0; k < MC_SHARD_NSTAT; ++k) h_sum[k] = g[k];
      for (int k = 0; k < MC_SHARD_NSTAT; ++k) h_max[k] = 0;
      h_max[3] = g[3]; h_max[4] = g[4]; h_max[5] = g[5]; h_max[6] = next_chunks;
      HIPCHK(hipMemcpyAsync(d_sum, h_sum, 2 * MC_SHARD_NSTAT * 8, hipMemcpyHostToDevice, stream_));
      if (W > 1) {
        NCCLCHK(R.GroupStart());
        NCCLCHK(R.AllReduce(d_sum, d_sum, MC_SHARD_NSTAT, ncclInt64, ncclSum, comm, stream_));
        NCCLCHK(R.AllReduce(d_max, d_max, 8, ncclInt64, ncclMax, comm, stream_));
        NCCLCHK(R.GroupEnd());
      }
      HIPCHK(hipMemcpyAsync(h_sum, d_sum, 2 * MC_SHARD_NSTAT * 8, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
      for (int k = 0; k < MC_SHARD_NSTAT; ++k) g[k] = h_sum[k];
      g[3] = h_max[3]; g[4] = h_max[4]; g[5] = h_max[5];
      chunks_out = h_max[6];
      return 0;
    };

    const u64 chunk = chunk_states_;
    auto rounds = [&](u64 n) -> int64_t { return (int64_t)((n + chunk - 1) / chunk); };
    int64_t nchunks = 0;
    {   // agree on the first level's chunk rounds (only the owner of Init holds a state)
      int64_t z[MC_SHARD_NSTAT] = {0};
      if (int rc = allreduce_level(z, rounds(sh_level_count_), nchunks)) return rc;
    }
    const u64 route_cap = chunk_states_ * S::NI;
    for (;;) {
      const u64 front = sh_level_count_;
      for (int64_t c = 0; c < nchunks; ++c) {
        const u64 begin = std::min<u64>((u64)c * chunk, front);
        const u64 count = std::min<u64>(chunk, front - begin);
        sh_chunk_begin_ = sh_level_begin_ + begin; sh_chunk_count_ = count;
        HIPCHK(hipMemsetAsync(d_rcnt_, 0, 16 * 8, stream_));
        if (count > 0) {
          const u64 nslots = count * (u64)S::NI;
          GenArgs g;
          g.states = d_states_; g.chunk_begin = sh_chunk_begin_; g.chunk_count = count; g.cand = d_cand_; g.seed = sres_.seed;
          g.rt = m_.rt; g.inv_oom = sopts_.inv_out_of_model ? 1u : 0u; g.ctr = (unsigned long long*)d_ctr_; g.viol = d_viol_;
          const unsigned nblk = (unsigned)((count + BS - 1) / BS);
          NAT_TIMED(0, hipLaunchKernelGGL((orig_generate<S, true>), dim3(nblk), dim3(BS), 0, stream_, g));
          sres_.kernels[0].algo_bytes += (double)count * NWP * 4 + (double)nslots * 8;
          RouteArgs ra;
          ra.cand = d_cand_; ra.nslots = nslots; ra.route = d_route_; ra.route_cap = route_cap; ra.world = (u32)W;
          ra.rcnt = (unsigned long long*)d_rcnt_;
          NAT_TIMED(1, hipLaunchKernelGGL((orig_route_blk<S::NI>), dim3(nblk), dim3(BS), 0, stream_, ra));
          sres_.kernels[1].algo_bytes += (double)nslots * 8;
        }
        // ---- ROUTE: (fp, slot) records to the fingerprints' owners
        if (int rc = xcounts(d_rcnt_)) return rc;
        u64 scnt[8], rcnt[8], sb[8], rb[8], rtot = 0;
        const char* src[8];
        for (int r = 0; r < W; ++r) {
          scnt[r] = h_xs[r]; rcnt[r] = h_xr[r]; rtot += rcnt[r];
          sb[r] = scnt[r] * 16; rb[r] = rcnt[r] * 16;
          src[r] = (const char*)(d_route_ + (u64)r * route_cap * 2);
          sres_.kernels[1].algo_bytes += (double)scnt[r] * 16;
        }
        if (rtot > route_cap) { err = "shard: received more ROUTE records than one chunk holds"; return MC_E_STATE; }
        if (int rc = grow(nat_recv_, nat_recv_cap_, rtot * 16)) return rc;
        if (int rc = xpay(src, sb, (char*)nat_recv_, rb)) return rc;
        // ---- owner-side dedup, one launch per source rank
        {
          u64 off = 0;
          for (int r = 0; r < W; ++r) {
            seg_off_[r] = off;
            const u64 n = rcnt[r];
            if (n) {
              DedupShArgs d;
              d.recv = r == me ? d_route_ + (u64)me * route_cap * 2 : (const u64*)nat_recv_ + 2 * off;
              d.n = n; d.table = d_table_; d.table_mask = table_mask_;
              d.reply = d_newrec_ + off; d.counter = (unsigned long long*)(d_rcnt_ + 8 + r); d.ctr = (unsigned long long*)d_ctr_;
              NAT_TIMED(2, hipLaunchKernelGGL(orig_dedup_sh, dim3((unsigned)((n + BS * DEDUP_PER - 1) / (BS * DEDUP_PER))), dim3(BS), 0, stream_, d));
            }
            off += n;
          }
        }
        // ---- REPLY: the new ones' slots back to the generating ranks
        if (int rc = xcounts(d_rcnt_ + 8)) return rc;
        u64 rep[8], ack[8], atot = 0, ntot = 0;
        for (int r = 0; r < W; ++r) {
          rep[r] = h_xs[r]; ack[r] = h_xr[r]; atot += ack[r]; ntot += rep[r];
          sb[r] = rep[r] * 8; rb[r] = ack[r] * 8;
          src[r] = (const char*)(d_newrec_ + seg_off_[r]);
        }
        sres_.kernels[2].algo_bytes += (double)rtot * 24 + (double)ntot * 16;
        if (int rc = grow(nat_acks_, nat_acks_cap_, atot * 8)) return rc;
        if (int rc = xpay(src, sb, (char*)nat_acks_, rb)) return rc;
        // ---- generator re-derives the acknowledged states
        {
          u64 off = 0;
          for (int r = 0; r < W; ++r) { seg_off_ack_[r] = off; off += ack[r]; }
          void* so = d_stout_;
          u64 socap = stout_cap_ * SBW;
          if (int rc = grow(so, socap, atot * SBW)) return rc;
          d_stout_ = (u32*)so; stout_cap_ = socap / SBW;
          for (int r = 0; r < W; ++r) {
            if (!ack[r]) continue;
            MatShArgs m;
            m.states = d_states_; m.acks = r == me ? d_newrec_ + seg_off_[me] : (const u64*)nat_acks_ + seg_off_ack_[r];
            m.n = ack[r]; m.chunk_begin = sh_chunk_begin_;
            m.chunk_count = sh_chunk_count_; m.out = d_stout_ + seg_off_ack_[r] * (NWP + 4); m.rank_bits = (u64)me << 37;
            m.seed = sres_.seed; m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_; m.viol = d_viol_;
            NAT_TIMED(3, hipLaunchKernelGGL((orig_materialize_sh<S>), dim3((unsigned)((ack[r] + BS - 1) / BS)), dim3(BS), 0, stream_, m));
          }
          sres_.kernels[3].algo_bytes += (double)atot * (8 + NWP * 4 + SBW);
        }
        // ---- STATES: packed states + parent pointers to their owners (sizes known: no sync)
        for (int r = 0; r < W; ++r) { sb[r] = ack[r] * SBW; rb[r] = rep[r] * SBW; src[r] = (const char*)(d_stout_ + seg_off_ack_[r] * (NWP + 4)); }
        if (int rc = grow(nat_stin_, nat_stin_cap_, ntot * SBW)) return rc;
        if (int rc = xpay(src, sb, (char*)nat_stin_, rb)) return rc;
        {   // the owner stores the states in source-rank order (its own ones straight from d_stout_)
          u64 in_off = 0;
          for (int r = 0; r < W; ++r) {
            const u64 n = rep[r];
            if (n) {
              StoreArgs a;
              a.in = r == me ? d_stout_ + seg_off_ack_[me] * (NWP + 4) : (const u32*)((const char*)nat_stin_ + in_off * SBW);
              a.n = n; a.dst = sh_next_write_; a.cap = cap_; a.states = d_states_; a.meta = d_meta_;
              a.ctr = (unsigned long long*)d_ctr_;
              NAT_TIMED(4, hipLaunchKernelGGL((orig_store<NWP>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_, a));
              sres_.kernels[4].algo_bytes += (double)n * (SBW + NWP * 4 + 8);
              sh_next_write_ += n; sh_new_ += n;
            }
            in_off += n;
          }
        }
      }
      HIPCHK(hipStreamSynchronize(stream_));
      harvest();
      int64_t g[MC_SHARD_NSTAT];
      if (int rc = shard_level_stats(g, err)) return rc;
      int64_t next_chunks = 0;
      if (int rc = allreduce_level(g, rounds(sh_new_), next_chunks)) return rc;
      int done = 0;
      if (int rc = shard_level_commit(g, &done, err)) return rc;
      if (done) break;
      nchunks = next_chunks;
    }
#undef NAT_TIMED
#undef NCCLCHK
    return 0;
  }

 private:
  OrigModel m_;
  u64* d_table_ = nullptr; u32* d_states_ = nullptr; u64* d_meta_ = nullptr; u64* d_ctr_ = nullptr; void* d_viol_ = nullptr;
  u64* d_cand_ = nullptr; u64* d_newrec_ = nullptr;
  u64* d_route_ = nullptr; u64* d_rcnt_ = nullptr; u32* d_stout_ = nullptr; u64 stout_cap_ = 0;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_[9] = {};
  u64 table_mask_ = 0, cap_ = 0, total_ = 0, chunk_states_ = 0;
  int dev_ = -1, alloc_world_ = 0; uint64_t req_table_ = 0, req_store_ = 0;
  // sharded-mode state
  int rank_ = 0, world_ = 1;
  RunOpts sopts_;
  RunResult sres_;
  std::chrono::steady_clock::time_point st0_;
  u64 sh_level_begin_ = 0, sh_level_count_ = 0, sh_next_write_ = 0, sh_new_ = 0, sh_chunk_begin_ = 0, sh_chunk_count_ = 0;
  u64 seg_off_[8] = {0}, seg_off_ack_[8] = {0}, fill_counts_reply_[8] = {0}, fill_counts_states_[8] = {0};
  u64 fill_counts_route_[8] = {0};
  u64 sviol_parent_ = 0; u32 sviol_bad_ = 0; std::string sviol_act_, sviol_text_;
  // native (RCCL) level loop buffers
  u64* d_nat_ = nullptr; u64* h_nat_ = nullptr;
  void* nat_recv_ = nullptr; void* nat_acks_ = nullptr; void* nat_stin_ = nullptr;
  u64 nat_recv_cap_ = 0, nat_acks_cap_ = 0, nat_stin_cap_ = 0;
  std::vector<hipEvent_t> nat_ev_;
  std::vector<hipEvent_t> lvl_ev_;
  // completed levels moved to host memory: global ids [0, base_) live in host_states_/host_meta_
  u64 base_ = 0;
  std::vector<u32> host_states_;
  std::vector<u64> host_meta_;

  void release() {
    for (void* p : {(void*)d_table_, (void*)d_states_, (void*)d_meta_, (void*)d_ctr_, d_viol_, (void*)d_cand_, (void*)d_newrec_,
                    (void*)d_route_, (void*)d_rcnt_, (void*)d_stout_})
      if (p) (void)hipFree(p);
    for (void* p : {(void*)d_nat_, nat_recv_, nat_acks_, nat_stin_})
      if (p) (void)hipFree(p);
    if (h_nat_) (void)hipHostFree(h_nat_);
    d_nat_ = nullptr; h_nat_ = nullptr; nat_recv_ = nat_acks_ = nat_stin_ = nullptr;
    nat_recv_cap_ = nat_acks_cap_ = nat_stin_cap_ = 0;
    for (auto& e : nat_ev_) (void)hipEventDestroy(e);
    nat_ev_.clear();
    for (auto& e : lvl_ev_) (void)hipEventDestroy(e);
    lvl_ev_.clear();
    for (auto& e : ev_) { if (e) (void)hipEventDestroy(e); e = nullptr; }
    if (stream_) (void)hipStreamDestroy(stream_);
    d_table_ = nullptr; d_states_ = nullptr; d_meta_ = nullptr; d_ctr_ = nullptr; d_viol_ = nullptr;
    d_cand_ = nullptr; d_newrec_ = nullptr; d_route_ = nullptr; d_rcnt_ = nullptr; d_stout_ = nullptr; stout_cap_ = 0;
    stream_ = nullptr; alloc_world_ = 0;
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

  // stored state `gid` (global id) and its parent pointer, from the host part or the device
  bool stored_state(u64 gid, u32 (&w)[NWP], u64& meta) const {
    if (gid < base_) {
      std::memcpy(w, host_states_.data() + gid * NWP, NWP * 4);
      meta = host_meta_[gid];
      return true;
    }
    const u64 d = gid - base_;
    return hipMemcpy(w, d_states_ + d * NWP, NWP * 4, hipMemcpyDeviceToHost) == hipSuccess &&
           hipMemcpy(&meta, d_meta_ + d, 8, hipMemcpyDeviceToHost) == hipSuccess;
  }

  // move the completed levels [base_, level_begin) to host memory and the frontier to the
  // front of the device store (left shift by d in blocks of <= d slots: each block's target
  // only overlaps blocks already moved)
  int spill(u64 level_begin, u64 level_count, std::string& err) {
    const u64 d = level_begin - base_;
    const u64 h0 = host_meta_.size();
    host_states_.resize((h0 + d) * NWP);
    host_meta_.resize(h0 + d);
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(host_states_.data() + h0 * NWP, d_states_, d * NWP * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(host_meta_.data() + h0, d_meta_, d * 8, hipMemcpyDeviceToHost));
    for (u64 off = 0; off < level_count; off += d) {
      const u64 n = std::min<u64>(d, level_count - off);
      HIPCHK(hipMemcpyAsync(d_states_ + off * NWP, d_states_ + (d + off) * NWP, n * NWP * 4, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(d_meta_ + off, d_meta_ + d + off, n * 8, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
    }
    base_ = level_begin;
    return 0;
  }

  // parent-pointer chase on the host (<= depth device reads of one state each)
  void build_trace(u64 parent, const char* last_act, const W& last, RunResult& r, std::string& err) {
    std::vector<std::pair<std::string, std::string>> tr;
    if (last_act) tr.push_back({last_act, state_text(last, true)});
    u64 g = parent;
    while (true) {
      u32 w[NWP]; u64 meta = 0;
      if (!stored_state(g, w, meta)) { err = "trace readback failed"; break; }
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
  X(2, 2, 3, 2, 6)          \
  X(5, 1, 3, 3, 4) /* C5 */
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
