// raftmc — gfx950 BFS backend for thirdparty/raft_original.tla.
//
// TLC's single-worker FIFO order, reproduced on a data-parallel GPU.  Every successor has the
// key  (global id of its parent) << 8 | instance,  where the instance index is its position in
// TLC's enumeration of the Next disjuncts (raft_original.tla:453-462; the order-preserving
// message codes of orig_spec.h make bag slot order the order of `\E m \in DOMAIN messages`).
// States are stored level by level in key order, so parent ids increase in FIFO order and the
// key is globally monotone over the whole search: the seen-set keeps the MINIMUM key per
// fingerprint (16-B entries {fp, ~key}, atomicMax on the complement), i.e. TLC's first-found
// parent, and every count, parent pointer, counterexample and stop point is TLC's.
//
// One BFS level is processed in frontier chunks; each chunk runs on one stream:
//
//  1. orig_generate  (compute): one lane per frontier state, a wave-uniform loop over the
//     action instances; constraint filter, TLC generated counts, out-of-model invariants (TLC
//     semantics, [ext] switch), canonical pack and FP64 of each in-model successor.  The
//     workgroup's in-model successors are compacted (wave ballot + one LDS atomic per wave and
//     instance) into its own record region: fp (8 B) + local key lane << 8 | instance (2 B).
//  2. orig_dedup     (HBM random access): workgroup b takes generate-workgroup b's records; a
//     workgroup-local LDS set {fp, min local key} merges the successors its 256 parents produce
//     more than once (diamonds of commuting actions, ~half of C2's), then every distinct fp of
//     the set probes the seen-set, 16 in flight per thread (lock-free linear probing over 16-B
//     entries, CAS insert of the fp, atomicMax of ~key).  Inserted entries' positions are
//     appended (one global atomic per workgroup).
//  3. orig_mark      lane per inserted entry: its final key names TLC's first-found producer;
//     set that (parent, instance) bit of the winner mask, count per workgroup of parents.
//  4. orig_scan      exclusive scan of the per-workgroup winner counts (one workgroup).
//  5. orig_materialize workgroup per 256 parents: winners in key order (parent-major, instance
//     order), re-derived from (parent, instance), stored with their parent pointers at their
//     FIFO position; invariants of the new states.
//  6. orig_advance   the level's running count of new states.
//
// The first *event* of a level in key order — a TLC evaluation error while computing a
// parent's successors, a deadlock, an invariant violation (new or out-of-model successor) — is
// a 64-bit atomicMin of key << 2 | kind; the host re-derives that successor with the same
// spec code and reproduces TLC's stop point (generated / distinct / per-action counts /
// left-on-queue) and counterexample.  All distinct states stay resident in HBM (completed
// levels spill to host memory when the store fills); traces chase parent pointers.
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <functional>
#include <map>
#include <sstream>
#include <type_traits>

#include "../../include/raftmc.h"
#include "backend.h"
#include "fp_gap.h"
#include "host_store.h"
#include "orig_spec.h"
#include "orig_text.h"
#include "rccl_api.h"
#include "shard_transport.h"

namespace rmc {

enum {
  K_NEW = 0, K_GEN_IN = 1, K_ERR = 2, K_EVENT = 3, K_ERRGID = 4, K_INS = 5, K_CHUNK_NEW = 6, K_LEVEL_NEW = 7,
  K_ACT = 8, K_PROF = K_ACT + 2 * OA_NACT,   // K_PROF: phase timers (RAFTMC_PROF, slots 0..5)
  K_PROBES = K_PROF + 6,                       // seen-set probes issued (fingerprints that reached the table)
  K_LEAD = K_PROF + 7,                         // the chunk's leader-work parents (orig_generate_lead)
  K_NCTR = K_PROF + 8
};
enum { EV_NEXT_ERROR = 0, EV_DEADLOCK = 1, EV_INV_ERROR = 2, EV_VIOLATION = 3 };
enum { OE_CAP_STORE = 0x100, OE_TABLE_FULL = 0x200 };
// Seen-set batches and the LDS filter (round 5, profiles/r05_dedup_ab.txt r5x-r6a): 4 probes in flight
// per thread at 50 VGPRs and a 2048-slot filter (18.4 KB of LDS) give 8 workgroups per CU, the wave
// limit, where 8 probes at 92 VGPRs and 4096 slots (34.8 KB) gave 4: orig_dedup_plain 11.5 -> 10.4 ms
// per C2 run although 3.5% more fingerprints get past the smaller filter (351M probes, not 339M); the
// FIFO path 35.9 -> 34.8 ms.  16 per thread (183 VGPRs) 16.4 ms, 1024 slots 11.1 ms.
constexpr int DEDUP_PER = 4;                  // probes in flight per dedup thread
constexpr int BS = 256;                       // workgroup size of every kernel (4 waves)
constexpr int LDS_FP_SLOTS = 2048;            // workgroup-local fingerprint set (8 B fp + 4 B key per slot)
constexpr int MAT_CAP = 2048;      // winners staged in LDS per materialize round
#ifndef RMC_RV_PATCH
#define RMC_RV_PATCH 0
#endif
#ifndef RMC_RV_WCOUNT
#define RMC_RV_WCOUNT 0
#endif
constexpr int SCAN_BS = 1024;      // orig_scan workgroup

// f(std::integral_constant<int, Q>) for Q = B .. E-1: a loop whose index is a compile-time constant
template <int B, int E, class F>
__device__ __forceinline__ void static_for(F&& f) {
  if constexpr (B < E) {
    f(std::integral_constant<int, B>{});
    static_for<B + 1, E>(f);
  }
}

// 64-bit event word: key << 2 | kind, key = parent gid << 8 | instance (gid < 2^40)
RMC_HD u64 ev_word(u64 gid, u32 inst, u32 kind) { return (((gid << 8) | (u64)inst) << 2) | (u64)kind; }

struct GenArgs {
  const u32* states;           // device store [cap][NWP]
  u64 chunk_begin, chunk_count;   // device index of the chunk's first parent, parents
  u64 gid0;                    // global id of the chunk's first parent
  u64* rfp;                    // [nblk][BS * NI] fingerprints of in-model successors (per-workgroup region)
  unsigned short* rkey;        // [nblk][BS * NI] local key: lane << 8 | instance
  u32* rcnt;                   // [nblk][4] records per wave (wave w's region starts at w * 64 * NI)
  u64 seed;
  OrigRuntime rt;
  u32 inv_oom, deadlock;
  unsigned long long* ctr;
  u32* lead;                   // [chunk] parents with leader work (chunk index | 1 << 31 if no other successor)
};

// One lane per frontier state; successor, constraints, TLC generated counts, out-of-model invariants,
// canonical pack and FP64 in one pass.  (A split expand + full-lane fingerprint pipeline measured
// 51.4 vs 49.4 ms/run on C2: apply, not the pack + hash, dominates this spec.)  Three sections:
//  * RequestVote(i, j): each lane's enabled instances one per trip (per-lane instance);
//  * a wave-uniform loop over the other instances (Restart, Timeout, Receive; the leader instances
//    [LEAD_LO, LEAD_HI) are orig_generate_lead's): k is a scalar, so the instance decode and the bag
//    slot selects are scalar work;
//  * DuplicateMessage / DropMessage unrolled per bag slot, without apply or pack.
// In-model successors leave as compacted records: per instance a wave ballot and consecutive stores
// into the wave's own region (only ~21% of C2's instance slots carry an in-model successor).
// Rejected designs (measured on MI355X; scripts/variants/orig_backend_experiments.hip builds them):
// instances binned by family for every family (19.5 vs 14.5 ms, round 4: a per-lane instance turns
// apply's whole dispatch into vector work), patch packing from the parent's words (14.45 vs 13.37 ms,
// round 5), per-wave aggregated action counts (+1.3 ms, round 2), DuplicateMessage / DropMessage
// through apply (13.37 -> 14.71 ms).
// 4 waves per SIMD (<= 128 VGPRs, no spill): 11.7 vs 13.4 ms per C2 run at 3 (round 5); 5 spills.
// Larger states (C5: 24 words) get no hint and keep the plain hash (the base terms would cost them
// occupancy: 45 vs 38 ms of expand time for C5 to depth 12).
template <class S>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(S::NW <= 15 ? 4 : 1))) orig_generate(GenArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  __shared__ unsigned int lds_cnt[OA_NACT + 1];   // per-action generated, in-model total
  for (int t = threadIdx.x; t < OA_NACT + 1; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 tid = (u64)blockIdx.x * BS + threadIdx.x;
  const bool active = tid < a.chunk_count;
  const u64 gid = a.gid0 + tid;
  const int lane = __lane_id();
  // each wave appends to its own region: the running count is wave-uniform, no LDS atomic per instance
  const u32 wave = __builtin_amdgcn_readfirstlane(threadIdx.x >> 6);   // wave-uniform (SGPR) region base
  const u64 wreg = (u64)blockIdx.x * (BS * S::NI) + (u64)wave * (64 * S::NI);
  u64* rfp = a.rfp + wreg;
  unsigned short* rkey = a.rkey + wreg;
  u32 wcount = 0;
  W s;
  u64 al[S::AW];
  u32 err = 0, nsucc = 0, nin = 0;
  unsigned long long ev = ~0ull;
  // the parent's packed words with allLogs' (every successor carries allLogs \cup {log[i]},
  // raft_original.tla:464) and their fingerprint terms: successors re-hash changed words only
  constexpr bool INC = NW <= 16;
  u32 bw[INC ? NW : 1];
  FpBase<INC ? NW : 2> fb;
  if (active) {
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(a.states + (a.chunk_begin + tid) * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    S::unpack(w, s);
    S::all_logs_next(s, al);
  } else {
    S::init(s);
#pragma unroll
    for (int q = 0; q < S::AW; ++q) al[q] = 0;
  }
  // bw = the parent with allLogs' (what every successor carries); a successor whose words equal bw is
  // the parent itself only when allLogs' = allLogs (no log of the parent is new to allLogs)
  bool al_same = true;
#pragma unroll
  for (int q = 0; q < S::AW; ++q) al_same &= al[q] == s.allLogs[q];
  if constexpr (INC) {
    W b = s;
#pragma unroll
    for (int q = 0; q < S::AW; ++q) b.allLogs[q] = al[q];
    S::pack(b, bw);
    fb.init(bw, a.seed);
  }
  // an in-model successor t (allLogs' applied): its fingerprint, and whether it leaves a record -- a
  // successor equal to its parent (Restart(i) of a server already in the reset state, allLogs' =
  // allLogs) is in the seen-set under an older key: no record, no probe (C2: 351M -> 313M seen-set
  // probes per run, round 6)
  auto fingerprint = [&](const W& t, u64& fp) -> bool {
    u32 pw[NW];
    S::pack(t, pw);
    if constexpr (INC) {
      bool changed;
      fp = fb.fp(pw, bw, a.seed, changed);
      return changed || !al_same;
    } else {
      fp = fp64(pw, a.seed);
      return true;
    }
  };
  // this wave's in-model successors of one trip into its record region (one ballot, consecutive stores)
  auto append = [&](bool have, u64 fp, int k) {
    const u64 mask = __ballot(have);
    if (have) {
      const u32 idx = wcount + __builtin_amdgcn_mbcnt_hi((u32)(mask >> 32), __builtin_amdgcn_mbcnt_lo((u32)mask, 0u));
      rfp[idx] = fp;
      rkey[idx] = (unsigned short)((threadIdx.x << 8) | (unsigned)k);
    }
    wcount += (u32)__popcll(mask);
  };
  // leader work (S::leader_work: a Leader or a Candidate with a quorum, ~1% of C2's states) is
  // left to orig_generate_lead, which runs those instances on full waves of just such parents: here
  // a wave with one leader lane would pay all of [LEAD_LO, LEAD_HI) for it (measured: a third of
  // this kernel's time for 0.7% of C2's successors)
  const bool lead = active && S::leader_work(s);
  {
    // RequestVote(i, j) [2N, 2N + N*N) (raft_original.tla:189-198): each lane's enabled instances one
    // per trip (S::request_vote_mask), so the wave runs as often as its busiest lane has RequestVote
    // instances instead of N*N times (C2: 6.3 trips per wave against 9, tests/native/orig_host_bfs.cpp
    // WAVE=64 "rv_waves"; orig_generate 11.1 -> 9.8 ms per run, round 6).  The handler is one short
    // function of (i, j) (S::request_vote), so a per-lane instance costs a few VALU ops here.
    u32 rvm = active ? S::request_vote_mask(s) : 0u;
#pragma unroll 1
    while (__ballot(rvm != 0u)) {
      const bool on = rvm != 0u;
      const int q = on ? __builtin_ctz(rvm) : 0;
      if (on) rvm &= rvm - 1u;
      const int k = 2 * S::N + q;
      bool have = false;
      u64 fp = 0;
      if (on) {
        W t = s;
        const int act = S::request_vote(s, q / S::N, q % S::N, t, err);
        if (act >= 0) {
#pragma unroll
          for (int w2 = 0; w2 < S::AW; ++w2) t.allLogs[w2] = al[w2];
          ++nsucc;
          if (!RMC_RV_WCOUNT) atomicAdd(&lds_cnt[act], 1u);
          if (S::in_model(t, a.rt)) {
            ++nin;
#if RMC_RV_PATCH
            if constexpr (INC) {
              // RequestVote changes only the bag: the parent's words with the bag re-packed, and only the
              // 64-bit words from the bag's first one re-hashed (both compile-time ranges)
              u32 pw[NW];
              S::pack_patch(t, 1u << S::PG_BAG, bw, pw);
              bool changed;
              fp = fb.template fp_tail<S::BAG_OFF / 64>(pw, bw, a.seed, changed);
              have = changed || !al_same;
            } else {
              have = fingerprint(t, fp);
            }
#else
            have = fingerprint(t, fp);
#endif
          }
          // out of the model: RequestVote writes only the bag, which no invariant reads (S::inv_frame)
        }
      }
      if (RMC_RV_WCOUNT) {   // every lane of the trip generates one RequestVote: one LDS atomic per wave
        const u64 gm = __ballot(on);
        if (lane == __ffsll((unsigned long long)gm) - 1) atomicAdd(&lds_cnt[OA_RequestVote], (unsigned)__popcll(gm));
      }
      append(have, fp, k);
    }
  }
  // DuplicateMessage / DropMessage [I_DUP, NI) change one message count and nothing else: with the
  // incremental fingerprint they are the unrolled section after this loop (no apply, no pack)
  constexpr int KEND = INC ? S::I_DUP : S::NI;
#pragma unroll 1
  for (int kk = 0; kk < KEND; ++kk) {
    if (kk == 2 * S::N) kk = S::LEAD_HI;   // RequestVote: the section above; leader work: orig_generate_lead
    const int k = kk;                      // wave-uniform
    const bool on = active;
    u64 fp = 0;
    bool have = false;
    const int qa = on ? S::quick_out_of_model(s, k, a.rt) : -1;
    if (qa >= 0) {      // generated, out of the model, no invariant to check: counted only
      ++nsucc;
      atomicAdd(&lds_cnt[qa], 1u);
    } else if (on) {
      W t;
      const int act = S::apply(s, k, t, err);
      if (act >= 0) {
#pragma unroll
        for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
        ++nsucc;
        atomicAdd(&lds_cnt[act], 1u);
        if (S::in_model(t, a.rt)) {
          ++nin;
          have = fingerprint(t, fp);
        } else if (a.inv_oom && S::violated(t, a.rt.invariants & S::inv_frame(act))) {
          // TLC checks invariants on out-of-model successors ([ext] switch (ii)); first in key order wins
          // (only those the action can change: the parent satisfies all of them, S::inv_frame)
          const u64 e = ev_word(gid, (u32)k, EV_VIOLATION);
          ev = e < ev ? e : ev;
        }
      }
    }
    append(have, fp, k);
  }
  if constexpr (KEND < S::NI) {
    // DuplicateMessage(m) / DropMessage(m) (raft_original.tla:442-449) for bag slot q, in instance
    // order, unrolled (q is a compile-time constant): the successor is the parent (allLogs' applied)
    // with one message count +-1 — the count field is the low CNTB bits of bag entry q, at the
    // compile-time bit offset BAG_OFF + q * ENTB of the packed state.  Every other constraint reads
    // what the parent already satisfies, so the successor is in the model iff BoundedMessages keeps
    // the new count in [MinMsgCount, MaxMsgCount]; no invariant reads the bag (S::inv_frame), so an
    // out-of-model one is only counted.  Its fingerprint re-mixes the one or two 64-bit words that
    // hold the field (FpBase::fp_add_bit): no apply, no pack.  (C2: 532M of the 1,348M generated
    // successors, 266M of the 590M in the model; orig_materialize_plain still re-derives the new
    // ones through S::apply.)  The per-action count is uniform over the wave: one ballot and one LDS
    // atomic per slot.
    const bool bounded = (a.rt.constraints & OC_BoundedMessages) != 0;
    static_for<0, 2 * S::MK>([&](auto qc) {
      constexpr int q = decltype(qc)::value;
      constexpr bool dup = q < S::MK;
      constexpr int slot = dup ? q : q - S::MK;
      constexpr int k = S::I_DUP + q;
      const typename S::BE ent = s.bag.v[slot];
      const bool on = active && ent != S::BEMPTY;
      const int c = S::ecount(ent) + (dup ? 1 : -1);
      bool have = false;
      u64 fp = 0;
      if (on) {
        ++nsucc;
        if (bounded && (c < a.rt.min_count || c > a.rt.max_count)) {
          // out of the model (S::quick_out_of_model): counted only
        } else if (c < -8 || c > 7) {
          err |= OE_CAP_COUNT;                              // the packed count field holds -8..7 (bag_add_at)
        } else {
          have = true;
          ++nin;
          fp = fb.template fp_add_bit<S::BAG_OFF + slot * S::ENTB>(bw, dup ? 1 : -1, a.seed);
        }
      }
      {
        const u64 om = __ballot(on);
        if (om && lane == __ffsll((unsigned long long)om) - 1)
          atomicAdd(&lds_cnt[dup ? OA_DuplicateMessage : OA_DropMessage], (unsigned)__popcll(om));
      }
      append(have, fp, k);
    });
  }
  if (active) {
    if (err & OE_EVAL_LOG_INDEX) { const u64 e = ev_word(gid, 0, EV_NEXT_ERROR); ev = e < ev ? e : ev; }
    if (nsucc == 0 && a.deadlock && !lead) { const u64 e = ev_word(gid, 0, EV_DEADLOCK); ev = e < ev ? e : ev; }
  }
  {   // leader-work parents to the chunk's list: one global atomic per wave
    const u64 lm = __ballot(lead);
    if (lm) {
      const int first = __ffsll((unsigned long long)lm) - 1;
      u32 base = 0;
      if (lane == first) base = (u32)atomicAdd(&a.ctr[K_LEAD], (unsigned long long)__popcll(lm));
      base = __shfl(base, first);
      if (lead) a.lead[base + (u32)__popcll(lm & ((1ull << lane) - 1ull))] = (u32)tid | (nsucc == 0 ? 0x80000000u : 0u);
    }
  }
  const u32 cap_err = err & ~(u32)OE_EVAL_LOG_INDEX;   // compiled-capacity limits, not TLC semantics
  if (cap_err) {
    atomicOr(&a.ctr[K_ERR], (unsigned long long)cap_err);
    atomicCAS(&a.ctr[K_ERRGID], 0ull, (unsigned long long)(gid + 1));
  }
  if (ev != ~0ull) atomicMin(&a.ctr[K_EVENT], ev);
  if (nin) atomicAdd(&lds_cnt[OA_NACT], nin);
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + t], (unsigned long long)lds_cnt[t]);
  if (threadIdx.x == 0 && lds_cnt[OA_NACT]) atomicAdd(&a.ctr[K_GEN_IN], (unsigned long long)lds_cnt[OA_NACT]);
  if (lane == 0) a.rcnt[blockIdx.x * 4 + wave] = wcount;
}

// The instances [LEAD_LO, LEAD_HI) of the chunk's leader-work parents (the list orig_generate wrote),
// one lane per parent on full waves: the same successor / constraint / count / pack / FP64 work as
// orig_generate, the in-model records appended to the parent's own wave region of its generate
// workgroup (global atomic on that wave's record count: the dedup kernels read whole regions, and
// record order inside a region is immaterial: the FIFO merge keeps the minimum key, the -workers N
// filter decides by key).
template <class S>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(S::NW <= 15 ? 4 : 1))) orig_generate_lead(GenArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  __shared__ unsigned int lds_cnt[OA_NACT + 1];
  for (int t = threadIdx.x; t < OA_NACT + 1; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 n = a.ctr[K_LEAD];
  constexpr bool INC = NW <= 16;
  u32 err = 0, nin = 0;
  unsigned long long ev = ~0ull;
  // grid-stride with a wave-uniform trip count (every lane of a wave runs the same instance loop)
  for (u64 i0 = (u64)blockIdx.x * BS; i0 < n; i0 += (u64)gridDim.x * BS) {
    const u64 i = i0 + threadIdx.x;
    const bool active = i < n;
    const u32 ent = active ? a.lead[i] : 0u;
    const u64 p = ent & 0x7fffffffu;                 // chunk index of the parent
    const u64 gid = a.gid0 + p;
    W s;
    u64 al[S::AW];
    if (active) {
      u32 w[NWP];
      const uint4* src = reinterpret_cast<const uint4*>(a.states + (a.chunk_begin + p) * NWP);
#pragma unroll
      for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
      S::unpack(w, s);
      S::all_logs_next(s, al);
    } else {
      S::init(s);
#pragma unroll
      for (int q = 0; q < S::AW; ++q) al[q] = 0;
    }
    u32 bw[INC ? NW : 1];
    FpBase<INC ? NW : 2> fb;
    bool al_same = true;   // allLogs' = allLogs: a successor equal to bw is the parent (orig_generate)
#pragma unroll
    for (int q = 0; q < S::AW; ++q) al_same &= al[q] == s.allLogs[q];
    if constexpr (INC) {
      W b = s;
#pragma unroll
      for (int q = 0; q < S::AW; ++q) b.allLogs[q] = al[q];
      S::pack(b, bw);
      fb.init(bw, a.seed);
    }
    const u32 blk = (u32)(p / BS), plane = (u32)(p % BS);
    const u64 wreg = (u64)blk * (BS * S::NI) + (u64)(plane >> 6) * (64 * S::NI);
    u32* wcnt = a.rcnt + blk * 4 + (plane >> 6);
    u32 nsucc = 0, perr = 0;
#pragma unroll 1
    for (int k = S::LEAD_LO; k < S::LEAD_HI; ++k) {
      if (!active) continue;
      W t;
      const int act = S::apply(s, k, t, perr);
      if (act < 0) continue;
#pragma unroll
      for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
      ++nsucc;
      atomicAdd(&lds_cnt[act], 1u);
      if (S::in_model(t, a.rt)) {
        ++nin;
        u32 pw[NW];
        S::pack(t, pw);
        u64 fp;
        if constexpr (INC) {
          bool changed;   // AdvanceCommitIndex(i) without an advance is its parent: no record
          fp = fb.fp(pw, bw, a.seed, changed);
          if (!changed && al_same) continue;
        } else {
          fp = fp64(pw, a.seed);
        }
        const u32 idx = atomicAdd(wcnt, 1u);
        a.rfp[wreg + idx] = fp;
        a.rkey[wreg + idx] = (unsigned short)((plane << 8) | (unsigned)k);
      } else if (a.inv_oom && S::violated(t, a.rt.invariants & S::inv_frame(act))) {
        const u64 e = ev_word(gid, (u32)k, EV_VIOLATION);
        ev = e < ev ? e : ev;
      }
    }
    if (active) {
      if (perr & OE_EVAL_LOG_INDEX) { const u64 e = ev_word(gid, 0, EV_NEXT_ERROR); ev = e < ev ? e : ev; }
      if ((ent >> 31) && nsucc == 0 && a.deadlock) { const u64 e = ev_word(gid, 0, EV_DEADLOCK); ev = e < ev ? e : ev; }
      const u32 ce = perr & ~(u32)OE_EVAL_LOG_INDEX;
      if (ce) { atomicCAS(&a.ctr[K_ERRGID], 0ull, (unsigned long long)(gid + 1)); err |= ce; }
    }
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
  if (ev != ~0ull) atomicMin(&a.ctr[K_EVENT], ev);
  if (nin) atomicAdd(&lds_cnt[OA_NACT], nin);
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + t], (unsigned long long)lds_cnt[t]);
  if (threadIdx.x == 0 && lds_cnt[OA_NACT]) atomicAdd(&a.ctr[K_GEN_IN], (unsigned long long)lds_cnt[OA_NACT]);
}

// Record i of workgroup b's four wave regions (concatenated in wave order): its offset in the
// workgroup's record region.  rc: the four per-wave counts; wreg = 64 * NI.
struct WaveRegions {
  u32 p1, p2, p3, n;
  u64 wreg;
  RMC_HD WaveRegions(const u32* rc, u64 wave_region) {
    p1 = rc[0]; p2 = p1 + rc[1]; p3 = p2 + rc[2]; n = p3 + rc[3]; wreg = wave_region;
  }
  RMC_HD u64 at(u32 i) const {
    const u32 w = (i >= p1) + (i >= p2) + (i >= p3);
    const u32 base = w == 0 ? 0u : w == 1 ? p1 : w == 2 ? p2 : p3;
    return (u64)w * wreg + (i - base);
  }
};

// Workgroup-local first-come fingerprint filter: answers only "certainly produced here before"
// (a full probe window lets the record through: the seen-set decides).  An empty slot is claimed
// by LDS CAS, so the set is exact up to the window: with plain stores (the round-4
// form, scripts/variants/orig_backend_experiments.hip RMC_LDS_PLAIN) two lanes inserting different fingerprints into one slot at once left one of them out of
// the set, and two lanes with the same fingerprint both passed.  Measured on C2 (round 5,
// profiles/r05_dedup_ab.txt): 339.5M seen-set probes per run instead of 367.0M, orig_dedup_plain
// 11.30 vs 11.51 ms; a 16-slot window changed nothing (366.5M: overflow is not the leak) and an
// 8192-slot set (64 KB) cost occupancy (14.96 ms).
constexpr int LDS_WIN = 8;   // probe window of the LDS filter
template <int SLOTS = LDS_FP_SLOTS>
__device__ __forceinline__ bool lds_first(unsigned long long* set, u64 fp) {
  u32 h = (u32)(fp >> 20) & (SLOTS - 1);
#pragma unroll 1
  for (int p = 0; p < LDS_WIN; ++p) {
    unsigned long long cur = set[h];
    if (cur == fp) return false;            // produced here before
    if (cur == 0ull) {                      // claim the slot; a lane that loses the race looks at the winner's fp
      cur = atomicCAS(&set[h], 0ull, (unsigned long long)fp);
      if (cur == 0ull) return true;
      if (cur == fp) return false;
    }
    h = (h + 1) & (SLOTS - 1);
  }
  return true;                              // window full: let the seen-set decide
}

// ------------------------------------------------------------------ seen-set probing
// The seen-set: 2^k entries of 16 B {fp, ~key} (0 = empty), linear probing.  probe_batch inserts
// or finds G fingerprints at once (independent probes in flight), then lowers each entry's key
// to the given one (atomicMax of the complement; a key only ever decreases, so an entry that
// already holds a smaller key needs no atomic: the common case, a duplicate of an older state).
// ins bit j = this call inserted fp[j]; pos[j] = its entry index.
template <int G, bool KEYED = true, int STRIDE = 2>
__device__ __forceinline__ u32 probe_batch(u64* table, u64 mask, const u64 (&fp)[G], const u64 (&nk)[G], u64 (&pos)[G], u32& err) {
  static_assert(!KEYED || STRIDE == 2, "keyed entries are {fp, ~key}");
  u64 cur[G], cnk[G];
#pragma unroll
  for (int j = 0; j < G; ++j) {
    pos[j] = fp[j] & mask;
    if (fp[j] && KEYED) {
      const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(table + 2 * pos[j]);
      cur[j] = e.x; cnk[j] = e.y;
    } else {
      cur[j] = fp[j] ? table[STRIDE * pos[j]] : ~0ull; cnk[j] = ~0ull;
    }
  }
  u32 ins = 0, lower = 0;
#pragma unroll
  for (int j = 0; j < G; ++j)
    if (fp[j] && cur[j] == 0ull) {
      cur[j] = (u64)atomicCAS((unsigned long long*)&table[STRIDE * pos[j]], 0ull, (unsigned long long)fp[j]);
      if (cur[j] == 0ull) { ins |= 1u << j; lower |= 1u << j; }
      else if (cur[j] == fp[j]) lower |= 1u << j;     // raced with another inserter of the same fp
    }
#pragma unroll
  for (int j = 0; j < G; ++j) {
    if (!fp[j] || ((lower >> j) & 1u)) continue;
    if (cur[j] == fp[j]) { if (KEYED && cnk[j] < nk[j]) lower |= 1u << j; continue; }
    u64 slot = (pos[j] + 1) & mask;
    for (u64 probe = 0;; ++probe) {
      if (probe > mask || probe >= (1u << 20)) { err |= OE_TABLE_FULL; break; }   // visited every entry
      u64 c, ck = ~0ull;
      if (KEYED) { const ulonglong2 e = *reinterpret_cast<const ulonglong2*>(table + 2 * slot); c = e.x; ck = e.y; }
      else c = table[STRIDE * slot];
      if (c == fp[j]) { if (KEYED && ck < nk[j]) lower |= 1u << j; break; }
      if (c == 0ull) {
        const u64 old = (u64)atomicCAS((unsigned long long*)&table[STRIDE * slot], 0ull, (unsigned long long)fp[j]);
        if (old == 0ull) { ins |= 1u << j; lower |= 1u << j; break; }
        if (old == fp[j]) { lower |= 1u << j; break; }
      }
      slot = (slot + 1) & mask;
    }
    pos[j] = slot;
  }
  if (KEYED) {
#pragma unroll
    for (int j = 0; j < G; ++j)
      if ((lower >> j) & 1u) atomicMax((unsigned long long*)&table[2 * pos[j] + 1], (unsigned long long)nk[j]);
  }
  return ins;
}

// one workgroup-wide exclusive scan of per-thread counts; returns this thread's offset, *total
__device__ __forceinline__ u32 block_excl_scan(u32 mine, u32* wave_tot, u32* total) {
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  u32 incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) { const u32 v = __shfl_up(incl, d); if (lane >= d) incl += v; }
  if (lane == 63) wave_tot[wave] = incl;
  __syncthreads();
  u32 base = 0, tot = 0;
#pragma unroll
  for (int w = 0; w < BS / 64; ++w) { const u32 x = wave_tot[w]; if (w < wave) base += x; tot += x; }
  *total = tot;
  __syncthreads();   // wave_tot may be reused
  return base + incl - mine;
}

struct DedupArgs {
  const u64* rfp;
  const unsigned short* rkey;
  const u32* rcnt;
  u64 region;                  // records per workgroup region (BS * NI)
  u64 gid0;                    // global id of the chunk's first parent
  ulonglong2* urec;            // [nblk][region] distinct (fp, ~key) of each workgroup's records
  u32* ucnt;                   // [nblk]
  u64* table;
  u64 table_mask;
  u64* newpos;                 // entry indices inserted by this chunk (ctr[K_INS] of them)
  unsigned long long* ctr;
  u32 prof;                    // accumulate per-workgroup wall-clock ticks into ctr[K_PROF..]
};

RMC_HD u64 nkey_of(u64 gid0, u32 blk, u32 lk) {   // ~(global key) of a local record key
  return ~(((gid0 + (u64)blk * BS + (lk >> 8)) << 8) | (u64)(lk & 255u));
}

// insert-or-find fp in the workgroup's LDS set and lower its slot's key to lk; false = window full
__device__ __forceinline__ bool lds_merge(unsigned long long* lfp, unsigned int* lkey, u64 fp, u32 lk) {
  u32 h = (u32)(fp >> 20) & (LDS_FP_SLOTS - 1);
#pragma unroll 1
  for (int p = 0; p < 8; ++p) {
    unsigned long long c = lfp[h];                                   // plain read first: most hits need no CAS
    if (c == 0ull) c = atomicCAS(&lfp[h], 0ull, (unsigned long long)fp);
    if (c == 0ull || c == fp) { atomicMin(&lkey[h], lk); return true; }
    h = (h + 1) & (LDS_FP_SLOTS - 1);
  }
  return false;
}

// Seen-set insertion, part 1 (LDS): workgroup b takes generate-workgroup b's records and merges
// them in an LDS set {fp, min local key} (exact: LDS CAS + LDS atomicMin; ~half of C2's
// successors repeat another successor of the same 256 parents).  The distinct (fp, ~global key)
// pairs are written compacted to the workgroup's region (a record whose probe window is full
// goes there with its own key: the seen-set keeps the minimum key anyway).  Splitting the merge
// from the probes lets the probe kernel run at the occupancy its registers allow, instead of
// the 3 workgroups per CU the 48-KB set allows (measured: fused merge + probes 17-21 ms of C2).
__global__ void __launch_bounds__(BS) orig_merge(DedupArgs a) {
  __shared__ unsigned long long lfp[LDS_FP_SLOTS];
  __shared__ unsigned int lkey[LDS_FP_SLOTS];
  __shared__ u32 wave_tot[BS / 64];
  __shared__ u32 ovf_cnt;
  for (int t = threadIdx.x; t < LDS_FP_SLOTS; t += BS) { lfp[t] = 0ull; lkey[t] = ~0u; }
  if (threadIdx.x == 0) ovf_cnt = 0;
  __syncthreads();
  const WaveRegions wr(a.rcnt + 4 * blockIdx.x, a.region / 4);
  const u32 n = wr.n;
  const u64* fps = a.rfp + (u64)blockIdx.x * a.region;
  const unsigned short* keys = a.rkey + (u64)blockIdx.x * a.region;
  ulonglong2* out = a.urec + (u64)blockIdx.x * a.region;
  // overflow records (probe window full) go to the END of the region, growing down
  constexpr int P1 = 8;
#pragma unroll 1
  for (u32 i0 = 0; i0 < n; i0 += P1 * BS) {
    u64 fp[P1];
    u32 lk[P1];
#pragma unroll
    for (int j = 0; j < P1; ++j) {
      const u32 i = i0 + (u32)j * BS + threadIdx.x;
      const u64 at = wr.at(i);
      fp[j] = i < n ? fps[at] : 0ull;
      lk[j] = i < n ? (u32)keys[at] : 0u;
    }
#pragma unroll
    for (int j = 0; j < P1; ++j) {
      if (fp[j] && !lds_merge(lfp, lkey, fp[j], lk[j])) {   // window full (rare): the record keeps its own key
        const u32 at = atomicAdd(&ovf_cnt, 1u);
        out[a.region - 1 - at] = make_ulonglong2((unsigned long long)fp[j], (unsigned long long)nkey_of(a.gid0, blockIdx.x, lk[j]));
      }
    }
  }
  __syncthreads();
  // compact the set's occupied slots to the front of the region
  constexpr int PER = LDS_FP_SLOTS / BS;
  u32 mine = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) mine += lfp[threadIdx.x * PER + j] ? 1u : 0u;
  u32 total = 0;
  u32 o = block_excl_scan(mine, wave_tot, &total);
#pragma unroll
  for (int j = 0; j < PER; ++j) {
    const int sl = threadIdx.x * PER + j;
    const u64 fp = lfp[sl];
    if (fp) out[o++] = make_ulonglong2((unsigned long long)fp, (unsigned long long)nkey_of(a.gid0, blockIdx.x, lkey[sl]));
  }
  const u32 nov = ovf_cnt;   // (read after the scan's barriers)
  __syncthreads();
  // move the overflow records (end of the region) behind the set's
  for (u32 q = threadIdx.x; q < nov; q += BS) out[total + q] = out[a.region - 1 - q];
  if (threadIdx.x == 0) a.ucnt[blockIdx.x] = total + nov;
}

// Seen-set insertion, part 2 (HBM random access): workgroup b probes the seen-set once per
// distinct fingerprint of region b, DEDUP_PER probes in flight per thread (insert-if-absent by CAS
// of the fp, then atomicMax of ~key: the entry keeps the minimum key), and appends the inserted
// entries' positions (one global atomic per workgroup and round).  COUNT: also count the probes
// (ctr[K_PROBES]; RAFTMC_COUNT_PROBES, a run of its own: timed runs leave the atomic out)
template <bool COUNT>
__global__ void __launch_bounds__(BS) orig_probe(DedupArgs a) {
  __shared__ u32 wave_tot[BS / 64];
  __shared__ unsigned long long base_sh;
  const u32 n = a.ucnt[blockIdx.x];
  const ulonglong2* in = a.urec + (u64)blockIdx.x * a.region;
  u32 err = 0;
  const u64 t0 = a.prof ? wall_clock64() : 0;
  if (COUNT && threadIdx.x == 0 && n) atomicAdd(&a.ctr[K_PROBES], (unsigned long long)n);
#pragma unroll 1
  for (u32 i0 = 0; i0 < n; i0 += DEDUP_PER * BS) {
    u64 fp[DEDUP_PER], nk[DEDUP_PER], pos[DEDUP_PER];
#pragma unroll
    for (int j = 0; j < DEDUP_PER; ++j) {
      const u32 i = i0 + (u32)j * BS + threadIdx.x;
      const ulonglong2 r = i < n ? in[i] : make_ulonglong2(0ull, 0ull);
      fp[j] = r.x; nk[j] = r.y;
    }
    const u32 ins = probe_batch<DEDUP_PER>(a.table, a.table_mask, fp, nk, pos, err);
    u32 total = 0;
    const u32 off = block_excl_scan((u32)__popc(ins), wave_tot, &total);
    if (threadIdx.x == 0) base_sh = total ? atomicAdd(&a.ctr[K_INS], (unsigned long long)total) : 0ull;
    __syncthreads();
    u64 o = base_sh + off;
#pragma unroll
    for (int j = 0; j < DEDUP_PER; ++j)
      if ((ins >> j) & 1u) a.newpos[o++] = pos[j];
    __syncthreads();   // base_sh reused
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
  if (a.prof && threadIdx.x == 0) {
    const u64 t3 = wall_clock64();
    atomicAdd(&a.ctr[K_PROF + 1], (unsigned long long)(t3 - t0));
    atomicAdd(&a.ctr[K_PROF + 3], 1ull);
  }
}

// ------------------------------------------------------------------ TLC -workers N semantics
// The order-independent pipeline (mc_opts.workers != 1): every count TLC prints without -coverage
// is the same, but which producer of a state is kept is not TLC's single-worker choice (as with
// TLC's own workers).  8-B seen-set entries, first-come LDS filter, no keys, no winner pass: the
// inserting thread numbers its new state directly.

// Fused variant for TLC -workers N (what the pipeline runs): records through a first-come LDS
// filter (lds_first: an LDS CAS claims each empty slot, 16 KB; a full window lets a record through to the
// seen-set, never drop a state), the survivors probe the 8-B seen-set DEDUP_PER at a time, and
// the new states' producers go out parent-major (an LDS winner mask per parent).  COUNT: also count the
// fingerprints that reach the seen-set (ctr[K_PROBES], one atomic per workgroup) -- a separate
// instantiation, because even one extra same-address atomic per wave costs ~3 ms of C2's
// 11 ms here (round 4, measured), so timed runs leave it off (RAFTMC_COUNT_PROBES).
template <int WW, bool COUNT>
__global__ void __launch_bounds__(BS) orig_dedup_plain(DedupArgs a) {
  __shared__ unsigned long long lfp[LDS_FP_SLOTS];
  __shared__ u32 wave_tot[BS / 64];
  __shared__ unsigned long long base_sh;
  __shared__ unsigned long long win[BS * WW];
  for (int t = threadIdx.x; t < LDS_FP_SLOTS; t += BS) lfp[t] = 0ull;
  for (int t = threadIdx.x; t < BS * WW; t += BS) win[t] = 0ull;
  __syncthreads();
  const WaveRegions wr(a.rcnt + 4 * blockIdx.x, a.region / 4);
  const u32 n = wr.n;
  const u64* fps = a.rfp + (u64)blockIdx.x * a.region;
  const unsigned short* keys = a.rkey + (u64)blockIdx.x * a.region;
  u32 err = 0;
  u32 probes = 0;   // this lane's (summed over the wave at the end)
#pragma unroll 1
  for (u32 i0 = 0; i0 < n; i0 += DEDUP_PER * BS) {
    u64 fp[DEDUP_PER], key[DEDUP_PER], pos[DEDUP_PER];
#pragma unroll
    for (int j = 0; j < DEDUP_PER; ++j) {
      const u32 i = i0 + (u32)j * BS + threadIdx.x;
      const u64 at = wr.at(i);
      fp[j] = i < n ? fps[at] : 0ull;
      key[j] = i < n ? (u64)keys[at] : 0ull;     // local key lane << 8 | instance
    }
#pragma unroll
    for (int j = 0; j < DEDUP_PER; ++j)
      if (fp[j] && !lds_first(lfp, fp[j])) fp[j] = 0ull;   // produced by this workgroup's parents before
    if constexpr (COUNT) {
#pragma unroll
      for (int j = 0; j < DEDUP_PER; ++j) probes += fp[j] ? 1u : 0u;
    }
    const u32 ins = probe_batch<DEDUP_PER, false, 1>(a.table, a.table_mask, fp, key, pos, err);
#pragma unroll
    for (int j = 0; j < DEDUP_PER; ++j)
      if ((ins >> j) & 1u) atomicOr(&win[(key[j] >> 8) * WW + ((key[j] & 255) >> 6)], 1ull << (key[j] & 63));
  }
  __shared__ u32 wave_probes[BS / 64];
  if constexpr (COUNT) {
    u32 wp = probes;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) wp += __shfl_xor(wp, d);
    if (__lane_id() == 0) wave_probes[threadIdx.x >> 6] = wp;
  }
  __syncthreads();
  if constexpr (COUNT) {
    if (threadIdx.x == 0) {
      u32 t = 0;
#pragma unroll
      for (int w = 0; w < BS / 64; ++w) t += wave_probes[w];
      if (t) atomicAdd(&a.ctr[K_PROBES], (unsigned long long)t);
    }
  }
  u64 wm[WW];
  u32 mine = 0;
#pragma unroll
  for (int q = 0; q < WW; ++q) { wm[q] = win[threadIdx.x * WW + q]; mine += (u32)__popcll(wm[q]); }
  u32 total = 0;
  const u32 off = block_excl_scan(mine, wave_tot, &total);
  if (threadIdx.x == 0) base_sh = total ? atomicAdd(&a.ctr[K_CHUNK_NEW], (unsigned long long)total) : 0ull;
  __syncthreads();
  u64 o = base_sh + off;
  const u64 pg = a.gid0 + (u64)blockIdx.x * BS + threadIdx.x;
#pragma unroll
  for (int q = 0; q < WW; ++q) {
    u64 m = wm[q];
    while (m) {
      const int k = q * 64 + __ffsll((unsigned long long)m) - 1;
      m &= m - 1;
      a.newpos[o++] = (pg << 8) | (u64)k;
    }
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
}

struct MatPlainArgs {
  u32* states;
  u64* meta;
  const u64* newrec;           // (parent gid << 8 | instance), ctr[K_CHUNK_NEW] of them
  u64 base;                    // global id of device slot 0
  u64 dst_base, cap;           // new state i of the chunk goes to dst_base + ctr[K_LEVEL_NEW] + i (device index)
  OrigRuntime rt;
  unsigned long long* ctr;
  u32 store;                   // 0: the last level of a depth-bounded search (count_final_level):
                               // counted and invariant-checked, not written
};

// grid-stride over the chunk's new states (their count stays on the device: no host wait)
template <class S>
__global__ void __launch_bounds__(BS) orig_materialize_plain(MatPlainArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  __shared__ unsigned int lds_cnt[OA_NACT];
  for (int t = threadIdx.x; t < OA_NACT; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 n_new = a.ctr[K_CHUNK_NEW];
  const u64 base = a.dst_base + a.ctr[K_LEVEL_NEW];
  u32 err = 0;
  unsigned long long ev = ~0ull;
  for (u64 i = (u64)blockIdx.x * BS + threadIdx.x; i < n_new; i += (u64)gridDim.x * BS) {
    const u64 rec = a.newrec[i], pgid = rec >> 8;
    const int k = (int)(rec & 0xff);
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(a.states + (pgid - a.base) * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    W s, t;
    u64 al[S::AW];
    S::unpack(w, s);
    S::all_logs_next(s, al);
    u32 e2 = 0;
    const int act = S::apply(s, k, t, e2);
#pragma unroll
    for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
    u32 pw[NW];
    S::pack(t, pw);
    const u64 dst = base + i;
    if (act >= 0 && (!a.store || dst < a.cap)) {
      if (a.store) {
        uint4* o = reinterpret_cast<uint4*>(a.states + dst * NWP);
#pragma unroll
        for (int q = 0; q < NWP / 4; ++q)
          o[q] = make_uint4(pw[4 * q], 4 * q + 1 < NW ? pw[4 * q + 1] : 0u, 4 * q + 2 < NW ? pw[4 * q + 2] : 0u, 4 * q + 3 < NW ? pw[4 * q + 3] : 0u);
        a.meta[dst] = (pgid << 24) | ((u64)act << 16) | (u64)k;
      }
      atomicAdd(&lds_cnt[act], 1u);
      if (S::violated(t, a.rt.invariants & S::inv_frame(act))) { const u64 e = ev_word(pgid, (u32)k, EV_VIOLATION); ev = e < ev ? e : ev; }
    } else {
      err |= dst >= a.cap ? (u32)OE_CAP_STORE : (u32)OE_TABLE_FULL;
    }
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
  if (ev != ~0ull) atomicMin(&a.ctr[K_EVENT], ev);
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + OA_NACT + t], (unsigned long long)lds_cnt[t]);
}

// Winners: an entry inserted by this chunk holds, after the chunk's dedup, the minimum key over
// all its producers (later chunks have larger keys), i.e. TLC's first-found (parent, instance).
// orig_mark sets that (parent, instance) bit; orig_count counts each workgroup's winners.
struct MarkArgs {
  const u64* newpos;
  const u64* table;
  u64 gid0, chunk_count;
  u64* winmask;                // [chunk][WW] instance bits of each parent's winning successors
  u32 ww;
  unsigned long long* ctr;
};

__global__ void __launch_bounds__(BS) orig_mark(MarkArgs a) {
  const u64 n = a.ctr[K_INS];
  for (u64 i = (u64)blockIdx.x * BS + threadIdx.x; i < n; i += (u64)gridDim.x * BS) {
    const u64 key = ~a.table[2 * a.newpos[i] + 1];
    const u64 p = (key >> 8) - a.gid0;
    const u32 k = (u32)(key & 255);
    if (p >= a.chunk_count) { atomicOr(&a.ctr[K_ERR], (unsigned long long)OE_TABLE_FULL); continue; }   // cannot happen
    atomicOr((unsigned long long*)&a.winmask[p * a.ww + (k >> 6)], 1ull << (k & 63));
  }
}

// winners per workgroup of 256 parents (popcount of their masks; coalesced, no atomics)
template <int WW>
__global__ void __launch_bounds__(BS) orig_count(const u64* winmask, u64 chunk_count, u32* wcnt) {
  __shared__ u32 wave_tot[BS / 64];
  const u64 p = (u64)blockIdx.x * BS + threadIdx.x;
  u32 mine = 0;
#pragma unroll
  for (int q = 0; q < WW; ++q) mine += p < chunk_count ? (u32)__popcll(winmask[p * WW + q]) : 0u;
  u32 total = 0;
  (void)block_excl_scan(mine, wave_tot, &total);
  if (threadIdx.x == 0) wcnt[blockIdx.x] = total;
}

// exclusive scan of the per-workgroup winner counts -> woff; the chunk's total -> ctr[K_CHUNK_NEW]
__global__ void __launch_bounds__(SCAN_BS) orig_scan(const u32* wcnt, u64* woff, u32 nblk, unsigned long long* ctr) {
  __shared__ unsigned long long part[SCAN_BS];
  const u32 per = (nblk + SCAN_BS - 1) / SCAN_BS, b0 = threadIdx.x * per;
  unsigned long long s = 0;
  for (u32 j = 0; j < per; ++j) if (b0 + j < nblk) s += wcnt[b0 + j];
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < SCAN_BS; d <<= 1) {
    const unsigned long long x = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0ull;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  unsigned long long run = part[threadIdx.x] - s;
  for (u32 j = 0; j < per; ++j) if (b0 + j < nblk) { woff[b0 + j] = run; run += wcnt[b0 + j]; }
  if (threadIdx.x == SCAN_BS - 1) ctr[K_CHUNK_NEW] = part[SCAN_BS - 1];
}

struct MatArgs {
  u32* states;
  u64* meta;
  u64 chunk_begin, chunk_count, gid0;   // parents: device index, count, global id of the first
  u64* winmask;                // read and re-zeroed
  const u64* woff;
  u32 ww;
  u64 dst_base, cap;           // new state i of the chunk goes to dst_base + ctr[K_LEVEL_NEW] + i (device index)
  OrigRuntime rt;
  unsigned long long* ctr;
};

// Workgroup per 256 parents (the generate workgroup's): the winners in key order — parent
// order, then instance order — are numbered by a workgroup scan plus the chunk offset, staged
// in LDS and spread over the workgroup's lanes; each is re-derived from (parent, instance) and
// stored at its FIFO position with its parent pointer; invariants of the new state.
template <class S>
__global__ void __launch_bounds__(BS) orig_materialize(MatArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3, WW = (S::NI + 63) / 64;
  __shared__ unsigned int lds_cnt[OA_NACT];
  __shared__ unsigned short items[MAT_CAP];
  __shared__ u32 wave_tot[BS / 64];
  for (int t = threadIdx.x; t < OA_NACT; t += BS) lds_cnt[t] = 0;
  const u64 p = (u64)blockIdx.x * BS + threadIdx.x;
  u64 wm[WW];
  u32 mine = 0;
#pragma unroll
  for (int q = 0; q < WW; ++q) {
    wm[q] = p < a.chunk_count ? a.winmask[p * WW + q] : 0ull;
    mine += (u32)__popcll(wm[q]);
  }
  if (p < a.chunk_count && mine) {
#pragma unroll
    for (int q = 0; q < WW; ++q) a.winmask[p * WW + q] = 0ull;   // ready for the next chunk
  }
  u32 total = 0;
  const u32 off = block_excl_scan(mine, wave_tot, &total);   // (also orders lds_cnt's clearing)
  const u64 base = a.dst_base + a.ctr[K_LEVEL_NEW] + a.woff[blockIdx.x];
  u32 err = 0;
  unsigned long long ev = ~0ull;
  for (u32 r0 = 0; r0 < total; r0 += MAT_CAP) {
    {   // stage this round's window [r0, r0 + MAT_CAP) of the workgroup's winners
      u32 idx = off;
#pragma unroll
      for (int q = 0; q < WW; ++q) {
        u64 m = wm[q];
        while (m) {
          const int k = q * 64 + __ffsll((unsigned long long)m) - 1;
          m &= m - 1;
          if (idx >= r0 && idx < r0 + MAT_CAP) items[idx - r0] = (unsigned short)((threadIdx.x << 8) | (unsigned)k);
          ++idx;
        }
      }
    }
    __syncthreads();
    const u32 nr = total - r0 < (u32)MAT_CAP ? total - r0 : (u32)MAT_CAP;
    for (u32 i = threadIdx.x; i < nr; i += BS) {
      const u32 x = items[i];
      const u64 par = (u64)blockIdx.x * BS + (x >> 8);
      const int k = (int)(x & 255);
      u32 w[NWP];
      const uint4* src = reinterpret_cast<const uint4*>(a.states + (a.chunk_begin + par) * NWP);
#pragma unroll
      for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
      W s, t;
      u64 al[S::AW];
      S::unpack(w, s);
      S::all_logs_next(s, al);
      u32 e2 = 0;
      const int act = S::apply(s, k, t, e2);
#pragma unroll
      for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
      u32 pw[NW];
      S::pack(t, pw);
      const u64 dst = base + r0 + i;
      if (act >= 0 && dst < a.cap) {
        uint4* o = reinterpret_cast<uint4*>(a.states + dst * NWP);
#pragma unroll
        for (int q = 0; q < NWP / 4; ++q)
          o[q] = make_uint4(pw[4 * q], 4 * q + 1 < NW ? pw[4 * q + 1] : 0u, 4 * q + 2 < NW ? pw[4 * q + 2] : 0u, 4 * q + 3 < NW ? pw[4 * q + 3] : 0u);
        const u64 pgid = a.gid0 + par;
        a.meta[dst] = (pgid << 24) | ((u64)act << 16) | (u64)k;
        atomicAdd(&lds_cnt[act], 1u);
        if (S::violated(t, a.rt.invariants & S::inv_frame(act))) {
          const u64 e = ev_word(pgid, (u32)k, EV_VIOLATION);
          ev = e < ev ? e : ev;
        }
      } else {
        err |= dst >= a.cap ? (u32)OE_CAP_STORE : (u32)OE_TABLE_FULL;   // a winner always re-derives
      }
    }
    __syncthreads();
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
  if (ev != ~0ull) atomicMin(&a.ctr[K_EVENT], ev);
  __syncthreads();
  for (int t = threadIdx.x; t < OA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[K_ACT + OA_NACT + t], (unsigned long long)lds_cnt[t]);
}

// after a chunk's materialize: fold its new-state count into the level's; re-arm the chunk's
// insert counter (the level's first chunk starts from the per-level counter reset)
// (Vector atomics only: with plain accesses the compiler reads the counters with a scalar load
// and may issue the vector store that zeroes K_CHUNK_NEW before that load has returned — on the
// GPU the load then sometimes sees the zero and the chunk's new states are lost.  Found when a
// fourth counter store moved the scalar wait behind the stores.)
__global__ void orig_advance(unsigned long long* ctr) {
  if (threadIdx.x == 0) {
    const unsigned long long n = atomicExch(&ctr[K_CHUNK_NEW], 0ull);
    atomicAdd(&ctr[K_LEVEL_NEW], n);
    atomicExch(&ctr[K_INS], 0ull);
    atomicExch(&ctr[K_LEAD], 0ull);
  }
}

// the level's counters back to their initial values (event word all ones); queued right after
// the level's counter readback, so it runs while the host looks at the counters and the next
// level starts with its generate kernel (one tiny kernel instead of two fills on the critical path)
__global__ void orig_reset_ctr(unsigned long long* ctr) {
  for (int t = threadIdx.x; t < K_NCTR; t += blockDim.x) ctr[t] = t == K_EVENT ? ~0ull : 0ull;
}

// ------------------------------------------------------------------ TLC's stop point
// On the level's first event (parent gid_stop, instance k_stop, kind): TLC's generated counts
// are the whole successor lists of the parents before it and of the event's parent (none when
// computing its successors raised the error), per-action generated counts stop at the event's
// successor.  out[0] = generated, out[1 + a] = per-action generated.
template <class S>
__global__ void __launch_bounds__(BS) orig_stop_generated(const u32* states, u64 first, u64 n, u64 gid0, u64 gid_stop,
                                                         u32 k_stop, u32 kind, unsigned long long* out) {
  using W = typename S::Work;
  constexpr int NWP = (S::NW + 3) & ~3;
  // counts in LDS, one global atomic per workgroup and action (a global atomic per successor on
  // 16 addresses serialises: minutes for C5v2's 93M-parent level 11)
  __shared__ unsigned int lds_cnt[1 + OA_NACT];
  for (int q = threadIdx.x; q < 1 + OA_NACT; q += BS) lds_cnt[q] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  const u64 gid = gid0 + i;
  if (i < n && !(gid == gid_stop && kind == EV_NEXT_ERROR)) {
    u32 w[NWP];
#pragma unroll
    for (int q = 0; q < NWP; ++q) w[q] = states[(first + i) * NWP + q];
    W s, t;
    S::unpack(w, s);
    u32 err = 0, tot = 0;
    for (int k = 0; k < S::NI; ++k) {
      const int act = S::apply(s, k, t, err);
      if (act < 0) continue;
      ++tot;
      if (gid < gid_stop || (u32)k <= k_stop) atomicAdd(&lds_cnt[1 + act], 1u);
    }
    if (tot) atomicAdd(&lds_cnt[0], tot);
  }
  __syncthreads();
  for (int q = threadIdx.x; q < 1 + OA_NACT; q += BS)
    if (lds_cnt[q]) atomicAdd(&out[q], (unsigned long long)lds_cnt[q]);
}

// per-action distinct counts of the level's first n new states (stored in key order)
__global__ void __launch_bounds__(BS) orig_stop_distinct(const u64* meta, u64 n, unsigned long long* out) {
  __shared__ unsigned int lds_cnt[OA_NACT];
  for (int q = threadIdx.x; q < OA_NACT; q += BS) lds_cnt[q] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i < n) atomicAdd(&lds_cnt[((meta[i] >> 16) & 0xff) % OA_NACT], 1u);
  __syncthreads();
  for (int q = threadIdx.x; q < OA_NACT; q += BS)
    if (lds_cnt[q]) atomicAdd(&out[q], (unsigned long long)lds_cnt[q]);
}

// ------------------------------------------------------------------ sharded (multi-GPU) kernels
// owner of a fingerprint: high half mod world (the seen-set index uses the low bits)
__device__ __host__ __forceinline__ u32 fp_owner(u64 fp, u32 world) { return (u32)((fp >> 32) % world); }

struct RouteArgs {
  const u64* rfp;
  const unsigned short* rkey;
  const u32* rcnt;
  u64 region;                  // records per workgroup region (BS * NI)
  u64* route;                  // [world][route_cap][2] (fp, slot)
  u64 route_cap;
  u32 world;
  unsigned long long* rcnt_out;   // [world]
};

// Sharded route over the compacted records: workgroup b takes generate-workgroup b's records,
// drops the successors its 256 parents produce more than once (the first-come LDS filter), and
// buckets the rest by owner, 16 records per thread at a time: LDS histogram, one global atomic
// per (workgroup, round, owner).  Records are (fp, state in chunk << 8 | instance).
// (its filter keeps 4096 slots: the route kernel's 16 records per thread make it VGPR-bound, so the
// larger set costs no occupancy here and saves the stores it filters: 7.1 vs 8.0 ms per C2 run at world 1)
constexpr int ROUTE_FP_SLOTS = 4096;
__global__ void __launch_bounds__(BS) orig_route_blk(RouteArgs a) {
  __shared__ unsigned long long lds_fp[ROUTE_FP_SLOTS];
  __shared__ unsigned int hist[8];
  __shared__ unsigned long long base[8];
  for (int t = threadIdx.x; t < ROUTE_FP_SLOTS; t += BS) lds_fp[t] = 0ull;
  const WaveRegions wr(a.rcnt + 4 * blockIdx.x, a.region / 4);
  const u32 n = wr.n;
  const u64* fps = a.rfp + (u64)blockIdx.x * a.region;
  const unsigned short* keys = a.rkey + (u64)blockIdx.x * a.region;
  constexpr int G = 16;
#pragma unroll 1
  for (u32 i0 = 0; i0 < n; i0 += G * BS) {
    if (threadIdx.x < 8) hist[threadIdx.x] = 0;
    __syncthreads();   // also orders the set's clearing before its first use
    u64 fp[G], slot[G];
    unsigned int off[G];
    int own[G];
#pragma unroll
    for (int j = 0; j < G; ++j) {
      const u32 i = i0 + (u32)j * BS + threadIdx.x;
      const u64 at = wr.at(i);
      fp[j] = i < n ? fps[at] : 0ull;
      const u32 lk = i < n ? keys[at] : 0u;
      slot[j] = (((u64)blockIdx.x * BS + (lk >> 8)) << 8) | (u64)(lk & 255u);
      // produced before by this workgroup's parents?  The first-come filter of orig_dedup_plain
      // (lds_first: a full probe window only lets a duplicate through to its owner's seen-set)
      if (fp[j] && !lds_first<ROUTE_FP_SLOTS>(lds_fp, fp[j])) fp[j] = 0;
      own[j] = fp[j] ? (int)fp_owner(fp[j], a.world) : -1;
      off[j] = own[j] >= 0 ? atomicAdd(&hist[own[j]], 1u) : 0u;
    }
    __syncthreads();
    if (threadIdx.x < a.world) base[threadIdx.x] = hist[threadIdx.x] ? atomicAdd(&a.rcnt_out[threadIdx.x], (unsigned long long)hist[threadIdx.x]) : 0ull;
    __syncthreads();
#pragma unroll
    for (int j = 0; j < G; ++j) {
      if (own[j] < 0) continue;
      // one 16-B store per record
      *reinterpret_cast<ulonglong2*>(a.route + ((u64)own[j] * a.route_cap + base[own[j]] + off[j]) * 2) =
          make_ulonglong2((unsigned long long)fp[j], (unsigned long long)slot[j]);
    }
    __syncthreads();   // hist / base reused by the next round
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

// owner-side insertion of one source rank's records into the seen-set as 8-B entries {fp} (no FIFO
// keys in sharded raft_original: twice the entries of the keyed table in the same bytes)
__global__ void __launch_bounds__(BS) orig_dedup_sh(DedupShArgs a) {
  __shared__ u32 wave_tot[BS / 64];
  __shared__ unsigned long long base_sh;
  const u64 tile = (u64)blockIdx.x * (BS * DEDUP_PER);
  u64 fp[DEDUP_PER], nk[DEDUP_PER], pos[DEDUP_PER];
#pragma unroll
  for (int j = 0; j < DEDUP_PER; ++j) {
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    fp[j] = idx < a.n ? a.recv[2 * idx] : 0ull;
    nk[j] = 0ull;
  }
  u32 err = 0;
  const u32 isnew = probe_batch<DEDUP_PER, false, 1>(a.table, a.table_mask, fp, nk, pos, err);
  u32 total = 0;
  const u32 off = block_excl_scan((u32)__popc(isnew), wave_tot, &total);
  if (threadIdx.x == 0) base_sh = total ? atomicAdd(a.counter, (unsigned long long)total) : 0ull;
  __syncthreads();
  u64 o = base_sh + off;
  for (int j = 0; j < DEDUP_PER; ++j) {
    if (!((isnew >> j) & 1u)) continue;
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    a.reply[o++] = a.recv[2 * idx + 1];
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
  // the generator's own segment (it owns these states): straight into its store at st_dst
  // instead of a STATES record, when st_states is set
  u32* st_states;
  u64* st_meta;
  u64 st_dst, st_cap;
  u32 store;                   // 0: the last level of a depth-bounded search (count_final_level):
                               // counted and invariant-checked, neither stored nor shipped
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
  unsigned long long ev = ~0ull;
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
    u32 e2 = 0;
    const int act = S::apply(s, (int)k, t, e2);
#pragma unroll
    for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
    u32 pw[NW];
    S::pack(t, pw);
    const u64 fp = fp64(pw, a.seed);
    const u64 meta = ((a.rank_bits | gid) << 24) | ((u64)(act < 0 ? 0 : act) << 16) | k;
    if (!a.store) {
      // counted only (count_final_level)
    } else if (a.st_states) {
      const u64 dst = a.st_dst + i;
      if (dst < a.st_cap) {
        uint4* o = reinterpret_cast<uint4*>(a.st_states + dst * NWP);
#pragma unroll
        for (int q = 0; q < NWP / 4; ++q)
          o[q] = make_uint4(pw[4 * q], 4 * q + 1 < NW ? pw[4 * q + 1] : 0u, 4 * q + 2 < NW ? pw[4 * q + 2] : 0u, 4 * q + 3 < NW ? pw[4 * q + 3] : 0u);
        a.st_meta[dst] = meta;
      } else {
        err |= OE_CAP_STORE;
      }
    } else {
      u32* o = a.out + i * RW;
#pragma unroll
      for (int q = 0; q < NWP / 4; ++q)
        reinterpret_cast<uint4*>(o)[q] = make_uint4(pw[4 * q], 4 * q + 1 < NW ? pw[4 * q + 1] : 0u, 4 * q + 2 < NW ? pw[4 * q + 2] : 0u, 4 * q + 3 < NW ? pw[4 * q + 3] : 0u);
      reinterpret_cast<uint4*>(o)[NWP / 4] = make_uint4((u32)meta, (u32)(meta >> 32), (u32)fp, (u32)(fp >> 32));
    }
    if (act >= 0) {
      atomicAdd(&lds_cnt[act], 1u);
      if (S::violated(t, a.rt.invariants & S::inv_frame(act))) ev = ev_word(gid, (u32)k, EV_VIOLATION);
    } else {
      err |= OE_TABLE_FULL;   // an acknowledged slot always re-derives
    }
  }
  if (err) atomicOr(&a.ctr[K_ERR], (unsigned long long)err);
  if (ev != ~0ull) atomicMin(&a.ctr[K_EVENT], ev);
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
template <class S, int STRIDE>
__global__ void __launch_bounds__(BS) orig_reinsert(const u32* states, u64 n, u64* table, u64 mask, u64 seed,
                                                    unsigned long long* ctr) {
  constexpr int NW = S::NW, NWP = (S::NW + 3) & ~3;
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  u32 w[NW];
#pragma unroll
  for (int q = 0; q < NW; ++q) w[q] = states[i * NWP + q];
  // stored states are older than any successor the search will generate: key 0 (~key = ~0)
  const u64 fp[1] = {fp64(w, seed)}, nk[1] = {~0ull};
  u64 pos[1];
  u32 err = 0;
  probe_batch<1, STRIDE == 2, STRIDE>(table, mask, fp, nk, pos, err);
  if (err) atomicOr(&ctr[K_ERR], (unsigned long long)err);
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
    return last_fifo_ ? fpgap::observed(d_table_, table_mask_ + 1, 2, stream_, v, err)
                      : fpgap::observed(d_table_, 2 * (table_mask_ + 1), 1, stream_, v, err);
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
    uint64_t slots = 1; while (slots * 2 * 16 <= tb) slots *= 2;   // 16-B entries {fp, ~key}
    if (slots < 1024) slots = 1024;
    uint64_t sb = o.state_store_bytes ? o.state_store_bytes : std::min<uint64_t>(32ull << 30, freeb / 3);
    cap_ = sb / (NWP * 4 + 8);
    if (cap_ < 16) cap_ = 16;
    // frontier chunk: the record regions hold chunk_states * NI records (10 B each), their
    // distinct pairs (16 B) and the inserted-position list as many 8-B entries (worst case: every
    // record new), sharded mode also world route regions of 16-B records: ~1/4 of the store
    chunk_states_ = std::max<u64>(4096, std::min<u64>(cap_, (sb / 4) / ((34 + 16 * (u64)world) * (u64)S::NI)));
    chunk_states_ = std::min<u64>(chunk_states_, (u64)SCAN_BS * 64 * BS);   // orig_scan: <= 64 blocks per lane
    chunk_states_ = (chunk_states_ / BS) * BS;   // whole workgroups: records are grouped per generate workgroup
    const u64 nblk = chunk_states_ / BS, nrec = chunk_states_ * (u64)S::NI;
    table_mask_ = slots - 1;
    HIPCHK(hipMalloc(&d_table_, slots * 16));
    HIPCHK(hipMalloc(&d_states_, cap_ * NWP * 4));
    HIPCHK(hipMalloc(&d_meta_, cap_ * 8));
    HIPCHK(hipMalloc(&d_rfp_, nrec * 8));
    HIPCHK(hipMalloc(&d_rkey_, nrec * 2));
    HIPCHK(hipMalloc(&d_rcnt_blk_, nblk * 16));
    HIPCHK(hipMalloc(&d_newrec_, nrec * 8));          // inserted entry positions (single GPU) / replies (sharded)
    HIPCHK(hipMalloc(&d_urec_, nrec * 16));           // distinct (fp, ~key) per workgroup region
    HIPCHK(hipMalloc(&d_ucnt_, nblk * 4));
    HIPCHK(hipMalloc(&d_winmask_, chunk_states_ * WW * 8));
    HIPCHK(hipMalloc(&d_wcnt_, nblk * 4));
    HIPCHK(hipMalloc(&d_woff_, nblk * 8));
    HIPCHK(hipMalloc(&d_lead_, chunk_states_ * 4));
    HIPCHK(hipMalloc(&d_ctr_, K_NCTR * 8));
    HIPCHK(hipHostMalloc((void**)&h_ctr_, K_NCTR * 8, hipHostMallocDefault));
    HIPCHK(hipMalloc(&d_stop_, (1 + OA_NACT) * 8));
    HIPCHK(hipMemset(d_winmask_, 0, chunk_states_ * WW * 8));
    if (world >= 1) {   // sharded mode
      HIPCHK(hipMalloc(&d_route_, (u64)world * nrec * 16));
      HIPCHK(hipMalloc(&d_rcnt_, 2 * 8 * 8));
    }
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (auto& e : ev_) HIPCHK(hipEventCreate(&e));
    dev_ = o.device; req_table_ = o.fp_table_bytes; req_store_ = o.state_store_bytes; alloc_world_ = world;
    return 0;
  }

  // event pairs (generate, dedup, winners = mark + scan, materialize) of chunk q of the current
  // level: lvl_ev_[8q .. 8q+8)
  int lvl_events(int q) {
    while ((int)lvl_ev_.size() < 8 * (q + 1)) {
      hipEvent_t e;
      if (hipEventCreate(&e) != hipSuccess) return MC_E_NO_DEVICE;
      lvl_ev_.push_back(e);
    }
    return 0;
  }

  GenArgs gen_args(u64 dev_begin, u64 count, u64 gid0, u64 seed, const RunOpts& o) const {
    GenArgs g;
    g.states = d_states_; g.chunk_begin = dev_begin; g.chunk_count = count; g.gid0 = gid0;
    g.rfp = d_rfp_; g.rkey = d_rkey_; g.rcnt = d_rcnt_blk_; g.seed = seed; g.rt = m_.rt;
    g.inv_oom = o.inv_out_of_model ? 1u : 0u; g.deadlock = o.check_deadlock ? 1u : 0u;
    g.ctr = (unsigned long long*)d_ctr_;
    g.lead = d_lead_;
    return g;
  }

  // the successor pass of one chunk: orig_generate over every parent, then orig_generate_lead over
  // the parents with leader work (its grid strides over the count the first kernel left on the
  // device); K_LEAD must be zero before (level start: orig_reset_ctr, later chunks: orig_advance)
  void launch_generate(const GenArgs& g, unsigned nblk) {
    hipLaunchKernelGGL((orig_generate<S>), dim3(nblk), dim3(BS), 0, stream_, g);
    const unsigned lblk = std::min<unsigned>(nblk, std::max<unsigned>(64u, nblk / 8));
    hipLaunchKernelGGL((orig_generate_lead<S>), dim3(lblk), dim3(BS), 0, stream_, g);
  }

  RouteArgs route_args(u32 world) const {
    RouteArgs ra;
    ra.rfp = d_rfp_; ra.rkey = d_rkey_; ra.rcnt = d_rcnt_blk_; ra.region = (u64)BS * S::NI; ra.route = d_route_;
    ra.route_cap = chunk_states_ * S::NI; ra.world = world; ra.rcnt_out = (unsigned long long*)d_rcnt_;
    return ra;
  }

  int run(const RunOpts& o, RunResult& r, std::string& err) override {
    unstored_ = 0;   // a previous run's unstored level must not outlive it (mc_dump_states)
    if (int rc = ensure_alloc(o, 0, err)) return rc;   // world 0 = single-GPU pipeline
    auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipMemsetAsync(d_table_, 0, (table_mask_ + 1) * 16, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    // TLC -workers 1: single-worker FIFO order (16-B {fp, ~key} entries); -workers N: 8-B entries
    const bool fifo = o.workers == 1;
    last_fifo_ = fifo;
    // RAFTMC_COUNT_PROBES: count the seen-set probes of the -workers N pipeline (an instrumented
    // kernel; read per run, so a caller can count in a run of its own outside a timed region)
    const bool count_probes = std::getenv("RAFTMC_COUNT_PROBES") != nullptr;
    const u64 tmask = fifo ? table_mask_ : 2 * (table_mask_ + 1) - 1;
    ctr_clean_ = false;

    r = RunResult();
    r.seed = o.seed ? o.seed : 0x5EED5EED2024ull;
    r.state_bytes = NWP * 4;
    for (int k = 0; k < OA_NACT; ++k) r.action_names.push_back(kOrigActNames[k]);
    r.act_generated.assign(OA_NACT, 0); r.act_distinct.assign(OA_NACT, 0);
    r.kernels = {{"orig_generate", 0, 0, 0}, {"orig_merge_probe", 0, 0, 0}, {"orig_mark_scan", 0, 0, 0}, {"orig_materialize", 0, 0, 0}};
    base_ = 0; host_.clear();

    W s0; S::init(s0);
    const u64 S_B = NWP * 4;
    u64 level_begin = 0, level_count = 1;
    if (!o.recover_path.empty()) {   // TLC -recover: continue the BFS saved by a checkpoint
      if (int rc = load_checkpoint(o.recover_path, fifo, r, level_begin, level_count, err)) return rc;
    } else {
    // ---- Init (raft_original.tla:139-159): one state, generated and distinct
    u32 w0[S::NW]; S::pack(s0, w0);
    u32 wp[NWP] = {0}; for (int q = 0; q < S::NW; ++q) wp[q] = w0[q];
    const u64 fp0 = fp64(w0, r.seed);
    const u64 e0[2] = {fp0, ~0ull};   // key 0
    if (fifo) HIPCHK(hipMemcpy(d_table_ + 2 * (fp0 & tmask), e0, 16, hipMemcpyHostToDevice));
    else HIPCHK(hipMemcpy(d_table_ + (fp0 & tmask), e0, 8, hipMemcpyHostToDevice));
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

    // count_final_level: the level at depth max_depth is never expanded, so the -workers N search
    // counts and checks its states without storing them (an event re-runs FIFO, which stores all)
    const bool count_last = o.count_final_level && !fifo && o.max_depth > 0 && o.checkpoint_path.empty();
    unstored_ = 0;
    while (level_count > 0) {
      if (o.max_depth && r.depth >= o.max_depth) { r.left_on_queue = (int64_t)level_count; r.verdict = MC_VERDICT_DEPTH_LIMIT; break; }
      const bool last = count_last && r.depth + 1 >= o.max_depth;
      // the device keeps what the search still reads (the frontier) and writes (the next
      // level); when the next level, predicted from the last growth ratio with a 1.5x margin,
      // might not fit behind what is stored, the completed levels move to host memory
      if (level_begin > base_ && !last) {
        const double prev = r.levels.size() >= 2 ? (double)r.levels[r.levels.size() - 2].states : 1.0;
        const double pred = (double)level_count * std::max(1.0, (double)level_count / std::max(prev, 1.0)) * 1.5;
        if ((double)(total_ - base_) + pred > (double)cap_) {
          if (progress_) std::fprintf(stderr, "spilling %llu completed states to host memory\n", (unsigned long long)(level_begin - base_));
          if (int rc = spill(level_begin, level_count, err)) return rc;
        }
      }
      if (!ctr_clean_) {
        hipLaunchKernelGGL(orig_reset_ctr, dim3(1), dim3(64), 0, stream_, (unsigned long long*)d_ctr_);
        HIPCHK(hipGetLastError());
      }
      ctr_clean_ = false;
      const u64 level_end = level_begin + level_count;
      // every chunk's kernels are queued without waiting: the chunk's insert and winner counts
      // stay on the device (grid-stride / scanned offsets), so the host synchronises once per
      // level, for the counters
      int nch = 0;
      for (u64 cb = level_begin; cb < level_end; cb += chunk_states_, ++nch) {
        const u64 cnt = std::min<u64>(chunk_states_, level_end - cb);
        const unsigned nblk = (unsigned)((cnt + BS - 1) / BS);
        if (int rc = lvl_events(nch)) { err = "hipEventCreate failed"; return rc; }
        hipEvent_t* e = &lvl_ev_[8 * nch];
        // kernels index the device store (global id - base_); keys and parent pointers are global
        const GenArgs g = gen_args(cb - base_, cnt, cb, r.seed, o);
        HIPCHK(hipEventRecord(e[0], stream_));
        launch_generate(g, nblk);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e[1], stream_));
        DedupArgs d;
        d.rfp = d_rfp_; d.rkey = d_rkey_; d.rcnt = d_rcnt_blk_; d.region = (u64)BS * S::NI; d.gid0 = cb;
        d.urec = (ulonglong2*)d_urec_; d.ucnt = d_ucnt_;
        d.table = d_table_; d.table_mask = tmask; d.newpos = d_newrec_; d.ctr = (unsigned long long*)d_ctr_;
        d.prof = prof_ ? 1u : 0u;
        // kernel boundaries share an event (each event record costs ~5 us of stream time)
        if (fifo) {
          hipLaunchKernelGGL(orig_merge, dim3(nblk), dim3(BS), 0, stream_, d);
          HIPCHK(hipGetLastError());
          if (count_probes) hipLaunchKernelGGL((orig_probe<true>), dim3(nblk), dim3(BS), 0, stream_, d);
          else hipLaunchKernelGGL((orig_probe<false>), dim3(nblk), dim3(BS), 0, stream_, d);
        } else {
          if (count_probes) {
            hipLaunchKernelGGL((orig_dedup_plain<WW, true>), dim3(nblk), dim3(BS), 0, stream_, d);
          } else {
            hipLaunchKernelGGL((orig_dedup_plain<WW, false>), dim3(nblk), dim3(BS), 0, stream_, d);
          }
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e[3], stream_));
        if (fifo) {
          MarkArgs mk;
          mk.newpos = d_newrec_; mk.table = d_table_; mk.gid0 = cb; mk.chunk_count = cnt; mk.winmask = d_winmask_;
          mk.ww = WW; mk.ctr = (unsigned long long*)d_ctr_;
          hipLaunchKernelGGL(orig_mark, dim3((unsigned)std::min<u64>(2048, (cnt * 2 + BS - 1) / BS)), dim3(BS), 0, stream_, mk);
          HIPCHK(hipGetLastError());
          hipLaunchKernelGGL((orig_count<WW>), dim3(nblk), dim3(BS), 0, stream_, (const u64*)d_winmask_, cnt, d_wcnt_);
          HIPCHK(hipGetLastError());
          hipLaunchKernelGGL(orig_scan, dim3(1), dim3(SCAN_BS), 0, stream_, (const u32*)d_wcnt_, d_woff_, (u32)nblk, (unsigned long long*)d_ctr_);
          HIPCHK(hipGetLastError());
        }
        if (fifo) HIPCHK(hipEventRecord(e[5], stream_));
        if (fifo) {
          MatArgs m;
          m.states = d_states_; m.meta = d_meta_; m.chunk_begin = cb - base_; m.chunk_count = cnt; m.gid0 = cb;
          m.winmask = d_winmask_; m.woff = d_woff_; m.ww = WW; m.dst_base = level_end - base_; m.cap = cap_;
          m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_;
          hipLaunchKernelGGL((orig_materialize<S>), dim3(nblk), dim3(BS), 0, stream_, m);
        } else {
          MatPlainArgs m;
          m.states = d_states_; m.meta = d_meta_; m.newrec = d_newrec_; m.base = base_; m.dst_base = level_end - base_;
          m.cap = cap_; m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_; m.store = last ? 0u : 1u;
          hipLaunchKernelGGL((orig_materialize_plain<S>), dim3((unsigned)std::min<u64>(4096, (cnt * 2 + BS - 1) / BS)), dim3(BS), 0, stream_, m);
        }
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(e[7], stream_));
        hipLaunchKernelGGL(orig_advance, dim3(1), dim3(64), 0, stream_, (unsigned long long*)d_ctr_);
        HIPCHK(hipGetLastError());
        for (size_t q = 0; q < r.kernels.size(); ++q) if (fifo || q != 2) r.kernels[q].launches += 1;
        r.kernels[0].algo_bytes += (double)cnt * S_B;        // + G_in * 10 record bytes per level below
      }
      u64* const c = h_ctr_;   // pinned: the readback is one direct copy
      HIPCHK(hipMemcpyAsync(c, d_ctr_, K_NCTR * 8, hipMemcpyDeviceToHost, stream_));
      hipLaunchKernelGGL(orig_reset_ctr, dim3(1), dim3(64), 0, stream_, (unsigned long long*)d_ctr_);
      HIPCHK(hipGetLastError());
      ctr_clean_ = true;
      HIPCHK(hipStreamSynchronize(stream_));
      double level_ms = 0;
      for (int q = 0; q < nch; ++q) {
        // event pairs per kernel: generate (e0, e1), dedup (e1, e3), mark/scan (e3, e5; FIFO only),
        // materialize (e5 or e3, e7)
        const hipEvent_t* e = &lvl_ev_[8 * q];
        const std::pair<int, int> pr[4] = {{0, 1}, {1, 3}, {3, fifo ? 5 : 3}, {fifo ? 5 : 3, 7}};
        for (int k = 0; k < 4; ++k) {
          float ms = 0;
          if (pr[k].first != pr[k].second) (void)hipEventElapsedTime(&ms, e[pr[k].first], e[pr[k].second]);
          r.kernels[k].ms += ms; level_ms += ms;
        }
      }
      const u64 nnew = c[K_LEVEL_NEW];
      const u64 next_write = level_end + nnew;
      if (progress_)   // TLC's progress line, per BFS level (RAFTMC_PROGRESS=1), on stderr
        std::fprintf(stderr, "Progress(%lld) at %.3f s: %lld states generated, %llu distinct states found, %llu states left on queue "
                             "(level kernels %.1f ms, %d chunk(s), store %llu/%llu, %llu on the host%s)\n",
                     (long long)r.depth + 1,
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count(),
                     (long long)(r.generated + (int64_t)[&] { u64 g = 0; for (int k = 0; k < OA_NACT; ++k) g += c[K_ACT + k]; return g; }()),
                     (unsigned long long)(level_end + nnew), (unsigned long long)nnew, level_ms, nch,
                     (unsigned long long)((last ? level_end : next_write) - base_), (unsigned long long)cap_, (unsigned long long)base_,
                     last ? "; the last level counted, not stored" : "");
      if (progress_ && (c[K_EVENT] != ~0ull || c[K_ERR]))
        std::fprintf(stderr, "level %lld: event word 0x%llx, error flags 0x%llx\n", (long long)r.depth + 1,
                     (unsigned long long)c[K_EVENT], (unsigned long long)c[K_ERR]);
      if (prof_) {
        for (int q = 0; q < 4; ++q) prof_acc_[q] += c[K_PROF + q];
        prof_acc_[4] = std::max<u64>(prof_acc_[4], c[K_PROF + 5]);
      }
      const u64 G_in = c[K_GEN_IN];
      // per-kernel algorithmic bytes: generate writes 10-B records; dedup reads them and probes
      // (8 B per in-model successor) and writes 16 B per new state; mark reads the
      // inserted positions + keys and sets winner bits; materialize re-reads the parent and writes
      // state + parent pointer
      r.kernels[0].algo_bytes += (double)G_in * 10;
      r.kernels[1].algo_bytes += (double)G_in * (10 + 8) + (double)nnew * (16 + 8);
      r.kernels[2].algo_bytes += (double)nnew * (8 + 16 + 8);
      r.kernels[3].algo_bytes += (double)level_count * WW * 8 + (double)nnew * (S_B + S_B + 8);
      r.seconds_kernels += level_ms / 1000.0;
      r.n_launches += 1;
      if (!last && next_write - base_ > cap_) c[K_ERR] |= OE_CAP_STORE;
      if (c[K_EVENT] != ~0ull && !fifo && (c[K_ERR] & ~(u64)OE_CAP_STORE) == 0) {
        // TLC -workers N found an event: TLC's counterexample and stop point are the single-worker
        // search's, so the model is searched again in FIFO order (it stops at this level)
        RunOpts o1 = o;
        o1.workers = 1;
        o1.recover_path.clear();        // a checkpoint of this search is in its order, not TLC's: start over
        o1.checkpoint_path.clear();
        const u64 evw = c[K_EVENT];
        const int64_t ev_depth = r.depth + 1;
        const int rc = run(o1, r, err);
        if (rc == 0 && r.verdict == MC_VERDICT_CAPACITY_OVERFLOW) {
          // the FIFO re-search stores every level (count_final_level included): when it does not
          // fit, the event the -workers N pass found is still reported, not lost
          static const char* const kind[4] = {"an evaluation error", "a deadlock", "an invariant evaluation error", "an invariant violation"};
          r.error = std::string("the -workers N search found ") + kind[evw & 3] + " at depth " + std::to_string(ev_depth) +
                    "; TLC's single-worker re-search of it (for TLC's counterexample and stop point) ran out of capacity: " + r.error;
        }
        return rc;
      }
      if (c[K_EVENT] != ~0ull && (c[K_ERR] & ~(u64)OE_CAP_STORE) == 0) {
        // the level's first event in TLC's order stops the search; a full state store only
        // matters when it cut off states that come before the event in key order
        const u64 stored = std::min<u64>(nnew, cap_ - std::min<u64>(cap_, level_end - base_));
        bool decided = false;
        if (int rc = handle_event(c[K_EVENT], level_begin, level_count, nnew, stored, r, decided, err)) return rc;
        if (decided) { total_ = level_end + stored; break; }
      }
      if (c[K_ERR]) {
        const u64 e = c[K_ERR];
        r.verdict = MC_VERDICT_CAPACITY_OVERFLOW;
        std::ostringstream os;
        os << "error flags 0x" << std::hex << e << std::dec << " while expanding state " << (c[K_ERRGID] ? (int64_t)(c[K_ERRGID] - 1) : -1) << ":";
        if (e & OE_CAP_ELECTIONS) os << " elections set exceeds the compiled capacity;";
        if (e & OE_CAP_COUNT) os << " message count / bag capacity exceeded;";
        if (e & OE_CAP_STORE)
          os << " state store full (raise state_store_bytes): " << cap_ << " state slots, " << base_
             << " states on the host, level ends at " << level_end << ", " << nnew << " new;";
        if (e & OE_TABLE_FULL) os << " fingerprint table full (raise fp_table_bytes);";
        // the summary counts the completed levels (their sizes sum to it, and the depth is theirs);
        // whatever part of the interrupted level reached the store is not a level of the search
        os << " the summary counts the " << level_end << " states of the " << r.depth << " completed levels;";
        r.error = os.str();
        total_ = level_end;
        r.distinct = (int64_t)total_;
        break;
      }
      int64_t gen = 0;
      for (int k = 0; k < OA_NACT; ++k) { r.act_generated[k] += (int64_t)c[K_ACT + k]; r.act_distinct[k] += (int64_t)c[K_ACT + OA_NACT + k]; gen += (int64_t)c[K_ACT + k]; }
      r.generated += gen;
      r.generated_in_model += (int64_t)G_in;
      r.seen_set_probes += (int64_t)c[K_PROBES];
      r.algo_bytes += (double)level_count * S_B + (double)G_in * 8 + (double)nnew * (16 + S_B);
      if (last) unstored_ = nnew;   // counted, not in the store (total_ counts stored states)
      else total_ += nnew;
      r.distinct = (int64_t)(total_ + unstored_);
      r.levels.back().generated = gen;
      r.levels.back().kernel_ms = level_ms;
      if (nnew > 0) { r.levels.push_back({(int64_t)nnew, 0, 0.0}); r.depth += 1; }
      level_begin += level_count;
      level_count = nnew;
      if (o.checkpoint_every > 0 && !o.checkpoint_path.empty() && r.depth % o.checkpoint_every == 0 && level_count > 0)
        if (int rc = save_checkpoint(o.checkpoint_path, r, level_begin, level_count, err)) return rc;
    }
    if (prof_ && prof_acc_[3])
      std::fprintf(stderr, "orig_probe per workgroup (us): %.2f  (%llu workgroups)\n",
                   prof_acc_[1] / 100.0 / prof_acc_[3], (unsigned long long)prof_acc_[3]);
    if (prof_) std::fprintf(stderr, "max concurrent dedup workgroups %llu\n", (unsigned long long)prof_acc_[4]);
    for (auto& x : prof_acc_) x = 0;
    finish(r, t0);
    return 0;
  }

  // TLC's stop point at the level's first event (key order = TLC's single-worker FIFO order):
  // generated = whole successor lists of the parents before the event's parent and of the
  // parent itself (none when computing its successors raised the error); per-action generated
  // stops at the event's successor; distinct = states inserted before it (the level's new
  // states are stored in key order: a binary search over their parent pointers); left on queue
  // = the level's parents after it + the new states found before it.
  // stored: how many of the level's nnew new states the store holds (a prefix in key order);
  // decided = false when the event may lie behind states the full store cut off
  int handle_event(u64 ev, u64 level_begin, u64 level_count, u64 nnew, u64 stored, RunResult& r, bool& decided,
                   std::string& err) {
    const int kind = (int)(ev & 3);
    const u64 key = ev >> 2, pg = key >> 8;
    const u32 k = (u32)(key & 255);
    const u64 level_end = level_begin + level_count;
    // distinct: this level's new states with key < event key (<= for a violation: the violating
    // state itself is new when it is in the model)
    auto key_at = [&](u64 i, u64& kk) -> int {
      u64 mt = 0;
      HIPCHK(hipMemcpy(&mt, d_meta_ + (level_end - base_) + i, 8, hipMemcpyDeviceToHost));
      kk = ((mt >> 24) << 8) | (mt & 0xff);
      return 0;
    };
    u64 lo = 0, hi = stored;   // first index whose key is beyond the stop point
    while (lo < hi) {
      const u64 mid = (lo + hi) / 2;
      u64 kk = 0;
      if (int rc = key_at(mid, kk)) return rc;
      const bool before = kk < key || (kk == key && kind >= EV_INV_ERROR);
      if (before) lo = mid + 1; else hi = mid;
    }
    const u64 before = lo;
    decided = before < stored || stored == nnew;
    const auto te0 = std::chrono::steady_clock::now();
    auto since = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - te0).count(); };
    if (progress_)
      std::fprintf(stderr, "event kind %d at parent %llu instance %u: %llu new states before it (%s)\n", kind,
                   (unsigned long long)pg, k, (unsigned long long)before, decided ? "decided" : "beyond the stored states");
    if (!decided) return 0;
    (void)nnew;
    // generated (device: re-derive the successor lists of the level's parents up to pg)
    HIPCHK(hipMemsetAsync(d_stop_, 0, (1 + OA_NACT) * 8, stream_));
    const u64 npar = pg - level_begin + 1;
    hipLaunchKernelGGL((orig_stop_generated<S>), dim3((unsigned)((npar + BS - 1) / BS)), dim3(BS), 0, stream_,
                       (const u32*)d_states_, level_begin - base_, npar, level_begin, pg, k, (u32)kind, (unsigned long long*)d_stop_);
    HIPCHK(hipGetLastError());
    u64 gs[1 + OA_NACT];
    HIPCHK(hipMemcpyAsync(gs, d_stop_, sizeof gs, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemsetAsync(d_stop_, 0, (1 + OA_NACT) * 8, stream_));
    if (before)
      hipLaunchKernelGGL(orig_stop_distinct, dim3((unsigned)((before + BS - 1) / BS)), dim3(BS), 0, stream_,
                         (const u64*)(d_meta_ + (level_end - base_)), before, (unsigned long long*)d_stop_);
    HIPCHK(hipGetLastError());
    u64 ds[1 + OA_NACT];
    HIPCHK(hipMemcpyAsync(ds, d_stop_, sizeof ds, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (progress_) std::fprintf(stderr, "stop-point counters over %llu parents: %.3f s\n", (unsigned long long)npar, since());
    r.generated += (int64_t)gs[0];
    for (int a = 0; a < OA_NACT; ++a) { r.act_generated[a] += (int64_t)gs[1 + a]; r.act_distinct[a] += (int64_t)ds[a]; }
    r.distinct = (int64_t)(level_end + before);
    r.left_on_queue = (int64_t)(level_end - pg - 1 + before);
    // the event's parent and (for a violation) successor, re-derived on the host
    u32 w[NWP]; u64 meta = 0;
    if (!stored_state(pg, w, meta)) { err = "event state readback failed"; return MC_E_NO_DEVICE; }
    W s; S::unpack(w, s);
    if (kind == EV_NEXT_ERROR) {
      r.verdict = MC_VERDICT_EVAL_ERROR;
      r.error = "TLC evaluation error while computing the successors of state " + std::to_string(pg) +
                ": log[i][prevLogIndex] applied outside its domain (raft_original.tla:207-210)";
      build_trace(pg, nullptr, s, r, err);
      return 0;
    }
    if (kind == EV_DEADLOCK) {
      r.verdict = MC_VERDICT_DEADLOCK;
      build_trace(pg, nullptr, s, r, err);
      return 0;
    }
    u64 al[S::AW]; S::all_logs_next(s, al);
    W t; u32 e2 = 0;
    const int act = S::apply(s, (int)k, t, e2);
    for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
    r.verdict = MC_VERDICT_INVARIANT_VIOLATION;
    r.violated = first_violated(S::violated(t, m_.rt.invariants));
    r.depth += 1;
    build_trace(pg, act >= 0 ? kOrigActNames[act] : "?", t, r, err);
    if (progress_) std::fprintf(stderr, "trace of %zu states: %.3f s\n", r.trace.size(), since());
    return 0;
  }

  // ---------------------------------------------------------------- checkpoint / recover
  // File: magic, the model's describe_json (a checkpoint only resumes the same model), the BFS
  // position (level_begin/count, stored states) and TLC's counters, then the stored states and
  // parent pointers [0, total).  The seen-set is rebuilt from the states on recovery.
  // fifo: the search order the stored levels are in — 1 = TLC's single-worker FIFO order (-workers 1:
  // kept parents, per-action distinct counts and counterexamples are TLC's), 0 = the -workers N
  // pipeline (first-come dedup).  A -workers N checkpoint cannot resume a -workers 1 search (its
  // kept parents are not TLC's); the reverse is safe.
  struct CkptHead {
    char magic[8];
    u64 nwp, total, level_begin, level_count, seed;
    int64_t generated, distinct, depth, generated_in_model, n_act, n_levels, desc_len, fifo;
  };
  int save_checkpoint(const std::string& path, const RunResult& r, u64 level_begin, u64 level_count, std::string& err) {
    const std::string desc = describe_json();
    CkptHead h;
    std::memcpy(h.magic, "RAFTMCK2", 8);
    h.fifo = last_fifo_ ? 1 : 0;
    h.nwp = NWP; h.total = total_; h.level_begin = level_begin; h.level_count = level_count; h.seed = r.seed;
    h.generated = r.generated; h.distinct = r.distinct; h.depth = r.depth; h.generated_in_model = r.generated_in_model;
    h.n_act = OA_NACT; h.n_levels = (int64_t)r.levels.size(); h.desc_len = (int64_t)desc.size();
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) { err = "cannot write checkpoint " + tmp; return MC_E_IO; }
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(desc.data(), 1, desc.size(), f) == desc.size() &&
              std::fwrite(r.act_generated.data(), 8, OA_NACT, f) == (size_t)OA_NACT &&
              std::fwrite(r.act_distinct.data(), 8, OA_NACT, f) == (size_t)OA_NACT;
    for (const auto& lv : r.levels) ok = ok && std::fwrite(&lv.states, 8, 1, f) == 1 && std::fwrite(&lv.generated, 8, 1, f) == 1;
    // the host part straight from host memory, the device part in bounded blocks (no second copy
    // of the store in host memory)
    constexpr u64 BLK = 1u << 20;
    ok = ok && host_.write_states(f);
    std::vector<u32> blk;
    for (u64 b = base_; ok && b < total_; b += BLK) {
      const u64 n = std::min<u64>(BLK, total_ - b);
      blk.resize(n * NWP);
      ok = hipMemcpy(blk.data(), d_states_ + (b - base_) * NWP, n * NWP * 4, hipMemcpyDeviceToHost) == hipSuccess &&
           std::fwrite(blk.data(), 4, n * NWP, f) == n * NWP;
    }
    ok = ok && host_.write_meta(f);
    std::vector<u64> mblk;
    for (u64 b = base_; ok && b < total_; b += BLK) {
      const u64 n = std::min<u64>(BLK, total_ - b);
      mblk.resize(n);
      ok = hipMemcpy(mblk.data(), d_meta_ + (b - base_), n * 8, hipMemcpyDeviceToHost) == hipSuccess &&
           std::fwrite(mblk.data(), 8, n, f) == n;
    }
    ok = (std::fclose(f) == 0) && ok;
    if (!ok || std::rename(tmp.c_str(), path.c_str()) != 0) { err = "writing checkpoint " + path + " failed"; return MC_E_IO; }
    return 0;
  }
  int load_checkpoint(const std::string& path, bool fifo, RunResult& r, u64& level_begin, u64& level_count, std::string& err) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) { err = "cannot read checkpoint " + path; return MC_E_IO; }
    CkptHead h;
    const std::string desc = describe_json();
    std::string fdesc;
    bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, "RAFTMCK2", 8) == 0 && h.nwp == (u64)NWP &&
              h.n_act == OA_NACT && h.desc_len >= 0 && h.desc_len < (1 << 20) && h.n_levels > 0 && h.n_levels < (1 << 20);
    if (ok) { fdesc.resize((size_t)h.desc_len); ok = std::fread(&fdesc[0], 1, fdesc.size(), f) == fdesc.size(); }
    if (!ok || fdesc != desc) { std::fclose(f); err = "checkpoint " + path + " is not a checkpoint of this model"; return MC_E_INVALID; }
    if (fifo && !h.fifo) {
      std::fclose(f);
      err = "checkpoint " + path + " was written by a -workers N search: its kept parents are not TLC's single-worker "
            "FIFO ones, so it cannot resume a -workers 1 search";
      return MC_E_INVALID;
    }
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
    // streamed: the host part into one host segment, the device part block by block into the
    // store (no second copy of the checkpoint in host memory)
    host_.clear();
    u32* hs = nullptr; u64* hm = nullptr;
    if (lb) host_.append(lb, &hs, &hm);
    ok = ok && std::fread(hs, 4, lb * NWP, f) == lb * NWP;
    constexpr u64 BLK = 1u << 20;
    std::vector<u32> blk;
    for (u64 b = lb; ok && b < h.total; b += BLK) {
      const u64 n = std::min<u64>(BLK, h.total - b);
      blk.resize(n * NWP);
      ok = std::fread(blk.data(), 4, n * NWP, f) == n * NWP &&
           hipMemcpy(d_states_ + (b - lb) * NWP, blk.data(), n * NWP * 4, hipMemcpyHostToDevice) == hipSuccess;
    }
    ok = ok && std::fread(hm, 8, lb, f) == lb;
    std::vector<u64> mblk;
    for (u64 b = lb; ok && b < h.total; b += BLK) {
      const u64 n = std::min<u64>(BLK, h.total - b);
      mblk.resize(n);
      ok = std::fread(mblk.data(), 8, n, f) == n &&
           hipMemcpy(d_meta_ + (b - lb), mblk.data(), n * 8, hipMemcpyHostToDevice) == hipSuccess;
    }
    std::fclose(f);
    if (!ok) { host_.clear(); err = "checkpoint " + path + " is truncated"; return MC_E_IO; }
    HIPCHK(hipMemsetAsync(d_ctr_, 0, K_NCTR * 8, stream_));
    // the host part's fingerprints go in through the (idle) candidate buffer, chunk by chunk
    const u64 stage = std::max<u64>(1, chunk_states_ * S::NI * 8 / (NWP * 4));
    for (u64 b = 0; b < lb; b += stage) {
      const u64 n = std::min<u64>(stage, lb - b);
      HIPCHK(hipMemcpy(d_rfp_, hs + b * NWP, n * NWP * 4, hipMemcpyHostToDevice));
      if (last_fifo_)
        hipLaunchKernelGGL((orig_reinsert<S, 2>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_,
                           (const u32*)d_rfp_, n, d_table_, table_mask_, (u64)h.seed, (unsigned long long*)d_ctr_);
      else
        hipLaunchKernelGGL((orig_reinsert<S, 1>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_,
                           (const u32*)d_rfp_, n, d_table_, 2 * table_mask_ + 1, (u64)h.seed, (unsigned long long*)d_ctr_);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(stream_));
    }
    if (h.total > lb) {
      if (last_fifo_)
        hipLaunchKernelGGL((orig_reinsert<S, 2>), dim3((unsigned)((h.total - lb + BS - 1) / BS)), dim3(BS), 0, stream_,
                           (const u32*)d_states_, (u64)(h.total - lb), d_table_, table_mask_, (u64)h.seed, (unsigned long long*)d_ctr_);
      else
        hipLaunchKernelGGL((orig_reinsert<S, 1>), dim3((unsigned)((h.total - lb + BS - 1) / BS)), dim3(BS), 0, stream_,
                           (const u32*)d_states_, (u64)(h.total - lb), d_table_, 2 * table_mask_ + 1, (u64)h.seed, (unsigned long long*)d_ctr_);
      HIPCHK(hipGetLastError());
    }
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
    if (unstored_) { err = "mc_dump_states: the last level was counted, not stored (count_final_level)"; return MC_E_STATE; }
    std::vector<u32> h(total_ * NWP);
    host_.for_each_segment([&](u64 g0, u64 n, const u32* st, const u64*) { std::memcpy(h.data() + g0 * NWP, st, n * NWP * 4); });
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
    unstored_ = 0;
    last_fifo_ = false;   // 8-B entries (observed_collision)
    HIPCHK(hipMemsetAsync(d_table_, 0, (table_mask_ + 1) * 16, stream_));
    HIPCHK(hipMemsetAsync(d_ctr_, 0, K_NCTR * 8, stream_));
    HIPCHK(hipMemsetAsync(d_ctr_ + K_EVENT, 0xFF, 8, stream_));
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
    base_ = 0; host_.clear();
    if ((int)fp_owner(fp0, (u32)world) == rank) {
      u32 wp[NWP] = {0}; for (int q = 0; q < S::NW; ++q) wp[q] = w0[q];
      HIPCHK(hipMemcpy(d_table_ + (fp0 & sh_table_mask()), &fp0, 8, hipMemcpyHostToDevice));
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
  u64 sh_table_mask() const { return 2 * table_mask_ + 1; }   // sharded seen-set: 8-B entries
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
      const GenArgs g = gen_args(sh_chunk_begin_, (u64)count, sh_chunk_begin_, sres_.seed, sopts_);
      const RouteArgs ra = route_args((u32)world_);
      const unsigned nblk = (unsigned)((count + BS - 1) / BS);
      HIPCHK(hipEventRecord(ev_[5], stream_));
      HIPCHK(hipMemsetAsync(d_ctr_ + K_LEAD, 0, 8, stream_));
      launch_generate(g, nblk);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(ev_[6], stream_));
      hipLaunchKernelGGL(orig_route_blk, dim3(nblk), dim3(BS), 0, stream_, ra);
      HIPCHK(hipGetLastError());
      HIPCHK(hipEventRecord(ev_[2], stream_));
    }
    u64 c[8] = {0};
    HIPCHK(hipMemcpyAsync(c, d_rcnt_, 8 * 8, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (count > 0) {
      u64 valid = 0; for (int r = 0; r < world_; ++r) valid += c[r];
      auto& ke = sres_.kernels[0]; ke.ms += time_ms(5, 6); ke.launches++; ke.algo_bytes += (double)count * NWP * 4;
      auto& kr = sres_.kernels[1]; kr.ms += time_ms(6, 2); kr.launches++; kr.algo_bytes += (double)valid * 16;
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
        d.recv = (const u64*)recv + 2 * off; d.n = n; d.table = d_table_; d.table_mask = sh_table_mask();
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
      m.seed = sres_.seed; m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_;
      m.st_states = nullptr; m.st_meta = nullptr; m.st_dst = 0; m.st_cap = 0; m.store = 1;
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
    // the sharded raft_original search is not FIFO-ranked across ranks: any event stops it
    sh_event_ = c[K_EVENT];
    const int kind = sh_event_ == ~0ull ? -1 : (int)(sh_event_ & 3);
    st[3] = (int64_t)(c[K_ERR] | (sh_next_write_ > cap_ ? (u64)OE_CAP_STORE : 0ull) | (kind == EV_NEXT_ERROR ? (u64)OE_EVAL_LOG_INDEX : 0ull));
    st[4] = kind == EV_VIOLATION ? 1 : 0; st[5] = kind == EV_DEADLOCK ? 1 : 0; st[6] = (int64_t)sh_level_count_;
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
      sh_event_ = ~0ull;
      std::ostringstream os; os << "error flags 0x" << std::hex << g[3] << " raised on some rank"; sres_.error = os.str();
      *done = 1;
    }
    if (*done && sres_.verdict == MC_VERDICT_CAPACITY_OVERFLOW) {
      // as on one GPU: the summary counts the completed levels; the interrupted one is not a level
      sres_.error += "; the summary counts the " + std::to_string(sres_.distinct) + " states of the " +
                     std::to_string(sres_.depth) + " completed levels";
    } else {
      sres_.distinct += g[0];
      if (g[0] > 0) { sres_.levels.push_back({g[0], 0, 0.0}); sres_.depth += 1; }
    }
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
    HIPCHK(hipMemset(d_ctr_ + K_EVENT, 0xFF, 8));
    sres_.n_launches += 1;
    if (*done) {
      sviol_act_.clear();
      if (sres_.verdict == MC_VERDICT_INVARIANT_VIOLATION && sh_event_ != ~0ull && (sh_event_ & 3) == EV_VIOLATION) {
        // this rank's violating successor, re-derived from (parent, instance)
        const u64 key = sh_event_ >> 2, par = key >> 8;
        const int k = (int)(key & 255);
        u32 w[NWP];
        if (hipMemcpy(w, d_states_ + par * NWP, NWP * 4, hipMemcpyDeviceToHost) == hipSuccess) {
          W s, t; S::unpack(w, s);
          u64 al[S::AW]; S::all_logs_next(s, al);
          u32 e2 = 0;
          const int act = S::apply(s, k, t, e2);
          for (int q = 0; q < S::AW; ++q) t.allLogs[q] = al[q];
          sviol_bad_ = S::violated(t, m_.rt.invariants);
          sviol_parent_ = ((u64)rank_ << 37) | par; sviol_act_ = act >= 0 ? kOrigActNames[act] : "?";
          sviol_text_ = state_text(t, true);
        }
      }
      if (sres_.verdict == MC_VERDICT_INVARIANT_VIOLATION) sres_.violated = sviol_act_.empty() ? "" : first_violated(sviol_bad_);
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

  // ---------------------------------------------------------------- native level loop
  // The whole sharded BFS of raft-tla_amd/shard.py (sharded_bfs) in C++ on one HIP stream:
  // per chunk generate+route -> counts exchange -> ROUTE payload -> dedup -> counts exchange ->
  // REPLY payload -> materialize -> STATES payload -> store, over a ShardTransport
  // (shard_transport.h: grouped ncclSend/ncclRecv straight from the kernels' buffers between
  // GPUs, or the in-process loopback of mc_shard_run_loopback) with two host synchronisations
  // per chunk (the counts) plus one per level (the all-reduce of the level statistics).
  int shard_run_native(ShardTransport& T, std::string& err) override {
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
        const char* src[8]; char* dst[8]; u64 n8[8];
        for (int r = 0; r < W; ++r) { src[r] = (const char*)(d_xs + r); dst[r] = (char*)(d_xr + r); n8[r] = 8; }
        if (T.exchange(me, W, src, n8, dst, n8, stream_, err)) return MC_E_NO_DEVICE;
      }
      HIPCHK(hipMemcpyAsync(h_xs, d_xs, 16 * 8, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
      return 0;
    };
    // payload exchange: segment r of the send side (bytes) goes to rank r, the receive side is
    // packed in source-rank order; the self segment is not copied (its consumer reads it in
    // place), so dst + roff[me] stays unused
    auto xpay = [&](const char* const* src, const u64* sbytes, char* dst, const u64* rbytes) -> int {
      char* dsts[8]; u64 acc = 0;
      for (int r = 0; r < W; ++r) { dsts[r] = dst + acc; acc += rbytes[r]; }
      if (sbytes[me] != rbytes[me]) { err = "sharded exchange: self segment size mismatch"; return MC_E_STATE; }
      if (W > 1 && T.exchange(me, W, src, sbytes, dsts, rbytes, stream_, err)) return MC_E_NO_DEVICE;
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
      // g: local stats in, global stats out; MAX slots: [3,6) flags, [6] chunk rounds of the next
      // level, [8, 8+32) one slot per bit of the error word (max per bit = bitwise OR over ranks:
      // two ranks' different capacity errors are both reported)
      static_assert(8 + 32 <= MC_SHARD_NSTAT, "max slots");
      for (int k = 0; k < MC_SHARD_NSTAT; ++k) h_sum[k] = g[k];
      for (int k = 0; k < MC_SHARD_NSTAT; ++k) h_max[k] = 0;
      h_max[3] = g[3]; h_max[4] = g[4]; h_max[5] = g[5]; h_max[6] = next_chunks;
      for (int b = 0; b < 32; ++b) h_max[8 + b] = (g[3] >> b) & 1;
      HIPCHK(hipMemcpyAsync(d_sum, h_sum, 2 * MC_SHARD_NSTAT * 8, hipMemcpyHostToDevice, stream_));
      if ((W > 1 || T.allreduce_at_world1()) && T.allreduce(d_sum, MC_SHARD_NSTAT, d_max, 8 + 32, stream_, err)) return MC_E_NO_DEVICE;
      HIPCHK(hipMemcpyAsync(h_sum, d_sum, 2 * MC_SHARD_NSTAT * 8, hipMemcpyDeviceToHost, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
      for (int k = 0; k < MC_SHARD_NSTAT; ++k) g[k] = h_sum[k];
      g[3] = 0;
      for (int b = 0; b < 32; ++b) g[3] |= (h_max[8 + b] ? 1ll : 0ll) << b;
      g[4] = h_max[4]; g[5] = h_max[5];
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
    // count_final_level: the level at depth max_depth is never expanded, so its new states are
    // deduplicated by their owners, counted and invariant-checked by the generating rank, but
    // neither shipped to the owners nor stored (no STATES exchange, no store kernel): the ranks'
    // stores hold the levels before it (BASELINE configs[4], C5v2 to depth 14 on 8 GPUs)
    const bool count_last = sopts_.count_final_level && sopts_.max_depth > 0;
    unstored_ = 0;
    for (;;) {
      const u64 front = sh_level_count_;
      const bool last = count_last && sres_.depth + 1 >= sopts_.max_depth;
      if (sopts_.test_fail_rank == me && sopts_.test_fail_depth == sres_.depth) {   // mc_set_fault_injection (tests)
        err = "injected failure (mc_set_fault_injection) at depth " + std::to_string(sres_.depth);
        return MC_E_STATE;
      }
      for (int64_t c = 0; c < nchunks; ++c) {
        const u64 begin = std::min<u64>((u64)c * chunk, front);
        const u64 count = std::min<u64>(chunk, front - begin);
        sh_chunk_begin_ = sh_level_begin_ + begin; sh_chunk_count_ = count;
        if (W == 1) {
          // World 1: every fingerprint is this rank's, so the route pass, both counts exchanges (the
          // chunk's two host synchronisations) and the acknowledged re-derivation collapse into the
          // single-GPU -workers N kernels: orig_dedup_plain's first-come LDS filter is the route's, its
          // probes the owner's, orig_materialize_plain stores the new states behind the level; the
          // counts stay on the device (orig_advance), the host waits once per level
          if (count == 0) continue;
          const GenArgs g = gen_args(sh_chunk_begin_, count, sh_chunk_begin_, sres_.seed, sopts_);
          const unsigned nblk = (unsigned)((count + BS - 1) / BS);
          HIPCHK(hipMemsetAsync(d_ctr_ + K_LEAD, 0, 8, stream_));
          NAT_TIMED(0, launch_generate(g, nblk));
          sres_.kernels[0].algo_bytes += (double)count * NWP * 4;
          DedupArgs d;
          d.rfp = d_rfp_; d.rkey = d_rkey_; d.rcnt = d_rcnt_blk_; d.region = (u64)BS * S::NI; d.gid0 = sh_chunk_begin_;
          d.urec = (ulonglong2*)d_urec_; d.ucnt = d_ucnt_;
          d.table = d_table_; d.table_mask = sh_table_mask(); d.newpos = d_newrec_; d.ctr = (unsigned long long*)d_ctr_;
          d.prof = 0;
          NAT_TIMED(2, hipLaunchKernelGGL((orig_dedup_plain<WW, false>), dim3(nblk), dim3(BS), 0, stream_, d));
          MatPlainArgs m;
          m.states = d_states_; m.meta = d_meta_; m.newrec = d_newrec_; m.base = 0; m.dst_base = sh_next_write_;
          m.cap = cap_; m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_; m.store = last ? 0u : 1u;
          NAT_TIMED(3, hipLaunchKernelGGL((orig_materialize_plain<S>), dim3((unsigned)std::min<u64>(4096, (count * 2 + BS - 1) / BS)),
                                          dim3(BS), 0, stream_, m));
          hipLaunchKernelGGL(orig_advance, dim3(1), dim3(64), 0, stream_, (unsigned long long*)d_ctr_);
          HIPCHK(hipGetLastError());
          continue;
        }
        HIPCHK(hipMemsetAsync(d_rcnt_, 0, 16 * 8, stream_));
        if (count > 0) {
          const GenArgs g = gen_args(sh_chunk_begin_, count, sh_chunk_begin_, sres_.seed, sopts_);
          const unsigned nblk = (unsigned)((count + BS - 1) / BS);
          HIPCHK(hipMemsetAsync(d_ctr_ + K_LEAD, 0, 8, stream_));
          NAT_TIMED(0, launch_generate(g, nblk));
          sres_.kernels[0].algo_bytes += (double)count * NWP * 4;
          const RouteArgs ra = route_args((u32)W);
          NAT_TIMED(1, hipLaunchKernelGGL(orig_route_blk, dim3(nblk), dim3(BS), 0, stream_, ra));
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
              d.n = n; d.table = d_table_; d.table_mask = sh_table_mask();
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
          if (!last) {
            void* so = d_stout_;
            u64 socap = stout_cap_ * SBW;
            if (int rc = grow(so, socap, atot * SBW)) return rc;
            d_stout_ = (u32*)so; stout_cap_ = socap / SBW;
          }
          for (int r = 0; r < W; ++r) {
            if (!ack[r]) continue;
            MatShArgs m;
            m.states = d_states_; m.acks = r == me ? d_newrec_ + seg_off_[me] : (const u64*)nat_acks_ + seg_off_ack_[r];
            m.n = ack[r]; m.chunk_begin = sh_chunk_begin_;
            m.chunk_count = sh_chunk_count_; m.out = last ? nullptr : d_stout_ + seg_off_ack_[r] * (NWP + 4); m.rank_bits = (u64)me << 37;
            m.seed = sres_.seed; m.rt = m_.rt; m.ctr = (unsigned long long*)d_ctr_;
            m.st_states = nullptr; m.st_meta = nullptr; m.st_dst = 0; m.st_cap = 0; m.store = last ? 0u : 1u;
            if (r == me && !last) {   // my own new states: into my store after the ones of lower ranks
              u64 before = 0; for (int q = 0; q < me; ++q) before += rep[q];
              m.st_states = d_states_; m.st_meta = d_meta_; m.st_dst = sh_next_write_ + before; m.st_cap = cap_;
            }
            NAT_TIMED(3, hipLaunchKernelGGL((orig_materialize_sh<S>), dim3((unsigned)((ack[r] + BS - 1) / BS)), dim3(BS), 0, stream_, m));
          }
          sres_.kernels[3].algo_bytes += (double)atot * (8 + NWP * 4 + (last ? 0 : SBW));
        }
        if (last) {   // the owners count their new states of the final level; nothing is shipped
          for (int r = 0; r < W; ++r) sh_new_ += rep[r];
          continue;
        }
        // ---- STATES: packed states + parent pointers to their owners (sizes known: no sync)
        for (int r = 0; r < W; ++r) { sb[r] = ack[r] * SBW; rb[r] = rep[r] * SBW; src[r] = (const char*)(d_stout_ + seg_off_ack_[r] * (NWP + 4)); }
        if (int rc = grow(nat_stin_, nat_stin_cap_, ntot * SBW)) return rc;
        if (int rc = xpay(src, sb, (char*)nat_stin_, rb)) return rc;
        {   // the owner stores the states in source-rank order (its own ones were materialized in place)
          u64 in_off = 0;
          for (int r = 0; r < W; ++r) {
            const u64 n = rep[r];
            if (n && r == me) { sh_next_write_ += n; sh_new_ += n; }
            else if (n) {
              StoreArgs a;
              a.in = (const u32*)((const char*)nat_stin_ + in_off * SBW);
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
      if (W == 1) {   // the level's new states (orig_advance's running count), stored behind the level
        u64 lvl_new = 0;
        HIPCHK(hipMemcpy(&lvl_new, d_ctr_ + K_LEVEL_NEW, 8, hipMemcpyDeviceToHost));
        sh_new_ = lvl_new;
        if (!last) sh_next_write_ += lvl_new;
      }
      int64_t g[MC_SHARD_NSTAT];
      if (int rc = shard_level_stats(g, err)) return rc;
      if (W == 1) {   // SURVEY.md §8(d) bytes of the fused kernels (the W > 1 ones count per exchange)
        sres_.kernels[2].algo_bytes += (double)g[2] * (10 + 8) + (double)sh_new_ * (16 + 8);
        sres_.kernels[3].algo_bytes += (double)sh_new_ * (2.0 * NWP * 4 + 8);
      }
      int64_t next_chunks = 0;
      if (int rc = allreduce_level(g, rounds(sh_new_), next_chunks)) return rc;
      if (last) unstored_ = sh_new_;   // this rank's share of the final level: counted, not in the store
      int done = 0;
      if (int rc = shard_level_commit(g, &done, err)) return rc;
      if (done) break;
      nchunks = next_chunks;
    }
#undef NAT_TIMED
    return 0;
  }

 private:
  OrigModel m_;
  static constexpr int WW = (S::NI + 63) / 64;   // winner-mask words per parent
  u64* d_table_ = nullptr; u32* d_states_ = nullptr; u64* d_meta_ = nullptr; u64* d_ctr_ = nullptr; u64* d_stop_ = nullptr;
  u64* h_ctr_ = nullptr;     // pinned host copy of the level counters
  bool ctr_clean_ = false;   // d_ctr_ already reset for the next level (queued after the readback)
  u64* d_rfp_ = nullptr; unsigned short* d_rkey_ = nullptr; u32* d_rcnt_blk_ = nullptr; u64* d_newrec_ = nullptr;
  u64* d_winmask_ = nullptr; u32* d_wcnt_ = nullptr; u64* d_woff_ = nullptr; u64* d_urec_ = nullptr; u32* d_ucnt_ = nullptr;
  u64* d_route_ = nullptr; u64* d_rcnt_ = nullptr; u32* d_stout_ = nullptr; u64 stout_cap_ = 0;
  u32* d_lead_ = nullptr;      // [chunk] the chunk's leader-work parents (orig_generate -> orig_generate_lead)
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_[9] = {};
  u64 table_mask_ = 0, cap_ = 0, total_ = 0, chunk_states_ = 0;
  u64 unstored_ = 0;   // states of the last level counted but not stored (count_final_level)
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
  u64 sh_event_ = ~0ull;
  bool last_fifo_ = true;   // seen-set layout of the last single-GPU run (16-B keyed / 8-B entries)
  // RAFTMC_PROF=1: per-phase wall-clock ticks (100 MHz) of orig_dedup, summed over workgroups
  const bool prof_ = std::getenv("RAFTMC_PROF") != nullptr;
  const bool progress_ = std::getenv("RAFTMC_PROGRESS") != nullptr;
  u64 prof_acc_[5] = {0, 0, 0, 0, 0};
  // native (RCCL) level loop buffers
  u64* d_nat_ = nullptr; u64* h_nat_ = nullptr;
  void* nat_recv_ = nullptr; void* nat_acks_ = nullptr; void* nat_stin_ = nullptr;
  u64 nat_recv_cap_ = 0, nat_acks_cap_ = 0, nat_stin_cap_ = 0;
  std::vector<hipEvent_t> nat_ev_;
  std::vector<hipEvent_t> lvl_ev_;
  // completed levels moved to host memory: global ids [0, base_) live in host_ (segments)
  u64 base_ = 0;
  HostStore host_{NWP};

  void release_device() override { release(); }
  void release() {
    for (void* p : {(void*)d_table_, (void*)d_states_, (void*)d_meta_, (void*)d_ctr_, (void*)d_stop_, (void*)d_rfp_, (void*)d_rkey_,
                    (void*)d_rcnt_blk_, (void*)d_newrec_, (void*)d_winmask_, (void*)d_wcnt_, (void*)d_woff_, (void*)d_urec_, (void*)d_ucnt_,
                    (void*)d_route_, (void*)d_rcnt_, (void*)d_stout_, (void*)d_lead_})
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
    if (h_ctr_) (void)hipHostFree(h_ctr_);
    h_ctr_ = nullptr; ctr_clean_ = false;
    d_table_ = nullptr; d_states_ = nullptr; d_meta_ = nullptr; d_ctr_ = nullptr; d_stop_ = nullptr;
    d_rfp_ = nullptr; d_rkey_ = nullptr; d_rcnt_blk_ = nullptr; d_newrec_ = nullptr; d_winmask_ = nullptr; d_wcnt_ = nullptr; d_woff_ = nullptr; d_urec_ = nullptr; d_ucnt_ = nullptr; d_route_ = nullptr; d_rcnt_ = nullptr; d_stout_ = nullptr; stout_cap_ = 0;
    d_lead_ = nullptr;
    stream_ = nullptr; alloc_world_ = 0;
  }

  std::string first_violated(u32 bad) const {
    for (auto& n : m_.inv_names) {
      if (bad & orig_inv_bit(n.c_str())) return n;
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
      std::memcpy(w, host_.state(gid), NWP * 4);
      meta = host_.meta(gid);
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
    u32* hs = nullptr; u64* hm = nullptr;
    const auto ts = std::chrono::steady_clock::now();
    auto since = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - ts).count(); };
    host_.append(d, &hs, &hm);   // a segment of its own: the host part is never reallocated
    if (progress_) std::fprintf(stderr, "spill: %.1f GB of host memory allocated in %.3f s\n", d * (NWP * 4.0 + 8) / 1e9, since());
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(hs, d_states_, d * NWP * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hm, d_meta_, d * 8, hipMemcpyDeviceToHost));
    if (progress_) std::fprintf(stderr, "spill: copied to host at %.3f s\n", since());
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
  X(5, 1, 3, 3, 4) /* C5 */ \
  X(5, 2, 3, 3, 8) /* C5 with 2 values and 8 messages (compact election records) */ \
  X(5, 2, 2, 4, 6) /* 5 servers, one election term, 6 messages: compact election records within reach */
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
