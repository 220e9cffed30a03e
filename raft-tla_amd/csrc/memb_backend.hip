// raftmc — gfx950 BFS backend for tlc_membership/raft.tla (SYMMETRY perms,
// VIEW vars, history summary automaton, scenario properties).
//
// Under VIEW the reachable set depends on WHICH successor of a view class is
// kept (history is outside the view but read by constraints, raft.tla:1105-1137),
// so the search reproduces TLC's single-worker FIFO first-found order
// (SURVEY.md §7 hard part 2): every successor has a key
//     key = (rank of its parent in the level) * NSLOT + slot(instance, sub)
// equal to its position in the oracle's enumeration order, the seen-set keeps
// the minimum key per fingerprint of the level (atomicMax on the complement),
// and the next level is written in key order.  Per frontier chunk:
//
//  1. memb_expand     lane per state, wave-uniform loop over the Next
//                     instances; constraint filter, out-of-model invariant
//                     checks; in-model cells compacted with wave ballots
//  1b memb_fingerprint lane per in-model successor (full lanes): re-derive it,
//                     symmetric FP64 of the view (min over Permutations(Server))
//                     into cand[slot][state]
//  1c memb_oom_check  lane per out-of-model successor: invariants (TLC [ext] (ii))
//  2. memb_dedup_cells workgroup b takes expand-workgroup b's in-model cells, 8
//                     independent seen-set probes per thread over 16-B entries
//                     (fp, ~level|key); insert-if-absent with CAS, then
//                     atomicMax of ~(level << 40 | key); cand := entry+1
//  3. memb_select     lane per state: which of its in-model slots (the slot
//                     mask memb_expand wrote) won its fingerprint (entry still
//                     holds its own key), per-block exclusive scan
//  4. memb_scan_blocks exclusive scan of the block totals (one workgroup)
//  5. memb_compact    lane per state: winners' (parent, slot) records in key order
//  6. memb_materialize lane per new state: re-derive, store packed state and
//                     parent pointer, per-action distinct counts, invariants
//
// The first "event" of a level in key order (TLC evaluation error while
// computing successors, deadlock, invariant error, invariant violation) is the
// 64-bit atomicMin of (key << 2 | kind); the host re-derives that successor
// with the same spec code to name the invariant and build the trace.
#include <hip/hip_runtime.h>
#include <rocprim/device/device_radix_sort.hpp>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstring>
#include <sstream>

#include "../../include/raftmc.h"
#include "backend.h"
#include "fifo_shard_loop.h"
#include "fp_gap.h"
#include "host_store.h"
#include "memb_prefix.h"
#include "memb_spec.h"
#include "memb_text.h"

namespace rmc {

namespace {
enum {
  C_CELLS = 0, C_ERR = 1, C_EVENT = 2, C_NEW = 3, C_ERRGID = 4, C_GEN_IN = 5, C_CELLS_OOM = 6,
  C_BIG = 7,   // the chunk's cells memb_fingerprint_lds left to memb_fingerprint_list (zeroed by memb_expand)
  C_ACT = 8, C_SHARD = C_ACT + 2 * MA_NACT, C_NCTR = C_SHARD + 8   // C_SHARD: per-rank bucket counters
};
enum { EV_NEXT_ERROR = 0, EV_DEADLOCK = 1, EV_INV_ERROR = 2, EV_VIOLATION = 3 };
enum { MERR_TABLE_FULL = 0x100, MERR_STORE = 0x200 };
constexpr int BS = 256;
constexpr int DPER = 16;               // probes in flight per dedup thread
constexpr u64 WINBIT = 1ull << 63;
constexpr int SCAN_MAX_BLOCKS = 4096;  // chunk <= 4096 * BS states
}  // namespace

struct MGenArgs {
  const u32* states;
  u64 chunk_begin, chunk_count, rank0;     // first state of the chunk: gid and rank in its level
  u64* cand;                               // [NSLOT][chunk] fingerprints, 0 = none
  u32* cells;                              // per workgroup: BS*NSLOT cells (slot * chunk + state) of in-model successors,
                                           // in four per-wave regions of 64*NSLOT
  u32* cells_oom;                          // ... of out-of-model successors (TLC checks their invariants, [ext] (ii))
  u32* cell_count;                         // per workgroup: in-model cells of waves 0-3, out-of-model cells of waves 0-3
  unsigned short* nsucc;                   // [chunk] successors per state (TLC "generated")
  u64 seed;
  MembRuntime rt;
  u32 inv_oom, deadlock;
  unsigned long long* ctr;
  unsigned long long* prof;                // RMC_FP_PROF builds: wave cycles per fingerprint stage (else null)
  u32* big;                                // TLC mode: cells whose parent's bag exceeds memb_fingerprint_lds's slice
  u32 slice_cap;                           // parent bag entries memb_fingerprint_lds keeps (<= its slice - 1)
  u64* smask;                              // [SMW][chunk] each state's in-model slots (bit per slot); null: the
                                           // dense form, every cand slot written (the sharded loop reads it so)
};

// Phase 1 for the instances [K0, K1) with NS successors each.  The bounds are compile-time so
// apply's dispatch is pruned to the range; launder() keeps the per-state decodes inside the
// loop body (hoisting them over ~100 instances exhausts the register file).
template <class S, int K0, int K1, int NS>
__device__ __forceinline__ void expand_group(typename S::Work& s, const MGenArgs& a, bool active, u64 tid, u32& err,
                                             u32& nsucc, u32& nin, unsigned int* lds_cnt, u32& wcin, u32& wcoom,
                                             u64& mcur, int& mwi) {
  using W = typename S::Work;
  // this wave's own regions of the workgroup's cell lists (64 * NSLOT cells each): a wave's cells stay
  // together, parent group by parent group (memb_fingerprint's lanes then share the 64 parents of one
  // expand wave, not the workgroup's 256: fewer parent lines re-fetched past L2)
  const u64 wreg = (u64)blockIdx.x * (BS * S::NSLOT) + (u64)(threadIdx.x >> 6) * (64 * S::NSLOT);
  u32* cells = a.cells + wreg;
  u32* cells_oom = a.cells_oom + wreg;
  for (int k = K0; k < K1; ++k) {
    const bool en = S::group_enabled(k, a.rt.next);                 // wave-uniform
    for (int sub = 0; sub < NS; ++sub) {
      const int slot = S::slot_of(k, sub);
      if (active && !a.smask) a.cand[(u64)slot * a.chunk_count + tid] = 0;   // (dense form only)
      // the slot mask one 64-bit word at a time: slots come in increasing order (slot_of), every one of them
      if ((slot >> 6) != mwi) {   // (wave-uniform)
        if (active && a.smask && mwi >= 0) a.smask[(u64)mwi * a.chunk_count + tid] = mcur;
        mcur = 0;
        mwi = slot >> 6;
      }
      if (!en) continue;
      S::launder(s);
      bool need = false, oom = false;
      if (active) {
        // the successor without its bag (round 6): the constraints read the bag's total and RequestVote
        // counts, which S::in_model_delta takes from the parent's bag and the change d, so no successor
        // bag is built (with_msg's sorted insertion over MK + 1 registers)
        W t;
        typename S::Delta d;
        const int bi = S::bag_slot_of(k);
        const u64 xent = bi >= 0 ? sel(s.bag, bi) : S::EMPTY;
        const int act = S::template apply_nobag<false>(s, k, sub, xent, t, d, err, a.rt);
        if (act >= 0) {
          // TLC's generated counters: the copies a disjunctive guard enumerates (S::tlc_copies)
          const int cp = (act == MA_HandleCheckOldConfig || act == MA_HandleCatchupResponse) ? S::template tlc_copies<true>(s, k, sub, a.rt, xent) : 1;
          nsucc += (u32)cp;
          atomicAdd(&lds_cnt[act], (unsigned)cp);
          if (S::in_model_delta(t, s, d, a.rt, err)) {   // (also flags a bag beyond the compiled capacity)
            need = true;
            ++nin;
          } else if (a.inv_oom) {
            oom = true;                                              // invariants checked by memb_oom_check
          }
        }
      }
      const u32 cell = (u32)((u64)slot * a.chunk_count + tid);
      mcur |= (u64)need << (slot & 63);
      // one ballot per list, consecutive stores at the wave's running count (wave-uniform: no atomic)
      const u64 mask = __ballot(need);
      if (need) cells[wcin + __builtin_amdgcn_mbcnt_hi((u32)(mask >> 32), __builtin_amdgcn_mbcnt_lo((u32)mask, 0u))] = cell;
      wcin += (u32)__popcll(mask);
      const u64 omask = __ballot(oom);
      if (oom) cells_oom[wcoom + __builtin_amdgcn_mbcnt_hi((u32)(omask >> 32), __builtin_amdgcn_mbcnt_lo((u32)omask, 0u))] = cell;
      wcoom += (u32)__popcll(omask);
    }
  }
}

// A workgroup's cells: its four waves' regions (wave w's at w * 64 * NSLOT, cnt[w] cells each),
// concatenated in wave order.
struct CellRegions {
  u32 p1, p2, p3, n, wreg;
  __device__ CellRegions(const u32* cnt, u32 wave_region) {   // (uniform: kept in SGPRs)
    p1 = __builtin_amdgcn_readfirstlane(cnt[0]); p2 = p1 + __builtin_amdgcn_readfirstlane(cnt[1]);
    p3 = p2 + __builtin_amdgcn_readfirstlane(cnt[2]); n = p3 + __builtin_amdgcn_readfirstlane(cnt[3]); wreg = wave_region;
  }
  __device__ u32 at(u32 i) const {   // w * wreg + (i - p_w), as three selects (no indexed table)
    return i + (i >= p1 ? wreg - p1 : 0u) + (i >= p2 ? wreg - (p2 - p1) : 0u) + (i >= p3 ? wreg - (p3 - p2) : 0u);
  }
};

// Phase 1: successors, constraints and TLC "generated" counts; in-model (and, for the
// invariant check, out-of-model) cells are appended with one atomic per wave and slot.
template <class S>
#ifndef RMC_MEXP_WAVES
#define RMC_MEXP_WAVES 1   // amdgpu_waves_per_eu hint of memb_expand (1: none; 3 spills 214 VGPRs)
#endif
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RMC_MEXP_WAVES))) memb_expand(MGenArgs a) {
  using W = typename S::Work;
  constexpr int NWP = S::NWP;
  __shared__ unsigned int lds_cnt[MA_NACT + 1];
  for (int t = threadIdx.x; t < MA_NACT + 1; t += BS) lds_cnt[t] = 0;
  if (blockIdx.x == 0 && threadIdx.x == 0) atomicExch(&a.ctr[C_BIG], 0ull);   // (the previous chunk's list kernel is done)
  __syncthreads();
  const u64 tid = (u64)blockIdx.x * BS + threadIdx.x;
  const bool active = tid < a.chunk_count;
  const u64 gid = a.chunk_begin + tid, kbase = (a.rank0 + tid) * (u64)S::NSLOT;
  W s;
  if (active) {
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(a.states + gid * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    S::unpack(w, s);
  } else {
    S::init(s);
  }
  u32 err = 0, nsucc = 0, nin = 0, wcin = 0, wcoom = 0;
  u64 mcur = 0;
  int mwi = -1;
  // three loops (instances before Receive, Receive with its two successor slots, the rest): the
  // compile-time ranges prune apply's dispatch while keeping the kernel within short-branch range
  expand_group<S, S::G_RV, S::G_RECV, 1>(s, a, active, tid, err, nsucc, nin, lds_cnt, wcin, wcoom, mcur, mwi);
  expand_group<S, S::G_RECV, S::G_TO, 2>(s, a, active, tid, err, nsucc, nin, lds_cnt, wcin, wcoom, mcur, mwi);
  expand_group<S, S::G_TO, S::NI, 1>(s, a, active, tid, err, nsucc, nin, lds_cnt, wcin, wcoom, mcur, mwi);
  if (active && a.smask) a.smask[(u64)mwi * a.chunk_count + tid] = mcur;   // the last word
  unsigned long long ev = ~0ull;
  if (active) {
    a.nsucc[tid] = (unsigned short)nsucc;
    if (err & ME_EVAL) { const u64 e = (kbase << 2) | EV_NEXT_ERROR; ev = e < ev ? e : ev; }
    if (nsucc == 0 && a.deadlock) { const u64 e = (kbase << 2) | EV_DEADLOCK; ev = e < ev ? e : ev; }
    if (err & ME_CAP) {
      atomicOr(&a.ctr[C_ERR], (unsigned long long)ME_CAP);
      atomicCAS(&a.ctr[C_ERRGID], 0ull, (unsigned long long)(gid + 1));
    }
  }
  if (ev != ~0ull) atomicMin(&a.ctr[C_EVENT], ev);
  if (nin) atomicAdd(&lds_cnt[MA_NACT], nin);
  __syncthreads();
  for (int t = threadIdx.x; t < MA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[C_ACT + t], (unsigned long long)lds_cnt[t]);
  if (threadIdx.x == 0 && lds_cnt[MA_NACT]) atomicAdd(&a.ctr[C_GEN_IN], (unsigned long long)lds_cnt[MA_NACT]);
  if (__lane_id() == 0) {   // per wave: [in-model x 4 waves, out-of-model x 4 waves]
    a.cell_count[8 * blockIdx.x + (threadIdx.x >> 6)] = wcin;
    a.cell_count[8 * blockIdx.x + 4 + (threadIdx.x >> 6)] = wcoom;
  }
}

// Phase 2: one lane per in-model successor (full lanes): re-derive it and store its
// symmetric FP64 into its cell (cand[slot][state]).
// TLC = MC_COMPAT_SYM_TLC (a kernel of its own, so the orbit mode keeps its registers).
template <class S, bool TLC>
__global__ void __launch_bounds__(BS) memb_fingerprint(MGenArgs a) {
  using W = typename S::Work;
  constexpr int NWP = S::NWP;
  const CellRegions cr(a.cell_count + 8 * blockIdx.x, 64 * S::NSLOT);
  const u32 n = cr.n;
  const u32* cells = a.cells + (u64)blockIdx.x * (BS * S::NSLOT);
  for (u32 i = threadIdx.x; i < n; i += BS) {
  const u32 cell = cells[cr.at(i)];
  const u64 slot = cell / a.chunk_count, st = cell - slot * a.chunk_count;
  int k, sub;
  S::inst_of_slot((int)slot, k, sub);
  u32 w[NWP];
  const uint4* src = reinterpret_cast<const uint4*>(a.states + (a.chunk_begin + st) * NWP);
#pragma unroll
  for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
  W s, t;
  unsigned long long pt = RMC_PROF_T();
  S::unpack(w, s);
  u32 err = 0;
  S::template apply<TLC>(s, k, sub, t, err, a.rt);
  RMC_PROF_ADD(a.prof, 0, pt);
#ifdef RMC_FP_DUP_APPLY   // timing experiment: the re-derivation twice
  { W t2; u32 e2 = 0; int k2 = k; asm volatile("" : "+v"(k2)); S::template apply<TLC>(s, k2, sub, t2, e2, a.rt); asm volatile("" :: "v"((u32)t2.hr0), "v"(t2.term), "v"(e2)); }
#endif
  a.cand[cell] = TLC ? S::fingerprint_tlc(t, a.seed, a.rt, a.prof) : S::fingerprint_orbit(t, a.seed, a.rt);
  }
}

// TLC's symmetry rule (the drop-in default) at 3 waves per SIMD: the same fingerprints as
// memb_fingerprint<S, true>, with the bag out of the registers.  The parent's bag entries go from the
// store straight to the lane's LDS slice (sorted, non-empty ones only: C3 states carry 3 messages on
// average), the re-derivation leaves the bag change to the caller (S::apply_nobag) and it is made on
// the slice (S::slice_with_msg / slice_without_msg), and the symmetry search and the view hash read the
// slice (S::fingerprint_tlc_slice).  Each Work is then ~70 VGPRs smaller: 168 VGPRs and a 24-entry slice
// (48 KB of LDS per workgroup) give 3 waves per SIMD where memb_fingerprint's 240 VGPRs and 64-KB bag
// stage gave 2.  A parent whose bag could overflow the slice leaves its cell to memb_fingerprint_list.
template <class S>
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(3))) memb_fingerprint_lds(MGenArgs a) {
  using W = typename S::Work;
  constexpr int SL = S::MK + 1 < 24 ? S::MK + 1 : 24;   // slice entries: any parent bag that fits, plus one insertion
                                                        // (a.slice_cap <= SL - 1 of them hold the parent's)
  __shared__ u64 sbag[SL * BS];
  u64* const p = sbag + threadIdx.x;                    // lane-interleaved: entry q at p[q * BS]
  const CellRegions cr(a.cell_count + 8 * blockIdx.x, 64 * S::NSLOT);
  const u32 n = cr.n;
  const u32* cells = a.cells + (u64)blockIdx.x * (BS * S::NSLOT);
  for (u32 i = threadIdx.x; i < n; i += BS) {
    const u32 cell = cells[cr.at(i)];
    const u64 slot = cell / a.chunk_count, st = cell - slot * a.chunk_count;
    int k, sub;
    S::inst_of_slot((int)slot, k, sub);
    const uint2* src = reinterpret_cast<const uint2*>(a.states + (a.chunk_begin + st) * S::NWP);
    u32 w[S::BAGW];
#pragma unroll
    for (int q = 0; q < S::BAGW / 2; ++q) { const uint2 v = src[q]; w[2 * q] = v.x; w[2 * q + 1] = v.y; }
    int len = 0;
    bool big = false;
#pragma unroll 1
    for (int q = 0; q < S::MK; ++q) {   // packed entries are sorted, empty (0) ones last
      const uint2 v = src[S::BAGW / 2 + q];
      const u64 x = (u64)v.x | (u64)v.y << 32;
      if (!x) break;
      if (len < (int)a.slice_cap) p[len * BS] = x; else big = true;
      ++len;
    }
    if (big) { a.big[atomicAdd(&a.ctr[C_BIG], 1ull)] = cell; continue; }
    W s, t;
    S::unpack_nobag(w, s);
    const int bi = S::bag_slot_of(k);
    const u64 xent = bi >= 0 && bi < len ? p[bi * BS] : S::EMPTY;
    u32 err = 0;
    typename S::Delta d;
    S::template apply_nobag<true>(s, k, sub, xent, t, d, err, a.rt);
    if (d.a) S::slice_with_msg(p, BS, len, SL, d.add);
    if (d.r) S::slice_without_msg(p, BS, len, d.rem);
    a.cand[cell] = S::fingerprint_tlc_slice(t, p, BS, len, a.seed, a.rt);
  }
}

// The cells memb_fingerprint_lds left (a parent bag longer than its slice): memb_fingerprint's
// TLC-mode path, grid-stride over the list (its length on the device; usually none)
template <class S>
__global__ void __launch_bounds__(BS) memb_fingerprint_list(MGenArgs a) {
  using W = typename S::Work;
  constexpr int NWP = S::NWP;
  const u64 n = a.ctr[C_BIG];
  for (u64 i = (u64)blockIdx.x * BS + threadIdx.x; i < n; i += (u64)gridDim.x * BS) {
    const u32 cell = a.big[i];
    const u64 slot = cell / a.chunk_count, st = cell - slot * a.chunk_count;
    int k, sub;
    S::inst_of_slot((int)slot, k, sub);
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(a.states + (a.chunk_begin + st) * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    W s, t;
    S::unpack(w, s);
    u32 err = 0;
    S::template apply<true>(s, k, sub, t, err, a.rt);
    a.cand[cell] = S::fingerprint_tlc(t, a.seed, a.rt);
  }
}

// Out-of-model successors: TLC still checks the invariants on them ([ext] switch (ii)); the
// first violation / evaluation error in key order becomes the level's event.
template <class S>
#ifndef RMC_MOOM_WAVES
#define RMC_MOOM_WAVES 4   // memb_oom_check at 4 waves per SIMD (round 6, without the bag: 128 VGPRs, no spill)
#endif
__global__ void __launch_bounds__(BS) __attribute__((amdgpu_waves_per_eu(RMC_MOOM_WAVES))) memb_oom_check(MGenArgs a) {
  using W = typename S::Work;
  constexpr int NWP = S::NWP;
  const CellRegions cr(a.cell_count + 8 * blockIdx.x + 4, 64 * S::NSLOT);
  const u32 n = cr.n;
  const u32* cells = a.cells_oom + (u64)blockIdx.x * (BS * S::NSLOT);
  for (u32 i = threadIdx.x; i < n; i += BS) {
  const u32 cell = cells[cr.at(i)];
  const u64 slot = cell / a.chunk_count, st = cell - slot * a.chunk_count;
  int k, sub;
  S::inst_of_slot((int)slot, k, sub);
  // no invariant reads the bag: the parent's words before it and the one entry the instance reads
  const uint2* src = reinterpret_cast<const uint2*>(a.states + (a.chunk_begin + st) * NWP);
  u32 w[S::BAGW];
#pragma unroll
  for (int q = 0; q < S::BAGW / 2; ++q) { const uint2 v = src[q]; w[2 * q] = v.x; w[2 * q + 1] = v.y; }
  const int bi = S::bag_slot_of(k);
  u64 xent = S::EMPTY;
  if (bi >= 0) { const uint2 v = src[S::BAGW / 2 + bi]; const u64 x = (u64)v.x | (u64)v.y << 32; xent = x ? x : S::EMPTY; }
  W s, t;
  S::unpack_nobag(w, s);
  u32 err = 0;
  typename S::Delta d;
  S::template apply_nobag<false>(s, k, sub, xent, t, d, err, a.rt);
  const u32 r = S::check_invariants(t, a.rt);
  if (r) {
    const u64 e = (((a.rank0 + st) * (u64)S::NSLOT + slot) << 2) | ((r >> 8) == IV_BAD ? EV_VIOLATION : EV_INV_ERROR);
    atomicMin(&a.ctr[C_EVENT], (unsigned long long)e);
  }
  }
}

struct MDedupArgs {
  const u32* cells;            // the in-model cells, per expand workgroup and wave (memb_dedup_cells)
  const u32* cell_count;
  u64* cand;
  u64 nslots, chunk_count, rank0, nslot, level;
  u64* table;                  // [2 * slots] (fp, ~(level << 40 | key)); zero = empty
  u64 table_mask;
  unsigned long long* ctr;
};

// memb_dedup over the in-model cells only: workgroup b takes expand-workgroup b's cell lists, DPER_C
// cells in flight per thread (round 6: the cand array is no longer zeroed, dedup'd, selected and
// compacted densely over every (slot, state) -- ~2% of C3's slots hold a successor)
constexpr int DPER_C = 8;
__global__ void __launch_bounds__(BS) memb_dedup_cells(MDedupArgs a) {
  const CellRegions cr(a.cell_count + 8 * blockIdx.x, 64 * (u32)a.nslot);
  const u32 n = cr.n;
  const u32* cells = a.cells + (u64)blockIdx.x * (BS * a.nslot);
  u32 err = 0;
  for (u32 i0 = 0; i0 < n; i0 += BS * DPER_C) {
    u64 fp[DPER_C], cur[DPER_C], pos[DPER_C];
    u32 cell[DPER_C];
#pragma unroll
    for (int j = 0; j < DPER_C; ++j) {
      const u32 i = i0 + (u32)j * BS + threadIdx.x;
      cell[j] = i < n ? cells[cr.at(i)] : 0u;
      fp[j] = i < n ? a.cand[cell[j]] : 0ull;
      pos[j] = fp[j] & a.table_mask;
    }
#pragma unroll
    for (int j = 0; j < DPER_C; ++j) cur[j] = fp[j] ? a.table[2 * pos[j]] : ~0ull;
#pragma unroll
    for (int j = 0; j < DPER_C; ++j)
      if (fp[j] && cur[j] == 0ull)
        cur[j] = (u64)atomicCAS((unsigned long long*)&a.table[2 * pos[j]], 0ull, (unsigned long long)fp[j]);
#pragma unroll
    for (int j = 0; j < DPER_C; ++j) {
      if (!fp[j]) continue;
      if (cur[j] == 0ull || cur[j] == fp[j]) continue;          // inserted here, or already present
      u64 slot = (pos[j] + 1) & a.table_mask;
      for (int probe = 0;; ++probe) {
        if (probe >= (1 << 20)) { err |= MERR_TABLE_FULL; break; }
        const u64 c = a.table[2 * slot];
        if (c == fp[j]) break;
        if (c == 0ull) {
          const u64 old = (u64)atomicCAS((unsigned long long*)&a.table[2 * slot], 0ull, (unsigned long long)fp[j]);
          if (old == 0ull || old == fp[j]) break;
        }
        slot = (slot + 1) & a.table_mask;
      }
      pos[j] = slot;
    }
    // FIFO first-found: keep the minimum (level, key) per fingerprint (older levels always win)
#pragma unroll
    for (int j = 0; j < DPER_C; ++j) {
      if (!fp[j]) continue;
      const u64 sl = cell[j] / a.chunk_count, st = cell[j] - sl * a.chunk_count;
      const u64 key = (a.rank0 + st) * a.nslot + sl;
      atomicMax((unsigned long long*)&a.table[2 * pos[j] + 1], (unsigned long long)~((a.level << 40) | key));
      a.cand[cell[j]] = pos[j] + 1;
    }
  }
  if (err) atomicOr(&a.ctr[C_ERR], (unsigned long long)err);
}

struct MSelArgs {
  const u64* smask;            // [smw][chunk] in-model slots per state (memb_expand)
  u32 smw;
  u64* cand;
  u64 chunk_count, rank0, nslot, level;
  const u64* table;
  unsigned int* woff;          // [chunk] block-local exclusive offsets
  unsigned long long* bsum;    // [blocks] block totals
};

__global__ void __launch_bounds__(BS) memb_select(MSelArgs a) {
  __shared__ unsigned int wave_tot[BS / 64];
  const u64 tid = (u64)blockIdx.x * BS + threadIdx.x;
  const int lane = __lane_id(), wave = threadIdx.x >> 6;
  unsigned int mine = 0;
  if (tid < a.chunk_count) {
    const u64 kb = (a.rank0 + tid) * a.nslot;
    for (u32 w = 0; w < a.smw; ++w) {   // only the state's in-model slots
      u64 m = a.smask[(u64)w * a.chunk_count + tid];
      while (m) {
        const u64 sl = (u64)w * 64 + (u64)__builtin_ctzll(m);
        m &= m - 1;
        const u64 c = a.cand[sl * a.chunk_count + tid];
        const u64 want = ~((a.level << 40) | (kb + sl));
        if (a.table[2 * (c - 1) + 1] == want) { a.cand[sl * a.chunk_count + tid] = c | WINBIT; ++mine; }
      }
    }
  }
  unsigned int incl = mine;
#pragma unroll
  for (int d = 1; d < 64; d <<= 1) { const unsigned int v = __shfl_up(incl, d); if (lane >= d) incl += v; }
  if (lane == 63) wave_tot[wave] = incl;
  __syncthreads();
  unsigned int base = 0;
  for (int w = 0; w < wave; ++w) base += wave_tot[w];
  if (tid < a.chunk_count) a.woff[tid] = base + incl - mine;
  if (threadIdx.x == BS - 1) a.bsum[blockIdx.x] = base + incl;
}

// exclusive scan of up to SCAN_MAX_BLOCKS block totals in one workgroup; total -> ctr[C_NEW]
__global__ void __launch_bounds__(BS) memb_scan_blocks(unsigned long long* bsum, u32 nblocks, unsigned long long* ctr) {
  __shared__ unsigned long long part[BS];
  constexpr int PER = SCAN_MAX_BLOCKS / BS;
  unsigned long long v[PER], s = 0;
#pragma unroll
  for (int j = 0; j < PER; ++j) { const u32 b = threadIdx.x * PER + j; v[j] = b < nblocks ? bsum[b] : 0ull; s += v[j]; }
  part[threadIdx.x] = s;
  __syncthreads();
  for (int d = 1; d < BS; d <<= 1) {
    const unsigned long long x = threadIdx.x >= (unsigned)d ? part[threadIdx.x - d] : 0ull;
    __syncthreads();
    part[threadIdx.x] += x;
    __syncthreads();
  }
  unsigned long long run = part[threadIdx.x] - s;
#pragma unroll
  for (int j = 0; j < PER; ++j) { const u32 b = threadIdx.x * PER + j; if (b < nblocks) bsum[b] = run; run += v[j]; }
  if (threadIdx.x == BS - 1) ctr[C_NEW] = part[BS - 1];
}

struct MCompArgs {
  const u64* smask;
  u32 smw;
  const u64* cand;
  u64 chunk_count, chunk_begin, nslot;
  const unsigned int* woff;
  const unsigned long long* bsum;
  u64* newrec;                 // (parent gid << 10 | slot), key order
};

__global__ void __launch_bounds__(BS) memb_compact(MCompArgs a) {
  const u64 tid = (u64)blockIdx.x * BS + threadIdx.x;
  if (tid >= a.chunk_count) return;
  u64 o = a.bsum[blockIdx.x] + a.woff[tid];
  const u64 gid = a.chunk_begin + tid;
  for (u32 w = 0; w < a.smw; ++w) {   // in-model slots in slot order: the winners in key order
    u64 m = a.smask[(u64)w * a.chunk_count + tid];
    while (m) {
      const u64 sl = (u64)w * 64 + (u64)__builtin_ctzll(m);
      m &= m - 1;
      if (a.cand[sl * a.chunk_count + tid] & WINBIT) a.newrec[o++] = (gid << 10) | sl;
    }
  }
}

struct MMatArgs {
  u32* states;
  u64* meta;
  const u64* newrec;
  u64 n_new, dst_base, cap, level_begin;   // level_begin: store index of rank 0 of the level (mod 2^64)
  u64 gid_tag;                             // sharded: owner rank << 37, or-ed into parent pointers
  MembRuntime rt;
  unsigned long long* ctr;
};

template <class S, bool TLC>
__global__ void __launch_bounds__(BS) memb_materialize(MMatArgs a) {
  using W = typename S::Work;
  constexpr int NW = S::NW, NWP = S::NWP;
  __shared__ unsigned int lds_cnt[MA_NACT];
  for (int t = threadIdx.x; t < MA_NACT; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  u32 err = 0;
  unsigned long long ev = ~0ull;
  if (i < a.n_new) {
    const u64 rec = a.newrec[i], gid = rec >> 10;
    const int slot = (int)(rec & 1023);
    int k, sub;
    S::inst_of_slot(slot, k, sub);
    // the state without its bag in registers (round 6): the words before the bag and the one entry the
    // instance reads; the successor's bag goes from the parent's packed entries to the store in one merge
    // pass with the change (S::bag_merge), its other words packed (no invariant reads the bag)
    const u32* src = a.states + gid * NWP;
    u32 w[S::BAGW];
#pragma unroll
    for (int q = 0; q < S::BAGW / 2; ++q) { const uint2 v = reinterpret_cast<const uint2*>(src)[q]; w[2 * q] = v.x; w[2 * q + 1] = v.y; }
    const u64* pbag = reinterpret_cast<const u64*>(src + S::BAGW);
    const int bi = S::bag_slot_of(k);
    u64 xent = S::EMPTY;
    if (bi >= 0) { const u64 x = pbag[bi]; xent = x ? x : S::EMPTY; }
    W s, t;
    S::unpack_nobag(w, s);
    typename S::Delta d;
    const int act = S::template apply_nobag<TLC>(s, k, sub, xent, t, d, err, a.rt);
    const u64 dst = a.dst_base + i;
    if (act >= 0 && dst < a.cap) {
      u32 pw[S::BAGW];
      S::pack_nobag(t, pw);
      u32* o = a.states + dst * NWP;
#pragma unroll
      for (int q = 0; q < S::BAGW / 2; ++q) reinterpret_cast<uint2*>(o)[q] = make_uint2(pw[2 * q], pw[2 * q + 1]);
      S::bag_merge(pbag, reinterpret_cast<u64*>(o + S::BAGW), d, err);
#pragma unroll
      for (int q = NW; q < NWP; ++q) o[q] = 0u;
      a.meta[dst] = ((gid | a.gid_tag) << 20) | ((u64)act << 10) | (u64)slot;
      atomicAdd(&lds_cnt[act], 1u);
      const u32 r = S::check_invariants(t, a.rt);
      if (r) ev = ((((gid - a.level_begin) * (u64)S::NSLOT + (u64)slot)) << 2) | ((r >> 8) == IV_BAD ? EV_VIOLATION : EV_INV_ERROR);
    } else {
      err |= dst >= a.cap ? (u32)MERR_STORE : (u32)ME_CAP;
    }
  }
  if (err) atomicOr(&a.ctr[C_ERR], (unsigned long long)err);
  if (ev != ~0ull) atomicMin(&a.ctr[C_EVENT], ev);
  __syncthreads();
  for (int t = threadIdx.x; t < MA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&a.ctr[C_ACT + MA_NACT + t], (unsigned long long)lds_cnt[t]);
}

// TLC's per-action counters at a stop point (oracle/engine.h: a parent's successors are counted in
// enumeration order up to the event's own successor; a next-state error counts none of the
// parent's).  Parents [0, n) of a level range starting at gid `first`; parent `stop` is the event's
// (n = stop + 1 when the event is in this range, else every parent counts whole).
template <class S, int K0, int K1, int NS>
__device__ __forceinline__ void stop_group(typename S::Work& s, const MembRuntime& rt, bool whole, int stop_slot, u32& err,
                                           unsigned int* lds_cnt) {
  using W = typename S::Work;
  for (int k = K0; k < K1; ++k) {
    const bool en = S::group_enabled(k, rt.next);                     // wave-uniform
    for (int sub = 0; sub < NS; ++sub) {
      if (!en) continue;
      S::launder(s);
      W t;
      const int act = S::template apply<false>(s, k, sub, t, err, rt);
      const int slot = S::slot_of(k, sub);
      if (act >= 0 && (whole || slot <= stop_slot)) {
        // a successor's TLC copies follow it in TLC's order: counted unless it is the event itself
        const int cp = (act == MA_HandleCheckOldConfig || act == MA_HandleCatchupResponse) ? S::tlc_copies(s, k, sub, rt) : 1;
        atomicAdd(&lds_cnt[act], (whole || slot < stop_slot) ? (unsigned)cp : 1u);
      }
    }
  }
}
template <class S>
__global__ void __launch_bounds__(BS) memb_stop_generated(const u32* states, u64 first, u64 n, u64 stop, int stop_slot, u32 kind,
                                                          MembRuntime rt, unsigned long long* out) {
  using W = typename S::Work;
  constexpr int NWP = S::NWP;
  __shared__ unsigned int lds_cnt[MA_NACT];
  for (int t = threadIdx.x; t < MA_NACT; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  const bool active = i < n && !(i == stop && kind == EV_NEXT_ERROR);
  W s;
  if (active) {
    u32 w[NWP];
    const uint4* src = reinterpret_cast<const uint4*>(states + (first + i) * NWP);
#pragma unroll
    for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
    S::unpack(w, s);
  } else {
    S::init(s);
  }
  u32 err = 0;
  if (active) {   // (active is per lane; the groups' loops are wave-uniform, inactive lanes idle)
    const bool whole = i < stop;
    stop_group<S, S::G_RV, S::G_RECV, 1>(s, rt, whole, stop_slot, err, lds_cnt);
    stop_group<S, S::G_RECV, S::G_TO, 2>(s, rt, whole, stop_slot, err, lds_cnt);
    stop_group<S, S::G_TO, S::NI, 1>(s, rt, whole, stop_slot, err, lds_cnt);
  }
  __syncthreads();
  for (int t = threadIdx.x; t < MA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&out[t], (unsigned long long)lds_cnt[t]);
}
// per-action distinct counts of n stored new states (their meta: parent << 20 | action << 10 | slot)
__global__ void __launch_bounds__(BS) memb_stop_distinct(const u64* meta, u64 n, unsigned long long* out) {
  __shared__ unsigned int lds_cnt[MA_NACT];
  for (int t = threadIdx.x; t < MA_NACT; t += BS) lds_cnt[t] = 0;
  __syncthreads();
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i < n) atomicAdd(&lds_cnt[((meta[i] >> 10) & 1023) % MA_NACT], 1u);
  __syncthreads();
  for (int t = threadIdx.x; t < MA_NACT; t += BS)
    if (lds_cnt[t]) atomicAdd(&out[t], (unsigned long long)lds_cnt[t]);
}

// Recovery from a checkpoint (TLC -recover): the fingerprints of the stored states [0, n) go back
// into the zeroed seen-set.  Their side value is ~0 (level 0, key 0): every stored state belongs to
// a completed level, so it beats any successor of the levels still to come, exactly as its own
// (older-level) entry did before the checkpoint.
template <class S, bool TLC>
__global__ void __launch_bounds__(BS) memb_reinsert(const u32* states, u64 n, u64 seed, MembRuntime rt, u64* table,
                                                    u64 table_mask, unsigned long long* ctr) {
  using W = typename S::Work;
  constexpr int NWP = S::NWP;
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  u32 w[NWP];
  const uint4* src = reinterpret_cast<const uint4*>(states + i * NWP);
#pragma unroll
  for (int q = 0; q < NWP / 4; ++q) { const uint4 v = src[q]; w[4 * q] = v.x; w[4 * q + 1] = v.y; w[4 * q + 2] = v.z; w[4 * q + 3] = v.w; }
  W s;
  S::unpack(w, s);
  const u64 fp = TLC ? S::fingerprint_tlc(s, seed, rt) : S::fingerprint_orbit(s, seed, rt);
  u64 slot = fp & table_mask;
  for (int probe = 0;; ++probe) {
    if (probe >= (1 << 20)) { atomicOr(&ctr[C_ERR], (unsigned long long)MERR_TABLE_FULL); return; }
    const u64 old = (u64)atomicCAS((unsigned long long*)&table[2 * slot], 0ull, (unsigned long long)fp);
    if (old == 0ull || old == fp) break;
    slot = (slot + 1) & table_mask;
  }
  table[2 * slot + 1] = ~0ull;
}

// ------------------------------------------------------------------ sharded (multi-GPU) kernels
// FIFO first-found across ranks: keys are global (global parent rank * NSLOT + slot),
// every fingerprint has one owner ((fp >> 32) mod world) whose seen-set entry keeps the minimum
// key of the level; after all chunks the owner sends each winning key back to the rank that
// generated it, which re-derives its winners in key order.
constexpr int RPER = 16;   // slots / records per thread in the bucketing kernels

struct MRouteArgs {
  const u64* cand;             // [NSLOT][chunk] fingerprints, 0 = none
  u64 nslots, chunk_count, rank0, nslot;
  u32 world;
  unsigned long long* counts;  // [world]: count pass totals / write pass cursors
  u64* out;                    // write pass: (fp, key) records, per-owner segments
};
RMC_HD u32 fp_owner(u64 fp, u32 world) { return (u32)((fp >> 32) % world); }

// per-owner bucketing in two passes (count, then write at reserved cursors); one global atomic
// per (workgroup, owner)
template <bool WRITE>
__global__ void __launch_bounds__(BS) memb_route(MRouteArgs a) {
  __shared__ unsigned int cnt[8], base[8];
  if (threadIdx.x < 8) cnt[threadIdx.x] = 0;
  __syncthreads();
  const u64 tile = (u64)blockIdx.x * (BS * RPER);
  u64 fp[RPER];
  unsigned int off[RPER];
#pragma unroll
  for (int j = 0; j < RPER; ++j) {
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    fp[j] = idx < a.nslots ? a.cand[idx] : 0ull;
    off[j] = fp[j] ? atomicAdd(&cnt[fp_owner(fp[j], a.world)], 1u) : 0u;
  }
  __syncthreads();
  if (threadIdx.x < a.world) {
    const unsigned int c = cnt[threadIdx.x];
    base[threadIdx.x] = c ? (unsigned int)atomicAdd(&a.counts[threadIdx.x], (unsigned long long)c) : 0u;
  }
  if (!WRITE) return;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPER; ++j) {
    if (!fp[j]) continue;
    const u64 idx = tile + (u64)j * BS + threadIdx.x;
    const u64 sl = idx / a.chunk_count, st = idx - sl * a.chunk_count;
    const u64 o = (u64)base[fp_owner(fp[j], a.world)] + off[j];
    a.out[2 * o] = fp[j];
    a.out[2 * o + 1] = (a.rank0 + st) * a.nslot + sl;
  }
}

struct MDedupShArgs {
  const u64* recv;             // (fp, key) records
  u64 n, level;
  u64* table;
  u64 table_mask;
  u64* lvl;                    // level records out: (table position + 1, key)
  unsigned long long* ctr;
};

// owner side: insert-if-absent, keep the minimum (level, key); remember (position, key) for select
__global__ void __launch_bounds__(BS) memb_dedup_sh(MDedupShArgs a) {
  const u64 tile = (u64)blockIdx.x * (BS * DPER);
  u64 fp[DPER], key[DPER], cur[DPER], pos[DPER];
#pragma unroll
  for (int j = 0; j < DPER; ++j) {
    const u64 i = tile + (u64)j * BS + threadIdx.x;
    fp[j] = i < a.n ? a.recv[2 * i] : 0ull;
    key[j] = i < a.n ? a.recv[2 * i + 1] : 0ull;
    pos[j] = fp[j] & a.table_mask;
  }
#pragma unroll
  for (int j = 0; j < DPER; ++j) cur[j] = fp[j] ? a.table[2 * pos[j]] : ~0ull;
#pragma unroll
  for (int j = 0; j < DPER; ++j)
    if (fp[j] && cur[j] == 0ull)
      cur[j] = (u64)atomicCAS((unsigned long long*)&a.table[2 * pos[j]], 0ull, (unsigned long long)fp[j]);
  u32 err = 0;
#pragma unroll
  for (int j = 0; j < DPER; ++j) {
    if (!fp[j]) continue;
    if (cur[j] == 0ull || cur[j] == fp[j]) continue;
    u64 slot = (pos[j] + 1) & a.table_mask;
    for (int probe = 0;; ++probe) {
      if (probe >= (1 << 20)) { err |= MERR_TABLE_FULL; break; }
      const u64 c = a.table[2 * slot];
      if (c == fp[j]) break;
      if (c == 0ull) {
        const u64 old = (u64)atomicCAS((unsigned long long*)&a.table[2 * slot], 0ull, (unsigned long long)fp[j]);
        if (old == 0ull || old == fp[j]) break;
      }
      slot = (slot + 1) & a.table_mask;
    }
    pos[j] = slot;
  }
#pragma unroll
  for (int j = 0; j < DPER; ++j) {
    if (!fp[j]) continue;
    const u64 i = tile + (u64)j * BS + threadIdx.x;
    atomicMax((unsigned long long*)&a.table[2 * pos[j] + 1], (unsigned long long)~((a.level << 40) | key[j]));
    a.lvl[2 * i] = pos[j] + 1;
    a.lvl[2 * i + 1] = key[j];
  }
  if (err) atomicOr(&a.ctr[C_ERR], (unsigned long long)err);
}

struct MSelShArgs {
  const u64* lvl;              // (position + 1, key) of the level
  u64 n, level;
  const u64* table;
  u64 kstart[8];               // first key of each generating rank's range (kstart[0] = 0)
  u32 world;
  unsigned long long* counts;  // [world]: count pass totals / write pass cursors
  u64* out;                    // write pass: winning keys, per-generator segments
};

// owner side, after every chunk of the level: the winners (entry still holds this level's key)
// bucketed by the rank that generated them
template <bool WRITE>
__global__ void __launch_bounds__(BS) memb_select_sh(MSelShArgs a) {
  __shared__ unsigned int cnt[8], base[8];
  if (threadIdx.x < 8) cnt[threadIdx.x] = 0;
  __syncthreads();
  const u64 tile = (u64)blockIdx.x * (BS * RPER);
  u64 key[RPER];
  unsigned int off[RPER], gen[RPER];
  bool win[RPER];
#pragma unroll
  for (int j = 0; j < RPER; ++j) {
    const u64 i = tile + (u64)j * BS + threadIdx.x;
    win[j] = false; key[j] = 0; gen[j] = 0; off[j] = 0;
    if (i < a.n) {
      const u64 p = a.lvl[2 * i] - 1;
      key[j] = a.lvl[2 * i + 1];
      win[j] = a.table[2 * p + 1] == ~((a.level << 40) | key[j]);
      u32 g = 0;
#pragma unroll
      for (int q = 1; q < 8; ++q) if ((u32)q < a.world && key[j] >= a.kstart[q]) g = (u32)q;
      gen[j] = g;
      if (win[j]) off[j] = atomicAdd(&cnt[g], 1u);
    }
  }
  __syncthreads();
  if (threadIdx.x < a.world) {
    const unsigned int c = cnt[threadIdx.x];
    base[threadIdx.x] = c ? (unsigned int)atomicAdd(&a.counts[threadIdx.x], (unsigned long long)c) : 0u;
  }
  if (!WRITE) return;
  __syncthreads();
#pragma unroll
  for (int j = 0; j < RPER; ++j)
    if (win[j]) a.out[(u64)base[gen[j]] + off[j]] = key[j];
}

// generating side: sorted winning keys -> (parent store index << 10 | slot) for memb_materialize
__global__ void __launch_bounds__(BS) memb_keys_to_newrec(const u64* keys, u64 n, u64 nslot, u64 rank_base, u64 level_begin,
                                                         u64* newrec) {
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  const u64 k = keys[i], r = k / nslot;
  newrec[i] = ((r - rank_base + level_begin) << 10) | (k - r * nslot);
}

// STATES records (packed state words, parent meta) <-> the store
template <int NWP>
__global__ void __launch_bounds__(BS) memb_pack_states(const u32* states, const u64* meta, u64 first, u64 n, u32* out) {
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  constexpr int RW = NWP + 2;
  const uint4* src = reinterpret_cast<const uint4*>(states + (first + i) * NWP);
#pragma unroll
  for (int q = 0; q < NWP / 4; ++q) {
    const uint4 v = src[q];
    out[i * RW + 4 * q] = v.x; out[i * RW + 4 * q + 1] = v.y; out[i * RW + 4 * q + 2] = v.z; out[i * RW + 4 * q + 3] = v.w;
  }
  const u64 m = meta[first + i];
  out[i * RW + NWP] = (u32)m; out[i * RW + NWP + 1] = (u32)(m >> 32);
}
template <int NWP>
__global__ void __launch_bounds__(BS) memb_unpack_states(const u32* in, u64 n, u64 first, u32* states, u64* meta) {
  const u64 i = (u64)blockIdx.x * BS + threadIdx.x;
  if (i >= n) return;
  constexpr int RW = NWP + 2;
  uint4* dst = reinterpret_cast<uint4*>(states + (first + i) * NWP);
#pragma unroll
  for (int q = 0; q < NWP / 4; ++q)
    dst[q] = make_uint4(in[i * RW + 4 * q], in[i * RW + 4 * q + 1], in[i * RW + 4 * q + 2], in[i * RW + 4 * q + 3]);
  meta[first + i] = (u64)in[i * RW + NWP] | ((u64)in[i * RW + NWP + 1] << 32);
}

#define HIPCHK(x)                                                                             \
  do {                                                                                        \
    hipError_t e_ = (x);                                                                      \
    if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); return MC_E_NO_DEVICE; } \
  } while (0)

template <class S>
class MembGpu : public Backend {
 public:
  using W = typename S::Work;
  static constexpr int NWP = S::NWP;
  explicit MembGpu(const MembModel& m) : m_(m), text_(m_) {}
  ~MembGpu() override { release(); }

  // ---- punctuated-search prefixes (memb_prefix.h): region 0 CommitWhenConcurrentLeaders_unique,
  // region 1 MajorityOfClusterRestarts_constraint
  std::vector<std::string> history_prefixes_needed() const override {
    std::vector<std::string> v;
    for (int r = 0; r < 2; ++r)
      if ((m_.rt.constraints >> kPrefixCon[r]) & 1u) v.push_back(kMembConNames[kPrefixCon[r]]);
    return v;
  }
  int set_history_prefix(const std::string& con, const TVal& trace, std::string& err) override {
    int r = -1;
    for (int q = 0; q < 2; ++q) if (con == kMembConNames[kPrefixCon[q]]) r = q;
    if (r < 0) { err = "'" + con + "' is not a punctuated-search prefix constraint"; return MC_E_INVALID; }
    try {
      const auto& g = trace_global(trace);
      if (g.size() > 1000) { err = "history prefix longer than the 10-bit history length field"; return MC_E_UNSUPPORTED; }
      int unmatched = 0;
      ptab_[r] = encode_prefix_table<S>(m_, g, &unmatched);
      plen_[r] = (u32)g.size();
      have_prefix_[r] = true;
    } catch (const CfgError& e) { err = e.what(); return e.code; }
    return 0;
  }
  // runtime descriptors with the prefix tables: host copies for host-side re-derivation, device
  // copies for the kernels
  int prepare_prefixes(std::string& err) {
    rt_host_ = m_.rt; rt_dev_ = m_.rt;
    u32 off = S::H_PREFIX;
    for (int r = 0; r < 2; ++r) {
      if (!((m_.rt.constraints >> kPrefixCon[r]) & 1u)) continue;
      if (!have_prefix_[r]) {
        err = std::string(kMembConNames[kPrefixCon[r]]) + " needs its golden history trace: place the reference's "
              "raft.tla next to the module, or pass the trace with mc_set_history_prefix";
        return MC_E_UNSUPPORTED;
      }
      if (off + S::NB > 64) { err = "both punctuated-search prefix constraints at once do not fit the history word for this |Server|"; return MC_E_UNSUPPORTED; }
      if (r == 1) rt_host_.preg1_off = rt_dev_.preg1_off = off;
      off += S::NB;
      if (d_ptab_[r]) { (void)hipFree(d_ptab_[r]); d_ptab_[r] = nullptr; }
      const size_t bytes = std::max<size_t>(16, ptab_[r].size() * 8);
      HIPCHK(hipMalloc(&d_ptab_[r], bytes));
      if (!ptab_[r].empty()) HIPCHK(hipMemcpy(d_ptab_[r], ptab_[r].data(), ptab_[r].size() * 8, hipMemcpyHostToDevice));
      const u32 len = plen_[r] ? plen_[r] : 0;
      if (r == 0) { rt_host_.ptab0 = ptab_[0].data(); rt_dev_.ptab0 = d_ptab_[0]; rt_host_.plen0 = rt_dev_.plen0 = len; }
      else { rt_host_.ptab1 = ptab_[1].data(); rt_dev_.ptab1 = d_ptab_[1]; rt_host_.plen1 = rt_dev_.plen1 = len; }
    }
    return 0;
  }

  std::string family() const override { return "tlc_membership"; }

  int observed_collision(double& v, std::string& err) override {
    if (!d_table_ || sharded_) { err = "after a single-GPU mc_run only"; return MC_E_STATE; }
    return fpgap::observed(d_table_, table_mask_ + 1, 2, stream_, v, err);
  }

  std::string describe_json() const override {
    std::ostringstream o;
    o << "{\"spec\": \"tlc_membership\", \"N\": " << S::N << ", \"NV\": " << S::NV << ", \"MK\": " << S::MK
      << ", \"next\": \"" << m_.next_name << "\", \"symmetry\": " << (m_.rt.symmetry ? "true" : "false")
      << ", \"permutations\": " << (m_.rt.symmetry ? S::NPERM : 1) << ", \"view\": \"vars\", \"init_server_mask\": " << m_.rt.init_cfg
      << ", \"num_rounds\": " << m_.rt.num_rounds << ", \"state_words\": " << S::NW << ", \"state_bytes_stored\": " << NWP * 4
      << ", \"instances\": " << S::NI << ", \"slots\": " << S::NSLOT << ", \"constraints\": [";
    for (size_t k = 0; k < m_.constraint_names.size(); ++k) o << (k ? ", " : "") << "\"" << m_.constraint_names[k] << "\"";
    o << "], \"action_constraints\": [";
    for (size_t k = 0; k < m_.action_constraint_names.size(); ++k) o << (k ? ", " : "") << "\"" << m_.action_constraint_names[k] << "\"";
    o << "], \"history_prefixes\": {";
    bool first = true;
    for (int q = 0; q < 2; ++q)
      if ((m_.rt.constraints >> kPrefixCon[q]) & 1u) {
        o << (first ? "" : ", ") << "\"" << kMembConNames[kPrefixCon[q]] << "\": " << (have_prefix_[q] ? (int)plen_[q] : -1);
        first = false;
      }
    o << "}, \"prefix_bindings\": " << S::NB << ", \"invariants\": [";
    for (size_t k = 0; k < m_.inv_names.size(); ++k) o << (k ? ", " : "") << "\"" << m_.inv_names[k] << "\"";
    o << "], \"actions\": [";
    for (int k = 0; k < MA_NACT; ++k) o << (k ? ", " : "") << "\"" << kMembActNames[k] << "\"";
    o << "]}";
    return o.str();
  }

  int ensure_alloc(const RunOpts& o, std::string& err) {
    int ndev = 0;
    if (hipGetDeviceCount(&ndev) != hipSuccess || ndev <= o.device) { err = "no HIP device available (raftmc has no CPU fallback)"; return MC_E_NO_DEVICE; }
    HIPCHK(hipSetDevice(o.device));
    if (d_table_ && o.device == dev_ && o.fp_table_bytes == req_table_ && o.state_store_bytes == req_store_) return 0;
    release();
    size_t freeb = 0, totalb = 0;
    HIPCHK(hipMemGetInfo(&freeb, &totalb));
    // defaults sized for one 288 GB MI355X: seen-set ~1/8 of free HBM (16-B entries), state store ~1/2
    const uint64_t tb = o.fp_table_bytes ? o.fp_table_bytes : std::min<uint64_t>(32ull << 30, freeb / 8);
    uint64_t slots = 1; while (slots * 2 * 16 <= tb) slots *= 2;
    if (slots < 1024) slots = 1024;
    const uint64_t sb = o.state_store_bytes ? o.state_store_bytes : std::min<uint64_t>(160ull << 30, freeb / 2);
    cap_ = std::max<u64>(16, sb / (NWP * 4 + 8));
    // chunk: cand + newrec hold NSLOT u64 per state; ~1/8 of the store bytes, <= SCAN_MAX_BLOCKS blocks
    chunk_ = std::max<u64>(BS, std::min<u64>({cap_, (sb / 8) / (16 * (u64)S::NSLOT), (u64)SCAN_MAX_BLOCKS * BS}));
    chunk_ = (chunk_ / BS) * BS;
    table_mask_ = slots - 1;
    HIPCHK(hipMalloc(&d_table_, slots * 16));
    HIPCHK(hipMalloc(&d_states_, cap_ * NWP * 4));
    HIPCHK(hipMalloc(&d_meta_, cap_ * 8));
    HIPCHK(hipMalloc(&d_cand_, chunk_ * S::NSLOT * 8));
    HIPCHK(hipMalloc(&d_newrec_, chunk_ * S::NSLOT * 8));
    HIPCHK(hipMalloc(&d_nsucc_, chunk_ * 2));
    HIPCHK(hipMalloc(&d_cells_, chunk_ * S::NSLOT * 4));
    HIPCHK(hipMalloc(&d_cells_oom_, chunk_ * S::NSLOT * 4));
    HIPCHK(hipMalloc(&d_cell_count_, 8 * ((chunk_ + BS - 1) / BS) * 4));
    HIPCHK(hipMalloc(&d_big_, chunk_ * S::NSLOT * 4));
    HIPCHK(hipMalloc(&d_smask_, chunk_ * SMW * 8));
    HIPCHK(hipMalloc(&d_woff_, chunk_ * 4));
    HIPCHK(hipMalloc(&d_bsum_, SCAN_MAX_BLOCKS * 8));
    HIPCHK(hipMalloc(&d_ctr_, C_NCTR * 8));
    HIPCHK(hipStreamCreateWithFlags(&stream_, hipStreamNonBlocking));
    for (auto& e : ev_) HIPCHK(hipEventCreate(&e));
    dev_ = o.device; req_table_ = o.fp_table_bytes; req_store_ = o.state_store_bytes;
    return 0;
  }

  float ms(int a, int b) { float x = 0; (void)hipEventElapsedTime(&x, ev_[a], ev_[b]); return x; }

  int run(const RunOpts& o, RunResult& r, std::string& err) override {
    sharded_ = false;
    for (int q = 0; q < 2; ++q)
      if (((m_.rt.constraints >> kPrefixCon[q]) & 1u) && !have_prefix_[q]) {
        err = std::string(kMembConNames[kPrefixCon[q]]) + " needs its golden history trace: place the reference's "
              "raft.tla next to the module, or pass the trace with mc_set_history_prefix";
        return MC_E_UNSUPPORTED;
      }
    if (int rc = ensure_alloc(o, err)) return rc;
    if (int rc = prepare_prefixes(err)) return rc;
    rt_host_.sym_tlc = rt_dev_.sym_tlc = (o.sym_tlc && m_.rt.symmetry) ? 1u : 0u;
    fp_slice_test_ = o.test_fp_slice;
    rt_host_.disjunct_copies = rt_dev_.disjunct_copies = o.disjunct_copies ? 1u : 0u;
    auto t0 = std::chrono::steady_clock::now();
    HIPCHK(hipMemsetAsync(d_table_, 0, (table_mask_ + 1) * 16, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    r = RunResult();
    r.seed = o.seed ? o.seed : 0x5EED5EED2024ull;
    r.state_bytes = NWP * 4;
    for (int k = 0; k < MA_NACT; ++k) r.action_names.push_back(kMembActNames[k]);
    r.act_generated.assign(MA_NACT, 0); r.act_distinct.assign(MA_NACT, 0);
    r.kernels = {{"memb_expand", 0, 0, 0}, {"memb_fingerprint", 0, 0, 0}, {"memb_dedup", 0, 0, 0},
                 {"memb_select", 0, 0, 0}, {"memb_compact", 0, 0, 0}, {"memb_materialize", 0, 0, 0}};
    const MembRuntime& rt = rt_host_;
    base_ = 0; host_.clear();
    u64 level_begin = 0, level_count = 1;
    u32 level = 0;

    if (!o.recover_path.empty()) {   // TLC -recover: continue the BFS saved by a checkpoint
      if (int rc = load_checkpoint(o.recover_path, r, level_begin, level_count, err)) return rc;
      level = (u32)(r.depth - 1);
    } else {
    // ---- Init (raft.tla:388-393): generated 1; constraints; invariants (TLC checks them on initial states)
    W s0; S::init(s0);
    r.generated = 1; r.depth = 1;
    r.levels.push_back({1, 0, 0.0});
    total_ = 0;
    if (!S::in_model(s0, s0, rt)) { r.distinct = 0; r.depth = 0; finish(r, t0); return 0; }
    {
      u32 w0[S::NW]; S::pack(s0, w0);
      u32 wp[NWP] = {0}; for (int q = 0; q < S::NW; ++q) wp[q] = w0[q];
      const u64 fp0 = S::fingerprint(s0, r.seed, rt);
      u64 e2[2] = {fp0, ~0ull};   // level 0, key 0: the stored side value is ~(0 << 40 | 0)
      HIPCHK(hipMemcpy(d_table_ + 2 * (fp0 & table_mask_), e2, 16, hipMemcpyHostToDevice));
      HIPCHK(hipMemcpy(d_states_, wp, NWP * 4, hipMemcpyHostToDevice));
      const u64 nometa = ~0ull;
      HIPCHK(hipMemcpy(d_meta_, &nometa, 8, hipMemcpyHostToDevice));
      total_ = 1; r.distinct = 1;
      if (u32 bad = S::check_invariants(s0, rt)) {
        if ((bad >> 8) == IV_BAD) { r.verdict = MC_VERDICT_INVARIANT_VIOLATION; r.violated = kMembInvNames[bad & 255]; }
        else { r.verdict = MC_VERDICT_EVAL_ERROR; r.error = std::string("TLC evaluation error in invariant ") + kMembInvNames[bad & 255]; }
        r.trace.push_back({"<Initial predicate>", text_.text(s0, true)});
        finish(r, t0); return 0;
      }
    }
    }

    const u64 S_B = NWP * 4;
    while (level_count > 0) {
      if (o.max_depth && r.depth >= o.max_depth) { r.left_on_queue = (int64_t)level_count; r.verdict = MC_VERDICT_DEPTH_LIMIT; break; }
      // the device keeps what the search still reads (the frontier) and writes (the next level);
      // when the next level, predicted from the last growth ratio with a 1.5x margin, might not
      // fit behind what is stored, the completed levels move to host memory
      if (level_begin > base_) {
        const double prev = r.levels.size() >= 2 ? (double)r.levels[r.levels.size() - 2].states : 1.0;
        const double pred = (double)level_count * std::max(1.0, (double)level_count / std::max(prev, 1.0)) * 1.5;
        if ((double)(total_ - base_) + pred > (double)cap_)
          if (int rc = spill(level_begin, level_count, err)) return rc;
      }
      // kernels index the store by global id: the device part holds [base_, base_ + cap_)
      u32* const sp = d_states_ - base_ * NWP;
      u64* const mp = d_meta_ - base_;
      const u64 cap_end = base_ + cap_;
      HIPCHK(hipMemsetAsync(d_ctr_, 0, C_NCTR * 8, stream_));
      HIPCHK(hipMemsetAsync(d_ctr_ + C_EVENT, 0xFF, 8, stream_));
      u64 next_write = level_begin + level_count;
      double level_ms = 0;
      int64_t gen_before_chunk = 0;       // generated in earlier chunks of this level
      std::vector<u64> act_before_chunk(2 * MA_NACT, 0);   // per-action generated / distinct in earlier chunks
      u64 gen_in_level = 0;               // in-model successors of this level (G_in)
      u64 gin_seen = 0;                   // ... counted up to the previous chunk
      u64 c[C_NCTR] = {0};
      bool stop = false;
      for (u64 cb = level_begin; cb < level_begin + level_count; cb += chunk_) {
        const u64 cnt = std::min<u64>(chunk_, level_begin + level_count - cb), rank0 = cb - level_begin;
        const u64 nslots = cnt * (u64)S::NSLOT;
        const u32 nblk = (u32)((cnt + BS - 1) / BS);
        MGenArgs g;
        g.states = sp; g.chunk_begin = cb; g.chunk_count = cnt; g.rank0 = rank0; g.cand = d_cand_; g.cells = d_cells_;
        g.cells_oom = d_cells_oom_; g.cell_count = d_cell_count_; g.nsucc = d_nsucc_;
        g.seed = r.seed; g.rt = rt_dev_; g.inv_oom = o.inv_out_of_model ? 1u : 0u; g.deadlock = o.check_deadlock ? 1u : 0u; g.ctr = (unsigned long long*)d_ctr_;
        g.smask = d_smask_;
        MDedupArgs d;
        d.cells = d_cells_; d.cell_count = d_cell_count_;
        d.cand = d_cand_; d.nslots = nslots; d.chunk_count = cnt; d.rank0 = rank0; d.nslot = S::NSLOT; d.level = level + 1;
        d.table = d_table_; d.table_mask = table_mask_; d.ctr = (unsigned long long*)d_ctr_;
        MSelArgs sa;
        sa.smask = d_smask_; sa.smw = (u32)SMW;
        sa.cand = d_cand_; sa.chunk_count = cnt; sa.rank0 = rank0; sa.nslot = S::NSLOT; sa.level = level + 1; sa.table = d_table_;
        sa.woff = d_woff_; sa.bsum = (unsigned long long*)d_bsum_;
        MCompArgs ca;
        ca.smask = d_smask_; ca.smw = (u32)SMW;
        ca.cand = d_cand_; ca.chunk_count = cnt; ca.chunk_begin = cb; ca.nslot = S::NSLOT; ca.woff = d_woff_;
        ca.bsum = (const unsigned long long*)d_bsum_; ca.newrec = d_newrec_;
        HIPCHK(hipEventRecord(ev_[7], stream_));
        hipLaunchKernelGGL((memb_expand<S>), dim3(nblk), dim3(BS), 0, stream_, g);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev_[8], stream_));
        if (o.inv_out_of_model) hipLaunchKernelGGL((memb_oom_check<S>), dim3(nblk), dim3(BS), 0, stream_, g);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev_[0], stream_));
        if (int rc = launch_fingerprint(g, nblk, err)) return rc;
        HIPCHK(hipEventRecord(ev_[1], stream_));
        hipLaunchKernelGGL(memb_dedup_cells, dim3(nblk), dim3(BS), 0, stream_, d);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev_[2], stream_));
        hipLaunchKernelGGL(memb_select, dim3(nblk), dim3(BS), 0, stream_, sa);
        HIPCHK(hipGetLastError());
        hipLaunchKernelGGL(memb_scan_blocks, dim3(1), dim3(BS), 0, stream_, (unsigned long long*)d_bsum_, nblk, (unsigned long long*)d_ctr_);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev_[3], stream_));
        hipLaunchKernelGGL(memb_compact, dim3(nblk), dim3(BS), 0, stream_, ca);
        HIPCHK(hipGetLastError());
        HIPCHK(hipEventRecord(ev_[4], stream_));
        u64 nnew = 0;
        HIPCHK(hipMemcpyAsync(&nnew, d_ctr_ + C_NEW, 8, hipMemcpyDeviceToHost, stream_));
        HIPCHK(hipStreamSynchronize(stream_));
        const float ms_x = ms(7, 8), ms_g = ms(0, 1), ms_d = ms(1, 2), ms_s = ms(2, 3), ms_c = ms(3, 4);

        float ms_m = 0;
        if (nnew && next_write + nnew <= cap_end) {
          MMatArgs m;
          m.states = sp; m.meta = mp; m.newrec = d_newrec_; m.n_new = nnew; m.dst_base = next_write; m.cap = cap_end;
          m.level_begin = level_begin; m.gid_tag = 0; m.rt = rt_dev_; m.ctr = (unsigned long long*)d_ctr_;
          HIPCHK(hipEventRecord(ev_[5], stream_));
          if (rt_dev_.sym_tlc) hipLaunchKernelGGL((memb_materialize<S, true>), dim3((unsigned)((nnew + BS - 1) / BS)), dim3(BS), 0, stream_, m);
          else hipLaunchKernelGGL((memb_materialize<S, false>), dim3((unsigned)((nnew + BS - 1) / BS)), dim3(BS), 0, stream_, m);
          HIPCHK(hipGetLastError());
          HIPCHK(hipEventRecord(ev_[6], stream_));
          HIPCHK(hipEventSynchronize(ev_[6]));
          ms_m = ms(5, 6);
        }
        HIPCHK(hipMemcpyAsync(c, d_ctr_, sizeof c, hipMemcpyDeviceToHost, stream_));
        HIPCHK(hipStreamSynchronize(stream_));
        level_ms += ms_x + ms_g + ms_d + ms_s + ms_c + ms_m;
        const u64 ncells = c[C_GEN_IN] - gin_seen;        // in-model successors of this chunk
        gin_seen = c[C_GEN_IN];
        r.kernels[0].ms += ms_x; r.kernels[0].launches++; r.kernels[0].algo_bytes += (double)cnt * S_B + (double)nslots * 8 + (double)ncells * 4;
        r.kernels[1].ms += ms_g; r.kernels[1].launches++; r.kernels[1].algo_bytes += (double)ncells * (4 + S_B + 8);
        r.kernels[2].ms += ms_d; r.kernels[2].launches++; r.kernels[2].algo_bytes += (double)nslots * 16 + (double)ncells * 16;
        r.kernels[3].ms += ms_s; r.kernels[3].launches++; r.kernels[3].algo_bytes += (double)nslots * 8 + (double)ncells * 16 + (double)cnt * 4;
        r.kernels[4].ms += ms_c; r.kernels[4].launches++; r.kernels[4].algo_bytes += (double)nslots * 8 + (double)nnew * 8;
        if (ms_m > 0) { r.kernels[5].ms += ms_m; r.kernels[5].launches++; r.kernels[5].algo_bytes += (double)nnew * (8 + 2 * S_B + 8); }
        if (next_write + nnew > cap_end) { c[C_ERR] |= MERR_STORE; stop = true; }
        if (c[C_EVENT] != ~0ull) {
          // first event of this chunk in key order (earlier chunks had none)
          handle_event(c, cnt, level_begin, level_count, rank0, gen_before_chunk, next_write - (level_begin + level_count), nnew, level, r);
          stop_action_counts(c, sp, mp, cb, level_begin, rank0, next_write, act_before_chunk, r);
          stop = true;
        }
        if (c[C_ERR]) stop = true;
        if (stop) break;
        next_write += nnew;
        int64_t g_all = 0; for (int k = 0; k < MA_NACT; ++k) g_all += (int64_t)c[C_ACT + k];
        gen_before_chunk = g_all;
        for (int k = 0; k < 2 * MA_NACT; ++k) act_before_chunk[k] = c[C_ACT + k];
      }
      r.seconds_kernels += level_ms / 1000.0;
      r.n_launches += 1;
      if (c[C_ERR] && r.verdict == MC_VERDICT_OK) {
        const u64 e = c[C_ERR];
        r.verdict = MC_VERDICT_CAPACITY_OVERFLOW;
        std::ostringstream os;
        os << "error flags 0x" << std::hex << e << std::dec << ":";
        if (e & ME_CAP) os << " a field, message count or the message bag exceeded its compiled capacity (state "
                           << (c[C_ERRGID] ? (int64_t)c[C_ERRGID] - 1 : -1) << ");";
        if (e & MERR_STORE) os << " state store full (raise state_store_bytes);";
        if (e & MERR_TABLE_FULL) os << " fingerprint table full (raise fp_table_bytes);";
        r.error = os.str();
      }
      if (stop) {
        if (r.verdict == MC_VERDICT_OK) r.verdict = MC_VERDICT_CAPACITY_OVERFLOW;
        break;
      }
      int64_t gen = 0;
      for (int k = 0; k < MA_NACT; ++k) { r.act_generated[k] += (int64_t)c[C_ACT + k]; r.act_distinct[k] += (int64_t)c[C_ACT + MA_NACT + k]; gen += (int64_t)c[C_ACT + k]; }
      r.generated += gen;
      gen_in_level = c[C_GEN_IN];
      r.generated_in_model += (int64_t)gen_in_level;
      const u64 nnew = next_write - (level_begin + level_count);
      r.algo_bytes += (double)level_count * S_B + (double)gen_in_level * 8 + (double)nnew * (16 + S_B);
      total_ = next_write;
      r.distinct = (int64_t)total_;
      r.levels.back().generated = gen;
      r.levels.back().kernel_ms = level_ms;
      if (nnew > 0) { r.levels.push_back({(int64_t)nnew, 0, 0.0}); r.depth += 1; }
      level_begin += level_count;
      level_count = nnew;
      ++level;
      if (o.checkpoint_every > 0 && !o.checkpoint_path.empty() && r.depth % o.checkpoint_every == 0 && level_count > 0)
        if (int rc = save_checkpoint(o.checkpoint_path, r, level_begin, level_count, err)) return rc;
    }
    finish(r, t0);
    return 0;
  }

  // ---------------------------------------------------------------- checkpoint / recover
  // TLC -checkpoint / -recover (its states/ directory, reference .gitignore:3).  File: magic, the
  // model's describe_json and symmetry mode (a checkpoint only resumes the same model), the BFS
  // position and TLC's counters, then the stored states [0, total) and their parent pointers.
  // Written straight from the host part and, in bounded blocks, from the device part (no second
  // copy of the store in host memory).  The seen-set is rebuilt from the states on recovery.
  struct CkptHead {
    char magic[8];
    u64 nwp, total, level_begin, level_count, seed, sym_tlc;
    int64_t generated, distinct, depth, generated_in_model, n_act, n_levels, desc_len;
  };
  static constexpr u64 kCkptBlock = 1u << 20;   // states per device<->file block
  int save_checkpoint(const std::string& path, const RunResult& r, u64 level_begin, u64 level_count, std::string& err) {
    const std::string desc = describe_json();
    CkptHead h;
    std::memcpy(h.magic, "RAFTMCM1", 8);
    h.nwp = NWP; h.total = total_; h.level_begin = level_begin; h.level_count = level_count; h.seed = r.seed;
    h.sym_tlc = rt_host_.sym_tlc;
    h.generated = r.generated; h.distinct = r.distinct; h.depth = r.depth; h.generated_in_model = r.generated_in_model;
    h.n_act = MA_NACT; h.n_levels = (int64_t)r.levels.size(); h.desc_len = (int64_t)desc.size();
    const std::string tmp = path + ".tmp";
    FILE* f = std::fopen(tmp.c_str(), "wb");
    if (!f) { err = "cannot write checkpoint " + tmp; return MC_E_IO; }
    bool ok = std::fwrite(&h, sizeof h, 1, f) == 1 && std::fwrite(desc.data(), 1, desc.size(), f) == desc.size() &&
              std::fwrite(r.act_generated.data(), 8, MA_NACT, f) == (size_t)MA_NACT &&
              std::fwrite(r.act_distinct.data(), 8, MA_NACT, f) == (size_t)MA_NACT;
    for (const auto& lv : r.levels) ok = ok && std::fwrite(&lv.states, 8, 1, f) == 1 && std::fwrite(&lv.generated, 8, 1, f) == 1;
    ok = ok && host_.write_states(f);
    std::vector<u32> blk;
    for (u64 b = base_; ok && b < total_; b += kCkptBlock) {
      const u64 n = std::min<u64>(kCkptBlock, total_ - b);
      blk.resize(n * NWP);
      ok = hipMemcpy(blk.data(), d_states_ + (b - base_) * NWP, n * NWP * 4, hipMemcpyDeviceToHost) == hipSuccess &&
           std::fwrite(blk.data(), 4, n * NWP, f) == n * NWP;
    }
    ok = ok && host_.write_meta(f);
    std::vector<u64> mblk;
    for (u64 b = base_; ok && b < total_; b += kCkptBlock) {
      const u64 n = std::min<u64>(kCkptBlock, total_ - b);
      mblk.resize(n);
      ok = hipMemcpy(mblk.data(), d_meta_ + (b - base_), n * 8, hipMemcpyDeviceToHost) == hipSuccess &&
           std::fwrite(mblk.data(), 8, n, f) == n;
    }
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
    bool ok = std::fread(&h, sizeof h, 1, f) == 1 && std::memcmp(h.magic, "RAFTMCM1", 8) == 0 && h.nwp == (u64)NWP &&
              h.n_act == MA_NACT && h.desc_len >= 0 && h.desc_len < (1 << 20) && h.n_levels > 0 && h.n_levels < (1 << 20) &&
              h.sym_tlc == rt_host_.sym_tlc;
    if (ok) { fdesc.resize((size_t)h.desc_len); ok = std::fread(&fdesc[0], 1, fdesc.size(), f) == fdesc.size(); }
    if (!ok || fdesc != desc) { std::fclose(f); err = "checkpoint " + path + " is not a checkpoint of this model"; return MC_E_INVALID; }
    // completed levels that do not fit the device store stay in host memory (spilled)
    const u64 lb = h.total > cap_ ? h.level_begin : 0;
    if (h.level_begin > h.total || h.total - lb > cap_) { std::fclose(f); err = "checkpoint frontier exceeds the state store (raise state_store_bytes)"; return MC_E_OOM; }
    ok = std::fread(r.act_generated.data(), 8, MA_NACT, f) == (size_t)MA_NACT &&
         std::fread(r.act_distinct.data(), 8, MA_NACT, f) == (size_t)MA_NACT;
    r.levels.clear();
    for (int64_t k = 0; ok && k < h.n_levels; ++k) {
      LevelStat lv;
      ok = std::fread(&lv.states, 8, 1, f) == 1 && std::fread(&lv.generated, 8, 1, f) == 1;
      r.levels.push_back(lv);
    }
    HIPCHK(hipMemsetAsync(d_ctr_, 0, C_NCTR * 8, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    // states: the host part stays on the host and its fingerprints go in through the (idle)
    // candidate buffer; the device part is read block by block into the store
    host_.clear();
    u32* hs = nullptr; u64* hm = nullptr;
    if (lb) host_.append(lb, &hs, &hm);
    ok = ok && std::fread(hs, 4, lb * NWP, f) == lb * NWP;
    const u64 stage = std::max<u64>(1, chunk_ * S::NSLOT * 8 / (NWP * 4));
    for (u64 b = 0; ok && b < lb; b += stage) {
      const u64 n = std::min<u64>(stage, lb - b);
      HIPCHK(hipMemcpy(d_cand_, hs + b * NWP, n * NWP * 4, hipMemcpyHostToDevice));
      if (int rc = launch_reinsert((const u32*)d_cand_, n, h.seed, err)) return rc;
      HIPCHK(hipStreamSynchronize(stream_));
    }
    std::vector<u32> blk;
    for (u64 b = lb; ok && b < h.total; b += kCkptBlock) {
      const u64 n = std::min<u64>(kCkptBlock, h.total - b);
      blk.resize(n * NWP);
      ok = std::fread(blk.data(), 4, n * NWP, f) == n * NWP;
      if (ok) HIPCHK(hipMemcpy(d_states_ + (b - lb) * NWP, blk.data(), n * NWP * 4, hipMemcpyHostToDevice));
    }
    ok = ok && std::fread(hm, 8, lb, f) == lb;
    std::vector<u64> mblk;
    for (u64 b = lb; ok && b < h.total; b += kCkptBlock) {
      const u64 n = std::min<u64>(kCkptBlock, h.total - b);
      mblk.resize(n);
      ok = std::fread(mblk.data(), 8, n, f) == n;
      if (ok) HIPCHK(hipMemcpy(d_meta_ + (b - lb), mblk.data(), n * 8, hipMemcpyHostToDevice));
    }
    std::fclose(f);
    if (!ok) { host_.clear(); err = "checkpoint " + path + " is truncated"; return MC_E_IO; }
    if (h.total > lb)
      if (int rc = launch_reinsert(d_states_, h.total - lb, h.seed, err)) return rc;
    u64 e = 0;
    HIPCHK(hipMemcpyAsync(&e, d_ctr_ + C_ERR, 8, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    if (e) { err = "fingerprint table too small for the checkpoint (raise fp_table_bytes)"; return MC_E_OOM; }
    base_ = lb;
    r.seed = h.seed; r.generated = h.generated; r.distinct = h.distinct; r.depth = h.depth;
    r.generated_in_model = h.generated_in_model;
    total_ = h.total; level_begin = h.level_begin; level_count = h.level_count;
    return 0;
  }
  int launch_reinsert(const u32* states, u64 n, u64 seed, std::string& err) {
    const dim3 grid((unsigned)((n + BS - 1) / BS));
    if (rt_dev_.sym_tlc)
      hipLaunchKernelGGL((memb_reinsert<S, true>), grid, dim3(BS), 0, stream_, states, n, seed, rt_dev_, d_table_, table_mask_, (unsigned long long*)d_ctr_);
    else
      hipLaunchKernelGGL((memb_reinsert<S, false>), grid, dim3(BS), 0, stream_, states, n, seed, rt_dev_, d_table_, table_mask_, (unsigned long long*)d_ctr_);
    HIPCHK(hipGetLastError());
    return 0;
  }

  // move the completed levels [base_, level_begin) to host memory and the frontier to the front
  // of the device store (left shift by d in blocks of <= d slots: each block's target only
  // overlaps blocks already moved)
  int spill(u64 level_begin, u64 level_count, std::string& err) {
    const u64 d = level_begin - base_;
    u32* hs = nullptr; u64* hm = nullptr;
    host_.append(d, &hs, &hm);   // a segment of its own: the host part is never reallocated
    HIPCHK(hipStreamSynchronize(stream_));
    HIPCHK(hipMemcpy(hs, d_states_, d * NWP * 4, hipMemcpyDeviceToHost));
    HIPCHK(hipMemcpy(hm, d_meta_, d * 8, hipMemcpyDeviceToHost));
    for (u64 off = 0; off < level_count; off += d) {
      const u64 n = std::min<u64>(d, level_count - off);
      HIPCHK(hipMemcpyAsync(d_states_ + off * NWP, d_states_ + (d + off) * NWP, n * NWP * 4, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipMemcpyAsync(d_meta_ + off, d_meta_ + d + off, n * 8, hipMemcpyDeviceToDevice, stream_));
      HIPCHK(hipStreamSynchronize(stream_));
    }
    base_ = level_begin;
    return 0;
  }

  // The first event of the level: reproduce TLC's (the oracle's) stop point, counts and trace.
  void handle_event(const u64* c, u64 cnt, u64 level_begin, u64 level_count, u64 rank0, int64_t gen_before_chunk,
                    u64 new_before_chunk, u64 nnew, u32 level, RunResult& r) {
    const u64 ev = c[C_EVENT], key = ev >> 2;
    const int kind = (int)(ev & 3);
    const u64 rank = key / S::NSLOT, slot = key % S::NSLOT, gid = level_begin + rank;
    // generated: whole successor lists of parents up to this one (next() errors abort before counting)
    std::vector<unsigned short> ns(cnt);
    (void)hipMemcpy(ns.data(), d_nsucc_, cnt * 2, hipMemcpyDeviceToHost);
    int64_t gen = gen_before_chunk;
    for (u64 q = 0; q < rank - rank0; ++q) gen += ns[q];
    if (kind != EV_NEXT_ERROR) gen += ns[rank - rank0];
    // distinct: this level's winners with key < k (<= k when the event state itself may be new)
    std::vector<u64> nr(nnew);
    if (nnew) (void)hipMemcpy(nr.data(), d_newrec_, nnew * 8, hipMemcpyDeviceToHost);
    auto key_of = [&](u64 rec) { return ((rec >> 10) - level_begin) * S::NSLOT + (rec & 1023); };
    u64 before = 0;
    for (u64 q = 0; q < nnew; ++q) {
      const u64 k = key_of(nr[q]);
      if (k < key || (k == key && kind >= EV_INV_ERROR)) ++before;
    }
    r.generated += gen;
    r.distinct = (int64_t)(total_ + new_before_chunk + before);
    // TLC's queue at the stop point (oracle/engine.h): the level's parents after this one and the
    // new states found before it
    r.left_on_queue = (int64_t)(level_count - rank - 1 + new_before_chunk + before);
    W s;
    read_state(gid, s);
    int k, sub;
    S::inst_of_slot((int)slot, k, sub);
    if (kind == EV_DEADLOCK) {
      r.verdict = MC_VERDICT_DEADLOCK;
      build_trace(gid, nullptr, s, r);
      return;
    }
    if (kind == EV_NEXT_ERROR) {
      r.verdict = MC_VERDICT_EVAL_ERROR;
      r.error = "TLC evaluation error while computing the successors of state " + std::to_string(gid) +
                " (SubSeq index out of domain, raft.tla:551/764)";
      build_trace(gid, nullptr, s, r);
      return;
    }
    W t; u32 e2 = 0;
    const int act = S::apply(s, k, sub, t, e2, rt_host_);
    const u32 res = S::check_invariants(t, rt_host_);
    const int id = (int)(res & 255);
    if (kind == EV_INV_ERROR) {
      r.verdict = MC_VERDICT_EVAL_ERROR;
      r.error = std::string("Evaluating invariant ") + kMembInvNames[id] +
                " failed: Committed(i) == SubSeq(log[i], 1, commitIndex[i]) or log[l][idx] outside its domain (raft.tla:969, :1099)";
    } else {
      r.verdict = MC_VERDICT_INVARIANT_VIOLATION;
      r.violated = kMembInvNames[id];
    }
    r.depth = (int64_t)level + 2;   // the successor's depth (oracle: level + 1, Init = 1)
    build_trace(gid, act >= 0 ? kMembActNames[act] : "?", t, r);
  }

  // TLC's per-action (generated, distinct) counters at the stop point: the level's earlier chunks
  // whole, this chunk's parents before the event's whole, the event's parent up to its own successor
  // (none for a next-state error), and the new states before the event (key order = store order)
  int stop_counts_dev(const u32* sp, u64 first, u64 npar, u64 stop, int stop_slot, u32 kind, const u64* meta, u64 before,
                      u64* gen, u64* dist) {
    unsigned long long* d = nullptr;
    if (hipMalloc(&d, 2 * MA_NACT * 8) != hipSuccess) return MC_E_OOM;
    int rc = 0;
    if (hipMemsetAsync(d, 0, 2 * MA_NACT * 8, stream_) != hipSuccess) rc = MC_E_NO_DEVICE;
    if (!rc && npar)
      hipLaunchKernelGGL((memb_stop_generated<S>), dim3((unsigned)((npar + BS - 1) / BS)), dim3(BS), 0, stream_, sp, first, npar, stop,
                         stop_slot, kind, rt_dev_, d);
    if (!rc && before)
      hipLaunchKernelGGL(memb_stop_distinct, dim3((unsigned)((before + BS - 1) / BS)), dim3(BS), 0, stream_, meta, before, d + MA_NACT);
    u64 h[2 * MA_NACT];
    if (!rc && (hipGetLastError() != hipSuccess || hipMemcpyAsync(h, d, sizeof h, hipMemcpyDeviceToHost, stream_) != hipSuccess ||
                hipStreamSynchronize(stream_) != hipSuccess)) rc = MC_E_NO_DEVICE;
    (void)hipFree(d);
    if (rc) return rc;
    for (int k = 0; k < MA_NACT; ++k) { gen[k] = h[k]; dist[k] = h[MA_NACT + k]; }
    return 0;
  }
  void stop_action_counts(const u64* c, const u32* sp, const u64* mp, u64 cb, u64 level_begin, u64 rank0, u64 next_write,
                          const std::vector<u64>& before_chunk, RunResult& r) {
    const u64 ev = c[C_EVENT], key = ev >> 2;
    const int kind = (int)(ev & 3);
    const u64 rank = key / S::NSLOT, slot = key % S::NSLOT;
    (void)level_begin;
    // the new states of this chunk before the event: r.distinct - (stored before this chunk)
    const u64 before = (u64)r.distinct - next_write;
    u64 gen[MA_NACT], dist[MA_NACT];
    if (stop_counts_dev(sp, cb, rank - rank0 + 1, rank - rank0, (int)slot, (u32)kind, mp + next_write, before, gen, dist)) return;
    for (int k = 0; k < MA_NACT; ++k) {
      r.act_generated[k] += (int64_t)(before_chunk[k] + gen[k]);
      r.act_distinct[k] += (int64_t)(before_chunk[MA_NACT + k] + dist[k]);
    }
  }

  int dump_states(const std::string& path, std::string& err) override {
    if (!d_states_) { err = "mc_dump_states before mc_run"; return MC_E_STATE; }
    std::vector<u32> h((total_ - base_) * NWP);
    HIPCHK(hipMemcpy(h.data(), d_states_, h.size() * 4, hipMemcpyDeviceToHost));
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) { err = "cannot write " + path; return MC_E_IO; }
    for (u64 g = 0; g < total_; ++g) {
      u32 w[NWP];
      const u32* src = g < base_ ? host_.state(g) : h.data() + (g - base_) * NWP;
      for (int q = 0; q < NWP; ++q) w[q] = src[q];
      W s; S::unpack(w, s);
      std::fprintf(f, "%s\n", text_.text(s, false).c_str());
    }
    std::fclose(f);
    return 0;
  }

  // ---- sharded mode: FIFO first-found across ranks.  Per level the driver
  // (raft-tla_amd/shard.py fifo_sharded_bfs) calls layout, then per chunk generate / fill(ROUTE) /
  // all-to-all / dedup, then select / fill(REPLY) / all-to-all / materialize, the level
  // statistics (+ event_stats on a stop), level_commit, and the rebalance fill(STATES) /
  // all-to-all / store that gives every rank an equal contiguous slice of the next level.
  int shard_open(const RunOpts& o, int rank, int world, std::string& err) override {
    if (world < 1 || world > 8 || rank < 0 || rank >= world) { err = "world must be 1..8"; return MC_E_INVALID; }
    base_ = 0; host_.clear();   // sharded runs keep every state on the device
    for (int q = 0; q < 2; ++q)
      if (((m_.rt.constraints >> kPrefixCon[q]) & 1u) && !have_prefix_[q]) {
        err = std::string(kMembConNames[kPrefixCon[q]]) + " needs its golden history trace (mc_set_history_prefix)";
        return MC_E_UNSUPPORTED;
      }
    RunOpts so = o;
    if (!so.state_store_bytes) {   // leave room for the level records and the sort (see below)
      size_t freeb = 0, totalb = 0;
      if (hipSetDevice(o.device) == hipSuccess && hipMemGetInfo(&freeb, &totalb) == hipSuccess)
        so.state_store_bytes = std::min<uint64_t>(96ull << 30, freeb / 4);
    }
    if (int rc = ensure_alloc(so, err)) return rc;
    if (int rc = prepare_prefixes(err)) return rc;
    rt_host_.sym_tlc = rt_dev_.sym_tlc = (o.sym_tlc && m_.rt.symmetry) ? 1u : 0u;
    fp_slice_test_ = o.test_fp_slice;
    rt_host_.disjunct_copies = rt_dev_.disjunct_copies = o.disjunct_copies ? 1u : 0u;
    sopts_ = o; s_rank_ = rank; s_world_ = world; s_finished_ = false; have_viol_ = false; sres_err_ = 0; sharded_ = true;
    // level records / sorted winners / newrec: lvl_cap_ entries each, plus the sort's scratch
    const u64 sb = so.state_store_bytes;
    const u64 want = std::max<u64>(4096, (sb / 4) / 16);
    if (!d_lvl_ || lvl_cap_ != want) {
      for (void* q : {(void*)d_lvl_, (void*)d_sorted_, (void*)d_newrec_lvl_, (void*)d_sort_tmp_, (void*)d_nsucc_lvl_}) if (q) (void)hipFree(q);
      lvl_cap_ = want;
      HIPCHK(hipMalloc(&d_lvl_, lvl_cap_ * 16));
      HIPCHK(hipMalloc(&d_sorted_, lvl_cap_ * 8));
      HIPCHK(hipMalloc(&d_newrec_lvl_, lvl_cap_ * 8));
      HIPCHK(hipMalloc(&d_nsucc_lvl_, cap_ * 2));
      sort_tmp_bytes_ = 0;
      HIPCHK(rocprim::radix_sort_keys(nullptr, sort_tmp_bytes_, (const u64*)nullptr, (u64*)nullptr, (size_t)lvl_cap_, 0, 48,
                                      stream_));
      HIPCHK(hipMalloc(&d_sort_tmp_, std::max<size_t>(sort_tmp_bytes_, 16)));
    }
    HIPCHK(hipMemsetAsync(d_table_, 0, (table_mask_ + 1) * 16, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    sres_ = RunResult();
    sres_.seed = o.seed ? o.seed : 0x5EED5EED2024ull;
    sres_.state_bytes = NWP * 4;
    for (int k = 0; k < MA_NACT; ++k) sres_.action_names.push_back(kMembActNames[k]);
    sres_.act_generated.assign(MA_NACT, 0); sres_.act_distinct.assign(MA_NACT, 0);
    sres_.kernels = {{"memb_expand", 0, 0, 0}, {"memb_fingerprint", 0, 0, 0}, {"memb_dedup_sh", 0, 0, 0},
                     {"memb_select_sh", 0, 0, 0}, {"memb_materialize", 0, 0, 0}};
    t0_ = std::chrono::steady_clock::now();
    // Init (raft.tla:388-393): every rank evaluates it; rank 0 stores it, its owner seeds the seen-set
    W s0; S::init(s0);
    sres_.generated = 1; sres_.depth = 1;
    sres_.levels.push_back({1, 0, 0.0});
    s_level_ = 0; s_level_begin_ = 0; s_level_count_ = 0; total_ = 0;
    if (!S::in_model(s0, s0, rt_host_)) { sres_.distinct = 0; sres_.depth = 0; s_finished_ = true; finish(sres_, t0_); return 0; }
    const u64 fp0 = S::fingerprint(s0, sres_.seed, rt_host_);
    if (fp_owner(fp0, (u32)world) == (u32)rank) {
      const u64 e2[2] = {fp0, ~0ull};
      HIPCHK(hipMemcpy(d_table_ + 2 * (fp0 & table_mask_), e2, 16, hipMemcpyHostToDevice));
    }
    if (rank == 0) {
      u32 w0[S::NW]; S::pack(s0, w0);
      u32 wp[NWP] = {0}; for (int q = 0; q < S::NW; ++q) wp[q] = w0[q];
      HIPCHK(hipMemcpy(d_states_, wp, NWP * 4, hipMemcpyHostToDevice));
      const u64 nometa = ~0ull;
      HIPCHK(hipMemcpy(d_meta_, &nometa, 8, hipMemcpyHostToDevice));
      total_ = 1; s_level_count_ = 1;
    }
    sres_.distinct = 1;
    if (u32 bad = S::check_invariants(s0, rt_host_)) {
      if ((bad >> 8) == IV_BAD) { sres_.verdict = MC_VERDICT_INVARIANT_VIOLATION; sres_.violated = kMembInvNames[bad & 255]; }
      else { sres_.verdict = MC_VERDICT_EVAL_ERROR; sres_.error = std::string("TLC evaluation error in invariant ") + kMembInvNames[bad & 255]; }
      if (rank == 0) { have_viol_ = true; viol_parent_ = ~0ull; viol_act_ = "<Initial predicate>"; viol_text_ = text_.text(s0, true); }
      s_finished_ = true; s_level_count_ = 0; finish(sres_, t0_);
    }
    return 0;
  }
  int shard_record_bytes(int what) const override {
    return what == MC_SHARD_ROUTE ? 16 : what == MC_SHARD_REPLY ? 8 : what == MC_SHARD_STATES ? NWP * 4 + 8 : -1;
  }
  int shard_frontier(int64_t* states, int64_t* chunk) const override {
    if (states) *states = s_finished_ ? 0 : (int64_t)s_level_count_;
    if (chunk) *chunk = (int64_t)chunk_;
    return 0;
  }
  // start of a level: every rank's frontier size (global ranks = concatenation in rank order)
  int shard_layout(const int64_t* counts, std::string& err) override {
    u64 acc = 0;
    for (int q = 0; q < 8; ++q) {
      if (q < s_world_) { if (q == s_rank_) s_B_ = acc; ks_[q] = acc * (u64)S::NSLOT; acc += (u64)counts[q]; }
      else ks_[q] = ~0ull;
    }
    s_F_ = acc;
    if (s_F_ * (u64)S::NSLOT >= (1ull << 40)) { err = "level too large for 40-bit FIFO keys"; return MC_E_UNSUPPORTED; }
    HIPCHK(hipMemsetAsync(d_ctr_, 0, C_NCTR * 8, stream_));
    HIPCHK(hipMemsetAsync(d_ctr_ + C_EVENT, 0xFF, 8, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    lvl_n_ = 0; n_sorted_ = 0; nnew_ = 0; level_ms_ = 0;
    return 0;
  }
  int shard_generate(int64_t begin, int64_t count, int64_t* counts, std::string& err) override {
    for (int q = 0; q < s_world_; ++q) counts[q] = 0;
    gen_cnt_ = (u64)std::max<int64_t>(0, count);
    gen_begin_ = (u64)begin;
    if (!gen_cnt_) return 0;
    const u64 cnt = gen_cnt_, nslots = cnt * (u64)S::NSLOT;
    const u32 nblk = (u32)((cnt + BS - 1) / BS);
    MGenArgs g;
    g.states = d_states_; g.chunk_begin = s_level_begin_ + gen_begin_; g.chunk_count = cnt; g.rank0 = s_B_ + gen_begin_;
    g.cand = d_cand_; g.cells = d_cells_; g.cells_oom = d_cells_oom_; g.cell_count = d_cell_count_; g.nsucc = d_nsucc_;
    g.seed = sres_.seed; g.rt = rt_dev_; g.inv_oom = sopts_.inv_out_of_model ? 1u : 0u;
    g.deadlock = sopts_.check_deadlock ? 1u : 0u; g.ctr = (unsigned long long*)d_ctr_;
    g.smask = nullptr;   // the dense cand form: memb_route / memb_dedup_sh / memb_select_sh read every slot
    HIPCHK(hipEventRecord(ev_[0], stream_));
    hipLaunchKernelGGL((memb_expand<S>), dim3(nblk), dim3(BS), 0, stream_, g);
    HIPCHK(hipGetLastError());
    if (sopts_.inv_out_of_model) hipLaunchKernelGGL((memb_oom_check<S>), dim3(nblk), dim3(BS), 0, stream_, g);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev_[1], stream_));
    if (int rc = launch_fingerprint(g, nblk, err)) return rc;
    HIPCHK(hipEventRecord(ev_[2], stream_));
    HIPCHK(hipMemcpyAsync(d_nsucc_lvl_ + gen_begin_, d_nsucc_, cnt * 2, hipMemcpyDeviceToDevice, stream_));
    route_.cand = d_cand_; route_.nslots = nslots; route_.chunk_count = cnt; route_.rank0 = s_B_ + gen_begin_;
    route_.nslot = S::NSLOT; route_.world = (u32)s_world_; route_.counts = (unsigned long long*)(d_ctr_ + C_SHARD);
    route_.out = nullptr;
    HIPCHK(hipMemsetAsync(d_ctr_ + C_SHARD, 0, 8 * 8, stream_));
    hipLaunchKernelGGL((memb_route<false>), dim3((unsigned)((nslots + BS * RPER - 1) / (BS * RPER))), dim3(BS), 0, stream_, route_);
    HIPCHK(hipGetLastError());
    u64 c[8];
    HIPCHK(hipMemcpyAsync(c, d_ctr_ + C_SHARD, sizeof c, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    sres_.kernels[0].ms += ms(0, 1); sres_.kernels[0].launches++;
    sres_.kernels[1].ms += ms(1, 2); sres_.kernels[1].launches++;
    level_ms_ += ms(0, 2);
    for (int q = 0; q < s_world_; ++q) counts[q] = (int64_t)c[q];
    return 0;
  }
  int shard_fill(int what, void* dst, const int64_t* offsets, std::string& err) override {
    if (what == MC_SHARD_ROUTE) {
      if (!gen_cnt_) return 0;
      u64 cur[8] = {0};
      for (int q = 0; q < s_world_; ++q) cur[q] = (u64)offsets[q];
      HIPCHK(hipMemcpyAsync(d_ctr_ + C_SHARD, cur, sizeof cur, hipMemcpyHostToDevice, stream_));
      route_.out = (u64*)dst;
      hipLaunchKernelGGL((memb_route<true>), dim3((unsigned)((route_.nslots + BS * RPER - 1) / (BS * RPER))), dim3(BS), 0, stream_, route_);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(stream_));
      return 0;
    }
    if (what == MC_SHARD_REPLY) {
      if (!lvl_n_) return 0;
      u64 cur[8] = {0};
      for (int q = 0; q < s_world_; ++q) cur[q] = (u64)offsets[q];
      HIPCHK(hipMemcpyAsync(d_ctr_ + C_SHARD, cur, sizeof cur, hipMemcpyHostToDevice, stream_));
      sel_.out = (u64*)dst;
      hipLaunchKernelGGL((memb_select_sh<true>), dim3((unsigned)((lvl_n_ + BS * RPER - 1) / (BS * RPER))), dim3(BS), 0, stream_, sel_);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(stream_));
      return 0;
    }
    if (what == MC_SHARD_STATES) {   // this rank's new states, in key order (one contiguous run)
      if (!nnew_) return 0;
      hipLaunchKernelGGL((memb_pack_states<NWP>), dim3((unsigned)((nnew_ + BS - 1) / BS)), dim3(BS), 0, stream_,
                         (const u32*)d_states_, (const u64*)d_meta_, total_, nnew_, (u32*)dst);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(stream_));
      return 0;
    }
    err = "unknown record kind";
    return MC_E_INVALID;
  }
  int shard_dedup(const void* recv, const int64_t* counts, int64_t* reply_counts, std::string& err) override {
    u64 n = 0;
    for (int q = 0; q < s_world_; ++q) { n += (u64)counts[q]; reply_counts[q] = 0; }   // winners are decided per level
    if (!n) return 0;
    if (lvl_n_ + n > lvl_cap_) { sres_err_ |= MERR_STORE; return 0; }
    MDedupShArgs d;
    d.recv = (const u64*)recv; d.n = n; d.level = s_level_ + 1; d.table = d_table_; d.table_mask = table_mask_;
    d.lvl = d_lvl_ + 2 * lvl_n_; d.ctr = (unsigned long long*)d_ctr_;
    HIPCHK(hipEventRecord(ev_[3], stream_));
    hipLaunchKernelGGL(memb_dedup_sh, dim3((unsigned)((n + BS * DPER - 1) / (BS * DPER))), dim3(BS), 0, stream_, d);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev_[4], stream_));
    HIPCHK(hipEventSynchronize(ev_[4]));
    sres_.kernels[2].ms += ms(3, 4); sres_.kernels[2].launches++; sres_.kernels[2].algo_bytes += (double)n * 48;
    level_ms_ += ms(3, 4);
    lvl_n_ += n;
    return 0;
  }
  // owner side, after the level's last chunk: winning keys per generating rank
  int shard_select(int64_t* reply_counts, std::string& err) override {
    for (int q = 0; q < s_world_; ++q) reply_counts[q] = 0;
    if (!lvl_n_) return 0;
    sel_.lvl = d_lvl_; sel_.n = lvl_n_; sel_.level = s_level_ + 1; sel_.table = d_table_;
    for (int q = 0; q < 8; ++q) sel_.kstart[q] = ks_[q];
    sel_.world = (u32)s_world_; sel_.counts = (unsigned long long*)(d_ctr_ + C_SHARD); sel_.out = nullptr;
    HIPCHK(hipMemsetAsync(d_ctr_ + C_SHARD, 0, 8 * 8, stream_));
    HIPCHK(hipEventRecord(ev_[3], stream_));
    hipLaunchKernelGGL((memb_select_sh<false>), dim3((unsigned)((lvl_n_ + BS * RPER - 1) / (BS * RPER))), dim3(BS), 0, stream_, sel_);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev_[4], stream_));
    u64 c[8];
    HIPCHK(hipMemcpyAsync(c, d_ctr_ + C_SHARD, sizeof c, hipMemcpyDeviceToHost, stream_));
    HIPCHK(hipStreamSynchronize(stream_));
    sres_.kernels[3].ms += ms(3, 4); sres_.kernels[3].launches++; sres_.kernels[3].algo_bytes += (double)lvl_n_ * 24;
    level_ms_ += ms(3, 4);
    for (int q = 0; q < s_world_; ++q) reply_counts[q] = (int64_t)c[q];
    return 0;
  }
  // generating side: sort the winning keys, re-derive them in key order at the store's end
  int shard_materialize(const void* acks, const int64_t* counts, std::string& err) override {
    u64 n = 0;
    for (int q = 0; q < s_world_; ++q) n += (u64)counts[q];
    n_sorted_ = n; nnew_ = 0;
    if (!n) return 0;
    if (n > lvl_cap_) { sres_err_ |= MERR_STORE; n_sorted_ = 0; return 0; }
    if (total_ + n > cap_) { sres_err_ |= MERR_STORE; n_sorted_ = 0; return 0; }
    size_t tb = sort_tmp_bytes_;
    HIPCHK(hipEventRecord(ev_[5], stream_));
    HIPCHK(rocprim::radix_sort_keys(d_sort_tmp_, tb, (const u64*)acks, d_sorted_, (size_t)n, 0, 48, stream_));
    hipLaunchKernelGGL(memb_keys_to_newrec, dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_, (const u64*)d_sorted_, n,
                       (u64)S::NSLOT, s_B_, s_level_begin_, d_newrec_lvl_);
    HIPCHK(hipGetLastError());
    MMatArgs m;
    m.states = d_states_; m.meta = d_meta_; m.newrec = d_newrec_lvl_; m.n_new = n; m.dst_base = total_; m.cap = cap_;
    m.level_begin = s_level_begin_ - s_B_;   // gid - level_begin = global rank (mod 2^64)
    m.gid_tag = (u64)s_rank_ << 37; m.rt = rt_dev_; m.ctr = (unsigned long long*)d_ctr_;
    if (rt_dev_.sym_tlc) hipLaunchKernelGGL((memb_materialize<S, true>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_, m);
    else hipLaunchKernelGGL((memb_materialize<S, false>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_, m);
    HIPCHK(hipGetLastError());
    HIPCHK(hipEventRecord(ev_[6], stream_));
    HIPCHK(hipEventSynchronize(ev_[6]));
    sres_.kernels[4].ms += ms(5, 6); sres_.kernels[4].launches++; sres_.kernels[4].algo_bytes += (double)n * (8 + 2 * NWP * 4 + 8);
    level_ms_ += ms(5, 6);
    nnew_ = n;
    return 0;
  }
  // the received slice of the next level, appended to the store (replacing the staged new states)
  int shard_store(const void* states, int64_t n, std::string& err) override {
    if (total_ + (u64)n > cap_) { err = "state store full (raise state_store_bytes)"; return MC_E_OOM; }
    if (n > 0) {
      hipLaunchKernelGGL((memb_unpack_states<NWP>), dim3((unsigned)((n + BS - 1) / BS)), dim3(BS), 0, stream_, (const u32*)states,
                         (u64)n, total_, d_states_, d_meta_);
      HIPCHK(hipGetLastError());
      HIPCHK(hipStreamSynchronize(stream_));
    }
    s_level_begin_ = total_;
    s_level_count_ = (u64)n;
    total_ += (u64)n;
    nnew_ = 0;
    return 0;
  }
  // stats layout (MC_SHARD_NSTAT): [0] winners materialised here, [1] generated, [2] in-model
  // generated, [3] error flags, [4] (1 << 62) - first event (0 = none; max-reduced = min event),
  // [6] frontier, [8..28) per-action generated, [40..60) per-action distinct, [30] / [31] the stop
  // point's generated / new-state counts and [32] 1 + the violated invariant's id (event_stats)
  int shard_level_stats(int64_t* st, std::string& err) override {
    u64 c[C_NCTR];
    HIPCHK(hipMemcpy(c, d_ctr_, sizeof c, hipMemcpyDeviceToHost));
    std::memset(st, 0, MC_SHARD_NSTAT * sizeof(int64_t));
    int64_t gen = 0;
    for (int k = 0; k < MA_NACT; ++k) { st[8 + k] = (int64_t)c[C_ACT + k]; st[40 + k] = (int64_t)c[C_ACT + MA_NACT + k]; gen += (int64_t)c[C_ACT + k]; }
    st[0] = (int64_t)nnew_; st[1] = gen; st[2] = (int64_t)c[C_GEN_IN];
    st[3] = (int64_t)(c[C_ERR] | sres_err_);
    st[4] = c[C_EVENT] == ~0ull ? 0 : (int64_t)((1ull << 62) - c[C_EVENT]);
    st[6] = (int64_t)s_level_count_;
    return 0;
  }
  // the global first event K: this rank's share of TLC's counters at the stop point; the rank
  // that generated K records the counterexample head
  int shard_event_stats(const int64_t* g, int64_t* st, std::string& err) override {
    std::memset(st, 0, MC_SHARD_NSTAT * sizeof(int64_t));
    if (!g[4]) return 0;
    const u64 ev = (1ull << 62) - (u64)g[4], key = ev >> 2;
    const int kind = (int)(ev & 3);
    const u64 R = key / S::NSLOT, slot = key % S::NSLOT;
    // generated: whole successor lists of the parents before R (and R's, unless next() failed)
    std::vector<unsigned short> ns(s_level_count_);
    if (s_level_count_) HIPCHK(hipMemcpy(ns.data(), d_nsucc_lvl_, s_level_count_ * 2, hipMemcpyDeviceToHost));
    int64_t gen = 0;
    for (u64 q = 0; q < s_level_count_; ++q) {
      const u64 r = s_B_ + q;
      if (r < R || (r == R && kind != EV_NEXT_ERROR)) gen += ns[q];
    }
    // distinct: this rank's winners with key < K (<= K when the event state itself may be new)
    std::vector<u64> ks(n_sorted_);
    if (n_sorted_) HIPCHK(hipMemcpy(ks.data(), d_sorted_, n_sorted_ * 8, hipMemcpyDeviceToHost));
    int64_t before = 0;
    for (u64 k : ks) if (k < key || (k == key && kind >= EV_INV_ERROR)) ++before;
    st[30] = gen; st[31] = before;
    {   // this rank's share of TLC's per-action counters at the stop point ([8, 8+A) generated, [40, 40+A) distinct)
      const u64 npar = R < s_B_ ? 0 : std::min<u64>(s_level_count_, R - s_B_ + 1);
      u64 ag[MA_NACT], ad[MA_NACT];
      if (int rc = stop_counts_dev(d_states_, s_level_begin_, npar, R - std::min<u64>(R, s_B_), (int)slot, (u32)kind,
                                   d_meta_ + total_, (u64)before, ag, ad)) { err = "stop-point counters"; return rc; }
      for (int k = 0; k < MA_NACT; ++k) { st[8 + k] = (int64_t)ag[k]; st[40 + k] = (int64_t)ad[k]; }
    }
    if (R >= s_B_ && R < s_B_ + s_level_count_) {   // the event's parent is ours: the counterexample head
      const u64 gid = s_level_begin_ + (R - s_B_);
      W s; read_state(gid, s);
      u64 meta = 0;
      HIPCHK(hipMemcpy(&meta, d_meta_ + gid, 8, hipMemcpyDeviceToHost));
      have_viol_ = true;
      if (kind == EV_DEADLOCK || kind == EV_NEXT_ERROR) {   // the trace ends at the parent itself
        viol_parent_ = meta == ~0ull ? ~0ull : (meta >> 20);
        viol_act_ = meta == ~0ull ? "<Initial predicate>" : kMembActNames[(meta >> 10) & 1023];
        viol_text_ = text_.text(s, true);
      } else {
        int k, sub;
        S::inst_of_slot((int)slot, k, sub);
        W t; u32 e2 = 0;
        const int act = S::apply(s, k, sub, t, e2, rt_host_);
        viol_parent_ = gid | ((u64)s_rank_ << 37);
        viol_act_ = act >= 0 ? kMembActNames[act] : "?";
        viol_text_ = text_.text(t, true);
        st[32] = 1 + (int64_t)(S::check_invariants(t, rt_host_) & 255);   // the invariant's id, for every rank
      }
    }
    return 0;
  }
  int shard_level_commit(const int64_t* g, int* done, std::string& err) override {
    *done = 0;
    if (s_finished_) { *done = 1; return 0; }
    sres_.seconds_kernels += level_ms_ / 1000.0;
    sres_.n_launches += 1;
    if (g[4]) {   // the level's first event in key order stops the search (single-GPU handle_event)
      const u64 ev = (1ull << 62) - (u64)g[4], key = ev >> 2;
      const int kind = (int)(ev & 3);
      const u64 R = key / S::NSLOT;
      sres_.generated += g[30];
      sres_.distinct += g[31];
      for (int k = 0; k < MA_NACT; ++k) { sres_.act_generated[k] += g[8 + k]; sres_.act_distinct[k] += g[40 + k]; }
      if (kind == EV_DEADLOCK) sres_.verdict = MC_VERDICT_DEADLOCK;
      else if (kind == EV_NEXT_ERROR) {
        sres_.verdict = MC_VERDICT_EVAL_ERROR;
        sres_.error = "TLC evaluation error while computing the successors of a state (SubSeq index out of domain, raft.tla:551/764)";
      } else if (kind == EV_INV_ERROR) {
        sres_.verdict = MC_VERDICT_EVAL_ERROR;
        sres_.error = std::string("Evaluating invariant ") + (g[32] ? kMembInvNames[g[32] - 1] : "?") +
                      " failed: Committed(i) == SubSeq(log[i], 1, commitIndex[i]) or log[l][idx] outside its domain (raft.tla:969, :1099)";
      } else {
        sres_.verdict = MC_VERDICT_INVARIANT_VIOLATION;
        sres_.violated = g[32] ? kMembInvNames[g[32] - 1] : "?";
      }
      if (kind >= EV_INV_ERROR) sres_.depth = (int64_t)s_level_ + 2;   // the successor's depth
      sres_.left_on_queue = (int64_t)(s_F_ - R - 1) + g[31];          // TLC's queue at the stop point
      s_finished_ = true; *done = 1;
      finish(sres_, t0_);
      return 0;
    }
    if (g[3]) {
      sres_.verdict = MC_VERDICT_CAPACITY_OVERFLOW;
      std::ostringstream os; os << "error flags 0x" << std::hex << g[3] << " raised on some rank"; sres_.error = os.str();
      s_finished_ = true; *done = 1;
      finish(sres_, t0_);
      return 0;
    }
    sres_.generated += g[1];
    sres_.generated_in_model += g[2];
    for (int k = 0; k < MA_NACT; ++k) { sres_.act_generated[k] += g[8 + k]; sres_.act_distinct[k] += g[40 + k]; }
    sres_.levels.back().generated = g[1];
    sres_.levels.back().kernel_ms = level_ms_;
    sres_.distinct += g[0];
    if (g[0] > 0) { sres_.levels.push_back({g[0], 0, 0.0}); sres_.depth += 1; }
    ++s_level_;
    if (g[0] == 0) *done = 1;
    else if (sopts_.max_depth && sres_.depth >= sopts_.max_depth) { sres_.verdict = MC_VERDICT_DEPTH_LIMIT; sres_.left_on_queue = g[0]; *done = 1; }
    if (*done) {   // the last level stays where it was generated (no rebalance follows)
      total_ += nnew_; nnew_ = 0;
      s_finished_ = true; finish(sres_, t0_);
    }
    return 0;
  }
  int shard_read_state(uint64_t gid, std::string& text, uint64_t* meta, std::string& err) const override {
    const u64 local = gid & ((1ull << 37) - 1);
    if (local >= total_) { err = "state id out of range"; return MC_E_INVALID; }
    W s; read_state(local, s);
    u64 m = 0;
    if (hipMemcpy(&m, d_meta_ + local, 8, hipMemcpyDeviceToHost) != hipSuccess) { err = "hipMemcpy failed"; return MC_E_NO_DEVICE; }
    text = text_.text(s, true);
    // normalised as the raft_original records: parent gid << 24 | action << 16
    if (meta) *meta = m == ~0ull ? ~0ull : ((m >> 20) << 24) | (((m >> 10) & 1023) << 16);
    return 0;
  }
  int shard_violation(uint64_t* parent, std::string& action, std::string& text) const override {
    if (!have_viol_) return MC_E_STATE;
    if (parent) *parent = viol_parent_;
    action = viol_act_; text = viol_text_;
    return 0;
  }
  const RunResult* shard_result() const override { return &sres_; }
  // the whole FIFO-ranked level loop natively over a transport (RCCL or the in-process loopback),
  // after shard_open: fifo_shard_loop.h
  int shard_run_native(ShardTransport& t, std::string& err) override {
    FifoShardLoop loop(*this, t, s_rank_, s_world_);
    return loop.run(err);
  }

 private:
  MembModel m_;
  MembText<S> text_;
  u64* d_table_ = nullptr; u32* d_states_ = nullptr; u64* d_meta_ = nullptr; u64* d_ctr_ = nullptr;
  u64* d_cand_ = nullptr; u64* d_newrec_ = nullptr; unsigned short* d_nsucc_ = nullptr; unsigned int* d_woff_ = nullptr;
  u32* d_cells_ = nullptr; u32* d_cells_oom_ = nullptr; u32* d_cell_count_ = nullptr; u32* d_big_ = nullptr;
  u64* d_smask_ = nullptr;   // [SMW][chunk] in-model slot masks (single-GPU loop)
  static constexpr int SMW = (S::NSLOT + 63) / 64;
  int fp_slice_test_ = -1;   // RunOpts::test_fp_slice of the current run
  u64* d_bsum_ = nullptr;
  hipStream_t stream_ = nullptr;
  hipEvent_t ev_[9] = {};
  u64 table_mask_ = 0, cap_ = 0, total_ = 0, chunk_ = 0;
  int dev_ = -1; uint64_t req_table_ = 0, req_store_ = 0;
  // completed levels moved to host memory: global ids [0, base_) live in host_ (segments)
  u64 base_ = 0;
  HostStore host_{NWP};

  // sharded mode
  RunOpts sopts_;
  RunResult sres_;
  std::chrono::steady_clock::time_point t0_;
  int s_rank_ = 0, s_world_ = 1;
  bool s_finished_ = false, have_viol_ = false, sharded_ = false;
  u32 s_level_ = 0;
  u64 s_level_begin_ = 0, s_level_count_ = 0, s_B_ = 0, s_F_ = 0, ks_[8] = {0};
  u64 gen_begin_ = 0, gen_cnt_ = 0, lvl_n_ = 0, lvl_cap_ = 0, n_sorted_ = 0, nnew_ = 0, sres_err_ = 0;
  double level_ms_ = 0;
  u64* d_lvl_ = nullptr; u64* d_sorted_ = nullptr; u64* d_newrec_lvl_ = nullptr; void* d_sort_tmp_ = nullptr;
  unsigned short* d_nsucc_lvl_ = nullptr;
  size_t sort_tmp_bytes_ = 0;
  MRouteArgs route_{};
  MSelShArgs sel_{};
  u64 viol_parent_ = 0; std::string viol_act_, viol_text_;

  MembRuntime rt_host_{}, rt_dev_{};
  std::vector<u64> ptab_[2];
  u32 plen_[2] = {0, 0};
  bool have_prefix_[2] = {false, false};
  u64* d_ptab_[2] = {nullptr, nullptr};

  // phase 2 on the stream: the symmetric fingerprints of the chunk's in-model cells.  (Round 4 tried
  // queueing the states with a ConfigEntry to a second kernel on full waves of their own: 1531 vs
  // 1267 ms of C3 fingerprint time, the re-derivation of the queued cells costing more than their
  // lanes' divergence had.)
  int launch_fingerprint(MGenArgs g, u32 nblk, std::string& err) {
    g.prof = nullptr;
#ifdef RMC_FP_PROF
    if (!d_prof_) { HIPCHK(hipMalloc(&d_prof_, 8 * 8)); HIPCHK(hipMemset(d_prof_, 0, 8 * 8)); }
    g.prof = d_prof_;
#endif
    g.big = d_big_;
    {   // room for one insertion; mc_set_fp_slice (tests) lowers the cap
      const int full = (S::MK + 1 < 24 ? S::MK + 1 : 24) - 1;
      const int t = fp_slice_test_;
      g.slice_cap = (u32)(t >= 0 && t < full ? t : full);
    }
    if (rt_dev_.sym_tlc && !g.prof) {
      hipLaunchKernelGGL((memb_fingerprint_lds<S>), dim3(nblk), dim3(BS), 0, stream_, g);
      HIPCHK(hipGetLastError());
      hipLaunchKernelGGL((memb_fingerprint_list<S>), dim3(std::min<u32>(nblk, 256u)), dim3(BS), 0, stream_, g);
    } else if (rt_dev_.sym_tlc) {   // (RMC_FP_PROF builds: the stage timers are memb_fingerprint's)
      hipLaunchKernelGGL((memb_fingerprint<S, true>), dim3(nblk), dim3(BS), 0, stream_, g);
    } else {
      hipLaunchKernelGGL((memb_fingerprint<S, false>), dim3(nblk), dim3(BS), 0, stream_, g);
    }
    HIPCHK(hipGetLastError());
    return 0;
  }
  unsigned long long* d_prof_ = nullptr;   // RMC_FP_PROF builds (printed to stderr by release)

  void release_device() override { release(); }
  void release() {
    if (d_prof_) {
      unsigned long long h[8] = {0};
      if (hipMemcpy(h, d_prof_, sizeof h, hipMemcpyDeviceToHost) == hipSuccess)
        std::fprintf(stderr, "FP_PROF apply %llu prologue %llu first %llu narrow %llu bagloops %llu tail %llu view %llu\n",
                     h[0], h[1], h[2], h[3], h[4], h[5], h[6]);
      (void)hipFree(d_prof_);
      d_prof_ = nullptr;
    }
    for (auto& p : d_ptab_) { if (p) (void)hipFree(p); p = nullptr; }
    for (void* q : {(void*)d_lvl_, (void*)d_sorted_, (void*)d_newrec_lvl_, (void*)d_sort_tmp_, (void*)d_nsucc_lvl_}) if (q) (void)hipFree(q);
    d_lvl_ = nullptr; d_sorted_ = nullptr; d_newrec_lvl_ = nullptr; d_sort_tmp_ = nullptr; d_nsucc_lvl_ = nullptr; lvl_cap_ = 0;
    for (void* p : {(void*)d_table_, (void*)d_states_, (void*)d_meta_, (void*)d_ctr_, (void*)d_cand_, (void*)d_newrec_,
                    (void*)d_nsucc_, (void*)d_woff_, (void*)d_bsum_, (void*)d_cells_, (void*)d_cells_oom_, (void*)d_cell_count_, (void*)d_big_, (void*)d_smask_})
      if (p) (void)hipFree(p);
    for (auto& e : ev_) { if (e) (void)hipEventDestroy(e); e = nullptr; }
    if (stream_) (void)hipStreamDestroy(stream_);
    d_table_ = nullptr; d_states_ = nullptr; d_meta_ = nullptr; d_ctr_ = nullptr; d_cand_ = nullptr; d_newrec_ = nullptr;
    d_nsucc_ = nullptr; d_woff_ = nullptr; d_bsum_ = nullptr; d_cells_ = nullptr; d_cells_oom_ = nullptr; d_cell_count_ = nullptr; d_big_ = nullptr; d_smask_ = nullptr; stream_ = nullptr;
  }
  // stored state `gid` (global id) and its parent pointer, from the host part or the device
  void read_state(u64 gid, W& s, u64* meta = nullptr) const {
    u32 w[NWP];
    if (gid < base_) {
      std::memcpy(w, host_.state(gid), NWP * 4);
      if (meta) *meta = host_.meta(gid);
    } else {
      (void)hipMemcpy(w, d_states_ + (gid - base_) * NWP, NWP * 4, hipMemcpyDeviceToHost);
      if (meta) (void)hipMemcpy(meta, d_meta_ + (gid - base_), 8, hipMemcpyDeviceToHost);
    }
    S::unpack(w, s);
  }
  void finish(RunResult& r, std::chrono::steady_clock::time_point t0) {
    const double M = (double)r.distinct, Ng = (double)r.generated;
    r.collision_optimistic = M * (Ng - M) / 18446744073709551616.0;
    r.seconds_total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  }
  // parent-pointer chase on the host (<= depth device reads)
  void build_trace(u64 parent, const char* last_act, const W& last, RunResult& r) {
    std::vector<std::pair<std::string, std::string>> tr;
    if (last_act) tr.push_back({last_act, text_.text(last, true)});
    u64 g = parent;
    while (true) {
      W s; u64 meta = 0;
      read_state(g, s, &meta);
      if (meta == ~0ull) { tr.push_back({"<Initial predicate>", text_.text(s, true)}); break; }
      tr.push_back({kMembActNames[(meta >> 10) & 1023], text_.text(s, true)});
      g = meta >> 20;
    }
    std::reverse(tr.begin(), tr.end());
    r.trace = tr;
  }
};

// ------------------------------------------------------------------ shapes compiled into this build: (N, NV)
#ifdef RMC_QUICK_BUILD
#define RMC_MEMB_SHAPES(X) X(3, 2)
#else
#define RMC_MEMB_SHAPES(X) \
  X(3, 2) /* shipped raft.cfg */ \
  X(2, 1)                        \
  X(2, 2)                        \
  X(3, 1)                        \
  X(4, 2) /* C3: 4 servers */
#endif

static Backend* memb_factory(const MembModel& m) {
#define X(n, nv) if (m.N == n && m.NV == nv) return new MembGpu<Memb<n, nv, 2 * n * n>>(m);
  RMC_MEMB_SHAPES(X)
#undef X
  return nullptr;
}

Backend* make_memb_backend(const CfgFile& cfg) {
  MembModel m = resolve_memb_model(cfg);
  Backend* b = memb_factory(m);
  if (!b) {
    std::string o;
#define X(n, nv) o += std::string(o.empty() ? "" : ", ") + "(" #n "," #nv ")";
    RMC_MEMB_SHAPES(X)
#undef X
    throw CfgError(MC_E_UNSUPPORTED, "tlc_membership shape (N=" + std::to_string(m.N) + ", |Value|=" + std::to_string(m.NV) +
                                         ") is not compiled into this build; compiled (N,|Value|): " + o);
  }
  return b;
}

}  // namespace rmc
