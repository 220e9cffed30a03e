// tlagen_kernels.h — the generated path's BFS kernels for gfx950 (appended to a generated spec
// in one translation unit; compiled by hiprtc at mc_open time or ahead of time by hipcc
// --genco; see tlagen_backend.cpp).
//
// One level = one launch of tlg_expand: a grid-stride loop gives each lane a frontier state,
// which it copies into its arena (a private slice of HBM) and enumerates with the generated
// tlg::next_states.  Each successor is laid out contiguously at the arena top, checked against
// the cfg's constraints, fingerprinted (tlv::fp_words over its canonical words) and inserted in
// the open-addressing seen-set (8-B entries, CAS on the empty slot: TLC -workers N semantics,
// every count order independent); a winner appends its words to the state store (one atomic for
// its id, one for its word range) with its parent id and action, and is checked against the
// invariants.  Per-lane counters are flushed once per lane.  The first event (invariant
// violation, evaluation error, deadlock) wins a flag, records itself, and stops the grid.
//
// Unlike the hand-compiled path (fixed-width packed states, one lane per (state, action
// instance)), a lane here runs a whole state's Next: the generality costs divergence and
// arena traffic; it is the fallback for specs nobody hand-compiled.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>   // hipcc --genco; hiprtc provides the device builtins itself
#endif
namespace tlk {
using namespace tlv;

enum : u32 {
  C_GEN = 0,       // generated successors
  C_GIN = 1,       // in-model successors
  C_ERR = 2,       // OR of arena error bits of failed lanes
  C_CAP = 3,       // store / seen-set capacity exhausted
  C_FLAG = 4,      // event claimed (0/1)
  C_KIND = 5,      // event kind: 1 violation (stored state), 2 violation (out-of-model successor), 3 eval error (computing
                   // the successors of C_SID, a constraint or an out-of-model invariant), 4 deadlock, 5 eval error of an
                   // invariant on the stored state C_SID (C_INV: the invariant)
  C_SID = 6,       // event state id (kind 1: the violating state; 2: its parent; 3/4: the state being expanded)
  C_INV = 7,       // kind 1/2: invariant index; kind 3: error bits
  C_EACT = 8,      // kind 2: action of the violating successor
  C_EWORDS = 9,    // kind 2: words of the violating successor in evbuf
  C_ACT = 16       // [C_ACT, C_ACT + NACT) generated per action, then NACT distinct per action
};

struct Args {
  u32* words;                       // state store: canonical words of every state, appended
  unsigned long long* words_used;
  unsigned long long words_cap;
  unsigned long long* offs;         // per state id: first word
  unsigned long long* parent;       // per state id: parent id (~0 for initial states)
  u32* act;                         // per state id: action that produced it
  unsigned long long states_cap;
  unsigned long long* n_states;     // state ids handed out (may pass states_cap on overflow)
  unsigned long long* n_committed;  // states whose words, offset, parent and action were written
  unsigned long long* table;        // seen-set of fingerprints (0 = empty)
  unsigned long long table_mask;
  u32* arena;                       // per lane: acap words
  u32 acap;
  u32* hstack;                      // per lane: hcap handles
  u32 hcap;
  unsigned long long* ctr;
  u32* evbuf;                       // words of an out-of-model violating successor
  u32 evcap;
  unsigned long long first, count;  // the level: state ids [first, first + count)
  unsigned long long seed;
  int inv_oom, deadlock;
};

__device__ inline bool claim(Args& a) { return atomicCAS(&a.ctr[C_FLAG], 0ull, 1ull) == 0ull; }

struct Em {
  Args* a;
  unsigned long long parent;
  unsigned long long gen, gin;
  unsigned long long act_gen[tlg::NACT > 0 ? tlg::NACT : 1], act_dist[tlg::NACT > 0 ? tlg::NACT : 1];

  __device__ __attribute__((noinline)) void operator()(tlg::Cx& c) {
    Ar& A = *c.A;
    if (A.err) return;   // computed after an evaluation error: not a successor (the parent reports the error)
    const u32 t0 = A.top;
    u32 n = 0;
    for (int i = 0; i < tlg::NV; ++i) n += sz(A, c.nxt[i]);
    const u32 w0 = alloc(A, n);
    if (A.err & E_OVF) return;
    u32 o = w0;
    for (int i = 0; i < tlg::NV; ++i) {
      const u32 h = c.nxt[i], m = sz(A, h);
      for (u32 q = 0; q < m; ++q) A.w[o + q] = A.w[h + q];
      o += m;
    }
    ++gen;
    ++act_gen[c.act];
    tlg::Cx d = c;
    for (int i = 0; i < tlg::NV; ++i) d.cur[i] = c.nxt[i];
    const bool im = tlg::constraints(d);
    if (A.err) {   // a constraint could not be evaluated on this successor: TLC's evaluation error
      if (!(A.err & E_OVF) && claim(*a)) { a->ctr[C_KIND] = 3; a->ctr[C_SID] = parent; a->ctr[C_INV] = A.err; }
      A.top = t0;
      return;
    }
    if (im) {
      ++gin;
      const unsigned long long fp = fp_words(A.w + w0, n, a->seed);
      unsigned long long slot = fp & a->table_mask;
      bool fresh = false;
      for (unsigned long long probe = 0;; ++probe) {
        if (probe > a->table_mask) { atomicOr(&a->ctr[C_CAP], 2ull); break; }
        const unsigned long long cur = a->table[slot];
        if (cur == fp) break;
        if (cur == 0ull) {
          const unsigned long long old = atomicCAS(&a->table[slot], 0ull, fp);
          if (old == 0ull) { fresh = true; break; }
          if (old == fp) break;
        }
        slot = (slot + 1) & a->table_mask;
      }
      if (fresh) {
        ++act_dist[c.act];
        const unsigned long long sid = atomicAdd(a->n_states, 1ull);
        const unsigned long long wp = atomicAdd(a->words_used, (unsigned long long)n);
        if (sid >= a->states_cap || wp + n > a->words_cap) {
          atomicOr(&a->ctr[C_CAP], 1ull);
        } else {
          for (u32 q = 0; q < n; ++q) a->words[wp + q] = A.w[w0 + q];
          a->offs[sid] = wp;
          a->parent[sid] = parent;
          a->act[sid] = (u32)c.act;
          atomicAdd(a->n_committed, 1ull);
          const int bad = tlg::invariants(d);
          if (A.err) {   // an invariant could not be evaluated on the new state: TLC's evaluation error
            if (!(A.err & E_OVF) && claim(*a)) { a->ctr[C_KIND] = 5; a->ctr[C_SID] = sid; a->ctr[C_INV] = (unsigned long long)bad; }
          } else if (bad >= 0 && claim(*a)) {
            a->ctr[C_KIND] = 1; a->ctr[C_SID] = sid; a->ctr[C_INV] = (unsigned long long)bad;
          }
        }
      }
    } else if (a->inv_oom) {
      const int bad = tlg::invariants(d);
      if (A.err) {   // evaluation error of an invariant on an out-of-model successor
        if (!(A.err & E_OVF) && claim(*a)) { a->ctr[C_KIND] = 3; a->ctr[C_SID] = parent; a->ctr[C_INV] = A.err; }
      } else if (bad >= 0 && claim(*a)) {
        a->ctr[C_KIND] = 2; a->ctr[C_SID] = parent; a->ctr[C_INV] = (unsigned long long)bad;
        a->ctr[C_EACT] = (unsigned long long)c.act;
        const u32 m = n < a->evcap ? n : a->evcap;
        for (u32 q = 0; q < m; ++q) a->evbuf[q] = A.w[w0 + q];
        a->ctr[C_EWORDS] = m;
      }
    }
    A.top = t0;
  }

  __device__ void flush() {
    atomicAdd(&a->ctr[C_GEN], gen);
    atomicAdd(&a->ctr[C_GIN], gin);
    for (int k = 0; k < tlg::NACT; ++k) {
      if (act_gen[k]) atomicAdd(&a->ctr[C_ACT + k], act_gen[k]);
      if (act_dist[k]) atomicAdd(&a->ctr[C_ACT + tlg::NACT + k], act_dist[k]);
    }
  }
};

__device__ inline void lane_init(Args& a, Ar& A, tlg::Cx& c, Em& em, unsigned long long lane) {
  init(A, a.arena + lane * a.acap, a.acap, a.hstack + lane * a.hcap, a.hcap);
  c.A = &A;
  tlg::init_consts(c);
  em.a = &a; em.gen = em.gin = 0;
  for (int k = 0; k < (tlg::NACT > 0 ? tlg::NACT : 1); ++k) { em.act_gen[k] = 0; em.act_dist[k] = 0; }
}

}  // namespace tlk

extern "C" __global__ void __launch_bounds__(64) tlg_init_k(tlk::Args a) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  tlv::Ar A;
  tlg::Cx c;
  tlk::Em em;
  tlk::lane_init(a, A, c, em, 0);
  em.parent = ~0ull;
  tlg::init_states(c, em);
  for (int k = 0; k < (tlg::NACT > 0 ? tlg::NACT : 1); ++k) { em.act_gen[k] = 0; em.act_dist[k] = 0; }   // initial states are no action's
  if (A.err) {
    if (A.err & tlv::E_OVF) atomicOr(&a.ctr[tlk::C_CAP], 4ull);
    else if (tlk::claim(a)) { a.ctr[tlk::C_KIND] = 3; a.ctr[tlk::C_SID] = ~0ull; a.ctr[tlk::C_INV] = A.err; }
  }
  em.flush();
}

extern "C" __global__ void __launch_bounds__(64) tlg_expand_k(tlk::Args a) {
  const unsigned long long lane = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  tlv::Ar A;
  tlg::Cx c;
  tlk::Em em;
  tlk::lane_init(a, A, c, em, lane);
  const tlv::u32 floor = A.top;
  for (unsigned long long i = lane; i < a.count; i += stride) {
    if (__atomic_load_n(&a.ctr[tlk::C_FLAG], __ATOMIC_RELAXED) || __atomic_load_n(&a.ctr[tlk::C_CAP], __ATOMIC_RELAXED)) break;
    const unsigned long long sid = a.first + i;
    A.top = floor; A.htop = 0; A.err = 0;
    const tlv::u32* p = a.words + a.offs[sid];
    for (int v = 0; v < tlg::NV; ++v) { c.cur[v] = tlv::copy_in(A, p); p += p[0] >> 3; }
    em.parent = sid;
    const unsigned long long g0 = em.gen;
    tlg::next_states(c, em);
    if (A.err) {
      if (A.err & tlv::E_OVF) atomicOr(&a.ctr[tlk::C_CAP], 4ull);
      else if (tlk::claim(a)) { a.ctr[tlk::C_KIND] = 3; a.ctr[tlk::C_SID] = sid; a.ctr[tlk::C_INV] = A.err; }
    } else if (a.deadlock && em.gen == g0 && tlk::claim(a)) {
      a.ctr[tlk::C_KIND] = 4; a.ctr[tlk::C_SID] = sid;
    }
  }
  em.flush();
}
