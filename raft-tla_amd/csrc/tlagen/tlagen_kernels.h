// tlagen_kernels.h — the generated path's BFS kernels for gfx950 (appended to a generated spec
// in one translation unit; compiled by hiprtc at mc_open time or ahead of time by hipcc
// --genco; see tlagen_backend.cpp).
//
// A lane takes a frontier state, copies it into its arena (a private slice of HBM) and
// enumerates its successors with the generated tlg::next_states; each successor is laid out
// contiguously at the arena top, checked against the cfg's constraints and fingerprinted
// (tlv::fp_words over its canonical words, or over the words of the cfg's VIEW of it).
//
// Two search orders, as TLC has them:
//  * -workers N (fifo = 0, one launch per level, tlg_expand_k): a new fingerprint is inserted in
//    the 8-B seen-set by CAS and the winning lane appends the state to the store at once (one
//    atomic for its id, one for its word range); every count TLC prints is order independent.
//  * -workers 1 (fifo = 1, TLC's single-worker FIFO order): pass 1 (tlg_expand_k)
//    gives every successor the key  rank of its parent in the level << 24 | its ordinal in the
//    parent's successor list  (TLC's dequeue-and-enumerate order) and inserts (fp, ~key) in a 16-B
//    seen-set that keeps the minimum key per fingerprint (atomicMax of the complement); the host
//    sorts the keys of the entries this level inserted (tlg_keys_k + a radix sort); pass 2
//    (tlg_mat_k) re-expands each parent that owns winners once and stores its winners at their
//    rank in key order, checking the invariants on them.  Which successor of a view class is
//    kept, the parent pointers, the counterexample and the stop point are then TLC's.
// The first event of a level (TLC's evaluation error, deadlock, invariant violation) is, in the
// FIFO order, the minimum of  key << 3 | kind  (C_EV); in the -workers N order the first lane to
// claim a flag wins and the host searches the model again in FIFO order for TLC's report.
// Initial states are enumerated by one lane, in Init's order (first-come = TLC's order).
//
// Unlike the hand-compiled path (fixed-width packed states, one lane per (state, action
// instance)), a lane here runs a whole state's Next: the generality costs divergence and
// arena traffic; it is the path for specs nobody hand-compiled.
#ifndef __HIPCC_RTC__
#include <hip/hip_runtime.h>   // hipcc --genco; hiprtc provides the device builtins itself
#endif
namespace tlk {
using namespace tlv;

enum : u32 {
  C_GEN = 0,       // generated successors
  C_GIN = 1,       // in-model successors
  C_ERR = 2,       // OR of arena error bits of failed lanes
  C_CAP = 3,       // capacity exhausted: 1 store, 2 seen-set, 4 lane arena, 8 successors per state (FIFO key)
  C_FLAG = 4,      // event claimed (0/1): -workers N order, and the initial states
  C_KIND = 5,      // event kind: 1 violation (stored state), 2 violation (out-of-model successor), 3 eval error (computing
                   // the successors of C_SID, a constraint or an out-of-model invariant), 4 deadlock, 5 eval error of an
                   // invariant on the stored state C_SID (C_INV: the invariant)
  C_SID = 6,       // event state id (kind 1: the violating state; 2: its parent; 3/4: the state being expanded)
  C_INV = 7,       // kind 1/2: invariant index; kind 3: error bits
  C_EACT = 8,      // kind 2 / stop capture: action of the violating successor
  C_EWORDS = 9,    // kind 2 / stop capture: words of the violating successor in evbuf
  C_EV = 10,       // FIFO order: min of key << 3 | EV_* over the level (~0 = none)
  C_EVINV = 11,    // FIFO stop capture: the first invariant the event successor violates (or fails to evaluate)
  C_NEWPOS = 12,   // FIFO pass 1: seen-set entries inserted this level
  C_ACT = 16       // [C_ACT, C_ACT + NACT) generated per action, then NACT distinct per action
};
// FIFO event kinds, in TLC's order at one key: errors while computing a state's successors come
// before its successors' checks
enum : u32 { EV_NEXT_ERROR = 0, EV_DEADLOCK = 1, EV_INV_ERROR_OOM = 2, EV_INV_ERROR_NEW = 3, EV_VIOLATION_OOM = 4, EV_VIOLATION_NEW = 5 };
enum : u32 { M_EXPAND = 0, M_MAT = 1, M_STOP = 2 };
constexpr u32 ORD_BITS = 24;   // successors per state (TLC key = parent rank << 24 | ordinal)

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
  unsigned long long* table;        // seen-set: 8-B {fp} (-workers N) or 16-B {fp, ~key} (FIFO), 0 = empty
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
  int fifo;                         // TLC's single-worker FIFO order (two passes per level)
  unsigned long long* newpos;       // FIFO pass 1: seen-set entries inserted this level (ctr[C_NEWPOS] of them)
  unsigned long long newpos_cap;
  const unsigned long long* wkeys;  // FIFO pass 2: the level's winner keys, ascending
  unsigned long long n_w;
  unsigned long long level_end;     // FIFO pass 2: id of the level's first new state
  unsigned long long stop_rank, stop_ord;   // tlg_stop_k: the event's parent rank and successor ordinal
  int stop_kind;
};

__device__ inline bool claim(Args& a) { return atomicCAS(&a.ctr[C_FLAG], 0ull, 1ull) == 0ull; }
__device__ inline void event(Args& a, unsigned long long key, u32 kind) { atomicMin(&a.ctr[C_EV], (key << 3) | kind); }

// keyed insert-if-absent (FIFO): the entry keeps the minimum key; true = this call inserted fp
__device__ inline bool insert_keyed(Args& a, unsigned long long fp, unsigned long long key, unsigned long long& pos) {
  unsigned long long slot = fp & a.table_mask;
  const unsigned long long nk = ~key;
  for (unsigned long long probe = 0;; ++probe) {
    if (probe > a.table_mask) { atomicOr(&a.ctr[C_CAP], 2ull); pos = ~0ull; return false; }
    unsigned long long cur = a.table[2 * slot];
    bool mine = false;
    if (cur == 0ull) {
      cur = atomicCAS(&a.table[2 * slot], 0ull, fp);
      mine = cur == 0ull;
      if (mine) cur = fp;
    }
    if (cur == fp) {
      if (a.table[2 * slot + 1] < nk) atomicMax(&a.table[2 * slot + 1], nk);
      pos = slot;
      return mine;
    }
    slot = (slot + 1) & a.table_mask;
  }
}

// plain insert-if-absent (-workers N): true = this call inserted fp
__device__ inline bool insert_plain(Args& a, unsigned long long fp) {
  unsigned long long slot = fp & a.table_mask;
  for (unsigned long long probe = 0;; ++probe) {
    if (probe > a.table_mask) { atomicOr(&a.ctr[C_CAP], 2ull); return false; }
    const unsigned long long cur = a.table[slot];
    if (cur == fp) return false;
    if (cur == 0ull) {
      const unsigned long long old = atomicCAS(&a.table[slot], 0ull, fp);
      if (old == 0ull) return true;
      if (old == fp) return false;
    }
    slot = (slot + 1) & a.table_mask;
  }
}

struct Em {
  Args* a;
  u32 mode;
  unsigned long long parent;        // the parent's state id (~0: Init)
  unsigned long long rank;          // its rank in the level (FIFO key)
  unsigned long long gen, gin, ord;
  unsigned long long j;             // M_MAT: the next winner key of this parent
  unsigned long long act_gen[tlg::NACT > 0 ? tlg::NACT : 1], act_dist[tlg::NACT > 0 ? tlg::NACT : 1];

  // the parent's per-variable fingerprint terms (expand_state), reused for the variables a
  // successor leaves unchanged
  unsigned long long ph[tlg::NV > 0 ? tlg::NV : 1];

  // the successor's canonical words laid out contiguously at the arena top (only for a state that
  // is stored or reported: the fingerprint and the checks work on the variables' own values)
  __device__ bool layout(Ar& A, tlg::Cx& c, u32& w0, u32& n) {
    n = 0;
    for (int i = 0; i < tlg::NV; ++i) n += sz(A, c.nxt[i]);
    w0 = alloc(A, n);
    if (A.err & E_OVF) return false;
    u32 q0 = w0;
    for (int i = 0; i < tlg::NV; ++i) {
      const u32 h = c.nxt[i], m = sz(A, h);
      for (u32 q = 0; q < m; ++q) A.w[q0 + q] = A.w[h + q];
      q0 += m;
    }
    return true;
  }

  __device__ __attribute__((noinline)) void operator()(tlg::Cx& c) {
    Ar& A = *c.A;
    if (A.err) return;   // computed after an evaluation error: not a successor (the parent reports the error)
    const unsigned long long o = ord++;   // this successor's ordinal in the parent's list
    const u32 t0 = A.top;
    // the variables this successor changed (a handle differs from the parent's; all for Init)
    unsigned long long chg = ~0ull;
    if (parent != ~0ull) {
      chg = 0;
      for (int i = 0; i < tlg::NV; ++i) chg |= (c.nxt[i] != c.cur[i] ? 1ull : 0ull) << i;
    }
    tlg::Cx d = c;
    for (int i = 0; i < tlg::NV; ++i) d.cur[i] = c.nxt[i];
    const unsigned long long key = (rank << ORD_BITS) | o;
    if (mode == M_MAT) { materialize(A, d, c, key, chg); A.top = t0; return; }
    if (mode == M_STOP) { stop_count(A, c, o, chg); A.top = t0; return; }
    const bool keyed = a->fifo && parent != ~0ull;   // FIFO pass 1 (initial states: stored at once)
    ++gen;
    ++act_gen[c.act];
    // in the model: the state constraints, then (a transition, not an initial state) the action
    // constraints over (parent, successor)
    const bool im = tlg::constraints(d, chg) && (parent == ~0ull || tlg::action_constraints(c));
    if (A.err) {   // a constraint could not be evaluated on this successor: TLC's evaluation error
      error_event(A, key, keyed);
      A.top = t0;
      return;
    }
    if (im) {
      ++gin;
      unsigned long long fp;
      if (tlg::HAS_VIEW || tlg::HAS_SYMMETRY) {   // TLC's VIEW / SYMMETRY: the fingerprint of what tells states apart
        const u32 vh = tlg::canon_view(d);
        if (A.err) { error_event(A, key, keyed); A.top = t0; return; }
        fp = fp_words(A.w + vh, sz(A, vh), a->seed);
      } else {
        fp = state_fp(A, c, chg);
      }
      if (keyed) {
        unsigned long long pos = 0;
        if (insert_keyed(*a, fp, key, pos)) {
          const unsigned long long k = atomicAdd(&a->ctr[C_NEWPOS], 1ull);
          if (k < a->newpos_cap) a->newpos[k] = pos; else atomicOr(&a->ctr[C_CAP], 2ull);
        }
      } else {
        unsigned long long pos = 0;
        const bool fresh = a->fifo ? insert_keyed(*a, fp, key, pos) : insert_plain(*a, fp);
        if (fresh) store_now(A, d, c, chg);
      }
    } else if (a->inv_oom) {
      const int bad = tlg::invariants(d, chg);
      if (A.err) {   // evaluation error of an invariant on an out-of-model successor
        error_event(A, key, keyed);
      } else if (bad >= 0) {
        if (keyed) event(*a, key, EV_VIOLATION_OOM);
        else if (claim(*a)) {
          a->ctr[C_KIND] = 2; a->ctr[C_SID] = parent; a->ctr[C_INV] = (unsigned long long)bad;
          a->ctr[C_EACT] = (unsigned long long)c.act;
          u32 w0 = 0, n = 0;
          const u32 m = layout(A, c, w0, n) ? (n < a->evcap ? n : a->evcap) : 0u;
          for (u32 q = 0; q < m; ++q) a->evbuf[q] = A.w[w0 + q];
          a->ctr[C_EWORDS] = m;
        }
      }
    }
    A.top = t0;
  }

  // a state's fingerprint: the sum of per-variable terms (fp_words of the variable's canonical
  // words under a per-variable seed), mixed; a variable the successor left unchanged reuses the
  // parent's term, so only changed variables are read and hashed
  __device__ static unsigned long long var_term(const Ar& A, u32 h, int v, unsigned long long seed) {
    return fp_words(A.w + h, sz(A, h), seed ^ (0x9E3779B97F4A7C15ull * (unsigned long long)(v + 1)));
  }
  __device__ unsigned long long state_fp(const Ar& A, tlg::Cx& c, unsigned long long chg) const {
    unsigned long long s = 0;
    for (int i = 0; i < tlg::NV; ++i) s += ((chg >> i) & 1ull) ? var_term(A, c.nxt[i], i, a->seed) : ph[i];
    s = fmix(s ^ a->seed);
    return s ? s : 1ull;
  }
  __device__ void parent_terms(const Ar& A, tlg::Cx& c) {
    for (int i = 0; i < tlg::NV; ++i) ph[i] = var_term(A, c.cur[i], i, a->seed);
  }

  // a constraint / VIEW / out-of-model invariant could not be evaluated on a successor
  __device__ void error_event(Ar& A, unsigned long long key, bool keyed) {
    if (!(A.err & E_OVF)) {
      if (keyed) event(*a, key, EV_INV_ERROR_OOM);
      else if (claim(*a)) { a->ctr[C_KIND] = 3; a->ctr[C_SID] = parent; a->ctr[C_INV] = A.err; }
    } else {
      atomicOr(&a->ctr[C_CAP], 4ull);
    }
    A.err = 0;   // (its siblings are still generated: TLC's counts at the stop point include them)
  }

  // -workers N (and the initial states): the inserting lane stores the new state at once
  __device__ void store_now(Ar& A, tlg::Cx& d, tlg::Cx& c, unsigned long long chg) {
    ++act_dist[c.act];
    u32 w0 = 0, n = 0;
    if (!layout(A, c, w0, n)) { atomicOr(&a->ctr[C_CAP], 4ull); return; }   // arena overflow: searched again, larger
    const unsigned long long sid = atomicAdd(a->n_states, 1ull);
    const unsigned long long wp = atomicAdd(a->words_used, (unsigned long long)n);
    if (sid >= a->states_cap || wp + n > a->words_cap) { atomicOr(&a->ctr[C_CAP], 1ull); return; }
    for (u32 q = 0; q < n; ++q) a->words[wp + q] = A.w[w0 + q];
    a->offs[sid] = wp;
    a->parent[sid] = parent;
    a->act[sid] = (u32)c.act;
    atomicAdd(a->n_committed, 1ull);
    const int bad = tlg::invariants(d, chg);
    if (A.err) {   // an invariant could not be evaluated on the new state: TLC's evaluation error
      if (!(A.err & E_OVF) && claim(*a)) { a->ctr[C_KIND] = 5; a->ctr[C_SID] = sid; a->ctr[C_INV] = (unsigned long long)bad; }
      A.err = 0;
    } else if (bad >= 0 && claim(*a)) {
      a->ctr[C_KIND] = 1; a->ctr[C_SID] = sid; a->ctr[C_INV] = (unsigned long long)bad;
    }
  }

  // FIFO pass 2: the successor is stored iff its key is this parent's next winner key
  __device__ void materialize(Ar& A, tlg::Cx& d, tlg::Cx& c, unsigned long long key, unsigned long long chg) {
    if (j >= a->n_w || a->wkeys[j] != key) return;
    const unsigned long long sid = a->level_end + j;
    ++j;
    ++act_dist[c.act];
    u32 w0 = 0, n = 0;
    if (!layout(A, c, w0, n)) { atomicOr(&a->ctr[C_CAP], 4ull); return; }
    const unsigned long long wp = atomicAdd(a->words_used, (unsigned long long)n);
    if (sid >= a->states_cap || wp + n > a->words_cap) { atomicOr(&a->ctr[C_CAP], 1ull); return; }
    for (u32 q = 0; q < n; ++q) a->words[wp + q] = A.w[w0 + q];
    a->offs[sid] = wp;
    a->parent[sid] = parent;
    a->act[sid] = (u32)c.act;
    atomicAdd(a->n_committed, 1ull);
    const int bad = tlg::invariants(d, chg);
    if (A.err) {
      if (!(A.err & E_OVF)) event(*a, key, EV_INV_ERROR_NEW);
      A.err = 0;
    } else if (bad >= 0) {
      event(*a, key, EV_VIOLATION_NEW);
    }
  }

  // tlg_stop_k: TLC's generated counts at the stop point (whole successor lists of the parents up
  // to the event's one; per action, the event parent's only up to the event's successor; none of
  // it when the event is an error computing those successors or a deadlock), and the words of the
  // event's successor
  __device__ void stop_count(Ar& A, tlg::Cx& c, unsigned long long o, unsigned long long chg) {
    const bool at_event = rank == a->stop_rank;
    if (at_event && (a->stop_kind == (int)EV_NEXT_ERROR || a->stop_kind == (int)EV_DEADLOCK)) return;
    ++gen;
    if (!at_event || o <= a->stop_ord) ++act_gen[c.act];
    if (at_event && o == a->stop_ord) {
      a->ctr[C_EACT] = (unsigned long long)c.act;
      u32 w0 = 0, n = 0;
      const u32 m = layout(A, c, w0, n) ? (n < a->evcap ? n : a->evcap) : 0u;
      for (u32 q = 0; q < m; ++q) a->evbuf[q] = A.w[w0 + q];
      a->ctr[C_EWORDS] = m;
      tlg::Cx d = c;
      for (int i = 0; i < tlg::NV; ++i) d.cur[i] = c.nxt[i];
      const int bad = tlg::invariants(d, chg);
      a->ctr[C_EVINV] = (unsigned long long)(bad < 0 ? 0 : bad);
      A.err = 0;
    }
  }

  __device__ void flush() {
    if (gen) atomicAdd(&a->ctr[C_GEN], gen);
    if (gin) atomicAdd(&a->ctr[C_GIN], gin);
    for (int k = 0; k < tlg::NACT; ++k) {
      if (act_gen[k]) atomicAdd(&a->ctr[C_ACT + k], act_gen[k]);
      if (act_dist[k]) atomicAdd(&a->ctr[C_ACT + tlg::NACT + k], act_dist[k]);
    }
  }
};

__device__ inline void lane_init(Args& a, Ar& A, tlg::Cx& c, Em& em, unsigned long long lane, u32 mode) {
  init(A, a.arena + lane * a.acap, a.acap, a.hstack + lane * a.hcap, a.hcap);
  c.A = &A;
  tlg::init_consts(c);
  em.a = &a; em.mode = mode; em.gen = em.gin = em.ord = 0; em.j = 0; em.rank = 0;
  for (int k = 0; k < (tlg::NACT > 0 ? tlg::NACT : 1); ++k) { em.act_gen[k] = 0; em.act_dist[k] = 0; }
}

// copy state sid into the lane's arena and enumerate its successors; the arena error bits
__device__ inline u32 expand_state(Args& a, Ar& A, tlg::Cx& c, Em& em, u32 floor, unsigned long long sid) {
  A.top = floor; A.htop = 0; A.err = 0;
  const tlv::u32* p = a.words + a.offs[sid];
  for (int v = 0; v < tlg::NV; ++v) { c.cur[v] = tlv::copy_in(A, p); p += p[0] >> 3; }
  if (!(tlg::HAS_VIEW || tlg::HAS_SYMMETRY)) em.parent_terms(A, c);
  em.parent = sid;
  em.ord = 0;
  tlg::next_states(c, em);
  return A.err;
}

}  // namespace tlk

extern "C" __global__ void __launch_bounds__(64) tlg_init_k(tlk::Args a) {
  if (blockIdx.x != 0 || threadIdx.x != 0) return;
  tlv::Ar A;
  tlg::Cx c;
  tlk::Em em;
  tlk::lane_init(a, A, c, em, 0, tlk::M_EXPAND);
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
  tlk::lane_init(a, A, c, em, lane, tlk::M_EXPAND);
  const tlv::u32 floor = A.top;
  for (unsigned long long i = lane; i < a.count; i += stride) {
    // -workers N: the first event ends the level; FIFO: every parent is expanded (the stop point
    // is the minimum over the whole level), capacity ends both
    if (__atomic_load_n(&a.ctr[tlk::C_CAP], __ATOMIC_RELAXED) || (!a.fifo && __atomic_load_n(&a.ctr[tlk::C_FLAG], __ATOMIC_RELAXED))) break;
    const unsigned long long sid = a.first + i;
    em.rank = i;
    const unsigned long long g0 = em.gen;
    const tlv::u32 e = tlk::expand_state(a, A, c, em, floor, sid);
    if (e) {
      if (e & tlv::E_OVF) atomicOr(&a.ctr[tlk::C_CAP], 4ull);
      else if (a.fifo) tlk::event(a, i << tlk::ORD_BITS, tlk::EV_NEXT_ERROR);
      else if (tlk::claim(a)) { a.ctr[tlk::C_KIND] = 3; a.ctr[tlk::C_SID] = sid; a.ctr[tlk::C_INV] = e; }
    } else if (a.deadlock && em.gen == g0) {
      if (a.fifo) tlk::event(a, i << tlk::ORD_BITS, tlk::EV_DEADLOCK);
      else if (tlk::claim(a)) { a.ctr[tlk::C_KIND] = 4; a.ctr[tlk::C_SID] = sid; }
    }
    if (em.ord >= (1ull << tlk::ORD_BITS)) atomicOr(&a.ctr[tlk::C_CAP], 8ull);   // more successors than a key holds
  }
  em.flush();
}

// FIFO: the level's winner keys, i.e. the minimum key each entry inserted by pass 1 ended with
extern "C" __global__ void __launch_bounds__(256) tlg_keys_k(const unsigned long long* table, const unsigned long long* newpos,
                                                            unsigned long long n, unsigned long long* keys) {
  for (unsigned long long i = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (unsigned long long)gridDim.x * blockDim.x)
    keys[i] = ~table[2 * newpos[i] + 1];
}

// FIFO pass 2: a lane per parent that owns winners (the first of its run of sorted keys)
extern "C" __global__ void __launch_bounds__(64) tlg_mat_k(tlk::Args a) {
  const unsigned long long lane = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  tlv::Ar A;
  tlg::Cx c;
  tlk::Em em;
  tlk::lane_init(a, A, c, em, lane, tlk::M_MAT);
  const tlv::u32 floor = A.top;
  for (unsigned long long i = lane; i < a.n_w; i += stride) {
    const unsigned long long r = a.wkeys[i] >> tlk::ORD_BITS;
    if (i > 0 && (a.wkeys[i - 1] >> tlk::ORD_BITS) == r) continue;
    em.rank = r;
    em.j = i;
    (void)tlk::expand_state(a, A, c, em, floor, a.first + r);
  }
  em.flush();
}

// the stop point: parents [0, stop_rank] of the level re-expanded for TLC's generated counts
extern "C" __global__ void __launch_bounds__(64) tlg_stop_k(tlk::Args a) {
  const unsigned long long lane = (unsigned long long)blockIdx.x * blockDim.x + threadIdx.x;
  const unsigned long long stride = (unsigned long long)gridDim.x * blockDim.x;
  tlv::Ar A;
  tlg::Cx c;
  tlk::Em em;
  tlk::lane_init(a, A, c, em, lane, tlk::M_STOP);
  const tlv::u32 floor = A.top;
  for (unsigned long long i = lane; i <= a.stop_rank && i < a.count; i += stride) {
    em.rank = i;
    (void)tlk::expand_state(a, A, c, em, floor, a.first + i);
  }
  em.flush();
}
