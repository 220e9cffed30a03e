// raftmc — thirdparty/raft_original.tla (Ongaro 2014) hand-compiled to a
// fixed-width packed state, shared by the gfx950 kernels and the host decoder.
//
// Shape parameters (compile time): N servers, NV values, MT = MaxTerm,
// ML = MaxLogLen, MK = MaxMsgDomain.  They come from the cfg (configs/*.cfg,
// the MC wrapper configs/raft_original_mc.tla) and size every field; the
// message-count range [MinMsgCount, MaxMsgCount] is a runtime parameter.
//
// Working state ("Work", registers): one scalar word per per-server array
// (currentTerm, state, votedFor, commitIndex, votesResponded, votesGranted),
// small per-row arrays for nextIndex/matchIndex/log/voterLog (read through
// select chains, never scratch), the allLogs bitmap over the log universe,
// and the elections / messages sets as sorted code arrays (~0 = empty slot).
// Out-of-model successors may hold one transient extra log entry / message /
// term, so working widths are one step wider than the packed (stored) ones.
//
// Canonical packed state: the concatenation of the fields below in a fixed
// bit order; equal TLA+ states <=> equal packed words (sets/bags sorted,
// unused slots zero).  Semantics cite raft_original.tla line numbers.
#pragma once
#include <type_traits>

#include "common.h"

namespace rmc {

enum OrigAct {
  OA_Restart, OA_Timeout, OA_RequestVote, OA_BecomeLeader, OA_ClientRequest, OA_AdvanceCommitIndex,
  OA_AppendEntries, OA_UpdateTerm, OA_HandleRequestVoteRequest, OA_DropStaleResponse,
  OA_HandleRequestVoteResponse, OA_HandleAppendEntriesRequest, OA_HandleAppendEntriesResponse,
  OA_DuplicateMessage, OA_DropMessage, OA_NACT
};
static const char* const kOrigActNames[OA_NACT] = {
    "Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex",
    "AppendEntries", "UpdateTerm", "HandleRequestVoteRequest", "DropStaleResponse",
    "HandleRequestVoteResponse", "HandleAppendEntriesRequest", "HandleAppendEntriesResponse",
    "DuplicateMessage", "DropMessage"};

// constraint / invariant selection bits (resolved from cfg names on the host)
enum { OC_BoundedTerms = 1, OC_BoundedLogs = 2, OC_BoundedMessages = 4 };
enum { OI_ElectionSafety = 1, OI_LogMatching = 2, OI_NoLeader = 4, OI_NoCommit = 8 };
static const char* const kOrigInvNames[4] = {"ElectionSafety", "LogMatching", "NoLeader", "NoCommit"};
// OI_* bit of an invariant name (configs/raft_original_mc.tla), 0 if unknown
inline u32 orig_inv_bit(const char* n) {
  for (int k = 0; k < 4; ++k) {
    const char* a = kOrigInvNames[k]; const char* b = n;
    while (*a && *a == *b) { ++a; ++b; }
    if (!*a && !*b) return 1u << k;
  }
  return 0;
}

// error flags raised by the successor function (TLC evaluation errors / capacity)
enum { OE_EVAL_LOG_INDEX = 1, OE_CAP_ELECTIONS = 2, OE_CAP_COUNT = 4 };

struct OrigRuntime {
  int min_count, max_count;   // MinMsgCount..MaxMsgCount
  u32 constraints;            // OC_* mask
  u32 invariants;             // OI_* mask (cfg order kept on host)
};

template <int N_, int NV_, int MT_, int ML_, int MK_>
struct Orig {
  static constexpr int N = N_, NV = NV_, MT = MT_, ML = ML_, MK = MK_;
  // ---- widths
  static constexpr int SB = bits_for(N - 1);        // server id 0..N-1
  static constexpr int VB = bits_for(N);            // votedFor 0..N (N = Nil)
  static constexpr int TB = bits_for(MT + 1);       // terms 0..MT+1 (transient MT+1)
  static constexpr int E = MT * NV;                 // entry kinds: (term, value)
  static constexpr int EB = bits_for(E);            // entry code 0 (none) / 1..E
  static constexpr int LLB = bits_for(ML + 1);      // working log length 0..ML+1
  static constexpr int SLLB = bits_for(ML);         // stored log length 0..ML
  static constexpr int CIB = bits_for(ML);          // commitIndex / matchIndex / indices 0..ML
  static constexpr int NIB = bits_for(ML + 1);      // nextIndex 1..ML+1
  static constexpr long long U = log_universe(E, ML);   // number of logs of length <= ML
  static constexpr int LIB = bits_for(U - 1);       // log universe index 0..U-1
  static constexpr int AW = (int)((U + 63) / 64);   // allLogs bitmap words
  static constexpr int EMAX = MT;                   // elections capacity (one per (term, leader))
  static constexpr int VLB = 1 + LIB;               // voterLog cell: present bit + log index
  static constexpr int CNTB = 4;                    // message count field (count + 8)
  // message code: class(2) << BODY | body, ORDER PRESERVING (see "messages" below)
  static constexpr int BODY_RVQ = SB + CIB + TB + SB + TB, BODY_RVP = SB + LIB + SB + TB + 1,
                       BODY_AEP = SB + CIB + SB + 1 + TB, BODY_AEQ = CIB + SB + EB + LIB + CIB + TB + SB + TB;
  static constexpr int BODY_A = BODY_RVQ > BODY_RVP ? BODY_RVQ : BODY_RVP, BODY_B = BODY_AEP > BODY_AEQ ? BODY_AEP : BODY_AEQ;
  static constexpr int BODY = BODY_A > BODY_B ? BODY_A : BODY_B;
  static constexpr int MSGB = 2 + BODY;
  static constexpr int ENTB = MSGB + CNTB;          // bag entry width
  using BE = typename std::conditional<(ENTB <= 31), u32, u64>::type;   // bag entry register type
  using MC = typename std::conditional<(MSGB <= 32), u32, u64>::type;   // message code register type
  using VR = typename std::conditional<(N * VLB <= 32), u32, u64>::type;   // voterLog row register type
  // election record [eterm, eleader, elog, evotes, evoterLog] (raft_original.tla:236-241).  When
  // the full voterLog row does not fit 64 bits (5 servers with 2 values: 69 bits), the row's
  // per-cell presence bits are left out: DOMAIN voterLog[i] = votesGranted[i] in every reachable
  // state (both change together in HandleRequestVoteResponse :313-318 and are emptied together by
  // Init, Restart and Timeout), so evotes already holds them; BecomeLeader checks the identity
  // and raises a capacity error if it ever failed (never a silent loss).
  // The compact form also stores eterm in bits_for(MT): BecomeLeader's parent is in the model, so
  // its term is <= MaxTerm (checked, like the voterLog identity).
  static constexpr bool ECOMPACT = TB + SB + LIB + N + N * VLB > 64;
  static constexpr int ETB = ECOMPACT ? bits_for(MT) : TB;        // eterm in a record
  static constexpr int EVB = ECOMPACT ? LIB : VLB;                // evoterLog cell in a record
  static constexpr int ELB = ETB + SB + LIB + N + N * EVB;        // election record width
  // ---- packed (stored) layout
  static constexpr int PBITS = N * TB + N * 2 + N * VB + N * CIB + N * N + N * N + N * N * NIB + N * N * CIB +
                               N * (SLLB + ML * EB) + N * N * VLB + (int)U + EMAX * ELB + MK * ENTB;
  static constexpr int NW = (PBITS + 31) / 32;      // u32 words per stored state
  static constexpr int BAG_OFF = PBITS - MK * ENTB; // bit offset of bag entry 0 (its count: the low CNTB bits)
  static constexpr int NI = 3 * N + 2 * N * N + N * NV + N + 3 * MK;   // action instances per state
  // the instances that need a Leader (ClientRequest, AdvanceCommitIndex, AppendEntries) or a
  // Candidate holding a quorum (BecomeLeader): one contiguous range [LEAD_LO, LEAD_HI) of apply's
  // order; rare states (C2: ~1% of the frontier), so the generate kernel skips the range and a
  // second pass runs it on full waves of just those parents (leader_work)
  static constexpr int LEAD_LO = 2 * N + N * N, LEAD_HI = LEAD_LO + N + N * NV + N + N * N;
  static constexpr int I_RECV = LEAD_HI, I_DUP = I_RECV + MK, I_DROP = I_DUP + MK;   // Receive / Duplicate / Drop

  static_assert(N >= 1 && N <= 7, "N");
  static_assert(N * TB <= 32 && N * VB <= 32 && N * CIB <= 32 && N * N <= 32, "scalar field words");
  static_assert(N * NIB <= 32 && N * CIB <= 32, "index rows");
  static_assert(LLB + (ML + 1) * EB <= 32, "working log word");
  static_assert(N * VLB <= 64, "voterLog row");
  static_assert(MSGB + CNTB <= 64, "message codes");
  static_assert(ELB <= 64, "election codes");

  struct Work {
    u32 term, st, voted, commit, vresp, vgrant;
    Arr<u32, N> nexti, matchi, log;
    Arr<VR, N> vl;
    u64 allLogs[AW];
    u64 el[EMAX];
    Arr<BE, MK + 1> bag;
  };
  static constexpr u32 F = 0, C = 1, L = 2;   // Follower, Candidate, Leader

  // ---------------------------------------------------------------- logs
  RMC_HD static int llen(u32 lw) { return (int)(lw & lomask(LLB)); }
  RMC_HD static int lent(u32 lw, int p) { return (int)((lw >> (LLB + p * EB)) & lomask(EB)); }   // 0-based p
  RMC_HD static int eterm(int e) { return e == 0 ? 0 : (e - 1) / NV + 1; }
  RMC_HD static int evalue(int e) { return (e - 1) % NV; }
  RMC_HD static int ecode(int term, int v) { return (term - 1) * NV + v + 1; }
  RMC_HD static int last_term(u32 lw) { int n = llen(lw); return n == 0 ? 0 : eterm(lent(lw, n - 1)); }
  RMC_HD static u32 lappend(u32 lw, int e) {
    int n = llen(lw);
    lw |= (u32)e << (LLB + n * EB);
    return (lw & ~(u32)lomask(LLB)) | (u32)(n + 1);
  }
  RMC_HD static u32 ldrop_last(u32 lw) {
    int n = llen(lw);
    lw &= ~((u32)lomask(EB) << (LLB + (n - 1) * EB));
    return (lw & ~(u32)lomask(LLB)) | (u32)(n - 1);
  }
  // universe index of a log of length <= ML (mixed radix over entry codes)
  RMC_HD static u32 lidx(u32 lw) {
    int n = llen(lw);
    u32 off = 0, pw = 1, d = 0;
#pragma unroll
    for (int k = 0; k < ML + 1; ++k) { if (k < n) { off += pw; pw *= (u32)E; } }
#pragma unroll
    for (int p = 0; p < ML + 1; ++p) if (p < n) d = d * (u32)E + (u32)(lent(lw, p) - 1);
    return off + d;
  }
  // host: index -> working log
  static u32 lfrom_idx(u32 idx) {
    u32 off = 0, pw = 1; int n = 0;
    while (n <= ML && idx >= off + pw) { off += pw; pw *= (u32)E; ++n; }
    u32 d = idx - off, lw = 0;
    int ent[ML + 2];
    for (int p = n - 1; p >= 0; --p) { ent[p] = (int)(d % (u32)E) + 1; d /= (u32)E; }
    for (int p = 0; p < n; ++p) lw = lappend(lw, ent[p]);
    return lw;
  }

  // ---------------------------------------------------------------- messages
  // The code is ORDER PRESERVING: numeric order of codes == the order of the message records
  // as TLA+ values (the oracle's value order, oracle/tla.h cmp: records by field count, then
  // field names, then field values in field-name order; sequences by length, then elements;
  // model values by their TLC intern order = the server index).  The bag is kept sorted by
  // code, so bag slot order is the enumeration order of `\E m \in DOMAIN messages` (Next,
  // raft_original.tla:460-462) and the instance index of a successor is its position in TLC's
  // single-worker FIFO order — the key the GPU uses to pick TLC's first-found parent and stop
  // point.  Field-name order of the four record shapes (raft_original.tla:191-197, 213-223,
  // 295-301, 352-357/368-373):
  //   RequestVoteRequest   mdest, mlastLogIndex, mlastLogTerm, msource, mterm, mtype   (6)
  //   RequestVoteResponse  mdest, mlog, msource, mterm, mtype, mvoteGranted            (6)
  //   AppendEntriesResp.   mdest, mmatchIndex, msource, msuccess, mterm, mtype         (6)
  //   AppendEntriesReq.    mcommitIndex, mdest, mentries, mlog, mprevLogIndex,
  //                        mprevLogTerm, msource, mterm, mtype                          (9)
  // so the class order is RVQ < RVP < AEP (second field name "mla" < "mlo" < "mma") < AEQ (more
  // fields); mtype is constant within a class.  Bodies are MSB-first in field-name order.
  enum { RVQ = 0, RVP = 1, AEP = 2, AEQ = 3 };
  RMC_HD static int mtype(MC c) { return (int)(c >> BODY); }
  RMC_HD static u32 fld(MC c, int off, int w) { return (u32)((c >> off) & (MC)lomask(w)); }
  // offsets from bit 0 (the last field of each body is its least significant)
  RMC_HD static int mterm(MC c) { return (int)fld(c, mtype(c) == RVP ? 1 : 0, TB); }
  RMC_HD static int msrc(MC c) { const int t = mtype(c); return (int)fld(c, TB + ((t == RVP || t == AEP) ? 1 : 0), SB); }
  RMC_HD static int mdst(MC c) {
    const int t = mtype(c);
    const int off = t == RVQ ? TB + SB + TB + CIB : t == RVP ? 1 + TB + SB + LIB : t == AEP ? TB + 1 + SB + CIB
                                                                                             : TB + SB + TB + CIB + LIB + EB;
    return (int)fld(c, off, SB);
  }
  RMC_HD static int rvq_llt(MC c) { return (int)fld(c, TB + SB, TB); }
  RMC_HD static int rvq_lli(MC c) { return (int)fld(c, TB + SB + TB, CIB); }
  RMC_HD static int rvp_granted(MC c) { return (int)fld(c, 0, 1); }
  RMC_HD static u32 rvp_log(MC c) { return (u32)fld(c, 1 + TB + SB, LIB); }
  RMC_HD static int aep_success(MC c) { return (int)fld(c, TB, 1); }
  RMC_HD static int aep_mmi(MC c) { return (int)fld(c, TB + 1 + SB, CIB); }
  RMC_HD static int aeq_plt(MC c) { return (int)fld(c, TB + SB, TB); }
  RMC_HD static int aeq_pli(MC c) { return (int)fld(c, TB + SB + TB, CIB); }
  RMC_HD static u32 aeq_log(MC c) { return (u32)fld(c, TB + SB + TB + CIB, LIB); }
  RMC_HD static int aeq_ent(MC c) { return (int)fld(c, TB + SB + TB + CIB + LIB, EB); }
  RMC_HD static int aeq_mci(MC c) { return (int)fld(c, TB + SB + TB + CIB + LIB + EB + SB, CIB); }
  RMC_HD static MC m_rvq(int term, int llt, int lli, int src, int dst) {
    MC b = (MC)dst;
    b = (b << CIB) | (MC)lli; b = (b << TB) | (MC)llt; b = (b << SB) | (MC)src; b = (b << TB) | (MC)term;
    return ((MC)RVQ << BODY) | b;
  }
  RMC_HD static MC m_rvp(int term, bool granted, u32 logidx, int src, int dst) {
    MC b = (MC)dst;
    b = (b << LIB) | (MC)logidx; b = (b << SB) | (MC)src; b = (b << TB) | (MC)term; b = (b << 1) | (MC)granted;
    return ((MC)RVP << BODY) | b;
  }
  RMC_HD static MC m_aeq(int term, int pli, int plt, int entry, u32 logidx, int commit, int src, int dst) {
    MC b = (MC)commit;
    b = (b << SB) | (MC)dst; b = (b << EB) | (MC)entry; b = (b << LIB) | (MC)logidx; b = (b << CIB) | (MC)pli;
    b = (b << TB) | (MC)plt; b = (b << SB) | (MC)src; b = (b << TB) | (MC)term;
    return ((MC)AEQ << BODY) | b;
  }
  RMC_HD static MC m_aep(int term, bool success, int mmi, int src, int dst) {
    MC b = (MC)dst;
    b = (b << CIB) | (MC)mmi; b = (b << SB) | (MC)src; b = (b << 1) | (MC)success; b = (b << TB) | (MC)term;
    return ((MC)AEP << BODY) | b;
  }
  // bag entries: code << CNTB | (count + 8); all ones = empty; kept sorted ascending.  32-bit
  // entries when they fit (C2: 29 bits), halving the bag's compare / select work
  static constexpr u64 EMPTY = ~0ull;
  static constexpr BE BEMPTY = (BE)~(BE)0;
  RMC_HD static MC ecode_of(BE ent) { return (MC)(ent >> CNTB); }
  RMC_HD static int ecount(BE ent) { return (int)((u64)ent & lomask(CNTB)) - 8; }
  // WithMessage (raft_original.tla:106-110)
  RMC_HD static void with_msg(Arr<BE, MK + 1>& bag, MC code, u32& err) {
    bool found = false;
#pragma unroll
    for (int k = 0; k < MK + 1; ++k) {
      if (bag.v[k] != BEMPTY && ecode_of(bag.v[k]) == code) {
        found = true;
        int c = ecount(bag.v[k]) + 1;
        if (c > 7) err |= OE_CAP_COUNT;
        bag.v[k] = (BE)(((BE)code << CNTB) | (BE)(c + 8));
      }
    }
    if (!found) {
      const BE x = (BE)(((BE)code << CNTB) | (BE)(1 + 8));
      if (bag.v[MK] != BEMPTY) err |= OE_CAP_COUNT;   // cannot happen from an in-model pre-state
      BE prev = 0; bool prev_lt = true;
#pragma unroll
      for (int k = 0; k < MK + 1; ++k) {
        const BE cur = bag.v[k];
        const bool cur_lt = cur < x;
        bag.v[k] = cur_lt ? cur : (prev_lt ? x : prev);
        prev = cur; prev_lt = cur_lt;
      }
    }
  }
  // WithoutMessage (raft_original.tla:114-118): decrement, entry stays (G1)
  RMC_HD static void without_msg(Arr<BE, MK + 1>& bag, MC code, u32& err) {
#pragma unroll
    for (int k = 0; k < MK + 1; ++k) {
      if (bag.v[k] != BEMPTY && ecode_of(bag.v[k]) == code) {
        int c = ecount(bag.v[k]) - 1;
        if (c < -8) err |= OE_CAP_COUNT;
        bag.v[k] = (BE)(((BE)code << CNTB) | (BE)(c + 8));
      }
    }
  }

  // the count of the message in bag slot k (k uniform: a select chain, no code search) changed by
  // delta: WithoutMessage (-1, G1: may go negative, the entry stays) / WithMessage of a message
  // already in the bag (+1) when the caller knows its slot
  RMC_HD static void bag_add_at(Arr<BE, MK + 1>& bag, int k, int delta, u32& err) {
    const BE e = sel(bag, k);
    const int c = ecount(e) + delta;
    if (c < -8 || c > 7) err |= OE_CAP_COUNT;
    put(bag, k, (BE)((e & ~(BE)lomask(CNTB)) | (BE)((c + 8) & (int)lomask(CNTB))));
  }

  // ---------------------------------------------------------------- per-server fields
  RMC_HD static int g_term(const Work& s, int i) { return (int)fget<TB>(s.term, i); }
  RMC_HD static int g_st(const Work& s, int i) { return (int)fget<2>(s.st, i); }
  RMC_HD static int g_voted(const Work& s, int i) { return (int)fget<VB>(s.voted, i); }
  RMC_HD static int g_commit(const Work& s, int i) { return (int)fget<CIB>(s.commit, i); }
  RMC_HD static u32 row_bits(u32 x, int i) { return (x >> (i * N)) & (u32)lomask(N); }
  RMC_HD static void set_row_bits(u32& x, int i, u32 v) { fset<N>(x, i, v); }
  RMC_HD static int g_ni(const Work& s, int i, int j) { return (int)fget<NIB>(sel(s.nexti, i), j); }
  RMC_HD static int g_mi(const Work& s, int i, int j) { return (int)fget<CIB>(sel(s.matchi, i), j); }
  RMC_HD static void s_ni(Work& t, int i, int j, int v) { u32 r = sel(t.nexti, i); fset<NIB>(r, j, (u32)v); put(t.nexti, i, r); }
  RMC_HD static void s_mi(Work& t, int i, int j, int v) { u32 r = sel(t.matchi, i); fset<CIB>(r, j, (u32)v); put(t.matchi, i, r); }

  // ---------------------------------------------------------------- Init (raft_original.tla:139-159)
  RMC_HD static void init(Work& s) {
    s.term = fsplat<TB, u32>(1, N); s.st = 0; s.voted = fsplat<VB, u32>((u32)N, N); s.commit = 0;
    s.vresp = 0; s.vgrant = 0;
    for (int i = 0; i < N; ++i) { s.nexti.v[i] = fsplat<NIB, u32>(1, N); s.matchi.v[i] = 0; s.log.v[i] = 0; s.vl.v[i] = 0; }
    for (int k = 0; k < AW; ++k) s.allLogs[k] = 0;
    for (int k = 0; k < EMAX; ++k) s.el[k] = EMPTY;
    for (int k = 0; k < MK + 1; ++k) s.bag.v[k] = BEMPTY;
  }

  // allLogs' = allLogs \cup {log[i] : i \in Server} (raft_original.tla:464, G3): same for every successor
  RMC_HD static void all_logs_next(const Work& s, u64 (&al)[AW]) {
#pragma unroll
    for (int k = 0; k < AW; ++k) al[k] = s.allLogs[k];
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const u32 ix = lidx(s.log.v[i]);
#pragma unroll
      for (int k = 0; k < AW; ++k) if ((int)(ix >> 6) == k) al[k] |= 1ull << (ix & 63);
    }
  }

  // true iff some instance in [LEAD_LO, LEAD_HI) can be enabled in s: a Leader (ClientRequest,
  // AdvanceCommitIndex, AppendEntries) or a Candidate with a vote quorum (BecomeLeader :228-231)
  RMC_HD static bool leader_work(const Work& s) {
    bool any = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int st = g_st(s, i);
      any |= st == L || (st == C && popc32(row_bits(s.vgrant, i)) * 2 > N);
    }
    return any;
  }

  // ---------------------------------------------------------------- instance families (generate's binning)
  // Which instances of a family can be enabled in s, as a bit mask over the family's instances: a
  // superset of those apply() enables (apply decides).  The generate kernel runs a family's set
  // bits one per iteration on every lane at once, so the lanes of an iteration share one handler
  // (SURVEY.md §7 hard part 8) and a lane with nothing left of a family costs no iterations.
  RMC_HD static u32 timeout_mask(const Work& s) {   // Timeout(i) :177-186: a Follower or Candidate
    u32 m = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) { const int st = g_st(s, i); m |= (st == (int)F || st == (int)C) ? 1u << i : 0u; }
    return m;
  }
  RMC_HD static u32 request_vote_mask(const Work& s) {   // RequestVote(i, j) :189-198: i a Candidate, j not responded
    u32 m = 0;
#pragma unroll
    for (int i = 0; i < N; ++i)
      if (g_st(s, i) == (int)C) m |= ((~row_bits(s.vresp, i)) & (u32)lomask(N)) << (i * N);
    return m;
  }
  // Receive(m) of bag slot km: -1 empty slot, 0 UpdateTerm (m.mterm > currentTerm[m.mdest], which
  // excludes every handler), else 1 + the message type (each type its own handler, :283-402)
  RMC_HD static int recv_class(const Work& s, int km) {
    const BE ent = sel(s.bag, km);
    if (ent == BEMPTY) return -1;
    const MC m = ecode_of(ent);
    return mterm(m) > g_term(s, mdst(m)) ? 0 : 1 + mtype(m);
  }
  static constexpr int RECV_CLASSES = 5;

  // DuplicateMessage(m) / DropMessage(m) change one message count and nothing else (:442-449): the
  // successor is out of the model iff BoundedMessages puts that count outside [MinMsgCount,
  // MaxMsgCount], and no invariant reads the bag (inv_frame).  Returns the action when instance k
  // (wave-uniform) yields such a successor, so the kernel counts it without building it (C2: most of
  // the 266M duplicates); -1 otherwise (apply decides).
  RMC_HD static int quick_out_of_model(const Work& s, int k, const OrigRuntime& rt) {
    if (k < I_DUP || !(rt.constraints & OC_BoundedMessages)) return -1;
    const bool dup = k < I_DROP;
    const BE ent = sel(s.bag, dup ? k - I_DUP : k - I_DROP);
    if (ent == BEMPTY) return -1;
    const int c = ecount(ent) + (dup ? 1 : -1);
    return (c < rt.min_count || c > rt.max_count) ? (dup ? (int)OA_DuplicateMessage : (int)OA_DropMessage) : -1;
  }

  // ---------------------------------------------------------------- instance -> successor
  // Returns the OrigAct id of the successor written to t, or -1 when instance
  // k is disabled in s.  Instances (uniform across a wave): Restart(i) N,
  // Timeout(i) N, RequestVote(i,j) N^2, BecomeLeader(i) N, ClientRequest(i,v)
  // N*NV, AdvanceCommitIndex(i) N, AppendEntries(i,j) N^2, Receive(slot) MK,
  // DuplicateMessage(slot) MK, DropMessage(slot) MK (Next, :453-462).
  RMC_HD static int apply(const Work& s, int k, Work& t, u32& err) {
    t = s;
    if (k < N) {                                                   // Restart(i) :166-174
      const int i = k;
      fset<2>(t.st, i, F);
      set_row_bits(t.vresp, i, 0); set_row_bits(t.vgrant, i, 0);
      put(t.vl, i, (VR)0);
      put(t.nexti, i, fsplat<NIB, u32>(1, N));
      put(t.matchi, i, (u32)0);
      fset<CIB>(t.commit, i, 0u);
      return OA_Restart;
    }
    k -= N;
    if (k < N) {                                                   // Timeout(i) :177-186
      const int i = k, st = g_st(s, i);
      if (!(st == F || st == C)) return -1;
      fset<2>(t.st, i, C);
      fset<TB>(t.term, i, (u32)(g_term(s, i) + 1));
      fset<VB>(t.voted, i, (u32)N);
      set_row_bits(t.vresp, i, 0); set_row_bits(t.vgrant, i, 0);
      put(t.vl, i, (VR)0);
      return OA_Timeout;
    }
    k -= N;
    if (k < N * N) return request_vote(s, k / N, k % N, t, err);   // RequestVote(i, j) :189-198
    k -= N * N;
    if (k < N) {                                                   // BecomeLeader(i) :228-242
      const int i = k;
      if (g_st(s, i) != C) return -1;
      const u32 vg = row_bits(s.vgrant, i);
      if (!(popc32(vg) * 2 > N)) return -1;
      fset<2>(t.st, i, L);
      const u32 li = sel(s.log, i);
      put(t.nexti, i, fsplat<NIB, u32>((u32)(llen(li) + 1), N));
      put(t.matchi, i, (u32)0);
      if (g_term(s, i) > (int)lomask(ETB)) err |= OE_CAP_ELECTIONS;
      const u64 rec = (u64)g_term(s, i) | ((u64)i << ETB) | ((u64)lidx(li) << (ETB + SB)) | ((u64)vg << (ETB + SB + LIB)) |
                      (evoter_code((u64)sel(s.vl, i), vg, err) << (ETB + SB + LIB + N));
      set_insert(t.el, rec, err);
      return OA_BecomeLeader;
    }
    k -= N;
    if (k < N * NV) {                                              // ClientRequest(i, v) :245-252
      const int i = k / NV, v = k % NV;
      if (g_st(s, i) != L) return -1;
      put(t.log, i, lappend(sel(s.log, i), ecode(g_term(s, i), v)));
      return OA_ClientRequest;
    }
    k -= N * NV;
    if (k < N) {                                                   // AdvanceCommitIndex(i) :258-275
      const int i = k;
      if (g_st(s, i) != L) return -1;
      const u32 li = sel(s.log, i), mrow = sel(s.matchi, i);
      const int n = llen(li);
      int best = 0;
#pragma unroll
      for (int index = 1; index <= ML + 1; ++index) {
        if (index > n) continue;
        u32 agree = 1u << i;                                       // Agree(index) == {i} \cup {k : matchIndex[i][k] >= index}
#pragma unroll
        for (int q = 0; q < N; ++q) if ((int)fget<CIB>(mrow, q) >= index) agree |= 1u << q;
        if (popc32(agree) * 2 > N) best = index;                   // Max(agreeIndexes)
      }
      int nci = g_commit(s, i);
      if (best > 0 && eterm(lent(li, best - 1)) == g_term(s, i)) nci = best;
      fset<CIB>(t.commit, i, (u32)nci);
      return OA_AdvanceCommitIndex;
    }
    k -= N;
    if (k < N * N) {                                               // AppendEntries(i, j) :203-225
      const int i = k / N, j = k % N;
      if (i == j || g_st(s, i) != L) return -1;
      const u32 li = sel(s.log, i);
      const int n = llen(li), ni = g_ni(s, i, j), pli = ni - 1;
      int plt = 0;
      if (pli > 0) {
        if (pli > n) { err |= OE_EVAL_LOG_INDEX; return -1; }     // log[i][prevLogIndex] out of domain (unguarded :207-210)
        plt = eterm(lent(li, pli - 1));
      }
      const int lastEntry = n < ni ? n : ni;
      const int entry = (ni <= lastEntry) ? lent(li, ni - 1) : 0;  // SubSeq(log[i], nextIndex, lastEntry): <= 1 entry
      const int ci = g_commit(s, i);
      with_msg(t.bag, m_aeq(g_term(s, i), pli, plt, entry, lidx(li), ci < lastEntry ? ci : lastEntry, i, j), err);
      return OA_AppendEntries;
    }
    k -= N * N;
    if (k < MK) {                                                  // Receive(m) :420-435
      const BE ent = sel(s.bag, k);
      if (ent == BEMPTY) return -1;
      return receive(s, k, ecode_of(ent), t, err);
    }
    k -= MK;
    if (k < MK) {                                                  // DuplicateMessage(m) :442-444
      const BE ent = sel(s.bag, k);
      if (ent == BEMPTY) return -1;
      bag_add_at(t.bag, k, +1, err);                               // WithMessage of a message in slot k
      return OA_DuplicateMessage;
    }
    k -= MK;
    {                                                              // DropMessage(m) :447-449
      const BE ent = sel(s.bag, k);
      if (ent == BEMPTY) return -1;
      bag_add_at(t.bag, k, -1, err);                               // WithoutMessage (G1)
      return OA_DropMessage;
    }
  }

  // RequestVote(i, j) (raft_original.tla:189-198) into t (= s on entry); i, j may differ per lane
  // (orig_generate's per-lane RequestVote section)
  RMC_HD static int request_vote(const Work& s, int i, int j, Work& t, u32& err) {
    if (g_st(s, i) != C) return -1;
    if ((row_bits(s.vresp, i) >> j) & 1u) return -1;
    const u32 li = sel(s.log, i);
    with_msg(t.bag, m_rvq(g_term(s, i), last_term(li), llen(li), i, j), err);
    return OA_RequestVote;
  }

  // the evoterLog field of an election record from voterLog[i]'s row (see ECOMPACT)
  RMC_HD static u64 evoter_code(u64 row, u32 vg, u32& err) {
    if constexpr (!ECOMPACT) { (void)vg; (void)err; return row; }
    u64 c = 0;
    u32 pres = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      pres |= (u32)((row >> (j * VLB)) & 1ull) << j;
      c |= ((row >> (j * VLB + 1)) & lomask(LIB)) << (j * LIB);
    }
    if (pres != vg) err |= OE_CAP_ELECTIONS;
    return c;
  }
  // ... and back to a voterLog row (text, traces)
  RMC_HD static u64 evoter_row(u64 code, u32 evotes) {
    if constexpr (!ECOMPACT) { (void)evotes; return code; }
    u64 row = 0;
#pragma unroll
    for (int j = 0; j < N; ++j)
      if ((evotes >> j) & 1u) row |= ((((code >> (j * LIB)) & lomask(LIB)) << 1) | 1ull) << (j * VLB);
    return row;
  }
  RMC_HD static void set_insert(u64 (&el)[EMAX], u64 x, u32& err) {   // elections' = elections \cup {x}
    bool found = false;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) found |= el[k] == x;
    if (found) return;
    if (el[EMAX - 1] != EMPTY) { err |= OE_CAP_ELECTIONS; return; }
    u64 prev = 0; bool prev_lt = true;
#pragma unroll
    for (int k = 0; k < EMAX; ++k) {
      const u64 cur = el[k]; const bool cur_lt = cur < x;
      el[k] = cur_lt ? cur : (prev_lt ? x : prev);
      prev = cur; prev_lt = cur_lt;
    }
  }

  // Receive(m): UpdateTerm excludes every handler (they need mterm <= currentTerm), so <= 1 successor.
  // m is the message in bag slot km: its own count is changed in place (before any reply is
  // inserted, which can shift the slots), the reply goes through WithMessage's search
  RMC_HD static int receive(const Work& s, int km, MC m, Work& t, u32& err) {
    const int i = mdst(m), j = msrc(m), mt = mterm(m), ct = g_term(s, i), ty = mtype(m);
    if (mt > ct) {                                                 // UpdateTerm :405-411
      fset<TB>(t.term, i, (u32)mt);
      fset<2>(t.st, i, F);
      fset<VB>(t.voted, i, (u32)N);
      return OA_UpdateTerm;
    }
    const u32 li = sel(s.log, i);
    const int n = llen(li);
    if (ty == RVQ) {                                               // HandleRequestVoteRequest :283-302
      const int llt = rvq_llt(m), lli = rvq_lli(m), lt = last_term(li);
      const bool logOk = llt > lt || (llt == lt && lli >= n);
      const int vf = g_voted(s, i);
      const bool grant = mt == ct && logOk && (vf == N || vf == j);
      if (grant) fset<VB>(t.voted, i, (u32)j);
      bag_add_at(t.bag, km, -1, err);                              // Reply (:128-129): discard m ...
      with_msg(t.bag, m_rvp(ct, grant, lidx(li), i, j), err);      // ... and send the response
      return OA_HandleRequestVoteRequest;
    }
    if (ty == RVP) {
      if (mt < ct) { bag_add_at(t.bag, km, -1, err); return OA_DropStaleResponse; }   // :414-417
      set_row_bits(t.vresp, i, row_bits(s.vresp, i) | (1u << j));                 // HandleRequestVoteResponse :306-320
      if (rvp_granted(m)) {
        set_row_bits(t.vgrant, i, row_bits(s.vgrant, i) | (1u << j));
        VR row = sel(s.vl, i);
        if (!((row >> (j * VLB)) & 1ull))                                         // voterLog[i] @@ (j :> m.mlog): left-biased
          row |= (VR)((((u64)rvp_log(m) << 1) | 1ull) << (j * VLB));
        put(t.vl, i, row);
      }
      bag_add_at(t.bag, km, -1, err);
      return OA_HandleRequestVoteResponse;
    }
    if (ty == AEQ) {                                               // HandleAppendEntriesRequest :326-388
      const int pli = aeq_pli(m), plt = aeq_plt(m), ment = aeq_ent(m);
      const int mci = aeq_mci(m);
      const int st = g_st(s, i);
      const bool logOk = pli == 0 || (pli > 0 && pli <= n && plt == eterm(lent(li, pli - 1)));
      if (mt < ct || (st == F && !logOk)) {                        // reject request
        bag_add_at(t.bag, km, -1, err);
        with_msg(t.bag, m_aep(ct, false, 0, i, j), err);
        return OA_HandleAppendEntriesRequest;
      }
      if (st == C) { fset<2>(t.st, i, F); return OA_HandleAppendEntriesRequest; }   // return to follower state
      if (st == F) {                                               // accept request (logOk)
        const int index = pli + 1;
        if (ment == 0 || (n >= index && eterm(lent(li, index - 1)) == eterm(ment))) {   // already done
          fset<CIB>(t.commit, i, (u32)mci);
          bag_add_at(t.bag, km, -1, err);
          with_msg(t.bag, m_aep(ct, true, pli + (ment ? 1 : 0), i, j), err);
          return OA_HandleAppendEntriesRequest;
        }
        if (n >= index) { put(t.log, i, ldrop_last(li)); return OA_HandleAppendEntriesRequest; }   // conflict: remove 1 entry
        if (n == pli) { put(t.log, i, lappend(li, ment)); return OA_HandleAppendEntriesRequest; }  // no conflict: append
      }
      return -1;                                                   // Leader in the same term: nothing enabled
    }
    // AppendEntriesResponse
    if (mt < ct) { bag_add_at(t.bag, km, -1, err); return OA_DropStaleResponse; }
    {                                                              // HandleAppendEntriesResponse :392-402
      const int mmi = aep_mmi(m);
      if (aep_success(m)) { s_ni(t, i, j, mmi + 1); s_mi(t, i, j, mmi); }
      else { const int ni = g_ni(s, i, j); s_ni(t, i, j, ni - 1 > 1 ? ni - 1 : 1); }
      bag_add_at(t.bag, km, -1, err);
      return OA_HandleAppendEntriesResponse;
    }
  }

  // ---------------------------------------------------------------- constraints (configs/raft_original_mc.tla)
  RMC_HD static bool in_model(const Work& t, const OrigRuntime& rt) {
    bool ok = true;
    if (rt.constraints & OC_BoundedTerms) {
#pragma unroll
      for (int i = 0; i < N; ++i) ok &= g_term(t, i) <= MT;
    }
    if (rt.constraints & OC_BoundedLogs) {
#pragma unroll
      for (int i = 0; i < N; ++i) ok &= llen(t.log.v[i]) <= ML;
    }
    if (rt.constraints & OC_BoundedMessages) {
      ok &= t.bag.v[MK] == BEMPTY;
#pragma unroll
      for (int k = 0; k < MK; ++k) {
        const int c = ecount(t.bag.v[k]);
        ok &= t.bag.v[k] == BEMPTY || (c >= rt.min_count && c <= rt.max_count);
      }
    }
    return ok;
  }

  // ---------------------------------------------------------------- invariants; returns OI_* bit of the first violated (cfg order
  // is applied on the host by the order mask), 0 if all hold
  RMC_HD static u32 violated(const Work& t, u32 invs) {
    u32 bad = 0;
    if (invs & OI_ElectionSafety) {   // \A e, f \in elections : e.eterm = f.eterm => e.eleader = f.eleader
      bool ok = true;
#pragma unroll
      for (int a = 0; a < EMAX; ++a)
#pragma unroll
        for (int b = a + 1; b < EMAX; ++b)
          if (t.el[a] != EMPTY && t.el[b] != EMPTY && (t.el[a] & lomask(ETB)) == (t.el[b] & lomask(ETB)) &&
              ((t.el[a] >> ETB) & lomask(SB)) != ((t.el[b] >> ETB) & lomask(SB)))
            ok = false;
      if (!ok) bad |= OI_ElectionSafety;
    }
    if (invs & OI_LogMatching) {      // \A i,j, n <= min: log[i][n].term = log[j][n].term => prefixes equal
      bool ok = true;
#pragma unroll
      for (int a = 0; a < N; ++a)
#pragma unroll
        for (int b = a + 1; b < N; ++b) {
          const u32 x = t.log.v[a], y = t.log.v[b];
          const int nx = llen(x), ny = llen(y), mn = nx < ny ? nx : ny;
          bool pref = true;   // entries 1..n-1 equal so far
#pragma unroll
          for (int p = 0; p < ML + 1; ++p) {
            if (p < mn) {
              const int ex = lent(x, p), ey = lent(y, p);
              if (eterm(ex) == eterm(ey) && !(pref && ex == ey)) ok = false;
              pref = pref && ex == ey;
            }
          }
        }
      if (!ok) bad |= OI_LogMatching;
    }
    if (invs & OI_NoLeader) {
      bool ok = true;
#pragma unroll
      for (int i = 0; i < N; ++i) ok &= g_st(t, i) != L;
      if (!ok) bad |= OI_NoLeader;
    }
    if (invs & OI_NoCommit) {         // \A i \in Server : commitIndex[i] = 0 (test-only scenario invariant)
      if (t.commit != 0u) bad |= OI_NoCommit;
    }
    return bad;
  }

  // The invariants an action can change (a frame condition over raft_original.tla's variables):
  // ElectionSafety reads elections (written only by BecomeLeader :236-241), LogMatching reads log
  // (ClientRequest :248, HandleAppendEntriesRequest :360-384), NoLeader reads state (Restart,
  // Timeout, BecomeLeader, UpdateTerm, HandleAppendEntriesRequest), NoCommit reads commitIndex
  // (Restart, AdvanceCommitIndex, HandleAppendEntriesRequest).  Every expanded parent satisfies every
  // invariant (a new state that violates one stops the search at its level), so a successor can
  // only violate the invariants its action may change: the others need no evaluation.
  RMC_HD static u32 inv_frame(int act) {
    u32 m = 0;
    if (act == OA_BecomeLeader) m |= OI_ElectionSafety;
    if (act == OA_ClientRequest || act == OA_HandleAppendEntriesRequest) m |= OI_LogMatching;
    if (act == OA_Restart || act == OA_Timeout || act == OA_BecomeLeader || act == OA_UpdateTerm ||
        act == OA_HandleAppendEntriesRequest) m |= OI_NoLeader;
    if (act == OA_Restart || act == OA_AdvanceCommitIndex || act == OA_HandleAppendEntriesRequest) m |= OI_NoCommit;
    return m;
  }

  // ---------------------------------------------------------------- pack / unpack (canonical stored form)
  RMC_HD static void pack(const Work& t, u32 (&w)[NW]) {
    BitOut<NW> o;
    o.put(t.term, N * TB); o.put(t.st, N * 2); o.put(t.voted, N * VB); o.put(t.commit, N * CIB);
    o.put(t.vresp, N * N); o.put(t.vgrant, N * N);
#pragma unroll
    for (int i = 0; i < N; ++i) o.put(t.nexti.v[i], N * NIB);
#pragma unroll
    for (int i = 0; i < N; ++i) o.put(t.matchi.v[i], N * CIB);
#pragma unroll
    for (int i = 0; i < N; ++i) {     // stored log: len (SLLB) + ML entries
      const u32 lw = t.log.v[i];
      o.put((u64)(lw & lomask(LLB)), SLLB);
      o.put((u64)(lw >> LLB) & lomask(ML * EB), ML * EB);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) o.put(t.vl.v[i], N * VLB);
#pragma unroll
    for (int k = 0; k < AW; ++k) o.put(t.allLogs[k], (k == AW - 1) ? (int)(U - 64 * (AW - 1)) : 64);
#pragma unroll
    for (int k = 0; k < EMAX; ++k) o.put(t.el[k] == EMPTY ? 0ull : t.el[k], ELB);
#pragma unroll
    for (int k = 0; k < MK; ++k) o.put(t.bag.v[k] == BEMPTY ? 0ull : (u64)t.bag.v[k], ENTB);
#pragma unroll
    for (int k = 0; k < NW; ++k) w[k] = o.w[k];
  }
  // ---------------------------------------------------------------- field groups of the packed layout
  // (pack's order and widths): a successor differs from its parent in a few groups only, so its packed
  // words can be the parent's with those groups re-inserted (pack_patch) instead of a whole pack
  enum { PG_TERM, PG_ST, PG_VOTED, PG_COMMIT, PG_VRESP, PG_VGRANT, PG_NEXTI, PG_MATCHI, PG_LOG, PG_VL, PG_EL, PG_BAG, NPG };
  static constexpr int LOGW = SLLB + ML * EB;   // a stored log: length + ML entries
  static constexpr int OFF_TERM = 0, OFF_ST = OFF_TERM + N * TB, OFF_VOTED = OFF_ST + N * 2, OFF_COMMIT = OFF_VOTED + N * VB,
                       OFF_VRESP = OFF_COMMIT + N * CIB, OFF_VGRANT = OFF_VRESP + N * N, OFF_NEXTI = OFF_VGRANT + N * N,
                       OFF_MATCHI = OFF_NEXTI + N * N * NIB, OFF_LOG = OFF_MATCHI + N * N * CIB, OFF_VL = OFF_LOG + N * LOGW,
                       OFF_ALL = OFF_VL + N * N * VLB, OFF_EL = OFF_ALL + (int)U, OFF_BAG = OFF_EL + EMAX * ELB;
  static_assert(OFF_BAG == BAG_OFF && OFF_BAG + MK * ENTB == PBITS, "pack_patch offsets follow pack");
  // the groups instance k can change when its action is the same for every state (a superset; ~0u for
  // Receive, whose handler depends on the message: dirty_of decides per successor)
  RMC_HD static u32 dirty_static(int k) {
    if (k < N) return 1u << PG_ST | 1u << PG_VRESP | 1u << PG_VGRANT | 1u << PG_VL | 1u << PG_NEXTI | 1u << PG_MATCHI | 1u << PG_COMMIT;   // Restart
    if (k < 2 * N) return 1u << PG_ST | 1u << PG_TERM | 1u << PG_VOTED | 1u << PG_VRESP | 1u << PG_VGRANT | 1u << PG_VL;      // Timeout
    if (k < 2 * N + N * N) return 1u << PG_BAG;                                                                              // RequestVote
    if (k < 3 * N + N * N) return 1u << PG_ST | 1u << PG_NEXTI | 1u << PG_MATCHI | 1u << PG_EL;                              // BecomeLeader
    if (k < 3 * N + N * N + N * NV) return 1u << PG_LOG;                                                                     // ClientRequest
    if (k < 4 * N + N * N + N * NV) return 1u << PG_COMMIT;                                                                  // AdvanceCommitIndex
    if (k < I_RECV) return 1u << PG_BAG;                                                                                     // AppendEntries
    if (k < I_DUP) return ~0u;                                                                                               // Receive
    return 1u << PG_BAG;                                                                                                     // Duplicate / Drop
  }
  // the groups in which t differs from s (field compares)
  RMC_HD static u32 dirty_of(const Work& s, const Work& t) {
    u32 d = (t.term != s.term ? 1u << PG_TERM : 0u) | (t.st != s.st ? 1u << PG_ST : 0u) | (t.voted != s.voted ? 1u << PG_VOTED : 0u) |
            (t.commit != s.commit ? 1u << PG_COMMIT : 0u) | (t.vresp != s.vresp ? 1u << PG_VRESP : 0u) |
            (t.vgrant != s.vgrant ? 1u << PG_VGRANT : 0u);
    bool ni = false, mi = false, lg = false, vl = false, el = false, bg = false;
#pragma unroll
    for (int i = 0; i < N; ++i) { ni |= t.nexti.v[i] != s.nexti.v[i]; mi |= t.matchi.v[i] != s.matchi.v[i]; lg |= t.log.v[i] != s.log.v[i]; vl |= t.vl.v[i] != s.vl.v[i]; }
#pragma unroll
    for (int q = 0; q < EMAX; ++q) el |= t.el[q] != s.el[q];
#pragma unroll
    for (int q = 0; q < MK; ++q) bg |= t.bag.v[q] != s.bag.v[q];
    return d | (ni ? 1u << PG_NEXTI : 0u) | (mi ? 1u << PG_MATCHI : 0u) | (lg ? 1u << PG_LOG : 0u) | (vl ? 1u << PG_VL : 0u) |
           (el ? 1u << PG_EL : 0u) | (bg ? 1u << PG_BAG : 0u);
  }
  // v (< 2^NB) into bits [P, P + NB) of w, the other bits kept (P, NB compile-time: shifts and masks only)
  template <int P, int NB>
  RMC_HD static void put_at(u32 (&w)[NW], u64 v) {
    constexpr int q = P >> 5, r = P & 31;
    constexpr u64 m = lomask(NB);
    w[q] = (w[q] & ~(u32)(m << r)) | (u32)(v << r);
    if constexpr (r + NB > 32) w[q + 1] = (w[q + 1] & ~(u32)(m >> (32 - r))) | (u32)(v >> (32 - r));
    if constexpr (r + NB > 64) w[q + 2] = (w[q + 2] & ~(u32)(m >> (64 - r))) | (u32)(v >> (64 - r));
  }
  template <int B, int E, class F>
  RMC_HD static void for_c(F&& f) { if constexpr (B < E) { f(std::integral_constant<int, B>{}); for_c<B + 1, E>(f); } }
  // pack(t) given base = pack of a state that equals t outside the groups of `dirty` (dirty is
  // wave-uniform on the device: each group is one scalar branch)
  RMC_HD static void pack_patch(const Work& t, u32 dirty, const u32 (&base)[NW], u32 (&w)[NW]) {
#pragma unroll
    for (int k = 0; k < NW; ++k) w[k] = base[k];
    if (dirty & 1u << PG_TERM) put_at<OFF_TERM, N * TB>(w, t.term);
    if (dirty & 1u << PG_ST) put_at<OFF_ST, N * 2>(w, t.st);
    if (dirty & 1u << PG_VOTED) put_at<OFF_VOTED, N * VB>(w, t.voted);
    if (dirty & 1u << PG_COMMIT) put_at<OFF_COMMIT, N * CIB>(w, t.commit);
    if (dirty & 1u << PG_VRESP) put_at<OFF_VRESP, N * N>(w, t.vresp);
    if (dirty & 1u << PG_VGRANT) put_at<OFF_VGRANT, N * N>(w, t.vgrant);
    if (dirty & 1u << PG_NEXTI) for_c<0, N>([&](auto ic) { constexpr int i = decltype(ic)::value; put_at<OFF_NEXTI + i * N * NIB, N * NIB>(w, t.nexti.v[i]); });
    if (dirty & 1u << PG_MATCHI) for_c<0, N>([&](auto ic) { constexpr int i = decltype(ic)::value; put_at<OFF_MATCHI + i * N * CIB, N * CIB>(w, t.matchi.v[i]); });
    if (dirty & 1u << PG_LOG)
      for_c<0, N>([&](auto ic) {
        constexpr int i = decltype(ic)::value;
        const u32 lw = t.log.v[i];
        put_at<OFF_LOG + i * LOGW, SLLB>(w, (u64)(lw & lomask(LLB)));
        put_at<OFF_LOG + i * LOGW + SLLB, ML * EB>(w, (u64)(lw >> LLB) & lomask(ML * EB));
      });
    if (dirty & 1u << PG_VL) for_c<0, N>([&](auto ic) { constexpr int i = decltype(ic)::value; put_at<OFF_VL + i * N * VLB, N * VLB>(w, (u64)t.vl.v[i]); });
    if (dirty & 1u << PG_EL) for_c<0, EMAX>([&](auto qc) { constexpr int q = decltype(qc)::value; put_at<OFF_EL + q * ELB, ELB>(w, t.el[q] == EMPTY ? 0ull : t.el[q]); });
    if (dirty & 1u << PG_BAG)
      for_c<0, MK>([&](auto qc) { constexpr int q = decltype(qc)::value; put_at<OFF_BAG + q * ENTB, ENTB>(w, t.bag.v[q] == BEMPTY ? 0ull : (u64)t.bag.v[q]); });
  }

  template <int M>
  RMC_HD static void unpack(const u32 (&w)[M], Work& t) {
    static_assert(M >= NW, "packed array too small");
    BitIn<M> in(w);
    t.term = (u32)in.get(N * TB); t.st = (u32)in.get(N * 2); t.voted = (u32)in.get(N * VB); t.commit = (u32)in.get(N * CIB);
    t.vresp = (u32)in.get(N * N); t.vgrant = (u32)in.get(N * N);
#pragma unroll
    for (int i = 0; i < N; ++i) t.nexti.v[i] = (u32)in.get(N * NIB);
#pragma unroll
    for (int i = 0; i < N; ++i) t.matchi.v[i] = (u32)in.get(N * CIB);
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const u32 len = (u32)in.get(SLLB);
      const u32 ents = (u32)in.get(ML * EB);
      t.log.v[i] = len | (ents << LLB);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) t.vl.v[i] = (VR)in.get(N * VLB);
#pragma unroll
    for (int k = 0; k < AW; ++k) t.allLogs[k] = in.get((k == AW - 1) ? (int)(U - 64 * (AW - 1)) : 64);
#pragma unroll
    for (int k = 0; k < EMAX; ++k) { const u64 x = in.get(ELB); t.el[k] = x ? x : EMPTY; }
#pragma unroll
    for (int k = 0; k < MK; ++k) { const u64 x = in.get(ENTB); t.bag.v[k] = x ? (BE)x : BEMPTY; }
    t.bag.v[MK] = BEMPTY;
  }
};

}  // namespace rmc
