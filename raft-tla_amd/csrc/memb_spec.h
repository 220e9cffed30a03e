// raftmc — tlc_membership/raft.tla (Ongaro + Ricketts + Amos/Zhang membership
// + Pirlea/Foo history) hand-compiled to fixed-width integer state, shared by
// the gfx950 kernels (memb_backend.hip) and the host decoder (memb_text.h).
//
// Shape parameters (compile time): N servers (|Server| <= 4), NV values and
// MK = message-bag capacity (2 * |Server|^2 = MaxInFlightMessages, raft.tla:30,
// G14).  The bounds MaxLogLength = 5, MaxTerms = 4, ... are operators of the
// spec itself (raft.tla:22-30) and size the fields; the cfg must enable the
// constraints that rely on them (memb_model.cpp checks).
//
// Representation choices:
//  * Messages are one u64 "code << CNTB | count" each; the code is ORDER
//    PRESERVING: numeric order of codes == the order of the message records
//    in the oracle's value model (records compare by field count, then field
//    names, then values in field-name order; sequences by length first).
//    The bag is kept sorted by code, so `\E m \in DOMAIN messages` visits
//    messages in the same order as the oracle's BFS (needed for TLC FIFO
//    first-found semantics under VIEW, SURVEY.md §7 hard part 2).
//  * `history` is not stored: VIEW vars (raft.cfg:30) excludes it from the
//    fingerprint, and every predicate that reads it (constraints :1105-1137,
//    scenario properties :1143-1278) is compiled to a fixed summary
//    automaton (h0/h1 below).
//  * Config values (SUBSET Server) in log entries are stored as their rank
//    in the oracle's set order (cardinality, then elements), so entry codes
//    are order preserving too; GetConfig converts ranks to masks.
//  * The fingerprint is symmetric: min over Permutations(Server) of a
//    permutation-aware hash of the VIEW (raft.tla:1281, raft.cfg:29), with
//    the bag hashed as a multiset sum so no re-sorting is needed per
//    permutation.  Equal fingerprints <=> same orbit of the view (up to
//    64-bit hash collisions, reported as TLC does).
#pragma once
// Cost attribution (RMC_FP_PROF builds only): wave cycles per stage of the TLC-mode fingerprint,
// summed into prof[stage] by one lane of each wave (memb_backend.hip RAFTMC fp profile)
#if defined(RMC_FP_PROF) && defined(__HIP_DEVICE_COMPILE__)
#define RMC_PROF_T() __builtin_readcyclecounter()
#define RMC_PROF_ADD(prof, i, t0)                                                                  \
  do {                                                                                             \
    const unsigned long long t1_ = __builtin_readcyclecounter();                                   \
    if ((prof) && __lane_id() == __ffsll((unsigned long long)__ballot(1)) - 1) atomicAdd(&(prof)[i], t1_ - (t0)); \
    (t0) = t1_;                                                                                    \
  } while (0)
#else
#define RMC_PROF_T() 0ull
#define RMC_PROF_ADD(prof, i, t0) do { (void)(prof); (void)(t0); } while (0)
#endif
// Host harness statistics (tests/native/memb_host_bfs.cpp built with -DRMC_FP_STATS): work counts of
// the TLC-mode canonical-permutation search
#if defined(RMC_FP_STATS) && !defined(__HIP_DEVICE_COMPILE__)
extern long long rmc_fp_stats[32];
#define RMC_FPS(i, v) (rmc_fp_stats[i] += (long long)(v))
#else
#define RMC_FPS(i, v) ((void)0)
#endif
#include "common.h"

namespace rmc {

enum MembAct {
  MA_RequestVote, MA_BecomeLeader, MA_ClientRequest, MA_AdvanceCommitIndex, MA_AppendEntries,
  MA_UpdateTerm, MA_HandleRequestVoteRequest, MA_DropStaleResponse, MA_HandleRequestVoteResponse,
  MA_HandleAppendEntriesRequest, MA_HandleAppendEntriesResponse, MA_HandleCatchupRequest,
  MA_HandleCatchupResponse, MA_HandleCheckOldConfig, MA_Timeout, MA_Restart,
  MA_DuplicateMessage, MA_DropMessage, MA_AddNewServer, MA_DeleteServer, MA_NACT
};
static const char* const kMembActNames[MA_NACT] = {
    "RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex", "AppendEntries",
    "UpdateTerm", "HandleRequestVoteRequest", "DropStaleResponse", "HandleRequestVoteResponse",
    "HandleAppendEntriesRequest", "HandleAppendEntriesResponse", "HandleCatchupRequest",
    "HandleCatchupResponse", "HandleCheckOldConfig", "Timeout", "Restart",
    "DuplicateMessage", "DropMessage", "AddNewServer", "DeleteServer"};

// state constraints, raft.tla:1105-1137 and :1182-1186
enum MembCon {
  MC_BoundedInFlightMessages, MC_BoundedRequestVote, MC_BoundedLogSize, MC_BoundedRestarts, MC_BoundedTimeouts,
  MC_BoundedTerms, MC_BoundedClientRequests, MC_BoundedTriedMembershipChanges, MC_BoundedMembershipChanges,
  MC_ElectionsUncontested, MC_CleanStartUntilFirstRequest, MC_CleanStartUntilTwoLeaders,
  MC_CommitWhenConcurrentLeaders_constraint, MC_CommitWhenConcurrentLeaders_unique, MC_MajorityOfClusterRestarts_constraint,
  MC_NCON
};
static const char* const kMembConNames[MC_NCON] = {
    "BoundedInFlightMessages", "BoundedRequestVote", "BoundedLogSize", "BoundedRestarts", "BoundedTimeouts",
    "BoundedTerms", "BoundedClientRequests", "BoundedTriedMembershipChanges", "BoundedMembershipChanges",
    "ElectionsUncontested", "CleanStartUntilFirstRequest", "CleanStartUntilTwoLeaders",
    "CommitWhenConcurrentLeaders_constraint", "CommitWhenConcurrentLeaders_unique",
    "MajorityOfClusterRestarts_constraint"};
// the punctuated-search prefix constraints (raft.tla:1198-1204, :1228-1234) in prefix-region order
static const int kPrefixCon[2] = {MC_CommitWhenConcurrentLeaders_unique, MC_MajorityOfClusterRestarts_constraint};
// action constraints, raft.tla:1207-1210
enum { MAC_CommitWhenConcurrentLeaders = 1 };

// invariants: Raft properties :969-1099 and scenario properties (negated goals) :1143-1278
enum MembInv {
  MI_LeaderVotesQuorum, MI_CandidateTermNotInLog, MI_ElectionSafety, MI_LogMatching, MI_VotesGrantedInv,
  MI_VotesGrantedInv_false, MI_QuorumLogInv, MI_MoreUpToDateCorrect, MI_LeaderCompleteness_false,
  MI_LeaderCompleteness, MI_BoundedTrace, MI_FirstBecomeLeader, MI_FirstCommit, MI_FirstRestart,
  MI_LeadershipChange, MI_MembershipChange, MI_MultipleMembershipChanges, MI_ConcurrentLeaders,
  MI_EntryCommitted, MI_CommitWhenConcurrentLeaders, MI_MajorityOfClusterRestarts, MI_AddSucessful,
  MI_MembershipChangeCommits, MI_MultipleMembershipChangesCommit, MI_AddCommits, MI_NewlyJoinedBecomeLeader,
  MI_LeaderChangesDuringConfChange, MI_NINV
};
static const char* const kMembInvNames[MI_NINV] = {
    "LeaderVotesQuorum", "CandidateTermNotInLog", "ElectionSafety", "LogMatching", "VotesGrantedInv",
    "VotesGrantedInv_false", "QuorumLogInv", "MoreUpToDateCorrect", "LeaderCompleteness_false",
    "LeaderCompleteness", "BoundedTrace", "FirstBecomeLeader", "FirstCommit", "FirstRestart",
    "LeadershipChange", "MembershipChange", "MultipleMembershipChanges", "ConcurrentLeaders",
    "EntryCommitted", "CommitWhenConcurrentLeaders", "MajorityOfClusterRestarts", "AddSucessful",
    "MembershipChangeCommits", "MultipleMembershipChangesCommit", "AddCommits", "NewlyJoinedBecomeLeader",
    "LeaderChangesDuringConfChange"};

// error flags: TLC evaluation error (a verdict) / compiled capacity exceeded
enum { ME_EVAL = 1, ME_CAP = 2 };
// NEXT relation pieces, raft.tla:909-943
enum { MN_ASYNC = 1, MN_CRASH = 2, MN_UNRELIABLE = 4, MN_DYNAMIC = 8 };
// outcome of one invariant on one state
enum { IV_OK = 0, IV_BAD = 1, IV_ERR = 2 };

struct MembRuntime {
  u32 constraints;          // 1 << MembCon
  u32 action_constraints;   // MAC_*
  u32 next;                 // MN_*
  u32 init_cfg;             // InitServer as a server mask
  u32 num_rounds;           // NumRounds (raft.cfg:11)
  u32 cfg_type;             // entry type bit of ConfigEntry (0 iff ConfigEntry sorts before ValueEntry)
  u32 symmetry;             // 1 = SYMMETRY perms
  u32 n_inv;                // invariants in cfg order
  u64 inv_order[4];         // invariant ids in cfg order, one byte each (read with selects, never a
                            // runtime-indexed array: that would put the kernel argument in scratch)
  // punctuated-search prefixes (region 0: CommitWhenConcurrentLeaders_unique, 1:
  // MajorityOfClusterRestarts_constraint): device tables of [position][binding] history-entry
  // codes (x, y), bindings = injective (s1, s2, s3) -> Server in lexicographic order; 0 length = off
  const u64* ptab0;
  const u64* ptab1;
  u32 plen0, plen1;
  u32 preg1_off;            // h1 bit offset of region 1's dead-binding mask
  u32 sym_tlc;              // SYMMETRY in TLC's mode (MC_COMPAT_SYM_TLC): least permuted full state, then VIEW
  u32 disjunct_copies;      // MC_COMPAT_DISJUNCT_COPIES: TLC's generated count of a disjunctive guard (tlc_copies)
};

// ------------------------------------------------------------------ small constexpr tables
// Config rank: subsets of {0..n-1} sorted by (cardinality, elements ascending) — the
// oracle's set order on sets of model values.  Packed as 4-bit nibbles (n <= 4).
constexpr long long subset_key(int m, int n) {
  long long key = 0; int c = 0;
  for (int k = 0; k < n; ++k) if ((m >> k) & 1) { key = key * 8 + k; ++c; }
  return (long long)c << 40 | key;
}
constexpr u64 mask_to_rank_lut(int n) {
  u64 lut = 0;
  for (int m = 0; m < (1 << n); ++m) {
    int r = 0;
    for (int x = 0; x < (1 << n); ++x) if (subset_key(x, n) < subset_key(m, n)) ++r;
    lut |= (u64)r << (4 * m);
  }
  return lut;
}
constexpr u64 rank_to_mask_lut(int n) {
  u64 m2r = mask_to_rank_lut(n), lut = 0;
  for (int m = 0; m < (1 << n); ++m) lut |= (u64)m << (4 * ((m2r >> (4 * m)) & 15));
  return lut;
}
constexpr int factorial(int n) { return n <= 1 ? 1 : n * factorial(n - 1); }

// Permutation tables in constant memory (a load each instead of a Lehmer decode or a 24-step
// scan per use in the symmetry code): perm[p] = the p-th permutation of N servers in Lehmer order,
// 2 bits per server; pos[s * 4 + l] = the permutations that send server s to l.
constexpr u32 lehmer_perm(int n, int p) {
  u32 avail = 0x3210u, pi = 0;
  int rem = p;
  for (int i = 0; i < n; ++i) {
    const int f = factorial(n - 1 - i), d = rem / f;
    rem -= d * f;
    pi |= ((avail >> (4 * d)) & 15u) << (2 * i);
    avail = (avail & (u32)lomask(4 * d)) | ((avail >> (4 * (d + 1))) << (4 * d));
  }
  return pi;
}
struct PermTables { u32 perm[24]; u32 pos[16]; };
constexpr PermTables make_perm_tables(int n) {
  PermTables t{};
  for (int p = 0; p < factorial(n) && p < 24; ++p) {
    t.perm[p] = lehmer_perm(n, p);
    for (int s = 0; s < n; ++s) t.pos[s * 4 + (int)((t.perm[p] >> (2 * s)) & 3u)] |= 1u << p;
  }
  return t;
}
#if defined(__HIPCC__)
__device__ constexpr PermTables kPermTables[5] = {make_perm_tables(0), make_perm_tables(1), make_perm_tables(2), make_perm_tables(3), make_perm_tables(4)};
#else
constexpr PermTables kPermTables[5] = {make_perm_tables(0), make_perm_tables(1), make_perm_tables(2), make_perm_tables(3), make_perm_tables(4)};
#endif

template <int N_, int NV_, int MK_>
struct Memb {
  static constexpr int N = N_, NV = NV_, MK = MK_;
  // raft.tla:22-30
  static constexpr int MAXLOG = 5, MAXRESTARTS = 2, MAXTIMEOUTS = 3, MAXCR = 3, MAXTERMS = 4, MAXMC = 3, MAXTMC = 4;
  static constexpr int MAXINFLIGHT = 2 * N * N;
  static constexpr int LMAXW = 2 * MAXLOG;          // longest working log (HandleCatchupRequest concat, out of model)
  // ---- widths
  static constexpr int SB = bits_for(N - 1);        // server index
  static constexpr int VB = bits_for(N);            // votedFor 0..N (N = Nil)
  static constexpr int TB = 3;                      // terms 0..7
  static constexpr int IB = 3;                      // indices / lengths 0..7
  static constexpr int RB = 2;                      // rounds 0..3
  static constexpr int VW = bits_for(NV - 1) > N ? bits_for(NV - 1) : N;   // entry value: Value index | config rank
  static constexpr int EW = 2 + 1 + VW;             // entry: term-1 (2b, terms 1..MaxTerms) | type | value
  static constexpr u32 EM = (u32)((1u << EW) - 1u);
  static constexpr int MLOGB = IB + MAXLOG * EW;    // log inside a message, MSB-first (length, e1, e2, ...)
  static constexpr int AEEB = 1 + EW;               // AppendEntries mentries: length (0/1) | entry
  static constexpr int CNTB = bits_for(MAXINFLIGHT + 1);
  static constexpr int CODEB = 64 - CNTB;
  static constexpr u64 R2M = rank_to_mask_lut(N), M2R = mask_to_rank_lut(N);
  static constexpr int NPERM = factorial(N);
  // ---- instance groups (Next order: NextAsync :909-916, NextCrash :918, NextUnreliable :924-932, NextDynamic :940-943)
  static constexpr int G_RV = 0, G_BL = G_RV + N * N, G_CR = G_BL + N, G_ACI = G_CR + N * NV, G_AE = G_ACI + N,
                       G_RECV = G_AE + N * N, G_TO = G_RECV + MK, G_RS = G_TO + N, G_DUP = G_RS + N, G_DROP = G_DUP + MK,
                       G_ADD = G_DROP + MK, G_DEL = G_ADD + N * N, NI = G_DEL + N * N;
  static constexpr int NSLOT = NI + MK;             // (instance, successor) slots; Receive has 2
  // ---- stored (packed) layout, u32 words: term st voted commit vr vg | nexti(2) matchi(2) | logs(2N) | h0(2) h1(2) |
  //      hr0(2) hr1(2) | bag(2MK)
  static constexpr int NW = 6 + 4 + 2 * N + 4 + 4 + 2 * MK;
  static constexpr int NWP = (NW + 3) & ~3;

  static_assert(N >= 1 && N <= 4, "1..4 servers");
  static_assert(N * N <= 16 && N * VB <= 32 && N * IB <= 32, "scalar words");
  static_assert(8 * EW <= 64 && 2 * EW <= 16, "working log words");
  static_assert(IB + MAXLOG * EW <= 60, "stored log word");
  static_assert(3 + IB + SB + MLOGB + IB + RB + SB + TB <= CODEB, "CatchupRequest code width");
  static_assert(3 + SB + MLOGB + SB + TB + 1 <= CODEB, "RequestVoteResponse code width");

  struct Work {
    u32 term, st, voted, commit, vr, vg;   // per-server fields (TB, 2, VB, IB bits; vr/vg rows of N bits)
    u64 nexti, matchi;                     // N*N fields of IB bits, index i*N+j
    Arr<u64, N> la;                        // log entries 0..7 (EW bits each)
    Arr<u32, N> lb;                        // entries 8..9 | length << 16
    u64 h0, h1;                            // history summary (see below)
    u64 hr0, hr1;                          // TLC-mode symmetry: ranks of the permuted histories (see below)
    Arr<u64, MK + 1> bag;                  // sorted (code << CNTB | count), EMPTY = ~0
  };
  static constexpr u32 F = 0, C = 1, L = 2;   // Follower, Candidate, Leader
  static constexpr u64 EMPTY = ~0ull;

  // ------------------------------------------------------------ per-server fields
  RMC_HD static int g_term(const Work& s, int i) { return (int)fget<TB>(s.term, i); }
  RMC_HD static int g_st(const Work& s, int i) { return (int)fget<2>(s.st, i); }
  RMC_HD static int g_voted(const Work& s, int i) { return (int)fget<VB>(s.voted, i); }
  RMC_HD static int g_commit(const Work& s, int i) { return (int)fget<IB>(s.commit, i); }
  RMC_HD static u32 g_vr(const Work& s, int i) { return fget<N>(s.vr, i); }
  RMC_HD static u32 g_vg(const Work& s, int i) { return fget<N>(s.vg, i); }
  RMC_HD static int g_next(const Work& s, int i, int j) { return (int)fget<IB>(s.nexti, i * N + j); }
  RMC_HD static int g_match(const Work& s, int i, int j) { return (int)fget<IB>(s.matchi, i * N + j); }
  RMC_HD static void s_term(Work& t, int i, int v, u32& err) { if (v > 7) err |= ME_CAP; fset<TB>(t.term, i, (u32)v); }
  RMC_HD static void s_st(Work& t, int i, u32 v) { fset<2>(t.st, i, v); }
  RMC_HD static void s_voted(Work& t, int i, int v) { fset<VB>(t.voted, i, (u32)v); }
  RMC_HD static void s_commit(Work& t, int i, int v, u32& err) { if (v > 7 || v < 0) err |= ME_CAP; fset<IB>(t.commit, i, (u32)v); }
  RMC_HD static void s_next(Work& t, int i, int j, int v, u32& err) { if (v > 7 || v < 0) err |= ME_CAP; fset<IB, u64>(t.nexti, i * N + j, (u64)v); }
  RMC_HD static void s_match(Work& t, int i, int j, int v, u32& err) { if (v > 7 || v < 0) err |= ME_CAP; fset<IB, u64>(t.matchi, i * N + j, (u64)v); }
  RMC_HD static u32 servers_in(u32 st, u32 x) {   // mask of servers whose state is x
    u32 m = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) if (fget<2>(st, i) == x) m |= 1u << i;
    return m;
  }

  // ------------------------------------------------------------ entries and logs
  RMC_HD static int eterm(u32 e) { return (int)(e >> (1 + VW)) + 1; }
  RMC_HD static u32 etype(u32 e) { return (e >> VW) & 1u; }
  RMC_HD static u32 evalue(u32 e) { return e & (u32)lomask(VW); }
  RMC_HD static u32 mkentry(int term, u32 type, u32 value, u32& err) {
    if (term < 1 || term > MAXTERMS) err |= ME_CAP;
    return ((u32)(term - 1) & 3u) << (1 + VW) | type << VW | value;
  }
  RMC_HD static u32 r2m(u32 r) { return (u32)((R2M >> (4 * r)) & 15u); }
  RMC_HD static u32 m2r(u32 m) { return (u32)((M2R >> (4 * m)) & 15u); }

  struct LogV { u64 a; u32 b; };
  RMC_HD static LogV getlog(const Work& s, int i) { return LogV{sel(s.la, i), sel(s.lb, i)}; }
  RMC_HD static void putlog(Work& t, int i, LogV l) { put(t.la, i, l.a); put(t.lb, i, l.b); }
  RMC_HD static int llen(LogV l) { return (int)(l.b >> 16); }
  RMC_HD static u32 lent(LogV l, int p) {   // 0-based
    return p < 8 ? (u32)((l.a >> (p * EW)) & EM) : (u32)((l.b >> ((p - 8) * EW)) & EM);
  }
  RMC_HD static LogV lset(LogV l, int p, u32 e) {
    if (p < 8) l.a = (l.a & ~((u64)EM << (p * EW))) | ((u64)e << (p * EW));
    else l.b = (l.b & ~(EM << ((p - 8) * EW))) | (e << ((p - 8) * EW));
    return l;
  }
  RMC_HD static LogV lsetlen(LogV l, int n) { l.b = (l.b & 0xFFFFu) | ((u32)n << 16); return l; }
  RMC_HD static LogV lappend(LogV l, u32 e, u32& err) {
    const int n = llen(l);
    if (n >= LMAXW) { err |= ME_CAP; return l; }
    return lsetlen(lset(l, n, e), n + 1);
  }
  RMC_HD static LogV lprefix(LogV l, int n) {     // SubSeq(log, 1, n), 0 <= n <= Len
    if (n < 8) { l.a &= lomask(n * EW); l.b = 0; }
    else l.b &= (u32)lomask((n - 8) * EW);
    return lsetlen(l, n);
  }
  RMC_HD static int last_term(LogV l) { const int n = llen(l); return n == 0 ? 0 : eterm(lent(l, n - 1)); }
  RMC_HD static bool leq(LogV x, LogV y) { return x.a == y.a && x.b == y.b; }
  // IsPrefix(SubSeq(x, 1, n), y) (SequencesExt.tla:134-140), n <= Len(x)
  RMC_HD static bool is_prefix_n(LogV x, int n, LogV y) {
    if (n > llen(y)) return false;
    const LogV px = lprefix(x, n), py = lprefix(y, n);
    return px.a == py.a && (px.b & 0xFFFFu) == (py.b & 0xFFFFu);
  }
  // GetHistoricalConfig / GetHistoricalMaxConfigIndex (raft.tla:346-360, G12) over the first n entries
  template <int LM>
  RMC_HD static u32 config_of(LogV l, int n, u32 init_cfg, u32 cfgt, int* maxidx) {
    u32 c = init_cfg; int mi = 0;
#pragma unroll
    for (int p = 0; p < LM; ++p)
      if (p < n) { const u32 e = lent(l, p); if (etype(e) == cfgt) { c = r2m(evalue(e)); mi = p + 1; } }
    if (maxidx) *maxidx = mi;
    return c;
  }
  // a message log field (MSB-first: length, e1, e2, ...; <= MaxLogLength entries)
  RMC_HD static u64 sub_to_mlog(LogV l, int m, int n, u32& err) {   // SubSeq(l, m, n)
    if (m > n) return 0;
    if (m < 1 || n > llen(l)) { err |= ME_EVAL; return 0; }          // TLC: SubSeq index out of domain
    const int cnt = n - m + 1;
    if (cnt > MAXLOG) { err |= ME_CAP; return 0; }
    u64 f = (u64)cnt << (MAXLOG * EW);
#pragma unroll
    for (int p = 0; p < MAXLOG; ++p) if (p < cnt) f |= (u64)lent(l, m - 1 + p) << ((MAXLOG - 1 - p) * EW);
    return f;
  }
  RMC_HD static int mlog_len(u64 f) { return (int)(f >> (MAXLOG * EW)); }
  RMC_HD static u32 mlog_ent(u64 f, int p) { return (u32)((f >> ((MAXLOG - 1 - p) * EW)) & EM); }
  RMC_HD static LogV mlog_append(LogV l, u64 f, u32& err) {        // l \o f
    const int c = mlog_len(f);
#pragma unroll
    for (int p = 0; p < MAXLOG; ++p) if (p < c) l = lappend(l, mlog_ent(f, p), err);
    return l;
  }

  // ------------------------------------------------------------ messages
  // classes in the oracle's record order (field count, then field names)
  enum { K_COC = 0, K_RVQ = 1, K_RVP = 2, K_AEP = 3, K_CRQ7 = 4, K_CRP = 5, K_CRQ8 = 6, K_AEQ = 7 };
  struct CB {   // MSB-first code builder
    u64 c; int n;
    RMC_HD explicit CB(int cls) : c((u64)cls), n(3) {}
    RMC_HD void put(long long v, int w, u32& err) {
      if (v < 0 || (u64)v > lomask(w)) err |= ME_CAP;
      c = (c << w) | ((u64)v & lomask(w)); n += w;
    }
    RMC_HD u64 done() const { return c << (CODEB - n); }
  };
  RMC_HD static u64 fld(u64 c, int off, int w) { return (c >> (CODEB - off - w)) & lomask(w); }
  RMC_HD static int mcls(u64 c) { return (int)(c >> (CODEB - 3)); }
  // field offsets (from the top, class bits included)
  static constexpr int O_COC_ADD = 3, O_COC_DST = 4, O_COC_SRV = 4 + SB, O_COC_SRC = 4 + 2 * SB, O_COC_TERM = 4 + 3 * SB;
  static constexpr int O_RVQ_DST = 3, O_RVQ_LLI = 3 + SB, O_RVQ_LLT = 3 + SB + IB, O_RVQ_SRC = 3 + SB + IB + TB, O_RVQ_TERM = 3 + 2 * SB + IB + TB;
  static constexpr int O_RVP_DST = 3, O_RVP_LOG = 3 + SB, O_RVP_SRC = 3 + SB + MLOGB, O_RVP_TERM = 3 + 2 * SB + MLOGB, O_RVP_GR = 3 + 2 * SB + MLOGB + TB;
  static constexpr int O_AEP_DST = 3, O_AEP_MMI = 3 + SB, O_AEP_SRC = 3 + SB + IB, O_AEP_SUC = 3 + 2 * SB + IB, O_AEP_TERM = 4 + 2 * SB + IB;
  static constexpr int O_CQ7_DST = 3, O_CQ7_ENT = 3 + SB, O_CQ7_LLEN = 3 + SB + MLOGB, O_CQ7_RND = 3 + SB + MLOGB + IB,
                       O_CQ7_SRC = 3 + SB + MLOGB + IB + RB, O_CQ7_TERM = 3 + 2 * SB + MLOGB + IB + RB;
  static constexpr int O_CRP_DST = 3, O_CRP_MMI = 3 + SB, O_CRP_RL = 3 + SB + IB, O_CRP_SRC = 3 + SB + IB + RB,
                       O_CRP_SUC = 3 + 2 * SB + IB + RB, O_CRP_TERM = 4 + 2 * SB + IB + RB;
  static constexpr int O_CQ8_CI = 3, O_CQ8_DST = 3 + IB, O_CQ8_ENT = 3 + IB + SB, O_CQ8_LLEN = 3 + IB + SB + MLOGB,
                       O_CQ8_RND = 3 + 2 * IB + SB + MLOGB, O_CQ8_SRC = 3 + 2 * IB + SB + MLOGB + RB, O_CQ8_TERM = 3 + 2 * IB + 2 * SB + MLOGB + RB;
  static constexpr int O_AEQ_CI = 3, O_AEQ_DST = 3 + IB, O_AEQ_ENT = 3 + IB + SB, O_AEQ_PLI = 3 + IB + SB + AEEB,
                       O_AEQ_PLT = 3 + 2 * IB + SB + AEEB, O_AEQ_SRC = 3 + 2 * IB + SB + AEEB + TB, O_AEQ_TERM = 3 + 2 * IB + 2 * SB + AEEB + TB;

  RMC_HD static u64 m_coc(bool add, int dst, int srv, int src, int term, u32& err) {
    CB b(K_COC); b.put(add, 1, err); b.put(dst, SB, err); b.put(srv, SB, err); b.put(src, SB, err); b.put(term, TB, err); return b.done();
  }
  RMC_HD static u64 m_rvq(int dst, int lli, int llt, int src, int term, u32& err) {
    CB b(K_RVQ); b.put(dst, SB, err); b.put(lli, IB, err); b.put(llt, TB, err); b.put(src, SB, err); b.put(term, TB, err); return b.done();
  }
  RMC_HD static u64 m_rvp(int dst, u64 mlog, int src, int term, bool granted, u32& err) {
    CB b(K_RVP); b.put(dst, SB, err); b.put((long long)mlog, MLOGB, err); b.put(src, SB, err); b.put(term, TB, err); b.put(granted, 1, err); return b.done();
  }
  RMC_HD static u64 m_aep(int dst, int mmi, int src, bool success, int term, u32& err) {
    CB b(K_AEP); b.put(dst, SB, err); b.put(mmi, IB, err); b.put(src, SB, err); b.put(success, 1, err); b.put(term, TB, err); return b.done();
  }
  RMC_HD static u64 m_crq7(int dst, u64 ents, int loglen, int rounds, int src, int term, u32& err) {
    CB b(K_CRQ7); b.put(dst, SB, err); b.put((long long)ents, MLOGB, err); b.put(loglen, IB, err); b.put(rounds, RB, err); b.put(src, SB, err); b.put(term, TB, err); return b.done();
  }
  RMC_HD static u64 m_crp(int dst, int mmi, int rl, int src, bool success, int term, u32& err) {
    CB b(K_CRP); b.put(dst, SB, err); b.put(mmi, IB, err); b.put(rl, RB, err); b.put(src, SB, err); b.put(success, 1, err); b.put(term, TB, err); return b.done();
  }
  RMC_HD static u64 m_crq8(int ci, int dst, u64 ents, int loglen, int rounds, int src, int term, u32& err) {
    CB b(K_CRQ8); b.put(ci, IB, err); b.put(dst, SB, err); b.put((long long)ents, MLOGB, err); b.put(loglen, IB, err); b.put(rounds, RB, err); b.put(src, SB, err); b.put(term, TB, err); return b.done();
  }
  RMC_HD static u64 m_aeq(int ci, int dst, u32 ents, int pli, int plt, int src, int term, u32& err) {
    CB b(K_AEQ); b.put(ci, IB, err); b.put(dst, SB, err); b.put(ents, AEEB, err); b.put(pli, IB, err); b.put(plt, TB, err); b.put(src, SB, err); b.put(term, TB, err); return b.done();
  }
  // positions of the fields every handler needs: (dst, src, term) offsets per class; plus the
  // permutation descriptor (server-valued fields and config-carrying logs)
  struct MDesc { int dst, src, term, srv, log, kind; };   // kind: 0 none, 1 message log, 2 AE entry
  RMC_HD static constexpr MDesc mdesc(int cls) {
    switch (cls) {
      case K_COC: return {O_COC_DST, O_COC_SRC, O_COC_TERM, O_COC_SRV, 0, 0};
      case K_RVQ: return {O_RVQ_DST, O_RVQ_SRC, O_RVQ_TERM, 0, 0, 0};
      case K_RVP: return {O_RVP_DST, O_RVP_SRC, O_RVP_TERM, 0, O_RVP_LOG, 1};
      case K_AEP: return {O_AEP_DST, O_AEP_SRC, O_AEP_TERM, 0, 0, 0};
      case K_CRQ7: return {O_CQ7_DST, O_CQ7_SRC, O_CQ7_TERM, 0, O_CQ7_ENT, 1};
      case K_CRP: return {O_CRP_DST, O_CRP_SRC, O_CRP_TERM, 0, 0, 0};
      case K_CRQ8: return {O_CQ8_DST, O_CQ8_SRC, O_CQ8_TERM, 0, O_CQ8_ENT, 1};
      default: return {O_AEQ_DST, O_AEQ_SRC, O_AEQ_TERM, 0, O_AEQ_ENT, 2};
    }
  }
  // one descriptor field of every class, a byte per class (class k in byte k): a field is one
  // 64-bit shift and mask on the lane's class, for the per-message hot loops of TLC's symmetry
  // rule (perm_code, canon_code), instead of the 8-way select chain below
  RMC_HD static constexpr u64 md_lut(int f) {
    u64 r = 0;
    for (int k = 0; k < 8; ++k) {
      const MDesc d = mdesc(k);
      const int v = f == 0 ? d.dst : f == 1 ? d.src : d.srv;
      r |= (u64)(v & 255) << (8 * k);
    }
    return r;
  }
  RMC_HD static int md_field(u64 lut, int cls) { return (int)((lut >> (8 * cls)) & 255u); }
  // a select-chain lookup of the descriptor (no divergence across lanes holding different classes)
  RMC_HD static u64 mdesc_packed(int cls) {
    u64 r = 0;
#pragma unroll
    for (int k = 0; k < 8; ++k) {
      const MDesc d = mdesc(k);
      const u64 w = (u64)d.dst | (u64)d.src << 7 | (u64)d.term << 14 | (u64)d.srv << 21 | (u64)d.log << 28 | (u64)d.kind << 35;
      r = cls == k ? w : r;
    }
    return r;
  }

  // ------------------------------------------------------------ bag (TypedBags, G2)
  RMC_HD static u64 mcode(u64 ent) { return ent >> CNTB; }
  RMC_HD static int mcount(u64 ent) { return (int)(ent & lomask(CNTB)); }
  // WithMessage (raft.tla:226, TypedBags.tla:51-57)
  RMC_HD static void with_msg(Arr<u64, MK + 1>& bag, u64 code, u32& err) {
    bool found = false;
#pragma unroll
    for (int k = 0; k < MK + 1; ++k) {
      if (bag.v[k] != EMPTY && mcode(bag.v[k]) == code) {
        found = true;
        if (mcount(bag.v[k]) + 1 > (int)lomask(CNTB)) err |= ME_CAP;
        bag.v[k] += 1;
      }
    }
    if (!found) {
      const u64 x = (code << CNTB) | 1ull;
      if (bag.v[MK] != EMPTY) err |= ME_CAP;
      u64 prev = 0; bool prev_lt = true;
#pragma unroll
      for (int k = 0; k < MK + 1; ++k) {
        const u64 cur = bag.v[k];
        const bool cur_lt = cur < x;
        bag.v[k] = cur_lt ? cur : (prev_lt ? x : prev);
        prev = cur; prev_lt = cur_lt;
      }
    }
  }
  // WithoutMessage (raft.tla:231, TypedBags.tla:60-69): a zero count leaves the domain (G2)
  RMC_HD static void without_msg(Arr<u64, MK + 1>& bag, u64 code) {
    int idx = -1;
#pragma unroll
    for (int k = 0; k < MK + 1; ++k) if (bag.v[k] != EMPTY && mcode(bag.v[k]) == code) idx = k;
    if (idx < 0) return;
    if (mcount(sel(bag, idx)) > 1) { put(bag, idx, sel(bag, idx) - 1); return; }
#pragma unroll
    for (int k = 0; k < MK; ++k) bag.v[k] = k >= idx ? bag.v[k + 1] : bag.v[k];
    bag.v[MK] = EMPTY;
  }

  // ------------------------------------------------------------ history summary (not in the VIEW)
  // h0: restarted[i] 2b @2i | timeout[i] 3b @2N+3i | hadNumLeaders 4b | hadNumClientRequests 3b |
  //     hadNumTriedMembershipChanges 3b | hadNumMembershipChanges 3b | Len(history["global"]) 10b
  static constexpr int H_TO = 2 * N, H_HL = 5 * N, H_CR = H_HL + 4, H_TMC = H_CR + 3, H_MC = H_TMC + 3, H_GLEN = H_MC + 3;
  // h1: flags | k0 (first CommitEntry position after a concurrent BecomeLeader) | last Restart position | added mask |
  //     dead-binding masks of the punctuated-search prefix constraints (NB bits per enabled region)
  enum { F_BL = 0, F_CE, F_CONCBL, F_RCLOSE, F_ADD, F_CMC, F_CMC2, F_ADDCOMMITS, F_NEWLEADER, F_PENDADD, F_LCDCC };
  static constexpr int H_K0 = 11, H_LASTR = 21, H_ADDED = 31, H_PREFIX = 36;
  static constexpr int NB = N >= 3 ? N * (N - 1) * (N - 2) : 0;   // bindings of s1, s2, s3 (raft.tla:1199, :1229)
  static constexpr u64 NBMASK = lomask(NB);
  RMC_HD static int hget(u64 h, int off, int w) { return (int)((h >> off) & lomask(w)); }
  RMC_HD static void hset(u64& h, int off, int w, int v, u32& err) {
    if (v < 0 || (u64)v > lomask(w)) { err |= ME_CAP; v &= (int)lomask(w); }
    h = (h & ~(lomask(w) << off)) | ((u64)v << off);
  }
  RMC_HD static bool hflag(u64 h1, int f) { return (h1 >> f) & 1ull; }
  RMC_HD static int restarted(const Work& s, int i) { return hget(s.h0, 2 * i, 2); }
  RMC_HD static int timeouts(const Work& s, int i) { return hget(s.h0, H_TO + 3 * i, 3); }
  RMC_HD static int glen(const Work& s) { return hget(s.h0, H_GLEN, 10); }
  RMC_HD static void h_bump(Work& t, int off, int w, u32& err) { hset(t.h0, off, w, hget(t.h0, off, w) + 1, err); }
  RMC_HD static int h_append(Work& t, int d, u32& err) { const int g = glen(t) + d; hset(t.h0, H_GLEN, 10, g, err); return g; }
  // History entries as (x, y) codes for the prefix constraints: x = kind | executedOn << 4 |
  // aux << 8, y = the message code (Send/Receive) or 0.  The host encodes the golden traces the
  // same way (memb_prefix.h).
  enum { HE_SEND = 1, HE_RECV, HE_TRYADD, HE_TRYREM, HE_ADD, HE_REM, HE_BL, HE_CE, HE_CMC, HE_RESTART, HE_TIMEOUT };
  RMC_HD static u64 hx(int kind, int exec, u32 aux) { return (u64)kind | (u64)exec << 4 | (u64)aux << 8; }
  // Bag changes of one successor are recorded as a delta (at most one message added, one
  // removed) and applied once at the end of apply(): one inlined copy of the 33-entry bag
  // loops instead of one per call site keeps every kernel within short-branch range.  The
  // history entries it appends are recorded the same way (hk: HK_* | entry x << 4).
  enum { HK_NONE = 0, HK_SEND, HK_DISCARD, HK_REPLY, HK_DISCARD_MC, HK_ONE };
  struct Delta { u64 add, rem; u32 hk; bool a, r; };
  // Send (raft.tla:247-263): TryAddServer/TryRemoveServer precede Send for CatchupRequest/CheckOldConfig
  RMC_HD static void send(Work& t, Delta& d, u64 code, u32& err) {
    d.add = code; d.a = true; d.hk = HK_SEND;
    const int c = mcls(code);
    if (c == K_CRQ7 || c == K_CRQ8 || c == K_COC) { h_bump(t, H_TMC, 3, err); h_append(t, 2, err); }
    else h_append(t, 1, err);
  }
  RMC_HD static void discard(Work& t, Delta& d, u64 code, u32& err) {   // :280-283
    d.rem = code; d.r = true; d.hk = HK_DISCARD; h_append(t, 1, err);
  }
  RMC_HD static void reply(Work& t, Delta& d, u64 resp, u64 req, u32& err) {   // :308-314: WithoutMessage(req, WithMessage(resp, .))
    d.add = resp; d.a = true; d.rem = req; d.r = true; d.hk = HK_REPLY; h_append(t, 2, err);
  }
  // DiscardDirectWithMembershipChange (:285-290) with AddServer/RemoveServer (:802-803)
  RMC_HD static void discard_mc(Work& t, Delta& d, u64 code, bool add, int srv, u32& err) {
    d.rem = code; d.r = true;
    d.hk = HK_DISCARD_MC | (u32)(add ? 1 : 0) << 4 | (u32)srv << 5;
    h_bump(t, H_MC, 3, err);
    h_append(t, 2, err);
    if (add) {
      t.h1 |= (1ull << F_ADD) | (1ull << F_PENDADD) | (1ull << (H_ADDED + srv));
    }
  }
  RMC_HD static void one_entry(Delta& d, int kind, int exec, u32 aux) { d.hk = HK_ONE | (u32)hx(kind, exec, aux) << 4; }
  RMC_HD static void ev_become_leader(Work& t, Delta& d, int i, u32 leaders, u32& err) {   // :479-483
    h_bump(t, H_HL, 4, err);
    h_append(t, 1, err);
    one_entry(d, HE_BL, i, leaders);
    t.h1 |= 1ull << F_BL;
    if (popc32(leaders) >= 2) t.h1 |= 1ull << F_CONCBL;
    if ((t.h1 >> (H_ADDED + i)) & 1ull) t.h1 |= 1ull << F_NEWLEADER;
    if (hflag(t.h1, F_PENDADD)) t.h1 |= 1ull << F_LCDCC;
  }
  RMC_HD static void ev_commit_entry(Work& t, Delta& d, int i, u32 entry, u32& err) {   // :537
    const int pos = h_append(t, 1, err);
    one_entry(d, HE_CE, i, entry);
    t.h1 |= 1ull << F_CE;
    if (hflag(t.h1, F_CONCBL) && hget(t.h1, H_K0, 10) == 0) hset(t.h1, H_K0, 10, pos, err);
  }
  RMC_HD static void ev_commit_membership(Work& t, Delta& d, int i, u32 cfgmask, u32& err) {   // :533-534
    h_append(t, 1, err);
    one_entry(d, HE_CMC, i, cfgmask);
    if (hflag(t.h1, F_CMC)) t.h1 |= 1ull << F_CMC2;
    t.h1 |= 1ull << F_CMC;
    if (((u32)(t.h1 >> H_ADDED) & cfgmask & (u32)lomask(N)) != 0) t.h1 |= 1ull << F_ADDCOMMITS;
    t.h1 &= ~(1ull << F_PENDADD);
  }
  RMC_HD static void ev_restart(Work& t, Delta& d, int i, u32& err) {   // :410
    h_bump(t, 2 * i, 2, err);
    const int pos = h_append(t, 1, err), last = hget(t.h1, H_LASTR, 10);
    one_entry(d, HE_RESTART, i, 0);
    if (last > 0 && pos - last < 6) t.h1 |= 1ull << F_RCLOSE;
    hset(t.h1, H_LASTR, 10, pos, err);
  }
  // executedOn of a Send (msource) / Receive (mdest), from the message code
  RMC_HD static int msg_src(u64 m) { return (int)fld(m, (int)((mdesc_packed(mcls(m)) >> 7) & 127), SB); }
  RMC_HD static int msg_dst(u64 m) { return (int)fld(m, (int)(mdesc_packed(mcls(m)) & 127), SB); }
  // One history entry at 0-based position p against one prefix region: clear the bindings whose
  // golden entry differs (IsPrefix(SubSeq(trace, 1, maxLen), history["global"]), raft.tla:1201-1204).
  RMC_HD static u64 prefix_match(u64 dead, const u64* tab, u32 plen, int p, u64 x, u64 y) {
    if (p >= (int)plen) return dead;
    const u64* row = tab + (u64)p * NB * 2;
#pragma unroll 1
    for (int b = 0; b < NB; ++b)
      if (row[2 * b] != x || row[2 * b + 1] != y) dead |= 1ull << b;
    return dead;
  }
  // The entries this successor appended (Delta.hk), at positions glen(s), glen(s)+1, against
  // every enabled prefix region.
  // the (x, y) codes of the 0, 1 or 2 entries a successor appended
  RMC_HD static int appended_entries(const Delta& d, u64& x0, u64& y0, u64& x1, u64& y1) {
    const u32 hk = d.hk & 15u;
    x0 = 0; y0 = 0; x1 = 0; y1 = 0;
    if (hk == HK_NONE) return 0;
    int n = 1;
    if (hk == HK_SEND) {
      const int c = mcls(d.add), src = msg_src(d.add);
      x0 = hx(HE_SEND, src, 0); y0 = d.add;
      if (c == K_CRQ7 || c == K_CRQ8 || c == K_COC) {   // TryAddServer (added = mdest) / TryRemoveServer (removed = mserver)
        x1 = x0; y1 = y0; n = 2;
        x0 = c == K_COC ? hx(HE_TRYREM, src, (u32)fld(d.add, O_COC_SRV, SB)) : hx(HE_TRYADD, src, (u32)msg_dst(d.add));
        y0 = 0;
      }
    } else if (hk == HK_ONE) {
      x0 = d.hk >> 4;
    } else {
      x0 = hx(HE_RECV, msg_dst(d.rem), 0); y0 = d.rem;
      if (hk == HK_REPLY) { x1 = hx(HE_SEND, msg_src(d.add), 0); y1 = d.add; n = 2; }
      if (hk == HK_DISCARD_MC) { x1 = hx((d.hk >> 4) & 1u ? HE_ADD : HE_REM, msg_dst(d.rem), d.hk >> 5); n = 2; }
    }
    return n;
  }
  RMC_HD static void prefix_step(const Work& s, Work& t, const Delta& d, const MembRuntime& rt) {
    u64 x0, y0, x1, y1;
    const int n = appended_entries(d, x0, y0, x1, y1);
    if (n == 0) return;
    const int p = glen(s);
    if (rt.plen0) {
      u64 dead = (t.h1 >> H_PREFIX) & NBMASK;
      dead = prefix_match(dead, rt.ptab0, rt.plen0, p, x0, y0);
      if (n == 2) dead = prefix_match(dead, rt.ptab0, rt.plen0, p + 1, x1, y1);
      t.h1 = (t.h1 & ~(NBMASK << H_PREFIX)) | dead << H_PREFIX;
    }
    if (rt.plen1) {
      const int off = (int)rt.preg1_off;
      u64 dead = (t.h1 >> off) & NBMASK;
      dead = prefix_match(dead, rt.ptab1, rt.plen1, p, x0, y0);
      if (n == 2) dead = prefix_match(dead, rt.ptab1, rt.plen1, p + 1, x1, y1);
      t.h1 = (t.h1 & ~(NBMASK << off)) | dead << off;
    }
  }

  // Opaque redefinition of the parent's registers (no instructions emitted): called at the top
  // of a per-instance loop so the compiler cannot hoist per-state decodes out of the loop
  // (loop-invariant code motion over ~100 instances otherwise exhausts the register file).
  RMC_HD static void launder(Work& s) {
#if defined(__HIP_DEVICE_COMPILE__)
    asm volatile("" : "+v"(s.term), "+v"(s.st), "+v"(s.voted), "+v"(s.commit), "+v"(s.vr), "+v"(s.vg));
    asm volatile("" : "+v"(s.nexti), "+v"(s.matchi), "+v"(s.h0), "+v"(s.h1), "+v"(s.hr0), "+v"(s.hr1));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("" : "+v"(s.la.v[i]), "+v"(s.lb.v[i]));
#pragma unroll
    for (int q = 0; q < MK + 1; ++q) asm volatile("" : "+v"(s.bag.v[q]));
#else
    (void)s;
#endif
  }

  // ------------------------------------------------------------ Init (raft.tla:367-393)
  RMC_HD static void init(Work& s) {
    s.term = fsplat<TB, u32>(1, N); s.st = 0; s.voted = fsplat<VB, u32>((u32)N, N); s.commit = 0; s.vr = 0; s.vg = 0;
    s.nexti = fsplat<IB, u64>(1, N * N); s.matchi = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) { s.la.v[i] = 0; s.lb.v[i] = 0; }
    s.h0 = 0; s.h1 = 0; s.hr0 = 0; s.hr1 = 0;
#pragma unroll
    for (int k = 0; k < MK + 1; ++k) s.bag.v[k] = EMPTY;
  }

  // ------------------------------------------------------------ instances
  // Slot of the sub-th successor of instance k (order = the oracle's enumeration order).
  RMC_HD static int slot_of(int k, int sub) { return k < G_RECV ? k : (k < G_TO ? G_RECV + 2 * (k - G_RECV) + sub : k + MK); }
  RMC_HD static void inst_of_slot(int slot, int& k, int& sub) {
    if (slot < G_RECV) { k = slot; sub = 0; }
    else if (slot < G_RECV + 2 * MK) { k = G_RECV + (slot - G_RECV) / 2; sub = (slot - G_RECV) & 1; }
    else { k = slot - MK; sub = 0; }
  }
  RMC_HD static bool group_enabled(int k, u32 next) {
    if (k < G_RS) return next & MN_ASYNC;
    if (k < G_DUP) return next & MN_CRASH;
    if (k < G_ADD) return next & MN_UNRELIABLE;
    return next & MN_DYNAMIC;
  }
  RMC_HD static int nsub(int k) { return (k >= G_RECV && k < G_TO) ? 2 : 1; }

  // The sub-th successor of instance k of s into t (t = s on entry is not assumed).
  // Returns its MembAct, or -1 when it does not exist.  HR = false: the TLC-mode history ranks of
  // t are left unrefined (kernels that never fingerprint or store t: no code for it).
  template <bool HR = true>
  RMC_HD static int apply(const Work& s, int k, int sub, Work& t, u32& err, const MembRuntime& rt) {
    t = s;
    Delta d{0, 0, HK_NONE, false, false};
    const int act = apply_inner(s, k, sub, t, d, err, rt);
    if (act >= 0) {
      if (d.a) with_msg(t.bag, d.add, err);
      if (d.r) without_msg(t.bag, d.rem);
      if (rt.plen0 | rt.plen1) prefix_step(s, t, d, rt);
      if (HR && rt.sym_tlc) tlc_refine(s, t, d, rt.cfg_type);
    }
    return act;
  }
  // XE: the bag entry of the instance's slot (Receive / DuplicateMessage / DropMessage) is xent, not read
  // from s.bag (memb_fingerprint_lds keeps the bag in LDS; EMPTY when the slot is past the bag's end)
  template <bool XE = false>
  RMC_HD static int apply_inner(const Work& s, int k, int sub, Work& t, Delta& d, u32& err, const MembRuntime& rt, u64 xent = EMPTY) {
    const u32 cfgt = rt.cfg_type;
    if (k < G_BL) {                                                   // RequestVote(i, j) :431-440
      const int i = k / N, j = k % N;
      if (g_st(s, i) != C) return -1;
      const LogV li = getlog(s, i);
      const u32 cfg = config_of<MAXLOG>(li, llen(li), rt.init_cfg, cfgt, nullptr);
      if (!((cfg >> j) & 1u) || ((g_vr(s, i) >> j) & 1u)) return -1;
      send(t, d, m_rvq(j, llen(li), last_term(li), i, g_term(s, i), err), err);
      return MA_RequestVote;
    }
    if (k < G_CR) {                                                   // BecomeLeader(i) :472-484
      const int i = k - G_BL;
      if (g_st(s, i) != C) return -1;
      const LogV li = getlog(s, i);
      const u32 cfg = config_of<MAXLOG>(li, llen(li), rt.init_cfg, cfgt, nullptr), vg = g_vg(s, i);
      if (!((vg & ~cfg) == 0 && popc32(vg) * 2 > popc32(cfg))) return -1;
      s_st(t, i, L);
#pragma unroll
      for (int j = 0; j < N; ++j) { s_next(t, i, j, llen(li) + 1, err); s_match(t, i, j, 0, err); }
      ev_become_leader(t, d, i, servers_in(s.st, L) | (1u << i), err);
      return MA_BecomeLeader;
    }
    if (k < G_ACI) {                                                  // ClientRequest(i, v) :488-497
      const int i = (k - G_CR) / NV, v = (k - G_CR) % NV;
      if (g_st(s, i) != L) return -1;
      putlog(t, i, lappend(getlog(s, i), mkentry(g_term(s, i), 1u - cfgt, (u32)v, err), err));
      h_bump(t, H_CR, 3, err);
      return MA_ClientRequest;
    }
    if (k < G_AE) {                                                   // AdvanceCommitIndex(i) :504-539
      const int i = k - G_ACI;
      if (g_st(s, i) != L) return -1;
      const LogV li = getlog(s, i);
      const int n = llen(li), ci = g_commit(s, i);
      const u32 cfg = config_of<MAXLOG>(li, n, rt.init_cfg, cfgt, nullptr);
      int best = 0;
#pragma unroll
      for (int index = 1; index <= MAXLOG; ++index) {
        if (index > n) continue;
        u32 agree = 1u << i;                                          // Agree(index)
#pragma unroll
        for (int q = 0; q < N; ++q) if (((cfg >> q) & 1u) && g_match(s, i, q) >= index) agree |= 1u << q;
        if ((agree & ~cfg) == 0 && popc32(agree) * 2 > popc32(cfg)) best = index;
      }
      int nci = ci;
      if (best > 0 && eterm(lent(li, best - 1)) == g_term(s, i)) nci = best;
      s_commit(t, i, nci, err);
      if (nci > ci) {
        const u32 e = lent(li, nci - 1);
        const bool cmc = etype(e) == cfgt && r2m(evalue(e)) != config_of<MAXLOG>(li, nci - 1, rt.init_cfg, cfgt, nullptr);
        if (cmc) ev_commit_membership(t, d, i, r2m(evalue(e)), err);   // G11
        else ev_commit_entry(t, d, i, e, err);
      }
      return MA_AdvanceCommitIndex;
    }
    if (k < G_RECV) {                                                 // AppendEntries(i, j) :446-468
      const int i = (k - G_AE) / N, j = (k - G_AE) % N;
      if (i == j || g_st(s, i) != L) return -1;
      const LogV li = getlog(s, i);
      const u32 cfg = config_of<MAXLOG>(li, llen(li), rt.init_cfg, cfgt, nullptr);
      if (!((cfg >> j) & 1u)) return -1;
      const int n = llen(li), ni = g_next(s, i, j), pli = ni - 1;
      const int plt = (pli > 0 && pli <= n) ? eterm(lent(li, pli - 1)) : 0;
      const int last = n < ni ? n : ni;
      const u32 ents = (ni <= last) ? ((1u << EW) | lent(li, ni - 1)) : 0u;   // SubSeq(log[i], ni, lastEntry): <= 1 entry
      const int ci = g_commit(s, i);
      send(t, d, m_aeq(ci < last ? ci : last, j, ents, pli, plt, i, g_term(s, i), err), err);
      return MA_AppendEntries;
    }
    if (k < G_TO) {                                                   // Receive(m) :842-863
      const u64 ent = XE ? xent : sel(s.bag, k - G_RECV);
      if (ent == EMPTY) return -1;
      return receive(s, mcode(ent), sub, t, d, err, rt);
    }
    if (k < G_RS) {                                                   // Timeout(i) :415-427
      const int i = k - G_TO, st = g_st(s, i);
      if (!(st == (int)F || st == (int)C)) return -1;
      const LogV li = getlog(s, i);
      if (!((config_of<MAXLOG>(li, llen(li), rt.init_cfg, cfgt, nullptr) >> i) & 1u)) return -1;
      s_st(t, i, C);
      s_term(t, i, g_term(s, i) + 1, err);
      s_voted(t, i, N);
      fset<N>(t.vr, i, 0u); fset<N>(t.vg, i, 0u);
      h_bump(t, H_TO + 3 * i, 3, err);
      h_append(t, 1, err);
      one_entry(d, HE_TIMEOUT, i, 0);
      return MA_Timeout;
    }
    if (k < G_DUP) {                                                  // Restart(i) :401-411
      const int i = k - G_RS;
      s_st(t, i, F);
      fset<N>(t.vr, i, 0u); fset<N>(t.vg, i, 0u);
#pragma unroll
      for (int j = 0; j < N; ++j) { s_next(t, i, j, 1, err); s_match(t, i, j, 0, err); }
      s_commit(t, i, 0, err);
      ev_restart(t, d, i, err);
      return MA_Restart;
    }
    if (k < G_DROP) {                                                 // DuplicateMessage(m), messages[m] = 1 :892-896, :926-928
      const u64 ent = XE ? xent : sel(s.bag, k - G_DUP);
      if (ent == EMPTY || mcount(ent) != 1) return -1;
      d.add = mcode(ent); d.a = true;
      return MA_DuplicateMessage;
    }
    if (k < G_ADD) {                                                  // DropMessage(m), messages[m] = 1 :900-904, :930-932
      const u64 ent = XE ? xent : sel(s.bag, k - G_DROP);
      if (ent == EMPTY || mcount(ent) != 1) return -1;
      d.rem = mcode(ent); d.r = true;
      return MA_DropMessage;
    }
    if (k < G_DEL) {                                                  // AddNewServer(i, j) :542-555 (G7, G8)
      const int i = (k - G_ADD) / N, j = (k - G_ADD) % N;
      if (g_st(s, i) != L) return -1;
      const LogV li = getlog(s, i);
      if ((config_of<MAXLOG>(li, llen(li), rt.init_cfg, cfgt, nullptr) >> j) & 1u) return -1;
      s_term(t, j, 1, err);
      s_voted(t, j, N);
      const int ci = g_commit(s, i);
      const u64 ents = sub_to_mlog(li, g_next(s, i, j), ci, err);
      send(t, d, m_crq8(ci, j, ents, g_match(s, i, j), (int)rt.num_rounds, i, g_term(s, i), err), err);
      return MA_AddNewServer;
    }
    {                                                                 // DeleteServer(i, j) :558-569
      const int i = (k - G_DEL) / N, j = (k - G_DEL) % N;
      if (g_st(s, i) != L) return -1;
      const int sj = g_st(s, j);
      if (!(sj == (int)F || sj == (int)C) || j == i) return -1;
      const LogV li = getlog(s, i);
      if (!((config_of<MAXLOG>(li, llen(li), rt.init_cfg, cfgt, nullptr) >> j) & 1u)) return -1;
      send(t, d, m_coc(false, i, j, i, g_term(s, i), err), err);
      return MA_DeleteServer;
    }
  }

  // The TLC-mode fingerprint kernel's re-derivation without the bag in registers (memb_fingerprint_lds):
  // apply's successor with the bag change left in d for the caller to make on its LDS copy of the
  // parent's bag (xent: the entry at the instance's bag slot).  Nothing after the bag change in apply
  // reads the bag (prefix_step reads d, tlc_refine the histories), so the order is apply's.
  template <bool HR = true>
  RMC_HD static int apply_nobag(const Work& s, int k, int sub, u64 xent, Work& t, Delta& d, u32& err, const MembRuntime& rt) {
    t = s;
    d = Delta{0, 0, HK_NONE, false, false};
    const int act = apply_inner<true>(s, k, sub, t, d, err, rt, xent);
    if (act >= 0) {
      if (rt.plen0 | rt.plen1) prefix_step(s, t, d, rt);
      if (HR && rt.sym_tlc) tlc_refine(s, t, d, rt.cfg_type);
    }
    return act;
  }
  // the bag slot instance k reads (Receive / DuplicateMessage / DropMessage), -1 for the others
  RMC_HD static int bag_slot_of(int k) {
    return k >= G_RECV && k < G_TO ? k - G_RECV : k >= G_DUP && k < G_DROP ? k - G_DUP : k >= G_DROP && k < G_ADD ? k - G_DROP : -1;
  }
  // with_msg / without_msg on a bag kept as len sorted entries p[q * stride] (a per-lane LDS slice of
  // cap entries): the same sorted order (entry value = code << CNTB | count, codes unique) and counts
  RMC_HD static void slice_with_msg(u64* p, int stride, int& len, int cap, u64 code) {
    int q = 0;
#pragma unroll 1
    while (q < len && mcode(p[q * stride]) < code) ++q;
    if (q < len && mcode(p[q * stride]) == code) { p[q * stride] += 1; return; }
    if (len >= cap) return;   // (the kernel sends parents that could overflow the slice elsewhere)
#pragma unroll 1
    for (int r = len; r > q; --r) p[r * stride] = p[(r - 1) * stride];
    p[q * stride] = (code << CNTB) | 1ull;
    ++len;
  }
  RMC_HD static void slice_without_msg(u64* p, int stride, int& len, u64 code) {
    int q = 0;
#pragma unroll 1
    while (q < len && mcode(p[q * stride]) != code) ++q;
    if (q == len) return;
    if (mcount(p[q * stride]) > 1) { p[q * stride] -= 1; return; }
#pragma unroll 1
    for (int r = q; r + 1 < len; ++r) p[r * stride] = p[(r + 1) * stride];
    --len;
  }

  // ReceiveDirect(m) :842-863: UpdateTerm first, then the type handler's successors in disjunct order.
  // How many times TLC's getNextStates generates the successor of instance k, sub-slot sub (>= 1 when
  // there is one): it enumerates every true disjunct of a disjunction inside an action as a branch of
  // its own, so a guard written as a disjunction yields the same successor once per true disjunct.
  // In this module that happens to two discards: HandleCheckOldConfig's `state[i] /= Leader \/
  // m.mterm = currentTerm[i]` (raft.tla:796) and HandleCatchupResponse's five-way list (:783-789).
  // The copies are one state, so only TLC's generated counters see them (distinct states, levels and
  // traces do not); the generic front end, which follows the text, counts them the same way.
  template <bool XE = false>
  RMC_HD static int tlc_copies(const Work& s, int k, int sub, const MembRuntime& rt, u64 xent = EMPTY) {
    if (!rt.disjunct_copies || k < G_RECV || k >= G_TO) return 1;
    const u64 ent = XE ? xent : sel(s.bag, k - G_RECV);
    if (ent == EMPTY) return 1;
    const u64 m = mcode(ent);
    const int cls = mcls(m);
    if (cls != K_COC && cls != K_CRP) return 1;
    const u64 dp = mdesc_packed(cls);
    const int i = (int)fld(m, (int)(dp & 127), SB), j = (int)fld(m, (int)((dp >> 7) & 127), SB);
    const int mt = (int)fld(m, (int)((dp >> 14) & 127), TB), ct = g_term(s, i);
    if (sub != (mt > ct ? 1 : 0)) return 1;   // (UpdateTerm, when enabled, takes the first sub-slot)
    const bool isLeader = g_st(s, i) == (int)L, termEq = mt == ct;
    if (cls == K_COC) return (!isLeader || termEq) ? (int)!isLeader + (int)termEq : 1;
    const LogV li = getlog(s, i);
    const int mmi = (int)fld(m, O_CRP_MMI, IB), ci = g_commit(s, i), mi = g_match(s, i, j);
    const bool succ = fld(m, O_CRP_SUC, 1);
    const bool inCfg = (config_of<MAXLOG>(li, llen(li), rt.init_cfg, rt.cfg_type, nullptr) >> j) & 1u;
    const bool c1 = succ && ((mmi != ci && mmi != mi) || mmi == ci) && isLeader && termEq && !inCfg;
    if (c1) return 1;
    return (int)!succ + (int)(mmi == mi && mmi != ci) + (int)!isLeader + (int)!termEq + (int)inCfg;
  }
#define RMC_EMIT(cond) if ((cond) && (idx++ == sub))
  RMC_HD static int receive(const Work& s, u64 m, int sub, Work& t, Delta& d, u32& err, const MembRuntime& rt) {
    const int cls = mcls(m);
    const u64 dp = mdesc_packed(cls);
    const int i = (int)fld(m, (int)(dp & 127), SB), j = (int)fld(m, (int)((dp >> 7) & 127), SB);
    const int mt = (int)fld(m, (int)((dp >> 14) & 127), TB), ct = g_term(s, i);
    const u32 cfgt = rt.cfg_type;
    int idx = 0;
    RMC_EMIT(mt > ct) {                                               // UpdateTerm :826-832 (G9): message kept
      s_term(t, i, mt, err); s_st(t, i, F); s_voted(t, i, N);
      return MA_UpdateTerm;
    }
    const LogV li = getlog(s, i);
    const int n = llen(li), st = g_st(s, i);
    switch (cls) {
      case K_RVQ: {                                                   // HandleRequestVoteRequest :578-597
        RMC_EMIT(mt <= ct) {
          const int llt = (int)fld(m, O_RVQ_LLT, TB), lli = (int)fld(m, O_RVQ_LLI, IB), lt = last_term(li);
          const bool logOk = llt > lt || (llt == lt && lli >= n);
          const int vf = g_voted(s, i);
          const bool grant = mt == ct && logOk && (vf == N || vf == j);
          if (grant) s_voted(t, i, j);
          reply(t, d, m_rvp(j, sub_to_mlog(li, 1, n, err), i, ct, grant, err), m, err);
          return MA_HandleRequestVoteRequest;
        }
        return -1;
      }
      case K_RVP: {
        RMC_EMIT(mt < ct) { discard(t, d, m, err); return MA_DropStaleResponse; }          // :836-839
        RMC_EMIT(mt == ct) {                                          // HandleRequestVoteResponse :602-614
          fset<N>(t.vr, i, g_vr(s, i) | (1u << j));
          if (fld(m, O_RVP_GR, 1)) fset<N>(t.vg, i, g_vg(s, i) | (1u << j));
          discard(t, d, m, err);
          return MA_HandleRequestVoteResponse;
        }
        return -1;
      }
      case K_AEQ: {                                                   // HandleAppendEntriesRequest :617-700
        const int pli = (int)fld(m, O_AEQ_PLI, IB), plt = (int)fld(m, O_AEQ_PLT, TB);
        const u32 ents = (u32)fld(m, O_AEQ_ENT, AEEB);
        const int elen = (int)(ents >> EW);
        const u32 e = ents & EM;
        const bool logOk = pli == 0 || (pli > 0 && pli <= n && plt == eterm(lent(li, pli - 1)));
        RMC_EMIT(mt <= ct && (mt < ct || (st == (int)F && !logOk))) {  // Reject :617-629
          reply(t, d, m_aep(j, 0, i, false, ct, err), m, err);
          return MA_HandleAppendEntriesRequest;
        }
        RMC_EMIT(mt == ct && st == (int)C) { s_st(t, i, F); return MA_HandleAppendEntriesRequest; }   // :632-636
        const bool acc = mt == ct && st == (int)F && logOk;           // Accept :675-683
        const int index = pli + 1;
        const bool has = elen > 0 && n >= index;
        const bool same = has && eterm(lent(li, index - 1)) == eterm(e);
        RMC_EMIT(acc && (elen == 0 || same)) {                        // AppendEntriesAlreadyDone :639-655
          s_commit(t, i, (int)fld(m, O_AEQ_CI, IB), err);
          reply(t, d, m_aep(j, pli + elen, i, true, ct, err), m, err);
          return MA_HandleAppendEntriesRequest;
        }
        RMC_EMIT(acc && has && !same) { putlog(t, i, lprefix(li, n - 1)); return MA_HandleAppendEntriesRequest; }   // :658-665
        RMC_EMIT(acc && elen > 0 && n == pli) { putlog(t, i, lappend(li, e, err)); return MA_HandleAppendEntriesRequest; }   // :668-672
        return -1;
      }
      case K_AEP: {
        RMC_EMIT(mt < ct) { discard(t, d, m, err); return MA_DropStaleResponse; }
        RMC_EMIT(mt == ct) {                                          // HandleAppendEntriesResponse :705-715
          const int mmi = (int)fld(m, O_AEP_MMI, IB);
          if (fld(m, O_AEP_SUC, 1)) { s_next(t, i, j, mmi + 1, err); s_match(t, i, j, mmi, err); }
          else { const int ni = g_next(s, i, j); s_next(t, i, j, ni - 1 > 1 ? ni - 1 : 1, err); }
          discard(t, d, m, err);
          return MA_HandleAppendEntriesResponse;
        }
        return -1;
      }
      case K_CRQ7:
      case K_CRQ8: {                                                  // HandleCatchupRequest :718-745 (G5)
        RMC_EMIT(mt < ct) {
          reply(t, d, m_crp(j, 0, 0, i, false, ct, err), m, err);
          return MA_HandleCatchupRequest;
        }
        RMC_EMIT(mt >= ct) {
          const bool c8 = cls == K_CRQ8;
          const u64 ments = fld(m, c8 ? O_CQ8_ENT : O_CQ7_ENT, MLOGB);
          const int mll = (int)fld(m, c8 ? O_CQ8_LLEN : O_CQ7_LLEN, IB), rnd = (int)fld(m, c8 ? O_CQ8_RND : O_CQ7_RND, RB);
          s_term(t, i, mt, err);
          LogV nl = n == 0 ? LogV{0ull, 0u} : lprefix(li, mll < n ? mll : n);
          putlog(t, i, mlog_append(nl, ments, err));
          reply(t, d, m_crp(j, n, rnd - 1, i, true, mt, err), m, err);
          return MA_HandleCatchupRequest;
        }
        return -1;
      }
      case K_CRP: {                                                   // HandleCatchupResponse :748-792
        const int mmi = (int)fld(m, O_CRP_MMI, IB), rl = (int)fld(m, O_CRP_RL, RB);
        const bool succ = fld(m, O_CRP_SUC, 1), isLeader = st == (int)L, termEq = mt == ct;
        const int ci = g_commit(s, i), mi = g_match(s, i, j), ni = g_next(s, i, j);
        const bool inCfg = (config_of<MAXLOG>(li, n, rt.init_cfg, cfgt, nullptr) >> j) & 1u;
        const bool c1 = succ && ((mmi != ci && mmi != mi) || mmi == ci) && isLeader && termEq && !inCfg;
        RMC_EMIT(c1) {
          s_next(t, i, j, mmi + 1, err); s_match(t, i, j, mmi, err);
          if (rl != 0) reply(t, d, m_crq7(j, sub_to_mlog(li, ni, ci, err), ni - 1, rl, i, ct, err), m, err);
          else reply(t, d, m_coc(true, i, j, i, ct, err), m, err);
          return MA_HandleCatchupResponse;
        }
        RMC_EMIT(!c1) { discard(t, d, m, err); return MA_HandleCatchupResponse; }
        return -1;
      }
      default: {                                                      // K_COC: HandleCheckOldConfig :795-822 (G6)
        const bool isLeader = st == (int)L, termEq = mt == ct;
        RMC_EMIT(!isLeader || termEq) { discard(t, d, m, err); return MA_HandleCheckOldConfig; }
        RMC_EMIT(isLeader && termEq) {
          int mci = 0;
          const u32 cfg = config_of<MAXLOG>(li, n, rt.init_cfg, cfgt, &mci);
          const bool add = fld(m, O_COC_ADD, 1);
          const int srv = (int)fld(m, O_COC_SRV, SB);
          if (mci <= g_commit(s, i)) {
            const u32 nc = add ? (cfg | (1u << srv)) : (cfg & ~(1u << srv));
            if (nc != cfg) {
              putlog(t, i, lappend(li, mkentry(ct, cfgt, m2r(nc), err), err));
              discard_mc(t, d, m, add, srv, err);
            } else {
              discard(t, d, m, err);
            }
          } else {
            reply(t, d, m_coc(add, i, srv, i, ct, err), m, err);
          }
          return MA_HandleCheckOldConfig;
        }
        return -1;
      }
    }
  }
#undef RMC_EMIT

  // ------------------------------------------------------------ constraints (cfg CONSTRAINTS) and action constraints
  RMC_HD static bool in_model(const Work& t, const Work& s, const MembRuntime& rt) {
    int tot = 0;
    bool rv1 = true;
#pragma unroll
    for (int q = 0; q < MK + 1; ++q) {
      const u64 e = t.bag.v[q];
      if (e != EMPTY) { tot += mcount(e); if (mcls(mcode(e)) == K_RVQ && mcount(e) > 1) rv1 = false; }
    }
    return in_model_bag(t, s, rt, tot, rv1);
  }
  // in_model of t = (s's successor by apply_nobag, bag change d) from s's bag and d, without t's bag:
  // the message total and RequestVote singleness of t's bag (with_msg then without_msg, as apply).  err
  // gets what apply and the expand kernel flag: a count beyond its field (with_msg, any successor) and,
  // for an in-model successor, a bag of more than MK messages (the expand kernel's check of entry MK)
  RMC_HD static bool in_model_delta(const Work& t, const Work& s, const Delta& d, const MembRuntime& rt, u32& err) {
    int tot = 0, n = 0;
    bool rv1 = true, found = false;
#pragma unroll
    for (int q = 0; q < MK; ++q) {
      const u64 e = s.bag.v[q];
      if (e == EMPTY) continue;
      const u64 code = mcode(e);
      int c = mcount(e);
      if (d.a && code == d.add) { found = true; if (c + 1 > (int)lomask(CNTB)) err |= ME_CAP; ++c; }
      if (d.r && code == d.rem) --c;
      tot += c;
      n += c > 0;   // (without_msg removes a message whose count reaches zero)
      if (mcls(code) == K_RVQ && c > 1) rv1 = false;
    }
    if (d.a && !found && !(d.r && d.rem == d.add)) { ++tot; ++n; }
    const bool ok = in_model_bag(t, s, rt, tot, rv1);
    if (ok && n > MK) err |= ME_CAP;
    return ok;
  }
  RMC_HD static bool in_model_bag(const Work& t, const Work& s, const MembRuntime& rt, int tot, bool rv1) {
    const u32 c = rt.constraints;
    bool ok = true;
    int sumr = 0, sumt = 0, cand = 0;
    bool anyr = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      sumr += restarted(t, i); sumt += timeouts(t, i); anyr |= restarted(t, i) != 0;
      if (g_st(t, i) == (int)C) ++cand;
      if (c & (1u << MC_BoundedLogSize)) ok &= llen(getlog(t, i)) <= MAXLOG;
      if (c & (1u << MC_BoundedRestarts)) ok &= restarted(t, i) <= MAXRESTARTS;
      if (c & (1u << MC_BoundedTimeouts)) ok &= timeouts(t, i) <= MAXTIMEOUTS;
      if (c & (1u << MC_BoundedTerms)) ok &= g_term(t, i) <= MAXTERMS;
    }
    const int hl = hget(t.h0, H_HL, 4), cr = hget(t.h0, H_CR, 3);
    if (c & (1u << MC_BoundedInFlightMessages)) ok &= tot <= MAXINFLIGHT;
    if (c & (1u << MC_BoundedRequestVote)) ok &= rv1;
    if (c & (1u << MC_BoundedClientRequests)) ok &= cr <= MAXCR;
    if (c & (1u << MC_BoundedTriedMembershipChanges)) ok &= hget(t.h0, H_TMC, 3) <= MAXTMC;
    if (c & (1u << MC_BoundedMembershipChanges)) ok &= hget(t.h0, H_MC, 3) <= MAXMC;
    if (c & (1u << MC_ElectionsUncontested)) ok &= cand <= 1;
    if (c & (1u << MC_CleanStartUntilFirstRequest))
      ok &= !(hl < 1 && cr < 1) || (!anyr && sumt <= 1 && cand <= 1);
    if (c & (1u << MC_CleanStartUntilTwoLeaders)) ok &= !(hl < 2) || (sumr <= 1 && sumt <= 2);
    if (c & (1u << MC_CommitWhenConcurrentLeaders_constraint)) ok &= glen(t) < 20 || hflag(t.h1, F_CONCBL);
    // \E s1, s2, s3 \in Server : distinct /\ the history extends the golden prefix (raft.tla:1198-1204, :1228-1234)
    if (c & (1u << MC_CommitWhenConcurrentLeaders_unique)) ok &= ((t.h1 >> H_PREFIX) & NBMASK) != NBMASK;
    if (c & (1u << MC_MajorityOfClusterRestarts_constraint)) ok &= ((t.h1 >> rt.preg1_off) & NBMASK) != NBMASK;
    if (rt.action_constraints & MAC_CommitWhenConcurrentLeaders) ok &= glen(s) < 20 || servers_in(t.st, C) == 0;
    return ok;
  }

  // ------------------------------------------------------------ invariants (TLC evaluation order; errors are verdicts)
  // Committed(i) == SubSeq(log[i], 1, commitIndex[i]) (:969): TLC error when commitIndex[i] > Len(log[i]).
  RMC_HD static int inv(const Work& t, int id, const MembRuntime& rt) {
    const u32 cfgt = rt.cfg_type;
    const u32 leaders = servers_in(t.st, L);
    switch (id) {
      case MI_LeaderVotesQuorum: {                                    // :988-993
        if (hget(t.h0, H_MC, 3) != 0) return IV_OK;
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (!((leaders >> i) & 1u)) continue;
          u32 q = 0;
#pragma unroll
          for (int j = 0; j < N; ++j)
            if (g_term(t, j) > g_term(t, i) || (g_term(t, j) == g_term(t, i) && g_voted(t, j) == i)) q |= 1u << j;
          const LogV li = getlog(t, i);
          const u32 cfg = config_of<LMAXW>(li, llen(li), rt.init_cfg, cfgt, nullptr);
          if (!((q & ~cfg) == 0 && popc32(q) * 2 > popc32(cfg))) return IV_BAD;
        }
        return IV_OK;
      }
      case MI_CandidateTermNotInLog: {                                // :997-1004
        if (hget(t.h0, H_MC, 3) != 0) return IV_OK;
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (g_st(t, i) != (int)C) continue;
          u32 q = 0;
#pragma unroll
          for (int j = 0; j < N; ++j)
            if (g_term(t, j) == g_term(t, i) && (g_voted(t, j) == i || g_voted(t, j) == N)) q |= 1u << j;
          const LogV li = getlog(t, i);
          const u32 cfg = config_of<LMAXW>(li, llen(li), rt.init_cfg, cfgt, nullptr);
          if (!((q & ~cfg) == 0 && popc32(q) * 2 > popc32(cfg))) continue;
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const LogV lj = getlog(t, j);
#pragma unroll 1
            for (int p = 0; p < LMAXW; ++p) if (p < llen(lj) && eterm(lent(lj, p)) == g_term(t, i)) return IV_BAD;
          }
        }
        return IV_OK;
      }
      case MI_ElectionSafety: {                                       // :1009-1014
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (!((leaders >> i) & 1u)) continue;
          const int ti = g_term(t, i);
          int mo[N];
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const LogV lj = getlog(t, j);
            int mx = 0;
#pragma unroll 1
            for (int p = 0; p < LMAXW; ++p) if (p < llen(lj) && eterm(lent(lj, p)) == ti) mx = p + 1;
            mo[j] = mx;
          }
#pragma unroll
          for (int j = 0; j < N; ++j) if (!(mo[i] >= mo[j])) return IV_BAD;
        }
        return IV_OK;
      }
      case MI_LogMatching: {                                          // :1017-1021
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const LogV li = getlog(t, i), lj = getlog(t, j);
            const int mn = llen(li) < llen(lj) ? llen(li) : llen(lj);
            bool pref = true;
#pragma unroll 1
            for (int p = 0; p < LMAXW; ++p) {
              if (p < mn) {
                const u32 x = lent(li, p), y = lent(lj, p);
                if (eterm(x) == eterm(y) && !(pref && x == y)) return IV_BAD;
                pref = pref && x == y;
              }
            }
          }
        return IV_OK;
      }
      case MI_VotesGrantedInv: {                                      // :1048-1052
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
          for (int j = 0; j < N; ++j) {
            if (g_voted(t, i) != j) continue;
            const LogV li = getlog(t, i);
            if (g_commit(t, i) > llen(li)) return IV_ERR;
            if (!is_prefix_n(li, g_commit(t, i), getlog(t, j))) return IV_BAD;
          }
        return IV_OK;
      }
      case MI_VotesGrantedInv_false: {                                // :1038-1046
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
          for (int j = 0; j < N; ++j) {
            if (!((g_vg(t, i) >> j) & 1u) || g_term(t, i) != g_term(t, j)) continue;
            const LogV lj = getlog(t, j);
            if (g_commit(t, j) > llen(lj)) return IV_ERR;
            if (!is_prefix_n(lj, g_commit(t, j), getlog(t, i))) return IV_BAD;
          }
        return IV_OK;
      }
      case MI_QuorumLogInv: {                                         // :1056-1060
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const LogV li = getlog(t, i);
          const u32 cfg = config_of<LMAXW>(li, llen(li), rt.init_cfg, cfgt, nullptr);
          if (cfg == 0) continue;                                     // Quorum({}) = {}
          if (g_commit(t, i) > llen(li)) return IV_ERR;
          u32 pre = 0;
#pragma unroll
          for (int j = 0; j < N; ++j) if (((cfg >> j) & 1u) && is_prefix_n(li, g_commit(t, i), getlog(t, j))) pre |= 1u << j;
          if (popc32(cfg & ~pre) * 2 > popc32(cfg)) return IV_BAD;     // a quorum avoiding every prefix holder
        }
        return IV_OK;
      }
      case MI_MoreUpToDateCorrect: {                                  // :1066-1071
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const LogV li = getlog(t, i), lj = getlog(t, j);
            const int a = last_term(li), b = last_term(lj);
            if (!(a > b || (a == b && llen(li) >= llen(lj)))) continue;
            if (g_commit(t, j) > llen(lj)) return IV_ERR;
            if (!is_prefix_n(lj, g_commit(t, j), li)) return IV_BAD;
          }
        return IV_OK;
      }
      case MI_LeaderCompleteness_false: {                             // :1079-1083
#pragma unroll
        for (int i = 0; i < N; ++i) {
          if (!((leaders >> i) & 1u)) continue;
#pragma unroll
          for (int j = 0; j < N; ++j) {
            const LogV lj = getlog(t, j);
            if (g_commit(t, j) > llen(lj)) return IV_ERR;
            if (!is_prefix_n(lj, g_commit(t, j), getlog(t, i))) return IV_BAD;
          }
        }
        return IV_OK;
      }
      case MI_LeaderCompleteness: {                                   // :1089-1099
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const LogV li = getlog(t, i);
          const int ci = g_commit(t, i);
          if (ci > llen(li)) return IV_ERR;
#pragma unroll 1
          for (int idx = 1; idx <= LMAXW; ++idx) {
            if (idx > ci) continue;
            const u32 e = lent(li, idx - 1);
#pragma unroll
            for (int l = 0; l < N; ++l) {
              if (!((leaders >> l) & 1u) || !(g_term(t, l) > eterm(e))) continue;
              const LogV ll = getlog(t, l);
              if (idx > llen(ll)) return IV_ERR;                      // log[l][idx] outside its domain
              if (lent(ll, idx - 1) != e) return IV_BAD;
            }
          }
        }
        return IV_OK;
      }
      case MI_BoundedTrace: return glen(t) <= 24 ? IV_OK : IV_BAD;   // :1143
      case MI_FirstBecomeLeader: return hflag(t.h1, F_BL) ? IV_BAD : IV_OK;
      case MI_FirstCommit: return t.commit == 0 ? IV_OK : IV_BAD;
      case MI_FirstRestart: {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) ok &= restarted(t, i) < 2;
        return ok ? IV_OK : IV_BAD;
      }
      case MI_LeadershipChange: return hget(t.h0, H_HL, 4) < 2 ? IV_OK : IV_BAD;
      case MI_MembershipChange: return hget(t.h0, H_MC, 3) < 1 ? IV_OK : IV_BAD;
      case MI_MultipleMembershipChanges: return hget(t.h0, H_MC, 3) < 2 ? IV_OK : IV_BAD;
      case MI_ConcurrentLeaders: return popc32(leaders) >= 2 ? IV_BAD : IV_OK;
      case MI_EntryCommitted: return hflag(t.h1, F_CE) ? IV_BAD : IV_OK;
      case MI_CommitWhenConcurrentLeaders: {                          // :1165-1176
        const int k0 = hget(t.h1, H_K0, 10);
        return (k0 > 0 && glen(t) >= k0 + 2 && popc32(leaders) >= 2) ? IV_BAD : IV_OK;
      }
      case MI_MajorityOfClusterRestarts: {                            // :1212-1226
        bool logs = false;
#pragma unroll
        for (int i = 0; i < N; ++i)
#pragma unroll
          for (int j = 0; j < N; ++j) if (i != j && llen(getlog(t, i)) >= 2 && llen(getlog(t, j)) >= 1) logs = true;
        if (!logs) return IV_OK;
        int rs = 0;
#pragma unroll
        for (int i = 0; i < N; ++i) rs += restarted(t, i) >= 1;
        if (!(rs * 2 > N)) return IV_OK;
        return hflag(t.h1, F_RCLOSE) ? IV_OK : IV_BAD;
      }
      case MI_AddSucessful: return hflag(t.h1, F_ADD) ? IV_BAD : IV_OK;
      case MI_MembershipChangeCommits: return hflag(t.h1, F_CMC) ? IV_BAD : IV_OK;
      case MI_MultipleMembershipChangesCommit: return hflag(t.h1, F_CMC2) ? IV_BAD : IV_OK;
      case MI_AddCommits: return hflag(t.h1, F_ADDCOMMITS) ? IV_BAD : IV_OK;
      case MI_NewlyJoinedBecomeLeader: return hflag(t.h1, F_NEWLEADER) ? IV_BAD : IV_OK;
      case MI_LeaderChangesDuringConfChange: return hflag(t.h1, F_LCDCC) ? IV_BAD : IV_OK;
      default: return IV_OK;
    }
  }
  // Invariants in cfg order (TLC stops at the first false or erroring one).
  // Returns 0 if all hold, else (kind << 8 | invariant id) with kind IV_BAD / IV_ERR.
  RMC_HD static u32 check_invariants(const Work& t, const MembRuntime& rt) {
    for (u32 q = 0; q < rt.n_inv; ++q) {
      const u64 w = q < 8 ? rt.inv_order[0] : q < 16 ? rt.inv_order[1] : q < 24 ? rt.inv_order[2] : rt.inv_order[3];
      const int id = (int)((w >> (8 * (q & 7))) & 255u);
      const int r = inv(t, id, rt);
      if (r != IV_OK) return ((u32)r << 8) | (u32)id;
    }
    return 0;
  }

  // ------------------------------------------------------------ symmetric fingerprint of the VIEW
  RMC_HD static int pi_of(u32 pi, int x) { return (int)((pi >> (2 * x)) & 3u); }
  RMC_HD static u32 pmask(u32 m, u32 pi) {
    u32 r = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) r |= ((m >> j) & 1u) << pi_of(pi, j);
    return r;
  }
  RMC_HD static u32 pentry(u32 e, u32 pi, u32 cfgt) {   // rename servers inside a config entry
    return etype(e) == cfgt ? (e & ~(u32)lomask(VW)) | m2r(pmask(r2m(evalue(e)), pi)) : e;
  }
  RMC_HD static u64 fmix(u64 h) { h ^= h >> 33; h *= P2; h ^= h >> 29; h *= P3; h ^= h >> 32; return h; }
  // any ConfigEntry (server-valued) inside a log or a log-carrying message?  Without one,
  // permuting the view only renames the server-valued fields (the cheap path).
  // a message code carrying a ConfigEntry (in its log / entries field): its permuted code renames
  // config values too (perm_entries), not only its server fields
  RMC_HD static bool msg_has_config(u64 c, u32 cfgt) {
    const u64 dp = mdesc_packed(mcls(c));
    const int ol = (int)((dp >> 28) & 127), kind = (int)((dp >> 35) & 3);
    bool any = false;
    if (kind == 1) {
      const int cnt = (int)fld(c, ol, IB);
#pragma unroll
      for (int p = 0; p < MAXLOG; ++p) if (p < cnt && etype((u32)fld(c, ol + IB + p * EW, EW)) == cfgt) any = true;
    } else if (kind == 2) {
      if (fld(c, ol, 1) && etype((u32)fld(c, ol + 1, EW)) == cfgt) any = true;
    }
    return any;
  }
  RMC_HD static bool logs_have_config(const Work& t, u32 cfgt) {
    bool any = false;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const LogV l = getlog(t, i);
#pragma unroll
      for (int p = 0; p < MAXLOG; ++p) if (p < llen(l) && etype(lent(l, p)) == cfgt) any = true;
    }
    return any;
  }
  RMC_HD static bool has_config_entries(const Work& t, u32 cfgt) {
    bool any = logs_have_config(t, cfgt);
#pragma unroll 1
    for (int q = 0; q < MK; ++q) {
      const u64 e = sel(t.bag, q);
      if (e == EMPTY) break;
      const u64 c = mcode(e), dp = mdesc_packed(mcls(c));
      const int ol = (int)((dp >> 28) & 127), kind = (int)((dp >> 35) & 3);
      if (kind == 1) {
        const int cnt = (int)fld(c, ol, IB);
#pragma unroll
        for (int p = 0; p < MAXLOG; ++p) if (p < cnt && etype((u32)fld(c, ol + IB + p * EW, EW)) == cfgt) any = true;
      } else if (kind == 2) {
        if (fld(c, ol, 1) && etype((u32)fld(c, ol + 1, EW)) == cfgt) any = true;
      }
    }
    return any;
  }
  // permutation number p (0 <= p < N!) -> pi packed 2 bits per server (Lehmer code)
  RMC_HD static u32 perm_of(int p) {   // the p-th permutation (Lehmer order), 2 bits per server
    static_assert(N <= 4, "permutation tables hold N <= 4");
    return kPermTables[N].perm[p];
  }
  // Permutation-aware hashing of the view (SYMMETRY perms): for every permutation p, the hash of
  // the permuted view is a sum of element hashes (servers, bag entries), so each element is
  // decoded once and then hashed under all permutations with pi a compile-time constant
  // (loop interchange: no per-permutation re-decoding, no re-sorting of the bag).
  //   server i: fmix(w0(p) ^ hl_i), w0 = (p(i), term, state, p(votedFor), commitIndex,
  //             p(votesResponded), p(votesGranted), nextIndex/matchIndex rows permuted),
  //             hl_i = hash of log[i] (permuted only when it holds ConfigEntry values)
  //   message:  fmix(p(entry) ^ K), entry = code << CNTB | count with mdest/msource/mserver renamed
  static constexpr u64 K_LOG = 0x243F6A8885A308D3ull, K_MSG = 0x13198A2E03707344ull;
  RMC_HD static u64 log_hash(LogV l, u64 seed) { return fmix((l.a * P1) ^ ((u64)l.b << 7) ^ seed ^ K_LOG); }
  RMC_HD static u64 server_word(const Work& t, int i, u32 pi) {
    const int vo = g_voted(t, i);
    u32 rn = 0, rm = 0;
#pragma unroll
    for (int j = 0; j < N; ++j) {
      rn |= (u32)g_next(t, i, j) << (IB * pi_of(pi, j));
      rm |= (u32)g_match(t, i, j) << (IB * pi_of(pi, j));
    }
    u32 pv = (u32)N;
#pragma unroll
    for (int j = 0; j < N; ++j) pv = vo == j ? (u32)pi_of(pi, j) : pv;
    return (u64)pi_of(pi, i) | (u64)g_term(t, i) << 2 | (u64)g_st(t, i) << 5 | (u64)pv << 7 | (u64)g_commit(t, i) << 10 |
           (u64)pmask(g_vr(t, i), pi) << 13 | (u64)pmask(g_vg(t, i), pi) << 17 | (u64)rn << 21 | (u64)rm << 33;
  }
  RMC_HD static LogV perm_log(LogV l, u32 pi, u32 cfgt) {
#pragma unroll
    for (int p = 0; p < MAXLOG; ++p) if (p < llen(l)) l = lset(l, p, pentry(lent(l, p), pi, cfgt));
    return l;
  }
  RMC_HD static u64 perm_entries(u64 c, u32 pi, u32 cfgt) {   // config values inside a message's log / entry
    const u64 dp = mdesc_packed(mcls(c));
    const int ol = (int)((dp >> 28) & 127), kind = (int)((dp >> 35) & 3);
    auto setf = [&](u64 x, int off, int w, u64 v) { const int sh = CODEB - off - w; return (x & ~(lomask(w) << sh)) | (v << sh); };
    if (kind == 1) {
      const int cnt = (int)fld(c, ol, IB);
#pragma unroll
      for (int p = 0; p < MAXLOG; ++p)
        if (p < cnt) { const int off = ol + IB + p * EW; c = setf(c, off, EW, pentry((u32)fld(c, off, EW), pi, cfgt)); }
    } else if (kind == 2) {
      if (fld(c, ol, 1)) c = setf(c, ol + 1, EW, pentry((u32)fld(c, ol + 1, EW), pi, cfgt));
    }
    return c;
  }
  // accumulate the hashes of pi_p(view) for p in [0, NP)
  template <int NP, bool CE>
  RMC_HD static void view_acc(const Work& t, u64 seed, u32 cfgt, u64 (&acc)[NPERM]) {
#pragma unroll
    for (int p = 0; p < NP; ++p) acc[p] = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const LogV l = getlog(t, i);
      const u64 hl = CE ? 0 : log_hash(l, seed);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const u64 h = CE ? log_hash(perm_log(l, perm_of(p), cfgt), seed) : hl;
        acc[p] += fmix(server_word(t, i, perm_of(p)) ^ h);
      }
    }
    // bag entries: sorted with EMPTY last, so stop at the first empty slot
#pragma unroll 1
    for (int q = 0; q < MK; ++q) {
      const u64 e = sel(t.bag, q);
      if (e == EMPTY) break;
      u64 c = mcode(e);
      const u64 dp = mdesc_packed(mcls(c));
      const int sd = CODEB + CNTB - (int)(dp & 127) - SB, ss = CODEB + CNTB - (int)((dp >> 7) & 127) - SB;
      const int ov = (int)((dp >> 21) & 127), sv = CODEB + CNTB - ov - SB;
      const u32 xd = (u32)((e >> sd) & lomask(SB)), xs = (u32)((e >> ss) & lomask(SB)), xv = ov ? (u32)((e >> sv) & lomask(SB)) : 0u;
      u64 base = e & ~(lomask(SB) << sd) & ~(lomask(SB) << ss);
      if (ov) base &= ~(lomask(SB) << sv);
#pragma unroll
      for (int p = 0; p < NP; ++p) {
        const u32 pi = perm_of(p);
        u64 x = CE ? ((perm_entries(mcode(base), pi, cfgt) << CNTB) | (base & lomask(CNTB))) : base;
        x |= (u64)pi_of(pi, (int)xd) << sd | (u64)pi_of(pi, (int)xs) << ss;
        if (ov) x |= (u64)pi_of(pi, (int)xv) << sv;
        acc[p] += fmix(x ^ seed ^ K_MSG);
      }
    }
  }
  // hash of pi(view) for one runtime permutation pi (same element hashes as view_acc)
  template <bool CE>
  RMC_HD static u64 view_hash1(const Work& t, u32 pi, u64 seed, u32 cfgt) {
    u64 acc = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const LogV l = getlog(t, i);
      acc += fmix(server_word(t, i, pi) ^ log_hash(CE ? perm_log(l, pi, cfgt) : l, seed));
    }
#pragma unroll 1
    for (int q = 0; q < MK; ++q) {
      const u64 e = sel(t.bag, q);
      if (e == EMPTY) break;
      const u64 dp = mdesc_packed(mcls(mcode(e)));
      const int sd = CODEB + CNTB - (int)(dp & 127) - SB, ss = CODEB + CNTB - (int)((dp >> 7) & 127) - SB;
      const int ov = (int)((dp >> 21) & 127), sv = CODEB + CNTB - ov - SB;
      u64 x = e & ~(lomask(SB) << sd) & ~(lomask(SB) << ss);
      if (ov) x &= ~(lomask(SB) << sv);
      if (CE) x = (perm_entries(mcode(x), pi, cfgt) << CNTB) | (x & lomask(CNTB));
      x |= (u64)pi_of(pi, (int)((e >> sd) & lomask(SB))) << sd | (u64)pi_of(pi, (int)((e >> ss) & lomask(SB))) << ss;
      if (ov) x |= (u64)pi_of(pi, (int)((e >> sv) & lomask(SB))) << sv;
      acc += fmix(x ^ seed ^ K_MSG);
    }
    return acc;
  }
  // view_hash1 with the bag read through an accessor (fingerprint_tlc: the per-lane LDS copy, so the
  // successor's bag registers are dead once staged and a runtime entry index is one LDS read instead of
  // a select chain over MK + 1 registers)
  template <bool CE, class Bag>
  RMC_HD static u64 view_hash1_bag(const Work& t, const Bag& bag, int len, u32 pi, u64 seed, u32 cfgt) {
    u64 acc = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const LogV l = getlog(t, i);
      acc += fmix(server_word(t, i, pi) ^ log_hash(CE ? perm_log(l, pi, cfgt) : l, seed));
    }
#pragma unroll 1
    for (int q = 0; q < len; ++q) {
      const u64 e = bag[q];
      const u64 dp = mdesc_packed(mcls(mcode(e)));
      const int sd = CODEB + CNTB - (int)(dp & 127) - SB, ss = CODEB + CNTB - (int)((dp >> 7) & 127) - SB;
      const int ov = (int)((dp >> 21) & 127), sv = CODEB + CNTB - ov - SB;
      u64 x = e & ~(lomask(SB) << sd) & ~(lomask(SB) << ss);
      if (ov) x &= ~(lomask(SB) << sv);
      if (CE) x = (perm_entries(mcode(x), pi, cfgt) << CNTB) | (x & lomask(CNTB));
      x |= (u64)pi_of(pi, (int)((e >> sd) & lomask(SB))) << sd | (u64)pi_of(pi, (int)((e >> ss) & lomask(SB))) << ss;
      if (ov) x |= (u64)pi_of(pi, (int)((e >> sv) & lomask(SB))) << sv;
      acc += fmix(x ^ seed ^ K_MSG);
    }
    return acc;
  }
  // Permutation-invariant signature of every server (sig_i(pi(t)) = sig_pi(i)(t)): its own fields,
  // its nextIndex/matchIndex rows as a multiset, its log with config values reduced to
  // (cardinality, membership of i), and the multiset of the messages it sends / receives.  The
  // bag is walked once; each message is credited to its destination and its source.
  RMC_HD static void server_sigs(const Work& t, u32 cfgt, u64 (&sig)[N]) {
    u64 ms[N];
#pragma unroll
    for (int i = 0; i < N; ++i) ms[i] = 0;
#pragma unroll 1
    for (int q = 0; q < MK; ++q) {
      const u64 e = sel(t.bag, q);
      if (e == EMPTY) break;
      const u64 c = mcode(e), dp = mdesc_packed(mcls(c));
      const int d = (int)fld(c, (int)(dp & 127), SB), sr = (int)fld(c, (int)((dp >> 7) & 127), SB);
      const u64 base = (u64)mcls(c) | (u64)fld(c, (int)((dp >> 14) & 127), TB) << 3 | (u64)mcount(e) << 6 | 0xA5ull << 16;
      const bool self = d == sr;
      const u64 hd = fmix(base | 1ull << 13 | (self ? (1ull << 14 | 1ull << 15) : 0ull));   // the destination's view
      const u64 hs = self ? 0ull : fmix(base | 1ull << 14);                                 // the source's view
#pragma unroll
      for (int i = 0; i < N; ++i) ms[i] += (d == i ? hd : 0ull) + (sr == i ? hs : 0ull);
    }
#pragma unroll
    for (int i = 0; i < N; ++i) {
      const int vo = g_voted(t, i);
      const u32 vr = g_vr(t, i), vg = g_vg(t, i);
      const u64 w = (u64)g_term(t, i) | (u64)g_st(t, i) << 3 | (u64)g_commit(t, i) << 5 | (u64)(vo == N) << 8 | (u64)(vo == i) << 9 |
                    (u64)popc32(vr) << 10 | (u64)popc32(vg) << 13 | (u64)((vr >> i) & 1u) << 16 | (u64)((vg >> i) & 1u) << 17 |
                    (u64)g_next(t, i, i) << 18 | (u64)g_match(t, i, i) << 21;
      u64 rows = 0;
#pragma unroll
      for (int j = 0; j < N; ++j)
        if (j != i) rows += fmix((u64)g_next(t, i, j) | (u64)g_match(t, i, j) << 3 | 0x5151ull << 8);
      const LogV l = getlog(t, i);
      u64 lh = (u64)llen(l);
#pragma unroll
      for (int p = 0; p < MAXLOG; ++p) {
        if (p >= llen(l)) continue;
        u32 en = lent(l, p);
        if (etype(en) == cfgt) { const u32 m = r2m(evalue(en)); en = (en & ~(u32)lomask(VW)) | (u32)popc32(m) << 1 | ((m >> i) & 1u); }
        lh = lh * P1 + (u64)en + 1;
      }
      sig[i] = fmix(w ^ fmix(rows ^ 0x9E37ull) ^ rotl64(fmix(lh), 17) ^ rotl64(ms[i], 31));
    }
  }
  // FP64 of raftmc for this spec.  With SYMMETRY: min over the permutations that respect the
  // order of the server signatures (ties permuted among themselves).  For pi(s) in the orbit of
  // s those are exactly the signature-respecting permutations of s composed with pi^-1, so the
  // minimum runs over the same set of permuted views: canonical, and usually over one
  // permutation instead of N!.  Without SYMMETRY: the identity.
  RMC_HD static u64 fingerprint(const Work& t, u64 seed, const MembRuntime& rt) {   // host entry: either mode
    return (rt.symmetry && rt.sym_tlc) ? fingerprint_tlc(t, seed, rt) : fingerprint_orbit(t, seed, rt);
  }
  RMC_HD static u64 fingerprint_orbit(const Work& t, u64 seed, const MembRuntime& rt) {
    const bool ce = has_config_entries(t, rt.cfg_type);
    u64 best;
    if (!rt.symmetry) {
      u64 acc[NPERM];
      if (ce) view_acc<1, true>(t, seed, rt.cfg_type, acc);
      else view_acc<1, false>(t, seed, rt.cfg_type, acc);
      best = acc[0];
    } else {
      u64 sig[N];
      server_sigs(t, rt.cfg_type, sig);
      u32 lo = 0, hi = 0, rank_pi = 0;                                 // packed 3-bit bounds per server
      bool distinct = true;
#pragma unroll
      for (int i = 0; i < N; ++i) {
        u32 l = 0, e = 0;
#pragma unroll
        for (int j = 0; j < N; ++j) { l += sig[j] < sig[i]; e += sig[j] == sig[i]; }
        lo |= l << (3 * i); hi |= (l + e) << (3 * i);
        rank_pi |= l << (2 * i);
        distinct &= e == 1;
      }
      if (distinct) {   // the one signature-respecting permutation: every server to its rank
        best = ce ? view_hash1<true>(t, rank_pi, seed, rt.cfg_type) : view_hash1<false>(t, rank_pi, seed, rt.cfg_type);
        const u64 fp = fmix(best ^ seed);
        return fp ? fp : 1ull;
      }
      auto valid = [&](u32 pi) {
        bool ok = true;
#pragma unroll
        for (int i = 0; i < N; ++i) {
          const u32 x = (u32)pi_of(pi, i);
          ok &= x >= ((lo >> (3 * i)) & 7u) && x < ((hi >> (3 * i)) & 7u);
        }
        return ok;
      };
      int nvalid = 0;
#pragma unroll 1
      for (int p = 0; p < NPERM; ++p) nvalid += valid(perm_of(p));
      best = ~0ull;
#pragma unroll 1
      for (int k = 0; k < nvalid; ++k) {
        u32 pi = 0;
        int c = 0;
#pragma unroll 1
        for (int p = 0; p < NPERM; ++p) { const u32 q = perm_of(p); if (valid(q)) { if (c == k) pi = q; ++c; } }
        const u64 h = ce ? view_hash1<true>(t, pi, seed, rt.cfg_type) : view_hash1<false>(t, pi, seed, rt.cfg_type);
        best = h < best ? h : best;
      }
    }
    const u64 fp = fmix(best ^ seed);
    return fp ? fp : 1ull;
  }

  // ------------------------------------------------------------ TLC-mode symmetry (MC_COMPAT_SYM_TLC)
  // TLC's rule ([ext], oracle/engine.h canon_key "tlc"): of the N! permuted states take the one
  // whose variable tuple, in declaration order (raft.tla:114-185: messages, history, currentTerm,
  // state, votedFor, log, commitIndex, votesResponded, votesGranted, nextIndex, matchIndex), is
  // least under TLC's value order (oracle tla.h cmp), then fingerprint its VIEW.  Unlike the orbit
  // mode this depends on history, which is not stored; what the comparison needs of it is: the
  // order of the permuted history["global"] sequences of THIS state (kept as hr0/hr1, a
  // competition rank per permutation, refined by every appended entry; a flag marks it discrete,
  // after which appends cannot change it), the permutation-invariant counters, and the per-server
  // [restarted, timeout] record (h0).
  static constexpr int RKB = NPERM <= 2 ? 1 : bits_for(NPERM - 1);   // bits per rank
  static constexpr int RPW = 60 / RKB;                                // ranks per word (bits 60..63 free)
  static_assert(NPERM <= 2 * RPW, "history ranks fit hr0/hr1");
  static constexpr u64 HR_DISCRETE = 1ull << 63;                     // in hr1: all ranks distinct
  RMC_HD static u32 hrank(const Work& t, int p) {
    return (u32)(((p < RPW ? t.hr0 : t.hr1) >> (RKB * (p < RPW ? p : p - RPW))) & lomask(RKB));
  }
  RMC_HD static int pinv(u32 pi, int s) {   // the server pi maps to s
    int r = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) r = pi_of(pi, i) == s ? i : r;
    return r;
  }
  // a message code with every server-valued field renamed by pi (and config values inside its
  // log / entry when ce); order preserving like the code itself
  RMC_HD static u64 perm_code(u64 c, u32 pi, bool ce, u32 cfgt) {
    constexpr u64 MD_DST = md_lut(0), MD_SRC = md_lut(1), MD_SRV = md_lut(2);
    RMC_FPS(13, 1); RMC_FPS(19, ce);
#if defined(RMC_FP_STATS) && !defined(__HIP_DEVICE_COMPILE__)
    RMC_FPS(26, ce && msg_has_config(c, cfgt));
#endif
    const int cl = mcls(c);
    const int od = md_field(MD_DST, cl), os = md_field(MD_SRC, cl), ov = md_field(MD_SRV, cl);
    const int sd = CODEB - od - SB, ss = CODEB - os - SB, sv = CODEB - ov - SB;
    u64 x = c & ~(lomask(SB) << sd) & ~(lomask(SB) << ss);
    if (ov) x &= ~(lomask(SB) << sv);
    if (ce) x = perm_entries(x, pi, cfgt);
    x |= (u64)pi_of(pi, (int)((c >> sd) & lomask(SB))) << sd | (u64)pi_of(pi, (int)((c >> ss) & lomask(SB))) << ss;
    if (ov) x |= (u64)pi_of(pi, (int)((c >> sv) & lomask(SB))) << sv;
    return x;
  }
  // Order key of pi(e) among the permutations of one history entry e = (x, y) (prefix_step's
  // codes): the entry record's server-valued fields in field-name order (records compare field
  // by field in name order; the invariant fields tie).
  // Branch-free on purpose: the kind differs from lane to lane, and the switch this replaces was
  // compiled for gfx950 into code that gave every lane another lane's case (tests/native/
  // tlc_refine_probe.hip: garbage keys on the device, correct ones on the host).
  RMC_HD static u64 entry_key(u64 x, u64 y, u32 pi, u32 cfgt) {
    const int kind = (int)(x & 15u);
    const u64 ex = (u64)pi_of(pi, (int)((x >> 4) & 15u));
    const u32 aux = (u32)(x >> 8);
    const bool msg = kind == HE_SEND || kind == HE_RECV;
    const u64 pa = (u64)pi_of(pi, (int)(aux & 3u));
    const u64 pm = m2r(pmask(aux & (u32)lomask(N), pi));
    const u64 kmsg = ex << CODEB | perm_code(msg ? y : 0ull, pi, true, cfgt);                 // action, executedOn, msg
    u64 k = ex;                                                                             // Restart, Timeout
    k = (kind == HE_TRYADD || kind == HE_ADD) ? (pa << 2 | ex) : k;                         // action, added, executedOn
    k = (kind == HE_TRYREM || kind == HE_REM) ? (ex << 2 | pa) : k;                         // action, executedOn, removed
    k = kind == HE_BL ? (ex << 4 | pm) : k;                                                 // action, executedOn, leaders
    k = kind == HE_CE ? ((u64)pentry(aux, pi, cfgt) << 2 | ex) : k;                         // action, entry, executedOn
    k = kind == HE_CMC ? (pm << 2 | ex) : k;                                                // action, config, executedOn
    return msg ? kmsg : k;
  }
  // refine the history ranks by the entries this successor appended (apply).  Runtime loops and
  // keys recomputed on the fly: small code in every kernel that inlines apply, no scratch arrays
  // (the work only happens while the ranks are not yet discrete, i.e. in the first few levels).
  RMC_HD static void tlc_refine(const Work& s, Work& t, const Delta& d, u32 cfgt) {
    (void)s;
    u64 x[2], y[2];
    const int n = appended_entries(d, x[0], y[0], x[1], y[1]);
#pragma unroll 1
    for (int e = 0; e < n && !(t.hr1 & HR_DISCRETE); ++e) {
      const u64 xe = e ? x[1] : x[0], ye = e ? y[1] : y[0];
      u64 w0 = 0, w1 = 0;
      bool distinct = true;
#pragma unroll 1
      for (int p = 0; p < NPERM; ++p) {
        const u32 rp = hrank(t, p);
        u32 r = 0, same = 0;   // permutations of a lower old rank; the others of p's rank class
#pragma unroll 1
        for (int q = 0; q < NPERM; ++q) {
          const u32 rq = hrank(t, q);
          r += rq < rp ? 1u : 0u;
          same |= (rq == rp && q != p) ? 1u << q : 0u;
        }
        if (same) {   // the new entry's keys order p's rank class (a singleton class needs none)
          const u64 kp = entry_key(xe, ye, perm_of(p), cfgt);
#pragma unroll 1
          for (u32 m = same; m; m &= m - 1u) {
            const u64 kq = entry_key(xe, ye, perm_of(__builtin_ctz(m)), cfgt);
            r += kq < kp ? 1u : 0u;
            distinct &= kq != kp;
          }
        }
        if (p < RPW) w0 |= (u64)r << (RKB * p); else w1 |= (u64)r << (RKB * (p - RPW));
      }
      t.hr0 = w0; t.hr1 = w1 | (distinct ? HR_DISCRETE : 0ull);
    }
  }
  RMC_HD static bool single(u32 cand) { return (cand & (cand - 1u)) == 0u; }
  // keep, among the candidate permutations, those whose key (p, pi) is least
  // (one pass: each candidate's key is evaluated once)
  template <class F>
  RMC_HD static u32 keep_min(u32 cand, F key, u64* least = nullptr) {
    u64 best = ~0ull;
    u32 out = 0;
#pragma unroll 1
    for (u32 m = cand; m; m &= m - 1u) {   // the candidates only (a lane's trip count is |cand|)
      const int p = __builtin_ctz(m);
      const u64 k = key(p, perm_of(p));
      out = k < best ? (1u << p) : k == best ? (out | 1u << p) : out;
      best = k < best ? k : best;
    }
    if (least) *least = best;   // the kept candidates' key
    return out;
  }
  // pi^-1 packed like pi (2 bits per server): pinv(pi, s) == pi_of(inv_of(pi), s)
  RMC_HD static u32 inv_of(u32 pi) {
    u32 r = 0;
#pragma unroll
    for (int i = 0; i < N; ++i) r |= (u32)i << (2 * pi_of(pi, i));
    return r;
  }
  // TLC's order over the variables after the messages, in as few integer keys as fit: a run of
  // consecutive keys of known widths packed most significant first into one u64 orders the run
  // exactly as comparing key by key does, so one keep_min settles a whole run (a wave's trip count
  // is the number of runs, not of keys).
  static constexpr int RTB = 2 + 3;   // server[x] = [restarted (<= MaxRestarts = 2), timeout (3 bits)]
  static constexpr int SCAL_BITS = RKB + N * (RTB + TB + 2 + VB);
  static constexpr int LOG_BITS = IB + MAXLOG * EW;
  static constexpr int CV_BITS = N * IB + 2 * N * 4;
  static constexpr int NM_BITS = N * N * IB;
  static_assert(SCAL_BITS <= 64 && LOG_BITS <= 64 && CV_BITS <= 64 && NM_BITS <= 64, "fused TLC keys fit 64 bits");
  // history (the rank of the permuted global sequence, then server[x] of the server mapped to x),
  // currentTerm, state ("Candidate" < "Follower" < "Leader"), votedFor (Nil = 0 sorts first)
  RMC_HD static u64 key_scalars(const Work& t, int p, u32 pi) {
    const u32 iv = inv_of(pi);
    u64 k = hrank(t, p);
#pragma unroll
    for (int x = 0; x < N; ++x) { const int i = pi_of(iv, x); k = k << RTB | (u64)restarted(t, i) << 3 | (u64)timeouts(t, i); }
#pragma unroll
    for (int x = 0; x < N; ++x) k = k << TB | (u64)g_term(t, pi_of(iv, x));
#pragma unroll
    for (int x = 0; x < N; ++x) { const int st = g_st(t, pi_of(iv, x)); k = k << 2 | (u64)(st == (int)C ? 0 : st == (int)F ? 1 : 2); }
#pragma unroll
    for (int x = 0; x < N; ++x) { const int v = g_voted(t, pi_of(iv, x)); k = k << VB | (u64)(v == N ? 0 : 1 + pi_of(pi, v)); }
    return k;
  }
  // log[x]: length, then the entries (config entries renamed), 0 past the end
  RMC_HD static u64 key_log(const Work& t, int x, u32 pi, u32 cfgt) {
    const LogV l = getlog(t, pinv(pi, x));
    const int n = llen(l);
    u64 k = (u64)n;
#pragma unroll
    for (int pos = 0; pos < MAXLOG; ++pos) k = k << EW | (pos < n ? (u64)pentry(lent(l, pos), pi, cfgt) : 0ull);
    return k;
  }
  // commitIndex, votesResponded, votesGranted (sets: cardinality, then elements: m2r)
  RMC_HD static u64 key_cv(const Work& t, u32 pi) {
    const u32 iv = inv_of(pi);
    u64 k = 0;
#pragma unroll
    for (int x = 0; x < N; ++x) k = k << IB | (u64)g_commit(t, pi_of(iv, x));
#pragma unroll
    for (int x = 0; x < N; ++x) k = k << 4 | (u64)m2r(pmask(g_vr(t, pi_of(iv, x)), pi));
#pragma unroll
    for (int x = 0; x < N; ++x) k = k << 4 | (u64)m2r(pmask(g_vg(t, pi_of(iv, x)), pi));
    return k;
  }
  // nextIndex (match: matchIndex)
  RMC_HD static u64 key_nm(const Work& t, u32 pi, bool match) {
    const u32 iv = inv_of(pi);
    u64 k = 0;
#pragma unroll
    for (int z = 0; z < N * N; ++z) {
      const int i = pi_of(iv, z / N), j = pi_of(iv, z % N);
      k = k << IB | (u64)(match ? g_match(t, i, j) : g_next(t, i, j));
    }
    return k;
  }
  // 64-bit hash of the permuted state pi(t) as far as TLC's order sees it: its VIEW (view_hash1), the
  // rank of its permuted history["global"] and its per-server [restarted, timeout] records
  template <bool CE>
  RMC_HD static u64 perm_state_hash(const Work& t, int p, u32 pi, u32 cfgt) {
    u64 h = view_hash1<CE>(t, pi, 0x243F6A8885A308D3ull, cfgt) ^ fmix((u64)hrank(t, p) ^ 0x13198A2E03707344ull);
#pragma unroll
    for (int x = 0; x < N; ++x) {
      const int i = pinv(pi, x);
      h += fmix(((u64)restarted(t, i) << 8 | (u64)timeouts(t, i)) ^ ((u64)(x + 1) * P1));
    }
    return h;
  }
  // Candidates whose permuted states coincide (pi' = pi o sigma, sigma an automorphism of t) tie on
  // every criterion, so a lane holding a symmetric state walked all of them (its wave with it).  Keep
  // one candidate per permuted state: equal hashes <=> equal permuted states up to a 2^-64
  // coincidence, the fingerprint's own collision class.  O(|cand|^2) hashes (small sets only), one
  // call site (the kernels stay within short-branch range); the config-entry hash variant is exact
  // for states without config entries too.
  RMC_HD static u32 dedup_auto(const Work& t, u32 cand, u32 cfgt) {
    u32 out = 0, todo = cand, cmp = 0;
    int p = 0;
    u64 hp = 0;
    bool placing = false;   // hp holds candidate p's hash; cmp: kept candidates not yet compared with p
#pragma unroll 1
    while (placing || todo) {
      if (!placing) { p = __builtin_ctz(todo); todo &= todo - 1u; cmp = out; }
      const int idx = placing ? __builtin_ctz(cmp) : p;
      const u64 h = perm_state_hash<true>(t, idx, perm_of(idx), cfgt);
      if (!placing) { hp = h; placing = true; }
      else {
        cmp &= cmp - 1u;
        if (h == hp) { placing = false; continue; }        // p repeats a kept candidate's state
      }
      if (!cmp) { out |= 1u << p; placing = false; }
    }
    return out;
  }
  // The bag as an array indexed at run time (tlc_min_perm reads entries by runtime index inside its
  // permutation loops; from the register array every read is a select chain over MK+1 entries): on
  // the device a per-lane slice of LDS (lane-interleaved, conflict-free), on the host a local array.
#ifndef RMC_TLC_CFG_MASK
#define RMC_TLC_CFG_MASK 1
#endif
// the one-pass narrowing's loop over a state's messages (RMC_TLC_QU: its unroll factor, so a lane has several LDS
// reads of bag entries in flight instead of one per iteration)
#ifndef RMC_TLC_QU
#define RMC_TLC_QU 1
#endif
#if RMC_TLC_QU == 4
#define RMC_QLOOP _Pragma("unroll 4")
#elif RMC_TLC_QU == 2
#define RMC_QLOOP _Pragma("unroll 2")
#else
#define RMC_QLOOP _Pragma("unroll 1")
#endif
  // cfgm: the entries whose message carries a ConfigEntry (the only ones perm_entries changes;
  // with RMC_TLC_CFG_MASK 0 every entry of a state with config entries anywhere, as in round 4)
  struct BagRef {
    const u64* p;
    int stride;
    u32 cfgm;
    RMC_HD u64 operator[](int q) const { return p[q * stride]; }
    RMC_HD bool cfg(int q) const { return (cfgm >> q) & 1u; }
  };
  RMC_HD static u64 next_perm_code(const BagRef& bag, int len, u32 pi, bool ce, u32 cfgt, bool have_last, u64 last) {
    u64 best = ~0ull;   // the least permuted message code above `last`
#pragma unroll 1
    for (int q = 0; q < len; ++q) {
      const u64 c = perm_code(mcode(bag[q]), pi, ce && bag.cfg(q), cfgt);
      if ((!have_last || c > last) && c < best) best = c;
    }
    return best;
  }
  // The least permuted code of one message over all permutations, without trying them: with no
  // ConfigEntry renamed (ce false) only its server-valued fields change, so the least code renames
  // them in order of significance -- the most significant to server 0, the next different one to 1,
  // the next to 2.  *lab: the servers of those fields and their labels (server | label << 4, per
  // field, most significant first), for cand_of.
  RMC_HD static u64 canon_code(u64 c, u32& lab) {
    constexpr u64 MD_DST = md_lut(0), MD_SRC = md_lut(1), MD_SRV = md_lut(2);
    const int cl = mcls(c);
    const int od = md_field(MD_DST, cl), os = md_field(MD_SRC, cl), ov = md_field(MD_SRV, cl);
    const int sd = CODEB - od - SB, ss = CODEB - os - SB, sv = CODEB - ov - SB;
    const bool has_v = ov != 0;
    // the fields (shift, server), most significant (largest shift) first: a 3-element sorting
    // network of selects (lanes hold different message classes: no divergent branches); a class
    // without a third server field gets shift -1 there, which sorts last
    int h0 = sd, h1 = ss, h2 = has_v ? sv : -1;
    int f0 = (int)((c >> sd) & lomask(SB)), f1 = (int)((c >> ss) & lomask(SB)), f2 = has_v ? (int)((c >> sv) & lomask(SB)) : 0;
    auto cswap = [](int& ha, int& fa, int& hb, int& fb) {
      const bool sw = hb > ha;
      const int th = sw ? hb : ha, tf = sw ? fb : fa;
      hb = sw ? ha : hb; fb = sw ? fa : fb; ha = th; fa = tf;
    };
    cswap(h0, f0, h1, f1); cswap(h1, f1, h2, f2); cswap(h0, f0, h1, f1);
    const int l0 = 0, l1 = f1 == f0 ? 0 : 1;
    const int l2 = f2 == f0 ? l0 : f2 == f1 ? l1 : l1 + 1;
    u64 x = c & ~(lomask(SB) << sd) & ~(lomask(SB) << ss);
    if (has_v) x &= ~(lomask(SB) << sv);
    x |= (u64)l0 << h0 | (u64)l1 << h1;
    if (h2 >= 0) x |= (u64)l2 << h2;
    lab = (u32)(f0 | l0 << 4) | (u32)(f1 | l1 << 4) << 8 | (h2 >= 0 ? ((u32)(f2 | l2 << 4) | 0x80u) << 16 : 0u);
    return x;
  }
  // the permutations that rename the fields as canon_code's labels say
  RMC_HD static u32 cand_of(u32 lab) {
    const u32* pos = kPermTables[N].pos;
    u32 m = pos[(lab & 15u) * 4 + ((lab >> 4) & 15u)] & pos[((lab >> 8) & 15u) * 4 + ((lab >> 12) & 15u)];
    if ((lab >> 23) & 1u) m &= pos[((lab >> 16) & 15u) * 4 + ((lab >> 20) & 7u)];
    return m;
  }
  // the permutation TLC picks: least permuted variable tuple, variable by variable
  RMC_HD static u32 tlc_min_perm(const Work& t, const BagRef& bag, int len, bool ce, u32 cfgt, unsigned long long* prof = nullptr) {
    unsigned long long pt = RMC_PROF_T();
    u32 cand = (u32)lomask(NPERM);
    RMC_FPS(0, 1); RMC_FPS(1, len);
    // messages: a function from message records to counts (oracle Fcn order: DOMAIN size — equal
    // for all — then the domain elements ascending, then the counts in domain order)
    u64 last = 0;
    bool have_last = false;
    int j0 = 0;
#ifndef RMC_TLC_NO_CANON
    if (len > 0) {
      // the first (least) permuted message in closed form: the least canonical code over the
      // messages, and the permutations that give some message of that code its canonical labels
      // (instead of the least permuted code under each of the N! permutations).  A message that
      // carries a ConfigEntry (only when ce) renames config values too: its least code and the
      // permutations reaching it are found by trying the N! permutations on it alone.
      u64 best = ~0ull;
      u32 cm = 0;   // one pass: the least code so far and the permutations reaching it
#pragma unroll 1
      for (int q = 0; q < len; ++q) {
        const u64 c = mcode(bag[q]);
        if (ce && (RMC_TLC_CFG_MASK ? bag.cfg(q) : msg_has_config(c, cfgt))) {
          RMC_FPS(25, 1);
#pragma unroll 1
          for (int p = 0; p < NPERM; ++p) {
            const u64 v = perm_code(c, perm_of(p), true, cfgt);
            cm = v < best ? 1u << p : v == best ? cm | 1u << p : cm;
            best = v < best ? v : best;
          }
        } else {
          u32 lab;
          const u64 cc = canon_code(c, lab);
          if (cc <= best) { const u32 m = cand_of(lab); cm = cc < best ? m : cm | m; best = cc; }
        }
      }
      cand = cm; last = best; have_last = true; j0 = 1;
    }
#endif
    RMC_FPS(2, __builtin_popcount(cand));
    // Automorphic candidates (symmetric states: servers in the same role): when every remaining
    // permutation maps the bag to the same function -- its permuted codes with their counts,
    // compared by a sum of 64-bit mixes (the fingerprint's own collision class) -- the domain and
    // count stages below tie for all of them: skipped (their cost is |cand| * len^2 code renamings)
    RMC_PROF_ADD(prof, 2, pt);
    // the bag under permutation pi as one 64-bit value: its permuted codes with their counts, a sum
    // of mixes (a function from codes to counts; equal values <=> equal permuted bags, up to the
    // fingerprint's own collision class)
    auto bag_hash = [&](u32 pi) -> u64 {
      u64 h = 0;
#pragma unroll 1
      for (int q = 0; q < len; ++q) { const u64 e = bag[q]; h += fmix(((perm_code(mcode(e), pi, ce && bag.cfg(q), cfgt) + 1ull) * P1) ^ (u64)mcount(e)); }
      return h;
    };
    // The next messages in domain order, a few at most: each usually halves the candidates (3:
    // memb_fingerprint 531 vs 546 ms per C3 run at 2, round 5; more saves nothing on the host counts)
#ifndef RMC_TLC_NARROW
#define RMC_TLC_NARROW 3
#endif
    int j = j0;
#ifndef RMC_TLC_ONEPASS
#define RMC_TLC_ONEPASS 1
#endif
#if RMC_TLC_ONEPASS
    // One pass per candidate instead of one per domain position: each candidate's next three permuted
    // codes (the 2nd..4th smallest, its permuted domain being a set: no repeats) in a sorted triple,
    // and the least triple kept.  Comparing the triples lexicographically keeps exactly what keeping
    // the least 2nd code, then the least 3rd, then the least 4th does; a lane pays one scan of the bag
    // per candidate, not one per position its wave's busiest lane needs (host counts: the narrowing
    // is 2.4x more work per wave than per lane).
    // The same pass hashes each candidate's permuted bag (bag_hash's sum of mixes): when every kept
    // candidate maps the bag to the same function, the bag stages below tie for all of them and are
    // skipped without the grouping pass (host counts: 92% of the states that reach the grouping).
    static_assert(RMC_TLC_NARROW == 3, "the one-pass narrowing keeps three codes");
    bool one_group = false;
    if (j0 == 1 && len > 1 && !single(cand)) {
      u64 b0 = ~0ull, b1 = ~0ull, b2 = ~0ull, hb = 0;
      u32 out = 0;
#pragma unroll 1
      for (u32 m = cand; m; m &= m - 1u) {
        const int p = __builtin_ctz(m);
        const u32 pi = perm_of(p);
        u64 k0 = ~0ull, k1 = ~0ull, k2 = ~0ull, h = 0;
RMC_QLOOP
        for (int q = 0; q < len; ++q) {
          const u64 e = bag[q];
          const u64 c = perm_code(mcode(e), pi, ce && bag.cfg(q), cfgt);
          h += fmix(((c + 1ull) * P1) ^ (u64)mcount(e));
          const bool ok = c > last, l0 = ok && c < k0, l1 = ok && c < k1, l2 = ok && c < k2;
          const u64 n2 = l1 ? k1 : l2 ? c : k2, n1 = l0 ? k0 : l1 ? c : k1;
          k0 = l0 ? c : k0; k1 = n1; k2 = n2;
        }
        const bool lt = k0 != b0 ? k0 < b0 : k1 != b1 ? k1 < b1 : k2 < b2;
        const bool eq = k0 == b0 && k1 == b1 && k2 == b2;
        one_group = lt ? true : eq ? (one_group && h == hb) : one_group;
        hb = lt ? h : hb;
        out = lt ? 1u << p : eq ? (out | 1u << p) : out;
        b0 = lt ? k0 : b0; b1 = lt ? k1 : b1; b2 = lt ? k2 : b2;
      }
      cand = out;
      const int nk = len - 1 < RMC_TLC_NARROW ? len - 1 : RMC_TLC_NARROW;
      j = 1 + nk;
      last = nk == 1 ? b0 : nk == 2 ? b1 : b2;
    }
    // (after it the loop below has nothing left: j reached len or j0 + RMC_TLC_NARROW)
#endif
#pragma unroll 1
    for (; (j == 0 || (j < len && !single(cand))) && j < j0 + RMC_TLC_NARROW; ++j) {   // (one pass even for an empty bag)
      u64 next = 0;
      RMC_FPS(15, 1); RMC_FPS(16, __builtin_popcount(cand));
      cand = keep_min(cand, [&](int, u32 pi) { return next_perm_code(bag, len, pi, ce, cfgt, have_last, last); }, &next);
      last = next;
      have_last = true;
    }
    RMC_FPS(3, __builtin_popcount(cand)); RMC_FPS(22, single(cand));
    RMC_PROF_ADD(prof, 3, pt);
    // Candidates that map the bag to the same function tie through the rest of the domain and all
    // the counts: a symmetric state (servers in the same role) keeps such groups to the last
    // message.  The stages below run on one representative per group and stop once one group is
    // left; its members all go on to the history.
    const u32 group_of_all = cand;
    bool grouped = false, bag_done = false;
#if RMC_TLC_ONEPASS
    if (one_group && !single(cand)) bag_done = true;   // (the narrowing's hashes: one group)
#endif
    // one message: every candidate gives it the least code the first stage found, with its one count
    if (len == 1 && !single(cand)) bag_done = true;
    // (also when the narrowing already compared the whole domain: the counts loop below would
    // otherwise run over every message for candidates that map the bag to the same function)
#ifndef RMC_TLC_GROUP_ALL
#define RMC_TLC_GROUP_ALL 1
#endif
    if (!bag_done && !single(cand) && (RMC_TLC_GROUP_ALL ? len > 0 : j < len)) {
      RMC_FPS(4, 1); RMC_FPS(14, len); RMC_FPS(20, __builtin_popcount(cand));
      u32 reps = 0, first_grp = 0;
#pragma unroll 1
      for (u32 left = cand; left;) {
        const int p = __builtin_ctz(left);
        const u64 h = bag_hash(perm_of(p));
        RMC_FPS(5, 1 + __builtin_popcount(left & (left - 1u)));
        u32 grp = 1u << p;
#pragma unroll 1
        for (u32 m = left & (left - 1u); m; m &= m - 1u) {
          const int q = __builtin_ctz(m);
          if (bag_hash(perm_of(q)) == h) grp |= 1u << q;
        }
        if (!reps) first_grp = grp;
        reps |= 1u << p;
        left &= ~grp;
      }
      if (single(reps)) { cand = first_grp; bag_done = true; RMC_FPS(6, 1); }   // one group: the bag stages tie for all of it
      else { cand = reps; grouped = true; RMC_FPS(7, 1); RMC_FPS(21, __builtin_popcount(reps)); }
    }
#pragma unroll 1
    for (; !bag_done && j < len && !single(cand); ++j) {
      RMC_FPS(8, 1); RMC_FPS(9, __builtin_popcount(cand));
      u64 next = 0;
      cand = keep_min(cand, [&](int, u32 pi) { return next_perm_code(bag, len, pi, ce, cfgt, have_last, last); }, &next);
      last = next;
      have_last = true;
    }
    have_last = false;
    RMC_FPS(23, !bag_done && !grouped && len > 0 && !single(cand));
#pragma unroll 1
    for (int jc = 0; !bag_done && jc < len && !single(cand); ++jc) {
      RMC_FPS(24, !grouped);   // same permuted domain: the counts in domain order
      const u64 code = next_perm_code(bag, len, perm_of(__builtin_ctz(cand)), ce, cfgt, have_last, last);
      RMC_FPS(10, 1); RMC_FPS(11, __builtin_popcount(cand));
      cand = keep_min(cand, [&](int, u32 pi) {
        u64 cnt = 0;
#pragma unroll 1
        for (int q = 0; q < len; ++q) {
          const u64 e = bag[q];
          if (perm_code(mcode(e), pi, ce && bag.cfg(q), cfgt) == code) cnt = (u64)mcount(e);
        }
        return cnt;
      });
      last = code; have_last = true;
    }
    if (grouped) {
      // the winning representative's whole group (members of other groups lost on the bag)
      const u64 h = bag_hash(perm_of(__builtin_ctz(cand)));
      u32 grp = cand;
      RMC_FPS(12, 1 + __builtin_popcount(group_of_all & ~cand));
#pragma unroll 1
      for (u32 m = group_of_all & ~cand; m; m &= m - 1u) {
        const int q = __builtin_ctz(m);
        if (bag_hash(perm_of(q)) == h) grp |= 1u << q;
      }
      cand = grp;
    }
    RMC_PROF_ADD(prof, 4, pt);
    // history: [global, hadNum* (invariant), server], currentTerm, state, votedFor, log, commitIndex,
    // votesResponded, votesGranted, nextIndex, matchIndex — each a function over the servers, in
    // the fused runs of key_scalars / key_log / key_cv / key_nm
    RMC_FPS(17, !single(cand)); RMC_FPS(18, single(cand) ? 0 : __builtin_popcount(cand));
    if (!single(cand)) cand = keep_min(cand, [&](int p, u32 pi) { return key_scalars(t, p, pi); });
#pragma unroll 1
    for (int x = 0; x < N && !single(cand); ++x)
      cand = keep_min(cand, [&](int, u32 pi) { return key_log(t, x, pi, cfgt); });
    if (!single(cand)) cand = keep_min(cand, [&](int, u32 pi) { return key_cv(t, pi); });
#pragma unroll 1
    for (int m = 0; m < 2 && !single(cand); ++m)
      cand = keep_min(cand, [&](int, u32 pi) { return key_nm(t, pi, m != 0); });
    RMC_PROF_ADD(prof, 5, pt);
    return perm_of(__builtin_ctz(cand));   // any remaining tie: identical permuted states
  }
  RMC_HD static u64 fingerprint_tlc(const Work& t, u64 seed, const MembRuntime& rt, unsigned long long* prof = nullptr) {
    unsigned long long pt = RMC_PROF_T();
    const bool ce = has_config_entries(t, rt.cfg_type);
#if defined(__HIP_DEVICE_COMPILE__)
    __shared__ u64 sbag[MK * 256];   // every kernel runs 256-lane workgroups; one slice per lane
    u64* const base = sbag + (threadIdx.x & 255u);
    constexpr int stride = 256;
#else
    u64 hbag[MK];
    u64* const base = hbag;
    constexpr int stride = 1;
#endif
    int len = 0;
    u32 cfgm = 0;
#pragma unroll
    for (int q = 0; q < MK; ++q) {
      base[q * stride] = t.bag.v[q];
      len += t.bag.v[q] != EMPTY;
      if (ce && t.bag.v[q] != EMPTY && (!RMC_TLC_CFG_MASK || msg_has_config(mcode(t.bag.v[q]), rt.cfg_type))) cfgm |= 1u << q;
    }
    RMC_PROF_ADD(prof, 1, pt);
    const BagRef bref{base, stride, cfgm};
    const u32 pi = tlc_min_perm(t, bref, len, ce, rt.cfg_type, prof);
    pt = RMC_PROF_T();
    const u64 best = ce ? view_hash1_bag<true>(t, bref, len, pi, seed, rt.cfg_type) : view_hash1_bag<false>(t, bref, len, pi, seed, rt.cfg_type);
    RMC_PROF_ADD(prof, 6, pt);
#if defined(__HIP_DEVICE_COMPILE__) && defined(RMC_FP_DUP_MINPERM)   // timing experiment: the search twice
    { int l2 = len; asm volatile("" : "+v"(l2)); const u32 p2 = tlc_min_perm(t, BagRef{base, stride, cfgm}, l2, ce, rt.cfg_type); asm volatile("" :: "v"(p2)); }
#endif
#if defined(__HIP_DEVICE_COMPILE__) && defined(RMC_FP_DUP_VIEW)      // timing experiment: the view hash twice
    { u32 p2 = pi; asm volatile("" : "+v"(p2)); const u64 b2 = ce ? view_hash1<true>(t, p2, seed, rt.cfg_type) : view_hash1<false>(t, p2, seed, rt.cfg_type); asm volatile("" :: "v"((u32)b2), "v"((u32)(b2 >> 32))); }
#endif
    const u64 fp = fmix(best ^ seed);
    return fp ? fp : 1ull;
  }

  // fingerprint_tlc of t whose bag is the len sorted entries p[q * stride] (memb_fingerprint_lds)
  RMC_HD static u64 fingerprint_tlc_slice(const Work& t, u64* p, int stride, int len, u64 seed, const MembRuntime& rt) {
    u32 cfgm = 0;
#pragma unroll 1
    for (int q = 0; q < len; ++q) if (msg_has_config(mcode(p[q * stride]), rt.cfg_type)) cfgm |= 1u << q;
    const bool ce = cfgm != 0 || logs_have_config(t, rt.cfg_type);
    const BagRef bref{p, stride, cfgm};
    const u32 pi = tlc_min_perm(t, bref, len, ce, rt.cfg_type);
    const u64 best = ce ? view_hash1_bag<true>(t, bref, len, pi, seed, rt.cfg_type) : view_hash1_bag<false>(t, bref, len, pi, seed, rt.cfg_type);
    const u64 fp = fmix(best ^ seed);
    return fp ? fp : 1ull;
  }
  // unpack without the bag (its words: NW - 2 * MK onwards)
  template <int M>
  RMC_HD static void unpack_nobag(const u32 (&w)[M], Work& t) {
    t.term = w[0]; t.st = w[1]; t.voted = w[2]; t.commit = w[3]; t.vr = w[4]; t.vg = w[5];
    t.nexti = (u64)w[6] | (u64)w[7] << 32; t.matchi = (u64)w[8] | (u64)w[9] << 32;
#pragma unroll
    for (int i = 0; i < N; ++i) { const LogV l = log_load((u64)w[10 + 2 * i] | (u64)w[11 + 2 * i] << 32); t.la.v[i] = l.a; t.lb.v[i] = l.b; }
    t.h0 = (u64)w[10 + 2 * N] | (u64)w[11 + 2 * N] << 32; t.h1 = (u64)w[12 + 2 * N] | (u64)w[13 + 2 * N] << 32;
    t.hr0 = (u64)w[14 + 2 * N] | (u64)w[15 + 2 * N] << 32; t.hr1 = (u64)w[16 + 2 * N] | (u64)w[17 + 2 * N] << 32;
  }
  static constexpr int BAGW = 18 + 2 * N;   // first packed word of the bag
  // pack without the bag (words [0, BAGW))
  RMC_HD static void pack_nobag(const Work& t, u32 (&w)[BAGW]) {
    w[0] = t.term; w[1] = t.st; w[2] = t.voted; w[3] = t.commit; w[4] = t.vr; w[5] = t.vg;
    w[6] = (u32)t.nexti; w[7] = (u32)(t.nexti >> 32); w[8] = (u32)t.matchi; w[9] = (u32)(t.matchi >> 32);
#pragma unroll
    for (int i = 0; i < N; ++i) { const u64 x = log_store(LogV{t.la.v[i], t.lb.v[i]}); w[10 + 2 * i] = (u32)x; w[11 + 2 * i] = (u32)(x >> 32); }
    w[10 + 2 * N] = (u32)t.h0; w[11 + 2 * N] = (u32)(t.h0 >> 32); w[12 + 2 * N] = (u32)t.h1; w[13 + 2 * N] = (u32)(t.h1 >> 32);
    w[14 + 2 * N] = (u32)t.hr0; w[15 + 2 * N] = (u32)(t.hr0 >> 32); w[16 + 2 * N] = (u32)t.hr1; w[17 + 2 * N] = (u32)(t.hr1 >> 32);
  }
  // the successor's packed bag from the parent's (MK sorted entries, 0 = empty, last) and apply's change
  // d: with_msg then without_msg as one merge pass, entry by entry (the bag never held in registers).
  // err: with_msg's count overflow and an (MK+1)-th message (that entry is dropped: expand reports it too)
  RMC_HD static void bag_merge(const u64* in, u64* out, const Delta& d, u32& err) {
    const u64 xa = (d.add << CNTB) | 1ull;
    bool pend = d.a;   // the new message not yet placed (or counted into its existing entry)
    int o = 0;
    auto emit = [&](u64 x) { if (o < MK) out[o] = x; else err |= ME_CAP; ++o; };
#pragma unroll 1
    for (int q = 0; q < MK; ++q) {
      u64 x = in[q];
      if (!x) break;
      const u64 code = mcode(x);
      if (pend && d.add < code) { if (!(d.r && d.rem == d.add)) emit(xa); pend = false; }
      if (pend && code == d.add) { if (mcount(x) + 1 > (int)lomask(CNTB)) err |= ME_CAP; x += 1; pend = false; }
      if (d.r && code == d.rem) { if (mcount(x) <= 1) continue; x -= 1; }
      emit(x);
    }
    if (pend && !(d.r && d.rem == d.add)) emit(xa);
#pragma unroll 1
    for (; o < MK; ++o) out[o] = 0ull;
  }

  // ------------------------------------------------------------ pack / unpack (word aligned)
  RMC_HD static u64 log_store(LogV l) { return (l.a & lomask(MAXLOG * EW)) | ((u64)llen(l) << 60); }
  RMC_HD static LogV log_load(u64 w) { return LogV{w & lomask(MAXLOG * EW), (u32)(w >> 60) << 16}; }
  RMC_HD static void pack(const Work& t, u32 (&w)[NW]) {
    w[0] = t.term; w[1] = t.st; w[2] = t.voted; w[3] = t.commit; w[4] = t.vr; w[5] = t.vg;
    w[6] = (u32)t.nexti; w[7] = (u32)(t.nexti >> 32); w[8] = (u32)t.matchi; w[9] = (u32)(t.matchi >> 32);
#pragma unroll
    for (int i = 0; i < N; ++i) { const u64 x = log_store(LogV{t.la.v[i], t.lb.v[i]}); w[10 + 2 * i] = (u32)x; w[11 + 2 * i] = (u32)(x >> 32); }
    w[10 + 2 * N] = (u32)t.h0; w[11 + 2 * N] = (u32)(t.h0 >> 32); w[12 + 2 * N] = (u32)t.h1; w[13 + 2 * N] = (u32)(t.h1 >> 32);
    w[14 + 2 * N] = (u32)t.hr0; w[15 + 2 * N] = (u32)(t.hr0 >> 32); w[16 + 2 * N] = (u32)t.hr1; w[17 + 2 * N] = (u32)(t.hr1 >> 32);
#pragma unroll
    for (int q = 0; q < MK; ++q) {
      const u64 x = t.bag.v[q] == EMPTY ? 0ull : t.bag.v[q];
      w[18 + 2 * N + 2 * q] = (u32)x; w[19 + 2 * N + 2 * q] = (u32)(x >> 32);
    }
  }
  template <int M>
  RMC_HD static void unpack(const u32 (&w)[M], Work& t) {
    static_assert(M >= NW, "packed array too small");
    t.term = w[0]; t.st = w[1]; t.voted = w[2]; t.commit = w[3]; t.vr = w[4]; t.vg = w[5];
    t.nexti = (u64)w[6] | (u64)w[7] << 32; t.matchi = (u64)w[8] | (u64)w[9] << 32;
#pragma unroll
    for (int i = 0; i < N; ++i) { const LogV l = log_load((u64)w[10 + 2 * i] | (u64)w[11 + 2 * i] << 32); t.la.v[i] = l.a; t.lb.v[i] = l.b; }
    t.h0 = (u64)w[10 + 2 * N] | (u64)w[11 + 2 * N] << 32; t.h1 = (u64)w[12 + 2 * N] | (u64)w[13 + 2 * N] << 32;
    t.hr0 = (u64)w[14 + 2 * N] | (u64)w[15 + 2 * N] << 32; t.hr1 = (u64)w[16 + 2 * N] | (u64)w[17 + 2 * N] << 32;
#pragma unroll
    for (int q = 0; q < MK; ++q) {
      const u64 x = (u64)w[18 + 2 * N + 2 * q] | (u64)w[19 + 2 * N + 2 * q] << 32;
      t.bag.v[q] = x ? x : EMPTY;
    }
    t.bag.v[MK] = EMPTY;
  }
};

}  // namespace rmc
