// ============================================================================
// TEST INFRASTRUCTURE ONLY (see oracle/tla.h header).
//
// Literal CPU restatement of tlc_membership/raft.tla (Ongaro + Ricketts +
// Amos/Zhang membership + Pîrlea/Foo history) over the value model of tla.h.
// Active message aliases are the *Direct ones (raft.tla:323-328, 883).
// Every function cites the lines it follows; gotchas G2, G4-G12 of SURVEY.md
// §8 are reproduced verbatim.
// ============================================================================
#pragma once
#include "engine.h"

namespace oracle {

struct RaftMembership : Spec {
  // VARIABLE declaration order, raft.tla:114-185
  enum { messages, history, currentTerm, state, votedFor, log, commitIndex,
         votesResponded, votesGranted, nextIndex, matchIndex, NVARS };
  enum { A_RequestVote, A_BecomeLeader, A_ClientRequest, A_AdvanceCommitIndex, A_AppendEntries,
         A_UpdateTerm, A_HandleRequestVoteRequest, A_DropStaleResponse, A_HandleRequestVoteResponse,
         A_HandleAppendEntriesRequest, A_HandleAppendEntriesResponse, A_HandleCatchupRequest,
         A_HandleCatchupResponse, A_HandleCheckOldConfig, A_Timeout, A_Restart,
         A_DuplicateMessage, A_DropMessage, A_AddNewServer, A_DeleteServer, NACT };

  const Cfg& cfg;
  V InitServer, Server, NumRounds, Nil, Value, ValueEntry, ConfigEntry, Follower, Candidate, Leader;
  V RVReq, RVResp, AEReq, AEResp, CReq, CResp, COC;
  std::vector<std::string> vn;
  bool use_async = true, use_crash = false, use_unreliable = false, use_dynamic = false;
  bool disjunct_copies = true;   // engine.h Options::disjunct_copies, [ext] switch (vi)
  std::vector<V> golden_cwcl, golden_morc;   // punctuated-search prefixes (raft.tla:1201, :1231)

  // Constraint bounds (raft.tla:23-30)
  static constexpr int64_t MaxLogLength = 5, MaxRestarts = 2, MaxTimeouts = 3, MaxClientRequests = 3,
                           MaxTerms = MaxTimeouts + 1, MaxMembershipChanges = 3,
                           MaxTriedMembershipChanges = MaxMembershipChanges + 1;
  int64_t MaxInFlightMessages() const { int64_t c = card(Server); return 2 * c * c; }

  explicit RaftMembership(const Cfg& c) : cfg(c) {
    InitServer = c.get("InitServer"); Server = c.get("Server"); NumRounds = c.get("NumRounds");
    Nil = c.get("Nil"); Value = c.get("Value"); ValueEntry = c.get("ValueEntry"); ConfigEntry = c.get("ConfigEntry");
    Follower = c.get("Follower"); Candidate = c.get("Candidate"); Leader = c.get("Leader");
    RVReq = c.get("RequestVoteRequest"); RVResp = c.get("RequestVoteResponse");
    AEReq = c.get("AppendEntriesRequest"); AEResp = c.get("AppendEntriesResponse");
    CReq = c.get("CatchupRequest"); CResp = c.get("CatchupResponse"); COC = c.get("CheckOldConfig");
    vn = {"messages", "history", "currentTerm", "state", "votedFor", "log", "commitIndex",
          "votesResponded", "votesGranted", "nextIndex", "matchIndex"};
    const std::string& n = c.next;                         // raft.tla:909-943
    if (n == "NextAsync") { use_async = true; }
    else if (n == "NextCrash") { use_async = false; use_crash = true; }
    else if (n == "NextAsyncCrash") { use_crash = true; }
    else if (n == "NextUnreliable") { use_async = false; use_unreliable = true; }
    else if (n == "Next") { use_crash = true; use_unreliable = true; }
    else if (n == "NextDynamic") { use_crash = true; use_unreliable = true; use_dynamic = true; }
    else throw EvalError("unknown NEXT " + n);
  }
  const std::vector<std::string>& var_names() const override { return vn; }
  std::vector<std::string> action_names() const override {
    return {"RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex", "AppendEntries",
            "UpdateTerm", "HandleRequestVoteRequest", "DropStaleResponse", "HandleRequestVoteResponse",
            "HandleAppendEntriesRequest", "HandleAppendEntriesResponse", "HandleCatchupRequest",
            "HandleCatchupResponse", "HandleCheckOldConfig", "Timeout", "Restart",
            "DuplicateMessage", "DropMessage", "AddNewServer", "DeleteServer"};
  }

  // ------------------------------------------------------------ helpers
  V fnOver(const V& dom, const V& val) const { std::vector<V> vs(dom->a.size(), val); return fcn(dom->a, vs); }
  // Quorum(config) membership: S \in {i \in SUBSET(config) : Cardinality(i) * 2 > Cardinality(config)} (:217)
  bool InQuorum(const V& S, const V& config) const { return subseteq(S, config) && card(S) * 2 > card(config); }
  int64_t LastTerm(const V& xlog) const { return len(xlog) == 0 ? 0 : as_int(ap(ap(xlog, len(xlog)), "term")); }   // :221
  // TypedBags (+)/(-) with SetToBag({m}) (:226-231, TypedBags.tla:51-69)   — G2
  V WithMessage(const V& m, const V& msgs) const {
    if (in_domain(msgs, m)) return except(msgs, m, Int(as_int(ap(msgs, m)) + 1));
    return at_at(msgs, colon_gt(m, Int(1)));
  }
  V WithoutMessage(const V& m, const V& msgs) const {
    if (!in_domain(msgs, m)) return msgs;
    int64_t c = as_int(ap(msgs, m)) - 1;
    if (c > 0) return except(msgs, m, Int(c));
    std::vector<V> ks, vs;
    for (size_t q = 0; q < msgs->a.size(); ++q) if (!eq(msgs->a[q], m)) { ks.push_back(msgs->a[q]); vs.push_back(msgs->b[q]); }
    return fcn(ks, vs);
  }
  V H(const State& s, const char* f) const { return ap(s[history], f); }
  V HGlobalAppend(const V& h, std::initializer_list<V> acts) const {
    V g = ap(h, "global"); for (auto& a : acts) g = append(g, a); return except(h, "global", g);
  }
  V HBump(const V& h, const char* f) const { return except(h, f, Int(as_int(ap(h, f)) + 1)); }
  // SendDirect (:247-263)   — G4
  void SendDirect(State& t, const State& s, const V& m) const {
    V msgA = rec({{"action", Str("Send")}, {"executedOn", ap(m, "msource")}, {"msg", m}});
    t[messages] = WithMessage(m, s[messages]);
    V ty = ap(m, "mtype");
    if (eq(ty, CReq)) {
      V ma = rec({{"action", Str("TryAddServer")}, {"executedOn", ap(m, "msource")}, {"added", ap(m, "mdest")}});
      t[history] = HGlobalAppend(HBump(s[history], "hadNumTriedMembershipChanges"), {ma, msgA});
    } else if (eq(ty, COC)) {
      V ma = rec({{"action", Str("TryRemoveServer")}, {"executedOn", ap(m, "msource")}, {"removed", ap(m, "mserver")}});
      t[history] = HGlobalAppend(HBump(s[history], "hadNumTriedMembershipChanges"), {ma, msgA});
    } else {
      t[history] = HGlobalAppend(s[history], {msgA});
    }
  }
  // DiscardDirect (:280-283)
  void DiscardDirect(State& t, const State& s, const V& m) const {
    V a = rec({{"action", Str("Receive")}, {"executedOn", ap(m, "mdest")}, {"msg", m}});
    t[messages] = WithoutMessage(m, s[messages]);
    t[history] = HGlobalAppend(s[history], {a});
  }
  // DiscardDirectWithMembershipChange (:285-290)
  void DiscardWithMC(State& t, const State& s, const V& m, const V& extra) const {
    V a = rec({{"action", Str("Receive")}, {"executedOn", ap(m, "mdest")}, {"msg", m}});
    t[messages] = WithoutMessage(m, s[messages]);
    t[history] = HGlobalAppend(HBump(s[history], "hadNumMembershipChanges"), {a, extra});
  }
  // ReplyDirect (:308-314)
  void ReplyDirect(State& t, const State& s, const V& resp, const V& req) const {
    V recvA = rec({{"action", Str("Receive")}, {"executedOn", ap(req, "mdest")}, {"msg", req}});
    V respA = rec({{"action", Str("Send")}, {"executedOn", ap(resp, "msource")}, {"msg", resp}});
    t[messages] = WithoutMessage(req, WithMessage(resp, s[messages]));
    t[history] = HGlobalAppend(s[history], {recvA, respA});
  }
  // GetHistoricalMaxConfigIndex / GetHistoricalConfig over a log (:346-360)  — G12
  int64_t MaxConfigIndex(const V& lg) const {
    int64_t mx = 0;
    for (int64_t q = 1; q <= len(lg); ++q) if (eq(ap(ap(lg, q), "type"), ConfigEntry)) mx = q;
    return mx;
  }
  V ConfigOfLog(const V& lg) const { int64_t q = MaxConfigIndex(lg); return q == 0 ? InitServer : ap(ap(lg, q), "value"); }
  V GetConfig(const State& s, const V& i) const { return ConfigOfLog(ap(s[log], i)); }
  int64_t GetMaxConfigIndex(const State& s, const V& i) const { return MaxConfigIndex(ap(s[log], i)); }
  V CurrentLeaders(const State& s) const {                                   // :362
    std::vector<V> xs; for (auto& i : Server->a) if (eq(ap(s[state], i), Leader)) xs.push_back(i); return set(xs);
  }
  V Committed(const State& s, const V& i) const { return subseq(ap(s[log], i), 1, as_int(ap(s[commitIndex], i))); }   // :969

  // ------------------------------------------------------------ Init (:367-393)
  std::vector<State> init() const override {
    State s(NVARS);
    s[messages] = fcn({}, {});                                          // EmptyBag
    s[history] = rec({{"server", fnOver(Server, rec({{"restarted", Int(0)}, {"timeout", Int(0)}}))},
                      {"global", empty_seq()}, {"hadNumLeaders", Int(0)}, {"hadNumClientRequests", Int(0)},
                      {"hadNumTriedMembershipChanges", Int(0)}, {"hadNumMembershipChanges", Int(0)}});
    s[currentTerm] = fnOver(Server, Int(1));
    s[state] = fnOver(Server, Follower);
    s[votedFor] = fnOver(Server, Nil);
    s[votesResponded] = fnOver(Server, empty_set());
    s[votesGranted] = fnOver(Server, empty_set());
    s[nextIndex] = fnOver(Server, fnOver(Server, Int(1)));
    s[matchIndex] = fnOver(Server, fnOver(Server, Int(0)));
    s[log] = fnOver(Server, empty_seq());
    s[commitIndex] = fnOver(Server, Int(0));
    return {s};
  }

  // ------------------------------------------------------------ actions
  void Restart(const State& s, const V& i, std::vector<Succ>& out) const {                          // :401-411
    State t = s;
    t[state] = except(s[state], i, Follower);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    t[commitIndex] = except(s[commitIndex], i, Int(0));
    V h = s[history], srv = ap(h, "server"), si = ap(srv, i);
    h = except(h, "server", except(srv, i, except(si, "restarted", Int(as_int(ap(si, "restarted")) + 1))));
    t[history] = HGlobalAppend(h, {rec({{"action", Str("Restart")}, {"executedOn", i}})});
    out.push_back({t, A_Restart});
  }
  void Timeout(const State& s, const V& i, std::vector<Succ>& out) const {                          // :415-427
    V st = ap(s[state], i);
    if (!(eq(st, Follower) || eq(st, Candidate))) return;
    if (!in_set(i, GetConfig(s, i))) return;
    State t = s;
    t[state] = except(s[state], i, Candidate);
    t[currentTerm] = except(s[currentTerm], i, Int(as_int(ap(s[currentTerm], i)) + 1));
    t[votedFor] = except(s[votedFor], i, Nil);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    V h = s[history], srv = ap(h, "server"), si = ap(srv, i);
    h = except(h, "server", except(srv, i, except(si, "timeout", Int(as_int(ap(si, "timeout")) + 1))));
    t[history] = HGlobalAppend(h, {rec({{"action", Str("Timeout")}, {"executedOn", i}})});
    out.push_back({t, A_Timeout});
  }
  void RequestVote(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {          // :431-440
    if (!eq(ap(s[state], i), Candidate)) return;
    if (!in_set(j, setminus(GetConfig(s, i), ap(s[votesResponded], i)))) return;
    V li = ap(s[log], i);
    V m = rec({{"mtype", RVReq}, {"mterm", ap(s[currentTerm], i)}, {"mlastLogTerm", Int(LastTerm(li))},
               {"mlastLogIndex", Int(len(li))}, {"msource", i}, {"mdest", j}});
    State t = s; SendDirect(t, s, m);
    out.push_back({t, A_RequestVote});
  }
  void AppendEntries(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {        // :446-468
    if (eq(i, j)) return;
    if (!eq(ap(s[state], i), Leader)) return;
    if (!in_set(j, GetConfig(s, i))) return;
    V li = ap(s[log], i);
    int64_t ni = as_int(ap(ap(s[nextIndex], i), j));
    int64_t prevLogIndex = ni - 1;
    int64_t prevLogTerm = (prevLogIndex > 0 && prevLogIndex <= len(li)) ? as_int(ap(ap(li, prevLogIndex), "term")) : 0;
    int64_t lastEntry = std::min(len(li), ni);
    V entries = subseq(li, ni, lastEntry);
    V m = rec({{"mtype", AEReq}, {"mterm", ap(s[currentTerm], i)}, {"mprevLogIndex", Int(prevLogIndex)},
               {"mprevLogTerm", Int(prevLogTerm)}, {"mentries", entries},
               {"mcommitIndex", Int(std::min(as_int(ap(s[commitIndex], i)), lastEntry))}, {"msource", i}, {"mdest", j}});
    State t = s; SendDirect(t, s, m);
    out.push_back({t, A_AppendEntries});
  }
  void BecomeLeader(const State& s, const V& i, std::vector<Succ>& out) const {                     // :472-484
    if (!eq(ap(s[state], i), Candidate)) return;
    if (!InQuorum(ap(s[votesGranted], i), GetConfig(s, i))) return;
    State t = s;
    t[state] = except(s[state], i, Leader);
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(len(ap(s[log], i)) + 1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    V a = rec({{"action", Str("BecomeLeader")}, {"executedOn", i}, {"leaders", cup(CurrentLeaders(s), set({i}))}});
    t[history] = HGlobalAppend(HBump(s[history], "hadNumLeaders"), {a});
    out.push_back({t, A_BecomeLeader});
  }
  void ClientRequest(const State& s, const V& i, const V& v, std::vector<Succ>& out) const {        // :488-497
    if (!eq(ap(s[state], i), Leader)) return;
    V entry = rec({{"term", ap(s[currentTerm], i)}, {"type", ValueEntry}, {"value", v}});
    State t = s;
    t[log] = except(s[log], i, append(ap(s[log], i), entry));
    t[history] = HBump(s[history], "hadNumClientRequests");
    out.push_back({t, A_ClientRequest});
  }
  void AdvanceCommitIndex(const State& s, const V& i, std::vector<Succ>& out) const {               // :504-539
    if (!eq(ap(s[state], i), Leader)) return;
    V cfgI = GetConfig(s, i), li = ap(s[log], i);
    std::vector<V> agree;
    for (int64_t index = 1; index <= len(li); ++index) {
      std::vector<V> ag = {i};
      for (auto& k : cfgI->a) if (as_int(ap(ap(s[matchIndex], i), k)) >= index) ag.push_back(k);
      if (InQuorum(set(ag), cfgI)) agree.push_back(Int(index));
    }
    V agreeIndexes = set(agree);
    int64_t ci = as_int(ap(s[commitIndex], i)), nci = ci;
    if (card(agreeIndexes) > 0 && eq(ap(ap(li, set_max(agreeIndexes)), "term"), ap(s[currentTerm], i)))
      nci = set_max(agreeIndexes);
    bool committed = nci > ci;
    bool cmc = committed && eq(ap(ap(li, nci), "type"), ConfigEntry) &&
               !eq(ap(ap(li, nci), "value"), ConfigOfLog(subseq(li, 1, nci - 1)));
    State t = s;
    t[commitIndex] = except(s[commitIndex], i, Int(nci));
    if (cmc)                                                                                         // G11
      t[history] = HGlobalAppend(s[history], {rec({{"action", Str("CommitMembershipChange")}, {"executedOn", i},
                                                   {"config", ap(ap(li, nci), "value")}})});
    else if (committed)
      t[history] = HGlobalAppend(s[history], {rec({{"action", Str("CommitEntry")}, {"executedOn", i}, {"entry", ap(li, nci)}})});
    out.push_back({t, A_AdvanceCommitIndex});
  }
  void AddNewServer(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {         // :542-555  G7 G8
    if (!eq(ap(s[state], i), Leader)) return;
    if (in_set(j, GetConfig(s, i))) return;
    State t = s;
    t[currentTerm] = except(s[currentTerm], j, Int(1));
    t[votedFor] = except(s[votedFor], j, Nil);
    V m = rec({{"mtype", CReq}, {"mterm", ap(s[currentTerm], i)}, {"mlogLen", ap(ap(s[matchIndex], i), j)},
               {"mentries", subseq(ap(s[log], i), as_int(ap(ap(s[nextIndex], i), j)), as_int(ap(s[commitIndex], i)))},
               {"mcommitIndex", ap(s[commitIndex], i)}, {"msource", i}, {"mdest", j}, {"mrounds", NumRounds}});
    SendDirect(t, s, m);
    out.push_back({t, A_AddNewServer});
  }
  void DeleteServer(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {         // :558-569
    if (!eq(ap(s[state], i), Leader)) return;
    V sj = ap(s[state], j);
    if (!(eq(sj, Follower) || eq(sj, Candidate))) return;
    if (!in_set(j, GetConfig(s, i))) return;
    if (eq(j, i)) return;
    V m = rec({{"mtype", COC}, {"mterm", ap(s[currentTerm], i)}, {"madd", Bool(false)}, {"mserver", j},
               {"msource", i}, {"mdest", i}});
    State t = s; SendDirect(t, s, m);
    out.push_back({t, A_DeleteServer});
  }
  // ------------------------------------------------------------ handlers, i = recipient, j = sender
  void HandleRequestVoteRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const {  // :578-597
    V li = ap(s[log], i);
    bool logOk = as_int(ap(m, "mlastLogTerm")) > LastTerm(li) ||
                 (as_int(ap(m, "mlastLogTerm")) == LastTerm(li) && as_int(ap(m, "mlastLogIndex")) >= len(li));
    V vf = ap(s[votedFor], i);
    bool grant = eq(ap(m, "mterm"), ap(s[currentTerm], i)) && logOk && (eq(vf, Nil) || eq(vf, j));
    if (!(as_int(ap(m, "mterm")) <= as_int(ap(s[currentTerm], i)))) return;
    State t = s;
    if (grant) t[votedFor] = except(s[votedFor], i, j);
    V resp = rec({{"mtype", RVResp}, {"mterm", ap(s[currentTerm], i)}, {"mvoteGranted", Bool(grant)},
                  {"mlog", li}, {"msource", i}, {"mdest", j}});
    ReplyDirect(t, s, resp, m);
    out.push_back({t, A_HandleRequestVoteRequest});
  }
  void HandleRequestVoteResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :602-614
    if (!eq(ap(m, "mterm"), ap(s[currentTerm], i))) return;
    State t = s;
    t[votesResponded] = except(s[votesResponded], i, cup(ap(s[votesResponded], i), set({j})));
    if (as_bool(ap(m, "mvoteGranted")))
      t[votesGranted] = except(s[votesGranted], i, cup(ap(s[votesGranted], i), set({j})));
    DiscardDirect(t, s, m);
    out.push_back({t, A_HandleRequestVoteResponse});
  }
  void HandleAppendEntriesRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :617-700
    V li = ap(s[log], i);
    int64_t pli = as_int(ap(m, "mprevLogIndex"));
    bool logOk = pli == 0 || (pli > 0 && pli <= len(li) && eq(ap(m, "mprevLogTerm"), ap(ap(li, pli), "term")));
    int64_t mterm = as_int(ap(m, "mterm")), ct = as_int(ap(s[currentTerm], i));
    V st = ap(s[state], i);
    if (!(mterm <= ct)) return;
    if (mterm < ct || (mterm == ct && eq(st, Follower) && !logOk)) {                  // Reject (:617-629)
      V resp = rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(false)}, {"mmatchIndex", Int(0)},
                    {"msource", i}, {"mdest", j}});
      State t = s; ReplyDirect(t, s, resp, m);
      out.push_back({t, A_HandleAppendEntriesRequest});
    }
    if (mterm == ct && eq(st, Candidate)) {                                          // ReturnToFollowerState (:632-636)
      State t = s; t[state] = except(s[state], i, Follower);
      out.push_back({t, A_HandleAppendEntriesRequest});
    }
    if (mterm == ct && eq(st, Follower) && logOk) {                                   // Accept (:675-683)
      int64_t index = pli + 1;
      V ents = ap(m, "mentries");
      if (len(ents) == 0 ||
          (len(ents) > 0 && len(li) >= index && eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term")))) {   // AlreadyDone (:639-655)
        State t = s;
        t[commitIndex] = except(s[commitIndex], i, ap(m, "mcommitIndex"));
        V resp = rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(true)},
                      {"mmatchIndex", Int(pli + len(ents))}, {"msource", i}, {"mdest", j}});
        ReplyDirect(t, s, resp, m);
        out.push_back({t, A_HandleAppendEntriesRequest});
      }
      if (len(ents) > 0 && len(li) >= index && !eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term"))) {  // Conflict (:658-665)
        State t = s; t[log] = except(s[log], i, subseq(li, 1, len(li) - 1));
        out.push_back({t, A_HandleAppendEntriesRequest});
      }
      if (len(ents) > 0 && len(li) == pli) {                                          // NoConflict (:668-672)
        State t = s; t[log] = except(s[log], i, append(li, ap(ents, 1)));
        out.push_back({t, A_HandleAppendEntriesRequest});
      }
    }
  }
  void HandleAppendEntriesResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :705-715
    if (!eq(ap(m, "mterm"), ap(s[currentTerm], i))) return;
    State t = s;
    if (as_bool(ap(m, "msuccess"))) {
      t[nextIndex] = except(s[nextIndex], i, except(ap(s[nextIndex], i), j, Int(as_int(ap(m, "mmatchIndex")) + 1)));
      t[matchIndex] = except(s[matchIndex], i, except(ap(s[matchIndex], i), j, ap(m, "mmatchIndex")));
    } else {
      int64_t ni = as_int(ap(ap(s[nextIndex], i), j));
      t[nextIndex] = except(s[nextIndex], i, except(ap(s[nextIndex], i), j, Int(std::max<int64_t>(ni - 1, 1))));
    }
    DiscardDirect(t, s, m);
    out.push_back({t, A_HandleAppendEntriesResponse});
  }
  void HandleCatchupRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const {       // :718-745  G5
    int64_t mterm = as_int(ap(m, "mterm")), ct = as_int(ap(s[currentTerm], i));
    if (mterm < ct) {
      V resp = rec({{"mtype", CResp}, {"mterm", Int(ct)}, {"msuccess", Bool(false)}, {"mmatchIndex", Int(0)},
                    {"msource", i}, {"mdest", j}, {"mroundsLeft", Int(0)}});
      State t = s; ReplyDirect(t, s, resp, m);
      out.push_back({t, A_HandleCatchupRequest});
    }
    if (mterm >= ct) {
      V li = ap(s[log], i), ents = ap(m, "mentries");
      State t = s;
      t[currentTerm] = except(s[currentTerm], i, ap(m, "mterm"));
      V nl = len(li) == 0 ? ents : concat(subseq(li, 1, std::min(as_int(ap(m, "mlogLen")), len(li))), ents);
      t[log] = except(s[log], i, nl);
      V resp = rec({{"mtype", CResp}, {"mterm", ap(m, "mterm")}, {"msuccess", Bool(true)}, {"mmatchIndex", Int(len(li))},
                    {"msource", i}, {"mdest", j}, {"mroundsLeft", Int(as_int(ap(m, "mrounds")) - 1)}});
      ReplyDirect(t, s, resp, m);
      out.push_back({t, A_HandleCatchupRequest});
    }
  }
  void HandleCatchupResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const {      // :748-792
    int64_t mmi = as_int(ap(m, "mmatchIndex")), ci = as_int(ap(s[commitIndex], i));
    int64_t mi = as_int(ap(ap(s[matchIndex], i), j)), ni = as_int(ap(ap(s[nextIndex], i), j));
    bool succ = as_bool(ap(m, "msuccess"));
    bool isLeader = eq(ap(s[state], i), Leader), termEq = eq(ap(m, "mterm"), ap(s[currentTerm], i));
    bool inCfg = in_set(j, GetConfig(s, i));
    if (succ && ((mmi != ci && mmi != mi) || mmi == ci) && isLeader && termEq && !inCfg) {
      State t = s;
      t[nextIndex] = except(s[nextIndex], i, except(ap(s[nextIndex], i), j, Int(mmi + 1)));
      t[matchIndex] = except(s[matchIndex], i, except(ap(s[matchIndex], i), j, Int(mmi)));
      int64_t rl = as_int(ap(m, "mroundsLeft"));
      if (rl != 0) {
        V r = rec({{"mtype", CReq}, {"mterm", ap(s[currentTerm], i)},
                   {"mentries", subseq(ap(s[log], i), ni, ci)}, {"mlogLen", Int(ni - 1)},
                   {"msource", i}, {"mdest", j}, {"mrounds", Int(rl)}});
        State u = t; ReplyDirect(u, s, r, m); out.push_back({u, A_HandleCatchupResponse});
      }
      if (rl == 0) {
        V r = rec({{"mtype", COC}, {"mterm", ap(s[currentTerm], i)}, {"madd", Bool(true)}, {"mserver", j},
                   {"msource", i}, {"mdest", i}});
        State u = t; ReplyDirect(u, s, r, m); out.push_back({u, A_HandleCatchupResponse});
      }
    }
    // TLC's getNextStates enumerates each true disjunct of this list as a branch of its own, so the
    // discard successor is generated once per true disjunct (:783-789; the inner disjunct
    // `mmi = ci \/ mmi = mi` is followed by `mmi /= ci`, which only its second branch passes)
    // (switch (vi) off: once)
    int copies = (!succ) + (mmi == mi && mmi != ci) + (!isLeader) + (!termEq) + inCfg;
    if (!disjunct_copies) copies = std::min(copies, 1);
    for (int q = 0; q < copies; ++q) {
      State t = s; DiscardDirect(t, s, m); out.push_back({t, A_HandleCatchupResponse});
    }
  }
  void HandleCheckOldConfig(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {                  // :795-822  G6
    bool isLeader = eq(ap(s[state], i), Leader), termEq = eq(ap(m, "mterm"), ap(s[currentTerm], i));
    // :796 `state[i] /= Leader \/ m.mterm = currentTerm[i]`: TLC enumerates each true disjunct as a
    // branch, so a non-leader receiving a current-term message generates the discard twice
    const int copies = disjunct_copies ? (int)(!isLeader) + (int)termEq : (int)(!isLeader || termEq);
    for (int q = 0; q < copies; ++q) {
      State t = s; DiscardDirect(t, s, m); out.push_back({t, A_HandleCheckOldConfig});
    }
    if (isLeader && termEq) {
      int64_t mci = GetMaxConfigIndex(s, i), ci = as_int(ap(s[commitIndex], i));
      if (mci <= ci) {
        bool madd = as_bool(ap(m, "madd"));
        V srv = ap(m, "mserver"), cfgI = GetConfig(s, i);
        V action = madd ? rec({{"action", Str("AddServer")}, {"executedOn", i}, {"added", srv}})
                        : rec({{"action", Str("RemoveServer")}, {"executedOn", i}, {"removed", srv}});
        V newConfig = madd ? cup(cfgI, set({srv})) : setminus(cfgI, set({srv}));
        bool changed = !eq(cfgI, newConfig);
        V newEntry = rec({{"term", ap(s[currentTerm], i)}, {"type", ConfigEntry}, {"value", newConfig}});
        State t = s;
        t[log] = except(s[log], i, changed ? append(ap(s[log], i), newEntry) : ap(s[log], i));
        if (changed) DiscardWithMC(t, s, m, action); else DiscardDirect(t, s, m);
        out.push_back({t, A_HandleCheckOldConfig});
      }
      if (mci > ci) {
        V r = rec({{"mtype", COC}, {"mterm", ap(s[currentTerm], i)}, {"madd", ap(m, "madd")}, {"mserver", ap(m, "mserver")},
                   {"msource", i}, {"mdest", i}});
        State t = s; ReplyDirect(t, s, r, m); out.push_back({t, A_HandleCheckOldConfig});
      }
    }
  }
  void UpdateTerm(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {            // :826-832  G9
    if (!(as_int(ap(m, "mterm")) > as_int(ap(s[currentTerm], i)))) return;
    State t = s;
    t[currentTerm] = except(s[currentTerm], i, ap(m, "mterm"));
    t[state] = except(s[state], i, Follower);
    t[votedFor] = except(s[votedFor], i, Nil);
    out.push_back({t, A_UpdateTerm});
  }
  void DropStaleResponse(const State& s, const V& m, std::vector<Succ>& out) const {                  // :836-839
    V i = ap(m, "mdest");
    if (!(as_int(ap(m, "mterm")) < as_int(ap(s[currentTerm], i)))) return;
    State t = s; DiscardDirect(t, s, m); out.push_back({t, A_DropStaleResponse});
  }
  void Receive(const State& s, const V& m, std::vector<Succ>& out) const {                            // :842-863
    V i = ap(m, "mdest"), j = ap(m, "msource"), ty = ap(m, "mtype");
    UpdateTerm(s, i, m, out);
    if (eq(ty, RVReq)) HandleRequestVoteRequest(s, i, j, m, out);
    if (eq(ty, RVResp)) { DropStaleResponse(s, m, out); HandleRequestVoteResponse(s, i, j, m, out); }
    if (eq(ty, AEReq)) HandleAppendEntriesRequest(s, i, j, m, out);
    if (eq(ty, AEResp)) { DropStaleResponse(s, m, out); HandleAppendEntriesResponse(s, i, j, m, out); }
    if (eq(ty, CReq)) HandleCatchupRequest(s, i, j, m, out);
    if (eq(ty, CResp)) HandleCatchupResponse(s, i, j, m, out);
    if (eq(ty, COC)) HandleCheckOldConfig(s, i, m, out);
  }

  // ------------------------------------------------------------ Next variants (:909-943)
  void next(const State& s, std::vector<Succ>& out) const override {
    if (use_async) {                                                        // NextAsync :909-916
      for (auto& i : Server->a) for (auto& j : Server->a) RequestVote(s, i, j, out);
      for (auto& i : Server->a) BecomeLeader(s, i, out);
      for (auto& i : Server->a) for (auto& v : Value->a) ClientRequest(s, i, v, out);
      for (auto& i : Server->a) AdvanceCommitIndex(s, i, out);
      for (auto& i : Server->a) for (auto& j : Server->a) AppendEntries(s, i, j, out);
      for (auto& m : domain_elems(s[messages])) Receive(s, m, out);
      for (auto& i : Server->a) Timeout(s, i, out);
    }
    if (use_crash) for (auto& i : Server->a) Restart(s, i, out);            // NextCrash :918
    if (use_unreliable) {                                                   // NextUnreliable :924-932
      for (auto& m : domain_elems(s[messages]))
        if (as_int(ap(s[messages], m)) == 1) { State t = s; t[messages] = WithMessage(m, s[messages]); out.push_back({t, A_DuplicateMessage}); }
      for (auto& m : domain_elems(s[messages]))
        if (as_int(ap(s[messages], m)) == 1) { State t = s; t[messages] = WithoutMessage(m, s[messages]); out.push_back({t, A_DropMessage}); }
    }
    if (use_dynamic) {                                                      // NextDynamic :940-943
      for (auto& i : Server->a) for (auto& j : Server->a) AddNewServer(s, i, j, out);
      for (auto& i : Server->a) for (auto& j : Server->a) DeleteServer(s, i, j, out);
    }
  }

  // ------------------------------------------------------------ constraints (:1105-1137, :1182-1234)
  int64_t SumServer(const State& s, const char* f) const {
    int64_t t = 0; V srv = H(s, "server");
    for (auto& i : Server->a) t += as_int(ap(ap(srv, i), f));
    return t;
  }
  bool ElectionsUncontested(const State& s) const {                        // :1126
    int64_t c = 0; for (auto& i : domain_elems(s[state])) if (eq(ap(s[state], i), Candidate)) c++;
    return c <= 1;
  }
  bool bound_prefix(const State& s, const std::vector<V>& golden) const {   // _unique / MajorityOfClusterRestarts_constraint
    V g = H(s, "global");
    // \E s1, s2, s3 \in Server : Cardinality({s1,s2,s3}) = 3 /\ IsPrefix(SubSeq(trace, 1, maxLen), g)
    auto& S = Server->a;
    size_t n = S.size();
    int id1 = Names::get().intern_mv("s1"), id2 = Names::get().intern_mv("s2"), id3 = Names::get().intern_mv("s3");
    for (size_t a = 0; a < n; ++a) for (size_t b = 0; b < n; ++b) for (size_t c = 0; c < n; ++c) {
      if (a == b || b == c || a == c) continue;
      std::vector<int> perm(Names::get().mv.size(), -1);
      perm[id1] = (int)S[a]->i; perm[id2] = (int)S[b]->i; perm[id3] = (int)S[c]->i;
      // the golden is written over placeholders s1,s2,s3: rename them to the bound servers
      size_t maxLen = std::min(golden.size(), g->a.size());
      bool ok = true;
      for (size_t q = 0; q < maxLen && ok; ++q) ok = eq(permute(golden[q], perm), g->a[q]);
      if (ok) return true;
    }
    return false;
  }
  bool constraint(const std::string& n, const State& s) const override {
    if (n == "BoundedInFlightMessages") {                                  // :1105 (BagCardinality = Sum)
      int64_t t = 0; for (auto& m : domain_elems(s[messages])) t += as_int(ap(s[messages], m));
      return t <= MaxInFlightMessages();
    }
    if (n == "BoundedRequestVote") {                                       // :1108-1110
      for (auto& m : domain_elems(s[messages]))
        if (eq(ap(m, "mtype"), RVReq) && as_int(ap(s[messages], m)) > 1) return false;
      return true;
    }
    if (n == "BoundedLogSize") { for (auto& i : Server->a) if (len(ap(s[log], i)) > MaxLogLength) return false; return true; }
    if (n == "BoundedRestarts") { for (auto& i : Server->a) if (as_int(ap(ap(H(s, "server"), i), "restarted")) > MaxRestarts) return false; return true; }
    if (n == "BoundedTimeouts") { for (auto& i : Server->a) if (as_int(ap(ap(H(s, "server"), i), "timeout")) > MaxTimeouts) return false; return true; }
    if (n == "BoundedTerms") { for (auto& i : Server->a) if (as_int(ap(s[currentTerm], i)) > MaxTerms) return false; return true; }
    if (n == "BoundedClientRequests") return as_int(H(s, "hadNumClientRequests")) <= MaxClientRequests;
    if (n == "BoundedTriedMembershipChanges") return as_int(H(s, "hadNumTriedMembershipChanges")) <= MaxTriedMembershipChanges;
    if (n == "BoundedMembershipChanges") return as_int(H(s, "hadNumMembershipChanges")) <= MaxMembershipChanges;
    if (n == "ElectionsUncontested") return ElectionsUncontested(s);
    if (n == "CleanStartUntilFirstRequest") {                              // :1128-1132
      if (!(as_int(H(s, "hadNumLeaders")) < 1 && as_int(H(s, "hadNumClientRequests")) < 1)) return true;
      for (auto& i : Server->a) if (as_int(ap(ap(H(s, "server"), i), "restarted")) != 0) return false;
      return SumServer(s, "timeout") <= 1 && ElectionsUncontested(s);
    }
    if (n == "CleanStartUntilTwoLeaders") {                                // :1134-1137
      if (!(as_int(H(s, "hadNumLeaders")) < 2)) return true;
      return SumServer(s, "restarted") <= 1 && SumServer(s, "timeout") <= 2;
    }
    if (n == "CommitWhenConcurrentLeaders_constraint") {                   // :1182-1186
      V g = H(s, "global");
      if (len(g) < 20) return true;
      for (auto& x : g->a) if (eq(ap(x, "action"), Str("BecomeLeader")) && card(ap(x, "leaders")) >= 2) return true;
      return false;
    }
    if (n == "CommitWhenConcurrentLeaders_unique") {
      if (golden_cwcl.empty()) throw EvalError("CommitWhenConcurrentLeaders_unique needs --golden-cwcl");
      return bound_prefix(s, golden_cwcl);
    }
    if (n == "MajorityOfClusterRestarts_constraint") {
      if (golden_morc.empty()) throw EvalError("MajorityOfClusterRestarts_constraint needs --golden-morc");
      return bound_prefix(s, golden_morc);
    }
    throw EvalError("unknown constraint " + n);
  }
  bool action_constraint(const std::string& n, const State& s, const State& t) const override {
    if (n == "CommitWhenConcurrentLeaders_action_constraint") {            // :1207-1210
      if (len(H(s, "global")) < 20) return true;
      for (auto& i : Server->a) if (eq(ap(t[state], i), Candidate)) return false;
      return true;
    }
    throw EvalError("unknown action constraint " + n);
  }

  // ------------------------------------------------------------ invariants (:969-1099, :1143-1278)
  static bool hasAction(const V& g, const char* a) { for (auto& x : g->a) if (eq(ap(x, "action"), Str(a))) return true; return false; }
  bool invariant(const std::string& n, const State& s) const override {
    const auto& S = Server->a;
    if (n == "LeaderVotesQuorum") {                                        // :988-993
      if (as_int(H(s, "hadNumMembershipChanges")) != 0) return true;
      for (auto& i : S) if (eq(ap(s[state], i), Leader)) {
        std::vector<V> xs;
        for (auto& j : S) {
          int64_t tj = as_int(ap(s[currentTerm], j)), ti = as_int(ap(s[currentTerm], i));
          if (tj > ti || (tj == ti && eq(ap(s[votedFor], j), i))) xs.push_back(j);
        }
        if (!InQuorum(set(xs), GetConfig(s, i))) return false;
      }
      return true;
    }
    if (n == "CandidateTermNotInLog") {                                    // :997-1004
      if (as_int(H(s, "hadNumMembershipChanges")) != 0) return true;
      for (auto& i : S) {
        if (!eq(ap(s[state], i), Candidate)) continue;
        std::vector<V> xs;
        for (auto& j : S) { V vf = ap(s[votedFor], j); if (eq(ap(s[currentTerm], j), ap(s[currentTerm], i)) && (eq(vf, i) || eq(vf, Nil))) xs.push_back(j); }
        if (!InQuorum(set(xs), GetConfig(s, i))) continue;
        for (auto& j : S) { V lj = ap(s[log], j); for (int64_t q = 1; q <= len(lj); ++q) if (eq(ap(ap(lj, q), "term"), ap(s[currentTerm], i))) return false; }
      }
      return true;
    }
    if (n == "ElectionSafety") {                                           // :1009-1014
      for (auto& i : S) if (eq(ap(s[state], i), Leader)) {
        V ti = ap(s[currentTerm], i);
        auto mo = [&](const V& lg) { int64_t mx = 0; for (int64_t q = 1; q <= len(lg); ++q) if (eq(ap(ap(lg, q), "term"), ti)) mx = q; return mx; };
        int64_t a = mo(ap(s[log], i));
        for (auto& j : S) if (!(a >= mo(ap(s[log], j)))) return false;
      }
      return true;
    }
    if (n == "LogMatching") {                                              // :1017-1021
      for (auto& i : S) for (auto& j : S) {
        V li = ap(s[log], i), lj = ap(s[log], j);
        for (int64_t q = 1; q <= std::min(len(li), len(lj)); ++q)
          if (eq(ap(ap(li, q), "term"), ap(ap(lj, q), "term")) && !eq(subseq(li, 1, q), subseq(lj, 1, q))) return false;
      }
      return true;
    }
    if (n == "VotesGrantedInv") {                                          // :1048-1052
      for (auto& i : S) for (auto& j : S) if (eq(ap(s[votedFor], i), j) && !is_prefix(Committed(s, i), ap(s[log], j))) return false;
      return true;
    }
    if (n == "VotesGrantedInv_false") {                                    // :1038-1046
      for (auto& i : S) for (auto& j : ap(s[votesGranted], i)->a)
        if (eq(ap(s[currentTerm], i), ap(s[currentTerm], j)) && !is_prefix(Committed(s, j), ap(s[log], i))) return false;
      return true;
    }
    if (n == "QuorumLogInv") {                                             // :1056-1060
      for (auto& i : S) {
        V cfgI = GetConfig(s, i);
        for (auto& Q : subsets(cfgI)) {
          if (!InQuorum(Q, cfgI)) continue;
          bool ok = false;
          for (auto& j : Q->a) if (is_prefix(Committed(s, i), ap(s[log], j))) { ok = true; break; }
          if (!ok) return false;
        }
      }
      return true;
    }
    if (n == "MoreUpToDateCorrect") {                                      // :1066-1071
      for (auto& i : S) for (auto& j : S) {
        V li = ap(s[log], i), lj = ap(s[log], j);
        if ((LastTerm(li) > LastTerm(lj) || (LastTerm(li) == LastTerm(lj) && len(li) >= len(lj))) &&
            !is_prefix(Committed(s, j), li)) return false;
      }
      return true;
    }
    if (n == "LeaderCompleteness_false") {                                 // :1079-1083
      for (auto& i : S) if (eq(ap(s[state], i), Leader)) for (auto& j : S) if (!is_prefix(Committed(s, j), ap(s[log], i))) return false;
      return true;
    }
    if (n == "LeaderCompleteness") {                                       // :1089-1099
      V leaders = CurrentLeaders(s);
      for (auto& i : S) {
        V committed = Committed(s, i);
        for (int64_t idx = 1; idx <= len(committed); ++idx) {
          V entry = ap(ap(s[log], i), idx);
          for (auto& l : leaders->a)
            if (as_int(ap(s[currentTerm], l)) > as_int(ap(entry, "term")) && !eq(ap(ap(s[log], l), idx), entry)) return false;
        }
      }
      return true;
    }
    V g = H(s, "global");
    if (n == "BoundedTrace") return len(g) <= 24;                          // :1143
    if (n == "FirstBecomeLeader") return !hasAction(g, "BecomeLeader");    // :1145
    if (n == "FirstCommit") { for (auto& i : S) if (as_int(ap(s[commitIndex], i)) > 0) return false; return true; }   // :1148
    if (n == "FirstRestart") { for (auto& i : S) if (as_int(ap(ap(H(s, "server"), i), "restarted")) >= 2) return false; return true; }
    if (n == "LeadershipChange") return as_int(H(s, "hadNumLeaders")) < 2;
    if (n == "MembershipChange") return as_int(H(s, "hadNumMembershipChanges")) < 1;
    if (n == "MultipleMembershipChanges") return as_int(H(s, "hadNumMembershipChanges")) < 2;
    if (n == "ConcurrentLeaders") return !(card(CurrentLeaders(s)) >= 2);  // :1158
    if (n == "EntryCommitted") return !hasAction(g, "CommitEntry");        // :1160-1163
    if (n == "CommitWhenConcurrentLeaders") {                              // :1165-1176
      int64_t L = len(g);
      for (int64_t i = 1; i <= L; ++i) for (int64_t k = i + 1; k <= L; ++k) {
        V x = ap(g, i), y = ap(g, k);
        if (eq(ap(x, "action"), Str("BecomeLeader")) && card(ap(x, "leaders")) >= 2 && eq(ap(y, "action"), Str("CommitEntry")) &&
            L >= k + 2 && card(CurrentLeaders(s)) >= 2) return false;
      }
      return true;
    }
    if (n == "MajorityOfClusterRestarts") {                                // :1212-1226
      bool logs = false;
      for (auto& i : S) for (auto& j : S) if (!eq(i, j) && len(ap(s[log], i)) >= 2 && len(ap(s[log], j)) >= 1) logs = true;
      if (!logs) return true;
      bool maj = false;
      for (auto& Q : subsets(Server)) {
        if (!InQuorum(Q, Server)) continue;
        bool all = true; for (auto& i : Q->a) if (as_int(ap(ap(H(s, "server"), i), "restarted")) < 1) all = false;
        if (all) { maj = true; break; }
      }
      if (!maj) return true;
      int64_t L = len(g);
      for (int64_t i = 1; i <= L; ++i) for (int64_t k = 1; k <= L; ++k)
        if (i < k && eq(ap(ap(g, i), "action"), Str("Restart")) && eq(ap(ap(g, k), "action"), Str("Restart")) && !(k - i >= 6)) return true;
      return false;
    }
    if (n == "AddSucessful") return !hasAction(g, "AddServer");            // :1236
    if (n == "MembershipChangeCommits") return !hasAction(g, "CommitMembershipChange");
    auto pairs = [&](auto pred) {
      int64_t L = len(g);
      for (int64_t i = 1; i <= L; ++i) for (int64_t j = i + 1; j <= L; ++j) if (pred(i, j, ap(g, i), ap(g, j))) return false;
      return true;
    };
    if (n == "MultipleMembershipChangesCommit")                            // :1242-1246
      return pairs([&](int64_t, int64_t, const V& x, const V& y) {
        return eq(ap(x, "action"), Str("CommitMembershipChange")) && eq(ap(y, "action"), Str("CommitMembershipChange")); });
    if (n == "AddCommits")                                                 // :1248-1256
      return pairs([&](int64_t, int64_t, const V& x, const V& y) {
        return eq(ap(x, "action"), Str("AddServer")) && eq(ap(y, "action"), Str("CommitMembershipChange")) && in_set(ap(x, "added"), ap(y, "config")); });
    if (n == "NewlyJoinedBecomeLeader")                                    // :1258-1266
      return pairs([&](int64_t, int64_t, const V& x, const V& y) {
        return eq(ap(x, "action"), Str("AddServer")) && eq(ap(y, "action"), Str("BecomeLeader")) && eq(ap(x, "added"), ap(y, "executedOn")); });
    if (n == "LeaderChangesDuringConfChange")                              // :1268-1278
      return pairs([&](int64_t i, int64_t k, const V& x, const V& y) {
        if (!(eq(ap(x, "action"), Str("AddServer")) && eq(ap(y, "action"), Str("BecomeLeader")))) return false;
        for (int64_t j = i; j <= k; ++j) if (eq(ap(ap(g, j), "action"), Str("CommitMembershipChange"))) return false;
        return true; });
    throw EvalError("unknown invariant " + n);
  }

  // Dumps and traces print history without its unbounded "global" sequence: the
  // product keeps a summary automaton of it (raft-tla_amd/csrc/memb_spec.h), so
  // state-set parity is checked on the view plus every history counter.
  std::string dump_line(const State& s) const override {
    State t = s;
    std::vector<V> ks, vs;
    const V& h = s[history];
    for (size_t q = 0; q < h->a.size(); ++q) if (!eq(h->a[q], Str("global"))) { ks.push_back(h->a[q]); vs.push_back(h->b[q]); }
    t[history] = fcn(ks, vs);
    return state_text(*this, t);
  }

  // ------------------------------------------------------------ VIEW vars / SYMMETRY perms (:193, :1281)
  std::vector<int> view_vars(const std::string& view) const override {
    if (view == "vars") return {messages, currentTerm, state, votedFor, votesResponded, votesGranted, nextIndex, matchIndex, log, commitIndex};
    throw EvalError("unknown VIEW " + view);
  }
  std::vector<std::vector<int>> symmetry_perms(const std::string& sym) const override {
    if (sym != "perms") throw EvalError("unknown SYMMETRY " + sym);
    std::vector<int> ids; for (auto& x : Server->a) { if (x->k != K::MV) throw EvalError("SYMMETRY over non-model values"); ids.push_back((int)x->i); }
    std::vector<int> p = ids; std::sort(p.begin(), p.end());
    std::vector<std::vector<int>> out;
    do {
      std::vector<int> m(Names::get().mv.size() + 16, -1);
      for (size_t q = 0; q < ids.size(); ++q) m[ids[q]] = p[q];
      out.push_back(m);
    } while (std::next_permutation(p.begin(), p.end()));
    return out;
  }
};

}  // namespace oracle
