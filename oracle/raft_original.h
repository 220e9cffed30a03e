// ============================================================================
// TEST INFRASTRUCTURE ONLY (see oracle/tla.h header).
//
// Literal CPU restatement of thirdparty/raft_original.tla (Ongaro 2014) over
// the explicit value model of tla.h.  Every function cites the lines it
// follows.  The model-checking wrapper operators (bounds, ElectionSafety,
// LogMatching) follow configs/raft_original_mc.tla, which the reference does
// not provide ("raft_original has none", "must be
// authored").
// ============================================================================
#pragma once
#include "engine.h"

namespace oracle {

struct RaftOriginal : Spec {
  // VARIABLE declaration order, raft_original.tla:32-85
  enum { messages, elections, allLogs, currentTerm, state, votedFor, log, commitIndex,
         votesResponded, votesGranted, voterLog, nextIndex, matchIndex, NVARS };
  // action ids (Next disjuncts raft_original.tla:453-462; Receive split by handler :420-435)
  enum { A_Restart, A_Timeout, A_RequestVote, A_BecomeLeader, A_ClientRequest, A_AdvanceCommitIndex,
         A_AppendEntries, A_UpdateTerm, A_HandleRequestVoteRequest, A_DropStaleResponse,
         A_HandleRequestVoteResponse, A_HandleAppendEntriesRequest, A_HandleAppendEntriesResponse,
         A_DuplicateMessage, A_DropMessage, NACT };

  const Cfg& cfg;
  V Server, Value, Follower, Candidate, Leader, Nil, RVReq, RVResp, AEReq, AEResp;
  int64_t MaxTerm = 0, MaxLogLen = 0, MaxMsgDomain = 0, MinMsgCount = 0, MaxMsgCount = 0;
  std::vector<std::string> vn;

  explicit RaftOriginal(const Cfg& c) : cfg(c) {
    Server = c.get("Server"); Value = c.get("Value");
    Follower = c.get("Follower"); Candidate = c.get("Candidate"); Leader = c.get("Leader");
    Nil = c.get("Nil");
    RVReq = c.get("RequestVoteRequest"); RVResp = c.get("RequestVoteResponse");
    AEReq = c.get("AppendEntriesRequest"); AEResp = c.get("AppendEntriesResponse");
    auto opt = [&](const char* n, int64_t& dst) { if (c.has(n)) dst = as_int(c.get(n)); };
    opt("MaxTerm", MaxTerm); opt("MaxLogLen", MaxLogLen); opt("MaxMsgDomain", MaxMsgDomain);
    opt("MinMsgCount", MinMsgCount); opt("MaxMsgCount", MaxMsgCount);
    vn = {"messages", "elections", "allLogs", "currentTerm", "state", "votedFor", "log", "commitIndex",
          "votesResponded", "votesGranted", "voterLog", "nextIndex", "matchIndex"};
  }
  const std::vector<std::string>& var_names() const override { return vn; }
  std::vector<std::string> action_names() const override {
    return {"Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex",
            "AppendEntries", "UpdateTerm", "HandleRequestVoteRequest", "DropStaleResponse",
            "HandleRequestVoteResponse", "HandleAppendEntriesRequest", "HandleAppendEntriesResponse",
            "DuplicateMessage", "DropMessage"};
  }

  // ---- helpers (raft_original.tla:97-134)
  V fnOver(const V& dom, const V& val) const {   // [i \in dom |-> val]
    std::vector<V> ks = dom->a, vs(dom->a.size(), val); return fcn(ks, vs);
  }
  bool IsQuorum(const V& s) const { return subseteq(s, Server) && card(s) * 2 > card(Server); }   // :99
  int64_t LastTerm(const V& xlog) const {                                                          // :102
    return len(xlog) == 0 ? 0 : as_int(ap(ap(xlog, len(xlog)), "term"));
  }
  V WithMessage(const V& m, const V& msgs) const {                                                 // :106-110
    if (in_domain(msgs, m)) return except(msgs, m, Int(as_int(ap(msgs, m)) + 1));
    return at_at(msgs, colon_gt(m, Int(1)));
  }
  V WithoutMessage(const V& m, const V& msgs) const {                                              // :114-118
    if (in_domain(msgs, m)) return except(msgs, m, Int(as_int(ap(msgs, m)) - 1));
    return msgs;
  }
  static V Min2(int64_t a, int64_t b) { return Int(std::min(a, b)); }

  // ---- Init (raft_original.tla:139-159)
  std::vector<State> init() const override {
    State s(NVARS);
    s[messages] = fcn({}, {});                               // [m \in {} |-> 0]
    s[elections] = empty_set(); s[allLogs] = empty_set();
    s[voterLog] = fnOver(Server, fcn({}, {}));               // [j \in {} |-> <<>>]
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

  // ---- actions; each returns successors into out (with allLogs' set by next())
  void Restart(const State& s, const V& i, std::vector<Succ>& out) const {                         // :166-174
    State t = s;
    t[state] = except(s[state], i, Follower);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    t[voterLog] = except(s[voterLog], i, fcn({}, {}));
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    t[commitIndex] = except(s[commitIndex], i, Int(0));
    out.push_back({t, A_Restart});
  }
  void Timeout(const State& s, const V& i, std::vector<Succ>& out) const {                         // :177-186
    V st = ap(s[state], i);
    if (!(eq(st, Follower) || eq(st, Candidate))) return;
    State t = s;
    t[state] = except(s[state], i, Candidate);
    t[currentTerm] = except(s[currentTerm], i, Int(as_int(ap(s[currentTerm], i)) + 1));
    t[votedFor] = except(s[votedFor], i, Nil);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    t[voterLog] = except(s[voterLog], i, fcn({}, {}));
    out.push_back({t, A_Timeout});
  }
  void RequestVote(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {         // :189-198
    if (!eq(ap(s[state], i), Candidate)) return;
    if (in_set(j, ap(s[votesResponded], i))) return;
    V li = ap(s[log], i);
    V m = rec({{"mtype", RVReq}, {"mterm", ap(s[currentTerm], i)}, {"mlastLogTerm", Int(LastTerm(li))},
               {"mlastLogIndex", Int(len(li))}, {"msource", i}, {"mdest", j}});
    State t = s; t[messages] = WithMessage(m, s[messages]);
    out.push_back({t, A_RequestVote});
  }
  void AppendEntries(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {       // :203-225
    if (eq(i, j)) return;
    if (!eq(ap(s[state], i), Leader)) return;
    V li = ap(s[log], i);
    int64_t ni = as_int(ap(ap(s[nextIndex], i), j));
    int64_t prevLogIndex = ni - 1;
    int64_t prevLogTerm = prevLogIndex > 0 ? as_int(ap(ap(li, prevLogIndex), "term")) : 0;   // unguarded (:207-210)
    int64_t lastEntry = std::min(len(li), ni);
    V entries = subseq(li, ni, lastEntry);
    V m = rec({{"mtype", AEReq}, {"mterm", ap(s[currentTerm], i)}, {"mprevLogIndex", Int(prevLogIndex)},
               {"mprevLogTerm", Int(prevLogTerm)}, {"mentries", entries}, {"mlog", li},
               {"mcommitIndex", Min2(as_int(ap(s[commitIndex], i)), lastEntry)}, {"msource", i}, {"mdest", j}});
    State t = s; t[messages] = WithMessage(m, s[messages]);
    out.push_back({t, A_AppendEntries});
  }
  void BecomeLeader(const State& s, const V& i, std::vector<Succ>& out) const {                    // :228-242
    if (!eq(ap(s[state], i), Candidate)) return;
    if (!IsQuorum(ap(s[votesGranted], i))) return;
    State t = s;
    t[state] = except(s[state], i, Leader);
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(len(ap(s[log], i)) + 1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    V e = rec({{"eterm", ap(s[currentTerm], i)}, {"eleader", i}, {"elog", ap(s[log], i)},
               {"evotes", ap(s[votesGranted], i)}, {"evoterLog", ap(s[voterLog], i)}});
    t[elections] = cup(s[elections], set({e}));
    out.push_back({t, A_BecomeLeader});
  }
  void ClientRequest(const State& s, const V& i, const V& v, std::vector<Succ>& out) const {       // :245-252
    if (!eq(ap(s[state], i), Leader)) return;
    V entry = rec({{"term", ap(s[currentTerm], i)}, {"value", v}});
    State t = s; t[log] = except(s[log], i, append(ap(s[log], i), entry));
    out.push_back({t, A_ClientRequest});
  }
  void AdvanceCommitIndex(const State& s, const V& i, std::vector<Succ>& out) const {              // :258-275
    if (!eq(ap(s[state], i), Leader)) return;
    V li = ap(s[log], i);
    std::vector<V> agree;
    for (int64_t index = 1; index <= len(li); ++index) {
      std::vector<V> ag = {i};                                       // Agree(index) == {i} \cup {k : matchIndex[i][k] >= index}
      for (auto& k : Server->a) if (as_int(ap(ap(s[matchIndex], i), k)) >= index) ag.push_back(k);
      if (IsQuorum(set(ag))) agree.push_back(Int(index));
    }
    V agreeIndexes = set(agree);
    int64_t nci = as_int(ap(s[commitIndex], i));
    if (card(agreeIndexes) > 0 && eq(ap(ap(li, set_max(agreeIndexes)), "term"), ap(s[currentTerm], i)))
      nci = set_max(agreeIndexes);
    State t = s; t[commitIndex] = except(s[commitIndex], i, Int(nci));
    out.push_back({t, A_AdvanceCommitIndex});
  }
  // ---- message handlers, i = recipient, j = sender (raft_original.tla:283-435)
  void HandleRequestVoteRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const {  // :283-302
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
    t[messages] = WithoutMessage(m, WithMessage(resp, s[messages]));    // Reply (:128-129)
    out.push_back({t, A_HandleRequestVoteRequest});
  }
  void HandleRequestVoteResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :306-320
    if (!eq(ap(m, "mterm"), ap(s[currentTerm], i))) return;
    State t = s;
    t[votesResponded] = except(s[votesResponded], i, cup(ap(s[votesResponded], i), set({j})));
    if (as_bool(ap(m, "mvoteGranted"))) {
      t[votesGranted] = except(s[votesGranted], i, cup(ap(s[votesGranted], i), set({j})));
      t[voterLog] = except(s[voterLog], i, at_at(ap(s[voterLog], i), colon_gt(j, ap(m, "mlog"))));
    }
    t[messages] = WithoutMessage(m, s[messages]);                       // Discard (:125)
    out.push_back({t, A_HandleRequestVoteResponse});
  }
  void HandleAppendEntriesRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :326-388
    V li = ap(s[log], i);
    int64_t pli = as_int(ap(m, "mprevLogIndex"));
    bool logOk = pli == 0 ||
                 (pli > 0 && pli <= len(li) && eq(ap(m, "mprevLogTerm"), ap(ap(li, pli), "term")));
    int64_t mterm = as_int(ap(m, "mterm")), ct = as_int(ap(s[currentTerm], i));
    V st = ap(s[state], i);
    if (!(mterm <= ct)) return;
    // reject request
    if (mterm < ct || (mterm == ct && eq(st, Follower) && !logOk)) {
      V resp = rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(false)}, {"mmatchIndex", Int(0)},
                    {"msource", i}, {"mdest", j}});
      State t = s; t[messages] = WithoutMessage(m, WithMessage(resp, s[messages]));
      out.push_back({t, A_HandleAppendEntriesRequest});
    }
    // return to follower state
    if (mterm == ct && eq(st, Candidate)) {
      State t = s; t[state] = except(s[state], i, Follower);
      out.push_back({t, A_HandleAppendEntriesRequest});
    }
    // accept request
    if (mterm == ct && eq(st, Follower) && logOk) {
      int64_t index = pli + 1;
      V ents = ap(m, "mentries");
      // already done with request
      if (len(ents) == 0 ||
          (len(ents) > 0 && len(li) >= index && eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term")))) {
        State t = s;
        t[commitIndex] = except(s[commitIndex], i, ap(m, "mcommitIndex"));
        V resp = rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(true)},
                      {"mmatchIndex", Int(pli + len(ents))}, {"msource", i}, {"mdest", j}});
        t[messages] = WithoutMessage(m, WithMessage(resp, s[messages]));
        out.push_back({t, A_HandleAppendEntriesRequest});
      }
      // conflict: remove 1 entry
      if (len(ents) > 0 && len(li) >= index && !eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term"))) {
        std::vector<V> ks, vs;                                          // [index2 \in 1..(Len(log[i]) - 1) |-> log[i][index2]]
        for (int64_t q = 1; q <= len(li) - 1; ++q) { ks.push_back(Int(q)); vs.push_back(ap(li, q)); }
        State t = s; t[log] = except(s[log], i, fcn(ks, vs));
        out.push_back({t, A_HandleAppendEntriesRequest});
      }
      // no conflict: append entry
      if (len(ents) > 0 && len(li) == pli) {
        State t = s; t[log] = except(s[log], i, append(li, ap(ents, 1)));
        out.push_back({t, A_HandleAppendEntriesRequest});
      }
    }
  }
  void HandleAppendEntriesResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :392-402
    if (!eq(ap(m, "mterm"), ap(s[currentTerm], i))) return;
    State t = s;
    if (as_bool(ap(m, "msuccess"))) {
      t[nextIndex] = except(s[nextIndex], i, except(ap(s[nextIndex], i), j, Int(as_int(ap(m, "mmatchIndex")) + 1)));
      t[matchIndex] = except(s[matchIndex], i, except(ap(s[matchIndex], i), j, ap(m, "mmatchIndex")));
    } else {
      int64_t ni = as_int(ap(ap(s[nextIndex], i), j));
      t[nextIndex] = except(s[nextIndex], i, except(ap(s[nextIndex], i), j, Int(std::max<int64_t>(ni - 1, 1))));
    }
    t[messages] = WithoutMessage(m, s[messages]);
    out.push_back({t, A_HandleAppendEntriesResponse});
  }
  void UpdateTerm(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {           // :405-411
    if (!(as_int(ap(m, "mterm")) > as_int(ap(s[currentTerm], i)))) return;
    State t = s;
    t[currentTerm] = except(s[currentTerm], i, ap(m, "mterm"));
    t[state] = except(s[state], i, Follower);
    t[votedFor] = except(s[votedFor], i, Nil);
    out.push_back({t, A_UpdateTerm});
  }
  void DropStaleResponse(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {    // :414-417
    if (!(as_int(ap(m, "mterm")) < as_int(ap(s[currentTerm], i)))) return;
    State t = s; t[messages] = WithoutMessage(m, s[messages]);
    out.push_back({t, A_DropStaleResponse});
  }
  void Receive(const State& s, const V& m, std::vector<Succ>& out) const {                          // :420-435
    V i = ap(m, "mdest"), j = ap(m, "msource"), ty = ap(m, "mtype");
    UpdateTerm(s, i, m, out);
    if (eq(ty, RVReq)) HandleRequestVoteRequest(s, i, j, m, out);
    if (eq(ty, RVResp)) { DropStaleResponse(s, i, m, out); HandleRequestVoteResponse(s, i, j, m, out); }
    if (eq(ty, AEReq)) HandleAppendEntriesRequest(s, i, j, m, out);
    if (eq(ty, AEResp)) { DropStaleResponse(s, i, m, out); HandleAppendEntriesResponse(s, i, j, m, out); }
  }

  // ---- Next (raft_original.tla:453-464)
  void next(const State& s, std::vector<Succ>& out) const override {
    size_t base = out.size();
    for (auto& i : Server->a) Restart(s, i, out);
    for (auto& i : Server->a) Timeout(s, i, out);
    for (auto& i : Server->a) for (auto& j : Server->a) RequestVote(s, i, j, out);
    for (auto& i : Server->a) BecomeLeader(s, i, out);
    for (auto& i : Server->a) for (auto& v : Value->a) ClientRequest(s, i, v, out);
    for (auto& i : Server->a) AdvanceCommitIndex(s, i, out);
    for (auto& i : Server->a) for (auto& j : Server->a) AppendEntries(s, i, j, out);
    auto dom = domain_elems(s[messages]);
    for (auto& m : dom) Receive(s, m, out);
    for (auto& m : dom) { State t = s; t[messages] = WithMessage(m, s[messages]); out.push_back({t, A_DuplicateMessage}); }   // :442-444
    for (auto& m : dom) { State t = s; t[messages] = WithoutMessage(m, s[messages]); out.push_back({t, A_DropMessage}); }     // :447-449
    // /\ allLogs' = allLogs \cup {log[i] : i \in Server}   (G3: conjoined to every step)
    std::vector<V> logs;
    for (auto& i : Server->a) logs.push_back(ap(s[log], i));
    V al = cup(s[allLogs], set(logs));
    for (size_t q = base; q < out.size(); ++q) out[q].s[allLogs] = al;
  }

  // ---- MC wrapper constraints (configs/raft_original_mc.tla)
  bool constraint(const std::string& n, const State& s) const override {
    if (n == "BoundedTerms") { for (auto& i : Server->a) if (as_int(ap(s[currentTerm], i)) > MaxTerm) return false; return true; }
    if (n == "BoundedLogs") { for (auto& i : Server->a) if (len(ap(s[log], i)) > MaxLogLen) return false; return true; }
    if (n == "BoundedMessages") {
      auto dom = domain_elems(s[messages]);
      if ((int64_t)dom.size() > MaxMsgDomain) return false;
      for (auto& m : dom) { int64_t c = as_int(ap(s[messages], m)); if (c < MinMsgCount || c > MaxMsgCount) return false; }
      return true;
    }
    throw EvalError("unknown constraint " + n);
  }
  bool invariant(const std::string& n, const State& s) const override {
    if (n == "ElectionSafety") {       // \A e, f \in elections : e.eterm = f.eterm => e.eleader = f.eleader
      for (auto& e : s[elections]->a) for (auto& f : s[elections]->a)
        if (eq(ap(e, "eterm"), ap(f, "eterm")) && !eq(ap(e, "eleader"), ap(f, "eleader"))) return false;
      return true;
    }
    if (n == "LogMatching") {          // tlc_membership/raft.tla:1017-1021, restated over raft_original logs
      for (auto& i : Server->a) for (auto& j : Server->a) {
        V li = ap(s[log], i), lj = ap(s[log], j);
        int64_t n2 = std::min(len(li), len(lj));
        for (int64_t q = 1; q <= n2; ++q)
          if (eq(ap(ap(li, q), "term"), ap(ap(lj, q), "term")) && !eq(subseq(li, 1, q), subseq(lj, 1, q))) return false;
      }
      return true;
    }
    if (n == "NoLeader") {            // test-only scenario invariant: ~\E i : state[i] = Leader
      for (auto& i : Server->a) if (eq(ap(s[state], i), Leader)) return false;
      return true;
    }
    if (n == "NoCommit") {            // test-only scenario invariant: \A i : commitIndex[i] = 0
      for (auto& i : Server->a) if (as_int(ap(s[commitIndex], i)) != 0) return false;
      return true;
    }
    throw EvalError("unknown invariant " + n);
  }
};

}  // namespace oracle
