// ============================================================================
// TEST INFRASTRUCTURE ONLY (see oracle/tla.h header).
//
// Literal CPU restatement of thirdparty/raft_dricketts.tla (Daniel Ricketts' TLAPS-proved copy of
// Ongaro's spec, module `raft`) over the explicit value model of tla.h.  Every function cites the
// lines it follows.  The reference ships no TLC cfg for it; the model-checking wrapper operators
// (bounds, NoLeader) follow configs/ricketts_mc.tla.  This is the oracle the generated path's
// Ricketts counts are checked against (tests/test_tlagen.py): the product runs the module through
// its SANY-subset front end, this file restates it by hand.
//
// Differences from raft_original.h that matter for the counts: `messages` is a Bags-module bag
// (WithoutMessage drops an element whose count reaches 0, raft_dricketts.tla:92), no history
// variables (elections, allLogs, voterLog), AppendEntries guards prevLogTerm and carries no mlog
// (:171-192), AppendEntriesAlreadyDone's UNCHANGED covers commitIndex (below), and the invariants
// are the spec's own (:1032-1135).  The AlreadyDone rule was first restated as in raft_original.h;
// the whole-space comparison with the generated path (which follows TLC's reading of UNCHANGED)
// found 6 states apart at depth 18, and TLC's semantics decide for the generated path.
// ============================================================================
#pragma once
#include "engine.h"

namespace oracle {

struct RaftRicketts : Spec {
  // VARIABLE declaration order, raft_dricketts.tla:31-67
  enum { messages, currentTerm, state, votedFor, log, commitIndex, votesResponded, votesGranted, nextIndex, matchIndex, NVARS };
  // action ids: Next's disjuncts (raft_dricketts.tla:421-430) as the generated path names TLC's
  // split points — inside Receive (:388-403) UpdateTerm is a disjunct of its own, each
  // `m.mtype = .. /\ Handle..` conjunction is named Receive
  enum { A_Restart, A_Timeout, A_RequestVote, A_BecomeLeader, A_ClientRequest, A_AdvanceCommitIndex,
         A_AppendEntries, A_Receive, A_UpdateTerm, A_DuplicateMessage, A_DropMessage, NACT };

  const Cfg& cfg;
  V Server, Value, Follower, Candidate, Leader, Nil, RVReq, RVResp, AEReq, AEResp;
  int64_t MaxTerm = 0, MaxLogLen = 0, MaxMsgs = 0;
  std::vector<std::string> vn;

  explicit RaftRicketts(const Cfg& c) : cfg(c) {
    Server = c.get("Server"); Value = c.get("Value");
    Follower = c.get("Follower"); Candidate = c.get("Candidate"); Leader = c.get("Leader");
    Nil = c.get("Nil");
    RVReq = c.get("RequestVoteRequest"); RVResp = c.get("RequestVoteResponse");
    AEReq = c.get("AppendEntriesRequest"); AEResp = c.get("AppendEntriesResponse");
    auto opt = [&](const char* n, int64_t& dst) { if (c.has(n)) dst = as_int(c.get(n)); };
    opt("MaxTerm", MaxTerm); opt("MaxLogLen", MaxLogLen); opt("MaxMsgs", MaxMsgs);
    vn = {"messages", "currentTerm", "state", "votedFor", "log", "commitIndex", "votesResponded", "votesGranted",
          "nextIndex", "matchIndex"};
  }
  const std::vector<std::string>& var_names() const override { return vn; }
  std::vector<std::string> action_names() const override {
    return {"Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex",
            "AppendEntries", "Receive", "UpdateTerm", "DuplicateMessage", "DropMessage"};
  }

  // ---- helpers (raft_dricketts.tla:79-108)
  V fnOver(const V& dom, const V& val) const { std::vector<V> ks = dom->a, vs(dom->a.size(), val); return fcn(ks, vs); }
  bool InQuorum(const V& s) const { return subseteq(s, Server) && card(s) * 2 > card(Server); }   // :81
  int64_t LastTerm(const V& xlog) const {                                                          // :84
    return len(xlog) == 0 ? 0 : as_int(ap(ap(xlog, len(xlog)), "term"));
  }
  // msgs (+) SetToBag({m}) (:88; Bags: B1 (+) B2 adds the counts over DOMAIN B1 \cup DOMAIN B2)
  V WithMessage(const V& m, const V& msgs) const {
    if (in_domain(msgs, m)) return except(msgs, m, Int(as_int(ap(msgs, m)) + 1));
    return at_at(msgs, colon_gt(m, Int(1)));
  }
  // msgs (-) SetToBag({m}) (:92; Bags: B1 (-) B2 keeps only the elements whose count stays > 0)
  V WithoutMessage(const V& m, const V& msgs) const {
    if (!in_domain(msgs, m)) return msgs;
    const int64_t c = as_int(ap(msgs, m));
    if (c > 1) return except(msgs, m, Int(c - 1));
    std::vector<V> ks, vs;
    for (auto& k : domain_elems(msgs)) if (!eq(k, m)) { ks.push_back(k); vs.push_back(ap(msgs, k)); }
    return fcn(ks, vs);
  }
  V Reply(const V& resp, const V& req, const V& msgs) const { return WithoutMessage(req, WithMessage(resp, msgs)); }   // :102-103

  // ---- Init (raft_dricketts.tla:113-129)
  std::vector<State> init() const override {
    State s(NVARS);
    s[messages] = fcn({}, {});   // EmptyBag
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

  // ---- actions
  void Restart(const State& s, const V& i, std::vector<Succ>& out) const {                          // :136-143
    State t = s;
    t[state] = except(s[state], i, Follower);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    t[commitIndex] = except(s[commitIndex], i, Int(0));
    out.push_back({t, A_Restart});
  }
  void Timeout(const State& s, const V& i, std::vector<Succ>& out) const {                          // :146-154
    V st = ap(s[state], i);
    if (!(eq(st, Follower) || eq(st, Candidate))) return;
    State t = s;
    t[state] = except(s[state], i, Candidate);
    t[currentTerm] = except(s[currentTerm], i, Int(as_int(ap(s[currentTerm], i)) + 1));
    t[votedFor] = except(s[votedFor], i, Nil);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    out.push_back({t, A_Timeout});
  }
  void RequestVote(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {          // :157-166
    if (!eq(ap(s[state], i), Candidate)) return;
    if (in_set(j, ap(s[votesResponded], i))) return;
    V li = ap(s[log], i);
    V m = rec({{"mtype", RVReq}, {"mterm", ap(s[currentTerm], i)}, {"mlastLogTerm", Int(LastTerm(li))},
               {"mlastLogIndex", Int(len(li))}, {"msource", i}, {"mdest", j}});
    State t = s; t[messages] = WithMessage(m, s[messages]);
    out.push_back({t, A_RequestVote});
  }
  void AppendEntries(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {        // :171-192
    if (eq(i, j)) return;
    if (!eq(ap(s[state], i), Leader)) return;
    V li = ap(s[log], i);
    int64_t ni = as_int(ap(ap(s[nextIndex], i), j));
    int64_t prevLogIndex = ni - 1;
    int64_t prevLogTerm = (prevLogIndex > 0 && prevLogIndex <= len(li)) ? as_int(ap(ap(li, prevLogIndex), "term")) : 0;
    int64_t lastEntry = std::min(len(li), ni);                 // Min({Len(log[i]), nextIndex[i][j]})
    V entries = subseq(li, ni, lastEntry);
    V m = rec({{"mtype", AEReq}, {"mterm", ap(s[currentTerm], i)}, {"mprevLogIndex", Int(prevLogIndex)},
               {"mprevLogTerm", Int(prevLogTerm)}, {"mentries", entries},
               {"mcommitIndex", Int(std::min(as_int(ap(s[commitIndex], i)), lastEntry))}, {"msource", i}, {"mdest", j}});
    State t = s; t[messages] = WithMessage(m, s[messages]);
    out.push_back({t, A_AppendEntries});
  }
  void BecomeLeader(const State& s, const V& i, std::vector<Succ>& out) const {                     // :195-203
    if (!eq(ap(s[state], i), Candidate)) return;
    if (!InQuorum(ap(s[votesGranted], i))) return;
    State t = s;
    t[state] = except(s[state], i, Leader);
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(len(ap(s[log], i)) + 1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    out.push_back({t, A_BecomeLeader});
  }
  void ClientRequest(const State& s, const V& i, const V& v, std::vector<Succ>& out) const {        // :206-213
    if (!eq(ap(s[state], i), Leader)) return;
    V entry = rec({{"term", ap(s[currentTerm], i)}, {"value", v}});
    State t = s; t[log] = except(s[log], i, append(ap(s[log], i), entry));
    out.push_back({t, A_ClientRequest});
  }
  void AdvanceCommitIndex(const State& s, const V& i, std::vector<Succ>& out) const {               // :219-236
    if (!eq(ap(s[state], i), Leader)) return;
    V li = ap(s[log], i);
    std::vector<V> agree;
    for (int64_t index = 1; index <= len(li); ++index) {
      std::vector<V> ag = {i};                                 // Agree(index) == {i} \cup {k : matchIndex[i][k] >= index}
      for (auto& k : Server->a) if (as_int(ap(ap(s[matchIndex], i), k)) >= index) ag.push_back(k);
      if (InQuorum(set(ag))) agree.push_back(Int(index));
    }
    V agreeIndexes = set(agree);
    int64_t nci = as_int(ap(s[commitIndex], i));
    if (card(agreeIndexes) > 0 && eq(ap(ap(li, set_max(agreeIndexes)), "term"), ap(s[currentTerm], i)))
      nci = set_max(agreeIndexes);
    State t = s; t[commitIndex] = except(s[commitIndex], i, Int(nci));
    out.push_back({t, A_AdvanceCommitIndex});
  }
  // ---- message handlers, i = recipient, j = sender (raft_dricketts.tla:244-403)
  void HandleRequestVoteRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const {  // :244-263
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
    t[messages] = Reply(resp, m, s[messages]);
    out.push_back({t, A_Receive});
  }
  void HandleRequestVoteResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :267-279
    if (!eq(ap(m, "mterm"), ap(s[currentTerm], i))) return;
    State t = s;
    t[votesResponded] = except(s[votesResponded], i, cup(ap(s[votesResponded], i), set({j})));
    if (as_bool(ap(m, "mvoteGranted"))) t[votesGranted] = except(s[votesGranted], i, cup(ap(s[votesGranted], i), set({j})));
    t[messages] = WithoutMessage(m, s[messages]);                 // Discard (:99)
    out.push_back({t, A_Receive});
  }
  void HandleAppendEntriesRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :347-356
    V li = ap(s[log], i);
    int64_t pli = as_int(ap(m, "mprevLogIndex"));
    bool logOk = pli == 0 || (pli > 0 && pli <= len(li) && eq(ap(m, "mprevLogTerm"), ap(ap(li, pli), "term")));
    int64_t mterm = as_int(ap(m, "mterm")), ct = as_int(ap(s[currentTerm], i));
    V st = ap(s[state], i);
    if (!(mterm <= ct)) return;
    if (mterm < ct || (mterm == ct && eq(st, Follower) && !logOk)) {                                // Reject (:281-293)
      V resp = rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(false)}, {"mmatchIndex", Int(0)},
                    {"msource", i}, {"mdest", j}});
      State t = s; t[messages] = Reply(resp, m, s[messages]);
      out.push_back({t, A_Receive});
    }
    if (mterm == ct && eq(st, Candidate)) {                                                          // ReturnToFollowerState (:295-299)
      State t = s; t[state] = except(s[state], i, Follower);
      out.push_back({t, A_Receive});
    }
    if (mterm == ct && eq(st, Follower) && logOk) {                                                  // Accept (:333-341)
      int64_t index = pli + 1;
      V ents = ap(m, "mentries");
      // AlreadyDone (:301-317).  It assigns commitIndex' and then asserts UNCHANGED <<serverVars,
      // logVars>> with logVars == <<log, commitIndex>> (:51): under TLC that conjunct is a test of
      // commitIndex' = commitIndex, so the step exists only when m.mcommitIndex equals the
      // follower's commitIndex (Ongaro's raft_original.tla leaves commitIndex out of the UNCHANGED)
      if ((len(ents) == 0 || (len(li) >= index && eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term")))) &&
          eq(ap(m, "mcommitIndex"), ap(s[commitIndex], i))) {
        State t = s;
        t[commitIndex] = except(s[commitIndex], i, ap(m, "mcommitIndex"));
        V resp = rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(true)},
                      {"mmatchIndex", Int(pli + len(ents))}, {"msource", i}, {"mdest", j}});
        t[messages] = Reply(resp, m, s[messages]);
        out.push_back({t, A_Receive});
      }
      if (len(ents) > 0 && len(li) >= index && !eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term"))) {     // Conflict (:319-325)
        std::vector<V> ks, vs;                                   // [index2 \in 1..(Len(log[i]) - 1) |-> log[i][index2]]
        for (int64_t q = 1; q <= len(li) - 1; ++q) { ks.push_back(Int(q)); vs.push_back(ap(li, q)); }
        State t = s; t[log] = except(s[log], i, fcn(ks, vs));
        out.push_back({t, A_Receive});
      }
      if (len(ents) > 0 && len(li) == pli) {                                                          // NoConflict (:327-331)
        State t = s; t[log] = except(s[log], i, append(li, ap(ents, 1)));
        out.push_back({t, A_Receive});
      }
    }
  }
  void HandleAppendEntriesResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :360-370
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
    out.push_back({t, A_Receive});
  }
  void UpdateTerm(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {            // :373-379
    if (!(as_int(ap(m, "mterm")) > as_int(ap(s[currentTerm], i)))) return;
    State t = s;
    t[currentTerm] = except(s[currentTerm], i, ap(m, "mterm"));
    t[state] = except(s[state], i, Follower);
    t[votedFor] = except(s[votedFor], i, Nil);
    out.push_back({t, A_UpdateTerm});
  }
  void DropStaleResponse(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {     // :382-385
    if (!(as_int(ap(m, "mterm")) < as_int(ap(s[currentTerm], i)))) return;
    State t = s; t[messages] = WithoutMessage(m, s[messages]);
    out.push_back({t, A_Receive});
  }
  void Receive(const State& s, const V& m, std::vector<Succ>& out) const {                          // :388-403
    V i = ap(m, "mdest"), j = ap(m, "msource"), ty = ap(m, "mtype");
    UpdateTerm(s, i, m, out);
    if (eq(ty, RVReq)) HandleRequestVoteRequest(s, i, j, m, out);
    if (eq(ty, RVResp)) { DropStaleResponse(s, i, m, out); HandleRequestVoteResponse(s, i, j, m, out); }
    if (eq(ty, AEReq)) HandleAppendEntriesRequest(s, i, j, m, out);
    if (eq(ty, AEResp)) { DropStaleResponse(s, i, m, out); HandleAppendEntriesResponse(s, i, j, m, out); }
  }

  // ---- Next (raft_dricketts.tla:421-430)
  void next(const State& s, std::vector<Succ>& out) const override {
    for (auto& i : Server->a) Restart(s, i, out);
    for (auto& i : Server->a) Timeout(s, i, out);
    for (auto& i : Server->a) for (auto& j : Server->a) RequestVote(s, i, j, out);
    for (auto& i : Server->a) BecomeLeader(s, i, out);
    for (auto& i : Server->a) for (auto& v : Value->a) ClientRequest(s, i, v, out);
    for (auto& i : Server->a) AdvanceCommitIndex(s, i, out);
    for (auto& i : Server->a) for (auto& j : Server->a) AppendEntries(s, i, j, out);
    auto dom = domain_elems(s[messages]);
    for (auto& m : dom) Receive(s, m, out);
    for (auto& m : dom) { State t = s; t[messages] = WithMessage(m, s[messages]); out.push_back({t, A_DuplicateMessage}); }   // :410-412
    for (auto& m : dom) { State t = s; t[messages] = WithoutMessage(m, s[messages]); out.push_back({t, A_DropMessage}); }     // :415-417
  }

  // ---- MC wrapper constraints (configs/ricketts_mc.tla)
  bool constraint(const std::string& n, const State& s) const override {
    if (n == "BoundedTerms") { for (auto& i : Server->a) if (as_int(ap(s[currentTerm], i)) > MaxTerm) return false; return true; }
    if (n == "BoundedLogs") { for (auto& i : Server->a) if (len(ap(s[log], i)) > MaxLogLen) return false; return true; }
    if (n == "BoundedMessages") {                              // BagCardinality(messages) <= MaxMsgs
      int64_t total = 0;
      for (auto& m : domain_elems(s[messages])) total += as_int(ap(s[messages], m));
      return total <= MaxMsgs;
    }
    throw EvalError("unknown constraint " + n);
  }
  // {n \in DOMAIN log[k] : log[k][n].term = t}, then Max of it (an error on {}: CHOOSE over {})
  int64_t MaxIndexOfTerm(const State& s, const V& k, const V& t) const {
    V lk = ap(s[log], k);
    std::vector<V> ns;
    for (int64_t n = 1; n <= len(lk); ++n) if (eq(ap(ap(lk, n), "term"), t)) ns.push_back(Int(n));
    return set_max(set(ns));
  }
  bool invariant(const std::string& n, const State& s) const override {
    if (n == "ElectionSafety") {                               // :1123-1128
      for (auto& i : Server->a) {
        if (!eq(ap(s[state], i), Leader)) continue;
        const V ti = ap(s[currentTerm], i);
        for (auto& j : Server->a)
          if (!(MaxIndexOfTerm(s, i, ti) >= MaxIndexOfTerm(s, j, ti))) return false;
      }
      return true;
    }
    if (n == "LogMatching") {                                  // :1131-1135
      for (auto& i : Server->a) for (auto& j : Server->a) {
        V li = ap(s[log], i), lj = ap(s[log], j);
        int64_t n2 = std::min(len(li), len(lj));
        for (int64_t q = 1; q <= n2; ++q)
          if (eq(ap(ap(li, q), "term"), ap(ap(lj, q), "term")) && !eq(subseq(li, 1, q), subseq(lj, 1, q))) return false;
      }
      return true;
    }
    if (n == "LeaderVotesQuorum") {                            // :1032-1036
      for (auto& i : Server->a) {
        if (!eq(ap(s[state], i), Leader)) continue;
        const int64_t ti = as_int(ap(s[currentTerm], i));
        std::vector<V> js;
        for (auto& j : Server->a) {
          const int64_t tj = as_int(ap(s[currentTerm], j));
          if (tj > ti || (tj == ti && eq(ap(s[votedFor], j), i))) js.push_back(j);
        }
        if (!InQuorum(set(js))) return false;
      }
      return true;
    }
    if (n == "CandidateTermNotInLog") {                        // :1040-1046
      for (auto& i : Server->a) {
        if (!eq(ap(s[state], i), Candidate)) continue;
        const V ti = ap(s[currentTerm], i);
        std::vector<V> js;
        for (auto& j : Server->a)
          if (eq(ap(s[currentTerm], j), ti) && (eq(ap(s[votedFor], j), i) || eq(ap(s[votedFor], j), Nil))) js.push_back(j);
        if (!InQuorum(set(js))) continue;
        for (auto& j : Server->a) {
          V lj = ap(s[log], j);
          for (int64_t q = 1; q <= len(lj); ++q) if (eq(ap(ap(lj, q), "term"), ti)) return false;
        }
      }
      return true;
    }
    if (n == "NoLeader") {                                     // configs/ricketts_mc.tla
      for (auto& i : Server->a) if (eq(ap(s[state], i), Leader)) return false;
      return true;
    }
    throw EvalError("unknown invariant " + n);
  }
};

}  // namespace oracle
