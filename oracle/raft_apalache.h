// ============================================================================
// TEST INFRASTRUCTURE ONLY (see oracle/tla.h header).
//
// Literal CPU restatement of apalache_no_membership/raft.tla (Ricketts' spec as annotated for the
// Apalache symbolic checker, with Pîrlea/Foo's history variable) over the explicit value model of
// tla.h, for its shipped raft.cfg (TLC syntax).  Every function cites the lines it follows.  This is
// the oracle the generated path's counts for that module are checked against (tests/test_tlagen.py,
// tests/test_gpu_tlagen.py): the product runs the module through its SANY-subset front end, this
// file restates it by hand.
//
// What differs from raft_dricketts.h (the same protocol):
//   * messages are wrapped records (WrapMsg :204-214): [wrapped, mtype, mterm, msource, mdest,
//     RVReq, RVResp, AEReq, AEResp], the unused halves filled with the Empty* records (:58-94); the
//     handlers receive the inner record (m.RVReq ...) and re-wrap it to discard it (:233-253);
//   * TypedBags (+)/(-) (TypedBags.tla:51-69): (-) drops an element whose count reaches 0;
//   * a history variable (:277-281): per-server restarted/timeout counters (Restart :303-305,
//     Timeout :318-320), the global action sequence (Send / Receive / Restart / Timeout records) and
//     hadAtLeastOneLeader (BecomeLeader :373); the constraints read it (:756-770);
//   * AdvanceCommitIndex ranges over 1..MaxLogLength (:398-410), so log[i][Max(agreeIndexes)] can be
//     outside the log: a TLC evaluation error, as here (ap throws);
//   * AppendEntriesAlreadyDone's UNCHANGED <<serverVars, logVars>> after commitIndex' (:489, :497,
//     logVars == <<log, commitIndex>> :147) is TLC's equality test, as in raft_dricketts.h;
//   * DuplicateMessage / DropMessage only when messages[m] = 1 (:621-628);
//   * ElectionSafety guards only empty logs (:691-699): Max({}) of a log without an entry of the
//     leader's term is an evaluation error.
// Action names follow TLC's split points as the generated path names them: Next's disjuncts, inside
// Receive (:577-592) UpdateTerm is a disjunct of its own and each `m.mtype = .. /\ ..` conjunction
// is Receive; the two `\E m : /\ messages[m] = 1 /\ ..` disjuncts are conjunctions, named Next.
// ============================================================================
#pragma once
#include "engine.h"

namespace oracle {

struct RaftApalache : Spec {
  // VARIABLE declaration order, apalache_no_membership/raft.tla:101-172
  enum { messages, history, currentTerm, state, votedFor, log, commitIndex, votesResponded, votesGranted, nextIndex, matchIndex, NVARS };
  enum { A_Next, A_Restart, A_Timeout, A_RequestVote, A_BecomeLeader, A_ClientRequest, A_AdvanceCommitIndex,
         A_AppendEntries, A_Receive, A_UpdateTerm, NACT };
  // MaxLogLength / MaxRestarts / MaxTimeouts (:19-21); MaxInFlightMessages (:22) = (2 |Server|)^2
  static constexpr int64_t MaxLogLength = 5, MaxRestarts = 2, MaxTimeouts = 2;

  const Cfg& cfg;
  V Server, Value, Follower, Candidate, Leader, Nil, RVReq, RVResp, AEReq, AEResp;
  V EmptyRVReqMsg, EmptyAEReqMsg, EmptyRVRespMsg, EmptyAERespMsg;
  std::vector<std::string> vn;

  explicit RaftApalache(const Cfg& c) : cfg(c) {
    Server = c.get("Server"); Value = c.get("Value");
    Follower = c.get("Follower"); Candidate = c.get("Candidate"); Leader = c.get("Leader");
    Nil = c.get("Nil");
    RVReq = c.get("RequestVoteRequest"); RVResp = c.get("RequestVoteResponse");
    AEReq = c.get("AppendEntriesRequest"); AEResp = c.get("AppendEntriesResponse");
    EmptyRVReqMsg = rec({{"mtype", RVReq}, {"mterm", Int(0)}, {"mlastLogTerm", Int(0)}, {"mlastLogIndex", Int(0)},   // :58-65
                         {"msource", Nil}, {"mdest", Nil}});
    EmptyAEReqMsg = rec({{"mtype", AEReq}, {"mterm", Int(0)}, {"mprevLogIndex", Int(0)}, {"mprevLogTerm", Int(0)},  // :67-76
                         {"mentries", empty_seq()}, {"mcommitIndex", Nil}, {"msource", Nil}, {"mdest", Nil}});
    EmptyRVRespMsg = rec({{"mtype", RVResp}, {"mterm", Nil}, {"mvoteGranted", Bool(false)}, {"mlog", empty_seq()}, // :78-85
                          {"msource", Nil}, {"mdest", Nil}});
    EmptyAERespMsg = rec({{"mtype", AEResp}, {"mterm", Int(0)}, {"msuccess", Bool(false)}, {"mmatchIndex", Int(0)}, // :87-94
                          {"msource", Nil}, {"mdest", Nil}});
    vn = {"messages", "history", "currentTerm", "state", "votedFor", "log", "commitIndex", "votesResponded", "votesGranted",
          "nextIndex", "matchIndex"};
  }
  const std::vector<std::string>& var_names() const override { return vn; }
  std::vector<std::string> action_names() const override {
    return {"Next", "Restart", "Timeout", "RequestVote", "BecomeLeader", "ClientRequest", "AdvanceCommitIndex",
            "AppendEntries", "Receive", "UpdateTerm"};
  }

  // ---- helpers (:187-260)
  V fnOver(const V& dom, const V& val) const { std::vector<V> ks = dom->a, vs(dom->a.size(), val); return fcn(ks, vs); }
  bool InQuorum(const V& s) const { return subseteq(s, Server) && card(s) * 2 > card(Server); }   // Quorum :187
  int64_t LastTerm(const V& xlog) const {                                                          // :191
    return len(xlog) == 0 ? 0 : as_int(ap(ap(xlog, len(xlog)), "term"));
  }
  // msgs (+) SetToBag({m}) (:196; TypedBags.tla:51-57)
  V WithMessage(const V& m, const V& msgs) const {
    if (in_domain(msgs, m)) return except(msgs, m, Int(as_int(ap(msgs, m)) + 1));
    return at_at(msgs, colon_gt(m, Int(1)));
  }
  // msgs (-) SetToBag({m}) (:201; TypedBags.tla:60-69: elements whose count drops to 0 leave the domain)
  V WithoutMessage(const V& m, const V& msgs) const {
    if (!in_domain(msgs, m)) return msgs;
    const int64_t c = as_int(ap(msgs, m));
    if (c > 1) return except(msgs, m, Int(c - 1));
    std::vector<V> ks, vs;
    for (auto& k : domain_elems(msgs)) if (!eq(k, m)) { ks.push_back(k); vs.push_back(ap(msgs, k)); }
    return fcn(ks, vs);
  }
  // WrapMsg (:204-214): an unwrapped record (no "wrapped" field) goes into the half of its type
  V WrapMsg(const V& m) const {
    if (in_domain(m, Str("wrapped"))) return m;
    const V ty = ap(m, "mtype");
    const bool rq = eq(ty, RVReq), rp = eq(ty, RVResp), aq = eq(ty, AEReq);
    return rec({{"wrapped", Bool(true)}, {"mtype", ty}, {"mterm", ap(m, "mterm")}, {"msource", ap(m, "msource")},
                {"mdest", ap(m, "mdest")}, {"RVReq", rq ? m : EmptyRVReqMsg}, {"RVResp", rp ? m : EmptyRVRespMsg},
                {"AEReq", aq ? m : EmptyAEReqMsg}, {"AEResp", (!rq && !rp && !aq) ? m : EmptyAERespMsg}});
  }
  V global_append(const V& h, const V& action) const { return except(h, "global", append(ap(h, "global"), action)); }
  // Send (:218-222): the wrapped message into the bag, a Send record onto history["global"]
  void Send(State& t, const V& m) const {
    const V w = WrapMsg(m);
    t[messages] = WithMessage(w, t[messages]);
    t[history] = global_append(t[history], rec({{"action", Str("Send")}, {"executedOn", ap(m, "msource")}, {"msg", w}}));
  }
  // Discard (:233-237)
  void Discard(State& t, const V& m) const {
    const V w = WrapMsg(m);
    t[messages] = WithoutMessage(w, t[messages]);
    t[history] = global_append(t[history], rec({{"action", Str("Receive")}, {"executedOn", ap(m, "mdest")}, {"msg", w}}));
  }
  // Reply (:247-253): WithoutMessage(wreq, WithMessage(wresp, messages)); Receive then Send appended
  void Reply(State& t, const V& response, const V& request) const {
    const V wreq = WrapMsg(request), wresp = WrapMsg(response);
    t[messages] = WithoutMessage(wreq, WithMessage(wresp, t[messages]));
    V h = global_append(t[history], rec({{"action", Str("Receive")}, {"executedOn", ap(request, "mdest")}, {"msg", wreq}}));
    t[history] = global_append(h, rec({{"action", Str("Send")}, {"executedOn", ap(response, "msource")}, {"msg", wresp}}));
  }
  // history["server"][i][field] + 1 (:303-304, :318-319)
  V bump_server(const V& h, const V& i, const char* field) const {
    const V srv = ap(h, "server"), si = ap(srv, i);
    return except(h, "server", except(srv, i, except(si, field, Int(as_int(ap(si, field)) + 1))));
  }

  // ---- Init (:265-288)
  std::vector<State> init() const override {
    State s(NVARS);
    s[messages] = fcn({}, {});   // EmptyBag == SetToBag({})
    s[history] = rec({{"server", fnOver(Server, rec({{"restarted", Int(0)}, {"timeout", Int(0)}}))},   // InitHistory :277-281
                      {"global", empty_seq()}, {"hadAtLeastOneLeader", Bool(false)}});
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

  // ---- actions (:296-411)
  void Restart(const State& s, const V& i, std::vector<Succ>& out) const {                          // :296-306
    State t = s;
    t[state] = except(s[state], i, Follower);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    t[commitIndex] = except(s[commitIndex], i, Int(0));
    t[history] = global_append(bump_server(s[history], i, "restarted"), rec({{"action", Str("Restart")}, {"executedOn", i}}));
    out.push_back({t, A_Restart});
  }
  void Timeout(const State& s, const V& i, std::vector<Succ>& out) const {                          // :310-321
    V st = ap(s[state], i);
    if (!(eq(st, Follower) || eq(st, Candidate))) return;
    State t = s;
    t[state] = except(s[state], i, Candidate);
    t[currentTerm] = except(s[currentTerm], i, Int(as_int(ap(s[currentTerm], i)) + 1));
    t[votedFor] = except(s[votedFor], i, Nil);
    t[votesResponded] = except(s[votesResponded], i, empty_set());
    t[votesGranted] = except(s[votesGranted], i, empty_set());
    t[history] = global_append(bump_server(s[history], i, "timeout"), rec({{"action", Str("Timeout")}, {"executedOn", i}}));
    out.push_back({t, A_Timeout});
  }
  void RequestVote(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {          // :325-334
    if (!eq(ap(s[state], i), Candidate)) return;
    if (in_set(j, ap(s[votesResponded], i))) return;
    V li = ap(s[log], i);
    State t = s;
    Send(t, rec({{"mtype", RVReq}, {"mterm", ap(s[currentTerm], i)}, {"mlastLogTerm", Int(LastTerm(li))},
                 {"mlastLogIndex", Int(len(li))}, {"msource", i}, {"mdest", j}}));
    out.push_back({t, A_RequestVote});
  }
  void AppendEntries(const State& s, const V& i, const V& j, std::vector<Succ>& out) const {        // :340-361
    if (eq(i, j)) return;
    if (!eq(ap(s[state], i), Leader)) return;
    V li = ap(s[log], i);
    int64_t ni = as_int(ap(ap(s[nextIndex], i), j));
    int64_t prevLogIndex = ni - 1;
    int64_t prevLogTerm = (prevLogIndex > 0 && prevLogIndex <= len(li)) ? as_int(ap(ap(li, prevLogIndex), "term")) : 0;
    int64_t lastEntry = std::min(len(li), ni);                 // Min({Len(log[i]), nextIndex[i][j]})
    V entries = subseq(li, ni, lastEntry);
    State t = s;
    Send(t, rec({{"mtype", AEReq}, {"mterm", ap(s[currentTerm], i)}, {"mprevLogIndex", Int(prevLogIndex)},
                 {"mprevLogTerm", Int(prevLogTerm)}, {"mentries", entries},
                 {"mcommitIndex", Int(std::min(as_int(ap(s[commitIndex], i)), lastEntry))}, {"msource", i}, {"mdest", j}}));
    out.push_back({t, A_AppendEntries});
  }
  void BecomeLeader(const State& s, const V& i, std::vector<Succ>& out) const {                     // :365-374
    if (!eq(ap(s[state], i), Candidate)) return;
    if (!InQuorum(ap(s[votesGranted], i))) return;
    State t = s;
    t[state] = except(s[state], i, Leader);
    t[nextIndex] = except(s[nextIndex], i, fnOver(Server, Int(len(ap(s[log], i)) + 1)));
    t[matchIndex] = except(s[matchIndex], i, fnOver(Server, Int(0)));
    t[history] = except(s[history], "hadAtLeastOneLeader", Bool(true));
    out.push_back({t, A_BecomeLeader});
  }
  void ClientRequest(const State& s, const V& i, const V& v, std::vector<Succ>& out) const {        // :378-385
    if (!eq(ap(s[state], i), Leader)) return;
    V entry = rec({{"term", ap(s[currentTerm], i)}, {"value", v}});
    State t = s; t[log] = except(s[log], i, append(ap(s[log], i), entry));
    out.push_back({t, A_ClientRequest});
  }
  void AdvanceCommitIndex(const State& s, const V& i, std::vector<Succ>& out) const {               // :392-411
    if (!eq(ap(s[state], i), Leader)) return;
    V li = ap(s[log], i);
    std::vector<V> agree;
    for (int64_t index = 1; index <= MaxLogLength; ++index) {   // agreeIndexes over 1..MaxLogLength (:400-401)
      std::vector<V> ag = {i};                                 // Agree(index) == {i} \cup {k : matchIndex[i][k] >= index}
      for (auto& k : Server->a) if (as_int(ap(ap(s[matchIndex], i), k)) >= index) ag.push_back(k);
      if (InQuorum(set(ag))) agree.push_back(Int(index));
    }
    V agreeIndexes = set(agree);
    int64_t nci = as_int(ap(s[commitIndex], i));
    // log[i][Max(agreeIndexes)] beyond Len(log[i]) raises TLC's evaluation error (ap throws)
    if (card(agreeIndexes) > 0 && eq(ap(ap(li, set_max(agreeIndexes)), "term"), ap(s[currentTerm], i)))
      nci = set_max(agreeIndexes);
    State t = s; t[commitIndex] = except(s[commitIndex], i, Int(nci));
    out.push_back({t, A_AdvanceCommitIndex});
  }

  // ---- message handlers, i = recipient, j = sender, m = the inner (unwrapped) record (:420-573)
  void HandleRequestVoteRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const {  // :420-439
    V li = ap(s[log], i);
    bool logOk = as_int(ap(m, "mlastLogTerm")) > LastTerm(li) ||
                 (as_int(ap(m, "mlastLogTerm")) == LastTerm(li) && as_int(ap(m, "mlastLogIndex")) >= len(li));
    V vf = ap(s[votedFor], i);
    bool grant = eq(ap(m, "mterm"), ap(s[currentTerm], i)) && logOk && (eq(vf, Nil) || eq(vf, j));
    if (!(as_int(ap(m, "mterm")) <= as_int(ap(s[currentTerm], i)))) return;
    State t = s;
    if (grant) t[votedFor] = except(s[votedFor], i, j);
    Reply(t, rec({{"mtype", RVResp}, {"mterm", ap(s[currentTerm], i)}, {"mvoteGranted", Bool(grant)},
                  {"mlog", li}, {"msource", i}, {"mdest", j}}), m);
    out.push_back({t, A_Receive});
  }
  void HandleRequestVoteResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :444-456
    if (!eq(ap(m, "mterm"), ap(s[currentTerm], i))) return;
    State t = s;
    t[votesResponded] = except(s[votesResponded], i, cup(ap(s[votesResponded], i), set({j})));
    if (as_bool(ap(m, "mvoteGranted"))) t[votesGranted] = except(s[votesGranted], i, cup(ap(s[votesGranted], i), set({j})));
    Discard(t, m);
    out.push_back({t, A_Receive});
  }
  void HandleAppendEntriesRequest(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :532-541
    V li = ap(s[log], i);
    int64_t pli = as_int(ap(m, "mprevLogIndex"));
    bool logOk = pli == 0 || (pli > 0 && pli <= len(li) && eq(ap(m, "mprevLogTerm"), ap(ap(li, pli), "term")));
    int64_t mterm = as_int(ap(m, "mterm")), ct = as_int(ap(s[currentTerm], i));
    V st = ap(s[state], i);
    if (!(mterm <= ct)) return;
    if (mterm < ct || (mterm == ct && eq(st, Follower) && !logOk)) {                                // Reject (:459-471)
      State t = s;
      Reply(t, rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(false)}, {"mmatchIndex", Int(0)},
                    {"msource", i}, {"mdest", j}}), m);
      out.push_back({t, A_Receive});
    }
    if (mterm == ct && eq(st, Candidate)) {                                                          // ReturnToFollowerState (:474-478)
      State t = s; t[state] = except(s[state], i, Follower);
      out.push_back({t, A_Receive});
    }
    if (mterm == ct && eq(st, Follower) && logOk) {                                                  // Accept (:517-525)
      int64_t index = pli + 1;
      V ents = ap(m, "mentries");
      // AlreadyDone (:481-497): UNCHANGED <<serverVars, logVars>> after commitIndex' is TLC's test of
      // commitIndex' = commitIndex (logVars == <<log, commitIndex>> :147)
      if ((len(ents) == 0 || (len(li) >= index && eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term")))) &&
          eq(ap(m, "mcommitIndex"), ap(s[commitIndex], i))) {
        State t = s;
        t[commitIndex] = except(s[commitIndex], i, ap(m, "mcommitIndex"));
        Reply(t, rec({{"mtype", AEResp}, {"mterm", Int(ct)}, {"msuccess", Bool(true)},
                      {"mmatchIndex", Int(pli + len(ents))}, {"msource", i}, {"mdest", j}}), m);
        out.push_back({t, A_Receive});
      }
      if (len(ents) > 0 && len(li) >= index && !eq(ap(ap(li, index), "term"), ap(ap(ents, 1), "term"))) {     // Conflict (:500-507)
        State t = s; t[log] = except(s[log], i, subseq(li, 1, len(li) - 1));
        out.push_back({t, A_Receive});
      }
      if (len(ents) > 0 && len(li) == pli) {                                                          // NoConflict (:510-514)
        State t = s; t[log] = except(s[log], i, append(li, ap(ents, 1)));
        out.push_back({t, A_Receive});
      }
    }
  }
  void HandleAppendEntriesResponse(const State& s, const V& i, const V& j, const V& m, std::vector<Succ>& out) const { // :546-556
    if (!eq(ap(m, "mterm"), ap(s[currentTerm], i))) return;
    State t = s;
    if (as_bool(ap(m, "msuccess"))) {
      t[nextIndex] = except(s[nextIndex], i, except(ap(s[nextIndex], i), j, Int(as_int(ap(m, "mmatchIndex")) + 1)));
      t[matchIndex] = except(s[matchIndex], i, except(ap(s[matchIndex], i), j, ap(m, "mmatchIndex")));
    } else {
      int64_t ni = as_int(ap(ap(s[nextIndex], i), j));
      t[nextIndex] = except(s[nextIndex], i, except(ap(s[nextIndex], i), j, Int(std::max<int64_t>(ni - 1, 1))));
    }
    Discard(t, m);
    out.push_back({t, A_Receive});
  }
  void UpdateTerm(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {            // :560-566 (m wrapped)
    if (!(as_int(ap(m, "mterm")) > as_int(ap(s[currentTerm], i)))) return;
    State t = s;
    t[currentTerm] = except(s[currentTerm], i, ap(m, "mterm"));
    t[state] = except(s[state], i, Follower);
    t[votedFor] = except(s[votedFor], i, Nil);
    out.push_back({t, A_UpdateTerm});
  }
  void DropStaleResponse(const State& s, const V& i, const V& m, std::vector<Succ>& out) const {     // :570-573
    if (!(as_int(ap(m, "mterm")) < as_int(ap(s[currentTerm], i)))) return;
    State t = s; Discard(t, m);
    out.push_back({t, A_Receive});
  }
  void Receive(const State& s, const V& m, std::vector<Succ>& out) const {                          // :577-592 (m wrapped)
    V i = ap(m, "mdest"), j = ap(m, "msource"), ty = ap(m, "mtype");
    UpdateTerm(s, i, m, out);
    if (eq(ty, RVReq)) HandleRequestVoteRequest(s, i, j, ap(m, "RVReq"), out);
    if (eq(ty, RVResp)) { DropStaleResponse(s, i, ap(m, "RVResp"), out); HandleRequestVoteResponse(s, i, j, ap(m, "RVResp"), out); }
    if (eq(ty, AEReq)) HandleAppendEntriesRequest(s, i, j, ap(m, "AEReq"), out);
    if (eq(ty, AEResp)) { DropStaleResponse(s, i, ap(m, "AEResp"), out); HandleAppendEntriesResponse(s, i, j, ap(m, "AEResp"), out); }
  }

  // ---- Next (:612-628)
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
    for (auto& m : dom)                                         // DuplicateMessage (:600-602): SendWithoutHistory (:226-228)
      if (as_int(ap(s[messages], m)) == 1) { State t = s; t[messages] = WithMessage(WrapMsg(m), s[messages]); out.push_back({t, A_Next}); }
    for (auto& m : dom)                                         // DropMessage (:606-608): DiscardWithoutHistory (:241-243)
      if (as_int(ap(s[messages], m)) == 1) { State t = s; t[messages] = WithoutMessage(WrapMsg(m), s[messages]); out.push_back({t, A_Next}); }
  }

  // ---- constraints (:756-770)
  int64_t srv(const State& s, const V& i, const char* f) const { return as_int(ap(ap(ap(s[history], "server"), i), f)); }
  bool uncontested(const State& s) const {                      // ElectionsUncontested :764
    int64_t c = 0;
    for (auto& i : domain_elems(s[state])) if (eq(ap(s[state], i), Candidate)) ++c;
    return c <= 1;
  }
  bool constraint(const std::string& n, const State& s) const override {
    if (n == "BoundedInFlightMessages") {                       // BagCardinality(messages) <= MaxInFlightMessages :756, :22
      int64_t total = 0;
      for (auto& m : domain_elems(s[messages])) total += as_int(ap(s[messages], m));
      const int64_t card2 = 2 * card(Server);
      return total <= card2 * card2;
    }
    if (n == "BoundedLogSize") { for (auto& i : Server->a) if (len(ap(s[log], i)) > MaxLogLength) return false; return true; }
    if (n == "BoundedRestarts") { for (auto& i : Server->a) if (srv(s, i, "restarted") > MaxRestarts) return false; return true; }
    if (n == "BoundedTimeouts") { for (auto& i : Server->a) if (srv(s, i, "timeout") > MaxTimeouts) return false; return true; }
    if (n == "ElectionsUncontested") return uncontested(s);
    if (n == "CleanFirstLeaderElection") {                      // :766-770
      if (as_bool(ap(s[history], "hadAtLeastOneLeader"))) return true;
      for (auto& i : Server->a) if (srv(s, i, "restarted") != 0) return false;
      for (auto& i : Server->a) if (srv(s, i, "restarted") > 1) return false;
      return uncontested(s);
    }
    throw EvalError("unknown constraint " + n);
  }

  // ---- invariants (:654-750)
  V Committed(const State& s, const V& i) const { return subseq(ap(s[log], i), 1, as_int(ap(s[commitIndex], i))); }   // :654
  bool invariant(const std::string& n, const State& s) const override {
    if (n == "LeaderVotesQuorum") {                             // :672-676
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
    if (n == "CandidateTermNotInLog") {                         // :680-686
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
    if (n == "ElectionSafety") {                                // :691-699
      for (auto& i : Server->a) {
        if (!eq(ap(s[state], i), Leader)) continue;
        const V ti = ap(s[currentTerm], i);
        auto max_of_term = [&](const V& k) {                    // Max({n \in DOMAIN log[k] : log[k][n].term = currentTerm[i]})
          V lk = ap(s[log], k);
          std::vector<V> ns;
          for (int64_t q = 1; q <= len(lk); ++q) if (eq(ap(ap(lk, q), "term"), ti)) ns.push_back(Int(q));
          return set_max(set(ns));                              // Max({}): TLC's evaluation error
        };
        for (auto& j : Server->a) {
          if (len(ap(s[log], i)) == 0 || len(ap(s[log], j)) == 0) continue;
          if (!(max_of_term(i) >= max_of_term(j))) return false;
        }
      }
      return true;
    }
    if (n == "LogMatching") {                                   // :702-706
      for (auto& i : Server->a) for (auto& j : Server->a) {
        V li = ap(s[log], i), lj = ap(s[log], j);
        int64_t n2 = std::min(len(li), len(lj));
        for (int64_t q = 1; q <= n2; ++q)
          if (eq(ap(ap(li, q), "term"), ap(ap(lj, q), "term")) && !eq(subseq(li, 1, q), subseq(lj, 1, q))) return false;
      }
      return true;
    }
    if (n == "VotesGrantedInv") {                               // :715-723
      for (auto& i : Server->a)
        for (auto& j : ap(s[votesGranted], i)->a)
          if (eq(ap(s[currentTerm], i), ap(s[currentTerm], j)) && !is_prefix(Committed(s, j), ap(s[log], i))) return false;
      return true;
    }
    if (n == "QuorumLogInv") {                                  // :727-731
      for (auto& i : Server->a) {
        const V ci = Committed(s, i);
        for (auto& S : subsets(Server)) {
          if (!InQuorum(S)) continue;
          bool any = false;
          for (auto& j : S->a) if (is_prefix(ci, ap(s[log], j))) { any = true; break; }
          if (!any) return false;
        }
      }
      return true;
    }
    if (n == "MoreUpToDateCorrect") {                           // :737-742
      for (auto& i : Server->a) for (auto& j : Server->a) {
        V li = ap(s[log], i), lj = ap(s[log], j);
        const bool upto = LastTerm(li) > LastTerm(lj) || (LastTerm(li) == LastTerm(lj) && len(li) >= len(lj));
        if (upto && !is_prefix(Committed(s, j), li)) return false;
      }
      return true;
    }
    if (n == "LeaderCompleteness") {                            // :746-750
      for (auto& i : Server->a) {
        if (!eq(ap(s[state], i), Leader)) continue;
        for (auto& j : Server->a) if (!is_prefix(Committed(s, j), ap(s[log], i))) return false;
      }
      return true;
    }
    if (n == "BoundedTrace") return len(ap(s[history], "global")) <= 12;   // :776
    if (n == "FirstBecomeLeader") {                             // :778-785
      const V g = ap(s[history], "global");
      auto rv_resp_received = [&](const V& x) { return eq(ap(x, "action"), Str("Receive")) && eq(ap(ap(x, "msg"), "mtype"), RVResp); };
      for (int64_t i = 1; i <= len(g); ++i)
        for (int64_t j = 1; j <= len(g); ++j) {
          if (i == j) continue;
          const V x = ap(g, i), y = ap(g, j);
          if (rv_resp_received(x) && rv_resp_received(y) && !eq(ap(ap(x, "msg"), "msource"), ap(ap(y, "msg"), "msource")) &&
              eq(ap(s[state], ap(ap(x, "msg"), "mdest")), Leader))
            return false;
        }
      return true;
    }
    throw EvalError("unknown invariant " + n);
  }
};

}  // namespace oracle
