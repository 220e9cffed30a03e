// raftmc host: encode the golden history trace of a punctuated-search constraint
// (tlc_membership/raft.tla:1198-1204 CommitWhenConcurrentLeaders_unique over the
// ConcurrentLeaders trace :1201, :1228-1234 MajorityOfClusterRestarts_constraint over
// the CommitWhenConcurrentLeaders trace :1231) into the device table the expand
// kernels compare appended history entries against (memb_spec.h prefix_step).
//
//   \E s1, s2, s3 \in Server : Cardinality({s1, s2, s3}) = 3 /\
//       IsPrefix(SubSeq(trace, 1, Min(Len(trace), Len(history["global"]))), history["global"])
//
// One row per trace position, one (x, y) pair per binding of (s1, s2, s3) to distinct
// servers, in lexicographic order of the server indices.  An entry that no history entry
// can equal under a binding (a field outside the compiled domains, a record of another
// shape) is encoded as (~0, ~0), which never matches.
#pragma once
#include <algorithm>
#include <array>
#include <string>
#include <vector>

#include "../../include/raftmc.h"

#include "memb_text.h"
#include "tla_value.h"

namespace rmc {

template <class S>
struct MembPrefix {
  const MembModel& m;
  int ph[3];   // servers bound to s1, s2, s3
  mutable bool ok = true;

  static std::vector<std::string> names(std::initializer_list<const char*> xs) {
    std::vector<std::string> v(xs.begin(), xs.end());
    std::sort(v.begin(), v.end());
    return v;
  }
  int server(const TVal* v) const {
    if (!v || v->kind != TVal::MV) { ok = false; return 0; }
    if (v->s == "s1") return ph[0];
    if (v->s == "s2") return ph[1];
    if (v->s == "s3") return ph[2];
    for (int k = 0; k < m.N; ++k) if (m.server[k] == v->s) return k;
    ok = false;
    return 0;
  }
  int integer(const TVal* v) const {
    if (!v || v->kind != TVal::Int) { ok = false; return 0; }
    return (int)v->i;
  }
  bool boolean(const TVal* v) const {
    if (!v || v->kind != TVal::Bool) { ok = false; return false; }
    return v->i != 0;
  }
  u32 server_mask(const TVal* v) const {
    if (!v || v->kind != TVal::Set) { ok = false; return 0; }
    u32 mask = 0;
    for (auto& e : v->elems) mask |= 1u << server(&e);
    return mask;
  }
  bool shape(const TVal* v, const std::vector<std::string>& fs) const {
    if (!v || v->kind != TVal::Rec || v->field_names() != fs) { ok = false; return false; }
    return true;
  }
  // a log entry [term, type, value] (raft.tla:490-492, :807)
  u32 entry(const TVal* v) const {
    if (!shape(v, names({"term", "type", "value"}))) return 0;
    const TVal* ty = v->field("type");
    const std::string tt = ty->text();
    u32 err = 0, type = 0, val = 0;
    if (tt == m.config_entry) {
      type = m.rt.cfg_type;
      val = S::m2r(server_mask(v->field("value")));
    } else if (tt == m.value_entry) {
      type = 1u - m.rt.cfg_type;
      const std::string vt = v->field("value")->text();
      auto it = std::find(m.value.begin(), m.value.end(), vt);
      if (it == m.value.end()) ok = false;
      val = (u32)(it - m.value.begin());
    } else {
      ok = false;
    }
    const u32 e = S::mkentry(integer(v->field("term")), type, val, err);
    if (err) ok = false;
    return e;
  }
  // a log inside a message: <= MaxLogLength entries, MSB-first (memb_spec.h sub_to_mlog)
  u64 mlog(const TVal* v) const {
    if (!v || v->kind != TVal::Seq || (int)v->elems.size() > S::MAXLOG) { ok = false; return 0; }
    const int n = (int)v->elems.size();
    u64 f = (u64)n << (S::MAXLOG * S::EW);
    for (int p = 0; p < n; ++p) f |= (u64)entry(&v->elems[p]) << ((S::MAXLOG - 1 - p) * S::EW);
    return f;
  }
  u64 message(const TVal* v) const {
    if (!v || v->kind != TVal::Rec || !v->field("mtype")) { ok = false; return 0; }
    const std::string ty = v->field("mtype")->text();
    auto F = [&](const char* f) { return v->field(f); };
    u32 err = 0;
    u64 c = 0;
    if (ty == m.t_rvq && shape(v, names({"mtype", "mterm", "mlastLogTerm", "mlastLogIndex", "msource", "mdest"})))
      c = S::m_rvq(server(F("mdest")), integer(F("mlastLogIndex")), integer(F("mlastLogTerm")), server(F("msource")),
                   integer(F("mterm")), err);
    else if (ty == m.t_rvp && shape(v, names({"mtype", "mterm", "mvoteGranted", "mlog", "msource", "mdest"})))
      c = S::m_rvp(server(F("mdest")), mlog(F("mlog")), server(F("msource")), integer(F("mterm")), boolean(F("mvoteGranted")), err);
    else if (ty == m.t_aeq && shape(v, names({"mtype", "mterm", "mprevLogIndex", "mprevLogTerm", "mentries", "mcommitIndex",
                                                "msource", "mdest"}))) {
      const TVal* es = F("mentries");
      u32 ents = 0;
      if (!es || es->kind != TVal::Seq || es->elems.size() > 1) ok = false;
      else if (es->elems.size() == 1) ents = (1u << S::EW) | entry(&es->elems[0]);
      c = S::m_aeq(integer(F("mcommitIndex")), server(F("mdest")), ents, integer(F("mprevLogIndex")), integer(F("mprevLogTerm")),
                   server(F("msource")), integer(F("mterm")), err);
    } else if (ty == m.t_aep && shape(v, names({"mtype", "mterm", "msuccess", "mmatchIndex", "msource", "mdest"})))
      c = S::m_aep(server(F("mdest")), integer(F("mmatchIndex")), server(F("msource")), boolean(F("msuccess")), integer(F("mterm")), err);
    else if (ty == m.t_crq && F("mcommitIndex") &&
             shape(v, names({"mtype", "mterm", "mlogLen", "mentries", "mcommitIndex", "msource", "mdest", "mrounds"})))
      c = S::m_crq8(integer(F("mcommitIndex")), server(F("mdest")), mlog(F("mentries")), integer(F("mlogLen")),
                    integer(F("mrounds")), server(F("msource")), integer(F("mterm")), err);
    else if (ty == m.t_crq && shape(v, names({"mtype", "mterm", "mlogLen", "mentries", "msource", "mdest", "mrounds"})))
      c = S::m_crq7(server(F("mdest")), mlog(F("mentries")), integer(F("mlogLen")), integer(F("mrounds")), server(F("msource")),
                    integer(F("mterm")), err);
    else if (ty == m.t_crp && shape(v, names({"mtype", "mterm", "msuccess", "mmatchIndex", "msource", "mdest", "mroundsLeft"})))
      c = S::m_crp(server(F("mdest")), integer(F("mmatchIndex")), integer(F("mroundsLeft")), server(F("msource")),
                   boolean(F("msuccess")), integer(F("mterm")), err);
    else if (ty == m.t_coc && shape(v, names({"mtype", "mterm", "madd", "mserver", "msource", "mdest"})))
      c = S::m_coc(boolean(F("madd")), server(F("mdest")), server(F("mserver")), server(F("msource")), integer(F("mterm")), err);
    else
      ok = false;
    if (err) ok = false;
    return c;
  }
  // one history entry (raft.tla:248-253, :281, :311-312, :410, :426, :483, :534, :537, :802-803)
  void history_entry(const TVal& e, u64& x, u64& y) const {
    x = ~0ull; y = ~0ull;
    ok = true;
    if (e.kind != TVal::Rec || !e.field("action") || e.field("action")->kind != TVal::Str) return;
    const std::string a = e.field("action")->s;
    const TVal* on = e.field("executedOn");
    u64 xx = 0, yy = 0;
    if (a == "Send" || a == "Receive") {
      if (!shape(&e, names({"action", "executedOn", "msg"}))) return;
      yy = message(e.field("msg"));
      const TVal* who = e.field("msg")->field(a == "Send" ? "msource" : "mdest");
      const int ex = server(on);
      if (!ok || server(who) != ex) return;   // executedOn is msource / mdest by construction
      xx = S::hx(a == "Send" ? S::HE_SEND : S::HE_RECV, ex, 0);
    } else if (a == "TryAddServer" || a == "AddServer") {
      if (!shape(&e, names({"action", "executedOn", "added"}))) return;
      xx = S::hx(a == "AddServer" ? S::HE_ADD : S::HE_TRYADD, server(on), (u32)server(e.field("added")));
    } else if (a == "TryRemoveServer" || a == "RemoveServer") {
      if (!shape(&e, names({"action", "executedOn", "removed"}))) return;
      xx = S::hx(a == "RemoveServer" ? S::HE_REM : S::HE_TRYREM, server(on), (u32)server(e.field("removed")));
    } else if (a == "BecomeLeader") {
      if (!shape(&e, names({"action", "executedOn", "leaders"}))) return;
      xx = S::hx(S::HE_BL, server(on), server_mask(e.field("leaders")));
    } else if (a == "CommitEntry") {
      if (!shape(&e, names({"action", "entry", "executedOn"}))) return;
      xx = S::hx(S::HE_CE, server(on), entry(e.field("entry")));
    } else if (a == "CommitMembershipChange") {
      if (!shape(&e, names({"action", "config", "executedOn"}))) return;
      xx = S::hx(S::HE_CMC, server(on), server_mask(e.field("config")));
    } else if (a == "Restart" || a == "Timeout") {
      if (!shape(&e, names({"action", "executedOn"}))) return;
      xx = S::hx(a == "Restart" ? S::HE_RESTART : S::HE_TIMEOUT, server(on), 0);
    } else {
      return;
    }
    if (ok) { x = xx; y = yy; }
  }
};

// [position][binding][x, y]; bindings of (s1, s2, s3) to distinct servers, lexicographic
template <class S>
std::vector<u64> encode_prefix_table(const MembModel& m, const std::vector<TVal>& trace, int* unmatched = nullptr) {
  std::vector<u64> tab;
  std::vector<std::array<int, 3>> binds;
  for (int a = 0; a < m.N; ++a)
    for (int b = 0; b < m.N; ++b)
      for (int c = 0; c < m.N; ++c)
        if (a != b && b != c && a != c) binds.push_back({a, b, c});
  if ((int)binds.size() != S::NB) throw CfgError(MC_E_INVALID, "binding count does not match the compiled shape");
  int bad = 0;
  tab.resize(trace.size() * binds.size() * 2);
  for (size_t p = 0; p < trace.size(); ++p)
    for (size_t b = 0; b < binds.size(); ++b) {
      MembPrefix<S> enc{m, {binds[b][0], binds[b][1], binds[b][2]}};
      u64 x, y;
      enc.history_entry(trace[p], x, y);
      if (x == ~0ull) ++bad;
      tab[(p * binds.size() + b) * 2] = x;
      tab[(p * binds.size() + b) * 2 + 1] = y;
    }
  if (unmatched) *unmatched = bad;
  return tab;
}

}  // namespace rmc
