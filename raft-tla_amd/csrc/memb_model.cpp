// raftmc host: resolve a TLC cfg into the tlc_membership model (memb_text.h).
// Every constant, NEXT variant, constraint and invariant of
// tlc_membership/raft.cfg:1-87 maps to a compiled field or predicate;
// anything else fails loudly (MC_E_UNSUPPORTED) instead of being ignored.
#include <algorithm>
#include <sstream>

#include "../../include/raftmc.h"
#include "memb_text.h"

namespace rmc {

namespace {
// order of values as the oracle's value model compares them (ints numerically, strings by
// text, model values by name — the cfgs list s1 < s2 < ... in this order)
bool value_less(const CVal& a, const CVal& b) {
  if (a.kind != b.kind) return a.kind < b.kind;
  if (a.kind == CVal::Int) return a.i < b.i;
  return a.text() < b.text();
}
}  // namespace

MembModel resolve_memb_model(const CfgFile& cfg) {
  MembModel m;
  const CVal& srv = cfg.get("Server");
  const CVal& init = cfg.get("InitServer");
  const CVal& val = cfg.get("Value");
  if (srv.kind != CVal::Set || init.kind != CVal::Set || val.kind != CVal::Set)
    throw CfgError(MC_E_UNSUPPORTED, "Server, InitServer and Value must be finite sets");
  for (auto& e : srv.elems) {
    if (e.kind != CVal::MV) throw CfgError(MC_E_UNSUPPORTED, "Server elements must be model values (e.g. {s1, s2, s3}, G13)");
    m.server.push_back(e.text());
  }
  std::sort(m.server.begin(), m.server.end());
  m.server.erase(std::unique(m.server.begin(), m.server.end()), m.server.end());
  m.N = (int)m.server.size();
  if (m.N < 1 || m.N > 4) throw CfgError(MC_E_UNSUPPORTED, "tlc_membership: 1..4 servers are compiled");
  for (auto& e : init.elems) {
    auto it = std::find(m.server.begin(), m.server.end(), e.text());
    if (it == m.server.end()) throw CfgError(MC_E_UNSUPPORTED, "InitServer must be a subset of Server");
    m.rt.init_cfg |= 1u << (it - m.server.begin());
  }
  std::vector<CVal> vals = val.elems;
  std::sort(vals.begin(), vals.end(), value_less);
  for (auto& e : vals) if (m.value.empty() || m.value.back() != e.text()) m.value.push_back(e.text());
  m.NV = (int)m.value.size();
  if (m.NV < 1) throw CfgError(MC_E_UNSUPPORTED, "Value must be non-empty");

  const CVal& nr = cfg.get("NumRounds");
  if (nr.kind != CVal::Int || nr.i < 1 || nr.i > 3) throw CfgError(MC_E_UNSUPPORTED, "NumRounds must be an integer in 1..3");
  m.rt.num_rounds = (u32)nr.i;
  m.nil = cfg.get("Nil").text();
  for (auto& s : m.server) if (s == m.nil) throw CfgError(MC_E_UNSUPPORTED, "Nil must not be a server");
  m.follower = cfg.get("Follower").text(); m.candidate = cfg.get("Candidate").text(); m.leader = cfg.get("Leader").text();
  const CVal& ve = cfg.get("ValueEntry");
  const CVal& ce = cfg.get("ConfigEntry");
  if (ve.kind != ce.kind || (ve.kind != CVal::Str && ve.kind != CVal::Int))
    throw CfgError(MC_E_UNSUPPORTED, "ValueEntry/ConfigEntry must both be strings (raft.cfg:13-14) or both integers");
  if (ve.text() == ce.text()) throw CfgError(MC_E_UNSUPPORTED, "ValueEntry and ConfigEntry must differ");
  m.value_entry = ve.text(); m.config_entry = ce.text();
  m.rt.cfg_type = value_less(ce, ve) ? 0u : 1u;   // the entry type bit is order preserving
  m.t_rvq = cfg.get("RequestVoteRequest").text(); m.t_rvp = cfg.get("RequestVoteResponse").text();
  m.t_aeq = cfg.get("AppendEntriesRequest").text(); m.t_aep = cfg.get("AppendEntriesResponse").text();
  m.t_crq = cfg.get("CatchupRequest").text(); m.t_crp = cfg.get("CatchupResponse").text();
  m.t_coc = cfg.get("CheckOldConfig").text();
  {
    // the message classes are ordered by their record shapes; mtype is constant per class, so the
    // order holds for any distinct type constants, but they must be distinct
    std::vector<std::string> ts = {m.t_rvq, m.t_rvp, m.t_aeq, m.t_aep, m.t_crq, m.t_crp, m.t_coc};
    std::sort(ts.begin(), ts.end());
    if (std::unique(ts.begin(), ts.end()) != ts.end()) throw CfgError(MC_E_UNSUPPORTED, "message type constants must be distinct");
  }

  if (!cfg.init.empty() && cfg.init != "Init") throw CfgError(MC_E_UNSUPPORTED, "INIT must be Init (raft.tla:388)");
  m.next_name = cfg.next;
  if (cfg.next == "NextAsync") m.rt.next = MN_ASYNC;
  else if (cfg.next == "NextCrash") m.rt.next = MN_CRASH;
  else if (cfg.next == "NextAsyncCrash") m.rt.next = MN_ASYNC | MN_CRASH;
  else if (cfg.next == "NextUnreliable") m.rt.next = MN_UNRELIABLE;
  else if (cfg.next == "Next") m.rt.next = MN_ASYNC | MN_CRASH | MN_UNRELIABLE;
  else if (cfg.next == "NextDynamic") m.rt.next = MN_ASYNC | MN_CRASH | MN_UNRELIABLE | MN_DYNAMIC;
  else throw CfgError(MC_E_UNSUPPORTED, "NEXT '" + cfg.next + "' is not one of the Next relations of raft.tla:909-943");
  m.rt.disjunct_copies = 1;   // TLC's counting (MC_COMPAT_DISJUNCT_COPIES); the run's opts decide
  if (cfg.symmetry == "perms") m.rt.symmetry = 1;
  else if (!cfg.symmetry.empty()) throw CfgError(MC_E_UNSUPPORTED, "SYMMETRY must be perms (raft.tla:1281)");
  if (cfg.view != "vars")
    throw CfgError(MC_E_UNSUPPORTED, "tlc_membership needs VIEW vars (raft.cfg:30): history is kept as a summary, not fingerprinted");
  if (!cfg.properties.empty()) throw CfgError(MC_E_UNSUPPORTED, "temporal PROPERTIES are not supported");

  for (auto& c : cfg.constraints) {
    int id = -1;
    for (int k = 0; k < MC_NCON; ++k) if (c == kMembConNames[k]) id = k;
    if (id < 0) throw CfgError(MC_E_UNSUPPORTED, "unknown state constraint '" + c + "' for tlc_membership");
    m.rt.constraints |= 1u << id;
    m.constraint_names.push_back(c);
  }
  for (auto& c : cfg.action_constraints) {
    if (c == "CommitWhenConcurrentLeaders_action_constraint") m.rt.action_constraints |= MAC_CommitWhenConcurrentLeaders;
    else throw CfgError(MC_E_UNSUPPORTED, "unknown action constraint '" + c + "'");
    m.action_constraint_names.push_back(c);
  }
  // each punctuated-search prefix constraint keeps a dead-binding mask of N(N-1)(N-2) bits in the
  // history word h1 from bit 36 (memb_spec.h H_PREFIX)
  {
    const int nb = m.N >= 3 ? m.N * (m.N - 1) * (m.N - 2) : 0;
    int regions = 0;
    for (int r = 0; r < 2; ++r) if ((m.rt.constraints >> kPrefixCon[r]) & 1u) ++regions;
    if (36 + regions * nb > 64)
      throw CfgError(MC_E_UNSUPPORTED, "CommitWhenConcurrentLeaders_unique and MajorityOfClusterRestarts_constraint together "
                                       "need more history bits than compiled for |Server| = " + std::to_string(m.N));
  }
  // the bounds that size the packed fields (raft.tla:22-30) must be in force
  for (int need : {MC_BoundedInFlightMessages, MC_BoundedLogSize, MC_BoundedTerms})
    if (!(m.rt.constraints & (1u << need)))
      throw CfgError(MC_E_UNSUPPORTED, std::string("tlc_membership needs the state constraint ") + kMembConNames[need] +
                                           " (it bounds a packed field; the state space is unbounded without it)");
  for (auto& n : cfg.invariants) {
    int id = -1;
    for (int k = 0; k < MI_NINV; ++k) if (n == kMembInvNames[k]) id = k;
    if (id < 0) throw CfgError(MC_E_UNSUPPORTED, "unknown invariant '" + n + "' for tlc_membership");
    if (m.rt.n_inv >= 32) throw CfgError(MC_E_UNSUPPORTED, "at most 32 invariants");
    m.rt.inv_order[m.rt.n_inv / 8] |= (u64)id << (8 * (m.rt.n_inv % 8));
    ++m.rt.n_inv;
    m.inv_names.push_back(n);
  }
  return m;
}

}  // namespace rmc
