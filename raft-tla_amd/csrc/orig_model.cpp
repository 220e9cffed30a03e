// raftmc host: resolve a cfg into the raft_original model (orig_text.h).
#include <algorithm>
#include <sstream>

#include "../../include/raftmc.h"
#include "orig_text.h"

namespace rmc {

OrigModel resolve_orig_model(const CfgFile& cfg) {
  OrigModel m;
  const CVal& srv = cfg.get("Server");
  const CVal& val = cfg.get("Value");
  if (srv.kind != CVal::Set || val.kind != CVal::Set) throw CfgError(MC_E_UNSUPPORTED, "Server and Value must be finite sets");
  for (auto& e : srv.elems) {
    if (e.kind != CVal::MV) throw CfgError(MC_E_UNSUPPORTED, "Server elements must be model values (e.g. {s1, s2, s3})");
    m.server.push_back(e.text());
  }
  for (auto& e : val.elems) m.value.push_back(e.text());
  std::sort(m.server.begin(), m.server.end());
  m.server.erase(std::unique(m.server.begin(), m.server.end()), m.server.end());
  std::sort(m.value.begin(), m.value.end());
  m.value.erase(std::unique(m.value.begin(), m.value.end()), m.value.end());
  m.N = (int)m.server.size(); m.NV = (int)m.value.size();
  m.follower = cfg.get("Follower").text(); m.candidate = cfg.get("Candidate").text(); m.leader = cfg.get("Leader").text();
  m.nil = cfg.get("Nil").text();
  m.t_rvq = cfg.get("RequestVoteRequest").text(); m.t_rvp = cfg.get("RequestVoteResponse").text();
  m.t_aeq = cfg.get("AppendEntriesRequest").text(); m.t_aep = cfg.get("AppendEntriesResponse").text();
  auto geti = [&](const char* n) {
    const CVal& v = cfg.get(n);
    if (v.kind != CVal::Int) throw CfgError(MC_E_UNSUPPORTED, std::string(n) + " must be an integer");
    return (int)v.i;
  };
  m.MT = geti("MaxTerm"); m.ML = geti("MaxLogLen"); m.MK = geti("MaxMsgDomain");
  m.rt.min_count = geti("MinMsgCount"); m.rt.max_count = geti("MaxMsgCount");
  if (m.rt.min_count < -7 || m.rt.max_count > 6 || m.rt.min_count > m.rt.max_count)
    throw CfgError(MC_E_UNSUPPORTED, "message count range must lie within -7..6");
  if (cfg.init != "Init") throw CfgError(MC_E_UNSUPPORTED, "INIT must be Init");
  if (cfg.next != "Next") throw CfgError(MC_E_UNSUPPORTED, "NEXT must be Next (raft_original.tla:453)");
  if (!cfg.symmetry.empty() || !cfg.view.empty()) throw CfgError(MC_E_UNSUPPORTED, "SYMMETRY/VIEW are not supported for raft_original in this build");
  if (!cfg.action_constraints.empty()) throw CfgError(MC_E_UNSUPPORTED, "ACTION_CONSTRAINTS are not supported for raft_original");
  if (!cfg.properties.empty()) throw CfgError(MC_E_UNSUPPORTED, "temporal PROPERTIES are not supported");
  for (auto& c : cfg.constraints) {
    if (c == "BoundedTerms") m.rt.constraints |= OC_BoundedTerms;
    else if (c == "BoundedLogs") m.rt.constraints |= OC_BoundedLogs;
    else if (c == "BoundedMessages") m.rt.constraints |= OC_BoundedMessages;
    else throw CfgError(MC_E_UNSUPPORTED, "unknown state constraint '" + c + "' for raft_original");
    m.constraint_names.push_back(c);
  }
  if (m.rt.constraints != (OC_BoundedTerms | OC_BoundedLogs | OC_BoundedMessages))
    throw CfgError(MC_E_UNSUPPORTED, "raft_original needs BoundedTerms, BoundedLogs and BoundedMessages (its state space is infinite otherwise, G1)");
  for (auto& n : cfg.invariants) {
    if (const u32 bit = orig_inv_bit(n.c_str())) m.rt.invariants |= bit;
    else throw CfgError(MC_E_UNSUPPORTED, "unknown invariant '" + n + "' for raft_original");
    m.inv_names.push_back(n);
  }
  return m;
}

}  // namespace rmc
