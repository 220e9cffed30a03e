// raftmc host: MembModel (tlc_membership model resolved from the cfg) and the
// canonical TLA+ text of a working state.  Printing follows TLC's value syntax
// with a canonical order (records by field name, sets and function keys by
// their own text, the empty function as <<>>), the same rule the oracle's
// dump uses, so state dumps compare as sets of strings.  `history` is printed
// without its unbounded "global" sequence (the product keeps a summary of it,
// memb_spec.h); the counters that constraints read are printed exactly.
#pragma once
#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "memb_spec.h"
#include "model.h"

namespace rmc {

struct MembModel {
  int N = 0, NV = 0;
  MembRuntime rt{};
  std::vector<std::string> server, value;                 // printed names, index order
  std::string nil, follower, candidate, leader, value_entry, config_entry;
  std::string t_rvq, t_rvp, t_aeq, t_aep, t_crq, t_crp, t_coc;
  std::vector<std::string> inv_names, constraint_names, action_constraint_names;
  std::string next_name;
};

MembModel resolve_memb_model(const CfgFile& cfg);   // memb_model.cpp; throws CfgError

template <class S>
struct MembText {
  using W = typename S::Work;
  using LogV = typename S::LogV;
  const MembModel& m_;
  explicit MembText(const MembModel& m) : m_(m) {}
  const std::string& sv(int i) const { return m_.server[i]; }
  static std::string join_sorted(std::vector<std::string> xs, const char* open, const char* sep, const char* close) {
    std::sort(xs.begin(), xs.end());
    std::string o = open;
    for (size_t k = 0; k < xs.size(); ++k) o += (k ? sep : "") + xs[k];
    return o + close;
  }
  static std::string record(std::vector<std::pair<std::string, std::string>> fs) {
    std::sort(fs.begin(), fs.end());
    std::string o = "[";
    for (size_t k = 0; k < fs.size(); ++k) o += (k ? ", " : "") + fs[k].first + " |-> " + fs[k].second;
    return o + "]";
  }
  std::string fn_servers(const std::function<std::string(int)>& f) const {
    std::vector<std::string> xs;
    for (int i = 0; i < S::N; ++i) xs.push_back(sv(i) + " :> " + f(i));
    return join_sorted(xs, "(", " @@ ", ")");
  }
  std::string server_set(u32 mask) const {
    std::vector<std::string> xs;
    for (int j = 0; j < S::N; ++j) if ((mask >> j) & 1u) xs.push_back(sv(j));
    return join_sorted(xs, "{", ", ", "}");
  }
  static std::string b(bool x) { return x ? "TRUE" : "FALSE"; }
  static std::string n(long long x) { return std::to_string(x); }
  std::string entry_text(u32 e) const {
    const bool cfg = S::etype(e) == m_.rt.cfg_type;
    return record({{"term", n(S::eterm(e))}, {"type", cfg ? m_.config_entry : m_.value_entry},
                   {"value", cfg ? server_set(S::r2m(S::evalue(e))) : m_.value[S::evalue(e)]}});
  }
  std::string log_text(LogV l) const {
    std::string o = "<<";
    for (int p = 0; p < S::llen(l); ++p) o += (p ? ", " : "") + entry_text(S::lent(l, p));
    return o + ">>";
  }
  std::string mlog_text(u64 f) const {
    std::string o = "<<";
    for (int p = 0; p < S::mlog_len(f); ++p) o += (p ? ", " : "") + entry_text(S::mlog_ent(f, p));
    return o + ">>";
  }
  std::string msg_text(u64 c) const {
    auto f = [&](int off, int w) { return (long long)S::fld(c, off, w); };
    switch (S::mcls(c)) {
      case S::K_COC:
        return record({{"madd", b(f(S::O_COC_ADD, 1))}, {"mdest", sv(f(S::O_COC_DST, S::SB))}, {"mserver", sv(f(S::O_COC_SRV, S::SB))},
                       {"msource", sv(f(S::O_COC_SRC, S::SB))}, {"mterm", n(f(S::O_COC_TERM, S::TB))}, {"mtype", m_.t_coc}});
      case S::K_RVQ:
        return record({{"mdest", sv(f(S::O_RVQ_DST, S::SB))}, {"mlastLogIndex", n(f(S::O_RVQ_LLI, S::IB))},
                       {"mlastLogTerm", n(f(S::O_RVQ_LLT, S::TB))}, {"msource", sv(f(S::O_RVQ_SRC, S::SB))},
                       {"mterm", n(f(S::O_RVQ_TERM, S::TB))}, {"mtype", m_.t_rvq}});
      case S::K_RVP:
        return record({{"mdest", sv(f(S::O_RVP_DST, S::SB))}, {"mlog", mlog_text((u64)f(S::O_RVP_LOG, S::MLOGB))},
                       {"msource", sv(f(S::O_RVP_SRC, S::SB))}, {"mterm", n(f(S::O_RVP_TERM, S::TB))}, {"mtype", m_.t_rvp},
                       {"mvoteGranted", b(f(S::O_RVP_GR, 1))}});
      case S::K_AEP:
        return record({{"mdest", sv(f(S::O_AEP_DST, S::SB))}, {"mmatchIndex", n(f(S::O_AEP_MMI, S::IB))},
                       {"msource", sv(f(S::O_AEP_SRC, S::SB))}, {"msuccess", b(f(S::O_AEP_SUC, 1))},
                       {"mterm", n(f(S::O_AEP_TERM, S::TB))}, {"mtype", m_.t_aep}});
      case S::K_CRQ7:
        return record({{"mdest", sv(f(S::O_CQ7_DST, S::SB))}, {"mentries", mlog_text((u64)f(S::O_CQ7_ENT, S::MLOGB))},
                       {"mlogLen", n(f(S::O_CQ7_LLEN, S::IB))}, {"mrounds", n(f(S::O_CQ7_RND, S::RB))},
                       {"msource", sv(f(S::O_CQ7_SRC, S::SB))}, {"mterm", n(f(S::O_CQ7_TERM, S::TB))}, {"mtype", m_.t_crq}});
      case S::K_CRP:
        return record({{"mdest", sv(f(S::O_CRP_DST, S::SB))}, {"mmatchIndex", n(f(S::O_CRP_MMI, S::IB))},
                       {"mroundsLeft", n(f(S::O_CRP_RL, S::RB))}, {"msource", sv(f(S::O_CRP_SRC, S::SB))},
                       {"msuccess", b(f(S::O_CRP_SUC, 1))}, {"mterm", n(f(S::O_CRP_TERM, S::TB))}, {"mtype", m_.t_crp}});
      case S::K_CRQ8:
        return record({{"mcommitIndex", n(f(S::O_CQ8_CI, S::IB))}, {"mdest", sv(f(S::O_CQ8_DST, S::SB))},
                       {"mentries", mlog_text((u64)f(S::O_CQ8_ENT, S::MLOGB))}, {"mlogLen", n(f(S::O_CQ8_LLEN, S::IB))},
                       {"mrounds", n(f(S::O_CQ8_RND, S::RB))}, {"msource", sv(f(S::O_CQ8_SRC, S::SB))},
                       {"mterm", n(f(S::O_CQ8_TERM, S::TB))}, {"mtype", m_.t_crq}});
      default: {
        const u32 ents = (u32)f(S::O_AEQ_ENT, S::AEEB);
        const std::string et = (ents >> S::EW) ? "<<" + entry_text(ents & S::EM) + ">>" : "<<>>";
        return record({{"mcommitIndex", n(f(S::O_AEQ_CI, S::IB))}, {"mdest", sv(f(S::O_AEQ_DST, S::SB))}, {"mentries", et},
                       {"mprevLogIndex", n(f(S::O_AEQ_PLI, S::IB))}, {"mprevLogTerm", n(f(S::O_AEQ_PLT, S::TB))},
                       {"msource", sv(f(S::O_AEQ_SRC, S::SB))}, {"mterm", n(f(S::O_AEQ_TERM, S::TB))}, {"mtype", m_.t_aeq}});
      }
    }
  }
  std::string bag_text(const W& s) const {
    std::vector<std::string> xs;
    for (int q = 0; q < S::MK + 1; ++q)
      if (s.bag.v[q] != S::EMPTY) xs.push_back(msg_text(S::mcode(s.bag.v[q])) + " :> " + n(S::mcount(s.bag.v[q])));
    if (xs.empty()) return "<<>>";
    return join_sorted(xs, "(", " @@ ", ")");
  }
  std::string history_text(const W& s) const {
    return record({{"hadNumClientRequests", n(S::hget(s.h0, S::H_CR, 3))}, {"hadNumLeaders", n(S::hget(s.h0, S::H_HL, 4))},
                   {"hadNumMembershipChanges", n(S::hget(s.h0, S::H_MC, 3))},
                   {"hadNumTriedMembershipChanges", n(S::hget(s.h0, S::H_TMC, 3))},
                   {"server", fn_servers([&](int i) { return record({{"restarted", n(S::restarted(s, i))}, {"timeout", n(S::timeouts(s, i))}}); })}});
  }
  std::string state_name(int st) const { return st == 0 ? m_.follower : st == 1 ? m_.candidate : m_.leader; }
  // one line per variable in declaration order (raft.tla:114-185), joined like the oracle's dump
  std::string text(const W& s, bool multiline) const {
    std::vector<std::pair<std::string, std::string>> v = {
        {"messages", bag_text(s)},
        {"history", history_text(s)},
        {"currentTerm", fn_servers([&](int i) { return n(S::g_term(s, i)); })},
        {"state", fn_servers([&](int i) { return state_name(S::g_st(s, i)); })},
        {"votedFor", fn_servers([&](int i) { const int x = S::g_voted(s, i); return x == S::N ? m_.nil : sv(x); })},
        {"log", fn_servers([&](int i) { return log_text(S::getlog(s, i)); })},
        {"commitIndex", fn_servers([&](int i) { return n(S::g_commit(s, i)); })},
        {"votesResponded", fn_servers([&](int i) { return server_set(S::g_vr(s, i)); })},
        {"votesGranted", fn_servers([&](int i) { return server_set(S::g_vg(s, i)); })},
        {"nextIndex", fn_servers([&](int i) { return fn_servers([&](int j) { return n(S::g_next(s, i, j)); }); })},
        {"matchIndex", fn_servers([&](int i) { return fn_servers([&](int j) { return n(S::g_match(s, i, j)); }); })}};
    std::string o;
    for (size_t k = 0; k < v.size(); ++k) {
      if (multiline) o += (k ? "\n" : "") + std::string("/\\ ") + v[k].first + " = " + v[k].second;
      else o += (k ? " /\\ " : "/\\ ") + v[k].first + " = " + v[k].second;
    }
    return o;
  }
};

}  // namespace rmc
