// raftmc host: OrigModel (raft_original model resolved from the cfg) and the
// canonical TLA+ text of a packed state.  Printing rules are TLC's value syntax
// with a canonical order: records print fields alphabetically, set elements
// and function keys print sorted by their own text, the empty function prints
// as <<>> (TLC: a function with domain 1..0 is the empty tuple).
#pragma once
#include <algorithm>
#include <functional>
#include <string>
#include <vector>

#include "model.h"
#include "orig_spec.h"

namespace rmc {

struct OrigModel {
  int N = 0, NV = 0, MT = 0, ML = 0, MK = 0;
  OrigRuntime rt{0, 0, 0, 0};
  std::vector<std::string> server, value;                 // printed names, index order
  std::string follower, candidate, leader, nil, t_rvq, t_rvp, t_aeq, t_aep;
  std::vector<std::string> inv_names;                     // cfg order
  std::vector<std::string> constraint_names;
};


OrigModel resolve_orig_model(const CfgFile& cfg);   // orig_model.cpp; throws CfgError

template <class S>
struct OrigText {
  using W = typename S::Work;
  const OrigModel& m_;
  explicit OrigText(const OrigModel& m) : m_(m) {}
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
  std::string entry_text(int e) const {
    return record({{"term", std::to_string(S::eterm(e))}, {"value", m_.value[S::evalue(e)]}});
  }
  std::string log_text(u32 lw) const {
    std::string o = "<<";
    for (int p = 0; p < S::llen(lw); ++p) o += (p ? ", " : "") + entry_text(S::lent(lw, p));
    return o + ">>";
  }
  std::string server_set(u32 mask) const {
    std::vector<std::string> xs;
    for (int j = 0; j < S::N; ++j) if ((mask >> j) & 1u) xs.push_back(sv(j));
    return join_sorted(xs, "{", ", ", "}");
  }
  std::string voterlog_text(u64 row) const {
    std::vector<std::string> xs;
    for (int j = 0; j < S::N; ++j) {
      const u64 cell = (row >> (j * S::VLB)) & lomask(S::VLB);
      if (cell & 1ull) xs.push_back(sv(j) + " :> " + log_text(S::lfrom_idx((u32)(cell >> 1))));
    }
    if (xs.empty()) return "<<>>";                              // the empty function is <<>>
    return join_sorted(xs, "(", " @@ ", ")");
  }
  std::string msg_text(u64 c) const {
    const std::string src = sv(S::msrc(c)), dst = sv(S::mdst(c)), term = std::to_string(S::mterm(c));
    switch (S::mtype(c)) {
      case S::RVQ:
        return record({{"mtype", m_.t_rvq}, {"mterm", term}, {"mlastLogTerm", std::to_string(S::rvq_llt(c))},
                       {"mlastLogIndex", std::to_string(S::rvq_lli(c))}, {"msource", src}, {"mdest", dst}});
      case S::RVP:
        return record({{"mtype", m_.t_rvp}, {"mterm", term}, {"mvoteGranted", S::rvp_granted(c) ? "TRUE" : "FALSE"},
                       {"mlog", log_text(S::lfrom_idx(S::rvp_log(c)))}, {"msource", src}, {"mdest", dst}});
      case S::AEQ: {
        const int ent = S::aeq_ent(c);
        return record({{"mtype", m_.t_aeq}, {"mterm", term}, {"mprevLogIndex", std::to_string(S::aeq_pli(c))},
                       {"mprevLogTerm", std::to_string(S::aeq_plt(c))},
                       {"mentries", ent ? "<<" + entry_text(ent) + ">>" : "<<>>"},
                       {"mlog", log_text(S::lfrom_idx(S::aeq_log(c)))},
                       {"mcommitIndex", std::to_string(S::aeq_mci(c))},
                       {"msource", src}, {"mdest", dst}});
      }
      default:
        return record({{"mtype", m_.t_aep}, {"mterm", term}, {"msuccess", S::aep_success(c) ? "TRUE" : "FALSE"},
                       {"mmatchIndex", std::to_string(S::aep_mmi(c))}, {"msource", src}, {"mdest", dst}});
    }
  }
  std::string state_text(const W& s, bool multiline) const {
    std::vector<std::pair<std::string, std::string>> v;
    {   // messages
      std::vector<std::string> xs;
      for (int k = 0; k < S::MK + 1; ++k)
        if (s.bag.v[k] != S::BEMPTY) xs.push_back(msg_text(S::ecode_of(s.bag.v[k])) + " :> " + std::to_string(S::ecount(s.bag.v[k])));
      v.push_back({"messages", xs.empty() ? "<<>>" : join_sorted(xs, "(", " @@ ", ")")});
    }
    {   // elections
      std::vector<std::string> xs;
      for (int k = 0; k < S::EMAX; ++k) {
        if (s.el[k] == S::EMPTY) continue;
        const u64 e = s.el[k];
        int off = 0;
        auto take = [&](int w) { u64 x = (e >> off) & lomask(w); off += w; return x; };
        const u64 et = take(S::ETB), el = take(S::SB), elog = take(S::LIB), ev = take(S::N);
        const u64 evl = S::evoter_row(take(S::N * S::EVB), (u32)ev);
        xs.push_back(record({{"eterm", std::to_string(et)}, {"eleader", sv((int)el)}, {"elog", log_text(S::lfrom_idx((u32)elog))},
                             {"evotes", server_set((u32)ev)}, {"evoterLog", voterlog_text(evl)}}));
      }
      v.push_back({"elections", join_sorted(xs, "{", ", ", "}")});
    }
    {   // allLogs
      std::vector<std::string> xs;
      for (long long ix = 0; ix < S::U; ++ix) if ((s.allLogs[ix >> 6] >> (ix & 63)) & 1ull) xs.push_back(log_text(S::lfrom_idx((u32)ix)));
      v.push_back({"allLogs", join_sorted(xs, "{", ", ", "}")});
    }
    v.push_back({"currentTerm", fn_servers([&](int i) { return std::to_string(S::g_term(s, i)); })});
    v.push_back({"state", fn_servers([&](int i) { int x = S::g_st(s, i); return x == 0 ? m_.follower : x == 1 ? m_.candidate : m_.leader; })});
    v.push_back({"votedFor", fn_servers([&](int i) { int x = S::g_voted(s, i); return x == S::N ? m_.nil : sv(x); })});
    v.push_back({"log", fn_servers([&](int i) { return log_text(s.log.v[i]); })});
    v.push_back({"commitIndex", fn_servers([&](int i) { return std::to_string(S::g_commit(s, i)); })});
    v.push_back({"votesResponded", fn_servers([&](int i) { return server_set(S::row_bits(s.vresp, i)); })});
    v.push_back({"votesGranted", fn_servers([&](int i) { return server_set(S::row_bits(s.vgrant, i)); })});
    v.push_back({"voterLog", fn_servers([&](int i) { return voterlog_text(s.vl.v[i]); })});
    v.push_back({"nextIndex", fn_servers([&](int i) { return fn_servers([&](int j) { return std::to_string(S::g_ni(s, i, j)); }); })});
    v.push_back({"matchIndex", fn_servers([&](int i) { return fn_servers([&](int j) { return std::to_string(S::g_mi(s, i, j)); }); })});
    std::string o;
    for (size_t k = 0; k < v.size(); ++k) {
      if (multiline) o += (k ? "\n" : "") + std::string("/\\ ") + v[k].first + " = " + v[k].second;
      else o += (k ? " /\\ " : "/\\ ") + v[k].first + " = " + v[k].second;
    }
    return o;
  }
};

template <class S>
std::string orig_state_text(const OrigModel& m, const typename S::Work& s, bool multiline) {
  return OrigText<S>(m).state_text(s, multiline);
}

}  // namespace rmc
