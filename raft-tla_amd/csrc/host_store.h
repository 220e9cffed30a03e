// raftmc host: the completed BFS levels that were moved out of HBM (the host spill, DESIGN.md
// §3c/§3d).  Global ids [0, size()) live here, one segment per spill (or per recovered
// checkpoint), so growing the host part never reallocates and copies what is already there: a
// spill of d states touches d states' worth of new host memory, not twice the whole host part.
#pragma once
#include <stdint.h>

#include <algorithm>
#include <cstdio>
#include <cstring>
#include <vector>

namespace rmc {

class HostStore {
 public:
  explicit HostStore(int words_per_state = 0) : nwp_(words_per_state) {}
  void set_words(int nwp) { nwp_ = nwp; }
  void clear() { st_.clear(); me_.clear(); first_.clear(); n_ = 0; }
  uint64_t size() const { return n_; }
  // a new segment of d states; the caller fills both arrays (states: d * nwp words, meta: d)
  void append(uint64_t d, uint32_t** states, uint64_t** meta) {
    first_.push_back(n_);
    st_.emplace_back((size_t)(d * (uint64_t)nwp_));
    me_.emplace_back((size_t)d);
    n_ += d;
    *states = st_.back().data();
    *meta = me_.back().data();
  }
  const uint32_t* state(uint64_t gid) const { const size_t k = seg(gid); return st_[k].data() + (gid - first_[k]) * (uint64_t)nwp_; }
  uint64_t meta(uint64_t gid) const { const size_t k = seg(gid); return me_[k][gid - first_[k]]; }
  // the states, then the parent pointers, in global-id order (the checkpoint layout)
  bool write_states(FILE* f) const {
    for (const auto& s : st_) if (!s.empty() && std::fwrite(s.data(), 4, s.size(), f) != s.size()) return false;
    return true;
  }
  bool write_meta(FILE* f) const {
    for (const auto& m : me_) if (!m.empty() && std::fwrite(m.data(), 8, m.size(), f) != m.size()) return false;
    return true;
  }
  // visit the segments in order: fn(first gid, count, states, meta)
  template <class F>
  void for_each_segment(F fn) const {
    for (size_t k = 0; k < st_.size(); ++k) fn(first_[k], (uint64_t)me_[k].size(), st_[k].data(), me_[k].data());
  }

 private:
  size_t seg(uint64_t gid) const { return (size_t)(std::upper_bound(first_.begin(), first_.end(), gid) - first_.begin()) - 1; }
  int nwp_;
  std::vector<std::vector<uint32_t>> st_;
  std::vector<std::vector<uint64_t>> me_;
  std::vector<uint64_t> first_;
  uint64_t n_ = 0;
};

}  // namespace rmc
