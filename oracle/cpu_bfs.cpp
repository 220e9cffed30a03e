// ============================================================================
// CPU BASELINE ONLY (bench.py's cpu_baseline leg; never part of the product, never a parity
// checker — oracle/main.cpp's restatement is the checker).
//
// cpu_bfs — a multithreaded, TLC-style breadth-first model checker for raft_original on the
// host: SURVEY.md §8(d)'s "builder's multithreaded C++ CPU BFS (same semantics as the oracle)
// with threads = nproc", the stand-in for `tlc2.TLC -workers N` (TLC itself cannot run offline,
// SURVEY.md §8c).  It does what TLC's workers do, with the data structures a tuned CPU checker
// would use: frontier states as fixed-width packed words, a lock-free open-addressing set of
// 64-bit fingerprints (CAS insert, linear probing), level-synchronous expansion with each
// thread taking frontier blocks from a shared cursor and appending its new states to its own
// next-level buffer.  The successor relation, constraints and packing are the product's
// (raft-tla_amd/csrc/orig_spec.h, checked against the oracle by tests/test_packed_semantics.py),
// so the comparison with the GPU is engine against engine, not spec encoding against spec encoding.
// Like the GPU pipeline (and TLC) it evaluates the cfg's invariants on every new state.
//
//   cpu_bfs CFG [--threads T] [--max-states N] [--max-depth D] [--table-log2 K]
//   -> one JSON line {generated, distinct, depth, seconds, threads, verdict}
// Shape from -DSHAPE_N.. like tests/native/orig_host_bfs.cpp.
// ============================================================================
#include <atomic>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "../raft-tla_amd/csrc/orig_text.h"

using namespace rmc;
using S = Orig<SHAPE_N, SHAPE_NV, SHAPE_MT, SHAPE_ML, SHAPE_MK>;
using W = S::Work;
constexpr int NW = S::NW;

struct Packed { u32 w[NW]; };

int main(int argc, char** argv) {
  if (argc < 2) { std::fprintf(stderr, "usage: cpu_bfs CFG [--threads T] [--max-states N] [--max-depth D]\n"); return 2; }
  CfgFile cfg = parse_cfg_text(read_text_file(argv[1]));
  OrigModel m = resolve_orig_model(cfg);
  int threads = (int)std::thread::hardware_concurrency();
  long long max_states = 0, max_depth = 0;
  int table_log2 = 0;
  for (int a = 2; a < argc; ++a) {
    const std::string k = argv[a];
    if (k == "--threads") threads = std::atoi(argv[++a]);
    else if (k == "--max-states") max_states = std::atoll(argv[++a]);
    else if (k == "--max-depth") max_depth = std::atoll(argv[++a]);
    else if (k == "--table-log2") table_log2 = std::atoi(argv[++a]);
  }
  if (threads < 1) threads = 1;
  // fingerprint set: 2^k u64 slots, <= 50% load for the sample bound (or 2^28 by default)
  if (!table_log2) {
    table_log2 = 20;
    const long long want = max_states ? 2 * max_states : (1ll << 28);
    while ((1ll << table_log2) < want && table_log2 < 34) ++table_log2;
  }
  const u64 mask = (1ull << table_log2) - 1;
  std::vector<std::atomic<u64>> table(mask + 1);
  for (auto& x : table) x.store(0, std::memory_order_relaxed);
  const u64 seed = 0x5EED5EED2024ull;
  auto insert = [&](u64 fp) -> bool {   // true if new
    u64 i = fp & mask;
    for (u64 p = 0; p <= mask; ++p) {
      u64 cur = table[i].load(std::memory_order_relaxed);
      if (cur == fp) return false;
      if (cur == 0) {
        if (table[i].compare_exchange_strong(cur, fp, std::memory_order_relaxed)) return true;
        if (cur == fp) return false;
      }
      i = (i + 1) & mask;
    }
    std::fprintf(stderr, "fingerprint table full\n");
    std::exit(3);
  };

  auto t0 = std::chrono::steady_clock::now();
  W s0; S::init(s0);
  Packed p0; S::pack(s0, p0.w);
  insert(fp64(p0.w, seed));
  std::vector<Packed> frontier{p0};
  std::atomic<long long> generated{1}, distinct{1};
  long long depth = 1;
  bool sample_stop = false;
  std::atomic<u32> err{0};
  std::atomic<bool> violation{false};
  while (!frontier.empty() && !sample_stop) {
    if (max_depth && depth >= max_depth) break;
    std::vector<std::vector<Packed>> next(threads);
    std::atomic<size_t> cursor{0};
    std::atomic<bool> stop{false};
    const size_t BLK = 256;
    auto work = [&](int t) {
      long long gen = 0;
      u32 e = 0;
      auto& out = next[t];
      for (;;) {
        const size_t b0 = cursor.fetch_add(BLK);
        if (b0 >= frontier.size() || stop.load(std::memory_order_relaxed)) break;
        const size_t b1 = std::min(frontier.size(), b0 + BLK);
        for (size_t i = b0; i < b1; ++i) {
          W s; S::unpack(frontier[i].w, s);
          u64 al[S::AW]; S::all_logs_next(s, al);
          for (int k = 0; k < S::NI; ++k) {
            W t2;
            const int act = S::apply(s, k, t2, e);
            if (act < 0) continue;
            ++gen;
            for (int q = 0; q < S::AW; ++q) t2.allLogs[q] = al[q];
            if (!S::in_model(t2, m.rt)) continue;
            Packed pk; S::pack(t2, pk.w);
            if (insert(fp64(pk.w, seed))) {
              // the configured invariants on every new state, as the GPU pipeline does (TLC: every
              // distinct state); a violation stops the search
              if (S::violated(t2, m.rt.invariants)) { violation.store(true, std::memory_order_relaxed); stop.store(true, std::memory_order_relaxed); }
              out.push_back(pk);
              const long long d = distinct.fetch_add(1, std::memory_order_relaxed) + 1;
              if (max_states && d >= max_states) stop.store(true, std::memory_order_relaxed);
            }
          }
        }
      }
      generated.fetch_add(gen);
      err.fetch_or(e);
    };
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) th.emplace_back(work, t);
    work(0);
    for (auto& x : th) x.join();
    sample_stop = stop.load();
    std::vector<Packed> nf;
    size_t tot = 0;
    for (auto& v : next) tot += v.size();
    nf.reserve(tot);
    for (auto& v : next) { nf.insert(nf.end(), v.begin(), v.end()); std::vector<Packed>().swap(v); }
    if (!nf.empty()) ++depth;
    frontier.swap(nf);
  }
  const double secs = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
  std::printf("{\"verdict\": \"%s\", \"generated\": %lld, \"distinct\": %lld, \"depth\": %lld, \"seconds\": %.6f, "
              "\"threads\": %d, \"err\": %u, \"table_log2\": %d}\n",
              violation.load() ? "INVARIANT_VIOLATION" : sample_stop ? "SAMPLE_LIMIT" : (max_depth && !frontier.empty() ? "DEPTH_LIMIT" : "OK"), generated.load(),
              distinct.load(), depth, secs, threads, err.load(), table_log2);
  return 0;
}
