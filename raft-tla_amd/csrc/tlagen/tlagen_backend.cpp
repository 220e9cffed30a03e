// tlagen_backend.cpp — the generated path behind the C ABI (mc_opts.frontend, SURVEY.md §8(f)
// rank 3): a module + cfg outside the hand-compiled families (or any module, on request) is
// parsed by the SANY-subset front end, compiled to C++ over tlv.h together with the BFS kernels
// of tlagen_kernels.h, turned into a gfx950 code object by hiprtc (cached by source hash next
// to the library, or prebuilt by the build for the repo's own test specs), and run level by
// level from here.  The same module text gives the same counts as the hand-compiled kernels
// (tests/test_tlagen.py, tests/test_gpu_tlagen.py).
#include <dlfcn.h>
#include <hip/hip_runtime.h>
#include <hip/hiprtc.h>
#include <sys/stat.h>
#include <unistd.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <memory>
#include <sstream>

#include "../../../include/raftmc.h"
#include "../backend.h"
#include "tla_gen.h"
#include "tlv_text.h"

namespace rmc {

int tlagen_sort_keys(const unsigned long long* keys_in, unsigned long long* keys_out, unsigned long long n, int bits,
                     void** tmp, size_t* tmp_bytes, hipStream_t s);   // tlagen_sort.hip

namespace {

using u32 = unsigned int;
using u64 = unsigned long long;

// counters of tlagen_kernels.h
enum { C_GEN = 0, C_GIN = 1, C_ERR = 2, C_CAP = 3, C_FLAG = 4, C_KIND = 5, C_SID = 6, C_INV = 7, C_EACT = 8, C_EWORDS = 9,
       C_EV = 10, C_EVINV = 11, C_NEWPOS = 12, C_ACT = 16 };

struct KArgs {   // tlk::Args, field for field
  u32* words; u64* words_used; u64 words_cap;
  u64* offs; u64* parent; u32* act; u64 states_cap;
  u64* n_states; u64* n_committed;
  u64* table; u64 table_mask;
  u32* arena; u32 acap;
  u32* hstack; u32 hcap;
  u64* ctr;
  u32* evbuf; u32 evcap;
  u64 first, count;
  u64 seed;
  int inv_oom, deadlock;
  int fifo;
  u64* newpos; u64 newpos_cap;
  const u64* wkeys; u64 n_w;
  u64 level_end;
  u64 stop_rank, stop_ord;
  int stop_kind;
};

std::string read_all(const std::string& p) {
  std::ifstream f(p, std::ios::binary);
  if (!f) return "";
  std::stringstream ss; ss << f.rdbuf();
  return ss.str();
}
u64 fnv64(const std::string& s) {
  u64 h = 1469598103934665603ull;
  for (unsigned char ch : s) { h ^= ch; h *= 1099511628211ull; }
  return h;
}
std::string hex(u64 v) { char b[17]; std::snprintf(b, sizeof b, "%016llx", v); return b; }
std::string dir_of(const std::string& p) { const size_t s = p.rfind('/'); return s == std::string::npos ? "." : p.substr(0, s); }

std::string lib_dir() {
  Dl_info info;
  if (dladdr((void*)&lib_dir, &info) && info.dli_fname) return dir_of(info.dli_fname);
  return ".";
}

const char* kOpts[] = {"--offload-arch=gfx950", "-O2", "-std=c++17"};
// per-lane stack of a kernel that evaluates recursive function definitions (tlv::kMaxRecDepth
// nested calls of a few hundred bytes each, over the kernel's own frame)
constexpr size_t kRecStackBytes = 16384;
// the text the generator emits into a recursive function definition's depth guard: a source holding
// it gets kRecStackBytes per lane (scripts/check_isa.py reads the same marker)
constexpr const char* kRecMarker = "kMaxRecDepth) {";

#define HIPOK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { err = std::string(#x) + ": " + hipGetErrorString(e_); return MC_E_NO_DEVICE; } } while (0)

struct Meta {
  std::vector<std::string> vars, actions, invariants, atoms;
};

// the generated source names its variables, actions, invariants and atoms in "//@" lines
Meta parse_meta(const std::string& src) {
  Meta m;
  std::istringstream in(src);
  std::string line;
  while (std::getline(in, line)) {
    if (line.rfind("//@", 0) != 0) { if (!line.empty() && line[0] != '/') break; continue; }
    const size_t sp = line.find(' ');
    const std::string kind = line.substr(3, sp - 3), val = sp == std::string::npos ? "" : line.substr(sp + 1);
    if (kind == "var") m.vars.push_back(val);
    else if (kind == "action") m.actions.push_back(val);
    else if (kind == "invariant") m.invariants.push_back(val);
    else if (kind == "atom") m.atoms.push_back(val);
  }
  return m;
}

// TLA+ text of a value, with the library's canonical print rule (the hand-compiled decoders' and
// the oracle's, oracle/tla.h show): records print their fields alphabetically, set elements and
// function pairs sorted by their text, so traces and state dumps compare as text
struct Printer {
  const Meta& m;
  std::string v(const u32* w) const {
    const u32 tag = w[0] & 7u, n = w[1];
    switch (tag) {
      case 1: return w[1] ? "TRUE" : "FALSE";
      case 2: return std::to_string((long long)(int)(w[1] ^ 0x80000000u));
      case 3: return w[1] < m.atoms.size() ? m.atoms[w[1]] : "?";
      case 4: case 6: {
        std::vector<std::string> el;
        const u32* e = w + 2;
        for (u32 i = 0; i < n; ++i) { el.push_back(v(e)); e += e[0] >> 3; }
        if (tag == 6) std::sort(el.begin(), el.end());
        std::string o = tag == 4 ? "<<" : "{";
        for (u32 i = 0; i < n; ++i) o += (i ? ", " : "") + el[i];
        return o + (tag == 4 ? ">>" : "}");
      }
      case 5: {
        bool rec = true;
        const u32* e = w + 2;
        for (u32 i = 0; i < n; ++i) {
          if ((e[0] & 7u) != 3 || e[1] >= m.atoms.size() || m.atoms[e[1]].empty() || m.atoms[e[1]][0] != '"') rec = false;
          e += e[0] >> 3; e += e[0] >> 3;
        }
        std::vector<std::pair<std::string, std::string>> fs;
        e = w + 2;
        for (u32 i = 0; i < n; ++i) {
          const u32* val = e + (e[0] >> 3);
          if (rec) { const std::string& k = m.atoms[e[1]]; fs.push_back({k.substr(1, k.size() - 2), v(val)}); }
          else fs.push_back({v(e), v(val)});
          e = val + (val[0] >> 3);
        }
        std::sort(fs.begin(), fs.end());
        std::string o = rec ? "[" : "(";
        for (u32 i = 0; i < n; ++i) o += (i ? (rec ? ", " : " @@ ") : "") + fs[i].first + (rec ? " |-> " : " :> ") + fs[i].second;
        return o + (rec ? "]" : ")");
      }
    }
    return "?";
  }
  std::string state(const u32* w) const {
    std::string o;
    for (size_t i = 0; i < m.vars.size(); ++i) {
      o += (i ? "\n" : "") + std::string("/\\ ") + m.vars[i] + " = " + v(w);
      w += w[0] >> 3;
    }
    return o;
  }
  static u32 words_of(const u32* w, size_t nv) { u32 n = 0; for (size_t i = 0; i < nv; ++i) { n += w[0] >> 3; w += w[0] >> 3; } return n; }
};

struct TlagenBackend : Backend {
  std::string src, key, src_origin;
  Meta meta;
  RunResult last;
  // device state kept after run() for dump_states / traces
  u32* d_words = nullptr; u64* d_offs = nullptr; u64 n_stored = 0, words_stored = 0;
  bool store_complete = true;   // false after a store overflow (ids handed out without words)
  int dev = 0;
  // The run's device buffers (store, seen-set, lane arenas, FIFO key arrays), kept from one run to the
  // next when the sizes and the device are unchanged: allocating a 200 GiB store costs ~2.5 s on
  // MI355X and freeing the buffers ~2.5 s more (scripts/hipmalloc_time.py), i.e. a quarter of C2's
  // run, so only a changed size (or a larger arena after an overflow) allocates again.
  struct Pool {
    int dev = -1;
    std::vector<u64> bytes;
    std::vector<void*> ptr;
    void free_all() {
      for (void* q : ptr) if (q) (void)hipFree(q);
      ptr.clear(); bytes.clear(); dev = -1;
    }
    // buffers of these sizes on device d (0 bytes: none); false = allocation failed (nothing kept)
    bool get(int d, const std::vector<u64>& want) {
      if (d == dev && want == bytes) return true;
      free_all();
      ptr.assign(want.size(), nullptr);
      for (size_t i = 0; i < want.size(); ++i)
        if (want[i] && hipMalloc(&ptr[i], want[i]) != hipSuccess) { ptr[i] = nullptr; free_all(); return false; }
      bytes = want; dev = d;
      return true;
    }
  } pool;

  TlagenBackend(const std::string& tla_path, const CfgFile& cfg) {
    if (tla_path.size() > 8 && tla_path.compare(tla_path.size() - 8, 8, ".gen.hip") == 0) {
      src = read_all(tla_path);
      if (src.empty()) throw CfgError(MC_E_IO, "cannot read " + tla_path);
      src_origin = "pregenerated " + tla_path;
    } else {
      std::vector<std::string> dirs;
      if (const char* e = std::getenv("RAFTMC_TLA_PATH")) {
        std::string s = e;
        size_t a = 0;
        while (a <= s.size()) { size_t b = s.find(':', a); if (b == std::string::npos) b = s.size(); if (b > a) dirs.push_back(s.substr(a, b - a)); a = b + 1; }
      }
      tlagen::Program prog;
      try { prog = tlagen::load_program(tla_path, dirs); }
      catch (const tlagen::ParseError& e) { throw CfgError(MC_E_PARSE, e.what()); }
      tlagen::Generated g = tlagen::generate(prog, cfg);
      src = tlagen::compose_source(g, kTlvText, kTlgKernelsText);
      src_origin = "front end: " + tla_path;
    }
    meta = parse_meta(src);
    if (meta.vars.empty()) throw CfgError(MC_E_PARSE, "generated source without metadata");
    std::string k = src;
    for (const char* o : kOpts) k += std::string("\n") + o;
    key = hex(fnv64(k));
  }
  ~TlagenBackend() override { release(); }
  void release_device() override { release(); }
  void release() {
    pool.free_all();
    d_words = nullptr; d_offs = nullptr;
  }

  std::string family() const override { return "tlagen"; }
  std::string describe_json() const override {
    std::string o = "{\"family\": \"tlagen\", \"origin\": \"" + src_origin + "\", \"code_object\": \"" + key + "\", \"variables\": [";
    for (size_t i = 0; i < meta.vars.size(); ++i) o += (i ? ", \"" : "\"") + meta.vars[i] + "\"";
    o += "], \"actions\": [";
    for (size_t i = 0; i < meta.actions.size(); ++i) o += (i ? ", \"" : "\"") + meta.actions[i] + "\"";
    return o + "]}";
  }

  // code object: cache file, else hiprtc
  int code_object(std::string& image, std::string& err) {
    std::vector<std::string> dirs;
    if (const char* e = std::getenv("RAFTMC_TLAGEN_CACHE")) dirs.push_back(e);
    dirs.push_back(lib_dir() + "/tlagen_co");
    for (auto& d : dirs) {
      image = read_all(d + "/" + key + ".hsaco");
      if (!image.empty()) return 0;
    }
    hiprtcProgram prog;
    if (hiprtcCreateProgram(&prog, src.c_str(), "tlagen.hip", 0, nullptr, nullptr) != HIPRTC_SUCCESS) { err = "hiprtcCreateProgram failed"; return MC_E_NO_DEVICE; }
    const hiprtcResult rc = hiprtcCompileProgram(prog, 3, kOpts);
    if (rc != HIPRTC_SUCCESS) {
      size_t n = 0; hiprtcGetProgramLogSize(prog, &n);
      std::string log(n, '\0'); if (n) hiprtcGetProgramLog(prog, &log[0]);
      hiprtcDestroyProgram(&prog);
      err = "hiprtc: " + log.substr(0, 4000);
      return MC_E_UNSUPPORTED;
    }
    size_t n = 0; hiprtcGetCodeSize(prog, &n);
    image.assign(n, '\0'); hiprtcGetCode(prog, &image[0]);
    hiprtcDestroyProgram(&prog);
    for (auto& d : dirs) {   // best effort: keep it for the next open (written aside, then renamed)
      ::mkdir(d.c_str(), 0755);
      const std::string path = d + "/" + key + ".hsaco", tmp = path + ".tmp" + std::to_string((long)::getpid());
      std::ofstream f(tmp, std::ios::binary);
      if (!f) continue;
      f.write(image.data(), (std::streamsize)image.size());
      f.close();
      if (f && std::rename(tmp.c_str(), path.c_str()) == 0) break;
      std::remove(tmp.c_str());
    }
    return 0;
  }

  int run(const RunOpts& o, RunResult& r, std::string& err) override {
    // a lane arena too small for one state's successors: searched again with 4x the arena per lane
    // on a quarter of the lanes (the same HBM), up to 64x (C2: 16K words; the Apalache spec's
    // states are ~1.4K words and need more)
    for (arena_scale = 1;; arena_scale *= 4) {
      bool again = false;
      int rc = run_once(o, r, err, again);
      if (rc == 0 && again) {
        // TLC -workers N found an event: TLC's counterexample and stop point are the single-worker
        // search's, so the model is searched again in FIFO order (as the hand-compiled paths do).
        // That search needs more HBM per state (44 B of bookkeeping instead of 20, 16-B seen-set
        // entries): when it does not fit, the event the first search found is still reported
        RunOpts o1 = o;
        o1.workers = 1;
        const std::string found = workers_event_;
        rc = run_once(o1, r, err, again);
        if (rc == 0 && r.verdict == MC_VERDICT_CAPACITY_OVERFLOW && !arena_overflow)
          r.error = "the -workers N search found " + found + "; TLC's single-worker re-search of it (for TLC's "
                    "counterexample and stop point) ran out of capacity: " + r.error;
      }
      if (rc != 0 || !arena_overflow || arena_scale >= 64) return rc;
    }
  }
  u32 arena_scale = 1;
  bool arena_overflow = false;
  std::string workers_event_;   // what a -workers N search stopped on (named if its FIFO re-search overflows)

  int run_once(const RunOpts& o, RunResult& r, std::string& err, bool& again) {
    again = false;
    arena_overflow = false;
    const auto t_start = std::chrono::steady_clock::now();
    if (!o.checkpoint_path.empty() || !o.recover_path.empty()) {
      err = "checkpoint / recover are not implemented on the generated path";
      return MC_E_UNSUPPORTED;
    }
    if (!o.disjunct_copies) {   // the generated code enumerates disjuncts as TLC does (MC_COMPAT_DISJUNCT_COPIES)
      err = "the generated path counts TLC's disjunct copies; MC_COMPAT_DISJUNCT_COPIES cannot be cleared on it";
      return MC_E_UNSUPPORTED;
    }
    // TLC -workers 1: the single-worker FIFO order (two passes per level, tlagen_kernels.h); any
    // other -workers: first-come insertion, every count TLC prints is order independent, and an
    // event is searched again in FIFO order for TLC's counterexample and stop point
    const bool fifo = o.workers == 1;
    dev = o.device;
    HIPOK(hipSetDevice(dev));
    std::string image;
    // RAFTMC_TLAGEN_TIMING=1: where mc_run's wall time goes outside the kernels (stderr)
    const bool timing = std::getenv("RAFTMC_TLAGEN_TIMING") != nullptr;
    auto since = [&]() { return std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count(); };
    if (int rc = code_object(image, err)) return rc;
    const double t_co = since();
    struct Scratch {   // freed on every return (the device buffers stay in the pool)
      hipModule_t mod = nullptr;
      void* sort_tmp = nullptr;
      hipEvent_t e0 = nullptr, e1 = nullptr;
      size_t prev_stack = 0;       // the device's stack limit before a recursive module raised it
      bool stack_raised = false;
      ~Scratch() {
        // hipLimitStackSize is process-wide: later kernels (the hand-compiled paths) get their limit back
        if (stack_raised) (void)hipDeviceSetLimit(hipLimitStackSize, prev_stack);
        if (sort_tmp) (void)hipFree(sort_tmp);
        if (e0) (void)hipEventDestroy(e0);
        if (e1) (void)hipEventDestroy(e1);
        if (mod) (void)hipModuleUnload(mod);
      }
    } sc;
    size_t sort_bytes = 0;
    // A spec with a recursive function definition compiles to kernels whose stack size the
    // compiler cannot bound (dynamic stack): give each lane room for tlv::kMaxRecDepth nested
    // calls (the generated code refuses deeper recursion with an evaluation error), instead of the
    // runtime's default, which the static part of such a kernel's frame already exceeds.
    // (scripts/check_isa.py fails the build for a code object with a dynamic stack whose source lacks
    // this marker, or with a static frame above kRecStackBytes)
    if (src.find(kRecMarker) != std::string::npos) {
      HIPOK(hipDeviceGetLimit(&sc.prev_stack, hipLimitStackSize));
      HIPOK(hipDeviceSetLimit(hipLimitStackSize, kRecStackBytes));
      sc.stack_raised = true;
    }
    HIPOK(hipModuleLoadData(&sc.mod, image.data()));
    hipFunction_t f_init, f_expand, f_keys, f_mat, f_stop;
    HIPOK(hipModuleGetFunction(&f_init, sc.mod, "tlg_init_k"));
    HIPOK(hipModuleGetFunction(&f_expand, sc.mod, "tlg_expand_k"));
    HIPOK(hipModuleGetFunction(&f_keys, sc.mod, "tlg_keys_k"));
    HIPOK(hipModuleGetFunction(&f_mat, sc.mod, "tlg_mat_k"));
    HIPOK(hipModuleGetFunction(&f_stop, sc.mod, "tlg_stop_k"));
    // HBM layout: store words + per-state offsets/parents/actions, seen-set, lanes' arenas (+ FIFO:
    // the level's inserted entries and their keys, unsorted and sorted)
    const u64 store = o.state_store_bytes ? o.state_store_bytes : (16ull << 30);
    // canonical words dominate (C2: ~350-450 words per state); 20 B per state for offsets, parents,
    // actions (+ 24 B of per-level key arrays in FIFO order)
    const u64 per_state = fifo ? 44 : 20;
    const u64 states_cap = store / 7 / per_state, words_cap = (store - states_cap * per_state) / 4;
    const u64 entry = fifo ? 16 : 8;
    u64 tbytes = o.fp_table_bytes ? o.fp_table_bytes : (2ull << 30);
    u64 slots = 1; while (slots * 2 * entry <= tbytes) slots *= 2;
    const u32 acap = 16384 * arena_scale, hcap = 4096 * arena_scale, evcap = 65536 * arena_scale;
    int ncu = 256;
    (void)hipDeviceGetAttribute(&ncu, hipDeviceAttributeMultiprocessorCount, dev);
    int waves = 8;   // per CU: 2 per SIMD (the expand kernel holds ~250 VGPRs)
    if (const char* e = std::getenv("RAFTMC_TLAGEN_WAVES")) waves = std::max(1, std::atoi(e));
    const u64 lanes = std::max<u64>(64, (u64)ncu * waves * 64 / arena_scale);
    u64 *d_parent = nullptr, *d_table = nullptr, *d_ctr = nullptr, *d_newpos = nullptr, *d_keys = nullptr, *d_sorted = nullptr;
    u32 *d_act = nullptr, *d_arena = nullptr, *d_hs = nullptr, *d_ev = nullptr;
    const int nact = (int)meta.actions.size();
    const size_t nctr = C_ACT + 2 * (size_t)nact + 4;   // + n_committed, n_states, words_used
    const u64 kcap = fifo ? std::min<u64>(states_cap, slots) : 1;
    const u64 kb = fifo ? kcap * 8 : 0;
    d_words = nullptr; d_offs = nullptr;
    if (!pool.get(dev, {words_cap * 4, states_cap * 8, states_cap * 8, states_cap * 4, slots * entry, nctr * 8,
                        lanes * acap * 4, lanes * hcap * 4, evcap * 4, kb, kb, kb})) {
      err = "device allocation failed";
      return MC_E_OOM;
    }
    d_words = (u32*)pool.ptr[0]; d_offs = (u64*)pool.ptr[1]; d_parent = (u64*)pool.ptr[2]; d_act = (u32*)pool.ptr[3];
    d_table = (u64*)pool.ptr[4]; d_ctr = (u64*)pool.ptr[5]; d_arena = (u32*)pool.ptr[6]; d_hs = (u32*)pool.ptr[7];
    d_ev = (u32*)pool.ptr[8]; d_newpos = (u64*)pool.ptr[9]; d_keys = (u64*)pool.ptr[10]; d_sorted = (u64*)pool.ptr[11];
    n_stored = 0; words_stored = 0; store_complete = false;
    HIPOK(hipMemset(d_table, 0, slots * entry));
    HIPOK(hipMemset(d_ctr, 0, nctr * 8));
    if (timing) HIPOK(hipDeviceSynchronize());
    const double t_setup = since();
    KArgs a{};
    a.words = d_words; a.words_used = d_ctr + nctr - 1; a.words_cap = words_cap;
    a.offs = d_offs; a.parent = d_parent; a.act = d_act; a.states_cap = states_cap;
    a.n_states = d_ctr + nctr - 2;
    a.n_committed = d_ctr + nctr - 3;
    a.table = d_table; a.table_mask = slots - 1;
    a.arena = d_arena; a.acap = acap; a.hstack = d_hs; a.hcap = hcap;
    a.ctr = d_ctr; a.evbuf = d_ev; a.evcap = evcap;
    a.seed = o.seed ? o.seed : 0x2545f4914f6cdd1dull;
    a.inv_oom = o.inv_out_of_model ? 1 : 0;
    a.deadlock = o.check_deadlock ? 1 : 0;
    a.fifo = fifo ? 1 : 0;
    a.newpos = d_newpos; a.newpos_cap = kcap;
    std::vector<u64> h(nctr);
    HIPOK(hipEventCreate(&sc.e0)); HIPOK(hipEventCreate(&sc.e1));
    hipEvent_t e0 = sc.e0, e1 = sc.e1;
    // every kernel but tlg_keys_k takes the Args block (tlk::Args)
    auto launch_with = [&](hipFunction_t f, u64 blocks, unsigned bs, void** params) -> int {
      HIPOK(hipEventRecord(e0, 0));
      HIPOK(hipModuleLaunchKernel(f, (unsigned)blocks, 1, 1, bs, 1, 1, 0, 0, params, nullptr));
      HIPOK(hipEventRecord(e1, 0));
      HIPOK(hipEventSynchronize(e1));
      float ms = 0; (void)hipEventElapsedTime(&ms, e0, e1);
      r.seconds_kernels += ms / 1e3;
      r.levels.empty() ? void() : void(r.levels.back().kernel_ms += ms);
      HIPOK(hipMemcpy(h.data(), d_ctr, nctr * 8, hipMemcpyDeviceToHost));
      return 0;
    };
    auto launch = [&](hipFunction_t f, u64 blocks, unsigned bs) -> int {
      void* params[] = {&a};
      return launch_with(f, blocks, bs, params);
    };
    auto set_ctr = [&](u32 k, u64 v) -> int { HIPOK(hipMemcpy(d_ctr + k, &v, 8, hipMemcpyHostToDevice)); return 0; };
    r = RunResult();
    r.action_names = meta.actions;
    if (int rc = launch(f_init, 1, 64)) return rc;
    u64 first = 0, count = h[nctr - 2], gen_prev = h[C_GEN];
    r.generated = (int64_t)h[C_GEN];
    if (count) { r.depth = 1; r.levels.push_back({(int64_t)count, (int64_t)h[C_GEN], 0}); }
    const u64 grid = lanes / 64;
    u64 fifo_ev = ~0ull;                              // FIFO: the stop point's event word
    std::vector<int64_t> prior_gen(nact, 0), prior_dist(nact, 0);
    int64_t prior_generated = 0;
    while (count && !h[C_FLAG] && !h[C_CAP]) {
      if (o.max_depth && r.depth >= o.max_depth) { r.verdict = MC_VERDICT_DEPTH_LIMIT; r.left_on_queue = (int64_t)count; break; }
      a.first = first; a.count = count;
      r.levels.push_back({0, 0, 0});
      u64 fresh = 0;
      if (!fifo) {
        if (int rc = launch(f_expand, grid, 64)) return rc;
        fresh = h[nctr - 2] - (first + count);
      } else {
        prior_generated = (int64_t)h[C_GEN];
        for (int k = 0; k < nact; ++k) { prior_gen[k] = (int64_t)h[C_ACT + k]; prior_dist[k] = (int64_t)h[C_ACT + nact + k]; }
        if (set_ctr(C_EV, ~0ull) || set_ctr(C_NEWPOS, 0)) return MC_E_NO_DEVICE;
        a.wkeys = nullptr; a.n_w = 0; a.level_end = first + count;
        if (int rc = launch(f_expand, grid, 64)) return rc;   // pass 1: keys into the seen-set
        if (h[C_CAP]) { r.levels.pop_back(); break; }
        const u64 nw = h[C_NEWPOS];
        const u64 level_end = first + count;
        if (nw) {
          {   // tlg_keys_k(table, newpos, n, keys)
            const u64* kt = d_table; const u64* kn = d_newpos; u64 kcount = nw; u64* kk = d_keys;
            void* kp[] = {(void*)&kt, (void*)&kn, (void*)&kcount, (void*)&kk};
            if (int rc = launch_with(f_keys, std::min<u64>(4096, (nw + 255) / 256), 256, kp)) return rc;
          }
          if (tlagen_sort_keys(d_keys, d_sorted, nw, 64, &sc.sort_tmp, &sort_bytes, 0)) { err = "radix sort of the level's keys failed"; return MC_E_NO_DEVICE; }
          a.wkeys = d_sorted; a.n_w = nw; a.level_end = level_end;
          if (int rc = launch(f_mat, grid, 64)) return rc;     // pass 2: the winners, in key order
          const u64 total = level_end + nw;
          if (hipMemcpy(d_ctr + nctr - 2, &total, 8, hipMemcpyHostToDevice) != hipSuccess) { err = "counter write failed"; return MC_E_NO_DEVICE; }
          h[nctr - 2] = total;
        }
        fresh = nw;
        // the level is not complete at a stop: only completed levels are reported (as TLC does)
        if (h[C_CAP]) { r.levels.pop_back(); break; }
        if (h[C_EV] != ~0ull) { fifo_ev = h[C_EV]; r.levels.pop_back(); break; }
      }
      ++r.n_launches;
      r.levels.back().states = (int64_t)fresh;
      r.levels.back().generated = (int64_t)(h[C_GEN] - gen_prev);
      gen_prev = h[C_GEN];
      first += count; count = fresh;
      if (fresh) ++r.depth; else r.levels.pop_back();
    }
    const double t_loop = since();
    if (timing)
      std::fprintf(stderr, "tlagen timing: code object %.3f s, module load + allocation + clears %.3f s, level loop %.3f s "
                           "(kernels %.3f s), store %.1f GiB, arena %.1f GiB\n", t_co, t_setup - t_co, t_loop - t_setup,
                   r.seconds_kernels, store / 1073741824.0, (double)lanes * (acap + hcap) * 4 / 1073741824.0);
    if (!fifo && h[C_FLAG] && !h[C_CAP]) {   // (searched again in FIFO order by run())
      // tlagen_kernels.h C_KIND: 1/2 violation, 3 evaluation error, 4 deadlock, 5 invariant evaluation error
      static const char* const kinds[] = {"an event", "an invariant violation", "an invariant violation",
                                          "an evaluation error", "a deadlock", "an invariant evaluation error"};
      const u64 kd = h[C_KIND];
      workers_event_ = std::string(kd < 6 ? kinds[kd] : "an event") + " at depth " + std::to_string(r.depth + 1);
      again = true;
      return 0;
    }
    // on a store overflow some ids were handed out without their words: only the committed states
    // are stored (and ids are no longer dense, so traces and dumps are refused below)
    store_complete = h[nctr - 3] == h[nctr - 2];
    n_stored = store_complete ? h[nctr - 2] : h[nctr - 3];
    words_stored = std::min<u64>(h[nctr - 1], words_cap);
    r.generated = (int64_t)h[C_GEN];
    r.generated_in_model = (int64_t)h[C_GIN];
    r.distinct = (int64_t)n_stored;
    r.act_generated.resize(nact); r.act_distinct.resize(nact);
    for (int k = 0; k < nact; ++k) { r.act_generated[k] = (int64_t)h[C_ACT + k]; r.act_distinct[k] = (int64_t)h[C_ACT + nact + k]; }
    Printer pr{meta};
    auto trace_to = [&](u64 sid) {
      std::vector<u64> path;
      if (sid != ~0ull) chase(sid, path, d_parent, err);
      for (size_t i = path.size(); i-- > 0;) trace_step(path[i], d_parent, d_act, pr, r);
    };
    auto inv_name = [&](u64 i) { return i < meta.invariants.size() ? meta.invariants[i] : std::string("?"); };
    if (h[C_CAP]) {
      arena_overflow = (h[C_CAP] & 4) != 0;
      r.verdict = MC_VERDICT_CAPACITY_OVERFLOW;
      r.error = (h[C_CAP] & 4) ? "lane arena too small for one state's successors" : (h[C_CAP] & 2) ? "seen-set full"
              : (h[C_CAP] & 8) ? "a state has more than 2^24 successors" : "state store full";
    } else if (fifo_ev != ~0ull) {
      if (int rc = fifo_stop(a, fifo_ev, first, count, f_stop, grid, launch, h, nctr, prior_generated, prior_gen, prior_dist,
                             trace_to, inv_name, r, err)) return rc;
    } else if (h[C_FLAG]) {   // an event among the initial states (one lane, Init's order: TLC's)
      const u64 kind = h[C_KIND], sid = h[C_SID];
      trace_to(sid);
      if (kind == 1 || kind == 2) {
        r.verdict = MC_VERDICT_INVARIANT_VIOLATION;
        r.violated = inv_name(h[C_INV]);
        if (kind == 2) {   // the violating successor is outside the constraints: printed from the event buffer
          std::vector<u32> w(h[C_EWORDS]);
          (void)hipMemcpy(w.data(), d_ev, w.size() * 4, hipMemcpyDeviceToHost);
          const u64 ak = h[C_EACT];
          r.trace.push_back({ak < meta.actions.size() ? meta.actions[ak] : "?", pr.state(w.data())});
        }
      } else if (kind == 3) {
        r.verdict = MC_VERDICT_EVAL_ERROR;
        r.error = "evaluation error (tlv error bits " + std::to_string(h[C_INV]) + ") while computing the initial states";
      } else if (kind == 5) {   // TLC: "Evaluating invariant X failed." with the behavior up to the state
        r.verdict = MC_VERDICT_EVAL_ERROR;
        r.violated = inv_name(h[C_INV]);
        r.error = "Evaluating invariant " + r.violated + " failed.";
      } else {
        r.verdict = MC_VERDICT_DEADLOCK;
      }
      r.left_on_queue = (int64_t)count;
    }
    r.seed = a.seed;
    r.state_bytes = 0;
    r.seconds_total = std::chrono::duration<double>(std::chrono::steady_clock::now() - t_start).count();
    last = r;
    return 0;
  }

  // TLC's report at the FIFO stop point: the level's first event in key order (tlagen_kernels.h
  // C_EV), its counters (generated = successor lists of the parents up to the event's; distinct =
  // the new states before it in key order, the violating one included; left on queue = the rest of
  // the level's parents plus the new states so far) and the counterexample
  template <class Launch, class TraceTo, class InvName>
  int fifo_stop(KArgs& a, u64 ev, u64 first, u64 count, hipFunction_t f_stop, u64 grid, Launch& launch, std::vector<u64>& h,
                size_t nctr, int64_t prior_generated, const std::vector<int64_t>& prior_gen, const std::vector<int64_t>& prior_dist,
                TraceTo& trace_to, InvName& inv_name, RunResult& r, std::string& err) {
    const u64 key = ev >> 3, kind = ev & 7, rank = key >> 24, ord = key & ((1ull << 24) - 1);
    const int nact = (int)meta.actions.size();
    const u64 level_end = first + count, nw = a.n_w;
    const bool new_state = kind == 3 || kind == 5;   // EV_INV_ERROR_NEW / EV_VIOLATION_NEW
    // the winners before the event in key order (binary search over the sorted keys)
    u64 lo = 0, hi = a.wkeys ? nw : 0;
    while (lo < hi) {
      const u64 mid = (lo + hi) / 2;
      u64 kk = 0;
      HIPOK(hipMemcpy(&kk, a.wkeys + mid, 8, hipMemcpyDeviceToHost));
      if (kk < key || (kk == key && new_state)) lo = mid + 1; else hi = mid;
    }
    const u64 before = lo;
    // generated counts: re-derived over the parents [0, rank] (and the event successor captured)
    for (size_t k = 0; k < nctr - 3; ++k) if (k == C_GEN || (k >= C_ACT && k < (size_t)C_ACT + nact)) h[k] = 0;
    HIPOK(hipMemcpy(a.ctr, h.data(), (nctr - 3) * 8, hipMemcpyHostToDevice));
    a.stop_rank = rank; a.stop_ord = ord; a.stop_kind = (int)kind;
    if (int rc = launch(f_stop, std::min<u64>(grid, (rank + 64) / 64), 64)) return rc;
    r.generated = prior_generated + (int64_t)h[C_GEN];
    for (int k = 0; k < nact; ++k) r.act_generated[k] = prior_gen[k] + (int64_t)h[C_ACT + k];
    std::vector<u32> acts(before);
    if (before) HIPOK(hipMemcpy(acts.data(), a.act + level_end, before * 4, hipMemcpyDeviceToHost));
    for (int k = 0; k < nact; ++k) r.act_distinct[k] = prior_dist[k];
    for (u32 x : acts) if (x < (u32)nact) ++r.act_distinct[x];
    r.distinct = (int64_t)(level_end + before);
    r.left_on_queue = (int64_t)(count - rank - 1 + before);
    n_stored = level_end + before;
    const u64 parent_sid = first + rank;
    auto successor = [&]() {   // the event's successor, captured by tlg_stop_k
      std::vector<u32> w(h[C_EWORDS]);
      if (w.empty()) { err = "the stop point's successor was not re-derived"; return; }
      (void)hipMemcpy(w.data(), a.evbuf, w.size() * 4, hipMemcpyDeviceToHost);
      const u64 ak = h[C_EACT];
      Printer pr{meta};
      r.trace.push_back({ak < meta.actions.size() ? meta.actions[ak] : "?", pr.state(w.data())});
    };
    switch (kind) {
      case 0:   // EV_NEXT_ERROR
        r.verdict = MC_VERDICT_EVAL_ERROR;
        r.error = "evaluation error while computing the successors of the last state";
        trace_to(parent_sid);
        break;
      case 1:   // EV_DEADLOCK
        r.verdict = MC_VERDICT_DEADLOCK;
        trace_to(parent_sid);
        break;
      case 2:   // EV_INV_ERROR_OOM: a constraint / VIEW / invariant could not be evaluated on a successor
        r.verdict = MC_VERDICT_EVAL_ERROR;
        r.violated = inv_name(h[C_EVINV]);
        r.error = "evaluation error on a successor of the last state (a constraint, the VIEW or invariant " + r.violated + ")";
        trace_to(parent_sid);
        successor();
        r.depth += 1;
        break;
      case 3:   // EV_INV_ERROR_NEW
        r.verdict = MC_VERDICT_EVAL_ERROR;
        r.violated = inv_name(h[C_EVINV]);
        r.error = "Evaluating invariant " + r.violated + " failed.";
        trace_to(level_end + before - 1);
        r.depth += 1;
        break;
      case 4:   // EV_VIOLATION_OOM
        r.verdict = MC_VERDICT_INVARIANT_VIOLATION;
        r.violated = inv_name(h[C_EVINV]);
        trace_to(parent_sid);
        successor();
        r.depth += 1;
        break;
      default:  // EV_VIOLATION_NEW
        r.verdict = MC_VERDICT_INVARIANT_VIOLATION;
        r.violated = inv_name(h[C_EVINV]);
        trace_to(level_end + before - 1);
        r.depth += 1;
        break;
    }
    (void)err;
    return 0;
  }

  void chase(u64 sid, std::vector<u64>& path, u64* d_parent, std::string& err) {
    (void)err;
    while (sid != ~0ull && path.size() < 100000) {
      path.push_back(sid);
      u64 p = ~0ull;
      (void)hipMemcpy(&p, d_parent + sid, 8, hipMemcpyDeviceToHost);
      sid = p;
    }
  }
  void trace_step(u64 sid, u64* d_parent, u32* d_act, const Printer& pr, RunResult& r) {
    u64 off = 0, par = 0;
    u32 act = 0;
    (void)hipMemcpy(&off, d_offs + sid, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&par, d_parent + sid, 8, hipMemcpyDeviceToHost);
    (void)hipMemcpy(&act, d_act + sid, 4, hipMemcpyDeviceToHost);
    std::vector<u32> w(std::min<u64>(1u << 20, words_stored - off));
    (void)hipMemcpy(w.data(), d_words + off, w.size() * 4, hipMemcpyDeviceToHost);
    r.trace.push_back({par == ~0ull ? "Initial predicate" : act < meta.actions.size() ? meta.actions[act] : "?", pr.state(w.data())});
  }

  int dump_states(const std::string& path, std::string& err) override {
    if (!d_words) { err = "no run"; return MC_E_STATE; }
    if (!store_complete) { err = "the state store overflowed: the stored states are incomplete"; return MC_E_STATE; }
    std::vector<u32> w(words_stored);
    std::vector<u64> off(n_stored);
    HIPOK(hipMemcpy(w.data(), d_words, w.size() * 4, hipMemcpyDeviceToHost));
    HIPOK(hipMemcpy(off.data(), d_offs, off.size() * 8, hipMemcpyDeviceToHost));
    FILE* f = std::fopen(path.c_str(), "w");
    if (!f) { err = "cannot write " + path; return MC_E_IO; }
    Printer pr{meta};
    for (u64 i = 0; i < n_stored; ++i) {
      std::string s = pr.state(w.data() + off[i]);
      for (char& ch : s) if (ch == '\n') ch = ' ';
      std::fprintf(f, "%s\n", s.c_str());
    }
    std::fclose(f);
    return 0;
  }

  // single-GPU only: the sharded entry points are the hand-compiled families'
  int shard_open(const RunOpts&, int, int, std::string& err) override { err = "the generated path runs on one GPU"; return MC_E_UNSUPPORTED; }
  int shard_record_bytes(int) const override { return 0; }
  int shard_frontier(int64_t*, int64_t*) const override { return MC_E_UNSUPPORTED; }
  int shard_generate(int64_t, int64_t, int64_t*, std::string& err) override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_fill(int, void*, const int64_t*, std::string& err) override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_dedup(const void*, const int64_t*, int64_t*, std::string& err) override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_materialize(const void*, const int64_t*, std::string& err) override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_store(const void*, int64_t, std::string& err) override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_level_stats(int64_t*, std::string& err) override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_level_commit(const int64_t*, int*, std::string& err) override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_read_state(uint64_t, std::string&, uint64_t*, std::string& err) const override { err = "unsupported"; return MC_E_UNSUPPORTED; }
  int shard_violation(uint64_t*, std::string&, std::string&) const override { return MC_E_UNSUPPORTED; }
  const RunResult* shard_result() const override { return &last; }
};

}  // namespace

Backend* make_tlagen_backend(const std::string& tla_path, const CfgFile& cfg) { return new TlagenBackend(tla_path, cfg); }

}  // namespace rmc
