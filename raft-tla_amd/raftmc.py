"""Host-side mirror of TLC's model-checking contract over the raftmc C ABI.

The reference path is TLC's command line:
    java -cp tla2tools.jar tlc2.TLC [-workers N] [-config F.cfg] [-deadlock] F.tla
This module exposes the same arguments with the same meaning:

    res = check("configs/raft_original_mc.tla", config="configs/c2.cfg")
    res.distinct, res.generated, res.depth, res.verdict, res.trace_text
    tlc_main(["-config", "c2.cfg", "raft_original_mc.tla"])   # TLC-style stdout + exit code

Every call goes to libraftmc.so (HIP kernels for gfx950).  There is no CPU
fallback: without the built library or a usable GPU the calls raise.
"""
import ctypes
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("RAFTMC_LIB") or os.path.join(_HERE, "_build", "libraftmc.so")   # RAFTMC_LIB: experiment builds only
ABI_VERSION = 3

VERDICTS = {0: "OK", 1: "INVARIANT_VIOLATION", 2: "EVAL_ERROR", 3: "CAPACITY_OVERFLOW", 4: "DEADLOCK", 5: "DEPTH_LIMIT"}
MC_COMPAT_INV_OUT_OF_MODEL = 0x1
MC_COMPAT_SYM_TLC = 0x2
MC_COMPAT_DISJUNCT_COPIES = 0x4

# every symbol include/raftmc.h declares
EXPORTS = ["mc_opts_init", "mc_default_opts", "mc_open", "mc_run", "mc_summary", "mc_action_stats", "mc_level_stats", "mc_kernel_stats",
           "mc_trace", "mc_report", "mc_dump_states", "mc_describe", "mc_exit_code", "mc_free",
           "mc_close", "mc_last_error", "mc_shard_open", "mc_shard_record_bytes", "mc_shard_frontier",
           "mc_shard_generate", "mc_shard_fill", "mc_shard_dedup", "mc_shard_materialize", "mc_shard_store",
           "mc_shard_level_stats", "mc_shard_level_commit", "mc_shard_read_state", "mc_shard_violation",
           "mc_set_history_prefix", "mc_shard_layout", "mc_shard_select", "mc_shard_event_stats",
           "mc_collision_observed", "mc_rccl_unique_id", "mc_shard_run_rccl", "mc_shard_run_loopback",
           "mc_set_checkpoint", "mc_set_recover", "mc_action_location", "mc_source_hash", "mc_set_fault_injection", "mc_release_device_memory", "mc_set_fp_slice"]


class McOpts(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("device", ctypes.c_int32), ("n_gpus", ctypes.c_int32),
                ("workers", ctypes.c_int32), ("fp_table_bytes", ctypes.c_uint64),
                ("state_store_bytes", ctypes.c_uint64), ("max_depth", ctypes.c_int64), ("seed", ctypes.c_uint64),
                ("tlc_compat_flags", ctypes.c_uint32), ("check_deadlock", ctypes.c_int32),
                ("block_size", ctypes.c_int32), ("same_device", ctypes.c_int32), ("frontend", ctypes.c_int32),
                ("count_final_level", ctypes.c_int32), ("reserved", ctypes.c_int32 * 4)]


class McSummary(ctypes.Structure):
    _fields_ = [("generated", ctypes.c_int64), ("distinct", ctypes.c_int64), ("left_on_queue", ctypes.c_int64),
                ("depth", ctypes.c_int64), ("verdict", ctypes.c_int32), ("n_actions", ctypes.c_int32),
                ("collision_prob_optimistic", ctypes.c_double), ("collision_prob_observed", ctypes.c_double),
                ("seconds_total", ctypes.c_double), ("seconds_kernels", ctypes.c_double),
                ("fp_seed", ctypes.c_uint64), ("algo_bytes", ctypes.c_double),
                ("generated_in_model", ctypes.c_int64), ("state_bytes", ctypes.c_int32), ("n_launches", ctypes.c_int32),
                ("violated", ctypes.c_char * 64), ("spec", ctypes.c_char * 32), ("seen_set_probes", ctypes.c_int64),
                ("reserved", ctypes.c_int64 * 8)]


class RaftMCError(RuntimeError):
    def __init__(self, code, msg):
        super().__init__("raftmc error %d: %s" % (code, msg))
        self.code = code


_lib = None


def source_hash():
    """The library's source identity as raft-tla_amd/Makefile computes it (SRCHASH), or None when the
    sources are not next to the package."""
    import hashlib
    here = os.path.dirname(os.path.abspath(__file__))
    csrc = os.path.join(here, "csrc")
    hdr = os.path.join(os.path.dirname(here), "include", "raftmc.h")
    if not (os.path.isdir(csrc) and os.path.exists(hdr)):
        return None
    names = [os.path.join("csrc", f) for f in os.listdir(csrc) if f.endswith((".h", ".cpp", ".hip"))]
    tg = os.path.join(csrc, "tlagen")   # the front end (tlv_text.h is derived from its sources)
    if os.path.isdir(tg):
        names += [os.path.join("csrc", "tlagen", f) for f in os.listdir(tg) if f.endswith((".h", ".cpp", ".hip")) and f != "tlv_text.h"]
    h = hashlib.sha256()
    for f in sorted(names):
        with open(os.path.join(here, f), "rb") as fh:
            h.update(fh.read())
    with open(hdr, "rb") as fh:
        h.update(fh.read())
    return h.hexdigest()[:16]


def load_library(path=LIB_PATH):
    """Load libraftmc.so (raises if it has not been built: there is no fallback)."""
    global _lib
    if _lib is not None:
        return _lib
    if not os.path.exists(path):
        raise RaftMCError(-5, "libraftmc.so not built at %s (run __graft_entry__.build())" % path)
    lib = ctypes.CDLL(path)
    lib.mc_source_hash.restype = ctypes.c_char_p
    want = source_hash()
    got = lib.mc_source_hash().decode()
    # RAFTMC_LIB names an experiment build (scripts/build_variant.sh) made beside the product: its
    # identity is the experiment's, not the tree's
    if want is not None and got != want and not os.environ.get("RAFTMC_LIB"):
        raise RaftMCError(-5, "libraftmc.so at %s was built from other sources (library %s, tree %s): rebuild it "
                              "(make -C raft-tla_amd)" % (path, got, want))
    P = ctypes.c_void_p
    lib.mc_default_opts.argtypes = [ctypes.POINTER(McOpts)]
    lib.mc_opts_init.argtypes = [ctypes.POINTER(McOpts), ctypes.c_int32]
    lib.mc_open.argtypes = [ctypes.c_char_p, ctypes.c_char_p, ctypes.POINTER(McOpts), ctypes.POINTER(P)]
    lib.mc_run.argtypes = [P]
    lib.mc_summary.argtypes = [P, ctypes.POINTER(McSummary)]
    lib.mc_action_stats.argtypes = [P, ctypes.c_int32, ctypes.POINTER(ctypes.c_char_p),
                                    ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_int64)]
    lib.mc_level_stats.argtypes = [P, ctypes.c_int32, ctypes.POINTER(ctypes.c_int64),
                                   ctypes.POINTER(ctypes.c_int64), ctypes.POINTER(ctypes.c_double)]
    lib.mc_kernel_stats.argtypes = [P, ctypes.c_int32, ctypes.POINTER(ctypes.c_char_p), ctypes.POINTER(ctypes.c_double),
                                    ctypes.POINTER(ctypes.c_double), ctypes.POINTER(ctypes.c_int64)]
    for f in ("mc_trace", "mc_report", "mc_describe"):
        getattr(lib, f).argtypes = [P, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.mc_dump_states.argtypes = [P, ctypes.c_char_p]
    lib.mc_action_location.argtypes = [P, ctypes.c_char_p, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t)]
    lib.mc_set_history_prefix.argtypes = [P, ctypes.c_char_p, ctypes.c_char_p]
    lib.mc_collision_observed.argtypes = [P, ctypes.POINTER(ctypes.c_double)]
    lib.mc_set_checkpoint.argtypes = [P, ctypes.c_char_p, ctypes.c_int32]
    lib.mc_set_recover.argtypes = [P, ctypes.c_char_p]
    lib.mc_set_fault_injection.argtypes = [P, ctypes.c_int32, ctypes.c_int64]
    lib.mc_set_fp_slice.argtypes = [P, ctypes.c_int32]
    lib.mc_release_device_memory.argtypes = [P]
    lib.mc_exit_code.argtypes = [P]
    lib.mc_free.argtypes = [P]
    lib.mc_close.argtypes = [P]
    lib.mc_last_error.argtypes = [P]
    lib.mc_last_error.restype = ctypes.c_char_p
    _lib = lib
    return lib


class Result:
    """Outcome of one model-checking run (TLC's summary lines + trace)."""

    def __init__(self, **kw):
        self.__dict__.update(kw)

    def __repr__(self):
        return "Result(verdict=%s, generated=%d, distinct=%d, depth=%d)" % (
            self.verdict, self.generated, self.distinct, self.depth)


class ModelChecker:
    """One raftmc handle: mc_open on construction, mc_run in run()."""

    # sym_tlc: SYMMETRY as TLC applies it (the default, MC_COMPAT_SYM_TLC); False = the orbit mode
    # disjunct_copies: TLC's generated count of a disjunctive guard (MC_COMPAT_DISJUNCT_COPIES, default)
    def __init__(self, spec, config=None, workers=1, deadlock=True, device=0, max_depth=0,
                 fp_table_bytes=0, state_store_bytes=0, seed=0, inv_out_of_model=True, sym_tlc=True, disjunct_copies=True, n_gpus=1,
                 same_device=False, frontend="auto", count_final_level=False):
        """n_gpus > 1: one search over the GPUs device .. device + n_gpus - 1 (owner-partitioned
        fingerprints, one host thread per GPU inside the library, in-process RCCL); same_device: all
        those ranks on `device` (the multi-GPU level loop on a one-GPU machine).  frontend: "auto"
        (hand-compiled kernels for the two Raft families, the generated path otherwise),
        "generated" (the SANY-subset front end for any module, or a .gen.hip source), "hand".
        count_final_level (raft_original, workers != 1, with max_depth): the last level's states are
        counted and checked but not stored, so the store needs room for the levels before it only."""
        self.lib = load_library()
        if config is None:
            config = spec[:-4] + ".cfg" if spec.endswith(".tla") else spec + ".cfg"
        o = McOpts()
        # the binding's own ABI version (the header it mirrors), not the library's (include/raftmc.h)
        if self.lib.mc_opts_init(ctypes.byref(o), ABI_VERSION):
            raise RaftMCError(-1, "libraftmc.so does not implement ABI version %d" % ABI_VERSION)
        o.device, o.workers, o.max_depth = device, workers, max_depth
        o.n_gpus, o.same_device = n_gpus, 1 if same_device else 0
        o.frontend = {"auto": 0, "generated": 1, "hand": 2}[frontend]
        o.count_final_level = 1 if count_final_level else 0
        o.fp_table_bytes, o.state_store_bytes, o.seed = fp_table_bytes, state_store_bytes, seed
        o.check_deadlock = 1 if deadlock else 0
        o.tlc_compat_flags = ((MC_COMPAT_INV_OUT_OF_MODEL if inv_out_of_model else 0) | (MC_COMPAT_SYM_TLC if sym_tlc else 0) |
                              (MC_COMPAT_DISJUNCT_COPIES if disjunct_copies else 0))
        self.h = ctypes.c_void_p()
        rc = self.lib.mc_open(spec.encode(), config.encode(), ctypes.byref(o), ctypes.byref(self.h))
        if rc:
            msg = self.lib.mc_last_error(self.h).decode() if self.h else "open failed"
            self.close()
            raise RaftMCError(rc, msg)

    def _text(self, fn):
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        rc = fn(self.h, ctypes.byref(p), ctypes.byref(n))
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())
        s = ctypes.string_at(p, n.value).decode()
        self.lib.mc_free(p)
        return s

    def set_history_prefix(self, constraint, trace_text):
        """Golden history trace (TLA+ value text) of a punctuated-search constraint
        (CommitWhenConcurrentLeaders_unique / MajorityOfClusterRestarts_constraint)."""
        rc = self.lib.mc_set_history_prefix(self.h, constraint.encode(), trace_text.encode())
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def set_checkpoint(self, path, every_levels=1):
        """TLC -checkpoint: write the BFS state to `path` every `every_levels` levels (None: off)."""
        rc = self.lib.mc_set_checkpoint(self.h, path.encode() if path else None, every_levels if path else 0)
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def set_recover(self, path):
        """TLC -recover: the next run() resumes the search saved in `path`."""
        rc = self.lib.mc_set_recover(self.h, path.encode() if path else None)
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def release_device_memory(self):
        """Free the device buffers this handle keeps between runs (the next run() allocates again)."""
        rc = self.lib.mc_release_device_memory(self.h)
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def set_fault_injection(self, rank, depth):
        """Tests only: in the next sharded run rank `rank` leaves the level loop at `depth` (rank < 0: off)."""
        rc = self.lib.mc_set_fault_injection(self.h, rank, depth)
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def set_fp_slice(self, entries):
        """Tests only: cap tlc_membership's LDS bag slice (0: every parent to the fallback kernel; < 0: default)."""
        rc = self.lib.mc_set_fp_slice(self.h, entries)
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def collision_observed(self):
        """TLC's "based on the actual fingerprints" estimate (1 / min fingerprint gap); GPU sort."""
        v = ctypes.c_double()
        rc = self.lib.mc_collision_observed(self.h, ctypes.byref(v))
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())
        return v.value

    def action_location(self, action):
        """TLC's trace-header location of `action` ("line L1, col C1 to line L2, col C2 of module M"),
        or None when the spec module (and the modules it EXTENDS) holds no definition of it."""
        p, n = ctypes.c_void_p(), ctypes.c_size_t()
        if self.lib.mc_action_location(self.h, action.encode(), ctypes.byref(p), ctypes.byref(n)):
            return None
        s = ctypes.string_at(p, n.value).decode()
        self.lib.mc_free(p)
        return s

    def describe(self):
        import json
        return json.loads(self._text(self.lib.mc_describe))

    def run(self):
        rc = self.lib.mc_run(self.h)
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())
        return self.summary()

    def summary(self):
        """Result of the last completed run (mc_run, or a finished sharded BFS)."""
        s = McSummary()
        self.lib.mc_summary(self.h, ctypes.byref(s))
        actions = {}
        for k in range(s.n_actions):
            name, g, d = ctypes.c_char_p(), ctypes.c_int64(), ctypes.c_int64()
            self.lib.mc_action_stats(self.h, k, ctypes.byref(name), ctypes.byref(g), ctypes.byref(d))
            actions[name.value.decode()] = [g.value, d.value]
        levels = []
        for k in range(s.depth):
            st, g, ms = ctypes.c_int64(), ctypes.c_int64(), ctypes.c_double()
            if self.lib.mc_level_stats(self.h, k, ctypes.byref(st), ctypes.byref(g), ctypes.byref(ms)) == 0:
                levels.append((st.value, g.value, ms.value))
        kernels = {}
        for k in range(16):
            name, ms, ab, nl = ctypes.c_char_p(), ctypes.c_double(), ctypes.c_double(), ctypes.c_int64()
            if self.lib.mc_kernel_stats(self.h, k, ctypes.byref(name), ctypes.byref(ms), ctypes.byref(ab), ctypes.byref(nl)):
                break
            kernels[name.value.decode()] = {"ms": ms.value, "algo_bytes": ab.value, "launches": nl.value}
        return Result(verdict=VERDICTS.get(s.verdict, str(s.verdict)), generated=s.generated, distinct=s.distinct,
                      kernels=kernels,
                      left_on_queue=s.left_on_queue, depth=s.depth, violated=s.violated.decode(),
                      spec=s.spec.decode(), actions=actions, levels=levels,
                      collision_prob_optimistic=s.collision_prob_optimistic,
                      collision_prob_observed=s.collision_prob_observed,
                      seconds=s.seconds_total, kernel_seconds=s.seconds_kernels, fp_seed=s.fp_seed,
                      algo_bytes=s.algo_bytes, generated_in_model=s.generated_in_model,
                      seen_set_probes=s.seen_set_probes,
                      state_bytes=s.state_bytes, n_launches=s.n_launches,
                      trace_text=self._text(self.lib.mc_trace), report=self._text(self.lib.mc_report),
                      error=self.lib.mc_last_error(self.h).decode(),
                      exit_code=self.lib.mc_exit_code(self.h))

    def dump_states(self, path):
        rc = self.lib.mc_dump_states(self.h, path.encode())
        if rc:
            raise RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def close(self):
        if getattr(self, "h", None) and self.h:
            self.lib.mc_close(self.h)
            self.h = ctypes.c_void_p()

    def __enter__(self):
        return self

    def __exit__(self, *a):
        self.close()


def check(spec, config=None, **kw):
    """Model-check `spec` with `config` (TLC: tlc2.TLC -config config spec)."""
    with ModelChecker(spec, config, **kw) as mc:
        return mc.run()


def tlc_main(argv):
    """TLC-compatible argv entry point; prints the report, returns TLC's exit code."""
    spec, config, kw = None, None, {}
    checkpoint, recover = None, None
    it = iter(argv)
    for a in it:
        if a == "-config":
            config = next(it)
        elif a == "-checkpoint":                 # raftmc: levels between checkpoints (TLC: minutes)
            checkpoint = int(next(it))
        elif a == "-recover":
            recover = next(it)
        elif a == "-workers":
            kw["workers"] = int(next(it))
        elif a == "-deadlock":
            kw["deadlock"] = False
        elif a == "-depth":
            kw["max_depth"] = int(next(it))
        elif a == "-countfinal":                 # raftmc: with -depth, the last level counted, not stored
            kw["count_final_level"] = True
        elif a == "-gpus":
            kw["n_gpus"] = int(next(it))
        elif a == "-frontend":                   # raftmc: auto (default) | generated | hand
            kw["frontend"] = next(it)
            if kw["frontend"] not in ("auto", "generated", "hand"):
                raise ValueError("-frontend auto|generated|hand")
        elif a == "-symmetry":                   # raftmc: tlc (TLC's rule, default) | orbit
            v = next(it)
            if v not in ("tlc", "orbit"):
                raise ValueError("-symmetry tlc|orbit")
            kw["sym_tlc"] = v == "tlc"
        else:
            spec = a
    with ModelChecker(spec, config, **kw) as mc:
        if checkpoint:   # TLC keeps its checkpoints under states/ next to the spec
            path = recover or os.path.join(os.path.dirname(os.path.abspath(spec)), "states", "raftmc.ckpt")
            os.makedirs(os.path.dirname(path), exist_ok=True)
            mc.set_checkpoint(path, checkpoint)
        if recover:
            mc.set_recover(recover)
        res = mc.run()
    print(res.report, end="")
    return res.exit_code
