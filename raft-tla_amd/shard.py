"""Multi-GPU BFS: owner-partitioned fingerprints, one process per GPU.

Per BFS level and frontier chunk every rank runs (include/raftmc.h mc_shard_*):

  generate   expand the local chunk; route in-model successor fingerprints to
             their owner ((fp >> 32) mod world)             -> ROUTE records
  exchange 1 all-to-all of ROUTE records (16 B: fp, slot)
  dedup      owner inserts them into its local seen-set      -> REPLY records
  exchange 2 all-to-all of REPLY records back (8 B: slot)
  materialize the generating rank re-derives the acknowledged new states
  exchange 3 all-to-all of STATES records to the owner (80 B: state, parent, fp)
  store      the owner appends them to its part of the next level

then one all-reduce of the level counters (sum; max for the error, violation
and deadlock flags).

tlc_membership (VIEW vars) needs TLC's single-worker FIFO first-found order,
so its driver (fifo_sharded_bfs) decides winners once per level: keys are
global (global parent rank * slots + slot), the owner keeps the minimum key per
fingerprint over all chunks, then sends each winning key back to the rank
that generated it (select + one all-to-all); the generator sorts and
re-derives its winners in key order, and a rebalancing all-to-all gives every
rank an equal contiguous slice of the next level.  The result (counts,
per-action distinct counts, the kept representatives, counterexamples) is the
single-GPU result.  All payloads are device tensors moved with
torch.distributed (backend "nccl" = RCCL over xGMI on MI355X); with the "gloo"
backend they are staged through host memory (used by the CPU tests and to
run several ranks on one GPU).  Parent pointers carry the owner rank, so a
counterexample is reassembled by chasing them across ranks.
"""
import ctypes

import torch
import torch.distributed as dist

from . import raftmc as _rm

ROUTE, REPLY, STATES = 0, 1, 2
RCCL_ID_BYTES = 128    # sizeof(ncclUniqueId)
NSTAT = 72
FLAG_SLICE = slice(3, 6)   # error flags, violation, deadlock: reduced with MAX


class LibShard:
    """ctypes view of the mc_shard_* entry points of one raftmc handle."""

    def __init__(self, checker, rank, world, open_shard=True):
        self.mc, self.lib, self.h = checker, checker.lib, checker.h
        self.world = world
        lib = self.lib
        P, I64P = ctypes.c_void_p, ctypes.POINTER(ctypes.c_int64)
        lib.mc_shard_open.argtypes = [P, ctypes.c_int32, ctypes.c_int32]
        lib.mc_shard_record_bytes.argtypes = [P, ctypes.c_int32]
        lib.mc_shard_frontier.argtypes = [P, I64P, I64P]
        lib.mc_shard_generate.argtypes = [P, ctypes.c_int64, ctypes.c_int64, I64P]
        lib.mc_shard_fill.argtypes = [P, ctypes.c_int32, P, I64P]
        lib.mc_shard_dedup.argtypes = [P, P, I64P, I64P]
        lib.mc_shard_materialize.argtypes = [P, P, I64P]
        lib.mc_shard_store.argtypes = [P, P, ctypes.c_int64]
        lib.mc_shard_level_stats.argtypes = [P, I64P]
        lib.mc_shard_level_commit.argtypes = [P, I64P, ctypes.POINTER(ctypes.c_int32)]
        lib.mc_shard_read_state.argtypes = [P, ctypes.c_uint64, ctypes.POINTER(P), ctypes.POINTER(ctypes.c_size_t),
                                            ctypes.POINTER(ctypes.c_uint64)]
        lib.mc_shard_violation.argtypes = [P, ctypes.POINTER(ctypes.c_uint64), ctypes.POINTER(P), ctypes.POINTER(P)]
        lib.mc_shard_layout.argtypes = [P, I64P]
        lib.mc_shard_select.argtypes = [P, I64P]
        lib.mc_shard_event_stats.argtypes = [P, I64P, I64P]
        lib.mc_rccl_unique_id.argtypes = [P, P, ctypes.c_size_t]
        lib.mc_shard_run_rccl.argtypes = [P, ctypes.c_int32, ctypes.c_int32, P, ctypes.c_size_t]
        if open_shard:
            self._check(lib.mc_shard_open(self.h, rank, world))
        self.rec_bytes = {w: lib.mc_shard_record_bytes(self.h, w) for w in (ROUTE, REPLY, STATES)}

    def _check(self, rc):
        if rc:
            raise _rm.RaftMCError(rc, self.lib.mc_last_error(self.h).decode())

    def _arr(self, xs=None):
        a = (ctypes.c_int64 * self.world)()
        if xs is not None:
            for i, x in enumerate(xs):
                a[i] = int(x)
        return a

    @staticmethod
    def _ptr(t):
        return ctypes.c_void_p(t.data_ptr() if t.numel() else 0)

    def rccl_unique_id(self):
        buf = ctypes.create_string_buffer(RCCL_ID_BYTES)
        self._check(self.lib.mc_rccl_unique_id(self.h, buf, RCCL_ID_BYTES))
        return buf.raw

    def run_rccl(self, rank, world, uid):
        buf = ctypes.create_string_buffer(uid, RCCL_ID_BYTES)
        self._check(self.lib.mc_shard_run_rccl(self.h, rank, world, buf, RCCL_ID_BYTES))

    def frontier(self):
        s, c = ctypes.c_int64(), ctypes.c_int64()
        self._check(self.lib.mc_shard_frontier(self.h, ctypes.byref(s), ctypes.byref(c)))
        return s.value, c.value

    def generate(self, begin, count):
        out = self._arr()
        self._check(self.lib.mc_shard_generate(self.h, begin, count, out))
        return list(out)

    def fill(self, what, dst, offsets):
        self._check(self.lib.mc_shard_fill(self.h, what, self._ptr(dst), self._arr(offsets)))

    def dedup(self, recv, counts):
        out = self._arr()
        self._check(self.lib.mc_shard_dedup(self.h, self._ptr(recv), self._arr(counts), out))
        return list(out)

    def materialize(self, acks, counts):
        self._check(self.lib.mc_shard_materialize(self.h, self._ptr(acks), self._arr(counts)))

    def store(self, states, n):
        self._check(self.lib.mc_shard_store(self.h, self._ptr(states), n))

    def layout(self, counts):
        self._check(self.lib.mc_shard_layout(self.h, self._arr(counts)))

    def select(self):
        out = self._arr()
        self._check(self.lib.mc_shard_select(self.h, out))
        return list(out)

    def event_stats(self, g):
        a = (ctypes.c_int64 * NSTAT)(*[int(x) for x in g])
        out = (ctypes.c_int64 * NSTAT)()
        self._check(self.lib.mc_shard_event_stats(self.h, a, out))
        return list(out)

    def level_stats(self):
        a = (ctypes.c_int64 * NSTAT)()
        self._check(self.lib.mc_shard_level_stats(self.h, a))
        return list(a)

    def level_commit(self, g):
        a = (ctypes.c_int64 * NSTAT)(*[int(x) for x in g])
        done = ctypes.c_int32()
        self._check(self.lib.mc_shard_level_commit(self.h, a, ctypes.byref(done)))
        return bool(done.value)

    def read_state(self, gid):
        p, n, meta = ctypes.c_void_p(), ctypes.c_size_t(), ctypes.c_uint64()
        self._check(self.lib.mc_shard_read_state(self.h, gid, ctypes.byref(p), ctypes.byref(n), ctypes.byref(meta)))
        s = ctypes.string_at(p, n.value).decode()
        self.lib.mc_free(p)
        return s, meta.value

    def violation(self):
        parent, a, t = ctypes.c_uint64(), ctypes.c_void_p(), ctypes.c_void_p()
        if self.lib.mc_shard_violation(self.h, ctypes.byref(parent), ctypes.byref(a), ctypes.byref(t)):
            return None
        act, text = ctypes.string_at(a).decode(), ctypes.string_at(t).decode()
        self.lib.mc_free(a)
        self.lib.mc_free(t)
        return parent.value, act, text


class Exchanger:
    """all-to-all of variable-size byte payloads between the ranks of a process group."""

    def __init__(self, world, device, group=None):
        self.world, self.device, self.group = world, device, group
        backend = dist.get_backend(group) if world > 1 else "local"
        self.host_staged = backend == "gloo"

    def counts(self, mine):
        if self.world == 1:
            return list(mine)
        dev = "cpu" if self.host_staged else self.device
        t = torch.tensor(mine, dtype=torch.int64, device=dev)
        out = torch.empty_like(t)
        dist.all_to_all_single(out, t, group=self.group)
        return out.tolist()

    def payload(self, send, send_counts, recv_counts, rec_bytes):
        """send: uint8 device tensor holding the per-destination segments in rank order."""
        rb = [c * rec_bytes for c in recv_counts]
        if self.world == 1:
            return send
        if self.host_staged:
            s = send.cpu()
            r = torch.empty(sum(rb), dtype=torch.uint8)
            dist.all_to_all_single(r, s, rb, [c * rec_bytes for c in send_counts], group=self.group)
            return r.to(self.device)
        r = torch.empty(sum(rb), dtype=torch.uint8, device=self.device)
        dist.all_to_all_single(r, send, rb, [c * rec_bytes for c in send_counts], group=self.group)
        torch.cuda.synchronize(self.device)
        return r

    def allreduce_stats(self, st):
        if self.world == 1:
            return list(st)
        dev = "cpu" if self.host_staged else self.device
        t = torch.tensor(st, dtype=torch.int64, device=dev)
        m = t[FLAG_SLICE].clone()
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        dist.all_reduce(m, op=dist.ReduceOp.MAX, group=self.group)
        t[FLAG_SLICE] = m
        out = t.tolist()
        if out[FLAG_SLICE.start]:
            # error flags are a bit set: report the OR over ranks, not the largest word
            # (every rank sees the same max, so every rank takes this extra all-gather)
            acc = 0
            for f in self.allgather(st[FLAG_SLICE.start]):
                acc |= f
            out[FLAG_SLICE.start] = acc
        return out

    def allreduce_sum(self, st):
        if self.world == 1:
            return list(st)
        dev = "cpu" if self.host_staged else self.device
        t = torch.tensor(st, dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.SUM, group=self.group)
        return t.tolist()

    def allgather(self, x):
        if self.world == 1:
            return [int(x)]
        dev = "cpu" if self.host_staged else self.device
        t = torch.tensor([int(x)], dtype=torch.int64, device=dev)
        out = [torch.empty_like(t) for _ in range(self.world)]
        dist.all_gather(out, t, group=self.group)
        return [int(o.item()) for o in out]

    def allreduce_max(self, x):
        if self.world == 1:
            return x
        dev = "cpu" if self.host_staged else self.device
        t = torch.tensor([x], dtype=torch.int64, device=dev)
        dist.all_reduce(t, op=dist.ReduceOp.MAX, group=self.group)
        return int(t.item())

    def broadcast_obj(self, obj, src):
        if self.world == 1:
            return obj
        box = [obj]
        dist.broadcast_object_list(box, src=src, group=self.group)
        return box[0]


def _offsets(counts):
    off, acc = [], 0
    for c in counts:
        off.append(acc)
        acc += c
    return off


def sharded_bfs(shard, ex, rank, device):
    """Drive the level loop; returns the (rank-0) trace list on a violation."""
    world = ex.world
    while True:
        front, chunk = shard.frontier()
        nchunks = ex.allreduce_max((front + chunk - 1) // chunk if front else 0)
        for c in range(nchunks):
            begin = c * chunk
            count = max(0, min(chunk, front - begin))
            send_counts = shard.generate(min(begin, front), count)
            recv_counts = ex.counts(send_counts)
            rb = shard.rec_bytes[ROUTE]
            send = torch.empty(sum(send_counts) * rb, dtype=torch.uint8, device=device)
            shard.fill(ROUTE, send, _offsets(send_counts))
            recv = ex.payload(send, send_counts, recv_counts, rb)
            reply_counts = shard.dedup(recv, recv_counts)           # replies[r] go back to rank r
            ack_counts = ex.counts(reply_counts)
            rb = shard.rec_bytes[REPLY]
            send = torch.empty(sum(reply_counts) * rb, dtype=torch.uint8, device=device)
            shard.fill(REPLY, send, _offsets(reply_counts))
            acks = ex.payload(send, reply_counts, ack_counts, rb)
            shard.materialize(acks, ack_counts)                      # states for owner r = acks from r
            rb = shard.rec_bytes[STATES]
            send = torch.empty(sum(ack_counts) * rb, dtype=torch.uint8, device=device)
            shard.fill(STATES, send, _offsets(ack_counts))
            states = ex.payload(send, ack_counts, reply_counts, rb)
            shard.store(states, sum(reply_counts))
        g = ex.allreduce_stats(shard.level_stats())
        if shard.level_commit(g):
            break
    return _trace(shard, ex, rank, world)


def _overlap(a0, a1, b0, b1):
    return max(0, min(a1, b1) - max(a0, b0))


def rebalance_counts(news, rank, world):
    """The level's new states are one key-ordered run per rank (news[g] states at global offset
    sum(news[:g])); the next level gives rank k the slice [k*D//W, (k+1)*D//W).  Returns
    (send_counts, recv_counts) of this rank, per peer in rank order."""
    total = sum(news)
    off = _offsets(news)
    tgt = [(k * total // world, (k + 1) * total // world) for k in range(world)]
    mine = (off[rank], off[rank] + news[rank])
    send = [_overlap(mine[0], mine[1], t0, t1) for t0, t1 in tgt]
    recv = [_overlap(off[g], off[g] + news[g], tgt[rank][0], tgt[rank][1]) for g in range(world)]
    return send, recv


def fifo_sharded_bfs(shard, ex, rank, device):
    """Level loop for FIFO-ranked specs (tlc_membership); returns the trace on a stop."""
    world = ex.world
    while True:
        front, chunk = shard.frontier()
        counts = ex.allgather(front)
        shard.layout(counts)
        nchunks = max((c + chunk - 1) // chunk for c in counts) if chunk else 0
        for c in range(nchunks):
            begin = c * chunk
            count = max(0, min(chunk, front - begin))
            send_counts = shard.generate(min(begin, front), count)
            recv_counts = ex.counts(send_counts)
            rb = shard.rec_bytes[ROUTE]
            send = torch.empty(sum(send_counts) * rb, dtype=torch.uint8, device=device)
            shard.fill(ROUTE, send, _offsets(send_counts))
            recv = ex.payload(send, send_counts, recv_counts, rb)
            shard.dedup(recv, recv_counts)
        reply_counts = shard.select()                              # winners generated by rank r go to r
        ack_counts = ex.counts(reply_counts)
        rb = shard.rec_bytes[REPLY]
        send = torch.empty(sum(reply_counts) * rb, dtype=torch.uint8, device=device)
        shard.fill(REPLY, send, _offsets(reply_counts))
        acks = ex.payload(send, reply_counts, ack_counts, rb)
        shard.materialize(acks, ack_counts)
        st = shard.level_stats()
        news = ex.allgather(st[0])
        g = ex.allreduce_stats(st)
        if g[4]:                                                   # the level's first event stops the search
            e = ex.allreduce_sum(shard.event_stats(g))
            g[30], g[31], g[32] = e[30], e[31], e[32]
            g[8:30], g[40:62] = e[8:30], e[40:62]                  # per-action counters at the stop point
        if shard.level_commit(g):
            break
        send_counts, recv_counts = rebalance_counts(news, rank, world)
        rb = shard.rec_bytes[STATES]
        send = torch.empty(sum(send_counts) * rb, dtype=torch.uint8, device=device)
        shard.fill(STATES, send, _offsets(send_counts))
        states = ex.payload(send, send_counts, recv_counts, rb)
        shard.store(states, sum(recv_counts))
    return _trace(shard, ex, rank, world)


def _local_trace(shards):
    """_trace for ranks that live in one process: the lowest violating rank's head, then the
    parent chain read from each state's owner (gid bits 37..39)."""
    head = next((v for v in (sh.violation() for sh in shards) if v is not None), None)
    if head is None:
        return None
    parent, act, text = head
    if parent == (1 << 64) - 1:
        return [("<Initial predicate>", text)]
    trace = [(act, text)]
    gid = parent
    names = shards[0].mc.describe()["actions"]
    for _ in range(1 << 20):
        text, meta = shards[(gid >> 37) & 7].read_state(gid)
        if meta == (1 << 64) - 1:
            trace.append(("<Initial predicate>", text))
            break
        trace.append((names[(meta >> 16) & 0xFF], text))
        gid = meta >> 24
    trace.reverse()
    return trace


def check_loopback(spec, config, world, device_index=0, history_prefixes=None, dump=None, **kw):
    """The library's native sharded level loop (the one mc_shard_run_rccl drives over RCCL; for
    tlc_membership the FIFO-ranked loop of csrc/fifo_shard_loop.h) for `world` ranks inside this
    process, all on one device, exchanging through device-to-device copies
    (mc_shard_run_loopback).  Returns one raftmc Result per rank, the counterexample (if any)
    reassembled across ranks as .trace_text on each; dump: a path prefix, each rank's kept states
    are written to dump.rank<r>."""
    mcs = [_rm.ModelChecker(spec, config, device=device_index, **kw) for _ in range(world)]
    try:
        for m in mcs:
            for con, text in (history_prefixes or {}).items():
                m.set_history_prefix(con, text)
        lib = mcs[0].lib
        lib.mc_shard_run_loopback.argtypes = [ctypes.POINTER(ctypes.c_void_p), ctypes.c_int32]
        hs = (ctypes.c_void_p * world)(*[m.h for m in mcs])
        rc = lib.mc_shard_run_loopback(hs, world)
        if rc:
            errs = [lib.mc_last_error(m.h).decode() for m in mcs]
            raise _rm.RaftMCError(rc, "; ".join(e for e in errs if e) or "loopback run failed")
        shards = [LibShard(m, r, world, open_shard=False) for r, m in enumerate(mcs)]
        trace = _local_trace(shards)
        out = [m.summary() for m in mcs]
        name = next((r.violated for r in out if r.violated), "")
        for m, res in zip(mcs, out):
            if res.verdict == "INVARIANT_VIOLATION":
                res.violated = name
            if trace:
                res.trace_text = trace_text(trace, m.action_location)
        if dump:
            for r, m in enumerate(mcs):
                m.dump_states("%s.rank%d" % (dump, r))
        return out
    finally:
        for m in mcs:
            m.close()


def _trace(shard, ex, rank, world):
    v = shard.violation()
    # the lowest rank that recorded a violation reports it
    top = ex.allreduce_max(world - rank if v is not None else 0)
    if top == 0:
        return None
    src = world - top
    head = ex.broadcast_obj(v, src)
    if head is None:
        return None
    parent, act, text = head
    if parent == (1 << 64) - 1:                  # the stop is at the initial state itself
        return [("<Initial predicate>", text)]
    trace = [(act, text)]
    gid = parent
    for _ in range(1 << 20):
        owner = (gid >> 37) & 7
        mine = shard.read_state(gid) if owner == rank else None
        text, meta = ex.broadcast_obj(mine, owner)
        if meta == (1 << 64) - 1:
            trace.append(("<Initial predicate>", text))
            break
        act_id = (meta >> 16) & 0xFF
        trace.append((shard.mc.describe()["actions"][act_id], text))
        gid = meta >> 24
    trace.reverse()
    return trace


def trace_text(trace, locate=None):
    """TLC's "State k: <Action line .. of module M>" blocks; `locate(action)` gives the location
    text (ModelChecker.action_location) or None, which leaves the header as "<Action>"."""
    out = []
    for k, (act, text) in enumerate(trace):
        loc = locate(act) if (locate and k) else None
        head = "<Initial predicate>" if k == 0 else ("<%s %s>" % (act, loc) if loc else "<%s>" % act)
        out.append("State %d: %s\n%s\n" % (k + 1, head, text))
    return "\n".join(out) + ("\n" if out else "")


class ShardedChecker:
    """One rank of a sharded model-checking job; run() may be called repeatedly
    (device buffers are kept, the seen-set is re-zeroed by mc_shard_open)."""

    def __init__(self, spec, config, rank, world, device_index=0, group=None, history_prefixes=None,
                 transport="auto", **kw):
        """transport: "rccl" = the library's native level loop over its own RCCL communicator
        (mc_shard_run_rccl; both spec families), "torch" = this module's level loop with
        torch.distributed collectives, "auto" = rccl when the process group's backend is nccl
        (RCCL), else torch."""
        self.rank, self.world = rank, world
        self.device = torch.device("cuda", device_index)
        if kw.get("count_final_level") and transport == "torch":
            raise ValueError("count_final_level runs in the library's native level loop (transport rccl), not shard.py's")
        self.mc = _rm.ModelChecker(spec, config, device=device_index, **kw)
        for con, text in (history_prefixes or {}).items():   # punctuated-search golden traces
            self.mc.set_history_prefix(con, text)
        self.ex = Exchanger(world, self.device, group)
        self.fifo = self.mc.describe()["spec"] == "tlc_membership"
        if transport == "auto":
            backend = dist.get_backend(group) if dist.is_initialized() else "none"
            transport = "rccl" if backend == "nccl" else "torch"
        self.transport = transport
        self._uid = None

    def run(self):
        if self.transport == "rccl":
            shard = LibShard(self.mc, self.rank, self.world, open_shard=False)
            if self._uid is None:   # one communicator per job, cached by the library across runs
                self._uid = self.ex.broadcast_obj(shard.rccl_unique_id() if self.rank == 0 else None, 0)
            shard.run_rccl(self.rank, self.world, self._uid)
            trace = _trace(shard, self.ex, self.rank, self.world)
        else:
            shard = LibShard(self.mc, self.rank, self.world)
            trace = (fifo_sharded_bfs if self.fifo else sharded_bfs)(shard, self.ex, self.rank, self.device)
        res = self.mc.summary()
        if res.verdict == "INVARIANT_VIOLATION":   # the name is known on the violating ranks only
            top = self.ex.allreduce_max(self.world - self.rank if res.violated else 0)
            if top:
                res.violated = self.ex.broadcast_obj(res.violated, self.world - top)
        if trace:
            res.trace_text = trace_text(trace, self.mc.action_location)
        return res

    def close(self):
        self.mc.close()


def check_sharded(spec, config, rank, world, device_index=0, group=None, **kw):
    # kw may carry transport= (see ShardedChecker)
    """Run one sharded BFS on this rank (call on every rank of the group).

    Returns the raftmc Result (identical on every rank) with .trace_text
    assembled across ranks."""
    sc = ShardedChecker(spec, config, rank, world, device_index, group, **kw)
    try:
        return sc.run()
    finally:
        sc.close()
