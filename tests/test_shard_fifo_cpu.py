"""N>1 path for FIFO-ranked specs (tlc_membership) on CPU: the level loop of
raft-tla_amd/shard.py (fifo_sharded_bfs: layout, per-chunk route + dedup,
per-level select + reply, key-ordered materialize, event stop point,
rebalancing all-to-all) with world_size 2-3 over gloo, driven by a host-side
stand-in implementing the same mc_shard_* contract as the membership backend.

The toy system is VIEW-like: a state is (v, h), only v is fingerprinted, and h
(a "history" register outside the view) feeds the successor relation and the
state constraint, so which representative of a view class is kept depends on
the exploration order.  The sharded run must reproduce the single-process FIFO
(TLC single worker) result exactly: counts, depth, level sizes, the kept
representatives and, on a violation, TLC's stop-point counters and a shortest
trace."""
import hashlib
import importlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

shard = importlib.import_module("raft-tla_amd.shard")

P = 4099
NI = 4
EV_VIOLATION = 3


def succ(s):
    v, h = s
    return [((3 * v + 1) % P, (h + 1) % 4), ((5 * v + 2) % P, h), ((v + 7) % P, (h * 2 + 1) % 4), ((v * v + 3) % P, 0)]


def in_model(s):
    v, h = s
    return not (h == 3 and v % 5 == 0)


def fp_of(v):
    return int.from_bytes(hashlib.blake2b(v.to_bytes(8, "little"), digest_size=8).digest(), "little") | 1


def reference_fifo(target=None):
    """Single-worker FIFO BFS with first-found representatives (TLC under VIEW)."""
    seen, kept, front, gen, depth, levels = {0}, {(0, 0)}, [(0, 0)], 1, 1, [1]
    while front:
        nxt = []
        for s in front:
            ys = succ(s)
            gen += len(ys)
            for y in ys:
                if in_model(y) and y[0] not in seen:
                    seen.add(y[0])
                    kept.add(y)
                    nxt.append(y)
                    if y[0] == target:
                        return dict(distinct=len(seen), generated=gen, depth=depth + 1, kept=kept, violation=True)
        if nxt:
            depth += 1
            levels.append(len(nxt))
        front = nxt
    return dict(distinct=len(seen), generated=gen, depth=depth, kept=kept, levels=levels, violation=False)


class FakeChecker:
    def describe(self):
        return {"spec": "tlc_membership", "actions": ["A0", "A1", "A2", "A3"]}


class FakeFifoShard:
    """Host stand-in for LibShard over the toy system, with the membership backend's contract."""

    def __init__(self, rank, world, chunk, target):
        self.rank, self.world, self.chunk, self.target = rank, world, chunk, target
        self.mc = FakeChecker()
        self.rec_bytes = {shard.ROUTE: 16, shard.REPLY: 8, shard.STATES: 16}
        self.store_states, self.meta = [], []
        self.table = {}                      # fp -> (level, key) of the kept representative
        self.level = 0
        self.viol = None
        self.res = dict(generated=1, distinct=1, depth=1, levels=[1], verdict="OK")
        if (fp_of(0) >> 32) % world == rank:
            self.table[fp_of(0)] = (0, 0)
        self.level_begin, self.level_count = 0, 0
        if rank == 0:
            self.store_states.append((0, 0))
            self.meta.append((1 << 64) - 1)
            self.level_count = 1
        self.done = False

    # -- the mc_shard_* contract
    def frontier(self):
        return (0 if self.done else self.level_count), self.chunk

    def layout(self, counts):
        self.B = sum(counts[:self.rank])
        self.F = sum(counts)
        self.kstart = [sum(counts[:g]) * NI for g in range(self.world)]
        self.lvl, self.nsucc, self.gen, self.gin = [], [0] * self.level_count, 0, 0
        self.event, self.new = None, []

    def generate(self, begin, count):
        self.route = [[] for _ in range(self.world)]
        for t in range(count):
            q = begin + t
            s = self.store_states[self.level_begin + q]
            ys = succ(s)
            self.nsucc[q] = len(ys)
            self.gen += len(ys)
            for k, y in enumerate(ys):
                if in_model(y):
                    self.gin += 1
                    f = fp_of(y[0])
                    self.route[(f >> 32) % self.world].append((f, (self.B + q) * NI + k))
        return [len(r) for r in self.route]

    def fill(self, what, dst, offsets):
        recs = {shard.ROUTE: getattr(self, "route", None), shard.REPLY: getattr(self, "replies", None),
                shard.STATES: getattr(self, "outstates", None)}[what]
        for r in range(self.world):
            if not recs or not recs[r]:
                continue
            flat = [v - (1 << 64) if v >= 1 << 63 else v
                    for rec in recs[r] for v in (rec if isinstance(rec, tuple) else (rec,))]
            t = torch.tensor(flat, dtype=torch.int64).view(torch.uint8)
            o = offsets[r] * self.rec_bytes[what]
            dst[o:o + t.numel()] = t

    def dedup(self, recv, counts):
        data = recv.view(torch.int64).tolist() if recv.numel() else []
        for i in range(sum(counts)):
            f, key = data[2 * i] & ((1 << 64) - 1), data[2 * i + 1]
            cur = self.table.get(f)
            if cur is None or (cur[0] == self.level + 1 and key < cur[1]):
                self.table[f] = (self.level + 1, key)
            self.lvl.append((f, key))
        return [0] * self.world

    def select(self):
        self.replies = [[] for _ in range(self.world)]
        for f, key in self.lvl:
            if self.table[f] == (self.level + 1, key):
                g = max(q for q in range(self.world) if key >= self.kstart[q])
                self.replies[g].append(key)
        return [len(r) for r in self.replies]

    def materialize(self, acks, counts):
        keys = sorted(acks.view(torch.int64).tolist() if acks.numel() else [])
        self.sorted = keys
        out = []
        for key in keys:
            R, k = divmod(key, NI)
            gid = self.level_begin + (R - self.B)
            y = succ(self.store_states[gid])[k]
            out.append((y, (((self.rank << 37) | gid) << 24) | (k << 16)))
            if y[0] == self.target:
                e = key << 2 | EV_VIOLATION
                self.event = e if self.event is None else min(self.event, e)
        self.new = out

    def level_stats(self):
        st = [0] * shard.NSTAT
        st[0], st[1], st[2] = len(self.new), self.gen, self.gin
        st[4] = (1 << 62) - self.event if self.event is not None else 0
        st[6] = self.level_count
        return st

    def event_stats(self, g):
        st = [0] * shard.NSTAT
        ev = (1 << 62) - g[4]
        key = ev >> 2
        R = key // NI
        st[30] = sum(n for q, n in enumerate(self.nsucc) if self.B + q <= R)
        st[31] = sum(1 for k in self.sorted if k <= key)
        if self.B <= R < self.B + self.level_count:
            gid = self.level_begin + (R - self.B)
            y = succ(self.store_states[gid])[key % NI]
            self.viol = ((self.rank << 37) | gid, "A%d" % (key % NI), "s = %r" % (y,))
        return st

    def level_commit(self, g):
        r = self.res
        if g[4]:
            r["generated"] += g[30]
            r["distinct"] += g[31]
            r["depth"] = self.level + 2
            r["verdict"] = "INVARIANT_VIOLATION"
            self.done = True
            return True
        r["generated"] += g[1]
        r["distinct"] += g[0]
        if g[0]:
            r["levels"].append(g[0])
            r["depth"] += 1
        self.level += 1
        self.outstates = None
        self.done = g[0] == 0
        return self.done

    def store(self, states, n):
        data = states.view(torch.int64).tolist() if states.numel() else []
        self.level_begin = len(self.store_states)
        for i in range(n):
            packed = data[2 * i]
            self.store_states.append((packed >> 8, packed & 255))
            self.meta.append(data[2 * i + 1] & ((1 << 64) - 1))
        self.level_count = n

    def read_state(self, gid):
        local = gid & ((1 << 37) - 1)
        return "s = %r" % (self.store_states[local],), self.meta[local]

    def violation(self):
        return self.viol


def _pack_states(fs):
    """STATES records for the rebalance: (v << 8 | h, meta) per new state, key order."""
    return [((y[0] << 8) | y[1], m) for y, m in fs.new]


class RecordingShard(FakeFifoShard):
    """Hooks fill(STATES) to emit the key-ordered new states as one run (as the backend does)."""

    def fill(self, what, dst, offsets):
        if what == shard.STATES:
            recs = _pack_states(self)
            flat = [v - (1 << 64) if v >= 1 << 63 else v for rec in recs for v in rec]
            if flat:
                t = torch.tensor(flat, dtype=torch.int64).view(torch.uint8)
                dst[:t.numel()] = t
            return
        super().fill(what, dst, offsets)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, chunk, target, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fs = RecordingShard(rank, world, chunk, target)
    ex = shard.Exchanger(world, torch.device("cpu"))
    trace = shard.fifo_sharded_bfs(fs, ex, rank, torch.device("cpu"))
    q.put((rank, fs.res, sorted(fs.store_states), trace))
    dist.destroy_process_group()


def run_world(world, chunk, target=None):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, chunk, target, q)) for r in range(world)]
    for p in ps:
        p.start()
    out = sorted(q.get(timeout=120) for _ in ps)
    for p in ps:
        p.join(timeout=60)
    return out


@pytest.mark.parametrize("world,chunk", [(2, 50), (2, 100000), (3, 37)])
def test_fifo_sharded_bfs_matches_single_worker(world, chunk):
    ref = reference_fifo()
    out = run_world(world, chunk)
    for rank, res, stored, trace in out:
        assert (res["distinct"], res["generated"], res["depth"]) == (ref["distinct"], ref["generated"], ref["depth"])
        assert res["levels"] == ref["levels"]
        assert trace is None
    kept = [s for o in out for s in o[2]]
    assert len(kept) == ref["distinct"] and set(kept) == ref["kept"]   # the same first-found representatives
    sizes = [len(o[2]) for o in out]
    assert min(sizes) > ref["distinct"] // (2 * world)                 # rebalancing spreads the levels


def test_fifo_sharded_stop_point_and_trace():
    target = 2024
    ref = reference_fifo(target)
    assert ref["violation"]
    out = run_world(2, 41, target)
    res, trace = out[0][1], out[0][3]
    assert res["verdict"] == "INVARIANT_VIOLATION"
    assert (res["distinct"], res["generated"], res["depth"]) == (ref["distinct"], ref["generated"], ref["depth"])
    assert trace is not None and len(trace) == ref["depth"]
    states = [eval(t[1].split("=", 1)[1]) for t in trace]
    assert states[0] == (0, 0) and states[-1][0] == target
    assert all(b in succ(a) for a, b in zip(states, states[1:]))
