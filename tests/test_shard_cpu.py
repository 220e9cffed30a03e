"""N>1 path on CPU: the sharded-BFS orchestration (raft-tla_amd/shard.py) with
world_size 2 over gloo, driven by a host-side stand-in for the per-rank device
work (a toy transition system with the same mc_shard_* contract).  Checks that
owner-partitioned exploration with the three all-to-all exchanges per chunk
finds exactly the single-process BFS result (distinct, generated, depth) and
reassembles a shortest counterexample across ranks."""
import hashlib
import importlib
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

shard = importlib.import_module("raft-tla_amd.shard")

P = 20011            # toy state space: integers mod P, Init = 0


def succ(x):
    return [(3 * x + 1) % P, (5 * x + 2) % P, (x + 7) % P, (x * x + 3) % P]


def fp_of(x):
    return int.from_bytes(hashlib.blake2b(x.to_bytes(8, "little"), digest_size=8).digest(), "little") | 1


def in_model(x):
    return x % 97 != 13


def reference_bfs(target=None):
    seen, front, gen, depth = {0}, [0], 1, 1
    while front:
        nxt = []
        for x in front:
            for y in succ(x):
                gen += 1
                if in_model(y) and y not in seen:
                    seen.add(y)
                    nxt.append(y)
                    if y == target:
                        return len(seen), gen, depth + 1
        if nxt:
            depth += 1
        front = nxt
    return len(seen), gen, depth


class FakeChecker:
    def describe(self):
        return {"actions": ["A0", "A1", "A2", "A3"]}


class FakeShard:
    """Host stand-in for LibShard: same calls, toy successor function."""
    NI = 4

    def __init__(self, rank, world, chunk, target):
        self.rank, self.world, self.chunk, self.target = rank, world, chunk, target
        self.mc = FakeChecker()
        self.rec_bytes = {shard.ROUTE: 16, shard.REPLY: 8, shard.STATES: 24}
        self.store_states, self.meta, self.seen = [], [], set()
        self.level_begin = self.level_count = 0
        self.new = 0
        self.gen = 0
        self.viol = None
        f0 = fp_of(0)
        if (f0 >> 32) % world == rank:
            self.store_states.append(0)
            self.meta.append((1 << 64) - 1)
            self.seen.add(f0)
            self.level_count = 1

    def frontier(self):
        return self.level_count, self.chunk

    def generate(self, begin, count):
        self.cb, self.cc = self.level_begin + begin, count
        self.route = [[] for _ in range(self.world)]
        for t in range(count):
            x = self.store_states[self.cb + t]
            for k, y in enumerate(succ(x)):
                self.gen += 1
                if in_model(y):
                    f = fp_of(y)
                    self.route[(f >> 32) % self.world].append((f, k * count + t))
        return [len(r) for r in self.route]

    def fill(self, what, dst, offsets):
        if what == shard.ROUTE:
            recs = self.route
        elif what == shard.REPLY:
            recs = self.replies
        else:
            recs = self.outstates
        for r in range(self.world):
            if not recs[r]:
                continue
            flat = [v - (1 << 64) if v >= 1 << 63 else v
                    for rec in recs[r] for v in (rec if isinstance(rec, tuple) else (rec,))]
            t = torch.tensor(flat, dtype=torch.int64).view(torch.uint8)
            o = offsets[r] * self.rec_bytes[what]
            dst[o:o + t.numel()] = t

    def dedup(self, recv, counts):
        data = recv.view(torch.int64).tolist() if recv.numel() else []
        self.replies, pos = [], 0
        for r in range(self.world):
            out = []
            for i in range(counts[r]):
                f, slot = data[2 * (pos + i)], data[2 * (pos + i) + 1]
                f &= (1 << 64) - 1
                if f not in self.seen:
                    self.seen.add(f)
                    out.append(slot)
            self.replies.append(out)
            pos += counts[r]
        return [len(x) for x in self.replies]

    def materialize(self, acks, counts):
        data = acks.view(torch.int64).tolist() if acks.numel() else []
        self.outstates, pos = [], 0
        for r in range(self.world):
            out = []
            for i in range(counts[r]):
                slot = data[pos + i]
                k, t = divmod(slot, self.cc)
                gid = self.cb + t
                y = succ(self.store_states[gid])[k]
                meta = ((self.rank << 37 | gid) << 24) | (k << 16) | k
                out.append((y, meta, 0))
                if y == self.target and self.viol is None:
                    self.viol = ((self.rank << 37) | gid, "A%d" % k, "x = %d" % y)
            self.outstates.append(out)
            pos += counts[r]

    def store(self, states, n):
        data = states.view(torch.int64).tolist() if states.numel() else []
        for i in range(n):
            self.store_states.append(data[3 * i])
            self.meta.append(data[3 * i + 1] & ((1 << 64) - 1))
        self.new += n

    def level_stats(self):
        st = [0] * shard.NSTAT
        st[0], st[1], st[4] = self.new, self.gen, 1 if self.viol else 0
        return st

    def level_commit(self, g):
        self.total_gen = getattr(self, "total_gen", 1) + g[1]
        self.gen = 0
        self.level_begin += self.level_count
        self.level_count, self.new = self.new, 0
        self.depth = getattr(self, "depth", 1) + (1 if g[0] else 0)
        self.distinct = getattr(self, "distinct", 1) + g[0]
        return g[0] == 0 or g[4] > 0

    def read_state(self, gid):
        local = gid & ((1 << 37) - 1)
        return "x = %d" % self.store_states[local], self.meta[local]

    def violation(self):
        return self.viol


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, chunk, target, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    fs = FakeShard(rank, world, chunk, target)
    ex = shard.Exchanger(world, torch.device("cpu"))
    trace = shard.sharded_bfs(fs, ex, rank, torch.device("cpu"))
    q.put((rank, fs.distinct, fs.total_gen, fs.depth, len(fs.store_states), trace))
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


@pytest.mark.parametrize("world,chunk", [(2, 64), (2, 100000), (3, 50)])
def test_sharded_bfs_matches_single_process(world, chunk):
    distinct, gen, depth = reference_bfs()
    out = run_world(world, chunk)
    for rank, d, g, dep, stored, trace in out:
        assert (d, g, dep) == (distinct, gen, depth)
        assert trace is None
    assert sum(o[4] for o in out) == distinct          # every state stored on exactly one owner
    assert all(o[4] > distinct // (3 * world) for o in out)   # owner partitioning spreads the states


def test_sharded_counterexample_spans_ranks():
    target = 4321
    distinct, gen, depth = reference_bfs(target)
    out = run_world(2, 37, target)
    trace = out[0][5]
    assert trace is not None and trace[-1][1] == "x = %d" % target
    assert len(trace) == depth                      # shortest: BFS depth of the target
    assert trace[0][1] == "x = 0"
    xs = [int(t[1].split("=")[1]) for t in trace]
    assert all(b in succ(a) for a, b in zip(xs, xs[1:]))
