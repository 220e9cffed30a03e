"""TEST INFRASTRUCTURE: an independent Python restatement of configs/tlagen/TokenRing.tla (the
repo's own front-end test module) — the expected counts for the generated path on the CPU
(test_tlagen.py) and the GPU (test_gpu_tlagen.py)."""

PROC = (1, 2, 3)
VAL = ("a", "b")
MAX_LOG = 2


def _succ(p):   # Succ(p): CASE p = Max(Proc) -> Min(Proc) [] OTHER -> Min({q \in Proc : q > p})
    return min(PROC) if p == max(PROC) else min(q for q in PROC if q > p)


def token_ring(max_depth=0, stop_when_all_full=False, view=False):
    """BFS over (token, logs, sent, passes, crashes); returns the run's counts.  view: TLC's
    `VIEW tokenlogs` (configs/tlagen/TokenRing_view.cfg) in TLC's single-worker FIFO
    order -- states are told apart by their view <<token, logs>>, and the one kept per view is the
    first found (parents in queue order, successors in Next's enumeration order), whose history
    (crashes) decides its own Lose successors."""
    init = (min(PROC), ((),) * len(PROC), frozenset(), 0, 0)
    key = (lambda s: (s[0], s[1])) if view else (lambda s: s)
    seen = {key(init)}
    frontier = [init]
    levels = [1]
    gen = {"Write": 0, "Pass": 0, "Lose": 0}
    dist = {"Write": 0, "Pass": 0, "Lose": 0}
    generated = 1
    depth = 1
    while frontier:
        nxt = []
        for (tok, logs, sent, passes, crashes) in frontier:
            succs = []
            for i, p in enumerate(PROC):   # Write(p, v)
                for v in VAL:
                    if tok == p and len(logs[i]) < MAX_LOG:
                        nl = logs[:i] + (logs[i] + ((v, p),),) + logs[i + 1:]
                        succs.append(("Write", (tok, nl, sent | {v}, passes, crashes)))
            for i, p in enumerate(PROC):   # Pass(p)
                if tok == p:
                    succs.append(("Pass", (_succ(p), logs, sent, passes + 1 if passes < 3 else passes, crashes)))
            for i, p in enumerate(PROC):   # Lose(p)
                if logs[i] and crashes < 2:
                    nl = logs[:i] + (logs[i][:-1],) + logs[i + 1:]
                    succs.append(("Lose", (tok, nl, sent, passes, crashes + 1)))
            for act, s in succs:
                generated += 1
                gen[act] += 1
                if key(s) not in seen:
                    seen.add(key(s))
                    dist[act] += 1
                    nxt.append(s)
                    if stop_when_all_full and all(len(l) == MAX_LOG for l in s[1]):
                        return dict(verdict="INVARIANT_VIOLATION", depth=depth + 1)
        if nxt:
            depth += 1
            levels.append(len(nxt))
        frontier = nxt
    return dict(verdict="OK", generated=generated, distinct=len(seen), depth=depth, levels=levels,
                actions={k: [gen[k], dist[k]] for k in gen})


FACT = {n: (1 if n == 0 else None) for n in range(7)}
for _n in range(1, 7):
    FACT[_n] = _n * FACT[_n - 1]


def rec_fun(invariant=None):
    """BFS over configs/tlagen/RecFun.tla (x, bag): Next = tick \\/ \\E k : decrement.  `invariant`:
    None, "FactNot24" or "SumNot7"; returns the run's counts, or the violation depth."""
    init = (0, (0, 0, 0))
    seen = {init}
    frontier = [init]
    levels = [1]
    generated = 1
    depth = 1
    bad = {None: lambda s: False, "FactNot24": lambda s: FACT[s[0]] == 24, "SumNot7": lambda s: sum(s[1]) == 7}[invariant]
    while frontier:
        nxt = []
        for (x, bag) in frontier:
            succs = []
            nb = list(bag)
            if sum(bag) < 9:
                nb[x % 3] += 1
            succs.append(((x + 1) % 7, tuple(nb)))
            if sum(bag) > 0:
                for k in range(3):
                    if bag[k] > 0:
                        b2 = list(bag)
                        b2[k] -= 1
                        succs.append((x, tuple(b2)))
            for s in succs:
                generated += 1
                if s not in seen:
                    seen.add(s)
                    nxt.append(s)
                    if bad(s):
                        return dict(verdict="INVARIANT_VIOLATION", depth=depth + 1)
        if nxt:
            depth += 1
            levels.append(len(nxt))
        frontier = nxt
    return dict(verdict="OK", generated=generated, distinct=len(seen), depth=depth, levels=levels)
