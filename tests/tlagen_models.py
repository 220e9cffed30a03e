"""TEST INFRASTRUCTURE: an independent Python restatement of configs/tlagen/TokenRing.tla (the
repo's own front-end test module) — the expected counts for the generated path on the CPU
(test_tlagen.py) and the GPU (test_gpu_tlagen.py)."""

PROC = (1, 2, 3)
VAL = ("a", "b")
MAX_LOG = 2


def _succ(p):   # Succ(p): CASE p = Max(Proc) -> Min(Proc) [] OTHER -> Min({q \in Proc : q > p})
    return min(PROC) if p == max(PROC) else min(q for q in PROC if q > p)


def token_ring(max_depth=0, stop_when_all_full=False):
    """BFS over (token, logs, sent, passes, crashes); returns the run's counts."""
    init = (min(PROC), ((),) * len(PROC), frozenset(), 0, 0)
    seen = {init}
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
                if s not in seen:
                    seen.add(s)
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
