---------------------------- MODULE TokenRing ----------------------------
\* A test module for raftmc's generated path (written for this repo; not part of the
\* reference).  Processes on a ring pass a token; the holder appends a value to its log or
\* passes the token on; a process with a non-empty log may lose its last entry.  It exercises
\* what the front end compiles: records, sequences, sets, functions, EXCEPT with @ and field
\* paths, CHOOSE, LET, CASE, IF, \E with two bound variables, UNCHANGED of a tuple definition.
EXTENDS Naturals, Sequences, FiniteSets, TLC

CONSTANTS Proc, Val, MaxLog

VARIABLES token, logs, sent, history

vars == <<token, logs, sent, history>>
static == <<logs, sent>>
tokenlogs == <<token, logs>>   \* a VIEW that leaves out sent and history (TokenRing_view.cfg)

Min(S) == CHOOSE x \in S : \A y \in S : x <= y
Max(S) == CHOOSE x \in S : \A y \in S : x >= y

Succ(p) == CASE p = Max(Proc) -> Min(Proc)
             [] OTHER -> Min({q \in Proc : q > p})

Init == /\ token = Min(Proc)
        /\ logs = [p \in Proc |-> <<>>]
        /\ sent = {}
        /\ history = [passes |-> 0, crashes |-> 0]

Write(p, v) ==
    /\ token = p
    /\ Len(logs[p]) < MaxLog
    /\ logs' = [logs EXCEPT ![p] = Append(@, [val |-> v, by |-> p])]
    /\ sent' = sent \cup {v}
    /\ UNCHANGED <<token, history>>

Pass(p) ==
    /\ token = p
    /\ LET q == Succ(p)
       IN token' = q
    /\ history' = [history EXCEPT !.passes = IF @ < 3 THEN @ + 1 ELSE @]
    /\ UNCHANGED static

Lose(p) ==
    /\ logs[p] /= <<>>
    /\ history.crashes < 2
    /\ logs' = [logs EXCEPT ![p] = SubSeq(@, 1, Len(@) - 1)]
    /\ history' = [history EXCEPT !["crashes"] = history.crashes + 1]
    /\ UNCHANGED <<token, sent>>

Next == \/ \E p \in Proc, v \in Val : Write(p, v)
        \/ \E p \in Proc : Pass(p)
        \/ \E p \in Proc : Lose(p)

TokenInRing == token \in Proc
LogsBounded == \A p \in Proc : Len(logs[p]) <= MaxLog
SentCoversLogs == \A p \in Proc : \A i \in DOMAIN logs[p] : logs[p][i].val \in sent /\ logs[p][i].by = p
\* test-only: reachable, so its check reports a violation
NotAllFull == ~ \A p \in Proc : Len(logs[p]) = MaxLog
=============================================================================
