---------------------------- MODULE FunSets ----------------------------
\* Generated-path test module (written for this repo): function sets [S -> T] and record sets
\* [f : S, ...] as values (Init's choices, \E over a function set) and in membership tests that
\* must not build the set (TypeOK-style predicates over Nat and Seq, as raft_dricketts.tla:482-492).
EXTENDS Naturals, Sequences

CONSTANT S

VARIABLES f, r, q

Cell == [a : 0..2, b : {FALSE, TRUE}]

Init == /\ f \in [S -> {0}]
        /\ r \in [a : {0}, b : {FALSE, TRUE}]
        /\ q = <<>>

Next == \/ \E s \in S : /\ f[s] < 2
                        /\ f' = [f EXCEPT ![s] = f[s] + 1]
                        /\ UNCHANGED <<r, q>>
        \/ /\ r.a < 2
           /\ r' = [r EXCEPT !.a = r.a + 1]
           /\ UNCHANGED <<f, q>>
        \/ \E g \in [S -> {1}] : /\ f' = g
                                 /\ UNCHANGED <<r, q>>
        \/ /\ Len(q) < 2
           /\ q' = Append(q, r)
           /\ UNCHANGED <<f, r>>

Positive == { n \in Nat : n >= 1 }

TypeOK == /\ f \in [S -> 0..2]
          /\ f \in [S -> Nat]
          /\ r \in Cell
          /\ q \in Seq(Cell)
          /\ {r} \subseteq [a : Nat, b : BOOLEAN]
          /\ [s \in S |-> f[s] + 1] \in [S -> Positive]
          /\ r \notin [a : Nat]

\* negative controls: violated once some f[s] reaches 2 (depth 3), r.a reaches 2 (depth 3), q is non-empty (depth 2)
FBelow2 == f \in [S -> 0..1]
RBelow2 == r \in [a : 0..1, b : BOOLEAN]
QEmpty == q \in [{} -> Cell]
=============================================================================
