---------------------------- MODULE HigherOrder ----------------------------
\* Generated-path test module (written for this repo): operators with operator parameters (F(_)),
\* LAMBDA, and SelectSeq, as SequencesExt's Remove uses them (apalache_no_membership/SequencesExt.tla:
\* 66-68: Remove(s, e) == SelectSeq(s, LAMBDA t: t # e)).  Operator arguments are a LAMBDA, a global
\* operator by name, a LET operator, a standard-module operator (Append), and an operator parameter
\* passed on (Count's P into SelectSeq).
EXTENDS Naturals, Sequences

VARIABLES s, n

Remove(q, e) == SelectSeq(q, LAMBDA t : t # e)
Count(q, P(_)) == Len(SelectSeq(q, P))
Fold2(F(_, _), x, y) == F(x, y)
IsEven(x) == x % 2 = 0

Init == /\ s = <<>>
        /\ n = 0

Next == \/ /\ Len(s) < 3
           /\ \E v \in 0..2 : s' = Append(s, v)
           /\ UNCHANGED n
        \/ /\ Len(s) > 0
           /\ s' = Remove(s, Head(s))
           /\ n' = Fold2(LAMBDA a, b : (a + b) % 3, n, Head(s))

LetArg == LET AtLeast(x) == x >= n IN Count(s, AtLeast) = Len(SelectSeq(s, AtLeast))

TypeOK == /\ Count(s, IsEven) + Count(s, LAMBDA x : ~IsEven(x)) = Len(s)
          /\ SelectSeq(s, IsEven) = Remove(Remove(s, 1), 3)
          /\ LetArg
          /\ Remove(Remove(s, 0), 0) = Remove(s, 0)
          /\ Len(Fold2(Append, s, 1)) = Len(s) + 1
          /\ n \in 0..2

\* negative controls: violated once s holds two zeros (depth 3), once n reaches 2
FewZeros == Count(s, LAMBDA x : x = 0) < 2
NBelow2 == n < 2
=============================================================================
