---------------------------- MODULE Recursive ----------------------------
\* Generated-path test module (written for this repo): RECURSIVE operators, self-recursive (SumSeq,
\* Fact) and mutually recursive (IsEven / IsOdd), bounded like TLC's stack: a runaway recursion is an
\* evaluation error, never a hang or a device fault (Runaway: Fact(-1)).
EXTENDS Integers, Sequences

VARIABLE s

RECURSIVE SumSeq(_)
SumSeq(q) == IF q = <<>> THEN 0 ELSE Head(q) + SumSeq(Tail(q))
RECURSIVE Fact(_)
Fact(k) == IF k = 0 THEN 1 ELSE k * Fact(k - 1)
RECURSIVE IsEven(_), IsOdd(_)
IsEven(k) == IF k = 0 THEN TRUE ELSE IsOdd(k - 1)
IsOdd(k) == IF k = 0 THEN FALSE ELSE IsEven(k - 1)

Init == s = <<>>

Next == \/ /\ Len(s) < 3
           /\ \E v \in 0..3 : s' = Append(s, v)
        \/ /\ Len(s) = 3
           /\ s' = Tail(s)

Inv == /\ SumSeq(s) <= 9
       /\ Fact(Len(s)) = IF Len(s) = 3 THEN 6 ELSE IF Len(s) = 2 THEN 2 ELSE 1
       /\ IsEven(SumSeq(s)) = (SumSeq(s) % 2 = 0)
       /\ IsOdd(SumSeq(s)) = ~IsEven(SumSeq(s))

\* negative controls: SumSeq(s) reaches 4 at depth 3 (<<1, 3>> or <<2, 2>> ..); Fact(-1) never ends
SumBelow4 == SumSeq(s) < 4
Runaway == Fact(Len(s) - 1) > 0
=============================================================================
