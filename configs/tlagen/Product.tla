---------------------------- MODULE Product ----------------------------
\* Generated-path test module (written for this repo): Cartesian products S \X T (\X is not
\* associative: A \X B \X C is a set of triples, (A \X B) \X C a set of pairs) and tuple-bound
\* quantifiers \E <<a, b>> \in S, in actions and in expressions.
EXTENDS Naturals, FiniteSets

VARIABLES p, q

Pairs == {0, 1} \X {0, 1, 2}

Init == /\ p \in Pairs
        /\ q = <<0, 0, 0>>

Next == \/ /\ \E <<a, b>> \in Pairs : /\ a # p[1]
                                      /\ p' = <<a, b>>
           /\ UNCHANGED q
        \/ /\ q' \in {t \in (0..1) \X (0..1) \X (0..1) : t[1] + t[2] + t[3] = q[1] + q[2] + q[3] + 1}
           /\ UNCHANGED p

Inv == /\ \A <<x, y, z>> \in {q} : x + y + z <= 3
       /\ \E <<a, b>> \in Pairs : <<a, b>> = p
       /\ Cardinality(Pairs) = 6
       /\ Cardinality((0..1) \X (0..1) \X (0..2)) = 12
       /\ <<0, 1, 2>> \in (0..1) \X (0..1) \X {2}
       /\ <<<<0, 1>>, 2>> \in ((0..1) \X (0..1)) \X {2}
       /\ <<0, 1, 2>> \notin ((0..1) \X (0..1)) \X {2}
       /\ {a + b : <<a, b>> \in Pairs} = 0..3

\* negative control: q's components sum to 2 at depth 3
QSumBelow2 == \A <<x, y, z>> \in {q} : x + y + z < 2
=============================================================================
