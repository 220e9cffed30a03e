---------------------------- MODULE Countdown ----------------------------
\* Generated-path test module (written for this repo): a counter that stops at zero, so the
\* search ends in TLC's deadlock report; with EvalError's cfg, a sequence read past its end is
\* TLC's evaluation error.
EXTENDS Naturals, Sequences

CONSTANT Start

VARIABLES x, seen

Init == /\ x = Start
        /\ seen = <<>>

Next == /\ x > 0
        /\ x' = x - 1
        /\ seen' = Append(seen, x)

\* reads one past the end of `seen` once x reaches 1: an evaluation error, not a violation
NextBad == /\ x > 0
           /\ x' = x - 1
           /\ seen' = Append(seen, IF x = 1 THEN seen[Len(seen) + 1] ELSE x)

Typed == x \in 0..Start
=============================================================================
