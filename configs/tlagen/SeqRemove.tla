---------------------------- MODULE SeqRemove ----------------------------
\* Generated-path test module (written for this repo): the reference's own SequencesExt Remove
\* (apalache_no_membership/SequencesExt.tla:66-68, a SelectSeq over a LAMBDA), found through -I.
EXTENDS Naturals, Sequences, SequencesExt

VARIABLE s

Init == s = <<>>

Next == \/ /\ Len(s) < 3
           /\ \E v \in 0..2 : s' = Append(s, v)
        \/ /\ Len(s) > 0
           /\ s' = Remove(s, Head(s))

TypeOK == /\ \A v \in 0..2 : \A i \in 1..Len(Remove(s, v)) : Remove(s, v)[i] # v
          /\ Len(Remove(s, 3)) = Len(s)

\* negative control: removing the head drops at most one element unless the head repeats
\* (violated at depth 3: <<0, 0>>)
NoRepeat == Len(Remove(s, Head(s \o <<9>>))) >= Len(s) - 1
=============================================================================
