--------------------------- MODULE raft_original_mc ---------------------------
\* raftmc-base: thirdparty/raft_original.tla
\*
\* Model-checking wrapper for Ongaro's raft_original.tla (module `raft` in the
\* reference, thirdparty/raft_original.tla).  The reference ships no cfg,
\* no constraints and no invariant for this spec (SURVEY.md §8 A21/A22), so
\* they are authored here and frozen.  To run this under TLC, place a copy of
\* thirdparty/raft_original.tla named raft.tla next to this file.
\*
\* G1: raft_original's message bag is a plain function; counts go negative
\* and DOMAIN messages never shrinks, so the message constraint bounds BOTH
\* the domain size and the per-message count range.
EXTENDS raft, Integers

CONSTANTS MaxTerm, MaxLogLen, MaxMsgDomain, MinMsgCount, MaxMsgCount

BoundedTerms == \A i \in Server : currentTerm[i] <= MaxTerm

BoundedLogs == \A i \in Server : Len(log[i]) <= MaxLogLen

BoundedMessages ==
    /\ Cardinality(DOMAIN messages) <= MaxMsgDomain
    /\ \A m \in DOMAIN messages : messages[m] \in MinMsgCount..MaxMsgCount

\* At most one leader per term, stated over the spec's own `elections`
\* history variable (raft_original.tla:39, :236-241).
ElectionSafety ==
    \A e, f \in elections : e.eterm = f.eterm => e.eleader = f.eleader

\* tlc_membership/raft.tla:1017-1021 restated over raft_original's logs.
LogMatching ==
    \A i, j \in Server :
        \A n \in (1..Len(log[i])) \cap (1..Len(log[j])) :
            log[i][n].term = log[j][n].term =>
            SubSeq(log[i],1,n) = SubSeq(log[j],1,n)

\* Test-only scenario invariant (a reachable "violation"): no leader ever.
NoLeader == ~ \E i \in Server : state[i] = Leader

\* Test-only scenario invariant reached only after a full replication round trip
\* (AppendEntries, HandleAppendEntriesRequest, HandleAppendEntriesResponse,
\* AdvanceCommitIndex): no server ever commits.  Its counterexamples exercise the
\* TLC order of every message type.
NoCommit == \A i \in Server : commitIndex[i] = 0
===============================================================================
