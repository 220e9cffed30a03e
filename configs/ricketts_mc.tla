---------------------------- MODULE ricketts_mc ----------------------------
\* raftmc-base: thirdparty/raft_dricketts.tla
\*
\* Model-checking wrapper for Daniel Ricketts' raft_dricketts.tla (module `raft` in the
\* reference), which the reference proves with TLAPS and ships without a TLC cfg.  It runs on the
\* generated path (the SANY-subset front end): the constraints bound terms, logs and the message
\* bag, as configs/raft_original_mc.tla does for Ongaro's spec.  To run this under TLC, place a
\* copy of thirdparty/raft_dricketts.tla named raft.tla next to this file.
EXTENDS raft

CONSTANTS MaxTerm, MaxLogLen, MaxMsgs

BoundedTerms == \A i \in Server : currentTerm[i] <= MaxTerm
BoundedLogs == \A i \in Server : Len(log[i]) <= MaxLogLen
BoundedMessages == BagCardinality(messages) <= MaxMsgs

\* Test-only scenario invariant (reachable): no leader ever.
NoLeader == ~ \E i \in Server : state[i] = Leader

\* Test-only negative control of TypeOK's function-set form: terms stay in 0..1 (false after the first Timeout).
BadTerm == currentTerm \in [Server -> 0..1]
=============================================================================
