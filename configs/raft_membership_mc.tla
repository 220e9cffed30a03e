-------------------------- MODULE raft_membership_mc --------------------------
\* raftmc-base: tlc_membership/raft.tla
\*
\* Wrapper that selects the reference's tlc_membership/raft.tla (module
\* `raft`) without copying it: every operator named by the membership_*.cfg
\* files (Init, Next*, the Bounded*/CleanStart* constraints, the Raft
\* invariants and the scenario properties, perms, vars) is defined in that
\* module.  To run under TLC, place tlc_membership/raft.tla and its helper
\* modules next to this file.
EXTENDS raft
===============================================================================
