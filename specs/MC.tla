---------------------------- MODULE MC ----------------------------
\* Model-checking wrapper for raft.tla (bernborgess/raft-tla,
\* sha256 683a120af29e3e5a805e291f756229d65914f8fb73dddd8c78bafef50a6f6b81).
\*
\* The reference's raft.cfg names INVARIANT NoTwoLeaders (raft.cfg:3) but
\* raft.tla never defines it, and raft.cfg has no CONSTRAINT while Timeout
\* (raft.tla:180) and Send (raft.tla:106-110) are unbounded.  These are the
\* build's own definitions; every state count this repository reports is
\* relative to them.  The MI355X checker (raft-tla_amd/) and both oracles
\* (oracle/raft_values.py, oracle/raft_cpu.c) implement exactly these.
EXTENDS raft, TLC

CONSTANTS MaxTerm,      \* currentTerm bound
          MaxLogLen,    \* Len(log) bound
          MaxCopies,    \* copies of one message in the bag
          MaxInFlight   \* 0 = unbounded; else total messages in the bag

BagCardinality(b) == LET S[D \in SUBSET DOMAIN b] ==
                           IF D = {} THEN 0
                           ELSE LET x == CHOOSE y \in D : TRUE IN b[x] + S[D \ {x}]
                     IN S[DOMAIN b]

StateConstraint ==
    /\ \A i \in Server : currentTerm[i] <= MaxTerm
    /\ \A i \in Server : Len(log[i]) <= MaxLogLen
    /\ \A m \in DOMAIN messages : messages[m] <= MaxCopies
    /\ MaxInFlight = 0 \/ BagCardinality(messages) <= MaxInFlight

\* Strict form: at most one server in state Leader at any time.
NoTwoLeaders == \A i, j \in Server :
                    (state[i] = Leader /\ state[j] = Leader) => i = j

\* History-variable form of Election Safety (raft.tla:34-39 `elections`).
ElectionSafety == \A e, f \in elections : e.eterm = f.eterm => e.eleader = f.eleader

\* Server symmetry (cfg: SYMMETRY Perms).  Every action of raft.tla treats
\* servers alike, so TLC may identify states that differ by a renaming of
\* Server: distinct-state counts become orbit counts.
Perms == Permutations(Server)

LogMatching == \A i, j \in Server :
                 \A n \in 1..(IF Len(log[i]) < Len(log[j]) THEN Len(log[i]) ELSE Len(log[j])) :
                    log[i][n].term = log[j][n].term =>
                        SubSeq(log[i], 1, n) = SubSeq(log[j], 1, n)
=====================================================================
