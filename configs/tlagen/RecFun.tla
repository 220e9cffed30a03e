---- MODULE RecFun ----
\* Recursive function definitions on the generated path (the form of TypedBags' Sum,
\* tlc_membership/TypedBags.tla:73-83): a global one (Fact) and one local to a LET (DSum).
EXTENDS Naturals, FiniteSets
VARIABLE x, bag
Fact[n \in 0..6] == IF n = 0 THEN 1 ELSE n * Fact[n - 1]
Sum(f) == LET DSum[S \in SUBSET DOMAIN f] ==
                LET elt == CHOOSE e \in S : TRUE
                IN  IF S = {} THEN 0 ELSE f[elt] + DSum[S \ {elt}]
          IN  DSum[DOMAIN f]
Init == x = 0 /\ bag = [k \in {1, 2, 3} |-> 0]
Next == \/ /\ x' = (x + 1) % 7
           /\ bag' = IF Sum(bag) < 9 THEN [bag EXCEPT ![1 + (x % 3)] = @ + 1] ELSE bag
        \/ /\ Sum(bag) > 0
           /\ \E k \in DOMAIN bag : bag[k] > 0 /\ bag' = [bag EXCEPT ![k] = @ - 1]
           /\ UNCHANGED x
FactBound == Fact[x] <= 720
SumBound == Sum(bag) <= 9
FactNot24 == Fact[x] /= 24
SumNot7 == Sum(bag) /= 7
OutOfDomain == Fact[x + 1] > 0
====
