"""Generate golden fixtures from the reference's own TLC output.

The reference (dranov/raft-tla) has no tests; the only machine-generated
results it holds are two TLC-produced ``history`` values pasted into
constraints of tlc_membership/raft.tla:

* raft.tla:1201 — the ConcurrentLeaders witness (20 history entries) used by
  ``CommitWhenConcurrentLeaders_unique``;
* raft.tla:1231 — the CommitWhenConcurrentLeaders witness (28 entries) used
  by ``MajorityOfClusterRestarts_constraint``.

This script (run here, where /root/reference exists) parses those TLA+ values
and writes them as JSON data under tests/golden/.  Nothing at test time reads
/root/reference.  Encoding of TLA+ values in JSON:
  int / bool -> JSON int / bool;  "str" -> {"str": s};  model value -> {"mv": n}
  <<..>> -> {"seq": [...]};  {..} -> {"set": [...]};  [f |-> v] -> {"rec": {f: v}}
  (k :> v @@ ...) -> {"fcn": [[k, v], ...]}
"""
import json
import os
import re
import sys

REF = "/root/reference/tlc_membership/raft.tla"
HERE = os.path.dirname(os.path.abspath(__file__))


class P:
    def __init__(self, s):
        self.s, self.p = s, 0

    def ws(self):
        while self.p < len(self.s) and self.s[self.p].isspace():
            self.p += 1

    def lit(self, t):
        self.ws()
        if self.s.startswith(t, self.p):
            self.p += len(t)
            return True
        return False

    def expect(self, t):
        if not self.lit(t):
            raise ValueError("expected %r at %d: %r" % (t, self.p, self.s[self.p:self.p + 40]))

    def ident(self):
        self.ws()
        m = re.compile(r"[A-Za-z0-9_]+").match(self.s, self.p)
        if not m:
            raise ValueError("identifier expected at %d" % self.p)
        self.p = m.end()
        return m.group(0)

    def primary(self):
        if self.lit("<<"):
            xs = []
            if self.lit(">>"):
                return {"seq": xs}
            while True:
                xs.append(self.value())
                if not self.lit(","):
                    break
            self.expect(">>")
            return {"seq": xs}
        if self.lit("["):
            r = {}
            while True:
                f = self.ident()
                self.expect("|->")
                r[f] = self.value()
                if not self.lit(","):
                    break
            self.expect("]")
            return {"rec": r}
        if self.lit("{"):
            xs = []
            if self.lit("}"):
                return {"set": xs}
            while True:
                xs.append(self.value())
                if not self.lit(","):
                    break
            self.expect("}")
            return {"set": xs}
        if self.lit("("):
            v = self.value()
            self.expect(")")
            return v
        self.ws()
        if self.s[self.p] == '"':
            q = self.s.index('"', self.p + 1)
            t = self.s[self.p + 1:q]
            self.p = q + 1
            return {"str": t}
        m = re.compile(r"-?[0-9]+").match(self.s, self.p)
        if m:
            self.p = m.end()
            return int(m.group(0))
        i = self.ident()
        if i == "TRUE":
            return True
        if i == "FALSE":
            return False
        return {"mv": i}

    def fn_term(self):
        a = self.primary()
        if self.lit(":>"):
            b = self.primary()
            return {"fcn": [[a, b]]}
        return a

    def value(self):
        v = self.fn_term()
        while self.lit("@@"):
            w = self.fn_term()
            v = {"fcn": v["fcn"] + w["fcn"]}
        return v


def extract(lines, lineno, name):
    text = lines[lineno - 1]
    m = re.search(name + r"\s*==\s*", text)
    if not m:
        raise SystemExit("trace %s not found on raft.tla:%d" % (name, lineno))
    p = P(text[m.end():])
    return p.value()


def main():
    if not os.path.exists(REF):
        sys.exit("reference not present; fixtures are already committed")
    lines = open(REF).read().split("\n")
    out = {
        "concurrent_leaders_trace.json": (1201, "ConcurrentLeaders_trace"),
        "commit_when_concurrent_leaders_trace.json": (1231, "CommitWhenConcurrentLeaders_trace"),
    }
    for fn, (ln, name) in out.items():
        v = extract(lines, ln, name)
        doc = {"source": "tlc_membership/raft.tla:%d (%s, TLC output pasted by the spec authors)" % (ln, name),
               "value": v}
        with open(os.path.join(HERE, fn), "w") as f:
            json.dump(doc, f, indent=1, sort_keys=True)
        print(fn, len(v["rec"]["global"]["seq"]), "history entries")


if __name__ == "__main__":
    main()
