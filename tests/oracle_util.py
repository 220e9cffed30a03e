"""Test helpers that drive the CPU oracle (test infrastructure only)."""
import json
import os
import subprocess
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(ROOT, "oracle")
ORACLE_BIN = os.path.join(ORACLE_DIR, "_build", "raft_oracle")
CONFIGS = os.path.join(ROOT, "configs")
GOLDEN = os.path.join(ROOT, "tests", "golden")
ORIG_MC = os.path.join(CONFIGS, "raft_original_mc.tla")
MEMB_MC = os.path.join(CONFIGS, "raft_membership_mc.tla")


def build_oracle():
    subprocess.run(["make", "-s", "-C", ORACLE_DIR], check=True)
    return ORACLE_BIN


def run_oracle(mode, tla, cfg, *extra, timeout=600):
    build_oracle()
    out = subprocess.run([ORACLE_BIN, mode, "--tla", tla, "--cfg", cfg, *map(str, extra)],
                         capture_output=True, text=True, timeout=timeout)
    line = out.stdout.strip().splitlines()[-1]
    return json.loads(line)


def tla_text(v):
    """JSON-encoded TLA+ value (tests/golden/make_golden.py) -> TLA+ text."""
    if isinstance(v, bool):
        return "TRUE" if v else "FALSE"
    if isinstance(v, int):
        return str(v)
    (k, x), = v.items()
    if k == "str":
        return '"%s"' % x
    if k == "mv":
        return x
    if k == "seq":
        return "<<" + ", ".join(tla_text(e) for e in x) + ">>"
    if k == "set":
        return "{" + ", ".join(tla_text(e) for e in x) + "}"
    if k == "rec":
        return "[" + ", ".join("%s |-> %s" % (f, tla_text(e)) for f, e in x.items()) + "]"
    if k == "fcn":
        return "(" + " @@ ".join("%s :> %s" % (tla_text(a), tla_text(b)) for a, b in x) + ")"
    raise ValueError(k)


def golden_file(name):
    """Write a golden JSON fixture as TLA+ value text into a temp file."""
    doc = json.load(open(os.path.join(GOLDEN, name)))
    fd, path = tempfile.mkstemp(suffix=".tla_value")
    with os.fdopen(fd, "w") as f:
        f.write(tla_text(doc["value"]))
    return path, doc


def cfg_variant(base_path, replace=(), append=""):
    """Copy a cfg with textual replacements; returns a temp path."""
    text = open(base_path).read()
    for a, b in replace:
        assert a in text, a
        text = text.replace(a, b)
    text += "\n" + append
    fd, path = tempfile.mkstemp(suffix=".cfg")
    with os.fdopen(fd, "w") as f:
        f.write(text)
    return path
