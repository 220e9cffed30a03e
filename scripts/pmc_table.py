"""Per-kernel counter table from rocprofv3 PMC databases (sum over the dispatches of one run).

    python scripts/pmc_table.py DB [DB ...]      -> one row per kernel, one column per counter
"""
import sqlite3
import sys
from collections import defaultdict

vals = defaultdict(dict)
calls = {}
for db in sys.argv[1:]:
    c = sqlite3.connect(db).cursor()
    for k, cn, n, s in c.execute("select kernel_name, counter_name, count(*), sum(value) from counters_collection "
                                 "group by kernel_name, counter_name").fetchall():
        vals[k][cn] = s
        calls[k] = n
cols = sorted({cn for v in vals.values() for cn in v})
for k, v in sorted(vals.items(), key=lambda kv: -max(kv[1].values())):
    short = k.split("(")[0].replace("void ", "")[-40:]
    print("%-40s %5d " % (short, calls[k]) + " ".join("%s=%.4g" % (cn, v.get(cn, 0)) for cn in cols))
