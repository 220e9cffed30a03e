"""Idle time between kernels on the device, from a rocprofv3 kernel trace in CSV form
(`rocprofv3 --kernel-trace --output-format csv -d DIR -o run -- python3 bench.py ...`): the union of
the kernels' busy intervals against the span, per run of the model (a run starts at the seen-set
clear, the first `fillBuffer` kernel after a gap), and the gaps between consecutive kernels.  A
development tool (profiles/r06_c2_kernel_gaps.json).

    python scripts/kernel_gaps.py KERNEL_TRACE.csv [OUT.json]
"""
import csv
import json
import sys


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    ks = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]) for r in rows)
    # runs: split at gaps above 2 ms (the host between bench steps)
    runs, cur = [], [ks[0]]
    for k in ks[1:]:
        if k[0] - max(e for _, e, _ in cur) > 2_000_000:
            runs.append(cur)
            cur = []
        cur.append(k)
    runs.append(cur)
    out = []
    for run in runs:
        span = max(e for _, e, _ in run) - run[0][0]
        busy, end = 0, run[0][0]
        gaps = []
        for s, e, n in run:
            if s > end:
                gaps.append(s - end)
            busy += max(0, e - max(s, end))
            end = max(end, e)
        gaps.sort(reverse=True)
        out.append({"kernels": len(run), "span_ms": span / 1e6, "busy_ms": busy / 1e6, "idle_ms": (span - busy) / 1e6,
                    "gaps": len(gaps), "gap_us_p50": gaps[len(gaps) // 2] / 1e3 if gaps else 0,
                    "gap_us_top5": [g / 1e3 for g in gaps[:5]],
                    "by_kernel_ms": {}})
        for s, e, n in run:
            key = n.split("(")[0].split("<")[0].replace("void ", "").strip()
            out[-1]["by_kernel_ms"][key] = round(out[-1]["by_kernel_ms"].get(key, 0) + (e - s) / 1e6, 3)
    doc = {"source": sys.argv[1], "runs": out}
    if len(sys.argv) > 2:
        json.dump(doc, open(sys.argv[2], "w"), indent=1)
    for r in out:
        print(json.dumps({k: r[k] for k in ("kernels", "span_ms", "busy_ms", "idle_ms", "gaps", "gap_us_p50")}))


if __name__ == "__main__":
    main()
