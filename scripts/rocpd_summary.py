"""Summarise rocprofv3 SQLite output (rocpd) into the files kept under profiles/.

    python scripts/rocpd_summary.py stats  RUN_DB OUT.csv          # per-kernel calls / total / avg (us)
    python scripts/rocpd_summary.py pmc    RUN_DB COUNTER OUT.csv  # per-kernel mean counter value per dispatch
    python scripts/rocpd_summary.py traffic FETCH_DB WRITE_DB KERNEL_SUBSTR OUT.json [WORKLOAD] [--random]
    python scripts/rocpd_summary.py valu   PMC_DB KERNEL_SUBSTR OUT.json [WORKLOAD]   # VALU/SALU wave-instructions per dispatch

WORKLOAD (default "c2.cfg") names the model the profiled command checked, as bench.py's workload key
(cfg basename, "@depth" when depth-bounded): bench.py only attaches a summary to its line when both the
kernel and the workload match.

`traffic` follows /opt/skills/guides/MI355X_MICROARCH.md (HBM/rocprofv3 section):
FETCH_SIZE and WRITE_SIZE come from separate --pmc passes, both in KiB per
dispatch; on gfx950 FETCH_SIZE reports half the bytes of wide coalesced reads,
so it is doubled; WRITE_SIZE is taken as is.
"""
import csv
import json
import sqlite3
import sys


def q(db, sql):
    return sqlite3.connect(db).cursor().execute(sql).fetchall()


def stats(db, out):
    rows = q(db, "select name, total_calls, total_duration, average, percentage from top_kernels order by total_duration desc")
    with open(out, "w", newline="") as f:
        w = csv.writer(f)
        w.writerow(["kernel", "calls", "total_us", "avg_us", "percent"])
        for r in rows:
            w.writerow([r[0], r[1], round(r[2], 3), round(r[3], 3), round(r[4], 3)])
    return rows


def pmc(db, counter):
    rows = q(db, "select kernel_name, count(*), avg(value), sum(value) from counters_collection where counter_name = '%s' "
                 "group by kernel_name order by sum(value) desc" % counter)
    return [(r[0], r[1], r[2], r[3]) for r in rows]


def main():
    mode = sys.argv[1]
    if mode == "stats":
        for r in stats(sys.argv[2], sys.argv[3]):
            print("%-70s %6d %12.1f us %10.1f us %6.2f%%" % (r[0][:70], r[1], r[2], r[3], r[4]))
    elif mode == "pmc":
        rows = pmc(sys.argv[2], sys.argv[3])
        with open(sys.argv[4], "w", newline="") as f:
            w = csv.writer(f)
            w.writerow(["kernel", "dispatches", "mean_value_per_dispatch", "sum"])
            for r in rows:
                w.writerow(r)
        for r in rows:
            print(r)
    elif mode == "traffic":
        args = [a for a in sys.argv if a != "--random"]
        random_probes = "--random" in sys.argv
        fetch = {r[0]: r for r in pmc(args[2], "FETCH_SIZE")}
        write = {r[0]: r for r in pmc(args[3], "WRITE_SIZE")}
        name = next(k for k in fetch if args[4] in k)
        f_kib, w_kib = fetch[name][2], write[name][2]
        # streaming reads: FETCH_SIZE is half the bytes (MI355X_MICROARCH.md); random 8-B probes: one
        # 64-B request per probe is charged 64 B (profiles/r04_fetch_size_calibration.json), so the
        # counter is taken as is (--random: the seen-set kernels)
        factor = 1 if random_probes else 2
        doc = {"kernel_name": args[4], "kernel_symbol": name, "dispatches": fetch[name][1],
               "workload": args[6] if len(args) > 6 else "c2.cfg",
               "fetch_bytes_per_launch_raw": f_kib * 1024, "write_bytes_per_launch": w_kib * 1024,
               "hbm_bytes_per_launch": factor * f_kib * 1024 + w_kib * 1024,
               "method": "rocprofv3 --pmc FETCH_SIZE and --pmc WRITE_SIZE in separate passes over `bench.py --steps 1 "
                         "--warmup 0 --no-extra`; KiB*1024 averaged over the kernel's dispatches; " +
                         ("FETCH_SIZE as is: random 8-B probes are charged 64 B per request, calibrated on "
                          "scripts/seen_set_bench.hip (profiles/r04_fetch_size_calibration.json)" if random_probes else
                          "FETCH_SIZE doubled per MI355X_MICROARCH.md (gfx950 tallies 128-B requests at 64 B)") +
                         ", WRITE_SIZE as is"}
        json.dump(doc, open(sys.argv[5], "w"), indent=1)
        print(json.dumps(doc, indent=1))
    elif mode == "valu":
        valu = {r[0]: r for r in pmc(sys.argv[2], "SQ_INSTS_VALU")}
        salu = {r[0]: r for r in pmc(sys.argv[2], "SQ_INSTS_SALU")}
        name = next(k for k in valu if sys.argv[3] in k)
        extra = {}
        for cn in ("SQ_ACTIVE_INST_VALU", "SQ_ACTIVE_INST_ANY", "SQ_WAVE_CYCLES", "SQ_BUSY_CYCLES", "SQ_WAIT_INST_ANY", "SQ_WAVES"):
            rows = {r[0]: r for r in pmc(sys.argv[2], cn)}
            if name in rows:
                extra[cn + "_per_launch"] = rows[name][2]
        doc = {"kernel_name": sys.argv[3], "kernel_symbol": name, "dispatches": valu[name][1],
               "workload": sys.argv[5] if len(sys.argv) > 5 else "c2.cfg",
               "valu_insts_per_launch": valu[name][2], "salu_insts_per_launch": salu[name][2] if name in salu else None,
               "sq_counters": extra,
               "peak_valu_insts_per_s": 256 * 2 * 2.4e9,
               "method": "rocprofv3 --pmc SQ_INSTS_VALU SQ_INSTS_SALU over `bench.py --steps 1 --warmup 0`; wave-instructions "
                         "per dispatch; peak per MI355X_MICROARCH.md: 4 SIMD-32 per CU, a wave64 VALU instruction "
                         "issues in 2 cycles, i.e. 2 wave-instructions per CU per cycle, 256 CUs at 2.4 GHz"}
        json.dump(doc, open(sys.argv[4], "w"), indent=1)
        print(json.dumps(doc, indent=1))


if __name__ == "__main__":
    main()
