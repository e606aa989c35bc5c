"""Summarise rocprofv3 SQLite outputs (run_results.db): per-kernel stats and PMC counters.

    python tools/rocpd_summary.py <db> [<db> ...] [--csv out.csv]

Prints, per kernel name: launches, total / average / min / max duration (ns), and for
every PMC counter collected its per-dispatch average.  Used to produce the summaries under
profiles/ (the raw .db files stay in gpurun_out/).
"""
import csv
import sqlite3
import sys
from collections import defaultdict


def kernel_stats(db):
    con = sqlite3.connect(db)
    rows = con.execute("select name, duration from kernels").fetchall()
    agg = defaultdict(list)
    for name, dur in rows:
        agg[name].append(dur)
    return {k: dict(calls=len(v), total_ns=sum(v), avg_ns=sum(v) / len(v), min_ns=min(v),
                    max_ns=max(v)) for k, v in agg.items()}


def pmc_stats(db):
    con = sqlite3.connect(db)
    try:
        rows = con.execute("select kernel_name, dispatch_id, counter_name, value, duration "
                           "from counters_collection").fetchall()
    except sqlite3.OperationalError:
        return {}
    per = defaultdict(lambda: defaultdict(float))
    disp = defaultdict(set)
    for name, did, cname, val, dur in rows:
        per[name][cname] += val
        disp[name].add(did)
    return {k: {c: v / len(disp[k]) for c, v in d.items()} for k, d in per.items()}


def short(name):
    return name.split("(")[0][:60]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    out_csv = sys.argv[sys.argv.index("--csv") + 1] if "--csv" in sys.argv else None
    if out_csv in args:
        args.remove(out_csv)
    lines = []
    for db in args:
        ks = kernel_stats(db)
        pm = pmc_stats(db)
        print(f"== {db}")
        for k, s in sorted(ks.items(), key=lambda kv: -kv[1]["total_ns"]):
            print(f"  {short(k):60s} calls={s['calls']:4d} avg={s['avg_ns'] / 1e6:10.3f} ms "
                  f"total={s['total_ns'] / 1e6:10.3f} ms")
            row = dict(db=db, kernel=short(k), **s)
            for c, v in sorted(pm.get(k, {}).items()):
                print(f"      {c:36s} {v:.6g}")
                row[c] = v
            lines.append(row)
    if out_csv:
        keys = sorted({k for r in lines for k in r}, key=lambda k: (k not in ("db", "kernel"), k))
        with open(out_csv, "w", newline="") as f:
            w = csv.DictWriter(f, fieldnames=keys)
            w.writeheader()
            w.writerows(lines)


if __name__ == "__main__":
    main()
