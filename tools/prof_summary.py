"""Summarise a rocprofv3 --kernel-trace database (results.db) into a per-kernel table."""
import glob
import json
import sqlite3
import sys


def summarize(db):
    c = sqlite3.connect(db)
    rows = c.execute(
        "select name, count(*), avg(end-start), sum(end-start), min(end-start), max(end-start), "
        "max(vgpr_count), max(sgpr_count), max(grid_x), max(workgroup_x) from kernels "
        "group by name order by sum(end-start) desc").fetchall()
    total = sum(r[3] for r in rows) or 1
    out = []
    for name, n, avg, tot, mn, mx, vg, sg, gx, wx in rows:
        out.append({"kernel": name, "calls": n, "avg_us": avg / 1e3, "total_ms": tot / 1e6,
                    "pct": 100.0 * tot / total, "min_us": mn / 1e3, "max_us": mx / 1e3,
                    "vgpr": vg, "sgpr": sg, "grid": gx, "block": wx})
    return out


if __name__ == "__main__":
    dbs = sorted(glob.glob(sys.argv[1] + "/**/*.db", recursive=True)) if not sys.argv[1].endswith(".db") else [sys.argv[1]]
    for db in dbs:
        res = summarize(db)
        if len(sys.argv) > 2 and sys.argv[2] == "--json":
            print(json.dumps(res, indent=1))
        else:
            print(f"# {db}")
            print(f"{'calls':>6} {'avg_us':>10} {'total_ms':>10} {'pct':>6} {'vgpr':>5}  kernel")
            for r in res:
                print(f"{r['calls']:6d} {r['avg_us']:10.2f} {r['total_ms']:10.3f} {r['pct']:6.1f} {r['vgpr']:5d}  {r['kernel'][:120]}")
