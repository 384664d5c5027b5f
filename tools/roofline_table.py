"""Kernel-by-kernel roofline table of one profiled configuration: rocprofv3
--kernel-trace --stats (calls, average duration) joined with the FETCH_SIZE /
WRITE_SIZE PMC passes (tools/pmc_summary.py JSON). HBM bytes per call = 2 FETCH_SIZE +
WRITE_SIZE (KiB; the gfx950 FETCH_SIZE width correction, MI355X_MICROARCH.md), GB/s =
bytes / average duration, frac against 8 TB/s.

  python tools/roofline_table.py STATS.csv PMC.json STEPS [--json OUT]
STEPS = solver steps in the profiled run (calls per step = calls / STEPS).
"""
import csv
import json
import sys

PEAK = 8000.0


def short(name):
    n = name.split("(")[0]
    for p in ("void ", "optamd::"):
        n = n.replace(p, "")
    return n[:60]


def main():
    stats, pmc, steps = sys.argv[1], sys.argv[2], float(sys.argv[3])
    out = sys.argv[5] if len(sys.argv) > 5 and sys.argv[4] == "--json" else None
    with open(pmc) as f:
        ks = json.load(f)["kernels"]
    pm = {short(k): v for k, v in ks.items()}
    rows = []
    with open(stats) as f:
        for r in csv.DictReader(f):
            n = short(r["Name"])
            calls = int(r["Calls"])
            avg_us = float(r["AverageNs"]) / 1e3
            c = pm.get(n, {})
            b = 1024 * (2 * c.get("FETCH_SIZE", 0.0) + c.get("WRITE_SIZE", 0.0)) if c else None
            gbs = b / (avg_us * 1e3) if b else None
            rows.append(dict(kernel=n, calls_per_step=calls / steps, avg_us=avg_us,
                             us_per_step=avg_us * calls / steps, hbm_bytes_per_call=b, gbs=gbs,
                             frac=gbs / PEAK if gbs else None))
    rows.sort(key=lambda r: -r["us_per_step"])
    tot = sum(r["us_per_step"] for r in rows)
    print(f"{'kernel':60s} {'calls/st':>8s} {'avg us':>8s} {'us/step':>8s} {'share':>6s} {'MB/call':>8s} {'GB/s':>7s} {'frac':>5s}")
    for r in rows:
        mb = f"{r['hbm_bytes_per_call'] / 1e6:8.1f}" if r["hbm_bytes_per_call"] else " " * 8
        g = f"{r['gbs']:7.0f} {r['frac']:5.2f}" if r["gbs"] else ""
        print(f"{r['kernel']:60s} {r['calls_per_step']:8.1f} {r['avg_us']:8.1f} {r['us_per_step']:8.1f} "
              f"{100 * r['us_per_step'] / tot:5.1f}% {mb} {g}")
    print(f"device time per step: {tot:.1f} us")
    if out:
        with open(out, "w") as f:
            json.dump({"stats": stats, "pmc": pmc, "steps": steps, "device_us_per_step": tot, "kernels": rows}, f,
                      indent=1)


if __name__ == "__main__":
    main()
