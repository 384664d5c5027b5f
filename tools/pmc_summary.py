"""Average rocprofv3 --pmc counters per kernel over the dispatches of one or more runs.

  python tools/pmc_summary.py OUT.json DIR [DIR ...]
Each DIR holds a run_counter_collection.csv (rocprofv3 -d DIR --output-format csv
--pmc COUNTER -- ...). FETCH_SIZE / WRITE_SIZE are in KiB per dispatch as rocprofv3
reports them; see MI355X_MICROARCH.md for the gfx950 FETCH_SIZE width caveat.
"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict


def collect(dirs):
    acc = defaultdict(lambda: defaultdict(list))
    for d in dirs:
        for path in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
            with open(path) as f:
                for row in csv.DictReader(f):
                    acc[row["Kernel_Name"]][row["Counter_Name"]].append(float(row["Counter_Value"]))
    out = {}
    for k, cs in acc.items():
        out[k] = {c: sum(v) / len(v) for c, v in cs.items()}
        out[k]["dispatches"] = max(len(v) for v in cs.values())
    return out


if __name__ == "__main__":
    res = collect(sys.argv[2:])
    with open(sys.argv[1], "w") as f:
        json.dump({"unit": "KiB per dispatch (rocprofv3 FETCH_SIZE / WRITE_SIZE)", "kernels": res}, f, indent=1)
    for k, v in sorted(res.items()):
        print(f"{k[:100]:100s} " + " ".join(f"{c}={x:.1f}" for c, x in v.items()))
