"""Print a rocprofv3 kernel_stats.csv as a short table (name, calls, avg us, total %)."""
import csv
import re
import sys

for path in sys.argv[1:]:
    print("==", path)
    for r in list(csv.DictReader(open(path)))[:int(__import__("os").environ.get("TOP", "16"))]:
        n = re.sub(r"\(.*", "", r["Name"]).replace("void ", "").replace("optamd::", "")[:70]
        print(f"{n:70s} {r['Calls']:>5} {float(r['AverageNs']) / 1000:9.1f} us {float(r['Percentage']):6.1f} %")
