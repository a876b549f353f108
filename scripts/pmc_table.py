"""Per-kernel mean of every counter in a rocprofv3 counter_collection.csv."""
import csv
import sys
from collections import defaultdict

agg = defaultdict(lambda: defaultdict(list))
for r in csv.DictReader(open(sys.argv[1])):
    agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
for k, v in sorted(agg.items()):
    print(k[:40].ljust(40), " ".join(f"{c}={sum(x) / len(x):.4g}" for c, x in sorted(v.items())))
