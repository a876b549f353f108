"""Per (kernel, grid-y) average durations from a rocprofv3 kernel trace: python scripts/trace_by_grid.py trace.csv"""
import collections
import csv
import sys

rows = list(csv.DictReader(open(sys.argv[1])))
d = collections.defaultdict(list)
for r in rows:
    d[(r["Kernel_Name"][:44], r["Grid_Size_X"], r["Grid_Size_Y"])].append(
        (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
for k, v in sorted(d.items(), key=lambda kv: -sum(kv[1]))[:int(sys.argv[2]) if len(sys.argv) > 2 else 30]:
    print(k[0].ljust(44), ("grid %sx%s" % (k[1], k[2])).ljust(20), str(len(v)).rjust(5), "%9.1f us" % (sum(v) / len(v)))
