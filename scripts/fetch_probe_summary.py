"""FETCH_SIZE (KB) per probe kernel vs the bytes it reads: python scripts/fetch_probe_summary.py <pmc_dir> <probe.json>"""
import csv
import glob
import json
import os
import sys

rows = []
for f in glob.glob(os.path.join(sys.argv[1], "**", "*counter_collection.csv"), recursive=True):
    rows += list(csv.DictReader(open(f)))
probe = {p["shape"]: p["bytes_read"] for p in json.loads(open(sys.argv[2]).read().strip().splitlines()[-1])}
names = {"probe_wide": "wide16", "probe_dword": "dword", "probe_byte": "byte", "probe_roi": "fast_roi"}
out = {}
for r in rows:
    k = r["Kernel_Name"].split("(")[0].replace("void ", "")
    if k in names and r["Counter_Name"] == "FETCH_SIZE":
        b = probe[names[k]]
        out[names[k]] = {"bytes_read": b, "fetch_size_bytes": float(r["Counter_Value"]) * 1024,
                         "fetch_over_bytes": float(r["Counter_Value"]) * 1024 / b}
print(json.dumps(out, indent=1))
