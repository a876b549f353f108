"""Summarise rocprofv3 rocpd databases into the files committed under profiles/.

    python scripts/profile_summary.py stats  <run_results.db> <out.csv>
        per-kernel Calls / TotalDurationNs / AverageNs / Percentage / Min / Max (the --stats summary)
    python scripts/profile_summary.py traffic <fetch.db> <write.db> <out.json>
        per-kernel HBM bytes per launch from the FETCH_SIZE and WRITE_SIZE passes (kilobytes in rocprofv3), with the
        gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of wide
        coalesced reads: x2), keyed by bench.py stage name for the single-kernel stages.
"""
from __future__ import annotations

import csv
import json
import sqlite3
import sys
from collections import defaultdict

# bench.py stage -> kernel symbol prefix (stages that are exactly one kernel launch)
STAGE_KERNELS = {
    "fast": "mam::k_fast_cells",
    "blur": "mam::k_blur7",
    "distribute": "mam::k_distribute",
    "describe": "mam::k_describe",
    "resolve": "mam::k_resolve",
    "grid": "mam::k_grid",
}


def stats(db: str, out: str) -> None:
    c = sqlite3.connect(db)
    rows = c.execute("select name, duration from kernels").fetchall()
    agg = defaultdict(list)
    for name, d in rows:
        agg[name].append(int(d))
    total = sum(sum(v) for v in agg.values())
    recs = []
    for name, v in agg.items():
        n = len(v)
        mean = sum(v) / n
        sd = (sum((x - mean) ** 2 for x in v) / n) ** 0.5
        recs.append((name, n, sum(v), mean, 100.0 * sum(v) / total, min(v), max(v), sd))
    recs.sort(key=lambda r: -r[2])
    with open(out, "w", newline="") as f:
        w = csv.writer(f, quoting=csv.QUOTE_NONNUMERIC)
        w.writerow(["Name", "Calls", "TotalDurationNs", "AverageNs", "Percentage", "MinNs", "MaxNs", "StdDev"])
        for r in recs:
            w.writerow(r)
    for r in recs[:12]:
        print(f"{r[3] / 1e3:10.1f} us x {r[1]:5d}  {r[4]:5.1f}%  {r[0][:90]}")


def _per_kernel(db: str, counter: str):
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, value from counters_collection where counter_name = ?", (counter,)).fetchall()
    agg = defaultdict(list)
    for name, v in rows:
        agg[name].append(float(v))
    return {k: sum(v) / len(v) for k, v in agg.items()}


def traffic(fetch_db: str, write_db: str, out: str) -> None:
    fe = _per_kernel(fetch_db, "FETCH_SIZE")
    wr = _per_kernel(write_db, "WRITE_SIZE")
    kernels = {}
    for name in sorted(set(fe) | set(wr)):
        f_kb, w_kb = fe.get(name, 0.0), wr.get(name, 0.0)
        kernels[name] = {"fetch_kb_raw": f_kb, "write_kb": w_kb,
                         "bytes_per_launch": 2.0 * f_kb * 1024.0 + w_kb * 1024.0}
    res = {"_note": "HBM bytes per launch = 2*FETCH_SIZE + WRITE_SIZE (KB->B); FETCH x2 per the gfx950 correction "
                    "for wide coalesced reads; Infinity-Cache hits are counted (MI355X_MICROARCH.md HBM section)",
           "kernels": kernels}
    for stage, prefix in STAGE_KERNELS.items():
        hits = [v["bytes_per_launch"] for k, v in kernels.items()
                if k.removeprefix("void ").startswith(prefix + "(") or k.removeprefix("void ").startswith(prefix + "<")]
        if hits:
            res[stage] = sum(hits) / len(hits)
    json.dump(res, open(out, "w"), indent=1)
    for k, v in sorted(kernels.items(), key=lambda kv: -kv[1]["bytes_per_launch"])[:10]:
        print(f"{v['bytes_per_launch'] / 1e6:10.2f} MB/launch  fetch {v['fetch_kb_raw']:10.0f} KB  write {v['write_kb']:10.0f} KB  {k[:70]}")


if __name__ == "__main__":
    if sys.argv[1] == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif sys.argv[1] == "traffic":
        traffic(sys.argv[2], sys.argv[3], sys.argv[4])
    else:
        raise SystemExit(__doc__)
