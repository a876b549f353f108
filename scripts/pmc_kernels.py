"""Per-kernel table of every counter in a set of rocprofv3 CSV runs (a kernel trace + one directory per --pmc pass):

    python scripts/pmc_kernels.py <trace_dir> <pmc_dir> [<pmc_dir> ...] [--match SUBSTR] [--json OUT]

Per kernel (name containing SUBSTR): launches, mean duration (us), the mean of every counter per launch, and derived
FETCH/WRITE MB per launch (FETCH doubled: the gfx950 correction of MI355X_MICROARCH.md for wide reads — an upper bound
for narrow loads), L2 hit rate = TCC_HIT / (TCC_HIT + TCC_MISS), and VALU busy from the SQ pass when present.
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS = 1024


def rows(d, pattern):
    for path in glob.glob(os.path.join(d, "**", pattern), recursive=True):
        yield from csv.DictReader(open(path))


def main():
    args = sys.argv[1:]
    match = ""
    out_json = None
    if "--match" in args:
        i = args.index("--match"); match = args[i + 1]; del args[i:i + 2]
    if "--json" in args:
        i = args.index("--json"); out_json = args[i + 1]; del args[i:i + 2]
    tdir, pdirs = args[0], args[1:]
    dur = collections.defaultdict(list)
    for r in rows(tdir, "*kernel_trace.csv"):
        dur[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    cnt = collections.defaultdict(lambda: collections.defaultdict(list))
    for d in pdirs:
        for r in rows(d, "*counter_collection.csv"):
            cnt[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    table = {}
    for k, v in sorted(dur.items(), key=lambda kv: -sum(kv[1])):
        if match not in k:
            continue
        e = {"launches": len(v), "us_mean": sum(v) / len(v)}
        for c, vals in cnt.get(k, {}).items():
            e[c] = sum(vals) / len(vals)
        if "FETCH_SIZE" in e:
            e["fetch_MB_x2"] = 2 * e["FETCH_SIZE"] * 1024 / 1e6
        if "WRITE_SIZE" in e:
            e["write_MB"] = e["WRITE_SIZE"] * 1024 / 1e6
        h, m = e.get("TCC_HIT_sum"), e.get("TCC_MISS_sum")
        if h is not None and m is not None and h + m > 0:
            e["l2_hit"] = h / (h + m)
        if "SQ_ACTIVE_INST_VALU" in e and e.get("GRBM_GUI_ACTIVE"):
            e["valu_busy"] = e["SQ_ACTIVE_INST_VALU"] * 4 / (SIMDS * e["GRBM_GUI_ACTIVE"])
        if e.get("SQ_WAVE_CYCLES"):
            for c in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
                if c in e:
                    e[c.lower() + "_frac"] = e[c] / e["SQ_WAVE_CYCLES"]
        table[k.removeprefix("void ").split("(")[0]] = e
    for k, e in table.items():
        keys = ("launches", "us_mean", "fetch_MB_x2", "write_MB", "l2_hit", "valu_busy", "sq_wait_inst_any_frac")
        print(k[:40].ljust(40), " ".join(f"{c}={e[c]:.3g}" for c in keys if c in e))
    if out_json:
        json.dump(table, open(out_json, "w"), indent=1)


if __name__ == "__main__":
    main()
