"""Per-solve timeline of lone LocalBundleAdjustment solves from a rocprofv3 kernel trace (CSV).

    python scripts/lone_trace.py <run_kernel_trace.csv> [--skip N]

A solve starts at k_struct_init and ends at k_finish; prints, per solve, the wall span on the GPU, the sum of kernel
durations, the gap share, and the mean duration of each kernel over the solves (after skipping N warm-up solves).
"""
import csv
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    skip = int(sys.argv[sys.argv.index("--skip") + 1]) if "--skip" in sys.argv else 1
    rows = list(csv.DictReader(open(path)))
    rows = [r for r in rows if "mam::lba" in r["Kernel_Name"]]
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    solves, cur = [], None
    for r in rows:
        n = r["Kernel_Name"]
        if "k_struct_init" in n:
            cur = []
            solves.append(cur)
        if cur is not None:
            cur.append(r)
    solves = [s for s in solves if any("k_finish" in r["Kernel_Name"] for r in s)][skip:]
    per = defaultdict(list)
    for i, s in enumerate(solves):
        t0, t1 = int(s[0]["Start_Timestamp"]), int(s[-1]["End_Timestamp"])
        ksum = sum(int(r["End_Timestamp"]) - int(r["Start_Timestamp"]) for r in s)
        print(f"solve {i}: span {(t1 - t0) / 1e3:8.1f} us, kernels {ksum / 1e3:8.1f} us, {len(s)} dispatches, "
              f"gaps {(t1 - t0 - ksum) / 1e3:7.1f} us")
        agg = defaultdict(float)
        cnt = defaultdict(int)
        for r in s:
            k = r["Kernel_Name"].split("(")[0].replace("void ", "")
            agg[k] += (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
            cnt[k] += 1
        for k in agg:
            per[k].append((agg[k], cnt[k]))
    print("per solve (mean over solves): total us, dispatches, us per dispatch")
    for k, v in sorted(per.items(), key=lambda kv: -sum(x[0] for x in kv[1])):
        tot = sum(x[0] for x in v) / len(v)
        n = sum(x[1] for x in v) / len(v)
        print(f"  {k[:50]:50s} {tot:9.1f} {n:6.1f} {tot / max(n, 1):8.1f}")


if __name__ == "__main__":
    main()
