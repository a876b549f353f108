"""Cross-check of bench.py's roofline line against a rocprofv3 kernel trace of the same bench command:

    python scripts/roofline_check.py <run_kernel_trace.csv> <bench.json> > roofline_check.json

bench.py times the dominant stage in its stage pass (after the timed region: the lanes one after another, each launch
standalone, HIP events on the launch stream). In the trace those are the last steps x lanes launches of the stage's
kernel with the batch-sized grid (the single-frame latency section launches smaller grids). Reports their mean
duration next to bench.py's avg_launch_ms, and the mean over the earlier (timed-region) launches, which overlap the
other lanes and the LocalMapping stream."""
import csv
import json
import sys

KERNELS = {"fast": "mam::k_fast_cells", "blur": "mam::k_blur7", "describe": "mam::k_describe",
           "distribute": "mam::k_distribute", "resolve": "mam::k_resolve", "pyramid": "mam::k_pyr_flat"}


def main():
    rows = list(csv.DictReader(open(sys.argv[1])))
    b = json.load(open(sys.argv[2]))
    rf = b["roofline"]
    kern = KERNELS[rf["kernel"]]
    ks = [r for r in rows if r["Kernel_Name"].removeprefix("void ").startswith(kern)]
    ks.sort(key=lambda r: int(r["Start_Timestamp"]))
    grid = max(int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) for r in ks)
    big = [r for r in ks if int(r["Grid_Size_X"]) * int(r["Grid_Size_Y"]) == grid]
    n_pass = b["steps"] * b["config"]["lanes"]
    if rf["kernel"] == "pyramid":
        n_pass *= 7
    dur = [(int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e6 for r in big]
    stage, timed = dur[-n_pass:], dur[:-n_pass]
    out = {"kernel": kern, "grid": grid, "bench_avg_launch_ms": rf["avg_launch_ms"],
           "trace_stage_pass_launches": len(stage), "trace_stage_pass_avg_ms": sum(stage) / len(stage),
           "agreement": (sum(stage) / len(stage)) / rf["avg_launch_ms"],
           "trace_timed_region_launches": len(timed),
           "trace_timed_region_avg_ms": sum(timed) / len(timed) if timed else None,
           "bytes_per_launch": rf["bytes_per_launch"]}
    if timed:
        out["timed_region_achieved_GBs"] = rf["bytes_per_launch"] / (out["trace_timed_region_avg_ms"] * 1e-3) / 1e9
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
