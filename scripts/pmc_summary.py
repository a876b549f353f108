"""Per-kernel PMC summary of rocprofv3 CSV runs (the kernel trace and the counter passes of scripts/gpu_fast_pmc.sh):

    python scripts/pmc_summary.py <trace_dir> <fetch_dir> <write_dir> <sq_dir> [--traffic <profiles/traffic_cN.json>]

For each kernel: mean duration (kernel trace), FETCH_SIZE / WRITE_SIZE per launch (raw KB; `hbm_bytes` applies the
gfx950 x2 FETCH correction of MI355X_MICROARCH.md §HBM for wide coalesced reads — an upper bound for narrower loads,
the raw value the lower; --traffic writes both per bench.py stage for roofline.traffic), and from the SQ pass: VALU busy = SQ_ACTIVE_INST_VALU x 4 / (1024 SIMDs x GRBM_GUI_ACTIVE)
(the gfx94x VALUBusy formula; SQ_* count quad-cycles), the fraction of wave cycles issuing VALU, waiting (s_waitcnt /
barrier) and stalled on issue, and VALU / LDS instructions per wave.
"""
import collections
import csv
import glob
import json
import os
import sys

SIMDS = 1024


def counters(d):
    f = glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True)
    agg = collections.defaultdict(lambda: collections.defaultdict(list))
    for path in f:
        for r in csv.DictReader(open(path)):
            agg[r["Kernel_Name"]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    return {k: {c: sum(v) / len(v) for c, v in cs.items()} for k, cs in agg.items()}


def trace(d):
    f = glob.glob(os.path.join(d, "**", "*kernel_trace.csv"), recursive=True)
    agg = collections.defaultdict(list)
    for path in f:
        for r in csv.DictReader(open(path)):
            agg[r["Kernel_Name"]].append((int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3)
    return {k: (sum(v) / len(v), len(v)) for k, v in agg.items()}


def short(name):
    n = name.removeprefix("void ")
    return n.split("(")[0]


# bench.py stage -> kernel (the stages that are one kernel launch)
STAGES = {"pyramid": "mam::k_pyr_flat", "fast": "mam::k_fast_cells", "blur": "mam::k_blur7",
          "distribute": "mam::k_distribute", "describe": "mam::k_describe", "grid": "mam::k_grid",
          "gather": "mam::k_gather", "resolve": "mam::k_resolve", "frustum": "mam::k_frustum"}


def write_traffic(out, path):
    t = {"_note": "HBM bytes per launch from FETCH_SIZE / WRITE_SIZE (separate rocprofv3 passes, KB): stage values "
                  "apply the gfx950 x2 FETCH_SIZE correction of MI355X_MICROARCH.md (exact for wide coalesced reads, "
                  "an upper bound for narrower loads); 'raw' holds the uncorrected lower bound",
         "frames_per_launch": 64,   # scripts/gpu_fast_pmc.sh: --lanes 1 --batch 64 (bench.py scales to its launches)
         "raw": {}, "valu_busy": {}, "wave_frac_wait": {}, "wave_frac_issue_stall": {}}
    for stage, kern in STAGES.items():
        for name, e in out.items():
            if name.startswith(kern) and "hbm_bytes_x2fetch" in e:
                t[stage] = e["hbm_bytes_x2fetch"]
                t["raw"][stage] = e["hbm_bytes_raw"]
            if name.startswith(kern) and "valu_busy" in e:
                t["valu_busy"][stage] = e["valu_busy"]
                t["wave_frac_wait"][stage] = e["wave_frac_wait"]
                t["wave_frac_issue_stall"][stage] = e["wave_frac_issue_stall"]
    with open(path, "w") as f:
        json.dump(t, f, indent=1)


def main():
    args = sys.argv[1:]
    tpath = None
    if "--traffic" in args:
        i = args.index("--traffic")
        tpath = args[i + 1]
        args = args[:i] + args[i + 2:]
    tr, fe, wr, sq = trace(args[0]), counters(args[1]), counters(args[2]), counters(args[3])
    out = {}
    for k in sorted(set(fe) | set(wr) | set(sq)):
        name = short(k)
        if not name.startswith("mam::"):
            continue
        e = out.setdefault(name, {})
        t = [v for kk, v in tr.items() if short(kk) == name]
        if t:
            e["avg_us"] = sum(x[0] * x[1] for x in t) / sum(x[1] for x in t)
        if k in fe:
            e["fetch_kb_raw"] = fe[k]["FETCH_SIZE"]
        if k in wr:
            e["write_kb"] = wr[k]["WRITE_SIZE"]
        if "fetch_kb_raw" in e and "write_kb" in e:
            e["hbm_bytes_x2fetch"] = (2 * e["fetch_kb_raw"] + e["write_kb"]) * 1024
            e["hbm_bytes_raw"] = (e["fetch_kb_raw"] + e["write_kb"]) * 1024
        if k in sq:
            s = sq[k]
            wc = max(s.get("SQ_WAVE_CYCLES", 0.0), 1.0)
            e["valu_busy"] = s.get("SQ_ACTIVE_INST_VALU", 0.0) * 4 / SIMDS / max(s.get("GRBM_GUI_ACTIVE", 1.0), 1.0)
            e["wave_frac_valu"] = s.get("SQ_ACTIVE_INST_VALU", 0.0) / wc
            e["wave_frac_active_any"] = s.get("SQ_ACTIVE_INST_ANY", 0.0) / wc
            e["wave_frac_wait"] = s.get("SQ_WAIT_ANY", 0.0) / wc
            e["wave_frac_issue_stall"] = s.get("SQ_WAIT_INST_ANY", 0.0) / wc
            e["sq_busy_cycles"] = s.get("SQ_BUSY_CYCLES")
            e["grbm_gui_active"] = s.get("GRBM_GUI_ACTIVE")
            e["insts_valu"] = s.get("SQ_INSTS_VALU")
            e["insts_lds"] = s.get("SQ_INSTS_LDS")
    print(json.dumps(out, indent=1))
    if tpath:
        write_traffic(out, tpath)


if __name__ == "__main__":
    main()
