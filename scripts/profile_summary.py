"""Summarise rocprofv3 rocpd databases into the files committed under profiles/.

    python scripts/profile_summary.py stats  <run_results.db> <out.csv>
        per-kernel Calls / TotalDurationNs / AverageNs / Percentage / Min / Max (the --stats summary)
    python scripts/profile_summary.py traffic <fetch.db> <write.db> <out.json>
        per-kernel HBM bytes per launch from the FETCH_SIZE and WRITE_SIZE passes (kilobytes in rocprofv3), with the
        gfx950 correction of /opt/skills/guides/MI355X_MICROARCH.md §HBM (FETCH_SIZE counts half the bytes of wide
        coalesced reads: x2), keyed by bench.py stage name for the single-kernel stages.
    python scripts/profile_summary.py gaps <run_results.db> [first_kernel]
        per-frame kernel timeline of a B=1 latency run (durations and inter-kernel gaps)
    python scripts/profile_summary.py mfma <pmc_results.db> <out.json>
        per-kernel FP64 MFMA flops (SQ_INSTS_VALU_MFMA_MOPS_F64 x 512), MFMA-busy fraction of the run
        (SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE x 1024 SIMDs)) and the achieved FP64-MFMA rate over the kernel's
        dispatch duration vs the gfx950 dense FP64 peak
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


def mfma(db: str, out: str, simds: int = 1024, fp64_peak_tflops: float = 78.6) -> None:
    c = sqlite3.connect(db)
    rows = c.execute("select kernel_name, counter_name, value, duration, dispatch_id from counters_collection").fetchall()
    agg = defaultdict(lambda: defaultdict(list))
    dur = defaultdict(dict)
    for name, cn, v, d, did in rows:
        agg[name][cn].append(float(v))
        dur[name][did] = float(d)
    res = {"_note": "FP64 MFMA flops = SQ_INSTS_VALU_MFMA_MOPS_F64 * 512 (rocprofv3 MfmaFlopsF64); busy = "
                    "SQ_VALU_MFMA_BUSY_CYCLES / (GRBM_GUI_ACTIVE * 1024 SIMDs) (rocprofv3 MfmaUtil, gfx94x formula); "
                    "tflops = flops / mean dispatch duration; peak = MI355X dense FP64 (78.6 TF/s)", "kernels": {}}
    for name, cs in agg.items():
        n = max(len(dur[name]), 1)
        flops = sum(cs.get("SQ_INSTS_VALU_MFMA_MOPS_F64", [0.0])) / n * 512.0
        busy = sum(cs.get("SQ_VALU_MFMA_BUSY_CYCLES", [0.0])) / n
        gui = sum(cs.get("GRBM_GUI_ACTIVE", [0.0])) / max(len(cs.get("GRBM_GUI_ACTIVE", [1])), 1)
        d_ns = sum(dur[name].values()) / n
        if flops <= 0 and busy <= 0:
            continue
        tf = flops / (d_ns * 1e-9) / 1e12 if d_ns > 0 else 0.0
        res["kernels"][name] = {"mfma_f64_flops_per_launch": flops, "mean_duration_us": d_ns / 1e3,
                                "mfma_f64_tflops": tf, "frac_of_fp64_peak": tf / fp64_peak_tflops,
                                "mfma_busy_frac": busy / (gui * simds) if gui > 0 else None}
    json.dump(res, open(out, "w"), indent=1)
    for k, v in res["kernels"].items():
        print(f"{k[:60]:60s} {v['mfma_f64_flops_per_launch'] / 1e6:8.2f} MFLOP {v['mean_duration_us']:8.1f} us "
              f"{v['mfma_f64_tflops']:6.3f} TF/s busy {v['mfma_busy_frac']}")


def gaps(db: str, first_kernel: str = "k_pyr_down", frames: int = 40) -> None:
    """Per-frame timeline of a B=1 latency run: the kernels of the last `frames` frames (a frame starts at each
    launch of `first_kernel` that follows a launch of another kernel), their mean durations in launch order, and the
    mean span first start -> last end vs the sum of kernel durations (the rest is inter-kernel gaps)."""
    if db.endswith(".csv"):   # rocprofv3 -f csv kernel trace
        with open(db) as f:
            rows = sorted(((r["Kernel_Name"], int(r["Start_Timestamp"]), int(r["End_Timestamp"]))
                           for r in csv.DictReader(f)), key=lambda r: r[1])
    else:
        c = sqlite3.connect(db)
        cols = [r[1] for r in c.execute("pragma table_info(kernels)").fetchall()]
        st = "start" if "start" in cols else "start_timestamp"
        en = "end" if "end" in cols else "end_timestamp"
        rows = c.execute(f"select name, {st}, {en} from kernels order by {st}").fetchall()
    starts = [i for i, r in enumerate(rows) if first_kernel in r[0] and (i == 0 or first_kernel not in rows[i - 1][0])]
    groups = [rows[a:b] for a, b in zip(starts, starts[1:] + [len(rows)])][-frames - 1:-1]
    sig = defaultdict(int)
    for g in groups:
        sig[tuple(r[0] for r in g)] += 1
    key = max(sig, key=sig.get)
    groups = [g for g in groups if tuple(r[0] for r in g) == key]
    n = len(groups)
    print(f"{n} frames with the modal launch sequence ({len(key)} kernels)")
    tot_k = 0.0
    for j, name in enumerate(key):
        d = sum(g[j][2] - g[j][1] for g in groups) / n / 1e3
        gap = sum(g[j][1] - g[j - 1][2] for g in groups) / n / 1e3 if j else 0.0
        tot_k += d
        print(f"  {j:2d} gap {gap:6.2f} us  dur {d:7.2f} us  {name[:80]}")
    span = sum(g[-1][2] - g[0][1] for g in groups) / n / 1e3
    print(f"span {span:.1f} us, kernels {tot_k:.1f} us, gaps {span - tot_k:.1f} us")


if __name__ == "__main__":
    mode = sys.argv[1]
    if mode == "stats":
        stats(sys.argv[2], sys.argv[3])
    elif mode == "traffic":
        traffic(sys.argv[2], sys.argv[3], sys.argv[4])
    elif mode == "mfma":
        mfma(sys.argv[2], sys.argv[3])
    elif mode == "gaps":
        gaps(sys.argv[2], *(sys.argv[3:4]))
    else:
        raise SystemExit(__doc__)
