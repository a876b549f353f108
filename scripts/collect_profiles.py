"""Copy the results of scripts/gpu_profiles.sh (gpurun_out/) into profiles/<round>/ and profiles/traffic_cN.json:

    python scripts/collect_profiles.py r03

bench lines, standalone benches, the rocprofv3 --stats summaries (CSV), the PMC summaries (per-kernel FETCH / WRITE,
VALU busy and wave-cycle fractions), the traffic files bench.py reads, the LBA FP64-MFMA counters and the GPU test
log."""
import csv
import json
import os
import shutil
import sys
from collections import defaultdict

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
G = os.path.join(ROOT, "gpurun_out")


def cp(src, dst):
    s = os.path.join(G, src)
    if os.path.exists(s):
        shutil.copyfile(s, dst)
        print("copied", src, "->", os.path.relpath(dst, ROOT))
    else:
        print("missing", src)


def mfma(dirname, out):
    f = None
    for r, _, fs in os.walk(os.path.join(G, dirname)):
        for x in fs:
            if x.endswith("counter_collection.csv"):
                f = os.path.join(r, x)
    if f is None:
        print("missing", dirname)
        return
    agg = defaultdict(lambda: defaultdict(list))
    for r in csv.DictReader(open(f)):
        agg[r["Kernel_Name"].split("(")[0]][r["Counter_Name"]].append(float(r["Counter_Value"]))
    res = {}
    for k, v in agg.items():
        mops = sum(v.get("SQ_INSTS_VALU_MFMA_MOPS_F64", [0.0])) / max(len(v.get("SQ_INSTS_VALU_MFMA_MOPS_F64", [1])), 1)
        if mops == 0:
            continue
        busy = v.get("SQ_VALU_MFMA_BUSY_CYCLES", [0.0])
        gui = v.get("GRBM_GUI_ACTIVE", [1.0])
        frac = (sum(busy) / len(busy)) / (1024 * max(sum(gui) / len(gui), 1.0))
        res[k] = {"fp64_mfma_flop_per_launch": mops * 512, "launches": len(v["SQ_INSTS_VALU_MFMA_MOPS_F64"]),
                  "mfma_busy_frac": frac,
                  # the batch of 32 runs as two stream groups: 16 workgroups (CUs) per k_ldlt launch
                  "mfma_busy_frac_of_16_cus": frac * 256 / 16,
                  "note": "SQ_VALU_MFMA_BUSY_CYCLES / (1024 SIMDs x GRBM_GUI_ACTIVE), whole GPU; x 256 / 16 for "
                          "the CUs a 16-window launch occupies"}
    json.dump(res, open(out, "w"), indent=1)
    print("wrote", os.path.relpath(out, ROOT))


def main():
    rnd = sys.argv[1] if len(sys.argv) > 1 else "r03"
    P = os.path.join(ROOT, "profiles", rnd)
    os.makedirs(P, exist_ok=True)
    for c in ("c1", "c2", "c3", "c4"):
        cp(f"bench_{c}.json", os.path.join(P, f"bench_{c}.json"))
    cp("bench_c2_world.json", os.path.join(P, "bench_c2_world.json"))
    cp(f"{rnd}pose.json", os.path.join(P, "pose_pmc_c2.json"))
    for n in ("lba_bench", "tri_bench", "pose_c2", "fuse_c2", "bow_c2"):
        cp(f"{n}.json", os.path.join(P, f"{n}.json"))
    cp("pytest_gpu.log", os.path.join(P, "pytest_gpu.log"))
    for c in ("c1", "c2"):
        cp(f"pmc_{rnd}{c}.json", os.path.join(P, f"pmc_{c}_64frame.json"))
        cp(f"prof_{rnd}{c}/run_kernel_stats.csv", os.path.join(P, f"kernel_stats_{c}_64frame.csv"))
        cp(f"traffic_{c}.json", os.path.join(ROOT, "profiles", f"traffic_{c}.json"))
    cp(f"prof_{rnd}default_c2/run_kernel_stats.csv", os.path.join(P, "kernel_stats_c2_default_command.csv"))
    cp("roofline_check_c2.json", os.path.join(P, "roofline_check_c2.json"))
    cp("bench_traced_c2.json", os.path.join(P, "bench_traced_c2.json"))
    cp(f"{rnd}lba_trace/run_kernel_stats.csv", os.path.join(P, "kernel_stats_lba_batch32.csv"))
    cp(f"{rnd}lba.json", os.path.join(P, "lba_pmc_batch32.json"))
    mfma(f"pmc_{rnd}lba", os.path.join(P, "lba_mfma_f64.json"))
    cp(f"{rnd}lba_ring/run_kernel_stats.csv", os.path.join(P, "kernel_stats_lba_ring32.csv"))
    mfma(f"pmc_{rnd}lba_ring", os.path.join(P, "lba_mfma_f64_ring.json"))


if __name__ == "__main__":
    main()
