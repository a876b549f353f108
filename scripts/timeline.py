"""Leg overlap from a rocprofv3 kernel trace (run_kernel_trace.csv): kernels classified into Tracking (ORB extraction,
motion / local-map searches, PoseOptimization), keyframe searches (BoW, SearchForTriangulation, Fuse) and
LocalBundleAdjustment (+ exchange); per tracking step (from one extraction pyramid launch to the next) the step's
span, each leg's busy time (union of its kernels' intervals), the time both legs are busy and the idle time.
Usage: python scripts/timeline.py <run_kernel_trace.csv> [first_kernel_substring]"""
import csv
import sys


def leg(name):
    n = name
    if "lba::" in n or "k_read_windows" in n or "k_pack" in n or "k_apply" in n:
        return "lba"
    if "bow" in n or "k_tri" in n or "fuse" in n or "distinct" in n:
        return "kfs"
    if "mam::" in n:
        return "trk"
    return "oth"   # torch / runtime copies and fills (either leg)


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def length(u):
    return sum(b - a for a, b in u)


def inter(u, v):
    i = j = 0
    s = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            s += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return s


rows = list(csv.DictReader(open(sys.argv[1])))
first = sys.argv[2] if len(sys.argv) > 2 else "k_pyr"
ks = []
for r in rows:
    ks.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"], r.get("Queue_Id", "")))
ks.sort()
starts = [k[0] for k in ks if first in k[2]]
# a step begins at the first pyramid launch after a gap (the lanes' pyramids are one step)
steps = []
for s in starts:
    if not steps or s - steps[-1] > 200_000:
        steps.append(s)
print(f"{len(ks)} kernels, {len(steps)} steps; queues: {sorted(set(k[3] for k in ks))}")
tot = {"span": 0, "trk": 0, "lba": 0, "kfs": 0, "oth": 0, "map": 0, "both": 0, "idle": 0}
n = 0
for a, b in zip(steps[:-1], steps[1:]):
    iv = {"trk": [], "lba": [], "kfs": [], "oth": []}
    for s, e, name, q in ks:
        if e <= a or s >= b:
            continue
        iv[leg(name)].append((max(s, a), min(e, b)))
    u = {k: union(v) for k, v in iv.items()}
    um = union(iv["lba"] + iv["kfs"])
    allu = union(iv["trk"] + iv["lba"] + iv["kfs"] + iv["oth"])
    span = b - a
    row = {"span": span, "trk": length(u["trk"]), "lba": length(u["lba"]), "kfs": length(u["kfs"]), "oth": length(u["oth"]),
           "map": length(um), "both": inter(u["trk"], um), "idle": span - length(allu)}
    for k in tot:
        tot[k] += row[k]
    n += 1
    print("step %3d" % n + "".join(f" {k} {v / 1e3:8.1f}us" for k, v in row.items()))
if n:
    print("mean    " + "".join(f" {k} {v / n / 1e3:8.1f}us" for k, v in tot.items()))
