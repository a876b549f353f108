"""Concurrency of kernel categories in a rocprofv3 results database: for the last --window ms of the trace, the busy
time of each category (union of its kernels' intervals), the time categories overlap, and a coarse timeline."""
import argparse
import sqlite3


def category(name):
    if "mam::lba::" in name:
        return "lba"
    if any(k in name for k in ("k_fuse", "k_distinct", "k_tri", "k_bow", "k_ring", "k_sin", "triang", "k_grid_kf",
                               "k_exchange", "k_pack", "k_apply", "k_copy_rows", "bow::")):
        return "search"
    if "at::native" in name or "rocclr" in name:
        return "other"
    return "track"


def union(iv):
    iv = sorted(iv)
    out = []
    for a, b in iv:
        if out and a <= out[-1][1]:
            out[-1][1] = max(out[-1][1], b)
        else:
            out.append([a, b])
    return out


def inter(u, v):
    i = j = 0
    tot = 0
    while i < len(u) and j < len(v):
        a, b = max(u[i][0], v[j][0]), min(u[i][1], v[j][1])
        if a < b:
            tot += b - a
        if u[i][1] < v[j][1]:
            i += 1
        else:
            j += 1
    return tot


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--window", type=float, default=60.0, help="ms at the end of the trace")
    ap.add_argument("--bin", type=float, default=0.5, help="timeline bin, ms")
    ap.add_argument("--names", action="store_true", help="list the kernel names per category")
    ap.add_argument("--end-at", default=None, help="end the window at the last kernel of this category")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    rows = list(c.execute("select name, start, end from kernels order by start"))
    t_end = max(r[2] for r in rows if a.end_at is None or category(r[0]) == a.end_at)
    t0 = t_end - a.window * 1e6
    cats = {}
    names = {}
    for n, s, e in rows:
        if e < t0 or s > t_end:
            continue
        k = category(n)
        cats.setdefault(k, []).append((max(s, t0), min(e, t_end)))
        names.setdefault(k, set()).add(n.split("(")[0][:60])
    U = {k: union(v) for k, v in cats.items()}
    span = (t_end - t0) / 1e6
    print(f"last {span:.1f} ms")
    for k, u in U.items():
        print(f"  {k:7s} busy {sum(b - a for a, b in u) / 1e6:8.2f} ms  kernels {len(cats[k])}")
    ks = sorted(U)
    for i in range(len(ks)):
        for j in range(i + 1, len(ks)):
            print(f"  overlap {ks[i]} & {ks[j]}: {inter(U[ks[i]], U[ks[j]]) / 1e6:.2f} ms")
    if a.names:
        for k, v in names.items():
            print(k, sorted(v))
    nb = int(a.window / a.bin)
    line = {k: [] for k in ks}
    for b in range(nb):
        lo, hi = t0 + b * a.bin * 1e6, t0 + (b + 1) * a.bin * 1e6
        for k in ks:
            f = inter(U[k], [[lo, hi]]) / (a.bin * 1e6)
            line[k].append(" .:-=#"[min(5, int(f * 5.999))])
    for k in ks:
        print(f"{k:7s} |" + "".join(line[k]) + "|")


if __name__ == "__main__":
    main()
