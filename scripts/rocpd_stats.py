"""Per-kernel statistics from a rocprofv3 results database (rocpd sqlite: the default output format of this image's
rocprofv3): name, calls, total / mean / min / max microseconds, sorted by total."""
import argparse
import sqlite3
import statistics


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("db")
    ap.add_argument("--top", type=int, default=30)
    ap.add_argument("--skip", type=int, default=0, help="ignore the first N dispatches of every kernel (warm-up)")
    ap.add_argument("--csv", default=None, help="also write the table as CSV here")
    a = ap.parse_args()
    c = sqlite3.connect(a.db)
    per = {}
    for name, dur in c.execute("select name, duration from kernels order by start"):
        per.setdefault(name, []).append(dur / 1e3)
    rows = []
    for name, v in per.items():
        v = v[a.skip:]
        if v:
            rows.append((name, len(v), sum(v), statistics.mean(v), min(v), max(v)))
    rows.sort(key=lambda r: -r[2])
    out = ["name,calls,total_us,mean_us,min_us,max_us"]
    for r in rows[:a.top]:
        print(f"{r[0][:70]:70s} {r[1]:6d} {r[2]:10.1f} {r[3]:8.2f} {r[4]:8.2f} {r[5]:8.2f}")
        out.append(f"\"{r[0]}\",{r[1]},{r[2]:.3f},{r[3]:.3f},{r[4]:.3f},{r[5]:.3f}")
    if a.csv:
        with open(a.csv, "w") as f:
            f.write("\n".join(out) + "\n")


if __name__ == "__main__":
    main()
