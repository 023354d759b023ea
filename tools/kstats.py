"""Print a rocprofv3 kernel_stats.csv (per-kernel calls, average / max us,
total ms), largest total first."""
import csv
import sys


def main(path, top=30):
    rows = list(csv.DictReader(open(path)))
    rows.sort(key=lambda r: -float(r["TotalDurationNs"]))
    tot = sum(float(r["TotalDurationNs"]) for r in rows)
    print(f"{'kernel':60s} {'calls':>7s} {'avg_us':>8s} {'max_us':>8s} {'total_ms':>9s}")
    for r in rows[:top]:
        print(f"{r['Name'][:60]:60s} {int(r['Calls']):7d} {float(r['AverageNs'])/1e3:8.2f} "
              f"{float(r['MaxNs'])/1e3:8.2f} {float(r['TotalDurationNs'])/1e6:9.2f}")
    print(f"{'TOTAL':60s} {'':7s} {'':8s} {'':8s} {tot/1e6:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
