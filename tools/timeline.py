"""Per-iteration timeline from a rocprofv3 kernel-trace CSV: kernel durations
and the idle gap before each kernel, over iterations [skip, skip+count) (an
iteration starts at each k_price launch)."""
import csv
import sys
from collections import defaultdict


def main(path, skip=100, count=1000, first="k_price"):
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    starts = [i for i, r in enumerate(rows) if first in r[2]]
    # skip the warmup solve's iterations: take the LAST run of iterations
    lo, hi = starts[skip], starts[min(skip + count, len(starts) - 1)]
    dur, gap, n = defaultdict(float), defaultdict(float), defaultdict(int)
    for i in range(lo, hi):
        s, e, name = rows[i]
        key = name.split("(")[0].replace("void ", "").replace("elp::", "")
        dur[key] += e - s
        gap[key] += max(0, s - rows[i - 1][1])
        n[key] += 1
    iters = hi - lo and len([i for i in starts if lo <= i < hi])
    wall = rows[hi][0] - rows[lo][0]
    print(f"iterations {iters}  wall/iter {wall / iters / 1e3:.2f} us")
    print(f"{'kernel':34s} {'calls/it':>8s} {'dur_us':>8s} {'gap_us':>8s}")
    for k in sorted(dur, key=lambda k: -dur[k]):
        print(f"{k[:34]:34s} {n[k] / iters:8.2f} {dur[k] / n[k] / 1e3:8.2f} {gap[k] / n[k] / 1e3:8.2f}")
    print(f"sum dur/iter {sum(dur.values()) / iters / 1e3:.2f} us  sum gap/iter {sum(gap.values()) / iters / 1e3:.2f} us")


if __name__ == "__main__":
    main(sys.argv[1], *(int(a) for a in sys.argv[2:4]))
