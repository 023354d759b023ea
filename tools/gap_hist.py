"""Idle time between consecutive kernels of the LAST full solve in a rocprofv3
kernel trace (bench.py --steps 1): span, busy time, and the idle time split by
gap size, with the kernel that follows the largest gaps.
usage: python tools/gap_hist.py kernel_trace.csv"""
import csv
import sys
from collections import Counter

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"].split("(")[0])
              for r in csv.DictReader(open(sys.argv[1])))
# the last solve: from the last k_init_cols (a load) to the end
starts = [i for i, r in enumerate(rows) if "k_init_cols" in r[2]]
lo = starts[-1] if starts else 0
rows = rows[lo:]
span = rows[-1][1] - rows[0][0]
busy = sum(e - s for s, e, _ in rows)
bins = [(0, 2e3), (2e3, 5e3), (5e3, 20e3), (20e3, 100e3), (100e3, 1e12)]
tot = Counter()
cnt = Counter()
after = Counter()
for a, b in zip(rows, rows[1:]):
    g = max(0, b[0] - a[1])
    for lo_, hi_ in bins:
        if lo_ <= g < hi_:
            tot[(lo_, hi_)] += g
            cnt[(lo_, hi_)] += 1
            if lo_ >= 5e3:
                after[b[2][-30:]] += g
print(f"kernels {len(rows)}  span {span / 1e6:.2f} ms  busy {busy / 1e6:.2f} ms  idle {(span - busy) / 1e6:.2f} ms")
for k in bins:
    print(f"  gaps {k[0] / 1e3:>6.0f}-{min(k[1], 1e9) / 1e3:<8.0f} us: {cnt[k]:6d} gaps, {tot[k] / 1e6:7.2f} ms")
print("idle >= 5 us before:")
for k, v in after.most_common(8):
    print(f"  {k:32s} {v / 1e6:7.2f} ms")
