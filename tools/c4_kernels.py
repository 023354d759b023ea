"""Per-kernel averages over the last N iterations of the 10000x500000 config in a
rocprofv3 kernel trace of bench.py (its k_price launches are the > 50 us ones)."""
import collections
import csv
import sys

rows = sorted((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"])
              for r in csv.DictReader(open(sys.argv[1])))
N = int(sys.argv[2]) if len(sys.argv) > 2 else 300
idx = [i for i, r in enumerate(rows) if "k_price" in r[2] and r[1] - r[0] > 50000][-N:]
i0, i1 = idx[0], idx[-1]
it = len(idx) - 1
dur = collections.defaultdict(list)
for a in rows[i0:i1]:
    dur[a[2].split("(")[0]].append(a[1] - a[0])
print(f"iterations {it}  wall/iter {(rows[i1][0] - rows[i0][0]) / it / 1e3:.2f} us")
for n in sorted(dur, key=lambda n: -sum(dur[n])):
    print(f"{n[-34:]:34s} {len(dur[n]) / it:5.2f} {sum(dur[n]) / len(dur[n]) / 1e3:8.2f}")
