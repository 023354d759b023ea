"""Per-kernel averages of a rocprofv3 kernel trace over bench.py's timed
solves, next to the bench line's own device-clock pricing figure.

bench.py --steps K --warmup W runs W + K identical full solves of L pricing
launches each (final.price_launches_per_solve); the timed solves are k_price
dispatches [W*L, (W+K)*L).  Every kernel dispatched between the first and the
last of those (loads included) is counted.
Usage: python tools/window_stats.py <kernel_trace.csv> <bench.json>
"""
import csv
import json
import sys
from collections import defaultdict


def main(trace, bench_json):
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    W, K = b["warmup"], b["steps"]
    L = b["final"]["price_launches_per_solve"]
    rows = []
    with open(trace) as f:
        for r in csv.DictReader(f):
            rows.append((int(r["Start_Timestamp"]), int(r["End_Timestamp"]), r["Kernel_Name"]))
    rows.sort()
    price = [i for i, r in enumerate(rows) if "k_price" in r[2]]
    lo, hi = price[W * L], price[(W + K) * L - 1]
    dur, n = defaultdict(float), defaultdict(int)
    for s, e, name in rows[lo:hi + 1]:
        key = name.split("(")[0].replace("void ", "").replace("elp::", "")
        dur[key] += e - s
        n[key] += 1
    wall = rows[hi][1] - rows[lo][0]
    kern = {k: {"calls": n[k], "avg_us": dur[k] / n[k] / 1e3, "total_ms": dur[k] / 1e6}
            for k in sorted(dur, key=lambda k: -dur[k])}
    # k_price<0> / k_price<1> (cached / non-temporal sweep loads): one figure
    kps = [k for k in kern if k.split("<")[0] == "k_price"]
    kp = {}
    if kps:
        calls = sum(kern[k]["calls"] for k in kps)
        tot = sum(kern[k]["total_ms"] for k in kps)
        kp = {"calls": calls, "avg_us": tot * 1e3 / calls, "total_ms": tot}
    out = {"timed_solves": K, "price_launches_per_solve": L, "window_wall_ms": wall / 1e6,
           "k_price_avg_us_rocprof": kp.get("avg_us"),
           "k_price_avg_us_bench": b["roofline"]["avg_launch_us"], "bench_timer": b["roofline"].get("timer"),
           "bytes_per_launch": b["roofline"]["bytes_per_launch"],
           "frac_from_rocprof": (b["roofline"]["bytes_per_launch"] / (kp["avg_us"] * 1e-6) / 8e12) if kp else None,
           "kernels": kern}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
