"""Per-kernel HBM traffic of one full solve from two rocprofv3 PMC passes
(FETCH_SIZE and WRITE_SIZE need separate passes: MI355X_MICROARCH.md, TCC
counter budget) of `bench.py --steps 1 --warmup 0 ...` -- the latency kernels
next to the pricing sweep.

FETCH_SIZE on gfx950 reports half the bytes of a wide (16 B per lane)
coalesced read; narrower or scattered reads (most of the latency kernels) are
uncalibrated, so both the raw 1024 x FETCH_SIZE and the doubled figure are
given.  Algorithmic bytes are evaluated at the solve's
final bump size k and |Y| (both grow nearly monotonically), i.e. an upper
bound per iteration.
Usage: python tools/pmc_kernels.py <fetch counter_collection.csv> <write counter_collection.csv> <bench.json>
"""
import csv
import json
import sys
from collections import defaultdict


def per_kernel(path, counter):
    acc = defaultdict(lambda: [0, 0.0])
    for r in csv.DictReader(open(path)):
        if r["Counter_Name"] != counter:
            continue
        name = r["Kernel_Name"].split("(")[0]
        acc[name][0] += 1
        acc[name][1] += float(r["Counter_Value"]) * 1024.0
    return acc


def main(fetch_csv, write_csv, bench_json):
    b = json.loads(open(bench_json).read().strip().splitlines()[-1])
    m, n = b["config"]["m"], b["config"]["n"]
    k, ny = b["final"]["bump_dim"], b["final"]["y_rows"]
    model = {  # per launch, at the final k and |Y|
        "k_price": 8.0 * ny * n + 9.0 * n + 12.0 * ny + 24.0 * n,
        "k_select_ftran": 8.0 * k * k + 32.0 * (n / 128 + 2),
        "k_ftran_zr": 8.0 * m * k,
        "k_ratio": 8.0 * k * k + 16.0 * n,
    }
    f = per_kernel(fetch_csv, "FETCH_SIZE")
    w = per_kernel(write_csv, "WRITE_SIZE")
    rows = []
    for name, (cnt, tot) in sorted(f.items(), key=lambda kv: -kv[1][1]):
        if cnt < 100:
            continue  # refactor / load kernels: a handful of dispatches
        base = name.replace("void ", "").replace("elp::", "").split("<")[0]
        wc, wt = w.get(name, (0, 0.0))
        rows.append({
            "kernel": name,
            "dispatches": cnt,
            "fetch_raw_bytes_per_launch": tot / cnt,
            "fetch_x2_bytes_per_launch": 2.0 * tot / cnt,
            "write_bytes_per_launch": wt / wc if wc else None,
            "algorithmic_bytes_at_final_k": model.get(base),
        })
    print(json.dumps({"m": m, "n": n, "final_k": k, "final_y_rows": ny,
                      "iterations": b["final"]["iterations_to_optimal"], "kernels": rows}, indent=1))


if __name__ == "__main__":
    main(*sys.argv[1:4])
