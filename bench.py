#!/usr/bin/env python3
"""bench.py -- simplex iterations/s on the dense random LP of BASELINE.json.

Workload (BASELINE.json configs[2], the config its metric is quoted on):
maximize c'x s.t. A x <= b, x >= 0, A dense 5000 x 50000 fp64 with
A_ij, c_j ~ U[0,1), b_i = n/8 + U n/4, generated on the device
by the counter-based generator (data: synthetic).  A "step" is one simplex
iteration (BTRAN, pricing sweep + argmin, FTRAN, ratio test, basis update;
periodic refactor included).  Inputs are resident in HBM before timing.

    python bench.py [--gpus N] [--steps K] [--warmup W]

Rank 0 prints one JSON line.  With N > 1 (torchrun) the columns of A are
sharded across ranks (one process per GPU, RCCL min-loc + entering-column
exchange per iteration) and all ranks run the same iterations: value is the
iteration rate of the one LP (strong scaling).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

METRIC = "simplex iterations/sec + time-to-optimal, dense LP m=5k n=50k at 1/2/4/8 GPUs"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=1000)
    ap.add_argument("--warmup", type=int, default=100)
    ap.add_argument("--m", type=int, default=5000)
    ap.add_argument("--n", type=int, default=50000)
    ap.add_argument("--seed", type=int, default=1)
    ap.add_argument("--cpu-iters", type=int, default=300,
                    help="iterations of the CPU oracle sample (after --warmup)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--no-optimal", action="store_true", help="skip the run to optimality")
    ap.add_argument("--profile-price", type=int, default=1,
                    help="HIP events around the pricing kernel (roofline)")
    ap.add_argument("--c4", type=int, default=1,
                    help="also time the 10000x500000 column-sharded config (SURVEY config 4)")
    ap.add_argument("--c4-steps", type=int, default=300)
    ap.add_argument("--c4-warmup", type=int, default=100)
    ap.add_argument("--p2p", type=int, default=1,
                    help="N>1: per-iteration min-loc through the xGMI mailbox (0: RCCL all-gather)")
    ap.add_argument("--force-sharded", action="store_true",
                    help="N=1: run the sharded pipeline on a 1-rank RCCL communicator (overhead probe)")
    ap.add_argument("--sparse", type=int, default=1,
                    help="also time the CSC path on a sparse LP (BASELINE config 5)")
    ap.add_argument("--sparse-m", type=int, default=1000)
    ap.add_argument("--sparse-n", type=int, default=10000)
    ap.add_argument("--sparse-steps", type=int, default=1000)
    ap.add_argument("--sparse-cpu-iters", type=int, default=200)
    ap.add_argument("--pricing", choices=["devex", "dantzig"], default="devex",
                    help="pricing rule (elp_control.pricing; devex is lp_solve's default)")
    ap.add_argument("--sync-every", type=int, default=32,
                    help="iterations enqueued between host polls (elp_control.sync_every)")
    ap.add_argument("--compare-rules", type=int, default=1,
                    help="N=1: also solve the LP to optimality with the other pricing rule")
    a = ap.parse_args()
    a.rule = 1 if a.pricing == "devex" else 0
    return a


def enable_p2p(p, rank):
    """xGMI mailbox for the min-loc; collective and agreed by all ranks, so on
    failure every rank falls back to the RCCL all-gather together."""
    from easylp_amd._lib import ElpError
    try:
        p.comm_enable_p2p()
        return True
    except ElpError as e:
        if rank == 0:
            print(f"xGMI mailbox unavailable ({e}); RCCL all-gather min-loc", file=sys.stderr)
        return False


def cpu_baseline(args):
    """The CPU oracle (same algorithm, 1 thread) on a bounded sample of the same LP."""
    import numpy as np
    from oracle import generate_dense, solve_dense
    A, b, c = generate_dense(args.seed, args.m, args.n)
    t0 = time.time()
    r = solve_dense(A, np.ones(args.m, np.int32), b, c, maximize=True, price_rule=args.rule,
                    max_iter=args.warmup + args.cpu_iters, t_mark_iter=args.warmup)
    wall = time.time() - t0
    it = r.stats["iterations"] - args.warmup
    secs = r.stats["seconds_at_mark"]
    return {
        "value": it / secs if secs > 0 else None,
        "unit": "iterations/s",
        "cores": 1,
        "kind": "port",
        "sample": (f"oracle/ (C, -O3, 1 thread) on the same LP, iterations "
                   f"[{args.warmup}, {args.warmup + it}) timed; {wall:.1f}s wall incl. "
                   f"iterations [0,{args.warmup})"),
    }


def committed_traffic(args):
    """HBM traffic per pricing launch from the committed rocprofv3 --pmc FETCH_SIZE
    pass of this same command (tools/gpu_check.sh -> profiles/pmc_traffic.json);
    only used when that pass measured the same LP and iteration window."""
    path = os.path.join(ROOT, "profiles", "pmc_traffic.json")
    try:
        t = json.load(open(path))
    except (OSError, ValueError):
        return None, None
    same = (t.get("m"), t.get("n"), t.get("warmup"), t.get("steps")) == (
        args.m, args.n, args.warmup, args.steps)
    if not same:
        return None, None
    return t["traffic_bytes_per_launch"], "profiles/pmc_traffic.json (rocprofv3 --pmc FETCH_SIZE, x2 gfx950)"


def c4_rate(args, lib, world, rank, local, barrier, dist):
    """Iterations/s of the north-star scaling config: dense LP m=10000 n=500000,
    columns sharded over the ranks.  Same step definition."""
    import torch
    from easylp_amd import Problem
    m, n = 10000, 500000
    from easylp_amd._lib import ELP_PROFILE_PRICE
    p = Problem(m, n, device=local, pricing=args.rule, verbose=ELP_PROFILE_PRICE if args.profile_price else 0)
    if world > 1 or args.force_sharded:
        from easylp_amd.dist import share_unique_id
        p.comm_init(share_unique_id(lib, rank), world, rank)
        if args.p2p:
            enable_p2p(p, rank)
    t_load = time.perf_counter()
    p.load_generated(args.seed)
    barrier()
    t_load = time.perf_counter() - t_load
    p.iterate(args.c4_warmup)
    barrier()
    s0 = p.stats()
    t0 = time.perf_counter()
    p.iterate(args.c4_steps)
    barrier()
    el = time.perf_counter() - t0
    s1 = p.stats()
    if world > 1:
        tt = torch.tensor([el], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        el = float(tt.item())
    it = s1["iterations"] - s0["iterations"]
    p.close()
    # this rank's pricing sweep over its column shard (device clock, as the headline roofline)
    price_s = s1["price_seconds"] - s0["price_seconds"]
    price_b = s1["price_timed_bytes"] - s0["price_timed_bytes"]
    price_n = s1["price_timed_launches"] - s0["price_timed_launches"]
    sweep = None
    if price_s > 0 and price_n > 0:
        gbs = price_b / price_s / 1e9
        sweep = {"achieved": gbs, "peak": 8000.0, "unit": "GB/s", "frac": gbs / 8000.0,
                 "bytes_per_launch": price_b / price_n, "avg_sweep_us": 1e6 * price_s / price_n, "rank": rank}
    return {"workload": "dense random LP m=10000 n=500000 (SURVEY config 4), columns sharded x%d" % world,
            "price_sweep": sweep,
            "value": it / el if el > 0 else None, "unit": "iterations/s", "iterations_timed": it,
            "warmup": args.c4_warmup, "ms_per_step": 1e3 * el / max(it, 1),
            "bump_dim": s1["bump_dim"], "y_rows": s1["y_rows"], "load_s": t_load}


def sparse_rate(args, local, with_cpu):
    """BASELINE config 5 on the CSC path: a seeded sparse LP of Netlib-like shape
    (easylp_amd.synth.sparse_packing, 5 nonzeros per column) plus the Klee-Minty
    cube n=12 (4095 pivots under Dantzig, a few dozen under Devex).  Same step definition; the CPU leg is the
    oracle in its CSC order (price_mode 1) over a bounded window."""
    import numpy as np
    from easylp_amd import Problem
    from easylp_amd.synth import dense_of, sparse_packing
    m, n = args.sparse_m, args.sparse_n
    cp, ri, v, b, c = sparse_packing(args.seed, m, n, 5)
    dirs = np.ones(m, np.int32)
    p = Problem(m, n, device=local, pricing=args.rule)
    p.load_csc(cp, ri, v, dirs, b, c, maximize=True)
    p.iterate(args.warmup)
    s0 = p.stats()
    t0 = time.perf_counter()
    p.iterate(args.sparse_steps)
    el = time.perf_counter() - t0
    s1 = p.stats()
    st = p.solve()
    s2 = p.stats()
    sol = p.solution(st)
    p.close()
    it = s1["iterations"] - s0["iterations"]
    out = {"workload": "sparse LP m=%d n=%d nnz=%d (CSC, BASELINE configs[4])" % (m, n, int(cp[-1])),
           "value": it / el if el > 0 else None, "unit": "iterations/s", "iterations_timed": it,
           "warmup": args.warmup, "ms_per_step": 1e3 * el / max(it, 1),
           "time_to_optimal_s": s2["seconds_loop"], "status": st, "objective": sol.objval,
           "iterations_to_optimal": s2["iterations"], "bump_dim": s2["bump_dim"]}
    # Klee-Minty cube (degenerate-path case): time to optimal on the GPU
    km = 12
    rows, cols, vals = [], [], []
    for i in range(km):
        for j in range(i + 1):
            rows.append(i)
            cols.append(j)
            vals.append(1.0 if i == j else 2.0 ** (i - j + 1))
    import scipy.sparse as sp
    K = sp.csc_matrix((vals, (rows, cols)), shape=(km, km))
    kb = np.array([5.0 ** (i + 1) for i in range(km)])
    kc = np.array([2.0 ** (km - 1 - j) for j in range(km)])
    with Problem(km, km, device=local, pricing=args.rule) as pk:
        pk.load_csc(K.indptr, K.indices, K.data, np.ones(km, np.int32), kb, kc, maximize=True)
        kst = pk.solve()
        ks = pk.stats()
        kobj = pk.solution(kst).objval
    out["klee_minty"] = {"n": km, "iterations": ks["iterations"], "seconds": ks["seconds_loop"],
                         "objective": kobj, "expected": 5.0 ** km}
    if with_cpu:
        from oracle import solve_dense
        A = dense_of(cp, ri, v, m, n)
        w = args.warmup
        r = solve_dense(A, dirs, b, c, maximize=True, price_mode=1, price_rule=args.rule,
                        max_iter=w + args.sparse_cpu_iters, t_mark_iter=w)
        cit = r.stats["iterations"] - w
        out["cpu_baseline"] = {"value": cit / r.stats["seconds_at_mark"], "unit": "iterations/s",
                               "cores": 1, "kind": "port",
                               "sample": "oracle/ (C, -O3, 1 thread, CSC order) iterations [%d, %d)" % (w, w + cit)}
        t0 = time.perf_counter()
        rk = solve_dense(K.toarray(), np.ones(km, np.int32), kb, kc, maximize=True, price_mode=1,
                         price_rule=args.rule)
        out["klee_minty"]["cpu_seconds"] = time.perf_counter() - t0
        out["klee_minty"]["cpu_iterations"] = rk.stats["iterations"]
    return out


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if args.gpus != world and world > 1:
        raise SystemExit(f"--gpus {args.gpus} but WORLD_SIZE={world}")

    import torch
    import torch.distributed as dist

    if world > 1:
        dist.init_process_group("gloo", init_method="env://")
    elif args.force_sharded:
        os.environ["ELP_RCCL_SINGLE"] = "1"
        os.environ.setdefault("MASTER_ADDR", "127.0.0.1")
        os.environ.setdefault("MASTER_PORT", "29533")
        dist.init_process_group("gloo", init_method="env://", rank=0, world_size=1)
    torch.cuda.set_device(local)

    from easylp_amd import Problem
    from easylp_amd._lib import ELP_PROFILE_PRICE, load

    lib = load()
    verbose = ELP_PROFILE_PRICE if args.profile_price else 0
    p = Problem(args.m, args.n, device=local, verbose=verbose, pricing=args.rule, sync_every=args.sync_every)
    if world > 1 or args.force_sharded:
        from easylp_amd.dist import share_unique_id
        p.comm_init(share_unique_id(lib, rank), world, rank)
        if args.p2p:
            args.p2p = int(enable_p2p(p, rank))

    p.load_generated(args.seed)

    def barrier():
        torch.cuda.synchronize()
        if world > 1:
            dist.barrier()

    # warmup (untimed)
    st = p.iterate(args.warmup)
    barrier()
    s0 = p.stats()
    t0 = time.perf_counter()
    st = p.iterate(args.steps)
    barrier()
    t1 = time.perf_counter()
    s1 = p.stats()
    elapsed = t1 - t0
    if world > 1:
        tt = torch.tensor([elapsed], dtype=torch.float64)
        dist.all_reduce(tt, op=dist.ReduceOp.MAX)
        elapsed = float(tt.item())
    iters = s1["iterations"] - s0["iterations"]
    value = iters / elapsed if elapsed > 0 else 0.0

    price_dev_bytes = (s1["price_bytes"] - s0["price_bytes"]) / max(iters, 1)
    price_s = s1["price_seconds"] - s0["price_seconds"]
    price_b = s1["price_timed_bytes"] - s0["price_timed_bytes"]
    price_n = s1["price_timed_launches"] - s0["price_timed_launches"]
    achieved = price_b / price_s / 1e9 if price_s > 0 else None

    # run on to optimality: time-to-optimal (device generation excluded)
    tto = None
    final = None
    if not args.no_optimal:
        st = p.solve()
        barrier()
        s2 = p.stats()
        sol = p.solution(st)
        tto = s2["seconds_loop"]
        final = {"status": st, "iterations_to_optimal": s2["iterations"],
                 "objective": sol.objval, "bump_dim": s2["bump_dim"], "y_rows": s2["y_rows"],
                 "refactors": s2["refactors"]}
        if world > 1:
            tt = torch.tensor([tto], dtype=torch.float64)
            dist.all_reduce(tt, op=dist.ReduceOp.MAX)
            tto = float(tt.item())

    traffic, traffic_src = committed_traffic(args) if world == 1 else (None, None)

    other = None  # the same LP to optimality under the other pricing rule
    if args.compare_rules and world == 1 and not args.no_optimal and not args.force_sharded:
        p.close()
        q = Problem(args.m, args.n, device=local, pricing=1 - args.rule, sync_every=args.sync_every)
        q.load_generated(args.seed)
        qst = q.solve()
        qs = q.stats()
        other = {"pricing": "dantzig" if args.rule else "devex", "status": qst,
                 "objective": q.solution(qst).objval, "iterations_to_optimal": qs["iterations"],
                 "time_to_optimal_s": qs["seconds_loop"]}
        q.close()

    c4 = None
    if args.c4:
        p.close()  # free the 5000x50000 problem first
        c4 = c4_rate(args, lib, world, rank, local, barrier, dist)

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu:
        cpu = cpu_baseline(args)

    sparse = None
    if args.sparse and world == 1:
        sparse = sparse_rate(args, local, rank == 0 and not args.no_cpu)

    if rank == 0:
        line = {
            "metric": METRIC,
            "value": value,
            "unit": "iterations/s",
            "n_gpus": world,
            "steps": args.steps,
            "warmup": args.warmup,
            "ms_per_step": 1e3 * elapsed / max(iters, 1),
            "higher_is_better": True,
            "scaling": "strong",
            "vs_baseline": None,
            "dtype": "f64",
            "data": "synthetic (counter-based generator on device, seed %d)" % args.seed,
            "config": {
                "workload": "dense random LP m=%d n=%d (BASELINE configs[2])" % (args.m, args.n),
                "m": args.m, "n": args.n, "seed": args.seed,
                "parallelism": ("column-shard x%d, %s min-loc" % (world, "xGMI mailbox" if args.p2p else "RCCL all-gather")
                                if world > 1 or args.force_sharded else "single GPU"),
                "iterations_timed": iters,
                "pricing": args.pricing,
            },
            "time_to_optimal_s": tto,
            "final": final,
            "other_pricing": other,
            "roofline": {
                "kernel": "k_price (pricing sweep + %s argmin)" % args.pricing,
                "bound": "hbm",
                "achieved": achieved,
                "peak": HBM_PEAK_GBS,
                "unit": "GB/s",
                "frac": (achieved / HBM_PEAK_GBS) if achieved else None,
                "traffic": traffic,
                "traffic_source": traffic_src,
                "bytes_per_launch": price_b / price_n if price_n else price_dev_bytes,
                "avg_launch_us": 1e6 * price_s / price_n if price_n else None,
                "launches_timed": price_n,
            },
            "cpu_baseline": cpu,
            "scaling_config": c4,
            "sparse_config": sparse,
        }
        print(json.dumps(line), flush=True)
    p.close()
    if world > 1:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
