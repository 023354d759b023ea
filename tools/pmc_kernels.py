"""Per-kernel averages of a rocprofv3 --pmc pass (counter_collection.csv):
counter value per dispatch, averaged over the dispatches of each kernel, plus
the wave-cycle split (SQ_WAIT_ANY / SQ_WAIT_INST_ANY / SQ_ACTIVE_INST_ANY over
SQ_WAVE_CYCLES) when those counters are present.  usage: pmc_kernels.py CSV"""
import collections
import csv
import sys


def main(path):
    per = collections.defaultdict(lambda: collections.defaultdict(float))
    disp = collections.defaultdict(set)
    for r in csv.DictReader(open(path)):
        name = r.get("Kernel_Name", "?").split("(")[0]
        ctr = r.get("Counter_Name")
        val = float(r.get("Counter_Value", 0) or 0)
        did = r.get("Dispatch_Id") or r.get("Correlation_Id")
        per[name][ctr] += val
        disp[name].add(did)
    for name in sorted(per, key=lambda n: -per[n].get("SQ_WAVE_CYCLES", 0)):
        n = max(1, len(disp[name]))
        c = per[name]
        line = f"{name[-30:]:30s} n {n:6d}"
        for k in sorted(c):
            line += f"  {k} {c[k] / n:.0f}"
        wc = c.get("SQ_WAVE_CYCLES", 0)
        if wc:
            line += "  | wait %.0f%% issue-stall %.0f%% active %.0f%%" % (
                100 * c.get("SQ_WAIT_ANY", 0) / wc, 100 * c.get("SQ_WAIT_INST_ANY", 0) / wc,
                100 * c.get("SQ_ACTIVE_INST_ANY", 0) / wc)
        print(line)


if __name__ == "__main__":
    main(sys.argv[1])
