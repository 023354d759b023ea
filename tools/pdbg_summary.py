"""Summary of ELP_PDBG pricing timelines (pdbg_dump's file): per launch, the
workgroup roles' start / end spread (us after the launch's first start) and the
tiles' phase times (ctl in, staged, chain done, reduced, end)."""
import sys

import numpy as np


def main(path):
    blocks, cur = [], None
    for line in open(path):
        if line.startswith("#"):
            cur = {"hdr": line.strip(), "rows": []}
            blocks.append(cur)
        elif cur is not None:
            f = line.split()
            cur["rows"].append((f[1], [int(x) for x in f[2:]]))
    for b in blocks:
        print(b["hdr"])
        for role in ("tile", "slack", "apply"):
            r = np.array([v for k, v in b["rows"] if k == role], dtype=float)
            if not len(r):
                continue
            st, en = r[:, 0] / 1e3, r[:, 5] / 1e3
            line = "  %-5s n %4d  start %6.2f..%6.2f  end %6.2f..%6.2f (median %.2f)" % (
                role, len(r), st.min(), st.max(), en.min(), en.max(), np.median(en))
            if role == "tile":
                ph = [np.median((r[:, i] - r[:, 0]) / 1e3) for i in range(1, 6)]
                line += "  tile phases (median after own start) ctl %.2f staged %.2f chain %.2f reduced %.2f end %.2f" % tuple(ph)
            print(line)


if __name__ == "__main__":
    main(sys.argv[1])
