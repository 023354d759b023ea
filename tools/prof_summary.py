"""Summarise a rocprofv3 kernel-trace database (or CSV) per kernel."""
import sqlite3
import sys


def main(path, top=25):
    con = sqlite3.connect(path)
    rows = con.execute(
        "select name, count(*), avg(end-start), sum(end-start), min(end-start), max(end-start) "
        "from kernels group by name order by sum(end-start) desc").fetchall()
    tot = sum(r[3] for r in rows)
    print(f"{'kernel':58s} {'calls':>7s} {'avg_us':>9s} {'min_us':>8s} {'max_us':>8s} {'total_ms':>9s} {'%':>6s}")
    for r in rows[:top]:
        print(f"{r[0][:58]:58s} {r[1]:7d} {r[2]/1e3:9.2f} {r[4]/1e3:8.2f} {r[5]/1e3:8.2f} {r[3]/1e6:9.2f} {100*r[3]/tot:6.1f}")
    print(f"{'TOTAL':58s} {'':7s} {'':9s} {'':8s} {'':8s} {tot/1e6:9.2f}")


if __name__ == "__main__":
    main(sys.argv[1])
