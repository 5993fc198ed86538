"""Per-kernel summary from a rocprofv3 rocpd database (default output format):
  python tools/rocpd_top.py <dir-or-db> [divisor] [n]
prints calls, average us and total us / divisor (e.g. timed steps) per kernel."""
import glob
import os
import sqlite3
import sys


def main():
    path = sys.argv[1]
    div = float(sys.argv[2]) if len(sys.argv) > 2 else 1.0
    n = int(sys.argv[3]) if len(sys.argv) > 3 else 25
    db = path if path.endswith(".db") else glob.glob(os.path.join(path, "**", "*.db"), recursive=True)[0]
    c = sqlite3.connect(db)
    q = ("select name, count(*), avg(end-start), sum(end-start), max(scratch_size), max(vgpr_count) "
         "from kernels group by name order by sum(end-start) desc limit ?")
    print(f"{'kernel':72s} {'calls':>6s} {'avg_us':>9s} {'tot_us/div':>10s} scr vgpr")
    for name, k, avg, tot, scr, vg in c.execute(q, (n,)):
        print(f"{name[:72]:72s} {k:6d} {avg / 1e3:9.1f} {tot / 1e3 / div:10.1f} {scr:3d} {vg}")


if __name__ == "__main__":
    main()
