#!/usr/bin/env python3
"""Per-kernel summary of a rocprofv3 database (the rocpd SQLite output that
rocprofv3 writes when no --output-format is given): dispatches, average and
total duration, by total time.

  python tools/rocpd_stats.py gpurun_out/<run>/prof/<name>_results.db [limit]
"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    limit = int(sys.argv[2]) if len(sys.argv) > 2 else 20
    c = sqlite3.connect(db)
    q = ("select name, count(*), avg(duration) / 1e3, sum(duration) / 1e6 from kernels "
         "group by name order by sum(duration) desc limit ?")
    print(f"{'calls':>5} {'avg_us':>10} {'total_ms':>9}  kernel")
    for name, n, avg_us, tot_ms in c.execute(q, (limit,)):
        print(f"{n:5d} {avg_us:10.1f} {tot_ms:9.2f}  {name}")


if __name__ == "__main__":
    main()
