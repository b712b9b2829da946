"""Per-kernel summary (calls, average / total microseconds) from a rocprofv3 results database
(``rocprofv3 --kernel-trace -o NAME`` writes NAME_results.db): usage ``db_stats.py DB [top]``."""
import os
import sqlite3
import sys


def main():
    db = sys.argv[1]
    if not os.path.isfile(db):  # (sqlite3.connect would create an empty database file)
        sys.exit(f"no such rocprofv3 database: {db}")
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    c = sqlite3.connect(db)
    rows = list(c.execute("select name, count(*), avg(end - start) / 1000.0, sum(end - start) / 1000.0 from kernels "
                          "group by name order by sum(end - start) desc limit ?", (top,)))
    total = sum(r[3] for r in c.execute("select name, count(*), 0, sum(end - start) / 1000.0 from kernels group by name"))
    print(f"{'calls':>6} {'avg_us':>10} {'total_us':>12} {'pct':>6}  kernel")
    for name, n, avg, tot in rows:
        print(f"{n:6d} {avg:10.1f} {tot:12.1f} {100 * tot / total:6.2f}  {name[:140]}")


if __name__ == "__main__":
    main()
