"""Per-kernel duration summary of a rocprofv3 rocpd database (run_results.db).

    python tools/rocpd_stats.py gpurun_out/prof_x/run_results.db [name-filter]
"""
import collections
import sqlite3
import sys


def main():
    con = sqlite3.connect(sys.argv[1])
    filt = sys.argv[2] if len(sys.argv) > 2 else ""
    tabs = [r[0] for r in con.execute("select name from sqlite_master where type='table'")]
    kd = next(t for t in tabs if t.startswith("rocpd_kernel_dispatch"))
    ks = next(t for t in tabs if t.startswith("rocpd_info_kernel_symbol"))
    rows = con.execute(f"select s.kernel_name, d.end - d.start from {kd} d join {ks} s on d.kernel_id = s.id")
    agg = collections.defaultdict(list)
    for name, dur in rows:
        if filt in name:
            agg[name].append(dur)
    print(f"{'calls':>6} {'avg_us':>10} {'min_us':>10} {'total_ms':>10}  kernel")
    for name, d in sorted(agg.items(), key=lambda kv: -sum(kv[1])):
        print(f"{len(d):6d} {sum(d) / len(d) / 1e3:10.2f} {min(d) / 1e3:10.2f} {sum(d) / 1e6:10.3f}  {name[:110]}")


if __name__ == "__main__":
    main()
