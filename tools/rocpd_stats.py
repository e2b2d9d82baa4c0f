"""Per-kernel time summary from a rocprofv3 SQLite (rocpd) database: name, calls, avg/min us,
total %.  Usage: python tools/rocpd_stats.py <results.db> [top N] [name filter]"""
import sqlite3
import sys


def main():
    db = sys.argv[1]
    top = int(sys.argv[2]) if len(sys.argv) > 2 else 40
    filt = sys.argv[3] if len(sys.argv) > 3 else ""
    c = sqlite3.connect(db)
    cols = [r[1] for r in c.execute("pragma table_info(kernels)")]
    name = "kernel_name" if "kernel_name" in cols else "name"
    rows = c.execute(f"select {name}, count(*), avg(end-start), min(end-start), sum(end-start) from kernels "
                     f"group by {name} order by sum(end-start) desc").fetchall()
    tot = sum(r[4] for r in rows) or 1
    print(f"{'kernel':70s} {'calls':>6s} {'avg_us':>9s} {'min_us':>9s} {'tot%':>6s}")
    for n, k, avg, mn, s in rows:
        if filt and filt not in n:
            continue
        print(f"{n[:70]:70s} {k:6d} {avg / 1e3:9.1f} {mn / 1e3:9.1f} {100 * s / tot:6.1f}")
        top -= 1
        if top == 0:
            break


if __name__ == "__main__":
    main()
