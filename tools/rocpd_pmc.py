"""Per-kernel counter summary from rocprofv3 --pmc databases (rocpd SQLite): for each kernel the
mean counter value per dispatch and, for byte counters (FETCH_SIZE / WRITE_SIZE, in KB), the rate
against the dispatch's duration.  Usage: python tools/rocpd_pmc.py <db> [<db> ...] [--filter S]"""
import sqlite3
import sys


def short(name):
    n = name.replace("(anonymous namespace)::", "").split("(")[0]
    return n.replace("void ", "")[:60]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--")]
    filt = ""
    if "--filter" in sys.argv:
        filt = sys.argv[sys.argv.index("--filter") + 1]
        args.remove(filt)
    rows = {}
    for db in args:
        c = sqlite3.connect(db)
        for name, cname, val, dur in c.execute("select name, counter_name, counter_value, duration from pmc_events"):
            if filt and filt not in name:
                continue
            r = rows.setdefault((short(name), cname), [0, 0.0, 0.0])
            r[0] += 1
            r[1] += val
            r[2] += dur
    print(f"{'kernel':60s} {'counter':11s} {'calls':>5s} {'mean':>12s} {'dur_us':>8s} {'GB/s':>8s}")
    for (k, cn), (cnt, v, d) in sorted(rows.items()):
        mean, dur = v / cnt, d / cnt
        rate = (mean * 1024 / dur) if cn.endswith("_SIZE") and dur else float("nan")
        print(f"{k:60s} {cn:11s} {cnt:5d} {mean:12.1f} {dur / 1e3:8.1f} {rate:8.1f}")


if __name__ == "__main__":
    main()
