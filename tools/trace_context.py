"""Print the kernels around each occurrence of a name pattern in one steady-state step of a
rocprofv3 kernel trace (CSV), to find which framework op launched an unexpected kernel.
Usage: python tools/trace_context.py <kernel_trace.csv> <pattern> [<pattern> ...] [--step N]"""
import csv
import sys


def main():
    args = [a for a in sys.argv[1:]]
    step = 6
    if "--step" in args:
        i = args.index("--step")
        step = int(args[i + 1])
        del args[i:i + 2]
    path, pats = args[0], args[1:]
    rows = sorted(csv.DictReader(open(path)), key=lambda r: int(r["Start_Timestamp"]))
    names = [r["Kernel_Name"] for r in rows]
    marks = [i for i, n in enumerate(names) if "k_sgd" in n]
    if len(marks) <= step:
        print("not enough steps")
        return
    lo, hi = marks[step - 1] + 1, marks[step] + 1
    for i in range(lo, hi):
        if any(p in names[i] for p in pats):
            print(f"--- #{i - lo} {names[i][:110]}  ({(int(rows[i]['End_Timestamp']) - int(rows[i]['Start_Timestamp'])) / 1e3:.1f} us)")
            for j in range(max(lo, i - 4), min(hi, i + 5)):
                print(f"   {'>' if j == i else ' '} {names[j][:120]}")


if __name__ == "__main__":
    main()
