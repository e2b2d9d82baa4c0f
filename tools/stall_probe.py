"""For each long GPU idle gap in a rocprofv3 kernel trace, show when the host LAUNCHED the kernel
that ended it (hip API trace, matched by correlation id) and the host API calls around the gap:
a launch after the gap began means the host was late; a launch before it means the GPU waited
on a dependency.
    python tools/stall_probe.py kernel_trace.csv hip_api_trace.csv out.txt [--min-us 300]"""
import argparse
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("ktrace")
    ap.add_argument("htrace")
    ap.add_argument("out")
    ap.add_argument("--min-us", type=float, default=300)
    ap.add_argument("--skip", type=int, default=5)
    a = ap.parse_args()
    ks = sorted(csv.DictReader(open(a.ktrace)), key=lambda r: int(r["Start_Timestamp"]))
    hs = sorted(csv.DictReader(open(a.htrace)), key=lambda r: int(r["Start_Timestamp"]))
    by_corr = {r["Correlation_Id"]: r for r in hs}
    marks = [int(r["Start_Timestamp"]) for r in ks if "k_pull_select" in r["Kernel_Name"]]
    t0 = marks[a.skip] if len(marks) > a.skip else int(ks[0]["Start_Timestamp"])
    lines, end, n = [], None, 0
    for r in ks:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if st < t0:
            end = en if end is None else max(end, en)
            continue
        if end is not None and st - end >= a.min_us * 1e3 and n < 10:
            n += 1
            h = by_corr.get(r["Correlation_Id"])
            lines.append(f"gap {(st - end) / 1e3:.1f} us before {r['Kernel_Name'][:80]}")
            if h is not None:
                lines.append(f"  its launch {h['Function']} (thread {h['Thread_Id']}) at {(int(h['Start_Timestamp']) - end) / 1e3:+.1f} us "
                             f"from the gap start, returned {(int(h['End_Timestamp']) - end) / 1e3:+.1f} us")
            for q in hs:
                qs, qe = int(q["Start_Timestamp"]), int(q["End_Timestamp"])
                if qe >= end - 100000 and qs <= st and qe - qs >= 20000:
                    lines.append(f"    host {q['Function'][:40]:40s} thread {q['Thread_Id']} {(qs - end) / 1e3:+9.1f} .. {(qe - end) / 1e3:+9.1f} us")
            # what every thread did last before the gap began (which thread launched the work the
            # GPU just finished, and how long before)
            lastb = {}
            for q in hs:
                qs = int(q["Start_Timestamp"])
                if end - 20_000_000 <= qs <= end:
                    lastb[q["Thread_Id"]] = q
            for tid, q in sorted(lastb.items()):
                lines.append(f"    before: thread {tid} last {q['Function'][:36]} at {(int(q['Start_Timestamp']) - end) / 1e3:+9.1f} us")
            # every HIP call of every thread inside the gap: per thread, the calls (count, time in
            # them) and the longest stretches with NO call (the thread ran Python / held or waited
            # for the GIL)
            per = {}
            for q in hs:
                qs, qe = int(q["Start_Timestamp"]), int(q["End_Timestamp"])
                if qe >= end and qs <= st:
                    per.setdefault(q["Thread_Id"], []).append((qs, qe, q["Function"]))
            for tid, calls in sorted(per.items()):
                calls.sort()
                busy = sum(min(qe, st) - max(qs, end) for qs, qe, _ in calls) / 1e3
                holes, prev = [], end
                for qs, qe, fn in calls:
                    if qs > prev:
                        holes.append(((qs - prev) / 1e3, (prev - end) / 1e3, fn))
                    prev = max(prev, qe)
                if st > prev:
                    holes.append(((st - prev) / 1e3, (prev - end) / 1e3, "<gap end>"))
                holes.sort(reverse=True)
                names = {}
                for _, _, fn in calls:
                    names[fn] = names.get(fn, 0) + 1
                top = ", ".join(f"{k} x{v}" for k, v in sorted(names.items(), key=lambda kv: -kv[1])[:6])
                lines.append(f"    thread {tid}: {len(calls)} HIP calls, {busy:.1f} us inside them ({top})")
                for dur, at, fn in holes[:3]:
                    lines.append(f"      no HIP call for {dur:7.1f} us from {at:+8.1f} us (next: {fn[:40]})")
        end = en if end is None else max(end, en)
    # host lead: for every kernel, GPU start minus the end of its launch call on the host -- how
    # far ahead of the GPU the launching thread was.  Small values for most kernels mean the host
    # (not the GPU) sets the pace; report percentiles per phase of the step
    leads = []
    for r in ks:
        st = int(r["Start_Timestamp"])
        if st < t0:
            continue
        h = by_corr.get(r["Correlation_Id"])
        if h is None:
            continue
        leads.append(((st - int(h["End_Timestamp"])) / 1e3, r["Kernel_Name"][:60]))
    if leads:
        v = sorted(x for x, _ in leads)
        pct = lambda q: v[min(len(v) - 1, int(q * len(v)))]  # noqa: E731
        lines.append(f"host lead (GPU start - launch return, us) over {len(v)} kernels: p5 {pct(0.05):.0f} "
                     f"p25 {pct(0.25):.0f} p50 {pct(0.5):.0f} p75 {pct(0.75):.0f} p95 {pct(0.95):.0f}")
        firsts = [x for x, nm in leads if "bfloat16_copy" in nm]
        if firsts:
            lines.append("host lead at the input casts (step starts), us: " + " ".join(f"{x:.0f}" for x in firsts[:20]))
    open(a.out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:80]))


if __name__ == "__main__":
    main()
