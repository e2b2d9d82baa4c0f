"""Summarize a rocprofv3 kernel trace to steady-state per-step costs.

Steps are delimited by a marker kernel that runs once per optimizer step (default: the async PS
pull-select kernel, once per worker step; k_sgd runs once per bucket update); the first `--skip` steps (warmup incl. MIOpen find) are dropped.
    python tools/steady_profile.py trace.csv out.txt [--marker k_sgd] [--skip 5]
"""
import argparse
import collections
import csv


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("trace")
    ap.add_argument("out")
    ap.add_argument("--marker", default="k_pull_select")
    ap.add_argument("--skip", type=int, default=5)
    ap.add_argument("--title", default="")
    ap.add_argument("--detail", default=None,
                    help="regex: list every call of the matching kernels in the last steady step (grid, us)")
    a = ap.parse_args()
    rows = list(csv.DictReader(open(a.trace)))
    rows.sort(key=lambda r: int(r["Start_Timestamp"]))
    marks = [int(r["Start_Timestamp"]) for r in rows if a.marker in r["Kernel_Name"]]
    if len(marks) < a.skip + 2:
        raise SystemExit(f"only {len(marks)} marker kernels")
    t0, t1 = marks[a.skip], marks[-1]
    n = len(marks) - 1 - a.skip
    steady = [r for r in rows if t0 <= int(r["Start_Timestamp"]) < t1]
    agg = collections.defaultdict(lambda: [0, 0])
    for r in steady:
        agg[r["Kernel_Name"]][0] += int(r["End_Timestamp"]) - int(r["Start_Timestamp"])
        agg[r["Kernel_Name"]][1] += 1
    tot = sum(v[0] for v in agg.values())
    cat = collections.defaultdict(float)
    for k, (d, c) in agg.items():
        if "hipps" in k:
            key = ("hipps-norm" if "k_bn_" in k else
                   "hipps-gemm" if ("conv1x1" in k or "wgrad" in k or "stem" in k or "k_gemm" in k) else "hipps-ps")
        elif "BatchNorm" in k:
            key = "miopen-batchnorm"
        elif any(s in k for s in ("conv", "igemm", "gemm", "Cijk", "xdl")):
            key = "conv/gemm"
        elif "elementwise" in k or "Functor" in k:
            key = "elementwise"
        else:
            key = "other"
        cat[key] += d
    lines = [a.title, f"steady steps={n} wall/step={(t1 - t0) / n / 1e6:.2f} ms kernel-sum/step={tot / n / 1e6:.2f} ms "
                      f"launches/step={len(steady) / n:.0f}"]
    for k, v in sorted(cat.items(), key=lambda x: -x[1]):
        lines.append(f"  {k:18s} {v / n / 1e6:8.3f} ms/step {100 * v / tot:5.1f}%")
    # GPU idle time: the wall time no kernel covers (side-stream kernels overlap, so the kernel
    # sum can exceed the wall), and the longest idle gaps with the kernel that ended before them
    busy, cur_s, cur_e, gaps = 0, None, None, collections.defaultdict(lambda: [0, 0])
    prev = ""
    for r in steady:
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if cur_e is None or st > cur_e:
            if cur_e is not None:
                busy += cur_e - cur_s
                g = gaps[prev[:60] + " -> " + r["Kernel_Name"][:60]]
                g[0] += st - cur_e
                g[1] += 1
            cur_s, cur_e = st, en
        else:
            cur_e = max(cur_e, en)
        if en >= cur_e:
            prev = r["Kernel_Name"]
    if cur_e is not None:
        busy += min(cur_e, t1) - cur_s
    lines.append(f"GPU busy/step={busy / n / 1e6:.2f} ms idle/step={((t1 - t0) - busy) / n / 1e6:.2f} ms")
    for k, (d, c) in sorted(gaps.items(), key=lambda x: -x[1][0])[:12]:
        lines.append(f"  idle {d / n / 1e3:7.1f} us/step gaps/step={c / n:5.1f}  {k}")
    # one steady step's idle gaps >= 40 us in context (stream / queue ids when the trace has them)
    sid = next((c for c in ("Stream_Id", "Queue_Id") if c in rows[0]), None)
    m0, m1 = marks[a.skip + n // 2], marks[a.skip + n // 2 + 1]
    one = [r for r in rows if m0 <= int(r["Start_Timestamp"]) < m1]
    lines.append(f"step timeline gaps (step {a.skip + n // 2}, {len(one)} kernels, t=0 at its marker):")
    end = None
    for j, r in enumerate(one):
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if end is not None and st - end >= 40000:
            for q in one[max(0, j - 2):j + 2]:
                lines.append(f"    t={(int(q['Start_Timestamp']) - m0) / 1e3:9.1f} us dur={(int(q['End_Timestamp']) - int(q['Start_Timestamp'])) / 1e3:7.1f}"
                             f" {('s' + str(q[sid])) if sid else ''} {q['Kernel_Name'][:70]}")
            lines.append(f"  ^ idle {(st - end) / 1e3:.1f} us")
        end = en if end is None else max(end, en)
    big, end = 0, None  # the long stalls (>= 200 us) anywhere in the steady steps, in context
    for j, r in enumerate(steady):
        st, en = int(r["Start_Timestamp"]), int(r["End_Timestamp"])
        if end is not None and st - end >= 200000 and big < 4:
            big += 1
            lines.append(f"stall {(st - end) / 1e3:.1f} us:")
            for q in steady[max(0, j - 6):j + 3]:
                lines.append(f"    t={(int(q['Start_Timestamp']) - t0) / 1e3:10.1f} us dur={(int(q['End_Timestamp']) - int(q['Start_Timestamp'])) / 1e3:7.1f}"
                             f" {('s' + str(q[sid])) if sid else ''} {q['Kernel_Name'][:70]}")
        end = en if end is None else max(end, en)
    lines.append("")
    for k, (d, c) in sorted(agg.items(), key=lambda x: -x[1][0])[:60]:
        lines.append(f"{d / n / 1e3:9.1f} us/step calls/step={c / n:6.1f}  {k[:140]}")
    if a.detail:
        import re

        pat = re.compile(a.detail)
        last = [r for r in rows if marks[-2] <= int(r["Start_Timestamp"]) < marks[-1]]
        gkey = next((k for k in ("Grid_Size_X", "Grid_Size", "grid_size_x") if rows and k in rows[0]), None)
        lines.append("")
        lines.append(f"calls of /{a.detail}/ in the last steady step (start us, grid, us):")
        for r in last:
            if pat.search(r["Kernel_Name"]):
                st = (int(r["Start_Timestamp"]) - marks[-2]) / 1e3
                du = (int(r["End_Timestamp"]) - int(r["Start_Timestamp"])) / 1e3
                lines.append(f"  {st:9.1f} {('s' + str(r[sid])) if sid else ''} grid={r.get(gkey, '?') if gkey else '?':>9} "
                             f"{du:8.1f}  {r['Kernel_Name'][:90]}")
    open(a.out, "w").write("\n".join(lines) + "\n")
    print("\n".join(lines[:24]))


if __name__ == "__main__":
    main()
