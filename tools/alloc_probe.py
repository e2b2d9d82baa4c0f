"""Which device allocations does the N=1 bench still make in steady state?  Snapshots the PyTorch
caching allocator's segments right before and right after the timed steps (bench.TIMED_HOOKS) and
prints the segments created in between, grouped by stream and size, plus the allocator counters.
Every new segment is a hipMalloc on the host path of some step.

    python tools/alloc_probe.py [--out file.txt] [bench args...]
"""
import collections
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    args = sys.argv[1:]
    out = None
    if "--out" in args:
        i = args.index("--out")
        out = args[i + 1]
        del args[i:i + 2]
    import torch

    import bench

    sys.argv = ["bench.py"] + args
    snaps = {}

    def timed(on: bool):
        torch.cuda.synchronize()
        snaps["on" if on else "off"] = (torch.cuda.memory_snapshot(), torch.cuda.memory_stats())

    bench.TIMED_HOOKS.append(timed)
    bench.main()
    (s0, m0), (s1, m1) = snaps["on"], snaps["off"]
    before = {seg["address"] for seg in s0}
    new = [seg for seg in s1 if seg["address"] not in before]
    groups = collections.Counter((seg.get("stream", 0), seg["segment_type"], seg["total_size"]) for seg in new)
    lines = [f"segments before {len(s0)} after {len(s1)} new {len(new)} "
             f"({sum(seg['total_size'] for seg in new) / 2**20:.1f} MiB)"]
    for k in ("num_device_alloc", "num_device_free", "num_alloc_retries", "num_sync_all_streams"):
        lines.append(f"  {k}: +{m1.get(k, 0) - m0.get(k, 0)}")
    lines.append("new segments by (stream, pool, size):")
    for (st, ty, sz), n in groups.most_common(40):
        lines.append(f"  stream {st:#x} {ty:5s} {sz / 2**20:9.2f} MiB x {n}")
    # what lives in the new segments now (active blocks: the allocation sizes that needed them)
    act = collections.Counter()
    for seg in new:
        for b in seg.get("blocks", []):
            if b.get("state") == "active_allocated":
                act[(seg.get("stream", 0), b["size"])] += 1
    lines.append("active blocks in the new segments by (stream, size):")
    for (st, sz), n in act.most_common(40):
        lines.append(f"  stream {st:#x} {sz / 2**20:9.3f} MiB x {n}")
    txt = "\n".join(lines)
    print(txt)
    if out:
        with open(out, "w") as f:
            f.write(txt + "\n")
    sys.stdout.flush()
    os._exit(0)


if __name__ == "__main__":
    main()
