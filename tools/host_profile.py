"""cProfile of the N=1 bench's host side (main thread) over the timed steps: which Python
functions take the host time per step.  The autograd engine thread and the PS thread are not
covered (cProfile follows one thread); their HIP calls are in the stall probe's API trace.

    python tools/host_profile.py [--out file.txt] [bench args...]
"""
import cProfile
import io
import os
import pstats
import sys

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main():
    args = sys.argv[1:]
    out = None
    if "--out" in args:
        i = args.index("--out")
        out = args[i + 1]
        del args[i:i + 2]
    import bench
    from hipps.parallel import dist as hdist

    sys.argv = ["bench.py"] + args
    prof = cProfile.Profile()
    orig_barrier = hdist.barrier
    calls = [0]

    def barrier(world):  # bench: barrier -> timed steps -> barrier
        r = orig_barrier(world)
        calls[0] += 1
        if calls[0] == 1:
            prof.enable()
        elif calls[0] == 2:
            prof.disable()
        return r

    hdist.barrier = barrier
    try:
        bench.main()
    finally:
        hdist.barrier = orig_barrier
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(40)
    s2 = io.StringIO()
    pstats.Stats(prof, stream=s2).sort_stats("cumulative").print_stats(40)
    txt = s.getvalue() + "\n\n" + s2.getvalue()
    if out:
        open(out, "w").write(txt)
    print(txt[:5000])


if __name__ == "__main__":
    main()
