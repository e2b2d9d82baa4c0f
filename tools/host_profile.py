"""Host profile of the N=1 bench over the timed steps, every thread: a sampler thread records
each Python thread's current stack every 0.5 ms (sys._current_frames), and cProfile covers the
main thread.  Prints, per thread (main / autograd engine / PS thread / ...), the share of samples
by innermost Python function and by the bench / hipps call site, so host time per step can be
attributed -- the autograd engine's backward launches and hooks run on its own thread.

    python tools/host_profile.py [--out file.txt] [bench args...]
"""
import collections
import cProfile
import io
import os
import pstats
import sys
import threading
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


class Sampler(threading.Thread):
    def __init__(self, period=5e-4):
        super().__init__(daemon=True, name="host-sampler")
        self.period, self.on, self.stop = period, False, False
        self.leaf = collections.defaultdict(collections.Counter)
        self.site = collections.defaultdict(collections.Counter)
        self.n = collections.Counter()

    def run(self):
        me = threading.get_ident()
        names = {}
        while not self.stop:
            time.sleep(self.period)
            if not self.on:
                continue
            for t in threading.enumerate():
                names[t.ident] = t.name
            for tid, f in sys._current_frames().items():
                if tid == me:
                    continue
                tn = names.get(tid, str(tid))
                self.n[tn] += 1
                code = f.f_code
                self.leaf[tn][f"{os.path.basename(code.co_filename)}:{code.co_name}"] += 1
                g = f  # innermost frame inside hipps / bench / models
                while g is not None:
                    fn = g.f_code.co_filename
                    if "/hipps/" in fn or fn.endswith("bench.py"):
                        self.site[tn][f"{os.path.relpath(fn, os.path.dirname(os.path.dirname(__file__)))}:"
                                      f"{g.f_code.co_name}:{g.f_lineno}"] += 1
                        break
                    g = g.f_back


def main():
    args = sys.argv[1:]
    out = None
    if "--out" in args:
        i = args.index("--out")
        out = args[i + 1]
        del args[i:i + 2]
    import bench

    sys.argv = ["bench.py"] + args
    prof = cProfile.Profile()
    smp = Sampler()
    smp.start()

    def timed(on: bool):  # bench.TIMED_HOOKS: around the timed steps
        smp.on = on
        if on:
            prof.enable()
        else:
            prof.disable()

    bench.TIMED_HOOKS.append(timed)
    try:
        bench.main()
    finally:
        smp.on = False
        smp.stop = True
        smp.join(timeout=2)
    lines = []
    for tn, n in smp.n.most_common():
        lines.append(f"== thread {tn}: {n} samples")
        for k, v in smp.leaf[tn].most_common(12):
            lines.append(f"   leaf {100.0 * v / n:5.1f}%  {k}")
        for k, v in smp.site[tn].most_common(12):
            lines.append(f"   site {100.0 * v / n:5.1f}%  {k}")
    s = io.StringIO()
    pstats.Stats(prof, stream=s).sort_stats("tottime").print_stats(30)
    txt = "\n".join(lines) + "\n\n== main thread cProfile (tottime)\n" + s.getvalue()
    if out:
        open(out, "w").write(txt)
    print(txt[:6000])
    sys.stdout.flush()
    sys.stderr.flush()


if __name__ == "__main__":
    main()
    # skip interpreter teardown: a sampled run once ended in std::terminate there after all output
    # was written (torch's atexit handlers racing the sampler's frame walks)
    os._exit(0)
