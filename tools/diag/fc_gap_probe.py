"""Where does the host spend the ~200 us before the ResNet fc backward GEMM (the largest idle gap
of the steady table, profiles/r5/final/steady.txt)?  Runs the N=1 bench with host timestamps at
loss.backward(), the cross-entropy backward, and the fc (_ShadowLinear) backward entry / after its
first GEMM launch, plus a GPU event at each, over the timed steps.  Prints per-interval means of
host time and of GPU time between the same points (GPU ~ host: the host is the bound there).

    python tools/diag/fc_gap_probe.py [bench args...]
"""
import collections
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__)))))


def main():
    import torch

    import bench
    import hipps.ops.nn as hnn

    sys.argv = ["bench.py"] + sys.argv[1:]
    on = [False]
    marks = []  # per step: list of (name, host t, event)

    def mark(name):
        if not on[0]:
            return
        ev = torch.cuda.Event(enable_timing=True)
        ev.record()
        marks[-1].append((name, time.perf_counter(), ev))

    orig_bwd = torch.Tensor.backward

    def backward(self, *a, **k):
        mark("backward() called")
        r = orig_bwd(self, *a, **k)
        mark("backward() returned")
        return r

    import hipps.optim as hopt

    zg, ost = hopt.MPI_PS.zero_grad, hopt.MPI_PS.step

    def zero_grad(self, *a, **k):
        if on[0]:
            marks.append([])
        mark("zero_grad (step start)")
        return zg(self, *a, **k)

    def opt_step(self, *a, **k):
        mark("opt.step entry")
        r = ost(self, *a, **k)
        mark("opt.step exit")
        return r

    hopt.MPI_PS.zero_grad = zero_grad
    hopt.MPI_PS.step = opt_step

    torch.Tensor.backward = backward
    xb = hnn._CrossEntropy.backward
    lb = hnn._ShadowLinear.backward

    def xent_bwd(ctx, *g):
        mark("xent backward entry")
        r = xb(ctx, *g)
        mark("xent backward exit")
        return r

    def lin_bwd(ctx, dy):  # hnn._ShadowLinear.backward with a mark after each statement
        mark("fc backward entry")
        x2, w_master = ctx.saved_tensors
        dy2 = dy.reshape(-1, dy.shape[-1])
        if dy2.dtype != torch.bfloat16:
            dy2 = dy2.to(torch.bfloat16)
        mark("fc saved tensors")
        wb = hnn.bf16_weight(w_master, idle=False)
        mark("fc bf16_weight")
        dx = torch.mm(dy2, wb).view(ctx.xshape)
        if dx.dtype != ctx.xdtype:
            dx = dx.to(ctx.xdtype)
        mark("fc dx mm")
        dw = hnn._linear_wgrad(dy2, x2)
        mark("fc dw mm")
        db = hnn.colsum_f32(dy2) if ctx.has_bias and ctx.needs_input_grad[2] else None
        mark("fc colsum")
        return dx, dw, db, None

    hnn._CrossEntropy.backward = staticmethod(xent_bwd)
    hnn._ShadowLinear.backward = staticmethod(lin_bwd)

    def timed(flag):
        on[0] = flag

    bench.TIMED_HOOKS.append(timed)
    import threading

    bench.TIMED_HOOKS.append(lambda f: f and print("threads:", [t.name for t in threading.enumerate()], flush=True))
    bench.main()
    torch.cuda.synchronize()
    host = collections.defaultdict(list)
    gpu = collections.defaultdict(list)
    for st in marks[:-1]:
        for (n0, t0, e0), (n1, t1, e1) in zip(st, st[1:]):
            key = f"{n0} -> {n1}"
            host[key].append((t1 - t0) * 1e6)
            gpu[key].append(e0.elapsed_time(e1) * 1e3)
    print(f"{len(marks)} steps")
    for key in host:
        h, g = host[key], gpu[key]
        print(f"  {key:50s} host {sum(h) / len(h):8.1f} us   gpu {sum(g) / len(g):8.1f} us")
    sys.stdout.flush()


if __name__ == "__main__":
    main()
    os._exit(0)
