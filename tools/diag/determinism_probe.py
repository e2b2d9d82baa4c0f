"""Which kernel makes two runs of the joined default differ on the tiny ResNet of
tests/test_ps_async_gpu.py::_resnet_defer?  Runs it three times in one process (the first only
warms the tuner) per environment variant and prints the largest parameter difference between runs
2 and 3 (0.0 = bitwise run-to-run deterministic).  TORCH_DET=1 runs under hipps.set_deterministic.

    python tools/diag/determinism_probe.py "" HIPPS_DGRAD_S2=1 TORCH_DET=1
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "tests"))


def _probe(rank, world, torch_det):
    from test_ps_async_gpu import _resnet_defer

    _resnet_defer(rank, world, False, False, torch_det)
    b = _resnet_defer(rank, world, False, False, torch_det)
    c = _resnet_defer(rank, world, False, False, torch_det)
    diffs = [float((y - z).abs().max()) for y, z in zip(b["params"], c["params"])]
    return {"max": max(diffs), "n_diff": sum(d > 0 for d in diffs), "n": len(diffs)}


def main():
    from dist_util import run_world

    for variant in sys.argv[1:] or [""]:
        saved = dict(os.environ)
        det = False
        for kv in variant.split(","):
            if not kv:
                continue
            k, v = kv.split("=", 1)
            if k == "TORCH_DET":
                det = v == "1"
            else:
                os.environ[k] = v
        r = run_world(_probe, 1, det)[0]
        print(f"variant [{variant or 'default'}]: max param diff {r['max']:.3g}, "
              f"{r['n_diff']}/{r['n']} tensors differ", flush=True)
        os.environ.clear()
        os.environ.update(saved)


if __name__ == "__main__":
    main()
