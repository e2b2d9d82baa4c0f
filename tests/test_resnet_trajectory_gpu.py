"""ResNet-50 trains: 40 steps on one fixed 224x224 batch of 64 (lr 0.1, momentum 0.9).

* hipps fused path (MFMA 1x1 convs with BN epilogues, fused BN/ReLU/residual kernels, hipps
  wgrad/dgrad, HIP max pool, fused SGD kernel) vs plain PyTorch (every fusion off, MIOpen
  convs, eager BN, torch.optim.SGD): per-step losses agree within 3 % -- or within three times
  the run-to-run spread of plain PyTorch itself at that step (MIOpen's default kernels use
  atomics; two identical plain runs already differ by ~1 % once the loss is below ~0.6; floor
  0.01 nats) -- for every step while the loss is above 0.1, at least 15 steps within 2 %, and
  both fall;
* ps_async at N=1 with max_delay=0 (rank 0 = PS + worker) is bit-identical to mode='local'
  (8 steps with MIOpen's deterministic algorithms: its default ones use atomics);
* free-running ps_async (GPU-time pull, one update of staleness per step) still trains the batch
  down, more slowly than local SGD (delayed gradients with momentum 0.9: 6.95 -> ~3.8 in 40
  steps where local SGD reaches ~0.1).

The fusion switches are read at import, so each side runs in a fresh child process.
"""
import json
import os
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _run(args, out, timeout=420):
    cmd = [sys.executable, "-u", os.path.join(ROOT, "tools", "trajectory.py"), "--out", out] + args
    r = subprocess.run(cmd, cwd=ROOT, timeout=timeout, capture_output=True, text=True)
    assert r.returncode == 0, r.stderr[-4000:]
    with open(out) as f:
        return {rec["variant"]: rec for rec in json.load(f)}


def test_resnet50_fused_trains_like_plain_pytorch(tmp_path):
    fused = _run(["--runs", "local,async"], str(tmp_path / "fused.json"))
    plain = _run(["--plain"], str(tmp_path / "plain.json"))["plain"]
    plain2 = _run(["--plain"], str(tmp_path / "plain2.json"))["plain"]
    det = _run(["--runs", "local,async_md0", "--steps", "8", "--deterministic"], str(tmp_path / "det.json"))
    a, b, b2 = fused["local"]["losses"], plain["losses"], plain2["losses"]
    assert len(a) == len(b) == 40
    checked = strict = 0
    for i, (u, v, v2) in enumerate(zip(a, b, b2)):
        if v < 0.1:
            break
        # one fused and one plain sample against one plain-vs-plain spread: 3 % or 3x that spread,
        # and never less than 0.01 nats (near the 0.1 cut-off 3 % is 0.003)
        tol = max(0.03 * v, 3 * abs(v2 - v), 0.01)
        assert abs(u - v) <= tol, f"step {i}: fused {u:.4f} vs plain {v:.4f} / {v2:.4f}"
        checked += 1
        strict += abs(u - v) <= 0.02 * v
    assert checked >= 20 and strict >= 15
    assert a[-1] < 0.5 * a[0] and b[-1] < 0.5 * b[0]
    # N=1 async PS with max_delay=0 applies exactly the local update sequence
    assert det["async_md0"]["param_sha"] == det["local"]["param_sha"]
    assert det["async_md0"]["losses"] == det["local"]["losses"]
    # free-running AsySG-InCon: staleness bounded by the pipeline, and the loss still falls
    fr = fused["async"]
    assert fr["ps"]["doorbells"] == "device" and fr["ps"]["pull"] == "device"
    lf = fr["losses"]
    assert min(lf[-5:]) < 0.6 * lf[0]
    assert sum(lf[-5:]) < sum(lf[15:20])  # still falling at the end
