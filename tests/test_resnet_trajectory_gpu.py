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
* the headline bench configuration (batch 256, bf16 wire, bf16 weight shadow, lr 0.1, momentum
  0.9, 60 steps): free-running ps_async running the reference's AsySG-InCon (plain read of the
  published parameters, GPU-time pull, one update of staleness per step) with the default
  per-bucket versions falls below half its first loss, never climbs more than 10 % above its
  running minimum after step 20, and ends at least as low as whole-model versions do (those
  oscillate around 4.3-5.3 under momentum 0.9: profiles/r4/traj_headline.json); the look-ahead
  publish (delay compensation, opt-in) converges too; max_delay=0 stays bit-identical to local.

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
    # the child's per-step progress goes to our stderr (visible with pytest -s: these runs take
    # minutes), and to a log whose tail is the failure message
    log = out + ".log"
    with open(log, "w") as f:
        p = subprocess.Popen(cmd, cwd=ROOT, stdout=subprocess.DEVNULL, stderr=subprocess.PIPE, text=True)
        try:
            for line in p.stderr:
                f.write(line)
                sys.stderr.write(line)
            p.wait(timeout=timeout)
        finally:
            if p.poll() is None:
                p.kill()
    with open(log) as f:
        assert p.returncode == 0, f.read()[-4000:]
    with open(out) as f:
        return {rec["variant"]: rec for rec in json.load(f)}


def test_resnet50_fused_trains_like_plain_pytorch(tmp_path):
    fused = _run(["--runs", "local"], str(tmp_path / "fused.json"))
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


def test_headline_config_async_converges(tmp_path):
    h = _run(["--headline", "--runs", "local,async,async_model,async_la"], str(tmp_path / "headline.json"),
             timeout=600)
    det = _run(["--headline", "--runs", "local,async_md0", "--steps", "6", "--deterministic"],
               str(tmp_path / "hdet.json"))
    assert det["async_md0"]["param_sha"] == det["local"]["param_sha"]
    assert det["async_md0"]["losses"] == det["local"]["losses"]
    fr = h["async"]
    assert fr["batch"] == 256 and fr["codec"] == "bf16" and fr["bf16_weights"] == "auto"
    assert fr["ps"]["doorbells"] == "device" and fr["ps"]["pull"] == "device"
    assert fr["ps"]["granularity"] == "bucket" and fr["ps"]["lookahead_tau_x1000"] == 0  # plain InCon
    lf = fr["losses"]
    assert len(lf) == 60 and lf[-1] < 0.5 * lf[0], lf
    for i in range(20, len(lf)):
        assert lf[i] <= 1.1 * min(lf[: i + 1]), f"step {i}: {lf[i]:.3f} rebounds above {min(lf[: i + 1]):.3f}"
    # per-bucket versions converge at least as well as whole-model versions
    lm = h["async_model"]["losses"]
    assert h["async_model"]["ps"]["granularity"] == "model"
    assert sum(lf[-20:]) <= sum(lm[-20:]), (lf[-20:], lm[-20:])
    la = h["async_la"]
    assert la["ps"]["lookahead_tau_x1000"] > 0 and la["losses"][-1] < 0.5 * la["losses"][0]
    # per-step staleness in the step data: one update at N=1
    assert fr["staleness"] and max(fr["staleness"][5:]) <= 2
    assert h["local"]["losses"][-1] < 0.2 * h["local"]["losses"][0]
