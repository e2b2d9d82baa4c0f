"""GPU numerics: every hipps HIP kernel vs the fp32 PyTorch reference of the same op.

Runs only on an MI355X (marker ``gpu``).  The native extension must be the code path under
test: the first test asserts ``hipps._C`` is loaded (no silent eager fallback).
"""
import pytest
import torch

from hipps import codecs, ops
from hipps.ops import _native
from hipps.ops import reference as ref

pytestmark = pytest.mark.gpu
DEV = "cuda"
SIZES = [1, 7, 1000, 4099, 1 << 20]


def test_native_extension_loaded():
    assert _native.available(), "hipps._C must be built and importable on the GPU box"
    import sys

    assert "hipps._C" in sys.modules


@pytest.mark.parametrize("n", SIZES)
@pytest.mark.parametrize("W", [1, 3, 8])
@pytest.mark.parametrize("dt", [torch.float32, torch.bfloat16])
def test_aggregate(n, W, dt):
    torch.manual_seed(n + W)
    slots = [torch.randn(n).to(dt) for _ in range(W)]
    want = torch.randn(n)
    got = want.clone().to(DEV)
    ref.aggregate(slots, want, 0.25, accumulate=True)
    ops.aggregate([s.to(DEV) for s in slots], got, 0.25, accumulate=True)
    torch.testing.assert_close(got.cpu(), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n", SIZES)
def test_convert_bf16_roundtrip_bitexact(n):
    x = torch.randn(n) * 10
    x[:1] = float("nan") if n > 3 else x[:1]
    y = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    ops.convert(x.to(DEV), y)
    want = x.to(torch.bfloat16)
    assert torch.equal(y.cpu().view(torch.int16)[~want.isnan()], want.view(torch.int16)[~want.isnan()])
    assert y.cpu().isnan().sum() == want.isnan().sum()
    z = torch.empty(n, device=DEV)
    ops.convert(y, z, 2.0)
    torch.testing.assert_close(z.cpu(), want.float() * 2, equal_nan=True)


@pytest.mark.parametrize("n", [5, 4096, 100003])
@pytest.mark.parametrize("mom,damp,nesterov,wd", [(0, 0, False, 0), (0.9, 0, False, 1e-4), (0.9, 0.1, True, 1e-4)])
@pytest.mark.parametrize("W,dt", [(1, torch.float32), (4, torch.bfloat16)])
def test_sgd_fused(n, mom, damp, nesterov, wd, W, dt):
    torch.manual_seed(n)
    p = torch.randn(n)
    buf = torch.zeros(n)
    pd, bd = p.to(DEV), buf.to(DEV)
    pub = torch.empty(n, dtype=torch.bfloat16, device=DEV)
    for t in range(3):
        grads = [torch.randn(n).to(dt) for _ in range(W)]
        kw = dict(lr=0.05, weight_decay=wd, momentum=mom, dampening=damp, nesterov=nesterov, first=(t == 0))
        ref.sgd_step(grads, p, buf if mom else None, None, False, 0.5, **kw)
        ops.sgd_step([g.to(DEV) for g in grads], pd, bd if mom else None, pub, False, 0.5, **kw)
    torch.testing.assert_close(pd.cpu(), p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(pub.cpu().float(), p.to(torch.bfloat16).float(), rtol=1e-2, atol=1e-2)
    if mom:
        torch.testing.assert_close(bd.cpu(), buf, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("masked", [False, True])
def test_sgd_zero_src(masked):
    """The async PS clears its accumulator in the update pass: the update must still use it."""
    n = 4099
    g = torch.randn(n, device=DEV)
    p = torch.randn(n, device=DEV)
    want, gc = p.cpu().clone(), g.cpu().clone()
    mask = torch.ones((n + 15) // 16, dtype=torch.uint8) if masked else None
    if masked:
        mask[::3] = 0
    ref.sgd_step([gc], want, None, None, True, 1.0, lr=0.1, weight_decay=0.01, mask=mask)
    ops.sgd_step([g], p, None, None, True, 1.0, lr=0.1, weight_decay=0.01, mask=None if mask is None else mask.to(DEV))
    assert g.abs().sum().item() == 0
    torch.testing.assert_close(p.cpu(), want, rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n", [3, 4096, 65537])
@pytest.mark.parametrize("amsgrad,torch_mode,wd", [(False, False, 0.0), (True, False, 1e-2), (False, True, 0.0)])
def test_adam_fused(n, amsgrad, torch_mode, wd):
    torch.manual_seed(n + 1)
    p, m, v, vm = torch.randn(n), torch.zeros(n), torch.zeros(n), torch.zeros(n)
    pd, md, vd, vmd = p.to(DEV), m.to(DEV), v.to(DEV), vm.to(DEV)
    for t in range(1, 4):
        g = torch.randn(n)
        kw = dict(lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=wd, step=t, amsgrad=amsgrad,
                  torch_mode=torch_mode)
        ref.adam_step([g], p, m, v, vm if amsgrad else None, None, False, 1.0, **kw)
        ops.adam_step([g.to(DEV)], pd, md, vd, vmd if amsgrad else None, None, False, 1.0, **kw)
    torch.testing.assert_close(pd.cpu(), p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(vd.cpu(), v, rtol=1e-5, atol=1e-7)


@pytest.mark.parametrize("opt", ["sgd", "adam"])
@pytest.mark.parametrize("n", [16 * 37 + 5, 1 << 18])
def test_masked_update_skips_chunks(opt, n):
    """Chunks (16 elements) whose mask byte is 0 keep p / state bit-exactly; publish gets p."""
    torch.manual_seed(3)
    nch = (n + 15) // 16
    mask = (torch.rand(nch) > 0.3).to(torch.uint8)
    p = torch.randn(n)
    p0 = p.clone()
    st = [torch.randn(n) * 0.1, torch.rand(n) * 0.1, torch.rand(n) * 0.1]
    g = torch.randn(n)
    pd, sd = p.to(DEV), [s.to(DEV) for s in st]
    s0 = [s.clone() for s in sd]
    pub = torch.empty(n, dtype=torch.float32, device=DEV)
    if opt == "sgd":
        kw = dict(lr=0.1, weight_decay=0.1, momentum=0.9)
        ref.sgd_step([g], p, st[0], None, False, 1.0, mask=mask, **kw)
        ops.sgd_step([g.to(DEV)], pd, sd[0], pub, False, 1.0, mask=mask.to(DEV), **kw)
    else:
        kw = dict(lr=1e-2, weight_decay=0.1, step=3, amsgrad=True)
        ref.adam_step([g], p, st[0], st[1], st[2], None, False, 1.0, mask=mask, **kw)
        ops.adam_step([g.to(DEV)], pd, sd[0], sd[1], sd[2], pub, False, 1.0, mask=mask.to(DEV), **kw)
    keep = ~mask.bool().repeat_interleave(16)[:n]
    assert torch.equal(pd.cpu()[keep], p0[keep])
    assert not torch.equal(pd.cpu()[~keep], p0[~keep])
    for a_, b_ in zip(sd, s0):
        assert torch.equal(a_.cpu()[keep], b_.cpu()[keep])
    torch.testing.assert_close(pd.cpu(), p, rtol=1e-5, atol=1e-6)
    assert torch.equal(pub.cpu(), pd.cpu())


@pytest.mark.parametrize("n", [1, 255, 256, 1000, 1 << 20, 9_000_001])
@pytest.mark.parametrize("ef,sr", [(False, False), (True, False), (False, True)])
def test_q8_encode_matches_reference(n, ef, sr):
    torch.manual_seed(n)
    x = torch.randn(n) * 3
    nb = (n + 255) // 256
    q, s = torch.empty(n, dtype=torch.int8), torch.empty(nb)
    r = torch.randn(n) * 0.01 if ef else None
    rd = r.to(DEV) if ef else None
    qd, sd = torch.empty(n, dtype=torch.int8, device=DEV), torch.empty(nb, device=DEV)
    ref.q8_encode(x, r, q, s, sr, 99)
    ops.q8_encode(x.to(DEV), rd, qd, sd, sr, 99)
    torch.testing.assert_close(sd.cpu(), s, rtol=1e-6, atol=0)
    mism = (qd.cpu().int() - q.int()).abs()
    assert mism.max() <= 1 and (mism > 0).float().mean() < 1e-3  # rint tie / fma corner cases only
    if ef:
        torch.testing.assert_close(rd.cpu(), r, rtol=0, atol=float(s.max()) * 1.01)
    acc = torch.zeros(n, device=DEV)
    ops.q8_aggregate([qd, qd], [sd, sd], acc, 0.5)
    torch.testing.assert_close(acc.cpu(), ref.q8_dequant(qd.cpu(), sd.cpu()), rtol=1e-6, atol=1e-6)


@pytest.mark.parametrize("n,k", [(10, 3), (1000, 10), (4099, 41), (1 << 20, 10486), (3_000_001, 30001)])
@pytest.mark.parametrize("vdt", [torch.float32, torch.bfloat16])
def test_topk_exact(n, k, vdt):
    torch.manual_seed(n)
    x = torch.randn(n)
    x[: n // 10] = x[0]  # force many ties at some magnitude
    idx, val = torch.empty(k, dtype=torch.int32), torch.empty(k, dtype=vdt)
    ref.topk_encode(x, None, k, idx, val)
    idd, vd = torch.empty(k, dtype=torch.int32, device=DEV), torch.empty(k, dtype=vdt, device=DEV)
    ops.topk_encode(x.to(DEV), None, k, idd, vd)
    assert torch.equal(idd.cpu(), idx)
    assert torch.equal(vd.cpu(), val)
    acc = torch.zeros(n, device=DEV)
    ops.topk_accumulate(idd, vd, acc, 2.0)
    want = torch.zeros(n)
    want[idx.long()] = val.float() * 2
    torch.testing.assert_close(acc.cpu(), want)


@pytest.mark.parametrize("case", ["mostly_zero", "all_equal", "two_levels"])
def test_topk_candidate_overflow_and_ties(case):
    """Threshold bins holding more elements than the candidate list (n/16): the candidate passes
    fall back to the whole bucket and ties are still admitted lowest-index-first."""
    n, k = 1 << 20, 20000
    torch.manual_seed(7)
    if case == "mostly_zero":
        x = torch.zeros(n)
        x[torch.randperm(n)[:5000]] = torch.randn(5000)
    elif case == "all_equal":
        x = torch.full((n,), -0.25)
    else:
        x = torch.where(torch.rand(n) < 0.5, torch.tensor(1.5), torch.tensor(-0.75))
    idx, val = torch.empty(k, dtype=torch.int32), torch.empty(k)
    ref.topk_encode(x, None, k, idx, val)
    idd, vd = torch.empty(k, dtype=torch.int32, device=DEV), torch.empty(k, device=DEV)
    ops.topk_encode(x.to(DEV), None, k, idd, vd)
    assert torch.equal(idd.cpu(), idx)
    assert torch.equal(vd.cpu(), val)


@pytest.mark.parametrize("vdt", [torch.float32, torch.bfloat16])
def test_topk_repeated_calls_speculative_list(vdt):
    """One workspace across calls, as a codec keeps it per bucket: call 1 has no previous threshold
    (P1 lists nothing, the repair pass lists bin B and up); later calls list from 0.95 x the
    previous threshold (the single-pass path); a 10x smaller gradient drops the threshold below that bound (every region
    repairs); a skewed bucket overflows a few regions' slots (shared pool); an all-equal bucket
    exhausts the pool (full-pass mode).  Every call must equal the CPU reference bit for bit,
    error-feedback residual included."""
    n, k = 3_000_001, 30001
    torch.manual_seed(3)
    ws = torch.zeros(ops.topk_workspace_bytes(n, k), dtype=torch.uint8, device=DEV)
    r_cpu, r_dev = torch.zeros(n), torch.zeros(n, device=DEV)
    gens = [lambda: torch.randn(n), lambda: torch.randn(n), lambda: torch.randn(n) * 1.3,
            lambda: torch.randn(n) * 0.1, lambda: torch.randn(n) * 0.1]

    def skew():
        x = torch.randn(n) * 0.01
        x[1_000_000:1_200_000] = torch.randn(200_000) * 10  # one layer with large gradients
        return x

    gens += [skew, skew, lambda: torch.full((n,), 0.5), lambda: torch.randn(n)]
    for step, gen in enumerate(gens):
        g = gen()
        idx, val = torch.empty(k, dtype=torch.int32), torch.empty(k, dtype=vdt)
        ref.topk_encode(g, r_cpu, k, idx, val)
        idd, vd = torch.empty(k, dtype=torch.int32, device=DEV), torch.empty(k, dtype=vdt, device=DEV)
        ops.topk_encode(g.to(DEV), r_dev, k, idd, vd, ws)
        assert torch.equal(idd.cpu(), idx), step
        assert torch.equal(vd.cpu(), val), step
        assert torch.equal(r_dev.cpu(), r_cpu), step


def test_topk_error_feedback_conserves_mass():
    n, k = 100_000, 1000
    g = torch.randn(n, device=DEV)
    r = torch.randn(n, device=DEV) * 0.1
    total = g + r
    idx = torch.empty(k, dtype=torch.int32, device=DEV)
    val = torch.empty(k, device=DEV)
    ops.topk_encode(g, r, k, idx, val)
    acc = torch.zeros(n, device=DEV)
    ops.topk_accumulate(idx, val, acc)
    torch.testing.assert_close(acc + r, total, rtol=0, atol=1e-6)


@pytest.mark.parametrize("spec", ["fp32", "bf16", "int8", "int8_sr", "topk:0.01", "topk_bf16:0.05", "topk_int8:0.02"])
def test_codec_gpu_matches_cpu(spec):
    torch.manual_seed(0)
    n = 50_000
    x = torch.randn(n)
    outs = []
    for dev in ("cpu", DEV):
        c = codecs.get_codec(spec)
        lay = c.layout(n)
        buf = torch.empty(lay.nbytes, dtype=torch.uint8, device=dev)
        st = c.init_state(n, dev)
        c.encode_into(x.to(dev), lay.views(buf), st)
        acc = torch.zeros(n, device=dev)
        c.accumulate([lay.views(buf)], acc)
        outs.append(acc.cpu())
    tol = 1e-6 if spec in ("fp32", "topk:0.01") else (2e-2 if "int8" in spec else 1e-2)
    torch.testing.assert_close(outs[1], outs[0], rtol=tol, atol=tol)


@pytest.mark.parametrize("n,tau,ratio", [(1000, 1.0, 0.5), (1 << 20, 2.0, 0.01), (1 << 20, 3.0, 0.5), (4099, 0.0, 0.1)])
@pytest.mark.parametrize("ef", [False, True])
def test_threshold_codec_gpu_matches_reference(n, tau, ratio, ef):
    from hipps.codecs import Threshold

    torch.manual_seed(n)
    x = torch.randn(n)
    outs = []
    for dev in ("cpu", DEV):
        c = Threshold(tau=tau, max_ratio=ratio, error_feedback=ef)
        lay = c.layout(n)
        buf = torch.zeros(lay.nbytes, dtype=torch.uint8, device=dev)
        v = lay.views(buf)
        st = c.init_state(n, dev)
        c.encode_into(x.to(dev), v, st)
        acc = torch.zeros(n, device=dev)
        c.accumulate([v], acc, 1.0, True)
        k = int(v["count"][0])
        outs.append((k, v["idx"][:k].cpu(), acc.cpu(), st["resid"].cpu() if ef else None))
    assert outs[0][0] == outs[1][0]
    assert torch.equal(outs[0][1], outs[1][1])
    torch.testing.assert_close(outs[1][2], outs[0][2])
    if ef:
        torch.testing.assert_close(outs[1][3], outs[0][3])


@pytest.mark.parametrize("opt", ["sgd", "adam"])
def test_chunk_steps_per_parameter_state(opt):
    """Per-chunk update counts (csteps): a chunk's first momentum step is buf = d_p and Adam's bias
    correction uses the chunk's own t, whatever the group step; counts advance under the mask."""
    torch.manual_seed(5)
    n = 16 * 4001
    nch = n // 16
    cs = torch.randint(0, 4, (nch,), dtype=torch.int32)
    p, st = torch.randn(n), [torch.randn(n) * 0.1, torch.rand(n) * 0.1]
    pd, sd, csd = p.to(DEV), [s.to(DEV) for s in st], cs.to(DEV)
    for t in range(3):
        mask = (torch.rand(nch) > 0.25).to(torch.uint8)
        g = torch.randn(n)
        if opt == "sgd":
            kw = dict(lr=0.1, weight_decay=0.01, momentum=0.9, dampening=0.3)
            ref.sgd_step([g], p, st[0], None, False, 1.0, mask=mask, csteps=cs, **kw)
            ops.sgd_step([g.to(DEV)], pd, sd[0], None, False, 1.0, mask=mask.to(DEV), csteps=csd, **kw)
        else:
            kw = dict(lr=1e-2, betas=(0.9, 0.999), eps=1e-8, weight_decay=0.01, step=t + 2)
            ref.adam_step([g], p, st[0], st[1], None, None, False, 1.0, mask=mask, csteps=cs, **kw)
            ops.adam_step([g.to(DEV)], pd, sd[0], sd[1], None, None, False, 1.0, mask=mask.to(DEV), csteps=csd, **kw)
    assert torch.equal(csd.cpu(), cs)
    torch.testing.assert_close(pd.cpu(), p, rtol=1e-5, atol=1e-6)
    torch.testing.assert_close(sd[0].cpu(), st[0], rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("masked", [False, True])
def test_sgd_lookahead_publish(masked):
    """Look-ahead publish: pub = p_new - c * buf_new (masked chunks: p - c * buf); master unchanged."""
    torch.manual_seed(6)
    n = 16 * 999
    p, buf = torch.randn(n), torch.randn(n) * 0.1
    g = torch.randn(n)
    mask = (torch.rand(n // 16) > 0.5).to(torch.uint8) if masked else None
    pd, bd = p.to(DEV), buf.to(DEV)
    pub = torch.empty(n, device=DEV)
    kw = dict(lr=0.1, weight_decay=1e-4, momentum=0.9)
    ref.sgd_step([g], p, buf, None, False, 1.0, mask=mask, **kw)
    ops.sgd_step([g.to(DEV)], pd, bd, pub, False, 1.0, mask=None if mask is None else mask.to(DEV), lookahead=0.09,
                 **kw)
    torch.testing.assert_close(pd.cpu(), p, rtol=1e-6, atol=1e-6)
    torch.testing.assert_close(pub.cpu(), p - 0.09 * buf, rtol=1e-5, atol=1e-6)


@pytest.mark.parametrize("n,k", [(1, 1), (10, 10), (17, 5), (10_000, 100), (32768, 3277), (32769, 3277)])
@pytest.mark.parametrize("vdt", [torch.float32, torch.bfloat16])
@pytest.mark.parametrize("case", ["randn", "ties", "zeros"])
def test_topk_small_single_workgroup(n, k, vdt, case):
    """n <= 32768 runs the one-launch LDS radix select (topk.hip k_topk_small): indices, values
    and the error-feedback residual equal the CPU reference bit for bit (32769 = the multi-pass
    path, same contract)."""
    torch.manual_seed(n + k)
    g = torch.randn(n) if case != "zeros" else torch.zeros(n)
    if case == "ties":
        g[::3] = 0.5
        g[1::7] = -0.5
    r0 = torch.randn(n) * 0.01 if case != "zeros" else torch.zeros(n)
    r_cpu, r_dev = r0.clone(), r0.to(DEV)
    idx, val = torch.empty(k, dtype=torch.int32), torch.empty(k, dtype=vdt)
    ref.topk_encode(g, r_cpu, k, idx, val)
    idd, vd = torch.empty(k, dtype=torch.int32, device=DEV), torch.empty(k, dtype=vdt, device=DEV)
    ops.topk_encode(g.to(DEV), r_dev, k, idd, vd)
    assert torch.equal(idd.cpu(), idx)
    assert torch.equal(vd.cpu(), val)
    assert torch.equal(r_dev.cpu(), r_cpu)


@pytest.mark.parametrize("n,k", [(32768, 328), (10_000, 100), (32768, 2900), (5000, 4000)])
@pytest.mark.parametrize("vdt", [torch.float32, torch.bfloat16])
def test_topk_small_repeated_calls_speculative_list(n, k, vdt):
    """One workspace across calls on the single-workgroup path: call 1 runs the full digit passes
    and leaves its threshold; later calls walk the short list of keys >= 0.95 x that threshold; a
    10x smaller gradient (too few listed keys), an all-equal bucket (more than the list holds) and
    ties fall back to the full passes.  Every call equals the CPU reference bit for bit."""
    torch.manual_seed(n + k)
    ws = torch.zeros(ops.topk_workspace_bytes(n, k), dtype=torch.uint8, device=DEV)
    r_cpu, r_dev = torch.zeros(n), torch.zeros(n, device=DEV)

    def ties():
        x = torch.randn(n)
        x[::3] = 2.0
        return x

    gens = [lambda: torch.randn(n), lambda: torch.randn(n), lambda: torch.randn(n) * 1.3,
            lambda: torch.randn(n) * 0.1, lambda: torch.randn(n) * 0.1, ties, lambda: torch.full((n,), 0.5),
            lambda: torch.randn(n), lambda: torch.randn(n)]
    for step, gen in enumerate(gens):
        g = gen()
        idx, val = torch.empty(k, dtype=torch.int32), torch.empty(k, dtype=vdt)
        ref.topk_encode(g, r_cpu, k, idx, val)
        idd, vd = torch.empty(k, dtype=torch.int32, device=DEV), torch.empty(k, dtype=vdt, device=DEV)
        ops.topk_encode(g.to(DEV), r_dev, k, idd, vd, ws)
        assert torch.equal(idd.cpu(), idx), step
        assert torch.equal(vd.cpu(), val), step
        assert torch.equal(r_dev.cpu(), r_cpu), step


@pytest.mark.parametrize("spec", ["fp32", "bf16", "int8", "topk:0.05", "topk_int8:0.05", "threshold:0.5:0.2"])
def test_codec_accumulate_acquire_path_matches(spec):
    """The PS's acquire path for peer-written mailbox slots (system-scope acquire in every
    workgroup before the first load, csrc/common.h) computes exactly what the plain path does."""
    n = 70001
    torch.manual_seed(3)
    c = codecs.get_codec(spec)
    lay = c.layout(n)
    msgs = []
    for w in range(3):
        buf = torch.zeros(lay.nbytes, dtype=torch.uint8, device=DEV)
        v = lay.views(buf)
        c.encode_into(torch.randn(n, device=DEV), v, c.init_state(n, torch.device(DEV)))
        msgs.append(v)
    base = torch.randn(n, device=DEV)
    a, b = base.clone(), base.clone()
    c.accumulate(msgs, a, 0.5, True)
    c.accumulate(msgs, b, 0.5, True, acquire=True)
    assert torch.equal(a, b)


@pytest.mark.parametrize("n", [1, 15, 16, 4097, 1 << 20])
def test_copy_acquire(n):
    src = torch.randint(0, 256, (n,), dtype=torch.uint8, device=DEV)
    dst = torch.zeros(n, dtype=torch.uint8, device=DEV)
    ops.copy_acquire(src, dst)
    assert torch.equal(src, dst)


@pytest.mark.parametrize("codec", ["dense_f32", "dense_bf16", "int8"])
def test_ps_accumulate_is_batch_invariant(codec):
    """The async PS adds arriving messages in launches of whatever arrived together: the result
    must not depend on that batching (one launch of [a, b, c] == [a] then [b, c], bitwise), and it
    matches the reference's per-message sequence."""
    torch.manual_seed(7)
    n = 5000
    acc0 = torch.randn(n, device=DEV)
    if codec == "int8":
        msgs = []
        for _ in range(3):
            x = torch.randn(n, device=DEV)
            q = torch.empty(n, dtype=torch.int8, device=DEV)
            s = torch.empty((n + 255) // 256, device=DEV)
            ops.q8_encode(x, None, q, s, False, 0)
            msgs.append((q, s))

        def add(ms, acc):
            ops.q8_aggregate([m[0] for m in ms], [m[1] for m in ms], acc, 1 / 3, True)
        want = acc0.cpu().clone()
        ref.q8_aggregate([m[0].cpu() for m in msgs], [m[1].cpu() for m in msgs], want, 1 / 3, True)
    else:
        dt = torch.float32 if codec == "dense_f32" else torch.bfloat16
        msgs = [torch.randn(n, device=DEV).to(dt) for _ in range(3)]

        def add(ms, acc):
            ops.aggregate(ms, acc, 1 / 3, True)
        want = acc0.cpu().clone()
        ref.aggregate([m.cpu() for m in msgs], want, 1 / 3, True)
    one = acc0.clone()
    add(msgs, one)
    two = acc0.clone()
    add(msgs[:1], two)
    add(msgs[1:], two)
    three = acc0.clone()
    for m in msgs:
        add([m], three)
    assert torch.equal(one, two) and torch.equal(one, three)
    # (the CPU reference scales by the Python double 1/3; the kernel by its float rounding)
    torch.testing.assert_close(one.cpu(), want, rtol=1e-6, atol=1e-6)
