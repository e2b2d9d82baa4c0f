"""Second-generation conv GEMM core (hipps/csrc/gemm2.hip) against the first core (gemm.hip,
itself checked against fp32 torch in test_conv1x1_gpu.py) and against fp32 torch directly.

Both cores accumulate each output over K in the same order (64-deep K tiles, two 16x16x32 MFMA
k-steps each), so the bf16 outputs must be bit-identical for every block tile; the statistics
partials are grouped by M tile (128 vs the gemm2 tile), so their sums agree to rounding.
"""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"
CL = torch.channels_last
TILES = [(128, 128), (256, 256), (256, 128), (128, 64), (256, 64)]


def C():
    from hipps.ops._native import native

    return native()


def _x(n, c, h, seed=0):
    g = torch.Generator(device="cpu").manual_seed(seed)
    return torch.randn(n, c, h, h, generator=g).to(DEV).to(torch.bfloat16).contiguous(memory_format=CL)


@pytest.mark.parametrize("bm,bn", TILES)
@pytest.mark.parametrize("cin,cout,stride", [(64, 256, 1), (256, 128, 1), (512, 256, 2)])
def test_gemm2_1x1_forward_stats_bitwise_first_core(bm, bn, cin, cout, stride):
    if cout % bn:
        pytest.skip("tile wider than Cout")
    n, h = 3, 13  # M tails: 3 * 13 * 13 = 507 rows (stride 2: 3 * 7 * 7)
    x = _x(n, cin, h)
    w = (torch.randn(cout, cin, device=DEV) / cin ** 0.5).to(torch.bfloat16)
    ho = (h - 1) // stride + 1
    M = n * ho * ho
    y1 = torch.empty(n, cout, ho, ho, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y2 = torch.full_like(y1, 7.0)
    p1 = torch.empty(2, cout, C().conv1x1_mtiles(M), device=DEV)
    p2 = torch.empty(2, cout, C().gemm2_mtiles(M, cout, cin, bm), device=DEV)
    C().conv1x1_forward(x, w, y1, p1, h, h, stride)
    C().gemm2_conv(x, w, y2, p2, None, None, h, h, stride, 1, 1, 0, bm, bn)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    torch.testing.assert_close(p2.sum(2), p1.sum(2), rtol=1e-5, atol=1e-3)
    ref = F.conv2d(x.float(), w.float().view(cout, cin, 1, 1), stride=stride)
    torch.testing.assert_close(y2.float(), ref, rtol=2e-2, atol=2e-2)
    # the statistics are those of the stored bf16 output
    yf = y2.float()
    torch.testing.assert_close(p2[0].sum(1), yf.sum((0, 2, 3)), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(p2[1].sum(1), (yf * yf).sum((0, 2, 3)), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("bm,bn", [(128, 128), (256, 256), (128, 64)])
@pytest.mark.parametrize("mode", ["add", "add_mask", "bst", "bst_bits", "bst_add"])
def test_gemm2_dgrad_epilogues_match_first_core(bm, bn, mode):
    n, h, cin, cout = 2, 15, 256, 256  # the dgrad GEMM: dy [M, cout] . wt [cin, cout]^T -> dx [M, cin]
    if cin % bn:
        pytest.skip("tile")
    dy = _x(n, cout, h, 1)
    wt = (torch.randn(cin, cout, device=DEV) / cout ** 0.5).to(torch.bfloat16)
    M = n * h * h
    add = _x(n, cin, h, 2) if "add" in mode else None
    amask = torch.randint(0, 256, (M * cin // 8,), dtype=torch.uint8, device=DEV) if mode == "add_mask" else None
    bx = bits = mean = inv = sc = sh = None
    if "bst" in mode:
        bx = _x(n, cin, h, 3)
        mean = torch.randn(cin, device=DEV) * 0.1
        inv = torch.rand(cin, device=DEV) + 0.5
        sc = torch.randn(cin, device=DEV)
        sh = torch.randn(cin, device=DEV) * 0.1
        if mode == "bst_bits":
            bits = torch.randint(0, 256, (M * cin // 8,), dtype=torch.uint8, device=DEV)
    y1 = torch.empty(n, cin, h, h, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y2 = torch.empty_like(y1)
    p1 = p2 = None
    if bx is not None:
        p1 = torch.empty(2, cin, C().conv1x1_mtiles(M), device=DEV)
        p2 = torch.empty(2, cin, C().gemm2_mtiles(M, cin, cout, bm), device=DEV)
    C().conv1x1_forward(dy, wt, y1, p1, h, h, 1, add, amask, bx, bits, mean, inv, sc, sh)
    C().gemm2_conv(dy, wt, y2, p2, add, amask, h, h, 1, 1, 1, 0, bm, bn, bx, bits, mean, inv, sc, sh)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    if p1 is not None:
        torch.testing.assert_close(p2.sum(2), p1.sum(2), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("bm,bn", TILES)
@pytest.mark.parametrize("cin,cout,h,stride", [(64, 128, 14, 1), (128, 128, 15, 2), (256, 256, 7, 1)])
def test_gemm2_3x3_implicit_gemm(bm, bn, cin, cout, h, stride):
    if cout % bn:
        pytest.skip("tile")
    n = 2
    x = _x(n, cin, h, 4)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) / (9 * cin) ** 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
    ho = (h + 2 - 3) // stride + 1
    M = n * ho * ho
    y1 = torch.empty(n, cout, ho, ho, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y2 = torch.full_like(y1, 3.0)
    p2 = torch.empty(2, cout, C().gemm2_mtiles(M, cout, 9 * cin, bm), device=DEV)
    C().convkxk_forward(x, w, y1, None, stride, 1)
    C().gemm2_conv(x, w, y2, p2, None, None, h, h, stride, 3, 3, 1, bm, bn)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)  # zero-page padding == the first core's masked loads
    ref = F.conv2d(x.float(), w.float(), stride=stride, padding=1)
    torch.testing.assert_close(y2.float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(p2[0].sum(1), y2.float().sum((0, 2, 3)), rtol=1e-4, atol=1e-2)


def test_tuner_picks_and_caches():
    from hipps.ops import nn as hnn

    x = _x(4, 256, 14)
    w = (torch.randn(512, 256, device=DEV) / 16).to(torch.bfloat16)
    y = torch.empty(4, 512, 14, 14, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    part = hnn._conv1x1_gemm(x, w, y, 14, 14, 1, True)
    keys = [k for k in hnn.TUNER.cache if k[:7] == ("1x1", 4 * 14 * 14, 256, 512, 1, 14, 14)]
    assert len(keys) == 1 and part.shape[:2] == (2, 512)
    ref = F.conv2d(x.float(), w.float().view(512, 256, 1, 1))
    torch.testing.assert_close(y.float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("cin,cout,k,h,stride", [(64, 256, 1, 14, 1), (256, 64, 1, 13, 1), (512, 256, 1, 15, 2),
                                                 (128, 128, 3, 14, 1), (256, 256, 3, 15, 2), (64, 64, 3, 9, 1)])
def test_gemm2_wgrad_bitwise_first_core(cin, cout, k, h, stride):
    """Same split-M slabs and per-slab accumulation order as gemm.hip's kernel: bit-identical."""
    n = 3
    pad = k // 2
    x = _x(n, cin, h, 5)
    ho = (h + 2 * pad - k) // stride + 1
    dy = _x(n, cout, ho, 6)
    if k == 1:
        d1 = torch.empty(cout, cin, device=DEV)
        d2 = torch.full_like(d1, 9.0)
        C().conv1x1_wgrad(dy, x, d1, h, h, stride)
    else:
        d1 = torch.empty(cout, cin, k, k, device=DEV).contiguous(memory_format=CL)
        d2 = torch.full_like(d1, 9.0)
        C().conv_wgrad(dy, x, d1, k, k, stride, pad)
    C().gemm2_wgrad(dy, x, d2, k, k, stride, pad, h, h)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), d1.view(cout, cin, k, k).float(), None,
                                              [stride, stride], [pad, pad], [1, 1], False, [0, 0], 1,
                                              [False, True, False])[1]
    torch.testing.assert_close(d2.view(cout, cin, k, k), ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("cfg", [1, 2])
@pytest.mark.parametrize("cin,cout,k,h,stride", [(256, 256, 1, 14, 1), (512, 512, 3, 7, 1), (256, 512, 3, 15, 2)])
def test_gemm2_wgrad_wide_tiles(cfg, cin, cout, k, h, stride):
    """256 x 128 / 256 x 256 output tiles (other slab split: fp32-close, not bitwise)."""
    if cfg == 2 and cin % 256:
        pytest.skip("tile")
    n = 2
    pad = k // 2
    x = _x(n, cin, h, 7)
    ho = (h + 2 * pad - k) // stride + 1
    dy = _x(n, cout, ho, 8)
    d0 = torch.empty(cout, cin, k, k, device=DEV).contiguous(memory_format=CL)
    d1 = torch.full_like(d0, 9.0)
    C().gemm2_wgrad(dy, x, d0, k, k, stride, pad, h, h, 0)
    C().gemm2_wgrad(dy, x, d1, k, k, stride, pad, h, h, cfg)
    torch.cuda.synchronize()
    torch.testing.assert_close(d1, d0, rtol=1e-5, atol=1e-4)


@pytest.mark.parametrize("bm,bn", [(128, 128), (256, 256), (128, 64)])
@pytest.mark.parametrize("bits", [False, True])
def test_gemm2_3x3_bn_backward_epilogue(bm, bn, bits):
    """Stride-1 3x3 input gradient run as a forward conv (rot180(W)^T) with the backward reduction
    of the BN whose output gradient it is in the epilogue (ResNet bn1 -> conv2): output equals the
    plain implicit GEMM bit for bit, partials equal fp32 torch sums of dz = dy * relu' and
    dz * x-hat on the stored bf16 dy."""
    n, h, cin, cout = 2, 13, 128, 256  # dgrad-as-forward: dy [n, cin, h, h] (*) wf [cout, cin, 3, 3]
    if cout % bn:
        pytest.skip("tile")
    dy = _x(n, cin, h, 11)
    wf = (torch.randn(cout, cin, 3, 3, device=DEV) / (9 * cin) ** 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
    M = n * h * h
    bx = _x(n, cout, h, 12)
    mean = torch.randn(cout, device=DEV) * 0.1
    inv = torch.rand(cout, device=DEV) + 0.5
    sc = torch.randn(cout, device=DEV)
    sh = torch.randn(cout, device=DEV) * 0.1
    mbits = torch.randint(0, 256, (M * cout // 8,), dtype=torch.uint8, device=DEV) if bits else None
    y0 = torch.empty(n, cout, h, h, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y1 = torch.full_like(y0, 5.0)
    C().gemm2_conv(dy, wf, y0, None, None, None, h, h, 1, 3, 3, 1, bm, bn)
    p = torch.empty(2, cout, C().gemm2_mtiles(M, cout, 9 * cin, bm), device=DEV)
    C().gemm2_conv(dy, wf, y1, p, None, None, h, h, 1, 3, 3, 1, bm, bn, bx, mbits, mean, inv, sc, sh)
    torch.cuda.synchronize()
    assert torch.equal(y0, y1)
    d = y1.permute(0, 2, 3, 1).reshape(M, cout).float()
    xv = bx.permute(0, 2, 3, 1).reshape(M, cout).float()
    if bits:
        on = ((mbits.view(-1, 1) >> torch.arange(8, device=DEV, dtype=torch.uint8)) & 1).view(M, cout).bool()
    else:
        on = xv * sc + sh > 0
    dz = torch.where(on, d, torch.zeros_like(d))
    torch.testing.assert_close(p[0].sum(1), dz.sum(0), rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(p[1].sum(1), (dz * (xv - mean) * inv).sum(0), rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize("bm,bn", [(256, 256), (256, 128), (128, 128), (128, 64), (256, 64)])
@pytest.mark.parametrize("kind", ["1x1", "1x1_k64", "1x1_k128", "3x3", "3x3_s2", "dgrad_bst_add"])
def test_gemm2_three_stage_pipeline_bitwise(bm, bn, kind):
    """3 LDS stages (one tile's DMA in flight across every barrier, counted vmcnt), the k-half
    units (stages=4: 32-deep units, two in flight) and the 256x256 ping-pong schedule (stages=5:
    two wave groups a phase apart) accumulate in the same order as the 2-stage loop: outputs and
    partials bit-identical, every K-tile count (1, 2, 3+ tiles: prologue / drain edges)."""
    n, h = 2, 11
    cin, cout, k, st = {"1x1": (320, 256, 1, 1), "1x1_k64": (64, 256, 1, 1), "1x1_k128": (128, 256, 1, 1),
                        "3x3": (128, 256, 3, 1), "3x3_s2": (64, 128, 3, 2), "dgrad_bst_add": (256, 256, 1, 1)}[kind]
    if cout % bn:
        pytest.skip("tile")
    x = _x(n, cin, h, 21)
    if k == 1:
        w = (torch.randn(cout, cin, device=DEV) / cin ** 0.5).to(torch.bfloat16)
    else:
        w = (torch.randn(cout, cin, k, k, device=DEV) / (k * k * cin) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=CL)
    pad = k // 2
    ho = (h + 2 * pad - k) // st + 1
    M = n * ho * ho
    extra = {}
    if kind == "dgrad_bst_add":
        extra = dict(add=_x(n, cout, ho, 22), bn_x=_x(n, cout, ho, 23), bn_mean=torch.randn(cout, device=DEV) * 0.1,
                     bn_invstd=torch.rand(cout, device=DEV) + 0.5, bn_scale=torch.randn(cout, device=DEV),
                     bn_shift=torch.randn(cout, device=DEV) * 0.1)
    outs = []
    for ns in ((2, 4, 5, 6) if (bm, bn) == (256, 256) else (2, 3, 4)):
        y = torch.full((n, cout, ho, ho), 3.0, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
        p = torch.empty(2, cout, C().gemm2_mtiles(M, cout, k * k * cin, bm), device=DEV)
        C().gemm2_conv(x, w, y, p, extra.get("add"), None, h, h, st, k, k, pad, bm, bn, extra.get("bn_x"), None,
                       extra.get("bn_mean"), extra.get("bn_invstd"), extra.get("bn_scale"), extra.get("bn_shift"),
                       stages=ns)
        outs.append((y, p))
    torch.cuda.synchronize()
    m32 = outs.pop() if (bm, bn) == (256, 256) else None  # stages 6: 32x32x16 MFMAs, another k order
    for o in outs[1:]:
        assert torch.equal(outs[0][0], o[0])
        assert torch.equal(outs[0][1], o[1])
    if m32 is not None:
        torch.testing.assert_close(m32[0].float(), outs[0][0].float(), rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(m32[1], outs[0][1], rtol=2e-2, atol=2e-1)
    if kind != "dgrad_bst_add":
        ref = F.conv2d(x.float(), w.float().view(cout, cin, k, k), stride=st, padding=pad)
        torch.testing.assert_close(outs[1][0].float(), ref, rtol=2e-2, atol=2e-2)


@pytest.mark.parametrize("M,K,N", [(1000, 512, 512), (4096, 2048, 768), (300, 64, 256)])
@pytest.mark.parametrize("bias", [False, True])
def test_gemm2_pingpong_linear_bitwise(M, K, N, bias):
    """The ping-pong 256x256 schedule (stages=5) on a Linear-shaped GEMM ([M, K] x [N, K]^T, several
    M tiles, masked tail rows, optional fp32 bias epilogue): bit-identical to the 2-stage loop and
    close to the fp32 reference."""
    if N % 256:
        pytest.skip("tile")
    g = torch.Generator(device=DEV).manual_seed(M + K)
    x = torch.randn(M, K, device=DEV, generator=g).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV, generator=g) / K ** 0.5).to(torch.bfloat16)
    b = torch.randn(N, device=DEV, generator=g) if bias else None
    outs = []
    for ns in (2, 5, 6):
        y = torch.full((M, N), 7.0, device=DEV, dtype=torch.bfloat16)
        C().gemm2_conv(x, w, y, None, None, None, 1, 1, 1, 1, 1, 0, 256, 256, stages=ns, bias=b)
        outs.append(y)
    torch.cuda.synchronize()
    assert torch.equal(outs[0], outs[1])
    ref = x.float() @ w.float().t() + (b if bias else 0.0)
    torch.testing.assert_close(outs[1].float(), ref, rtol=2e-2, atol=2e-2)
    torch.testing.assert_close(outs[2].float(), ref, rtol=2e-2, atol=2e-2)  # (32x32x16: another k order)


@pytest.mark.parametrize("cfg", [0, 1])
@pytest.mark.parametrize("cin,cout,k,h,stride", [(256, 256, 1, 14, 1), (128, 256, 3, 15, 2), (64, 64, 3, 9, 1)])
def test_gemm2_wgrad_three_stages_bitwise(cfg, cin, cout, k, h, stride):
    """3-stage weight gradient: same slabs and per-slab order as 2 stages -> bit-identical when the
    slab split matches (it can differ: 3 stages use more LDS, fewer resident blocks) else fp32-close."""
    if cfg == 1 and (cout % 256 or cin % 128):
        pytest.skip("tile")
    n = 2
    pad = k // 2
    x = _x(n, cin, h, 31)
    ho = (h + 2 * pad - k) // stride + 1
    dy = _x(n, cout, ho, 32)
    d2 = torch.empty(cout, cin, k, k, device=DEV).contiguous(memory_format=CL)
    d3 = torch.full_like(d2, 9.0)
    d4 = torch.full_like(d2, 9.0)
    C().gemm2_wgrad(dy, x, d2, k, k, stride, pad, h, h, cfg, 2)
    C().gemm2_wgrad(dy, x, d3, k, k, stride, pad, h, h, cfg, 3)
    C().gemm2_wgrad(dy, x, d4, k, k, stride, pad, h, h, cfg, 4)  # k-half units: same slabs, same order
    torch.cuda.synchronize()
    torch.testing.assert_close(d3, d2, rtol=1e-5, atol=1e-4)
    assert torch.equal(d4, d2)
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), d2.float(), None, [stride, stride], [pad, pad],
                                              [1, 1], False, [0, 0], 1, [False, True, False])[1]
    torch.testing.assert_close(d3, ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("bm,bn", [(128, 128), (256, 256), (128, 64)])
@pytest.mark.parametrize("h,bst", [(14, False), (13, True)])
def test_gemm2_add_s2_compact_stride2_gradient(bm, bn, h, bst):
    """conv1 dgrad + the downsample's compact stride-2 input gradient added on the even (h, w)
    rows (kAddS2), odd sizes included: equals the same GEMM with the zero-filled full-size addend."""
    n, cin, cout = 2, 256, 128  # dgrad: dy [M, cout] . wt [cin, cout]^T -> dx [M, cin]
    if cin % bn:
        pytest.skip("tile")
    dy = _x(n, cout, h, 41)
    wt = (torch.randn(cin, cout, device=DEV) / cout ** 0.5).to(torch.bfloat16)
    hs = (h + 1) // 2
    comp = _x(n, cin, hs, 42)
    full = torch.zeros(n, cin, h, h, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    full[:, :, ::2, ::2] = comp
    M = n * h * h
    extra = ()
    p1 = p2 = None
    if bst:
        bx = _x(n, cin, h, 43)
        bits = torch.randint(0, 256, (M * cin // 8,), dtype=torch.uint8, device=DEV)
        mean = torch.randn(cin, device=DEV) * 0.1
        inv = torch.rand(cin, device=DEV) + 0.5
        extra = (bx, bits, mean, inv, torch.ones_like(mean), torch.zeros_like(mean))
        p1 = torch.empty(2, cin, C().gemm2_mtiles(M, cin, cout, bm), device=DEV)
        p2 = torch.empty_like(p1)
    y1 = torch.empty(n, cin, h, h, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y2 = torch.full_like(y1, 7.0)
    C().gemm2_conv(dy, wt, y1, p1, full, None, h, h, 1, 1, 1, 0, bm, bn, *extra)
    C().gemm2_conv(dy, wt, y2, p2, comp, None, h, h, 1, 1, 1, 0, bm, bn, *extra, add_s2=True)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    if bst:
        assert torch.equal(p1, p2)


@pytest.mark.parametrize("cfg", [3, 4, 5, 6])
@pytest.mark.parametrize("ns", [2, 3, 4])
@pytest.mark.parametrize("cin,cout,k,h,stride", [(256, 256, 1, 14, 1), (256, 256, 3, 9, 1), (128, 256, 3, 15, 2),
                                                 (64, 64, 3, 13, 1), (64, 128, 3, 9, 2)])
def test_gemm2_wgrad_eight_wave_and_multitap(cfg, ns, cin, cout, k, h, stride):
    """8-wave 128x256 / 256x128 weight-gradient tiles (cfg 3 / 4) and the multi-tap tiles of the
    64-channel KxK layers (cfg 5 / 6: two taps per 128-wide tile, K padded) against fp32 torch."""
    ok = {3: cout % 128 == 0 and cin % 256 == 0, 4: cout % 256 == 0 and cin % 128 == 0,
          5: cin == 64 and k > 1, 6: cin == 64 and k > 1}
    if not ok[cfg]:
        pytest.skip("tile")
    n = 2
    pad = k // 2
    x = _x(n, cin, h, 51)
    ho = (h + 2 * pad - k) // stride + 1
    dy = _x(n, cout, ho, 52)
    d = torch.full((cout, cin, k, k), 9.0, device=DEV).contiguous(memory_format=CL)
    C().gemm2_wgrad(dy, x, d, k, k, stride, pad, h, h, cfg, ns)
    torch.cuda.synchronize()
    ref = torch.ops.aten.convolution_backward(dy.float(), x.float(), d.float(), None, [stride, stride], [pad, pad],
                                              [1, 1], False, [0, 0], 1, [False, True, False])[1]
    torch.testing.assert_close(d, ref, rtol=1e-3, atol=1e-2)


@pytest.mark.parametrize("bm,bn", [(128, 128), (256, 256), (128, 64), (256, 64)])
@pytest.mark.parametrize("cin,cout,h,bst", [(128, 128, 14, False), (256, 128, 15, True), (64, 64, 9, False),
                                            (128, 256, 8, True)])
def test_gemm2_dgrad_stride2_parity_classes(bm, bn, cin, cout, h, bst):
    """Stride-2 3x3 input gradient as four output-parity GEMMs (odd and even sizes) against fp32
    torch, and its BN-backward epilogue partials against fp32 sums."""
    if cin % bn:
        pytest.skip("tile")
    n = 2
    ho = (h - 1) // 2 + 1
    dy = _x(n, cout, ho, 61)
    w = (torch.randn(cout, cin, 3, 3, device=DEV) / (9 * cout) ** 0.5).to(torch.bfloat16).contiguous(memory_format=CL)
    wf = torch.flip(w, (2, 3)).transpose(0, 1).contiguous(memory_format=CL)
    dx = torch.full((n, cin, h, h), 7.0, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    extra = ()
    if bst:
        bx = _x(n, cin, h, 62)
        mean = torch.randn(cin, device=DEV) * 0.1
        inv = torch.rand(cin, device=DEV) + 0.5
        sc = torch.randn(cin, device=DEV)
        sh = torch.randn(cin, device=DEV) * 0.1
        extra = (bx, None, mean, inv, sc, sh)
    part = C().gemm2_dgrad_s2(dy, wf, dx, bm, bn, *extra)
    torch.cuda.synchronize()
    ref = torch.ops.aten.convolution_backward(dy.float(), torch.zeros(n, cin, h, h, device=DEV), w.float(), None,
                                              [2, 2], [1, 1], [1, 1], False, [0, 0], 1, [True, False, False])[0]
    torch.testing.assert_close(dx.float(), ref, rtol=2e-2, atol=2e-2)
    if bst:
        M = n * h * h
        d = dx.permute(0, 2, 3, 1).reshape(M, cin).float()
        xv = bx.permute(0, 2, 3, 1).reshape(M, cin).float()
        dz = torch.where(xv * sc + sh > 0, d, torch.zeros_like(d))
        torch.testing.assert_close(part[0].sum(1), dz.sum(0), rtol=1e-4, atol=1e-2)
        torch.testing.assert_close(part[1].sum(1), (dz * (xv - mean) * inv).sum(0), rtol=1e-4, atol=1e-2)


def _bn_apply_ref(x, sc, sh):
    """bf16(relu(x * sc + sh)) exactly as the fused BN apply kernel rounds it (channels-last)."""
    y = torch.empty_like(x)
    C().bn_apply(x, None, y, sc, sh, x.shape[1], True)
    return y


@pytest.mark.parametrize("bm,bn", [(128, 128), (256, 256), (128, 64), (256, 64)])
@pytest.mark.parametrize("cin,cout,k,h,stride", [(128, 256, 1, 13, 1), (64, 64, 3, 11, 1), (128, 128, 3, 15, 2),
                                                 (256, 256, 3, 7, 1)])
def test_gemm2_bn_prologue_bitwise(bm, bn, cin, cout, k, h, stride):
    """kPro: relu(x * scale + shift) applied to the staged A tiles in LDS gives the same output and
    statistics as the BN apply pass followed by the plain GEMM (padding taps stay zero)."""
    if cout % bn:
        pytest.skip("tile")
    n = 2
    x = _x(n, cin, h, 71)
    sc = torch.randn(cin, device=DEV)
    sh = torch.randn(cin, device=DEV) * 0.5
    if k == 1:
        w = (torch.randn(cout, cin, device=DEV) / cin ** 0.5).to(torch.bfloat16)
    else:
        w = (torch.randn(cout, cin, k, k, device=DEV) / (k * k * cin) ** 0.5).to(torch.bfloat16).contiguous(
            memory_format=CL)
    pad = k // 2
    ho = (h + 2 * pad - k) // stride + 1
    M = n * ho * ho
    y1 = torch.empty(n, cout, ho, ho, device=DEV, dtype=torch.bfloat16).contiguous(memory_format=CL)
    y2 = torch.full_like(y1, 3.0)
    p1 = torch.empty(2, cout, C().gemm2_mtiles(M, cout, k * k * cin, bm), device=DEV)
    p2 = torch.empty_like(p1)
    C().gemm2_conv(_bn_apply_ref(x, sc, sh), w, y1, p1, None, None, h, h, stride, k, k, pad, bm, bn)
    C().gemm2_conv(x, w, y2, p2, None, None, h, h, stride, k, k, pad, bm, bn, pro_scale=sc, pro_shift=sh)
    torch.cuda.synchronize()
    assert torch.equal(y1, y2)
    assert torch.equal(p1, p2)


@pytest.mark.parametrize("cfg", [0, 1, 3, 4, 5, 6])
@pytest.mark.parametrize("cin,cout,k,h,stride", [(128, 256, 1, 13, 1), (64, 64, 3, 11, 1), (128, 256, 3, 15, 2),
                                                 (256, 256, 3, 7, 1)])
def test_gemm2_wgrad_bn_prologue_bitwise(cfg, cin, cout, k, h, stride):
    """Weight gradient with the BN + ReLU applied to the X tiles in LDS == apply pass + plain kernel."""
    ok = {0: True, 1: cout % 256 == 0 and cin % 128 == 0, 3: cout % 128 == 0 and cin % 256 == 0,
          4: cout % 256 == 0 and cin % 128 == 0, 5: cin == 64 and k > 1, 6: cin == 64 and k > 1}
    if not ok[cfg]:
        pytest.skip("tile")
    n = 2
    pad = k // 2
    x = _x(n, cin, h, 72)
    sc = torch.randn(cin, device=DEV)
    sh = torch.randn(cin, device=DEV) * 0.5
    ho = (h + 2 * pad - k) // stride + 1
    dy = _x(n, cout, ho, 73)
    d1 = torch.empty(cout, cin, k, k, device=DEV).contiguous(memory_format=CL)
    d2 = torch.full_like(d1, 9.0)
    C().gemm2_wgrad(dy, _bn_apply_ref(x, sc, sh), d1, k, k, stride, pad, h, h, cfg, 2)
    C().gemm2_wgrad(dy, x, d2, k, k, stride, pad, h, h, cfg, 2, sc, sh)
    torch.cuda.synchronize()
    assert torch.equal(d1, d2)


@pytest.mark.parametrize("cfg", [0, 2])
@pytest.mark.parametrize("cin,cout,k,h,stride", [(256, 256, 1, 28, 1), (256, 256, 3, 14, 2)])
def test_gemm2_wgrad_fewer_slabs(cfg, cin, cout, k, h, stride):
    """sdiv=2 (half as many, twice as long M slabs) == the default split to fp32 rounding."""
    n = 8
    pad = k // 2
    x = _x(n, cin, h, 81)
    ho = (h + 2 * pad - k) // stride + 1
    dy = _x(n, cout, ho, 82)
    d1 = torch.empty(cout, cin, k, k, device=DEV).contiguous(memory_format=CL)
    d2 = torch.full_like(d1, 9.0)
    C().gemm2_wgrad(dy, x, d1, k, k, stride, pad, h, h, cfg, 2)
    C().gemm2_wgrad(dy, x, d2, k, k, stride, pad, h, h, cfg, 2, sdiv=2)
    torch.cuda.synchronize()
    torch.testing.assert_close(d2, d1, rtol=1e-5, atol=1e-4)
