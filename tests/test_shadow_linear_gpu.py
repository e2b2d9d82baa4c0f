"""hipps.ops.nn.Linear / linear on the bf16 weight shadow (_ShadowLinear) against F.linear under
bf16 autocast, the transformer models on it, and weight sharing on the weight-gradient side
stream (a weight used twice in one graph)."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

DEV = "cuda"


def _shadowed(*shapes):
    """fp32 parameters as views of one flat buffer with a registered bf16 shadow."""
    from hipps.ops import nn as hnn

    n = sum(torch.Size(s).numel() for s in shapes)
    flat = torch.randn(n, device=DEV) * 0.05
    shadow = flat.to(torch.bfloat16)
    hnn.register_weight_shadow(flat, shadow)
    out, o = [], 0
    for s in shapes:
        k = torch.Size(s).numel()
        out.append(torch.nn.Parameter(flat[o:o + k].view(s)))
        o += k
    return flat, shadow, out


def test_shadow_linear_matches_autocast_linear():
    from hipps.ops import nn as hnn

    torch.manual_seed(0)
    flat, shadow, (w, b) = _shadowed((96, 64), (96,))
    try:
        x = torch.randn(4, 33, 64, device=DEV, requires_grad=True)
        x0 = x.detach().clone().requires_grad_(True)
        w0 = torch.nn.Parameter(w.detach().clone())
        b0 = torch.nn.Parameter(b.detach().clone())
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert hnn.shadow_linear_ok(x, w, b)
            y = hnn.linear(x, w, b)
            y0 = F.linear(x0, w0, b0)
        assert y.dtype == torch.bfloat16 and y.shape == y0.shape
        torch.testing.assert_close(y.float(), y0.float(), rtol=1e-2, atol=1e-2)
        g = torch.randn_like(y)
        y.backward(g)
        y0.backward(g)
        assert w.grad.dtype == torch.float32 and x.grad.dtype == torch.float32
        torch.testing.assert_close(x.grad, x0.grad, rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(w.grad, w0.grad, rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(b.grad, b0.grad, rtol=2e-2, atol=2e-2)
        # fp32 reference of the same op
        ref = torch.nn.functional.linear(x0.detach().double(), w0.detach().double(), b0.detach().double())
        torch.testing.assert_close(y.double(), ref, rtol=3e-2, atol=3e-2)
    finally:
        hnn.unregister_weight_shadow(shadow)


def test_shadow_linear_tied_weight_used_twice():
    """A weight used twice in one forward (tied decoder): both contributions summed exactly once."""
    from hipps.ops import nn as hnn

    torch.manual_seed(1)
    flat, shadow, (w,) = _shadowed((80, 48))
    try:
        x = torch.randn(16, 48, device=DEV)
        w0 = torch.nn.Parameter(w.detach().clone())
        with torch.autocast("cuda", dtype=torch.bfloat16):
            h = hnn.linear(x, w)             # [16, 80]
            y = hnn.linear(h[:, :48], w)
            h0 = F.linear(x, w0)
            y0 = F.linear(h0[:, :48], w0)
        y.float().sum().backward()
        y0.float().sum().backward()
        torch.testing.assert_close(w.grad, w0.grad, rtol=3e-2, atol=3e-2)
    finally:
        hnn.unregister_weight_shadow(shadow)


def test_conv_weight_shared_twice_on_side_stream():
    """The same hipps 3x3 conv applied twice in one graph: its two weight-gradient contributions
    (both on the side stream) are summed by autograd on the caller's stream only after both
    finished -- bit-identical to the same kernels run in line (side stream off)."""
    from hipps.ops import nn as hnn

    def run(side):
        saved = hnn._WGRAD_SIDE
        hnn._WGRAD_SIDE = side
        try:
            torch.manual_seed(2)
            conv = torch.nn.Conv2d(64, 64, 3, padding=1, bias=False).cuda().to(memory_format=torch.channels_last)
            x = torch.randn(8, 64, 14, 14, device=DEV).to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
            with torch.autocast("cuda", dtype=torch.bfloat16):
                y = hnn.conv2d(conv, hnn.conv2d(conv, x, fuse=True), fuse=True)
            y.backward(torch.randn(y.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3)).to(y.dtype))
            torch.cuda.synchronize()
            return conv.weight.grad.clone()
        finally:
            hnn._WGRAD_SIDE = saved

    a, b = run(True), run(False)
    assert torch.isfinite(a).all()
    assert torch.equal(a, b)


@pytest.mark.parametrize("name", ["bert-tiny", "llama-tiny"])
def test_transformer_steps_shadow_linear_vs_autocast(name):
    """Four steps of the tiny transformers with the bf16 shadow on: the Linear layers on
    _ShadowLinear track plain autocast F.linear (the dW precision differs: fp32 from the GEMM vs
    a bf16 dW cast up), and the loss goes down."""
    import hipps
    from hipps.models.transformer import build
    from hipps.ops import nn as hnn

    def run(shadow_linear):
        saved = hnn._SHADOW_LINEAR
        hnn._SHADOW_LINEAR = shadow_linear
        torch.manual_seed(3)
        m = build(name).cuda()
        opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="local", bf16_weights="on")
        ids = torch.randint(0, 512, (4, 32), device=DEV, generator=torch.Generator(device=DEV).manual_seed(4))
        losses = []
        try:
            for _ in range(4):
                opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = m(ids, ids)
                loss.backward()
                opt.step()
                losses.append(loss.item())
        finally:
            opt.close()
            hnn._SHADOW_LINEAR = saved
        return losses

    on, off = run(True), run(False)
    assert all(v == v for v in on) and on[-1] < on[0]
    torch.testing.assert_close(torch.tensor(on), torch.tensor(off), rtol=2e-2, atol=2e-2)


def test_transformer_async_step_on_shadow_linear():
    """The default async path (bf16 shadow auto-on for ps_async on a GPU) with the tiny BERT."""
    import hipps
    from hipps.models.transformer import build

    torch.manual_seed(5)
    m = build("bert-tiny").cuda()
    opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="ps_async", max_delay=0)
    ids = torch.randint(0, 512, (4, 32), device=DEV)
    losses = []
    try:
        for _ in range(6):
            opt.zero_grad()
            with torch.autocast("cuda", dtype=torch.bfloat16):
                loss = m(ids, ids)
            loss.backward()
            opt.step()
            losses.append(loss.item())
    finally:
        opt.close()
    assert all(v == v for v in losses) and losses[-1] < losses[0]


@pytest.mark.parametrize("m,n,k", [(4096, 768, 768), (2048, 3072, 768), (2048, 768, 3072), (1024, 192, 64), (100, 96, 48)])
def test_linear_wgrad_matches_fp32(m, n, k):
    """The tuner-picked Linear weight gradient (hipBLASLt or a gemm2 split-M kernel) against fp64."""
    from hipps.ops import nn as hnn

    torch.manual_seed(m + n + k)
    dy = torch.randn(m, n, device=DEV).to(torch.bfloat16)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    dw = hnn._linear_wgrad(dy, x)
    ref = dy.double().t() @ x.double()
    assert dw.dtype == torch.float32 and dw.shape == (n, k)
    torch.testing.assert_close(dw.double(), ref, rtol=1e-3, atol=1e-2 * (m ** 0.5) / 16)


@pytest.mark.parametrize("m,n,k", [(4096, 768, 768), (2048, 3072, 1024), (1024, 4096, 512), (200, 128, 64)])
def test_linear_fwd_nobias_matches_fp32(m, n, k):
    """The tuner-picked bias-free Linear forward (hipBLASLt or a hipps 1x1 GEMM core) against fp64."""
    from hipps.ops import nn as hnn

    torch.manual_seed(m + n)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) / k ** 0.5).to(torch.bfloat16)
    y = hnn._linear_fwd_nobias(x, w)
    ref = x.double() @ w.double().t()
    assert y.dtype == torch.bfloat16 and y.shape == (m, n)
    torch.testing.assert_close(y.double(), ref, rtol=1e-2, atol=1e-2)


@pytest.mark.parametrize("m,n,k", [(4096, 768, 768), (2048, 3072, 768), (4096, 768, 3072), (200, 128, 64)])
def test_linear_fwd_bias_matches_fp32(m, n, k):
    """The tuner-picked biased Linear forward (hipBLASLt addmm or a hipps 1x1 GEMM core with the
    fp32 kBias epilogue) against fp64; every gemm2 candidate is also checked on its own."""
    from hipps.ops import nn as hnn
    from hipps.ops._native import native

    torch.manual_seed(m + n + 7)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) / k ** 0.5).to(torch.bfloat16)
    b = torch.randn(n, device=DEV)
    y = hnn._linear_fwd(x, w, b)
    ref = x.double() @ w.double().t() + b.double()
    assert y.dtype == torch.bfloat16 and y.shape == (m, n)
    torch.testing.assert_close(y.double(), ref, rtol=1e-2, atol=1e-2)
    if m >= 1024:
        for name in hnn._g2_names(n):
            bm, bn, ns = hnn._g2_parse(name)
            y2 = torch.full_like(y, float("nan"))
            native().gemm2_conv(x, w, y2, None, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns, bias=b)
            torch.testing.assert_close(y2.double(), ref, rtol=1e-2, atol=1e-2, msg=name)


@pytest.mark.parametrize("m,n,k,bias", [(4096, 768, 768, True), (4096, 768, 3072, True), (2048, 1024, 512, False),
                                        (200, 128, 64, True)])
def test_linear_fwd_residual_matches_fp32(m, n, k, bias):
    """y = x w^T (+ b) + r: the tuner-picked route (hipBLASLt with r as C, or a gemm2 core with the
    kBias | kAdd epilogue) and every gemm2 candidate on its own, against fp64."""
    from hipps.ops import nn as hnn
    from hipps.ops._native import native

    torch.manual_seed(m + n + k)
    x = torch.randn(m, k, device=DEV).to(torch.bfloat16)
    w = (torch.randn(n, k, device=DEV) / k ** 0.5).to(torch.bfloat16)
    b = torch.randn(n, device=DEV) if bias else None
    r = torch.randn(m, n, device=DEV).to(torch.bfloat16)
    y = hnn._linear_fwd(x, w, b, r)
    ref = x.double() @ w.double().t() + r.double() + (b.double() if bias else 0)
    torch.testing.assert_close(y.double(), ref, rtol=2e-2, atol=2e-2)
    if m >= 1024:
        for name in hnn._g2_names(n):
            bm, bn, ns = hnn._g2_parse(name)
            y2 = torch.full_like(y, float("nan"))
            native().gemm2_conv(x, w, y2, None, r, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns, bias=b)
            torch.testing.assert_close(y2.double(), ref, rtol=2e-2, atol=2e-2, msg=name)


def test_shadow_linear_residual_gradients():
    """linear(x, w, b, residual=r) under autocast on the shadow: r's gradient is dy itself."""
    from hipps.ops import nn as hnn

    torch.manual_seed(11)
    flat, shadow, (w, b) = _shadowed((64, 64), (64,))
    try:
        x = torch.randn(2, 40, 64, device=DEV, requires_grad=True)
        r = torch.randn(2, 40, 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert hnn.shadow_linear_ok(x, w, b, r)
            y = hnn.linear(x, w, b, residual=r)
        g = torch.randn_like(y)
        y.backward(g)
        assert r.grad.dtype == torch.bfloat16 and torch.equal(r.grad, g)
        ref = F.linear(x.detach().double(), w.detach().double(), b.detach().double()) + r.detach().double()
        torch.testing.assert_close(y.double(), ref, rtol=3e-2, atol=3e-2)
    finally:
        hnn.unregister_weight_shadow(shadow)


def test_shadow_linear_fp32_residual():
    """An fp32 residual stream (Llama: x + wo(a)) is added by the GEMM itself (hipBLASLt C, fp32
    output): y is fp32 and equals residual + x w^T; the residual's gradient is dy (fp32), and the
    input / weight gradients match autocast's F.linear."""
    from hipps.ops import nn as hnn

    torch.manual_seed(12)
    flat, shadow, (w,) = _shadowed((128, 64))
    try:
        x = torch.randn(2, 48, 64, device=DEV).to(torch.bfloat16).requires_grad_(True)
        r = torch.randn(2, 48, 128, device=DEV, requires_grad=True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            assert hnn.shadow_linear_ok(x, w, None, r)
            y = hnn.linear(x, w, residual=r)
        assert y.dtype == torch.float32
        ref = F.linear(x.detach().double(), w.detach().to(torch.bfloat16).double()) + r.detach().double()
        torch.testing.assert_close(y.double(), ref, rtol=1e-3, atol=5e-3)
        g = torch.randn_like(y)
        y.backward(g)
        assert r.grad.dtype == torch.float32 and torch.equal(r.grad, g)
        x0 = x.detach().clone().requires_grad_(True)
        w0 = torch.nn.Parameter(w.detach().clone())
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y0 = F.linear(x0, w0)
        y0.backward(g.to(torch.bfloat16))
        torch.testing.assert_close(x.grad.float(), x0.grad.float(), rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(w.grad, w0.grad, rtol=2e-2, atol=2e-2)
    finally:
        hnn.unregister_weight_shadow(shadow)


@pytest.mark.parametrize("name", ["g2_256x256", "g2_256x256s5", "g2_256x256s6", "g2_256x128", "g2_256x128s3",
                                  "g2_128x128", "g2_128x128s3", "g2_256x64", "g2_128x64", "g2_128x64s3"])
def test_gemm2_gelu_epilogues_every_tile(name):
    """gemm2.hip kGelu (y = gelu(x w^T + b), pre kept) and kGeluB (gelu'(pre) * (dy w)) on every
    tile against the fp32 formula over the same bf16 operands (M not a tile multiple)."""
    from hipps.ops import _native
    from hipps.ops import nn as hnn

    C = _native.native()
    bm, bn, ns = hnn._g2_parse(name)
    torch.manual_seed(bm + bn + ns)
    M, K, N = 1000, 256, 512
    x = (torch.randn(M, K, device=DEV) * 0.5).to(torch.bfloat16)
    w = (torch.randn(N, K, device=DEV) * 0.1).to(torch.bfloat16)
    b = torch.randn(N, device=DEV) * 0.5
    pre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    post = torch.empty_like(pre)
    C.gemm2_conv(x, w, post, None, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns, bias=b, gelu_pre=pre, gelu=1)
    ref_pre = x.float() @ w.float().t() + b
    torch.testing.assert_close(pre.float(), ref_pre, rtol=1e-2, atol=1e-2)
    # the GELU of the stored bf16 pre-activation, as F.gelu on it rounds it
    torch.testing.assert_close(post.float(), F.gelu(pre.float()).to(torch.bfloat16).float(), rtol=0, atol=1e-2)
    # backward: dy [M, K2] through w2 [K2, N] (the next Linear, transposed for the kernel)
    K2 = 256
    dy = torch.randn(M, K2, device=DEV).to(torch.bfloat16)
    w2 = (torch.randn(K2, N, device=DEV) * 0.1).to(torch.bfloat16)
    dpre = torch.empty(M, N, device=DEV, dtype=torch.bfloat16)
    C.gemm2_conv(dy, w2.t().contiguous(), dpre, None, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns,
                 gelu_pre=pre, gelu=2)
    dpost = (dy.float() @ w2.float())
    prf = pre.float()
    ref = dpost * (0.5 * (1 + torch.erf(prf * 0.7071067811865476)) + prf * torch.exp(-0.5 * prf * prf) * 0.3989422804014327)
    torch.testing.assert_close(dpre.float(), ref, rtol=2e-2, atol=2e-2)
    # kGeluBS: the same output plus per-m-tile column sums of it (the first Linear's bias gradient)
    part = torch.empty((C.gemm2_mtiles(M, N, K2, bm), N), device=DEV, dtype=torch.float32)
    dpre2 = torch.empty_like(dpre)
    C.gemm2_conv(dy, w2.t().contiguous(), dpre2, part, None, None, 1, 1, 1, 1, 1, 0, bm, bn, stages=ns,
                 gelu_pre=pre, gelu=2)
    assert torch.equal(dpre2, dpre)
    db = torch.empty(N, device=DEV, dtype=torch.float32)
    C.colsum_fold(part, db)
    torch.testing.assert_close(db.double(), dpre.double().sum(0), rtol=1e-5, atol=1e-3)


def test_gelu_mlp_matches_fp32_and_composition():
    """hnn.gelu_mlp (one _GeluMLP node: kGelu / kGeluB epilogues, the residual gradient folded
    into the input-gradient addmm) against the fp32 formula over the bf16 shadows, forward and
    every gradient; the tuner runs (M >= 1024)."""
    from hipps.ops import nn as hnn

    torch.manual_seed(3)
    D, F4 = 256, 1024
    flat, shadow, (w1, b1, w2, b2) = _shadowed((F4, D), (F4,), (D, F4), (D,))
    try:
        l1 = hnn.Linear(D, F4).to(DEV)
        l2 = hnn.Linear(F4, D).to(DEV)
        l1.weight, l1.bias, l2.weight, l2.bias = w1, b1, w2, b2
        # the W^T copies the flat store keeps for marked Linears (gemm2 input-gradient epilogues)
        for w in (w1, w2):
            hnn.register_transposed_weight(w, w.detach().t().contiguous().to(torch.bfloat16))
        x = (torch.randn(4, 512, D, device=DEV)).to(torch.bfloat16).requires_grad_(True)
        with torch.autocast("cuda", dtype=torch.bfloat16):
            y = hnn.gelu_mlp(x, l1, l2, residual_x=True)
        assert y.grad_fn is not None and "GeluMLP" in type(y.grad_fn).__name__
        g = torch.randn_like(y)
        y.backward(g)
        xs = x.detach().double().requires_grad_(True)
        sw = [t.detach().to(torch.bfloat16).double().requires_grad_(True) for t in (w1, b1, w2, b2)]
        ref = F.linear(F.gelu(F.linear(xs, sw[0], sw[1])), sw[2], sw[3]) + xs
        ref.backward(g.double())
        torch.testing.assert_close(y.double(), ref, rtol=3e-2, atol=3e-2)
        torch.testing.assert_close(x.grad.double(), xs.grad, rtol=3e-2, atol=3e-2)
        for p, r in zip((w1, b1, w2, b2), sw):
            assert p.grad.dtype == torch.float32
            tol = 2e-2 * r.grad.abs().max().item() + 1e-3
            torch.testing.assert_close(p.grad.double(), r.grad, rtol=3e-2, atol=tol)
    finally:
        hnn.unregister_weight_shadow(shadow)
        for w in (w1, w2):
            hnn.unregister_transposed_weight(w)


def test_residual_link_folds_the_residual_gradient():
    """ResidualLink: qkv(x, link) ... out(a, residual=x, link) gives x the same gradient as the
    unlinked pair (the residual's gradient added inside qkv's input-gradient addmm), and an
    unarmed link (reader off the shadow path) leaves the residual's gradient to autograd."""
    from hipps.ops import nn as hnn

    torch.manual_seed(5)
    D = 128
    flat, shadow, (w1, w2) = _shadowed((D, D), (D, D))
    hnn.register_transposed_weight(w1, w1.detach().t().contiguous().to(torch.bfloat16))
    try:
        x0 = torch.randn(8, 256, D, device=DEV).to(torch.bfloat16)
        g = torch.randn(8, 256, D, device=DEV).to(torch.bfloat16)

        def run(use_link, arm=True):
            x = x0.clone().requires_grad_(True)
            link = hnn.ResidualLink() if use_link else None
            with torch.autocast("cuda", dtype=torch.bfloat16):
                h = hnn.linear(x, w1, None, link=link if arm else None)
                y = hnn.linear(torch.tanh(h), w2, None, residual=x, link=link)
            y.backward(g)
            return x.grad.float()

        ref = run(False)
        torch.testing.assert_close(run(True), ref, rtol=2e-2, atol=2e-2)
        torch.testing.assert_close(run(True, arm=False), ref, rtol=0, atol=0)
    finally:
        hnn.unregister_weight_shadow(shadow)
        hnn.unregister_transposed_weight(w1)


def test_bert_fused_tail_matches_compositions_at_gemm2_sizes(monkeypatch):
    """A small BERT (1024 tokens: the gemm2 candidates are live) with the round-6 transformer tail
    -- GELU MLP node (kGelu / kGeluB / kGeluBS over the W^T shadows), residual links, LayerNorm dx
    column sums, fused embedding -- against the same model on the module compositions: the first
    step's gradients agree and three steps' losses track each other."""
    import hipps
    from hipps.models.transformer import Bert, BertConfig
    from hipps.ops import nn as hnn

    def run(fused):
        for flag in ("_GELU_MLP", "_RES_LINK", "_FUSED_EMBED"):
            monkeypatch.setattr(hnn, flag, fused)
        torch.manual_seed(21)
        m = Bert(BertConfig(vocab=1000, hidden=128, layers=2, heads=2, ffn=512, max_pos=128)).cuda()
        opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="local", bf16_weights="on")
        ids = torch.randint(0, 1000, (8, 128), device=DEV, generator=torch.Generator(device=DEV).manual_seed(22))
        losses, grads = [], None
        try:
            for i in range(3):
                opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = m(ids, ids)
                loss.backward()
                if i == 0:
                    grads = {n: p.grad.detach().float().clone() for n, p in m.named_parameters() if p.grad is not None}
                opt.step()
                losses.append(loss.item())
        finally:
            opt.close()
        return losses, grads

    (l1, g1), (l0, g0) = run(True), run(False)
    assert g1.keys() == g0.keys()
    for n in g0:
        scale = g0[n].abs().max().item() + 1e-6
        assert (g1[n] - g0[n]).abs().max().item() <= 5e-2 * scale + 1e-4, n
    torch.testing.assert_close(torch.tensor(l1), torch.tensor(l0), rtol=2e-2, atol=2e-2)
    assert l1[-1] < l1[0]
