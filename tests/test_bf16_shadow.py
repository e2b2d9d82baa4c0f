"""bf16 weight shadow (FlatStore.enable_bf16_shadow / ops.nn.bf16_weight): the conv kernels read a
flat bf16 copy of the fp32 params refreshed once per step instead of casting every layer's weight
in every forward.  The cast is the same round-to-nearest, so training must match to summation-order rounding."""
import pytest
import torch
import torch.nn.functional as F

import hipps
from hipps.ops import nn as hnn


def _conv_model():
    torch.manual_seed(0)
    return torch.nn.Sequential(torch.nn.Conv2d(8, 16, 3, bias=False), torch.nn.Conv2d(16, 4, 1, bias=False))


def test_shadow_views_follow_steps_cpu():
    m = _conv_model().to(memory_format=torch.channels_last)
    opt = hipps.SGD(m.named_parameters(), lr=0.1, momentum=0.9, mode="local", bf16_weights="on")
    try:
        for p in m.parameters():
            v = hnn.bf16_weight(p)
            assert v.dtype == torch.bfloat16 and v.shape == p.shape and v.stride() == p.stride()
            assert torch.equal(v, p.detach().to(torch.bfloat16))
        x = torch.randn(2, 8, 6, 6).contiguous(memory_format=torch.channels_last)
        m(x).square().mean().backward()
        opt.step()
        for p in m.parameters():  # refreshed by step()
            assert torch.equal(hnn.bf16_weight(p), p.detach().to(torch.bfloat16))
        with torch.no_grad():
            for p in m.parameters():
                p.mul_(0.5)
        opt.refresh_bf16_weights()
        for p in m.parameters():
            assert torch.equal(hnn.bf16_weight(p), p.detach().to(torch.bfloat16))
        foreign = torch.randn(3, 3)
        assert torch.equal(hnn.bf16_weight(foreign), foreign.to(torch.bfloat16))
    finally:
        opt.close()
    assert not hnn._SHADOWS  # close() unregisters


def test_shadow_auto_off_for_sync_modes_cpu():
    m = _conv_model()
    opt = hipps.SGD(m.named_parameters(), lr=0.1, mode="local")
    try:
        assert getattr(opt.store, "shadow", None) is None
    finally:
        opt.close()


@pytest.mark.gpu
def test_shadow_resnet_bit_identical_gpu():
    from hipps.models import resnet_tiny

    from hipps.ops import nn as hnn

    def run(flag):
        torch.manual_seed(0)
        m = resnet_tiny().cuda().to(memory_format=torch.channels_last)
        opt = hipps.SGD(m.named_parameters(), lr=0.05, momentum=0.9, mode="local", bf16_weights=flag)
        # the conv path only: the fc layer on the shadow computes an fp32 weight gradient (vs a bf16
        # one cast up), a deliberate numeric difference covered by tests/test_shadow_linear_gpu.py
        saved = hnn._SHADOW_LINEAR
        hnn._SHADOW_LINEAR = False
        g = torch.Generator(device="cuda").manual_seed(1)
        losses = []
        try:
            for _ in range(3):
                x = torch.randn(8, 3, 32, 32, device="cuda", generator=g).contiguous(memory_format=torch.channels_last)
                y = torch.randint(0, 10, (8,), device="cuda", generator=g)
                opt.zero_grad()
                with torch.autocast("cuda", dtype=torch.bfloat16):
                    loss = F.cross_entropy(m(x), y)
                loss.backward()
                opt.step()
                losses.append(loss.item())
            return losses, opt.store.data.clone()
        finally:
            hnn._SHADOW_LINEAR = saved
            opt.close()

    l_on, p_on = run("on")
    l_off, p_off = run("off")
    # same bf16 rounding of the weights; MIOpen may pick solvers with a different summation order
    # between the two runs, so the parameters are compared to fp32 rounding, not bitwise
    torch.testing.assert_close(torch.tensor(l_on), torch.tensor(l_off), rtol=1e-3, atol=1e-4)
    torch.testing.assert_close(p_on, p_off, rtol=1e-3, atol=1e-5)


@pytest.mark.gpu
def test_transposed_shadow_matches_torch_gpu():
    torch.manual_seed(0)
    convs = torch.nn.ModuleList([torch.nn.Conv2d(130, 70, 1, bias=False), torch.nn.Conv2d(64, 256, 1, bias=False),
                                 torch.nn.Conv2d(8, 8, 3, bias=False), torch.nn.Conv2d(2048, 512, 1, bias=False),
                                 torch.nn.Conv2d(192, 72, 3, bias=False), torch.nn.Conv2d(3, 64, 7, bias=False)])
    convs = convs.cuda().to(memory_format=torch.channels_last)
    opt = hipps.SGD(convs.named_parameters(), lr=0.1, mode="local", bf16_weights="on")
    try:
        for c in convs:
            w = c.weight
            t = hnn._TSHADOWS.get(w.data_ptr())
            if w.shape[2] != 1:  # rot180(W)^T, channels-last
                ref = torch.flip(w.detach(), (2, 3)).transpose(0, 1).to(torch.bfloat16)
                assert t.shape == ref.shape and t.is_contiguous(memory_format=torch.channels_last)
                assert torch.equal(t, ref)
                continue
            ref = w.detach().reshape(w.shape[0], w.shape[1]).t().to(torch.bfloat16)
            assert t.shape == ref.shape and torch.equal(t, ref)
        with torch.no_grad():
            for c in convs:
                c.weight.mul_(-3.0)
        opt.refresh_bf16_weights()
        for c in convs:
            w = c.weight
            if w.shape[2] == 1:
                ref = w.detach().reshape(w.shape[0], w.shape[1]).t().to(torch.bfloat16)
                assert torch.equal(hnn._TSHADOWS[w.data_ptr()], ref)
    finally:
        opt.close()
    assert not hnn._TSHADOWS


def test_watch_module_refreshes_shadow_after_model_load():
    """a model.load_state_dict after the optimizer exists must reach the bf16 shadow."""
    import hipps

    m = torch.nn.Sequential(torch.nn.Linear(16, 16), torch.nn.Linear(16, 4))
    opt = hipps.SGD(m.named_parameters(), lr=0.1, mode="local", bf16_weights="on")
    if getattr(opt.store, "shadow", None) is None:
        opt.close()
        return  # (no shadow on this device)
    opt.watch_module(m)
    sd = {k: torch.full_like(v, 0.5) for k, v in m.state_dict().items()}
    m.load_state_dict(sd)
    assert torch.equal(opt.store.shadow.float(), opt.store.data.to(torch.bfloat16).float())
    opt.close()
