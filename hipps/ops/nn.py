"""Fused model ops backed by hipps HIP kernels.

``conv_bn`` runs a 1x1 convolution feeding such a BN as an MFMA GEMM whose epilogue emits the
BN batch statistics (hipps/csrc/gemm.hip).

``FusedBatchNorm2d`` is a drop-in ``nn.BatchNorm2d`` that can also apply a residual add and a
ReLU in the same pass (``forward(x, residual=None)``).  On a HIP device with a channels-last
bf16 input (the autocast ResNet path) it runs hipps/csrc/norm.hip: one statistics pass, one
apply pass, and a backward that recomputes the ReLU mask instead of storing it.  Anything
else (CPU, fp32, NCHW, odd channel counts, eval with grad) takes the standard PyTorch path, so
models stay portable and the CPU test suite exercises the same module.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from ._native import native

import os as _os

# weight gradient of the MFMA 1x1 path: own split-M kernel (1) or MIOpen (0, default: measured
# faster in the full step, profiles/conv1x1_wgrad_r1.json)
_OWN_WGRAD = _os.environ.get("HIPPS_CONV_WGRAD", "0") != "0"

MASK_NONE, MASK_X, MASK_Y, MASK_BITS = 0, 1, 2, 3


class _Conv1x1(torch.autograd.Function):
    """1x1 convolution on channels-last bf16 as an MFMA GEMM (hipps/csrc/gemm.hip) that also
    emits the per-channel batch statistics of its output for the BatchNorm that follows.
    Backward: the input gradient of a stride-1 conv is the same NT GEMM against the transposed
    weight (dX[M,Cin] = dY[M,Cout] . W[Cout,Cin]); the weight gradient is the split-M MFMA
    reduction with transposing LDS reads (conv1x1_wgrad), written straight into an fp32 grad
    for an fp32 master weight (no bf16 round trip); strided dgrad goes to MIOpen."""

    @staticmethod
    def forward(ctx, x, w_master, stride):
        w = w_master if w_master.dtype == torch.bfloat16 else w_master.to(torch.bfloat16)
        ctx.wdtype = w_master.dtype
        N, Cin, H, W = x.shape
        Cout = w.shape[0]
        Ho, Wo = (H - 1) // stride + 1, (W - 1) // stride + 1
        y = torch.empty((N, Cout, Ho, Wo), dtype=torch.bfloat16, device=x.device, memory_format=torch.channels_last)
        mt = native().conv1x1_mtiles(N * Ho * Wo)
        part = torch.empty((2, Cout, mt), dtype=torch.float32, device=x.device)
        native().conv1x1_forward(x, w.reshape(Cout, Cin), y, part, H, W, stride)
        ctx.stride = stride
        ctx.save_for_backward(x, w)
        ctx.mark_non_differentiable(part)
        return y, part

    @staticmethod
    def backward(ctx, dy, _dpart):
        x, w = ctx.saved_tensors
        s = ctx.stride
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = dw = None
        own_dx = ctx.needs_input_grad[0] and s == 1
        if ctx.needs_input_grad[0] and not own_dx:
            dx = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                     [True, False, False])[0]
        if ctx.needs_input_grad[1] and not _OWN_WGRAD:
            dw = torch.ops.aten.convolution_backward(dy, x, w, None, [s, s], [0, 0], [1, 1], False, [0, 0], 1,
                                                     [False, True, False])[1].to(ctx.wdtype)
        elif ctx.needs_input_grad[1]:
            dw = torch.empty(w.shape, dtype=torch.float32, device=w.device)
            native().conv1x1_wgrad(dy, x, dw.view(w.shape[0], w.shape[1]), x.shape[2], x.shape[3], s)
            if ctx.wdtype != torch.float32:
                dw = dw.to(ctx.wdtype)
        if own_dx:
            cout, cin = w.shape[0], w.shape[1]
            wt = w.reshape(cout, cin).t().contiguous()  # [Cin, Cout]: K-contiguous B operand
            dx = torch.empty_like(x, memory_format=torch.channels_last)
            native().conv1x1_forward(dy, wt, dx, None, x.shape[2], x.shape[3], 1)
        return dx, dw, None


def conv1x1_ok(conv: nn.Conv2d, x: torch.Tensor) -> bool:
    """Can the MFMA 1x1 path run this convolution on this input?"""
    if not (x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4 and
            x.is_contiguous(memory_format=torch.channels_last)):
        return False
    if conv.kernel_size != (1, 1) or conv.padding != (0, 0) or conv.dilation != (1, 1) or conv.groups != 1:
        return False
    if conv.bias is not None or conv.stride[0] != conv.stride[1]:
        return False
    return conv.in_channels % 64 == 0 and conv.out_channels % 64 == 0


def conv1x1_stats(x, weight, stride=1):
    """(y, part): bf16 1x1 conv output and its [2, Cout, m_tiles] BN partial statistics."""
    return _Conv1x1.apply(x, weight, int(stride))


class _FusedBNAct(torch.autograd.Function):
    @staticmethod
    def forward(ctx, x, res, weight, bias, running_mean, running_var, eps, momentum, relu, part=None):
        C = x.shape[1]
        y = torch.empty_like(x, memory_format=torch.channels_last)
        f32 = dict(dtype=torch.float32, device=x.device)
        mean, invstd = torch.empty(C, **f32), torch.empty(C, **f32)
        scale, shift = torch.empty(C, **f32), torch.empty(C, **f32)
        # relu(bn(x) + res): the mask depends on res, so keep 1 bit per element instead of
        # re-reading the bf16 output in the backward
        mode = MASK_NONE if not relu else (MASK_BITS if res is not None else MASK_X)
        mask = torch.empty(x.numel() // 8, dtype=torch.uint8, device=x.device) if mode == MASK_BITS else None
        if part is not None:  # statistics already reduced by the producing 1x1 conv
            native().bn_forward_partials(part, part.shape[2], x, res, y, weight, bias, running_mean, running_var,
                                         mean, invstd, scale, shift, C, float(eps), float(momentum), bool(relu), mask)
        else:
            native().bn_forward_train(x, res, y, weight, bias, running_mean, running_var, mean, invstd, scale, shift,
                                      C, float(eps), float(momentum), bool(relu), mask)
        ctx.mode, ctx.C, ctx.has_res = mode, C, res is not None
        ctx.save_for_backward(x, mask, weight, mean, invstd, scale, shift)
        return y

    @staticmethod
    def backward(ctx, dy):
        x, mask, weight, mean, invstd, scale, shift = ctx.saved_tensors
        dy = dy.to(torch.bfloat16).contiguous(memory_format=torch.channels_last)
        dx = torch.empty_like(x, memory_format=torch.channels_last)
        dres = torch.empty_like(x, memory_format=torch.channels_last) if ctx.has_res else None
        dw = torch.empty_like(weight)
        db = torch.empty_like(weight)
        native().bn_backward(dy, x, None, ctx.mode, weight, mean, invstd, scale, shift, dx, dres, dw, db, ctx.C, mask)
        return dx, dres, dw, db, None, None, None, None, None, None


def fused_bn_act(x, weight, bias, running_mean, running_var, eps=1e-5, momentum=0.1, relu=True, residual=None,
                 part=None):
    """Training-mode BN (+residual) (+ReLU) on a channels-last bf16 HIP tensor.  ``part``: the
    [2, C, nrb] partial statistics when the producer (conv1x1_stats) already reduced them."""
    return _FusedBNAct.apply(x, residual, weight, bias, running_mean, running_var, eps, momentum, relu, part)


class FusedBatchNorm2d(nn.BatchNorm2d):
    """nn.BatchNorm2d with optional fused residual add and ReLU."""

    def __init__(self, num_features, relu: bool = False, fused: bool = True, **kw):
        super().__init__(num_features, **kw)
        self.relu = relu
        self.fused = fused
        # num_batches_tracked is only read when momentum is None; bumping the device buffer costs
        # one kernel launch per BN per step (53 per ResNet-50 step), so count on the host and fold
        # the count in whenever the state is read.
        self._nbt_pending = 0
        self.register_state_dict_pre_hook(lambda mod, *a, **k: mod.sync_num_batches_tracked())

    def sync_num_batches_tracked(self):
        if self._nbt_pending and self.num_batches_tracked is not None:
            self.num_batches_tracked.add_(self._nbt_pending)
        self._nbt_pending = 0

    def extra_repr(self):
        return super().extra_repr() + f", relu={self.relu}, fused={self.fused}"

    def _fast_ok(self, x, residual) -> bool:
        if not (self.fused and x.is_cuda and x.dtype == torch.bfloat16 and x.dim() == 4):
            return False
        C = x.shape[1]
        if C % 8 or C > 2048 or not self.affine or not x.is_contiguous(memory_format=torch.channels_last):
            return False
        if self.training and (not self.track_running_stats or self.momentum is None):
            return False
        if residual is not None and (residual.dtype != torch.bfloat16 or residual.shape != x.shape or
                                     not residual.is_contiguous(memory_format=torch.channels_last)):
            return False
        if x.numel() % 16:
            return False
        return True

    def forward(self, x, residual=None, stats=None):
        if self._fast_ok(x, residual):
            if self.training:
                self._nbt_pending += 1
                return fused_bn_act(x, self.weight, self.bias, self.running_mean, self.running_var, self.eps,
                                    self.momentum, self.relu, residual, stats)
            if not torch.is_grad_enabled() or not (x.requires_grad or (residual is not None and
                                                                       residual.requires_grad)):
                scale = self.weight / torch.sqrt(self.running_var + self.eps)
                shift = self.bias - self.running_mean * scale
                y = torch.empty_like(x, memory_format=torch.channels_last)
                native().bn_apply(x, residual, y, scale.float().contiguous(), shift.float().contiguous(),
                                  x.shape[1], self.relu)
                return y
        y = super().forward(x)
        if residual is not None:
            y = y + residual
        if self.relu:
            y = F.relu(y)
        return y


def conv_bn(conv: nn.Conv2d, bn: FusedBatchNorm2d, x, residual=None, fuse: bool = True):
    """bn(conv(x), residual): a 1x1 conv that feeds a training-mode fused BN runs as the MFMA GEMM
    with the BN statistics in its epilogue (one fewer pass over the conv output)."""
    if fuse and bn.training and conv1x1_ok(conv, x):
        y, part = conv1x1_stats(x, conv.weight, conv.stride[0])
        if bn._fast_ok(y, residual):
            return bn(y, residual, stats=part)
        return bn(y, residual)
    return bn(conv(x), residual)
