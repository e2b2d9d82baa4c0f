"""ResNet-50 (and family) for the synthetic-ImageNet async-PS benchmark.

The reference has no model zoo (SURVEY.md §1 "Missing layers"); BASELINE.json names
"ResNet-50 synthetic-ImageNet async PS (AsySG-InCon) bf16" as the headline config, so the
framework ships its own ResNet definition (random init, no checkpoints, no torchvision).

MI355X notes: convolutions go to MIOpen (library path), run channels_last in bf16 under
autocast; parameters stay fp32 so the PS keeps an exact fp32 master copy and the wire codec
decides the transport precision.
"""
from __future__ import annotations

import torch
import torch.nn as nn
import torch.nn.functional as F

from hipps.ops.nn import (FusedBatchNorm2d, Linear, MaxPool2d, ResidualTap, bn_pro_pays, bn_relu_conv, bn_relu_conv1x1_ok,
                          bn_relu_conv_bn, bn_relu_conv_ok, bn_relu_maxpool, conv1x1_bn_input, conv1x1_ok, conv2d,
                          conv2d_bn, conv2d_stats, conv_bn, dual_bn_relu, dual_bn_relu_ok, global_avg_pool,
                          stem_block, stem_block_ok)

# One switch for the whole zoo: fused BN(+residual)(+ReLU) HIP kernels on channels-last bf16,
# standard PyTorch elsewhere.  HIPPS_FUSED_BN=0 restores the eager MIOpen path for A/B runs.
import os as _os

_FUSED = _os.environ.get("HIPPS_FUSED_BN", "1") != "0"
# 1x1 convolutions feeding a fused BN: MFMA GEMM with the BN statistics in its epilogue
_FUSED_CONV = _FUSED and _os.environ.get("HIPPS_FUSED_CONV", "1") != "0"
# residual-gradient sums folded into the 1x1 dgrad epilogue (ResidualTap / alias)
_FUSED_GRAD = _FUSED_CONV and _os.environ.get("HIPPS_FUSED_GRAD", "1") != "0"
# stem max pool on the hipps kernels
_FUSED_POOL = _FUSED and _os.environ.get("HIPPS_FUSED_POOL", "1") != "0"
# BN backward reductions done in the consuming 1x1 conv's dgrad epilogue (BNGradTap)
_FUSED_BNGRAD = _os.environ.get("HIPPS_FUSED_BNGRAD", "1") != "0"
# 3x3 convolutions: weight gradient on the hipps implicit-GEMM kernel (fwd / dgrad stay on MIOpen)
_FUSED_WGRAD = _os.environ.get("HIPPS_FUSED_WGRAD", "1") != "0"
# bn2 -> conv3: BN apply + ReLU in the 1x1 GEMM's operand prologue (the BN output is never written).
# Opt-in: measured on ResNet-50 bs256 it removes 16 apply passes (-0.23 ms/step) but the prologue
# GEMMs lose about as much (+0.10..0.17 ms/step), profiles/ab_r2/prologue_*.txt
# stem conv on the hipps MFMA stem kernels (BN statistics in the forward epilogue); HIPPS_OWN_STEM=0
# keeps it on MIOpen
_FUSED_STEM = _FUSED
# stem BN apply + ReLU folded into the max pool's load (the BN output is never materialised)
_FUSED_STEM_POOL = _FUSED_STEM and _os.environ.get("HIPPS_FUSED_STEMPOOL", "1") != "0"
# ... and the stem's backward as one node (_StemBlock): the pool gradient is never materialised; 2 (default)
# writes the BN input gradient in one pass for the plain weight gradient, 1 recomputes it inside the
# weight gradient's staging (latency-bound there: 10308 vs 10342 img/s in round 2,
# profiles/ab_r2/stembwd_*; 12020 / 12037 vs 12171 / 12089 in round 5, profiles/r5/stem/), 0 = pool backward + BN
# backward kernels
_FUSED_STEM_BWD = _FUSED_STEM_POOL and _os.environ.get("HIPPS_FUSED_STEMBWD", "2") != "0"
_FUSED_PRO = _FUSED_CONV and _os.environ.get("HIPPS_FUSED_PRO", "0") != "0"
# downsample blocks: the downsample BN applied inside bn3's apply pass (its output, the residual,
# is never materialised) and both BNs' backward in two passes (ops.nn._DualBNRelu)
_FUSED_DUAL = _FUSED_GRAD and _os.environ.get("HIPPS_FUSED_DUAL", "1") != "0"
# bn1 -> conv2 and bn2 -> conv3 with the BN + ReLU applied to the conv's staged A tiles in LDS
# (ops.nn._BNReluConv): the bn1 / bn2 outputs are never written.  Opt-in: bit-identical to the
# apply pass + plain GEMM (tests), but the in-LDS transform sits between each tile's DMA and its
# barrier and the compute-bound 3x3 GEMMs lose 15-47 % (forward and weight gradient) -- more
# than the 32 apply passes cost (same box: 11070 off vs 10629 img/s on, profiles/r3b/bnpro/)
_BN_PRO = _FUSED_DUAL and _os.environ.get("HIPPS_BN_PRO", "0") == "1"
# HIPPS_BN_PRO=2: only bn2 -> conv3 (the 1x1, memory-bound side) takes the prologue; bn1 is applied
# by its own pass and conv2 (the compute-bound 3x3 GEMM that the in-LDS transform slows) stays plain
_BN_PRO2 = _FUSED_DUAL and _os.environ.get("HIPPS_BN_PRO", "0") == "2"


def _bn(c, relu=False):
    return FusedBatchNorm2d(c, relu=relu, fused=_FUSED)


def _conv(cin, cout, k, stride=1, groups=1):
    return nn.Conv2d(cin, cout, k, stride=stride, padding=k // 2, groups=groups, bias=False)


class Bottleneck(nn.Module):
    expansion = 4

    def __init__(self, cin, width, stride=1, downsample=False):
        super().__init__()
        cout = width * self.expansion
        self.conv1 = _conv(cin, width, 1)
        self.bn1 = _bn(width, relu=True)
        self.conv2 = _conv(width, width, 3, stride=stride)
        self.bn2 = _bn(width, relu=True)
        self.conv3 = _conv(width, cout, 1)
        self.bn3 = _bn(cout, relu=True)  # relu(bn3(conv3) + identity), one fused pass
        self.downsample = None
        if downsample:
            self.downsample = nn.Sequential(_conv(cin, cout, 1, stride=stride), _bn(cout))

    def _forward_pro(self, x, bng):
        """conv1 (statistics) -> [bn1 + ReLU inside conv2] -> [bn2 + ReLU inside conv3] -> bn3 (+
        residual / downsample BN) -> ReLU; every gradient tap of forward() kept."""
        ds = self.downsample
        if ds is None:
            tap = ResidualTap() if _FUSED_GRAD else None
            y1, p1 = conv1x1_bn_input(self.conv1, x, tap=tap, bn_grad=bng)
            xd = pd = None
        else:
            tap = None
            y1, p1, xa = conv1x1_bn_input(self.conv1, x, alias=True, bn_grad=bng)
            xd, pd = conv1x1_bn_input(ds[0], xa)
        x2, p2 = bn_relu_conv(self.bn1, self.conv2, y1, p1)
        x3, p3 = bn_relu_conv(self.bn2, self.conv3, x2, p2)
        if ds is None:
            return self.bn3(x3, x, stats=p3, res_tap=tap) if self.bn3._fast_ok(x3, x) else self.bn3(x3, x)
        if dual_bn_relu_ok(self.bn3, ds[1], x3, xd):
            return dual_bn_relu(self.bn3, x3, p3, ds[1], xd, pd)
        return self.bn3(x3, ds[1](xd, stats=pd), stats=p3)

    def _forward_pro2(self, x, bng):
        """bn2 + ReLU inside conv3 only: conv1 -> bn1 (apply pass) -> conv2 (statistics) ->
        [bn2 + ReLU inside conv3] -> bn3 (+ residual / downsample BN) -> ReLU."""
        ds = self.downsample
        if ds is None:
            tap = ResidualTap() if _FUSED_GRAD else None
            y = conv_bn(self.conv1, self.bn1, x, fuse=_FUSED_CONV, tap=tap, bn_grad=bng)
            xd = pd = None
        else:
            tap = None
            y1, p1, xa = conv1x1_bn_input(self.conv1, x, alias=True, bn_grad=bng)
            y = self.bn1(y1, stats=p1) if self.bn1._fast_ok(y1, None) else self.bn1(y1)
            xd, pd = conv1x1_bn_input(ds[0], xa)
        x2, p2 = conv2d_stats(self.conv2, y, fuse=_FUSED_WGRAD, bn_grad=bng)
        if p2 is None or not bn_relu_conv_ok(self.bn2, self.conv3, x2):  # (MIOpen forward: no statistics)
            y = self.bn2(x2, stats=p2) if p2 is not None and self.bn2._fast_ok(x2, None) else self.bn2(x2)
            if ds is None:
                return conv_bn(self.conv3, self.bn3, y, residual=x, fuse=_FUSED_CONV, res_tap=tap, bn_grad=bng)
            x3, p3 = conv1x1_bn_input(self.conv3, y, bn_grad=bng)
        else:
            x3, p3 = bn_relu_conv(self.bn2, self.conv3, x2, p2)
        if ds is None:
            return self.bn3(x3, x, stats=p3, res_tap=tap) if self.bn3._fast_ok(x3, x) else self.bn3(x3, x)
        if dual_bn_relu_ok(self.bn3, ds[1], x3, xd):
            return dual_bn_relu(self.bn3, x3, p3, ds[1], xd, pd)
        return self.bn3(x3, ds[1](xd, stats=pd), stats=p3)

    def forward(self, x):
        # Gradient of x = conv1's dgrad + the residual path's gradient.  Instead of autograd's add
        # (read 2, write 1 full-size tensors per block) conv1's dgrad epilogue sums them: the
        # identity residual's gradient (bn3's dy * ReLU bits) arrives through a ResidualTap, a
        # downsample branch's input gradient through an alias of x.
        # With every gradient path into x summed there, conv1's dgrad epilogue also reduces the
        # previous block's bn3 backward statistics, and conv3's those of bn2 (BNGradTap).
        ds = self.downsample
        bng = _FUSED_GRAD and _FUSED_BNGRAD
        if (_BN_PRO and bng and self.training and conv1x1_ok(self.conv1, x) and conv1x1_ok(self.conv3, x) and
                (ds is None or conv1x1_ok(ds[0], x)) and bn_relu_conv_ok(self.bn1, self.conv2, x) and
                bn_relu_conv_ok(self.bn2, self.conv3, x)):
            return self._forward_pro(x, bng)
        if (_BN_PRO2 and bng and self.training and conv1x1_ok(self.conv1, x) and conv1x1_ok(self.conv3, x) and
                (ds is None or conv1x1_ok(ds[0], x))):
            return self._forward_pro2(x, bng)
        if ds is None:
            tap = ResidualTap() if _FUSED_GRAD else None
            y = conv_bn(self.conv1, self.bn1, x, fuse=_FUSED_CONV, tap=tap, bn_grad=bng)
            idt = x
        elif (_FUSED_DUAL and self.training and self.bn1.training and conv1x1_ok(self.conv1, x) and
              conv1x1_ok(ds[0], x) and conv1x1_ok(self.conv3, x)):  # (conv3's input: bf16 channels-last too)
            # downsample block with the downsample BN folded into bn3's apply (_DualBNRelu)
            y1, p1, xa = conv1x1_bn_input(self.conv1, x, alias=True, bn_grad=bng)
            y = self.bn1(y1, stats=p1) if self.bn1._fast_ok(y1, None) else self.bn1(y1)
            xd, pd = conv1x1_bn_input(ds[0], xa)
            x2, p2 = conv2d_stats(self.conv2, y, fuse=_FUSED_WGRAD, bn_grad=bng)
            if bng and bn_pro_pays(self.bn2, self.conv3, x2, p2):  # measured per layer
                x3, p3 = bn_relu_conv(self.bn2, self.conv3, x2, p2)
            else:
                y = self.bn2(x2, stats=p2) if p2 is not None and self.bn2._fast_ok(x2, None) else self.bn2(x2)
                x3, p3 = conv1x1_bn_input(self.conv3, y, bn_grad=bng)
            if dual_bn_relu_ok(self.bn3, ds[1], x3, xd):
                return dual_bn_relu(self.bn3, x3, p3, ds[1], xd, pd)
            return self.bn3(x3, ds[1](xd, stats=pd), stats=p3)
        else:
            if _FUSED_GRAD:
                y, xa = conv_bn(self.conv1, self.bn1, x, fuse=_FUSED_CONV, alias=True, bn_grad=bng)
            else:
                y, xa = conv_bn(self.conv1, self.bn1, x, fuse=_FUSED_CONV), x
            tap = None
            idt = conv_bn(ds[0], ds[1], xa, fuse=_FUSED_CONV)
        if _FUSED_PRO:
            y = conv2d(self.conv2, y, fuse=_FUSED_WGRAD)
            if bn_relu_conv1x1_ok(self.bn2, self.conv3, y):
                # bn2's apply happens in conv3's operand prologue: its output is never written
                return bn_relu_conv_bn(self.bn2, self.conv3, self.bn3, y, residual=idt, res_tap=tap)
            y = self.bn2(y)
        else:
            # bn1's output only feeds conv2: its backward reduction rides conv2's input-gradient GEMM
            x2, p2 = conv2d_stats(self.conv2, y, fuse=_FUSED_WGRAD, bn_grad=bng)
            if (bng and self.training and _FUSED_CONV and conv1x1_ok(self.conv3, x2) and
                    bn_pro_pays(self.bn2, self.conv3, x2, p2)):
                # bn2 + ReLU in conv3's operand prologue (this layer measured faster that way)
                x3, p3 = bn_relu_conv(self.bn2, self.conv3, x2, p2)
                return self.bn3(x3, idt, stats=p3, res_tap=tap) if self.bn3._fast_ok(x3, idt) else self.bn3(x3, idt)
            if p2 is not None and self.bn2.training and self.bn2._fast_ok(x2, None):
                y = self.bn2(x2, stats=p2)
            else:
                y = self.bn2(x2)
        return conv_bn(self.conv3, self.bn3, y, residual=idt, fuse=_FUSED_CONV, res_tap=tap, bn_grad=bng)


class BasicBlock(nn.Module):
    expansion = 1

    def __init__(self, cin, width, stride=1, downsample=False):
        super().__init__()
        self.conv1 = _conv(cin, width, 3, stride=stride)
        self.bn1 = _bn(width, relu=True)
        self.conv2 = _conv(width, width, 3)
        self.bn2 = _bn(width, relu=True)
        self.downsample = None
        if downsample:
            self.downsample = nn.Sequential(_conv(cin, width, 1, stride=stride), _bn(width))

    def forward(self, x):
        idt = x if self.downsample is None else self.downsample(x)
        y = conv2d_bn(self.conv1, self.bn1, x, fuse=_FUSED_WGRAD)
        return conv2d_bn(self.conv2, self.bn2, y, residual=idt, fuse=_FUSED_WGRAD)


class ResNet(nn.Module):
    def __init__(self, block, layers, num_classes=1000, width=64, zero_init_residual=True):
        super().__init__()
        self.conv1 = nn.Conv2d(3, width, 7, stride=2, padding=3, bias=False)
        self.bn1 = _bn(width, relu=True)
        self.maxpool = MaxPool2d(3, stride=2, padding=1, fused=_FUSED_POOL)
        cin = width
        stages = []
        for i, n in enumerate(layers):
            w = width * (2 ** i)
            blocks = []
            for j in range(n):
                stride = 2 if (j == 0 and i > 0) else 1
                ds = j == 0 and (stride != 1 or cin != w * block.expansion)
                blocks.append(block(cin, w, stride=stride, downsample=ds))
                cin = w * block.expansion
            stages.append(nn.Sequential(*blocks))
        self.num_stages = len(stages)
        for i, st in enumerate(stages):
            setattr(self, f"layer{i + 1}", st)
        self.fc = Linear(cin, num_classes)  # hipps.ops.nn.Linear: reads the bf16 weight shadow
        for m in self.modules():
            if isinstance(m, nn.Conv2d):
                nn.init.kaiming_normal_(m.weight, mode="fan_out", nonlinearity="relu")
            elif isinstance(m, nn.BatchNorm2d):
                nn.init.ones_(m.weight)
                nn.init.zeros_(m.bias)
        if zero_init_residual:
            for m in self.modules():
                if isinstance(m, Bottleneck):
                    nn.init.zeros_(m.bn3.weight)
                elif isinstance(m, BasicBlock):
                    nn.init.zeros_(m.bn2.weight)

    def forward(self, x):
        if _FUSED_STEM_BWD and stem_block_ok(self.conv1, self.bn1, self.maxpool, x):
            x = stem_block(self.conv1, self.bn1, self.maxpool, x)
        else:
            y, part = conv2d_stats(self.conv1, x, fuse=_FUSED_STEM)
            x = bn_relu_maxpool(self.bn1, self.maxpool, y, part if _FUSED_STEM_POOL else None)
        for i in range(self.num_stages):
            x = getattr(self, f"layer{i + 1}")(x)
        x = global_avg_pool(x)
        return self.fc(x)


def resnet50(num_classes=1000, **kw):
    return ResNet(Bottleneck, [3, 4, 6, 3], num_classes=num_classes, **kw)


def resnet18(num_classes=1000, **kw):
    return ResNet(BasicBlock, [2, 2, 2, 2], num_classes=num_classes, **kw)


def resnet_tiny(num_classes=10, **kw):
    """A 2-stage toy ResNet for CPU tests (same block code as ResNet-50)."""
    return ResNet(Bottleneck, [1, 1], num_classes=num_classes, width=8, **kw)
