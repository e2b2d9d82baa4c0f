"""Transformer models for BASELINE configs 4 and 5 (random init, synthetic tokens).

  bert-base   BertModel layout (12 x 768, 12 heads, FFN 3072, vocab 30522, 512 positions, pooler)
              = 109,482,240 params + a tied-decoder MLM head; the query / key /
              value projections are one fused [2304, 768] Linear per layer (175 tensors instead
              of the 199 of separate q / k / v -- same parameter count and math).
              Config 4 ("BERT-base async PS, variable-size per-layer grad buckets").
  llama3-8b   Llama-3 8B (32 x 4096, 32 q / 8 kv heads, SwiGLU 14336, RMSNorm, RoPE theta 5e5,
              vocab 128256) = 8.03 B params.  Config 5 ("Llama-3 8B pure-DP async PS").  The
              q / k / v and gate / up projections are fused Linears (same parameters and math).
  *-tiny      same code, small widths, for CPU tests.

Attention is ``hipps.ops.nn.attention`` (csrc/attn.hip: MFMA flash attention, forward and a
deterministic backward, causal + grouped-query heads for Llama, key padding for BERT) on the
[B, S, H, hd] views of the projection outputs (no transposes); the
projections and MLPs are ``hipps.ops.nn.Linear`` (per shape hipBLASLt or the hipps gemm2 cores,
reading the engine's bf16 weight shadow, fp32 weight gradients written directly, the residual add
in the output projections' epilogue; plain ``nn.Linear`` behaviour without a shadow).  The loss
is the fused bf16 cross-entropy (csrc/xent.hip), the norms csrc/ln.hip (LayerNorm / RMSNorm), the
Llama SwiGLU gate and RoPE csrc/act.hip.  These models exercise the PS engine's bucketing /
codec / transport at 100 M - 8 B parameters (BASELINE configs 4 and 5).
"""
from __future__ import annotations

import math
from dataclasses import dataclass

import torch
import torch.nn as nn
import torch.nn.functional as F

from hipps.ops import nn as hnn


def _ln(mod: nn.LayerNorm, x: torch.Tensor, colsum_dx: bool = False) -> torch.Tensor:
    """LayerNorm on the autocast dtype: PyTorch's kernel reads bf16, computes in fp32 and writes
    bf16, where autocast's fp32 policy for layer_norm would cast the activation up, write fp32 and
    cast it back down for the next GEMM (two extra passes per norm, fp32 residual adds)."""
    if x.is_cuda and torch.is_autocast_enabled():
        dt = torch.get_autocast_dtype("cuda")
        with torch.autocast("cuda", enabled=False):
            xd = x.to(dt)
            if len(mod.normalized_shape) == 1 and hnn.layer_norm_ok(xd, mod.weight, mod.bias):
                return hnn.layer_norm(xd, mod.weight, mod.bias, mod.eps, colsum_dx)  # csrc/ln.hip
            return F.layer_norm(xd, mod.normalized_shape, mod.weight.to(dt), mod.bias.to(dt), mod.eps)
    return mod(x)


# ------------------------------------------------------------------------------------- BERT
@dataclass
class BertConfig:
    vocab: int = 30522
    hidden: int = 768
    layers: int = 12
    heads: int = 12
    ffn: int = 3072
    max_pos: int = 512
    type_vocab: int = 2
    eps: float = 1e-12


class BertLayer(nn.Module):
    def __init__(self, c: BertConfig):
        super().__init__()
        self.heads = c.heads
        # the query / key / value projections as ONE [3 * hidden, hidden] weight (+ [3 * hidden]
        # bias): same parameters and math as three Linears, one GEMM each way instead of three,
        # and the input gradient comes out of one GEMM (no two autograd adds per layer)
        self.qkv = hnn.Linear(c.hidden, 3 * c.hidden)
        self.attn_out = hnn.Linear(c.hidden, c.hidden)
        self.attn_ln = nn.LayerNorm(c.hidden, eps=c.eps)
        self.inter = hnn.Linear(c.hidden, c.ffn)
        self.out = hnn.Linear(c.ffn, c.hidden)
        self.out_ln = nn.LayerNorm(c.hidden, eps=c.eps)
        # bf16 W^T copies (refreshed with the shadow) for the input-gradient GEMMs that carry an
        # epilogue: qkv's and inter's add the residual's gradient, out's the GELU backward
        hnn.mark_transposed_reader(self.qkv.weight, self.inter.weight, self.out.weight)

    def forward(self, x, mask=None):
        B, S, D = x.shape
        h = self.heads

        link = hnn.ResidualLink()  # x's gradient from attn_out's residual joins qkv's input-gradient GEMM
        qkv = self.qkv(x, link=link).view(B, S, 3, h, D // h)
        if mask is None or (torch.is_tensor(mask) and mask.dtype == torch.int32 and mask.dim() == 1):
            # the packed [B, S, 3, H, hd] projection straight into the hipps flash-attention
            # kernels (csrc/attn.hip); ``mask`` may be the int32 [B] key lengths of a padded batch
            a = hnn.attention_qkv(qkv, kv_len=mask)
        else:
            q, k, v = (t.transpose(1, 2) for t in qkv.unbind(2))
            a = F.scaled_dot_product_attention(q, k, v, attn_mask=mask).transpose(1, 2)
        a = a.reshape(B, S, D)
        # residual adds ride in the output projections (GEMM epilogue / hipBLASLt C)
        # (colsum_dx: the LayerNorm backward also sums its dx -- attn_out's / out's bias gradient)
        x = _ln(self.attn_ln, self.attn_out(a, residual=x, link=link), colsum_dx=True)
        # intermediate -> GELU -> output (+ x) as one node: GELU in the GEMM epilogues both ways
        return _ln(self.out_ln, hnn.gelu_mlp(x, self.inter, self.out, residual_x=True), colsum_dx=True)


class Bert(nn.Module):
    def __init__(self, c: BertConfig = BertConfig(), mlm: bool = True):
        super().__init__()
        self.c = c
        self.word = nn.Embedding(c.vocab, c.hidden)
        self.pos = nn.Embedding(c.max_pos, c.hidden)
        self.tok_type = nn.Embedding(c.type_vocab, c.hidden)
        self.emb_ln = nn.LayerNorm(c.hidden, eps=c.eps)
        self.layers = nn.ModuleList([BertLayer(c) for _ in range(c.layers)])
        self.pooler = hnn.Linear(c.hidden, c.hidden)
        self.mlm = mlm
        if mlm:
            self.mlm_dense = hnn.Linear(c.hidden, c.hidden)
            self.mlm_ln = nn.LayerNorm(c.hidden, eps=c.eps)
            self.mlm_bias = nn.Parameter(torch.zeros(c.vocab))
            hnn.mark_shadow_reader(self.word.weight, self.mlm_bias)  # the tied decoder's hnn.linear
        self.apply(self._init)

    @staticmethod
    def _init(m):
        if isinstance(m, (nn.Linear, nn.Embedding)):
            nn.init.normal_(m.weight, std=0.02)
        if isinstance(m, nn.Linear) and m.bias is not None:
            nn.init.zeros_(m.bias)

    def forward(self, ids, labels=None, kv_len=None):
        """``kv_len``: optional int32 [B] valid lengths of a right-padded batch (key padding mask)."""
        B, S = ids.shape
        if hnn.bert_embed_ok(ids, self.word.weight, self.pos.weight, self.tok_type.weight):
            # one gather-add pass, deterministic table gradients (csrc/embed.hip); type ids all 0
            x = hnn.bert_embed(ids, self.word.weight, self.pos.weight, self.tok_type.weight)
        else:
            pos = torch.arange(S, device=ids.device)
            x = self.word(ids) + self.pos(pos)[None] + self.tok_type(torch.zeros_like(ids))
        x = _ln(self.emb_ln, x)
        for layer in self.layers:
            x = layer(x, kv_len)
        pooled = torch.tanh(self.pooler(x[:, 0]))
        if not self.mlm:
            return x, pooled
        h = _ln(self.mlm_ln, F.gelu(self.mlm_dense(x)))
        logits = hnn.linear(h, self.word.weight, self.mlm_bias)  # tied decoder
        if labels is None:
            return logits
        return hnn.cross_entropy(logits, labels, ignore_index=-100)


# ------------------------------------------------------------------------------------- Llama
@dataclass
class LlamaConfig:
    vocab: int = 128256
    dim: int = 4096
    layers: int = 32
    heads: int = 32
    kv_heads: int = 8
    ffn: int = 14336
    eps: float = 1e-5
    theta: float = 500000.0
    max_seq: int = 8192


class RMSNorm(nn.Module):
    def __init__(self, d, eps):
        super().__init__()
        self.weight = nn.Parameter(torch.ones(d))
        self.eps = eps

    def forward(self, x, add=None):
        """RMSNorm(x); with ``add``, returns (x + add, RMSNorm(x + add)) -- the residual add of the
        block before folded into this norm (one fused pass each way on the device)."""
        if add is not None:
            if x.is_cuda and torch.is_autocast_enabled() and hnn.add_rms_norm_ok(x, add, self.weight):
                return hnn.add_rms_norm(x, add, self.weight, self.eps)
            x = x + add
            return x, self(x)
        if x.is_cuda and torch.is_autocast_enabled() and hnn.rms_norm_ok(x, self.weight):
            # csrc/ln.hip: reads the fp32 residual stream directly, writes bf16 (no cast kernels)
            return hnn.rms_norm(x, self.weight, self.eps)
        if x.is_cuda:
            # one fused kernel (aten._fused_rms_norm, fp32 math) on the activation dtype instead of
            # six eager ops over an fp32 copy
            dt = torch.get_autocast_dtype("cuda") if torch.is_autocast_enabled() else x.dtype
            with torch.autocast("cuda", enabled=False):
                return F.rms_norm(x.to(dt), (x.shape[-1],), self.weight.to(dt), self.eps)
        xf = x.float()
        return (xf * torch.rsqrt(xf.pow(2).mean(-1, keepdim=True) + self.eps)).to(x.dtype) * self.weight.to(x.dtype)


def _rope(x, cos, sin):
    """Rotary embedding of interleaved pairs; cos / sin are fp32 [S, hd/2].  One fused HIP pass
    (hipps.ops.nn.rope) for bf16 device activations, the eager composition otherwise."""
    if hnn.rope_ok(x, cos):
        return hnn.rope(x, cos, sin)
    c, s_ = cos[None, :x.shape[1], None, :].to(x.dtype), sin[None, :x.shape[1], None, :].to(x.dtype)
    x1, x2 = x[..., ::2], x[..., 1::2]
    return torch.stack((x1 * c - x2 * s_, x1 * s_ + x2 * c), dim=-1).flatten(-2)


class LlamaBlock(nn.Module):
    def __init__(self, c: LlamaConfig):
        super().__init__()
        self.c = c
        hd = c.dim // c.heads
        # q | k | v as ONE [(heads + 2 kv_heads) * hd, dim] projection and the SwiGLU gate | up as
        # ONE [2 ffn, dim] projection: the same parameters and math as wq / wk / wv and w1 / w3,
        # one GEMM each way instead of three (two), and their input gradients come out of one
        # GEMM (no autograd adds of the slices' gradients)
        self.wqkv = hnn.Linear(c.dim, (c.heads + 2 * c.kv_heads) * hd, bias=False)
        self.wo = hnn.Linear(c.heads * hd, c.dim, bias=False)
        self.w13 = hnn.Linear(c.dim, 2 * c.ffn, bias=False)
        self.w2 = hnn.Linear(c.ffn, c.dim, bias=False)
        self.attn_norm = RMSNorm(c.dim, c.eps)
        self.ffn_norm = RMSNorm(c.dim, c.eps)

    def forward(self, x, cos, sin, y=None):
        """Returns (x', y') with the block's output = x' + y': the residual add of each branch is
        deferred into the norm that reads it next (RMSNorm(x, add=...)), so ``y`` is the previous
        block's pending branch output (None for the first block)."""
        B, S, D = x.shape
        c = self.c
        hd = D // c.heads
        if y is None:
            h = self.attn_norm(x)
        else:
            x, h = self.attn_norm(x, add=y)
        y = self.wqkv(h)  # [B, S, (heads + 2 kv_heads) * hd]
        if hnn.rope_attention_packed_ok(y, cos, c.heads, c.kv_heads):
            # RoPE + causal GQA flash attention on the packed projection (csrc/act.hip, attn.hip)
            a = hnn.rope_attention_packed(y, cos, sin, c.heads, c.kv_heads)
        else:
            q, k, v = y.split([c.heads * hd, c.kv_heads * hd, c.kv_heads * hd], dim=-1)
            q = _rope(q.reshape(B, S, c.heads, hd).contiguous(), cos, sin)
            k = _rope(k.reshape(B, S, c.kv_heads, hd).contiguous(), cos, sin)
            a = hnn.attention(q, k, v.reshape(B, S, c.kv_heads, hd), causal=True)
        x, h = self.ffn_norm(x, add=self.wo(a.reshape(B, S, D)))
        return x, self.w2(hnn.swiglu_packed(self.w13(h)))


class Llama(nn.Module):
    def __init__(self, c: LlamaConfig = LlamaConfig()):
        super().__init__()
        self.c = c
        self.tok = nn.Embedding(c.vocab, c.dim)
        self.blocks = nn.ModuleList([LlamaBlock(c) for _ in range(c.layers)])
        self.norm = RMSNorm(c.dim, c.eps)
        self.head = hnn.Linear(c.dim, c.vocab, bias=False)
        for m in self.modules():
            if isinstance(m, (nn.Linear, nn.Embedding)):
                nn.init.normal_(m.weight, std=0.02)

    def rope_tables(self, S, device):
        """fp32 cos / sin [S, hd/2] (cached per length and device: built once, not every forward)."""
        key = (S, str(device))
        cache = self.__dict__.setdefault("_rope_cache", {})
        if key not in cache:
            hd = self.c.dim // self.c.heads
            inv = 1.0 / (self.c.theta ** (torch.arange(0, hd, 2, device=device, dtype=torch.float32) / hd))
            t = torch.arange(S, device=device, dtype=torch.float32)
            f = torch.outer(t, inv)
            cache[key] = (f.cos().contiguous(), f.sin().contiguous())
        return cache[key]

    def forward(self, ids, labels=None):
        B, S = ids.shape
        x = self.tok(ids)
        cos, sin = self.rope_tables(S, ids.device)
        y = None
        for b in self.blocks:
            x, y = b(x, cos, sin, y)
        logits = self.head(self.norm(x) if y is None else self.norm(x, add=y)[1])
        if labels is None:
            return logits
        return hnn.cross_entropy(logits, labels)


def build(name: str, **kw):
    name = name.lower()
    if name in ("bert", "bert-base", "bert_base"):
        return Bert(BertConfig(**kw))
    if name in ("bert-tiny", "bert_tiny"):
        return Bert(BertConfig(vocab=512, hidden=64, layers=2, heads=4, ffn=128, max_pos=64, **kw))
    if name in ("llama3-8b", "llama-3-8b", "llama3_8b"):
        return Llama(LlamaConfig(**kw))
    if name in ("llama3-1b", "llama-3.2-1b"):
        return Llama(LlamaConfig(dim=2048, layers=16, heads=32, kv_heads=8, ffn=8192, **kw))
    if name in ("llama-tiny", "llama_tiny"):
        return Llama(LlamaConfig(vocab=512, dim=64, layers=2, heads=4, kv_heads=2, ffn=128, max_seq=128, **kw))
    raise ValueError(f"unknown transformer {name!r}")
