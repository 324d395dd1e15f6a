"""Dropout on the fused path (reference ``perceiver/model.py:47-56`` residual dropout and
``:66-71`` attention-probability dropout), checked on CPU through the kernel emulation.

The fused kernels draw their masks from a counter-based hash of (device seed, call site,
element index) — ``csrc/common.h`` ``DropCfg`` / ``drop_key``; ``ops/emulation.py`` reproduces
the hash bit-exactly.  So a plain-PyTorch re-statement of the layer maths with the SAME masks
(``emulation.attn_drop_mask`` / ``row_drop_mask``) is an exact oracle for the fused layer's
outputs and gradients with dropout on.  The GPU tests (``test_kernels_gpu.py``) check the HIP
kernels against the same emulation.
"""
import math

import pytest
import torch
import torch.nn.functional as F

from perceiver_io_amd import ops
from perceiver_io_amd.models.blocks import cross_attention_layer, self_attention_block
from perceiver_io_amd.ops import emulation


def _ref_layer(layer, xq, xkv, pad, seed, site, p):
    """Residual(attention) → Residual(mlp) with the kernels' masks applied explicitly."""
    att, mlp = layer.attn, layer.mlp
    mha = att.attention.attention
    C, H = mha.embed_dim, mha.num_heads
    D = C // H
    if hasattr(att, "q_norm"):
        qn = F.layer_norm(xq, (C,), att.q_norm.weight, att.q_norm.bias, 1e-5)
        kvn = F.layer_norm(xkv, (xkv.shape[-1],), att.kv_norm.weight, att.kv_norm.bias, 1e-5)
    else:
        qn = kvn = F.layer_norm(xq, (C,), att.norm.weight, att.norm.bias, 1e-5)
    q = F.linear(qn, mha.q_weight(), mha.in_proj_bias[:C])
    k, v = F.linear(kvn, mha.kv_weight(), mha.in_proj_bias[C:]).split(C, dim=-1)
    B, Nq, Nk = k.shape[0], q.shape[1], k.shape[1]
    q = q.expand(B, -1, -1)
    xq = xq.expand(B, -1, -1)
    qh, kh, vh = (t.reshape(B, -1, H, D).transpose(1, 2) for t in (q, k, v))
    s = qh @ kh.transpose(-1, -2) / math.sqrt(D)
    if pad is not None:
        s = s.masked_fill(pad.view(B, 1, 1, Nk), float("-inf"))
    a = torch.softmax(s, -1)
    if p > 0:
        a = a * emulation.attn_drop_mask(seed, site, B, H, Nq, Nk, p)
    o = (a @ vh).transpose(1, 2).reshape(B, Nq, C)
    att_out = F.linear(o, mha.out_proj.weight, mha.out_proj.bias)
    if p > 0:
        att_out = att_out * emulation.row_drop_mask(seed, site, 0, B * Nq, C, p).view(B, Nq, C)
    y = xq + att_out
    f = mlp(y)
    if p > 0:
        f = f * emulation.row_drop_mask(seed, site, 1, B * Nq, C, p).view(B, Nq, C)
    return y + f


def _grads(mod):
    return {n: p.grad.clone() for n, p in mod.named_parameters() if p.grad is not None}


def _check(fused, ref, mods, w):
    assert fused.shape == ref.shape
    assert (fused - ref).abs().max() <= 0.03 * ref.abs().max()
    (ref * w).sum().backward()
    g_ref = [_grads(m) for m in mods]
    for m in mods:
        m.zero_grad()
    (fused * w).sum().backward()
    for m, gr in zip(mods, g_ref):
        for n, p in m.named_parameters():
            if n in gr:
                # per-tensor relative error (bf16 GEMM operands in the emulation)
                err = (p.grad - gr[n]).norm() / (gr[n].norm() + 1e-12)
                assert err < 0.03, (n, err.item())


@pytest.fixture
def fixed_seed(monkeypatch):
    seed = torch.tensor([0x1234_5678_9ABC_DEF], dtype=torch.int64)
    monkeypatch.setattr(ops.fused, "_seed", lambda p, device: seed if p > 0 else None)
    return seed


@pytest.mark.parametrize("p", [0.1, 0.4])
def test_fused_cross_layer_dropout_matches_masked_reference(p, fixed_seed):
    torch.manual_seed(0)
    C, Ckv, B, N, M = 64, 48, 3, 16, 40
    layer = cross_attention_layer(C, Ckv, 4, p).train()
    lat = torch.randn(1, N, C, requires_grad=True)
    xkv = torch.randn(B, M, Ckv)
    pad = torch.zeros(B, M, dtype=torch.bool)
    pad[1, 25:] = True
    fused = ops.fused.cross_attention_layer(layer, lat, xkv, pad)
    ref = _ref_layer(layer, lat, xkv, pad, fixed_seed, 0, p)
    _check(fused, ref, [layer], torch.randn_like(ref))


@pytest.mark.parametrize("p", [0.1, 0.3])
def test_fused_self_attention_block_dropout_matches_masked_reference(p, fixed_seed):
    torch.manual_seed(1)
    C, B, N = 64, 2, 32
    block = self_attention_block(3, C, 4, p).train()
    x = torch.randn(B, N, C)
    fused = ops.fused.self_attention_block(block, x)
    ref = x
    for i, layer in enumerate(block):  # layer i of the block uses site i of the block's seed
        ref = _ref_layer(layer, ref, ref, None, fixed_seed, i, p)
    _check(fused, ref, [block], torch.randn_like(ref))


def test_dropout_off_in_eval_and_at_p0():
    torch.manual_seed(2)
    C, B, N = 64, 2, 32
    block = self_attention_block(2, C, 4, 0.3)
    x = torch.randn(B, N, C)
    block.eval()
    a = ops.fused.self_attention_block(block, x)
    b = block(x)  # eager, eval: dropout is the identity
    assert (a - b).abs().max() < 0.03 * b.abs().max()
    for layer in block:
        layer.attn.attention.attention.dropout = 0.0
        for r in layer:
            r.dropout.p = 0.0
    block.train()
    assert torch.equal(ops.fused.self_attention_block(block, x), a)


def test_device_seed_is_drawn_per_call():
    """Two fused forwards draw two different device seeds (so masks change every step, also
    inside a replayed hipGraph where the draw is a graph node)."""
    s1, s2 = ops.fused._seed(0.1, torch.device("cpu")), ops.fused._seed(0.1, torch.device("cpu"))
    assert s1.dtype == torch.int64 and s1.numel() == 1 and not torch.equal(s1, s2)
    assert ops.fused._seed(0.0, torch.device("cpu")) is None


def test_encoder_pass_draws_one_seed_pool(monkeypatch):
    """Inside an encoder pass (ops.fused._encode) the fused calls take distinct slots of ONE drawn
    pool (one generator launch per pass, not per layer); every pass draws a fresh pool; outside a
    pass each call draws its own seed."""
    from perceiver_io_amd.models import PerceiverEncoder, TextInputAdapter

    torch.manual_seed(0)
    enc = PerceiverEncoder(TextInputAdapter(300, 64, 64), (16, 64), 3, num_self_attention_layers_per_block=2,
                           dropout=0.1).train()
    x = torch.randint(3, 300, (2, 64))
    draws = []
    real = torch.randint

    def counting(*a, **k):
        draws.append(1)
        return real(*a, **k)

    monkeypatch.setattr(torch, "randint", counting)
    seeds = []
    real_seed = ops.fused._seed

    def spy(p, device):
        s = real_seed(p, device)
        if s is not None:
            seeds.append(s.clone())
        return s

    monkeypatch.setattr(ops.fused, "_seed", spy)
    o1 = ops.fused.encoder_forward(enc, x)
    n1, s1 = len(draws), list(seeds)
    o2 = ops.fused.encoder_forward(enc, x)
    assert n1 == 1 and len(draws) == 2, (n1, len(draws))
    assert len(s1) >= 4 and len({int(t) for t in s1}) == len(s1)  # distinct slots
    assert not torch.equal(o1, o2)  # a fresh pool: different masks
    assert not ops.fused._SEED_POOL["armed"]
    ops.fused._seed(0.1, torch.device("cpu"))
    assert len(draws) == 3


def test_mask_statistics_and_hash_reproducibility():
    seed = torch.tensor([7], dtype=torch.int64)
    m = emulation.row_drop_mask(seed, 3, 0, 512, 64, 0.25)
    keep = (m > 0).float().mean().item()
    assert abs(keep - 0.75) < 0.01
    assert torch.allclose(m[m > 0], torch.full_like(m[m > 0], 1 / 0.75))
    assert torch.equal(m, emulation.row_drop_mask(seed, 3, 0, 512, 64, 0.25))
    assert not torch.equal(m, emulation.row_drop_mask(seed, 3, 1, 512, 64, 0.25))
    a = emulation.attn_drop_mask(seed, 0, 2, 4, 33, 70, 0.5)
    assert abs((a > 0).float().mean().item() - 0.5) < 0.02
