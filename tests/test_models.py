"""Model semantics on CPU: checkpoint key layout, adapters, masking, encoder
weight sharing, MLM loss parity with the full-logits reference path, fused-executor parity
through the kernel emulation."""
import math

import pytest
import torch

from perceiver_io_amd import ops
from perceiver_io_amd.models import (ClassificationOutputAdapter, ImageInputAdapter, PerceiverDecoder, PerceiverEncoder,
                                     PerceiverIO, PerceiverMLM, SemanticSegOutputAdapter, TextInputAdapter, TextMasking,
                                     TextOutputAdapter)


def mnist_model(latents=32, c=128, layers=3, sa=3):
    enc = PerceiverEncoder(ImageInputAdapter((28, 28, 1), 32), (latents, c), layers, num_self_attention_layers_per_block=sa)
    dec = PerceiverDecoder(ClassificationOutputAdapter(10, num_output_channels=c), (latents, c), num_cross_attention_heads=1)
    return PerceiverIO(enc, dec)


def mlm_model(v=300, L=64, n=16, c=64, layers=2, sa=2):
    enc = PerceiverEncoder(TextInputAdapter(v, L, c), (n, c), layers, num_self_attention_layers_per_block=sa)
    dec = PerceiverDecoder(TextOutputAdapter(v, L, c), (n, c))
    return PerceiverMLM(enc, dec, TextMasking(v))


def test_state_dict_layout_image():
    keys = set(mnist_model().state_dict())
    # separate q/k/v projection weights in the image encoder cross-attention (Cin != C)
    assert "0.layer_1.0.0.module.attention.attention.q_proj_weight" in keys
    assert "0.layer_1.0.0.module.attention.attention.k_proj_weight" in keys
    assert "0.layer_1.0.0.module.attention.attention.in_proj_bias" in keys
    assert "0.layer_1.0.0.module.q_norm.weight" in keys and "0.layer_1.0.0.module.kv_norm.bias" in keys
    assert "0.layer_1.0.1.module.0.weight" in keys and "0.layer_1.0.1.module.3.bias" in keys
    assert "0.layer_1.1.2.0.module.norm.weight" in keys
    assert "0.layer_1.1.2.0.module.attention.attention.in_proj_weight" in keys
    assert "0.layer_n.1.0.1.module.1.weight" in keys
    assert "0.input_adapter.position_encoding" in keys and "0.latent" in keys
    assert "1.output" in keys and "1.output_adapter.linear.weight" in keys
    assert "1.cross_attention.0.module.attention.attention.in_proj_weight" in keys
    assert "1.cross_attention.1.module.3.weight" in keys
    assert not any("in_proj_weight" in k and "layer_1.0.0" in k for k in keys)


def test_state_dict_layout_mlm_and_aliases():
    m = mlm_model()
    keys = set(m.state_dict())
    assert "encoder.input_adapter.text_embedding.weight" in keys
    assert "encoder.input_adapter.pos_encoding" in keys
    assert "encoder.layer_1.0.0.module.attention.attention.in_proj_weight" in keys
    assert "decoder.output_adapter.linear.bias" in keys
    io = PerceiverIO(m.encoder, m.decoder)
    assert io.encoder is io[0] and io.decoder is io[1]  # defect D3
    assert set(io.state_dict()) == {k.replace("encoder.", "0.", 1).replace("decoder.", "1.", 1) for k in keys}


def test_param_counts_match_survey():
    # SURVEY §6.3 parameter counts (MNIST 32x128: 904,086; MLM 64x64 vocab 10003 L 512: 1,738,643)
    assert sum(p.numel() for p in mnist_model().parameters()) == 904_086
    m = mlm_model(v=10003, L=512, n=64, c=64, layers=3, sa=6)
    assert sum(p.numel() for p in m.parameters()) == 1_738_643


def test_fourier_encoding_layout():
    ad = ImageInputAdapter((28, 28, 1), 32)
    assert ad.num_input_channels == 1 + 2 * (2 * 32 + 1)
    pe = ad.position_encoding
    assert pe.shape == (784, 130)
    # positions first (row-major ij grid in [-1, 1]); then sin for dim0 bands, sin dim1, cos dim0, cos dim1
    assert torch.allclose(pe[0, :2], torch.tensor([-1.0, -1.0]))
    assert torch.allclose(pe[27, :2], torch.tensor([-1.0, 1.0]))
    f0 = torch.linspace(1.0, 14.0, 32)
    p = pe[5, 0]
    assert torch.allclose(pe[5, 2:34], torch.sin(math.pi * p * f0), atol=1e-5)
    assert torch.allclose(pe[5, 66:98], torch.cos(math.pi * p * f0), atol=1e-5)
    x = torch.randn(2, 28, 28, 1)
    y = ad(x)
    assert y.shape == (2, 784, 131) and torch.equal(y[:, :, 0], x.reshape(2, -1))
    with pytest.raises(ValueError):
        ad(torch.randn(2, 27, 28, 1))


def test_text_adapter_and_masking_semantics():
    torch.manual_seed(0)
    ad = TextInputAdapter(100, 16, 8)
    ids = torch.randint(0, 100, (3, 10))
    y = ad(ids)
    assert torch.allclose(y, ad.text_embedding.weight[ids] * math.sqrt(8) + ad.pos_encoding[:10])
    mk = TextMasking(1000)
    x = torch.randint(3, 1000, (64, 512))
    x[:, -50:] = 0
    x[:, :5] = 1  # UNK never selected
    pad = x == 0
    x0 = x.clone()
    xm, lab = mk(x, pad)
    assert torch.equal(x, x0)  # out of place (defect D4)
    sel = lab != -100
    assert not sel[pad].any() and not sel[:, :5].any()
    frac = sel.float().sum() / (~pad & (x != 1)).float().sum()
    assert abs(frac.item() - 0.15) < 0.01
    masked = (xm == 2) & sel
    assert abs(masked.float().sum().item() / sel.float().sum().item() - 0.8) < 0.03
    assert torch.equal(lab[sel], x[sel]) and torch.equal(xm[~sel], x[~sel])
    rnd = sel & (xm != 2) & (xm != x)
    assert rnd.any() and (xm[rnd] >= 3).all() and (xm[rnd] < 1000).all()
    kept = sel & (xm == x)  # the 10 % left unchanged
    assert abs(kept.float().sum().item() / sel.float().sum().item() - 0.1) < 0.02


def test_masking_counter_state_and_generator():
    """The device-resident counter advances per call (fresh masks, as on every replay of a
    captured step); an explicit generator reproduces a masking and leaves the state alone."""
    from perceiver_io_amd.ops import masking

    masking.reset_mask_state()
    torch.manual_seed(11)
    mk = TextMasking(500)
    x = torch.randint(3, 500, (8, 256))
    st = masking.mask_state(x.device)
    c0 = int(st[1])
    _, l1 = mk(x)
    _, l2 = mk(x)
    assert int(st[1]) == c0 + 2 and not torch.equal(l1, l2)
    masking.reset_mask_state()
    torch.manual_seed(11)
    torch.randint(3, 500, (8, 256))  # the same generator draws as before the first state
    _, l1b = mk(x)
    assert torch.equal(l1, l1b)  # torch.manual_seed reproduces the state's seed
    g1, g2 = torch.Generator().manual_seed(3), torch.Generator().manual_seed(3)
    c1 = int(masking.mask_state(x.device)[1])
    a = mk(x, generator=g1)
    b = mk(x, generator=g2)
    assert torch.equal(a[0], b[0]) and torch.equal(a[1], b[1])
    assert int(masking.mask_state(x.device)[1]) == c1


def test_encoder_weight_sharing():
    enc = PerceiverEncoder(TextInputAdapter(50, 16, 32), (8, 32), 4, num_self_attention_layers_per_block=1)
    layers = enc.layers()
    assert len(layers) == 4 and layers[1] is layers[2] is layers[3] is enc.layer_n


def test_decoder_latent_shape_check():
    dec = PerceiverDecoder(ClassificationOutputAdapter(5, num_output_channels=16), (8, 16))
    with pytest.raises(ValueError):
        dec(torch.randn(2, 7, 16))
    assert dec(torch.randn(2, 8, 16)).shape == (2, 5)


def test_semantic_seg_adapter_identity():
    ad = SemanticSegOutputAdapter(3, num_outputs=4, num_output_channels=8)
    x = torch.randn(2, 4, 8)
    assert ad(x) is x


def test_all_masked_rows_are_zero_not_nan():
    q = torch.randn(2, 4, 16)
    k = torch.randn(2, 6, 16)
    pad = torch.zeros(2, 6, dtype=torch.bool)
    pad[0] = True
    o = ops.attention.mha_core(q, k, k, 4, key_padding_mask=pad)
    assert torch.isfinite(o).all() and o[0].abs().max() == 0


def test_mlm_loss_matches_full_logit_reference():
    torch.manual_seed(1)
    m = mlm_model()
    x = torch.randint(3, 300, (4, 64))
    pad = torch.zeros(4, 64, dtype=torch.bool)
    pad[1, 40:] = True
    xm, lab = m.masking(x, pad)
    fast = m.loss(x, pad, labels=lab, x_masked=xm)
    with ops.backend("reference"):
        ref = m.loss(x, pad, labels=lab, x_masked=xm)
        logits, _ = m(xm, pad, masking=False)
    full = torch.nn.functional.cross_entropy(logits.transpose(1, 2), lab, ignore_index=-100)
    assert torch.allclose(fast, ref, atol=1e-5) and torch.allclose(fast, full, atol=1e-5)


@pytest.mark.parametrize("mask_p", [0.5, 0.9])
def test_mlm_loss_capacity_follows_mask_p(mask_p):
    """Capacities derive from TextMasking.mask_p: at high masking rates every selected position
    still reaches the loss (no silent truncation), and the persistent overflow flag stays clear."""
    from perceiver_io_amd.ops import mlm_head

    torch.manual_seed(5)
    m = mlm_model()
    m.masking.mask_p = mask_p
    x = torch.randint(3, 300, (4, 64))
    pad = torch.zeros(4, 64, dtype=torch.bool)
    pad[2, 50:] = True
    xm, lab = m.masking(x, pad)
    assert (lab != -100).float().mean() > 0.6 * mask_p
    mlm_head.check_overflow(reset=True)
    fast = m.loss(x, pad, labels=lab, x_masked=xm)
    logits, _ = m(xm, pad, masking=False)
    full = torch.nn.functional.cross_entropy(logits.transpose(1, 2), lab, ignore_index=-100)
    assert torch.allclose(fast, full, atol=1e-5)
    assert mlm_head.check_overflow() is False


def test_mlm_capacity_overflow_fails_loudly():
    from perceiver_io_amd.ops import mlm_head

    mlm_head.check_overflow(reset=True)
    labels = torch.full((2, 32), -100, dtype=torch.long)
    labels[:, :20] = 7  # 40 selected positions
    mlm_head.compact_rows(labels, 16)
    with pytest.raises(RuntimeError, match="capacity"):
        mlm_head.check_overflow(reset=True)
    assert mlm_head.check_overflow() is False  # reset cleared it


def test_reference_backend_matches_nn_multihead_attention():
    torch.manual_seed(2)
    from perceiver_io_amd.models.blocks import MultiHeadAttention

    mha = MultiHeadAttention(32, 48, 4, 0.0)
    ref = torch.nn.MultiheadAttention(32, 4, kdim=48, vdim=48, batch_first=True)
    ref.load_state_dict(mha.attention.state_dict())
    q, kv = torch.randn(2, 5, 32), torch.randn(2, 7, 48)
    pad = torch.zeros(2, 7, dtype=torch.bool)
    pad[1, 4:] = True
    want = ref(q, kv, kv, key_padding_mask=pad)[0]
    assert torch.allclose(mha(q, kv, pad), want, atol=1e-5)
    with ops.backend("reference"):
        assert torch.allclose(mha(q, kv, pad), want, atol=1e-6)


@pytest.mark.parametrize("slab", [True, False])
@pytest.mark.parametrize("kind", ["mlm", "image", "image128", "image128_materialised"])
def test_fused_executor_matches_eager_via_emulation(kind, slab, monkeypatch):
    """image128: head dim 32, the encoder cross-attention over implicit K/V (attention_pe.hip);
    image128_materialised: the same with the K/V tensor written by pe_proj_fwd."""
    monkeypatch.setattr(ops.fused, "WGRAD_SLAB", slab)
    monkeypatch.setattr(ops.fused, "PE_IMPLICIT", kind != "image128_materialised")
    kind = kind.replace("_materialised", "")
    torch.manual_seed(3)
    if kind == "mlm":
        m = mlm_model()
        x = torch.randint(3, 300, (3, 64))
        pad = torch.zeros(3, 64, dtype=torch.bool)
        pad[2, 30:] = True
        enc = m.encoder
    elif kind == "image128":  # head dim 32: cross-attention bwd fused into the PE reductions
        m = mnist_model(latents=16, c=128, layers=3, sa=1)
        x = torch.randn(2, 28, 28, 1)
        pad = None
        enc = m.encoder
    else:
        m = mnist_model(latents=16, c=64, layers=2, sa=1)
        x = torch.randn(2, 28, 28, 1)
        pad = None
        enc = m.encoder
    ref = enc(x, pad)[0]
    fused = ops.fused.encoder_forward(enc, x, pad)
    w = torch.randn_like(ref)
    (ref * w).sum().backward()
    g_ref = {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None}
    enc.zero_grad()
    (fused * w).sum().backward()
    assert (fused - ref).abs().max() < 0.03 * ref.abs().max()
    gmax = max(g.abs().max() for g in g_ref.values())
    for n, p in enc.named_parameters():
        if n in g_ref:
            assert (p.grad - g_ref[n]).abs().max() < 0.03 * gmax, n


@pytest.mark.parametrize("latents", [16, 64])
def test_cross_self_attention_boundary_fusion(latents, monkeypatch):
    """Layer-boundary fusion between the encoder's cross-attention layers and self-attention
    blocks, both ways: a cross layer runs the next block's LN1/QKV in its post-attention kernel
    and that block hands the LN1/QKV backward back to it; with 64 latents (the fused layer
    kernel's shape) a block's last kernel also computes the next cross layer's LN + query
    projection, whose backward comes back to the block.  Same outputs / gradients as unfused."""
    monkeypatch.setattr(ops.fused, "WGRAD_SLAB", True)
    # the attention-backward fusion of 64-latent blocks changes which dQKV are bf16 (its own test:
    # tests/test_models.py test_chain_fused_attention_plumbing_emulated)
    monkeypatch.setattr(ops.fused, "CHAIN_ATT", False)
    torch.manual_seed(4)
    m = mlm_model(n=latents, layers=3, sa=2)
    enc = m.encoder
    x = torch.randint(3, 300, (3, 64))
    pad = torch.zeros(3, 64, dtype=torch.bool)
    pad[1, 40:] = True
    emu = ops.emulation
    calls = {}

    class Counting:  # the executor's kernel calls (not the emulation's internal compositions)
        def __getattr__(self, name):
            calls[name] = calls.get(name, 0) + 1
            return getattr(emu, name)

    w = None
    res = []
    for fuse in (False, True):
        with monkeypatch.context() as mp:
            mp.setattr(ops.fused, "kernels", lambda t: Counting())
            if not fuse:
                mp.setattr(ops.fused, "sa_block_lookahead", lambda block, rows, *a: None)
                mp.setattr(ops.fused, "cross_q_lookahead", lambda cross, src, **kw: None)
            calls.clear()
            enc.zero_grad(set_to_none=True)
            out = ops.fused.encoder_forward(enc, x, pad)
            if w is None:
                w = torch.randn_like(out)
            (out * w).sum().backward()
            res.append((out.detach(), {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None},
                        dict(calls)))
    (o0, g0, c0), (o1, g1, c1) = res
    # 3 cross → block boundaries (+ 2 block → cross boundaries with the fused layer kernel)
    k = 3 + (2 if latents == 64 else 0)
    assert c0["ln_linear_fwd"] - c1["ln_linear_fwd"] == k, (c0, c1)
    assert c1["ln_linear_post_attn_bwd"] - c0.get("ln_linear_post_attn_bwd", 0) == k, (c0, c1)
    torch.testing.assert_close(o1, o0, rtol=1e-5, atol=1e-5)
    assert set(g0) == set(g1)
    for n in g0:
        torch.testing.assert_close(g1[n], g0[n], rtol=1e-4, atol=1e-5 * (g0[n].abs().max().item() + 1e-6), msg=n)


@pytest.mark.parametrize("slab", [False, True])
def test_fused_executor_replicated_gradients_fold_to_eager(slab, monkeypatch):
    """Flat parameter space with 8-way replicated gradient accumulators for the fused layers:
    after fold() the gradients equal the eager ones, and non-layer parameters are untouched
    by the replica mechanism.  With per-tile slabs (slab=True) the layer gradients bypass the
    replicas and land in the flat gradient through slab_reduce."""
    from perceiver_io_amd.ops.optim import FlatParameterSpace

    monkeypatch.setattr(ops.fused, "WGRAD_SLAB", slab)
    torch.manual_seed(4)
    m = mlm_model()
    x = torch.randint(3, 300, (3, 64))
    pad = torch.zeros(3, 64, dtype=torch.bool)
    pad[1, 40:] = True
    enc = m.encoder
    ref = enc(x, pad)[0]
    w = torch.randn_like(ref)
    (ref * w).sum().backward()
    g_ref = {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None}
    flat = FlatParameterSpace(enc.parameters(), with_shadow=False, replicate=True)
    assert flat.grad_rep is not None and flat.n_rep > 0
    rep_params = [p for p in flat.params if getattr(p, "_pio_grad_rep", None) is not None]
    assert rep_params and all(getattr(p, "_pio_replicate", False) for p in rep_params)
    flat.zero_grad()
    fused = ops.fused.encoder_forward(enc, x, pad)
    (fused * w).sum().backward()
    if not slab:
        assert flat.grad_rep.abs().sum() > 0  # layer kernels accumulated into the replicas
    else:
        assert flat.grad_rep.abs().sum() == 0 and flat.grad.abs().sum() > 0
    flat.fold()
    assert flat.grad_rep.abs().sum() == 0
    gmax = max(g.abs().max() for g in g_ref.values())
    for n, p in enc.named_parameters():
        if n in g_ref:
            assert (p.grad - g_ref[n]).abs().max() < 0.03 * gmax, n


def check_factored_pe_projection(K, device, channels, B=3, M=120, O=64, tol=2e-3):
    """ops/fused.py _pe_proj_fwd/_pe_proj_bwd (csrc/pe_proj.hip: per-step PE GEMM + per-sample
    epilogue + one streaming backward pass) against fp32 autograd of LayerNorm + Linear over the
    materialised [pixels ‖ PE] rows (reference adapter.py:106-109, model.py:89-99)."""
    import torch.nn.functional as F

    g = torch.Generator().manual_seed(channels)
    kin = channels + 40
    pe = torch.zeros(M, (kin + 7) // 8 * 8)
    pe[:, channels:kin] = torch.rand(M, kin - channels, generator=g) * 2 - 1
    pix = torch.randn(B * M, channels, generator=g)
    lnw = 1 + 0.3 * torch.randn(kin, generator=g)
    lnb = 0.3 * torch.randn(kin, generator=g)
    W = torch.randn(O, kin, generator=g) / kin ** 0.5
    bias = 0.3 * torch.randn(O, generator=g)
    dy = torch.randn(B * M, O, generator=g)
    t = [v.double().requires_grad_() for v in (lnw, lnb, W, bias)]
    full = pe[:, :kin].repeat(B, 1).double()
    full[:, :channels] += pix.double()
    y = F.linear(F.layer_norm(full, (kin,), t[0], t[1], 1e-5), t[2], t[3])
    y.backward(dy.double())
    dev = [v.to(device) for v in (pix, pe, lnw, lnb, W, bias, dy)]
    yk, mean, rstd = ops.fused._pe_proj_fwd(K, *dev[:6])
    assert (yk.float().cpu().double() - y.detach()).abs().max() < 1e-2 * y.abs().max()
    got = ops.fused._pe_proj_bwd(K, dev[6], dev[0], mean, rstd, dev[1], dev[2], dev[3], dev[4], M)
    for name, a, ref in zip(("dW", "db", "dln_w", "dln_b"), got, (t[2].grad, t[3].grad, t[0].grad, t[1].grad)):
        err = (a.cpu().double() - ref).abs().max() / ref.abs().max()
        assert err < tol, (name, err.item())


@pytest.mark.parametrize("channels", [1, 3, 4])
def test_factored_pe_projection_matches_autograd(channels):
    from perceiver_io_amd.ops import emulation

    check_factored_pe_projection(emulation, "cpu", channels)


def test_classifier_loss_matches_logits_cross_entropy():
    """PerceiverIO.loss (the fused-head entry point) equals cross_entropy of the logits, value and
    gradients, for image and text classifiers (CPU: the eager path; GPU coverage in
    tests/test_model_gpu.py)."""
    import torch.nn.functional as F

    from perceiver_io_amd.models import ClassificationOutputAdapter

    torch.manual_seed(6)
    m = mnist_model(latents=8, c=64, layers=2, sa=2)
    x = torch.randn(3, 28, 28, 1)
    y = torch.tensor([1, 7, 3])
    ref = F.cross_entropy(m(x).float(), y)
    ref.backward()
    g = {n: p.grad.clone() for n, p in m.named_parameters() if p.grad is not None}
    m.zero_grad()
    out = m.loss(x, y)
    out.backward()
    torch.testing.assert_close(out, ref)
    for n, p in m.named_parameters():
        if n in g:
            torch.testing.assert_close(p.grad, g[n], msg=n)
    assert isinstance(m.decoder.output_adapter, ClassificationOutputAdapter)


def test_chain_fused_attention_plumbing_emulated(monkeypatch):
    """64-latent blocks (``ops.fused.CHAIN_ATT``): the executor hands each boundary kernel the
    layer below's Q|K|V, LSE and a bf16 dQKV buffer and skips that layer's attention-backward
    launch (emulated kernels; the HIP kernel is compared in tests/test_attn_bwd_selfattn_gpu.py):
    same forward, gradients within the bf16 rounding of the handed-on dQKV, and one
    attention-backward launch per block instead of one per layer."""
    monkeypatch.setattr(ops.fused, "WGRAD_SLAB", True)
    torch.manual_seed(5)
    m = mlm_model(n=64, layers=3, sa=3)
    enc = m.encoder
    x = torch.randint(3, 300, (2, 64))
    pad = torch.zeros(2, 64, dtype=torch.bool)
    pad[1, 40:] = True
    emu = ops.emulation
    calls = {}

    class Counting:  # not the emulation module itself: the executor takes the kernel paths
        def __getattr__(self, name):
            calls[name] = calls.get(name, 0) + 1
            return getattr(emu, name)

    w = None
    res = []
    for flag in (False, True):
        with monkeypatch.context() as mp:
            mp.setattr(ops.fused, "kernels", lambda t: Counting())
            mp.setattr(ops.fused, "CHAIN_ATT", flag)
            calls.clear()
            enc.zero_grad(set_to_none=True)
            out = ops.fused.encoder_forward(enc, x, pad)
            if w is None:
                w = torch.randn_like(out)
            (out * w).sum().backward()
            res.append((out.detach(), {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None},
                        dict(calls)))
    (o0, g0, c0), (o1, g1, c1) = res
    torch.testing.assert_close(o1, o0, rtol=0, atol=0)
    # 3 blocks × 3 layers + 3 cross layers: 12 attention-backward launches unfused; fused, the 3
    # cross layers' and one self-attention layer's (the decoder-side block's last layer, whose
    # post-attention backward is not a chain kernel) remain
    assert (c0["attn_bwd"], c1["attn_bwd"]) == (12, 4), (c0["attn_bwd"], c1["attn_bwd"])
    assert set(g0) == set(g1)
    for n in g0:
        e = ((g1[n] - g0[n]).norm() / (g0[n].norm() + 1e-12)).item()
        assert e < 2e-2, (n, e)
