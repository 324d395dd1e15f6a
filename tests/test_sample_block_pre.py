"""The encoder cross-attention layer's post-attention half folded into the per-sample block after it
(ops/fused.py "want_pa" / "have_pa" / "bwd_pa"; csrc/sample_block.hip pre stage) and the next cross
layer's LN + query projection into the block before it ("want_q" / "have_q" / "bwd_q"; the post
stage), run on the CPU
through the kernel emulation with the per-sample block routing forced on (it needs CUDA tensors
otherwise): same outputs and gradients as the unfolded executor and as eager fp32, and the folded
layers launch no post-attention kernels of their own."""
import pytest
import torch

from perceiver_io_amd import ops
from perceiver_io_amd.models import (ClassificationOutputAdapter, ImageInputAdapter, PerceiverDecoder,
                                     PerceiverEncoder, PerceiverIO)


def _model(c, layers, sa, cross_heads=4):
    enc = PerceiverEncoder(ImageInputAdapter((28, 28, 1), 32), (32, c), layers, num_cross_attention_heads=cross_heads,
                           num_self_attention_layers_per_block=sa)
    dec = PerceiverDecoder(ClassificationOutputAdapter(10, num_output_channels=c), (32, c), num_cross_attention_heads=1)
    return PerceiverIO(enc, dec)


@pytest.mark.parametrize("c,cross_heads", [(64, 4), (128, 4), (128, 1)])
def test_cross_post_attention_folded_into_sample_block(c, cross_heads, monkeypatch):
    """cross_heads = 1: δ of the cross attention is not in the block's 4-head layout, no fold."""
    torch.manual_seed(c)
    enc = _model(c, 3, 2, cross_heads).encoder
    x = torch.randn(3, 28, 28, 1)
    ok = ops.fused._sample_block_ok
    monkeypatch.setattr(ops.fused, "_sample_block_ok", lambda specs, n, p, cuda: ok(specs, n, p, True))
    emu = ops.emulation
    calls = {}

    class Counting:  # the executor's kernel calls
        def __getattr__(self, name):
            calls[name] = calls.get(name, 0) + 1
            return getattr(emu, name)

    ref = enc(x, None)[0]
    w = torch.randn_like(ref)
    (ref * w).sum().backward()
    g_ref = {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None}
    res = []
    for fold in (False, True):
        with monkeypatch.context() as mp:
            mp.setattr(ops.fused, "kernels", lambda t: Counting())
            mp.setattr(ops.fused, "SB_PRE", fold)
            mp.setattr(ops.fused, "SB_POST", fold)
            calls.clear()
            enc.zero_grad(set_to_none=True)
            out = ops.fused.encoder_forward(enc, x, None)
            (out * w).sum().backward()
            res.append((out.detach(), {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None},
                        dict(calls)))
    (o0, g0, c0), (o1, g1, c1) = res
    assert c0.get("sb_fwd", 0) == 3 and c1.get("sb_fwd", 0) == 3, (c0, c1)
    # every cross layer is followed by a per-sample block: no post-attention kernels at all
    folded = 3 if cross_heads == 4 else 0
    assert c0.get("post_attn_fwd", 0) == 3 and c1.get("post_attn_fwd", 0) == 3 - folded, (c0, c1)
    assert c0.get("post_attn_bwd", 0) == 3 and c1.get("post_attn_bwd", 0) == 3 - folded, (c0, c1)
    # the query paths of the 2nd and 3rd cross layers run in the preceding blocks' kernels
    assert c0["ln_linear_fwd"] - c1["ln_linear_fwd"] == 2, (c0, c1)
    assert c0["ln_linear_bwd"] - c1["ln_linear_bwd"] == 2, (c0, c1)
    assert set(g0) == set(g1) == set(g_ref)
    torch.testing.assert_close(o1, o0, rtol=2e-3, atol=2e-3 * o0.abs().max().item())
    gmax = max(g.abs().max() for g in g_ref.values())
    assert (o1 - ref).abs().max() < 0.03 * ref.abs().max()
    for n in g0:
        assert (g1[n] - g0[n]).abs().max() < 0.01 * gmax, n
        assert (g1[n] - g_ref[n]).abs().max() < 0.03 * gmax, n


@pytest.mark.parametrize("c", [64, 128])
def test_decoder_kv_folded_into_last_sample_block(c, monkeypatch):
    """An image classifier's decoder K|V projection (LN_kv + the 2C-wide in-projection rows) runs
    in the encoder's last per-sample block both ways ("want_kv" → the post stage with N = 2C): same
    loss and gradients as the unfolded executor and eager fp32, one LN + projection kernel fewer
    each way; with a DDP ready point armed on the decoder input only the forward is folded."""
    from perceiver_io_amd.ops import emulation, ext
    from perceiver_io_amd.parallel import reducer as red_mod

    torch.manual_seed(c + 1)
    model = _model(c, 3, 2)
    x = torch.randn(3, 28, 28, 1)
    y = torch.tensor([1, 7, 3])
    ref = torch.nn.functional.cross_entropy(model(x), y)
    ref.backward()
    g_ref = {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None}
    ok = ops.fused._sample_block_ok
    monkeypatch.setattr(ops.fused, "_sample_block_ok", lambda specs, n, p, cuda: ok(specs, n, p, True))
    monkeypatch.setattr(ext, "_mod", emulation)
    monkeypatch.setattr(ops, "use_hip", lambda t: True)
    calls = {}

    class Counting:
        def __getattr__(self, name):
            calls[name] = calls.get(name, 0) + 1
            return getattr(emulation, name)

    monkeypatch.setattr(ops.fused, "kernels", lambda t: Counting())
    res = []
    for fold, armed in ((False, False), (True, False), (True, True)):
        with monkeypatch.context() as mp:
            mp.setattr(ops.fused, "SB_POST", fold)
            mp.setattr(red_mod, "ready_point_armed", lambda m, n: armed)
            mp.setattr("perceiver_io_amd.models.perceiver.ready_point_armed", lambda m, n: armed)
            calls.clear()
            model.zero_grad(set_to_none=True)
            loss = model.loss(x, y)
            loss.backward()
            res.append((loss.detach(), {n: p.grad.clone() for n, p in model.named_parameters() if p.grad is not None},
                        dict(calls)))
            assert ops.fused._LOOKAHEAD["bwd_q"] is None and ops.fused._LOOKAHEAD["have_q"] is None
    (l0, g0, c0), (l1, g1, c1), (l2, g2, c2) = res
    # unfolded: 2 next-cross query paths + the decoder's query and K/V paths
    assert c0["ln_linear_fwd"] - c1["ln_linear_fwd"] == 3, (c0, c1)
    assert c0["ln_linear_bwd"] - c1["ln_linear_bwd"] == 3, (c0, c1)
    assert c2["ln_linear_fwd"] == c1["ln_linear_fwd"] and c2["ln_linear_bwd"] == c1["ln_linear_bwd"] + 1, (c1, c2)
    gmax = max(g.abs().max() for g in g_ref.values())
    for l_, g_ in ((l1, g1), (l2, g2)):
        assert abs(l_.item() - l0.item()) < 2e-3 * max(1.0, abs(l0.item()))
        assert set(g_) == set(g0) == set(g_ref)
        for n in g0:
            assert (g_[n] - g0[n]).abs().max() < 0.01 * gmax, n
            assert (g_[n] - g_ref[n]).abs().max() < 0.03 * gmax, n
