"""LArTPC sparse execution (``models/lartpc.py``, ``data/lartpc.py``) against the dense reference
computation, and the coupled-L2 fused Adam of the experiment (CPU)."""
import pytest
import torch
import torch.nn.functional as F

from perceiver_io_amd.data.lartpc import sparse_collate
from perceiver_io_amd.data.synthetic import lartpc_event
from perceiver_io_amd.models.lartpc import LArPerceiver, accuracies, class_weights


def _events(n, size, seed=0):
    return [lartpc_event(seed * 1000 + i, size) for i in range(n)]


def test_sparse_collate_layout():
    ev = _events(3, 32)
    values, index, kmask, qidx, qlab = sparse_collate(ev, bucket=64)
    assert values.shape[1] % 64 == 0 and qidx.shape[1] % 64 == 0
    for i, (img, lab) in enumerate(ev):
        nz = torch.nonzero(img.reshape(-1) != 0).squeeze(1)
        n = len(nz)
        assert torch.equal(index[i, :n], nz) and not kmask[i, :n].any() and kmask[i, n:].all()
        assert torch.equal(values[i, :n, 0], img.reshape(-1)[nz])
        q = torch.nonzero(lab > 0).squeeze(1)  # background weight 0
        assert torch.equal(qidx[i, :len(q)], q) and torch.equal(qlab[i, :len(q)], lab[q])
        assert (qlab[i, len(q):] == -100).all()


@pytest.mark.parametrize("weights", [(0.0, 1.0, 1.0), (0.0, 1.0, 2.5)])
def test_sparse_loss_and_grads_match_dense(weights):
    """Encoder over the non-zero pixels only + decoder over the weighted pixels only == the
    reference's dense computation (all keys with zero pixels masked, all queries, weighted CE)."""
    torch.manual_seed(0)
    size = 32
    model = LArPerceiver(size)
    ev = _events(2, size, seed=3)
    w = class_weights("cpu", weights)
    img = torch.stack([e[0] for e in ev])
    lab = torch.stack([e[1] for e in ev])
    dense = F.cross_entropy(model(img), lab, weight=w)
    dense.backward()
    g_dense = {n: p.grad.clone() for n, p in model.perceiver.named_parameters()}
    model.zero_grad()
    loss, acc = model.sparse_loss(sparse_collate(ev, bucket=64, weights=weights), w)
    loss.backward()
    pred = model(img).argmax(1)
    for k, v in accuracies(pred, lab).items():
        assert abs(float(acc[k]) - float(v)) < 1e-6, k
    assert torch.allclose(loss, dense, rtol=1e-5, atol=1e-6), (float(loss), float(dense))
    for n, p in model.perceiver.named_parameters():
        gd, gs = g_dense[n], p.grad
        assert gs is not None, n
        tol = 1e-5 * max(1.0, float(gd.abs().max()))
        assert torch.allclose(gs, gd, atol=tol, rtol=1e-4), (n, float((gs - gd).abs().max()))
    # the 262,144-row (here 1,024) output-query table: only weighted pixels carry gradient
    out_grad = model.perceiver.decoder.output.grad
    hit = torch.zeros(size * size, dtype=torch.bool)
    for _, lb in ev:
        hit |= lb > 0
    assert (out_grad[~hit] == 0).all()


def test_sparse_logits_equal_dense_at_selected_pixels():
    torch.manual_seed(1)
    size = 32
    model = LArPerceiver(size).eval()
    ev = _events(2, size, seed=5)
    img = torch.stack([e[0] for e in ev])
    values, index, kmask, qidx, qlab = sparse_collate(ev, bucket=64)
    with torch.no_grad():
        dense = model(img).permute(0, 2, 1)  # (B, HW, 3)
        sp = model.sparse_logits(values, index, kmask, qidx)
    for i in range(2):
        m = qlab[i] != -100
        assert torch.allclose(sp[i][m], dense[i][qidx[i][m]], atol=1e-5)


def test_accuracies_match_reference_definition():
    pred = torch.tensor([0, 1, 2, 1, 2, 0])
    lab = torch.tensor([0, 1, 2, 2, -100, 1])
    acc = {k: float(v) for k, v in accuracies(pred, lab).items()}
    assert acc["acc"] == pytest.approx(2 / 4) and acc["acc1"] == pytest.approx(1 / 2)
    assert acc["acc2"] == pytest.approx(1 / 2)
    assert float(accuracies(pred, torch.full((6,), -100))["acc"]) == 0.0


def test_fused_adam_l2_matches_torch_adam_with_clip():
    """FusedAdam (coupled L2 decay, clip folded into the update) == clip_grad_norm_ + torch Adam."""
    from perceiver_io_amd.ops.optim import FusedAdam

    torch.manual_seed(2)
    ps = [torch.nn.Parameter(torch.randn(37, 5)), torch.nn.Parameter(torch.randn(11))]
    ref = [torch.nn.Parameter(p.detach().clone()) for p in ps]
    opt = FusedAdam(ps, lr=1e-2, weight_decay=1e-2, max_grad_norm=0.5)
    topt = torch.optim.Adam(ref, lr=1e-2, weight_decay=1e-2)
    for it in range(3):
        gs = [torch.randn_like(p) * (3.0 if it == 0 else 0.01) for p in ps]  # clip active, then not
        opt.flat.zero_grad()
        for p, g in zip(ps, gs):
            p.grad.copy_(g)
        opt.step()
        topt.zero_grad()
        for p, g in zip(ref, gs):
            p.grad = g.clone()
        torch.nn.utils.clip_grad_norm_(ref, 0.5)
        topt.step()
        for p, r in zip(ps, ref):
            assert torch.allclose(p.detach(), r.detach(), atol=1e-6, rtol=1e-5), (it, (p - r).abs().max())


def test_sparse_loss_fused_executor_emulated(monkeypatch):
    """The fused path (fused layers, pixel head + weighted CE kernels, row-gather backward) through
    the kernel emulation on the CPU equals the plain PyTorch path."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops import emulation, ext

    torch.manual_seed(3)
    size = 32
    model = LArPerceiver(size)
    ev = _events(3, size, seed=7)
    w = class_weights("cpu", (0.0, 1.0, 2.0))
    batch = sparse_collate(ev, bucket=64, weights=(0.0, 1.0, 2.0))
    loss_ref, acc_ref = model.sparse_loss(batch, w)
    loss_ref.backward()
    g_ref = {n: p.grad.clone() for n, p in model.perceiver.named_parameters()}
    model.zero_grad()
    monkeypatch.setattr(ext, "_mod", emulation)
    monkeypatch.setattr(ops, "use_hip", lambda t: True)
    loss, acc = model.sparse_loss(batch, w)
    loss.backward()
    assert abs(float(loss) - float(loss_ref)) < 2e-2 * float(loss_ref)
    for k in acc_ref:
        assert abs(float(acc[k]) - float(acc_ref[k])) < 0.05, k
    head = model.perceiver.decoder.output_adapter.linear
    for n, p in model.perceiver.named_parameters():
        gr = g_ref[n]
        if gr.norm() < 1e-4:  # e.g. the decoder query-LN affine at init (|g| ~ 1e-7): noise only
            assert (p.grad - gr).norm() < 1e-4, n
            continue
        err = float((p.grad - gr).norm() / gr.norm())
        # decoder + head (the new fused pieces: row gather, pixel CE) within 5 %; the encoder's
        # cross-attention query side is ill-conditioned in bf16 at random init (near-uniform
        # attention over ~1,000 keys; the GPU test bounds it by the emulation's own error)
        assert err < (5e-2 if n.startswith("1.") else 0.25), (n, err)
    assert head.weight.grad is not None and head.bias.grad is not None


def test_pixel_ce_emulation_matches_torch():
    from perceiver_io_amd.ops import emulation

    torch.manual_seed(4)
    h, W, b = torch.randn(50, 64), torch.randn(3, 64) * 0.2, torch.randn(3) * 0.1
    lab = torch.randint(0, 3, (50,))
    lab[::7] = -100
    wts = torch.tensor([0.0, 1.0, 2.5])
    stats, loss = emulation.pixel_ce_fwd(h, W, b, lab, wts)
    ref = F.cross_entropy(h @ W.t() + b, lab, weight=wts, ignore_index=-100)
    assert torch.allclose(loss, ref, atol=1e-6)
    hh, WW, bb = (t.clone().requires_grad_() for t in (h, W, b))
    F.cross_entropy(hh @ WW.t() + bb, lab, weight=wts, ignore_index=-100).backward()
    dH, dW, db = torch.empty_like(h), torch.zeros_like(W), torch.zeros_like(b)
    emulation.pixel_ce_bwd(h, W, b, lab, wts, torch.tensor([1.0]), stats, dH, dW, db)
    assert torch.allclose(dH, hh.grad, atol=1e-6)
    assert torch.allclose(dW, WW.grad, atol=1e-5)
    assert torch.allclose(db, bb.grad, atol=1e-6)
