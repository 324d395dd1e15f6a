"""Replayed steps return their loss through the update kernel's loss ring (CPU, closure graphs).

``StepEngine`` replays hand back ``loss_ring[slot]`` (written by the captured AdamW kernel from
``hyper[7]``) instead of cloning the graph's static loss after every replay.  Pinned here: the
returned losses equal the eager path's bitwise and each stays valid while later steps overwrite
the static output.
"""
import pytest
import torch

V, L = 101, 64


def _fused_on_cpu(monkeypatch):
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops import emulation, ext

    monkeypatch.setattr(ext, "_mod", emulation)
    monkeypatch.setattr(ops, "use_hip", lambda t: True)


def _model():
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    torch.manual_seed(0)
    return LitMaskedLanguageModel(vocab_size=V, max_seq_len=L,
                                  optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                  num_latents=64, num_latent_channels=64, num_encoder_layers=2,
                                  num_encoder_self_attention_layers_per_block=1).model


def _batches(model, steps):
    out = []
    for s in range(steps):
        g = torch.Generator().manual_seed(10 + s)
        x = torch.randint(3, V, (2, L), generator=g)
        pad = torch.zeros(2, L, dtype=torch.bool)
        xm, lab = model.masking(x, pad, generator=torch.Generator().manual_seed(77 + s))
        out.append((x, pad, lab, xm))
    return out


def _run(graph, steps=5, ring_view=True):
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    model = _model()
    opt = FusedAdamW(model.parameters(), lr=1e-2, eps=0.1, weight_decay=0.01)

    def loss_fn(b):
        x, pad, lab, xm = b
        return model.loss(x, pad, labels=lab, x_masked=xm)

    eng = StepEngine(loss_fn, opt, graph=graph, warmup_eager=1, graph_impl="closure" if graph else None)
    data = _batches(model, steps)
    losses, snap = [], []
    for s in range(steps):
        out = eng.step(data[s], ring_view=ring_view)
        losses.append(out)
        snap.append(float(out))
    return eng, losses, snap


def test_replayed_losses_from_the_ring_equal_eager(monkeypatch):
    _fused_on_cpu(monkeypatch)
    _, eager, eager_snap = _run(False)
    eng, graph, graph_snap = _run(True)
    assert eng.replays >= 3 and eng._loss_ring is not None
    assert graph_snap == eager_snap  # bitwise: the closure replay runs the same arithmetic
    # every returned loss still holds its own step's value after the later steps
    assert [float(t) for t in graph] == graph_snap
    # the replayed steps' losses are ring slots, not copies of the static output
    assert all(t.data_ptr() != graph[-1].data_ptr() for t in graph[1:-1])


def test_default_step_returns_an_independent_loss(monkeypatch):
    """Without ring_view the caller owns its loss tensor (a copy, like an eager step's): a later
    step's update kernel rewriting the ring slot cannot change it."""
    _fused_on_cpu(monkeypatch)
    eng, graph, snap = _run(True, ring_view=False)
    assert eng.replays >= 3
    assert all(t._base is None or t._base is not eng._loss_ring for t in graph)
    eng._loss_ring.fill_(-1.0)  # what LOSS_RING later steps would do to every slot
    assert [float(t) for t in graph] == snap
