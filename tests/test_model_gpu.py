"""End-to-end GPU checks: fused HIP path vs the eager fp32 path of the same model, and the
hipGraph step engine vs eager steps."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _mlm(vocab=500, L=96, latents=64, c=64, layers=2, sa=2):
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    return LitMaskedLanguageModel(vocab_size=vocab, max_seq_len=L,
                                  optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                  num_latents=latents, num_latent_channels=c, num_encoder_layers=layers,
                                  num_encoder_self_attention_layers_per_block=sa).cuda()


def _grads(m):
    return {n: p.grad.detach().clone() for n, p in m.named_parameters() if p.grad is not None}


def test_mlm_fused_matches_eager():
    from perceiver_io_amd import ops

    torch.manual_seed(0)
    lit = _mlm()
    m = lit.model
    ids = torch.randint(3, 500, (6, 96), device="cuda")
    pad = torch.zeros(6, 96, dtype=torch.bool, device="cuda")
    pad[2, 60:] = True
    xm, lab = m.masking(ids, pad)
    with ops.backend("torch"):
        l_ref = m.loss(ids, pad, labels=lab, x_masked=xm)
        l_ref.backward()
    g_ref = _grads(m)
    m.zero_grad()
    with ops.backend("hip"):
        l_hip = m.loss(ids, pad, labels=lab, x_masked=xm)
        l_hip.backward()
    g_hip = _grads(m)
    assert abs(l_hip.item() - l_ref.item()) < 2e-2 * abs(l_ref.item())
    gmax = max(g.abs().max().item() for g in g_ref.values())
    for n, g in g_ref.items():
        assert n in g_hip, n
        err = (g_hip[n] - g).abs().max().item()
        assert err < 3e-2 * gmax, (n, err, gmax)


def test_image_classifier_fused_matches_eager():
    from perceiver_io_amd import ops
    from perceiver_io_amd.tasks import LitImageClassifier

    torch.manual_seed(1)
    lit = LitImageClassifier(image_shape=(28, 28, 1), num_classes=10,
                             optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                             num_latents=32, num_latent_channels=128, num_encoder_layers=2,
                             num_encoder_self_attention_layers_per_block=2, num_decoder_cross_attention_heads=1).cuda()
    x = torch.randn(4, 28, 28, 1, device="cuda")
    y = torch.randint(0, 10, (4,), device="cuda")
    outs = []
    for be in ("torch", "hip"):
        lit.zero_grad()
        with ops.backend(be):
            loss, _ = lit.step((x, y))
            loss.backward()
        outs.append((loss.item(), _grads(lit)))
    (l0, g0), (l1, g1) = outs
    assert abs(l0 - l1) < 2e-2 * abs(l0)
    gmax = max(g.abs().max().item() for g in g0.values())
    for n, g in g0.items():
        assert (g1[n] - g).abs().max().item() < 3e-2 * gmax, n


def test_image_classifier_replicated_flat_grads_match_eager():
    """Separate q/k/v projections (Cin ≠ C) with the flat space's replicated accumulators."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops.optim import FlatParameterSpace
    from perceiver_io_amd.tasks import LitImageClassifier

    torch.manual_seed(2)
    lit = LitImageClassifier(image_shape=(28, 28, 1), num_classes=10,
                             optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                             num_latents=32, num_latent_channels=128, num_encoder_layers=2,
                             num_encoder_self_attention_layers_per_block=1, num_decoder_cross_attention_heads=1).cuda()
    x = torch.randn(4, 28, 28, 1, device="cuda")
    y = torch.randint(0, 10, (4,), device="cuda")
    with ops.backend("torch"):
        loss, _ = lit.step((x, y))
        loss.backward()
    g0 = _grads(lit)
    flat = FlatParameterSpace(lit.parameters(), replicate=True)
    assert flat.grad_rep is not None
    flat.zero_grad()
    with ops.backend("hip"):
        loss, _ = lit.step((x, y))
        loss.backward()
    flat.fold()
    g1 = _grads(lit)
    gmax = max(g.abs().max().item() for g in g0.values())
    for n, g in g0.items():
        assert (g1[n] - g).abs().max().item() < 3e-2 * gmax, n


def test_graph_engine_matches_eager_steps():
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    torch.manual_seed(2)
    ids = torch.randint(3, 500, (4, 96), device="cuda")
    pad = torch.zeros(4, 96, dtype=torch.bool, device="cuda")
    states = []
    for graph in (False, True):
        torch.manual_seed(3)
        lit = _mlm()
        opt = FusedAdamW(lit.model.parameters(), lr=1e-3)
        gen_state = torch.cuda.get_rng_state()
        eng = StepEngine(lambda b: lit.model.loss(b[1], b[2]), opt, device="cuda", graph=graph, warmup_eager=1)
        torch.manual_seed(4)
        losses = [eng.step((None, ids, pad)).item() for _ in range(4)]
        states.append((losses, [p.detach().clone() for p in lit.model.parameters()]))
        del gen_state
    (la, pa), (lb, pb) = states
    # masking RNG streams differ between eager and replay, so compare trajectories loosely
    assert all(abs(a - b) < 0.5 for a, b in zip(la, lb)), (la, lb)
    assert all(torch.isfinite(p).all() for p in pb)
