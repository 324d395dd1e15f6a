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


def _rel(a, b):
    """per-tensor relative Frobenius error ‖a − b‖ / ‖b‖"""
    return ((a.float() - b.float()).norm() / (b.float().norm() + 1e-12)).item()


def _check_grads(g_hip, g_ref, tol=2e-2, floor=None):
    """every gradient tensor within ``tol`` of ITS OWN norm (small-gradient tensors — LN
    biases, latents, biases — are checked as strictly as the large ones).  ``floor``: per-tensor
    bf16 rounding floor (the kernel emulation's own error vs fp32), added twice to ``tol`` —
    a few tensors are ill-conditioned in bf16 (e.g. the decoder query-LN affine: its gradient
    is a sum of dQ = dS·(K − K̄) over near-identical keys, where bf16 keys lose most bits)."""
    bad = {}
    for n, g in g_ref.items():
        assert n in g_hip, n
        if g.norm() == 0:
            assert g_hip[n].norm() == 0, n
            continue
        e = _rel(g_hip[n], g)
        t = tol + (2 * floor[n] if floor is not None else 0.0)
        if e > t:
            bad[n] = (e, t)
    assert not bad, bad


class _emulated:
    """Run the fused executor on ops.emulation (fp32 maths, the kernels' bf16 rounding points
    and dropout hash) instead of the HIP extension, on the same GPU tensors."""

    def __enter__(self):
        from perceiver_io_amd import ops
        from perceiver_io_amd.ops import emulation, ext

        self.saved = (ext._mod, ops.fused.kernels)
        ext._mod = emulation
        ops.fused.kernels = lambda t: emulation
        return self

    def __exit__(self, *exc):
        from perceiver_io_amd import ops
        from perceiver_io_amd.ops import ext

        ext._mod, ops.fused.kernels = self.saved


def _three_way(mod, run, loss_tol=1e-2, tol=2e-2, jitter_run=None):
    """``run()`` → loss (backward inside) on: eager fp32 (reference maths), HIP kernels, and the
    kernels' emulation.  Checks HIP vs emulation per tensor at ``tol`` (kernel correctness) and
    HIP vs fp32 per tensor at ``tol`` + 2 × the emulation's own bf16 error (precision).

    ``jitter_run`` (optional): ``run`` on inputs perturbed by ~1e-6 relative.  The emulation's
    gradient change under that perturbation measures each tensor's conditioning: a gradient
    formed as a small difference of bf16-rounded terms (e.g. the decoder query-LN affine over
    near-identical latent keys, where a one-ulp flip of one key moves it by percent) changes by
    percent under ANY perturbation, so that change is added to the floor."""
    from perceiver_io_amd import ops

    res = {}
    for name in ("torch", "hip", "emu") + (("jit",) if jitter_run is not None else ()):
        mod.zero_grad()
        if name in ("emu", "jit"):
            with ops.backend("hip"), _emulated():
                loss = run() if name == "emu" else jitter_run()
        else:
            with ops.backend(name):
                loss = run()
        res[name] = (loss.item(), _grads(mod))
    (l0, g0), (l1, g1), (l2, g2) = res["torch"], res["hip"], res["emu"]
    assert abs(l1 - l0) < loss_tol * abs(l0), (l0, l1)
    assert abs(l1 - l2) < 1e-3 * abs(l2), (l1, l2)
    floor = {n: _rel(g2[n], g) for n, g in g0.items()}
    if jitter_run is not None:
        gj = res["jit"][1]
        floor = {n: f + _rel(gj[n], g2[n]) for n, f in floor.items()}
    _check_grads(g1, g2, tol=tol, floor=floor)
    _check_grads(g1, g0, tol=tol, floor=floor)


@pytest.mark.parametrize("latents,L,B", [(64, 96, 6), (512, 96, 6), (64, 2048, 2)])
def test_mlm_fused_matches_eager(latents, L, B):
    """(512 latents: the self-attention backward has 2 key blocks and query splits, whose
    accumulators the preceding kernel clears — csrc attn_bwd_zero_plan; L = 2048: ~300 selected
    positions per sequence, so the decoder's attention backward splits its queries and adds into
    dK / dV, which the decoder's post-attention backward clears on the way)"""
    from perceiver_io_amd import ops

    torch.manual_seed(0)
    lit = _mlm(latents=latents, L=L)
    m = lit.model
    ids = torch.randint(3, 500, (B, L), device="cuda")
    pad = torch.zeros(B, L, dtype=torch.bool, device="cuda")
    pad[B // 2, 2 * L // 3:] = True
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
    m.zero_grad()
    with ops.backend("hip"), _emulated():
        l_emu = m.loss(ids, pad, labels=lab, x_masked=xm)
        l_emu.backward()
    g_emu = _grads(m)
    assert abs(l_hip.item() - l_ref.item()) < 1e-2 * abs(l_ref.item())
    assert abs(l_hip.item() - l_emu.item()) < 1e-3 * abs(l_emu.item())
    # per-tensor bf16 noise floor: how far an independent bf16 implementation (the emulation)
    # lands from fp32; the kernels must be as close to fp32 AND to the emulation
    floor = {n: _rel(g_emu[n], g) for n, g in g_ref.items()}
    _check_grads(g_hip, g_emu, floor=floor)
    _check_grads(g_hip, g_ref, floor=floor)


@pytest.mark.parametrize("heads,shape,sa", [(1, (28, 28, 1), 2), (4, (28, 28, 1), 2), (4, (64, 64, 3), 2),
                                            (4, (28, 28, 1), 4)])
def test_image_classifier_fused_matches_eager(heads, shape, sa):
    """heads = 4 (head dim 32): the encoder cross-attention runs over implicit K/V
    (attention_pe.hip), both directions, the weight-shared layer_n applied twice.  sa = 4
    self-attention layers per block: past the per-sample block kernels' limits, the block runs
    on the layer-boundary kernels."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.tasks import LitImageClassifier

    torch.manual_seed(1)
    lit = LitImageClassifier(image_shape=shape, num_classes=10,
                             optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                             num_latents=32, num_latent_channels=128, num_encoder_layers=2 if heads == 1 else 3,
                             num_encoder_cross_attention_heads=heads,
                             num_encoder_self_attention_layers_per_block=sa, num_decoder_cross_attention_heads=1).cuda()
    x = torch.randn(4, *shape, device="cuda")
    y = torch.randint(0, 10, (4,), device="cuda")

    def run(xx=x):
        loss, _ = lit.step((xx, y))
        loss.backward()
        return loss

    xj = x * (1 + 1e-6 * torch.randn_like(x))
    _three_way(lit, run, jitter_run=lambda: run(xj))


@pytest.mark.parametrize("kind", ["image", "text"])
def test_classifier_fused_head_loss(kind):
    """PerceiverIO.loss through the fused CE head (ce_fwd / ce_bwd over the decoder rows, the
    query stream broadcast inside the fused decoder layer) vs the same loss in fp32 eager maths
    (= cross_entropy of the logits) and vs the kernels' emulation: loss and every gradient."""
    import torch.nn.functional as F

    from perceiver_io_amd import ops
    from perceiver_io_amd.tasks import LitImageClassifier, LitTextClassifier

    torch.manual_seed(2)
    opt = {"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}}
    if kind == "image":
        lit = LitImageClassifier(image_shape=(28, 28, 1), num_classes=10, optimizer_init=opt, num_latents=32,
                                 num_latent_channels=128, num_encoder_layers=2,
                                 num_encoder_self_attention_layers_per_block=2,
                                 num_decoder_cross_attention_heads=1).cuda()
        args = (torch.randn(6, 28, 28, 1, device="cuda"),)
        y = torch.randint(0, 10, (6,), device="cuda")
    else:
        lit = LitTextClassifier(num_classes=2, vocab_size=300, max_seq_len=64, optimizer_init=opt, num_latents=64,
                                num_latent_channels=64, num_encoder_layers=2,
                                num_encoder_self_attention_layers_per_block=2,
                                num_decoder_cross_attention_heads=1).cuda()
        ids = torch.randint(3, 300, (6, 64), device="cuda")
        pad = torch.zeros(6, 64, dtype=torch.bool, device="cuda")
        pad[2, 40:] = True
        args = (ids, pad)
        y = torch.randint(0, 2, (6,), device="cuda")
    m = lit.model
    with ops.backend("torch"):  # the fused head's value = cross_entropy of the logits
        ref = F.cross_entropy(m(*args).float(), y).item()
    assert abs(m.loss(args[0], y, *args[1:]).item() - ref) < 1e-2 * max(1.0, abs(ref))

    def run(a0=args[0]):
        loss = m.loss(a0, y, *args[1:])
        loss.backward()
        return loss

    jit = None
    if kind == "image":  # conditioning floor of the decoder query-LN affine (see _three_way)
        xj = args[0] * (1 + 1e-6 * torch.randn_like(args[0]))
        jit = lambda: run(xj)  # noqa: E731
    _three_way(m, run, jitter_run=jit)


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
    lit.zero_grad()
    with ops.backend("hip"), _emulated():
        loss, _ = lit.step((x, y))
        loss.backward()
    floor = {n: _rel(g, g0[n]) for n, g in _grads(lit).items()}
    lit.zero_grad()
    flat = FlatParameterSpace(lit.parameters(), replicate=True)
    assert flat.grad_rep is not None
    flat.zero_grad()
    with ops.backend("hip"):
        loss, _ = lit.step((x, y))
        loss.backward()
    flat.fold()
    g1 = _grads(lit)
    _check_grads(g1, g0, floor=floor)


def _fixed_mask_engine(lit, graph, ids, pad, lr=1e-3, warmup=1):
    """StepEngine whose loss replays ONE precomputed masking (no RNG inside the step)."""
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    m = lit.model
    with torch.no_grad():  # a fixed generator: every engine of a test sees the same masking
        xm, lab = m.masking(ids, pad, generator=torch.Generator(device="cuda").manual_seed(7))
    opt = FusedAdamW(m.parameters(), lr=lr)
    return StepEngine(lambda b: m.loss(b[1], b[2], labels=lab, x_masked=xm), opt, device="cuda", graph=graph,
                      warmup_eager=warmup)


def test_graph_engine_matches_eager_steps():
    """Replayed hipGraph steps vs eager steps from the same initial state with identical
    inputs and masks: losses and parameters agree to fp32-atomic reordering noise."""
    torch.manual_seed(2)
    ids = torch.randint(3, 500, (4, 96), device="cuda")
    pad = torch.zeros(4, 96, dtype=torch.bool, device="cuda")
    pad[1, 70:] = True
    states = []
    for graph in (False, True):
        torch.manual_seed(3)
        lit = _mlm()
        eng = _fixed_mask_engine(lit, graph, ids, pad)
        losses = [eng.step((None, ids, pad)).item() for _ in range(5)]
        states.append((losses, [p.detach().clone() for p in lit.model.parameters()]))
        if graph:
            assert eng.num_graphs == 1
    (la, pa), (lb, pb) = states
    # identical up to fp32-atomic summation order (which Adam's sign-like first steps amplify
    # for near-zero gradient elements); the deterministic mode test pins bitwise equality
    for a, b in zip(la, lb):
        assert abs(a - b) <= 5e-3 * abs(a), (la, lb)
    # per element, Adam turns pure-rounding-noise gradients (true value ≈ 0) into ±lr steps, so
    # the parameters are compared as a whole here; bitwise per-element equality is pinned by
    # the deterministic-mode test
    assert _rel(torch.cat([t.reshape(-1) for t in pb]), torch.cat([t.reshape(-1) for t in pa])) < 1e-2


def test_graph_engine_variable_shapes():
    """One captured graph per batch shape (LRU), each replayed with its own static buffers."""
    torch.manual_seed(5)
    lit = _mlm(L=128)
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    opt = FusedAdamW(lit.model.parameters(), lr=1e-3)
    eng = StepEngine(lambda b: lit.model.loss(b[1], b[2]), opt, device="cuda", graph=True, warmup_eager=0,
                     max_graphs=2)
    shapes = [(4, 64), (4, 128), (4, 64), (3, 64), (4, 128)]
    for b, L in shapes:
        ids = torch.randint(3, 500, (b, L), device="cuda")
        pad = torch.zeros(b, L, dtype=torch.bool, device="cuda")
        loss = eng.step((None, ids, pad))
        assert torch.isfinite(loss)
    assert eng.captures == 4 and eng.num_graphs == 2  # (4,128) was evicted by (3,64) and recaptured


def test_graph_replays_draw_fresh_dropout_masks():
    """Dropout under graph capture: with lr = 0 the parameters never change, so consecutive
    replays of one graph differ ONLY through the dropout masks — they must differ (seed slots
    restaged before each replay) — while at p = 0 they are bit-identical."""
    ids = torch.randint(3, 500, (4, 96), device="cuda")
    pad = torch.zeros(4, 96, dtype=torch.bool, device="cuda")
    for p in (0.0, 0.2):
        torch.manual_seed(6)
        lit = _mlm_dropout(p)
        eng = _fixed_mask_engine(lit, True, ids, pad, lr=0.0, warmup=0)
        losses = [eng.step((None, ids, pad)).item() for _ in range(4)]
        # the seeds are static slots of the graph, restaged with fresh values before each replay
        # (no generator kernel inside the graph)
        ent = next(iter(eng._graphs.values()))
        assert (ent.drop_seeds is not None) == (p > 0), ent.drop_seeds
        if p == 0.0:
            assert len(set(losses)) == 1, losses
        else:
            assert len(set(losses)) == 4, losses


def test_two_engines_keep_private_dropout_seed_pools():
    """Two step engines (e.g. two models trained in one process) capture dropout graphs: each
    captured graph reads its OWN static seed slots, so staging one engine's seeds before its
    replay cannot change the masks of the other's (interleaved replays, both still drawing fresh
    masks every step)."""
    ids = torch.randint(3, 500, (4, 96), device="cuda")
    pad = torch.zeros(4, 96, dtype=torch.bool, device="cuda")
    engs = []
    for s in (6, 7):
        torch.manual_seed(s)
        engs.append(_fixed_mask_engine(_mlm_dropout(0.2), True, ids, pad, lr=0.0, warmup=0))
    losses = [[], []]
    for _ in range(3):
        for k, e in enumerate(engs):
            losses[k].append(e.step((None, ids, pad)).item())
    pools = [next(iter(e._graphs.values())).drop_seeds[0] for e in engs]
    assert pools[0].data_ptr() != pools[1].data_ptr()
    assert all(len(set(ls)) == 3 for ls in losses), losses


def _mlm_dropout(p, **kw):
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    return LitMaskedLanguageModel(vocab_size=500, max_seq_len=96,
                                  optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                  num_latents=64, num_latent_channels=64, num_encoder_layers=2,
                                  num_encoder_self_attention_layers_per_block=2, dropout=p, **kw).cuda()


def test_dropout_fused_matches_masked_emulation_end_to_end(monkeypatch):
    """Whole MLM encoder with dropout 0.1 on the HIP kernels vs the same executor on the
    kernel emulation (bit-identical hashed masks, fp32 oracle maths)."""
    from perceiver_io_amd import ops

    seed = torch.tensor([123456789], dtype=torch.int64, device="cuda")
    monkeypatch.setattr(ops.fused, "_seed", lambda p, device: seed if p > 0 else None)
    torch.manual_seed(7)
    lit = _mlm_dropout(0.1)
    enc = lit.model.encoder.train()
    ids = torch.randint(3, 500, (4, 96), device="cuda")
    pad = torch.zeros(4, 96, dtype=torch.bool, device="cuda")
    pad[2, 50:] = True
    outs = []
    for K in ("hip", "emu"):
        enc.zero_grad()
        if K == "emu":
            monkeypatch.setattr(ops.fused, "kernels", lambda t: ops.emulation)
        z = ops.fused.encoder_forward(enc, ids, pad)
        w = torch.randn(z.shape, generator=torch.Generator(device="cuda").manual_seed(1), device="cuda")
        (z * w).sum().backward()
        outs.append((z.detach().clone(), _grads(enc)))
    (z1, g1), (z2, g2) = outs
    assert _rel(z1, z2) < 1e-2
    _check_grads(g1, g2, tol=3e-2)


def test_headline_shape_fused_matches_eager_fp32():
    """The benchmark configuration itself (B = 64, L = 512, 256 × 64 latents, 3 × (1 + 6)
    layers, vocab 10003): fused bf16 loss + gradients vs the eager fp32 path."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    torch.manual_seed(8)
    lit = LitMaskedLanguageModel(vocab_size=10003, max_seq_len=512,
                                 optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                 num_latents=256, num_latent_channels=64, num_encoder_layers=3,
                                 num_encoder_self_attention_layers_per_block=6).cuda()
    m = lit.model
    ids = torch.randint(3, 10003, (64, 512), device="cuda")
    pad = torch.zeros(64, 512, dtype=torch.bool, device="cuda")
    pad[::3, 400:] = True
    xm, lab = m.masking(ids, pad)

    def run():
        loss = m.loss(ids, pad, labels=lab, x_masked=xm)
        loss.backward()
        return loss

    _three_way(m, run, loss_tol=5e-3)


def _det_run(graph, steps=4, image=False):
    from perceiver_io_amd.ops.optim import FusedAdamW
    from perceiver_io_amd.train.engine import StepEngine

    torch.manual_seed(11)
    if image:
        from perceiver_io_amd.tasks import LitImageClassifier

        lit = LitImageClassifier(image_shape=(28, 28, 1), num_classes=10,
                                 optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                 num_latents=32, num_latent_channels=128, num_encoder_layers=3,
                                 num_encoder_self_attention_layers_per_block=2,
                                 num_decoder_cross_attention_heads=1).cuda()
        x = torch.randn(16, 28, 28, 1, device="cuda")
        y = torch.randint(0, 10, (16,), device="cuda")
        opt = FusedAdamW(lit.parameters(), lr=1e-3, max_grad_norm=0.5)
        eng = StepEngine(lambda b: lit.step(b)[0], opt, device="cuda", graph=graph, warmup_eager=1)
        batch = (x, y)
    else:
        lit = _mlm(L=96)
        ids = torch.randint(3, 500, (8, 96), device="cuda")
        pad = torch.zeros(8, 96, dtype=torch.bool, device="cuda")
        pad[3, 40:] = True
        m = lit.model
        with torch.no_grad():
            xm, lab = m.masking(ids, pad, generator=torch.Generator(device="cuda").manual_seed(7))
        opt = FusedAdamW(m.parameters(), lr=1e-3, max_grad_norm=0.5)
        eng = StepEngine(lambda b: m.loss(b[1], b[2], labels=lab, x_masked=xm), opt, device="cuda", graph=graph,
                         warmup_eager=1)
        batch = (None, ids, pad)
    losses = [eng.step(batch).item() for _ in range(steps)]
    return losses, [p.detach().clone() for p in lit.parameters()]


@pytest.mark.parametrize("image", [False, True])
def test_deterministic_mode_bitwise(image):
    """``--trainer.deterministic=true`` (reference trainer.yaml:57): with the
    atomics-free reductions two identical runs give bitwise-identical parameters, and a replayed
    hipGraph step equals the eager step bit for bit."""
    from perceiver_io_amd import ops

    ops.set_deterministic(True)
    torch.use_deterministic_algorithms(True, warn_only=True)
    try:
        la, pa = _det_run(True, image=image)
        lb, pb = _det_run(True, image=image)
        lc, pc = _det_run(False, image=image)
    finally:
        ops.set_deterministic(False)
        torch.use_deterministic_algorithms(False)
    assert la == lb, (la, lb)
    assert all(torch.equal(a, b) for a, b in zip(pa, pb))
    assert la == lc, (la, lc)
    assert all(torch.equal(a, c) for a, c in zip(pa, pc))


def test_lartpc_sparse_fused_matches_eager():
    """LArTPC sparse execution (non-zero keys, weighted queries, 1,300+ keys per sample with
    capacity padding masked) on the fused kernels vs eager fp32 vs the emulation.  Sparse ==
    dense is pinned on the CPU (tests/test_lartpc.py)."""
    from perceiver_io_amd.data.lartpc import sparse_collate
    from perceiver_io_amd.data.synthetic import lartpc_event
    from perceiver_io_amd.models.lartpc import LArPerceiver, class_weights

    torch.manual_seed(4)
    model = LArPerceiver(64).cuda()
    ev = [lartpc_event(i, 64) for i in range(3)]
    batch = tuple(t.cuda() for t in sparse_collate(ev, bucket=256))
    w = class_weights("cuda")
    _three_way(model.perceiver, lambda: model.sparse_loss(batch, w)[0])


def test_lartpc_dense_inference_fused_matches_eager():
    from perceiver_io_amd import ops
    from perceiver_io_amd.data.synthetic import lartpc_event
    from perceiver_io_amd.models.lartpc import LArPerceiver

    torch.manual_seed(5)
    model = LArPerceiver(64).cuda().eval()
    img = torch.stack([lartpc_event(10 + i, 64)[0] for i in range(2)]).cuda()
    with torch.no_grad():
        with ops.backend("torch"):
            ref = model(img)
        with ops.backend("hip"):
            out = model(img)
    assert _rel(out, ref) < 2e-2


def test_lartpc_run_graph_engine(tmp_path):
    """run.py on the fused graph path: sparse batches of varying capacity, FusedAdam (L2 + clip),
    plateau scheduler on the previous loss, validation, checkpoint."""
    import run

    ck = tmp_path / "ckpt"
    run.main(["--epochs", "1", "--events", "16", "--val-events", "4", "--size", "128", "--batch-size", "4",
              "--max-steps", "4", "--bucket", "256", "--log-dir", str(tmp_path / "runs"), "--ckpt-dir", str(ck),
              "--device", "cuda", "--workers", "0"])
    state = torch.load(ck / "model_0.ckpt", weights_only=True)
    assert all(torch.isfinite(v).all() for v in state["model_state_dict"].values() if v.is_floating_point())


def test_bf16_dqkv_handoff_is_bitwise_neutral(monkeypatch):
    """The self-attention backward stores dQKV as bf16 for the chain-layout boundary kernel
    (``ops.fused.BF16_DQKV``): that kernel rounds a fp32 dQKV to the same bf16 values itself, so
    the gradients are bitwise those of the fp32 hand-off (deterministic mode: no atomics)."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops import fused

    ops.set_deterministic(True)
    try:
        res = []
        for flag in (True, False):
            monkeypatch.setattr(fused, "BF16_DQKV", flag)
            torch.manual_seed(5)
            lit = _mlm(L=96, latents=128, sa=3)
            m = lit.model
            ids = torch.randint(3, 500, (8, 96), device="cuda")
            pad = torch.zeros(8, 96, dtype=torch.bool, device="cuda")
            pad[1, 50:] = True
            with torch.no_grad():
                xm, lab = m.masking(ids, pad, generator=torch.Generator(device="cuda").manual_seed(3))
            m.loss(ids, pad, labels=lab, x_masked=xm).backward()
            res.append(_grads(m))
    finally:
        ops.set_deterministic(False)
    a, b = res
    assert a.keys() == b.keys()
    for n in a:
        assert torch.equal(a[n], b[n]), n


@pytest.mark.parametrize("p", [0.0, 0.1])
def test_chain_fused_attention_backward_matches_separate(monkeypatch, p):
    """64-latent blocks (``ops.fused.CHAIN_ATT``): the boundary kernel that also runs the layer
    below's attention backward gives the gradients of the separate attention-backward launches
    (same kernels' maths, bf16 dQKV hand-off), with and without dropout."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops import fused

    seed = torch.tensor([24681357], dtype=torch.int64, device="cuda")
    monkeypatch.setattr(ops.fused, "_seed", lambda p_, device: seed if p_ > 0 else None)
    res = []
    for flag in (False, True):
        monkeypatch.setattr(fused, "CHAIN_ATT", flag)
        torch.manual_seed(6)
        lit = _mlm_dropout(p)
        m = lit.model.train()
        ids = torch.randint(3, 500, (6, 96), device="cuda")
        pad = torch.zeros(6, 96, dtype=torch.bool, device="cuda")
        pad[2, 60:] = True
        with torch.no_grad():
            xm, lab = m.masking(ids, pad, generator=torch.Generator(device="cuda").manual_seed(2))
        loss = m.loss(ids, pad, labels=lab, x_masked=xm)
        loss.backward()
        res.append((loss.item(), _grads(m)))
    (l0, g0), (l1, g1) = res
    assert l0 == l1
    _check_grads(g1, g0, tol=2e-2)
