"""Remaining SURVEY §2.1 components on CPU: the LArTPC experiment (run.py, #34) with its U-ResNet
(#35), tokenizer utilities (#21, #37), masked-token prediction (#20), and the fused executor's
bookkeeping that the GPU path relies on (deferred weight-gradient slab jobs, the self-attention
block node) through the kernel emulation."""
import os

import pytest
import torch

from perceiver_io_amd.ops import emulation
from perceiver_io_amd.ops import fused as F

REF_TOKENIZER = "/root/reference/.cache/imdb-tokenizer-10003.json"


def test_lartpc_run_cpu_smoke(tmp_path):
    """run.py end to end on a tiny synthetic event set: train steps, validation, reference-layout
    checkpoint ({'epoch', 'model_state_dict', 'optimizer_state_dict'}, run.py:278-281)."""
    import run

    ck = tmp_path / "ckpt"
    run.main(["--epochs", "1", "--events", "4", "--val-events", "2", "--size", "32", "--batch-size", "2",
              "--max-steps", "2", "--log-dir", str(tmp_path / "runs"), "--ckpt-dir", str(ck), "--device", "cpu"])
    files = os.listdir(ck)
    assert files == ["model_0.ckpt"]
    state = torch.load(ck / files[0], weights_only=True)
    assert set(state) == {"epoch", "model_state_dict", "optimizer_state_dict"}
    assert any(k.startswith("perceiver.") for k in state["model_state_dict"])
    assert any(k.startswith("uresnet.") for k in state["model_state_dict"])  # built, unused in forward


def test_lartpc_logits_are_permuted_not_reshaped():
    """Defect D6: (B, H·W, 3) logits become (B, 3, H·W) by a permute."""
    import run

    torch.manual_seed(0)
    m = run.LArPerceiver(16)
    img = torch.rand(2, 16 * 16)
    img[img < 0.7] = 0
    out = m(img)
    assert out.shape == (2, 3, 256)
    raw = m.perceiver(img.reshape(2, 16, 16, 1), (img == 0).reshape(2, -1))
    assert torch.equal(out, raw.permute(0, 2, 1))


def test_uresnet_shapes():
    from perceiver_io_amd.models.uresnet import UResNet

    net = UResNet(num_classes=3, input_channels=3, inplanes=16)
    y = net(torch.randn(1, 3, 64, 64))
    assert y.shape == (1, 3, 64, 64)


def test_tokenizer_train_save_load_roundtrip(tmp_path):
    from tokenizers.normalizers import Replace

    from perceiver_io_amd.utils.tokenizer import (MASK_TOKEN, PAD_TOKEN, UNK_TOKEN, create_tokenizer, load_tokenizer,
                                                  save_tokenizer, train_tokenizer)

    tok = create_tokenizer(Replace("<br />", " "))
    corpus = ["The movie was great<br />and the acting superb", "a terrible film", "great great acting"] * 20
    train_tokenizer(tok, corpus, vocab_size=120)
    assert [tok.token_to_id(t) for t in (PAD_TOKEN, UNK_TOKEN, MASK_TOKEN)] == [0, 1, 2]
    path = str(tmp_path / "tok.json")
    save_tokenizer(tok, path)
    tok2 = load_tokenizer(path)
    ids = tok2.encode("The MOVIE<br />was Great").ids
    assert ids == tok.encode("the movie was great").ids  # normalizers: Replace, NFD, Lowercase, StripAccents
    assert tok2.decode(ids) == "the movie was great"


@pytest.mark.skipif(not os.path.exists(REF_TOKENIZER), reason="reference tokenizer JSON not mounted")
def test_reference_tokenizer_json_loads():
    """The tokenizer shipped in the reference tree (SURVEY #37) loads with the JSON loader."""
    from perceiver_io_amd.utils.tokenizer import load_tokenizer

    tok = load_tokenizer(REF_TOKENIZER)
    assert tok.get_vocab_size() == 10003
    assert [tok.token_to_id(t) for t in ("[PAD]", "[UNK]", "[MASK]")] == [0, 1, 2]


def test_predict_masked_samples_topk_fill_ins():
    from perceiver_io_amd.models import (PerceiverDecoder, PerceiverEncoder, PerceiverMLM, TextInputAdapter,
                                         TextMasking, TextOutputAdapter)
    from perceiver_io_amd.utils.misc import predict_masked_samples
    from perceiver_io_amd.utils.tokenizer import create_tokenizer, train_tokenizer

    tok = create_tokenizer()
    train_tokenizer(tok, ["i have watched this movie and it was awesome", "a show", "the film"] * 10, vocab_size=60)
    V, L = tok.get_vocab_size(), 16
    enc = PerceiverEncoder(TextInputAdapter(V, L, 32), (8, 32), 1, num_self_attention_layers_per_block=1)
    dec = PerceiverDecoder(TextOutputAdapter(V, L, 32), (8, 32))
    model = PerceiverMLM(enc, dec, TextMasking(V))

    def encode(texts):
        rows = [tok.encode(t).ids[:L] for t in texts]
        x = torch.zeros(len(rows), L, dtype=torch.long)
        for i, r in enumerate(rows):
            x[i, :len(r)] = torch.tensor(r)
        return x, x == 0

    out = predict_masked_samples(["i have watched this [MASK] and it was awesome", "a [MASK]"], encode, tok, model,
                                 num_predictions=3)
    assert len(out) == 2 and all(len(o) == 3 for o in out)
    assert all(isinstance(s, str) and "[MASK]" not in s for o in out for s in o)
    # the i-th variant fills every [MASK] with its i-th most likely token
    x, pad = encode(["i have watched this [MASK] and it was awesome", "a [MASK]"])
    model.eval()
    logits, _ = model(x, pad, masking=False)
    at = x == tok.token_to_id("[MASK]")
    for i in range(3):
        y = x.clone()
        y[at] = logits[at].topk(3, dim=-1).indices[:, i]
        assert [out[j][i] for j in range(2)] == [tok.decode(r.tolist(), skip_special_tokens=True) for r in y]


def _fake_imdb(root, n=3):
    for split in ("train", "test"):
        for lab in ("neg", "pos"):
            d = root / "IMDB" / "aclImdb" / split / lab
            d.mkdir(parents=True)
            for i in range(n):
                (d / f"{i}_1.txt").write_text(f"this movie was {'bad' if lab == 'neg' else 'great'}<br />film {i}")


@pytest.mark.skipif(not os.path.exists(REF_TOKENIZER), reason="reference tokenizer not mounted")
@pytest.mark.parametrize("explicit", [False, True])
def test_imdb_uses_shipped_tokenizer(tmp_path, explicit):
    """The reference's shipped tokenizer (``.cache/imdb-tokenizer-10003.json``) is loaded as is —
    at ``<data_dir>/imdb-tokenizer-10003.json`` or via ``tokenizer_path`` — and never retrained."""
    import shutil

    from perceiver_io_amd.data.imdb import IMDBDataModule

    _fake_imdb(tmp_path)
    if explicit:
        tok_path = tmp_path / "user-tok.json"
        shutil.copy(REF_TOKENIZER, tok_path)
        dm = IMDBDataModule(data_dir=str(tmp_path), batch_size=2, num_workers=0, tokenizer_path=str(tok_path))
    else:
        tok_path = tmp_path / "imdb-tokenizer-10003.json"
        shutil.copy(REF_TOKENIZER, tok_path)
        dm = IMDBDataModule(data_dir=str(tmp_path), batch_size=2, num_workers=0)
    before = tok_path.read_bytes()
    dm.prepare_data()
    dm.setup()
    assert tok_path.read_bytes() == before  # not retrained
    assert dm.tokenizer.get_vocab_size() == 10003
    assert [dm.tokenizer.token_to_id(t) for t in ("[PAD]", "[UNK]", "[MASK]")] == [0, 1, 2]
    y, ids, pad = next(iter(dm.train_dataloader()))
    assert ids.shape[0] == 2 and int(ids.max()) < 10003 and pad.dtype == torch.bool
    with pytest.raises(FileNotFoundError):
        IMDBDataModule(data_dir=str(tmp_path), tokenizer_path=str(tmp_path / "missing.json")).prepare_data()


class _DeferInBackward(torch.autograd.Function):
    """Defers a slab job from inside backward; the job must be complete when backward returns."""

    @staticmethod
    def forward(ctx, x, slab, dst):
        ctx.slab, ctx.dst = slab, dst
        return x * 2

    @staticmethod
    def backward(ctx, g):
        F.defer_slab(emulation, ctx.slab, [ctx.dst[:5], ctx.dst[5:]], [0, 8])
        assert F._pending, "job must be queued, not run, inside backward"
        return g * 2, None, None


def test_slab_jobs_deferred_to_backward_end_and_run_outside_backward():
    slab = torch.arange(3 * 16, dtype=torch.float32).view(3, 16)
    want = torch.cat([slab[:, :5].sum(0), slab[:, 8:13].sum(0)])
    dst = torch.ones(10)
    x = torch.ones(4, requires_grad=True)
    _DeferInBackward.apply(x, slab, dst).sum().backward()
    assert not F._pending and torch.allclose(dst, 1 + want)
    dst2 = torch.zeros(10)
    F.defer_slab(emulation, slab, [dst2[:5], dst2[5:]], [0, 8])  # outside backward: runs immediately
    assert not F._pending and torch.allclose(dst2, want)


def test_self_attention_block_node_matches_layerwise():
    """The one-node self-attention block (fused layer boundaries, slab gradients) equals the
    layer-by-layer executor in outputs and parameter gradients (kernel emulation)."""
    from perceiver_io_amd.models.blocks import self_attention_block as make_block

    torch.manual_seed(5)
    block = make_block(3, 64, 4, 0.0)
    x = torch.randn(3, 20, 64, requires_grad=True)
    w = torch.randn(3, 20, 64)
    outs, grads = [], []
    for mode in ("block", "layers"):
        block.zero_grad()
        x.grad = None
        if mode == "block":
            y = F.self_attention_block(block, x)
        else:
            y = x
            for layer in block:
                y = F.self_attention_layer(layer, y)
        (y * w).sum().backward()
        outs.append(y.detach())
        grads.append([x.grad.clone()] + [p.grad.clone() for p in block.parameters()])
    assert torch.allclose(outs[0], outs[1], atol=1e-5)
    for a, b in zip(*grads):
        assert torch.allclose(a, b, atol=1e-4, rtol=1e-4)


@pytest.mark.gpu
def test_lartpc_run_gpu(tmp_path):
    """run.py on the MI355X through the HIP path: Fourier-PE image input with the zero-pixel
    key-padding mask, a one-query-per-pixel decoder, weighted CE, grad clipping."""
    import run
    from perceiver_io_amd.ops import ext

    ext.require()
    ck = tmp_path / "ckpt"
    run.main(["--epochs", "1", "--events", "4", "--val-events", "2", "--size", "128", "--batch-size", "2",
              "--max-steps", "2", "--log-dir", str(tmp_path / "runs"), "--ckpt-dir", str(ck), "--device", "cuda"])
    state = torch.load(ck / "model_0.ckpt", weights_only=True)
    assert all(torch.isfinite(v).all() for v in state["model_state_dict"].values() if v.is_floating_point())


def test_checked_variant_is_built_and_flagged():
    """build.py --check produces _C_check (PIO_CHECKS=1, host binding under UBSan) next to the
    release _C; each reports which it is (the loader picks _C_check with PERCEIVER_CHECKED=1)."""
    import importlib

    import pytest

    try:
        rel = importlib.import_module("perceiver_io_amd._C")
        chk = importlib.import_module("perceiver_io_amd._C_check")
    except ImportError as e:  # pragma: no cover - depends on the build state
        pytest.skip(f"extension not built: {e}")
    assert not rel.checked_build() and chk.checked_build()


def test_shipped_reference_tokenizer_installed_for_real_data(tmp_path):
    """A real-data IMDB run at vocab 10003 without a tokenizer in data_dir installs the shipped
    reference vocabulary (reference .cache/imdb-tokenizer-10003.json) instead of training one."""
    import filecmp
    import os

    from perceiver_io_amd.data.imdb import IMDBDataModule, shipped_tokenizer
    from perceiver_io_amd.utils.tokenizer import MASK_TOKEN, PAD_TOKEN, UNK_TOKEN

    for split in ("train", "test"):
        for lab in ("neg", "pos"):
            d = tmp_path / "IMDB" / "aclImdb" / split / lab
            d.mkdir(parents=True)
            (d / "0_1.txt").write_text("a tiny review<br />of a movie")
    dm = IMDBDataModule(data_dir=str(tmp_path), vocab_size=10003, max_seq_len=16, batch_size=2, num_workers=0)
    dm.prepare_data()
    path = os.path.join(str(tmp_path), "imdb-tokenizer-10003.json")
    assert filecmp.cmp(path, shipped_tokenizer(10003), shallow=False)
    dm.setup("fit")
    tok = dm.tokenizer
    assert tok.get_vocab_size() == 10003
    assert [tok.token_to_id(t) for t in (PAD_TOKEN, UNK_TOKEN, MASK_TOKEN)] == [0, 1, 2]
    ref = "/root/reference/.cache/imdb-tokenizer-10003.json"
    if os.path.exists(ref):  # byte-identical to the reference's shipped file
        assert filecmp.cmp(ref, shipped_tokenizer(10003), shallow=False)
    ids = tok.encode("i have watched this [MASK] and it was awesome").ids
    assert 2 in ids and 1 not in ids
