"""Overlapped, bucketed gradient all-reduce and gradient clipping under data parallelism
(gloo on CPU, 2 and 4 ranks).

* The ready-point buckets (decoder + head, the tail of the flat buffer; then layer_n) are launched
  from the backward pass when autograd reaches the decoder input / layer_n's input (``parallel/reducer.py`` ``_ReadyFn``).  If any
  decoder-side gradient were still incomplete at that point the reduced values would differ, so
  bit-identity with the non-overlapped reducer pins the readiness ordering — here with the FUSED
  executor (kernel emulation on CPU: deferred weight-gradient slab jobs, in-place gradient
  accumulation), which is the path the GPU runs.
* Clipping applies to the norm of the averaged gradient (``max_grad_norm`` under DDP equals
  single-process clipping of the large-batch gradient), for the fused AdamW and the eager path.
"""
import os
import socket

import pytest
import torch
import torch.multiprocessing as mp


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _env(rank, world, port):
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1",
                      MASTER_PORT=str(port))


def _fused_on_cpu():
    """Route the model through the fused executor with the kernel emulation (CPU)."""
    from perceiver_io_amd import ops
    from perceiver_io_amd.ops import emulation, ext

    ext._mod = emulation
    ops.use_hip = lambda t: True


def _mlm(seed):
    from perceiver_io_amd.tasks import LitMaskedLanguageModel

    torch.manual_seed(seed)
    return LitMaskedLanguageModel(vocab_size=200, max_seq_len=32,
                                  optimizer_init={"class_path": "torch.optim.AdamW", "init_args": {"lr": 1e-3}},
                                  num_latents=16, num_latent_channels=32, num_encoder_layers=2,
                                  num_encoder_self_attention_layers_per_block=2)


def _worker_overlap(rank, world, port, fused, out):
    _env(rank, world, port)
    if fused:
        _fused_on_cpu()
    from perceiver_io_amd.ops.optim import FlatParameterSpace
    from perceiver_io_amd.parallel import FlatGradReducer, dist

    dist.init(device_type="cpu")
    lit = _mlm(seed=0)
    model = lit.model
    flat = FlatParameterSpace(model.parameters(), with_shadow=False, replicate=False)
    g = torch.Generator().manual_seed(100 + rank)
    x = torch.randint(3, 200, (4, 32), generator=g)
    pad = torch.zeros(4, 32, dtype=torch.bool)
    pad[1, 20:] = True
    xm, lab = model.masking(x, pad, generator=torch.Generator().manual_seed(5 + rank))
    res = {}
    for overlap in (False, True):
        red = FlatGradReducer(flat, bucket_bytes=16 << 10, overlap=overlap)
        red.plan(model)
        flat.zero_grad()
        red.arm()
        loss = model.loss(x, pad, labels=lab, x_masked=xm)
        loss.backward()
        red.finish()
        res[overlap] = (flat.grad.clone(), red.early_launches, len(red.buckets), red.early)
        red.close()
    out[rank] = res
    dist.shutdown()


@pytest.mark.parametrize("world,fused", [(2, True), (4, True), (2, False)])
def test_overlapped_buckets_bit_identical(world, fused):
    port = _port()
    out = mp.Manager().dict()
    mp.spawn(_worker_overlap, args=(world, port, fused, out), nprocs=world, join=True)
    for r in range(world):
        (g0, n0, nb0, e0), (g1, n1, nb1, e1) = out[r][False], out[r][True]
        assert e1 is not None and e1[1] > e1[0]  # the decoder is a contiguous tail bucket
        assert n0 == 0 and n1 == 3  # only the overlapped reducer launched from the backward (decoder, layer_n, layer_1_sa)
        assert nb0 == nb1 >= 2  # an explicit bucket size: the same layout without overlap
        assert torch.equal(g0, g1), (r, (g0 - g1).abs().max())
    assert all(torch.equal(out[0][True][0], out[r][True][0]) for r in range(world))


def _worker_clip(rank, world, port, fused, out):
    _env(rank, world, port)
    from perceiver_io_amd.ops.optim import FlatParameterSpace, FusedAdamW
    from perceiver_io_amd.parallel import FlatGradReducer, dist

    dist.init(device_type="cpu")
    lit = _mlm(seed=0)
    model = lit.model
    params = list(model.parameters())
    g = torch.Generator().manual_seed(200 + rank)
    x = torch.randint(3, 200, (4, 32), generator=g)
    pad = torch.zeros(4, 32, dtype=torch.bool)
    xm, lab = model.masking(x, pad, generator=torch.Generator().manual_seed(9 + rank))
    clip = 0.05
    if fused:
        opt = FusedAdamW(params, lr=1.0, eps=0.1, weight_decay=0.0, max_grad_norm=clip)
        red = FlatGradReducer(opt.flat)
        opt.grad_scale = red.grad_scale()
        opt.flat.zero_grad()
        model.loss(x, pad, labels=lab, x_masked=xm).backward()
        red.finish()
        opt.step()
    else:  # the trainer's eager clip path (precision 32)
        from perceiver_io_amd.train.trainer import Trainer

        flat = FlatParameterSpace(params, with_shadow=False)
        red = FlatGradReducer(flat)
        opt = torch.optim.AdamW(params, lr=1.0, eps=0.1, weight_decay=0.0)
        tr = Trainer.__new__(Trainer)
        tr.optimizers, tr.lr_schedulers, tr.gradient_clip_val, tr.model = [opt], [], clip, lit

        class _E:
            reducer = red

        tr._engine = _E()
        tr._training_loss = lambda b: model.loss(x, pad, labels=lab, x_masked=xm)
        tr._batch_idx = 0
        flat.zero_grad()
        tr._eager_clip_step([None])
    red.close()
    out[rank] = (torch.cat([p.detach().reshape(-1) for p in params]), x, xm, lab)
    dist.shutdown()


@pytest.mark.parametrize("fused", [True, False])
def test_clip_under_ddp_matches_single_process(fused):
    world, port = 2, _port()
    out = mp.Manager().dict()
    mp.spawn(_worker_clip, args=(world, port, fused, out), nprocs=world, join=True)
    # single process: mean of the per-rank mean losses (= the DDP averaged gradient), clipped
    lit = _mlm(seed=0)
    model = lit.model
    params = list(model.parameters())
    loss = sum(model.loss(out[r][1], torch.zeros(4, 32, dtype=torch.bool), labels=out[r][3], x_masked=out[r][2])
               for r in range(world)) / world
    loss.backward()
    norm = torch.nn.utils.clip_grad_norm_(params, 0.05)
    assert norm > 0.05 * 2  # clipping is active
    # eps ≫ |g|: the update is ~linear in the (clipped) gradient, so a wrong clip factor shows
    opt = torch.optim.AdamW(params, lr=1.0, eps=0.1, weight_decay=0.0)
    opt.step()
    ref = torch.cat([p.detach().reshape(-1) for p in params])
    for r in range(world):
        assert torch.allclose(out[r][0], ref, atol=2e-6, rtol=1e-5), (r, (out[r][0] - ref).abs().max())
