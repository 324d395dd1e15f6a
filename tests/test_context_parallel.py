"""Context parallelism (parallel/context.py) on CPU with gloo: the encoder with its
inputs sharded over 2 and 3 ranks gives the single-process encoder's latents and — after the
ordinary data-parallel gradient average — its parameter gradients, for text and image inputs,
with ragged and fully masked key-padding rows."""
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


def _encoder(kind):
    from perceiver_io_amd.models import ImageInputAdapter, PerceiverEncoder, TextInputAdapter

    torch.manual_seed(0)
    if kind == "text":
        ad = TextInputAdapter(vocab_size=50, max_seq_len=31, num_input_channels=32)
    else:
        ad = ImageInputAdapter((6, 5, 2), num_frequency_bands=3)
    return PerceiverEncoder(ad, (8, 32), num_layers=3, num_cross_attention_heads=4, num_self_attention_heads=4,
                            num_self_attention_layers_per_block=1, dropout=0.0)


def _inputs(kind):
    g = torch.Generator().manual_seed(5)
    if kind == "text":
        x = torch.randint(3, 50, (3, 31), generator=g)
        pad = torch.zeros(3, 31, dtype=torch.bool)
        pad[1, 20:] = True  # ragged suffix padding: the last rank's shard is fully masked for row 1
        pad[2, :] = True    # every key masked → zero attention output (D10)
        return x, pad
    return torch.randn(3, 6, 5, 2, generator=g), None


def _worker(rank, world, port, kind, out, impl="torch"):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from perceiver_io_amd import ops
    from perceiver_io_amd.parallel.context import ContextParallelEncoder

    dist.init_process_group("gloo", rank=rank, world_size=world)
    ops.set_backend("torch")
    enc = _encoder(kind)
    x, pad = _inputs(kind)
    w = torch.randn(3, 8, 32, generator=torch.Generator().manual_seed(9))
    # single-process reference (full input on this rank)
    ref, _ = enc(x, pad)
    (ref * w).sum().backward()
    ref_grads = {n: p.grad.clone() for n, p in enc.named_parameters() if p.grad is not None}
    enc.zero_grad(set_to_none=True)
    # context parallel: this rank's input shard, then the data-parallel gradient average
    lat, _ = ContextParallelEncoder(enc, impl=impl)(x, pad)
    (lat * w).sum().backward()
    err_g = 0.0
    for n, p in enc.named_parameters():
        if p.grad is None:
            continue
        dist.all_reduce(p.grad)
        p.grad /= world
        err_g = max(err_g, (p.grad - ref_grads[n]).abs().max().item() / (ref_grads[n].abs().max().item() + 1e-6))
    out[rank] = ((lat - ref).abs().max().item(), err_g, lat[2].abs().max().item() if kind == "text" else None,
                 set(ref_grads) == {n for n, p in enc.named_parameters() if p.grad is not None})
    dist.destroy_process_group()


@pytest.mark.parametrize("kind,world", [("text", 2), ("text", 3), ("image", 2)])
def test_context_parallel_encoder_matches_full(kind, world):
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _port(), kind, out), nprocs=world, join=True)
    for r in range(world):
        err_out, err_g, _, same_params = out[r]
        assert err_out < 1e-5, (r, err_out)
        assert err_g < 1e-4, (r, err_g)
        assert same_params


@pytest.mark.parametrize("kind,world", [("text", 3), ("image", 2)])
def test_context_parallel_flash_merge_matches_full(kind, world):
    """The kernel implementation (shard-local flash attention + LSE merge; the CPU runs the
    kernels' emulation, bf16 operands) against the fp32 single-process encoder."""
    out = mp.Manager().dict()
    mp.spawn(_worker, args=(world, _port(), kind, out, "kernel"), nprocs=world, join=True)
    for r in range(world):
        err_out, err_g, dead, same_params = out[r]
        assert err_out < 3e-2, (r, err_out)
        assert err_g < 5e-2, (r, err_g)
        assert same_params


def test_shard_range_covers_inputs():
    from perceiver_io_amd.parallel.context import shard_range

    for m in (1, 7, 31, 512):
        for w in (1, 2, 3, 8):
            parts = [shard_range(m, r, w) for r in range(w)]
            assert parts[0][0] == 0 and parts[-1][1] == m
            assert all(a[1] == b[0] for a, b in zip(parts, parts[1:]))


def _worker_gpu(rank, world, port, out):
    os.environ.update(RANK=str(rank), WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    import torch.distributed as dist

    from perceiver_io_amd.ops import ext
    from perceiver_io_amd.parallel.context import ContextParallelEncoder

    ext.require()
    dist.init_process_group("gloo", rank=rank, world_size=world)  # 2 ranks share the box's one GPU
    dev = torch.device("cuda:0")
    enc = _encoder("text").to(dev)
    x, pad = (t.to(dev) for t in _inputs("text"))
    w = torch.randn(3, 8, 32, generator=torch.Generator().manual_seed(9)).to(dev)
    ref, _ = enc(x, pad)  # fused HIP encoder on the full input
    (ref * w).sum().backward()
    def flat_grads():
        return torch.cat([(p.grad if p.grad is not None else torch.zeros_like(p)).reshape(-1).clone()
                          for p in enc.parameters()])

    ref_g = flat_grads()
    enc.zero_grad(set_to_none=False)
    # CP cross-attention on the flash kernels (shard-local attention + LSE merge) + fused HIP
    # self-attention blocks
    lat, _ = ContextParallelEncoder(enc)(x, pad)
    (lat * w).sum().backward()
    g = flat_grads()
    dist.all_reduce(g)
    g /= 2
    torch.cuda.synchronize()
    out[rank] = ((lat - ref).abs().max().item() / ref.abs().max().item(), bool(torch.isfinite(g).all().item()),
                 ((g - ref_g).norm() / ref_g.norm()).item())
    dist.destroy_process_group()


@pytest.mark.gpu
def test_context_parallel_encoder_gpu_two_ranks():
    out = mp.Manager().dict()
    mp.spawn(_worker_gpu, args=(2, _port(), out), nprocs=2, join=True)
    for r in range(2):
        rel, finite, grel = out[r]
        assert rel < 3e-2 and finite, (r, rel)
        assert grel < 3e-2, (r, grel)
