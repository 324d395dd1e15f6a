"""Fused layer executor: one autograd node per Perceiver sublayer.

The module tree (``models/blocks.py``) only holds parameters.  On an MI355X each
``Residual(attention) → Residual(mlp)`` pair (reference ``perceiver/model.py:29-44``) runs as
a single :class:`_LayerFn` whose forward is

    LN+QKV projection (ln_linear_fwd) → flash attention (attn_fwd) →
    out-proj + residual + LN2 + MLP(GELU) + residual (post_attn_fwd)

i.e. 3 kernel launches, and whose backward is the hand-written reverse chain
(post_attn_bwd → attn_bwd → ln_linear_bwd), 3 launches as well: each weight gradient is an
extra MFMA pass over LDS tiles the producing kernel already holds.  Parameter gradients go
through per-tile slabs by default (``WGRAD_SLAB``, see ``_GradSlab``): each 64-row tile STORES
its partial into one slab row, and the slab rows are summed into ``p.grad`` (views of the flat
gradient buffer) by extra workgroups appended to the next backward kernel, or by an
end-of-backward flush — no float atomics, no per-parameter autograd accumulation
(``WGRAD_SLAB = False`` selects in-kernel atomics into replicated accumulators).
Self-attention blocks run as one node (``_SABlockFn``): one launch per layer forward and per
layer boundary backward.  Activations kept for backward: the bf16 Q/K/V and attention output,
fp32 post-attention residual, LN statistics, the bf16 pre-GELU tensor — LN outputs and GELU
outputs are recomputed.

Encoder-specific savings over the reference forward:
  * the learned latent array enters the first layer un-expanded (batch stride 0): its
    LayerNorm + Q projection runs on N rows instead of B·N (SURVEY K-04);
  * the decoder's output queries likewise (K rows, not B·K).

``kernels`` is either the HIP extension or :mod:`.emulation` (same signatures in plain
PyTorch), so the executor's bookkeeping is testable on CPU.
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass
from typing import List, Optional

import torch

from . import emulation, ext
from ..parallel.reducer import bucket_ready_point

EPS = 1e-5
# per-tile weight-gradient partials go to a slab whose reduction rides the next backward kernel
# (see _GradSlab); False: in-kernel float atomics into the replicated accumulators
WGRAD_SLAB = True
# self-attention dQKV stored as bf16 for the chain-layout boundary kernel (identical results)
BF16_DQKV = True
# the bf16 self-attention backward carries the pending slab reduction in appended workgroups
# (1.429 → 1.377 ms on the headline step against the next chain kernel carrying it, r5)
ATTN_SLAB = True
# 64-latent blocks (one sample per 64-row tile): the boundary kernel of layers i → i-1 also runs
# layer i-1's attention backward (csrc/chain.hip phase D) and hands its dQKV on as bf16 — one
# launch per layer instead of two (tests/test_model_gpu.py compares both settings)
CHAIN_ATT = True
TALL_ROWS = 1 << 17  # kTallRows in csrc/binding.cpp: taller projections stream their dW (wgrad kernel)


def kernels(t: torch.Tensor):
    return ext.require() if t.is_cuda else emulation


# ------------------------------------------------------------------------------------------
# bf16 weight shadows
# ------------------------------------------------------------------------------------------
class WeightCache:
    """bf16 copies of fp32 parameters used as GEMM operands.

    An entry is refreshed when the parameter's version counter or storage changes.  The
    fused optimizer (``ops.optim.FusedAdamW``) writes shadows in the same pass as the
    parameter update and binds them here, so steady-state training never re-casts.
    """

    def __init__(self):
        self._d = {}

    def bind(self, p: torch.Tensor, shadow: torch.Tensor):
        self._d[id(p)] = [p._version, p.data_ptr(), shadow, p]
        with torch.no_grad():
            shadow.copy_(p.detach().reshape(shadow.shape))

    def get(self, p: torch.Tensor) -> torch.Tensor:
        ent = self._d.get(id(p))
        if ent is not None and ent[3] is p and ent[0] == p._version and ent[1] == p.data_ptr():
            return ent[2]
        with torch.no_grad():
            if ent is not None and ent[3] is p and ent[2].shape == p.shape:
                ent[2].copy_(p.detach())
                ent[0], ent[1] = p._version, p.data_ptr()
                return ent[2]
            t = p.detach().to(torch.bfloat16).contiguous()
        self._d[id(p)] = [p._version, p.data_ptr(), t, p]
        return t

    def clear(self):
        self._d.clear()


weight_cache = WeightCache()


# ------------------------------------------------------------------------------------------
# weight-gradient slabs
# ------------------------------------------------------------------------------------------
_pending = []          # deferred slab reductions: (K, slab, dsts, offsets, stream)
_flush_queued = [False]


def _flush_pending():
    """Run every deferred slab reduction as a standalone launch (end of a backward pass)."""
    _flush_queued[0] = False
    while _pending:
        K, t, ds, os_, st = _pending.pop(0)
        if st is None:
            K.slab_reduce(t, ds, os_)
        else:
            with torch.cuda.stream(st):
                K.slab_reduce(t, ds, os_)


def flush_pending(stream=None, inside=None):
    """Launch every deferred slab reduction now (e.g. before a gradient bucket that depends on
    them is all-reduced mid-backward, parallel/reducer.py).

    ``stream`` (the reducer's side stream, the only consumer of a completed bucket): the jobs whose
    every destination satisfies ``inside`` (lies in the bucket, so nothing on the main stream adds
    to it any more) run there, after the caller has made ``stream`` wait for the current stream;
    the slabs are recorded on it so the allocator keeps them until it is done.  Every other job —
    destinations still being accumulated by later kernels of the backward (e.g. ``layer_n``'s
    query path, finished inside ``layer_1``'s block), or straddling the bucket — runs on the
    current stream NOW, before that wait, so it stays ordered with those kernels.  In
    deterministic mode everything runs on the current stream (fixed order, plain adds).
    Returns the jobs to run on ``stream`` as a callable (call it after the wait)."""
    from . import deterministic

    if stream is None or inside is None or deterministic():
        _flush_pending()
        return lambda: None
    _flush_queued[0] = False
    side = []
    while _pending:
        job = _pending.pop(0)
        K, t, ds, os_, st = job
        if all(inside(d) for d in ds):
            side.append(job)
        elif st is None:
            K.slab_reduce(t, ds, os_)
        else:
            with torch.cuda.stream(st):
                K.slab_reduce(t, ds, os_)

    def run_side():
        with torch.cuda.stream(stream):
            for K, t, ds, os_, _ in side:
                t.record_stream(stream)
                K.slab_reduce(t, ds, os_)

    return run_side


def defer_slab(K, t: torch.Tensor, dsts, offs):
    """Queue ``dsts[j] += Σ_rows t[:, offs[j]:offs[j] + dsts[j].numel()]`` (a slab job) for the
    next backward kernel of the chain, or the end-of-backward flush."""
    if not dsts:
        return
    st = torch.cuda.current_stream(t.device) if t.is_cuda else None
    _pending.append((K, t, list(dsts), list(offs), st))
    if not _flush_queued[0]:
        try:
            torch.autograd.Variable._execution_engine.queue_callback(_flush_pending)
            _flush_queued[0] = True
        except RuntimeError:  # not inside a backward pass
            _flush_pending()


def _take_job() -> dict:
    """kwargs handing the oldest deferred slab reduction to the next backward kernel, which
    runs it in extra workgroups appended to its own grid (csrc/common.h SlabJob)."""
    if not _pending:
        return {}
    _, t, ds, os_, _ = _pending.pop(0)
    return dict(job_slab=t, job_dsts=ds, job_offs=os_)


class _GradSlab:
    """(tiles, P) fp32 slab holding one backward kernel's per-64-row-tile parameter-gradient
    partials (one row per workgroup, segments 4-float aligned).  The kernel stores its partials
    with plain stores instead of float atomics (which run at ≈1.3 TB/s chip-wide: ≈10 µs of a
    ≈25 µs post-attention / QKV backward at the headline shape).  ``defer`` queues the
    reduction of the slab into the parameter gradients; the next backward kernel of the chain
    runs it in appended workgroups, overlapped with its own latency-bound tiles, on the same
    stream (a side-stream branch costs 10–15 µs of cross-queue hand-off per fork in a
    replayed hipGraph; round 5 re-measured every reduction on a side stream: 1.712 against
    1.424 ms per headline step, profiles/r5_slab_side_ab.md).  Reductions still pending when the backward pass ends are launched by
    an autograd final callback, so gradients are complete when ``backward()`` returns."""

    def __init__(self, R: int, sizes, like: torch.Tensor):
        self.offs, P = [], 0
        for n in sizes:
            self.offs.append(P)
            P += (n + 3) // 4 * 4
        self.sizes = list(sizes)
        self.t = torch.empty(((R + 63) // 64, P), dtype=torch.float32, device=like.device)

    def targets(self):
        return [self.t[:, o:o + n] for o, n in zip(self.offs, self.sizes)]

    def defer(self, K, dsts):
        """dsts[i]: None (frozen: dropped), a contiguous tensor of sizes[i] elements, or a list
        of (tensor, offset within segment i) pieces."""
        ds, os_ = [], []
        for i, d in enumerate(dsts):
            if d is None:
                continue
            for t, extra in (d if isinstance(d, list) else [(d, 0)]):
                ds.append(t.view(-1))
                os_.append(self.offs[i] + extra)
        defer_slab(K, self.t, ds, os_)


def _grad_of(p: torch.Tensor):
    """p's fp32 gradient tensor (created if absent); None for frozen parameters."""
    if not p.requires_grad:
        return None
    if p.grad is None:
        p.grad = torch.zeros_like(p)
    return p.grad


# ------------------------------------------------------------------------------------------
# layer specs
# ------------------------------------------------------------------------------------------
@dataclass(frozen=True)
class LayerSpec:
    cross: bool
    packed: bool      # packed in_proj_weight (kdim == vdim == embed_dim)
    C: int            # embed / latent channels
    heads: int
    dropout: float


def layer_spec_and_params(layer):
    att = layer.attn
    mha = att.attention.attention
    m = layer.mlp
    cross = hasattr(att, "q_norm")
    packed = mha._qkv_same_embed_dim
    spec = LayerSpec(cross=cross, packed=packed, C=mha.embed_dim, heads=mha.num_heads, dropout=float(mha.dropout))
    ps: List[torch.Tensor] = []
    if cross:
        ps += [att.q_norm.weight, att.q_norm.bias, att.kv_norm.weight, att.kv_norm.bias]
    else:
        ps += [att.norm.weight, att.norm.bias]
    if packed:
        ps += [mha.in_proj_weight]
    else:
        ps += [mha.q_proj_weight, mha.k_proj_weight, mha.v_proj_weight]
    ps += [mha.in_proj_bias, mha.out_proj.weight, mha.out_proj.bias,
           m[0].weight, m[0].bias, m[1].weight, m[1].bias, m[3].weight, m[3].bias]
    return spec, ps


def _kv_weight(spec: LayerSpec, ps):
    """bf16 K‖V projection weight of a cross layer with kdim ≠ embed_dim, rows zero padded to a
    multiple of 8 columns (vectorised weight staging in the kernels).  Built only where the K/V
    projection runs (once per forward for a weight-shared layer)."""
    wc = weight_cache
    wk, wv = wc.get(ps[5]), wc.get(ps[6])
    kin = wk.shape[1]
    both = _adjacent_rows(wk, wv)
    if both is not None:
        # adjacent bf16 shadows in the optimizer's flat shadow buffer: K‖V is already one
        # (2C, kin) matrix (unpadded rows: the kernels take the row stride) — no per-step copy
        return both
    wkv = torch.zeros((2 * spec.C, (kin + 7) // 8 * 8), dtype=wk.dtype, device=wk.device)
    wkv[: spec.C, :kin] = wk
    wkv[spec.C:, :kin] = wv
    return wkv


def _bf16_weights(spec: LayerSpec, ps):
    """bf16 GEMM operands: (w_q_or_qkv, w_kv (packed layers; None otherwise, see _kv_weight),
    w_o, w_1, w_2)."""
    wc = weight_cache
    if spec.cross:
        if spec.packed:
            win = wc.get(ps[4])
            wq, wkv = win[: spec.C], win[spec.C:]
            rest = ps[5:]
        else:
            wq, wkv = wc.get(ps[4]), None
            rest = ps[7:]
    else:
        wq, wkv = wc.get(ps[2]), None
        rest = ps[3:]
    # rest = [bin, Wo, bo, g2, be2, W1, b1, W2, b2]
    return wq, wkv, wc.get(rest[1]), wc.get(rest[5]), wc.get(rest[7])


class KVSource:
    """The key/value input of the encoder's cross-attention layers for one forward pass.

    * K-06 (reference ``model.py:186-187`` applies the same ``layer_n`` to the same input
      ``num_layers - 1`` times): the LayerNorm + K/V projection of a cross layer runs once per
      forward; later applications reuse the K/V, their dK/dV are accumulated into one buffer
      (attention backward in accumulate mode) and the projection's backward runs once — in the
      backward of the first application, which autograd schedules after the later ones (their
      queries depend on its output).
    * K-03 (``adapter.py:99-109`` materialises ``[pixels ‖ Fourier PE]``): with ``pe`` given, ``x``
      holds only the pixels ``(B, M, C_img)`` and the projection kernels add them into the
      zero leading columns of the padded PE table ``pe`` ``(M, round_up(Kin, 8))``; with ``index``
      (B, M) int64 given (sparse images, ``models/lartpc.py``) row (b, m) reads PE row
      ``index[b, m]`` instead of ``m``, so the gathered ``[pixel ‖ PE]`` rows are never formed.
    """

    def __init__(self, x: torch.Tensor, pe: Optional[torch.Tensor] = None, kin: Optional[int] = None,
                 index: Optional[torch.Tensor] = None):
        self.x = x
        self.pe = pe
        self.index = index
        self.kin = kin if kin is not None else x.shape[-1]
        self.entries = {}
        # input-gradient hand-off between the projections of different layers (layer_1 and
        # layer_n both project this input): each backward adds the previous one's dX as the
        # residual of its ln_linear_bwd, and only the last returns the total to autograd
        self.pending_dx = None
        self.owners_left = None

    @property
    def channels(self) -> int:
        return self.kin

    def materialize(self) -> torch.Tensor:
        """The (B, M, Kin) input the unfused path consumes."""
        if self.pe is None:
            return self.x
        b, m = self.x.shape[0], self.x.shape[1]
        if self.index is not None:
            full = self.pe[:, : self.kin].index_select(0, self.index.reshape(-1)).view(b, m, self.kin)
        else:
            full = self.pe[:, : self.kin].unsqueeze(0).repeat(b, 1, 1)
        full[:, :, : self.x.shape[2]] += self.x
        return full


# K/V projection over [pixels ‖ Fourier PE] in factored form (csrc/pe_proj.hip): the PE part of
# LN(x)·Wᵀ is batch-independent, so it is one (M × Kin)·(Kin × O) GEMM per step and each sample
# only pays a bandwidth-bound epilogue.
PE_FACTORED = True


def _adjacent_rows(a: torch.Tensor, b: torch.Tensor):
    """(2N, K) view over two contiguous (N, K) tensors that lie back to back in one storage (e.g.
    the k / v projection gradients in the optimizer's flat buffer), else None."""
    if not (a.is_contiguous() and b.is_contiguous() and a.shape == b.shape and a.dim() == 2 and a.dtype == b.dtype):
        return None
    if a.untyped_storage().data_ptr() != b.untyped_storage().data_ptr():
        return None
    if b.data_ptr() != a.data_ptr() + a.numel() * a.element_size():
        return None
    return torch.as_strided(a, (2 * a.shape[0], a.shape[1]), (a.shape[1], 1))


def _pe_index(src):
    """(R,) int64 PE row of every K/V input row of a sparse source, else None."""
    if src is None or src.index is None:
        return None
    return src.index.reshape(-1)


def _pe_table(pe, nc: int, kin: int):
    """Step-invariant PE operands, cached ON the PE table tensor (so they live exactly as long as
    it does; refreshed if it is modified): the bf16 table Ebf (M, Kp) with only the PE columns
    [nc, kin) kept (Kp = kin rounded up to 32) and the row sums Σe, Σe² over those columns."""
    key = (pe._version, nc, kin)
    ent = getattr(pe, "_pio_pe_table", None)
    if ent is not None and ent[0] == key:
        return ent[1]
    kp = -(-kin // 32) * 32
    pe_e = pe[:, nc:kin]
    ebf = torch.zeros((pe.shape[0], kp), device=pe.device, dtype=torch.bfloat16)
    ebf[:, nc:kin] = pe_e.to(torch.bfloat16)
    tab = (ebf, pe_e.sum(1).contiguous(), (pe_e * pe_e).sum(1).contiguous())
    pe._pio_pe_table = (key, tab)
    return tab


def _pe_proj_fwd(K, pix, pe, g, b, W, bias):
    """pix (B·M, nc) pixel channels, pe (M, ≥Kin) padded PE table with zero pixel columns,
    g/b (Kin) kv_norm affine, W (O, Kin) fp32 K‖V weights, bias (O) → bf16 (B·M, O), mean, rstd.

    Per step: one weight-prep kernel (W⊙γ in bf16 + the epilogue vectors) and the in-tree MFMA
    GEMM P' = Ebf·(W⊙γ)ᵀ over the cached bf16 PE table (bf16 operands, fp32 accumulation: the
    precision of the bf16 K/V it feeds); then the per-sample epilogue (pe_proj_fwd)."""
    nc, kin = pix.shape[1], g.shape[0]
    ebf, pes, pesq = _pe_table(pe, nc, kin)
    O = W.shape[0]
    if O % 128 == 0 and hasattr(K, "pe_gemm"):
        wg, wpg, gw, bw = K.pe_weight_prep(W.contiguous(), g.contiguous(), b.contiguous(), bias.contiguous(), nc,
                                           ebf.shape[1])[:4]
        P = K.pe_gemm(ebf, wg)
    else:
        wg, wpg, gw, bw = emulation.pe_weight_prep(W, g, b, bias, nc, ebf.shape[1])[:4]
        P = torch.mm(ebf, wg.t()).float()
    return K.pe_proj_fwd(pix, P, pes, pesq, wpg, gw, bw, kin, EPS)


# implicit K/V for the encoder cross-attention over [pixels ‖ Fourier PE] (csrc/attention_pe.hip):
# both attention directions factor their products over the bf16 PE product P' = Ebf·(W⊙γ)ᵀ plus a
# per-sample augmentation from the sample's pixels and a per-column table, so the (B·M, 2C) K/V
# tensor (0.8 GB at ImageNet shape) is never written or read, nor any K/V tile formed.  PE_IMPLICIT = False selects the materialised factored path (tests).
PE_IMPLICIT = True


PE_PAD_ROWS = 64  # zero rows after P' (the forward kernel's last prefetch reads them)


def _pe_implicit_operands(K, nc, pe, g, b, W, bias):
    """(P' (M, 2C) bf16, Σe, Σe², column table (6, 2C), Kin) of one K/V projection; W = (W_k, W_v)
    (read in place by the weight prep kernel) or the stacked (2C, Kin) weight."""
    kin = g.shape[0]
    ebf, pes, pesq = _pe_table(pe, nc, kin)
    Wk, Wv = W if isinstance(W, tuple) else (W, None)
    O = Wk.shape[0] + (0 if Wv is None else Wv.shape[0])
    if O % 128 == 0 and hasattr(K, "pe_gemm"):
        wg, _, _, _, wt = K.pe_weight_prep(Wk.contiguous(), g.contiguous(), b.contiguous(), bias.contiguous(), nc,
                                           ebf.shape[1], None if Wv is None else Wv.contiguous())
        P = K.pe_gemm(ebf, wg, bf16_out=True, pad_rows=PE_PAD_ROWS)
    else:
        wg, _, _, _, wt = emulation.pe_weight_prep(Wk, g, b, bias, nc, ebf.shape[1], Wv)
        P = emulation.pe_gemm(ebf, wg, bf16_out=True, pad_rows=PE_PAD_ROWS)
    return P, pes, pesq, wt, kin




def _mm_tn_split(a, b):
    """aᵀ·b for tall a (M, K1), b (M, K2): the long contraction is split into batches of a
    bmm (split-K) so the small (K1 × K2) output still spreads over the whole GPU."""
    M = a.shape[0]
    s = max((d for d in range(1, 65) if M % d == 0 and M // d >= 256), default=1)
    if s == 1:
        return torch.mm(a.t(), b)
    return torch.bmm(a.reshape(s, M // s, a.shape[1]).transpose(1, 2), b.reshape(s, M // s, b.shape[1])).sum(0)


def _pe_proj_bwd(K, dy, pix, mean, rstd, pe, g, b, W, M):
    """Gradients of _pe_proj_fwd w.r.t. W, bias, g, b from one streaming pass over dy (B·M, O)."""
    D, part = K.pe_proj_bwd(dy, pix, mean, rstd, M)
    return _pe_proj_grads(D, part, pix.shape[1], pe, g, b, W)


# the encoder cross-attention backward folds dK/dV straight into the factored projection's
# reductions (csrc/attention_pe.hip): no fp32 (B·M, 2C) dK/dV tensor.
PE_ATTN_FUSED = True


def pe_attn_bsplit(B: int, M: int, H: int) -> int:
    """Batch groups of the fused PE attention backward: ≥ 512 workgroups when the image is small."""
    from . import deterministic

    if deterministic():  # batch groups would add into D with atomics
        return 1
    nkb = (M + 255) // 256
    return max(1, min(B, -(-512 // (nkb * H))))


def _pe_proj_grads(D, part, nc, pe, g, b, W):
    """W, bias, g, b gradients of the factored projection from its reductions
    D[m,o] = Σ_b dY·rσ and part rows [Σ dY | Σ dY·μ·rσ | Σ dY·x̂_c]:
    G[o,c] = Σ dY_o·x̂_c (pixel channels from the partials, PE channels = E_cᵀ·D − e),
    dW = G⊙γ + S⊗β, db = S, dγ = Σ_o W⊙G, dβ = Wᵀ·S."""
    kin, O = g.shape[0], D.shape[1]
    tot = part.sum(0)
    S, e, Gp = tot[:O], tot[O:2 * O], tot[2 * O:].view(nc, O)
    Ge = _mm_tn_split(pe, D)[nc:kin] - e[None, :]
    G = torch.cat([Gp, Ge], 0).t()  # (O, Kin)
    dW = G * g[None, :] + S[:, None] * b[None, :]
    return dW, S, (W * G).sum(0), torch.mv(W.t(), S)


_ZERO_STAND_INS = {}


def _zero_stand_in(r: int, c: int, device) -> torch.Tensor:
    """A persistent (r, c) fp32 zero tensor returned as an input gradient a later kernel overwrites
    in effect (it only adds it): never written, so one tensor serves every step (no fill launch;
    the reference kept here also stops autograd from accumulating into it in place)."""
    key = (r, c, str(device))
    t = _ZERO_STAND_INS.get(key)
    if t is None:
        t = _ZERO_STAND_INS[key] = torch.zeros((r, c), device=device, dtype=torch.float32)
    return t


def _cross_zero_bufs(ctx, device):
    """(zbuf, dq_pre, d_pre) of a fused cross-attention layer's backward: the attention backward's
    atomically accumulated dQ — and, for the first backward application of a PE layer whose batch
    groups add into its factored reduction D, that (M, 2C) buffer too; for the first application
    of a plain layer whose query splits add into dK / dV (many queries over few keys: the MLM
    decoder's selected positions over the latents), that (B, M, 2C) buffer — in one fp32 span
    that the kernel before the attention backward clears on the way (no fill launch);
    (None, None, None) for self-attention layers and in deterministic mode.  Broadcast latent
    queries on the fused PE path come back summed over the batch."""
    from . import deterministic

    if not ctx.spec.cross or deterministic():
        return None, None, None
    B, Bq, Nq, C, H, D, scale = ctx.dims
    pe_fused, pm = ctx.zplan
    f32 = dict(device=device, dtype=torch.float32)
    nq = (Bq if pe_fused else B) * Nq * C
    d_pre = None
    K = ext.require() if torch.device(device).type == "cuda" else emulation
    if pe_fused and ctx.kv_entry.get("pe_D") is None and pe_attn_bsplit(B, pm, H) > 1:
        zbuf = torch.empty(nq + pm * 2 * C, **f32)
        d_pre = zbuf[nq:].view(pm, 2 * C)
    elif (not pe_fused and ctx.kv_entry.get("dkv") is None and hasattr(K, "attn_bwd_zero_plan")
          and int(K.attn_bwd_zero_plan(B, H, Nq, pm, D)) & 2):
        zbuf = torch.empty(nq + B * pm * 2 * C, **f32)
        d_pre = zbuf[nq:].view(B, pm, 2 * C)
    else:
        zbuf = torch.empty(nq, **f32)
    return zbuf, zbuf[:nq].view(-1, Nq, C), d_pre


class _LayerFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, spec: LayerSpec, bw, seed, p_attn, src, x_q, x_kv, kmask, *ps):
        K = kernels(x_q)
        # broadcast queries that are a leaf parameter's (1, N, C) view (the encoder's latent array):
        # the backward adds their gradient straight into the parameter's gradient buffer (no
        # autograd AccumulateGrad add kernel) — only when that buffer is an optimizer's flat
        # gradient view (FlatParameterSpace sets _pio_flat); otherwise the gradient goes back
        # through autograd, so torch.autograd.grad(..., inputs=[latent]) and hooks still work
        base = x_q._base
        ctx.q_leaf = (base if spec.cross and base is not None and base.is_leaf and base.requires_grad
                      and getattr(base, "_pio_flat", False)
                      and x_q.shape[0] == 1 and tuple(base.shape) == tuple(x_q.shape[1:]) else None)
        C, H = spec.C, spec.heads
        D = C // H
        scale = 1.0 / math.sqrt(D)
        wq, wkv, wo, w1, w2 = bw
        if spec.cross:
            g_q, b_q, g_kv, b_kv = ps[0:4]
            rest = ps[5:] if spec.packed else ps[7:]
        else:
            g_q, b_q = ps[0:2]
            rest = ps[3:]
        bin_, _, bo, g2, be2, _, b1, _, b2 = rest
        Bq, Nq = x_q.shape[0], x_q.shape[1]
        xq2 = x_q.reshape(Bq * Nq, C)
        if not xq2.is_contiguous():
            xq2 = xq2.contiguous()
        if spec.cross:
            B, M = x_kv.shape[0], x_kv.shape[1]
            xkv2 = x_kv.reshape(B * M, x_kv.shape[2])
            hq = _LOOKAHEAD["have_q"]
            if hq is not None and hq[4] is g_q and hq[0].data_ptr() == xq2.data_ptr() and hq[0].numel() == xq2.numel():
                # LN + query projection computed by the producing self-attention block's last kernel
                q, mean_q, rstd_q = hq[1:4]
                _LOOKAHEAD["have_q"] = None
                ctx.q_handoff = True
            else:
                q, mean_q, rstd_q = K.ln_linear_fwd(xq2, g_q, b_q, EPS, wq, bin_[:C], 0, None, True, True)
            key = id(ps[0])
            ent = src.entries.get(key) if src is not None else None
            ctx.kv_owner = ent is None
            if ent is None:  # first application of this layer: project K/V (LN over [pixels ‖ PE] if split)
                kv_sb = False
                factored = (PE_FACTORED and src is not None and src.pe is not None and src.index is None
                            and not spec.packed
                            and not ctx.needs_input_grad[6] and 1 <= xkv2.shape[1] <= 4 and 2 * C <= 512)
                implicit = (factored and PE_IMPLICIT and PE_ATTN_FUSED and D == 32 and Nq <= 32 and kmask is None
                            and p_attn == 0.0 and hasattr(K, "attn_fwd_pe"))
                imp = None
                if implicit:
                    imp = _pe_implicit_operands(K, xkv2.shape[1], src.pe, g_kv, b_kv, (ps[5], ps[6]), bin_[C:])
                    kv = mean_kv = rstd_kv = None
                elif factored:
                    kv, mean_kv, rstd_kv = _pe_proj_fwd(K, xkv2, src.pe, g_kv, b_kv,
                                                        torch.cat([ps[5], ps[6]], 0), bin_[C:])
                else:
                    if wkv is None:
                        wkv = _kv_weight(spec, ps)
                    hk = _LOOKAHEAD["have_q"]
                    if (src is None and hk is not None and hk[4] is g_kv and hk[0].data_ptr() == xkv2.data_ptr()
                            and hk[0].numel() == xkv2.numel()):
                        # K/V of a decoder over the encoder output: computed by the encoder's last
                        # self-attention kernel.  Its backward stays here (plain ln_linear_bwd) unless
                        # that kernel was a per-sample block offering to run it (hk[5])
                        kv, mean_kv, rstd_kv = hk[1:4]
                        kv_sb = len(hk) > 5 and bool(hk[5]) and spec.packed and ctx.needs_input_grad[6]
                        _LOOKAHEAD["have_q"] = None
                    else:
                        kv, mean_kv, rstd_kv = K.ln_linear_fwd(xkv2, g_kv, b_kv, EPS, wkv, bin_[C:], 0, None, True,
                                                               True, src.pe if src is not None else None,
                                                               g_kv.shape[0], _pe_index(src))
                ent = {"kv": kv, "mean": mean_kv, "rstd": rstd_kv, "dkv": None, "factored": factored, "wkv": wkv,
                       "implicit": imp, "sb_bwd": kv_sb}
                if src is not None:
                    src.entries[key] = ent
            kv, mean_kv, rstd_kv = ent["kv"], ent["mean"], ent["rstd"]
            ctx.kv_entry = ent
            # the backward's accumulator plan (known here so a following per-sample block that runs
            # this layer's post-attention backward can clear the accumulators: _cross_zero_bufs)
            ctx.zplan = (bool(ent.get("factored") and PE_ATTN_FUSED and D == 32 and Nq <= 32 and kmask is None
                              and p_attn == 0.0 and xkv2.shape[1] <= 4),
                         ent["implicit"][1].shape[0] if ent.get("implicit") is not None else ent["kv"].shape[0] // B)
            ctx.kv_pe = src.pe if src is not None else None
            ctx.kv_pe_index = _pe_index(src)
            q3 = q.view(Bq, Nq, C)
            if ent.get("implicit") is None:
                kv3 = kv.view(B, M, 2 * C)
                k3, v3 = kv3[:, :, :C], kv3[:, :, C:]
        else:
            B = Bq
            qkv, mean_q, rstd_q = K.ln_linear_fwd(xq2, g_q, b_q, EPS, wq, bin_, 0, None, True, True)
            qkv3 = qkv.view(B, Nq, 3 * C)
            q3, k3, v3 = qkv3[:, :, :C], qkv3[:, :, C:2 * C], qkv3[:, :, 2 * C:]
            xkv2 = kv = mean_kv = rstd_kv = None
        from .attention import pick_splits

        imp = ent.get("implicit") if spec.cross else None
        if imp is not None:
            P, pes, pesq, wt, kin = imp
            o, lse = K.attn_fwd_pe(q3, P, xkv2, pes, pesq, wt, H, scale, kin, EPS, 0)  # 0: one round of waves
        else:
            nsplit = pick_splits(B, H, Nq, k3.shape[1], p_attn > 0)
            o, lse = K.attn_fwd(q3, k3, v3, kmask, H, D, scale, p_attn, seed, nsplit)
        o2 = o.view(B * Nq, C)
        # a batch-broadcast query stream (Bq = 1) is added as the residual without expanding it;
        # residual dropout (p_attn: the layer's one dropout rate) in the kernel epilogues
        nxt, _LOOKAHEAD["want"] = _LOOKAHEAD["want"], None
        want_pa, _LOOKAHEAD["want_pa"] = _LOOKAHEAD["want_pa"], None
        if (want_pa and spec.cross and nxt is None and p_attn == 0.0 and Nq == 32 and H == 4 and Bq in (1, B)
                and o2.is_contiguous()):  # 4 heads: δ in the block's head layout
            # the following per-sample block (_SampleBlockFn) runs this layer's post-attention half
            # as the prologue of its kernels, forward and backward: z is its placeholder, written
            # by that block's forward before anything reads it
            z = torch.empty((B * Nq, C), device=o2.device, dtype=torch.float32)
            _LOOKAHEAD["have_pa"] = dict(key=z.data_ptr(), ctx=ctx, pre=[o2, xq2, wo, bo, g2, be2, w1, b1, w2, b2],
                                         ps=(rest[1], bo, g2, be2, rest[5], b1, rest[7], b2))
            ctx.pa_key = z.data_ptr()
            y = m2 = r2 = u = torch.empty(0, device=o2.device)
        elif nxt is not None and spec.cross:
            # the following self-attention block's LN1 + QKV projection in the same launch (its
            # forward picks the result up instead of launching ln_linear_fwd)
            z, y, m2, r2, u, qkv_n, mean_n, rstd_n = K.post_attn_ln_linear_fwd(
                o2, xq2, wo, bo, g2, be2, EPS, w1, b1, w2, b2, nxt[0], nxt[1], nxt[2], nxt[3], seed=seed, p=p_attn)
            _LOOKAHEAD["have"] = (z, qkv_n, mean_n, rstd_n, nxt[0])
            ctx.lookahead_z = z.data_ptr()  # the block's backward hands its LN1/QKV backward back here
        else:
            z, y, m2, r2, u = K.post_attn_fwd(o2, xq2, wo, bo, g2, be2, EPS, w1, b1, w2, b2, seed=seed, p=p_attn)
        ctx.spec, ctx.bw, ctx.seed, ctx.p_attn = spec, bw, seed, p_attn
        ctx.src = src if spec.cross else None
        ctx.dims = (B, Bq, Nq, C, H, D, scale)
        ctx.kv_grad = x_kv is not None and ctx.needs_input_grad[6]
        ctx.has_mask = kmask is not None
        ctx.save_for_backward(xq2, xkv2 if xkv2 is not None else torch.empty(0), q3 if spec.cross else qkv,
                              kv if kv is not None else torch.empty(0), o, lse, y, m2, r2, u, mean_q, rstd_q,
                              mean_kv if mean_kv is not None else torch.empty(0),
                              rstd_kv if rstd_kv is not None else torch.empty(0),
                              kmask if kmask is not None else torch.empty(0), *ps)
        return z.view(B, Nq, C)

    @staticmethod
    def backward(ctx, dz):
        K = kernels(dz)
        spec = ctx.spec
        B, Bq, Nq, C, H, D, scale = ctx.dims
        (xq2, xkv2, qx, kv, o, lse, y, m2, r2, u, mean_q, rstd_q, mean_kv, rstd_kv, kmask, *ps) = ctx.saved_tensors
        kmask = kmask if ctx.has_mask else None
        wq, wkv, wo, w1, w2 = ctx.bw
        if spec.cross:
            g_q, b_q, g_kv, b_kv = ps[0:4]
            rest = ps[5:] if spec.packed else ps[7:]
            ibias = 5 if spec.packed else 7
            if wkv is None:
                wkv = ctx.kv_entry.get("wkv")
        else:
            g_q, b_q = ps[0:2]
            rest = ps[3:]
            ibias = 3
        bin_, Wo, bo, g2, be2, W1, b1, W2, b2 = rest
        dz2 = dz.reshape(B * Nq, C)
        if not dz2.is_contiguous():
            dz2 = dz2.contiguous()
        o2 = o.view(B * Nq, C)
        R = B * Nq
        f32 = dict(device=dz.device, dtype=torch.float32)
        scratch = {}

        # gradient targets: the parameter's replicated accumulator (8, numel) when the flat
        # parameter space gave it one (ops/optim.py), else its .grad; frozen parameters get a
        # throw-away buffer of the same kind.  All targets of one kernel call share the kind.
        rep_mode = any(getattr(p, "_pio_grad_rep", None) is not None for p in ps if p.requires_grad)

        def gb(p):
            if not p.requires_grad:
                t = scratch.get(id(p))
                if t is None:
                    shape = (8, p.numel()) if rep_mode else p.shape
                    t = scratch[id(p)] = torch.zeros(shape, **f32)
                return t
            if rep_mode:
                return p._pio_grad_rep
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            return p.grad

        def rows(t, a, b, width):
            """rows [a, b) of an (N, width) gradient target (plain or replicated)."""
            return t[:, a * width:b * width] if rep_mode else t[a:b]

        def flat(p, a=None, b=None):
            """final gradient destination p.grad (flattened [a:b]); None if p is frozen."""
            g = _grad_of(p)
            return None if g is None else g.view(-1)[a:b]

        drop = dict(seed=ctx.seed, p=ctx.p_attn)
        # the cross-attention backward's dQ accumulator (atomic key-block partials) is cleared by
        # the post-attention backward kernel on the way (no fill launch on the chain)
        from . import deterministic

        pe_fused = spec.cross and ctx.zplan[0]
        pa = None
        if getattr(ctx, "pa_key", None) is not None:
            pa, _LOOKAHEAD["bwd_pa"] = _LOOKAHEAD["bwd_pa"], None
            if pa is None or pa["key"] != ctx.pa_key:
                raise RuntimeError("fused encoder: the per-sample block that ran this cross-attention layer's "
                                   "post-attention half did not hand its backward back")
            zbuf, dq_pre, d_pre = pa["zbuf"]  # cleared by that block's backward kernel
        else:
            zbuf, dq_pre, d_pre = _cross_zero_bufs(ctx, dz.device)
        if zbuf is not None and pa is None:
            drop["zero_out"] = zbuf
        ho, _LOOKAHEAD["bwd"] = _LOOKAHEAD["bwd"], None
        if ho is not None and ho["key"] != getattr(ctx, "lookahead_z", None):
            raise RuntimeError("fused encoder: a self-attention block handed its LN1/QKV backward to the wrong "
                               "cross-attention layer")
        if pa is not None:
            if ho is not None:
                raise RuntimeError("fused encoder: a cross-attention layer with two backward hand-offs")
            # post-attention backward done by the block: dY (the residual path) arrives as dz
            dy, do, delta = dz2, pa["do"], pa["delta"]
        elif ho is not None:
            # the following block's first LN1/QKV backward (its dX = this layer's dZ) and this
            # layer's post-attention backward in one launch; both weight-gradient sets in one slab
            sl = _GradSlab(R, LL_SIZES(C) + PA_SIZES(C), dz2)
            tg = sl.targets()
            dy, do, delta = K.ln_linear_post_attn_bwd(ho["g"], ho["wq"], ho["x"], ho["mean1"], ho["rstd1"], ho["lnw"],
                                                      ho["lnb"], ho["dres"], tg[:4], y, m2, r2, u, o2, wo, w1, w2, g2,
                                                      be2, H, tg[4:], **_take_job(), **drop)
            sl.defer(K, ho["ll_dsts"] + [flat(p) for p in (Wo, bo, g2, be2, W1, b1, W2, b2)])
        elif WGRAD_SLAB and R < TALL_ROWS:
            sl = _GradSlab(R, [C * C, C, C, C, C * C, C, C * C, C], dz2)
            dy, do, delta = K.post_attn_bwd(dz2, y, m2, r2, u, o2, wo, w1, w2, g2, be2, H, sl.targets(), slab=True,
                                            **_take_job(), **drop)
            sl.defer(K, [flat(p) for p in (Wo, bo, g2, be2, W1, b1, W2, b2)])
        else:
            dy, do, delta = K.post_attn_bwd(dz2, y, m2, r2, u, o2, wo, w1, w2, g2, be2, H,
                                            [gb(Wo), gb(bo), gb(g2), gb(be2), gb(W1), gb(b1), gb(W2), gb(b2)], **drop)
        delta3 = delta.view(B, Nq, H)
        # --- attention backward + input-side projections (weight grads fused into ln_linear_bwd) ----
        if spec.cross:
            ent = ctx.kv_entry
            imp = ent.get("implicit")
            M = imp[1].shape[0] if imp is not None else kv.shape[0] // B
            kv3 = kv.view(B, M, 2 * C) if imp is None else None
            if pe_fused:
                # dK/dV folded into the factored projection's reductions (D, partials), which every
                # application of this layer accumulates (attention_pe.hip): no dK/dV tensor
                acc = ent.get("pe_D") is not None
                if not acc:
                    bs = pe_attn_bsplit(B, M, H)
                    ent["pe_D"] = d_pre if d_pre is not None else torch.empty((M, 2 * C), **f32)
                    prows = (K.attn_bwd_pe_part_rows(M, H, B, bs) if hasattr(K, "attn_bwd_pe_part_rows")
                             else ((M + 255) // 256) * bs)
                    ent["pe_part"] = torch.empty((prows, (2 + xkv2.shape[1]) * 2 * C), **f32)
                    ent["pe_bsplit"] = bs
                # broadcast latent queries (layer_1): dq comes back summed over the batch
                dq = dq_pre if dq_pre is not None else torch.empty((Bq, Nq, C), **f32)
                if imp is not None:
                    P, pes, pesq, wt, kin = imp
                    K.attn_bwd_pe_implicit(qx, P, pes, pesq, wt, do.view(B, Nq, C), lse, delta3, xkv2, dq, ent["pe_D"],
                                           ent["pe_part"], H, scale, kin, EPS, acc, ent["pe_bsplit"],
                                           dq_zeroed=dq_pre is not None, d_zeroed=d_pre is not None)
                else:
                    K.attn_bwd_pe(qx, kv, do.view(B, Nq, C), lse, delta3, mean_kv, rstd_kv, xkv2, dq, ent["pe_D"],
                                  ent["pe_part"], H, scale, acc, ent["pe_bsplit"], dq_zeroed=dq_pre is not None,
                                  d_zeroed=d_pre is not None)
            else:
                # dK/dV of every application of this layer land in one buffer (K-06); the first
                # writer stores, later ones accumulate
                acc = ent["dkv"] is not None
                kv_pre = not acc and d_pre is not None and d_pre.dim() == 3  # cleared with dQ (_cross_zero_bufs)
                if not acc:
                    ent["dkv"] = d_pre if kv_pre else torch.empty((B, M, 2 * C), **f32)
                dkv = ent["dkv"]
                dq, _, _ = K.attn_bwd(qx, kv3[:, :, :C], kv3[:, :, C:], kmask, o, do.view(B, Nq, C), lse, delta3, H,
                                      D, scale, ctx.p_attn, ctx.seed, dq_pre, dkv[:, :, :C], dkv[:, :, C:], acc,
                                      dq_zeroed=dq_pre is not None, kv_zeroed=kv_pre)
            # the latent array's gradient, written by the kernels below in place: += Σ_b dY by the
            # batch sum, then dX = LN_bwd(·) + that into the same buffer
            leaf_g = None
            if ctx.q_leaf is not None and Bq == 1 and B > 1 and not getattr(ctx, "q_handoff", False):
                leaf_g = _grad_of(ctx.q_leaf)
                if leaf_g is not None and not (leaf_g.is_contiguous() and leaf_g.data_ptr() % 16 == 0):
                    leaf_g = None
            if Bq == 1 and B > 1 and dq.shape[0] == B:
                # broadcast latent queries: both batch sums in one deterministic kernel
                dq2, dres = K.batch_sum2(dq.contiguous(), dy.view(B, Nq, C), ob_acc=leaf_g)
            elif Bq == 1 and B > 1:  # dq already summed (fused pe path)
                dq2 = dq.reshape(Nq, C)
                _, dres = K.batch_sum2(None, dy.view(B, Nq, C).contiguous(), ob_acc=leaf_g)
            else:
                dq2, dres = dq.reshape(B * Nq, C), dy
            q_out = dict(dx_out=dres.view(Nq, C)) if leaf_g is not None else {}
            Ckv = g_kv.shape[0]
            Rq = dq2.shape[0]
            if getattr(ctx, "q_handoff", False):
                # the producing self-attention block runs this LN + query-projection backward
                # fused with its last post-attention backward; dres stands in for dx_q (same
                # shape, no fill launch) and is ignored by that block
                _LOOKAHEAD["bwd_q"] = dict(key=xq2.data_ptr(), g=dq2.contiguous(), wq=wq, x=xq2, mean1=mean_q,
                                           rstd1=rstd_q, lnw=g_q, lnb=b_q, dres=dres.contiguous(),
                                           ll_dsts=[flat(g_q), flat(b_q), flat(ps[4], 0, C * C), flat(bin_, 0, C)])
                dx_q = dres
            elif WGRAD_SLAB and Rq < TALL_ROWS:
                sl = _GradSlab(Rq, [C, C, C * C, C], dz2)
                dx_q = K.ln_linear_bwd(dq2, wq, xq2, mean_q, rstd_q, g_q, b_q, dres, True, *sl.targets(), slab=True,
                                       **_take_job(), **q_out)
                sl.defer(K, [flat(g_q), flat(b_q), flat(ps[4], 0, C * C), flat(bin_, 0, C)])
            else:
                gwq = rows(gb(ps[4]), 0, C, C) if spec.packed else gb(ps[4])
                dx_q = K.ln_linear_bwd(dq2, wq, xq2, mean_q, rstd_q, g_q, b_q, dres, True, gb(g_q), gb(b_q), gwq,
                                       rows(gb(bin_), 0, C, 1), **q_out)
            dx_kv = None
            if ctx.kv_owner and ent.get("sb_bwd") and ent.get("pe_D") is None:
                # a decoder's K/V projected by the encoder's last per-sample block: that block runs
                # this LN + K|V projection backward first in its own backward (sample_block.hip post
                # stage, 2C wide) and the gradient of its output arrives there; the input gradient
                # returned here is a zero stand-in the block adds (no fill launch)
                _LOOKAHEAD["bwd_q"] = dict(key=xkv2.data_ptr(), g=dkv.view(B * M, 2 * C), dres=None,
                                           ll_dsts=[flat(g_kv), flat(b_kv), flat(ps[4], C * C, 3 * C * C),
                                                    flat(bin_, C, 3 * C)])
                dx_kv = _zero_stand_in(B * M, Ckv, dkv.device)
                ent["dkv"] = None
            elif ctx.kv_owner:  # the projection's backward, once, over the summed dK/dV
                if ent.get("pe_D") is not None:
                    dkv2, Rkv = None, B * M
                else:
                    dkv2 = dkv.view(B * M, 2 * C)
                    Rkv = dkv2.shape[0]
                if ent.get("factored"):
                    # (D, partials) from the fused attention backward or a pe_proj_bwd pass, then
                    # the weight / LN gradients in three kernels, added straight into the targets
                    if ent.get("pe_D") is not None:
                        Dm, part = ent["pe_D"], ent["pe_part"]
                    else:
                        Dm, part = K.pe_proj_bwd(dkv2, xkv2, mean_kv, rstd_kv, M)
                    nc = xkv2.shape[1]
                    ebf = _pe_table(ctx.kv_pe, nc, g_kv.shape[0])[0]

                    def tg(p):
                        t = gb(p)
                        return t[0] if rep_mode else t

                    gbias = gb(bin_)
                    K.pe_grads(Dm, part, ebf, ps[5].detach(), ps[6].detach(), g_kv.detach(), b_kv.detach(), nc,
                               tg(ps[5]), tg(ps[6]), gbias[0, C:3 * C] if rep_mode else gbias[C:3 * C], tg(g_kv),
                               tg(b_kv))
                elif WGRAD_SLAB and Rkv < TALL_ROWS:
                    sl = _GradSlab(Rkv, [Ckv, Ckv, 2 * C * Ckv, 2 * C], dz2)
                    src = ctx.src
                    chain = src is not None and ctx.kv_grad and ctx.kv_pe is None
                    if chain and src.owners_left is None:
                        src.owners_left = len(src.entries)
                    dx_kv = K.ln_linear_bwd(dkv2, wkv, xkv2, mean_kv, rstd_kv, g_kv, b_kv,
                                            src.pending_dx if chain else None, ctx.kv_grad,
                                            *sl.targets(), ctx.kv_pe, Ckv, slab=True, pe_index=ctx.kv_pe_index,
                                            **_take_job())
                    if chain:  # hand the partial input gradient on; the last projection returns it
                        src.owners_left -= 1
                        if src.owners_left > 0:
                            src.pending_dx, dx_kv = dx_kv, None
                        else:
                            src.pending_dx = src.owners_left = None
                    if spec.packed:
                        dwkv = flat(ps[4], C * C, 3 * C * C)
                    else:
                        gk, gv = flat(ps[5]), flat(ps[6])
                        dwkv = [(t, o) for t, o in ((gk, 0), (gv, C * Ckv)) if t is not None] or None
                    sl.defer(K, [flat(g_kv), flat(b_kv), dwkv, flat(bin_, C, 3 * C)])
                else:
                    gbias = gb(bin_)
                    sep = False
                    if spec.packed:
                        gwkv = rows(gb(ps[4]), C, 3 * C, C)
                    else:
                        gwkv = None if rep_mode else _adjacent_rows(gb(ps[5]), gb(ps[6]))
                        sep = gwkv is None
                        if sep:
                            gwkv = torch.zeros((8, 2 * C * Ckv) if rep_mode else (2 * C, Ckv), **f32)
                    dx_kv = K.ln_linear_bwd(dkv2, wkv, xkv2, mean_kv, rstd_kv, g_kv, b_kv, None, ctx.kv_grad,
                                            gb(g_kv), gb(b_kv), gwkv, rows(gbias, C, 3 * C, 1), ctx.kv_pe, Ckv,
                                            pe_index=ctx.kv_pe_index)
                    if sep:
                        gb(ps[5]).add_(rows(gwkv, 0, C, Ckv))
                        gb(ps[6]).add_(rows(gwkv, C, 2 * C, Ckv))
                ent["dkv"] = ent["pe_D"] = ent["pe_part"] = None
            dx_q = None if leaf_g is not None else dx_q.view(Bq, Nq, C)  # already in the leaf's gradient
            dx_kv = dx_kv.view(B, M, -1) if (ctx.kv_grad and dx_kv is not None) else None
        else:
            qkv3 = qx.view(B, Nq, 3 * C)
            dqkv = torch.empty((B, Nq, 3 * C), **f32)  # every column block is written by attn_bwd
            K.attn_bwd(qkv3[:, :, :C], qkv3[:, :, C:2 * C], qkv3[:, :, 2 * C:], kmask, o, do.view(B, Nq, C), lse,
                       delta3, H, D, scale, ctx.p_attn, ctx.seed, dqkv[:, :, :C], dqkv[:, :, C:2 * C],
                       dqkv[:, :, 2 * C:])
            if WGRAD_SLAB and R < TALL_ROWS:
                sl = _GradSlab(R, [C, C, 3 * C * C, 3 * C], dz2)
                dx_q = K.ln_linear_bwd(dqkv.view(R, 3 * C), wq, xq2, mean_q, rstd_q, g_q, b_q, dy, True, *sl.targets(),
                                       slab=True, **_take_job())
                sl.defer(K, [flat(g_q), flat(b_q), flat(ps[2]), flat(ps[3])])
            else:
                dx_q = K.ln_linear_bwd(dqkv.view(R, 3 * C), wq, xq2, mean_q, rstd_q, g_q, b_q, dy, True, gb(g_q),
                                       gb(b_q), gb(ps[2]), gb(ps[3]))
            dx_q = dx_q.view(B, Nq, C)
            dx_kv = None
        # parameter gradients were accumulated in place (no autograd AccumulateGrad pass)
        return (None, None, None, None, None, dx_q, dx_kv, None) + (None,) * len(ps)


# the fused latent self-attention layer forward (chain.hip sa_layer_fwd_chain8_kernel);
# PERCEIVER_SA_LAYER_FUSED=0 restores attn_fwd + post_attn(_ln_linear)_fwd
SA_LAYER_FUSED = True
PA_SIZES = lambda C: [C * C, C, C, C, C * C, C, C * C, C]  # noqa: E731  (Wo bo γ2 β2 W1 b1 W2 b2)
LL_SIZES = lambda C: [C, C, 3 * C * C, 3 * C]                 # noqa: E731  (γ1 β1 Wqkv bqkv)
SA_NP = 12  # parameters per self-attention layer (layer_spec_and_params order)
# the fused C = 64 stacks with N <= 256 latents run every layer of a block in ONE persistent launch
# (csrc/persist.hip); False: one launch per layer (chain.hip; the N = 512 path, and the reference the
# persistent kernel is bitwise checked against in tests/test_persist_gpu.py).  Same-box A/B, round 6:
# 1.342 / 1.346 ms per headline step against 1.372 / 1.373 with the per-layer launches
PERSIST_BLOCK = True
# channel widths run as one fused self-attention block node (PERCEIVER_SA_BLOCK_C128=0 keeps C = 128
# stacks layer by layer)
SA_BLOCK_CHANNELS = (32, 64, 128)


class _SABlockFn(torch.autograd.Function):
    """A whole self-attention block (reference ``model.py:43-44``: ``num_layers`` self-attention
    layers) as ONE autograd node, so that the row-local kernels of adjacent layers fuse across
    the layer boundary:

        forward : ln_linear(0) → [attn(l) → post_attn(l)+ln_linear(l+1)]… → attn(L-1) → post_attn(L-1)
        backward: post_attn_bwd(L-1) → [attn_bwd(l) → ln_linear_bwd(l)+post_attn_bwd(l-1)]… → attn_bwd(0)
                  → ln_linear_bwd(0)

    i.e. 2L+1 launches each way instead of 3L; the residual stream between layers never
    leaves registers at a boundary.  Weight gradients go through per-tile slabs (slab jobs)."""

    @staticmethod
    def forward(ctx, specs, bws, seed, pdrop, x, *ps):
        K = kernels(x)
        L = len(specs)
        spec = specs[0]
        C, H = spec.C, spec.heads
        D = C // H
        scale = 1.0 / math.sqrt(D)
        B, N = x.shape[0], x.shape[1]
        R = B * N
        from .attention import pick_splits

        nsplit = pick_splits(B, H, N, N)
        P = [ps[SA_NP * i:SA_NP * (i + 1)] for i in range(L)]
        xl = x.reshape(R, C)
        if not xl.is_contiguous():
            xl = xl.contiguous()
        have, _LOOKAHEAD["have"] = _LOOKAHEAD["have"], None
        if (have is not None and have[4] is P[0][0] and have[0].data_ptr() == xl.data_ptr()
                and have[0].numel() == xl.numel()):
            qkv, mean1, rstd1 = have[1:4]  # computed by the preceding cross-attention layer's kernel
            ctx.handoff = xl.data_ptr()
        else:
            qkv, mean1, rstd1 = K.ln_linear_fwd(xl, P[0][0], P[0][1], EPS, bws[0][0], P[0][3], 0, None, True, True)
        saved = []
        # one fused launch per layer (attention + post-attention + next LN1/QKV) for the
        # C = 64, H = 4 latent stacks, attention-probability dropout included (csrc/chain.hip
        # sa_layer_fwd_chain8_kernel: up to 512 latents)
        fused_layer = SA_LAYER_FUSED and C == 64 and H == 4 and N <= 512 and N % 64 == 0
        res = None
        if fused_layer and PERSIST_BLOCK and N <= 256 and hasattr(K, "sa_block_fwd"):
            wantq = _LOOKAHEAD["want_q"]
            nxt = [(P[i + 1][0], P[i + 1][1], bws[i + 1][0], P[i + 1][3]) for i in range(L - 1)]
            if wantq is not None:  # the following cross-attention layer's LN + query projection
                nxt.append(tuple(wantq[:4]))
            res = K.sa_block_fwd(qkv, xl, N, scale, EPS, [b[2] for b in bws], [p[5] for p in P], [p[6] for p in P],
                                 [p[7] for p in P], [b[3] for b in bws], [p[9] for p in P], [b[4] for b in bws],
                                 [p[11] for p in P], [n[0] for n in nxt], [n[1] for n in nxt], [n[2] for n in nxt],
                                 [n[3] for n in nxt], seed=seed, p=pdrop)
        if res:
            k = 0
            for i in range(L):
                o, lse, z, y, m2, r2, u = res[k:k + 7]
                k += 7
                qkv_n = mean_n = rstd_n = None
                if i < len(nxt):
                    qkv_n, mean_n, rstd_n = res[k:k + 3]
                    k += 3
                saved += [xl, qkv, mean1, rstd1, o, lse, y, m2, r2, u]
                if i == L - 1 and wantq is not None:
                    _LOOKAHEAD["want_q"] = None
                    _LOOKAHEAD["have_q"] = (z, qkv_n, mean_n, rstd_n, wantq[0])
                    ctx.out_ptr = z.data_ptr()
                    qkv_n = mean_n = rstd_n = None
                xl, qkv, mean1, rstd1 = z, qkv_n, mean_n, rstd_n
        for i in range(L if not res else 0):
            p = P[i]
            _, _, wo, w1, w2 = bws[i]
            bo, g2, be2, b1, b2 = p[5], p[6], p[7], p[9], p[11]
            if fused_layer:
                if i + 1 < L:
                    pn = P[i + 1]
                    o, lse, z, y, m2, r2, u, qkv_n, mean_n, rstd_n = K.sa_layer_fwd(
                        qkv, xl, N, scale, wo, bo, g2, be2, EPS, w1, b1, w2, b2, pn[0], pn[1], bws[i + 1][0], pn[3],
                        seed=seed, site=i, p=pdrop)
                else:
                    wantq, _LOOKAHEAD["want_q"] = _LOOKAHEAD["want_q"], None
                    if wantq is not None:  # the following cross-attention layer's LN + query projection
                        o, lse, z, y, m2, r2, u, qn, mq, rq = K.sa_layer_fwd(
                            qkv, xl, N, scale, wo, bo, g2, be2, EPS, w1, b1, w2, b2, wantq[0], wantq[1], wantq[2],
                            wantq[3], seed=seed, site=i, p=pdrop)
                        _LOOKAHEAD["have_q"] = (z, qn, mq, rq, wantq[0])
                        ctx.out_ptr = z.data_ptr()
                    else:
                        o, lse, z, y, m2, r2, u = K.sa_layer_fwd(qkv, xl, N, scale, wo, bo, g2, be2, EPS, w1, b1, w2,
                                                                 b2, seed=seed, site=i, p=pdrop)
                    qkv_n = mean_n = rstd_n = None
                saved += [xl, qkv, mean1, rstd1, o, lse, y, m2, r2, u]
                xl, qkv, mean1, rstd1 = z, qkv_n, mean_n, rstd_n
                continue
            qkv3 = qkv.view(B, N, 3 * C)
            # layer i of the block draws its masks from site i of the block's device seed
            o, lse = K.attn_fwd(qkv3[:, :, :C], qkv3[:, :, C:2 * C], qkv3[:, :, 2 * C:], None, H, D, scale, pdrop, seed,
                                nsplit, site=i)
            o2 = o.view(R, C)
            if i + 1 < L:
                pn = P[i + 1]
                z, y, m2, r2, u, qkv_n, mean_n, rstd_n = K.post_attn_ln_linear_fwd(
                    o2, xl, wo, bo, g2, be2, EPS, w1, b1, w2, b2, pn[0], pn[1], bws[i + 1][0], pn[3],
                    seed=seed, site=i, p=pdrop)
            else:
                z, y, m2, r2, u = K.post_attn_fwd(o2, xl, wo, bo, g2, be2, EPS, w1, b1, w2, b2, seed=seed, site=i, p=pdrop)
                qkv_n = mean_n = rstd_n = None
            saved += [xl, qkv, mean1, rstd1, o, lse, y, m2, r2, u]
            xl, qkv, mean1, rstd1 = z, qkv_n, mean_n, rstd_n
        ctx.specs, ctx.bws, ctx.dims = specs, bws, (B, N, C, H, D, scale)
        ctx.seed, ctx.p = seed, pdrop
        ctx.save_for_backward(*saved, *ps)
        return xl.view(B, N, C)

    @staticmethod
    def backward(ctx, dz):
        K = kernels(dz)
        B, N, C, H, D, scale = ctx.dims
        R = B * N
        L = len(ctx.specs)
        bws = ctx.bws
        t = ctx.saved_tensors
        S = [t[10 * i:10 * (i + 1)] for i in range(L)]
        ps = t[10 * L:]
        P = [ps[SA_NP * i:SA_NP * (i + 1)] for i in range(L)]
        f32 = dict(device=dz.device, dtype=torch.float32)

        def flat(p):
            g = _grad_of(p)
            return None if g is None else g.view(-1)

        def pa_dsts(p):  # Wo bo γ2 β2 W1 b1 W2 b2
            return [flat(p[4]), flat(p[5]), flat(p[6]), flat(p[7]), flat(p[8]), flat(p[9]), flat(p[10]), flat(p[11])]

        def ll_dsts(p):  # γ1 β1 Wqkv bqkv
            return [flat(p[0]), flat(p[1]), flat(p[2]), flat(p[3])]

        def pa_args(i):
            xl, qkv, mean1, rstd1, o, lse, y, m2, r2, u = S[i]
            _, _, wo, w1, w2 = bws[i]
            return (y, m2, r2, u, o.view(R, C), wo, w1, w2, P[i][6], P[i][7])

        def drop(i):
            return dict(seed=ctx.seed, site=i, p=ctx.p)

        dz2 = dz.reshape(R, C)
        if not dz2.is_contiguous():
            dz2 = dz2.contiguous()
        # attention-backward accumulators the launcher would clear itself (several key blocks /
        # query splits adding up, e.g. 512 latents): cleared instead by the kernel before it
        zp = _zero_plan(K, B, H, N, N, D)
        # dQKV of layers 1..L-1 feeds the chain-layout boundary kernel, which reads it as bf16
        # MFMA operands only: the attention backward stores it as bf16 (half the bytes both
        # ways, identical results) when it writes every element once (zp == 0: one key block)
        g_bf16 = (BF16_DQKV and K is not emulation and zp == 0 and C == 64 and H == 4 and R % 64 == 0
                  and 64 < N <= 256)

        def new_dqkv(i):  # every column block is written (or accumulated onto a cleared buffer) by attn_bwd
            # layer 0's dQKV goes to the producing cross-attention layer's chain kernel when there
            # is a hand-off (bf16 operand too), else to ln_linear_bwd (fp32)
            if g_bf16 and (i > 0 or getattr(ctx, "handoff", None) is not None):
                return torch.empty((B, N, 3 * C), device=dz.device, dtype=torch.bfloat16), {}
            t_ = torch.empty((B, N, 3 * C), **f32)
            return t_, (dict(zero_out=t_) if zp else {})

        # N = 64: layer i-1's attention backward runs inside the boundary kernel of layers i → i-1
        fuse_att = (CHAIN_ATT and K is not emulation and zp == 0 and C == 64 and H == 4 and N == 64 and D == 16
                    and R % 64 == 0 and hasattr(K, "ln_linear_post_attn_bwd"))
        dqkv_next, zkw = new_dqkv(L - 1)
        ho, _LOOKAHEAD["bwd_q"] = _LOOKAHEAD["bwd_q"], None
        if ho is not None and ho["key"] != getattr(ctx, "out_ptr", None):
            raise RuntimeError("fused encoder: a cross-attention layer handed its query-path backward to the wrong "
                               "self-attention block")
        att_first = {}  # layer L-1's attention backward inside the first boundary kernel (fused)
        if ho is not None:
            # the next cross-attention layer's LN + query-projection backward (dX = this block's
            # dZ) fused with the last layer's post-attention backward
            # (the chain kernel takes a query-projection hand-off: a C-row wq, fp32 G; a decoder's
            # 2C-wide K|V hand-off runs on the row-pass kernel, without phase D)
            if fuse_att and ho["g"].dtype == torch.float32 and ho["wq"].shape[0] in (C, 3 * C):
                dqkv_next, zkw = torch.empty((B, N, 3 * C), device=dz.device, dtype=torch.bfloat16), {}
                att_first = dict(att_qkv=S[L - 1][1], att_lse=S[L - 1][5], att_out=dqkv_next, att_scale=scale)
            sl = _GradSlab(R, [C, C, C * C, C] + PA_SIZES(C), dz2)
            tg = sl.targets()
            dy, do, delta = K.ln_linear_post_attn_bwd(ho["g"], ho["wq"], ho["x"], ho["mean1"], ho["rstd1"], ho["lnw"],
                                                      ho["lnb"], ho["dres"], tg[:4], *pa_args(L - 1), H, tg[4:],
                                                      **_take_job(), **drop(L - 1), **zkw, **att_first)
            sl.defer(K, ho["ll_dsts"] + pa_dsts(P[L - 1]))
        else:
            sl = _GradSlab(R, PA_SIZES(C), dz2)
            dy, do, delta = K.post_attn_bwd(dz2, *pa_args(L - 1), H, sl.targets(), slab=True, **_take_job(),
                                            **drop(L - 1), **zkw)
            sl.defer(K, pa_dsts(P[L - 1]))
        dx = None
        for i in range(L - 1, -1, -1):
            xl, qkv, mean1, rstd1, o, lse, y, m2, r2, u = S[i]
            qkv3 = qkv.view(B, N, 3 * C)
            dqkv = dqkv_next
            if not (fuse_att and (i < L - 1 or att_first)):  # (fused: a boundary kernel already ran it)
                # the bf16 variant carries the previous kernel's slab reduction on the CUs it shares
                # with its tiles (two workgroups per CU); the chain kernel after it then carries none
                K.attn_bwd(qkv3[:, :, :C], qkv3[:, :, C:2 * C], qkv3[:, :, 2 * C:], None, o, do.view(B, N, C), lse,
                           delta.view(B, N, H), H, D, scale, ctx.p, ctx.seed, dqkv[:, :, :C], dqkv[:, :, C:2 * C],
                           dqkv[:, :, 2 * C:], site=i, dq_zeroed=bool(zp & 1), kv_zeroed=bool(zp & 2),
                           **(_take_job() if ATTN_SLAB and dqkv.dtype == torch.bfloat16 else {}))
            if i > 0:
                att = {}
                if fuse_att:  # layer i-1's attention backward in phase D: its dQKV out, bf16
                    dqkv_next, zkw = torch.empty((B, N, 3 * C), device=dz.device, dtype=torch.bfloat16), {}
                    att = dict(att_qkv=S[i - 1][1], att_lse=S[i - 1][5], att_out=dqkv_next, att_scale=scale)
                else:
                    dqkv_next, zkw = new_dqkv(i - 1)
                sl = _GradSlab(R, LL_SIZES(C) + PA_SIZES(C), dz2)
                tg = sl.targets()
                dy, do, delta = K.ln_linear_post_attn_bwd(dqkv.view(R, 3 * C), bws[i][0], xl, mean1, rstd1, P[i][0],
                                                          P[i][1], dy, tg[:4], *pa_args(i - 1), H, tg[4:],
                                                          **_take_job(), **drop(i - 1), **zkw, **att)
                sl.defer(K, ll_dsts(P[i]) + pa_dsts(P[i - 1]))
            elif getattr(ctx, "handoff", None) is not None:
                # the producing cross-attention layer runs this LN1/QKV backward fused with its
                # post-attention backward (ln_linear_post_attn_bwd); it ignores the gradient
                # returned here (dy stands in as a correctly shaped tensor: no fill launch)
                _LOOKAHEAD["bwd"] = dict(key=ctx.handoff, g=dqkv.view(R, 3 * C), wq=bws[0][0], x=xl, mean1=mean1,
                                         rstd1=rstd1, lnw=P[0][0], lnb=P[0][1], dres=dy, ll_dsts=ll_dsts(P[0]))
                dx = dy
            else:
                sl = _GradSlab(R, LL_SIZES(C), dz2)
                dx = K.ln_linear_bwd(dqkv.view(R, 3 * C), bws[0][0], xl, mean1, rstd1, P[0][0], P[0][1], dy, True,
                                     *sl.targets(), slab=True, **_take_job())
                sl.defer(K, ll_dsts(P[0]))
        return (None, None, None, None, dx.view(B, N, C)) + (None,) * len(ps)


# cross-layer hand-off between a fused cross-attention layer and the self-attention block that
# follows it (_encode): "want" = the block's first-layer (γ1, β1, Wqkv bf16, bqkv), consumed by the
# cross layer's forward, which then runs post_attn + LN1/QKV in one launch and leaves
# "have" = (z, qkv, mean1, rstd1, γ1) for the block's forward.  Backward, the block hands its first
# LN1/QKV backward back ("bwd"), which the cross layer runs fused with its post-attention backward.
# The same in the other direction ("want_q" / "have_q" / "bwd_q"): a block's last fused layer
# computes the next cross-attention layer's LN + query projection, and that layer hands the
# backward of it back to the block.
# "want_pa" / "have_pa" / "bwd_pa": a cross-attention layer's post-attention half run by the
# per-sample block after it (forward prologue / backward epilogue of sb_fwd / sb_bwd).
_LOOKAHEAD = {"want": None, "have": None, "bwd": None, "want_q": None, "have_q": None, "bwd_q": None,
              "want_pa": None, "have_pa": None, "bwd_pa": None,
              "want_kv": None}


def _sa_block_plan(block, rows: int):
    """(layers, specs, param lists, fused?) of a self-attention block applied to ``rows`` rows."""
    layers = list(block)
    specs, pss = [], []
    for layer in layers:
        spec, ps = layer_spec_and_params(layer)
        specs.append(spec)
        pss.append(ps)
    ok = (WGRAD_SLAB and len(layers) > 1 and all(_fusable(lay) for lay in layers)
          and all(sp == specs[0] for sp in specs) and specs[0].C in SA_BLOCK_CHANNELS and not specs[0].cross
          and rows < TALL_ROWS)
    return layers, specs, pss, ok


def sa_block_lookahead(block, rows: int, n: Optional[int] = None, device=None):
    """The (γ1, β1, Wqkv bf16, bqkv) a preceding cross-attention layer can fuse into its
    post-attention kernel, or None when the block will not run fused (or runs as a per-sample
    block, which projects its own first layer)."""
    layers, specs, pss, ok = _sa_block_plan(block, rows)
    if not ok:
        return None
    p = specs[0].dropout if layers[0].training else 0.0
    if n is not None and _sample_block_ok(specs, n, p, device is not None and torch.device(device).type == "cuda"):
        return None
    ps = pss[0]
    return (ps[0], ps[1], _bf16_weights(specs[0], ps)[0], ps[3])


# a cross-attention layer's post-attention half folded into the per-sample block after it
# (PIO_SB_PRE=0: the cross layer runs it, A/B)
SB_PRE = os.environ.get("PIO_SB_PRE", "1") != "0"
# the next cross layer's LN + query projection in the per-sample block's kernels (PIO_SB_POST=0: A/B)
SB_POST = os.environ.get("PIO_SB_POST", "1") != "0"
# ... and a decoder's K|V projection into the encoder's last block (PerceiverIO.loss; MNIST −11 µs, r5)
SB_KV = True


def sample_block_runs(block, b: int, n: int, device) -> bool:
    """True when ``block`` over (b, n) latents will run as a per-sample block (_SampleBlockFn)
    that can take the preceding cross layer's post-attention half."""
    if not SB_PRE:
        return False
    layers, specs, pss, ok = _sa_block_plan(block, b * n)
    if not ok:
        return False
    p = specs[0].dropout if layers[0].training else 0.0
    return _sample_block_ok(specs, n, p, device is not None and torch.device(device).type == "cuda")


def _zero_plan(K, B, H, Nq, Nk, D) -> int:
    """Bits of the attention-backward accumulators the launcher would clear (1: dQ, 2: dK/dV),
    0 in deterministic mode (partial slices, no atomics) or on the emulation."""
    from . import deterministic

    if deterministic() or not hasattr(K, "attn_bwd_zero_plan"):
        return 0
    return int(K.attn_bwd_zero_plan(B, H, Nq, Nk, D))


def self_attention_block(block, x):
    """All layers of a self-attention block; one fused autograd node when every layer is
    fusable at C ≤ 64 (slab gradients on), else layer by layer."""
    layers, specs, pss, ok = _sa_block_plan(block, x.shape[1] * x.shape[0] if x.dim() == 3 else TALL_ROWS)
    ok = ok and x.dim() == 3
    if not ok:
        for layer in layers:
            x = self_attention_layer(layer, x)
        return x
    if x.dtype != torch.float32:
        x = x.float()
    bws = tuple(_bf16_weights(sp, ps) for sp, ps in zip(specs, pss))
    flat_ps = [p for ps in pss for p in ps]
    p = specs[0].dropout if layers[0].training else 0.0
    if _sample_block_ok(specs, x.shape[1], p, x.is_cuda):
        return _SampleBlockFn.apply(tuple(specs), bws, x, *flat_ps)
    return _SABlockFn.apply(tuple(specs), bws, _seed(p, x.device), p, x, *flat_ps)


# the image configs' latent blocks (C = 128, H = 4, 32 latents, no dropout): one workgroup per
# sample runs every layer of the block, forward and backward (csrc/sample_block.hip), plus one
# grouped weight-gradient GEMM launch; PERCEIVER_SAMPLE_BLOCK=0 keeps the per-layer kernels
SAMPLE_BLOCK = os.environ.get("PERCEIVER_SAMPLE_BLOCK", "1") != "0"


def _sample_block_ok(specs, n: int, p: float, cuda: bool) -> bool:
    from . import deterministic

    sp = specs[0]
    # ≤ 3 layers: with the cross layers' pre / post folds a block's backward fills 4L + 4 slab
    # segments (common.h kMaxSlabSegs = 16) and 4L + 3 weight-gradient jobs (sb_args.h
    # kSBMaxJobs); 4 layers would overflow both, so such blocks keep the per-layer kernels
    return (SAMPLE_BLOCK and cuda and sp.C in (64, 128) and sp.heads == 4 and n == 32 and p == 0.0 and not sp.cross
            and 1 <= len(specs) <= 3 and all(s == sp for s in specs) and not deterministic())


class _SampleBlockFn(torch.autograd.Function):
    """A C ∈ {64, 128}, 4-head, 32-latent self-attention block as per-sample kernels (reference model.py:36-44):
    forward saves, per layer, the rows the backward and the weight-gradient GEMMs read (LN1(x),
    QKV, O, LN2(y), u, GELU(u) in bf16; y, z and the LayerNorm statistics in fp32); backward runs
    the per-sample backward (activation gradients + LayerNorm affine gradients) and one grouped
    GEMM launch for every weight / bias gradient of the block."""

    @staticmethod
    def forward(ctx, specs, bws, x, *ps):
        K = kernels(x)
        B, N, C = x.shape
        L = len(specs)
        xl = x.reshape(B * N, C)
        if not xl.is_contiguous():
            xl = xl.contiguous()
        params = []
        for i in range(L):
            p = ps[SA_NP * i:SA_NP * (i + 1)]
            wq, _, wo, w1, w2 = bws[i]
            params += [p[0], p[1], wq, p[3], wo, p[5], p[6], p[7], w1, p[9], w2, p[11]]
        scale = 1.0 / math.sqrt(C // specs[0].heads)
        hp = _LOOKAHEAD["have_pa"]
        ctx.pa = None
        pre = []
        if hp is not None and hp["key"] == xl.data_ptr():
            # the preceding cross layer's post-attention half: x is its placeholder output, written
            # by this launch before the block's first layer reads it
            _LOOKAHEAD["have_pa"] = None
            ctx.pa = hp
            pre = hp["pre"]
        # the next cross layer's LN + query projection of the block output (its backward comes
        # back as "bwd_q" and runs first in this block's backward)
        wq_n = _LOOKAHEAD["want_q"] if SB_POST else None
        # (a decoder's K|V projection: a (2C, C) weight, the backward offered when wq_n[4])
        post = ([wq_n[0], wq_n[1], wq_n[2], wq_n[3]]
                if wq_n is not None and tuple(wq_n[2].shape) in ((C, C), (2 * C, C)) else [])
        saved = K.sb_fwd(xl, params, scale, EPS, pre=pre, post=post)
        ctx.pre_saved = saved[12 * L:12 * L + 6] if pre else None
        ctx.post, ctx.post_saved = (post, saved[-3:]) if post else (None, None)
        if post:
            _LOOKAHEAD["want_q"] = None
        post_q = saved[-4] if post else None
        saved = saved[:12 * L]
        z = saved[12 * (L - 1) + 7]
        if post:
            _LOOKAHEAD["have_q"] = (z, post_q, ctx.post_saved[1], ctx.post_saved[2], post[0],
                                    len(wq_n) > 4 and bool(wq_n[4]))
            ctx.out_ptr = z.data_ptr()
            # the block output is the query path's LayerNorm input: kept for the backward
            ctx.save_for_backward(xl, *saved)
        else:
            # the block output is not a backward operand: a placeholder in its slot
            ctx.save_for_backward(xl, *saved[:12 * (L - 1) + 7], xl, *saved[12 * (L - 1) + 8:])
        ctx.params, ctx.ps, ctx.dims = params, ps, (B, N, C, L, scale)
        return z.view(B, N, C)

    @staticmethod
    def backward(ctx, dz):
        K = kernels(dz)
        B, N, C, L, scale = ctx.dims
        xl, *saved = ctx.saved_tensors
        ps = ctx.ps
        dz2 = dz.reshape(B * N, C)
        if not dz2.is_contiguous():
            dz2 = dz2.contiguous()
        scratch = []

        def target(p, n):
            g = _grad_of(p)
            if g is None:
                g = torch.zeros(n, device=dz.device, dtype=torch.float32)
                scratch.append(g)
            return g.view(-1)

        pa = ctx.pa
        hq = None
        if ctx.post is not None:
            hq, _LOOKAHEAD["bwd_q"] = _LOOKAHEAD["bwd_q"], None
            if hq is not None and hq["key"] != ctx.out_ptr:
                raise RuntimeError("fused encoder: a cross-attention layer handed its query-path backward to the "
                                   "wrong per-sample block")
        kw = {}
        if hq is not None:
            _, mean_q, rstd_q = ctx.post_saved
            # a decoder's K/V path hands no residual: the gradient arriving here (its zero stand-in
            # plus any other consumer's) is the residual
            dres = hq["dres"] if hq["dres"] is not None else dz2
            kw = dict(post=ctx.post, post_io=[hq["g"], dres, mean_q, rstd_q])
        zb = None
        if pa is not None:
            # the cross layer's post-attention backward last: its dO / δ and cleared accumulators go
            # to that layer's backward, the returned gradient is its residual path dY
            zb = _cross_zero_bufs(pa["ctx"], dz.device)
            kw.update(pre=pa["pre"], pre_saved=ctx.pre_saved, zero_out=zb[0])
        out = K.sb_bwd(dz2, xl, saved, ctx.params, scale, EPS, **kw)
        dqb = out.pop() if hq is not None else None
        if pa is not None:
            _LOOKAHEAD["bwd_pa"] = dict(key=pa["key"], do=out[-5], delta=out[-4], zbuf=zb)
        # the per-sample LayerNorm affine partials (B, 4·L·C [+ 2C]): summed into the gradients by
        # the grouped weight-gradient launch's appended workgroups (or a deferred slab reduction)
        dsts, offs = [], []
        for i in range(L):
            p = ps[SA_NP * i:SA_NP * (i + 1)]
            for j, q in enumerate((p[0], p[1], p[6], p[7])):
                g = _grad_of(q)
                if g is not None:
                    dsts.append(g.view(-1))
                    offs.append((4 * i + j) * C)
        jobs = []
        for i in range(L):
            p = ps[SA_NP * i:SA_NP * (i + 1)]
            dq, dy, du, dzz = out[2 + 4 * i:6 + 4 * i]
            sv = saved[12 * i:12 * (i + 1)]
            for G, A, W, b in ((dq, sv[0], p[2], p[3]), (dy, sv[2], p[4], p[5]), (du, sv[3], p[8], p[9]),
                               (dzz, sv[5], p[10], p[11])):
                if W.requires_grad or b.requires_grad:
                    jobs += [G, A, target(W, W.numel()), target(b, b.numel())]
        if hq is not None:  # the query path: LN_q affine partials after the pre stage's, dWq / dbq
            o = (4 * L + (2 if pa is not None else 0)) * C
            for j in range(2):
                if hq["ll_dsts"][j] is not None:
                    dsts.append(hq["ll_dsts"][j])
                    offs.append(o + j * C)
            if hq["ll_dsts"][2] is not None or hq["ll_dsts"][3] is not None:
                Nq = dqb.shape[1]  # C (a query projection) or 2C (a decoder's K|V)
                jobs += [dqb, ctx.post_saved[0],
                         hq["ll_dsts"][2] if hq["ll_dsts"][2] is not None else torch.zeros(Nq * C, device=dz.device),
                         hq["ll_dsts"][3] if hq["ll_dsts"][3] is not None else torch.zeros(Nq, device=dz.device)]
        if pa is not None:
            Wo, bo, g2, be2, W1, b1, W2, b2 = pa["ps"]
            for j, q in enumerate((g2, be2)):
                g = _grad_of(q)
                if g is not None:
                    dsts.append(g.view(-1))
                    offs.append((4 * L + j) * C)
            dyp, dup, dzp = out[-3:]
            o_pre = pa["pre"][0]
            ln2y, _, gu = ctx.pre_saved[:3]
            for G, A, W, b in ((dyp, o_pre, Wo, bo), (dup, ln2y, W1, b1), (dzp, gu, W2, b2)):
                if W.requires_grad or b.requires_grad:
                    jobs += [G, A, target(W, W.numel()), target(b, b.numel())]
        if jobs:
            K.sb_wgrad(jobs, job_slab=out[1] if dsts else None, job_dsts=dsts, job_offs=offs)
        else:
            defer_slab(K, out[1], dsts, offs)
        return (None, None, out[0].view(B, N, C)) + (None,) * len(ps)


def _seed(p: float, device) -> Optional[torch.Tensor]:
    """Device seed of one fused call's dropout masks (None when p == 0).

    Drawn ON THE DEVICE by torch's generator: under hipGraph capture the draw is a graph node
    whose Philox offset torch advances on every replay, so each replayed step gets fresh masks
    (a host integer would be frozen into the graph).  The backward reads the same tensor, so
    masks are regenerated, never stored."""
    if p <= 0.0:
        return None
    st = _STATIC_SEEDS
    if st["on"] and torch.cuda.is_current_stream_capturing():
        # a StepEngine capture: this call's own slot of the persistent pool the engine stages
        # fresh values into before every replay (no generator kernel in the graph, no generator
        # bookkeeping launches per replay)
        i = st["n"]
        if i >= _STATIC_SEED_SLOTS or st["t"] is None or st["t"].device != torch.device(device):
            raise RuntimeError(f"fused dropout: more than {_STATIC_SEED_SLOTS} seeded calls in one captured step")
        st["n"] = i + 1
        return st["t"][i:i + 1]
    pool = _SEED_POOL
    if pool["armed"]:
        # inside one encoder pass: one draw of a small pool serves every fused call of the pass
        # (one generator launch instead of one per layer / block; each call its own slot)
        t = pool["t"]
        if t is None or t.device != torch.device(device) or pool["i"] >= t.numel():
            t = pool["t"] = torch.randint(-(2**62), 2**62, (_SEED_POOL_SIZE,), device=device, dtype=torch.int64)
            pool["i"] = 0
        pool["i"] += 1
        return t[pool["i"] - 1:pool["i"]]
    return torch.randint(-(2**62), 2**62, (1,), device=device, dtype=torch.int64)


# dropout seeds of one encoder pass (_encode arms the pool on entry and disarms it on exit, so a
# pass always draws a fresh pool: a replayed step graph re-runs that draw; calls outside an
# encoder pass draw their own seed)
_SEED_POOL_SIZE = 16
_STATIC_SEED_SLOTS = 64  # csrc/elementwise.hip kStageSeeds
_STATIC_SEEDS = {"on": False, "t": None, "n": 0}


def begin_static_seeds(device) -> None:
    """Start a graph capture's static dropout seeds (train/engine.py StepEngine): every seeded
    fused call captured until end_static_seeds() reads its own slot of an int64 pool that belongs
    to THIS capture only (a fresh tensor per captured graph: two engines — e.g. a train and an
    eval model — or two graphs of one engine never share slots, so staging one graph's seeds can
    not change what another graph reads).  Call OUTSIDE the capture (the pool is allocated here)."""
    t = torch.zeros(_STATIC_SEED_SLOTS, dtype=torch.int64, device=device)
    _STATIC_SEEDS.update(on=True, t=t, n=0)


def end_static_seeds():
    """(pool, slots used) of the capture just ended; the engine stages slots [0, used) — fresh
    random values — in the launch before each replay (stage_step seed_dst / seeds)."""
    _STATIC_SEEDS["on"] = False
    t, n = _STATIC_SEEDS["t"], _STATIC_SEEDS["n"]
    _STATIC_SEEDS["t"] = None  # the captured graph keeps its pool (drop_seeds); the next capture gets a new one
    return t, n
_SEED_POOL = {"armed": False, "t": None, "i": 0}


def _run_layer(layer, x_q, x_kv=None, pad_mask=None, src: Optional[KVSource] = None):
    spec, ps = layer_spec_and_params(layer)
    kmask = pad_mask.to(torch.bool).contiguous() if pad_mask is not None else None
    bw = _bf16_weights(spec, ps)
    p_attn = spec.dropout if layer.training else 0.0
    if x_q.dtype != torch.float32:
        x_q = x_q.float()
    if x_kv is not None and x_kv.dtype != torch.float32:
        x_kv = x_kv.float()
    return _LayerFn.apply(spec, bw, _seed(p_attn, x_q.device), p_attn, src, x_q, x_kv, kmask, *ps)


def _fusable(layer, x=None) -> bool:
    spec, _ = layer_spec_and_params(layer)
    d = spec.C // spec.heads
    return spec.C in (32, 64, 128) and d in (16, 32, 64, 128)


def can_fuse(layer, x_kv=None) -> bool:
    ch = x_kv.channels if isinstance(x_kv, KVSource) else (x_kv.shape[-1] if x_kv is not None else 0)
    return _fusable(layer) and ch <= 160


def self_attention_layer(layer, x):
    if not _fusable(layer, x):
        return layer.eager_forward(x)
    return _run_layer(layer, x)


def cross_attention_layer(layer, x_q, x_kv, pad_mask=None):
    """``x_kv`` is a tensor or a :class:`KVSource` (shared K/V projection, split PE input)."""
    src = x_kv if isinstance(x_kv, KVSource) else None
    if not can_fuse(layer, x_kv):
        if src is not None:
            x_kv = src.materialize()
        return layer.eager_forward(x_q, x_kv, pad_mask)
    if x_q.dim() == 3 and x_q.shape[0] > 1 and x_q.stride(0) == 0:
        x_q = x_q[:1]  # batch-broadcast queries (decoder output array): project once
    return _run_layer(layer, x_q, src.x if src is not None else x_kv, pad_mask, src)


# ------------------------------------------------------------------------------------------
# text embedding
# ------------------------------------------------------------------------------------------
class _TextEmbedFn(torch.autograd.Function):
    @staticmethod
    def forward(ctx, ids, emb, pos, scale):
        K = kernels(emb)
        ids = ids.contiguous()
        out = K.embed_fwd(ids, emb, pos[: ids.shape[1]].contiguous(), scale)
        ctx.save_for_backward(ids)
        ctx.scale, ctx.emb, ctx.pos = scale, emb, pos
        return out

    @staticmethod
    def backward(ctx, g):
        (ids,) = ctx.saved_tensors
        K = kernels(g)
        targets = []
        for p, need in ((ctx.emb, ctx.needs_input_grad[1]), (ctx.pos, ctx.needs_input_grad[2])):
            if need and p.grad is None:
                p.grad = torch.zeros_like(p)
            targets.append(p.grad if need else None)
        from . import deterministic

        if deterministic() and g.is_cuda:  # sorted segment sums instead of fp32 atomics
            C = g.shape[-1]
            if targets[0] is not None:
                targets[0].index_put_((ids.reshape(-1),), g.reshape(-1, C) * ctx.scale, accumulate=True)
            if targets[1] is not None:
                targets[1][: ids.shape[1]] += g.sum(0)
            return None, None, None, None
        # scatter-add straight into the (flat-buffer) gradients
        K.embed_bwd(ids, g.contiguous(), targets[0], targets[1], ctx.scale, **_take_job())
        return None, None, None, None


def text_embed(adapter, ids):
    return _TextEmbedFn.apply(ids, adapter.text_embedding.weight, adapter.pos_encoding, float(adapter.scale))


# ------------------------------------------------------------------------------------------
# encoder
# ------------------------------------------------------------------------------------------
def encoder_forward(encoder, x, pad_mask=None):
    from ..models.adapters import ImageInputAdapter, TextInputAdapter

    ad = encoder.input_adapter
    if isinstance(ad, TextInputAdapter):
        src = KVSource(text_embed(ad, x))
    elif isinstance(ad, ImageInputAdapter) and not x.requires_grad:
        ad.check_shape(x)
        pix = x.reshape(x.shape[0], -1, ad.num_image_channels).float().contiguous()
        src = KVSource(pix, pe=ad.padded_position_encoding(), kin=ad.num_input_channels)
    else:
        src = KVSource(ad(x))
    return _encode(encoder, src, pad_mask)


def encode_inputs(encoder, x_in, pad_mask=None):
    """The encoder body over already adapted inputs ``x_in`` (B, M, Kin) — e.g. the gathered
    ``[pixel ‖ PE]`` rows of a sparse image (``models/lartpc.py``)."""
    return _encode(encoder, KVSource(x_in.float().contiguous()), pad_mask)


def encode_sparse(encoder, values, index, pad_mask=None):
    """The encoder over a sparse image: ``values`` (B, K, C_img) pixel values at flat pixel
    positions ``index`` (B, K) int64; the K/V projections read the Fourier PE rows at ``index``
    from the adapter's padded table inside their kernels (no gathered input rows).

    ``index`` must lie in [0, H·W) (``data/lartpc.py`` ``sparse_collate`` builds it from the
    non-zero pixels).  The kernels clamp an index outside the table instead of faulting, where
    the eager path's ``index_select`` raises; the checked build (``PERCEIVER_CHECKED=1``) flags
    it and raises (``ops.check_device_errors``)."""
    ad = encoder.input_adapter
    pix = values.reshape(values.shape[0], values.shape[1], ad.num_image_channels).float().contiguous()
    idx = index if index.dtype == torch.int64 and index.is_contiguous() else index.long().contiguous()
    src = KVSource(pix, pe=ad.padded_position_encoding(), kin=ad.num_input_channels, index=idx)
    return _encode(encoder, src, pad_mask)


def _encode(encoder, src: KVSource, pad_mask):
    _SEED_POOL.update(armed=True, t=None, i=0)
    try:
        return _encode_layers(encoder, src, pad_mask)
    finally:
        _SEED_POOL.update(armed=False, t=None, i=0)


def _encode_layers(encoder, src: KVSource, pad_mask):
    lat = encoder.latent.unsqueeze(0)  # (1, N, C): projected once, broadcast inside the kernels
    b = src.x.shape[0]
    n = lat.shape[1]
    layers = list(encoder.layers())
    for li, layer in enumerate(layers):
        cross, block = layer[0], layer[1]
        if li == 1:  # DDP: every layer_n gradient but its query path is final here (parallel/reducer.py)
            lat = bucket_ready_point(lat, encoder, "layer_n")
        if lat.shape[0] == 1 and not can_fuse(cross, src):
            lat = lat.expand(b, -1, -1)
        # the block's first LN1 + QKV projection rides on the cross layer's post-attention kernel,
        # or a per-sample block runs that post-attention half itself
        _LOOKAHEAD["want"] = sa_block_lookahead(block, b * n, n, lat.device) if can_fuse(cross, src) else None
        sb_runs = sample_block_runs(block, b, n, lat.device)
        _LOOKAHEAD["want_pa"] = can_fuse(cross, src) and sb_runs
        try:
            lat = cross_attention_layer(cross, lat, src, pad_mask)
        finally:
            _LOOKAHEAD["want"] = _LOOKAHEAD["want_pa"] = None
        if lat.shape[0] == 1 and b > 1:
            lat = lat.expand(b, -1, -1)
        nxt_cross = layers[li + 1][0] if li + 1 < len(layers) else None
        if nxt_cross is not None and can_fuse(nxt_cross, src):
            _LOOKAHEAD["want_q"] = cross_q_lookahead(nxt_cross, src, sample_block=sb_runs)
        elif nxt_cross is None:  # a decoder's K/V over the encoder output, when its caller asked for it
            _LOOKAHEAD["want_q"] = _LOOKAHEAD["want_kv"]
        if li == 0 and len(layers) > 1:  # DDP: layer_1's block gradients (but its first LN1/QKV) final here
            lat = bucket_ready_point(lat, encoder, "layer_1_sa")
        try:
            lat = self_attention_block(block, lat)
            if _LOOKAHEAD["have_pa"] is not None:
                raise RuntimeError("fused encoder: a cross-attention layer left its post-attention half to a "
                                   "per-sample block that did not run it")
        finally:
            _LOOKAHEAD["have"] = _LOOKAHEAD["want_q"] = _LOOKAHEAD["have_pa"] = None
    if _LOOKAHEAD["want_kv"] is None:
        _LOOKAHEAD["have_q"] = None
    return lat


def decoder_kv_lookahead(cross, sample_block: bool = False, backward: bool = False):
    """(γkv, βkv, Wkv bf16 (2C, C), bkv[, backward]) of a decoder cross-attention over the encoder's
    latents, for the encoder's last self-attention kernel (C = 64, H = 4 latents: the fused layer
    kernel's shape; a per-sample block (sample_block): C ∈ {64, 128}), or None.  backward: that
    block may also run the projection's backward (packed in-projection only; the caller passes False
    while a DDP ready point on the decoder input is armed — the decoder's gradients must be final
    when it fires).  Set by the caller for the duration of one encoder + decoder call only
    (PerceiverMLM.loss, PerceiverIO.loss), so the stashed K/V never outlives it."""
    if sample_block and not SB_KV:
        return None
    spec, ps = layer_spec_and_params(cross)
    if not spec.cross or spec.C not in ((64, 128) if sample_block else (64,)) or ps[2].shape[0] != spec.C:
        return None
    wkv = _bf16_weights(spec, ps)[1]
    if wkv is None:
        wkv = _kv_weight(spec, ps)
    bin_ = ps[5] if spec.packed else ps[7]
    if not wkv.is_contiguous() or tuple(wkv.shape) != (2 * spec.C, spec.C):
        return None
    return (ps[2], ps[3], wkv, bin_[spec.C:], backward and spec.packed)


def cross_q_lookahead(cross, src, sample_block: bool = False):
    """(γq, βq, Wq bf16 (C, C), bq) of a cross-attention layer's query path, for the preceding
    self-attention block's last kernel (C = 64, H = 4: the fused layer kernel's shape; a per-sample
    block (sample_block): C ∈ {64, 128}, any head count)."""
    spec, ps = layer_spec_and_params(cross)
    if not spec.cross or (spec.C not in (64, 128) if sample_block else (spec.C != 64 or spec.heads != 4)):
        return None
    bw = _bf16_weights(spec, ps)
    bin_ = ps[5] if spec.packed else ps[7]
    return (ps[0], ps[1], bw[0], bin_[:spec.C])
