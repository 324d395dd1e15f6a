"""Plain-PyTorch emulation of every HIP kernel entry point (same signatures as ``_C``).

Two uses: (1) the fused executor runs on CPU through this module, so its bookkeeping
(strides, packed buffers, batch-broadcast queries, in-place gradient accumulation) is
covered by the CPU test-suite; (2) it is the fp32 oracle the GPU numerics tests compare
the hand-written kernels against.  Rounding points mirror the kernels: GEMM operands are
rounded to bf16 exactly where the kernels stage bf16 tiles, accumulation is fp32.
"""
from __future__ import annotations

import math
import torch
import torch.nn.functional as F

LOG2E = 1.4426950408889634


def _bf(x):
    return x.to(torch.bfloat16).to(torch.float32)


# ---- the kernels' counter-based dropout RNG (csrc/common.h hash3 / drop_key), bit-exact --------
M32 = 0xFFFFFFFF


def _u32(x):
    return x & M32


def hash3(a, b, c):
    """uint32 murmur-style mixer over int64 tensors / ints holding uint32 values."""
    h = _u32(_u32(a * 0x9E3779B1) ^ _u32(b + 0x7F4A7C15))
    h = h ^ _u32(c * 0x85EBCA77)
    h = _u32((h ^ (h >> 15)) * 0x2C1B3C6D)
    h = _u32((h ^ (h >> 12)) * 0x297A2D39)
    return h ^ (h >> 15)


def drop_key(seed, site: int, sub: int) -> int:
    s = int(seed.reshape(-1)[0].item()) & 0xFFFFFFFFFFFFFFFF
    return int(hash3(torch.tensor(s & M32), torch.tensor(s >> 32), torch.tensor(_u32(site * 4 + sub))).item())


def drop_thresh(p: float) -> int:
    return min(M32, int(p * 4294967296.0)) if p > 0 else 0


def keep_mask(key: int, stream, idx, p: float):
    """bool keep mask: hash3(key, stream, idx) >= p·2^32 (stream / idx int64 tensors)."""
    return hash3(torch.as_tensor(key, dtype=torch.int64), stream, idx) >= drop_thresh(p)


def row_drop_mask(seed, site: int, sub: int, R: int, C: int, p: float, device=None):
    """(R, C) float mask·1/(1-p) of a fused post-attention kernel's residual dropout."""
    idx = torch.arange(R * C, dtype=torch.int64, device=device).view(R, C)
    keep = keep_mask(drop_key(seed, site, sub), torch.zeros((), dtype=torch.int64), idx, p)
    return keep.float() / (1.0 - p)


def attn_drop_mask(seed, site: int, B: int, H: int, Nq: int, Nk: int, p: float, device=None):
    """(B, H, Nq, Nk) float mask·1/(1-p) of the attention kernels' probability dropout."""
    stream = torch.arange(B * H, dtype=torch.int64, device=device).view(B, H, 1, 1)
    idx = (torch.arange(Nq, dtype=torch.int64, device=device).view(Nq, 1) * Nk
           + torch.arange(Nk, dtype=torch.int64, device=device).view(1, Nk))
    keep = keep_mask(drop_key(seed, site, 2), stream, _u32(idx), p)
    return keep.float() / (1.0 - p)


def _ln(x, w, b, eps):
    mean = x.mean(-1)
    var = x.var(-1, unbiased=False)
    rstd = torch.rsqrt(var + eps)
    return (x - mean[:, None]) * rstd[:, None] * w + b, mean, rstd


def _split_x(x, pe, kin, pe_index=None):
    """Logical input rows: x itself, or pe[r mod M] — pe[pe_index[r]] when given (sparse
    images) — (first kin columns) with x's pixel channels added into the leading columns
    (SURVEY K-03 split input)."""
    if pe is None:
        return x.float()
    r, m = x.shape[0], pe.shape[0]
    if pe_index is not None:
        full = pe.index_select(0, pe_index.reshape(-1).clamp(0, m - 1))[:, :kin].clone()
    else:
        full = pe.repeat(r // m, 1)[:, :kin].clone()
    full[:, : x.shape[1]] += x.float()
    return full


def ln_linear_fwd(x, lnw, lnb, eps, w, bias, act, res, out_bf16, save_stats, pe=None, kin=-1, pe_index=None):
    if kin >= 0:
        w = w[:, :kin]
    xf = _split_x(x, pe, w.shape[1], pe_index)
    mean = rstd = None
    if lnw is not None:
        xn, mean, rstd = _ln(xf, lnw, lnb, eps)
    else:
        xn = xf
    y = _bf(xn) @ _bf(w.float()).t()
    if bias is not None:
        y = y + bias
    if act == 1:
        y = F.gelu(y)
    if res is not None:
        y = y + res
    y = y.to(torch.bfloat16) if out_bf16 else y
    out = [y]
    if save_stats and lnw is not None:
        out += [mean, rstd]
    return out


def pe_gemm(A, B, bf16_out=False, pad_rows=0):
    """bf16 operands, fp32 accumulation, fp32 (or bf16) output (csrc/pe_proj.hip pe_gemm_kernel),
    pad_rows zero rows appended."""
    y = A.float() @ B.float().t()
    if pad_rows:
        y = torch.cat([y, y.new_zeros(pad_rows, y.shape[1])])
    return y.to(torch.bfloat16) if bf16_out else y


def pe_weight_prep(W, g, b, bias, nc, Kp, W2=None):
    if W2 is not None:  # separate K / V weights (the kernel reads the two row blocks in place)
        W = torch.cat([W, W2], 0)
    O, kin = W.shape
    wg = W * g[None, :]
    Wg = torch.zeros((O, Kp), device=W.device, dtype=torch.float32)
    Wg[:, nc:kin] = wg[:, nc:]
    wpg, gw, bw = wg[:, :nc].t().contiguous(), wg.sum(1), W @ b + bias
    wt = torch.zeros((6, O), device=W.device, dtype=torch.float32)  # implicit-K/V generation table
    wt[:nc] = wpg
    wt[4] = wpg.sum(0) - gw
    wt[5] = bw
    return [Wg.to(torch.bfloat16), wpg, gw, bw, wt]


def pe_grads(D, part, E, Wa, Wb, g, b, nc, dWa=None, dWb=None, db=None, dg=None, dbeta=None):
    """csrc/pe_proj.hip pe_grads: factored-projection weight / LN gradients added into targets
    (the PE GEMM with bf16 operands, fp32 accumulation)."""
    O, kin, Ch = D.shape[1], g.shape[0], Wa.shape[0]
    graw = E.float().t() @ D.to(torch.bfloat16).float()
    tot = part.sum(0)
    S, e, Gp = tot[:O], tot[O:2 * O], tot[2 * O:].view(nc, O)
    G = torch.cat([Gp, graw[nc:kin] - e[None, :]], 0).t()  # (O, kin)
    W = torch.cat([Wa, Wb], 0)
    dW = G * g[None, :] + S[:, None] * b[None, :]
    for t, v in ((dWa, dW[:Ch]), (dWb, dW[Ch:]), (db, S), (dg, (W * G).sum(0)), (dbeta, W.t() @ S)):
        if t is not None:
            t.view(-1).add_(v.reshape(-1))


def pe_proj_fwd(pix, P, pes, pesq, wpg, gw, bw, kin, eps):
    """csrc/pe_proj.hip forward: factored LN + K/V projection over [pixels ‖ PE]."""
    M = P.shape[0]
    R = pix.shape[0]
    m = torch.arange(R, device=pix.device) % M
    s = pes[m] + pix.sum(1)
    sq = pesq[m] + (pix * pix).sum(1)
    mu = s / kin
    rs = torch.rsqrt((sq / kin - mu * mu).clamp(min=0) + eps)
    y = (P[m] + pix @ wpg) * rs[:, None] - (mu * rs)[:, None] * gw + bw
    return [y.to(torch.bfloat16), mu, rs]


def pe_proj_bwd(dy, pix, mean, rstd, M):
    """csrc/pe_proj.hip backward: D = Σ_b dY·rσ and one 'partial' row [ΣdY | ΣdY·μ·rσ | ΣdY·x̂_c]."""
    R, O = dy.shape
    B = R // M
    D = (dy * rstd[:, None]).view(B, M, O).sum(0)
    xh = (pix - mean[:, None]) * rstd[:, None]
    part = torch.cat([dy.sum(0), (dy * (mean * rstd)[:, None]).sum(0), (xh.t() @ dy).reshape(-1)])
    return [D, part[None]]


def pe_kv(P, pix, pes, pesq, wt, kin, eps):
    """csrc/attention_pe.hip pe_key_stats / pe_kv_elem: the implicit K/V rows (B·M, 2C) bf16 from
    the bf16 PE product P' (M, 2C), the pixel channels and the generation table, plus μ, rσ."""
    M = pes.shape[0]  # P may carry zero pad rows past M
    R, nc = pix.shape
    m = torch.arange(R, device=pix.device) % M
    mu = (pes[m] + pix.sum(1)) / kin
    rs = torch.rsqrt(((pesq[m] + (pix * pix).sum(1)) / kin - mu * mu).clamp(min=0) + eps)
    xh = (pix - mu[:, None]) * rs[:, None]
    y = rs[:, None] * P[m].float() + xh @ wt[:nc] + (mu * rs)[:, None] * wt[4] + wt[5]
    return y.to(torch.bfloat16), mu, rs


def attn_fwd_pe(q, P, pix, pes, pesq, wt, H, scale, kin, eps, nsplit):
    """csrc/attention_pe.hip attn_fwd_pe_kernel: encoder cross-attention over implicit K/V."""
    C, M = H * 32, pes.shape[0]
    B = pix.shape[0] // M
    kv = pe_kv(P, pix, pes, pesq, wt, kin, eps)[0].view(B, M, 2 * C)
    return attn_fwd(q, kv[:, :, :C], kv[:, :, C:], None, H, 32, scale, 0.0, None, nsplit)


def attn_bwd_pe_implicit(q, P, pes, pesq, wt, dO, lse, delta, pix, dq, D, part, H, scale, kin, eps, accumulate, bsplit,
                         dq_zeroed=False, d_zeroed=False):
    """attn_bwd_pe over implicit K/V (the same generation as attn_fwd_pe)."""
    kv, mu, rs = pe_kv(P, pix, pes, pesq, wt, kin, eps)
    attn_bwd_pe(q, kv, dO, lse, delta, mu, rs, pix, dq, D, part, H, scale, accumulate, bsplit)


def attn_bwd_pe_part_rows(M, H, B, bsplit):
    """rows of attn_bwd_pe's partial buffer (the kernel's grid mode; the emulation fills row 0)."""
    return ((M + 255) // 256) * bsplit


def attn_bwd_pe(q, kv, dO, lse, delta, mean, rstd, pix, dq, D, part, H, scale, accumulate, bsplit, dq_zeroed=False,
                d_zeroed=False):
    """csrc/attention_pe.hip: encoder cross-attention backward whose dK/dV are folded into the
    factored projection's reductions D = Σ_b dY·rσ and [Σ dY | Σ dY·μ·rσ | Σ dY·x̂_c] (one
    partial row here; the kernel writes one per (key block, batch group)).  q is batch-broadcast
    (1, Nq, C) and dq (Nq, C) receives the gradient summed over the batch."""
    C = H * 32
    B = dO.shape[0]
    M = kv.shape[0] // B
    kv3 = kv.view(B, M, -1)
    g = attn_bwd(q, kv3[:, :, :C], kv3[:, :, C:2 * C], None, None, dO, lse, delta, H, 32, scale, 0.0, None, None,
                 None, None)
    dq.copy_((g[0].sum(0) if q.shape[0] == 1 else g[0]).reshape(dq.shape))
    dy = torch.cat([g[1], g[2]], -1).reshape(B * M, 2 * C)
    Dn, pn = pe_proj_bwd(dy, pix, mean, rstd, M)
    full = torch.zeros_like(part)
    full[0] = pn[0]
    if accumulate:
        D += Dn
        part += full
    else:
        D.copy_(Dn)
        part.copy_(full)


_SLAB = [False]


def _acc(t, v):
    """t += v for a gradient target: plain (any shape with v's numel) or an (8, numel)
    replicated accumulator (the emulation adds into replica 0).  In slab mode the target is a
    (tiles, numel) slab view: the emulation stores the whole sum into row 0, zeros elsewhere
    (the HIP kernels store one partial per 64-row tile; slab_reduce sums either form)."""
    if _SLAB[0]:
        t[0] = v.reshape(-1)
        t[1:] = 0
    elif t.dim() == 2 and t.shape[0] == 8 and t.shape[1] == v.numel():
        t[0] += v.reshape(-1)
    else:
        t += v.reshape(t.shape)


def sa_layer_fwd(qkv, x, N, scale, wo, bo, g2, be2, eps, w1, b1, w2, b2, lnw=None, lnb=None, wq=None, bq=None,
                 seed=None, site=0, p=0.0):
    """The fused self-attention layer forward (chain.hip sa_layer_fwd_chain8_kernel): attention of the
    packed qkv (C = 64, H = 4, probability dropout p), then the post-attention block and, when the
    next layer's LN1 / in-projection are given, its QKV."""
    C, H = 64, 4
    R = x.shape[0]
    q3 = qkv.view(R // N, N, 3 * C)
    o, lse = attn_fwd(q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:], None, H, C // H, scale, p, seed, 1, site=site)
    o2 = o.reshape(R, C)
    if wq is None:
        return [o, lse] + list(post_attn_fwd(o2, x, wo, bo, g2, be2, eps, w1, b1, w2, b2, seed, site, p))
    return [o, lse] + list(post_attn_ln_linear_fwd(o2, x, wo, bo, g2, be2, eps, w1, b1, w2, b2, lnw, lnb, wq, bq, seed,
                                                    site, p))


def sa_block_fwd(qkv0, x0, N, scale, eps, wo, bo, g2, be2, w1, b1, w2, b2, lnw, lnb, wq, bq, seed=None, p=0.0):
    """The persistent block forward (persist.hip sa_block_fwd_kernel): sa_layer_fwd of every layer
    in one call, layer i's next projection from (lnw, lnb, wq, bq)[i] when present.  Returns the
    per-layer outputs flattened ([o, lse, z, y, m2, r2, u] + [qkv_n, mean_n, rstd_n])."""
    out, qkv, x = [], qkv0, x0
    for i in range(len(wo)):
        nx = i < len(wq)
        r = sa_layer_fwd(qkv, x, N, scale, wo[i], bo[i], g2[i], be2[i], eps, w1[i], b1[i], w2[i], b2[i],
                         lnw[i] if nx else None, lnb[i] if nx else None, wq[i] if nx else None,
                         bq[i] if nx else None, seed=seed, site=i, p=p)
        out += list(r)
        x = r[2]
        qkv = r[7] if nx else None
    return out


def post_attn_ln_linear_fwd(o, x, wo, bo, g2, be2, eps, w1, b1, w2, b2, lnw, lnb, wq, bq, seed=None, site=0, p=0.0):
    """post_attn_fwd of layer l, then ln_linear_fwd (LN1 + packed QKV) of layer l+1."""
    z, y, m2, r2, u = post_attn_fwd(o, x, wo, bo, g2, be2, eps, w1, b1, w2, b2, seed, site, p)
    qkv, mean1, rstd1 = ln_linear_fwd(z, lnw, lnb, eps, wq, bq, 0, None, True, True)
    return z, y, m2, r2, u, qkv, mean1, rstd1


def ln_linear_post_attn_bwd(g, wq, x, mean1, rstd1, lnw, lnb, dres, ll_grads, y, m2, r2, u, o, wo, w1, w2, g2, be2,
                            H, pa_grads, job_slab=None, job_dsts=(), job_offs=(), seed=None, site=0, p=0.0,
                            zero_out=None, att_qkv=None, att_lse=None, att_out=None, att_scale=0.0):
    """ln_linear_bwd of layer l+1 (dX = dZ of layer l, incl. dres) → post_attn_bwd of layer l,
    both into slab targets.  att_out: layer l's attention backward too (64 latents per sample,
    csrc/chain.hip phase D), its dQKV written into att_out (R, 3C) bf16."""
    _run_job(job_slab, job_dsts, job_offs)
    dz = ln_linear_bwd(g, wq, x, mean1, rstd1, lnw, lnb, dres, True, *ll_grads, slab=True)
    dy, do, delta = post_attn_bwd(dz, y, m2, r2, u, o, wo, w1, w2, g2, be2, H, pa_grads, slab=True, seed=seed,
                                  site=site, p=p)
    if att_out is not None:
        R, C = y.shape
        B, N = R // 64, 64
        q3 = att_qkv.view(B, N, 3 * C)
        d3 = torch.empty(B, N, 3 * C, device=y.device)
        attn_bwd(q3[:, :, :C], q3[:, :, C:2 * C], q3[:, :, 2 * C:], None, o.view(B, N, C), do.view(B, N, C),
                 att_lse.view(B, N, H), delta.view(B, N, H), H, C // H, att_scale, p, seed, d3[:, :, :C],
                 d3[:, :, C:2 * C], d3[:, :, 2 * C:], site=site)
        att_out.view(R, 3 * C).copy_(d3.view(R, 3 * C))
    return dy, do, delta


def _heads(x, H):
    b, n, _ = x.shape
    return x[:, :, : x.shape[2]].reshape(b, n, H, -1).permute(0, 2, 1, 3)


def _qkv(q, k, v, H, D):
    B = max(q.shape[0], k.shape[0])
    qf = q[:, :, : H * D].float().expand(B, -1, -1).reshape(B, q.shape[1], H, D).permute(0, 2, 1, 3)
    kf = k[:, :, : H * D].float().reshape(B, k.shape[1], H, D).permute(0, 2, 1, 3)
    vf = v[:, :, : H * D].float().reshape(B, v.shape[1], H, D).permute(0, 2, 1, 3)
    return B, qf, kf, vf


def _scores(qf, kf, kmask, scale):
    s = torch.matmul(qf, kf.transpose(-1, -2)) * scale
    if kmask is not None:
        s = s.masked_fill(kmask.view(kmask.shape[0], 1, 1, -1).bool(), float("-inf"))
    return s


def attn_fwd(q, k, v, kmask, H, D, scale, dropout_p, seed, nsplit, site=0):
    B, qf, kf, vf = _qkv(q, k, v, H, D)
    s = _scores(qf, kf, kmask, scale)
    lse = torch.logsumexp(s, -1)  # (B, H, Nq), -inf for dead rows
    p = torch.exp(s - lse[..., None])
    p = torch.nan_to_num(p, nan=0.0)
    if dropout_p > 0:
        p = p * attn_drop_mask(seed, site, B, H, q.shape[1], k.shape[1], dropout_p, q.device)
    o = torch.matmul(_bf(p), vf)
    lse2 = torch.where(torch.isfinite(lse), lse * LOG2E, torch.full_like(lse, float("inf")))
    o = o.permute(0, 2, 1, 3).reshape(B, q.shape[1], H * D).to(torch.bfloat16)
    return o, lse2.permute(0, 2, 1).contiguous()


def attn_bwd(q, k, v, kmask, o, dO, lse, delta_in, H, D, scale, dropout_p, seed, dq_out, dk_out, dv_out,
             kv_accumulate=False, site=0, dq_zeroed=False, kv_zeroed=False, job_slab=None, job_dsts=(), job_offs=()):
    _run_job(job_slab, job_dsts, job_offs)
    B, qf, kf, vf = _qkv(q, k, v, H, D)
    s = _scores(qf, kf, kmask, scale)
    l2 = lse.permute(0, 2, 1)  # (B, H, Nq)
    p = torch.exp2(s * LOG2E - l2[..., None])
    p = torch.nan_to_num(p, nan=0.0)
    dof = dO.float().reshape(B, -1, H, D).permute(0, 2, 1, 3)
    if delta_in is not None:  # rowsum(dO∘O) from the post-attention backward
        delta = delta_in.float().reshape(B, -1, H).permute(0, 2, 1)[..., None]
    else:
        of = o.float().reshape(B, -1, H, D).permute(0, 2, 1, 3)
        delta = (dof * of).sum(-1, keepdim=True)
    dp = torch.matmul(dof, vf.transpose(-1, -2))
    if dropout_p > 0:
        m = attn_drop_mask(seed, site, B, H, q.shape[1], k.shape[1], dropout_p, q.device)
        ds = p * (dp * m - delta)
        pd = p * m
    else:
        ds = p * (dp - delta)
        pd = p
    dq = torch.matmul(ds, kf) * scale
    dk = torch.matmul(ds.transpose(-1, -2), qf) * scale
    dv = torch.matmul(pd.transpose(-1, -2), dof)

    def merge(t):
        return t.permute(0, 2, 1, 3).reshape(B, t.shape[2], H * D)

    res = []
    for i, (t, out) in enumerate(((dq, dq_out), (dk, dk_out), (dv, dv_out))):
        t = merge(t)
        if out is not None:
            if kv_accumulate and i > 0:
                out[:, :, : H * D] += t
            else:
                out[:, :, : H * D].copy_(t)
            t = out
        res.append(t)
    return res


def post_attn_fwd(o, x, wo, bo, g2, be2, eps, w1, b1, w2, b2, seed=None, site=0, p=0.0):
    """x may have R / k rows (batch-broadcast residual): row r adds x[r % rows(x)].
    p > 0: residual dropout with the kernels' hashed masks (sub-streams 0 / 1)."""
    if x.shape[0] != o.shape[0]:
        x = x.repeat(o.shape[0] // x.shape[0], 1)
    R, C = o.shape
    a = _bf(o.float()) @ _bf(wo.float()).t() + bo
    if p > 0:
        a = a * row_drop_mask(seed, site, 0, R, C, p, o.device)
    y = x + a
    xn, m, r = _ln(y, g2, be2, eps)
    u = _bf(xn) @ _bf(w1.float()).t() + b1
    h = F.gelu(u)
    f = _bf(h) @ _bf(w2.float()).t() + b2
    if p > 0:
        f = f * row_drop_mask(seed, site, 1, R, C, p, o.device)
    z = y + f
    return z, y, m, r, u.to(torch.bfloat16)


def _gelu_grad(u):
    cdf = 0.5 * (1.0 + torch.erf(u * 0.7071067811865476))
    pdf = 0.3989422804014327 * torch.exp(-0.5 * u * u)
    return cdf + u * pdf


def _ln_bwd(dxn, x, mean, rstd, w):
    xh = (x - mean[:, None]) * rstd[:, None]
    g = dxn * w
    s1 = g.mean(-1, keepdim=True)
    s2 = (g * xh).mean(-1, keepdim=True)
    return rstd[:, None] * (g - s1 - xh * s2), xh


def _run_job(job_slab, job_dsts, job_offs):
    """the slab-reduction job a HIP backward kernel runs in its appended workgroups"""
    if job_slab is not None:
        slab_reduce(job_slab, job_dsts, job_offs)


def post_attn_bwd(dz, y, m2, r2, u, o, wo, w1, w2, g2, be2, H, grads, slab=False, job_slab=None, job_dsts=(),
                  job_offs=(), seed=None, site=0, p=0.0, zero_out=None):
    """Returns (dy, dO, delta); parameter grads are ACCUMULATED into
    grads = [dWo, dbo, dg2, dbe2, dW1, db1, dW2, db2] (or stored into slab views)."""
    _run_job(job_slab, job_dsts, job_offs)
    _SLAB[0] = slab
    try:
        return _post_attn_bwd(dz, y, m2, r2, u, o, wo, w1, w2, g2, be2, H, grads, seed, site, p)
    finally:
        _SLAB[0] = False


def _post_attn_bwd(dz, y, m2, r2, u, o, wo, w1, w2, g2, be2, H, grads, seed=None, site=0, p=0.0):
    dWo, dbo, dg2, dbe2, dW1, db1, dW2, db2 = grads
    R, C = dz.shape
    uf = u.float()
    dzm = dz * row_drop_mask(seed, site, 1, R, C, p, dz.device) if p > 0 else dz
    dh = _bf(dzm) @ _bf(w2.float())
    _acc(dW2, _bf(dzm).t() @ _bf(F.gelu(uf)))
    _acc(db2, dzm.sum(0))
    du = dh * _gelu_grad(uf)
    dxn = _bf(du) @ _bf(w1.float())
    xn = (y - m2[:, None]) * r2[:, None] * g2 + be2
    _acc(dW1, _bf(du).t() @ _bf(xn))
    _acc(db1, du.sum(0))
    dln, xh = _ln_bwd(dxn, y, m2, r2, g2)
    dy = dz + dln
    dym = dy * row_drop_mask(seed, site, 0, R, C, p, dz.device) if p > 0 else dy
    do = (_bf(dym) @ _bf(wo.float())).to(torch.bfloat16)
    _acc(dWo, _bf(dym).t() @ _bf(o.float()))
    _acc(dbo, dym.sum(0))
    D = C // H
    delta = (do.float().view(R, H, D) * o.float().view(R, H, D)).sum(-1)
    _acc(dg2, (dxn * xh).sum(0))
    _acc(dbe2, dxn.sum(0))
    return dy, do, delta


def ln_linear_bwd(g, w, x, mean, rstd, lnw, lnb, dres, need_dx, dlnw=None, dlnb=None, dW=None, db=None, pe=None,
                  kin=-1, slab=False, job_slab=None, job_dsts=(), job_offs=(), dx_out=None, pe_index=None):
    """Returns dX (or None); LN grads accumulate into dlnw / dlnb and, when given,
    dW += gᵀ·LN(x), db += Σ_rows g (slab: stored into (tiles, ·) slab views)."""
    _run_job(job_slab, job_dsts, job_offs)
    _SLAB[0] = slab
    try:
        dx = _ln_linear_bwd(g, w, x, mean, rstd, lnw, lnb, dres, need_dx, dlnw, dlnb, dW, db, pe, kin, pe_index)
    finally:
        _SLAB[0] = False
    if dx is not None and dx_out is not None:
        dx_out.copy_(dx)
        return dx_out
    return dx


def _ln_linear_bwd(g, w, x, mean, rstd, lnw, lnb, dres, need_dx, dlnw, dlnb, dW, db, pe, kin, pe_index=None):
    if kin >= 0:
        w = w[:, :kin]
    gf = g.float()
    dxn = _bf(gf) @ _bf(w.float())
    xf = _split_x(x, pe, w.shape[1], pe_index)
    if dW is not None:
        xn = (xf - mean[:, None]) * rstd[:, None] * lnw + lnb if lnw is not None else xf
        _acc(dW, _bf(gf).t() @ _bf(xn))
        if db is not None:
            _acc(db, gf.sum(0))
    if lnw is not None:
        d, xh = _ln_bwd(dxn, xf, mean, rstd, lnw)
        _acc(dlnw, (dxn * xh).sum(0))
        _acc(dlnb, dxn.sum(0))
    else:
        d = dxn
    if need_dx:
        return d + dres if dres is not None else d
    return None


def wgrad(g, a, amode, mean, rstd, lnw, lnb, rows_per_wg, dW, db=None, pe=None, kin=-1, pe_index=None):
    """dW += Gᵀ·A(transformed), db += Σ_rows G (accumulated in place)."""
    af = _split_x(a, pe, kin if kin >= 0 else a.shape[1], pe_index)
    if amode == 1:
        af = (af - mean[:, None]) * rstd[:, None] * lnw + lnb
    elif amode == 2:
        af = F.gelu(af)
    _acc(dW, _bf(g.float()).t() @ _bf(af))
    if db is not None:
        _acc(db, g.float().sum(0))


def mlm_select(labels, cap, gcap, sticky=None, queries=None):
    B, L = labels.shape
    sel = labels != -100
    pos = torch.cumsum(sel.to(torch.int64), 1) - 1
    idx_b = (torch.arange(cap, device=labels.device) % L).repeat(B, 1)
    lab_b = torch.full((B, cap), -100, dtype=torch.int64, device=labels.device)
    keep = sel & (pos < cap)
    rows = torch.arange(B, device=labels.device)[:, None].expand(B, L)
    cols = torch.arange(L, device=labels.device).expand(B, L)
    idx_b[rows[keep], pos[keep]] = cols[keep]
    lab_b[rows[keep], pos[keep]] = labels[keep]
    count = sel.sum(1)
    n = count.clamp(max=cap)
    slot_ok = torch.arange(cap, device=labels.device)[None, :] < n[:, None]
    flat = torch.nonzero(slot_ok.reshape(-1)).reshape(-1)
    gidx = torch.zeros(gcap, dtype=torch.int64, device=labels.device)
    glab = torch.full((gcap,), -100, dtype=torch.int64, device=labels.device)
    m = min(gcap, flat.numel())
    gidx[:m] = flat[:m]
    glab[:m] = lab_b.reshape(-1)[flat[:m]]
    total = count.sum().float().reshape(1)
    ovf = ((count > cap).any() | (n.sum() > gcap)).reshape(1)
    if sticky is not None:
        sticky.logical_or_(ovf.reshape(sticky.shape))
    if queries is not None:
        return idx_b, lab_b, gidx, glab, total, ovf, queries.index_select(0, idx_b.reshape(-1)).view(B, cap, -1)
    return idx_b, lab_b, gidx, glab, total, ovf


def _ce_rows(h, idx):
    return h if idx is None else h.index_select(0, idx)


def ce_fwd(h, idx, labels, w, bias, count, zero_out=None, count_labels=False):
    """→ (mean loss Σ rows / max(count, 1) as a 0-dim tensor, per-row lse); rows of ``h`` are
    gathered through ``idx`` when given; ``zero_out`` (the backward's dH accumulator) is cleared.
    ``count_labels``: ``count`` is written with the number of rows whose label is ≥ 0."""
    if zero_out is not None:
        zero_out.zero_()
    if count_labels:
        count.reshape(-1)[0] = (labels >= 0).sum()
    logits = _bf(_ce_rows(h, idx).float()) @ _bf(w.float()).t() + bias
    lse = torch.logsumexp(logits, -1)
    valid = labels >= 0
    picked = logits.gather(1, labels.clamp(min=0)[:, None])[:, 0]
    loss = torch.where(valid, lse - picked, torch.zeros_like(lse))
    return loss.sum() / count.reshape(()).clamp(min=1), lse, _ce_rows(h, idx).to(torch.bfloat16).contiguous()


def ce_bwd(h, labels, w, bias, lse, gout, count, dH, dW, db, accumulate, rowmap=None, slab=False, u=None, u_ml=None):
    """h: the compact bf16 rows returned by ce_fwd.  slab=True: dW | db are returned as a one-row
    (1, V·C + V₄) slab instead of being added.  ``u`` / ``u_ml`` (the HIP two-pass head's forward
    outputs) are not needed here: dH is formed from the logits."""
    if slab:
        gw, gb = torch.zeros_like(dW), torch.zeros_like(db)
        ce_bwd(h, labels, w, bias, lse, gout, count, dH, gw, gb, False, rowmap)
        V = w.shape[0]
        out = torch.zeros(1, dW.numel() + (V + 3) // 4 * 4, dtype=dW.dtype, device=dW.device)
        out[0, :dW.numel()] = gw.reshape(-1)
        out[0, dW.numel():dW.numel() + V] = gb
        return out
    gscale = gout.reshape(()) / count.reshape(()).clamp(min=1)
    logits = _bf(h.float()) @ _bf(w.float()).t() + bias
    p = torch.exp(logits - lse[:, None])
    valid = (labels >= 0).float()[:, None]
    onehot = F.one_hot(labels.clamp(min=0), w.shape[0]).float()
    dl = (p - onehot) * valid * gscale
    rows = _bf(dl) @ _bf(w.float())
    if rowmap is None:
        dH.add_(rows)
    else:
        keep = labels >= 0
        dH.index_add_(0, rowmap[keep], rows[keep])
    gw = _bf(dl).t() @ _bf(h.float())
    gb = dl.sum(0)
    if accumulate:
        dW.add_(gw)
        db.add_(gb)
    else:
        dW.copy_(gw)
        db.copy_(gb)
    return None


def embed_fwd(ids, E, P, scale):
    return E[ids] * scale + P[: ids.shape[1]].unsqueeze(0)


def embed_bwd(ids, g, dE, dP, scale, job_slab=None, job_dsts=(), job_offs=()):
    _run_job(job_slab, job_dsts, job_offs)
    C = g.shape[-1]
    if dE is not None:
        dE.index_add_(0, ids.reshape(-1), g.reshape(-1, C) * scale)
    if dP is not None:
        dP[: ids.shape[1]] += g.sum(0)


def _unit24(h):
    return (h >> 8).to(torch.float32) * (1.0 / 16777216.0)


def _mulhi32(a, b: int):
    """floor(a · b / 2^32) for uint32 a (int64 tensor) and b < 2^32, exact in int64."""
    return ((a >> 16) * b + (((a & 0xFFFF) * b) >> 16)) >> 16


def text_mask(x, pad, state, unk, mask, p, lo, hi, advance=True):
    """Counter-hash BERT masking, bit-exact with ``text_mask_kernel`` (elementwise.hip)."""
    seed = int(state[0].item()) & 0xFFFFFFFFFFFFFFFF
    ctr = int(state[1].item())
    key = hash3(torch.tensor(seed & M32), torch.tensor(seed >> 32), torch.tensor(ctr & M32))
    i = torch.arange(x.numel(), device=x.device, dtype=torch.int64).view(x.shape)
    h = [hash3(key.to(x.device), torch.tensor(k, device=x.device), i) for k in range(4)]
    special = x == unk
    if pad is not None:
        special = special | pad
    sel = ~special & (_unit24(h[0]) < p)
    msk = sel & (_unit24(h[1]) < 0.9)
    rnd = msk & (_unit24(h[2]) < 1.0 / 9.0)
    rid = lo + _mulhi32(h[3], hi - lo)
    xm = torch.where(rnd, rid, torch.where(msk, torch.full_like(x, mask), x))
    if advance:
        state[1] += 1
    return xm, torch.where(sel, x, torch.full_like(x, -100))


def sumsq(g, part):
    """Σ g² as the kernel's partial buffer (csrc elementwise.hip sumsq_kernel): here one partial."""
    part.zero_()
    part[0] = (g.float() ** 2).sum()


def adamw(p, g, m, v, shadow, hyper, eps, wd, clip, gscale, l2=False, zero_grad=False, loss_src=None, loss_ring=None,
          norm_part=None):
    lr, step, b1, b2 = float(hyper[0]), float(hyper[1]), float(hyper[3]), float(hyper[4])
    if loss_src is not None:  # the step's loss into the engine's ring slot hyper[7]
        loss_ring.view(-1)[int(float(hyper[7])) % loss_ring.numel()] = loss_src.reshape(())
    gs = gscale
    if clip > 0:
        norm = math.sqrt(float(norm_part.sum())) * gscale  # norm of the mean (all-reduced sum × 1/world)
        f = clip / (norm + 1e-6)
        if f < 1:
            gs *= f
    gg = g * gs
    if zero_grad:
        g.zero_()
    if l2:  # torch.optim.Adam: coupled L2 decay added to the (clipped) gradient
        gg = gg + wd * p
    else:
        p.mul_(1 - lr * wd)
    m.mul_(b1).add_(gg, alpha=1 - b1)
    v.mul_(b2).addcmul_(gg, gg, value=1 - b2)
    bc1, bc2 = 1 - b1 ** step, 1 - b2 ** step
    denom = (v.sqrt() / math.sqrt(bc2)).add_(eps)
    p.addcdiv_(m, denom, value=-lr / bc1)
    if shadow is not None:
        shadow.copy_(p.to(shadow.dtype))


def fold_replicas(grad, rep):
    n = rep.shape[1]
    grad[:n] += rep.sum(0)
    rep.zero_()


def slab_reduce(slab, dsts, offs):
    for d, o in zip(dsts, offs):
        n = d.numel()
        if n:
            d += slab[:, o:o + n].float().sum(0).view(d.shape)  # bf16 slabs are summed in fp32


def set_deterministic(flag):
    """the emulation has no atomics: nothing to switch"""


def get_deterministic():
    return False


def cast_bf16(x, y):
    y.copy_(x.to(torch.bfloat16).view(y.shape))


def batch_sum2(a, b, ob_acc=None):
    sb = b.sum(0)
    if ob_acc is not None:
        ob_acc.add_(sb.view_as(ob_acc))
        sb = ob_acc.view_as(sb)
    return (a.sum(0) if a is not None else None), sb


def index_add_rows(dst, idx, src):
    dst.index_add_(0, idx, src.to(dst.dtype))


def gather_rows(src, idx):
    ok = (idx >= 0) & (idx < src.shape[0])
    return torch.where(ok[:, None], src.index_select(0, idx.clamp(0, src.shape[0] - 1)), torch.zeros((), dtype=src.dtype))


def _pixel_logits(h, w, b):
    return h.float() @ w.float().t() + b.float()


def pixel_ce_fwd(h, w, b, labels, wts):
    """(stats, loss): stats = [Σ w·ce, Σ w, n(lab>0), hit(lab>0), (n_k, hit_k)… | acc, acc_1…]
    (pixel_head.hip), loss = Σ w·ce / Σ w."""
    part = _pixel_ce_sums(h, w, b, labels, wts)
    K = w.shape[0]

    def ratio(hit, n):
        return torch.where(n > 0, hit / n.clamp(min=1), torch.zeros_like(n))

    accs = [ratio(part[3], part[2])] + [ratio(part[5 + 2 * k], part[4 + 2 * k]) for k in range(1, K)]
    return torch.cat([part, torch.stack(accs)]), part[0] / part[1]


def _pixel_ce_sums(h, w, b, labels, wts):
    K = w.shape[0]
    z = _pixel_logits(h, w, b)
    valid = (labels >= 0) & (labels < K)
    lab = labels.clamp(0, K - 1)
    ce = torch.logsumexp(z, -1) - z.gather(1, lab[:, None])[:, 0]
    wl = torch.where(valid, wts[lab], torch.zeros_like(ce))
    hit = (z.argmax(-1) == lab) & valid
    out = [(wl * ce).sum(), wl.sum(), (valid & (lab > 0)).sum().float(), (hit & (lab > 0)).sum().float()]
    for k in range(K):
        out += [(valid & (lab == k)).sum().float(), (hit & (lab == k)).sum().float()]
    return torch.stack(out)


def pixel_ce_bwd(h, w, b, labels, wts, gout, stats, dH, dW, db):
    gscale = gout.reshape(1).float() / stats[1]
    K, C = w.shape
    z = _pixel_logits(h, w, b)
    valid = (labels >= 0) & (labels < K)
    lab = labels.clamp(0, K - 1)
    p = torch.softmax(z, -1)
    coef = p - torch.nn.functional.one_hot(lab, K).float()
    coef = coef * (torch.where(valid, wts[lab], torch.zeros_like(p[:, 0])) * gscale.float())[:, None]
    dH.copy_(coef @ w.float())
    dW += (coef.t() @ h.float()).view_as(dW)
    db += coef.sum(0)


# ---- per-sample latent-block kernels (csrc/sample_block.hip): 32 latents, 4 heads -------------
# the same operands, bf16 rounding points and outputs as sb_fwd / sb_bwd / sb_wgrad
_SB_N, _SB_H = 32, 4


def _sb_unpack(params, i):
    return params[12 * i:12 * (i + 1)]


def _sb_heads(t, B, C):  # (B·32, C) → (B, H, 32, d)
    return t.view(B, _SB_N, _SB_H, C // _SB_H).transpose(1, 2)


def _sb_probs(q, k, scale):
    """normalised softmax probabilities (fp32) from bf16 q, k (B, H, 32, d)"""
    s = q @ k.transpose(-1, -2)
    return torch.softmax(s * scale, dim=-1)


def _sb_pre_fwd(pre, R, C, eps):
    """the pre stage: the cross layer's post-attention half (O, x_q → y, LN2, MLP → z0)."""
    o, xq, wo, bo, g2, be2, w1, b1, w2, b2 = pre
    if xq.shape[0] != R:  # broadcast latents
        xq = xq.repeat(R // xq.shape[0], 1)
    y = o.float() @ wo.float().t() + bo + xq
    t2, mean2, rstd2 = _ln(y, g2, be2, eps)
    ln2y = _bf(t2)
    u = ln2y @ w1.float().t() + b1
    gu = _bf(F.gelu(u))
    z = gu @ w2.float().t() + b2 + y
    bf = torch.bfloat16
    return z, [ln2y.to(bf), u.to(bf), gu.to(bf), y, mean2, rstd2]


def sb_fwd(x, params, scale, eps, pre=(), post=()):
    """pre (10 tensors): the cross layer's post-attention half first; x (the block input) is
    written with its output and its 6 saved tensors are appended."""
    R, C = x.shape
    B = R // _SB_N
    L = len(params) // 12
    out = []
    pre_saved = []
    if pre:
        z0, pre_saved = _sb_pre_fwd(pre, R, C, eps)
        x.copy_(z0)
    for i in range(L):
        g1, be1, wqkv, bqkv, wo, bo, g2, be2, w1, b1, w2, b2 = _sb_unpack(params, i)
        t, mean1, rstd1 = _ln(x, g1, be1, eps)
        ln1x = _bf(t)
        qkv = _bf(ln1x @ wqkv.float().t() + bqkv)
        q, k, v = (_sb_heads(qkv[:, j * C:(j + 1) * C], B, C) for j in range(3))
        p = _sb_probs(q, k, scale)
        # O = Σ bf16(p̃)·v / Σ p̃ with p̃ = exp(s − max): the kernel rounds the unnormalised probabilities
        s = (q @ k.transpose(-1, -2)) * scale
        pt = torch.exp(s - s.amax(-1, keepdim=True))
        o = (_bf(pt) @ v) / pt.sum(-1, keepdim=True)
        o = _bf(o.transpose(1, 2).reshape(R, C))
        y = o @ wo.float().t() + bo + x
        t2, mean2, rstd2 = _ln(y, g2, be2, eps)
        ln2y = _bf(t2)
        u = ln2y @ w1.float().t() + b1
        gu = _bf(F.gelu(u))
        z = gu @ w2.float().t() + b2 + y
        bf = torch.bfloat16
        out += [ln1x.to(bf), qkv.to(bf), o.to(bf), ln2y.to(bf), u.to(bf), gu.to(bf), y, z, mean1, rstd1, mean2, rstd2]
        del p
        x = z
    post_out = []
    if post:  # the next cross layer's LN + query projection of the block output
        g, b, wq, bq = post
        t, mean, rstd = _ln(x, g, b, eps)
        lnx = _bf(t)
        q = _bf(lnx @ wq.float().t() + bq)
        post_out = [q.to(torch.bfloat16), lnx.to(torch.bfloat16), mean, rstd]
    return out + pre_saved + post_out


def sb_bwd(dz, x0, saved, params, scale, eps, pre=(), pre_saved=(), zero_out=None, post=(), post_io=()):
    R, C = x0.shape
    B = R // _SB_N
    L = len(params) // 12
    grads = [None] * L
    lns = torch.empty(B, 4 * L * C + (2 * C if pre else 0) + (2 * C if post else 0), dtype=torch.float32,
                      device=x0.device)
    if zero_out is not None:
        zero_out.zero_()
    post_tail = []
    if post:  # the next cross layer's query-path backward first: dz = dres + LN_q backward of dQ·Wq
        g, _, wq, _ = post
        dq, dres, mean, rstd = post_io
        dqb = _bf(dq.float())
        dxn = dqb @ wq.float()
        dxl, xh = _ln_bwd(dxn, saved[12 * (L - 1) + 7], mean, rstd, g)
        o = (4 * L + (2 if pre else 0)) * C
        lns[:, o:o + C] = (dxn * xh).view(B, _SB_N, C).sum(1)
        lns[:, o + C:o + 2 * C] = dxn.view(B, _SB_N, C).sum(1)
        dz = dres.float() + dxl
        post_tail = [dqb.to(torch.bfloat16)]

    def per_sample(t):  # (B·32, C) → the sample sums (B, C)
        return t.view(B, _SB_N, C).sum(1)
    dz = dz.float()
    for i in reversed(range(L)):
        g1, be1, wqkv, bqkv, wo, bo, g2, be2, w1, b1, w2, b2 = _sb_unpack(params, i)
        ln1x, qkv, o, ln2y, u, gu, y, z, mean1, rstd1, mean2, rstd2 = saved[12 * i:12 * (i + 1)]
        x = saved[12 * (i - 1) + 7] if i > 0 else x0
        dzb = _bf(dz)
        du = _bf((dzb @ w2.float()) * _gelu_grad(u.float()))
        dxn2 = du @ w1.float()
        dyl, yh = _ln_bwd(dxn2, y, mean2, rstd2, g2)
        dy = dz + dyl
        lns[:, (4 * i + 2) * C:(4 * i + 3) * C] = per_sample(dxn2 * yh)
        lns[:, (4 * i + 3) * C:(4 * i + 4) * C] = per_sample(dxn2)
        dyb = _bf(dy)
        do = _bf(dyb @ wo.float())
        qf = qkv.float()
        q, k, v = (_sb_heads(qf[:, j * C:(j + 1) * C], B, C) for j in range(3))
        doh = _sb_heads(do, B, C)
        oh = _sb_heads(o.float(), B, C)
        p = _sb_probs(q, k, scale)
        dp = doh @ v.transpose(-1, -2)
        delta = (doh * oh).sum(-1, keepdim=True)
        ds = p * (dp - delta)
        dv = _bf(p).transpose(-1, -2) @ doh
        dq = (_bf(ds) @ k) * scale
        dk = (_bf(ds).transpose(-1, -2) @ q) * scale
        dqkv = torch.cat([t.transpose(1, 2).reshape(R, C) for t in (dq, dk, dv)], 1)
        dqkvb = _bf(dqkv)
        dxn1 = dqkvb @ wqkv.float()
        dxl, xh = _ln_bwd(dxn1, x, mean1, rstd1, g1)
        lns[:, 4 * i * C:(4 * i + 1) * C] = per_sample(dxn1 * xh)
        lns[:, (4 * i + 1) * C:(4 * i + 2) * C] = per_sample(dxn1)
        bf = torch.bfloat16
        grads[i] = [dqkvb.to(bf), dyb.to(bf), du.to(bf), dzb.to(bf)]
        dz = dy + dxl
    tail = []
    if pre:  # the cross layer's post-attention backward: dO, δ, and dX = dY (the x_q residual path)
        o, _, wo, bo, g2, be2, w1, b1, w2, b2 = pre
        ln2y, u, gu, y, mean2, rstd2 = pre_saved
        dzb = _bf(dz)
        du = _bf((dzb @ w2.float()) * _gelu_grad(u.float()))
        dxn2 = du @ w1.float()
        dyl, yh = _ln_bwd(dxn2, y, mean2, rstd2, g2)
        dy = dz + dyl
        lns[:, 4 * L * C:(4 * L + 1) * C] = per_sample(dxn2 * yh)
        lns[:, (4 * L + 1) * C:(4 * L + 2) * C] = per_sample(dxn2)
        dyb = _bf(dy)
        do = _bf(dyb @ wo.float())
        delta = (do * o.float()).view(R, 4, C // 4).sum(-1)
        bf = torch.bfloat16
        tail = [do.to(bf), delta, dyb.to(bf), du.to(bf), dzb.to(bf)]
        dz = dy
    out = [dz, lns]
    for g in grads:
        out += g
    return out + tail + post_tail


def sb_wgrad(jobs, job_slab=None, job_dsts=(), job_offs=()):
    _run_job(job_slab, job_dsts, job_offs)
    for j in range(0, len(jobs), 4):
        G, A, dW, db = jobs[j:j + 4]
        Gf = G.float()
        dW.view(Gf.shape[1], A.shape[1]).add_(Gf.t() @ A.float())
        db.view(-1).add_(Gf.sum(0))
