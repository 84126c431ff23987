"""CPU: the host logic of the GEMM-composed maf backward (naz_amd/flows/maf_grad_wide.py) — the
per-layer order of the D - 1 input chains, the degree blocks (4-unit boundaries, the forward's input
ranges, the transposed products' output ranges, the input chains' unit prefixes) and the flat dW
layout — against torch autograd of a float64 restatement of the maf log-density (pyro
AffineAutoregressive._inverse per layer, naz transforms.py:133-198; the clamp of pyro's
clamp_preserve_gradients and jnp.clip's zero gradient, bflow_jax_maf.py:177-192).

The native kernels the class launches are replaced here by float64 torch stand-ins of their C-ABI
contracts (include/naz_hip.h): this checks the composition, not the kernels, which
tests/test_gpu_train.py::test_wide_maf_train_path_vs_oracle_and_walk covers on the GPU."""
import numpy as np
import pytest
import torch

from naz_amd import ops
from naz_amd.flows import maf_grad_wide as mgw


def _stand_ins(monkeypatch):
    def linear_act(x, weight, bias, act="identity", context=None, mask=None, out=None):
        w = weight if mask is None else weight * mask
        inp = x
        if context is not None:
            c = context.reshape(1, -1).expand(x.shape[0], -1) if context.dim() == 1 or context.shape[0] == 1 else context
            inp = torch.cat([c, x], 1)
        y = inp @ w.t() + bias
        y = torch.tanh(y) if act == "tanh" else y
        out.copy_(y)
        return out

    def gemm_dact(a, weight, y, act, mask=None, out=None):
        assert act == "tanh" and out.data_ptr() % 16 == 0 and out.stride(0) % 4 == 0  # the kernel's contract
        w = weight if mask is None else weight * mask
        out.copy_((a @ w) * (1 - y * y))
        return out

    def gemm(a, b, out=None, mask=None, mask_b=False, accumulate=False, split_k=None, rowsum=None):
        bb = b * mask if (mask is not None and mask_b) else b
        r = a @ bb
        if accumulate:
            out.add_(r)
        else:
            out.copy_(r)
        if rowsum is not None:
            rowsum.add_(a.sum(1)) if accumulate else rowsum.copy_(a.sum(1))
        return out

    def maf_dim_vjp(raw, s, g, g_lp, dim, g_next, tot, chain=None, clip_zero=False):
        D = s.shape[1]
        a = raw[:, D + dim]
        ls = a.clamp(-5, 3)
        gy = g[:, dim] * torch.exp(-ls)
        ga = -g_lp - g[:, dim] * s[:, dim]
        if clip_zero:
            ga = torch.where((a >= -5) & (a <= 3), ga, torch.zeros_like(ga))
        g_next[:, dim] = gy
        tot[:, dim] = -gy
        tot[:, D + dim] = ga
        if chain is not None:
            chain.zero_()
            chain[:, dim] = -gy
            chain[:, D + dim] = ga

    monkeypatch.setattr(ops, "linear_act", linear_act)
    monkeypatch.setattr(ops, "gemm_dact", gemm_dact)
    monkeypatch.setattr(ops, "gemm", gemm)
    monkeypatch.setattr(ops, "maf_dim_vjp", maf_dim_vjp)
    monkeypatch.setattr(ops, "base_log_prob_bwd", lambda z, g_lp: -z * g_lp[:, None])


def _flow(desc, seed):
    """Random masked flat weights [L * per], the mask, per-layer permutations (pyro's masks for the
    compiled hidden degrees, naz_oracle.py:185-209)."""
    D, C, H, L, NH = desc.D, desc.C, desc.H, desc.L, desc.n_hidden
    rng = np.random.default_rng(seed)
    deg = ops.ar_flow_degrees(desc).astype(np.int64)
    flats, masks, perms = [], [], []
    for _ in range(L):
        perm = rng.permutation(D)
        order = np.empty(D, dtype=np.int64)
        order[perm] = np.arange(D)
        in_idx = np.concatenate([np.zeros(C, dtype=np.int64), order + 1])
        out_idx = np.tile(order + 1, 2)
        ms = [deg[:, None] >= in_idx[None, :]] + [deg[:, None] >= deg[None, :]] * (NH - 1) + \
             [out_idx[:, None] > deg[None, :]]
        for m in ms:
            w = rng.normal(0, 0.6 / np.sqrt(m.shape[1]), m.shape)
            flats += [w.ravel(), rng.normal(0, 0.1, m.shape[0])]
            masks += [m.astype(np.float64).ravel(), np.ones(m.shape[0])]
        perms.append(perm)
    return (torch.as_tensor(np.concatenate(flats)), torch.as_tensor(np.concatenate(masks)),
            np.stack(perms).astype(np.int32))


def _reference(g, flat, mask, perms, x, ctx, g_lp, clip_zero):
    """Σ g_lp · log p(x | ctx) of the L-layer maf (float64, the D-pass inverse per layer, autograd),
    its gradient in the flat order, and every layer's output [L, B, D]."""
    D, C, H, L, NH = g.desc.D, g.desc.C, g.desc.H, g.desc.L, g.desc.n_hidden
    w = (flat * mask).clone().requires_grad_(True)
    B = x.shape[0]
    cb = ctx.reshape(1, -1).expand(B, C)

    def made(l, v):
        Ws = g._views(w, l)
        h = torch.cat([cb, v], 1)
        for i in range(NH):
            h = torch.tanh(h @ Ws[i][0].t() + Ws[i][1])
        return h @ Ws[NH][0].t() + Ws[NH][1]

    def clip(a):
        if clip_zero:
            return a.clamp(-5, 3)
        return a + (a.clamp(-5, 3) - a).detach()  # clamp_preserve_gradients

    y = x
    states = [None] * L
    ld = torch.zeros(B, dtype=torch.float64)
    for l in range(L - 1, -1, -1):
        v = torch.zeros_like(y)
        for p in range(D):
            raw = made(l, v)
            dp = int(perms[l, p])
            col = (y[:, dp] - raw[:, dp]) * torch.exp(-clip(raw[:, D + dp]))
            v = torch.cat([v[:, :dp], col[:, None], v[:, dp + 1:]], 1)
        raw = made(l, v)
        ld = ld + clip(raw[:, D:]).sum(1)
        y = v
        states[l] = v.detach()
    lp = -(y * y).sum(1) / 2 - D * 0.91893853320467274178 - ld
    (gw,) = torch.autograd.grad((g_lp * lp).sum(), [w])
    return gw * mask, torch.stack(states)


@pytest.mark.parametrize("blocks,clip_zero,ctx_rows", [(True, False, True), (False, False, True),
                                                        (True, True, False)])
def test_wide_backward_composition_matches_autograd(monkeypatch, blocks, clip_zero, ctx_rows):
    _stand_ins(monkeypatch)
    desc = ops.ar_flow_desc("maf", 4, 2, 512, 2, n_hidden=5)
    flat, mask, perms = _flow(desc, seed=3)
    g = mgw.WideMafGrad(desc, perms, mask.float(), clip_zero=clip_zero, blocks=blocks)
    assert g.blocked == blocks
    if blocks:  # D=4, H=512: hidden degrees 0 | 1 | 2 | 3 over 86 | 170 | 170 | 86 units
        assert [(a, b) for a, b, _, _ in g.blocks] == [(0, 84), (84, 256), (256, 424), (424, 512)]
        assert [fk for *_, fk, _ in g.blocks] == [88, 256, 432, 512]
        assert [k0 for *_, k0 in g.blocks] == [0, 0, 256, 256]
        assert (g.prefix[1], g.prefix[2], g.prefix[3]) == (256, 428, 512)
    B = 12
    rng = np.random.default_rng(7)
    x = torch.as_tensor(rng.normal(0, 1.5, (B, 4)))
    ctx = torch.as_tensor(rng.normal(0, 1, (B if ctx_rows else 1, 2)))
    g_lp = torch.as_tensor(rng.normal(0, 1, B))
    if not ctx_rows:
        ref, states = _reference(g, flat, mask, perms, x, ctx, g_lp, clip_zero)
    else:  # per-row contexts: the reference with each row's own context
        refs, sts = [], []
        for r in range(B):
            gr, st = _reference(g, flat, mask, perms, x[r:r + 1], ctx[r], g_lp[r:r + 1], clip_zero)
            refs.append(gr)
            sts.append(st)
        ref, states = sum(refs), torch.cat(sts, 1)
    wflat = flat * mask
    imgs = (None, wflat, wflat[g.fidx])
    g.ws = g.ws.double()
    g.mask = g.mask.double()
    f64 = dict(dtype=torch.float64)
    g._bufs[B] = dict(g=torch.empty((B, 4), **f64), g_next=torch.empty((B, 4), **f64),
                      h=[torch.zeros((B, 512), **f64) for _ in range(5)], da=torch.empty((B, 512), **f64),
                      db=torch.empty((B, 512), **f64), raw=torch.empty((B, 8), **f64),
                      tot=torch.empty((B, 8), **f64), chain=torch.empty((B, 8), **f64), ones=torch.ones(B, **f64))
    grad, gx = g.backward(imgs, states, ctx, g_lp)
    err = (grad - ref).abs().max() / ref.abs().max()
    assert float(err) < 1e-9, f"blocks={blocks}: max rel error {float(err):.2e}"
    # entries outside the masks stay exact zeros
    assert bool((grad[mask == 0] == 0).all())
