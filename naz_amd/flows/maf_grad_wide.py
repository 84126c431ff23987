"""The maf NLL gradient at fused-inverse shapes without a fused backward kernel (SURVEY.md §8a a10,
VERDICT r03 Next #7: MLE training of naz's production MAFs, D=4 | C=2, H=[512]*5, L=18 —
examples/papers/2506.05657/train_mle_all_data_4param.py:87-92, eposydon/train_maf_mle.py:84-90).

naz's ``train`` differentiates ``flow.log_prob`` every minibatch (train_flows.py:194-213).  The
autograd walk re-runs the D-pass inverse per layer and records every partial GEMM; here the same
gradient is the algorithm of the fused maf backward (made_ar_bwd.h, flows/maf_grad.py) composed of
native GEMM launches, one layer at a time:

  * forward: the fused wide inverse kernel (naz_ar_flow_log_prob_train) saving each layer's
    output s_l [L, B, D] — one launch for all L layers;
  * per layer l = 0 .. L-1 (reverse flow order):
      1. ONE dense MADE pass on (ctx, s_l) (naz_linear_act x (n_hidden + 1)): the masks make every
         hidden unit and every dim's (mean, log_scale) equal to the D-pass inverse's final values;
      2. for order p = D-1 .. 1: dim d_p's VJP (naz_maf_dim_vjp) and its input chain through the
         MADE (naz_gemm_dact per hidden layer, naz_gemm into dL/ds) — the masked weights give
         exact zeros to every dim of order >= p, so the chain adds only what the inverse's
         sequential dependence routes back;
      3. dim d_0's VJP, then ONE chain with every dim's output gradient (the total δ's by
         linearity) whose GEMMs also reduce dW_i = δ_iᵀ h_i and db_i into the flat workspace
         (naz_gemm with the row sum fused);
  * the gradient = workspace ⊙ masks (pyro MaskedLinear's gradient is mask ⊙ δᵀh).

Degree blocks.  pyro's hidden degrees (round(linspace(1, D, H)), oracle/naz_oracle.py:185-189)
never decrease along the unit index, so a degree class is a contiguous run of units and every mask
is block-triangular in that order: hidden unit k reads unit j iff deg(j) <= deg(k).  Each GEMM
therefore runs per class on only its non-zero blocks — forward: out class c over inputs [0, e_c);
transposed products: in class c over outputs [s_c, P) — the input chain of order p only over the
units of degree <= p (the only ones that reach the outputs of order p); units of degree >= D (if
any: they reach no output) not at all.  At D=4, H=[512]x5 that is 136 of the unrestricted 228
MFLOP per row and 18 layers (``flop_per_row``).
``blocks=False`` (NAZ_MAF_WIDE_BLOCKS=0) is the unrestricted A/B: one class of all H units.

No [L, B, ...] operand buffers: each layer's dW is reduced while its activations are live
(n_hidden + 2 [B, H] buffers per row count).  Exact-fp32 MFMA GEMMs throughout (the forward kernel
is the f16x3 split).
"""
from __future__ import annotations

import os
from typing import Optional, Tuple

import numpy as np
import torch
from torch import Tensor

from .. import ops

# dW: one strided GEMM per block (measured faster than the batch-reduction kernel on these strided
# views: 222 vs 254 ms per 2^16-row maf4 step, profiles/r04_s10_*); NAZ_MAF_WIDE_WGRAD=1 = the latter
_ONE_DW_GEMM = os.environ.get("NAZ_MAF_WIDE_WGRAD", "0") != "1"
# the dW reductions on a side stream beside the chain's next transposed product (NAZ_MAF_WIDE_DW_STREAM)
_DW_STREAM = os.environ.get("NAZ_MAF_WIDE_DW_STREAM", "1") == "1"
# ... and the next layer's dense pass on a second stream (NAZ_MAF_WIDE_DENSE_STREAM; needs the first)
_DENSE_STREAM = os.environ.get("NAZ_MAF_WIDE_DENSE_STREAM", "1") == "1"
_SIDE = {}


class WideMafGrad:
    """Same interface as ``maf_grad.MafGrad`` (images / forward / backward / __call__) for an affine
    naz_ar_desc whose inverse is fused (``ops.ar_flow_supported(desc) == 1``) but whose backward is
    not.  ``perms`` [L, D] (dim of order p per layer), ``mask`` [L * per] (MADE masks in the
    naz_ar_flow_pack_host flat layout, 1 on biases); weights arrive as that flat layout."""

    def __init__(self, desc, perms: np.ndarray, mask: Tensor, clip_zero: bool = False, keep_sizes: int = 2,
                 blocks: Optional[bool] = None):
        if desc.kind != ops.AR_KIND["maf"] or ops.ar_flow_supported(desc) != 1:
            raise RuntimeError("WideMafGrad: needs an affine flow with a fused inverse")
        self.desc = desc
        self.clip_zero = bool(clip_zero)
        self.keep_sizes = max(1, int(keep_sizes))
        dev = mask.device
        self.dev = dev
        D, C, H, L, NH = desc.D, desc.C, desc.H, desc.L, desc.n_hidden
        self.shapes = [(H, C + D)] + [(H, H)] * (NH - 1) + [(2 * D, H)]
        offs, o = [], 0
        for (r, c) in self.shapes:
            offs.append((o, o + r * c))
            o += r * c + r
        self.per, self.offs = o, offs
        self.perms = np.ascontiguousarray(np.asarray(perms), dtype=np.int32)
        if self.perms.shape != (L, D):
            raise ValueError(f"WideMafGrad: perms must be [{L}, {D}]")
        self.mask = mask.to(dev, torch.float32).reshape(-1).contiguous()
        if self.mask.numel() != L * o:
            raise ValueError("WideMafGrad: mask does not match the flow's flat parameter count")
        self.ws = torch.zeros(L * o, device=dev, dtype=torch.float32)
        self._bufs = {}
        self._main = self._side = self._dense = None  # streams of the running backward (side: dW
        # reductions; dense: the next layer's dense pass)
        self._evs = []                   # side-stream events, one per submitted reduction
        # unit blocks [a, b) on 4-unit boundaries (the GEMMs store 16-byte row pieces): one per
        # degree class, a class start rounded down; the units past the last class of degree < D are
        # dropped (rounded up).  Per block: fwd_k = the inputs its forward product reads, k0 = the
        # first output its transposed product reads (supersets of the masks' non-zero blocks: the
        # masked weights make the extra terms exact zeros)
        if blocks is None:
            blocks = os.environ.get("NAZ_MAF_WIDE_BLOCKS", "1") != "0"
        deg = ops.ar_flow_degrees(desc).astype(np.int64)
        blocks = bool(blocks) and bool((np.diff(deg) >= 0).all()) and H % 4 == 0
        c4 = lambda v: min(H, (v + 3) // 4 * 4)
        if blocks:
            act = int(np.searchsorted(deg, D, side="left"))  # units of degree < D
            A = c4(act)
            bounds = sorted({int(np.searchsorted(deg, v, side="left")) // 4 * 4 for v in np.unique(deg[:act])} | {A})
            self.blocks = []
            for a, b in zip(bounds[:-1], bounds[1:]):
                live = deg[a:b][deg[a:b] < D]
                fk = min(A, (int(np.searchsorted(deg, live.max(), side="right")) + 7) // 8 * 8)
                k0 = int(np.searchsorted(deg, deg[a], side="left")) // 4 * 4
                self.blocks.append((a, b, fk, k0))
            self.act = A
            self.prefix = {p: c4(int(np.searchsorted(deg, p, side="right"))) for p in range(D)}
        else:
            self.blocks, self.act, self.prefix = [(0, H, H, 0)], H, {p: H for p in range(D)}
        self.blocked = blocks
        # the forward blocks as one contiguous image (naz_linear_act takes dense weights): per layer,
        # W_i[a:b, :fwd_k] per block for i = 1..NH-1, then W_out[:, :act]
        fidx, self.foff = [], []
        fo = 0
        for l in range(L):
            base = l * o
            lay = []
            for i in range(1, NH):
                ow = offs[i][0]
                blk = []
                for (a, b, fk, _) in self.blocks:
                    ii = base + ow + np.arange(a, b)[:, None] * H + np.arange(fk)[None, :]
                    fidx.append(ii.reshape(-1))
                    blk.append(fo)
                    fo += (b - a) * fk
                lay.append(blk)
            ow = offs[NH][0]
            ii = base + ow + np.arange(2 * D)[:, None] * H + np.arange(self.act)[None, :]
            fidx.append(ii.reshape(-1))
            lay.append([fo])
            fo += 2 * D * self.act
            self.foff.append(lay)
        self.fidx = torch.from_numpy(np.concatenate(fidx).astype(np.int64)).to(dev)

    def flop_per_row(self) -> int:
        """FLOPs per row the backward's GEMMs execute (the blocks included, padding and all)."""
        d = self.desc
        D, C, NH, A = d.D, d.C, d.n_hidden, self.act
        fwd_h = sum(2 * (b - a) * fk for (a, b, fk, _) in self.blocks)

        def tr(P):  # one transposed hidden product over the units [0, P)
            return sum(2 * (min(b, P) - a) * (P - k0) for (a, b, _, k0) in self.blocks if a < P)

        dense = 2 * A * (C + D) + (NH - 1) * fwd_h + 2 * 2 * D * A
        chains = sum(2 * 2 * D * P + (NH - 1) * tr(P) + 2 * P * D
                     for P in (self.prefix[p] for p in range(1, D)))
        final = 2 * 2 * D * A + (NH - 1) * tr(A)
        dw = 2 * 2 * D * A + (NH - 1) * fwd_h + 2 * A * (C + D)
        return d.L * (dense + chains + final + dw)

    def _views(self, flat: Tensor, l: int):
        """[(W [r, c], b [r])] of layer l in a flat [L * per] tensor."""
        base = l * self.per
        return [(flat[base + ow:base + ow + r * c].view(r, c), flat[base + ob:base + ob + r])
                for (r, c), (ow, ob) in zip(self.shapes, self.offs)]

    def _buffers(self, B: int) -> dict:
        b = self._bufs.pop(B, None)
        if b is None:
            while len(self._bufs) >= self.keep_sizes:
                self._bufs.pop(next(iter(self._bufs)))
            d = self.desc
            f32 = dict(device=self.dev, dtype=torch.float32)
            b = dict(states=torch.empty((d.L, B, d.D), **f32), lp=torch.empty((B,), **f32),
                     g=torch.empty((B, d.D), **f32), g_next=torch.empty((B, d.D), **f32),
                     h=[torch.zeros((B, d.H), **f32) for _ in range(d.n_hidden)],
                     h2=[torch.zeros((B, d.H), **f32) for _ in range(d.n_hidden)] if _DW_STREAM else None,
                     raw2=torch.empty((B, 2 * d.D), **f32) if _DW_STREAM else None,
                     da=torch.empty((B, d.H), **f32), db=torch.empty((B, d.H), **f32),
                     raw=torch.empty((B, 2 * d.D), **f32), tot=torch.empty((B, 2 * d.D), **f32),
                     chain=torch.empty((B, 2 * d.D), **f32), ones=torch.ones((B,), **f32))
        self._bufs[B] = b  # most recently used last
        return b

    def images(self, flat: Tensor) -> Tuple[Tensor, Tensor, Tensor]:
        """(inverse image, the masked flat weights, the forward block image) on the device."""
        flat = flat.to(self.dev, torch.float32).reshape(-1).contiguous()
        inv = ops.ar_flow_pack_batched(self.desc, flat[None], self.perms, mask=self.mask)[0]
        wflat = flat * self.mask
        return inv, wflat, wflat[self.fidx]

    def forward(self, imgs, x: Tensor, ctx: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
        b = self._buffers(x.shape[0])
        ops.ar_flow_log_prob_train(self.desc, imgs[0], x, ctx, b["states"], out=b["lp"])
        return b["lp"], b["states"]

    @staticmethod
    def _wgrad(gv: Tensor, xv: Tensor, out: Tensor, rowsum: Optional[Tensor]) -> None:
        """out += gvᵀ xv (+ rowsum += Σ_rows gv) in pieces of <= 256 x 256 outputs (the bias column
        rides with the last column piece): the batch-reduction kernel's shape limits (gemm_rows.hip
        wgrad: N1 <= 256, N2 + 1 <= 256), which take strided row views."""
        n1, n2 = gv.shape[1], xv.shape[1]
        if _ONE_DW_GEMM:  # one strided GEMM per block (the generic 64 x 64 tile kernel)
            ops.gemm(gv.t(), xv, out=out, accumulate=True, rowsum=rowsum)
            return
        for r0 in range(0, n1, 256):
            r1 = min(n1, r0 + 256)
            cuts = list(range(0, n2, 255)) + [n2]
            for j, (c0, c1) in enumerate(zip(cuts[:-1], cuts[1:])):
                last = j == len(cuts) - 2
                ops.gemm(gv[:, r0:r1].t(), xv[:, c0:c1], out=out[r0:r1, c0:c1], accumulate=True,
                         rowsum=rowsum[r0:r1] if (last and rowsum is not None) else None)

    def _wg(self, gv: Tensor, xv: Tensor, out: Tensor, rowsum: Optional[Tensor]) -> None:
        """_wgrad on the side stream (after everything the main stream has queued), or inline."""
        if self._side is None:
            self._wgrad(gv, xv, out, rowsum)
            return
        ev = torch.cuda.Event()
        ev.record(self._main)
        self._side.wait_event(ev)
        with torch.cuda.stream(self._side):
            self._wgrad(gv, xv, out, rowsum)
        done = torch.cuda.Event()
        done.record(self._side)
        self._evs.append(done)

    def _after(self, k: int) -> None:
        """The main stream waits for the side stream's first k reductions (in order: the k-th)."""
        if self._side is not None and 0 < k <= len(self._evs):
            self._main.wait_event(self._evs[k - 1])

    def _chain(self, a: Tensor, W, h, P: int, b: dict, dw=None) -> Tensor:
        """The transposed products of one chain, output layer first, over the units [0, P): a = dL/d
        (MADE output) [B, 2D] -> dL/d(first hidden pre-activation) [B, :P].  ``dw``: the layer's dW
        views — each step also reduces dW_i = δ_iᵀ h_{i-1} (+ db_i) on the forward's blocks."""
        NH = self.desc.n_hidden
        blks = [(a0, min(b0, P), fk, k0) for (a0, b0, fk, k0) in self.blocks if a0 < P]
        dl = ops.gemm_dact(a, W[NH][0][:, :P], h[NH - 1][:, :P], "tanh", out=b["da"][:, :P])
        prev = len(self._evs)  # reductions submitted before the previous step's
        for i in range(NH - 1, 0, -1):
            if dw is not None:
                # (reads dl and h[i - 1]; dl's buffer is written again two steps on)
                for (a0, b0, fk, _) in blks:
                    self._wg(dl[:, a0:b0], h[i - 1][:, :fk], dw[i][0][a0:b0, :fk], dw[i][1][a0:b0])
            nxt = b["db"] if dl.data_ptr() == b["da"].data_ptr() else b["da"]
            if dw is not None:  # nxt was the previous step's dl: its reductions must be over
                self._after(prev)
                prev = len(self._evs)
            for (a0, b0, _, k0) in blks:
                ops.gemm_dact(dl[:, k0:P], W[i][0][k0:P, a0:b0], h[i - 1][:, a0:b0], "tanh", out=nxt[:, a0:b0])
            dl = nxt[:, :P]
        return dl

    def backward(self, imgs, states: Tensor, ctx: Optional[Tensor],
                 g_lp: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
        """(dL/dθ in the flat order, dL/dx [B, D]) for L = Σ_rows g_lp · log p (g_lp None: 1)."""
        d = self.desc
        D, C, NH, L = d.D, d.C, d.n_hidden, d.L
        B = states.shape[1]
        b = self._buffers(B)
        wflat, fimg = imgs[1], imgs[2]
        self.ws.zero_()
        if B == 0:
            return self.ws * self.mask, torch.zeros((0, D), device=self.dev)
        g_lp = b["ones"] if g_lp is None else g_lp.to(self.dev).contiguous()  # fp32 (checked by the kernels)
        if _DW_STREAM and self.dev.type == "cuda":
            self._main = torch.cuda.current_stream(self.dev)
            i = self.dev.index if self.dev.index is not None else torch.cuda.current_device()
            if i not in _SIDE:
                _SIDE[i] = torch.cuda.Stream(self.dev)
            if (i, 1) not in _SIDE:
                _SIDE[(i, 1)] = torch.cuda.Stream(self.dev)
            self._side, self._dense, self._evs = _SIDE[i], _SIDE[(i, 1)], []
        else:
            self._main = self._side = None
        g, g_next = b["g"], b["g_next"]
        g.copy_(ops.base_log_prob_bwd(states[0], g_lp))  # d/dz of the Normal(0, I) base log-density
        h, raw, tot, chain = b["h"], b["raw"], b["tot"], b["chain"]
        A = self.act
        cb = None
        if ctx is not None and C > 0:
            cb = ctx.reshape(1, C).expand(B, C) if ctx.dim() == 1 or ctx.shape[0] == 1 else ctx
        def dense(l, h, raw):
            # 1. the dense MADE pass on (ctx, s_l), the units that reach an output only
            W, fo = self._views(wflat, l), self.foff[l]
            ops.linear_act(states[l], W[0][0][:A], W[0][1][:A], "tanh", context=ctx if C > 0 else None, out=h[0][:, :A])
            for i in range(1, NH):
                for (a0, b0, fk, _), o0 in zip(self.blocks, fo[i - 1]):
                    ops.linear_act(h[i - 1][:, :fk], fimg[o0:o0 + (b0 - a0) * fk].view(b0 - a0, fk), W[i][1][a0:b0],
                                   "tanh", out=h[i][:, a0:b0])
            o0 = fo[NH - 1][0]
            ops.linear_act(h[NH - 1][:, :A], fimg[o0:o0 + 2 * D * A].view(2 * D, A), W[NH][1], "identity", out=raw)

        # with the side streams: layer l + 1's dense pass (it reads only s_{l+1} and the weights) runs on
        # a second stream into the other activation set while layer l's chains run
        two = _DENSE_STREAM and self._side is not None and b["h2"] is not None
        sets = [(h, raw), (b["h2"], b["raw2"])] if two else [(h, raw)]
        dense_ev = {}

        def submit_dense(l):
            ev = torch.cuda.Event()
            ev.record(self._main)
            self._dense.wait_event(ev)
            with torch.cuda.stream(self._dense):
                dense(l, *sets[l % 2])
            dense_ev[l] = torch.cuda.Event()
            dense_ev[l].record(self._dense)

        if len(sets) == 2:
            submit_dense(0)
        for l in range(L):
            self._after(len(self._evs))  # the previous layer's reductions read h, tot and da / db
            s = states[l]
            W = self._views(wflat, l)
            G = self._views(self.ws, l)
            h, raw = sets[l % len(sets)]
            if len(sets) == 2:
                self._main.wait_event(dense_ev.pop(l))
                if l + 1 < L:  # (its set's readers: layer l - 1's chains and reductions, all behind us)
                    submit_dense(l + 1)
            else:
                dense(l, h, raw)
            # 2. the inverse's sequential dependence, last order first: dim d_p's outputs reach the
            #    units of degree <= p only
            for p in range(D - 1, 0, -1):
                ops.maf_dim_vjp(raw, s, g, g_lp, int(self.perms[l, p]), g_next, tot, chain=chain,
                                clip_zero=self.clip_zero)
                P = self.prefix[p]
                if P > 0:  # (p >= 1: at least the degree-1 units)
                    dl = self._chain(chain, W, h, P, b)
                    ops.gemm(dl, W[0][0][:P, C:], out=g, accumulate=True)
            ops.maf_dim_vjp(raw, s, g, g_lp, int(self.perms[l, 0]), g_next, tot, chain=None,
                            clip_zero=self.clip_zero)
            # 3. the total δ's and this layer's dW / db
            self._wg(tot, h[NH - 1][:, :A], G[NH][0][:, :A], G[NH][1])
            dl = self._chain(tot, W, h, A, b, dw=G)
            if cb is not None:
                self._wg(dl, cb, G[0][0][:A, :C], None)
            self._wg(dl, s, G[0][0][:A, C:], G[0][1][:A])
            g, g_next = g_next, g
        self._after(len(self._evs))  # the workspace is read on the main stream
        self._main = self._side = None
        return self.ws * self.mask, g

    def __call__(self, flat: Tensor, x: Tensor, ctx: Optional[Tensor]) -> Tuple[Tensor, Tensor]:
        """(Σ_rows log p(x | ctx), ∇θ) of one flat θ."""
        imgs = self.images(flat)
        lp, states = self.forward(imgs, x, ctx)
        grad, _ = self.backward(imgs, states, ctx, None)
        return lp.sum(), grad
