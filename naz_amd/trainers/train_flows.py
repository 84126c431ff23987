"""naz's MLE trainer (naz/trainers/train_flows.py:20-242), data-parallel over one process per GPU.

Only the NLL step is on the hot path:

    zero_grad -> loss = -log_prob(x_b | y_b).mean() (+ L1)  -> backward
              -> all-reduce grads (RCCL over xGMI, one flat bucket) -> clip_grad_norm_(1.0) -> Adam

``log_prob`` records the autograd walk whose every node is a HIP kernel with a HIP backward
(naz_amd.autograd).  Data parallelism: every rank sees the SAME shuffled global minibatch
order (a generator seeded identically on all ranks) and evaluates its contiguous slice of each
minibatch; the local loss is ``-sum(lp_local) / global_batch`` so a SUM all-reduce yields the
exact gradient of the global mean even when the slices are ragged.  Gradients are reduced
before clipping, so every rank clips and steps identically and the replicas never diverge.
The all-reduce is one flat fp32 bucket (config 4: ~1.5 MB): latency-bound on xGMI, so one
collective per step beats per-tensor buckets.
"""
from __future__ import annotations

import copy
from typing import List, Optional

import torch
import torch.optim as optim
from torch import nn

__all__ = ["DataParallel", "GraphedNllStep", "get_params", "set_params", "nll_step", "train", "train_lightning",
           "predict"]


def _transforms(flow):
    return flow.flow_dist.transforms


def get_params(flow) -> List[dict]:
    """naz/trainers/train_flows.py:20-45: per-transform {name: copy of parameter}."""
    out = []
    for t in _transforms(flow):
        if isinstance(t, nn.Module):
            out.append({n: copy.deepcopy(p) for n, p in t.named_parameters()})
        else:
            out.append({})
    return out


def set_params(flow, params, sample_idx: Optional[int] = None) -> None:
    """naz/trainers/train_flows.py:47-71."""
    from ..nn import invalidate_caches
    invalidate_caches()
    for i, t in enumerate(_transforms(flow)):
        if not isinstance(t, nn.Module):
            continue
        for name, param in t.named_parameters():
            with torch.no_grad():
                src = params[i][name] if sample_idx is None else params[f"flow_{i}_{name}"][sample_idx]
                param.copy_(torch.as_tensor(src))


def _flow_parameters(flow) -> List[torch.Tensor]:
    """train_flows.py:166-168: the union of the transforms' parameters (deduplicated)."""
    seen, out = set(), []
    for t in _transforms(flow):
        if isinstance(t, nn.Module):
            for p in t.parameters():
                if id(p) not in seen:
                    seen.add(id(p))
                    out.append(p)
    return out


def _module_parameters(flow) -> List[torch.Tensor]:
    """train_flows.py:270 (Lightning ``Learner.configure_optimizers``): ``self.model.parameters()``
    — every parameter of the flow module, the embedding net's included — deduplicated, plus any
    transform parameter the module does not register."""
    seen, out = set(), []
    for p in list(flow.parameters()) + _flow_parameters(flow):
        if id(p) not in seen:
            seen.add(id(p))
            out.append(p)
    return out


class DataParallel:
    """Rank layout and the gradient all-reduce.  ``group=None`` with an initialised default
    process group uses it; without torch.distributed this is the single-process identity."""

    def __init__(self, group=None):
        import torch.distributed as dist
        self.dist = dist if dist.is_available() and dist.is_initialized() else None
        self.group = group
        self.world = self.dist.get_world_size(group) if self.dist else 1
        self.rank = self.dist.get_rank(group) if self.dist else 0

    def shard(self, n: int):
        """Contiguous slice [lo, hi) of n rows owned by this rank (ragged when n % world != 0)."""
        base, rem = divmod(n, self.world)
        lo = self.rank * base + min(self.rank, rem)
        return lo, lo + base + (1 if self.rank < rem else 0)

    def all_reduce_grads(self, params: List[torch.Tensor]) -> None:
        if self.dist is None or self.world == 1:
            return
        grads = [p.grad if p.grad is not None else torch.zeros_like(p) for p in params]
        flat = torch.cat([g.reshape(-1) for g in grads])
        self.dist.all_reduce(flat, group=self.group)
        off = 0
        for p, g in zip(params, grads):
            n = g.numel()
            if p.grad is None:
                p.grad = flat[off:off + n].view_as(p).clone()
            else:
                p.grad.copy_(flat[off:off + n].view_as(p))
            off += n

    def all_reduce_sum(self, t: torch.Tensor) -> torch.Tensor:
        if self.dist is not None and self.world > 1:
            self.dist.all_reduce(t, group=self.group)
        return t

    def broadcast_params(self, params: List[torch.Tensor]) -> None:
        """Start every replica from rank 0's weights."""
        if self.dist is None or self.world == 1:
            return
        flat = torch.cat([p.detach().reshape(-1) for p in params])
        self.dist.broadcast(flat, 0, group=self.group)
        off = 0
        with torch.no_grad():
            for p in params:
                p.copy_(flat[off:off + p.numel()].view_as(p))
                off += p.numel()


def nll_step(flow, x_b: torch.Tensor, y_b: Optional[torch.Tensor], optimizer, params: List[torch.Tensor],
             dp: DataParallel, global_batch: int, clip_val: Optional[float] = 1.0,
             lambda_l1: float = 0.0, micro_batch: Optional[int] = None) -> torch.Tensor:
    """One NLL training step on this rank's slice (x_b, y_b) of a global minibatch of
    ``global_batch`` rows (train_flows.py:194-213).  Returns the GLOBAL mean NLL (+ L1) as a
    0-dim tensor on the device (no host sync).

    ``micro_batch``: the slice runs forward + backward in chunks of that many rows whose
    gradients accumulate in ``.grad`` before the single all-reduce — the same gradient as one
    pass over the slice (up to fp32 summation order), with activation memory bounded by the
    chunk (a 2^23-row global batch on one GPU)."""
    optimizer.zero_grad(set_to_none=False)
    n = x_b.shape[0]
    step = max(1, n if not micro_batch or micro_batch >= n else int(micro_batch))
    loss = torch.zeros((), device=x_b.device)
    if lambda_l1 > 0.0:
        reg = 0.0
        for name, p in flow.named_parameters():
            if name.endswith("weight"):
                reg = reg + lambda_l1 * p.abs().sum()
        part = reg / dp.world  # every rank adds its share; the SUM reduce restores one copy
        part.backward()
        loss = loss + part.detach()
    for s in range(0, n, step):
        cond = y_b if y_b is None or y_b.dim() == 1 else y_b[s:s + step]
        part = -flow.log_prob(x_b[s:s + step], condition=cond).sum() / global_batch
        part.backward()
        loss = loss + part.detach()
    dp.all_reduce_grads(params)
    if clip_val is not None:
        nn.utils.clip_grad_norm_(params, clip_val)
    optimizer.step()
    return dp.all_reduce_sum(loss)


class GraphedNllStep:
    """``nll_step`` replayed as ONE captured HIP graph (forward kernels, the composed or fused
    backward, the gradient all-reduce, clip and Adam) for a fixed minibatch shape: naz's ``train``
    runs the same ``batch_frac`` minibatch shape every step (train_flows.py:194-213), and at naz's
    batch sizes (e.g. 10.7 k rows for the 4-parameter MLE MAF, train_mle_all_data_4param.py:95) the
    composed wide-MAF backward is hundreds of small launches per layer.

    The rows are copied into static buffers and the graph replays; the first call for a shape is
    an eager step on a side stream (it creates the gradients, the optimizer state and the paths'
    caches: schedules, packs, buffers) after which one step is captured without running, so every
    call is exactly one optimizer step.  The fused paths check that the rows fit their f16 input
    split (|x|, |ctx| < 2^15) with a host read-back, which a capture cannot do: the check runs
    eagerly before every replay, and an out-of-range minibatch takes the eager step instead.

    Captured: the fused maf paths and the fused nsc step (the weights are re-packed by a device
    kernel inside the graph, in the MFMA mode the eager step resolved).  A flow whose step reads
    device values back on the host (a CNF's adaptive solver, the per-layer walk's checks) cannot be
    captured: the first failed capture is reported once and every later call runs the eager step
    (``self.eager_only``), still exactly one optimizer step per call.

    Limits (fixed at capture time): the optimizer must be capturable — ``torch.optim.Adam(...,
    capturable=True)``, set here when the optimizer has no state yet (an optimizer that already
    stepped keeps its host-side step counters and is refused); the learning rate and the other
    hyper-parameters are baked into the graph (changing ``param_groups[i]['lr']`` later, e.g. naz
    train's ``lr_decay``, needs ``recapture()``); the gradients must not be set to None outside the
    step (``zero_grad(set_to_none=True)`` would free the buffers the graph writes); the naz_tuning
    launch choices and the fused / walk path choice are those of the capture."""

    def __init__(self, flow, optimizer, params: List[torch.Tensor], dp: "DataParallel", global_batch: int,
                 clip_val: Optional[float] = 1.0, micro_batch: Optional[int] = None):
        self.flow, self.opt, self.params, self.dp = flow, optimizer, params, dp
        self.global_batch, self.clip_val, self.micro_batch = global_batch, clip_val, micro_batch
        if any(len(st) for st in optimizer.state.values()):
            raise ValueError("GraphedNllStep: the optimizer has already stepped (its state is not capturable); "
                             "pass a fresh optimizer")
        for g in optimizer.param_groups:
            if "capturable" in g:
                g["capturable"] = True
        self._key, self._graph = None, None
        self._stream = None
        self.replays = 0
        self.eager_steps = 0
        self.eager_only = False
        self.capture_error = None

    def recapture(self) -> None:
        """Drop the graph: the next call captures again (after a hyper-parameter change)."""
        self._key, self._graph = None, None

    def _eager(self, x_b, y_b):
        self.eager_steps += 1
        return nll_step(self.flow, x_b, y_b, self.opt, self.params, self.dp, self.global_batch, self.clip_val,
                        micro_batch=self.micro_batch)

    def _in_range(self, x_b, y_b) -> bool:
        """The rows and the context the fused kernels will see: with an embedding net that is the
        net's output (flow.py NormalizingFlow._pdf conditions on embedding_net(condition)), formed
        here once more, eagerly (a dropout embedding net's draw differs from the graph's)."""
        from .. import ops
        emb = getattr(self.flow, "embedding_net", None)
        ctx = None
        if y_b is not None and emb is not None and not isinstance(emb, nn.Identity):
            with torch.no_grad():
                ctx = emb(y_b)
        return ops.absmax(x_b, y_b, ctx) < 32768.0

    def __call__(self, x_b: torch.Tensor, y_b: Optional[torch.Tensor]) -> torch.Tensor:
        from ..flows import flow as flow_mod
        key = (tuple(x_b.shape), None if y_b is None else tuple(y_b.shape), x_b.device)
        if self.eager_only or not self._in_range(x_b, y_b):
            return self._eager(x_b, y_b)
        if key != self._key:
            dev = x_b.device
            self._x = x_b.detach().clone()
            self._y = None if y_b is None else y_b.detach().clone()
            if self._stream is None:  # one warm-up stream for every (re)capture
                self._stream = torch.cuda.Stream(dev)
            side = self._stream
            side.wait_stream(torch.cuda.current_stream(dev))
            with torch.cuda.stream(side):
                loss = self._eager(self._x, self._y).clone()  # this call's step
            torch.cuda.current_stream(dev).wait_stream(side)
            graph = torch.cuda.CUDAGraph()
            tok = flow_mod._RANGE_CHECKED.set(True)
            try:
                with torch.cuda.graph(graph):  # recorded, not run
                    self._loss = nll_step(self.flow, self._x, self._y, self.opt, self.params, self.dp,
                                          self.global_batch, self.clip_val, micro_batch=self.micro_batch)
            except RuntimeError as e:  # a host read-back inside the step: eager from now on
                import warnings
                self.eager_only, self.capture_error = True, str(e)[:300]
                warnings.warn(f"GraphedNllStep: this flow's step cannot be captured ({self.capture_error}); "
                              "running it eagerly", RuntimeWarning)
                # caches (packed images, plans) touched inside the aborted capture were never filled:
                # a new cache epoch makes every path re-pack eagerly
                from ..nn import invalidate_caches
                invalidate_caches()
                torch.cuda.synchronize(dev)
                return loss
            finally:
                flow_mod._RANGE_CHECKED.reset(tok)
            self._graph, self._key = graph, key
            return loss
        self._x.copy_(x_b)
        if y_b is not None:
            self._y.copy_(y_b)
        self._graph.replay()
        self.replays += 1
        return self._loss


def train(flow, x, y, opt=optim.Adam, lr=0.001, num_epochs=1024, train_frac=0.7, batch_frac=0.005,
          lambda_l1=0., lambda_l2=0., patience=32, min_epochs=128, clip_val=1.0, lr_decay=0.5, min_lr=None,
          return_final=False, seed: int = 0, group=None, verbose: bool = True):
    """naz/trainers/train_flows.py:73-242 with the same arguments and return value
    ``(flow, history, history_val, best_mse, best_epoch)``.  Under torch.distributed (one process
    per GPU, backend "nccl" = RCCL) every rank passes the SAME full x, y and the step runs data
    parallel; the train/test split and the per-epoch shuffles come from ``seed`` (the reference
    used unseeded sklearn/torch shuffles, which cannot agree across ranks)."""
    dp = DataParallel(group)
    params = _flow_parameters(flow)
    dp.broadcast_params(params)
    optimizer = opt(params, lr=lr, weight_decay=lambda_l2)
    scheduler = optim.lr_scheduler.ReduceLROnPlateau(optimizer, mode="min", factor=lr_decay,
                                                     patience=int(patience / 2))
    gen = torch.Generator().manual_seed(seed)
    n = x.shape[0]
    perm = torch.randperm(n, generator=gen)
    n_train = int(round(n * train_frac))
    tr, te = perm[:n_train], perm[n_train:]
    dev = next(iter(params)).device if params else x.device
    x_train, x_test = x[tr.to(x.device)].to(dev), x[te.to(x.device)].to(dev)
    has_y = y is not None
    y_train = y[tr.to(y.device)].to(dev) if has_y else None
    y_test = y[te.to(y.device)].to(dev) if has_y else None
    batch_size = max(1, int(len(x_train) * batch_frac))
    starts = list(range(0, len(x_train), batch_size))
    t_lo, t_hi = dp.shard(len(x_test))
    best_mse, best_weights, best_epoch, n_noimprove = float("inf"), None, 0, 0
    history, history_val = [], []
    min_lr = lr * 1e-3 if min_lr is None else min_lr
    for epoch in range(num_epochs):
        flow.train()
        shuffle = torch.randperm(len(x_train), generator=gen).to(dev)
        total = torch.zeros((), device=dev)
        for s in starts:
            idx = shuffle[s:s + batch_size]
            lo, hi = dp.shard(len(idx))
            mine = idx[lo:hi]
            total = total + nll_step(flow, x_train[mine], y_train[mine] if has_y else None, optimizer, params, dp,
                                     len(idx), clip_val, lambda_l1)
        flow.flow_dist.clear_cache()
        flow.eval()
        with torch.no_grad():
            acc = torch.zeros(2, device=dev, dtype=torch.float64)
            if t_hi > t_lo:
                lp = flow.log_prob(x_test[t_lo:t_hi], condition=y_test[t_lo:t_hi] if has_y else None)
                acc[0] = lp.double().sum()
            acc[1] = t_hi - t_lo
            dp.all_reduce_sum(acc)
            mse = float(-acc[0] / acc[1])
        current_lr = optimizer.param_groups[0]["lr"]
        scheduler.step(mse)
        if verbose and dp.rank == 0:
            print(f"epoch: {epoch}, validation_loss: {mse}, best validation_loss:{best_mse},"
                  f"training_loss: {float(total)}, learning_rate: {float(current_lr)}, min_lr: {min_lr}, "
                  f"no imrovement for {n_noimprove}")
        history.append(float(total) / len(starts))
        history_val.append(mse)
        if mse < best_mse:
            best_epoch, best_mse = epoch, mse
            best_weights = copy.deepcopy(get_params(flow))
            n_noimprove = 0
        elif epoch > min_epochs:
            n_noimprove += 1
        if epoch > min_epochs and n_noimprove > patience and current_lr < min_lr:
            if verbose and dp.rank == 0:
                print(f"network converged after {epoch} eopchs")
            break
    if not return_final and best_weights is not None:
        set_params(flow, best_weights)
    return flow, history, history_val, best_mse, best_epoch


def train_lightning(flow, theta_train, condition_train, opt=optim.AdamW, lr=2e-3, lambda_l2=1e-5, batch_size=10240,
                    num_epochs=600, seed: int = 0, group=None):
    """naz/trainers/train_flows.py:244-278 without PyTorch-Lightning (not a dependency here):
    the same loop its ``Learner`` defines — per epoch a shuffled pass in minibatches of
    ``batch_size`` rows (DataLoader(shuffle=True), last batch partial), loss = -mean log_prob,
    ``opt(params, lr, weight_decay=lambda_l2)``, no clipping (Lightning's default) — as the
    data-parallel NLL step (one process per GPU under torch.distributed).  Returns the flow."""
    dp = DataParallel(group)
    params = _module_parameters(flow)
    dp.broadcast_params(params)
    optimizer = opt(params, lr=lr, weight_decay=lambda_l2)
    gen = torch.Generator().manual_seed(seed)
    dev = next(iter(params)).device if params else theta_train.device
    x = theta_train.to(dev)
    y = condition_train.to(dev) if condition_train is not None else None
    n = x.shape[0]
    flow.train()
    for _ in range(num_epochs):
        order = torch.randperm(n, generator=gen).to(dev)
        for s in range(0, n, batch_size):
            idx = order[s:s + batch_size]
            lo, hi = dp.shard(len(idx))
            mine = idx[lo:hi]
            nll_step(flow, x[mine], y[mine] if y is not None else None, optimizer, params, dp, len(idx),
                     clip_val=None)
    flow.flow_dist.clear_cache()
    return flow


def _draw_params(posterior_samples, l: int, names: List[str], p0: int, p1: int, dev):
    """One flow layer's (W, b) pairs for draws [p0, p1) from naz's posterior dict
    (keys ``flow_{l}_{name}``, a leading draw axis; bflow.py:66-78 / train_flows.py:414)."""
    out = []
    for i in range(len(names) // 2):
        w = torch.as_tensor(posterior_samples[f"flow_{l}_nn.layers.{i}.weight"][p0:p1])
        b = torch.as_tensor(posterior_samples[f"flow_{l}_nn.layers.{i}.bias"][p0:p1])
        out.append((w.to(dev, torch.float32), b.to(dev, torch.float32)))
    return out


def predict(flow, cond, posterior_samples, Nsamples, seed: Optional[int] = None,
            rows_per_launch: int = 1 << 25):
    """naz/trainers/train_flows.py:384-422: ``Nsamples`` draws of theta ~ p(theta | cond) under
    every posterior sample of the flow parameters -> numpy [N_posterior, Nsamples, D].

    The reference loops over posterior samples, ``set_params`` then ``flow.sample(cond,
    [Nsamples])`` (a positional ``cond`` that its conditional ``sample`` asserts against; the
    evident intent ``sample([Nsamples], condition=cond)`` is what runs here).  For naz's affine
    MAF (``maf``, the Bayesian flows of bflow.py) all draws of a chunk run together: one batched
    masked-MADE forward + affine launch per layer over (draws × samples) — the fused
    ``naz_made_affine_fwd`` kernel when the shape fits it, else ``naz_linear_act_batched`` GEMMs
    (``flows.bflow_maf.sampler_batched``).  Other flow types take the reference's per-draw loop
    over the HIP sampling path.  The flow's own parameters are left at the last posterior sample,
    as the reference's loop leaves them."""
    import numpy as np
    key0 = "flow_0_nn.layers.0.weight"
    P = len(posterior_samples[key0])
    if getattr(flow, "flow_type", None) == "maf" and flow.embedding_net.__class__.__name__ == "Identity":
        from ..flows import bflow_maf as BM
        ts = list(flow.flow_dist.transforms)
        arn0 = ts[0].nn
        dev = arn0.layers[0].weight.device
        spec = BM.MAFSpec(arn0.input_dim, arn0.context_dim, arn0.hidden_dims, arn0.act)
        _, _, masks, _, perms = BM.torch_to_jax(flow)
        D = arn0.input_dim
        ctx = None
        if arn0.context_dim:
            ctx = torch.as_tensor(cond, dtype=torch.float32, device=dev).reshape(-1)
        bm = BM.make_normalizing_flow(spec, torch.zeros((1, D), device=dev), masks, [None] * len(ts), perms,
                                      context=ctx)
        names = [n for n, _ in ts[0].named_parameters()]
        out = np.empty((P, int(Nsamples), D), dtype=np.float32)
        gen = torch.Generator(device=dev)
        gen.manual_seed(int(torch.randint(0, 2 ** 62, ()).item()) if seed is None else int(seed))
        per = max(1, rows_per_launch // max(int(Nsamples), 1))
        for p0 in range(0, P, per):
            p1 = min(P, p0 + per)
            params = [_draw_params(posterior_samples, l, names, p0, p1, dev) for l in range(len(ts))]
            y = bm["sampler_batched"](params, gen, int(Nsamples))[0]
            if flow.bounds is not None:
                from ..flows.transforms import inverse_bounding_transform
                b = flow._bounds_dev(y)
                y = inverse_bounding_transform(y, b["low"], b["high"])
            out[p0:p1] = y.cpu().numpy()
        set_params(flow, posterior_samples, sample_idx=P - 1)
        return out
    samples = []
    for i in range(P):
        set_params(flow, posterior_samples, sample_idx=i)
        with torch.no_grad():
            samples.append(flow.sample([int(Nsamples)], condition=cond).cpu().numpy())
    return np.array(samples)
