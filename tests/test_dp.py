"""CPU: the data-parallel NLL step over torch.distributed with
world_size 2 on gloo.  The HIP kernels are not involved here: the flow is a tiny pure-torch
test double exposing naz's flow surface (log_prob(x, condition=), flow_dist.transforms), so
these tests cover the orchestration — sharding, the flat-bucket gradient all-reduce, clipping
after the reduce, identical optimizer steps — against a single-process run."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp
from torch import nn

from naz_amd.trainers import train_flows as T


class _Dist:
    def __init__(self, transforms):
        self.transforms = transforms

    def clear_cache(self):
        pass


class _TinyFlow(nn.Module):
    """Conditional diagonal Gaussian whose mean/log-scale come from an MLP on the condition."""

    def __init__(self, D=3, C=2, seed=0):
        super().__init__()
        torch.manual_seed(seed)
        self.net = nn.Sequential(nn.Linear(C, 16), nn.Tanh(), nn.Linear(16, 2 * D))
        self.D = D
        self.flow_dist = _Dist([self.net])

    def log_prob(self, x, condition=None):
        out = self.net(condition)
        mean, ls = out[:, :self.D], out[:, self.D:].clamp(-5, 3)
        z = (x - mean) * torch.exp(-ls)
        return (-0.5 * z ** 2 - 0.9189385332046727 - ls).sum(-1)


def _data(n=203, D=3, C=2):
    g = torch.Generator().manual_seed(42)
    y = torch.randn(n, C, generator=g)
    x = torch.randn(n, D, generator=g) * 0.5 + y[:, :1]
    return x, y


def _steps(flow, x, y, dp, steps=5, batch=37, micro_batch=None):
    params = T._flow_parameters(flow)
    opt = torch.optim.Adam(params, lr=1e-2)
    losses = []
    for s in range(steps):
        idx = torch.arange(s * batch, (s + 1) * batch) % x.shape[0]
        lo, hi = dp.shard(len(idx))
        mine = idx[lo:hi]
        losses.append(float(T.nll_step(flow, x[mine], y[mine], opt, params, dp, len(idx), 1.0, lambda_l1=1e-3,
                                       micro_batch=micro_batch)))
    return losses, [p.detach().clone() for p in params]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, q, mode):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        torch.manual_seed(100 + rank)  # replicas start different: train() must broadcast rank 0
        x, y = _data()
        if mode.startswith("steps") or mode == "tiny":
            flow = _TinyFlow(seed=0)
            dp = T.DataParallel()
            mb = None if mode in ("steps", "tiny") else int(mode.split(":")[1])
            losses, params = _steps(flow, x, y, dp, micro_batch=mb, batch=2 if mode == "tiny" else 37)
            q.put((rank, losses, [p.numpy() for p in params]))
        else:
            flow = _TinyFlow(seed=rank)
            _, hist, hist_val, best, _ = T.train(flow, x, y, num_epochs=3, batch_frac=0.2, seed=5, verbose=False,
                                                return_final=True)
            q.put((rank, hist_val, [p.detach().numpy().copy() for p in flow.parameters()]))
    finally:
        dist.destroy_process_group()


def _run(world, mode):
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q, mode)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=120) for _ in range(world)]
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    res = [(r, a, [torch.as_tensor(v) for v in ps]) for r, a, ps in res]
    return sorted(res, key=lambda r: r[0])


@pytest.mark.parametrize("micro_batch", [None, 64, 7])
def test_dp_step_matches_single_process(micro_batch):
    """2 ranks on ragged slices of each global minibatch == one process on the whole batch; with
    a micro-batch larger than a rank's 18-19-row slice (64: one chunk, what 8 ranks of bench --train
    run) and smaller (7: chunks accumulated before the one all-reduce)."""
    x, y = _data()
    ref_losses, ref_params = _steps(_TinyFlow(seed=0), x, y, T.DataParallel(), micro_batch=micro_batch)
    res = _run(2, "steps" if micro_batch is None else f"steps:{micro_batch}")
    for _, losses, params in res:
        assert losses == pytest.approx(ref_losses, rel=1e-5, abs=1e-6)
        for a, b in zip(params, ref_params):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for a, b in zip(res[0][2], res[1][2]):
        assert torch.equal(a, b), "replicas diverged"


def test_dp_step_with_an_empty_rank_matches_single_process():
    """3 ranks over 2-row global minibatches: one rank's slice is empty every step (what 8 ranks
    see on a minibatch smaller than 8 rows).  It adds zero gradients to the flat all-reduce (its
    .grad is materialised as zeros, so every rank posts the same bucket) and steps identically."""
    x, y = _data()
    ref_losses, ref_params = _steps(_TinyFlow(seed=0), x, y, T.DataParallel(), batch=2)
    res = _run(3, "tiny")
    for _, losses, params in res:
        assert losses == pytest.approx(ref_losses, rel=1e-5, abs=1e-6)
        for a, b in zip(params, ref_params):
            torch.testing.assert_close(a, b, rtol=1e-5, atol=1e-6)
    for r in res[1:]:
        for a, b in zip(res[0][2], r[2]):
            assert torch.equal(a, b), "replicas diverged"


def test_dp_train_replicas_agree():
    """naz's train() under 2 ranks: rank 0's weights are broadcast, validation loss is the
    all-reduced mean, and both replicas end bitwise identical."""
    res = _run(2, "train")
    (_, hv0, p0), (_, hv1, p1) = res
    assert hv0 == hv1
    for a, b in zip(p0, p1):
        assert torch.equal(a, b)
    # single-process run from rank 0's init with the same seed reaches the same weights
    x, y = _data()
    flow = _TinyFlow(seed=0)
    _, _, hv, _, _ = T.train(flow, x, y, num_epochs=3, batch_frac=0.2, seed=5, verbose=False, return_final=True)
    assert hv == pytest.approx(hv0, rel=1e-5)
    for a, b in zip(flow.parameters(), p0):
        torch.testing.assert_close(a.detach(), b, rtol=1e-5, atol=1e-6)


def test_shard_covers_rows():
    class _DP(T.DataParallel):
        def __init__(self, rank, world):
            self.rank, self.world, self.dist, self.group = rank, world, None, None
    for n in (0, 1, 7, 64, 65):
        for w in (1, 2, 3, 8):
            spans = [_DP(r, w).shard(n) for r in range(w)]
            assert spans[0][0] == 0 and spans[-1][1] == n
            assert all(spans[i][1] == spans[i + 1][0] for i in range(w - 1))
