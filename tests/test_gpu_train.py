"""GPU: the config-3/4 NLL training step end to end — full-size flow
gradient parity, micro-batching, data parallelism over two ranks on one device (gloo), the
``naz`` import-compatible trainers, and posterior-predictive ``predict``."""
import os
import socket

import numpy as np
import pytest
import torch

from oracle import naz_oracle as O
from tests.parity import assert_parity, grad_floor

pytestmark = pytest.mark.gpu
DEV = "cuda"


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    if not torch.cuda.is_available():
        pytest.skip("no HIP device")
    from naz_amd import _lib
    _lib.lib()


def _np(t):
    return t.detach().double().cpu().numpy()


CFG3 = dict(flow_type="nsc", D=16, C=32, hidden=[128, 128], L=8, K=8, split=8)


def _cfg3_flow(state):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    f = NormalizingFlow("nsc", None, 16, 32, [128, 128], 8, 8, 8)
    fio.load_state(f, state)
    return f


def _oracle_grads(spec, state, x, ctx, dt):
    st = {k: (torch.as_tensor(np.asarray(v)) if np.asarray(v).dtype.kind in "iu" else
              torch.as_tensor(np.asarray(v)).to(dt).requires_grad_(True)) for k, v in state.items()}
    of = O.build_flow(spec, st, dt)
    lp = of.log_prob(torch.as_tensor(x).to(dt), torch.as_tensor(ctx).to(dt))
    keys = [k for k in st if st[k].requires_grad]
    return lp.detach(), dict(zip(keys, torch.autograd.grad(-lp.mean(), [st[k] for k in keys])))


def test_config3_full_flow_gradient_vs_oracle():
    """BASELINE configs[2]/[3] flow at full depth (L=8, D=16|C=32, K=8, H=[128,128]) on 4096
    rows: every parameter's NLL gradient against the oracle's float64 autograd."""
    from naz_amd.flows import io as fio
    state = {k: v.numpy() for k, v in O.random_state(CFG3, seed=1234).items()}
    x = O.gaussian_mixture(4096, 16, seed=0)
    c = O.context_normal(4096, 32, seed=1)
    f = _cfg3_flow(state)
    lp = f.log_prob(torch.as_tensor(x, device=DEV), condition=torch.as_tensor(c, device=DEV))
    (-lp.mean()).backward()
    lp64, g64 = _oracle_grads(CFG3, state, x, c, torch.float64)
    lp32, g32 = _oracle_grads(CFG3, state, x, c, torch.float32)
    assert_parity(_np(lp), _np(lp64), _np(lp32), what="config-3 L=8 walk log_prob")
    params = fio.named_state_params(f)
    assert set(params) == set(g64)
    for k, p in params.items():
        g = _np(g64[k])
        assert_parity(_np(p.grad), g, _np(g32[k]), what=f"config-3 L=8 d/d{k}", floor=grad_floor(g),
                      count_factor=None)


def test_nll_step_micro_batch_matches_one_pass():
    """nll_step(micro_batch=m) accumulates the same gradient as one pass over the slice."""
    from naz_amd.trainers import DataParallel, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    state = {k: v.numpy() for k, v in O.random_state(CFG3, seed=7).items()}
    x = torch.as_tensor(O.gaussian_mixture(6000, 16, seed=3), device=DEV)
    c = torch.as_tensor(O.context_normal(6000, 32, seed=4), device=DEV)
    grads = []
    for mb in (None, 2048):
        f = _cfg3_flow(state)
        f.set_fused(False)
        ps = _flow_parameters(f)
        opt = torch.optim.SGD(ps, lr=0.0)
        nll_step(f, x, c, opt, ps, DataParallel(), 6000, clip_val=None, micro_batch=mb)
        grads.append([p.grad.detach().clone() for p in ps])
    for a, b in zip(*grads):
        torch.testing.assert_close(a, b, rtol=2e-5, atol=1e-6 * float(b.abs().max()) + 1e-12)


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _dp_steps(rank, world, steps=2, micro_batch=None, side=None):
    """`steps` nll_steps of the HIP nsc flow (the fused step; the dW side stream on / off with `side`,
    else as configured) on this rank's slice of fixed global batches, in `micro_batch`-row chunks."""
    from naz_amd.flows import flow as flow_mod
    if side is not None:
        flow_mod._DW_STREAM = bool(side)
    from naz_amd.trainers import DataParallel, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    state = {k: v.numpy() for k, v in O.random_state(CFG3, seed=99).items()}
    f = _cfg3_flow(state)
    if rank > 0:  # replicas start different: the DP path must broadcast rank 0's weights
        with torch.no_grad():
            for p in f.parameters():
                p.add_(0.01)
    dp = DataParallel()
    ps = _flow_parameters(f)
    dp.broadcast_params(ps)
    # SGD: the update difference between DP and one process is then lr x the gradient's fp32
    # summation-order difference (Adam's normalised step amplifies it on near-zero gradients);
    # compared norm-wise per tensor (single elements of near-cancelling sums are noise-dominated)
    # lr 1e-4: this randomly initialised flow's NLL is steep (pre-clip gradient norms >> 1), so an
    # fp32-level parameter difference after one step grows ~1e4x in the next step's gradient
    # (measured, scripts/diag_dp2.py: lr 1e-2 gives 7e-4 at step 2, 6e-2 at step 3)
    opt = torch.optim.SGD(ps, lr=1e-4)
    G = 3001  # ragged over 2 ranks
    x = torch.as_tensor(O.gaussian_mixture(G * steps, 16, seed=5), device=DEV)
    c = torch.as_tensor(O.context_normal(G * steps, 32, seed=6), device=DEV)
    losses, grads = [], []
    for s in range(steps):
        lo, hi = dp.shard(G)
        rows = slice(s * G + lo, s * G + hi)
        assert f._plan.train_ready(x[rows], c[rows])  # the fused nsc step, not the walk
        losses.append(float(nll_step(f, x[rows], c[rows], opt, ps, dp, G, clip_val=1.0, micro_batch=micro_batch)))
        grads.append(torch.cat([p.grad.reshape(-1) for p in ps]).cpu().numpy())  # reduced + clipped
    return losses, grads, [p.detach().cpu().numpy() for p in ps]


def _dp_worker(rank, world, port, q, micro_batch=None, side=None):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        q.put((rank,) + _dp_steps(rank, world, micro_batch=micro_batch, side=side))
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("micro_batch,side", [(None, False), (4096, False), (4096, True), (1024, True)])
def test_dp_two_ranks_on_one_gpu_match_single_process(micro_batch, side):
    """Config 4's DP step with the real HIP flow: two gloo ranks sharing cuda:0, each on its
    ragged slice, one flat gradient all-reduce, clip, SGD == one process on the whole batch;
    the replicas stay bitwise identical.  VERDICT r05 Next #7: the fused nsc step, the dW side stream
    off (the default since r06) and on, with a micro-batch larger than a rank's slice (4096 > 1501
    rows: what 8 ranks of bench --train's 2^23 rows in 2^22-row micro-batches run) or smaller (1024:
    chunks)."""
    import torch.multiprocessing as mp
    from naz_amd.flows import flow as flow_mod
    prev = flow_mod._DW_STREAM
    try:
        ref_losses, ref_grads, _ = _dp_steps(0, 1, micro_batch=micro_batch, side=side)
    finally:
        flow_mod._DW_STREAM = prev
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_dp_worker, args=(r, 2, port, q, micro_batch, side)) for r in range(2)]
    for p in procs:
        p.start()
    res = sorted([q.get(timeout=100) for _ in range(2)], key=lambda r: r[0])
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    for _, losses, grads, _ in res:
        np.testing.assert_allclose(losses, ref_losses, rtol=1e-5)
        for s, (a, b) in enumerate(zip(grads, ref_grads)):  # the reduced, clipped gradient of each step
            rel = np.linalg.norm(a - b) / np.linalg.norm(b)
            assert rel <= 1e-4, f"step {s}: DP gradient differs from one process by {rel:.2e} (norm-wise)"
    for a, b in zip(res[0][3], res[1][3]):
        assert np.array_equal(a, b), "replicas diverged"


@pytest.mark.parametrize("micro_batch", [None, 4096])
def test_nll_step_empty_rank_slice(micro_batch):
    """A rank whose slice of the global batch is empty (8 ranks over a batch smaller than 8 rows, or
    the ragged tail of DataParallel.shard): the fused nsc step contributes a zero loss and zero
    gradients to the all-reduce, takes no NaN from 0 / 0, and leaves the weights as SGD on a zero
    gradient does."""
    from naz_amd.trainers import DataParallel, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    state = {k: v.numpy() for k, v in O.random_state(CFG3, seed=99).items()}
    f = _cfg3_flow(state)
    ps = _flow_parameters(f)
    before = [p.detach().clone() for p in ps]
    opt = torch.optim.SGD(ps, lr=1e-2)
    x = torch.as_tensor(O.gaussian_mixture(4, 16, seed=5), device=DEV)[:0]
    c = torch.as_tensor(O.context_normal(4, 32, seed=6), device=DEV)[:0]
    loss = nll_step(f, x, c, opt, ps, DataParallel(), 4, clip_val=1.0, micro_batch=micro_batch)
    assert float(loss) == 0.0
    for p, b in zip(ps, before):
        assert p.grad is None or (torch.isfinite(p.grad).all() and float(p.grad.abs().max()) == 0.0)
        assert torch.equal(p.detach(), b)


def test_naz_compat_front_end_runs_unchanged():
    """The import paths and calls of examples/papers/2506.05657/train_mle_all_data.py:1-20,
    62-89 (at a toy size): construction, train(), sample(), log_prob; train_lightning too."""
    from naz.flows.flow import NormalizingFlow
    from naz.trainers.train_flows import train, train_lightning
    from naz.utils import set_device
    rng = np.random.default_rng(0)
    lam = rng.standard_normal((2000, 2)).astype(np.float32)
    th = (lam[:, :1] + 0.3 * rng.standard_normal((2000, 2))).astype(np.float32)
    flow = NormalizingFlow('maf', None, 2, 2, [32, 32], 3)
    model, history, history_val, best_mse, best_epoch = train(flow, set_device(th), set_device(lam), train_frac=0.89,
                                                              patience=64, lr=1e-3, min_lr=1e-9, num_epochs=2,
                                                              batch_frac=0.05, lr_decay=0.5, verbose=False)
    assert len(history_val) == 2 and np.isfinite(best_mse)
    s = model.sample([500], condition=set_device(lam[0]))
    assert s.shape == (500, 2) and bool(torch.isfinite(s).all())
    lp = model.log_prob(set_device(th[:64]), condition=set_device(lam[:64]))
    assert lp.shape == (64,) and bool(torch.isfinite(lp).all())
    before = [p.detach().clone() for p in model.parameters()]
    train_lightning(model, set_device(th), set_device(lam), num_epochs=1, batch_size=512)
    assert any(not torch.equal(a, p.detach()) for a, p in zip(before, model.parameters()))


def test_train_lightning_updates_embedding_net():
    """The Lightning Learner optimises ``self.model.parameters()`` (train_flows.py:269-270), the
    embedding net included: its weights must move (they were left out)."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.trainers import train_lightning
    torch.manual_seed(0)
    emb = torch.nn.Linear(3, 2).to(DEV)
    flow = NormalizingFlow('maf', None, 2, 2, [32, 32], 2, embedding_net=emb)
    rng = np.random.default_rng(0)
    lam = torch.as_tensor(rng.standard_normal((1024, 3)).astype(np.float32), device=DEV)
    th = torch.as_tensor(rng.standard_normal((1024, 2)).astype(np.float32), device=DEV)
    w0 = emb.weight.detach().clone()
    t0 = [p.detach().clone() for p in flow.flow_dist.transforms[0].parameters()]
    train_lightning(flow, th, lam, num_epochs=1, batch_size=256)
    assert not torch.equal(w0, emb.weight.detach()), "embedding net not optimised"
    assert any(not torch.equal(a, p.detach()) for a, p in zip(t0, flow.flow_dist.transforms[0].parameters()))


def test_predict_batched_matches_oracle_per_draw():
    """predict (train_flows.py:384-422) for a maf: all posterior draws in one batched sampler
    call; draw p's samples equal the oracle flow under draw p's weights applied to the same
    base draws z (regenerated from the seed)."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from naz_amd.trainers import predict
    spec = dict(flow_type="maf", D=2, C=2, hidden=[48, 48], L=4)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=3).items()}
    f = NormalizingFlow("maf", None, 2, 2, [48, 48], 4)
    fio.load_state(f, state)
    P, N = 5, 700
    rng = np.random.default_rng(1)
    post = {}
    for l in range(4):
        for i in range(3):
            for n in ("weight", "bias"):
                v = state[f"layers.{l}.nn.layers.{i}.{n}"]
                post[f"flow_{l}_nn.layers.{i}.{n}"] = (v * (1 + 0.2 * rng.uniform(-1, 1, (P,) + v.shape))).astype(
                    np.float32)
    cond = np.array([0.4, -1.1], dtype=np.float32)
    y = predict(f, torch.as_tensor(cond, device=DEV), post, N, seed=17)
    assert y.shape == (P, N, 2)
    g = torch.Generator(device=DEV).manual_seed(17)
    z = torch.randn((P, N, 2), device=DEV, generator=g).double().cpu()
    for p in range(P):
        st = dict(state)
        for k, v in post.items():
            l, rest = k[5:].split("_", 1)
            st[f"layers.{l}.{rest}"] = v[p]
        of = O.build_flow(spec, st, torch.float64)
        ref = of.sample_from_base(z[p], torch.as_tensor(cond).double().expand(N, 2)).numpy()
        np.testing.assert_allclose(y[p], ref, rtol=1e-4, atol=2e-4, err_msg=f"draw {p}")


@pytest.mark.parametrize("shape", [(16, 32, 8, 8), (8, 0, 4, 6)])
def test_fused_train_path_vs_oracle_and_walk(monkeypatch, shape):
    """The fused NLL step (naz_coupling_log_prob_train + naz_coupling_bwd_layer + dW GEMMs, the
    inference kernel's math) against the oracle's float64 autograd with the gradient criterion
    of tests/parity.py, on a ragged batch; and within 5e-3 (norm-wise) of the per-node walk,
    which uses libm-grade math (two valid fp32 evaluations of the same gradient)."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import flow as flow_mod
    from naz_amd.flows import io as fio
    D, C, S, L = shape
    spec = dict(flow_type="nsc", D=D, C=C, hidden=[128, 128], L=L, K=8, split=S)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=21).items()}
    xh = O.gaussian_mixture(3001, D, seed=2)
    ch = O.context_normal(3001, C, seed=3) if C else None
    x = torch.as_tensor(xh, device=DEV)
    c = torch.as_tensor(ch, device=DEV) if C else None
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setattr(flow_mod, "_TRAIN_FUSED", fused)
        f = NormalizingFlow("nsc", None, D, C, [128, 128], L, 8, S)
        fio.load_state(f, state)
        assert f.fused and f._plan.train_ready(x, c) == (fused == "1")
        lp = f.log_prob(x, condition=c)
        (-lp.mean()).backward()
        res[fused] = (lp.detach(), {k: p.grad.detach().clone() for k, p in fio.named_state_params(f).items()})
    st = {k: (torch.as_tensor(np.asarray(v)) if np.asarray(v).dtype.kind in "iu" else
              torch.as_tensor(np.asarray(v))) for k, v in state.items()}
    g64, g32 = {}, {}
    for dt, out in ((torch.float64, g64), (torch.float32, g32)):
        sd = {k: (v if v.dtype == torch.int64 else v.to(dt).requires_grad_(True)) for k, v in st.items()}
        of = O.build_flow(spec, sd, dt)
        lpo = of.log_prob(torch.as_tensor(xh).to(dt), None if ch is None else torch.as_tensor(ch).to(dt))
        keys = [k for k in sd if sd[k].requires_grad]
        out.update(zip(keys, torch.autograd.grad(-lpo.mean(), [sd[k] for k in keys])))
        out["lp"] = lpo.detach()
    assert_parity(_np(res["1"][0]), _np(g64["lp"]), _np(g32["lp"]), what=f"{shape} fused train log_prob")
    for k, g in res["0"][1].items():
        a = res["1"][1][k]
        ref = _np(g64[k])
        assert_parity(_np(a), ref, _np(g32[k]), what=f"{shape} fused d/d{k}", floor=grad_floor(ref), count_factor=None)
        rel = float((a - g).norm() / g.norm().clamp_min(1e-30))
        assert rel < 5e-3, f"{k}: fused vs walk {rel:.2e}"


@pytest.mark.parametrize("shape", [(16, 32, 8, 8), (8, 0, 4, 6)])
def test_fused_train_dw_side_stream_matches(monkeypatch, shape):
    """NAZ_TRAIN_DW_STREAM: layer l's dW reductions on a side stream while layer l + 1's backward
    runs (two operand sets, event fork / join) give the gradients of the one-stream backward (to the
    dW kernels' atomic-order rounding), on a batch large enough for the kernels to overlap."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import flow as flow_mod
    from naz_amd.flows import io as fio
    D, C, S, L = shape
    spec = dict(flow_type="nsc", D=D, C=C, hidden=[128, 128], L=L, K=8, split=S)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=23).items()}
    x = torch.as_tensor(O.gaussian_mixture(1 << 16, D, seed=4), device=DEV)
    c = torch.as_tensor(O.context_normal(1 << 16, C, seed=5), device=DEV) if C else None
    res = {}
    for side in (False, True):
        monkeypatch.setattr(flow_mod, "_DW_STREAM", side)
        f = NormalizingFlow("nsc", None, D, C, [128, 128], L, 8, S)
        fio.load_state(f, state)
        assert f._plan.train_ready(x, c)
        lp = f.log_prob(x, condition=c)
        (-lp.mean()).backward()
        torch.cuda.synchronize()
        res[side] = {k: p.grad.detach().clone() for k, p in fio.named_state_params(f).items()}
    for k, a in res[False].items():
        b = res[True][k]
        rel = float((a - b).norm() / a.norm().clamp_min(1e-30))
        assert rel < 1e-5, f"{k}: side-stream dW vs one stream {rel:.2e}"


def test_fused_train_full_size_properties():
    """The training forward (coupling_r16_kernel VAR=1, the ring protocol of the metric kernel)
    and the fused backward at BASELINE's 2^20 rows: finite, deterministic and chunk-invariant
    log_prob and saved states; the log_prob agrees with the inference kernel (libm-grade vs
    hardware-transcendental spline math: within 1e-4 of max(|lp|, 1)); every gradient finite."""
    from naz_amd import ops
    from naz_amd.flows import io as fio
    state = {k: v.numpy() for k, v in O.random_state(CFG3, seed=1234).items()}
    f = _cfg3_flow(state)
    B = 1 << 20
    x = torch.as_tensor(O.gaussian_mixture(B, 16, seed=31), device=DEV)
    c = torch.as_tensor(O.context_normal(B, 32, seed=32), device=DEV)
    plan = f._plan
    assert plan.train_ready(x, c)
    packed, _, _ = plan.packed_bwd()
    d = plan.desc

    def fwd(xx, cc):
        st = torch.empty((d.L + 1, xx.shape[0], d.D), device=DEV)
        return ops.coupling_log_prob_train(d, packed, xx, cc, None, None, st), st

    lp, st = fwd(x, c)
    bad = torch.nonzero(~torch.isfinite(lp) | ~torch.isfinite(st).all(dim=2).all(dim=0)).reshape(-1)
    assert bad.numel() == 0, f"non-finite training forward in rows {bad[:8].tolist()} (workgroups {(bad // 128).unique()[:8].tolist()})"
    lp2, st2 = fwd(x, c)
    assert torch.equal(lp, lp2) and torch.equal(st, st2), "training forward not deterministic"
    h = B // 2 + 12345
    la, sa = fwd(x[:h], c[:h])
    lb, sb = fwd(x[h:], c[h:])
    assert torch.equal(torch.cat([la, lb]), lp) and torch.equal(torch.cat([sa, sb], 1), st), "chunking"
    with torch.no_grad():
        lpi = f.log_prob(x, condition=c)
    rel = ((lp - lpi).abs() / lpi.abs().clamp_min(1.0)).max()
    assert float(rel) < 1e-4, f"training forward vs inference kernel: {float(rel):.2e}"
    lpg = f.log_prob(x, condition=c)
    (-lpg.mean()).backward()
    for k, p in fio.named_state_params(f).items():
        assert p.grad is not None and bool(torch.isfinite(p.grad).all()), f"d/d{k} not finite at 2^20 rows"


GOLDEN = os.path.join(os.path.dirname(__file__), "golden")


def _tail_layer_case(B, tail_frac):
    """Layer 2 of a config-3 flow whose lower splines are all the one that broke training in r06
    (tests/golden/nsc_tail_vjp_lower.npz, dim 6), and a state whose rows [0, tail_frac B) put
    every input in the identity tails: the lower dims on consecutive fp32 values around the input
    where the extrapolated map's F_theta is exactly 0 (y = 3.0040803, B = 3) and their negatives,
    the upper dims on a sweep of (B, B + 0.05].  The other rows lie inside the box."""
    from naz_amd.flows import io as fio
    gold = np.load(os.path.join(GOLDEN, "nsc_tail_vjp_lower.npz"))
    state = {k: v.numpy() for k, v in O.random_state(CFG3, seed=1234).items()}
    d6 = int(gold["dim_fail"])
    for l in range(8):
        state[f"layers.{l}.lower_spline.unnormalized_widths"] = np.repeat(gold["uw"][d6:d6 + 1], 8, 0)
        state[f"layers.{l}.lower_spline.unnormalized_heights"] = np.repeat(gold["uh"][d6:d6 + 1], 8, 0)
        state[f"layers.{l}.lower_spline.unnormalized_derivatives"] = np.repeat(gold["ud"][d6:d6 + 1], 8, 0)
    f = _cfg3_flow(state)
    rng = np.random.default_rng(5)
    st = rng.uniform(-2.9, 2.9, size=(B, 16)).astype(np.float32)
    nt = int(B * tail_frac)
    steps = np.arange(nt, dtype=np.int64) - nt // 2
    y0 = np.float32(gold["y_fail"]).view(np.int32).astype(np.int64)
    yl = (y0 + (steps // 2)).astype(np.int32).view(np.float32)  # consecutive fp32 values around y_fail
    yl = np.where(steps % 2 == 0, yl, -yl)
    st[:nt, :8] = yl[:, None] + np.zeros((1, 8), np.float32)
    st[:nt, 8:] = np.float32(3.0) + rng.uniform(1e-6, 0.05, size=(nt, 8)).astype(np.float32)
    assert (np.abs(st[:nt]) > 3.0).all()
    return f, torch.as_tensor(st, device=DEV), nt


def _bwd_layer(f, state, ctx, g_in, layer=2, g_lp_value=-1.0 / (1 << 16)):
    from naz_amd import ops
    plan = f._plan
    assert plan.train_ready(state, ctx)
    packed, pbwd, flat = plan.packed_bwd()
    d = plan.desc
    B = state.shape[0]
    ncol = ops.coupling_dp3_columns(d).numel()
    bufs = {k: torch.empty((B, n), device=DEV) for k, n in
            (("h1", 128), ("h2", 128), ("dp1", 128), ("dp2", 128), ("dp3", ncol), ("x0", 40))}
    g_out = torch.empty_like(g_in)
    g_low = torch.zeros((8 * 23,), device=DEV)
    g_lp = torch.full((B,), g_lp_value, device=DEV)
    ops.coupling_bwd_layer(d, packed, pbwd, flat, layer, state, ctx, g_in, g_lp, bufs, g_out, g_low)
    torch.cuda.synchronize()
    return bufs, g_out, g_low


def test_fused_bwd_tail_inputs_are_the_identity():
    """r06 (VERDICT r05 Next #1): the configs[3] NLL step went non-finite after ~27 Adam steps
    because the spline VJP (rqs_vjp_select_inv) evaluated the bin arithmetic at out-of-box inputs and
    multiplied the results by an inside flag: at y = 3.0040803 (B = 3) the extrapolated F_theta is
    exactly 0, r = inf and 0 * inf = NaN in the lower spline's shared gradient.  With every input of
    a layer in the identity tails its backward IS the identity: g_out == g_in, no parameter
    gradient (g_low and dPre3 exactly 0), everything finite."""
    f, st, nt = _tail_layer_case(1 << 16, 1.0)
    ctx = torch.as_tensor(O.context_normal(st.shape[0], 32, seed=8), device=DEV)
    g_in = torch.randn(st.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    bufs, g_out, g_low = _bwd_layer(f, st, ctx, g_in)
    assert bool(torch.isfinite(g_low).all()), "lower-spline gradient not finite on tail inputs"
    assert int(torch.count_nonzero(g_low)) == 0, "tail inputs gave the lower spline a gradient"
    assert int(torch.count_nonzero(bufs["dp3"])) == 0, "tail inputs gave the conditioner a gradient"
    for k, v in bufs.items():
        assert bool(torch.isfinite(v).all()), f"{k} not finite"
    assert torch.equal(g_out, g_in), "the identity tails' VJP must pass g through"


def test_fused_bwd_tail_rows_add_nothing():
    """Half the rows in the tails (around the r06 singular input), half inside: the layer's
    lower-spline gradient equals that of the inside rows alone (to the atomic adds' rounding), and
    the tail rows' g_out is their g_in."""
    f, st, nt = _tail_layer_case(1 << 16, 0.5)
    ctx = torch.as_tensor(O.context_normal(st.shape[0], 32, seed=8), device=DEV)
    g_in = torch.randn(st.shape, device=DEV, generator=torch.Generator(device=DEV).manual_seed(3))
    bufs, g_out, g_low = _bwd_layer(f, st, ctx, g_in)
    _, g_out_i, g_low_i = _bwd_layer(f, st[nt:].contiguous(), ctx[nt:].contiguous(), g_in[nt:].contiguous())
    assert bool(torch.isfinite(g_low).all()) and bool(torch.isfinite(g_out).all())
    assert torch.equal(g_out[:nt], g_in[:nt]) and torch.equal(g_out[nt:], g_out_i)
    rel = float((g_low - g_low_i).norm() / g_low_i.norm())
    assert rel < 1e-5, f"tail rows changed the lower-spline gradient: {rel:.2e}"
    assert int(torch.count_nonzero(bufs["dp3"][:nt])) == 0


def _bench_train_losses(steps, rows, micro_batch, side):
    """bench.py --train's step (its flow, rows, Adam lr 1e-4, clip 1) for `steps` steps: the
    losses and whether every parameter is finite after each step."""
    import bench
    from naz_amd.flows import flow as flow_mod
    from naz_amd.trainers import DataParallel, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    old = flow_mod._DW_STREAM
    flow_mod._DW_STREAM = side
    try:
        f = bench.build_flow()
        x = torch.as_tensor(bench.mixture_rows(0, rows, 16, seed=0), device=DEV)
        c = torch.as_tensor(bench.normal_rows(0, rows, 32, seed=1), device=DEV)
        ps = _flow_parameters(f)
        assert f._plan.train_ready(x, c)
        opt = torch.optim.Adam(ps, lr=1e-4)
        losses, pfin = [], []
        for _ in range(steps):
            losses.append(nll_step(f, x, c, opt, ps, DataParallel(), rows, clip_val=1.0, micro_batch=micro_batch))
            pfin.append(torch.stack([torch.isfinite(p).all() for p in ps]).all())
        return torch.stack(losses).cpu().numpy(), torch.stack(pfin).cpu().numpy()
    finally:
        flow_mod._DW_STREAM = old


def test_fused_nsc_training_30_steps_finite_2e20():
    """VERDICT r05 Next #1: 30 fused nsc optimizer steps (Adam lr 1e-4, clip 1) of bench.py
    --train's flow at 2^20 rows: every loss and every parameter finite, with the dW side stream on
    and off; the first loss identical (same weights, deterministic forward) and the trajectories
    within 2e-3 of each other (the dW atomics' rounding, amplified by Adam's normalised step on
    near-zero gradients: ~3e-4 after 27 steps between runs, r06_g1)."""
    la, pa = _bench_train_losses(30, 1 << 20, None, True)
    lb, pb = _bench_train_losses(30, 1 << 20, None, False)
    assert np.isfinite(la).all() and pa.all(), f"side stream: first non-finite step {np.argmin(np.isfinite(la) & pa)}"
    assert np.isfinite(lb).all() and pb.all(), f"one stream: first non-finite step {np.argmin(np.isfinite(lb) & pb)}"
    assert la[0] == lb[0]
    assert (np.abs(la - lb) / np.abs(lb)).max() < 2e-3
    assert la[-1] < la[0] - 1.0, "the NLL did not decrease"


def test_fused_nsc_training_40_steps_finite_default_micro_batch():
    """The bench default: 2^23 rows in 2^22-row micro-batches, 40 steps (the r06_g1 failure was at
    step 27 of this configuration), every loss and parameter finite."""
    la, pa = _bench_train_losses(40, 1 << 23, 1 << 22, False)  # the shipped configuration (one stream)
    assert np.isfinite(la).all() and pa.all(), f"first non-finite step {np.argmin(np.isfinite(la) & pa)}"


def _maf_train_vs_oracle_and_walk(monkeypatch, D, C, hidden, L, B, ctx_rows, what):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import flow as flow_mod
    from naz_amd.flows import io as fio
    spec = dict(flow_type="maf", D=D, C=C, hidden=list(hidden), L=L)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=23).items()}
    xh = O.gaussian_mixture(B, D, seed=4)
    ch = O.context_normal(B if ctx_rows else 1, C, seed=5)
    x = torch.as_tensor(xh, device=DEV)
    c = torch.as_tensor(ch if ctx_rows else ch[0], device=DEV)
    res = {}
    for fused in ("1", "0"):
        monkeypatch.setattr(flow_mod, "_TRAIN_FUSED", fused)
        f = NormalizingFlow("maf", None, D, C, list(hidden), L)
        fio.load_state(f, state)
        assert f.fused and f._plan.train_ready(x, c) == (fused == "1")
        lp = f.log_prob(x, condition=c)
        (-lp.mean()).backward()
        res[fused] = (lp.detach(), {k: p.grad.detach().clone() for k, p in fio.named_state_params(f).items()})
    st = {k: torch.as_tensor(np.asarray(v)) for k, v in state.items()}
    g64, g32 = {}, {}
    cb = np.broadcast_to(ch, (B, C)) if not ctx_rows else ch
    for dt, out in ((torch.float64, g64), (torch.float32, g32)):
        sd = {k: (v if v.dtype == torch.int64 else v.to(dt).requires_grad_(True)) for k, v in st.items()}
        of = O.build_flow(spec, sd, dt)
        lpo = of.log_prob(torch.as_tensor(xh).to(dt), torch.as_tensor(np.ascontiguousarray(cb)).to(dt))
        keys = [k for k in sd if sd[k].requires_grad]
        out.update(zip(keys, torch.autograd.grad(-lpo.mean(), [sd[k] for k in keys])))
        out["lp"] = lpo.detach()
    assert_parity(_np(res["1"][0]), _np(g64["lp"]), _np(g32["lp"]), what=f"{what} train log_prob")
    for k, g in res["0"][1].items():
        a = res["1"][1][k]
        ref = _np(g64[k])
        assert_parity(_np(a), ref, _np(g32[k]), what=f"{what} d/d{k}", floor=grad_floor(ref), count_factor=None)
        rel = float((a - g).norm() / g.norm().clamp_min(1e-30))
        assert rel < 5e-3, f"{k}: {what} vs walk {rel:.2e}"


@pytest.mark.parametrize("ctx_rows,B", [(True, 3001), (False, 777)])
def test_fused_maf_train_path_vs_oracle_and_walk(monkeypatch, ctx_rows, B):
    """The maf NLL step on the fused maf backward (flows/maf_grad.py: saved-state inverse kernel,
    made_ar_bwd_kernel per layer, batched bf16x6 dW) at the paper shape (D=2 | C=2, H=[150]x3)
    against the oracle's float64 autograd (tests/parity.py gradient criterion) and the per-node
    walk; ragged batches, per-row and broadcast contexts."""
    _maf_train_vs_oracle_and_walk(monkeypatch, 2, 2, [150] * 3, 4, B, ctx_rows, "fused maf")


@pytest.mark.parametrize("ctx_rows,B", [(True, 1027), (False, 300), (True, 2311)])
def test_wide_maf_train_path_vs_oracle_and_walk(monkeypatch, ctx_rows, B):
    """The MLE maf's NLL step (train_mle_all_data_4param.py:87-92: D=4 | C=2, H=[512]x5) on the
    saved-state wide inverse kernel + the GEMM-composed backward (flows/maf_grad_wide.py: one dense
    MADE pass, D - 1 input chains and one dW chain per layer) against the oracle's float64 autograd
    and the per-node walk, at L=3; ragged batches, per-row and broadcast contexts.  B = 2311 puts the
    dW reductions (K = B >= 2048) on gemm_tn128_kernel."""
    _maf_train_vs_oracle_and_walk(monkeypatch, 4, 2, [512] * 5, 3, B, ctx_rows, "wide maf")


@pytest.mark.parametrize("ctx_rows,B", [(True, 1500), (False, 333)])
def test_config3_ar_maf_train_path_vs_oracle_and_walk(monkeypatch, ctx_rows, B):
    """SURVEY §8d's config-3 AR variant as a maf (D=16 | C=32, H=[128,128]): its inverse is fused but
    made_ar_bwd is not compiled for it, so its NLL step takes the GEMM-composed backward
    (flows/maf_grad_wide.py: 15 input chains per layer, a 32-wide context in the dW of W_0) -- checked
    here against the oracle's float64 autograd and the per-node walk."""
    _maf_train_vs_oracle_and_walk(monkeypatch, 16, 32, [128, 128], 3, B, ctx_rows, "composed maf D16C32")


def test_wide_maf_dw_side_stream_matches():
    """NAZ_MAF_WIDE_DW_STREAM: the composed wide-maf backward's dW reductions on a side stream beside
    the chain's next transposed product (event-ordered reuse of the two delta buffers and of the layer's
    activations) give the one-stream gradients, to the reductions' atomic-order rounding."""
    from naz_amd.flows import maf_grad_wide as mgw
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    spec = dict(flow_type="maf", D=4, C=2, hidden=[512] * 5, L=3)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=33).items()}
    B = 10752
    x = torch.as_tensor(O.gaussian_mixture(B, 4, seed=6), device=DEV)
    c = torch.as_tensor(O.context_normal(B, 2, seed=7), device=DEV)
    res = {}
    prev = mgw._DW_STREAM
    try:
        for side in (False, True):
            mgw._DW_STREAM = side
            f = NormalizingFlow("maf", None, 4, 2, [512] * 5, 3)
            fio.load_state(f, state)
            f = f.to(DEV)
            lp = f.log_prob(x, condition=c)
            (-lp.mean()).backward()
            torch.cuda.synchronize()
            res[side] = {k: p.grad.detach().clone() for k, p in fio.named_state_params(f).items()}
    finally:
        mgw._DW_STREAM = prev
    for k, a in res[False].items():
        b = res[True][k]
        rel = float((a - b).norm() / a.norm().clamp_min(1e-30))
        assert rel < 1e-5, f"{k}: side-stream dW vs one stream {rel:.2e}"


def test_graphed_nll_step_matches_eager_steps():
    """trainers.GraphedNllStep (the whole NLL step -- wide maf forward kernel, the GEMM-composed
    backward, clip, capturable Adam -- replayed as one captured HIP graph) takes the same steps as
    eager nll_step calls: same losses and parameters after 4 steps (to the split-K reductions'
    atomic ordering), new minibatch rows through the static buffers, and an out-of-range
    minibatch runs eagerly."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from naz_amd.trainers import DataParallel, GraphedNllStep, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    spec = dict(flow_type="maf", D=4, C=2, hidden=[512] * 5, L=2)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=31).items()}
    B = 2048
    xs = [torch.as_tensor(O.gaussian_mixture(B, 4, seed=40 + i), device=DEV) for i in range(4)]
    cs = [torch.as_tensor(O.context_normal(B, 2, seed=50 + i), device=DEV) for i in range(4)]
    runs = {}
    for graphed in (False, True):
        f = NormalizingFlow("maf", None, 4, 2, [512] * 5, 2)
        fio.load_state(f, state)
        f = f.to(DEV)
        params = _flow_parameters(f)
        dp = DataParallel()
        opt = torch.optim.Adam(params, lr=1e-3, capturable=graphed)
        g = GraphedNllStep(f, opt, params, dp, B) if graphed else None
        losses = []
        for x, c in zip(xs, cs):
            loss = g(x, c) if graphed else nll_step(f, x, c, opt, params, dp, B)
            losses.append(float(loss))
        runs[graphed] = (losses, [p.detach().clone() for p in params])
        if graphed:
            assert g.replays == 3 and g.eager_steps == 1
            big = xs[0].clone()
            big[0, 0] = 1e6  # outside the fused kernel's f16 input split: the eager walk
            assert torch.isfinite(g(big, cs[0]))
            assert g.eager_steps == 2 and g.replays == 3
    le, pe = runs[False]
    lg, pg = runs[True]
    assert np.allclose(le, lg, rtol=1e-5, atol=1e-5), (le, lg)
    for a, b in zip(pe, pg):
        rel = float((a - b).norm() / a.norm().clamp_min(1e-30))
        assert rel < 1e-5, rel


def test_graphed_nll_step_nsc_matches_eager_steps():
    """GraphedNllStep on the fused nsc step (config-3 shape, L = 2): the weights are
    re-packed by the device packer inside the graph (the eager step's MFMA mode, no host read-back
    while capturing), and 4 calls = 1 eager step + 3 replays give the losses and parameters of 4
    eager nll_step calls (to the dW atomics' rounding, amplified by Adam)."""
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from naz_amd.trainers import DataParallel, GraphedNllStep, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    spec = dict(CFG3, L=2)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=33).items()}
    B = 4096
    xs = [torch.as_tensor(O.gaussian_mixture(B, 16, seed=60 + i), device=DEV) for i in range(4)]
    cs = [torch.as_tensor(O.context_normal(B, 32, seed=70 + i), device=DEV) for i in range(4)]
    runs = {}
    for graphed in (False, True):
        f = NormalizingFlow("nsc", None, 16, 32, [128, 128], 2, 8, 8)
        fio.load_state(f, state)
        params = _flow_parameters(f)
        dp = DataParallel()
        opt = torch.optim.Adam(params, lr=1e-4, capturable=graphed)
        g = GraphedNllStep(f, opt, params, dp, B) if graphed else None
        assert f._plan.train_ready(xs[0], cs[0])
        losses = [float(g(x, c) if graphed else nll_step(f, x, c, opt, params, dp, B)) for x, c in zip(xs, cs)]
        runs[graphed] = (losses, [p.detach().clone() for p in params])
        if graphed:
            assert not g.eager_only, g.capture_error
            assert g.replays == 3 and g.eager_steps == 1
            with torch.no_grad():  # the inference kernel reads the image the graph's packer rewrote
                lp = f.log_prob(xs[0], condition=cs[0])
            assert bool(torch.isfinite(lp).all())
    le, pe = runs[False]
    lg, pg = runs[True]
    assert np.allclose(le, lg, rtol=1e-5, atol=1e-5), (le, lg)
    for a, b in zip(pe, pg):
        rel = float((a - b).norm() / a.norm().clamp_min(1e-30))
        assert rel < 1e-4, rel


@pytest.mark.parametrize("scale", [1.0, 1e5])
def test_graphed_nll_step_range_checks_the_embedded_context(scale):
    """with an embedding net the fused step's f16 range applies to the net's output,
    not to the raw condition.  A net that maps in-range conditions past 2^15 must send every call to
    the eager step (no replay of a graph captured without the check); an in-range net captures."""
    from torch import nn
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from naz_amd.trainers import DataParallel, GraphedNllStep
    from naz_amd.trainers.train_flows import _flow_parameters
    spec = dict(CFG3, L=2)
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=33).items()}
    B = 1024
    emb = nn.Linear(32, 32)
    with torch.no_grad():
        emb.weight.copy_(torch.eye(32) * scale)
        emb.bias.zero_()
    f = NormalizingFlow("nsc", None, 16, 32, [128, 128], 2, 8, 8, embedding_net=emb)
    fio.load_state(f, state)
    f.to(DEV)
    params = _flow_parameters(f)
    opt = torch.optim.Adam(params, lr=1e-4, capturable=True)
    g = GraphedNllStep(f, opt, params, DataParallel(), B)
    xs = [torch.as_tensor(O.gaussian_mixture(B, 16, seed=80 + i), device=DEV) for i in range(3)]
    cs = [torch.as_tensor(O.context_normal(B, 32, seed=90 + i), device=DEV) for i in range(3)]
    losses = [float(g(x, c)) for x, c in zip(xs, cs)]
    assert all(np.isfinite(losses)), losses
    if scale > 1.0:
        assert g.replays == 0 and g.eager_steps == 3
    else:
        assert not g.eager_only, g.capture_error
        assert g.eager_steps == 1 and g.replays == 2


@pytest.mark.parametrize("solver", ["rk4", "dopri5"])
def test_graphed_nll_step_cnf_captures_or_runs_eagerly(solver):
    """GraphedNllStep on a CNF.  The RK4 step (fused solve, discrete adjoint) captures
    and replays; the dopri5 step (torchdyn's batch-global controller polls its `done` flag on the
    host) cannot be captured, so the first failed capture is reported once and every call runs
    eagerly — one optimizer step per call either way, the losses of plain nll_step calls, and no
    stale packed image after the aborted capture."""
    import warnings
    from naz_amd.flows import NormalizingFlow
    from naz_amd.trainers import DataParallel, GraphedNllStep, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    B = 1024
    xs = [torch.as_tensor(O.gaussian_mixture(B, 4, seed=80 + i), device=DEV) * 0.5 for i in range(3)]
    runs = {}
    for graphed in (False, True):
        torch.manual_seed(5)
        f = NormalizingFlow("cnf", None, 4, 0, [32, 32], 1, steps=2, solver=solver)
        params = _flow_parameters(f)
        dp = DataParallel()
        opt = torch.optim.Adam(params, lr=1e-3, capturable=graphed)
        g = GraphedNllStep(f, opt, params, dp, B) if graphed else None
        with warnings.catch_warnings():
            warnings.simplefilter("ignore", RuntimeWarning)
            losses = [float(g(x, None) if graphed else nll_step(f, x, None, opt, params, dp, B)) for x in xs]
        runs[graphed] = losses
        if graphed:
            if solver == "rk4":
                assert not g.eager_only and g.replays == 2 and g.eager_steps == 1, g.capture_error
            else:
                assert g.eager_only and g.replays == 0 and g.eager_steps == 3
    assert np.allclose(runs[False], runs[True], rtol=1e-4, atol=1e-5), runs
