"""diagnostic: the configs[3] NLL step going non-finite (VERDICT r05 Next #1).

Runs bench.py --train's step (the config-3 nsc flow, 2^23 rows, Adam lr 1e-4, clip 1) for
``--steps`` steps per trial, checking the loss and the parameters after every step.  On the
first non-finite step it restores the parameters and Adam state from before that step and
  1. re-runs the step's forward (train path and inference path) per micro-batch, 3 times, and
     reports the non-finite rows and whether repeats agree bit for bit;
  2. re-runs the backward with every launch synchronised and checked (per layer: g_next, the six
     dW operand buffers, the lower-spline gradients; each dW GEMM output), naming the first
     non-finite tensor;
  3. re-runs the whole step plainly 3 times (does the NaN reproduce from the same state?).
Independently of a NaN it checks, once per trial, that the deterministic kernels ARE
deterministic: the training forward's lp and one layer's backward outputs (no atomics in
them) over 5 repeats, bitwise.  Writes gpurun_out/<tag>/diag_train_nan.json (+ a .pt of the
failing state)."""
import argparse
import json
import sys
import time
from pathlib import Path

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import torch  # noqa: E402

import bench  # noqa: E402
from naz_amd import ops  # noqa: E402
from naz_amd.flows import flow as flow_mod  # noqa: E402
from naz_amd.trainers import DataParallel, nll_step  # noqa: E402
from naz_amd.trainers.train_flows import _flow_parameters  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--steps", type=int, default=40)
ap.add_argument("--trials", type=int, default=3)
ap.add_argument("--micro-batch", type=int, default=1 << 22)
ap.add_argument("--batch", type=int, default=1 << 23)
ap.add_argument("--tag", default="diag")
ap.add_argument("--det-repeats", type=int, default=5)
args = ap.parse_args()
out_dir = ROOT / "gpurun_out" / args.tag
out_dir.mkdir(parents=True, exist_ok=True)
dev = torch.device("cuda:0")
torch.cuda.set_device(dev)

G = args.batch
x = torch.as_tensor(bench.mixture_rows(0, G, bench.D, seed=0), device=dev)
c = torch.as_tensor(bench.normal_rows(0, G, bench.C, seed=1), device=dev)
mb = args.micro_batch
report = {"args": vars(args), "trials": []}


def finite(t):
    return bool(torch.isfinite(t).all())


def nonfinite_rows(t):
    bad = ~torch.isfinite(t)
    if bad.dim() > 1:
        bad = bad.reshape(bad.shape[0], -1).any(1)
    idx = torch.nonzero(bad).reshape(-1)
    return int(idx.numel()), idx[:16].tolist()


def snapshot(params, opt):
    st = {k: {kk: (vv.clone() if torch.is_tensor(vv) else vv) for kk, vv in v.items()}
          for k, v in opt.state_dict()["state"].items()}
    return [p.detach().clone() for p in params], st


def restore(params, opt, snap):
    ps, st = snap
    with torch.no_grad():
        for p, s in zip(params, ps):
            p.copy_(s)
    sd = opt.state_dict()
    sd["state"] = {k: {kk: (vv.clone() if torch.is_tensor(vv) else vv) for kk, vv in v.items()} for k, v in st.items()}
    opt.load_state_dict(sd)


def det_check(flow, params):
    """Bitwise repeatability of the kernels without atomics: the training forward's lp and states,
    and layer 3's backward outputs (g_next, h1, h2, dp1, dp2, dp3, x0)."""
    plan = flow._plan
    res = {}
    xb, cb = x[:mb], c[:mb]
    packed, pbwd, flat = plan.packed_bwd()
    d = plan.desc
    lps, sts = [], []
    for _ in range(args.det_repeats):
        states = torch.empty((d.L + 1, mb, d.D), device=dev)
        lp = ops.coupling_log_prob_train(d, packed, xb, cb, None, None, states)
        torch.cuda.synchronize()
        lps.append(lp.clone())
        sts.append(states.clone())
    res["fwd_lp_nonfinite"] = nonfinite_rows(lps[0])[0]
    res["fwd_lp_rows_differing"] = [int((l.view(torch.int32) != lps[0].view(torch.int32)).sum()) for l in lps[1:]]
    res["fwd_states_rows_differing"] = [int((s.view(torch.int32) != sts[0].view(torch.int32)).any(-1).any(0).sum())
                                        for s in sts[1:]]
    D, C, S, K, H, act, lower, bound = plan.shape
    rows = ops.coupling_dp3_columns(d).to(dev)
    states = sts[0]
    g_lp = torch.full((mb,), -1.0 / G, device=dev)
    g0 = ((-states[0]) * g_lp[:, None]).contiguous()
    outs = []
    for _ in range(args.det_repeats):
        bufs = {"h1": torch.empty((mb, H), device=dev), "h2": torch.empty((mb, H), device=dev),
                "dp1": torch.empty((mb, H), device=dev), "dp2": torch.empty((mb, H), device=dev),
                "dp3": torch.empty((mb, rows.numel()), device=dev), "x0": torch.empty((mb, C + S), device=dev)}
        gn = torch.empty_like(g0)
        glow = torch.zeros((S * (3 * K - 1),), device=dev) if lower else None
        ops.coupling_bwd_layer(d, packed, pbwd, flat, 0, states[1], cb, g0, g_lp, bufs, gn, glow)
        torch.cuda.synchronize()
        outs.append(dict(bufs, g_next=gn))
    res["bwd_nonfinite"] = {k: nonfinite_rows(v)[0] for k, v in outs[0].items()}
    res["bwd_rows_differing"] = [{k: int((o[k].view(torch.int32) != outs[0][k].view(torch.int32)).reshape(mb, -1)
                                        .any(1).sum()) for k in o} for o in outs[1:]]
    return res


def instrumented_backward(flow, xb, cb):
    """One micro-batch's forward + backward with every backward launch synchronised and checked."""
    events = []
    orig_bwd, orig_gemm = ops.coupling_bwd_layer, ops.gemm
    first = {}

    def bwd(d, packed, pbwd, flat, layer, state, context, g_in, g_lp, bufs, g_out, g_low):
        torch.cuda.synchronize()
        pre = {"state": nonfinite_rows(state)[0], "g_in": nonfinite_rows(g_in)[0]}
        orig_bwd(d, packed, pbwd, flat, layer, state, context, g_in, g_lp, bufs, g_out, g_low)
        torch.cuda.synchronize()
        post = {k: nonfinite_rows(v) for k, v in bufs.items()}
        post["g_next"] = nonfinite_rows(g_out)
        if g_low is not None:
            post["g_low"] = (0 if finite(g_low) else 1, [])
        e = {"layer": int(layer), "in": pre, "out": {k: v[0] for k, v in post.items()},
             "rows": {k: v[1] for k, v in post.items() if v[0]}}
        events.append(e)
        if not first and (any(pre.values()) or any(v[0] for v in post.values())):
            first.update(e)

    def gemm(a, b, out=None, **kw):
        r = orig_gemm(a, b, out=out, **kw)
        torch.cuda.synchronize()
        o = out if out is not None else r
        ok = finite(o) and (kw.get("rowsum") is None or finite(kw["rowsum"]))
        events.append({"gemm": list(o.shape), "finite": ok, "a_finite": finite(a), "b_finite": finite(b)})
        if not ok and not first:
            first.update(events[-1])
        return r

    ops.coupling_bwd_layer, ops.gemm = bwd, gemm
    try:
        lp = flow.log_prob(xb, condition=cb)
        torch.cuda.synchronize()
        lpn = nonfinite_rows(lp)
        (-lp.sum() / G).backward()
        torch.cuda.synchronize()
    finally:
        ops.coupling_bwd_layer, ops.gemm = orig_bwd, orig_gemm
    return {"lp_nonfinite": lpn, "first_nonfinite": first, "events": events[:64]}


for trial in range(args.trials):
    flow = bench.build_flow()
    params = _flow_parameters(flow)
    dp = DataParallel()
    opt = torch.optim.Adam(params, lr=1e-4)
    tr = {"trial": trial, "losses": []}
    if trial == 0:
        tr["determinism_step0"] = det_check(flow, params)
    t0 = time.time()
    bad_step = None
    for s in range(args.steps):
        snap = snapshot(params, opt)
        loss = nll_step(flow, x, c, opt, params, dp, G, clip_val=1.0, micro_batch=mb)
        lf = float(loss)
        pf = all(finite(p) for p in params)
        gf = all(p.grad is None or finite(p.grad) for p in params)
        tr["losses"].append(lf)
        if not (lf == lf and abs(lf) != float("inf")) or not pf or not gf:
            bad_step = s
            tr["bad"] = {"step": s, "loss": lf, "params_finite": pf, "grads_finite": gf}
            break
    tr["seconds"] = time.time() - t0
    print(json.dumps({"trial": trial, "steps_run": len(tr["losses"]), "bad_step": bad_step,
                      "last_loss": tr["losses"][-1]}), flush=True)
    if bad_step is not None:
        restore(params, opt, snap)
        torch.save({"params": snap[0], "opt": snap[1], "step": bad_step}, out_dir / f"nan_state_t{trial}.pt")
        fw = []
        for rep in range(3):
            per = []
            for s0 in range(0, G, mb):
                xb, cb = x[s0:s0 + mb], c[s0:s0 + mb]
                lp_t = flow.log_prob(xb, condition=cb)  # grad mode: the training forward
                with torch.no_grad():
                    lp_i = flow.log_prob(xb, condition=cb)  # inference kernel
                torch.cuda.synchronize()
                nt, rt = nonfinite_rows(lp_t)
                ni, ri = nonfinite_rows(lp_i)
                per.append({"chunk": s0, "train_nonfinite": nt, "train_rows": [r + s0 for r in rt],
                            "infer_nonfinite": ni, "infer_rows": [r + s0 for r in ri],
                            "lp_t_sum": float(lp_t.detach().double().sum()),
                            "lp_i_sum": float(lp_i.double().sum())})
            fw.append(per)
        tr["forward_repeats"] = fw
        ib = []
        for s0 in range(0, G, mb):
            for p in params:
                p.grad = None
            ib.append(instrumented_backward(flow, x[s0:s0 + mb], c[s0:s0 + mb]))
        tr["instrumented"] = ib
        rr = []
        for rep in range(3):
            restore(params, opt, snap)
            loss = nll_step(flow, x, c, opt, params, dp, G, clip_val=1.0, micro_batch=mb)
            rr.append({"loss": float(loss), "params_finite": all(finite(p) for p in params)})
        tr["replays"] = rr
    report["trials"].append(tr)
    (out_dir / "diag_train_nan.json").write_text(json.dumps(report, indent=1))
print(json.dumps({"done": True, "bad": [t.get("bad") for t in report["trials"]]}), flush=True)
