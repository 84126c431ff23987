"""diagnostic (CPU): why layer 2's lower-spline gradient went non-finite in r06_g1.

Loads the parameters saved by scripts/diag_train_nan.py before the failing step, runs the oracle
flow (fp32) over the failing micro-batch down to layer ``--layer``'s input, and evaluates a numpy
float32 restatement of rqs_vjp_select_inv (spline_bwd.h) on every lower-spline input.  Prints
how many rows give non-finite intermediates, split by inside / outside [-B, B]."""
import argparse
import sys
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parents[1]
sys.path.insert(0, str(ROOT))
import bench  # noqa: E402
from naz_amd.flows import io as fio  # noqa: E402
from naz_amd.trainers.train_flows import _flow_parameters  # noqa: E402
from oracle import naz_oracle as O  # noqa: E402

ap = argparse.ArgumentParser()
ap.add_argument("--state", default="gpurun_out/r06_g1/nan_state_t0.pt")
ap.add_argument("--layer", type=int, default=2)
ap.add_argument("--lo", type=int, default=1 << 22)
ap.add_argument("--rows", type=int, default=1 << 22)
args = ap.parse_args()

f = bench.build_flow()
st = torch.load(args.state, weights_only=True, map_location="cpu")
with torch.no_grad():
    for p, v in zip(_flow_parameters(f), st["params"]):
        p.copy_(v)
state = {k: torch.as_tensor(v).clone() for k, v in fio.export_state(f).items()}
spec = dict(flow_type="nsc", D=bench.D, C=bench.C, hidden=[bench.H, bench.H], L=bench.L, K=bench.K, split=bench.S)
of = O.build_flow(spec, state, torch.float32)
K, S, B = bench.K, bench.S, 3.0
lay = of.layers[args.layer]
uw, uh, ud = [t.numpy().astype(np.float32) for t in lay.lower]
f32 = np.float32
mw = f32(1e-3)  # pyro min bin width / height
md = f32(1e-3)
cA = f32(2 * B) * (f32(1) - mw * f32(K))
ms = f32(2 * B) * mw
nb = f32(-B)
key = np.array([0] + [ms * f32(k) + nb + f32(1e-6) for k in range(1, K)], dtype=f32)


def vjp_select_inv(uw, uh, ud, y):
    """numpy fp32 restatement of rqs_vjp_select_inv's intermediates for one dim (vector y)."""
    ew = np.exp(uw - uw.max()).astype(f32)
    eh = np.exp(uh - uh.max()).astype(f32)
    Ew = np.concatenate([[0], np.cumsum(ew)]).astype(f32)
    Eh = np.concatenate([[0], np.cumsum(eh)]).astype(f32)
    rw, rh = f32(1) / Ew[K], f32(1) / Eh[K]
    Aw, Ah = cA * rw, cA * rh
    idx = np.zeros(y.shape, np.int64)
    for k in range(1, K):
        idx += (y >= Ah * Eh[k] + key[k])
    fi = idx.astype(f32)
    first, last = idx == 0, idx == K - 1
    ch0 = Ah * Eh[idx] + (ms * fi + nb)
    ch1 = np.where(last, f32(B), Ah * Eh[idx + 1] + (ms * (fi + 1) + nb))
    cw0 = Aw * Ew[idx] + (ms * fi + nb)
    cw1 = np.where(last, f32(B), Aw * Ew[idx + 1] + (ms * (fi + 1) + nb))
    sp = lambda u: np.logaddexp(0, u).astype(f32)  # noqa: E731
    udp = np.concatenate([ud, ud[-1:]])
    d0 = np.where(first, f32(1) - md, md + sp(ud[np.maximum(idx - 1, 0)]))
    d1 = np.where(last, f32(1) - md, md + sp(udp[np.minimum(idx, K - 2)]))
    W, H = cw1 - cw0, ch1 - ch0
    delta = H / W
    T1 = (d0 + d1) - f32(2) * delta
    dy = y - ch0
    a = dy * T1 + H * (delta - d0)
    b = H * d0 - dy * T1
    c = -delta * dy
    th = (f32(2) * c) / (-b - np.sqrt(np.maximum(b * b - f32(4) * a * c, 0)))
    om = f32(1) - th
    tt = th * om
    N = delta * th * th + d0 * tt
    Dn = delta + T1 * tt
    G = d1 * th * th + f32(2) * delta * tt + d0 * om * om
    Np = f32(2) * delta * th + d0 * (f32(1) - f32(2) * th)
    Dp = T1 * (f32(1) - f32(2) * th)
    F_th = H * (Np * Dn - N * Dp) / (Dn * Dn)
    return {"th": th, "Dn": Dn, "G": G, "F_th": F_th, "idx": idx}


x = torch.as_tensor(bench.mixture_rows(args.lo, args.lo + args.rows, bench.D, seed=0))
c = torch.as_tensor(bench.normal_rows(args.lo, args.lo + args.rows, bench.C, seed=1))
np.seterr(all="ignore")
tot = {"rows": 0, "tail_vals": 0, "tail_nonfinite": 0, "inside_nonfinite": 0}
worst = []
with torch.no_grad():
    for s0 in range(0, args.rows, 1 << 18):
        y = x[s0:s0 + (1 << 18)]
        cc = c[s0:s0 + (1 << 18)]
        for li in range(len(of.layers) - 1, args.layer, -1):
            y, _ = of.layers[li].inverse(y, cc)
        y1 = y[:, :S].numpy()
        tot["rows"] += y1.shape[0]
        for dim in range(S):
            v = y1[:, dim]
            r = vjp_select_inv(uw[dim], uh[dim], ud[dim], v)
            bad = ~(np.isfinite(r["th"]) & np.isfinite(r["Dn"]) & np.isfinite(r["F_th"]) & np.isfinite(r["G"])
                    & (r["Dn"] != 0) & (r["G"] != 0) & (r["F_th"] != 0))
            inside = (v >= -B) & (v <= B)
            tot["tail_vals"] += int((~inside).sum())
            tot["tail_nonfinite"] += int((bad & ~inside).sum())
            tot["inside_nonfinite"] += int((bad & inside).sum())
            for i in np.nonzero(bad)[0][:4]:
                worst.append({"row": args.lo + s0 + int(i), "dim": dim, "y": float(v[i]), "th": float(r["th"][i]),
                              "Dn": float(r["Dn"][i]), "F_th": float(r["F_th"][i]), "idx": int(r["idx"][i])})
print(tot)
for w in worst[:20]:
    print(w)
