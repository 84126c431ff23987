"""Diagnostic: the multi-step DP test's per-step reduced gradient and update vs one process."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oracle import naz_oracle as O  # noqa: E402

CFG3 = dict(flow_type="nsc", D=16, C=32, hidden=[128, 128], L=8, K=8, split=8)


def steps_(rank, world, steps=3):
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from naz_amd.trainers import DataParallel, nll_step
    from naz_amd.trainers.train_flows import _flow_parameters
    state = {k: v.numpy() for k, v in O.random_state(CFG3, seed=99).items()}
    f = NormalizingFlow("nsc", None, 16, 32, [128, 128], 8, 8, 8)
    fio.load_state(f, state)
    dp = DataParallel()
    ps = _flow_parameters(f)
    opt = torch.optim.SGD(ps, lr=1e-2)
    G = 3001
    x = torch.as_tensor(O.gaussian_mixture(G * steps, 16, seed=5), device="cuda")
    c = torch.as_tensor(O.context_normal(G * steps, 32, seed=6), device="cuda")
    out = []
    for s in range(steps):
        lo, hi = dp.shard(G)
        rows = slice(s * G + lo, s * G + hi)
        before = torch.cat([p.detach().reshape(-1) for p in ps]).clone()
        nll_step(f, x[rows], c[rows], opt, ps, dp, G, clip_val=1.0)
        g = torch.cat([p.grad.reshape(-1) for p in ps]).cpu().numpy()
        upd = (torch.cat([p.detach().reshape(-1) for p in ps]) - before).cpu().numpy()
        out.append((g, upd))
    return out


def worker(rank, world, port, q):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q.put((rank, steps_(rank, world)))
    dist.destroy_process_group()


if __name__ == "__main__":
    ref = steps_(0, 1)
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        port = s.getsockname()[1]
    ps = [ctx.Process(target=worker, args=(r, 2, port, q)) for r in range(2)]
    [p.start() for p in ps]
    res = dict(q.get(timeout=100) for _ in range(2))
    [p.join() for p in ps]
    r = lambda a, b: np.linalg.norm(a - b) / np.linalg.norm(b)
    for s in range(3):
        print("step", s, "grad", r(res[0][s][0], ref[s][0]), "upd", r(res[0][s][1], ref[s][1]),
              "gnorm dp/ref", np.linalg.norm(res[0][s][0]), np.linalg.norm(ref[s][0]),
              "upd ratio", float(np.dot(res[0][s][1], ref[s][1]) / np.dot(ref[s][1], ref[s][1])))
