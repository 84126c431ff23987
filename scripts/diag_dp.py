"""Diagnostic: one DP NLL step over 2 gloo ranks on cuda:0 vs one process (reduced gradients)."""
import os
import socket
import sys
from pathlib import Path

import numpy as np
import torch
import torch.multiprocessing as mp

sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from oracle import naz_oracle as O  # noqa: E402

spec = dict(flow_type="nsc", D=16, C=32, hidden=[128, 128], L=2, K=8, split=8)
G = 3001


def grads(rank, world, mode):
    import torch.distributed as dist
    from naz_amd.flows import NormalizingFlow
    from naz_amd.flows import io as fio
    from naz_amd.trainers import DataParallel
    from naz_amd.trainers.train_flows import _flow_parameters
    state = {k: v.numpy() for k, v in O.random_state(spec, seed=99).items()}
    f = NormalizingFlow("nsc", None, 16, 32, [128, 128], 2, 8, 8)
    fio.load_state(f, state)
    dp = DataParallel()
    ps = _flow_parameters(f)
    if mode == "bcast":
        if rank > 0:
            with torch.no_grad():
                for p in f.parameters():
                    p.add_(0.01)
        dp.broadcast_params(ps)
    x = O.gaussian_mixture(G, 16, seed=5)
    c = O.context_normal(G, 32, seed=6)
    lo, hi = dp.shard(G)
    lp = f.log_prob(torch.as_tensor(x[lo:hi], device="cuda"), condition=torch.as_tensor(c[lo:hi], device="cuda"))
    (-lp.sum() / G).backward()
    if world > 1:
        if mode == "cpu":
            flat = torch.cat([p.grad.reshape(-1) for p in ps]).cpu()
            dist.all_reduce(flat)
            out = flat.numpy()
        elif mode == "sync":
            flat = torch.cat([p.grad.reshape(-1) for p in ps])
            torch.cuda.synchronize()
            dist.all_reduce(flat)
            torch.cuda.synchronize()
            out = flat.cpu().numpy()
        else:
            dp.all_reduce_grads(ps)
            out = torch.cat([p.grad.reshape(-1) for p in ps]).cpu().numpy()
    else:
        out = torch.cat([p.grad.reshape(-1) for p in ps]).cpu().numpy()
    return out


def worker(rank, world, port, q, mode):
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    q.put((rank, grads(rank, world, mode)))
    dist.destroy_process_group()


if __name__ == "__main__":
    ref = grads(0, 1, None)
    for mode in ("bcast",):
        ctx = mp.get_context("spawn")
        q = ctx.Queue()
        with socket.socket() as s:
            s.bind(("127.0.0.1", 0))
            port = s.getsockname()[1]
        ps = [ctx.Process(target=worker, args=(r, 2, port, q, mode)) for r in range(2)]
        [p.start() for p in ps]
        res = dict(q.get(timeout=100) for _ in range(2))
        [p.join() for p in ps]
        for r in (0, 1):
            print(mode, r, "rel norm diff", np.linalg.norm(res[r] - ref) / np.linalg.norm(ref),
                  "ratio", float(np.dot(res[r], ref) / np.dot(ref, ref)))
