"""Benchmark: samples/sec through log_prob + log|det J| of the 16|32 conditional RQ-spline
coupling flow (BASELINE.json metric, configs[2] = "Conditional SBI flow: 16-dim params | 32-dim
context, RQ-spline, batch 2^20, 1 MI355X"; shapes pinned in SURVEY.md §8: K=8, L=8, H=[128,128],
split 8, tanh, bound 3).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--batch B] [--no-cpu-baseline]

One step = one fused log_prob launch over one batch of 2^20 rows per GPU, inputs resident in
HBM.  N > 1 runs under torch.distributed.run, one process per GPU: each rank owns an
independent shard of 2^20 rows (log_prob has no cross-row term: SURVEY.md §8e) — no data-path
collective, "weak" scaling.  The timed region is bracketed by barrier + synchronize on both
sides; the max over ranks is reported.  Rank 0 prints ONE JSON line.
"""
from __future__ import annotations

import argparse
import json
import math
import os
import statistics
import sys
import time
from pathlib import Path

import numpy as np
import torch

ROOT = Path(__file__).resolve().parent
sys.path.insert(0, str(ROOT))

METRIC = "samples/sec through log_prob+log|detJ|, 16-dim RQ-spline flow, batch 2^20"
D, C, S, K, L, H = 16, 32, 8, 8, 8, 128
FP32_PEAK_TFLOPS = 157.3   # MI355X_MICROARCH.md: dense FP32 (matrix == vector)
BF16_PEAK_TFLOPS = 2500.0  # MI355X_MICROARCH.md: dense BF16 MFMA
X6_PRODUCTS = 6            # bf16x6: every fp32 product costs six bf16 MFMA products
HBM_PEAK_GBS = 8000.0


def flops_per_row() -> int:
    """Algorithmic conditioner FLOPs per row: 2·L·(in·H + H·H + H·out)."""
    out = (D - S) * (3 * K - 1)
    return 2 * L * ((C + S) * H + H * H + H * out)


def bytes_per_row() -> int:
    """Algorithmic HBM bytes per row: x (D) + context (C) in, log p out, fp32."""
    return 4 * (D + C) + 4


def gaussian_mixture(n: int, dim: int, seed: int) -> np.ndarray:
    """BASELINE.md synthetic x: 8-component mixture, means ~ N(0, 2^2 I), sigma ~ U(0.3, 1)."""
    rng = np.random.default_rng(seed)
    means = rng.normal(0.0, 2.0, size=(8, dim))
    sig = rng.uniform(0.3, 1.0, size=(8, dim))
    comp = rng.integers(0, 8, size=n)
    return (means[comp] + sig[comp] * rng.standard_normal(size=(n, dim))).astype(np.float32)


def build_flow():
    from naz_amd.flows import NormalizingFlow
    torch.manual_seed(1234)
    f = NormalizingFlow("nsc", None, D, C, [H, H], L, K, S)
    with torch.no_grad():  # last conditioner layer x3 so bins are non-uniform
        for t in f.flow_dist.transforms:
            t.nn.layers[-1].weight.mul_(3.0)
            t.nn.layers[-1].bias.mul_(3.0)
    assert f.fused, "bench: the metric configuration must run the fused kernel"
    return f


def cpu_baseline(flow, x_host: np.ndarray, c_host: np.ndarray, budget_rows: int = 1 << 18):
    """The reference's CPU path (the oracle: pure-torch restatement of pyro's eager per-layer
    semantics, fp32) timed on this host's cores over a bounded sample of the same workload."""
    from naz_amd.flows import io as fio
    from oracle import naz_oracle as O  # baseline + checker only
    spec = dict(flow_type="nsc", D=D, C=C, hidden=[H, H], L=L, K=K, split=S)
    state = fio.export_state(flow)
    of = O.build_flow(spec, state, torch.float32)
    threads = torch.get_num_threads()
    chunk = 1 << 16
    xs = torch.as_tensor(x_host[:budget_rows])
    cs = torch.as_tensor(c_host[:budget_rows])
    with torch.inference_mode():
        of.log_prob(xs[:chunk], cs[:chunk])  # warm-up
        runs = []
        for _ in range(3):
            t0 = time.perf_counter()
            for i in range(0, budget_rows, chunk):
                of.log_prob(xs[i:i + chunk], cs[i:i + chunk])
            runs.append(time.perf_counter() - t0)
    med = statistics.median(runs)
    # parity spot check of the measured GPU path on the first 4096 rows (checker use)
    n = 4096
    of64 = O.build_flow(spec, state, torch.float64)
    with torch.inference_mode():
        ref = of64.log_prob(xs[:n].double(), cs[:n].double()).numpy()
        ref32 = of.log_prob(xs[:n], cs[:n]).numpy()
    with torch.no_grad():
        gpu = flow.log_prob(torch.as_tensor(x_host[:n], device="cuda"),
                            condition=torch.as_tensor(c_host[:n], device="cuda")).cpu().numpy()
    rel = np.abs(gpu - ref) / np.maximum(np.abs(ref), 1.0)
    rel32 = np.abs(ref32 - ref) / np.maximum(np.abs(ref), 1.0)
    return {
        "value": budget_rows / med, "unit": "samples/s", "cores": threads, "kind": "port",
        "sample": f"{budget_rows} rows of the same workload in 2^16-row chunks, torch.inference_mode, "
                  f"{threads} threads, median of 3 after 1 warm-up chunk ({med:.2f} s)",
    }, {"rows": n, "gpu_rel_median": float(np.median(rel)), "gpu_rel_q99": float(np.quantile(rel, 0.99)),
        "gpu_rel_max": float(rel.max()), "ref_fp32_rel_max": float(rel32.max())}


def load_traffic(mode: str):
    """HBM bytes per launch measured with rocprofv3 PMC passes for this kernel variant
    (profiles/traffic_config3_<mode>.json, written by scripts/pmc_summary.py), if present."""
    p = ROOT / "profiles" / f"traffic_config3_{mode}.json"
    if p.exists():
        try:
            d = json.loads(p.read_text())
            return d.get("hbm_bytes_per_launch"), str(p.relative_to(ROOT))
        except Exception:
            pass
    return None, None


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--batch", type=int, default=1 << 20, help="rows per GPU")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--mfma", choices=["auto", "f16x3", "bf16x6", "f32"], default="auto",
                    help="auto (default): f16x3 when the hidden-layer weights fit fp16 (GEMM1 bf16x6, GEMM2/3 as "
                         "three exact-split fp16 products), else bf16x6; f32: exact FP32 MFMA")
    args = ap.parse_args()

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = None
    if world > 1:
        import torch.distributed as dist
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device(f"cuda:{local}"))
    dev = torch.device(f"cuda:{local}")
    torch.cuda.set_device(dev)

    flow = build_flow()
    B = args.batch
    x_host = gaussian_mixture(B, D, seed=0 + rank)
    c_host = np.random.default_rng(1 + 1000 * rank).standard_normal(size=(B, C)).astype(np.float32)
    x = torch.as_tensor(x_host, device=dev)
    c = torch.as_tensor(c_host, device=dev)
    out = torch.empty(B, device=dev)
    plan = flow._plan
    plan.set_mfma(args.mfma)
    packed = plan.packed()
    mode = plan.mode

    from naz_amd import ops

    def step():
        ops.coupling_log_prob(plan.desc, packed, x, c, out=out)

    for _ in range(args.warmup):
        step()
    # per-launch kernel time with HIP events on the launch stream (the current stream)
    stream = torch.cuda.current_stream(dev)
    evs = [(torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)) for _ in range(args.steps)]

    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for i in range(args.steps):
        evs[i][0].record(stream)
        step()
        evs[i][1].record(stream)
    torch.cuda.synchronize(dev)
    if dist is not None:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = time.perf_counter() - t0
    kern_ms = [a.elapsed_time(b) for a, b in evs]
    avg_kern_s = sum(kern_ms) / len(kern_ms) / 1e3

    if dist is not None:
        t = torch.tensor([elapsed, avg_kern_s], device=dev, dtype=torch.float64)
        dist.all_reduce(t, op=dist.ReduceOp.MAX)
        elapsed, avg_kern_s = float(t[0]), float(t[1])

    if rank == 0:
        total_rows = B * world * args.steps
        flop_launch = flops_per_row() * B
        achieved = flop_launch / avg_kern_s / 1e12
        # ceiling for algorithmic FP32 FLOPs on the pipe the kernel actually uses: bf16/fp16 dense
        # MFMA peak divided by the products per fp32 product, weighted by each GEMM's FLOP share
        g1 = 2 * L * (C + S) * H / flops_per_row()  # GEMM1 share (always bf16x6 in the split modes)
        if mode == "f32":
            peak = FP32_PEAK_TFLOPS
        elif mode == "bf16x6":
            peak = BF16_PEAK_TFLOPS / X6_PRODUCTS
        else:
            peak = BF16_PEAK_TFLOPS / (g1 * X6_PRODUCTS + (1 - g1) * 3)
        traffic, traffic_src = load_traffic(mode)
        rec = {
            "metric": METRIC, "value": total_rows / elapsed, "unit": "samples/s", "n_gpus": world,
            "steps": args.steps, "warmup": args.warmup, "ms_per_step": elapsed / args.steps * 1e3,
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "dtype": "f32",
            "data": "synthetic: x ~ 8-component Gaussian mixture (numpy rng(rank)), context ~ N(0, I); "
                    "random-init weights (nn.Linear default, torch seed 1234, last layer x3)",
            "config": {"workload": "BASELINE configs[2]: conditional RQ-spline coupling flow D=16 | C=32, K=8, "
                                   "L=8, H=[128,128], split 8, tanh; fused log_prob (naz_coupling_log_prob)",
                       "batch_per_gpu": B, "global_batch": B * world,
                       "parallelism": f"dp{world} (independent row shards, no collective)"},
            "roofline": {"bound": "mfma", "achieved": achieved, "peak": peak, "unit": "TFLOP/s",
                         "frac": achieved / peak, "traffic": traffic, "traffic_source": traffic_src,
                         "mfma_mode": mode,
                         "peak_note": ("exact FP32 MFMA (v_mfma_f32_32x32x2_f32) peak" if mode == "f32" else
                                       "algorithmic fp32 FLOP/s vs the dense bf16/fp16 MFMA peak (2.5 PF) divided by "
                                       "the MFMA products per fp32 product (bf16x6: 6; f16x3: 3 on GEMM2/3, 6 on "
                                       f"GEMM1); the exact-FP32 MFMA peak is {FP32_PEAK_TFLOPS}"),
                         "kernel": ("coupling_flow_kernel" if mode == "f32" else "coupling_x6_kernel")
                                   + f"<16,32,8,8,128,lower,inv,{mode}>",
                         "flop_per_row": flops_per_row(), "avg_kernel_ms": avg_kern_s * 1e3,
                         "hbm_alg_GBps": bytes_per_row() * B / avg_kern_s / 1e9},
        }
        if world == 1 and not args.no_cpu_baseline:
            base, parity = cpu_baseline(flow, x_host, c_host)
            rec["cpu_baseline"] = base
            rec["parity_spot_check"] = parity
        print(json.dumps(rec), flush=True)
    if dist is not None:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
