"""Diagnose the fused nsa log_prob: kernel time (events) vs whole-call time, and host cProfile."""
import cProfile, pstats, sys, time
from pathlib import Path
import torch
sys.path.insert(0, str(Path(__file__).resolve().parent.parent))
from naz_amd.flows import NormalizingFlow  # noqa: E402
from naz_amd import ops  # noqa: E402

torch.manual_seed(0)
f = NormalizingFlow("nsa", None, 16, 32, [128, 128], 8, 8).to("cuda")
B = 1 << 18
x = torch.randn(B, 16, device="cuda"); c = torch.randn(B, 32, device="cuda")
print("fused", f.fused, flush=True)
with torch.no_grad():
    for _ in range(2):
        f.log_prob(x, condition=c)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(3):
        f.log_prob(x, condition=c)
    torch.cuda.synchronize()
    print("call ms", (time.perf_counter() - t0) / 3 * 1e3, flush=True)
    plan = f._plan
    packed = plan.packed()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    out = torch.empty(B, device="cuda")
    e0.record()
    for _ in range(3):
        ops.ar_flow_log_prob(plan.desc, packed, x, c, out=out)
    e1.record(); torch.cuda.synchronize()
    print("kernel ms", e0.elapsed_time(e1) / 3, flush=True)
    pr = cProfile.Profile(); pr.enable()
    f.log_prob(x, condition=c); torch.cuda.synchronize()
    pr.disable()
    pstats.Stats(pr).sort_stats("cumulative").print_stats(12)
