"""Probe: streaming-read rates torch reaches on the dW operand shapes (2^20 rows), for comparison with
the bf16x6 dW kernels (scripts/wgrad_probe.py)."""
import torch

B = 1 << 20
dev = "cuda"
for (n1, n2) in [(192, 128), (128, 40)]:
    g = torch.randn(B, n1, device=dev)
    x = torch.randn(B, n2, device=dev)
    o = torch.empty_like(g)
    nbytes = (g.numel() + x.numel()) * 4
    for name, fn, by in [("copy g (r+w)", lambda: o.copy_(g), 2 * g.numel() * 4),
                         ("sum rows g,x", lambda: (g.sum(0), x.sum(0)), nbytes),
                         ("g^T 1 (mv)", lambda: (torch.mv(g.t(), x[:, 0]),), g.numel() * 4 + B * 4)]:
        for _ in range(3):
            fn()
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        for _ in range(10):
            fn()
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / 10
        print(f"{n1}x{n2} {name}: {ms:.3f} ms  {by / ms / 1e9:.2f} TB/s", flush=True)
