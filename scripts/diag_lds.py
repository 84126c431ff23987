"""diagnostic: poison every CU's LDS with NaN words, then run each fused kernel at full size and
count non-finite outputs (a kernel reading LDS it never wrote in that workgroup shows up here)"""
import ctypes
import torch
from oracle import naz_oracle as O
from tests.test_gpu_parity import _config3_flow

DEV = "cuda"
lib = ctypes.CDLL("scripts/poison/_lds_poison.so")
lib.lds_poison.argtypes = [ctypes.c_uint, ctypes.c_int, ctypes.c_void_p]


def poison():
    s = torch.cuda.current_stream().cuda_stream
    assert lib.lds_poison(0x7FC07FC0, 4096, s) == 0
    torch.cuda.synchronize()


f, spec, state = _config3_flow()
f = f.to(DEV)
B = 1 << 20
g = torch.Generator(device=DEV).manual_seed(0)
x = torch.as_tensor(O.gaussian_mixture(B, 16, seed=0), device=DEV)
c = torch.randn(B, 32, device=DEV, generator=g)
with torch.no_grad():
    for trial in range(3):
        poison()
        lp = f.log_prob(x, condition=c)
        torch.cuda.synchronize()
        bad = torch.nonzero(~torch.isfinite(lp)).reshape(-1)
        print("nsc log_prob trial", trial, "non-finite", bad.numel(), bad[:8].tolist(), flush=True)
    poison()
    lp2 = f.log_prob(x, condition=c)
    clean = f.log_prob(x, condition=c)
    fin = torch.isfinite(lp2)
    print("poisoned vs clean (finite rows) equal:", bool(torch.equal(lp2[fin], clean[fin])), flush=True)
