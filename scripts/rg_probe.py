import sys, torch
sys.path.insert(0, '.')
from naz_amd import ops
from scripts.gemm_bench import timeit
dev = torch.device('cuda')
M = 1 << 18
for K, N, act, masked in [(4, 150, 'tanh', True), (150, 150, 'tanh', True), (150, 150, 'tanh', False), (150, 150, 'identity', False), (160, 160, 'tanh', False), (128, 128, 'tanh', False)]:
    X = torch.randn(M, K, device=dev)
    W = torch.randn(N, K, device=dev) / K ** 0.5
    b = torch.randn(N, device=dev)
    m = (torch.rand(N, K, device=dev) > 0.5).float() if masked else None
    t = timeit(lambda: ops.linear_act(X, W, b, act, mask=m))
    print(f"K={K} N={N} {act} mask={masked}: {t:.1f} us  {2*M*N*K/t/1e6:.1f} TF  {(M*(K+N))*4/t/1e3:.0f} GB/s")
