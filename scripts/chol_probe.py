"""How fast is a library batched dense Cholesky (torch.linalg -> rocSOLVER) at the ring windows' reduced-system size
(16 windows of n = 288..384)? A probe for DESIGN §6's factorization choice, not part of the product path."""
import time

import torch

dev = torch.device("cuda", 0)
for n in (288, 336, 384):
    g = torch.Generator(device="cpu").manual_seed(n)
    a = torch.randn(16, n, n, dtype=torch.float64, generator=g)
    s = (a @ a.transpose(1, 2) + n * torch.eye(n, dtype=torch.float64)).to(dev)
    b = torch.randn(16, n, 1, dtype=torch.float64, generator=g).to(dev)
    for _ in range(3):
        L, info = torch.linalg.cholesky_ex(s)
        x = torch.cholesky_solve(b, L)
    torch.cuda.synchronize()
    ts = []
    for _ in range(10):
        t0 = time.perf_counter()
        L, info = torch.linalg.cholesky_ex(s)
        x = torch.cholesky_solve(b, L)
        torch.cuda.synchronize()
        ts.append((time.perf_counter() - t0) * 1e6)
    ts.sort()
    print(f"n {n} batch 16: cholesky_ex + cholesky_solve median {ts[5]:.0f} us min {ts[0]:.0f} us", flush=True)
