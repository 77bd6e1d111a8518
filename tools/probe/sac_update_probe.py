"""Where a FusedSAC update's time goes (timing only; results are wrong in the ablated
variants): the update captured as a HIP graph and replayed, in full, without its rocBLAS
GEMMs, without its tools/sac_fused.hip launches, and the Adam launches alone.  GPU only:
  python tools/probe/sac_update_probe.py [obs_dim act_dim]"""
import os
import sys
import time

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), ".."))
import sac_torch  # noqa: E402

od = int(sys.argv[1]) if len(sys.argv) > 1 else 4
ad = int(sys.argv[2]) if len(sys.argv) > 2 else 1
dev = torch.device("cuda", 0)
torch.backends.cuda.preferred_blas_library("cublas")


def make():
    s = sac_torch.FusedSAC(od, ad, dev, seed=0, lr=1e-3, buffer=100000)
    n = 8192
    s.insert(torch.randn((n, od), device=dev), torch.rand((n, ad), device=dev) * 2 - 1,
             torch.randn((n,), device=dev), torch.randn((n, od), device=dev),
             (torch.rand((n,), device=dev) < 0.05).float())
    return s


def timed(fn, reps=300):
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(side):
        for _ in range(3):
            fn()
    torch.cuda.current_stream().wait_stream(side)
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        fn()
    for _ in range(20):
        g.replay()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


s = make()
print(f"obs {od} act {ad}: full update {timed(lambda: s.update(losses=False)):.1f} us")
mm, bmm = torch.mm, torch.bmm
torch.mm = lambda *a, **k: None
torch.bmm = lambda *a, **k: None
print(f"  without the GEMMs        {timed(lambda: s.update(losses=False)):.1f} us")
torch.mm, torch.bmm = mm, bmm
call = s._call
s._call = lambda *a, **k: None
print(f"  without sac_fused launches {timed(lambda: s.update(losses=False)):.1f} us")
s._call = call
print(f"  critic Adam alone        {timed(lambda: s.opt_q.step()):.1f} us")
print(f"  actor Adam alone         {timed(lambda: s.opt_a.step()):.1f} us")
x = torch.zeros(256, 256, device=dev)
y = torch.zeros(256, 256, device=dev)
o = torch.zeros(256, 256, device=dev)
print(f"  one 256^3 mm alone       {timed(lambda: torch.mm(x, y, out=o)):.1f} us")
def ten():
    for _ in range(10):
        torch.mm(x, y, out=o)
print(f"  ten dependent 256^3 mm   {timed(ten):.1f} us")
z = torch.zeros(1, device=dev)
def tiny():
    for _ in range(10):
        z.add_(1.0)
print(f"  ten tiny launches        {timed(tiny):.1f} us")
