"""Debug: where a captured-then-replayed step first departs from the inline batch."""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd"), os.path.join(os.getcwd(), "tests")]
import torch
from test_gpu_lookahead import _batch, _snap

def diff(x, y):
    out = []
    for k in x:
        a, b = x[k], y[k]
        if a.dtype.is_floating_point:
            a = a.view(torch.int64 if a.element_size() == 8 else torch.int32)
            b = b.view(torch.int64 if b.element_size() == 8 else torch.int32)
        if not torch.equal(a, b):
            nz = torch.nonzero(a != b)
            envs = sorted(set(nz[:, 0].tolist()))[:8]
            out.append(f"{k}: {nz.shape[0]} entries, envs {envs}")
    return out

def run(la_on, capture, replay_odd=True, E=128, N=32):
    ref, la = _batch(E, N, False), _batch(E, N, la_on)
    g = torch.Generator(device="cuda").manual_seed(5)
    ref.reset(); la.reset()
    a = torch.zeros((E, la.act_dim), dtype=torch.float64, device="cuda")
    for t in range(5):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a); la.step(a)
    s = torch.cuda.Stream()
    s.wait_stream(torch.cuda.current_stream())
    with torch.cuda.stream(s):
        la.step(a)
    torch.cuda.current_stream().wait_stream(s)
    ref.step(a)
    graph = None
    if capture:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            la.step(a)
    for t in range(6, 40):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a)
        if graph is not None and (t % 2 or not replay_odd):
            graph.replay()
        else:
            la.step(a)
        d = diff(_snap(ref), _snap(la))
        if d:
            print(f"  la={la_on} capture={capture} replay_odd={replay_odd}: first diff at t={t} ({'replay' if graph is not None and (t % 2 or not replay_odd) else 'direct'}):")
            for line in d[:12]:
                print("    ", line)
            return
    print(f"  la={la_on} capture={capture} replay_odd={replay_odd}: identical through t=39")

run(True, False)
run(False, True)
run(True, True)
run(True, True, replay_odd=False)
