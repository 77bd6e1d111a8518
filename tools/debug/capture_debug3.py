"""Debug: isolate the replay divergence (la batch, warm-up step on a side stream, capture)."""
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
            out.append(k)
    return out

def run(name, warm_side, capture, replay_all, la_on=True, E=128, N=32, T=46):
    ref, la = _batch(E, N, False), _batch(E, N, la_on)
    g = torch.Generator(device="cuda").manual_seed(5)
    ref.reset(); la.reset()
    a = torch.zeros((E, la.act_dim), dtype=torch.float64, device="cuda")
    for t in range(5):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a); la.step(a)
    if warm_side:
        s = torch.cuda.Stream()
        s.wait_stream(torch.cuda.current_stream())
        with torch.cuda.stream(s):
            la.step(a)
        torch.cuda.current_stream().wait_stream(s)
    else:
        la.step(a)
    ref.step(a)
    graph = None
    if capture:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            la.step(a)
    for t in range(6, T):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a)
        if graph is not None and (replay_all or t % 2):
            graph.replay()
        else:
            la.step(a)
        d = diff(_snap(ref), _snap(la))
        if d:
            print(f"  {name}: first diff at t={t}: {d[:8]}")
            return
    print(f"  {name}: identical through t={T-1}")

#run("V0 side warm-up, capture, replay all", True, True, True)
#run("V2 current-stream warm-up, capture, replay all", False, True, True)
#run("V3 side warm-up, no capture", True, False, False)
run("V5 side warm-up, capture, direct only after", True, True, False, T=46) if False else None

def run_memo(name, la_on, T=46, E=128, N=32):
    ref, la = _batch(E, N, False), _batch(E, N, la_on)
    g = torch.Generator(device="cuda").manual_seed(5)
    ref.reset(); la.reset()
    a = torch.zeros((E, la.act_dim), dtype=torch.float64, device="cuda")
    for t in range(5):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a); la.step(a)
    la.step(a); ref.step(a)
    for t in range(6, T):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a)
        la.memo_cache.fill_(float("nan"))
        la.step(a)
        d = diff(_snap(ref), _snap(la))
        if d:
            print(f"  {name}: first diff at t={t}: {d[:8]}")
            return
    print(f"  {name}: identical through t={T-1}")

#run_memo("M1 no lookahead, memo NaN before every step from t=6", False)

import ctypes as C
def run_g(name, off_api, T=46, E=128, N=32):
    ref, la = _batch(E, N, False), _batch(E, N, True)
    g = torch.Generator(device="cuda").manual_seed(5)
    ref.reset(); la.reset()
    a = torch.zeros((E, la.act_dim), dtype=torch.float64, device="cuda")
    for t in range(5):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a); la.step(a)
    la.step(a); ref.step(a)
    if off_api:
        assert la.lib.bsg_set_lookahead(la._ctx, None, C.c_int64(0)) == 0
        la.step(a); ref.step(a)          # the transition's memset runs here, outside any graph
    graph = torch.cuda.CUDAGraph()
    with torch.cuda.graph(graph):
        la.step(a)
    for t in range(6, T):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a)
        graph.replay()
        d = diff(_snap(ref), _snap(la))
        if d:
            print(f"  {name}: first diff at t={t}: {d[:8]}")
            return
    print(f"  {name}: identical through t={T-1}")

run_g("G0 la batch captured (la off by capture), replay all", False)
#run_g("G1 la batch, la off by API first, then capture, replay all", True)

def run_f(name, fill, in_graph, T=46, E=128, N=32):
    ref, la = _batch(E, N, False), _batch(E, N, False)
    g = torch.Generator(device="cuda").manual_seed(5)
    ref.reset(); la.reset()
    a = torch.zeros((E, la.act_dim), dtype=torch.float64, device="cuda")
    for t in range(5):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a); la.step(a)
    la.step(a); ref.step(a)
    def body():
        if fill == "ones":
            la.memo_cache.view(torch.int64).fill_(-1)
        else:
            la.memo_cache.fill_(float("nan"))
        la.step(a)
    graph = None
    if in_graph:
        graph = torch.cuda.CUDAGraph()
        with torch.cuda.graph(graph):
            body()
    for t in range(6, T):
        a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
        ref.step(a)
        graph.replay() if graph is not None else body()
        d = diff(_snap(ref), _snap(la))
        if d:
            print(f"  {name}: first diff at t={t}: {d[:8]}")
            return
    print(f"  {name}: identical through t={T-1}")

#run_f("F1 no-la batch, 0xFF fill + step, direct", "ones", False)
#run_f("F2 no-la batch, NaN fill + step, direct", "nan", False)
#run_f("F3 no-la batch, 0xFF fill + step, in graph", "ones", True)
