"""Debug: magnitude of the replay divergence (la batch captured at t=5)."""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd"), os.path.join(os.getcwd(), "tests")]
import torch
from test_gpu_lookahead import _batch
E, N = 128, 32
ref, la = _batch(E, N, False), _batch(E, N, True)
g = torch.Generator(device="cuda").manual_seed(5)
ref.reset(); la.reset()
a = torch.zeros((E, 2), dtype=torch.float64, device="cuda")
for t in range(6):
    a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
    ref.step(a); la.step(a)
graph = torch.cuda.CUDAGraph()
with torch.cuda.graph(graph):
    la.step(a)
for t in range(6, 27):
    a.copy_(torch.rand(a.shape, dtype=torch.float64, device="cuda", generator=g) * 2 - 1)
    ref.step(a)
    graph.replay()
    torch.cuda.synchronize()
    dl = (ref.state["lat"] - la.state["lat"]).abs()
    dh = (ref.state["hdg"] - la.state["hdg"]).abs()
    nav_r, nav_l = ref.state["nav"], la.state["nav"]
    sc_r, sc_l = ref.envs["step_count"], la.envs["step_count"]
    print(f"t={t} max|dlat|={dl.max().item():.3e} max|dhdg|={dh.max().item():.3e} "
          f"nav diff={int((nav_r != nav_l).sum())} step_count ref/la env0 {int(sc_r[0])}/{int(sc_l[0])} "
          f"episode ref/la {int(ref.envs['episode'][0]) if 'episode' in ref.envs else -1}/{int(la.envs['episode'][0]) if 'episode' in la.envs else -1}")
    if dl.max().item() > 0:
        i = int(torch.argmax(dl.view(E, N).max(dim=1).values))
        print("  env", i, "ref lat", ref.state["lat"].view(E, N)[i, :4].tolist())
        print("  env", i, "la  lat", la.state["lat"].view(E, N)[i, :4].tolist())
        print("  ref hdg", ref.state["hdg"].view(E, N)[i, :4].tolist())
        print("  la  hdg", la.state["hdg"].view(E, N)[i, :4].tolist())
        break
