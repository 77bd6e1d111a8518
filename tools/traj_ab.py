"""A/B of the trajectory store at C4's shard sizes (one GPU): per RL step wall time and
HIP-event time of the bare launch loop, 100 steps after a reset (inside the episodes the
reset's own producer launch flies) and 400 steps on (the async producers in steady state),
with the store off, on, and on without the async producers (BSG_TRAJ_NOASYNC=1 is read by
bsg_set_trajectory, so each mode runs in its own process).

    python tools/traj_ab.py [E ...]            (runs the three modes as child processes)
    python tools/traj_ab.py --mode on|off|noasync E
"""
import os
import subprocess
import sys
import time

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]


def one(mode, E):
    import torch
    from bluesky_gym import config, core
    b = core.DeviceBatch(config.merge_config(num_ac=32), E, compute_cd=True, seed=1234,
                         trajectory=(mode != "off"))     # (explicit: the default is off)
    bank = torch.rand((16, E, 2), dtype=torch.float64, device="cuda") * 2 - 1
    b.reset()
    ev0 = torch.cuda.Event(enable_timing=True)
    ev1 = torch.cuda.Event(enable_timing=True)

    def timed(n, k0):
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        ev0.record()
        for k in range(n):
            b.step(bank[(k0 + k) % 16])
        ev1.record()
        torch.cuda.synchronize()
        return (time.perf_counter() - t0) / n * 1e6, ev0.elapsed_time(ev1) / n * 1e3

    for k in range(5):
        b.step(bank[k % 16])
    w1, e1 = timed(100, 5)
    for k in range(100):
        b.step(bank[k % 16])
    w2, e2 = timed(300, 205)
    info = b.trajectory_info() if b.trajectory else {"copies": None, "producer_launches": 0}
    cp = int(info["copies"].sum()) if info["copies"] is not None else 0
    print(f"E={E:5d} store {mode:8s} steps 5..105: wall {w1:6.1f} us event {e1:6.1f} us | "
          f"steps 205..505: wall {w2:6.1f} us event {e2:6.1f} us | copies {cp} "
          f"producer launches {info['producer_launches']}", flush=True)
    b.close()


def main():
    if sys.argv[1:2] == ["--mode"]:
        return one(sys.argv[2], int(sys.argv[3]))
    sizes = [int(x) for x in sys.argv[1:]] or [512, 1024]
    for E in sizes:
        for mode in ("off", "on", "noasync"):
            env = dict(os.environ, BSG_TRAJ_NOASYNC="1" if mode == "noasync" else "0")
            r = subprocess.run([sys.executable, __file__, "--mode", mode, str(E)], env=env,
                               timeout=300)
            if r.returncode != 0:
                sys.exit(r.returncode)


if __name__ == "__main__":
    main()
