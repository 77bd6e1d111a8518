"""Run one configuration for PMC collection: python tools/one_config.py KIND N E S CD STEPS"""
import os, sys
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import torch
from bluesky_gym import config, core
kind, N, E, S, cd, steps = sys.argv[1], int(sys.argv[2]), int(sys.argv[3]), int(sys.argv[4]), int(sys.argv[5]), int(sys.argv[6])
cfg = {"merge": lambda: config.merge_config(num_ac=N, action_frequency=S),
       "vertical": lambda: config.vertical_config(num_intruders=N - 1, action_frequency=S),
       "descent": lambda: config.descent_config(action_frequency=S)}[kind]()
b = core.DeviceBatch(cfg, E, compute_cd=bool(cd), seed=1)   # lookahead: DeviceBatch default
b.reset()
act = torch.rand((8, E, b.act_dim), dtype=torch.float64, device="cuda") * 2 - 1
for k in range(steps):
    b.step(act[k % 8])
torch.cuda.synchronize()
