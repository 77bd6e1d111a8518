"""Step time (Merge 32 aircraft by default; AB_KIND=vertical|descent|horizontal) (HIP events around 300 back-to-back launches after 100 warm-up
steps, the DeviceBatch defaults: lookahead up to 2,048 envs) of the tree in the current
directory -- run from another checkout's root to A/B two builds on one box:

    (cd <other tree> && python /root/repo/tools/ab_tree.py 512 1024) ; python tools/ab_tree.py 512 1024
"""
import os
import sys

sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import torch
from bluesky_gym import config, core

tag = os.environ.get("AB_TAG", os.path.basename(os.getcwd()))
kind = os.environ.get("AB_KIND", "merge")        # merge | vertical | descent | horizontal
cfgs = {"merge": lambda: config.merge_config(num_ac=32),
        "vertical": lambda: config.vertical_config(num_intruders=31),
        "descent": lambda: config.descent_config(),
        "horizontal": lambda: config.horizontal_config(num_intruders=31)}
for E in [int(x) for x in sys.argv[1:]] or [512, 1024, 2048, 4096]:
    b = core.DeviceBatch(cfgs[kind](), E, compute_cd=kind != "descent", seed=1)
    b.reset()
    bank = torch.rand((16, E, b.act_dim), dtype=torch.float64, device="cuda") * 2 - 1
    for k in range(100):
        b.step(bank[k % 16])
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    e0.record()
    for k in range(300):
        b.step(bank[k % 16])
    e1.record()
    torch.cuda.synchronize()
    print(f"{tag:8s} {kind:10s} E={E:5d} event {e0.elapsed_time(e1) / 300 * 1e3:6.2f} us/step "
          f"(lookahead {b.lookahead})", flush=True)
    b.close()
