"""Time DeviceBatch.step under configuration ablations (kernel time via HIP events)."""
import sys, os, json, time
WALL = [0.0]
sys.path[:0] = [os.getcwd(), os.path.join(os.getcwd(), "bluesky-gym-hallucination_amd")]
import torch
from bluesky_gym import core, config

def run(cfg, E, cd, steps=60, warm=10, la=None):
    b = core.DeviceBatch(cfg, E, compute_cd=cd, seed=1,
                         memo_cache=os.environ.get("BSG_NO_MEMO", "0") != "1", lookahead=la)
    b.reset()
    act = torch.rand((8, E, b.act_dim), dtype=torch.float64, device="cuda") * 2 - 1
    for k in range(warm):
        b.step(act[k % 8])
    torch.cuda.synchronize(); b.step_timing(); b.set_timing(True)
    for k in range(steps):
        b.step(act[k % 8])
    torch.cuda.synchronize()
    ms, n = b.step_timing()
    b.set_timing(False)
    t0 = time.perf_counter()
    for k in range(steps):
        b.step(act[k % 8])
    torch.cuda.synchronize()
    WALL[0] = (time.perf_counter() - t0) / steps * 1e3
    return ms / n

only = set(sys.argv[1:])
res = {}
for spec in [
    ("merge32_full", config.merge_config(num_ac=32), 4096, True),
    ("merge32_nocd", config.merge_config(num_ac=32), 4096, False),
    ("merge32_S1", config.merge_config(num_ac=32, action_frequency=1), 4096, True),
    ("merge32_S1_nocd", config.merge_config(num_ac=32, action_frequency=1), 4096, False),
    ("merge32_S0_nocd", config.merge_config(num_ac=32, action_frequency=0), 4096, False),
    ("merge16_full_1024", config.merge_config(num_ac=16), 1024, True),
    ("vert32_full_2048", config.vertical_config(num_intruders=31), 2048, True),
    ("descent_4096", config.descent_config(), 4096, False),
    ("horiz32_full_4096", config.horizontal_config(num_intruders=31), 4096, True),
    ("merge32_full_512", config.merge_config(num_ac=32), 512, True),      # C4 shard at 8 GPUs
    ("merge32_full_1024", config.merge_config(num_ac=32), 1024, True),    # C4 shard at 4 GPUs
    ("merge32_full_2048", config.merge_config(num_ac=32), 2048, True),    # C4 shard at 2 GPUs
    ("descent_512", config.descent_config(), 512, False),                 # C5 shard at 8 GPUs
    ("merge32_nocd_512", config.merge_config(num_ac=32), 512, False),
    ("merge32_nocd_1024", config.merge_config(num_ac=32), 1024, False),
    ("merge32_nocd_2048", config.merge_config(num_ac=32), 2048, False),
    ("merge32_full_8192", config.merge_config(num_ac=32), 8192, True),
    ("merge32_full_16384", config.merge_config(num_ac=32), 16384, True),
    # the Merge lookahead forced off / on (DeviceBatch's default: on up to 2048 envs)
    ("merge32_full_512_nola", config.merge_config(num_ac=32), 512, True, False),
    # C4 shards without episode ends in the timed window (no spawns: what resets cost)
    ("merge32_full_512_noreset", config.merge_config(num_ac=32, max_episode_steps=1000000), 512, True),
    ("merge32_full_2048_noreset", config.merge_config(num_ac=32, max_episode_steps=1000000), 2048, True),
    ("merge32_full_1024_nola", config.merge_config(num_ac=32), 1024, True, False),
    ("merge32_full_2048_nola", config.merge_config(num_ac=32), 2048, True, False),
    ("merge32_full_la", config.merge_config(num_ac=32), 4096, True, True),
    # Vertical (C3) with the lookahead forced off (DeviceBatch's default: on up to 2048 envs)
    ("vert32_full_2048_nola", config.vertical_config(num_intruders=31), 2048, True, False),
    ("vert32_full_1024", config.vertical_config(num_intruders=31), 1024, True),
    ("vert32_full_1024_nola", config.vertical_config(num_intruders=31), 1024, True, False),
]:
    name, cfg, E, cd = spec[:4]
    la = spec[4] if len(spec) > 4 else None
    if only and name not in only:
        continue
    res[name] = run(cfg, E, cd, la=la)
    print(name, f"{res[name]*1e3:.1f} us  (wall/step untimed {WALL[0]*1e3:.1f} us)", flush=True)
json.dump(res, open(os.environ.get("ABLATE_OUT", "gpurun_out/ablate.json"), "w"), indent=1)
