import sys, numpy as np
import os; R = os.path.dirname(os.path.dirname(os.path.abspath(__file__))); sys.path[:0] = [R, os.path.join(R, 'tests')]
import ref_policy as sp
from oracle import batched_areas as oba
import test_ref_logs as trl
W = sp.load()
for alt in (350.0, 0.0):
    oba.C_ALTITUDE = alt
    for tag in ("sector", "sector_ppo"):
        E = 200
        rec = trl.rollout_oracle(oba.SectorOracle(E, seed=5, compute_cd=False), tag, W, E)
        lines, bad, rows = sp.compare(W, tag, rec)
        print(f"== C_ALTITUDE {alt} {tag}")
        print("\n".join(lines))
