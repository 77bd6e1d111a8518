"""Which docs/BLUESKY_SUBSET_SPEC.md A.3 decision moves a held-out log statistic?

Rolls the reference's saved actors out on the CPU oracle (tests/test_ref_logs.py) with
one or more oracle/bluesky_subset.py constants overridden, and prints every statistic's
z against the actor's own training log.  A diagnostic for DESIGN.md §5 only: the product
constants stay frozen (the held-out check must not be re-fitted).

    python tools/envelope_sensitivity.py descent_ddpg vertical_ppo --set VSMAX=15 --envs 400
"""
from __future__ import annotations

import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "tests")]

import ref_policy as sp  # noqa: E402
from oracle import bluesky_subset as bsx  # noqa: E402
from test_ref_logs import MAKERS, rollout_oracle  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("tags", nargs="+")
    ap.add_argument("--set", action="append", default=[], help="CONST=value (bluesky_subset)")
    ap.add_argument("--envs", type=int, default=0, help="envs per rollout (0 = the test's)")
    args = ap.parse_args()
    for kv in args.set:
        k, v = kv.split("=")
        if not hasattr(bsx, k):
            raise SystemExit(f"bluesky_subset has no {k}")
        setattr(bsx, k, float(v))
        if k == "VSMAX":
            bsx.VSMIN = -float(v)
    W = sp.load()
    from test_ref_logs import CASES
    for tag in args.tags:
        E = args.envs or CASES.get(tag, 400)
        rec = rollout_oracle(MAKERS[sp.env_of(tag)](E), tag, W, E)
        lines, _, _ = sp.compare(W, tag, rec)
        print(f"# {' '.join(args.set) or 'frozen'}")
        print("\n".join(lines), flush=True)


if __name__ == "__main__":
    main()
