"""The trajectory store (bsg_set_trajectory; csrc/bsg_kernels.hip produce_kernel and the
lookahead's copy path): MergeEnv's intruders fly whole future episodes ahead -- a Merge
intruder's episode depends only on (seed, env, Philox episode counter), merge_env.py:148-158
with RESO OFF -- and the lookahead copies the next step's state (and the intruder pairs'
conflict rows) instead of propagating it.  It must be invisible: every output and state
buffer bit-identical to the inline path, step by step, through NEXT_STEP autoresets, masked
resets, host spawn rows (which retire the store), patched env constants, with the producers
on the launch stream ("sync") and on their own low-priority stream (the default)."""
import numpy as np
import pytest
import torch

from test_gpu_lookahead import _same, _snap

pytestmark = pytest.mark.gpu


def _batch(E, N, la, tj, seed=11, maxep=12, params=None):
    from bluesky_gym import config, core
    cfg = config.merge_config(num_ac=N, max_episode_steps=maxep, params=params)
    return core.DeviceBatch(cfg, E, compute_cd=True, seed=seed, learner=True, lookahead=la,
                            trajectory=tj)


def _run(E, N, T, tj, maxep, params=None, host_rows_at=None, mask_reset_at=None):
    ref, b = _batch(E, N, False, False, maxep=maxep, params=params), \
        _batch(E, N, True, tj, maxep=maxep, params=params)
    assert b.lookahead and b.trajectory and not ref.lookahead
    g = torch.Generator(device="cuda").manual_seed(3)
    ref.reset()
    b.reset()
    _same(_snap(ref), _snap(b), -1)
    gen0 = b.trajectory_info()["generation"]
    for t in range(T):
        a = torch.rand((E, 2), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
        ref.step(a)
        b.step(a)
        _same(_snap(ref), _snap(b), t)
        if t == mask_reset_at:               # an explicit masked reset with device spawns
            m = (torch.arange(E, device="cuda") % 4 == 1).to(torch.uint8)
            ref.reset(m)
            b.reset(m)
            _same(_snap(ref), _snap(b), t)
        if t == host_rows_at:                # a masked reset from host spawn rows
            m = (torch.arange(E, device="cuda") % 5 == 2).to(torch.uint8)
            rng = np.random.default_rng(t)
            sp = np.zeros((E, 2 * N))
            sp[:, 0::2] = rng.uniform(-15, 15, (E, N))
            sp[:, 1::2] = rng.uniform(20, 200, (E, N))
            sp = torch.from_numpy(sp)
            ref.reset(m, spawn=sp)
            b.reset(m, spawn=sp)
            _same(_snap(ref), _snap(b), t)
            assert b.trajectory_info()["generation"] != gen0     # the store was retired
    torch.cuda.synchronize()
    return b.trajectory_info()


def test_trajectory_sync_bit_identical():
    """Producers on the launch stream: every episode after the first few steps is served
    from the store; 5 TimeLimits of 12 steps, a masked reset mid-run."""
    E, N = 256, 32
    info = _run(E, N, 70, "sync", maxep=12, mask_reset_at=30)
    # most lookahead slots came from the store (the first episode's are flown by the
    # reset's own producer launch too)
    assert int(info["copies"].sum()) > E * 40, int(info["copies"].sum())
    assert info["producer_launches"] > 1


def test_trajectory_async_bit_identical():
    """The product path: producers on their own least-priority stream, each publishing itself
    on the device when its last wave ends; the reference TimeLimit (50) over three episodes."""
    E, N = 512, 32
    info = _run(E, N, 160, True, maxep=50)
    assert info["producer_launches"] > 2
    assert int(info["copies"].sum()) > E * 60, int(info["copies"].sum())


def test_trajectory_host_rows_retire_the_store():
    """A reset from host spawn rows (the parity mode's draws) is another episode under the
    same Philox counter: the store is retired (new generation) and the outputs stay the
    inline path's; later episodes are served again."""
    E, N = 128, 20
    info = _run(E, N, 60, "sync", maxep=10, host_rows_at=17, mask_reset_at=35)
    assert int(info["copies"].sum()) > 0


def test_trajectory_with_patched_constants():
    """The producers fly with the patched module constants too (bsg_set_params)."""
    E, N = 256, 32
    params = {"D_HEADING": 30.0, "INTRUDER_DISTANCE_MAX": 150.0, "INTRUSION_DISTANCE": 9.0}
    info = _run(E, N, 40, "sync", maxep=12, params=params)
    assert int(info["copies"].sum()) > E * 20


@pytest.mark.parametrize("N", [8, 16])
def test_trajectory_small_groups(N):
    """Env groups of 8 / 4 envs per wave (GS 8, 16): the producers' and the copy's indexing."""
    info = _run(200, N, 40, "sync", maxep=9)
    assert int(info["copies"].sum()) > 200 * 20


def test_trajectory_async_host_ahead():
    """The bench's regime: the host enqueues steps far ahead of the GPU (no synchronisation
    in the loop), so the lookahead waves meet producers that finish while the step launches
    enqueued before them run.  Every step's outputs and state are snapshotted on the device
    and compared after the loop."""
    E, N, T = 512, 32, 220
    ref, b = _batch(E, N, False, False, maxep=50), _batch(E, N, True, True, maxep=50)
    g = torch.Generator(device="cuda").manual_seed(9)
    acts = torch.rand((T, E, 2), dtype=torch.float64, device="cuda", generator=g) * 2 - 1
    ref.reset()
    b.reset()
    sa, sb = [], []
    for t in range(T):
        ref.step(acts[t])
        b.step(acts[t])
        sa.append(_snap(ref))
        sb.append(_snap(b))
    torch.cuda.synchronize()
    for t in range(T):
        _same(sa[t], sb[t], t)
    info = b.trajectory_info()
    assert int(info["copies"].sum()) > E * 120, int(info["copies"].sum())
