"""C-ABI checks that need no GPU: libbsg.so loads, exports every entry point declared in
include/bsg.h, the ctypes mirror has the C struct layout (checked against gcc), and the
shape helpers agree with the reference observation/action spaces."""
import ctypes as C
import os
import re
import subprocess

import pytest

from bluesky_gym import _native as nat
from bluesky_gym.obs_layout import ObsLayout

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(REPO, "include", "bsg.h")


def declared_functions():
    src = open(HDR).read()
    return sorted(set(re.findall(r"^\s*(?:int32_t|int64_t|const char\*)\s+(bsg_\w+)\s*\(", src, re.M)))


def test_header_declares_the_ctypes_symbol_set():
    assert declared_functions() == sorted(nat.EXPORTED_SYMBOLS)


def test_library_exports_every_declared_symbol():
    lib = nat.load_library()
    out = subprocess.run(["nm", "-D", "--defined-only", nat.LIB_PATH], capture_output=True,
                         text=True, check=True).stdout
    exported = set(re.findall(r"\bT (bsg_\w+)", out))
    for sym in declared_functions():
        assert sym in exported, sym
        getattr(lib, sym)
    assert lib.bsg_abi_version() == nat.ABI_VERSION


def test_shape_helpers_match_reference_spaces():
    lib = nat.load_library()
    # merge_env.py:59-74 (K=5 -> 40), vertical_cr_env.py:67-83 (5 intruders -> 39), descent 4
    assert lib.bsg_obs_dim(nat.ENV_MERGE, 20, 5) == 40
    assert lib.bsg_obs_dim(nat.ENV_VERTICAL_CR, 6, 0) == 39
    assert lib.bsg_obs_dim(nat.ENV_VERTICAL_CR, 32, 0) == 221
    assert lib.bsg_obs_dim(nat.ENV_DESCENT, 1, 0) == 4
    assert lib.bsg_obs_dim(nat.ENV_MERGE, 4, 5) < 0            # fewer intruders than K
    assert lib.bsg_action_dim(nat.ENV_MERGE) == 2
    assert lib.bsg_action_dim(nat.ENV_DESCENT) == 1
    assert lib.bsg_spawn_width(nat.ENV_MERGE, 32) == 64
    assert lib.bsg_spawn_width(nat.ENV_VERTICAL_CR, 6) == 22
    for kind, n, k in ((nat.ENV_MERGE, 32, 5), (nat.ENV_VERTICAL_CR, 32, 0), (nat.ENV_DESCENT, 1, 0),
                       (nat.ENV_HORIZONTAL_CR, 6, 0), (nat.ENV_HORIZONTAL_CR, 32, 0),
                       (nat.ENV_STATIC_OBSTACLE, 1, 0), (nat.ENV_SECTOR_CR, 32, 4)):
        assert ObsLayout(kind, n, k).dim == lib.bsg_obs_dim(kind, n, k)


def test_ctypes_struct_layout_matches_c(tmp_path):
    prog = tmp_path / "layout.c"
    fields_c = [f[0] for f in nat.BsgConfig._fields_]
    fields_b = [f[0] for f in nat.BsgBuffers._fields_]
    fields_w = [f[0] for f in nat.BsgWind._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', "int main(void){",
             'printf("%zu %zu %zu\\n", sizeof(bsg_config), sizeof(bsg_buffers), sizeof(bsg_wind));']
    lines += [f'printf("%zu\\n", offsetof(bsg_config, {f}));' for f in fields_c]
    lines += [f'printf("%zu\\n", offsetof(bsg_buffers, {f}));' for f in fields_b]
    lines += [f'printf("%zu\\n", offsetof(bsg_wind, {f}));' for f in fields_w]
    lines += ["return 0;}"]
    prog.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(prog)], check=True)
    vals = subprocess.run([str(exe)], capture_output=True, text=True, check=True).stdout.split()
    assert int(vals[0]) == C.sizeof(nat.BsgConfig)
    assert int(vals[1]) == C.sizeof(nat.BsgBuffers)
    assert int(vals[2]) == C.sizeof(nat.BsgWind)
    offs = [int(v) for v in vals[3:]]
    nc, nb = len(fields_c), len(fields_b)
    assert offs[:nc] == [getattr(nat.BsgConfig, f).offset for f in fields_c]
    assert offs[nc:nc + nb] == [getattr(nat.BsgBuffers, f).offset for f in fields_b]
    assert offs[nc + nb:] == [getattr(nat.BsgWind, f).offset for f in fields_w]


def test_create_fails_cleanly_without_device_or_bad_config():
    lib = nat.load_library()
    from bluesky_gym import config
    ctx = C.c_void_p()
    bad = config.merge_config(num_ac=70).to_c(16, 1, 1, 0, 0)      # > 64 aircraft
    rc = lib.bsg_create(C.byref(bad), C.byref(ctx))
    assert rc == -1 and b"num_ac" in lib.bsg_last_error()
    cfg = config.merge_config(num_ac=32).to_c(16, 1, 1, 0, 0)
    cfg.abi_version = 99
    assert lib.bsg_create(C.byref(cfg), C.byref(ctx)) == -1
    assert lib.bsg_step(None, None, None, None) == -1               # null ctx -> error, no crash


def test_empty_batch_and_bad_timing_interval_rejected():
    """num_envs = 0 (an empty batch) is refused at bsg_create with a message, before any
    device work; a negative timing interval is refused on a null ctx without a crash."""
    lib = nat.load_library()
    from bluesky_gym import config
    ctx = C.c_void_p()
    cfg = config.merge_config(num_ac=32).to_c(0, 1, 1, 0, 0)
    assert lib.bsg_create(C.byref(cfg), C.byref(ctx)) == -1
    assert b"num_envs" in lib.bsg_last_error()
    assert lib.bsg_set_timing(None, -1) == -1


def test_policy_host_validation_without_gpu():
    """The fused SAC actor's host layer: no CPU fallback, and the C entry point rejects bad
    shapes before touching a device."""
    import ctypes as C
    import numpy as np
    from bluesky_gym.policy import SACPolicy
    with np.load(os.path.join(os.path.dirname(__file__), "golden", "sac_actors.npz")) as z:
        W = {k.split("/", 1)[1]: z[k] for k in z.files if k.startswith("descent/") and "/log" not in k
             and not k.endswith("obs_dim")}
    with pytest.raises(nat.BsgError):
        SACPolicy(W, "cpu")
    lib = nat.load_library()
    buf = (C.c_float * 70000)()
    p = C.cast(buf, C.c_void_p).value
    w = nat.BsgSacActor(4, 1, 128, 0, *([p] * 8))        # hidden must be 256
    act = (C.c_double * 8)()
    rc = lib.bsg_policy_sac(C.byref(w), p, 8, 4, None, C.cast(act, C.c_void_p), None, None)
    assert rc == -1                                      # BSG_E_INVALID_ARG
    assert b"hidden" in lib.bsg_last_error()
    w = nat.BsgSacActor(4, 5, 256, 0, *([p] * 8))        # act_dim <= 4
    assert lib.bsg_policy_sac(C.byref(w), p, 8, 4, None, C.cast(act, C.c_void_p), None, None) == -1
    w = nat.BsgSacActor(4, 1, 256, 0, *([p] * 8))
    assert lib.bsg_policy_sac(C.byref(w), p, 8, 3, None, C.cast(act, C.c_void_p), None, None) == -1
    assert lib.bsg_policy_sac(C.byref(w), p, 0, 4, None, C.cast(act, C.c_void_p), None, None) == 0


def test_policy_rejects_every_bad_pointer_argument():
    """SACPolicy._check runs before any raw pointer reaches bsg_policy_sac: narrow obs
    views, eps / out / log_prob on another device, strided log_prob.  The
    policy object is built without a device (the checks are host logic), with the CPU as
    its 'device' so that tensors on another device can be made here."""
    import torch
    from bluesky_gym.policy import SACPolicy
    pol = SACPolicy.__new__(SACPolicy)
    pol.device, pol.obs_dim, pol.act_dim = torch.device("cpu"), 4, 1
    E = 8
    big = torch.zeros((E, 10), dtype=torch.float32)
    ok = dict(eps=torch.zeros((E, 1)), out=torch.zeros((E, 1), dtype=torch.float64),
              log_prob=torch.zeros(E))
    assert pol._check(big[:, 2:6], **ok) == E           # a 4-wide column view: stride 10, fine
    with pytest.raises(ValueError, match="features"):
        pol._check(big[:, 7:10], **ok)                   # 3 < obs_dim: would read past the row
    with pytest.raises(ValueError, match="log_prob"):
        pol._check(big, ok["eps"], ok["out"], torch.zeros((E, 2))[:, 0])   # strided [E] view
    with pytest.raises(ValueError, match="obs"):
        pol._check(big.double(), **ok)
    meta = torch.device("meta")                          # "another device" without a GPU
    with pytest.raises(ValueError, match="eps"):
        pol._check(big, torch.zeros((E, 1), device=meta), ok["out"], ok["log_prob"])
    with pytest.raises(ValueError, match="log_prob"):
        pol._check(big, ok["eps"], ok["out"], torch.zeros(E, device=meta))
    with pytest.raises(ValueError, match="out"):
        pol._check(big, ok["eps"], torch.zeros((E, 1), dtype=torch.float64, device=meta),
                   ok["log_prob"])


def test_load_sb3_actor_from_zip(tmp_path):
    """SACPolicy.from_sb3_zip's loader: policy.pth inside an SB3 archive, weights only, actor.*
    keys (a synthetic archive of the SB3 layout; critic keys and the pickled `data` member
    are ignored)."""
    import io
    import zipfile
    import numpy as np
    import torch
    from bluesky_gym.policy import load_sb3_actor
    shapes = {"latent_pi.0.weight": (256, 4), "latent_pi.0.bias": (256,),
              "latent_pi.2.weight": (256, 256), "latent_pi.2.bias": (256,),
              "mu.weight": (1, 256), "mu.bias": (1,), "log_std.weight": (1, 256), "log_std.bias": (1,)}
    g = torch.Generator().manual_seed(0)
    sd = {f"actor.{k}": torch.randn(s, generator=g) for k, s in shapes.items()}
    sd["critic.qf0.0.weight"] = torch.zeros(256, 5)
    buf = io.BytesIO()
    torch.save(sd, buf)
    zp = tmp_path / "model.zip"
    with zipfile.ZipFile(zp, "w") as z:
        z.writestr("policy.pth", buf.getvalue())
        z.writestr("data", b"not read")
    w = load_sb3_actor(zp)
    assert sorted(w) == sorted(shapes)
    for k in shapes:
        assert np.array_equal(np.asarray(w[k]), sd[f"actor.{k}"].numpy())
    with zipfile.ZipFile(tmp_path / "bad.zip", "w") as z:
        b2 = io.BytesIO()
        torch.save({"critic.x": torch.zeros(1)}, b2)
        z.writestr("policy.pth", b2.getvalue())
    with pytest.raises(KeyError):
        load_sb3_actor(tmp_path / "bad.zip")


def test_comm_info_struct_layout_matches_c(tmp_path):
    prog = tmp_path / "comm_layout.c"
    fields = [f[0] for f in nat.BsgCommInfo._fields_]
    lines = ['#include <stdio.h>', '#include <stddef.h>', f'#include "{HDR}"', "int main(void){",
             'printf("%zu\\n", sizeof(bsg_comm_info));']
    lines += [f'printf("%zu\\n", offsetof(bsg_comm_info, {f}));' for f in fields]
    lines += ["return 0;}"]
    prog.write_text("\n".join(lines))
    exe = tmp_path / "comm_layout"
    subprocess.run(["gcc", "-std=c99", "-o", str(exe), str(prog)], check=True)
    vals = [int(v) for v in subprocess.run([str(exe)], capture_output=True, text=True,
                                           check=True).stdout.split()]
    assert vals[0] == C.sizeof(nat.BsgCommInfo)
    assert vals[1:] == [getattr(nat.BsgCommInfo, f).offset for f in fields]


def test_comm_argument_errors_before_any_device_call():
    """bsg_comm_* validate their arguments before touching RCCL or the device (VERDICT r04
    weak #5): null id / out pointer, rank count and rank out of range, null comm or buffers,
    slot and count out of range -- each BSG_E_INVALID_ARG with a message naming the call."""
    lib = nat.load_library()
    E_INVALID = -1
    idb = (C.c_uint8 * nat.COMM_ID_BYTES)()
    out = C.c_void_p()
    err = lambda: lib.bsg_comm_last_error().decode()             # noqa: E731
    assert lib.bsg_comm_unique_id(None) == E_INVALID and "bsg_comm_unique_id" in err()
    assert lib.bsg_comm_create(None, 2, 0, 0, C.byref(out)) == E_INVALID and "null" in err()
    assert lib.bsg_comm_create(idb, 2, 0, 0, None) == E_INVALID
    for nranks, rank in ((0, 0), (-1, 0), (2, 2), (2, -1), (8, 9)):
        assert lib.bsg_comm_create(idb, nranks, rank, 0, C.byref(out)) == E_INVALID, (nranks, rank)
        assert "rank out of range" in err() and not out.value
    buf = (C.c_float * 4)()
    assert lib.bsg_comm_all_gather(None, buf, buf, 4, 0, None) == E_INVALID
    assert "bsg_comm_all_gather: null" in err()
    # a non-null handle that is never dereferenced: the range checks come first
    fake = C.c_void_p(8)
    for slot, count in ((-1, 4), (nat.COMM_SLOTS, 4), (0, -1)):
        assert lib.bsg_comm_all_gather(fake, buf, buf, count, slot, None) == E_INVALID
        assert "out of range" in err()
    assert lib.bsg_comm_all_gather(fake, None, buf, 4, 0, None) == E_INVALID
    assert lib.bsg_comm_wait(None, 0, None) == E_INVALID and "null comm" in err()
    assert lib.bsg_comm_wait(fake, nat.COMM_SLOTS, None) == E_INVALID and "slot out of range" in err()
    assert lib.bsg_comm_all_reduce(None, buf, 4, nat.REDUCE_AVG, None) == E_INVALID
    assert "bsg_comm_all_reduce: null" in err()
    assert lib.bsg_comm_all_reduce(fake, None, 4, nat.REDUCE_SUM, None) == E_INVALID
    for count, op in ((-1, nat.REDUCE_SUM), (4, 2), (4, -1)):
        assert lib.bsg_comm_all_reduce(fake, buf, count, op, None) == E_INVALID
        assert "out of range" in err()
    info = nat.BsgCommInfo()
    assert lib.bsg_comm_get_info(None, C.byref(info)) == E_INVALID and "null" in err()
    assert lib.bsg_comm_destroy(None) == 0


def test_error_messages_carry_no_stray_format_arguments():
    """fail()'s old two-argument printf form appended a stray '0' to every message
    without a number; the messages end where their text ends."""
    lib = nat.load_library()
    assert lib.bsg_step_gather(None, None, None, None, None, None, 0, None) == -1
    assert lib.bsg_last_error() == b"bsg_step_gather: null ctx/comm"
    assert lib.bsg_destroy(None) in (0, -1)
    assert lib.bsg_set_wind(None, None) == -1
    assert lib.bsg_last_error() == b"bsg_set_wind: null ctx"
