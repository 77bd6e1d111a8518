"""Device policy: an SB3 SAC actor evaluated on the batch's observation rows by one fused
HIP kernel (``bsg_policy_sac``, csrc/bsg_policy.hip), writing the fp64 action rows that
``bsg_step`` reads -- the batched form of what the reference does per env with

    action, _states = model.predict(obs, deterministic=True)     # main.py:54,
                                                                 # scripts/multi_processing_example.py:70

and of the stochastic action SB3 SAC draws per collected step (``Actor.action_log_prob``,
stable_baselines3 2.x sac/policies.py; the library is not vendored in the reference).

The weights are read through device pointers on every call, so a learner that updates the
actor's parameters in place (torch optimizers do) is seen by the next call, also inside a
captured HIP graph.  The observation rows are the kernel's flat fp32 obs (sorted-key
order = SB3 MultiInputPolicy's flattening).  No CPU fallback: without libbsg.so or a HIP
device this raises.
"""
from __future__ import annotations

import ctypes as C

import numpy as np
import torch

from . import _native as nat

_KEYS = ("latent_pi.0.weight", "latent_pi.0.bias", "latent_pi.2.weight", "latent_pi.2.bias",
         "mu.weight", "mu.bias", "log_std.weight", "log_std.bias")


def load_sb3_actor(path) -> dict:
    """The actor weights of a saved SB3 SAC model (``model.save(...)`` -> ``<name>.zip``):
    ``policy.pth`` inside the archive, read with ``torch.load(weights_only=True)`` (tensors
    only; nothing in the file is executed), keys ``actor.*`` with the prefix removed.  The
    archive's pickled ``data`` member is never read."""
    import io
    import zipfile
    with zipfile.ZipFile(path) as z:
        with z.open("policy.pth") as f:
            sd = torch.load(io.BytesIO(f.read()), map_location="cpu", weights_only=True)
    w = {k[len("actor."):]: v for k, v in sd.items() if k.startswith("actor.")}
    missing = [k for k in _KEYS if k not in w]
    if missing:
        raise KeyError(f"{path}: no SAC actor weights {missing} in policy.pth")
    return {k: w[k] for k in _KEYS}


class SACPolicy:
    """SAC actor (net_arch [256, 256]) on the device.

    ``weights`` maps SB3's actor parameter names (``latent_pi.0.weight`` ...; an ``actor.``
    prefix is accepted) to arrays or tensors; they are copied to fp32 device tensors.
    ``from_module`` instead shares the parameters of a live torch actor (no copy)."""

    def __init__(self, weights, device="cuda"):
        dev = torch.device(device)
        if dev.type != "cuda":
            raise nat.BsgError("SACPolicy runs on a HIP device (no CPU fallback)")
        if dev.index is None:                     # "cuda" -> the current device, as tensors report it
            dev = torch.device("cuda", torch.cuda.current_device())
        w = {k[len("actor."):] if k.startswith("actor.") else k: v for k, v in weights.items()}
        missing = [k for k in _KEYS if k not in w]
        if missing:
            raise KeyError(f"SACPolicy: missing actor weights {missing}")
        self._t = [torch.as_tensor(np.asarray(w[k]) if not torch.is_tensor(w[k]) else w[k])
                   .to(device=dev, dtype=torch.float32).contiguous() for k in _KEYS]
        self._setup(dev)

    @classmethod
    def from_npz(cls, path, tag, device="cuda"):
        """Weights from an .npz holding ``{tag}/{name}`` arrays (tests/golden/sac_actors.npz:
        the reference's saved SAC actors, extracted weights-only)."""
        with np.load(path) as z:
            return cls({k: z[f"{tag}/{k}"] for k in _KEYS}, device)

    @classmethod
    def from_sb3_zip(cls, path, device="cuda"):
        """The actor of a saved SB3 SAC model (the reference's ``model.save`` archives,
        e.g. ``scripts/common/results/models_backup/*/model.zip``), weights only."""
        return cls(load_sb3_actor(path), device)

    @classmethod
    def from_module(cls, actor):
        """Share the parameters of a torch actor with ``latent`` (Linear, ReLU, Linear,
        ReLU), ``mu`` and ``log_std`` Linear layers (tools/sac_torch.Actor)."""
        self = cls.__new__(cls)
        ps = [actor.latent[0].weight, actor.latent[0].bias, actor.latent[2].weight,
              actor.latent[2].bias, actor.mu.weight, actor.mu.bias, actor.log_std.weight,
              actor.log_std.bias]
        for p in ps:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device.type != "cuda":
                raise nat.BsgError("SACPolicy.from_module: parameters must be contiguous fp32 "
                                   "on a HIP device")
        self._t = [p.detach() for p in ps]
        self._setup(ps[0].device)
        return self

    def _setup(self, dev):
        t = self._t
        hidden, obs_dim = t[0].shape
        act_dim = t[4].shape[0]
        shapes = [(hidden, obs_dim), (hidden,), (hidden, hidden), (hidden,), (act_dim, hidden),
                  (act_dim,), (act_dim, hidden), (act_dim,)]
        for k, x, s in zip(_KEYS, t, shapes):
            if tuple(x.shape) != s:
                raise ValueError(f"SACPolicy: {k} has shape {tuple(x.shape)}, expected {s}")
        self.device, self.obs_dim, self.act_dim, self.hidden = dev, int(obs_dim), int(act_dim), int(hidden)
        self._lib = nat.load_library()
        self._w = nat.BsgSacActor(self.obs_dim, self.act_dim, self.hidden, 0,
                                  *[x.data_ptr() for x in t])

    def __call__(self, obs: torch.Tensor, eps: torch.Tensor | None = None, *,
                 out: torch.Tensor | None = None, log_prob: torch.Tensor | None = None) -> torch.Tensor:
        """Actions [E, act_dim] fp64 for fp32 obs rows [E, >= obs_dim] (row stride = obs's).
        ``eps``: fp32 [E, act_dim] standard normals (stochastic SAC sample) or None
        (deterministic, tanh(mu)).  ``log_prob``: optional fp32 [E] output."""
        E = self._check(obs, eps, out, log_prob)
        if out is None:
            out = torch.empty((E, self.act_dim), dtype=torch.float64, device=self.device)
        if E == 0:
            return out
        ptr = lambda x: None if x is None else C.c_void_p(x.data_ptr())  # noqa: E731
        with torch.cuda.device(self.device):       # the launch goes to the policy's device
            stream = C.c_void_p(torch.cuda.current_stream(self.device).cuda_stream)
            nat.check(self._lib.bsg_policy_sac(C.byref(self._w), ptr(obs), E, obs.stride(0),
                                               ptr(eps), ptr(out), ptr(log_prob), stream),
                      "bsg_policy_sac")
        return out

    def _check(self, obs, eps, out, log_prob) -> int:
        """Every tensor the kernel reads or writes by raw pointer: dtype, shape, layout and
        device (the kernel reads obs_dim floats per row at obs.stride(0) and writes out /
        log_prob at unit stride)."""
        dev = self.device
        if obs.dtype != torch.float32 or obs.dim() != 2 or obs.stride(1) != 1 or obs.device != dev:
            raise ValueError("SACPolicy: obs must be fp32 [E, D] rows (unit column stride) on the "
                             "policy's device")
        if obs.shape[1] < self.obs_dim:
            raise ValueError(f"SACPolicy: obs rows hold {obs.shape[1]} features, the actor reads "
                             f"{self.obs_dim}")
        E = obs.shape[0]
        if out is not None and (out.dtype != torch.float64 or tuple(out.shape) != (E, self.act_dim)
                                or not out.is_contiguous() or out.device != dev):
            raise ValueError("SACPolicy: out must be contiguous fp64 [E, act_dim] on the policy's "
                             "device")
        if eps is not None and (eps.dtype != torch.float32 or tuple(eps.shape) != (E, self.act_dim)
                                or not eps.is_contiguous() or eps.device != dev):
            raise ValueError("SACPolicy: eps must be contiguous fp32 [E, act_dim] on the policy's "
                             "device")
        if log_prob is not None and (log_prob.dtype != torch.float32 or tuple(log_prob.shape) != (E,)
                                     or not log_prob.is_contiguous() or log_prob.device != dev):
            raise ValueError("SACPolicy: log_prob must be contiguous fp32 [E] on the policy's device")
        return E

    def predict(self, obs: torch.Tensor, deterministic: bool = True, generator=None):
        """SB3's ``predict`` shape: (actions, None)."""
        eps = None if deterministic else torch.randn(
            (obs.shape[0], self.act_dim), dtype=torch.float32, device=self.device, generator=generator)
        return self(obs, eps), None
