"""Soft Actor-Critic in plain torch, on the device that holds the env batch -- the learner
of BASELINE configs[4] ("DescentEnv-v0 + SB3 SAC learner, 4096 envs"), for measuring
end-to-end RL throughput with the MI355X env path (bench.py --workload descent-sac).

stable-baselines3 is not installed here; this restates the part of SB3 2.x SAC that runs
per environment step with the hyper-parameters of the reference's training script
(scripts/descent_env_sac.py:25-34 -> SB3 defaults): MultiInputPolicy (the Dict obs
flattened in sorted-key order = the kernel's flat rows), actor and twin critics
Linear-ReLU 256-256, squashed Gaussian with log_std clamped to [-20, 2], Adam (lr 1e-3 in
the reference script, descent_env_sac.py:29),
batch 256, buffer 1e6, gamma 0.99, tau 0.005, entropy coefficient 'auto' (target
entropy -dim(A)), train_freq 1 / gradient_steps 1 -- one gradient step per vector step.

The twin critics are one TwinQ (weights stacked, one batched GEMM per layer for both).

Per iteration: sample actions for every env (actor forward) -> one env step on the
device (SAME_STEP autoreset, terminal obs from final_obs as SB3's VecEnv gives it) ->
insert the E transitions into a device ring buffer -> one SAC update.  The whole
iteration is captured once as a HIP graph (torch.cuda.graph; the env kernel is launched
on the capture stream through the C ABI), so a step costs one graph launch instead of
~60 small kernel launches.  With torch.distributed initialised, each rank learns on its
env shard's buffer and the gradients are all-reduced (RCCL) before the optimizer step --
data-parallel SAC with the per-rank batch 256 / world.
"""
from __future__ import annotations

import ctypes
import math
import os

import torch
import torch.nn as nn
import torch.nn.functional as F

LOG_STD_MIN, LOG_STD_MAX = -20.0, 2.0
_HERE = os.path.dirname(os.path.abspath(__file__))
ADAM_LIB = os.path.join(_HERE, "_lib", "libsacadam.so")
_MAXT = 16


class _AdamTable(ctypes.Structure):
    _fields_ = [("n", ctypes.c_int32), ("start", ctypes.c_int32 * (_MAXT + 1)),
                ("numel", ctypes.c_int64 * _MAXT), ("p", ctypes.c_void_p * _MAXT),
                ("g", ctypes.c_void_p * _MAXT), ("m", ctypes.c_void_p * _MAXT),
                ("v", ctypes.c_void_p * _MAXT)]


class HipAdam:
    """torch.optim.Adam (lr, betas (0.9, 0.999), eps 1e-8; no weight decay / amsgrad) over
    several parameter groups, one launch of tools/sac_adam.hip per step() instead of one
    torch fused-Adam launch per group at ~28 us each.  The step count t lives on the device
    and is advanced by tick() (once per update: every group here steps once per update), so
    the whole update can be captured in a HIP graph.  Gradients are read at step() time from
    p.grad (set_to_none gradients included: the pointers are taken at launch/capture)."""

    _lib = None

    def __init__(self, params, lr, betas=(0.9, 0.999), eps=1e-8, step=None, targets=None, tau=0.0):
        if HipAdam._lib is None:
            if not os.path.exists(ADAM_LIB):
                raise RuntimeError(f"{ADAM_LIB} missing: run __graft_entry__.build()")
            lib = ctypes.CDLL(ADAM_LIB)
            lib.sac_adam_step.restype = ctypes.c_int32
            lib.sac_adam_step.argtypes = [ctypes.POINTER(_AdamTable), ctypes.c_void_p, ctypes.c_float,
                                          ctypes.c_float, ctypes.c_float, ctypes.c_float, ctypes.c_void_p]
            lib.sac_adam_step_polyak.restype = ctypes.c_int32
            lib.sac_adam_step_polyak.argtypes = [ctypes.POINTER(_AdamTable), ctypes.c_void_p, ctypes.c_float,
                                                 ctypes.c_float, ctypes.c_float, ctypes.c_float,
                                                 ctypes.c_void_p * _MAXT, ctypes.c_float, ctypes.c_void_p]
            lib.sac_replay_insert.restype = ctypes.c_int32
            lib.sac_replay_insert.argtypes = ([ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int32,
                                               ctypes.c_int32] + [ctypes.c_void_p] * 7 +
                                              [ctypes.c_int32] + [ctypes.c_void_p] * 4)
            lib.sac_replay_insert_obs.restype = ctypes.c_int32
            lib.sac_replay_insert_obs.argtypes = ([ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int32,
                                                   ctypes.c_int32] + [ctypes.c_void_p] * 7 +
                                                  [ctypes.c_int32] + [ctypes.c_void_p] * 5)
            lib.sac_replay_sample.restype = ctypes.c_int32
            lib.sac_replay_sample.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int32,
                                              ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                              ctypes.c_void_p, ctypes.c_void_p]
            lib.sac_replay_sample_tick.restype = ctypes.c_int32
            lib.sac_replay_sample_tick.argtypes = [ctypes.c_void_p, ctypes.c_longlong, ctypes.c_int32,
                                                   ctypes.c_void_p, ctypes.c_int32, ctypes.c_void_p,
                                                   ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            lib.sac_td_target.restype = ctypes.c_int32
            lib.sac_td_target.argtypes = ([ctypes.c_void_p] * 4 + [ctypes.c_int32] * 3 +
                                          [ctypes.c_float, ctypes.c_int32, ctypes.c_void_p, ctypes.c_void_p])
            lib.sac_twin_mse_fwd.restype = ctypes.c_int32
            lib.sac_twin_mse_fwd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                             ctypes.c_void_p, ctypes.c_void_p, ctypes.c_void_p]
            lib.sac_twin_mse_bwd.restype = ctypes.c_int32
            lib.sac_twin_mse_bwd.argtypes = [ctypes.c_void_p, ctypes.c_void_p, ctypes.c_int32,
                                             ctypes.c_void_p, ctypes.c_void_p]
            lib.sac_actor_loss_fwd.restype = ctypes.c_int32
            lib.sac_actor_loss_fwd.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int32] + [ctypes.c_void_p] * 2
            lib.sac_actor_loss_bwd.restype = ctypes.c_int32
            lib.sac_actor_loss_bwd.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int32] + [ctypes.c_void_p] * 3
            lib.sac_sq_gauss_fwd.restype = ctypes.c_int32
            lib.sac_sq_gauss_fwd.argtypes = [ctypes.c_void_p] * 3 + [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 3
            lib.sac_sq_gauss_bwd.restype = ctypes.c_int32
            lib.sac_sq_gauss_bwd.argtypes = [ctypes.c_void_p] * 6 + [ctypes.c_int32] * 2 + [ctypes.c_void_p] * 3
            HipAdam._lib = lib
        self.params = list(params)
        if len(self.params) > _MAXT:
            raise ValueError("HipAdam: at most 16 tensors")
        for p in self.params:
            if p.dtype != torch.float32 or not p.is_contiguous() or p.device.type != "cuda":
                raise ValueError("HipAdam: contiguous fp32 device parameters only")
        self.m = [torch.zeros_like(p) for p in self.params]
        self.v = [torch.zeros_like(p) for p in self.params]
        self.lr, self.b1, self.b2, self.eps = float(lr), float(betas[0]), float(betas[1]), float(eps)
        self.t = step if step is not None else torch.zeros((), dtype=torch.float32,
                                                             device=self.params[0].device)
        # targets: a target copy per parameter, polyak-updated in the same launch behind the
        # parameter's Adam step (target = target (1 - tau) + tau p_new, SB3's polyak_update)
        self.targets, self.tau = None, float(tau)
        if targets is not None:
            targets = list(targets)
            if len(targets) != len(self.params) or any(
                    t.shape != p.shape or t.dtype != p.dtype or not t.is_contiguous()
                    for t, p in zip(targets, self.params)):
                raise ValueError("HipAdam: one contiguous target per parameter, of its shape")
            self.targets = targets

    def tick(self):
        self.t.add_(1.0)

    def zero_grad(self, set_to_none=True):
        for p in self.params:
            p.grad = None

    def step(self):
        T = _AdamTable()
        T.n = len(self.params)
        acc = 0
        T.start[0] = 0
        for i, (p, m, v) in enumerate(zip(self.params, self.m, self.v)):
            g = p.grad
            if g is None or not g.is_contiguous():
                raise RuntimeError("HipAdam: every parameter needs a contiguous gradient")
            T.numel[i] = p.numel()
            acc += (p.numel() + 255) // 256
            T.start[i + 1] = acc
            T.p[i], T.g[i], T.m[i], T.v[i] = p.data_ptr(), g.data_ptr(), m.data_ptr(), v.data_ptr()
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.params[0].device).cuda_stream)
        if self.targets is not None:
            tg = (ctypes.c_void_p * _MAXT)(*[t.data_ptr() for t in self.targets])
            rc = self._lib.sac_adam_step_polyak(ctypes.byref(T), ctypes.c_void_p(self.t.data_ptr()),
                                                self.lr, self.b1, self.b2, self.eps, tg, self.tau, stream)
        else:
            rc = self._lib.sac_adam_step(ctypes.byref(T), ctypes.c_void_p(self.t.data_ptr()), self.lr,
                                         self.b1, self.b2, self.eps, stream)
        if rc != 0:
            raise RuntimeError(f"sac_adam_step failed ({rc})")


def mlp(i, o, h=256):
    return nn.Sequential(nn.Linear(i, h), nn.ReLU(), nn.Linear(h, h), nn.ReLU(), nn.Linear(h, o))


class SquashedGaussian(torch.autograd.Function):
    """(tanh(u), log_prob) of SB3's squashed Gaussian from (mu, raw log_std, eps) as one
    forward and one backward launch of tools/sac_adam.hip (Actor.forward's torch form is
    ~13 kernels each way)."""

    @staticmethod
    def forward(ctx, mu, lsr, eps):
        mu, lsr, eps = mu.contiguous(), lsr.contiguous(), eps.contiguous()
        N, A = mu.shape
        a = torch.empty_like(mu)
        lp = torch.empty((N,), device=mu.device, dtype=mu.dtype)
        st = ctypes.c_void_p(torch.cuda.current_stream(mu.device).cuda_stream)
        p = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        if HipAdam._lib.sac_sq_gauss_fwd(p(mu), p(lsr), p(eps), N, A, p(a), p(lp), st) != 0:
            raise RuntimeError("sac_sq_gauss_fwd failed")
        ctx.save_for_backward(mu, lsr, eps, a)
        return a, lp

    @staticmethod
    def backward(ctx, ga, gl):
        mu, lsr, eps, a = ctx.saved_tensors
        N, A = mu.shape
        gmu, glsr = torch.empty_like(mu), torch.empty_like(lsr)
        ga = ga.contiguous() if ga is not None else None
        gl = gl.contiguous() if gl is not None else None
        st = ctypes.c_void_p(torch.cuda.current_stream(mu.device).cuda_stream)
        p = lambda t: None if t is None else ctypes.c_void_p(t.data_ptr())  # noqa: E731
        if HipAdam._lib.sac_sq_gauss_bwd(p(mu), p(lsr), p(eps), p(a), p(ga), p(gl), N, A, p(gmu),
                                         p(glsr), st) != 0:
            raise RuntimeError("sac_sq_gauss_bwd failed")
        return gmu, glsr, None


class Actor(nn.Module):
    def __init__(self, obs_dim, act_dim, h=256):
        super().__init__()
        self.latent = nn.Sequential(nn.Linear(obs_dim, h), nn.ReLU(), nn.Linear(h, h), nn.ReLU())
        self.mu = nn.Linear(h, act_dim)
        self.log_std = nn.Linear(h, act_dim)

    fused_dist = False       # SquashedGaussian launches (set by SAC on the HIP path)

    def forward(self, obs):
        """(tanh-squashed sample, log-prob) of the SB3 squashed diagonal Gaussian."""
        h = self.latent(obs)
        mu = self.mu(h)
        if self.fused_dist:
            lsr = self.log_std(h)
            return SquashedGaussian.apply(mu, lsr, torch.randn_like(mu))
        log_std = torch.clamp(self.log_std(h), LOG_STD_MIN, LOG_STD_MAX)
        std = log_std.exp()
        u = mu + std * torch.randn_like(mu)
        a = torch.tanh(u)
        logp = (-0.5 * ((u - mu) / std) ** 2 - log_std - 0.5 * math.log(2 * math.pi)).sum(-1)
        logp = logp - torch.log(1 - a * a + 1e-6).sum(-1)
        return a, logp

    def load_sb3(self, W, tag):
        """Weights of the reference's saved SB3 actor (tests/golden/sac_actors.npz)."""
        g = lambda k: torch.as_tensor(W[f"{tag}/{k}"])  # noqa: E731
        with torch.no_grad():
            self.latent[0].weight.copy_(g("latent_pi.0.weight")); self.latent[0].bias.copy_(g("latent_pi.0.bias"))
            self.latent[2].weight.copy_(g("latent_pi.2.weight")); self.latent[2].bias.copy_(g("latent_pi.2.bias"))
            self.mu.weight.copy_(g("mu.weight")); self.mu.bias.copy_(g("mu.bias"))
            self.log_std.weight.copy_(g("log_std.weight")); self.log_std.bias.copy_(g("log_std.bias"))


class TwinMSE(torch.autograd.Function):
    """(q - y).pow(2).mean(-1).sum() for q [2, B], y [B] (no grad) as one forward and one
    backward launch of tools/sac_adam.hip; the gradient is bit-identical to torch's."""

    @staticmethod
    def forward(ctx, q, y):
        q, y = q.contiguous(), y.contiguous()
        B = y.shape[0]
        diff = torch.empty_like(q)
        loss = torch.empty((), device=q.device, dtype=q.dtype)
        st = ctypes.c_void_p(torch.cuda.current_stream(q.device).cuda_stream)
        if HipAdam._lib.sac_twin_mse_fwd(ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(y.data_ptr()), B,
                                         ctypes.c_void_p(diff.data_ptr()), ctypes.c_void_p(loss.data_ptr()),
                                         st) != 0:
            raise RuntimeError("sac_twin_mse_fwd failed")
        ctx.save_for_backward(diff)
        return loss

    @staticmethod
    def backward(ctx, g):
        (diff,) = ctx.saved_tensors
        g = g.contiguous()
        dq = torch.empty_like(diff)
        st = ctypes.c_void_p(torch.cuda.current_stream(diff.device).cuda_stream)
        if HipAdam._lib.sac_twin_mse_bwd(ctypes.c_void_p(diff.data_ptr()), ctypes.c_void_p(g.data_ptr()),
                                         diff.shape[1], ctypes.c_void_p(dq.data_ptr()), st) != 0:
            raise RuntimeError("sac_twin_mse_bwd failed")
        return dq, None


class ActorLoss(torch.autograd.Function):
    """(alpha * logp - q.amin(0)).mean() for q [2, B], logp [B], alpha a detached 0-dim
    tensor, as one forward and one backward launch of tools/sac_adam.hip."""

    @staticmethod
    def forward(ctx, q, logp, alpha):
        q, logp = q.contiguous(), logp.contiguous()
        B = logp.shape[0]
        loss = torch.empty((), device=q.device, dtype=q.dtype)
        st = ctypes.c_void_p(torch.cuda.current_stream(q.device).cuda_stream)
        if HipAdam._lib.sac_actor_loss_fwd(ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(logp.data_ptr()),
                                           ctypes.c_void_p(alpha.data_ptr()), B,
                                           ctypes.c_void_p(loss.data_ptr()), st) != 0:
            raise RuntimeError("sac_actor_loss_fwd failed")
        ctx.save_for_backward(q, alpha)
        return loss

    @staticmethod
    def backward(ctx, g):
        q, alpha = ctx.saved_tensors
        g = g.contiguous()
        B = q.shape[1]
        dq = torch.empty_like(q)
        dlogp = torch.empty((B,), device=q.device, dtype=q.dtype)
        st = ctypes.c_void_p(torch.cuda.current_stream(q.device).cuda_stream)
        if HipAdam._lib.sac_actor_loss_bwd(ctypes.c_void_p(q.data_ptr()), ctypes.c_void_p(alpha.data_ptr()),
                                           ctypes.c_void_p(g.data_ptr()), B, ctypes.c_void_p(dq.data_ptr()),
                                           ctypes.c_void_p(dlogp.data_ptr()), st) != 0:
            raise RuntimeError("sac_actor_loss_bwd failed")
        return dq, dlogp, None


class TwinQ(nn.Module):
    """SB3's twin critics (two Linear-ReLU 256-256 MLPs over [obs, act], each initialised as
    nn.Linear does) with their weights stacked on a leading axis of 2: every layer is one
    batched GEMM for both critics (baddbmm) and every elementwise op, reduction and their
    backward run once on [2, B, .] -- half the launches of two separate critics, which is
    what a batch-256 update costs (a few microseconds per kernel).  forward -> [2, B]."""

    def __init__(self, i, h=256):
        super().__init__()
        a, b = mlp(i, 1, h), mlp(i, 1, h)
        w = lambda k: nn.Parameter(torch.stack([a[k].weight.detach().t(), b[k].weight.detach().t()]).contiguous())  # noqa: E731
        c = lambda k: nn.Parameter(torch.stack([a[k].bias.detach(), b[k].bias.detach()])[:, None, :].contiguous())  # noqa: E731
        self.w0, self.w1, self.w2 = w(0), w(2), w(4)
        self.b0, self.b1, self.b2 = c(0), c(2), c(4)

    def forward(self, x):
        h = torch.relu(torch.baddbmm(self.b0, x.expand(2, *x.shape), self.w0))
        h = torch.relu(torch.baddbmm(self.b1, h, self.w1))
        return torch.baddbmm(self.b2, h, self.w2).squeeze(-1)


class QView(nn.Module):
    """Critic `idx` of a TwinQ as a module (forward -> [B, 1]); parameters() are the shared
    stacked tensors (not registered here, so an optimizer over the TwinQ sees them once)."""

    def __init__(self, twin, idx):
        super().__init__()
        object.__setattr__(self, "_twin", twin)
        self.idx = idx

    def forward(self, x):
        return self._twin(x)[self.idx][:, None]

    def parameters(self, recurse=True):
        return self._twin.parameters(recurse)


class SAC:
    def __init__(self, obs_dim, act_dim, device, *, lr=3e-4, batch=256, buffer=1_000_000,
                 gamma=0.99, tau=0.005, group=None, seed=0, comm=None):
        """group: the data-parallel process group (None: one rank).  comm: an object with
        all_reduce(t, avg) -- bluesky_gym.parallel.RcclGather, libbsg's RCCL communicator --
        that reduces the gradients on the current stream (graph-capturable; also at one rank,
        where it is the identity); without it several ranks reduce through torch.distributed
        (eager).  seed: this rank's sampling seed (replay draws, noise); the parameters are
        those of rank 0, broadcast over `group` (every rank starts from the same networks)."""
        torch.manual_seed(seed)
        self.dev = torch.device(device)
        self.actor = Actor(obs_dim, act_dim).to(self.dev)
        self.q = TwinQ(obs_dim + act_dim).to(self.dev)
        self.qt = TwinQ(obs_dim + act_dim).to(self.dev)
        self.qt.load_state_dict(self.q.state_dict())
        self.q1, self.q2 = QView(self.q, 0), QView(self.q, 1)
        self.log_alpha = torch.zeros(1, device=self.dev, requires_grad=True)
        self.target_entropy = -float(act_dim)
        # fused Adam: one kernel per parameter group instead of a foreach chain per tensor
        # (the update is launch-bound: batch 256 through 256-wide MLPs)
        # hip: tools/sac_adam.hip (one launch per step over every tensor of the groups that
        # step together); fused | foreach: torch's Adam (A/B; the CPU tests use torch's)
        impl = os.environ.get("SAC_ADAM", "hip" if self.dev.type == "cuda" else "torch")
        self.hip_adam = impl == "hip"
        # SB3's squashed Gaussian as one launch each way (on by default once the whole-update
        # equivalence test, tests/test_gpu_sac_adam.py, covers it; SAC_FUSED_DIST=0 = autograd)
        self.actor.fused_dist = self.hip_adam and os.environ.get("SAC_FUSED_DIST", "1") == "1"
        if self.hip_adam:
            t = torch.zeros((), dtype=torch.float32, device=self.dev)
            self.opt_q = HipAdam(self.q.parameters(), lr, step=t)
            # the actor and the entropy coefficient step back to back: one launch for both
            self.opt_a = HipAdam(list(self.actor.parameters()) + [self.log_alpha], lr, step=t)
            self.opt_al = None
        else:
            opt = dict(lr=lr, capturable=True, **{impl: True}) if self.dev.type == "cuda" else dict(lr=lr)
            self.opt_a = torch.optim.Adam(self.actor.parameters(), **opt)
            self.opt_q = torch.optim.Adam(self.q.parameters(), **opt)
            self.opt_al = torch.optim.Adam([self.log_alpha], **opt)
        self.gamma, self.tau = gamma, tau
        self.group = group
        self.comm = comm
        world = torch.distributed.get_world_size(group) if group is not None else 1
        if comm is not None and group is None:
            world = int(getattr(comm, "world", 1))
        self.world = world
        if group is not None and world > 1:
            # data-parallel SAC: one set of networks.  Each rank seeded its own (seed = its
            # sampling seed), so rank 0's are broadcast before any step
            src = torch.distributed.get_global_rank(group, 0)
            with torch.no_grad():
                for t in (list(self.actor.parameters()) + list(self.q.parameters()) +
                          list(self.qt.parameters()) + [self.log_alpha]):
                    torch.distributed.broadcast(t.data, src=src, group=group)
        self.batch = max(1, batch // world)
        self.cap = buffer // world
        d = self.dev
        # one packed row per transition [obs | act | rew | next_obs | done]: an insert is one
        # index_copy and a sample one gather (the named buffers are column views)
        self.buf = torch.zeros((self.cap, 2 * obs_dim + act_dim + 2), device=d)
        o0, o1 = 0, obs_dim
        self.buf_obs = self.buf[:, o0:o1]
        self.buf_act = self.buf[:, o1:o1 + act_dim]
        self.buf_rew = self.buf[:, o1 + act_dim]
        self.buf_next = self.buf[:, o1 + act_dim + 1:o1 + act_dim + 1 + obs_dim]
        self.buf_done = self.buf[:, -1]
        self.od, self.ad = obs_dim, act_dim
        self.pos = torch.zeros((), dtype=torch.long, device=d)
        self.size = torch.zeros((), dtype=torch.long, device=d)

    # -------------------------------------------------------------- replay buffer
    def insert(self, obs, act, rew, next_obs, term):
        n = obs.shape[0]
        idx = (self.pos + torch.arange(n, device=self.dev)) % self.cap
        row = torch.cat([obs.to(self.buf.dtype), act.to(self.buf.dtype), rew.to(self.buf.dtype)[:, None],
                         next_obs.to(self.buf.dtype), term.to(self.buf.dtype)[:, None]], -1)
        self.buf.index_copy_(0, idx, row)
        self.pos.copy_((self.pos + n) % self.cap)
        self.size.copy_(torch.clamp(self.size + n, max=self.cap))

    def insert_step(self, obs, act, batch, obs_out=None):
        """The E transitions of one SAME_STEP vector step (obs before the step, fp64 actions,
        the batch's reward / terminated / truncated / obs / final_obs) in one launch of
        tools/sac_adam.hip's replay insert; the same rows and pos/size as insert() with
        next_obs = final_obs where terminated | truncated and done = terminated."""
        if not hasattr(self, "_ticket"):
            self._ticket = torch.zeros((), dtype=torch.int32, device=self.dev)
            HipAdam([torch.zeros(1, device=self.dev)], 0.0)      # loads the library
        E = obs.shape[0]
        for t, dt in ((obs, torch.float32), (act, torch.float64), (batch.reward, torch.float32),
                      (batch.terminated, torch.uint8), (batch.truncated, torch.uint8),
                      (batch.obs, torch.float32), (batch.final_obs, torch.float32)):
            if t.dtype != dt or not t.is_contiguous() or t.shape[0] != E:
                raise ValueError("insert_step: unexpected tensor layout")
        ptr = lambda t: ctypes.c_void_p(t.data_ptr())  # noqa: E731
        stream = ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream)
        if obs_out is not None:
            # (and obs_out <- batch.obs in the same launch: RLLoop's copy of the new observations)
            if obs_out.dtype != torch.float32 or not obs_out.is_contiguous() or obs_out.shape != obs.shape:
                raise ValueError("insert_step: obs_out must be an fp32 tensor of obs's shape")
            rc = HipAdam._lib.sac_replay_insert_obs(
                ptr(self.buf), self.cap, self.od, self.ad, ptr(obs), ptr(act), ptr(batch.reward),
                ptr(batch.terminated), ptr(batch.truncated), ptr(batch.obs), ptr(batch.final_obs), E,
                ptr(self.pos), ptr(self.size), ptr(self._ticket), ptr(obs_out), stream)
        else:
            rc = HipAdam._lib.sac_replay_insert(
                ptr(self.buf), self.cap, self.od, self.ad, ptr(obs), ptr(act), ptr(batch.reward),
                ptr(batch.terminated), ptr(batch.truncated), ptr(batch.obs), ptr(batch.final_obs), E,
                ptr(self.pos), ptr(self.size), ptr(self._ticket), stream)
        if rc != 0:
            raise RuntimeError(f"sac_replay_insert failed ({rc})")

    def sample(self):
        u = torch.rand(self.batch, device=self.dev)
        if self.hip_adam:
            # the gather below as one launch of tools/sac_adam.hip (same index arithmetic)
            if not hasattr(self, "_rows"):
                self._rows = torch.empty((self.batch, self.buf.shape[1]), device=self.dev)
                HipAdam([torch.zeros(1, device=self.dev)], 0.0)  # loads the library
            t = self._rows
            rc = HipAdam._lib.sac_replay_sample(
                ctypes.c_void_p(self.buf.data_ptr()), self.cap, self.buf.shape[1],
                ctypes.c_void_p(u.data_ptr()), self.batch, ctypes.c_void_p(self.size.data_ptr()),
                ctypes.c_void_p(t.data_ptr()),
                ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream))
            if rc != 0:
                raise RuntimeError(f"sac_replay_sample failed ({rc})")
        else:
            idx = torch.clamp((u * self.size.float()).long(), max=self.cap - 1)
            t = self.buf[idx]
        od, ad = self.od, self.ad
        return (t[:, :od], t[:, od:od + ad], t[:, od + ad], t[:, od + ad + 1:2 * od + ad + 1], t[:, -1])

    def _td_target(self, q2, ll, alpha):
        """r + gamma (1 - d) (min(q_t) - alpha logp') in one launch (tools/sac_adam.hip),
        bit-identical to the torch expression; r, d from the sampled rows (self._rows), logp'
        the first B entries of the actor pass's log-probs."""
        B = self.batch
        if not hasattr(self, "_y"):
            self._y = torch.empty(B, device=self.dev)
        q2 = q2.contiguous()
        W = self._rows.shape[1]
        rc = HipAdam._lib.sac_td_target(
            ctypes.c_void_p(q2.data_ptr()), ctypes.c_void_p(ll.data_ptr()), ctypes.c_void_p(alpha.data_ptr()),
            ctypes.c_void_p(self._rows.data_ptr()), W, self.od + self.ad, W - 1, self.gamma, B,
            ctypes.c_void_p(self._y.data_ptr()), ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream))
        if rc != 0:
            raise RuntimeError(f"sac_td_target failed ({rc})")
        return self._y

    # -------------------------------------------------------------- SAC update
    def _reduce_flat(self, flat):
        """flat <- the mean over the ranks (in place)"""
        if self.comm is not None:
            self.comm.all_reduce(flat, avg=True)
        elif self.world > 1:
            torch.distributed.all_reduce(flat, group=self.group)
            flat /= self.world

    def _allreduce(self, params):
        if self.world == 1 and self.comm is None:
            return
        grads = [p.grad for p in params if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        self._reduce_flat(flat)
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    def update(self, losses=True):
        """One SAC gradient step; returns (critic loss, actor loss) as device scalars."""
        o, a, r, o2, d = self.sample()
        alpha = self.log_alpha.exp().detach()
        # the actor's two evaluations of the update (next obs for the target, obs for the
        # actor loss) in one pass: its parameters do not change in between (its optimizer
        # steps after both); the target half is detached
        B = o.shape[0]
        aa, ll = self.actor(torch.cat([o2, o]))
        with torch.no_grad():
            a2, logp2 = aa[:B].detach(), ll[:B].detach()
            x2 = torch.cat([o2, a2], -1)
            if self.hip_adam:
                y = self._td_target(self.qt(x2), ll, alpha)
            else:
                qt = self.qt(x2).amin(0) - alpha * logp2
                y = r + self.gamma * (1.0 - d) * qt
        x = torch.cat([o, a], -1)
        # F.mse_loss(q1, y) + F.mse_loss(q2, y)
        lq = TwinMSE.apply(self.q(x), y) if self.hip_adam else (self.q(x) - y).pow(2).mean(-1).sum()
        if self.hip_adam:
            self.opt_q.tick()                     # shared step count: every group steps once
        self.opt_q.zero_grad(set_to_none=True)
        lq.backward()
        self._allreduce(list(self.q.parameters()))
        self.opt_q.step()
        ap, logp = aa[B:], ll[B:]
        xp = torch.cat([o, ap], -1)
        # the critics only pass the actor loss's gradient through: SB3 lets it land on
        # their .grad too (cleared before their next step); freezing them skips that work
        for p_ in self.q.parameters():
            p_.requires_grad_(False)
        la = ActorLoss.apply(self.q(xp), logp, alpha) if self.hip_adam else \
            (alpha * logp - self.q(xp).amin(0)).mean()
        self.opt_a.zero_grad(set_to_none=True)
        la.backward()
        for p_ in self.q.parameters():
            p_.requires_grad_(True)
        self._allreduce(list(self.actor.parameters()))
        if not self.hip_adam:
            self.opt_a.step()
        lal = -(self.log_alpha * (logp.detach() + self.target_entropy)).mean()
        if self.hip_adam:
            self.log_alpha.grad = None
        else:
            self.opt_al.zero_grad(set_to_none=True)
        lal.backward()
        self._allreduce([self.log_alpha])
        if self.hip_adam:
            self.opt_a.step()                     # actor + log_alpha in one launch
        else:
            self.opt_al.step()
        with torch.no_grad():
            # SB3 polyak_update (target * (1 - tau), then + tau * param), as two multi-tensor
            # kernels over all target parameters instead of two kernels per tensor
            src = list(self.q.parameters())
            tgt = list(self.qt.parameters())
            torch._foreach_mul_(tgt, 1.0 - self.tau)
            torch._foreach_add_(tgt, src, alpha=self.tau)
        return lq.detach(), la.detach()


FUSED_LIB = os.environ.get("SAC_FUSED_LIB", os.path.join(_HERE, "_lib", "libsacfused.so"))


class FusedSAC(SAC):
    """SAC.update with its forward and backward passes written out (one rank, the HIP path):
    the 256 x 256 products are MFMA launches of tools/sac_fused.hip gemm256_kernel (SAC_GEMM=blas:
    rocBLAS, torch.mm / bmm into preallocated outputs) and
    everything between two GEMMs is one launch of tools/sac_fused.hip -- 19 launches per
    update instead of autograd's ~100, each of which paid the dependent-kernel boundary.
    Same parameters, replay buffer, HipAdam optimizers, step count and RNG draws (torch.rand
    for the sample, torch.randn for the squashed Gaussian, in SAC.update's order), so an
    update equals SAC.update's to fp32 rounding (tests/test_gpu_sac_adam.py).  Parameter
    gradients live in persistent .grad buffers the kernels overwrite; every buffer is
    preallocated, so the update is graph-capturable."""

    _lib = None

    def __init__(self, obs_dim, act_dim, device, noise=None, **kw):
        super().__init__(obs_dim, act_dim, device, **kw)
        # noise: "philox" = the update's uniforms and normals (and an attached action sample's)
        # from one launch of tools/sac_fused.hip; "torch" = torch.rand / torch.randn in
        # SAC.update's order (the equivalence test draws both updates' numbers that way)
        # gemm: "mfma" = the update's 256-wide products by tools/sac_fused.hip gemm256_kernel
        # (batch 256 only; v_mfma_f32_16x16x4_f32, split K over four waves), "blas" = rocBLAS
        self.gemm = os.environ.get("SAC_GEMM", "mfma")
        self.noise = noise or os.environ.get("SAC_NOISE", "philox")
        if self.noise not in ("philox", "torch"):
            raise ValueError("FusedSAC: noise is 'philox' or 'torch'")
        self._launch = torch.zeros(1, dtype=torch.int64, device=self.dev)
        self._seed = int(kw.get("seed", 0)) * 0x9E3779B97F4A7C15 % (1 << 64) ^ 0x5AC0FFEE
        self._pol_eps = None
        if not self.hip_adam or self.dev.type != "cuda":
            raise ValueError("FusedSAC: the HIP Adam path (SAC_ADAM=hip) on a HIP device")
        # (several ranks: the gradients are all-reduced before each Adam launch, _reduce_flat:
        # with an RCCL comm on the update's stream, so RLLoop.capture records it too)
        if FusedSAC._lib is None:
            if not os.path.exists(FUSED_LIB):
                raise RuntimeError(f"{FUSED_LIB} missing: run __graft_entry__.build()")
            lib = ctypes.CDLL(FUSED_LIB)
            for name in ("sf_in_layer", "sf_actor_head", "sf_critic_head",
                         "sf_critic_bwd_in", "sf_actor_bwd_head", "sf_actor_bwd_in",
                         "sf_td_critic_head", "sf_in_layer_pair", "sf_noise", "sf_noise_sample",
                         "sf_gemm"):
                getattr(lib, name).restype = ctypes.c_int32
            FusedSAC._lib = lib
        HipAdam([torch.zeros(1, device=self.dev)], 0.0)         # loads sac_adam.hip's library
        d, B, od, A = self.dev, self.batch, self.od, self.ad
        H = 256
        z = lambda *shape: torch.zeros(shape, dtype=torch.float32, device=d)  # noqa: E731
        # the target critics' and the online critics' second layers in one [4, H, H] tensor
        # (qt.w1 = [0:2], q.w1 = [2:4], views): the TD target's and the critic loss's hidden
        # products are one bmm and one head launch
        self._w1 = torch.cat([self.qt.w1.detach(), self.q.w1.detach()]).contiguous()
        self.qt.w1 = nn.Parameter(self._w1[0:2], requires_grad=self.qt.w1.requires_grad)
        self.q.w1 = nn.Parameter(self._w1[2:4])
        # the critic's optimizer is rebuilt over the new q.w1 (fresh moments, as at creation)
        # with SB3's polyak_update of the targets fused behind its Adam step: the critics'
        # parameters do not change between their step and the update's polyak
        self.opt_q = HipAdam(self.q.parameters(), self.opt_q.lr, step=self.opt_q.t,
                             targets=self.qt.parameters(), tau=self.tau)
        self._u = z(B)
        self._rows = z(B, self.buf.shape[1])
        self._eps = z(2 * B, A)
        self._h0, self._p1a, self._h1 = z(2 * B, H), z(2 * B, H), z(2 * B, H)
        self._mu, self._lsr, self._act, self._logp = z(2 * B, A), z(2 * B, A), z(2 * B, A), z(2 * B)
        self._g04, self._p14, self._g1 = z(4, B, H), z(4, B, H), z(2, B, H)
        self._g0, self._p1c = self._g04[2:4], self._p14[2:4]
        self._q, self._y, self._dq = z(2, B), z(B), z(2, B)
        self._dlogp, self._lossq, self._lossa = z(B), z(B), z(B)
        self._dg1, self._dg0 = z(2, B, H), z(2, B, H)
        self._dh1, self._dh0, self._dmu, self._dlsr = z(B, H), z(B, H), z(B, A), z(B, A)
        # the gradients as views of two flat buffers -- the critics', and the actor's with the
        # entropy coefficient's (the groups each Adam launch steps): the data-parallel
        # reduction is one all-reduce per group, on the update's stream (graph-capturable with
        # an RCCL comm)
        def flat_grads(params):
            n = sum(p.numel() for p in params)
            flat = torch.zeros(n, dtype=torch.float32, device=d)
            off = 0
            for p in params:
                p.grad = flat[off:off + p.numel()].view_as(p)
                off += p.numel()
            return flat
        self._gq = flat_grads(list(self.q.parameters()))
        self._ga = flat_grads(list(self.actor.parameters()) + [self.log_alpha])

    def attach_policy_noise(self, eps):
        """Philox noise: each update also fills `eps` (fp32, contiguous) with N(0, 1) draws for
        the next vector step's action sample (RLLoop), in the same launch."""
        if eps.dtype != torch.float32 or not eps.is_contiguous() or eps.device != self.dev:
            raise ValueError("attach_policy_noise: contiguous fp32 tensor on the learner's device")
        self._pol_eps = eps

    def _call(self, name, *args):
        c = []
        for x in args:
            if isinstance(x, ctypes._SimpleCData):
                c.append(x)
            elif isinstance(x, torch.Tensor):
                c.append(ctypes.c_void_p(x.data_ptr()))
            elif x is None:
                c.append(ctypes.c_void_p(None))
            elif isinstance(x, float):
                c.append(ctypes.c_float(x))
            else:
                c.append(ctypes.c_int32(int(x)))
        c.append(ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream))
        rc = getattr(self._lib, name)(*c)
        if rc != 0:
            raise RuntimeError(f"{name} failed ({rc})")

    def _mm(self, ta, tb, a, b, c, M, batch=1):
        """c[i] = op(a[i]) op(b[i]) for the update's products (K = N = 256): gemm256_kernel at
        batch 256, rocBLAS (torch.mm / bmm into c) otherwise.  a, b, c: the operands as stored
        (op = transpose where ta / tb)."""
        if self.gemm == "mfma" and self.batch == 256:
            sa = a.shape[-2] * a.shape[-1] if batch > 1 else 0
            sb = b.shape[-2] * b.shape[-1] if batch > 1 else 0
            sc = c.shape[-2] * c.shape[-1] if batch > 1 else 0
            self._call("sf_gemm", int(ta), int(tb), a, b, c, M, batch, ctypes.c_longlong(sa),
                       ctypes.c_longlong(sb), ctypes.c_longlong(sc))
            return
        x = a.transpose(-2, -1) if ta else a
        y = b.transpose(-2, -1) if tb else b
        (torch.bmm if batch > 1 else torch.mm)(x, y, out=c)

    def update(self, losses=True):
        """SAC.update's gradient step (same order of evaluation; with noise="torch" the same
        RNG draws)."""
        with torch.no_grad():
            return self._update(losses)

    def _update(self, losses):
        B, od, A = self.batch, self.od, self.ad
        H = 256
        W = self.buf.shape[1]
        ic = od + A
        rows = self._rows
        L = HipAdam._lib
        f = self._call
        if self.noise == "philox":
            # the update's random numbers, the replay sample they draw and the shared Adam step
            # count's tick (opt_q.tick()) in one launch
            pe = self._pol_eps
            f("sf_noise_sample", self._launch, ctypes.c_uint64(self._seed), self._u, B, self._eps,
              2 * B * A, pe, 0 if pe is None else pe.numel(), self.buf, ctypes.c_longlong(self.cap), W,
              self.size, rows, self.opt_q.t)
        else:
            torch.rand(B, device=self.dev, out=self._u)
            # the sample, with the shared Adam step count advanced in the same launch
            rc = L.sac_replay_sample_tick(ctypes.c_void_p(self.buf.data_ptr()), self.cap, W,
                                          ctypes.c_void_p(self._u.data_ptr()), B,
                                          ctypes.c_void_p(self.size.data_ptr()),
                                          ctypes.c_void_p(rows.data_ptr()),
                                          ctypes.c_void_p(self.opt_q.t.data_ptr()),
                                          ctypes.c_void_p(torch.cuda.current_stream(self.dev).cuda_stream))
            if rc != 0:
                raise RuntimeError(f"sac_replay_sample_tick failed ({rc})")
            torch.randn((2 * B, A), device=self.dev, out=self._eps)
        o = rows                                    # columns 0..od of the row
        a = rows[:, od:]                            # the stored action (ld = W)
        o2 = rows[:, od + A + 1:]                   # next obs
        act, logp = self._act, self._logp
        la_, lat = self.actor.latent, self.actor
        # ---- actor on [o2; o] (one pass: its parameters do not change before its step) ----
        q, qt = self.q, self.qt
        # (the online critics' first layer on [o, a] in the same launch as the actor's)
        f("sf_in_layer_pair", o2, o, B, W, od, 2 * B, la_[0].weight, la_[0].bias, self._h0,
          o, W, od, a, W, A, B, q.w0, q.b0, self._g0)
        self._mm(0, 1, self._h0, la_[2].weight, self._p1a, 2 * B)
        # (the target critics' first layer on [o2, a2] inside the actor's head launch)
        f("sf_actor_head", self._p1a, la_[2].bias, lat.mu.weight, lat.mu.bias, lat.log_std.weight,
          lat.log_std.bias, self._eps, 2 * B, A, self._h1, self._mu, self._lsr, act, logp,
          B, o2, W, od, qt.w0, qt.b0, self._g04[0:2])
        # ---- TD target from the target critics on [o2, a2] and the critics on [o, a]: one
        # bmm over the four second layers, one head (y, then the twin MSE's gradient) ---------
        self._mm(0, 0, self._g04, self._w1, self._p14, B, 4)
        f("sf_td_critic_head", self._p14, qt.b1, qt.w2, qt.b2, q.b1, q.w2, q.b2, B, rows, W, od + A,
          W - 1, self.gamma, self.log_alpha, logp, self._y, self._g1, self._q, self._dq, self._lossq,
          self._dg1)
        # ---- the critics' backward and step (polyak of the targets in the same launch) ---------
        # (dg1 came from the TD head's launch; the head's column sums ride in critic_bwd_in)
        self._mm(1, 0, self._g0, self._dg1, q.w1.grad, H, 2)
        self._mm(0, 1, self._dg1, q.w1, self._dg0, B, 2)
        f("sf_critic_bwd_in", self._dg0, self._g0, o, W, od, a, W, A, B, q.w0.grad, q.b0.grad,
          self._g1, self._dq, q.w2, q.w2.grad, q.b1.grad, q.b2.grad)
        if self.world > 1 or self.comm is not None:
            self._reduce_flat(self._gq)
        self.opt_q.step()                            # (the step count was advanced by the sample)
        # ---- actor loss through the updated critics on [o, ap] (critics frozen) ----------------
        ap, lp = act[B:], logp[B:]
        f("sf_in_layer", o, None, B, W, od, ap, A, A, B, 2, q.w0, 1, q.b0, self._g0)
        self._mm(0, 0, self._g0, q.w1, self._p1c, B, 2)
        # (the head's backward, dg1, in the same launch: g1 itself is not needed)
        f("sf_critic_head", self._p1c, q.b1, q.w2, q.b2, B, 2, None, W, 0, 0, self.gamma,
          self.log_alpha, lp, None, None, self._q, self._dq, self._dlogp, self._lossa, self._dg1)
        self._mm(0, 1, self._dg1, q.w1, self._dg0, B, 2)
        # ---- actor backward (the o half of the pass; the critics' action gradient computed in
        # its head launch), entropy coefficient, their step ----------------------------------
        h0b, h1b = self._h0[B:], self._h1[B:]
        f("sf_actor_bwd_head", None, self._dlogp, self._mu[B:], self._lsr[B:], self._eps[B:], ap,
          h1b, lat.mu.weight, lat.log_std.weight, B, A, self._dmu, self._dlsr, self._dh1,
          self._dg0, self._g0, q.w0, ic, od)
        self._mm(1, 0, self._dh1, h0b, la_[2].weight.grad, H)
        self._mm(0, 0, self._dh1, la_[2].weight, self._dh0, B)
        # (with the heads' and b1's column sums and d log_alpha in the same launch)
        f("sf_actor_bwd_in", self._dh0, h0b, o, W, od, B, la_[0].weight.grad, la_[0].bias.grad,
          self._dmu, self._dlsr, h1b, self._dh1, lp, float(self.target_entropy), A,
          lat.mu.weight.grad, lat.log_std.weight.grad, la_[2].bias.grad, lat.mu.bias.grad,
          lat.log_std.bias.grad, self.log_alpha.grad)
        if self.world > 1 or self.comm is not None:
            self._reduce_flat(self._ga)
        self.opt_a.step()                            # actor + log_alpha in one launch
        if losses:
            return self._lossq.sum(), self._lossa.sum()
        return None


class RLLoop:
    """One RL iteration over a core.DeviceBatch in SAME_STEP mode (final_obs on) with
    the SAC above; step() runs it eagerly, capture() records it as one HIP graph."""

    def __init__(self, batch, sac: SAC, learn=True, fused_policy=False):
        self.b, self.sac, self.learn = batch, sac, learn
        self.obs = batch.obs.clone()
        self.act = torch.zeros((batch.E, batch.act_dim), dtype=torch.float64, device=batch.device)
        self.graph, self.iters = None, 1
        # fused_policy: the action sample is one HIP kernel (bluesky_gym.policy.SACPolicy,
        # bsg_policy_sac) reading the live actor's parameters, instead of ~25 torch kernels
        self.pol = None
        # (FusedSAC with Philox noise draws the next step's eps inside its update: one launch less)
        self.own_noise = True
        if fused_policy:
            from bluesky_gym.policy import SACPolicy
            self.pol = SACPolicy.from_module(sac.actor)
            self.eps = torch.randn((batch.E, batch.act_dim), dtype=torch.float32, device=batch.device)
            if learn and isinstance(sac, FusedSAC) and sac.noise == "philox":
                sac.attach_policy_noise(self.eps)
                self.own_noise = False

    def step(self):
        b, s = self.b, self.sac
        if self.pol is not None:
            if self.own_noise:
                torch.randn(self.eps.shape, device=self.eps.device, out=self.eps)
            a = self.pol(self.obs, self.eps, out=self.act)
        else:
            with torch.no_grad():
                a, _ = s.actor(self.obs)
            self.act.copy_(a)
        b.step(self.act)
        copied = False
        if self.learn:
            if s.hip_adam:
                # one launch (tools/sac_adam.hip), which also copies the new observations
                s.insert_step(self.obs, self.act, b, obs_out=self.obs)
                copied = True
            else:
                done = (b.terminated | b.truncated).bool()
                nxt = torch.where(done[:, None], b.final_obs, b.obs)
                s.insert(self.obs, a, b.reward, nxt, b.terminated.float())
            s.update(losses=False)
        if not copied:
            self.obs.copy_(b.obs)

    def capture(self, warm=3, iters=1):
        """iters: RL iterations per graph (each replay runs that many, in order, each with its
        own RNG offsets).  A replay costs host-side submission and torch's two RNG-state fills
        ahead of the graph -- gaps on the GPU that more iterations per graph amortise."""
        side = torch.cuda.Stream(device=self.b.device)
        side.wait_stream(torch.cuda.current_stream(self.b.device))
        with torch.cuda.stream(side):
            for _ in range(warm):
                self.step()
        torch.cuda.current_stream(self.b.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            for _ in range(iters):
                self.step()
        self.graph, self.iters = g, iters

    def replay(self):
        self.graph.replay()
