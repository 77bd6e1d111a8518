"""Soft Actor-Critic in plain torch, on the device that holds the env batch -- the learner
of BASELINE configs[4] ("DescentEnv-v0 + SB3 SAC learner, 4096 envs"), for measuring
end-to-end RL throughput with the MI355X env path (bench.py --workload descent-sac).

stable-baselines3 is not installed here; this restates the part of SB3 2.x SAC that runs
per environment step with the hyper-parameters of the reference's training script
(scripts/descent_env_sac.py:25-34 -> SB3 defaults): MultiInputPolicy (the Dict obs
flattened in sorted-key order = the kernel's flat rows), actor and twin critics
Linear-ReLU 256-256, squashed Gaussian with log_std clamped to [-20, 2], Adam lr 3e-4,
batch 256, buffer 1e6, gamma 0.99, tau 0.005, entropy coefficient 'auto' (target
entropy -dim(A)), train_freq 1 / gradient_steps 1 -- one gradient step per vector step.

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

import math

import torch
import torch.nn as nn
import torch.nn.functional as F

LOG_STD_MIN, LOG_STD_MAX = -20.0, 2.0


def mlp(i, o, h=256):
    return nn.Sequential(nn.Linear(i, h), nn.ReLU(), nn.Linear(h, h), nn.ReLU(), nn.Linear(h, o))


class Actor(nn.Module):
    def __init__(self, obs_dim, act_dim, h=256):
        super().__init__()
        self.latent = nn.Sequential(nn.Linear(obs_dim, h), nn.ReLU(), nn.Linear(h, h), nn.ReLU())
        self.mu = nn.Linear(h, act_dim)
        self.log_std = nn.Linear(h, act_dim)

    def forward(self, obs):
        """(tanh-squashed sample, log-prob) of the SB3 squashed diagonal Gaussian."""
        h = self.latent(obs)
        mu = self.mu(h)
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


class SAC:
    def __init__(self, obs_dim, act_dim, device, *, lr=3e-4, batch=256, buffer=1_000_000,
                 gamma=0.99, tau=0.005, group=None, seed=0):
        torch.manual_seed(seed)
        self.dev = torch.device(device)
        self.actor = Actor(obs_dim, act_dim).to(self.dev)
        self.q1, self.q2 = mlp(obs_dim + act_dim, 1).to(self.dev), mlp(obs_dim + act_dim, 1).to(self.dev)
        self.q1t, self.q2t = mlp(obs_dim + act_dim, 1).to(self.dev), mlp(obs_dim + act_dim, 1).to(self.dev)
        self.q1t.load_state_dict(self.q1.state_dict())
        self.q2t.load_state_dict(self.q2.state_dict())
        self.log_alpha = torch.zeros(1, device=self.dev, requires_grad=True)
        self.target_entropy = -float(act_dim)
        # fused Adam: one kernel per parameter group instead of a foreach chain per tensor
        # (the update is launch-bound: batch 256 through 256-wide MLPs)
        opt = dict(lr=lr, fused=True, capturable=True) if self.dev.type == "cuda" else dict(lr=lr)
        self.opt_a = torch.optim.Adam(self.actor.parameters(), **opt)
        self.opt_q = torch.optim.Adam(list(self.q1.parameters()) + list(self.q2.parameters()), **opt)
        self.opt_al = torch.optim.Adam([self.log_alpha], **opt)
        self.gamma, self.tau = gamma, tau
        self.group = group
        world = torch.distributed.get_world_size(group) if group is not None else 1
        self.world = world
        self.batch = max(1, batch // world)
        self.cap = buffer // world
        d = self.dev
        self.buf_obs = torch.zeros((self.cap, obs_dim), device=d)
        self.buf_next = torch.zeros((self.cap, obs_dim), device=d)
        self.buf_act = torch.zeros((self.cap, act_dim), device=d)
        self.buf_rew = torch.zeros((self.cap,), device=d)
        self.buf_done = torch.zeros((self.cap,), device=d)
        self.pos = torch.zeros((), dtype=torch.long, device=d)
        self.size = torch.zeros((), dtype=torch.long, device=d)

    # -------------------------------------------------------------- replay buffer
    def insert(self, obs, act, rew, next_obs, term):
        n = obs.shape[0]
        idx = (self.pos + torch.arange(n, device=self.dev)) % self.cap
        self.buf_obs.index_copy_(0, idx, obs)
        self.buf_next.index_copy_(0, idx, next_obs)
        self.buf_act.index_copy_(0, idx, act)
        self.buf_rew.index_copy_(0, idx, rew)
        self.buf_done.index_copy_(0, idx, term)
        self.pos.copy_((self.pos + n) % self.cap)
        self.size.copy_(torch.clamp(self.size + n, max=self.cap))

    def sample(self):
        u = torch.rand(self.batch, device=self.dev)
        idx = torch.clamp((u * self.size.float()).long(), max=self.cap - 1)
        return (self.buf_obs[idx], self.buf_act[idx], self.buf_rew[idx], self.buf_next[idx],
                self.buf_done[idx])

    # -------------------------------------------------------------- SAC update
    def _allreduce(self, params):
        if self.world == 1:
            return
        grads = [p.grad for p in params if p.grad is not None]
        flat = torch.cat([g.reshape(-1) for g in grads])
        torch.distributed.all_reduce(flat, group=self.group)
        flat /= self.world
        off = 0
        for g in grads:
            n = g.numel()
            g.copy_(flat[off:off + n].view_as(g))
            off += n

    def update(self):
        o, a, r, o2, d = self.sample()
        alpha = self.log_alpha.exp().detach()
        with torch.no_grad():
            a2, logp2 = self.actor(o2)
            x2 = torch.cat([o2, a2], -1)
            qt = torch.min(self.q1t(x2), self.q2t(x2)).squeeze(-1) - alpha * logp2
            y = r + self.gamma * (1.0 - d) * qt
        x = torch.cat([o, a], -1)
        lq = F.mse_loss(self.q1(x).squeeze(-1), y) + F.mse_loss(self.q2(x).squeeze(-1), y)
        self.opt_q.zero_grad(set_to_none=False)
        lq.backward()
        self._allreduce(list(self.q1.parameters()) + list(self.q2.parameters()))
        self.opt_q.step()
        ap, logp = self.actor(o)
        xp = torch.cat([o, ap], -1)
        la = (alpha * logp - torch.min(self.q1(xp), self.q2(xp)).squeeze(-1)).mean()
        self.opt_a.zero_grad(set_to_none=False)
        la.backward()
        self._allreduce(list(self.actor.parameters()))
        self.opt_a.step()
        lal = -(self.log_alpha * (logp.detach() + self.target_entropy)).mean()
        self.opt_al.zero_grad(set_to_none=False)
        lal.backward()
        self._allreduce([self.log_alpha])
        self.opt_al.step()
        with torch.no_grad():
            # SB3 polyak_update (target * (1 - tau), then + tau * param), as two multi-tensor
            # kernels over all target parameters instead of two kernels per tensor
            src = list(self.q1.parameters()) + list(self.q2.parameters())
            tgt = list(self.q1t.parameters()) + list(self.q2t.parameters())
            torch._foreach_mul_(tgt, 1.0 - self.tau)
            torch._foreach_add_(tgt, src, alpha=self.tau)
        return lq.detach(), la.detach()


class RLLoop:
    """One RL iteration over a core.DeviceBatch in SAME_STEP mode (final_obs on) with
    the SAC above; step() runs it eagerly, capture() records it as one HIP graph."""

    def __init__(self, batch, sac: SAC, learn=True):
        self.b, self.sac, self.learn = batch, sac, learn
        self.obs = batch.obs.clone()
        self.act = torch.zeros((batch.E, batch.act_dim), dtype=torch.float64, device=batch.device)
        self.graph = None

    def step(self):
        b, s = self.b, self.sac
        with torch.no_grad():
            a, _ = s.actor(self.obs)
        self.act.copy_(a)
        b.step(self.act)
        done = (b.terminated | b.truncated).bool()
        if self.learn:
            nxt = torch.where(done[:, None], b.final_obs, b.obs)
            s.insert(self.obs, a, b.reward, nxt, b.terminated.float())
            s.update()
        self.obs.copy_(b.obs)

    def capture(self, warm=3):
        side = torch.cuda.Stream(device=self.b.device)
        side.wait_stream(torch.cuda.current_stream(self.b.device))
        with torch.cuda.stream(side):
            for _ in range(warm):
                self.step()
        torch.cuda.current_stream(self.b.device).wait_stream(side)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g):
            self.step()
        self.graph = g

    def replay(self):
        self.graph.replay()
