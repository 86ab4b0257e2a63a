"""On-GPU PPO rollout over BatchControllerEnv (BASELINE config 5).

The reference trains `PPO('MlpPolicy', env)` from stable-baselines3 with `hp = {}` (the
hyperparams table is keyed by the string 'PPO', neural/setups.py:29, so `PPO in hyperparams` is
False at neural/agent.py:48): SB3 1.4 defaults -- separate pi/vf MLPs [64, 64] with tanh,
orthogonal init, state-independent log_std (init 0), n_steps 2048, gamma 0.99, gae_lambda 0.95,
clip 0.2, ent 0.0, vf 0.5, max_grad_norm 0.5, Adam lr 3e-4, 10 epochs, batch 64.

Here the policy, the rollout buffer and the env all live on the GPU: one rollout step is
policy forward -> Gaussian sample -> clip to the action space -> b747_env_step, with every
tensor preallocated so the whole n_steps rollout can be captured in one HIP graph.  GAE and the
clipped-surrogate update run on device too (batch size scaled to the env count: SB3's batch of
64 is meant for 4 envs).

Data-parallel over ranks (SURVEY 8(e), config 5 on several GPUs): every rank steps its own env
shard (global env ids rank*N + i, so the Philox streams never overlap) and collects its own rollout;
`process_group` makes the ranks start from rank 0's parameters and average their gradients with
ONE all-reduce of the flat gradient bucket (~9k fp32, 36 KB) per minibatch before clipping and the
Adam step -- the only collective, once per minibatch, never on the rollout path.
"""
import math
from dataclasses import dataclass
from typing import Callable, Optional

import torch
import torch.distributed as dist
from torch import nn

from .ctrl_env import BatchControllerEnv


class ActorCritic(nn.Module):
    """SB3 MlpPolicy for a 1-D Box action: pi/vf extractors [64, 64] tanh, action_net, value_net,
    log_std parameter; orthogonal init with SB3's gains (sqrt 2 / 0.01 / 1)."""

    def __init__(self, obs_dim: int, act_dim: int = 1, hidden=(64, 64), log_std_init: float = 0.0):
        super().__init__()

        def mlp():
            layers, d = [], obs_dim
            for h in hidden:
                layers += [nn.Linear(d, h), nn.Tanh()]
                d = h
            return nn.Sequential(*layers)
        self.pi_net, self.vf_net = mlp(), mlp()
        self.action_net = nn.Linear(hidden[-1], act_dim)
        self.value_net = nn.Linear(hidden[-1], 1)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))
        for m, g in ((self.pi_net, math.sqrt(2)), (self.vf_net, math.sqrt(2)), (self.action_net, 0.01),
                     (self.value_net, 1.0)):
            for lin in m.modules():
                if isinstance(lin, nn.Linear):
                    nn.init.orthogonal_(lin.weight, gain=g)
                    nn.init.zeros_(lin.bias)

    def flat_params(self):
        """The parameters in the order b747_policy_act reads them (include/b747.h): pi_net layers,
        vf_net layers, action_net, value_net (weight then bias each), log_std."""
        seq = []
        for m in (self.pi_net, self.vf_net):
            for lin in m:
                if isinstance(lin, nn.Linear):
                    seq += [lin.weight, lin.bias]
        seq += [self.action_net.weight, self.action_net.bias, self.value_net.weight, self.value_net.bias,
                self.log_std]
        return torch.cat([p.detach().reshape(-1) for p in seq])

    def forward(self, obs):
        mean = self.action_net(self.pi_net(obs))
        value = self.value_net(self.vf_net(obs)).squeeze(-1)
        return mean, value

    def log_prob(self, mean, actions):
        std = self.log_std.exp()
        return (-((actions - mean) ** 2) / (2 * std * std) - self.log_std - 0.5 * math.log(2 * math.pi)).sum(-1)

    def entropy(self):
        return (0.5 + 0.5 * math.log(2 * math.pi) + self.log_std).sum()


def _world(group) -> int:
    return dist.get_world_size(group) if dist.is_available() and dist.is_initialized() else 1


def broadcast_parameters(module: nn.Module, group=None, src_rank: int = 0):
    """Every rank takes the parameters of rank `src_rank` of `group` (one flat broadcast)."""
    params = [p.data for p in module.parameters()]
    flat = torch.cat([p.reshape(-1) for p in params])
    src = dist.get_global_rank(group, src_rank) if group is not None else src_rank
    dist.broadcast(flat, src=src, group=group)
    off = 0
    for p in params:
        p.copy_(flat[off:off + p.numel()].view_as(p))
        off += p.numel()


def check_env_shards(env, group=None):
    """Data-parallel PPO needs every rank on its OWN env shard of the SAME size: equal counts,
    or the ranks run different numbers of minibatches and the per-minibatch all-reduce hangs; disjoint
    global env ids [env_offset, env_offset + n) under one reset seed, or the Philox reset draws and policy
    noise (both keyed by the global env id) repeat on every rank and the all-reduce silently averages
    duplicate experience.  One all-gather of (n, env_offset, seed) at construction; every rank sees the
    same table, so every rank raises together (no rank is left waiting in a collective)."""
    world = _world(group)
    if world == 1:
        return
    dev = env.device if dist.get_backend(group) == "nccl" else torch.device("cpu")
    seed = int(getattr(getattr(env, "cfg", None), "seed", 0)) & ((1 << 64) - 1)
    seed = seed - (1 << 64) if seed >= 1 << 63 else seed    # the uint64 Philox key as int64 (same bits)
    mine = torch.tensor([int(env.n), int(getattr(env, "env_offset", 0)), seed], dtype=torch.int64, device=dev)
    rows = [torch.zeros_like(mine) for _ in range(world)]
    dist.all_gather(rows, mine, group=group)
    rows = [tuple(int(v) for v in r.cpu().tolist()) for r in rows]
    if len({r[0] for r in rows}) != 1:
        raise ValueError(f"data-parallel PPO: env counts differ across ranks {[r[0] for r in rows]} "
                         "(every rank must run the same number of minibatches)")
    for a in range(world):
        for b in range(a + 1, world):
            (n, oa, sa), (_, ob, sb) = rows[a], rows[b]
            if sa == sb and oa < ob + n and ob < oa + n:
                raise ValueError(f"data-parallel PPO: ranks {a} and {b} hold overlapping env ids "
                                 f"[{oa}, {oa + n}) and [{ob}, {ob + n}) under the same seed -- their experience "
                                 "would be identical; give rank r env_offset = r * n")


def allreduce_gradients(params, group=None):
    """Average the gradients of `params` over the ranks of `group` through ONE flat bucket (a single
    all-reduce of ~36 KB for the 64-64 policy instead of one per parameter tensor)."""
    world = _world(group)
    grads = [p.grad for p in params if p.grad is not None]
    if world == 1 or not grads:
        return
    flat = torch.cat([g.reshape(-1) for g in grads])
    dist.all_reduce(flat, op=dist.ReduceOp.SUM, group=group)
    flat.div_(world)
    off = 0
    for g in grads:
        g.copy_(flat[off:off + g.numel()].view_as(g))
        off += g.numel()


@dataclass
class PPOConfig:
    n_steps: int = 2048
    gamma: float = 0.99
    gae_lambda: float = 0.95
    clip_range: float = 0.2
    ent_coef: float = 0.0
    vf_coef: float = 0.5
    max_grad_norm: float = 0.5
    learning_rate: float = 3e-4
    n_epochs: int = 10
    batch_size: int = 65536


class PPO:
    """Device-resident PPO on a BatchControllerEnv (action space [-1, 1] with norm_act)."""

    def __init__(self, env: BatchControllerEnv, cfg: Optional[PPOConfig] = None, seed: int = 0, fused: bool = True,
                 rollout_kernel: Optional[bool] = None, process_group=None, data_parallel: Optional[bool] = None):
        """fused=True: one b747_policy_act launch per rollout step (HIP kernel, include/b747.h);
        fused=False: the same policy as torch modules (reference implementation of the math).
        rollout_kernel (fused only; None = wherever it applies): the whole rollout as ONE
        b747_ppo_rollout launch (policy + env step fused, state in registers across steps) for the
        configuration that kernel covers; False keeps two launches per step.
        data_parallel (None = whenever torch.distributed is initialised with more than one rank):
        average the gradients over `process_group` (module docstring); every rank must hold an env
        shard of the same size so that all ranks run the same number of minibatches."""
        self.env, self.cfg = env, cfg or PPOConfig()
        self.fused, self.seed = bool(fused), int(seed)
        dev, n, T, od = env.device, env.n, self.cfg.n_steps, env.obs_dim
        torch.manual_seed(seed)
        self.policy = ActorCritic(od).to(dev)
        self.group = process_group
        self.data_parallel = (_world(process_group) > 1) if data_parallel is None else bool(data_parallel)
        if self.data_parallel:
            check_env_shards(env, process_group)
            broadcast_parameters(self.policy, process_group)
        self.opt = torch.optim.Adam(self.policy.parameters(), lr=self.cfg.learning_rate, eps=1e-5)
        lo, hi = env.action_space.low, env.action_space.high
        self.act_lo, self.act_hi = float(lo), float(hi)
        z = lambda *s, dt=torch.float32: torch.zeros(*s, dtype=dt, device=dev)
        self.obs_buf, self.act_buf = z(T, n, od), z(T, n, 1)
        self.logp_buf, self.val_buf, self.rew_buf = z(T, n), z(T, n), z(T, n)
        self.done_buf = z(T, n, dt=torch.bool)
        self.adv_buf, self.ret_buf = z(T, n), z(T, n)
        self.last_obs = z(n, od)
        self._last_obs_from_env = False   # (rollout kernel: last_obs is env.obs, copied when compute_gae reads it)
        self.last_done = z(n, dt=torch.bool)
        self.noise = z(n, 1)
        self._graph = None
        self._graph_steps = 0
        if self.fused:
            from . import _lib
            self._lib = _lib
            self._L = _lib.lib()
            self.flat = z(int(self._L.b747_policy_num_params(od)))
            self.step_base = torch.zeros(1, dtype=torch.int64, device=dev)   # Philox counter base
            self.sync_params()
        self.rollout_kernel = False
        if self.fused and rollout_kernel is not False:
            ok = self._ppo_rollout(0) == 0                # T = 0: validates the configuration, launches nothing
            if rollout_kernel and not ok:
                raise ValueError(f"b747_ppo_rollout does not cover this env: {self._L.b747_last_error().decode()}")
            self.rollout_kernel = ok

    def sync_params(self):
        """Copy the policy parameters into the flat fp32 buffer the fused kernel reads."""
        if self.fused:
            with torch.no_grad():
                fp = self.policy.flat_params()
                self.flat[:fp.numel()].copy_(fp)
            self._lib.check(self._L.b747_policy_pack(self.flat.data_ptr(), self.env.obs_dim,
                                                     torch.cuda.current_stream().cuda_stream), "b747_policy_pack")

    # --------------------------------------------------------------- rollout --
    @torch.no_grad()
    def _rollout_step(self, t: int, noise: Optional[torch.Tensor] = None):
        """One policy + env step into rollout row t.  noise [n] (optional, on the env's device): the standard
        normal draws to sample with instead of the generator's -- e.g. a recorded run's own action noise
        (tests/tb_training.py replays the reference's SB3 rollouts this way)."""
        if self.fused:
            return self._rollout_step_fused(t, noise)
        obs = self.last_obs
        mean, value = self.policy(obs)
        if noise is None:
            self.noise.normal_()                  # default CUDA generator: graph-capture safe
        else:
            self.noise.copy_(noise.reshape(self.noise.shape))
        action = mean + self.policy.log_std.exp() * self.noise
        self.obs_buf[t].copy_(obs)
        self.act_buf[t].copy_(action)
        self.logp_buf[t].copy_(self.policy.log_prob(mean, action))
        self.val_buf[t].copy_(value)
        clipped = action.clamp(self.act_lo, self.act_hi)          # SB3 clips before env.step
        o, r, d, _ = self.env.step(clipped.view(-1))
        self.rew_buf[t].copy_(r)
        self.done_buf[t].copy_(d)
        self.last_obs.copy_(o)

    def _rollout_step_fused(self, t: int, noise: Optional[torch.Tensor] = None):
        """Two launches per step: the policy reads the env's current obs and writes the rollout
        row + the env's action buffer; the env step writes reward / done straight into the
        rollout buffers (b747_env_rollout with K = 1).  noise [n] fp32 on the device (optional): the
        kernel's standard normal draws instead of its Philox ones (b747_policy_act's noise argument)."""
        env, p = self.env, lambda x: x.data_ptr()
        stream = torch.cuda.current_stream().cuda_stream
        if noise is not None:
            assert noise.dtype == torch.float32 and noise.is_contiguous() and noise.numel() == env.n \
                and noise.device == env.device, "noise: [n] contiguous fp32 on the env's device"
        self._lib.check(self._L.b747_policy_act(
            p(self.flat), env.obs_dim, env.n, p(env.obs), None if noise is None else p(noise), self.seed,
            p(self.step_base), t,
            env.env_offset, p(self.obs_buf[t]), p(self.act_buf[t]), p(self.logp_buf[t]), p(self.val_buf[t]),
            p(env.action), self.act_lo, self.act_hi, stream), "b747_policy_act")
        env.rollout(env.action.view(1, -1), None, self.rew_buf[t], self.done_buf[t])

    def _ppo_rollout(self, T: int) -> int:
        env, p = self.env, lambda x: x.data_ptr()
        env._batch()
        return self._L.b747_ppo_rollout(env._bref, env._cref, env._kref, p(self.flat), self.seed, p(self.step_base), T,
                                        p(self.obs_buf), p(self.act_buf), p(self.logp_buf), p(self.val_buf),
                                        p(self.rew_buf), p(self.done_buf), self.act_lo, self.act_hi,
                                        torch.cuda.current_stream().cuda_stream)

    def _end_rollout(self, T: int):
        if self.fused:
            self.step_base.add_(T)                    # fresh Philox counters for the next rollout
            self.last_obs.copy_(self.env.obs)         # bootstrap observation for GAE

    def _end_kernel_rollout(self):
        # b747_ppo_rollout advances step_base itself (ABI 10), and the bootstrap observation is the env's, taken
        # when compute_gae needs it: the captured rollout is then its two kernels and nothing else
        self._last_obs_from_env = True

    def _bootstrap_obs(self) -> torch.Tensor:
        if self._last_obs_from_env:
            self.last_obs.copy_(self.env.obs)
            self._last_obs_from_env = False
        return self.last_obs

    def _graph_key(self, T: int):
        """What a captured rollout graph baked in: the step count, the env's C descriptor (rebuilt when buffers are added,
        e.g. track_episodes / record_signals), the configuration and constants, and the kernel specialisation -- a
        change of any of them re-captures instead of replaying stale arguments"""
        from . import _lib
        env, L = self.env, _lib.lib()
        spec = int(L.b747_set_specialization(1))   # (the ABI has no query: read it by setting, then restore)
        L.b747_set_specialization(spec)
        return (T, env._batch(), bytes(env.cfg), bytes(env.consts), spec)   # (the descriptor itself: no id reuse)

    def collect_rollouts(self, n_steps: Optional[int] = None, use_graph: bool = True):
        """n_steps (default cfg.n_steps) policy+env steps for every env, all on device.  With the rollout kernel the
        bootstrap observation stays in env.obs until compute_gae copies it into last_obs (no copy node in the graph)."""
        T = n_steps or self.cfg.n_steps
        assert T <= self.cfg.n_steps
        if self.rollout_kernel:                      # one launch for the whole rollout
            if not use_graph:
                with torch.no_grad():
                    self._lib.check(self._ppo_rollout(T), "b747_ppo_rollout")
                self._end_kernel_rollout()
                return T
            # ... and with use_graph, that launch and the value pass replayed as one HIP graph: no host work between
            # the call and the GPU (the configuration, seed and buffers are the capture's, as for the two-launch graph
            # below; the value pass advances step_base on the device)
            if self._graph is None or self._graph_steps != self._graph_key(T):
                s = torch.cuda.Stream(device=self.env.device)
                s.wait_stream(torch.cuda.current_stream())
                g = torch.cuda.CUDAGraph()
                with torch.cuda.graph(g, stream=s), torch.no_grad():
                    self._lib.check(self._ppo_rollout(T), "b747_ppo_rollout")
                self._graph, self._graph_steps = g, self._graph_key(T)
            self._graph.replay()
            self._end_kernel_rollout()
            return T
        if not use_graph:
            for t in range(T):
                self._rollout_step(t)
            self._end_rollout(T)
            return T
        if self._graph is None or self._graph_steps != self._graph_key(T):
            s = torch.cuda.Stream(device=self.env.device)
            s.wait_stream(torch.cuda.current_stream())
            with torch.cuda.stream(s), torch.no_grad():     # warm up the policy kernels (no env step)
                mean, _ = self.policy(self.last_obs)
                self.policy.log_prob(mean, mean)
            torch.cuda.current_stream().wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with torch.cuda.graph(g, stream=s):
                for t in range(T):
                    self._rollout_step(t)
                self._end_rollout(T)
            self._graph, self._graph_steps = g, self._graph_key(T)
        self._graph.replay()
        return T

    @torch.no_grad()
    def compute_gae(self, T: Optional[int] = None):
        """Generalized advantage estimation (SB3 RolloutBuffer.compute_returns_and_advantage)."""
        T = T or self.cfg.n_steps
        c = self.cfg
        _, last_value = self.policy(self._bootstrap_obs())
        gae = torch.zeros_like(last_value)
        for t in reversed(range(T)):
            next_value = last_value if t == T - 1 else self.val_buf[t + 1]
            nonterminal = (~self.done_buf[t]).float()
            delta = self.rew_buf[t] + c.gamma * next_value * nonterminal - self.val_buf[t]
            gae = delta + c.gamma * c.gae_lambda * nonterminal * gae
            self.adv_buf[t] = gae
        self.ret_buf[:T] = self.adv_buf[:T] + self.val_buf[:T]

    def train(self, T: Optional[int] = None, minibatch_order: Optional[Callable[[int, int, int], torch.Tensor]] = None):
        """Clipped-surrogate PPO epochs over the rollout (SB3 1.4 PPO.train).

        minibatch_order(epoch, T, n) -> [T * n] indices into the time-major rollout (row t * n + env) giving
        the epoch's sample order; default torch.randperm.  (SB3 draws np.random.permutation over its env-major
        flattening, RolloutBuffer.get / swap_and_flatten; tests/tb_transfer.py passes that order to replay a
        recorded SB3 update.)
        Returns SB3's train/* log values: entropy_loss, policy_gradient_loss, value_loss and clip_fraction
        (means over every minibatch), approx_kl (mean over the last epoch's minibatches), loss (the last
        minibatch), explained_variance (of the rollout's values against its returns) and std; policy_loss /
        value_loss repeat the means.  Beside them (not SB3 log values): pg_term_scale = mean |A ratio| over every
        minibatch and kl_term_scale = mean (|ratio| + 1 + |log ratio|) over the last epoch's, the magnitude of the
        terms the two cancelling means sum (the float32 rounding scale of policy_gradient_loss and approx_kl, which the
        replay gates of tests/tb_training.py use).  One host synchronisation at the end."""
        T = T or self.cfg.n_steps
        c = self.cfg
        N = T * self.env.n
        views = (self.obs_buf[:T].reshape(N, -1), self.act_buf[:T].reshape(N, -1), self.logp_buf[:T].reshape(N),
                 self.adv_buf[:T].reshape(N), self.ret_buf[:T].reshape(N))
        n_mb = -(-N // c.batch_size)
        rows = torch.empty(c.n_epochs * n_mb, 7, dtype=torch.float32, device=views[0].device)
        loss, k = None, 0
        for epoch in range(c.n_epochs):
            if minibatch_order is None:
                perm = torch.randperm(N, device=views[0].device)
            else:
                perm = torch.as_tensor(minibatch_order(epoch, T, self.env.n), device=views[0].device)
            for i in range(0, N, c.batch_size):
                idx = perm[i:i + c.batch_size]
                loss, st = self._minibatch(idx, views)
                rows[k].copy_(st)
                k += 1
        self.sync_params()
        with torch.no_grad():
            v, r = self.val_buf[:T].reshape(N), views[4]
            var_r = r.var(unbiased=False)
            ev = 1 - (r - v).var(unbiased=False) / var_r if float(var_r) != 0 else torch.tensor(float("nan"))
            mean = rows.double().mean(0).tolist()
            stats = {"entropy_loss": mean[2], "policy_gradient_loss": mean[0], "value_loss": mean[1],
                     "approx_kl": float(rows[(c.n_epochs - 1) * n_mb:, 4].double().mean()), "clip_fraction": mean[3],
                     "loss": float(loss) if loss is not None else float("nan"),
                     "explained_variance": float(ev), "std": float(self.policy.log_std.exp().mean()),
                     "pg_term_scale": mean[5], "kl_term_scale": float(rows[(c.n_epochs - 1) * n_mb:, 6].double().mean())}
        stats["policy_loss"] = stats["policy_gradient_loss"]
        return stats

    def _minibatch(self, idx, views):
        """One clipped-surrogate step on the rows `idx` of the rollout views -> (loss, [pg, vf, entropy loss,
        clip fraction, approx_kl, mean |A ratio|, mean (|ratio| + 1 + |log ratio|)])."""
        c = self.cfg
        obs, act, old_logp, adv, ret = views
        mean, value = self.policy(obs[idx])
        logp = self.policy.log_prob(mean, act[idx])
        a = adv[idx]
        a = (a - a.mean()) / (a.std() + 1e-8)
        log_ratio = logp - old_logp[idx]
        ratio = torch.exp(log_ratio)
        pg = -torch.min(a * ratio, a * ratio.clamp(1 - c.clip_range, 1 + c.clip_range)).mean()
        vf = ((ret[idx] - value) ** 2).mean()
        ent_loss = -self.policy.entropy()
        loss = pg + c.ent_coef * ent_loss + c.vf_coef * vf
        with torch.no_grad():
            st = torch.stack([pg, vf, ent_loss, ((ratio - 1).abs() > c.clip_range).float().mean(),
                              ((ratio - 1) - log_ratio).mean(), (a * ratio).abs().mean(),
                              (ratio.abs() + 1 + log_ratio.abs()).mean()])
        self.opt.zero_grad(set_to_none=True)
        loss.backward()
        if self.data_parallel:
            allreduce_gradients(self.policy.parameters(), self.group)
        nn.utils.clip_grad_norm_(self.policy.parameters(), c.max_grad_norm)
        self.opt.step()
        return loss.detach(), st

    def learn(self, iterations: int, n_steps: Optional[int] = None):
        T = n_steps or self.cfg.n_steps
        self.last_obs.copy_(self.env.reset())
        self._last_obs_from_env = False
        hist = []
        for _ in range(iterations):
            self.collect_rollouts(T)
            self.compute_gae(T)
            hist.append(self.train(T) | {"mean_reward": float(self.rew_buf[:T].mean())})
        return hist
