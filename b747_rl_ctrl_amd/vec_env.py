"""SB3-style VecEnv adapter over BatchControllerEnv -- what `neural/agent.py` trains on.

The reference wraps 4 ControllerEnv copies in `SubprocVecEnv` + `VecMonitor`
(neural/agent.py:63-82).  `B747VecEnv` replaces that stack for N envs on one MI355X with the
stable-baselines3 VecEnv contract (SB3 1.4, requirements.txt:145):

  reset() -> obs [N, obs_dim] float32
  step_async(actions [N, 1]) / step_wait() -> (obs, rewards [N] float32, dones [N] bool, infos)
  infos[i] for a finished env: {"terminal_observation": last obs, "episode": {"r", "l", "t"},
                                "TimeLimit.truncated": False}   (VecEnv auto-reset + VecMonitor: "r" is
                                VecMonitor's float32 return, accumulated per step as float32(r + float64 reward))
  ep_rew_mean(infos...) : SB3's rollout/ep_rew_mean over the recorded episodes (safe_mean: a float32 numpy mean)
  seed(s), close(), get_attr / set_attr / env_method, env_is_wrapped, render

numpy in/out is the SB3 surface (one device->host copy of obs/reward/done per step).  GPU
training loops should call `step_torch`, which returns the device tensors without any copy.
When stable_baselines3 is importable the class derives from its VecEnv, so `isinstance` checks
and SB3 wrappers accept it; otherwise it is a duck-typed stand-in (SB3 is not a dependency).
"""
import time
from typing import Optional, Sequence

import numpy as np
import torch

from .ctrl_env import BatchControllerEnv

try:  # optional: real SB3 base class and gym spaces when present
    from stable_baselines3.common.vec_env.base_vec_env import VecEnv as _SB3VecEnv  # type: ignore
except Exception:  # pragma: no cover - SB3 absent in this image
    _SB3VecEnv = object

try:
    import gym  # type: ignore

    def _box(space):
        return gym.spaces.Box(low=np.asarray(space.low, np.float32) * np.ones(space.shape, np.float32),
                              high=np.asarray(space.high, np.float32) * np.ones(space.shape, np.float32),
                              dtype=np.float32)
except Exception:  # pragma: no cover - gym absent in this image
    def _box(space):
        return space


class B747VecEnv(_SB3VecEnv):
    """N ControllerEnvs behind the SB3 VecEnv interface (auto-reset, VecMonitor episode info)."""

    def __init__(self, env: BatchControllerEnv, monitor_path: Optional[str] = None):
        self.env = env
        self.num_envs = env.n
        self.observation_space = _box(env.observation_space)
        self.action_space = _box(env.action_space)
        self._actions = None
        self._t0 = time.time()
        self._monitor = None
        if monitor_path:
            import json
            self._monitor = open(monitor_path, "w")
            self._monitor.write("#" + json.dumps({"t_start": self._t0, "env_id": "B747VecEnv"}) + "\n")
            self._monitor.write("r,l,t\n")

    # ------------------------------------------------------------ VecEnv contract --
    def reset(self):
        obs = self.env.reset()
        return obs.cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        obs, rew, done, info = self.step_torch(self._actions)
        obs_h, rew_h, done_h = obs.cpu().numpy(), rew.cpu().numpy(), done.cpu().numpy()
        infos = [{} for _ in range(self.num_envs)]
        idx = np.flatnonzero(done_h)
        if idx.size:
            term = info["terminal_observation"][idx].cpu().numpy()
            ret = info["episode_return"][idx].cpu().numpy()
            length = info["episode_length"][idx].cpu().numpy()
            t = round(time.time() - self._t0, 6)
            for j, i in enumerate(idx):
                # VecMonitor's record: its float32 episode_returns / int32 episode_lengths entries (the kernels
                # accumulate the return exactly as VecMonitor does: float32(return + float64 reward) per step)
                ep = {"r": np.float32(ret[j]), "l": np.int32(length[j]), "t": t}
                infos[i] = {"terminal_observation": term[j], "episode": ep, "TimeLimit.truncated": False}
                if self._monitor:
                    self._monitor.write(f"{ep['r']},{ep['l']},{ep['t']}\n")
        return obs_h, rew_h, done_h, infos

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def step_torch(self, actions):
        """Device-resident step: actions as a tensor (or array) [N] / [N, 1]; returns the env's own
        obs / reward / done tensors and info dict (no host copy)."""
        a = torch.as_tensor(actions, dtype=torch.float32, device=self.env.device).reshape(self.num_envs)
        return self.env.step(a)

    def seed(self, seed: Optional[int] = None):
        """Re-key the reset RNG (Philox key = seed; streams stay per global env id)."""
        if seed is not None:
            self.env.cfg.seed = int(seed) & 0xFFFFFFFFFFFFFFFF
        return [seed] * self.num_envs

    def close(self):
        if self._monitor:
            self._monitor.close()
            self._monitor = None

    def render(self, mode: str = "human"):
        return None

    def get_attr(self, attr_name: str, indices=None):
        return [getattr(self.env, attr_name)] * len(self._indices(indices))

    def set_attr(self, attr_name: str, value, indices=None):
        setattr(self.env, attr_name, value)

    def env_method(self, method_name: str, *method_args, indices=None, **method_kwargs):
        out = getattr(self.env, method_name)(*method_args, **method_kwargs)
        return [out] * len(self._indices(indices))

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def get_images(self) -> Sequence[np.ndarray]:
        return []

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices


def ep_rew_mean(episodes) -> np.float32:
    """SB3's `rollout/ep_rew_mean` (OnPolicyAlgorithm logging: safe_mean over ep_info_buffer): numpy's mean of the
    episodes' float32 "r" values, itself float32 (numpy sums float32 pairwise in float32)."""
    r = np.asarray([e["r"] for e in episodes], dtype=np.float32)
    return np.float32(np.nan) if r.size == 0 else np.mean(r)


def make_vec_env(n: int, *args, monitor_path: Optional[str] = None, **kwargs) -> B747VecEnv:
    """`Agent._wrap_env` replacement: B747VecEnv over BatchControllerEnv(n, *args, **kwargs)."""
    return B747VecEnv(BatchControllerEnv(n, *args, **kwargs), monitor_path=monitor_path)


class B747GymVectorEnv(B747VecEnv):
    """gym 0.19 `VectorEnv` facade (requirements.txt:51 pins gym 0.19): the same N envs
    with gym's vector API -- batched `observation_space` [N, obs_dim] / `action_space` [N, 1], the per-env
    `single_observation_space` / `single_action_space`, reset() / step() with reset_async / reset_wait
    and step_async / step_wait, and SyncVectorEnv's auto-reset (infos[i] of a finished env carries the
    terminal observation).  gym is not importable in this image, so the spaces are duck-typed Box
    stand-ins unless gym is present."""

    def __init__(self, env: BatchControllerEnv):
        super().__init__(env)
        self.single_observation_space = self.observation_space
        self.single_action_space = self.action_space
        self.observation_space = _batched(env.observation_space, self.num_envs)
        self.action_space = _batched(env.action_space, self.num_envs)
        self.closed = False

    def reset_async(self):
        pass

    def reset_wait(self, **kwargs):
        return B747VecEnv.reset(self)

    def step(self, actions):
        self.step_async(actions)
        obs, rew, done, infos = self.step_wait()
        for info in infos:                      # gym's infos carry no VecMonitor episode record
            info.pop("episode", None)
            info.pop("TimeLimit.truncated", None)
        return obs, rew, done, infos

    def close(self):
        super().close()
        self.closed = True


def _batched(space, n):
    """gym.vector.utils.batch_space for a Box: the same bounds stacked n times."""
    lo = np.broadcast_to(np.asarray(space.low, np.float32), space.shape)
    hi = np.broadcast_to(np.asarray(space.high, np.float32), space.shape)
    try:
        import gym  # type: ignore
        return gym.spaces.Box(low=np.stack([lo] * n), high=np.stack([hi] * n), dtype=np.float32)
    except Exception:
        from .ctrl_env import Box
        return Box(np.stack([lo] * n), np.stack([hi] * n), (n,) + tuple(space.shape))
