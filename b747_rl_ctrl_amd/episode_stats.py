"""Episode statistics of a (sharded) env batch: SURVEY 8(e)'s optional gather of scalar episode stats.

The reference logs episode returns / lengths through SB3's VecMonitor around its SubprocVecEnv
(neural/agent.py:63-82), one host-side info dict per env step.  Here the step kernel adds every
finished episode to per-env device accumulators (b747_env_batch.ep_stats: count, return sum,
length sum; written on done lanes only, so the per-step path pays nothing), and `collect()` reduces
them every M steps: a sum over the envs of this rank, then ONE all-reduce of 3 doubles over the
ranks (RCCL over xGMI with the nccl backend, 24 B) -- no collective on the env-step path itself.
"""
from typing import Optional

import torch
import torch.distributed as dist


def reduce_episode_stats(local: torch.Tensor, group=None) -> torch.Tensor:
    """Sum a rank's [3] (episodes, return sum, length sum) over every rank of `group` (in place;
    a no-op without an initialised process group or with one rank)."""
    if dist.is_available() and dist.is_initialized() and dist.get_world_size(group) > 1:
        dist.all_reduce(local, op=dist.ReduceOp.SUM, group=group)
    return local


def summarize(totals) -> dict:
    """{episodes, mean_return, mean_length} from summed (episodes, return sum, length sum)."""
    count, ret, length = (float(v) for v in totals)
    return {"episodes": int(round(count)), "mean_return": ret / count if count else float("nan"),
            "mean_length": length / count if count else float("nan")}


class EpisodeStats:
    """Turns on the env's episode accumulators and reduces them on demand."""

    def __init__(self, env, group=None):
        self.env, self.group = env, group
        env.track_episodes(True)

    def collect(self, reset: bool = True, stream: Optional[torch.cuda.Stream] = None) -> dict:
        """Episodes finished since the last collect (all envs, all ranks): count, mean return and mean
        length.  Synchronises the calling stream with the host (one 24-byte read-back)."""
        acc = self.env.ep_stats
        local = acc.sum(dim=1)
        if dist.is_available() and dist.is_initialized() and dist.get_backend(self.group) == "gloo":
            local = local.cpu()
        totals = reduce_episode_stats(local, self.group)
        if reset:
            acc.zero_()
        return summarize(totals.tolist())
