"""Multi-process (world size 2, gloo, CPU) coverage of the N>1 path.

The env batch shards over GPUs by contiguous global env ids with no data-path collective
(SURVEY.md 8e).  What must hold for that to be correct, checked here on the CPU:
  * every rank's shard draws exactly the episodes the same global envs get in one big batch
    (Philox streams keyed by seed x global env id -- host build of b747_env.h's draw_reset);
  * every rank STEPS its shard (host build of the product's per-lane dynamics and env read-out,
    tests/native/hostcheck.cpp b747h_bench_shard) across several auto-resets, and the gathered
    shards are bit-identical to stepping the whole batch in one process;
  * the bench's timing reduction is a MAX over ranks and the aggregate throughput sums ranks
    (bench.reduce_max, bench.aggregate_rate).
On hardware the same split runs one rank per MI355X (tests/test_gpu_fullsize.py checks 8 device
shards against one device batch); 8-GPU timing itself is unmeasured here.
"""
import os
import socket

import numpy as np
import torch
import torch.distributed as dist
import torch.multiprocessing as mp

import oracle_lib as O

N_PER_RANK, SEED = 4096, 1234


def _draws(offset, n, episode=0, mode=0, dist_mode=0):
    return O.draw_resets(SEED, offset, n, episode, mode, dist_mode)


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    s0, ref, ae, _ = _draws(rank * N_PER_RANK, N_PER_RANK, episode=3, mode=1, dist_mode=0)
    t = torch.from_numpy(np.concatenate([s0.ravel(), ref.ravel().astype(np.float64), ae.ravel().astype(np.float64)]))
    out = [torch.zeros_like(t) for _ in range(world)]
    dist.all_gather(out, t)
    import bench
    wall = bench.reduce_max(0.5 + rank, dist, torch.device("cpu"))
    if rank == 0:
        q.put((torch.cat(out).numpy(), wall))
    dist.barrier()
    dist.destroy_process_group()


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_two_rank_shards_reproduce_the_single_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, wall = q.get(timeout=120)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    s0, ref, ae, _ = _draws(0, world * N_PER_RANK, episode=3, mode=1, dist_mode=0)
    per = [np.concatenate([s0[r * N_PER_RANK:(r + 1) * N_PER_RANK].ravel(),
                           ref[r * N_PER_RANK:(r + 1) * N_PER_RANK].ravel().astype(np.float64),
                           ae[r * N_PER_RANK:(r + 1) * N_PER_RANK].ravel().astype(np.float64)]) for r in range(world)]
    assert np.array_equal(gathered, np.concatenate(per))
    assert wall == 1.5                                   # max over ranks (0.5, 1.5)


def test_draw_distributions_match_controller_reset():
    """core/controller.py:148-191 distributions for CONST / OSCILLATING / HYBRID + AERO."""
    n = 200000
    s0, ref, ae, fl = _draws(0, n, mode=0, dist_mode=0)
    vmax = 10 * np.pi / 180
    assert s0[:, 1].min() >= 1000 and s0[:, 1].max() <= 11000 and abs(s0[:, 1].mean() - 6000) < 30
    assert s0[:, 2].min() >= 100 and s0[:, 2].max() <= 265 and abs(s0[:, 3].mean()) < 0.2
    assert np.abs(s0[:, 5]).max() <= 1e-3 and np.all(s0[:, 0] == 0) and np.all(s0[:, 4] == 0)
    r = ref[:, 0]
    assert np.abs(r).min() >= np.float32(np.pi / 180) * (1 - 1e-6) and np.abs(r).max() <= np.float32(vmax) * (1 + 1e-6)
    assert abs((r > 0).mean() - 0.5) < 0.01
    assert np.allclose(ae.mean(0), [-0.1, 0.1, -0.1, -0.1, 0.1], atol=0.01) and np.allclose(ae.std(0), 0.5, atol=0.01)
    _, ref, _, _ = _draws(0, n, mode=1, dist_mode=-1)
    A = ref[:, 1:4].astype(np.float64)
    assert np.all(A >= 0) and np.all(A.sum(1) <= vmax * (1 + 1e-6))
    assert ref[:, 4:7].min() >= 0.01 - 1e-7 and ref[:, 4:7].max() <= 0.5 + 1e-7
    s0, ref, ae, fl = _draws(0, n, mode=2, dist_mode=-1)
    cs = (fl & 2) != 0
    assert abs(cs.mean() - 0.5) < 0.01
    assert np.all(np.abs(ref[cs, 7] - s0[cs, 1]) <= 1000 + 1e-3)
    assert np.all(np.abs(ref[~cs, 0]) <= vmax)
    assert np.all(ae == 0)


STEP_N, STEP_T, STEP_TK = 256, 300, 1.0           # 100 env steps per episode: 3 auto-resets per env


def _actions(world):
    """The full-width action stream (every rank slices its envs out of it)."""
    return np.random.default_rng(77).uniform(-1, 1, (STEP_T, world * STEP_N)).astype(np.float32)


def _step_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import time
    t0 = time.perf_counter()
    a = _actions(world)[:, rank * STEP_N:(rank + 1) * STEP_N]
    X, k, ep, obs, rew, done, ret = O.bench_shard(STEP_N, rank * STEP_N, SEED, STEP_TK, a)
    local = torch.from_numpy(np.concatenate([X.ravel(), k.astype(np.float64), ep.astype(np.float64),
                                             obs.ravel().astype(np.float64), rew.astype(np.float64),
                                             done.astype(np.float64), ret]))
    out = [torch.zeros_like(local) for _ in range(world)]
    dist.all_gather(out, local)
    import bench
    wall = bench.reduce_max(time.perf_counter() - t0, dist, torch.device("cpu"))
    if rank == 0:
        q.put((torch.stack(out).numpy(), wall, bench.aggregate_rate(STEP_N, STEP_T, world, wall)))
    dist.barrier()
    dist.destroy_process_group()


def test_two_ranks_step_their_shards_bit_identical_to_one_batch():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_step_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    gathered, wall, rate = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    X, k, ep, obs, rew, done, ret = O.bench_shard(world * STEP_N, 0, SEED, STEP_TK, _actions(world))
    assert np.all(ep == 4) and np.isfinite(X).all()                   # 1 reset + 3 auto-resets per env
    for r in range(world):
        sl = slice(r * STEP_N, (r + 1) * STEP_N)
        ref = np.concatenate([X[:, sl].ravel(), k[sl].astype(np.float64), ep[sl].astype(np.float64),
                              obs[sl].ravel().astype(np.float64), rew[sl].astype(np.float64),
                              done[sl].astype(np.float64), ret[sl]])
        assert np.array_equal(gathered[r].view(np.int64), ref.view(np.int64)), f"rank {r} shard differs"
    assert wall > 0 and rate == world * STEP_N * STEP_T / wall          # whole-job env-steps/s (weak scaling)


# ------------------------------------------------------------------ SURVEY 8(e) optional collectives --
class _HostEnv:
    """What PPO.train reads of an env (the rollout buffers are filled by the test)."""

    class _Box:
        low, high = -1.0, 1.0

    def __init__(self, n, obs_dim=3, env_offset=0, seed=0):
        self.n, self.obs_dim, self.device, self.action_space = n, obs_dim, torch.device("cpu"), self._Box()
        self.env_offset = env_offset
        self.cfg = type("Cfg", (), {"seed": seed})()     # b747_env_config.seed: a uint64 Philox key


def _fill_rollout(ppo, T, seed):
    g = torch.Generator().manual_seed(seed)
    for buf in (ppo.obs_buf, ppo.act_buf, ppo.logp_buf, ppo.val_buf, ppo.rew_buf):
        buf.copy_(torch.randn(buf.shape, generator=g))
    ppo.done_buf.copy_(torch.rand(ppo.done_buf.shape, generator=g) < 0.05)
    ppo.last_obs.copy_(torch.randn(ppo.last_obs.shape, generator=g))
    ppo.compute_gae(T)


def _flat(module):
    return torch.cat([p.detach().reshape(-1) for p in module.parameters()])


def _ppo_worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from b747_rl_ctrl_amd.episode_stats import reduce_episode_stats, summarize
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig, allreduce_gradients
    T, n = 8, 64
    cfg = PPOConfig(n_steps=T, n_epochs=2, batch_size=128)
    # different seeds per rank: the broadcast must still start every rank from rank 0's parameters
    ppo = PPO(_HostEnv(n, env_offset=rank * n), cfg, seed=10 + rank, fused=False)
    assert ppo.data_parallel
    # shard checks: duplicate env ids and unequal counts are refused on every rank, together
    refused = []
    for bad in (_HostEnv(n, env_offset=0), _HostEnv(n + 64 * rank, env_offset=rank * 4096)):
        try:
            PPO(bad, cfg, seed=10, fused=False)
        except ValueError as e:
            refused.append("overlapping" in str(e) or "counts differ" in str(e))
    assert refused == [True, True], refused
    # a reset seed >= 2**63 (the uint64 key packed into an int64 tensor) constructs on every rank
    assert PPO(_HostEnv(n, env_offset=rank * n, seed=2 ** 64 - 1), cfg, seed=10, fused=False).data_parallel
    start = _flat(ppo.policy)
    _fill_rollout(ppo, T, seed=100 + rank)          # each rank's own shard of experience
    torch.manual_seed(5 + rank)                      # rank-local minibatch permutations
    ppo.train(T)
    after = _flat(ppo.policy)
    # the bucketed all-reduce itself: gradients rank + 1 average to (1 + world) / 2
    lin = torch.nn.Linear(4, 3)
    for p in lin.parameters():
        p.grad = torch.full_like(p, float(rank + 1))
    allreduce_gradients(lin.parameters())
    grads = torch.cat([p.grad.reshape(-1) for p in lin.parameters()])
    # episode statistics: rank r finished r + 2 episodes of return 10 (r + 1) and length 100 each
    stats = reduce_episode_stats(torch.tensor([rank + 2.0, 10.0 * (rank + 1) * (rank + 2), 100.0 * (rank + 2)],
                                              dtype=torch.float64))
    both = torch.cat([start, after])
    out = [torch.zeros_like(both) for _ in range(world)]
    dist.all_gather(out, both)
    if rank == 0:
        q.put((torch.stack(out).numpy(), grads.numpy(), summarize(stats.tolist())))
    dist.barrier()
    dist.destroy_process_group()


def test_data_parallel_ppo_ranks_stay_in_lockstep_and_episode_stats_reduce():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_ppo_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    params, grads, stats = q.get(timeout=180)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    half = params.shape[1] // 2
    start, after = params[:, :half], params[:, half:]
    assert np.array_equal(start[0], start[1])                  # broadcast from rank 0
    assert np.array_equal(after[0], after[1])                  # identical averaged updates on both ranks
    assert not np.array_equal(after[0], start[0])              # and training did move the policy
    # reference: rank 0 alone on its own shard ends elsewhere (the other rank's gradients mattered)
    from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
    T = 8
    solo = PPO(_HostEnv(64), PPOConfig(n_steps=T, n_epochs=2, batch_size=128), seed=10, fused=False)
    assert not solo.data_parallel
    _fill_rollout(solo, T, seed=100)
    torch.manual_seed(5)
    solo.train(T)
    assert not np.allclose(_flat(solo.policy).numpy(), after[0])
    assert np.all(grads == 1.5)
    assert stats["episodes"] == 5 and stats["mean_length"] == 100.0
    assert abs(stats["mean_return"] - (10 * 1 * 2 + 10 * 2 * 3) / 5) < 1e-12
