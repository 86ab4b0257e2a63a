import time, torch, sys
sys.path.insert(0, '.')
import bench
from b747_rl_ctrl_amd.ppo import PPO, PPOConfig
dev = torch.device('cuda', 0)
env = bench.make_env(65536, 0, True, dev, seed=99, variant='fast')
ppo = PPO(env, PPOConfig(n_steps=64), seed=0)
ppo.last_obs.copy_(env.obs)
ppo.collect_rollouts(64); torch.cuda.synchronize()
for _ in range(3):
    t0 = time.perf_counter(); k = ppo._graph_key(64); t1 = time.perf_counter()
    ppo._graph.replay(); t2 = time.perf_counter(); torch.cuda.synchronize(); t3 = time.perf_counter()
    print(f"graph_key {1e6*(t1-t0):.1f} us  replay host {1e6*(t2-t1):.1f} us  to sync {1e6*(t3-t2):.1f} us  total {1e6*(t3-t0):.1f}")
for _ in range(3):
    t0 = time.perf_counter(); ppo.collect_rollouts(64); t1 = time.perf_counter(); torch.cuda.synchronize(); t2 = time.perf_counter()
    print(f"collect host {1e6*(t1-t0):.1f} us total {1e6*(t2-t0):.1f} us -> {1e6*(t2-t0)/64:.3f} us/step")
