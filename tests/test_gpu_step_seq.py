"""b747_env_step_seq (K per-step launches from one C call) == K step() calls, bit for bit, across an
auto-reset (GPU).  The sequence entry point is the bench's launch path for short timed regions."""
import pytest
import torch

pytestmark = pytest.mark.gpu


def _env(n, seed=5):
    import bench
    return bench.make_env(n, 0, True, torch.device("cuda", 0))


@pytest.mark.parametrize("n", [1000, 65536])
def test_step_seq_equals_step_loop(n):
    T = 40
    a = _env(n)
    b = _env(n)
    g = torch.Generator(device="cuda").manual_seed(11)
    acts = torch.rand(T, n, generator=g, device="cuda") * 2 - 1
    # move both envs near the episode end so that the sequence crosses auto-resets
    for env in (a, b):
        env.k.fill_(1985)
    for t in range(T):
        a.step(acts[t])
    b.step_seq(acts)
    torch.cuda.synchronize()
    assert int(a.done.sum().item()) == int(b.done.sum().item())
    for name in ("X", "disc", "k", "obs", "reward", "done", "ep_return", "episode", "terminal_obs"):
        ta, tb = getattr(a, name), getattr(b, name)
        assert torch.equal(ta, tb), name
    b.step_seq(acts[:0])   # empty sequence: no launch
