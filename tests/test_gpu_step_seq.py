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


@pytest.mark.parametrize("src", ["host_f32", "device_f64"])
@pytest.mark.parametrize("entry", ["rollout", "step_seq"])
def test_converted_actions_on_a_side_stream_are_ordered(entry, src):
    """rollout / step_seq on an explicit, busy side stream with actions that need a conversion (a freshly
    allocated host tensor, or a float64 device tensor): the converted temporary must be made on the launch
    stream.  Made on the current stream, it returns to that stream's pool when the call
    returns, and the junk tensor allocated right after reuses its block and overwrites it while the kernel
    still waits behind torch.cuda._sleep on the side stream."""
    n, T = 4096, 16
    ref, env = _env(n), _env(n)
    acts = torch.rand(T, n, generator=torch.Generator().manual_seed(3)) * 2 - 1      # host tensor
    getattr(ref, entry)(acts.cuda())         # the same entry point, device float32 actions, current stream
    torch.cuda.synchronize()
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        torch.cuda._sleep(100_000_000)      # the side stream is busy when the call enqueues on it
    fresh = acts.clone() if src == "host_f32" else acts.to("cuda", torch.float64)
    getattr(env, entry)(fresh, stream=s)
    junk = torch.full((T, n), 0.75, device="cuda")   # current stream: reuses a block it freed, if any
    torch.cuda.synchronize()
    del junk
    for name in ("X", "disc", "k", "obs", "reward", "done", "episode", "ep_return"):
        assert torch.equal(getattr(ref, name), getattr(env, name)), name
