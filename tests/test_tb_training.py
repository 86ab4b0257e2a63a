"""The reference's recorded training run replayed through the product's PPO and the oracle env (CPU); see
tests/tb_training.py.  The first iterations track the record to float32 rounding: SB3's test metrics and episode
returns bit for bit or within 1e-6, the update's loss statistics within 1e-5 relative (approx_kl and the
policy-gradient loss, means of small signed terms, within 1e-4; the explained variance, a difference near 0,
within 1e-5 absolute).  The full 62-iteration report is profiles/r04/tb_training_replay_oracle.txt (the
float32 differences between the reference's torch 1.10 / Windows and this torch grow through the 62 updates of
chaotic PPO training: ~1e-7 in the first iterations, ~1e-4 - 1e-3 by the end)."""
import pytest

import tb_training as TT

RUN = "PID_LIKE_MANUAL_ADD_DIRECT_CONTROL_CONST_None_2"
ITERATIONS = 2
@pytest.fixture(scope="module")
def replay():
    rp = TT.TrainingReplay(RUN, "oracle")
    return rp, [rp.step_iteration() for _ in range(ITERATIONS)]


def test_first_iterations_track_the_record(replay):
    rec = TT.load_curves(RUN)
    _, entries = replay
    exact = total = 0
    for step, entry in entries:
        cmp_ = TT.check_entry(entry, rec, step)
        exact += sum(c[2] for c in cmp_.values())
        total += len(cmp_)
    assert total == 4 + 12 and exact >= 9        # measured 10 of 16 float32-equal

