"""b747_rl_ctrl_amd -- MI355X-native batched B747 pitch-control environment.

Drop-in for the hot path of kllmagn/B747_RL_CTRL: the Simulink dynamics behind core/model.py
(model_simple_win64.dll) and the env/ctrl_env.py step()/reset() loop, re-derived as HIP kernels
(libb747.so, C ABI in include/b747.h) that advance N environments per launch.
"""
from ._lib import B747Error, F_PID_CS, F_PID_SS, F_RL, F_RP  # noqa: F401
from .model import BatchModel  # noqa: F401
from .ctrl_env import (BatchControllerEnv, CtrlMode, CtrlType, DisturbanceMode, ObservationType,  # noqa: F401
                       ResetRefMode, RewardType)
from .vec_env import B747GymVectorEnv, B747VecEnv, ep_rew_mean, make_vec_env  # noqa: F401
from .storage import BatchStorage, Storage  # noqa: F401

__version__ = "0.1.0"
