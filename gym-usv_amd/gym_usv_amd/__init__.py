"""gym_usv_amd — MI355X-native batched USV path-following environment.

Registry mirroring gym_usv/__init__.py:3-39 for the ids on the accelerated path:

    make("usv-simple")                         -> UsvSimpleEnv with TimeLimit(500)
    make("usv-asmc-simple")                    -> UsvSimpleASMCEnv with TimeLimit(1000)
    make("usv-asmc-v0")                        -> legacy UsvAsmcEnv (old gym API, no TimeLimit)
    make("usv-pid-v0")                         -> legacy UsvPidEnv (float64 PID plant)
    make("usv-asmc-ye-int-v0")                 -> legacy UsvAsmcYeIntEnv (float64, ye integral)
    make_vec("usv-simple", num_envs=65536)     -> UsvVectorEnv (one HIP launch per step)
    make_sb3_vec_env("usv-simple", 4096, 5)    -> SB3 VecEnv (NumPy out, Monitor infos, VecFrameStack(5))

The compute lives in libusvhip.so (HIP, gfx950) behind the C-ABI in include/usv_hip.h.
"""
from ._lib import UsvLibError, load as load_library  # noqa: F401
from .vector_env import ENV_SPECS, UsvVectorEnv  # noqa: F401

__all__ = ["make", "make_vec", "make_sb3_vec_env", "registry", "UsvVectorEnv", "UsvLibError", "ENV_SPECS"]

registry = {k: {"entry_point": f"gym_usv_amd.envs:{cls}", "max_episode_steps": v[1] or None}
            for (k, v), cls in zip(ENV_SPECS.items(), ("UsvSimpleEnv", "UsvSimpleASMCEnv", "UsvAsmcEnv",
                                                       "UsvPidEnv", "UsvAsmcYeIntEnv"))}


def make(env_id, max_episode_steps=None, **kwargs):
    from . import envs
    cls = {"usv-simple": envs.UsvSimpleEnv, "usv-asmc-simple": envs.UsvSimpleASMCEnv,
           "usv-asmc-v0": envs.UsvAsmcEnv, "usv-pid-v0": envs.UsvPidEnv,
           "usv-asmc-ye-int-v0": envs.UsvAsmcYeIntEnv}[env_id]
    limit = registry[env_id]["max_episode_steps"] if max_episode_steps is None else max_episode_steps
    limit = limit or 0
    return cls(max_episode_steps=limit, **kwargs)


def make_vec(env_id, num_envs, **kwargs):
    return UsvVectorEnv(env_id, num_envs=num_envs, **kwargs)


def make_sb3_vec_env(env_id, n_envs, frame_stack=0, seed=0, **kwargs):
    """SB3 ``VecEnv`` counterpart of ``VecFrameStack(make_vec_env(env_id, n_envs), frame_stack)``
    (train_test/sb3_train_vec.py:67-70): one HIP-stepped batch with Monitor/TimeLimit infos."""
    from .sb3 import Sb3VecEnv
    return Sb3VecEnv(env_id, num_envs=n_envs, frame_stack=frame_stack, seed=seed, **kwargs)
