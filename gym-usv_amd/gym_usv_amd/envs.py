"""Single-env classes with the reference's Gymnasium ``Env`` API, backed by the HIP library.

``UsvSimpleEnv`` / ``UsvSimpleASMCEnv`` keep the reference names and call signatures
(gym_usv/envs/simple_env.py:7, simple_env_asmc.py:7): ``reset(seed=None, options=None) ->
(obs float32[143], info)`` and ``step(action) -> (obs, reward, terminated, truncated, info)``
with NumPy in/out.  Each is a 1-env ``UsvVectorEnv`` with autoreset off and no TimeLimit
(``gym_usv_amd.make`` adds the registered TimeLimit, like ``gymnasium.make``).  By default
(``reset_rng="numpy"``) a usv-simple / usv-asmc-simple env draws its resets from
``Generator(PCG64(SeedSequence(seed)))`` exactly like the reference (the legacy ids from np.random's
MT19937 after ``np.random.seed(seed)``), so ``make(id).reset(seed=s)`` followed by the same actions
reproduces the reference's episode; ``reset_rng="philox"`` selects the in-kernel Philox resets of the
vector env.  They exist for API compatibility and debugging; throughput lives in ``UsvVectorEnv``.
"""
from __future__ import annotations

import numpy as np
import torch

from .vector_env import LEGACY_IDS, UsvVectorEnv


class _SingleEnv:
    env_id = None
    metadata = {"render_modes": [], "render_fps": 30}

    def __init__(self, render_mode=None, options=None, device=0, precision="f32",
                 max_episode_steps=0, seed=None, reset_rng="numpy", obstacle_cap=32, perturb=False):
        if render_mode not in (None, "rgb_array"):
            raise NotImplementedError("render_mode 'human' (a pygame window) is out of scope; use 'rgb_array'")
        self.render_mode = render_mode
        self.options = options or {}
        self._venv = UsvVectorEnv(self.env_id, num_envs=1, device=device, precision=precision,
                                  autoreset=False, max_episode_steps=max_episode_steps,
                                  seed=0 if seed is None else seed, reset_rng=reset_rng,
                                  obstacle_cap=obstacle_cap, options=self.options, info=True,
                                  perturb=perturb)
        self.observation_space = self._venv.single_observation_space
        self.action_space = self._venv.single_action_space
        self._seeded = False

    def reset(self, seed=None, options=None):
        if seed is None and not self._seeded:
            # an unseeded first reset draws fresh entropy (gymnasium's np_random(None)); the legacy ids
            # seed np.random's MT19937, which takes seeds below 2**32 only (usv_asmc_env.py:258)
            bound = 1 << (32 if self.env_id in LEGACY_IDS else 63)
            seed = int(np.random.SeedSequence().entropy % bound)
        if seed is not None:
            self._seeded = True
        obs, info = self._venv.reset(seed=seed, options=options)
        return obs[0].cpu().numpy(), self._host_info(info)

    def step(self, action):
        a = torch.as_tensor(np.asarray(action, dtype=np.float32).reshape(1, self._venv.act_dim),
                            device=self._venv.device)
        obs, rew, term, trunc, info = self._venv.step(a)
        return (obs[0].cpu().numpy(), float(rew[0].item()), bool(term[0].item()),
                bool(trunc[0].item()), self._host_info(info))

    @staticmethod
    def _host_info(info):
        """The reference's info dict for env 0 (simple_env.py:102-115, 189-199): arrays for
        position / velocity / path_start / path_end, Python floats for the rest."""
        out = {}
        for k, v in info.items():
            if k in ("final_obs", "_final_obs"):
                continue
            x = v[0].detach().cpu().numpy().astype(np.float64)
            out[k] = x if x.ndim else float(x)
        return out

    def render(self):
        """simple_env.py:117-119: an rgb_array frame when render_mode == "rgb_array"."""
        if self.render_mode == "rgb_array":
            return self._venv.render(0)
        return None

    def close(self):
        self._venv.close()


class UsvSimpleEnv(_SingleEnv):
    """HIP-backed ``UsvSimpleEnv`` (id usv-simple)."""
    env_id = "usv-simple"


class UsvSimpleASMCEnv(_SingleEnv):
    """HIP-backed ``UsvSimpleASMCEnv`` (id usv-asmc-simple)."""
    env_id = "usv-asmc-simple"


class UsvAsmcEnv(_SingleEnv):
    """HIP-backed legacy ``UsvAsmcEnv`` (id usv-asmc-v0, usv_asmc_env.py:14) with the reference's
    old gym API: ``reset() -> obs`` and ``step(action) -> (obs, reward, done, info)``."""
    env_id = "usv-asmc-v0"

    def reset(self, seed=None, options=None):
        obs, _ = super().reset(seed=seed, options=options)
        return obs

    def step(self, action):
        obs, r, term, trunc, info = super().step(action)
        return obs, r, term or trunc, info


class UsvPidEnv(UsvAsmcEnv):
    """HIP-backed legacy ``UsvPidEnv`` (id usv-pid-v0, usv_pid_env.py:14), old gym API."""
    env_id = "usv-pid-v0"


class UsvAsmcYeIntEnv(UsvAsmcEnv):
    """HIP-backed legacy ``UsvAsmcYeIntEnv`` (id usv-asmc-ye-int-v0, usv_asmc_ye_int_env.py:14),
    old gym API."""
    env_id = "usv-asmc-ye-int-v0"
