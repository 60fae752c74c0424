"""Import harness for the read-only reference (romi2002/gym-usv) — THIS CONTAINER ONLY.

Test infrastructure, never shipped to the GPU box and never imported by the product
package.  It registers minimal stand-in modules for the reference's uninstalled
third-party imports so that the reference's own files under /root/reference run
unmodified:

* ``gymnasium``   -- ``Env`` with the gymnasium seeding rule
                     ``np_random = Generator(PCG64(SeedSequence(seed)))``, ``spaces.Box``,
                     ``register`` (records kwargs).
* ``gym``         -- old-API ``Env`` / ``spaces`` / ``utils.seeding`` (usv_asmc_env.py:9-11).
* ``numba``       -- ``njit`` = identity (same float64 semantics, just slower).
* ``pygame``      -- attribute sink (renderers are never called with render_mode=None).
* ``usv_libs_py`` -- placeholders; AITSMC / usv-asmc-ca-v0 dynamics stay unpinned.

NumPy >= 2 removed ``np.math``; the reference uses it (usv_asmc.py:72), so it is
re-attached here.  Nothing in the reference is edited or copied.
"""
from __future__ import annotations

import math
import sys
import types

import numpy as np

REF_ROOT = "/root/reference"


class _Sink(types.ModuleType):
    """Module whose every attribute is a callable sink (pygame stand-in)."""

    def __getattr__(self, name):  # pragma: no cover - only hit by renderers
        if name.startswith("__"):
            raise AttributeError(name)
        return _Sink(name)

    def __call__(self, *a, **k):  # pragma: no cover
        return _Sink("call")


class Box:
    def __init__(self, low=None, high=None, shape=None, dtype=np.float32):
        self.low, self.high, self.dtype = low, high, dtype
        if shape is None and low is not None:
            shape = np.shape(low)
        self.shape = tuple(shape) if shape is not None else ()


def _install_stubs():
    if getattr(sys.modules.get("gymnasium"), "_graft_stub", False):
        return

    # --- gymnasium -----------------------------------------------------------------
    gymnasium = types.ModuleType("gymnasium")
    gymnasium._graft_stub = True
    spaces = types.ModuleType("gymnasium.spaces")
    spaces.Box = Box
    registry = {}

    def register(id, entry_point=None, **kwargs):
        registry[id] = dict(entry_point=entry_point, **kwargs)

    class Env:
        _np_random = None

        @property
        def np_random(self):
            if self._np_random is None:
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(None)))
            return self._np_random

        def reset(self, *, seed=None, options=None):
            if seed is not None:
                self._np_random = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
            return None

    gymnasium.Env = Env
    gymnasium.spaces = spaces
    gymnasium.register = register
    gymnasium.registry = registry
    sys.modules["gymnasium"] = gymnasium
    sys.modules["gymnasium.spaces"] = spaces

    # --- gym (old API, legacy envs) ---------------------------------------------------
    gym = types.ModuleType("gym")
    gym_spaces = types.ModuleType("gym.spaces")
    gym_spaces.Box = Box
    gym_utils = types.ModuleType("gym.utils")
    gym_seeding = types.ModuleType("gym.utils.seeding")
    gym_utils.seeding = gym_seeding
    gym.Env = type("Env", (), {})
    gym.spaces = gym_spaces
    gym.utils = gym_utils
    gym.error = types.ModuleType("gym.error")
    sys.modules.update({"gym": gym, "gym.spaces": gym_spaces, "gym.utils": gym_utils,
                        "gym.utils.seeding": gym_seeding, "gym.error": gym.error})

    # --- numba ----------------------------------------------------------------------
    numba = types.ModuleType("numba")
    numba.njit = lambda f=None, **k: (f if f is not None else (lambda g: g))
    sys.modules["numba"] = numba

    # --- pygame ---------------------------------------------------------------------
    pygame = _Sink("pygame")
    sys.modules["pygame"] = pygame

    # --- usv_libs_py (absent external C++ lib) -------------------------------------------
    usv = types.ModuleType("usv_libs_py")
    usv.controller = types.ModuleType("usv_libs_py.controller")
    usv.model = types.ModuleType("usv_libs_py.model")
    usv.controller.ASMC = type("ASMC", (), {})
    usv.controller.AITSMC = type("AITSMC", (), {})
    usv.model.DynamicModel = type("DynamicModel", (), {})
    sys.modules.update({"usv_libs_py": usv, "usv_libs_py.controller": usv.controller,
                        "usv_libs_py.model": usv.model})


def load_reference():
    """Return the reference ``gym_usv`` package (imported read-only from /root/reference)."""
    np.math = math  # NumPy 2 removed np.math; usv_asmc.py:72, usv_asmc_env.py:234 use it
    _install_stubs()
    if REF_ROOT not in sys.path:
        sys.path.insert(0, REF_ROOT)
    import gym_usv  # noqa: F401  (registers ids via the stub)
    import gym_usv.envs  # noqa: F401
    import gym_usv.control  # noqa: F401
    return sys.modules["gym_usv"]
