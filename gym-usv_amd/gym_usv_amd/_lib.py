"""ctypes binding of libusvhip.so (C-ABI declared in include/usv_hip.h).

The library is built in-tree (``__graft_entry__.build()`` / ``python -m gym_usv_amd.build``)
and loaded from this package directory.  There is no fallback: if the HIP library is missing
or fails to load, every env constructor raises ``UsvLibError``.
"""
from __future__ import annotations

import ctypes
import os

LIB_NAME = "libusvhip.so"
LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), LIB_NAME)
# diagnostic builds (tools/) may point at another in-tree copy of the library
LIB_PATH = os.environ.get("USV_LIB_PATH", LIB_PATH)

ABI_VERSION = 5
MODE_SIMPLE, MODE_ASMC_SIMPLE, MODE_ASMC_V0, MODE_ASMC_YE_INT_V0, MODE_PID_V0 = 0, 1, 2, 3, 4
F32, F64 = 0, 1
AUTORESET_SAME_STEP, AUTORESET_DISABLED = 0, 1
LIDAR_BRUTE, LIDAR_WINDOW = 0, 1
RESET_PHILOX, RESET_NUMPY_PCG64 = 0, 1
OBS_DIM, SENSOR_COUNT, ACT_DIM, ASMC_STATE = 143, 128, 2, 16
FLAG_PERTURB = 1
# usv_info_key order (include/usv_hip.h): reference info keys (simple_env.py:102-115, 189-199) -> column
INFO_KEYS = ("x", "y", "psi", "u", "v", "r", "path_x0", "path_y0", "path_x1", "path_y1", "action0",
             "action1", "ye", "angle_to_target", "ye_reward", "angle_to_target_reward",
             "delta_action_reward", "delta_action", "velocity_track_reward", "reference_velocity",
             "reward_velocity", "reference_velocity_error")
INFO_DIM = len(INFO_KEYS)
EXP_MAX_OBS = 64


class UsvLibError(RuntimeError):
    pass


class UsvConfig(ctypes.Structure):
    _fields_ = [("abi_version", ctypes.c_int32), ("mode", ctypes.c_int32),
                ("precision", ctypes.c_int32), ("num_envs", ctypes.c_int32),
                ("obstacle_cap", ctypes.c_int32), ("max_episode_steps", ctypes.c_int32),
                ("autoreset", ctypes.c_int32), ("lidar_algo", ctypes.c_int32),
                ("seed", ctypes.c_uint64), ("env_id_offset", ctypes.c_uint64),
                ("flags", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class UsvResetOptions(ctypes.Structure):
    _fields_ = [("place_obstacles_on_path", ctypes.c_int32), ("reserved", ctypes.c_int32)]


class UsvExperiment(ctypes.Structure):
    _fields_ = [("n_obs", ctypes.c_int32), ("reserved", ctypes.c_int32),
                ("obstacle_x", ctypes.c_double * EXP_MAX_OBS), ("obstacle_y", ctypes.c_double * EXP_MAX_OBS),
                ("obstacle_r", ctypes.c_double * EXP_MAX_OBS), ("path_start", ctypes.c_double * 2),
                ("angle", ctypes.c_double), ("position", ctypes.c_double * 3)]


# (name, restype, argtypes) for every function in include/usv_hip.h
_vp, _i32, _u64, _sz = ctypes.c_void_p, ctypes.c_int32, ctypes.c_uint64, ctypes.c_size_t
SIGNATURES = [
    ("usv_abi_version", ctypes.c_int, []),
    ("usv_last_error", ctypes.c_char_p, []),
    ("usv_config_default", None, [ctypes.POINTER(UsvConfig), _i32, _i32]),
    ("usv_create", ctypes.c_int, [ctypes.POINTER(UsvConfig), _i32, ctypes.POINTER(_vp)]),
    ("usv_destroy", None, [_vp]),
    ("usv_num_envs", ctypes.c_int, [_vp]),
    ("usv_obs_dim", ctypes.c_int, [_vp]),
    ("usv_act_dim", ctypes.c_int, [_vp]),
    ("usv_reward_bytes", ctypes.c_int, [_vp]),
    ("usv_seed", ctypes.c_int, [_vp, _u64]),
    ("usv_set_reset_rng", ctypes.c_int, [_vp, _i32]),
    ("usv_reset", ctypes.c_int, [_vp, _vp, _vp, _vp]),
    ("usv_reset_ex", ctypes.c_int, [_vp, _vp, _vp, ctypes.POINTER(UsvResetOptions), _vp, _vp]),
    ("usv_set_experiment", ctypes.c_int, [_vp, ctypes.POINTER(UsvExperiment)]),
    ("usv_step", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("usv_step_ex", ctypes.c_int, [_vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp, _vp]),
    ("usv_field_info", ctypes.c_int, [_vp, _i32, ctypes.POINTER(_i32), ctypes.POINTER(_i32),
                                      ctypes.POINTER(ctypes.c_char_p)]),
    ("usv_get_field", ctypes.c_int, [_vp, _i32, _vp, _sz]),
    ("usv_set_field", ctypes.c_int, [_vp, _i32, _vp, _sz]),
    ("usv_state_bytes", _sz, [_vp]),
    ("usv_get_state", ctypes.c_int, [_vp, _vp, _sz]),
    ("usv_set_state", ctypes.c_int, [_vp, _vp, _sz]),
    ("usv_set_kernel_variant", ctypes.c_int, [_vp, _i32, _i32, _i32]),
    ("usv_config_size", _sz, []),
    ("usv_asmc_compute", ctypes.c_int, [_i32, _i32, _vp, _vp, _vp, _vp, _vp, _i32, _i32, _vp]),
]

_LIBS = {}


def load(path=None):
    """Load (once per path) and return the HIP library; raise UsvLibError if it is unavailable.
    ``path`` selects another build of the same C-ABI (e.g. libusvhip_safe.so); each path is its
    own ctypes handle (RTLD_LOCAL), so two builds can be used side by side."""
    path = path or LIB_PATH
    if path in _LIBS:
        return _LIBS[path]
    if not os.path.exists(path):
        raise UsvLibError(f"{path} not built: run `python -c 'import __graft_entry__ as g; g.build()'`")
    try:
        lib = ctypes.CDLL(path)
    except OSError as e:  # pragma: no cover
        raise UsvLibError(f"cannot load {path}: {e}") from e
    for name, res, args in SIGNATURES:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    if lib.usv_abi_version() != ABI_VERSION:
        raise UsvLibError("libusvhip ABI version mismatch")
    if lib.usv_config_size() != ctypes.sizeof(UsvConfig):
        raise UsvLibError(f"usv_config is {lib.usv_config_size()} B in the library, "
                          f"{ctypes.sizeof(UsvConfig)} B in this binding")
    _LIBS[path] = lib
    return lib


SAFE_LIB_PATH = os.path.join(os.path.dirname(os.path.abspath(__file__)), "libusvhip_safe.so")


def check(rc, lib=None):
    if rc != 0:
        msg = (lib or load()).usv_last_error().decode(errors="replace")
        raise UsvLibError(f"libusvhip error {rc}: {msg}")
    return rc
