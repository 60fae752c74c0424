"""C-ABI checks that need no GPU: the library builds/loads, exports every function declared in
include/usv_hip.h, and reports errors through its return codes instead of crashing."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared_functions():
    src = open(os.path.join(ROOT, "include", "usv_hip.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"^\s*(?:const\s+)?\w+\**\s+\**(usv_\w+)\s*\(", src, flags=re.M)))


@pytest.fixture(scope="module")
def lib():
    from gym_usv_amd import _lib
    from gym_usv_amd.build import build_library
    build_library(verbose=False)
    return _lib.load()


def test_header_declares_full_api():
    names = _declared_functions()
    assert {"usv_create", "usv_step", "usv_reset", "usv_get_state", "usv_set_state",
            "usv_last_error", "usv_abi_version"} <= set(names)


def test_every_declared_symbol_exported(lib):
    from gym_usv_amd import _lib
    bound = {n for n, _, _ in _lib.SIGNATURES}
    for name in _declared_functions():
        assert hasattr(lib, name), f"{name} declared in usv_hip.h but not exported"
        assert name in bound, f"{name} declared in usv_hip.h but not bound in _lib.py"


def test_abi_version_and_defaults(lib):
    from gym_usv_amd import _lib
    assert lib.usv_abi_version() == _lib.ABI_VERSION
    cfg = _lib.UsvConfig()
    lib.usv_config_default(ctypes.byref(cfg), _lib.MODE_SIMPLE, 128)
    assert (cfg.abi_version, cfg.num_envs, cfg.obstacle_cap, cfg.max_episode_steps) == (_lib.ABI_VERSION, 128, 32, 500)
    assert (cfg.flags, cfg.reserved) == (0, 0)
    lib.usv_config_default(ctypes.byref(cfg), _lib.MODE_ASMC_SIMPLE, 8)
    assert cfg.max_episode_steps == 1000          # gym_usv/__init__.py:33
    for mode in (_lib.MODE_ASMC_V0, _lib.MODE_PID_V0, _lib.MODE_ASMC_YE_INT_V0):
        lib.usv_config_default(ctypes.byref(cfg), mode, 8)
        assert cfg.max_episode_steps == 0         # registered without a TimeLimit (:3-16)


def test_create_rejects_bad_config_without_gpu(lib):
    from gym_usv_amd import _lib
    cfg = _lib.UsvConfig()
    lib.usv_config_default(ctypes.byref(cfg), _lib.MODE_SIMPLE, 16)
    h = ctypes.c_void_p()
    cfg.obstacle_cap = 8                           # reference draws up to 29 obstacles
    assert lib.usv_create(ctypes.byref(cfg), 0, ctypes.byref(h)) != 0
    assert b"obstacle_cap" in lib.usv_last_error()
    cfg.obstacle_cap = 32
    cfg.mode = 5                                   # no such id
    assert lib.usv_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -1
    assert b"mode" in lib.usv_last_error()
    cfg.mode = _lib.MODE_SIMPLE
    cfg.abi_version = 99
    assert lib.usv_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -3
    assert not h.value
    # null handles are reported, not dereferenced
    assert lib.usv_step(None, None, None, None, None, None, None, None) == -1
    assert lib.usv_reset(None, None, None, None) == -1
    assert lib.usv_step_ex(None, None, None, None, None, None, None, None, None, None) == -1
    assert lib.usv_reset_ex(None, None, None, None, None, None) == -1
    assert lib.usv_set_experiment(None, None) == -1
    cfg.abi_version = _lib.ABI_VERSION
    cfg.flags = 4                                  # unknown flag bit
    assert lib.usv_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -1
    cfg.flags = _lib.FLAG_PERTURB                  # do_perturb is usv-asmc-simple's
    assert lib.usv_create(ctypes.byref(cfg), 0, ctypes.byref(h)) == -1


def test_vector_env_fails_loudly_without_gpu():
    import torch
    if torch.cuda.is_available():
        pytest.skip("GPU present")
    import gym_usv_amd
    with pytest.raises(gym_usv_amd.UsvLibError):
        gym_usv_amd.make_vec("usv-simple", 8)


def test_safe_vmcnt_build_same_abi():
    """libusvhip_safe.so (the vmcnt(0) debug build the GPU tests compare bitwise with the product)
    exports the same C-ABI and loads side by side with the product library (own ctypes handle)."""
    from gym_usv_amd import _lib
    from gym_usv_amd.build import build_all
    build_all(verbose=False)
    prod, safe = _lib.load(), _lib.load(_lib.SAFE_LIB_PATH)
    assert prod is not safe and _lib.load(_lib.SAFE_LIB_PATH) is safe
    assert safe.usv_abi_version() == prod.usv_abi_version() == _lib.ABI_VERSION
    for name in _declared_functions():
        assert hasattr(safe, name), name


def integration_snippet():
    """The reference-side binding of INTEGRATION.md §2, verbatim."""
    src = open(os.path.join(ROOT, "INTEGRATION.md")).read()
    sec = src.split("## 2.", 1)[1]
    return sec.split("```python\n", 1)[1].split("```", 1)[0]


def test_config_struct_layout(lib):
    """usv_config as compiled into the library = the binding's ctypes struct (a size check, plus
    usv_config_default writing the trailing fields where the binding reads them)."""
    from gym_usv_amd import _lib
    assert lib.usv_config_size() == ctypes.sizeof(_lib.UsvConfig) == 56
    buf = (ctypes.c_uint8 * 64)(*([0xAB] * 64))
    lib.usv_config_default(ctypes.cast(buf, ctypes.POINTER(_lib.UsvConfig)), _lib.MODE_SIMPLE, 7)
    assert all(b == 0xAB for b in bytes(buf)[56:]), "usv_config_default wrote past the struct"
    cfg = _lib.UsvConfig.from_buffer_copy(bytes(buf)[:56])
    assert (cfg.num_envs, cfg.flags, cfg.reserved, cfg.lidar_algo) == (7, 0, 0, _lib.LIDAR_WINDOW)


def test_integration_snippet_runs_verbatim_to_create(lib):
    """INTEGRATION.md §2's binding, executed as written up to usv_create (no GPU here: the create
    must fail through its return code and usv_last_error, after the struct-size check passed)."""
    import subprocess
    import sys
    code = integration_snippet()
    head = code.split("h = ctypes.c_void_p()", 1)[0]
    assert "usv_config_size" in head and '("flags", ctypes.c_int32)' in head
    prog = head + ("h = ctypes.c_void_p()\n"
                   "rc = lib.usv_create(ctypes.byref(cfg), 0, ctypes.byref(h))\n"
                   "print('RC', rc, lib.usv_last_error().decode())\n")
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.dirname(lib._name))
    out = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0, out.stderr
    line = [ln for ln in out.stdout.splitlines() if ln.startswith("RC")][-1]
    import torch
    if not torch.cuda.is_available():
        assert line.split()[1] != "0" and len(line.split()) > 2, line


def test_div_const_is_ieee_division_on_host(tmp_path):
    """div_const (usv_device.hpp), the f64 build's division by compile-time constants, restated in C with
    the same fma sequence: equal to x / c for 1e6 random operands per divisor (tools/micro/div_const_check.c;
    round 6 ran 2e8 per divisor)."""
    import os
    import shutil
    import subprocess
    cc = shutil.which("gcc")
    if cc is None:
        import pytest
        pytest.skip("no gcc")
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    exe = str(tmp_path / "div_const_check")
    subprocess.run([cc, "-O2", "-ffp-contract=off", "-o", exe, os.path.join(root, "tools", "micro", "div_const_check.c"),
                    "-lm"], check=True)
    p = subprocess.run([exe, "1000000"], capture_output=True, text=True, timeout=120)
    assert p.returncode == 0, p.stdout
    assert p.stdout.count(": 0 mismatches") == 10
