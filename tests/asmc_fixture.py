"""Injection of tests/golden/asmc_highspeed.npz (make_golden.py gen_asmc_highspeed) into the oracle
and into the HIP vector env: the reference's UsvSimpleASMCEnv stepped from high-speed,
large-heading, large-gain states, with and without do_perturb.  Test infrastructure."""
import numpy as np

from oracle import usv_oracle as O


def asmc_state(so, last, aux):
    """so_filter / last / aux_vars (usv_asmc.py:43-49) -> the 16-value state (ASMC_FIELDS order)."""
    np.testing.assert_array_equal(so[..., 3], so[..., 4])
    return np.concatenate([so[..., [0, 4, 5, 6]], last, aux], axis=-1)


def env_state(g, idx):
    """Per-env state dict (include/usv_hip.h field names) of the fixture's envs ``idx``."""
    p, v, la, ma = (g[k][idx] for k in ("inj_position", "inj_velocity", "inj_last_action", "init_max_action"))
    return {"x": p[:, 0], "y": p[:, 1], "psi": p[:, 2], "u": v[:, 0], "v": v[:, 1], "r": v[:, 2],
            "last_u": la[:, 0], "last_r": la[:, 2], "progress": g["init_progress"][idx],
            "path_x0": g["init_path_start"][idx, 0], "path_y0": g["init_path_start"][idx, 1],
            "path_x1": g["init_path_end"][idx, 0], "path_y1": g["init_path_end"][idx, 1],
            "max_u": ma[:, 0], "max_r": ma[:, 2], "ref_v": g["init_ref_v"][idx],
            "n_obs": g["init_n_obs"][idx], "obs_x": g["init_ox"][idx], "obs_y": g["init_oy"][idx],
            "obs_r": g["init_orad"][idx], "sensor_last": g["init_sensors"][idx],
            "elapsed": g["inj_elapsed"][idx].astype(np.int32), "scan_valid": 1,
            "asmc": asmc_state(g["inj_so_in"][idx], g["inj_last_in"][idx], g["inj_aux_in"][idx])}


def oracle_env(g, idx, perturb):
    """An oracle SimpleAsmcEnvBatch holding the fixture's injected state for envs ``idx``."""
    n = len(idx)
    e = O.SimpleAsmcEnvBatch(n, perturb=perturb)
    st = env_state(g, idx)
    e.position = np.stack([st["x"], st["y"], st["psi"]], 1)
    e.velocity = np.stack([st["u"], st["v"], st["r"]], 1)
    e.last_action = g["inj_last_action"][idx].copy()
    e.max_action = g["init_max_action"][idx].copy()
    e.ref_v, e.progress = st["ref_v"].copy(), st["progress"].copy()
    e.path_start, e.path_end = g["init_path_start"][idx].copy(), g["init_path_end"][idx].copy()
    e.target = g["init_target"][idx].copy()
    e.n_obs = st["n_obs"].astype(np.int64)
    e.ox, e.oy, e.orad = st["obs_x"].copy(), st["obs_y"].copy(), st["obs_r"].copy()
    e.sensors = st["sensor_last"].copy()
    e.asmc.state = st["asmc"].copy()
    e.asmc.perturb_step = 20 * g["inj_elapsed"][idx].astype(np.int64)
    return e
