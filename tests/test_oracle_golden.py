"""Pin the CPU oracle (oracle/usv_oracle.py) against golden vectors generated from the
reference itself (tests/golden/make_golden.py).  CPU only."""
import numpy as np
import pytest

from oracle import usv_oracle as O


def test_lidar_matches_reference(golden):
    g = golden("lidar.npz")
    p = g["pos"]
    keys, sens = O.lidar(p[:, 0], p[:, 1], p[:, 2], g["ox"], g["oy"], g["orad"], g["n_obs"])
    np.testing.assert_allclose(keys, g["keys"], rtol=0, atol=1e-12)
    np.testing.assert_allclose(sens, g["sensors"], rtol=0, atol=1e-10)
    # coverage: hits, misses and negative readings (boat inside an obstacle) all present
    assert (g["sensors"] == 100).any() and (g["sensors"] < 100).any() and (g["sensors"] < 0).any()


def test_asmc_single_compute_matches_reference(golden):
    g = golden("asmc_compute.npz")
    n = g["action"].shape[0]
    a = O.AsmcBatch(n)
    so, last, aux = g["so_in"], g["last_in"], g["aux_in"]
    # so_filter = [psi_d_last, o_dd_last, o_d_last, o_last, o, o_d, o_dd] (usv_asmc.py:58)
    np.testing.assert_array_equal(so[:, 3], so[:, 4])
    a.state = np.concatenate([so[:, [0, 4, 5, 6]], last, aux], axis=1)
    pos, vel = a.compute(g["action"], g["pos_in"], g["vel_in"])
    np.testing.assert_allclose(pos, g["pos_out"], rtol=1e-11, atol=1e-11)
    np.testing.assert_allclose(vel, g["vel_out"], rtol=1e-11, atol=1e-11)
    ref_state = np.concatenate([g["so_out"][:, [0, 4, 5, 6]], g["last_out"], g["aux_out"]], axis=1)
    np.testing.assert_allclose(a.state, ref_state, rtol=1e-10, atol=1e-10)


@pytest.mark.parametrize("name", ["kat_zero", "kat_fwd", "kat_rot"])
def test_asmc_reference_kats(golden, name):
    """Adapted reference tests (tests/test_usv_asmc.py:8-37): 1000 compute() calls."""
    g = golden("asmc_compute.npz")
    act = {"kat_zero": [0, 0], "kat_fwd": [10, 0], "kat_rot": [0, 10]}[name]
    a = O.AsmcBatch(1)
    pos, vel = np.zeros((1, 3)), np.zeros((1, 3))
    traj = []
    for k in range(1000):
        pos, vel = a.compute(np.array([act], dtype=np.float64), pos, vel)
        if k < 50 or k % 50 == 49:
            traj.append(np.concatenate([pos[0], vel[0]]))
    traj = np.stack(traj)
    # first 300 calls pinned tightly; after that ulp differences (constant M^-1 instead of a
    # per-substep inv, fused C/D products) get amplified through sign() switches (chaotic)
    np.testing.assert_allclose(traj[:55], g[name][:55], rtol=1e-9, atol=1e-9)
    if name == "kat_zero":
        assert np.allclose(traj[-1], 0)
    elif name == "kat_fwd":
        assert traj[-1, 0] > 10 and np.all(np.abs(traj[-1, 1:3]) < 1) and traj[-1, 3] > 1
    else:
        assert traj[-1, 2] > 5


@pytest.mark.parametrize("fname,env_id", [("simple_traj.npz", "usv-simple"),
                                          ("simple_traj_tl.npz", "usv-simple"),
                                          ("asmc_simple_traj.npz", "usv-asmc-simple")])
def test_trajectories_match_reference(golden, fname, env_id):
    g = golden(fname)
    n, T = g["actions"].shape[:2]
    venv = O.OracleVectorEnv(env_id, n)
    if int(g["limit"]) > 0:
        venv.limit = int(g["limit"])
    obs = venv.reset([int(s) for s in g["seeds"]])
    np.testing.assert_allclose(obs, g["obs0"], rtol=1e-6, atol=1e-6)
    e = venv.env
    np.testing.assert_allclose(e.position, g["init_position"], atol=1e-13)
    np.testing.assert_array_equal(e.n_obs, g["init_n_obs"])
    np.testing.assert_allclose(e.ox, g["init_ox"], atol=1e-13)
    np.testing.assert_allclose(e.orad, g["init_orad"], atol=1e-13)
    for t in range(T):
        obs, rew, term, trunc, fobs, done = venv.step(g["actions"][:, t])
        np.testing.assert_array_equal(term, g["terminated"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(trunc, g["truncated"][:, t], err_msg=f"t={t}")
        np.testing.assert_allclose(rew, g["reward"][:, t], rtol=1e-9, atol=1e-9, err_msg=f"t={t}")
        np.testing.assert_allclose(fobs, g["final_obs"][:, t], rtol=1e-6, atol=1e-6, err_msg=f"t={t}")
        np.testing.assert_allclose(obs, g["obs"][:, t], rtol=1e-6, atol=1e-6, err_msg=f"t={t}")


def test_asmc_v0_trajectories_match_reference(golden):
    """Legacy usv-asmc-v0 (usv_asmc_env.py:99-300): seeded resets (np.random), 3000 scalar-action
    steps per env with resets on done; float32 state rounding reproduced."""
    g = golden("asmc_v0_traj.npz")
    n, T = g["actions"].shape
    o = O.AsmcV0Batch(n)
    obs = o.reset([int(s) for s in g["seeds"]])
    np.testing.assert_array_equal(obs, g["obs0"])
    np.testing.assert_allclose(o.position, g["init_position"], atol=0)
    np.testing.assert_allclose(o.target, g["init_target"], atol=0)
    for t in range(T):
        ob, rw, dn = o.step(g["actions"][:, t])
        np.testing.assert_array_equal(dn, g["done"][:, t], err_msg=f"t={t}")
        np.testing.assert_allclose(ob, g["final_obs"][:, t], rtol=0, atol=5e-6, err_msg=f"t={t}")
        np.testing.assert_allclose(rw, g["reward"][:, t], rtol=0, atol=1e-6, err_msg=f"t={t}")
        if dn.any():
            idx = np.flatnonzero(dn)
            o.reset(idx=idx)
            np.testing.assert_array_equal(o.state[idx].astype(np.float32), g["obs"][idx, t])
    assert g["done"].sum() >= 5


@pytest.mark.parametrize("fname,family", [("asmc_ye_int_traj.npz", "ye_int"), ("pid_traj.npz", "pid")])
def test_legacy_f64_trajectories_match_reference(golden, fname, family):
    """usv-asmc-ye-int-v0 (usv_asmc_ye_int_env.py:92-296) and usv-pid-v0 (usv_pid_env.py:89-276):
    float64 state, seeded np.random resets, 2000 float32 scalar-action steps per env with resets
    on done.  The restatement reproduces the reference's float64 arithmetic order, so obs match
    bitwise after the float32 cast and rewards to 1 ulp-scale (the reference's np.linalg.inv /
    BLAS matmul may round its last bit differently)."""
    g = golden(fname)
    n, T = g["actions"].shape
    o = O.LegacyF64Batch(n, family)
    obs = o.reset([int(s) for s in g["seeds"]])
    np.testing.assert_array_equal(obs, g["obs0"])
    for k in ("position", "target", "state"):
        np.testing.assert_array_equal(getattr(o, k), g[f"init_{k}"])
    for t in range(T):
        ob, rw, dn = o.step(g["actions"][:, t])
        np.testing.assert_array_equal(dn, g["done"][:, t], err_msg=f"t={t}")
        np.testing.assert_allclose(ob, g["final_obs"][:, t], rtol=0, atol=1e-6, err_msg=f"t={t}")
        np.testing.assert_allclose(rw, g["reward"][:, t], rtol=0, atol=1e-12, err_msg=f"t={t}")
        if dn.any():
            idx = np.flatnonzero(dn)
            o.reset(idx=idx)
            np.testing.assert_array_equal(o.state[idx].astype(np.float32), g["obs"][idx, t])
    assert g["done"].sum() >= 2


# --------------------------------------------------------------------------- round-2 fixtures
def test_asmc_perturb_compute_matches_reference(golden):
    """UsvAsmc.compute(..., do_perturb=True) (usv_asmc.py:184-199) from fresh controllers:
    120 consecutive calls (perturb_step 0, 10, ..., 1190)."""
    g = golden("asmc_perturb_traj.npz")
    seq, act = g["compute_seq"], g["compute_act"]
    a = O.AsmcBatch(seq.shape[0])
    pos, vel = seq[:, 0, :3].copy(), seq[:, 0, 3:].copy()
    for k in range(1, seq.shape[1]):
        pos, vel = a.compute(act, pos, vel, do_perturb=True)
        # chaotic sign() switches amplify last-bit differences late in the sequence
        tol = 1e-9 if k <= 40 else 1e-6
        np.testing.assert_allclose(np.concatenate([pos, vel], axis=1), seq[:, k], rtol=tol, atol=tol,
                                   err_msg=f"call {k}")
    assert np.all(a.perturb_step == 10 * (seq.shape[1] - 1))


def test_asmc_perturb_trajectories_match_reference(golden):
    g = golden("asmc_perturb_traj.npz")
    n, T = g["actions"].shape[:2]
    venv = O.OracleVectorEnv("usv-asmc-simple", n, perturb=True)
    obs = venv.reset([int(s) for s in g["seeds"]])
    np.testing.assert_allclose(obs, g["obs0"], rtol=1e-6, atol=1e-6)
    for t in range(T):
        obs, rew, term, trunc, fobs, done = venv.step(g["actions"][:, t])
        np.testing.assert_array_equal(term, g["terminated"][:, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(trunc, g["truncated"][:, t], err_msg=f"t={t}")
        np.testing.assert_allclose(rew, g["reward"][:, t], rtol=1e-8, atol=1e-8, err_msg=f"t={t}")
        np.testing.assert_allclose(fobs, g["final_obs"][:, t], rtol=1e-6, atol=1e-6, err_msg=f"t={t}")
        np.testing.assert_allclose(obs, g["obs"][:, t], rtol=1e-6, atol=1e-6, err_msg=f"t={t}")


def test_step_and_reset_info_match_reference(golden):
    """The info dicts of reset and step (simple_env.py:102-115, 189-199), every key."""
    g = golden("simple_info_traj.npz")
    n, T = g["actions"].shape[:2]
    e = O.SimpleEnvBatch(n)
    e.reset(seeds=[int(s) for s in g["seeds"]])
    inf = e.reset_info()
    for k in ("position", "velocity", "path_start", "path_end", "reward", "action0", "action1", "ye",
              "angle_to_target"):
        np.testing.assert_allclose(inf[k], g["info0_" + k], rtol=1e-12, atol=1e-12, err_msg=k)
    alive = np.ones(n, bool)
    for t in range(T):
        e.step(g["actions"][:, t])
        for k, v in e.info.items():
            np.testing.assert_allclose(v[alive], g["info_" + k][alive, t], rtol=1e-9, atol=1e-9,
                                       err_msg=f"{k} t={t}")
        alive &= ~(g["terminated"][:, t] | g["truncated"][:, t])
        if not alive.any():
            break


def test_reset_place_obstacles_on_path_matches_reference(golden):
    g = golden("reset_options.npz")
    for i in range(len(g["seed"])):
        e = O.SimpleEnvBatch(1, cap=64)
        obs = e.reset(seeds=[int(g["seed"][i])], options={"place_obstacles_on_path": int(g["k"][i])})
        np.testing.assert_allclose(obs[0], g["obs"][i], rtol=1e-6, atol=1e-6)
        assert e.n_obs[0] == g["snap_n_obs"][i]
        np.testing.assert_allclose(e.ox[0], g["snap_ox"][i], atol=1e-12)
        np.testing.assert_allclose(e.oy[0], g["snap_oy"][i], atol=1e-12)
        np.testing.assert_allclose(e.orad[0], g["snap_orad"][i], atol=1e-12)
        np.testing.assert_allclose(e.position[0], g["snap_position"][i], atol=1e-12)


def experiment_of(g):
    return dict(obstacle_positions=g["exp_obstacle_positions"], obstacle_radius=g["exp_obstacle_radius"],
                path_start=g["exp_path_start"], angle=float(g["exp_angle"]), position=g["exp_position"])


def test_custom_experiment_matches_reference(golden):
    """UsvSimpleEnv(options={'run_custom_experiment': True, 'experiment': ...}) (simple_env.py:292-300)."""
    g = golden("experiment.npz")
    n, T = g["actions"].shape[:2]
    e = O.SimpleEnvBatch(n, options={"run_custom_experiment": True, "experiment": experiment_of(g)})
    obs = e.reset(seeds=[int(s) for s in g["seeds"]])
    np.testing.assert_allclose(obs, g["obs0"], rtol=1e-6, atol=1e-6)
    np.testing.assert_allclose(e.position, g["init_position"], atol=1e-12)
    np.testing.assert_allclose(e.path_end, g["init_path_end"], atol=1e-12)
    np.testing.assert_array_equal(e.n_obs, g["init_n_obs"])
    alive = np.ones(n, bool)
    for t in range(T):
        o, r, te, tr = e.step(g["actions"][:, t])
        np.testing.assert_allclose(o[alive], g["final_obs"][alive, t], rtol=1e-6, atol=1e-6)
        np.testing.assert_allclose(r[alive], g["reward"][alive, t], rtol=1e-9, atol=1e-9)
        alive &= ~(te | tr)


# --------------------------------------------------------------------------- round-3 fixtures
def test_place_obstacles_on_path_rollouts_match_reference(golden):
    """Rollouts after reset(seed, options={'place_obstacles_on_path': k}) (simple_env.py:276-288,
    310-346), k up to 35 (61 obstacles): the lidar over every obstacle (usv_asmc_ca_env.py:411-461)."""
    g = golden("path_traj.npz")
    n, T = g["actions"].shape[:2]
    assert g["init_n_obs"].max() > 32           # the > 32-obstacle path is what this pins
    for k in np.unique(g["k"]):
        idx = np.flatnonzero(g["k"] == k)
        e = O.SimpleEnvBatch(len(idx), cap=64)
        obs = e.reset(seeds=[int(s) for s in g["seeds"][idx]], options={"place_obstacles_on_path": int(k)})
        np.testing.assert_allclose(obs, g["obs0"][idx], rtol=1e-6, atol=1e-6)
        np.testing.assert_array_equal(e.n_obs, g["init_n_obs"][idx])
        np.testing.assert_allclose(e.ox, g["init_ox"][idx], atol=1e-12)
        alive = np.ones(len(idx), bool)
        for t in range(T):
            o, r, te, tr = e.step(g["actions"][idx, t])
            m = alive
            np.testing.assert_array_equal(te[m], g["terminated"][idx][m, t], err_msg=f"k={k} t={t}")
            np.testing.assert_array_equal(tr[m], g["truncated"][idx][m, t], err_msg=f"k={k} t={t}")
            np.testing.assert_allclose(o[m], g["final_obs"][idx][m, t], rtol=1e-6, atol=1e-6, err_msg=f"k={k} t={t}")
            np.testing.assert_allclose(r[m], g["reward"][idx][m, t], rtol=1e-9, atol=1e-9, err_msg=f"k={k} t={t}")
            alive &= ~(g["terminated"][idx][:, t] | g["truncated"][idx][:, t])
            if not alive.any():
                break


def test_asmc_simple_step_info_matches_reference(golden):
    """usv-asmc-simple's step info: UsvSimpleEnv.step's info after the two ASMC computes
    (simple_env_asmc.py:18-27, simple_env.py:102-115, 189-199)."""
    g = golden("asmc_info_traj.npz")
    n, T = g["actions"].shape[:2]
    e = O.SimpleAsmcEnvBatch(n)
    e.reset(seeds=[int(s) for s in g["seeds"]])
    inf = e.reset_info()
    for k in ("position", "velocity", "path_start", "path_end", "reward", "ye", "angle_to_target"):
        np.testing.assert_allclose(inf[k], g["info0_" + k], rtol=1e-12, atol=1e-12, err_msg=k)
    alive = np.ones(n, bool)
    for t in range(T):
        e.step(g["actions"][:, t])
        for k, v in e.info.items():
            np.testing.assert_allclose(v[alive], g["info_" + k][alive, t], rtol=1e-8, atol=1e-8,
                                       err_msg=f"{k} t={t}")
        alive &= ~(g["terminated"][:, t] | g["truncated"][:, t])
        if not alive.any():
            break


# --------------------------------------------------------------------------- round-4 fixtures
@pytest.mark.parametrize("fixture", ["asmc_highspeed.npz", "asmc_highspeed_240.npz"], ids=["48", "240"])
@pytest.mark.parametrize("perturb", [False, True], ids=["plain", "perturb"])
def test_asmc_highspeed_steps_match_reference(golden, perturb, fixture):
    """usv-asmc-simple from injected states outside the action space's low-speed regime
    (make_golden.py gen_asmc_highspeed): |u| > 1.2 hydrodynamics (usv_asmc.py:95-99), headings to
    400 rad, adaptive gains to 5, u_d to 10; with and without do_perturb (:184-199)."""
    from asmc_fixture import asmc_state, oracle_env
    g = golden(fixture)
    idx = np.flatnonzero(g["perturb"] == perturb)
    e = oracle_env(g, idx, perturb)
    elapsed = g["inj_elapsed"][idx].copy()
    alive = np.ones(len(idx), bool)
    for t in range(g["actions"].shape[1]):
        o, r, te, tr = e.step(g["actions"][idx, t])
        elapsed += 1
        tr = tr | (elapsed >= 1000)
        m = alive
        np.testing.assert_array_equal(te[m], g["terminated"][idx][m, t], err_msg=f"t={t}")
        np.testing.assert_array_equal(tr[m], g["truncated"][idx][m, t], err_msg=f"t={t}")
        np.testing.assert_allclose(o[m], g["final_obs"][idx][m, t], rtol=1e-6, atol=1e-6, err_msg=f"t={t}")
        np.testing.assert_allclose(r[m], g["reward"][idx][m, t], rtol=1e-9, atol=1e-9, err_msg=f"t={t}")
        np.testing.assert_allclose(e.info["position"][m], g["info_position"][idx][m, t], rtol=1e-10, atol=1e-10)
        np.testing.assert_allclose(e.info["velocity"][m], g["info_velocity"][idx][m, t], rtol=1e-10, atol=1e-10)
        ref = asmc_state(g["so_out"][idx][m, t], g["last_out"][idx][m, t], g["aux_out"][idx][m, t])
        np.testing.assert_allclose(e.asmc.state[m], ref, rtol=1e-9, atol=1e-9, err_msg=f"t={t}")
        alive &= ~(g["terminated"][idx][:, t] | g["truncated"][idx][:, t])
    # the regime this fixture exists for is actually reached
    assert (e.asmc.fast_substeps > 0).sum() >= len(idx) // 3, e.asmc.fast_substeps
    assert np.abs(g["inj_position"][idx, 2]).max() > 300
