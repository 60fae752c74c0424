"""Generate golden vectors from the reference (romi2002/gym-usv) — build container only.

Run:  python tests/golden/make_golden.py      (needs /root/reference; writes tests/golden/*.npz)

The reference is imported read-only through ``refharness`` (stand-ins for its uninstalled
third-party imports).  Only inputs and outputs are stored; no
reference source travels.  Fixtures:

* ``asmc_compute.npz``   -- UsvAsmc.compute (usv_asmc.py:53-244) on injected random states,
                            plus the three adapted reference KATs (tests/test_usv_asmc.py:8-37).
* ``lidar.npz``          -- UsvAsmcCaEnv.compute_sensor_measurments (usv_asmc_ca_env.py:411-461)
                            on random scenes as UsvSimpleEnv calls it (simple_env.py:203-226).
* ``simple_traj.npz``    -- UsvSimpleEnv (usv-simple) seeded reset + random-action rollouts with
                            TimeLimit + same-step autoreset (SB3 DummyVecEnv semantics).
* ``asmc_simple_traj.npz`` -- the same for UsvSimpleASMCEnv (usv-asmc-simple).
* ``asmc_v0_traj.npz``   -- legacy UsvAsmcEnv (usv-asmc-v0) seeded rollouts with resets on done.
* ``asmc_ye_int_traj.npz`` / ``pid_traj.npz`` -- the float64 legacy envs UsvAsmcYeIntEnv
                            (usv-asmc-ye-int-v0) and UsvPidEnv (usv-pid-v0), same protocol
                            (``python tests/golden/make_golden.py --legacy-f64`` makes only these).

Round 4 (``--r4``): ``asmc_highspeed.npz`` -- usv-asmc-simple steps from injected high-speed /
large-heading / large-gain states, with and without do_perturb (gen_asmc_highspeed).

Round 2 (``--r2`` makes only these):

* ``asmc_perturb_traj.npz`` -- usv-asmc-simple rollouts with UsvAsmc.compute(..., do_perturb=True)
                            (usv_asmc.py:184-199), plus raw compute() sequences from fresh controllers.
* ``simple_info_traj.npz``  -- usv-simple rollouts recording the reset / step info dicts
                            (simple_env.py:102-115, 189-199).
* ``reset_options.npz``     -- reset(seed, options={'place_obstacles_on_path': k}) (:276-288).
* ``experiment.npz``        -- UsvSimpleEnv(options={'run_custom_experiment': True, ...}) resets and
                            rollouts (:292-300).
"""
from __future__ import annotations

import os
import sys

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, HERE)
import refharness  # noqa: E402

CAP = 32


def gen_asmc(E):
    from gym_usv.control.usv_asmc import UsvAsmc
    rng = np.random.default_rng(1234)
    n = 192
    out = {k: [] for k in ("action", "pos_in", "vel_in", "last_in", "so_in", "aux_in",
                           "pos_out", "vel_out", "last_out", "so_out", "aux_out")}
    for i in range(n):
        c = UsvAsmc()
        # warm the controller from zero state with a random action so its internal state
        # is realistic, then inject a perturbed state (covers both Xu regimes, Ka switches)
        pos = np.array([rng.uniform(0, 20), rng.uniform(0, 20), rng.uniform(-4, 4)])
        vel = np.array([rng.uniform(-0.5, 2.5), rng.uniform(-0.3, 0.3), rng.uniform(-1, 1)])
        warm = np.array([rng.uniform(0.2, 1.0), rng.uniform(-1, 1)], dtype=np.float32)
        for _ in range(int(rng.integers(0, 6))):
            pos, vel, _ = c.compute(warm, pos, vel, False)
        act = np.array([rng.uniform(0.2, 1.0), rng.uniform(-1, 1)], dtype=np.float32)
        out["action"].append(act.astype(np.float64))
        out["pos_in"].append(np.array(pos, dtype=np.float64))
        out["vel_in"].append(np.array(vel, dtype=np.float64))
        out["last_in"].append(np.array(c.last, dtype=np.float64))
        out["so_in"].append(np.array(c.so_filter, dtype=np.float64))
        out["aux_in"].append(np.array(c.aux_vars, dtype=np.float64))
        p2, v2, _ = c.compute(act, pos, vel, False)
        out["pos_out"].append(p2)
        out["vel_out"].append(v2)
        out["last_out"].append(np.array(c.last, dtype=np.float64))
        out["so_out"].append(np.array(c.so_filter, dtype=np.float64))
        out["aux_out"].append(np.array(c.aux_vars, dtype=np.float64))
    res = {k: np.stack(v) for k, v in out.items()}
    # adapted reference KATs: compute(a, p, v, False), 1000 calls from zero state
    for name, a in (("kat_zero", [0, 0]), ("kat_fwd", [10, 0]), ("kat_rot", [0, 10])):
        c = UsvAsmc()
        pos, vel = np.zeros(3), np.zeros(3)
        traj = []
        for k in range(1000):
            pos, vel, _ = c.compute(np.array(a, dtype=np.float64), pos, vel, False)
            if k < 50 or k % 50 == 49:
                traj.append(np.concatenate([pos, vel]))
        res[name] = np.stack(traj)
    np.savez_compressed(os.path.join(HERE, "asmc_compute.npz"), **res)
    print("asmc_compute.npz", {k: v.shape for k, v in res.items()})


def gen_lidar(E):
    UsvAsmcCaEnv = E.UsvAsmcCaEnv
    rng = np.random.default_rng(99)
    n_scenes = 256
    pos = np.zeros((n_scenes, 3))
    ox, oy, orad = np.zeros((n_scenes, CAP)), np.zeros((n_scenes, CAP)), np.zeros((n_scenes, CAP))
    nob = np.zeros(n_scenes, dtype=np.int64)
    keys = np.full((n_scenes, CAP), np.inf)
    sens = np.zeros((n_scenes, 128))
    for i in range(n_scenes):
        n = int(rng.integers(1, 30))
        p = np.array([rng.uniform(-1, 21), rng.uniform(-1, 21), rng.uniform(-20, 20)])
        xy = rng.uniform(0, 20, size=(n, 2))
        r = rng.uniform(0.15, 0.5, size=n)
        if i % 8 == 0:          # put the boat inside / touching an obstacle
            xy[0] = p[:2] + rng.normal(scale=0.2, size=2)
        sensor_count, span = 128, (2 / 3) * (2 * np.pi)
        d = np.hypot(xy[:, 0] - p[0], xy[:, 1] - p[1]) - r      # simple_env.py:205-206
        s = UsvAsmcCaEnv.compute_sensor_measurments(p, sensor_count, 100, r, span / sensor_count,
                                                    xy[:, 0].reshape(-1, 1), xy[:, 1].reshape(-1, 1),
                                                    n, d)
        pos[i], nob[i] = p, n
        ox[i, :n], oy[i, :n], orad[i, :n] = xy[:, 0], xy[:, 1], r
        keys[i, :n] = d
        sens[i] = s[:, 1]
    np.savez_compressed(os.path.join(HERE, "lidar.npz"), pos=pos, ox=ox, oy=oy, orad=orad,
                        n_obs=nob, keys=keys, sensors=sens)
    print("lidar.npz", n_scenes)


def snapshot(env):
    n = env.obstacle_n
    ox, oy, r = np.zeros(CAP), np.zeros(CAP), np.zeros(CAP)
    ox[:n], oy[:n], r[:n] = env.obstacle_positions[:, 0], env.obstacle_positions[:, 1], env.obstacle_radius
    return dict(position=np.array(env.position, dtype=np.float64),
                velocity=np.array(env.velocity, dtype=np.float64),
                last_action=np.array(env.last_action, dtype=np.float64),
                progress=float(env.progress), path_start=np.array(env.path_start),
                path_end=np.array(env.path_end), target=np.array(env.target_position),
                max_action=np.array(env.max_action, dtype=np.float64),
                ref_v=float(env.reference_velocity), n_obs=int(n), ox=ox, oy=oy, orad=r,
                sensors=np.array(env.sensor_data[:, 1], dtype=np.float64))


def gen_traj(E, cls, fname, limit, n_env=8, T=96):
    """Per env: seeded reset, then T random-action steps under TimeLimit(limit) with
    same-step autoreset (SB3 DummyVecEnv: reset() with no seed continues the stream)."""
    rng = np.random.default_rng(7)
    acts = np.stack([rng.uniform([0.2, -1], [1, 1], size=(T, 2)) for _ in range(n_env)]).astype(np.float32)
    seeds = np.arange(n_env) + 1000
    obs0 = np.zeros((n_env, 143), np.float32)
    obs = np.zeros((n_env, T, 143), np.float32)
    fobs = np.zeros((n_env, T, 143), np.float32)
    rew = np.zeros((n_env, T))
    term = np.zeros((n_env, T), bool)
    trunc = np.zeros((n_env, T), bool)
    st0 = []
    for e in range(n_env):
        env = cls(render_mode=None)
        o, _ = env.reset(seed=int(seeds[e]))
        obs0[e] = o
        st0.append(snapshot(env))
        elapsed = 0
        for t in range(T):
            o, r, te, tr, _ = env.step(acts[e, t])
            elapsed += 1
            tr = bool(tr) or (limit is not None and elapsed >= limit)
            fobs[e, t], rew[e, t], term[e, t], trunc[e, t] = o, r, bool(te), tr
            if te or tr:
                o, _ = env.reset()
                elapsed = 0
            obs[e, t] = o
    st = {f"init_{k}": np.stack([np.asarray(s[k]) for s in st0]) for k in st0[0]}
    np.savez_compressed(os.path.join(HERE, fname), seeds=seeds, actions=acts, obs0=obs0, obs=obs,
                        final_obs=fobs, reward=rew, terminated=term, truncated=trunc,
                        limit=-1 if limit is None else limit, **st)
    print(fname, "episodes ended:", int((term | trunc).sum()), "terminated:", int(term.sum()))


def gen_asmc_v0(E, fname="asmc_v0_traj.npz", n_env=4, T=3000):
    """Legacy UsvAsmcEnv (usv-asmc-v0, usv_asmc_env.py:99-300): old gym API, scalar action,
    np.random global RNG for resets (seeded per env here), no TimeLimit.  On done the env is
    reset (continuing the global stream), like a DummyVecEnv would."""
    rng = np.random.default_rng(11)
    acts = rng.uniform(-np.pi / 2, np.pi / 2, size=(n_env, T))
    # envs 1.. steer off the path (heading offsets biased away) so episodes end (|ye| > 10)
    for e in range(1, n_env):
        acts[e] = np.clip(rng.normal((-1) ** e * (0.6 + 0.3 * e), 0.3, size=T), -np.pi / 2, np.pi / 2)
    acts = acts.astype(np.float32)
    seeds = np.arange(n_env) + 2000
    obs0 = np.zeros((n_env, 6), np.float32)
    obs = np.zeros((n_env, T, 6), np.float32)
    fobs = np.zeros((n_env, T, 6), np.float32)
    rew = np.zeros((n_env, T))
    done = np.zeros((n_env, T), bool)
    init = {k: [] for k in ("state", "velocity", "position", "aux_vars", "last", "target")}
    for e in range(n_env):
        np.random.seed(int(seeds[e]))
        env = E.UsvAsmcEnv()
        obs0[e] = env.reset()
        for k in init:
            init[k].append(np.array(getattr(env, k), dtype=np.float64))
        for t in range(T):
            o, r, d, _ = env.step(acts[e, t])      # scalar action (shape-(1,) raises on NumPy >= 1.24)
            fobs[e, t], rew[e, t], done[e, t] = o, r, bool(d)
            if d:
                o = env.reset()
            obs[e, t] = o
    np.savez_compressed(os.path.join(HERE, fname), seeds=seeds, actions=acts, obs0=obs0, obs=obs,
                        final_obs=fobs, reward=rew, done=done,
                        **{f"init_{k}": np.stack(v) for k, v in init.items()})
    print(fname, "episodes ended:", int(done.sum()))


def gen_legacy_f64(E, cls, fname, n_env=4, T=2000, seed0=3000):
    """Legacy float64 path-following envs on the usv-asmc-v0 template: UsvAsmcYeIntEnv
    (usv-asmc-ye-int-v0, usv_asmc_ye_int_env.py:92-296) and UsvPidEnv (usv-pid-v0,
    usv_pid_env.py:89-278).  Same protocol as gen_asmc_v0: per-env np.random.seed, float32
    scalar actions, reset on done; the reference's obs are float64, stored here as float32 (the
    Box dtype, and what the C-ABI returns)."""
    rng = np.random.default_rng(seed0)
    acts = rng.uniform(-np.pi / 2, np.pi / 2, size=(n_env, T))
    # envs 1.. hold a heading offset near +-pi/2 so |ye| passes 10 within the rollout
    for e in range(1, n_env):
        acts[e] = np.clip(rng.normal((-1) ** e * (1.2 + 0.1 * e), 0.15, size=T), -np.pi / 2, np.pi / 2)
    acts = acts.astype(np.float32)
    seeds = np.arange(n_env) + seed0
    obs0 = np.zeros((n_env, 6), np.float32)
    obs = np.zeros((n_env, T, 6), np.float32)
    fobs = np.zeros((n_env, T, 6), np.float32)
    rew = np.zeros((n_env, T))
    done = np.zeros((n_env, T), bool)
    init = {k: [] for k in ("state", "velocity", "position", "aux_vars", "last", "target")}
    for e in range(n_env):
        np.random.seed(int(seeds[e]))
        env = cls()
        obs0[e] = env.reset()
        for k in init:
            init[k].append(np.array(getattr(env, k), dtype=np.float64))
        for t in range(T):
            o, r, d, _ = env.step(acts[e, t])
            fobs[e, t], rew[e, t], done[e, t] = o, float(r), bool(d)
            if d:
                o = env.reset()
            obs[e, t] = o
    np.savez_compressed(os.path.join(HERE, fname), seeds=seeds, actions=acts, obs0=obs0, obs=obs,
                        final_obs=fobs, reward=rew, done=done,
                        **{f"init_{k}": np.stack(v) for k, v in init.items()})
    print(fname, "episodes ended:", int(done.sum()))


# --------------------------------------------------------------------------- round-2 fixtures
CAP2 = 64


def snapshot64(env):
    """snapshot() with room for 29 + k obstacles (place_obstacles_on_path)."""
    n = env.obstacle_n
    ox, oy, r = np.zeros(CAP2), np.zeros(CAP2), np.zeros(CAP2)
    ox[:n], oy[:n], r[:n] = env.obstacle_positions[:, 0], env.obstacle_positions[:, 1], env.obstacle_radius
    return dict(position=np.array(env.position, dtype=np.float64), velocity=np.array(env.velocity, dtype=np.float64),
                path_start=np.array(env.path_start, dtype=np.float64), path_end=np.array(env.path_end, dtype=np.float64),
                target=np.array(env.target_position, dtype=np.float64),
                max_action=np.array(env.max_action, dtype=np.float64), ref_v=float(env.reference_velocity),
                n_obs=int(n), ox=ox, oy=oy, orad=r)


INFO_VEC = ("position", "velocity", "path_start", "path_end")
INFO_SCALAR = ("reward", "action0", "action1", "ye", "angle_to_target", "ye_reward", "angle_to_target_reward",
               "delta_action_reward", "delta_action", "velocity_track_reward", "reference_velocity",
               "reward_velocity", "reference_velocity_error")


def gen_asmc_perturb(E, n_env=6, T=160, fname="asmc_perturb_traj.npz"):
    """usv-asmc-simple with UsvAsmc.compute(..., do_perturb=True) (usv_asmc.py:184-199): the
    env's step (simple_env_asmc.py:18-27) with the reference's own compute called with the
    flag set; plus raw compute() sequences from a fresh controller (perturb_step 0, 10, 20, ...)."""
    from gym_usv.control.usv_asmc import UsvAsmc

    class PerturbedASMCEnv(E.UsvSimpleASMCEnv):
        def step(self, action):
            for _ in range(2):
                self.position, self.velocity, _ = self.asmc.compute(action, self.position, self.velocity, True)
            return E.UsvSimpleEnv.step(self, np.zeros(2))

    gen_traj(E, PerturbedASMCEnv, fname, 1000, n_env=n_env, T=T)
    rng = np.random.default_rng(77)
    seqs, acts = [], []
    for i in range(8):
        c = UsvAsmc()
        pos = np.array([rng.uniform(0, 20), rng.uniform(0, 20), rng.uniform(-3, 3)])
        vel = np.array([rng.uniform(0, 1.5), rng.uniform(-0.2, 0.2), rng.uniform(-0.5, 0.5)])
        a = np.array([rng.uniform(0.2, 1.0), rng.uniform(-1, 1)], dtype=np.float32)
        traj = [np.concatenate([pos, vel])]
        for k in range(120):
            pos, vel, _ = c.compute(a, pos, vel, True)
            traj.append(np.concatenate([pos, vel]))
        seqs.append(np.stack(traj))
        acts.append(a.astype(np.float64))
    d = dict(np.load(os.path.join(HERE, fname)))
    d.update(compute_seq=np.stack(seqs), compute_act=np.stack(acts))
    np.savez_compressed(os.path.join(HERE, fname), **d)
    print(fname, "+ compute sequences", d["compute_seq"].shape)


def gen_info_traj(E, n_env=4, T=64, fname="simple_info_traj.npz", cls=None, seed0=5000):
    """usv-simple rollouts (as gen_traj, TimeLimit 500) recording the reset and step info dicts
    (simple_env.py:102-115, 189-199, 305).  ``cls`` = UsvSimpleASMCEnv records usv-asmc-simple's,
    which is UsvSimpleEnv.step's info after the two ASMC computes (simple_env_asmc.py:18-27)."""
    cls = cls or E.UsvSimpleEnv
    rng = np.random.default_rng(17 + seed0 - 5000)
    acts = np.stack([rng.uniform([0.2, -1], [1, 1], size=(T, 2)) for _ in range(n_env)]).astype(np.float32)
    seeds = np.arange(n_env) + seed0
    out = {"obs0": np.zeros((n_env, 143), np.float32), "final_obs": np.zeros((n_env, T, 143), np.float32),
           "reward": np.zeros((n_env, T)), "terminated": np.zeros((n_env, T), bool),
           "truncated": np.zeros((n_env, T), bool)}
    for k in INFO_VEC:
        n = 3 if k in ("position", "velocity") else 2
        out["info0_" + k] = np.zeros((n_env, n))
        out["info_" + k] = np.zeros((n_env, T, n))
    for k in INFO_SCALAR:
        out["info_" + k] = np.zeros((n_env, T))
    for k in ("reward", "action0", "action1", "ye", "angle_to_target"):
        out["info0_" + k] = np.zeros(n_env)
    st0 = []
    for e in range(n_env):
        env = cls(render_mode=None)
        o, inf = env.reset(seed=int(seeds[e]))
        out["obs0"][e] = o
        st0.append(snapshot(env))
        for k in INFO_VEC:
            out["info0_" + k][e] = inf[k]
        for k in ("reward", "action0", "action1", "ye", "angle_to_target"):
            out["info0_" + k][e] = inf[k]
        for t in range(T):
            o, r, te, tr, inf = env.step(acts[e, t])
            out["final_obs"][e, t], out["reward"][e, t] = o, r
            out["terminated"][e, t], out["truncated"][e, t] = bool(te), bool(tr)
            for k in INFO_VEC:
                out["info_" + k][e, t] = inf[k]
            for k in INFO_SCALAR:
                out["info_" + k][e, t] = inf[k]
            if te or tr:
                break
    st = {f"init_{k}": np.stack([np.asarray(s[k]) for s in st0]) for k in st0[0]}
    np.savez_compressed(os.path.join(HERE, fname), seeds=seeds, actions=acts, **out, **st)
    print(fname, {k: v.shape for k, v in out.items() if k.startswith("info_p")})


def gen_reset_options(E, fname="reset_options.npz"):
    """UsvSimpleEnv.reset(seed, options={'place_obstacles_on_path': k}) (simple_env.py:276-288)."""
    ks = (3, 8, 20, 35)
    res = {k: [] for k in ("seed", "k", "obs")}
    snaps = []
    for k in ks:
        for sd in range(6):
            env = E.UsvSimpleEnv(render_mode=None)
            o, _ = env.reset(seed=100 + sd, options={"place_obstacles_on_path": k})
            res["seed"].append(100 + sd)
            res["k"].append(k)
            res["obs"].append(o)
            snaps.append(snapshot64(env))
    out = {k: np.stack([np.asarray(v) for v in vs]) for k, vs in res.items()}
    out.update({f"snap_{k}": np.stack([np.asarray(s[k]) for s in snaps]) for k in snaps[0]})
    np.savez_compressed(os.path.join(HERE, fname), **out)
    print(fname, out["snap_n_obs"])


def gen_experiment(E, fname="experiment.npz", T=40):
    """UsvSimpleEnv(options={'run_custom_experiment': True, 'experiment': ...}) (simple_env.py:292-300):
    seeded resets (each keeps its draws, then takes the experiment's obstacles, path and pose) and a
    short random-action rollout from each."""
    rng = np.random.default_rng(5)
    n = 12
    exp = dict(obstacle_positions=rng.uniform(2, 18, size=(n, 2)), obstacle_radius=rng.uniform(0.15, 0.5, n),
               path_start=np.array([3.0, 4.0]), angle=0.6, position=np.array([3.2, 3.7, 0.4]))
    seeds = np.arange(4) + 600
    acts = rng.uniform([0.2, -1], [1, 1], size=(len(seeds), T, 2)).astype(np.float32)
    obs0 = np.zeros((len(seeds), 143), np.float32)
    fobs = np.zeros((len(seeds), T, 143), np.float32)
    rew = np.zeros((len(seeds), T))
    term = np.zeros((len(seeds), T), bool)
    trunc = np.zeros((len(seeds), T), bool)
    snaps = []
    for i, sd in enumerate(seeds):
        env = E.UsvSimpleEnv(render_mode=None, options={"run_custom_experiment": True, "experiment": exp})
        obs0[i], _ = env.reset(seed=int(sd))
        snaps.append(snapshot(env))
        for t in range(T):
            o, r, te, tr, _ = env.step(acts[i, t])
            fobs[i, t], rew[i, t], term[i, t], trunc[i, t] = o, r, bool(te), bool(tr)
            if te or tr:
                break
    st = {f"init_{k}": np.stack([np.asarray(s[k]) for s in snaps]) for k in snaps[0]}
    np.savez_compressed(os.path.join(HERE, fname), seeds=seeds, actions=acts, obs0=obs0, final_obs=fobs,
                        reward=rew, terminated=term, truncated=trunc,
                        exp_obstacle_positions=exp["obstacle_positions"], exp_obstacle_radius=exp["obstacle_radius"],
                        exp_path_start=exp["path_start"], exp_angle=exp["angle"], exp_position=exp["position"], **st)
    print(fname, "steps until end:", (term | trunc).argmax(axis=1))


# --------------------------------------------------------------------------- round-3 fixtures
def snapshot_full(env, cap=CAP2):
    """Everything the step reads, with room for 29 + k obstacles: the state-injection image."""
    n = env.obstacle_n
    ox, oy, r = np.zeros(cap), np.zeros(cap), np.zeros(cap)
    ox[:n], oy[:n], r[:n] = env.obstacle_positions[:, 0], env.obstacle_positions[:, 1], env.obstacle_radius
    return dict(position=np.array(env.position, dtype=np.float64), velocity=np.array(env.velocity, dtype=np.float64),
                last_action=np.array(env.last_action, dtype=np.float64), progress=float(env.progress),
                path_start=np.array(env.path_start, dtype=np.float64), path_end=np.array(env.path_end, dtype=np.float64),
                target=np.array(env.target_position, dtype=np.float64),
                max_action=np.array(env.max_action, dtype=np.float64), ref_v=float(env.reference_velocity),
                n_obs=int(n), ox=ox, oy=oy, orad=r, sensors=np.array(env.sensor_data[:, 1], dtype=np.float64))


def gen_path_rollouts(E, fname="path_traj.npz", per_k=6, T=100):
    """Rollouts after reset(seed, options={'place_obstacles_on_path': k}) (simple_env.py:276-288),
    k in {3, 8, 20, 35} (up to 29 + 35 = 64 obstacles): random-action steps (:310-346) with the
    lidar over every obstacle (usv_asmc_ca_env.py:411-461), recorded up to each env's first episode
    end (no autoreset: SB3 would reset without the option)."""
    ks = (3, 8, 20, 35)
    n_env = len(ks) * per_k
    rng = np.random.default_rng(31)
    acts = rng.uniform([0.2, -1], [1, 1], size=(n_env, T, 2)).astype(np.float32)
    seeds = np.arange(n_env) + 700
    kk = np.repeat(np.array(ks), per_k)
    obs0 = np.zeros((n_env, 143), np.float32)
    fobs = np.zeros((n_env, T, 143), np.float32)
    rew = np.zeros((n_env, T))
    term = np.zeros((n_env, T), bool)
    trunc = np.zeros((n_env, T), bool)
    steps = np.zeros(n_env, np.int64)
    snaps = []
    for e in range(n_env):
        env = E.UsvSimpleEnv(render_mode=None)
        obs0[e], _ = env.reset(seed=int(seeds[e]), options={"place_obstacles_on_path": int(kk[e])})
        snaps.append(snapshot_full(env))
        for t in range(T):
            o, r, te, tr, _ = env.step(acts[e, t])
            fobs[e, t], rew[e, t], term[e, t], trunc[e, t] = o, r, bool(te), bool(tr)
            steps[e] = t + 1
            if te or tr:
                break
    st = {f"init_{k}": np.stack([np.asarray(s[k]) for s in snaps]) for k in snaps[0]}
    np.savez_compressed(os.path.join(HERE, fname), seeds=seeds, k=kk, actions=acts, obs0=obs0, final_obs=fobs,
                        reward=rew, terminated=term, truncated=trunc, steps=steps, **st)
    print(fname, "n_obs", st["init_n_obs"], "steps", steps)


# --------------------------------------------------------------------------- round-4 fixtures
def _f32(x):
    """Round to the nearest float32 (kept as float64): injected states every precision holds exactly."""
    return np.asarray(x, dtype=np.float32).astype(np.float64)


def gen_asmc_highspeed(E, fname="asmc_highspeed.npz", n_env=48, T=8, seed=4040, seed0=8000):
    """usv-asmc-simple steps (simple_env_asmc.py:18-27) from harness-injected states outside the
    low-speed regime the action space reaches: u in [-1, 4] (UsvAsmc's |u| > 1.2 hydrodynamics,
    usv_asmc.py:95-99), r in [-1, 1], v in [-0.1, 0.1] (the reference's explicit integrator diverges
    for |v| above ~0.3: Yv's damping, ~19 880 |v| over m - Y_v_dot = 53.13 (:101-102, :172-174), puts
    h * lambda past its stability bound), headings up to +-400 rad, adaptive gains up to 5, filter and
    integral states far from zero, desired speeds u_d up to 10 (the reference KATs'
    tests/test_usv_asmc.py:18-37).  Odd envs run UsvAsmc.compute(..., do_perturb=True)
    (usv_asmc.py:184-199) with perturb_step = 20 * elapsed.  Every injected value is a float32, so the
    f32 kernel starts from the state the reference starts from.  Recorded per step up to each env's
    first episode end: obs, reward, flags, the info position / velocity and the ASMC state."""
    from gym_usv.control.usv_asmc import UsvAsmc

    class PerturbedASMCEnv(E.UsvSimpleASMCEnv):
        def step(self, action):
            for _ in range(2):
                self.position, self.velocity, _ = self.asmc.compute(action, self.position, self.velocity, True)
            return E.UsvSimpleEnv.step(self, np.zeros(2))

    rng = np.random.default_rng(seed)
    perturb = (np.arange(n_env) % 2) == 1
    seeds = np.arange(n_env) + seed0
    acts = np.zeros((n_env, T, 2), np.float32)
    acts[:, :, 0] = np.where(rng.uniform(size=(n_env, T)) < 0.6, rng.uniform(0.2, 10, (n_env, T)),
                             rng.uniform(0.2, 1, (n_env, T)))
    acts[:, :, 1] = rng.uniform(-1, 1, (n_env, T))
    out = {k: [] for k in ("position", "velocity", "last_action", "so_in", "last_in", "aux_in", "elapsed")}
    rec = {"final_obs": np.zeros((n_env, T, 143), np.float32), "reward": np.zeros((n_env, T)),
           "terminated": np.zeros((n_env, T), bool), "truncated": np.zeros((n_env, T), bool),
           "info_position": np.zeros((n_env, T, 3)), "info_velocity": np.zeros((n_env, T, 3)),
           "so_out": np.zeros((n_env, T, 7)), "last_out": np.zeros((n_env, T, 9)),
           "aux_out": np.zeros((n_env, T, 3)), "steps": np.zeros(n_env, np.int64)}
    snaps = []
    for e in range(n_env):
        env = (PerturbedASMCEnv if perturb[e] else E.UsvSimpleASMCEnv)(render_mode=None)
        env.reset(seed=int(seeds[e]))
        band = e % 3                                  # heading scale: a turn, 30 rad, 400 rad
        psi = rng.uniform(-np.pi, np.pi) if band == 0 else rng.uniform(-30, 30) if band == 1 else \
            rng.choice([-1, 1]) * rng.uniform(300, 400)
        pos = _f32([rng.uniform(4, 16), rng.uniform(4, 16), psi])
        vel = _f32([rng.uniform(-1, 4), rng.uniform(-0.1, 0.1), rng.uniform(-1, 1)])
        mx = env.max_action
        la = _f32([rng.uniform(0, 0.5) * mx[0], 0.0, rng.uniform(-0.5, 0.5) * mx[2]])
        pdl, o, od, odd = _f32([psi + rng.uniform(-0.5, 0.5), rng.uniform(-2, 2), rng.uniform(-20, 20),
                                rng.uniform(-200, 200)])
        so = np.array([pdl, odd, od, o, o, od, odd])
        last = _f32(np.concatenate([rng.uniform(-4, 4, 3), rng.uniform(-5, 5, 3), [rng.uniform(-5, 5)],
                                    [rng.choice([-0.1, 0.1, 0.05])], [rng.choice([-0.2, 0.2])]]))
        aux = _f32([rng.uniform(-20, 20), rng.choice([0.02, rng.uniform(0, 5)]), rng.choice([0.1, rng.uniform(0, 5)])])
        elapsed = int(rng.integers(0, 990))
        env.position, env.velocity, env.last_action = pos.copy(), vel.copy(), la.copy()
        env.asmc.so_filter, env.asmc.last, env.asmc.aux_vars = so.copy(), last.copy(), aux.copy()
        env.asmc.perturb_step = 20 * elapsed
        for k, v in (("position", pos), ("velocity", vel), ("last_action", la), ("so_in", so), ("last_in", last),
                     ("aux_in", aux), ("elapsed", elapsed)):
            out[k].append(v)
        snaps.append(snapshot(env))
        for t in range(T):
            o_, r, te, tr, inf = env.step(acts[e, t])
            tr = bool(tr) or elapsed + t + 1 >= 1000
            rec["final_obs"][e, t], rec["reward"][e, t] = o_, r
            rec["terminated"][e, t], rec["truncated"][e, t] = bool(te), tr
            rec["info_position"][e, t], rec["info_velocity"][e, t] = inf["position"], inf["velocity"]
            rec["so_out"][e, t], rec["last_out"][e, t] = env.asmc.so_filter, env.asmc.last
            rec["aux_out"][e, t] = env.asmc.aux_vars
            rec["steps"][e] = t + 1
            if te or tr:
                break
    st = {f"init_{k}": np.stack([np.asarray(s[k]) for s in snaps]) for k in snaps[0]
          if k not in ("position", "velocity", "last_action")}
    np.savez_compressed(os.path.join(HERE, fname), seeds=seeds, actions=acts, perturb=perturb,
                        **{f"inj_{k}": np.stack([np.asarray(v) for v in vs]) for k, vs in out.items()}, **rec, **st)
    print(fname, "steps", rec["steps"], "max |u| after a step", np.abs(rec["info_velocity"][..., 0]).max())
    del UsvAsmc


def main():
    refharness.load_reference()
    import gym_usv.envs as E
    if "--r5" in sys.argv:              # round-5 fixture only: the high-speed generator at 240 envs
        gen_asmc_highspeed(E, fname="asmc_highspeed_240.npz", n_env=240, seed=4041, seed0=9000)
        return
    if "--r4" in sys.argv:              # round-4 fixtures only (existing files untouched)
        gen_asmc_highspeed(E)
        return
    if "--r3" in sys.argv:              # round-3 fixtures only (existing files untouched)
        gen_path_rollouts(E)
        gen_info_traj(E, fname="asmc_info_traj.npz", cls=E.UsvSimpleASMCEnv, seed0=5100)
        return
    if "--r2" in sys.argv:              # round-2 fixtures only (existing files untouched)
        gen_asmc_perturb(E)
        gen_info_traj(E)
        gen_reset_options(E)
        gen_experiment(E)
        return
    if "--legacy-f64" in sys.argv:      # only the usv-asmc-ye-int-v0 / usv-pid-v0 fixtures
        gen_legacy_f64(E, E.UsvAsmcYeIntEnv, "asmc_ye_int_traj.npz")
        gen_legacy_f64(E, E.UsvPidEnv, "pid_traj.npz", seed0=4000)
        return
    gen_asmc(E)
    gen_lidar(E)
    gen_traj(E, E.UsvSimpleEnv, "simple_traj.npz", 500, n_env=8, T=256)
    gen_traj(E, E.UsvSimpleASMCEnv, "asmc_simple_traj.npz", 1000, n_env=6, T=160)
    # short time limit variant exercises TimeLimit truncation + autoreset path
    gen_traj(E, E.UsvSimpleEnv, "simple_traj_tl.npz", 20, n_env=4, T=64)
    gen_asmc_v0(E)


if __name__ == "__main__":
    main()
