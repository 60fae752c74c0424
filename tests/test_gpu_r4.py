"""Round-4 GPU parity: the HIP ASMC outside the low-speed regime, and the controller on its own.

* ``asmc_highspeed.npz`` (make_golden.py gen_asmc_highspeed): the reference's UsvSimpleASMCEnv
  stepped from injected states with |u| up to 4 (the |u| > 1.2 hydrodynamics, usv_asmc.py:95-99),
  headings to 400 rad, adaptive gains to 5 and u_d to 10, with and without do_perturb
  (:184-199), replayed through the env's usv_set_state / usv_step.
* ``gym_usv_amd.control.UsvAsmc`` (usv_asmc_compute): the reference's three tests
  (tests/test_usv_asmc.py:8-37, adapted to compute(a, p, v, False) as SURVEY §4 states) and the
  192 injected states and perturbed sequences of asmc_compute.npz / asmc_perturb_traj.npz.

Tolerances: f64 to the reference's float64 arithmetic (the oracle matches the reference to 1e-9 on
these fixtures); f32 per SURVEY §8(c) on obs / reward (obs 1e-5 + 1e-4 |ref|, reward 1e-4), the
ASMC state relative to max(1, |ref|), each bound ~5x the measured error printed by the test.
"""
import numpy as np
import pytest
import torch

from asmc_fixture import asmc_state, env_state, oracle_env

pytestmark = pytest.mark.gpu


def make(env_id, n, **kw):
    import gym_usv_amd
    return gym_usv_amd.make_vec(env_id, n, device=0, **kw)


def to_np(*ts):
    torch.cuda.synchronize()
    return [t.detach().cpu().numpy() for t in ts]


# (Round 4 / 5 history.)  Bounds ~5x the worst case measured on the round-4 tree (printed by the test; profiles/r04_gpu_errors.txt),
# capped by SURVEY 8(c) where that is tighter.  f64 measured: obs header exact, reward 3.6e-15, pose /
# velocity 2.5e-16, ASMC state 1.8e-13 (OCML's exp / asin / sin / cos against glibc's differ in the last
# bit, and 20 substeps carry it); f32: header 7.1e-6 (8(c) 1e-5), reward 3.5e-5 (8(c) 1e-4), pose /
# velocity 3.5e-5 relative, state 1.6e-3.
# Round 5 (240-env fixture, 5x more envs): f64 reward 4.0e-14, state 6.2e-13; f32 state 7.4e-3 (row 7,
# the surge acceleration u_dot_last, relative to max(1, |ref|)) -- bounds raised to ~5x / ~3x those.
# Round 6: the ASMC state bound is per row (verdict r5 #4): 2x the largest error each row
# showed over both fixtures and both modes (round-6 tree, gpurun_out/r6a; the test prints every row).
# Rows (usv_hip.h usv_asmc_compute): 0 psi_d_last, 1-3 the heading filter o, o', o'', 4-6 eta_dot_last,
# 7-9 upsilon_dot_last (the surge / sway / yaw accelerations, which jump with every Ka-switch-adjacent
# rounding), 10 e_u_last, 13 e_u_int, 14-15 Ka_u, Ka_psi (11, 12 are the switches: counted as flips).
# Measured f32 maxima: 2.3e-4 2.2e-4 1.1e-3 3.6e-3 | 6.1e-4 1.3e-3 2.1e-4 | 7.4e-3 5.6e-4 1.5e-3 |
# 3.2e-4 6.7e-5 2.5e-3 6.4e-6 (rows 7 and 3 from the perturbed 240-env half).
HS_STATE_ROWS_F32 = {0: 5e-4, 1: 5e-4, 2: 2.5e-3, 3: 7.5e-3, 4: 1.5e-3, 5: 3e-3, 6: 5e-4,
                     7: 1.5e-2, 8: 1.5e-3, 9: 3e-3, 10: 7e-4, 13: 1.5e-4, 14: 5e-3, 15: 1.5e-5}
# measured (round 6): f64 reward 4.0e-14, state 6.2e-13 (row 3), velocity 4.4e-16, position 1.1e-15;
# f32 header 7.9e-6, reward 3.5e-5, velocity 6.3e-6, position 5.7e-5
HS_TOL = {"f64": dict(hdr=0.0, rew=8e-14, vel=1e-15, pos=2.5e-15, state=1.2e-12),
          "f32": dict(hdr=1e-5, rew=7e-5, vel=1.5e-5, pos=1e-4, state=None)}


# f32 envs whose Ka switch lands on the other branch (the round-5 240-env fixture gives the rate
# statistical weight): bound = 2x the measured count per fixture and mode (round 5: 48-env fixture
# 1/24 plain, 0/24 perturbed; 240-env fixture 4/120 plain, 3/120 perturbed, i.e. 2.5-3.3 %)
HS_FLIPS = {("asmc_highspeed.npz", False): 2, ("asmc_highspeed.npz", True): 1,
            ("asmc_highspeed_240.npz", False): 8, ("asmc_highspeed_240.npz", True): 6}


@pytest.mark.parametrize("fixture", ["asmc_highspeed.npz", "asmc_highspeed_240.npz"], ids=["48", "240"])
@pytest.mark.parametrize("precision", ["f64", "f32"])
@pytest.mark.parametrize("perturb", [False, True], ids=["plain", "perturb"])
def test_asmc_highspeed_replay(golden, precision, perturb, fixture):
    """Up to each env's first episode end.  The adaptive-gain derivatives Ka_dot_u / Ka_dot_psi
    (usv_asmc.py:137-140) are switches (+-k, k_min): in f32 a sliding surface within rounding of
    its threshold mu picks the other branch, after which that env follows another control law.
    Such envs are counted (a branch-flip rate, bounded) and compared no further; the others
    are held to the stated bounds."""
    g = golden(fixture)
    idx = np.flatnonzero(g["perturb"] == perturb)
    n, T = len(idx), g["actions"].shape[1]
    env = make("usv-asmc-simple", n, precision=precision, autoreset=False, info=True, perturb=perturb)
    env.set_state(env_state(g, idx))
    orc = oracle_env(g, idx, perturb)           # the checker: counts the |u| > 1.2 substeps
    alive = np.ones(n, bool)
    flipped = np.zeros(n, bool)
    worst = dict(hdr=0.0, rew=0.0, vel=0.0, pos=0.0, state=0.0)
    flips = rays = 0
    worst_entry = -1
    cont = np.array([k for k in range(16) if k not in (11, 12)])    # continuous state entries
    rows = np.zeros(16)                         # per state row: max relative error
    band = idx % 3                              # gen_asmc_highspeed: |psi| <= pi, <= 30, 300..400 rad
    bw = {b: dict(hdr=0.0, rew=0.0, flips=0) for b in range(3)}
    for t in range(T):
        a = torch.from_numpy(g["actions"][idx, t]).cuda()
        obs, rew, term, trunc, info = env.step(a)
        obs, rew, term, trunc, ipos, ivel = to_np(obs, rew, term, trunc, info["position"], info["velocity"])
        orc.step(g["actions"][idx, t])
        st = env.get_field("asmc")
        rs = asmc_state(g["so_out"][idx][:, t], g["last_out"][idx][:, t], g["aux_out"][idx][:, t])
        flipped |= alive & (np.abs(st[:, [11, 12]] - rs[:, [11, 12]]) > 1e-6).any(axis=1)
        m = alive & ~flipped
        if m.any():
            ref = g["final_obs"][idx][m, t]
            worst["hdr"] = max(worst["hdr"], float((np.abs(obs[m, :15] - ref[:, :15]) - 1e-4 * np.abs(ref[:, :15])).max()))
            flips += int((np.abs(obs[m, 15:] - ref[:, 15:]) > 1e-5 + 1e-4 * np.abs(ref[:, 15:])).sum())
            rays += int(m.sum()) * 128
            worst["rew"] = max(worst["rew"], float(np.abs(rew[m] - g["reward"][idx][m, t]).max()))
            rv, rp = g["info_velocity"][idx][m, t], g["info_position"][idx][m, t]
            worst["vel"] = max(worst["vel"], float((np.abs(ivel[m] - rv) / np.maximum(1, np.abs(rv))).max()))
            worst["pos"] = max(worst["pos"], float((np.abs(ipos[m] - rp) / np.maximum(1, np.abs(rp))).max()))
            d = np.abs(st[m][:, cont] - rs[m][:, cont]) / np.maximum(1, np.abs(rs[m][:, cont]))
            rows[cont] = np.maximum(rows[cont], d.max(axis=0))
            if float(d.max()) > worst["state"]:
                worst["state"] = float(d.max())
                worst_entry = int(cont[np.unravel_index(np.argmax(d), d.shape)[1]])
            for b in range(3):
                mb = m & (band == b)
                if mb.any():
                    rb = g["final_obs"][idx][mb, t]
                    bw[b]["hdr"] = max(bw[b]["hdr"], float((np.abs(obs[mb, :15] - rb[:, :15]) - 1e-4 * np.abs(rb[:, :15])).max()))
                    bw[b]["rew"] = max(bw[b]["rew"], float(np.abs(rew[mb] - g["reward"][idx][mb, t]).max()))
                    bw[b]["flips"] += int((np.abs(obs[mb, 15:] - rb[:, 15:]) > 1e-5 + 1e-4 * np.abs(rb[:, 15:])).sum())
            np.testing.assert_array_equal(term[m], g["terminated"][idx][m, t], err_msg=f"t={t}")
            np.testing.assert_array_equal(trunc[m], g["truncated"][idx][m, t], err_msg=f"t={t}")
        alive &= ~(g["terminated"][idx][:, t] | g["truncated"][idx][:, t])
    fast = int(orc.asmc.fast_substeps.sum())
    print(f"\n[asmc highspeed {fixture} {precision} perturb={perturb}] {fast} substeps with |u| > 1.2 over {n} envs; "
          f"Ka-switch flips {int(flipped.sum())}/{n} envs (rate {flipped.mean():.3f}); "
          + ", ".join(f"{k} {v:.2e}" for k, v in worst.items()) + f" (state row {worst_entry})"
          + f"; sensor flips {flips}/{rays}; by |psi| band "
          + "; ".join(f"{b}: hdr {v['hdr']:.2e} rew {v['rew']:.2e} flips {v['flips']}" for b, v in bw.items())
          + "; state rows " + " ".join(f"{k}:{rows[k]:.1e}" for k in cont))
    assert fast > 0 and (orc.asmc.fast_substeps > 0).sum() >= n // 3
    assert flipped.sum() <= (0 if precision == "f64" else HS_FLIPS.get((fixture, perturb), max(2, n // 8))), \
        flipped.sum()
    tol = HS_TOL[precision]
    assert worst["hdr"] <= tol["hdr"] and worst["rew"] <= tol["rew"], worst
    assert worst["vel"] <= tol["vel"] and worst["pos"] <= tol["pos"], worst
    if precision == "f64":
        assert worst["state"] <= tol["state"], worst
    else:
        over = {k: (float(rows[k]), b) for k, b in HS_STATE_ROWS_F32.items() if rows[k] > b}
        assert not over, f"ASMC state rows over their bounds: {over}"
    assert flips <= (0 if precision == "f64" else max(2, rays // 10000))
    env.close()


# --------------------------------------------------------------------------- the controller on its own
# calls 350..1000 of the reference KATs (round 5; measured in parentheses): kat_fwd stays smooth
# (f64 5.2e-15, f32 1.9e-5); kat_rot's heading-rate switching makes even f64 drift (9.3e-2 on psi,
# u, r at call 1000), f32 8.6e-2 -- a band around the reference trajectory, not a tolerance
# Round 6: ~1.5x the measured values -- f64 kat_fwd 5.2e-15, kat_rot 9.25e-2; f32 kat_fwd
# 1.85e-5, kat_rot 7.3e-2 (8.6-10.8 % across round 5's substep edits).  The f32 kat_rot trajectory against
# this library's own f64 one drifts as far (8.3e-2 over 1000 calls): the switching, not the reference, sets
# the band, so it is bounded the same way (KAT_ROT_VS_F64).
KAT_BAND = {"f64": {"kat_zero": 0.0, "kat_fwd": 8e-15, "kat_rot": 0.14},
            "f32": {"kat_zero": 0.0, "kat_fwd": 3e-5, "kat_rot": 0.12}}
KAT_ROT_VS_F64 = 0.13


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_reference_asmc_tests_on_hip(golden, precision):
    """The reference's own tests (tests/test_usv_asmc.py:8-37: 1000 compute() calls from rest),
    adapted to the signature the reference code has (compute(a, p, v, False), three return values;
    SURVEY §4), run on the HIP controller.  f64 additionally follows the reference's trajectories
    (the first 300 calls, before chaotic sign() switches amplify last-bit differences)."""
    from gym_usv_amd.control import UsvAsmc
    g = golden("asmc_compute.npz")
    worst = 0.0
    band = {}
    def run(prec, act):
        asmc = UsvAsmc(precision=prec)
        position, velocity = np.zeros(3), np.zeros(3)
        traj = []
        for k in range(1000):
            position, velocity, _ = asmc.compute(np.array(act, dtype=np.float64), position, velocity, False)
            if k < 50 or k % 50 == 49:
                traj.append(np.concatenate([position, velocity]))
        return position, velocity, np.stack(traj)
    vs64 = None
    for name, act in (("kat_zero", [0, 0]), ("kat_fwd", [10, 0]), ("kat_rot", [0, 10])):
        position, velocity, traj = run(precision, act)
        if name == "kat_rot" and precision == "f32":
            # the f32 controller against this library's own f64 one on the same calls: f64 follows
            # the reference to 5.7e-15 over the first 300 calls, so this tracks the f32 arithmetic alone
            t64 = run("f64", act)[2]
            vs64 = float((np.abs(traj - t64) / np.maximum(1, np.abs(t64)))[:, [2, 3, 5]].max())
        if name == "kat_zero":                                       # test_no_movement :8-16
            assert np.allclose(position, np.zeros(3)) and np.allclose(velocity, np.zeros(3))
        elif name == "kat_fwd":                                      # test_forward_movement :18-28
            assert position[0] > 10 and np.all(np.abs(position[1:]) < 1)
            assert velocity[0] > 1 and np.all(np.abs(velocity[1:]) < 1)
        else:                                                        # test_rotation :30-37
            assert position[2] > 5
        ref = g[name]
        err = np.abs(traj[:55] - ref[:55]) / np.maximum(1, np.abs(ref[:55]))
        worst = max(worst, float(err.max()))
        # calls 350..1000 (round 5): a property band, since sign() switches amplify last-bit
        # differences there (f64 too).  kat_fwd stays smooth: relative error on every entry;
        # kat_rot: surge speed u, yaw rate r and heading psi (x, y wander around 0 and are bounded
        # by the reference test itself)
        late = np.abs(traj[55:] - ref[55:]) / np.maximum(1, np.abs(ref[55:]))
        if name == "kat_rot":
            late = late[:, [2, 3, 5]]
        band[name] = float(late.max())
        print(f"\n[KAT {name} {precision}] final pos {position}, vel {velocity}; ref final {ref[-1]}; "
              f"first 300 calls max rel err {err.max():.2e}; calls 350-1000 band {band[name]:.2e}"
              + (f"; f32 vs own f64 (psi, u, r) over 1000 calls {vs64:.2e}" if name == "kat_rot" and vs64 is not None else ""))
    # measured: f64 5.7e-15, f32 4.5e-5 (kat_rot)
    assert worst <= (9e-15 if precision == "f64" else 7e-5), worst
    if vs64 is not None:
        assert vs64 <= KAT_ROT_VS_F64, vs64
    # calls 350-1000, measured (round 5): see KAT_BAND
    for name, lim in KAT_BAND[precision].items():
        assert band[name] <= lim, (name, band[name])


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_asmc_compute_injected_states(golden, precision):
    """UsvAsmc.compute on the 192 injected states of asmc_compute.npz (both Xu regimes, Ka switches),
    one batched launch (UsvAsmcBatch)."""
    from gym_usv_amd.control import UsvAsmcBatch
    g = golden("asmc_compute.npz")
    n = g["action"].shape[0]
    b = UsvAsmcBatch(n, precision=precision)
    b.state.copy_(torch.from_numpy(asmc_state(g["so_in"], g["last_in"], g["aux_in"]).T.copy()))
    p, v = b.compute(g["action"], g["pos_in"], g["vel_in"])
    p, v, st = to_np(p, v, b.state)
    ref_st = asmc_state(g["so_out"], g["last_out"], g["aux_out"])
    rel = lambda a, r: float((np.abs(a - r) / np.maximum(1, np.abs(r))).max())
    e = dict(pos=rel(p, g["pos_out"]), vel=rel(v, g["vel_out"]), state=rel(st.T, ref_st))
    print(f"\n[asmc compute 192 {precision}] " + ", ".join(f"{k} {x:.2e}" for k, x in e.items())
          + f"; |u| > 1.2 inputs: {int((np.abs(g['vel_in'][:, 0]) > 1.2).sum())}")
    # measured: f64 pos 1.5e-16, vel 6.3e-16, state 7.3e-14; f32 pos 9.8e-8, vel 2.5e-7, state 5.1e-5
    tol = 5e-13 if precision == "f64" else dict(pos=5e-7, vel=1.5e-6, state=2.5e-4)
    for k, x in e.items():
        assert x <= (tol if precision == "f64" else tol[k]), (k, x)


@pytest.mark.parametrize("precision", ["f64", "f32"])
def test_asmc_compute_perturbed_sequences(golden, precision):
    """UsvAsmc.compute(..., do_perturb=True) from fresh controllers, 120 calls (perturb_step 0 ..
    1190; usv_asmc.py:184-199): the reference's sequences of asmc_perturb_traj.npz."""
    from gym_usv_amd.control import UsvAsmcBatch
    g = golden("asmc_perturb_traj.npz")
    seq, act = g["compute_seq"], g["compute_act"]
    b = UsvAsmcBatch(seq.shape[0], precision=precision)
    pos = torch.from_numpy(seq[:, 0, :3].copy()).cuda().to(b.dtype)
    vel = torch.from_numpy(seq[:, 0, 3:].copy()).cuda().to(b.dtype)
    worst = 0.0
    for k in range(1, 41):
        b.compute(act, pos, vel, do_perturb=True)
        got = np.concatenate(to_np(pos, vel), axis=1)
        worst = max(worst, float((np.abs(got - seq[:, k]) / np.maximum(1, np.abs(seq[:, k]))).max()))
    (ps,) = to_np(b.perturb_step)
    print(f"\n[asmc perturb seq {precision}] 40 calls, max rel err {worst:.2e}")
    assert np.all(ps == 400)
    assert worst <= (2e-15 if precision == "f64" else 5e-6), worst     # measured 3.4e-16 / 9.6e-7


def test_asmc_compute_matches_env_step_f64():
    """The standalone controller and the env step run the same substep function: two compute()
    calls from an env's state give the env step's ASMC state bit for bit (f64)."""
    from gym_usv_amd.control import UsvAsmcBatch
    n = 256
    env = make("usv-asmc-simple", n, precision="f64", seed=3, autoreset=False)
    env.reset(seed=3)
    gen = torch.Generator(device="cuda").manual_seed(2)
    for _ in range(5):
        env.step(torch.rand(n, 2, device="cuda", generator=gen) * torch.tensor([0.8, 2.0], device="cuda")
                 + torch.tensor([0.2, -1.0], device="cuda"))
    st = env.get_state()
    a = torch.rand(n, 2, device="cuda", generator=gen) * torch.tensor([0.8, 2.0], device="cuda") \
        + torch.tensor([0.2, -1.0], device="cuda")
    b = UsvAsmcBatch(n, precision="f64")
    b.state.copy_(torch.from_numpy(st["asmc"].T.copy()))
    pos = torch.from_numpy(np.stack([st["x"], st["y"], st["psi"]], 1)).cuda()
    vel = torch.from_numpy(np.stack([st["u"], st["v"], st["r"]], 1)).cuda()
    b.compute(a.double(), pos, vel, calls=2)
    env.step(a)
    (bst,) = to_np(b.state)
    np.testing.assert_array_equal(bst.T, env.get_field("asmc"))
    env.close()


def test_integration_snippet_runs_verbatim_on_gpu():
    """INTEGRATION.md §2's reference-side binding, executed as written (a fresh process with
    libusvhip.so on LD_LIBRARY_PATH): create, reset, step, step_ex with info and done outputs."""
    import os
    import subprocess
    import sys
    from test_abi import integration_snippet
    from gym_usv_amd import _lib
    prog = integration_snippet() + ("torch.cuda.synchronize()\n"
                                    "assert torch.isfinite(obs).all() and torch.isfinite(rew).all()\n"
                                    "assert bool(((term | trunc) == done).all())\n"
                                    "lib.usv_destroy.argtypes = [ctypes.c_void_p]\nlib.usv_destroy(h)\nprint('SNIPPET OK')\n")
    env = dict(os.environ, LD_LIBRARY_PATH=os.path.dirname(_lib.LIB_PATH))
    out = subprocess.run([sys.executable, "-c", prog], env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode == 0 and "SNIPPET OK" in out.stdout, out.stderr[-2000:]


@pytest.mark.parametrize("env_id", ["usv-asmc-v0", "usv-pid-v0", "usv-asmc-ye-int-v0", "usv-simple"])
def test_unseeded_single_env_reset(env_id):
    """gym_usv_amd.make(id).reset() with no seed, the reference's usual first call: the legacy ids
    seed np.random's MT19937 (seeds below 2**32, usv_asmc_env.py:258) from fresh entropy."""
    import gym_usv_amd
    for _ in range(4):
        env = gym_usv_amd.make(env_id)
        out = env.reset()
        obs = out if env_id != "usv-simple" else out[0]
        assert np.isfinite(obs).all()
        env.close()


@pytest.mark.parametrize("n", [1, 77, 1077, 40000])
def test_asmc_split_chain_bit_identical(n):
    """usv-asmc-simple kind 6 (asmc_chain_kernel, then the fused block-queue step running
    UsvSimpleEnv.step(zeros(2)) in its phase 1; both block shapes) against the fused wave kernel
    and the split block queue (kind 4), over a rollout with TimeLimit resets and ragged env counts:
    bitwise equal outputs, terminal rows and info rows."""
    T = 30
    gen = torch.Generator(device="cuda").manual_seed(8)
    acts = [torch.rand(n, 2, device="cuda", generator=gen) * torch.tensor([0.8, 2.0], device="cuda")
            + torch.tensor([0.2, -1.0], device="cuda") for _ in range(T)]
    ref = None
    for v in ("64,7,1", "128,7,4", "128,7,6", "16,7,6", "128,263,6", None):
        env = make("usv-asmc-simple", n, seed=6, max_episode_steps=11, kernel_variant=v, copy=False, info=True)
        env.reset(seed=6)
        outs = []
        for a in acts:
            o, r, te, tr, info = env.step(a)
            outs.append([x.clone() for x in (o, r, te, tr, info["final_obs"], info["position"], info["ye_reward"])])
        outs.append([torch.from_numpy(env.get_field("asmc"))])
        env.close()
        if ref is None:
            ref = outs
            continue
        for t, (a_, b_) in enumerate(zip(ref, outs)):
            for x, y in zip(a_, b_):
                assert torch.equal(x, y), f"variant {v} differs at step {t} (n={n})"


@pytest.mark.parametrize("env_id", ["usv-simple", "usv-asmc-simple"])
def test_f32_heading_turns_roundtrip_and_spin(env_id):
    """The f32 state holds the heading as phi + 2 pi k: a heading of ~400 rad set through the state
    interface reads back to float precision of phi (not float32's 3e-5 at 400 rad), psi_d_last
    keeps its value across a frame change (usv-asmc-simple), and a usv-simple rollout spinning at
    full yaw (the heading passing tens of turns) keeps the f32 obs header within 2e-5 of the f64
    kernel's."""
    n = 64
    envs = {p: make(env_id, n, precision=p, autoreset=False, reset_rng="numpy", max_episode_steps=0)
            for p in ("f32", "f64")}
    for e in envs.values():
        e.reset(seed=list(range(900, 900 + n)))
    e32 = envs["f32"]
    psi = np.linspace(-400.3, 400.7, n)
    e32.set_field("psi", psi)
    assert np.abs(e32.get_field("psi") - psi).max() < 1e-6
    if env_id == "usv-asmc-simple":
        st = e32.get_field("asmc")
        st[:, 0] = psi + 0.25
        e32.set_field("asmc", st)
        e32.set_field("psi", psi + 12.0)                 # a new frame: psi_d_last keeps its value
        assert np.abs(e32.get_field("asmc")[:, 0] - (psi + 0.25)).max() < 1e-5
        e32.set_field("psi", psi)
        e32.set_field("asmc", np.zeros((n, 16)))
    if env_id != "usv-simple":          # (the ASMC's switching law makes f32 and f64 rollouts part ways)
        for e in envs.values():
            e.close()
        return
    envs["f64"].set_state(e32.get_state())
    a = torch.tensor([[0.3, 1.0]] * n, device="cuda")
    alive = np.ones(n, bool)
    worst = 0.0
    for t in range(300):
        o32, _, te, tr, _ = e32.step(a)
        o64, _, te64, tr64, _ = envs["f64"].step(a)
        o32, o64, te, tr, te64, tr64 = to_np(o32, o64, te, tr, te64, tr64)
        alive &= ~(te | tr | te64 | tr64)
        if not alive.any():
            break
        worst = max(worst, float(np.abs(o32[alive, :15] - o64[alive, :15]).max()))
    spin = np.abs(e32.get_field("psi") - psi).max()
    print(f"\n[{env_id} heading turns] |psi| up to {np.abs(e32.get_field('psi')).max():.1f} rad "
          f"(moved {spin:.1f} rad), f32 vs f64 obs header max err {worst:.2e}, {int(alive.sum())} envs alive")
    assert alive.sum() >= n // 4 and spin > 20
    assert worst <= 2e-5, worst
    for e in envs.values():
        e.close()
