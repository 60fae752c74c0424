"""CPU restatement of romi2002/gym-usv's hot path — TEST INFRASTRUCTURE, NOT PRODUCT.

Only ``tests/``, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline`` leg may
import this module, and only as the checker (or the timed CPU baseline).  The product
path (``gym-usv_amd``) never routes through it: it fails loudly without its HIP library.

Parity pinning: this restatement is checked against golden vectors generated from the
reference itself (``tests/golden/make_golden.py`` imports /root/reference read-only in the
build container; fixtures ``tests/golden/*.npz``; checks in ``tests/test_oracle_golden.py``).

Everything is float64 and batched over N envs (struct-of-arrays, one row per env), so the
same code serves as the single-env oracle (N = 1) and as the 4096-env parity checker.
Reference citations are ``path:line`` under the reference repo.
"""
from __future__ import annotations

import math

import numpy as np

# --------------------------------------------------------------------------- constants
SENSOR_COUNT = 128                                   # simple_env.py:11
SENSOR_SPAN = (2 / 3) * (2 * np.pi)                  # simple_env.py:12
SENSOR_MAX_RANGE = 100.0                             # simple_env.py:13
SENSOR_RES = SENSOR_SPAN / SENSOR_COUNT              # simple_env.py:14
SENSOR_START = -np.pi * 2 / 3                        # usv_asmc_ca_env.py:420
DT = 1 / 25                                          # simple_env.py:35
BOUND_HI = 20.0                                      # simple_env.py:56 env_bounds = (0, 20)
MAX_ACC = np.array([1.75, 0.0, 3.0])                 # simple_env.py:34 (+ [1] = 0 at :253)
TARGET_NORM = np.array([np.pi, np.hypot(20.0, 20.0), 10.0, 10.0])   # simple_env.py:80
LOOKAHEAD = (0.005 / 10) * 20                        # simple_env.py:146
OBS_DIM = 15 + SENSOR_COUNT                          # simple_env.py:27
TIME_LIMITS = {"usv-simple": 500, "usv-asmc-simple": 1000, "usv-asmc-v0": None}  # gym_usv/__init__.py

# UsvAsmc coefficients (usv_asmc.py:7-41)
X_U_DOT, Y_V_DOT, Y_R_DOT, N_V_DOT, N_R_DOT = -2.25, -23.13, -1.31, -16.41, -2.79
YVV, YVR, YRV, YRR = -99.99, -5.49, -5.49, -8.8
NVV, NVR, NRV, NRR = -5.49, -8.8, -8.8, -3.49
MASS, IZ, B_TH, C_TH = 30.0, 4.1, 0.41, 0.78
K_U, K_PSI, KMIN_U, KMIN_PSI = 0.1, 0.2, 0.05, 0.2
K2_U, K2_PSI, MU_U, MU_PSI = 0.02, 0.1, 0.05, 0.1
LAMBDA_U, LAMBDA_PSI = 0.001, 1.0
F1, F2, F3 = 2.0, 2.0, 2.0
H = 0.01                                             # usv_asmc.py:47 integral_step
M_MAT = np.array([[MASS - X_U_DOT, 0, 0],
                  [0, MASS - Y_V_DOT, 0 - Y_R_DOT],
                  [0, 0 - N_V_DOT, IZ - N_R_DOT]])   # usv_asmc.py:172-174
M_INV = np.linalg.inv(M_MAT)                         # constant; ref inverts per substep (:226)
# Yv / Yr / Nv / Nr scale factors (usv_asmc.py:101-108)
YV_K = 0.5 * (-40 * 1000) * (1.1 + 0.0045 * (1.01 / 0.09) - 0.1 * (0.27 / 0.09)
                             + 0.016 * ((0.27 / 0.09) ** 2))
YR_K = 6 * (-3.141592 * 1000) * 0.09 * 0.09 * 1.01
NV_K = 0.06 * (-3.141592 * 1000) * 0.09 * 0.09 * 1.01
NR_K = 0.02 * (-3.141592 * 1000) * 0.09 * 0.09 * 1.01 * 1.01

# ASMC per-env persistent state layout (16 unique values; usv_asmc.py:43-49, :237-242)
ASMC_FIELDS = ("psi_d_last", "o", "o_dot", "o_dot_dot",
               "x_dot_last", "y_dot_last", "psi_dot_last",
               "u_dot_last", "v_dot_last", "r_dot_last",
               "e_u_last", "ka_dot_u_last", "ka_dot_psi_last",
               "e_u_int", "ka_u", "ka_psi")
ASMC_N = len(ASMC_FIELDS)


def wrap_angle(a):
    """simple_env.py:63-65 — atan2(sin, cos)."""
    return np.arctan2(np.sin(a), np.cos(a))


def wrap_once(e):
    """Single wrap sign(e)(|e|-2pi) if |e|>pi (usv_asmc.py:120)."""
    return np.where(np.abs(e) > np.pi, np.sign(e) * (np.abs(e) - 2 * np.pi), e)


# --------------------------------------------------------------------------- lidar
def lidar(px, py, psi, ox, oy, orad, n_obs):
    """Batched 128-ray lidar.

    Restates simple_env.py:203-226 -> usv_asmc_ca_env.py:411-437 (compute_sensor_measurments)
    -> :500-519 (compute_obstacle_positions) -> :439-461 (_compute_sensor_distances).

    The reference sorts obstacles by key d_j = |c_j - p| - r_j (argsort, :417) and, per ray,
    takes the first obstacle in that order with proj >= 0, r^2 - perp^2 >= 0 and reading
    proj - sqrt(r^2 - perp^2) < max range.  That is the hit obstacle with the smallest key
    (the "min-key rule"), which is what this restatement and the HIP kernel compute.

    Args: px, py, psi [N]; ox, oy, orad [N, cap] (entries j >= n_obs[i] ignored); n_obs [N].
    Returns: keys [N, cap] (inf where padded), readings [N, 128].
    """
    px, py, psi = (np.asarray(a, dtype=np.float64) for a in (px, py, psi))
    cap = ox.shape[1]
    valid = np.arange(cap)[None, :] < np.asarray(n_obs)[:, None]
    dx = ox - px[:, None]
    dy = oy - py[:, None]
    keys = np.where(valid, np.hypot(dx, dy) - orad, np.inf)             # simple_env.py:205-206
    ang = (SENSOR_START + np.arange(SENSOR_COUNT) * SENSOR_RES)[None, :] + psi[:, None]  # :420-423
    c, s = np.cos(ang)[:, :, None], np.sin(ang)[:, :, None]             # [N, 128, 1]
    # inverse rotation of the obstacle offset, y mirrored (usv_asmc_ca_env.py:506-518)
    proj = c * dx[:, None, :] + s * dy[:, None, :]
    perp = s * dx[:, None, :] - c * dy[:, None, :]
    delta = orad[:, None, :] ** 2 - perp * perp                         # :453
    with np.errstate(invalid="ignore"):
        reading = proj - np.sqrt(np.where(delta >= 0, delta, 0.0))      # :457
    hit = valid[:, None, :] & (proj >= 0) & (delta >= 0) & (reading < SENSOR_MAX_RANGE)
    kk = np.where(hit, keys[:, None, :], np.inf)
    best = np.argmin(kk, axis=2)                                        # min-key == sorted first hit
    any_hit = np.take_along_axis(hit, best[:, :, None], axis=2)[:, :, 0]
    val = np.take_along_axis(reading, best[:, :, None], axis=2)[:, :, 0]
    readings = np.where(any_hit, val, SENSOR_MAX_RANGE)
    return keys, readings


# --------------------------------------------------------------------------- ASMC
class AsmcBatch:
    """Batched restatement of ``UsvAsmc`` (usv_asmc.py:4-244), N independent controllers.

    ``state`` is [N, 16] in ASMC_FIELDS order (psi_d_last, o, o', o'', eta_dot_last(3),
    upsilon_dot_last(3), e_u_last, Ka_dot_u_last, Ka_dot_psi_last, e_u_int, Ka_u, Ka_psi).
    The reference keeps o_last == o, o_dot_last == o_dot, o_dot_dot_last == o_dot_dot after
    every substep (:89-92), so 16 values carry the full state.
    """

    def __init__(self, n):
        self.state = np.zeros((n, ASMC_N))
        self.perturb_step = np.zeros(n, dtype=np.int64)                   # usv_asmc.py:49
        self.fast_substeps = np.zeros(n, dtype=np.int64)   # checker statistic: substeps with |u| > 1.2

    def reset(self, idx=None):
        if idx is None:
            self.state[:] = 0.0
            self.perturb_step[:] = 0
        else:
            self.state[idx] = 0.0
            self.perturb_step[idx] = 0

    def compute(self, action, pos, vel, substeps=10, do_perturb=False):
        """usv_asmc.py:53-244. action [N,2] = (u_d, psi offset)."""
        st = self.state
        a0, a1 = action[:, 0].astype(np.float64), action[:, 1].astype(np.float64)
        x, y, psi = pos[:, 0].copy(), pos[:, 1].copy(), pos[:, 2].copy()
        u, v, r = vel[:, 0].copy(), vel[:, 1].copy(), vel[:, 2].copy()
        (psi_d_last, o, o_d, o_dd, xd_l, yd_l, psid_l, ud_l, vd_l, rd_l,
         e_u_last, kdu_l, kdp_l, e_u_int, ka_u, ka_psi) = (st[:, k].copy() for k in range(ASMC_N))
        for _ in range(substeps):
            speed = np.hypot(u, v)
            beta = np.arcsin(v / (0.001 + speed))                         # :72
            psi_d = psi + beta + a1                                       # :73-77
            r_d = (psi_d - psi_d_last) / H                                # :84
            psi_d_last = psi_d
            o_dd_new = ((r_d - o) * F1 - F3 * o_d) * F2                   # :86
            o_d_new = H * (o_dd_new + o_dd) / 2 + o_d                     # :87
            o = H * (o_d_new + o_d) / 2 + o                               # :88 (uses old o_dot_last)
            o_d, o_dd = o_d_new, o_dd_new
            r_d = o                                                       # :89
            fast = np.abs(u) > 1.2                                        # :95-99
            self.fast_substeps += fast
            xu = np.where(fast, 64.55, -25.0)
            xuu = np.where(fast, -70.92, 0.0)
            vmag = np.sqrt(u * u + v * v)
            yv = YV_K * np.abs(v)                                         # :101-102
            yr, nv, nr = YR_K * vmag, NV_K * vmag, NR_K * vmag            # :103-108
            f_u = ((MASS - Y_V_DOT) * v * r + (xuu * np.abs(u) + xu * u)) / (MASS - X_U_DOT)  # :113
            f_psi = ((-X_U_DOT + Y_V_DOT) * u * v + nr * r) / (IZ - N_R_DOT)                 # :115
            e_psi = wrap_once(psi_d - psi)                                # :119-120
            e_psi_dot = r_d - r                                           # :121
            e_u = a0 - u                                                  # :128
            e_u_int = H * (e_u + e_u_last) / 2 + e_u_int                  # :129
            e_u_last = e_u
            sig_u = e_u + LAMBDA_U * e_u_int                              # :133
            sig_p = e_psi_dot + LAMBDA_PSI * e_psi                        # :134
            kdu = np.where(ka_u > KMIN_U, K_U * np.sign(np.abs(sig_u) - MU_U), KMIN_U)       # :137
            kdp = np.where(ka_psi > KMIN_PSI, K_PSI * np.sign(np.abs(sig_p) - MU_PSI), KMIN_PSI)
            ka_u = H * (kdu + kdu_l) / 2 + ka_u                           # :143
            ka_psi = H * (kdp + kdp_l) / 2 + ka_psi                       # :146
            kdu_l, kdp_l = kdu, kdp
            ua_u = -ka_u * np.sqrt(np.abs(sig_u)) * np.sign(sig_u) - K2_U * sig_u            # :150
            ua_p = -ka_psi * np.sqrt(np.abs(sig_p)) * np.sign(sig_p) - K2_PSI * sig_p        # :151
            tx = (LAMBDA_U * e_u - f_u - ua_u) * (MASS - X_U_DOT)         # :154 (/g_u)
            tz = (LAMBDA_PSI * e_psi - f_psi - ua_p) * (IZ - N_R_DOT)     # :155
            tport = tx / 2 + tz / B_TH                                    # :158
            tstbd = tx / (2 * C_TH) - tz / (B_TH * C_TH)                  # :159
            t0 = tport + C_TH * tstbd                                     # :176
            t2 = 0.5 * B_TH * (tport - C_TH * tstbd)
            t1 = np.zeros_like(t0)
            if do_perturb:                                                # :184-198, T += F @ J
                t = self.perturb_step * H
                k = 10 * (2 * np.pi)
                fx = np.cos(t * k) * 5
                fy = np.cos(t + k + 10) * 5
                cps, sps = np.cos(psi), np.sin(psi)
                t0 = t0 + (fx * cps + fy * sps)
                t1 = t1 + (fx * -sps + fy * cps)
            self.perturb_step = self.perturb_step + 1                     # :199
            # C(nu) = CRB + CA (:201-211), D = Dl - Dn (:213-223); rhs = T - C nu - D nu
            c02 = -MASS * v + 2 * (Y_V_DOT * v + ((Y_R_DOT + N_V_DOT) / 2) * r)
            c12 = MASS * u - X_U_DOT * MASS * u
            c20 = MASS * v + 2 * ((-Y_V_DOT) * v - ((Y_R_DOT + N_V_DOT) / 2) * r)
            c21 = -MASS * u + X_U_DOT * MASS * u
            d00 = -xu - xuu * np.abs(u)
            d11 = -yv - (YVV * np.abs(v) + YVR * np.abs(r))
            d12 = -yr - (YRV * np.abs(v) + YRR * np.abs(r))
            d21 = -nv - (NVV * np.abs(v) + NVR * np.abs(r))
            d22 = -nr - (NRV * np.abs(v) + NRR * np.abs(r))
            rhs0 = t0 - c02 * r - d00 * u
            rhs1 = t1 - c12 * r - (d11 * v + d12 * r)
            rhs2 = t2 - (c20 * u + c21 * v) - (d21 * v + d22 * r)
            ud = M_INV[0, 0] * rhs0 + M_INV[0, 1] * rhs1 + M_INV[0, 2] * rhs2               # :226
            vd = M_INV[1, 0] * rhs0 + M_INV[1, 1] * rhs1 + M_INV[1, 2] * rhs2
            rd = M_INV[2, 0] * rhs0 + M_INV[2, 1] * rhs1 + M_INV[2, 2] * rhs2
            u = H * (ud + ud_l) / 2 + u                                   # :228-229
            v = H * (vd + vd_l) / 2 + v
            r = H * (rd + rd_l) / 2 + r
            ud_l, vd_l, rd_l = ud, vd, rd
            cp, sp = np.cos(psi), np.sin(psi)                             # J(psi_old) :179-181
            xd = cp * u - sp * v                                          # :233
            yd = sp * u + cp * v
            pd = r
            x = H * (xd + xd_l) / 2 + x                                   # :234
            y = H * (yd + yd_l) / 2 + y
            psi = H * (pd + psid_l) / 2 + psi
            xd_l, yd_l, psid_l = xd, yd, pd
        self.state = np.stack([psi_d_last, o, o_d, o_dd, xd_l, yd_l, psid_l, ud_l, vd_l, rd_l,
                               e_u_last, kdu_l, kdp_l, e_u_int, ka_u, ka_psi], axis=1)
        return np.stack([x, y, psi], axis=1), np.stack([u, v, r], axis=1)


# --------------------------------------------------------------------------- usv-simple
class SimpleEnvBatch:
    """Batched restatement of ``UsvSimpleEnv`` (simple_env.py:7-349), N envs.

    Per-env state mirrors the reference attributes: position (x, y, psi), velocity (u, v, r),
    last_action (3; [1] is always 0), progress, path_start / path_end, target_position,
    max_action (3; [1] = 0 after reset), reference_velocity, obstacles (n, xy, radius) and
    the stale ``sensor_data`` distances (:47, returned in the reset obs).
    Each env owns a numpy Generator with gymnasium's seeding rule (PCG64(SeedSequence)).
    """

    obs_dim = OBS_DIM
    act_dim = 2

    def __init__(self, n, cap=32, options=None):
        self.n, self.cap = n, cap
        self.options = dict(options or {})                                # simple_env.py:10,15
        self.info = {}
        z = lambda *s: np.zeros((n,) + s)
        self.position, self.velocity, self.last_action = z(3), z(3), z(3)
        self.max_action = np.tile(np.array([3.0, 0.0, 3.0]), (n, 1))       # simple_env.py:32
        self.ref_v = z()
        self.progress = z()
        self.path_start, self.path_end, self.target = z(2), z(2), z(2)
        self.n_obs = np.zeros(n, dtype=np.int64)
        self.ox, self.oy, self.orad = z(cap), z(cap), z(cap)
        self.sensors = z(SENSOR_COUNT)                                    # stale scan (:47)
        self.rngs = [None] * n

    # ---- observation pieces (simple_env.py:67-96, 133-148) ----
    def ye(self):
        ak = np.arctan2(self.path_end[:, 1] - self.path_start[:, 1],
                        self.path_end[:, 0] - self.path_start[:, 0])      # :134
        return (-(self.position[:, 0] - self.path_start[:, 0]) * np.sin(ak)
                + (self.position[:, 1] - self.path_start[:, 1]) * np.cos(ak))

    def angle_to_target(self):
        d = self.target - self.position[:, :2]                            # :68-69
        return wrap_angle(np.arctan2(d[:, 1], d[:, 0]) - self.position[:, 2])

    def target_state(self):
        dist = np.hypot(self.position[:, 0] - self.target[:, 0],
                        self.position[:, 1] - self.target[:, 1])          # :74
        ts = np.stack([self.angle_to_target(), dist, self.ye(), self.ref_v], axis=1)
        return ts / TARGET_NORM                                           # :79-80

    def obs(self, action):
        """_get_obs(action) (:91-96); ``action`` is [N,3]."""
        act = action[:, [0, 2]] / self.max_action[:, [0, 2]]
        kin = np.concatenate([self.max_action / 10, np.tile(MAX_ACC / 10, (self.n, 1))], axis=1)
        return np.concatenate([self.velocity / 10, self.target_state(), act, kin,
                               self.sensors / SENSOR_MAX_RANGE], axis=1).astype(np.float32)

    def closest_point(self):
        """_get_closest_point (:139-148)."""
        x1, y1 = self.path_start[:, 0], self.path_start[:, 1]
        dx = self.path_end[:, 0] - x1
        dy = self.path_end[:, 1] - y1
        a = (dy * (self.position[:, 1] - y1) + dx * (self.position[:, 0] - x1)) / (dx * dx + dy * dy)
        a = a + LOOKAHEAD
        a = np.clip(a, self.progress, 1)
        return np.stack([x1 + a * dx, y1 + a * dy], axis=1), a

    def reward(self, action):
        """_get_reward (:150-201); action [N,3] is the new filtered action."""
        min_sensor = self.sensors.min(axis=1)
        collision = np.where(min_sensor < 0.2, -20.0, 0.0)                # :153-156
        delta = np.abs(self.last_action - action).sum(axis=1)             # :160
        angle = self.angle_to_target()
        ye = self.ye()
        k = 0.075
        ye_r = np.maximum(np.exp(-np.abs(ye / k)), np.exp(-np.power(ye / k, 2)))   # :167-170
        ang_r = np.exp(-np.abs(angle))                                    # :172
        dact_r = -(delta / 2) * 0.15                                      # :176
        vel_r = np.exp(-np.abs(np.hypot(self.velocity[:, 0], self.velocity[:, 1]) - self.ref_v)) * 0.05
        return 0.0 + collision + ye_r + ang_r + vel_r + dact_r            # :181-186

    # ---- reset (simple_env.py:228-308) ----
    def reset_env(self, i, seed=None, options=None):
        if seed is not None or self.rngs[i] is None:
            self.rngs[i] = np.random.Generator(np.random.PCG64(np.random.SeedSequence(seed)))
        g = self.rngs[i]
        start = g.normal(scale=0.5, size=2) + np.array([BOUND_HI, BOUND_HI]) / 2      # :234
        g.normal(start, scale=0.75); g.uniform(-np.pi, np.pi)                        # :236-237 discarded
        psi = g.uniform(-np.pi, np.pi)                                               # :238
        angle = g.uniform(-np.pi, np.pi)                                             # :241
        dist = g.uniform(100, 110)                                                   # :242
        self.path_start[i] = start
        self.position[i] = [start[0], start[1], psi]
        self.path_end[i] = start + np.array([np.cos(angle), np.sin(angle)]) * dist  # :243
        self.target[i] = g.uniform(0, BOUND_HI, size=2)                              # :245
        self.velocity[i] = g.uniform(0.0, 0.15, size=3)                              # :246
        self.progress[i] = 0.0
        ma = g.uniform(1.50, 3, size=3)                                              # :249
        ma[2] = g.uniform(3, 6)                                                      # :250
        self.ref_v[i] = g.uniform(0.75, ma[0])                                       # :251
        ma[1] = 0.0                                                                  # :254
        self.max_action[i] = ma
        n = int(g.integers(15, 30))                                                  # :257
        pos = g.uniform(0, BOUND_HI, size=(n, 2))                                    # :258
        d_pos = np.hypot(start[0] - pos[:, 0], start[1] - pos[:, 1])
        d_tgt = np.hypot(self.target[i, 0] - pos[:, 0], self.target[i, 1] - pos[:, 1])
        keep = ~((d_pos < 0.5) | (d_tgt < 0.5))                                     # :261-268
        pos = pos[keep]
        if pos.shape[0] == 0:                                                        # :270-274
            pos = g.uniform(0, BOUND_HI, size=(1, 2))
        if options and options.get("place_obstacles_on_path"):                       # :276-288
            k = options["place_obstacles_on_path"]
            mag = g.uniform(0, np.hypot(0.0, BOUND_HI), k)                # hypot(*env_bounds) = 20
            lx = g.normal(np.cos(angle) * mag + start[0], 1)
            ly = g.normal(np.sin(angle) * mag + start[1], 1)
            pos = np.concatenate([pos, np.stack([lx, ly], axis=1)])
        n = pos.shape[0]
        if n > self.cap:
            raise ValueError(f"obstacle count {n} exceeds cap {self.cap}")
        rad = g.uniform(0.15, 0.5, size=n)                                           # :290
        if self.options.get("run_custom_experiment"):                                # :292-300
            x = self.options["experiment"]
            pos = np.asarray(x["obstacle_positions"], dtype=np.float64).reshape(-1, 2)
            rad = np.asarray(x["obstacle_radius"], dtype=np.float64).reshape(-1)
            self.path_start[i] = x["path_start"]
            self.path_end[i] = self.path_start[i] + np.array([np.cos(x["angle"]), np.sin(x["angle"])]) * 100
            self.position[i] = x["position"]
            n = pos.shape[0]
        self.n_obs[i] = n
        self.ox[i], self.oy[i], self.orad[i] = 0.0, 0.0, 0.0
        self.ox[i, :n], self.oy[i, :n], self.orad[i, :n] = pos[:, 0], pos[:, 1], rad

    def reset(self, seeds=None, idx=None, options=None):
        idx = range(self.n) if idx is None else idx
        for k, i in enumerate(idx):
            s = None if seeds is None else seeds[k]
            self.reset_env(i, s, options)
        return self.obs(np.zeros((self.n, 3)))                            # :302 (stale sensors)

    # ---- step (simple_env.py:310-346) ----
    def kinematics(self, action):
        """Action scaling + filter + accel/speed clip + pose update (:311-324)."""
        a3 = np.stack([action[:, 0], np.zeros(self.n), action[:, 1]], axis=1).astype(np.float64)
        a3 = self.max_action * a3
        a3 = 0.8 * self.last_action + 0.2 * a3
        dv = np.clip(a3 - self.velocity, -MAX_ACC, MAX_ACC)
        self.velocity = np.clip(self.velocity + dv, -self.max_action, self.max_action)
        th = self.position[:, 2]
        rot = np.stack([self.velocity[:, 0] * np.cos(th), self.velocity[:, 0] * np.sin(th),
                        self.velocity[:, 2]], axis=1)
        self.position = self.position + rot * DT
        return a3

    def step(self, action):
        a3 = self.kinematics(np.asarray(action, dtype=np.float64))
        return self._finish_step(a3)

    def _finish_step(self, a3):
        self.target, self.progress = self.closest_point()                 # :328
        keys, self.sensors = lidar(self.position[:, 0], self.position[:, 1], self.position[:, 2],
                                   self.ox, self.oy, self.orad, self.n_obs)   # :329
        terminated = keys.min(axis=1) < 0.05                              # :334
        pxy = self.position[:, :2]
        truncated = np.any((pxy > BOUND_HI) | (pxy < 0), axis=1)          # :336
        obs = self.obs(self.last_action)                                  # :338 (previous action)
        rew = self.reward(a3)                                             # :339
        self.info = self.step_info(a3, rew)                               # :341-342
        self.last_action = a3                                             # :343
        return obs, rew, terminated, truncated

    def reset_info(self):
        """_get_info(-1, zeros(3)) of the reset (:102-115, :305)."""
        return {"position": self.position.copy(), "velocity": self.velocity.copy(),
                "path_start": self.path_start.copy(), "path_end": self.path_end.copy(),
                "reward": np.full(self.n, -1.0), "action0": np.zeros(self.n), "action1": np.zeros(self.n),
                "ye": self.ye(), "angle_to_target": self.target_state()[:, 0]}

    def step_info(self, a3, rew):
        """_get_info(reward, action) + reward_info of a step (:102-115, :189-199); ``a3`` is the
        new filtered action, ``self.last_action`` still the previous one."""
        info = {"position": self.position.copy(), "velocity": self.velocity.copy(),
                "path_start": self.path_start.copy(), "path_end": self.path_end.copy(),
                "reward": rew, "action0": a3[:, 0], "action1": a3[:, 2],
                "ye": self.ye(), "angle_to_target": self.target_state()[:, 0]}
        ye = self.ye()
        k = 0.075
        delta = np.abs(self.last_action - a3).sum(axis=1)
        info.update(ye_reward=np.maximum(np.exp(-np.abs(ye / k)), np.exp(-np.power(ye / k, 2))),
                    angle_to_target_reward=np.exp(-np.abs(self.angle_to_target())),
                    delta_action_reward=-(delta / 2) * 0.15, delta_action=delta,
                    velocity_track_reward=np.exp(-np.abs(np.hypot(self.velocity[:, 0], self.velocity[:, 1])
                                                         - self.ref_v)) * 0.05,
                    reference_velocity=self.ref_v.copy(), reward_velocity=self.last_action[:, 0].copy(),
                    reference_velocity_error=self.last_action[:, 0] - self.ref_v)
        return info

    # ---- state exchange with the HIP library (field names = include/usv_hip.h) ----
    def get_state(self):
        return {
            "x": self.position[:, 0], "y": self.position[:, 1], "psi": self.position[:, 2],
            "u": self.velocity[:, 0], "v": self.velocity[:, 1], "r": self.velocity[:, 2],
            "last_u": self.last_action[:, 0], "last_r": self.last_action[:, 2],
            "progress": self.progress,
            "path_x0": self.path_start[:, 0], "path_y0": self.path_start[:, 1],
            "path_x1": self.path_end[:, 0], "path_y1": self.path_end[:, 1],
            "max_u": self.max_action[:, 0], "max_r": self.max_action[:, 2], "ref_v": self.ref_v,
            "n_obs": self.n_obs, "obs_x": self.ox, "obs_y": self.oy, "obs_r": self.orad,
            "sensor_last": self.sensors,
        }


class SimpleAsmcEnvBatch(SimpleEnvBatch):
    """Batched ``UsvSimpleASMCEnv`` (simple_env_asmc.py:7-27): 2x UsvAsmc.compute (20 substeps
    of 0.01 s) then ``UsvSimpleEnv.step(zeros(2))``.  Reset re-creates the controller
    (zero state) and drops ``options`` (:14-16)."""

    def __init__(self, n, cap=32, options=None, perturb=False):
        super().__init__(n, cap, options)
        self.asmc = AsmcBatch(n)
        self.perturb = perturb           # compute(..., do_perturb) (the reference env passes False)

    def reset_env(self, i, seed=None, options=None):
        self.asmc.reset([i])
        super().reset_env(i, seed, None)

    def step(self, action):
        action = np.asarray(action, dtype=np.float64)
        for _ in range(2):                                                # simple_env_asmc.py:19-25
            self.position, self.velocity = self.asmc.compute(action, self.position, self.velocity,
                                                             do_perturb=self.perturb)
        a3 = self.kinematics(np.zeros((self.n, 2)))                       # :27 super().step(zeros)
        return self._finish_step(a3)

    def get_state(self):
        st = super().get_state()
        st["asmc"] = self.asmc.state
        return st


# --------------------------------------------------------------------------- vector wrapper
class OracleVectorEnv:
    """N oracle envs behind the SB3/gymnasium vector semantics the HIP VectorEnv implements:
    TimeLimit(max_episode_steps) (gym_usv/__init__.py:24-34) and same-step autoreset
    (``final_obs`` = the terminal obs; the returned obs is the reset obs)."""

    def __init__(self, env_id, num_envs, cap=32, options=None, perturb=False):
        if env_id == "usv-simple":
            assert not perturb, "do_perturb is usv-asmc-simple's"
            self.env = SimpleEnvBatch(num_envs, cap, options)
        else:
            self.env = SimpleAsmcEnvBatch(num_envs, cap, options, perturb)
        self.limit = TIME_LIMITS[env_id]
        self.elapsed = np.zeros(num_envs, dtype=np.int64)

    def reset(self, seeds):
        self.elapsed[:] = 0
        return self.env.reset(seeds)

    def step(self, actions):
        obs, rew, term, trunc = self.env.step(actions)
        self.elapsed += 1
        if self.limit:
            trunc = trunc | (self.elapsed >= self.limit)
        done = term | trunc
        final_obs = obs.copy()
        if done.any():
            idx = np.flatnonzero(done)
            self.env.reset(idx=idx)
            self.elapsed[idx] = 0
            obs = obs.copy()
            obs[idx] = self.env.obs(np.zeros((self.env.n, 3)))[idx]
        return obs, rew, term, trunc, final_obs, done


# --------------------------------------------------------------------------- usv-asmc-v0 (legacy)
# UsvAsmcEnv coefficients that differ from UsvAsmc (usv_asmc_env.py:20,51-53,74-78)
V0_MIN_SPEED = 0.3
V0_K_AK, V0_K_YE, V0_SIGMA_YE = 5.72, 0.5, 1.0
V0_MAX_ACTION = np.pi / 2
V0_C_ACTION = 1.0 / np.power((V0_MAX_ACTION / 2 - (-V0_MAX_ACTION) / 2) / H, 2)   # :77
V0_W_ACTION = 0.2                                                                 # :78
V0_T_MIN, V0_T_MAX = -30.0, 36.5                                                  # :182-185
f32 = np.float32


class AsmcV0Batch:
    """Batched restatement of the legacy ``UsvAsmcEnv`` (id usv-asmc-v0, usv_asmc_env.py:14-401).

    One 0.01 s ASMC + Gonzalez-Garcia plant step per env step with a sigmoid desired speed
    (:151-156), no r_d filter (e_psi_dot = -r, :149), thrust saturation (:182-185) and the
    float32 rounding the reference applies: T, CRB, CA, Dl, Dn, J are float32 arrays
    (:191-222) and the whole state is stored as float32 after every step (:247-251).  Scalars
    follow NumPy 2 promotion (a float32 operand with Python scalars stays float32).  Quirk:
    e_u_last is never updated (:159, :251).  obs = [u, v_ak, r, ye, psi_ak, action_last].
    Resets draw from a per-env ``np.random.RandomState`` exactly like the reference's global
    ``np.random.uniform`` calls (:260-279) after ``np.random.seed(seed)``.
    """

    obs_dim = 6
    act_dim = 1

    def __init__(self, n):
        self.n = n
        z = lambda *s: np.zeros((n,) + s)
        self.velocity, self.position, self.aux = z(3), z(3), z(3)
        self.last = z(9)
        self.target = z(6)          # x_0, y_0, desired_speed, ak, x_d, y_d
        self.state = z(6)
        self.first = np.ones(n, bool)   # reference state is float64 until the first step
        self.rngs = [None] * n

    def reset_env(self, i, seed=None):
        if seed is not None or self.rngs[i] is None:
            self.rngs[i] = np.random.RandomState(seed)
        g = self.rngs[i]
        x, y = g.uniform(-2.5, 2.5), g.uniform(-2.5, 2.5)                  # :260-261
        psi = g.uniform(-np.pi, np.pi)                                     # :262
        x0, y0 = g.uniform(-2.5, 2.5), g.uniform(-2.5, 2.5)                # :275-276
        xd = g.uniform(15, 30)                                             # :277
        yd = y0                                                            # :278
        ds = g.uniform(1.4, 2.4)                                           # :279
        ak = float(f32(math.atan2(yd - y0, xd - x0)))                      # :281-282
        psi_ak = float(f32(wrap_once(np.float64(psi - ak))))              # :284-286
        ye = -(x - x0) * math.sin(ak) + (y - y0) * math.cos(ak)            # :287
        self.velocity[i] = 0.0
        self.position[i] = [x, y, psi]
        self.aux[i] = 0.0
        self.last[i] = 0.0
        self.target[i] = [x0, y0, ds, ak, xd, yd]
        # body_to_path(0, 0, psi_ak) -> v_ak = 0 (:289)
        self.state[i] = [0.0, 0.0, 0.0, ye, psi_ak, 0.0]
        self.first[i] = True

    def reset(self, seeds=None, idx=None):
        idx = range(self.n) if idx is None else idx
        for k, i in enumerate(idx):
            self.reset_env(i, None if seeds is None else seeds[k])
        return self.state.astype(np.float32)

    def step(self, action):
        """action [N] (or [N,1]) heading offsets; returns obs [N,6] f32, reward [N], done [N]."""
        a = np.asarray(action, dtype=np.float32).reshape(self.n)
        fs = ~self.first                         # envs whose stored state is float32
        u, v, r = (self.velocity[:, k] for k in range(3))
        x, y, psi = (self.position[:, k] for k in range(3))
        e_u_int, ka_u, ka_psi = (self.aux[:, k] for k in range(3))
        xd_l, yd_l, pd_l, ud_l, vd_l, rd_l, e_u_last, kdu_l, kdp_l = (self.last[:, k] for k in range(9))
        x0, y0, ds, ak = (self.target[:, k] for k in range(4))
        a_last = self.state[:, 5]
        # action_dot: float32 once the stored state is float32 (:120)
        ad64 = (a.astype(np.float64) - a_last) / H
        ad32 = ((a - a_last.astype(np.float32)) / np.float32(H)).astype(np.float64)
        action_dot = np.where(fs, ad32, ad64)
        psi_d = wrap_once(a.astype(np.float64) + ak)                      # :123-124
        fast = np.abs(u) > 1.2                                             # :126-130

        def f32ops(vals):
            """Evaluate in float32 where the env's state is float32 (NumPy 2 promotion)."""
            return np.where(fs, vals(np.float32).astype(np.float64), vals(np.float64))

        def hydro(dt):
            uu, vv, rr = u.astype(dt), v.astype(dt), r.astype(dt)
            mag = np.sqrt(np.power(uu, 2) + np.power(vv, 2))
            yv = dt(0.5) * (dt(-40 * 1000) * np.abs(vv)) * dt(1.1 + 0.0045 * (1.01 / 0.09) - 0.1 * (0.27 / 0.09) + 0.016 * np.power((0.27 / 0.09), 2))
            yr = dt(6 * (-3.141592 * 1000)) * mag * dt(0.09) * dt(0.09) * dt(1.01)
            nv = dt(0.06 * (-3.141592 * 1000)) * mag * dt(0.09) * dt(0.09) * dt(1.01)
            nr = dt(0.02 * (-3.141592 * 1000)) * mag * dt(0.09) * dt(0.09) * dt(1.01) * dt(1.01)
            return yv, yr, nv, nr
        y64, y32 = hydro(np.float64), hydro(np.float32)
        yv, yr, nv, nr = (np.where(fs, b.astype(np.float64), c) for b, c in zip(y32, y64))   # :132-139
        xu = np.where(fast, 64.55, -25.0)
        xuu = np.where(fast, -70.92, 0.0)

        def fpart(dt):
            uu, vv, rr = u.astype(dt), v.astype(dt), r.astype(dt)
            fu = (dt(MASS - Y_V_DOT) * vv * rr + (xuu.astype(dt) * np.abs(uu) + xu.astype(dt) * uu)) / dt(MASS - X_U_DOT)
            fp = (dt(-X_U_DOT + Y_V_DOT) * uu * vv + (nr.astype(dt) * rr)) / dt(IZ - N_R_DOT)
            return fu, fp
        fu32, fp32 = fpart(np.float32)
        fu64, fp64 = fpart(np.float64)
        f_u = np.where(fs, fu32.astype(np.float64), fu64)                  # :144
        f_psi = np.where(fs, fp32.astype(np.float64), fp64)                # :145
        e_psi = wrap_once(psi_d - psi)                                     # :147-148
        e_psi_dot = 0 - r                                                  # :149
        u_psi = 1 / (1 + np.exp(10 * (np.abs(e_psi) * (2 / np.pi) - 0.5)))    # :153
        u_d = (ds - V0_MIN_SPEED) * u_psi + V0_MIN_SPEED                   # :155-156
        e_u = u_d - u                                                      # :158
        e_u_int = H * (e_u + e_u_last) / 2 + e_u_int                       # :159 (e_u_last stale)
        sig_u = e_u + LAMBDA_U * e_u_int                                   # :161
        sig_p = e_psi_dot + LAMBDA_PSI * e_psi                             # :162
        kdu = np.where(ka_u > KMIN_U, K_U * np.sign(np.abs(sig_u) - MU_U), KMIN_U)       # :164
        kdp = np.where(ka_psi > KMIN_PSI, K_PSI * np.sign(np.abs(sig_p) - MU_PSI), KMIN_PSI)
        ka_u = H * (kdu + kdu_l) / 2 + ka_u                                # :167
        ka_psi = H * (kdp + kdp_l) / 2 + ka_psi                            # :170
        ua_u = -ka_u * np.sqrt(np.abs(sig_u)) * np.sign(sig_u) - K2_U * sig_u            # :173
        ua_p = -ka_psi * np.sqrt(np.abs(sig_p)) * np.sign(sig_p) - K2_PSI * sig_p        # :174
        tx = (LAMBDA_U * e_u - f_u - ua_u) / (1 / (MASS - X_U_DOT))       # :176
        tz = (LAMBDA_PSI * e_psi - f_psi - ua_p) / (1 / (IZ - N_R_DOT))   # :177
        tport = np.clip(tx / 2 + tz / B_TH, V0_T_MIN, V0_T_MAX)            # :179-185
        tstbd = np.clip(tx / (2 * C_TH) - tz / (B_TH * C_TH), V0_T_MIN, V0_T_MAX)
        t0 = (tport + C_TH * tstbd).astype(np.float32)                     # :191 float32 T
        t2 = (0.5 * B_TH * (tport - C_TH * tstbd)).astype(np.float32)
        # CRB, CA, Dl, Dn as float32 arrays (:193-212), entries computed in the stored dtype
        uu, vv, rr = u.astype(np.float32), v.astype(np.float32), r.astype(np.float32)

        def cast(z):
            return z.astype(np.float32)
        m = np.float32(MASS)
        c02 = cast(np.where(fs, (0 - m * vv).astype(np.float64), 0 - MASS * v)) + cast(np.where(fs, (np.float32(2) * (np.float32(Y_V_DOT) * vv + np.float32((Y_R_DOT + N_V_DOT) / 2) * rr)).astype(np.float64), 2 * (Y_V_DOT * v + ((Y_R_DOT + N_V_DOT) / 2) * r)))
        c12 = cast(np.where(fs, (m * uu).astype(np.float64), MASS * u)) + cast(np.where(fs, (0 - np.float32(X_U_DOT * MASS) * uu).astype(np.float64), 0 - X_U_DOT * MASS * u))
        c20 = cast(np.where(fs, (m * vv).astype(np.float64), MASS * v)) + cast(np.where(fs, (np.float32(2) * ((np.float32(-Y_V_DOT) * vv) - np.float32((Y_R_DOT + N_V_DOT) / 2) * rr)).astype(np.float64), 2 * ((-Y_V_DOT) * v - ((Y_R_DOT + N_V_DOT) / 2) * r)))
        c21 = cast(np.where(fs, (0 - m * uu).astype(np.float64), 0 - MASS * u)) + cast(np.where(fs, (np.float32(X_U_DOT * MASS) * uu).astype(np.float64), X_U_DOT * MASS * u))
        av = np.where(fs, np.abs(vv).astype(np.float64), np.abs(v))
        ar = np.where(fs, np.abs(rr).astype(np.float64), np.abs(r))
        d00 = cast(0 - xu) - cast(xuu * np.abs(u))
        d11 = cast(0 - yv) - cast(f32ops(lambda dt: dt(YVV) * av.astype(dt) + dt(YVR) * ar.astype(dt)))
        d12 = cast(0 - yr) - cast(f32ops(lambda dt: dt(YRV) * av.astype(dt) + dt(YRR) * ar.astype(dt)))
        d21 = cast(0 - nv) - cast(f32ops(lambda dt: dt(NVV) * av.astype(dt) + dt(NVR) * ar.astype(dt)))
        d22 = cast(0 - nr) - cast(f32ops(lambda dt: dt(NRV) * av.astype(dt) + dt(NRR) * ar.astype(dt)))
        # T - C nu - D nu: float32 products/sums where nu is float32, float64 on the first step
        def rhs(dt):
            U, V, Rr = u.astype(dt), v.astype(dt), r.astype(dt)
            cn0 = c02.astype(dt) * Rr
            cn1 = c12.astype(dt) * Rr
            cn2 = c20.astype(dt) * U + c21.astype(dt) * V
            dn0 = d00.astype(dt) * U
            dn1 = d11.astype(dt) * V + d12.astype(dt) * Rr
            dn2 = d21.astype(dt) * V + d22.astype(dt) * Rr
            return ((t0.astype(dt) - cn0) - dn0, (dt(0) - cn1) - dn1, (t2.astype(dt) - cn2) - dn2)
        r32, r64 = rhs(np.float32), rhs(np.float64)
        rhs0, rhs1, rhs2 = (np.where(fs, b.astype(np.float64), c) for b, c in zip(r32, r64))
        ud = M_INV[0, 0] * rhs0 + M_INV[0, 1] * rhs1 + M_INV[0, 2] * rhs2               # :214-215
        vd = M_INV[1, 0] * rhs0 + M_INV[1, 1] * rhs1 + M_INV[1, 2] * rhs2
        rd = M_INV[2, 0] * rhs0 + M_INV[2, 1] * rhs1 + M_INV[2, 2] * rhs2
        u = H * (ud + ud_l) / 2 + u                                        # :216-217
        v = H * (vd + vd_l) / 2 + v
        r = H * (rd + rd_l) / 2 + r
        # J is a float32 array (:220-222): cos/sin of the stored (float32) heading, or of the
        # float64 reset heading on the first step, rounded to float32
        psif = psi.astype(np.float32)
        cj = np.where(fs, np.cos(psif).astype(np.float64), np.cos(psi).astype(np.float32).astype(np.float64))
        sj = np.where(fs, np.sin(psif).astype(np.float64), np.sin(psi).astype(np.float32).astype(np.float64))
        xd = cj * u - sj * v                                               # :224
        yd = sj * u + cj * v
        pd = r
        x = H * (xd + xd_l) / 2 + x                                        # :225
        y = H * (yd + yd_l) / 2 + y
        psi = H * (pd + pd_l) / 2 + psi
        psi = wrap_once(psi)                                               # :228-229
        psi_ak = wrap_once(psi - ak)                                       # :231-232
        ye = -(x - x0) * np.sin(ak) + (y - y0) * np.cos(ak)                # :234
        ye_abs = np.abs(ye)
        # compute_reward (:364-374)
        pa = np.abs(psi_ak)
        ad = np.where(fs, np.power(action_dot.astype(np.float32), 2).astype(np.float64), np.power(action_dot, 2))
        cad = np.where(fs, (np.float32(-V0_C_ACTION) * ad.astype(np.float32)).astype(np.float64), -V0_C_ACTION * ad)
        r_act = V0_W_ACTION * np.tanh(cad)
        r_ye = np.where(ye_abs > V0_SIGMA_YE, np.exp(-V0_K_YE * ye_abs), np.exp(-V0_K_YE * np.power(ye_abs, 2) / V0_SIGMA_YE))
        r_ak = -np.exp(V0_K_AK * (pa - np.pi))
        reward = np.where(pa < np.pi / 2, r_act + r_ye, r_ak)
        v_ak = np.sin(psi_ak) * u + np.cos(psi_ak) * v                     # body_to_path :376-390
        done = (ye_abs > 10) | (np.abs(x) > 30)                             # :241-245
        reward = np.where(done, -1.0, reward)
        q = lambda z: z.astype(np.float32).astype(np.float64)              # stored float32 (:247-251)
        self.state = np.stack([q(u), q(v_ak), q(r), q(ye), q(psi_ak), a.astype(np.float64)], axis=1)
        self.velocity = np.stack([q(u), q(v), q(r)], axis=1)
        self.position = np.stack([q(x), q(y), q(psi)], axis=1)
        self.aux = np.stack([q(e_u_int), q(ka_u), q(ka_psi)], axis=1)
        self.last = np.stack([q(xd), q(yd), q(pd), q(ud), q(vd), q(rd), q(e_u_last), q(kdu), q(kdp)], axis=1)
        self.first[:] = False
        return self.state.astype(np.float32), reward, done


# --------------------------------------------------------------------------- legacy float64 family
PID_KP_U, PID_KI_U, PID_KD_U, PID_KP_PSI, PID_KD_PSI = 1.1, 0.2, 0.1, 0.8, 3.0   # usv_pid_env.py:40-44
YE_INT_K_I = 0.001                                                               # usv_asmc_ye_int_env.py:51
LEGACY_MAX_YE, LEGACY_MIN_X = 10.0, -10.0    # usv_asmc_ye_int_env.py:63,78 / usv_pid_env.py:60


class LegacyF64Batch:
    """Batched restatement of the float64 legacy path-following envs built on the usv-asmc-v0
    template:

    * ``family="ye_int"`` -- ``UsvAsmcYeIntEnv`` (id usv-asmc-ye-int-v0,
      usv_asmc_ye_int_env.py:92-253): the usv-asmc-v0 ASMC + plant step in float64 (no float32
      arrays), plus a cross-track integral that restarts when ye changes sign (:230-235); the
      obs carries ye_ss = ye + k_i * ye_int (:235, :247); reward r_act + (exp(-k_ye |ye|) or
      the heading penalty) (:350-360); reset ranges x, y ~ U(-5, 5), speed ~ U(0.4, 1.4)
      (:256-296).
    * ``family="pid"`` -- ``UsvPidEnv`` (id usv-pid-v0, usv_pid_env.py:89-233): the same plant
      driven by a PID surge/heading law (:148-155; e_u_last is never updated, so e_u_dot =
      e_u / h), the usv-asmc-v0 reward (:329-338), reset ranges as usv-asmc-v0 but speed ~
      U(0.4, 1.4) (:236-276).

    Both end an episode when |ye| > 10 or x < -10 with reward -1 (ye_int :241-245, pid
    :219-223).  The state is float64 throughout; only ``ak`` and the reset ``psi_ak`` are
    rounded to float32 (ye_int :282-286, pid :260-264).  Citations below are
    usv_asmc_ye_int_env.py lines; usv_pid_env.py has the same statements 4 (step) or
    20 (reset) lines earlier.  Actions are float32 scalars (promoted to float64 against the
    float64 state).  Resets draw from a per-env ``np.random.RandomState`` in the reference order.
    """

    obs_dim = 6
    act_dim = 1

    def __init__(self, n, family):
        assert family in ("ye_int", "pid")
        self.n, self.family = n, family
        z = lambda *s: np.zeros((n,) + s)
        self.velocity, self.position = z(3), z(3)
        self.aux = z(4)             # e_u_int, Ka_u, Ka_psi, ye_int (ye_int: ye-int env only)
        self.last = z(10)           # eta_dot_last(3), upsilon_dot_last(3), e_u_last, Ka_dot_u/psi_last, ye_last
        self.target = z(6)          # x_0, y_0, desired_speed, ak, x_d, y_d
        self.state = z(6)
        self.rngs = [None] * n

    def reset_env(self, i, seed=None):
        if seed is not None or self.rngs[i] is None:
            self.rngs[i] = np.random.RandomState(seed)
        g = self.rngs[i]
        lim = 5.0 if self.family == "ye_int" else 2.5
        x, y = g.uniform(-lim, lim), g.uniform(-lim, lim)                  # :258-259
        psi = g.uniform(-np.pi, np.pi)
        x0, y0 = g.uniform(-2.5, 2.5), g.uniform(-2.5, 2.5)
        xd = g.uniform(15, 30)
        yd = y0
        ds = g.uniform(0.4, 1.4)                                           # :279
        ak = float(f32(math.atan2(yd - y0, xd - x0)))                      # :281-282
        psi_ak = float(f32(wrap_once(np.float64(psi - ak))))              # :284-286
        ye = -(x - x0) * math.sin(ak) + (y - y0) * math.cos(ak)            # :287-288
        self.velocity[i] = 0.0
        self.position[i] = [x, y, psi]
        self.aux[i] = 0.0
        self.last[i] = 0.0
        self.target[i] = [x0, y0, ds, ak, xd, yd]
        self.state[i] = [0.0, 0.0, 0.0, ye, psi_ak, 0.0]                   # body_to_path(0, 0) = 0 (:289-291)

    def reset(self, seeds=None, idx=None):
        idx = range(self.n) if idx is None else idx
        for k, i in enumerate(idx):
            self.reset_env(i, None if seeds is None else seeds[k])
        return self.state.astype(np.float32)

    def step(self, action):
        """action [N] heading offsets (float32); returns obs [N,6] f32, reward [N], done [N]."""
        a = np.asarray(action, dtype=np.float32).reshape(self.n).astype(np.float64)
        u, v, r = (self.velocity[:, k] for k in range(3))
        x, y, psi = (self.position[:, k] for k in range(3))
        e_u_int, ka_u, ka_psi, ye_int = (self.aux[:, k] for k in range(4))
        xd_l, yd_l, pd_l, ud_l, vd_l, rd_l, e_u_last, kdu_l, kdp_l, ye_last = (self.last[:, k] for k in range(10))
        x0, y0, ds, ak = (self.target[:, k] for k in range(4))
        action_dot = (a - self.state[:, 5]) / H                            # :113
        psi_d = wrap_once(a + ak)                                          # :116-117
        fast = np.abs(u) > 1.2                                             # :119-123
        xu = np.where(fast, 64.55, -25.0)
        xuu = np.where(fast, -70.92, 0.0)
        mag = np.sqrt(np.power(u, 2) + np.power(v, 2))
        yv = 0.5 * (-40 * 1000 * np.abs(v)) * (1.1 + 0.0045 * (1.01 / 0.09) - 0.1 * (0.27 / 0.09) + 0.016 * np.power((0.27 / 0.09), 2))
        yr = 6 * (-3.141592 * 1000) * mag * 0.09 * 0.09 * 1.01            # :125-132
        nv = 0.06 * (-3.141592 * 1000) * mag * 0.09 * 0.09 * 1.01
        nr = 0.02 * (-3.141592 * 1000) * mag * 0.09 * 0.09 * 1.01 * 1.01
        g_u, g_psi = 1 / (MASS - X_U_DOT), 1 / (IZ - N_R_DOT)              # :134-138
        f_u = ((MASS - Y_V_DOT) * v * r + (xuu * np.abs(u) + xu * u)) / (MASS - X_U_DOT)
        f_psi = ((-X_U_DOT + Y_V_DOT) * u * v + (nr * r)) / (IZ - N_R_DOT)
        e_psi = wrap_once(psi_d - psi)                                     # :140-152
        e_psi_dot = 0 - r
        u_psi = 1 / (1 + np.exp(10 * (np.abs(e_psi) * (2 / np.pi) - 0.5)))
        u_d = (ds - V0_MIN_SPEED) * u_psi + V0_MIN_SPEED
        e_u = u_d - u
        e_u_int = H * (e_u + e_u_last) / 2 + e_u_int
        if self.family == "ye_int":                                        # ASMC, :154-170
            sig_u = e_u + LAMBDA_U * e_u_int
            sig_p = e_psi_dot + LAMBDA_PSI * e_psi
            kdu = np.where(ka_u > KMIN_U, K_U * np.sign(np.abs(sig_u) - MU_U), KMIN_U)
            kdp = np.where(ka_psi > KMIN_PSI, K_PSI * np.sign(np.abs(sig_p) - MU_PSI), KMIN_PSI)
            ka_u = H * (kdu + kdu_l) / 2 + ka_u
            ka_psi = H * (kdp + kdp_l) / 2 + ka_psi
            ua_u = (-ka_u * np.power(np.abs(sig_u), 0.5) * np.sign(sig_u)) - (K2_U * sig_u)
            ua_p = (-ka_psi * np.power(np.abs(sig_p), 0.5) * np.sign(sig_p)) - (K2_PSI * sig_p)
            tx = ((LAMBDA_U * e_u) - f_u - ua_u) / g_u
            tz = ((LAMBDA_PSI * e_psi) - f_psi - ua_p) / g_psi
        else:                                                              # PID, usv_pid_env.py:149-155
            kdu, kdp = kdu_l, kdp_l
            e_u_dot = (e_u - e_u_last) / H
            ua_u = (PID_KP_U * e_u) + (PID_KI_U * e_u_int) + (PID_KD_U * e_u_dot)
            ua_p = (PID_KP_PSI * e_psi) + (PID_KD_PSI * e_psi_dot)
            tx = (-f_u + ua_u) / g_u
            tz = (-f_psi + ua_p) / g_psi
        tport = tx / 2 + tz / B_TH                                         # :172-178
        tstbd = tx / (2 * C_TH) - tz / (B_TH * C_TH)
        tport = np.where(tport > 36.5, 36.5, tport)
        tport = np.where(tport < -30, -30.0, tport)
        tstbd = np.where(tstbd > 36.5, 36.5, tstbd)
        tstbd = np.where(tstbd < -30, -30.0, tstbd)
        t0 = tport + C_TH * tstbd                                          # :184
        t2 = 0.5 * B_TH * (tport - C_TH * tstbd)
        # C = CRB + CA, D = Dl - Dn (:186-205); only their non-zero entries enter C nu, D nu
        c02 = (0 - MASS * v) + 2 * ((Y_V_DOT * v) + ((Y_R_DOT + N_V_DOT) / 2) * r)
        c12 = (MASS * u) + (0 - X_U_DOT * MASS * u)
        c20 = (MASS * v) + 2 * (((0 - Y_V_DOT) * v) - ((Y_R_DOT + N_V_DOT) / 2) * r)
        c21 = (0 - MASS * u) + (X_U_DOT * MASS * u)
        av, ar = np.abs(v), np.abs(r)
        d00 = (0 - xu) - xuu * np.abs(u)
        d11 = (0 - yv) - (YVV * av + YVR * ar)
        d12 = (0 - yr) - (YRV * av + YRR * ar)
        d21 = (0 - nv) - (NVV * av + NVR * ar)
        d22 = (0 - nr) - (NRV * av + NRR * ar)
        rhs0 = (t0 - c02 * r) - d00 * u                                    # :207-208
        rhs1 = (0 - c12 * r) - (d11 * v + d12 * r)
        rhs2 = (t2 - (c20 * u + c21 * v)) - (d21 * v + d22 * r)
        ud = M_INV[0, 0] * rhs0 + M_INV[0, 1] * rhs1 + M_INV[0, 2] * rhs2
        vd = M_INV[1, 0] * rhs0 + M_INV[1, 1] * rhs1 + M_INV[1, 2] * rhs2
        rd = M_INV[2, 0] * rhs0 + M_INV[2, 1] * rhs1 + M_INV[2, 2] * rhs2
        u = H * (ud + ud_l) / 2 + u                                        # :209-211
        v = H * (vd + vd_l) / 2 + v
        r = H * (rd + rd_l) / 2 + r
        cj, sj = np.cos(psi), np.sin(psi)                                  # J(psi) :213-215
        xd, yd, pd = cj * u - sj * v, sj * u + cj * v, r
        x = H * (xd + xd_l) / 2 + x                                        # :217-219
        y = H * (yd + yd_l) / 2 + y
        psi = wrap_once(H * (pd + pd_l) / 2 + psi)                         # :221-222
        psi_ak = wrap_once(psi - ak)                                       # :224-225
        ye = -(x - x0) * np.sin(ak) + (y - y0) * np.cos(ak)               # :227
        ye_abs = np.abs(ye)
        pa = np.abs(psi_ak)
        r_act = V0_W_ACTION * np.tanh(-V0_C_ACTION * np.power(action_dot, 2))
        r_ak = -np.exp(V0_K_AK * (pa - np.pi))
        if self.family == "ye_int":
            ye_int = np.where(np.sign(ye) != np.sign(ye_last), 0.0, ye_int)   # :230-232
            ye_int = H * (ye + ye_last) + ye_int
            ye_last = ye
            ye_obs = ye + YE_INT_K_I * ye_int                              # ye_ss (:235)
            reward = r_act + np.where(pa < np.pi / 2, np.exp(-V0_K_YE * ye_abs), r_ak)   # :350-360
        else:
            ye_obs = ye
            r_ye = np.where(ye_abs > V0_SIGMA_YE, np.exp(-V0_K_YE * ye_abs),
                            np.exp(-V0_K_YE * np.power(ye_abs, 2) / V0_SIGMA_YE))
            reward = np.where(pa < np.pi / 2, r_act + r_ye, r_ak)         # usv_pid_env.py:329-338
        v_ak = np.sin(psi_ak) * u + np.cos(psi_ak) * v                     # body_to_path :239, :362-376
        done = (ye_abs > LEGACY_MAX_YE) | (x < LEGACY_MIN_X)                # :241-245
        reward = np.where(done, -1.0, reward)
        self.state = np.stack([u, v_ak, r, ye_obs, psi_ak, a], axis=1)
        self.velocity = np.stack([u, v, r], axis=1)
        self.position = np.stack([x, y, psi], axis=1)
        self.aux = np.stack([e_u_int, ka_u, ka_psi, ye_int], axis=1)
        self.last = np.stack([xd, yd, pd, ud, vd, rd, e_u_last, kdu, kdp, ye_last], axis=1)
        return self.state.astype(np.float32), reward, done
