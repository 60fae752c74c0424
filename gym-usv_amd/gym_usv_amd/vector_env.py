"""Batched HIP vector env: the gymnasium ``VectorEnv`` reset()/step() surface over libusvhip.

Replaces N x ``UsvSimpleEnv`` / ``UsvSimpleASMCEnv`` (gym_usv/envs/simple_env.py:7-349,
simple_env_asmc.py:7-32) stepped one by one by SB3's DummyVecEnv
(train_test/sb3_train_vec.py:67): one kernel launch steps every env, outputs stay in HBM as
torch tensors, done envs are reset inside the same launch (same-step autoreset, the terminal
observation in ``info["final_obs"]``), and the TimeLimit of the registered id
(gym_usv/__init__.py:24-34) is applied in-kernel.
"""
from __future__ import annotations

import ctypes
import sys
import warnings
import weakref

import numpy as np
import torch

from . import _lib
from .spaces import Box

# storage use count (a private torch binding): a copy=True output set is reused only when its storage
# has no view outside the env; without the binding every copy=True step allocates a fresh set
_STORAGE_USE_COUNT = getattr(torch._C, "_storage_Use_Count", None)

ENV_SPECS = {
    # id: (mode, max_episode_steps)  -- gym_usv/__init__.py:3-34
    "usv-simple": (_lib.MODE_SIMPLE, 500),
    "usv-asmc-simple": (_lib.MODE_ASMC_SIMPLE, 1000),
    "usv-asmc-v0": (_lib.MODE_ASMC_V0, 0),      # registered without max_episode_steps (:3-6)
    "usv-pid-v0": (_lib.MODE_PID_V0, 0),        # :8-11
    "usv-asmc-ye-int-v0": (_lib.MODE_ASMC_YE_INT_V0, 0),   # :13-16
}
LEGACY_IDS = ("usv-asmc-v0", "usv-pid-v0", "usv-asmc-ye-int-v0")


def _spaces(env_id):
    """Observation / action spaces as the reference declares them."""
    if env_id in LEGACY_IDS:    # usv_asmc_env.py:74-96, usv_pid_env.py:75-86, usv_asmc_ye_int_env.py:80-90
        lo = np.array([-1.5, -1.5, -1.0, -10, -np.pi, -np.pi / 2], dtype=np.float32)
        hi = np.array([1.5, 1.5, 1.0, 10, np.pi, np.pi / 2], dtype=np.float32)
        return (Box(lo, hi, dtype=np.float32),
                Box(-np.pi / 2, np.pi / 2, shape=(1,), dtype=np.float32))
    return (Box(-1, 1, shape=(_lib.OBS_DIM,), dtype=np.float32),          # simple_env.py:27,30
            Box(np.array([0.2, -1]), np.array([1, 1]), shape=(2,), dtype=np.float32))


def np_rng_words(seeds):
    """USV_FIELD_NP_RNG rows for numpy Generator(PCG64(SeedSequence(seed))) per seed: the state
    and increment as 32-bit halves, has_uint32, uinteger (include/usv_hip.h)."""
    out = np.zeros((len(seeds), 10), dtype=np.uint32)
    m64, m32 = (1 << 64) - 1, (1 << 32) - 1
    for i, sd in enumerate(seeds):
        st = np.random.PCG64(np.random.SeedSequence(int(sd))).state
        a, b = st["state"]["state"], st["state"]["inc"]
        for k, w in enumerate((a >> 64, a & m64, b >> 64, b & m64)):
            out[i, 2 * k], out[i, 2 * k + 1] = w & m32, w >> 32
        out[i, 8], out[i, 9] = st["has_uint32"], st["uinteger"]
    return out.view(np.int32)


def np_mt_words(seeds):
    """USV_FIELD_NP_MT rows: np.random.RandomState(seed)'s MT19937 key[624] and pos, i.e. the
    global stream after np.random.seed(seed) that the legacy envs' resets draw from."""
    out = np.zeros((len(seeds), 625), dtype=np.uint32)
    for i, sd in enumerate(seeds):
        _, key, pos, _, _ = np.random.RandomState(int(sd)).get_state(legacy=True)
        out[i, :624], out[i, 624] = key, pos
    return out.view(np.int32)


def _stream_ptr(device):
    return ctypes.c_void_p(torch.cuda.current_stream(device).cuda_stream)


def _ptr(t):
    return ctypes.c_void_p(t.data_ptr()) if t is not None else ctypes.c_void_p(0)


class _OutSet:
    """A copy=True output set (UsvVectorEnv._fresh_outputs): the tensors, their storage, ctypes
    pointers, the reference-state baseline, and whether a tensor of it was recorded on a stream."""
    __slots__ = ("ts", "tl", "st", "ptrs", "base", "exposed", "__weakref__")

    @classmethod
    def make(cls, n, d, dev, rdt, info_enabled):
        ent = cls()
        rb = torch.empty((), dtype=rdt).element_size()
        ob = n * d * 4
        info_b = n * _lib.INFO_DIM * rb if info_enabled else 0
        # byte layout: rewards and info rows first (8-B aligned), then obs, final obs, the flags
        sizes = (n * rb, info_b, ob, ob, 3 * n)
        buf = torch.empty(sum(sizes), dtype=torch.uint8, device=dev)
        rew_b, info_bytes, obs_b, fobs_b, flags = buf.split(sizes)
        term, trunc, done = flags.view(torch.bool).view(3, n).unbind(0)
        ent.ts = (obs_b.view(torch.float32).view(n, d), rew_b.view(rdt), term, trunc, done,
                  fobs_b.view(torch.float32).view(n, d),
                  info_bytes.view(rdt).view(n, _lib.INFO_DIM) if info_enabled else None)
        ent.tl = tuple(t for t in ent.ts if t is not None)
        ent.st = buf.untyped_storage()
        ent.ptrs = tuple(_ptr(t) for t in ent.ts)
        ent.base, ent.exposed = None, False
        _install_record_stream_hook()
        _RING_SETS[ent.st.data_ptr()] = ent            # (weak: the entry goes with the set)
        return ent

    def state(self, h0, h1, h2):
        """Reference counts of the set: the tuple, each tensor (less the env's own references, whose
        ids are h0..h2), each tensor's TensorImpl, the storage."""
        out = [sys.getrefcount(self.ts), _STORAGE_USE_COUNT(self.st._cdata)]
        for t in self.tl:
            i = id(t)
            out.append(sys.getrefcount(t) - (i == h0) - (i == h1) - (i == h2))
            out.append(t._use_count())
        return out

    def unchanged(self, h0, h1, h2):
        """state(h0, h1, h2) == base, stopping at the first difference."""
        b = self.base
        if sys.getrefcount(self.ts) != b[0] or _STORAGE_USE_COUNT(self.st._cdata) != b[1]:
            return False
        k = 2
        for t in self.tl:
            i = id(t)
            if sys.getrefcount(t) - (i == h0) - (i == h1) - (i == h2) != b[k] or t._use_count() != b[k + 1]:
                return False
            k += 2
        return True


# Storage address -> live copy=True output set.  Tensor.record_stream is wrapped once (the first time a
# set is made) so that recording any tensor or view of a set's storage on a stream retires that set from
# the ring; the original method then runs unchanged.  A class-level wrapper, not a per-tensor attribute:
# the outputs stay plain tensors (pickling, deepcopy and views behave as usual).
_RING_SETS = weakref.WeakValueDictionary()
_RECORD_STREAM = None


def _install_record_stream_hook():
    global _RECORD_STREAM
    if _RECORD_STREAM is not None:
        return
    orig = _RECORD_STREAM = torch.Tensor.record_stream

    def record_stream(self, stream):
        if _RING_SETS:
            ent = _RING_SETS.get(self.untyped_storage().data_ptr())
            if ent is not None:
                ent.exposed = True
        return orig(self, stream)
    record_stream.__doc__ = orig.__doc__
    torch.Tensor.record_stream = record_stream


class UsvVectorEnv:
    """``num_envs`` USV path-following envs on one GPU.

    reset(seed=None, options=None, mask=None) -> (obs [N,143] f32, info)
    step(actions [N,2] f32)  -> (obs, reward [N], terminated [N] bool, truncated [N] bool, info)

    ``copy=True`` (default, gymnasium's ``SyncVectorEnv(copy=True)`` convention): every call returns
    tensors of its own -- the kernel writes straight into freshly allocated device tensors, so this
    costs no extra copy.  ``copy=False``: the env's persistent device buffers are returned and the next
    call overwrites them (no allocation; for loops that consume each step before the next).
    ``info["final_obs"]`` holds the terminal obs rows of envs that ended this step
    (``info["_final_obs"]`` is the mask; rows where it is False are unspecified).
    """

    metadata = {"render_modes": [], "autoreset_mode": "same-step"}

    def __init__(self, env_id="usv-simple", num_envs=4096, device=0, seed=0, precision="f32",
                 autoreset=True, max_episode_steps=None, obstacle_cap=32, lidar="window",
                 env_id_offset=0, reset_rng="philox", options=None, info=False, perturb=False,
                 copy=True, kernel_variant=None, lib_path=None):
        """``options`` are UsvSimpleEnv's constructor options (simple_env.py:10): only
        ``run_custom_experiment`` / ``experiment`` (:292-300) exist there.  ``info=True`` returns the
        reference's per-step info keys (simple_env.py:102-115, 189-199) as device tensors.
        ``perturb=True`` runs usv-asmc-simple's UsvAsmc.compute with do_perturb (usv_asmc.py:184-199).
        ``kernel_variant="epb,lid,kind"`` selects a step-kernel variant (usv_set_kernel_variant; all
        variants give bit-identical outputs, the GPU tests compare them); None = the tuned default."""
        if env_id not in ENV_SPECS:
            raise ValueError(f"unknown env id {env_id!r}; known: {sorted(ENV_SPECS)}")
        if not torch.cuda.is_available():
            raise _lib.UsvLibError("UsvVectorEnv needs a ROCm GPU (torch.cuda.is_available() is False)")
        self.lib = _lib.load(lib_path)    # lib_path: another build of the C-ABI (e.g. _lib.SAFE_LIB_PATH)
        mode, limit = ENV_SPECS[env_id]
        self.env_id, self.num_envs = env_id, int(num_envs)
        self.device = torch.device("cuda", device)
        cfg = _lib.UsvConfig()
        self.lib.usv_config_default(ctypes.byref(cfg), mode, self.num_envs)
        cfg.precision = {"f32": _lib.F32, "f64": _lib.F64}[precision]
        cfg.obstacle_cap = obstacle_cap
        cfg.max_episode_steps = limit if max_episode_steps is None else int(max_episode_steps)
        cfg.autoreset = _lib.AUTORESET_SAME_STEP if autoreset else _lib.AUTORESET_DISABLED
        cfg.lidar_algo = {"brute": _lib.LIDAR_BRUTE, "window": _lib.LIDAR_WINDOW}[lidar]
        cfg.seed = int(seed)
        cfg.env_id_offset = int(env_id_offset)
        cfg.flags = _lib.FLAG_PERTURB if perturb else 0
        self.cfg = cfg
        h = ctypes.c_void_p()
        with torch.cuda.device(self.device):
            self._check(self.lib.usv_create(ctypes.byref(cfg), self.device.index, ctypes.byref(h)))
        self._h = h
        if kernel_variant is not None:
            epb, lid, kind = (int(v) for v in str(kernel_variant).split(","))
            self._check(self.lib.usv_set_kernel_variant(h, kind, epb, lid))
        n = self.num_envs
        self.obs_dim = self.lib.usv_obs_dim(h)
        self.act_dim = self.lib.usv_act_dim(h)
        rdt = torch.float32 if precision == "f32" else torch.float64
        self._rdt = rdt
        self.copy = bool(copy)
        kw = dict(device=self.device)
        self.obs = torch.zeros((n, self.obs_dim), dtype=torch.float32, **kw)
        self.final_obs = torch.zeros((n, self.obs_dim), dtype=torch.float32, **kw)
        self.reward = torch.zeros(n, dtype=rdt, **kw)
        self._term = torch.zeros(n, dtype=torch.uint8, **kw)
        self._trunc = torch.zeros(n, dtype=torch.uint8, **kw)
        self._done = torch.zeros(n, dtype=torch.uint8, **kw)   # terminated | truncated, written by the step kernel
        self.max_episode_steps = cfg.max_episode_steps
        self.single_observation_space, self.single_action_space = _spaces(env_id)
        self._fields = self._field_table()
        if reset_rng not in ("philox", "numpy"):
            raise ValueError("reset_rng must be 'philox' or 'numpy'")
        self.reset_rng = reset_rng
        self._np_seeded = False
        if reset_rng == "numpy":
            self._check(self.lib.usv_set_reset_rng(self._h, _lib.RESET_NUMPY_PCG64))
        self.info_enabled = bool(info) and env_id not in LEGACY_IDS   # the legacy ids return {}
        # info rows in the handle's precision (f64 build: float64 rows, like the reference's values)
        self.info_buf = torch.zeros((n, _lib.INFO_DIM), dtype=rdt, **kw) if self.info_enabled else None
        # step() hot path: the persistent buffers' pointers and bool views, made once
        self._out_ptrs = (_ptr(self.obs), _ptr(self.reward), _ptr(self._term), _ptr(self._trunc),
                          _ptr(self._done), _ptr(self.final_obs), _ptr(self.info_buf))
        self._term_b, self._trunc_b = self._term.view(torch.bool), self._trunc.view(torch.bool)
        self._done_b = self._done.view(torch.bool)
        self._last_obs = self.obs              # the latest obs rows (a masked reset keeps the others)
        self._last_rew = self.reward
        self.options = dict(options or {})
        # the reference reads only these keys and ignores any other (simple_env.py:292)
        unknown = set(self.options) - {"run_custom_experiment", "experiment"}
        if unknown:
            warnings.warn(f"constructor options {sorted(unknown)} are ignored (UsvSimpleEnv reads only "
                          "'run_custom_experiment' and 'experiment', simple_env.py:292-300)", stacklevel=2)
        if self.options.get("run_custom_experiment"):
            if env_id != "usv-simple":
                raise ValueError("run_custom_experiment exists for usv-simple only (UsvSimpleASMCEnv.__init__ "
                                 "takes no options, simple_env_asmc.py:10)")
            self.set_experiment(self.options["experiment"])

    def _check(self, rc):
        return _lib.check(rc, self.lib)

    def set_experiment(self, exp):
        """Install a custom experiment (simple_env.py:292-300) for every env: each reset keeps its
        draws but takes obstacles, path and pose from ``exp`` (keys obstacle_positions [n,2],
        obstacle_radius [n], path_start [2], angle, position [3]); ``None`` removes it."""
        if exp is None:
            self._check(self.lib.usv_set_experiment(self._h, None))
            return
        x = _lib.UsvExperiment()
        pos = np.asarray(exp["obstacle_positions"], dtype=np.float64).reshape(-1, 2)
        rad = np.asarray(exp["obstacle_radius"], dtype=np.float64).reshape(-1)
        if pos.shape[0] != rad.shape[0] or not 1 <= pos.shape[0] <= min(self.cfg.obstacle_cap, _lib.EXP_MAX_OBS):
            raise ValueError(f"experiment needs 1..{self.cfg.obstacle_cap} obstacles with one radius each")
        x.n_obs = pos.shape[0]
        for j in range(x.n_obs):
            x.obstacle_x[j], x.obstacle_y[j], x.obstacle_r[j] = pos[j, 0], pos[j, 1], rad[j]
        ps = np.asarray(exp["path_start"], dtype=np.float64).reshape(2)
        x.path_start[0], x.path_start[1] = ps
        x.angle = float(exp["angle"])
        p3 = np.asarray(exp["position"], dtype=np.float64).reshape(3)
        x.position[0], x.position[1], x.position[2] = p3
        self._check(self.lib.usv_set_experiment(self._h, ctypes.byref(x)))

    def _info_dict(self, b, reward=None, reset=False, mask=None):
        """The reference's info keys as device tensors (views of the info rows ``b``).  After a reset
        the reward is -1 (_get_info(-1, ...), simple_env.py:305) in the rows of the reset envs; rows of
        envs a masked reset left alone keep their last values."""
        n = self.num_envs
        if reset:
            rew = torch.full((n,), -1.0, dtype=self._rdt, device=self.device)
            if mask is not None:
                rew = torch.where(mask, rew, self._last_rew)
        else:
            rew = reward
        col = {k: i for i, k in enumerate(_lib.INFO_KEYS)}
        z = torch.zeros(n, dtype=self._rdt, device=self.device)
        d = {"position": b[:, 0:3], "velocity": b[:, 3:6], "path_start": b[:, 6:8], "path_end": b[:, 8:10],
             "reward": rew, "action0": b[:, col["action0"]], "action1": b[:, col["action1"]],
             "left_thruster": z, "right_thruster": z,
             "ye": b[:, col["ye"]], "angle_to_target": b[:, col["angle_to_target"]]}
        if not reset:
            for k in ("ye_reward", "angle_to_target_reward", "delta_action_reward", "delta_action",
                      "velocity_track_reward", "reference_velocity", "reward_velocity", "reference_velocity_error"):
                d[k] = b[:, col[k]]
            d["angle_action_reward"] = z
        return d

    # ------------------------------------------------------------------ API
    def reset(self, seed=None, options=None, mask=None):
        """UsvSimpleEnv.reset (simple_env.py:228-308) for every env (or those where ``mask``);
        ``options={'place_obstacles_on_path': k}`` (:276-288) needs ``obstacle_cap >= 29 + k``.
        Other option keys are ignored, as the reference ignores them; UsvSimpleASMCEnv.reset drops its
        options altogether (simple_env_asmc.py:14-16: super().reset(seed=seed))."""
        ropt = _lib.UsvResetOptions()
        if self.env_id == "usv-simple" and options:
            ropt.place_obstacles_on_path = int(dict(options).get("place_obstacles_on_path") or 0)
        if self.reset_rng == "numpy":
            # each env owns a numpy Generator(PCG64(SeedSequence(seed_i))), like gymnasium's
            # Env.reset(seed) (simple_env.py:229); an int seed gives env i seed + global id (the
            # make_vec_env / DummyVecEnv convention), a sequence gives one seed per env
            if seed is None and not self._np_seeded:
                seed = int(self.cfg.seed)
            if seed is not None:
                if np.ndim(seed) == 0:
                    seeds = int(seed) + int(self.cfg.env_id_offset) + np.arange(self.num_envs)
                else:
                    seeds = np.asarray(seed, dtype=np.int64).reshape(self.num_envs)
                if self.env_id in LEGACY_IDS:      # np.random.seed(seed_i) (usv_asmc_env.py:258)
                    self.set_field("np_mt", np_mt_words(seeds))
                else:
                    self.set_field("np_rng", np_rng_words(seeds))
                self._np_seeded = True
        elif seed is not None:
            self._check(self.lib.usv_seed(self._h, ctypes.c_uint64(int(seed))))
        m = None
        if mask is not None:
            m = torch.as_tensor(mask, device=self.device).to(torch.uint8).contiguous()
        # rows of envs that are not reset keep the latest obs (and info) rows; a full reset rewrites
        # every row, so with copy=True it only needs fresh tensors
        obs, ib = self._last_obs, self.info_buf
        if self.copy:
            fresh = torch.empty_like if m is None else torch.clone
            obs = fresh(obs)
            if self.info_enabled:
                ib = fresh(ib)
        self._check(self.lib.usv_reset_ex(self._h, _ptr(m), _ptr(obs), ctypes.byref(ropt),
                                         _ptr(ib), _stream_ptr(self.device)))
        self._last_obs = obs
        if not self.info_enabled:
            return obs, {}
        self.info_buf = ib
        return obs, self._info_dict(ib, reset=True, mask=None if m is None else m.bool())

    def step(self, actions):
        if isinstance(actions, torch.Tensor) and actions.device == self.device:
            a = actions
        else:
            a = torch.as_tensor(actions, device=self.device)
        if a.dtype != torch.float32 or not a.is_contiguous():
            a = a.to(torch.float32).contiguous()
        if self.act_dim == 1 and a.shape == (self.num_envs,):
            a = a.reshape(self.num_envs, 1)
        if a.shape != (self.num_envs, self.act_dim):
            raise ValueError(f"actions must be [{self.num_envs}, {self.act_dim}], got {tuple(a.shape)}")
        if self.copy:
            # fresh outputs: tensors no one else references (the kernel writes every row of obs /
            # reward / flags and of the info rows, so they need no copy)
            (obs, rew, term, trunc, done, fobs, ib), ptrs = self._fresh_outputs()
        else:
            obs, rew, fobs, ib = self.obs, self.reward, self.final_obs, self.info_buf
            term, trunc, done = self._term_b, self._trunc_b, self._done_b
            ptrs = self._out_ptrs
        o, r, te, tr, dn, fo, inf = ptrs
        # the kernel also writes the done mask (terminated | truncated): no extra launch per step
        self._check(self.lib.usv_step_ex(self._h, ctypes.c_void_p(a.data_ptr()), o, r, te, tr, dn, fo, inf,
                                        _stream_ptr(self.device)))
        self._last_obs, self._last_rew = obs, rew
        info = {"final_obs": fobs, "_final_obs": done}
        if self.info_enabled:
            self.info_buf = ib
            info.update(self._info_dict(ib, rew))
        return obs, rew, term, trunc, info

    _RING = 3

    def _fresh_outputs(self):
        """One output set of a copy=True step: (obs, reward, terminated, truncated, done, final_obs,
        info rows) and their ctypes pointers.  A set is one device allocation viewed as the outputs;
        a set returned earlier is handed out again only when nothing outside this env can still read
        it, i.e. its reference state is back at the baseline taken when it was made (_OutSet.state):
          * no Python reference to the tuple or to one of its tensors (sys.getrefcount, read by the
            same code at creation and at reuse, so the interpreter's own counting cancels out);
          * no other view of the storage (the storage use count);
          * no C++ holder of a tensor (TensorImpl use count: a DLPack capsule, an autograd graph);
          * no other stream recorded on it: ``record_stream`` on a handed-out tensor (or a view) retires its
            set from the ring for good, so the caching allocator frees it only after that stream's
            work, exactly as for any tensor it owns.
        Otherwise a new set is allocated: the caller always gets tensors that alias nothing it holds
        or still reads (gymnasium's copy=True), at the cost of a few reference-count reads instead of
        an allocation and seven views per step."""
        ring = self.__dict__.setdefault("_out_ring", [])
        if _STORAGE_USE_COUNT is not None:
            # the env's own references to the last step's outputs (reset(mask=) keeps the rows of the
            # envs it does not reset) are not the caller's: ids, so that reading them adds none
            d = self.__dict__
            h0, h1, h2 = id(d.get("_last_obs")), id(d.get("_last_rew")), id(d.get("info_buf"))
            for ent in ring:
                if not ent.exposed and ent.unchanged(h0, h1, h2):
                    return ent.ts, ent.ptrs
        ent = _OutSet.make(self.num_envs, self.obs_dim, self.device, self._rdt, self.info_enabled)
        if len(ring) >= self._RING:
            ring.pop(0)                                # (still the caller's if it holds it)
        ring.append(ent)
        ring[:] = [e for e in ring if not e.exposed]   # retired sets: the allocator's from now on
        if _STORAGE_USE_COUNT is not None:
            ent.base = ent.state(0, 0, 0)
        return ent.ts, ent.ptrs

    def step_raw(self, actions, obs, reward, term, trunc, final_obs=None, stream=None):
        """Launch one step into caller-owned buffers (no checks, no allocation): bench / graphs."""
        st = ctypes.c_void_p(stream) if stream is not None else _stream_ptr(self.device)
        return self.lib.usv_step(self._h, _ptr(actions), _ptr(obs), _ptr(reward), _ptr(term),
                                 _ptr(trunc), _ptr(final_obs), st)

    # ------------------------------------------------------------------ state exchange
    def _field_table(self):
        tab = {}
        per, isint, name = ctypes.c_int32(), ctypes.c_int32(), ctypes.c_char_p()
        for f in range(64):
            if self.lib.usv_field_info(self._h, f, ctypes.byref(per), ctypes.byref(isint),
                                       ctypes.byref(name)) != 0:
                break
            tab[name.value.decode()] = (f, per.value, bool(isint.value))
        return tab

    @property
    def field_names(self):
        return list(self._fields)

    def get_field(self, name):
        f, per, isint = self._fields[name]
        shape = (self.num_envs,) if per == 1 else (self.num_envs, per)
        out = np.zeros(shape, dtype=np.int32 if isint else np.float64)
        self._check(self.lib.usv_get_field(self._h, f, out.ctypes.data_as(ctypes.c_void_p), out.nbytes))
        return out

    def set_field(self, name, value):
        f, per, isint = self._fields[name]
        shape = (self.num_envs,) if per == 1 else (self.num_envs, per)
        arr = np.ascontiguousarray(np.broadcast_to(np.asarray(value), shape),
                                   dtype=np.int32 if isint else np.float64)
        self._check(self.lib.usv_set_field(self._h, f, arr.ctypes.data_as(ctypes.c_void_p), arr.nbytes))

    def render(self, i=0, window_size=512):
        """rgb_array frame of env i (uint8 [H, W, 3]; gym_usv_amd.render, host-side), for
        VecVideoRecorder.  usv-simple / usv-asmc-simple only."""
        from .render import frame_from_state
        if self.env_id not in ("usv-simple", "usv-asmc-simple"):
            raise NotImplementedError("the legacy ids' renderer (gym's classic_control viewer) is out of scope")
        names = ("x", "y", "psi", "path_x0", "path_y0", "path_x1", "path_y1", "progress", "n_obs",
                 "obs_x", "obs_y", "obs_r")
        f = {k: self.get_field(k) for k in names}
        return frame_from_state(f, i, self._last_obs[i].detach().cpu().numpy(), window_size)

    def get_state(self):
        """All per-env state as {field: ndarray} (env checkpoint / parity inspection)."""
        return {k: self.get_field(k) for k in self._fields}

    def set_state(self, state):
        for k, v in state.items():
            self.set_field(k, v)

    def state_blob(self):
        n = self.lib.usv_state_bytes(self._h)
        buf = np.zeros(n, dtype=np.uint8)
        self._check(self.lib.usv_get_state(self._h, buf.ctypes.data_as(ctypes.c_void_p), n))
        return buf

    def load_state_blob(self, blob):
        blob = np.ascontiguousarray(blob, dtype=np.uint8)
        self._check(self.lib.usv_set_state(self._h, blob.ctypes.data_as(ctypes.c_void_p), blob.nbytes))

    def close(self):
        if getattr(self, "_h", None):
            torch.cuda.synchronize(self.device)
            self.lib.usv_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
