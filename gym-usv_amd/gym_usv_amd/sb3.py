"""Stable-Baselines3 integration: a ``VecEnv`` over the HIP vector env.

The reference trains with::

    env = make_vec_env(env_id, n_envs=4, vec_env_cls=DummyVecEnv)     # sb3_train_vec.py:67
    env = VecVideoRecorder(env, ...)                                   # :68-69
    env = VecFrameStack(env, 5)                                        # :70

i.e. N Python envs stepped one by one, each wrapped in ``Monitor`` (episode stats) and
``TimeLimit`` (gym_usv/__init__.py:27,33), with DummyVecEnv's same-step autoreset.  The
counterpart here is one object::

    from gym_usv_amd.sb3 import Sb3VecEnv
    env = Sb3VecEnv("usv-simple", num_envs=4096, frame_stack=5)

It duck-types ``stable_baselines3.common.vec_env.VecEnv`` (SB3 itself is not importable in this
image, so it is not subclassed; ``as_sb3()`` subclasses it where SB3 is installed).  Semantics
restated from SB3 2.x:

* ``step_wait`` -> (obs ndarray, rewards float32 ndarray, dones bool ndarray, infos list);
* a done env's info holds ``terminal_observation`` (the final obs; frame-stacked when stacking)
  and ``TimeLimit.truncated`` (truncated and not terminated), as DummyVecEnv + TimeLimit do;
* ``episode = {"r", "l", "t"}`` in the info of a done env, as ``Monitor`` writes it;
* ``frame_stack=k`` is ``VecFrameStack(k)`` (channels-last: the newest obs is the last block,
  a done env's stack is zeroed before the reset obs is pushed), computed on the device.

The step itself stays on the GPU; only the arrays SB3 consumes are copied to the host, into
page-locked buffers: the stacked obs on a copy stream while the host builds the done envs' infos,
the small arrays (reward, done) first, and the terminal rows of the done envs only.  The returned
arrays alternate between two such buffer sets, so each stays valid until the second-next step
(SB3's collectors consume or copy them within one step).  ``infos`` is a new list every step; a done
env's info is a new dict; an env that did not end gets an empty dict that is reused across steps
only while it stays empty: a dict a wrapper or callback wrote into BEFORE the next ``step_wait`` is
replaced by a new one there (one C-level ``any()`` over the list detects it), so such a write never
shows up in a later step's infos, without building 4096 dicts per step (~0.1-0.2 ms of Python).
A write into step t's empty dict made AFTER step t+1 has returned (a consumer that keeps infos lists
and annotates them later) does show up in step t+1's infos, which DummyVecEnv's fresh dicts never
do: pass ``fresh_infos=True`` for a new dict per env and step, as DummyVecEnv builds them.
The env's device is the current device for the whole call (events and copies are ordered on its
stream even when another device is current in the caller).
"""
from __future__ import annotations

import time

import numpy as np
import torch

from .spaces import Box


class DeviceFrameStack:
    """``VecFrameStack`` on device tensors (SB3 ``StackedObservations``, channels-last 1-D obs).

    ``buf`` is [N, k*D]; two buffers alternate so the shift is one out-of-place copy."""

    def __init__(self, num_envs, obs_dim, n_stack, device, dtype=torch.float32):
        self.n, self.d, self.k = num_envs, obs_dim, n_stack
        self._bufs = [torch.zeros((num_envs, n_stack * obs_dim), device=device, dtype=dtype) for _ in range(2)]
        self._i = 0

    @property
    def buf(self):
        return self._bufs[self._i]

    def reset(self, obs):
        b = self.buf
        b.zero_()
        b[:, -self.d:] = obs
        return b

    def step(self, obs, done, final_obs=None):
        """Push `obs`; returns (stacked obs, stacked terminal obs rows of done envs or None)."""
        old, new = self._bufs[self._i], self._bufs[1 - self._i]
        d = self.d
        new[:, :-d] = old[:, d:]                       # np.roll(stacked, -D, axis=-1)
        term = None
        if final_obs is not None and bool(done.any()):
            idx = done.nonzero().flatten()
            term = torch.cat((new[idx, :-d], final_obs[idx]), dim=1)
            new[idx] = 0
        elif bool(done.any()):
            new[done] = 0
        new[:, -d:] = obs
        self._i = 1 - self._i
        return new, term


def _to_gym_box(box):
    """The env's Box as a gymnasium Box when gymnasium is importable (SB3 checks spaces)."""
    try:
        import gymnasium
        return gymnasium.spaces.Box(low=box.low, high=box.high, shape=box.shape, dtype=box.dtype)
    except Exception:
        return box


class Sb3VecEnv:
    """SB3 ``VecEnv`` of ``num_envs`` HIP-stepped USV envs (+ Monitor, TimeLimit, VecFrameStack).

    ``venv`` may be passed instead of ``env_id`` (anything with the ``UsvVectorEnv`` surface:
    ``num_envs``, ``obs_dim``, ``act_dim``, ``single_*_space``, ``reset(seed=)``, ``step()`` with
    same-step autoreset and ``info["final_obs"]``)."""

    def __init__(self, env_id="usv-simple", num_envs=4096, frame_stack=0, seed=0, venv=None,
                 fresh_infos=False, **kw):
        if venv is None:
            from .vector_env import UsvVectorEnv
            # each step is consumed (copied to the host) before the next: the persistent buffers do
            kw.setdefault("copy", False)
            venv = UsvVectorEnv(env_id, num_envs=num_envs, seed=seed, autoreset=True, **kw)
        self.venv = venv
        self.num_envs = venv.num_envs
        self.render_mode = "rgb_array"               # VecVideoRecorder: env 0 (render.py)
        d = venv.obs_dim
        self._stack = DeviceFrameStack(self.num_envs, d, frame_stack, venv.device) if frame_stack else None
        obs_space = venv.single_observation_space
        if frame_stack:
            obs_space = Box(np.tile(obs_space.low, frame_stack), np.tile(obs_space.high, frame_stack),
                            dtype=np.float32)
        self.observation_space = _to_gym_box(obs_space)
        self.action_space = _to_gym_box(venv.single_action_space)
        self._seed = seed
        self._actions = None
        dev = venv.device
        n = self.num_envs
        self._ep_ret = torch.zeros(n, dtype=torch.float64, device=dev)
        self._ep_len = torch.zeros(n, dtype=torch.int64, device=dev)
        self._t0 = time.time()
        # host side: page-locked buffers (two sets, alternating) and a copy stream on a GPU
        self._cuda = dev.type == "cuda"
        pin = self._cuda
        w = d * (frame_stack or 1)
        self._host = [dict(obs=torch.empty((n, w), dtype=torch.float32, pin_memory=pin),
                           rew=torch.empty(n, dtype=torch.float32, pin_memory=pin),
                           done=torch.empty(n, dtype=torch.bool, pin_memory=pin)) for _ in range(2)]
        self._hb = 0
        self._act_host = torch.empty((n, venv.act_dim), dtype=torch.float32, pin_memory=pin)
        self._act_dev = torch.empty((n, venv.act_dim), dtype=torch.float32, device=dev)
        self._rew32 = torch.empty(n, dtype=torch.float32, device=dev)
        self._copy_stream = torch.cuda.Stream(dev) if self._cuda else None
        self._fresh_infos = bool(fresh_infos)
        self._infos = [{} for _ in range(n)]            # per env: empty unless it ended this step
        self._filled = np.empty(0, dtype=np.int64)

    # ---------------------------------------------------------------- VecEnv API
    def reset(self):
        obs, _ = self.venv.reset(seed=self._seed)
        self._seed = None                              # SB3: the seed applies to the next reset only
        self._ep_ret.zero_()
        self._ep_len.zero_()
        if self._stack is not None:
            obs = self._stack.reset(obs)
        return obs.cpu().numpy()

    def step_async(self, actions):
        self._actions = actions

    def step_wait(self):
        if self._cuda:
            with torch.cuda.device(self.venv.device):
                return self._step_wait()
        return self._step_wait()

    def _step_wait(self):
        venv, n, dev = self.venv, self.num_envs, self.venv.device
        np.copyto(self._act_host.numpy(), np.asarray(self._actions, dtype=np.float32).reshape(n, -1))
        self._act_dev.copy_(self._act_host, non_blocking=self._cuda)
        obs, rew, term, trunc, info = venv.step(self._act_dev)
        done = info["_final_obs"]                       # terminated | truncated, written by the step kernel
        final = info.get("final_obs")
        self._ep_ret += rew
        self._ep_len += 1
        st = self._stack
        old = None
        if st is not None:
            # VecFrameStack: roll by one obs, zero the done envs' stacks, push the new obs; `old` keeps
            # the previous stacks for the done envs' terminal observations below
            old, new, d = st.buf, st._bufs[1 - st._i], st.d
            torch.mul(old[:, d:], (~done)[:, None], out=new[:, :-d])
            new[:, -d:] = obs
            st._i = 1 - st._i
            obs = new
        h = self._host[self._hb]
        self._hb ^= 1
        if self._cuda:
            # the stacked obs (the big copy) on the copy stream, overlapping the rest of this call
            main = torch.cuda.current_stream(dev)
            ready = torch.cuda.Event()
            ready.record(main)
            cs = self._copy_stream
            cs.wait_event(ready)
            with torch.cuda.stream(cs):
                h["obs"].copy_(obs, non_blocking=True)
                obs_done = torch.cuda.Event()
                obs_done.record(cs)
            obs.record_stream(cs)
            self._rew32.copy_(rew)
            h["rew"].copy_(self._rew32, non_blocking=True)
            h["done"].copy_(done, non_blocking=True)
            small = torch.cuda.Event()
            small.record(main)
            small.synchronize()
        else:
            h["obs"].copy_(obs)
            h["rew"].copy_(rew)
            h["done"].copy_(done)
        if self._fresh_infos:                           # DummyVecEnv: a new dict per env and step
            infos = self._infos = [{} for _ in range(n)]
        else:
            infos = self._infos
            for i in self._filled:                      # last step's done envs: new empty dicts
                infos[i] = {}
            if any(infos):                              # a consumer wrote into an empty info dict:
                for i, d in enumerate(infos):           # replace it (theirs keeps the write)
                    if d:
                        infos[i] = {}
        done_np = h["done"].numpy()
        idx = np.flatnonzero(done_np)
        if idx.size:
            ti = torch.from_numpy(idx).to(dev)
            rows = final[ti] if old is None else torch.cat((old[ti, st.d:], final[ti]), dim=1)
            w = rows.shape[1]
            # one device->host copy: terminal rows, TimeLimit.truncated, episode return and length
            pack = torch.cat((rows.to(torch.float64), (trunc & ~term)[ti, None].to(torch.float64),
                              self._ep_ret[ti, None], self._ep_len[ti, None].to(torch.float64)), dim=1).cpu().numpy()
            self._ep_ret[ti] = 0
            self._ep_len[ti] = 0
            t = round(time.time() - self._t0, 6)
            term_obs = pack[:, :w].astype(np.float32)
            for j, i in enumerate(idx):
                infos[i] = {"terminal_observation": term_obs[j], "TimeLimit.truncated": bool(pack[j, w]),
                                  "episode": {"r": round(float(pack[j, w + 1]), 6), "l": int(pack[j, w + 2]), "t": t}}
        self._filled = idx
        if self._cuda:
            obs_done.synchronize()
        return h["obs"].numpy(), h["rew"].numpy(), done_np, list(infos)

    def step(self, actions):
        self.step_async(actions)
        return self.step_wait()

    def close(self):
        self.venv.close()

    def seed(self, seed=None):
        self._seed = seed
        return [seed] * self.num_envs

    def get_attr(self, attr_name, indices=None):
        val = getattr(self.venv, attr_name)
        return [val] * len(self._indices(indices))

    def set_attr(self, attr_name, value, indices=None):
        setattr(self.venv, attr_name, value)

    def env_method(self, method_name, *args, indices=None, **kwargs):
        raise NotImplementedError("per-env methods: the envs are one batched GPU object")

    def env_is_wrapped(self, wrapper_class, indices=None):
        return [False] * len(self._indices(indices))

    def get_images(self):
        """One rgb_array frame per env would copy every env's state off the GPU; like
        VecVideoRecorder needs, this returns env 0's frame (gym_usv_amd.render)."""
        return [self.venv.render(0)]

    def render(self, mode=None):
        return self.venv.render(0)

    def _indices(self, indices):
        if indices is None:
            return range(self.num_envs)
        if isinstance(indices, int):
            return [indices]
        return indices

    # ---------------------------------------------------------------- SB3 proper
    def as_sb3(self):
        """A real ``stable_baselines3`` VecEnv subclass instance wrapping this one (SB3 needed)."""
        from stable_baselines3.common.vec_env import VecEnv

        outer = self

        class _Sb3(VecEnv):
            def __init__(self):
                super().__init__(outer.num_envs, outer.observation_space, outer.action_space)

            def reset(self):
                return outer.reset()

            def step_async(self, actions):
                outer.step_async(actions)

            def step_wait(self):
                return outer.step_wait()

            def close(self):
                outer.close()

            def get_attr(self, attr_name, indices=None):
                return outer.get_attr(attr_name, indices)

            def set_attr(self, attr_name, value, indices=None):
                outer.set_attr(attr_name, value, indices)

            def env_method(self, method_name, *method_args, indices=None, **method_kwargs):
                return outer.env_method(method_name, *method_args, indices=indices, **method_kwargs)

            def env_is_wrapped(self, wrapper_class, indices=None):
                return outer.env_is_wrapped(wrapper_class, indices)

        return _Sb3()
