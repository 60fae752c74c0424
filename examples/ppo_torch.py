"""Torch-native PPO on the HIP vector env: config C5 without stable-baselines3.

The reference trains SB3 PPO on ``VecFrameStack(make_vec_env("usv-simple", n_envs), 5)`` with
``config_ppo`` (train_test/sb3_train_vec.py:67-81, train_test/config.py:3-15).  SB3 is absent from
this image, so this is a compact PPO with the same hyper-parameters where they carry over:

* policy / value: separate MLPs, ``net_arch=dict(pi=[256, 256], vf=[256, 256])``, ReLU,
  ``ortho_init=False`` (torch default init), Gaussian policy with ``log_std_init=-2``;
* SB3 PPO defaults for the rest: lr 3e-4, gamma 0.99, GAE lambda 0.95, clip 0.2, 10 epochs,
  vf_coef 0.5, ent_coef 0, max_grad_norm 0.5, advantage normalisation, Box-action clipping;
* TimeLimit truncation bootstrapped from the terminal observation's value (SB3 does the same with
  ``infos[i]["terminal_observation"]``); VecFrameStack(5) via ``DeviceFrameStack``.

Not reproduced: gSDE (``use_sde``/``sde_sample_freq``, a state-dependent exploration noise of
SB3's) -- this policy uses a state-independent log-std.  Parity with SB3 itself is unpinned (SB3
is not installed): the test checks finite losses, episode statistics and throughput only.

Everything stays on the device: observations, actions, rewards and dones are the env's HBM
tensors; the only host sync per update is the loss/statistics read-back.

    python examples/ppo_torch.py --envs 4096 --updates 50
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for _p in (ROOT, os.path.join(ROOT, "gym-usv_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

import torch  # noqa: E402
import torch.nn as nn  # noqa: E402

CONFIG_PPO = {"n_stack": 5, "hidden": (256, 256), "log_std_init": -2.0, "lr": 3e-4, "gamma": 0.99,
              "gae_lambda": 0.95, "clip": 0.2, "n_epochs": 10, "vf_coef": 0.5, "ent_coef": 0.0,
              "max_grad_norm": 0.5}


def mlp(inp, hidden, out):
    layers, d = [], inp
    for h in hidden:
        layers += [nn.Linear(d, h), nn.ReLU()]
        d = h
    layers.append(nn.Linear(d, out))
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    def __init__(self, obs_dim, act_dim, hidden, log_std_init):
        super().__init__()
        self.pi = mlp(obs_dim, hidden, act_dim)
        self.vf = mlp(obs_dim, hidden, 1)
        self.log_std = nn.Parameter(torch.full((act_dim,), float(log_std_init)))

    def dist(self, obs):
        return torch.distributions.Normal(self.pi(obs), self.log_std.exp())

    def value(self, obs):
        return self.vf(obs).squeeze(-1)


class PPO:
    """Rollout + update over a ``UsvVectorEnv`` (any registered id with a Box action space)."""

    def __init__(self, env, n_steps=16, batch_size=4096, seed=0, **cfg):
        from gym_usv_amd.sb3 import DeviceFrameStack
        self.cfg = dict(CONFIG_PPO, **cfg)
        self.env, self.n_steps, self.batch_size = env, n_steps, batch_size
        self.device = env.device
        self.N, D, A = env.num_envs, env.obs_dim, env.act_dim
        self.stack = DeviceFrameStack(self.N, D, self.cfg["n_stack"], self.device)
        torch.manual_seed(seed)
        self.model = ActorCritic(D * self.cfg["n_stack"], A, self.cfg["hidden"], self.cfg["log_std_init"]).to(self.device)
        self.opt = torch.optim.Adam(self.model.parameters(), lr=self.cfg["lr"])
        lo, hi = env.single_action_space.low, env.single_action_space.high
        self.a_lo = torch.as_tensor(lo, device=self.device, dtype=torch.float32)
        self.a_hi = torch.as_tensor(hi, device=self.device, dtype=torch.float32)
        obs, _ = env.reset(seed=seed)
        self.obs = self.stack.reset(obs).clone()
        T, N = n_steps, self.N
        z = lambda *s: torch.zeros(s, device=self.device)   # noqa: E731
        self.b_obs = z(T, N, D * self.cfg["n_stack"])
        self.b_act, self.b_logp, self.b_val = z(T, N, A), z(T, N), z(T, N)
        self.b_rew, self.b_done = z(T, N), z(T, N)
        self.ep_ret, self.ep_len = z(N), z(N)
        self.finished = []                              # (return, length) of completed episodes
        self.env_steps = 0

    @torch.no_grad()
    def rollout(self):
        g = self.cfg["gamma"]
        for t in range(self.n_steps):
            dist = self.model.dist(self.obs)
            a = dist.sample()
            self.b_obs[t] = self.obs
            self.b_act[t] = a
            self.b_logp[t] = dist.log_prob(a).sum(-1)
            self.b_val[t] = self.model.value(self.obs)
            a_env = torch.max(torch.min(a, self.a_hi), self.a_lo)          # SB3 clips Box actions
            obs, rew, term, trunc, info = self.env.step(a_env)
            done = term | trunc
            nxt, term_rows = self.stack.step(obs, done, info["final_obs"])
            r = rew.float().clone()
            if bool(trunc.any()):                       # bootstrap time-limit truncations
                idx = done.nonzero().flatten()
                tr = trunc[idx]
                if bool(tr.any()):
                    r[idx[tr]] += g * self.model.value(term_rows[tr])
            self.b_rew[t] = r
            self.b_done[t] = done.float()
            self.ep_ret += rew.float()
            self.ep_len += 1
            if bool(done.any()):
                d = done.nonzero().flatten()
                self.finished.append(torch.stack((self.ep_ret[d], self.ep_len[d]), 1))
                self.ep_ret[d] = 0
                self.ep_len[d] = 0
            self.obs = nxt.clone()
            self.env_steps += self.N

    def advantages(self):
        g, lam = self.cfg["gamma"], self.cfg["gae_lambda"]
        with torch.no_grad():
            last_v = self.model.value(self.obs)
        adv = torch.zeros_like(self.b_rew)
        gae = torch.zeros(self.N, device=self.device)
        for t in reversed(range(self.n_steps)):
            nv = last_v if t == self.n_steps - 1 else self.b_val[t + 1]
            nonterm = 1.0 - self.b_done[t]
            delta = self.b_rew[t] + g * nv * nonterm - self.b_val[t]
            gae = delta + g * lam * nonterm * gae
            adv[t] = gae
        return adv, adv + self.b_val

    def update(self):
        c = self.cfg
        adv, ret = self.advantages()
        M = self.n_steps * self.N
        obs = self.b_obs.reshape(M, -1)
        act = self.b_act.reshape(M, -1)
        logp0, adv, ret = self.b_logp.reshape(M), adv.reshape(M), ret.reshape(M)
        stats = []
        for _ in range(c["n_epochs"]):
            perm = torch.randperm(M, device=self.device)
            for k in range(0, M, self.batch_size):
                i = perm[k:k + self.batch_size]
                a_ = adv[i]
                a_ = (a_ - a_.mean()) / (a_.std() + 1e-8)
                dist = self.model.dist(obs[i])
                logp = dist.log_prob(act[i]).sum(-1)
                ratio = (logp - logp0[i]).exp()
                pg = -torch.min(ratio * a_, ratio.clamp(1 - c["clip"], 1 + c["clip"]) * a_).mean()
                vl = ((self.model.value(obs[i]) - ret[i]) ** 2).mean()
                ent = dist.entropy().sum(-1).mean()
                loss = pg + c["vf_coef"] * vl - c["ent_coef"] * ent
                self.opt.zero_grad(set_to_none=True)
                loss.backward()
                nn.utils.clip_grad_norm_(self.model.parameters(), c["max_grad_norm"])
                self.opt.step()
                stats.append(torch.stack((pg.detach(), vl.detach(), ent.detach())))
        s = torch.stack(stats).mean(0).tolist()
        return {"policy_loss": s[0], "value_loss": s[1], "entropy": s[2]}

    def episode_stats(self):
        if not self.finished:
            return {"episodes": 0}
        f = torch.cat(self.finished)
        self.finished = []
        return {"episodes": int(f.shape[0]), "ep_rew_mean": float(f[:, 0].mean()), "ep_len_mean": float(f[:, 1].mean())}


def train(env_id="usv-simple", envs=4096, updates=10, n_steps=16, batch_size=4096, seed=0, log=print):
    import gym_usv_amd
    env = gym_usv_amd.make_vec(env_id, envs, seed=seed, copy=False)   # each step is consumed at once
    ppo = PPO(env, n_steps=n_steps, batch_size=batch_size, seed=seed)
    hist = []
    t0 = time.perf_counter()
    for u in range(updates):
        ppo.rollout()
        rec = {"update": u + 1, **ppo.update(), **ppo.episode_stats(), "env_steps": ppo.env_steps}
        torch.cuda.synchronize()
        rec["wall_s"] = round(time.perf_counter() - t0, 3)
        hist.append(rec)
        log(json.dumps(rec))
    env.close()
    return hist


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env-id", default="usv-simple")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--updates", type=int, default=50)
    ap.add_argument("--n-steps", type=int, default=16)
    ap.add_argument("--batch-size", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=0)
    a = ap.parse_args()
    train(a.env_id, a.envs, a.updates, a.n_steps, a.batch_size, a.seed)


if __name__ == "__main__":
    main()
