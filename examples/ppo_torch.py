"""Torch-native PPO with gSDE on the HIP vector env: config C5 without stable-baselines3.

The reference trains SB3 PPO on ``VecFrameStack(make_vec_env("usv-simple", n_envs), 5)`` with
``config_ppo`` (train_test/sb3_train_vec.py:67-81, train_test/config.py:3-15).  SB3 is absent from
this image, so this is a compact PPO with the same hyper-parameters where they carry over:

* policy / value: separate MLPs, ``net_arch=dict(pi=[256, 256], vf=[256, 256])``, ReLU,
  ``ortho_init=False`` (torch default init);
* gSDE (``use_sde=True``, ``sde_sample_freq=4``, ``log_std_init=-2``), as SB3's
  ``StateDependentNoiseDistribution`` (full_std, no expln, latent not learned through the noise):
  a per-env exploration matrix W ~ N(0, exp(log_std)^2) of shape [256, act_dim] is drawn at the
  start of every rollout and every 4 steps; the action is mean(s) + latent(s) @ W, where latent(s)
  is the policy's last hidden layer (detached); its log-probability is under
  N(mean(s), sqrt(latent(s)^2 @ exp(log_std)^2 + 1e-6)).  SB3 reports no entropy for gSDE and uses
  -mean(log_prob) in its place; with ent_coef 0 it does not enter the loss;
* SB3 PPO defaults for the rest: lr 3e-4, gamma 0.99, GAE lambda 0.95, clip 0.2, 10 epochs,
  vf_coef 0.5, ent_coef 0, max_grad_norm 0.5, per-minibatch advantage normalisation, Box-action
  clipping;
* TimeLimit truncation bootstrapped from the terminal observation's value for envs that were
  truncated and not terminated (SB3: ``infos[i]["terminal_observation"]`` and
  ``TimeLimit.truncated``); VecFrameStack(5) via ``DeviceFrameStack``.

Rollout size at 4096 envs.  config_ppo's ``n_steps=2048, batch_size=64`` are for the reference's 4
envs: 8 192 samples per update in 128 minibatches.  With 4096 envs the same n_steps would put 8.4 M
samples (24 GB of stacked obs) into every update, so this scales the other way, as massively
parallel PPO does: ``n_steps=32`` (131 072 samples per update, 16x config_ppo's) in minibatches of
4096 (64x config_ppo's, 32 per epoch): updates stay frequent in env-steps and each gradient step
averages over many envs.  Both stay configurable (``--n-steps``, ``--batch-size``).

Parity with SB3 itself is unpinned (SB3 is not installed).  Everything stays on the device:
observations, actions, rewards and dones are the env's HBM tensors; the host reads back only the
per-update statistics.

    python examples/ppo_torch.py --envs 4096 --updates 80 --log profiles/r03_ppo_4096.jsonl
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

CONFIG_PPO = {"n_stack": 5, "hidden": (256, 256), "log_std_init": -2.0, "use_sde": True, "sde_sample_freq": 4,
              "lr": 3e-4, "gamma": 0.99, "gae_lambda": 0.95, "clip": 0.2, "n_epochs": 10, "vf_coef": 0.5,
              "ent_coef": 0.0, "max_grad_norm": 0.5}
SDE_EPS = 1e-6        # StateDependentNoiseDistribution.epsilon


def mlp(inp, hidden, out=None):
    layers, d = [], inp
    for h in hidden:
        layers += [nn.Linear(d, h), nn.ReLU()]
        d = h
    if out is not None:
        layers.append(nn.Linear(d, out))
    return nn.Sequential(*layers)


class ActorCritic(nn.Module):
    def __init__(self, obs_dim, act_dim, hidden, log_std_init, use_sde=True):
        super().__init__()
        self.use_sde = use_sde
        self.pi_body = mlp(obs_dim, hidden)                 # latent_pi (gSDE's latent_sde, detached)
        self.mu = nn.Linear(hidden[-1], act_dim)
        self.vf = mlp(obs_dim, hidden, 1)
        shape = (hidden[-1], act_dim) if use_sde else (act_dim,)
        self.log_std = nn.Parameter(torch.full(shape, float(log_std_init)))

    def dist(self, obs):
        """(Normal over actions, latent_sde)."""
        lat = self.pi_body(obs)
        mean = self.mu(lat)
        if not self.use_sde:
            return torch.distributions.Normal(mean, self.log_std.exp().expand_as(mean)), None
        lat_sde = lat.detach()
        var = (lat_sde * lat_sde) @ (self.log_std.exp() ** 2)
        return torch.distributions.Normal(mean, torch.sqrt(var + SDE_EPS)), lat_sde

    def sample_weights(self, n):
        """gSDE exploration matrices, one per env: [n, latent, act] ~ N(0, exp(log_std)^2)."""
        std = self.log_std.exp().detach()
        return torch.randn((n,) + tuple(std.shape), device=std.device) * std

    def value(self, obs):
        return self.vf(obs).squeeze(-1)


class PPO:
    """Rollout + update over a ``UsvVectorEnv`` (any registered id with a Box action space)."""

    def __init__(self, env, n_steps=32, batch_size=4096, seed=0, **cfg):
        from gym_usv_amd.sb3 import DeviceFrameStack
        self.cfg = dict(CONFIG_PPO, **cfg)
        self.env, self.n_steps, self.batch_size = env, n_steps, batch_size
        self.device = env.device
        self.N, D, A = env.num_envs, env.obs_dim, env.act_dim
        self.D = D
        self.stack = DeviceFrameStack(self.N, D, self.cfg["n_stack"], self.device)
        torch.manual_seed(seed)
        self.model = ActorCritic(D * self.cfg["n_stack"], A, self.cfg["hidden"], self.cfg["log_std_init"],
                                 self.cfg["use_sde"]).to(self.device)
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
        self.abs_ye = []                                # mean |ye| (m) of every step's obs
        self.env_steps = 0
        self.W = None

    @torch.no_grad()
    def rollout(self):
        g, sde, freq = self.cfg["gamma"], self.cfg["use_sde"], self.cfg["sde_sample_freq"]
        for t in range(self.n_steps):
            if sde and (t == 0 or (freq > 0 and t % freq == 0)):   # reset_noise (SB3 collect_rollouts)
                self.W = self.model.sample_weights(self.N)
            dist, lat = self.model.dist(self.obs)
            if sde:
                a = dist.mean + torch.bmm(lat.unsqueeze(1), self.W).squeeze(1)
            else:
                a = dist.sample()
            self.b_obs[t] = self.obs
            self.b_act[t] = a
            self.b_logp[t] = dist.log_prob(a).sum(-1)
            self.b_val[t] = self.model.value(self.obs)
            a_env = torch.max(torch.min(a, self.a_hi), self.a_lo)          # SB3 clips Box actions
            obs, rew, term, trunc, info = self.env.step(a_env)
            done = info["_final_obs"]                                     # terminated | truncated
            self.abs_ye.append(obs[:, 5].abs().mean() * 10.0)   # obs[5] = ye / 10 (simple_env.py:79-80)
            nxt, term_rows = self.stack.step(obs, done, info["final_obs"])
            r = rew.float().clone()
            if bool(trunc.any()):
                # bootstrap envs truncated (TimeLimit / out of the field) and not terminated (SB3:
                # TimeLimit.truncated and not done-by-termination)
                idx = done.nonzero().flatten()
                tr = (trunc & ~term)[idx]
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
                dist, _ = self.model.dist(obs[i])
                logp = dist.log_prob(act[i]).sum(-1)
                ratio = (logp - logp0[i]).exp()
                pg = -torch.min(ratio * a_, ratio.clamp(1 - c["clip"], 1 + c["clip"]) * a_).mean()
                vl = ((self.model.value(obs[i]) - ret[i]) ** 2).mean()
                ent = -logp.mean() if c["use_sde"] else dist.entropy().sum(-1).mean()
                loss = pg + c["vf_coef"] * vl - c["ent_coef"] * ent
                self.opt.zero_grad(set_to_none=True)
                loss.backward()
                nn.utils.clip_grad_norm_(self.model.parameters(), c["max_grad_norm"])
                self.opt.step()
                stats.append(torch.stack((pg.detach(), vl.detach(), ent.detach())))
        s = torch.stack(stats).mean(0).tolist()
        return {"policy_loss": s[0], "value_loss": s[1], "entropy": s[2],
                "std_mean": float(self.model.log_std.detach().exp().mean())}

    def episode_stats(self):
        out = {"mean_abs_ye": float(torch.stack(self.abs_ye).mean())} if self.abs_ye else {}
        self.abs_ye = []
        if not self.finished:
            return {"episodes": 0, **out}
        f = torch.cat(self.finished)
        self.finished = []
        return {"episodes": int(f.shape[0]), "ep_rew_mean": float(f[:, 0].mean()),
                "ep_len_mean": float(f[:, 1].mean()), **out}


def train(env_id="usv-simple", envs=4096, updates=10, n_steps=32, batch_size=4096, seed=0, log=print, **cfg):
    import gym_usv_amd
    env = gym_usv_amd.make_vec(env_id, envs, seed=seed, copy=False)   # each step is consumed at once
    ppo = PPO(env, n_steps=n_steps, batch_size=batch_size, seed=seed, **cfg)
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
    ap.add_argument("--updates", type=int, default=80)
    ap.add_argument("--n-steps", type=int, default=32)
    ap.add_argument("--batch-size", type=int, default=4096)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--no-sde", action="store_true", help="state-independent log-std instead of gSDE")
    ap.add_argument("--log", default=None, help="also append the JSON lines to this file")
    a = ap.parse_args()
    f = open(a.log, "a") if a.log else None

    def log(s):
        print(s, flush=True)
        if f:
            f.write(s + "\n")
            f.flush()
    if f:
        log(json.dumps({"config": {**CONFIG_PPO, "use_sde": not a.no_sde, "env_id": a.env_id, "envs": a.envs,
                                   "n_steps": a.n_steps, "batch_size": a.batch_size, "seed": a.seed}}))
    train(a.env_id, a.envs, a.updates, a.n_steps, a.batch_size, a.seed, log=log, use_sde=not a.no_sde)


if __name__ == "__main__":
    main()
