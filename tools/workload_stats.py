"""Steady-state lidar workload of the bench configuration (diagnostic).

Runs the bench's random-action rollout on the GPU, then pulls the state and reports per env:
obstacle count, the fraction of envs with an obstacle >= 99 m away (range-checked lidar), and the
angular-window pair count W (pairs the window lidar tests; brute tests 128 * n).

    python tools/workload_stats.py [--envs 65536] [--steps 2000]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-usv_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402

RES = (4 * np.pi / 3) / 128


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--env-id", default="usv-simple")
    args = ap.parse_args()
    import gym_usv_amd
    env = gym_usv_amd.make_vec(args.env_id, args.envs, seed=1)
    env.reset(seed=1)
    g = torch.Generator(device="cuda").manual_seed(0)
    lo = torch.tensor([0.2, -1.0], device="cuda")
    for _ in range(args.steps):
        env.step(torch.rand(args.envs, 2, device="cuda", generator=g) * torch.tensor([0.8, 2.0], device="cuda") + lo)
    st = env.get_state()
    x, y, psi = st["x"], st["y"], st["psi"]
    n = st["n_obs"].astype(int)
    ox, oy, orr = st["obs_x"], st["obs_y"], st["obs_r"]
    valid = np.arange(ox.shape[1])[None, :] < n[:, None]
    dx, dy = ox - x[:, None], oy - y[:, None]
    d = np.hypot(dx, dy)
    far = ((d >= 99) & valid).any(1)
    phi = np.angle(np.exp(1j * (np.arctan2(dy, dx) - (psi[:, None] - 2 * np.pi / 3))))   # (-pi, pi]
    half = np.where(d <= orr * 1.001, np.pi / 2,
                    np.arcsin(np.minimum(orr / np.maximum(d, 1e-9), 1))) + 0.25 * RES
    cnt = np.zeros_like(d)
    for c in (phi, phi + 2 * np.pi):
        lo_i = np.maximum(0, np.ceil((c - half) / RES))
        hi_i = np.minimum(127, np.floor((c + half) / RES))
        cnt += np.maximum(0, hi_i - lo_i + 1)
    W = (cnt * valid).sum(1)
    out = {"envs": args.envs, "steps": args.steps, "n_obs_mean": float(n.mean()),
           "far_frac": float(far.mean()), "pairs_mean": float(W.mean()),
           "pairs_pcts": np.percentile(W, [50, 90, 99, 100]).tolist(),
           "passes_mean": float(np.ceil(W / 64).mean()), "brute_pairs_mean": float(128 * n.mean())}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
