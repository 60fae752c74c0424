"""Same-step resets per launch (terminated | truncated envs per step) in a steady random-action
rollout, per env id: the block-queue step runs each reset inside its pair loop, so the q kernel's
time depends on this rate (DESIGN: usv-asmc-simple's q kernel vs usv-simple's).

    python tools/done_rate.py [--envs 65536] [--steps 3000]
"""
import argparse
import json
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-usv_amd"))
import gym_usv_amd  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=3000)
    ap.add_argument("--skip", type=int, default=1000)
    a = ap.parse_args()
    out = {}
    for env_id in ("usv-simple", "usv-asmc-simple"):
        env = gym_usv_amd.make_vec(env_id, a.envs, seed=2, copy=False)
        env.reset(seed=2)
        g = torch.Generator(device="cuda").manual_seed(0)
        lo, span = torch.tensor([0.2, -1.0], device="cuda"), torch.tensor([0.8, 2.0], device="cuda")
        term = trunc = 0
        for k in range(a.steps):
            _, _, te, tr, _ = env.step(torch.rand(a.envs, 2, device="cuda", generator=g) * span + lo)
            if k >= a.skip:
                term += int(te.sum())
                trunc += int((tr & ~te).sum())
        n = a.steps - a.skip
        out[env_id] = {"terminated_per_step": round(term / n, 1), "truncated_only_per_step": round(trunc / n, 1),
                       "resets_per_step": round((term + trunc) / n, 1),
                       "resets_per_block_per_step": round((term + trunc) / n / (a.envs / 128), 3)}
        env.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
