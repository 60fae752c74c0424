"""Env-steps/s at one env count through the three host surfaces (config C2/C5 scale):

* ``step_raw``  -- the C-ABI launch into caller-owned buffers (what bench.py times);
* ``step``      -- the public UsvVectorEnv.step (torch.as_tensor / dtype / shape checks, outputs in HBM;
                   fresh tensors), ``step_nocopy`` the same with copy=False (persistent buffers);
* ``sb3``       -- Sb3VecEnv.step (VecFrameStack(5) on device, NumPy host copies + Monitor infos per
                   step, i.e. what an SB3 algorithm consumes).

    python tools/api_throughput.py [--envs 4096] [--steps 2000]
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-usv_amd")]

import numpy as np  # noqa: E402
import torch  # noqa: E402


def rate(fn, steps, n):
    for k in range(20):
        fn(k)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for k in range(steps):
        fn(k)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    return {"env_steps_per_s": round(n * steps / dt, 1), "us_per_step": round(dt / steps * 1e6, 2)}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=2000)
    ap.add_argument("--env-id", default="usv-simple")
    a = ap.parse_args()
    import gym_usv_amd
    n = a.envs
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = torch.rand((64, n, 2), device="cuda", generator=g) * torch.tensor([0.8, 2.0], device="cuda") + \
        torch.tensor([0.2, -1.0], device="cuda")
    env = gym_usv_amd.make_vec(a.env_id, n, seed=0)
    env.reset(seed=0)
    obs, fobs = torch.empty((n, env.obs_dim), device="cuda"), torch.empty((n, env.obs_dim), device="cuda")
    rew = torch.empty(n, device="cuda")
    te, tr = torch.empty(n, dtype=torch.uint8, device="cuda"), torch.empty(n, dtype=torch.uint8, device="cuda")
    out = {"env_id": a.env_id, "envs": n, "steps": a.steps}
    out["step_raw"] = rate(lambda k: env.step_raw(acts[k % 64], obs, rew, te, tr, fobs), a.steps, n)
    out["step"] = rate(lambda k: env.step(acts[k % 64]), a.steps, n)               # copy=True (default)
    env.close()
    env = gym_usv_amd.make_vec(a.env_id, n, seed=0, copy=False)
    env.reset(seed=0)
    out["step_nocopy"] = rate(lambda k: env.step(acts[k % 64]), a.steps, n)        # persistent buffers
    env.close()
    sb = gym_usv_amd.make_sb3_vec_env(a.env_id, n, frame_stack=5, seed=0)
    sb.reset()
    acts_np = acts.cpu().numpy()
    out["sb3"] = rate(lambda k: sb.step(acts_np[k % 64]), max(1, a.steps // 4), n)
    sb.close()
    print(json.dumps(out))


if __name__ == "__main__":
    main()
