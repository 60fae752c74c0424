"""Step-kernel variant sweep (usv_set_kernel_variant: envs per block, lidar variant, kind) on one GPU.

For every variant: check the outputs of a short seeded rollout are bit-identical to the first
variant's, then time back-to-back launches with HIP events.  Prints one JSON line per variant.

    python tools/sweep_variants.py [--envs 65536] [--steps 500] [--env-id usv-simple]
"""
import argparse
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-usv_amd")]

import torch  # noqa: E402

import gym_usv_amd  # noqa: E402


def run(variant, args, acts):
    env = gym_usv_amd.make_vec(args.env_id, args.envs, seed=3, precision=args.precision, kernel_variant=variant,
                               copy=False)
    env.reset(seed=3)
    outs = []
    for k in range(16):
        o, r, te, tr, _ = env.step(acts[k])
        outs.append((o.clone(), r.clone(), te.clone(), tr.clone()))
    n = args.envs
    obs = torch.empty((n, 143), device="cuda")
    fobs = torch.empty((n, 143), device="cuda")
    rew = torch.empty(n, device="cuda", dtype=env.reward.dtype)
    te = torch.empty(n, device="cuda", dtype=torch.uint8)
    tr = torch.empty(n, device="cuda", dtype=torch.uint8)
    for k in range(30):
        env.step_raw(acts[k % len(acts)], obs, rew, te, tr, fobs)
    s, e = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    torch.cuda.synchronize()
    s.record()
    for k in range(args.steps):
        env.step_raw(acts[k % len(acts)], obs, rew, te, tr, fobs)
    e.record()
    torch.cuda.synchronize()
    ms = s.elapsed_time(e) / args.steps
    env.close()
    return ms, outs


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--steps", type=int, default=500)
    ap.add_argument("--env-id", default="usv-simple")
    ap.add_argument("--precision", default="f32")
    ap.add_argument("--variants", default="64,7,1 16,7,1 16,7,2 128,7,4 128,7,5 16,7,5",
                    help="epb,lid,kind triples (include/usv_hip.h usv_set_kernel_variant)")
    args = ap.parse_args()
    g = torch.Generator(device="cuda").manual_seed(0)
    acts = [torch.rand(args.envs, 2, device="cuda", generator=g) * torch.tensor([0.8, 2.0], device="cuda")
            + torch.tensor([0.2, -1.0], device="cuda") for _ in range(64)]
    ref = None
    for v in args.variants.split():
        ms, outs = run(v, args, acts)
        same = True
        if ref is None:
            ref = outs
        else:
            for a, b in zip(ref, outs):
                same &= all(torch.equal(x, y) for x, y in zip(a, b))
        print(json.dumps({"variant": v, "env_id": args.env_id, "envs": args.envs, "precision": args.precision,
                          "ms_per_step": round(ms, 5), "env_steps_per_s": round(args.envs / ms * 1e3),
                          "bit_identical_to_first": bool(same)}), flush=True)


if __name__ == "__main__":
    main()
