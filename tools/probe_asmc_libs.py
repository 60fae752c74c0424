"""Checksums of a short usv-asmc-simple f32 rollout per library build (same seed, same actions):
shows whether two builds' ASMC substeps differ on the env path.   USV_LIB_PATH=... python tools/probe_asmc_libs.py"""
import os
import sys

import torch

sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "gym-usv_amd"))
import gym_usv_amd  # noqa: E402

for info in (False, True):
    for variant in (None, "128,7,4", "16,7,1"):
        env = gym_usv_amd.make_vec("usv-asmc-simple", 256, seed=3, info=info, kernel_variant=variant, copy=False)
        env.reset(seed=3)
        g = torch.Generator(device="cuda").manual_seed(1)
        acc = 0.0
        for _ in range(20):
            a = torch.rand(256, 2, device="cuda", generator=g) * torch.tensor([0.8, 2.0], device="cuda") + \
                torch.tensor([0.2, -1.0], device="cuda")
            o, r, *_ = env.step(a)
            acc += float(o[:, :15].double().sum()) + float(r.double().sum())
        print(os.environ.get("USV_LIB_PATH", "product"), "info", info, "variant", variant, repr(acc))
        env.close()
