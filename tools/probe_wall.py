"""Where the fixed host-side cost of bench.py's timed region goes (diagnostic; no GPU work changed).

    python tools/probe_wall.py [--envs 65536]

Prints, in µs: an idle torch.cuda.synchronize(); one ctypes usv_step call's host time; the wall of
1 and of 20 back-to-back step launches bracketed by synchronize() (as bench.py's timed region);
the same with the stream's synchronize instead of the device's; and the HIP-event time of the 20.
"""
import argparse
import ctypes
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-usv_amd")]

import torch  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=65536)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    import gym_usv_amd
    N = args.envs
    env = gym_usv_amd.make_vec("usv-simple", N, seed=0, copy=False)
    env.reset(seed=0)
    dev = torch.device("cuda", 0)
    acts = torch.rand((N, 2), device=dev) * torch.tensor([0.8, 2.0], device=dev) + torch.tensor([0.2, -1.0], device=dev)
    obs, fobs = torch.empty((N, 143), device=dev), torch.empty((N, 143), device=dev)
    rew = torch.empty(N, device=dev)
    term, trunc = torch.empty(N, device=dev, dtype=torch.uint8), torch.empty(N, device=dev, dtype=torch.uint8)
    stream = torch.cuda.current_stream(dev)
    vp = ctypes.c_void_p
    args_ = (env._h, vp(acts.data_ptr()), vp(obs.data_ptr()), vp(rew.data_ptr()), vp(term.data_ptr()),
             vp(trunc.data_ptr()), vp(fobs.data_ptr()), vp(stream.cuda_stream))
    step = env.lib.usv_step
    for _ in range(3000):                      # clocks up
        step(*args_)
    torch.cuda.synchronize(dev)
    out = {}

    def med(xs):
        xs = sorted(xs)
        return round(xs[len(xs) // 2] * 1e6, 2)

    xs = []
    for _ in range(args.reps):
        t = time.perf_counter(); torch.cuda.synchronize(dev); xs.append(time.perf_counter() - t)
    out["sync_idle_us"] = med(xs)
    xs = []
    for _ in range(args.reps):
        torch.cuda.synchronize(dev)
        t = time.perf_counter(); step(*args_); xs.append(time.perf_counter() - t)
    torch.cuda.synchronize(dev)
    out["launch_call_us"] = med(xs)
    for K in (1, 20):
        for how in ("device", "stream"):
            xs, ev = [], []
            for _ in range(args.reps):
                e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
                torch.cuda.synchronize(dev)
                t = time.perf_counter()
                e0.record(stream)
                for _ in range(K):
                    step(*args_)
                e1.record(stream)
                if how == "device":
                    torch.cuda.synchronize(dev)
                else:
                    stream.synchronize()
                xs.append(time.perf_counter() - t)
                ev.append(e0.elapsed_time(e1) * 1e-3)
            out[f"wall_{K}_{how}_sync_us"] = med(xs)
            out[f"event_{K}_{how}_sync_us"] = med(ev)
    # bench.py's round-3/4 layout: events after the first launch and after launch 17 (markers between kernels)
    for how in ("mid_events", "edge_events", "no_events"):
        xs = []
        for _ in range(args.reps):
            e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
            torch.cuda.synchronize(dev)
            t = time.perf_counter()
            if how == "edge_events":
                e0.record(stream)
            step(*args_)
            for k in range(1, 20):
                if how == "mid_events" and k == 1:
                    e0.record(stream)
                step(*args_)
                if how == "mid_events" and k == 16:
                    e1.record(stream)
            if how == "edge_events":
                e1.record(stream)
            torch.cuda.synchronize(dev)
            xs.append(time.perf_counter() - t)
        out[f"wall_20_{how}_us"] = med(xs)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
