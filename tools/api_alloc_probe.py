"""Host cost of the output allocation of a copy=True step (verdict r4 #7), no kernel: the five
separate caching-allocator calls of round 4 against one allocation viewed as the outputs.

    python tools/api_alloc_probe.py [--envs 4096]
"""
import argparse
import time

import torch


def five(n, d, dev):
    obs = torch.empty((n, d), dtype=torch.float32, device=dev)
    fobs = torch.empty((n, d), dtype=torch.float32, device=dev)
    rew = torch.empty(n, dtype=torch.float32, device=dev)
    term, trunc, done = torch.empty((3, n), dtype=torch.bool, device=dev).unbind(0)
    return obs, fobs, rew, term, trunc, done


def one_split(n, d, dev):
    # rows [0, n) obs, [n, 2n) final obs, then the reward and the flags in the tail rows
    tail = (n + (3 * n + 3) // 4 + d - 1) // d
    buf = torch.empty((2 * n + tail, d), dtype=torch.float32, device=dev)
    obs, fobs, t = buf.split((n, n, tail))
    flat = t.view(-1)
    rew = flat[:n]
    term, trunc, done = flat[n:].view(torch.bool)[:3 * n].view(3, n).unbind(0)
    return obs, fobs, rew, term, trunc, done


def one_bytes(n, d, dev):
    ob = n * d * 4
    buf = torch.empty(2 * ob + 4 * n + 3 * n, dtype=torch.uint8, device=dev)
    obs, fobs, rew, flags = buf.split((ob, ob, 4 * n, 3 * n))
    return (obs.view(torch.float32).view(n, d), fobs.view(torch.float32).view(n, d), rew.view(torch.float32),
            *flags.view(torch.bool).view(3, n).unbind(0))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--iters", type=int, default=2000)
    a = ap.parse_args()
    dev = torch.device("cuda", 0)
    n, d = a.envs, 143
    out = {}
    for f in (five, one_split, one_bytes):
        for _ in range(100):
            f(n, d, dev)
        torch.cuda.synchronize()
        t = time.perf_counter()
        for _ in range(a.iters):
            f(n, d, dev)
        out[f.__name__] = round((time.perf_counter() - t) / a.iters * 1e6, 2)
    print(out)


if __name__ == "__main__":
    main()
