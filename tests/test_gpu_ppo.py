"""C5 without stable-baselines3: torch-native gSDE PPO (examples/ppo_torch.py, config_ppo of
train_test/config.py:3-15) driven by the 4096-env HIP vector env's device tensors.

Parity with SB3's PPO is unpinned (SB3 is not installed); these check that the env drives a full
training loop (finite losses, Monitor-style episode statistics, every env-step accounted for) and
that a seeded run learns (return and episode length rise within 12 updates)."""
import math
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "examples"), os.path.join(ROOT, "gym-usv_amd")]

pytestmark = pytest.mark.gpu


def test_ppo_4096_envs_updates():
    from ppo_torch import train
    hist = train("usv-simple", envs=4096, updates=3, n_steps=16, batch_size=4096, seed=0, log=print)
    assert len(hist) == 3
    for h in hist:
        for k in ("policy_loss", "value_loss", "entropy"):
            assert math.isfinite(h[k]), h
    assert hist[-1]["env_steps"] == 3 * 16 * 4096
    eps = sum(h["episodes"] for h in hist)
    assert eps > 0                                    # collisions / out-of-field end episodes early
    done = [h for h in hist if h["episodes"]]
    assert all(math.isfinite(h["ep_rew_mean"]) and 1 <= h["ep_len_mean"] <= 48 for h in done)


def test_ppo_gsde_learns_path_following():
    """Seeded gSDE PPO at 4096 envs (config_ppo's policy, n_steps 32): within 12 updates (1.6 M
    env-steps) the episodes get longer and the return rises (the random policy collides or leaves
    the field within ~20 steps).  The committed 10 M-step curve is profiles/r03_ppo_4096.jsonl."""
    from ppo_torch import train
    hist = train("usv-simple", envs=4096, updates=12, n_steps=32, batch_size=4096, seed=0, log=print)
    first, last = hist[:3], hist[-3:]
    r0 = sum(h["ep_rew_mean"] for h in first) / 3
    r1 = sum(h["ep_rew_mean"] for h in last) / 3
    l0 = sum(h["ep_len_mean"] for h in first) / 3
    l1 = sum(h["ep_len_mean"] for h in last) / 3
    print(f"ep_rew_mean {r0:.1f} -> {r1:.1f}, ep_len_mean {l0:.1f} -> {l1:.1f}")
    assert r1 > r0 + 30 and l1 > 2 * l0


def test_ppo_asmc_simple_runs():
    from ppo_torch import train
    hist = train("usv-asmc-simple", envs=1024, updates=1, n_steps=8, batch_size=2048, seed=1, log=print)
    assert math.isfinite(hist[0]["value_loss"])
