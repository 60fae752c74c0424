"""PPO on the HIP vector env: the counterpart of the reference's train_test/sb3_train_vec.py.

The reference builds ``make_vec_env("usv-simple", n_envs=4, vec_env_cls=DummyVecEnv)``, wraps it
in ``VecVideoRecorder`` and ``VecFrameStack(env, 5)`` (sb3_train_vec.py:67-70) and trains with the
``config_ppo`` dict (train_test/config.py:3-15).  Here the env line becomes one HIP-stepped batch;
everything SB3-side is unchanged.  Video recording is out of scope (no rendering) and wandb logging
is left to the caller.  Needs stable-baselines3 (not installed in this image):

    python examples/sb3_train_vec_hip.py --envs 4096 --steps 2000000
"""
import argparse
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT, os.path.join(ROOT, "gym-usv_amd")]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--env-id", default="usv-simple")
    ap.add_argument("--envs", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=2_000_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--n-steps", type=int, default=16)
    ap.add_argument("--batch-size", type=int, default=4096)
    args = ap.parse_args()
    from stable_baselines3 import PPO                     # noqa: E402  (optional dependency)
    import gym_usv_amd

    env = gym_usv_amd.make_sb3_vec_env(args.env_id, args.envs, frame_stack=5, seed=args.seed).as_sb3()
    # config_ppo (config.py:3-15).  n_steps is per env: the reference's 2048 x 4 envs = 8192
    # samples per rollout; at 4096 envs the same rollout size is n_steps = 2 (raise it with
    # --n-steps), and the reference's batch_size 64 is scaled with the env count.
    import torch.nn as nn
    config_ppo = {"use_sde": True, "sde_sample_freq": 4,
                  "n_steps": args.n_steps, "batch_size": args.batch_size,
                  "policy_kwargs": dict(log_std_init=-2, ortho_init=False, activation_fn=nn.ReLU,
                                        net_arch=dict(pi=[256, 256], vf=[256, 256]))}
    model = PPO("MlpPolicy", env, verbose=1, seed=args.seed, **config_ppo)
    model.learn(total_timesteps=args.steps)
    model.save(f"ppo_{args.env_id}_hip")


if __name__ == "__main__":
    main()
