"""Round-5 GPU tests.

* Same-step autoreset ordering: in the fused block queue (kinds 5 and 6) and in kind 3,
  one wave's phase-1 dynamics store an env's state and another wave may reset that env in the same
  launch.  The reset now waits for an LDS flag the dynamics wave sets once its stores are
  acknowledged.  Checked at 524 288 envs (state in DRAM, not the Infinity Cache) with a 3-step
  TimeLimit, so every env resets every third step, against the split kinds whose dynamics run in
  their own launch (kinds 4 and 2): whole state blobs and step outputs bit-identical.
"""
import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu


def make(env_id, n, **kw):
    import gym_usv_amd
    return gym_usv_amd.make_vec(env_id, n, device=0, **kw)


def _rollout(env_id, n, variant, precision, T, limit, seed=21):
    gen = torch.Generator(device="cuda").manual_seed(seed)
    env = make(env_id, n, seed=seed, precision=precision, max_episode_steps=limit, kernel_variant=variant,
               copy=False)
    env.reset(seed=seed)
    digest = []
    for _ in range(T):
        a = torch.rand(n, 2, device="cuda", generator=gen) * torch.tensor([0.8, 2.0], device="cuda") \
            + torch.tensor([0.2, -1.0], device="cuda")
        o, r, te, tr, info = env.step(a)
        # per-step digests of the outputs (full tensors would not fit 2 x T copies at this size)
        digest.append(tuple(float(x.double().sum()) for x in (o, r, te.to(torch.int32), tr.to(torch.int32))))
    torch.cuda.synchronize()
    blob = env.state_blob()
    done = int((env.get_field("episode") > 0).sum())
    env.close()
    return digest, blob, done


@pytest.mark.parametrize("env_id,precision,n,fused,split", [
    ("usv-simple", "f32", 524288, "128,7,5", "128,7,4"),
    ("usv-asmc-simple", "f32", 524288, "128,7,6", "128,7,4"),
    ("usv-simple", "f64", 131072, "64,7,3", "64,7,2"),
])
def test_same_step_reset_after_dynamics_bit_identical_at_dram_size(env_id, precision, n, fused, split):
    T, limit = 7, 3
    d_f, b_f, done_f = _rollout(env_id, n, fused, precision, T, limit)
    d_s, b_s, done_s = _rollout(env_id, n, split, precision, T, limit)
    assert done_f == done_s and done_f >= n          # every env reset at least twice (episode counter)
    assert d_f == d_s
    assert b_f.shape == b_s.shape
    bad = np.flatnonzero(b_f != b_s)
    assert bad.size == 0, f"state blobs differ in {bad.size} bytes (first at byte {bad[:4]})"


@pytest.mark.parametrize("bad", [float("nan"), float("inf"), 1e11])
def test_heading_set_rejects_unrepresentable_turns(bad):
    """The f32 build stores the heading as phi + 2 pi k with k an int32 (DESIGN 'Heading in the f32
    build'): a non-finite heading or one whose turn count overflows int32 is refused
    and leaves the state untouched."""
    import gym_usv_amd
    env = make("usv-simple", 64, seed=3)
    env.reset(seed=3)
    before = env.get_field("psi").copy()
    psi = before.copy()
    psi[5] = bad
    with pytest.raises(gym_usv_amd.UsvLibError):
        env.set_field("psi", psi)
    np.testing.assert_array_equal(env.get_field("psi"), before)
    psi[5] = 1e9                                       # large but representable: exact round trip of k
    env.set_field("psi", psi)
    got = env.get_field("psi")
    assert abs(got[5] - 1e9) <= 2 * np.pi * 2 ** -23 * 4   # phi in [-pi, pi] rounded to f32
    env.close()


@pytest.mark.parametrize("env_id,n", [("usv-simple", 40000), ("usv-simple", 65536), ("usv-simple", 60001),
                                      ("usv-asmc-simple", 65536), ("usv-asmc-simple", 33001)])
def test_one_round_grid_bit_identical(env_id, n):
    """One-round grids of the 128-env block queue (<= 2 blocks per CU) run the round-5 priority path
    (phase-1 priority, the second blocks' raised waves, the dynamics waves' drain and flag):
    bit-identical to the split kind 4 (same queue, dynamics in their own launch) and to the fused
    wave kernel (kind 1), over a rollout with same-step resets, at full and ragged counts."""
    T, limit = 24, 9
    fused = "128,7,6" if env_id == "usv-asmc-simple" else "128,7,5"
    ref = None
    for v in (fused, "128,7,4", "16,7,1"):
        gen = torch.Generator(device="cuda").manual_seed(4)
        env = make(env_id, n, seed=31, max_episode_steps=limit, kernel_variant=v, copy=False)
        env.reset(seed=31)
        outs = []
        for _ in range(T):
            a = torch.rand(n, 2, device="cuda", generator=gen) * torch.tensor([0.8, 2.0], device="cuda") \
                + torch.tensor([0.2, -1.0], device="cuda")
            o, r, te, tr, info = env.step(a)
            outs.append(torch.cat([o.flatten(), r, te.float(), tr.float()]).cpu())
        blob = env.state_blob()
        env.close()
        if ref is None:
            ref = (outs, blob)
            continue
        for t, (x, y) in enumerate(zip(ref[0], outs)):
            assert torch.equal(x, y), f"variant {v} differs from {fused} at step {t} (n={n})"
        assert np.array_equal(ref[1], blob), f"variant {v}: state differs (n={n})"
