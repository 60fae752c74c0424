"""Round-6 GPU tests: the bench launcher on a real box, the copy=True output ring under a side
stream, the SB3 adapter under a non-default current stream, and usv_asmc_compute's pointer checks.
"""
import ctypes
import os
import subprocess
import sys

import numpy as np
import pytest
import torch

pytestmark = pytest.mark.gpu

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def make(env_id, n, **kw):
    import gym_usv_amd
    return gym_usv_amd.make_vec(env_id, n, device=0, **kw)


def rand_actions(n, gen):
    return torch.rand(n, 2, device="cuda", generator=gen) * torch.tensor([0.8, 2.0], device="cuda") \
        + torch.tensor([0.2, -1.0], device="cuda")


def test_bench_refuses_more_gpus_than_the_box_has():
    """bench.py --gpus N with N beyond this box's GPUs exits 1 with a message and prints no line
    (verdict r5 #1: an N-GPU line is never a 1-GPU measurement)."""
    have = torch.cuda.device_count()
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(have + 1), "--steps", "3"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 1, p.stderr[-2000:]
    assert f"needs {have + 1} visible GPUs, this node shows {have}" in p.stderr and p.stdout == ""


def _sleep_on(stream, ms=30):
    """Keep `stream` busy for about `ms` milliseconds."""
    with torch.cuda.stream(stream):
        if hasattr(torch.cuda, "_sleep"):
            torch.cuda._sleep(int(ms * 2.4e6))            # clock cycles at ~2.4 GHz
        else:
            x = torch.randn(2048, 2048, device="cuda")
            for _ in range(40):
                x = x @ x
                x = x / x.norm()


def test_copy_true_side_stream_read_of_a_dropped_output():
    """copy=True outputs read on another stream (recorded with record_stream) and then dropped by the
    caller: later steps must not write into them before that read ran (verdict r5 #6).  Without the
    side stream the ring still hands the same set back (the fast path is kept)."""
    n = 4096
    env = make("usv-simple", n, seed=3)
    env.reset(seed=3)
    gen = torch.Generator(device="cuda").manual_seed(1)
    a = rand_actions(n, gen)
    # fast path: a dropped set comes back
    out = env.step(a)
    p0 = out[0].data_ptr()
    del out
    out = env.step(a)
    assert out[0].data_ptr() == p0
    del out
    # side-stream read of a dropped output
    obs, rew, term, trunc, info = env.step(a)
    expect_obs, expect_rew = obs.clone(), rew.clone()
    side = torch.cuda.Stream()
    side.wait_stream(torch.cuda.current_stream())
    _sleep_on(side, 50)
    with torch.cuda.stream(side):
        seen_obs = obs * 1.0
        seen_rew = rew * 1.0
    obs.record_stream(side)
    rew.record_stream(side)
    p_obs = obs.data_ptr()
    del obs, rew, term, trunc, info
    reused = False
    for _ in range(6):                            # each would be a chance to reuse the set
        o2, *_rest = env.step(rand_actions(n, gen))
        reused |= o2.data_ptr() == p_obs
        del o2, _rest
    side.synchronize()
    torch.cuda.synchronize()
    assert torch.equal(seen_obs, expect_obs) and torch.equal(seen_rew, expect_rew)
    print(f"\n[copy=True side stream] the recorded set handed out again before the read: {reused}")
    env.close()


def test_copy_true_dlpack_export_keeps_the_set():
    """A copy=True output exported by DLPack and dropped as a tensor is not overwritten while the
    capsule lives."""
    from torch.utils import dlpack
    n = 1024
    env = make("usv-simple", n, seed=4)
    env.reset(seed=4)
    gen = torch.Generator(device="cuda").manual_seed(2)
    obs, *_ = env.step(rand_actions(n, gen))
    expect = obs.clone()
    cap = dlpack.to_dlpack(obs)
    del obs, _
    for _ in range(5):
        o, *r = env.step(rand_actions(n, gen))
        del o, r
    back = dlpack.from_dlpack(cap)
    torch.cuda.synchronize()
    assert torch.equal(back, expect)
    env.close()


def test_sb3_step_wait_under_a_non_default_current_stream():
    """Sb3VecEnv.step_wait called while a side stream is current on the env's device: the step is
    launched on that stream and the copies wait for it; outputs bit-identical to the raw env stepped on
    the default stream."""
    import gym_usv_amd
    from gym_usv_amd.sb3 import Sb3VecEnv
    n = 512
    env = Sb3VecEnv("usv-simple", num_envs=n, seed=5)
    raw = gym_usv_amd.make_vec("usv-simple", n, seed=5)
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        env.reset()
    raw.reset(seed=5)
    rng = np.random.default_rng(0)
    for t in range(30):
        a = rng.uniform([0.2, -1], [1, 1], size=(n, 2)).astype(np.float32)
        with torch.cuda.stream(side):
            _sleep_on(side, 2)                      # the step queues behind work on that stream
            o, r, dn, _ = env.step(a)
        ro, rr, rte, rtr, _ = raw.step(torch.from_numpy(a).cuda())
        np.testing.assert_array_equal(o, ro.cpu().numpy(), err_msg=f"t={t}")
        np.testing.assert_array_equal(r, rr.cpu().numpy())
        np.testing.assert_array_equal(dn, (rte | rtr).cpu().numpy())
    env.close()
    raw.close()


def test_asmc_compute_rejects_host_pointers():
    """usv_asmc_compute checks every buffer: a pageable host pointer for the state, or for an input,
    returns USV_ERR_ARG before any launch."""
    from gym_usv_amd import _lib
    lib = _lib.load()
    n = 8
    vp = ctypes.c_void_p
    act = torch.zeros(n, 2, dtype=torch.float64, device="cuda")
    pos = torch.zeros(n, 3, dtype=torch.float64, device="cuda")
    vel = torch.zeros(n, 3, dtype=torch.float64, device="cuda")
    st = torch.zeros(16, n, dtype=torch.float64, device="cuda")
    host = np.zeros((16, n))
    hp = vp(host.ctypes.data)
    s0 = vp(torch.cuda.current_stream().cuda_stream)
    F64 = 1
    assert lib.usv_asmc_compute(F64, n, vp(act.data_ptr()), vp(pos.data_ptr()), vp(vel.data_ptr()), hp,
                                None, 0, 1, s0) == -1
    assert b"state" in lib.usv_last_error()
    assert lib.usv_asmc_compute(F64, n, hp, vp(pos.data_ptr()), vp(vel.data_ptr()), vp(st.data_ptr()),
                                None, 0, 1, s0) == -1
    assert lib.usv_asmc_compute(F64, n, vp(act.data_ptr()), vp(pos.data_ptr()), hp, vp(st.data_ptr()),
                                None, 0, 1, s0) == -1
    # the same call with device buffers runs
    assert lib.usv_asmc_compute(F64, n, vp(act.data_ptr()), vp(pos.data_ptr()), vp(vel.data_ptr()),
                                vp(st.data_ptr()), None, 0, 1, s0) == 0
    torch.cuda.synchronize()
    assert torch.isfinite(pos).all()


def test_bench_line_at_n1_has_the_contract_fields():
    """python bench.py --gpus 1 (short): one JSON line with the contract's fields, the roofline and
    API objects, one rank, a single-process launcher (the driver's N = 1 form)."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "1", "--steps", "20",
                        "--warmup", "5", "--no-cpu-baseline", "--f64-steps", "50", "--api-steps", "20",
                        "--steady-steps", "100"], capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    for k in ("metric", "value", "unit", "n_gpus", "steps", "warmup", "ms_per_step", "higher_is_better",
              "scaling", "vs_baseline", "dtype", "data", "config", "roofline", "cpu_baseline"):
        assert k in d, k
    assert d["n_gpus"] == 1 and d["ranks_seen"] == 1 and d["launcher"] == "single process"
    assert d["steps"] == 20 and d["value"] > 0 and d["scaling"] == "weak"
    r = d["roofline"]
    assert r["bound"] == "hbm" and 0 < r["frac"] < 1 and r["unit"] == "GB/s" and r["peak"] == 8000.0
    assert d["config"]["envs_per_gpu"] == 65536 and d["f64"]["dtype"] == "f64"
    assert d["value"] == pytest.approx(65536 * 20 / (d["ms_per_step"] * 20 / 1e3), rel=1e-3)


@pytest.mark.parametrize("env_id", ["usv-simple", "usv-asmc-simple"])
def test_max_size_batch_matches_its_shard(env_id):
    """2^23 envs on one GPU (~20 GB of HBM for the state and the persistent outputs): the last 4 096 envs
    of the batch step bit-identically to a 4 096-env batch with env_id_offset = N - 4096 (resets keyed by
    global id; a 3-step TimeLimit so every env resets twice), i.e. no indexing overflows at the top of the
    range and the DRAM-size kernel (row spans, multi-round grid) agrees with the small-count one."""
    N, n, T = 1 << 23, 4096, 7
    big = make(env_id, N, seed=21, max_episode_steps=3, copy=False)
    small = make(env_id, n, seed=21, max_episode_steps=3, copy=False, env_id_offset=N - n)
    ob, _ = big.reset(seed=21)
    os_, _ = small.reset(seed=21)
    assert torch.equal(ob[N - n:], os_)
    gen = torch.Generator(device="cuda").manual_seed(9)
    for t in range(T):
        a = rand_actions(N, gen)
        ob, rb, tb, trb, ib = big.step(a)
        os_, rs, ts, trs, is_ = small.step(a[N - n:].contiguous())
        torch.cuda.synchronize()
        assert torch.equal(ob[N - n:], os_), f"obs differ at step {t}"
        assert torch.equal(rb[N - n:], rs) and torch.equal(tb[N - n:], ts) and torch.equal(trb[N - n:], trs)
        done = ib["_final_obs"][N - n:]
        assert torch.equal(done, is_["_final_obs"])
        if bool(done.any()):
            assert torch.equal(ib["final_obs"][N - n:][done], is_["final_obs"][done])
    assert bool(torch.isfinite(ob).all()) and bool(torch.isfinite(rb).all())
    big.close()
    small.close()


def test_spawned_rank_runs_the_real_bench():
    """bench.spawn_ranks with one rank on the real GPU (the machinery `--gpus N > 1` uses on a
    multi-GPU node, here at N = 1): the spawned interpreter gets the launcher environment, binds
    cuda:0, runs the timed window and prints the line; the parent returns its exit status."""
    import json
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    argv = ["--gpus", "1", "--steps", "20", "--warmup", "5", "--no-cpu-baseline", "--f64-steps", "0",
            "--api-steps", "0", "--steady-steps", "0"]
    prog = ("import sys; sys.path.insert(0, %r); import bench; sys.exit(bench.spawn_ranks(1, %r))" % (ROOT, argv))
    p = subprocess.run([sys.executable, "-c", prog], capture_output=True, text=True, env=env, timeout=300,
                       cwd=ROOT)
    assert p.returncode == 0, p.stderr[-2000:]
    lines = [ln for ln in p.stdout.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    d = json.loads(lines[0])
    assert d["launcher"] == "bench.py spawn" and d["ranks_seen"] == 1 and d["n_gpus"] == 1
    assert d["value"] > 0 and 0 < d["roofline"]["frac"] < 1
