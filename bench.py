"""Benchmark: env-steps/s of the batched HIP USV step at 65 536 envs per GPU (BASELINE.json).

    python bench.py [--gpus N] [--steps K] [--warmup W] [--envs 65536] [--env-id usv-simple]
    python -m torch.distributed.run --nproc-per-node N --master-addr 127.0.0.1 bench.py --gpus N

--gpus N without a launcher starts N rank processes itself (spawn_ranks: fresh interpreters, the
same environment torch.distributed.run gives its ranks); under a launcher --gpus must equal
WORLD_SIZE, and --gpus beyond the visible GPUs is refused (resolve_world), so an N-GPU line is
always N ranks on N GPUs.

A "step" is one launch of the fused step kernel over every env of the rank (config C3:
usv-simple, 65 536 envs, random actions in [0.2,1]x[-1,1], in-kernel TimeLimit + same-step
autoreset).  Actions for all K timed steps are generated on the device before the timed
region (inputs resident in HBM).  Multi-GPU: one process per GPU, envs sharded by global id
(env_id_offset = rank * N), no collective on the step path (weak scaling); the only
collectives are the barrier and the max-over-ranks of the elapsed time.

Warm-up: the W warm-up steps, then more untimed steps until --clock-warmup seconds have passed
(the GPU clock ramps over the first few hundred milliseconds of work; a short --warmup would
otherwise time a cold chip).  The line reports both counts.

Rank 0 prints one JSON line: value = all ranks' env-steps / max-rank time, plus
  roofline:     algorithmic bytes per launch / mean launch duration (HIP events on the env's stream
                around groups of back-to-back launches 2..K; --event-layout edge: one pair around
                all K launches, no timing marker between two launches)
                vs 8 TB/s; traffic from the committed
                rocprofv3 PMC summary (profiles/pmc_summary.json) when it matches the workload;
                valu_frac = VALU wave-instructions per launch (same summary, SQ_INSTS_VALU) x 2
                cycles (a wave64 VALU instruction on a SIMD-32) / (1024 SIMDs x 2.4 GHz x launch time).
  api_step:     the public UsvVectorEnv.step() (ctypes call, checks, output tensors) timed over the
                same envs, copy=True (fresh output tensors) and copy=False (persistent buffers).
  cpu_baseline: the CPU oracle (per-env NumPy restatement of the reference step, oracle/) timed
                on this host's cores for a bounded sample.
"""
from __future__ import annotations

import argparse
import json
import math
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
for _p in (ROOT, os.path.join(ROOT, "gym-usv_amd")):
    if _p not in sys.path:
        sys.path.insert(0, _p)

HBM_PEAK_GBS = 8000.0      # MI355X HBM3E spec peak (MI355X_MICROARCH.md, chip-level table)
SIMDS, CLOCK_GHZ, VALU_CYCLES = 1024, 2.4, 2   # 256 CUs x 4 SIMD-32; max clock; wave64 VALU issue
METRIC = "env-steps/sec at 65 536 parallel envs; 1/2/4/8 MI355X scaling"


# --------------------------------------------------------------------------- byte model
LEGACY_IDS = ("usv-asmc-v0", "usv-pid-v0", "usv-asmc-ye-int-v0")


def algorithmic_bytes_per_env_step(env_id, mean_obs, precision="f32"):
    """Bytes one env-step must move (DESIGN.md 'Algorithmic bytes'): action in, obs/reward/flags
    out, dynamic state read+write, obstacle read (x, y, r per obstacle).  Reset traffic excluded."""
    w = 4 if precision == "f32" else 8
    if env_id in LEGACY_IDS:
        # action 4, obs 6 f32, reward, flags; state read: pose+velocity (6) + last/aux/target/
        # action_last (19) + elapsed; write: 6 + 13 (target is read-only) + elapsed;
        # usv-asmc-ye-int-v0 also reads and writes ye_int, ye_last
        ye = 2 * w if env_id == "usv-asmc-ye-int-v0" else 0
        return 4 + 6 * 4 + w + 2 + (25 * w + 4 + ye) + (19 * w + 4 + ye)
    act, obs, rew, flags = 8, 143 * 4, w, 2
    state_rd = 16 * w + 2 * 4          # 16 real fields + n_obs + elapsed
    state_wr = 9 * w + 2 * 4           # pose, velocity, last action, progress + elapsed, scan flag
    obst = 3 * w * mean_obs
    asmc = 2 * 16 * w if env_id == "usv-asmc-simple" else 0
    return act + obs + rew + flags + state_rd + state_wr + obst + asmc


# --------------------------------------------------------------------------- multi-rank plumbing
def shard(rank, envs_per_rank):
    """Global env ids owned by `rank`: [rank*N, (rank+1)*N) (DESIGN.md 'Multi-GPU').  The reset
    RNG is keyed by global id, so results do not depend on the number of ranks."""
    return rank * envs_per_rank, (rank + 1) * envs_per_rank


def reduce_max(values, device=None):
    """Max over ranks of a few floats (elapsed time, kernel time); identity when not distributed."""
    import torch
    import torch.distributed as dist
    if not (dist.is_available() and dist.is_initialized()) or dist.get_world_size() == 1:
        return [float(v) for v in values]
    t = torch.tensor(values, dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return [float(v) for v in t.tolist()]


def aggregate_rate(envs_per_rank, world, steps, max_elapsed):
    """Whole-job env-steps/s: every rank's env-steps over the slowest rank's time (weak scaling)."""
    return envs_per_rank * world * steps / max_elapsed


def timed_window(launch, K, sync, barrier):
    """The timed region: sync, barrier, sync, then t0; K launches; sync, then t1.  The barrier
    lines the ranks up before t0, and nothing between t0 and t1 is a collective: the max over ranks
    (reduce_max) and the closing barrier come after t1, so an N-rank curve times kernels, not RCCL
    (tests/test_multirank.py::test_timed_window_is_collective_free)."""
    sync()
    barrier()
    sync()
    t0 = time.perf_counter()
    for k in range(K):
        launch(k)
    sync()
    t1 = time.perf_counter()
    barrier()          # (outside the window) every rank has finished before the reductions
    return t0, t1


# --------------------------------------------------------------------------- CPU baseline
def _cpu_worker(args):
    env_id, seconds, seed = args
    os.environ.setdefault("OMP_NUM_THREADS", "1")
    import numpy as np
    from oracle import usv_oracle as O
    rng = np.random.default_rng(seed)
    if env_id in LEGACY_IDS:
        o = O.AsmcV0Batch(1) if env_id == "usv-asmc-v0" else \
            O.LegacyF64Batch(1, "pid" if env_id == "usv-pid-v0" else "ye_int")
        o.reset([seed])

        def one():
            _, _, d = o.step(rng.uniform(-np.pi / 2, np.pi / 2, 1).astype(np.float32))
            if d[0]:
                o.reset(idx=[0])
    else:
        venv = O.OracleVectorEnv(env_id, 1)
        venv.reset([seed])

        def one():
            venv.step(rng.uniform([0.2, -1], [1, 1], size=(1, 2)).astype(np.float32))
    n, t0 = 0, time.perf_counter()
    while True:
        one()
        n += 1
        if n % 32 == 0 and time.perf_counter() - t0 >= seconds:
            break
    return n, time.perf_counter() - t0


def host_cores():
    """Cores this process may use: the affinity set, capped by a cgroup CPU quota when one is set
    and by the host's declared CPU share (OMP_NUM_THREADS, which the GPU pool sets to the box's
    share of the node: its affinity mask lists every CPU of the machine)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        q, p = open("/sys/fs/cgroup/cpu.max").read().split()[:2]       # cgroup v2: "max 100000"
        if q != "max":
            quota = float(q) / float(p)
    except (OSError, ValueError):
        try:                                                            # cgroup v1
            q = int(open("/sys/fs/cgroup/cpu/cpu.cfs_quota_us").read())
            p = int(open("/sys/fs/cgroup/cpu/cpu.cfs_period_us").read())
            quota = q / p if q > 0 else None
        except (OSError, ValueError):
            quota = None
    cores = aff if quota is None else max(1, min(aff, int(quota)))
    share = os.environ.get("OMP_NUM_THREADS", "")
    if share.isdigit() and int(share) > 0:
        cores = min(cores, int(share))
    return cores, aff, quota


def cpu_model():
    try:
        for line in open("/proc/cpuinfo"):
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    except OSError:
        pass
    return "unknown"


def cpu_baseline(env_id, seconds, procs, affinity=None, quota=None):
    ctx = mp.get_context("spawn")
    with ctx.Pool(procs) as pool:
        res = pool.map(_cpu_worker, [(env_id, seconds, 1000 + i) for i in range(procs)])
    steps = sum(r[0] for r in res)
    rate = sum(r[0] / r[1] for r in res)
    out = {"value": round(rate, 1), "unit": "env-steps/s", "cores": procs, "kind": "port",
           "cpu_model": cpu_model(), "affinity_cpus": affinity, "cgroup_quota_cpus": quota,
           "declared_share": os.environ.get("OMP_NUM_THREADS"),
           "sample": f"{procs} single-threaded processes (one per usable host core) x 1 env x ~{seconds:.0f}s "
                     f"of random-action {env_id} steps with TimeLimit+autoreset ({steps} env-steps total); "
                     "oracle/usv_oracle.py per-env float64 NumPy restatement of the reference step"}
    # per-core speed of this restatement relative to the reference itself, measured in the build
    # container (tools/calibrate_cpu.py; the reference does not exist on the GPU box)
    cal_p = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    if os.path.exists(cal_p):
        cal = json.load(open(cal_p)).get(env_id)
        if cal:
            ratio = cal["ratio_oracle_over_reference"]
            out["calibration"] = {"oracle_over_reference_per_core": ratio,
                                  "reference_equivalent_value": round(rate / ratio, 1),
                                  "source": "profiles/cpu_calibration.json (tools/calibrate_cpu.py)",
                                  "note": "reference timed without numba (not importable here), so its "
                                          "@njit lidar (usv_asmc_ca_env.py:439-440) ran as pure Python: "
                                          "reference_equivalent_value is a lower bound (unpinned)"}
    return out


# --------------------------------------------------------------------------- reference precision
def pmc_entry(path, key):
    """(traffic bytes per launch, SQ_INSTS_VALU per launch) of `key` in the committed PMC summary."""
    try:
        d = json.load(open(path)).get(key)
    except (OSError, ValueError):
        return None, None
    if not d:
        return None, None
    return d.get("hbm_bytes_per_launch"), d.get("sq_insts_valu_per_launch")


def f64_leg(args, N, rank, dev, stream, acts, pool):
    """The default float64 step kernel (the reference's precision) on the same env count and
    actions: env-steps/s and the roofline from one HIP event pair around --f64-steps back-to-back
    launches (after --warmup + 64 untimed ones)."""
    import ctypes
    import torch
    import gym_usv_amd
    env = gym_usv_amd.make_vec(args.env_id, N, device=dev.index, seed=args.seed, precision="f64",
                               lidar=args.lidar, env_id_offset=shard(rank, N)[0])
    env.reset(seed=args.seed)
    mean_obs = float(env.get_field("n_obs").mean())
    D = env.obs_dim
    obs = torch.empty((N, D), device=dev)
    fobs = torch.empty((N, D), device=dev)
    rew = torch.empty(N, device=dev, dtype=torch.float64)
    term = torch.empty(N, device=dev, dtype=torch.uint8)
    trunc = torch.empty(N, device=dev, dtype=torch.uint8)
    vp = ctypes.c_void_p
    outs = (vp(obs.data_ptr()), vp(rew.data_ptr()), vp(term.data_ptr()), vp(trunc.data_ptr()),
            vp(fobs.data_ptr()), vp(stream.cuda_stream))
    bound = [(env._h, vp(acts[i].data_ptr())) + outs for i in range(pool)]
    step_fn = env.lib.usv_step

    def launch(k):
        rc = step_fn(*bound[k % pool])
        if rc != 0:
            raise RuntimeError(env.lib.usv_last_error().decode())
    for k in range(args.warmup + 64):
        launch(k)
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record(stream)
    for k in range(args.f64_steps):
        launch(k)
    b.record(stream)
    b.synchronize()
    ms = a.elapsed_time(b) / args.f64_steps
    env.close()
    bpe = algorithmic_bytes_per_env_step(args.env_id, mean_obs, "f64")
    achieved = bpe * N / (ms * 1e-3) / 1e9
    traffic, valu = pmc_entry(args.pmc, f"{args.env_id}/{N}/f64/{args.lidar}")
    return {"dtype": "f64", "env_steps_per_s": round(N / (ms * 1e-3), 1), "kernel_ms": round(ms, 5),
            "launches": args.f64_steps, "mean_obstacles": round(mean_obs, 2),
            "algorithmic_bytes_per_env_step": round(bpe, 1), "achieved": round(achieved, 1),
            "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic,
            "valu_frac": (round(valu * VALU_CYCLES / (SIMDS * CLOCK_GHZ * 1e9 * ms * 1e-3), 4) if valu else None),
            "note": "the default float64 step kernel (the reference's arithmetic, bit-exact obs parity) on the "
                    "same env count and actions; one HIP event pair around that many launches, untimed by "
                    "the contract; traffic from profiles/pmc_summary.json"}


# --------------------------------------------------------------------------- launch
BACKEND = "nccl"            # RCCL on ROCm; tests/test_multirank.py runs the same ranks under gloo


def parse_args(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1,
                    help="ranks, one per GPU: under torch.distributed.run it must equal WORLD_SIZE; "
                         "without a launcher N > 1 starts N rank processes itself")
    ap.add_argument("--steps", type=int, default=10000)
    ap.add_argument("--warmup", type=int, default=200)
    ap.add_argument("--envs", type=int, default=65536, help="envs per GPU")
    ap.add_argument("--env-id", default="usv-simple", choices=["usv-simple", "usv-asmc-simple", *LEGACY_IDS])
    ap.add_argument("--precision", default="f32", choices=["f32", "f64"])
    ap.add_argument("--lidar", default="window", choices=["brute", "window"])
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--cpu-seconds", type=float, default=10.0)
    ap.add_argument("--cpu-procs", type=int, default=0, help="0 = every usable host core")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--event-every", type=int, default=16, help="launches per HIP-event-timed group (mid layout)")
    ap.add_argument("--event-layout", default="mid", choices=["edge", "mid"],
                    help="edge: one event pair around all K timed launches; mid: groups inside the loop")
    ap.add_argument("--pmc", default=os.path.join(ROOT, "profiles", "pmc_summary.json"))
    ap.add_argument("--clock-warmup", type=float, default=0.3,
                    help="untimed steps after --warmup until this many seconds have passed")
    ap.add_argument("--steady-steps", type=int, default=1000,
                    help="untimed launches after the timed region for roofline.steady (0 = skip)")
    ap.add_argument("--f64-steps", type=int, default=500,
                    help="launches of the f64 (reference-precision) leg after the timed region (0 = skip)")
    ap.add_argument("--api-steps", type=int, default=200, help="steps of the public-API leg (0 = skip)")
    ap.add_argument("--variant", default=None, help="step-kernel variant epb,lid,kind (tools; default: tuned)")
    return ap.parse_args(argv)


def resolve_world(gpus, environ, device_count):
    """How this process takes part, from --gpus and the launcher's environment:
      ("rank", world)  -- this process is one rank: WORLD_SIZE set by torch.distributed.run (or by
                          spawn_ranks) and equal to --gpus, or a plain single-GPU run;
      ("spawn", gpus)  -- --gpus N > 1 with no launcher: start N rank processes (spawn_ranks).
    Refuses (SystemExit with a message, exit status 1) a WORLD_SIZE that differs from --gpus, and
    --gpus N beyond the visible GPUs, so an N-GPU line is never measured on fewer GPUs.
    `device_count` is called only in the spawn case (torch.cuda.device_count() does not initialise
    the GPU, so the parent stays GPU-free before it starts its children)."""
    if gpus < 1:
        raise SystemExit(f"bench.py: --gpus must be >= 1, got {gpus}")
    ws = environ.get("WORLD_SIZE")
    if ws is not None:
        if int(ws) != gpus:
            raise SystemExit(f"bench.py: --gpus {gpus} but the launcher started WORLD_SIZE={ws} ranks; "
                             f"pass --gpus {ws} (or --nproc-per-node {gpus})")
        return "rank", int(ws)
    if gpus == 1:
        return "rank", 1
    have = int(device_count())
    if have < gpus:
        raise SystemExit(f"bench.py: --gpus {gpus} needs {gpus} visible GPUs, this node shows {have}; "
                         "refusing to report a smaller run as an N-GPU one")
    return "spawn", gpus


def _free_port():
    import socket
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    port = s.getsockname()[1]
    s.close()
    return port


def _rank_entry(rank, world, port, argv):
    """Body of one spawned rank: the environment torch.distributed.run would give it, then main()."""
    os.environ.update(RANK=str(rank), LOCAL_RANK=str(rank), WORLD_SIZE=str(world),
                      LOCAL_WORLD_SIZE=str(world), MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port),
                      USV_BENCH_LAUNCHER="bench.py spawn")
    main(argv)


def spawn_ranks(n, argv, target=_rank_entry, port=None):
    """Start n rank processes (multiprocessing "spawn": each child execs a fresh interpreter at once, so
    no rank inherits this process's state, and nothing is exec'd over this process, which has made no
    GPU call) and wait for them.  Returns 0, or the exit
    status of the first rank that fails, after terminating the others (a rank left waiting in a
    barrier for a dead peer would otherwise hang)."""
    from multiprocessing.connection import wait
    ctx = mp.get_context("spawn")
    port = port or _free_port()
    procs = [ctx.Process(target=target, args=(r, n, port, list(argv)), name=f"bench-rank{r}") for r in range(n)]
    rc, live = 0, []
    try:
        for p in procs:
            p.start()
            live.append(p)
        while live:
            wait([p.sentinel for p in live])
            for p in [p for p in live if not p.is_alive()]:
                p.join()
                live.remove(p)
                if p.exitcode != 0 and rc == 0:
                    rc = p.exitcode if p.exitcode > 0 else 1
                    print(f"bench.py: {p.name} exited with status {p.exitcode}; stopping the other ranks",
                          file=sys.stderr, flush=True)
                    for q in live:
                        q.terminate()
    finally:                       # (an interrupted parent leaves no rank behind)
        for q in live:
            q.terminate()
            q.join(30)
    return rc


def init_dist(local):
    """One process group over the ranks (BACKEND); the NCCL (RCCL) group is bound to this rank's GPU."""
    import torch
    import torch.distributed as dist
    if BACKEND == "nccl":
        torch.cuda.set_device(local)
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        dist.init_process_group(BACKEND)


# --------------------------------------------------------------------------- the timed workload
class _StreamEvent:
    """A HIP event recorded on the env's stream (torch.cuda.Event sees only what it is recorded on)."""

    def __init__(self, stream):
        import torch
        self.e, self.s = torch.cuda.Event(enable_timing=True), stream

    def record(self):
        self.e.record(self.s)

    def elapsed_time(self, other):
        return self.e.elapsed_time(other.e)

    def synchronize(self):
        self.e.synchronize()


class StepWorkload:
    """Config C3 on one rank: the vector env over this rank's shard of global env ids, the actions of
    every timed step resident in HBM, and the C-ABI step call with its arguments bound once per action
    buffer (usv_step, include/usv_hip.h), so the host path of a launch is one ctypes call."""

    def __init__(self, args, rank, local):
        import ctypes
        import torch
        import gym_usv_amd
        self.args, self.rank = args, rank
        dev = self.dev = torch.device("cuda", local)
        torch.cuda.set_device(dev)
        self.collective_device = dev
        N = self.N = args.envs
        env = self.env = gym_usv_amd.make_vec(args.env_id, N, device=local, seed=args.seed,
                                              precision=args.precision, lidar=args.lidar,
                                              env_id_offset=shard(rank, N)[0], kernel_variant=args.variant)
        env.reset(seed=args.seed)
        self.mean_obs = float(env.get_field("n_obs").mean())
        A, D = env.act_dim, env.obs_dim
        # actions for every timed step resident in HBM before timing (cycled pool if huge)
        pool = self.pool = max(1, min(args.steps, (8 << 30) // (N * 4 * A)))
        gen = torch.Generator(device=dev).manual_seed(args.seed * 7919 + rank)
        if A == 2:
            lo, span = torch.tensor([0.2, -1.0], device=dev), torch.tensor([0.8, 2.0], device=dev)
        else:                                   # legacy heading offset (usv_asmc_env.py:74-75)
            lo, span = torch.tensor([-math.pi / 2], device=dev), torch.tensor([math.pi], device=dev)
        self.acts = torch.rand((pool, N, A), device=dev, generator=gen) * span + lo
        self.obs = torch.empty((N, D), device=dev)
        self.fobs = torch.empty((N, D), device=dev)
        self.rew = torch.empty(N, device=dev, dtype=torch.float32 if args.precision == "f32" else torch.float64)
        self.term = torch.empty(N, device=dev, dtype=torch.uint8)
        self.trunc = torch.empty(N, device=dev, dtype=torch.uint8)
        self.stream = torch.cuda.current_stream(dev)
        vp = ctypes.c_void_p
        outs = (vp(self.obs.data_ptr()), vp(self.rew.data_ptr()), vp(self.term.data_ptr()),
                vp(self.trunc.data_ptr()), vp(self.fobs.data_ptr()), vp(self.stream.cuda_stream))
        self.bound = [(env._h, vp(self.acts[i].data_ptr())) + outs for i in range(pool)]
        self.step_fn = env.lib.usv_step

    def launch(self, k):
        rc = self.step_fn(*self.bound[k % self.pool])
        if rc != 0:
            raise RuntimeError(self.env.lib.usv_last_error().decode())

    def sync(self):
        import torch
        torch.cuda.synchronize(self.dev)

    def event(self):
        return _StreamEvent(self.stream)

    def extras(self):
        """The legs after the timed region, untimed by the contract: the f64 (reference-precision)
        kernel and the public-API step."""
        import torch
        args, env, N, pool, acts = self.args, self.env, self.N, self.pool, self.acts
        # the reference's precision (float64, simple_env.py:32-54) on the same workload: its own env
        # and the same launch path, one event pair around --f64-steps launches
        f64 = None
        if args.f64_steps > 0 and args.precision == "f32" and args.env_id not in LEGACY_IDS:
            f64 = f64_leg(args, N, self.rank, self.dev, self.stream, acts, pool)
        # public API leg: UsvVectorEnv.step on the same envs
        api = None
        if args.api_steps > 0:
            api = {}
            for copy in (True, False):
                env.copy = copy
                for k in range(8):
                    env.step(acts[k % pool])
                torch.cuda.synchronize(self.dev)
                t1 = time.perf_counter()
                for k in range(args.api_steps):
                    env.step(acts[k % pool])
                torch.cuda.synchronize(self.dev)
                dt = (time.perf_counter() - t1) / args.api_steps
                api["copy" if copy else "nocopy"] = {"env_steps_per_s": round(N / dt, 1),
                                                     "us_per_step": round(dt * 1e6, 2)}
            api["steps"] = args.api_steps
            api["note"] = ("UsvVectorEnv.step(actions) -> (obs, reward, terminated, truncated, info) with "
                           "torch tensors on the device; copy=True returns fresh tensors (gymnasium default), "
                           "copy=False the persistent buffers")
        return {"f64": f64, "api_step": api}

    def close(self):
        self.env.close()


# --------------------------------------------------------------------------- main
def run(args, rank, world, local, workload_cls=None):
    """One rank of the bench: warm-up, the timed window, the kernel timing, the max over ranks; rank 0
    returns (and prints) the JSON line, the other ranks return None."""
    import torch.distributed as dist
    if world > 1:
        init_dist(local)
    ranks_seen = dist.get_world_size() if dist.is_available() and dist.is_initialized() else 1
    wl = (workload_cls or StepWorkload)(args, rank, local)
    N, K, W = wl.N, args.steps, args.warmup
    launch = wl.launch

    for k in range(W):
        launch(k)
    # clock warm-up (untimed): keep stepping until the GPU has been busy for --clock-warmup seconds
    wl.sync()
    extra, tw = 0, time.perf_counter()
    while time.perf_counter() - tw < args.clock_warmup:
        for _ in range(64):
            launch(W + extra)
            extra += 1
        wl.sync()
    W2 = W + extra
    # HIP events on the env's stream bracket groups of G back-to-back launches (one event pair
    # per group; a pair around every single launch would add its own gap to each launch)
    # groups start after the first launch, so nothing but that launch sits between t0 and the GPU
    G = max(1, args.event_every)
    edge = args.event_layout == "edge"
    groups = 1 if edge else (K - 1) // G
    ev = [(wl.event(), wl.event()) for _ in range(groups)]
    for a, b in ev:                                   # the events exist before the timed region
        a.record()
        b.record()

    def timed_launch(k):
        if edge:
            # one timing marker before the first launch and one after the last: a marker between two
            # launches makes the second wait for the first's end-of-kernel release (tools/probe_wall.py)
            if k == 0:
                ev[0][0].record()
            launch(W2 + k)
            if k == K - 1:
                ev[0][1].record()
            return
        g, r = divmod(k - 1, G)
        if k > 0 and g < groups and r == 0:
            ev[g][0].record()
        launch(W2 + k)
        if k > 0 and g < groups and r == G - 1:
            ev[g][1].record()

    t0, t1 = timed_window(timed_launch, K, wl.sync, dist.barrier if world > 1 else (lambda: None))
    elapsed = t1 - t0
    if edge:
        kern_ms = ev[0][0].elapsed_time(ev[0][1]) / K
    else:
        kern_ms = (sum(a.elapsed_time(b) for a, b in ev) / (groups * G)) if groups else elapsed / K * 1e3
    # steady-state kernel time (after the timed region, untimed by the contract): one event pair
    # around --steady-steps more back-to-back launches, so the roofline is not read off a single
    # 16-launch group when the driver runs --steps 20
    steady_ms = None
    if args.steady_steps > 0:
        sa, sb = wl.event(), wl.event()
        sa.record()
        for k in range(args.steady_steps):
            launch(W2 + K + k)
        sb.record()
        sb.synchronize()
        steady_ms = sa.elapsed_time(sb) / args.steady_steps
    elapsed, kern_ms, steady_ms = reduce_max([elapsed, kern_ms, steady_ms or 0.0], device=wl.collective_device)
    legs = wl.extras()

    out = None
    if rank == 0:
        value = aggregate_rate(N, world, K, elapsed)
        bpe = algorithmic_bytes_per_env_step(args.env_id, wl.mean_obs, args.precision)
        bytes_per_launch = bpe * N
        achieved = bytes_per_launch / (kern_ms * 1e-3) / 1e9
        traffic, valu = pmc_entry(args.pmc, f"{args.env_id}/{N}/{args.precision}/{args.lidar}")
        valu_frac = None
        if valu:
            valu_frac = round(valu * VALU_CYCLES / (SIMDS * CLOCK_GHZ * 1e9 * kern_ms * 1e-3), 4)
        out = {
            "metric": METRIC, "value": round(value, 1), "unit": "env-steps/s", "n_gpus": world,
            "steps": K, "warmup": W, "clock_warmup_steps": extra, "ms_per_step": round(elapsed / K * 1e3, 5),
            "higher_is_better": True, "scaling": "weak", "vs_baseline": None, "ranks_seen": ranks_seen,
            "launcher": os.environ.get("USV_BENCH_LAUNCHER",
                                       "torch.distributed.run" if world > 1 or "TORCHELASTIC_RUN_ID" in os.environ
                                       else "single process"),
            "dtype": args.precision, "data": "synthetic (on-device uniform random actions, Philox env resets)",
            "config": {"workload": f"C3: {args.env_id}, {N} envs per GPU, random-action rollout, "
                                   f"in-kernel TimeLimit + same-step autoreset",
                       "env_id": args.env_id, "envs_per_gpu": N, "global_envs": N * world,
                       "parallelism": f"env-sharded x{world}, no step-path collective",
                       "lidar": args.lidar, "mean_obstacles": round(wl.mean_obs, 2)},
            "roofline": {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS,
                         "unit": "GB/s", "frac": round(achieved / HBM_PEAK_GBS, 4),
                         "traffic": traffic, "kernel_ms": round(kern_ms, 5),
                         "kernel_timing": ("HIP events around all K timed launches / K" if edge else
                                           f"HIP events around {groups} group(s) of {G} launches"),
                         "algorithmic_bytes_per_env_step": round(bpe, 1),
                         "valu_frac": valu_frac,
                         "steady": ({"kernel_ms": round(steady_ms, 5), "launches": args.steady_steps,
                                     "frac": round(bytes_per_launch / (steady_ms * 1e-3) / 1e9 / HBM_PEAK_GBS, 4),
                                     "timing": "one HIP event pair around that many back-to-back launches "
                                               "after the timed region"} if steady_ms else None),
                         "valu_basis": "SQ_INSTS_VALU per launch (profiles/pmc_summary.json) x 2 cycles / "
                                       "(1024 SIMDs x 2.4 GHz x kernel_ms)" if valu_frac is not None else None},
            "api_step": legs["api_step"],
            "f64": legs["f64"],
        }
        if args.env_id in LEGACY_IDS:
            out["config"].pop("lidar")
            out["config"].pop("mean_obstacles")
        if not args.no_cpu_baseline and world == 1:        # the CPU leg runs at N = 1 only
            cores, aff, quota = host_cores()
            out["cpu_baseline"] = cpu_baseline(args.env_id, args.cpu_seconds, args.cpu_procs or cores, aff, quota)
        else:
            out["cpu_baseline"] = None
        print(json.dumps(out), flush=True)
    wl.close()
    if world > 1:
        dist.destroy_process_group()
    return out


def main(argv=None):
    argv = sys.argv[1:] if argv is None else list(argv)
    args = parse_args(argv)

    def device_count():
        import torch
        return torch.cuda.device_count()
    mode, world = resolve_world(args.gpus, os.environ, device_count)
    if mode == "spawn":
        sys.exit(spawn_ranks(world, argv))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    run(args, rank, world, local)


if __name__ == "__main__":
    main()
