"""World-size-2 gloo test of the multi-GPU bench plumbing on CPU: env sharding by global id,
max-over-ranks timing and the whole-job rate (bench.py)."""
import os
import socket

import pytest
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    lo, hi = bench.shard(rank, 1000)
    # each rank reports a different elapsed; every rank must see the max
    el, km = bench.reduce_max([1.0 + rank, 0.5 * (rank + 1)])
    rate = bench.aggregate_rate(1000, world, 10, el)
    q.put((rank, lo, hi, el, km, rate))
    dist.barrier()
    dist.destroy_process_group()


def test_two_rank_gloo_sharding_and_timing():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    assert [(r[1], r[2]) for r in res] == [(0, 1000), (1000, 2000)]     # disjoint, contiguous shards
    for r in res:
        assert r[3] == 2.0 and r[4] == 1.0                                # max over ranks
        assert r[5] == pytest.approx(1000 * 2 * 10 / 2.0)                 # all ranks' env-steps / slowest


def _window_worker(rank, world, port, q):
    """bench.timed_window under gloo with every torch.distributed collective wrapped by a counter
    that stamps perf_counter(): none may fall inside [t0, t1]."""
    import time
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    import bench
    calls = []
    names = ("barrier", "all_reduce", "all_gather", "broadcast", "reduce", "all_gather_object",
             "all_to_all", "reduce_scatter", "gather", "scatter", "monitored_barrier")
    orig = {n: getattr(dist, n) for n in names if hasattr(dist, n)}

    def wrap(n, f):
        def g(*a, **k):
            calls.append((n, time.perf_counter()))
            return f(*a, **k)
        return g
    for n, f in orig.items():
        setattr(dist, n, wrap(n, f))
    launches = []

    def launch(k):
        launches.append(time.perf_counter())
        time.sleep(0.002 * (1 + rank))          # ranks of different speed
    try:
        t0, t1 = bench.timed_window(launch, 5, lambda: None, dist.barrier)
        el, = bench.reduce_max([t1 - t0])
    finally:
        for n, f in orig.items():
            setattr(dist, n, f)
    inside = [c for c in calls if t0 <= c[1] <= t1]
    q.put((rank, len(launches), inside, [c[0] for c in calls], t1 - t0, el))
    dist.destroy_process_group()


def test_timed_window_is_collective_free():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_window_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(60)
        assert p.exitcode == 0
    for rank, nl, inside, names, mine, el in res:
        assert nl == 5
        assert inside == [], f"rank {rank}: collectives inside the timed window: {inside}"
        assert names.count("barrier") == 2 and "all_reduce" in names   # before t0, after t1, the max
        assert el == pytest.approx(max(r[4] for r in res))


def test_committed_counters_cover_the_driver_line():
    """The driver's bench line reads roofline.traffic / valu_frac for the headline workload and the
    f64 leg from profiles/pmc_summary.json: both keys exist there with per-launch bytes above the
    algorithmic bytes (counter-backed traffic, not a model)."""
    import json
    import os
    import bench
    pmc = os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "profiles", "pmc_summary.json")
    for prec in ("f32", "f64"):
        traffic, valu = bench.pmc_entry(pmc, f"usv-simple/65536/{prec}/window")
        assert traffic and valu, prec
        algo = bench.algorithmic_bytes_per_env_step("usv-simple", 21.9, prec) * 65536
        assert 1.0 <= traffic / algo < 1.6, (prec, traffic / algo)
    for key in ("usv-asmc-simple/65536/f32/window", "usv-asmc-simple/65536/f64/window",
                "usv-simple/524288/f32/window"):
        assert all(bench.pmc_entry(pmc, key)), key
    assert bench.pmc_entry(pmc, "no/such/key") == (None, None)
    assert json.load(open(pmc))["usv-simple/65536/f32/window"]["round"].startswith("r06")


# --------------------------------------------------------------------------- bench.py --gpus N launcher
class _WallEvent:
    def record(self):
        import time
        self.t = time.perf_counter()

    def elapsed_time(self, other):
        return (other.t - self.t) * 1e3

    def synchronize(self):
        pass


class _StubWorkload:
    """CPU stand-in for bench.StepWorkload (same interface): launches sleep, events read the wall clock,
    and close() reports what the rank saw to $USV_TEST_OUT/rank<r>.json."""

    def __init__(self, args, rank, local):
        import bench
        self.N, self.rank, self.local, self.mean_obs = args.envs, rank, local, 20.0
        self.collective_device = None
        self.lo, self.hi = bench.shard(rank, self.N)
        self.launches = 0

    def launch(self, k):
        import time
        self.launches += 1
        time.sleep(0.0005 * (1 + self.rank))

    def sync(self):
        pass

    def event(self):
        return _WallEvent()

    def extras(self):
        return {"f64": None, "api_step": None}

    def close(self):
        import json
        self.report = {"rank": self.rank, "local": self.local, "lo": self.lo, "hi": self.hi,
                       "launches": self.launches, "world": dist.get_world_size()}


def _stub_rank(rank, world, port, argv):
    """bench._rank_entry with the CPU workload, gloo, and every collective timestamped."""
    import json
    import time
    import bench
    bench.BACKEND = "gloo"
    bench.StepWorkload = _StubWorkload
    calls, win, wls = [], {}, []
    names = ("barrier", "all_reduce", "all_gather", "broadcast", "reduce", "all_to_all", "reduce_scatter")
    for n in names:
        f = getattr(dist, n)
        setattr(dist, n, (lambda n, f: lambda *a, **k: (calls.append((n, time.perf_counter())), f(*a, **k))[1])(n, f))
    orig_tw = bench.timed_window

    def tw(*a, **k):
        win["t"] = orig_tw(*a, **k)
        return win["t"]
    bench.timed_window = tw
    orig_close = _StubWorkload.close

    def close(self):
        orig_close(self)
        wls.append(self.report)
    _StubWorkload.close = close
    bench._rank_entry(rank, world, port, argv)
    t0, t1 = win["t"]
    rep = dict(wls[0], inside=[c for c in calls if t0 <= c[1] <= t1], n_calls=len(calls),
               env_rank=os.environ["RANK"], env_world=os.environ["WORLD_SIZE"])
    with open(os.path.join(os.environ["USV_TEST_OUT"], f"rank{rank}.json"), "w") as f:
        json.dump(rep, f)


def test_bench_gpus_n_spawns_n_ranks(tmp_path, monkeypatch, capfd):
    """bench.py --gpus 2 without a launcher: two rank processes start (spawn_ranks), own disjoint
    shards, form a 2-rank group (ranks_seen 2, n_gpus 2), time a collective-free window, and only
    rank 0 prints the line."""
    import json
    import bench
    monkeypatch.setenv("USV_TEST_OUT", str(tmp_path))
    argv = ["--gpus", "2", "--steps", "5", "--warmup", "2", "--envs", "1000", "--clock-warmup", "0",
            "--steady-steps", "0", "--no-cpu-baseline", "--event-every", "2"]
    mode, world = bench.resolve_world(2, {}, lambda: 2)
    assert (mode, world) == ("spawn", 2)
    assert bench.spawn_ranks(world, argv, target=_stub_rank) == 0
    reps = [json.load(open(tmp_path / f"rank{r}.json")) for r in range(2)]
    assert [(r["lo"], r["hi"]) for r in reps] == [(0, 1000), (1000, 2000)]
    assert [r["local"] for r in reps] == [0, 1] and all(r["world"] == 2 for r in reps)
    assert [(r["env_rank"], r["env_world"]) for r in reps] == [("0", "2"), ("1", "2")]
    for r in reps:
        assert r["launches"] == 2 + 5
        assert r["inside"] == [], r["inside"]
        assert r["n_calls"] >= 3                # barrier before t0, barrier after t1, the max
    lines = [ln for ln in capfd.readouterr().out.splitlines() if ln.startswith("{")]
    assert len(lines) == 1
    line = json.loads(lines[0])
    assert line["n_gpus"] == 2 and line["ranks_seen"] == 2 and line["launcher"] == "bench.py spawn"
    assert line["config"]["global_envs"] == 2000 and line["scaling"] == "weak"
    # whole-job rate: both ranks' env-steps over the slower rank's window
    assert line["value"] == pytest.approx(2 * 1000 * 5 / (line["ms_per_step"] * 5 / 1e3), rel=1e-3)


def _failing_rank(rank, world, port, argv):
    import sys
    import time
    if rank == 1:
        sys.exit(3)
    time.sleep(600)                             # a rank that would wait forever for its dead peer


def test_spawn_ranks_stops_on_a_failed_rank():
    import time
    import bench
    t = time.perf_counter()
    assert bench.spawn_ranks(2, [], target=_failing_rank) == 3
    assert time.perf_counter() - t < 120


def test_bench_gpus_refusals():
    """--gpus N is never silently fewer GPUs: beyond the visible count, or != the launcher's
    WORLD_SIZE, bench.py exits non-zero with a message before touching a GPU."""
    import subprocess
    import sys
    import bench
    assert bench.resolve_world(1, {}, lambda: 0) == ("rank", 1)
    assert bench.resolve_world(4, {"WORLD_SIZE": "4"}, lambda: 0) == ("rank", 4)
    with pytest.raises(SystemExit, match="needs 8 visible GPUs, this node shows 1"):
        bench.resolve_world(8, {}, lambda: 1)
    with pytest.raises(SystemExit, match="WORLD_SIZE=2"):
        bench.resolve_world(4, {"WORLD_SIZE": "2"}, lambda: 8)
    with pytest.raises(SystemExit):
        bench.resolve_world(0, {}, lambda: 8)
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--steps", "3"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 1 and "needs 2 visible GPUs" in p.stderr and p.stdout == ""
    env["WORLD_SIZE"] = "2"
    p = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "1"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert p.returncode == 1 and "WORLD_SIZE=2" in p.stderr and p.stdout == ""
