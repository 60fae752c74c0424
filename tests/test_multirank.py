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
    assert json.load(open(pmc))["usv-simple/65536/f32/window"]["round"].startswith("r05")
