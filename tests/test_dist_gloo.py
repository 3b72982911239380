"""Multi-GPU path on CPU: world_size-2 gloo ranks run bench.py's sharding and
timing reduction.  Streams partition across ranks with no data-path
collective; the only exchange is the max over ranks of the
timed region."""
import os
import socket

import pytest
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, q):
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    import torch
    import torch.distributed as dist
    import bench
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    seeds = bench.shard_seeds(rank, 8)
    gathered = [None] * world
    dist.all_gather_object(gathered, seeds)
    t = bench.max_over_ranks(dist, torch, 1.0 + rank)
    dist.barrier()
    dist.destroy_process_group()
    q.put((rank, gathered, t))


@pytest.mark.timeout(120)
def test_two_rank_sharding_and_max():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = [q.get(timeout=100) for _ in range(world)]
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    for rank, gathered, t in res:
        assert t == 2.0                              # max over ranks
        flat = [s for g in gathered for s in g]
        assert len(flat) == len(set(flat)) == 16     # disjoint stream sets
        assert sorted(flat) == list(range(100, 116))  # config 4: seeds 100.. 8 per GPU


def _bench_worker(rank, world, port, q, one_device=False):
    """One rank of `bench.py --gpus 2 --dry-run` (torch.distributed.run's
    environment): sharding, host parse, warmup + timed step loop, the
    max-over-ranks timing and the summed verification counts, no device."""
    import contextlib
    import io
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    sys.path.insert(0, root)
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port), RANK=str(rank), LOCAL_RANK=str(rank),
                      WORLD_SIZE=str(world))
    if one_device:
        os.environ["BENCH_ONE_DEVICE"] = "1"
    import bench
    out = io.StringIO()
    with contextlib.redirect_stdout(out):
        bench.main(["--gpus", str(world), "--dry-run", "--streams", "2", "--warmup", "1", "--steps", "3",
                    "--config", "2", "--gen", "w_mbs=6,h_mbs=4,crop_bottom=0"])
    q.put((rank, out.getvalue()))


@pytest.mark.timeout(180)
def test_bench_dry_run_two_ranks():
    import json
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=160) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    assert res[1].strip() == ""                      # only rank 0 prints
    line = json.loads(res[0].strip().splitlines()[-1])
    assert line["n_gpus"] == 2 and line["steps"] == 3 and line["warmup"] == 1
    assert line["config"]["total_streams"] == 4 and line["config"]["seeds"] == "100..103"
    # GOP phases 0 and 30 of the 60-picture streams (three steps per launch):
    # 30 pre-roll launches + 1 warmup step + the 3 timed ones as one launch,
    # then the aligned P-only leg (3 pre-roll + 1 warmup step + a triple)
    assert line["dry_run"]["preroll_launches"] == 30 and line["dry_run"]["seeds"] == [100, 101]
    assert line["dry_run"]["launches"] == 30 + 1 + 1 + 3 + 1 + 1
    assert line["kernels"]["k_wgpp"]["trace_steps"] == [3]
    assert line["value"] > 0 and line["scaling"] == "weak"
    assert line["bitexact_check"]["frames_expected"] == 2 * 2 * 4
    assert line["p_only"]["i_pictures_timed"] == 0
    # every rank's record, coefficient and descriptor buffers on its own GPU
    # (rank r -> LOCAL_RANK r), allocated through its engine
    place = {p["rank"]: p for p in line["device_placement"]}
    assert sorted(place) == [0, 1]
    for r in (0, 1):
        assert place[r]["device"] == r
        assert [d for _, d in place[r]["buffers"]] == [r, r, r]
    # the end-to-end drop-in leg of every rank: its own GPU and a host-core
    # share disjoint from every other rank's
    import bench
    plan = {p["rank"]: p for p in line["end_to_end_plan"]}
    assert sorted(plan) == [0, 1]
    cores = {r: set(bench.parse_cpulist(plan[r]["cpus"])) for r in (0, 1)}
    for r in (0, 1):
        assert plan[r]["device"] == r
        assert cores[r] and len(cores[r]) == plan[r]["host_cores"]
        assert cores[r] <= os.sched_getaffinity(0)
    assert not cores[0] & cores[1]


@pytest.mark.timeout(180)
def test_bench_one_device_rehearsal_disjoint_cores():
    """BENCH_ONE_DEVICE=1 (the N-rank rehearsal on one GPU): every rank's GPU
    is device 0, but each rank still pins its end-to-end decoder processes to
    its own disjoint share of that device's host cores."""
    import json
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_bench_worker, args=(r, world, port, q, True)) for r in range(world)]
    for p in procs:
        p.start()
    res = dict(q.get(timeout=160) for _ in range(world))
    for p in procs:
        p.join(timeout=30)
        assert p.exitcode == 0
    line = json.loads(res[0].strip().splitlines()[-1])
    plan = {p["rank"]: p for p in line["end_to_end_plan"]}
    assert sorted(plan) == [0, 1]
    assert all(plan[r]["device"] == 0 for r in (0, 1))
    cores = {r: set(bench.parse_cpulist(plan[r]["cpus"])) for r in (0, 1)}
    assert cores[0] and cores[1] and not cores[0] & cores[1]


def test_e2e_core_plan_numa():
    """Ranks whose GPUs share a NUMA node split that node's cores; a node
    with no usable cores falls back to an equal share of all allowed cores."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    assert bench.parse_cpulist("0-3,8,10-11") == [0, 1, 2, 3, 8, 10, 11]
    assert bench.format_cpulist([11, 0, 1, 2, 3, 8, 10]) == "0-3,8,10-11"
    allowed = list(range(16))
    mine, plan = bench.e2e_core_plan(1, [-1, -1, -1, -1], allowed)
    assert mine == [4, 5, 6, 7] and len(plan) == 4
    assert sorted(c for p in plan for c in p) == allowed
    # a NUMA node the sysfs does not know: the fallback
    mine, plan = bench.e2e_core_plan(0, [99, 99], allowed)
    assert mine == list(range(8)) and plan[1] == list(range(8, 16))


def test_e2e_process_cpus_one_l3_each(monkeypatch):
    """End-to-end decoder processes: one L3 domain (CCD) each when the share
    has one per process, round-robin in order; otherwise the whole share."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    share = list(range(64))
    monkeypatch.setattr(bench, "l3_groups", lambda cpus: [list(range(k, k + 8)) for k in range(0, 64, 8)])
    per = bench.process_cpus(share, 8)
    assert per == [list(range(k, k + 8)) for k in range(0, 64, 8)]
    assert bench.process_cpus(share, 4) == per[:4]
    monkeypatch.setattr(bench, "l3_groups", lambda cpus: [sorted(cpus)])
    assert bench.process_cpus(share, 8) == [share] * 8
    # this container's real sysfs: every group lies inside the share
    monkeypatch.undo()
    allowed = sorted(os.sched_getaffinity(0))
    for g in bench.l3_groups(allowed):
        assert g and set(g) <= set(allowed)


def test_bench_gpus_mismatch_refused(monkeypatch):
    """--gpus N inside a torch.distributed environment of another size fails
    loudly instead of reporting the wrong n_gpus."""
    import sys
    sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
    import bench
    monkeypatch.setenv("WORLD_SIZE", "1")
    with pytest.raises(SystemExit):
        bench.dist_setup(8)
