"""World-size-2 gloo test of the multi-GPU bench logic on CPU: disjoint payload
ranges per rank, barrier + max-over-ranks timing, whole-job aggregate, and the
per-rank work itself (checked with the CPU oracle as the stand-in compute, since
there is no GPU here).  The GPU run uses the same functions over RCCL."""
import os
import socket
import sys

import numpy as np
import pytest
import torch.multiprocessing as mp

ROOT = os.path.abspath(os.path.join(os.path.dirname(__file__), ".."))
sys.path[:0] = [ROOT, os.path.join(ROOT, "oracle"), os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python")]


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def _worker(rank, world, port, per_rank, q):
    import time

    import torch
    import torch.distributed as dist

    import bench
    import np_oracle
    from novelpoly_amd import synth

    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    lo, hi = bench.partition(per_rank, world, rank)
    orc = np_oracle.Oracle()
    n, k, plen = 16, 8, 600
    dist.barrier()
    t0 = time.perf_counter()
    ok = True
    for i in range(lo, hi):
        pl = synth.payload(i, plen)
        st, shards = orc.encode(pl, n, k, n)
        pres = synth.present_mask(i, n, 8)
        st2, rec = orc.reconstruct([s if pres[j] else None for j, s in enumerate(shards)], n, k)
        ok &= st == 0 and st2 == 0 and rec[:plen] == pl
    time.sleep(0.05 * (rank + 1))  # make the ranks' clocks differ
    mine = time.perf_counter() - t0
    dist.barrier()
    job = bench.max_over_ranks(mine, dist, torch.device("cpu"))
    q.put((rank, lo, hi, mine, job, ok, bench.aggregate_gib_s(world, per_rank, plen, job, 1)))
    dist.destroy_process_group()


def test_two_rank_weak_scaling_logic():
    world, per_rank = 2, 3
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_worker, args=(r, world, port, per_rank, q)) for r in range(world)]
    for p in procs:
        p.start()
    res = sorted(q.get(timeout=120) for _ in range(world))
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    ranges = [(r[1], r[2]) for r in res]
    assert ranges == [(0, 3), (3, 6)]  # disjoint, covering the global batch
    assert all(r[5] for r in res)  # every rank's payloads round-trip
    slowest = max(r[3] for r in res)
    for r in res:
        assert r[4] == pytest.approx(slowest)  # every rank reports the max
        assert r[6] == pytest.approx(world * per_rank * 600 / slowest / 2**30)


def test_partition_is_disjoint_and_complete():
    import bench

    for world in (1, 2, 4, 8):
        got = [bench.partition(1024, world, r) for r in range(world)]
        assert got[0][0] == 0 and got[-1][1] == 1024 * world
        assert all(a[1] == b[0] for a, b in zip(got, got[1:]))


def test_bench_gpus_flag_spawns_ranks():
    """`python bench.py --gpus 2` outside torchrun starts two ranks under
    torch.distributed.run (bench.launch_replicas); each takes a disjoint payload
    range and the job reports n_gpus = 2 (NP_BENCH_DRYRUN: gloo, no GPU)."""
    import json
    import subprocess

    env = dict(os.environ, NP_BENCH_DRYRUN="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "2", "--batch", "8"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert [tuple(x) for x in line["ranges"]] == [(0, 8), (8, 16)]


def test_bench_rejects_mismatched_world_size():
    import subprocess

    env = dict(os.environ, NP_BENCH_DRYRUN="1", WORLD_SIZE="1", RANK="0")
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8"], capture_output=True,
                       text=True, env=env, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr


def test_bench_labels_eight_gpus_as_config5():
    """`--gpus 8` at the default config is BASELINE config 5 (8192 payloads of
    1 MiB over 8 GPUs); its metric stays the headline one."""
    import json
    import subprocess

    import bench

    assert bench.workload_name(3, 8, 1024).startswith("BASELINE config 5")
    assert bench.workload_name(3, 1, 1024) == "BASELINE config 3"
    assert bench.metric_name(1024, 1 << 20) == bench.METRIC
    assert "n=4096 shards, 4 MiB msgs" in bench.metric_name(4096, 4 << 20)
    assert "n=256 shards, 64 KiB msgs" in bench.metric_name(256, 64 << 10)
    env = dict(os.environ, NP_BENCH_DRYRUN="1", OMP_NUM_THREADS="1")
    env.pop("WORLD_SIZE", None)
    r = subprocess.run([sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", "8", "--batch", "2"],
                       capture_output=True, text=True, env=env, timeout=300)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([ln for ln in r.stdout.splitlines() if ln.startswith("{")][-1])
    assert line["n_gpus"] == 8
    assert line["workload"].startswith("BASELINE config 5") and "16 payloads over 8 GPUs" in line["workload"]
    assert line["metric"] == bench.METRIC


def test_host_cores_reports_affinity_and_quota():
    import bench

    hc = bench.host_cores()
    assert hc["affinity"] >= 1 and 1 <= hc["used"] <= hc["affinity"]
    if hc["quota"] is not None:
        assert hc["used"] <= max(1, int(hc["quota"]))
