#!/usr/bin/env python3
"""Headline benchmark: payload GiB/s (device-resident) encode+reconstruct,
n=1024 shards, 1 MiB messages (BASELINE.json `metric`, config 3; config 5
is the same workload on 8 GPUs).

One step = encode a batch of payloads into n shards each, evaluate the
erasure locator of every payload, and reconstruct every payload from the
shards that survive a random erasure of 342 of them -- all on the GPU with
inputs already resident in HBM.  Payloads are independent, so N GPUs run N
replicas on disjoint payload sets (weak scaling, no data-path collective);
only the barrier and the max-over-ranks timing use torch.distributed.

Usage: python bench.py [--gpus N] [--steps K] [--warmup W]
       torchrun --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, os.path.join(ROOT, "reed-solomon-novelpoly_amd", "python"))

METRIC = "payload GiB/s (device-resident) encode+reconstruct, n=1024 shards, 1 MiB msgs"


def metric_name(n_wanted: int, payload: int) -> str:
    """BASELINE.json's metric for its headline shape (n = 1024 shards, 1 MiB
    payloads: configs 3 and 5); other shapes name their own (n, payload)."""
    if n_wanted == 1024 and payload == 1 << 20:
        return METRIC
    size = f"{payload >> 20} MiB" if payload % (1 << 20) == 0 else (
        f"{payload >> 10} KiB" if payload % 1024 == 0 else f"{payload} B")
    return f"payload GiB/s (device-resident) encode+reconstruct, n={n_wanted} shards, {size} msgs"


def workload_name(cfg_id, world: int, batch: int) -> str:
    """The BASELINE config a run measures: config 3 on N GPUs is config 5's
    workload (1 MiB x 1024 payloads per GPU, 8192 on 8 GPUs)."""
    if cfg_id in (3, 5) and world > 1:
        return f"BASELINE config 5 shape: {world * batch} payloads over {world} GPUs ({batch}/GPU)"
    return f"BASELINE config {cfg_id}"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md: HBM3E 8.0 TB/s spec


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=5)
    ap.add_argument("--config", type=int, default=3, help="BASELINE config id (workload shape)")
    ap.add_argument("--batch", type=int, default=0, help="payloads per GPU (default: the config's)")
    ap.add_argument("--cpu-seconds", type=float, default=10.0, help="CPU baseline budget (rank 0, N=1)")
    ap.add_argument("--no-cpu", action="store_true")
    ap.add_argument("--out", default="", help="also write the JSON line to this file")
    # ad-hoc shapes for DESIGN measurements (never the headline): override the config's
    ap.add_argument("--n-wanted", type=int, default=0)
    ap.add_argument("--k-wanted", type=int, default=0)
    ap.add_argument("--payload", type=int, default=0, help="payload bytes")
    ap.add_argument("--erase", type=int, default=-1, help="erasures per payload")
    return ap.parse_args()


def partition(per_rank: int, world: int, rank: int):
    """Payload index range of `rank` (weak scaling: every rank owns `per_rank`
    payloads of the global batch world * per_rank; ranges are disjoint)."""
    assert 0 <= rank < world
    return rank * per_rank, (rank + 1) * per_rank


def max_over_ranks(elapsed: float, dist, device) -> float:
    """The job's wall time: the slowest rank (no data-path collective exists;
    this scalar all-reduce is the only communication)."""
    import torch

    if not dist.is_available() or not dist.is_initialized() or dist.get_world_size() == 1:
        return elapsed
    t = torch.tensor([elapsed], dtype=torch.float64, device=device)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def aggregate_gib_s(world: int, per_rank: int, payload_len: int, elapsed: float, steps: int) -> float:
    """Whole-job payload GiB/s over all ranks."""
    return world * per_rank * payload_len / (elapsed / steps) / 2**30


# Profile tags, newest first: round 6's closing profiles (r06: configs 3, 4
# and 2), then round 4's (r04g: configs 3 and 4; r04: config 2).
ROUND_TAGS = ("r06", "r05", "r04g", "r04")


def load_traffic(config: int):
    """Per-launch HBM bytes (FETCH_SIZE + WRITE_SIZE, calibrated) of each kernel
    from the newest committed PMC summary of this round for this config
    (tools/profile_round.sh + tools/pmc_summary.py, measured on this same bench
    command: profiles/<tag>_pmc_summary.json for config 3, <tag>_cfg<c>_...
    else)."""
    for rt in ROUND_TAGS:
        tag = rt if config == 3 else f"{rt}_cfg{config}"
        p = os.path.join(ROOT, "profiles", f"{tag}_pmc_summary.json")
        if os.path.exists(p):
            with open(p) as f:
                summary = json.load(f)
            return {k: v.get("traffic_bytes") for k, v in summary.get("kernels", {}).items()}
    return {}


def host_cores():
    """The host cores this process may run on: its CPU affinity set, capped by
    the cgroup CPU quota where one is set (cpu.max: the lease's share of a
    larger machine).  The CPU baseline runs one thread per such core."""
    try:
        affinity = len(os.sched_getaffinity(0))
    except AttributeError:
        affinity = os.cpu_count() or 1
    quota = None
    for path in ("/sys/fs/cgroup/cpu.max", "/sys/fs/cgroup/cpu/cpu.cfs_quota_us"):
        try:
            with open(path) as f:
                parts = f.read().split()
        except OSError:
            continue
        if path.endswith("cpu.max") and parts and parts[0] != "max":
            quota = int(parts[0]) / int(parts[1])
        elif path.endswith("cfs_quota_us") and parts and int(parts[0]) > 0:
            with open("/sys/fs/cgroup/cpu/cpu.cfs_period_us") as f:
                quota = int(parts[0]) / int(f.read().split()[0])
        break
    used = affinity if quota is None else max(1, min(affinity, int(quota)))
    return {"affinity": affinity, "quota": quota, "used": used}


def cpu_baseline(cfg, params, seconds):
    """The reference's own C implementation (oracle/_ref/cpu_bench_ref, built from
    /root/reference by oracle/Makefile) -- or, where that build is absent, the C
    restatement (oracle/cpu_bench_port) -- on a bounded sample of the same
    workload: whole payloads encoded and reconstructed with the crate's glue
    (oracle/cpu_bench.c), one payload per host thread at a time, every
    reconstruction checked.  Timed on all host cores of this GPU's share and on
    one core."""
    import subprocess

    ref = os.path.join(ROOT, "oracle", "_ref", "cpu_bench_ref")
    port = os.path.join(ROOT, "oracle", "cpu_bench_port")
    exe = ref if os.path.exists(ref) else port
    if not os.path.exists(exe):
        raise RuntimeError("CPU baseline harness missing: run __graft_entry__.build()")
    hc = host_cores()
    threads = hc["used"]
    # OMP_NUM_THREADS caps it (16 on the GPU boxes, equal to their cgroup quota;
    # rounds 1-2 used min(affinity, OMP_NUM_THREADS, 16), round 3 the quota alone)
    omp = os.environ.get("OMP_NUM_THREADS", "")
    if omp.isdigit() and int(omp) > 0:
        threads = min(threads, int(omp))
    n, k, plen = params.n(), params.k(), cfg["payload"]
    erase = cfg["erase"] if cfg["erase"] is not None else n - k  # as the GPU workload (main)

    def run(t, secs):
        out = subprocess.run([exe, str(n), str(k), str(plen), str(erase), str(t), str(secs)],
                             check=True, capture_output=True, text=True, timeout=secs + 300)
        r = json.loads(out.stdout.strip().splitlines()[-1])
        assert r["failures"] == 0 and r["payloads"] > 0, r
        return r

    multi = run(threads, seconds)
    single = run(1, max(1.0, seconds / 3))
    return {
        "value": round(multi["gib_s"], 6),
        "unit": "GiB/s",
        "cores": threads,
        "omp_num_threads": omp or None,
        "cores_available": hc["affinity"],
        "cpu_quota": hc["quota"],
        "kind": multi["kind"],
        "single_core_value": round(single["gib_s"], 6),
        "sample": f"{multi['payloads']} payloads of config {cfg['id']} in {multi['seconds']:.1f}s on {threads} threads "
                  f"({hc['affinity']} cores in the affinity set, cgroup CPU quota {hc['quota']}) "
                  f"(+{single['payloads']} in {single['seconds']:.1f}s on 1 thread): encode + reconstruct with "
                  f"{erase} erasures, {'reference cxx/RSErasureCode.c' if multi['kind'] == 'reference' else 'oracle/np_oracle.c'} "
                  f"+ crate glue (oracle/cpu_bench.c), every payload round-trip checked",
    }


def launch_replicas(args) -> int:
    """`python bench.py --gpus N` (N > 1) outside torchrun: start N ranks under
    torch.distributed.run as a child process -- before this process touches the
    GPU -- and return its exit code.  Each rank then runs main() below."""
    import socket
    import subprocess

    with socket.socket() as so:
        so.bind(("127.0.0.1", 0))
        port = so.getsockname()[1]
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={args.gpus}",
           "--master-addr", "127.0.0.1", "--master-port", str(port), os.path.abspath(__file__)] + sys.argv[1:]
    env = dict(os.environ, HSA_ENABLE_IPC_MODE_LEGACY=os.environ.get("HSA_ENABLE_IPC_MODE_LEGACY", "0"))
    return subprocess.run(cmd, env=env).returncode


def dry_run(args):
    """NP_BENCH_DRYRUN=1 (CPU tests): the launch and partition logic without a
    GPU -- each rank joins a gloo group, takes its payload range and rank 0
    prints the ranges of every rank with n_gpus."""
    import torch
    import torch.distributed as dist

    from novelpoly_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    batch = args.batch or (synth.CONFIGS[args.config]["batch"] if args.config != 5 else
                           synth.CONFIGS[5]["batch"] // 8)
    lo, hi = partition(batch, world, rank)
    ranges = [(lo, hi)]
    if world > 1:
        dist.init_process_group("gloo")
        t = torch.tensor([lo, hi], dtype=torch.int64)
        out = [torch.zeros(2, dtype=torch.int64) for _ in range(world)]
        dist.all_gather(out, t)
        ranges = [tuple(int(v) for v in o) for o in out]
        dist.destroy_process_group()
    if rank == 0:
        cfg = synth.CONFIGS[args.config]
        print(json.dumps({"dry_run": True, "n_gpus": world, "ranges": ranges, "batch_per_gpu": batch,
                          "metric": metric_name(cfg["n_wanted"], cfg["payload"]),
                          "workload": workload_name(args.config, world, batch)}), flush=True)


def main():
    args = parse()
    world_env = os.environ.get("WORLD_SIZE")
    if world_env is None and args.gpus > 1:
        sys.exit(launch_replicas(args))
    if world_env is not None and int(world_env) != args.gpus:
        sys.exit(f"bench.py: --gpus {args.gpus} but WORLD_SIZE={world_env}; launch one rank per GPU")
    if os.environ.get("NP_BENCH_DRYRUN"):
        return dry_run(args)
    import torch
    import torch.distributed as dist

    import novelpoly_amd as npa
    from novelpoly_amd import synth

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world > 1:
        dist.init_process_group("nccl", device_id=torch.device("cuda", local))
    torch.cuda.set_device(local)
    dev = torch.device("cuda", local)
    # a dedicated stream: kernels, events and torch copies share one queue
    torch.cuda.set_stream(torch.cuda.Stream(dev))

    cfg = dict(synth.CONFIGS[args.config])
    cfg["id"] = args.config
    if args.n_wanted or args.k_wanted or args.payload or args.erase >= 0:  # ad-hoc shape
        cfg["id"] = f"{args.config}+override"
        cfg["n_wanted"] = args.n_wanted or cfg["n_wanted"]
        cfg["k_wanted"] = args.k_wanted or npa.recoverablity_subset_size(cfg["n_wanted"])
        cfg["payload"] = args.payload or cfg["payload"]
        if args.erase >= 0:
            cfg["erase"] = args.erase
    params = npa.CodeParams.derive_parameters(cfg["n_wanted"], cfg["k_wanted"])
    n, k = params.n(), params.k()
    batch = args.batch or (cfg["batch"] if args.config != 5 else cfg["batch"] // 8)
    plen = cfg["payload"]
    erase = cfg["erase"] if cfg["erase"] is not None else n - k
    ctx = npa.Context(local)
    rs = params.make_encoder(ctx)
    sl = rs.shard_len(plen)
    out_len = (sl // 2) * 2 * k
    lo, hi = partition(batch, world, rank)

    # SURVEY.md §8(d) synthetic inputs: payload i = splitmix64 stream with seed
    # 0x5EED_0000 + i (global payload index), erasures by partial Fisher-Yates
    # with seed 0xE7A5_0000 + i
    payloads = synth.payload_batch_dev(lo, hi, plen, dev)
    shards = torch.empty((batch, n, sl), dtype=torch.uint8, device=dev)
    np_ = __import__("numpy")
    wn = params.wanted_n  # rows >= wanted_n are never produced: absent (BASELINE configs: wanted_n == n)
    pres_np = np_.zeros((hi - lo, n), np_.uint8)
    for i in range(lo, hi):
        pres_np[i - lo, :wn] = synth.present_mask(i, wn, erase)
    present_h = torch.from_numpy(pres_np)
    present = present_h.to(dev)
    out = torch.empty((batch, out_len), dtype=torch.uint8, device=dev)
    stream = torch.cuda.current_stream(dev)
    sptr = stream.cuda_stream

    ev = {name: [] for name in ("encode", "reconstruct")}

    def step(record):
        # encode, then reconstruct with the erasure locators computed on the
        # device (d_locators = NULL: fused into the fast reconstruct kernel)
        if record:
            e = [torch.cuda.Event(enable_timing=True) for _ in range(3)]
            e[0].record(stream)
        npa.encode_batch_dev(params, payloads.data_ptr(), plen, plen, batch, shards.data_ptr(), n * sl, ctx=ctx,
                             stream=sptr)
        if record:
            e[1].record(stream)
        npa.reconstruct_batch_dev2(params, shards.data_ptr(), sl, n * sl, present.data_ptr(), 0, batch,
                                   out.data_ptr(), out_len, ctx=ctx, stream=sptr)
        if record:
            e[2].record(stream)
            ev["encode"].append((e[0], e[1]))
            ev["reconstruct"].append((e[1], e[2]))

    for _ in range(args.warmup):
        step(False)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(args.steps):
        step(True)
    torch.cuda.synchronize(dev)
    if world > 1:
        dist.barrier()
    torch.cuda.synchronize(dev)
    elapsed = max_over_ranks(time.perf_counter() - t0, dist, dev)

    # correctness guard on the measured buffers: every payload round-trips
    ok = bool(torch.equal(out[:, :plen], payloads))

    ms_step = elapsed / args.steps * 1e3
    value = aggregate_gib_s(world, batch, plen, elapsed, args.steps)

    kt = {name: sum(a.elapsed_time(b) for a, b in pairs) / len(pairs) for name, pairs in ev.items()}
    nshard = params.wanted_n  # == n for the BASELINE configs
    # SURVEY.md §8(d) algorithmic bytes per payload: encode = P + n * shard_len;
    # reconstruct = present * shard_len + (shard_len / 2) * 2k (every present
    # row is read: the reference decodes from all of them)
    present_rows = int(present_h.sum())
    algo = {
        "encode": batch * (plen + nshard * sl),
        # + the present mask (batch x n bytes) the locator reads
        "reconstruct": present_rows * sl + batch * out_len + batch * n,
    }
    # the committed PMC summaries were measured at each config's BASELINE batch:
    # other batches report traffic null
    traffic = load_traffic(args.config) if batch == cfg["batch"] and cfg["id"] == args.config else {}
    roof = {}
    for name in kt:
        achieved = algo[name] / (kt[name] / 1e3) / 1e9
        roof[name] = {"bound": "hbm", "achieved": round(achieved, 2), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                      "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic.get(name),
                      "ms": round(kt[name], 4), "algorithmic_bytes": algo[name]}
    dominant = max(kt, key=kt.get)

    line = {
        "metric": metric_name(cfg["n_wanted"], plen),
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u16",
        "data": "synthetic",
        "config": {"workload": f"{workload_name(cfg['id'], world, batch)}: n_wanted={cfg['n_wanted']} "
                               f"k_wanted={cfg['k_wanted']} (effective n={n}, k={k}), {plen} B payloads, "
                               f"batch {batch}/GPU, encode + error locator + reconstruct with {erase} "
                               f"random erasures per payload",
                   "n": n, "k": k, "payload_bytes": plen, "batch_per_gpu": batch, "global_batch": world * batch,
                   "erasures": erase, "parallelism": f"replicas x{world} (no collective)",
                   "fast_path": params.is_faster8()},
        "roofline": dict(roof[dominant], kernel=dominant),
        "kernels": roof,
        "roundtrip_ok": ok,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        line["cpu_baseline"] = cpu_baseline(cfg, params, args.cpu_seconds)
    if rank == 0:
        s = json.dumps(line)
        print(s, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                f.write(s + "\n")
    if world > 1:
        dist.destroy_process_group()
    if not ok:
        sys.exit(3)


if __name__ == "__main__":
    main()
