"""bench.py — device-resident SST block encode + bloom build, 64 MiB sorted KV per SST.

Metric (BASELINE.json): GiB/s of logical KV bytes Σ(|key|+|value|) encoded per second, whole job,
inputs resident in HBM when the timed region starts.  One step = every rank encodes one complete
64 MiB D1 SST (configs[1]: 578,524 entries of 16 B keys / 100 B values -> 17,016 V2 blocks with
CRC32 + a 10 bits/key bloom) through the C ABI (sdb_encode_sst).  Ranks encode independent SSTs
(the compaction sharding of configs[4]); no collective is on the data path — the only RCCL calls
are the timing barrier and the max-over-ranks of the elapsed time.

  python bench.py [--gpus N --steps K --warmup W]
  python -m torch.distributed.run --nproc-per-node N bench.py --gpus N ...
"""
import argparse
import ctypes as C
import json
import os
import subprocess
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.abspath(__file__))
sys.path.insert(0, ROOT)

from slatedb_amd import _abi, datasets, runtime  # noqa: E402

PEAK_HBM_GBS = 8000.0  # MI355X HBM3E spec (MI355X_MICROARCH.md: 8.0 TB/s)


def parse():
    p = argparse.ArgumentParser()
    p.add_argument("--gpus", type=int, default=1)
    p.add_argument("--steps", type=int, default=20)
    p.add_argument("--warmup", type=int, default=5)
    p.add_argument("--ssts", type=int, default=4, help="distinct resident input SSTs per rank (rotated)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="budget of the CPU baseline sample")
    p.add_argument("--cpu-threads", type=int, default=0, help="CPU baseline threads (0: min(16, cpus))")
    p.add_argument("--no-cpu", action="store_true")
    p.add_argument("--no-verify", action="store_true")
    p.add_argument("--bpk", type=int, default=10, help="bloom bits per key (0 = no filter; diagnostics)")
    return p.parse_args()


def cpu_baseline(budget_s, threads):
    """The oracle (C restatement of EncodedSsTableBuilder + BloomFilterBuilder, oracle/sdb_oracle.c)
    encoding whole D1 SSTs: once on 1 thread, then on `threads` threads with one SST per thread (the
    l0_flush_parallelism / subcompaction shape).  ctypes releases the GIL during the
    C call, so the threads run in parallel."""
    import threading
    from oracle import oracle as O
    prm = O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    logical = None

    def run(batch, deadline, out, i):
        done, t_used = 0, 0.0
        while True:
            t0 = time.perf_counter()
            r = O.encode_sst(batch, prm)
            t_used += time.perf_counter() - t0
            assert r.status == 0
            done += 1
            if time.perf_counter() >= deadline:
                break
        out[i] = (done, t_used)

    # 1 thread
    b0 = datasets.d1(sst_index=9000)
    logical = b0.logical_bytes()
    out1 = [None]
    run(b0, time.perf_counter() + budget_s / 2, out1, 0)
    single = out1[0][0] * logical / out1[0][1] / 2**30
    # T threads, one SST each
    batches = [b0] + [datasets.d1(sst_index=9001 + i) for i in range(threads - 1)]
    outs = [None] * threads
    t0 = time.perf_counter()
    deadline = t0 + budget_s / 2
    ths = [threading.Thread(target=run, args=(batches[i], deadline, outs, i)) for i in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    wall = time.perf_counter() - t0
    multi = sum(o[0] for o in outs) * logical / wall / 2**30
    try:
        model = [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        model = "unknown"
    return {"value": round(multi, 4), "unit": "GiB/s", "cores": threads, "kind": "port",
            "single_thread_value": round(single, 4),
            "sample": "whole D1 SSTs (64 MiB logical KV each, encode + 10 bits/key bloom) by "
                      "oracle/sdb_oracle.c: %d SSTs on 1 thread (%.1f s), then %d threads x 1 SST each "
                      "for %.1f s wall (%d SSTs), on %s" % (out1[0][0], out1[0][1], threads, wall,
                                                          sum(o[0] for o in outs), model)}


def pmc_traffic(kernel):
    """HBM bytes per launch of `kernel` from the committed PMC passes over this same bench command
    (profiles/r1_pmc_traffic.json, written by scripts/collect_profiles.py; FETCH_SIZE/WRITE_SIZE
    corrected per MI355X_MICROARCH.md).  PMC counters cannot be read from inside the timed run."""
    try:
        d = json.load(open(os.path.join(ROOT, "profiles", "r1_pmc_traffic.json")))
        return d["per_dispatch"][kernel]["traffic_bytes"]
    except (OSError, KeyError, ValueError):
        return None


def main():
    args = parse()
    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    dist = world > 1
    if dist:
        import torch.distributed as tdist
        torch.cuda.set_device(local)
        tdist.init_process_group("nccl", device_id=torch.device("cuda", local))
    else:
        torch.cuda.set_device(0)
    dev = torch.device("cuda", torch.cuda.current_device())
    runtime.require_device()
    lib = runtime.lib()
    prm = runtime.params(block_size=4096, sst_version=2, restart_interval=16, bloom_bits_per_key=args.bpk)

    # resident inputs: distinct D1 SSTs per rank
    hosts = [datasets.d1(sst_index=rank * 64 + j) for j in range(args.ssts)]
    dbs = [h.to_device(dev) for h in hosts]
    logical = hosts[0].logical_bytes()
    outs = [runtime.DeviceSstOutput(hosts[0].n, logical, logical, prm, device=dev) for _ in range(2)]
    stream = torch.cuda.Stream(device=dev)

    def step(i):
        runtime.encode_sst_device(dbs[i % len(dbs)], outs[i % 2], stream)

    with torch.cuda.stream(stream):
        for i in range(args.warmup):
            step(i)
    torch.cuda.synchronize()

    # verify one SST against the oracle (bit-exact) before timing
    verified = None
    if not args.no_verify:
        step(0)
        torch.cuda.synchronize()
        got = outs[0].to_host()
        sm = got["summary"]
        assert sm.status == 0, "encode failed: %s" % _abi.STATUS_NAMES.get(sm.status)
        if rank == 0:
            from oracle import oracle as O
            ref = O.encode_sst(hosts[0], O.params(block_size=4096, sst_version=2, bloom_bits_per_key=args.bpk))
            verified = bool(np.array_equal(got["data"], ref.data) and np.array_equal(got["bloom"], ref.bloom)
                            and np.array_equal(got["block_off"], ref.block_off))
            assert verified, "GPU output differs from the oracle"
    sm = outs[0].summary_host()
    alg_bytes = hosts[0].algorithmic_input_bytes() + sm.data_len + sm.bloom_len

    # timed region
    if dist:
        tdist.barrier()
    torch.cuda.synchronize()
    ev0, ev1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    t0 = time.perf_counter()
    ev0.record(stream)
    for i in range(args.steps):
        step(i)
    ev1.record(stream)
    torch.cuda.synchronize()
    if dist:
        tdist.barrier()
    t1 = time.perf_counter()
    elapsed = t1 - t0
    dev_ms = ev0.elapsed_time(ev1)
    if dist:
        t = torch.tensor([elapsed], dtype=torch.float64, device=dev)
        tdist.all_reduce(t, op=tdist.ReduceOp.MAX)
        elapsed = float(t.item())

    # stage timing pass (HIP events around each kernel on the encode stream)
    lib.sdb_diag_enable_stage_timing(1)
    for i in range(args.steps):
        step(i)
    torch.cuda.synchronize()
    lib.sdb_diag_enable_stage_timing(0)
    ms = (C.c_double * 16)()
    launches = C.c_uint64(0)
    ns = lib.sdb_diag_stage_times(ms, 16, C.byref(launches))
    nl = max(launches.value, 1)
    stage_ms = {_abi.STAGES[i]: ms[i] / nl for i in range(ns)}
    emit_ms = stage_ms["emit"]
    # algorithmic bytes of the emit kernel: read keys+values(+seq/flags), write the data section
    emit_bytes = hosts[0].algorithmic_input_bytes() + sm.data_len
    emit_gbs = emit_bytes / (emit_ms * 1e-3) / 1e9

    total_logical = world * args.steps * logical
    value = total_logical / elapsed / 2**30
    ms_per_step = elapsed / args.steps * 1e3
    pipe_gbs = alg_bytes / (dev_ms / args.steps * 1e-3) / 1e9
    line = {
        "metric": "GiB/s device-resident SST block encode+bloom, 64 MiB sorted KV, 1/2/4/8 GPU",
        "value": round(value, 3),
        "unit": "GiB/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": round(ms_per_step, 4),
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "u8",
        "data": "synthetic (D1: seeded 12-byte BE counter keys + 4-byte SST index, 100 random value bytes)",
        "config": {"workload": "configs[1]: encode one 64 MiB L0 SST (578,524 x 16 B key / 100 B value) "
                               "-> 17,016 V2 4 KiB blocks + CRC32 + bloom 10 bits/key, per GPU per step",
                   "entries_per_sst": hosts[0].n, "block_size": 4096, "sst_version": 2,
                   "bloom_bits_per_key": 10, "resident_ssts_per_gpu": args.ssts,
                   "parallelism": "independent SSTs per GPU (no collective)"},
        "roofline": {"bound": "hbm", "kernel": "k_emit", "achieved": round(emit_gbs, 1),
                     "peak": PEAK_HBM_GBS, "unit": "GB/s", "frac": round(emit_gbs / PEAK_HBM_GBS, 4),
                     "traffic": pmc_traffic("k_emit"), "algorithmic_bytes_per_launch": emit_bytes,
                     "avg_launch_ms": round(emit_ms, 5),
                     "pipeline": {"algorithmic_bytes_per_sst": alg_bytes, "device_ms_per_sst": round(dev_ms / args.steps, 5),
                                  "achieved_GBps": round(pipe_gbs, 1), "frac": round(pipe_gbs / PEAK_HBM_GBS, 4),
                                  "stage_ms": {k: round(v, 5) for k, v in stage_ms.items()}}},
        "verified_vs_oracle": verified,
    }
    if rank == 0 and world == 1 and not args.no_cpu:
        threads = args.cpu_threads or min(16, os.cpu_count() or 1)
        line["cpu_baseline"] = cpu_baseline(args.cpu_seconds, threads)
    if rank == 0:
        print(json.dumps(line), flush=True)
    if dist:
        tdist.destroy_process_group()


if __name__ == "__main__":
    main()
