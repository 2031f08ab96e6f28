"""Multi-rank sharding of a compaction job (configs[4]) on CPU with the gloo backend.

SSTs are independent, so the job shards with no data-path collective: SST j -> rank j mod N
(slatedb_amd/job.py), each rank encodes its share, and the whole-job rate is Σ bytes ÷ max wall time.
bench.py runs exactly this partition over RCCL on the GPU box; here world_size 2 runs over gloo with
the CPU oracle standing in as the per-rank encoder (test-only), and the ranks' outputs are checked
against a single-process encode of the whole job.
"""
import os
import socket
import zlib

import pytest
import torch.multiprocessing as mp

from slatedb_amd import job

JOB_SSTS = 6
N_ENTRIES = 3000


def test_assign_partition():
    for world in (1, 2, 3, 8):
        a = job.assign(64, world)
        assert sorted(sum(a, [])) == list(range(64))
        assert all(j % world == r for r, ids in enumerate(a) for j in ids)
    assert job.assign(64, 8)[3] == [3, 11, 19, 27, 35, 43, 51, 59]
    assert job.job_rate_gibs(2**31, 2.0) == 1.0
    with pytest.raises(ValueError):
        job.assign(4, 0)


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _encode_digest(j):
    from oracle import oracle as O
    from slatedb_amd import datasets
    b = datasets.d1(sst_index=j, n=N_ENTRIES)
    r = O.encode_sst(b, O.params())
    assert r.status == 0
    return b.logical_bytes(), zlib.crc32(r.data.tobytes()) ^ (zlib.crc32(r.bloom.tobytes()) << 1)


def _rank_main(rank, world, port, q):
    import time

    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        mine = job.share(JOB_SSTS, world, rank)
        dist.barrier()
        t0 = time.perf_counter()
        got = {j: _encode_digest(j) for j in mine}
        elapsed = time.perf_counter() - t0
        dist.barrier()
        total, tmax = job.aggregate(dist, sum(v[0] for v in got.values()), elapsed)
        everything = [None] * world
        dist.all_gather_object(everything, got)
        if rank == 0:
            q.put((total, tmax, everything))
    finally:
        dist.destroy_process_group()


def test_job_sharding_gloo_world2():
    world = 2
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, world, port, q)) for r in range(world)]
    for p in procs:
        p.start()
    total, tmax, everything = q.get(timeout=240)
    for p in procs:
        p.join(timeout=60)
        assert p.exitcode == 0
    merged = {}
    for r, d in enumerate(everything):
        assert sorted(d) == job.share(JOB_SSTS, world, r)
        merged.update(d)
    assert sorted(merged) == list(range(JOB_SSTS))       # every SST exactly once
    single = {j: _encode_digest(j) for j in range(JOB_SSTS)}
    assert merged == single                               # sharding changes no byte
    assert total == sum(v[0] for v in single.values())   # Σ bytes over ranks
    assert tmax > 0 and job.job_rate_gibs(total, tmax) > 0


def test_bench_spawns_gpus_ranks_dry_run():
    """`python bench.py --gpus 2` without a launcher starts two ranks itself (before any GPU call); in
    --dry-run they meet over gloo, take their share of the job and aggregate, and n_gpus == --gpus."""
    import json
    import subprocess
    import sys
    root = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
    env = {k: v for k, v in os.environ.items() if k not in ("WORLD_SIZE", "RANK", "LOCAL_RANK")}
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run",
                        "--job-ssts", "64"], env=env, capture_output=True, text=True, timeout=180)
    assert r.returncode == 0, r.stderr[-2000:]
    line = json.loads([l for l in r.stdout.splitlines() if l.startswith("{")][-1])
    assert line["n_gpus"] == 2
    assert line["ssts_per_rank"] == [job.share(64, 2, 0), job.share(64, 2, 1)]
    assert line["total_logical_bytes"] == 64 * (578524 * 116)
    # a launcher world that disagrees with --gpus is refused
    env["WORLD_SIZE"] = "1"
    r = subprocess.run([sys.executable, os.path.join(root, "bench.py"), "--gpus", "2", "--dry-run"], env=env,
                       capture_output=True, text=True, timeout=120)
    assert r.returncode != 0 and "WORLD_SIZE" in r.stderr
