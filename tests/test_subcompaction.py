"""Subcompactions (RFC-0028; slatedb/src/subcompaction.rs): the boundary planner and the key-range split of one
compaction over ranks.

CPU tests: the reference's own planner cases (subcompaction.rs:377-578) restated as data against
slatedb_amd/subcompaction.py, the planner over encoded SSTs, and a world-2 gloo job in which each rank
compacts its ranges (the oracle standing in for the per-rank sdb_compactor, test-only) — the ranges' merged
outputs concatenate to the unsplit compaction's, entry for entry.  The device path of the same split is
tests/test_gpu_compaction.py::test_compactor_subcompactions."""
import os
import socket

import numpy as np
import pytest
import torch.multiprocessing as mp

from oracle import oracle as O
from slatedb_amd import datasets
from slatedb_amd import subcompaction as S
from slatedb_amd.batch import Run


def k(i):
    return b"k%010d" % i


def assert_covering(ranges):
    assert ranges[0].start is None and ranges[-1].end is None
    for a, b in zip(ranges, ranges[1:]):
        assert a.end is not None and a.end == b.start
    for r in ranges:
        assert r.start is None or r.end is None or r.start < r.end


def test_reference_select_boundaries_cases():
    U = [S.UNBOUNDED]
    # test_should_not_split_when_subcompactions_disabled / _inputs_below_floor / _single_anchor
    assert S.select_boundaries([(k(0), 100), (k(100), 100)], 1, 1) == U
    assert S.select_boundaries([(k(0), 100), (k(100), 100)], 4, 1000) == U
    assert S.select_boundaries([(k(0), 1000)], 4, 1000) == U
    # test_should_split_evenly_weighted_anchors
    r = S.select_boundaries([(k(0), 100), (k(10), 100), (k(20), 100), (k(30), 100)], 4, 1)
    assert_covering(r)
    assert [x.end for x in r[:3]] == [k(10), k(20), k(30)] and len(r) == 4
    # test_should_divide_evenly_with_many_anchors_per_subcompaction
    r = S.select_boundaries([(k(i), 10) for i in range(16)], 4, 25)
    assert_covering(r)
    assert [x.end for x in r[:3]] == [k(4), k(8), k(12)] and len(r) == 4
    # test_should_split_into_fewer_ranges_when_floor_binds
    r = S.select_boundaries([(k(i), 50) for i in range(8)], 8, 100)
    assert_covering(r)
    assert [x.end for x in r[:3]] == [k(2), k(4), k(6)] and len(r) == 4
    # test_should_cap_splits_at_max_subcompactions
    r = S.select_boundaries([(k(i), 100) for i in range(100)], 4, 1)
    assert_covering(r)
    assert len(r) == 4
    # test_should_isolate_heavy_region
    r = S.select_boundaries([(k(0), 1000), (k(10), 10), (k(20), 10), (k(30), 10), (k(40), 10)], 2, 1)
    assert_covering(r)
    assert len(r) == 2 and r[0].end == k(10)
    # test_should_not_emit_boundary_on_smallest_key
    r = S.select_boundaries([(k(0), 400), (k(0), 400), (k(0), 400), (k(10), 400), (k(20), 400)], 4, 1)
    assert_covering(r)
    assert r[0].end == k(10) and len(r) > 1
    # test_should_handle_duplicate_keys_without_empty_ranges
    r = S.select_boundaries([(k(0), 500), (k(0), 500), (k(10), 500), (k(10), 500), (k(20), 500), (k(20), 500)], 4, 1)
    assert_covering(r)
    assert len(r) > 1


def test_reference_sample_anchors_cases():
    keys, offs = [k(0), k(10), k(20), k(30)], [0, 100, 200, 300]
    # test_sample_anchors_keeps_all_blocks_without_projection
    assert S.sample_anchors(keys, offs, 400) == [(k(0), 100), (k(10), 100), (k(20), 100), (k(30), 100)]
    # test_sample_anchors_clips_to_projected_effective_range
    assert S.sample_anchors(keys, offs, 400, effective_range=S.KeyRange(k(10), k(30))) == [(k(10), 100), (k(20), 100)]
    # grouping: 4 blocks at <= 2 anchors -> groups of 2, weighted by the group's bytes
    assert S.sample_anchors(keys, offs, 400, max_anchors=2) == [(k(0), 200), (k(20), 200)]


def _job(n=6000, nruns=4):
    batches = datasets.overwrite_runs(nruns=nruns, n=n)
    runs = [Run.from_batch(b) for b in batches]
    prm = O.params(block_size=4096)
    metas = []
    for b in batches:
        e = O.encode_sst(b, prm)
        assert e.status == 0
        metas.append(S.SstMeta.from_encoded(b, e))
    return batches, runs, metas, prm


def merged_entries(b):
    return [(b.key(i), int(b.kind[i]), int(b.seq[i]), b.value(i)) for i in range(b.n)]


def test_planner_over_encoded_ssts():
    _, runs, metas, _ = _job()
    ranges = S.plan_subcompaction_ranges(metas, 4)
    assert_covering(ranges)
    assert 2 <= len(ranges) <= 4
    # each range holds a comparable share of the input entries
    share = [sum(np.subtract(*S.run_bounds(r, x)[::-1]) for r in runs) for x in ranges]
    assert sum(share) == sum(r.n for r in runs)
    assert max(share) <= 2.5 * min(share), share


def test_ranges_concatenate_to_the_unsplit_compaction():
    _, runs, metas, prm = _job()
    ret = O.retention(filter_tombstone=True)
    whole, wsm, _, _ = O.compact(runs, ret, prm, 64 << 20)
    assert wsm.status == 0
    ranges = S.plan_subcompaction_ranges(metas, 4)
    got = []
    for x in ranges:
        part, sm, cuts, ssts = O.compact([S.slice_run(r, x) for r in runs], ret, prm, 64 << 20)
        assert sm.status == 0 and all(s.status == 0 for s in ssts)
        got += merged_entries(part)
    assert got == merged_entries(whole)


# --- world 2 over gloo: range r -> rank r mod 2 ---------------------------------------------------------------
def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _rank_main(rank, world, port, q):
    import torch.distributed as dist
    os.environ["MASTER_ADDR"] = "127.0.0.1"
    os.environ["MASTER_PORT"] = str(port)
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        _, runs, metas, prm = _job()
        ranges = S.plan_subcompaction_ranges(metas, 4)
        ret = O.retention(filter_tombstone=True)
        mine = S.assign_ranges(ranges, world)[rank]
        out = {}
        for ri in mine:
            part, sm, _, _ = O.compact([S.slice_run(r, ranges[ri]) for r in runs], ret, prm, 64 << 20)
            assert sm.status == 0
            out[ri] = merged_entries(part)
        gathered = [None] * world
        dist.all_gather_object(gathered, out)
        if rank == 0:
            allr = {}
            for g in gathered:
                allr.update(g)
            q.put((len(ranges), [e for ri in sorted(allr) for e in allr[ri]]))
    finally:
        dist.destroy_process_group()


def test_subcompactions_over_two_ranks_gloo():
    ctx = mp.get_context("spawn")
    q = ctx.Queue()
    port = _free_port()
    procs = [ctx.Process(target=_rank_main, args=(r, 2, port, q)) for r in range(2)]
    for p in procs:
        p.start()
    nranges, got = q.get(timeout=300)
    for p in procs:
        p.join(timeout=120)
        assert p.exitcode == 0
    _, runs, _, prm = _job()
    whole, wsm, _, _ = O.compact(runs, O.retention(filter_tombstone=True), prm, 64 << 20)
    assert nranges >= 2
    assert got == merged_entries(whole)


def test_assign_ranges():
    assert S.assign_ranges(list(range(5)), 2) == [[0, 2, 4], [1, 3]]
    with pytest.raises(ValueError):
        S.assign_ranges([S.UNBOUNDED], 0)
