"""GPU parity of the compaction output side (sdb_merge_runs, sdb_sst_cuts, sdb_compactor_*;
slatedb_amd/csrc/sdb_compact.hip, sdb_compactor.cpp) against the oracle restatement (orc_merge_runs,
orc_sst_cuts, orc_encode_sst per output SST): the merged + retained stream field by field, the cut
list, and every output SST byte for byte — on the reference's retention table, random multi-run
inputs (duplicate seqs, merges, expiry, tombstone filtering), multi-chunk / multi-group streams, and
SSTs encoded then decoded on the device as the inputs."""
import json
import os
import random
import types

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi
from slatedb_amd.batch import Batch, Run

from .test_compaction_oracle import GOLDEN, entries_of, rand_runs, to_entry
from .test_gpu_parity import assert_same

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from slatedb_amd import runtime
    runtime.require_device()
    return runtime


def assert_batch_same(got, ref, what=""):
    assert got.n == ref.n, (what, got.n, ref.n)
    for f in ("key_off", "val_off", "kind", "seq", "ts_mask", "create_ts", "expire_ts"):
        assert np.array_equal(np.asarray(getattr(got, f)), np.asarray(getattr(ref, f))), (what, f)
    assert np.array_equal(got.key_bytes, ref.key_bytes), what
    assert np.array_equal(got.val_bytes, ref.val_bytes), what


def merge_both(rt, runs, ret):
    import torch
    druns = [rt.DeviceRun.from_host(r) for r in runs]
    o, sm = rt.merge_runs_device(druns, ret)
    torch.cuda.synchronize()
    ref, rsm = O.merge_runs(runs, ret)
    assert sm.status == rsm.status, (sm.status, rsm.status)
    assert sm.first_error_entry == rsm.first_error_entry
    assert sm.num_in == rsm.num_in
    if rsm.status == 0:
        for f in ("num_out", "key_bytes", "val_bytes", "expired_values", "expired_merges"):
            assert getattr(sm, f) == getattr(rsm, f), f
        assert_batch_same(rt.merged_to_host(o, sm), ref)
    return ref, rsm


@pytest.mark.parametrize("case", GOLDEN, ids=[c["name"] for c in GOLDEN])
def test_retention_golden_device(rt, case):
    to = case["timeout_s"]
    ret = O.retention(min_seq=case["retention_min_seq"], time_seq=0 if to else None,
                      compaction_start_ts=case["compaction_start_ts"], filter_tombstone=case["filter_tombstone"],
                      merge_operands=True)
    run = Run.from_entries([to_entry(e) for e in case["input"]])
    ref, _ = merge_both(rt, [run], ret)
    assert entries_of(ref) == [to_entry(e) for e in case["expected"]]


@pytest.mark.parametrize("seed", range(10))
def test_merge_retention_random_device(rt, seed):
    rng = random.Random(100 + seed)
    runs = rand_runs(rng, rng.randrange(1, 9), 300, 5, merge=0.2, dup_seq=seed % 3 == 0)
    ret = O.retention(min_seq=rng.choice([None, 0, 200, 700]), time_seq=rng.choice([None, 0, 400]),
                      compaction_start_ts=rng.choice([0, 1000, 5000]), filter_tombstone=bool(seed % 2),
                      merge_operands=True)
    merge_both(rt, [Run.from_entries(r) for r in runs], ret)


def test_merge_errors_device(rt):
    runs = [[(b"a", 0, b"1", 3, None, None), (b"b", 1, b"x", 2, None, None), (b"c", 1, b"y", 1, None, None)],
            [(b"a", 0, b"0", 1, None, None), (b"bb", 1, b"z", 5, None, None)]]
    _, sm = merge_both(rt, [Run.from_entries(r) for r in runs], O.retention())
    assert sm.status == _abi.SDB_MERGE_OPERATOR_MISSING and sm.first_error_entry == 2
    bad = Run.from_entries([(b"b", 0, b"1", 3, None, None), (b"a", 0, b"0", 1, None, None)])
    _, sm = merge_both(rt, [Run.from_entries(runs[0][:1]), bad], O.retention())
    assert sm.status == _abi.SDB_INVALID_ARGUMENT and sm.first_error_entry == 2


def test_merge_empty_runs(rt):
    e = Run.from_entries([])
    merge_both(rt, [e, e], O.retention())
    ret = O.retention(compaction_start_ts=10 ** 9, filter_tombstone=True)  # everything expires and goes
    merge_both(rt, [Run.from_entries([(b"k", 0, b"v", 1, None, 5)])], ret)


def big_runs(seed, nkeys, nruns, maxver=3, vmax=120, tomb=0.1, expire=0.05):
    """numpy-built sorted runs: 16-byte keys (8-byte BE random prefix + 8-byte BE counter), 1..maxver
    versions each spread over the runs, unique seqs, values of 0..vmax bytes."""
    rng = np.random.default_rng(seed)
    pre = np.sort(rng.integers(0, 1 << 62, nkeys, dtype=np.int64).astype(np.uint64))
    nver = rng.integers(1, maxver + 1, nkeys)
    kidx = np.repeat(np.arange(nkeys), nver)
    m = len(kidx)
    seq = rng.permutation(m).astype(np.uint64) + 1
    # within a key: seqs descending
    order = np.lexsort((-seq.astype(np.int64), kidx))
    seq = seq[order]
    run = rng.integers(0, nruns, m)
    kb = np.zeros((m, 16), np.uint8)
    kb[:, :8] = pre[kidx].byteswap().view(np.uint8).reshape(-1, 8)
    kb[:, 8:] = np.arange(nkeys, dtype=np.uint64)[kidx].byteswap().view(np.uint8).reshape(-1, 8)
    vlen = rng.integers(0, vmax + 1, m)
    kind = np.where(rng.random(m) < tomb, _abi.KIND_TOMBSTONE, _abi.KIND_VALUE).astype(np.uint8)
    vlen[kind == _abi.KIND_TOMBSTONE] = 0
    pool = rng.integers(0, 256, int(vlen.sum()) + 16, dtype=np.uint8)
    ets = rng.integers(0, 2000, m).astype(np.int64)
    mask = np.where(rng.random(m) < expire, _abi.TS_EXPIRE, 0).astype(np.uint8)
    runs = []
    vstart = np.concatenate([[0], np.cumsum(vlen)])
    for r in range(nruns):
        sel = np.nonzero(run == r)[0]
        n = len(sel)
        koff = np.arange(n + 1, dtype=np.uint64) * 16
        vl = vlen[sel]
        voff = np.concatenate([[0], np.cumsum(vl)]).astype(np.uint64)
        vb = np.concatenate([pool[vstart[i]:vstart[i] + vlen[i]] for i in sel]) if n else np.zeros(0, np.uint8)
        runs.append(Run.from_batch(Batch(kb[sel].reshape(-1), koff, vb, voff, kind[sel], seq[sel],
                                         np.zeros(n, np.int64), ets[sel], mask[sel])))
    return runs


@pytest.mark.parametrize("nruns", [2, 7])
def test_merge_big_device(rt, nruns):
    runs = big_runs(nruns, 60000, nruns)
    merge_both(rt, runs, O.retention(min_seq=50000, compaction_start_ts=1000, filter_tombstone=nruns == 7))


def cuts_both(rt, batch, prm, max_sst):
    got = rt.sst_cuts_device(batch.to_device(), prm, max_sst)
    st, ref = O.sst_cuts(batch, prm, max_sst)
    assert st == 0
    assert got == ref, (len(got), len(ref), [(a, b) for a, b in zip(got, ref) if a != b][:4])
    return ref


@pytest.mark.parametrize("max_sst", [1, 5000, 300000, 10 ** 12])
@pytest.mark.parametrize("version,bs", [(2, 4096), (2, 512), (1, 4096)])
def test_sst_cuts_device(rt, max_sst, version, bs):
    runs = big_runs(5, 40000, 1, maxver=1)
    r = runs[0]
    b = Batch(r.key_arena, r.key_off, r.val_base, np.concatenate([r.val_off, [r.val_off[-1] + r.val_len[-1]]]),
              np.where(r.flags & 1, 2, 0).astype(np.uint8), r.seq, r.create_ts, r.expire_ts,
              np.where(r.flags & 2, 2, 0).astype(np.uint8))
    cuts = cuts_both(rt, b, O.params(sst_version=version, block_size=bs), max_sst)
    if max_sst == 10 ** 12:
        assert cuts == [0, b.n]


def test_sst_cuts_long_blocks_device(rt):
    """64 KiB blocks of tiny rows: the chain tables are off (serial walk mode)."""
    n = 30000
    ents = [(b"%08d" % i, 0, b"", 1, None, None) for i in range(n)]
    b = Batch.from_entries(ents)
    cuts_both(rt, b, O.params(block_size=65536), 100000)


@pytest.mark.parametrize("max_sst", [3000, 100000, 10 ** 12])
def test_sst_cuts_tables_in_hbm_device(rt, max_sst):
    """~315 tiny rows per 4 KiB block: ~316 candidate entry points per chunk, so a group's chunk tables
    (and, with 123 chunks, the group tables) outgrow k_cut's LDS and the walk reads them from HBM."""
    n = 250000
    ents = [(b"%08d" % i, 0, b"", 1, None, None) for i in range(n)]
    b = Batch.from_entries(ents)
    cuts_both(rt, b, O.params(block_size=4096), max_sst)


def sst_view(d):
    return types.SimpleNamespace(status=d["summary"].status,
                                 summary={f: getattr(d["summary"], f) for f, _ in _abi.SstSummary._fields_},
                                 data=d["data"], block_off=d["block_off"], block_first_entry=d["block_first_entry"],
                                 index_key_len=d["index_key_len"], block_stats=d["block_stats"], bloom=d["bloom"])


def compact_both(rt, runs, ret, prm_kw, max_sst, druns=None):
    import torch
    druns = druns or [rt.DeviceRun.from_host(r) for r in runs]
    comp = rt.Compactor()
    st, ns = comp.run(druns, ret, rt.params(**prm_kw), max_sst)
    torch.cuda.synchronize()
    merged, msum, cuts, ssts = O.compact(runs, ret, O.params(**prm_kw), max_sst)
    assert st == msum.status, (st, msum.status)
    if st:
        return comp, ssts
    gm, gsm = comp.merged()
    assert_batch_same(gm, merged, "merged")
    assert ns == len(ssts), (ns, len(ssts))
    for i, ref in enumerate(ssts):
        d = comp.sst(i)
        assert (d["entry_start"], d["entry_end"]) == (cuts[i], cuts[i + 1])
        assert_same(ref, sst_view(d), "sst %d" % i)
    return comp, ssts


@pytest.mark.parametrize("version", [1, 2])
def test_compactor_big(rt, version):
    runs = big_runs(11, 80000, 5)
    comp, ssts = compact_both(rt, runs, O.retention(min_seq=100000, compaction_start_ts=1000, filter_tombstone=True),
                              dict(sst_version=version, block_size=4096, bloom_bits_per_key=10), 2 << 20)
    assert len(ssts) >= 3
    comp.close()


def test_compactor_small_cases(rt):
    rng = random.Random(5)
    runs = [Run.from_entries(r) for r in rand_runs(rng, 4, 500, 4)]
    for max_sst in (1, 700, 10 ** 9):
        compact_both(rt, runs, O.retention(min_seq=100, compaction_start_ts=900), dict(block_size=256), max_sst)
    # merge operands without a merge operator fail the job
    mruns = [Run.from_entries(r) for r in rand_runs(rng, 2, 50, 3, merge=0.3)]
    compact_both(rt, mruns, O.retention(), dict(), 10 ** 9)
    # everything filtered: no output SST
    compact_both(rt, [Run.from_entries([(b"k", 2, b"", 1, None, None)])], O.retention(filter_tombstone=True),
                 dict(), 100)


def test_compactor_from_device_decoded_ssts(rt):
    """The whole device path: input SSTs encoded on the GPU, decoded on the GPU (sdb_decode_blocks),
    merged / retained / cut / re-encoded on the GPU; checked against the oracle on the host runs."""
    import torch
    runs = big_runs(21, 30000, 3)
    prm_kw = dict(block_size=4096, bloom_bits_per_key=10)
    druns = []
    keep = []
    for r in runs:
        n = r.n
        b = Batch(r.key_arena, r.key_off, r.val_base, np.concatenate([r.val_off, [r.val_off[-1] + r.val_len[-1]]]),
                  np.where(r.flags & 1, 2, 0).astype(np.uint8), r.seq, r.create_ts, r.expire_ts,
                  np.where(r.flags & 2, 2, 0).astype(np.uint8))
        enc = O.encode_sst(b, O.params(**prm_kw))
        blocks = torch.from_numpy(np.concatenate([enc.data, np.zeros(64, np.uint8)])).cuda()
        boff = torch.from_numpy(enc.block_off.view(np.int64)).cuda()
        nb = len(enc.block_off) - 1
        dout = rt.DeviceDecodeOutput(nb, n + 16, int(r.key_off[-1]) + 64)
        st = rt.lib().sdb_decode_blocks(blocks.data_ptr(), boff.data_ptr(), nb, 2, __import__("ctypes").byref(dout.out),
                                        dout.workspace.data_ptr(), dout.workspace.numel(), None)
        assert st == 0
        torch.cuda.synchronize()
        assert dout.summary_host().num_entries == n
        druns.append(rt.DeviceRun.from_decoded(dout, blocks, n))
        keep.append((blocks, boff, dout))
    compact_both(rt, runs, O.retention(min_seq=40000, compaction_start_ts=1000), prm_kw, 1 << 20, druns=druns)


def test_v1_blocks_past_block_size(rt):
    """V1 blocks may hold block_size + 2 bytes (the new entry's offset is not counted, block.rs:117-123):
    their CRC runs through the windowed path with a 1-2 byte first window (encode and decode)."""
    from .test_gpu_parity import assert_decode_same
    runs = big_runs(11, 80000, 5)
    merged, _ = O.merge_runs(runs, O.retention(min_seq=100000, compaction_start_ts=1000, filter_tombstone=True))
    b = merged.slice(0, 30000)
    prm = dict(sst_version=1, block_size=4096)
    ref = O.encode_sst(b, O.params(**prm))
    lens = np.diff(ref.block_off.astype(np.int64)) - 4
    assert (lens > 4096).any()
    enc = rt.Encoder(rt.params(**prm))
    got = enc.encode(b)
    enc.close()
    assert_same(ref, got, "v1 oversized")
    dref = O.decode_blocks(ref.data, ref.block_off, 1)
    dec = rt.Decoder()
    assert_decode_same(dref, dec.decode(ref.data, ref.block_off, 1), "v1 oversized decode")


def encoded_inputs(rt, runs, prm_kw, split=1):
    """Each run encoded by the oracle as `split` consecutive SSTs, uploaded: (inputs, run_start, ref_runs) with
    ref_runs = the runs as the reference reads them back (the oracle's decode of each run's SSTs: V0 rows
    drop a tombstone's expire_ts)."""
    import torch
    inputs, run_start, ref_runs = [], [0], []
    for r in runs:
        datas, offs, base = [], [], 0
        b = Batch(r.key_arena, r.key_off, r.val_base, np.concatenate([r.val_off, [r.val_off[-1] + r.val_len[-1]]]),
                  np.where(r.flags & 1, 2, 0).astype(np.uint8), r.seq, r.create_ts, r.expire_ts,
                  np.where(r.flags & 2, 2, 0).astype(np.uint8))
        cuts = np.linspace(0, b.n, split + 1).astype(int)
        for i in range(split):
            enc = O.encode_sst(b.slice(cuts[i], cuts[i + 1]), O.params(**prm_kw))
            sm = enc.summary
            inputs.append(types.SimpleNamespace(
                data=torch.from_numpy(np.concatenate([enc.data, np.zeros(16, np.uint8)])).cuda(),
                block_off=torch.from_numpy(enc.block_off.view(np.int64)).cuda(),
                num_entries=int(sm.num_entries), key_bytes=int(sm.raw_key_size), val_bytes=int(sm.raw_val_size)))
            bo = enc.block_off.astype(np.uint64)
            datas.append(enc.data[:int(bo[-1])])
            offs.append((bo if i == split - 1 else bo[:-1]) + np.uint64(base))
            base += int(bo[-1])
        run_start.append(len(inputs))
        blocks = np.concatenate(datas) if datas else np.zeros(0, np.uint8)
        d = O.decode_blocks(blocks, np.concatenate(offs), prm_kw.get("sst_version", 2))
        assert d.status == 0 and d.n == r.n
        ref_runs.append(Run(d.key_arena, d.key_off, blocks, d.val_off, d.val_len, d.seq, d.flags, d.create_ts,
                            d.expire_ts))
    return inputs, run_start, ref_runs


def compact_ssts_both(rt, runs, ret, prm_kw, max_sst, split=1, version=2, out_kw=None):
    """sdb_compactor_run_ssts on the runs' encoded SSTs vs O.compact on the runs."""
    import torch
    inputs, run_start, runs = encoded_inputs(rt, runs, dict(prm_kw, sst_version=version), split)
    out_kw = out_kw or prm_kw
    comp = rt.Compactor()
    st, ns = comp.run_ssts(inputs, ret, rt.params(**out_kw), max_sst, input_version=version,
                           run_start=run_start if split > 1 else None)
    torch.cuda.synchronize()
    merged, msum, cuts, ssts = O.compact(runs, ret, O.params(**out_kw), max_sst)
    assert st == msum.status, (st, msum.status)
    if not st:
        gm, _ = comp.merged()
        assert_batch_same(gm, merged, "merged")
        assert ns == len(ssts), (ns, len(ssts))
        for i, ref in enumerate(ssts):
            d = comp.sst(i)
            assert (d["entry_start"], d["entry_end"]) == (cuts[i], cuts[i + 1])
            assert_same(ref, sst_view(d), "sst %d" % i)
    comp.close()
    return st, ns, inputs


@pytest.mark.parametrize("version", [1, 2])
def test_compactor_run_ssts(rt, version):
    """Decode inside the job: L0 SSTs encoded by the oracle, decoded + merged + retained + cut + encoded on
    the device, compared with the oracle's compaction of the same runs."""
    runs = big_runs(31, 40000, 4)
    _, ns, _ = compact_ssts_both(rt, runs, O.retention(min_seq=50000, compaction_start_ts=1000, filter_tombstone=True),
                                 dict(block_size=4096, bloom_bits_per_key=10), 1 << 20, version=version)
    assert ns >= 3


def test_compactor_run_ssts_sorted_runs(rt):
    """Sorted runs of three SSTs each (run_start), small blocks, several output SSTs."""
    runs = big_runs(32, 20000, 3)
    compact_ssts_both(rt, runs, O.retention(min_seq=10000, compaction_start_ts=500), dict(block_size=1024), 300000,
                      split=3)


def test_compactor_run_ssts_edges(rt):
    rng = random.Random(9)
    small = [Run.from_entries(r) for r in rand_runs(rng, 3, 400, 4)]
    for max_sst in (1, 10 ** 9):  # one SST per block / one SST
        compact_ssts_both(rt, small, O.retention(min_seq=100, compaction_start_ts=900), dict(block_size=256), max_sst)
    # everything dropped: no output SST
    compact_ssts_both(rt, [Run.from_entries([(b"k", 2, b"", 1, None, None)])], O.retention(filter_tombstone=True),
                      dict(), 100)
    # merge operands without a merge operator
    mruns = [Run.from_entries(r) for r in rand_runs(rng, 2, 50, 3, merge=0.3)]
    compact_ssts_both(rt, mruns, O.retention(), dict(), 10 ** 9)


def test_compactor_run_ssts_bad_inputs(rt):
    """A corrupt input block fails the job with its read error (lowest block first); counts that
    disagree with the blocks fail it with SDB_INVALID_ARGUMENT; nothing is merged either way."""
    import torch
    runs = big_runs(33, 8000, 3)
    prm_kw = dict(block_size=4096, bloom_bits_per_key=10)
    inputs, _, _ = encoded_inputs(rt, runs, prm_kw)
    prm, ret = rt.params(**prm_kw), O.retention()
    comp = rt.Compactor()
    # flip a byte inside block 3 of input 1 (job block index = input 0's blocks + 3)
    bo = inputs[1].block_off.cpu().numpy()
    inputs[1].data[int(bo[3]) + 10] ^= 0x5A
    st, ns = comp.run_ssts(inputs, ret, prm, 1 << 30)
    torch.cuda.synchronize()
    assert st == _abi.SDB_CHECKSUM_MISMATCH and ns == 0
    _, sm = comp.merged()
    assert sm.first_error_entry == inputs[0].block_off.numel() - 1 + 3
    inputs[1].data[int(bo[3]) + 10] ^= 0x5A
    st, ns = comp.run_ssts(inputs, ret, prm, 1 << 30)
    assert st == 0 and ns == 1
    for f, d in (("num_entries", 1), ("key_bytes", -1)):
        setattr(inputs[2], f, getattr(inputs[2], f) + d)
        st, ns = comp.run_ssts(inputs, ret, prm, 1 << 30)
        torch.cuda.synchronize()
        assert st == _abi.SDB_INVALID_ARGUMENT and ns == 0, (f, st)
        setattr(inputs[2], f, getattr(inputs[2], f) - d)
    comp.close()


def test_compactor_overwrites_drop(rt):
    """Retention that drops: four L0 runs over one key space (most keys in several runs), tombstones in the
    newest, no snapshot and filter_tombstone (the bench_configs.py overwrite job at reduced size): both
    device jobs bit-exact, and the merged stream holds only each key's newest live version."""
    from slatedb_amd import datasets
    runs = [Run.from_batch(b) for b in datasets.overwrite_runs(n=30000)]
    ret = O.retention(filter_tombstone=True)
    prm_kw = dict(block_size=4096, bloom_bits_per_key=10)
    comp, ssts = compact_both(rt, runs, ret, prm_kw, 1 << 20)
    _, msum = comp.merged()
    assert msum.num_out < msum.num_in // 3 and len(ssts) >= 2
    comp.close()
    st, ns, _ = compact_ssts_both(rt, runs, ret, prm_kw, 1 << 20)
    assert st == 0 and ns == len(ssts)


# ------------------------------------------------------------------------------------------------
# limits: one sdb_merge_runs call takes SDB_MAX_RUNS (32) runs; the compactor merges more in groups of
# 32 first (sdb_compactor.cpp group_runs) and takes any number of input SSTs
# ------------------------------------------------------------------------------------------------
def test_merge_runs_limit(rt):
    """33 runs in one sdb_merge_runs call: SDB_LIMIT_EXCEEDED (documented per-call limit)."""
    import ctypes as C
    runs = [Run.from_entries([(b"k%03d" % i, 0, b"v", 1, None, None)]) for i in range(33)]
    druns = [rt.DeviceRun.from_host(r) for r in runs]
    cr = (_abi.Run * 33)(*[r.to_ctypes() for r in druns])
    assert rt.lib().sdb_merge_runs(cr, 33, C.byref(O.retention()), C.byref(_abi.MergedOut()), None, 0, None) == \
        _abi.SDB_LIMIT_EXCEEDED
    merged, sm = rt.merge_runs_device(druns[:32], O.retention())
    assert sm.status == 0 and sm.num_out == 32


@pytest.mark.parametrize("nruns", [32, 33, 70])
def test_compactor_many_runs(rt, nruns):
    """Jobs of 32, 33 and 70 runs (one merge; groups of 32 merged first): bit-exact with the oracle's
    single merge of every run, including versions with equal seqs in different groups (run order)."""
    rng = random.Random(100 + nruns)
    runs = [Run.from_entries(r) for r in rand_runs(rng, nruns, 600, 5, dup_seq=True)]
    compact_both(rt, runs, O.retention(min_seq=300, compaction_start_ts=900, filter_tombstone=True),
                 dict(block_size=1024), 4000)
    compact_both(rt, runs, O.retention(min_seq=10 ** 9), dict(block_size=4096, bloom_bits_per_key=10), 10 ** 9)


@pytest.mark.parametrize("ninputs,split", [(64, 1), (65, 1), (70, 5)])
def test_compactor_run_ssts_many_inputs(rt, ninputs, split):
    """64, 65 and 70 input SSTs (70 as 14 sorted runs of 5 SSTs): the decode takes every input's blocks,
    the runs beyond 32 merge in groups."""
    rng = random.Random(200 + ninputs)
    nruns = ninputs // split
    runs = [Run.from_entries(r) for r in rand_runs(rng, nruns, 3000, 4, dup_seq=True) if len(r) >= split]
    if split == 1:
        runs = [r for r in runs if r.n > 0]
    st, ns, _ = compact_ssts_both(rt, runs, O.retention(min_seq=500, compaction_start_ts=900), dict(block_size=512),
                                  20000, split=split)
    assert st == 0 and ns >= 1


def test_compactor_many_runs_order_error(rt):
    """A run out of order in the second group fails the job at its global entry index, as one merge would."""
    rng = random.Random(7)
    runs = [Run.from_entries(r) for r in rand_runs(rng, 40, 400, 3)]
    ents = [(b"zz", 0, b"x", 5, None, None), (b"aa", 0, b"y", 4, None, None)]  # descending keys
    runs[35] = Run.from_entries(ents)
    compact_both(rt, runs, O.retention(), dict(), 10 ** 9)


def test_compactor_subcompactions(rt):
    """RFC-0028 subcompactions on the device: the planner's key ranges (slatedb_amd/subcompaction.py over
    the inputs' block indexes), each range compacted by its own sdb_compactor job from the input runs cut to
    the range — every range bit-exact vs the oracle (merged stream, cut list, every output SST), and the
    ranges' merged streams concatenate to the unsplit job's."""
    from slatedb_amd import subcompaction as S

    from .test_subcompaction import _job, merged_entries
    _, runs, metas, _ = _job(n=20000)
    ranges = S.plan_subcompaction_ranges(metas, 4)
    assert len(ranges) >= 2
    ret = O.retention(filter_tombstone=True)
    got = []
    for x in ranges:
        part = [S.slice_run(r, x) for r in runs]
        comp, ssts = compact_both(rt, part, ret, dict(block_size=4096, bloom_bits_per_key=10), 2 << 20)
        gm, _ = comp.merged()
        got += merged_entries(gm)
        comp.close()
    whole, wsm, _, _ = O.compact(runs, ret, O.params(block_size=4096, bloom_bits_per_key=10), 2 << 20)
    assert got == merged_entries(whole)
