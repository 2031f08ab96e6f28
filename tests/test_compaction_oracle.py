"""CPU tests of the compaction restatement (oracle/): MergeIterator order, RetentionIterator against the
reference's own table (tests/golden/retention_cases.json, retention_iterator.rs:655-1024), and the
compactor's max_sst_size cut rule (compactor_executor.rs:833-858) checked structurally."""
import json
import os
import random

import numpy as np
import pytest

from oracle import oracle
from slatedb_amd import _abi
from slatedb_amd.batch import Batch, Run

HERE = os.path.dirname(os.path.abspath(__file__))
V, M, T = _abi.KIND_VALUE, _abi.KIND_MERGE, _abi.KIND_TOMBSTONE


def entries_of(b):
    out = []
    for i in range(b.n):
        mask = int(b.ts_mask[i])
        out.append((b.key(i), int(b.kind[i]), b.value(i) if b.kind[i] != T else b"", int(b.seq[i]),
                    int(b.create_ts[i]) if mask & _abi.TS_CREATE else None,
                    int(b.expire_ts[i]) if mask & _abi.TS_EXPIRE else None))
    return out


def to_entry(e):
    k, kind, val, seq, c, x = e
    return (k.encode(), kind, val.encode() if kind != T else b"", seq, c, x)


GOLDEN = json.load(open(os.path.join(HERE, "golden", "retention_cases.json")))["cases"]


@pytest.mark.parametrize("case", GOLDEN, ids=[c["name"] for c in GOLDEN])
def test_retention_golden(case):
    """apply_retention_filter cases of the reference (empty SequenceTracker: a timeout > 0 keeps every
    seq in the time window, a zero timeout none)."""
    to = case["timeout_s"]
    ret = oracle.retention(min_seq=case["retention_min_seq"], time_seq=0 if to else None,
                           compaction_start_ts=case["compaction_start_ts"],
                           filter_tombstone=case["filter_tombstone"], merge_operands=True)
    run = Run.from_entries([to_entry(e) for e in case["input"]])
    merged, sm = oracle.merge_runs([run], ret)
    assert sm.status == 0
    assert entries_of(merged) == [to_entry(e) for e in case["expected"]]


def rand_runs(rng, nruns, nkeys, maxver, tomb=0.15, merge=0.0, expire=0.2, dup_seq=False):
    """Sorted runs over a shared key space; seqs unique per key unless dup_seq."""
    keys = sorted({bytes(rng.randrange(97, 100) for _ in range(rng.randrange(1, 6))) for _ in range(nkeys)})
    runs = [[] for _ in range(nruns)]
    seq = 1
    for k in keys:
        for _ in range(rng.randrange(1, maxver + 1)):
            r = rng.randrange(nruns)
            u = rng.random()
            kind = T if u < tomb else (M if u < tomb + merge else V)
            val = bytes(rng.randrange(256) for _ in range(rng.randrange(0, 12))) if kind != T else b""
            c = rng.randrange(0, 2000) if rng.random() < 0.7 else None
            x = rng.randrange(0, 2000) if rng.random() < expire else None
            s = seq if not (dup_seq and rng.random() < 0.2) else max(1, seq - 1)
            seq += 1
            runs[r].append((k, kind, val, s, c, x))
    for r in runs:
        r.sort(key=lambda e: (e[0], -e[3]))
    return runs


def py_merge(runs):
    tagged = [(e[0], -e[3], ri, i, e) for ri, r in enumerate(runs) for i, e in enumerate(r)]
    tagged.sort(key=lambda t: t[:4])
    return [t[4] for t in tagged]


def py_retention(stream, min_seq, time_seq, cst, filter_tombstone):
    """apply_retention_filter (retention_iterator.rs:91-204) restated in Python over the merged stream."""
    out, g = [], 0
    while g < len(stream):
        ge = g
        while ge < len(stream) and stream[ge][0] == stream[g][0]:
            ge += 1
        versions = {}
        for e in stream[g:ge]:  # BTreeMap::insert: a later equal seq replaces
            versions[e[3]] = e
        kept = []
        for s in sorted(versions, reverse=True):
            k, kind, val, seq, c, x = versions[s]
            if x is not None and x <= cst:
                if kind == M:
                    continue
                e = (k, T, b"", seq, c, None)
            else:
                e = versions[s]
            kept.append(e)
            cont = (time_seq is not None and seq >= time_seq) or (min_seq is not None and seq > min_seq) or kind == M
            if not cont:
                break
        if filter_tombstone:
            while kept and kept[-1][1] == T:
                kept.pop()
        out += kept
        g = ge
    return out


@pytest.mark.parametrize("seed", range(12))
def test_merge_retention_random(seed):
    rng = random.Random(seed)
    runs = rand_runs(rng, rng.randrange(1, 6), 60, 5, merge=0.2, dup_seq=seed % 3 == 0)
    min_seq = rng.choice([None, 0, 40, 120])
    time_seq = rng.choice([None, 0, 80])
    cst = rng.choice([0, 1000, 5000])
    ft = bool(seed % 2)
    ret = oracle.retention(min_seq=min_seq, time_seq=time_seq, compaction_start_ts=cst, filter_tombstone=ft,
                           merge_operands=True)
    merged, sm = oracle.merge_runs([Run.from_entries(r) for r in runs], ret)
    assert sm.status == 0
    assert sm.num_in == sum(len(r) for r in runs)
    assert entries_of(merged) == py_retention(py_merge(runs), min_seq, time_seq, cst, ft)


def test_merge_order_keep_all():
    rng = random.Random(7)
    runs = rand_runs(rng, 4, 80, 4, expire=0.0)
    ret = oracle.retention(time_seq=0)
    merged, sm = oracle.merge_runs([Run.from_entries(r) for r in runs], ret)
    assert entries_of(merged) == py_merge(runs)
    assert sm.expired_values == 0 and sm.expired_merges == 0


def test_merge_operator_missing():
    runs = [[(b"a", V, b"1", 3, None, None), (b"b", M, b"x", 2, None, None)], [(b"a", V, b"0", 1, None, None)]]
    merged, sm = oracle.merge_runs([Run.from_entries(r) for r in runs], oracle.retention())
    assert sm.status == _abi.SDB_MERGE_OPERATOR_MISSING
    assert sm.first_error_entry == 2  # merged position of the operand


def test_unsorted_run_rejected():
    run = Run.from_entries([(b"b", V, b"1", 3, None, None), (b"a", V, b"0", 1, None, None)])
    _, sm = oracle.merge_runs([run], oracle.retention())
    assert sm.status == _abi.SDB_INVALID_ARGUMENT and sm.first_error_entry == 1


def check_cuts(batch, prm, max_sst, cuts):
    """The cut rule, structurally: every SST but the last ends with a one-entry block whose add finished
    the block that pushed the bytes past max_sst; no earlier finished block did."""
    assert cuts[0] == 0 and cuts[-1] == batch.n
    for i in range(len(cuts) - 1):
        r = oracle.encode_sst(batch.slice(cuts[i], cuts[i + 1]), prm)
        assert r.status == 0
        blen = np.diff(r.block_off.astype(np.int64))
        finished = blen[:-1]  # the last block is built by close()
        if i + 1 < len(cuts) - 1 or finished.sum() > max_sst:  # (the last entry may be a trigger too)
            assert r.block_first_entry[-2] == r.block_first_entry[-1] - 1, "tail block holds the trigger only"
            assert finished.sum() > max_sst
            assert finished[:-1].sum() <= max_sst
        else:
            assert np.cumsum(finished).max(initial=0) <= max_sst


@pytest.mark.parametrize("max_sst", [1, 300, 2000, 10 ** 9])
@pytest.mark.parametrize("version", [1, 2])
def test_sst_cuts(max_sst, version):
    rng = random.Random(max_sst + version)
    ents = sorted({(b"k%05d" % rng.randrange(100000), V, bytes(rng.randrange(256) for _ in range(rng.randrange(0, 40))),
                    1, None, None) for _ in range(600)}, key=lambda e: e[0])
    ents = [e for i, e in enumerate(ents) if i == 0 or e[0] != ents[i - 1][0]]
    b = Batch.from_entries(ents)
    prm = oracle.params(block_size=256, sst_version=version)
    st, cuts = oracle.sst_cuts(b, prm, max_sst)
    assert st == 0
    check_cuts(b, prm, max_sst, cuts)
    if max_sst == 10 ** 9:
        assert cuts == [0, b.n]
    if max_sst == 1:  # every finished block rolls over: SSTs of one block + the trigger
        assert len(cuts) > 10


def test_sst_cuts_empty():
    b = Batch.from_entries([])
    st, cuts = oracle.sst_cuts(b, oracle.params(), 100)
    assert st == 0 and cuts == []


def test_compact_end_to_end_oracle():
    rng = random.Random(3)
    runs = rand_runs(rng, 3, 400, 3)
    ret = oracle.retention(min_seq=300, compaction_start_ts=1000)
    merged, sm, cuts, ssts = oracle.compact([Run.from_entries(r) for r in runs], ret,
                                            oracle.params(block_size=512), 1024)
    assert sm.status == 0 and len(ssts) == len(cuts) - 1 >= 2
    assert sum(s.summary.num_entries for s in ssts) == merged.n


@pytest.mark.skipif(not os.path.exists("/root/reference/slatedb/src/retention_iterator.rs"),
                    reason="reference sources not present (GPU box)")
def test_retention_fixture_reproducible():
    """tests/golden/retention_cases.json is what make_retention_cases.py extracts from the reference."""
    import subprocess
    import sys
    r = subprocess.run([sys.executable, os.path.join(HERE, "golden", "make_retention_cases.py"), "--check"],
                       capture_output=True, text=True, timeout=60)
    assert r.returncode == 0, r.stderr + r.stdout
