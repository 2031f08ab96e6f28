"""CPU checks of the point-lookup restatement (oracle/sdb_oracle.c orc_sst_lookup) against properties of
the reference read path on sorted SSTs (key asc, seq desc):

  * ascending (BlockIteratorV2::seek, block_iterator_v2.rs:269-313, with the restart back-up of
    :157-176 that keeps duplicate keys straddling restarts): FOUND iff the key is present, positioned
    on its FIRST occurrence (the newest version);
  * descending (DescendingBlockIteratorV2::seek, :430-469, forward duplicate scan :178-208): FOUND iff
    present, positioned on its LAST occurrence (the order a descending scan returns it first);
  * a bloom-filtered key is never FOUND; absent keys are POSITIONED / EXHAUSTED, never FOUND.
The GPU kernels are compared with this oracle bit for bit in tests/test_gpu_configs.py.
"""
import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets
from slatedb_amd.batch import Batch


def dup_batch(n=4000, seed=5):
    """Sorted entries with long runs of duplicate keys (up to 40 versions: they straddle restart points
    and blocks), tombstones, merges and timestamps — the shape of block_iterator_v2.rs's proptest (:1522)."""
    rng = np.random.default_rng(seed)
    es, k = [], 0
    while len(es) < n:
        key = b"k%07d" % k + (b"x" * int(rng.integers(0, 40)) if rng.random() < 0.1 else b"")
        for v in range(int(rng.integers(1, 41)) if rng.random() < 0.2 else 1):
            kind = int(rng.choice([0, 0, 0, 1, 2]))
            es.append((key, kind, bytes(rng.integers(0, 256, int(rng.integers(0, 60)), dtype=np.uint8)),
                       10**6 - len(es), int(rng.integers(0, 2**40)) if rng.random() < 0.2 else None,
                       int(rng.integers(0, 2**40)) if rng.random() < 0.2 else None))
        k += int(rng.integers(1, 3))
    return Batch.from_entries(es[:n])


def queries(b, rng, extra=400):
    present = [b.key(i) for i in range(0, b.n, 3)]
    absent = [b"k%07d" % int(rng.integers(0, 10**7)) + bytes(rng.integers(0, 3, int(rng.integers(0, 3)), dtype=np.uint8))
              for _ in range(extra)]
    return present + absent + [b"", b"\x00", b"k", b"\xff" * 9, b.key(0), b.key(b.n - 1)]


@pytest.mark.parametrize("version,bs", [(2, 256), (2, 1024), (2, 4096), (1, 512)])
def test_lookup_properties(version, bs):
    b = dup_batch()
    e = O.encode_sst(b, O.params(block_size=bs, sst_version=version))
    assert e.status == 0
    ik, iko = O.sst_index_keys(b, e)
    keys = queries(b, np.random.default_rng(bs))
    allk = [b.key(i) for i in range(b.n)]
    first, last = {}, {}
    for i, k in enumerate(allk):
        first.setdefault(k, i)
        last[k] = i
    for desc in (False, True):
        r = O.sst_lookup(e.data, e.block_off, ik, iko, keys, descending=desc, sst_version=version)
        assert (r.status == 0).all()
        for q, k in enumerate(keys):
            if k in first:
                assert r.state[q] == _abi.LOOKUP_FOUND, (desc, k)
                g = int(e.block_first_entry[r.block[q]]) + int(r.entry[q])
                assert g == (last[k] if desc else first[k]), (desc, k, g)
                assert r.key_len[q] == len(k) and r.seq[q] == b.seq[g]
            else:
                assert r.state[q] in (_abi.LOOKUP_POSITIONED, _abi.LOOKUP_EXHAUSTED), (desc, k)


def test_lookup_bloom_and_corruption():
    b = datasets.d1(n=20000)
    e = O.encode_sst(b, O.params())
    ik, iko = O.sst_index_keys(b, e)
    keys = [b.key(i) for i in range(0, b.n, 97)] + [b"absent%d" % i for i in range(2000)]
    r = O.sst_lookup(e.data, e.block_off, ik, iko, keys, bloom=e.bloom, num_probes=6)
    assert (r.state[:len(keys) - 2000] == _abi.LOOKUP_FOUND).all()
    fp = r.state[len(keys) - 2000:]
    assert (fp != _abi.LOOKUP_FOUND).all() and (fp == _abi.LOOKUP_FILTERED).sum() > 1900
    data = e.data.copy()
    data[int(e.block_off[5]) + 7] ^= 1
    r = O.sst_lookup(data, e.block_off, ik, iko, [b.key(int(e.block_first_entry[5]) + 3), b.key(0)])
    assert r.status[0] == _abi.SDB_CHECKSUM_MISMATCH and r.status[1] == 0 and r.state[1] == _abi.LOOKUP_FOUND
