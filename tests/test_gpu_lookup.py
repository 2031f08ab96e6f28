"""GPU parity of the batched point lookups / seeks (sdb_sst_lookup, slatedb_amd/csrc/sdb_lookup.hip)
against the oracle restatement (orc_sst_lookup), field by field: state, status, block, entry, key
length, value reference, seq, flags, timestamps.  Ascending and descending, V1 and V2, duplicate keys
straddling restarts and blocks, bloom filtering, a corrupted block."""
import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets

from .test_lookup_oracle import dup_batch, queries

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from slatedb_amd import runtime
    runtime.require_device()
    return runtime


def _dev(a, dt=None):
    import torch
    a = np.ascontiguousarray(a)
    if a.dtype == np.uint64:
        a = a.view(np.int64)
    if not a.size:
        a = np.zeros(16, a.dtype)
    return torch.from_numpy(a).cuda()


def run_both(rt, data, e, ik, iko, keys, version, desc, bloom=None):
    import torch
    koff = np.zeros(len(keys) + 1, np.uint64)
    koff[1:] = np.cumsum([len(k) for k in keys])
    kb = np.frombuffer(b"".join(keys) or b"\0", np.uint8).copy()
    vt = {"data": _dev(data), "block_off": _dev(e.block_off), "num_blocks": len(e.block_off) - 1,
          "index_keys": _dev(ik), "index_key_off": _dev(iko), "sst_version": version}
    if bloom is not None:
        vt.update(bloom=_dev(bloom), bloom_len=len(bloom), num_probes=6)
    got = rt.sst_lookup_device(vt, _dev(kb), _dev(koff), len(keys), desc)
    torch.cuda.synchronize()
    ref = O.sst_lookup(data, e.block_off, ik, iko, keys, descending=desc, sst_version=version,
                       bloom=bloom, num_probes=6 if bloom is not None else 0)
    for f, _ in O.LOOKUP_FIELDS:
        g = got[f][:len(keys)].cpu().numpy()
        r = getattr(ref, f)
        if f in ("create_ts", "expire_ts"):
            bit = _abi.FLAG_HAS_CREATE_TS if f == "create_ts" else _abi.FLAG_HAS_EXPIRE_TS
            m = (ref.flags & bit) != 0
            g, r = g[m], r[m]
        assert np.array_equal(g.astype(np.int64), r.astype(np.int64)), (f, desc, version)
    return ref


@pytest.mark.parametrize("version,bs", [(2, 256), (2, 1024), (2, 4096), (1, 512)])
@pytest.mark.parametrize("desc", [False, True])
def test_lookup_dups(rt, version, bs, desc):
    b = dup_batch()
    e = O.encode_sst(b, O.params(block_size=bs, sst_version=version))
    ik, iko = O.sst_index_keys(b, e)
    keys = queries(b, np.random.default_rng(bs + desc))
    ref = run_both(rt, e.data, e, ik, iko, keys, version, desc)
    assert (ref.state == _abi.LOOKUP_FOUND).sum() >= b.n // 3


@pytest.mark.parametrize("desc", [False, True])
def test_lookup_d1_bloom_corrupt(rt, desc):
    b = datasets.d1(n=60000)
    e = O.encode_sst(b, O.params())
    ik, iko = O.sst_index_keys(b, e)
    rng = np.random.default_rng(3)
    keys = [b.key(int(i)) for i in rng.integers(0, b.n, 3000)] + [bytes(rng.integers(0, 256, 16, dtype=np.uint8)) for _ in range(3000)]
    ref = run_both(rt, e.data, e, ik, iko, keys, 2, desc, bloom=e.bloom)
    assert (ref.state == _abi.LOOKUP_FILTERED).sum() > 2900
    data = e.data.copy()
    for k in (2, 40, 1000):
        data[int(e.block_off[k]) + 100] ^= 0x10
    keys = [b.key(int(e.block_first_entry[k]) + 5) for k in (2, 3, 40, 1000, 1001)]
    ref = run_both(rt, data, e, ik, iko, keys, 2, desc)
    assert (ref.status == _abi.SDB_CHECKSUM_MISMATCH).sum() == 3


def test_lookup_d3_mixed(rt):
    b = datasets.d3(n=3000)
    for version in (1, 2):
        e = O.encode_sst(b, O.params(block_size=1024, sst_version=version))
        ik, iko = O.sst_index_keys(b, e)
        keys = queries(b, np.random.default_rng(version))
        for desc in (False, True):
            run_both(rt, e.data, e, ik, iko, keys, version, desc)
