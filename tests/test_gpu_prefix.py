"""GPU parity of prefix-extractor filters (§8 f4): the device builder (sdb_bloom_build_prefix, and the
encoder with prefix params) and Filter::might_match (sdb_bloom_might_match) against the oracle, bit for
bit, for the fixed / first-delimiter families and caller-supplied lengths, with and without whole-key
filtering."""
import numpy as np
import pytest

from oracle import footer as F
from oracle import oracle as O
from slatedb_amd import datasets
from slatedb_amd.batch import Batch

from .test_gpu_configs import _host_view
from .test_gpu_parity import assert_same, encode_both

pytestmark = pytest.mark.gpu
FIXED, DELIM, LENGTHS = 1, 2, 3


@pytest.fixture(scope="module")
def rt():
    from slatedb_amd import runtime
    runtime.require_device()
    return runtime


def grouped(n=30000, seed=1):
    """GroupId ‖ ':' ‖ suffix keys (the reference's prefix workload), sorted; some without a delimiter."""
    rng = np.random.default_rng(seed)
    keys = set()
    while len(keys) < n:
        g = int(rng.integers(0, n // 20))
        keys.add(b"g%05d:%d" % (g, int(rng.integers(0, 10**6))) if rng.random() > 0.05 else b"nodelim%07d" % g)
    keys = sorted(keys)
    off = np.zeros(len(keys) + 1, np.uint64)
    off[1:] = np.cumsum([len(k) for k in keys])
    return np.frombuffer(b"".join(keys), np.uint8).copy(), off, keys


def lens_of(keys):
    return np.array([(k.index(b":") + 1) if b":" in k else -1 for k in keys], np.int32)


@pytest.mark.parametrize("kind,arg", [(FIXED, 6), (DELIM, ord(":")), (LENGTHS, 0)])
@pytest.mark.parametrize("whole", [True, False])
def test_prefix_build_and_match(rt, kind, arg, whole):
    import torch
    kb, ko, keys = grouped()
    lens = lens_of(keys) if kind == LENGTHS else None
    ref = O.bloom_build_prefix(kb, ko, 10, kind, arg, whole, lens)
    dk, do = torch.from_numpy(kb).cuda(), torch.from_numpy(ko.view(np.int64)).cuda()
    dl = None if lens is None else torch.from_numpy(lens).cuda()
    got = rt.bloom_build_prefix_device(dk, do, len(keys), 10, kind, arg, whole, dl)
    assert np.array_equal(got.cpu().numpy(), ref)
    # might_match over points and prefixes: stored, absent, short, no-delimiter
    rng = np.random.default_rng(2)
    qs = [keys[int(i)] for i in rng.integers(0, len(keys), 500)] + [b"g%05d:" % i for i in range(600)]
    qs += [b"h%05d:x" % i for i in range(300)] + [b"g0", b"", b"nodelim0000001", b"zz"]
    isp = np.array([i % 3 == 0 for i in range(len(qs))], np.uint8)
    ql = lens_of(qs) if kind == LENGTHS else None
    qo = np.zeros(len(qs) + 1, np.uint64)
    qo[1:] = np.cumsum([len(q) for q in qs])
    qb = np.frombuffer(b"".join(qs), np.uint8).copy()
    res = rt.might_match_device(torch.from_numpy(np.ascontiguousarray(ref)).cuda() if len(ref) else torch.zeros(0, dtype=torch.uint8, device="cuda"),
                                6, whole, kind, arg, torch.from_numpy(qb).cuda(), torch.from_numpy(qo.view(np.int64)).cuda(),
                                len(qs), torch.from_numpy(isp).cuda(), None if ql is None else torch.from_numpy(ql).cuda())
    want = [O.might_match(ref, 6, whole, kind, arg, q, bool(isp[i]), -1 if ql is None else int(ql[i])) for i, q in enumerate(qs)]
    assert np.array_equal(res.cpu().numpy().astype(bool), np.array(want))


@pytest.mark.parametrize("kind,arg,whole", [(FIXED, 7, True), (DELIM, ord(":"), False), (LENGTHS, 0, True)])
def test_encode_with_prefix_filter(rt, kind, arg, whole):
    """The encoder with prefix params: data section + device-counted filter, and the whole SST object
    under the policy's name."""
    kb, ko, keys = grouped(20000, seed=4)
    lens = lens_of(keys) if kind == LENGTHS else None
    rng = np.random.default_rng(5)
    vals = [bytes(rng.integers(0, 256, 40, dtype=np.uint8)) for _ in keys]
    b = Batch.from_entries([(k, 0, v, 0, None, None) for k, v in zip(keys, vals)])
    b.prefix_len = lens
    kw = dict(block_size=4096, prefix_kind=kind, prefix_arg=arg, no_whole_key=0 if whole else 1)
    ref, got = encode_both(rt, b, **kw)
    assert ref.summary.bloom_len > 0
    assert_same(ref, got, "prefix encode")
    prm = rt.params(**kw)
    name = rt.filter_name(prm)
    assert rt.sst_object(b, got, filter_name=name) == F.sst_object(b, ref, filter_name=name)
