"""GPU parity: the HIP path (through the C ABI) against the CPU oracle, bit for bit.

Byte/integer work, so the bar is exact equality of every output array: data section (blocks +
CRC32), block offsets, first entries, index-key lengths, block stats, bloom bitmap, summary
counters and error codes; decode outputs field by field.  Cases mirror the reference's tests
(sst_builder.rs:593-1892, format/block_v2.rs:282-630, filter.rs:250-367, sst_iter.rs) plus the
datasets of SURVEY.md §8d.
"""
import struct
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets
from slatedb_amd.batch import Batch

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from slatedb_amd import runtime
    runtime.require_device()
    return runtime


def encode_both(rt, batch, **kw):
    prm = O.params(**kw)
    ref = O.encode_sst(batch, prm)
    enc = rt.Encoder(rt.params(**kw))
    got = enc.encode(batch)
    enc.close()
    return ref, got


def assert_same(ref, got, what=""):
    assert got.status == ref.status, (what, got.status, ref.status, got.summary)
    if ref.status != 0:
        assert got.summary["first_error_entry"] == ref.summary.first_error_entry, what
        return
    for f in ("data_len", "num_blocks", "num_entries", "raw_key_size", "raw_val_size", "num_puts",
              "num_deletes", "num_merges", "bloom_len", "num_probes", "filter_built", "max_block_entries"):
        if f == "max_block_entries":
            # device reports the longest candidate block, the oracle the longest actual one
            assert got.summary[f] >= getattr(ref.summary, f), (what, f)
            continue
        assert got.summary[f] == getattr(ref.summary, f), (what, f, got.summary[f], getattr(ref.summary, f))
    assert np.array_equal(got.block_off, ref.block_off), what
    assert np.array_equal(got.block_first_entry, ref.block_first_entry), what
    assert np.array_equal(got.index_key_len, ref.index_key_len), what
    assert np.array_equal(got.block_stats, ref.block_stats), what
    if not np.array_equal(got.data, ref.data):
        bad = np.nonzero(got.data != ref.data)[0]
        blk = np.searchsorted(ref.block_off, bad[0], side="right") - 1
        raise AssertionError("%s: data differs at byte %d (block %d), %d bytes differ" % (what, bad[0], blk, len(bad)))
    assert np.array_equal(got.bloom, ref.bloom), what


def ent(key, value=b"", seq=0, kind=0, create=None, expire=None):
    key = key.encode() if isinstance(key, str) else key
    value = value.encode() if isinstance(value, str) else value
    return (key, kind, value, seq, create, expire)


# ------------------------------------------------------------------------------------------------
# encode
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("n", [1, 2, 33, 34, 35, 1000, 20000])
def test_d1_prefixes(rt, n):
    ref, got = encode_both(rt, datasets.d1(n=n))
    assert_same(ref, got, "d1 n=%d" % n)


def test_d1_full_64mib(rt):
    """configs[1]: one 64 MiB L0 SST, bit-exact vs the oracle (578,524 entries, 17,016 blocks)."""
    b = datasets.d1()
    ref, got = encode_both(rt, b)
    assert ref.summary.num_blocks == 17016 and ref.summary.bloom_len == 723155
    assert_same(ref, got, "d1 full")


def test_d1_seq_desc_and_d2(rt):
    ref, got = encode_both(rt, datasets.d1(n=50000, seq_desc=True))
    assert_same(ref, got, "d1 seq desc")
    ref, got = encode_both(rt, datasets.d2(n=50000))
    assert_same(ref, got, "d2")


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("block_size", [64, 256, 1024, 4096])
def test_d3_mixed(rt, version, block_size):
    b = datasets.d3(n=3000)
    ref, got = encode_both(rt, b, sst_version=version, block_size=block_size)
    assert_same(ref, got, "d3 v%d bs%d" % (version, block_size))


@pytest.mark.parametrize("ri", [1, 2, 4, 32])
def test_restart_intervals(rt, ri):
    ref, got = encode_both(rt, datasets.d3(n=2000), restart_interval=ri, block_size=2048)
    assert_same(ref, got, "ri=%d" % ri)


def test_sst500(rt):
    from tests.test_oracle_kats import sst500_batch
    ref, got = encode_both(rt, sst500_batch(), block_size=1024)
    assert ref.summary.data_len == 21998
    assert_same(ref, got, "sst500")


def test_oversize_and_large_blocks(rt):
    rng = np.random.default_rng(5)
    es = []
    for i in range(300):
        vlen = 6000 if i % 17 == 0 else int(rng.integers(0, 200))
        es.append(ent(b"k%06d" % i, bytes(rng.integers(0, 256, vlen, dtype=np.uint8)), i))
    b = Batch.from_entries(es)
    for bs in (4096, 16384, 65536):
        ref, got = encode_both(rt, b, block_size=bs)
        assert_same(ref, got, "oversize bs=%d" % bs)
    ref, got = encode_both(rt, b, block_size=4096, sst_version=1)
    assert_same(ref, got, "oversize v1")


def test_long_keys_and_tiny_entries(rt):
    es = [ent(b"p" * 300 + b"%05d" % i, b"", i) for i in range(500)]
    ref, got = encode_both(rt, Batch.from_entries(es), block_size=4096)
    assert_same(ref, got, "long keys")
    es = [ent(bytes([65 + i % 26]) + struct.pack(">I", i), b"", i) for i in range(5000)]
    es.sort(key=lambda e: e[0])
    ref, got = encode_both(rt, Batch.from_entries(es), block_size=4096)
    assert_same(ref, got, "tiny entries")


def test_empty_and_min_filter_keys(rt):
    ref, got = encode_both(rt, Batch.from_entries([]))
    assert_same(ref, got, "empty")
    b = datasets.d1(n=500)
    ref, got = encode_both(rt, b, min_filter_keys=1000)  # num_rows < min_filter_keys: no filter
    assert not ref.summary.filter_built
    assert_same(ref, got, "min_filter_keys")
    ref, got = encode_both(rt, b, bloom_bits_per_key=0)
    assert_same(ref, got, "no policy")


def test_error_codes(rt):
    cases = [
        [ent(b"", "v")],                                  # EmptyKey (block_v2.rs:168)
        [ent("a", "v"), ent("b", "v"), ent(b"", "v")],    # assert in compute_lower_bound
        [ent("abc", "v"), ent("ab", "v")],                # out-of-bounds panic in compute_lower_bound
    ]
    for es in cases:
        ref, got = encode_both(rt, Batch.from_entries(es))
        assert ref.status != 0
        assert_same(ref, got, "errors")
    ref, got = encode_both(rt, Batch.from_entries([ent("a", "v"), ent(b"k" * 70000, "v")]), sst_version=1)
    assert ref.status == _abi.SDB_LIMIT_EXCEEDED
    assert_same(ref, got, "v1 u16")
    bad = Batch.from_entries([ent("a", "v"), ent("b", "v")])
    bad.kind[1] = 7
    ref, got = encode_both(rt, bad)
    assert ref.status == _abi.SDB_INVALID_ARGUMENT
    assert_same(ref, got, "bad kind")


def test_builder_mirror(rt):
    """EncodedSsTableBuilder-style add()/build()/next_block() (sst_builder.rs:224-276)."""
    b = datasets.d3(n=700)
    bld = rt.SstBuilder(rt.params(block_size=512))
    for i in range(b.n):
        m = int(b.ts_mask[i])
        bld.add(b.key(i), b.value(i), int(b.seq[i]), int(b.kind[i]),
                int(b.create_ts[i]) if m & 1 else None, int(b.expire_ts[i]) if m & 2 else None)
    got = bld.build()
    ref = O.encode_sst(b, O.params(block_size=512))
    assert_same(ref, got, "builder")
    blocks = []
    while True:
        x = got.next_block()
        if x is None:
            break
        assert struct.unpack(">I", x[-4:])[0] == zlib.crc32(x[:-4])
        blocks.append(x)
    assert b"".join(blocks) == ref.data.tobytes()


# ------------------------------------------------------------------------------------------------
# bloom
# ------------------------------------------------------------------------------------------------
# (n, bpk): tiny filters (one slice), the dense build at k <= 7 (8 keys per thread) and k 8..15 (4 per
# thread), several slices per k_bloom_or workgroup (2 M keys: 306 slices), and k = 16 (no binned plan:
# the atomic build)
@pytest.mark.parametrize("n,bpk", [(1, 10), (7, 10), (1000, 10), (200000, 10), (100000, 7), (5, 1), (300000, 12),
                                   (50000, 21), (20000, 24), (2000000, 10), (8193, 10)])
def test_bloom_bitmap(rt, n, bpk):
    kb, ko = datasets.c4_keys(n=n, seed=11 + n)
    ref = O.bloom_build(kb, ko, bpk)
    got = rt.BloomFilterPolicy(bpk).build(Batch(kb, ko, np.zeros(0, np.uint8), np.zeros(len(ko), np.uint64)))
    assert got[:2] == struct.pack(">H", O.optimal_num_probes(bpk))
    assert got[2:] == ref.tobytes()


def test_bloom_bitmap_ragged_keys(rt):
    """Keys of 0..40 bytes at unaligned offsets (the generic SipHash path of the dense build)."""
    rng = np.random.default_rng(5)
    lens = rng.integers(0, 41, 150000).astype(np.uint64)
    ko = np.concatenate([[0], np.cumsum(lens)]).astype(np.uint64)
    kb = rng.integers(0, 256, int(ko[-1]), dtype=np.uint8)
    ref = O.bloom_build(kb, ko, 10)
    got = rt.BloomFilterPolicy(10).build(Batch(kb, ko, np.zeros(0, np.uint8), np.zeros(len(ko), np.uint64)))
    assert got[2:] == ref.tobytes()


def test_bloom_fp_kat_on_gpu(rt):
    # filter.rs:331-367 on the device builder + device prober: exactly 870 false positives
    n = 100000
    keys = np.arange(n, dtype=">u4").view(np.uint8).copy()
    off = np.arange(n + 1, dtype=np.uint64) * np.uint64(4)
    enc = rt.BloomFilterPolicy(10).build(Batch(keys, off, np.zeros(0, np.uint8), np.zeros(n + 1, np.uint64)))
    bm = np.frombuffer(enc[2:], np.uint8)
    assert rt.might_contain(bm, 6, [struct.pack(">I", i) for i in range(n)]).all()
    fp = rt.might_contain(bm, 6, [struct.pack(">I", i) for i in range(n, 2 * n)]).sum()
    assert fp == 870
    assert not rt.might_contain(np.zeros(0, np.uint8), 6, [b"x"]).any()  # empty bitmap guard


# ------------------------------------------------------------------------------------------------
# decode
# ------------------------------------------------------------------------------------------------
def assert_decode_same(ref, got, what=""):
    assert got.status == ref.status, (what, got.status, ref.status)
    assert got.n == ref.n, what
    assert np.array_equal(got.block_entry_start, ref.block_entry_start), what
    for f in ("key_off", "val_off", "val_len", "seq", "flags"):
        assert np.array_equal(getattr(got, f), getattr(ref, f)), (what, f)
    # timestamps are valid iff the row's flag says so (include/slatedb_amd.h, sdb_decoded_out)
    for f, bit in (("create_ts", _abi.FLAG_HAS_CREATE_TS), ("expire_ts", _abi.FLAG_HAS_EXPIRE_TS)):
        m = (ref.flags & bit) != 0
        assert np.array_equal(getattr(got, f)[m], getattr(ref, f)[m]), (what, f)
    assert np.array_equal(got.key_arena, ref.key_arena), what
    assert sorted(got.bad_block.tolist()) == sorted(ref.bad_block.tolist()), what


@pytest.mark.parametrize("version", [1, 2])
def test_decode_d3(rt, version):
    b = datasets.d3(n=3000)
    enc = O.encode_sst(b, O.params(sst_version=version, block_size=1024))
    ref = O.decode_blocks(enc.data, enc.block_off, version)
    dec = rt.Decoder()
    got = dec.decode(enc.data, enc.block_off, version)
    assert_decode_same(ref, got, "d3 v%d" % version)


def test_decode_d1_and_corruption(rt):
    b = datasets.d1(n=40000)
    enc = O.encode_sst(b, O.params())
    dec = rt.Decoder()
    got = dec.decode(enc.data, enc.block_off, 2)
    ref = O.decode_blocks(enc.data, enc.block_off, 2)
    assert_decode_same(ref, got, "d1")
    data = enc.data.copy()
    for k in (3, 77, 500):
        data[int(enc.block_off[k]) + 11] ^= 0x40
    got = dec.decode(data, enc.block_off, 2)
    ref = O.decode_blocks(data, enc.block_off, 2)
    assert ref.status == _abi.SDB_CHECKSUM_MISMATCH
    assert_decode_same(ref, got, "corrupt")


def test_decode_large_blocks_and_flags(rt):
    rng = np.random.default_rng(9)
    es = [ent(b"k%06d" % i, bytes(rng.integers(0, 256, 9000 if i % 5 == 0 else 50, dtype=np.uint8)), i)
          for i in range(200)]
    enc = O.encode_sst(Batch.from_entries(es), O.params(block_size=65536))
    dec = rt.Decoder()
    assert_decode_same(O.decode_blocks(enc.data, enc.block_off, 2), dec.decode(enc.data, enc.block_off, 2), "big")
    blk = bytearray(O.encode_row(2, 0, b"k", 0, b"v", 7))
    blk[-1] = 0x10
    body = bytes(blk) + struct.pack(">HH", 0, 1)
    body += struct.pack(">I", zlib.crc32(body))
    arr = np.frombuffer(body, np.uint8)
    off = np.array([0, len(body)], np.uint64)
    assert_decode_same(O.decode_blocks(arr, off, 2), dec.decode(arr, off, 2), "flags")


def test_device_round_trip_full_d1(rt):
    """Encode on the GPU, decode on the GPU: size-independent round-trip property at full size."""
    b = datasets.d1()
    enc = rt.Encoder(rt.params()).encode(b)
    assert enc.status == 0
    d = rt.Decoder().decode(enc.data, enc.block_off, 2)
    assert d.status == 0 and d.n == b.n
    assert np.array_equal(d.key_arena, b.key_bytes)
    assert np.array_equal(d.key_off, b.key_off)
    assert (d.val_len == 100).all()
    vals = enc.data[(d.val_off[:, None] + np.arange(100, dtype=np.uint64)).astype(np.int64)]
    assert np.array_equal(vals.reshape(-1), b.val_bytes)


@pytest.mark.gpu
@pytest.mark.parametrize("n", [5000, 100000, datasets.D1_N])
def test_bloom_slots_do_not_overflow(rt, n):
    """The fused bloom's (tile, slice) slots are sized for uniform probes: D1-shaped batches must take
    the slotted fill (no overflowing run), not the rebuild-from-keys fallback."""
    import ctypes as C
    import torch
    runtime = rt
    b = datasets.d1(n=n)
    prm = runtime.params(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    out = runtime.DeviceSstOutput(b.n, b.logical_bytes(), b.logical_bytes(), prm)
    runtime.encode_sst_device(b.to_device("cuda"), out)
    torch.cuda.synchronize()
    got = out.to_host()
    ref = O.encode_sst(b, O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10))
    assert np.array_equal(got["bloom"], ref.bloom)
    cd = C.CDLL(runtime.LIB_PATH)
    cd.sdb_diag_bloom_slots.restype = C.c_uint64
    cd.sdb_diag_bloom_slots.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    tiles, nsl, cap = C.c_uint32(), C.c_uint32(), C.c_uint32()
    off = cd.sdb_diag_bloom_slots(b.n, C.byref(prm), C.byref(tiles), C.byref(nsl), C.byref(cap))
    cnt = out.workspace[off: off + 4 * tiles.value * nsl.value].cpu().numpy().view(np.uint32)
    assert (cnt <= cap.value).all(), "a bloom slot overflowed"
    assert int(cnt.sum()) == n * 6


# ------------------------------------------------------------------------------------------------
# whole SST object (§8 f1): GPU data section + host footer from the device's per-block outputs
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("case", ["d1", "d3v1", "d3v2", "sst500", "sst500_wal", "wal_insertion_order"])
def test_whole_sst_object(rt, case):
    from oracle import footer as F
    from .test_oracle_kats import sst500_batch
    kw, sst_type = {}, _abi.SST_COMPACTED
    if case == "d1":
        b = datasets.d1()
    elif case.startswith("d3"):
        b = datasets.d3(n=3000)
        kw = dict(sst_version=int(case[-1]), block_size=512)
    elif case == "wal_insertion_order":
        from .test_footer import _wal_batch
        b, kw, sst_type = _wal_batch(), dict(block_size=1024), _abi.SST_WAL
    else:
        b = sst500_batch()
        kw = dict(block_size=1024)
        if case.endswith("wal"):
            sst_type = _abi.SST_WAL
    ref, got = encode_both(rt, b, sst_type=sst_type, **kw)
    assert_same(ref, got, case)
    v = kw.get("sst_version", 2)
    want = F.sst_object(b, ref, sst_version=v, sst_type=sst_type)
    obj = rt.sst_object(b, got, sst_version=v, sst_type=sst_type)
    assert obj == want, case
    if case == "sst500":
        assert len(obj) == 23794
    if case == "sst500_wal":
        assert len(obj) == 22928


def test_decode_small_batches(rt):
    """<= 1024 blocks take the fused path (scan inside k_dec_emit, last workgroup finishes): the
    2 MiB read_blocks granularity (~520 blocks, format/sst.rs:919-978); 1025 takes the scan kernels."""
    b = datasets.d1(n=40000)
    enc = O.encode_sst(b, O.params())
    dec = rt.Decoder()
    for b0, b1 in [(0, 1), (0, 520), (520, 1040), (0, 1024), (0, 1025), (100, 1124), (1170, enc.summary.num_blocks)]:
        off = enc.block_off[b0:b1 + 1]
        got = dec.decode(enc.data, off, 2)
        assert_decode_same(O.decode_blocks(enc.data, off, 2), got, "range %d-%d" % (b0, b1))
    data = enc.data.copy()
    data[int(enc.block_off[600]) + 5] ^= 1
    off = enc.block_off[520:1040 + 1]
    ref = O.decode_blocks(data, off, 2)
    assert ref.status == _abi.SDB_CHECKSUM_MISMATCH
    assert_decode_same(ref, dec.decode(data, off, 2), "small corrupt")
