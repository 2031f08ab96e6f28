"""Pin the CPU oracle (oracle/sdb_oracle.c) against every exact fixture the reference holds for this
path.  CPU only.

Reference tests restated here (paths relative to slatedb/src):
  utils.rs:1615-1680 varint KATs          utils.rs:846-887 index-key KATs
  format/block.rs:250-350 V1 snapshots    format/row.rs:288-465 V0 row snapshots
  format/block_v2.rs:282-630 V2 builder   format/block_v2.rs:636-890 V1-vs-V2 size table
  filter.rs:250-367 bloom bit/probe/FP    sst_builder.rs:484-584 500-entry SST size
"""
import os
import struct
import subprocess
import sys
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi
from slatedb_amd.batch import Batch


def ent(key, value=b"", seq=0, kind=0, create=None, expire=None):
    if isinstance(key, str):
        key = key.encode()
    if isinstance(value, str):
        value = value.encode()
    return (key, kind, value, seq, create, expire)


# ------------------------------------------------------------------------------------------------
# utils.rs
# ------------------------------------------------------------------------------------------------
def test_varint_kats(golden):
    for v, n in golden["varint_len_kat"]:
        assert O.varint_len(v) == n
    for v, hx in golden["varint_encode_kat"]:
        assert O.encode_varint(v).hex() == hx


def test_index_key_kats(golden):
    for prev, first, exp in golden["index_key_kat"]:
        p = None if prev is None else prev.encode("latin-1")
        assert O.index_key(p, first.encode("latin-1")) == exp.encode("latin-1")
    for prev, first in golden["index_key_panics"]:
        assert O.index_key(prev.encode(), first.encode()) is None


def test_compute_prefix_kats(golden):
    for a, b, n in golden["prefix_kat"]:
        assert O.compute_prefix(a.encode(), b.encode()) == n
    # chunked path (>128 B) of compute_prefix_chunks::<128> (block_v2.rs:65-75)
    a = b"x" * 300 + b"a"
    assert O.compute_prefix(a, b"x" * 300 + b"b") == 300
    assert O.compute_prefix(b"y" * 256, b"y" * 256) == 256


# ------------------------------------------------------------------------------------------------
# filter.rs
# ------------------------------------------------------------------------------------------------
def test_probes_kat(golden):
    k = golden["probes_kat"]
    assert O.probes_for_key(k["hash"], k["num_probes"], k["filter_bits"]) == k["probes"]


def test_optimal_num_probes_and_sizes():
    assert O.optimal_num_probes(10) == 6          # (10 as f32 * 0.69) as u16
    assert O.optimal_num_probes(1) == 0
    assert O.optimal_num_probes(20) == 13
    assert O.filter_size_bytes(0, 10) == 0        # estimate_encoded_size(0,10) - 2 (filter.rs:414)
    assert O.filter_size_bytes(1, 10) == 2
    assert O.filter_size_bytes(100, 10) == 125
    assert O.filter_size_bytes(578524, 10) == 723155
    assert O.filter_size_bytes(10_000_000, 10) == 12_500_000


def test_set_bit_is_lsb_first(golden):
    # set_bit KATs (filter.rs:250-266): bit b lives in byte b/8 at position b%8.
    for before, after, bit in golden["set_bit_kat"]:
        buf = bytearray(bytes.fromhex(before))
        buf[bit // 8] |= 1 << (bit % 8)
        assert buf.hex() == after
    # The oracle's bitmap uses exactly that convention for every probe of a key.
    keys = np.frombuffer(b"somekey!", np.uint8).copy()
    bm = O.bloom_build(keys, np.array([0, 8], np.uint64), 10)
    m = len(bm) * 8
    for p in O.probes_for_key(O.filter_hash(b"somekey!"), 6, m):
        assert bm[p // 8] & (1 << (p % 8))
    assert O.might_contain(bm, 6, b"somekey!")


SIPHASH24_VECTORS = {  # SipHash-2-4 reference vectors (Aumasson & Bernstein), key 00..0f, msg 00..n-1
    0: 0x726FDB47DD0E0E31,
    1: 0x74F839C593DC67FD,
}


def test_siphash_machinery_pinned():
    key = bytes(range(16))
    k0, k1 = struct.unpack("<QQ", key)
    for n, exp in SIPHASH24_VECTORS.items():
        assert O.siphash(bytes(range(n)), k0, k1, 2, 4) == exp
    # CPython 3.10 hashes bytes with zero-key SipHash-2-4 under PYTHONHASHSEED=0
    msgs = [b"a", b"slatedb", bytes(range(15)), bytes(range(16)), b"x" * 33]
    code = "import sys\nfor m in %r: print(hash(m))" % (msgs,)
    env = dict(os.environ, PYTHONHASHSEED="0")
    outs = subprocess.check_output([sys.executable, "-c", code], env=env).split()
    for m, o in zip(msgs, outs):
        h = O.siphash(m, 0, 0, 2, 4)
        s = h - (1 << 64) if h >= 1 << 63 else h
        if s == -1:
            s = -2
        assert int(o) == s


def test_bloom_fp_rate_kat(golden):
    # filter.rs:331-367: 100k u32 BE keys at 10 bpk, FP over the next 100k keys < 1 % (observed .0087)
    kat = golden["bloom_fp_kat"]
    n = kat["keys"]
    keys = np.arange(n, dtype=">u4").view(np.uint8).copy()
    off = np.arange(n + 1, dtype=np.uint64) * np.uint64(4)
    bm = O.bloom_build(keys, off, kat["bits_per_key"])
    for i in range(0, n, 997):
        assert O.might_contain(bm, 6, struct.pack(">I", i))
    fp = sum(O.might_contain(bm, 6, struct.pack(">I", i)) for i in range(n, 2 * n))
    assert fp / n < kat["bound"]
    # The reference comment records the observed rate 0.0087; SipHash-1-3 outputs are otherwise
    # unpinned, so report how close the restatement lands (see DESIGN.md "Parity").
    # 0.0087 of 100,000 queries is exactly 870 false positives: a wrong hash, probe sequence or
    # bitmap size would land on 870 only by chance (~1/75), so this is the end-to-end bloom KAT.
    assert fp == round(kat["observed_fp"] * n) == 870


def test_crc32_matches_zlib():
    rng = np.random.default_rng(7)
    for n in (0, 1, 7, 8, 9, 63, 64, 4019, 70000):
        b = rng.integers(0, 256, n, dtype=np.uint8).tobytes()
        assert O.crc32(b) == zlib.crc32(b)


# ------------------------------------------------------------------------------------------------
# format/block.rs + format/row.rs snapshots
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("name", ["test_block", "block_with_tombstone", "block_with_merge"])
def test_v1_block_snapshots(golden, name):
    snap = golden["v1_block_snapshots"][name]
    es = [ent(e["key"], e["value"], e["seq"], e["kind"], e["create_ts"], e["expire_ts"])
          for e in snap["entries"]]
    st, enc, acc = O.build_block(Batch.from_entries(es), version=1, block_size=4096)
    assert st == 0 and acc.all()
    data = bytes.fromhex(snap["data_hex"])
    assert len(enc) == snap["size"]
    assert enc[:len(data)] == data
    offs = list(struct.unpack(">%dH" % len(snap["offsets"]), enc[len(data):-2]))
    assert offs == snap["offsets"]
    assert struct.unpack(">H", enc[-2:])[0] == len(snap["offsets"])


def _lossy(b):
    return b.decode("utf-8", errors="replace")


def test_v0_row_snapshots(golden):
    rows = golden["v0_row_snapshots"]
    assert len(rows) == 10
    for name, r in rows.items():
        i = r["input"]
        val = None if i["value_hex"] is None else bytes.fromhex(i["value_hex"])
        kind = 2 if val is None else 0
        enc = O.encode_row(1, i["prefix"], bytes.fromhex(i["suffix_hex"]), kind, val, i["seq"],
                           i["create_ts"], i["expire_ts"])
        assert _lossy(enc) == r["encoded_lossy"], name
        # decode through a 2-row V1 block whose first row carries the first key
        first = bytes.fromhex(i["first_key_hex"])
        row0 = O.encode_row(1, 0, first, 0, b"", 0)
        data = row0 + enc
        blk = data + struct.pack(">HHH", 0, len(row0), 2)
        blk += struct.pack(">I", zlib.crc32(blk))
        if not first:
            continue  # an empty first key cannot head a real block; the encode half is pinned above
        d = O.decode_blocks(np.frombuffer(blk, np.uint8), np.array([0, len(blk)], np.uint64), 1)
        assert d.status == 0 and d.n == 2, name
        key = d.key_arena[int(d.key_off[1]):int(d.key_off[2])].tobytes()
        assert key.hex() == r["full_key_hex"], name
        assert int(d.seq[1]) == r["seq"]
        fl = int(d.flags[1])
        assert bool(fl & 1) == r["tombstone"]
        assert (int(d.create_ts[1]) if fl & 4 else None) == r["create_ts"]
        assert (int(d.expire_ts[1]) if fl & 2 else None) == r["expire_ts"]


# ------------------------------------------------------------------------------------------------
# format/block_v2.rs structure tests and the V1/V2 size table
# ------------------------------------------------------------------------------------------------
def _v2_rows(enc):
    cnt = struct.unpack(">H", enc[-2:])[0]
    offs = struct.unpack(">%dH" % cnt, enc[-2 - 2 * cnt:-2]) if cnt else ()
    return enc[:len(enc) - 2 - 2 * cnt], list(offs)


def test_v2_builder_structure():
    # should_build_single_entry_block
    st, enc, _ = O.build_block(Batch.from_entries([ent("key1", "value1", 1)]), 2, 4096)
    assert _v2_rows(enc)[1] == [0]
    # should_handle_various_restart_intervals: restarts == ceil(50 / interval)
    es = [ent("key_%05d" % i, "value_%d" % i, i) for i in range(50)]
    for interval in (1, 2, 4, 16, 32):
        st, enc, _ = O.build_block(Batch.from_entries(es), 2, 8192, interval)
        assert len(_v2_rows(enc)[1]) == -(-50 // interval)
    # should_use_prefix_compression_between_restarts: shared=9, suffix b"b"
    st, enc, _ = O.build_block(Batch.from_entries([ent("prefix_aaa", "v1", 1), ent("prefix_aab", "v2", 2)]), 2, 4096)
    data, offs = _v2_rows(enc)
    row0 = O.encode_row(2, 0, b"prefix_aaa", 0, b"v1", 1)
    assert data[:len(row0)] == row0
    assert data[len(row0):len(row0) + 4] == bytes([9, 1, 2]) + b"b"
    # should_store_full_key_at_restart_points (interval 2)
    st, enc, _ = O.build_block(Batch.from_entries(
        [ent("prefix_aaa", "v1", 1), ent("prefix_aab", "v2", 2), ent("prefix_bbb", "v3", 3)]), 2, 4096, 2)
    data, offs = _v2_rows(enc)
    assert data[offs[1]:offs[1] + 3] == bytes([0, 10, 2])
    # should_reject_entry_exceeding_block_size / should_accept_first_entry_exceeding_block_size
    st, enc, acc = O.build_block(Batch.from_entries([ent("key1", "value1", 1), ent("key2", b"x" * 200, 2)]), 2, 100)
    assert list(acc) == [1, 0]
    st, enc, acc = O.build_block(Batch.from_entries([ent("key1", b"x" * 200, 1)]), 2, 10)
    assert list(acc) == [1]
    # should_encode_with_varints (row_codec_v2.rs:352-381)
    r = O.encode_row(2, 3, b"abc", 0, b"xyz", 1)
    assert r[:9] == bytes([3, 3, 3]) + b"abcxyz"
    assert len(r) == 3 + 3 + 3 + 8 + 1
    # 2-/3-byte varints
    r = O.encode_row(2, 20000, b"k" * 20000, 0, b"v" * 20000, 1)
    assert r[:3] == O.encode_varint(20000)
    # large key requiring u32 varint lengths
    big = b"k" * (3 * 1024 * 1024)
    st, enc, acc = O.build_block(Batch.from_entries([ent(big, "small_value", 1)]), 2, 4 * 1024 * 1024)
    assert st == 0 and enc[:1] == b"\x00" and enc[1:5] == O.encode_varint(len(big))


def _size_scenarios():
    """Entry lists of block_size_comparison (format/block_v2.rs:747-890)."""
    E = lambda k, v, s: ent(k, v, s)
    S = {}
    S["Sequential keys (key0001..key0100)"] = [E("key%04d" % i, "value", i) for i in range(1, 101)]
    S["Sequential keys, 100-byte values"] = [E("key%04d" % i, b"v" * 100, i) for i in range(1, 101)]
    pre = "com.example.application.module.submodule."
    S["Long common prefix (90% shared)"] = [E("%s%04d" % (pre, i), "value", i) for i in range(1, 101)]
    S["Random keys (no common prefix)"] = [
        E("%08x%08x" % (i * 2654435761, i * 1597334677), "value", i) for i in range(1, 101)]
    S["Few entries (10 sequential)"] = [E("key%04d" % i, "value", i) for i in range(1, 11)]
    S["Many small entries (500)"] = [E("k%04d" % i, "v", i) for i in range(1, 501)]
    S["Tombstones (100 sequential keys)"] = [ent("key%04d" % i, b"", i, 2) for i in range(1, 101)]
    S["Mixed: 50% values, 50% tombstones"] = [
        E("key%04d" % i, "value", i) if i % 2 == 0 else ent("key%04d" % i, b"", i, 2) for i in range(1, 101)]
    S["Varying value sizes (1-500 bytes)"] = [E("key%04d" % i, b"v" * ((i * 5) % 500 + 1), i) for i in range(1, 101)]
    S["Large values (1KB each)"] = [E("key%04d" % i, b"v" * 1024, i) for i in range(1, 51)]
    S["Short keys (1-3 chars)"] = [E(chr(ord("a") + i % 26), "value", i) for i in range(1, 101)]
    S["UUID-like keys"] = [E("%08x-%04x-%04x-%04x-%012x" % (i * 12345, i * 67, i * 89, i * 101, i * 112131),
                             "value", i) for i in range(1, 101)]
    S["Hierarchical paths (/a/b/c/...)"] = [
        E("".join("/level%d" % d for d in range(i % 5 + 1)) + "/item%04d" % i, "value", i) for i in range(1, 101)]
    S["With create timestamps"] = [ent("key%04d" % i, "value", i, 0, 1700000000000 + i) for i in range(1, 101)]
    S["With create and expire timestamps"] = [
        ent("key%04d" % i, "value", i, 0, 1700000000000 + i, 1800000000000 + i) for i in range(1, 101)]
    return S


def test_block_size_table(golden):
    scen = _size_scenarios()
    table = golden["block_size_table_64k"]
    assert len(table) == 15
    for row in table:
        es = scen[row["scenario"]]
        assert len(es) == row["entries"]
        b = Batch.from_entries(es)
        st1, e1, _ = O.build_block(b, 1, 64 * 1024)
        st2, e2, _ = O.build_block(b, 2, 64 * 1024)
        assert (len(e1), len(e2)) == (row["v1"], row["v2"]), row["scenario"]


# ------------------------------------------------------------------------------------------------
# sst_builder.rs:484-584 — 500-entry SST at block_size 1024
# ------------------------------------------------------------------------------------------------
def _bitrev64(i):
    return int("{:064b}".format(i)[::-1], 2)


def sst500_batch():
    keys = sorted(struct.pack(">QQ", _bitrev64(i), i) for i in range(500))
    return Batch.from_entries([ent(k, b"val%013d" % i, i + 1) for i, k in enumerate(keys)])


def test_sst500_data_section():
    r = O.encode_sst(sst500_batch(), O.params(block_size=1024, bloom_bits_per_key=10, min_filter_keys=0))
    assert r.status == 0
    # derived from the reference's estimate-vs-actual assertion: data 21,998 B in 22
    # blocks (23 entries each except the last); composite filter block 646 B = 2+2+3+8+(2+625)+4.
    assert r.summary.data_len == 21998
    assert r.summary.num_blocks == 22
    assert list(np.diff(r.block_first_entry)[:-1]) == [23] * 21
    assert r.summary.bloom_len == 625 and 2 + 2 + 3 + 8 + 2 + 625 + 4 == 646
    # every block ends with its CRC32 (BE) over Block::encode (format/sst.rs:541-552)
    for k in range(22):
        s, e = int(r.block_off[k]), int(r.block_off[k + 1])
        blk = r.data[s:e].tobytes()
        assert struct.unpack(">I", blk[-4:])[0] == zlib.crc32(blk[:-4])
    assert r.index_key_len[0] == 0


def test_encode_errors():
    p = O.params()
    r = O.encode_sst(Batch.from_entries([ent(b"", "v")]), p)
    assert r.status == _abi.SDB_EMPTY_KEY
    r = O.encode_sst(Batch.from_entries([ent("a", "v"), ent(b"", "v")]), p)
    assert r.status == _abi.SDB_EMPTY_KEY and r.summary.first_error_entry == 1
    r = O.encode_sst(Batch.from_entries([ent("abc", "v"), ent("ab", "v")]), p)  # panics in compute_lower_bound
    assert r.status == _abi.SDB_INVALID_ARGUMENT
    # V1 u16 asserts (row.rs:73-85)
    r = O.encode_sst(Batch.from_entries([ent(b"k" * 70000, "v")]), O.params(sst_version=1))
    assert r.status == _abi.SDB_LIMIT_EXCEEDED
    r = O.encode_sst(Batch.from_entries([]), p)
    assert r.status == 0 and r.summary.num_blocks == 0 and r.summary.bloom_len == 0


# ------------------------------------------------------------------------------------------------
# decode round trips + failure detection (format/sst.rs:1029-1038, sst_builder.rs:1140-1155)
# ------------------------------------------------------------------------------------------------
@pytest.mark.parametrize("version", [1, 2])
def test_decode_round_trip_d3(version):
    from slatedb_amd.datasets import d3
    b = d3(n=1500)
    r = O.encode_sst(b, O.params(sst_version=version, block_size=1024))
    assert r.status == 0
    d = O.decode_blocks(r.data, r.block_off, version)
    assert d.status == 0 and d.n == b.n
    assert (d.block_entry_start.astype(np.uint32) == r.block_first_entry).all()
    for i in range(b.n):
        assert d.key_arena[int(d.key_off[i]):int(d.key_off[i + 1])].tobytes() == b.key(i)
        kind = int(b.kind[i])
        fl = int(d.flags[i])
        assert (fl & 1) == (kind == 2) and bool(fl & 8) == (kind == 1)
        if kind != 2:
            assert r.data[int(d.val_off[i]):int(d.val_off[i]) + int(d.val_len[i])].tobytes() == b.value(i)
        assert int(d.seq[i]) == int(b.seq[i])
        m = int(b.ts_mask[i])
        assert bool(fl & 4) == bool(m & 1)
        if m & 1:
            assert int(d.create_ts[i]) == int(b.create_ts[i])
        exp_has_expire = bool(m & 2) and not (version == 1 and kind == 2)  # V0 drops tombstone expire
        assert bool(fl & 2) == exp_has_expire
        if exp_has_expire:
            assert int(d.expire_ts[i]) == int(b.expire_ts[i])


def test_decode_detects_corruption():
    from slatedb_amd.datasets import d1
    b = d1(n=2000)
    r = O.encode_sst(b, O.params())
    data = r.data.copy()
    data[int(r.block_off[3]) + 5] ^= 1
    d = O.decode_blocks(data, r.block_off, 2)
    assert d.status == _abi.SDB_CHECKSUM_MISMATCH and list(d.bad_block) == [3]
    assert d.n == b.n - (r.block_first_entry[4] - r.block_first_entry[3])
    # invalid row flags with a valid CRC -> InvalidRowFlags
    blk = bytearray(O.encode_row(2, 0, b"k", 0, b"v", 7))
    blk[-1] = 0x10
    body = bytes(blk) + struct.pack(">HH", 0, 1)
    body += struct.pack(">I", zlib.crc32(body))
    d = O.decode_blocks(np.frombuffer(body, np.uint8), np.array([0, len(body)], np.uint64), 2)
    assert d.status == _abi.SDB_INVALID_ROW_FLAGS
