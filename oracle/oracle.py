"""ctypes front-end of oracle/liboracle.so — the CPU restatement used as the parity checker.

TEST INFRASTRUCTURE ONLY: imported by tests/, __graft_entry__.smoke() and bench.py's cpu_baseline
leg; never by slatedb_amd/.
"""
import ctypes as C
import os
import subprocess

import numpy as np

from slatedb_amd import _abi

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "liboracle.so")


def build():
    subprocess.check_call(["make", "-s", "-C", HERE])


def _load():
    if not os.path.exists(LIB):
        build()
    lib = C.CDLL(LIB)
    V, P = C.c_void_p, C.POINTER
    sig = {
        "orc_varint_len": (C.c_uint32, [C.c_uint32]),
        "orc_encode_varint": (C.c_size_t, [V, C.c_uint32]),
        "orc_crc32": (C.c_uint32, [V, C.c_size_t]),
        "orc_siphash": (C.c_uint64, [V, C.c_size_t, C.c_uint64, C.c_uint64, C.c_int, C.c_int]),
        "orc_filter_hash": (C.c_uint64, [V, C.c_size_t]),
        "orc_probes_for_key": (None, [C.c_uint64, C.c_uint16, C.c_uint32, V]),
        "orc_optimal_num_probes": (C.c_uint16, [C.c_uint32]),
        "orc_filter_size_bytes": (C.c_uint64, [C.c_uint64, C.c_uint32]),
        "orc_compute_prefix": (C.c_size_t, [V, C.c_size_t, V, C.c_size_t]),
        "orc_index_key_len": (C.c_int64, [V, C.c_size_t, C.c_int, V, C.c_size_t]),
        "orc_encode_row": (C.c_size_t, [C.c_uint16, C.c_uint32, V, C.c_size_t, C.c_uint8, V,
                                        C.c_size_t, C.c_uint64, C.c_int, C.c_int64, C.c_int,
                                        C.c_int64, V, C.c_size_t]),
        "orc_build_block": (C.c_int, [P(_abi.KvBatch), C.c_uint16, C.c_uint32, C.c_uint16, V,
                                      C.c_uint64, P(C.c_uint64), V]),
        "orc_encode_sst": (C.c_int, [P(_abi.KvBatch), P(_abi.SstParams), P(_abi.SstOut)]),
        "orc_bloom_build": (C.c_int, [V, V, C.c_uint64, C.c_uint32, V, C.c_uint64]),
        "orc_bloom_build_range": (C.c_int, [V, V, C.c_uint64, C.c_uint64, C.c_uint64, C.c_uint32, V, C.c_uint64]),
        "orc_bloom_might_contain": (C.c_int, [V, C.c_uint64, C.c_uint32, V, C.c_size_t]),
        "orc_decode_blocks": (C.c_int, [V, V, C.c_uint64, C.c_uint16, P(_abi.DecodedOut)]),
        "orc_decode_blocks_desc": (C.c_int, [V, V, C.c_uint64, C.c_uint16, P(_abi.DecodedOut)]),
        "orc_sst_lookup": (C.c_int, [P(_abi.SstView), V, V, C.c_uint64, C.c_int, P(_abi.LookupOut)]),
        "orc_bloom_build_prefix": (C.c_int, [V, V, V, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_int, V,
                                             C.c_uint64, P(C.c_uint64)]),
        "orc_bloom_might_match": (C.c_int, [V, C.c_uint64, C.c_uint32, C.c_int, C.c_uint32, C.c_uint32, V,
                                            C.c_size_t, C.c_int, C.c_int64]),
        "orc_prefix_len": (C.c_int64, [C.c_uint32, C.c_uint32, V, C.c_size_t, C.c_int64]),
        "orc_decompressed_len": (C.c_int64, [C.c_uint32, V, C.c_size_t]),
        "orc_xxh64": (C.c_uint64, [V, C.c_size_t, C.c_uint64]),
        "orc_decompress": (C.c_int, [C.c_uint32, V, C.c_size_t, V, C.c_size_t, P(C.c_size_t)]),
        "orc_decompress_blocks": (C.c_int, [C.c_uint32, V, V, C.c_uint64, V, C.c_uint64, V, V, P(C.c_uint64)]),
        "orc_merge_runs": (C.c_int, [P(_abi.Run), C.c_uint32, P(_abi.Retention), P(_abi.MergedOut)]),
        "orc_sst_cuts": (C.c_int, [P(_abi.KvBatch), P(_abi.SstParams), C.c_uint64, V, C.c_uint64, P(C.c_uint64)]),
    }
    for k, (r, a) in sig.items():
        f = getattr(lib, k)
        f.restype, f.argtypes = r, a
    return lib


_lib = None


def lib():
    global _lib
    if _lib is None:
        _lib = _load()
    return _lib


def _buf(b):
    b = bytes(b)
    return C.create_string_buffer(b, max(len(b), 1)), len(b)


def varint_len(v):
    return lib().orc_varint_len(v)


def encode_varint(v):
    out = C.create_string_buffer(8)
    n = lib().orc_encode_varint(out, v)
    return out.raw[:n]


def crc32(data):
    b, n = _buf(data)
    return lib().orc_crc32(b, n)


def siphash(data, k0=0, k1=0, c=1, d=3):
    b, n = _buf(data)
    return lib().orc_siphash(b, n, k0, k1, c, d)


def filter_hash(key):
    b, n = _buf(key)
    return lib().orc_filter_hash(b, n)


def probes_for_key(h, k, m):
    out = (C.c_uint32 * k)()
    lib().orc_probes_for_key(h, k, m, out)
    return list(out)


def optimal_num_probes(bpk):
    return lib().orc_optimal_num_probes(bpk)


def filter_size_bytes(n, bpk):
    return lib().orc_filter_size_bytes(n, bpk)


def compute_prefix(a, b):
    ba, na = _buf(a)
    bb, nb = _buf(b)
    return lib().orc_compute_prefix(ba, na, bb, nb)


def index_key(prev, first):
    """compute_index_key; returns bytes, or None where the reference panics."""
    bf, nf = _buf(first)
    if prev is None:
        r = lib().orc_index_key_len(None, 0, 0, bf, nf)
    else:
        bp, npv = _buf(prev)
        r = lib().orc_index_key_len(bp, npv, 1, bf, nf)
    return None if r < 0 else bytes(first)[:r]


def encode_row(version, shared, suffix, kind, value, seq, create_ts=None, expire_ts=None):
    bs, ns = _buf(suffix)
    bv, nv = _buf(value or b"")
    cap = ns + nv + 64
    out = C.create_string_buffer(cap)
    n = lib().orc_encode_row(version, shared, bs, ns, kind, bv, nv, seq, create_ts is not None,
                             create_ts or 0, expire_ts is not None, expire_ts or 0, out, cap)
    return out.raw[:n]


def build_block(batch, version=2, block_size=4096, restart_interval=16):
    cap = int(batch.key_off[-1] + batch.val_off[-1]) + 64 * (batch.n + 1)
    out = (C.c_uint8 * cap)()
    ln = C.c_uint64(0)
    acc = np.zeros(max(batch.n, 1), np.uint8)
    kb = batch.to_ctypes()
    st = lib().orc_build_block(C.byref(kb), version, block_size, restart_interval, out, cap,
                               C.byref(ln), acc.ctypes.data)
    return st, bytes(out)[:ln.value] if st == 0 else b"", acc[:batch.n]


class SstResult:
    def __init__(self, status, summary, data, block_off, block_first_entry, index_key_len,
                 block_stats, bloom):
        self.status = status
        self.summary = summary
        self.data = data
        self.block_off = block_off
        self.block_first_entry = block_first_entry
        self.index_key_len = index_key_len
        self.block_stats = block_stats
        self.bloom = bloom


def bounds(batch, params):
    """Same upper bounds as sdb_encode_bounds (restated so the oracle needs no GPU library)."""
    n = batch.n
    kb = int(batch.key_off[-1] - batch.key_off[0])
    vb = int(batch.val_off[-1] - batch.val_off[0])
    data_cap = kb + vb + n * 64 + 64
    block_cap = n + 1
    hashes = (n if params.prefix_kind else 0) + (0 if params.no_whole_key else n)
    bloom_cap = filter_size_bytes(hashes, params.bloom_bits_per_key) + 16 if params.bloom_bits_per_key else 16
    return data_cap, block_cap, bloom_cap


def params(block_size=4096, sst_version=2, restart_interval=16, bloom_bits_per_key=10,
           min_filter_keys=0, sst_type=0, prefix_kind=0, prefix_arg=0, no_whole_key=0):
    return _abi.SstParams(block_size, sst_version, restart_interval, bloom_bits_per_key,
                          min_filter_keys, sst_type, prefix_kind, prefix_arg, no_whole_key)


def bloom_build_prefix(key_bytes, key_off, bpk, kind, arg=0, whole=True, prefix_len=None):
    """BloomFilterBuilder with a prefix extractor (filter.rs:40-90): the bitmap (size from the hash count)."""
    n = len(key_off) - 1
    cap = filter_size_bytes(2 * n, bpk) + 16
    bm = np.zeros(max(cap, 1), np.uint8)
    ln = C.c_uint64(0)
    pl = None if prefix_len is None else np.ascontiguousarray(prefix_len, np.int32)
    kb = np.ascontiguousarray(key_bytes, np.uint8)
    st = lib().orc_bloom_build_prefix(kb.ctypes.data if kb.size else None, np.ascontiguousarray(key_off, np.uint64).ctypes.data,
                                      None if pl is None else pl.ctypes.data, n, bpk, kind, arg, int(whole),
                                      bm.ctypes.data, cap, C.byref(ln))
    assert st == 0, st
    return bm[:ln.value].copy()


def might_match(bitmap, num_probes, whole, kind, arg, query, is_prefix=False, given=-1):
    """Filter::might_match (filter.rs:149-175) for FilterQuery::point / ::prefix."""
    bq, nq = _buf(query)
    bm = np.ascontiguousarray(bitmap, np.uint8)
    return bool(lib().orc_bloom_might_match(bm.ctypes.data if bm.size else None, bm.size, num_probes, int(whole),
                                            kind, arg, bq, nq, int(is_prefix), given))


def encode_sst(batch, prm):
    data_cap, block_cap, bloom_cap = bounds(batch, prm)
    data = np.zeros(data_cap, np.uint8)
    block_off = np.zeros(block_cap + 1, np.uint64)
    bfe = np.zeros(block_cap + 1, np.uint32)
    ikl = np.zeros(block_cap, np.uint32)
    bst = np.zeros(3 * block_cap, np.uint16)
    bloom = np.zeros(bloom_cap, np.uint8)
    sm = _abi.SstSummary()
    out = _abi.SstOut(data.ctypes.data, data_cap, block_off.ctypes.data, bfe.ctypes.data,
                      ikl.ctypes.data, bst.ctypes.data, block_cap, bloom.ctypes.data, bloom_cap,
                      C.addressof(sm))
    kb = batch.to_ctypes()
    st = lib().orc_encode_sst(C.byref(kb), C.byref(prm), C.byref(out))
    nb = sm.num_blocks
    return SstResult(st, sm, data[:sm.data_len].copy(), block_off[:nb + 1].copy(),
                     bfe[:nb + 1].copy(), ikl[:nb].copy(), bst[:3 * nb].reshape(-1, 3).copy(),
                     bloom[:sm.bloom_len].copy())


def bloom_build(key_bytes, key_off, bpk):
    n = len(key_off) - 1
    fb = filter_size_bytes(n, bpk)
    bm = np.zeros(max(fb, 1), np.uint8)
    st = lib().orc_bloom_build(key_bytes.ctypes.data, key_off.ctypes.data, n, bpk, bm.ctypes.data, fb)
    assert st == 0
    return bm[:fb]


def bloom_build_threads(key_bytes, key_off, bpk, threads):
    """build_filter split by key range over `threads` threads (private bitmaps, OR-merged): the
    multi-thread CPU baseline of configs[3].  ctypes drops the GIL inside the C call."""
    import threading
    n = len(key_off) - 1
    fb = filter_size_bytes(n, bpk)
    parts = [np.zeros(max(fb, 1), np.uint8) for _ in range(threads)]
    cuts = [n * t // threads for t in range(threads + 1)]

    def run(t):
        st = lib().orc_bloom_build_range(key_bytes.ctypes.data, key_off.ctypes.data, n, cuts[t], cuts[t + 1],
                                         bpk, parts[t].ctypes.data, fb)
        assert st == 0

    ths = [threading.Thread(target=run, args=(t,)) for t in range(threads)]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    out = parts[0]
    for q in parts[1:]:
        np.bitwise_or(out, q, out=out)
    return out[:fb]


def might_contain(bitmap, num_probes, key):
    bk, nk = _buf(key)
    bm = np.ascontiguousarray(bitmap, np.uint8)
    return bool(lib().orc_bloom_might_contain(bm.ctypes.data if bm.size else None, bm.size,
                                              num_probes, bk, nk))


class DecodeResult:
    pass


def decode_blocks(blocks, block_off, version=2, cap_entries=None, key_cap=None, descending=False):
    blocks = np.ascontiguousarray(blocks, np.uint8)
    total = int(np.asarray(block_off)[-1] - np.asarray(block_off)[0]) if len(block_off) > 1 else 0
    key_cap = key_cap or (total * 4 + 4096)
    while True:
        r = _decode_blocks(blocks, block_off, version, cap_entries, key_cap, descending)
        if r.status != _abi.SDB_INVALID_ARGUMENT or key_cap > (total + 1) * 1024:
            return r
        key_cap *= 8


def _decode_blocks(blocks, block_off, version, cap_entries, key_cap, descending=False):
    block_off = np.ascontiguousarray(block_off, np.uint64)
    nb = len(block_off) - 1
    total = int(block_off[-1] - block_off[0]) if nb else 0
    cap_entries = cap_entries or (total // 12 + 16)
    key_cap = key_cap or (total * 64 + 64)
    r = DecodeResult()
    r.block_entry_start = np.zeros(nb + 1, np.uint64)
    r.key_arena = np.zeros(key_cap, np.uint8)
    r.key_off = np.zeros(cap_entries + 1, np.uint64)
    r.val_off = np.zeros(cap_entries, np.uint64)
    r.val_len = np.zeros(cap_entries, np.uint32)
    r.seq = np.zeros(cap_entries, np.uint64)
    r.flags = np.zeros(cap_entries, np.uint8)
    r.create_ts = np.zeros(cap_entries, np.int64)
    r.expire_ts = np.zeros(cap_entries, np.int64)
    r.bad_block = np.zeros(max(nb, 1), np.uint32)
    sm = _abi.DecodeSummary()
    out = _abi.DecodedOut(r.block_entry_start.ctypes.data, r.key_arena.ctypes.data, key_cap,
                          r.key_off.ctypes.data, r.val_off.ctypes.data, r.val_len.ctypes.data,
                          r.seq.ctypes.data, r.flags.ctypes.data, r.create_ts.ctypes.data,
                          r.expire_ts.ctypes.data, cap_entries, r.bad_block.ctypes.data,
                          max(nb, 1), C.addressof(sm))
    fn = lib().orc_decode_blocks_desc if descending else lib().orc_decode_blocks
    st = fn(blocks.ctypes.data if blocks.size else None, block_off.ctypes.data, nb, version, C.byref(out))
    r.status = st
    r.summary = sm
    n = sm.num_entries
    r.n = n
    r.key_off = r.key_off[:n + 1]
    r.key_arena = r.key_arena[:sm.key_bytes]
    for f in ("val_off", "val_len", "seq", "flags", "create_ts", "expire_ts"):
        setattr(r, f, getattr(r, f)[:n])
    r.bad_block = r.bad_block[:min(sm.num_bad_blocks, max(nb, 1))]
    return r


LOOKUP_FIELDS = (("state", np.uint8), ("status", np.int32), ("block", np.uint32), ("entry", np.uint32),
                 ("key_len", np.uint32), ("val_off", np.uint64), ("val_len", np.uint32), ("seq", np.uint64),
                 ("flags", np.uint8), ("create_ts", np.int64), ("expire_ts", np.int64))


class LookupResult:
    pass


def sst_index_keys(batch, enc):
    """BlockMeta.first_key of every block (index key = first key[:index_key_len]) -> (bytes, offsets)."""
    nb = len(enc.block_off) - 1
    starts = np.asarray(enc.block_first_entry[:nb], np.int64)
    ikl = np.asarray(enc.index_key_len[:nb], np.uint64)
    off = np.zeros(nb + 1, np.uint64)
    off[1:] = np.cumsum(ikl)
    parts = [batch.key_bytes[int(batch.key_off[s]):int(batch.key_off[s]) + int(l)] for s, l in zip(starts, ikl)]
    kb = np.concatenate(parts) if parts else np.zeros(0, np.uint8)
    return np.ascontiguousarray(kb, np.uint8), off


def sst_lookup(data, block_off, index_keys, index_key_off, keys, descending=False, sst_version=2,
               bloom=None, num_probes=0):
    """orc_sst_lookup over host arrays; keys: list of bytes.  Returns a LookupResult of numpy arrays."""
    data = np.ascontiguousarray(data, np.uint8)
    block_off = np.ascontiguousarray(block_off, np.uint64)
    ik = np.ascontiguousarray(index_keys, np.uint8)
    iko = np.ascontiguousarray(index_key_off, np.uint64)
    bm = None if bloom is None else np.ascontiguousarray(bloom, np.uint8)
    v = _abi.SstView(data.ctypes.data if data.size else None, block_off.ctypes.data, len(block_off) - 1,
                     ik.ctypes.data if ik.size else None, iko.ctypes.data,
                     bm.ctypes.data if bm is not None and bm.size else (None if bm is None else 1),
                     0 if bm is None else bm.size, num_probes, sst_version, 0)
    if bm is not None and not bm.size:
        v.bloom = C.cast(C.create_string_buffer(1), C.c_void_p).value
    n = len(keys)
    koff = np.zeros(n + 1, np.uint64)
    koff[1:] = np.cumsum([len(k) for k in keys]) if n else []
    kb = np.frombuffer(b"".join(bytes(k) for k in keys) or b"\0", np.uint8).copy()
    r = LookupResult()
    for f, dt in LOOKUP_FIELDS:
        setattr(r, f, np.zeros(max(n, 1), dt))
    out = _abi.LookupOut(*[getattr(r, f).ctypes.data for f, _ in LOOKUP_FIELDS])
    lib().orc_sst_lookup(C.byref(v), kb.ctypes.data, koff.ctypes.data, n, int(bool(descending)), C.byref(out))
    for f, _ in LOOKUP_FIELDS:
        setattr(r, f, getattr(r, f)[:n])
    return r


def retention(min_seq=None, time_seq=None, compaction_start_ts=0, filter_tombstone=False, merge_operands=False):
    """sdb_retention: min_seq = retention_min_seq (None: no seq window); time_seq = the first seq inside the
    retention_timeout window (None: no time window, 0: every seq)."""
    return _abi.Retention(min_seq or 0, time_seq or 0, compaction_start_ts, int(min_seq is not None),
                          int(time_seq is not None), int(bool(filter_tombstone)), int(bool(merge_operands)), 0)


def merge_runs(runs, ret):
    """orc_merge_runs over host Runs -> (Batch of the merged, retained stream, MergeSummary)."""
    from slatedb_amd.batch import Batch
    total = sum(r.n for r in runs)
    kcap = sum(int(r.key_off[-1]) for r in runs) + 1
    vcap = sum(int(r.val_len.sum()) for r in runs) + 1
    kb, vb = np.zeros(kcap, np.uint8), np.zeros(vcap, np.uint8)
    ko, vo = np.zeros(total + 1, np.uint64), np.zeros(total + 1, np.uint64)
    kind, seq = np.zeros(max(total, 1), np.uint8), np.zeros(max(total, 1), np.uint64)
    cts, ets, mask = np.zeros(max(total, 1), np.int64), np.zeros(max(total, 1), np.int64), np.zeros(max(total, 1), np.uint8)
    sm = _abi.MergeSummary()
    out = _abi.MergedOut(kb.ctypes.data, kcap, ko.ctypes.data, vb.ctypes.data, vcap, vo.ctypes.data, kind.ctypes.data,
                         seq.ctypes.data, cts.ctypes.data, ets.ctypes.data, mask.ctypes.data, total, C.addressof(sm))
    cr = (_abi.Run * max(len(runs), 1))(*[r.to_ctypes() for r in runs])
    lib().orc_merge_runs(cr, len(runs), C.byref(ret), C.byref(out))
    n = sm.num_out
    b = Batch(kb[:sm.key_bytes], ko[:n + 1], vb[:sm.val_bytes], vo[:n + 1], kind[:n], seq[:n], cts[:n], ets[:n], mask[:n])
    return b, sm


def sst_cuts(batch, prm, max_sst_size):
    """orc_sst_cuts -> (status, list of SST start entries + [n])."""
    cap = batch.n + 2
    cuts = np.zeros(cap, np.uint64)
    ns = C.c_uint64(0)
    kb = batch.to_ctypes()
    st = lib().orc_sst_cuts(C.byref(kb), C.byref(prm), max_sst_size, cuts.ctypes.data, cap, C.byref(ns))
    return st, [int(x) for x in cuts[:ns.value + 1]] if ns.value else []


def compact(runs, ret, prm, max_sst_size):
    """The compaction output side: merge + retention, cuts, then encode_sst per output SST.
    Returns (merged Batch, MergeSummary, cuts, [SstResult])."""
    merged, sm = merge_runs(runs, ret)
    if sm.status:
        return merged, sm, [], []
    st, cuts = sst_cuts(merged, prm, max_sst_size)
    assert st == 0, st
    ssts = [encode_sst(merged.slice(cuts[i], cuts[i + 1]), prm) for i in range(len(cuts) - 1)]
    return merged, sm, cuts, ssts


# --- f3: block decompression (format/sst.rs:884-917) -----------------------------------------------
CODEC_SNAPPY, CODEC_ZLIB, CODEC_LZ4, CODEC_ZSTD = 1, 2, 3, 4  # CompressionFormat (schemas/sst.fbs)


def decompress(codec, data):
    """SsTableFormat::decompress of one payload -> (status, bytes)."""
    b = np.frombuffer(bytes(data), np.uint8)
    n = lib().orc_decompressed_len(codec, b.ctypes.data if b.size else None, b.size)
    if n < 0 and codec in (CODEC_ZLIB, CODEC_ZSTD):  # the length comes from decoding: it failed
        return _abi.SDB_DECOMPRESSION_ERROR, b""
    cap = max(int(n), 0) + 1
    out = np.zeros(cap, np.uint8)
    ol = C.c_size_t(0)
    st = lib().orc_decompress(codec, b.ctypes.data if b.size else None, b.size, out.ctypes.data, cap, C.byref(ol))
    return st, out[:ol.value].tobytes() if st == 0 else b""


class DecompressResult:
    pass


def decompress_blocks(codec, blocks, block_off, out_cap=None):
    """decode_block's first half over a block run: (status, out, out_start, out_end, first_err)."""
    blocks = np.ascontiguousarray(blocks, np.uint8)
    block_off = np.ascontiguousarray(block_off, np.uint64)
    nb = len(block_off) - 1
    cap = out_cap if out_cap is not None else int(blocks.size) * 64 + 4 * nb + 64
    r = DecompressResult()
    r.out = np.zeros(max(cap, 1), np.uint8)
    r.out_start = np.zeros(nb + 1, np.uint64)
    r.out_end = np.zeros(max(nb, 1), np.uint64)
    fe = C.c_uint64(0)
    r.status = lib().orc_decompress_blocks(codec, blocks.ctypes.data if blocks.size else None, block_off.ctypes.data,
                                           nb, r.out.ctypes.data, cap, r.out_start.ctypes.data, r.out_end.ctypes.data,
                                           C.byref(fe))
    r.first_err = fe.value
    r.out_end = r.out_end[:nb]
    return r
