"""GPU parity at BASELINE.json's full sizes and on the fallback paths, plus the batched (launch-set)
encoder and graph capture.  Every case compares the HIP path (through the C ABI) with the CPU oracle
bit for bit.

  configs[2]  decode + iterate 16 D1 SSTs (272,256 blocks, ~1.095 GB): every decoded column
  configs[3]  bloom over 10 M random 16 B keys at 10 bits/key: the 12,500,000 B bitmap
  slot overflow   one hot key with 6,000 versions (legal compaction output; filter.rs:60-62 hashes
                  every duplicate): the bloom's (tile, slice) slots overflow and the slice rebuild runs
  long blocks     64 KiB blocks of 13 B rows: blocks longer than k_seg's lookahead (HBM continuation)
                  and than a chunk (k_group's serial walk, mode 0), emitted by the slow path
"""
import ctypes as C
from concurrent.futures import ThreadPoolExecutor

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets
from slatedb_amd.batch import Batch

from .test_gpu_parity import assert_decode_same, assert_same, encode_both

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def rt():
    from slatedb_amd import runtime
    runtime.require_device()
    return runtime


def _host_view(d):
    """DeviceSstOutput.to_host() dict -> an object assert_same understands."""
    class V:
        pass
    v = V()
    sm = d["summary"]
    v.status = sm.status
    v.summary = {f: getattr(sm, f) for f, _ in _abi.SstSummary._fields_}
    for k in ("data", "block_off", "block_first_entry", "index_key_len", "block_stats", "bloom"):
        setattr(v, k, d[k])
    if sm.status:
        v.summary["first_error_entry"] = sm.first_error_entry
    return v


# ------------------------------------------------------------------------------------------------
# configs[2]: decode + iterate 1 GiB of 4 KiB blocks
# ------------------------------------------------------------------------------------------------
def test_configs2_full_decode(rt):
    prm = O.params()
    with ThreadPoolExecutor(8) as ex:  # the oracle releases the GIL
        encs = list(ex.map(lambda j: O.encode_sst(datasets.d1(sst_index=j), prm), range(16)))
    data = np.concatenate([e.data for e in encs])
    offs = [np.zeros(1, np.uint64)]
    base = 0
    for e in encs:
        offs.append(e.block_off[1:] + np.uint64(base))
        base += len(e.data)
    block_off = np.concatenate(offs)
    assert len(block_off) - 1 == 272256 and len(data) > 1_095_000_000  # ~1 GiB (exact size depends on the LCPs)
    got = rt.Decoder().decode(data, block_off, 2)
    ref = O.decode_blocks(data, block_off, 2)
    assert ref.status == 0 and ref.n == 9256384
    assert_decode_same(ref, got, "configs[2]")


# ------------------------------------------------------------------------------------------------
# configs[3]: bloom over 10 M keys
# ------------------------------------------------------------------------------------------------
def test_configs3_bloom_10m(rt):
    kb, ko = datasets.c4_keys()
    assert len(ko) - 1 == 10_000_000
    ref = O.bloom_build(kb, ko, 10)
    assert len(ref) == 12_500_000
    got = rt.BloomFilterPolicy(10).build(Batch(kb, ko, np.zeros(0, np.uint8), np.zeros(len(ko), np.uint64)))
    assert got[:2] == b"\x00\x06"
    assert got[2:] == ref.tobytes()


# ------------------------------------------------------------------------------------------------
# bloom slot overflow: one hot key with thousands of versions
# ------------------------------------------------------------------------------------------------
def hot_key_batch(n=50000, hot=6000, at=10000):
    b = datasets.d1(n=n)
    keys = b.key_bytes.reshape(-1, 16).copy()
    keys[at:at + hot] = keys[at]
    seq = np.zeros(n, np.uint64)
    seq[at:at + hot] = np.arange(hot, 0, -1, dtype=np.uint64)  # key asc / seq desc
    return Batch(keys.reshape(-1), b.key_off, b.val_bytes, b.val_off, b.kind, seq)


def test_bloom_slot_overflow_rebuild(rt):
    import torch
    b = hot_key_batch()
    prm = rt.params()
    out = rt.DeviceSstOutput(b.n, b.logical_bytes(), b.logical_bytes(), prm)
    rt.encode_sst_device(b.to_device("cuda"), out)
    torch.cuda.synchronize()
    got = _host_view(out.to_host())
    ref = O.encode_sst(b, O.params())
    assert_same(ref, got, "hot key (fused bloom)")
    cd = C.CDLL(rt.LIB_PATH)
    cd.sdb_diag_bloom_slots.restype = C.c_uint64
    cd.sdb_diag_bloom_slots.argtypes = [C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]
    tiles, nsl, cap = C.c_uint32(), C.c_uint32(), C.c_uint32()
    off = cd.sdb_diag_bloom_slots(b.n, C.byref(prm), C.byref(tiles), C.byref(nsl), C.byref(cap))
    cnt = out.workspace[off: off + 4 * tiles.value * nsl.value].cpu().numpy().view(np.uint32)
    assert (cnt == 0xFFFFFFFF).any(), "the hot key must overflow a slot (the rebuild path is the subject)"
    # the standalone filter build (sdb_bloom_build) on the same keys
    std = rt.BloomFilterPolicy(10).build(b)
    assert std[2:] == ref.bloom.tobytes()


def test_fused_bloom_u32_slots_two_pass(rt):
    """The fused bloom's other binning mode: a filter of > 256 x 2^16 bits has slices of 2^17 bits, so
    the slots hold u32 bit positions and k_facts bins by the two-pass counting sort (the one-pass LDS
    buckets take u16 offsets only)."""
    n = 1_000_000
    keys = np.arange(n, dtype=">u8").view(np.uint8).copy()
    b = Batch(keys, np.arange(n + 1, dtype=np.uint64) * np.uint64(8), np.zeros(0, np.uint8),
              np.zeros(n + 1, np.uint64), np.zeros(n, np.uint8), np.arange(n, dtype=np.uint64))
    ref, got = encode_both(rt, b, bloom_bits_per_key=20)
    assert ref.status == 0 and ref.summary.num_probes == 13
    assert ref.summary.bloom_len * 8 > 256 * (1 << 16)  # slices of 2^17 bits: u32 slots
    assert_same(ref, got, "fused bloom, u32 slots")


# ------------------------------------------------------------------------------------------------
# long blocks: k_seg's HBM continuation, k_group's serial walk, the emit slow path
# ------------------------------------------------------------------------------------------------
def tiny_rows_batch(n=30000):
    keys = np.arange(n, dtype=">u4").view(np.uint8).copy()  # consecutive keys share 3 bytes: 13 B V2 rows
    return Batch(keys, np.arange(n + 1, dtype=np.uint64) * np.uint64(4), np.zeros(0, np.uint8),
                 np.zeros(n + 1, np.uint64), np.zeros(n, np.uint8), np.arange(n, dtype=np.uint64))


@pytest.mark.parametrize("version", [2, 1])
def test_long_blocks_serial_walk(rt, version):
    b = tiny_rows_batch()
    ref, got = encode_both(rt, b, block_size=65536, sst_version=version)
    assert ref.status == 0 and ref.summary.num_blocks >= 3
    assert ref.summary.max_block_entries > 2048  # longer than a chunk and than the lookahead
    assert got.summary["max_block_entries"] > 1024
    assert_same(ref, got, "64 KiB blocks of tiny rows v%d" % version)


# ------------------------------------------------------------------------------------------------
# the launch-set encoder (sdb_encode_ssts): several SSTs per launch sequence, errors isolated
# ------------------------------------------------------------------------------------------------
def _encode_set(rt, batches, prm):
    import torch
    dbs = [x.to_device("cuda") for x in batches]
    outs = [rt.DeviceSstOutput(x.n, max(x.logical_bytes(), 1), max(x.logical_bytes(), 1), prm, workspace=False)
            for x in batches]
    ws = rt.ssts_workspace(dbs, prm)
    rt.encode_ssts_device(dbs, outs, prm, ws)
    torch.cuda.synchronize()
    return [_host_view(o.to_host()) for o in outs]


def test_encode_ssts_set(rt):
    bad = Batch.from_entries([(b"abc", 0, b"v", 0, None, None), (b"ab", 0, b"v", 0, None, None)])
    batches = [datasets.d1(n=40000, sst_index=1), datasets.d3(n=2000), bad, Batch.from_entries([]),
               datasets.d1(n=3, sst_index=2), datasets.d2(n=30000), datasets.d1(n=70000, sst_index=3)]
    prm = rt.params(block_size=4096)
    gots = _encode_set(rt, batches, prm)
    for i, (x, got) in enumerate(zip(batches, gots)):
        ref = O.encode_sst(x, O.params(block_size=4096))
        assert_same(ref, got, "set member %d" % i)


def test_encode_ssts_more_than_one_set(rt):
    batches = [datasets.d1(n=5000 + 997 * j, sst_index=10 + j) for j in range(11)]  # 8 + 3
    prm = rt.params(block_size=1024, restart_interval=4)
    gots = _encode_set(rt, batches, prm)
    for j, (x, got) in enumerate(zip(batches, gots)):
        assert_same(O.encode_sst(x, O.params(block_size=1024, restart_interval=4)), got, "sst %d" % j)


def test_encode_ssts_full_d1_set(rt):
    """The bench's shape: 8 distinct full 64 MiB D1 SSTs in one launch sequence, all bit-exact."""
    batches = [datasets.d1(sst_index=j) for j in range(8)]
    gots = _encode_set(rt, batches, rt.params())
    with ThreadPoolExecutor(8) as ex:
        refs = list(ex.map(lambda x: O.encode_sst(x, O.params()), batches))
    for j, (ref, got) in enumerate(zip(refs, gots)):
        assert ref.summary.num_blocks == 17016
        assert_same(ref, got, "d1 set %d" % j)


def test_encode_ssts_concurrent_streams(rt):
    """bench.py's default shape: two builders in flight, each a launch set on its own stream with its own
    workspace and outputs; the sets alternate for several rounds and every SST stays bit-exact."""
    import torch
    sets = [[datasets.d1(n=60000 + 1000 * j, sst_index=60 + 4 * q + j) for j in range(4)] for q in range(2)]
    prm = rt.params()
    dsets = [[x.to_device("cuda") for x in s] for s in sets]
    outs = [[rt.DeviceSstOutput(x.n, x.logical_bytes(), x.logical_bytes(), prm, workspace=False) for x in s]
            for s in sets]
    wss = [rt.ssts_workspace(d, prm) for d in dsets]
    streams = [torch.cuda.Stream() for _ in range(2)]
    for _ in range(5):
        for q in range(2):
            rt.encode_ssts_device(dsets[q], outs[q], prm, wss[q], streams[q])
    torch.cuda.synchronize()
    for q in range(2):
        for x, o in zip(sets[q], outs[q]):
            assert_same(O.encode_sst(x, O.params()), _host_view(o.to_host()), "stream %d" % q)


def test_encode_graph_capture_replay(rt):
    """The device entry points launch only on the caller's stream: a captured encode replays."""
    import torch
    batches = [datasets.d1(n=30000, sst_index=40), datasets.d1(n=20000, sst_index=41)]
    prm = rt.params()
    dbs = [x.to_device("cuda") for x in batches]
    outs = [rt.DeviceSstOutput(x.n, x.logical_bytes(), x.logical_bytes(), prm, workspace=False) for x in batches]
    ws = rt.ssts_workspace(dbs, prm)
    s = torch.cuda.Stream()
    with torch.cuda.stream(s):
        rt.encode_ssts_device(dbs, outs, prm, ws, s)  # warm-up outside the capture
    torch.cuda.synchronize()
    for o in outs:
        o.data.zero_()
        o.bloom.zero_()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g, stream=s):
        rt.encode_ssts_device(dbs, outs, prm, ws, s)
    g.replay()
    g.replay()
    torch.cuda.synchronize()
    for x, o in zip(batches, outs):
        assert_same(O.encode_sst(x, O.params()), _host_view(o.to_host()), "graph replay")


# ------------------------------------------------------------------------------------------------
# many read_blocks ranges in one arena (sdb_decode_blocks_at): §8 C1 at the 2 MiB GET granularity
# ------------------------------------------------------------------------------------------------
def test_decode_blocks_at_scattered_ranges(rt):
    import torch
    rng = np.random.default_rng(17)
    encs = [O.encode_sst(datasets.d1(n=30000, sst_index=50 + j), O.params()) for j in range(3)]
    encs.append(O.encode_sst(datasets.d3(n=2500), O.params(block_size=1024)))
    # ranges of ~520 blocks (one 2 MiB GET each), placed in the arena in shuffled order with gaps
    ranges = []
    for e in encs:
        nb = len(e.block_off) - 1
        for b0 in range(0, nb, 520):
            ranges.append((e, b0, min(nb, b0 + 520)))
    order = rng.permutation(len(ranges))
    arena = np.zeros(0, np.uint8)
    starts, ends, contig, coff = [], [], [], [0]
    for i in order:
        e, b0, b1 = ranges[i]
        lo, hi = int(e.block_off[b0]), int(e.block_off[b1])
        base = len(arena) + int(rng.integers(1, 300))                  # a gap before every range
        arena = np.concatenate([arena, rng.integers(0, 256, base - len(arena), dtype=np.uint8), e.data[lo:hi]])
        starts += [base + int(e.block_off[k]) - lo for k in range(b0, b1)]
        ends += [base + int(e.block_off[k + 1]) - lo for k in range(b0, b1)]
        contig.append(e.data[lo:hi])
    nb = len(starts)
    # the oracle decodes the same blocks laid out back to back
    cdata = np.concatenate(contig)
    cl = np.array([e - s for s, e in zip(starts, ends)], np.uint64)
    coff = np.concatenate([[0], np.cumsum(cl)]).astype(np.uint64)
    ref = O.decode_blocks(cdata, coff, 2)
    assert ref.status == 0
    dev = torch.device("cuda")
    out = rt.DeviceDecodeOutput(nb, ref.n + 16, len(ref.key_arena) + 16)
    rt.decode_blocks_at_device(torch.from_numpy(arena).to(dev), torch.from_numpy(np.array(starts, np.uint64).view(np.int64)).to(dev),
                               torch.from_numpy(np.array(ends, np.uint64).view(np.int64)).to(dev), nb, out)
    torch.cuda.synchronize()
    got = out.to_host()
    # value references are arena offsets: map them back to the contiguous layout block by block
    blk = np.searchsorted(ref.block_entry_start, np.arange(ref.n), side="right") - 1
    shift = np.array(starts, np.uint64)[blk] - coff[:-1][blk]
    got.val_off = np.where(got.val_len > 0, got.val_off - shift, got.val_off)
    assert_decode_same(ref, got, "scattered ranges")


def test_encode_host_many_pipelined(rt):
    """sdb_encoder_encode_host_many (overlapped H2D / kernels / D2H, two staging slots): every SST equals
    the oracle's, with sizes that grow and shrink across the slots and an empty SST in the middle."""
    from .test_gpu_parity import assert_same
    import types
    sizes = [3000, 40000, 0, 578524, 7, 20000, 120000]
    hosts = [datasets.d1(sst_index=i, n=n) if n else Batch.from_entries([]) for i, n in enumerate(sizes)]
    prm = dict(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    enc = rt.Encoder(rt.params(**prm))
    for rep in range(2):  # the second call reuses (and partly regrows) the slots
        got = enc.encode_many(hosts if rep == 0 else hosts[::-1])
        src = hosts if rep == 0 else hosts[::-1]
        for i, (b, g) in enumerate(zip(src, got)):
            ref = O.encode_sst(b, O.params(**prm))
            assert_same(ref, g, "many[%d] rep %d" % (i, rep))
    enc.close()


def test_encode_host_many_grows_output_slots(rt):
    """A call with more SSTs than any earlier one grows the encoder's pinned output buffers; the buffers
    of the earlier SSTs must survive the growth (they are moved, not copied and freed)."""
    prm = dict(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    enc = rt.Encoder(rt.params(**prm))
    for sizes in ([5000, 9000], [5000, 9000, 300, 7000, 12000, 1, 4000], [800, 700]):
        hosts = [datasets.d1(sst_index=i, n=n) for i, n in enumerate(sizes)]
        got = enc.encode_many(hosts)
        for i, (b, g) in enumerate(zip(hosts, got)):
            assert_same(O.encode_sst(b, O.params(**prm)), g, "grow %d/%d" % (i, len(sizes)))
    enc.close()
