"""Every SstBlockSize (config.rs:231-267) against the oracle, bit for bit.  Blocks over one k_emit wave
image take the piece path (k_emit_big: pieces of <= 64 rows / 4 KiB, CRC chained across pieces, short
trailers gathered in LDS, long ones read back), chains whose chunk tables exceed k_enum's LDS take the
HBM table walk (mode 2), and blocks with rows too large for a piece the workgroup path."""
import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import datasets
from slatedb_amd.batch import Batch

from .test_gpu_parity import assert_same, encode_both, rt  # noqa: F401

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("block_size", [8192, 16384, 32768, 65536])
def test_d1_large_blocks(rt, block_size):  # noqa: F811
    b = datasets.d1(n=150000, sst_index=11)
    ref, got = encode_both(rt, b, block_size=block_size, sst_version=2, bloom_bits_per_key=10)
    assert_same(ref, got, "d1 bs=%d" % block_size)


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("block_size", [8192, 16384])
def test_mixed_large_blocks(rt, version, block_size):  # noqa: F811
    # tombstones, merges, timestamps, long keys, values of 0-299 bytes
    b = datasets.d3(n=6000)
    ref, got = encode_both(rt, b, block_size=block_size, sst_version=version, bloom_bits_per_key=10)
    assert_same(ref, got, "d3 v%d bs=%d" % (version, block_size))


@pytest.mark.parametrize("restart_interval", [1, 3, 16])
def test_piece_trailer_paths(rt, restart_interval):  # noqa: F811
    # 64 KiB blocks of ~40-byte rows: ~1600 rows per block; restart interval 1 makes a 3 KiB trailer
    # (read back through the image), 16 a ~200-byte one
    rng = np.random.default_rng(8)
    ents = [(b"key%012d" % i, 0, bytes(rng.integers(0, 256, 20, dtype=np.uint8)), 5000 - i, None, None)
            for i in range(5000)]
    b = Batch.from_entries(ents)
    ref, got = encode_both(rt, b, block_size=65536, sst_version=2, restart_interval=restart_interval,
                           bloom_bits_per_key=10)
    assert_same(ref, got, "ri=%d" % restart_interval)


def test_blocks_with_rows_too_large_for_a_piece(rt):  # noqa: F811
    # 16 KiB blocks where some rows carry 5 KiB values: those blocks stay on the workgroup path, the
    # others take pieces
    rng = np.random.default_rng(9)
    ents = []
    for i in range(3000):
        vlen = 5000 if i % 97 == 5 else int(rng.integers(10, 200))
        ents.append((b"row%08d" % i, 0, bytes(rng.integers(0, 256, vlen, dtype=np.uint8)), 1, None, None))
    b = Batch.from_entries(ents)
    ref, got = encode_both(rt, b, block_size=16384, sst_version=2, bloom_bits_per_key=10)
    assert_same(ref, got, "huge rows")


# ------------------------------------------------------------------------------------------------
# decode of blocks over one wave image: restart-region pieces staged in LDS (sdb_decode.hip
# for_each_piece), and the HBM walk for blocks a piece cannot hold
# ------------------------------------------------------------------------------------------------
def _decode_cases():
    rng = np.random.default_rng(21)
    small_rows = Batch.from_entries([(b"key%012d" % i, 0, bytes(rng.integers(0, 256, 20, dtype=np.uint8)), 9000 - i,
                                      None, None) for i in range(9000)])
    big_rows = Batch.from_entries([(b"row%08d" % i, 0, bytes(rng.integers(0, 256, 5000 if i % 97 == 5 else
                                                                      int(rng.integers(10, 200)), dtype=np.uint8)),
                                    1, None, None) for i in range(3000)])
    return [("d1", datasets.d1(n=120000, sst_index=3), {}), ("d3", datasets.d3(n=6000), {}),
            ("tiny-ri1", small_rows, {"restart_interval": 1}), ("tiny-ri3", small_rows, {"restart_interval": 3}),
            ("huge-rows", big_rows, {})]


@pytest.mark.parametrize("block_size", [8192, 16384, 32768, 65536])
def test_decode_large_blocks(rt, block_size):  # noqa: F811
    from .test_descending import device_desc
    from .test_gpu_parity import assert_decode_same
    for name, b, kw in _decode_cases():
        e = O.encode_sst(b, O.params(block_size=block_size, **kw))
        ref = O.decode_blocks(e.data, e.block_off, 2)
        assert ref.status == 0
        got = rt.Decoder().decode(e.data, e.block_off, 2)
        assert_decode_same(ref, got, "%s bs=%d" % (name, block_size))
        assert np.array_equal(got.key_arena, b.key_bytes)
        desc = O.decode_blocks(e.data, e.block_off, 2, descending=True)
        assert_decode_same(desc, device_desc(rt, e.data, e.block_off, 2), "%s desc bs=%d" % (name, block_size))


def test_decode_large_blocks_corrupt(rt):  # noqa: F811
    """Corruption inside big blocks: a CRC mismatch, and a row whose varint header runs past its region
    with the CRC recomputed (the piece walk must report what the whole-block walk reports)."""
    import struct
    import zlib
    from .test_gpu_parity import assert_decode_same
    b = datasets.d1(n=40000, sst_index=4)
    e = O.encode_sst(b, O.params(block_size=16384))
    data = e.data.copy()
    data[int(e.block_off[3]) + 1000] ^= 0x10  # CRC mismatch in block 3
    k = 7
    s, t = int(e.block_off[k]), int(e.block_off[k + 1])
    blk = bytearray(data[s:t - 4].tobytes())
    blk[200] = 0xFF  # a byte inside the first region's rows
    data[s:t - 4] = np.frombuffer(bytes(blk), np.uint8)
    data[t - 4:t] = np.frombuffer(struct.pack(">I", zlib.crc32(bytes(blk))), np.uint8)
    ref = O.decode_blocks(data, e.block_off, 2)
    got = rt.Decoder().decode(data, e.block_off, 2)
    assert ref.status != 0
    assert_decode_same(ref, got, "corrupt big blocks")


def test_decode_64k_block_corrupt(rt):  # noqa: F811
    """A 64 KiB block (its CRC through sixteen 4 KiB LDS windows, its rows as restart-region pieces):
    a flipped byte in each part of the block, a flipped CRC byte, a corrupt trailer count and a corrupt
    region offset (CRC recomputed: the whole-block walk decides), each alone and in descending order."""
    import struct
    import zlib
    from .test_descending import device_desc
    from .test_gpu_parity import assert_decode_same
    b = datasets.d1(n=60000, sst_index=5)
    e = O.encode_sst(b, O.params(block_size=65536))
    k = 2
    s, t = int(e.block_off[k]), int(e.block_off[k + 1])
    n = t - s - 4
    variants = []
    for frac in (0.0, 0.1, 0.3, 0.55, 0.8, 0.99):  # a byte in each part of the block (incl. its trailer)
        d = e.data.copy()
        d[s + min(n - 1, int(frac * n))] ^= 0x04
        variants.append(("flip %.2f" % frac, d))
    d = e.data.copy()
    d[t - 1] ^= 0x01
    variants.append(("crc byte", d))
    for what, pos, val in (("count", n - 2, 0x7F), ("offset", n - 2 - 2 * 3, 0xFF)):
        blk = bytearray(e.data[s:t - 4].tobytes())
        blk[pos] = val
        d = e.data.copy()
        d[s:t - 4] = np.frombuffer(bytes(blk), np.uint8)
        d[t - 4:t] = np.frombuffer(struct.pack(">I", zlib.crc32(bytes(blk))), np.uint8)
        variants.append((what, d))
    for what, d in variants:
        ref = O.decode_blocks(d, e.block_off, 2)
        assert ref.status != 0 or what in ("count", "offset"), what  # (a bad offset may not matter ascending)
        assert_decode_same(ref, rt.Decoder().decode(d, e.block_off, 2), "64k " + what)
        desc = O.decode_blocks(d, e.block_off, 2, descending=True)
        assert_decode_same(desc, device_desc(rt, d, e.block_off, 2), "64k desc " + what)


# ------------------------------------------------------------------------------------------------
# size boundaries of the two passes' LDS staging (count: whole blocks up to 4096 bytes, emit: up to
# 6144): a block staged whole is walked in place, never cut into pieces over the same LDS image; and
# rows that straddle a piece boundary (the whole-block walk decides, exactly as the reference iterates)
# ------------------------------------------------------------------------------------------------
TAIL_SIZES = [4086, 4090, 4093, 4096, 4100, 4250, 5000, 5900, 6100, 6144, 6150, 7000]


@pytest.mark.parametrize("restart_interval", [1, 16])
def test_decode_tail_block_sizes(rt, restart_interval):  # noqa: F811
    from .decode_cases import tail_block_case
    from .test_descending import device_desc
    from .test_gpu_parity import assert_decode_same
    for target in TAIL_SIZES:
        for seed in (0, 1):
            b, e, _ = tail_block_case(target, restart_interval, seed=seed)
            what = "tail %d B ri=%d seed=%d" % (target, restart_interval, seed)
            ref = O.decode_blocks(e.data, e.block_off, 2)
            assert ref.status == 0
            got = rt.Decoder().decode(e.data, e.block_off, 2)
            assert_decode_same(ref, got, what)
            assert np.array_equal(got.key_arena, b.key_bytes), what
            desc = O.decode_blocks(e.data, e.block_off, 2, descending=True)
            assert_decode_same(desc, device_desc(rt, e.data, e.block_off, 2), what + " desc")


@pytest.mark.parametrize("block_size", [8192, 16384])
def test_decode_row_straddles_piece(rt, block_size):  # noqa: F811
    from .decode_cases import _rows, straddle_variants
    from .test_gpu_parity import assert_decode_same
    e = O.encode_sst(_rows(3000, 5), O.params(block_size=block_size, bloom_bits_per_key=0))
    statuses = set()
    for d, data in straddle_variants(e, 1, range(1, 88, 3)):
        ref = O.decode_blocks(data, e.block_off, 2)
        got = rt.Decoder().decode(data, e.block_off, 2)
        statuses.add(ref.status)
        assert_decode_same(ref, got, "straddle +%d bs=%d" % (d, block_size))
    assert len(statuses) >= 1
