"""f3 on the device: sdb_decompress_plan / sdb_decompress_blocks against the oracle (and through
sdb_decode_blocks_at), bit-exact.  Compressed runs: tests/codec_util.py."""
import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets, runtime

from .codec_util import compress_run, frame

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CODECS = [O.CODEC_LZ4, O.CODEC_SNAPPY, O.CODEC_ZLIB, O.CODEC_ZSTD]


def _dev(a, dt=None):
    t = torch.from_numpy(np.ascontiguousarray(a).view(dt) if dt else np.ascontiguousarray(a))
    return t.to("cuda")


def _run(codec, comp, coff):
    out, start, end, err = runtime.decompress_blocks_device(codec, _dev(comp), _dev(coff, np.int64))
    torch.cuda.synchronize()
    return (out.cpu().numpy(), start.cpu().numpy().view(np.uint64), end.cpu().numpy().view(np.uint64),
            int(err.cpu().numpy().view(np.uint64)[0]))


def _check(codec, comp, coff):
    out, start, end, err = _run(codec, comp, coff)
    r = O.decompress_blocks(codec, comp, coff)
    assert err == r.first_err
    assert np.array_equal(start, r.out_start) and np.array_equal(end, r.out_end)
    for k in range(len(coff) - 1):
        a, b = int(start[k]), int(end[k])
        assert np.array_equal(out[a:b], r.out[a:b]), k
    return out, start, end, err


@pytest.mark.parametrize("codec", CODECS)
@pytest.mark.parametrize("version,block_size,n", [(2, 4096, 20000), (1, 1024, 3000), (2, 65536, 6000),
                                                  (2, 256, 3000)])
def test_decompress_matches_oracle(codec, version, block_size, n):
    b = datasets.d3(n=n) if version == 1 or block_size == 256 else datasets.d1(n=n, sst_index=7)
    enc = O.encode_sst(b, O.params(block_size=block_size, sst_version=version, bloom_bits_per_key=0))
    comp, coff = compress_run(codec, enc.data, enc.block_off)
    out, start, end, err = _check(codec, comp, coff)
    assert err == 2**64 - 1
    nb = len(coff) - 1
    assert np.array_equal(out[: int(start[nb])], enc.data)  # the uncompressed data section, bit for bit


@pytest.mark.parametrize("codec", CODECS)
def test_decompress_then_decode_on_device(codec):
    b = datasets.d1(n=30000, sst_index=2)
    enc = O.encode_sst(b, O.params(block_size=4096, bloom_bits_per_key=0))
    comp, coff = compress_run(codec, enc.data, enc.block_off)
    out, start, end, err = runtime.decompress_blocks_device(codec, _dev(comp), _dev(coff, np.int64))
    nb = len(coff) - 1
    dout = runtime.DeviceDecodeOutput(nb, b.n + 16, int(b.key_off[-1]) + 4096)
    runtime.decode_blocks_at_device(out, start[:nb], end, nb, dout, 2)
    torch.cuda.synchronize()
    got = dout.to_host()
    ref = O.decode_blocks(enc.data, enc.block_off, 2)
    assert got.status == 0 and got.summary["num_entries"] == ref.n
    assert np.array_equal(got.key_arena, ref.key_arena) and np.array_equal(got.seq, ref.seq)
    assert np.array_equal(got.val_len, ref.val_len) and np.array_equal(got.val_off, ref.val_off)


def test_big_blocks_single_lane_path():
    # 64 KiB blocks of 2 KiB random values: payloads over the 8 KiB stage / 16 KiB image
    rng = np.random.default_rng(4)
    from slatedb_amd.batch import Batch
    ents = [(b"k%08d" % i, 0, bytes(rng.integers(0, 256, 2048, dtype=np.uint8)) * (1 + (i % 3)), 100 - i, None, None)
            for i in range(60)]
    b = Batch.from_entries(ents)
    enc = O.encode_sst(b, O.params(block_size=65536, bloom_bits_per_key=0))
    for codec in CODECS:
        comp, coff = compress_run(codec, enc.data, enc.block_off)
        assert max(np.diff(coff)) > 8192
        out, start, end, err = _check(codec, comp, coff)
        assert err == 2**64 - 1


@pytest.mark.parametrize("codec", CODECS)
def test_device_errors_match_oracle(codec):
    enc = O.encode_sst(datasets.d1(n=3000, sst_index=5), O.params(block_size=4096, bloom_bits_per_key=0))
    comp, coff = compress_run(codec, enc.data, enc.block_off)
    c2 = comp.copy()
    c2[int(coff[5]) + 9] ^= 0x01  # CRC mismatch in block 5
    _, _, _, err = _check(codec, c2, coff)
    assert err == (5 << 8) | _abi.SDB_CHECKSUM_MISMATCH
    parts = [comp[int(coff[k]):int(coff[k + 1])].tobytes() for k in range(len(coff) - 1)]
    p = parts[1][:-4]
    parts[1] = frame(p[: len(p) - 7])  # re-framed truncated stream: decompression error in block 1
    c3 = np.frombuffer(b"".join(parts), np.uint8).copy()
    o3 = np.cumsum([0] + [len(x) for x in parts]).astype(np.uint64)
    _, _, _, err = _check(codec, c3, o3)
    if codec == O.CODEC_ZLIB:  # flate2's read_to_end keeps what a cut stream decodes to (no error)
        assert err == 2**64 - 1
    else:
        assert err == (1 << 8) | _abi.SDB_DECOMPRESSION_ERROR


def test_unknown_codec():
    lib = runtime.lib()
    z = torch.zeros(64, dtype=torch.uint8, device="cuda")
    for c in (0, 5):
        assert lib.sdb_decompress_plan(c, z.data_ptr(), z.data_ptr(), 0, z.data_ptr(), z.data_ptr(), 64, None) == \
            _abi.SDB_INVALID_ARGUMENT


def _raw_run(codec, payloads):
    """Arbitrary payloads (not SST blocks) framed with the CRC, as a block run."""
    parts = [frame(p) for p in payloads]
    return (np.frombuffer(b"".join(parts), np.uint8).copy(),
            np.cumsum([0] + [len(x) for x in parts]).astype(np.uint64))


def test_entropy_codecs_levels_and_frames():
    """zlib at every level / window and strategy, zstd at negative to high levels, multi-block zstd frames
    (repeat tables, treeless literals), hand-built frames (raw / RLE blocks, checksum, skippable and
    concatenated frames) and error streams: device == oracle, and the decoded bytes == the input."""
    import struct
    import zlib
    from .test_codec_entropy import frame as zframe, payloads, zstd_compress
    ps = payloads()
    rng = np.random.default_rng(3)
    words = [bytes(rng.integers(97, 123, rng.integers(2, 9), dtype=np.uint8)) for _ in range(300)]
    big = b" ".join(words[i] for i in rng.integers(0, 300, 60000))  # ~300 KiB: three zstd blocks
    zl = []
    for i, p in enumerate(ps + [big]):
        c = zlib.compressobj([0, 1, 6, 9][i % 4], zlib.DEFLATED, [9, 12, 15][i % 3], 8,
                             [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE][i % 4])
        zl.append(c.compress(p) + c.flush())
    zl.append(zlib.compress(ps[8])[:-9])                # cut stream: the bytes decoded so far
    bad = bytearray(zlib.compress(ps[8]))
    bad[-1] ^= 1
    zl.append(bytes(bad))                               # Adler-32 mismatch
    comp, coff = _raw_run(O.CODEC_ZLIB, zl)
    out, start, end, err = _check(O.CODEC_ZLIB, comp, coff)
    assert err == ((len(zl) - 1) << 8) | _abi.SDB_DECOMPRESSION_ERROR
    for k, p in enumerate(ps + [big]):
        assert out[int(start[k]):int(end[k]) - 4].tobytes() == p, k
    zs = [zstd_compress(p, [-5, 1, 3, 9, 19][i % 5]) for i, p in enumerate(ps)]
    zs += [zstd_compress(big, 1), zstd_compress(big, 12)]
    f = zframe([(0, b"hello world", b"hello world"), (1, bytes([0x41, 200]), b"A" * 200)], checksum=True)
    skip = struct.pack("<II", 0x184D2A53, 5) + b"12345"
    zs += [f, skip + zs[8] + f + skip, zs[8][:-3]]
    comp, coff = _raw_run(O.CODEC_ZSTD, zs)
    out, start, end, err = _check(O.CODEC_ZSTD, comp, coff)
    assert err == ((len(zs) - 1) << 8) | _abi.SDB_DECOMPRESSION_ERROR
    want = ps + [big, big, b"hello world" + b"A" * 200, ps[8] + b"hello world" + b"A" * 200]
    for k, p in enumerate(want):
        assert out[int(start[k]):int(end[k]) - 4].tobytes() == p, k


def test_zstd_plan_from_frame_content_size():
    """The zstd plan reads Frame_Content_Size from the frame headers (zstd::bulk::compress writes it,
    format/sst.rs:590) and decodes in count mode only for frames without one: device == oracle for
    frames with and without a content size, a content size above / below what the frame decodes to,
    and concatenated frames mixing both."""
    from .test_codec_entropy import frame as zframe, payloads, zstd_compress
    raw = (0, b"hello world", b"hello world")
    rle = (1, bytes([0x41, 200]), b"A" * 200)
    ps = payloads()
    cases = [
        ([zstd_compress(ps[8], 3), zframe([raw, rle]), zframe([raw], fcs=False)], None),
        ([zframe([raw, rle], fcs=False) + zstd_compress(ps[8], 1)], None),
        ([zframe([raw], content=b"hello world!")], 0),   # declares more than it decodes to
        ([zframe([raw, rle], content=b"hello")], 0),     # declares less: overflows its slot
        ([zstd_compress(ps[3], 3), zframe([raw], content=b"hello world!!", checksum=True)], 1),
    ]
    for i, (streams, bad) in enumerate(cases):
        comp, coff = _raw_run(O.CODEC_ZSTD, streams)
        out, start, end, err = _check(O.CODEC_ZSTD, comp, coff)
        if bad is None:
            assert err == 2**64 - 1, i
        else:
            assert err == (bad << 8) | _abi.SDB_DECOMPRESSION_ERROR, i
