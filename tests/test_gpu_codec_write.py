"""f3 write side: sdb_compress_blocks (compress_and_transform with SsTableFormat::compress,
format/sst.rs:525-594) on the device, every codec.  The crates that define the reference's compressed
bytes (lz4_flex, snap, flate2, zstd) are not in /root/reference, so byte parity with them is unpinned;
validity is pinned instead: every compressed block carries the CRC32 of its compressed bytes, and
decompresses to the uncompressed block through the oracle's decompressors, through this image's
canonical codecs (pyarrow LZ4 / Snappy / zstd, Python zlib) and through the device decompressor, after
which the SST decodes (sdb_decompress_* -> sdb_decode_blocks_at) to the oracle's columns."""
import struct
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import datasets

from .test_gpu_parity import assert_decode_same, rt  # noqa: F401

pytestmark = pytest.mark.gpu

CODECS = [O.CODEC_LZ4, O.CODEC_SNAPPY, O.CODEC_ZLIB, O.CODEC_ZSTD]


def canonical_decompress(codec, payload, n):
    import pyarrow as pa
    if codec == O.CODEC_LZ4:
        assert struct.unpack("<I", payload[:4])[0] == n
        return pa.decompress(payload[4:], decompressed_size=n, codec="lz4_raw", asbytes=True)
    if codec == O.CODEC_SNAPPY:
        return pa.decompress(payload, decompressed_size=n, codec="snappy", asbytes=True)
    if codec == O.CODEC_ZLIB:
        return zlib.decompress(payload)
    return pa.Codec("zstd").decompress(payload, decompressed_size=n, asbytes=True)


def compressed_on_device(rt, codec, data, off):  # noqa: F811
    import torch
    d = torch.from_numpy(np.concatenate([np.asarray(data, np.uint8), np.zeros(64, np.uint8)])).cuda()
    o = torch.from_numpy(np.asarray(off, np.uint64).view(np.int64)).cuda()
    out, out_off, err = rt.compress_blocks_device(codec, d, o)
    torch.cuda.synchronize()
    assert int(err.item()) == -1, hex(int(err.item()))
    coff = out_off.cpu().numpy().view(np.uint64)
    comp = out[:int(coff[-1])].cpu().numpy()
    return comp, coff


def canonical_compress(codec, raw):
    """The canonical library's stream for one block, framed like compress_and_transform (lz4: + the u32 size
    prefix of lz4_flex::compress_prepend_size); the CRC is not counted."""
    import pyarrow as pa
    if codec == O.CODEC_ZLIB:
        return zlib.compress(raw, 6)                  # flate2's default level
    if codec == O.CODEC_ZSTD:
        return pa.Codec("zstd", compression_level=3).compress(raw, asbytes=True)  # zstd::bulk::compress(data, 3)
    if codec == O.CODEC_LZ4:
        return b"\0\0\0\0" + pa.Codec("lz4_raw").compress(raw, asbytes=True)
    return pa.Codec("snappy").compress(raw, asbytes=True)


# device bytes / library bytes on the same blocks: zstd and zlib within 5 % of zstd level 3 / zlib level 6;
# lz4 / snappy (single-probe like lz4_flex / snap) within 10 % of the C libraries
RATIO_BOUND = {O.CODEC_LZ4: 1.10, O.CODEC_SNAPPY: 1.10, O.CODEC_ZLIB: 1.05, O.CODEC_ZSTD: 1.05}


def datasets_for_write():
    d3 = datasets.d3(n=3000)
    yield "d1", datasets.d1(n=20000, sst_index=4), 4096
    yield "text", datasets.text_kv(n=8000), 4096
    yield "d3", d3, 4096
    yield "d3-1k", d3, 1024
    # compressible blocks: repeated values and runs of equal bytes
    b = datasets.d1(n=8000, sst_index=5)
    v = np.asarray(b.val_bytes, np.uint8).reshape(-1, 100)
    v[:, 40:] = v[:, :1]
    v[::3] = 7
    b.val_bytes = v.reshape(-1).copy()
    yield "repetitive", b, 4096


@pytest.mark.parametrize("codec", CODECS)
def test_compressed_blocks_decompress_everywhere(rt, codec):  # noqa: F811
    for name, b, bs in datasets_for_write():
        e = O.encode_sst(b, O.params(block_size=bs))
        comp, coff = compressed_on_device(rt, codec, e.data, e.block_off)
        nb = len(e.block_off) - 1
        assert len(coff) == nb + 1 and coff[0] == 0
        for k in range(nb):
            blk = comp[int(coff[k]):int(coff[k + 1])]
            payload, crc = blk[:-4].tobytes(), struct.unpack(">I", blk[-4:].tobytes())[0]
            assert crc == zlib.crc32(payload), (name, k)
            raw = e.data[int(e.block_off[k]):int(e.block_off[k + 1]) - 4].tobytes()
            assert canonical_decompress(codec, payload, len(raw)) == raw, (name, codec, k)
        # the oracle's decompressors, then its decode
        r = O.decompress_blocks(codec, comp, coff)
        assert r.status == 0 and r.first_err == 0xFFFFFFFFFFFFFFFF, (r.status, r.first_err)
        for k in range(nb):
            got = r.out[int(r.out_start[k]):int(r.out_end[k])]
            assert np.array_equal(got, e.data[int(e.block_off[k]):int(e.block_off[k + 1])]), (name, k)
        if name in ("repetitive", "text"):
            assert int(coff[-1]) < len(e.data) * (0.8 if name == "repetitive" else 0.5), (name, codec, int(coff[-1]))
        if name in ("d1", "text"):
            # compression ratio against the canonical library on the same blocks (parity of the bytes: unpinned)
            lib = sum(len(canonical_compress(codec, e.data[int(e.block_off[k]):int(e.block_off[k + 1]) - 4].tobytes()))
                      for k in range(nb))
            dev = int(coff[-1]) - 4 * nb
            print("ratio %s %s device %d library %d -> %.4f" % (name, codec, dev, lib, dev / lib))
            assert dev <= RATIO_BOUND[codec] * lib, (name, codec, dev, lib)


@pytest.mark.parametrize("codec", CODECS)
def test_compressed_sst_decodes_on_device(rt, codec):  # noqa: F811
    import torch
    b = datasets.d1(n=30000, sst_index=6)
    e = O.encode_sst(b, O.params())
    comp, coff = compressed_on_device(rt, codec, e.data, e.block_off)
    nb = len(coff) - 1
    blocks = torch.from_numpy(np.concatenate([comp, np.zeros(64, np.uint8)])).cuda()
    boff = torch.from_numpy(coff.view(np.int64)).cuda()
    out, out_start, out_end, err = rt.decompress_blocks_device(codec, blocks, boff)
    torch.cuda.synchronize()
    assert int(err.item()) == -1
    n_ent = b.n
    dout = rt.DeviceDecodeOutput(nb, n_ent + 64, len(b.key_bytes) + 4096)
    rt.decode_blocks_at_device(out, out_start[:nb].contiguous(), out_end.contiguous(), nb, dout, 2)
    torch.cuda.synchronize()
    got = dout.to_host()
    ref = O.decode_blocks(e.data, e.block_off, 2)
    assert got.status == 0 and got.n == ref.n
    assert np.array_equal(got.key_arena, ref.key_arena) and np.array_equal(got.seq, ref.seq)
    assert np.array_equal(got.val_len, ref.val_len)


def _big_value_batch(n=40, vlen=20000, seed=21):
    """Values far longer than a 4 KiB window of random bytes: windows with no match at all."""
    from slatedb_amd.batch import Batch
    rng = np.random.default_rng(seed)
    es = [(b"big:%06d" % i, 0, rng.integers(0, 256, vlen, dtype=np.uint8).tobytes(), 7, None, None) for i in range(n)]
    return Batch.from_entries(es)


@pytest.mark.parametrize("block_size", [8192, 16384, 65536])
def test_big_blocks_windows(rt, block_size):  # noqa: F811
    """SstBlockSize 8-64 KiB: a block over 4 KiB is compressed as consecutive 4 KiB windows (zstd blocks of one
    frame, deflate blocks of one stream, snappy elements, lz4 windows that end at their last match; lz4 falls back
    to a literal-only stream when a window has no match to end on)."""
    text = datasets.text_kv(n=4000, seed=13)
    for name, b in (("text", text), ("d1", datasets.d1(n=6000, sst_index=8)), ("random", _big_value_batch())):
        e = O.encode_sst(b, O.params(block_size=block_size))
        for codec in CODECS:
            comp, coff = compressed_on_device(rt, codec, e.data, e.block_off)
            for k in range(len(coff) - 1):
                blk = comp[int(coff[k]):int(coff[k + 1])]
                payload = blk[:-4].tobytes()
                assert struct.unpack(">I", blk[-4:].tobytes())[0] == zlib.crc32(payload), (name, codec, k)
                raw = e.data[int(e.block_off[k]):int(e.block_off[k + 1]) - 4].tobytes()
                assert canonical_decompress(codec, payload, len(raw)) == raw, (name, codec, k)
            r = O.decompress_blocks(codec, comp, coff)
            assert r.status == 0 and r.first_err == 0xFFFFFFFFFFFFFFFF, (name, codec, r.status)
            if name == "text":
                assert int(coff[-1]) < 0.5 * len(e.data), (codec, block_size, int(coff[-1]), len(e.data))


def test_capacity_and_arguments(rt):  # noqa: F811
    import torch
    from slatedb_amd import _abi
    b = datasets.d1(n=3000, sst_index=9)
    e = O.encode_sst(b, O.params())
    d = torch.from_numpy(np.concatenate([e.data, np.zeros(64, np.uint8)])).cuda()
    o = torch.from_numpy(np.asarray(e.block_off, np.uint64).view(np.int64)).cuda()
    out, out_off, err = rt.compress_blocks_device(O.CODEC_LZ4, d, o, out_cap=100)
    torch.cuda.synchronize()
    assert (int(err.item()) & 0xFF) == _abi.SDB_LIMIT_EXCEEDED
    with pytest.raises(rt.SdbError):
        rt.compress_blocks_device(0, d, o)
    # in_bytes smaller than the blocks span: the blocks past it are refused, nothing is written past the slots
    out, out_off, err = rt.compress_blocks_device(O.CODEC_ZSTD, d, o, in_bytes=int(e.block_off[-1]) // 2)
    torch.cuda.synchronize()
    assert (int(err.item()) & 0xFF) == _abi.SDB_INVALID_ARGUMENT
