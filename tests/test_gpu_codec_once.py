"""f3 decode-once on the device: sdb_decompress_blocks_once (no host synchronisation between sizing and
decompressing; Zlib inflates each block once into a fixed slot and re-plans only the blocks that overflow
it) against the oracle, block for block: the same bytes, the same out_end - out_start and the same first
error as sdb_decompress_plan + sdb_decompress_blocks."""
import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets, runtime

from .codec_util import compress_run, frame

pytestmark = pytest.mark.gpu
torch = pytest.importorskip("torch")

CODECS = [O.CODEC_LZ4, O.CODEC_SNAPPY, O.CODEC_ZLIB, O.CODEC_ZSTD]
NONE = 2**64 - 1


def _dev(a, dt=None):
    t = torch.from_numpy(np.ascontiguousarray(a).view(dt) if dt else np.ascontiguousarray(a))
    return t.to("cuda")


def _once(codec, comp, coff, slot_bytes, out_cap=None):
    out, start, end, err = runtime.decompress_blocks_once_device(codec, _dev(comp), _dev(coff, np.int64), slot_bytes,
                                                                 out_cap=out_cap)
    torch.cuda.synchronize()
    return (out.cpu().numpy(), start.cpu().numpy().view(np.uint64), end.cpu().numpy().view(np.uint64),
            int(err.cpu().numpy().view(np.uint64)[0]))


def _check(codec, comp, coff, slot_bytes, out_cap=None):
    """once == the oracle block for block; returns (out, start, end, err, blocks past their slot)."""
    out, start, end, err = _once(codec, comp, coff, slot_bytes, out_cap)
    r = O.decompress_blocks(codec, comp, coff)
    nb = len(coff) - 1
    assert err == r.first_err
    spilled = 0
    for k in range(nb):
        a, b = int(start[k]), int(end[k])
        ra, rb = int(r.out_start[k]), int(r.out_end[k])
        assert b - a == rb - ra, k
        assert np.array_equal(out[a:b], r.out[ra:rb]), k
        if codec == O.CODEC_ZLIB:
            if a != k * slot_bytes:
                spilled += 1
                assert a >= nb * slot_bytes and b <= int(start[nb]), k
            else:
                assert b <= a + slot_bytes, k
    if codec != O.CODEC_ZLIB:
        assert np.array_equal(start, r.out_start)
    return out, start, end, err, spilled


@pytest.mark.parametrize("codec", CODECS)
@pytest.mark.parametrize("version,block_size,n", [(2, 4096, 20000), (1, 1024, 3000), (2, 65536, 6000)])
def test_once_matches_oracle(codec, version, block_size, n):
    b = datasets.d3(n=n) if version == 1 else datasets.d1(n=n, sst_index=7)
    enc = O.encode_sst(b, O.params(block_size=block_size, sst_version=version, bloom_bits_per_key=0))
    comp, coff = compress_run(codec, enc.data, enc.block_off)
    nb = len(coff) - 1
    sizes = np.diff(enc.block_off.astype(np.int64))
    # slots that fit every block, about half of them, and none
    for slot in (int(sizes.max()) + 8, int(np.median(sizes)) & ~7, 8):
        out, start, end, err, spilled = _check(codec, comp, coff, slot)
        assert err == NONE
        if codec == O.CODEC_ZLIB:
            assert spilled == int((sizes > slot).sum()), slot
        got = b"".join(out[int(start[k]):int(end[k])].tobytes() for k in range(nb))
        assert got == enc.data.tobytes()


@pytest.mark.parametrize("codec", CODECS)
def test_once_then_decode_on_device(codec):
    b = datasets.d1(n=30000, sst_index=2)
    enc = O.encode_sst(b, O.params(block_size=4096, bloom_bits_per_key=0))
    comp, coff = compress_run(codec, enc.data, enc.block_off)
    nb = len(coff) - 1
    out, start, end, err = runtime.decompress_blocks_once_device(codec, _dev(comp), _dev(coff, np.int64), 4096)
    dout = runtime.DeviceDecodeOutput(nb, b.n + 16, int(b.key_off[-1]) + 4096)
    runtime.decode_blocks_at_device(out, start[:nb], end, nb, dout, 2)
    torch.cuda.synchronize()
    assert int(err.cpu().numpy().view(np.uint64)[0]) == NONE
    got = dout.to_host()
    ref = O.decode_blocks(enc.data, enc.block_off, 2)
    assert got.status == 0 and got.summary["num_entries"] == ref.n
    assert np.array_equal(got.key_arena, ref.key_arena) and np.array_equal(got.seq, ref.seq)
    assert np.array_equal(got.val_len, ref.val_len)


@pytest.mark.parametrize("slot", [8, 64, 4096])
def test_once_errors_match_oracle(slot):
    enc = O.encode_sst(datasets.d1(n=3000, sst_index=5), O.params(block_size=4096, bloom_bits_per_key=0))
    for codec in CODECS:
        comp, coff = compress_run(codec, enc.data, enc.block_off)
        c2 = comp.copy()
        c2[int(coff[5]) + 9] ^= 0x01  # CRC mismatch in block 5
        err = _check(codec, c2, coff, slot)[3]
        assert err == (5 << 8) | _abi.SDB_CHECKSUM_MISMATCH
        parts = [comp[int(coff[k]):int(coff[k + 1])].tobytes() for k in range(len(coff) - 1)]
        p = parts[1][:-4]
        parts[1] = frame(p[: len(p) - 7])  # truncated stream in block 1
        c3 = np.frombuffer(b"".join(parts), np.uint8).copy()
        o3 = np.cumsum([0] + [len(x) for x in parts]).astype(np.uint64)
        _check(codec, c3, o3, slot)


def test_once_zlib_streams():
    """zlib at every level / window / strategy, a cut stream and an Adler-32 mismatch, at slots that every
    block, some blocks and no block overflows: once == the oracle."""
    import zlib
    from .test_codec_entropy import payloads
    ps = payloads()
    zl = []
    for i, p in enumerate(ps):
        c = zlib.compressobj([0, 1, 6, 9][i % 4], zlib.DEFLATED, [9, 12, 15][i % 3], 8,
                             [zlib.Z_DEFAULT_STRATEGY, zlib.Z_FIXED, zlib.Z_HUFFMAN_ONLY, zlib.Z_RLE][i % 4])
        zl.append(c.compress(p) + c.flush())
    zl.append(zlib.compress(ps[8])[:-9])
    bad = bytearray(zlib.compress(ps[8]))
    bad[-1] ^= 1
    zl.append(bytes(bad))
    parts = [frame(p) for p in zl]
    comp = np.frombuffer(b"".join(parts), np.uint8).copy()
    coff = np.cumsum([0] + [len(x) for x in parts]).astype(np.uint64)
    big = max(len(p) for p in ps) + 16
    for slot in (8, 256, 4096, big):
        err = _check(O.CODEC_ZLIB, comp, coff, slot)[3]
        assert err == ((len(zl) - 1) << 8) | _abi.SDB_DECOMPRESSION_ERROR


def test_once_capacity_and_arguments():
    enc = O.encode_sst(datasets.d1(n=3000, sst_index=5), O.params(block_size=4096, bloom_bits_per_key=0))
    comp, coff = compress_run(O.CODEC_ZLIB, enc.data, enc.block_off)
    nb = len(coff) - 1
    # room for the slots only: every overflowing block fails with SDB_INVALID_ARGUMENT (the first in order)
    sizes = np.diff(enc.block_off.astype(np.int64))
    slot = int(np.median(sizes)) & ~7
    first = int(np.nonzero(sizes > slot)[0][0])
    _, start, end, err = _once(O.CODEC_ZLIB, comp, coff, slot, out_cap=nb * slot)
    assert err == (first << 8) | _abi.SDB_INVALID_ARGUMENT
    for k in range(nb):
        if sizes[k] <= slot:
            assert int(end[k]) - int(start[k]) == sizes[k]
        else:
            assert int(end[k]) == int(start[k])
    lib = runtime.lib()
    z = torch.zeros(1 << 16, dtype=torch.uint8, device="cuda")
    ws = torch.zeros(int(lib.sdb_decompress_once_workspace_bytes(4)), dtype=torch.uint8, device="cuda")
    p = z.data_ptr()
    for codec, slot_bytes, cap in ((0, 64, 4096), (5, 64, 4096), (O.CODEC_ZLIB, 4, 4096), (O.CODEC_ZLIB, 2048, 4096)):
        assert lib.sdb_decompress_blocks_once(codec, p, p, 4, slot_bytes, p, cap, p, p, p, ws.data_ptr(), ws.numel(),
                                              None) == _abi.SDB_INVALID_ARGUMENT
    assert lib.sdb_decompress_blocks_once(O.CODEC_ZLIB, p, p, 4, 64, p, 4096, p, p, p, ws.data_ptr(), 16,
                                          None) == _abi.SDB_INVALID_ARGUMENT


def _device_compressed(codec, data, block_off):
    cz, czoff, err = runtime.compress_blocks_device(codec, _dev(data), _dev(block_off, np.int64))
    torch.cuda.synchronize()
    assert int(err.cpu().numpy().view(np.uint64)[0]) == NONE
    nb = len(block_off) - 1
    off = czoff.cpu().numpy().view(np.uint64)[: nb + 1].copy()
    return cz.cpu().numpy()[: int(off[nb])].copy(), off


@pytest.mark.parametrize("slot", [8, 2048, 4160])
def test_once_zlib_wide_pass(slot):
    """The wide pass (every lane a decoder against the fixed code's shared tables): blocks the device write
    side compressed (fixed-Huffman / stored deflate), alone and interleaved with Python-zlib blocks (dynamic
    Huffman, listed for the per-decoder-table pass), at slots every block, some blocks and no block
    overflows: once == the oracle, and the bytes == the uncompressed blocks."""
    b = datasets.d1(n=20000, sst_index=3)
    enc = O.encode_sst(b, O.params(block_size=4096, bloom_bits_per_key=0))
    nb = len(enc.block_off) - 1
    fixed, foff = _device_compressed(O.CODEC_ZLIB, enc.data, enc.block_off)
    dyn, doff = compress_run(O.CODEC_ZLIB, enc.data, enc.block_off)
    parts = [(fixed[int(foff[k]):int(foff[k + 1])] if k % 3 else dyn[int(doff[k]):int(doff[k + 1])]).tobytes()
             for k in range(nb)]
    mixed = np.frombuffer(b"".join(parts), np.uint8).copy()
    moff = np.cumsum([0] + [len(x) for x in parts]).astype(np.uint64)
    for comp, coff in ((fixed, foff), (mixed, moff)):
        out, start, end, err, _ = _check(O.CODEC_ZLIB, comp, coff, slot)
        assert err == NONE
        got = b"".join(out[int(start[k]):int(end[k])].tobytes() for k in range(nb))
        assert got == enc.data.tobytes()
    # a corrupt fixed-code block (CRC) and a truncated one among them
    c2 = mixed.copy()
    c2[int(moff[4]) + 5] ^= 0x40
    assert _check(O.CODEC_ZLIB, c2, moff, slot)[3] == (4 << 8) | _abi.SDB_CHECKSUM_MISMATCH
    p = parts[5][:-4]
    parts2 = list(parts)
    parts2[5] = frame(p[: len(p) // 2])
    c3 = np.frombuffer(b"".join(parts2), np.uint8).copy()
    o3 = np.cumsum([0] + [len(x) for x in parts2]).astype(np.uint64)
    _check(O.CODEC_ZLIB, c3, o3, slot)
