"""f3 oracle: LZ4 block / Snappy raw decompression (format/sst.rs:884-917) and the compressed-block
read step (decode_block, format/sst.rs:980-999), pinned by round trips through the canonical C++
codecs (pyarrow) — see tests/codec_util.py."""
import struct

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets

from .codec_util import compress_payload, compress_run, frame

CODECS = [O.CODEC_LZ4, O.CODEC_SNAPPY]


def _inputs():
    rng = np.random.default_rng(11)
    yield b""
    yield b"x"
    yield b"abcd" * 3
    yield bytes(rng.integers(0, 256, 4096, dtype=np.uint8))                # incompressible: literals only
    yield bytes(rng.integers(0, 3, 5000, dtype=np.uint8))                   # short matches
    yield b"a" * 10000                                                      # offset-1 overlapping matches
    yield (b"0123456789abcdefghij" * 400)[:7777]                            # offset 20 < match length
    yield bytes(rng.integers(0, 256, 300, dtype=np.uint8)) * 40              # offset 300, long matches
    yield bytes(rng.integers(0, 256, 70000, dtype=np.uint8))                # long literal runs (extensions)


@pytest.mark.parametrize("codec", CODECS)
def test_round_trip_canonical_codecs(codec):
    for raw in _inputs():
        st, out = O.decompress(codec, compress_payload(codec, raw))
        assert st == 0 and out == raw


def test_snappy_hand_built_elements():
    # varint 20; literal "abcd" (tag 0x0C); copy-1 len 8 off 4 (tag 0x11, 0x04); copy-2 len 4 off 6
    # (tag 0x0E, 06 00); copy-4 len 4 off 2 (tag 0x0F, 02 00 00 00)
    s = bytes([20, 0x0C]) + b"abcd" + bytes([0x11, 0x04, 0x0E, 0x06, 0x00, 0x0F, 0x02, 0, 0, 0])
    st, out = O.decompress(O.CODEC_SNAPPY, s)
    assert st == 0
    ref = bytearray(b"abcd")
    for ln, off in ((8, 4), (4, 6), (4, 2)):
        for _ in range(ln):
            ref.append(ref[-off])
    assert out == bytes(ref) and len(out) == 20
    # 60..63 literal tags: 1..4 little-endian length bytes
    lit = bytes(range(200))
    st, out = O.decompress(O.CODEC_SNAPPY, bytes([200, 1]) + bytes([60 << 2, 199]) + lit)
    assert st == 0 and out == lit


def test_lz4_hand_built_sequences():
    # token 0x4F: 4 literals, match length 15 + 4 + ext (255, 3) = 277, offset 2; then 3 trailing literals
    blk = bytes([0x4F]) + b"wxyz" + struct.pack("<H", 2) + bytes([255, 3]) + bytes([0x30]) + b"END"
    ref = bytearray(b"wxyz")
    for _ in range(15 + 4 + 255 + 3):
        ref.append(ref[-2])
    ref += b"END"
    st, out = O.decompress(O.CODEC_LZ4, struct.pack("<I", len(ref)) + blk)
    assert st == 0 and out == bytes(ref)
    # lz4_flex truncates to what was written when the declared size is larger
    st, out = O.decompress(O.CODEC_LZ4, struct.pack("<I", len(ref) + 100) + blk)
    assert st == 0 and out == bytes(ref)


@pytest.mark.parametrize("codec", CODECS)
def test_malformed_payloads_fail(codec):
    good = compress_payload(codec, b"hello hello hello hello hello world")
    bad = [good[: len(good) - 3], good[:1]]
    if codec == O.CODEC_LZ4:
        bad.append(struct.pack("<I", 8) + bytes([0x10]) + b"a" + struct.pack("<H", 0))   # offset 0
        bad.append(struct.pack("<I", 8) + bytes([0x10]) + b"a" + struct.pack("<H", 5))   # offset past output
        bad.append(struct.pack("<I", 2) + bytes([0x30]) + b"abc")                        # past declared size
    else:
        bad.append(bytes([8, 0x00]) + b"a" + bytes([0x01 | (0 << 2), 0]))                # offset 0
        bad.append(bytes([5, 0x00]) + b"a")                                              # short output
        bad.append(bytes([1, 0x04]) + b"ab")                                             # past declared size
    for b in bad:
        st, _ = O.decompress(codec, b)
        assert st == _abi.SDB_DECOMPRESSION_ERROR, b


@pytest.mark.parametrize("codec", CODECS)
@pytest.mark.parametrize("version,block_size", [(2, 4096), (1, 1024), (2, 65536)])
def test_compressed_block_run_restores_the_data_section(codec, version, block_size):
    b = datasets.d3(n=2500) if version == 1 else datasets.d1(n=6000, sst_index=3)
    enc = O.encode_sst(b, O.params(block_size=block_size, sst_version=version, bloom_bits_per_key=0))
    assert enc.status == 0
    comp, coff = compress_run(codec, enc.data, enc.block_off)
    r = O.decompress_blocks(codec, comp, coff)
    assert r.status == 0 and r.first_err == 2**64 - 1
    nb = len(coff) - 1
    assert np.array_equal(r.out_end, r.out_start[1:])  # declared == actual: a contiguous run
    # the decompressed blocks re-framed with the CRC of their bytes are the uncompressed data section
    assert np.array_equal(r.out[: int(r.out_start[nb])], enc.data)
    d = O.decode_blocks(r.out[: int(r.out_start[nb])], r.out_start, version)
    ref = O.decode_blocks(enc.data, enc.block_off, version)
    assert d.status == 0 and np.array_equal(d.key_arena, ref.key_arena) and np.array_equal(d.seq, ref.seq)


@pytest.mark.parametrize("codec", CODECS)
def test_block_run_errors(codec):
    enc = O.encode_sst(datasets.d1(n=800, sst_index=5), O.params(block_size=4096, bloom_bits_per_key=0))
    comp, coff = compress_run(codec, enc.data, enc.block_off)
    # a flipped byte in block 3: validate_checksum fails there first
    c2 = comp.copy()
    c2[int(coff[3]) + 7] ^= 0x40
    r = O.decompress_blocks(codec, c2, coff)
    assert r.status == _abi.SDB_CHECKSUM_MISMATCH and r.first_err == (3 << 8) | _abi.SDB_CHECKSUM_MISMATCH
    assert r.out_end[3] == r.out_start[3]
    # a payload that passes the CRC but does not decode (truncated stream, re-framed): block 2
    parts = [comp[int(coff[k]):int(coff[k + 1])].tobytes() for k in range(len(coff) - 1)]
    p2 = parts[2][:-4]
    parts[2] = frame(p2[: len(p2) // 2])
    c3 = np.frombuffer(b"".join(parts), np.uint8)
    o3 = np.cumsum([0] + [len(p) for p in parts]).astype(np.uint64)
    r = O.decompress_blocks(codec, c3, o3)
    assert r.first_err == (2 << 8) | _abi.SDB_DECOMPRESSION_ERROR
    # an unknown codec number
    assert O.decompress_blocks(9, comp, coff).status == _abi.SDB_UNSUPPORTED
