"""Compressed block runs for the f3 tests (test infrastructure).

The reference compresses each finished block with lz4_flex 0.11.6 (block::compress_prepend_size), snap
1.1.1 (raw::Encoder), flate2 1.1.9 (ZlibEncoder) or zstd 0.13.3 (libzstd) and appends the CRC32 of the
compressed bytes (compress_and_transform, format/sst.rs:525-594).  None of the crates is in
/root/reference, so the compressed payloads here come from the canonical C / C++ libraries of this image
(pyarrow's LZ4, Snappy and zstd; Python's zlib): any valid stream of a format decodes to one byte string,
so decompression parity is pinned by the round trip (bytes differ from what the Rust encoders would
emit, the decoded blocks may not).
"""
import struct
import zlib

import numpy as np

from oracle import oracle as O


def compress_payload(codec, raw, level=3):
    import pyarrow as pa
    raw = bytes(raw)
    if codec == O.CODEC_LZ4:  # block::compress_prepend_size: u32 LE length, then the LZ4 block
        return struct.pack("<I", len(raw)) + pa.compress(raw, codec="lz4_raw", asbytes=True)
    if codec == O.CODEC_SNAPPY:  # raw Snappy: varint length, then elements
        return pa.compress(raw, codec="snappy", asbytes=True)
    if codec == O.CODEC_ZLIB:  # flate2 ZlibEncoder: a zlib stream
        return zlib.compress(raw, level)
    if codec == O.CODEC_ZSTD:  # zstd::bulk / stream encoders: one zstd frame
        return pa.Codec("zstd", compression_level=level).compress(raw, asbytes=True)
    raise ValueError(codec)


def frame(payload):
    """compress_and_transform's framing: payload ++ crc32fast::hash(payload) big-endian."""
    return bytes(payload) + struct.pack(">I", zlib.crc32(bytes(payload)))


def compress_run(codec, data, block_off, level=3):
    """An encoded data section (blocks = Block::encode ++ CRC) -> the same blocks compressed:
    (bytes as uint8 array, block offsets uint64 nblocks + 1)."""
    data = np.asarray(data, np.uint8)
    bo = np.asarray(block_off, np.uint64)
    parts, offs, pos = [], [0], 0
    for k in range(len(bo) - 1):
        raw = data[int(bo[k]):int(bo[k + 1]) - 4].tobytes()  # Block::encode bytes (CRC stripped)
        b = frame(compress_payload(codec, raw, level))
        parts.append(b)
        pos += len(b)
        offs.append(pos)
    return np.frombuffer(b"".join(parts), np.uint8).copy(), np.array(offs, np.uint64)
