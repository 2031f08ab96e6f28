"""Hand-shaped SSTs for the decoder's size boundaries (sdb_decode.hip): a last block of an exact byte size
(around the count pass's 4096-byte staging cap and the emit pass's 6144-byte one, where the piece walk
must not run over a block staged whole in the same LDS image), and V2 blocks whose rows straddle a
restart region that is also a piece boundary (for_each_piece cuts pieces at <= 3968 bytes)."""
import functools
import struct
import zlib

import numpy as np

from oracle import oracle as O
from slatedb_amd.batch import Batch

PIECE_BYTES = 3968  # sdb_decode.hip kPieceBytes


@functools.lru_cache(maxsize=8)
def _entries(seed, n=4000):
    rng = np.random.default_rng(seed)
    return [(b"key%05d/%06d" % (i // 7, i), 0, bytes(rng.integers(0, 256, int(rng.integers(8, 40)), dtype=np.uint8)),
             100000 - i, None, None) for i in range(n)]


def _rows(n, seed, last_vlen=None):
    ents = list(_entries(seed)[:n])
    if last_vlen is not None:
        k, kind, v, sq, c, x = ents[-1]
        ents[-1] = (k, kind, (v * 8)[:last_vlen], sq, c, x)
    return Batch.from_entries(ents)


def _tail_size(e):
    nb = len(e.block_off) - 1
    return int(e.block_off[nb] - e.block_off[nb - 1])


def tail_block_case(target, restart_interval, block_size=8192, seed=0, lead_blocks=2):
    """A batch whose encoded SST (V2, `block_size`) is `lead_blocks` full blocks then a last block of
    exactly `target` bytes (CRC included), so the last block starts at an offset the seed decides.  The
    last entry's value length tunes the size byte for byte (1-byte varint)."""
    prm = O.params(block_size=block_size, restart_interval=restart_interval, bloom_bits_per_key=0)
    enc = lambda n, lv=None: O.encode_sst(_rows(n, seed, lv), prm)
    nblk = lambda n: len(enc(n).block_off) - 1
    lo, hi = 2, len(_entries(seed))
    while lo < hi:  # the first n with lead_blocks + 1 blocks
        mid = (lo + hi) // 2
        lo, hi = (mid + 1, hi) if nblk(mid) <= lead_blocks else (lo, mid)
    first = lo
    lo, hi = first, len(_entries(seed))
    while lo < hi:  # then the first n whose last block reaches target - 60 bytes
        mid = (lo + hi) // 2
        e = enc(mid)
        if len(e.block_off) - 1 == lead_blocks + 1 and _tail_size(e) < target - 60:
            lo = mid + 1
        else:
            hi = mid
    for n in range(max(lo - 2, first), lo + 3):
        e = enc(n)
        if len(e.block_off) - 1 != lead_blocks + 1:
            continue
        base = _rows(n, seed)
        lastv = int(base.val_off[n] - base.val_off[n - 1])
        need = lastv + target - _tail_size(e)
        if 0 <= need < 128:
            e = enc(n, need)
            if len(e.block_off) - 1 == lead_blocks + 1 and _tail_size(e) == target:
                return _rows(n, seed, need), e, prm
    raise AssertionError("no tail block of %d bytes" % target)


def _varint(d, p):
    v = sh = 0
    while True:
        b = d[p]
        p += 1
        v |= (b & 0x7F) << sh
        if not b & 0x80:
            return v, p
        sh += 7


def v2_rows(blk, start, end):
    """Row start positions of a V2 restart region [start, end) of a CRC-stripped block."""
    out, p = [], start
    while p < end:
        out.append(p)
        _, p = _varint(blk, p)
        uns, p = _varint(blk, p)
        vl, p = _varint(blk, p)
        p += uns + vl
        flags = blk[p + 8]
        p += 9 + (8 if flags & 2 else 0) + (8 if flags & 4 else 0)  # HAS_EXPIRE_TS 2, HAS_CREATE_TS 4
    assert p == end
    return out


def piece_cuts(offs, data_end):
    """for_each_piece's greedy cut of a block's restart regions: the first region of each piece."""
    R = len(offs)
    cuts, qa = [], 0
    while qa < R:
        cuts.append(qa)
        base, q = offs[qa], qa
        while q < R and q - qa < 64 and (offs[q + 1] if q + 1 < R else data_end) - base <= PIECE_BYTES:
            q += 1
        qa = q
    return cuts


def straddle_variants(e, block, bumps):
    """Copies of SST `e`'s data where the value-length varint of the last row before a piece boundary in
    `block` is raised by each of `bumps` (the row then runs into the next piece), CRC recomputed."""
    s, t = int(e.block_off[block]), int(e.block_off[block + 1])
    blk = bytearray(e.data[s:t - 4].tobytes())
    cnt = struct.unpack(">H", blk[-2:])[0]
    data_end = len(blk) - 2 - 2 * cnt
    offs = [struct.unpack(">H", blk[data_end + 2 * i:data_end + 2 * i + 2])[0] for i in range(cnt)]
    cuts = piece_cuts(offs, data_end)
    assert len(cuts) >= 2, "block %d is one piece" % block
    q = cuts[1] - 1  # the last region of the first piece
    rows = v2_rows(blk, offs[q], offs[q + 1])
    p = rows[-1]
    _, p1 = _varint(blk, p)
    _, p2 = _varint(blk, p1)
    vl, p3 = _varint(blk, p2)
    assert p3 == p2 + 1, "one-byte value length expected"
    out = []
    for d in bumps:
        nv = vl + d
        assert nv < 128
        b2 = bytearray(blk)
        b2[p2] = nv
        data = e.data.copy()
        data[s:t - 4] = np.frombuffer(bytes(b2), np.uint8)
        data[t - 4:t] = np.frombuffer(struct.pack(">I", zlib.crc32(bytes(b2))), np.uint8)
        out.append((d, data))
    return out
