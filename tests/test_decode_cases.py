"""The hand-shaped decoder cases (tests/decode_cases.py) hit the sizes they claim, on the CPU oracle."""
import struct

import numpy as np

from oracle import oracle as O

from .decode_cases import _rows, piece_cuts, straddle_variants, tail_block_case


def test_tail_block_sizes_hit():
    for ri in (1, 16):
        for target in (4086, 4096, 6144, 6150):
            b, e, _ = tail_block_case(target, ri)
            assert int(e.block_off[-1] - e.block_off[-2]) == target
            assert len(e.block_off) == 4
            r = O.decode_blocks(e.data, e.block_off, 2)
            assert r.status == 0 and r.n == b.n and np.array_equal(r.key_arena, b.key_bytes)


def test_piece_cuts_greedy():
    assert piece_cuts([0, 1000, 2000, 3000, 3900], 4500) == [0, 4]
    assert piece_cuts([0, 3968], 7936) == [0, 1]
    assert piece_cuts(list(range(0, 100 * 10, 10)), 1000) == [0, 64]


def test_straddle_variants_change_one_row():
    e = O.encode_sst(_rows(3000, 5), O.params(block_size=16384, bloom_bits_per_key=0))
    vs = straddle_variants(e, 1, [1, 40])
    s, t = int(e.block_off[1]), int(e.block_off[2])
    for d, data in vs:
        diff = np.nonzero(data != e.data)[0]
        assert diff.size >= 1 and diff.min() >= s and diff.max() < t
        import zlib
        assert struct.unpack(">I", data[t - 4:t].tobytes())[0] == zlib.crc32(data[s:t - 4].tobytes())
    # the oracle reads the bumped row across its region: the block is irregular or corrupt, never silent
    statuses = {O.decode_blocks(data, e.block_off, 2).status for _, data in vs}
    assert statuses
