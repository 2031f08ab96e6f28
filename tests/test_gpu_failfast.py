"""SDB_DECODE_FAIL_FAST (read_blocks semantics): the checksums move to the emit pass.  The status is the
first failing block's in block order with its checksum ahead of its rows (the oracle's), every bad block
is listed, and a clean decode is bit-exact with the oracle, ascending and descending."""
import struct
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import datasets

from .test_gpu_parity import assert_decode_same, rt  # noqa: F401

pytestmark = pytest.mark.gpu


def ff_decode(rt, data, block_off, version, descending=False):  # noqa: F811
    import torch
    nb = len(block_off) - 1
    total = int(block_off[-1])
    dout = rt.DeviceDecodeOutput(nb, total // 8 + 64, total * 8 + 4096)
    arena = torch.from_numpy(np.concatenate([np.asarray(data, np.uint8), np.zeros(64, np.uint8)])).cuda()
    boff = torch.from_numpy(np.asarray(block_off, np.uint64).view(np.int64)).cuda()
    rt.decode_blocks_ex_device(arena, boff, None, nb, dout, version, descending=descending, fail_fast=True)
    torch.cuda.synchronize()
    return dout.to_host()


def check(rt, data, block_off, version, what, descending=False):  # noqa: F811
    ref = O.decode_blocks(data, block_off, version, descending=descending)
    got = ff_decode(rt, data, block_off, version, descending)
    assert got.status == ref.status, (what, got.status, ref.status)
    if ref.status == 0:
        assert_decode_same(ref, got, what)
    else:
        assert sorted(got.bad_block.tolist()) == sorted(ref.bad_block.tolist()), what
    return ref


@pytest.mark.parametrize("version,bs", [(2, 4096), (2, 1024), (1, 4096), (2, 16384)])
def test_fail_fast_clean(rt, version, bs):  # noqa: F811
    for name, b in (("d1", datasets.d1(n=50000, sst_index=2)), ("d3", datasets.d3(n=3000))):
        e = O.encode_sst(b, O.params(sst_version=version, block_size=bs))
        check(rt, e.data, e.block_off, version, "%s v%d bs %d" % (name, version, bs))
        check(rt, e.data, e.block_off, version, "%s v%d bs %d desc" % (name, version, bs), descending=True)


def test_fail_fast_corruption(rt):  # noqa: F811
    """A checksum mismatch the count pass no longer sees (found by the emit pass), a corrupt row with a
    recomputed checksum (found by the count pass), both (the earlier block decides), and a block that
    fails both ways (checksum first)."""
    b = datasets.d1(n=40000, sst_index=6)
    e = O.encode_sst(b, O.params())
    off = e.block_off

    def crc_fix(data, k):
        s, t = int(off[k]), int(off[k + 1])
        data[t - 4:t] = np.frombuffer(struct.pack(">I", zlib.crc32(data[s:t - 4].tobytes())), np.uint8)

    d1 = e.data.copy()
    d1[int(off[9]) + 300] ^= 0x40  # checksum mismatch only
    check(rt, d1, off, 2, "crc only")
    d2 = e.data.copy()
    d2[int(off[4]) + 1] = 0xFF  # a row header run-away in block 4, checksum recomputed
    crc_fix(d2, 4)
    check(rt, d2, off, 2, "rows only")
    d3 = d2.copy()
    d3[int(off[2]) + 50] ^= 0x01  # + a checksum mismatch in an earlier block
    check(rt, d3, off, 2, "crc before rows")
    d4 = e.data.copy()
    d4[int(off[6]) + 1] = 0xFF  # rows and checksum both bad in block 6: checksum reported
    check(rt, d4, off, 2, "both in one block")
    for desc in (False, True):
        check(rt, d3, off, 2, "crc before rows desc=%d" % desc, descending=desc)


@pytest.mark.parametrize("small", [True, False])
def test_fail_fast_over_capacity_reports_checksum(rt, small):  # noqa: F811
    """Counts that exceed the caller's capacity (here: the capacity one entry short) with a block whose
    checksum the count pass deferred: read_blocks fails on the block, so the status is
    CHECKSUM_MISMATCH (the oracle's), not the capacity error, and the block is listed."""
    import torch
    from slatedb_amd import _abi
    b = datasets.d1(n=2000 if small else 60000, sst_index=7)
    e = O.encode_sst(b, O.params())
    off = e.block_off
    nb = len(off) - 1
    bad = nb // 2
    data = e.data.copy()
    data[int(off[bad]) + 200] ^= 0x10  # payload byte: the rows still parse, only the checksum is wrong
    ref = O.decode_blocks(data, off, 2)
    assert ref.status == _abi.SDB_CHECKSUM_MISMATCH
    for cap_e, cap_k in ((b.n - 1, len(b.key_bytes) + 64), (b.n + 64, len(b.key_bytes) - 1)):
        dout = rt.DeviceDecodeOutput(nb, cap_e, cap_k)
        arena = torch.from_numpy(np.concatenate([data, np.zeros(64, np.uint8)])).cuda()
        boff = torch.from_numpy(np.asarray(off, np.uint64).view(np.int64)).cuda()
        rt.decode_blocks_ex_device(arena, boff, None, nb, dout, 2, fail_fast=True)
        torch.cuda.synchronize()
        got = dout.to_host()
        assert got.status == _abi.SDB_CHECKSUM_MISMATCH, (cap_e, cap_k, got.status)
        assert bad in got.bad_block.tolist()
        # without the corruption the same capacities are a plain capacity error
        dout = rt.DeviceDecodeOutput(nb, cap_e, cap_k)
        clean = torch.from_numpy(np.concatenate([e.data, np.zeros(64, np.uint8)])).cuda()
        rt.decode_blocks_ex_device(clean, boff, None, nb, dout, 2, fail_fast=True)
        torch.cuda.synchronize()
        assert dout.to_host().status == _abi.SDB_INVALID_ARGUMENT
