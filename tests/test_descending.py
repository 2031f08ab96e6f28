"""Descending iteration over decoded blocks (sdb_decode_blocks_ex + SDB_DECODE_DESCENDING): the oracle
restatement of SstIterator Descending / DescendingBlockIteratorV2 (block_iterator_v2.rs:318-430) and
BlockIterator Descending (block_iterator.rs:159-224) on the CPU, and the device against it."""
import struct
import zlib

import numpy as np
import pytest

from oracle import oracle as O
from slatedb_amd import _abi, datasets
from slatedb_amd.batch import Batch

from .test_lookup_oracle import dup_batch


def rows(d):
    """(key, val_off, val_len, seq, flags, cts, ets) per entry, timestamps masked by the flags."""
    out = []
    for i in range(d.n):
        f = int(d.flags[i])
        out.append((d.key_arena[int(d.key_off[i]):int(d.key_off[i + 1])].tobytes(), int(d.val_off[i]),
                    int(d.val_len[i]), int(d.seq[i]), f,
                    int(d.create_ts[i]) if f & _abi.FLAG_HAS_CREATE_TS else None,
                    int(d.expire_ts[i]) if f & _abi.FLAG_HAS_EXPIRE_TS else None))
    return out


def irregular_v2(b, bs=512):
    """An encoded V2 SST whose first multi-region block gets restart 1 moved one byte into a row (CRC
    recomputed): the ascending walk ignores restarts, descending iteration cannot."""
    e = O.encode_sst(b, O.params(block_size=bs, restart_interval=2))
    data = bytearray(e.data.tobytes())
    for k in range(len(e.block_off) - 1):
        s, t = int(e.block_off[k]), int(e.block_off[k + 1])
        blen = t - s - 4
        cnt = struct.unpack(">H", data[s + blen - 2:s + blen])[0]
        if cnt >= 2:
            at = s + blen - 2 - 2 * cnt + 2
            r1 = struct.unpack(">H", data[at:at + 2])[0]
            data[at:at + 2] = struct.pack(">H", r1 + 1)
            data[t - 4:t] = struct.pack(">I", zlib.crc32(bytes(data[s:s + blen])))
            return np.frombuffer(bytes(data), np.uint8).copy(), e.block_off, k
    raise AssertionError("no multi-region block")


@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("bs", [256, 4096])
def test_descending_is_reversed_ascending(version, bs):
    for b in (datasets.d3(n=3000), dup_batch()):
        e = O.encode_sst(b, O.params(sst_version=version, block_size=bs))
        asc = O.decode_blocks(e.data, e.block_off, version)
        desc = O.decode_blocks(e.data, e.block_off, version, descending=True)
        assert asc.status == desc.status == 0
        assert rows(desc) == rows(asc)[::-1]
        assert np.array_equal(desc.block_entry_start, asc.block_entry_start)


def test_descending_irregular_oracle_runs():
    data, off, _ = irregular_v2(datasets.d3(n=2000))
    asc = O.decode_blocks(data, off, 2)
    assert asc.status == 0  # the sequential walk ignores the restart table
    O.decode_blocks(data, off, 2, descending=True)  # restated literally; no crash


# ------------------------------------------------------------------------------------------------
# device
# ------------------------------------------------------------------------------------------------
@pytest.fixture(scope="module")
def rt():
    from slatedb_amd import runtime
    runtime.require_device()
    return runtime


def device_desc(rt, data, block_off, version):
    import torch
    nb = len(block_off) - 1
    total = int(block_off[-1])
    dout = rt.DeviceDecodeOutput(nb, total // 8 + 64, total * 8 + 4096)
    arena = torch.from_numpy(np.concatenate([np.asarray(data, np.uint8), np.zeros(64, np.uint8)])).cuda()
    boff = torch.from_numpy(np.asarray(block_off, np.uint64).view(np.int64)).cuda()
    rt.decode_blocks_ex_device(arena, boff, None, nb, dout, version, descending=True)
    torch.cuda.synchronize()
    return dout.to_host()


@pytest.mark.gpu
@pytest.mark.parametrize("version", [1, 2])
@pytest.mark.parametrize("bs", [256, 4096, 16384])
def test_descending_device(rt, version, bs):
    from .test_gpu_parity import assert_decode_same
    for b in (datasets.d3(n=3000), dup_batch(), datasets.d1(n=60000)):
        e = O.encode_sst(b, O.params(sst_version=version, block_size=bs))
        ref = O.decode_blocks(e.data, e.block_off, version, descending=True)
        got = device_desc(rt, e.data, e.block_off, version)
        assert_decode_same(ref, got, "desc v%d bs %d" % (version, bs))


@pytest.mark.gpu
def test_descending_device_bad_blocks(rt):
    from .test_gpu_parity import assert_decode_same
    b = datasets.d3(n=3000)
    e = O.encode_sst(b, O.params(block_size=512))
    data = e.data.copy()
    mid = int(e.block_off[5]) + 7
    data[mid] ^= 0x40  # CRC mismatch in block 5
    ref = O.decode_blocks(data, e.block_off, 2, descending=True)
    got = device_desc(rt, data, e.block_off, 2)
    assert ref.status == _abi.SDB_CHECKSUM_MISMATCH
    assert_decode_same(ref, got, "desc crc")
    # a restart table the descending iterator cannot follow: reported, not decoded
    data, off, k = irregular_v2(b)
    got = device_desc(rt, data, off, 2)
    assert got.status == _abi.SDB_CORRUPT_BLOCK and k in got.bad_block.tolist()
