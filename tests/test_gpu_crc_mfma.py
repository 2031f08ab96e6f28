"""The matrix-core block CRC (sdb_crc_mfma.h) against Python's zlib.crc32 and the slicing-by-8 wave CRC,
and the i8 MFMA lane maps it relies on (A[l&31][16(l>>5)+j], B[16(l>>5)+j][l&31], D[(i&3)+8(i>>2)+4(l>>5)][l&31])."""
import zlib

import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def dev():
    import torch
    from slatedb_amd import runtime
    runtime.require_device()
    return torch, runtime.lib()


def test_mfma_i8_lane_maps(dev):
    torch, L = dev
    rng = np.random.default_rng(5)
    A = rng.integers(-128, 128, (32, 32), dtype=np.int8)
    B = rng.integers(-128, 128, (32, 32), dtype=np.int8)
    a = np.zeros((64, 16), np.int8)
    b = np.zeros((64, 16), np.int8)
    for l in range(64):
        r, h = l & 31, l >> 5
        a[l] = A[r, 16 * h:16 * h + 16]
        b[l] = B[16 * h:16 * h + 16, r]
    ta = torch.from_numpy(a.view(np.int32).copy()).cuda()
    tb = torch.from_numpy(b.view(np.int32).copy()).cuda()
    td = torch.zeros(64 * 16, dtype=torch.int32, device="cuda")
    assert L.sdb_diag_mfma_i8(ta.data_ptr(), tb.data_ptr(), td.data_ptr(), None) == 0
    torch.cuda.synchronize()
    d = td.cpu().numpy().reshape(64, 16)
    ref = A.astype(np.int32) @ B.astype(np.int32)
    got = np.zeros((32, 32), np.int32)
    for l in range(64):
        for i in range(16):
            got[(i & 3) + 8 * (i >> 2) + 4 * (l >> 5), l & 31] = d[l, i]
    assert np.array_equal(got, ref)


@pytest.mark.parametrize("method", [0, 1])
def test_block_crc32(dev, method):
    torch, L = dev
    rng = np.random.default_rng(11 + method)
    lens = [4, 5, 7, 8, 15, 16, 17, 31, 32, 33, 63, 64, 65, 127, 128, 129, 1000, 2047, 2048, 2049, 4023, 4095, 4096]
    lens += [int(x) for x in rng.integers(4, 4097, 2000)]
    off = np.zeros(len(lens) + 1, np.uint64)
    off[1:] = np.cumsum(lens)
    data = rng.integers(0, 256, int(off[-1]) + 64, dtype=np.uint8)
    data[off[5]:off[6]] = 0xFF  # constant blocks too
    data[off[6]:off[7]] = 0
    td = torch.from_numpy(data).cuda()
    to = torch.from_numpy(off.view(np.int64)).cuda()
    out = torch.zeros(len(lens), dtype=torch.int32, device="cuda")
    assert L.sdb_diag_crc32_blocks(td.data_ptr(), to.data_ptr(), len(lens), out.data_ptr(), method, None) == 0
    torch.cuda.synchronize()
    got = out.cpu().numpy().view(np.uint32)
    ref = np.array([zlib.crc32(data[int(off[i]):int(off[i + 1])].tobytes()) for i in range(len(lens))], np.uint32)
    bad = np.nonzero(got != ref)[0]
    assert len(bad) == 0, [(lens[i], hex(got[i]), hex(ref[i])) for i in bad[:8]]
