"""Diagnostic: fused-bloom encode vs the oracle on a small D1 batch; dumps the per-entry (h0, d0)
words k_seg wrote into the workspace and the first differing bitmap bytes."""
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from slatedb_amd import datasets, runtime  # noqa: E402

n = int(sys.argv[1]) if len(sys.argv) > 1 else 5000
b = datasets.d1(n=n)
prm = runtime.params(block_size=4096, sst_version=2, bloom_bits_per_key=10)
db = b.to_device("cuda:0")
out = runtime.DeviceSstOutput(b.n, b.logical_bytes(), b.logical_bytes(), prm)
runtime.encode_sst_device(db, out)
torch.cuda.synchronize()
got = out.to_host()
ref = O.encode_sst(b, O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10))
gb, rb = got["bloom"], ref.bloom
print("status", got["summary"].status, "bloom_len", got["summary"].bloom_len, len(rb))
diff = np.nonzero(gb != rb)[0]
print("differing bytes:", len(diff), "first:", diff[:10])
print("popcount got/ref:", int(np.unpackbits(gb).sum()), int(np.unpackbits(rb).sum()))
m = len(rb) * 8
for i in range(3):
    h = O.filter_hash(b.key(i))
    print("key", i, "hash %016x" % h, "h0", (h & 0xFFFFFFFF) % m, "d0", (h >> 32) % m, "probes", O.probes_for_key(h, 6, m))
ws = out.workspace.cpu().numpy()
# search the workspace for the (h0, d0) word of key 0
h = O.filter_hash(b.key(0))
w0 = np.uint64(((h & 0xFFFFFFFF) % m) | (((h >> 32) % m) << 32))
u64 = ws[: len(ws) // 8 * 8].view(np.uint64)
hit = np.nonzero(u64 == w0)[0]
print("hd word of key 0 found at u64 index", hit[:5])
import ctypes as C  # noqa: E402
cd = C.CDLL(runtime.LIB_PATH)
cd.sdb_diag_bloom_ws_offset.restype = C.c_uint64
cd.sdb_diag_bloom_ws_offset.argtypes = [C.c_uint64, C.c_void_p]
off = cd.sdb_diag_bloom_ws_offset(b.n, C.byref(prm))
off = (off + 255) // 256 * 256
cur = ws[off: off + 4 * 64].view(np.uint32)
print("cursors (first 24):", cur[:24])
