"""Which deflate block types sdb_compress_blocks' zlib writes for D1 blocks (diagnostic): the first block's
BTYPE per stream, and the share of output in stored blocks (walking the stored blocks' headers only)."""
import collections
import os
import sys
import zlib

import numpy as np
import torch

sys.path.insert(0, os.path.join(os.path.dirname(__file__), ".."))
from oracle import oracle as O  # noqa: E402
from slatedb_amd import datasets, runtime  # noqa: E402

b = datasets.d1(n=60000, sst_index=1)
enc = O.encode_sst(b, O.params(block_size=4096, bloom_bits_per_key=0))
cz, off, err = runtime.compress_blocks_device(O.CODEC_ZLIB, torch.from_numpy(enc.data).cuda(),
                                              torch.from_numpy(enc.block_off.view(np.int64)).cuda())
torch.cuda.synchronize()
nb = len(enc.block_off) - 1
off = off.cpu().numpy().view(np.uint64)[: nb + 1]
cz = cz.cpu().numpy()
kinds = collections.Counter()
ratio = []
for k in range(nb):
    blk = cz[int(off[k]):int(off[k + 1]) - 4].tobytes()
    kinds[(blk[2] >> 1) & 3] += 1
    ratio.append(len(blk) / (int(enc.block_off[k + 1]) - int(enc.block_off[k])))
    assert zlib.decompress(blk) == enc.data[int(enc.block_off[k]):int(enc.block_off[k + 1]) - 4].tobytes()
print({"blocks": nb, "first_btype": dict(kinds), "mean_ratio": float(np.mean(ratio))})
