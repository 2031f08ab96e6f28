"""Diagnostic: per-phase s_memtime ticks of the compressor (k_cz) from a -DSDB_CZ_PT build
(SDB_LIBRARY=libslatedb_amd_czpt.so).  Phases: 0 stage, 1 matches, 2 parse, 3 elements (entropy coding),
4 CRC + slot; zlib inside 3: 5 histograms, 6 ll/d lengths, 7 run-length items, 8 cl lengths, 9 sizes + header,
10 body.  Prints mean ticks per block per phase for D1 and text_kv blocks."""
import ctypes as C
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
sys.path.insert(0, os.path.join(ROOT, "scripts"))
from slatedb_amd import datasets, runtime  # noqa: E402
from bench_configs import _encoded_blocks  # noqa: E402
from oracle import oracle as O  # noqa: E402

lib = C.CDLL(runtime.LIB_PATH)
lib.sdb_diag_cz_phase.argtypes = [C.c_void_p, C.c_int]
dev = torch.device("cuda", 0)
for name, batches in (("d1", [datasets.d1(sst_index=j) for j in range(2)]), ("text", [datasets.text_kv(n=100_000)])):
    data, off = _encoded_blocks(batches, dev)
    nb = len(off) - 1
    dd = torch.from_numpy(np.concatenate([data, np.zeros(64, np.uint8)])).to(dev)
    db = torch.from_numpy(off.view(np.int64)).to(dev)
    for codec, cn in ((O.CODEC_LZ4, "lz4"), (O.CODEC_ZLIB, "zlib"), (O.CODEC_ZSTD, "zstd")):
        runtime.compress_blocks_device(codec, dd, db)
        torch.cuda.synchronize()
        buf = (C.c_uint64 * 16)()
        assert lib.sdb_diag_cz_phase(buf, 1) == 0
        runtime.compress_blocks_device(codec, dd, db)
        torch.cuda.synchronize()
        assert lib.sdb_diag_cz_phase(buf, 0) == 0
        v = np.array(list(buf), np.float64) / nb
        print("%-5s %-6s blocks %d ticks/block: " % (name, cn, nb) + " ".join("%d:%.0f" % (i, x) for i, x in enumerate(v) if x),
              flush=True)
