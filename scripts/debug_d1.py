"""Diagnostic: first divergence between the GPU encoder and the oracle on full D1."""
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from oracle import oracle as O  # noqa: E402
from slatedb_amd import datasets, runtime as rt  # noqa: E402

b = datasets.d1(sst_index=int(os.environ.get("SST", "0")))
enc = rt.Encoder(rt.params(bloom_bits_per_key=0)).encode(b)
ref = O.encode_sst(b, O.params(block_size=4096, sst_version=2, bloom_bits_per_key=0))
print("status", enc.status, "blocks gpu/ref", len(enc.block_off) - 1, len(ref.block_off) - 1)
gf = np.asarray(enc.block_first_entry) if hasattr(enc, "block_first_entry") else None
print("attrs", [a for a in dir(enc) if not a.startswith("_")])
go = np.asarray(enc.block_off)
ro = np.asarray(ref.block_off)
m = min(len(go), len(ro))
d = np.nonzero(go[:m] != ro[:m])[0]
print("first block_off mismatch", d[:5])
if hasattr(ref, "block_first_entry"):
    rf = np.asarray(ref.block_first_entry)
    if gf is not None:
        dd = np.nonzero(gf[:m] != rf[:m])[0]
        print("first block_first mismatch", dd[:5])
        if len(dd):
            i = dd[0]
            print("gpu firsts", gf[max(0, i - 3):i + 4], "ref firsts", rf[max(0, i - 3):i + 4], "chunk", rf[i] // 2048)
