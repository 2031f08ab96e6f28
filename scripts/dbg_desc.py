import sys, os
sys.path.insert(0, os.getcwd())
import numpy as np
from tests.test_descending import device_desc, dup_batch
from slatedb_amd import datasets, runtime as rt
from oracle import oracle as O
for name, b, bs in (("d3-800", datasets.d3(n=800), 256), ("dup-bs64", dup_batch(), 64), ("dup-bs4096", dup_batch(), 4096), ("dup-1500", dup_batch(n=1500), 256)):
    for desc in (False,):
        e = O.encode_sst(b, O.params(sst_version=2, block_size=bs))
        ref = O.decode_blocks(e.data, e.block_off, 2, descending=desc)
        if desc:
            got = device_desc(rt, e.data, e.block_off, 2)
        else:
            import torch
            nb = len(e.block_off) - 1; total = int(e.block_off[-1])
            dout = rt.DeviceDecodeOutput(nb, total // 8 + 64, total * 8 + 4096)
            arena = torch.from_numpy(np.concatenate([np.asarray(e.data, np.uint8), np.zeros(64, np.uint8)])).cuda()
            boff = torch.from_numpy(np.asarray(e.block_off, np.uint64).view(np.int64)).cuda()
            rt.decode_blocks_ex_device(arena, boff, None, nb, dout, 2, descending=False)
            torch.cuda.synchronize(); got = dout.to_host()
        bad = {}
        for f in ("key_off", "val_off", "val_len", "seq", "flags"):
            a_, b_ = getattr(ref, f), getattr(got, f)
            if not np.array_equal(a_, b_):
                idx = np.nonzero(a_ != b_)[0] if len(a_) == len(b_) else [-1]
                bad[f] = (len(idx), int(idx[0]), int(idx[-1]))
        print(name, "desc" if desc else "asc", "nblocks", len(e.block_off) - 1, "n", ref.n, got.n, "status", ref.status, got.status, "bad", bad, flush=True)
        if bad and "key_off" in bad:
            i = bad["key_off"][1]
            print("  ref key_off[i-2:i+3]", ref.key_off[max(0,i-2):i+3], "got", got.key_off[max(0,i-2):i+3])
            bes = ref.block_entry_start
            blk = int(np.searchsorted(bes, i, side="right") - 1)
            print("  entry", i, "block", blk, "bes ref", ref.block_entry_start[blk:blk+3], "got", got.block_entry_start[blk:blk+3])
