"""Diagnostic: HBM bandwidth probes (sdb_diag_bw) on a 2 GiB buffer pair -> one JSON line per (mode, grid).
Bytes counted: copy = read + write, read only = read, write only = write."""
import json
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slatedb_amd import runtime  # noqa: E402

L = runtime.lib()
n = 1 << 31
a = torch.empty(n, dtype=torch.uint8, device="cuda").fill_(1)
b = torch.empty_like(a)
st = torch.cuda.current_stream().cuda_stream
names = {0: "copy nt (sdb_diag_copy)", 1: "copy plain", 2: "copy 4 KiB per wave", 3: "read only", 4: "write only"}
for mode in range(5):
    for wpc in (4, 8, 16, 32):
        assert L.sdb_diag_bw(b.data_ptr(), a.data_ptr(), n, mode, wpc, st) == 0
        torch.cuda.synchronize()
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record()
        for _ in range(reps):
            L.sdb_diag_bw(b.data_ptr(), a.data_ptr(), n, mode, wpc, st)
        e1.record()
        torch.cuda.synchronize()
        ms = e0.elapsed_time(e1) / reps
        moved = 2 * n if mode <= 2 else n
        print(json.dumps({"mode": names[mode], "wg_per_cu": wpc, "ms": round(ms, 4), "GBps": round(moved / ms / 1e6, 1)}), flush=True)
