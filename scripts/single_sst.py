"""configs[1] literal shape: one 64 MiB D1 SST per sdb_encode_sst call, back to back on one stream
(the L0 flush rate).  For rocprofv3 --kernel-trace --stats (per-kernel durations of the single-SST sequence)."""
import os
import sys

import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from slatedb_amd import datasets, runtime  # noqa: E402

torch.cuda.set_device(0)
runtime.require_device()
dev = torch.device("cuda", 0)
prm = runtime.params(block_size=4096, sst_version=2, restart_interval=16, bloom_bits_per_key=10)
hosts = [datasets.d1(sst_index=j) for j in range(4)]
dbs = [h.to_device(dev) for h in hosts]
one = runtime.DeviceSstOutput(hosts[0].n, hosts[0].logical_bytes(), hosts[0].logical_bytes(), prm, device=dev)
st = torch.cuda.current_stream()
n = int(os.environ.get("SDB_SINGLE_STEPS", "100"))
for i in range(10):
    runtime.encode_sst_device(dbs[i % 4], one, st)
torch.cuda.synchronize()
e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
e0.record(st)
for i in range(n):
    runtime.encode_sst_device(dbs[i % 4], one, st)
e1.record(st)
torch.cuda.synchronize()
print("single SST: %.2f us per SST" % (1e3 * e0.elapsed_time(e1) / n), flush=True)
