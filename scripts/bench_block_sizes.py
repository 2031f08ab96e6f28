"""Encode time of the configs[1] SST (D1) at every SstBlockSize (config.rs:231-267): 8 SSTs per launch
sequence, device-resident, HIP events.  Checks the first SST of each size against the oracle."""
import json
import os
import sys

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from slatedb_amd import datasets, runtime  # noqa: E402


def main():
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    hosts = [datasets.d1(sst_index=j) for j in range(8)]
    dbs = [h.to_device(dev) for h in hosts]
    s = torch.cuda.Stream(device=dev)
    for bs in (1024, 2048, 4096, 8192, 16384, 32768, 65536):
        prm = runtime.params(block_size=bs, sst_version=2, bloom_bits_per_key=10)
        outs = [runtime.DeviceSstOutput(h.n, h.logical_bytes(), h.logical_bytes(), prm, device=dev, workspace=False)
                for h in hosts]
        ws = runtime.ssts_workspace(dbs, prm, device=dev)
        with torch.cuda.stream(s):
            for _ in range(3):
                runtime.encode_ssts_device(dbs, outs, prm, ws, s)
        torch.cuda.synchronize()
        got = outs[0].to_host()
        ref = O.encode_sst(hosts[0], O.params(block_size=bs, sst_version=2, bloom_bits_per_key=10))
        ok = np.array_equal(got["data"], ref.data) and np.array_equal(got["bloom"], ref.bloom)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        reps = 10
        e0.record(s)
        with torch.cuda.stream(s):
            for _ in range(reps):
                runtime.encode_ssts_device(dbs, outs, prm, ws, s)
        e1.record(s)
        torch.cuda.synchronize()
        us = e0.elapsed_time(e1) / reps / 8 * 1000
        print(json.dumps({"block_size": bs, "us_per_sst": round(us, 1), "blocks": int(got["summary"].num_blocks),
                          "GiB_per_s": round(hosts[0].logical_bytes() / (us * 1e-6) / 2**30, 1), "bit_exact": bool(ok)}),
              flush=True)
        del outs, ws


if __name__ == "__main__":
    main()
