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
    sizes = [int(x) for x in os.environ.get("SDB_BLOCK_SIZES", "1024,2048,4096,8192,16384,32768,65536").split(",")]
    for bs in sizes:
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
        # decode of SST 0 (sdb_decode_blocks over its data section)
        nb = int(got["summary"].num_blocks)
        dout = runtime.DeviceDecodeOutput(nb, hosts[0].n + 16, int(hosts[0].key_off[-1]) + 4096, device=dev)
        data = outs[0].data[:int(got["summary"].data_len)]
        boff = outs[0].block_off[:nb + 1]

        def dec():
            runtime.decode_blocks_at_device(data, boff[:nb], boff[1:], nb, dout, 2, stream=s)

        with torch.cuda.stream(s):
            dec()
        torch.cuda.synchronize()
        dh = dout.to_host()
        dok = dh.status == 0 and np.array_equal(dh.key_arena, hosts[0].key_bytes)
        d0, d1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        d0.record(s)
        with torch.cuda.stream(s):
            for _ in range(reps):
                dec()
        d1.record(s)
        torch.cuda.synchronize()
        dus = d0.elapsed_time(d1) / reps * 1000
        print(json.dumps({"block_size": bs, "us_per_sst": round(us, 1), "blocks": nb,
                          "GiB_per_s": round(hosts[0].logical_bytes() / (us * 1e-6) / 2**30, 1), "bit_exact": bool(ok),
                          "decode_us_per_sst": round(dus, 1), "decode_keys_ok": bool(dok)}), flush=True)
        del outs, ws


if __name__ == "__main__":
    main()
