"""Diagnostic: per-phase k_seg timings from a -DSDB_PHASE_TIMING build (SDB_LIBRARY=libslatedb_amd_pt.so)."""
import ctypes as C
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from slatedb_amd import datasets, runtime  # noqa: E402

lib = runtime.lib()
dev = torch.device("cuda", 0)
prm = runtime.params(block_size=4096, sst_version=2, restart_interval=16, bloom_bits_per_key=int(os.environ.get('BPK', '10')))
h = datasets.d1(sst_index=1)
db = h.to_device(dev)
out = runtime.DeviceSstOutput(h.n, h.logical_bytes(), h.logical_bytes(), prm, device=dev)
s = torch.cuda.Stream()
for _ in range(5):
    runtime.encode_sst_device(db, out, s)
torch.cuda.synchronize()
nb = (h.n + 2047) // 2048
buf = (C.c_uint64 * (8 * 1024))()
f = lib._lib.sdb_diag_phase_times if hasattr(lib, "_lib") else None
cdll = C.CDLL(runtime.LIB_PATH)
cdll.sdb_diag_phase_times.argtypes = [C.c_void_p, C.c_int]
assert cdll.sdb_diag_phase_times(C.addressof(buf), 1024) == 0
t = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8)[:nb].astype(np.int64)
marks = 7
d = np.diff(t[:, :marks], axis=1)
print("phase durations (s_memtime ticks) mean/max over %d workgroups:" % nb)
for i in range(marks - 1):
    print("  %d->%d  mean %8.0f  max %8.0f" % (i, i + 1, d[:, i].mean(), d[:, i].max()))
tot = t[:, marks - 1] - t[:, 0]
r = np.frombuffer(buf, dtype=np.uint64).reshape(1024, 8)[1023].astype(np.int64)
print("resolve phases:", list(np.diff(r[:6])), "total", r[5] - r[0])
print("  total   mean %8.0f  max %8.0f ; spread of starts %d, of ends %d" % (tot.mean(), tot.max(), t[:, 0].max() - t[:, 0].min(), t[:, marks - 1].max() - t[:, marks - 1].min()))

wb = (C.c_uint64 * (8 * 8192))()
cdll.sdb_diag_wave_phase.argtypes = [C.c_void_p, C.c_int]
assert cdll.sdb_diag_wave_phase(C.addressof(wb), 8192) == 0
w = np.frombuffer(wb, dtype=np.uint64).reshape(8192, 8).astype(np.int64)
w = w[w[:, 6] > 0]
print("emit waves %d, blocks/wave %.2f; mean ticks per block per phase:" % (len(w), w[:, 6].mean()))
names = ["desc+meta+sizes", "rows(hdr/keys)", "wait stage", "value copy", "crc", "store"]
per = w[:, :6].sum(axis=0) / w[:, 6].sum()
for n, v in zip(names, per):
    print("  %-16s %8.0f" % (n, v))
print("  total            %8.0f  (per-wave total mean %.0f)" % (per.sum(), w[:, :6].sum(axis=1).mean()))

rb = (C.c_uint64 * (4 * 8192))()
cdll.sdb_diag_wave_rt.argtypes = [C.c_void_p, C.c_int]
assert cdll.sdb_diag_wave_rt(C.addressof(rb), 8192) == 0
r = np.frombuffer(rb, dtype=np.uint64).reshape(8192, 4).astype(np.int64)
r = r[r[:, 1] > 0][:len(w)]
st, en = (r[:, 0] - r[:, 0].min()) / 100.0, (r[:, 1] - r[:, 0].min()) / 100.0  # 100 MHz -> us
clk = (r[:, 3] - r[:, 2]) / np.maximum(r[:, 1] - r[:, 0], 1) * 100.0
print("k_emit waves (us from first start): start p50 %.1f p90 %.1f max %.1f; end p10 %.1f p50 %.1f max %.1f; "
      "wave duration p50 %.1f; shader clock %.0f MHz (median)" % (np.percentile(st, 50), np.percentile(st, 90), st.max(),
      np.percentile(en, 10), np.percentile(en, 50), en.max(), np.median(en - st), np.median(clk)))

eb = (C.c_uint64 * (8 * 1024))()
cdll.sdb_diag_enum_phase.argtypes = [C.c_void_p, C.c_int]
assert cdll.sdb_diag_enum_phase(C.addressof(eb), 1024) == 0
t = np.frombuffer(eb, dtype=np.uint64).reshape(1024, 8)[:nb].astype(np.int64)
d = np.diff(t[:, :6], axis=1)
print("k_enum phases (ticks) mean/max: " + "  ".join("%d->%d %.0f/%.0f" % (i, i + 1, d[:, i].mean(), d[:, i].max()) for i in range(5)))

# per-workgroup end time of k_emit (max over its waves), grouped by workgroup % 8 (XCD round-robin)
wpb = 16
nwg = len(r) // wpb
wend = en[: nwg * wpb].reshape(nwg, wpb).max(axis=1)
print("k_emit workgroup end (us) by wg%%8: " + "  ".join("%d:%.1f/%.1f" % (x, np.median(wend[x::8]), wend[x::8].max()) for x in range(8)))
print("k_emit workgroup end (us) percentiles p0 %.1f p10 %.1f p50 %.1f p90 %.1f p100 %.1f" % tuple(np.percentile(wend, [0, 10, 50, 90, 100])))
slow = np.argsort(wend)[-8:]
print("slowest workgroups:", list(slow), [round(float(wend[i]), 1) for i in slow])
