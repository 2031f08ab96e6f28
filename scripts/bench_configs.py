"""Secondary measurements for BASELINE.json configs[2..3] and the host-memory (E2E) encode path.

  python scripts/bench_configs.py [--decode] [--bloom] [--e2e] [--reps R]

Prints one JSON line per measurement.  Not the headline bench (bench.py is); these numbers feed
DESIGN.md:
  decode  configs[2]: 16 D1 SSTs (suffix 0..15) encoded on the GPU, their 272,256 blocks decoded in
          one sdb_decode_blocks launch sequence (device-resident in and out); also 2 MiB ranges.
          Algorithmic bytes = encoded bytes read + Σ(|k| + 8 + 1 + 8·ts) + value refs are not
          counted.
  bloom   configs[3]: 10 M sorted random 16 B keys, 10 bits/key; bitmap bit-exact vs the oracle.
  e2e     configs[1] from pinned host memory: sdb_encoder_encode_host (H2D + kernels + D2H).
  hbm     the box's measured HBM copy / read bandwidth (torch copy_ and a sum over 4 GiB), beside the
          8.0 TB/s spec that every roofline fraction uses (BASELINE.md reporting rules).
CPU baselines (oracle/sdb_oracle.c, a restatement — not the Rust binary) are timed beside decode and
bloom on 1 thread and on the process's CPU share (one SST / one key range per thread).
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np
import torch

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from slatedb_amd import _abi, datasets, runtime  # noqa: E402

PEAK = 8000.0


def cpu_share():
    if os.environ.get("OMP_NUM_THREADS", "").isdigit():
        return max(1, int(os.environ["OMP_NUM_THREADS"]))
    try:
        return len(os.sched_getaffinity(0))
    except AttributeError:
        return os.cpu_count() or 1


def cpu_model():
    try:
        return [l.split(":", 1)[1].strip() for l in open("/proc/cpuinfo") if l.startswith("model name")][0]
    except Exception:
        return "unknown"


def threaded(fn, items, deadline_s):
    """Run fn(item) repeatedly on one thread per item until the deadline; returns (calls, wall s)."""
    import threading
    counts = [0] * len(items)
    t0 = time.perf_counter()

    def run(i):
        while True:
            fn(items[i])
            counts[i] += 1
            if time.perf_counter() - t0 >= deadline_s:
                break

    ths = [threading.Thread(target=run, args=(i,)) for i in range(len(items))]
    for t in ths:
        t.start()
    for t in ths:
        t.join()
    return sum(counts), time.perf_counter() - t0


def timed(fn, reps, stream):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record(stream)
    for _ in range(reps):
        fn()
    e1.record(stream)
    torch.cuda.synchronize()
    return e0.elapsed_time(e1) / reps


def decode_bench(reps, granular=True, cpu_s=0.0):
    lib = runtime.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    prm = runtime.params(block_size=4096, sst_version=2, bloom_bits_per_key=0)
    chunks, offs, keys, nent = [], [], [], 0
    base = 0
    for j in range(16):
        h = datasets.d1(sst_index=j)
        db = h.to_device(dev)
        out = runtime.DeviceSstOutput(h.n, h.logical_bytes(), h.logical_bytes(), prm, device=dev)
        runtime.encode_sst_device(db, out)
        torch.cuda.synchronize()
        sm = out.summary_host()
        assert sm.status == 0
        chunks.append(out.data[:sm.data_len].clone())
        bo = out.block_off[:sm.num_blocks + 1].clone()
        offs.append(bo[:-1] + base if j < 15 else bo + base)
        base += sm.data_len
        keys.append(h.key_bytes)
        nent += h.n
        del db, out
    blocks = torch.cat(chunks)
    block_off = torch.cat(offs)
    nb = block_off.numel() - 1
    kbytes = int(sum(k.size for k in keys))
    o = lambda n, dt: torch.empty(n, dtype=dt, device=dev)
    bes, ka, ko = o(nb + 1, torch.int64), o(kbytes + 16, torch.uint8), o(nent + 1, torch.int64)
    vo, vl, sq = o(nent, torch.int64), o(nent, torch.int32), o(nent, torch.int64)
    fl, ct, et = o(nent, torch.uint8), o(nent, torch.int64), o(nent, torch.int64)
    bad, smy = o(nb + 1, torch.int32), torch.zeros(64, dtype=torch.uint8, device=dev)
    dout = _abi.DecodedOut(bes.data_ptr(), ka.data_ptr(), kbytes + 16, ko.data_ptr(), vo.data_ptr(),
                           vl.data_ptr(), sq.data_ptr(), fl.data_ptr(), ct.data_ptr(), et.data_ptr(), nent,
                           bad.data_ptr(), nb + 1, smy.data_ptr())
    wsb = lib.sdb_decode_workspace_bytes(nb)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

    def run(b0=0, b1=nb):
        st = lib.sdb_decode_blocks(blocks.data_ptr(), block_off[b0:].data_ptr(), b1 - b0, 2, C.byref(dout),
                                   ws.data_ptr(), wsb, s.cuda_stream)
        assert st == 0, st

    with torch.cuda.stream(s):
        ms = timed(run, reps, s)
    torch.cuda.synchronize()
    if os.environ.get("SDB_DEC_PHASE"):  # phase ticks of one full decode (timing build only)
        cd = C.CDLL(runtime.LIB_PATH)
        cd.sdb_diag_dec_phase.argtypes = [C.c_void_p]
        b0 = np.zeros((2, 8192, 4), np.uint64)
        b1 = np.zeros((2, 8192, 4), np.uint64)
        cd.sdb_diag_dec_phase(b0.ctypes.data)
        with torch.cuda.stream(s):
            run()
        torch.cuda.synchronize()
        cd.sdb_diag_dec_phase(b1.ctypes.data)
        d = (b1 - b0).astype(np.int64)
        for pas, name, labels in ((0, "count", ["stage+crc", "tally", "-"]), (1, "emit", ["stage", "walk+cols", "keystore"])):
            nbk = max(int(d[pas, :, 3].sum()), 1)
            per = d[pas, :, :3].sum(axis=0) / nbk
            print("%s: %d blocks; ticks per block: %s" % (name, nbk, "  ".join("%s %.0f" % (l, v) for l, v in zip(labels, per))), flush=True)
    sm = _abi.DecodeSummary.from_buffer_copy(smy.cpu().numpy().tobytes()[:C.sizeof(_abi.DecodeSummary)])
    ok = sm.status == 0 and sm.num_entries == nent and sm.num_bad_blocks == 0
    ok = ok and np.array_equal(ka[:kbytes].cpu().numpy(), np.concatenate(keys))
    enc = int(blocks.numel())
    alg = enc + nent * (16 + 8 + 1 + 8)  # encoded bytes + Σ(|k| + 8 + 1 + 8·ts) (val refs 8)
    gbs = alg / (ms * 1e-3) / 1e9
    print(json.dumps({"what": "decode configs[2]", "blocks": nb, "entries": nent, "encoded_bytes": enc,
                      "ms": round(ms, 4), "GiB_per_s_encoded": round(enc / (ms * 1e-3) / 2**30, 2),
                      "algorithmic_bytes": alg, "achieved_GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4),
                      "verified_keys": bool(ok)}), flush=True)
    # read_blocks semantics (SDB_DECODE_FAIL_FAST): the checksums verified by the emit pass
    def run_ff():
        st = lib.sdb_decode_blocks_ex(blocks.data_ptr(), block_off.data_ptr(), None, nb, 2, _abi.DECODE_FAIL_FAST,
                                      C.byref(dout), ws.data_ptr(), wsb, s.cuda_stream)
        assert st == 0, st

    with torch.cuda.stream(s):
        ms_ff = timed(run_ff, reps, s)
    torch.cuda.synchronize()
    sm_ff = _abi.DecodeSummary.from_buffer_copy(smy.cpu().numpy().tobytes()[:C.sizeof(_abi.DecodeSummary)])
    ok_ff = sm_ff.status == 0 and sm_ff.num_entries == nent and np.array_equal(ka[:kbytes].cpu().numpy(), np.concatenate(keys))
    gbs_ff = alg / (ms_ff * 1e-3) / 1e9
    print(json.dumps({"what": "decode configs[2], fail-fast (read_blocks semantics: checksums in the emit pass)",
                      "ms": round(ms_ff, 4), "GiB_per_s_encoded": round(enc / (ms_ff * 1e-3) / 2**30, 2),
                      "achieved_GBps": round(gbs_ff, 1), "frac": round(gbs_ff / PEAK, 4), "verified_keys": bool(ok_ff)}),
          flush=True)
    # descending iteration order (SDB_DECODE_DESCENDING): written mirrored by the emit pass
    asc_keys = ka[:kbytes].cpu().numpy().copy()
    asc_seq = sq[:nent].cpu().numpy().copy()

    def run_desc():
        st = lib.sdb_decode_blocks_ex(blocks.data_ptr(), block_off.data_ptr(), None, nb, 2, _abi.DECODE_DESCENDING,
                                      C.byref(dout), ws.data_ptr(), wsb, s.cuda_stream)
        assert st == 0, st

    with torch.cuda.stream(s):
        ms_d = timed(run_desc, reps, s)
    torch.cuda.synchronize()
    smd = _abi.DecodeSummary.from_buffer_copy(smy.cpu().numpy().tobytes()[:C.sizeof(_abi.DecodeSummary)])
    okd = smd.status == 0 and smd.num_entries == nent and np.array_equal(
        ka[:kbytes].cpu().numpy().reshape(-1, 16), asc_keys.reshape(-1, 16)[::-1]) and np.array_equal(
        sq[:nent].cpu().numpy(), asc_seq[::-1])
    print(json.dumps({"what": "decode configs[2], descending order", "ms": round(ms_d, 4),
                      "GiB_per_s_encoded": round(enc / (ms_d * 1e-3) / 2**30, 2),
                      "verified_keys_seq_reversed": bool(okd)}), flush=True)
    if cpu_s > 0:  # CPU baseline: the oracle decoding whole D1 SSTs (read_blocks -> DataBlockIterator)
        from oracle import oracle as O
        host = []
        for j in range(16):
            lo = int(offs[j][0])
            hi = int(offs[j][-1]) if j == 15 else int(offs[j + 1][0])
            bo = np.append(offs[j].cpu().numpy(), hi) if j < 15 else offs[j].cpu().numpy()
            host.append((blocks[lo:hi].cpu().numpy(), (bo - lo).astype(np.uint64)))
        enc_sst = host[0][0].size
        dec = lambda hb: O.decode_blocks(hb[0], hb[1], 2, cap_entries=600000, key_cap=10 << 20)
        r = dec(host[0])
        assert r.status == 0 and r.n == nent // 16
        n1, w1 = threaded(dec, host[:1], cpu_s / 4)
        th = cpu_share()
        nt, wt = threaded(dec, [host[i % 16] for i in range(th)], cpu_s * 3 / 4)
        print(json.dumps({"what": "decode configs[2] CPU baseline (oracle, port)", "kind": "port",
                          "single_thread_GiB_per_s_encoded": round(n1 * enc_sst / w1 / 2**30, 3),
                          "threads": th, "GiB_per_s_encoded": round(nt * enc_sst / wt / 2**30, 3),
                          "configs2_ms_at_threads": round(16 * wt / nt * 1e3, 1),
                          "sample": "%d D1 SSTs on 1 thread (%.1f s), then %d threads x 1 SST for %.1f s (%d SSTs)"
                                    % (n1, w1, th, wt, nt), "cpu": cpu_model(), "nproc": os.cpu_count()}),
              flush=True)
    if not granular:
        return
    # 2 MiB ranged-GET granularity (≈ 520 blocks per call), launched back to back
    per = 520
    ranges = [(b, min(nb, b + per)) for b in range(0, nb, per)]

    # arguments prepared outside the timed region (a Rust caller pays no per-call interpreter cost)
    fn, bp, dref, wsp, cs = lib.sdb_decode_blocks, blocks.data_ptr(), C.byref(dout), ws.data_ptr(), s.cuda_stream
    args = [(block_off[b0:].data_ptr(), b1 - b0) for b0, b1 in ranges]

    def run_ranges():
        for op, n in args:
            if fn(bp, op, n, 2, dref, wsp, wsb, cs):
                raise RuntimeError("sdb_decode_blocks failed")

    with torch.cuda.stream(s):
        ms2 = timed(run_ranges, max(1, reps // 4), s)
    print(json.dumps({"what": "decode configs[2] at 2 MiB granularity, one sdb_decode_blocks call per range",
                      "calls": len(ranges), "ms": round(ms2, 4),
                      "GiB_per_s_encoded": round(enc / (ms2 * 1e-3) / 2**30, 2)}), flush=True)
    # the same 2 MiB ranges uploaded into one arena (each GET at a 4 KiB-aligned slot, gaps between
    # them) and decoded by ONE sdb_decode_blocks_at call
    bo = block_off.cpu().numpy().view(np.uint64)
    starts, ends, pieces, pos = [], [], [], 0
    for b0, b1 in ranges:
        lo, hi = int(bo[b0]), int(bo[b1])
        pos = (pos + 4095) & ~4095
        starts.append(bo[b0:b1] - np.uint64(lo) + np.uint64(pos))
        ends.append(bo[b0 + 1:b1 + 1] - np.uint64(lo) + np.uint64(pos))
        pieces.append((pos, lo, hi))
        pos += hi - lo
    arena = torch.zeros(pos + 16, dtype=torch.uint8, device=dev)
    for p0, lo, hi in pieces:
        arena[p0:p0 + hi - lo].copy_(blocks[lo:hi])
    ds = torch.from_numpy(np.concatenate(starts).view(np.int64)).to(dev)
    de = torch.from_numpy(np.concatenate(ends).view(np.int64)).to(dev)
    fn_at = lib.sdb_decode_blocks_at

    def run_at():
        if fn_at(arena.data_ptr(), ds.data_ptr(), de.data_ptr(), nb, 2, dref, wsp, wsb, cs):
            raise RuntimeError("sdb_decode_blocks_at failed")

    with torch.cuda.stream(s):
        ms3 = timed(run_at, reps, s)
    sm = _abi.DecodeSummary.from_buffer_copy(smy.cpu().numpy().tobytes()[:C.sizeof(_abi.DecodeSummary)])
    ok3 = sm.status == 0 and sm.num_entries == nent and np.array_equal(ka[:kbytes].cpu().numpy(), np.concatenate(keys))
    print(json.dumps({"what": "decode configs[2] as %d 2 MiB ranges in one arena, one sdb_decode_blocks_at call" % len(ranges),
                      "ms": round(ms3, 4), "GiB_per_s_encoded": round(enc / (ms3 * 1e-3) / 2**30, 2),
                      "verified_keys": bool(ok3)}), flush=True)


def bloom_bench(reps):
    from oracle import oracle as O
    lib = runtime.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    kb, ko = datasets.c4_keys()
    n = len(ko) - 1
    dk = torch.from_numpy(kb).to(dev)
    do = torch.from_numpy(ko.view(np.uint8)).to(dev)
    fb = lib.sdb_bloom_filter_bytes(n, 10)
    bm = torch.empty(fb + 16, dtype=torch.uint8, device=dev)
    wsb = lib.sdb_bloom_workspace_bytes(n, 10)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)

    def run():
        st = lib.sdb_bloom_build(dk.data_ptr(), do.data_ptr(), n, 10, bm.data_ptr(), fb, ws.data_ptr(), wsb,
                                 s.cuda_stream)
        assert st == 0

    def run_atomic():  # no workspace: k_bloom_atomic, device-scope atomicOr per probe (comparison only)
        st = lib.sdb_bloom_build(dk.data_ptr(), do.data_ptr(), n, 10, bm.data_ptr(), fb, 0, 0, s.cuda_stream)
        assert st == 0

    with torch.cuda.stream(s):
        ms_at = timed(run_atomic, reps, s)
        got_at = bm[:fb].cpu().numpy()
        ms = timed(run, reps, s)
    got = bm[:fb].cpu().numpy()
    print(json.dumps({"what": "bloom configs[3], device-atomic path (no workspace)", "ms": round(ms_at, 4),
                      "same_bitmap_as_dense": bool(np.array_equal(got_at, got))}), flush=True)
    t0 = time.perf_counter()
    ref = O.bloom_build(kb, ko, 10)
    cpu_s = time.perf_counter() - t0
    ok = np.array_equal(got, np.frombuffer(bytes(ref), np.uint8) if not isinstance(ref, np.ndarray) else ref)
    th = cpu_share()
    t0 = time.perf_counter()
    ref_t = O.bloom_build_threads(kb, ko, 10, th)
    cpu_t = time.perf_counter() - t0
    ok = ok and np.array_equal(ref_t, ref)
    alg = n * 16 + fb
    gbs = alg / (ms * 1e-3) / 1e9
    print(json.dumps({"what": "bloom configs[3]", "keys": n, "bitmap_bytes": fb, "ms": round(ms, 4),
                      "Mkeys_per_s": round(n / (ms * 1e-3) / 1e6, 1), "algorithmic_bytes": alg,
                      "achieved_GBps": round(gbs, 1), "frac": round(gbs / PEAK, 4), "bit_exact": bool(ok),
                      "cpu_baseline": {"kind": "port", "single_thread_s": round(cpu_s, 3),
                                       "single_thread_Mkeys_per_s": round(n / cpu_s / 1e6, 2), "threads": th,
                                       "threads_s": round(cpu_t, 3), "threads_Mkeys_per_s": round(n / cpu_t / 1e6, 2),
                                       "sample": "the whole 10 M-key build, 1 thread then key ranges over %d "
                                                 "threads OR-merged" % th, "cpu": cpu_model(),
                                       "nproc": os.cpu_count()}}), flush=True)


def e2e_bench(reps):
    """Host -> host (the boundary a Rust caller uses): pageable batches in, host SST bytes out."""
    hs = [datasets.d1(sst_index=j) for j in range(8)]
    h = hs[0]
    enc = runtime.Encoder(runtime.params(block_size=4096, sst_version=2, bloom_bits_per_key=10))
    for _ in range(2):
        enc.encode(h)
    ev, walls = [], []
    for _ in range(reps):
        t0 = time.perf_counter()
        st, res = enc.encode(h, copy=False)
        walls.append((time.perf_counter() - t0) * 1e3)
        assert st == 0
        ev.append({"h2d": res.h2d_ms, "kernel": res.kernel_ms, "d2h": res.d2h_ms})
    r = enc.encode(h)
    med = {k: round(float(np.median([e[k] for e in ev])), 4) for k in ev[0]}
    wall = float(np.median(walls))
    print(json.dumps({"what": "e2e configs[1] host->host, one SST per call (marshal into pinned staging, H2D, kernels, D2H)",
                      "ms_wall": round(wall, 3), "GiB_per_s_logical": round(h.logical_bytes() / (wall * 1e-3) / 2**30, 2),
                      "events_ms_median": med, "marshal_ms": round(wall - sum(med.values()), 3),
                      "num_blocks": r.num_blocks}), flush=True)
    # the pipelined path: 8 SSTs per call, transfers overlapped (sdb_encoder_encode_host_many)
    single = [enc.encode(x) for x in hs[:2]]
    got = enc.encode_many(hs)
    ok = all(g.status == 0 for g in got) and all(
        np.array_equal(got[q].data, single[q].data) and np.array_equal(got[q].bloom, single[q].bloom) for q in range(2))
    walls = []
    for _ in range(max(2, reps // 4)):
        t0 = time.perf_counter()
        st, _ = enc.encode_many(hs, copy=False)
        walls.append((time.perf_counter() - t0) * 1e3)
        assert st == 0
    wall = float(np.median(walls))
    print(json.dumps({"what": "e2e configs[1] host->host, 8 SSTs per sdb_encoder_encode_host_many call (overlapped)",
                      "ms_wall_per_call": round(wall, 3), "ms_per_sst": round(wall / len(hs), 3),
                      "GiB_per_s_logical": round(len(hs) * h.logical_bytes() / (wall * 1e-3) / 2**30, 2),
                      "matches_single_path": bool(ok)}), flush=True)
    enc.close()


def compact_bench(reps):
    """f2: a compaction job on the device -- 4 L0 SSTs of the configs[1] shape (D1, 578,524 x 16 B key /
    100 B value each, key ranges interleaved) merged, retention applied, cut at max_sst_size = 256 MiB
    (config.rs:1383) and encoded (4 KiB blocks, 10 bits/key bloom); runs resident in HBM."""
    from slatedb_amd.batch import Run
    hosts = [datasets.d1(sst_index=j) for j in range(4)]
    druns = [runtime.DeviceRun.from_host(Run.from_batch(h)) for h in hosts]
    prm = runtime.params(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    ret = _abi.Retention(0, 0, 0, 1, 0, 0, 0, 0)  # retention_min_seq Some(0), compaction_clock_tick 0
    comp = runtime.Compactor()
    logical = sum(h.logical_bytes() for h in hosts)
    st, ns = comp.run(druns, ret, prm, 256 << 20)
    assert st == 0, st
    torch.cuda.synchronize()
    walls = []
    for _ in range(reps):
        t0 = time.perf_counter()
        st, ns = comp.run(druns, ret, prm, 256 << 20)
        walls.append((time.perf_counter() - t0) * 1e3)
        assert st == 0
    ms = float(np.median(walls))
    # CPU baseline: the oracle's merge + retention + cuts + encode of the same job, one thread
    from oracle import oracle as O
    runs = [Run.from_batch(hh) for hh in hosts]
    oret = O.retention(min_seq=0)
    t0 = time.perf_counter()
    _, osm, ocuts, ossts = O.compact(runs, oret, O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10),
                                     256 << 20)
    cpu_s = time.perf_counter() - t0
    merged, msum = comp.merged()
    same = len(ossts) == ns and all(np.array_equal(comp.sst(i)["data"], ossts[i].data) for i in range(ns))
    print(json.dumps({"what": "compaction job (f2): 4 x configs[1] L0 SSTs -> merge + retention + cuts + encode",
                      "entries_in": int(msum.num_in), "entries_out": int(msum.num_out), "output_ssts": ns,
                      "logical_bytes_in": logical, "ms_wall": round(ms, 3),
                      "GiB_per_s_logical": round(logical / (ms * 1e-3) / 2**30, 2), "bit_exact_vs_oracle": bool(same),
                      "cpu_baseline": {"kind": "port", "cores": 1, "s": round(cpu_s, 3),
                                       "GiB_per_s_logical": round(logical / cpu_s / 2**30, 3),
                                       "sample": "the whole job, oracle compact (merge + retention + cuts + encode)"}}),
          flush=True)
    # the same job from the encoded input SSTs (sdb_compactor_run_ssts: decode inside the job), the four
    # SSTs encoded on the device and resident; CPU baseline: the oracle's decode of the four SSTs + compact
    import types
    dev = torch.device("cuda", 0)
    inputs, enc_host = [], []
    for h in hosts:
        db = h.to_device(dev)
        out = runtime.DeviceSstOutput(h.n, h.logical_bytes(), h.logical_bytes(), prm, device=dev)
        runtime.encode_sst_device(db, out)
        torch.cuda.synchronize()
        sm = out.summary_host()
        nb = int(sm.num_blocks)
        inputs.append(types.SimpleNamespace(data=out.data, block_off=out.block_off[:nb + 1],
                                            num_entries=int(sm.num_entries), key_bytes=int(sm.raw_key_size),
                                            val_bytes=int(sm.raw_val_size), keep=out))
        r = out.to_host()
        enc_host.append((r["data"], r["block_off"].astype(np.uint64)))
        del db
    encoded = sum(int(x.block_off[-1].item()) for x in inputs)
    comp2 = runtime.Compactor()
    st2, ns2 = comp2.run_ssts(inputs, ret, prm, 256 << 20)
    assert st2 == 0, st2
    torch.cuda.synchronize()
    walls2 = []
    for _ in range(reps):
        t0 = time.perf_counter()
        st2, ns2 = comp2.run_ssts(inputs, ret, prm, 256 << 20)
        walls2.append((time.perf_counter() - t0) * 1e3)
        assert st2 == 0
    ms2 = float(np.median(walls2))
    t0 = time.perf_counter()
    druns_o = []
    for data, bo in enc_host:
        d = O.decode_blocks(data, bo, 2)
        druns_o.append(Run(d.key_arena, d.key_off, data, d.val_off, d.val_len, d.seq, d.flags, d.create_ts, d.expire_ts))
    _, osm2, ocuts2, ossts2 = O.compact(druns_o, oret, O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10),
                                        256 << 20)
    cpu2_s = time.perf_counter() - t0
    same2 = len(ossts2) == ns2 and all(np.array_equal(comp2.sst(i)["data"], ossts2[i].data) for i in range(ns2))
    print(json.dumps({"what": "compaction job (f2) from encoded SSTs: 4 x configs[1] L0 SSTs -> decode + merge + "
                              "retention + cuts + encode (sdb_compactor_run_ssts, two host synchronisations)",
                      "encoded_bytes_in": encoded, "logical_bytes_in": logical, "output_ssts": ns2, "ms_wall": round(ms2, 3),
                      "GiB_per_s_logical": round(logical / (ms2 * 1e-3) / 2**30, 2), "bit_exact_vs_oracle": bool(same2),
                      "cpu_baseline": {"kind": "port", "cores": 1, "s": round(cpu2_s, 3),
                                       "GiB_per_s_logical": round(logical / cpu2_s / 2**30, 3),
                                       "sample": "the whole job, oracle decode of the 4 SSTs + compact"}}), flush=True)
    comp2.close()
    comp.close()
    # a job whose retention drops: four L0 runs over one key space (each key in ~3 runs), tombstones in the
    # newest, no snapshot, the destination is the last run (filter_tombstone)
    ohosts = datasets.overwrite_runs(nruns=4)
    oruns = [Run.from_batch(h) for h in ohosts]
    odruns = [runtime.DeviceRun.from_host(r) for r in oruns]
    oret_d = _abi.Retention(0, 0, 0, 0, 0, 1, 0, 0)  # retention_min_seq None, no time window, filter_tombstone
    ological = sum(h.logical_bytes() for h in ohosts)
    comp3 = runtime.Compactor()
    st3, ns3 = comp3.run(odruns, oret_d, prm, 256 << 20)
    assert st3 == 0, st3
    torch.cuda.synchronize()
    walls3 = []
    for _ in range(reps):
        t0 = time.perf_counter()
        st3, ns3 = comp3.run(odruns, oret_d, prm, 256 << 20)
        walls3.append((time.perf_counter() - t0) * 1e3)
        assert st3 == 0
    ms3 = float(np.median(walls3))
    _, msum3 = comp3.merged()
    t0 = time.perf_counter()
    _, osm3, ocuts3, ossts3 = O.compact(oruns, O.retention(filter_tombstone=True),
                                        O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10), 256 << 20)
    cpu3_s = time.perf_counter() - t0
    same3 = len(ossts3) == ns3 and all(np.array_equal(comp3.sst(i)["data"], ossts3[i].data) for i in range(ns3))
    print(json.dumps({"what": "compaction job (f2), overwrites: 4 L0 runs over one key space, tombstones in the newest, "
                              "no snapshot, filter_tombstone -> merge + retention (drops) + cuts + encode",
                      "entries_in": int(msum3.num_in), "entries_out": int(msum3.num_out), "output_ssts": ns3,
                      "logical_bytes_in": ological, "ms_wall": round(ms3, 3),
                      "GiB_per_s_logical": round(ological / (ms3 * 1e-3) / 2**30, 2), "bit_exact_vs_oracle": bool(same3),
                      "cpu_baseline": {"kind": "port", "cores": 1, "s": round(cpu3_s, 3),
                                       "GiB_per_s_logical": round(ological / cpu3_s / 2**30, 3),
                                       "sample": "the whole job, oracle compact"}}), flush=True)
    comp3.close()


def codec_bench(reps):
    """f3: 4 D1 SSTs (68,064 blocks) compressed per block (LZ4 / Snappy via the canonical C++ codecs in
    pyarrow, framed as compress_and_transform does), then on the device: sdb_decompress_blocks
    (CRC check + decompress + re-frame) and the decode of the result.  Device-resident, HIP events."""
    sys.path.insert(0, os.path.join(ROOT, "tests"))
    from codec_util import compress_run
    from oracle import oracle as O
    lib = runtime.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    prm = runtime.params(block_size=4096, sst_version=2, bloom_bits_per_key=0)
    datas, offs, base, nent, kbytes = [], [], 0, 0, 0
    for j in range(4):
        h = datasets.d1(sst_index=j)
        db = h.to_device(dev)
        out = runtime.DeviceSstOutput(h.n, h.logical_bytes(), h.logical_bytes(), prm, device=dev)
        runtime.encode_sst_device(db, out)
        torch.cuda.synchronize()
        r = out.to_host()
        datas.append(r["data"])
        bo = r["block_off"].astype(np.uint64)
        offs.append((bo[:-1] if j < 3 else bo) + np.uint64(base))
        base += int(r["data"].size)
        nent += h.n
        kbytes += int(h.key_off[-1])
        del db, out
    data, block_off = np.concatenate(datas), np.concatenate(offs)
    nb = len(block_off) - 1
    only = os.environ.get("SDB_CODECS", "lz4,snappy,zlib,zstd").split(",")  # (per-codec PMC passes)
    for codec, name in ((O.CODEC_LZ4, "lz4"), (O.CODEC_SNAPPY, "snappy"), (O.CODEC_ZLIB, "zlib"), (O.CODEC_ZSTD, "zstd")):
        if name not in only:
            continue
        comp, coff = compress_run(codec, data, block_off)
        dc = torch.from_numpy(comp).to(dev)
        do = torch.from_numpy(coff.view(np.int64)).to(dev)
        with torch.cuda.stream(s):
            o, start, end, err = runtime.decompress_blocks_device(codec, dc, do, stream=s)
        torch.cuda.synchronize()
        total = int(start[nb].item())
        ok = int(err.cpu().numpy().view(np.uint64)[0]) == 2**64 - 1 and np.array_equal(o[:total].cpu().numpy(), data)
        fn = lib.sdb_decompress_blocks

        def run():
            if fn(codec, dc.data_ptr(), do.data_ptr(), nb, o.data_ptr(), total, start.data_ptr(), end.data_ptr(),
                  err.data_ptr(), s.cuda_stream):
                raise RuntimeError("sdb_decompress_blocks")

        with torch.cuda.stream(s):
            ms = timed(run, reps, s)
        plan_ws = torch.empty(lib.sdb_decompress_workspace_bytes(nb), dtype=torch.uint8, device=dev)

        def plan():  # the output plan (zlib / zstd decode to count)
            if lib.sdb_decompress_plan(codec, dc.data_ptr(), do.data_ptr(), nb, start.data_ptr(), plan_ws.data_ptr(),
                                       plan_ws.numel(), s.cuda_stream):
                raise RuntimeError("sdb_decompress_plan")

        with torch.cuda.stream(s):
            ms_plan = timed(plan, max(3, reps // 4), s)
        # CPU baselines on a bounded sample of the same blocks: the oracle (one thread), and for zlib /
        # zstd the canonical C decoders of this image (Python's zlib, pyarrow's zstd) per block
        ns = min(nb, 4000)
        t0 = time.perf_counter()
        rs = O.decompress_blocks(codec, comp[: int(coff[ns])], coff[: ns + 1])
        cpu_s = time.perf_counter() - t0
        cpu_bytes = int(rs.out_start[ns])
        canon = None
        if codec in (O.CODEC_ZLIB, O.CODEC_ZSTD):
            import pyarrow as pa
            zc = pa.Codec("zstd")
            blk = [comp[int(coff[k]):int(coff[k + 1]) - 4].tobytes() for k in range(ns)]
            t0 = time.perf_counter()
            for k, x in enumerate(blk):
                if codec == O.CODEC_ZLIB:
                    __import__("zlib").decompress(x)
                else:
                    zc.decompress(x, decompressed_size=int(rs.out_start[k + 1] - rs.out_start[k]) - 4, asbytes=True)
            canon = round(cpu_bytes / (time.perf_counter() - t0) / 2**30, 3)
        # decode-once (sdb_decompress_blocks_once): no read-back between sizing and decompressing; zlib inflates
        # into 4160-byte slots (block_size + 64) and re-plans the blocks past theirs
        slot = 4096 + 64
        once_ws = torch.empty(lib.sdb_decompress_once_workspace_bytes(nb), dtype=torch.uint8, device=dev)
        ocap = nb * slot + 8 * int(comp.size)
        o1 = torch.empty(ocap + 16, dtype=torch.uint8, device=dev)
        s1 = torch.empty(nb + 1, dtype=torch.int64, device=dev)
        e1 = torch.empty(nb, dtype=torch.int64, device=dev)
        r1 = torch.empty(1, dtype=torch.int64, device=dev)

        def once():
            if lib.sdb_decompress_blocks_once(codec, dc.data_ptr(), do.data_ptr(), nb, slot, o1.data_ptr(), ocap,
                                              s1.data_ptr(), e1.data_ptr(), r1.data_ptr(), once_ws.data_ptr(),
                                              once_ws.numel(), s.cuda_stream):
                raise RuntimeError("sdb_decompress_blocks_once")

        with torch.cuda.stream(s):
            ms_once = timed(once, reps, s)
        torch.cuda.synchronize()
        st1 = s1.cpu().numpy().view(np.uint64)
        spilled = int((st1[:nb] != np.arange(nb, dtype=np.uint64) * np.uint64(slot)).sum()) if codec == O.CODEC_ZLIB else 0
        ok_once = (int(r1.cpu().numpy().view(np.uint64)[0]) == 2**64 - 1 and
                   np.array_equal((e1 - s1[:nb]).cpu().numpy(), (end - start[:nb]).cpu().numpy()))
        del o1
        dev_line = None
        if codec == O.CODEC_ZLIB:
            # the same blocks compressed by the device write side (sdb_compress_blocks: fixed-Huffman / stored
            # deflate), decoded once: every lane of the wide pass decodes a block against shared tables
            dd = torch.from_numpy(data).to(dev)
            db = torch.from_numpy(block_off.view(np.int64)).to(dev)
            cz, czoff, czerr = runtime.compress_blocks_device(codec, dd, db)
            torch.cuda.synchronize()
            czo = czoff[: nb + 1].contiguous()
            ccap = nb * slot + 8 * int(czo[nb].item())
            o2 = torch.empty(ccap + 16, dtype=torch.uint8, device=dev)

            def once2():
                if lib.sdb_decompress_blocks_once(codec, cz.data_ptr(), czo.data_ptr(), nb, slot, o2.data_ptr(), ccap,
                                                  s1.data_ptr(), e1.data_ptr(), r1.data_ptr(), once_ws.data_ptr(),
                                                  once_ws.numel(), s.cuda_stream):
                    raise RuntimeError("sdb_decompress_blocks_once")

            with torch.cuda.stream(s):
                ms_once2 = timed(once2, reps, s)
            torch.cuda.synchronize()
            st2, en2 = s1.cpu().numpy().view(np.uint64), e1.cpu().numpy().view(np.uint64)
            oh = o2.cpu().numpy()
            ok2 = int(r1.cpu().numpy().view(np.uint64)[0]) == 2**64 - 1 and all(
                np.array_equal(oh[int(st2[k]):int(en2[k])], data[int(block_off[k]):int(block_off[k + 1])])
                for k in range(0, nb, 97))
            dev_line = {"compressed_bytes": int(czo[nb].item()), "once_ms": round(ms_once2, 4),
                        "GiB_per_s_decompressed": round(total / (ms_once2 * 1e-3) / 2**30, 2), "ok_sampled": bool(ok2)}
            del o2, cz, dd
        dout = runtime.DeviceDecodeOutput(nb, nent + 16, kbytes + 4096, device=dev)

        def dec():
            runtime.decode_blocks_at_device(o, start[:nb], end, nb, dout, 2, stream=s)

        with torch.cuda.stream(s):
            ms_dec = timed(dec, reps, s)
        print(json.dumps({"what": "f3 decompress (%s) of 4 D1 SSTs" % name, "blocks": nb, "compressed_bytes": int(comp.size),
                          "decompressed_bytes": total, "ratio": round(total / comp.size, 4), "ms": round(ms, 4),
                          "GiB_per_s_decompressed": round(total / (ms * 1e-3) / 2**30, 2),
                          "plan_ms": round(ms_plan, 4), "once_ms": round(ms_once, 4), "once_spilled_blocks": spilled,
                          "once_ok": bool(ok_once), "device_compressed_once": dev_line,
                          "decode_after_ms": round(ms_dec, 4), "bit_exact": bool(ok),
                          "cpu_baseline": {"kind": "port", "GiB_per_s": round(cpu_bytes / cpu_s / 2**30, 3),
                                           "cores": 1, "sample": "first %d blocks, oracle orc_decompress_blocks" % ns,
                                           "canonical_lib_GiB_per_s_1_thread": canon}}), flush=True)


def _encoded_blocks(batches, dev):
    """Encode batches on the device (4 KiB V2 blocks, no filter); returns the concatenated data section and
    the block offsets (one run of blocks)."""
    prm = runtime.params(block_size=4096, sst_version=2, bloom_bits_per_key=0)
    datas, offs, base = [], [], 0
    for j, h in enumerate(batches):
        db = h.to_device(dev)
        out = runtime.DeviceSstOutput(h.n, h.logical_bytes(), h.logical_bytes(), prm, device=dev)
        runtime.encode_sst_device(db, out)
        torch.cuda.synchronize()
        r = out.to_host()
        datas.append(r["data"])
        bo = r["block_off"].astype(np.uint64)
        offs.append((bo[:-1] if j < len(batches) - 1 else bo) + np.uint64(base))
        base += int(r["data"].size)
        del db, out
    return np.concatenate(datas), np.concatenate(offs)


def compress_bench(reps, sets=("d1", "text")):
    """f3 write side: sdb_compress_blocks over 4 D1 SSTs (random values) and over a compressible set
    (datasets.text_kv: JSON documents, ~60 MiB), every codec.  Device bytes and ratio beside the canonical
    library's on the same blocks (zstd level 3 = zstd::bulk::compress(data, 3); zlib level 6 = flate2's
    default; pyarrow LZ4 raw / Snappy), sampled every 4th block; device GB/s by HIP events; the canonical
    library's one-thread speed as the CPU baseline.  Validity: every block of the device output decompresses
    (device decompressor) to the input."""
    import zlib
    import pyarrow as pa
    from oracle import oracle as O
    lib = runtime.lib()
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    canon = {O.CODEC_LZ4: pa.Codec("lz4_raw"), O.CODEC_SNAPPY: pa.Codec("snappy"),
             O.CODEC_ZSTD: pa.Codec("zstd", compression_level=3)}
    only = os.environ.get("SDB_CODECS", "lz4,snappy,zlib,zstd").split(",")
    sets = os.environ.get("SDB_SETS", ",".join(sets)).split(",")
    for name in sets:
        if name == "d1":
            batches = [datasets.d1(sst_index=j) for j in range(4)]
        else:
            batches = [datasets.text_kv(n=200_000, seed=11 + j) for j in range(2)]
        data, block_off = _encoded_blocks(batches, dev)
        del batches
        nb = len(block_off) - 1
        in_bytes = int(block_off[-1] - block_off[0])
        dd = torch.from_numpy(np.concatenate([data, np.zeros(64, np.uint8)])).to(dev)
        db = torch.from_numpy(block_off.view(np.int64)).to(dev)
        sample = range(0, nb, 4)
        raws = [data[int(block_off[k]):int(block_off[k + 1]) - 4].tobytes() for k in sample]
        for codec, cname in ((O.CODEC_LZ4, "lz4"), (O.CODEC_SNAPPY, "snappy"), (O.CODEC_ZLIB, "zlib"), (O.CODEC_ZSTD, "zstd")):
            if cname not in only:
                continue
            with torch.cuda.stream(s):
                out, out_off, err = runtime.compress_blocks_device(codec, dd, db, stream=s)
            torch.cuda.synchronize()
            ok_err = int(err.item()) == -1
            ws = torch.empty(int(lib.sdb_compress_workspace_bytes(nb, in_bytes)), dtype=torch.uint8, device=dev)
            cap = out.numel() - 16

            def run():
                if lib.sdb_compress_blocks(codec, dd.data_ptr(), db.data_ptr(), nb, in_bytes, out.data_ptr(), cap,
                                           out_off.data_ptr(), err.data_ptr(), ws.data_ptr(), ws.numel(), s.cuda_stream):
                    raise RuntimeError("sdb_compress_blocks")

            with torch.cuda.stream(s):
                ms = timed(run, reps, s)
            coff = out_off.cpu().numpy().view(np.uint64)
            total = int(coff[nb])
            # validity: the device decompressor restores every block
            with torch.cuda.stream(s):
                o, st, en, derr = runtime.decompress_blocks_device(codec, out[:total + 64].contiguous(), out_off, stream=s)
            torch.cuda.synchronize()
            ok = ok_err and int(derr.item()) == -1 and int(st[nb].item()) == data.size and \
                np.array_equal(o[:data.size].cpu().numpy(), data)
            # the canonical library on the sampled blocks (+ the same framing: lz4 size prefix, CRC)
            t0 = time.perf_counter()
            lib_bytes = 0
            for x in raws:
                if codec == O.CODEC_ZLIB:
                    c = zlib.compress(x, 6)
                else:
                    c = canon[codec].compress(x, asbytes=True)
                lib_bytes += len(c) + 4 + (4 if codec == O.CODEC_LZ4 else 0)
            cpu_s = time.perf_counter() - t0
            raw_bytes = sum(len(x) + 4 for x in raws)
            dev_bytes = int(sum(int(coff[k + 1] - coff[k]) for k in sample))
            print(json.dumps({
                "what": "f3 compress (%s) of %s" % (cname, "4 D1 SSTs" if name == "d1" else "text_kv (JSON values)"),
                "blocks": nb, "input_bytes": in_bytes, "compressed_bytes": total, "ratio_device": round(in_bytes / total, 4),
                "sample_blocks": len(raws), "sample_ratio_device": round(raw_bytes / dev_bytes, 4),
                "sample_ratio_library": round(raw_bytes / lib_bytes, 4),
                "device_over_library_bytes": round(dev_bytes / lib_bytes, 4),
                "library": {O.CODEC_ZLIB: "zlib level 6", O.CODEC_ZSTD: "zstd level 3 (pyarrow)",
                            O.CODEC_LZ4: "lz4 raw (pyarrow)", O.CODEC_SNAPPY: "snappy (pyarrow)"}[codec],
                "ms": round(ms, 4), "GB_per_s": round(in_bytes / (ms * 1e-3) / 1e9, 2),
                "frac_hbm": round((in_bytes + total) / (ms * 1e-3) / 1e9 / PEAK * 1000 / 1000, 5),
                "valid_device_roundtrip": bool(ok),
                "cpu_baseline": {"kind": "canonical library", "GiB_per_s": round(raw_bytes / cpu_s / 2**30, 3), "cores": 1,
                                 "sample": "every 4th block, %d blocks" % len(raws)}}), flush=True)
            del out, ws, o
        del dd, db


def lookup_bench(reps):
    """Point lookups (sdb_sst_lookup: bloom -> index partition -> block CRC -> restart search -> seek) of
    1 M keys into one D1 SST (configs[1] shape): half present, half absent (bloom-filtered or seeking past),
    device-resident, HIP events; the oracle on a bounded sample as the CPU baseline."""
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    h = datasets.d1(sst_index=5)
    enc = O.encode_sst(h, O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10))
    ik, iko = O.sst_index_keys(h, enc)
    rng = np.random.default_rng(17)
    nq = 1 << 20
    pick = rng.integers(0, h.n, nq)
    kb = np.empty(nq * 16, np.uint8)
    for q in range(nq):  # present keys, and the same keys with the last byte flipped (absent)
        k0 = int(h.key_off[pick[q]])
        kb[16 * q:16 * q + 16] = h.key_bytes[k0:k0 + 16]
    kb[16 * np.arange(1, nq, 2) + 15] ^= 0xA5
    koff = (np.arange(nq + 1, dtype=np.uint64) * np.uint64(16))
    t = lambda a: torch.from_numpy(np.ascontiguousarray(a).view(np.int64) if a.dtype == np.uint64 else a).to(dev)
    vt = {"data": t(enc.data), "block_off": t(enc.block_off), "num_blocks": len(enc.block_off) - 1,
          "index_keys": t(ik), "index_key_off": t(iko), "sst_version": 2, "bloom": t(enc.bloom),
          "bloom_len": len(enc.bloom), "num_probes": O.optimal_num_probes(10)}
    dk, do = t(kb), t(koff)
    with torch.cuda.stream(s):
        res = runtime.sst_lookup_device(vt, dk, do, nq, stream=s)
    torch.cuda.synchronize()
    ns = 20000
    keys = [kb[16 * q:16 * q + 16].tobytes() for q in range(ns)]
    t0 = time.perf_counter()
    ref = O.sst_lookup(enc.data, enc.block_off, ik, iko, keys, bloom=enc.bloom, num_probes=O.optimal_num_probes(10))
    cpu_s = time.perf_counter() - t0
    ok = all(np.array_equal(res[f][:ns].cpu().numpy().astype(np.int64), getattr(ref, f).astype(np.int64))
             for f in ("state", "block", "entry", "val_off", "seq"))

    def run():
        runtime.sst_lookup_device(vt, dk, do, nq, stream=s)

    with torch.cuda.stream(s):
        ms = timed(run, reps, s)
    print(json.dumps({"what": "point lookups into one D1 SST (bloom, index, CRC, restart search, seek)",
                      "keys": nq, "present_fraction": 0.5, "ms": round(ms, 4),
                      "Mlookups_per_s": round(nq / (ms * 1e-3) / 1e6, 1), "matches_oracle_on_sample": bool(ok),
                      "cpu_baseline": {"kind": "port", "cores": 1, "Mlookups_per_s": round(ns / cpu_s / 1e6, 3),
                                       "sample": "first %d of the same keys, oracle orc_sst_lookup" % ns}}), flush=True)


def encode_variants_bench(reps):
    """Headline-shaped encode (8 SSTs per sdb_encode_ssts call, resident) on the other SURVEY §8(d)
    datasets: D2 (sorted random 16 B keys, shared prefix ~2 B) and D1-L0 (N = 489,740, the memtable size
    at which a real L0 flush freezes).  SST 0 of each set is checked bit-exact against the oracle."""
    from oracle import oracle as O
    dev = torch.device("cuda", 0)
    s = torch.cuda.Stream(device=dev)
    prm = runtime.params(block_size=4096, sst_version=2, restart_interval=16, bloom_bits_per_key=10)
    oprm = O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    variants = [("D2 random-sorted", lambda j: datasets.d2(seed=datasets.SEED_D2 + j)),
                ("D1-L0 (N=489,740)", lambda j: datasets.d1(sst_index=j, n=489_740))]
    for name, make in variants:
        hosts = [make(j) for j in range(8)]
        dbs = [h.to_device(dev) for h in hosts]
        outs = [runtime.DeviceSstOutput(h.n, h.logical_bytes(), h.logical_bytes(), prm, device=dev,
                                        workspace=False) for h in hosts]
        ws = runtime.ssts_workspace(dbs, prm, device=dev)
        run = lambda: runtime.encode_ssts_device(dbs, outs, prm, ws, s)
        run()
        torch.cuda.synchronize()
        got = outs[0].to_host()
        ref = O.encode_sst(hosts[0], oprm)
        ok = (got["summary"].status == 0 and np.array_equal(got["data"], ref.data)
              and np.array_equal(got["bloom"], ref.bloom) and np.array_equal(got["block_off"], ref.block_off))
        ms = timed(run, reps, s)
        logical = sum(h.logical_bytes() for h in hosts)
        alg = 0
        for h, o in zip(hosts, outs):
            sm = o.summary_host()
            alg += h.algorithmic_input_bytes() + sm.data_len + sm.bloom_len
        print(json.dumps({"what": "encode %s, 8 SSTs per call (headline shape)" % name, "entries_per_sst": hosts[0].n,
                          "ms_per_call": round(ms, 4), "ms_per_sst": round(ms / 8, 4),
                          "GiBps_logical": round(logical / (ms * 1e-3) / 2**30, 1),
                          "alg_GBps": round(alg / (ms * 1e-3) / 1e9, 1),
                          "frac_of_8TBps": round(alg / (ms * 1e-3) / 1e9 / PEAK, 3),
                          "matches_oracle_sst0": bool(ok)}), flush=True)
        del dbs, outs, ws
        torch.cuda.empty_cache()


def hbm_bench(reps):
    """STREAM-like: torch's copy kernel over 4 GiB (read + write) and a read-only int64 sum."""
    dev = torch.device("cuda", 0)
    nbytes = 4 << 30
    a = torch.randint(0, 255, (nbytes,), dtype=torch.uint8, device=dev)
    b = torch.empty_like(a)
    s = torch.cuda.current_stream()
    ms_copy = timed(lambda: b.copy_(a), reps, s)
    a64 = a.view(torch.int64)
    ms_read = timed(lambda: a64.sum(), reps, s)
    cp = 2 * nbytes / (ms_copy * 1e-3) / 1e9
    rd = nbytes / (ms_read * 1e-3) / 1e9
    print(json.dumps({"what": "measured HBM bandwidth (4 GiB buffers)", "copy_GBps": round(cp, 1),
                      "read_GBps": round(rd, 1), "spec_GBps": PEAK, "copy_frac_of_spec": round(cp / PEAK, 3),
                      "note": "roofline fractions use the 8.0 TB/s spec; this is the attainable ceiling"}),
          flush=True)
    del a, b, a64


def footer_bench(reps):
    """Host footer of one D1 SST (sdb_sst_footer: filter block, index, stats, SsTableInfo; 17,016 blocks):
    the C call alone, its inputs prepared once (the first keys gathered as runtime.sst_footer does)."""
    from oracle import oracle as O
    b = datasets.d1(sst_index=3)
    e = O.encode_sst(b, O.params())
    ref = runtime.sst_footer(b, e)
    sm = e.summary if isinstance(e.summary, _abi.SstSummary) else _abi.SstSummary(**e.summary)
    nb = len(e.block_off) - 1
    starts = np.asarray(e.block_first_entry[:nb], np.int64)
    ikl = np.asarray(e.index_key_len[:nb], np.uint64)
    fko = np.zeros(nb + 1, np.uint64)
    fko[1:] = np.cumsum(ikl)
    idx = np.repeat(b.key_off[starts] - fko[:-1], ikl.astype(np.int64)) + np.arange(int(fko[-1]), dtype=np.uint64)
    fk = np.ascontiguousarray(b.key_bytes[idx.astype(np.int64)])
    boff = np.ascontiguousarray(e.block_off[:nb], np.uint64)
    bst = np.ascontiguousarray(np.asarray(e.block_stats, np.uint16).reshape(-1))
    bloom = np.ascontiguousarray(np.asarray(e.bloom, np.uint8))
    first, last = b.key(0), b.key(b.n - 1)
    fi = _abi.FooterIn(2, _abi.SST_COMPACTED, 1, sm.num_probes, int(sm.data_len), nb, boff.ctypes.data,
                       fk.ctypes.data, fko.ctypes.data, first, len(first), last, len(last), C.addressof(sm),
                       bst.ctypes.data, bloom.ctypes.data, int(sm.bloom_len), None)
    L = runtime.lib()
    cap = L.sdb_sst_footer_bound(C.byref(fi))
    out = np.empty(cap, np.uint8)
    n = C.c_uint64(0)
    ts = []
    for _ in range(reps + 3):
        t0 = time.perf_counter()
        st = L.sdb_sst_footer(C.byref(fi), out.ctypes.data, cap, C.byref(n))
        ts.append(time.perf_counter() - t0)
        assert st == 0
    assert out[:n.value].tobytes() == ref, "footer bytes changed"
    ts = sorted(ts[3:])
    print(json.dumps({"what": "host SST footer (sdb_sst_footer) of one D1 SST", "blocks": nb, "footer_bytes": n.value,
                      "ms_median": round(1e3 * ts[len(ts) // 2], 3), "ms_min": round(1e3 * ts[0], 3),
                      "cpu": cpu_model()}), flush=True)


def main():
    p = argparse.ArgumentParser()
    p.add_argument("--decode", action="store_true")
    p.add_argument("--bloom", action="store_true")
    p.add_argument("--e2e", action="store_true")
    p.add_argument("--compact", action="store_true")
    p.add_argument("--hbm", action="store_true")
    p.add_argument("--codec", action="store_true")
    p.add_argument("--compress", action="store_true", help="f3 write side: device vs canonical library ratio and speed")
    p.add_argument("--lookup", action="store_true")
    p.add_argument("--encode", action="store_true", help="encode D2 and D1-L0 (headline shape)")
    p.add_argument("--footer", action="store_true", help="host footer of one D1 SST (no device)")
    p.add_argument("--cpu-seconds", type=float, default=12.0, help="decode CPU baseline budget (0: skip)")
    p.add_argument("--reps", type=int, default=20)
    p.add_argument("--no-granular", action="store_true", help="decode: skip the 2 MiB granularity run")
    a = p.parse_args()
    allp = not (a.decode or a.bloom or a.e2e or a.compact or a.hbm or a.codec or a.compress or a.lookup or a.encode or
                a.footer)
    if a.footer or allp:
        footer_bench(max(a.reps, 20))
    if a.footer and not allp:
        return
    torch.cuda.set_device(0)
    runtime.require_device()
    if a.bloom or allp:
        bloom_bench(a.reps)
    if a.decode or allp:
        decode_bench(a.reps, not a.no_granular, a.cpu_seconds)
    if a.e2e or allp:
        e2e_bench(a.reps)
    if a.hbm or allp:
        hbm_bench(a.reps)
    if a.codec or allp:
        codec_bench(max(3, a.reps // 2))
    if a.compress or allp:
        compress_bench(max(3, a.reps // 4))
    if a.compact or allp:
        compact_bench(max(3, a.reps // 4))
    if a.lookup or allp:
        lookup_bench(a.reps)
    if a.encode or allp:
        encode_variants_bench(a.reps)


if __name__ == "__main__":
    main()
