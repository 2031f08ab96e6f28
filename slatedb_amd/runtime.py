"""Host-side front-end of libslatedb_amd.so (ctypes over the C ABI in include/slatedb_amd.h).

Mirrors the reference's surface for this path:
  * SstBuilder            <- EncodedSsTableBuilder add()/build()/next_block() (sst_builder.rs:224-417)
  * BloomFilterPolicy     <- FilterPolicy "_bf" / BloomFilterBuilder (filter_policy.rs:170-283,
                             filter.rs:40-90); encode() = Filter::encode (filter.rs:177-180)
  * read_blocks()         <- SsTableFormat::read_blocks + DataBlockIterator (format/sst.rs:938-999)
  * encode_sst_device()   <- the batched device entry point used by bench.py

The HIP library is mandatory: a missing .so or a machine without a HIP device raises; nothing
falls back to a CPU implementation.
"""
import ctypes as C
import os

import numpy as np

from . import _abi
from .batch import Batch

HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.path.join(HERE, "libslatedb_amd.so")
# tuning experiments only: an alternative in-tree build of the same library
if os.environ.get("SDB_LIBRARY"):
    LIB_PATH = os.path.join(HERE, os.path.basename(os.environ["SDB_LIBRARY"]))

_lib = None


class SdbError(RuntimeError):
    def __init__(self, status, what=""):
        self.status = status
        super().__init__("%s: %s" % (what or "slatedb_amd", _abi.STATUS_NAMES.get(status, status)))


def lib():
    """Load libslatedb_amd.so (fails loudly if it has not been built).

    torch is imported first on purpose: torch ships its own libamdhip64.so with the same soname
    (libamdhip64.so.7) as /opt/rocm's, so loading it first makes our library bind to the HIP runtime
    torch already uses — one runtime per process, so torch streams, events and allocations are
    valid handles for our kernels.  (The Rust/C host links /opt/rocm's runtime as usual.)"""
    global _lib
    if _lib is None:
        try:
            import torch  # noqa: F401
            if torch.cuda.is_available():
                torch.cuda.init()
        except ImportError:
            pass
        if not os.path.exists(LIB_PATH):
            raise ImportError("libslatedb_amd.so not built: run `python __graft_entry__.py build` "
                              "(hipcc --offload-arch=gfx950)")
        _lib = _abi.bind(C.CDLL(LIB_PATH), partial=bool(os.environ.get("SDB_LIBRARY")))
    return _lib


def device_count():
    return lib().sdb_device_count()


def require_device():
    if device_count() <= 0:
        raise SdbError(_abi.SDB_DEVICE_ERROR, "no HIP device visible")


def params(block_size=4096, sst_version=2, restart_interval=16, bloom_bits_per_key=10,
           min_filter_keys=0, sst_type=_abi.SST_COMPACTED, prefix_kind=0, prefix_arg=0, no_whole_key=0):
    return _abi.SstParams(block_size, sst_version, restart_interval, bloom_bits_per_key,
                          min_filter_keys, sst_type, prefix_kind, prefix_arg, no_whole_key)


def filter_name(prm, extractor_name=None):
    """FilterPolicy::name of BloomFilterPolicy (filter_policy.rs:237-250): "_bf[:p=<extractor>][:wh=0]"."""
    name = "_bf"
    if prm.prefix_kind:
        name += ":p=" + (extractor_name or {1: "fixed%d" % prm.prefix_arg, 2: "delim%d" % prm.prefix_arg,
                                            3: "custom"}[prm.prefix_kind])
    if prm.no_whole_key:
        name += ":wh=0"
    return name.encode()


def bloom_build_prefix_device(key_bytes, key_off, n, bpk, kind, arg=0, whole=True, prefix_len=None, stream=None):
    """sdb_bloom_build_prefix over device tensors -> the bitmap (torch uint8, device-counted length)."""
    import torch
    dev = key_bytes.device
    cap = lib().sdb_bloom_filter_bytes(2 * n, bpk) + 16
    bm = torch.empty((cap + 3) // 4 * 4, dtype=torch.uint8, device=dev)
    ln = torch.zeros(1, dtype=torch.int64, device=dev)
    wsb = lib().sdb_bloom_prefix_workspace_bytes(n)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    sp = None if stream is None else (stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
    st = lib().sdb_bloom_build_prefix(key_bytes.data_ptr(), key_off.data_ptr(),
                                      None if prefix_len is None else prefix_len.data_ptr(), n, bpk, kind, arg,
                                      int(whole), bm.data_ptr(), cap, ln.data_ptr(), ws.data_ptr(), wsb, sp)
    if st:
        raise SdbError(st, "sdb_bloom_build_prefix")
    torch.cuda.synchronize()
    L = int(ln.item())
    if L < 0:
        raise SdbError(_abi.SDB_INVALID_ARGUMENT, "sdb_bloom_build_prefix (prefix longer than its key)")
    return bm[:L]


def might_match_device(bitmap, num_probes, whole, kind, arg, key_bytes, key_off, n, is_prefix=None,
                       query_prefix_len=None, stream=None):
    """sdb_bloom_might_match over device tensors -> torch uint8 results."""
    import torch
    res = torch.zeros(max(n, 1), dtype=torch.uint8, device=key_bytes.device)
    sp = None if stream is None else (stream.cuda_stream if hasattr(stream, "cuda_stream") else stream)
    st = lib().sdb_bloom_might_match(bitmap.data_ptr() if bitmap.numel() else None, bitmap.numel(), num_probes,
                                     int(whole), kind, arg, key_bytes.data_ptr(), key_off.data_ptr(),
                                     None if is_prefix is None else is_prefix.data_ptr(),
                                     None if query_prefix_len is None else query_prefix_len.data_ptr(), n,
                                     res.data_ptr(), sp)
    if st:
        raise SdbError(st, "sdb_bloom_might_match")
    return res[:n]


def _u8(ptr, n):
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(C.c_uint8)), (n,)) if n else np.zeros(0, np.uint8)


def _arr(ptr, ctype, n, dtype):
    if not n:
        return np.zeros(0, dtype)
    return np.ctypeslib.as_array(C.cast(ptr, C.POINTER(ctype)), (n,)).view(dtype)


class EncodedSst:
    """Data section + bloom of one SST (host copies)."""

    def __init__(self, res, params_):
        sm = res.summary
        self.status = sm.status
        self.summary = {f: getattr(sm, f) for f, _ in _abi.SstSummary._fields_}
        ok = sm.status == 0
        nb = sm.num_blocks if ok else 0
        self.data = _u8(res.data, sm.data_len if ok else 0).copy()
        self.block_off = _arr(res.block_off, C.c_uint64, nb + 1 if ok else 0, np.uint64).copy()
        self.block_first_entry = _arr(res.block_first_entry, C.c_uint32, nb + 1 if ok else 0, np.uint32).copy()
        self.index_key_len = _arr(res.index_key_len, C.c_uint32, nb, np.uint32).copy()
        self.block_stats = _arr(res.block_stats, C.c_uint16, 3 * nb, np.uint16).reshape(-1, 3).copy()
        self.bloom = _u8(res.bloom, sm.bloom_len if sm.status == 0 else 0).copy()
        self.num_probes = sm.num_probes
        self.filter_built = bool(sm.filter_built)
        self.timings_ms = {"h2d": res.h2d_ms, "kernel": res.kernel_ms, "d2h": res.d2h_ms}
        self.sst_version = params_.sst_version
        self._next = 0

    @property
    def num_blocks(self):
        return len(self.index_key_len)

    def block(self, k):
        """Encoded block k: Block::encode() ++ crc32 BE (EncodedSsTableBlock.encoded_bytes)."""
        return self.data[int(self.block_off[k]):int(self.block_off[k + 1])].tobytes()

    def next_block(self):
        """EncodedSsTableBuilder::next_block (sst_builder.rs:274-276)."""
        if self._next >= self.num_blocks:
            return None
        b = self.block(self._next)
        self._next += 1
        return b

    def filter_block(self, name="_bf"):
        """Composite filter block bytes incl. CRC (format/sst.rs:394-421, 525-554)."""
        import struct
        import zlib
        if not self.filter_built:
            return b""
        enc = struct.pack(">H", self.num_probes) + self.bloom.tobytes()
        comp = struct.pack(">HH", 1, len(name)) + name.encode() + struct.pack(">Q", len(enc)) + enc
        return comp + struct.pack(">I", zlib.crc32(comp))


def sst_footer(batch, enc, sst_version=2, sst_type=_abi.SST_COMPACTED, filter_name=None, compression=0):
    """Footer bytes after the data section (sdb_sst_footer; EncodedSsTableFooterBuilder::build,
    format/sst.rs:383-487).  `enc` is an encode result with host arrays (EncodedSst, the
    DeviceSstOutput.to_host() dict wrapped by `_FooterView`, or anything with data/block_off/
    block_first_entry/index_key_len/block_stats/bloom/summary).  For SST_WAL the block first keys
    are the first entries' seq numbers, big-endian (wal/slatedb/sst_builder.rs:137-155), and there
    is no last entry, stats or filter.  Host code: no device needed."""
    sm = enc.summary if isinstance(enc.summary, _abi.SstSummary) else _abi.SstSummary(**enc.summary)
    nb = len(enc.block_off) - 1 if len(enc.block_off) else 0
    starts = np.asarray(enc.block_first_entry[:nb], np.int64)
    if sst_type == _abi.SST_WAL:
        seqs = (np.zeros(batch.n, np.uint64) if batch.seq is None else batch.seq)[starts]
        fk = seqs.astype(">u8").view(np.uint8).copy()
        fko = np.arange(nb + 1, dtype=np.uint64) * 8
        first = fk[:8].tobytes() if nb else None
        last = None
    else:
        ikl = np.asarray(enc.index_key_len[:nb], np.uint64)
        fko = np.zeros(nb + 1, np.uint64)
        fko[1:] = np.cumsum(ikl)
        ks = batch.key_off[starts] if nb else np.zeros(0, np.uint64)
        idx = np.repeat(ks - fko[:-1], ikl.astype(np.int64)) + np.arange(int(fko[-1]), dtype=np.uint64)
        fk = batch.key_bytes[idx.astype(np.int64)].copy() if len(idx) else np.zeros(1, np.uint8)
        first = batch.key(0) if batch.n else None
        last = batch.key(batch.n - 1) if batch.n else None
    boff = np.ascontiguousarray(enc.block_off[:nb], np.uint64)
    bst = np.ascontiguousarray(np.asarray(enc.block_stats, np.uint16).reshape(-1))
    bloom = np.ascontiguousarray(np.asarray(enc.bloom, np.uint8))
    fk = np.ascontiguousarray(fk if len(fk) else np.zeros(1, np.uint8))
    wal = sst_type == _abi.SST_WAL
    fi = _abi.FooterIn(sst_version, sst_type, 0 if wal else int(bool(sm.filter_built)), sm.num_probes,
                       int(sm.data_len), nb, boff.ctypes.data, fk.ctypes.data, fko.ctypes.data,
                       first, len(first or b""), last, len(last or b""),
                       None if wal else C.addressof(sm), bst.ctypes.data if len(bst) else None,
                       bloom.ctypes.data if len(bloom) else None, 0 if wal else int(sm.bloom_len),
                       filter_name, compression, 0)
    n = C.c_uint64(0)
    cap = lib().sdb_sst_footer_bound(C.byref(fi))
    out = np.empty(max(cap, 1), np.uint8)
    st = lib().sdb_sst_footer(C.byref(fi), out.ctypes.data, cap, C.byref(n))
    if st:
        raise SdbError(st, "sdb_sst_footer")
    return out[:n.value].tobytes()


def sst_object(batch, enc, sst_version=2, sst_type=_abi.SST_COMPACTED, filter_name=None):
    """The whole SST object (data section ++ footer) that write_sst stores."""
    return np.asarray(enc.data, np.uint8).tobytes() + sst_footer(batch, enc, sst_version, sst_type, filter_name)


class Encoder:
    """Host-buffer encoder (device arena + pinned staging + its own stream)."""

    def __init__(self, prm=None, device=0):
        require_device()
        self.params = prm or params()
        self._h = lib().sdb_encoder_create(device, C.byref(self.params))
        if not self._h:
            raise SdbError(_abi.SDB_DEVICE_ERROR, "sdb_encoder_create")

    def encode(self, batch, copy=True):
        kb = batch.to_ctypes()
        res = _abi.SstHostResult()
        st = lib().sdb_encoder_encode_host(self._h, C.byref(kb), C.byref(res))
        if not copy:  # the raw SstHostResult view (valid until the next call)
            return st, res
        out = EncodedSst(res, self.params)
        out.status = st
        return out

    def encode_many(self, batches, copy=True):
        """sdb_encoder_encode_host_many: several SSTs with overlapped transfers.  copy=False returns the
        raw SstHostResult views (valid until the next call) instead of EncodedSst copies."""
        kbs = (_abi.KvBatch * max(len(batches), 1))(*[b.to_ctypes() for b in batches])
        res = (_abi.SstHostResult * max(len(batches), 1))()
        st = lib().sdb_encoder_encode_host_many(self._h, len(batches), kbs, res)
        self.last_status = st
        if not copy:
            return st, res
        return [EncodedSst(res[i], self.params) for i in range(len(batches))]

    def close(self):
        if self._h:
            lib().sdb_encoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class SstBuilder:
    """EncodedSsTableBuilder mirror: add() entries in order, then build() encodes on the GPU."""

    def __init__(self, prm=None, device=0):
        require_device()
        self.params = prm or params()
        self._h = lib().sdb_sst_builder_new(device, C.byref(self.params))
        if not self._h:
            raise SdbError(_abi.SDB_DEVICE_ERROR, "sdb_sst_builder_new")

    def add(self, key, value=b"", seq=0, kind=_abi.KIND_VALUE, create_ts=None, expire_ts=None):
        key = bytes(key)
        value = bytes(value or b"")
        st = lib().sdb_sst_builder_add(self._h, key, len(key), kind, value, len(value), seq,
                                       create_ts is not None, create_ts or 0, expire_ts is not None,
                                       expire_ts or 0)
        if st:
            raise SdbError(st, "add")

    def add_value(self, key, value, create_ts=None, expire_ts=None):
        """EncodedSsTableBuilder::add_value (sst_builder.rs:257-272): seq 0."""
        self.add(key, value, 0, _abi.KIND_VALUE, create_ts, expire_ts)

    def build(self):
        res = _abi.SstHostResult()
        st = lib().sdb_sst_builder_build(self._h, C.byref(res))
        out = EncodedSst(res, self.params)
        out.status = st
        return out

    def close(self):
        if self._h:
            lib().sdb_sst_builder_free(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class BloomFilterPolicy:
    """FilterPolicy "_bf" with whole-key filtering (filter_policy.rs:170-283)."""

    NAME = "_bf"

    def __init__(self, bits_per_key=10):
        self.bits_per_key = bits_per_key

    def name(self):
        return self.NAME

    def num_probes(self):
        return lib().sdb_bloom_num_probes(self.bits_per_key)

    def estimate_size(self, num_keys):
        return lib().sdb_bloom_filter_bytes(num_keys, self.bits_per_key) + 2

    def build_device(self, key_bytes, key_off, n, stream=None):
        """Bitmap over device-resident keys -> torch uint8 tensor (device)."""
        import torch
        fb = lib().sdb_bloom_filter_bytes(n, self.bits_per_key)
        bm = torch.empty((fb + 3) // 4 * 4 or 4, dtype=torch.uint8, device=key_bytes.device)
        wsb = lib().sdb_bloom_workspace_bytes(n, self.bits_per_key)
        ws = torch.empty(wsb, dtype=torch.uint8, device=key_bytes.device)
        st = lib().sdb_bloom_build(key_bytes.data_ptr(), key_off.data_ptr(), n, self.bits_per_key,
                                   bm.data_ptr(), fb, ws.data_ptr(), wsb, stream)
        if st:
            raise SdbError(st, "sdb_bloom_build")
        return bm[:fb]

    def build(self, batch_or_keys):
        """Filter::encode bytes: u16 BE num_probes ++ bitmap (filter.rs:177-180)."""
        import struct
        import torch
        require_device()
        if isinstance(batch_or_keys, Batch):
            kbytes, koff = batch_or_keys.key_bytes, batch_or_keys.key_off
        else:
            keys = [bytes(k) for k in batch_or_keys]
            koff = np.zeros(len(keys) + 1, np.uint64)
            koff[1:] = np.cumsum([len(k) for k in keys]) if keys else []
            kbytes = np.frombuffer(b"".join(keys) or b"\0", np.uint8)
        n = len(koff) - 1
        dk = torch.from_numpy(np.ascontiguousarray(kbytes)).cuda() if kbytes.size else torch.zeros(16, dtype=torch.uint8, device="cuda")
        do = torch.from_numpy(np.ascontiguousarray(koff).view(np.uint8)).cuda()
        bm = self.build_device(dk, do, n)
        torch.cuda.synchronize()
        return struct.pack(">H", self.num_probes()) + bm.cpu().numpy().tobytes()


def might_contain(bitmap, num_probes, keys):
    """Batched BloomFilter::might_contain over host keys; returns a bool array."""
    import torch
    require_device()
    keys = [bytes(k) for k in keys]
    koff = np.zeros(len(keys) + 1, np.uint64)
    koff[1:] = np.cumsum([len(k) for k in keys]) if keys else []
    kb = np.frombuffer(b"".join(keys) or b"\0", np.uint8).copy()
    dk = torch.from_numpy(kb).cuda()
    do = torch.from_numpy(koff.view(np.uint8)).cuda()
    bm = np.ascontiguousarray(bitmap, np.uint8)
    dbm = torch.from_numpy(np.concatenate([bm, np.zeros(4, np.uint8)])).cuda()
    res = torch.zeros(max(len(keys), 1), dtype=torch.uint8, device="cuda")
    st = lib().sdb_bloom_might_contain(dbm.data_ptr(), bm.size, num_probes, dk.data_ptr(), do.data_ptr(),
                                       len(keys), res.data_ptr(), None)
    if st:
        raise SdbError(st, "sdb_bloom_might_contain")
    torch.cuda.synchronize()
    return res.cpu().numpy()[:len(keys)].astype(bool)


class Decoded:
    pass


class Decoder:
    def __init__(self, device=0):
        require_device()
        self._h = lib().sdb_decoder_create(device)
        if not self._h:
            raise SdbError(_abi.SDB_DEVICE_ERROR, "sdb_decoder_create")

    def decode(self, blocks, block_off, sst_version=2):
        blocks = np.ascontiguousarray(blocks, np.uint8)
        block_off = np.ascontiguousarray(block_off, np.uint64)
        nb = len(block_off) - 1
        res = _abi.DecodeHostResult()
        st = lib().sdb_decoder_decode_host(self._h, blocks.ctypes.data if blocks.size else None,
                                           block_off.ctypes.data, nb, sst_version, C.byref(res))
        d = Decoded()
        d.status = st
        sm = res.summary
        d.summary = {f: getattr(sm, f) for f, _ in _abi.DecodeSummary._fields_}
        n = sm.num_entries if st in (0, 3, 4, 9) else 0
        d.n = n
        d.block_entry_start = _arr(res.block_entry_start, C.c_uint64, nb + 1, np.uint64).copy()
        d.key_off = _arr(res.key_off, C.c_uint64, n + 1, np.uint64).copy()
        d.key_arena = _u8(res.key_arena, sm.key_bytes).copy()
        d.val_off = _arr(res.val_off, C.c_uint64, n, np.uint64).copy()
        d.val_len = _arr(res.val_len, C.c_uint32, n, np.uint32).copy()
        d.seq = _arr(res.seq, C.c_uint64, n, np.uint64).copy()
        d.flags = _u8(res.flags, n).copy()
        d.create_ts = _arr(res.create_ts, C.c_int64, n, np.int64).copy()
        d.expire_ts = _arr(res.expire_ts, C.c_int64, n, np.int64).copy()
        d.bad_block = _arr(res.bad_block, C.c_uint32, min(sm.num_bad_blocks, nb + 1), np.uint32).copy()
        return d

    def close(self):
        if self._h:
            lib().sdb_decoder_destroy(self._h)
            self._h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


# ------------------------------------------------------------------------------------------------
# Device-resident batched entry point (bench / multi-SST pipelines)
# ------------------------------------------------------------------------------------------------
class DeviceSstOutput:
    """Caller-owned device outputs + workspace for sdb_encode_sst (allocated once, reused)."""

    def __init__(self, n, total_key_bytes, total_val_bytes, prm, device="cuda", workspace=True):
        import torch
        dc, bc, fc = C.c_uint64(), C.c_uint64(), C.c_uint64()
        st = lib().sdb_encode_bounds(n, total_key_bytes, total_val_bytes, C.byref(prm), C.byref(dc),
                                     C.byref(bc), C.byref(fc))
        if st:
            raise SdbError(st, "sdb_encode_bounds")
        self.params = prm
        self.data = torch.empty(dc.value, dtype=torch.uint8, device=device)
        self.block_off = torch.empty(bc.value + 1, dtype=torch.int64, device=device)
        self.block_first = torch.empty(bc.value + 1, dtype=torch.int32, device=device)
        self.index_key_len = torch.empty(bc.value + 1, dtype=torch.int32, device=device)
        self.block_stats = torch.empty(3 * (bc.value + 1), dtype=torch.int16, device=device)
        self.bloom = torch.empty(fc.value, dtype=torch.uint8, device=device)
        self.summary = torch.zeros(C.sizeof(_abi.SstSummary), dtype=torch.uint8, device=device)
        self.workspace = None
        if workspace:  # own scratch for sdb_encode_sst (a set shares one, see encode_ssts_device)
            ws = lib().sdb_encode_workspace_bytes(n, C.byref(prm))
            self.workspace = torch.empty(max(ws, 256), dtype=torch.uint8, device=device)
        self.out = _abi.SstOut(self.data.data_ptr(), dc.value, self.block_off.data_ptr(),
                               self.block_first.data_ptr(), self.index_key_len.data_ptr(),
                               self.block_stats.data_ptr(), bc.value, self.bloom.data_ptr(), fc.value,
                               self.summary.data_ptr())

    def summary_host(self):
        raw = self.summary.cpu().numpy().tobytes()
        return _abi.SstSummary.from_buffer_copy(raw)

    def to_host(self):
        sm = self.summary_host()
        nb = sm.num_blocks
        r = {
            "summary": sm,
            "data": self.data[:sm.data_len].cpu().numpy(),
            "block_off": self.block_off[:nb + 1].cpu().numpy().view(np.uint64),
            "block_first_entry": self.block_first[:nb + 1].cpu().numpy().view(np.uint32),
            "index_key_len": self.index_key_len[:nb].cpu().numpy().view(np.uint32),
            "block_stats": self.block_stats[:3 * nb].cpu().numpy().view(np.uint16).reshape(-1, 3),
            "bloom": self.bloom[:sm.bloom_len].cpu().numpy(),
        }
        return r


def encode_sst_device(dbatch, out, stream=None):
    """Enqueue one SST encode (device batch -> device outputs) on `stream` (torch stream or None)."""
    sp = None
    if stream is not None:
        sp = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    kb = dbatch.to_ctypes()
    st = lib().sdb_encode_sst(C.byref(kb), C.byref(out.params), C.byref(out.out), out.workspace.data_ptr(),
                              out.workspace.numel(), sp)
    if st:
        raise SdbError(st, "sdb_encode_sst")


def ssts_workspace(dbatches, prm, device="cuda"):
    """Scratch for sdb_encode_ssts over these device batches (sdb_encode_ssts_workspace_bytes)."""
    import torch
    kbs = (_abi.KvBatch * max(len(dbatches), 1))(*[b.to_ctypes() for b in dbatches])
    n = lib().sdb_encode_ssts_workspace_bytes(len(dbatches), kbs, C.byref(prm))
    return torch.empty(max(n, 256), dtype=torch.uint8, device=device)


def encode_ssts_device(dbatches, outs, prm, workspace, stream=None):
    """Enqueue the encode of several independent SSTs (same params) as ONE launch sequence
    (sdb_encode_ssts): outs[i] receives batches[i]."""
    assert len(dbatches) == len(outs)
    sp = None
    if stream is not None:
        sp = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    kbs = (_abi.KvBatch * max(len(dbatches), 1))(*[b.to_ctypes() for b in dbatches])
    os_ = (_abi.SstOut * max(len(outs), 1))(*[o.out for o in outs])
    st = lib().sdb_encode_ssts(len(dbatches), kbs, C.byref(prm), os_, workspace.data_ptr(), workspace.numel(), sp)
    if st:
        raise SdbError(st, "sdb_encode_ssts")


class DeviceDecodeOutput:
    """Caller-owned device outputs + workspace for sdb_decode_blocks / sdb_decode_blocks_at."""

    def __init__(self, nblocks, cap_entries, key_cap, device="cuda"):
        import torch
        o = lambda n, dt: torch.empty(max(n, 1), dtype=dt, device=device)
        self.nblocks = nblocks
        self.block_entry_start = o(nblocks + 1, torch.int64)
        self.key_arena = o(key_cap + 16, torch.uint8)
        self.key_off = o(cap_entries + 1, torch.int64)
        self.val_off = o(cap_entries, torch.int64)
        self.val_len = o(cap_entries, torch.int32)
        self.seq = o(cap_entries, torch.int64)
        self.flags = o(cap_entries, torch.uint8)
        self.create_ts = o(cap_entries, torch.int64)
        self.expire_ts = o(cap_entries, torch.int64)
        self.bad_block = o(nblocks + 1, torch.int32)
        self.summary = torch.zeros(64, dtype=torch.uint8, device=device)
        self.out = _abi.DecodedOut(self.block_entry_start.data_ptr(), self.key_arena.data_ptr(), key_cap,
                                   self.key_off.data_ptr(), self.val_off.data_ptr(), self.val_len.data_ptr(),
                                   self.seq.data_ptr(), self.flags.data_ptr(), self.create_ts.data_ptr(),
                                   self.expire_ts.data_ptr(), cap_entries, self.bad_block.data_ptr(),
                                   nblocks + 1, self.summary.data_ptr())
        wsb = lib().sdb_decode_workspace_bytes(nblocks)
        self.workspace = torch.empty(max(wsb, 256), dtype=torch.uint8, device=device)

    def summary_host(self):
        return _abi.DecodeSummary.from_buffer_copy(self.summary.cpu().numpy().tobytes()[:C.sizeof(_abi.DecodeSummary)])

    def to_host(self):
        """A Decoded with the same fields as Decoder.decode (numpy)."""
        sm = self.summary_host()
        d = Decoded()
        d.status = sm.status
        d.summary = {f: getattr(sm, f) for f, _ in _abi.DecodeSummary._fields_}
        n = sm.num_entries if sm.status in (0, 3, 4, 9) else 0
        d.n = n
        v = lambda t, k, dt: t[:k].cpu().numpy().view(dt)
        d.block_entry_start = v(self.block_entry_start, self.nblocks + 1, np.uint64)
        d.key_off = v(self.key_off, n + 1, np.uint64)
        d.key_arena = v(self.key_arena, sm.key_bytes, np.uint8)
        d.val_off = v(self.val_off, n, np.uint64)
        d.val_len = v(self.val_len, n, np.uint32)
        d.seq = v(self.seq, n, np.uint64)
        d.flags = v(self.flags, n, np.uint8)
        d.create_ts = v(self.create_ts, n, np.int64)
        d.expire_ts = v(self.expire_ts, n, np.int64)
        d.bad_block = v(self.bad_block, min(sm.num_bad_blocks, self.nblocks + 1), np.uint32)
        return d


def decode_blocks_at_device(arena, block_start, block_end, nblocks, out, sst_version=2, stream=None):
    """Enqueue sdb_decode_blocks_at: blocks at arbitrary places of one device arena (torch tensors)."""
    sp = None
    if stream is not None:
        sp = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    st = lib().sdb_decode_blocks_at(arena.data_ptr(), block_start.data_ptr(), block_end.data_ptr(), nblocks,
                                    sst_version, C.byref(out.out), out.workspace.data_ptr(), out.workspace.numel(), sp)
    if st:
        raise SdbError(st, "sdb_decode_blocks_at")


def decode_blocks_ex_device(arena, block_start, block_end, nblocks, out, sst_version=2, descending=False, stream=None,
                            fail_fast=False):
    """Enqueue sdb_decode_blocks_ex (block_end None: contiguous blocks, block_start has nblocks + 1 entries).
    fail_fast: read_blocks semantics (SDB_DECODE_FAIL_FAST: columns unspecified when the call fails)."""
    flags = (_abi.DECODE_DESCENDING if descending else 0) | (_abi.DECODE_FAIL_FAST if fail_fast else 0)
    st = lib().sdb_decode_blocks_ex(arena.data_ptr(), block_start.data_ptr(),
                                    None if block_end is None else block_end.data_ptr(), nblocks, sst_version, flags,
                                    C.byref(out.out), out.workspace.data_ptr(), out.workspace.numel(), _sp(stream))
    if st:
        raise SdbError(st, "sdb_decode_blocks_ex")


def decompress_blocks_device(codec, blocks, block_off, stream=None):
    """Compressed blocks -> a plain block run (sdb_decompress_plan + sdb_decompress_blocks; the first half
    of decode_block, format/sst.rs:980-999).  blocks: device u8 tensor, block_off: device int64 tensor of
    nblocks + 1.  Synchronises once to size the output.  Returns (out, out_start, out_end, err) device
    tensors (err: block << 8 | status of the first failing block, ~0 none) — decode them with
    decode_blocks_at_device(out, out_start, out_end, ...)."""
    import torch
    dev = blocks.device
    nb = block_off.numel() - 1
    sp = _sp(stream)
    ws = torch.empty(int(lib().sdb_decompress_workspace_bytes(nb)), dtype=torch.uint8, device=dev)
    out_start = torch.empty(nb + 1, dtype=torch.int64, device=dev)
    st = lib().sdb_decompress_plan(codec, blocks.data_ptr(), block_off.data_ptr(), nb, out_start.data_ptr(),
                                   ws.data_ptr(), ws.numel(), sp)
    if st:
        raise SdbError(st, "sdb_decompress_plan")
    if stream is not None and hasattr(stream, "synchronize"):
        stream.synchronize()
    else:
        torch.cuda.synchronize(dev)
    total = int(out_start[nb].item())
    out = torch.empty(max(total, 1) + 16, dtype=torch.uint8, device=dev)
    out_end = torch.empty(max(nb, 1), dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    st = lib().sdb_decompress_blocks(codec, blocks.data_ptr(), block_off.data_ptr(), nb, out.data_ptr(), total,
                                     out_start.data_ptr(), out_end.data_ptr(), err.data_ptr(), sp)
    if st:
        raise SdbError(st, "sdb_decompress_blocks")
    return out, out_start, out_end[:nb], err


def decompress_blocks_once_device(codec, blocks, block_off, slot_bytes, out_cap=None, stream=None, out=None):
    """sdb_decompress_blocks_once: decompress_blocks_device without the host synchronisation between the plan
    and the run.  Zlib inflates every block once into a slot of slot_bytes and re-plans only the blocks that
    overflowed theirs (packed after the slots; out_start then is not monotone, out_start[nblocks] = the bytes
    used); the other codecs run plan + run back to back.  out_cap defaults to nblocks * slot_bytes plus the
    compressed section's length * 8 for overflows.  Returns (out, out_start, out_end, err) as
    decompress_blocks_device."""
    import torch
    dev = blocks.device
    nb = block_off.numel() - 1
    if out_cap is None:
        out_cap = nb * slot_bytes + 8 * int(blocks.numel()) + 64
    ws = torch.empty(int(lib().sdb_decompress_once_workspace_bytes(nb)), dtype=torch.uint8, device=dev)
    if out is None:
        out = torch.empty(max(out_cap, 1) + 16, dtype=torch.uint8, device=dev)
    out_start = torch.empty(nb + 1, dtype=torch.int64, device=dev)
    out_end = torch.empty(max(nb, 1), dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    st = lib().sdb_decompress_blocks_once(codec, blocks.data_ptr(), block_off.data_ptr(), nb, slot_bytes,
                                          out.data_ptr(), out_cap, out_start.data_ptr(), out_end.data_ptr(),
                                          err.data_ptr(), ws.data_ptr(), ws.numel(), _sp(stream))
    if st:
        raise SdbError(st, "sdb_decompress_blocks_once")
    return out, out_start, out_end[:nb], err


def compress_blocks_device(codec, blocks, block_off, in_bytes=None, out_cap=None, stream=None):
    """An encoded data section -> the same blocks compressed (sdb_compress_blocks; compress_and_transform,
    format/sst.rs:525-594).  blocks: device u8 tensor, block_off: device int64 tensor of nblocks + 1.
    Returns (out, out_off, err) device tensors; out_off[nblocks] = the compressed section's length."""
    import torch
    dev = blocks.device
    nb = block_off.numel() - 1
    if in_bytes is None:
        in_bytes = int(block_off[nb].item() - block_off[0].item()) if nb else 0
    if out_cap is None:
        out_cap = in_bytes + in_bytes // 8 + 64 * (nb + 1)
    ws = torch.empty(int(lib().sdb_compress_workspace_bytes(nb, in_bytes)), dtype=torch.uint8, device=dev)
    out = torch.empty(max(out_cap, 1) + 16, dtype=torch.uint8, device=dev)
    out_off = torch.empty(nb + 1, dtype=torch.int64, device=dev)
    err = torch.empty(1, dtype=torch.int64, device=dev)
    st = lib().sdb_compress_blocks(codec, blocks.data_ptr(), block_off.data_ptr(), nb, in_bytes, out.data_ptr(), out_cap,
                                   out_off.data_ptr(), err.data_ptr(), ws.data_ptr(), ws.numel(), _sp(stream))
    if st:
        raise SdbError(st, "sdb_compress_blocks")
    return out, out_off, err


LOOKUP_FIELDS = (("state", "uint8"), ("status", "int32"), ("block", "int32"), ("entry", "int32"),
                 ("key_len", "int32"), ("val_off", "int64"), ("val_len", "int32"), ("seq", "int64"),
                 ("flags", "uint8"), ("create_ts", "int64"), ("expire_ts", "int64"))


def sst_lookup_device(view_tensors, key_bytes, key_off, nkeys, descending=False, stream=None):
    """sdb_sst_lookup over device tensors.  view_tensors: dict with data, block_off, index_keys,
    index_key_off (torch device tensors), num_blocks, sst_version and optionally bloom (device
    tensor) + num_probes.  Returns a dict of device result tensors (LOOKUP_FIELDS)."""
    import torch
    dev = key_bytes.device
    vt = view_tensors
    bloom = vt.get("bloom")
    v = _abi.SstView(vt["data"].data_ptr(), vt["block_off"].data_ptr(), vt["num_blocks"],
                     vt["index_keys"].data_ptr(), vt["index_key_off"].data_ptr(),
                     bloom.data_ptr() if bloom is not None else None,
                     int(vt.get("bloom_len", 0)) if bloom is not None else 0, int(vt.get("num_probes", 0)),
                     int(vt.get("sst_version", 2)), 0)
    res = {f: torch.zeros(max(nkeys, 1), dtype=getattr(torch, dt), device=dev) for f, dt in LOOKUP_FIELDS}
    out = _abi.LookupOut(*[res[f].data_ptr() for f, _ in LOOKUP_FIELDS])
    wsb = lib().sdb_sst_lookup_workspace_bytes(vt["num_blocks"], nkeys)
    ws = torch.empty(wsb, dtype=torch.uint8, device=dev)
    sp = None
    if stream is not None:
        sp = stream.cuda_stream if hasattr(stream, "cuda_stream") else stream
    st = lib().sdb_sst_lookup(C.byref(v), key_bytes.data_ptr(), key_off.data_ptr(), nkeys, int(bool(descending)),
                              C.byref(out), ws.data_ptr(), wsb, sp)
    if st:
        raise SdbError(st, "sdb_sst_lookup")
    res["_ws"] = ws
    return res


# ------------------------------------------------------------------------------------------------
# Compaction (sdb_merge_runs / sdb_sst_cuts / sdb_compactor_*)
# ------------------------------------------------------------------------------------------------
def _sync(stream, dev):
    """Wait for work queued on `stream` (a torch stream, a raw handle or None) before a host read."""
    import torch
    if stream is not None and hasattr(stream, "synchronize"):
        stream.synchronize()
    else:
        torch.cuda.synchronize(dev)  # device-wide: covers a raw stream handle too


def _sp(stream):
    if stream is None:
        return None
    return stream.cuda_stream if hasattr(stream, "cuda_stream") else stream


_hip = None


def _d2h(ptr, nbytes):
    """Copy nbytes at a raw device pointer to a host numpy uint8 array (hipMemcpy D2H)."""
    global _hip
    if _hip is None:
        _hip = C.CDLL("libamdhip64.so")
        _hip.hipMemcpy.argtypes = [C.c_void_p, C.c_void_p, C.c_size_t, C.c_int]
        _hip.hipMemcpy.restype = C.c_int
    out = np.empty(max(nbytes, 1), np.uint8)
    if nbytes:
        st = _hip.hipMemcpy(out.ctypes.data, ptr, nbytes, 2)
        if st:
            raise SdbError(_abi.SDB_DEVICE_ERROR, "hipMemcpy D2H")
    return out[:nbytes]


class DeviceRun:
    """A sorted run on the device in the sdb_run layout (torch tensors)."""

    def __init__(self, n, key_arena, key_off, val_base, val_off, val_len, seq, flags, create_ts, expire_ts,
                 key_bytes, val_bytes):
        self.n = n
        self.t = (key_arena, key_off, val_base, val_off, val_len, seq, flags, create_ts, expire_ts)
        self.key_bytes, self.val_bytes = key_bytes, val_bytes

    @classmethod
    def from_host(cls, run, device="cuda"):
        import torch
        up = lambda a: torch.from_numpy(np.concatenate([np.ascontiguousarray(a).view(np.uint8),
                                                        np.zeros(16, np.uint8)])).to(device)
        return cls(run.n, up(run.key_arena), up(run.key_off), up(run.val_base), up(run.val_off), up(run.val_len),
                   up(run.seq), up(run.flags), up(run.create_ts), up(run.expire_ts),
                   int(run.key_off[-1]) if run.n else 0, int(run.val_len.sum()))

    @classmethod
    def from_decoded(cls, dout, blocks, n):
        """A DeviceDecodeOutput of `n` entries whose values live in the `blocks` device tensor."""
        sm = dout.summary_host()
        vb = int(dout.val_len[:n].to(dtype=__import__("torch").int64).sum().item()) if n else 0
        return cls(n, dout.key_arena, dout.key_off, blocks, dout.val_off, dout.val_len, dout.seq, dout.flags,
                   dout.create_ts, dout.expire_ts, int(sm.key_bytes), vb)

    def to_ctypes(self):
        return _abi.Run(self.n, *[t.data_ptr() for t in self.t])


def merge_runs_device(druns, ret, stream=None):
    """sdb_merge_runs over DeviceRuns -> (dict of device tensors of the merged batch, MergeSummary)."""
    import torch
    dev = druns[0].t[0].device if druns else "cuda"
    total = sum(r.n for r in druns)
    kcap = sum(r.key_bytes for r in druns)
    vcap = sum(r.val_bytes for r in druns)
    e = lambda k, dt: torch.empty(max(k, 1), dtype=dt, device=dev)
    o = {"key_bytes": e(kcap + 16, torch.uint8), "key_off": e(total + 1, torch.int64),
         "val_bytes": e(vcap + 16, torch.uint8), "val_off": e(total + 1, torch.int64),
         "kind": e(total, torch.uint8), "seq": e(total, torch.int64), "create_ts": e(total, torch.int64),
         "expire_ts": e(total, torch.int64), "ts_mask": e(total, torch.uint8),
         "summary": torch.zeros(C.sizeof(_abi.MergeSummary), dtype=torch.uint8, device=dev)}
    out = _abi.MergedOut(o["key_bytes"].data_ptr(), kcap, o["key_off"].data_ptr(), o["val_bytes"].data_ptr(), vcap,
                         o["val_off"].data_ptr(), o["kind"].data_ptr(), o["seq"].data_ptr(), o["create_ts"].data_ptr(),
                         o["expire_ts"].data_ptr(), o["ts_mask"].data_ptr(), total, o["summary"].data_ptr())
    cr = (_abi.Run * max(len(druns), 1))(*[r.to_ctypes() for r in druns])
    wsb = lib().sdb_merge_runs_workspace_bytes(cr, len(druns))
    ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
    st = lib().sdb_merge_runs(cr, len(druns), C.byref(ret), C.byref(out), ws.data_ptr(), ws.numel(), _sp(stream))
    if st:
        raise SdbError(st, "sdb_merge_runs")
    _sync(stream, dev)
    sm = _abi.MergeSummary.from_buffer_copy(o["summary"].cpu().numpy().tobytes())
    o["_ws"] = ws
    return o, sm


def merged_to_host(o, sm):
    from .batch import Batch
    n = sm.num_out
    v = lambda k, m, dt: o[k][:m].cpu().numpy().view(dt)
    return Batch(v("key_bytes", sm.key_bytes, np.uint8), v("key_off", n + 1, np.uint64),
                 v("val_bytes", sm.val_bytes, np.uint8), v("val_off", n + 1, np.uint64), v("kind", n, np.uint8),
                 v("seq", n, np.uint64), v("create_ts", n, np.int64), v("expire_ts", n, np.int64),
                 v("ts_mask", n, np.uint8))


def sst_cuts_device(dbatch, prm, max_sst_size, stream=None):
    """sdb_sst_cuts over a device batch -> list of SST start entries + [n] (synchronises)."""
    import torch
    n = dbatch.n
    dev = dbatch.key_bytes.device if hasattr(dbatch, "key_bytes") else "cuda"
    cut = torch.zeros(n + 2, dtype=torch.int64, device=dev)
    num = torch.zeros(1, dtype=torch.int64, device=dev)
    wsb = lib().sdb_sst_cuts_workspace_bytes(n, C.byref(prm))
    ws = torch.empty(max(wsb, 256), dtype=torch.uint8, device=dev)
    kb = dbatch.to_ctypes()
    st = lib().sdb_sst_cuts(C.byref(kb), C.byref(prm), max_sst_size, cut.data_ptr(), n + 1, num.data_ptr(),
                            ws.data_ptr(), ws.numel(), _sp(stream))
    if st:
        raise SdbError(st, "sdb_sst_cuts")
    _sync(stream, dev)
    ns = int(num.item())
    return [int(x) for x in cut[:ns + 1].cpu().numpy()] if ns else []


class Compactor:
    """sdb_compactor_*: one compaction job (merge + retention + cuts + encode) per run()."""

    def __init__(self, device=0):
        require_device()
        self.h = lib().sdb_compactor_create(device)
        if not self.h:
            raise SdbError(_abi.SDB_DEVICE_ERROR, "sdb_compactor_create")

    def run(self, druns, ret, prm, max_sst_size, stream=None):
        cr = (_abi.Run * max(len(druns), 1))(*[r.to_ctypes() for r in druns])
        ns = C.c_uint32(0)
        st = lib().sdb_compactor_run(self.h, cr, len(druns), C.byref(ret), C.byref(prm), max_sst_size, _sp(stream),
                                     C.byref(ns))
        self.status = st
        return st, ns.value

    def run_ssts(self, inputs, ret, prm, max_sst_size, input_version=2, run_start=None, stream=None):
        """sdb_compactor_run_ssts: the job from encoded input SSTs (decode included).  inputs: objects with
        .data / .block_off (device tensors: the data section, block_off u64[num_blocks + 1]) and the
        SstStats counts .num_entries / .key_bytes / .val_bytes; run_start: inputs of each sorted run."""
        ci = (_abi.CompactionInput * max(len(inputs), 1))(*[
            _abi.CompactionInput(x.data.data_ptr(), x.block_off.data_ptr(), x.block_off.numel() - 1, x.num_entries,
                                 x.key_bytes, x.val_bytes) for x in inputs])
        rs = None
        nruns = len(inputs)
        if run_start is not None:
            rs = (C.c_uint32 * len(run_start))(*run_start)
            nruns = len(run_start) - 1
        ns = C.c_uint32(0)
        st = lib().sdb_compactor_run_ssts(self.h, ci, len(inputs), rs, nruns, input_version, C.byref(ret), C.byref(prm),
                                          max_sst_size, _sp(stream), C.byref(ns))
        self.status = st
        return st, ns.value

    def merged(self):
        kb, sm = _abi.KvBatch(), _abi.MergeSummary()
        st = lib().sdb_compactor_merged(self.h, C.byref(kb), C.byref(sm))
        if st:
            raise SdbError(st, "sdb_compactor_merged")
        from .batch import Batch
        n = kb.n
        if not n:
            return Batch(np.zeros(0, np.uint8), np.zeros(1, np.uint64), np.zeros(0, np.uint8), np.zeros(1, np.uint64),
                         np.zeros(0, np.uint8), np.zeros(0, np.uint64), np.zeros(0, np.int64), np.zeros(0, np.int64),
                         np.zeros(0, np.uint8)), sm
        g = lambda p, k, dt: _d2h(p, k * np.dtype(dt).itemsize).view(dt)
        return Batch(g(kb.key_bytes, sm.key_bytes, np.uint8), g(kb.key_off, n + 1, np.uint64),
                     g(kb.val_bytes, sm.val_bytes, np.uint8), g(kb.val_off, n + 1, np.uint64), g(kb.kind, n, np.uint8),
                     g(kb.seq, n, np.uint64), g(kb.create_ts, n, np.int64), g(kb.expire_ts, n, np.int64),
                     g(kb.ts_mask, n, np.uint8)), sm

    def sst(self, i):
        """SST i of the last run as host arrays (the fields of DeviceSstOutput.to_host) + entry range."""
        v = _abi.CompactedSst()
        st = lib().sdb_compactor_sst(self.h, i, C.byref(v))
        if st:
            raise SdbError(st, "sdb_compactor_sst")
        sm = v.summary
        nb = sm.num_blocks
        g = lambda p, k, dt: _d2h(p, k * np.dtype(dt).itemsize).view(dt)
        return {"summary": sm, "entry_start": v.entry_start, "entry_end": v.entry_end,
                "data": g(v.data, sm.data_len, np.uint8), "block_off": g(v.block_off, nb + 1, np.uint64),
                "block_first_entry": g(v.block_first_entry, nb + 1, np.uint32),
                "index_key_len": g(v.index_key_len, nb, np.uint32),
                "block_stats": g(v.block_stats, 3 * nb, np.uint16).reshape(-1, 3),
                "bloom": g(v.bloom, sm.bloom_len, np.uint8)}

    def close(self):
        if getattr(self, "h", None):
            lib().sdb_compactor_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass
