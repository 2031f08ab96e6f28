"""Columnar sorted-run batches (the input side of the C ABI, `sdb_kv_batch`).

A batch is the Arrow-style columnar form of a run of RowEntry (slatedb/src/types.rs:17-29):
entry i's key is key_bytes[key_off[i]:key_off[i+1]], likewise for values; kind is
ValueDeletable::{Value, Merge, Tombstone} = {0, 1, 2}; ts_mask bit0 = create_ts present,
bit1 = expire_ts present.  The same layout is used for host (numpy) and device (torch) buffers.
"""
import ctypes as C

import numpy as np

from . import _abi


class Batch:
    __slots__ = ("key_bytes", "key_off", "val_bytes", "val_off", "kind", "seq", "create_ts",
                 "expire_ts", "ts_mask", "prefix_len")

    def __init__(self, key_bytes, key_off, val_bytes, val_off, kind=None, seq=None,
                 create_ts=None, expire_ts=None, ts_mask=None, prefix_len=None):
        self.key_bytes = np.ascontiguousarray(key_bytes, dtype=np.uint8)
        self.key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
        self.val_bytes = np.ascontiguousarray(val_bytes, dtype=np.uint8)
        self.val_off = np.ascontiguousarray(val_off, dtype=np.uint64)
        self.kind = None if kind is None else np.ascontiguousarray(kind, dtype=np.uint8)
        self.seq = None if seq is None else np.ascontiguousarray(seq, dtype=np.uint64)
        self.create_ts = None if create_ts is None else np.ascontiguousarray(create_ts, dtype=np.int64)
        self.expire_ts = None if expire_ts is None else np.ascontiguousarray(expire_ts, dtype=np.int64)
        self.ts_mask = None if ts_mask is None else np.ascontiguousarray(ts_mask, dtype=np.uint8)
        self.prefix_len = None if prefix_len is None else np.ascontiguousarray(prefix_len, dtype=np.int32)
        n = len(self.key_off) - 1
        assert len(self.val_off) == n + 1, "val_off must have n+1 entries"
        for name in ("kind", "seq", "create_ts", "expire_ts", "ts_mask", "prefix_len"):
            a = getattr(self, name)
            assert a is None or len(a) == n, name

    @property
    def n(self):
        return len(self.key_off) - 1

    @classmethod
    def from_entries(cls, entries):
        """entries: iterable of (key, kind, value, seq, create_ts|None, expire_ts|None)."""
        entries = list(entries)
        n = len(entries)
        keys = [bytes(e[0]) for e in entries]
        vals = [b"" if e[1] == _abi.KIND_TOMBSTONE else bytes(e[2] or b"") for e in entries]
        key_off = np.zeros(n + 1, np.uint64)
        val_off = np.zeros(n + 1, np.uint64)
        key_off[1:] = np.cumsum([len(k) for k in keys], dtype=np.uint64) if n else []
        val_off[1:] = np.cumsum([len(v) for v in vals], dtype=np.uint64) if n else []
        kb = np.frombuffer(b"".join(keys), np.uint8) if n else np.zeros(0, np.uint8)
        vb = np.frombuffer(b"".join(vals), np.uint8) if n else np.zeros(0, np.uint8)
        kind = np.array([e[1] for e in entries], np.uint8)
        seq = np.array([e[3] for e in entries], np.uint64)
        cts = np.array([e[4] if e[4] is not None else 0 for e in entries], np.int64)
        ets = np.array([e[5] if e[5] is not None else 0 for e in entries], np.int64)
        mask = np.array([(e[4] is not None) * _abi.TS_CREATE + (e[5] is not None) * _abi.TS_EXPIRE
                         for e in entries], np.uint8)
        return cls(kb.copy(), key_off, vb.copy(), val_off, kind, seq, cts, ets, mask)

    def key(self, i):
        return self.key_bytes[int(self.key_off[i]):int(self.key_off[i + 1])].tobytes()

    def value(self, i):
        return self.val_bytes[int(self.val_off[i]):int(self.val_off[i + 1])].tobytes()

    def slice(self, lo, hi):
        """Entries [lo, hi) as a new batch (offsets rebased)."""
        ko, vo = self.key_off[lo:hi + 1], self.val_off[lo:hi + 1]
        kb = self.key_bytes[int(ko[0]):int(ko[-1])]
        vb = self.val_bytes[int(vo[0]):int(vo[-1])]
        pick = lambda a: None if a is None else a[lo:hi]
        return Batch(kb, ko - ko[0], vb, vo - vo[0], pick(self.kind), pick(self.seq),
                     pick(self.create_ts), pick(self.expire_ts), pick(self.ts_mask), pick(self.prefix_len))

    def logical_bytes(self):
        """Σ(|key| + |value|) — the headline GiB/s numerator."""
        return int(self.key_off[-1] - self.key_off[0]) + int(self.val_off[-1] - self.val_off[0])

    def algorithmic_input_bytes(self):
        """Σ(|k|+|v|+8+1+8·ts): SURVEY.md §8(d) input term."""
        n = self.n
        ts = 0
        if self.ts_mask is not None:
            ts = int(np.count_nonzero(self.ts_mask & 1) + np.count_nonzero(self.ts_mask & 2))
        return self.logical_bytes() + 9 * n + 8 * ts

    def to_ctypes(self):
        """Host-pointer sdb_kv_batch.  The numpy arrays must outlive the returned struct."""
        p = lambda a: None if a is None else a.ctypes.data
        return _abi.KvBatch(self.n, p(self.key_bytes), p(self.key_off), p(self.val_bytes),
                            p(self.val_off), p(self.kind), p(self.seq), p(self.create_ts),
                            p(self.expire_ts), p(self.ts_mask), p(self.prefix_len))

    def to_device(self, device="cuda"):
        return DeviceBatch(self, device)


class DeviceBatch:
    """The same batch resident in HBM (torch tensors as plain device allocations)."""

    def __init__(self, host, device="cuda"):
        import torch
        t = lambda a: None if a is None else torch.from_numpy(a.view(np.uint8)).to(device)
        self.n = host.n
        self.key_bytes = t(host.key_bytes) if host.key_bytes.size else torch.zeros(16, dtype=torch.uint8, device=device)
        self.key_off = t(host.key_off)
        self.val_bytes = t(host.val_bytes) if host.val_bytes.size else torch.zeros(16, dtype=torch.uint8, device=device)
        self.val_off = t(host.val_off)
        self.kind = t(host.kind)
        self.seq = t(host.seq)
        self.create_ts = t(host.create_ts)
        self.expire_ts = t(host.expire_ts)
        self.ts_mask = t(host.ts_mask)
        self.prefix_len = t(host.prefix_len)

    def to_ctypes(self):
        p = lambda a: None if a is None else a.data_ptr()
        return _abi.KvBatch(self.n, p(self.key_bytes), p(self.key_off), p(self.val_bytes),
                            p(self.val_off), p(self.kind), p(self.seq), p(self.create_ts),
                            p(self.expire_ts), p(self.ts_mask), p(self.prefix_len))


class Run:
    """A sorted input run of a compaction in the decoded layout (`sdb_run`): value i is
    val_base[val_off[i]:val_off[i] + val_len[i]], flags are RowFlags (row_codec_v2.rs:67-80)."""
    __slots__ = ("key_arena", "key_off", "val_base", "val_off", "val_len", "seq", "flags", "create_ts",
                 "expire_ts")

    def __init__(self, key_arena, key_off, val_base, val_off, val_len, seq, flags, create_ts, expire_ts):
        self.key_arena = np.ascontiguousarray(key_arena, dtype=np.uint8)
        self.key_off = np.ascontiguousarray(key_off, dtype=np.uint64)
        self.val_base = np.ascontiguousarray(val_base, dtype=np.uint8)
        self.val_off = np.ascontiguousarray(val_off, dtype=np.uint64)
        self.val_len = np.ascontiguousarray(val_len, dtype=np.uint32)
        self.seq = np.ascontiguousarray(seq, dtype=np.uint64)
        self.flags = np.ascontiguousarray(flags, dtype=np.uint8)
        self.create_ts = np.ascontiguousarray(create_ts, dtype=np.int64)
        self.expire_ts = np.ascontiguousarray(expire_ts, dtype=np.int64)

    @property
    def n(self):
        return len(self.key_off) - 1

    @classmethod
    def from_batch(cls, b):
        n = b.n
        kind = b.kind if b.kind is not None else np.zeros(n, np.uint8)
        mask = b.ts_mask if b.ts_mask is not None else np.zeros(n, np.uint8)
        flags = np.where(kind == _abi.KIND_TOMBSTONE, _abi.FLAG_TOMBSTONE,
                         np.where(kind == _abi.KIND_MERGE, _abi.FLAG_MERGE_OPERAND, 0)).astype(np.uint8)
        flags |= np.where(mask & _abi.TS_CREATE, _abi.FLAG_HAS_CREATE_TS, 0).astype(np.uint8)
        flags |= np.where(mask & _abi.TS_EXPIRE, _abi.FLAG_HAS_EXPIRE_TS, 0).astype(np.uint8)
        vlen = np.diff(b.val_off).astype(np.uint32)
        vlen[kind == _abi.KIND_TOMBSTONE] = 0
        zeros = np.zeros(n, np.int64)
        cts = b.create_ts if b.create_ts is not None else zeros
        ets = b.expire_ts if b.expire_ts is not None else zeros
        return cls(b.key_bytes, b.key_off, b.val_bytes, b.val_off[:n], vlen,
                   b.seq if b.seq is not None else np.zeros(n, np.uint64), flags, cts, ets)

    @classmethod
    def from_entries(cls, entries):
        return cls.from_batch(Batch.from_entries(entries))

    def to_ctypes(self):
        p = lambda a: a.ctypes.data if a.size else None
        return _abi.Run(self.n, p(self.key_arena), self.key_off.ctypes.data, p(self.val_base), p(self.val_off),
                        p(self.val_len), p(self.seq), p(self.flags), p(self.create_ts), p(self.expire_ts))
