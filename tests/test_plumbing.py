"""configs[0] — the plumbing round trip on the CPU (SURVEY.md §8(d) "Config 1").

The reference's bencher writes SSTs through the DB into an object store and reads them back
(`slatedb-bencher`, `compaction_execute_bench.rs:84-86,168-177`); that harness needs cargo and an
object store, so this is its counterpart over the same formats:

  write:  D1-shaped batches -> CPU encode (oracle: EncodedSsTableBuilder restated) -> SST footer
          (`sdb_sst_footer`, host code of the product library) -> an in-memory object map
          (path -> bytes, standing in for object_store `put`, `tablestore.rs` write_sst)
  read:   ranged GETs only — the 10-byte tail (meta offset + version), the SsTableInfo, the index
          (`format/sst.rs:600-760` read_info / read_index), then the data blocks grouped into
          `read_blocks` ranges of at most 2 MiB (`format/sst.rs:938-978`, `config.rs:1323-1337`)
  decode: every range -> validate_checksum -> DataBlockIterator (oracle decode), and the iterated
          rows must equal the written batch (key, value, seq, kind) in order.

Test infrastructure (it runs the oracle, never the device); `python -m tests.test_plumbing` times the
full-size round trip on one thread and prints one JSON line.
"""
import json
import struct
import time
import zlib

import numpy as np

from oracle import footer as F
from oracle import oracle as O
from slatedb_amd import _abi, datasets, runtime

READ_RANGE = 2 << 20  # object_store_cache_part_size_bytes / read_blocks range (config.rs:1323-1337)


class ObjectMap:
    """object_store::memory::InMemory stand-in: whole-object put, ranged get, byte accounting."""

    def __init__(self):
        self.objs, self.gets, self.bytes_read = {}, 0, 0

    def put(self, path, data):
        self.objs[path] = bytes(data)

    def size(self, path):
        return len(self.objs[path])

    def get_range(self, path, lo, hi):
        self.gets += 1
        self.bytes_read += hi - lo
        return self.objs[path][lo:hi]


def _unck(b):
    assert struct.unpack(">I", b[-4:])[0] == zlib.crc32(b[:-4]), "checksum mismatch"
    return b[:-4]


def write_ssts(store, batches, prm):
    for j, b in enumerate(batches):
        r = O.encode_sst(b, prm)
        assert r.status == 0, _abi.STATUS_NAMES.get(r.status)
        store.put("compacted/%06d.sst" % j, runtime.sst_object(b, r, prm.sst_version))


def read_sst(store, path, version=2):
    """read_info -> read_index -> read_blocks in <= 2 MiB ranges -> decode; returns the rows."""
    size = store.size(path)
    tail = store.get_range(path, size - 10, size)
    assert struct.unpack(">H", tail[8:])[0] == version
    meta = struct.unpack(">Q", tail[:8])[0]
    info = F.parse_info(_unck(store.get_range(path, meta, size - 10)))
    io, il = info["index_offset"], info["index_len"]
    index = F.parse_index(_unck(store.get_range(path, io, io + il)))
    offs = [o for o, _ in index] + [info["filter_offset"] if info["filter_len"] else io]
    rows = []
    b = 0
    while b < len(index):  # group consecutive blocks into one ranged GET of at most READ_RANGE bytes
        e = b + 1
        while e < len(index) and offs[e + 1] - offs[b] <= READ_RANGE:
            e += 1
        data = np.frombuffer(store.get_range(path, offs[b], offs[e]), np.uint8)
        bo = np.array(offs[b:e + 1], np.uint64) - np.uint64(offs[b])
        d = O.decode_blocks(data, bo, version)
        assert d.status == 0 and d.summary.num_bad_blocks == 0
        rows.append((d, data))
        b = e
    return rows


def check_rows(batch, rows):
    """Iterated rows == the written batch, in order (keys, values, seq, kind)."""
    i = 0
    for d, data in rows:
        ko = d.key_off.astype(np.int64)
        keys = d.key_arena
        for q in range(d.n):
            assert keys[ko[q]:ko[q + 1]].tobytes() == batch.key(i)
            vo, vl = int(d.val_off[q]), int(d.val_len[q])
            assert data[vo:vo + vl].tobytes() == batch.value(i)
            assert int(d.seq[q]) == (0 if batch.seq is None else int(batch.seq[i]))
            kind = 0 if batch.kind is None else int(batch.kind[i])
            fl = int(d.flags[q])  # RowFlags (format/row.rs): kind -> TOMBSTONE / MERGE_OPERAND bits
            assert bool(fl & _abi.FLAG_TOMBSTONE) == (kind == _abi.KIND_TOMBSTONE)
            assert bool(fl & _abi.FLAG_MERGE_OPERAND) == (kind == _abi.KIND_MERGE)
            i += 1
    assert i == batch.n


def round_trip(batches, prm):
    store = ObjectMap()
    t0 = time.perf_counter()
    write_ssts(store, batches, prm)
    t1 = time.perf_counter()
    for j, b in enumerate(batches):
        check_rows(b, read_sst(store, "compacted/%06d.sst" % j, prm.sst_version))
    t2 = time.perf_counter()
    return store, t1 - t0, t2 - t1


def test_plumbing_round_trip_small():
    prm = O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    batches = [datasets.d1(sst_index=j, n=20000) for j in range(3)]
    store, _, _ = round_trip(batches, prm)
    assert len(store.objs) == 3
    # 20,000 x 116 B logical -> ~2.3 MB of blocks per SST: more than one 2 MiB ranged GET each
    assert store.gets >= 3 * 4


def test_plumbing_mixed_kinds_v1():
    prm = O.params(block_size=1024, sst_version=1, bloom_bits_per_key=10)
    b = datasets.d3(n=3000)
    store, _, _ = round_trip([b], prm)
    assert store.bytes_read < store.size("compacted/000000.sst")  # the filter is never fetched


def main():
    import argparse
    p = argparse.ArgumentParser()
    p.add_argument("--ssts", type=int, default=4)
    a = p.parse_args()
    prm = O.params(block_size=4096, sst_version=2, bloom_bits_per_key=10)
    batches = [datasets.d1(sst_index=j) for j in range(a.ssts)]
    logical = sum(b.logical_bytes() for b in batches)
    round_trip([datasets.d1(sst_index=99, n=1000)], prm)  # load both libraries outside the timing
    store, tw, tr = round_trip(batches, prm)
    print(json.dumps({"what": "configs[0] plumbing round trip (CPU, 1 thread): encode -> footer -> object map -> "
                              "ranged read_blocks (<= 2 MiB) -> decode -> row equality",
                      "ssts": a.ssts, "logical_bytes": logical, "object_bytes": sum(map(len, store.objs.values())),
                      "ranged_gets": store.gets, "write_s": round(tw, 3), "read_check_s": round(tr, 3),
                      "write_GiB_per_s": round(logical / tw / 2**30, 3)}), flush=True)


if __name__ == "__main__":
    main()
