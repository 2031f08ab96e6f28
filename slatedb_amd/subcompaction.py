"""Subcompactions: one compaction split by key range over GPUs.

The reference splits a logical compaction into disjoint key ranges that run in parallel
(slatedb/src/subcompaction.rs): each input SST's block index is sampled into at most 128 weighted
anchors (block first key, on-disk bytes of the block group; `sample_anchors`, :268-316), the anchors of
all inputs are swept in key order and a boundary opens a new range each time the bytes of the closed
ranges reach the next multiple of max(total / max_subcompactions, largest input SST)
(`select_boundaries`, :186-257; `plan_subcompaction_ranges`, :97-171).  The ranges cover the key space:
(-inf, b1), [b1, b2), ..., [bk, +inf).

Here the planner is host code over the same metadata this repo's footer writes (block first keys =
index keys, BlockMeta offsets, the data section's end), and a subcompaction is a compaction of every
input run cut to its range (`slice_run`: a binary search on the run's sorted keys; runs are views, nothing
is copied).  Range r goes to rank r mod N (the same dealing as job.assign for SSTs), each rank runs its
ranges through its own sdb_compactor, and there is no collective on the data path: the ranges are
independent, and their outputs concatenate to the unsplit compaction's merged stream (the retention
filter sees every version of a key inside one range, since a key never straddles a boundary).
"""
import numpy as np

from .batch import Run

MAX_ANCHORS_PER_SST = 128  # subcompaction.rs:81-86


class KeyRange:
    """[start, end): start None = unbounded below, end None = unbounded above (BytesRange)."""
    __slots__ = ("start", "end")

    def __init__(self, start=None, end=None):
        self.start, self.end = start, end

    def contains(self, key):
        return (self.start is None or key >= self.start) and (self.end is None or key < self.end)

    def __eq__(self, o):
        return isinstance(o, KeyRange) and (self.start, self.end) == (o.start, o.end)

    def __repr__(self):
        return "KeyRange(%r, %r)" % (self.start, self.end)


UNBOUNDED = KeyRange()


def sample_anchors(first_keys, offsets, data_end_offset, max_anchors=MAX_ANCHORS_PER_SST, effective_range=None):
    """An SST's block index -> [(group first key, bytes of the group)] (subcompaction.rs:268-316): blocks
    grouped by ceil(nblocks / max_anchors); a block ends at the next block's offset, the last one at the end
    of the data section; anchors outside `effective_range` dropped."""
    nb = len(first_keys)
    if nb == 0:
        return []
    max_anchors = max(int(max_anchors), 1)
    stride = -(-nb // max_anchors)
    out = []
    for b in range(0, nb, stride):
        g_end = min(b + stride, nb)
        end = int(offsets[g_end]) if g_end < nb else int(data_end_offset)
        nbytes = max(end - int(offsets[b]), 0)
        key = bytes(first_keys[b])
        if effective_range is None or effective_range.contains(key):
            out.append((key, nbytes))
    return out


def select_boundaries(anchors, max_subcompactions, min_range_bytes):
    """Covering ranges with roughly equal input bytes (subcompaction.rs:186-257)."""
    if max_subcompactions <= 1:
        return [UNBOUNDED]
    total = sum(b for _, b in anchors)
    target = max(total // max_subcompactions, min_range_bytes)
    if target == 0 or target >= total:
        return [UNBOUNDED]
    anchors = sorted(anchors, key=lambda a: a[0])
    first_key = anchors[0][0]
    boundaries = []
    threshold, cumulative = target, 0
    for key, nbytes in anchors:
        distinct = key > boundaries[-1] if boundaries else key > first_key
        if cumulative >= threshold and len(boundaries) < max_subcompactions - 1 and distinct:
            boundaries.append(key)
            threshold += target
        cumulative += nbytes
    if not boundaries:
        return [UNBOUNDED]
    ranges, start = [], None
    for b in boundaries:
        ranges.append(KeyRange(start, b))
        start = b
    ranges.append(KeyRange(start, None))
    return ranges


class SstMeta:
    """What the planner reads of one input SST: its index (block first keys, BlockMeta offsets), the end of
    the data section (filter_offset) and its size estimate (index_offset + index_len, db_state.rs:50-52)."""
    __slots__ = ("first_keys", "offsets", "data_len", "size")

    def __init__(self, first_keys, offsets, data_len, size=None):
        self.first_keys, self.offsets, self.data_len = list(first_keys), np.asarray(offsets), int(data_len)
        self.size = int(size) if size is not None else int(data_len)

    @classmethod
    def from_encoded(cls, batch, enc, footer_len=0):
        """From an encode result (oracle EncodedSst or a device output moved to the host): the index keys are
        each block's first key cut to its index-key length (compute_index_key)."""
        nb = len(enc.block_off) - 1
        starts = np.asarray(enc.block_first_entry[:nb], np.int64)
        ikl = np.asarray(enc.index_key_len[:nb], np.int64)
        keys = [batch.key(int(s))[:int(k)] for s, k in zip(starts, ikl)]
        data_len = int(enc.block_off[nb])
        return cls(keys, np.asarray(enc.block_off[:nb], np.uint64), data_len, data_len + footer_len)


def plan_subcompaction_ranges(ssts, max_subcompactions, max_anchors=MAX_ANCHORS_PER_SST):
    """subcompaction.rs:97-171: anchors of every input SST, floor = the largest input's size estimate."""
    if max_subcompactions <= 1:
        return [UNBOUNDED]
    min_range_bytes = max((s.size for s in ssts), default=0)
    anchors = []
    for s in ssts:
        anchors += sample_anchors(s.first_keys, s.offsets, s.data_len, max_anchors)
    return select_boundaries(anchors, max_subcompactions, min_range_bytes)


def assign_ranges(ranges, world):
    """Range r -> rank r mod world (job.assign's dealing): [[range index, ...] per rank]."""
    if world < 1:
        raise ValueError("world must be >= 1")
    return [list(range(r, len(ranges), world)) for r in range(world)]


def _key_index(run, key):
    """First entry of the sorted run whose key is >= key (binary search over the key arena)."""
    lo, hi = 0, run.n
    ko, arena = run.key_off, run.key_arena
    while lo < hi:
        mid = (lo + hi) // 2
        k = arena[int(ko[mid]):int(ko[mid + 1])].tobytes()
        if k < key:
            lo = mid + 1
        else:
            hi = mid
    return lo


def run_bounds(run, rng):
    """[lo, hi) entries of a sorted run inside the range."""
    lo = 0 if rng.start is None else _key_index(run, rng.start)
    hi = run.n if rng.end is None else _key_index(run, rng.end)
    return lo, max(lo, hi)


def slice_run(run, rng):
    """The entries of a sorted run inside the range, as a Run view (key offsets rebased to a sliced arena,
    value references unchanged)."""
    lo, hi = run_bounds(run, rng)
    k0, k1 = int(run.key_off[lo]), int(run.key_off[hi])
    return Run(run.key_arena[k0:k1], run.key_off[lo:hi + 1] - np.uint64(k0), run.val_base, run.val_off[lo:hi],
               run.val_len[lo:hi], run.seq[lo:hi], run.flags[lo:hi], run.create_ts[lo:hi], run.expire_ts[lo:hi])
