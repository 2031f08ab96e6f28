"""Seeded synthetic sorted runs.  numpy-vectorised, deterministic across hosts.

PRNG: counter-based splitmix64, word i = mix64(seed + (i+1)·0x9E3779B97F4A7C15) — the sequential
splitmix64 stream written in closed form so it vectorises.

D1  "bench-ordered": mirrors slatedb's compaction bench loader (compaction_execute_bench.rs:158-187,
    bytes_generator.rs:32-47): a 12-byte big-endian counter starting at a seeded random value,
    suffixed with the 4-byte big-endian SST index; 100 random value bytes; seq 0; kind Value.
    N = floor(64 MiB / (16 + 100)) = 578,524.
D2  "random-sorted": N uniform random 16-byte keys, sorted, unique; 100-byte random values.
C4  bloom config: 10,000,000 uniform random 16-byte keys (seed 0x5EED0004), sorted.
"""
import numpy as np

from .batch import Batch

GAMMA = np.uint64(0x9E3779B97F4A7C15)
MIB64 = 64 * 1024 * 1024
D1_N = MIB64 // 116
SEED_D1 = 0x5EED0001
SEED_D2 = 0x5EED0002
SEED_C4 = 0x5EED0004


def splitmix64(seed, start, count):
    """Words [start, start+count) of the splitmix64 stream for `seed`."""
    with np.errstate(over="ignore"):
        i = np.arange(start + 1, start + count + 1, dtype=np.uint64)
        z = np.uint64(seed) + i * GAMMA
        z = (z ^ (z >> np.uint64(30))) * np.uint64(0xBF58476D1CE4E5B9)
        z = (z ^ (z >> np.uint64(27))) * np.uint64(0x94D049BB133111EB)
        return z ^ (z >> np.uint64(31))


def _be_bytes_u64(x):
    return x.astype(">u8").view(np.uint8).reshape(-1, 8)


def random_bytes(seed, start_word, nbytes):
    words = splitmix64(seed, start_word, (nbytes + 7) // 8)
    return words.view(np.uint8)[:nbytes].copy()


def d1(sst_index=0, n=D1_N, value_len=100, seed=SEED_D1, seq_desc=False):
    """D1 bench-ordered SST `sst_index` (distinct data per index, like the bench's per-SST suffix)."""
    s = seed + 0x1000003 * sst_index
    start = splitmix64(s, 0, 2)
    hi = np.uint64(int(start[0]) >> 32)          # top 32 bits of the 96-bit counter
    lo0 = start[1]                               # low 64 bits
    with np.errstate(over="ignore"):
        idx = np.arange(n, dtype=np.uint64)
        lo = lo0 + idx
        carry = (lo < lo0).astype(np.uint64)
        hiv = hi + carry
    keys = np.empty((n, 16), np.uint8)
    keys[:, 0:4] = hiv.astype(">u4").view(np.uint8).reshape(-1, 4)
    keys[:, 4:12] = _be_bytes_u64(lo)
    keys[:, 12:16] = np.frombuffer(np.uint32(sst_index).astype(">u4").tobytes(), np.uint8)
    stride = (value_len + 7) // 8 * 8
    vals = random_bytes(s, 2, n * stride).reshape(n, stride)[:, :value_len]
    key_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(16)
    val_off = np.arange(n + 1, dtype=np.uint64) * np.uint64(value_len)
    seq = (np.arange(n, 0, -1, dtype=np.uint64) if seq_desc else np.zeros(n, np.uint64))
    return Batch(keys.reshape(-1), key_off, np.ascontiguousarray(vals).reshape(-1), val_off,
                 np.zeros(n, np.uint8), seq, None, None, None)


def sorted_random_keys(seed, n, key_len=16, unique=True):
    raw = random_bytes(seed, 0, n * key_len).reshape(n, key_len)
    # sort lexicographically via big-endian u64 columns
    cols = []
    for c in range(0, key_len, 8):
        w = np.zeros((n, 8), np.uint8)
        w[:, :min(8, key_len - c)] = raw[:, c:c + 8]
        cols.append(w.view(">u8").reshape(-1).astype(np.uint64))
    order = np.lexsort(cols[::-1])
    raw = raw[order]
    if unique and n > 1:
        keep = np.ones(n, bool)
        keep[1:] = np.any(raw[1:] != raw[:-1], axis=1)
        raw = raw[keep]
    return raw


def d2(n=D1_N, value_len=100, seed=SEED_D2):
    keys = sorted_random_keys(seed, n)
    m = len(keys)
    stride = (value_len + 7) // 8 * 8
    vals = random_bytes(seed + 1, 0, m * stride).reshape(m, stride)[:, :value_len]
    return Batch(keys.reshape(-1), np.arange(m + 1, dtype=np.uint64) * np.uint64(16),
                 np.ascontiguousarray(vals).reshape(-1),
                 np.arange(m + 1, dtype=np.uint64) * np.uint64(value_len),
                 np.zeros(m, np.uint8), np.zeros(m, np.uint64))


def c4_keys(n=10_000_000, seed=SEED_C4):
    """Config 4 keys: returns (key_bytes, key_off)."""
    keys = sorted_random_keys(seed, n, unique=False)
    return keys.reshape(-1), np.arange(len(keys) + 1, dtype=np.uint64) * np.uint64(16)


def d3(seed=3, n=3000):
    """D3 parity-mixed: tombstones, merges, timestamps, empty values, duplicate keys with descending
    seq across restart/block boundaries, long keys (>128 B, chunked LCP), variable lengths."""
    rng = np.random.default_rng(seed)
    entries = []
    base = b"user:"
    i = 0
    while len(entries) < n:
        r = rng.random()
        if r < 0.05:
            key = base + b"L" * int(rng.integers(120, 400)) + b"%08d" % i
        elif r < 0.1:
            key = bytes(rng.integers(0, 256, int(rng.integers(1, 8)), dtype=np.uint8))
            key = base + b"\xff" + key
        else:
            key = base + b"%010d" % i
        dup = int(rng.integers(1, 4)) if rng.random() < 0.15 else 1
        for d in range(dup):
            kr = rng.random()
            kind = 2 if kr < 0.15 else (1 if kr < 0.3 else 0)
            vlen = 0 if rng.random() < 0.05 else int(rng.integers(1, 300))
            val = bytes(rng.integers(0, 256, vlen, dtype=np.uint8))
            seq = 10_000_000 - len(entries)
            cts = int(rng.integers(-2**40, 2**40)) if rng.random() < 0.3 else None
            ets = int(rng.integers(0, 2**40)) if rng.random() < 0.3 else None
            entries.append((key, kind, val, seq, cts, ets))
        i += 1
    entries.sort(key=lambda e: (e[0], -e[3]))
    return Batch.from_entries(entries[:n])


def overwrite_runs(nruns=4, n=D1_N, value_len=100, overlap=0.75, tomb_frac=0.1, seed=SEED_D1 + 77):
    """A compaction whose retention drops entries: `nruns` L0 runs (newest first) of n entries each, drawn
    from one key space of n / overlap 16-byte keys (D1's BE counter layout), so most keys have versions in
    several runs; run r's seqs are (nruns - r) << 32 | position (newer runs are higher); the newest run
    deletes tomb_frac of its keys (tombstones, no value).  With no snapshot (retention_min_seq None) and
    filter_tombstone (the destination is the last run), retention keeps each key's newest version and
    drops its tombstones (retention_iterator.rs:91-204, 381-398)."""
    u = int(n / overlap)
    start = splitmix64(seed, 0, 2)
    hi0, lo0 = np.uint64(int(start[0]) >> 32), start[1]
    runs = []
    for r in range(nruns):
        rng = np.random.default_rng(seed + r)
        idx = np.sort(rng.choice(u, size=n, replace=False)).astype(np.uint64)
        with np.errstate(over="ignore"):
            lo = lo0 + idx
            hiv = hi0 + (lo < lo0).astype(np.uint64)
        keys = np.empty((n, 16), np.uint8)
        keys[:, 0:4] = hiv.astype(">u4").view(np.uint8).reshape(-1, 4)
        keys[:, 4:12] = _be_bytes_u64(lo)
        keys[:, 12:16] = 0
        kind = np.zeros(n, np.uint8)
        if r == 0 and tomb_frac > 0:
            kind[rng.random(n) < tomb_frac] = 2  # SDB_KIND_TOMBSTONE
        vlen = np.where(kind == 2, 0, value_len).astype(np.uint64)
        val_off = np.zeros(n + 1, np.uint64)
        val_off[1:] = np.cumsum(vlen)
        vals = random_bytes(seed + 1000 + r, 0, int(val_off[-1]))
        seq = (np.uint64(nruns - r) << np.uint64(32)) | np.arange(n, dtype=np.uint64)
        runs.append(Batch(keys.reshape(-1), np.arange(n + 1, dtype=np.uint64) * np.uint64(16), vals, val_off,
                          kind, seq))
    return runs


_FIRST = ["alice", "bob", "carol", "dave", "erin", "frank", "grace", "heidi", "ivan", "judy", "mallory",
          "niaj", "olivia", "peggy", "rupert", "sybil", "trent", "victor", "walter", "yolanda"]
_LAST = ["smith", "jones", "garcia", "miller", "davis", "lopez", "wilson", "taylor", "thomas", "moore",
         "martin", "lee", "walker", "hall", "young", "king", "wright", "scott", "green", "baker"]
_CITY = ["amsterdam", "berlin", "chicago", "denver", "edinburgh", "florence", "geneva", "houston",
         "istanbul", "jakarta", "kyoto", "lisbon", "madrid", "nairobi", "oslo", "paris"]
_TAGS = ["admin", "beta", "churned", "trial", "premium", "verified", "mobile", "eu", "us", "apac"]


def text_kv(n=200_000, seed=11):
    """A compressible set for the codec write side (f3): ASCII keys "user:%010d" (sorted, gaps) and JSON
    documents of 90-200 bytes drawn from small vocabularies — the kind of values a KV store actually
    compresses, unlike D1's random bytes."""
    rng = np.random.default_rng(seed)
    ids = np.cumsum(rng.integers(1, 50, n))
    f, l, c = rng.integers(0, len(_FIRST), n), rng.integers(0, len(_LAST), n), rng.integers(0, len(_CITY), n)
    age, score = rng.integers(18, 90, n), rng.integers(0, 100000, n)
    nt = rng.integers(0, 4, n)
    tg = rng.integers(0, len(_TAGS), (n, 3))
    entries = []
    for i in range(n):
        tags = ",".join('"%s"' % _TAGS[t] for t in tg[i, :nt[i]])
        v = ('{"name":"%s %s","email":"%s.%s@example.com","city":"%s","age":%d,"score":%d,"tags":[%s]}' %
             (_FIRST[f[i]], _LAST[l[i]], _FIRST[f[i]], _LAST[l[i]], _CITY[c[i]], age[i], score[i], tags))
        entries.append((b"user:%010d" % ids[i], 0, v.encode(), 0, None, None))
    return Batch.from_entries(entries)
