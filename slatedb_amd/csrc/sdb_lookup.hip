// sdb_lookup.hip — batched point lookups / seeks on one encoded SST for gfx950.
//
// Replaces the read path of Db::get / an SstIterator positioned on a key:
//   filter      BloomFilter::might_contain(filter_hash(key))            filter.rs:124-136
//   blocks      partitions_covering_range([key, key]) over the index     partitioned_keyspace.rs:16-110
//   seek        BlockIteratorV2::seek asc / DescendingBlockIteratorV2    block_iterator_v2.rs:138-208,
//               ::seek; BlockIterator::seek (V1)                         269-313, 318-469;
//                                                                        block_iterator.rs:130-190
//   next block  only the first block of the range is seeked; an exhausted seek enters the next block
//               at its first (asc) / last (desc) entry                   sst_iter.rs:501-516
//   checksum    every block read is CRC-checked                          format/sst.rs:1029-1038
// Three launches: k_lk_locate (thread per query: filter + index -> the <= 2 blocks the seek can
// touch, marked), k_lk_check (wave per marked block: the shared wave CRC), k_lk_seek (thread per
// query: the seek itself).  Keys are never materialised: a seek step compares the next key
// prev[..shared] ++ suffix with the target from the running (common prefix, order) state of the
// previous key, reading only the suffix bytes.
#include <mutex>

#include "sdb_bloom.h"
#include "sdb_crc.h"
#include "sdb_device.h"

namespace sdb {

struct LookupArgs {
    sdb_sst_view v;
    const uint8_t *key_bytes;
    const uint64_t *key_off;
    uint64_t nkeys;
    uint32_t desc;
    sdb_lookup_out out;
    uint32_t *qrange;     // per query: start, end (block range; end == start: empty)
    uint8_t *mark;        // per block: 1 = a seek reads it
    int32_t *bstat;       // per block: sdb_status of Block::decode + CRC
};

SDB_DEV uint64_t be_at(const uint8_t *p, int n) {
    uint64_t v = 0;
    for (int i = 0; i < n; i++) v = (v << 8) | p[i];
    return v;
}

// Order of a and b (<[u8] as Ord>) and their common prefix, from global memory.
struct Cmp {
    uint32_t m;  // common prefix of key and target
    int c;       // sign(key cmp target)
    uint32_t len;
};
SDB_DEV Cmp cmp_bytes(const uint8_t *a, uint32_t na, const uint8_t *t, uint32_t nt, uint32_t base) {
    // a is the key from byte `base` on; t the whole target
    Cmp r;
    const uint32_t rest = nt > base ? nt - base : 0;
    const uint32_t l = lcp_bytes(a, na, t + base, rest);
    r.m = base + l;
    r.len = base + na;
    if (l < na && l < rest) r.c = a[l] < t[base + l] ? -1 : 1;
    else r.c = na < rest ? -1 : (na > rest ? 1 : 0);
    return r;
}
// The key K' = K[..sh] ++ S given K's state s against the target.
SDB_DEV Cmp cmp_next(Cmp s, uint32_t sh, const uint8_t *S, uint32_t un, const uint8_t *t, uint32_t nt) {
    if (sh > s.m) {  // K' agrees with K on [0, m]: same order; T a proper prefix of K' when m == |T|
        Cmp r;
        r.m = s.m;
        r.len = sh + un;
        r.c = s.m < nt ? s.c : 1;
        return r;
    }
    return cmp_bytes(S, un, t, nt, sh);  // K'[0, sh) == T[0, sh)
}

struct Blk {  // Block::decode of a checked block
    const uint8_t *d;
    uint32_t data_end, count;
    const uint8_t *offs;
    uint64_t base;
};
SDB_DEV int blk_open(const LookupArgs &a, uint64_t k, Blk &b) {
    const uint64_t s = a.v.block_off[k], e = a.v.block_off[k + 1];
    if (e < s || e - s < 6) return SDB_CORRUPT_BLOCK;
    const uint32_t blen = (uint32_t)(e - s - 4);
    b.d = a.v.data + s;
    b.base = s;
    b.count = (uint32_t)be_at(b.d + blen - 2, 2);
    if (2 + 2 * (uint64_t)b.count > blen) return SDB_CORRUPT_BLOCK;
    b.data_end = blen - 2 - 2 * b.count;
    b.offs = b.d + b.data_end;
    return 0;
}
SDB_DEV uint32_t boff(const Blk &b, uint32_t i) { return (uint32_t)be_at(b.offs + 2 * i, 2); }

SDB_DEV bool rdv(const uint8_t *d, uint32_t end, uint32_t &pos, uint32_t &v) {  // decode_varint
    uint32_t r = 0;
    for (int sh = 0; sh <= 28; sh += 7) {
        if (pos >= end) return false;
        const uint8_t x = d[pos++];
        r |= (uint32_t)(x & 0x7F) << sh;
        if (!(x & 0x80)) {
            v = r;
            return true;
        }
    }
    return false;
}
SDB_DEV bool flags_valid(uint8_t f) { return !(f & ~0x0Fu) && !((f & SDB_FLAG_TOMBSTONE) && (f & SDB_FLAG_MERGE_OPERAND)); }

struct Row {
    uint32_t sh, un, vl, suf, vpos, next;
    uint64_t seq;
    int64_t cts, ets;
    uint8_t flags;
};
SDB_DEV int v2_row(const Blk &b, uint32_t pos, Row &r) {  // SstRowCodecV2::decode (row_codec_v2.rs:172-220)
    if (!rdv(b.d, b.data_end, pos, r.sh) || !rdv(b.d, b.data_end, pos, r.un) || !rdv(b.d, b.data_end, pos, r.vl))
        return SDB_CORRUPT_BLOCK;
    if ((uint64_t)pos + r.un + r.vl + 9 > b.data_end) return SDB_CORRUPT_BLOCK;
    r.suf = pos;
    pos += r.un;
    r.vpos = pos;
    pos += r.vl;
    r.seq = be_at(b.d + pos, 8);
    pos += 8;
    r.flags = b.d[pos++];
    if (!flags_valid(r.flags)) return SDB_INVALID_ROW_FLAGS;
    const uint32_t need = ((r.flags & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((r.flags & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
    if ((uint64_t)pos + need > b.data_end) return SDB_CORRUPT_BLOCK;
    r.ets = r.cts = 0;
    if (r.flags & SDB_FLAG_HAS_EXPIRE_TS) {
        r.ets = (int64_t)be_at(b.d + pos, 8);
        pos += 8;
    }
    if (r.flags & SDB_FLAG_HAS_CREATE_TS) {
        r.cts = (int64_t)be_at(b.d + pos, 8);
        pos += 8;
    }
    r.next = pos;
    return 0;
}
// decode_first_key_at_restart (block_iterator_v2.rs:73-80): key = d[*kp, *kp + *kn), shared == 0
SDB_DEV int v2_restart_key(const Blk &b, uint32_t ri, uint32_t &kp, uint32_t &kn) {
    uint32_t p = boff(b, ri), sh, un, vl;
    if (p > b.data_end || !rdv(b.d, b.data_end, p, sh) || !rdv(b.d, b.data_end, p, un) || !rdv(b.d, b.data_end, p, vl) ||
        sh != 0 || (uint64_t)p + un > b.data_end)
        return SDB_CORRUPT_BLOCK;
    kp = p;
    kn = un;
    return 0;
}
SDB_DEV uint32_t region_end(const Blk &b, uint32_t ri) { return ri + 1 < b.count ? boff(b, ri + 1) : b.data_end; }

struct Pos {
    bool ok;         // positioned
    uint32_t at;     // V2: byte offset of the entry; V1: its index
    Cmp key;         // the entry's key against the target
};

// binary_search_restarts (block_iterator_v2.rs:138-154)
SDB_DEV int v2_bsearch(const Blk &b, const uint8_t *t, uint32_t nt, uint32_t &low) {
    uint32_t lo = 0, hi = b.count;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        uint32_t kp, kn;
        if (int st = v2_restart_key(b, mid, kp, kn)) return st;
        if (cmp_bytes(b.d + kp, kn, t, nt, 0).c < 0) lo = mid + 1;
        else hi = mid;
    }
    low = lo;
    return 0;
}

// BlockIteratorV2::seek ascending (block_iterator_v2.rs:157-176, 269-313)
SDB_DEV int v2_seek_asc(const Blk &b, const uint8_t *t, uint32_t nt, Pos &P) {
    P.ok = false;
    if (b.count == 0) return 0;
    uint32_t low;
    if (int st = v2_bsearch(b, t, nt, low)) return st;
    for (uint32_t ri = low ? low - 1 : 0; ri < b.count; ri++) {  // find_restart_for_key_ascending
        uint32_t kp, kn;
        if (int st = v2_restart_key(b, ri, kp, kn)) return st;
        uint32_t off = boff(b, ri);
        const Cmp rk = cmp_bytes(b.d + kp, kn, t, nt, 0);  // seek_to_restart
        if (off >= b.data_end) return 0;                   // exhausted
        if (rk.c >= 0) {
            P.ok = true;
            P.at = off;
            P.key = rk;
            return 0;
        }
        const uint32_t rend = region_end(b, ri);
        Cmp prev = rk;
        while (off < rend && off < b.data_end) {
            uint32_t p = off, sh, un, vl;  // decode_key_at_offset (:115-126)
            if (!rdv(b.d, b.data_end, p, sh) || !rdv(b.d, b.data_end, p, un) || !rdv(b.d, b.data_end, p, vl) ||
                sh > prev.len || (uint64_t)p + un > b.data_end)
                return SDB_CORRUPT_BLOCK;
            const Cmp cur = cmp_next(prev, sh, b.d + p, un, t, nt);
            if (cur.c >= 0) {
                P.ok = true;
                P.at = off;
                P.key = cur;
                return 0;
            }
            Row r;  // advance_past_current_entry
            if (int st = v2_row(b, off, r)) return st;
            off = r.next;
            prev = cur;
        }
    }
    return 0;
}

// DescendingBlockIteratorV2::seek (block_iterator_v2.rs:178-208, 430-469)
SDB_DEV int v2_seek_desc(const Blk &b, const uint8_t *t, uint32_t nt, Pos &P) {
    P.ok = false;
    if (b.count == 0) return 0;
    uint32_t low;
    if (int st = v2_bsearch(b, t, nt, low)) return st;
    uint32_t start = low ? low - 1 : 0;
    if (low < b.count) {  // find_restart_for_key_descending
        uint32_t kp, kn;
        if (int st = v2_restart_key(b, low, kp, kn)) return st;
        if (cmp_bytes(b.d + kp, kn, t, nt, 0).c == 0) {
            uint32_t last = low;
            while (last + 1 < b.count) {
                if (int st = v2_restart_key(b, last + 1, kp, kn)) return st;
                if (cmp_bytes(b.d + kp, kn, t, nt, 0).c != 0) break;
                last++;
            }
            start = last;
        }
    }
    for (uint32_t ri = start + 1; ri-- > 0;) {
        uint32_t kp, kn;
        if (int st = v2_restart_key(b, ri, kp, kn)) return st;
        Cmp cur{0, 0, kn};
        cur = cmp_bytes(b.d + kp, kn, t, nt, 0);
        uint32_t off = boff(b, ri);
        const uint32_t rend = region_end(b, ri);
        bool have = false;
        while (off < rend && off < b.data_end) {  // load_restart_region (:375-394)
            Row r;
            if (int st = v2_row(b, off, r)) return st;
            if (r.sh > cur.len) return SDB_CORRUPT_BLOCK;
            cur = cmp_next(cur, r.sh, b.d + r.suf, r.un, t, nt);
            if (cur.c > 0) break;  // the last entry before the first key > target
            have = true;
            P.at = off;
            P.key = cur;
            off = r.next;
        }
        if (have) {
            P.ok = true;
            return 0;
        }
    }
    return 0;
}

// V1 key i = first_key[..prefix] ++ suffix (decode_key_at_index, block_iterator.rs:249-265)
SDB_DEV int v1_cmp(const Blk &b, uint32_t i, const uint8_t *t, uint32_t nt, Cmp &c) {
    if (b.data_end < 4 || be_at(b.d, 2) != 0) return SDB_CORRUPT_BLOCK;  // decode_first_key
    const uint32_t fk = (uint32_t)be_at(b.d + 2, 2);
    if (4 + fk > b.data_end) return SDB_CORRUPT_BLOCK;
    const uint32_t p = boff(b, i);
    if (p + 4 > b.data_end) return SDB_CORRUPT_BLOCK;
    const uint32_t pre = (uint32_t)be_at(b.d + p, 2), sl = (uint32_t)be_at(b.d + p + 2, 2);
    if (pre > fk || p + 4 + sl > b.data_end) return SDB_CORRUPT_BLOCK;
    Cmp f = cmp_bytes(b.d + 4, pre, t, nt, 0);  // the prefix part
    if (f.m < pre) {
        f.len = pre + sl;
        c = f;
        return 0;
    }
    c = cmp_bytes(b.d + p + 4, sl, t, nt, pre);
    return 0;
}
// BlockIterator::seek (block_iterator.rs:130-190)
SDB_DEV int v1_seek(const Blk &b, const uint8_t *t, uint32_t nt, bool desc, Pos &P) {
    P.ok = false;
    uint32_t lo = 0, hi = b.count;
    while (lo < hi) {
        const uint32_t mid = lo + (hi - lo) / 2;
        Cmp c;
        if (int st = v1_cmp(b, mid, t, nt, c)) return st;
        if (desc ? c.c <= 0 : c.c < 0) lo = mid + 1;
        else hi = mid;
    }
    if (!desc && lo < b.count) {
        P.ok = true;
        P.at = lo;
    }
    if (desc && lo > 0) {
        P.ok = true;
        P.at = lo - 1;
    }
    if (P.ok) return v1_cmp(b, P.at, t, nt, P.key);
    return 0;
}

// partition_point (partitioned_keyspace.rs:16-39); le: first_key <= key, else first_key < key
SDB_DEV uint64_t partition_point(const LookupArgs &a, const uint8_t *t, uint32_t nt, bool le) {
    const uint64_t n = a.v.num_blocks;
    if (n == 0) return 0;
    uint64_t lo = 0, hi = n - 1, pp = 0;
    while (lo <= hi) {
        const uint64_t mid = lo + (hi - lo) / 2;
        const uint64_t f0 = a.v.index_key_off[mid], f1 = a.v.index_key_off[mid + 1];
        const int c = cmp_bytes(a.v.index_keys + f0, (uint32_t)(f1 - f0), t, nt, 0).c;
        if (le ? c <= 0 : c < 0) {
            lo = mid + 1;
            pp = mid + 1;
        } else if (mid > lo) {
            hi = mid - 1;
        } else {
            break;
        }
    }
    return pp;
}

__global__ __launch_bounds__(256) void k_lk_locate(LookupArgs a) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.nkeys) return;
    const uint8_t *t = a.key_bytes + a.key_off[q];
    const uint32_t nt = (uint32_t)(a.key_off[q + 1] - a.key_off[q]);
    uint32_t start = 0, end = 0;
    bool filtered = false;
    if (a.v.bloom) {  // might_contain (filter.rs:124-136): an empty bitmap answers false
        const uint32_t m = (uint32_t)(a.v.bloom_len * 8);
        filtered = true;
        if (m) {
            const uint64_t h = siphash13(t, nt);  // filter_hash (filter.rs:196-204)
            uint32_t hh = (uint32_t)h % m, d = (uint32_t)(h >> 32) % m;
            filtered = false;
            for (uint32_t i = 0; i < a.v.num_probes; i++) {
                d = (uint32_t)(((uint64_t)d + i) % m);
                if (!((a.v.bloom[hh >> 3] >> (hh & 7)) & 1)) {
                    filtered = true;
                    break;
                }
                hh = (uint32_t)(((uint64_t)hh + d) % m);
            }
        }
    }
    if (!filtered) {  // partitions_covering_range(Included(k), Included(k))
        const uint64_t lt = partition_point(a, t, nt, false), le = partition_point(a, t, nt, true);
        start = (uint32_t)(lt > 0 ? lt - 1 : 0);
        end = (uint32_t)(le > 0 ? le : start);
        if (end > start) {  // the seeked block and the one after it in iteration order
            const uint32_t b0 = a.desc ? end - 1 : start;
            a.mark[b0] = 1;
            if (end - start >= 2) a.mark[a.desc ? end - 2 : start + 1] = 1;
        }
    }
    a.qrange[2 * q] = start;
    a.qrange[2 * q + 1] = filtered ? 0xFFFFFFFFu : end;
}

// One wave per marked block: Block::decode bounds + CRC (the shared wave CRC over an LDS image).
constexpr uint32_t kLkThreads = 256;
constexpr uint32_t kLkImg = 4096 + 32;
__global__ __launch_bounds__(kLkThreads) void k_lk_check(LookupArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    crc_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, l = (uint32_t)lane_id();
    lu8 *img = (lu8 *)smem + kCrcTablesLds + wave * (kLkImg + 64) + 64;
    if (l < 16) ((lu32 *)(img - 64))[l] = 0;  // zero lead-in of the right-aligned CRC segments
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k < a.v.num_blocks; k += nw) {
        if (!a.mark[k]) continue;
        const uint64_t s = a.v.block_off[k], e = a.v.block_off[k + 1];
        int st = 0;
        if (e < s || e - s < 6) {
            st = SDB_CORRUPT_BLOCK;
        } else {
            const uint32_t blen = (uint32_t)(e - s - 4);
            uint32_t crc;
            if (blen + 16 <= 4096 && blen >= 4) {
                const uint32_t p0 = (uint32_t)(s & 15), Lc = p0 + blen;
                const uint64_t a0 = s & ~15ull;
                const uint32_t ng = (uint32_t)((((s + blen + 15) & ~15ull) - a0) >> 4);
                for (uint32_t g = l; g < ng; g += 64) {
                    const uint4 v = ((const uint4 *)(a.v.data + a0))[g];
                    u32x4 w;
                    w.x = v.x;
                    w.y = v.y;
                    w.z = v.z;
                    w.w = v.w;
                    ((lu128 *)img)[g] = w;
                }
                __builtin_amdgcn_wave_barrier();
                if (l < p0) img[l] = 0;
                if (l < 4) img[p0 + l] ^= 0xFF;  // crc32fast's init
                __builtin_amdgcn_wave_barrier();
                crc = wave_crc_image_ra(img, Lc);
                __builtin_amdgcn_wave_barrier();
            } else {  // large blocks: one lane, byte-wise
                uint32_t x = 0xFFFFFFFFu;
                if (l == 0)
                    for (uint32_t i = 0; i < blen; i++) x = c_crc.t[0][(x ^ a.v.data[s + i]) & 0xFF] ^ (x >> 8);
                crc = (uint32_t)__builtin_amdgcn_readfirstlane((int)(x ^ 0xFFFFFFFFu));
            }
            if (crc != (uint32_t)be_at(a.v.data + s + blen, 4)) st = SDB_CHECKSUM_MISMATCH;
        }
        if (l == 0) {
            a.bstat[k] = st;
            a.mark[k] = 0;  // ready for the next call
        }
    }
}

SDB_DEV void report(const LookupArgs &a, uint64_t q, const Blk &b, uint32_t blk, const Pos &P, int &st) {
    Row r;
    uint32_t phys = 0;
    if (a.v.sst_version == 2) {
        if ((st = v2_row(b, P.at, r))) return;
        for (uint32_t p = 0; p < P.at; phys++) {  // the entry's index: rows before it
            Row x;
            if ((st = v2_row(b, p, x))) return;
            p = x.next;
        }
        if (r.flags & SDB_FLAG_TOMBSTONE) r.vl = 0;
        a.out.val_off[q] = r.vl ? b.base + r.vpos : 0;
        a.out.val_len[q] = r.vl;
    } else {
        phys = P.at;
        uint32_t p = boff(b, P.at) + 4;
        const uint32_t sl = (uint32_t)be_at(b.d + p - 2, 2);
        p += sl;
        if ((uint64_t)p + 9 > b.data_end) {
            st = SDB_CORRUPT_BLOCK;
            return;
        }
        r.seq = be_at(b.d + p, 8);
        p += 8;
        uint8_t f = b.d[p++];
        if (!flags_valid(f)) {
            st = SDB_INVALID_ROW_FLAGS;
            return;
        }
        const uint32_t need = ((f & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((f & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
        if ((uint64_t)p + need > b.data_end) {
            st = SDB_CORRUPT_BLOCK;
            return;
        }
        r.ets = r.cts = 0;
        if (f & SDB_FLAG_HAS_EXPIRE_TS) {
            r.ets = (int64_t)be_at(b.d + p, 8);
            p += 8;
        }
        if (f & SDB_FLAG_HAS_CREATE_TS) {
            r.cts = (int64_t)be_at(b.d + p, 8);
            p += 8;
        }
        uint32_t vl = 0;
        uint64_t vp = 0;
        if (f & SDB_FLAG_TOMBSTONE) {
            f = (uint8_t)(f & ~SDB_FLAG_HAS_EXPIRE_TS);  // V0 decode drops expire_ts (row.rs:223-231)
        } else {
            if ((uint64_t)p + 4 > b.data_end) {
                st = SDB_CORRUPT_BLOCK;
                return;
            }
            vl = (uint32_t)be_at(b.d + p, 4);
            p += 4;
            if ((uint64_t)p + vl > b.data_end) {
                st = SDB_CORRUPT_BLOCK;
                return;
            }
            vp = b.base + p;
        }
        r.flags = f;
        a.out.val_off[q] = vl ? vp : 0;
        a.out.val_len[q] = vl;
    }
    a.out.flags[q] = r.flags;
    a.out.seq[q] = r.seq;
    a.out.create_ts[q] = (r.flags & SDB_FLAG_HAS_CREATE_TS) ? r.cts : 0;
    a.out.expire_ts[q] = (r.flags & SDB_FLAG_HAS_EXPIRE_TS) ? r.ets : 0;
    a.out.block[q] = blk;
    a.out.entry[q] = phys;
    a.out.key_len[q] = P.key.len;
    a.out.state[q] = P.key.c == 0 ? SDB_LOOKUP_FOUND : SDB_LOOKUP_POSITIONED;
}

__global__ __launch_bounds__(256) void k_lk_seek(LookupArgs a) {
    const uint64_t q = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (q >= a.nkeys) return;
    const uint8_t *t = a.key_bytes + a.key_off[q];
    const uint32_t nt = (uint32_t)(a.key_off[q + 1] - a.key_off[q]);
    const uint32_t start = a.qrange[2 * q], end = a.qrange[2 * q + 1];
    a.out.status[q] = 0;
    a.out.state[q] = SDB_LOOKUP_EXHAUSTED;
    a.out.block[q] = a.out.entry[q] = a.out.key_len[q] = 0;
    a.out.val_off[q] = 0;
    a.out.val_len[q] = 0;
    a.out.seq[q] = 0;
    a.out.flags[q] = 0;
    a.out.create_ts[q] = a.out.expire_ts[q] = 0;
    if (end == 0xFFFFFFFFu) {
        a.out.state[q] = SDB_LOOKUP_FILTERED;
        return;
    }
    int st = 0;
    for (uint32_t i = 0; end > start && i < 2 && i < end - start; i++) {  // seeked block, then its successor
        const uint32_t blk = a.desc ? end - 1 - i : start + i;
        Blk b;
        if ((st = a.bstat[blk]) || (st = blk_open(a, blk, b))) break;
        Pos P;
        P.ok = false;
        if (i == 0) {
            if (a.v.sst_version == 2) st = a.desc ? v2_seek_desc(b, t, nt, P) : v2_seek_asc(b, t, nt, P);
            else st = v1_seek(b, t, nt, a.desc, P);
        } else if (b.count > 0) {  // a fresh block iterator: first entry (asc) or last (desc)
            if (a.v.sst_version == 1) {
                P.ok = true;
                P.at = a.desc ? b.count - 1 : 0;
                st = v1_cmp(b, P.at, t, nt, P.key);
            } else {
                uint32_t kp, kn;
                if (!(st = v2_restart_key(b, a.desc ? b.count - 1 : 0, kp, kn))) {
                    Cmp cur = cmp_bytes(b.d + kp, kn, t, nt, 0);
                    if (!a.desc) {
                        if (b.data_end > 0) {
                            P.ok = true;
                            P.at = 0;
                            P.key = cur;
                        }
                    } else {  // the last region's last entry
                        uint32_t off = boff(b, b.count - 1);
                        while (!st && off < b.data_end) {
                            Row r;
                            if ((st = v2_row(b, off, r))) break;
                            if (r.sh > cur.len) {
                                st = SDB_CORRUPT_BLOCK;
                                break;
                            }
                            cur = cmp_next(cur, r.sh, b.d + r.suf, r.un, t, nt);
                            P.ok = true;
                            P.at = off;
                            P.key = cur;
                            off = r.next;
                        }
                    }
                }
            }
        }
        if (!st && P.ok) report(a, q, b, blk, P, st);
        if (st || P.ok) break;
    }
    if (st) {
        a.out.status[q] = st;
        a.out.state[q] = SDB_LOOKUP_EXHAUSTED;
    }
}

uint64_t lookup_workspace_bytes(uint64_t num_blocks, uint64_t nkeys) {
    return ((8 * (nkeys + 1) + 255) & ~255ull) + ((num_blocks + 256) & ~255ull) + ((4 * (num_blocks + 1) + 255) & ~255ull);
}

hipError_t launch_lookup(LookupArgs a, hipStream_t st) {
    if (!a.nkeys) return hipSuccess;
    static std::once_flag once;
    std::call_once(once, [] {
        (void)hipFuncSetAttribute((const void *)k_lk_check, hipFuncAttributeMaxDynamicSharedMemorySize,
                                  (int)(kCrcTablesLds + (kLkThreads / 64) * (kLkImg + 64)));
        (void)hipGetLastError();
    });
    if (a.v.num_blocks) {
        hipError_t e = hipMemsetAsync(a.mark, 0, a.v.num_blocks, st);
        if (e != hipSuccess) return e;
    }
    const uint32_t qb = (uint32_t)((a.nkeys + 255) / 256);
    hipLaunchKernelGGL(k_lk_locate, dim3(qb), dim3(256), 0, st, a);
    if (a.v.num_blocks) {
        uint64_t wgs = (a.v.num_blocks + 3) / 4;
        if (wgs > 4096) wgs = 4096;
        hipLaunchKernelGGL(k_lk_check, dim3((uint32_t)wgs), dim3(kLkThreads), kCrcTablesLds + (kLkThreads / 64) * (kLkImg + 64),
                           st, a);
    }
    hipLaunchKernelGGL(k_lk_seek, dim3(qb), dim3(256), 0, st, a);
    return hipGetLastError();
}

}  // namespace sdb
