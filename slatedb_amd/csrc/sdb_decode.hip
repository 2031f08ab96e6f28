// sdb_decode.hip — batched SST block decode for gfx950.
//
// Replaces SsTableFormat::read_blocks -> decode_block -> validate_checksum -> Block::decode
// (slatedb/src/format/sst.rs:938-1038, format/block.rs:28-46) followed by draining
// DataBlockIterator ascending (block_iterator.rs:54-267, block_iterator_v2.rs:33-113,235-267) into
// columnar RowEntry output (the SstFile::read_block contract, sst_reader.rs:287-309).
//
// D1 count   one wave per block: stage the block into LDS with 16-byte loads, CRC32 check
//            (same wave CRC as the encoder), parse the trailer and every row (V2: one lane per
//            restart region; V1: one lane per entry offset) -> entries and restored-key bytes.
// D2 scan    exclusive scans over blocks (tile sums -> tile scan -> apply).
// D3 emit    one wave per block: parse again and write keys (restored against the previous key),
//            value references into `blocks`, seq, flags and timestamps.
#include "sdb_decode.h"
#include "sdb_device.h"

namespace sdb {

constexpr uint32_t kDecCap = 8192;  // LDS staging per wave (bytes); larger blocks parse from HBM

SDB_DEV uint64_t rd_be(const uint8_t *p, int nb) {
    uint64_t v = 0;
    for (int i = 0; i < nb; i++) v = (v << 8) | p[i];
    return v;
}

// Parse one varint (decode_varint, utils.rs:622-634) from d[*pos] (bounded by end).
SDB_DEV bool rd_varint(const uint8_t *d, uint32_t end, uint32_t *pos, uint32_t *v) {
    uint32_t r = 0;
    int sh = 0;
    for (;;) {
        if (*pos >= end || sh > 28) return false;
        uint8_t b = d[(*pos)++];
        r |= (uint32_t)(b & 0x7F) << sh;
        if (!(b & 0x80)) break;
        sh += 7;
    }
    *v = r;
    return true;
}

SDB_DEV bool flags_ok(uint8_t f) {  // decode_flags (row_codec_v2.rs:234-249)
    return !(f & ~0x0Fu) && !((f & SDB_FLAG_TOMBSTONE) && (f & SDB_FLAG_MERGE_OPERAND));
}

struct RowV2 {
    uint32_t shared, unshared, vlen, suf_pos, val_pos, next;
    uint64_t seq;
    int64_t ets, cts;
    uint8_t flags;
};

// SstRowCodecV2::decode (row_codec_v2.rs:172-220).  Returns 0 or an sdb_status.
SDB_DEV int parse_v2(const uint8_t *d, uint32_t end, uint32_t pos, RowV2 *r) {
    if (!rd_varint(d, end, &pos, &r->shared) || !rd_varint(d, end, &pos, &r->unshared) ||
        !rd_varint(d, end, &pos, &r->vlen))
        return SDB_CORRUPT_BLOCK;
    if ((uint64_t)pos + r->unshared + r->vlen + 9 > end) return SDB_CORRUPT_BLOCK;
    r->suf_pos = pos;
    pos += r->unshared;
    r->val_pos = pos;
    pos += r->vlen;
    r->seq = rd_be(d + pos, 8);
    pos += 8;
    uint8_t f = d[pos++];
    if (!flags_ok(f)) return SDB_INVALID_ROW_FLAGS;
    uint32_t need = ((f & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((f & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
    if ((uint64_t)pos + need > end) return SDB_CORRUPT_BLOCK;
    r->ets = 0;
    r->cts = 0;
    if (f & SDB_FLAG_HAS_EXPIRE_TS) {
        r->ets = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    if (f & SDB_FLAG_HAS_CREATE_TS) {
        r->cts = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    r->flags = f;
    r->next = pos;
    return 0;
}

struct RowV0 {
    uint32_t prefix, suf, suf_pos, vlen, val_pos;
    uint64_t seq;
    int64_t ets, cts;
    uint8_t flags;  // as returned by the iterator (V0 tombstones drop expire_ts, row.rs:223-231)
};

// SstRowCodecV0::decode (row.rs:200-249).
SDB_DEV int parse_v0(const uint8_t *d, uint32_t end, uint32_t pos, RowV0 *r) {
    if ((uint64_t)pos + 4 > end) return SDB_CORRUPT_BLOCK;
    r->prefix = (uint32_t)rd_be(d + pos, 2);
    r->suf = (uint32_t)rd_be(d + pos + 2, 2);
    pos += 4;
    if ((uint64_t)pos + r->suf + 9 > end) return SDB_CORRUPT_BLOCK;
    r->suf_pos = pos;
    pos += r->suf;
    r->seq = rd_be(d + pos, 8);
    pos += 8;
    uint8_t f = d[pos++];
    if (!flags_ok(f)) return SDB_INVALID_ROW_FLAGS;
    uint32_t need = ((f & SDB_FLAG_HAS_EXPIRE_TS) ? 8 : 0) + ((f & SDB_FLAG_HAS_CREATE_TS) ? 8 : 0);
    if ((uint64_t)pos + need > end) return SDB_CORRUPT_BLOCK;
    r->ets = 0;
    r->cts = 0;
    if (f & SDB_FLAG_HAS_EXPIRE_TS) {
        r->ets = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    if (f & SDB_FLAG_HAS_CREATE_TS) {
        r->cts = (int64_t)rd_be(d + pos, 8);
        pos += 8;
    }
    r->vlen = 0;
    r->val_pos = 0;
    r->flags = f;
    if (f & SDB_FLAG_TOMBSTONE) {
        r->flags = (uint8_t)(f & ~SDB_FLAG_HAS_EXPIRE_TS);
    } else {
        if ((uint64_t)pos + 4 > end) return SDB_CORRUPT_BLOCK;
        r->vlen = (uint32_t)rd_be(d + pos, 4);
        pos += 4;
        if ((uint64_t)pos + r->vlen > end) return SDB_CORRUPT_BLOCK;
        r->val_pos = pos;
    }
    return 0;
}

SDB_DEV void wave_sync_d() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Block parse plan shared by count and emit: where the data lives and how rows are split on lanes.
struct BlockView {
    const uint8_t *d;      // block bytes (LDS or global), CRC stripped
    uint32_t data_end;     // end of rows
    uint32_t count;        // trailer count (restarts for V2, entries for V1)
    const uint8_t *offs;   // trailer offsets (big-endian u16)
    int status;
};

// Stage + CRC-check block k; fills the view.  Called by a whole wave.
SDB_DEV BlockView load_block(const DecodeArgs &a, uint64_t k, uint8_t *stage, const uint32_t (*crc)[256]) {
    BlockView v{};
    const uint64_t s = a.block_off[k], e = a.block_off[k + 1];
    const uint64_t len = e - s;
    if (len < 4) {
        v.status = SDB_CORRUPT_BLOCK;
        return v;
    }
    const uint8_t *g = a.blocks + s;
    const uint32_t blen = (uint32_t)(len - 4);
    uint32_t c;
    const uint8_t *d;
    if (len + 32 <= kDecCap) {
        // 16-byte granules covering [s, e); stage[pad + i] = g[i]
        uint64_t a0 = s & ~15ull, a1 = (e + 15) & ~15ull;
        uint32_t nchunk = (uint32_t)((a1 - a0) >> 4);
        const uint4 *src = (const uint4 *)(a.blocks + a0);
        for (uint32_t q = lane_id(); q < nchunk; q += 64) ((uint4 *)stage)[q] = src[q];
        wave_sync_d();
        d = stage + (s & 15);
        c = blen >= 4 ? wave_crc32_lds(d, blen, crc) : 0;
    } else {
        // big block: CRC through 4 KiB LDS windows, parse straight from HBM
        uint64_t nwin = (blen + 4095) >> 12;
        uint64_t first = blen - ((nwin - 1) << 12);
        uint32_t acc = 0;
        for (uint64_t w = 0; w < nwin; w++) {
            uint64_t wbeg = (w == 0) ? 0 : first + ((w - 1) << 12);
            uint32_t wlen = (uint32_t)((w == 0) ? first : 4096);
            for (uint32_t q = lane_id(); q < wlen; q += 64) stage[16 + q] = g[wbeg + q];
            wave_sync_d();
            uint32_t raw = wave_crc_raw_lds(stage + 16, wlen, crc, w == 0);
            acc = (w == 0) ? raw : (gf_mul(c_shift.window, acc) ^ raw);
            wave_sync_d();
        }
        c = acc ^ 0xFFFFFFFFu;
        d = g;
    }
    if (blen < 4) {  // the wave CRC folds the init into 4 message bytes; tiny blocks go byte-wise
        uint32_t x = 0xFFFFFFFFu;
        for (uint32_t q = 0; q < blen; q++) x = crc[0][(x ^ d[q]) & 0xFF] ^ (x >> 8);
        c = x ^ 0xFFFFFFFFu;
    }
    uint32_t stored = (uint32_t)rd_be(d + blen, 4);
    if (c != stored) {
        v.status = SDB_CHECKSUM_MISMATCH;  // validate_checksum (format/sst.rs:1029-1038)
        return v;
    }
    if (blen < 2) {
        v.status = SDB_CORRUPT_BLOCK;
        return v;
    }
    uint32_t cnt = (uint32_t)rd_be(d + blen - 2, 2);  // Block::decode (format/block.rs:28-46)
    if (2 + 2 * (uint64_t)cnt > blen) {
        v.status = SDB_CORRUPT_BLOCK;
        return v;
    }
    v.d = d;
    v.count = cnt;
    v.data_end = blen - 2 - 2 * cnt;
    v.offs = d + v.data_end;
    v.status = 0;
    return v;
}

// V2 plan: lane q parses restart region q when the block is "regular" (restart 0 at offset 0,
// strictly increasing restarts, regions ending exactly on the next restart, shared == 0 at every
// region start); otherwise lane 0 walks the whole block like BlockIteratorV2::next does.
// Returns (entries, key bytes, status) reduced over the wave.
struct Tally {
    uint64_t entries, key_bytes;
    int status;
    bool sequential;
};

SDB_DEV Tally tally_v2(const BlockView &v) {
    Tally t{0, 0, 0, false};
    const int l = lane_id();
    const uint32_t R = v.count;
    bool regular = R > 0 && rd_be(v.offs, 2) == 0;
    uint32_t my_entries = 0, my_kb = 0;
    int my_status = 0;
    bool my_regular = true;
    for (uint32_t q = l; q < R && regular; q += 64) {
        uint32_t pos = (uint32_t)rd_be(v.offs + 2 * q, 2);
        uint32_t end = (q + 1 < R) ? (uint32_t)rd_be(v.offs + 2 * q + 2, 2) : v.data_end;
        if (end <= pos || end > v.data_end) {
            my_regular = false;
            break;
        }
        uint32_t prevlen = 0;
        bool firstrow = true;
        while (pos < end) {
            RowV2 r;
            int st = parse_v2(v.d, v.data_end, pos, &r);
            if (st) {
                my_status = st;
                break;
            }
            if (firstrow && r.shared != 0) my_regular = false;
            if (!firstrow && r.shared > prevlen) {
                my_status = SDB_CORRUPT_BLOCK;
                break;
            }
            firstrow = false;
            prevlen = r.shared + r.unshared;
            my_entries++;
            my_kb += prevlen;
            pos = r.next;
        }
        if (pos != end && !my_status) my_regular = false;
        if (my_status || !my_regular) break;
    }
    // wave-reduce: regular only if every lane stayed regular
    bool all_regular = regular && (__ballot(!my_regular) == 0);
    if (all_regular) {
        // lowest-lane error wins (rows are in lane order within the block)
        uint64_t bad = __ballot(my_status != 0);
        if (bad) {
            int first = __builtin_ctzll(bad);
            t.status = __shfl(my_status, first, 64);
            return t;
        }
        t.entries = wave_sum((uint64_t)my_entries);
        t.key_bytes = wave_sum((uint64_t)my_kb);
        return t;
    }
    // sequential walk (lane 0)
    t.sequential = true;
    uint64_t ent = 0, kb = 0;
    int st = 0;
    if (l == 0) {
        uint32_t curlen = 0;
        if (R > 0) {  // decode_first_key_at_restart(0) asserts shared == 0
            uint32_t p = (uint32_t)rd_be(v.offs, 2);
            uint32_t sh = 0, un = 0, vl = 0;
            if (!rd_varint(v.d, v.data_end, &p, &sh) || !rd_varint(v.d, v.data_end, &p, &un) ||
                !rd_varint(v.d, v.data_end, &p, &vl) || sh != 0 || (uint64_t)p + un > v.data_end)
                st = SDB_CORRUPT_BLOCK;
            curlen = un;
        }
        uint32_t pos = 0;
        while (!st && pos < v.data_end) {
            RowV2 r;
            st = parse_v2(v.d, v.data_end, pos, &r);
            if (st) break;
            if (r.shared > curlen) {
                st = SDB_CORRUPT_BLOCK;
                break;
            }
            curlen = r.shared + r.unshared;
            ent++;
            kb += curlen;
            pos = r.next;
        }
    }
    t.status = __shfl(st, 0, 64);
    t.entries = __shfl(ent, 0, 64);
    t.key_bytes = __shfl(kb, 0, 64);
    return t;
}

SDB_DEV Tally tally_v1(const BlockView &v) {
    Tally t{0, 0, 0, false};
    const int l = lane_id();
    const uint32_t R = v.count;
    if (R == 0) return t;
    // decode_first_key (block_iterator.rs:235-242)
    if (v.data_end < 4 || rd_be(v.d, 2) != 0 || 4 + rd_be(v.d + 2, 2) > v.data_end) {
        t.status = SDB_CORRUPT_BLOCK;
        return t;
    }
    const uint32_t fk = (uint32_t)rd_be(v.d + 2, 2);
    uint64_t kb = 0;
    int st = 0;
    uint64_t bad_first = ~0ull;
    for (uint32_t i = l; i < R; i += 64) {
        RowV0 r;
        int s = parse_v0(v.d, v.data_end, (uint32_t)rd_be(v.offs + 2 * i, 2), &r);
        if (!s && r.prefix > fk) s = SDB_CORRUPT_BLOCK;
        if (s) {
            if (i < bad_first) {
                bad_first = i;
                st = s;
            }
            continue;
        }
        kb += r.prefix + r.suf;
    }
    // lowest failing entry wins
    uint64_t mn = bad_first;
#pragma unroll
    for (int d = 32; d >= 1; d >>= 1) {
        uint64_t o = __shfl_xor(mn, d, 64);
        mn = o < mn ? o : mn;
    }
    if (mn != ~0ull) {
        uint64_t owner = __ballot(bad_first == mn);
        t.status = __shfl(st, __builtin_ctzll(owner), 64);
        return t;
    }
    t.entries = R;
    t.key_bytes = wave_sum(kb);
    return t;
}

__global__ __launch_bounds__(256) void k_dec_count(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t(*crc)[256] = (uint32_t(*)[256])smem;
    for (uint32_t q = threadIdx.x; q < 8 * 256; q += blockDim.x) ((uint32_t *)crc)[q] = (&c_crc.t[0][0])[q];
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    uint8_t *stage = smem + 8192 + wave * (kDecCap + 64);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k < a.nblocks; k += nwaves) {
        BlockView v = load_block(a, k, stage, crc);
        Tally t{0, 0, v.status, false};
        if (!v.status) t = (a.version == 2) ? tally_v2(v) : tally_v1(v);
        if (lane_id() == 0) {
            if (t.status) {
                a.cnt[k] = 0;
                a.kbytes[k] = 0;
                a.flag[k] = 0;
                atomicMin(a.err, (unsigned long long)((k << 8) | (uint64_t)t.status));
                unsigned long long slot = atomicAdd(a.nbad, 1ull);
                if (slot < a.bad_cap) a.bad_block[slot] = (uint32_t)k;
            } else {
                a.cnt[k] = t.entries;
                a.kbytes[k] = t.key_bytes;
                a.flag[k] = t.sequential ? 1 : 0;
            }
        }
        wave_sync_d();
    }
}

// --- emit -----------------------------------------------------------------------------------------
SDB_DEV void put_entry(const DecodeArgs &a, uint64_t idx, uint64_t kpos, uint32_t klen, uint64_t vref,
                       uint32_t vlen, uint64_t seq, uint8_t flags, int64_t cts, int64_t ets) {
    a.out.key_off[idx] = kpos;
    a.out.val_off[idx] = vlen ? vref : 0;
    a.out.val_len[idx] = vlen;
    a.out.seq[idx] = seq;
    a.out.flags[idx] = flags;
    a.out.create_ts[idx] = (flags & SDB_FLAG_HAS_CREATE_TS) ? cts : 0;
    a.out.expire_ts[idx] = (flags & SDB_FLAG_HAS_EXPIRE_TS) ? ets : 0;
    (void)klen;
}

__global__ __launch_bounds__(256) void k_dec_emit(DecodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    uint32_t(*crc)[256] = (uint32_t(*)[256])smem;
    for (uint32_t q = threadIdx.x; q < 8 * 256; q += blockDim.x) ((uint32_t *)crc)[q] = (&c_crc.t[0][0])[q];
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6;
    const int l = lane_id();
    uint8_t *stage = smem + 8192 + wave * (kDecCap + 64);
    const uint64_t nwaves = (uint64_t)gridDim.x * (blockDim.x >> 6);
    // capacity guard: if the counted output does not fit the caller's arrays, write nothing
    if (a.ent_start[a.nblocks] > a.out.cap_entries || a.key_start[a.nblocks] > a.out.key_arena_cap) return;
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k < a.nblocks; k += nwaves) {
        const uint64_t ent0 = a.ent_start[k];
        const uint64_t n_ent = a.ent_start[k + 1] - ent0;
        if (l == 0) a.out.block_entry_start[k] = ent0;
        if (n_ent == 0) continue;
        BlockView v = load_block(a, k, stage, crc);
        if (v.status) continue;  // cannot happen: count pass accepted it
        const uint64_t kb0 = a.key_start[k];
        const uint64_t gbase = a.block_off[k];
        // value references are offsets into `blocks`; d may be LDS (staged) or HBM
        const uint8_t *g = a.blocks + gbase;
        if (a.version == 1) {
            const uint32_t R = v.count;
            const uint32_t fk = (uint32_t)rd_be(v.d + 2, 2);
            // key positions: exclusive scan of restored key lengths over the entries
            uint64_t carry = kb0;
            for (uint32_t g0 = 0; g0 < R; g0 += 64) {
                uint32_t i = g0 + l;
                RowV0 r;
                uint32_t kl = 0;
                if (i < R) {
                    parse_v0(v.d, v.data_end, (uint32_t)rd_be(v.offs + 2 * i, 2), &r);
                    kl = r.prefix + r.suf;
                }
                uint64_t inc = wave_incl_scan((uint64_t)kl);
                if (i < R) {
                    uint64_t kp = carry + inc - kl;
                    uint8_t *dst = a.out.key_arena + kp;
                    for (uint32_t q = 0; q < r.prefix; q++) dst[q] = v.d[4 + q];
                    for (uint32_t q = 0; q < r.suf; q++) dst[r.prefix + q] = v.d[r.suf_pos + q];
                    put_entry(a, ent0 + i, kp, kl, gbase + r.val_pos, r.vlen, r.seq, r.flags, r.cts, r.ets);
                }
                carry += __shfl(inc, 63, 64);
            }
            (void)fk;
            (void)g;
        } else if (!a.flag[k]) {
            // regular: lane q owns restart region q; entry/key bases by wave scans over regions
            const uint32_t R = v.count;
            uint64_t ecarry = ent0, kcarry = kb0;
            for (uint32_t q0 = 0; q0 < R; q0 += 64) {
                uint32_t q = q0 + l;
                uint32_t pos = 0, end = 0, ne = 0, nk = 0;
                if (q < R) {
                    pos = (uint32_t)rd_be(v.offs + 2 * q, 2);
                    end = (q + 1 < R) ? (uint32_t)rd_be(v.offs + 2 * q + 2, 2) : v.data_end;
                    uint32_t p = pos;
                    while (p < end) {
                        RowV2 r;
                        parse_v2(v.d, v.data_end, p, &r);
                        ne++;
                        nk += r.shared + r.unshared;
                        p = r.next;
                    }
                }
                uint64_t ie = wave_incl_scan((uint64_t)ne), ik = wave_incl_scan((uint64_t)nk);
                uint64_t idx = ecarry + ie - ne, kp = kcarry + ik - nk;
                if (q < R) {
                    uint64_t prev_kp = 0;
                    uint32_t p = pos;
                    while (p < end) {
                        RowV2 r;
                        parse_v2(v.d, v.data_end, p, &r);
                        uint8_t *dst = a.out.key_arena + kp;
                        const uint8_t *pk = a.out.key_arena + prev_kp;
                        for (uint32_t x = 0; x < r.shared; x++) dst[x] = pk[x];
                        for (uint32_t x = 0; x < r.unshared; x++) dst[r.shared + x] = v.d[r.suf_pos + x];
                        uint32_t vl = (r.flags & SDB_FLAG_TOMBSTONE) ? 0 : r.vlen;
                        put_entry(a, idx, kp, r.shared + r.unshared, gbase + r.val_pos, vl, r.seq, r.flags, r.cts,
                                  r.ets);
                        prev_kp = kp;
                        kp += r.shared + r.unshared;
                        idx++;
                        p = r.next;
                    }
                }
                ecarry += __shfl(ie, 63, 64);
                kcarry += __shfl(ik, 63, 64);
            }
        } else if (l == 0) {
            // sequential walk (BlockIteratorV2 ascending)
            uint64_t idx = ent0, kp = kb0, prev_kp = 0;
            uint32_t pos = 0;
            // initial current_key = key at restart 0
            uint32_t p0 = (uint32_t)rd_be(v.offs, 2), sh = 0, un = 0, vl0 = 0;
            rd_varint(v.d, v.data_end, &p0, &sh);
            rd_varint(v.d, v.data_end, &p0, &un);
            rd_varint(v.d, v.data_end, &p0, &vl0);
            const uint8_t *init_key = v.d + p0;
            bool first = true;
            while (pos < v.data_end) {
                RowV2 r;
                parse_v2(v.d, v.data_end, pos, &r);
                uint8_t *dst = a.out.key_arena + kp;
                for (uint32_t x = 0; x < r.shared; x++) dst[x] = first ? init_key[x] : a.out.key_arena[prev_kp + x];
                for (uint32_t x = 0; x < r.unshared; x++) dst[r.shared + x] = v.d[r.suf_pos + x];
                uint32_t vl = (r.flags & SDB_FLAG_TOMBSTONE) ? 0 : r.vlen;
                put_entry(a, idx, kp, r.shared + r.unshared, gbase + r.val_pos, vl, r.seq, r.flags, r.cts, r.ets);
                prev_kp = kp;
                kp += r.shared + r.unshared;
                idx++;
                first = false;
                pos = r.next;
            }
        }
        wave_sync_d();
    }
}

// --- scans ------------------------------------------------------------------------------------------
constexpr uint32_t kScanTile = 1024;

__global__ __launch_bounds__(1024) void k_scan_tiles(const uint64_t *x, const uint64_t *y, uint64_t n,
                                                     uint64_t *tx, uint64_t *ty) {
    __shared__ uint64_t s_w[17];
    uint64_t i = (uint64_t)blockIdx.x * kScanTile + threadIdx.x;
    uint64_t vx = i < n ? x[i] : 0, vy = i < n ? y[i] : 0;
    uint64_t sx, sy;
    block_excl_scan_u64(vx, s_w, &sx);
    block_excl_scan_u64(vy, s_w, &sy);
    if (threadIdx.x == 0) {
        tx[blockIdx.x] = sx;
        ty[blockIdx.x] = sy;
    }
}

__global__ __launch_bounds__(1024) void k_scan_top(uint64_t *tx, uint64_t *ty, uint64_t nt) {
    __shared__ uint64_t s_w[17];
    uint64_t cx = 0, cy = 0;
    for (uint64_t b = 0; b < nt; b += kScanTile) {
        uint64_t i = b + threadIdx.x;
        uint64_t vx = i < nt ? tx[i] : 0, vy = i < nt ? ty[i] : 0;
        uint64_t sx, sy;
        uint64_t ex = block_excl_scan_u64(vx, s_w, &sx);
        uint64_t ey = block_excl_scan_u64(vy, s_w, &sy);
        if (i < nt) {
            tx[i] = cx + ex;
            ty[i] = cy + ey;
        }
        cx += sx;
        cy += sy;
    }
    if (threadIdx.x == 0) {
        tx[nt] = cx;
        ty[nt] = cy;
    }
}

__global__ __launch_bounds__(1024) void k_scan_apply(const uint64_t *x, const uint64_t *y, uint64_t n,
                                                     const uint64_t *tx, const uint64_t *ty, uint64_t nt,
                                                     uint64_t *ox, uint64_t *oy) {
    __shared__ uint64_t s_w[17];
    uint64_t i = (uint64_t)blockIdx.x * kScanTile + threadIdx.x;
    uint64_t vx = i < n ? x[i] : 0, vy = i < n ? y[i] : 0;
    uint64_t sx, sy;
    uint64_t ex = block_excl_scan_u64(vx, s_w, &sx);
    uint64_t ey = block_excl_scan_u64(vy, s_w, &sy);
    if (i < n) {
        ox[i] = tx[blockIdx.x] + ex;
        oy[i] = ty[blockIdx.x] + ey;
    }
    if (i == n - 1) {
        ox[n] = tx[nt];
        oy[n] = ty[nt];
    }
}

__global__ void k_dec_init(DecodeArgs a) {
    if (threadIdx.x == 0) {
        *a.err = ~0ull;
        *a.nbad = 0;
    }
}

__global__ void k_dec_finish(DecodeArgs a) {
    if (threadIdx.x == 0) {
        sdb_decode_summary *s = a.out.summary;
        uint64_t ne = a.ent_start[a.nblocks], kb = a.key_start[a.nblocks];
        s->num_entries = ne;
        s->key_bytes = kb;
        s->num_bad_blocks = *a.nbad;
        unsigned long long e = *a.err;
        s->status = e == ~0ull ? 0 : (int32_t)(e & 0xFF);
        s->pad = 0;
        a.out.block_entry_start[a.nblocks] = ne;
        if (ne > a.out.cap_entries || kb > a.out.key_arena_cap) s->status = SDB_INVALID_ARGUMENT;
        else a.out.key_off[ne] = kb;
    }
}

hipError_t launch_decode(DecodeArgs a, hipStream_t st) {
    hipLaunchKernelGGL(k_dec_init, dim3(1), dim3(64), 0, st, a);
    const size_t lds = 8192 + 4 * (kDecCap + 64);
    uint64_t waves = a.nblocks;
    uint64_t wgs = (waves + 3) / 4;
    if (wgs > 4096) wgs = 4096;
    if (wgs == 0) wgs = 1;
    if (a.nblocks) hipLaunchKernelGGL(k_dec_count, dim3((uint32_t)wgs), dim3(256), lds, st, a);
    // scans: ent_start = excl(cnt), key_start = excl(kbytes)
    uint64_t nt = (a.nblocks + kScanTile - 1) / kScanTile;
    if (a.nblocks) {
        hipLaunchKernelGGL(k_scan_tiles, dim3((uint32_t)nt), dim3(kScanTile), 0, st, a.cnt, a.kbytes, a.nblocks,
                           a.tile_x, a.tile_y);
        hipLaunchKernelGGL(k_scan_top, dim3(1), dim3(kScanTile), 0, st, a.tile_x, a.tile_y, nt);
        hipLaunchKernelGGL(k_scan_apply, dim3((uint32_t)nt), dim3(kScanTile), 0, st, a.cnt, a.kbytes, a.nblocks,
                           a.tile_x, a.tile_y, nt, a.ent_start, a.key_start);
    } else {
        hipMemsetAsync(a.ent_start, 0, 8, st);
        hipMemsetAsync(a.key_start, 0, 8, st);
    }
    if (a.nblocks) hipLaunchKernelGGL(k_dec_emit, dim3((uint32_t)wgs), dim3(256), lds, st, a);
    hipLaunchKernelGGL(k_dec_finish, dim3(1), dim3(64), 0, st, a);
    return hipGetLastError();
}

}  // namespace sdb
