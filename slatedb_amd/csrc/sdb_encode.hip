// sdb_encode.hip — SST data-section encoder for gfx950.
//
// Replaces EncodedSsTableBuilder::{add, finish_block, build} (slatedb/src/sst_builder.rs:224-417)
// with BlockBuilderV2/V1 (format/block_v2.rs:118-240, format/block.rs:76-218), the row codecs
// (format/row_codec_v2.rs:127-169, format/row.rs:159-198) and the per-block CRC32 of
// compress_and_transform (format/sst.rs:525-554).
//
// The greedy block fill of the reference (BlockBuilderV2::would_fit, block_v2.rs:151-164) is a
// sequential chain b -> next(b).  It is parallelised as:
//   K1 prep     one thread per entry: LCP vs previous key, restart/non-restart row sizes, checks,
//               stats.
//   K2 next     one thread per entry b: next(b) = end of a block that would start at b, and its
//               encoded size.
//   K3 chunk    one workgroup per chunk of kChunk entries: pointer jumping in LDS gives, for every
//               entry point e of the chunk, the first block start past the chunk plus the blocks
//               and bytes on the way (a chunk transfer table).
//   K4 resolve  one workgroup: the chunk tables are composed by a Blelloch up-sweep in LDS and the
//               single chain from entry 0 is pushed down the tree (O(log K) depth) -> per-chunk
//               anchors (first block start, block index, byte offset).
//   K5 emit     one workgroup per chunk: binary lifting enumerates the chunk's block starts, then
//               one wave per block stages the block's keys/values in LDS with 16-byte loads,
//               assembles the rows, restart table and count in an LDS image, computes the CRC32
//               (slicing-by-8 per lane + GF(2) shift-combine across the wave) and writes the block
//               with 16-byte stores.
//   K6 slow     blocks larger than the LDS image (oversized first entries, huge block sizes) are
//               assembled directly in HBM by one workgroup each.
#include "sdb_device.h"
#include "sdb_encode.h"

namespace sdb {


// ------------------------------------------------------------------------------------------------
// K1: per-entry prep
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_prep(EncodeArgs a) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    uint64_t rk = 0, rv = 0;
    uint32_t puts = 0, dels = 0, merges = 0;
    if (i < a.n) {
        uint64_t ko0 = a.key_off[i], ko1 = a.key_off[i + 1];
        uint64_t klen = ko1 - ko0;
        uint8_t kd = a.kind ? a.kind[i] : 0;
        uint8_t m = a.ts_mask ? a.ts_mask[i] : 0;
        uint64_t vlen = (kd == SDB_KIND_TOMBSTONE) ? 0 : (a.val_off[i + 1] - a.val_off[i]);
        uint32_t lcp = 0;
        int err = 0;
        if (kd > SDB_KIND_TOMBSTONE) err = SDB_INVALID_ARGUMENT;
        if (!err && i > 0) {
            uint64_t pko = a.key_off[i - 1];
            uint64_t plen = ko0 - pko;
            uint32_t nmin = (uint32_t)((plen < klen ? plen : klen) > 0xFFFFFFFFull ? 0xFFFFFFFFull
                                                                                  : (plen < klen ? plen : klen));
            lcp = lcp_bytes(a.key_bytes + pko, nmin, a.key_bytes + ko0, nmin);
            // compute_index_key runs on every entry (sst_builder.rs:228): assert on empty keys and
            // out-of-bounds panic when this key is a proper prefix of the previous one (utils.rs:210-216)
            if (klen == 0) err = SDB_EMPTY_KEY;
            else if (plen > 0 && lcp == klen && klen < plen) err = SDB_INVALID_ARGUMENT;
        }
        if (!err && klen == 0) err = SDB_EMPTY_KEY;  // BlockBuilder*::add (block_v2.rs:168-170)
        const uint32_t ts8 = 8u * (((m & SDB_TS_CREATE) != 0) + ((m & SDB_TS_EXPIRE) != 0));
        if (a.version == 2) {
            if (!err && (klen > 0xFFFFFFFFull || vlen > 0xFFFFFFFFull)) err = SDB_LIMIT_EXCEEDED;
            uint32_t kl = (uint32_t)klen, vl = (uint32_t)vlen, suf = kl - lcp;
            // SstRowEntryV2::encoded_size (row_codec_v2.rs:92-116)
            a.s_nr[i] = varint_len(lcp) + varint_len(suf) + varint_len(vl) + suf + vl + 9 + ts8;
            a.s_r[i] = 1 + varint_len(kl) + varint_len(vl) + kl + vl + 9 + ts8;
        } else {
            // SstRowEntry::new asserts (row.rs:73-85)
            if (!err && (klen > 0xFFFF || vlen > 0xFFFFFFFFull)) err = SDB_LIMIT_EXCEEDED;
            // RowEntry::encoded_size with key_prefix_len = 0 (types.rs:64-83)
            a.s_r[i] = (uint32_t)(4 + klen + 9 + ts8 + (kd == SDB_KIND_TOMBSTONE ? 0 : 4 + vlen));
        }
        a.lcp[i] = lcp;
        if (err) report_error(a.err, i, err);
        rk = klen;
        rv = vlen;
        puts = kd == SDB_KIND_VALUE;
        merges = kd == SDB_KIND_MERGE;
        dels = kd == SDB_KIND_TOMBSTONE;
    }
    // SstStats (sst_builder.rs:225-226, 315-317): per-workgroup partials, summed in k_resolve
    __shared__ uint64_t s_part[4][5];
    rk = wave_sum(rk);
    rv = wave_sum(rv);
    uint32_t c = wave_sum(puts | (dels << 10) | (merges << 20));  // <= 64 each per wave
    const uint32_t w = threadIdx.x >> 6;
    if (lane_id() == 0) {
        s_part[w][0] = rk;
        s_part[w][1] = rv;
        s_part[w][2] = c & 0x3FF;
        s_part[w][3] = (c >> 10) & 0x3FF;
        s_part[w][4] = (c >> 20) & 0x3FF;
    }
    __syncthreads();
    if (threadIdx.x < 5) {
        uint64_t t = 0;
        for (uint32_t q = 0; q < (blockDim.x >> 6); q++) t += s_part[q][threadIdx.x];
        a.stat_part[5 * (uint64_t)blockIdx.x + threadIdx.x] = t;
    }
}

// ------------------------------------------------------------------------------------------------
// K2: next(b) for every entry b (BlockBuilderV2::would_fit / BlockBuilderV1::would_fit)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_next(EncodeArgs a) {
    // sizes of [b0, b0 + kNextSpan) staged in LDS; a scan that runs past it continues from HBM
    __shared__ uint32_t s_r[kNextSpan], s_nr[kNextSpan];
    const uint64_t b0 = (uint64_t)blockIdx.x * blockDim.x;
    const uint64_t b = b0 + threadIdx.x;
    const uint64_t lim = b0 + kNextSpan < a.n ? b0 + kNextSpan : a.n;
    for (uint64_t j = b0 + threadIdx.x; j < lim; j += blockDim.x) {
        s_r[j - b0] = a.s_r[j];
        if (a.version == 2) s_nr[j - b0] = a.s_nr[j];
    }
    __syncthreads();
    uint32_t len = 0;
    if (b < a.n) {
        const uint64_t bs = a.block_size;
        uint64_t acc = 2;  // Block::size of an empty block: data 0 + offsets 0 + count 2
        uint64_t j = b;
        uint32_t p = 0;
        if (a.version == 2) {
            const uint32_t ri = a.restart_interval;
            uint32_t ph = 0;  // p % ri
            while (j < a.n) {
                bool rs = ph == 0;
                uint32_t sz;
                if (j < lim) sz = rs ? s_r[j - b0] : s_nr[j - b0];
                else sz = rs ? a.s_r[j] : a.s_nr[j];
                uint64_t add = (uint64_t)sz + (rs ? 2 : 0);
                if (p > 0 && acc + add > bs) break;
                acc += add;
                j++;
                p++;
                if (++ph == ri) ph = 0;
            }
        } else {
            const uint64_t fko = a.key_off[b];
            const uint32_t fkl = (uint32_t)(a.key_off[b + 1] - fko);
            while (j < a.n) {
                uint32_t prefix = 0;
                if (p > 0) {
                    uint64_t ko = a.key_off[j];
                    prefix = lcp_bytes(a.key_bytes + fko, fkl, a.key_bytes + ko, (uint32_t)(a.key_off[j + 1] - ko));
                }
                uint64_t sz = (uint64_t)(j < lim ? s_r[j - b0] : a.s_r[j]) - prefix;
                if (p > 0 && acc + sz > bs) break;  // the new entry's 2-byte offset is not counted (block.rs:117-123)
                acc += sz + 2;
                j++;
                p++;
            }
        }
        a.next[b] = (uint32_t)j;
        a.bbytes[b] = (uint32_t)(acc + 4);  // + CRC32 (format/sst.rs:541-552)
        len = (uint32_t)(j - b);
    }
    // longest candidate block: per-workgroup partial (a single global atomicMax target would
    // serialise ~10^4 wave atomics at the memory side), reduced in k_resolve
    __shared__ uint32_t s_len[4];
    len = wave_max(len);
    if (lane_id() == 0) s_len[threadIdx.x >> 6] = len;
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t m = 0;
        for (uint32_t q = 0; q < (blockDim.x >> 6); q++) m = s_len[q] > m ? s_len[q] : m;
        a.wmax_part[blockIdx.x] = m;
    }
}

// ------------------------------------------------------------------------------------------------
// K3: chunk transfer tables by pointer jumping in LDS
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(512) void k_chunk(EncodeArgs a) {
    __shared__ uint32_t s_s[2][kChunk];
    __shared__ uint32_t s_c[2][kChunk];
    __shared__ uint64_t s_b[2][kChunk];
    const uint64_t cs = (uint64_t)blockIdx.x * kChunk;
    const uint64_t ce = cs + kChunk < a.n ? cs + kChunk : a.n;
    const uint32_t cn = (uint32_t)(ce - cs);
    for (uint32_t e = threadIdx.x; e < cn; e += blockDim.x) {
        s_s[0][e] = a.next[cs + e];
        s_c[0][e] = 1;
        s_b[0][e] = a.bbytes[cs + e];
    }
    __syncthreads();
    int cur = 0;
    for (int round = 0; round < 24; round++) {
        int changed = 0;
        for (uint32_t e = threadIdx.x; e < cn; e += blockDim.x) {
            uint32_t s = s_s[cur][e], c = s_c[cur][e];
            uint64_t by = s_b[cur][e];
            if (s < ce) {
                uint32_t t = s - (uint32_t)cs;
                c += s_c[cur][t];
                by += s_b[cur][t];
                s = s_s[cur][t];
                changed = 1;
            }
            s_s[cur ^ 1][e] = s;
            s_c[cur ^ 1][e] = c;
            s_b[cur ^ 1][e] = by;
        }
        cur ^= 1;
        if (!__syncthreads_or(changed)) break;
    }
    for (uint32_t e = threadIdx.x; e < cn; e += blockDim.x) {
        a.tab_exit[cs + e] = s_s[cur][e];
        a.tab_cnt[cs + e] = s_c[cur][e];
        a.tab_bytes[cs + e] = s_b[cur][e];
    }
}

// ------------------------------------------------------------------------------------------------
// K4: resolve chunk anchors (single workgroup)
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(1024) void k_resolve(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    __shared__ uint64_t s_w[17];
    __shared__ uint32_t s_fast;
    const uint32_t K = a.nchunks;
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    uint32_t KP = 1;
    while (KP < K) KP <<= 1;
    __shared__ uint32_t s_wmax;
    if (tid == 0) s_wmax = 0;
    __syncthreads();
    {
        uint32_t m = 0;
        for (uint32_t q = tid; q < a.nprep_wg; q += nt) m = a.wmax_part[q] > m ? a.wmax_part[q] : m;
        m = wave_max(m);
        if (lane_id() == 0) atomicMax(&s_wmax, m);
    }
    __syncthreads();
    const uint32_t W = s_wmax;
    if (tid == 0) *a.wmax = W;
    // LDS: ex (KP*W u16) + v (KP u32) + tmp (KP/2*W u16), each 16-byte aligned
    if (tid == 0)
        s_fast = (W <= kChunk && (((uint64_t)KP * W * 2 + 15) & ~15ull) + ((4ull * KP + 15) & ~15ull) +
                                         (uint64_t)KP * W + 16 <= kResolveLds)
                     ? 1u
                     : 0u;
    __syncthreads();
    if (s_fast) {
        uint16_t *ex = (uint16_t *)smem;                               // KP x W exit offsets
        uint32_t *v = (uint32_t *)(smem + (((uint64_t)KP * W * 2 + 15) & ~15ull));  // KP entry offsets
        // ex[k][o] = entry offset into chunk k+1 reached from entry offset o into chunk k
        for (uint64_t idx = tid; idx < (uint64_t)KP * W; idx += nt) {
            uint32_t k = (uint32_t)(idx / W), o = (uint32_t)(idx % W);
            uint16_t val = (uint16_t)o;  // identity for the padding chunks k >= K
            if (k < K) {
                uint64_t cs = (uint64_t)k * kChunk;
                uint64_t ce = cs + kChunk < a.n ? cs + kChunk : a.n;
                val = 0;
                if (cs + o < ce) val = (uint16_t)(a.tab_exit[cs + o] - ce);
            }
            ex[idx] = val;
        }
        __syncthreads();
        // Blelloch up-sweep: ex[k] <- ex[k] o ex[k-d] for k = 2d-1 (mod 2d).  A level reads entries
        // of ex[k] that other threads of the same level overwrite, so results go through `tmp`.
        uint16_t *tmp = (uint16_t *)(smem + (((uint64_t)KP * W * 2 + 15) & ~15ull) + (((uint64_t)KP * 4 + 15) & ~15ull));
        for (uint32_t d = 1; d < KP; d <<= 1) {
            uint32_t nodes = KP / (2 * d);
            for (uint64_t idx = tid; idx < (uint64_t)nodes * W; idx += nt) {
                uint32_t q = (uint32_t)(idx / W), o = (uint32_t)(idx % W);
                uint32_t k = 2 * d * q + 2 * d - 1;
                uint16_t mid = ex[(uint64_t)(k - d) * W + o];
                tmp[idx] = ex[(uint64_t)k * W + mid];
            }
            __syncthreads();
            for (uint64_t idx = tid; idx < (uint64_t)nodes * W; idx += nt) {
                uint32_t q = (uint32_t)(idx / W), o = (uint32_t)(idx % W);
                uint32_t k = 2 * d * q + 2 * d - 1;
                ex[(uint64_t)k * W + o] = tmp[idx];
            }
            __syncthreads();
        }
        // down-sweep of the single chain that starts at entry 0
        if (tid == 0) v[0] = 0;
        __syncthreads();
        for (uint32_t d = KP >> 1; d >= 1; d >>= 1) {
            for (uint32_t q = tid; q < KP / (2 * d); q += nt) {
                uint32_t k = 2 * d * q;
                v[k + d] = ex[(uint64_t)(k + d - 1) * W + v[k]];
            }
            __syncthreads();
        }
        for (uint32_t k = tid; k < K; k += nt) a.anchor_e[k] = (uint32_t)((uint64_t)k * kChunk + v[k]);
    } else if (tid == 0) {
        // general fallback (a block longer than a chunk, or too many chunk tables): serial walk
        uint64_t e = 0;
        for (uint32_t k = 0; k < K; k++) {
            uint64_t cs = (uint64_t)k * kChunk;
            uint64_t ce = cs + kChunk < a.n ? cs + kChunk : a.n;
            a.anchor_e[k] = (uint32_t)e;
            if (e < ce) e = a.tab_exit[e];
        }
    }
    __threadfence();
    __syncthreads();
    // per-chunk block counts / bytes from the entry point; exclusive scans give the anchors
    uint64_t cb = 0, cy = 0;
    for (uint32_t k0 = 0; k0 < K; k0 += nt) {
        uint32_t k = k0 + tid;
        uint64_t c = 0, by = 0;
        if (k < K) {
            uint64_t cs = (uint64_t)k * kChunk;
            uint64_t ce = cs + kChunk < a.n ? cs + kChunk : a.n;
            uint64_t e = a.anchor_e[k];
            if (e < ce) {
                c = a.tab_cnt[e];
                by = a.tab_bytes[e];
            }
        }
        uint64_t tc, ty;
        uint64_t xc = block_excl_scan_u64(c, s_w, &tc);
        uint64_t xy = block_excl_scan_u64(by, s_w, &ty);
        if (k < K) {
            a.anchor_blk[k] = (uint32_t)(cb + xc);
            a.anchor_byte[k] = cy + xy;
        }
        cb += tc;
        cy += ty;
    }
    // SstStats totals from the k_prep partials
    for (uint32_t f = 0; f < 5; f++) {
        uint64_t t = 0;
        for (uint32_t q = tid; q < a.nprep_wg; q += nt) t += a.stat_part[5 * (uint64_t)q + f];
        uint64_t tot;
        block_excl_scan_u64(t, s_w, &tot);
        if (tid == 0) {
            if (f == 0) a.summary->raw_key_size = tot;
            if (f == 1) a.summary->raw_val_size = tot;
            if (f == 2) a.summary->num_puts = tot;
            if (f == 3) a.summary->num_deletes = tot;
            if (f == 4) a.summary->num_merges = tot;
        }
    }
    if (tid == 0) {
        a.anchor_blk[K] = (uint32_t)cb;
        a.anchor_byte[K] = cy;
        a.anchor_e[K] = (uint32_t)a.n;
        a.summary->num_blocks = cb;
        a.summary->data_len = cy;
        a.summary->num_entries = a.n;
        if (cb > a.block_cap || cy > a.data_cap) report_error(a.err, 0, SDB_INVALID_ARGUMENT);
    }
}

// ------------------------------------------------------------------------------------------------
// K5: emit
// ------------------------------------------------------------------------------------------------
struct RowInfo {
    uint64_t key_src;   // global byte offset (into key_bytes) of the key suffix
    uint64_t val_src;   // global byte offset (into val_bytes) of the value
    uint32_t suf, vlen; // suffix / value length
    uint32_t shared;
    uint32_t row_off;   // offset of the row in the block
    uint32_t size;
    uint8_t flags;
};

// Encode the row described by (r, seq, ts) into `dst` (LDS or global) byte by byte for the small
// fields; values and key suffixes come from `ksrc`/`vsrc` (LDS staging or global).
template <int V>
SDB_DEV void write_row_small(uint8_t *dst, const RowInfo &r, uint64_t seq, int64_t ets, int64_t cts,
                             uint32_t *hdr_len_out) {
    uint32_t p = 0;
    if (V == 2) {  // SstRowCodecV2::encode (row_codec_v2.rs:127-169)
        uint32_t vals[3] = {r.shared, r.suf, r.vlen};
#pragma unroll
        for (int f = 0; f < 3; f++) {
            uint32_t x = vals[f];
            while (x >= 0x80) {
                dst[p++] = (uint8_t)(x | 0x80);
                x >>= 7;
            }
            dst[p++] = (uint8_t)x;
        }
    } else {  // SstRowCodecV0::encode (row.rs:159-198)
        dst[p++] = (uint8_t)(r.shared >> 8);
        dst[p++] = (uint8_t)r.shared;
        dst[p++] = (uint8_t)(r.suf >> 8);
        dst[p++] = (uint8_t)r.suf;
    }
    *hdr_len_out = p;
    // trailer after key suffix (+ value for V2)
    uint32_t t = p + r.suf + (V == 2 ? r.vlen : 0);
#pragma unroll
    for (int q = 0; q < 8; q++) dst[t++] = (uint8_t)(seq >> (56 - 8 * q));
    dst[t++] = r.flags;
    if (r.flags & SDB_FLAG_HAS_EXPIRE_TS)
#pragma unroll
        for (int q = 0; q < 8; q++) dst[t++] = (uint8_t)((uint64_t)ets >> (56 - 8 * q));
    if (r.flags & SDB_FLAG_HAS_CREATE_TS)
#pragma unroll
        for (int q = 0; q < 8; q++) dst[t++] = (uint8_t)((uint64_t)cts >> (56 - 8 * q));
    if (V == 1 && !(r.flags & SDB_FLAG_TOMBSTONE)) {
        dst[t++] = (uint8_t)(r.vlen >> 24);
        dst[t++] = (uint8_t)(r.vlen >> 16);
        dst[t++] = (uint8_t)(r.vlen >> 8);
        dst[t++] = (uint8_t)r.vlen;
    }
}

// Byte-granular copy between LDS regions with dword realignment (dst, src arbitrary alignment).
SDB_DEV void lds_copy(uint8_t *dst, const uint8_t *src, uint32_t n) {
    uint32_t i = 0;
    while (i < n && (((uintptr_t)(dst + i)) & 3)) {
        dst[i] = src[i];
        i++;
    }
    if (i + 4 <= n) {
        uintptr_t sa = (uintptr_t)(src + i);
        uint32_t sh = (uint32_t)(sa & 3);
        const uint32_t *sw = (const uint32_t *)(sa - sh);
        uint32_t *dw = (uint32_t *)(dst + i);
        uint32_t nw = (n - i) >> 2;
        if (sh == 0) {
            for (uint32_t w = 0; w < nw; w++) dw[w] = sw[w];
        } else {
            uint32_t lo = sw[0];
            for (uint32_t w = 0; w < nw; w++) {
                uint32_t hi = sw[w + 1];
                dw[w] = __builtin_amdgcn_alignbyte(hi, lo, sh);
                lo = hi;
            }
        }
        i += nw * 4;
    }
    while (i < n) {
        dst[i] = src[i];
        i++;
    }
}

SDB_DEV void wave_sync() {
    __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
    __builtin_amdgcn_wave_barrier();
    __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
}

// Stage global bytes [g0, g1) into LDS so that stage[x - (g0 & ~15)] = g[x].  One wave, 16-byte
// loads (every loaded 16-byte granule holds at least one requested byte).
SDB_DEV void wave_stage(uint8_t *stage, const uint8_t *g, uint64_t g0, uint64_t g1) {
    if (g1 <= g0) return;
    uint64_t a0 = g0 & ~15ull, a1 = (g1 + 15) & ~15ull;
    uint32_t nchunk = (uint32_t)((a1 - a0) >> 4);
    const uint4 *src = (const uint4 *)(g + a0);
    uint4 *dst = (uint4 *)stage;
    for (uint32_t c = lane_id(); c < nchunk; c += 64) dst[c] = src[c];
}

// Store LDS image bytes [0, len) to global [dst, dst+len); image byte 0 sits at img + (dst & 15).
SDB_DEV void wave_store(uint8_t *gdst, const uint8_t *img, uint64_t len) {
    uintptr_t d0 = (uintptr_t)gdst, d1 = d0 + len;
    uintptr_t a0 = d0 & ~(uintptr_t)15, a1 = (d1 + 15) & ~(uintptr_t)15;
    uint32_t nchunk = (uint32_t)((a1 - a0) >> 4);
    for (uint32_t c = lane_id(); c < nchunk; c += 64) {
        uintptr_t ga = a0 + 16 * (uintptr_t)c;
        const uint8_t *li = img + 16 * c;
        if (ga >= d0 && ga + 16 <= d1) {
            *(uint4 *)ga = *(const uint4 *)li;
        } else {
            for (int q = 0; q < 16; q++)
                if (ga + q >= d0 && ga + q < d1) ((uint8_t *)ga)[q] = li[q];
        }
    }
}

// ------------------------------------------------------------------------------------------------
// K5a: enumerate the blocks of each chunk (binary lifting over next()) -> BlockMeta offsets and the
//      per-block descriptors the emitter streams.
// ------------------------------------------------------------------------------------------------
__global__ __launch_bounds__(256) void k_enum(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    const uint32_t k = blockIdx.x;
    if (*a.err != ~0ull) return;
    const uint64_t cs = (uint64_t)k * kChunk;
    const uint64_t ce = cs + kChunk < a.n ? cs + kChunk : a.n;
    const uint32_t cn = (uint32_t)(ce - cs);
    const uint64_t e0 = a.anchor_e[k];
    const uint32_t blk0 = a.anchor_blk[k];
    const uint32_t nb = a.anchor_blk[k + 1] - blk0;
    const uint64_t byte0 = a.anchor_byte[k];
    const uint32_t tid = threadIdx.x, nt = blockDim.x;
    if (k + 1 == a.nchunks && tid == 0) {
        a.out_block_off[a.anchor_blk[k + 1]] = a.anchor_byte[k + 1];
        a.out_block_first[a.anchor_blk[k + 1]] = (uint32_t)a.n;
    }
    if (!nb) return;
    uint32_t *bl_s = (uint32_t *)smem;
    uint32_t *bl_b = bl_s + kChunk;
    uint64_t *bl_o = (uint64_t *)(bl_b + kChunk);
    uint16_t *lv = (uint16_t *)(bl_o + kChunk);
    uint32_t levels = 1;
    while ((1u << levels) < nb) levels++;
    for (uint32_t x = tid; x < cn; x += nt) {
        uint64_t nx = a.next[cs + x];
        lv[x] = (uint16_t)(nx >= ce ? cn : (uint32_t)(nx - cs));
    }
    __syncthreads();
    for (uint32_t j = 1; j < levels; j++) {
        uint16_t *src = lv + (uint64_t)(j - 1) * kChunk, *dst = lv + (uint64_t)j * kChunk;
        for (uint32_t x = tid; x < cn; x += nt) {
            uint16_t y = src[x];
            dst[x] = (y >= cn) ? (uint16_t)cn : src[y];
        }
        __syncthreads();
    }
    for (uint32_t t = tid; t < nb; t += nt) {
        uint32_t x = (uint32_t)(e0 - cs);
        for (uint32_t j = 0; j < levels; j++)
            if ((t >> j) & 1) x = lv[(uint64_t)j * kChunk + x];
        bl_s[t] = (uint32_t)cs + x;
        bl_b[t] = a.bbytes[cs + x];
    }
    __syncthreads();
    if (tid < 64) {
        uint64_t carry = byte0;
        for (uint32_t g = 0; g < nb; g += 64) {
            uint32_t t = g + tid;
            uint64_t v = t < nb ? bl_b[t] : 0;
            uint64_t inc = wave_incl_scan(v);
            if (t < nb) bl_o[t] = carry + inc - v;
            carry += __shfl(inc, 63, 64);
        }
    }
    __syncthreads();
    for (uint32_t t = tid; t < nb; t += nt) {
        uint64_t s = bl_s[t], e = a.next[s];
        uint32_t blk = blk0 + t;
        a.out_block_off[blk] = bl_o[t];
        a.out_block_first[blk] = (uint32_t)s;
        BlockDesc d;
        d.s = (uint32_t)s;
        d.e = (uint32_t)e;
        d.off = bl_o[t];
        d.vs = a.val_off[s];
        d.ve = a.val_off[e];
        d.ks = a.key_off[s];
        d.ke = a.key_off[e];
        d.bb = bl_b[t];
        d.pad = 0;
        a.desc[blk] = d;
    }
}

// ------------------------------------------------------------------------------------------------
// K5b: emit.  Persistent waves stream blocks (one block per wave at a time); each wave prefetches the
//      next block's values, keys and row metadata into registers while it assembles the current one
//      in LDS, so HBM latency overlaps the byte work.
// ------------------------------------------------------------------------------------------------
struct Pre {
    // wave-uniform block descriptor
    uint32_t blk, s, e, bb, nv16, nk16;
    uint64_t off, vs, ks;
    bool valid, fast;
    // staged 16-byte granules (value range: lane + 64 r; key range: lane)
    uint4 v[4];
    uint4 k;
    // this lane's row (lane < e - s)
    uint64_t ko, vo, seq;
    int64_t cts, ets;
    uint32_t klen, vlen, lcp, prev_klen;
    uint8_t kind, mask;
};

SDB_DEV void load_pre(const EncodeArgs &a, uint32_t blk, uint32_t nb, Pre &p) {
    const int l = lane_id();
    p.valid = blk < nb;
    p.fast = false;
    if (!p.valid) return;
    const BlockDesc d = a.desc[blk];
    p.blk = blk;
    p.s = d.s;
    p.e = d.e;
    p.bb = d.bb;
    p.off = d.off;
    p.vs = d.vs;
    p.ks = d.ks;
    const uint32_t ne = d.e - d.s;
    const uint64_t va = d.vs & ~15ull, ka = d.ks & ~15ull;
    p.nv16 = (uint32_t)((((d.ve + 15) & ~15ull) - va) >> 4);
    p.nk16 = (uint32_t)((((d.ke + 15) & ~15ull) - ka) >> 4);
    if (d.ve == d.vs) p.nv16 = 0;
    if (d.ke == d.ks) p.nk16 = 0;
    p.fast = ne <= 64 && p.nv16 <= 256 && p.nk16 <= 64 && (p.nv16 + p.nk16) * 16 <= kStageCap &&
             d.bb + 32 <= kImgCap;
    if (!p.fast) return;
    const uint4 *vsrc = (const uint4 *)(a.val_bytes + va);
#pragma unroll
    for (int r = 0; r < 4; r++) {
        uint32_t c = (uint32_t)l + 64u * r;
        p.v[r] = c < p.nv16 ? vsrc[c] : make_uint4(0, 0, 0, 0);
    }
    p.k = (uint32_t)l < p.nk16 ? ((const uint4 *)(a.key_bytes + ka))[l] : make_uint4(0, 0, 0, 0);
    if ((uint32_t)l < ne) {
        uint64_t j = d.s + l;
        p.ko = a.key_off[j];
        p.klen = (uint32_t)(a.key_off[j + 1] - p.ko);
        p.vo = a.val_off[j];
        p.kind = a.kind ? a.kind[j] : 0;
        p.mask = a.ts_mask ? a.ts_mask[j] : 0;
        p.vlen = p.kind == SDB_KIND_TOMBSTONE ? 0 : (uint32_t)(a.val_off[j + 1] - p.vo);
        p.lcp = a.lcp[j];
        p.seq = a.seq ? a.seq[j] : 0;
        p.cts = (p.mask & SDB_TS_CREATE) ? a.create_ts[j] : 0;
        p.ets = (p.mask & SDB_TS_EXPIRE) ? a.expire_ts[j] : 0;
        p.prev_klen = (l == 0 && d.s > 0) ? (uint32_t)(p.ko - a.key_off[j - 1]) : 0;
    } else {
        p.klen = p.vlen = p.lcp = p.prev_klen = 0;
        p.kind = p.mask = 0;
        p.ko = p.vo = p.seq = 0;
        p.cts = p.ets = 0;
    }
}

template <int V>
SDB_DEV void process_block(const EncodeArgs &a, const Pre &p, uint8_t *stage, uint8_t *img,
                           const uint32_t (*crc)[256]) {
    const int l = lane_id();
    const uint32_t ne = p.e - p.s;
    // 1. staged granules -> LDS
#pragma unroll
    for (int r = 0; r < 4; r++) {
        uint32_t c = (uint32_t)l + 64u * r;
        if (c < p.nv16) ((uint4 *)stage)[c] = p.v[r];
    }
    uint8_t *kst = stage + 16 * p.nv16;
    if ((uint32_t)l < p.nk16) ((uint4 *)kst)[l] = p.k;
    wave_sync();
    const uint64_t va = p.vs & ~15ull, ka = p.ks & ~15ull;
    // 2. row sizes and offsets (lane = row)
    const bool row = (uint32_t)l < ne;
    const uint32_t ri = a.restart_interval;
    uint32_t shared = 0;
    if (V == 2 && row) shared = (l % ri == 0) ? 0 : p.lcp;
    if (V == 1) {  // prefix vs the block's first key (block.rs:117-123)
        uint32_t fkl = __shfl(p.klen, 0, 64);
        if (row && l > 0) {
            const uint8_t *fk = kst + (p.ks - ka);
            const uint8_t *mk = kst + (p.ko - ka);
            shared = lcp_bytes(fk, fkl, mk, p.klen);
        }
    }
    RowInfo r;
    r.shared = shared;
    r.suf = p.klen - shared;
    r.vlen = p.vlen;
    r.flags = (uint8_t)((p.kind == SDB_KIND_MERGE ? SDB_FLAG_MERGE_OPERAND : 0) |
                        (p.kind == SDB_KIND_TOMBSTONE ? SDB_FLAG_TOMBSTONE : 0) |
                        ((p.mask & SDB_TS_EXPIRE) ? SDB_FLAG_HAS_EXPIRE_TS : 0) |
                        ((p.mask & SDB_TS_CREATE) ? SDB_FLAG_HAS_CREATE_TS : 0));
    const uint32_t ts8 = 8u * (((p.mask & SDB_TS_CREATE) != 0) + ((p.mask & SDB_TS_EXPIRE) != 0));
    uint32_t size = 0;
    if (row) {
        if (V == 2) size = varint_len(shared) + varint_len(r.suf) + varint_len(r.vlen) + r.suf + r.vlen + 9 + ts8;
        else size = 4 + r.suf + 9 + ts8 + (p.kind == SDB_KIND_TOMBSTONE ? 0 : 4 + r.vlen);
    }
    r.size = size;
    const uint32_t inc = wave_incl_scan(size);
    const uint32_t row_off = inc - size;
    const uint32_t D = __shfl(inc, 63, 64);
    uint8_t *gdst = a.out_data + p.off;
    uint8_t *im = img + ((uintptr_t)gdst & 15);
    // 3. rows
    if (row) {
        uint8_t *rowp = im + row_off;
        uint32_t h;
        write_row_small<V>(rowp, r, p.seq, p.ets, p.cts, &h);
        lds_copy(rowp + h, kst + (p.ko + shared - ka), r.suf);
        if (r.vlen) {
            uint32_t voff = (V == 2) ? h + r.suf : (size - r.vlen);
            lds_copy(rowp + voff, stage + (p.vo - va), r.vlen);
        }
    }
    // 4. offsets + count (Block::encode, format/block.rs:17-26)
    uint32_t noffs;
    if (V == 2) {
        noffs = (ne + ri - 1) / ri;
        if (row && l % ri == 0) {
            uint32_t q = l / ri;
            if (row_off > 0xFFFF) report_error(a.err, p.s + l, SDB_LIMIT_EXCEEDED);  // block_v2.rs:195
            im[D + 2 * q] = (uint8_t)(row_off >> 8);
            im[D + 2 * q + 1] = (uint8_t)row_off;
        }
    } else {
        noffs = ne;
        if (row) {
            im[D + 2 * l] = (uint8_t)(row_off >> 8);  // `as u16` (block.rs:163)
            im[D + 2 * l + 1] = (uint8_t)row_off;
        }
    }
    if (l == 0) {
        im[D + 2 * noffs] = (uint8_t)(noffs >> 8);
        im[D + 2 * noffs + 1] = (uint8_t)noffs;
    }
    wave_sync();
    // 5. CRC32 (format/sst.rs:541-552) and store
    const uint32_t Lc = D + 2 * noffs + 2;
    const uint32_t c = wave_crc32_lds(im, Lc, crc);
    if (l == 0) {
        im[Lc] = (uint8_t)(c >> 24);
        im[Lc + 1] = (uint8_t)(c >> 16);
        im[Lc + 2] = (uint8_t)(c >> 8);
        im[Lc + 3] = (uint8_t)c;
        if (Lc + 4 != p.bb) report_error(a.err, p.s, SDB_DEVICE_ERROR);  // internal consistency
    }
    wave_sync();
    wave_store(gdst, img, (uint64_t)Lc + 4);
    // 6. BlockStats (sst_stats.rs:9-16) and the index key (compute_index_key, utils.rs:198-226)
    const uint64_t pu = __ballot(row && p.kind == SDB_KIND_VALUE);
    const uint64_t de = __ballot(row && p.kind == SDB_KIND_TOMBSTONE);
    const uint64_t me = __ballot(row && p.kind == SDB_KIND_MERGE);
    if (l == 0) {
        a.out_block_stats[3 * (uint64_t)p.blk] = (uint16_t)__popcll(pu);
        a.out_block_stats[3 * (uint64_t)p.blk + 1] = (uint16_t)__popcll(de);
        a.out_block_stats[3 * (uint64_t)p.blk + 2] = (uint16_t)__popcll(me);
        uint32_t ik = 0;
        if (p.s > 0) ik = (p.lcp == p.prev_klen && p.prev_klen == p.klen) ? p.klen : p.lcp + 1;
        a.out_index_key_len[p.blk] = ik;
    }
    wave_sync();
}

template <int V>
__global__ __launch_bounds__(512, 4) void k_emit(EncodeArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    if (*a.err != ~0ull) return;  // any earlier error (incl. capacity): write nothing
    const uint32_t nb = a.anchor_blk[a.nchunks];
    uint32_t(*crc)[256] = (uint32_t(*)[256])smem;
    for (uint32_t q = threadIdx.x; q < 8 * 256; q += blockDim.x) ((uint32_t *)crc)[q] = (&c_crc.t[0][0])[q];
    __syncthreads();
    const uint32_t wave = threadIdx.x >> 6, wpb = blockDim.x >> 6;
    uint8_t *stage = smem + kCrcLds + (uint64_t)wave * (kStageCap + kImgCap);
    uint8_t *img = stage + kStageCap;
    const uint32_t gw = blockIdx.x * wpb + wave, G = gridDim.x * wpb;
    Pre cur, nxt;
    load_pre(a, gw, nb, cur);
    for (uint32_t blk = gw; blk < nb; blk += G) {
        load_pre(a, blk + G, nb, nxt);  // in flight while `cur` is assembled
        if (cur.fast) {
            process_block<V>(a, cur, stage, img, crc);
        } else if (lane_id() == 0) {
            uint32_t slot = atomicAdd(a.slow_count, 1u);
            a.slow_list[slot] = blk;
        }
        cur = nxt;
    }
}

// ------------------------------------------------------------------------------------------------
// K6: slow path for blocks that do not fit the LDS image: assemble straight into HBM.
// ------------------------------------------------------------------------------------------------
template <int V>
__global__ __launch_bounds__(256) void k_emit_slow(EncodeArgs a) {
    __shared__ __attribute__((aligned(16))) uint32_t s_crc[8][256];
    __shared__ __attribute__((aligned(16))) uint8_t s_win[4096 + 64];  // window at +16
    const uint32_t nslow = *a.slow_count;
    if (a.anchor_blk[a.nchunks] > a.block_cap || a.anchor_byte[a.nchunks] > a.data_cap) return;
    for (uint32_t q = threadIdx.x; q < 8 * 256; q += blockDim.x) ((uint32_t *)s_crc)[q] = (&c_crc.t[0][0])[q];
    __syncthreads();
    for (uint32_t it = blockIdx.x; it < nslow; it += gridDim.x) {
        const uint32_t blk = a.slow_list[it];
        const uint64_t b = a.out_block_first[blk];
        const uint64_t e = a.next[b];
        const uint64_t off = a.out_block_off[blk];
        const uint32_t ne = (uint32_t)(e - b);
        uint8_t *dst = a.out_data + off;
        const uint32_t ri = a.restart_interval;
        const uint64_t fko = a.key_off[b];
        const uint32_t fkl = (uint32_t)(a.key_off[b + 1] - fko);
        uint64_t D = 0;
        for (uint32_t i0 = 0; i0 < ne; i0 += blockDim.x) {
            uint32_t i = i0 + threadIdx.x;
            // each thread writes its own row; row offsets need a prefix sum -> do it serially per round
            __shared__ uint64_t s_size[256];
            __shared__ uint64_t s_off[256];
            RowInfo r;
            uint64_t seq = 0;
            int64_t ets = 0, cts = 0;
            if (i < ne) {
                uint64_t j = b + i;
                uint64_t ko = a.key_off[j];
                uint32_t klen = (uint32_t)(a.key_off[j + 1] - ko);
                uint8_t kd = a.kind ? a.kind[j] : 0;
                uint8_t m = a.ts_mask ? a.ts_mask[j] : 0;
                uint32_t vlen = kd == SDB_KIND_TOMBSTONE ? 0 : (uint32_t)(a.val_off[j + 1] - a.val_off[j]);
                uint32_t shared;
                if (V == 2) shared = (i % ri == 0) ? 0 : a.lcp[j];
                else shared = (i == 0) ? 0 : lcp_bytes(a.key_bytes + fko, fkl, a.key_bytes + ko, klen);
                r.shared = shared;
                r.suf = klen - shared;
                r.vlen = vlen;
                r.key_src = ko + shared;
                r.val_src = a.val_off[j];
                r.flags = (uint8_t)((kd == SDB_KIND_MERGE ? SDB_FLAG_MERGE_OPERAND : 0) |
                                    (kd == SDB_KIND_TOMBSTONE ? SDB_FLAG_TOMBSTONE : 0) |
                                    ((m & SDB_TS_EXPIRE) ? SDB_FLAG_HAS_EXPIRE_TS : 0) |
                                    ((m & SDB_TS_CREATE) ? SDB_FLAG_HAS_CREATE_TS : 0));
                const uint32_t ts8 = 8u * (((m & SDB_TS_CREATE) != 0) + ((m & SDB_TS_EXPIRE) != 0));
                if (V == 2) r.size = varint_len(shared) + varint_len(r.suf) + varint_len(vlen) + r.suf + vlen + 9 + ts8;
                else r.size = 4 + r.suf + 9 + ts8 + (kd == SDB_KIND_TOMBSTONE ? 0 : 4 + vlen);
                seq = a.seq ? a.seq[j] : 0;
                ets = (m & SDB_TS_EXPIRE) ? a.expire_ts[j] : 0;
                cts = (m & SDB_TS_CREATE) ? a.create_ts[j] : 0;
                s_size[threadIdx.x] = r.size;
            } else {
                s_size[threadIdx.x] = 0;
            }
            __syncthreads();
            if (threadIdx.x == 0) {
                uint64_t c = D;
                for (uint32_t q = 0; q < blockDim.x; q++) {
                    s_off[q] = c;
                    c += s_size[q];
                }
            }
            __syncthreads();
            if (i < ne) {
                uint64_t ro = s_off[threadIdx.x];
                r.row_off = (uint32_t)ro;
                uint8_t *row = dst + ro;
                uint32_t h;
                write_row_small<V>(row, r, seq, ets, cts, &h);
                for (uint32_t q = 0; q < r.suf; q++) row[h + q] = a.key_bytes[r.key_src + q];
                uint32_t voff = (V == 2) ? h + r.suf : (r.size - r.vlen);
                for (uint32_t q = 0; q < r.vlen; q++) row[voff + q] = a.val_bytes[r.val_src + q];
                // offsets
                if (V == 2) {
                    if (i % ri == 0) {
                        if (ro > 0xFFFF) report_error(a.err, b + i, SDB_LIMIT_EXCEEDED);
                        // placed after all rows: remember in s_off reuse below
                    }
                }
            }
            __syncthreads();
            // offsets table entries for this round are written after D is known: store row offsets
            // temporarily in the workspace `lcp` is still needed, so stash into tab_cnt (per entry)
            if (i < ne) a.tab_cnt[b + i] = (uint32_t)s_off[threadIdx.x];
            D = s_off[blockDim.x - 1] + s_size[blockDim.x - 1];
            __syncthreads();
        }
        __threadfence();
        __syncthreads();
        if (threadIdx.x == 0) {  // BlockStats + compute_index_key for this block
            uint32_t pu = 0, de = 0, me = 0;
            for (uint64_t j = b; j < e; j++) {
                uint8_t kd = a.kind ? a.kind[j] : 0;
                pu += kd == SDB_KIND_VALUE;
                de += kd == SDB_KIND_TOMBSTONE;
                me += kd == SDB_KIND_MERGE;
            }
            a.out_block_stats[3 * (uint64_t)blk] = (uint16_t)pu;
            a.out_block_stats[3 * (uint64_t)blk + 1] = (uint16_t)de;
            a.out_block_stats[3 * (uint64_t)blk + 2] = (uint16_t)me;
            uint32_t ik = 0;
            if (b > 0) {
                uint64_t fl = a.key_off[b + 1] - a.key_off[b];
                uint64_t pl = a.key_off[b] - a.key_off[b - 1];
                uint32_t lc = a.lcp[b];
                ik = (lc == pl && pl == fl) ? (uint32_t)fl : lc + 1;
            }
            a.out_index_key_len[blk] = ik;
        }
        uint32_t noffs = (V == 2) ? (ne + ri - 1) / ri : ne;
        for (uint32_t q = threadIdx.x; q < noffs; q += blockDim.x) {
            uint32_t ro = a.tab_cnt[b + (V == 2 ? (uint64_t)q * ri : q)];
            dst[D + 2 * q] = (uint8_t)(ro >> 8);
            dst[D + 2 * q + 1] = (uint8_t)ro;
        }
        if (threadIdx.x == 0) {
            dst[D + 2 * noffs] = (uint8_t)(noffs >> 8);
            dst[D + 2 * noffs + 1] = (uint8_t)noffs;
        }
        __threadfence();
        __syncthreads();
        // CRC over [dst, dst + Lc) with 4 KiB right-aligned windows staged through LDS by wave 0
        const uint64_t Lc = D + 2 * (uint64_t)noffs + 2;
        if (threadIdx.x < 64) {
            uint64_t nwin = (Lc + 4095) >> 12;
            uint64_t first = Lc - ((nwin - 1) << 12);
            uint32_t acc = 0;
            for (uint64_t w = 0; w < nwin; w++) {
                uint64_t wbeg = (w == 0) ? 0 : first + ((w - 1) << 12);
                uint32_t wlen = (uint32_t)((w == 0) ? first : 4096);
                for (uint32_t q = threadIdx.x; q < wlen; q += 64) s_win[16 + q] = dst[wbeg + q];
                wave_sync();
                uint32_t raw = wave_crc_raw_lds(s_win + 16, wlen, (const uint32_t(*)[256])s_crc, w == 0);
                // R(A || B) = R(A) * x^(8|B|) + R(B); every window after the first is 4096 bytes
                acc = (w == 0) ? raw : (gf_mul(c_shift.window, acc) ^ raw);
                wave_sync();
            }
            uint32_t crc = acc ^ 0xFFFFFFFFu;
            if (threadIdx.x == 0) {
                dst[Lc] = (uint8_t)(crc >> 24);
                dst[Lc + 1] = (uint8_t)(crc >> 16);
                dst[Lc + 2] = (uint8_t)(crc >> 8);
                dst[Lc + 3] = (uint8_t)crc;
            }
        }
        __syncthreads();
    }
}

template __global__ void k_emit<1>(EncodeArgs);
template __global__ void k_emit<2>(EncodeArgs);
template __global__ void k_emit_slow<1>(EncodeArgs);
template __global__ void k_emit_slow<2>(EncodeArgs);

// ------------------------------------------------------------------------------------------------
// Launcher
// ------------------------------------------------------------------------------------------------
__global__ void k_init_summary(EncodeArgs a) {
    if (threadIdx.x == 0) {
        sdb_sst_summary *s = a.summary;
        s->data_len = 0;
        s->num_blocks = 0;
        s->num_entries = a.n;
        s->raw_key_size = 0;
        s->raw_val_size = 0;
        s->num_puts = s->num_deletes = s->num_merges = 0;
        s->bloom_len = 0;
        s->num_probes = 0;
        s->filter_built = 0;
        s->status = 0;
        s->max_block_entries = 0;
        s->first_error_entry = ~0ull;
        *a.err = ~0ull;
        *a.wmax = 0;
        *a.slow_count = 0;
        if (a.n == 0 && a.block_cap + 1 > 0) {  // empty SST: BlockMeta list is empty, offsets = [0]
            a.out_block_off[0] = 0;
            a.out_block_first[0] = 0;
        }
    }
}

__global__ void k_finish_summary(EncodeArgs a, uint64_t bloom_len, uint32_t num_probes, uint32_t built) {
    if (threadIdx.x == 0) {
        sdb_sst_summary *s = a.summary;
        unsigned long long e = *a.err;
        s->max_block_entries = *a.wmax;
        s->bloom_len = bloom_len;
        s->num_probes = num_probes;
        s->filter_built = built;
        if (e != ~0ull) {
            s->status = (int32_t)(e & 0xFF);
            s->first_error_entry = e >> 8;
        }
    }
}

static bool lds_attrs_set = false;
static int g_cus = 0;
static uint32_t emit_grid() { return (uint32_t)(g_cus > 0 ? 2 * g_cus : 512); }
static void set_lds_attrs() {
    if (lds_attrs_set) return;
    int dev = 0;
    hipGetDevice(&dev);
    hipDeviceGetAttribute(&g_cus, hipDeviceAttributeMultiprocessorCount, dev);
    hipFuncSetAttribute((const void *)k_emit<1>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEmitLds);
    hipFuncSetAttribute((const void *)k_emit<2>, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEmitLds);
    hipFuncSetAttribute((const void *)k_enum, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kEnumLds);
    hipFuncSetAttribute((const void *)k_resolve, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kResolveLds);
    lds_attrs_set = true;
}

hipError_t launch_encode(EncodeArgs a, hipStream_t st) {
    const uint32_t tpb = 256;
    set_lds_attrs();
    hipLaunchKernelGGL(k_init_summary, dim3(1), dim3(64), 0, st, a);
    if (a.n == 0) {
        hipLaunchKernelGGL(k_finish_summary, dim3(1), dim3(64), 0, st, a, a.bloom_len, a.num_probes, a.filter_built);
        return hipGetLastError();
    }
    const uint32_t g = (uint32_t)((a.n + tpb - 1) / tpb);
    a.nprep_wg = g;
    stage_mark(st, kStPrep, true);
    hipLaunchKernelGGL(k_prep, dim3(g), dim3(tpb), 0, st, a);
    stage_mark(st, kStPrep, false);
    stage_mark(st, kStNext, true);
    hipLaunchKernelGGL(k_next, dim3(g), dim3(tpb), 0, st, a);
    stage_mark(st, kStNext, false);
    stage_mark(st, kStChunk, true);
    hipLaunchKernelGGL(k_chunk, dim3(a.nchunks), dim3(512), 0, st, a);
    stage_mark(st, kStChunk, false);
    stage_mark(st, kStResolve, true);
    hipLaunchKernelGGL(k_resolve, dim3(1), dim3(1024), kResolveLds, st, a);
    stage_mark(st, kStResolve, false);
    stage_mark(st, kStEnum, true);
    hipLaunchKernelGGL(k_enum, dim3(a.nchunks), dim3(256), kEnumLds, st, a);
    stage_mark(st, kStEnum, false);
    stage_mark(st, kStEmit, true);
    if (a.version == 2) hipLaunchKernelGGL(k_emit<2>, dim3(emit_grid()), dim3(kEmitThreads), kEmitLds, st, a);
    else hipLaunchKernelGGL(k_emit<1>, dim3(emit_grid()), dim3(kEmitThreads), kEmitLds, st, a);
    stage_mark(st, kStEmit, false);
    stage_mark(st, kStEmitSlow, true);
    if (a.version == 2) hipLaunchKernelGGL(k_emit_slow<2>, dim3(64), dim3(256), 0, st, a);
    else hipLaunchKernelGGL(k_emit_slow<1>, dim3(64), dim3(256), 0, st, a);
    stage_mark(st, kStEmitSlow, false);
    hipLaunchKernelGGL(k_finish_summary, dim3(1), dim3(64), 0, st, a, a.bloom_len, a.num_probes, a.filter_built);
    return hipGetLastError();
}

}  // namespace sdb
