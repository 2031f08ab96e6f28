// sdb_bloom.hip — bloom filter build / probe for gfx950.
//
// Replaces BloomFilterBuilder (slatedb/src/filter.rs:40-90) and BloomFilter::might_contain
// (filter.rs:124-136): filter_hash = SipHash-1-3 with a zero key over the raw key bytes
// (siphasher 1.0.3, filter.rs:196-204); probes by enhanced double hashing (filter.rs:206-221);
// LSB-first bit order (filter.rs:223-233).  Bit p of the byte-addressed bitmap is bit (p & 31) of the
// little-endian 32-bit word p >> 5, so setting it is one 32-bit atomicOr.
#include <mutex>

#include "sdb_bloom.h"

namespace sdb {

__global__ __launch_bounds__(256) void k_bloom_atomic(const uint8_t *__restrict__ key_bytes,
                                                      const uint64_t *__restrict__ key_off, uint64_t n,
                                                      uint32_t k, uint32_t m, uint32_t *bitmap) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint64_t ko = key_off[i];
        uint64_t h = siphash13(key_bytes + ko, key_off[i + 1] - ko);
        for_each_probe(h, k, m, [&](uint32_t p) {
            atomicOr(bitmap + (p >> 5), 1u << (p & 31));
            return true;
        });
    }
}

__global__ __launch_bounds__(kBinThreads) void k_bloom_bin(const uint8_t *__restrict__ key_bytes,
                                                           const uint64_t *__restrict__ key_off, uint64_t n,
                                                           BloomPlan pl, BloomSlots q) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    bloom_bin_tile(blockIdx.x, key_bytes, key_off, n, pl, q, lds);
}

__global__ __launch_bounds__(kFillThreads) void k_bloom_fill(const uint8_t *__restrict__ key_bytes,
                                                             const uint64_t *__restrict__ key_off, uint64_t n,
                                                             BloomPlan pl, BloomSlots q, uint8_t *bitmap,
                                                             uint64_t bytes) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    bloom_fill_slice(blockIdx.x, key_bytes, key_off, n, pl, q, bitmap, bytes, lds);
}

// Byte-granular probe reads: the bitmap may sit at any address (e.g. 17 bytes into an SST's filter
// block, format/sst.rs:394-421) and is read only inside [0, ceil(m / 8)).
__global__ __launch_bounds__(256) void k_bloom_query(const uint8_t *bitmap, uint32_t k, uint32_t m,
                                                     const uint8_t *__restrict__ key_bytes,
                                                     const uint64_t *__restrict__ key_off, uint64_t n,
                                                     uint8_t *result) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n;
         i += (uint64_t)gridDim.x * blockDim.x) {
        uint8_t r = 0;
        if (m) {
            uint64_t ko = key_off[i];
            uint64_t h = siphash13(key_bytes + ko, key_off[i + 1] - ko);
            r = 1;
            for_each_probe(h, k, m, [&](uint32_t p) {
                if (!((bitmap[p >> 3] >> (p & 7)) & 1u)) {
                    r = 0;
                    return false;
                }
                return true;
            });
        }
        result[i] = r;
    }
}

// ------------------------------------------------------------------------------------------------
// Standalone build, dense records (configs[3]: 10 M keys, 100 M bits).  The bitmap is cut into
// slices of 2^16 bits, so a probe is stored as its u16 offset inside its slice.
//   k_bloom_sort  one 512-thread workgroup per tile of T = 4096 keys (two per CU): the key offsets,
//                 then the 16-byte key words, all loads in flight before the first use; SipHash-1-3
//                 and the k probes of every key held in registers; an LDS counting sort by slice (one
//                 returning LDS add per probe gives its rank in the slice, so the scatter needs no
//                 second atomic); the tile's T*k u16 offsets are written as ONE dense, slice-ordered
//                 array with 16-byte stores, and the tile's run starts (S + 1 u16, T*k < 2^16) as its
//                 table row.
//   k_bloom_or    one 512-thread workgroup per pair of slices (kOrNs): the pair's run starts in every
//                 tile staged in LDS, then every tile's contiguous run of the pair's records (a wave
//                 reads eight tiles' runs per load instruction, 16 bytes per lane, eight such loads in
//                 flight) ORed into an LDS copy of the pair, written with plain stores.
// No per-slot capacity, hence no overflow case.  Records cost 2 B written + 2 B read per probe, the
// half of u32 records.  Measured (configs[3]): sort ~115 us, or ~70 us; one workgroup per
// slice or per four slices, 256- or 1024-thread sort workgroups were all slower.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kDenseThreads = 512, kDenseSliceBits = 16, kDenseMaxSlices = 4096;
constexpr uint32_t kOrThreads = 512;
#ifndef SDB_OR_NS
#define SDB_OR_NS 2
#endif
#ifndef SDB_OR_LANES
#define SDB_OR_LANES 8
#endif
constexpr uint32_t kOrNs = SDB_OR_NS, kOrLanes = SDB_OR_LANES, kOrSeg = 64 / kOrLanes, kOrUnroll = 8;
static_assert(kOrNs >= 1 && kOrNs <= 7, "a tile row of kOrNs + 1 u16 run starts fits 16 bytes");
constexpr uint32_t kOrLds = 150 * 1024;

struct DensePlan {
    uint32_t k, m, S;        // probes per key, bits, slices of 2^16 bits
    uint32_t kpt, T, tiles;  // keys per thread, keys per tile, tiles
    uint32_t tab_stride;     // u16 per table row (>= S + 1, multiple of 8)
    uint32_t W;              // k_bloom_or workgroups
    uint64_t rec_stride;     // u16 records per tile (T * k rounded to 8)
    uint64_t mmod;
    uint16_t *rec;           // tiles x rec_stride
    uint16_t *tab;           // tiles x tab_stride
};

static DensePlan dense_plan(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    DensePlan d{};
    d.k = k;
    d.m = (uint32_t)(bitmap_bytes * 8);
    d.S = (uint32_t)(((uint64_t)d.m + (1u << kDenseSliceBits) - 1) >> kDenseSliceBits);
    d.kpt = k <= 7 ? 8 : 4;
    d.T = kDenseThreads * d.kpt;
    d.tiles = (uint32_t)((n + d.T - 1) / d.T);
    d.tab_stride = (d.S + 1 + 7) & ~7u;
    d.rec_stride = ((uint64_t)d.T * k + 7) & ~7ull;
    d.W = (d.S + kOrNs - 1) / kOrNs;  // k_bloom_or: kOrNs slices per workgroup
    d.mmod = d.m ? ~0ull / d.m + 1 : 0;
    return d;
}
// k_bloom_sort's LDS: S + 1 counts, then the sorted records 16-byte aligned
__host__ __device__ inline uint32_t dense_sorted_at(uint32_t S) { return (S + 1 + 3) & ~3u; }
static size_t dense_sort_lds(const DensePlan &d) { return 4 * (size_t)dense_sorted_at(d.S) + 2 * (size_t)d.rec_stride; }
static size_t dense_or_lds(const DensePlan &d);
static bool dense_fits(const DensePlan &d) {
    return d.k >= 1 && d.k <= 15 && d.m >= 2 && d.S <= kDenseMaxSlices && (uint64_t)d.T * d.k < 65536 &&
           dense_sort_lds(d) <= kBinLds && dense_or_lds(d) <= kOrLds;
}
static uint64_t dense_ws_bytes(const DensePlan &d) {
    return 256 + (((uint64_t)d.tiles * d.rec_stride * 2 + 255) & ~255ull) + (uint64_t)d.tiles * d.tab_stride * 2;
}
static void dense_carve(DensePlan &d, void *ws) {
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    d.rec = (uint16_t *)w;
    d.tab = (uint16_t *)(w + (((uint64_t)d.tiles * d.rec_stride * 2 + 255) & ~255ull));
}

// (h0, d0) of keys k0 + tid + j * kDenseThreads (j < KPT, only those < nk are meaningful).  Every load
// is unconditional, so all of them are in flight before the first use: the KPT offset pairs, then
// the KPT 16-byte key words (a key that is not 16 bytes at an 8-byte aligned offset reads the 16
// in-bounds bytes of its own offset pair instead, and is hashed by the generic path afterwards).
template <uint32_t KPT>
SDB_DEV void dense_hash_keys(const uint8_t *__restrict__ key_bytes, const uint64_t *__restrict__ key_off, uint64_t k0,
                             uint32_t nk, const BloomPlan &pl, uint32_t (&hh)[KPT], uint32_t (&dd)[KPT]) {
    const uint32_t tid = threadIdx.x;
    uint64_t ko[KPT], ke[KPT];
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
        const uint32_t x = tid + j * kDenseThreads;
        const uint64_t i = k0 + (x < nk ? x : nk - 1);
        ko[j] = key_off[i];
        ke[j] = key_off[i + 1];
    }
    uint4 w[KPT];
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
        const uint32_t x = tid + j * kDenseThreads;
        const uint64_t i = k0 + (x < nk ? x : nk - 1);
        const bool fast = ke[j] - ko[j] == 16 && (ko[j] & 7) == 0;
        w[j] = *(const uint4 *)(fast ? key_bytes + ko[j] : (const uint8_t *)(key_off + i));
    }
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
        const bool fast = ke[j] - ko[j] == 16 && (ko[j] & 7) == 0;
        uint64_t h;
        if (fast) h = siphash13_16((uint64_t)w[j].x | (uint64_t)w[j].y << 32, (uint64_t)w[j].z | (uint64_t)w[j].w << 32);
        else h = siphash13(key_bytes + ko[j], ke[j] - ko[j]);
        hh[j] = fastmod_u32((uint32_t)h, pl.mmod, pl.m);
        dd[j] = fastmod_u32((uint32_t)(h >> 32), pl.mmod, pl.m);
    }
}

// KMAX: probes per key the registers hold (k <= KMAX; EXACT: k == KMAX, the loops fully unrolled with no
// uniform branches between the probes); KPT keys per thread.
template <uint32_t KMAX, uint32_t KPT, bool EXACT>
SDB_DEV void bloom_sort_tile(const uint8_t *__restrict__ key_bytes, const uint64_t *__restrict__ key_off, uint64_t n,
                             const DensePlan &d, uint32_t *lds) {
    uint32_t *hist = lds;  // S: counts, then run starts; hist[S]: the count of dead lanes' probes (unused)
    uint16_t *sorted = (uint16_t *)(lds + dense_sorted_at(d.S));  // T * k offsets, slice order
    __shared__ uint64_t s_w[17];
    const uint32_t tid = threadIdx.x, tile = blockIdx.x, S = d.S, k = EXACT ? KMAX : d.k;
    const uint64_t k0 = (uint64_t)tile * d.T;
    const uint32_t nk = (uint32_t)((k0 + d.T < n ? k0 + d.T : n) - k0);
    for (uint32_t x = tid; x <= S; x += kDenseThreads) hist[x] = 0;
    // hash: key tid + j * 1024 of the tile (consecutive lanes read consecutive keys)
    BloomPlan pl{};
    pl.m = d.m;
    pl.mmod = d.mmod;
    uint32_t hh[KPT], dd[KPT];
    dense_hash_keys<KPT>(key_bytes, key_off, k0, nk, pl, hh, dd);
    __syncthreads();
    // every probe (u32) and its rank inside its slice (u16: T * k < 2^16, two per register) stay in
    // registers from the counting pass to the scatter.  The probes are generated first, then each key's
    // rank reservations are issued back to back (a dead lane counts into hist[S]), so a wave has many LDS
    // adds in flight instead of one round trip per probe
    uint32_t pr[KPT * KMAX], rk[(KPT * KMAX + 1) / 2];
#pragma unroll
    for (uint32_t x = 0; x < (KPT * KMAX + 1) / 2; x++) rk[x] = 0;
    if constexpr (EXACT) {
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++) {
            uint32_t h = hh[j], dl = dd[j];
            const uint32_t m = d.m;
#pragma unroll
            for (uint32_t i = 0; i < KMAX; i++) {
                dl += i;
                const uint32_t dm = dl - m;
                dl = dm < dl ? dm : dl;
                pr[j * KMAX + i] = h;
                h += dl;
                const uint32_t hm = h - m;
                h = hm < h ? hm : h;
            }
        }
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++) {
            const bool live = tid + j * kDenseThreads < nk;
            uint32_t r[KMAX];
#pragma unroll
            for (uint32_t i = 0; i < KMAX; i++) r[i] = atomicAdd(&hist[live ? pr[j * KMAX + i] >> kDenseSliceBits : S], 1u);
#pragma unroll
            for (uint32_t i = 0; i < KMAX; i++) rk[(j * KMAX + i) / 2] |= r[i] << (16 * ((j * KMAX + i) & 1));
        }
    } else {  // one LDS round trip per probe, in fewer registers
#pragma unroll
        for (uint32_t j = 0; j < KPT; j++) {
            const bool live = tid + j * kDenseThreads < nk;
            uint32_t h = hh[j], dl = dd[j];
            const uint32_t m = d.m;
#pragma unroll
            for (uint32_t i = 0; i < KMAX; i++) {
                pr[j * KMAX + i] = h;
                if (live && i < k) {
                    dl += i;
                    const uint32_t dm = dl - m;
                    dl = dm < dl ? dm : dl;
                    const uint32_t r = atomicAdd(&hist[h >> kDenseSliceBits], 1u);
                    rk[(j * KMAX + i) / 2] |= r << (16 * ((j * KMAX + i) & 1));
                    h += dl;
                    const uint32_t hm = h - m;
                    h = hm < h ? hm : h;
                }
            }
        }
    }
    __syncthreads();
    // run starts: exclusive scan of the counts (each thread sums its consecutive ceil(S / 512) counts,
    // one block scan); the table row gets S + 1 of them
    const uint32_t per = (S + kDenseThreads - 1) / kDenseThreads, x0 = tid * per;
    uint32_t mine = 0;
    for (uint32_t x = x0; x < x0 + per && x < S; x++) mine += hist[x];
    uint64_t tot;
    uint32_t run = (uint32_t)block_excl_scan_u64(mine, s_w, &tot);
    uint16_t *trow = d.tab + (uint64_t)tile * d.tab_stride;
    for (uint32_t x = x0; x < x0 + per && x < S; x++) {
        const uint32_t c = hist[x];
        hist[x] = run;
        trow[x] = (uint16_t)run;
        run += c;
    }
    const uint32_t carry = (uint32_t)tot;
    if (tid == 0) trow[S] = (uint16_t)carry;
    __syncthreads();
    // scatter: each probe's offset to its slice's run start + its rank
#pragma unroll
    for (uint32_t j = 0; j < KPT; j++) {
        if (tid + j * kDenseThreads < nk) {
#pragma unroll
            for (uint32_t i = 0; i < KMAX; i++) {
                if (i < k) {
                    const uint32_t p = pr[j * KMAX + i];
                    const uint32_t r = (rk[(j * KMAX + i) / 2] >> (16 * ((j * KMAX + i) & 1))) & 0xFFFFu;
                    sorted[hist[p >> kDenseSliceBits] + r] = (uint16_t)p;
                }
            }
        }
    }
    __syncthreads();
    // the dense record array of the tile: 16-B stores (rec_stride is a multiple of 8 u16)
    const uint32_t n16 = (carry + 7) >> 3;
    const uint4 *src = (const uint4 *)sorted;
    uint4 *dst = (uint4 *)(d.rec + (uint64_t)tile * d.rec_stride);
    for (uint32_t x = tid; x < n16; x += kDenseThreads) dst[x] = src[x];
}

// the default plan (k = 6) at two workgroups per CU: its 48 probes' rank reservations in flight fit 128 VGPRs
__global__ __launch_bounds__(kDenseThreads) __attribute__((amdgpu_waves_per_eu(4))) void k_bloom_sort6(
    const uint8_t *__restrict__ key_bytes, const uint64_t *__restrict__ key_off, uint64_t n, DensePlan d) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    bloom_sort_tile<6, 8, true>(key_bytes, key_off, n, d, lds);
}
template <uint32_t KMAX, uint32_t KPT>
__global__ __launch_bounds__(kDenseThreads) void k_bloom_sort(const uint8_t *__restrict__ key_bytes,
                                                              const uint64_t *__restrict__ key_off, uint64_t n,
                                                              DensePlan d) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    bloom_sort_tile<KMAX, KPT, false>(key_bytes, key_off, n, d, lds);
}

// Workgroup b -> its run of slices, XCD-aware: the dispatcher places workgroup b on XCD b mod 8, so
// the runs are dealt out so that each XCD holds consecutive slices (neighbouring runs share the edge
// lines of every tile's records in that XCD's L2).
SDB_DEV uint32_t dense_run_of(uint32_t b, uint32_t W) {
    const uint32_t x = b & 7, q = b >> 3;
    uint32_t start = 0;  // runs of XCDs 0 .. x - 1: XCD y holds ceil((W - y) / 8) workgroups
    for (uint32_t y = 0; y < x; y++) start += (W - y + 7) / 8;
    return start + q;
}

// kOrNs consecutive 2^16-bit slices per workgroup.  Every tile holds one run of those slices'
// records (run starts row[s0 .. s0 + kOrNs], u16), staged in LDS first.  A wave reads kOrSeg tiles'
// runs per load instruction: lane group q (kOrLanes lanes) reads tile t0 + q, 16 bytes (eight
// records) per lane, kOrUnroll such loads in flight per lane before the first OR; runs over
// 8 * kOrLanes records loop on.  A record's slice is the number of the row's inner starts at or below
// its position.
__global__ __launch_bounds__(kOrThreads) void k_bloom_or(DensePlan d, uint8_t *bitmap, uint64_t bytes) {
    extern __shared__ __attribute__((aligned(16))) uint32_t lds[];
    constexpr uint32_t kWords = 1u << (kDenseSliceBits - 5);
    constexpr uint32_t kRowU16 = kOrNs + 1 <= 2 ? 2 : kOrNs + 1 <= 4 ? 4 : 8;  // u16 per staged row
    const uint32_t run = dense_run_of(blockIdx.x, d.W);
    const uint32_t s0 = run * kOrNs, s1 = s0 + kOrNs < d.S ? s0 + kOrNs : d.S, ns = s1 - s0;
    uint32_t *bits = lds;                                // kOrNs x 2^16 bits
    uint16_t *rows = (uint16_t *)(lds + kOrNs * kWords);  // per tile: run starts s0 .. s0 + kOrNs
    const uint32_t tid = threadIdx.x, T = d.tiles;
    for (uint32_t x = tid; x < kOrNs * kWords; x += kOrThreads) bits[x] = 0;
    for (uint32_t t0 = tid; t0 < T; t0 += 4 * kOrThreads) {  // four rows' loads in flight per thread
        uint32_t e[4][kOrNs + 1];
#pragma unroll
        for (uint32_t u = 0; u < 4; u++) {
            const uint32_t t = t0 + u * kOrThreads;
            const uint16_t *row = d.tab + (uint64_t)(t < T ? t : 0) * d.tab_stride + s0;
#pragma unroll
            for (uint32_t j = 0; j <= kOrNs; j++) e[u][j] = row[j <= ns ? j : ns];
        }
#pragma unroll
        for (uint32_t u = 0; u < 4; u++)
            if (t0 + u * kOrThreads < T)
#pragma unroll
                for (uint32_t j = 0; j <= kOrNs; j++) rows[(t0 + u * kOrThreads) * kRowU16 + j] = (uint16_t)e[u][j];
    }
    __syncthreads();
    const uint32_t w = tid >> 6, nw = kOrThreads >> 6, l = tid & 63, q = l / kOrLanes, sl = l % kOrLanes;
    // lane sl of a group covers records [a8 + 8 sl, a8 + 8 sl + 8) of its tile, a8 = a & ~7 (16-byte
    // aligned: rec_stride is a multiple of 8 records); records outside [a, b) are skipped
    const uint64_t rlim = (uint64_t)T * d.rec_stride;  // u16 records in the workspace
    for (uint32_t t0 = w * kOrSeg; t0 < T; t0 += nw * kOrSeg * kOrUnroll) {
        uint4 v[kOrUnroll];
        uint32_t rb[kOrUnroll][kOrNs + 1];
        // unconditional loads (lanes past their run read an in-bounds clamped address, masked at use):
        // a load under a branch makes the compiler wait for every earlier load at the join
#pragma unroll
        for (uint32_t u = 0; u < kOrUnroll; u++) {
            const uint32_t t = t0 + u * nw * kOrSeg + q, tc = t < T ? t : T - 1;
#pragma unroll
            for (uint32_t j = 0; j <= kOrNs; j++) rb[u][j] = t < T ? rows[tc * kRowU16 + j] : 0;
            uint64_t x = (uint64_t)tc * d.rec_stride + (rb[u][0] & ~7u) + 8 * sl;
            x = x + 8 <= rlim ? x : 0;
            v[u] = *(const uint4 *)(d.rec + x);
        }
#pragma unroll
        for (uint32_t u = 0; u < kOrUnroll; u++) {
            const uint32_t t = t0 + u * nw * kOrSeg + q;
            const uint32_t a = rb[u][0], b = rb[u][kOrNs];
            auto put = [&](uint32_t i, uint32_t o) {  // record i of the tile, offset o in its slice
                uint32_t sub = 0;
#pragma unroll
                for (uint32_t j = 1; j < kOrNs; j++) sub += i >= rb[u][j] ? 1u : 0u;
                atomicOr(&bits[sub * kWords + (o >> 5)], 1u << (o & 31));
            };
            uint32_t i = (a & ~7u) + 8 * sl;  // first record of this lane's 16 bytes
            const uint32_t wv[4] = {v[u].x, v[u].y, v[u].z, v[u].w};
#pragma unroll
            for (uint32_t j = 0; j < 8; j++)
                if (i + j >= a && i + j < b) put(i + j, (wv[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
            if (t < T) {
                for (i += 8 * kOrLanes; i < b; i += 8 * kOrLanes) {  // runs over 8 * kOrLanes records
                    const uint4 y = *(const uint4 *)(d.rec + (uint64_t)t * d.rec_stride + i);
                    const uint32_t yw[4] = {y.x, y.y, y.z, y.w};
#pragma unroll
                    for (uint32_t j = 0; j < 8; j++)
                        if (i + j < b) put(i + j, (yw[j >> 1] >> (16 * (j & 1))) & 0xFFFFu);
                }
            }
        }
    }
    __syncthreads();
    // bitmap bytes [s0 * 8 KiB, s1 * 8 KiB) clipped to the filter (bitmap 4-byte aligned)
    const uint64_t b0 = (uint64_t)s0 << (kDenseSliceBits - 3);
    const uint64_t b1 = ((uint64_t)s1 << (kDenseSliceBits - 3)) < bytes ? ((uint64_t)s1 << (kDenseSliceBits - 3)) : bytes;
    const uint64_t nfull = (b1 - b0) >> 2;
    for (uint64_t x = tid; x < nfull; x += kOrThreads) ((uint32_t *)(bitmap + b0))[x] = bits[x];
    for (uint64_t x = b0 + 4 * nfull + tid; x < b1; x += kOrThreads) {
        const uint64_t r = x - b0;
        bitmap[x] = (uint8_t)(bits[r >> 2] >> (8 * (r & 3)));
    }
}

static size_t dense_or_lds(const DensePlan &d) {  // the slices' bits, then one row of run starts per tile
    constexpr uint32_t kRowU16 = kOrNs + 1 <= 2 ? 2 : kOrNs + 1 <= 4 ? 4 : 8;
    return 4 * (size_t)kOrNs * (1u << (kDenseSliceBits - 5)) + 2 * (size_t)kRowU16 * d.tiles;
}

static hipError_t launch_bloom_dense(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n, DensePlan d,
                                     uint8_t *bitmap, uint64_t bitmap_bytes, void *ws, hipStream_t st) {
    static std::once_flag attrs;
    static hipError_t attr_err = hipSuccess;
    std::call_once(attrs, [] {
        const void *f[] = {(const void *)k_bloom_sort6, (const void *)k_bloom_sort<7, 8>,
                           (const void *)k_bloom_sort<15, 4>};
        for (const void *x : f)
            if (attr_err == hipSuccess)
                attr_err = hipFuncSetAttribute(x, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBinLds);
        if (attr_err == hipSuccess)
            attr_err = hipFuncSetAttribute((const void *)k_bloom_or, hipFuncAttributeMaxDynamicSharedMemorySize,
                                           (int)kOrLds);
    });
    if (attr_err != hipSuccess) return attr_err;
    dense_carve(d, ws);
    if (d.k == 6)  // 10 bits per key
        hipLaunchKernelGGL(k_bloom_sort6, dim3(d.tiles), dim3(kDenseThreads), dense_sort_lds(d), st, key_bytes,
                           key_off, n, d);
    else if (d.k <= 7)
        hipLaunchKernelGGL((k_bloom_sort<7, 8>), dim3(d.tiles), dim3(kDenseThreads), dense_sort_lds(d), st, key_bytes,
                           key_off, n, d);
    else
        hipLaunchKernelGGL((k_bloom_sort<15, 4>), dim3(d.tiles), dim3(kDenseThreads), dense_sort_lds(d), st, key_bytes,
                           key_off, n, d);
    hipLaunchKernelGGL(k_bloom_or, dim3(d.W), dim3(kOrThreads), dense_or_lds(d), st, d, bitmap, bitmap_bytes);
    return hipGetLastError();
}

// one pass also when its buckets take more LDS than the counting sort but no more than this (two binning
// workgroups per CU either way)
#ifndef SDB_BIN_ONEPASS_LDS
#define SDB_BIN_ONEPASS_LDS (64 * 1024)
#endif
constexpr uint64_t kBinOnePassLds = SDB_BIN_ONEPASS_LDS;

BloomPlan bloom_plan(uint64_t n, uint32_t k, uint64_t bitmap_bytes, uint32_t tile_keys) {
    BloomPlan pl{};
    pl.k = k ? k : 1;
    pl.m = (uint32_t)(bitmap_bytes * 8);
    // slices of 2^sb bits: at least 4 KiB, at most 64 KiB of LDS, and at most 256 of them
    pl.sb = 15;
    while (pl.sb < 19 && (((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb) > 256) pl.sb++;
    pl.nslices = (uint32_t)(((uint64_t)pl.m + (1ull << pl.sb) - 1) >> pl.sb);
    if (pl.nslices == 0) pl.nslices = 1;
    uint32_t T = tile_keys;
    if (!T) {  // kBinKeysPerThread keys per thread, fewer when the sorted probes outgrow LDS
        T = kBinThreads * kBinKeysPerThread;
        while (T > kBinThreads && 4ull * (2 * pl.nslices + (uint64_t)T * pl.k) > kBinLds) T -= kBinThreads;
    }
    pl.T = T;
    pl.tiles = (uint32_t)((n + T - 1) / T);
    if (pl.tiles == 0) pl.tiles = 1;
    pl.mmod = pl.m ? ~0ull / pl.m + 1 : 0;
    // one pass (probes straight into per-slice LDS buckets of the slot capacity) when the offsets are
    // u16 and the buckets take no more LDS than the two-pass counting sort
    const uint64_t bk = 4ull * ((pl.nslices + 3) & ~3u) + 2ull * pl.nslices * bloom_slot_cap(pl);
    pl.one_pass = pl.sb <= 16 && (bk <= 4ull * (2ull * pl.nslices + (uint64_t)pl.T * pl.k) || bk <= kBinOnePassLds) ? 1u : 0u;
    return pl;
}

uint32_t bloom_slot_cap(const BloomPlan &pl) {
    // uniform probes: a slot (slice, tile) receives the probes of the tile's T keys that land in the
    // slice (2^sb of the m bits); + 6 sigma + 16
    const double frac = pl.m ? (double)(1ull << pl.sb) / pl.m : 1.0;
    const double mean = (double)pl.T * pl.k * (frac < 1.0 ? frac : 1.0);
    uint64_t cap = (uint64_t)(mean + 6.0 * __builtin_sqrt(mean + 1.0)) + 16;
    // a multiple of 32: u16 slots start 64-byte aligned, so the binning writes whole 64-byte granules (a
    // partial one costs the memory a read-modify-write) and bloom_fill_slice's 16-byte loads stay aligned
    cap = (cap + 31) & ~31ull;
    const uint64_t most = (uint64_t)pl.T * pl.k;  // a slot never holds more than the tile's probes
    if (cap > most) cap = (most + 31) & ~31ull;
    return (uint32_t)cap;
}

bool bloom_plan_fits(const BloomPlan &pl) {
    return pl.k <= kBinMaxK && pl.sb <= 19 && pl.m >= 2 && bloom_bin_lds(pl) <= kBinLds &&
           bloom_fill_lds(pl) <= 96 * 1024;
}

uint64_t bloom_slots_bytes(const BloomPlan &pl) {
    const uint64_t counts = ((uint64_t)pl.tiles * pl.nslices * 4 + 255) & ~255ull;
    return 256 + counts + (uint64_t)pl.nslices * pl.tiles * bloom_slot_cap(pl) * 4;
}

uint64_t bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    const DensePlan d = dense_plan(n, k, bitmap_bytes);
    const uint64_t a = bloom_slots_bytes(bloom_plan(n, k, bitmap_bytes));
    const uint64_t b = dense_fits(d) ? dense_ws_bytes(d) : 0;
    return a > b ? a : b;
}

BloomSlots bloom_slots(void *ws, const BloomPlan &pl) {
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    BloomSlots q;
    q.count = (uint32_t *)w;
    q.slot = (uint32_t *)(w + (((uint64_t)pl.tiles * pl.nslices * 4 + 255) & ~255ull));
    q.cap = bloom_slot_cap(pl);
    return q;
}

size_t bloom_bin_lds(const BloomPlan &pl) {
    // counts (padded to 16 bytes), then the buckets
    if (pl.one_pass) return 4 * (size_t)((pl.nslices + 3) & ~3u) + 2 * (size_t)pl.nslices * bloom_slot_cap(pl);
    return 4 * (2 * (size_t)pl.nslices + (size_t)pl.T * pl.k);
}
size_t bloom_fill_lds(const BloomPlan &pl) { return 4 * ((size_t)(1u << (pl.sb - 5)) + pl.tiles); }

hipError_t launch_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint32_t num_probes, uint8_t *bitmap, uint64_t bitmap_bytes, void *ws,
                              hipStream_t st) {
    if (bitmap_bytes == 0) return hipSuccess;
    if (n == 0 || num_probes == 0) return hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
    if (ws) {
        const DensePlan d = dense_plan(n, num_probes, bitmap_bytes);
        if (dense_fits(d) && !((uintptr_t)bitmap & 3)) return launch_bloom_dense(key_bytes, key_off, n, d, bitmap, bitmap_bytes, ws, st);
    }
    BloomPlan pl = bloom_plan(n, num_probes, bitmap_bytes);
    if (!ws || !bloom_plan_fits(pl)) {
        // no workspace (or a plan the binning cannot hold): device-scope atomics into the bitmap
        hipError_t e = hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
        if (e != hipSuccess) return e;
        uint64_t blocks = (n + 255) / 256;
        if (blocks > 65536) blocks = 65536;
        hipLaunchKernelGGL(k_bloom_atomic, dim3((uint32_t)blocks), dim3(256), 0, st, key_bytes, key_off, n,
                           num_probes, pl.m, (uint32_t *)bitmap);
        return hipGetLastError();
    }
    static std::once_flag attrs;
    std::call_once(attrs, [] {
        (void)hipFuncSetAttribute((const void *)k_bloom_bin, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kBinLds);
        (void)hipFuncSetAttribute((const void *)k_bloom_fill, hipFuncAttributeMaxDynamicSharedMemorySize, 96 * 1024);
        (void)hipGetLastError();  // an unsupported attribute value must not poison the launch status
    });
    const BloomSlots q = bloom_slots(ws, pl);
    hipLaunchKernelGGL(k_bloom_bin, dim3(pl.tiles), dim3(kBinThreads), bloom_bin_lds(pl), st, key_bytes, key_off, n, pl, q);
    hipLaunchKernelGGL(k_bloom_fill, dim3(pl.nslices), dim3(kFillThreads), bloom_fill_lds(pl), st, key_bytes, key_off, n, pl,
                       q, bitmap, bitmap_bytes);
    return hipGetLastError();
}

hipError_t launch_bloom_query(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes,
                              const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint8_t *result, hipStream_t st) {
    if (n == 0) return hipSuccess;
    uint32_t m = (uint32_t)(bitmap_bytes * 8);
    uint64_t blocks = (n + 255) / 256;
    if (blocks > 65536) blocks = 65536;
    hipLaunchKernelGGL(k_bloom_query, dim3((uint32_t)blocks), dim3(256), 0, st, bitmap,
                       num_probes, m, key_bytes, key_off, n, result);
    return hipGetLastError();
}

}  // namespace sdb

namespace sdb {
// The encode workspace serves either build: the fused one (tiles = k_seg's chunks) or the standalone
// kernels (sdb_encode_sst falls back to them when the fused plan does not fit).
uint64_t encode_bloom_workspace_bytes(uint64_t n, uint32_t k, uint64_t bitmap_bytes) {
    const uint64_t a = bloom_workspace_bytes(n, k, bitmap_bytes);
    const uint64_t b = bloom_slots_bytes(bloom_plan(n, k, bitmap_bytes, kChunk));
    return a > b ? a : b;
}
}  // namespace sdb

namespace sdb {

// ------------------------------------------------------------------------------------------------
// Prefix-extractor filters (BloomFilterBuilder::add_key with an extractor, filter.rs:40-63; build
// filter.rs:71-90): every stored key contributes hash(key[..prefix_len]) when that prefix differs from
// the last stored prefix (keys without a prefix do not reset it) and hash(key) under whole-key
// filtering.  The filter size follows the hash count, so the device counts before it sizes:
//   k_pf_last   per 1024-entry chunk: the last entry that has a prefix
//   k_pf_count  per entry: the previous entry with a prefix (in-chunk scan, else the chunks before),
//               new-prefix flag; per chunk: hashes
//   k_pf_plan   one workgroup: total hashes -> filter_size_bytes (u32 arithmetic), m, fastmod constant
//   k_pf_set    per entry: the probes of its hashes, device-scope atomicOr into the zeroed bitmap
// ------------------------------------------------------------------------------------------------
struct PrefixSpec {
    uint32_t kind, arg, whole, pad;
    const int32_t *lens;  // SDB_PREFIX_LENGTHS
};
struct PrefixWs {
    int64_t *chunk_last;   // per chunk: last entry with a prefix (-1: none)
    int64_t *prev_last;    // per chunk: last entry with a prefix before the chunk
    uint64_t *chunk_cnt;   // per chunk: hashes
    uint8_t *is_new;       // per entry: its prefix hash is stored
    uint64_t *plan;        // [0] hashes, [1] filter bytes, [2] m, [3] fastmod constant, [4] error
};
constexpr uint32_t kPfChunk = 1024;

SDB_DEV int64_t pf_len(const PrefixSpec &ps, const uint8_t *k, uint32_t kl, uint64_t i) {  // -1 = None
    if (ps.kind == SDB_PREFIX_FIXED) return kl >= ps.arg ? (int64_t)ps.arg : -1;
    if (ps.kind == SDB_PREFIX_DELIM) {
        for (uint32_t x = 0; x < kl; x++)
            if (k[x] == (uint8_t)ps.arg) return (int64_t)x + 1;
        return -1;
    }
    if (ps.kind == SDB_PREFIX_LENGTHS) return ps.lens ? (int64_t)ps.lens[i] : -1;
    return -1;
}

// Entry indices travel as i + 1 (0 = none) so the scans are unsigned maxima with identity 0 (the DPP
// lanes without a source read 0).
SDB_DEV uint64_t umax64(uint64_t x, uint64_t y) { return x > y ? x : y; }
SDB_DEV int64_t block_max_i64(int64_t v, int64_t *s_w) {  // every thread gets the workgroup max (v >= -1)
    const uint32_t tid = threadIdx.x, w = tid >> 6, nw = (blockDim.x + 63) >> 6;
    const uint64_t u = wave_readlane(wave_incl_scan_op((uint64_t)(v + 1), umax64), 63);
    __syncthreads();
    if ((tid & 63) == 0) s_w[w] = (int64_t)u;
    __syncthreads();
    uint64_t r = (uint64_t)s_w[0];
    for (uint32_t q = 1; q < nw; q++) r = umax64(r, (uint64_t)s_w[q]);
    __syncthreads();
    return (int64_t)r - 1;
}

__global__ __launch_bounds__(kPfChunk) void k_pf_last(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                                                      PrefixSpec ps, PrefixWs w) {
    __shared__ int64_t s_w[16];
    const uint64_t i = (uint64_t)blockIdx.x * kPfChunk + threadIdx.x;
    int64_t v = -1;
    if (i < n) {
        const uint64_t ko = key_off[i];
        if (pf_len(ps, key_bytes + ko, (uint32_t)(key_off[i + 1] - ko), i) >= 0) v = (int64_t)i;
    }
    v = block_max_i64(v, s_w);
    if (threadIdx.x == 0) w.chunk_last[blockIdx.x] = v;
}

__global__ __launch_bounds__(1024) void k_pf_prev(uint64_t nchunks, PrefixWs w) {  // exclusive max-scan
    if (threadIdx.x == 0) {
        int64_t m = -1;
        for (uint64_t c = 0; c < nchunks; c++) {
            w.prev_last[c] = m;
            const int64_t x = w.chunk_last[c];
            m = x > m ? x : m;
        }
    }
}

__global__ __launch_bounds__(kPfChunk) void k_pf_count(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                                                       PrefixSpec ps, PrefixWs w) {
    __shared__ int64_t s_last[16];
    __shared__ uint64_t s_w[17];
    const uint32_t tid = threadIdx.x, lane = (uint32_t)lane_id(), wv = tid >> 6;
    const uint64_t i = (uint64_t)blockIdx.x * kPfChunk + tid;
    int64_t pl = -1;
    uint64_t ko = 0;
    uint32_t kl = 0;
    if (i < n) {
        ko = key_off[i];
        kl = (uint32_t)(key_off[i + 1] - ko);
        pl = pf_len(ps, key_bytes + ko, kl, i);
    }
    // j = the last entry < i with a prefix: inclusive max-scan of (has ? i : -1), shifted by one
    const uint64_t mine = pl >= 0 ? i + 1 : 0;  // i + 1, 0 = none
    const uint64_t inc = wave_incl_scan_op(mine, umax64);
    if (lane == 63) s_last[wv] = (int64_t)inc;
    __syncthreads();
    uint64_t before = (uint64_t)(w.prev_last[blockIdx.x] + 1);
    for (uint32_t q = 0; q < wv; q++) before = umax64(before, (uint64_t)s_last[q]);
    uint64_t jp = wave_prev_lane(inc);
    if (lane == 0) jp = 0;
    const int64_t j = (int64_t)umax64(jp, before) - 1;
    uint64_t cnt = 0;
    uint8_t isnew = 0;
    if (i < n) {
        if (pl >= 0) {
            if (pl > kl) atomicMax((unsigned long long *)&w.plan[4], 1ull);  // the reference asserts
            isnew = 1;
            if (j >= 0) {
                const uint64_t jo = key_off[j];
                const uint32_t jl = (uint32_t)(key_off[j + 1] - jo);
                const int64_t pj = pf_len(ps, key_bytes + jo, jl, (uint64_t)j);
                if (pj == pl && pl <= kl && pj <= jl &&
                    lcp_bytes(key_bytes + ko, (uint32_t)pl, key_bytes + jo, (uint32_t)pj) == (uint32_t)pl)
                    isnew = 0;
            }
        }
        w.is_new[i] = isnew;
        cnt = isnew + (ps.whole ? 1 : 0);
    }
    uint64_t tot;
    block_excl_scan_u64(cnt, s_w, &tot);
    if (tid == 0) w.chunk_cnt[blockIdx.x] = tot;
}

__global__ __launch_bounds__(64) void k_pf_plan(uint64_t nchunks, uint32_t bpk, uint64_t cap, uint64_t *bloom_len,
                                                PrefixWs w) {
    if (threadIdx.x) return;
    uint64_t h = 0;
    for (uint64_t c = 0; c < nchunks; c++) h += w.chunk_cnt[c];
    const uint32_t bits = (uint32_t)h * bpk;  // key_hashes.len() as u32 (filter.rs:65-69)
    const uint64_t fb = bits / 8u + (bits % 8u != 0);
    const uint64_t m = fb * 8;
    w.plan[0] = h;
    w.plan[1] = fb;
    w.plan[2] = m;
    w.plan[3] = m ? ~0ull / m + 1 : 0;
    if (fb > cap) w.plan[4] = 1;
    *bloom_len = w.plan[4] ? ~0ull : fb;  // ~0: a prefix longer than its key, or the bitmap too small
}

__global__ __launch_bounds__(256) void k_pf_zero(uint8_t *bitmap, uint64_t cap, PrefixWs w) {
    const uint64_t fb = w.plan[4] ? 0 : w.plan[1];
    for (uint64_t x = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; 4 * x < fb && 4 * x < cap;
         x += (uint64_t)gridDim.x * blockDim.x)
        ((uint32_t *)bitmap)[x] = 0;
}

SDB_DEV void pf_set_hash(uint32_t *bm, uint64_t h, uint32_t k, uint32_t m, uint64_t mmod) {
    const uint32_t h0 = fastmod_u32((uint32_t)h, mmod, m), d0 = fastmod_u32((uint32_t)(h >> 32), mmod, m);
    probes_hd(h0, d0, k, m, [&](uint32_t p) { atomicOr(bm + (p >> 5), 1u << (p & 31)); });
}

__global__ __launch_bounds__(256) void k_pf_set(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                                                PrefixSpec ps, uint32_t k, uint8_t *bitmap, PrefixWs w) {
    if (w.plan[4]) return;
    const uint32_t m = (uint32_t)w.plan[2];
    const uint64_t mmod = w.plan[3];
    if (!m) return;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t ko = key_off[i];
        const uint32_t kl = (uint32_t)(key_off[i + 1] - ko);
        if (w.is_new[i]) {
            const int64_t pl = pf_len(ps, key_bytes + ko, kl, i);
            pf_set_hash((uint32_t *)bitmap, siphash13(key_bytes + ko, (uint64_t)pl), k, m, mmod);
        }
        if (ps.whole) pf_set_hash((uint32_t *)bitmap, siphash13(key_bytes + ko, kl), k, m, mmod);
    }
}

uint64_t prefix_workspace_bytes(uint64_t n) {
    const uint64_t nc = (n + kPfChunk - 1) / kPfChunk + 1;
    return 3 * ((8 * nc + 255) & ~255ull) + ((n + 256) & ~255ull) + 256;
}
static PrefixWs prefix_ws(void *ws, uint64_t n) {
    const uint64_t nc = (n + kPfChunk - 1) / kPfChunk + 1, a = (8 * nc + 255) & ~255ull;
    uint8_t *b = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    PrefixWs w;
    w.plan = (uint64_t *)b;
    w.chunk_last = (int64_t *)(b + 256);
    w.prev_last = (int64_t *)(b + 256 + a);
    w.chunk_cnt = (uint64_t *)(b + 256 + 2 * a);
    w.is_new = b + 256 + 3 * a;
    return w;
}

hipError_t launch_bloom_prefix(const uint8_t *key_bytes, const uint64_t *key_off, const int32_t *lens, uint64_t n,
                               uint32_t bpk, uint32_t kind, uint32_t arg, uint32_t whole, uint8_t *bitmap, uint64_t cap,
                               uint64_t *bloom_len, void *ws, hipStream_t st) {
    PrefixSpec ps{kind, arg, whole, 0, lens};
    PrefixWs w = prefix_ws(ws, n);
    const uint64_t nc = (n + kPfChunk - 1) / kPfChunk;
    hipError_t e = hipMemsetAsync(w.plan, 0, 64, st);
    if (e != hipSuccess) return e;
    const uint32_t k = (uint32_t)((float)bpk * 0.69f);  // optimal_num_probes (filter.rs:235-239)
    if (nc) {
        hipLaunchKernelGGL(k_pf_last, dim3((uint32_t)nc), dim3(kPfChunk), 0, st, key_bytes, key_off, n, ps, w);
        hipLaunchKernelGGL(k_pf_prev, dim3(1), dim3(1024), 0, st, nc, w);
        hipLaunchKernelGGL(k_pf_count, dim3((uint32_t)nc), dim3(kPfChunk), 0, st, key_bytes, key_off, n, ps, w);
    }
    hipLaunchKernelGGL(k_pf_plan, dim3(1), dim3(64), 0, st, nc, bpk, cap, bloom_len, w);
    uint64_t zb = (cap / 4 + 255) / 256;
    zb = zb < 1 ? 1 : (zb > 8192 ? 8192 : zb);
    hipLaunchKernelGGL(k_pf_zero, dim3((uint32_t)zb), dim3(256), 0, st, bitmap, cap, w);
    if (n) {
        uint64_t sb = (n + 255) / 256;
        sb = sb > 65536 ? 65536 : sb;
        hipLaunchKernelGGL(k_pf_set, dim3((uint32_t)sb), dim3(256), 0, st, key_bytes, key_off, n, ps, k, bitmap, w);
    }
    return hipGetLastError();
}

// Filter::might_match (filter.rs:149-175)
__global__ __launch_bounds__(256) void k_bloom_match(const uint8_t *bitmap, uint64_t bytes, uint32_t k, uint32_t whole,
                                                     PrefixSpec ps, const uint8_t *key_bytes, const uint64_t *key_off,
                                                     const uint8_t *is_prefix, uint64_t n, uint8_t *result) {
    const uint32_t m = (uint32_t)(bytes * 8);
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t ko = key_off[i];
        const uint32_t kl = (uint32_t)(key_off[i + 1] - ko);
        const bool pfx = is_prefix && is_prefix[i];
        int64_t len = -1;
        if (!pfx && whole) len = kl;
        else if (ps.kind != SDB_PREFIX_NONE) len = pf_len(ps, key_bytes + ko, kl, i);
        uint8_t r = 1;  // nothing to probe: no false negative
        if (len >= 0) {
            r = 0;
            if (m) {  // might_contain: an empty bitmap answers false
                r = 1;
                const uint64_t h = siphash13(key_bytes + ko, (uint64_t)len);
                for_each_probe(h, k, m, [&](uint32_t p) {
                    if (!((bitmap[p >> 3] >> (p & 7)) & 1u)) {
                        r = 0;
                        return false;
                    }
                    return true;
                });
            }
        }
        result[i] = r;
    }
}

hipError_t launch_bloom_match(const uint8_t *bitmap, uint64_t bytes, uint32_t k, uint32_t whole, uint32_t kind,
                              uint32_t arg, const uint8_t *key_bytes, const uint64_t *key_off, const uint8_t *is_prefix,
                              const int32_t *qlens, uint64_t n, uint8_t *result, hipStream_t st) {
    if (!n) return hipSuccess;
    PrefixSpec ps{kind, arg, whole, 0, qlens};
    uint64_t b = (n + 255) / 256;
    b = b > 65536 ? 65536 : b;
    hipLaunchKernelGGL(k_bloom_match, dim3((uint32_t)b), dim3(256), 0, st, bitmap, bytes, k, whole, ps, key_bytes, key_off,
                       is_prefix, n, result);
    return hipGetLastError();
}

}  // namespace sdb
