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
    const uint64_t bk = 4ull * pl.nslices + 2ull * pl.nslices * bloom_slot_cap(pl);
    pl.one_pass = pl.sb <= 16 && bk <= 4ull * (2ull * pl.nslices + (uint64_t)pl.T * pl.k) ? 1u : 0u;
    return pl;
}

uint32_t bloom_slot_cap(const BloomPlan &pl) {
    // uniform probes: a slot (slice, tile) receives the probes of the tile's T keys that land in the
    // slice (2^sb of the m bits); + 6 sigma + 16
    const double frac = pl.m ? (double)(1ull << pl.sb) / pl.m : 1.0;
    const double mean = (double)pl.T * pl.k * (frac < 1.0 ? frac : 1.0);
    uint64_t cap = (uint64_t)(mean + 6.0 * __builtin_sqrt(mean + 1.0)) + 16;
    cap = (cap + 3) & ~3ull;
    const uint64_t most = (uint64_t)pl.T * pl.k;  // a slot never holds more than the tile's probes
    if (cap > most) cap = (most + 3) & ~3ull;
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
    return bloom_slots_bytes(bloom_plan(n, k, bitmap_bytes));
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
    if (pl.one_pass) return 4 * (size_t)pl.nslices + 2 * (size_t)pl.nslices * bloom_slot_cap(pl);
    return 4 * (2 * (size_t)pl.nslices + (size_t)pl.T * pl.k);
}
size_t bloom_fill_lds(const BloomPlan &pl) { return 4 * ((size_t)(1u << (pl.sb - 5)) + pl.tiles); }

hipError_t launch_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                              uint32_t num_probes, uint8_t *bitmap, uint64_t bitmap_bytes, void *ws,
                              hipStream_t st) {
    if (bitmap_bytes == 0) return hipSuccess;
    if (n == 0 || num_probes == 0) return hipMemsetAsync(bitmap, 0, bitmap_bytes, st);
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
