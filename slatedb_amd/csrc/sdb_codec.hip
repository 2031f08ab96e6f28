// sdb_codec.hip — per-block decompression of a read_blocks range for gfx950.
//
// Replaces the first half of SsTableFormat::decode_block (slatedb/src/format/sst.rs:980-999):
// validate_checksum over the stored (compressed) block, then SsTableFormat::decompress
// (format/sst.rs:884-917) for the LZ-family codecs:
//   CompressionFormat::Lz4    = lz4_flex 0.11.6 block::decompress_size_prepended (Cargo.lock:1945):
//                               u32 little-endian uncompressed size, then one LZ4 block;
//   CompressionFormat::Snappy = snap 1.1.1 raw::Decoder::decompress_vec (Cargo.lock:3406): varint
//                               uncompressed size, then Snappy raw elements.
// Zlib / Zstd (entropy-coded) run in sdb_codec_ent.hip.  Every output block is re-framed as
// Block::encode() ++ CRC32 BE of those bytes, so the output is a plain uncompressed block run that
// sdb_decode_blocks_at decodes unchanged (values then reference the decompressed arena).
//
//   Z1 plan   one thread per block: the declared length from the header -> slot = length + 4
//             (0: unreadable header or more than kMaxBlockOut), exclusive scan -> out_start.
//   Z2 run    one wave per block: the compressed block staged in LDS, wave CRC32 check, then the
//             token stream parsed in lock-step by every lane (wave-uniform reads of the LDS bytes)
//             while literal and match copies are spread over the 64 lanes (a match of offset d copies
//             byte i from op - d + (i mod d): the d bytes before op are complete, so overlapping
//             matches need no serialisation); the image's CRC32 and 16-byte stores.  Blocks larger
//             than the LDS images are decoded by one lane straight between HBM buffers.
#include <mutex>

#include "sdb_crc.h"
#include "sdb_decode.h"
#include "sdb_device.h"

namespace sdb {

constexpr uint32_t kDzThreads = 1024;                   // 16 waves per workgroup, one workgroup per CU
constexpr uint32_t kDzIn = 4096 + 256;                  // compressed bytes staged per wave (a 4 KiB block)
constexpr uint32_t kDzOut = 4096 + 256;                 // decompressed image per wave
constexpr uint64_t kMaxBlockOut = 64ull << 20;          // larger declared lengths: SDB_LIMIT_EXCEEDED
constexpr uint32_t kDzWaveLds = kDzIn + 32 + kDzOut;
constexpr uint32_t kDzLds = 8 * 1024 + (kDzThreads / 64) * kDzWaveLds;  // slicing tables, then the waves
static_assert(kDzLds <= 160 * 1024, "decompress LDS");

struct DzArgs {
    uint32_t codec;
    const uint8_t *blocks;
    const uint64_t *block_off;  // nblocks + 1
    uint64_t nblocks;
    uint64_t *slot;             // workspace: per block slot bytes (nblocks + 1)
    uint8_t *out;
    uint64_t out_cap;
    const uint64_t *out_start;  // nblocks + 1 (the plan)
    uint64_t *out_end;          // nblocks
    unsigned long long *err;    // min (block << 8 | status), ~0 = none
};

// Declared uncompressed length from the payload header (lz4_flex block::uncompressed_size,
// snap raw::decompress_len); -1 when unreadable.
template <typename P>
SDB_DEV int64_t dz_declared(uint32_t codec, P in, uint64_t n) {
    if (codec == SDB_CODEC_LZ4) {
        if (n < 4) return -1;
        return (int64_t)((uint32_t)in[0] | (uint32_t)in[1] << 8 | (uint32_t)in[2] << 16 | (uint32_t)in[3] << 24);
    }
    uint64_t v = 0;
    for (uint32_t i = 0; i < 5; i++) {
        if (i >= n) return -1;
        v |= (uint64_t)(in[i] & 0x7F) << (7 * i);
        if (!(in[i] & 0x80)) return v > 0xFFFFFFFFull ? -1 : (int64_t)v;
    }
    return -1;
}
template <typename P>
SDB_DEV uint32_t dz_header_len(uint32_t codec, P in) {
    if (codec == SDB_CODEC_LZ4) return 4;
    uint32_t i = 0;
    while (in[i] & 0x80) i++;
    return i + 1;
}

__global__ __launch_bounds__(256) void k_dz_plan(DzArgs a) {
    const uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (k > a.nblocks) return;
    uint64_t slot = 0;
    if (k < a.nblocks) {
        const uint64_t s = a.block_off[k], e = a.block_off[k + 1];
        if (e >= s && e - s >= 4) {
            const int64_t len = dz_declared(a.codec, a.blocks + s, e - s - 4);
            if (len >= 0 && (uint64_t)len <= kMaxBlockOut) slot = (uint64_t)len + 4;
        }
    }
    a.slot[k] = slot;
}

// The byte of `p` every lane reads (a wave-uniform LDS broadcast, or one lane's global read), kept scalar.
template <typename P>
SDB_DEV uint32_t ub(P p) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)*p); }

// The 8 bytes at p as one wave-uniform little-endian word: eight byte reads issued together (one LDS
// round trip instead of one per header byte).  Wave mode only: p lies in the staged block, which has
// slack past its end.
template <typename P>
SDB_DEV uint64_t win8(P p) {
    uint32_t b[8];
#pragma unroll
    for (int i = 0; i < 8; i++) b[i] = p[i];
    const uint32_t lo = b[0] | b[1] << 8 | b[2] << 16 | b[3] << 24, hi = b[4] | b[5] << 8 | b[6] << 16 | b[7] << 24;
    return (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)lo) |
           (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)hi) << 32;
}

// Copies of one decoder step: lanes first, first + step, ... (64-lane wave mode, or one lane: 0, 1).
template <typename PI, typename PO>
SDB_DEV void dz_literal(PO out, uint32_t op, PI in, uint32_t ip, uint32_t len, uint32_t first, uint32_t step) {
    for (uint32_t i = first; i < len; i += step) out[op + i] = in[ip + i];
}
template <typename PO>
SDB_DEV void dz_match(PO out, uint32_t op, uint32_t off, uint32_t len, uint32_t first, uint32_t step) {
    if (off >= len) {
        for (uint32_t i = first; i < len; i += step) out[op + i] = out[op - off + i];
    } else {  // overlapping: byte i repeats byte i mod off of the off bytes before op
        uint32_t r = first % off;
        const uint32_t adv = step % off;
        for (uint32_t i = first; i < len; i += step) {
            out[op + i] = out[op - off + r];
            r += adv;
            if (r >= off) r -= off;
        }
    }
}
SDB_DEV void dz_sync(bool wave) {
    if (wave) {
        __builtin_amdgcn_fence(__ATOMIC_RELEASE, "wavefront");
        __builtin_amdgcn_wave_barrier();
        __builtin_amdgcn_fence(__ATOMIC_ACQUIRE, "wavefront");
    }
}

// LZ4 block (lz4_flex decompress_into): token, literal length extension bytes of 255, literals, then
// (unless the input ends there) a u16 LE offset and the match; output may end short of `cap` (the
// declared size: lz4_flex truncates), never past it.  Returns 0 or SDB_DECOMPRESSION_ERROR.
template <typename PI, typename PO>
SDB_DEV int dz_lz4(PI in, uint32_t n, PO out, uint32_t cap, uint32_t *olen, uint32_t first, uint32_t step) {
    const bool wave = step > 1;
    uint32_t ip = 0, op = 0;
    for (;;) {
        if (ip >= n) return SDB_DECOMPRESSION_ERROR;
        const uint32_t tok = ub(in + ip++);
        uint32_t lit = tok >> 4;
        if (lit == 15) {
            uint32_t b;
            do {
                if (ip >= n) return SDB_DECOMPRESSION_ERROR;
                b = ub(in + ip++);
                lit += b;
            } while (b == 255);
        }
        if (lit > n - ip || lit > cap - op) return SDB_DECOMPRESSION_ERROR;
        dz_literal(out, op, in, ip, lit, first, step);
        ip += lit;
        op += lit;
        if (ip == n) break;
        if (n - ip < 2) return SDB_DECOMPRESSION_ERROR;
        const uint32_t off = ub(in + ip) | ub(in + ip + 1) << 8;
        ip += 2;
        uint32_t ml = (tok & 15) + 4;
        if ((tok & 15) == 15) {
            uint32_t b;
            do {
                if (ip >= n) return SDB_DECOMPRESSION_ERROR;
                b = ub(in + ip++);
                ml += b;
            } while (b == 255);
        }
        if (off == 0 || off > op || ml > cap - op) return SDB_DECOMPRESSION_ERROR;
        dz_sync(wave);  // the literals (other lanes' writes) before the match reads them
        dz_match(out, op, off, ml, first, step);
        dz_sync(wave);
        op += ml;
    }
    *olen = op;
    return 0;
}

// Snappy raw elements (snap raw::Decoder): literal (length - 1 in the tag, or 1..4 LE bytes for tags
// 60..63), copies with 1-, 2- and 4-byte offsets; the output must end exactly at `len`.
template <typename PI, typename PO>
SDB_DEV int dz_snappy(PI in, uint32_t n, PO out, uint32_t len, uint32_t first, uint32_t step) {
    const bool wave = step > 1;
    uint32_t ip = 0, op = 0;
    while (ip < n) {
        const uint32_t tag = ub(in + ip++);
        if ((tag & 3) == 0) {
            uint32_t l = tag >> 2;
            if (l >= 60) {
                const uint32_t nb = l - 59;
                if (n - ip < nb) return SDB_DECOMPRESSION_ERROR;
                l = 0;
                for (uint32_t i = 0; i < nb; i++) l |= ub(in + ip + i) << (8 * i);
                ip += nb;
                if (l == 0xFFFFFFFFu) return SDB_DECOMPRESSION_ERROR;
            }
            l += 1;
            if (l > n - ip || l > len - op) return SDB_DECOMPRESSION_ERROR;
            dz_literal(out, op, in, ip, l, first, step);
            ip += l;
            op += l;
            continue;
        }
        uint32_t l, off;
        if ((tag & 3) == 1) {
            if (ip >= n) return SDB_DECOMPRESSION_ERROR;
            l = 4 + ((tag >> 2) & 7);
            off = ((tag >> 5) << 8) | ub(in + ip++);
        } else if ((tag & 3) == 2) {
            if (n - ip < 2) return SDB_DECOMPRESSION_ERROR;
            l = 1 + (tag >> 2);
            off = ub(in + ip) | ub(in + ip + 1) << 8;
            ip += 2;
        } else {
            if (n - ip < 4) return SDB_DECOMPRESSION_ERROR;
            l = 1 + (tag >> 2);
            off = ub(in + ip) | ub(in + ip + 1) << 8 | ub(in + ip + 2) << 16 | ub(in + ip + 3) << 24;
            ip += 4;
        }
        if (off == 0 || off > op || l > len - op) return SDB_DECOMPRESSION_ERROR;
        dz_sync(wave);
        dz_match(out, op, off, l, first, step);
        dz_sync(wave);
        op += l;
    }
    return op == len ? 0 : SDB_DECOMPRESSION_ERROR;
}

// The same LZ4 decode for the wave mode (input staged in LDS): each sequence reads its header through two
// 8-byte windows, the second issued before the literal copy so its latency overlaps it.
template <typename PI, typename PO>
SDB_DEV int dz_lz4_win(PI in, uint32_t n, PO out, uint32_t cap, uint32_t *olen, uint32_t first) {
    uint32_t ip = 0, op = 0;
    for (;;) {
        if (ip >= n) return SDB_DECOMPRESSION_ERROR;
        uint64_t w = win8(in + ip);
        const uint32_t tok = (uint32_t)w & 0xFF;
        uint32_t c = 1, lit = tok >> 4;
        if (lit == 15) {
            uint32_t b;
            do {
                if (ip + c >= n) return SDB_DECOMPRESSION_ERROR;
                if (c == 8) {
                    ip += 8;
                    c = 0;
                    w = win8(in + ip);
                }
                b = (uint32_t)(w >> (8 * c)) & 0xFF;
                c++;
                lit += b;
            } while (b == 255);
        }
        ip += c;
        if (lit > n - ip || lit > cap - op) return SDB_DECOMPRESSION_ERROR;
        const bool last = ip + lit == n;
        const uint64_t w2 = last ? 0 : win8(in + ip + lit);  // offset + match extension, in flight over the copy
        dz_literal(out, op, in, ip, lit, first, 64u);
        ip += lit;
        op += lit;
        if (last) break;
        if (n - ip < 2) return SDB_DECOMPRESSION_ERROR;
        const uint32_t off = (uint32_t)w2 & 0xFFFF;
        uint32_t ml = (tok & 15) + 4;
        c = 2;
        w = w2;
        if ((tok & 15) == 15) {
            uint32_t b;
            do {
                if (ip + c >= n) return SDB_DECOMPRESSION_ERROR;
                if (c == 8) {
                    ip += 8;
                    c = 0;
                    w = win8(in + ip);
                }
                b = (uint32_t)(w >> (8 * c)) & 0xFF;
                c++;
                ml += b;
            } while (b == 255);
        }
        ip += c;
        if (off == 0 || off > op || ml > cap - op) return SDB_DECOMPRESSION_ERROR;
        dz_sync(true);  // the literals and earlier matches (other lanes' writes) before the match reads them
        dz_match(out, op, off, ml, first, 64u);
        op += ml;
    }
    *olen = op;
    return 0;
}

// Snappy for the wave mode: one 8-byte window per element (tag + up to four length / offset bytes).
template <typename PI, typename PO>
SDB_DEV int dz_snappy_win(PI in, uint32_t n, PO out, uint32_t len, uint32_t first) {
    uint32_t ip = 0, op = 0;
    while (ip < n) {
        const uint64_t w = win8(in + ip);
        const uint32_t tag = (uint32_t)w & 0xFF;
        const uint32_t rest = n - ip - 1;  // bytes after the tag
        if ((tag & 3) == 0) {
            uint32_t l = tag >> 2, nb = 0;
            if (l >= 60) {
                nb = l - 59;
                if (rest < nb) return SDB_DECOMPRESSION_ERROR;
                l = (uint32_t)(w >> 8) & (nb == 4 ? 0xFFFFFFFFu : ((1u << (8 * nb)) - 1));
                if (l == 0xFFFFFFFFu) return SDB_DECOMPRESSION_ERROR;
            }
            l += 1;
            ip += 1 + nb;
            if (l > n - ip || l > len - op) return SDB_DECOMPRESSION_ERROR;
            dz_literal(out, op, in, ip, l, first, 64u);
            ip += l;
            op += l;
            continue;
        }
        uint32_t l, off, nb;
        if ((tag & 3) == 1) {
            nb = 1;
            l = 4 + ((tag >> 2) & 7);
            off = ((tag >> 5) << 8) | ((uint32_t)(w >> 8) & 0xFF);
        } else if ((tag & 3) == 2) {
            nb = 2;
            l = 1 + (tag >> 2);
            off = (uint32_t)(w >> 8) & 0xFFFF;
        } else {
            nb = 4;
            l = 1 + (tag >> 2);
            off = (uint32_t)(w >> 8);
        }
        if (rest < nb) return SDB_DECOMPRESSION_ERROR;
        ip += 1 + nb;
        if (off == 0 || off > op || l > len - op) return SDB_DECOMPRESSION_ERROR;
        dz_sync(true);
        dz_match(out, op, off, l, first, 64u);
        op += l;
    }
    return op == len ? 0 : SDB_DECOMPRESSION_ERROR;
}

template <typename PI, typename PO>
SDB_DEV int dz_payload(uint32_t codec, PI in, uint32_t n, PO out, uint32_t decl, uint32_t *olen, uint32_t first,
                       uint32_t step) {
    const uint32_t h = dz_header_len(codec, in);
    if (codec == SDB_CODEC_LZ4)
        return step > 1 ? dz_lz4_win(in + h, n - h, out, decl, olen, first) : dz_lz4(in + h, n - h, out, decl, olen, first, step);
    *olen = decl;
    return step > 1 ? dz_snappy_win(in + h, n - h, out, decl, first) : dz_snappy(in + h, n - h, out, decl, first, step);
}

// crc32fast::hash of msg[0, n) (generic pointer: LDS or HBM), every lane; tab: slicing tables in LDS.
SDB_DEV uint32_t dz_crc(const uint8_t *msg, uint64_t n, const uint32_t (*tab)[256]) {
    if (n >= 4) return wave_crc32_lds(msg, (uint32_t)n, tab);
    uint32_t x = 0xFFFFFFFFu;
    for (uint32_t q = 0; q < n; q++) x = tab[0][(x ^ msg[q]) & 0xFF] ^ (x >> 8);
    return x ^ 0xFFFFFFFFu;
}

__global__ __launch_bounds__(kDzThreads) void k_dz_run(DzArgs a) {
    extern __shared__ __attribute__((aligned(16))) uint8_t smem[];
    crc_slice_tables_to_lds((lu32 *)smem);
    __syncthreads();
    const uint32_t(*tab)[256] = (const uint32_t(*)[256])smem;
    const uint32_t l = (uint32_t)lane_id(), wave = threadIdx.x >> 6;
    uint8_t *stage = smem + 8 * 1024 + wave * kDzWaveLds;  // 16-byte granules of the compressed block
    uint8_t *img = stage + kDzIn + 32;                      // the decompressed block
    const uint64_t nw = (uint64_t)gridDim.x * (blockDim.x >> 6);
    for (uint64_t k = (uint64_t)blockIdx.x * (blockDim.x >> 6) + wave; k < a.nblocks; k += nw) {
        const uint64_t s = a.block_off[k], e = a.block_off[k + 1], o = a.out_start[k];
        const uint64_t slot = a.out_start[k + 1] - o;
        int st = 0;
        uint32_t ol = 0;
        const uint8_t *in = nullptr;
        uint64_t bl = 0;
        if (e < s || e - s < 4 || e - s > 0xFFFFFFFFull) {
            st = SDB_CORRUPT_BLOCK;
        } else {
            bl = e - s - 4;
            const bool staged = bl <= kDzIn;
            if (staged) {
                const uint64_t a0 = s & ~15ull;
                const uint32_t ng = (uint32_t)((((e + 15) & ~15ull) - a0) >> 4);
                const uint4 *src = (const uint4 *)(a.blocks + a0);
                for (uint32_t q = l; q < ng; q += 64) ((uint4 *)stage)[q] = src[q];
                dz_sync(true);
                in = stage + (s & 15);
            } else {
                in = a.blocks + s;
            }
            const uint32_t stored = (uint32_t)in[bl] << 24 | (uint32_t)in[bl + 1] << 16 | (uint32_t)in[bl + 2] << 8 |
                                    (uint32_t)in[bl + 3];
            if (dz_crc(in, bl, tab) != stored) {
                st = SDB_CHECKSUM_MISMATCH;  // validate_checksum (format/sst.rs:1029-1038)
            } else if (slot == 0) {
                st = dz_declared(a.codec, in, bl) < 0 ? SDB_DECOMPRESSION_ERROR : SDB_LIMIT_EXCEEDED;
            } else if (o + slot > a.out_cap) {
                st = SDB_INVALID_ARGUMENT;
            } else {
                const uint32_t decl = (uint32_t)(slot - 4);
                if (staged && decl <= kDzOut) {
                    st = dz_payload(a.codec, (const uint8_t *)in, (uint32_t)bl, img, decl, &ol, l, 64u);
                    dz_sync(true);
                    if (!st) {
                        const uint32_t c = dz_crc(img, ol, tab);
                        if (l == 0) {
                            img[ol] = (uint8_t)(c >> 24);
                            img[ol + 1] = (uint8_t)(c >> 16);
                            img[ol + 2] = (uint8_t)(c >> 8);
                            img[ol + 3] = (uint8_t)c;
                        }
                        dz_sync(true);
                        // 16-byte stores (unaligned in HBM, aligned in LDS), the < 16-byte tail by bytes
                        uint8_t *g = a.out + o;
                        const uint32_t L = ol + 4, nfull = L >> 4;
                        for (uint32_t q = l; q < nfull; q += 64) {
                            const uint4 v = ((const uint4 *)img)[q];
                            __builtin_memcpy(g + 16 * q, &v, 16);
                        }
                        if (l < (L & 15)) g[(nfull << 4) + l] = img[(nfull << 4) + l];
                    }
                } else {
                    // one lane, HBM to HBM (the match reads see the lane's own earlier stores)
                    uint8_t *g = a.out + o;
                    int r = 0;
                    uint32_t w = 0;
                    if (l == 0) r = dz_payload(a.codec, in, (uint32_t)bl, g, decl, &w, 0u, 1u);
                    st = __shfl(r, 0, 64);
                    ol = (uint32_t)__shfl((int)w, 0, 64);
                    __threadfence_block();
                    dz_sync(true);
                    if (!st) {
                        const uint32_t c = dz_crc(g, ol, tab);
                        if (l == 0) {
                            g[ol] = (uint8_t)(c >> 24);
                            g[ol + 1] = (uint8_t)(c >> 16);
                            g[ol + 2] = (uint8_t)(c >> 8);
                            g[ol + 3] = (uint8_t)c;
                        }
                    }
                }
            }
        }
        if (l == 0) {
            a.out_end[k] = st ? o : o + ol + 4;
            if (st) atomicMin(a.err, (unsigned long long)((k << 8) | (uint64_t)st));
        }
        dz_sync(true);
    }
}

__global__ void k_dz_init(unsigned long long *err) {
    if (threadIdx.x == 0) *err = ~0ull;
}

uint64_t decompress_workspace_bytes(uint64_t nblocks) {
    const uint64_t nt = (nblocks + 1023) / 1024 + 1;
    return 256 + 8 * (nblocks + 2) * 2 + 16 * (nt + 2) + 256;
}

static std::once_flag g_dz_once;

// entropy-coded codecs (sdb_codec_ent.hip)
hipError_t launch_ent_slots(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                            uint64_t *slot, hipStream_t st);
hipError_t launch_ent_run(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks, uint8_t *out,
                          uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end, unsigned long long *err,
                          hipStream_t st);
static bool ent_codec(uint32_t codec) { return codec == SDB_CODEC_ZLIB || codec == SDB_CODEC_ZSTD; }

hipError_t launch_decompress_plan(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                  uint64_t *out_start, void *ws, hipStream_t st) {
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    const uint64_t nt = (nblocks + 1023) / 1024 + 1;
    DzArgs a{};
    a.codec = codec;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
    a.slot = (uint64_t *)w;
    uint64_t *scratch = a.slot + (nblocks + 2);
    uint64_t *tx = scratch + (nblocks + 2), *ty = tx + (nt + 1);
    if (ent_codec(codec)) {
        const hipError_t e = launch_ent_slots(codec, blocks, block_off, nblocks, a.slot, st);
        if (e != hipSuccess) return e;
    } else {
        hipLaunchKernelGGL(k_dz_plan, dim3((uint32_t)((nblocks + 256) / 256)), dim3(256), 0, st, a);
    }
    return launch_excl_scan2(a.slot, a.slot, nblocks, tx, ty, out_start, scratch, st);
}

hipError_t launch_decompress_run(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                 uint8_t *out, uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end,
                                 unsigned long long *err, hipStream_t st) {
    std::call_once(g_dz_once, [] {
        (void)hipFuncSetAttribute((const void *)k_dz_run, hipFuncAttributeMaxDynamicSharedMemorySize, (int)kDzLds);
        (void)hipGetLastError();
    });
    DzArgs a{};
    a.codec = codec;
    a.blocks = blocks;
    a.block_off = block_off;
    a.nblocks = nblocks;
    a.out = out;
    a.out_cap = out_cap;
    a.out_start = out_start;
    a.out_end = out_end;
    a.err = err;
    hipLaunchKernelGGL(k_dz_init, dim3(1), dim3(64), 0, st, err);
    if (ent_codec(codec)) return launch_ent_run(codec, blocks, block_off, nblocks, out, out_cap, out_start, out_end, err, st);
    if (nblocks) {
        int dev = 0, cus = 0;
        (void)hipGetDevice(&dev);
        (void)hipDeviceGetAttribute(&cus, hipDeviceAttributeMultiprocessorCount, dev);
        uint64_t wgs = (nblocks + 15) / 16;
        const uint64_t most = (uint64_t)(cus > 0 ? cus : 256) * 2;
        if (wgs > most) wgs = most;
        hipLaunchKernelGGL(k_dz_run, dim3((uint32_t)wgs), dim3(kDzThreads), kDzLds, st, a);
    }
    return hipGetLastError();
}

// ---- decode once: no host synchronisation between sizing and decompressing --------------------------------
// zlib's plan is a whole inflate (the stream does not record its length), so decode-once inflates every block
// once into a fixed slot of slot_bytes (out_start[k] = k * slot_bytes), lists the blocks whose output overflowed
// their slot, and only those are planned and inflated again, packed after the slots.  The other codecs' plans
// read a length header, so for them it is the plan and the run back to back on the stream.
bool zl_once_supported();
hipError_t launch_zl_once_slots(const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks, const uint32_t *list,
                                const unsigned long long *nlist, uint64_t *slot, hipStream_t st);
hipError_t launch_zl_once_run(int mode, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks, uint8_t *out,
                              uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end, unsigned long long *err,
                              const uint32_t *list, const unsigned long long *nlist, bool out_by_block, uint32_t *ovf_list,
                              unsigned long long *ovf_count, uint32_t *dyn_list, unsigned long long *dyn_count,
                              uint64_t *wres, hipStream_t st);

uint64_t decompress_once_workspace_bytes(uint64_t nblocks) {
    return decompress_workspace_bytes(nblocks) + 8 * (nblocks + 2) + 8 * (nblocks + 2) + 16 * (nblocks + 2) + 1024;
}

#ifndef SDB_ZL_WIDE
#define SDB_ZL_WIDE 1
#endif

__global__ void k_zo_init(uint64_t *out_start, uint64_t nblocks, uint64_t slot_bytes, unsigned long long *err,
                          unsigned long long *nlist, unsigned long long *ndyn) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i <= nblocks) out_start[i] = i * slot_bytes;
    if (i == 0) {
        *err = ~0ull;
        *nlist = 0;
        *ndyn = 0;
    }
}

// pos: the overflow list's exclusive scan (nblocks + 1 values, zero past the list) -> absolute positions after
// the slots; the listed blocks' out_start, and out_start[nblocks] = the bytes of out the call used
__global__ void k_zo_fix(uint64_t *pos, uint64_t *out_start, uint64_t nblocks, uint64_t base, const uint32_t *list,
                         const unsigned long long *nlist) {
    const uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x;
    if (i > nblocks) return;
    const uint64_t n = *nlist < nblocks ? *nlist : nblocks;
    const uint64_t p = base + pos[i];
    pos[i] = p;
    if (i < n) out_start[list[i]] = p;
    if (i == nblocks) out_start[nblocks] = p;
}

hipError_t launch_decompress_once(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                  uint64_t slot_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_start,
                                  uint64_t *out_end, unsigned long long *err, void *ws, hipStream_t st) {
    if (codec != SDB_CODEC_ZLIB || !zl_once_supported()) {
        const hipError_t e = launch_decompress_plan(codec, blocks, block_off, nblocks, out_start, ws, st);
        if (e != hipSuccess) return e;
        return launch_decompress_run(codec, blocks, block_off, nblocks, out, out_cap, out_start, out_end, err, st);
    }
    uint8_t *w = (uint8_t *)(((uintptr_t)ws + 255) & ~(uintptr_t)255);
    const uint64_t nt = (nblocks + 1023) / 1024 + 1;
    uint64_t *slot = (uint64_t *)w;
    uint64_t *scratch = slot + (nblocks + 2);
    uint64_t *tx = scratch + (nblocks + 2), *ty = tx + (nt + 1);
    uint64_t *pos = ty + (nt + 1);
    unsigned long long *nlist = (unsigned long long *)(pos + (nblocks + 2));
    unsigned long long *ndyn = nlist + 1;
    uint32_t *list = (uint32_t *)(ndyn + 1);
    uint32_t *dyn = list + (nblocks + 2);
    uint64_t *wres = (uint64_t *)(((uintptr_t)(dyn + (nblocks + 2)) + 15) & ~(uintptr_t)15);
    const uint32_t g = (uint32_t)((nblocks + 256) / 256);
    hipLaunchKernelGGL(k_zo_init, dim3(g), dim3(256), 0, st, out_start, nblocks, slot_bytes, err, nlist, ndyn);
    hipError_t e;
    if (SDB_ZL_WIDE) {
        // 1. every block once into its slot, all 64 lanes decoding against the fixed code's shared tables;
        //    blocks with dynamic-Huffman deflate blocks listed, then decoded by the per-decoder-table run into
        //    their slots (out_start[block]); overflowed blocks listed by both
        e = launch_zl_once_run(1, blocks, block_off, nblocks, out, out_cap, out_start, out_end, err, nullptr, nullptr,
                               false, list, nlist, dyn, ndyn, wres, st);
        if (e == hipSuccess)
            e = launch_zl_once_run(0, blocks, block_off, nblocks, out, out_cap, out_start, out_end, err, dyn, ndyn, true,
                                   list, nlist, nullptr, nullptr, nullptr, st);
    } else {
        // 1. every block once into its slot; the overflowed ones listed
        e = launch_zl_once_run(0, blocks, block_off, nblocks, out, out_cap, out_start, out_end, err, nullptr, nullptr,
                               false, list, nlist, nullptr, nullptr, nullptr, st);
    }
    // 2. the listed blocks' exact sizes, packed after the slots, and their inflate
    if (e == hipSuccess) e = launch_zl_once_slots(blocks, block_off, nblocks, list, nlist, slot, st);
    if (e == hipSuccess) e = launch_excl_scan2(slot, slot, nblocks, tx, ty, pos, scratch, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_zo_fix, dim3(g), dim3(256), 0, st, pos, out_start, nblocks, nblocks * slot_bytes, list, nlist);
    return launch_zl_once_run(0, blocks, block_off, nblocks, out, out_cap, pos, out_end, err, list, nlist, false, nullptr,
                              nullptr, nullptr, nullptr, nullptr, st);
}

}  // namespace sdb
