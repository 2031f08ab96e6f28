// sdb_decode.h — kernel arguments of the batched block decoder.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../../include/slatedb_amd.h"

namespace sdb {

struct DecodeArgs {
    const uint8_t *blocks;
    const uint64_t *block_off;  // nblocks+1 (contiguous) or nblocks starts (with block_end)
    const uint64_t *block_end;  // nblocks ends, or NULL: block k ends at block_off[k + 1]
    uint64_t nblocks;
    uint32_t version;
    sdb_decoded_out out;  // device pointers
    // workspace
    uint64_t *cnt, *kbytes;            // per block
    uint8_t *flag;                     // per block: 1 = sequential V2 walk
    uint64_t *rcnt;                    // per block: rows of restart regions 0..3 (16 bits each; ~0: not recorded)
    uint16_t *rowpos;                  // per block: 4 x 32 row positions (region q, row i at q * 32 + i)
    uint64_t *ent_start, *key_start;   // nblocks+1
    uint64_t *tile_x, *tile_y;         // per 1024-block tile (+1)
    unsigned long long *err, *nbad;
    uint32_t *done;                    // k_dec_emit workgroups finished (small batches: the last one finishes)
    uint32_t small;                    // 1: nblocks <= 1024 and one block per wave: k_dec_emit scans the counts itself
    uint32_t descending;               // 1: output in descending iteration order (written mirrored by k_dec_emit)
    uint32_t fail_fast, pad_ff;        // 1: read_blocks semantics (the first failing block fails the call, the
                                       //    columns are unspecified then): the checksums move to the emit pass
    uint32_t *bad_block;
    uint64_t bad_cap;
    uint64_t dn, dkb;                  // descending: entries and key bytes of the whole output (k_dec_emit)
};

struct DecodeWorkspace {
    uint64_t cnt, kbytes, flag, rcnt, rowpos, ent_start, key_start, tile_x, tile_y, err, nbad, done, total;
};
inline DecodeWorkspace decode_workspace_layout(uint64_t nblocks) {
    DecodeWorkspace w{};
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        uint64_t r = off;
        off += (bytes + 255) & ~255ull;
        return r;
    };
    uint64_t nt = (nblocks + 1023) / 1024 + 1;
    w.cnt = take(8 * (nblocks + 1));
    w.kbytes = take(8 * (nblocks + 1));
    w.flag = take(nblocks + 1);
    w.rcnt = take(8 * (nblocks + 1));
    w.rowpos = take(256 * (nblocks + 1));
    w.ent_start = take(8 * (nblocks + 1));
    w.key_start = take(8 * (nblocks + 1));
    w.tile_x = take(8 * (nt + 1));
    w.tile_y = take(8 * (nt + 1));
    w.err = take(8);
    w.nbad = take(8);
    w.done = take(8);
    w.total = off;
    return w;
}

hipError_t launch_decode(DecodeArgs a, hipStream_t st);
hipError_t launch_excl_scan2(const uint64_t *x, const uint64_t *y, uint64_t n, uint64_t *tx, uint64_t *ty,
                             uint64_t *ox, uint64_t *oy, hipStream_t st);

// f3: per-block decompression (sdb_codec.hip)
uint64_t decompress_workspace_bytes(uint64_t nblocks);
hipError_t launch_decompress_plan(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                  uint64_t *out_start, void *ws, hipStream_t st);
hipError_t launch_decompress_run(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                 uint8_t *out, uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end,
                                 unsigned long long *err, hipStream_t st);
uint64_t decompress_once_workspace_bytes(uint64_t nblocks);
hipError_t launch_decompress_once(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                  uint64_t slot_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_start,
                                  uint64_t *out_end, unsigned long long *err, void *ws, hipStream_t st);
// f3: per-block compression, the write side (sdb_codec_enc.hip)
uint64_t compress_workspace_bytes(uint64_t nblocks, uint64_t in_bytes);
hipError_t launch_compress(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                           uint64_t in_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_off,
                           unsigned long long *err, void *ws, hipStream_t st);

}  // namespace sdb
