// sdb_api.cpp — the C ABI (include/slatedb_amd.h): argument checks, workspace carving, launches,
// and the host-buffer runtime (device arena + pinned staging + stream per handle).
//
// Host side of the drop-in for slatedb's EncodedSsTableBuilder / SsTableFormat::read_blocks
// (slatedb/src/sst_builder.rs:224-417, format/sst.rs:938-1038).  No CPU fallback: without a HIP
// device every compute entry point returns SDB_DEVICE_ERROR.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <mutex>
#include <thread>
#include <vector>

#include "../../include/slatedb_amd.h"
#include "sdb_decode.h"
#include "sdb_bloom.h"
#include "sdb_compact.h"

namespace sdb {
struct LookupArgs {
    sdb_sst_view v;
    const uint8_t *key_bytes;
    const uint64_t *key_off;
    uint64_t nkeys;
    uint32_t desc;
    sdb_lookup_out out;
    uint32_t *qrange;
    uint8_t *mark;
    int32_t *bstat;
};
uint64_t lookup_workspace_bytes(uint64_t num_blocks, uint64_t nkeys);
hipError_t launch_lookup(LookupArgs a, hipStream_t st);
}  // namespace sdb

using namespace sdb;

namespace {

inline hipStream_t S(void *s) { return reinterpret_cast<hipStream_t>(s); }

uint16_t num_probes_for(uint32_t bpk) { return (uint16_t)((float)bpk * 0.69f); }  // filter.rs:235-239

uint64_t filter_bytes_for(uint64_t n, uint32_t bpk) {  // filter.rs:65-69 (u32 arithmetic)
    uint32_t bits = (uint32_t)n * bpk;
    return bits / 8u + (bits % 8u != 0);
}

bool device_ok() {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return false;
    return n > 0;
}

sdb_status check_params(const sdb_sst_params *p) {
    if (!p) return SDB_INVALID_ARGUMENT;
    if (p->sst_version != 1 && p->sst_version != 2) return SDB_INVALID_ARGUMENT;
    if (p->block_size == 0) return SDB_INVALID_ARGUMENT;
    if (p->sst_version == 2 && p->restart_interval == 0) return SDB_INVALID_ARGUMENT;
    if (p->sst_type > SDB_SST_WAL || (p->sst_type == SDB_SST_WAL && p->sst_version != 2)) return SDB_INVALID_ARGUMENT;
    if (p->prefix_kind > SDB_PREFIX_LENGTHS || (p->prefix_kind == SDB_PREFIX_DELIM && p->prefix_arg > 255))
        return SDB_INVALID_ARGUMENT;
    if (p->no_whole_key && p->prefix_kind == SDB_PREFIX_NONE) return SDB_INVALID_ARGUMENT;  // nothing to hash
    return SDB_OK;
}

template <typename T>
T *carve(void *base, uint64_t off) {
    return reinterpret_cast<T *>(reinterpret_cast<uint8_t *>(base) + off);
}

}  // namespace

extern "C" {

uint32_t sdb_abi_version(void) { return SDB_ABI_VERSION; }

int sdb_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

const char *sdb_status_name(int s) {
    switch (s) {
        case SDB_OK: return "OK";
        case SDB_EMPTY_KEY: return "EMPTY_KEY";
        case SDB_EMPTY_BLOCK: return "EMPTY_BLOCK";
        case SDB_CHECKSUM_MISMATCH: return "CHECKSUM_MISMATCH";
        case SDB_INVALID_ROW_FLAGS: return "INVALID_ROW_FLAGS";
        case SDB_INVALID_VERSION: return "INVALID_VERSION";
        case SDB_LIMIT_EXCEEDED: return "LIMIT_EXCEEDED";
        case SDB_UNSUPPORTED: return "UNSUPPORTED";
        case SDB_INVALID_ARGUMENT: return "INVALID_ARGUMENT";
        case SDB_CORRUPT_BLOCK: return "CORRUPT_BLOCK";
        case SDB_MERGE_OPERATOR_MISSING: return "MERGE_OPERATOR_MISSING";
        case SDB_DECOMPRESSION_ERROR: return "DECOMPRESSION_ERROR";
        case SDB_DEVICE_ERROR: return "DEVICE_ERROR";
        default: return "UNKNOWN";
    }
}

uint64_t sdb_bloom_filter_bytes(uint64_t num_keys, uint32_t bits_per_key) {
    return filter_bytes_for(num_keys, bits_per_key);
}
uint32_t sdb_bloom_num_probes(uint32_t bits_per_key) { return num_probes_for(bits_per_key); }

sdb_status sdb_encode_bounds(uint64_t n, uint64_t total_key_bytes, uint64_t total_val_bytes,
                             const sdb_sst_params *params, uint64_t *data_cap, uint64_t *block_cap,
                             uint64_t *bloom_cap) {
    sdb_status st = check_params(params);
    if (st) return st;
    // every row <= 15 B of varints/headers + key + value + 25 B trailer; each entry may be its own
    // block (+2 offset +2 count +4 crc).  V0 rows: 4 + key + 9 + 16 + 4 + value, +2 offset.
    if (data_cap) *data_cap = total_key_bytes + total_val_bytes + 64 * n + 64;
    if (block_cap) *block_cap = n + 1;
    // a prefix-extractor filter holds up to one prefix hash per key besides the full-key hash
    const uint64_t hashes = (params->prefix_kind ? n : 0) + (params->no_whole_key ? 0 : n);
    if (bloom_cap)
        *bloom_cap = params->bloom_bits_per_key ? ((filter_bytes_for(hashes, params->bloom_bits_per_key) + 3) & ~3ull) + 16
                                                : 16;
    return SDB_OK;
}

}  // extern "C"

namespace {
// One SST's workspace region (256-byte multiple) inside a set's workspace.
bool prefix_filter(const sdb_sst_params *p) { return p->prefix_kind != SDB_PREFIX_NONE || p->no_whole_key; }
uint64_t sst_ws_bytes(uint64_t n, const sdb_sst_params *p) {
    if (prefix_filter(p))  // the prefix filter's scratch instead of the fused bloom's slots
        return (encode_workspace_offsets(n, false).bloom_rep + prefix_workspace_bytes(n) + 511) & ~255ull;
    const uint64_t fb = p->bloom_bits_per_key ? filter_bytes_for(n, p->bloom_bits_per_key) : 0;
    return (encode_workspace_layout(n, fb, num_probes_for(p->bloom_bits_per_key)).total + 255) & ~255ull;
}

sdb_status check_sst(const sdb_kv_batch *b, const sdb_sst_params *p, const sdb_sst_out *out) {
    if (!b || !out || !out->summary) return SDB_INVALID_ARGUMENT;
    const uint64_t n = b->n;
    if (n >= (1ull << 31)) return SDB_LIMIT_EXCEEDED;
    if (n && (!b->key_bytes || !b->key_off || !b->val_off)) return SDB_INVALID_ARGUMENT;
    const bool want_filter = p->sst_type != SDB_SST_WAL && p->bloom_bits_per_key > 0 && n >= p->min_filter_keys;
    const uint64_t hashes = prefix_filter(p) ? (p->prefix_kind ? n : 0) + (p->no_whole_key ? 0 : n) : n;
    const uint64_t fb = want_filter ? filter_bytes_for(hashes, p->bloom_bits_per_key) : 0;
    if (want_filter && fb && (!out->bloom || out->bloom_cap < fb)) return SDB_INVALID_ARGUMENT;
    if (want_filter && prefix_filter(p) && ((uintptr_t)out->bloom & 3)) return SDB_INVALID_ARGUMENT;
    if (want_filter && p->prefix_kind == SDB_PREFIX_LENGTHS && n && !b->prefix_len) return SDB_INVALID_ARGUMENT;
    if (n && (!out->data || !out->block_off || !out->block_first_entry || !out->index_key_len || !out->block_stats))
        return SDB_INVALID_ARGUMENT;
    return SDB_OK;
}

// The slot of one SST (no launches); *standalone_bloom: the filter needs the standalone build first.
SstSlot plan_slot(const sdb_kv_batch *b, const sdb_sst_params *p, const sdb_sst_out *out, uint8_t *ws,
                  bool *standalone_bloom) {
    const uint64_t n = b->n;
    const bool want_filter = p->sst_type != SDB_SST_WAL && p->bloom_bits_per_key > 0 && n >= p->min_filter_keys;
    const uint64_t fb = want_filter ? filter_bytes_for(n, p->bloom_bits_per_key) : 0;
    SstSlot s{};
    s.key_bytes = b->key_bytes;
    s.key_off = b->key_off;
    s.val_bytes = b->val_bytes;
    s.val_off = b->val_off;
    s.kind = b->kind;
    s.seq = b->seq;
    s.create_ts = b->create_ts;
    s.expire_ts = b->expire_ts;
    s.ts_mask = b->ts_mask;
    s.n = n;
    s.out_data = out->data;
    s.out_block_off = out->block_off;
    s.out_block_first = out->block_first_entry;
    s.out_index_key_len = out->index_key_len;
    s.out_block_stats = out->block_stats;
    s.data_cap = out->data_cap;
    s.block_cap = out->block_cap;
    s.summary = out->summary;
    s.bloom_out = out->bloom;
    s.bloom_len = fb;
    s.ws = ws;
    s.num_probes = want_filter ? num_probes_for(p->bloom_bits_per_key) : 0;
    s.filter_built = want_filter ? 1 : 0;
    s.has_filter_ws = (p->bloom_bits_per_key && filter_bytes_for(n, p->bloom_bits_per_key)) ? 1 : 0;
    s.nchunks = (uint32_t)((n + kChunk - 1) / kChunk);
    s.nfacts = (uint32_t)((n + kFactsEntries - 1) / kFactsEntries);
    fill_ws_layout(s);
    {   // chunks per group: about sqrt(nchunks), so k_enum walks <= ~2 sqrt(nchunks) tables
        uint32_t g = 16;
        while ((uint64_t)g * g < s.nchunks) g++;
        s.group = g;
    }
    *standalone_bloom = false;
    if (want_filter && prefix_filter(p)) {  // device-counted size: built before the set (sdb_bloom.hip)
        s.prefix_bloom = 1;
        s.bloom_len = 0;
        *standalone_bloom = true;
    } else if (want_filter && n) {
        // the bloom is fused with the encode (k_facts hashes, binned per chunk) when the binned build
        // fits; otherwise the standalone build runs before the set
        const BloomPlan pl = bloom_plan(n, s.num_probes, fb, kChunk);
        if (bloom_plan_fits(pl)) {
            s.bloom_fused = 1;
            s.bpl = pl;
            s.slot_cap = bloom_slot_cap(pl);
        } else {
            *standalone_bloom = true;
        }
    }
    return s;
}

SstSet set_header(const sdb_sst_params *p) {
    SstSet P{};
    P.block_size = p->block_size;
    P.restart_interval = p->sst_version == 2 ? p->restart_interval : 1;
    P.version = p->sst_version;
    P.wal = p->sst_type == SDB_SST_WAL;
    // a block holds at most (block_size - 2) / 12 + 1 entries (smallest row: 12 bytes in V2, 13 in V1);
    // blocks longer than the lookahead continue from HBM inside k_seg
    const uint64_t look = (uint64_t)p->block_size / 12 + 2;
    P.seg_look = (uint32_t)(look < kSegLook ? look : kSegLook);
    return P;
}
}  // namespace

extern "C" {

uint64_t sdb_encode_workspace_bytes(uint64_t n, const sdb_sst_params *params) {
    if (!params) return 0;
    return sst_ws_bytes(n, params) + 256;
}

uint64_t sdb_encode_ssts_workspace_bytes(uint32_t count, const sdb_kv_batch *batches, const sdb_sst_params *params) {
    if (!params || (count && !batches)) return 0;
    uint64_t t = 256;
    for (uint32_t i = 0; i < count; i++) t += sst_ws_bytes(batches[i].n, params);
    return t;
}

sdb_status sdb_encode_ssts(uint32_t count, const sdb_kv_batch *batches, const sdb_sst_params *p,
                           const sdb_sst_out *outs, void *workspace, uint64_t workspace_bytes, void *stream) {
    sdb_status st = check_params(p);
    if (st) return st;
    if (count && (!batches || !outs)) return SDB_INVALID_ARGUMENT;
    for (uint32_t i = 0; i < count; i++)
        if ((st = check_sst(&batches[i], p, &outs[i]))) return st;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    if (!workspace || workspace_bytes < sdb_encode_ssts_workspace_bytes(count, batches, p)) return SDB_INVALID_ARGUMENT;
    hipStream_t s = S(stream);
    uint8_t *ws = (uint8_t *)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    SstSet P = set_header(p);
    size_t bin_lds = 0, fill_lds = 0;
    auto flush = [&]() -> bool {
        const bool ok = launch_encode_set(P, bin_lds, fill_lds, s) == hipSuccess;
        SstSet q = set_header(p);
        P = q;
        bin_lds = fill_lds = 0;
        return ok;
    };
    for (uint32_t i = 0; i < count; i++) {
        bool standalone = false;
        const SstSlot slot = plan_slot(&batches[i], p, &outs[i], ws, &standalone);
        ws += sst_ws_bytes(batches[i].n, p);
        if (standalone) {
            SstSet one = set_header(p);
            one.count = 1;
            one.s[0] = slot;
            const EncodeArgs a = make_args(one, 0);
            stage_mark(s, kStBloom, true);
            hipError_t e;
            if (slot.prefix_bloom)
                e = launch_bloom_prefix(slot.key_bytes, slot.key_off, batches[i].prefix_len, slot.n, p->bloom_bits_per_key,
                                        p->prefix_kind, p->prefix_arg, p->no_whole_key ? 0 : 1, slot.bloom_out,
                                        outs[i].bloom_cap, (uint64_t *)a.bloom_len_dev, (void *)a.bq.count, s);
            else
                e = launch_bloom_build(slot.key_bytes, slot.key_off, slot.n, slot.num_probes, slot.bloom_out, slot.bloom_len,
                                       (void *)a.bq.count, s);
            if (e != hipSuccess) return SDB_DEVICE_ERROR;
            stage_mark(s, kStBloom, false);
        }
        if (!slot.n) {  // empty SST: summary only (a filter of an empty SST has no bytes)
            SstSet one = set_header(p);
            one.count = 1;
            one.s[0] = slot;
            if (launch_encode_empty(make_args(one, 0), s) != hipSuccess) return SDB_DEVICE_ERROR;
            continue;
        }
        P.s[P.count++] = slot;
        P.max_facts = std::max(P.max_facts, slot.nfacts);
        P.max_chunks = std::max(P.max_chunks, slot.nchunks);
        P.max_groups = std::max(P.max_groups, (slot.nchunks + slot.group - 1) / slot.group);
        if (slot.bloom_fused) {
            P.max_tiles = std::max(P.max_tiles, slot.bpl.tiles);
            P.max_slices = std::max(P.max_slices, slot.bpl.nslices);
            bin_lds = std::max(bin_lds, bloom_bin_lds(slot.bpl));
            fill_lds = std::max(fill_lds, bloom_fill_lds(slot.bpl));
        }
        if (P.count == kMaxSsts && !flush()) return SDB_DEVICE_ERROR;
    }
    if (P.count && !flush()) return SDB_DEVICE_ERROR;
    return SDB_OK;
}

uint64_t sdb_bloom_workspace_bytes(uint64_t n, uint32_t bits_per_key) {
    return bloom_workspace_bytes(n, num_probes_for(bits_per_key), filter_bytes_for(n, bits_per_key)) + 256;
}

sdb_status sdb_encode_sst(const sdb_kv_batch *b, const sdb_sst_params *p, const sdb_sst_out *out,
                          void *workspace, uint64_t workspace_bytes, void *stream) {
    if (!b || !out) return SDB_INVALID_ARGUMENT;
    return sdb_encode_ssts(1, b, p, out, workspace, workspace_bytes, stream);
}

sdb_status sdb_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                           uint32_t bits_per_key, uint8_t *bitmap, uint64_t bitmap_bytes, void *workspace,
                           uint64_t workspace_bytes, void *stream) {
    if (!device_ok()) return SDB_DEVICE_ERROR;
    uint64_t fb = filter_bytes_for(n, bits_per_key);
    if (bitmap_bytes < fb || (fb && !bitmap) || (n && (!key_bytes || !key_off))) return SDB_INVALID_ARGUMENT;
    // the build writes 32-bit words: a 4-byte aligned bitmap, and (atomic path, no workspace) room for
    // the word that holds the last byte
    if (((uintptr_t)bitmap & 3) || (!workspace && fb && bitmap_bytes < ((fb + 3) & ~3ull))) return SDB_INVALID_ARGUMENT;
    if (workspace && workspace_bytes < sdb_bloom_workspace_bytes(n, bits_per_key)) return SDB_INVALID_ARGUMENT;
    if (launch_bloom_build(key_bytes, key_off, n, num_probes_for(bits_per_key), bitmap, fb, workspace, S(stream)) != hipSuccess)
        return SDB_DEVICE_ERROR;
    return SDB_OK;
}

uint64_t sdb_bloom_prefix_workspace_bytes(uint64_t n) { return prefix_workspace_bytes(n) + 256; }

sdb_status sdb_bloom_build_prefix(const uint8_t *key_bytes, const uint64_t *key_off, const int32_t *prefix_len,
                                  uint64_t n, uint32_t bits_per_key, uint32_t prefix_kind, uint32_t prefix_arg,
                                  uint32_t whole_key, uint8_t *bitmap, uint64_t bitmap_cap, uint64_t *bloom_len,
                                  void *workspace, uint64_t workspace_bytes, void *stream) {
    if (!device_ok()) return SDB_DEVICE_ERROR;
    if (prefix_kind > SDB_PREFIX_LENGTHS || (prefix_kind == SDB_PREFIX_NONE && !whole_key) || !bloom_len ||
        (n && (!key_bytes || !key_off)) || (prefix_kind == SDB_PREFIX_LENGTHS && n && !prefix_len) ||
        (prefix_kind == SDB_PREFIX_DELIM && prefix_arg > 255) || !bitmap || ((uintptr_t)bitmap & 3) ||
        !workspace || workspace_bytes < sdb_bloom_prefix_workspace_bytes(n))
        return SDB_INVALID_ARGUMENT;
    if (launch_bloom_prefix(key_bytes, key_off, prefix_len, n, bits_per_key, prefix_kind, prefix_arg, whole_key ? 1 : 0,
                            bitmap, bitmap_cap, bloom_len, workspace, S(stream)) != hipSuccess)
        return SDB_DEVICE_ERROR;
    return SDB_OK;
}

sdb_status sdb_bloom_might_match(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes, uint32_t whole_key,
                                 uint32_t prefix_kind, uint32_t prefix_arg, const uint8_t *key_bytes,
                                 const uint64_t *key_off, const uint8_t *is_prefix, const int32_t *query_prefix_len,
                                 uint64_t n, uint8_t *result, void *stream) {
    if (!device_ok()) return SDB_DEVICE_ERROR;
    if (prefix_kind > SDB_PREFIX_LENGTHS || (n && (!key_bytes || !key_off || !result)) ||
        (prefix_kind == SDB_PREFIX_LENGTHS && n && !query_prefix_len) || (bitmap_bytes && !bitmap))
        return SDB_INVALID_ARGUMENT;
    if (launch_bloom_match(bitmap, bitmap_bytes, num_probes, whole_key ? 1 : 0, prefix_kind, prefix_arg, key_bytes, key_off,
                           is_prefix, query_prefix_len, n, result, S(stream)) != hipSuccess)
        return SDB_DEVICE_ERROR;
    return SDB_OK;
}

sdb_status sdb_bloom_might_contain(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes,
                                   const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                                   uint8_t *result, void *stream) {
    if (!device_ok()) return SDB_DEVICE_ERROR;
    if (n && (!key_bytes || !key_off || !result)) return SDB_INVALID_ARGUMENT;
    if (launch_bloom_query(bitmap, bitmap_bytes, num_probes, key_bytes, key_off, n, result, S(stream)) != hipSuccess)
        return SDB_DEVICE_ERROR;
    return SDB_OK;
}

uint64_t sdb_decode_workspace_bytes(uint64_t nblocks) { return decode_workspace_layout(nblocks).total; }

static sdb_status decode_common(const uint8_t *blocks, const uint64_t *block_off, const uint64_t *block_end,
                                uint64_t nblocks, uint16_t sst_version, const sdb_decoded_out *out, void *workspace,
                                uint64_t workspace_bytes, void *stream, uint32_t flags = 0) {
    if (!out || !out->summary || !out->block_entry_start) return SDB_INVALID_ARGUMENT;
    if (sst_version != 1 && sst_version != 2) return SDB_INVALID_VERSION;  // block_iterator.rs:60-77
    if (nblocks && (!blocks || !block_off)) return SDB_INVALID_ARGUMENT;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    DecodeWorkspace wl = decode_workspace_layout(nblocks);
    if (!workspace || workspace_bytes < wl.total) return SDB_INVALID_ARGUMENT;
    DecodeArgs a{};
    a.blocks = blocks;
    a.block_off = block_off;
    a.block_end = block_end;
    a.nblocks = nblocks;
    a.version = sst_version;
    a.descending = (flags & SDB_DECODE_DESCENDING) ? 1u : 0u;
    a.fail_fast = (flags & SDB_DECODE_FAIL_FAST) ? 1u : 0u;
    a.out = *out;
    a.cnt = carve<uint64_t>(workspace, wl.cnt);
    a.kbytes = carve<uint64_t>(workspace, wl.kbytes);
    a.flag = carve<uint8_t>(workspace, wl.flag);
    a.rcnt = carve<uint64_t>(workspace, wl.rcnt);
    a.rowpos = carve<uint16_t>(workspace, wl.rowpos);
    a.ent_start = carve<uint64_t>(workspace, wl.ent_start);
    a.key_start = carve<uint64_t>(workspace, wl.key_start);
    a.tile_x = carve<uint64_t>(workspace, wl.tile_x);
    a.tile_y = carve<uint64_t>(workspace, wl.tile_y);
    a.err = carve<unsigned long long>(workspace, wl.err);
    a.nbad = carve<unsigned long long>(workspace, wl.nbad);
    a.done = carve<uint32_t>(workspace, wl.done);
    a.bad_block = out->bad_block;
    a.bad_cap = out->bad_cap;
    if (launch_decode(a, S(stream)) != hipSuccess) return SDB_DEVICE_ERROR;
    return SDB_OK;
}

sdb_status sdb_decode_blocks(const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                             uint16_t sst_version, const sdb_decoded_out *out, void *workspace,
                             uint64_t workspace_bytes, void *stream) {
    return decode_common(blocks, block_off, nullptr, nblocks, sst_version, out, workspace, workspace_bytes, stream);
}

sdb_status sdb_decode_blocks_ex(const uint8_t *arena, const uint64_t *block_start, const uint64_t *block_end,
                                uint64_t nblocks, uint16_t sst_version, uint32_t flags, const sdb_decoded_out *out,
                                void *workspace, uint64_t workspace_bytes, void *stream) {
    if (flags & ~(uint32_t)(SDB_DECODE_DESCENDING | SDB_DECODE_FAIL_FAST)) return SDB_INVALID_ARGUMENT;
    if (block_end && nblocks && !block_start) return SDB_INVALID_ARGUMENT;
    return decode_common(arena, block_start, block_end, nblocks, sst_version, out, workspace, workspace_bytes, stream,
                         flags);
}

sdb_status sdb_decode_blocks_at(const uint8_t *arena, const uint64_t *block_start, const uint64_t *block_end,
                                uint64_t nblocks, uint16_t sst_version, const sdb_decoded_out *out,
                                void *workspace, uint64_t workspace_bytes, void *stream) {
    if (nblocks && !block_end) return SDB_INVALID_ARGUMENT;
    return decode_common(arena, block_start, block_end, nblocks, sst_version, out, workspace, workspace_bytes, stream);
}

uint64_t sdb_decompress_workspace_bytes(uint64_t nblocks) { return decompress_workspace_bytes(nblocks); }

static bool lz_codec(uint32_t codec) {  // every compressing codec of CompressionCodec (format/sst.rs:884-917)
    return codec == SDB_CODEC_LZ4 || codec == SDB_CODEC_SNAPPY || codec == SDB_CODEC_ZLIB || codec == SDB_CODEC_ZSTD;
}

sdb_status sdb_decompress_plan(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                               uint64_t *out_start, void *workspace, uint64_t workspace_bytes, void *stream) {
    if (!lz_codec(codec)) return SDB_INVALID_ARGUMENT;
    if (!out_start || (nblocks && (!blocks || !block_off))) return SDB_INVALID_ARGUMENT;
    if (!workspace || workspace_bytes < decompress_workspace_bytes(nblocks)) return SDB_INVALID_ARGUMENT;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    return launch_decompress_plan(codec, blocks, block_off, nblocks, out_start, workspace, S(stream)) == hipSuccess
               ? SDB_OK : SDB_DEVICE_ERROR;
}

sdb_status sdb_decompress_blocks(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                 uint8_t *out, uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end,
                                 uint64_t *err, void *stream) {
    if (!lz_codec(codec)) return SDB_INVALID_ARGUMENT;
    if (!err || !out_start || (nblocks && (!blocks || !block_off || !out_end || (out_cap && !out)))) return SDB_INVALID_ARGUMENT;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    return launch_decompress_run(codec, blocks, block_off, nblocks, out, out_cap, out_start, out_end,
                                 (unsigned long long *)err, S(stream)) == hipSuccess ? SDB_OK : SDB_DEVICE_ERROR;
}

uint64_t sdb_decompress_once_workspace_bytes(uint64_t nblocks) { return decompress_once_workspace_bytes(nblocks); }

sdb_status sdb_decompress_blocks_once(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                      uint64_t slot_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_start,
                                      uint64_t *out_end, uint64_t *err, void *workspace, uint64_t workspace_bytes,
                                      void *stream) {
    if (!lz_codec(codec)) return SDB_INVALID_ARGUMENT;
    if (!err || !out_start || (nblocks && (!blocks || !block_off || !out_end || (out_cap && !out)))) return SDB_INVALID_ARGUMENT;
    if (!workspace || workspace_bytes < decompress_once_workspace_bytes(nblocks)) return SDB_INVALID_ARGUMENT;
    if (codec == SDB_CODEC_ZLIB && (slot_bytes < 8 || slot_bytes > (1ull << 32) ||
                                    (nblocks && out_cap / nblocks < slot_bytes)))
        return SDB_INVALID_ARGUMENT;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    return launch_decompress_once(codec, blocks, block_off, nblocks, slot_bytes, out, out_cap, out_start, out_end,
                                  (unsigned long long *)err, workspace, S(stream)) == hipSuccess ? SDB_OK
                                                                                                 : SDB_DEVICE_ERROR;
}

uint64_t sdb_compress_workspace_bytes(uint64_t nblocks, uint64_t in_bytes) {
    return compress_workspace_bytes(nblocks, in_bytes) + 256;
}

sdb_status sdb_compress_blocks(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                               uint64_t in_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *err,
                               void *workspace, uint64_t workspace_bytes, void *stream) {
    if (!lz_codec(codec)) return SDB_INVALID_ARGUMENT;
    if (!out_off || !err || (nblocks && (!blocks || !block_off || (out_cap && !out)))) return SDB_INVALID_ARGUMENT;
    if (!workspace || workspace_bytes < sdb_compress_workspace_bytes(nblocks, in_bytes)) return SDB_INVALID_ARGUMENT;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    return launch_compress(codec, blocks, block_off, nblocks, in_bytes, out, out_cap, out_off,
                           (unsigned long long *)err, workspace, S(stream)) == hipSuccess ? SDB_OK : SDB_DEVICE_ERROR;
}

uint64_t sdb_merge_runs_workspace_bytes(const sdb_run *runs, uint32_t nruns) {
    if (nruns && !runs) return 0;
    uint64_t total = 0;
    for (uint32_t r = 0; r < nruns; r++) total += runs[r].n;
    return merge_workspace_layout(total).total + 256;
}

sdb_status sdb_merge_runs(const sdb_run *runs, uint32_t nruns, const sdb_retention *ret, const sdb_merged_out *out,
                          void *workspace, uint64_t workspace_bytes, void *stream) {
    MergeArgs a;
    sdb_status st = build_merge_args(runs, nruns, ret, out, workspace, workspace_bytes, &a);
    if (st) return st;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    if (launch_merge(a, true, S(stream)) != hipSuccess) return SDB_DEVICE_ERROR;
    return SDB_OK;
}

uint64_t sdb_sst_cuts_workspace_bytes(uint64_t n, const sdb_sst_params *params) {
    if (!params) return 0;
    sdb_sst_params p = *params;
    p.bloom_bits_per_key = 0;
    p.prefix_kind = SDB_PREFIX_NONE;
    p.no_whole_key = 0;
    return sst_ws_bytes(n, &p) + 512 + 256;
}

sdb_status sdb_sst_cuts(const sdb_kv_batch *batch, const sdb_sst_params *params, uint64_t max_sst_size,
                        uint64_t *cut_start, uint64_t cut_cap, uint64_t *num_ssts, void *workspace,
                        uint64_t workspace_bytes, void *stream) {
    return sst_cuts_padded(batch, params, max_sst_size, cut_start, cut_cap, num_ssts, workspace, workspace_bytes,
                           S(stream), nullptr);
}

}  // extern "C"

namespace sdb {
sdb_status sst_cuts_padded(const sdb_kv_batch *batch, const sdb_sst_params *params, uint64_t max_sst_size,
                           uint64_t *cut_start, uint64_t cut_cap, uint64_t *num_ssts, void *workspace,
                           uint64_t workspace_bytes, hipStream_t s, const uint64_t *n_real) {
    if (!batch || !params || !cut_start || !num_ssts) return SDB_INVALID_ARGUMENT;
    sdb_sst_params p = *params;  // the chain only: no filter
    p.bloom_bits_per_key = 0;
    p.prefix_kind = SDB_PREFIX_NONE;
    p.no_whole_key = 0;
    sdb_status st = check_params(&p);
    if (st) return st;
    const uint64_t n = batch->n;
    if (n >= (1ull << 31)) return SDB_LIMIT_EXCEEDED;
    if (cut_cap < n + 1 || (n && (!batch->key_bytes || !batch->key_off || !batch->val_off))) return SDB_INVALID_ARGUMENT;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    if (!workspace || workspace_bytes < sdb_sst_cuts_workspace_bytes(n, params)) return SDB_INVALID_ARGUMENT;
    uint8_t *ws = (uint8_t *)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    if (!n) {
        if (hipMemsetAsync(cut_start, 0, 8, s) != hipSuccess || hipMemsetAsync(num_ssts, 0, 8, s) != hipSuccess)
            return SDB_DEVICE_ERROR;
        return SDB_OK;
    }
    // the prep kernels write an SST summary: a scratch one after the encode workspace
    sdb_sst_summary *scratch = (sdb_sst_summary *)(ws + sst_ws_bytes(n, &p));
    sdb_sst_out out{};
    out.data_cap = ~0ull;
    out.block_cap = ~0ull;
    out.summary = scratch;
    bool standalone = false;
    SstSet P = set_header(&p);
    P.s[0] = plan_slot(batch, &p, &out, ws, &standalone);
    P.count = 1;
    P.max_facts = P.s[0].nfacts;
    P.max_chunks = P.s[0].nchunks;
    P.max_groups = (P.s[0].nchunks + P.s[0].group - 1) / P.s[0].group;
    if (launch_cuts(P, max_sst_size, cut_start, cut_cap, num_ssts, s, n_real) != hipSuccess) return SDB_DEVICE_ERROR;
    return SDB_OK;
}
}  // namespace sdb

extern "C" {

uint64_t sdb_sst_lookup_workspace_bytes(uint64_t num_blocks, uint64_t nkeys) {
    return lookup_workspace_bytes(num_blocks, nkeys) + 256;
}

sdb_status sdb_sst_lookup(const sdb_sst_view *sst, const uint8_t *key_bytes, const uint64_t *key_off,
                          uint64_t nkeys, int32_t descending, const sdb_lookup_out *out, void *workspace,
                          uint64_t workspace_bytes, void *stream) {
    if (!sst || !out) return SDB_INVALID_ARGUMENT;
    if (sst->sst_version != 1 && sst->sst_version != 2) return SDB_INVALID_VERSION;
    if (sst->num_blocks >= 0xFFFFFFFFull) return SDB_LIMIT_EXCEEDED;
    if (sst->num_blocks && (!sst->data || !sst->block_off || !sst->index_keys || !sst->index_key_off))
        return SDB_INVALID_ARGUMENT;
    if (nkeys && (!key_bytes || !key_off || !out->state || !out->status || !out->block || !out->entry ||
                  !out->key_len || !out->val_off || !out->val_len || !out->seq || !out->flags || !out->create_ts ||
                  !out->expire_ts))
        return SDB_INVALID_ARGUMENT;
    if (!device_ok()) return SDB_DEVICE_ERROR;
    if (!workspace || workspace_bytes < sdb_sst_lookup_workspace_bytes(sst->num_blocks, nkeys)) return SDB_INVALID_ARGUMENT;
    uint8_t *w = (uint8_t *)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    LookupArgs a{};
    a.v = *sst;
    a.key_bytes = key_bytes;
    a.key_off = key_off;
    a.nkeys = nkeys;
    a.desc = descending ? 1 : 0;
    a.out = *out;
    a.qrange = (uint32_t *)w;
    w += (8 * (nkeys + 1) + 255) & ~255ull;
    a.mark = w;
    w += (sst->num_blocks + 256) & ~255ull;
    a.bstat = (int32_t *)w;
    if (launch_lookup(a, S(stream)) != hipSuccess) return SDB_DEVICE_ERROR;
    return SDB_OK;
}

}  // extern "C"

// =================================================================================================
// Stage timing (diagnostics)
// =================================================================================================
#include <mutex>
namespace sdb {
namespace {
std::mutex g_diag_mu;
bool g_diag_on = false;
struct StageRec {
    int stage;
    hipEvent_t a, b;
};
std::vector<StageRec> g_recs;
std::vector<hipEvent_t> g_open(kNumStages, nullptr);
uint64_t g_launches = 0;
}  // namespace
bool stage_timing_on() { return g_diag_on; }
void stage_mark(hipStream_t st, int stage, bool begin) {
    if (!g_diag_on) return;
    std::lock_guard<std::mutex> lk(g_diag_mu);
    hipEvent_t e;
    hipEventCreate(&e);
    hipEventRecord(e, st);
    if (begin) {
        g_open[stage] = e;
        if (stage == kStFacts) g_launches++;
    } else {
        g_recs.push_back({stage, g_open[stage], e});
        g_open[stage] = nullptr;
    }
}
}  // namespace sdb

extern "C" {
void sdb_diag_enable_stage_timing(int on) {
    std::lock_guard<std::mutex> lk(g_diag_mu);
    g_diag_on = on != 0;
}
int sdb_diag_stage_times(double *ms, int max_stages, uint64_t *launches) {
    std::lock_guard<std::mutex> lk(g_diag_mu);
    std::vector<double> acc(kNumStages, 0.0);
    for (auto &r : g_recs) {
        hipEventSynchronize(r.b);
        float t = 0;
        hipEventElapsedTime(&t, r.a, r.b);
        acc[r.stage] += t;
        hipEventDestroy(r.a);
        hipEventDestroy(r.b);
    }
    g_recs.clear();
    for (int i = 0; i < max_stages && i < kNumStages; i++) ms[i] = acc[i];
    if (launches) *launches = g_launches;
    g_launches = 0;
    return kNumStages;
}
}  // extern "C"

// =================================================================================================
// Host-buffer runtime
// =================================================================================================
namespace {

struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) hipFree(p);
        p = nullptr;
        cap = 0;
        uint64_t want = std::max<uint64_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipMalloc(&p, want);
        if (e == hipSuccess) cap = want;
        return e;
    }
    DevBuf() = default;
    DevBuf(const DevBuf &) = delete;
    DevBuf &operator=(const DevBuf &) = delete;
    DevBuf(DevBuf &&o) noexcept : p(o.p), cap(o.cap) {
        o.p = nullptr;
        o.cap = 0;
    }
    DevBuf &operator=(DevBuf &&o) noexcept {
        if (this != &o) {
            if (p) hipFree(p);
            p = o.p;
            cap = o.cap;
            o.p = nullptr;
            o.cap = 0;
        }
        return *this;
    }
    ~DevBuf() {
        if (p) hipFree(p);
    }
};
struct PinBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    hipError_t ensure(uint64_t bytes) {
        if (bytes <= cap) return hipSuccess;
        if (p) hipHostFree(p);
        p = nullptr;
        cap = 0;
        uint64_t want = std::max<uint64_t>(bytes + bytes / 4, 4096);
        hipError_t e = hipHostMalloc(&p, want, hipHostMallocDefault);
        if (e == hipSuccess) cap = want;
        return e;
    }
    PinBuf() = default;
    PinBuf(const PinBuf &) = delete;
    PinBuf &operator=(const PinBuf &) = delete;
    PinBuf(PinBuf &&o) noexcept : p(o.p), cap(o.cap) {
        o.p = nullptr;
        o.cap = 0;
    }
    PinBuf &operator=(PinBuf &&o) noexcept {
        if (this != &o) {
            if (p) hipHostFree(p);
            p = o.p;
            cap = o.cap;
            o.p = nullptr;
            o.cap = 0;
        }
        return *this;
    }
    ~PinBuf() {
        if (p) hipHostFree(p);
    }
};

}  // namespace

// One in-flight SST of the pipelined host path (sdb_encoder_encode_host_many).
struct EncSlot {
    PinBuf h_in;
    DevBuf d_in, d_out, d_ws;
    hipEvent_t h2d_done = nullptr, comp_done = nullptr, d2h_done = nullptr;
    bool used = false;
};

struct sdb_encoder {
    int device = 0;
    sdb_sst_params params{};
    hipStream_t stream = nullptr;  // kernels (and the whole single-SST path)
    hipEvent_t ev[4] = {};
    // device: input, output, workspace
    DevBuf d_in, d_out, d_ws;
    PinBuf h_in, h_out;
    // pipelined path: H2D and D2H on their own streams (the two copy directions overlap each other
    // and the kernels), two slots of staging / device buffers, one pinned output area per SST
    hipStream_t s_h2d = nullptr, s_d2h = nullptr;
    EncSlot slot[2];
    std::vector<PinBuf> outs;
    PinBuf sums;
};

namespace {

struct InLayout {  // packed input arrays inside one allocation (256-byte aligned pieces)
    uint64_t key_bytes, key_off, val_bytes, val_off, kind, seq, cts, ets, mask, plen, total;
};
// Only the columns the batch has take space (and H2D bytes).
InLayout in_layout(const sdb_kv_batch *hb, uint64_t kb, uint64_t vb) {
    const uint64_t n = hb->n;
    InLayout l{};
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        uint64_t r = off;
        off += (bytes + 255) & ~255ull;
        return r;
    };
    l.key_bytes = take(kb + 16);
    l.key_off = take(8 * (n + 1));
    l.val_bytes = take(vb + 16);
    l.val_off = take(8 * (n + 1));
    l.kind = take(hb->kind ? n + 1 : 0);
    l.seq = take(hb->seq ? 8 * (n + 1) : 0);
    l.cts = take(hb->create_ts ? 8 * (n + 1) : 0);
    l.ets = take(hb->expire_ts ? 8 * (n + 1) : 0);
    l.mask = take(hb->ts_mask ? n + 1 : 0);
    l.plen = take(hb->prefix_len ? 4 * (n + 1) : 0);
    l.total = off;
    return l;
}

// The caller's (pageable) batch into pinned staging, offsets rebased to 0.  Large copies are split
// over a few host threads: one thread's memcpy bandwidth is below the PCIe rate.
void marshal(const sdb_kv_batch *hb, const InLayout &il, uint8_t *hi, uint64_t k0, uint64_t kb, uint64_t v0, uint64_t vb) {
    const uint64_t n = hb->n;
    if (!n) return;
    std::vector<std::pair<uint8_t *, const uint8_t *>> dst_src;
    std::vector<uint64_t> len;
    auto add = [&](uint8_t *d, const void *s, uint64_t l) {
        if (s && l) {
            dst_src.push_back({d, (const uint8_t *)s});
            len.push_back(l);
        }
    };
    add(hi + il.key_bytes, hb->key_bytes + k0, kb);
    add(hi + il.val_bytes, hb->val_bytes ? hb->val_bytes + v0 : nullptr, vb);
    add(hi + il.kind, hb->kind, n);
    add(hi + il.seq, hb->seq, 8 * n);
    add(hi + il.cts, hb->create_ts, 8 * n);
    add(hi + il.ets, hb->expire_ts, 8 * n);
    add(hi + il.mask, hb->ts_mask, n);
    add(hi + il.plen, hb->prefix_len, 4 * n);
    uint64_t total = 0;
    for (uint64_t l : len) total += l;
    const unsigned nt = total >= (16u << 20) ? 8 : 1;
    auto work = [&](unsigned t) {
        // byte range [t * total / nt, (t + 1) * total / nt) of the concatenated copies
        const uint64_t lo = total * t / nt, hi_ = total * (t + 1) / nt;
        uint64_t base = 0;
        for (size_t q = 0; q < len.size(); q++) {
            const uint64_t a = std::max(lo, base), b = std::min(hi_, base + len[q]);
            if (a < b) memcpy(dst_src[q].first + (a - base), dst_src[q].second + (a - base), b - a);
            base += len[q];
        }
        // and entries [t * (n + 1) / nt, ...) of the rebased offsets
        uint64_t *ko = (uint64_t *)(hi + il.key_off), *vo = (uint64_t *)(hi + il.val_off);
        const uint64_t e0 = (n + 1) * t / nt, e1 = (n + 1) * (t + 1) / nt;
        for (uint64_t i = e0; i < e1; i++) {
            ko[i] = hb->key_off[i] - k0;
            vo[i] = hb->val_off[i] - v0;
        }
    };
    if (nt == 1) {
        work(0);
        return;
    }
    std::vector<std::thread> th;
    for (unsigned t = 1; t < nt; t++) th.emplace_back(work, t);
    work(0);
    for (auto &x : th) x.join();
}

sdb_kv_batch dev_batch(const sdb_kv_batch *hb, const InLayout &il, uint8_t *di) {
    sdb_kv_batch db{};
    db.n = hb->n;
    db.key_bytes = di + il.key_bytes;
    db.key_off = (const uint64_t *)(di + il.key_off);
    db.val_bytes = di + il.val_bytes;
    db.val_off = (const uint64_t *)(di + il.val_off);
    db.kind = hb->kind ? di + il.kind : nullptr;
    db.seq = hb->seq ? (const uint64_t *)(di + il.seq) : nullptr;
    db.create_ts = hb->create_ts ? (const int64_t *)(di + il.cts) : nullptr;
    db.expire_ts = hb->expire_ts ? (const int64_t *)(di + il.ets) : nullptr;
    db.ts_mask = hb->ts_mask ? di + il.mask : nullptr;
    db.prefix_len = hb->prefix_len ? (const int32_t *)(di + il.plen) : nullptr;
    return db;
}
struct OutLayout {
    uint64_t data, block_off, block_first, index_key_len, block_stats, bloom, summary, total;
};
OutLayout out_layout(uint64_t data_cap, uint64_t block_cap, uint64_t bloom_cap) {
    OutLayout l{};
    uint64_t off = 0;
    auto take = [&](uint64_t bytes) {
        uint64_t r = off;
        off += (bytes + 255) & ~255ull;
        return r;
    };
    l.data = take(data_cap);
    l.block_off = take(8 * (block_cap + 1));
    l.block_first = take(4 * (block_cap + 1));
    l.index_key_len = take(4 * (block_cap + 1));
    l.block_stats = take(6 * (block_cap + 1));
    l.bloom = take(bloom_cap);
    l.summary = take(sizeof(sdb_sst_summary));
    l.total = off;
    return l;
}

}  // namespace

extern "C" {

sdb_encoder *sdb_encoder_create(int device, const sdb_sst_params *params) {
    if (check_params(params) || !device_ok()) return nullptr;
    if (hipSetDevice(device) != hipSuccess) return nullptr;
    sdb_encoder *e = new sdb_encoder();
    e->device = device;
    e->params = *params;
    if (hipStreamCreateWithFlags(&e->stream, hipStreamNonBlocking) != hipSuccess) {
        delete e;
        return nullptr;
    }
    for (auto &x : e->ev) hipEventCreate(&x);
    if (hipStreamCreateWithFlags(&e->s_h2d, hipStreamNonBlocking) != hipSuccess ||
        hipStreamCreateWithFlags(&e->s_d2h, hipStreamNonBlocking) != hipSuccess) {
        sdb_encoder_destroy(e);
        return nullptr;
    }
    for (EncSlot &sl : e->slot) {
        hipEventCreateWithFlags(&sl.h2d_done, hipEventDisableTiming);
        hipEventCreateWithFlags(&sl.comp_done, hipEventDisableTiming);
        hipEventCreateWithFlags(&sl.d2h_done, hipEventDisableTiming);
    }
    return e;
}

void sdb_encoder_destroy(sdb_encoder *e) {
    if (!e) return;
    hipSetDevice(e->device);
    for (hipStream_t st : {e->stream, e->s_h2d, e->s_d2h})
        if (st) hipStreamSynchronize(st);
    for (auto &x : e->ev) hipEventDestroy(x);
    for (EncSlot &sl : e->slot)
        for (hipEvent_t x : {sl.h2d_done, sl.comp_done, sl.d2h_done})
            if (x) hipEventDestroy(x);
    for (hipStream_t st : {e->stream, e->s_h2d, e->s_d2h})
        if (st) hipStreamDestroy(st);
    delete e;
}

sdb_status sdb_encoder_encode_host(sdb_encoder *e, const sdb_kv_batch *hb, sdb_sst_host_result *r) {
    if (!e || !hb || !r) return SDB_INVALID_ARGUMENT;
    hipSetDevice(e->device);
    const uint64_t n = hb->n;
    const uint64_t k0 = n ? hb->key_off[0] : 0, kb = n ? hb->key_off[n] - k0 : 0;
    const uint64_t v0 = n ? hb->val_off[0] : 0, vb = n ? hb->val_off[n] - v0 : 0;
    uint64_t data_cap, block_cap, bloom_cap;
    sdb_encode_bounds(n, kb, vb, &e->params, &data_cap, &block_cap, &bloom_cap);
    if (data_cap >= (1ull << 32)) return SDB_LIMIT_EXCEEDED;  // u32 per-block/chunk byte counters
    InLayout il = in_layout(hb, kb, vb);
    OutLayout ol = out_layout(data_cap, block_cap, bloom_cap);
    uint64_t wsb = sdb_encode_workspace_bytes(n, &e->params);
    if (e->h_in.ensure(il.total) || e->d_in.ensure(il.total) || e->h_out.ensure(ol.total) ||
        e->d_out.ensure(ol.total) || e->d_ws.ensure(wsb))
        return SDB_DEVICE_ERROR;
    uint8_t *hi = (uint8_t *)e->h_in.p;
    marshal(hb, il, hi, k0, kb, v0, vb);
    uint8_t *di = (uint8_t *)e->d_in.p, *dout = (uint8_t *)e->d_out.p;
    hipEventRecord(e->ev[0], e->stream);
    hipMemcpyAsync(di, hi, il.total, hipMemcpyHostToDevice, e->stream);
    hipEventRecord(e->ev[1], e->stream);
    const sdb_kv_batch db = dev_batch(hb, il, di);
    sdb_sst_out o{};
    o.data = dout + ol.data;
    o.data_cap = data_cap;
    o.block_off = (uint64_t *)(dout + ol.block_off);
    o.block_first_entry = (uint32_t *)(dout + ol.block_first);
    o.index_key_len = (uint32_t *)(dout + ol.index_key_len);
    o.block_stats = (uint16_t *)(dout + ol.block_stats);
    o.block_cap = block_cap;
    o.bloom = dout + ol.bloom;
    o.bloom_cap = bloom_cap;
    o.summary = (sdb_sst_summary *)(dout + ol.summary);
    sdb_status st = sdb_encode_sst(&db, &e->params, &o, e->d_ws.p, e->d_ws.cap, e->stream);
    if (st) return st;
    hipEventRecord(e->ev[2], e->stream);
    // D2H: summary first (sizes), then only the used parts
    uint8_t *ho = (uint8_t *)e->h_out.p;
    hipMemcpyAsync(ho + ol.summary, dout + ol.summary, sizeof(sdb_sst_summary), hipMemcpyDeviceToHost, e->stream);
    if (hipStreamSynchronize(e->stream) != hipSuccess) return SDB_DEVICE_ERROR;
    sdb_sst_summary sm;
    memcpy(&sm, ho + ol.summary, sizeof sm);
    if (sm.status == SDB_OK) {
        uint64_t nb = sm.num_blocks;
        hipMemcpyAsync(ho + ol.data, dout + ol.data, sm.data_len, hipMemcpyDeviceToHost, e->stream);
        hipMemcpyAsync(ho + ol.block_off, dout + ol.block_off, 8 * (nb + 1), hipMemcpyDeviceToHost, e->stream);
        hipMemcpyAsync(ho + ol.block_first, dout + ol.block_first, 4 * (nb + 1), hipMemcpyDeviceToHost, e->stream);
        hipMemcpyAsync(ho + ol.index_key_len, dout + ol.index_key_len, 4 * nb, hipMemcpyDeviceToHost, e->stream);
        hipMemcpyAsync(ho + ol.block_stats, dout + ol.block_stats, 6 * nb, hipMemcpyDeviceToHost, e->stream);
        if (sm.bloom_len)
            hipMemcpyAsync(ho + ol.bloom, dout + ol.bloom, sm.bloom_len, hipMemcpyDeviceToHost, e->stream);
    }
    hipEventRecord(e->ev[3], e->stream);
    if (hipStreamSynchronize(e->stream) != hipSuccess) return SDB_DEVICE_ERROR;
    float t01 = 0, t12 = 0, t23 = 0;
    hipEventElapsedTime(&t01, e->ev[0], e->ev[1]);
    hipEventElapsedTime(&t12, e->ev[1], e->ev[2]);
    hipEventElapsedTime(&t23, e->ev[2], e->ev[3]);
    r->summary = sm;
    r->data = ho + ol.data;
    r->block_off = (const uint64_t *)(ho + ol.block_off);
    r->block_first_entry = (const uint32_t *)(ho + ol.block_first);
    r->index_key_len = (const uint32_t *)(ho + ol.index_key_len);
    r->block_stats = (const uint16_t *)(ho + ol.block_stats);
    r->bloom = ho + ol.bloom;
    r->h2d_ms = t01;
    r->kernel_ms = t12;
    r->d2h_ms = t23;
    return (sdb_status)sm.status;
}

// Several host batches, transfers overlapped: while SST i's kernels run, SST i+1 is marshalled
// into the other slot's pinned staging and copied H2D, and SST i-1's outputs come back D2H (three
// streams; the copy engines serve both directions at once).  The host waits only for each SST's
// summary (to size its D2H) and for the last D2H.
sdb_status sdb_encoder_encode_host_many(sdb_encoder *e, uint32_t count, const sdb_kv_batch *hbs,
                                        sdb_sst_host_result *results) {
    if (!e || (count && (!hbs || !results))) return SDB_INVALID_ARGUMENT;
    if (hipSetDevice(e->device) != hipSuccess) return SDB_DEVICE_ERROR;
    if (e->outs.size() < count) e->outs.resize(count);
    if (e->sums.ensure(sizeof(sdb_sst_summary) * (count + 1))) return SDB_DEVICE_ERROR;
    sdb_sst_summary *sums = (sdb_sst_summary *)e->sums.p;
    struct Job {
        InLayout il;
        OutLayout ol;
        uint64_t data_cap, block_cap, bloom_cap;
    };
    std::vector<Job> jobs(count);
    sdb_status first = SDB_OK;
    auto fail = [&](sdb_status st) {
        for (hipStream_t x : {e->s_h2d, e->stream, e->s_d2h}) hipStreamSynchronize(x);
        return st;
    };
    for (uint32_t i = 0; i <= count; i++) {
        if (i < count) {
            const sdb_kv_batch *hb = &hbs[i];
            EncSlot &sl = e->slot[i & 1];
            Job &jb = jobs[i];
            const uint64_t n = hb->n;
            const uint64_t k0 = n ? hb->key_off[0] : 0, kb = n ? hb->key_off[n] - k0 : 0;
            const uint64_t v0 = n ? hb->val_off[0] : 0, vb = n ? hb->val_off[n] - v0 : 0;
            if (sdb_encode_bounds(n, kb, vb, &e->params, &jb.data_cap, &jb.block_cap, &jb.bloom_cap)) return fail(SDB_INVALID_ARGUMENT);
            if (jb.data_cap >= (1ull << 32)) return fail(SDB_LIMIT_EXCEEDED);
            jb.il = in_layout(hb, kb, vb);
            jb.ol = out_layout(jb.data_cap, jb.block_cap, jb.bloom_cap);
            const uint64_t wsb = sdb_encode_workspace_bytes(n, &e->params);
            // the slot's previous SST (i - 2) must be out of its staging (H2D) before the marshal
            // overwrites it; buffers only grow after every use of the slot has drained
            if (sl.used) hipEventSynchronize(sl.h2d_done);
            const bool grow = sl.h_in.cap < jb.il.total || sl.d_in.cap < jb.il.total || sl.d_out.cap < jb.ol.total ||
                              sl.d_ws.cap < wsb;
            if (grow && sl.used) {
                hipEventSynchronize(sl.comp_done);
                hipEventSynchronize(sl.d2h_done);
            }
            if (sl.h_in.ensure(jb.il.total) || sl.d_in.ensure(jb.il.total) || sl.d_out.ensure(jb.ol.total) ||
                sl.d_ws.ensure(wsb))
                return fail(SDB_DEVICE_ERROR);
            marshal(hb, jb.il, (uint8_t *)sl.h_in.p, k0, kb, v0, vb);
            // H2D once the slot's previous kernels no longer read d_in
            if (sl.used) hipStreamWaitEvent(e->s_h2d, sl.comp_done, 0);
            hipMemcpyAsync(sl.d_in.p, sl.h_in.p, jb.il.total, hipMemcpyHostToDevice, e->s_h2d);
            hipEventRecord(sl.h2d_done, e->s_h2d);
            // kernels once the input is there and the slot's previous outputs are back on the host
            hipStreamWaitEvent(e->stream, sl.h2d_done, 0);
            if (sl.used) hipStreamWaitEvent(e->stream, sl.d2h_done, 0);
            const sdb_kv_batch db = dev_batch(hb, jb.il, (uint8_t *)sl.d_in.p);
            uint8_t *dout = (uint8_t *)sl.d_out.p;
            sdb_sst_out o{};
            o.data = dout + jb.ol.data;
            o.data_cap = jb.data_cap;
            o.block_off = (uint64_t *)(dout + jb.ol.block_off);
            o.block_first_entry = (uint32_t *)(dout + jb.ol.block_first);
            o.index_key_len = (uint32_t *)(dout + jb.ol.index_key_len);
            o.block_stats = (uint16_t *)(dout + jb.ol.block_stats);
            o.block_cap = jb.block_cap;
            o.bloom = dout + jb.ol.bloom;
            o.bloom_cap = jb.bloom_cap;
            o.summary = (sdb_sst_summary *)(dout + jb.ol.summary);
            const sdb_status st = sdb_encode_sst(&db, &e->params, &o, sl.d_ws.p, sl.d_ws.cap, e->stream);
            if (st) return fail(st);
            hipMemcpyAsync(&sums[i], o.summary, sizeof(sdb_sst_summary), hipMemcpyDeviceToHost, e->stream);
            hipEventRecord(sl.comp_done, e->stream);
            sl.used = true;
        }
        if (i >= 1) {  // SST j's outputs: sized by its summary, copied on the D2H stream
            const uint32_t j = i - 1;
            EncSlot &sl = e->slot[j & 1];
            const Job &jb = jobs[j];
            if (hipEventSynchronize(sl.comp_done) != hipSuccess) return fail(SDB_DEVICE_ERROR);
            const sdb_sst_summary sm = sums[j];
            PinBuf &ho = e->outs[j];
            if (ho.ensure(jb.ol.total)) return fail(SDB_DEVICE_ERROR);
            uint8_t *h = (uint8_t *)ho.p, *d = (uint8_t *)sl.d_out.p;
            hipStreamWaitEvent(e->s_d2h, sl.comp_done, 0);
            if (sm.status == SDB_OK) {
                const uint64_t nb = sm.num_blocks;
                hipMemcpyAsync(h + jb.ol.data, d + jb.ol.data, sm.data_len, hipMemcpyDeviceToHost, e->s_d2h);
                hipMemcpyAsync(h + jb.ol.block_off, d + jb.ol.block_off, 8 * (nb + 1), hipMemcpyDeviceToHost, e->s_d2h);
                hipMemcpyAsync(h + jb.ol.block_first, d + jb.ol.block_first, 4 * (nb + 1), hipMemcpyDeviceToHost, e->s_d2h);
                hipMemcpyAsync(h + jb.ol.index_key_len, d + jb.ol.index_key_len, 4 * nb, hipMemcpyDeviceToHost, e->s_d2h);
                hipMemcpyAsync(h + jb.ol.block_stats, d + jb.ol.block_stats, 6 * nb, hipMemcpyDeviceToHost, e->s_d2h);
                if (sm.bloom_len)
                    hipMemcpyAsync(h + jb.ol.bloom, d + jb.ol.bloom, sm.bloom_len, hipMemcpyDeviceToHost, e->s_d2h);
            }
            hipEventRecord(sl.d2h_done, e->s_d2h);
            sdb_sst_host_result &r = results[j];
            r.summary = sm;
            r.data = h + jb.ol.data;
            r.block_off = (const uint64_t *)(h + jb.ol.block_off);
            r.block_first_entry = (const uint32_t *)(h + jb.ol.block_first);
            r.index_key_len = (const uint32_t *)(h + jb.ol.index_key_len);
            r.block_stats = (const uint16_t *)(h + jb.ol.block_stats);
            r.bloom = h + jb.ol.bloom;
            r.h2d_ms = r.kernel_ms = r.d2h_ms = 0;
            if (!first && sm.status) first = (sdb_status)sm.status;
        }
    }
    if (hipStreamSynchronize(e->s_d2h) != hipSuccess) return SDB_DEVICE_ERROR;
    return first;
}

}  // extern "C"

// -------------------------------------------------------------------------------------------------
// EncodedSsTableBuilder mirror
// -------------------------------------------------------------------------------------------------
struct sdb_sst_builder {
    sdb_encoder *enc = nullptr;
    std::vector<uint8_t> keys, vals, kind, mask;
    std::vector<uint64_t> koff{0}, voff{0}, seq;
    std::vector<int64_t> cts, ets;
};

extern "C" {

sdb_sst_builder *sdb_sst_builder_new(int device, const sdb_sst_params *params) {
    sdb_encoder *e = sdb_encoder_create(device, params);
    if (!e) return nullptr;
    sdb_sst_builder *b = new sdb_sst_builder();
    b->enc = e;
    return b;
}

void sdb_sst_builder_free(sdb_sst_builder *b) {
    if (!b) return;
    sdb_encoder_destroy(b->enc);
    delete b;
}

sdb_status sdb_sst_builder_add(sdb_sst_builder *b, const uint8_t *key, uint64_t key_len, uint8_t kind,
                               const uint8_t *val, uint64_t val_len, uint64_t seq, int32_t has_create_ts,
                               int64_t create_ts, int32_t has_expire_ts, int64_t expire_ts) {
    if (!b || kind > SDB_KIND_TOMBSTONE) return SDB_INVALID_ARGUMENT;
    b->keys.insert(b->keys.end(), key, key + key_len);
    if (kind != SDB_KIND_TOMBSTONE && val_len) b->vals.insert(b->vals.end(), val, val + val_len);
    b->koff.push_back(b->keys.size());
    b->voff.push_back(b->vals.size());
    b->kind.push_back(kind);
    b->seq.push_back(seq);
    b->cts.push_back(create_ts);
    b->ets.push_back(expire_ts);
    b->mask.push_back((uint8_t)((has_create_ts ? SDB_TS_CREATE : 0) | (has_expire_ts ? SDB_TS_EXPIRE : 0)));
    return SDB_OK;
}

sdb_status sdb_sst_builder_build(sdb_sst_builder *b, sdb_sst_host_result *r) {
    if (!b) return SDB_INVALID_ARGUMENT;
    sdb_kv_batch hb{};
    hb.n = b->kind.size();
    static const uint8_t zero16[16] = {0};
    hb.key_bytes = b->keys.empty() ? zero16 : b->keys.data();
    hb.key_off = b->koff.data();
    hb.val_bytes = b->vals.empty() ? zero16 : b->vals.data();
    hb.val_off = b->voff.data();
    hb.kind = b->kind.data();
    hb.seq = b->seq.data();
    hb.create_ts = b->cts.data();
    hb.expire_ts = b->ets.data();
    hb.ts_mask = b->mask.data();
    return sdb_encoder_encode_host(b->enc, &hb, r);
}

}  // extern "C"

// -------------------------------------------------------------------------------------------------
// Host decode
// -------------------------------------------------------------------------------------------------
struct sdb_decoder {
    int device = 0;
    hipStream_t stream = nullptr;
    DevBuf d_in, d_out, d_ws;
    PinBuf h_in, h_out;
};

extern "C" {

sdb_decoder *sdb_decoder_create(int device) {
    if (!device_ok() || hipSetDevice(device) != hipSuccess) return nullptr;
    sdb_decoder *d = new sdb_decoder();
    d->device = device;
    if (hipStreamCreateWithFlags(&d->stream, hipStreamNonBlocking) != hipSuccess) {
        delete d;
        return nullptr;
    }
    return d;
}

void sdb_decoder_destroy(sdb_decoder *d) {
    if (!d) return;
    hipSetDevice(d->device);
    hipStreamSynchronize(d->stream);
    hipStreamDestroy(d->stream);
    delete d;
}

sdb_status sdb_decoder_decode_host(sdb_decoder *d, const uint8_t *blocks, const uint64_t *block_off,
                                   uint64_t nblocks, uint16_t sst_version, sdb_decode_host_result *r) {
    if (!d || !r || (nblocks && (!blocks || !block_off))) return SDB_INVALID_ARGUMENT;
    hipSetDevice(d->device);
    const uint64_t b0 = nblocks ? block_off[0] : 0;
    const uint64_t total = nblocks ? block_off[nblocks] - b0 : 0;
    // capacities: every row >= 12 bytes; restored keys can exceed encoded bytes (shared prefixes),
    // bounded by rows x (64 KiB V0 keys) — use a generous first guess and retry once if too small.
    uint64_t cap_e = total / 12 + 16;
    uint64_t key_cap = total * 4 + 4096;
    for (int attempt = 0; attempt < 2; attempt++) {
        uint64_t off = 0;
        auto take = [&](uint64_t bytes) {
            uint64_t rr = off;
            off += (bytes + 255) & ~255ull;
            return rr;
        };
        uint64_t o_bes = take(8 * (nblocks + 1)), o_ka = take(key_cap), o_ko = take(8 * (cap_e + 1));
        uint64_t o_vo = take(8 * cap_e), o_vl = take(4 * cap_e), o_seq = take(8 * cap_e), o_fl = take(cap_e);
        uint64_t o_ct = take(8 * cap_e), o_et = take(8 * cap_e), o_bad = take(4 * (nblocks + 1));
        uint64_t o_sm = take(sizeof(sdb_decode_summary));
        uint64_t out_total = off;
        uint64_t in_total = ((total + 16 + 255) & ~255ull) + 8 * (nblocks + 1);
        uint64_t wsb = sdb_decode_workspace_bytes(nblocks);
        if (d->h_in.ensure(in_total) || d->d_in.ensure(in_total) || d->h_out.ensure(out_total) ||
            d->d_out.ensure(out_total) || d->d_ws.ensure(wsb))
            return SDB_DEVICE_ERROR;
        uint8_t *hi = (uint8_t *)d->h_in.p;
        uint64_t o_boff = (total + 16 + 255) & ~255ull;
        memcpy(hi, blocks + b0, total);
        uint64_t *bo = (uint64_t *)(hi + o_boff);
        for (uint64_t k = 0; k <= nblocks; k++) bo[k] = block_off[k] - b0;
        uint8_t *di = (uint8_t *)d->d_in.p, *dout = (uint8_t *)d->d_out.p;
        hipMemcpyAsync(di, hi, in_total, hipMemcpyHostToDevice, d->stream);
        sdb_decoded_out o{};
        o.block_entry_start = (uint64_t *)(dout + o_bes);
        o.key_arena = dout + o_ka;
        o.key_arena_cap = key_cap;
        o.key_off = (uint64_t *)(dout + o_ko);
        o.val_off = (uint64_t *)(dout + o_vo);
        o.val_len = (uint32_t *)(dout + o_vl);
        o.seq = (uint64_t *)(dout + o_seq);
        o.flags = dout + o_fl;
        o.create_ts = (int64_t *)(dout + o_ct);
        o.expire_ts = (int64_t *)(dout + o_et);
        o.cap_entries = cap_e;
        o.bad_block = (uint32_t *)(dout + o_bad);
        o.bad_cap = nblocks + 1;
        o.summary = (sdb_decode_summary *)(dout + o_sm);
        sdb_status st = sdb_decode_blocks(di, (const uint64_t *)(di + o_boff), nblocks, sst_version, &o, d->d_ws.p,
                                          d->d_ws.cap, d->stream);
        if (st) return st;
        uint8_t *ho = (uint8_t *)d->h_out.p;
        hipMemcpyAsync(ho, dout, out_total, hipMemcpyDeviceToHost, d->stream);
        if (hipStreamSynchronize(d->stream) != hipSuccess) return SDB_DEVICE_ERROR;
        sdb_decode_summary sm;
        memcpy(&sm, ho + o_sm, sizeof sm);
        if (sm.status == SDB_INVALID_ARGUMENT && attempt == 0 &&
            (sm.num_entries > cap_e || sm.key_bytes > key_cap)) {
            cap_e = sm.num_entries + 16;
            key_cap = sm.key_bytes + 4096;
            continue;
        }
        // value references are positions in the caller's `blocks` (block_off[0] was rebased to 0)
        uint64_t *vo_h = (uint64_t *)(ho + o_vo);
        const uint32_t *vl_h = (const uint32_t *)(ho + o_vl);
        if (b0)
            for (uint64_t i = 0; i < sm.num_entries && i < cap_e; i++)
                if (vl_h[i]) vo_h[i] += b0;
        r->summary = sm;
        r->block_entry_start = (const uint64_t *)(ho + o_bes);
        r->key_arena = ho + o_ka;
        r->key_off = (const uint64_t *)(ho + o_ko);
        r->val_off = (const uint64_t *)(ho + o_vo);
        r->val_len = (const uint32_t *)(ho + o_vl);
        r->seq = (const uint64_t *)(ho + o_seq);
        r->flags = ho + o_fl;
        r->create_ts = (const int64_t *)(ho + o_ct);
        r->expire_ts = (const int64_t *)(ho + o_et);
        r->bad_block = (const uint32_t *)(ho + o_bad);
        return (sdb_status)sm.status;
    }
    return SDB_INVALID_ARGUMENT;
}

}  // extern "C"

// Diagnostics: the fused bloom's slot plan inside sdb_encode_sst's workspace: byte offset of the run
// counts (tiles x nslices u32), tiles, slices and slot capacity.
extern "C" uint64_t sdb_diag_bloom_slots(uint64_t n, const sdb_sst_params *p, uint32_t *tiles, uint32_t *nslices,
                                         uint32_t *cap) {
    const uint64_t fb = p && p->bloom_bits_per_key ? filter_bytes_for(n, p->bloom_bits_per_key) : 0;
    const uint32_t k = p ? num_probes_for(p->bloom_bits_per_key) : 0;
    const BloomPlan pl = bloom_plan(n, k, fb, kChunk);
    *tiles = pl.tiles;
    *nslices = pl.nslices;
    *cap = bloom_slot_cap(pl);
    const uint64_t off = sdb::encode_workspace_layout(n, fb, k).bloom_rep;
    return (off + 255) & ~255ull;
}
