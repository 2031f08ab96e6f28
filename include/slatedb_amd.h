/*
 * slatedb_amd.h — C ABI of the MI355X-native SST block codec + bloom-filter builder.
 *
 * This is the drop-in boundary for slatedb's SST encode/decode hot path.  Every entry point is
 * plain C (no HIP/torch types): pointers, sizes, an opaque stream handle and a status code.
 * Citations are `path:line` relative to the slatedb reference (workspace 0.15.0).
 *
 * What each group replaces (the reference side is Rust; the binding a maintainer would add is in
 * INTEGRATION.md):
 *   - sdb_encode_sst*          -> EncodedSsTableBuilder::{add, finish_block, build}
 *                                 (slatedb/src/sst_builder.rs:224-254, 284-326, 370-417) with
 *                                 BlockBuilderV2 / BlockBuilderV1 (format/block_v2.rs:118-240,
 *                                 format/block.rs:76-218), SstRowCodecV2 / SstRowCodecV0
 *                                 (format/row_codec_v2.rs:127-169, format/row.rs:159-198), the
 *                                 per-block CRC32 of compress_and_transform (format/sst.rs:525-554)
 *                                 and BloomFilterBuilder (filter.rs:40-90).
 *   - sdb_bloom_build*         -> FilterBuilder::build for BloomFilterPolicy "_bf"
 *                                 (filter_policy.rs:170-283, filter.rs:71-90, 196-239).
 *   - sdb_bloom_might_contain  -> BloomFilter::might_contain (filter.rs:124-136).
 *   - sdb_decode_blocks*       -> SsTableFormat::read_blocks/decode_block + validate_checksum
 *                                 (format/sst.rs:938-999, 1029-1038) followed by draining
 *                                 DataBlockIterator ascending (block_iterator.rs:54-101,
 *                                 block_iterator_v2.rs:235-267) — the contract of the public
 *                                 SstFile::read_block (sst_reader.rs:287-309).
 *   - sdb_sst_builder_*        -> host-side mirror of EncodedSsTableBuilder's add()/build()/
 *                                 next_block() call order (sst_builder.rs:224-276), batching
 *                                 entries into a columnar pinned buffer and encoding on the GPU.
 *
 * Conventions
 *   - "device" entry points take device pointers and enqueue on `stream` (a hipStream_t passed as
 *     void*; NULL = the legacy default stream).  They never allocate, never synchronise, launch only
 *     on `stream` (no side streams, no cross-stream events; concurrent calls on different streams
 *     share nothing), and are safe to capture into a HIP graph.  Results that the host needs
 *     (lengths, status) are written
 *     to a device-resident summary struct the caller copies back.
 *   - "host" entry points take host pointers, manage a per-handle device arena + pinned staging and
 *     return synchronously.
 *   - Keys/values are Arrow-style columnar: entry i's key is key_bytes[key_off[i] .. key_off[i+1]).
 *     Offsets are monotone (n+1 entries, key_off[0] may be non-zero).
 *   - The library fails loudly: if no HIP device is present every compute entry point returns
 *     SDB_DEVICE_ERROR.  There is no CPU fallback.
 */
#ifndef SLATEDB_AMD_H
#define SLATEDB_AMD_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define SDB_ABI_VERSION 2u

/* Status codes.  Mirrors the hot-path variants of SlateDBError (slatedb/src/error.rs:23-38,
 * 142-152, 197); the reference *panics* where SDB_LIMIT_EXCEEDED is returned. */
typedef enum sdb_status {
    SDB_OK = 0,
    SDB_EMPTY_KEY = 1,              /* SlateDBError::EmptyKey (block_v2.rs:168-170) / assert in
                                       compute_lower_bound (utils.rs:210) */
    SDB_EMPTY_BLOCK = 2,            /* SlateDBError::EmptyBlock */
    SDB_CHECKSUM_MISMATCH = 3,      /* SlateDBError::ChecksumMismatch (format/sst.rs:1029-1038) */
    SDB_INVALID_ROW_FLAGS = 4,      /* SlateDBError::InvalidRowFlags (row_codec_v2.rs:234-249) */
    SDB_INVALID_VERSION = 5,        /* SlateDBError::InvalidVersion (block_iterator.rs:60-77) */
    SDB_LIMIT_EXCEEDED = 6,         /* reference panics: u16 asserts row.rs:73-85, block_v2.rs:195 */
    SDB_UNSUPPORTED = 7,            /* compression / block transformer (not on this path) */
    SDB_INVALID_ARGUMENT = 8,       /* bad kind byte, capacity too small, NULL pointer, ... */
    SDB_CORRUPT_BLOCK = 9,          /* block bytes that the reference would panic on while parsing */
    SDB_MERGE_OPERATOR_MISSING = 10,/* SlateDBError::MergeOperatorMissing (merge_operator.rs:213-223) */
    SDB_DECOMPRESSION_ERROR = 11,   /* SlateDBError::BlockDecompressionError (format/sst.rs:884-917) */
    SDB_DEVICE_ERROR = 100          /* no HIP device / launch failure */
} sdb_status;

/* Entry kinds: ValueDeletable::{Value, Merge, Tombstone} (types.rs:166-173). */
enum { SDB_KIND_VALUE = 0, SDB_KIND_MERGE = 1, SDB_KIND_TOMBSTONE = 2 };
/* Row flags, RowFlags (format/row.rs:8-16). */
enum { SDB_FLAG_TOMBSTONE = 1, SDB_FLAG_HAS_EXPIRE_TS = 2, SDB_FLAG_HAS_CREATE_TS = 4,
       SDB_FLAG_MERGE_OPERAND = 8 };
/* ts_mask bits. */
enum { SDB_TS_CREATE = 1, SDB_TS_EXPIRE = 2 };

/* A sorted run of RowEntry (types.rs:17-29), key asc / seq desc (mem_table.rs:38-44), columnar. */
typedef struct sdb_kv_batch {
    uint64_t n;
    const uint8_t *key_bytes;
    const uint64_t *key_off;    /* n+1 */
    const uint8_t *val_bytes;   /* tombstones: value bytes are ignored (treated as empty) */
    const uint64_t *val_off;    /* n+1 */
    const uint8_t *kind;        /* n; NULL = all SDB_KIND_VALUE */
    const uint64_t *seq;        /* n; NULL = all 0 */
    const int64_t *create_ts;   /* n (NULL = none); used where ts_mask & SDB_TS_CREATE, any entry may be read */
    const int64_t *expire_ts;   /* n (NULL = none); used where ts_mask & SDB_TS_EXPIRE, any entry may be read */
    const uint8_t *ts_mask;     /* n; NULL = no timestamps */
    const int32_t *prefix_len;  /* n; SDB_PREFIX_LENGTHS only: PrefixExtractor::prefix_len(Point(key))
                                   computed by the caller's extractor (-1 = None); else NULL */
} sdb_kv_batch;

enum { SDB_SST_COMPACTED = 0, SDB_SST_WAL = 1 };   /* SstType (schemas/sst.fbs) */
/* Prefix extractor of BloomFilterPolicy::with_prefix_extractor (filter_policy.rs:213-224, filter.rs:
 * 40-63, prefix_extractor.rs:41-95).  The extractor is a user trait object in the reference; the
 * device evaluates the two stateless families the reference's tests use, or takes the lengths the
 * caller's own extractor returned (SDB_PREFIX_LENGTHS), which covers any extractor. */
enum { SDB_PREFIX_NONE = 0,
       SDB_PREFIX_FIXED = 1,    /* prefix_len = key.len() >= arg ? Some(arg) : None */
       SDB_PREFIX_DELIM = 2,    /* first byte == arg at i: Some(i + 1), else None */
       SDB_PREFIX_LENGTHS = 3 };/* sdb_kv_batch.prefix_len / the query lengths */

/* SsTableFormat knobs on this path (format/sst.rs:620-643, db/builder.rs:439-531). */
typedef struct sdb_sst_params {
    uint32_t block_size;         /* SstBlockSize, default 4096 (config.rs:231-267) */
    uint16_t sst_version;        /* 1 = BlockBuilderV1 + SstRowCodecV0, 2 = BlockBuilderV2 + V2 */
    uint16_t restart_interval;   /* V2 only; reference constant 16 (block_v2.rs:8) */
    uint32_t bloom_bits_per_key; /* BloomFilterPolicy::new(bpk) (filter_policy.rs:201); 0 = none */
    uint32_t min_filter_keys;    /* filter built iff num_rows >= min_filter_keys (sst_builder.rs:390) */
    uint32_t sst_type;           /* SDB_SST_COMPACTED, or SDB_SST_WAL: EncodedWalSsTableBuilder
                                    (wal/slatedb/sst_builder.rs:68-205): entries in insertion order,
                                    no compute_index_key (so no prefix panic), no filter; V2 only */
    uint32_t prefix_kind;        /* SDB_PREFIX_*: prefix hashes (deduplicated against the previous
                                    key's prefix) join the filter (filter.rs:40-58) */
    uint32_t prefix_arg;         /* FIXED: the length; DELIM: the delimiter byte */
    uint32_t no_whole_key;       /* 1 = with_whole_key_filtering(false) (filter_policy.rs:226-235):
                                    full keys are not hashed; 0 (default) = they are */
} sdb_sst_params;

/* Scalar results of one SST encode, written by the device. */
typedef struct sdb_sst_summary {
    uint64_t data_len;           /* bytes of data section (all blocks incl. CRC) */
    uint64_t num_blocks;
    uint64_t num_entries;
    uint64_t raw_key_size;       /* SstStats::raw_key_size (sst_builder.rs:225) */
    uint64_t raw_val_size;       /* SstStats::raw_val_size (sst_builder.rs:226) */
    uint64_t num_puts, num_deletes, num_merges;
    uint64_t bloom_len;          /* bitmap bytes (0 if no filter) */
    uint32_t num_probes;         /* optimal_num_probes(bpk) (filter.rs:235-239) */
    uint32_t filter_built;       /* 1 iff a filter was built */
    int32_t status;              /* sdb_status of the device-side checks */
    uint32_t max_block_entries;  /* diagnostics: longest block in entries */
    uint64_t first_error_entry;  /* entry index that raised `status` (UINT64_MAX if none) */
} sdb_sst_summary;

/* Caller-owned outputs.  For sdb_encode_sst (device) every pointer is device memory. */
typedef struct sdb_sst_out {
    uint8_t *data;               /* data section: blocks (Block::encode ++ crc32 BE), contiguous */
    uint64_t data_cap;
    uint64_t *block_off;         /* num_blocks+1 byte offsets into data (BlockMeta.offset) */
    uint32_t *block_first_entry; /* num_blocks+1 entry indices (last = n) */
    uint32_t *index_key_len;     /* per block: BlockMeta.first_key = key(first entry)[..len]
                                    (compute_index_key, utils.rs:198-226); block 0 -> 0 */
    uint16_t *block_stats;       /* 3 per block: num_puts, num_deletes, num_merges (sst_stats.rs:9-16) */
    uint64_t block_cap;          /* capacity (in blocks) of the four arrays above */
    uint8_t *bloom;              /* bloom bitmap (BloomFilter.buffer; the u16 BE num_probes header of
                                    Filter::encode is NOT included) */
    uint64_t bloom_cap;
    sdb_sst_summary *summary;    /* device-writable */
} sdb_sst_out;

/* ---------------------------------------------------------------------------------------------
 * Sizing (pure host arithmetic, no device needed)
 * ------------------------------------------------------------------------------------------- */
uint32_t sdb_abi_version(void);
/* Upper bounds on the output arrays for a batch of n entries holding the given key/value bytes. */
sdb_status sdb_encode_bounds(uint64_t n, uint64_t total_key_bytes, uint64_t total_val_bytes,
                             const sdb_sst_params *params, uint64_t *data_cap,
                             uint64_t *block_cap, uint64_t *bloom_cap);
/* Device scratch needed by sdb_encode_sst for n entries. */
uint64_t sdb_encode_workspace_bytes(uint64_t n, const sdb_sst_params *params);
/* BloomFilterBuilder::filter_size_bytes (filter.rs:65-69): ceil(u32(n*bpk)/8). */
uint64_t sdb_bloom_filter_bytes(uint64_t num_keys, uint32_t bits_per_key);
/* optimal_num_probes (filter.rs:235-239). */
uint32_t sdb_bloom_num_probes(uint32_t bits_per_key);

/* ---------------------------------------------------------------------------------------------
 * Device entry points (device pointers, async on `stream`)
 * ------------------------------------------------------------------------------------------- */
/* Encode one SST's data section + bloom bitmap from a device-resident sorted batch.  Host-side
 * argument errors are returned directly; data-dependent errors (empty key, V1 u16 overflow, bad
 * kind) are reported in out->summary->status after the stream completes. */
sdb_status sdb_encode_sst(const sdb_kv_batch *batch, const sdb_sst_params *params,
                          const sdb_sst_out *out, void *workspace, uint64_t workspace_bytes,
                          void *stream);

/* Encode `count` independent SSTs that share `params` in ONE launch sequence on `stream` (the SSTs of
 * one compaction job or of concurrent L0 flushes: l0_flush_parallelism / subcompactions,
 * config.rs:1081, 1383-1390).  Same per-SST contract as sdb_encode_sst (outs[i] for batches[i]; the
 * device checks land in outs[i].summary).  The kernels of up to 8 SSTs share each launch, so the
 * latency-bound segmentation of small grids fills the chip; larger counts run as consecutive sets.
 * workspace: sdb_encode_ssts_workspace_bytes(count, batches, params) bytes (only batches[i].n is read
 * on the host). */
uint64_t sdb_encode_ssts_workspace_bytes(uint32_t count, const sdb_kv_batch *batches,
                                         const sdb_sst_params *params);
sdb_status sdb_encode_ssts(uint32_t count, const sdb_kv_batch *batches, const sdb_sst_params *params,
                           const sdb_sst_out *outs, void *workspace, uint64_t workspace_bytes,
                           void *stream);
/* Scheduling hint: the caller keeps `builders` encode launch sequences (sdb_encode_sst / _ssts on distinct
 * streams, e.g. the concurrent SST writers of compactions and flushes) in flight on the current device.
 * The block-assembly kernel then takes 1/builders of the CUs (at least 1 workgroup), so one sequence's
 * segmentation kernels run on the CUs another sequence's assembly leaves free (1, the default: every
 * CU).  Process-wide per device; results do not depend on it.  SDB_INVALID_ARGUMENT for 0. */
sdb_status sdb_set_concurrent_builders(uint32_t builders);

/* Bloom bitmap over n keys (BloomFilterBuilder with whole-key filtering, filter.rs:40-90).
 * bitmap must hold sdb_bloom_filter_bytes(n, bpk) bytes and be 4-byte aligned (the build stores
 * 32-bit words); it is zeroed and filled on `stream`.  workspace (sdb_bloom_workspace_bytes) holds
 * the binned probes; NULL selects the slower device-scope-atomic build, which also needs
 * bitmap_bytes >= the filter size rounded up to 4.  Otherwise SDB_INVALID_ARGUMENT. */
uint64_t sdb_bloom_workspace_bytes(uint64_t num_keys, uint32_t bits_per_key);
sdb_status sdb_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                           uint32_t bits_per_key, uint8_t *bitmap, uint64_t bitmap_bytes,
                           void *workspace, uint64_t workspace_bytes, void *stream);

/* Filter over whole keys and/or extracted prefixes (BloomFilterBuilder::add_key with a prefix
 * extractor, filter.rs:40-90): the filter's size follows the number of hashes (full keys + distinct
 * consecutive prefixes), which the device counts, so the byte length is written to *bloom_len (device
 * u64).  bitmap: 4-byte aligned, >= sdb_bloom_filter_bytes(2 n, bpk) bytes (the bound).  prefix_len:
 * per-key lengths for SDB_PREFIX_LENGTHS (else NULL).  Keys must be sorted for the prefix dedup. */
uint64_t sdb_bloom_prefix_workspace_bytes(uint64_t n);
sdb_status sdb_bloom_build_prefix(const uint8_t *key_bytes, const uint64_t *key_off, const int32_t *prefix_len,
                                  uint64_t n, uint32_t bits_per_key, uint32_t prefix_kind,
                                  uint32_t prefix_arg, uint32_t whole_key, uint8_t *bitmap,
                                  uint64_t bitmap_cap, uint64_t *bloom_len, void *workspace,
                                  uint64_t workspace_bytes, void *stream);
/* Filter::might_match (filter.rs:149-175) for FilterQuery targets: is_prefix[i] = 0 -> Point(key),
 * 1 -> Prefix(key) (a scan prefix; NULL = all points).  With whole-key filtering a point probes the
 * full key; otherwise the extracted prefix (query_prefix_len for SDB_PREFIX_LENGTHS, -1 = None); no
 * extractable prefix answers 1 (no false negative).  result[i] = 1 iff the key may be present. */
sdb_status sdb_bloom_might_match(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes,
                                 uint32_t whole_key, uint32_t prefix_kind, uint32_t prefix_arg,
                                 const uint8_t *key_bytes, const uint64_t *key_off,
                                 const uint8_t *is_prefix, const int32_t *query_prefix_len, uint64_t n,
                                 uint8_t *result, void *stream);

/* Batched BloomFilter::might_contain(filter_hash(key)) (filter.rs:124-136, 150-175): result[i]=1
 * iff every probe bit is set.  An empty bitmap answers 0.  The bitmap may start at any byte address
 * (e.g. inside an SST's filter block); only bytes [0, bitmap_bytes) are read. */
sdb_status sdb_bloom_might_contain(const uint8_t *bitmap, uint64_t bitmap_bytes,
                                   uint32_t num_probes, const uint8_t *key_bytes,
                                   const uint64_t *key_off, uint64_t n, uint8_t *result,
                                   void *stream);

/* Decoded entries, columnar, ascending order within and across blocks. */
typedef struct sdb_decode_summary {
    uint64_t num_entries;
    uint64_t key_bytes;
    uint64_t num_bad_blocks;
    int32_t status;              /* error of the lowest-index failing block (try_join_all order) */
    uint32_t pad;
} sdb_decode_summary;

typedef struct sdb_decoded_out {
    uint64_t *block_entry_start; /* nblocks+1 */
    uint8_t *key_arena;          /* full keys restored (restore_full_key, row_codec_v2.rs:83-89) */
    uint64_t key_arena_cap;
    uint64_t *key_off;           /* cap_entries+1 */
    uint64_t *val_off;           /* byte offset of the value inside `blocks` (zero-copy, like
                                    Bytes::slice); tombstones -> 0 */
    uint32_t *val_len;
    uint64_t *seq;
    uint8_t *flags;              /* RowFlags of the row; kind = tombstone/merge/value from it */
    int64_t *create_ts;          /* valid iff flags & HAS_CREATE_TS */
    int64_t *expire_ts;          /* valid iff flags & HAS_EXPIRE_TS (V0 tombstones: never) */
    uint64_t cap_entries;
    uint32_t *bad_block;         /* indices of blocks that failed (CRC / flags / parse) */
    uint64_t bad_cap;
    sdb_decode_summary *summary; /* device-writable */
} sdb_decoded_out;

uint64_t sdb_decode_workspace_bytes(uint64_t nblocks);
/* Decode nblocks encoded blocks (each = Block::encode ++ crc32 BE) located at
 * blocks[block_off[k] .. block_off[k+1]).  sst_version 1 or 2 selects the row codec. */
sdb_status sdb_decode_blocks(const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                             uint16_t sst_version, const sdb_decoded_out *out, void *workspace,
                             uint64_t workspace_bytes, void *stream);

/* Decode nblocks blocks placed anywhere in one device arena: block k = arena[block_start[k] ..
 * block_end[k]).  The read path fetches an SST's blocks as ~2 MiB ranged GETs (read_blocks,
 * format/sst.rs:919-978; bytes_to_fetch / max_fetch_tasks, config.rs:1323-1337) and splits each per
 * BlockMeta.offset; uploading many such ranges into one arena and decoding them here costs one launch
 * sequence instead of one per range.  Same output contract as sdb_decode_blocks; val_off is relative to
 * `arena`.  Workspace: sdb_decode_workspace_bytes(nblocks). */
sdb_status sdb_decode_blocks_at(const uint8_t *arena, const uint64_t *block_start, const uint64_t *block_end,
                                uint64_t nblocks, uint16_t sst_version, const sdb_decoded_out *out,
                                void *workspace, uint64_t workspace_bytes, void *stream);

/* Decode with options.  block_end == NULL: contiguous blocks (block_start has nblocks + 1 entries),
 * else as sdb_decode_blocks_at.  flags:
 *   SDB_DECODE_DESCENDING  entries in descending iteration order, as SstIterator in
 *     IterationOrder::Descending yields them (sst_iter.rs:460, 557): blocks last to first, each
 *     through DescendingBlockIteratorV2 (block_iterator_v2.rs:318-430) / BlockIterator Descending
 *     (block_iterator.rs:159-224).  Keys / columns are in that order; block_entry_start keeps the
 *     ascending prefix of the per-block counts, so block k's entries are [N - bes[k+1], N - bes[k]).
 *     A V2 block whose restart regions do not start at restarts with shared == 0 and end at the next
 *     one reports SDB_CORRUPT_BLOCK (the reference asserts there, block_iterator_v2.rs:76).
 *   SDB_DECODE_FAIL_FAST   read_blocks semantics (format/sst.rs:938-1038, all or nothing): the status is
 *     the first failing block's, in block order, with its checksum verified before its rows as
 *     decode_block does, and every column is unspecified when the call fails (without the flag the
 *     good blocks are still decoded and the bad ones listed).  The checksums are then verified by the
 *     emit pass, which re-reads every block anyway, instead of the count pass. */
enum { SDB_DECODE_DESCENDING = 1, SDB_DECODE_FAIL_FAST = 2 };
sdb_status sdb_decode_blocks_ex(const uint8_t *arena, const uint64_t *block_start, const uint64_t *block_end,
                                uint64_t nblocks, uint16_t sst_version, uint32_t flags, const sdb_decoded_out *out,
                                void *workspace, uint64_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Compressed blocks (SsTableInfo.compression_format != None): the first half of decode_block
 * (format/sst.rs:980-999) — validate_checksum over the stored bytes, then SsTableFormat::decompress
 * (format/sst.rs:884-917) — on the device, for every codec:
 *   SDB_CODEC_LZ4     lz4_flex 0.11.6 block::decompress_size_prepended (u32 LE size, then an LZ4 block;
 *                     output shorter than the declared size is kept, as lz4_flex truncates);
 *   SDB_CODEC_SNAPPY  snap 1.1.1 raw::Decoder::decompress_vec (varint size, then Snappy raw elements);
 *   SDB_CODEC_ZLIB    flate2 1.1.9 read::ZlibDecoder::read_to_end (zlib header, deflate, Adler-32; input
 *                     that ends inside the stream yields the bytes decoded so far, as flate2's read does);
 *   SDB_CODEC_ZSTD    zstd 0.13.3 stream::decode_all (zstd frames and skippable frames in sequence).
 * Two steps, so the caller can size the output:
 *   1. sdb_decompress_plan writes out_start[0..nblocks] (device): block k's output slot starts at
 *      out_start[k] and holds its decompressed length + 4 (the declared length for Lz4 / Snappy, the
 *      frames' Frame_Content_Size for Zstd — zstd::bulk::compress writes it — and a count-mode decode
 *      for Zlib and for Zstd frames without one; Adler-32 / XXH64 checksums are verified in step 2);
 *      out_start[nblocks] = the bytes `out` needs.  A header that cannot be read, a Zlib / Zstd stream
 *      that fails to decode, or more than 64 MiB gets an empty slot (that block then fails in step 2).
 *   2. sdb_decompress_blocks fills out[out_start[k] .. out_end[k]) with the uncompressed block followed
 *      by the CRC32 (BE) of those bytes — Block::encode() ++ crc, so sdb_decode_blocks_at(out,
 *      out_start, out_end, ...) decodes the run (value references then point into `out`).  *err
 *      (device u64) = block << 8 | status of the first failing block in block order (~0: none):
 *      SDB_CHECKSUM_MISMATCH, SDB_DECOMPRESSION_ERROR, SDB_CORRUPT_BLOCK (fewer than 4 bytes),
 *      SDB_LIMIT_EXCEEDED (over 64 MiB) or SDB_INVALID_ARGUMENT (slot past out_cap); a failing block's
 *      out_end[k] = out_start[k].
 * blocks / block_off (nblocks + 1) as sdb_decode_blocks.  Workspace (step 1 only):
 * sdb_decompress_workspace_bytes(nblocks). */
enum { SDB_CODEC_NONE = 0, SDB_CODEC_SNAPPY = 1, SDB_CODEC_ZLIB = 2, SDB_CODEC_LZ4 = 3, SDB_CODEC_ZSTD = 4 };
uint64_t sdb_decompress_workspace_bytes(uint64_t nblocks);
sdb_status sdb_decompress_plan(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                               uint64_t *out_start, void *workspace, uint64_t workspace_bytes, void *stream);
sdb_status sdb_decompress_blocks(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                 uint8_t *out, uint64_t out_cap, const uint64_t *out_start, uint64_t *out_end,
                                 uint64_t *err, void *stream);
/* Both steps without a host synchronisation between them (out sized by the caller up front).  For
 * SDB_CODEC_ZLIB, whose plan is a whole inflate, each block is inflated once into a slot of slot_bytes
 * (out_start[k] = k * slot_bytes, 8 <= slot_bytes <= 4 GiB, out_cap >= nblocks * slot_bytes); the blocks
 * whose output + 4 does not fit their slot are planned and inflated again, packed from
 * nblocks * slot_bytes on, and their out_start[k] rewritten — so out_start is not monotone and
 * out_start[nblocks] = the bytes of out the call used.  A block past out_cap fails with
 * SDB_INVALID_ARGUMENT as in step 2.  Zlib blocks coded with deflate's fixed code or stored (what
 * sdb_compress_blocks writes) are inflated one per lane against shared tables; dynamic-Huffman blocks (what
 * flate2 at its default level writes) take the per-decoder-table kernel.  The other codecs ignore
 * slot_bytes: the plan and the run back to
 * back (out_start as step 1 writes it).  out_start / out_end / *err then mean what step 2 says, and
 * sdb_decode_blocks_at(out, out_start, out_end, ...) decodes the run.  Workspace:
 * sdb_decompress_once_workspace_bytes(nblocks). */
uint64_t sdb_decompress_once_workspace_bytes(uint64_t nblocks);
sdb_status sdb_decompress_blocks_once(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                      uint64_t slot_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_start,
                                      uint64_t *out_end, uint64_t *err, void *workspace, uint64_t workspace_bytes,
                                      void *stream);

/* The compressing write side: compress_and_transform (format/sst.rs:525-554) with SsTableFormat::compress
 * (format/sst.rs:557-594) for every block of an encoded data section (each Block::encode() ++ CRC32 BE, as
 * sdb_encode_sst writes it): block k becomes the codec's bytes of its Block::encode() followed by the CRC32
 * (BE) of those compressed bytes, at out[out_off[k], out_off[k + 1]):
 *   SDB_CODEC_LZ4     u32 LE length ++ one LZ4 block (lz4_flex block::compress_prepend_size);
 *   SDB_CODEC_SNAPPY  varint length ++ Snappy raw elements (snap raw::Encoder::compress_vec);
 *   SDB_CODEC_ZLIB    78 9C ++ deflate (a dynamic-Huffman, fixed-Huffman or stored block per 4 KiB window,
 *                     whichever is shortest) ++ Adler-32 BE (flate2 ZlibEncoder, default level 6);
 *   SDB_CODEC_ZSTD    one zstd frame with Frame_Content_Size, a compressed block per 4 KiB window (Huffman
 *                     or raw / RLE literals, sequences with predefined / RLE / FSE-compressed tables) or a
 *                     raw / RLE block when shorter (zstd::bulk::compress at level 3).
 * One wave per block: hash-chain LZ77 with lazy matching in the wave's LDS, entropy codes built by the wave
 * (compression ratio within a few per cent of the canonical libraries).  The streams are valid for their formats and
 * decode (the crates' decompressors, sdb_decompress_blocks) to the block; they are not the crates' own
 * bytes (a match finder's choices are its own).  in_bytes = block_off[nblocks] - block_off[0];
 * out_off (device, nblocks + 1) = the compressed blocks' offsets from out (BlockMeta.offset when the data
 * section starts the SST), out_off[nblocks] = the compressed data section's length.  *err (device u64) =
 * block << 8 | status of the first failing block (~0: none): SDB_CORRUPT_BLOCK (a block under 4 bytes),
 * SDB_LIMIT_EXCEEDED (the section is over out_cap: nothing is written).
 * Workspace: sdb_compress_workspace_bytes(nblocks, in_bytes). */
uint64_t sdb_compress_workspace_bytes(uint64_t nblocks, uint64_t in_bytes);
sdb_status sdb_compress_blocks(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                               uint64_t in_bytes, uint8_t *out, uint64_t out_cap, uint64_t *out_off, uint64_t *err,
                               void *workspace, uint64_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Point lookups / seeks on one encoded SST (device): the read path of Db::get and of an SstIterator
 * positioned on a key:
 *   1. filter: BloomFilter::might_contain(filter_hash(key)) (filter.rs:124-136, sst_iter.rs:201-227);
 *   2. blocks: partitions_covering_range([key, key]) over BlockMeta.first_key (partitioned_keyspace.rs:
 *      16-110), i.e. [first_partition_including_or_after_key, last_partition_including_key + 1);
 *   3. the first block of that range in iteration order is seeked (sst_iter.rs:501-516):
 *      BlockIteratorV2::seek (block_iterator_v2.rs:138-208, 269-313) ascending or
 *      DescendingBlockIteratorV2::seek (:318-469); BlockIterator::seek for V1 (block_iterator.rs:
 *      130-190); when it is exhausted the next block of the range is entered at its first entry
 *      (ascending) or its last (descending);
 *   4. the entry the iterator returns next is reported, and FOUND if its key equals the query.
 * Each block read is CRC-checked first (validate_checksum, format/sst.rs:1029-1038).
 * ------------------------------------------------------------------------------------------- */
enum { SDB_LOOKUP_FILTERED = 0,     /* the bloom filter rules the key out (no block read) */
       SDB_LOOKUP_EXHAUSTED = 1,    /* no entry at or past the key in iteration order */
       SDB_LOOKUP_POSITIONED = 2,   /* positioned on an entry whose key differs from the query */
       SDB_LOOKUP_FOUND = 3 };      /* positioned on an entry with key == query (newest version) */
typedef struct sdb_sst_view {       /* device pointers into one encoded SST */
    const uint8_t *data;            /* data section (blocks ++ crc) */
    const uint64_t *block_off;      /* num_blocks + 1: BlockMeta.offset, then the data length */
    uint64_t num_blocks;
    const uint8_t *index_keys;      /* BlockMeta.first_key of block k = */
    const uint64_t *index_key_off;  /*   index_keys[index_key_off[k] .. index_key_off[k + 1]) */
    const uint8_t *bloom;           /* bitmap (filter without its u16 header); NULL = no filter */
    uint64_t bloom_len;
    uint32_t num_probes;
    uint16_t sst_version;           /* 1 or 2 */
    uint16_t pad;
} sdb_sst_view;
typedef struct sdb_lookup_out {     /* device arrays, one element per query */
    uint8_t *state;                 /* SDB_LOOKUP_* */
    int32_t *status;                /* sdb_status of the blocks read (CHECKSUM_MISMATCH, ...) */
    uint32_t *block;                /* block of the positioned entry */
    uint32_t *entry;                /* index of that entry inside its block (physical order) */
    uint32_t *key_len;              /* its key length */
    uint64_t *val_off;              /* its value: data[val_off .. val_off + val_len) (tombstone: 0, 0) */
    uint32_t *val_len;
    uint64_t *seq;
    uint8_t *flags;                 /* RowFlags as the iterator returns them */
    int64_t *create_ts;             /* valid iff flags & HAS_CREATE_TS */
    int64_t *expire_ts;             /* valid iff flags & HAS_EXPIRE_TS */
} sdb_lookup_out;
uint64_t sdb_sst_lookup_workspace_bytes(uint64_t num_blocks, uint64_t nkeys);
sdb_status sdb_sst_lookup(const sdb_sst_view *sst, const uint8_t *key_bytes, const uint64_t *key_off,
                          uint64_t nkeys, int32_t descending, const sdb_lookup_out *out,
                          void *workspace, uint64_t workspace_bytes, void *stream);

/* ---------------------------------------------------------------------------------------------
 * Compaction (device): the output side of CompactionExecutor::run_subcompaction_merge
 * (compactor_executor.rs:386-410, 818-871) over decoded inputs:
 *   1. MergeIterator over the sorted runs, dedup off (merge_iterator.rs:56-69): key ascending, seq
 *      descending; equal (key, seq) pairs (which the store never writes) in run order;
 *   2. MergeOperatorRequiredIterator (merge_operator.rs:213-223): a merge operand fails the job with
 *      SDB_MERGE_OPERATOR_MISSING, unless `merge_operands` passes operands on unmerged;
 *   3. RetentionIterator (retention_iterator.rs:91-204, 381-398): per key, versions newest first,
 *      a later equal-seq version replacing an earlier one (BTreeMap::insert); expired merges are
 *      skipped, expired values / tombstones become tombstones without expire_ts; the walk stops
 *      after the first non-merge version outside both the seq and the time window; trailing
 *      tombstones are dropped when filter_tombstone;
 *   4. output SSTs cut where the bytes of the blocks the writer finished exceed max_sst_size: the
 *      entry whose add finished that block closes the SST as its one-entry tail block
 *      (compactor_executor.rs:833-858, sst_builder.rs:224-325); every SST then encodes as above.
 * sdb_merge_runs and sdb_sst_cuts are asynchronous on the caller's stream; sdb_compactor_run
 * orchestrates the whole job over decoded runs, sdb_compactor_run_ssts over encoded input SSTs.
 * ------------------------------------------------------------------------------------------- */
/* One sorted input run in the layout sdb_decode_blocks produces (a decoded SST, or a sorted run's
 * SSTs decoded into one output): value i = val_base[val_off[i] .. val_off[i] + val_len[i]). */
typedef struct sdb_run {
    uint64_t n;
    const uint8_t *key_arena;
    const uint64_t *key_off;        /* n+1 */
    const uint8_t *val_base;
    const uint64_t *val_off;        /* n */
    const uint32_t *val_len;        /* n */
    const uint64_t *seq;            /* n */
    const uint8_t *flags;           /* n: RowFlags (SDB_FLAG_*) */
    const int64_t *create_ts;       /* n: valid iff flags & HAS_CREATE_TS (NULL: none anywhere) */
    const int64_t *expire_ts;       /* n: valid iff flags & HAS_EXPIRE_TS (NULL: none anywhere) */
} sdb_run;
enum { SDB_MAX_RUNS = 32 };        /* runs of one sdb_merge_runs call; the compactor merges more in groups of
                                      this many first (up to SDB_MAX_RUNS^2 runs per job) */
typedef struct sdb_retention {
    uint64_t min_seq;               /* retention_min_seq: the walk continues past seq > min_seq
                                       (retention_iterator.rs:188-190) when has_min_seq */
    uint64_t time_seq;              /* retention_timeout resolved on the host: the walk continues past
                                       seq >= time_seq when has_time_window (create_sys_ts + timeout > now,
                                       :171-187; SequenceTracker::find_ts(.., RoundUp) is monotone in seq,
                                       so the seqs inside the window are an up-set; 0 = every seq) */
    int64_t compaction_start_ts;    /* compaction_clock_tick: expire_ts <= this has expired */
    uint8_t has_min_seq, has_time_window;
    uint8_t filter_tombstone;       /* is_dest_last_run */
    uint8_t merge_operands;         /* 0: MergeOperatorRequiredIterator; 1: operands pass unmerged */
    uint32_t pad;
} sdb_retention;
typedef struct sdb_merge_summary {
    uint64_t num_in;                /* entries of all runs */
    uint64_t num_out;               /* entries after retention */
    uint64_t key_bytes, val_bytes;  /* bytes written to the output arenas */
    uint64_t expired_values;        /* RetentionMetrics::expired_entries_purged_value */
    uint64_t expired_merges;        /* RetentionMetrics::expired_entries_purged_merge */
    int32_t status;                 /* SDB_OK | SDB_MERGE_OPERATOR_MISSING | SDB_INVALID_ARGUMENT (a run
                                       out of order: first_error_entry = its global index) */
    uint32_t pad;
    uint64_t first_error_entry;     /* merged position (or run entry) that raised status */
} sdb_merge_summary;
/* Merged, retained stream: an sdb_kv_batch (n = summary.num_out) in caller-owned device memory.
 * Capacities: cap_entries >= sum n, key_cap >= sum key bytes, val_cap >= sum value bytes. */
typedef struct sdb_merged_out {
    uint8_t *key_bytes;
    uint64_t key_cap;
    uint64_t *key_off;              /* cap_entries + 1 */
    uint8_t *val_bytes;
    uint64_t val_cap;
    uint64_t *val_off;              /* cap_entries + 1 */
    uint8_t *kind;
    uint64_t *seq;
    int64_t *create_ts;
    int64_t *expire_ts;
    uint8_t *ts_mask;
    uint64_t cap_entries;
    sdb_merge_summary *summary;     /* device-writable */
} sdb_merged_out;
uint64_t sdb_merge_runs_workspace_bytes(const sdb_run *runs, uint32_t nruns);
sdb_status sdb_merge_runs(const sdb_run *runs, uint32_t nruns, const sdb_retention *retention,
                          const sdb_merged_out *out, void *workspace, uint64_t workspace_bytes, void *stream);
/* SST boundaries of a compaction output stream: cut_start[0..*num_ssts] (device) are entry indices
 * with cut_start[0] = 0 and cut_start[*num_ssts] = n; SST i = entries [cut_start[i], cut_start[i+1]).
 * cut_cap >= n + 1 always suffices.  params: the output format (block size, restart interval). */
uint64_t sdb_sst_cuts_workspace_bytes(uint64_t n, const sdb_sst_params *params);
sdb_status sdb_sst_cuts(const sdb_kv_batch *batch, const sdb_sst_params *params, uint64_t max_sst_size,
                        uint64_t *cut_start, uint64_t cut_cap, uint64_t *num_ssts, void *workspace,
                        uint64_t workspace_bytes, void *stream);

/* A compaction job on the device: merge + retention + cuts + encode of every output SST, with the
 * outputs in the handle's device memory (valid until the next run or destroy). */
typedef struct sdb_compactor sdb_compactor;
typedef struct sdb_compacted_sst {
    uint64_t entry_start, entry_end;   /* range of the merged stream (sdb_compactor_merged) */
    const uint8_t *data;               /* device: the SST's data section */
    const uint64_t *block_off;         /* device: num_blocks + 1 */
    const uint32_t *block_first_entry; /* device: num_blocks + 1 (relative to entry_start) */
    const uint32_t *index_key_len;     /* device: num_blocks */
    const uint16_t *block_stats;       /* device: 3 per block */
    const uint8_t *bloom;              /* device: summary.bloom_len bytes */
    sdb_sst_summary summary;           /* host copy */
} sdb_compacted_sst;
sdb_compactor *sdb_compactor_create(int device);
void sdb_compactor_destroy(sdb_compactor *c);
sdb_status sdb_compactor_run(sdb_compactor *c, const sdb_run *runs, uint32_t nruns, const sdb_retention *retention,
                             const sdb_sst_params *params, uint64_t max_sst_size, void *stream, uint32_t *num_ssts);
/* The same job from the encoded input SSTs, decode included (compactor_executor.rs:327-390, load_iterators:
 * each input SST is read block by block and decoded; an L0 SST is a sorted run, a sorted run of several
 * SSTs is their concatenation).  Every input's blocks are decoded by one launch sequence (CRC check,
 * V1/V2 rows, key restore; values stay in place, like Bytes::slice), straight into the merge's runs; the
 * merged stream is sized from the inputs' SstStats, so the job synchronises with the host twice: for the
 * merged count with the cut list, and for the output SSTs' summaries.  Input i: an uncompressed data
 * section on the device and the counts its footer holds.  Runs: inputs [run_start[r], run_start[r+1]),
 * run_start == NULL: one run per input.  A failing input block fails the job with its status (lowest
 * block first; the merged summary's first_error_entry = that block's index among all inputs' blocks);
 * counts that disagree with the decoded blocks fail it with SDB_INVALID_ARGUMENT.  Any number of inputs
 * (their block tables go to device memory); more than SDB_MAX_RUNS runs are merged in groups first (one
 * more host synchronisation per group), up to SDB_MAX_RUNS^2 runs. */
typedef struct sdb_compaction_input {
    const uint8_t *data;            /* device: the data section (encoded blocks, each ++ crc32) */
    const uint64_t *block_off;      /* device: num_blocks + 1 (BlockMeta.offset of each block, then the
                                       data section length) */
    uint64_t num_blocks;
    uint64_t num_entries;           /* SstStats::num_rows() (num_puts + num_deletes + num_merges) */
    uint64_t key_bytes;             /* SstStats.raw_key_size */
    uint64_t val_bytes;             /* SstStats.raw_val_size */
} sdb_compaction_input;
sdb_status sdb_compactor_run_ssts(sdb_compactor *c, const sdb_compaction_input *inputs, uint32_t ninputs,
                                  const uint32_t *run_start, uint32_t nruns, uint16_t input_sst_version,
                                  const sdb_retention *retention, const sdb_sst_params *params,
                                  uint64_t max_sst_size, void *stream, uint32_t *num_ssts);
sdb_status sdb_compactor_sst(const sdb_compactor *c, uint32_t i, sdb_compacted_sst *out);
/* The merged stream of the last run (device batch view) and its summary (host copy). */
sdb_status sdb_compactor_merged(const sdb_compactor *c, sdb_kv_batch *batch, sdb_merge_summary *summary);

/* ---------------------------------------------------------------------------------------------
 * SST footer (host): everything after the data section, so data ++ footer is the whole SST object
 * EncodedSsTableBuilder::build / EncodedWalSsTableBuilder::build hand to write_sst.
 * Replaces EncodedSsTableFooterBuilder::build (format/sst.rs:383-487) plus the index the builders
 * accumulate per block (sst_builder.rs:228-237, 307-313; wal/slatedb/sst_builder.rs:129-205),
 * SstStats::encode (sst_stats.rs:52-86) and SsTableInfo::encode (format/sst.rs:195-199).
 * Layout: [filter block + crc]? [index + crc] [stats + crc]? [SsTableInfo + crc] [u64 BE meta
 * offset] [u16 BE version]; flatbuffer bytes identical to the `flatbuffers` 25.12.19 crate.
 * ------------------------------------------------------------------------------------------- */
typedef struct sdb_footer_in {
    uint16_t sst_version;             /* trailing u16 (SST_FORMAT_VERSION: 1 or 2) */
    uint8_t sst_type;                 /* SDB_SST_COMPACTED | SDB_SST_WAL */
    uint8_t has_filter;               /* write the composite "_bf" filter block */
    uint32_t num_probes;              /* Filter::encode header (filter.rs:177-180) */
    uint64_t data_len;                /* blocks_size: bytes of the data section before the footer */
    uint64_t num_blocks;
    const uint64_t *block_off;        /* num_blocks: BlockMeta.offset */
    const uint8_t *first_key_bytes;   /* BlockMeta.first_key of block k = */
    const uint64_t *first_key_off;    /*   first_key_bytes[first_key_off[k] .. first_key_off[k+1]) */
    const uint8_t *first_entry;       /* SsTableInfo.first_entry; NULL = None */
    uint64_t first_entry_len;
    const uint8_t *last_entry;        /* SsTableInfo.last_entry; NULL = None (WAL) */
    uint64_t last_entry_len;
    const sdb_sst_summary *stats;     /* SstStats totals; NULL = no stats block (WAL) */
    const uint16_t *block_stats;      /* 3 per block (puts, deletes, merges) */
    const uint8_t *bloom;             /* bitmap (has_filter) */
    uint64_t bloom_len;
    const char *filter_name;          /* FilterPolicy::name: NULL = "_bf"; a prefix / no-whole-key policy
                                         is "_bf:p=<extractor>[:wh=0]" (filter_policy.rs:237-250) */
    uint32_t compression;             /* SsTableInfo.compression_format (SDB_CODEC_*): the filter, index and
                                         stats blocks go through compress_and_transform with that codec: zlib
                                         level 6, hash-chain LZ4 / Snappy, zstd with predefined FSE sequences,
                                         each kept only when shorter than the literal-only stream (host code,
                                         sdb_host_codec.cpp; the data blocks: sdb_compress_blocks) */
    uint32_t pad;
} sdb_footer_in;
/* Writes the footer into out[0..cap) and its length into *len.  out == NULL: size query only.
 * cap too small: SDB_LIMIT_EXCEEDED (with *len set). */
sdb_status sdb_sst_footer(const sdb_footer_in *in, uint8_t *out, uint64_t cap, uint64_t *len);
/* Upper bound on the footer length (arithmetic only), to size `out` for a single sdb_sst_footer call. */
uint64_t sdb_sst_footer_bound(const sdb_footer_in *in);

/* ---------------------------------------------------------------------------------------------
 * Host entry points: device arena + pinned staging per handle (E2E path: H2D -> kernels -> D2H)
 * ------------------------------------------------------------------------------------------- */
typedef struct sdb_encoder sdb_encoder;

/* Host-memory view of one encoded SST (arrays owned by the encoder, valid until the next call). */
typedef struct sdb_sst_host_result {
    sdb_sst_summary summary;
    const uint8_t *data;
    const uint64_t *block_off;
    const uint32_t *block_first_entry;
    const uint32_t *index_key_len;
    const uint16_t *block_stats;
    const uint8_t *bloom;
    double h2d_ms, kernel_ms, d2h_ms;   /* hipEvent timings of the last call */
} sdb_sst_host_result;

sdb_encoder *sdb_encoder_create(int device, const sdb_sst_params *params);
void sdb_encoder_destroy(sdb_encoder *enc);
/* Encode a host batch; returns the first error (host-side or device-side). */
sdb_status sdb_encoder_encode_host(sdb_encoder *enc, const sdb_kv_batch *host_batch,
                                   sdb_sst_host_result *result);
/* Encode `count` host batches (the SSTs of one L0 flush or of a compaction's output, config.rs:
 * 1081, 1383-1390) with their transfers overlapped: SST i+1's marshal and H2D and SST i-1's D2H run
 * while SST i's kernels do (two slots of pinned staging, separate H2D / kernel / D2H streams).
 * results[i] views host memory owned by the encoder, valid until the next call; returns the first
 * SST status that is not SDB_OK (every SST is still attempted); the *_ms timings are 0. */
sdb_status sdb_encoder_encode_host_many(sdb_encoder *enc, uint32_t count, const sdb_kv_batch *host_batches,
                                        sdb_sst_host_result *results);

/* Mirror of EncodedSsTableBuilder's per-entry surface (sst_builder.rs:224-276,370-417). */
typedef struct sdb_sst_builder sdb_sst_builder;
sdb_sst_builder *sdb_sst_builder_new(int device, const sdb_sst_params *params);
void sdb_sst_builder_free(sdb_sst_builder *b);
/* add(entry): kind per SDB_KIND_*, timestamps present iff the has_* flags are non-zero. */
sdb_status sdb_sst_builder_add(sdb_sst_builder *b, const uint8_t *key, uint64_t key_len,
                               uint8_t kind, const uint8_t *val, uint64_t val_len, uint64_t seq,
                               int32_t has_create_ts, int64_t create_ts, int32_t has_expire_ts,
                               int64_t expire_ts);
/* build(): encode everything added so far on the GPU. */
sdb_status sdb_sst_builder_build(sdb_sst_builder *b, sdb_sst_host_result *result);

/* Host decode of encoded blocks (H2D, decode kernels, D2H).  Arrays owned by the handle. */
typedef struct sdb_decoder sdb_decoder;
typedef struct sdb_decode_host_result {
    sdb_decode_summary summary;
    const uint64_t *block_entry_start;
    const uint8_t *key_arena;
    const uint64_t *key_off;
    const uint64_t *val_off;
    const uint32_t *val_len;
    const uint64_t *seq;
    const uint8_t *flags;
    const int64_t *create_ts;
    const int64_t *expire_ts;
    const uint32_t *bad_block;
} sdb_decode_host_result;
sdb_decoder *sdb_decoder_create(int device);
void sdb_decoder_destroy(sdb_decoder *dec);
sdb_status sdb_decoder_decode_host(sdb_decoder *dec, const uint8_t *blocks,
                                   const uint64_t *block_off, uint64_t nblocks,
                                   uint16_t sst_version, sdb_decode_host_result *result);

/* ---------------------------------------------------------------------------------------------
 * Diagnostics (bench / profiling only)
 * ------------------------------------------------------------------------------------------- */
/* Stage timing of sdb_encode_sst: when enabled, hipEvents are recorded around each kernel stage
 * (bloom, k_facts, k_seg, k_anchor, k_blocks, k_emit, k_emit_big, bloom_fill).  sdb_diag_stage_times synchronises the
 * recorded events, writes the summed milliseconds per stage into ms[0..max_stages), the number of
 * encodes measured into *launches, clears the record, and returns the number of stages. */
void sdb_diag_enable_stage_timing(int on);
int sdb_diag_stage_times(double *ms, int max_stages, uint64_t *launches);
/* The block CRC32 (crc32fast::hash, the checksum compress_and_transform appends, format/sst.rs:541-552)
 * of n device ranges data[off[i], off[i+1]), 4 <= length <= 4096, one wave per range: method 0 the
 * slicing-by-8 wave CRC, 1 the matrix-core (MFMA) wave CRC the kernels use.  Results in out[0, n). */
sdb_status sdb_diag_crc32_blocks(const uint8_t *data, const uint64_t *off, uint64_t n, uint32_t *out, int method,
                                 void *stream);
/* One v_mfma_i32_32x32x32_i8 with lane-supplied operands (a, b: 64 lanes x 4 dwords; d: 64 x 16
 * dwords, lane-major): pins the operand / result lane maps the MFMA CRC relies on. */
sdb_status sdb_diag_mfma_i8(const int32_t *a, const int32_t *b, int32_t *d, void *stream);
/* A hand-written STREAM copy (16 bytes per lane, grid-stride) of `bytes` (a multiple of 16, 16-byte aligned):
 * bench.py's attainable-HBM ceiling beside the 8 TB/s spec. */
sdb_status sdb_diag_copy(void *dst, const void *src, uint64_t bytes, void *stream);
/* Bandwidth probes over `bytes` (a multiple of 4096, 16-byte aligned), wg_per_cu x CUs workgroups of 256
 * threads: mode 0 sdb_diag_copy, 1 the same copy with plain loads / stores, 2 a copy by 4 KiB per wave
 * and step, 3 read only, 4 write only. */
sdb_status sdb_diag_bw(void *dst, const void *src, uint64_t bytes, int mode, int wg_per_cu, void *stream);

/* Device query: number of visible HIP devices (0 on a machine without a GPU). */
int sdb_device_count(void);
/* Human-readable name of a status code. */
const char *sdb_status_name(int status);

#ifdef __cplusplus
}
#endif
#endif /* SLATEDB_AMD_H */
