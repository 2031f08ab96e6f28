/*
 * sdb_oracle.h — CPU restatement of slatedb's SST codec + bloom builder.
 *
 * TEST INFRASTRUCTURE ONLY.  Nothing in slatedb_amd/ links or calls this; it is the checker used by
 * tests/, __graft_entry__.smoke() and bench.py's cpu_baseline leg.  Every function cites the
 * reference file:line it restates (paths relative to /root/reference/slatedb/src).
 */
#ifndef SDB_ORACLE_H
#define SDB_ORACLE_H
#include <stddef.h>
#include <stdint.h>
#include "../include/slatedb_amd.h"

#ifdef __cplusplus
extern "C" {
#endif

uint32_t orc_varint_len(uint32_t v);                                   /* utils.rs:638-645 */
size_t orc_encode_varint(uint8_t *out, uint32_t v);                    /* utils.rs:609-615 */
uint32_t orc_crc32(const uint8_t *p, size_t n);                        /* crc32fast::hash */
uint64_t orc_siphash(const uint8_t *p, size_t n, uint64_t k0, uint64_t k1, int c, int d);
uint64_t orc_filter_hash(const uint8_t *p, size_t n);                  /* filter.rs:196-204 */
void orc_probes_for_key(uint64_t h, uint16_t k, uint32_t m, uint32_t *out); /* filter.rs:206-221 */
uint16_t orc_optimal_num_probes(uint32_t bpk);                         /* filter.rs:235-239 */
uint64_t orc_filter_size_bytes(uint64_t num_keys, uint32_t bpk);       /* filter.rs:65-69 */
size_t orc_compute_prefix(const uint8_t *a, size_t na, const uint8_t *b, size_t nb); /* block_v2.rs:52-75 */
/* compute_index_key (utils.rs:198-226).  Returns index-key length, or -1 where the reference panics. */
int64_t orc_index_key_len(const uint8_t *prev, size_t nprev, int has_prev, const uint8_t *first,
                          size_t nfirst);

size_t orc_encode_row(uint16_t version, uint32_t shared, const uint8_t *suffix, size_t suffix_len,
                      uint8_t kind, const uint8_t *val, size_t vlen, uint64_t seq, int has_create,
                      int64_t create_ts, int has_expire, int64_t expire_ts, uint8_t *out, size_t cap);

/* Build ONE block from entries [0, batch->n) in order (BlockBuilder V1/V2 add(); entries that do not
 * fit are skipped exactly like `let _ = builder.add(e)`).  Writes Block::encode() bytes
 * (format/block.rs:17-26), no CRC.  accepted[i] = 1 if entry i was added (may be NULL). */
sdb_status orc_build_block(const sdb_kv_batch *batch, uint16_t version, uint32_t block_size,
                           uint16_t restart_interval, uint8_t *out, uint64_t cap, uint64_t *len,
                           uint8_t *accepted);

/* EncodedSsTableBuilder::{add, finish_block, build} data section + bloom (sst_builder.rs:224-417).
 * Host pointers; same output contract as sdb_encode_sst.  `summary` is written directly. */
sdb_status orc_encode_sst(const sdb_kv_batch *batch, const sdb_sst_params *params,
                          const sdb_sst_out *out);

/* Bloom bitmap (filter.rs:71-90) over keys. */
sdb_status orc_bloom_build(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n,
                           uint32_t bpk, uint8_t *bitmap, uint64_t bitmap_bytes);
sdb_status orc_bloom_build_range(const uint8_t *key_bytes, const uint64_t *key_off, uint64_t n, uint64_t lo,
                                 uint64_t hi, uint32_t bpk, uint8_t *bitmap, uint64_t bitmap_bytes);
int orc_bloom_might_contain(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes,
                            const uint8_t *key, size_t klen);
/* Prefix filters (filter.rs:40-90, 149-175; prefix_extractor.rs:41-95). */
int64_t orc_prefix_len(uint32_t kind, uint32_t arg, const uint8_t *key, size_t klen, int64_t given);
sdb_status orc_bloom_build_prefix(const uint8_t *key_bytes, const uint64_t *key_off, const int32_t *plens,
                                  uint64_t n, uint32_t bpk, uint32_t kind, uint32_t arg, int whole,
                                  uint8_t *bitmap, uint64_t cap, uint64_t *len);
int orc_bloom_might_match(const uint8_t *bitmap, uint64_t bitmap_bytes, uint32_t num_probes, int whole,
                          uint32_t kind, uint32_t arg, const uint8_t *q, size_t qn, int is_prefix,
                          int64_t given);

/* SsTableFormat::decompress (format/sst.rs:884-917) for the two LZ-family codecs, restated from their
 * format specifications: codec 3 = lz4_flex 0.11.6 block::decompress_size_prepended (u32 LE size, then
 * an LZ4 block), codec 1 = snap 1.1.1 raw::Decoder::decompress_vec (varint size, then Snappy
 * elements).  orc_decompressed_len: the declared length (-1: bad header / other codec). */
int64_t orc_decompressed_len(uint32_t codec, const uint8_t *in, size_t n);
sdb_status orc_decompress(uint32_t codec, const uint8_t *in, size_t n, uint8_t *out, size_t cap, size_t *out_len);
/* decode_block's first half over a block run (format/sst.rs:980-999): validate_checksum over the stored
 * bytes, decompress, then the block re-framed with the CRC32 of its uncompressed bytes, so that
 * [out_start[k], out_end[k]) is a plain block for orc_decode_blocks / sdb_decode_blocks_at.  out_start
 * (nblocks+1) is the plan: slots of declared length + 4 (0 for an unreadable header or one over 64 MiB).
 * *first_err: (block << 8 | status) of the first failing block (~0: none); a failing block is empty. */
sdb_status orc_decompress_blocks(uint32_t codec, const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                 uint8_t *out, uint64_t out_cap, uint64_t *out_start, uint64_t *out_end,
                                 uint64_t *first_err);

/* read_blocks/decode_block + DataBlockIterator (format/sst.rs:938-1038, block_iterator*.rs). */
sdb_status orc_decode_blocks(const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                             uint16_t sst_version, const sdb_decoded_out *out);

/* The same blocks in descending iteration order (SstIterator Descending over
 * DescendingBlockIteratorV2 / BlockIterator Descending); block_entry_start keeps the ascending
 * prefix of the per-block counts (block k's entries: [N - bes[k + 1], N - bes[k])). */
sdb_status orc_decode_blocks_desc(const uint8_t *blocks, const uint64_t *block_off, uint64_t nblocks,
                                  uint16_t sst_version, const sdb_decoded_out *out);

/* Point lookups on one SST (host pointers in `sst`): the same contract as sdb_sst_lookup, following
 * filter.rs:124-136, partitioned_keyspace.rs:16-110, sst_iter.rs:501-516, block_iterator_v2.rs:
 * 138-469 and block_iterator.rs:130-190 literally (materialised keys). */
sdb_status orc_sst_lookup(const sdb_sst_view *sst, const uint8_t *key_bytes, const uint64_t *key_off,
                          uint64_t nkeys, int descending, const sdb_lookup_out *out);

/* Compaction output side over host runs: MergeIterator (merge_iterator.rs:55-69, dedup off) ->
 * MergeOperatorRequiredIterator (merge_operator.rs:213-223) -> RetentionIterator
 * (retention_iterator.rs:91-204, 381-398); the same contract as sdb_merge_runs. */
sdb_status orc_merge_runs(const sdb_run *runs, uint32_t nruns, const sdb_retention *ret, const sdb_merged_out *out);
/* Output SST boundaries by EncodedSsTableWriter::add and the compactor's max_sst_size rule
 * (compactor_executor.rs:833-858, sst_builder.rs:224-325); the same contract as sdb_sst_cuts. */
sdb_status orc_sst_cuts(const sdb_kv_batch *batch, const sdb_sst_params *p, uint64_t max_sst_size,
                        uint64_t *cut_start, uint64_t cap, uint64_t *num_ssts);

#ifdef __cplusplus
}
#endif
#endif
