"""ctypes mirror of include/slatedb_amd.h (the C ABI of libslatedb_amd.so).

Only plain C types cross this boundary; torch is used by callers merely to own device memory and
streams.  Struct layouts must stay byte-identical to the header (checked by tests/test_abi.py).
"""
import ctypes as C

SDB_OK = 0
SDB_EMPTY_KEY = 1
SDB_EMPTY_BLOCK = 2
SDB_CHECKSUM_MISMATCH = 3
SDB_INVALID_ROW_FLAGS = 4
SDB_INVALID_VERSION = 5
SDB_LIMIT_EXCEEDED = 6
SDB_UNSUPPORTED = 7
SDB_INVALID_ARGUMENT = 8
SDB_CORRUPT_BLOCK = 9
SDB_MERGE_OPERATOR_MISSING = 10
SDB_DECOMPRESSION_ERROR = 11
SDB_DEVICE_ERROR = 100
CODEC_NONE, CODEC_SNAPPY, CODEC_ZLIB, CODEC_LZ4, CODEC_ZSTD = 0, 1, 2, 3, 4  # CompressionFormat

STATUS_NAMES = {
    0: "OK", 1: "EMPTY_KEY", 2: "EMPTY_BLOCK", 3: "CHECKSUM_MISMATCH", 4: "INVALID_ROW_FLAGS",
    5: "INVALID_VERSION", 6: "LIMIT_EXCEEDED", 7: "UNSUPPORTED", 8: "INVALID_ARGUMENT",
    9: "CORRUPT_BLOCK", 10: "MERGE_OPERATOR_MISSING", 11: "DECOMPRESSION_ERROR", 100: "DEVICE_ERROR",
}

KIND_VALUE, KIND_MERGE, KIND_TOMBSTONE = 0, 1, 2
FLAG_TOMBSTONE, FLAG_HAS_EXPIRE_TS, FLAG_HAS_CREATE_TS, FLAG_MERGE_OPERAND = 1, 2, 4, 8
TS_CREATE, TS_EXPIRE = 1, 2

u8p = C.POINTER(C.c_uint8)
u16p = C.POINTER(C.c_uint16)
u32p = C.POINTER(C.c_uint32)
u64p = C.POINTER(C.c_uint64)
i64p = C.POINTER(C.c_int64)


class KvBatch(C.Structure):
    _fields_ = [
        ("n", C.c_uint64),
        ("key_bytes", C.c_void_p), ("key_off", C.c_void_p),
        ("val_bytes", C.c_void_p), ("val_off", C.c_void_p),
        ("kind", C.c_void_p), ("seq", C.c_void_p),
        ("create_ts", C.c_void_p), ("expire_ts", C.c_void_p), ("ts_mask", C.c_void_p),
        ("prefix_len", C.c_void_p),
    ]


class SstParams(C.Structure):
    _fields_ = [
        ("block_size", C.c_uint32), ("sst_version", C.c_uint16), ("restart_interval", C.c_uint16),
        ("bloom_bits_per_key", C.c_uint32), ("min_filter_keys", C.c_uint32), ("sst_type", C.c_uint32),
        ("prefix_kind", C.c_uint32), ("prefix_arg", C.c_uint32), ("no_whole_key", C.c_uint32),
    ]


class SstSummary(C.Structure):
    _fields_ = [
        ("data_len", C.c_uint64), ("num_blocks", C.c_uint64), ("num_entries", C.c_uint64),
        ("raw_key_size", C.c_uint64), ("raw_val_size", C.c_uint64),
        ("num_puts", C.c_uint64), ("num_deletes", C.c_uint64), ("num_merges", C.c_uint64),
        ("bloom_len", C.c_uint64), ("num_probes", C.c_uint32), ("filter_built", C.c_uint32),
        ("status", C.c_int32), ("max_block_entries", C.c_uint32), ("first_error_entry", C.c_uint64),
    ]


class SstOut(C.Structure):
    _fields_ = [
        ("data", C.c_void_p), ("data_cap", C.c_uint64),
        ("block_off", C.c_void_p), ("block_first_entry", C.c_void_p),
        ("index_key_len", C.c_void_p), ("block_stats", C.c_void_p), ("block_cap", C.c_uint64),
        ("bloom", C.c_void_p), ("bloom_cap", C.c_uint64),
        ("summary", C.c_void_p),
    ]


class DecodeSummary(C.Structure):
    _fields_ = [
        ("num_entries", C.c_uint64), ("key_bytes", C.c_uint64), ("num_bad_blocks", C.c_uint64),
        ("status", C.c_int32), ("pad", C.c_uint32),
    ]


class DecodedOut(C.Structure):
    _fields_ = [
        ("block_entry_start", C.c_void_p),
        ("key_arena", C.c_void_p), ("key_arena_cap", C.c_uint64), ("key_off", C.c_void_p),
        ("val_off", C.c_void_p), ("val_len", C.c_void_p), ("seq", C.c_void_p),
        ("flags", C.c_void_p), ("create_ts", C.c_void_p), ("expire_ts", C.c_void_p),
        ("cap_entries", C.c_uint64),
        ("bad_block", C.c_void_p), ("bad_cap", C.c_uint64),
        ("summary", C.c_void_p),
    ]


class SstHostResult(C.Structure):
    _fields_ = [
        ("summary", SstSummary),
        ("data", C.c_void_p), ("block_off", C.c_void_p), ("block_first_entry", C.c_void_p),
        ("index_key_len", C.c_void_p), ("block_stats", C.c_void_p), ("bloom", C.c_void_p),
        ("h2d_ms", C.c_double), ("kernel_ms", C.c_double), ("d2h_ms", C.c_double),
    ]


class DecodeHostResult(C.Structure):
    _fields_ = [
        ("summary", DecodeSummary),
        ("block_entry_start", C.c_void_p), ("key_arena", C.c_void_p), ("key_off", C.c_void_p),
        ("val_off", C.c_void_p), ("val_len", C.c_void_p), ("seq", C.c_void_p), ("flags", C.c_void_p),
        ("create_ts", C.c_void_p), ("expire_ts", C.c_void_p), ("bad_block", C.c_void_p),
    ]


class FooterIn(C.Structure):
    _fields_ = [
        ("sst_version", C.c_uint16), ("sst_type", C.c_uint8), ("has_filter", C.c_uint8),
        ("num_probes", C.c_uint32), ("data_len", C.c_uint64), ("num_blocks", C.c_uint64),
        ("block_off", C.c_void_p), ("first_key_bytes", C.c_void_p), ("first_key_off", C.c_void_p),
        ("first_entry", C.c_char_p), ("first_entry_len", C.c_uint64),
        ("last_entry", C.c_char_p), ("last_entry_len", C.c_uint64),
        ("stats", C.c_void_p), ("block_stats", C.c_void_p), ("bloom", C.c_void_p),
        ("bloom_len", C.c_uint64), ("filter_name", C.c_char_p), ("compression", C.c_uint32), ("pad", C.c_uint32),
    ]


class SstView(C.Structure):
    _fields_ = [
        ("data", C.c_void_p), ("block_off", C.c_void_p), ("num_blocks", C.c_uint64),
        ("index_keys", C.c_void_p), ("index_key_off", C.c_void_p),
        ("bloom", C.c_void_p), ("bloom_len", C.c_uint64), ("num_probes", C.c_uint32),
        ("sst_version", C.c_uint16), ("pad", C.c_uint16),
    ]


class LookupOut(C.Structure):
    _fields_ = [
        ("state", C.c_void_p), ("status", C.c_void_p), ("block", C.c_void_p), ("entry", C.c_void_p),
        ("key_len", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p), ("seq", C.c_void_p),
        ("flags", C.c_void_p), ("create_ts", C.c_void_p), ("expire_ts", C.c_void_p),
    ]


class Run(C.Structure):
    _fields_ = [
        ("n", C.c_uint64), ("key_arena", C.c_void_p), ("key_off", C.c_void_p),
        ("val_base", C.c_void_p), ("val_off", C.c_void_p), ("val_len", C.c_void_p),
        ("seq", C.c_void_p), ("flags", C.c_void_p), ("create_ts", C.c_void_p), ("expire_ts", C.c_void_p),
    ]


MAX_RUNS = 32
U64_MAX = (1 << 64) - 1


class Retention(C.Structure):
    _fields_ = [
        ("min_seq", C.c_uint64), ("time_seq", C.c_uint64), ("compaction_start_ts", C.c_int64),
        ("has_min_seq", C.c_uint8), ("has_time_window", C.c_uint8), ("filter_tombstone", C.c_uint8),
        ("merge_operands", C.c_uint8), ("pad", C.c_uint32),
    ]


class MergeSummary(C.Structure):
    _fields_ = [
        ("num_in", C.c_uint64), ("num_out", C.c_uint64), ("key_bytes", C.c_uint64), ("val_bytes", C.c_uint64),
        ("expired_values", C.c_uint64), ("expired_merges", C.c_uint64),
        ("status", C.c_int32), ("pad", C.c_uint32), ("first_error_entry", C.c_uint64),
    ]


class MergedOut(C.Structure):
    _fields_ = [
        ("key_bytes", C.c_void_p), ("key_cap", C.c_uint64), ("key_off", C.c_void_p),
        ("val_bytes", C.c_void_p), ("val_cap", C.c_uint64), ("val_off", C.c_void_p),
        ("kind", C.c_void_p), ("seq", C.c_void_p), ("create_ts", C.c_void_p), ("expire_ts", C.c_void_p),
        ("ts_mask", C.c_void_p), ("cap_entries", C.c_uint64), ("summary", C.c_void_p),
    ]


class CompactedSst(C.Structure):
    _fields_ = [
        ("entry_start", C.c_uint64), ("entry_end", C.c_uint64),
        ("data", C.c_void_p), ("block_off", C.c_void_p), ("block_first_entry", C.c_void_p),
        ("index_key_len", C.c_void_p), ("block_stats", C.c_void_p), ("bloom", C.c_void_p),
        ("summary", SstSummary),
    ]


class CompactionInput(C.Structure):
    _fields_ = [
        ("data", C.c_void_p), ("block_off", C.c_void_p), ("num_blocks", C.c_uint64), ("num_entries", C.c_uint64),
        ("key_bytes", C.c_uint64), ("val_bytes", C.c_uint64),
    ]



DECODE_DESCENDING = 1
DECODE_FAIL_FAST = 2  # SDB_DECODE_FAIL_FAST

LOOKUP_FILTERED, LOOKUP_EXHAUSTED, LOOKUP_POSITIONED, LOOKUP_FOUND = 0, 1, 2, 3

SST_COMPACTED, SST_WAL = 0, 1


# Every symbol include/slatedb_amd.h declares, with its ctypes signature.
SIGNATURES = {
    "sdb_abi_version": (C.c_uint32, []),
    "sdb_encode_bounds": (C.c_int, [C.c_uint64, C.c_uint64, C.c_uint64, C.POINTER(SstParams),
                                    u64p, u64p, u64p]),
    "sdb_encode_workspace_bytes": (C.c_uint64, [C.c_uint64, C.POINTER(SstParams)]),
    "sdb_bloom_filter_bytes": (C.c_uint64, [C.c_uint64, C.c_uint32]),
    "sdb_bloom_num_probes": (C.c_uint32, [C.c_uint32]),
    "sdb_encode_sst": (C.c_int, [C.POINTER(KvBatch), C.POINTER(SstParams), C.POINTER(SstOut),
                                 C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_encode_ssts_workspace_bytes": (C.c_uint64, [C.c_uint32, C.POINTER(KvBatch), C.POINTER(SstParams)]),
    "sdb_encode_ssts": (C.c_int, [C.c_uint32, C.POINTER(KvBatch), C.POINTER(SstParams), C.POINTER(SstOut),
                                  C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_bloom_workspace_bytes": (C.c_uint64, [C.c_uint64, C.c_uint32]),
    "sdb_bloom_build": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                  C.c_uint64, C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_bloom_prefix_workspace_bytes": (C.c_uint64, [C.c_uint64]),
    "sdb_bloom_build_prefix": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32,
                                         C.c_uint32, C.c_uint32, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                         C.c_uint64, C.c_void_p]),
    "sdb_bloom_might_match": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_uint32, C.c_uint32, C.c_uint32,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p,
                                        C.c_void_p]),
    "sdb_bloom_might_contain": (C.c_int, [C.c_void_p, C.c_uint64, C.c_uint32, C.c_void_p,
                                          C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p]),
    "sdb_decode_workspace_bytes": (C.c_uint64, [C.c_uint64]),
    "sdb_decode_blocks": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint16,
                                    C.POINTER(DecodedOut), C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_decode_blocks_at": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint16,
                                       C.POINTER(DecodedOut), C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_decode_blocks_ex": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint16, C.c_uint32,
                                       C.POINTER(DecodedOut), C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_decompress_workspace_bytes": (C.c_uint64, [C.c_uint64]),
    "sdb_decompress_plan": (C.c_int, [C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_void_p,
                                      C.c_uint64, C.c_void_p]),
    "sdb_decompress_blocks": (C.c_int, [C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_uint64,
                                        C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sdb_decompress_once_workspace_bytes": (C.c_uint64, [C.c_uint64]),
    "sdb_decompress_blocks_once": (C.c_int, [C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                             C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                             C.c_void_p]),
    "sdb_sst_lookup_workspace_bytes": (C.c_uint64, [C.c_uint64, C.c_uint64]),
    "sdb_sst_lookup": (C.c_int, [C.POINTER(SstView), C.c_void_p, C.c_void_p, C.c_uint64, C.c_int32,
                                 C.POINTER(LookupOut), C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_merge_runs_workspace_bytes": (C.c_uint64, [C.POINTER(Run), C.c_uint32]),
    "sdb_merge_runs": (C.c_int, [C.POINTER(Run), C.c_uint32, C.POINTER(Retention), C.POINTER(MergedOut),
                                 C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_sst_cuts_workspace_bytes": (C.c_uint64, [C.c_uint64, C.POINTER(SstParams)]),
    "sdb_sst_cuts": (C.c_int, [C.POINTER(KvBatch), C.POINTER(SstParams), C.c_uint64, C.c_void_p, C.c_uint64,
                               C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_compactor_create": (C.c_void_p, [C.c_int]),
    "sdb_compactor_destroy": (None, [C.c_void_p]),
    "sdb_compactor_run": (C.c_int, [C.c_void_p, C.POINTER(Run), C.c_uint32, C.POINTER(Retention),
                                    C.POINTER(SstParams), C.c_uint64, C.c_void_p, u32p]),
    "sdb_compactor_run_ssts": (C.c_int, [C.c_void_p, C.POINTER(CompactionInput), C.c_uint32, u32p, C.c_uint32,
                                         C.c_uint16, C.POINTER(Retention), C.POINTER(SstParams), C.c_uint64,
                                         C.c_void_p, u32p]),
    "sdb_compactor_sst": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(CompactedSst)]),
    "sdb_compactor_merged": (C.c_int, [C.c_void_p, C.POINTER(KvBatch), C.POINTER(MergeSummary)]),
    "sdb_sst_footer": (C.c_int, [C.POINTER(FooterIn), C.c_void_p, C.c_uint64, u64p]),
    "sdb_sst_footer_bound": (C.c_uint64, [C.POINTER(FooterIn)]),
    "sdb_encoder_create": (C.c_void_p, [C.c_int, C.POINTER(SstParams)]),
    "sdb_encoder_destroy": (None, [C.c_void_p]),
    "sdb_encoder_encode_host": (C.c_int, [C.c_void_p, C.POINTER(KvBatch), C.POINTER(SstHostResult)]),
    "sdb_encoder_encode_host_many": (C.c_int, [C.c_void_p, C.c_uint32, C.POINTER(KvBatch), C.POINTER(SstHostResult)]),
    "sdb_sst_builder_new": (C.c_void_p, [C.c_int, C.POINTER(SstParams)]),
    "sdb_sst_builder_free": (None, [C.c_void_p]),
    "sdb_sst_builder_add": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint8, C.c_void_p,
                                      C.c_uint64, C.c_uint64, C.c_int32, C.c_int64, C.c_int32,
                                      C.c_int64]),
    "sdb_sst_builder_build": (C.c_int, [C.c_void_p, C.POINTER(SstHostResult)]),
    "sdb_decoder_create": (C.c_void_p, [C.c_int]),
    "sdb_decoder_destroy": (None, [C.c_void_p]),
    "sdb_decoder_decode_host": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64,
                                          C.c_uint16, C.POINTER(DecodeHostResult)]),
    "sdb_diag_enable_stage_timing": (None, [C.c_int]),
    "sdb_diag_stage_times": (C.c_int, [C.POINTER(C.c_double), C.c_int, u64p]),
    "sdb_diag_crc32_blocks": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p, C.c_int, C.c_void_p]),
    "sdb_diag_mfma_i8": (C.c_int, [C.c_void_p, C.c_void_p, C.c_void_p, C.c_void_p]),
    "sdb_diag_copy": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_diag_bw": (C.c_int, [C.c_void_p, C.c_void_p, C.c_uint64, C.c_int, C.c_int, C.c_void_p]),
    "sdb_set_concurrent_builders": (C.c_int, [C.c_uint32]),
    "sdb_compress_workspace_bytes": (C.c_uint64, [C.c_uint64, C.c_uint64]),
    "sdb_compress_blocks": (C.c_int, [C.c_uint32, C.c_void_p, C.c_void_p, C.c_uint64, C.c_uint64, C.c_void_p,
                                      C.c_uint64, C.c_void_p, C.c_void_p, C.c_void_p, C.c_uint64, C.c_void_p]),
    "sdb_device_count": (C.c_int, []),
    "sdb_status_name": (C.c_char_p, [C.c_int]),
}


STAGES = ["bloom", "facts", "seg", "anchor", "blocks", "emit", "emit_big", "bloom_fill"]  # k_anchor, k_blocks (round 5 on); emit = k_emit alone


def bind(lib, partial=False):
    """Sets restype/argtypes on every entry point. ``partial`` (diagnostic
    variant libraries picked with SDB_LIBRARY, possibly built from an older
    tree) skips symbols the library does not export instead of failing."""
    for name, (res, args) in SIGNATURES.items():
        fn = getattr(lib, name, None) if partial else getattr(lib, name)
        if fn is None:
            continue
        fn.restype = res
        fn.argtypes = args
    return lib
