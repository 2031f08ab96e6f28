// sdb_compactor.cpp — host orchestration of one compaction job on the device (sdb_compactor_*):
// CompactionExecutor::run_subcompaction_merge's output side (compactor_executor.rs:818-871) as
//   merge + retention (sized, then emitted) -> SST cuts -> sdb_encode_ssts over the cut ranges,
// with three host synchronisations (merged sizes, cut count, SST summaries).  The outputs stay in
// the handle's device memory; every SST of the job is encoded by one launch sequence per 8 SSTs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/slatedb_amd.h"
#include "sdb_compact.h"

using namespace sdb;

namespace {

struct DevBuf {
    void *p = nullptr;
    uint64_t cap = 0;
    bool ensure(uint64_t bytes) {
        if (bytes <= cap && p) return true;
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
        const uint64_t c = bytes + bytes / 4 + 256;
        if (hipMalloc(&p, c) != hipSuccess) {
            p = nullptr;
            return false;
        }
        cap = c;
        return true;
    }
    void release() {
        if (p) (void)hipFree(p);
        p = nullptr;
        cap = 0;
    }
    template <typename T>
    T *at(uint64_t off) const {
        return reinterpret_cast<T *>(reinterpret_cast<uint8_t *>(p) + off);
    }
};

uint64_t al256(uint64_t x) { return (x + 255) & ~255ull; }

}  // namespace

struct sdb_compactor {
    int device = 0;
    DevBuf merge_ws, cols, keys, vals, cut_ws, cuts, sst_meta, sst_data, sst_bloom, enc_ws;
    sdb_kv_batch merged{};
    sdb_merge_summary msum{};
    std::vector<sdb_compacted_sst> ssts;
    ~sdb_compactor() {
        (void)hipSetDevice(device);
        for (DevBuf *b : {&merge_ws, &cols, &keys, &vals, &cut_ws, &cuts, &sst_meta, &sst_data, &sst_bloom, &enc_ws})
            b->release();
    }
};

extern "C" {

sdb_compactor *sdb_compactor_create(int device) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || device < 0 || device >= n) return nullptr;
    sdb_compactor *c = new sdb_compactor();
    c->device = device;
    return c;
}

void sdb_compactor_destroy(sdb_compactor *c) { delete c; }

sdb_status sdb_compactor_run(sdb_compactor *c, const sdb_run *runs, uint32_t nruns, const sdb_retention *ret,
                             const sdb_sst_params *params, uint64_t max_sst_size, void *stream, uint32_t *num_ssts) {
    if (!c || !params || !num_ssts) return SDB_INVALID_ARGUMENT;
    *num_ssts = 0;
    c->ssts.clear();
    c->merged = sdb_kv_batch{};
    c->msum = sdb_merge_summary{};
    if (params->sst_type != SDB_SST_COMPACTED) return SDB_INVALID_ARGUMENT;  // compactions write compacted SSTs
    if (hipSetDevice(c->device) != hipSuccess) return SDB_DEVICE_ERROR;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint64_t total = 0;
    for (uint32_t r = 0; r < nruns && runs; r++) total += runs[r].n;

    // 1. merge + retention, sized with unbounded byte capacities, then emitted
    const uint64_t o_koff = 0, o_voff = al256(8 * (total + 1)), o_kind = o_voff + al256(8 * (total + 1));
    const uint64_t o_seq = o_kind + al256(total + 1), o_cts = o_seq + al256(8 * (total + 1));
    const uint64_t o_ets = o_cts + al256(8 * (total + 1)), o_mask = o_ets + al256(8 * (total + 1));
    const uint64_t o_sum = o_mask + al256(total + 1), cols_bytes = o_sum + al256(sizeof(sdb_merge_summary));
    if (!c->cols.ensure(cols_bytes)) return SDB_DEVICE_ERROR;
    sdb_merged_out out{};
    out.key_cap = ~0ull;
    out.key_off = c->cols.at<uint64_t>(o_koff);
    out.val_cap = ~0ull;
    out.val_off = c->cols.at<uint64_t>(o_voff);
    out.kind = c->cols.at<uint8_t>(o_kind);
    out.seq = c->cols.at<uint64_t>(o_seq);
    out.create_ts = c->cols.at<int64_t>(o_cts);
    out.expire_ts = c->cols.at<int64_t>(o_ets);
    out.ts_mask = c->cols.at<uint8_t>(o_mask);
    out.cap_entries = total;
    out.summary = c->cols.at<sdb_merge_summary>(o_sum);
    const uint64_t mws = sdb_merge_runs_workspace_bytes(runs, nruns);
    if (!c->merge_ws.ensure(mws)) return SDB_DEVICE_ERROR;
    MergeArgs a;
    sdb_status st = build_merge_args(runs, nruns, ret, &out, c->merge_ws.p, c->merge_ws.cap, &a);
    if (st) return st;
    if (launch_merge(a, false, s) != hipSuccess) return SDB_DEVICE_ERROR;
    if (hipMemcpyAsync(&c->msum, out.summary, sizeof(sdb_merge_summary), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return SDB_DEVICE_ERROR;
    if (c->msum.status) return (sdb_status)c->msum.status;
    if (!c->keys.ensure(c->msum.key_bytes + 16) || !c->vals.ensure(c->msum.val_bytes + 16)) return SDB_DEVICE_ERROR;
    a.out.key_bytes = c->keys.at<uint8_t>(0);
    a.out.key_cap = c->msum.key_bytes;
    a.out.val_bytes = c->vals.at<uint8_t>(0);
    a.out.val_cap = c->msum.val_bytes;
    if (launch_merge_emit(a, s) != hipSuccess) return SDB_DEVICE_ERROR;
    const uint64_t n = c->msum.num_out;
    sdb_kv_batch &m = c->merged;
    m.n = n;
    m.key_bytes = a.out.key_bytes;
    m.key_off = out.key_off;
    m.val_bytes = a.out.val_bytes;
    m.val_off = out.val_off;
    m.kind = out.kind;
    m.seq = out.seq;
    m.create_ts = out.create_ts;
    m.expire_ts = out.expire_ts;
    m.ts_mask = out.ts_mask;
    m.prefix_len = nullptr;
    if (!n) return hipStreamSynchronize(s) == hipSuccess ? SDB_OK : SDB_DEVICE_ERROR;

    // 2. cuts (and the byte offsets of every cut, to size the SSTs)
    const uint64_t cws = sdb_sst_cuts_workspace_bytes(n, params);
    const uint64_t o_num = 0, o_cut = 256, o_off = o_cut + al256(8 * (n + 2));
    if (!c->cut_ws.ensure(cws) || !c->cuts.ensure(o_off + al256(16 * (n + 2)))) return SDB_DEVICE_ERROR;
    uint64_t *d_num = c->cuts.at<uint64_t>(o_num), *d_cut = c->cuts.at<uint64_t>(o_cut);
    uint64_t *d_off = c->cuts.at<uint64_t>(o_off);
    st = sdb_sst_cuts(&m, params, max_sst_size, d_cut, n + 1, d_num, c->cut_ws.p, c->cut_ws.cap, stream);
    if (st) return st;
    // the cut count, the cuts and their byte offsets in one synchronisation: every SST but the last holds
    // more than max_sst_size bytes of blocks, and a block costs at most its keys, values and 64 bytes
    // per row, so g bounds the count (a larger one takes a second copy)
    const uint64_t g = max_sst_size ? std::min<uint64_t>(n, 2 + (c->msum.key_bytes + c->msum.val_bytes + 64 * n) / max_sst_size) : n;
    uint64_t ns = 0;
    std::vector<uint64_t> cut(g + 1), off(2 * (g + 1));
    if (launch_cut_offsets(d_cut, d_num, m.key_off, m.val_off, d_off, s) != hipSuccess ||
        hipMemcpyAsync(&ns, d_num, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(cut.data(), d_cut, 8 * (g + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipMemcpyAsync(off.data(), d_off, 16 * (g + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return SDB_DEVICE_ERROR;
    if (ns == 0 || ns > n) return SDB_DEVICE_ERROR;
    if (ns > g) {
        cut.resize(ns + 1);
        off.resize(2 * (ns + 1));
        if (hipMemcpyAsync(cut.data(), d_cut, 8 * (ns + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipMemcpyAsync(off.data(), d_off, 16 * (ns + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return SDB_DEVICE_ERROR;
    }

    // 3. encode every output SST (sets of up to 8 per launch sequence)
    std::vector<sdb_kv_batch> batches(ns);
    std::vector<sdb_sst_out> outs(ns);
    std::vector<uint64_t> data_at(ns), bloom_at(ns), meta_at(ns);
    uint64_t data_total = 0, bloom_total = 0, meta_total = al256(ns * sizeof(sdb_sst_summary));
    for (uint64_t i = 0; i < ns; i++) {
        const uint64_t b = cut[i], e = cut[i + 1], ni = e - b;
        sdb_kv_batch &x = batches[i];
        x = m;
        x.n = ni;
        x.key_off = m.key_off + b;
        x.val_off = m.val_off + b;
        x.kind = m.kind + b;
        x.seq = m.seq + b;
        x.create_ts = m.create_ts + b;
        x.expire_ts = m.expire_ts + b;
        x.ts_mask = m.ts_mask + b;
        uint64_t dcap = 0, bcap = 0, fcap = 0;
        st = sdb_encode_bounds(ni, off[2 * (i + 1)] - off[2 * i], off[2 * (i + 1) + 1] - off[2 * i + 1], params, &dcap,
                               &bcap, &fcap);
        if (st) return st;
        outs[i].data_cap = dcap;
        outs[i].block_cap = bcap;
        outs[i].bloom_cap = fcap;
        data_at[i] = data_total;
        data_total += al256(dcap);
        bloom_at[i] = bloom_total;
        bloom_total += al256(fcap);
        meta_at[i] = meta_total;
        meta_total += al256(8 * (bcap + 1)) + al256(4 * (bcap + 1)) + al256(4 * bcap) + al256(6 * bcap);
    }
    if (!c->sst_data.ensure(data_total) || !c->sst_bloom.ensure(bloom_total) || !c->sst_meta.ensure(meta_total))
        return SDB_DEVICE_ERROR;
    for (uint64_t i = 0; i < ns; i++) {
        sdb_sst_out &o = outs[i];
        const uint64_t bcap = o.block_cap;
        uint64_t q = meta_at[i];
        o.data = c->sst_data.at<uint8_t>(data_at[i]);
        o.bloom = c->sst_bloom.at<uint8_t>(bloom_at[i]);
        o.block_off = c->sst_meta.at<uint64_t>(q);
        q += al256(8 * (bcap + 1));
        o.block_first_entry = c->sst_meta.at<uint32_t>(q);
        q += al256(4 * (bcap + 1));
        o.index_key_len = c->sst_meta.at<uint32_t>(q);
        q += al256(4 * bcap);
        o.block_stats = c->sst_meta.at<uint16_t>(q);
        o.summary = c->sst_meta.at<sdb_sst_summary>(i * sizeof(sdb_sst_summary));
    }
    const uint64_t ews = sdb_encode_ssts_workspace_bytes((uint32_t)ns, batches.data(), params);
    if (!c->enc_ws.ensure(ews)) return SDB_DEVICE_ERROR;
    st = sdb_encode_ssts((uint32_t)ns, batches.data(), params, outs.data(), c->enc_ws.p, c->enc_ws.cap, stream);
    if (st) return st;
    std::vector<sdb_sst_summary> sums(ns);
    if (hipMemcpyAsync(sums.data(), c->sst_meta.p, ns * sizeof(sdb_sst_summary), hipMemcpyDeviceToHost, s) != hipSuccess ||
        hipStreamSynchronize(s) != hipSuccess)
        return SDB_DEVICE_ERROR;
    c->ssts.resize(ns);
    sdb_status first = SDB_OK;
    for (uint64_t i = 0; i < ns; i++) {
        sdb_compacted_sst &v = c->ssts[i];
        v.entry_start = cut[i];
        v.entry_end = cut[i + 1];
        v.data = outs[i].data;
        v.block_off = outs[i].block_off;
        v.block_first_entry = outs[i].block_first_entry;
        v.index_key_len = outs[i].index_key_len;
        v.block_stats = outs[i].block_stats;
        v.bloom = outs[i].bloom;
        v.summary = sums[i];
        if (!first && sums[i].status) first = (sdb_status)sums[i].status;
    }
    *num_ssts = (uint32_t)ns;
    return first;
}

sdb_status sdb_compactor_sst(const sdb_compactor *c, uint32_t i, sdb_compacted_sst *out) {
    if (!c || !out || i >= c->ssts.size()) return SDB_INVALID_ARGUMENT;
    *out = c->ssts[i];
    return SDB_OK;
}

sdb_status sdb_compactor_merged(const sdb_compactor *c, sdb_kv_batch *batch, sdb_merge_summary *summary) {
    if (!c) return SDB_INVALID_ARGUMENT;
    if (batch) *batch = c->merged;
    if (summary) *summary = c->msum;
    return SDB_OK;
}

}  // extern "C"
