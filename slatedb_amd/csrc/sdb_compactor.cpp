// sdb_compactor.cpp — host orchestration of one compaction job on the device (sdb_compactor_*):
// CompactionExecutor::run_subcompaction_merge (compactor_executor.rs:327-390 load_iterators, 818-871
// the output side) as
//   sdb_compactor_run:       merge + retention (sized, then emitted) -> SST cuts -> sdb_encode_ssts over
//                            the cut ranges; three host synchronisations (merged sizes, cuts, summaries);
//   sdb_compactor_run_ssts:  decode of every input SST's blocks (one launch sequence) -> gate -> merge +
//                            retention + emit into buffers sized by the inputs' SstStats -> SST cuts over the
//                            merged stream padded to the input count -> sdb_encode_ssts; two host
//                            synchronisations (merged count + cuts together, summaries).
// The outputs stay in the handle's device memory; every SST of the job is encoded by one launch sequence
// per 8 SSTs.
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include <algorithm>
#include <vector>

#include "../../include/slatedb_amd.h"
#include "sdb_compact.h"
#include "sdb_decode.h"

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

struct PinBuf {  // pinned host staging (async device -> host copies)
    void *p = nullptr;
    uint64_t cap = 0;
    PinBuf() = default;
    PinBuf(const PinBuf &) = delete;
    PinBuf &operator=(const PinBuf &) = delete;
    bool ensure(uint64_t bytes) {
        if (bytes <= cap && p) return true;
        release();
        const uint64_t c = bytes + bytes / 4 + 256;
        if (hipHostMalloc(&p, c, hipHostMallocDefault) != hipSuccess) {
            p = nullptr;
            return false;
        }
        cap = c;
        return true;
    }
    void release() {
        if (p) (void)hipHostFree(p);
        p = nullptr;
        cap = 0;
    }
};

struct GroupBufs {  // a group of runs merged ahead of the job (runs beyond SDB_MAX_RUNS)
    DevBuf cols, keys, vals, asrun;
};

struct sdb_compactor {
    int device = 0;
    DevBuf merge_ws, cols, keys, vals, cut_ws, cuts, sst_meta, sst_data, sst_bloom, enc_ws, dec, dec_ws, cx_tab;
    std::vector<GroupBufs> groups;
    PinBuf pin, pin_tab;
    // recorded on the job's stream when a run_ssts job returns (every path): the next job waits for it
    // before it rewrites pin_tab / cx_tab, which that job's upload and kernels may still be reading
    hipEvent_t tab_ev = nullptr;
    bool tab_ev_live = false;
    sdb_kv_batch merged{};
    sdb_merge_summary msum{};
    std::vector<sdb_compacted_sst> ssts;
    ~sdb_compactor() {
        (void)hipSetDevice(device);
        for (DevBuf *b : {&merge_ws, &cols, &keys, &vals, &cut_ws, &cuts, &sst_meta, &sst_data, &sst_bloom, &enc_ws,
                          &dec, &dec_ws, &cx_tab})
            b->release();
        for (GroupBufs &g : groups)
            for (DevBuf *b : {&g.cols, &g.keys, &g.vals, &g.asrun}) b->release();
        if (tab_ev) (void)hipEventSynchronize(tab_ev);
        pin.release();
        pin_tab.release();
        if (tab_ev) (void)hipEventDestroy(tab_ev);
    }
};

namespace {

// merged-stream columns for `total` entries in `cols`: the sdb_merged_out (byte arenas unset)
sdb_status merged_columns_in(DevBuf &cols, uint64_t total, sdb_merged_out *out) {
    const uint64_t o_koff = 0, o_voff = al256(8 * (total + 1)), o_kind = o_voff + al256(8 * (total + 1));
    const uint64_t o_seq = o_kind + al256(total + 1), o_cts = o_seq + al256(8 * (total + 1));
    const uint64_t o_ets = o_cts + al256(8 * (total + 1)), o_mask = o_ets + al256(8 * (total + 1));
    const uint64_t o_sum = o_mask + al256(total + 1), cols_bytes = o_sum + al256(sizeof(sdb_merge_summary));
    if (!cols.ensure(cols_bytes)) return SDB_DEVICE_ERROR;
    *out = sdb_merged_out{};
    out->key_cap = ~0ull;
    out->key_off = cols.at<uint64_t>(o_koff);
    out->val_cap = ~0ull;
    out->val_off = cols.at<uint64_t>(o_voff);
    out->kind = cols.at<uint8_t>(o_kind);
    out->seq = cols.at<uint64_t>(o_seq);
    out->create_ts = cols.at<int64_t>(o_cts);
    out->expire_ts = cols.at<int64_t>(o_ets);
    out->ts_mask = cols.at<uint8_t>(o_mask);
    out->cap_entries = total;
    out->summary = cols.at<sdb_merge_summary>(o_sum);
    return SDB_OK;
}
sdb_status merged_columns(sdb_compactor *c, uint64_t total, sdb_merged_out *out) {
    return merged_columns_in(c->cols, total, out);
}

// A job with more runs than one merge takes (SDB_MAX_RUNS): groups of SDB_MAX_RUNS consecutive runs are
// merged first without retention (every entry kept as it is, in the group's MergeIterator order: key asc,
// seq desc, run), and the group streams become the job's runs.  Groups are consecutive runs, so equal keys
// with equal seqs keep their run order and the job's merged stream is the one a single merge of every run
// would give (merge_iterator.rs:55-69).  One host synchronisation per group (its byte sizes).  A run out
// of order fails the job like the single merge: *fail = the group merge's summary, first_error_entry
// rebased to the job's entry numbering.  gate: the decode gate of sdb_compactor_run_ssts (or NULL).
sdb_status group_runs(sdb_compactor *c, const sdb_run *runs, uint32_t nruns, const unsigned long long *gate,
                      std::vector<sdb_run> &grouped, sdb_merge_summary *fail, hipStream_t s) {
    const uint32_t ng = (nruns + kMaxRuns - 1) / kMaxRuns;
    if (ng > kMaxRuns) return SDB_LIMIT_EXCEEDED;
    uint64_t job_total = 0;
    for (uint32_t r = 0; r < nruns; r++) job_total += runs[r].n;
    if (c->groups.size() < ng) c->groups.resize(ng);
    grouped.clear();
    uint64_t base = 0;
    const sdb_retention none{};
    for (uint32_t g = 0; g < ng; g++) {
        const uint32_t r0 = g * kMaxRuns, r1 = std::min(nruns, r0 + kMaxRuns);
        GroupBufs &B = c->groups[g];
        uint64_t total = 0;
        for (uint32_t r = r0; r < r1; r++) total += runs[r].n;
        sdb_merged_out out{};
        sdb_status st = merged_columns_in(B.cols, total, &out);
        if (st) return st;
        if (!c->merge_ws.ensure(sdb_merge_runs_workspace_bytes(runs + r0, r1 - r0))) return SDB_DEVICE_ERROR;
        MergeArgs a;
        st = build_merge_args(runs + r0, r1 - r0, &none, &out, c->merge_ws.p, c->merge_ws.cap, &a, true);
        if (st) return st;
        a.gate = gate;
        sdb_merge_summary sm{};
        if (launch_merge(a, false, s) != hipSuccess ||
            hipMemcpyAsync(&sm, out.summary, sizeof(sm), hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess)
            return SDB_DEVICE_ERROR;
        if (sm.status) {
            *fail = sm;
            fail->num_in = job_total;
            // the group's entry numbering starts at `base` in the job's (a gate error can only come from
            // group 0, whose base is 0)
            if (sm.status == SDB_INVALID_ARGUMENT && sm.first_error_entry != ~0ull) fail->first_error_entry += base;
            return (sdb_status)sm.status;
        }
        if (!B.keys.ensure(sm.key_bytes + 16) || !B.vals.ensure(sm.val_bytes + 16) ||
            !B.asrun.ensure(al256(4 * (total + 1)) + al256(total + 1)))
            return SDB_DEVICE_ERROR;
        a.out.key_bytes = B.keys.at<uint8_t>(0);
        a.out.key_cap = sm.key_bytes;
        a.out.val_bytes = B.vals.at<uint8_t>(0);
        a.out.val_cap = sm.val_bytes;
        uint32_t *vlen = B.asrun.at<uint32_t>(0);
        uint8_t *flags = B.asrun.at<uint8_t>(al256(4 * (total + 1)));
        if (launch_merge_emit(a, s) != hipSuccess || launch_merged_as_run(a.out, total, vlen, flags, s) != hipSuccess)
            return SDB_DEVICE_ERROR;
        sdb_run R{};
        R.n = total;
        R.key_arena = a.out.key_bytes;
        R.key_off = a.out.key_off;
        R.val_base = a.out.val_bytes;
        R.val_off = a.out.val_off;
        R.val_len = vlen;
        R.seq = a.out.seq;
        R.flags = flags;
        R.create_ts = a.out.create_ts;
        R.expire_ts = a.out.expire_ts;
        grouped.push_back(R);
        base += total;
    }
    return SDB_OK;
}

sdb_kv_batch batch_of(const sdb_merged_out &o, uint64_t n) {
    sdb_kv_batch m{};
    m.n = n;
    m.key_bytes = o.key_bytes;
    m.key_off = o.key_off;
    m.val_bytes = o.val_bytes;
    m.val_off = o.val_off;
    m.kind = o.kind;
    m.seq = o.seq;
    m.create_ts = o.create_ts;
    m.expire_ts = o.expire_ts;
    m.ts_mask = o.ts_mask;
    m.prefix_len = nullptr;
    return m;
}

// step 3 of both jobs: encode every output SST (sets of up to 8 per launch sequence) over the cut
// ranges of c->merged, then read the summaries back (one synchronisation)
sdb_status encode_outputs(sdb_compactor *c, const uint64_t *cut, const uint64_t *off, uint64_t ns,
                          const sdb_sst_params *params, void *stream) {
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const sdb_kv_batch &m = c->merged;
    sdb_status st = SDB_OK;
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
    if (!c->pin.ensure(ns * sizeof(sdb_sst_summary))) return SDB_DEVICE_ERROR;
    sdb_sst_summary *sums = static_cast<sdb_sst_summary *>(c->pin.p);
    if (hipMemcpyAsync(sums, c->sst_meta.p, ns * sizeof(sdb_sst_summary), hipMemcpyDeviceToHost, s) != hipSuccess ||
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
    return first;
}

}  // namespace

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
    if ((nruns && !runs) || !ret) return SDB_INVALID_ARGUMENT;  // before group_runs reads runs[]
    if (hipSetDevice(c->device) != hipSuccess) return SDB_DEVICE_ERROR;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    uint64_t total = 0;
    for (uint32_t r = 0; r < nruns && runs; r++) total += runs[r].n;
    std::vector<sdb_run> grouped;
    if (nruns > kMaxRuns) {  // more runs than one merge takes: groups merged ahead (group_runs)
        const sdb_status gs = group_runs(c, runs, nruns, nullptr, grouped, &c->msum, s);
        if (gs) return gs;
        runs = grouped.data();
        nruns = (uint32_t)grouped.size();
    }

    // 1. merge + retention, sized with unbounded byte capacities, then emitted
    sdb_merged_out out{};
    sdb_status st = merged_columns(c, total, &out);
    if (st) return st;
    const uint64_t mws = sdb_merge_runs_workspace_bytes(runs, nruns);
    if (!c->merge_ws.ensure(mws)) return SDB_DEVICE_ERROR;
    MergeArgs a;
    st = build_merge_args(runs, nruns, ret, &out, c->merge_ws.p, c->merge_ws.cap, &a);
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
    m = batch_of(a.out, n);
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

    // 3. encode every output SST
    const sdb_status first = encode_outputs(c, cut.data(), off.data(), ns, params, stream);
    if (first == SDB_OK || c->ssts.size() == ns) *num_ssts = (uint32_t)ns;
    return first;
}

sdb_status sdb_compactor_run_ssts(sdb_compactor *c, const sdb_compaction_input *inputs, uint32_t ninputs,
                                  const uint32_t *run_start, uint32_t nruns, uint16_t input_sst_version,
                                  const sdb_retention *ret, const sdb_sst_params *params, uint64_t max_sst_size,
                                  void *stream, uint32_t *num_ssts) {
    if (!c || !params || !num_ssts || !ret || (ninputs && !inputs)) return SDB_INVALID_ARGUMENT;
    *num_ssts = 0;
    c->ssts.clear();
    c->merged = sdb_kv_batch{};
    c->msum = sdb_merge_summary{};
    if (params->sst_type != SDB_SST_COMPACTED) return SDB_INVALID_ARGUMENT;
    if (input_sst_version != 1 && input_sst_version != 2) return SDB_INVALID_VERSION;
    if (!run_start) nruns = ninputs;
    if ((uint64_t)nruns > (uint64_t)kMaxRuns * kMaxRuns) return SDB_LIMIT_EXCEEDED;  // two merge levels
    if (run_start) {
        if (run_start[0] != 0 || run_start[nruns] != ninputs) return SDB_INVALID_ARGUMENT;
        for (uint32_t r = 0; r < nruns; r++)
            if (run_start[r + 1] < run_start[r]) return SDB_INVALID_ARGUMENT;
    }
    if (hipSetDevice(c->device) != hipSuccess) return SDB_DEVICE_ERROR;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);

    // the inputs' blocks, in input order, as offsets from the lowest data address; the per-input and per-run
    // tables go to device memory (any number of inputs)
    CxInputs in{};
    in.n = ninputs;
    in.nruns = nruns;
    const uint64_t t_data = 0, t_boff = al256(8ull * ninputs), t_first = t_boff + al256(8ull * ninputs);
    const uint64_t t_rblk = t_first + al256(8ull * (ninputs + 1)), t_rent = t_rblk + al256(8ull * (nruns + 1));
    const uint64_t t_total = t_rent + al256(8ull * (nruns + 1));
    // the previous job's upload and kernels may still read pin_tab / cx_tab (a job that failed early
    // returns without a synchronisation, and the caller may alternate streams)
    if (c->tab_ev_live && hipEventSynchronize(c->tab_ev) != hipSuccess) return SDB_DEVICE_ERROR;
    c->tab_ev_live = false;
    if (!c->tab_ev && hipEventCreateWithFlags(&c->tab_ev, hipEventDisableTiming) != hipSuccess) {
        c->tab_ev = nullptr;
        return SDB_DEVICE_ERROR;
    }
    if (!c->pin_tab.ensure(t_total) || !c->cx_tab.ensure(t_total)) return SDB_DEVICE_ERROR;
    uint8_t *th = static_cast<uint8_t *>(c->pin_tab.p);
    const uint8_t **h_data = reinterpret_cast<const uint8_t **>(th + t_data);
    const uint64_t **h_boff = reinterpret_cast<const uint64_t **>(th + t_boff);
    uint64_t *h_first = reinterpret_cast<uint64_t *>(th + t_first), *h_rblk = reinterpret_cast<uint64_t *>(th + t_rblk);
    uint64_t *h_rent = reinterpret_cast<uint64_t *>(th + t_rent);
    uint64_t E = 0, K = 0, V = 0, B = 0;
    uintptr_t base = ~(uintptr_t)0;
    for (uint32_t i = 0; i < ninputs; i++) {
        const sdb_compaction_input &x = inputs[i];
        if (x.num_blocks && (!x.data || !x.block_off)) return SDB_INVALID_ARGUMENT;
        if (x.num_blocks && (uintptr_t)x.data < base) base = (uintptr_t)x.data;
        h_data[i] = x.data;
        h_boff[i] = x.block_off;
        h_first[i] = B;
        B += x.num_blocks;
        E += x.num_entries;
        K += x.key_bytes;
        V += x.val_bytes;
    }
    h_first[ninputs] = B;
    if (base == ~(uintptr_t)0) base = 0;
    in.base = base;
    in.nblocks = B;
    std::vector<uint64_t> run_entry(nruns + 1);
    {
        uint64_t e = 0;
        for (uint32_t r = 0; r < nruns; r++) {
            const uint32_t i0 = run_start ? run_start[r] : r, i1 = run_start ? run_start[r + 1] : r + 1;
            h_rblk[r] = h_first[i0];
            h_rent[r] = run_entry[r] = e;
            for (uint32_t i = i0; i < i1; i++) e += inputs[i].num_entries;
        }
        h_rblk[nruns] = B;
        h_rent[nruns] = run_entry[nruns] = e;
    }
    in.key_bytes = K;
    if (E >= (1ull << 31)) return SDB_LIMIT_EXCEEDED;
    if (hipMemcpyAsync(c->cx_tab.p, th, t_total, hipMemcpyHostToDevice, s) != hipSuccess) return SDB_DEVICE_ERROR;
    struct TabRelease {  // on every return from here: everything enqueued so far precedes the event
        sdb_compactor *c;
        hipStream_t s;
        ~TabRelease() { c->tab_ev_live = hipEventRecord(c->tab_ev, s) == hipSuccess; }
    } tab_release{c, s};
    in.data = c->cx_tab.at<const uint8_t *const>(t_data);
    in.block_off = c->cx_tab.at<const uint64_t *const>(t_boff);
    in.first_block = c->cx_tab.at<const uint64_t>(t_first);
    in.run_block = c->cx_tab.at<const uint64_t>(t_rblk);
    in.run_entry = c->cx_tab.at<const uint64_t>(t_rent);

    // 1. decode every input block into one columnar output (run r = entries [run_entry[r], run_entry[r+1]))
    const uint64_t o_bs = 0, o_be = o_bs + al256(8 * (B + 1)), o_bes = o_be + al256(8 * (B + 1));
    const uint64_t o_ka = o_bes + al256(8 * (B + 2)), o_ko = o_ka + al256(K + 64);
    const uint64_t o_vo = o_ko + al256(8 * (E + 1)), o_vl = o_vo + al256(8 * (E + 1));
    const uint64_t o_sq = o_vl + al256(4 * (E + 1)), o_fl = o_sq + al256(8 * (E + 1));
    const uint64_t o_ct = o_fl + al256(E + 1), o_et = o_ct + al256(8 * (E + 1)), o_bad = o_et + al256(8 * (E + 1));
    const uint64_t o_ds = o_bad + al256(4 * 16), o_gate = o_ds + al256(sizeof(sdb_decode_summary));
    const uint64_t dec_bytes = o_gate + 256;
    const uint64_t dws = sdb_decode_workspace_bytes(B);
    if (!c->dec.ensure(dec_bytes) || !c->dec_ws.ensure(dws)) return SDB_DEVICE_ERROR;
    uint64_t *bstart = c->dec.at<uint64_t>(o_bs), *bend = c->dec.at<uint64_t>(o_be);
    sdb_decoded_out dout{};
    dout.block_entry_start = c->dec.at<uint64_t>(o_bes);
    dout.key_arena = c->dec.at<uint8_t>(o_ka);
    dout.key_arena_cap = K;
    dout.key_off = c->dec.at<uint64_t>(o_ko);
    dout.val_off = c->dec.at<uint64_t>(o_vo);
    dout.val_len = c->dec.at<uint32_t>(o_vl);
    dout.seq = c->dec.at<uint64_t>(o_sq);
    dout.flags = c->dec.at<uint8_t>(o_fl);
    dout.create_ts = c->dec.at<int64_t>(o_ct);
    dout.expire_ts = c->dec.at<int64_t>(o_et);
    dout.cap_entries = E;
    dout.bad_block = c->dec.at<uint32_t>(o_bad);
    dout.bad_cap = 16;
    dout.summary = c->dec.at<sdb_decode_summary>(o_ds);
    unsigned long long *gate = c->dec.at<unsigned long long>(o_gate);
    const uint8_t *arena = reinterpret_cast<const uint8_t *>(base);
    if (launch_cx_blocks(in, bstart, bend, s) != hipSuccess) return SDB_DEVICE_ERROR;
    // fail-fast (a failing block fails the job anyway, as load_iterators' reads would): checksums in the emit pass
    sdb_status st = sdb_decode_blocks_ex(arena, bstart, bend, B, input_sst_version, SDB_DECODE_FAIL_FAST, &dout,
                                         c->dec_ws.p, c->dec_ws.cap,
                                         stream);
    if (st) return st;
    const unsigned long long *dec_err =
        reinterpret_cast<const unsigned long long *>(static_cast<uint8_t *>(c->dec_ws.p) + decode_workspace_layout(B).err);
    if (launch_cx_gate(in, dout.summary, dec_err, dout.block_entry_start, gate, s) != hipSuccess)
        return SDB_DEVICE_ERROR;
    std::vector<sdb_run> runs(nruns);
    for (uint32_t r = 0; r < nruns; r++) {
        const uint64_t e0 = run_entry[r];
        sdb_run &R = runs[r];
        R.n = run_entry[r + 1] - e0;
        R.key_arena = dout.key_arena;
        R.key_off = dout.key_off + e0;
        R.val_base = arena;
        R.val_off = dout.val_off + e0;
        R.val_len = dout.val_len + e0;
        R.seq = dout.seq + e0;
        R.flags = dout.flags + e0;
        R.create_ts = dout.create_ts + e0;
        R.expire_ts = dout.expire_ts + e0;
    }

    // 2. merge + retention + emit into buffers of the declared sizes (retention only drops entries and
    //    values), gated on the decode; the stream padded to E entries for the cut walk
    sdb_merged_out out{};
    st = merged_columns(c, E, &out);
    if (st) return st;
    if (!c->keys.ensure(K + 16) || !c->vals.ensure(V + 16)) return SDB_DEVICE_ERROR;
    out.key_bytes = c->keys.at<uint8_t>(0);
    out.key_cap = K;
    out.val_bytes = c->vals.at<uint8_t>(0);
    out.val_cap = V;
    const sdb_run *mruns = runs.data();
    uint32_t mn = nruns;
    std::vector<sdb_run> grouped;
    if (nruns > kMaxRuns) {  // more runs than one merge takes: groups merged ahead (group_runs)
        const sdb_status gs = group_runs(c, mruns, nruns, gate, grouped, &c->msum, s);
        if (gs) return gs;
        mruns = grouped.data();
        mn = (uint32_t)grouped.size();
    }
    if (!c->merge_ws.ensure(sdb_merge_runs_workspace_bytes(mruns, mn))) return SDB_DEVICE_ERROR;
    MergeArgs a;
    st = build_merge_args(mruns, mn, ret, &out, c->merge_ws.p, c->merge_ws.cap, &a);
    if (st) return st;
    a.gate = gate;
    if (launch_merge(a, true, s) != hipSuccess || launch_merge_pad(out, E, s) != hipSuccess) return SDB_DEVICE_ERROR;
    const sdb_kv_batch padded = batch_of(out, E);

    // cuts over the padded stream, ending at the merged count; merged summary, cut count, cuts and their
    // byte offsets read back in one synchronisation
    const uint64_t cws = sdb_sst_cuts_workspace_bytes(E, params);
    const uint64_t o_num = 0, o_cut = 256, o_off = o_cut + al256(8 * (E + 2));
    if (!c->cut_ws.ensure(cws) || !c->cuts.ensure(o_off + al256(16 * (E + 2)))) return SDB_DEVICE_ERROR;
    uint64_t *d_num = c->cuts.at<uint64_t>(o_num), *d_cut = c->cuts.at<uint64_t>(o_cut);
    uint64_t *d_off = c->cuts.at<uint64_t>(o_off);
    if (E) {
        st = sst_cuts_padded(&padded, params, max_sst_size, d_cut, E + 1, d_num, c->cut_ws.p, c->cut_ws.cap, s,
                             &out.summary->num_out);
        if (st) return st;
        if (launch_cut_offsets(d_cut, d_num, out.key_off, out.val_off, d_off, s) != hipSuccess) return SDB_DEVICE_ERROR;
    }
    const uint64_t g = max_sst_size ? std::min<uint64_t>(E, 2 + (K + V + 64 * E) / max_sst_size) : E;
    const uint64_t h_sum = 0, h_num = al256(sizeof(sdb_merge_summary)), h_cut = h_num + 256;
    const uint64_t h_off = h_cut + al256(8 * (g + 2)), h_total = h_off + al256(16 * (g + 2));
    if (!c->pin.ensure(h_total)) return SDB_DEVICE_ERROR;
    uint8_t *hp = static_cast<uint8_t *>(c->pin.p);
    sdb_merge_summary *hsum = reinterpret_cast<sdb_merge_summary *>(hp + h_sum);
    uint64_t *hnum = reinterpret_cast<uint64_t *>(hp + h_num);
    *hnum = 0;
    if (hipMemcpyAsync(hsum, out.summary, sizeof(sdb_merge_summary), hipMemcpyDeviceToHost, s) != hipSuccess ||
        (E && (hipMemcpyAsync(hnum, d_num, 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
               hipMemcpyAsync(hp + h_cut, d_cut, 8 * (g + 1), hipMemcpyDeviceToHost, s) != hipSuccess ||
               hipMemcpyAsync(hp + h_off, d_off, 16 * (g + 1), hipMemcpyDeviceToHost, s) != hipSuccess)) ||
        hipStreamSynchronize(s) != hipSuccess)
        return SDB_DEVICE_ERROR;
    c->msum = *hsum;
    if (c->msum.status) return (sdb_status)c->msum.status;
    const uint64_t n = c->msum.num_out;
    c->merged = batch_of(out, n);
    const uint64_t ns = *hnum;
    if (!n) return SDB_OK;
    if (ns == 0 || ns > n) return SDB_DEVICE_ERROR;
    std::vector<uint64_t> cut(ns + 1), off(2 * (ns + 1));
    if (ns > g) {
        if (hipMemcpy(cut.data(), d_cut, 8 * (ns + 1), hipMemcpyDeviceToHost) != hipSuccess ||
            hipMemcpy(off.data(), d_off, 16 * (ns + 1), hipMemcpyDeviceToHost) != hipSuccess)
            return SDB_DEVICE_ERROR;
    } else {
        memcpy(cut.data(), hp + h_cut, 8 * (ns + 1));
        memcpy(off.data(), hp + h_off, 16 * (ns + 1));
    }

    // 3. encode every output SST
    const sdb_status first = encode_outputs(c, cut.data(), off.data(), ns, params, stream);
    if (first == SDB_OK || c->ssts.size() == ns) *num_ssts = (uint32_t)ns;
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
