// sdb_compact.hip — the compaction output side on the device: merge of sorted runs, retention, and
// the SST cuts of the output stream (include/slatedb_amd.h, "Compaction").
//
//   k_mg_prefix   per input entry: 8-byte big-endian key prefix; run order check
//   k_mg_rank     per input entry: its merged position = own index + one binary search per other run
//                 (MergeIterator order, merge_iterator.rs:55-69: key asc, seq desc, then run)
//   k_mg_keys     per merged position: first version of its key?; merge operand check
//                 (MergeOperatorRequiredIterator, merge_operator.rs:213-223); per key, on its first
//                 version's thread: apply_retention_filter (retention_iterator.rs:91-204) -> keep / drop /
//                 keep as a tombstone per version, and the kept entries / key / value bytes per
//                 kMergeTile positions
//   k_mg_scan     one workgroup: tile offsets, the summary
//   k_mg_emit     per kMergeTile positions: the output batch (metadata + key / value bytes)
//   k_cut         one lane: the compactor's max_sst_size walk (compactor_executor.rs:833-858) over
//                 the chain tables of the encoder's k_seg / k_group (group, chunk, then block steps)
//
// The work here is integer / byte movement bound by HBM and by the dependent loads of the binary
// searches; nothing is GEMM-shaped.
#include <hip/hip_runtime.h>

#include "sdb_compact.h"
#include "sdb_device.h"

namespace sdb {

namespace {

constexpr uint32_t kPfxThreads = 256;

// The run holding global entry g: the number of runs after the first that start at or below g (bases
// ascend; an empty run shares its successor's base).  The loop index is uniform, so the bases are
// scalar loads of the kernel arguments and no load waits on g.
SDB_DEV uint32_t run_of(const MergeArgs &a, uint64_t g) {
    uint32_t r = 0;
    for (uint32_t k = 1; k < a.nruns; k++) r += g >= a.r[k].base ? 1u : 0u;
    return r;
}

// The descriptor of a lane's run (run: per lane) by a uniform walk over the runs (their fields come by scalar
// loads) and selects, instead of a per-lane vector load of the kernel-argument array: one dependent memory
// round trip less in front of every gather that starts from a global entry index.
SDB_DEV RunDesc run_desc(const MergeArgs &a, uint32_t run) {
    RunDesc d = a.r[0];
    for (uint32_t k = 1; k < a.nruns; k++) {
        const RunDesc &c = a.r[k];
        const bool m = run == k;
        d.n = m ? c.n : d.n;
        d.base = m ? c.base : d.base;
        d.key_arena = m ? c.key_arena : d.key_arena;
        d.key_off = m ? c.key_off : d.key_off;
        d.val_base = m ? c.val_base : d.val_base;
        d.val_off = m ? c.val_off : d.val_off;
        d.val_len = m ? c.val_len : d.val_len;
        d.seq = m ? c.seq : d.seq;
        d.flags = m ? c.flags : d.flags;
        d.create_ts = m ? c.create_ts : d.create_ts;
        d.expire_ts = m ? c.expire_ts : d.expire_ts;
    }
    return d;
}

SDB_DEV uint64_t key_prefix(const uint8_t *p, uint32_t n) {  // first 8 bytes, big-endian, zero padded
    if (!n) return 0;
    const uint32_t need = n < 8 ? n : 8;
    uint64_t v = load8(p, need);
    if (need < 8) v &= (~0ull) >> (8 * (8 - need));
    return bswap64(v);
}

struct KeyAt {
    const uint8_t *p;
    uint32_t n;
};
SDB_DEV KeyAt key_at(const RunDesc &R, uint64_t i) {
    const uint64_t o = R.key_off[i];
    return {R.key_arena + o, (uint32_t)(R.key_off[i + 1] - o)};
}

// <[u8] as Ord>::cmp given the prefixes of bytes [s, s + 8) of two keys whose bytes [0, s) are equal:
// -1, 0, 1
SDB_DEV int cmp_key(uint64_t pa, const uint8_t *a, uint32_t na, uint64_t pb, const uint8_t *b, uint32_t nb,
                    uint32_t s = 0) {
    if (pa != pb) return pa < pb ? -1 : 1;
    const uint32_t t = s + 8;
    if (na > t && nb > t) {
        const uint32_t l = lcp_bytes(a + t, na - t, b + t, nb - t), m = (na < nb ? na : nb) - t;
        if (l < m) return a[t + l] < b[t + l] ? -1 : 1;
    }
    return na < nb ? -1 : (na > nb ? 1 : 0);
}

// L0 = the common prefix of the first and last keys of every run, with run 0's first key: every key of
// sorted runs lies between its run's first and last, so it shares L0 bytes with them.  The merge's
// 8-byte prefixes start there (keys with a long common prefix, e.g. big-endian counters, would otherwise
// tie on every prefix and compare their bytes from HBM).  Checked by k_mg_prefix's full run-order test:
// the rank and group kernels only run when every run is sorted.
__global__ void k_mg_lcp0(MergeArgs a) {
    for (uint64_t x = threadIdx.x; x < 3 * (uint64_t)a.ntiles; x += blockDim.x) a.tile_sum[x] = 0;  // k_mg_keys adds
    if (threadIdx.x) return;
    if (a.gate && *a.gate != ~0ull) {  // a failed input: the job fails with its status, nothing is merged
        *a.err = *a.gate;
        *a.lcp0 = 0;
        return;
    }
    uint32_t L = ~0u;
    const uint8_t *e0 = nullptr;
    uint32_t n0 = 0;
    for (uint32_t r = 0; r < a.nruns; r++) {
        const RunDesc &R = a.r[r];
        if (!R.n) continue;
        const KeyAt f = key_at(R, 0), l = key_at(R, R.n - 1);
        if (!e0) {
            e0 = f.p;
            n0 = f.n;
            L = n0;
        }
        const uint32_t x = lcp_bytes(e0, n0, f.p, f.n), y = lcp_bytes(e0, n0, l.p, l.n);
        L = x < L ? x : L;
        L = y < L ? y : L;
    }
    *a.lcp0 = e0 ? L : 0;
}


__global__ __launch_bounds__(kPfxThreads) void k_mg_prefix(MergeArgs a) {
    const uint64_t g = (uint64_t)blockIdx.x * kPfxThreads + threadIdx.x;
    if (g >= a.total || (a.gate && *a.gate != ~0ull)) return;
    const uint32_t r = run_of(a, g);
    const RunDesc &R = a.r[r];
    const uint64_t i = g - R.base;
    const KeyAt k = key_at(R, i);
    const uint64_t pk = key_prefix(k.p, k.n);
    const uint32_t L0 = *a.lcp0;
    a.pfx[g] = k.n >= L0 ? key_prefix(k.p + L0, k.n - L0) : 0;  // n >= L0 whenever the runs are sorted
    if (i > 0) {  // sorted-run precondition: key asc, seq desc (full keys)
        const KeyAt q = key_at(R, i - 1);
        const int c = cmp_key(key_prefix(q.p, q.n), q.p, q.n, pk, k.p, k.n);
        if (c > 0 || (c == 0 && R.seq[i - 1] < R.seq[i])) report_error(a.err, g, SDB_INVALID_ARGUMENT);
    }
}

// Entries of run Q (= run r2) in [lo, hi) that come before (key k, seq sq, run r): key less, or equal
// with a larger seq, or an equal seq in an earlier run; the count is known to lie in [lo, hi].
SDB_DEV uint64_t rank_in(const MergeArgs &a, uint32_t r2, uint32_t r, uint64_t pk, const KeyAt &k, uint64_t sq,
                         uint32_t L0, uint64_t lo, uint64_t hi) {
    const RunDesc &Q = a.r[r2];
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const KeyAt f = key_at(Q, mid);
        const int c = cmp_key(a.pfx[Q.base + mid], f.p, f.n, pk, k.p, k.n, L0);
        bool before = c < 0;
        if (c == 0) {
            const uint64_t s2 = Q.seq[mid];
            before = s2 > sq || (s2 == sq && r2 < r);
        }
        if (before) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// rank_in over a window whose prefixes are staged in LDS (w: the window's a.pfx values, from run index lo):
// a step whose prefix differs from the key's is decided in LDS, a tie compares the full keys and seqs in
// HBM as rank_in does
SDB_DEV uint64_t rank_in_lds(const MergeArgs &a, uint32_t r2, uint32_t r, uint64_t pk, const KeyAt &k, uint64_t sq,
                             uint32_t L0, uint64_t lo, uint64_t hi, const uint64_t *w) {
    const RunDesc &Q = a.r[r2];
    const uint64_t base = lo;
    while (lo < hi) {
        const uint64_t mid = (lo + hi) >> 1;
        const uint64_t pm = w[mid - base];
        bool before;
        if (pm != pk) {
            before = pm < pk;
        } else {
            const KeyAt f = key_at(Q, mid);
            const int c = cmp_key(pm, f.p, f.n, pk, k.p, k.n, L0);
            before = c < 0;
            if (c == 0) {
                const uint64_t s2 = Q.seq[mid];
                before = s2 > sq || (s2 == sq && r2 < r);
            }
        }
        if (before) lo = mid + 1;
        else hi = mid;
    }
    return lo;
}

// Merged position = own index + the entries of every other run that come before.  A workgroup's
// entries are consecutive in one run, so their counts in run r2 lie between those of its first and
// last entry: two full binary searches per workgroup and run, then each entry searches that window —
// in LDS when the windows' prefixes fit (kRankLds; staged with coalesced loads), so a search step is an
// LDS read instead of a dependent HBM gather.
constexpr uint32_t kRankLds = 16 * 1024;
// The two full searches of every k_mg_rank workgroup and run, one thread each, all in flight at once (inside
// the rank workgroups each one was a 20-step chain of dependent gathers in front of the workgroup's work):
// bound[(b * 2 + side) * nruns + r2] = the count in run r2 of workgroup b's first (side 0) / last entry.
__global__ __launch_bounds__(256) void k_mg_bounds(MergeArgs a) {
    if (*a.err != ~0ull) return;
    const uint64_t gb = (a.total + kPfxThreads - 1) / kPfxThreads, nr = a.nruns;
    const uint64_t t = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x, q = t / nr;
    const uint32_t r2 = (uint32_t)(t - q * nr), side = (uint32_t)(q & 1);
    const uint64_t b = q >> 1;
    if (b >= gb) return;
    const uint64_t g0 = b * kPfxThreads, gl = (g0 + kPfxThreads < a.total ? g0 + kPfxThreads : a.total) - 1;
    const uint64_t ge = side ? gl : g0;
    const uint32_t r = run_of(a, ge);
    uint64_t v = 0;
    if (r2 != r) {
        const RunDesc &R = a.r[r];
        const uint64_t i = ge - R.base;
        v = rank_in(a, r2, r, a.pfx[ge], key_at(R, i), R.seq[i], *a.lcp0, 0, a.r[r2].n);
    }
    a.bound[t] = v;
}

__global__ __launch_bounds__(kPfxThreads) void k_mg_rank(MergeArgs a) {
    __shared__ uint64_t s_win[2][kMaxRuns];
    __shared__ uint64_t s_pf[kRankLds / 8];
    __shared__ uint32_t s_woff[kMaxRuns];  // window r2's offset in s_pf (~0: searched in HBM)
    if (*a.err != ~0ull) return;
    const uint64_t g0 = (uint64_t)blockIdx.x * kPfxThreads;
    const uint64_t gl = (g0 + kPfxThreads < a.total ? g0 + kPfxThreads : a.total) - 1;
    const uint32_t r = run_of(a, g0), tid = threadIdx.x;
    const bool one_run = run_of(a, gl) == r;  // uniform
    const uint32_t L0 = *a.lcp0;
    if (one_run) {
        // thread t < nruns: the first entry's count in run t; thread 64 + t: the last entry's (k_mg_bounds)
        const uint32_t side = tid >> 6, r2 = tid & 63;
        if (side < 2 && r2 < a.nruns && r2 != r) s_win[side][r2] = a.bound[((uint64_t)blockIdx.x * 2 + side) * a.nruns + r2];
        __syncthreads();
        if (tid == 0) {  // pack the windows that fit
            uint32_t off = 0;
            for (uint32_t r2 = 0; r2 < a.nruns; r2++) {
                const uint64_t c = r2 == r ? 0 : s_win[1][r2] - s_win[0][r2];
                s_woff[r2] = ~0u;
                if (r2 != r && off + c <= kRankLds / 8) {
                    s_woff[r2] = off;
                    off += (uint32_t)c;
                }
            }
        }
        __syncthreads();
        for (uint32_t r2 = 0; r2 < a.nruns; r2++) {  // (uniform)
            const uint32_t off = s_woff[r2];
            if (off == ~0u) continue;
            const uint64_t lo = s_win[0][r2], c = s_win[1][r2] - lo, b = a.r[r2].base + lo;
            for (uint64_t x = tid; x < c; x += kPfxThreads) s_pf[off + x] = a.pfx[b + x];
        }
        __syncthreads();
    }
    const uint64_t g = g0 + tid;
    if (g >= a.total) return;
    const uint32_t rg = one_run ? r : run_of(a, g);
    const RunDesc &R = a.r[rg];
    const uint64_t i = g - R.base;
    const KeyAt k = key_at(R, i);
    const uint64_t pk = a.pfx[g], sq = R.seq[i];
    uint64_t pos = i;
    for (uint32_t r2 = 0; r2 < a.nruns; r2++) {
        if (r2 == rg) continue;
        const uint64_t lo = one_run ? s_win[0][r2] : 0, hi = one_run ? s_win[1][r2] : a.r[r2].n;
        const uint32_t off = one_run ? s_woff[r2] : ~0u;
        pos += off != ~0u ? rank_in_lds(a, r2, rg, pk, k, sq, L0, lo, hi, s_pf + off)
                          : rank_in(a, r2, rg, pk, k, sq, L0, lo, hi);
    }
    a.perm[pos] = g;
}

struct Ver {
    uint64_t seq;
    int64_t ets;
    uint8_t flags;
};
SDB_DEV Ver ver_at(const MergeArgs &a, uint64_t p) {
    const uint64_t g = a.perm[p];
    const RunDesc &R = a.r[run_of(a, g)];
    const uint64_t i = g - R.base;
    Ver v;
    v.seq = R.seq[i];
    v.flags = R.flags[i];
    v.ets = (v.flags & SDB_FLAG_HAS_EXPIRE_TS) ? R.expire_ts[i] : 0;
    return v;
}

static_assert(kMergeTile % kPfxThreads == 0, "a k_mg_keys workgroup lies in one tile");

// What k_mg_keys needs of the entry at merged position q: one level of gathers after perm[q].
struct PosInfo {
    uint64_t pf, seq;
    const uint8_t *kp;
    const int64_t *ets_src;
    uint32_t kn, vlen;
    uint8_t flags;
};
SDB_DEV PosInfo pos_info(const MergeArgs &a, uint64_t q) {
    const uint64_t g = a.perm[q];
    const RunDesc R = run_desc(a, run_of(a, g));
    const uint64_t i = g - R.base;
    PosInfo x;
    const uint64_t k0 = R.key_off[i], k1 = R.key_off[i + 1];
    x.pf = a.pfx[g];
    x.seq = R.seq[i];
    x.flags = R.flags[i];
    x.vlen = R.val_len[i];
    x.ets_src = R.expire_ts ? R.expire_ts + i : nullptr;  // read only when the flags carry one (rare)
    x.kp = R.key_arena + k0;
    x.kn = (uint32_t)(k1 - k0);
    return x;
}

// Per merged position p: is it the first version of its key (its key differs from position p - 1's,
// MergeIterator order)?  The merge operand check (MergeOperatorRequiredIterator, merge_operator.rs:
// 213-223).  The thread of a key's first version then runs retention over the key's versions, newest
// first (retention_iterator.rs:91-204 over the RetentionBuffer's BTreeMap, :381-398), writes dec[] per
// version and sums the kept entries / key bytes / value bytes into the tile of kMergeTile positions
// each version lies in (k_mg_lcp0 zeroed the tile sums; one atomic per workgroup and field, a version
// past the workgroup's tile adds on its own).  Lanes hold consecutive positions: the neighbours' keys
// come by DPP (lanes 0 / 63 gather theirs alongside their own), and a key with one version (the common
// case) is decided from the lane's own gathers.
__global__ __launch_bounds__(kPfxThreads) void k_mg_keys(MergeArgs a) {
    __shared__ unsigned long long s_sum[3];
    const uint32_t tid = threadIdx.x, lane = tid & 63;
    if (tid < 3) s_sum[tid] = 0;
    __syncthreads();
    const uint64_t p0 = (uint64_t)blockIdx.x * kPfxThreads, p = p0 + tid, T0 = p0 / kMergeTile;
    unsigned long long *ts = (unsigned long long *)a.tile_sum;
    uint64_t c = 0, kb = 0, vb = 0;  // this workgroup's tile
    if (*a.err == ~0ull && a.total) {  // (uniform: the DPP exchanges below run on every lane)
        const uint32_t L0 = *a.lcp0;
        const uint64_t n = a.total;
        const bool live = p < n;
        // lane 0 also gathers position p - 1, lane 63 position p + 1 (the others re-read their own)
        const uint64_t qo = lane == 0 ? (p > 0 ? p - 1 : p) : lane == 63 ? (p + 1 < n ? p + 1 : p) : p;
        // both gathers unconditional (a lane past the end reads position n - 1): under a branch the
        // compiler waited for the first gather's loads before issuing the second's
        const uint64_t pc = live ? p : n - 1, qc = live ? qo : n - 1;
        const PosInfo me = pos_info(a, pc), ot = pos_info(a, qc);
        uint64_t ppf = wave_prev_lane(me.pf), pkp = wave_prev_lane((uint64_t)me.kp);
        uint32_t pkn = wave_prev_lane(me.kn);
        uint64_t npf = wave_next_lane(me.pf), nkp = wave_next_lane((uint64_t)me.kp);
        uint32_t nkn = wave_next_lane(me.kn);
        if (lane == 0) {
            ppf = ot.pf;
            pkp = (uint64_t)ot.kp;
            pkn = ot.kn;
        } else if (lane == 63) {
            npf = ot.pf;
            nkp = (uint64_t)ot.kp;
            nkn = ot.kn;
        }
        if (live && a.raw) {  // a group of a job's runs merged ahead of the job (no retention): keep it
            a.dec[p] = 1;
            c = 1;
            kb = me.kn;
            vb = (me.flags & SDB_FLAG_TOMBSTONE) ? 0 : me.vlen;
        } else if (live) {
            if (!a.ret.merge_operands && (me.flags & SDB_FLAG_MERGE_OPERAND))
                report_error(a.err_merge, p, SDB_MERGE_OPERATOR_MISSING);
            const bool first = p == 0 || cmp_key(ppf, (const uint8_t *)pkp, pkn, me.pf, me.kp, me.kn, L0) != 0;
            const bool more = p + 1 < n && cmp_key(npf, (const uint8_t *)nkp, nkn, me.pf, me.kp, me.kn, L0) == 0;
            const sdb_retention &rt = a.ret;
            if (first && !more) {  // one version: it is the newest, so only expiry and the tombstone filter apply
                uint8_t d = 1;
                if ((me.flags & SDB_FLAG_HAS_EXPIRE_TS) && (me.ets_src ? *me.ets_src : 0) <= rt.compaction_start_ts) {
                    const bool is_merge = (me.flags & SDB_FLAG_MERGE_OPERAND) != 0;
                    atomicAdd(&a.metric[is_merge ? 1 : 0], 1ull);
                    d = is_merge ? 0 : 2;
                }
                if (rt.filter_tombstone && (d == 2 || (d && (me.flags & SDB_FLAG_TOMBSTONE)))) d = 0;
                a.dec[p] = d;
                if (d) {
                    c = 1;
                    kb = me.kn;
                    vb = (d == 1 && !(me.flags & SDB_FLAG_TOMBSTONE)) ? me.vlen : 0;
                }
            } else if (first) {  // several versions: walk them from HBM
                auto same = [&](uint64_t q) {  // position q holds this key
                    const uint64_t h = a.perm[q];
                    const RunDesc &Q = a.r[run_of(a, h)];
                    const KeyAt x = key_at(Q, h - Q.base);
                    return cmp_key(a.pfx[h], x.p, x.n, me.pf, me.kp, me.kn, L0) == 0;
                };
                uint64_t end = p + 2;
                while (end < n && same(end)) end++;
                uint64_t nv = 0, nm = 0;
                bool broken = false;
                Ver cur = ver_at(a, p);
                for (uint64_t q = p; q < end; q++) {
                    Ver nxt{};
                    if (q + 1 < end) nxt = ver_at(a, q + 1);
                    uint8_t d = 0;
                    // a later version with the same seq replaces this one (BTreeMap::insert)
                    if (!broken && !(q + 1 < end && nxt.seq == cur.seq)) {
                        const bool is_merge = (cur.flags & SDB_FLAG_MERGE_OPERAND) != 0;
                        bool skip = false;
                        d = 1;
                        if ((cur.flags & SDB_FLAG_HAS_EXPIRE_TS) && cur.ets <= rt.compaction_start_ts) {
                            if (is_merge) {  // expired merge operands are skipped
                                nm++;
                                skip = true;
                                d = 0;
                            } else {         // expired values / tombstones become tombstones
                                nv++;
                                d = 2;
                            }
                        }
                        if (!skip) {
                            const bool cont = (rt.has_time_window && cur.seq >= rt.time_seq) ||
                                              (rt.has_min_seq && cur.seq > rt.min_seq) || is_merge;
                            if (!cont) broken = true;
                        }
                    }
                    a.dec[q] = d;
                    cur = nxt;
                }
                if (rt.filter_tombstone) {  // pop the tombstones in the tail
                    for (uint64_t q = end; q-- > p;) {
                        const uint8_t d = a.dec[q];
                        if (!d) continue;
                        if (d == 2 || (ver_at(a, q).flags & SDB_FLAG_TOMBSTONE)) a.dec[q] = 0;
                        else break;
                    }
                }
                if (nv) atomicAdd(&a.metric[0], (unsigned long long)nv);
                if (nm) atomicAdd(&a.metric[1], (unsigned long long)nm);
                // output sizes of the kept versions (all of them carry this key)
                for (uint64_t q = p; q < end; q++) {
                    const uint8_t d = a.dec[q];
                    if (!d) continue;
                    const uint64_t h = a.perm[q];
                    const RunDesc &Q = a.r[run_of(a, h)];
                    const uint64_t qi = h - Q.base;
                    const uint64_t v = (d == 1 && !(Q.flags[qi] & SDB_FLAG_TOMBSTONE)) ? Q.val_len[qi] : 0;
                    const uint64_t T = q / kMergeTile;
                    if (T == T0) {
                        c++;
                        kb += me.kn;
                        vb += v;
                    } else {
                        atomicAdd(&ts[3 * T + 0], 1ull);
                        atomicAdd(&ts[3 * T + 1], (unsigned long long)me.kn);
                        if (v) atomicAdd(&ts[3 * T + 2], (unsigned long long)v);
                    }
                }
            }
        }
    }
    c = wave_sum(c);
    kb = wave_sum(kb);
    vb = wave_sum(vb);
    if (lane == 0) {
        if (c) atomicAdd(&s_sum[0], (unsigned long long)c);
        if (kb) atomicAdd(&s_sum[1], (unsigned long long)kb);
        if (vb) atomicAdd(&s_sum[2], (unsigned long long)vb);
    }
    __syncthreads();
    if (tid < 3 && s_sum[tid]) atomicAdd(&ts[3 * T0 + tid], s_sum[tid]);
}

constexpr uint32_t kPerT = kMergeTile / kMergeThreads;

// One workgroup: exclusive tile offsets, the totals and the summary.
__global__ __launch_bounds__(kMergeThreads) void k_mg_scan(MergeArgs a) {
    __shared__ uint64_t s_w[17];
    sdb_merge_summary *sm = a.out.summary;
    unsigned long long e1 = *a.err;
    const unsigned long long e2 = *a.err_merge;
    if (e1 == ~0ull && a.gate && *a.gate != ~0ull) e1 = *a.gate;  // (no entries: k_mg_lcp0 did not run)
    uint64_t carry[3] = {0, 0, 0};
    if (e1 == ~0ull && e2 == ~0ull) {
        for (uint32_t base = 0; base < a.ntiles; base += kMergeThreads) {
            const uint32_t t = base + threadIdx.x;
#pragma unroll
            for (int f = 0; f < 3; f++) {
                const uint64_t v = t < a.ntiles ? a.tile_sum[3 * (uint64_t)t + f] : 0;
                uint64_t tot;
                const uint64_t ex = block_excl_scan_u64(v, s_w, &tot);
                if (t < a.ntiles) a.tile_sum[3 * (uint64_t)t + f] = carry[f] + ex;
                carry[f] += tot;
            }
        }
    }
    if (threadIdx.x) return;
    // (a job that fails reports no retention counts: k_mg_keys ran its walks before the errors were known)
    const bool clean = e1 == ~0ull && e2 == ~0ull;
    sm->num_in = a.total;
    sm->expired_values = clean ? a.metric[0] : 0;
    sm->expired_merges = clean ? a.metric[1] : 0;
    sm->pad = 0;
    sm->first_error_entry = ~0ull;
    int32_t st = SDB_OK;
    if (e1 != ~0ull) {
        st = (int32_t)(e1 & 0xFF);
        sm->first_error_entry = e1 >> 8;
    } else if (e2 != ~0ull) {
        st = (int32_t)(e2 & 0xFF);
        sm->first_error_entry = e2 >> 8;
    } else if (carry[0] > a.out.cap_entries || carry[1] > a.out.key_cap || carry[2] > a.out.val_cap) {
        st = SDB_INVALID_ARGUMENT;
    }
    sm->status = st;
    // a capacity failure still reports the sizes the output needs
    const bool sized = e1 == ~0ull && e2 == ~0ull;
    sm->num_out = sized ? carry[0] : 0;
    sm->key_bytes = sized ? carry[1] : 0;
    sm->val_bytes = sized ? carry[2] : 0;
    if (!st) {
        a.out.key_off[carry[0]] = carry[1];
        a.out.val_off[carry[0]] = carry[2];
    }
}

// Unaligned vector / scalar accesses for byte ranges at any alignment (unaligned global access is
// enabled on gfx9).
typedef uint32_t u32x4_u __attribute__((ext_vector_type(4), aligned(1)));
typedef uint32_t u32x2_u __attribute__((ext_vector_type(2), aligned(1)));
typedef uint32_t u32_u __attribute__((aligned(1)));

// Key / value copies of the merge emit: the entries' descriptors sit in LDS and a wave copies 64 of them
// at a time, eight lanes per entry and 16 bytes per lane per step, so a load instruction reads eight
// contiguous 128-byte spans (a thread copying its own entries, one load in flight, ran at 0.7 TB/s).
struct CopyDesc {
    const uint8_t *ks, *vs;
    uint8_t *kd, *vd;
    uint32_t kb, vb;
};
// <= 16 bytes as independent loads (16, or 8 / 4 / 2 / 1 pieces: never past the range), so a lane's
// chunks of several entries are all in flight before the first store waits
struct Chunk {  // (its length is recomputed at the store from the descriptor: fewer live registers)
    uint64_t lo, hi;
};
typedef uint16_t u16_u __attribute__((aligned(1)));
typedef uint64_t u64_u __attribute__((aligned(1)));
SDB_DEV void chunk_load(Chunk &c, const uint8_t *src, uint32_t n) {
    if (n >= 16) {  // one 16-byte access
        const u32x4_u v = *(const u32x4_u *)src;
        c.lo = (uint64_t)v.x | ((uint64_t)v.y << 32);
        c.hi = (uint64_t)v.z | ((uint64_t)v.w << 32);
        return;
    }
    const uint32_t o = n & 8, b4 = n & 4, b2 = n & 2;
    c.lo = o ? *(const u64_u *)src : 0;
    uint64_t t = 0;
    if (b4) t = *(const u32_u *)(src + o);
    if (b2) t |= (uint64_t)*(const u16_u *)(src + o + b4) << (8 * b4);
    if (n & 1) t |= (uint64_t)src[o + b4 + b2] << (8 * (b4 + b2));
    if (o) c.hi = t;
    else c.lo = t;
}
SDB_DEV void chunk_store(const Chunk &c, uint8_t *dst, uint32_t n) {
    if (n >= 16) {
        u32x4_u v;
        v.x = (uint32_t)c.lo, v.y = (uint32_t)(c.lo >> 32), v.z = (uint32_t)c.hi, v.w = (uint32_t)(c.hi >> 32);
        *(u32x4_u *)dst = v;
        return;
    }
    const uint32_t o = n & 8, b4 = n & 4, b2 = n & 2;
    if (o) *(u64_u *)dst = c.lo;
    const uint64_t t = o ? c.hi : c.lo;
    if (b4) *(u32_u *)(dst + o) = (uint32_t)t;
    if (b2) *(u16_u *)(dst + o + b4) = (uint16_t)(t >> (8 * b4));
    if (n & 1) dst[o + b4 + b2] = (uint8_t)(t >> (8 * (b4 + b2)));
}
// The unconditional form of a lane chunk (a load under a branch makes the compiler wait for every earlier
// load at the join, so the chunks of eight entries went out one at a time): a range of >= 16 bytes reads
// the 16 bytes at x, or for its tail the 16 ending at its end (shifted down at the store); a lane with no
// chunk, or a range under 16 bytes, reads g_safe16 and (the latter) copies piecewise afterwards.
__device__ uint4 g_safe16;
SDB_DEV const uint8_t *chunk_src(const uint8_t *src, uint32_t len, uint32_t x) {
    const bool live = x < len && len >= 16;
    return live ? src + (x + 16 <= len ? x : len - 16) : (const uint8_t *)&g_safe16;
}
// global (not flat) accesses: a flat access also counts on lgkmcnt, so every LDS descriptor read after the
// stores waited for all of them
typedef __attribute__((address_space(1))) u32x4_u g_u32x4_u;
typedef __attribute__((address_space(1))) u64_u g_u64_u;
typedef __attribute__((address_space(1))) u32_u g_u32_u;
typedef __attribute__((address_space(1))) u16_u g_u16_u;
typedef __attribute__((address_space(1))) uint8_t g_u8;
SDB_DEV u32x4_u chunk_ld(const uint8_t *p) { return *(const g_u32x4_u *)(uintptr_t)p; }
SDB_DEV void chunk_store_g(const Chunk &c, uint8_t *dst0, uint32_t n) {
    const uintptr_t dst = (uintptr_t)dst0;
    if (n >= 16) {
        u32x4_u v;
        v.x = (uint32_t)c.lo, v.y = (uint32_t)(c.lo >> 32), v.z = (uint32_t)c.hi, v.w = (uint32_t)(c.hi >> 32);
        *(g_u32x4_u *)dst = v;
        return;
    }
    const uint32_t o = n & 8, b4 = n & 4, b2 = n & 2;
    if (o) *(g_u64_u *)dst = c.lo;
    const uint64_t t = o ? c.hi : c.lo;
    if (b4) *(g_u32_u *)(dst + o) = (uint32_t)t;
    if (b2) *(g_u16_u *)(dst + o + b4) = (uint16_t)(t >> (8 * b4));
    if (n & 1) *(g_u8 *)(dst + o + b4 + b2) = (uint8_t)(t >> (8 * (b4 + b2)));
}
// store bytes [x, min(len, x + 16)) of the range from the chunk_src window w
SDB_DEV void chunk_put(const u32x4_u &w, const uint8_t *src, uint8_t *dst, uint32_t len, uint32_t x) {
    if (x >= len) return;
    const uint32_t n = len - x < 16 ? len - x : 16;
    if (len < 16) {  // a short range: exact pieces (rare for keys and values)
        Chunk c;
        chunk_load(c, src + x, n);
        chunk_store(c, dst + x, n);
        return;
    }
    uint64_t lo = (uint64_t)w.x | ((uint64_t)w.y << 32), hi = (uint64_t)w.z | ((uint64_t)w.w << 32);
    const uint32_t sh = 16 - n;  // bytes of the window before x (a tail window ends at len)
    if (sh >= 8) {
        lo = hi >> (8 * (sh - 8));
        hi = 0;
    } else if (sh) {
        lo = (lo >> (8 * sh)) | (hi << (64 - 8 * sh));
        hi >>= 8 * sh;
    }
    Chunk c;
    c.lo = lo;
    c.hi = hi;
    chunk_store_g(c, dst + x, n);
}
// lane chunk x of every listed entry's key and value bytes: all sixteen loads, then the stores
SDB_DEV void copy_group_chunks_kv(const CopyDesc *cd, uint32_t l, uint32_t x) {
    u32x4_u ck[8], cv[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) {
        const CopyDesc &c = cd[8 * q + (l >> 3)];
        ck[q] = chunk_ld(chunk_src(c.ks, c.kb, x));
        cv[q] = chunk_ld(chunk_src(c.vs, c.vb, x));
    }
    asm volatile("" ::: "memory");  // re-read the descriptors from LDS rather than hold 8 of them
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) {
        const CopyDesc &c = cd[8 * q + (l >> 3)];
        chunk_put(ck[q], c.ks, c.kd, c.kb, x);
        chunk_put(cv[q], c.vs, c.vd, c.vb, x);
    }
}
// lane chunk x of every listed entry's key (K) or value bytes: all eight loads, then the stores
template <bool K>
SDB_DEV void copy_group_chunks(const CopyDesc *cd, uint32_t l, uint32_t x) {
    u32x4_u ch[8];
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) {
        const CopyDesc &c = cd[8 * q + (l >> 3)];
        ch[q] = chunk_ld(chunk_src(K ? c.ks : c.vs, K ? c.kb : c.vb, x));
    }
    asm volatile("" ::: "memory");
#pragma unroll
    for (uint32_t q = 0; q < 8; q++) {
        const CopyDesc &c = cd[8 * q + (l >> 3)];
        chunk_put(ch[q], K ? c.ks : c.vs, K ? c.kd : c.vd, K ? c.kb : c.vb, x);
    }
}

// One merged entry's inputs, every load issued before any output store (the output may alias nothing
// the compiler can prove, so loads after a store would wait for it).
struct EntIn {
    const uint8_t *ks, *vs;
    uint64_t seq;
    uint32_t kb, vb, run, i;  // timestamps (rare) are read at the store from (run, i)
    uint8_t d, f;
};
SDB_DEV void ent_load(const MergeArgs &a, uint64_t p, EntIn &x) {
    x.d = 0;
    x.kb = x.vb = 0;
    if (p >= a.total) return;
    x.d = a.dec[p];
    const uint64_t g = a.perm[p];
    if (!x.d) return;
    x.run = run_of(a, g);
    const RunDesc &R = a.r[x.run];
    const uint64_t i = g - R.base;
    x.i = (uint32_t)i;
    x.f = R.flags[i];
    const uint64_t k0 = R.key_off[i], k1 = R.key_off[i + 1];
    x.ks = R.key_arena + k0;
    x.kb = (uint32_t)(k1 - k0);
    const uint32_t vl = R.val_len[i];
    x.vs = R.val_base + R.val_off[i];
    x.seq = R.seq[i];
    x.vb = (x.d == 1 && !(x.f & SDB_FLAG_TOMBSTONE)) ? vl : 0;
}

// Columns from each thread's kPerT consecutive positions; the key / value bytes then move half a tile at
// a time: every entry's copy descriptor goes to LDS and each wave copies a contiguous run of entries, so
// the output is written as one stream per wave (a thread's strided entries left lines half-written).
constexpr uint32_t kCopyHalf = kMergeTile / 2;

__global__ __launch_bounds__(kMergeThreads) void k_mg_emit(MergeArgs a) {
    if (a.out.summary->status != SDB_OK) return;
    __shared__ uint64_t s_w[17];
    __shared__ CopyDesc s_cd[kCopyHalf];
    const uint64_t p0 = (uint64_t)blockIdx.x * kMergeTile + (uint64_t)threadIdx.x * kPerT;
    EntIn x[kPerT];
#pragma unroll
    for (uint32_t u = 0; u < kPerT; u++) ent_load(a, p0 + u, x[u]);
    uint64_t c = 0, kb = 0, vb = 0, tot;
#pragma unroll
    for (uint32_t u = 0; u < kPerT; u++) {
        c += x[u].d != 0;
        kb += x[u].kb;
        vb += x[u].vb;
    }
    uint64_t j = a.tile_sum[3 * (uint64_t)blockIdx.x + 0] + block_excl_scan_u64(c, s_w, &tot);
    uint64_t ko = a.tile_sum[3 * (uint64_t)blockIdx.x + 1] + block_excl_scan_u64(kb, s_w, &tot);
    uint64_t vo = a.tile_sum[3 * (uint64_t)blockIdx.x + 2] + block_excl_scan_u64(vb, s_w, &tot);
    const sdb_merged_out &o = a.out;
    CopyDesc cds[kPerT];
#pragma unroll
    for (uint32_t u = 0; u < kPerT; u++) {
        CopyDesc &cd = cds[u];
        cd = CopyDesc{nullptr, nullptr, nullptr, nullptr, 0, 0};
        const EntIn &e = x[u];
        if (!e.d) continue;
        const bool tomb = e.d == 2 || (e.f & SDB_FLAG_TOMBSTONE);
        uint8_t mask = 0;
        if (e.f & SDB_FLAG_HAS_CREATE_TS) mask |= SDB_TS_CREATE;
        if ((e.f & SDB_FLAG_HAS_EXPIRE_TS) && e.d == 1) mask |= SDB_TS_EXPIRE;  // converted: expire_ts None
        {
        o.key_off[j] = ko;
        o.val_off[j] = vo;
        o.kind[j] = tomb ? SDB_KIND_TOMBSTONE : (e.f & SDB_FLAG_MERGE_OPERAND) ? SDB_KIND_MERGE : SDB_KIND_VALUE;
        o.seq[j] = e.seq;
        o.ts_mask[j] = mask;
        o.create_ts[j] = (mask & SDB_TS_CREATE) ? a.r[e.run].create_ts[e.i] : 0;
        o.expire_ts[j] = (mask & SDB_TS_EXPIRE) ? a.r[e.run].expire_ts[e.i] : 0;
        }
        cd.ks = e.ks;
        cd.kd = o.key_bytes + ko;
        cd.kb = e.kb;
        if (e.vb) {
            cd.vs = e.vs;
            cd.vd = o.val_bytes + vo;
            cd.vb = e.vb;
        }
        j++;
        ko += e.kb;
        vo += e.vb;
    }
    const uint32_t l = threadIdx.x & 63, w = threadIdx.x >> 6;
    constexpr uint32_t kPerWave = kCopyHalf / (kMergeThreads / 64);  // entries a wave copies per half
#pragma unroll
    for (uint32_t h = 0; h < kMergeTile / kCopyHalf; h++) {
#pragma unroll
        for (uint32_t u = 0; u < kPerT; u++) {
            const uint32_t idx = threadIdx.x * kPerT + u;  // position in the tile
            if (idx / kCopyHalf == h) s_cd[idx - h * kCopyHalf] = cds[u];
        }
        __syncthreads();
        for (uint32_t g = 0; g < kPerWave; g += 64) {
            // lanes 8q' .. 8q' + 7 copy entry 8q + q' of these 64; lane l's 16-byte chunks start at
            // 16 (l & 7) and step by 128 (entries over 128 bytes take more steps, wave-uniformly)
            const CopyDesc *cd = s_cd + w * kPerWave + g;
            const uint32_t mk = wave_max(cd[l].kb), mv = wave_max(cd[l].vb);
            const uint32_t mb = mk < mv ? mk : mv;  // chunk steps every entry's key and value share
            uint32_t x0 = 0;
            for (; x0 < mb; x0 += 128) copy_group_chunks_kv(cd, l, x0 + 16 * (l & 7));
            for (uint32_t xk = x0; xk < mk; xk += 128) copy_group_chunks<true>(cd, l, xk + 16 * (l & 7));
            for (uint32_t xv = x0; xv < mv; xv += 128) copy_group_chunks<false>(cd, l, xv + 16 * (l & 7));
        }
        __syncthreads();
    }
}

// ------------------------------------------------------------------------------------------------
// SST cuts: one lane walks the block chain the writer builds, restarting it after every cut.  A
// chain that enters a chunk (or a group of chunks) from the one before sits at one of the table
// entry points, so whole chunks / groups whose bytes keep the SST at or under max_sst_size are
// skipped with one lookup; near a cut the walk steps block by block through next() / bbytes.
// ------------------------------------------------------------------------------------------------
constexpr uint32_t kCutThreads = 256, kCutTab = 2048;
constexpr uint64_t kCutDone = ~1ull, kCutTables = 1ull << 62;  // staging requests: chunk k, or kCutTables | group g
__global__ __launch_bounds__(kCutThreads) void k_cut(SstSet P, uint64_t max_sst, uint64_t *cut, uint64_t *num,
                                                      const uint64_t *n_real) {
    // Thread 0 walks; the workgroup stages what the next steps read into LDS first: the group tables
    // (once), the chunk tables of the group the walk is in, and a chunk's next() / block bytes before
    // thread 0 steps block by block through it (one HBM round trip per table set or chunk instead of one
    // per step).  Tables larger than kCutTab entries stay in HBM.
    __shared__ uint32_t s_next[kChunk], s_bb[kChunk];
    __shared__ uint32_t s_gx[kCutTab], s_cx[kCutTab];
    __shared__ uint64_t s_gb[kCutTab], s_cb[kCutTab];
    __shared__ uint64_t s_stage;  // the next staging request (kCutDone: the walk is done)
    const EncodeArgs a = make_args(P, 0);
    // the walk ends at the stream's true length: every block that ends before it is the same in a padded
    // stream, the one that reaches it is the tail block (never counted), and a chunk / group skip past it
    // adds no cut in either stream
    const uint64_t n = n_real ? *n_real : a.n;
    const bool fast = *a.mode >= 1;  // 1 and 2: the chunk / group tables describe the chain
    const uint32_t W = *a.wmax, G = a.group, L = a.seg_look;
    const uint32_t K = a.nchunks, ngroups = (K + G - 1) / G;
    const bool glds = fast && (uint64_t)ngroups * W <= kCutTab, clds = fast && (uint64_t)G * W <= kCutTab;
    const uint32_t tid = threadIdx.x;
    if (glds)
        for (uint32_t x = tid; x < ngroups * W; x += kCutThreads) {
            const uint32_t g = x / W, o = x - g * W;
            s_gx[x] = a.gtab_exit[(uint64_t)g * L + o];
            s_gb[x] = a.gtab_bytes[(uint64_t)g * L + o];
        }
    __syncthreads();
    uint64_t e = 0, acc = 0, ns = 0;
    bool entry_pt = true;  // reached from the previous chunk (or the stream start): the tables apply
    uint64_t staged = ~0ull, gstaged = ~0ull;
    if (tid == 0) cut[0] = 0;
    for (;;) {
        if (tid == 0) {
            uint64_t want = kCutDone;
            while (e < n) {
                const uint64_t k = e / kChunk, o = e - k * kChunk;
                if (fast && entry_pt && o < W) {
                    const uint64_t g = k / G;
                    if (k % G == 0) {
                        uint64_t b;
                        uint32_t gx;
                        if (glds) {
                            b = s_gb[g * W + o];
                            gx = s_gx[g * W + o];
                        } else {
                            b = a.gtab_bytes[g * L + o];
                            gx = a.gtab_exit[g * L + o];
                        }
                        if (acc + b <= max_sst) {
                            acc += b;
                            e = (k + G) * kChunk + gx;
                            continue;
                        }
                    }
                    if (clds && gstaged != g) {  // the group is entered chunk by chunk: its tables to LDS
                        want = kCutTables | g;
                        break;
                    }
                    uint32_t ex;
                    uint64_t cb;
                    if (clds) {
                        ex = s_cx[(k - g * G) * W + o];
                        cb = s_cb[(k - g * G) * W + o];
                    } else {
                        ex = a.tab_exit[k * L + o];
                        cb = a.tab_bytes[k * L + o];
                    }
                    if (ex != 0xFFFFFFFFu && acc + cb <= max_sst) {
                        acc += cb;
                        e = ex;
                        continue;
                    }
                }
                if (staged != k) {  // the block steps of this chunk come from LDS
                    want = k;
                    break;
                }
                const uint64_t j = s_next[o];
                if (j >= n) {  // the tail block: built by close(), never counted
                    e = n;
                    break;
                }
                acc += s_bb[o];
                if (acc > max_sst) {
                    // entry j's add finished the block: the writer closes with j as its one-entry tail
                    if (j + 1 < n) cut[++ns] = j + 1;
                    acc = 0;
                    e = j + 1;
                    entry_pt = (e % kChunk) == 0;
                    continue;
                }
                entry_pt = j / kChunk != k;
                e = j;
            }
            s_stage = want;
        }
        __syncthreads();
        // the loop around the barriers exits on a scalar (wave-uniform) value
        const uint64_t sv = s_stage;
        const uint64_t want = (uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)sv) |
                              ((uint64_t)(uint32_t)__builtin_amdgcn_readfirstlane((int)(uint32_t)(sv >> 32)) << 32);
        if (want == kCutDone) break;
        if (want & kCutTables) {
            const uint64_t g = want & ~kCutTables, k0 = g * G, nk = k0 + G < K ? G : K - k0;
            for (uint32_t x = tid; x < nk * W; x += kCutThreads) {
                const uint32_t q = x / W, o = x - q * W;
                const uint64_t kk = k0 + q, ccs = kk * kChunk, cce = ccs + kChunk < n ? ccs + kChunk : n;
                // candidates past a short last chunk were never written: no table entry
                s_cx[x] = ccs + o < cce ? a.tab_exit[kk * L + o] : 0xFFFFFFFFu;
                s_cb[x] = ccs + o < cce ? a.tab_bytes[kk * L + o] : 0;
            }
            gstaged = g;
        } else {
            const uint64_t cs = want * kChunk, ce = cs + kChunk < n ? cs + kChunk : n;
            for (uint64_t x = cs + tid; x < ce; x += kCutThreads) {
                s_next[x - cs] = a.next[x];
                s_bb[x - cs] = a.bbytes[x];
            }
            staged = want;
        }
        __syncthreads();
    }
    if (tid == 0) {
        if (n) cut[++ns] = n;
        *num = ns;
    }
}

// The key / value byte offset of every cut; the cut count is read on the device (the host learns it
// with the offsets, in one synchronisation).
__global__ void k_cut_offsets(const uint64_t *cut, const uint64_t *num, const uint64_t *key_off, const uint64_t *val_off,
                              uint64_t *out) {
    const uint64_t ns = *num;
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= ns; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint64_t c = cut[i];
        out[2 * i] = key_off[c];
        out[2 * i + 1] = val_off[c];
    }
}

// ------------------------------------------------------------------------------------------------
// sdb_compactor_run_ssts: the input SSTs' blocks as one decode, the gate between decode and merge, and
// the padding of the merged stream for the cut walk.
// ------------------------------------------------------------------------------------------------
__global__ void k_cx_blocks(CxInputs in, uint64_t *start, uint64_t *end) {
    const uint64_t nb = in.nblocks;
    for (uint64_t k = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; k < nb; k += (uint64_t)gridDim.x * blockDim.x) {
        uint32_t lo = 0, hi = in.n - 1;  // the input holding block k: last first_block <= k
        while (lo < hi) {
            const uint32_t mid = (lo + hi + 1) >> 1;
            if (in.first_block[mid] <= k) lo = mid;
            else hi = mid - 1;
        }
        const uint64_t j = k - in.first_block[lo], d = (uint64_t)(uintptr_t)in.data[lo] - in.base;
        start[k] = d + in.block_off[lo][j];
        end[k] = d + in.block_off[lo][j + 1];
    }
}

// ~0 when the decode succeeded and agrees with the declared counts; else the decode's first failure
// (block << 8 | status), or SDB_INVALID_ARGUMENT at the first run whose boundary disagrees
__global__ void k_cx_gate(CxInputs in, const sdb_decode_summary *dsum, const unsigned long long *dec_err,
                          const uint64_t *bes, unsigned long long *gate) {
    if (threadIdx.x) return;
    unsigned long long g = ~0ull;
    if (dsum->status != SDB_OK) {
        g = *dec_err != ~0ull ? *dec_err : (unsigned long long)(uint32_t)dsum->status;
    } else if (dsum->num_entries != in.run_entry[in.nruns] || dsum->key_bytes != in.key_bytes) {
        g = SDB_INVALID_ARGUMENT;
    } else {
        for (uint32_t r = 0; r < in.nruns; r++)
            if (bes[in.run_block[r]] != in.run_entry[r]) {
                g = ((unsigned long long)in.run_block[r] << 8) | SDB_INVALID_ARGUMENT;
                break;
            }
    }
    *gate = g;
}

// RowFlags and value lengths of a merged stream (kind + ts_mask, val_off[i + 1] - val_off[i]).
__global__ void k_mg_asrun(sdb_merged_out o, uint64_t n, uint32_t *val_len, uint8_t *flags) {
    for (uint64_t i = (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i < n; i += (uint64_t)gridDim.x * blockDim.x) {
        const uint8_t k = o.kind[i], m = o.ts_mask[i];
        flags[i] = (uint8_t)((k == SDB_KIND_TOMBSTONE ? SDB_FLAG_TOMBSTONE : 0) | (k == SDB_KIND_MERGE ? SDB_FLAG_MERGE_OPERAND : 0) |
                             ((m & SDB_TS_EXPIRE) ? SDB_FLAG_HAS_EXPIRE_TS : 0) | ((m & SDB_TS_CREATE) ? SDB_FLAG_HAS_CREATE_TS : 0));
        val_len[i] = (uint32_t)(o.val_off[i + 1] - o.val_off[i]);
    }
}

__global__ void k_mg_pad(sdb_merged_out o, uint64_t cap) {
    const sdb_merge_summary *sm = o.summary;
    const bool ok = sm->status == SDB_OK;
    // from the first padding entry (its offset slot num_out already holds the totals: rewritten with the
    // same value); a failed merge: the whole stream is empty entries
    const uint64_t from = ok ? sm->num_out : 0;
    const uint64_t kt = ok ? sm->key_bytes : 0, vt = ok ? sm->val_bytes : 0;
    for (uint64_t i = from + (uint64_t)blockIdx.x * blockDim.x + threadIdx.x; i <= cap;
         i += (uint64_t)gridDim.x * blockDim.x) {
        o.key_off[i] = kt;
        o.val_off[i] = vt;
        if (i < cap) {
            o.kind[i] = SDB_KIND_VALUE;
            o.seq[i] = 0;
            o.ts_mask[i] = 0;
        }
    }
}

}  // namespace

hipError_t launch_merged_as_run(const sdb_merged_out &out, uint64_t n, uint32_t *val_len, uint8_t *flags, hipStream_t st) {
    if (n) {
        const uint64_t g = (n + 255) / 256;
        hipLaunchKernelGGL(k_mg_asrun, dim3((uint32_t)(g < 4096 ? g : 4096)), dim3(256), 0, st, out, n, val_len, flags);
    }
    return hipGetLastError();
}

hipError_t launch_cx_blocks(const CxInputs &in, uint64_t *start, uint64_t *end, hipStream_t st) {
    const uint64_t nb = in.nblocks;
    if (nb) {
        uint64_t g = (nb + 255) / 256;
        hipLaunchKernelGGL(k_cx_blocks, dim3((uint32_t)(g < 2048 ? g : 2048)), dim3(256), 0, st, in, start, end);
    }
    return hipGetLastError();
}

hipError_t launch_cx_gate(const CxInputs &in, const sdb_decode_summary *dsum, const unsigned long long *dec_err,
                          const uint64_t *block_entry_start, unsigned long long *gate, hipStream_t st) {
    hipLaunchKernelGGL(k_cx_gate, dim3(1), dim3(64), 0, st, in, dsum, dec_err, block_entry_start, gate);
    return hipGetLastError();
}

hipError_t launch_merge_pad(const sdb_merged_out &out, uint64_t cap, hipStream_t st) {
    hipLaunchKernelGGL(k_mg_pad, dim3(256), dim3(256), 0, st, out, cap);
    return hipGetLastError();
}

hipError_t launch_cut_offsets(const uint64_t *cut, const uint64_t *num, const uint64_t *key_off, const uint64_t *val_off,
                              uint64_t *out, hipStream_t st) {
    hipLaunchKernelGGL(k_cut_offsets, dim3(64), dim3(256), 0, st, cut, num, key_off, val_off, out);
    return hipGetLastError();
}

sdb_status build_merge_args(const sdb_run *runs, uint32_t nruns, const sdb_retention *ret, const sdb_merged_out *out,
                            void *workspace, uint64_t workspace_bytes, MergeArgs *pa, bool raw) {
    if (nruns > kMaxRuns) return SDB_LIMIT_EXCEEDED;  // per call (the compactor merges more in groups)
    if ((nruns && !runs) || !ret || !out || !out->summary || !out->key_off || !out->val_off || !pa)
        return SDB_INVALID_ARGUMENT;
    MergeArgs &a = *pa;
    a = MergeArgs{};
    a.nruns = nruns;
    a.raw = raw ? 1u : 0u;
    uint64_t total = 0;
    for (uint32_t r = 0; r < nruns; r++) {
        const sdb_run &R = runs[r];
        if (R.n && (!R.key_arena || !R.key_off || !R.val_off || !R.val_len || !R.seq || !R.flags))
            return SDB_INVALID_ARGUMENT;
        RunDesc &d = a.r[r];
        d.n = R.n;
        d.base = total;
        d.key_arena = R.key_arena;
        d.key_off = R.key_off;
        d.val_base = R.val_base;
        d.val_off = R.val_off;
        d.val_len = R.val_len;
        d.seq = R.seq;
        d.flags = R.flags;
        d.create_ts = R.create_ts;
        d.expire_ts = R.expire_ts;
        total += R.n;
    }
    if (total >= (1ull << 40)) return SDB_LIMIT_EXCEEDED;
    if (total && (!out->kind || !out->seq || !out->create_ts || !out->expire_ts || !out->ts_mask)) return SDB_INVALID_ARGUMENT;
    const MergeWorkspace w = merge_workspace_layout(total);
    if (!workspace || workspace_bytes < w.total + 256) return SDB_INVALID_ARGUMENT;
    uint8_t *ws = (uint8_t *)(((uintptr_t)workspace + 255) & ~(uintptr_t)255);
    a.total = total;
    a.ntiles = (uint32_t)((total + kMergeTile - 1) / kMergeTile);
    a.ret = *ret;
    a.out = *out;
    a.pfx = (uint64_t *)(ws + w.pfx);
    a.perm = (uint64_t *)(ws + w.perm);
    a.start = ws + w.start;
    a.dec = ws + w.dec;
    a.tile_sum = (uint64_t *)(ws + w.tile_sum);
    a.bound = (uint64_t *)(ws + w.bound);
    a.err = (unsigned long long *)(ws + w.err);
    a.err_merge = (unsigned long long *)(ws + w.err_merge);
    a.metric = (unsigned long long *)(ws + w.metric);
    a.lcp0 = (uint32_t *)(ws + w.lcp0);
    return SDB_OK;
}

hipError_t launch_merge(const MergeArgs &a, bool emit, hipStream_t st) {
    if (hipMemsetAsync(a.err, 0xFF, 8, st) != hipSuccess || hipMemsetAsync(a.err_merge, 0xFF, 8, st) != hipSuccess ||
        hipMemsetAsync(a.metric, 0, 16, st) != hipSuccess)
        return hipErrorUnknown;
    const uint32_t gb = (uint32_t)((a.total + kPfxThreads - 1) / kPfxThreads);
    if (gb) {
        hipLaunchKernelGGL(k_mg_lcp0, dim3(1), dim3(256), 0, st, a);
        hipLaunchKernelGGL(k_mg_prefix, dim3(gb), dim3(kPfxThreads), 0, st, a);
        const uint64_t nb = (uint64_t)gb * 2 * a.nruns;
        hipLaunchKernelGGL(k_mg_bounds, dim3((uint32_t)((nb + 255) / 256)), dim3(256), 0, st, a);
        hipLaunchKernelGGL(k_mg_rank, dim3(gb), dim3(kPfxThreads), 0, st, a);
        hipLaunchKernelGGL(k_mg_keys, dim3(gb), dim3(kPfxThreads), 0, st, a);
    }
    hipLaunchKernelGGL(k_mg_scan, dim3(1), dim3(kMergeThreads), 0, st, a);
    if (emit && a.ntiles) hipLaunchKernelGGL(k_mg_emit, dim3(a.ntiles), dim3(kMergeThreads), 0, st, a);
    return hipGetLastError();
}

// The emit alone, after launch_merge(a, false) sized the output with unbounded capacities (the
// caller then points a.out at buffers of exactly the reported sizes).
hipError_t launch_merge_emit(const MergeArgs &a, hipStream_t st) {
    if (a.ntiles) hipLaunchKernelGGL(k_mg_emit, dim3(a.ntiles), dim3(kMergeThreads), 0, st, a);
    return hipGetLastError();
}

hipError_t launch_cuts(const SstSet &P, uint64_t max_sst_size, uint64_t *cut, uint64_t cap, uint64_t *num,
                       hipStream_t st, const uint64_t *n_real) {
    (void)cap;  // the host checks cap >= n + 1
    hipError_t e = launch_encode_prep(P, st);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_cut, dim3(1), dim3(kCutThreads), 0, st, P, max_sst_size, cut, num, n_real);
    return hipGetLastError();
}

}  // namespace sdb
