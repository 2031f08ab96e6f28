// sdb_footer.cpp — host builder of the SST footer (filter block, index block, stats block,
// SsTableInfo, meta offset, version) that follows the data section written by sdb_encode_sst.
//
// Replaces EncodedSsTableFooterBuilder::build (slatedb/src/format/sst.rs:383-487) together with the
// index the reference accumulates block by block in EncodedSsTableBuilder (sst_builder.rs:228-237,
// 307-313) or EncodedWalSsTableBuilder (wal/slatedb/sst_builder.rs:129-205), SstStats::encode
// (sst_stats.rs:52-86) and SsTableInfo::encode (format/sst.rs:195-199, flatbuffer_types.rs:775-800).
//
// The bytes are those of the `flatbuffers` crate 25.12.19 (the reference's Cargo.lock) driven in the
// reference's creation order: the buffer is filled back to front, scalars equal to their schema
// default are omitted, every push pads to its own size, vtables follow the table's soffset and are
// shared when byte-identical, and `finish` pads the root offset to the largest alignment seen.
// Field add order per table = the generated create() functions (generated/root_generated.rs:
// 1238-1255 SsTableInfo, 1497-1506 BlockStats, 1631-1643 SstStats, 1809-1817 BlockMeta,
// 1923-1930 SsTableIndex).  Host code: a footer is O(num_blocks) small writes (≈ 1 MB for a
// 64 MiB SST), produced after the device encode from its per-block outputs.
#include <cstdint>
#include <cstring>
#include <utility>
#include <thread>
#include <vector>
#if defined(__x86_64__)
#include <immintrin.h>
#endif

#include "../../include/slatedb_amd.h"

namespace sdb {
void host_compress(uint32_t codec, const uint8_t *in, uint64_t n, std::vector<uint8_t> &o);  // sdb_host_codec.cpp
}

namespace {

// crc32fast::hash (IEEE, reflected, init/xorout 0xFFFFFFFF) on the host: carry-less multiply folding
// (PCLMULQDQ, four 128-bit lanes, then Barrett reduction) where the CPU has it, slicing-by-8 otherwise.
// A D1 footer checksums ~1.7 MB (bitmap, index, stats): 1.3 ms by tables, ~0.1 ms folded.
struct HostCrc {
    uint32_t t[8][256];
    bool clmul;
    HostCrc() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; i++)
            for (int s = 1; s < 8; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
#if defined(__x86_64__)
        clmul = __builtin_cpu_supports("pclmul") && __builtin_cpu_supports("sse4.1");
#else
        clmul = false;
#endif
    }
    uint32_t update_tab(uint32_t c, const uint8_t *p, size_t n) const {  // raw register update
        while (n >= 8) {
            uint32_t lo, hi;
            memcpy(&lo, p, 4);
            memcpy(&hi, p + 4, 4);
            lo ^= c;
            c = t[7][lo & 0xFF] ^ t[6][(lo >> 8) & 0xFF] ^ t[5][(lo >> 16) & 0xFF] ^ t[4][lo >> 24] ^
                t[3][hi & 0xFF] ^ t[2][(hi >> 8) & 0xFF] ^ t[1][(hi >> 16) & 0xFF] ^ t[0][hi >> 24];
            p += 8;
            n -= 8;
        }
        while (n--) c = (c >> 8) ^ t[0][(c ^ *p++) & 0xFF];
        return c;
    }
    uint32_t update(uint32_t c, const uint8_t *p, size_t n) const;
    uint32_t operator()(const uint8_t *p, size_t n) const { return ~update(0xFFFFFFFFu, p, n); }
};

#if defined(__x86_64__)
__attribute__((target("pclmul,sse4.1"))) inline __m128i clmul_fold(__m128i a, __m128i b, __m128i k) {
    const __m128i lo = _mm_clmulepi64_si128(a, k, 0x00), hi = _mm_clmulepi64_si128(a, k, 0x11);
    return _mm_xor_si128(_mm_xor_si128(hi, lo), b);
}
// The raw register after `n` >= 64 bytes (a multiple of 16 folded, the rest by table).  Constants:
// x^(k) mod P for the 512- and 128-bit folds, the 64 -> 32 bit fold and Barrett's mu / P (reflected).
__attribute__((target("pclmul,sse4.1"))) uint32_t clmul_update(const HostCrc &h, uint32_t crc, const uint8_t *p,
                                                                size_t n) {
    const __m128i k1k2 = _mm_set_epi64x(0x1c6e41596ll, 0x154442bd4ll);
    const __m128i k3k4 = _mm_set_epi64x(0x0ccaa009ell, 0x1751997d0ll);
    const __m128i k5 = _mm_set_epi64x(0, 0x163cd6124ll);
    const __m128i poly = _mm_set_epi64x(0x1F7011641ll, 0x1DB710641ll);
    const __m128i mask32 = _mm_set_epi32(0, 0, 0, -1);
    auto ld = [](const uint8_t *q) { return _mm_loadu_si128((const __m128i *)q); };
    __m128i x1 = _mm_xor_si128(ld(p), _mm_cvtsi32_si128((int)crc)), x2 = ld(p + 16), x3 = ld(p + 32), x4 = ld(p + 48);
    p += 64;
    n -= 64;
    for (; n >= 64; p += 64, n -= 64) {
        x1 = clmul_fold(x1, ld(p), k1k2);
        x2 = clmul_fold(x2, ld(p + 16), k1k2);
        x3 = clmul_fold(x3, ld(p + 32), k1k2);
        x4 = clmul_fold(x4, ld(p + 48), k1k2);
    }
    x1 = clmul_fold(clmul_fold(clmul_fold(x1, x2, k3k4), x3, k3k4), x4, k3k4);
    for (; n >= 16; p += 16, n -= 16) x1 = clmul_fold(x1, ld(p), k3k4);
    x1 = _mm_xor_si128(_mm_srli_si128(x1, 8), _mm_clmulepi64_si128(x1, k3k4, 0x10));  // 128 -> 64 (+ 32 zero bits)
    __m128i hi = _mm_srli_si128(x1, 4);
    x1 = _mm_xor_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), k5, 0x00), hi);  // -> 64
    hi = x1;  // Barrett 64 -> 32
    x1 = _mm_and_si128(_mm_clmulepi64_si128(_mm_and_si128(x1, mask32), poly, 0x10), mask32);
    x1 = _mm_xor_si128(_mm_clmulepi64_si128(x1, poly, 0x00), hi);
    return h.update_tab((uint32_t)_mm_extract_epi32(x1, 1), p, n);
}
#endif

uint32_t HostCrc::update(uint32_t c, const uint8_t *p, size_t n) const {
#if defined(__x86_64__)
    if (clmul && n >= 64) return clmul_update(*this, c, p, n);
#endif
    return update_tab(c, p, n);
}
const HostCrc &host_crc() {
    static const HostCrc c;
    return c;
}

// Back-to-front flatbuffer writer.  Positions are "reverse offsets": bytes from the end of the
// finished buffer, which do not move when the buffer grows.
class BackWriter {
  public:
    // `storage` is reused across calls (a thread's scratch): its bytes are not assumed zero, every byte
    // taken below head is written, padding included
    BackWriter(std::vector<uint8_t> &storage, size_t cap) : buf_(storage) {
        if (buf_.size() < cap) buf_.resize(cap);
        head_ = buf_.size();
    }
    uint32_t rev() const { return (uint32_t)(buf_.size() - head_); }

    void pad_for(size_t len, size_t align) {  // room for `len` bytes that must end `align`-aligned
        if (align > max_align_) max_align_ = align;
        const size_t p = ((size_t)0 - (rev() + len)) & (align - 1);
        reserve(p);
        memset(&buf_[head_], 0, p);
    }
    template <class T>
    uint32_t scalar(T v) {
        pad_for(sizeof(T), sizeof(T));
        reserve(sizeof(T));
        memcpy(&buf_[head_], &v, sizeof(T));  // little-endian host
        return rev();
    }
    uint32_t uoffset(uint32_t target) {
        pad_for(4, 4);
        reserve(4);
        const uint32_t v = rev() - target;
        memcpy(&buf_[head_], &v, 4);
        return rev();
    }
    uint32_t bytes_vector(const uint8_t *p, size_t n) {
        pad_for(n, 4);
        reserve(n);
        if (n) memcpy(&buf_[head_], p, n);
        return scalar<uint32_t>((uint32_t)n);
    }
    uint32_t offsets_vector(const std::vector<uint32_t> &targets) {
        const size_t n = targets.size();
        pad_for(4 * n, 4);
        reserve(4 * n);
        const uint32_t top = rev();
        for (size_t i = 0; i < n; i++) {
            const uint32_t v = top - 4 * (uint32_t)i - targets[i];
            memcpy(&buf_[head_ + 4 * i], &v, 4);
        }
        return scalar<uint32_t>((uint32_t)n);
    }

    // tables
    uint32_t begin() {
        nf_ = 0;
        return rev();
    }
    template <class T>
    void field(uint16_t slot, T v) {  // omitted when equal to the default (0 for every field here)
        if (v != 0) fields_[nf_++] = {slot, scalar<T>(v)};
    }
    void field_offset(uint16_t slot, uint32_t target) { fields_[nf_++] = {slot, uoffset(target)}; }
    uint32_t end(uint32_t tail) {
        const uint32_t obj = scalar<uint32_t>(0);  // soffset to the vtable, patched below
        uint16_t vlen = 4;
        for (uint32_t i = 0; i < nf_; i++) vlen = fields_[i].slot + 2 > vlen ? (uint16_t)(fields_[i].slot + 2) : vlen;
        VTable vt;
        memset(vt.b, 0, vlen);
        vt.len = vlen;
        const uint16_t hdr[2] = {vlen, (uint16_t)(obj - tail)};
        memcpy(vt.b, hdr, 4);
        for (uint32_t i = 0; i < nf_; i++) {
            const uint16_t d = (uint16_t)(obj - fields_[i].rev);
            memcpy(vt.b + fields_[i].slot, &d, 2);
        }
        nf_ = 0;
        return link_vtable(obj, vt.b, vlen);
    }
    // The index loop's body, byte for byte what bytes_vector(key) + begin + field<u64>(4, off) +
    // field_offset(6, key) + end write, with one capacity check (a D1 index has 17,016 of them).
    uint32_t block_meta(uint64_t off, const uint8_t *key, uint32_t n) {
        ensure(n + 48);
        uint8_t *const e = buf_.data() + buf_.size();
        uint32_t r = rev();
        if (max_align_ < 4) max_align_ = 4;
        const uint32_t p0 = (0u - (r + n)) & 3u;  // the key vector: bytes, then its u32 length
        memset(e - r - 4, 0, 4);  // the padding (bytes below it are written next)
        r += p0;
        if (n <= 16) {
            for (uint32_t i = 0; i < n; i++) e[(int64_t)i - r - n] = key[i];
        } else {
            memcpy(e - r - n, key, n);
        }
        r += n;
        memcpy(e - r - 4, &n, 4);
        r += 4;
        const uint32_t keyr = r, tail = r;
        uint32_t f4 = 0;
        if (off) {  // BlockMeta.offset (omitted when 0)
            if (max_align_ < 8) max_align_ = 8;
            const uint32_t p8 = (0u - (r + 8)) & 7u;
            memset(e - r - 8, 0, 8);
            r += p8;
            memcpy(e - r - 8, &off, 8);
            r += 8;
            f4 = r;
        }
        // BlockMeta.first_key, then the soffset: r is 4-aligned here (no padding)
        const uint32_t ko = r + 4 - keyr;
        memcpy(e - r - 4, &ko, 4);
        r += 4;
        const uint32_t f6 = r;
        memset(e - r - 4, 0, 4);  // the soffset, patched by link_vtable
        r += 4;
        head_ = buf_.size() - r;
        const uint16_t vt[4] = {8, (uint16_t)(r - tail), (uint16_t)(f4 ? r - f4 : 0), (uint16_t)(r - f6)};
        return link_vtable(r, (const uint8_t *)vt, 8);
    }
    // The stats loop's body: BlockStats{puts, deletes, merges} as begin + field<u16>(8), (6), (4) + end.
    uint32_t block_stats(uint16_t puts, uint16_t dels, uint16_t merges) {
        ensure(32);
        uint8_t *const e = buf_.data() + buf_.size();
        uint32_t r = rev();
        const uint32_t tail = r;
        uint32_t f[3] = {0, 0, 0};
        const uint16_t v[3] = {merges, dels, puts};
        for (int i = 0; i < 3; i++)
            if (v[i]) {
                if (max_align_ < 2) max_align_ = 2;
                if (r & 1u) e[-(int64_t)++r] = 0;
                memcpy(e - r - 2, &v[i], 2);
                r += 2;
                f[i] = r;
            }
        if (max_align_ < 4) max_align_ = 4;
        const uint32_t p4 = (0u - (r + 4)) & 3u;
        memset(e - r - 8, 0, 8);
        r += p4 + 4;
        head_ = buf_.size() - r;
        const uint16_t vlen = merges ? 10 : dels ? 8 : puts ? 6 : 4;
        const uint16_t vt[5] = {vlen, (uint16_t)(r - tail), (uint16_t)(f[2] ? r - f[2] : 0),
                                (uint16_t)(f[1] ? r - f[1] : 0), (uint16_t)(f[0] ? r - f[0] : 0)};
        return link_vtable(r, (const uint8_t *)vt, vlen);
    }
    // finish(root, None): pad so the root uoffset ends aligned to the largest alignment seen
    void finish(uint32_t root, const uint8_t **data, uint64_t *len) {
        vtables_.clear();
        hit_ = 0;
        pad_for(4, max_align_);
        uoffset(root);
        *data = &buf_[head_];
        *len = buf_.size() - head_;
    }

  private:
    // the table at `obj` gets the vtable `vb[0, vlen)`: an identical one written before, else this one
    // (a footer has a handful of distinct vtables, one per padding pattern: linear search, most recent first)
    uint32_t link_vtable(uint32_t obj, const uint8_t *vb, uint16_t vlen) {
        auto same = [&](const VTable &t) {
            if (t.len != vlen) return false;
            for (uint16_t i = 0; i < vlen; i += 2)
                if (t.b[i] != vb[i] || t.b[i + 1] != vb[i + 1]) return false;
            return true;
        };
        uint32_t vt_rev = 0;
        bool found = false;
        if (hit_ < vtables_.size() && same(vtables_[hit_])) {  // the block loops alternate a few vtables
            vt_rev = vtables_[hit_].rev;
            found = true;
        } else {
            for (size_t i = vtables_.size(); i-- > 0;)
                if (same(vtables_[i])) {
                    vt_rev = vtables_[i].rev;
                    found = true;
                    hit_ = i;
                    break;
                }
        }
        if (!found) {
            reserve(vlen);
            memcpy(&buf_[head_], vb, vlen);
            VTable vt;
            memcpy(vt.b, vb, vlen);
            vt.len = vlen;
            vt_rev = vt.rev = rev();
            vtables_.push_back(vt);
        }
        const int32_t so = (int32_t)vt_rev - (int32_t)obj;
        memcpy(&buf_[buf_.size() - obj], &so, 4);
        return obj;
    }
    void ensure(size_t n) {  // room for n more bytes below head (reserve without taking them)
        reserve(n);
        head_ += n;
    }
    struct Field {
        uint16_t slot;
        uint32_t rev;
    };
    struct VTable {
        uint8_t b[32];  // widest vtable here: SsTableInfo, 26 bytes
        uint16_t len;
        uint32_t rev;
    };
    void reserve(size_t n) {
        if (__builtin_expect(head_ < n, 0)) grow(n);
        head_ -= n;  // the caller writes all n bytes
    }
    __attribute__((noinline)) void grow(size_t n) {
        {
            size_t cap = buf_.size();
            const size_t used = cap - head_;
            while (cap - used < n) cap = cap ? 2 * cap : 1024;
            std::vector<uint8_t> nb(cap);
            memcpy(&nb[cap - used], &buf_[head_], used);
            buf_.swap(nb);
            head_ = cap - used;
        }
    }
    std::vector<uint8_t> &buf_;
    size_t head_;
    size_t max_align_ = 1;
    Field fields_[16];  // the widest table here has 11 fields
    uint32_t nf_ = 0;
    std::vector<VTable> vtables_;
    size_t hit_ = 0;
};

uint8_t *put_be(uint8_t *o, uint64_t v, int nbytes) {
    for (int i = nbytes - 1; i >= 0; i--) *o++ = (uint8_t)(v >> (8 * i));
    return o;
}

// compress_and_transform's codec step for the footer's blocks (format/sst.rs:557-594): a literal-only
// stream of the format — the stored / raw form every decoder of it reads (zlib: stored deflate blocks +
// Adler-32; zstd: a frame of raw blocks with Frame_Content_Size; lz4: one literal sequence after the u32 LE
// length; snappy: the varint length and one literal element).  Appended to `o`.
void literal_stream(uint32_t codec, const uint8_t *in, uint64_t n, std::vector<uint8_t> &o) {
    auto le = [&](uint64_t v, int nb) {
        for (int i = 0; i < nb; i++) o.push_back((uint8_t)(v >> (8 * i)));
    };
    if (codec == SDB_CODEC_LZ4) {
        le(n, 4);
        o.push_back((uint8_t)((n >= 15 ? 15 : n) << 4));
        if (n >= 15) {
            uint64_t x = n - 15;
            for (; x >= 255; x -= 255) o.push_back(255);
            o.push_back((uint8_t)x);
        }
        o.insert(o.end(), in, in + n);
    } else if (codec == SDB_CODEC_SNAPPY) {
        for (uint64_t x = n;; x >>= 7) {
            o.push_back((uint8_t)(x >= 0x80 ? (x & 0x7F) | 0x80 : x));
            if (x < 0x80) break;
        }
        if (n) {
            const uint64_t v = n - 1;
            const int nb = v < 60 ? 0 : v < 256 ? 1 : v < 65536 ? 2 : v < (1u << 24) ? 3 : 4;
            o.push_back((uint8_t)((nb ? 59 + nb : v) << 2));
            le(v, nb);
            o.insert(o.end(), in, in + n);
        }
    } else if (codec == SDB_CODEC_ZLIB) {
        o.push_back(0x78);
        o.push_back(0x9C);
        uint64_t a = 1, b = 0, done = 0;
        for (uint64_t i = 0; i < n; i++) {
            a = (a + in[i]) % 65521;
            b = (b + a) % 65521;
        }
        do {
            const uint64_t c = n - done < 65535 ? n - done : 65535;
            o.push_back(done + c == n ? 1 : 0);
            le(c, 2);
            le(~c & 0xFFFF, 2);
            o.insert(o.end(), in + done, in + done + c);
            done += c;
        } while (done < n);
        put_be(&*o.insert(o.end(), 4, 0), (b << 16) | a, 4);
    } else {  // zstd
        le(0xFD2FB528u, 4);
        if (n < 256) {
            o.push_back(0x20);
            le(n, 1);
        } else if (n < 65536 + 256) {
            o.push_back(0x60);
            le(n - 256, 2);
        } else {
            o.push_back(0xA0);
            le(n, 4);
        }
        uint64_t done = 0;
        do {
            const uint64_t c = n - done < (128u << 10) ? n - done : (128u << 10);
            le((done + c == n ? 1u : 0u) | (c << 3), 3);  // Raw_Block
            o.insert(o.end(), in + done, in + done + c);
            done += c;
        } while (done < n);
    }
}

// A thread's reusable buffers: a footer is ~1.7 MB of flatbuffer bytes for a D1 SST, and fresh buffers
// cost it a page fault per 4 KiB on every call.
struct FooterScratch {
    std::vector<uint8_t> index, stats, info;
    std::vector<uint32_t> metas, tabs;
};

}  // namespace

extern "C" uint64_t sdb_sst_footer_bound(const sdb_footer_in *in) {
    if (!in) return 0;
    const uint64_t nb = in->num_blocks;
    const uint64_t keys = nb && in->first_key_off ? in->first_key_off[nb] - in->first_key_off[0] : 0;
    uint64_t b = 256 + in->first_entry_len + in->last_entry_len;  // SsTableInfo, crcs, trailer
    if (in->has_filter) b += 32 + in->bloom_len + (in->filter_name ? strlen(in->filter_name) : 3);  // composite filter block
    b += 64 + keys + 48 * nb;                                      // index: key, len, pads, BlockMeta, vtable, slot
    if (in->stats) b += 128 + 32 * nb;                             // stats: BlockStats tables + vector
    if (in->compression) b += b / 64 + 256;                        // the codecs' framing (literal streams)
    return b;
}

extern "C" sdb_status sdb_sst_footer(const sdb_footer_in *in, uint8_t *out, uint64_t cap,
                                     uint64_t *len) {
    if (!in || !len) return SDB_INVALID_ARGUMENT;
    const uint64_t nb = in->num_blocks;
    if (nb && (!in->block_off || !in->first_key_off || !in->first_key_bytes)) return SDB_INVALID_ARGUMENT;
    if (in->stats && nb && !in->block_stats) return SDB_INVALID_ARGUMENT;
    if (in->has_filter && in->bloom_len && !in->bloom) return SDB_INVALID_ARGUMENT;
    if (in->sst_type > 1 || in->compression > SDB_CODEC_ZSTD) return SDB_INVALID_ARGUMENT;
    for (uint64_t k = 0; k < nb; k++)
        if (in->first_key_off[k + 1] < in->first_key_off[k]) return SDB_INVALID_ARGUMENT;
    const HostCrc &crc = host_crc();
    const uint64_t base = in->data_len;
    // the caller's thread-local scratch, bound by reference: the stats lambda may run on a worker thread,
    // and a lambda names a thread_local directly (it is not captured), so it must see this reference
    thread_local FooterScratch tl_sc;
    FooterScratch &sc = tl_sc;

    // 1. composite filter block [u16 count][u16 name_len]["_bf"][u64 len][Filter::encode]
    //    (format/sst.rs:394-421; Filter::encode = u16 BE num_probes ++ bitmap, filter.rs:177-180)
    const uint64_t filter_offset = base;
    uint64_t filter_len = 0;
    const char *name = in->filter_name ? in->filter_name : "_bf";
    const size_t nl = strlen(name);
    std::vector<uint8_t> fh;
    if (in->has_filter) {
        if (nl > 0xFFFF) return SDB_INVALID_ARGUMENT;
        fh.resize(14 + nl);
        uint8_t *q = put_be(fh.data(), 1, 2);
        q = put_be(q, nl, 2);
        memcpy(q, name, nl);
        q = put_be(q + nl, in->bloom_len + 2, 8);
        put_be(q, in->num_probes, 2);
        filter_len = fh.size() + in->bloom_len + 4;
    }

    // 2. index: per block the first_key vector then its BlockMeta (creation order of the reference);
    // 3. stats (SstStats::encode): BlockStats tables, their vector, then SstStats.  Built side by side
    //    on two threads for large SSTs (they are independent until the offsets in SsTableInfo).
    const uint8_t *idx_p = nullptr, *st_p = nullptr;
    uint64_t idx_n = 0, st_n = 0;
    uint32_t idx_crc = 0, st_crc = 0;
    auto build_index = [&]() {
        BackWriter w(sc.index, 64 + nb * 48);
        sc.metas.resize(nb);
        for (uint64_t k = 0; k < nb; k++) {
            const uint64_t a = in->first_key_off[k], b = in->first_key_off[k + 1];
            sc.metas[k] = w.block_meta(in->block_off[k], in->first_key_bytes + a, (uint32_t)(b - a));
        }
        const uint32_t vec = w.offsets_vector(sc.metas);
        const uint32_t t = w.begin();
        w.field_offset(4, vec);  // SsTableIndex.block_meta
        w.finish(w.end(t), &idx_p, &idx_n);
        idx_crc = crc(idx_p, idx_n);
    };
    auto build_stats = [&]() {
        BackWriter w(sc.stats, 128 + nb * 24);
        sc.tabs.resize(nb);
        for (uint64_t k = 0; k < nb; k++) {
            const uint16_t *s = in->block_stats + 3 * k;
            sc.tabs[k] = w.block_stats(s[0], s[1], s[2]);  // fields added merges, deletes, puts
        }
        uint32_t vec = 0;
        if (nb) vec = w.offsets_vector(sc.tabs);
        const sdb_sst_summary *s = in->stats;
        const uint32_t t = w.begin();
        w.field<uint64_t>(12, s->raw_val_size);
        w.field<uint64_t>(10, s->raw_key_size);
        w.field<uint64_t>(8, s->num_merges);
        w.field<uint64_t>(6, s->num_deletes);
        w.field<uint64_t>(4, s->num_puts);
        if (nb) w.field_offset(14, vec);
        w.finish(w.end(t), &st_p, &st_n);
        st_crc = crc(st_p, st_n);
    };
    uint32_t filter_crc = 0;
    if (in->stats && nb >= 2048) {
        std::thread th(build_stats);
        build_index();
        if (in->has_filter) filter_crc = ~crc.update(crc.update(0xFFFFFFFFu, fh.data(), fh.size()), in->bloom, in->bloom_len);
        th.join();
    } else {
        build_index();
        if (in->stats) build_stats();
    }
    if (in->has_filter && !(in->stats && nb >= 2048))
        filter_crc = ~crc.update(crc.update(0xFFFFFFFFu, fh.data(), fh.size()), in->bloom, in->bloom_len);
    // a compression codec (format/sst.rs:557-594): the three blocks become the codec's streams, checksummed
    // after compression
    const uint32_t codec = in->compression;
    std::vector<uint8_t> zf, zi, zs;
    if (codec) {
        if (in->has_filter) {
            std::vector<uint8_t> composite(fh);
            composite.insert(composite.end(), in->bloom, in->bloom + in->bloom_len);
            literal_stream(codec, composite.data(), composite.size(), zf);
            sdb::host_compress(codec, composite.data(), composite.size(), zf);
            filter_crc = crc(zf.data(), zf.size());
            filter_len = zf.size() + 4;
        }
        literal_stream(codec, idx_p, idx_n, zi);
        sdb::host_compress(codec, idx_p, idx_n, zi);
        idx_p = zi.data();
        idx_n = zi.size();
        idx_crc = crc(idx_p, idx_n);
        if (in->stats) {
            literal_stream(codec, st_p, st_n, zs);
            sdb::host_compress(codec, st_p, st_n, zs);
            st_p = zs.data();
            st_n = zs.size();
            st_crc = crc(st_p, st_n);
        }
    }
    const uint64_t index_offset = base + filter_len, index_len = idx_n + 4;
    uint64_t stats_offset = 0, stats_len = 0;
    if (in->stats) {
        stats_offset = index_offset + index_len;
        stats_len = st_n + 4;
    }

    // 4. SsTableInfo (DbFlatBufferBuilder::add_sst_info), its CRC, meta offset and version
    const uint64_t meta_offset = index_offset + index_len + stats_len;
    const uint8_t *info_p = nullptr;
    uint64_t info_n = 0;
    {
        BackWriter w(sc.info, 256);
        uint32_t fe = 0, le = 0;
        if (in->first_entry) fe = w.bytes_vector(in->first_entry, (size_t)in->first_entry_len);
        if (in->last_entry) le = w.bytes_vector(in->last_entry, (size_t)in->last_entry_len);
        const uint32_t t = w.begin();
        w.field<uint64_t>(22, stats_len);
        w.field<uint64_t>(20, stats_offset);
        w.field<uint64_t>(12, filter_len);
        w.field<uint64_t>(10, filter_offset);
        w.field<uint64_t>(8, index_len);
        w.field<uint64_t>(6, index_offset);
        if (in->last_entry) w.field_offset(18, le);
        if (in->first_entry) w.field_offset(4, fe);
        w.field<uint8_t>(24, 1);  // FilterFormat::Composite
        w.field<uint8_t>(16, in->sst_type);
        w.field<uint8_t>(14, (uint8_t)codec);  // CompressionFormat (None is the default: omitted)
        w.finish(w.end(t), &info_p, &info_n);
    }
    const uint64_t total = meta_offset - base + info_n + 4 + 10;
    *len = total;
    if (!out) return SDB_OK;  // size query
    if (cap < total) return SDB_LIMIT_EXCEEDED;
    // compress_and_transform with no codec / transformer: bytes ++ crc32 BE (format/sst.rs:525-554)
    uint8_t *o = out;
    if (in->has_filter && codec) {
        memcpy(o, zf.data(), zf.size());
        o = put_be(o + zf.size(), filter_crc, 4);
    } else if (in->has_filter) {
        memcpy(o, fh.data(), fh.size());
        o += fh.size();
        if (in->bloom_len) memcpy(o, in->bloom, in->bloom_len);
        o = put_be(o + in->bloom_len, filter_crc, 4);
    }
    memcpy(o, idx_p, idx_n);
    o = put_be(o + idx_n, idx_crc, 4);
    if (in->stats) {
        memcpy(o, st_p, st_n);
        o = put_be(o + st_n, st_crc, 4);
    }
    memcpy(o, info_p, info_n);
    o = put_be(o + info_n, crc(info_p, info_n), 4);
    o = put_be(o, meta_offset, 8);
    put_be(o, in->sst_version, 2);
    return SDB_OK;
}
