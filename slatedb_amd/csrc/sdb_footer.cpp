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
#include <vector>

#include "../../include/slatedb_amd.h"

namespace {

// crc32fast::hash (IEEE, reflected, init/xorout 0xFFFFFFFF), slicing-by-8 on the host.
struct HostCrc {
    uint32_t t[8][256];
    HostCrc() {
        for (uint32_t i = 0; i < 256; i++) {
            uint32_t c = i;
            for (int k = 0; k < 8; k++) c = (c >> 1) ^ (0xEDB88320u & (0u - (c & 1u)));
            t[0][i] = c;
        }
        for (uint32_t i = 0; i < 256; i++)
            for (int s = 1; s < 8; s++) t[s][i] = (t[s - 1][i] >> 8) ^ t[0][t[s - 1][i] & 0xFF];
    }
    uint32_t operator()(const uint8_t *p, size_t n) const {
        uint32_t c = 0xFFFFFFFFu;
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
        return ~c;
    }
};
const HostCrc &host_crc() {
    static const HostCrc c;
    return c;
}

// Back-to-front flatbuffer writer.  Positions are "reverse offsets": bytes from the end of the
// finished buffer, which do not move when the buffer grows.
class BackWriter {
  public:
    explicit BackWriter(size_t cap = 1024) : buf_(cap), head_(cap) {}
    uint32_t rev() const { return (uint32_t)(buf_.size() - head_); }

    void pad_for(size_t len, size_t align) {  // room for `len` bytes that must end `align`-aligned
        if (align > max_align_) max_align_ = align;
        reserve(((size_t)0 - (rev() + len)) & (align - 1));
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
        fields_.clear();
        return rev();
    }
    template <class T>
    void field(uint16_t slot, T v) {  // omitted when equal to the default (0 for every field here)
        if (v != 0) fields_.push_back({slot, scalar<T>(v)});
    }
    void field_offset(uint16_t slot, uint32_t target) { fields_.push_back({slot, uoffset(target)}); }
    uint32_t end(uint32_t tail) {
        const uint32_t obj = scalar<uint32_t>(0);  // soffset to the vtable, patched below
        uint16_t vlen = 4;
        for (const auto &f : fields_) vlen = f.slot + 2 > vlen ? (uint16_t)(f.slot + 2) : vlen;
        VTable vt{};
        vt.len = vlen;
        const uint16_t hdr[2] = {vlen, (uint16_t)(obj - tail)};
        memcpy(vt.b, hdr, 4);
        for (const auto &f : fields_) {
            const uint16_t d = (uint16_t)(obj - f.rev);
            memcpy(vt.b + f.slot, &d, 2);
        }
        // a footer has a handful of distinct vtables (one per padding pattern): linear search,
        // most recent first
        uint32_t vt_rev = 0;
        bool found = false;
        for (size_t i = vtables_.size(); i-- > 0;)
            if (vtables_[i].len == vlen && !memcmp(vtables_[i].b, vt.b, vlen)) {
                vt_rev = vtables_[i].rev;
                found = true;
                if (i + 1 != vtables_.size()) std::swap(vtables_[i], vtables_.back());
                break;
            }
        if (!found) {
            reserve(vlen);
            memcpy(&buf_[head_], vt.b, vlen);
            vt_rev = vt.rev = rev();
            vtables_.push_back(vt);
        }
        const int32_t so = (int32_t)vt_rev - (int32_t)obj;
        memcpy(&buf_[buf_.size() - obj], &so, 4);
        fields_.clear();
        return obj;
    }
    // finish(root, None): pad so the root uoffset ends aligned to the largest alignment seen
    void finish(uint32_t root, std::vector<uint8_t> &out) {
        vtables_.clear();
        pad_for(4, max_align_);
        uoffset(root);
        out.insert(out.end(), buf_.begin() + (ptrdiff_t)head_, buf_.end());
    }

  private:
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
        if (head_ < n) {
            size_t cap = buf_.size();
            const size_t used = cap - head_;
            while (cap - used < n) cap = cap ? 2 * cap : 1024;
            std::vector<uint8_t> nb(cap);
            memcpy(&nb[cap - used], &buf_[head_], used);
            buf_.swap(nb);
            head_ = cap - used;
        }
        head_ -= n;  // fresh bytes are zero (padding stays zero)
    }
    std::vector<uint8_t> buf_;
    size_t head_;
    size_t max_align_ = 1;
    std::vector<Field> fields_;
    std::vector<VTable> vtables_;
};

void put_be(std::vector<uint8_t> &o, uint64_t v, int nbytes) {
    for (int i = nbytes - 1; i >= 0; i--) o.push_back((uint8_t)(v >> (8 * i)));
}
// compress_and_transform with no codec / transformer: bytes ++ crc32 BE (format/sst.rs:525-554)
uint64_t append_checked(std::vector<uint8_t> &o, const uint8_t *p, size_t n) {
    o.insert(o.end(), p, p + n);
    put_be(o, host_crc()(p, n), 4);
    return n + 4;
}

}  // namespace

extern "C" uint64_t sdb_sst_footer_bound(const sdb_footer_in *in) {
    if (!in) return 0;
    const uint64_t nb = in->num_blocks;
    const uint64_t keys = nb && in->first_key_off ? in->first_key_off[nb] - in->first_key_off[0] : 0;
    uint64_t b = 256 + in->first_entry_len + in->last_entry_len;  // SsTableInfo, crcs, trailer
    if (in->has_filter) b += 32 + in->bloom_len + (in->filter_name ? strlen(in->filter_name) : 3);  // composite filter block
    b += 64 + keys + 48 * nb;                                      // index: key, len, pads, BlockMeta, vtable, slot
    if (in->stats) b += 128 + 32 * nb;                             // stats: BlockStats tables + vector
    return b;
}

extern "C" sdb_status sdb_sst_footer(const sdb_footer_in *in, uint8_t *out, uint64_t cap,
                                     uint64_t *len) {
    if (!in || !len) return SDB_INVALID_ARGUMENT;
    const uint64_t nb = in->num_blocks;
    if (nb && (!in->block_off || !in->first_key_off || !in->first_key_bytes)) return SDB_INVALID_ARGUMENT;
    if (in->stats && nb && !in->block_stats) return SDB_INVALID_ARGUMENT;
    if (in->has_filter && in->bloom_len && !in->bloom) return SDB_INVALID_ARGUMENT;
    if (in->sst_type > 1) return SDB_INVALID_ARGUMENT;
    const uint64_t base = in->data_len;
    std::vector<uint8_t> o;
    o.reserve(sdb_sst_footer_bound(in));

    // 1. composite filter block [u16 count][u16 name_len]["_bf"][u64 len][Filter::encode]
    //    (format/sst.rs:394-421; Filter::encode = u16 BE num_probes ++ bitmap, filter.rs:177-180)
    const uint64_t filter_offset = base;
    uint64_t filter_len = 0;
    if (in->has_filter) {
        std::vector<uint8_t> c;
        const char *name = in->filter_name ? in->filter_name : "_bf";
        const size_t nl = strlen(name);
        if (nl > 0xFFFF) return SDB_INVALID_ARGUMENT;
        c.reserve(in->bloom_len + 14 + nl);
        put_be(c, 1, 2);
        put_be(c, nl, 2);
        c.insert(c.end(), (const uint8_t *)name, (const uint8_t *)name + nl);
        put_be(c, in->bloom_len + 2, 8);
        put_be(c, in->num_probes, 2);
        if (in->bloom_len) c.insert(c.end(), in->bloom, in->bloom + in->bloom_len);
        filter_len = append_checked(o, c.data(), c.size());
    }

    // 2. index: per block the first_key vector then its BlockMeta (creation order of the reference)
    std::vector<uint8_t> fb;
    {
        BackWriter w(64 + nb * 48);
        std::vector<uint32_t> metas(nb);
        for (uint64_t k = 0; k < nb; k++) {
            const uint64_t a = in->first_key_off[k], b = in->first_key_off[k + 1];
            if (b < a) return SDB_INVALID_ARGUMENT;
            const uint32_t key = w.bytes_vector(in->first_key_bytes + a, (size_t)(b - a));
            const uint32_t t = w.begin();
            w.field<uint64_t>(4, in->block_off[k]);  // BlockMeta.offset
            w.field_offset(6, key);                  // BlockMeta.first_key
            metas[k] = w.end(t);
        }
        const uint32_t vec = w.offsets_vector(metas);
        const uint32_t t = w.begin();
        w.field_offset(4, vec);  // SsTableIndex.block_meta
        w.finish(w.end(t), fb);
    }
    const uint64_t index_offset = base + o.size();
    const uint64_t index_len = append_checked(o, fb.data(), fb.size());

    // 3. stats (SstStats::encode): BlockStats tables, their vector, then SstStats
    uint64_t stats_offset = 0, stats_len = 0;
    if (in->stats) {
        fb.clear();
        BackWriter w(64 + nb * 20);
        std::vector<uint32_t> tabs(nb);
        for (uint64_t k = 0; k < nb; k++) {
            const uint16_t *s = in->block_stats + 3 * k;
            const uint32_t t = w.begin();
            w.field<uint16_t>(8, s[2]);  // num_merges
            w.field<uint16_t>(6, s[1]);  // num_deletes
            w.field<uint16_t>(4, s[0]);  // num_puts
            tabs[k] = w.end(t);
        }
        uint32_t vec = 0;
        if (nb) vec = w.offsets_vector(tabs);
        const sdb_sst_summary *s = in->stats;
        const uint32_t t = w.begin();
        w.field<uint64_t>(12, s->raw_val_size);
        w.field<uint64_t>(10, s->raw_key_size);
        w.field<uint64_t>(8, s->num_merges);
        w.field<uint64_t>(6, s->num_deletes);
        w.field<uint64_t>(4, s->num_puts);
        if (nb) w.field_offset(14, vec);
        w.finish(w.end(t), fb);
        stats_offset = base + o.size();
        stats_len = append_checked(o, fb.data(), fb.size());
    }

    // 4. SsTableInfo (DbFlatBufferBuilder::add_sst_info), its CRC, meta offset and version
    const uint64_t meta_offset = base + o.size();
    fb.clear();
    {
        BackWriter w(256);
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
        w.field<uint8_t>(14, 0);  // CompressionFormat::None
        w.finish(w.end(t), fb);
    }
    append_checked(o, fb.data(), fb.size());
    put_be(o, meta_offset, 8);
    put_be(o, in->sst_version, 2);

    *len = o.size();
    if (!out) return SDB_OK;  // size query
    if (cap < o.size()) return SDB_LIMIT_EXCEEDED;
    memcpy(out, o.data(), o.size());
    return SDB_OK;
}
