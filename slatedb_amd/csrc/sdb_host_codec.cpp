// sdb_host_codec.cpp — host compressors for the footer's blocks.
//
// The filter, index and stats blocks are built on the host (sdb_footer.cpp) and go through the SST's codec
// before their checksums exactly like the data blocks (compress_and_transform, format/sst.rs:394-452 ->
// SsTableFormat::compress, format/sst.rs:557-594).  They are small (a D1 SST's footer is 1.5 MB, most of it
// the filter's random bits), so they are compressed here rather than on the device:
//   Zlib    the image's zlib at level 6 (flate2's default level; zlib.h / libz, present on every box);
//   Lz4     a hash-chain greedy parse into LZ4 block sequences (lz4_flex::compress_prepend_size framing);
//   Snappy  the same parse into Snappy literal / copy elements;
//   Zstd    one frame (Frame_Content_Size), 128 KiB blocks: raw literals and sequences coded with the
//           predefined FSE distributions (RFC 8878 3.1.1.3.2.2), repeat offsets, or a raw block when that is
//           shorter.
// Every stream is checked against the literal-only stream's size and replaced by it when not shorter.
// The bytes are valid for the formats (decoded by the reference's crates; the tests decode them with
// pyarrow / Python zlib) but are not the crates' bytes: byte parity is unpinned, as for the data blocks.
#include <stdint.h>
#include <string.h>
#include <zlib.h>

#include <vector>

#include "../../include/slatedb_amd.h"

namespace sdb {

namespace {

struct HSeq {
    uint32_t lit, len, off;  // literal run before the match, match length, offset
};

// Greedy parse with a depth-limited hash chain over in[0, n): sequences + the tail literals.
// lz4: matches start 12+ bytes before the end and end 5+ before it.
uint64_t parse(const uint8_t *in, uint64_t n, uint32_t max_off, int depth, bool lz4, std::vector<HSeq> &seqs) {
    constexpr int kBits = 16;
    std::vector<int64_t> head(1u << kBits, -1), prev(n ? n : 1, -1);
    auto hash = [&](uint64_t p) {
        uint32_t v;
        memcpy(&v, in + p, 4);
        return (v * 2654435761u) >> (32 - kBits);
    };
    auto insert = [&](uint64_t p) {
        const uint32_t h = hash(p);
        prev[p] = head[h];
        head[h] = (int64_t)p;
    };
    seqs.clear();
    uint64_t p = 0, ls = 0;
    while (p + 4 <= n) {
        if (lz4 && p + 12 > n) break;
        uint64_t lim = n - p;
        if (lz4) lim = n - 5 - p;
        if (lim > 65535) lim = 65535;
        uint32_t blen = 0, boff = 0;
        int64_t c = head[hash(p)];
        for (int d = 0; d < depth && c >= 0 && p - (uint64_t)c <= max_off; d++, c = prev[c]) {
            if (memcmp(in + c, in + p, 4)) continue;
            uint64_t len = 4;
            while (len < lim && in[c + len] == in[p + len]) len++;
            if (len > blen) {
                blen = (uint32_t)len;
                boff = (uint32_t)(p - (uint64_t)c);
                if (len >= 258) break;
            }
        }
        insert(p);
        if (blen >= 4) {
            seqs.push_back({(uint32_t)(p - ls), blen, boff});
            for (uint64_t q = p + 1; q < p + blen && q + 4 <= n; q++) insert(q);
            p += blen;
            ls = p;
        } else {
            p++;
        }
    }
    return n - ls;
}

void le(std::vector<uint8_t> &o, uint64_t v, int nb) {
    for (int i = 0; i < nb; i++) o.push_back((uint8_t)(v >> (8 * i)));
}

void lz4_block(const uint8_t *in, uint64_t n, std::vector<uint8_t> &o) {
    std::vector<HSeq> seqs;
    const uint64_t tail = parse(in, n, 65535, 4, true, seqs);
    le(o, n, 4);
    auto lenx = [&](uint64_t x) {  // the length bytes past a token's 15
        for (; x >= 255; x -= 255) o.push_back(255);
        o.push_back((uint8_t)x);
    };
    uint64_t pos = 0;
    for (const HSeq &s : seqs) {
        const uint32_t ml = s.len - 4;
        o.push_back((uint8_t)(((s.lit >= 15 ? 15 : s.lit) << 4) | (ml >= 15 ? 15 : ml)));
        if (s.lit >= 15) lenx(s.lit - 15);
        o.insert(o.end(), in + pos, in + pos + s.lit);
        le(o, s.off, 2);
        if (ml >= 15) lenx(ml - 15);
        pos += s.lit + s.len;
    }
    o.push_back((uint8_t)((tail >= 15 ? 15 : tail) << 4));
    if (tail >= 15) lenx(tail - 15);
    o.insert(o.end(), in + pos, in + n);
}

void snappy_block(const uint8_t *in, uint64_t n, std::vector<uint8_t> &o) {
    std::vector<HSeq> seqs;
    const uint64_t tail = parse(in, n, 65535, 4, false, seqs);
    for (uint64_t x = n;; x >>= 7) {
        o.push_back((uint8_t)(x >= 0x80 ? (x & 0x7F) | 0x80 : x));
        if (x < 0x80) break;
    }
    auto literal = [&](const uint8_t *p, uint64_t len) {
        if (!len) return;
        const uint64_t v = len - 1;
        const int nb = v < 60 ? 0 : v < 256 ? 1 : v < 65536 ? 2 : v < (1u << 24) ? 3 : 4;
        o.push_back((uint8_t)((nb ? 59 + nb : v) << 2));
        le(o, v, nb);
        o.insert(o.end(), p, p + len);
    };
    auto copy2 = [&](uint32_t len, uint32_t off) {
        o.push_back((uint8_t)(2 | ((len - 1) << 2)));
        le(o, off, 2);
    };
    uint64_t pos = 0;
    for (const HSeq &s : seqs) {
        literal(in + pos, s.lit);
        uint32_t r = s.len;
        while (r >= 68) {
            copy2(64, s.off);
            r -= 64;
        }
        if (r > 64) {
            copy2(60, s.off);
            r -= 60;
        }
        if (r < 12 && s.off < 2048) {
            o.push_back((uint8_t)(1 | ((r - 4) << 2) | ((s.off >> 8) << 5)));
            o.push_back((uint8_t)s.off);
        } else {
            copy2(r, s.off);
        }
        pos += s.lit + s.len;
    }
    literal(in + pos, tail);
}

// --- zstd: predefined FSE distributions (RFC 8878 3.1.1.3.2.2), tables in lane order LL, ML, OF -----------
const int16_t kDef[3][53] = {
    {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2, 2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1},
    {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
     1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1},
    {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1}};
const uint32_t kDefN[3] = {36, 53, 29}, kDefAl[3] = {6, 6, 5};
const uint32_t kLLBase[36] = {0,  1,  2,  3,  4,  5,  6,  7,  8,   9,   10,  11,   12,   13,   14,   15,    16,    18,
                              20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096, 8192, 16384, 32768, 65536};
const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
const uint32_t kMLBase[53] = {3,  4,  5,  6,  7,  8,  9,  10, 11, 12,  13,  14,  15,   16,   17,   18,   19,    20,
                              21, 22, 23, 24, 25, 26, 27, 28, 29, 30,  31,  32,  33,   34,   35,   37,   39,    41,
                              43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051, 4099, 8195, 16387, 32771, 65539};
const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                             0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};

struct FseCT {  // FSE_buildCTable for one predefined distribution
    uint32_t al = 0;
    std::vector<uint16_t> stab;
    std::vector<int32_t> dnb, dfs;
    void build(const int16_t *norm, uint32_t ns, uint32_t a) {
        al = a;
        const uint32_t size = 1u << al, mask = size - 1, step = (size >> 1) + (size >> 3) + 3;
        std::vector<uint32_t> cumul(ns + 1);
        std::vector<uint8_t> spread(size);
        uint32_t high = size - 1;
        for (uint32_t u = 1; u <= ns; u++) {
            if (norm[u - 1] == -1) {
                cumul[u] = cumul[u - 1] + 1;
                spread[high--] = (uint8_t)(u - 1);
            } else {
                cumul[u] = cumul[u - 1] + (uint32_t)norm[u - 1];
            }
        }
        uint32_t pos = 0;
        for (uint32_t s = 0; s < ns; s++)
            for (int i = 0; i < norm[s]; i++) {
                spread[pos] = (uint8_t)s;
                pos = (pos + step) & mask;
                while (pos > high) pos = (pos + step) & mask;
            }
        stab.assign(size, 0);
        for (uint32_t u = 0; u < size; u++) stab[cumul[spread[u]]++] = (uint16_t)(size + u);
        dnb.assign(ns, 0);
        dfs.assign(ns, 0);
        int total = 0;
        for (uint32_t s = 0; s < ns; s++) {
            const int nc = norm[s];
            if (nc == -1 || nc == 1) {
                dnb[s] = (int32_t)((al << 16) - size);
                dfs[s] = total - 1;
                total++;
            } else if (nc > 1) {
                const uint32_t mbo = al - (31u - (uint32_t)__builtin_clz((uint32_t)nc - 1)), msp = (uint32_t)nc << mbo;
                dnb[s] = (int32_t)((mbo << 16) - msp);
                dfs[s] = total - nc;
                total += nc;
            } else {
                dnb[s] = (int32_t)(((al + 1) << 16) - size);
            }
        }
    }
    uint32_t init(uint32_t sym) const {
        const uint32_t nbo = (uint32_t)((dnb[sym] + (1 << 15)) >> 16);
        const uint32_t v = (nbo << 16) - (uint32_t)dnb[sym];
        return stab[(int)(v >> nbo) + dfs[sym]];
    }
};

struct BitW {  // BIT_CStream: forward, read backwards by the decoder
    std::vector<uint8_t> &o;
    uint64_t acc = 0;
    uint32_t bc = 0;
    void add(uint64_t v, uint32_t nb) {
        if (!nb) return;
        if (nb < 64) v &= (1ull << nb) - 1;
        while (nb) {
            const uint32_t take = nb < 32 ? nb : 32;
            acc |= (v & ((1ull << take) - 1)) << bc;
            bc += take;
            v >>= take;
            nb -= take;
            while (bc >= 8) {
                o.push_back((uint8_t)acc);
                acc >>= 8;
                bc -= 8;
            }
        }
    }
    void close() {
        add(1, 1);
        if (bc) o.push_back((uint8_t)acc);
        acc = 0;
        bc = 0;
    }
};

uint32_t ll_code(uint32_t v) {
    if (v < 16) return v;
    uint32_t c = 16;
    while (c < 35 && kLLBase[c + 1] <= v) c++;
    return c;
}
uint32_t ml_code(uint32_t len) {
    if (len < 35) return len - 3;
    uint32_t c = 32;
    while (c < 52 && kMLBase[c + 1] <= len) c++;
    return c;
}

// one compressed block's content for in[0, n), or false when it is not shorter than n
bool zstd_block(const uint8_t *in, uint64_t n, uint32_t (&rep)[3], const FseCT (&ct)[3], std::vector<uint8_t> &o) {
    std::vector<HSeq> seqs;
    const uint64_t tail = parse(in, n, (uint32_t)n, 8, false, seqs);
    std::vector<uint8_t> lit;
    uint64_t pos = 0;
    for (const HSeq &s : seqs) {
        lit.insert(lit.end(), in + pos, in + pos + s.lit);
        pos += s.lit + s.len;
    }
    lit.insert(lit.end(), in + pos, in + n);
    (void)tail;
    const size_t o0 = o.size();
    const uint64_t nl = lit.size();
    if (nl < 32) o.push_back((uint8_t)(nl << 3));
    else if (nl < 4096) le(o, (1u << 2) | (nl << 4), 2);
    else le(o, (3u << 2) | (nl << 4), 3);
    o.insert(o.end(), lit.begin(), lit.end());
    const uint64_t ns = seqs.size();
    if (ns < 128) o.push_back((uint8_t)ns);
    else if (ns < 0x7F00) {
        o.push_back((uint8_t)((ns >> 8) + 128));
        o.push_back((uint8_t)ns);
    } else {
        o.push_back(255);
        le(o, ns - 0x7F00, 2);
    }
    uint32_t r0 = rep[0], r1 = rep[1], r2 = rep[2];
    if (ns) {
        o.push_back(0);  // LL, OF, ML: predefined
        std::vector<uint32_t> ob(ns), lc(ns), mc(ns), oc(ns);
        for (uint64_t i = 0; i < ns; i++) {  // repeat offsets (RFC 8878 3.1.2.5)
            const uint32_t L = seqs[i].lit, off = seqs[i].off;
            uint32_t b;
            if (L) b = off == r0 ? 1 : off == r1 ? 2 : off == r2 ? 3 : off + 3;
            else b = off == r1 ? 1 : off == r2 ? 2 : off == r0 - 1 ? 3 : off + 3;
            const uint32_t idx = b > 3 ? 4 : (L ? b - 1 : b);
            if (idx == 1) {
                r1 = r0;
                r0 = off;
            } else if (idx >= 2) {
                r2 = r1;
                r1 = r0;
                r0 = off;
            }
            ob[i] = b;
            lc[i] = ll_code(L);
            mc[i] = ml_code(seqs[i].len);
            oc[i] = 31u - (uint32_t)__builtin_clz(b);
        }
        BitW bw{o};
        uint32_t sll = ct[0].init(lc[ns - 1]), sml = ct[1].init(mc[ns - 1]), sof = ct[2].init(oc[ns - 1]);
        auto extras = [&](uint64_t i) {
            bw.add(seqs[i].lit - kLLBase[lc[i]], kLLBits[lc[i]]);
            bw.add(seqs[i].len - kMLBase[mc[i]], kMLBits[mc[i]]);
            bw.add(ob[i] - (1u << oc[i]), oc[i]);
        };
        auto enc = [&](const FseCT &t, uint32_t &st, uint32_t sym) {
            const uint32_t nb = (uint32_t)((int)st + t.dnb[sym]) >> 16;
            bw.add(st, nb);
            st = t.stab[(int)(st >> nb) + t.dfs[sym]];
        };
        extras(ns - 1);
        for (int64_t i = (int64_t)ns - 2; i >= 0; i--) {
            enc(ct[2], sof, oc[i]);
            enc(ct[1], sml, mc[i]);
            enc(ct[0], sll, lc[i]);
            extras((uint64_t)i);
        }
        bw.add(sml - (1u << ct[1].al), ct[1].al);
        bw.add(sof - (1u << ct[2].al), ct[2].al);
        bw.add(sll - (1u << ct[0].al), ct[0].al);
        bw.close();
    }
    if (o.size() - o0 >= n) {
        o.resize(o0);
        return false;
    }
    rep[0] = r0;
    rep[1] = r1;
    rep[2] = r2;
    return true;
}

struct PredefTables {
    FseCT t[3];
    PredefTables() {
        for (int i = 0; i < 3; i++) t[i].build(kDef[i], kDefN[i], kDefAl[i]);
    }
};

void zstd_frame(const uint8_t *in, uint64_t n, std::vector<uint8_t> &o) {
    static const PredefTables tabs;
    const FseCT(&ct)[3] = tabs.t;
    le(o, 0xFD2FB528u, 4);
    if (n < 256) {
        o.push_back(0x20);
        le(o, n, 1);
    } else if (n < 65536 + 256) {
        o.push_back(0x60);
        le(o, n - 256, 2);
    } else {
        o.push_back(0xA0);
        le(o, n, 4);
    }
    uint32_t rep[3] = {1, 4, 8};
    uint64_t done = 0;
    do {
        const uint64_t c = n - done < (128u << 10) ? n - done : (128u << 10);
        const bool last = done + c == n;
        const size_t h = o.size();
        le(o, 0, 3);
        uint32_t type = 0, size = (uint32_t)c;
        if (c >= 16 && zstd_block(in + done, c, rep, ct, o)) {
            type = 2;
            size = (uint32_t)(o.size() - h - 3);
        } else {
            o.insert(o.end(), in + done, in + done + c);
        }
        const uint32_t bh = (last ? 1u : 0u) | (type << 1) | (size << 3);
        o[h] = (uint8_t)bh;
        o[h + 1] = (uint8_t)(bh >> 8);
        o[h + 2] = (uint8_t)(bh >> 16);
        done += c;
    } while (done < n);
}

}  // namespace

// The codec's stream of in[0, n) (the footer blocks): `o` holds the literal-only stream on entry and is
// replaced by the compressed one when that is shorter.
void host_compress(uint32_t codec, const uint8_t *in, uint64_t n, std::vector<uint8_t> &o) {
    std::vector<uint8_t> c;
    if (codec == SDB_CODEC_ZLIB) {
        uLongf cap = compressBound((uLong)n);
        c.resize(cap);
        if (compress2(c.data(), &cap, in, (uLong)n, 6) == Z_OK) c.resize(cap);
        else c.clear();
    } else if (codec == SDB_CODEC_LZ4) {
        lz4_block(in, n, c);
    } else if (codec == SDB_CODEC_SNAPPY) {
        snappy_block(in, n, c);
    } else if (codec == SDB_CODEC_ZSTD) {
        zstd_frame(in, n, c);
    }
    if (!c.empty() && c.size() < o.size()) o.swap(c);
}

}  // namespace sdb
