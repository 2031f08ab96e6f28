/*
 * sdb_oracle_entropy.c — CPU restatement of the entropy-coded block codecs of
 * SsTableFormat::decompress (slatedb/src/format/sst.rs:884-917).  TEST INFRASTRUCTURE ONLY: loaded by
 * tests/, smoke() and bench.py's cpu_baseline leg as the checker, never by the product.
 *
 * The reference delegates both codecs to third-party crates that are absent from /root/reference:
 *   CompressionCodec::Zlib = flate2 1.1.9 read::ZlibDecoder (miniz_oxide 0.8.9 backend, Cargo.lock:1017,
 *                            2012), read_to_end: a zlib stream (RFC 1950: CMF/FLG header, deflate data
 *                            RFC 1951, Adler-32 trailer);
 *   CompressionCodec::Zstd = zstd 0.13.3 stream::decode_all (libzstd 1.5.7, Cargo.lock:4847-4866):
 *                            a sequence of zstd frames (RFC 8878) and skippable frames.
 * Both are restated here from the published formats.  Parity is pinned by round trips through the
 * canonical C implementations available in this image (Python zlib; pyarrow's zstd codec) plus hand-built
 * frames for the elements those encoders do not emit (tests/test_codec_entropy.py).
 *
 * Semantics of the corners (documented, parity of the corners unpinned where marked):
 *   zlib  header: CM 8, CINFO <= 7, FCHECK, no preset dictionary; otherwise an error.  Input that ends
 *         before the stream does is NOT an error: flate2's read() maps miniz_oxide's BufError at EOF to
 *         Ok(0), so read_to_end returns the bytes decoded so far (unpinned: no flate2 here).  Bytes after
 *         the Adler-32 trailer are ignored.  Adler-32 mismatch: error.  Incomplete or oversubscribed
 *         Huffman codes with more than one used symbol: error (miniz_oxide's table check).
 *   zstd  every frame of the input in order; skippable frames skipped; a frame with a dictionary ID, a
 *         reserved bit set, a window over 2^27 (ZSTD_WINDOWLOG_LIMIT_DEFAULT), a content-size mismatch,
 *         a checksum mismatch or trailing bytes that do not form a frame: error; input that ends inside
 *         a frame: error (zstd-rs "incomplete frame").  Legacy (pre-v0.8) frames: error (unpinned).
 */
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#include "sdb_oracle.h"

/* ------------------------------------------------------------------------------------------- */
/* Output sink: out == NULL counts only (the plan's decompressed length).                       */
/* ------------------------------------------------------------------------------------------- */
typedef struct {
    uint8_t *p;
    size_t cap, len;
    int overflow;
} sink;

static int put_byte(sink *o, uint8_t b) {
    if (o->len >= o->cap) { o->overflow = 1; return -1; }
    if (o->p) o->p[o->len] = b;
    o->len++;
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* zlib / deflate (RFC 1950, RFC 1951)                                                          */
/* ------------------------------------------------------------------------------------------- */
typedef struct {
    const uint8_t *in;
    size_t n, pos;
    uint64_t buf;
    int cnt;
} lsb_bits;

/* k (<= 16) bits LSB-first; -1 when the input ends first (truncation). */
static int lsb_get(lsb_bits *s, int k, uint32_t *v) {
    while (s->cnt < k) {
        if (s->pos >= s->n) return -1;
        s->buf |= (uint64_t)s->in[s->pos++] << s->cnt;
        s->cnt += 8;
    }
    *v = (uint32_t)(s->buf & ((1ull << k) - 1));
    s->buf >>= k;
    s->cnt -= k;
    return 0;
}

/* canonical Huffman code by lengths: count[len] and the symbols in code order */
typedef struct {
    uint16_t count[16];
    uint16_t sym[320];
} canon;

/* 0: usable; -1: incomplete / oversubscribed with more than one used symbol */
static int canon_build(canon *h, const uint8_t *len, int n) {
    uint16_t offs[16];
    memset(h->count, 0, sizeof(h->count));
    for (int s = 0; s < n; s++) h->count[len[s]]++;
    int used = n - h->count[0];
    int left = 1;
    for (int l = 1; l < 16; l++) {
        left <<= 1;
        left -= h->count[l];
        if (left < 0) return used > 1 ? -1 : 0;
    }
    if (left > 0 && used > 1) return -1;
    offs[1] = 0;
    for (int l = 1; l < 15; l++) offs[l + 1] = offs[l] + h->count[l];
    for (int s = 0; s < n; s++)
        if (len[s]) h->sym[offs[len[s]]++] = (uint16_t)s;
    return 0;
}

/* one symbol, code bits MSB-first of the code read one at a time; -1 truncated, -2 invalid code */
static int canon_decode(lsb_bits *s, const canon *h) {
    int code = 0, first = 0, index = 0;
    for (int l = 1; l < 16; l++) {
        uint32_t b;
        if (lsb_get(s, 1, &b)) return -1;
        code |= (int)b;
        const int c = h->count[l];
        if (code - first < c) return h->sym[index + code - first];
        index += c;
        first += c;
        first <<= 1;
        code <<= 1;
    }
    return -2;
}

static const uint16_t kLenBase[29] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 13, 15, 17, 19, 23, 27, 31,
                                      35, 43, 51, 59, 67, 83, 99, 115, 131, 163, 195, 227, 258};
static const uint8_t kLenExtra[29] = {0, 0, 0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 2, 2, 3, 3, 3, 3, 4, 4, 4, 4, 5, 5, 5, 5, 0};
static const uint16_t kDistBase[30] = {1, 2, 3, 4, 5, 7, 9, 13, 17, 25, 33, 49, 65, 97, 129, 193, 257, 385, 513, 769,
                                       1025, 1537, 2049, 3073, 4097, 6145, 8193, 12289, 16385, 24577};
static const uint8_t kDistExtra[30] = {0, 0, 0, 0, 1, 1, 2, 2, 3, 3, 4, 4, 5, 5, 6, 6, 7, 7, 8, 8, 9, 9, 10, 10, 11, 11, 12, 12, 13, 13};

enum { Z_OK = 0, Z_TRUNC = 1, Z_ERR = -1 };

/* inflate into o; the output so far is o->p[0, o->len) (count mode: history not kept, distances are
 * still checked against the bytes produced).  Z_TRUNC: the input ended before the final block did. */
static int inflate_raw(lsb_bits *s, sink *o) {
    static const uint8_t kOrder[19] = {16, 17, 18, 0, 8, 7, 9, 6, 10, 5, 11, 4, 12, 3, 13, 2, 14, 1, 15};
    canon lit, dist;
    uint32_t last = 0;
    do {
        uint32_t type;
        if (lsb_get(s, 1, &last) || lsb_get(s, 2, &type)) return Z_TRUNC;
        if (type == 0) {  /* stored: to the byte boundary, LEN, NLEN, bytes */
            s->buf >>= s->cnt & 7;
            s->cnt -= s->cnt & 7;
            uint32_t ln, nl;
            if (lsb_get(s, 16, &ln) || lsb_get(s, 16, &nl)) return Z_TRUNC;
            if ((ln ^ 0xFFFF) != nl) return Z_ERR;
            for (uint32_t i = 0; i < ln; i++) {  /* a truncated stored block yields what is there */
                uint32_t b;
                if (lsb_get(s, 8, &b)) return Z_TRUNC;
                if (put_byte(o, (uint8_t)b)) return Z_ERR;
            }
            continue;
        }
        if (type == 3) return Z_ERR;
        uint8_t lens[320];
        int nlen, ndist;
        if (type == 1) {  /* fixed codes */
            int i = 0;
            for (; i < 144; i++) lens[i] = 8;
            for (; i < 256; i++) lens[i] = 9;
            for (; i < 280; i++) lens[i] = 7;
            for (; i < 288; i++) lens[i] = 8;
            for (i = 0; i < 32; i++) lens[288 + i] = 5;  /* 32 five-bit codes; 30 and 31 never occur */
            nlen = 288;
            ndist = 32;
        } else {  /* dynamic: code length code, then the literal/length and distance lengths */
            uint32_t hlit, hdist, hclen;
            if (lsb_get(s, 5, &hlit) || lsb_get(s, 5, &hdist) || lsb_get(s, 4, &hclen)) return Z_TRUNC;
            nlen = (int)hlit + 257;
            ndist = (int)hdist + 1;
            if (nlen > 286 || ndist > 30) return Z_ERR;
            uint8_t cl[19];
            memset(cl, 0, sizeof(cl));
            for (uint32_t i = 0; i < hclen + 4; i++) {
                uint32_t v;
                if (lsb_get(s, 3, &v)) return Z_TRUNC;
                cl[kOrder[i]] = (uint8_t)v;
            }
            canon clc;
            if (canon_build(&clc, cl, 19)) return Z_ERR;
            int i = 0;
            while (i < nlen + ndist) {
                const int sym = canon_decode(s, &clc);
                if (sym == -1) return Z_TRUNC;
                if (sym < 0) return Z_ERR;
                if (sym < 16) { lens[i++] = (uint8_t)sym; continue; }
                uint32_t rep, v;
                uint8_t val = 0;
                if (sym == 16) {
                    if (i == 0) return Z_ERR;
                    val = lens[i - 1];
                    if (lsb_get(s, 2, &v)) return Z_TRUNC;
                    rep = 3 + v;
                } else if (sym == 17) {
                    if (lsb_get(s, 3, &v)) return Z_TRUNC;
                    rep = 3 + v;
                } else {
                    if (lsb_get(s, 7, &v)) return Z_TRUNC;
                    rep = 11 + v;
                }
                if (i + (int)rep > nlen + ndist) return Z_ERR;
                while (rep--) lens[i++] = val;
            }
            if (lens[256] == 0) return Z_ERR;  /* no end-of-block code */
            memmove(lens + 288, lens + nlen, (size_t)ndist);
        }
        if (canon_build(&lit, lens, nlen) || canon_build(&dist, lens + 288, ndist)) return Z_ERR;
        for (;;) {
            int sym = canon_decode(s, &lit);
            if (sym == -1) return Z_TRUNC;
            if (sym < 0) return Z_ERR;
            if (sym < 256) {
                if (put_byte(o, (uint8_t)sym)) return Z_ERR;
                continue;
            }
            if (sym == 256) break;
            sym -= 257;
            if (sym >= 29) return Z_ERR;
            uint32_t v;
            if (lsb_get(s, kLenExtra[sym], &v)) return Z_TRUNC;
            const uint32_t len = kLenBase[sym] + v;
            const int ds = canon_decode(s, &dist);
            if (ds == -1) return Z_TRUNC;
            if (ds < 0 || ds >= 30) return Z_ERR;
            if (lsb_get(s, kDistExtra[ds], &v)) return Z_TRUNC;
            const uint32_t d = kDistBase[ds] + v;
            if (d > o->len) return Z_ERR;
            for (uint32_t i = 0; i < len; i++) {
                const uint8_t b = o->p ? o->p[o->len - d] : 0;
                if (put_byte(o, b)) return Z_ERR;
            }
        }
    } while (!last);
    return Z_OK;
}

static uint32_t adler32(const uint8_t *p, size_t n) {
    uint32_t a = 1, b = 0;
    for (size_t i = 0; i < n; i++) {
        a = (a + p[i]) % 65521u;
        b = (b + a) % 65521u;
    }
    return b << 16 | a;
}

/* flate2 ZlibDecoder::read_to_end -> 0 or -1 (error); o holds the output.  Adler-32 is checked only
 * when the bytes are kept (o->p != NULL). */
static int zlib_decode(const uint8_t *in, size_t n, sink *o) {
    if (n < 2) return 0;  /* EOF before the header: no output, no error */
    const uint32_t cmf = in[0], flg = in[1];
    if ((cmf & 0x0F) != 8 || (cmf >> 4) > 7 || ((cmf << 8) | flg) % 31 != 0 || (flg & 0x20)) return -1;
    lsb_bits s = {in, n, 2, 0, 0};
    const int r = inflate_raw(&s, o);
    if (r == Z_ERR) return -1;
    if (r == Z_TRUNC) return 0;
    /* Adler-32, big-endian, at the next byte boundary */
    s.buf >>= s.cnt & 7;
    s.cnt -= s.cnt & 7;
    uint32_t a = 0;
    for (int i = 0; i < 4; i++) {
        uint32_t b;
        if (lsb_get(&s, 8, &b)) return 0;  /* truncated trailer: not checked */
        a = a << 8 | b;
    }
    if (o->p && adler32(o->p, o->len) != a) return -1;
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* zstd (RFC 8878)                                                                              */
/* ------------------------------------------------------------------------------------------- */
static uint64_t xxh_rotl(uint64_t x, int r) { return (x << r) | (x >> (64 - r)); }
static const uint64_t P1 = 11400714785074694791ull, P2 = 14029467366897019727ull, P3 = 1609587929392839161ull,
                      P4 = 9650029242287828579ull, P5 = 2870177450012600261ull;
static uint64_t rd64(const uint8_t *p) { uint64_t v; memcpy(&v, p, 8); return v; }
static uint32_t rd32(const uint8_t *p) { uint32_t v; memcpy(&v, p, 4); return v; }
static uint64_t xxh_round(uint64_t acc, uint64_t in) { acc += in * P2; acc = xxh_rotl(acc, 31); return acc * P1; }
static uint64_t xxh_merge(uint64_t acc, uint64_t v) { acc ^= xxh_round(0, v); return acc * P1 + P4; }

uint64_t orc_xxh64(const uint8_t *p, size_t n, uint64_t seed) {
    const uint8_t *e = p + n;
    uint64_t h;
    if (n >= 32) {
        uint64_t v1 = seed + P1 + P2, v2 = seed + P2, v3 = seed, v4 = seed - P1;
        while (p + 32 <= e) {
            v1 = xxh_round(v1, rd64(p));
            v2 = xxh_round(v2, rd64(p + 8));
            v3 = xxh_round(v3, rd64(p + 16));
            v4 = xxh_round(v4, rd64(p + 24));
            p += 32;
        }
        h = xxh_rotl(v1, 1) + xxh_rotl(v2, 7) + xxh_rotl(v3, 12) + xxh_rotl(v4, 18);
        h = xxh_merge(h, v1);
        h = xxh_merge(h, v2);
        h = xxh_merge(h, v3);
        h = xxh_merge(h, v4);
    } else {
        h = seed + P5;
    }
    h += (uint64_t)n;
    while (p + 8 <= e) {
        h ^= xxh_round(0, rd64(p));
        h = xxh_rotl(h, 27) * P1 + P4;
        p += 8;
    }
    if (p + 4 <= e) {
        h ^= (uint64_t)rd32(p) * P1;
        h = xxh_rotl(h, 23) * P2 + P3;
        p += 4;
    }
    while (p < e) {
        h ^= (*p++) * P5;
        h = xxh_rotl(h, 11) * P1;
    }
    h ^= h >> 33;
    h *= P2;
    h ^= h >> 29;
    h *= P3;
    h ^= h >> 32;
    return h;
}

static int highbit32(uint32_t v) { return 31 - __builtin_clz(v); }

/* backward bitstream (Huffman streams, FSE sequences): bits are read from the last byte toward the
 * first, most significant first; the last byte's highest set bit is the start marker. */
typedef struct {
    const uint8_t *p;
    int64_t pos;  /* bits not yet read: bit indices [0, pos) */
} rev_bits;

static int rev_init(rev_bits *b, const uint8_t *p, size_t n) {
    if (n == 0 || p[n - 1] == 0) return -1;
    b->p = p;
    b->pos = (int64_t)(n - 1) * 8 + highbit32(p[n - 1]);
    return 0;
}
/* k (<= 32) bits; bits past the start read as zero (pos goes negative: checked by the callers) */
static uint32_t rev_get(rev_bits *b, int k) {
    uint32_t v = 0;
    for (int i = 0; i < k; i++) {
        const int64_t q = b->pos - 1 - i;
        const uint32_t bit = q >= 0 ? (b->p[q >> 3] >> (q & 7)) & 1u : 0u;
        v = v << 1 | bit;
    }
    b->pos -= k;
    return v;
}
static uint32_t rev_peek(const rev_bits *b, int k) {
    rev_bits c = *b;
    return rev_get(&c, k);
}

/* FSE */
typedef struct {
    uint8_t sym, nb;
    uint16_t base;
} fse_cell;
typedef struct {
    int al;            /* accuracy log */
    fse_cell t[512];
} fse_table;

/* normalized counts -> decoding table (RFC 8878 4.1.1) */
static int fse_build(fse_table *ft, const int16_t *norm, int nsym, int al) {
    const int size = 1 << al;
    int high = size - 1;
    uint16_t next[256];
    ft->al = al;
    for (int s = 0; s < nsym; s++) {
        if (norm[s] == -1) {
            ft->t[high--].sym = (uint8_t)s;
            next[s] = 1;
        } else {
            next[s] = (uint16_t)norm[s];
        }
    }
    const int step = (size >> 1) + (size >> 3) + 3, mask = size - 1;
    int pos = 0;
    for (int s = 0; s < nsym; s++)
        for (int i = 0; i < norm[s]; i++) {
            ft->t[pos].sym = (uint8_t)s;
            do pos = (pos + step) & mask; while (pos > high);
        }
    if (pos != 0) return -1;
    for (int u = 0; u < size; u++) {
        const int s = ft->t[u].sym;
        const uint32_t x = next[s]++;
        const int nb = al - highbit32(x);
        ft->t[u].nb = (uint8_t)nb;
        ft->t[u].base = (uint16_t)((x << nb) - (uint32_t)size);
    }
    return 0;
}

/* FSE table description (forward bitstream) -> normalized counts; returns bytes used or -1 */
static int fse_read_ncount(const uint8_t *in, size_t n, int16_t *norm, int *nsym, int max_sym, int max_al, int *al_out) {
    if (n < 1) return -1;
    size_t bitpos = 0;
    #define FBITS(k) ({ uint32_t _v = 0; for (int _i = 0; _i < (k); _i++) { size_t _q = bitpos + _i; \
        if ((_q >> 3) < n) _v |= (uint32_t)((in[_q >> 3] >> (_q & 7)) & 1u) << _i; } _v; })
    const int al = (int)FBITS(4) + 5;
    bitpos += 4;
    if (al > max_al) return -1;
    int remaining = (1 << al) + 1, threshold = 1 << al, nbits = al + 1, s = 0;
    while (remaining > 1 && s <= max_sym) {
        const int mx = (2 * threshold - 1) - remaining;
        int v;
        const uint32_t low = FBITS(nbits - 1);
        if ((int)low < mx) {
            v = (int)low;
            bitpos += nbits - 1;
        } else {
            v = (int)FBITS(nbits);
            if (v >= threshold) v -= mx;
            bitpos += nbits;
        }
        const int proba = v - 1;
        remaining -= proba < 0 ? -proba : proba;
        norm[s++] = (int16_t)proba;
        if (proba == 0) {  /* repeat flags: 2 bits, 3 = another flag follows */
            for (;;) {
                const int r = (int)FBITS(2);
                bitpos += 2;
                for (int i = 0; i < r && s <= max_sym; i++) norm[s++] = 0;
                if (r != 3) break;
            }
        }
        while (remaining < threshold) {
            nbits--;
            threshold >>= 1;
        }
    }
    #undef FBITS
    if (remaining != 1 || s > max_sym + 1) return -1;
    if ((bitpos + 7) / 8 > n) return -1;
    *nsym = s;
    *al_out = al;
    return (int)((bitpos + 7) / 8);
}

/* Huffman literal table */
typedef struct {
    int maxbits;
    uint8_t sym[2048], nb[2048];
} huf_table;

static int huf_from_weights(huf_table *h, const uint8_t *w, int nw) {
    uint32_t total = 0;
    for (int i = 0; i < nw; i++) {
        if (w[i] > 11) return -1;
        if (w[i]) total += 1u << (w[i] - 1);
    }
    if (total == 0) return -1;
    const int maxbits = highbit32(total) + 1;
    if (maxbits > 11) return -1;
    const uint32_t rest = (1u << maxbits) - total;
    if (rest & (rest - 1)) return -1;  /* the implied last weight must complete the code */
    uint8_t wt[256];
    memcpy(wt, w, (size_t)nw);
    wt[nw] = (uint8_t)(highbit32(rest) + 1);
    const int ns = nw + 1;
    h->maxbits = maxbits;
    uint32_t start[13];
    uint32_t next = 0;
    for (int wv = 1; wv <= maxbits; wv++) {
        start[wv] = next;
        for (int s = 0; s < ns; s++)
            if (wt[s] == wv) next += 1u << (wv - 1);
    }
    for (int wv = 1; wv <= maxbits; wv++) {
        uint32_t p = start[wv];
        for (int s = 0; s < ns; s++) {
            if (wt[s] != wv) continue;
            for (uint32_t i = 0; i < (1u << (wv - 1)); i++, p++) {
                h->sym[p] = (uint8_t)s;
                h->nb[p] = (uint8_t)(maxbits + 1 - wv);
            }
        }
    }
    return 0;
}

/* Huffman tree description -> table; returns bytes used or -1 */
static int huf_read(huf_table *h, const uint8_t *in, size_t n) {
    if (n < 1) return -1;
    const int hb = in[0];
    uint8_t w[256];
    int nw = 0;
    if (hb >= 128) {  /* direct 4-bit weights */
        nw = hb - 127;
        const int nb = (nw + 1) / 2;
        if ((size_t)nb + 1 > n) return -1;
        for (int i = 0; i < nw; i++) w[i] = (i & 1) ? (in[1 + i / 2] & 15) : (in[1 + i / 2] >> 4);
        if (huf_from_weights(h, w, nw)) return -1;
        return 1 + nb;
    }
    /* FSE-compressed weights: hb bytes = table description + backward stream, two interleaved states */
    if ((size_t)hb + 1 > n || hb == 0) return -1;
    const uint8_t *p = in + 1;
    int16_t norm[256];
    int nsym, al;
    const int used = fse_read_ncount(p, (size_t)hb, norm, &nsym, 255, 6, &al);
    if (used < 0) return -1;
    fse_table ft;
    if (fse_build(&ft, norm, nsym, al)) return -1;
    rev_bits b;
    if (rev_init(&b, p + used, (size_t)(hb - used))) return -1;
    uint32_t s1 = rev_get(&b, al), s2 = rev_get(&b, al);
    if (b.pos < 0) return -1;
    for (;;) {  /* weights alternate between the states until the stream is exhausted */
        if (nw >= 255) return -1;
        w[nw++] = ft.t[s1].sym;
        s1 = ft.t[s1].base + rev_get(&b, ft.t[s1].nb);
        if (b.pos < 0) {
            if (nw >= 255) return -1;
            w[nw++] = ft.t[s2].sym;
            break;
        }
        if (nw >= 255) return -1;
        w[nw++] = ft.t[s2].sym;
        s2 = ft.t[s2].base + rev_get(&b, ft.t[s2].nb);
        if (b.pos < 0) {
            if (nw >= 255) return -1;
            w[nw++] = ft.t[s1].sym;
            break;
        }
    }
    if (huf_from_weights(h, w, nw)) return -1;
    return 1 + hb;
}

static int huf_stream(const huf_table *h, const uint8_t *in, size_t n, uint8_t *out, size_t cnt) {
    rev_bits b;
    if (rev_init(&b, in, n)) return -1;
    for (size_t i = 0; i < cnt; i++) {
        const uint32_t x = rev_peek(&b, h->maxbits);
        out[i] = h->sym[x];
        b.pos -= h->nb[x];
        if (b.pos < 0) return -1;
    }
    return b.pos == 0 ? 0 : -1;
}

static const int16_t kLLDefault[36] = {4, 3, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 2, 1, 1, 1, 2, 2,
                                       2, 2, 2, 2, 2, 2, 2, 3, 2, 1, 1, 1, 1, 1, -1, -1, -1, -1};
static const int16_t kMLDefault[53] = {1, 4, 3, 2, 2, 2, 2, 2, 2, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1, -1, -1};
static const int16_t kOFDefault[29] = {1, 1, 1, 1, 1, 1, 2, 2, 2, 1, 1, 1, 1, 1, 1,
                                       1, 1, 1, 1, 1, 1, 1, 1, 1, -1, -1, -1, -1, -1};
static const uint32_t kLLBase[36] = {0, 1, 2, 3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 18,
                                     20, 22, 24, 28, 32, 40, 48, 64, 128, 256, 512, 1024, 2048, 4096,
                                     8192, 16384, 32768, 65536};
static const uint8_t kLLBits[36] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 1, 1,
                                    1, 1, 2, 2, 3, 3, 4, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16};
static const uint32_t kMLBase[53] = {3, 4, 5, 6, 7, 8, 9, 10, 11, 12, 13, 14, 15, 16, 17, 18, 19, 20,
                                     21, 22, 23, 24, 25, 26, 27, 28, 29, 30, 31, 32, 33, 34, 35, 37,
                                     39, 41, 43, 47, 51, 59, 67, 83, 99, 131, 259, 515, 1027, 2051,
                                     4099, 8195, 16387, 32771, 65539};
static const uint8_t kMLBits[53] = {0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0, 0,
                                    0, 0, 0, 0, 0, 0, 1, 1, 1, 1, 2, 2, 3, 3, 4, 4, 5, 7, 8, 9, 10, 11,
                                    12, 13, 14, 15, 16};

typedef struct {
    fse_table ll, of, ml;
    int have_ll, have_of, have_ml;
    huf_table huf;
    int have_huf;
    uint32_t rep[3];
} zstd_ctx;

/* one sequence table by its mode (0 predefined, 1 RLE, 2 FSE description, 3 repeat); bytes or -1 */
static int seq_table(fse_table *ft, int *have, int mode, const uint8_t *in, size_t n, const int16_t *def, int ndef,
                     int def_al, int max_sym, int max_al) {
    if (mode == 0) {
        if (fse_build(ft, def, ndef, def_al)) return -1;
        *have = 1;
        return 0;
    }
    if (mode == 1) {
        if (n < 1 || in[0] > max_sym) return -1;
        ft->al = 0;
        ft->t[0].sym = in[0];
        ft->t[0].nb = 0;
        ft->t[0].base = 0;
        *have = 1;
        return 1;
    }
    if (mode == 2) {
        int16_t norm[64];
        int nsym, al;
        const int used = fse_read_ncount(in, n, norm, &nsym, max_sym, max_al, &al);
        if (used < 0 || fse_build(ft, norm, nsym, al)) return -1;
        *have = 1;
        return used;
    }
    return *have ? 0 : -1;
}

/* a compressed block -> appended to the frame's output o (frame bytes o->p[fstart, o->len)) */
static int zstd_block(zstd_ctx *z, const uint8_t *in, size_t n, sink *o, size_t fstart, uint64_t window) {
    if (n < 1) return -1;
    /* literals section */
    const int ltype = in[0] & 3, sf = (in[0] >> 2) & 3;
    size_t hdr, regen, csize = 0;
    int streams = 1;
    if (ltype < 2) {
        if (sf == 0 || sf == 2) { hdr = 1; regen = in[0] >> 3; }
        else if (sf == 1) { if (n < 2) return -1; hdr = 2; regen = (in[0] >> 4) + ((size_t)in[1] << 4); }
        else { if (n < 3) return -1; hdr = 3; regen = (in[0] >> 4) + ((size_t)in[1] << 4) + ((size_t)in[2] << 12); }
    } else {
        if (sf <= 1) {
            if (n < 3) return -1;
            const uint32_t h = in[0] | (uint32_t)in[1] << 8 | (uint32_t)in[2] << 16;
            hdr = 3; regen = (h >> 4) & 0x3FF; csize = (h >> 14) & 0x3FF; streams = sf == 0 ? 1 : 4;
        } else if (sf == 2) {
            if (n < 4) return -1;
            const uint32_t h = rd32(in);
            hdr = 4; regen = (h >> 4) & 0x3FFF; csize = h >> 18; streams = 4;
        } else {
            if (n < 5) return -1;
            const uint64_t h = (uint64_t)rd32(in) | (uint64_t)in[4] << 32;
            hdr = 5; regen = (size_t)((h >> 4) & 0x3FFFF); csize = (size_t)((h >> 22) & 0x3FFFF); streams = 4;
        }
    }
    if (regen > 128 * 1024) return -1;
    uint8_t *lit = (uint8_t *)malloc(regen + 1);
    size_t ip = hdr;
    int rc = -1;
    if (ltype == 0) {
        if (ip + regen > n) goto out;
        memcpy(lit, in + ip, regen);
        ip += regen;
    } else if (ltype == 1) {
        if (ip + 1 > n) goto out;
        memset(lit, in[ip], regen);
        ip += 1;
    } else {
        if (ip + csize > n) goto out;
        const uint8_t *c = in + ip;
        size_t cn = csize;
        if (ltype == 2) {
            const int used = huf_read(&z->huf, c, cn);
            if (used < 0) goto out;
            z->have_huf = 1;
            c += used;
            cn -= (size_t)used;
        } else if (!z->have_huf) {
            goto out;
        }
        if (streams == 1) {
            if (huf_stream(&z->huf, c, cn, lit, regen)) goto out;
        } else {
            if (cn < 10 || regen < 6) goto out;  /* jump table + a byte per stream; a 4-way split of >= 6 */
            const size_t s1 = c[0] | (size_t)c[1] << 8, s2 = c[2] | (size_t)c[3] << 8, s3 = c[4] | (size_t)c[5] << 8;
            if (6 + s1 + s2 + s3 > cn) goto out;
            const size_t s4 = cn - 6 - s1 - s2 - s3, q = (regen + 3) / 4;
            const uint8_t *p = c + 6;
            if (huf_stream(&z->huf, p, s1, lit, q) || huf_stream(&z->huf, p + s1, s2, lit + q, q) ||
                huf_stream(&z->huf, p + s1 + s2, s3, lit + 2 * q, q) ||
                huf_stream(&z->huf, p + s1 + s2 + s3, s4, lit + 3 * q, regen - 3 * q))
                goto out;
        }
        ip += csize;
    }
    /* sequences section */
    {
        if (ip >= n) goto out;
        size_t nseq = in[ip++];
        if (nseq >= 128) {
            if (nseq < 255) {
                if (ip >= n) goto out;
                nseq = ((nseq - 128) << 8) + in[ip++];
            } else {
                if (ip + 2 > n) goto out;
                nseq = in[ip] + ((size_t)in[ip + 1] << 8) + 0x7F00;
                ip += 2;
            }
        }
        size_t lp = 0;  /* literals consumed */
        const size_t block_start = o->len;
        if (nseq > 0) {
            if (ip >= n) goto out;
            const int modes = in[ip++];
            if (modes & 3) goto out;
            int u;
            u = seq_table(&z->ll, &z->have_ll, modes >> 6, in + ip, n - ip, kLLDefault, 36, 6, 35, 9);
            if (u < 0) goto out;
            ip += (size_t)u;
            u = seq_table(&z->of, &z->have_of, (modes >> 4) & 3, in + ip, n - ip, kOFDefault, 29, 5, 31, 8);
            if (u < 0) goto out;
            ip += (size_t)u;
            u = seq_table(&z->ml, &z->have_ml, (modes >> 2) & 3, in + ip, n - ip, kMLDefault, 53, 6, 52, 9);
            if (u < 0) goto out;
            ip += (size_t)u;
            rev_bits b;
            if (rev_init(&b, in + ip, n - ip)) goto out;
            uint32_t sll = rev_get(&b, z->ll.al), sof = rev_get(&b, z->of.al), sml = rev_get(&b, z->ml.al);
            for (size_t k = 0; k < nseq; k++) {
                const uint32_t ofc = z->of.t[sof].sym, mlc = z->ml.t[sml].sym, llc = z->ll.t[sll].sym;
                if (ofc > 31 || mlc > 52 || llc > 35) goto out;
                uint32_t ofv = (1u << ofc) + rev_get(&b, (int)ofc);
                const uint32_t ml = kMLBase[mlc] + rev_get(&b, kMLBits[mlc]);
                const uint32_t ll = kLLBase[llc] + rev_get(&b, kLLBits[llc]);
                if (k + 1 < nseq) {  /* state updates: literal length, match length, offset */
                    sll = z->ll.t[sll].base + rev_get(&b, z->ll.t[sll].nb);
                    sml = z->ml.t[sml].base + rev_get(&b, z->ml.t[sml].nb);
                    sof = z->of.t[sof].base + rev_get(&b, z->of.t[sof].nb);
                }
                if (b.pos < 0) goto out;
                uint32_t off;
                if (ofv > 3) {
                    off = ofv - 3;
                    z->rep[2] = z->rep[1];
                    z->rep[1] = z->rep[0];
                    z->rep[0] = off;
                } else {
                    const uint32_t idx = ll == 0 ? ofv : ofv - 1;  /* ll == 0: repeat codes shift by one */
                    if (idx == 0) {
                        off = z->rep[0];
                    } else {
                        off = idx == 3 ? z->rep[0] - 1 : z->rep[idx];
                        if (idx > 1) z->rep[2] = z->rep[1];
                        z->rep[1] = z->rep[0];
                        z->rep[0] = off;
                    }
                }
                if (ll > regen - lp) goto out;
                for (uint32_t i = 0; i < ll; i++)
                    if (put_byte(o, lit[lp + i])) goto out;
                lp += ll;
                if (off == 0 || off > o->len - fstart || off > window) goto out;
                for (uint32_t i = 0; i < ml; i++) {
                    const uint8_t x = o->p ? o->p[o->len - off] : 0;
                    if (put_byte(o, x)) goto out;
                }
            }
            if (b.pos != 0) goto out;
        } else if (ip != n) {
            goto out;
        }
        for (; lp < regen; lp++)
            if (put_byte(o, lit[lp])) goto out;
        if (o->len - block_start > 128 * 1024) goto out;
    }
    rc = 0;
out:
    free(lit);
    return rc;
}

/* zstd::stream::decode_all -> 0 or -1 */
static int zstd_decode(const uint8_t *in, size_t n, sink *o) {
    size_t ip = 0;
    while (ip < n) {
        if (n - ip < 4) return -1;
        const uint32_t magic = rd32(in + ip);
        ip += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {  /* skippable frame */
            if (n - ip < 4) return -1;
            const uint32_t sz = rd32(in + ip);
            ip += 4;
            if (n - ip < sz) return -1;
            ip += sz;
            continue;
        }
        if (magic != 0xFD2FB528u) return -1;
        if (ip >= n) return -1;
        const uint32_t fhd = in[ip++];
        const int fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
        if (fhd & 8) return -1;  /* reserved bit */
        uint64_t window = 0;
        if (!single) {
            if (ip >= n) return -1;
            const uint32_t wd = in[ip++];
            const int wlog = 10 + (int)(wd >> 3);
            const uint64_t base = 1ull << wlog;
            window = base + (base / 8) * (wd & 7);
        }
        static const int kDid[4] = {0, 1, 2, 4};
        if (n - ip < (size_t)kDid[did_flag]) return -1;
        uint32_t did = 0;
        for (int i = 0; i < kDid[did_flag]; i++) did |= (uint32_t)in[ip + i] << (8 * i);
        ip += kDid[did_flag];
        if (did) return -1;  /* no dictionary loaded */
        const int fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (n - ip < (size_t)fcs_len) return -1;
        uint64_t fcs = 0;
        int has_fcs = fcs_len > 0;
        for (int i = 0; i < fcs_len; i++) fcs |= (uint64_t)in[ip + i] << (8 * i);
        if (fcs_len == 2) fcs += 256;
        ip += fcs_len;
        if (single) window = fcs;
        if (window > (1ull << 27) + 1) return -1;  /* ZSTD_MAXWINDOWSIZE_DEFAULT */
        zstd_ctx z;
        memset(&z, 0, sizeof(z));
        z.rep[0] = 1;
        z.rep[1] = 4;
        z.rep[2] = 8;
        const size_t fstart = o->len;
        const uint64_t bmax = window < 128 * 1024 ? window : 128 * 1024;
        for (;;) {
            if (n - ip < 3) return -1;
            const uint32_t bh = in[ip] | (uint32_t)in[ip + 1] << 8 | (uint32_t)in[ip + 2] << 16;
            ip += 3;
            const int last = bh & 1, type = (bh >> 1) & 3;
            const size_t bs = bh >> 3;
            if (type == 3) return -1;
            if (type == 1) {  /* RLE: one byte, bs times */
                if (bs > bmax || ip >= n) return -1;
                for (size_t i = 0; i < bs; i++)
                    if (put_byte(o, in[ip])) return -1;
                ip += 1;
            } else {
                if (n - ip < bs || bs > bmax) return -1;
                if (type == 0) {
                    for (size_t i = 0; i < bs; i++)
                        if (put_byte(o, in[ip + i])) return -1;
                } else if (zstd_block(&z, in + ip, bs, o, fstart, window)) {
                    return -1;
                }
                ip += bs;
            }
            if (last) break;
        }
        if (has_fcs && o->len - fstart != fcs) return -1;
        if (checksum) {
            if (n - ip < 4) return -1;
            if (o->p && (uint32_t)orc_xxh64(o->p + fstart, o->len - fstart, 0) != rd32(in + ip)) return -1;
            ip += 4;
        }
    }
    return 0;
}

/* ------------------------------------------------------------------------------------------- */
/* Entry points for the codec dispatch in sdb_oracle.c                                          */
/* ------------------------------------------------------------------------------------------- */
/* The decoded size of a zstd stream from its frame headers alone (RFC 8878 3.1.1.1.4 Frame_Content_Size;
 * the reference's encoder, zstd::bulk::compress at format/sst.rs:590, always writes it): frame and
 * block headers are walked, nothing is entropy-decoded.  -1 when a frame has no content size or a
 * header is malformed (the plan then decodes in count mode). */
static int64_t zstd_frames_size(const uint8_t *in, size_t n) {
    size_t ip = 0;
    uint64_t sum = 0;
    while (ip < n) {
        if (n - ip < 4) return -1;
        const uint32_t magic = rd32(in + ip);
        ip += 4;
        if ((magic & 0xFFFFFFF0u) == 0x184D2A50u) {
            if (n - ip < 4) return -1;
            const uint32_t sz = rd32(in + ip);
            ip += 4;
            if (n - ip < sz) return -1;
            ip += sz;
            continue;
        }
        if (magic != 0xFD2FB528u || ip >= n) return -1;
        const unsigned fhd = in[ip++];
        const unsigned fcs_flag = fhd >> 6, single = (fhd >> 5) & 1, checksum = (fhd >> 2) & 1, did_flag = fhd & 3;
        if (fhd & 8) return -1;
        const size_t fcs_len = fcs_flag == 0 ? (single ? 1 : 0) : fcs_flag == 1 ? 2 : fcs_flag == 2 ? 4 : 8;
        if (!fcs_len) return -1;
        const size_t skip = (single ? 0 : 1) + (did_flag == 3 ? 4 : did_flag);
        if (n - ip < skip + fcs_len) return -1;
        ip += skip;
        uint64_t fcs = 0;
        for (size_t i = 0; i < fcs_len; i++) fcs |= (uint64_t)in[ip + i] << (8 * i);
        if (fcs_len == 2) fcs += 256;
        ip += fcs_len;
        for (;;) {
            if (n - ip < 3) return -1;
            const uint32_t bh = in[ip] | (uint32_t)in[ip + 1] << 8 | (uint32_t)in[ip + 2] << 16;
            ip += 3;
            const unsigned type = (bh >> 1) & 3;
            const size_t csz = type == 1 ? 1 : (size_t)(bh >> 3);
            if (type == 3 || n - ip < csz) return -1;
            ip += csz;
            if (bh & 1) break;
        }
        if (checksum) {
            if (n - ip < 4) return -1;
            ip += 4;
        }
        sum += fcs;
        if (sum > (64ull << 20)) return -1;
    }
    return (int64_t)sum;
}

int64_t orc_entropy_len(uint32_t codec, const uint8_t *in, size_t n) {
    if (codec != 2) {
        const int64_t f = zstd_frames_size(in, n);
        if (f >= 0) return f;
    }
    /* count mode, as the device plan: the bytes are not kept, so Adler-32 / XXH64 are verified only by
     * the decode proper (a stream whose checksum fails gets a slot here and fails in step 2) */
    sink o = {NULL, (size_t)1 << 40, 0, 0};
    const int r = codec == 2 ? zlib_decode(in, n, &o) : zstd_decode(in, n, &o);
    return r || o.overflow ? -1 : (int64_t)o.len;
}

sdb_status orc_entropy_decompress(uint32_t codec, const uint8_t *in, size_t n, uint8_t *out, size_t cap,
                                  size_t *out_len) {
    sink o = {out, cap, 0, 0};
    const int r = codec == 2 ? zlib_decode(in, n, &o) : zstd_decode(in, n, &o);
    *out_len = o.len;
    /* zstd: a slot sized from the frames' content sizes overflows only when a frame decodes to more than
     * it declares, which libzstd reports as corruption (the reference: BlockDecompressionError) */
    if (o.overflow) return codec == 2 ? SDB_INVALID_ARGUMENT : SDB_DECOMPRESSION_ERROR;
    return r ? SDB_DECOMPRESSION_ERROR : SDB_OK;
}
