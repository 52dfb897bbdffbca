/* Host half of the hybrid JPEG decode (include/hkp_jpeg.h): marker parsing and
 * Huffman entropy decoding of baseline JPEGs into quantised DCT coefficients.
 * Plain C (gcc), no GPU runtime: the data loader's forked workers call it.
 *
 * Follows ITU-T T.81 (the JPEG standard): Annex B (syntax: SOI, DQT, SOF0/1,
 * DHT, DRI, SOS, RSTn, EOI), Annex C (canonical Huffman tables from BITS /
 * HUFFVAL), F.2.2 (DC difference and AC run/size decoding, EXTEND), and the
 * behaviour of libjpeg-turbo 3.1 (the decoder behind the reference's
 * cv2.imread, dataset.py:71, and Pillow) where T.81 leaves a choice: a marker
 * met inside entropy-coded data ends the data and the remaining bits read as
 * zeros; restart markers reset the DC predictors.  The decode table layout
 * (a 9-bit lookahead table plus per-length maxcode / value offsets) is the
 * usual canonical-code scheme of T.81 Figure F.16. */
#include <stdint.h>
#include <stdio.h>
#include <stdarg.h>
#include <string.h>

#include "../../../include/hkp_jpeg.h"

static __thread char g_err[256];

static int fail(int code, const char* fmt, ...) {
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(g_err, sizeof g_err, fmt, ap);
    va_end(ap);
    return code;
}

const char* hkpj_last_error(void) { return g_err; }

/* zig-zag scan position -> natural (row-major) index, T.81 Figure A.6 */
static const uint8_t k_natural[64] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,
    12, 19, 26, 33, 40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28,
    35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23, 30, 37, 44, 51,
    58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63};

#define LOOK 9
#define FAST 10                    /* AC symbol + its extra bits decoded by one lookup */

typedef struct {
    int present;
    uint8_t look_len[1 << LOOK];   /* code length of a LOOK-bit prefix, 0: longer code */
    uint8_t look_sym[1 << LOOK];
    /* AC tables: for a FAST-bit prefix holding a whole nonzero run/size code and
     * its extra bits, (value << 16) | (run << 8) | bits consumed; 0 otherwise */
    int32_t fast_ac[1 << FAST];
    int32_t maxcode[18];           /* largest code of each length, -1: none */
    int32_t valoff[17];            /* HUFFVAL index = code + valoff[len] */
    int32_t nval;
    uint8_t val[256];
} htab;

typedef struct {
    const uint8_t* p;              /* next unread byte of entropy-coded data */
    const uint8_t* end;
    uint64_t buf;                  /* bits, MSB-aligned at bit 63 */
    int nbits;
    int hit_marker;                /* a marker ended the data: feed zeros */
} bitreader;

typedef struct {
    uint16_t qt[4][64];
    int qt_present[4];
    htab dc[4], ac[4];
    int sof;                       /* SOF marker seen */
    int cid[3];                    /* component identifiers */
    int adobe_transform;           /* APP14 Adobe transform flag, -1: no marker */
    int scan_seen;
    int scan_td[3], scan_ta[3];    /* per component (frame order) */
    const uint8_t* scan_data;      /* first byte of the first scan's entropy-coded data */
} parser;

static int build_htab(htab* t, const uint8_t* bits, const uint8_t* vals, int nvals) {
    int huffsize[257], huffcode[257];
    int p = 0;
    for (int l = 1; l <= 16; ++l)
        for (int i = 0; i < bits[l - 1]; ++i) huffsize[p++] = l;
    huffsize[p] = 0;
    if (p != nvals) return fail(HKPJ_ERR_FORMAT, "DHT: %d symbols counted, %d given", p, nvals);
    int code = 0, si = huffsize[0];
    p = 0;
    while (huffsize[p]) {
        while (huffsize[p] == si) {
            huffcode[p++] = code;
            ++code;
        }
        if (code >= (1 << si)) return fail(HKPJ_ERR_FORMAT, "DHT: bad code lengths");
        code <<= 1;
        ++si;
    }
    p = 0;
    for (int l = 1; l <= 16; ++l) {
        if (bits[l - 1]) {
            t->valoff[l] = p - huffcode[p];
            p += bits[l - 1];
            t->maxcode[l] = huffcode[p - 1];
        } else {
            t->maxcode[l] = -1;
        }
    }
    t->maxcode[17] = 0x7FFFFFFF;
    memcpy(t->val, vals, (size_t)nvals);
    t->nval = nvals;
    memset(t->look_len, 0, sizeof t->look_len);
    p = 0;
    for (int l = 1; l <= LOOK; ++l)
        for (int i = 0; i < bits[l - 1]; ++i, ++p) {
            const int base = huffcode[p] << (LOOK - l);
            for (int k = 0; k < (1 << (LOOK - l)); ++k) {
                t->look_len[base + k] = (uint8_t)l;
                t->look_sym[base + k] = vals[p];
            }
        }
    memset(t->fast_ac, 0, sizeof t->fast_ac);
    p = 0;
    for (int l = 1; l <= FAST; ++l)
        for (int i = 0; i < bits[l - 1]; ++i, ++p) {
            const int r = vals[p] >> 4, sz = vals[p] & 15;
            if (sz == 0 || l + sz > FAST) continue;        /* EOB / ZRL / too long: the table walk */
            const int base = huffcode[p] << (FAST - l);
            for (int k = 0; k < (1 << (FAST - l)); ++k) {
                const int extra = k >> (FAST - l - sz);
                const int v = extra < (1 << (sz - 1)) ? extra - (1 << sz) + 1 : extra;
                t->fast_ac[base + k] = (int32_t)((uint32_t)v << 16) | (r << 8) | (l + sz);
            }
        }
    t->present = 1;
    return HKPJ_OK;
}

static inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

/* Headers up to (and including) the first SOS. */
static int parse_headers(const uint8_t* data, int64_t size, parser* ps, hkpj_geom* g) {
    memset(ps, 0, sizeof *ps);
    memset(g, 0, sizeof *g);
    ps->adobe_transform = -1;
    if (size < 4 || data[0] != 0xFF || data[1] != 0xD8) return fail(HKPJ_ERR_FORMAT, "no SOI marker");
    const uint8_t* p = data + 2;
    const uint8_t* end = data + size;
    for (;;) {
        while (p < end && *p != 0xFF) ++p;                 /* tolerate garbage between segments */
        while (p < end && *p == 0xFF) ++p;                 /* fill bytes */
        if (p >= end) return fail(HKPJ_ERR_FORMAT, "no SOS before the end of the data");
        const int m = *p++;
        if (m == 0xD8 || (m >= 0xD0 && m <= 0xD7) || m == 0x01) continue;   /* parameterless */
        if (m == 0xD9) return fail(HKPJ_ERR_FORMAT, "EOI before any scan");
        if (end - p < 2) return fail(HKPJ_ERR_FORMAT, "truncated segment");
        const int len = be16(p);
        if (len < 2 || end - p < len) return fail(HKPJ_ERR_FORMAT, "truncated segment (marker %02X)", m);
        const uint8_t* s = p + 2;
        const uint8_t* se = p + len;
        switch (m) {
            case 0xDB:                                     /* DQT */
                while (s < se) {
                    const int pq = s[0] >> 4, tq = s[0] & 15;
                    ++s;
                    if (tq > 3 || pq > 1) return fail(HKPJ_ERR_FORMAT, "DQT: bad table %d / precision %d", tq, pq);
                    if (se - s < (pq ? 128 : 64)) return fail(HKPJ_ERR_FORMAT, "DQT: truncated");
                    for (int i = 0; i < 64; ++i) {
                        ps->qt[tq][k_natural[i]] = pq ? be16(s + 2 * i) : s[i];
                    }
                    s += pq ? 128 : 64;
                    ps->qt_present[tq] = 1;
                }
                break;
            case 0xC4:                                     /* DHT */
                while (s < se) {
                    if (se - s < 17) return fail(HKPJ_ERR_FORMAT, "DHT: truncated");
                    const int tc = s[0] >> 4, th = s[0] & 15;
                    if (tc > 1 || th > 3) return fail(HKPJ_ERR_FORMAT, "DHT: bad class %d / table %d", tc, th);
                    int n = 0;
                    for (int i = 0; i < 16; ++i) n += s[1 + i];
                    if (n > 256 || se - s < 17 + n) return fail(HKPJ_ERR_FORMAT, "DHT: truncated values");
                    const int rc = build_htab(tc ? &ps->ac[th] : &ps->dc[th], s + 1, s + 17, n);
                    if (rc) return rc;
                    s += 17 + n;
                }
                break;
            case 0xC0:
            case 0xC1: {                                   /* SOF0 baseline, SOF1 extended sequential */
                if (ps->sof) return fail(HKPJ_ERR_FORMAT, "two SOF markers");
                if (len < 8) return fail(HKPJ_ERR_FORMAT, "SOF: truncated");
                if (s[0] != 8) return fail(HKPJ_ERR_UNSUPPORTED, "%d-bit samples (8-bit only)", s[0]);
                g->height = be16(s + 1);
                g->width = be16(s + 3);
                g->ncomp = s[5];
                if (g->width <= 0 || g->height <= 0)
                    return fail(HKPJ_ERR_UNSUPPORTED, "image size %dx%d (DNL not supported)", g->width, g->height);
                if ((int64_t)g->width * g->height > (int64_t)1 << 26)
                    return fail(HKPJ_ERR_UNSUPPORTED, "image size %dx%d (at most 64 Mpixel)", g->width, g->height);
                if (g->ncomp != 1 && g->ncomp != 3)
                    return fail(HKPJ_ERR_UNSUPPORTED, "%d components (1 or 3 only)", g->ncomp);
                if (len < 8 + 3 * g->ncomp) return fail(HKPJ_ERR_FORMAT, "SOF: truncated");
                g->hmax = g->vmax = 1;
                for (int c = 0; c < g->ncomp; ++c) {
                    ps->cid[c] = s[6 + 3 * c];
                    g->hs[c] = s[7 + 3 * c] >> 4;
                    g->vs[c] = s[7 + 3 * c] & 15;
                    g->tq[c] = s[8 + 3 * c];
                    if (g->hs[c] < 1 || g->hs[c] > 4 || g->vs[c] < 1 || g->vs[c] > 4 || g->tq[c] > 3)
                        return fail(HKPJ_ERR_FORMAT, "SOF: bad component %d", c);
                    if (g->hs[c] > g->hmax) g->hmax = g->hs[c];
                    if (g->vs[c] > g->vmax) g->vmax = g->vs[c];
                }
                ps->sof = 1;
                break;
            }
            case 0xC2: case 0xC3: case 0xC5: case 0xC6: case 0xC7:
            case 0xC9: case 0xCA: case 0xCB: case 0xCD: case 0xCE: case 0xCF:
                return fail(HKPJ_ERR_UNSUPPORTED, "SOF%d (progressive / lossless / hierarchical / arithmetic)",
                            m - 0xC0);
            case 0xDD:                                     /* DRI */
                if (len < 4) return fail(HKPJ_ERR_FORMAT, "DRI: truncated");
                g->restart_interval = be16(s);
                break;
            case 0xEE:                                     /* APP14: Adobe colour transform flag */
                if (len >= 14 && memcmp(s, "Adobe", 5) == 0) ps->adobe_transform = s[11];
                break;
            case 0xDA: {                                   /* SOS */
                if (!ps->sof) return fail(HKPJ_ERR_FORMAT, "SOS before SOF");
                if (len < 6 + 2 * g->ncomp) return fail(HKPJ_ERR_FORMAT, "SOS: truncated");
                const int ns = s[0];
                if (ns != g->ncomp)
                    return fail(HKPJ_ERR_UNSUPPORTED, "scan of %d of %d components (one interleaved scan only)", ns,
                                g->ncomp);
                if (len < 6 + 2 * ns) return fail(HKPJ_ERR_FORMAT, "SOS: truncated");
                for (int i = 0; i < ns; ++i) {
                    int c = 0;
                    while (c < g->ncomp && ps->cid[c] != s[1 + 2 * i]) ++c;
                    if (c == g->ncomp || c != i)
                        return fail(HKPJ_ERR_UNSUPPORTED, "scan component order differs from the frame's");
                    ps->scan_td[c] = s[2 + 2 * i] >> 4;
                    ps->scan_ta[c] = s[2 + 2 * i] & 15;
                    if (ps->scan_td[c] > 3 || ps->scan_ta[c] > 3) return fail(HKPJ_ERR_FORMAT, "SOS: bad table");
                }
                const int ss = s[1 + 2 * ns], se_ = s[2 + 2 * ns], a = s[3 + 2 * ns];
                if (ss != 0 || se_ != 63 || a != 0)
                    return fail(HKPJ_ERR_UNSUPPORTED, "scan Ss=%d Se=%d Ah/Al=%02X (sequential only)", ss, se_, a);
                ps->scan_seen = 1;
                ps->scan_data = p + len;
                goto done;
            }
            default:                                       /* APPn, COM, DNL, ... */
                break;
        }
        p += len;
    }
done:
    if (g->ncomp == 3 && ps->adobe_transform == 0)
        return fail(HKPJ_ERR_UNSUPPORTED, "Adobe RGB (untransformed) colour");
    for (int c = 0; c < g->ncomp; ++c) {
        const int fh = g->hmax / g->hs[c], fv = g->vmax / g->vs[c];
        if (g->hmax % g->hs[c] || g->vmax % g->vs[c] || fh > 2 || fv > fh)
            return fail(HKPJ_ERR_UNSUPPORTED, "chroma sampling %dx%d of %dx%d (4:4:4, 4:2:2, 4:2:0 only)", g->hs[c],
                        g->vs[c], g->hmax, g->vmax);
        if (!ps->qt_present[g->tq[c]]) return fail(HKPJ_ERR_FORMAT, "missing quantisation table %d", g->tq[c]);
        if (!ps->dc[ps->scan_td[c]].present || !ps->ac[ps->scan_ta[c]].present)
            return fail(HKPJ_ERR_FORMAT, "missing Huffman table for component %d", c);
    }
    const int mcux = (g->width + 8 * g->hmax - 1) / (8 * g->hmax);
    const int mcuy = (g->height + 8 * g->vmax - 1) / (8 * g->vmax);
    int64_t off = 0;
    for (int c = 0; c < g->ncomp; ++c) {
        g->dw[c] = (g->width * g->hs[c] + g->hmax - 1) / g->hmax;
        g->dh[c] = (g->height * g->vs[c] + g->vmax - 1) / g->vmax;
        if (g->ncomp == 1) {                               /* non-interleaved: the component's own block grid */
            g->bw[c] = (g->dw[c] + 7) / 8;
            g->bh[c] = (g->dh[c] + 7) / 8;
        } else {
            g->bw[c] = mcux * g->hs[c];
            g->bh[c] = mcuy * g->vs[c];
        }
        g->blk_off[c] = off;
        off += (int64_t)g->bw[c] * g->bh[c];
    }
    g->nblocks = off;
    return HKPJ_OK;
}

int hkpj_probe(const uint8_t* data, int64_t size, hkpj_geom* g) {
    if (!data || !g || size <= 0) return fail(HKPJ_ERR_ARG, "hkpj_probe: bad arguments");
    parser ps;
    return parse_headers(data, size, &ps, g);
}

/* ---- bit reader: byte-stuffed entropy-coded data (T.81 F.1.2.3) ---- */
static inline void fill(bitreader* br) {
    /* fast path: the next 8 bytes hold no 0xFF (no stuffing, no marker) */
    if (!br->hit_marker && br->end - br->p >= 8) {
        uint64_t v;
        memcpy(&v, br->p, 8);
        const uint64_t inv = ~v;                           /* a 0xFF byte is a zero byte of ~v */
        if (!((inv - 0x0101010101010101ULL) & ~inv & 0x8080808080808080ULL)) {
            v = __builtin_bswap64(v);
            const int take = (64 - br->nbits) >> 3;        /* whole bytes that fit */
            br->buf |= (v >> (64 - 8 * take)) << (64 - br->nbits - 8 * take);
            br->nbits += 8 * take;
            br->p += take;
            return;
        }
    }
    while (br->nbits <= 56) {
        unsigned byte = 0;
        if (!br->hit_marker && br->p < br->end) {
            byte = *br->p;
            if (byte == 0xFF) {
                const unsigned nxt = br->p + 1 < br->end ? br->p[1] : 0xD9;
                if (nxt == 0x00) {
                    br->p += 2;                            /* stuffed zero */
                } else {
                    br->hit_marker = 1;                    /* a marker: the data ends, zeros follow */
                    byte = 0;
                }
            } else {
                ++br->p;
            }
        } else if (!br->hit_marker) {
            br->hit_marker = 1;                            /* out of bytes: zeros */
        }
        br->buf |= (uint64_t)byte << (56 - br->nbits);
        br->nbits += 8;
    }
}

static inline unsigned peek(bitreader* br, int n) { return (unsigned)(br->buf >> (64 - n)); }

static inline void skip(bitreader* br, int n) {
    br->buf <<= n;
    br->nbits -= n;
}

static inline int get_bits(bitreader* br, int n) {
    if (n == 0) return 0;
    if (br->nbits < n) fill(br);
    const int v = (int)peek(br, n);
    skip(br, n);
    return v;
}

/* one Huffman symbol; -1 on an invalid code */
static inline int decode_sym(bitreader* br, const htab* t) {
    if (br->nbits < 16) fill(br);
    const unsigned look = peek(br, LOOK);
    const int l0 = t->look_len[look];
    if (l0) {
        skip(br, l0);
        return t->look_sym[look];
    }
    int l = LOOK + 1;
    int code = (int)peek(br, l);
    while (l <= 16 && code > t->maxcode[l]) {
        ++l;
        code = (int)peek(br, l);
    }
    if (l > 16) return -1;
    const int idx = code + t->valoff[l];
    if (idx < 0 || idx >= t->nval) return -1;              /* corrupt data: never index outside HUFFVAL */
    skip(br, l);
    return t->val[idx];
}

/* EXTEND (T.81 Figure F.12) */
static inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v - (1 << s) + 1 : v; }

/* a symbol (<= 16 bits) and its extra bits (<= 15) need at most 31 bits: one
 * refill check per symbol, none inside */
static inline int take_bits(bitreader* br, int n) {
    if (n == 0) return 0;
    const int v = (int)peek(br, n);
    skip(br, n);
    return v;
}

static int decode_block(bitreader* br, const htab* dc, const htab* ac, int* pred, int16_t* out) {
    memset(out, 0, 64 * sizeof(int16_t));
    if (br->nbits < 32) fill(br);
    int s = decode_sym(br, dc);
    if (s < 0 || s > 15) return fail(HKPJ_ERR_CORRUPT, "bad DC code");
    const int diff = s ? extend(take_bits(br, s), s) : 0;
    *pred += diff;
    out[0] = (int16_t)*pred;
    for (int k = 1; k < 64;) {
        if (br->nbits < 32) fill(br);
        const int32_t f = ac->fast_ac[peek(br, FAST)];
        if (f) {
            k += (f >> 8) & 15;
            if (k > 63) return fail(HKPJ_ERR_CORRUPT, "AC run past the block");
            out[k_natural[k]] = (int16_t)(f >> 16);
            skip(br, f & 255);
            ++k;
            continue;
        }
        const int rs = decode_sym(br, ac);
        if (rs < 0) return fail(HKPJ_ERR_CORRUPT, "bad AC code");
        const int r = rs >> 4;
        s = rs & 15;
        if (s) {
            k += r;
            if (k > 63) return fail(HKPJ_ERR_CORRUPT, "AC run past the block");
            out[k_natural[k]] = (int16_t)extend(take_bits(br, s), s);
            ++k;
        } else if (r == 15) {
            k += 16;                                       /* ZRL */
        } else {
            break;                                         /* EOB */
        }
    }
    return HKPJ_OK;
}

/* At a restart boundary: drop the buffered bits (byte alignment), step over the
 * RSTn marker and any fill bytes, clear the marker state. */
static int restart(bitreader* br, int expect) {
    br->buf = 0;
    br->nbits = 0;
    br->hit_marker = 0;
    const uint8_t* p = br->p;
    while (p < br->end && *p == 0xFF && p + 1 < br->end && p[1] == 0xFF) ++p;
    if (p + 1 < br->end && p[0] == 0xFF && p[1] == (uint8_t)(0xD0 + expect)) {
        br->p = p + 2;
        return HKPJ_OK;
    }
    return fail(HKPJ_ERR_CORRUPT, "expected RST%d marker", expect);
}

int hkpj_decode(const uint8_t* data, int64_t size, const hkpj_geom* g, int16_t* coefs, uint16_t* qt) {
    if (!data || !g || !coefs || !qt || size <= 0) return fail(HKPJ_ERR_ARG, "hkpj_decode: bad arguments");
    parser ps;
    hkpj_geom gg;
    int rc = parse_headers(data, size, &ps, &gg);
    if (rc) return rc;
    if (gg.nblocks != g->nblocks || gg.width != g->width || gg.height != g->height || gg.ncomp != g->ncomp)
        return fail(HKPJ_ERR_ARG, "hkpj_decode: geometry differs from these bytes' headers");
    for (int c = 0; c < gg.ncomp; ++c) memcpy(qt + 64 * c, ps.qt[gg.tq[c]], 64 * sizeof(uint16_t));

    bitreader br = {ps.scan_data, data + size, 0, 0, 0};
    int pred[3] = {0, 0, 0};
    const int ri = gg.restart_interval;
    int to_go = ri, next_rst = 0;
    if (gg.ncomp == 1) {
        const htab* dc = &ps.dc[ps.scan_td[0]];
        const htab* ac = &ps.ac[ps.scan_ta[0]];
        const int64_t n = gg.nblocks;
        for (int64_t b = 0; b < n; ++b) {
            if (ri && to_go == 0) {
                if ((rc = restart(&br, next_rst))) return rc;
                next_rst = (next_rst + 1) & 7;
                pred[0] = 0;
                to_go = ri;
            }
            if ((rc = decode_block(&br, dc, ac, &pred[0], coefs + 64 * b))) return rc;
            --to_go;
        }
        return HKPJ_OK;
    }
    const int mcux = gg.bw[0] / gg.hs[0], mcuy = gg.bh[0] / gg.vs[0];
    for (int my = 0; my < mcuy; ++my)
        for (int mx = 0; mx < mcux; ++mx) {
            if (ri && to_go == 0) {
                if ((rc = restart(&br, next_rst))) return rc;
                next_rst = (next_rst + 1) & 7;
                pred[0] = pred[1] = pred[2] = 0;
                to_go = ri;
            }
            for (int c = 0; c < gg.ncomp; ++c) {
                const htab* dc = &ps.dc[ps.scan_td[c]];
                const htab* ac = &ps.ac[ps.scan_ta[c]];
                for (int v = 0; v < gg.vs[c]; ++v)
                    for (int h = 0; h < gg.hs[c]; ++h) {
                        const int64_t bx = (int64_t)mx * gg.hs[c] + h, by = (int64_t)my * gg.vs[c] + v;
                        int16_t* out = coefs + 64 * (gg.blk_off[c] + by * gg.bw[c] + bx);
                        if ((rc = decode_block(&br, dc, ac, &pred[c], out))) return rc;
                    }
            }
            --to_go;
        }
    return HKPJ_OK;
}
