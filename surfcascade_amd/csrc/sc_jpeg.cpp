// sc_jpeg.cpp -- JPEG -> 8-bit grayscale, the input side of the detect path
// (SURVEY.md 8f row f4): ObjDetector reads every FDDB image with
// cv::imread(prefix + path + ".jpg", cv::IMREAD_GRAYSCALE) (ObjDetector.cpp:164).
//
// OpenCV 3.0.0 decodes JPEG with its bundled IJG libjpeg; for a grayscale
// read of a 1- or 3-component (YCbCr) file it asks libjpeg for
// out_color_space = JCS_GRAYSCALE, which is the luma component as decoded:
// Huffman entropy decoding (baseline, extended-sequential or progressive),
// dequantisation, the default JDCT_ISLOW integer inverse DCT (LL&M,
// CONST_BITS 13, PASS1_BITS 2) and the post-IDCT range-limit table.  The
// chroma planes are entropy-decoded (to walk the bitstream) but never
// transformed.  libjpeg itself is not in /root/reference: this is a
// restatement of the published algorithm (ITU T.81 Annex F/G, IJG jidctint.c
// islow, jdphuff.c refinement rules), pinned in tests/test_jpeg.py against
// libjpeg-turbo (Pillow's decoder, bit-compatible with IJG islow) on
// baseline, restart-interval, subsampled and progressive files.
//
// Host code: entropy decoding is a serial bit stream per scan, and the
// frames reach the detector as u8 planes either way.  Arithmetic coding,
// 12-bit, lossless, CMYK/YCCK and subsampled luma are rejected.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "sc_jpeg.hpp"

namespace sc {
namespace {

// natural order of the zig-zag index (T.81 Figure A.6); the extra entries
// absorb a corrupt run past position 63 as libjpeg's jpeg_natural_order does
const int kZigzag[80] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33,
    40, 48, 41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36,
    29, 22, 15, 23, 30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54,
    47, 55, 62, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

constexpr long long kMaxPixels = 1ll << 28;

struct Fail {
    std::string msg;
};

struct Huff {  // T.81 Annex C canonical code, decoded by length (F.2.2.3)
    bool present = false;
    int mincode[17], maxcode[18], valptr[17];
    uint8_t vals[256];
    // fast path: the first 9 bits -> (length << 8 | symbol), 0 = longer code
    uint16_t look[512];
};

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0;
    int bw = 0, bh = 0;  // blocks across / down in the padded MCU grid
    int dc_tbl = 0, ac_tbl = 0;
    int dc_pred = 0;
};

// Entropy-coded segment reader: byte stuffing (FF 00 -> FF); a marker ends the
// data and, as in libjpeg, zeros are fed from there on.
struct Bits {
    const uint8_t *p, *end;
    uint32_t acc = 0;
    int n = 0;
    bool hit_marker = false;
    int marker = 0;
    void fill() {
        while (n <= 24) {
            int b = 0;
            if (!hit_marker && p < end) {
                b = *p;
                if (b == 0xFF) {
                    int b2 = p + 1 < end ? p[1] : 0xD9;
                    while (b2 == 0xFF && p + 2 < end) {  // fill bytes
                        p++;
                        b2 = p[1];
                    }
                    if (b2 == 0x00) {
                        p += 2;
                    } else {
                        hit_marker = true;
                        marker = b2;
                        b = 0;
                    }
                } else {
                    p++;
                }
            }
            acc |= (uint32_t)b << (24 - n);
            n += 8;
        }
    }
    int bit() {
        if (n < 1) fill();
        const int r = (int)(acc >> 31);
        acc <<= 1;
        n--;
        return r;
    }
    int get(int s) {  // s <= 16
        if (s == 0) return 0;
        if (n < s) fill();
        const int r = (int)(acc >> (32 - s));
        acc <<= s;
        n -= s;
        return r;
    }
    int peek9() {
        if (n < 9) fill();
        return (int)(acc >> 23);
    }
    void skip(int s) {
        acc <<= s;
        n -= s;
    }
    // restart: drop the partial byte, consume the RSTn marker
    void restart(int expect) {
        acc = 0;
        n = 0;
        if (!hit_marker) {  // find the marker (tolerate trailing padding)
            while (p < end) {
                if (*p == 0xFF && p + 1 < end && p[1] != 0x00 && p[1] != 0xFF) break;
                p++;
            }
            if (p + 1 < end) {
                hit_marker = true;
                marker = p[1];
            }
        }
        if (hit_marker && marker == 0xD0 + expect) {
            // p points at FF of the marker
            while (p < end && *p != 0xFF) p++;
            p = end - p > 2 ? p + 2 : end;
            hit_marker = false;
        }
        // a missing / wrong RSTn: continue (libjpeg resyncs; corrupt input)
    }
};

int decode_huff(Bits &b, const Huff &h) {
    const int lk = h.look[b.peek9()];
    if (lk) {
        b.skip(lk >> 8);
        return lk & 0xff;
    }
    int code = b.get(9);
    for (int l = 10; l <= 16; l++) {
        code = (code << 1) | b.bit();
        if (code <= h.maxcode[l]) return h.vals[h.valptr[l] + code - h.mincode[l]];
    }
    return 0;  // corrupt data: libjpeg warns and returns 0
}

inline int extend(int v, int s) {  // F.2.2.1 EXTEND
    return (s > 0 && v < (1 << (s - 1))) ? v - (1 << s) + 1 : v;
}

// jidctint.c jpeg_idct_islow (IJG; 6b / turbo / 9a produce the same values):
// dequantise, columns then rows, DESCALE with round-half-up, range-limit.
constexpr int kConstBits = 13, kPass1Bits = 2;
constexpr int32_t F0_298 = 2446, F0_390 = 3196, F0_541 = 4433, F0_765 = 6270, F0_899 = 7373,
                  F1_175 = 9633, F1_501 = 12299, F1_847 = 15137, F1_961 = 16069, F2_053 = 16819,
                  F2_562 = 20995, F3_072 = 25172;

// The IDCT's products and sums in 32-bit two's-complement arithmetic that
// wraps (unsigned ops, then an arithmetic shift of the signed value): IJG's
// INT32 is `long`, 32 bits on the reference's Win64 build, where corrupt
// coefficients overflow silently; the same bits here, with no signed overflow.
typedef uint32_t u32;
inline int32_t descale(u32 x, int n) { return (int32_t)(x + (1u << (n - 1))) >> n; }

// post-IDCT range limit (jdmaster.c prepare_range_limit_table, masked by 1023)
inline uint8_t range_limit(int32_t v) {
    const int x = v & 1023;
    if (x < 128) return (uint8_t)(x + 128);
    if (x < 512) return 255;
    if (x < 896) return 0;
    return (uint8_t)(x - 896);
}

void idct_islow(const int16_t *coef, const uint16_t *q, uint8_t *out, int ostride) {
    u32 ws[64];
    for (int c = 0; c < 8; c++) {  // pass 1: columns
        const int16_t *in = coef + c;
        const uint16_t *qt = q + c;
        u32 *w = ws + c;
        if (!in[8] && !in[16] && !in[24] && !in[32] && !in[40] && !in[48] && !in[56]) {
            const u32 dc = (u32)in[0] * qt[0] * (1u << kPass1Bits);
            for (int r = 0; r < 8; r++) w[8 * r] = dc;
            continue;
        }
        u32 z2 = (u32)in[16] * qt[16], z3 = (u32)in[48] * qt[48];
        u32 z1 = (z2 + z3) * F0_541;
        u32 tmp2 = z1 + z3 * -F1_847;
        u32 tmp3 = z1 + z2 * F0_765;
        z2 = (u32)in[0] * qt[0];
        z3 = (u32)in[32] * qt[32];
        u32 tmp0 = (z2 + z3) * (1u << kConstBits);
        u32 tmp1 = (z2 - z3) * (1u << kConstBits);
        const u32 tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = (u32)in[56] * qt[56];
        tmp1 = (u32)in[40] * qt[40];
        tmp2 = (u32)in[24] * qt[24];
        tmp3 = (u32)in[8] * qt[8];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        u32 z4 = tmp1 + tmp3;
        const u32 z5 = (z3 + z4) * F1_175;
        tmp0 *= F0_298;
        tmp1 *= F2_053;
        tmp2 *= F3_072;
        tmp3 *= F1_501;
        z1 *= -F0_899;
        z2 *= -F2_562;
        z3 *= -F1_961;
        z4 *= -F0_390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        const int sh = kConstBits - kPass1Bits;
        w[0] = descale(tmp10 + tmp3, sh);
        w[56] = descale(tmp10 - tmp3, sh);
        w[8] = descale(tmp11 + tmp2, sh);
        w[48] = descale(tmp11 - tmp2, sh);
        w[16] = descale(tmp12 + tmp1, sh);
        w[40] = descale(tmp12 - tmp1, sh);
        w[24] = descale(tmp13 + tmp0, sh);
        w[32] = descale(tmp13 - tmp0, sh);
    }
    for (int r = 0; r < 8; r++) {  // pass 2: rows
        const u32 *w = ws + 8 * r;
        uint8_t *o = out + (size_t)r * ostride;
        if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
            const uint8_t v = range_limit(descale(w[0], kPass1Bits + 3));
            for (int c = 0; c < 8; c++) o[c] = v;
            continue;
        }
        u32 z2 = w[2], z3 = w[6];
        u32 z1 = (z2 + z3) * F0_541;
        u32 tmp2 = z1 + z3 * -F1_847;
        u32 tmp3 = z1 + z2 * F0_765;
        u32 tmp0 = (w[0] + w[4]) * (1u << kConstBits);
        u32 tmp1 = (w[0] - w[4]) * (1u << kConstBits);
        const u32 tmp10 = tmp0 + tmp3, tmp13 = tmp0 - tmp3, tmp11 = tmp1 + tmp2, tmp12 = tmp1 - tmp2;
        tmp0 = w[7];
        tmp1 = w[5];
        tmp2 = w[3];
        tmp3 = w[1];
        z1 = tmp0 + tmp3;
        z2 = tmp1 + tmp2;
        z3 = tmp0 + tmp2;
        u32 z4 = tmp1 + tmp3;
        const u32 z5 = (z3 + z4) * F1_175;
        tmp0 *= F0_298;
        tmp1 *= F2_053;
        tmp2 *= F3_072;
        tmp3 *= F1_501;
        z1 *= -F0_899;
        z2 *= -F2_562;
        z3 *= -F1_961;
        z4 *= -F0_390;
        z3 += z5;
        z4 += z5;
        tmp0 += z1 + z3;
        tmp1 += z2 + z4;
        tmp2 += z2 + z3;
        tmp3 += z1 + z4;
        const int sh = kConstBits + kPass1Bits + 3;
        o[0] = range_limit(descale(tmp10 + tmp3, sh));
        o[7] = range_limit(descale(tmp10 - tmp3, sh));
        o[1] = range_limit(descale(tmp11 + tmp2, sh));
        o[6] = range_limit(descale(tmp11 - tmp2, sh));
        o[2] = range_limit(descale(tmp12 + tmp1, sh));
        o[5] = range_limit(descale(tmp12 - tmp1, sh));
        o[3] = range_limit(descale(tmp13 + tmp0, sh));
        o[4] = range_limit(descale(tmp13 - tmp0, sh));
    }
}

struct Decoder {
    const uint8_t *d;
    size_t n, pos = 0;
    uint16_t qt[4][64] = {};  // natural order
    bool qt_set[4] = {};
    Huff dc[4], ac[4];
    std::vector<Comp> comps;
    int W = 0, H = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0;
    bool progressive = false, have_frame = false;
    int restart = 0;
    std::vector<int16_t> coef;  // component 0, [bh][bw][64] natural order
    uint16_t q0[64];             // component 0's table, latched at its first scan
    bool q0_latched = false;
    int eobrun = 0;

    int u8() {
        if (pos >= n) throw Fail{"truncated JPEG"};
        return d[pos++];
    }
    int u16() {
        const int a = u8();
        return (a << 8) | u8();
    }

    void read_dqt(size_t end) {
        while (pos < end) {
            const int pq = u8(), prec = pq >> 4, t = pq & 15;
            if (t > 3 || prec > 1) throw Fail{"bad DQT"};
            for (int i = 0; i < 64; i++) qt[t][kZigzag[i]] = (uint16_t)(prec ? u16() : u8());
            qt_set[t] = true;
        }
    }
    void read_dht(size_t end) {
        while (pos < end) {
            const int tc = u8(), cls = tc >> 4, t = tc & 15;
            if (cls > 1 || t > 3) throw Fail{"bad DHT"};
            Huff &h = cls ? ac[t] : dc[t];
            int counts[17] = {}, total = 0;
            for (int l = 1; l <= 16; l++) total += counts[l] = u8();
            if (total > 256) throw Fail{"bad DHT"};
            for (int i = 0; i < total; i++) h.vals[i] = (uint8_t)u8();
            // canonical codes (C.2) and the decoding tables (F.2.2.3)
            int code = 0, k = 0;
            std::memset(h.look, 0, sizeof(h.look));
            for (int l = 1; l <= 16; l++) {
                h.valptr[l] = k;
                h.mincode[l] = code;
                for (int i = 0; i < counts[l]; i++, k++, code++) {
                    // more codes of length l than l bits hold (libjpeg
                    // jdhuff.c: JERR_BAD_HUFF_TABLE); the lookahead fill
                    // below would index past its 512 entries
                    if (code >= (1 << l)) throw Fail{"bad Huffman table"};
                    if (l <= 9) {
                        const int sh = 9 - l;
                        for (int f = 0; f < (1 << sh); f++)
                            h.look[(code << sh) | f] = (uint16_t)((l << 8) | h.vals[k]);
                    }
                }
                h.maxcode[l] = counts[l] ? code - 1 : -1;
                code <<= 1;
            }
            h.maxcode[17] = 0x7fffffff;
            h.present = true;
        }
    }
    void read_sof(int m) {
        if (have_frame) throw Fail{"more than one frame"};
        const int p = u8();
        if (p != 8) throw Fail{"only 8-bit JPEG is supported"};
        H = u16();
        W = u16();
        const int nf = u8();
        if (W <= 0 || H <= 0) throw Fail{"JPEG without dimensions (DNL) is not supported"};
        // the coefficient plane is allocated from these two header fields:
        // bound it (twice the largest frame a detector accepts, about 2^27
        // px: sc_api.cpp's 32-bit table offsets) so a 20-byte file cannot
        // ask for gigabytes
        if ((long long)W * H > kMaxPixels) throw Fail{"JPEG larger than 2^28 pixels"};
        if (nf != 1 && nf != 3) throw Fail{"only 1- and 3-component JPEG are supported"};
        comps.resize(nf);
        for (Comp &c : comps) {
            c.id = u8();
            const int hv = u8();
            c.h = hv >> 4;
            c.v = hv & 15;
            c.tq = u8();
            if (c.h < 1 || c.h > 4 || c.v < 1 || c.v > 4 || c.tq > 3) throw Fail{"bad SOF"};
            hmax = std::max(hmax, c.h);
            vmax = std::max(vmax, c.v);
        }
        if (comps[0].h != hmax || comps[0].v != vmax)
            throw Fail{"subsampled luma is not supported"};
        mcux = (W + 8 * hmax - 1) / (8 * hmax);
        mcuy = (H + 8 * vmax - 1) / (8 * vmax);
        for (Comp &c : comps) {
            c.bw = mcux * c.h;
            c.bh = mcuy * c.v;
        }
        progressive = m == 0xC2;
        coef.assign((size_t)comps[0].bw * comps[0].bh * 64, 0);
        have_frame = true;
    }

    // one block of one component: sequential (F.2.2) or a progressive pass (G.1.2)
    void block(Bits &b, Comp &c, int16_t *blk, int ss, int se, int ah, int al) {
        if (!progressive) {
            const int t = decode_huff(b, dc[c.dc_tbl]);
            const int s = t & 15;
            c.dc_pred = (int)((unsigned)c.dc_pred + (unsigned)extend(b.get(s), s));  // (wraps as IJG's int)
            if (blk) blk[0] = (int16_t)c.dc_pred;
            const Huff &ha = ac[c.ac_tbl];
            for (int k = 1; k < 64; k++) {
                const int rs = decode_huff(b, ha), r = rs >> 4, sz = rs & 15;
                if (sz) {
                    k += r;
                    const int v = extend(b.get(sz), sz);
                    if (blk) blk[kZigzag[k]] = (int16_t)v;
                } else {
                    if (r != 15) break;
                    k += 15;
                }
            }
            return;
        }
        if (ss == 0) {  // DC scans
            if (ah == 0) {
                const int t = decode_huff(b, dc[c.dc_tbl]);
                const int s = t & 15;
                c.dc_pred = (int)((unsigned)c.dc_pred + (unsigned)extend(b.get(s), s));
                if (blk) blk[0] = (int16_t)((unsigned)c.dc_pred << al);  // (IJG's LEFT_SHIFT)
            } else if (b.bit() && blk) {
                blk[0] = (int16_t)(blk[0] | (1 << al));
            }
            return;
        }
        const Huff &ha = ac[c.ac_tbl];
        if (ah == 0) {  // AC first pass (jdphuff.c decode_mcu_AC_first)
            if (eobrun > 0) {
                eobrun--;
                return;
            }
            for (int k = ss; k <= se; k++) {
                const int rs = decode_huff(b, ha), r = rs >> 4, sz = rs & 15;
                if (sz) {
                    k += r;
                    const int v = extend(b.get(sz), sz);
                    if (blk) blk[kZigzag[k]] = (int16_t)(v * (1 << al));
                } else if (r == 15) {
                    k += 15;
                } else {
                    eobrun = 1 << r;
                    if (r) eobrun += b.get(r);
                    eobrun--;
                    break;
                }
            }
            return;
        }
        // AC refinement (jdphuff.c decode_mcu_AC_refine)
        const int p1 = 1 << al, m1 = -1 * (1 << al);
        int16_t dummy[64];
        int16_t *bk = blk ? blk : dummy;
        if (!blk) std::memset(dummy, 0, sizeof(dummy));
        int k = ss;
        if (eobrun == 0) {
            for (; k <= se; k++) {
                const int rs = decode_huff(b, ha);
                int r = rs >> 4, s = rs & 15;
                if (s) {
                    s = b.bit() ? p1 : m1;  // (s must be 1; corrupt data tolerated)
                } else if (r != 15) {
                    eobrun = 1 << r;
                    if (r) eobrun += b.get(r);
                    break;
                }
                do {
                    int16_t &cf = bk[kZigzag[k]];
                    if (cf != 0) {
                        if (b.bit() && (cf & p1) == 0) cf = (int16_t)(cf >= 0 ? cf + p1 : cf + m1);
                    } else {
                        if (--r < 0) break;
                    }
                    k++;
                } while (k <= se);
                if (s) bk[kZigzag[k]] = (int16_t)s;
            }
        }
        if (eobrun > 0) {
            for (; k <= se; k++) {
                int16_t &cf = bk[kZigzag[k]];
                if (cf != 0 && b.bit() && (cf & p1) == 0) cf = (int16_t)(cf >= 0 ? cf + p1 : cf + m1);
            }
            eobrun--;
        }
    }

    void read_sos() {
        if (!have_frame) throw Fail{"SOS before SOF"};
        const int ns = u8();
        if (ns < 1 || ns > 4) throw Fail{"bad SOS"};
        std::vector<Comp *> sc;
        for (int i = 0; i < ns; i++) {
            const int id = u8(), tt = u8();
            Comp *c = nullptr;
            for (Comp &x : comps)
                if (x.id == id) c = &x;
            if (!c) throw Fail{"SOS names an unknown component"};
            c->dc_tbl = tt >> 4;
            c->ac_tbl = tt & 15;
            if (c->dc_tbl > 3 || c->ac_tbl > 3) throw Fail{"bad SOS"};
            sc.push_back(c);
        }
        const int ss = u8(), se = u8(), a = u8(), ah = a >> 4, al = a & 15;
        if (progressive) {
            if (ss > se || se > 63 || (ss == 0 && se != 0) || (ss > 0 && ns != 1) || al > 13)
                throw Fail{"bad progressive scan"};
        }
        const bool has0 = std::find(sc.begin(), sc.end(), &comps[0]) != sc.end();
        if (!has0) {  // a chroma-only scan: nothing of it reaches the gray plane
            const uint8_t *p = d + pos;
            while (p + 1 < d + n && !(p[0] == 0xFF && p[1] != 0x00 && p[1] != 0xFF &&
                                      !(p[1] >= 0xD0 && p[1] <= 0xD7)))
                p++;
            pos = (size_t)(p - d);
            return;
        }
        if (has0 && !q0_latched) {  // libjpeg latches a component's table at its first scan
            if (!qt_set[comps[0].tq]) throw Fail{"missing quantisation table"};
            std::memcpy(q0, qt[comps[0].tq], sizeof(q0));
            q0_latched = true;
        }
        for (Comp *c : sc) {
            const bool need_dc = !progressive || (ss == 0 && ah == 0);
            const bool need_ac = !progressive ? true : ss > 0;
            if ((need_dc && !dc[c->dc_tbl].present) || (need_ac && !ac[c->ac_tbl].present))
                throw Fail{"missing Huffman table"};
            c->dc_pred = 0;
        }
        eobrun = 0;
        Bits b{d + pos, d + n};
        // blocks of the scan: interleaved (ns > 1): MCUs of h x v blocks per
        // component; a single component: its own block grid (A.2.2)
        const Comp &c0 = comps[0];
        int since = 0, rst = 0;
        auto tick = [&]() {
            if (restart && ++since == restart) {
                b.restart(rst);
                rst = (rst + 1) & 7;
                since = 0;
                eobrun = 0;
                for (Comp *c : sc) c->dc_pred = 0;
            }
        };
        if (ns == 1) {
            Comp &c = *sc[0];
            // the component's own block grid: ceil(ceil(W*h/hmax) / 8) across
            const int sw = (W * c.h + hmax - 1) / hmax, sh = (H * c.v + vmax - 1) / vmax;
            const int nbx = (sw + 7) / 8, nby = (sh + 7) / 8;
            for (int by = 0; by < nby; by++)
                for (int bx = 0; bx < nbx; bx++) {
                    int16_t *blk = &c == &c0 ? &coef[((size_t)by * c0.bw + bx) * 64] : nullptr;
                    block(b, c, blk, ss, se, ah, al);
                    tick();
                }
        } else {
            for (int my = 0; my < mcuy; my++)
                for (int mx = 0; mx < mcux; mx++) {
                    for (Comp *cp : sc) {
                        Comp &c = *cp;
                        for (int v = 0; v < c.v; v++)
                            for (int h = 0; h < c.h; h++) {
                                int16_t *blk = nullptr;
                                if (&c == &c0)
                                    blk = &coef[((size_t)(my * c.v + v) * c0.bw + mx * c.h + h) * 64];
                                block(b, c, blk, ss, se, ah, al);
                            }
                    }
                    tick();
                }
        }
        // continue after the entropy-coded segment, at its terminating marker
        const uint8_t *p = b.p;
        while (p + 1 < d + n && !(p[0] == 0xFF && p[1] != 0x00 && p[1] != 0xFF &&
                                  !(p[1] >= 0xD0 && p[1] <= 0xD7)))
            p++;
        pos = (size_t)(p - d);
    }

    void run() {
        if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) throw Fail{"not a JPEG file (no SOI)"};
        pos = 2;
        bool scanned = false;
        for (;;) {
            if (pos >= n) {
                if (scanned) break;  // (missing EOI: libjpeg warns and finishes)
                throw Fail{"truncated JPEG"};
            }
            if (d[pos] != 0xFF) {  // garbage between markers: skip (libjpeg warns)
                pos++;
                continue;
            }
            while (pos < n && d[pos] == 0xFF) pos++;
            if (pos >= n) break;
            const int m = d[pos++];
            if (m == 0xD9) break;                      // EOI
            if (m == 0x01 || (m >= 0xD0 && m <= 0xD7)) continue;  // TEM, stray RSTn
            const size_t len = (size_t)u16();
            if (len < 2 || pos + len - 2 > n) throw Fail{"truncated marker segment"};
            const size_t end = pos + len - 2;
            switch (m) {
                case 0xDB: read_dqt(end); break;
                case 0xC4: read_dht(end); break;
                case 0xC0: case 0xC1: case 0xC2: read_sof(m); break;
                case 0xC3: case 0xC5: case 0xC6: case 0xC7: case 0xC9: case 0xCA: case 0xCB:
                case 0xCD: case 0xCE: case 0xCF:
                    throw Fail{"lossless / hierarchical / arithmetic-coded JPEG is not supported"};
                case 0xDD: restart = u16(); break;
                case 0xDA:
                    read_sos();
                    scanned = true;
                    continue;  // pos is at the next marker
                case 0xDC: throw Fail{"DNL marker is not supported"};
                default: break;  // APPn, COM, ...
            }
            pos = end;
        }
        if (!scanned) throw Fail{"JPEG without image data"};
    }

    void render(uint8_t *out) {
        const Comp &c0 = comps[0];
        const uint16_t *q = q0_latched ? q0 : qt[c0.tq];
        uint8_t tile[64];
        for (int by = 0; by * 8 < H; by++)
            for (int bx = 0; bx * 8 < W; bx++) {
                idct_islow(&coef[((size_t)by * c0.bw + bx) * 64], q, tile, 8);
                const int h = std::min(8, H - by * 8), w = std::min(8, W - bx * 8);
                for (int r = 0; r < h; r++)
                    std::memcpy(out + (size_t)(by * 8 + r) * W + bx * 8, tile + 8 * r, w);
            }
    }
};

}  // namespace

int jpeg_gray(const uint8_t *data, size_t len, std::vector<uint8_t> *out, int *w, int *h,
              std::string *err) {
    Decoder dec;
    dec.d = data;
    dec.n = len;
    try {
        dec.run();
    } catch (const Fail &f) {
        *err = f.msg;
        return -1;
    }
    *w = dec.W;
    *h = dec.H;
    if (out) {
        out->resize((size_t)dec.W * dec.H);
        dec.render(out->data());
    }
    return 0;
}

}  // namespace sc
