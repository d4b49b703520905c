// pt_jpeg.cpp — JPEG decoding as the reference's FreeImage_Load(FIF_JPEG, path, 0) produces it
// (Others/image_loader.cpp:31-95; FreeImage.h:693 "JPEG_DEFAULT: loading (see JPEG_FAST)").
//
// FreeImage 3.17 decodes with its bundled IJG libjpeg 9a. Without JPEG_ACCURATE in the flags (the
// reference passes 0), its loader asks libjpeg for the fast integer IDCT and no fancy upsampling.
// That output is restated here:
//   - baseline, extended-sequential and progressive Huffman scans (SOF0/SOF1/SOF2, 8-bit; spectral
//     selection, successive approximation, end-of-band runs), interleaved or not, restart intervals,
//     1 (grey) or 3 (YCbCr, or RGB by Adobe transform 0 / component ids 'R','G','B') components;
//   - the AAN "ifast" IDCT (jidctfst.c) on the scaled quantisation table of jddctmgr.c;
//   - chroma replicated to full size (jdsample.c int_upsample; jdmerge.c merged upsampling is the
//     same arithmetic);
//   - the integer YCbCr -> RGB tables of jdcolor.c.
// Grey images come out as r = g = b (FreeImage_ConvertTo24Bits of an 8-bit grey bitmap).
// Arithmetic-coded, lossless, hierarchical, 12-bit and CMYK files are rejected with an error.
//
// Two arithmetic variants (pt_jpeg_decode):
//   PT_JPEG_IJG9 — libjpeg 9a, what the reference ran (the default of pt_image_load). Its IDCT
//     rounds the final descale (a fudge term on the DC input) and writes the odd part with positive
//     constants; its colour tables use the TIFF 6.0 coefficients 0.344136286 and 0.714136286.
//   PT_JPEG_IJG6 — libjpeg 6b arithmetic, which libjpeg-turbo keeps: a truncating final descale, a
//     negated-constant odd part, and the coefficients 0.34414 and 0.71414. This variant is
//     test infrastructure. tests/test_jpeg.py checks it bit for bit against PIL (libjpeg-turbo)
//     in the same fast mode, which pins everything the two variants share: markers, Huffman
//     decoding, dequantisation, block layout, upsampling and colour conversion.
// Neither libjpeg 9a nor FreeImage is in the checkout. The 9a-specific lines are restated from the
// published source and are unpinned.
// The IDCT, table and colour-conversion arithmetic follow the Independent JPEG Group's libjpeg: this
// software is based in part on the work of the Independent JPEG Group.
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pt_loader.h"
#include "pt_jpeg.h"

namespace {

// zigzag position -> natural (row-major) index, with overrun padding (jutils.c jpeg_natural_order)
const int kNatural[64 + 16] = {
    0,  1,  8,  16, 9,  2,  3,  10, 17, 24, 32, 25, 18, 11, 4,  5,  12, 19, 26, 33, 40, 48,
    41, 34, 27, 20, 13, 6,  7,  14, 21, 28, 35, 42, 49, 56, 57, 50, 43, 36, 29, 22, 15, 23,
    30, 37, 44, 51, 58, 59, 52, 45, 38, 31, 39, 46, 53, 60, 61, 54, 47, 55, 62, 63, 63, 63,
    63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63, 63};

// AAN scale factors scaled by 2^14 (jddctmgr.c aanscales)
const int kAanScales[64] = {
    16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  22725, 31521, 29692, 26722, 22725, 17855, 12299, 6270,
    21407, 29692, 27969, 25172, 21407, 16819, 11585, 5906,  19266, 26722, 25172, 22654, 19266, 15137, 10426, 5315,
    16384, 22725, 21407, 19266, 16384, 12873, 8867,  4520,  12873, 17855, 16819, 15137, 12873, 10114, 6967,  3552,
    8867,  12299, 11585, 10426, 8867,  6967,  4799,  2446,  4520,  6270,  5906,  5315,  4520,  3552,  2446,  1247};

struct Huff {
    bool defined = false;
    int maxcode[18];   // largest code of each length, -1 if none; maxcode[17] sentinel
    int valoffset[18]; // value index = code + valoffset[len]
    uint8_t vals[256];
    int look_len[256]; // 8-bit lookahead: code length (0: longer than 8)
    uint8_t look_val[256];
};

bool build_huff(const uint8_t* counts, const uint8_t* vals, int nvals, Huff& h) {
    // jdhuff.c jpeg_make_d_derived_tbl: canonical codes in order of length
    int code = 0, k = 0;
    std::memset(h.look_len, 0, sizeof(h.look_len));
    for (int l = 1; l <= 16; l++) {
        if (counts[l - 1]) {
            h.valoffset[l] = k - code;
            if (code + counts[l - 1] > (1 << l)) return false;  // more codes than the length allows
            for (int i = 0; i < counts[l - 1]; i++, k++, code++) {
                if (l <= 8) {
                    const int lo = code << (8 - l), n = 1 << (8 - l);
                    for (int j = 0; j < n; j++) { h.look_len[lo + j] = l; h.look_val[lo + j] = vals[k]; }
                }
            }
            h.maxcode[l] = code - 1;
        } else {
            h.maxcode[l] = -1;
            h.valoffset[l] = 0;
        }
        code <<= 1;
    }
    h.maxcode[17] = 0x7fffffff;
    std::memcpy(h.vals, vals, (size_t)nvals);
    h.defined = true;
    return true;
}

// Entropy-coded bits (jdhuff.c fill_bit_buffer): FF 00 is a data FF; a marker ends the data and
// zeros are supplied after it, as libjpeg does on a premature marker.
struct Bits {
    const uint8_t* d;
    size_t n, pos;
    uint32_t acc = 0;
    int cnt = 0;
    bool at_marker = false;
    void fill() {
        while (cnt <= 24) {
            uint32_t b = 0;
            if (!at_marker && pos < n) {
                b = d[pos];
                if (b == 0xFF) {
                    const uint8_t nx = pos + 1 < n ? d[pos + 1] : 0xD9;
                    if (nx == 0x00) pos += 2;
                    else { at_marker = true; b = 0; }
                } else {
                    pos++;
                }
            }
            acc |= b << (24 - cnt);
            cnt += 8;
        }
    }
    int bits(int k) {  // k in 0..16
        if (k == 0) return 0;
        if (cnt < k) fill();
        const int v = (int)(acc >> (32 - k));
        acc <<= k;
        cnt -= k;
        return v;
    }
    int decode(const Huff& h) {
        if (cnt < 16) fill();
        const int peek = (int)(acc >> 24);
        if (h.look_len[peek]) {
            const int l = h.look_len[peek];
            acc <<= l;
            cnt -= l;
            return h.look_val[peek];
        }
        int code = bits(8);
        int l = 8;
        do {
            code = (code << 1) | bits(1);
            l++;
        } while (l <= 16 && code > h.maxcode[l]);
        if (l > 16) return 0;  // corrupt data: libjpeg warns and takes a zero
        return h.vals[(code + h.valoffset[l]) & 0xff];
    }
    // restart marker: drop the partial byte, consume RSTn if it is the next marker
    void restart() {
        acc = 0;
        cnt = 0;
        if (!at_marker) {
            while (pos + 1 < n && !(d[pos] == 0xFF && d[pos + 1] != 0x00 && d[pos + 1] != 0xFF)) pos++;
        }
        while (pos + 1 < n && d[pos] == 0xFF && d[pos + 1] == 0xFF) pos++;
        if (pos + 1 < n && d[pos] == 0xFF && d[pos + 1] >= 0xD0 && d[pos + 1] <= 0xD7) pos += 2;
        at_marker = false;
    }
};

inline int extend(int v, int s) { return v < (1 << (s - 1)) ? v + (int)(~0u << s) + 1 : v; }

struct Comp {
    int id = 0, h = 1, v = 1, tq = 0;
    int bw = 0, bh = 0;        // blocks per row / column, MCU-padded
    int wib = 0, hib = 0;      // blocks covering the component's own samples (non-interleaved scans)
    std::vector<int16_t> coef; // bw * bh blocks of 64, natural order
    int dc_pred = 0, td = 0, ta = 0;
};

// jidctfst.c: MULTIPLY = product descaled by a truncating shift (USE_ACCURATE_ROUNDING unset). The
// IDCT runs in 64-bit integers: equal to libjpeg's int arithmetic wherever that does not overflow
// (every valid file), and defined where a corrupt file would overflow it.
typedef long long i64;
inline i64 fmul(i64 v, int c) { return (v * c) >> 8; }
const int F1_082 = 277, F1_414 = 362, F1_847 = 473, F2_613 = 669;

// The 10-bit (6b) or 9-bit (9a) wrapped range limit of the IDCT output, s = the centred sample.
inline uint8_t limit6(i64 s) {
    const int i = (int)(s & 1023);
    if (i < 128) return (uint8_t)(i + 128);
    if (i < 384) return 255;
    if (i < 896) return 0;
    return (uint8_t)(i - 896);
}
inline uint8_t limit9(i64 s) {
    const int j = (int)((s + 256) & 511) - 128;
    return (uint8_t)(j < 0 ? 0 : (j > 255 ? 255 : j));
}

// One 8x8 block: coefficients (natural order) * the scaled quantisation table -> samples.
template <bool IJG9>
void idct_ifast(const int16_t* in, const int* q, uint8_t* out, int stride) {
    i64 ws[64];
    for (int c = 0; c < 8; c++) {  // pass 1: columns
        const int16_t* ip = in + c;
        const int* qp = q + c;
        i64* wp = ws + c;
        if (!ip[8] && !ip[16] && !ip[24] && !ip[32] && !ip[40] && !ip[48] && !ip[56]) {
            const i64 dc = (i64)ip[0] * qp[0];
            for (int r = 0; r < 8; r++) wp[8 * r] = dc;
            continue;
        }
        i64 t0 = (i64)ip[0] * qp[0], t1 = (i64)ip[16] * qp[16], t2 = (i64)ip[32] * qp[32], t3 = (i64)ip[48] * qp[48];
        i64 t10 = t0 + t2, t11 = t0 - t2, t13 = t1 + t3;
        i64 t12 = fmul(t1 - t3, F1_414) - t13;
        t0 = t10 + t13; t3 = t10 - t13; t1 = t11 + t12; t2 = t11 - t12;
        i64 t4 = (i64)ip[8] * qp[8], t5 = (i64)ip[24] * qp[24], t6 = (i64)ip[40] * qp[40], t7 = (i64)ip[56] * qp[56];
        const i64 z13 = t6 + t5, z10 = t6 - t5, z11 = t4 + t7, z12 = t4 - t7;
        t7 = z11 + z13;
        t11 = fmul(z11 - z13, F1_414);
        const i64 z5 = fmul(z10 + z12, F1_847);
        if (IJG9) {
            t10 = z5 - fmul(z12, F1_082);
            t12 = z5 - fmul(z10, F2_613);
            t6 = t12 - t7; t5 = t11 - t6; t4 = t10 - t5;
            wp[24] = t3 + t4; wp[32] = t3 - t4;
        } else {
            t10 = fmul(z12, F1_082) - z5;
            t12 = fmul(z10, -F2_613) + z5;
            t6 = t12 - t7; t5 = t11 - t6; t4 = t10 + t5;
            wp[32] = t3 + t4; wp[24] = t3 - t4;
        }
        wp[0] = t0 + t7; wp[56] = t0 - t7;
        wp[8] = t1 + t6; wp[48] = t1 - t6;
        wp[16] = t2 + t5; wp[40] = t2 - t5;
    }
    for (int r = 0; r < 8; r++) {  // pass 2: rows, descale by PASS1_BITS + 3 = 5
        const i64* w = ws + 8 * r;
        uint8_t* o = out + (size_t)r * stride;
        // 9a: the rounding term (1 << 4) rides on the DC input; 6b truncates
        const i64 dc = IJG9 ? w[0] + 16 : w[0];
        auto lim = [](i64 v) { return IJG9 ? limit9(v >> 5) : limit6(v >> 5); };
        if (!w[1] && !w[2] && !w[3] && !w[4] && !w[5] && !w[6] && !w[7]) {
            const uint8_t v = lim(dc);
            for (int c = 0; c < 8; c++) o[c] = v;
            continue;
        }
        i64 t10 = dc + w[4], t11 = dc - w[4], t13 = w[2] + w[6];
        i64 t12 = fmul(w[2] - w[6], F1_414) - t13;
        const i64 t0 = t10 + t13, t3 = t10 - t13, t1 = t11 + t12, t2 = t11 - t12;
        const i64 z13 = w[5] + w[3], z10 = w[5] - w[3], z11 = w[1] + w[7], z12 = w[1] - w[7];
        const i64 t7 = z11 + z13;
        t11 = fmul(z11 - z13, F1_414);
        const i64 z5 = fmul(z10 + z12, F1_847);
        i64 t4, t5, t6;
        if (IJG9) {
            t10 = z5 - fmul(z12, F1_082);
            t12 = z5 - fmul(z10, F2_613);
            t6 = t12 - t7; t5 = t11 - t6; t4 = t10 - t5;
            o[3] = lim(t3 + t4); o[4] = lim(t3 - t4);
        } else {
            t10 = fmul(z12, F1_082) - z5;
            t12 = fmul(z10, -F2_613) + z5;
            t6 = t12 - t7; t5 = t11 - t6; t4 = t10 + t5;
            o[4] = lim(t3 + t4); o[3] = lim(t3 - t4);
        }
        o[0] = lim(t0 + t7); o[7] = lim(t0 - t7);
        o[1] = lim(t1 + t6); o[6] = lim(t1 - t6);
        o[2] = lim(t2 + t5); o[5] = lim(t2 - t5);
    }
}

inline uint16_t be16(const uint8_t* p) { return (uint16_t)((p[0] << 8) | p[1]); }

// One scan's parameters: progressive frames code the coefficients in bands (Ss..Se) and bit planes
// (Ah: the previous scan's low bit, Al: this scan's), jdphuff.c; sequential scans take every
// coefficient of a block at once (jdhuff.c decode_mcu).
struct ScanSpec {
    bool prog;
    int ss, se, ah, al;
};

void block_sequential(Bits& br, Comp& cp, int16_t* blk, const Huff* dc_t, const Huff* ac_t) {
    int s = br.decode(dc_t[cp.td]);
    if (s > 15) s = 15;  // corrupt table value (a baseline DC size is at most 11)
    int diff = 0;
    if (s) diff = extend(br.bits(s), s);
    cp.dc_pred = (int)((unsigned)cp.dc_pred + (unsigned)diff);  // libjpeg's int, wrapped
    blk[0] = (int16_t)cp.dc_pred;
    for (int k = 1; k < 64; k++) {
        const int rs = br.decode(ac_t[cp.ta]);
        const int r = rs >> 4, sz = rs & 15;
        if (sz) {
            k += r;
            blk[kNatural[k]] = (int16_t)extend(br.bits(sz), sz);
        } else {
            if (r != 15) break;
            k += 15;
        }
    }
}

// jdphuff.c decode_mcu_DC_first / _DC_refine
void block_dc_prog(Bits& br, Comp& cp, int16_t* blk, const Huff* dc_t, const ScanSpec& sp) {
    if (sp.ah == 0) {
        int s = br.decode(dc_t[cp.td]);
        if (s > 15) s = 15;
        int diff = 0;
        if (s) diff = extend(br.bits(s), s);
        cp.dc_pred = (int)((unsigned)cp.dc_pred + (unsigned)diff);
        blk[0] = (int16_t)((unsigned)cp.dc_pred << sp.al);
    } else if (br.bits(1)) {
        blk[0] = (int16_t)(blk[0] | (1 << sp.al));
    }
}

// jdphuff.c decode_mcu_AC_first: one band of one block, or one block of an end-of-band run
void block_ac_first(Bits& br, const Comp& cp, int16_t* blk, const Huff* ac_t, const ScanSpec& sp, unsigned& eobrun) {
    if (eobrun > 0) {
        eobrun--;
        return;
    }
    for (int k = sp.ss; k <= sp.se; k++) {
        const int rs = br.decode(ac_t[cp.ta]);
        int r = rs >> 4;
        const int sz = rs & 15;
        if (sz) {
            k += r;
            blk[kNatural[k]] = (int16_t)((unsigned)extend(br.bits(sz), sz) << sp.al);
        } else if (r == 15) {
            k += 15;
        } else {
            eobrun = 1u << r;
            if (r) eobrun += (unsigned)br.bits(r);
            eobrun--;
            break;
        }
    }
}

// jdphuff.c decode_mcu_AC_refine: correction bits for the coefficients already nonzero, and the
// newly nonzero ones (magnitude 1 << Al) placed after their run of still-zero coefficients
void block_ac_refine(Bits& br, const Comp& cp, int16_t* blk, const Huff* ac_t, const ScanSpec& sp, unsigned& eobrun) {
    const int p1 = 1 << sp.al, m1 = -(1 << sp.al);
    auto correct = [&](int16_t& c) {
        if (br.bits(1) && (c & p1) == 0) c = (int16_t)(c >= 0 ? c + p1 : c + m1);
    };
    int k = sp.ss;
    if (eobrun == 0) {
        for (; k <= sp.se; k++) {
            const int rs = br.decode(ac_t[cp.ta]);
            int r = rs >> 4;
            int s = rs & 15;
            if (s) {
                s = br.bits(1) ? p1 : m1;  // the new coefficient's sign (its size is 1)
            } else if (r != 15) {
                eobrun = 1u << r;
                if (r) eobrun += (unsigned)br.bits(r);
                break;  // the rest of the band is handled by the end-of-band logic below
            }
            do {
                int16_t& c = blk[kNatural[k]];
                if (c != 0) {
                    correct(c);
                } else if (--r < 0) {
                    break;  // the zero coefficient that becomes nonzero
                }
                k++;
            } while (k <= sp.se);
            if (s) blk[kNatural[k]] = (int16_t)s;
        }
    }
    if (eobrun > 0) {
        for (; k <= sp.se; k++) {
            int16_t& c = blk[kNatural[k]];
            if (c != 0) correct(c);
        }
        eobrun--;
    }
}

bool decode_scan(Bits& br, std::vector<Comp>& comps, const std::vector<int>& sc, const Huff* dc_t, const Huff* ac_t,
                 int mcux, int mcuy, int restart_interval, const ScanSpec& sp) {
    const bool inter = sc.size() > 1;
    int nx, ny;
    if (inter) {
        nx = mcux;
        ny = mcuy;
    } else {
        nx = comps[sc[0]].wib;
        ny = comps[sc[0]].hib;
    }
    for (int c : sc) comps[c].dc_pred = 0;
    unsigned eobrun = 0;
    const long total = (long)nx * ny;
    int todo = restart_interval;
    for (long m = 0; m < total; m++) {
        if (restart_interval) {
            if (todo == 0) {
                br.restart();
                for (int c : sc) comps[c].dc_pred = 0;
                eobrun = 0;
                todo = restart_interval;
            }
            todo--;
        }
        const int mx = (int)(m % nx), my = (int)(m / nx);
        for (int c : sc) {
            Comp& cp = comps[c];
            const int bh = inter ? cp.v : 1, bwid = inter ? cp.h : 1;
            for (int by = 0; by < bh; by++)
                for (int bx = 0; bx < bwid; bx++) {
                    const int col = mx * bwid + bx, row = my * bh + by;
                    int16_t* blk = &cp.coef[((size_t)row * cp.bw + col) * 64];
                    if (!sp.prog) block_sequential(br, cp, blk, dc_t, ac_t);
                    else if (sp.ss == 0) block_dc_prog(br, cp, blk, dc_t, sp);
                    else if (sp.ah == 0) block_ac_first(br, cp, blk, ac_t, sp, eobrun);
                    else block_ac_refine(br, cp, blk, ac_t, sp, eobrun);
                }
        }
    }
    return true;
}

}  // namespace

namespace pt {

bool decode_jpeg(const unsigned char* d, size_t n, int variant, int* out_w, int* out_h,
                 std::vector<unsigned char>& rgba, std::string& err) {
    if (n < 4 || d[0] != 0xFF || d[1] != 0xD8) { err = "not a JPEG file"; return false; }
    int qt[4][64];
    bool qt_def[4] = {false, false, false, false};
    Huff dc_t[4], ac_t[4];
    std::vector<Comp> comps;
    int W = 0, H = 0, hmax = 1, vmax = 1, mcux = 0, mcuy = 0, restart_interval = 0;
    bool frame = false, prog = false, jfif = false, adobe = false, any_scan = false;
    int adobe_transform = -1;
    size_t p = 2;
    while (p + 4 <= n) {
        if (d[p] != 0xFF) { p++; continue; }  // garbage between markers (libjpeg: warning, skip)
        const uint8_t m = d[p + 1];
        if (m == 0xFF) { p++; continue; }
        p += 2;
        if (m == 0xD9) break;                      // EOI
        if (m >= 0xD0 && m <= 0xD7) continue;      // stray RSTn
        if (p + 2 > n) break;
        const size_t len = be16(d + p);
        if (len < 2 || p + len > n) { err = "truncated JPEG segment"; return false; }
        const uint8_t* s = d + p + 2;
        const size_t sl = len - 2;
        if (m == 0xC0 || m == 0xC1 || m == 0xC2) {
            prog = m == 0xC2;
            if (sl < 6 || s[0] != 8) { err = "only 8-bit JPEG is supported"; return false; }
            H = be16(s + 1);
            W = be16(s + 3);
            const int nc = s[5];
            if (W <= 0 || H <= 0 || (nc != 1 && nc != 3) || sl < 6 + 3 * (size_t)nc) {
                err = W <= 0 || H <= 0 ? "bad JPEG frame size" : "only 1- or 3-component JPEG is supported";
                return false;
            }
            comps.assign(nc, Comp());
            for (int i = 0; i < nc; i++) {
                comps[i].id = s[6 + 3 * i];
                comps[i].h = s[7 + 3 * i] >> 4;
                comps[i].v = s[7 + 3 * i] & 15;
                comps[i].tq = s[8 + 3 * i] & 3;
                if (comps[i].h < 1 || comps[i].h > 4 || comps[i].v < 1 || comps[i].v > 4) {
                    err = "bad JPEG sampling factors";
                    return false;
                }
                hmax = std::max(hmax, comps[i].h);
                vmax = std::max(vmax, comps[i].v);
            }
            for (auto& c : comps)
                if (hmax % c.h || vmax % c.v) { err = "fractional JPEG sampling is not supported"; return false; }
            if ((long long)W * H > (1ll << 28)) { err = "JPEG too large"; return false; }
            mcux = (W + 8 * hmax - 1) / (8 * hmax);
            mcuy = (H + 8 * vmax - 1) / (8 * vmax);
            for (auto& c : comps) {
                c.bw = mcux * c.h;
                c.bh = mcuy * c.v;
                c.wib = ((W * c.h + hmax - 1) / hmax + 7) / 8;
                c.hib = ((H * c.v + vmax - 1) / vmax + 7) / 8;
                c.coef.assign((size_t)c.bw * c.bh * 64, 0);
            }
            frame = true;
        } else if (m == 0xC3 || (m >= 0xC5 && m <= 0xC7) || (m >= 0xC9 && m <= 0xCB) || (m >= 0xCD && m <= 0xCF)) {
            err = "this JPEG coding process (lossless, hierarchical or arithmetic) is not supported";
            return false;
        } else if (m == 0xC4) {
            size_t q = 0;
            while (q + 17 <= sl) {
                const int tc = s[q] >> 4, th = s[q] & 15;
                int cnt = 0;
                for (int i = 0; i < 16; i++) cnt += s[q + 1 + i];
                if (th > 3 || tc > 1 || cnt > 256 || q + 17 + cnt > sl) { err = "bad JPEG Huffman table"; return false; }
                Huff& h = tc ? ac_t[th] : dc_t[th];
                if (!build_huff(s + q + 1, s + q + 17, cnt, h)) { err = "bad JPEG Huffman table"; return false; }
                q += 17 + cnt;
            }
        } else if (m == 0xDB) {
            size_t q = 0;
            while (q < sl) {
                const int pq = s[q] >> 4, tq = s[q] & 15;
                if (tq > 3 || q + 1 + 64 * (pq + 1) > sl) { err = "bad JPEG quantisation table"; return false; }
                for (int i = 0; i < 64; i++)
                    qt[tq][kNatural[i]] = pq ? be16(s + q + 1 + 2 * i) : s[q + 1 + i];
                qt_def[tq] = true;
                q += 1 + 64 * (pq + 1);
            }
        } else if (m == 0xDD) {
            if (sl < 2) { err = "bad JPEG restart interval"; return false; }
            restart_interval = be16(s);
        } else if (m == 0xE0) {
            if (sl >= 5 && !std::memcmp(s, "JFIF\0", 5)) jfif = true;
        } else if (m == 0xEE) {
            if (sl >= 12 && !std::memcmp(s, "Adobe", 5)) { adobe = true; adobe_transform = s[11]; }
        } else if (m == 0xDA) {
            if (!frame) { err = "JPEG scan before frame"; return false; }
            const int ns = sl ? s[0] : 0;
            if (ns < 1 || ns > 4 || sl < 1 + 2 * (size_t)ns + 3) { err = "bad JPEG scan header"; return false; }
            ScanSpec sp{prog, s[1 + 2 * ns], s[2 + 2 * ns], s[3 + 2 * ns] >> 4, s[3 + 2 * ns] & 15};
            if (prog && (sp.se > 63 || sp.ss > sp.se || (sp.ss == 0 && sp.se != 0) || (sp.ss > 0 && ns != 1) ||
                         sp.al > 13 || (sp.ah != 0 && sp.ah != sp.al + 1))) {
                err = "bad progressive JPEG scan";
                return false;
            }
            const bool need_dc = !prog || (sp.ss == 0 && sp.ah == 0), need_ac = !prog || sp.ss > 0;
            std::vector<int> sc;
            for (int i = 0; i < ns; i++) {
                const int cid = s[1 + 2 * i];
                int ci = -1;
                for (int k = 0; k < (int)comps.size(); k++)
                    if (comps[k].id == cid) ci = k;
                if (ci < 0) { err = "bad JPEG scan component"; return false; }
                comps[ci].td = s[2 + 2 * i] >> 4;
                comps[ci].ta = s[2 + 2 * i] & 15;
                if (comps[ci].td > 3 || comps[ci].ta > 3 || (need_dc && !dc_t[comps[ci].td].defined) ||
                    (need_ac && !ac_t[comps[ci].ta].defined)) {
                    err = "JPEG Huffman table missing";
                    return false;
                }
                sc.push_back(ci);
            }
            Bits br{d, n, p + len};
            decode_scan(br, comps, sc, dc_t, ac_t, mcux, mcuy, restart_interval, sp);
            any_scan = true;
            // continue after the entropy-coded data: the next marker that is not RSTn
            size_t q = br.pos;
            while (q + 1 < n && !(d[q] == 0xFF && d[q + 1] != 0x00 && !(d[q + 1] >= 0xD0 && d[q + 1] <= 0xD7) &&
                                  d[q + 1] != 0xFF))
                q++;
            p = q;
            continue;
        }
        p += len;
    }
    if (!frame || !any_scan) { err = "JPEG has no image data"; return false; }
    for (auto& c : comps)
        if (!qt_def[c.tq]) { err = "JPEG quantisation table missing"; return false; }

    // IDCT of every block into the component planes (jddctmgr.c: ifast table = q * aan >> 12, rounded)
    std::vector<std::vector<uint8_t>> planes(comps.size());
    for (size_t ci = 0; ci < comps.size(); ci++) {
        Comp& c = comps[ci];
        int q[64];
        for (int i = 0; i < 64; i++) q[i] = (qt[c.tq][i] * kAanScales[i] + (1 << 11)) >> 12;
        const int stride = c.bw * 8;
        planes[ci].assign((size_t)stride * c.bh * 8, 0);
        for (int by = 0; by < c.bh; by++)
            for (int bx = 0; bx < c.bw; bx++) {
                const int16_t* blk = &c.coef[((size_t)by * c.bw + bx) * 64];
                uint8_t* o = &planes[ci][(size_t)by * 8 * stride + bx * 8];
                if (variant == PT_JPEG_IJG6) idct_ifast<false>(blk, q, o, stride);
                else idct_ifast<true>(blk, q, o, stride);
            }
    }

    // colour space (jdapimin.c default_decompress_parms)
    bool rgb_space = false;
    if (comps.size() == 3) {
        if (jfif) rgb_space = false;
        else if (adobe) rgb_space = adobe_transform == 0;
        else rgb_space = comps[0].id == 'R' && comps[1].id == 'G' && comps[2].id == 'B';
    }
    // jdcolor.c build_ycc_rgb_table (SCALEBITS 16)
    const bool v9 = variant != PT_JPEG_IJG6;
    auto FIX = [](double x) { return (int32_t)(x * 65536.0 + 0.5); };
    const int32_t k_cr_r = FIX(1.40200), k_cb_b = FIX(1.77200);
    const int32_t k_cr_g = v9 ? FIX(0.714136286) : FIX(0.71414), k_cb_g = v9 ? FIX(0.344136286) : FIX(0.34414);
    int cr_r[256], cb_b[256];
    int32_t cr_g[256], cb_g[256];
    for (int i = 0; i < 256; i++) {
        const int32_t x = i - 128;
        cr_r[i] = (int)((k_cr_r * x + (1 << 15)) >> 16);
        cb_b[i] = (int)((k_cb_b * x + (1 << 15)) >> 16);
        cr_g[i] = -k_cr_g * x;
        cb_g[i] = -k_cb_g * x + (1 << 15);
    }
    auto clamp8 = [](int v) { return (unsigned char)(v < 0 ? 0 : (v > 255 ? 255 : v)); };
    rgba.assign((size_t)W * H * 4, 255);
    for (int y = 0; y < H; y++) {
        for (int x = 0; x < W; x++) {
            int s[3];
            for (size_t ci = 0; ci < comps.size(); ci++) {
                const Comp& c = comps[ci];
                const int sx = x / (hmax / c.h), sy = y / (vmax / c.v);
                s[ci] = planes[ci][(size_t)sy * c.bw * 8 + sx];
            }
            unsigned char* o = &rgba[((size_t)y * W + x) * 4];
            if (comps.size() == 1) {
                o[0] = o[1] = o[2] = (unsigned char)s[0];
            } else if (rgb_space) {
                o[0] = (unsigned char)s[0]; o[1] = (unsigned char)s[1]; o[2] = (unsigned char)s[2];
            } else {
                const int Y = s[0], cb = s[1], cr = s[2];
                o[0] = clamp8(Y + cr_r[cr]);
                o[1] = clamp8(Y + (int)((cb_g[cb] + cr_g[cr]) >> 16));
                o[2] = clamp8(Y + cb_b[cb]);
            }
        }
    }
    *out_w = W;
    *out_h = H;
    return true;
}

}  // namespace pt

extern "C" int pt_jpeg_decode(const unsigned char* data, size_t size, int variant, int* width, int* height,
                              unsigned char** rgba) {
    if (!data || !width || !height || !rgba || (variant != PT_JPEG_IJG9 && variant != PT_JPEG_IJG6)) return -1;
    *rgba = nullptr;
    std::vector<unsigned char> px;
    std::string err;
    if (!pt::decode_jpeg(data, size, variant, width, height, px, err)) {
        std::fprintf(stderr, "[Error]%s.\n", err.c_str());
        return -3;
    }
    *rgba = (unsigned char*)std::malloc(px.size());
    if (!*rgba) return -4;
    std::memcpy(*rgba, px.data(), px.size());
    return 0;
}
