// pt_image.cpp — image decoding for scene ingestion and PNG output (include/pt_loader.h).
//
// The reference decodes textures and cube-map faces with FreeImage 3.17 (Others/image_loader.cpp:31-95):
// FreeImage_Load, FreeImage_ConvertTo24Bits, then a copy to RGBA8 with alpha forced to 255 and the
// top row first. FreeImage itself is a binary-only dependency that is not in the checkout, so the
// formats the reference's assets use are decoded here directly, producing the pixel values
// FreeImage's 24-bit conversion defines:
//   BMP  1/4/8-bit palette, 16-bit 555/565 (bit fields), 24-bit, 32-bit; uncompressed or bit fields
//   TGA  types 1/2/3 and their RLE forms 9/10/11; 8/15/16/24/32 bpp; either origin
//   PNG  every colour type and bit depth, Adam7 interlacing (zlib inflate)
// 16-bit channels keep their high byte and 5/6-bit channels expand as c * 255 / 31 (or 63), as
// FreeImage's ConvertTo24Bits does. JPEG: pt_jpeg.cpp (libjpeg 9a's fast IDCT, FreeImage's default).
// The PNG writer stores the 8-bit framebuffer (the reference's screenshot, Main/window.cpp:712-740).
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/pt_loader.h"
#include "pt_jpeg.h"

namespace {

bool read_file(const char* path, std::vector<unsigned char>& out) {
    FILE* f = std::fopen(path, "rb");
    if (!f) return false;
    std::fseek(f, 0, SEEK_END);
    long n = std::ftell(f);
    std::fseek(f, 0, SEEK_SET);
    if (n < 0) { std::fclose(f); return false; }
    out.resize((size_t)n);
    size_t got = n > 0 ? std::fread(out.data(), 1, (size_t)n, f) : 0;
    std::fclose(f);
    return got == (size_t)n;
}

inline unsigned rd16le(const unsigned char* p) { return p[0] | (p[1] << 8); }
inline unsigned rd32le(const unsigned char* p) { return p[0] | (p[1] << 8) | (p[2] << 16) | ((unsigned)p[3] << 24); }
inline unsigned rd32be(const unsigned char* p) { return ((unsigned)p[0] << 24) | (p[1] << 16) | (p[2] << 8) | p[3]; }

// 5- and 6-bit channel expansion of FreeImage's 16 -> 24 bit conversion
inline unsigned char x5(unsigned v) { return (unsigned char)((v * 0xFF) / 0x1F); }
inline unsigned char x6(unsigned v) { return (unsigned char)((v * 0xFF) / 0x3F); }

struct Image {
    int w = 0, h = 0;
    std::vector<unsigned char> rgba;  // top row first
    void alloc(int W, int H) { w = W; h = H; rgba.assign((size_t)W * H * 4, 255); }
    unsigned char* px(int x, int y) { return rgba.data() + ((size_t)y * w + x) * 4; }
    void set(int x, int y, unsigned char r, unsigned char g, unsigned char b) {
        unsigned char* p = px(x, y);
        p[0] = r; p[1] = g; p[2] = b; p[3] = 255;
    }
};

// ---- BMP ----------------------------------------------------------------------------------------
int mask_shift(unsigned m) { int s = 0; if (!m) return 0; while (!(m & 1u)) { m >>= 1; s++; } return s; }
int mask_bits(unsigned m) { int b = 0; m >>= mask_shift(m); while (m & 1u) { m >>= 1; b++; } return b; }
unsigned char mask_channel(unsigned v, unsigned m) {
    if (!m) return 0;
    unsigned c = (v & m) >> mask_shift(m);
    int bits = mask_bits(m);
    if (bits == 8) return (unsigned char)c;
    if (bits == 5) return x5(c);
    if (bits == 6) return x6(c);
    if (bits > 8) return (unsigned char)(c >> (bits - 8));
    return (unsigned char)((c * 0xFF) / ((1u << bits) - 1u));
}

bool decode_bmp(const std::vector<unsigned char>& d, Image& im, std::string& err) {
    if (d.size() < 26 || d[0] != 'B' || d[1] != 'M') { err = "not a BMP file"; return false; }
    const unsigned off = rd32le(&d[10]);
    const unsigned hsize = rd32le(&d[14]);
    int w, h, bpp;
    unsigned comp = 0, ncolors = 0;
    size_t pal_off = 14 + hsize;
    int pal_entry = 4;
    if (hsize == 12) {  // BITMAPCOREHEADER
        w = (int)rd16le(&d[18]); h = (int)(short)rd16le(&d[20]); bpp = (int)rd16le(&d[24]);
        pal_entry = 3;
    } else {
        if (d.size() < 54) { err = "truncated BMP header"; return false; }
        w = (int)rd32le(&d[18]); h = (int)rd32le(&d[22]); bpp = (int)rd16le(&d[28]);
        comp = rd32le(&d[30]);
        ncolors = rd32le(&d[46]);
    }
    const bool top_down = h < 0;
    if (top_down) h = -h;
    if (w <= 0 || h <= 0) { err = "bad BMP size"; return false; }
    unsigned rm = 0, gm = 0, bm = 0;
    if (bpp == 16) { rm = 0x7C00; gm = 0x03E0; bm = 0x001F; }
    if (bpp == 32) { rm = 0x00FF0000; gm = 0x0000FF00; bm = 0x000000FF; }
    if (comp == 3) {  // BI_BITFIELDS: masks follow a 40-byte header, or live inside a V4/V5 header
        if (d.size() < 54 + 12) { err = "truncated BMP masks"; return false; }
        rm = rd32le(&d[54]); gm = rd32le(&d[58]); bm = rd32le(&d[62]);
        if (hsize == 40) pal_off += 12;
    } else if (comp != 0) {
        err = "compressed BMP (RLE) is not supported";
        return false;
    }
    std::vector<unsigned char> pal;
    if (bpp <= 8) {
        unsigned n = ncolors ? ncolors : (1u << bpp);
        if (pal_off + (size_t)n * pal_entry > d.size()) { err = "truncated BMP palette"; return false; }
        pal.resize((size_t)n * 3);
        for (unsigned i = 0; i < n; i++) {
            pal[i * 3 + 0] = d[pal_off + i * pal_entry + 2];
            pal[i * 3 + 1] = d[pal_off + i * pal_entry + 1];
            pal[i * 3 + 2] = d[pal_off + i * pal_entry + 0];
        }
    } else if (bpp != 16 && bpp != 24 && bpp != 32) {
        err = "unsupported BMP bit depth";
        return false;
    }
    const size_t stride = (((size_t)w * bpp + 31) / 32) * 4;
    if ((size_t)off + stride * h > d.size()) { err = "BMP file too small for its pixels"; return false; }
    im.alloc(w, h);
    for (int row = 0; row < h; row++) {
        const unsigned char* s = &d[off + stride * row];
        const int y = top_down ? row : h - 1 - row;
        for (int x = 0; x < w; x++) {
            if (bpp <= 8) {
                unsigned bit = (unsigned)x * bpp;
                unsigned idx = (s[bit >> 3] >> (8 - bpp - (bit & 7))) & ((1u << bpp) - 1u);
                if ((size_t)idx * 3 + 2 >= pal.size()) idx = 0;
                im.set(x, y, pal[idx * 3], pal[idx * 3 + 1], pal[idx * 3 + 2]);
            } else if (bpp == 24) {
                im.set(x, y, s[x * 3 + 2], s[x * 3 + 1], s[x * 3]);
            } else if (bpp == 16) {
                unsigned v = rd16le(s + x * 2);
                im.set(x, y, mask_channel(v, rm), mask_channel(v, gm), mask_channel(v, bm));
            } else {
                unsigned v = rd32le(s + x * 4);
                im.set(x, y, mask_channel(v, rm), mask_channel(v, gm), mask_channel(v, bm));
            }
        }
    }
    return true;
}

// ---- TGA ----------------------------------------------------------------------------------------
bool decode_tga(const std::vector<unsigned char>& d, Image& im, std::string& err) {
    if (d.size() < 18) { err = "truncated TGA header"; return false; }
    const int idlen = d[0], cmtype = d[1], type = d[2];
    const int cm_first = (int)rd16le(&d[3]), cm_len = (int)rd16le(&d[5]), cm_bits = d[7];
    const int w = (int)rd16le(&d[12]), h = (int)rd16le(&d[14]), bpp = d[16], desc = d[17];
    const bool rle = type >= 9;
    const int base = rle ? type - 8 : type;
    if (base < 1 || base > 3 || w <= 0 || h <= 0) { err = "unsupported TGA type"; return false; }
    size_t p = 18 + (size_t)idlen;
    std::vector<unsigned char> pal;
    if (cmtype == 1) {
        const int eb = (cm_bits + 7) / 8;
        if (p + (size_t)cm_len * eb > d.size()) { err = "truncated TGA palette"; return false; }
        pal.resize((size_t)(cm_first + cm_len) * 3, 0);
        for (int i = 0; i < cm_len; i++) {
            const unsigned char* e = &d[p + (size_t)i * eb];
            unsigned char* o = &pal[(size_t)(cm_first + i) * 3];
            if (eb == 2) {
                unsigned v = rd16le(e);
                o[0] = x5((v >> 10) & 31); o[1] = x5((v >> 5) & 31); o[2] = x5(v & 31);
            } else {
                o[0] = e[2]; o[1] = e[1]; o[2] = e[0];
            }
        }
        p += (size_t)cm_len * eb;
    }
    const int pb = (bpp + 7) / 8;
    if (pb < 1 || pb > 4) { err = "unsupported TGA depth"; return false; }
    const size_t n = (size_t)w * h;
    std::vector<unsigned char> raw(n * pb);
    if (!rle) {
        if (p + raw.size() > d.size()) { err = "truncated TGA pixels"; return false; }
        std::memcpy(raw.data(), &d[p], raw.size());
    } else {
        size_t o = 0;
        while (o < raw.size()) {
            if (p >= d.size()) { err = "truncated TGA RLE stream"; return false; }
            const int hdr = d[p++];
            const size_t cnt = (size_t)(hdr & 0x7f) + 1;
            if (hdr & 0x80) {
                if (p + pb > d.size()) { err = "truncated TGA RLE packet"; return false; }
                for (size_t k = 0; k < cnt && o < raw.size(); k++, o += pb) std::memcpy(&raw[o], &d[p], pb);
                p += pb;
            } else {
                size_t bytes = cnt * pb;
                if (p + bytes > d.size()) { err = "truncated TGA raw packet"; return false; }
                if (o + bytes > raw.size()) bytes = raw.size() - o;
                std::memcpy(&raw[o], &d[p], bytes);
                o += bytes;
                p += cnt * pb;
            }
        }
    }
    const bool top = (desc & 0x20) != 0, right_to_left = (desc & 0x10) != 0;
    im.alloc(w, h);
    for (int r = 0; r < h; r++) {
        const int y = top ? r : h - 1 - r;
        for (int c = 0; c < w; c++) {
            const int x = right_to_left ? w - 1 - c : c;
            const unsigned char* s = &raw[((size_t)r * w + c) * pb];
            if (base == 1) {
                unsigned idx = pb == 2 ? rd16le(s) : s[0];
                if ((size_t)idx * 3 + 2 >= pal.size()) idx = 0;
                im.set(x, y, pal[idx * 3], pal[idx * 3 + 1], pal[idx * 3 + 2]);
            } else if (base == 3) {
                im.set(x, y, s[0], s[0], s[0]);
            } else if (pb == 2) {
                unsigned v = rd16le(s);
                im.set(x, y, x5((v >> 10) & 31), x5((v >> 5) & 31), x5(v & 31));
            } else {
                im.set(x, y, s[2], s[1], s[0]);
            }
        }
    }
    return true;
}

// ---- PNG ----------------------------------------------------------------------------------------
inline int paeth(int a, int b, int c) {
    int p = a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    if (pa <= pb && pa <= pc) return a;
    return pb <= pc ? b : c;
}

bool unfilter(unsigned char* data, size_t stride, int rows, int bpp_bytes, std::string& err) {
    std::vector<unsigned char> prev(stride, 0);
    for (int r = 0; r < rows; r++) {
        unsigned char* line = data + r * (stride + 1);
        const int f = line[0];
        unsigned char* x = line + 1;
        for (size_t i = 0; i < stride; i++) {
            const int a = i >= (size_t)bpp_bytes ? x[i - bpp_bytes] : 0;
            const int b = prev[i];
            const int c = i >= (size_t)bpp_bytes ? prev[i - bpp_bytes] : 0;
            switch (f) {
                case 0: break;
                case 1: x[i] = (unsigned char)(x[i] + a); break;
                case 2: x[i] = (unsigned char)(x[i] + b); break;
                case 3: x[i] = (unsigned char)(x[i] + ((a + b) >> 1)); break;
                case 4: x[i] = (unsigned char)(x[i] + paeth(a, b, c)); break;
                default: err = "bad PNG filter"; return false;
            }
        }
        std::memcpy(prev.data(), x, stride);
    }
    return true;
}

bool decode_png(const std::vector<unsigned char>& d, Image& im, std::string& err) {
    static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    if (d.size() < 33 || std::memcmp(d.data(), sig, 8) != 0) { err = "not a PNG file"; return false; }
    int w = 0, h = 0, depth = 0, ctype = 0, interlace = 0;
    std::vector<unsigned char> idat, pal;
    size_t p = 8;
    while (p + 8 <= d.size()) {
        const unsigned len = rd32be(&d[p]);
        const unsigned char* t = &d[p + 4];
        if (p + 12 + (size_t)len > d.size()) { err = "truncated PNG chunk"; return false; }
        const unsigned char* c = &d[p + 8];
        if (!std::memcmp(t, "IHDR", 4)) {
            w = (int)rd32be(c); h = (int)rd32be(c + 4); depth = c[8]; ctype = c[9]; interlace = c[12];
        } else if (!std::memcmp(t, "PLTE", 4)) {
            pal.assign(c, c + len);
        } else if (!std::memcmp(t, "IDAT", 4)) {
            idat.insert(idat.end(), c, c + len);
        } else if (!std::memcmp(t, "IEND", 4)) {
            break;
        }
        p += 12 + (size_t)len;
    }
    static const int chans_of[7] = {1, 0, 3, 1, 2, 0, 4};
    if (w <= 0 || h <= 0 || ctype > 6 || chans_of[ctype] == 0) { err = "bad PNG header"; return false; }
    const int chans = chans_of[ctype];
    const int bits = chans * depth;
    const int bpp_bytes = bits >= 8 ? bits / 8 : 1;
    // pass geometry (Adam7 or one pass)
    static const int ax0[7] = {0, 4, 0, 2, 0, 1, 0}, ay0[7] = {0, 0, 4, 0, 2, 0, 1};
    static const int adx[7] = {8, 8, 4, 4, 2, 2, 1}, ady[7] = {8, 8, 8, 4, 4, 2, 2};
    const int passes = interlace ? 7 : 1;
    size_t need = 0;
    int pw[7], ph[7];
    for (int k = 0; k < passes; k++) {
        pw[k] = interlace ? (w - ax0[k] + adx[k] - 1) / adx[k] : w;
        ph[k] = interlace ? (h - ay0[k] + ady[k] - 1) / ady[k] : h;
        if (pw[k] > 0 && ph[k] > 0) need += (size_t)ph[k] * ((((size_t)pw[k] * bits + 7) / 8) + 1);
    }
    std::vector<unsigned char> raw(need);
    uLongf got = (uLongf)need;
    if (uncompress(raw.data(), &got, idat.data(), (uLong)idat.size()) != Z_OK || got != need) {
        err = "PNG inflate failed";
        return false;
    }
    im.alloc(w, h);
    size_t off = 0;
    for (int k = 0; k < passes; k++) {
        if (pw[k] <= 0 || ph[k] <= 0) continue;
        const size_t stride = ((size_t)pw[k] * bits + 7) / 8;
        if (!unfilter(&raw[off], stride, ph[k], bpp_bytes, err)) return false;
        for (int r = 0; r < ph[k]; r++) {
            const unsigned char* s = &raw[off + r * (stride + 1) + 1];
            const int y = interlace ? ay0[k] + r * ady[k] : r;
            for (int cidx = 0; cidx < pw[k]; cidx++) {
                const int x = interlace ? ax0[k] + cidx * adx[k] : cidx;
                unsigned v[4] = {0, 0, 0, 255};
                for (int ch = 0; ch < chans; ch++) {
                    if (depth == 16) {
                        v[ch] = s[((size_t)cidx * chans + ch) * 2];  // high byte
                    } else if (depth == 8) {
                        v[ch] = s[(size_t)cidx * chans + ch];
                    } else {
                        const size_t bit = (size_t)cidx * depth;
                        v[ch] = (s[bit >> 3] >> (8 - depth - (bit & 7))) & ((1u << depth) - 1u);
                    }
                }
                unsigned char r8, g8, b8;
                if (ctype == 3) {
                    const unsigned idx = v[0];
                    if ((size_t)idx * 3 + 2 < pal.size()) { r8 = pal[idx * 3]; g8 = pal[idx * 3 + 1]; b8 = pal[idx * 3 + 2]; }
                    else { r8 = g8 = b8 = 0; }
                } else if (ctype == 0 || ctype == 4) {
                    unsigned g = v[0];
                    if (depth < 8) g = g * 255 / ((1u << depth) - 1u);
                    r8 = g8 = b8 = (unsigned char)g;
                } else {
                    r8 = (unsigned char)v[0]; g8 = (unsigned char)v[1]; b8 = (unsigned char)v[2];
                }
                im.set(x, y, r8, g8, b8);
            }
        }
        off += (size_t)ph[k] * (stride + 1);
    }
    return true;
}

std::string lower_ext(const char* path) {
    std::string s(path);
    size_t dot = s.find_last_of('.');
    std::string e = dot == std::string::npos ? "" : s.substr(dot + 1);
    for (auto& ch : e) ch = (char)std::tolower((unsigned char)ch);
    return e;
}

}  // namespace

// FreeImage_GetFileType sniffs the signature first, then falls back to the extension
// (image_loader.cpp:35-40); the same order here.
extern "C" int pt_image_load(const char* path, int* width, int* height, unsigned char** rgba) {
    if (!path || !width || !height || !rgba) return -1;
    *rgba = nullptr;
    std::vector<unsigned char> d;
    if (!read_file(path, d)) {
        std::fprintf(stderr, "[Error]Failed to load image file %s.\n", path);
        return -2;
    }
    Image im;
    std::string err;
    bool ok;
    static const unsigned char png_sig[4] = {137, 80, 78, 71};
    if (d.size() >= 4 && !std::memcmp(d.data(), png_sig, 4)) ok = decode_png(d, im, err);
    else if (d.size() >= 2 && d[0] == 'B' && d[1] == 'M') ok = decode_bmp(d, im, err);
    else if (d.size() >= 3 && d[0] == 0xFF && d[1] == 0xD8 && d[2] == 0xFF) {
        ok = pt::decode_jpeg(d.data(), d.size(), PT_JPEG_IJG9, &im.w, &im.h, im.rgba, err);
    }
    else if (lower_ext(path) == "tga") ok = decode_tga(d, im, err);
    else { ok = false; err = "Unsupported image file format"; }
    if (!ok) {
        std::fprintf(stderr, "[Error]%s: %s.\n", path, err.c_str());
        return -3;
    }
    *width = im.w;
    *height = im.h;
    *rgba = (unsigned char*)std::malloc(im.rgba.size());
    if (!*rgba) return -4;
    std::memcpy(*rgba, im.rgba.data(), im.rgba.size());
    return 0;
}

extern "C" void pt_image_free(unsigned char* rgba) { std::free(rgba); }

// 8-bit RGB (channels 3) or RGBA (4), top row first.
extern "C" int pt_image_write_png(const char* path, int width, int height, const unsigned char* pixels, int channels) {
    if (!path || width <= 0 || height <= 0 || !pixels || (channels != 3 && channels != 4)) return -1;
    const size_t stride = (size_t)width * channels;
    std::vector<unsigned char> raw((stride + 1) * height);
    for (int y = 0; y < height; y++) {
        raw[y * (stride + 1)] = 0;
        std::memcpy(&raw[y * (stride + 1) + 1], pixels + stride * y, stride);
    }
    uLongf clen = compressBound((uLong)raw.size());
    std::vector<unsigned char> z(clen);
    if (compress2(z.data(), &clen, raw.data(), (uLong)raw.size(), 6) != Z_OK) return -2;
    FILE* f = std::fopen(path, "wb");
    if (!f) return -3;
    auto be32 = [](unsigned v, unsigned char* o) { o[0] = v >> 24; o[1] = (v >> 16) & 255; o[2] = (v >> 8) & 255; o[3] = v & 255; };
    auto chunk = [&](const char* type, const unsigned char* data, unsigned len) {
        unsigned char hdr[8];
        be32(len, hdr);
        std::memcpy(hdr + 4, type, 4);
        std::fwrite(hdr, 1, 8, f);
        if (len) std::fwrite(data, 1, len, f);
        uLong crc = crc32(0L, (const Bytef*)type, 4);
        if (len) crc = crc32(crc, data, len);
        unsigned char c[4];
        be32((unsigned)crc, c);
        std::fwrite(c, 1, 4, f);
    };
    static const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    std::fwrite(sig, 1, 8, f);
    unsigned char ihdr[13];
    be32((unsigned)width, ihdr);
    be32((unsigned)height, ihdr + 4);
    ihdr[8] = 8; ihdr[9] = channels == 4 ? 6 : 2; ihdr[10] = 0; ihdr[11] = 0; ihdr[12] = 0;
    chunk("IHDR", ihdr, 13);
    chunk("IDAT", z.data(), (unsigned)clen);
    chunk("IEND", nullptr, 0);
    const bool ok = std::ferror(f) == 0;
    std::fclose(f);
    return ok ? 0 : -4;
}
