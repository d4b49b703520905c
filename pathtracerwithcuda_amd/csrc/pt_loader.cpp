// pt_loader.cpp — the reference's JSON configuration / scene loaders and its OBJ loader, restated
// as host C++ behind include/pt_loader.h.
//
//   JSON      nlohmann/json 3.0.1 as the loaders use it: objects, arrays, strings; a missing key reads
//             as null (operator[] on a non-const object), a duplicate key keeps the last value.
//   config    Core/config_parser.cpp:8-124 (every value a string; parse_int / parse_float /
//             parse_bool("true") / parse_float3 via istringstream), :159-187 (copy to configuration)
//   scene     Core/scene_parser.cpp:37-442 (Background / Texture / Material / Sphere / Mesh, checked in
//             that order), :465-528 (device data: meshes, then one BVH per mesh)
//   presets   Core/material.cpp:12-577
//   OBJ       tinyobjloader 1.1.0 as vendored (lib/tiny_obj_loader/tiny_obj_loader.h): its number parser
//             (tryParseDouble :498-611), index fix-up (:432-453), face triples (:747-798), shape
//             splitting on g/o (:1849-1905), ear-clipping triangulation (:1004-1152); then
//             triangle_mesh::load_obj (Core/triangle_mesh.cpp:8-213)
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <sstream>
#include <string>
#include <vector>

#include "../../include/pt_loader.h"

namespace {

// ---- JSON ---------------------------------------------------------------------------------------
struct JVal {
    enum Type { Null, Bool, Num, Str, Arr, Obj } t = Null;
    bool b = false;
    double n = 0.0;
    std::string s;
    std::vector<JVal> a;
    std::vector<std::pair<std::string, JVal>> o;

    const JVal& operator[](const char* key) const {
        static const JVal null_value;
        if (t != Obj) return null_value;
        for (auto it = o.rbegin(); it != o.rend(); ++it)
            if (it->first == key) return it->second;
        return null_value;
    }
    bool is_null() const { return t == Null; }
};

struct JParser {
    const char* p;
    const char* e;
    std::string err;

    void ws() { while (p < e && (*p == ' ' || *p == '\t' || *p == '\n' || *p == '\r')) p++; }
    bool fail(const char* m) { if (err.empty()) err = m; return false; }

    bool str(std::string& out) {
        if (p >= e || *p != '"') return fail("expected string");
        p++;
        while (p < e && *p != '"') {
            char c = *p++;
            if (c != '\\') { out.push_back(c); continue; }
            if (p >= e) return fail("bad escape");
            c = *p++;
            switch (c) {
                case '"': out.push_back('"'); break;
                case '\\': out.push_back('\\'); break;
                case '/': out.push_back('/'); break;
                case 'b': out.push_back('\b'); break;
                case 'f': out.push_back('\f'); break;
                case 'n': out.push_back('\n'); break;
                case 'r': out.push_back('\r'); break;
                case 't': out.push_back('\t'); break;
                case 'u': {
                    if (e - p < 4) return fail("bad \\u escape");
                    unsigned cp = (unsigned)std::strtoul(std::string(p, p + 4).c_str(), nullptr, 16);
                    p += 4;
                    if (cp >= 0xD800 && cp < 0xDC00 && e - p >= 6 && p[0] == '\\' && p[1] == 'u') {
                        unsigned lo = (unsigned)std::strtoul(std::string(p + 2, p + 6).c_str(), nullptr, 16);
                        if (lo >= 0xDC00 && lo < 0xE000) { cp = 0x10000 + ((cp - 0xD800) << 10) + (lo - 0xDC00); p += 6; }
                    }
                    if (cp < 0x80) out.push_back((char)cp);
                    else if (cp < 0x800) { out.push_back((char)(0xC0 | (cp >> 6))); out.push_back((char)(0x80 | (cp & 63))); }
                    else if (cp < 0x10000) {
                        out.push_back((char)(0xE0 | (cp >> 12))); out.push_back((char)(0x80 | ((cp >> 6) & 63)));
                        out.push_back((char)(0x80 | (cp & 63)));
                    } else {
                        out.push_back((char)(0xF0 | (cp >> 18))); out.push_back((char)(0x80 | ((cp >> 12) & 63)));
                        out.push_back((char)(0x80 | ((cp >> 6) & 63))); out.push_back((char)(0x80 | (cp & 63)));
                    }
                    break;
                }
                default: return fail("bad escape");
            }
        }
        if (p >= e) return fail("unterminated string");
        p++;
        return true;
    }

    bool value(JVal& v, int depth) {
        if (depth > 512) return fail("nesting too deep");
        ws();
        if (p >= e) return fail("unexpected end of input");
        const char c = *p;
        if (c == '{') {
            v.t = JVal::Obj;
            p++;
            ws();
            if (p < e && *p == '}') { p++; return true; }
            while (true) {
                ws();
                std::string k;
                if (!str(k)) return false;
                ws();
                if (p >= e || *p != ':') return fail("expected ':'");
                p++;
                JVal child;
                if (!value(child, depth + 1)) return false;
                v.o.emplace_back(std::move(k), std::move(child));
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == '}') { p++; return true; }
                return fail("expected ',' or '}'");
            }
        }
        if (c == '[') {
            v.t = JVal::Arr;
            p++;
            ws();
            if (p < e && *p == ']') { p++; return true; }
            while (true) {
                JVal child;
                if (!value(child, depth + 1)) return false;
                v.a.push_back(std::move(child));
                ws();
                if (p < e && *p == ',') { p++; continue; }
                if (p < e && *p == ']') { p++; return true; }
                return fail("expected ',' or ']'");
            }
        }
        if (c == '"') { v.t = JVal::Str; return str(v.s); }
        if (e - p >= 4 && !std::strncmp(p, "true", 4)) { v.t = JVal::Bool; v.b = true; p += 4; return true; }
        if (e - p >= 5 && !std::strncmp(p, "false", 5)) { v.t = JVal::Bool; v.b = false; p += 5; return true; }
        if (e - p >= 4 && !std::strncmp(p, "null", 4)) { v.t = JVal::Null; p += 4; return true; }
        if (c == '-' || (c >= '0' && c <= '9')) {
            char* end = nullptr;
            std::string tmp(p, (size_t)std::min<ptrdiff_t>(e - p, 64));
            v.t = JVal::Num;
            v.n = std::strtod(tmp.c_str(), &end);
            if (end == tmp.c_str()) return fail("bad number");
            p += end - tmp.c_str();
            return true;
        }
        return fail("unexpected character");
    }
};

bool parse_json_file(const std::string& path, JVal& root, std::string& err) {
    std::ifstream f(path, std::ios::in | std::ios::binary);
    if (!f) { err = "cannot open " + path; return false; }
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string text = ss.str();
    JParser jp{text.data(), text.data() + text.size(), {}};
    // a UTF-8 byte-order mark is skipped, as nlohmann's input adapter does
    if (text.size() >= 3 && (unsigned char)text[0] == 0xEF && (unsigned char)text[1] == 0xBB && (unsigned char)text[2] == 0xBF)
        jp.p += 3;
    if (!jp.value(root, 0)) { err = "parse error: " + jp.err; return false; }
    jp.ws();
    if (jp.p != jp.e) { err = "parse error: trailing characters"; return false; }
    return true;
}

// ---- value parsing exactly as the loaders do it (istringstream >>, "true") -----------------------
float parse_float(const std::string& s) {
    std::istringstream st(s);
    float v = 0.0f;
    st >> v;
    return v;
}
int parse_int(const std::string& s) {
    std::istringstream st(s);
    int v = 0;
    st >> v;
    return v;
}
bool parse_bool(const std::string& s) { return s == "true"; }
pt_float3 parse_float3(const std::string& s) {
    std::istringstream st(s);
    float x = 0.0f, y = 0.0f, z = 0.0f;
    st >> x >> y >> z;
    return {x, y, z};
}
float clampf_(float v, float lo, float hi) { return v < lo ? lo : (v > hi ? hi : v); }

// std::string conversion of a json value: anything but a string is a type error in nlohmann
bool as_string(const JVal& v, std::string& out) {
    if (v.t != JVal::Str) return false;
    out = v.s;
    return true;
}

// ---- materials (Core/material.cpp:12-577) ------------------------------------------------------
struct Preset {
    const char* name;
    float d[3], e[3], s[3];
    bool transparent;
    float roughness, n, k, ab[3], rs[3];
};
const Preset kPresets[] = {
    {"titanium", {0, 0, 0}, {0, 0, 0}, {0.542f, 0.497f, 0.499f}, false, 0.3f, 2.2670f, 3.0385f, {0, 0, 0}, {0, 0, 0}},
    {"chromium", {0, 0, 0}, {0, 0, 0}, {0.549f, 0.556f, 0.554f}, false, 0.3f, 2.3230f, 3.1350f, {0, 0, 0}, {0, 0, 0}},
    {"iron", {0, 0, 0}, {0, 0, 0}, {0.562f, 0.556f, 0.578f}, false, 0.3f, 2.5845f, 2.7670f, {0, 0, 0}, {0, 0, 0}},
    {"nickel", {0, 0, 0}, {0, 0, 0}, {0.662f, 0.609f, 0.526f}, false, 0.3f, 1.7290f, 2.9435f, {0, 0, 0}, {0, 0, 0}},
    {"platinum", {0, 0, 0}, {0, 0, 0}, {0.673f, 0.637f, 0.585f}, false, 0.3f, 1.3400f, 1.0300f, {0, 0, 0}, {0, 0, 0}},
    {"copper", {0, 0, 0}, {0, 0, 0}, {0.955f, 0.638f, 0.538f}, false, 0.3f, 1.2404f, 2.3929f, {0, 0, 0}, {0, 0, 0}},
    {"palladium", {0, 0, 0}, {0, 0, 0}, {0.733f, 0.697f, 0.652f}, false, 0.3f, 1.4080f, 3.2540f, {0, 0, 0}, {0, 0, 0}},
    {"zinc", {0, 0, 0}, {0, 0, 0}, {0.664f, 0.824f, 0.850f}, false, 0.3f, 0.67767f, 4.01220f, {0, 0, 0}, {0, 0, 0}},
    {"gold", {0, 0, 0}, {0, 0, 0}, {1.022f, 0.782f, 0.344f}, false, 0.3f, 0.89863f, 2.4584f, {0, 0, 0}, {0, 0, 0}},
    {"aluminum", {0, 0, 0}, {0, 0, 0}, {0.913f, 0.922f, 0.924f}, false, 0.3f, 0.63324f, 5.4544f, {0, 0, 0}, {0, 0, 0}},
    {"silver", {0, 0, 0}, {0, 0, 0}, {0.972f, 0.960f, 0.915f}, false, 0.3f, 0.04f, 2.6484f, {0, 0, 0}, {0, 0, 0}},
    {"glass", {1, 1, 1}, {0, 0, 0}, {0.045f, 0.045f, 0.045f}, true, 0.1f, 1.5319f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"green_glass", {1, 1, 1}, {0, 0, 0}, {0.045f, 0.045f, 0.045f}, true, 0.1f, 1.5319f, 0.0f, {0.8f, 0.01f, 0.8f}, {0, 0, 0}},
    {"diamond", {1, 1, 1}, {0, 0, 0}, {1, 1, 1}, true, 0.01f, 2.4392f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"red", {0.87f, 0.15f, 0.15f}, {0, 0, 0}, {1, 1, 1}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"green", {0.15f, 0.87f, 0.15f}, {0, 0, 0}, {1, 1, 1}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"orange", {0.93f, 0.33f, 0.04f}, {0, 0, 0}, {1, 1, 1}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"purple", {0.5f, 0.1f, 0.9f}, {0, 0, 0}, {1, 1, 1}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"wall_blue", {0.4f, 0.6f, 0.8f}, {0, 0, 0}, {0, 0, 0}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"wall_red", {0.87f, 0.15f, 0.15f}, {0, 0, 0}, {0, 0, 0}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"wall_green", {0.15f, 0.87f, 0.15f}, {0, 0, 0}, {0, 0, 0}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"wall_white", {1, 1, 1}, {0, 0, 0}, {0, 0, 0}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"blue", {0.4f, 0.6f, 0.8f}, {0, 0, 0}, {1, 1, 1}, false, 0.01f, 1.491f, 0.0f, {0, 0, 0}, {0, 0, 0}},
    {"marble", {0, 0, 0}, {0, 0, 0}, {1, 1, 1}, true, 0.01f, 1.486f, 0.0f, {0.6f, 0.6f, 0.6f}, {8, 8, 8}},
    {"something_blue", {0, 0, 0}, {0, 0, 0}, {1, 1, 1}, true, 0.01f, 1.333f, 0.0f, {0.9f, 0.3f, 0.02f}, {2, 2, 2}},
    {"something_red", {0, 0, 0}, {0, 0, 0}, {1, 1, 1}, true, 0.01f, 1.35f, 0.0f, {0.02f, 5.1f, 5.7f}, {9, 9, 9}},
    {"light", {0, 0, 0}, {13, 13, 11}, {0, 0, 0}, false, 0.01f, 1.000293f, 0.0f, {0, 0, 0}, {0, 0, 0}},
};

pt_material to_material(const Preset& p) {
    pt_material m;
    std::memset(&m, 0, sizeof(m));
    m.diffuse_color = {p.d[0], p.d[1], p.d[2]};
    m.emission_color = {p.e[0], p.e[1], p.e[2]};
    m.specular_color = {p.s[0], p.s[1], p.s[2]};
    m.is_transparent = p.transparent ? 1 : 0;
    m.roughness = p.roughness;
    m.medium.refraction_index = p.n;
    m.medium.extinction_coefficient = p.k;
    m.medium.scattering.absorption_coefficient = {p.ab[0], p.ab[1], p.ab[2]};
    m.medium.scattering.reduced_scattering_coefficient = {p.rs[0], p.rs[1], p.rs[2]};
    m.diffuse_texture_id = -1;
    m.specular_texture_id = -1;
    return m;
}

// ---- OBJ (tinyobjloader 1.1.0 semantics) ---------------------------------------------------------
// try_parse_double, pnpoly and export_group below follow tinyobjloader 1.1.0 (the OBJ loader the
// reference vendors, lib/tiny_obj_loader/tiny_obj_loader.h:498-611, :975-1166) closely, because the
// parsed floats and the triangulation must be bit-identical to it. Its licence:
//
//   The MIT License (MIT)
//
//   Copyright (c) 2012-2017 Syoyo Fujita and many contributors.
//
//   Permission is hereby granted, free of charge, to any person obtaining a copy
//   of this software and associated documentation files (the "Software"), to deal
//   in the Software without restriction, including without limitation the rights
//   to use, copy, modify, merge, publish, distribute, sublicense, and/or sell
//   copies of the Software, and to permit persons to whom the Software is
//   furnished to do so, subject to the following conditions:
//
//   The above copyright notice and this permission notice shall be included in
//   all copies or substantial portions of the Software.
//
//   THE SOFTWARE IS PROVIDED "AS IS", WITHOUT WARRANTY OF ANY KIND, EXPRESS OR
//   IMPLIED, INCLUDING BUT NOT LIMITED TO THE WARRANTIES OF MERCHANTABILITY,
//   FITNESS FOR A PARTICULAR PURPOSE AND NONINFRINGEMENT. IN NO EVENT SHALL THE
//   AUTHORS OR COPYRIGHT HOLDERS BE LIABLE FOR ANY CLAIM, DAMAGES OR OTHER
//   LIABILITY, WHETHER IN AN ACTION OF CONTRACT, TORT OR OTHERWISE, ARISING FROM,
//   OUT OF OR IN CONNECTION WITH THE SOFTWARE OR THE USE OR OTHER DEALINGS IN
//   THE SOFTWARE.
inline bool is_space(char c) { return c == ' ' || c == '\t'; }
inline bool is_digit(char c) { return (unsigned)(c - '0') < 10u; }
inline bool is_new_line(char c) { return c == '\r' || c == '\n' || c == '\0'; }

// tryParseDouble (tiny_obj_loader.h:498-611): mantissa accumulated in double, fraction digits
// scaled by a table of negative powers of ten, exponent applied as ldexp(m * 5^e, e).
bool try_parse_double(const char* s, const char* s_end, double* result) {
    if (s >= s_end) return false;
    double mantissa = 0.0;
    int exponent = 0;
    char sign = '+', exp_sign = '+';
    const char* curr = s;
    int read = 0;
    bool end_not_reached = false;
    if (*curr == '+' || *curr == '-') { sign = *curr; curr++; }
    else if (!is_digit(*curr)) return false;
    end_not_reached = curr != s_end;
    while (end_not_reached && is_digit(*curr)) {
        mantissa *= 10;
        mantissa += (int)(*curr - 0x30);
        curr++; read++;
        end_not_reached = curr != s_end;
    }
    if (read == 0) return false;
    if (!end_not_reached) goto assemble;
    if (*curr == '.') {
        curr++;
        read = 1;
        end_not_reached = curr != s_end;
        while (end_not_reached && is_digit(*curr)) {
            static const double pow_lut[] = {1.0, 0.1, 0.01, 0.001, 0.0001, 0.00001, 0.000001, 0.0000001};
            mantissa += (int)(*curr - 0x30) * (read < 8 ? pow_lut[read] : std::pow(10.0, -read));
            read++; curr++;
            end_not_reached = curr != s_end;
        }
    } else if (*curr == 'e' || *curr == 'E') {
    } else {
        goto assemble;
    }
    if (!end_not_reached) goto assemble;
    if (*curr == 'e' || *curr == 'E') {
        curr++;
        end_not_reached = curr != s_end;
        if (end_not_reached && (*curr == '+' || *curr == '-')) { exp_sign = *curr; curr++; }
        else if (!is_digit(*curr)) return false;
        read = 0;
        end_not_reached = curr != s_end;
        while (end_not_reached && is_digit(*curr)) {
            exponent *= 10;
            exponent += (int)(*curr - 0x30);
            curr++; read++;
            end_not_reached = curr != s_end;
        }
        exponent *= (exp_sign == '+' ? 1 : -1);
        if (read == 0) return false;
    }
assemble:
    *result = (sign == '+' ? 1 : -1) * (exponent ? std::ldexp(mantissa * std::pow(5.0, exponent), exponent) : mantissa);
    return true;
}

float parse_real(const char** token, double dflt) {
    *token += std::strspn(*token, " \t");
    const char* end = *token + std::strcspn(*token, " \t\r");
    double val = dflt;
    try_parse_double(*token, end, &val);
    *token = end;
    return (float)val;
}

inline bool fix_index(int idx, int n, int* ret) {
    if (idx > 0) { *ret = idx - 1; return true; }
    if (idx == 0) return false;
    *ret = n + idx;
    return true;
}

struct VIdx { int v = -1, vt = -1, vn = -1; };

bool parse_triple(const char** token, int vsize, int vnsize, int vtsize, VIdx* ret) {
    VIdx vi;
    if (!fix_index(std::atoi(*token), vsize, &vi.v)) return false;
    *token += std::strcspn(*token, "/ \t\r");
    if ((*token)[0] != '/') { *ret = vi; return true; }
    (*token)++;
    if ((*token)[0] == '/') {  // i//k
        (*token)++;
        if (!fix_index(std::atoi(*token), vnsize, &vi.vn)) return false;
        *token += std::strcspn(*token, "/ \t\r");
        *ret = vi;
        return true;
    }
    if (!fix_index(std::atoi(*token), vtsize, &vi.vt)) return false;  // i/j/k or i/j
    *token += std::strcspn(*token, "/ \t\r");
    if ((*token)[0] != '/') { *ret = vi; return true; }
    (*token)++;
    if (!fix_index(std::atoi(*token), vnsize, &vi.vn)) return false;
    *token += std::strcspn(*token, "/ \t\r");
    *ret = vi;
    return true;
}

// pnpoly (tiny_obj_loader.h:975-984)
int pnpoly(int nvert, const float* vx, const float* vy, float tx, float ty) {
    int c = 0;
    for (int i = 0, j = nvert - 1; i < nvert; j = i++) {
        if (((vy[i] > ty) != (vy[j] > ty)) && (tx < (vx[j] - vx[i]) * (ty - vy[i]) / (vy[j] - vy[i]) + vx[i])) c = !c;
    }
    return c;
}

struct ObjShape { std::vector<VIdx> idx; };  // 3 per triangle

// exportFaceGroupToShape with triangulate = true (tiny_obj_loader.h:986-1166). A face naming a vertex
// that does not exist (yet) sets *bad: tinyobjloader reads past its vertex array there (undefined
// behaviour, found by the sanitizer build, tests/test_sanitizers.py); this loader rejects the file.
bool export_group(ObjShape& shape, std::vector<std::vector<VIdx>>& group, const std::vector<float>& v,
                  bool* bad = nullptr) {
    if (group.empty()) return false;
    const long long nv = (long long)(v.size() / 3);
    for (const auto& face : group)
        for (const VIdx& c : face)
            if (c.v < 0 || c.v >= nv) {
                if (bad) *bad = true;
                return false;
            }
    for (const auto& face : group) {
        size_t npolys = face.size();
        if (npolys < 3) {  // the reference reads face[1] and walks (k+2)%npolys; a degenerate face emits nothing
            continue;
        }
        size_t axes[2] = {1, 2};
        for (size_t k = 0; k < npolys; ++k) {
            const VIdx i0 = face[(k + 0) % npolys], i1 = face[(k + 1) % npolys], i2 = face[(k + 2) % npolys];
            const float* p0 = &v[(size_t)i0.v * 3];
            const float* p1 = &v[(size_t)i1.v * 3];
            const float* p2 = &v[(size_t)i2.v * 3];
            float e0x = p1[0] - p0[0], e0y = p1[1] - p0[1], e0z = p1[2] - p0[2];
            float e1x = p2[0] - p1[0], e1y = p2[1] - p1[1], e1z = p2[2] - p1[2];
            float cx = std::fabs(e0y * e1z - e0z * e1y);
            float cy = std::fabs(e0z * e1x - e0x * e1z);
            float cz = std::fabs(e0x * e1y - e0y * e1x);
            const float eps = 0.0001f;
            if (cx > eps || cy > eps || cz > eps) {
                if (!(cx > cy && cx > cz)) {
                    axes[0] = 0;
                    if (cz > cx && cz > cy) axes[1] = 1;
                }
                break;
            }
        }
        float area = 0;
        for (size_t k = 0; k < npolys; ++k) {
            const VIdx i0 = face[(k + 0) % npolys], i1 = face[(k + 1) % npolys];
            float v0x = v[(size_t)i0.v * 3 + axes[0]], v0y = v[(size_t)i0.v * 3 + axes[1]];
            float v1x = v[(size_t)i1.v * 3 + axes[0]], v1y = v[(size_t)i1.v * 3 + axes[1]];
            area += (v0x * v1y - v0y * v1x) * 0.5f;
        }
        int max_rounds = 10;
        std::vector<VIdx> rem = face;
        size_t guess = 0;
        VIdx ind[3];
        float vx[3], vy[3];
        while (rem.size() > 3 && max_rounds > 0) {
            npolys = rem.size();
            if (guess >= npolys) { max_rounds -= 1; guess -= npolys; }
            for (size_t k = 0; k < 3; k++) {
                ind[k] = rem[(guess + k) % npolys];
                vx[k] = v[(size_t)ind[k].v * 3 + axes[0]];
                vy[k] = v[(size_t)ind[k].v * 3 + axes[1]];
            }
            float e0x = vx[1] - vx[0], e0y = vy[1] - vy[0];
            float e1x = vx[2] - vx[1], e1y = vy[2] - vy[1];
            float cross = e0x * e1y - e0y * e1x;
            if (cross * area < 0.0f) { guess += 1; continue; }
            bool overlap = false;
            for (size_t other = 3; other < npolys; ++other) {
                const size_t ovi = (size_t)rem[(guess + other) % npolys].v;
                if (pnpoly(3, vx, vy, v[ovi * 3 + axes[0]], v[ovi * 3 + axes[1]])) { overlap = true; break; }
            }
            if (overlap) { guess += 1; continue; }
            shape.idx.push_back(ind[0]); shape.idx.push_back(ind[1]); shape.idx.push_back(ind[2]);
            size_t removed = (guess + 1) % npolys;
            while (removed + 1 < npolys) { rem[removed] = rem[removed + 1]; removed += 1; }
            rem.pop_back();
        }
        if (rem.size() == 3) { shape.idx.push_back(rem[0]); shape.idx.push_back(rem[1]); shape.idx.push_back(rem[2]); }
    }
    return true;
}

std::string dir_of(const std::string& path) {
    size_t s = path.find_last_of("/\\");
    return s == std::string::npos ? std::string() : path.substr(0, s + 1);
}

// material names of the .mtl files named by mtllib (the MaterialFileReader's map; only the ids
// matter here: they decide whether usemtl flushes the current face group)
void read_mtl_names(const std::string& path, std::map<std::string, int>& mm, int& count, bool& ok) {
    std::ifstream f(path);
    if (!f) { ok = false; return; }
    ok = true;
    std::string line;
    while (std::getline(f, line)) {
        const char* t = line.c_str();
        t += std::strspn(t, " \t");
        if (!std::strncmp(t, "newmtl", 6) && is_space(t[6])) {
            t += 7;
            std::string name(t);
            while (!name.empty() && (name.back() == '\r' || name.back() == '\n')) name.pop_back();
            mm[name] = count++;
        }
    }
}

bool load_obj_file(const std::string& path, std::vector<float>& v, std::vector<float>& vn, std::vector<float>& vt,
                   std::vector<ObjShape>& shapes, std::string& err) {
    std::ifstream in(path, std::ios::in | std::ios::binary);
    if (!in) { err = "Cannot open file [" + path + "]"; return false; }
    std::vector<std::vector<VIdx>> group;
    std::map<std::string, int> material_map;
    int material_count = 0;
    int material = -1;
    ObjShape shape;
    std::string line;
    while (std::getline(in, line)) {
        if (!line.empty() && line.back() == '\r') line.pop_back();
        if (line.empty()) continue;
        const char* token = line.c_str();
        token += std::strspn(token, " \t");
        if (token[0] == '\0' || token[0] == '#') continue;
        if (token[0] == 'v' && is_space(token[1])) {
            token += 2;
            float x = parse_real(&token, 0.0), y = parse_real(&token, 0.0), z = parse_real(&token, 0.0);
            v.push_back(x); v.push_back(y); v.push_back(z);
            continue;
        }
        if (token[0] == 'v' && token[1] == 'n' && is_space(token[2])) {
            token += 3;
            float x = parse_real(&token, 0.0), y = parse_real(&token, 0.0), z = parse_real(&token, 0.0);
            vn.push_back(x); vn.push_back(y); vn.push_back(z);
            continue;
        }
        if (token[0] == 'v' && token[1] == 't' && is_space(token[2])) {
            token += 3;
            float x = parse_real(&token, 0.0), y = parse_real(&token, 0.0);
            vt.push_back(x); vt.push_back(y);
            continue;
        }
        if (token[0] == 'f' && is_space(token[1])) {
            token += 2;
            token += std::strspn(token, " \t");
            std::vector<VIdx> face;
            while (!is_new_line(token[0])) {
                VIdx vi;
                if (!parse_triple(&token, (int)(v.size() / 3), (int)(vn.size() / 3), (int)(vt.size() / 2), &vi)) {
                    err = "Failed parse `f' line(e.g. zero value for face index).";
                    return false;
                }
                face.push_back(vi);
                token += std::strspn(token, " \t\r");
            }
            group.push_back(std::move(face));
            continue;
        }
        if (!std::strncmp(token, "usemtl", 6) && is_space(token[6])) {
            std::string name(token + 7);
            int id = -1;
            auto it = material_map.find(name);
            if (it != material_map.end()) id = it->second;
            if (id != material) {
                bool bad = false;
                export_group(shape, group, v, &bad);
                if (bad) { err = "face index out of range"; return false; }
                group.clear();
                material = id;
            }
            continue;
        }
        if (!std::strncmp(token, "mtllib", 6) && is_space(token[6])) {
            std::istringstream names(std::string(token + 7));
            std::string fn;
            while (names >> fn) {
                bool ok = false;
                read_mtl_names(dir_of(path) + fn, material_map, material_count, ok);
                if (ok) break;
            }
            continue;
        }
        if (token[0] == 'g' && is_space(token[1])) {
            bool bad = false;
            export_group(shape, group, v, &bad);
            if (bad) { err = "face index out of range"; return false; }
            if (!shape.idx.empty()) shapes.push_back(shape);
            shape = ObjShape();
            group.clear();
            continue;
        }
        if (token[0] == 'o' && is_space(token[1])) {
            // the face group is flushed, but the shape is kept only if that flush exported faces
            // (tiny_obj_loader.h:1886-1905)
            bool bad = false;
            if (export_group(shape, group, v, &bad)) shapes.push_back(shape);
            if (bad) { err = "face index out of range"; return false; }
            group.clear();
            shape = ObjShape();
            continue;
        }
    }
    bool bad = false;
    const bool ret = export_group(shape, group, v, &bad);
    if (bad) { err = "face index out of range"; return false; }
    if (ret || !shape.idx.empty()) shapes.push_back(shape);
    return true;
}

// ---- scene loading ------------------------------------------------------------------------------
std::string fix_path(std::string p, const char* root) {
    std::replace(p.begin(), p.end(), '\\', '/');
    if (root && *root && !p.empty() && p[0] != '/') {
        std::string r(root);
        if (r.back() != '/') r.push_back('/');
        p = r + p;
    }
    return p;
}

#define LOAD_ERROR(...)                                    \
    do {                                                   \
        std::fprintf(stderr, "[Error]" __VA_ARGS__);       \
        std::fprintf(stderr, "\n");                        \
        return -10;                                        \
    } while (0)

// CHECK_PROPERTY (Others/utilities.hpp:64-69)
#define CHECK_PROPERTY(cat, val, tok)                                                  \
    if ((val).is_null()) {                                                             \
        std::fprintf(stderr, "[Error]%s property <%s> not defined!\n", cat, tok);      \
        return -11;                                                                    \
    }

struct MeshSpec {
    std::string path;
    std::vector<std::string> mats;
    pt_float3 position, scale, rotate;
};

}  // namespace

extern "C" int pt_material_preset(const char* name, pt_material* out) {
    if (!name || !out) return -1;
    for (const auto& p : kPresets) {
        if (!std::strcmp(p.name, name)) { *out = to_material(p); return 0; }
    }
    return -2;
}

extern "C" int pt_config_load(const char* path, pt_configuration* cfg) {
    if (!path || !cfg) return -1;
    // config_parser member defaults (Core/config_parser.h:71-93)
    std::memset(cfg, 0, sizeof(*cfg));
    cfg->width = 1024; cfg->height = 768; cfg->use_fullscreen = 0; cfg->block_size = 64; cfg->max_block_size = 1024;
    cfg->max_tracer_depth = 20; cfg->vector_bias_length = 0.0001f; cfg->energy_exist_threshold = 0.000001f;
    cfg->sss_threshold = 0.000001f; cfg->use_sky_box = 1; cfg->use_bilinear = 0; cfg->use_sky = 0;
    cfg->gamma_correction = 1; cfg->use_anti_alias = 1; cfg->fov = 45.0f; cfg->bvh_leaf_node_triangle_num = 1;
    cfg->bvh_bucket_max_divide_internal_num = 12; cfg->bvh_build_block_size = 32; cfg->bvh_build = PT_BVH_MORTON_CODE_CUDA;
    cfg->air_refraction_index = 1.000293f; cfg->air_absorption_coef = {0, 0, 0};
    cfg->air_reduced_scattering_coef = {0, 0, 0}; cfg->cuda_acceleration = 1;

    JVal root;
    std::string err;
    if (!parse_json_file(path, root, err)) {
        std::fprintf(stderr, "[Error]%s\n", err.c_str());
        return -2;
    }
    static const char* keys[] = {"Height", "Width", "FullScreen", "BlockSize", "MaxBlockSize", "MaxDepth", "BiasLength",
                                 "EnergyThreshold", "SSSThreshold", "Skybox", "BilinearSample", "Sky", "GammaCorrection",
                                 "AntiAlias", "FOV", "BvhLeafNodeTriangleNum", "BvhBucketMaxDivideInternalNum",
                                 "BvhBuildBlockSize", "BvhBuildMethod", "AirRefractionIndex", "AirAbsorptionCoef",
                                 "AirReducedScatteringCoef", "CUDAAcceleration"};
    std::map<std::string, std::string> v;
    for (const char* k : keys) {
        const JVal& x = root[k];
        // the reference's message for BvhBuildMethod names BvhBuildBlockSize (config_parser.cpp:67)
        CHECK_PROPERTY("Config", x, std::strcmp(k, "BvhBuildMethod") ? k : "BvhBuildBlockSize");
        std::string s;
        if (!as_string(x, s)) {
            std::fprintf(stderr, "[Error]Config property <%s> must be a string\n", k);
            return -3;
        }
        v[k] = s;
    }
    pt_configuration c = *cfg;
    c.height = parse_int(v["Height"]);
    c.width = parse_int(v["Width"]);
    c.use_fullscreen = parse_bool(v["FullScreen"]);
    c.block_size = parse_int(v["BlockSize"]);
    c.max_block_size = parse_int(v["MaxBlockSize"]);
    c.max_tracer_depth = parse_int(v["MaxDepth"]);
    c.vector_bias_length = parse_float(v["BiasLength"]);
    c.energy_exist_threshold = parse_float(v["EnergyThreshold"]);
    c.sss_threshold = parse_float(v["SSSThreshold"]);
    c.use_sky_box = parse_bool(v["Skybox"]);
    c.use_bilinear = parse_bool(v["BilinearSample"]);
    c.use_sky = parse_bool(v["Sky"]);
    c.gamma_correction = parse_bool(v["GammaCorrection"]);
    c.use_anti_alias = parse_bool(v["AntiAlias"]);
    c.fov = parse_bool(v["FOV"]) ? 1.0f : 0.0f;  // config_parser.cpp:111
    c.bvh_leaf_node_triangle_num = parse_int(v["BvhLeafNodeTriangleNum"]);
    c.bvh_bucket_max_divide_internal_num = parse_int(v["BvhBucketMaxDivideInternalNum"]);
    c.bvh_build_block_size = parse_int(v["BvhBuildBlockSize"]);
    {  // parse_bvh_build_method (Bvh/bvh_build_config.cpp:7-27): case-insensitive, default NaiveCPU
        std::string m = v["BvhBuildMethod"];
        std::transform(m.begin(), m.end(), m.begin(), [](unsigned char ch) { return (char)std::tolower(ch); });
        // "SAH" (not a reference value): PT_BVH_SAH, this build's surface-area tree; every other
        // unknown value falls back to NaiveCPU as in the reference
        c.bvh_build = m == "mortoncodecpu" ? PT_BVH_MORTON_CODE_CPU
                    : m == "mortoncodecuda" ? PT_BVH_MORTON_CODE_CUDA : m == "sah" ? PT_BVH_SAH : PT_BVH_NAIVE_CPU;
    }
    c.air_refraction_index = parse_float(v["AirRefractionIndex"]);
    c.air_absorption_coef = parse_float3(v["AirAbsorptionCoef"]);
    c.air_reduced_scattering_coef = parse_float3(v["AirReducedScatteringCoef"]);
    c.cuda_acceleration = parse_bool(v["CUDAAcceleration"]);
    *cfg = c;
    return 0;
}

extern "C" int pt_obj_load(const char* path, pt_obj_mesh* out) {
    if (!path || !out) return -1;
    std::memset(out, 0, sizeof(*out));
    std::vector<float> v, vn, vt;
    std::vector<ObjShape> shapes;
    std::string err;
    if (!load_obj_file(path, v, vn, vt, shapes, err)) {
        std::fprintf(stderr, "[TinyObj]\n%s\n[Info]Load file %s failed.\n", err.c_str(), path);
        return -2;
    }
    if (vt.empty()) std::fprintf(stderr, "[Warn]Mesh does not have texcoords!\n");
    if (vn.empty()) {
        std::fprintf(stderr, "[Error]Mesh does not have normal!\n");
        return -3;
    }
    size_t tris = 0;
    for (const auto& s : shapes) tris += s.idx.size() / 3;
    out->triangle_num = (int)tris;
    out->shape_num = (int)shapes.size();
    out->vertex_num = (int)(v.size() / 3);
    out->vertices = (float*)std::malloc(std::max<size_t>(tris, 1) * 9 * sizeof(float));
    out->normals = (float*)std::malloc(std::max<size_t>(tris, 1) * 9 * sizeof(float));
    out->uvs = vt.empty() ? nullptr : (float*)std::malloc(std::max<size_t>(tris, 1) * 6 * sizeof(float));
    out->shape_of_triangle = (int*)std::malloc(std::max<size_t>(tris, 1) * sizeof(int));
    if (!out->vertices || !out->normals || (!vt.empty() && !out->uvs) || !out->shape_of_triangle) {
        pt_obj_free(out);
        return -4;
    }
    size_t t = 0;
    for (size_t si = 0; si < shapes.size(); si++) {
        const auto& s = shapes[si];
        for (size_t k = 0; k < s.idx.size(); k += 3, t++) {
            out->shape_of_triangle[t] = (int)si;
            for (int c = 0; c < 3; c++) {
                const VIdx& x = s.idx[k + c];
                for (int a = 0; a < 3; a++) out->vertices[t * 9 + c * 3 + a] = v[(size_t)x.v * 3 + a];
                // a face without normal index reads attrib.normals[-3..-1] in the reference (undefined);
                // here it reads as the zero vector
                for (int a = 0; a < 3; a++)
                    out->normals[t * 9 + c * 3 + a] = (x.vn >= 0 && (size_t)x.vn * 3 + 2 < vn.size()) ? vn[(size_t)x.vn * 3 + a] : 0.0f;
                if (out->uvs) {
                    for (int a = 0; a < 2; a++)
                        out->uvs[t * 6 + c * 2 + a] = (x.vt >= 0 && (size_t)x.vt * 2 + 1 < vt.size()) ? vt[(size_t)x.vt * 2 + a] : 0.0f;
                }
            }
        }
    }
    return 0;
}

extern "C" void pt_obj_free(pt_obj_mesh* m) {
    if (!m) return;
    std::free(m->vertices);
    std::free(m->normals);
    std::free(m->uvs);
    std::free(m->shape_of_triangle);
    std::memset(m, 0, sizeof(*m));
}

extern "C" int pt_scene_load(pt_scene_builder* b, const char* scene_path, const pt_scene_load_options* opt) {
    if (!b || !scene_path) return -1;
    pt_scene_load_options o;
    std::memset(&o, 0, sizeof(o));
    o.leaf_size = 1;
    o.bvh_method = PT_BVH_MORTON_CODE_CUDA;
    o.bucket_num = 12;
    if (opt) o = *opt;
    const char* root = o.root_dir;

    JVal js;
    std::string err;
    if (!parse_json_file(fix_path(scene_path, nullptr), js, err)) LOAD_ERROR("%s", err.c_str());

    std::map<std::string, pt_material> materials;
    for (const auto& p : kPresets) materials[p.name] = to_material(p);

    // Background (scene_parser.cpp:79-111)
    const JVal& bg = js["Background"];
    if (bg.is_null()) LOAD_ERROR("Background not defined!");
    if (bg.t == JVal::Arr) LOAD_ERROR("Background can not be array!");
    const JVal &bname = bg["Name"], &bpath = bg["Path"], &bformat = bg["Format"];
    CHECK_PROPERTY("Background", bname, "Name");
    CHECK_PROPERTY("Background", bpath, "Path");
    CHECK_PROPERTY("Background", bformat, "Format");
    std::string name_s, path_s, format_s;
    if (!as_string(bname, name_s) || !as_string(bpath, path_s) || !as_string(bformat, format_s))
        LOAD_ERROR("Background properties must be strings");
    std::string cube_dir = o.background_override ? std::string(o.background_override) : path_s + name_s;
    if (o.background_format) format_s = o.background_format;
    static const char* faces[6] = {"xpos", "xneg", "ypos", "yneg", "zpos", "zneg"};
    std::string cube_paths[6];
    for (int f = 0; f < 6; f++) cube_paths[f] = fix_path(cube_dir + "\\" + faces[f] + "." + format_s, root);

    // Texture (:113-127)
    std::vector<std::string> texture_paths;
    const JVal& tex = js["Texture"];
    if (!tex.is_null()) {
        if (tex.t != JVal::Arr) LOAD_ERROR("Texture must be array!");
        for (const auto& t : tex.a) {
            std::string s;
            if (!as_string(t, s)) LOAD_ERROR("Texture entries must be strings");
            texture_paths.push_back(s);
        }
    }

    // Material (:129-234)
    const JVal& mat = js["Material"];
    if (!mat.is_null()) {
        if (mat.t != JVal::Arr) LOAD_ERROR("Material must be array!");
        for (const auto& m : mat.a) {
            static const char* mk[10] = {"Name", "Diffuse", "Emission", "Specular", "Transparent", "Roughness",
                                         "RefractionIndex", "ExtinctionCoef", "AbsorptionCoef", "ReducedScatteringCoef"};
            std::string s[10];
            for (int i = 0; i < 10; i++) {
                CHECK_PROPERTY("Material", m[mk[i]], mk[i]);
                if (!as_string(m[mk[i]], s[i])) LOAD_ERROR("Material property <%s> must be a string", mk[i]);
            }
            if (materials.count(s[0])) std::fprintf(stderr, "[Warning]Built-in materail <%s> is overlapped!\n", s[0].c_str());
            pt_material x;
            std::memset(&x, 0, sizeof(x));
            x.diffuse_color = parse_float3(s[1]);
            x.emission_color = parse_float3(s[2]);
            x.specular_color = parse_float3(s[3]);
            x.is_transparent = parse_bool(s[4]);
            x.roughness = clampf_(parse_float(s[5]), 0.0f, 1.0f);
            x.medium.refraction_index = parse_float(s[6]);
            x.medium.extinction_coefficient = parse_float(s[7]);
            x.medium.scattering.absorption_coefficient = parse_float3(s[8]);
            x.medium.scattering.reduced_scattering_coefficient = parse_float3(s[9]);
            x.diffuse_texture_id = -1;
            x.specular_texture_id = -1;
            static const char* tk[2] = {"DiffuseTextureId", "SpecularTextureId"};
            for (int k = 0; k < 2; k++) {
                const JVal& id = m[tk[k]];
                if (id.is_null()) continue;
                std::string ids;
                if (!as_string(id, ids)) LOAD_ERROR("Material property <%s> must be a string", tk[k]);
                const int tid = parse_int(ids);
                if (tid != -1 && (tid >= (int)texture_paths.size() || tid < 0))
                    LOAD_ERROR("Materail <%s>: Texture index out of range!", s[0].c_str());
                (k == 0 ? x.diffuse_texture_id : x.specular_texture_id) = tid;
            }
            if (x.is_transparent && x.medium.extinction_coefficient > 0.0f)
                LOAD_ERROR("Materail <%s>: Extinction coefficient of transparent material should be zero!", s[0].c_str());
            materials[s[0]] = x;
        }
    }

    // Sphere (:236-266)
    std::vector<std::pair<pt_float3, float>> spheres;
    std::vector<std::string> sphere_mats;
    const JVal& sph = js["Sphere"];
    if (!sph.is_null()) {
        if (sph.t != JVal::Arr) LOAD_ERROR("Sphere must be array!");
        for (const auto& s : sph.a) {
            CHECK_PROPERTY("Sphere", s["Center"], "Center");
            CHECK_PROPERTY("Sphere", s["Radius"], "Radius");
            CHECK_PROPERTY("Sphere", s["Material"], "Material");
            std::string c, r, m;
            if (!as_string(s["Center"], c) || !as_string(s["Radius"], r) || !as_string(s["Material"], m))
                LOAD_ERROR("Sphere properties must be strings");
            spheres.push_back({parse_float3(c), clampf_(parse_float(r), 0.0f, INFINITY)});
            sphere_mats.push_back(m);
        }
    }

    // Mesh (:268-317)
    std::vector<MeshSpec> meshes;
    const JVal& msh = js["Mesh"];
    if (!msh.is_null()) {
        if (msh.t != JVal::Arr) LOAD_ERROR("Mesh must be array!");
        for (const auto& m : msh.a) {
            CHECK_PROPERTY("Mesh", m["Path"], "Path");
            CHECK_PROPERTY("Mesh", m["Material"], "Material");
            CHECK_PROPERTY("Mesh", m["Position"], "Material");  // the reference's token (scene_parser.cpp:287)
            CHECK_PROPERTY("Mesh", m["Scale"], "Scale");
            CHECK_PROPERTY("Mesh", m["Rotate"], "Rotate");
            MeshSpec ms;
            std::string pos, scl, rot;
            if (!as_string(m["Path"], ms.path) || !as_string(m["Position"], pos) || !as_string(m["Scale"], scl) ||
                !as_string(m["Rotate"], rot))
                LOAD_ERROR("Mesh properties must be strings");
            if (m["Material"].t != JVal::Arr) LOAD_ERROR("Material of mesh must be array!");
            for (const auto& x : m["Material"].a) {
                std::string s;
                if (!as_string(x, s)) LOAD_ERROR("Mesh materials must be strings");
                ms.mats.push_back(s);
            }
            ms.position = parse_float3(pos);
            pt_float3 sc = parse_float3(scl);
            ms.scale = {clampf_(sc.x, 0.0f, INFINITY), clampf_(sc.y, 0.0f, INFINITY), clampf_(sc.z, 0.0f, INFINITY)};
            ms.rotate = parse_float3(rot);
            meshes.push_back(ms);
        }
    }

    // Background images: square, all the same size (cube_map_loader.cpp:3-102)
    std::vector<unsigned char> cube;
    int cube_len = 0;
    for (int f = 0; f < 6; f++) {
        int w = 0, h = 0;
        unsigned char* px = nullptr;
        std::fprintf(stderr, "[Info]Loading file %s....\n", cube_paths[f].c_str());
        const int rc = pt_image_load(cube_paths[f].c_str(), &w, &h, &px);
        const bool bad = rc != 0 || w != h || (f > 0 && w != cube_len);
        if (bad) {
            pt_image_free(px);
            LOAD_ERROR("Background load fail, please check the <Path> and <Name>!");
        }
        if (f == 0) { cube_len = w; cube.resize((size_t)6 * w * w * 4); }
        std::memcpy(cube.data() + (size_t)f * w * w * 4, px, (size_t)w * w * 4);
        pt_image_free(px);
    }

    // Textures (:339-368)
    std::vector<int> tex_ids;
    std::vector<std::vector<unsigned char>> tex_px;
    std::vector<int> tex_w, tex_h;
    for (const auto& tp : texture_paths) {
        int w = 0, h = 0;
        unsigned char* px = nullptr;
        const std::string p = fix_path(tp, root);
        std::fprintf(stderr, "[Info]Load texture %s...\n", p.c_str());
        if (pt_image_load(p.c_str(), &w, &h, &px) != 0) LOAD_ERROR("Texture %s load fail.", p.c_str());
        tex_px.emplace_back(px, px + (size_t)w * h * 4);
        tex_w.push_back(w);
        tex_h.push_back(h);
        pt_image_free(px);
    }

    // every material must exist (:370-402)
    bool missing = false;
    for (const auto& m : sphere_mats)
        if (!materials.count(m)) { std::fprintf(stderr, "[Error]Material <%s> not found!\n", m.c_str()); missing = true; }
    for (const auto& ms : meshes)
        for (const auto& m : ms.mats)
            if (!materials.count(m)) { std::fprintf(stderr, "[Error]Material <%s> not found!\n", m.c_str()); missing = true; }
    if (missing) return -12;

    // meshes (:404-427): each mesh owns copies of its materials; shape i uses material
    // min(i, count - 1); a mesh without texcoords disables the diffuse texture of the materials
    // its shapes use (triangle_mesh.cpp:131-137)
    std::vector<pt_obj_mesh> objs(meshes.size());
    for (size_t i = 0; i < meshes.size(); i++) {
        const std::string p = fix_path(meshes[i].path, root);
        std::fprintf(stderr, "[Info]Loading file %s....\n", p.c_str());
        if (meshes[i].mats.empty() || pt_obj_load(p.c_str(), &objs[i]) != 0) {
            for (auto& ob : objs) pt_obj_free(&ob);
            return -13;
        }
    }

    pt_scene_builder_set_cube_map(b, cube_len, cube.data());
    for (size_t t = 0; t < tex_px.size(); t++) pt_scene_builder_add_texture(b, tex_w[t], tex_h[t], tex_px[t].data());
    int rc = 0;
    for (size_t i = 0; i < meshes.size() && rc == 0; i++) {
        const pt_obj_mesh& ob = objs[i];
        const int nm = (int)meshes[i].mats.size();
        std::vector<pt_material> mm(nm);
        for (int k = 0; k < nm; k++) mm[k] = materials[meshes[i].mats[k]];
        if (!ob.uvs)
            for (int t = 0; t < ob.triangle_num; t++) mm[std::min(ob.shape_of_triangle[t], nm - 1)].diffuse_texture_id = -1;
        int base = -1;
        for (int k = 0; k < nm; k++) {
            int id = pt_scene_builder_add_material(b, &mm[k]);
            if (k == 0) base = id;
        }
        std::vector<int> tri_mat((size_t)std::max(ob.triangle_num, 1));
        for (int t = 0; t < ob.triangle_num; t++) tri_mat[t] = base + std::min(ob.shape_of_triangle[t], nm - 1);
        if (ob.triangle_num > 0 &&
            pt_scene_builder_add_mesh(b, ob.triangle_num, ob.vertices, ob.normals, ob.uvs, tri_mat.data(),
                                      meshes[i].position, meshes[i].scale, meshes[i].rotate) < 0)
            rc = -14;
    }
    for (auto& ob : objs) pt_obj_free(&ob);
    if (rc) return rc;
    for (size_t i = 0; i < spheres.size(); i++) {
        const pt_material m = materials[sphere_mats[i]];
        pt_scene_builder_add_sphere(b, spheres[i].first, spheres[i].second, &m);
    }
    return pt_scene_builder_build_ex(b, o.leaf_size, o.bvh_method, o.bucket_num);
}
