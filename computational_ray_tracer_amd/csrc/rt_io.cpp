// Scene ingest and image output around the hot path, host-only C-ABI entry points:
//   rt_load_obj / rt_mesh_free  — Wavefront OBJ → the MeshCache::Mesh layout the reference builds with assimp
//                                 (AssetManager.cpp:67-190: aiProcess_Triangulate | aiProcess_GenNormals, one
//                                 vertex per face corner, flat face normals when the file has none)
//   rt_image_write              — 8-bit RGB to PNG (stored deflate blocks, no zlib dependency) or binary PPM
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "rt_guard.h"
#include "../../include/rtmi355x.h"

namespace {

struct V3f { float x, y, z; };

// OBJ index: 1-based, negative = relative to the end of the list so far
bool resolve_index(long v, size_t n, size_t* out) {
    if (v > 0 && (size_t)v <= n) { *out = (size_t)v - 1; return true; }
    if (v < 0 && (size_t)(-v) <= n) { *out = n - (size_t)(-v); return true; }
    return false;
}

struct Corner { size_t v; long vt; long vn; };

bool parse_corner(const char* tok, size_t nv, size_t nvt, size_t nvn, Corner* c) {
    char* end;
    long v = std::strtol(tok, &end, 10);
    if (end == tok || !resolve_index(v, nv, &c->v)) return false;
    c->vt = -1; c->vn = -1;
    if (*end != '/') return *end == 0;
    const char* p = end + 1;
    if (*p != '/') {
        long t = std::strtol(p, &end, 10);
        size_t r;
        if (end != p && resolve_index(t, nvt, &r)) c->vt = (long)r;
        p = end;
    }
    if (*p == '/') {
        ++p;
        long nn = std::strtol(p, &end, 10);
        size_t r;
        if (end != p && resolve_index(nn, nvn, &r)) c->vn = (long)r;
    }
    return true;
}

void crc_table(uint32_t* t) {
    for (uint32_t n = 0; n < 256; ++n) {
        uint32_t c = n;
        for (int k = 0; k < 8; ++k) c = (c & 1) ? 0xedb88320u ^ (c >> 1) : c >> 1;
        t[n] = c;
    }
}

void put32(std::vector<unsigned char>& b, uint32_t v) {
    b.push_back((unsigned char)(v >> 24)); b.push_back((unsigned char)(v >> 16));
    b.push_back((unsigned char)(v >> 8)); b.push_back((unsigned char)v);
}

void chunk(std::vector<unsigned char>& out, const char* type, const std::vector<unsigned char>& data, const uint32_t* crc) {
    put32(out, (uint32_t)data.size());
    size_t s = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    uint32_t c = 0xffffffffu;
    for (size_t i = s; i < out.size(); ++i) c = crc[(c ^ out[i]) & 0xff] ^ (c >> 8);
    put32(out, c ^ 0xffffffffu);
}

}  // namespace

extern "C" {

static void impl_rt_mesh_free(rt_mesh* m);
static int impl_rt_load_obj(const char* path, rt_mesh** out) {
    if (!path || !out) return RT_E_ARG;
    *out = nullptr;
    FILE* f = std::fopen(path, "rb");
    if (!f) return RT_E_ARG;
    std::vector<V3f> v, vn;
    std::vector<float> vt;
    std::vector<Corner> corners;  // 3 per triangle, fan-triangulated (aiProcess_Triangulate)
    char line[4096];
    bool ok = true;
    while (ok && std::fgets(line, sizeof(line), f)) {
        char* s = line;
        while (*s == ' ' || *s == '\t') ++s;
        if (s[0] == 'v' && (s[1] == ' ' || s[1] == '\t')) {
            V3f p{0, 0, 0};
            if (std::sscanf(s + 2, "%f %f %f", &p.x, &p.y, &p.z) < 3) ok = false;
            v.push_back(p);
        } else if (s[0] == 'v' && s[1] == 'n') {
            V3f p{0, 0, 0};
            if (std::sscanf(s + 3, "%f %f %f", &p.x, &p.y, &p.z) < 3) ok = false;
            vn.push_back(p);
        } else if (s[0] == 'v' && s[1] == 't') {
            float a = 0, b = 0;
            std::sscanf(s + 3, "%f %f", &a, &b);
            vt.push_back(a); vt.push_back(b);
        } else if (s[0] == 'f' && (s[1] == ' ' || s[1] == '\t')) {
            std::vector<Corner> poly;
            char* save = nullptr;
            for (char* tok = strtok_r(s + 2, " \t\r\n", &save); tok; tok = strtok_r(nullptr, " \t\r\n", &save)) {
                Corner c;
                if (!parse_corner(tok, v.size(), vt.size() / 2, vn.size(), &c)) { ok = false; break; }
                poly.push_back(c);
            }
            if (ok && poly.size() < 3) ok = false;
            for (size_t k = 1; ok && k + 1 < poly.size(); ++k) {
                corners.push_back(poly[0]); corners.push_back(poly[k]); corners.push_back(poly[k + 1]);
            }
        }
    }
    std::fclose(f);
    if (!ok || corners.empty()) return RT_E_ARG;
    size_t nc = corners.size();
    rt_mesh* m = (rt_mesh*)std::calloc(1, sizeof(rt_mesh));
    if (!m) return RT_E_OOM;
    m->n_vertices = (int)nc;
    m->n_triangles = (int)(nc / 3);
    m->positions = (float*)std::malloc(sizeof(float) * 3 * nc);
    m->normals = (float*)std::malloc(sizeof(float) * 3 * nc);
    m->texcoords = (float*)std::malloc(sizeof(float) * 2 * nc);
    m->indices = (uint32_t*)std::malloc(sizeof(uint32_t) * nc);
    if (!m->positions || !m->normals || !m->texcoords || !m->indices) {
        impl_rt_mesh_free(m);
        return RT_E_OOM;
    }
    for (size_t t = 0; t < nc / 3; ++t) {
        const V3f& a = v[corners[3 * t].v];
        const V3f& b = v[corners[3 * t + 1].v];
        const V3f& c = v[corners[3 * t + 2].v];
        // aiProcess_GenNormals without shared vertices: the face normal normalize((b - a) x (c - a))
        V3f e1{b.x - a.x, b.y - a.y, b.z - a.z}, e2{c.x - a.x, c.y - a.y, c.z - a.z};
        V3f fnrm{e1.y * e2.z - e1.z * e2.y, e1.z * e2.x - e1.x * e2.z, e1.x * e2.y - e1.y * e2.x};
        float l = std::sqrt(fnrm.x * fnrm.x + fnrm.y * fnrm.y + fnrm.z * fnrm.z);
        if (l > 0) { fnrm.x /= l; fnrm.y /= l; fnrm.z /= l; }
        for (int k = 0; k < 3; ++k) {
            const Corner& cr = corners[3 * t + k];
            size_t i = 3 * t + k;
            const V3f& p = v[cr.v];
            m->positions[3 * i] = p.x; m->positions[3 * i + 1] = p.y; m->positions[3 * i + 2] = p.z;
            V3f n = cr.vn >= 0 ? vn[(size_t)cr.vn] : fnrm;
            m->normals[3 * i] = n.x; m->normals[3 * i + 1] = n.y; m->normals[3 * i + 2] = n.z;
            m->texcoords[2 * i] = cr.vt >= 0 ? vt[2 * (size_t)cr.vt] : 0.f;
            m->texcoords[2 * i + 1] = cr.vt >= 0 ? vt[2 * (size_t)cr.vt + 1] : 0.f;
            m->indices[i] = (uint32_t)i;
        }
    }
    *out = m;
    return RT_OK;
}

static void impl_rt_mesh_free(rt_mesh* m) {
    if (!m) return;
    std::free(m->positions); std::free(m->normals); std::free(m->texcoords); std::free(m->indices);
    std::free(m);
}

static int impl_rt_image_write(const char* path, int w, int h, const uint8_t* rgb, int flip_y) {
    if (!path || !rgb || w <= 0 || h <= 0) return RT_E_ARG;
    std::string p(path);
    bool png = p.size() >= 4 && (p.compare(p.size() - 4, 4, ".png") == 0 || p.compare(p.size() - 4, 4, ".PNG") == 0);
    FILE* f = std::fopen(path, "wb");
    if (!f) return RT_E_ARG;
    auto row = [&](int y) { return rgb + (size_t)3 * w * (flip_y ? h - 1 - y : y); };
    if (!png) {
        std::fprintf(f, "P6\n%d %d\n255\n", w, h);
        for (int y = 0; y < h; ++y) std::fwrite(row(y), 1, (size_t)3 * w, f);
        std::fclose(f);
        return RT_OK;
    }
    uint32_t crc[256];
    crc_table(crc);
    std::vector<unsigned char> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'}, ihdr, idat;
    put32(ihdr, (uint32_t)w); put32(ihdr, (uint32_t)h);
    ihdr.insert(ihdr.end(), {8, 2, 0, 0, 0});  // 8-bit RGB, no interlace
    chunk(out, "IHDR", ihdr, crc);
    // zlib stream of stored deflate blocks over the filtered scanlines (filter byte 0)
    std::vector<unsigned char> raw;
    raw.reserve((size_t)h * (3 * w + 1));
    for (int y = 0; y < h; ++y) { raw.push_back(0); raw.insert(raw.end(), row(y), row(y) + (size_t)3 * w); }
    idat.push_back(0x78); idat.push_back(0x01);
    size_t pos = 0;
    do {
        size_t len = std::min<size_t>(65535, raw.size() - pos);
        bool last = pos + len == raw.size();
        idat.push_back(last ? 1 : 0);
        idat.push_back((unsigned char)(len & 0xff)); idat.push_back((unsigned char)(len >> 8));
        idat.push_back((unsigned char)(~len & 0xff)); idat.push_back((unsigned char)((~len >> 8) & 0xff));
        idat.insert(idat.end(), raw.begin() + pos, raw.begin() + pos + len);
        pos += len;
    } while (pos < raw.size());
    uint32_t a = 1, b = 0;  // adler32
    for (unsigned char c : raw) { a = (a + c) % 65521u; b = (b + a) % 65521u; }
    put32(idat, (b << 16) | a);
    chunk(out, "IDAT", idat, crc);
    chunk(out, "IEND", {}, crc);
    size_t wrote = std::fwrite(out.data(), 1, out.size(), f);
    std::fclose(f);
    return wrote == out.size() ? RT_OK : RT_E_ARG;
}

}  // extern "C"

// ---- the exception firewall around every entry point (rt_guard.h)
using rtmi::guarded;
extern "C" {
int rt_load_obj(const char* path, rt_mesh** out) {
    return guarded([&] { return impl_rt_load_obj(path, out); }, [](const std::string&) {});
}
int rt_image_write(const char* path, int w, int h, const uint8_t* rgb, int flip_y) {
    return guarded([&] { return impl_rt_image_write(path, w, h, rgb, flip_y); }, [](const std::string&) {});
}
void rt_mesh_free(rt_mesh* m) {
    guarded([&] { impl_rt_mesh_free(m); return 0; }, [](const std::string&) {}, /*inject=*/false);
}

}  // extern "C"
