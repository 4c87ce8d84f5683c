// RGB -> RGBSigmoidPolynomial coefficients.  The reference's RGBToSpectrumTable (color.cpp:26-72)
// trilinearly interpolates a 3 x 64^3 x 3 coefficient table that RGBToSpectrumTable::Init (color.cpp:107-171) reads
// from "../rgb2spec/sRGB64binary" — a file the repository does not contain.  The build regenerates that table with
// the generator's method (tools/rgb2spec_gen.cpp over the fit of rt_rgb2spec.h; file layout exactly the one Init
// reads: a big-endian int resolution, 64 float z-nodes, the float[3][64][64][64][3] coefficients; checksum in
// data/srgb64.rgbspec.sha256) and restates the reference's lookup over it:
//   rt_rgb_to_sigmoid  = RGBToSpectrumTable::operator() — uniform-RGB closed form (color.cpp:35-37), else the largest
//                        component's table, (x, y) = the other two scaled by (res - 1) / z, z's interval by
//                        FindInterval over the z-nodes (helpers.h:159-172), then float trilinear Lerps;
//   rt_rgb_fit_sigmoid = the fit itself, for one colour (the table generator's per-entry solve).
// The table is found next to the library (../data/srgb64.rgbspec) or through RTMI_RGBSPEC_TABLE.
#include <dlfcn.h>

#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <mutex>
#include <string>
#include <vector>

#include "rt_guard.h"
#include "rt_rgb2spec.h"
#include "../../include/rtmi355x.h"

namespace {

struct RgbTable {
    int res = 0;
    std::vector<float> z, coeffs;  // res z-nodes; [3][res][res][res][3]
};

// RGBToSpectrumTable::Init's reader (color.cpp:107-171): 4-byte big-endian int, res floats, 3 * res^3 * 3 floats
bool load_table(const std::string& path, RgbTable& t) {
    FILE* f = std::fopen(path.c_str(), "rb");
    if (!f) return false;
    unsigned char b[4];
    bool ok = std::fread(b, 1, 4, f) == 4;
    const int res = (b[0] << 24) | (b[1] << 16) | (b[2] << 8) | b[3];  // UtoInt
    ok = ok && res == 64;
    if (ok) {
        t.res = res;
        t.z.resize(res);
        t.coeffs.resize((size_t)3 * res * res * res * 3);
        ok = std::fread(t.z.data(), 4, t.z.size(), f) == t.z.size() &&
             std::fread(t.coeffs.data(), 4, t.coeffs.size(), f) == t.coeffs.size();
    }
    std::fclose(f);
    return ok;
}

std::string table_path() {
    if (const char* e = std::getenv("RTMI_RGBSPEC_TABLE")) return e;
    Dl_info info;
    if (dladdr((void*)&table_path, &info) && info.dli_fname) {
        std::string so(info.dli_fname);
        size_t p = so.find_last_of('/');
        std::string dir = p == std::string::npos ? "." : so.substr(0, p);
        return dir + "/../data/srgb64.rgbspec";
    }
    return "srgb64.rgbspec";
}

const RgbTable* table() {
    static RgbTable t;
    static bool ok = false;
    static std::once_flag once;
    std::call_once(once, [] { ok = load_table(table_path(), t); });
    return ok ? &t : nullptr;
}

inline float lerp(float x, float a, float b) { return (1 - x) * a + x * b; }  // helpers.h:154-157

// color.cpp:26-72 RGBToSpectrumTable::operator() (non-uniform branch)
void table_lookup(const RgbTable& T, const float* rgb, float* c) {
    const int res = T.res;
    const int maxc = (rgb[0] > rgb[1]) ? ((rgb[0] > rgb[2]) ? 0 : 2) : ((rgb[1] > rgb[2]) ? 1 : 2);
    const float z = rgb[maxc];
    const float x = rgb[(maxc + 1) % 3] * (res - 1) / z;
    const float y = rgb[(maxc + 2) % 3] * (res - 1) / z;
    const int xi = std::min((int)x, res - 2), yi = std::min((int)y, res - 2);
    long size = (long)res - 2, first = 1;  // FindInterval(res, zNodes[i] < z)
    while (size > 0) {
        const long half = size >> 1, middle = first + half;
        const bool r = T.z[middle] < z;
        first = r ? middle + 1 : first;
        size = r ? size - (half + 1) : half;
    }
    const int zi = (int)std::min(std::max(first - 1, 0L), (long)res - 2);
    const float dx = x - xi, dy = y - yi, dz = (z - T.z[zi]) / (T.z[zi + 1] - T.z[zi]);
    for (int i = 0; i < 3; ++i) {
        auto co = [&](int ox, int oy, int oz) {
            const size_t index = (size_t)maxc * 64 * 64 * 64 * 3 + (size_t)(zi + oz) * 64 * 64 * 3 +
                                 (size_t)(yi + oy) * 64 * 3 + (size_t)(xi + ox) * 3 + i;
            return T.coeffs[index];
        };
        c[i] = lerp(dz, lerp(dy, lerp(dx, co(0, 0, 0), co(1, 0, 0)), lerp(dx, co(0, 1, 0), co(1, 1, 0))),
                    lerp(dy, lerp(dx, co(0, 0, 1), co(1, 0, 1)), lerp(dx, co(0, 1, 1), co(1, 1, 1))));
    }
}

bool valid_rgb(const float* rgb) {
    for (int k = 0; k < 3; ++k)
        if (!(rgb[k] >= 0.f && rgb[k] <= 1.f)) return false;
    return true;
}

}  // namespace

extern "C" {

static int impl_rt_rgb_to_sigmoid(const float* rgb, float* coeffs) {
    if (!rgb || !coeffs || !valid_rgb(rgb)) return RT_E_ARG;
    if (rgb[0] == rgb[1] && rgb[1] == rgb[2]) {  // color.cpp:35-37, in float like the reference
        float g = rgb[0];
        coeffs[0] = 0; coeffs[1] = 0;
        coeffs[2] = (g - .5f) / std::sqrt(g * (1 - g));  // +-inf at 0 and 1: s(+-inf) = 1, 0
        return RT_OK;
    }
    const RgbTable* T = table();
    if (!T) return RT_E_STATE;  // the coefficient table was not generated (python __graft_entry__.py build)
    table_lookup(*T, rgb, coeffs);
    return RT_OK;
}

static int impl_rt_rgb_fit_sigmoid(const float* rgb, float* coeffs) {
    if (!rgb || !coeffs || !valid_rgb(rgb)) return RT_E_ARG;
    if (rgb[0] == rgb[1] && rgb[1] == rgb[2]) return impl_rt_rgb_to_sigmoid(rgb, coeffs);
    // continuation from the grey of equal mean towards the target (rgb2spec_opt marches from a solved neighbour)
    double c[3] = {0, 0, 0};
    double mean = (rgb[0] + rgb[1] + rgb[2]) / 3.0;
    double mc = std::fmin(std::fmax(mean, 1e-3), 1 - 1e-3);
    c[2] = (mc - .5) / std::sqrt(mc * (1 - mc));
    const int steps = 16;
    for (int s = 1; s <= steps; ++s) {
        double f = (double)s / steps, t[3];
        for (int k = 0; k < 3; ++k) t[k] = mc + f * (rgb[k] - mc);
        rgb2spec::gauss_newton(t, c);
    }
    double nm[3];
    rgb2spec::to_nm(c, nm);
    for (int k = 0; k < 3; ++k) coeffs[k] = (float)nm[k];
    return RT_OK;
}

}  // extern "C"

// ---- the exception firewall around every entry point (rt_guard.h)
using rtmi::guarded;
extern "C" {
int rt_rgb_to_sigmoid(const float* rgb, float* coeffs) {
    return guarded([&] { return impl_rt_rgb_to_sigmoid(rgb, coeffs); }, [](const std::string&) {});
}
int rt_rgb_fit_sigmoid(const float* rgb, float* coeffs) {
    return guarded([&] { return impl_rt_rgb_fit_sigmoid(rgb, coeffs); }, [](const std::string&) {});
}

}  // extern "C"
