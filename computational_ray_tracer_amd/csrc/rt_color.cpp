// RGB -> RGBSigmoidPolynomial coefficients: the reference's RGBToSpectrumTable
// (color.cpp:26-72) interpolates a precomputed 3 x 64^3 coefficient table loaded from "rgb2spec/sRGB64binary"
// (color.cpp:114), which is not in the repository.  This fits the coefficients for one colour directly with the
// table generator's method (Jakob & Hanika 2019, pbrt-v4 rgb2spec_opt): Gauss-Newton on the CIELAB difference
// between the target sRGB colour and the sigmoid spectrum under D65, wavelength normalised to [0, 1] over
// 360..830 nm, then re-expressed in nm so that R(λ) = s(c0 λ² + c1 λ + c2) (color.h:363-403).  Grey inputs take
// the reference's closed-form branch (color.cpp:35-37).  Host only; double precision.
#include <cmath>
#include <cstring>
#include <utility>

#include "rt_guard.h"
#include "../../include/rtmi355x.h"
#include "../data/spectra_data.h"

namespace {

constexpr int kN = 471;  // 360..830 nm, 1 nm
constexpr double kLmin = 360.0, kLmax = 830.0;

// sRGB (D65) from XYZ, IEC 61966-2-1
const double kXYZ2RGB[3][3] = {{3.2404542, -1.5371385, -0.4985314},
                               {-0.9692660, 1.8760108, 0.0415560},
                               {0.0556434, -0.2040259, 1.0572252}};
const double kRGB2XYZ[3][3] = {{0.4124564, 0.3575761, 0.1804375},
                               {0.2126729, 0.7151522, 0.0721750},
                               {0.0193339, 0.1191920, 0.9503041}};

struct Tables {
    double w[3][kN];   // CIE x/y/z * D65, normalised so that a unit spectrum has Y = 1
    double white[3];   // XYZ of the unit spectrum
    Tables() {
        const float* il = rtdata::illum_d65;  // interleaved (λ, value)
        int n = rtdata::illum_d65_n / 2;
        auto d65 = [&](double l) {
            if (l <= il[0]) return (double)il[1];
            for (int i = 0; i + 1 < n; ++i)
                if (l <= il[2 * (i + 1)]) {
                    double t = (l - il[2 * i]) / (il[2 * (i + 1)] - il[2 * i]);
                    return (1 - t) * il[2 * i + 1] + t * il[2 * (i + 1) + 1];
                }
            return (double)il[2 * n - 1];
        };
        const float* cie[3] = {rtdata::cie_x, rtdata::cie_y, rtdata::cie_z};
        double norm = 0;
        for (int i = 0; i < kN; ++i) norm += cie[1][i] * d65(kLmin + i);
        for (int c = 0; c < 3; ++c) {
            white[c] = 0;
            for (int i = 0; i < kN; ++i) {
                w[c][i] = cie[c][i] * d65(kLmin + i) / norm;
                white[c] += w[c][i];
            }
        }
    }
};

const Tables& tables() {
    static Tables t;
    return t;
}

double lab_f(double t) {
    const double d = 6.0 / 29.0;
    return t > d * d * d ? std::cbrt(t) : t / (3 * d * d) + 4.0 / 29.0;
}
void xyz_to_lab(const double* xyz, double* lab) {
    const Tables& T = tables();
    double fx = lab_f(xyz[0] / T.white[0]), fy = lab_f(xyz[1] / T.white[1]), fz = lab_f(xyz[2] / T.white[2]);
    lab[0] = 116 * fy - 16;
    lab[1] = 500 * (fx - fy);
    lab[2] = 200 * (fy - fz);
}
double sigmoid(double x) { return 0.5 + x / (2 * std::sqrt(1 + x * x)); }

void spectrum_lab(const double* c, double* lab) {
    const Tables& T = tables();
    double xyz[3] = {0, 0, 0};
    for (int i = 0; i < kN; ++i) {
        double l = i / (kLmax - kLmin);
        double s = sigmoid((c[0] * l + c[1]) * l + c[2]);
        for (int k = 0; k < 3; ++k) xyz[k] += T.w[k][i] * s;
    }
    xyz_to_lab(xyz, lab);
}

void residual(const double* c, const double* target_lab, double* r) {
    double lab[3];
    spectrum_lab(c, lab);
    for (int k = 0; k < 3; ++k) r[k] = target_lab[k] - lab[k];
}

bool solve3(double A[3][3], double* b) {  // Gaussian elimination with partial pivoting, A x = b
    for (int col = 0; col < 3; ++col) {
        int p = col;
        for (int r = col + 1; r < 3; ++r)
            if (std::fabs(A[r][col]) > std::fabs(A[p][col])) p = r;
        if (std::fabs(A[p][col]) < 1e-15) return false;
        if (p != col) {
            for (int k = 0; k < 3; ++k) std::swap(A[p][k], A[col][k]);
            std::swap(b[p], b[col]);
        }
        for (int r = col + 1; r < 3; ++r) {
            double f = A[r][col] / A[col][col];
            for (int k = col; k < 3; ++k) A[r][k] -= f * A[col][k];
            b[r] -= f * b[col];
        }
    }
    for (int r = 2; r >= 0; --r) {
        for (int k = r + 1; k < 3; ++k) b[r] -= A[r][k] * b[k];
        b[r] /= A[r][r];
    }
    return true;
}

void gauss_newton(const double* rgb, double* c) {
    double xyz[3], lab[3];
    for (int k = 0; k < 3; ++k) xyz[k] = kRGB2XYZ[k][0] * rgb[0] + kRGB2XYZ[k][1] * rgb[1] + kRGB2XYZ[k][2] * rgb[2];
    xyz_to_lab(xyz, lab);
    for (int it = 0; it < 30; ++it) {
        double r[3];
        residual(c, lab, r);
        double J[3][3];
        for (int j = 0; j < 3; ++j) {  // central differences, eps 1e-5 (rgb2spec_opt eval_jacobian)
            double cp[3] = {c[0], c[1], c[2]}, cm[3] = {c[0], c[1], c[2]}, rp[3], rm[3];
            cp[j] += 1e-5; cm[j] -= 1e-5;
            residual(cp, lab, rp);
            residual(cm, lab, rm);
            for (int i = 0; i < 3; ++i) J[i][j] = (rp[i] - rm[i]) / 2e-5;
        }
        double x[3] = {r[0], r[1], r[2]};
        if (!solve3(J, x)) break;
        for (int k = 0; k < 3; ++k) c[k] -= x[k];
        double m = std::fmax(std::fmax(std::fabs(c[0]), std::fabs(c[1])), std::fabs(c[2]));
        if (m > 200) for (int k = 0; k < 3; ++k) c[k] *= 200 / m;  // rgb2spec_opt's coefficient clamp
        if (std::sqrt(r[0] * r[0] + r[1] * r[1] + r[2] * r[2]) < 1e-6) break;
    }
}

}  // namespace

extern "C" {

static int impl_rt_rgb_to_sigmoid(const float* rgb, float* coeffs) {
    if (!rgb || !coeffs) return RT_E_ARG;
    for (int k = 0; k < 3; ++k)
        if (!(rgb[k] >= 0.f && rgb[k] <= 1.f)) return RT_E_ARG;
    if (rgb[0] == rgb[1] && rgb[1] == rgb[2]) {  // color.cpp:35-37, in float like the reference
        float g = rgb[0];
        coeffs[0] = 0; coeffs[1] = 0;
        coeffs[2] = (g - .5f) / std::sqrt(g * (1 - g));  // +-inf at 0 and 1: s(+-inf) = 1, 0
        return RT_OK;
    }
    // continuation from the grey of equal mean towards the target (rgb2spec_opt marches from the grey axis)
    double c[3] = {0, 0, 0};
    double mean = (rgb[0] + rgb[1] + rgb[2]) / 3.0;
    double mc = std::fmin(std::fmax(mean, 1e-3), 1 - 1e-3);
    c[2] = (mc - .5) / std::sqrt(mc * (1 - mc));
    const int steps = 16;
    for (int s = 1; s <= steps; ++s) {
        double f = (double)s / steps, t[3];
        for (int k = 0; k < 3; ++k) t[k] = mc + f * (rgb[k] - mc);
        gauss_newton(t, c);
    }
    // λ_n = (λ - 360) / 470  ->  coefficients of λ in nm
    double s = 1.0 / (kLmax - kLmin);
    double A = c[0] * s * s, B = c[1] * s - 2 * c[0] * kLmin * s * s, C = c[2] - c[1] * kLmin * s + c[0] * kLmin * kLmin * s * s;
    coeffs[0] = (float)A; coeffs[1] = (float)B; coeffs[2] = (float)C;
    return RT_OK;
}

}  // extern "C"

// ---- the exception firewall around every entry point (rt_guard.h)
using rtmi::guarded;
extern "C" {
int rt_rgb_to_sigmoid(const float* rgb, float* coeffs) {
    return guarded([&] { return impl_rt_rgb_to_sigmoid(rgb, coeffs); }, [](const std::string&) {});
}

}  // extern "C"
