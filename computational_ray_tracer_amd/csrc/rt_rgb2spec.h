// The RGB -> RGBSigmoidPolynomial fit (Jakob & Hanika 2019, the method of pbrt-v4's rgb2spec_opt, which generates the
// coefficient table the reference loads from "rgb2spec/sRGB64binary", color.cpp:107-171): Gauss-Newton on the
// CIELAB difference between the target sRGB colour and the sigmoid spectrum under D65, wavelength normalised to
// [0, 1] over 360..830 nm.  Shared by rt_color.cpp (rt_rgb_fit_sigmoid) and the table generator
// (tools/rgb2spec_gen.cpp).  Host only; double precision.
#pragma once
#include <cmath>
#include <cstring>
#include <utility>

#include "../data/spectra_data.h"

namespace rgb2spec {


constexpr int kN = 471;  // 360..830 nm, 1 nm
constexpr double kLmin = 360.0, kLmax = 830.0;

// sRGB (D65) from XYZ, IEC 61966-2-1
inline const double kXYZ2RGB[3][3] = {{3.2404542, -1.5371385, -0.4985314},
                               {-0.9692660, 1.8760108, 0.0415560},
                               {0.0556434, -0.2040259, 1.0572252}};
inline const double kRGB2XYZ[3][3] = {{0.4124564, 0.3575761, 0.1804375},
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

inline const Tables& tables() {
    static Tables t;
    return t;
}

inline double lab_f(double t) {
    const double d = 6.0 / 29.0;
    return t > d * d * d ? std::cbrt(t) : t / (3 * d * d) + 4.0 / 29.0;
}
inline void xyz_to_lab(const double* xyz, double* lab) {
    const Tables& T = tables();
    double fx = lab_f(xyz[0] / T.white[0]), fy = lab_f(xyz[1] / T.white[1]), fz = lab_f(xyz[2] / T.white[2]);
    lab[0] = 116 * fy - 16;
    lab[1] = 500 * (fx - fy);
    lab[2] = 200 * (fy - fz);
}
inline double sigmoid(double x) { return 0.5 + x / (2 * std::sqrt(1 + x * x)); }

inline void spectrum_lab(const double* c, double* lab) {
    const Tables& T = tables();
    double xyz[3] = {0, 0, 0};
    for (int i = 0; i < kN; ++i) {
        double l = i / (kLmax - kLmin);
        double s = sigmoid((c[0] * l + c[1]) * l + c[2]);
        for (int k = 0; k < 3; ++k) xyz[k] += T.w[k][i] * s;
    }
    xyz_to_lab(xyz, lab);
}

inline void residual(const double* c, const double* target_lab, double* r) {
    double lab[3];
    spectrum_lab(c, lab);
    for (int k = 0; k < 3; ++k) r[k] = target_lab[k] - lab[k];
}

inline bool solve3(double A[3][3], double* b) {  // Gaussian elimination with partial pivoting, A x = b
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

inline void gauss_newton(const double* rgb, double* c) {
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


// coefficients of the normalised wavelength -> coefficients of λ in nm, so that R(λ) = s(c0 λ² + c1 λ + c2)
inline void to_nm(const double* c, double* out) {
    const double s = 1.0 / (kLmax - kLmin);
    out[0] = c[0] * s * s;
    out[1] = c[1] * s - 2 * c[0] * kLmin * s * s;
    out[2] = c[2] - c[1] * kLmin * s + c[0] * kLmin * kLmin * s * s;
}

}  // namespace rgb2spec
