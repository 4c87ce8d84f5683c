// =====================================================================================================
//  rtcore — ORACLE.  TEST INFRASTRUCTURE ONLY.
//
//  A plain, scalar, AoS C++ restatement of the reference's Monte Carlo ray-tracing inner loop
//  (GiboDidact/Computational_ray_tracer).  Every function cites the reference file:line it follows.
//  It is the parity checker for the HIP product path (computational_ray_tracer_amd/) and the
//  `cpu_baseline` leg of bench.py.  Nothing in the product may include, link or call this file.
//
//  Parity status: the reference cannot be compiled here (MSVC-only C++,
//  glm/assimp/GLFW absent — SURVEY.md §8c), so this restatement is pinned by known-answer tests
//  (tests/test_oracle_known_answers.py) and by golden fixtures it generated (tests/golden/).
//  glm operation order is restated explicitly (glm itself is not vendored: parity is unpinned at the
//  glm boundary).  Transcendentals (cos/sin/atanh/cosh) are evaluated in double and
//  rounded to float on BOTH sides, a documented build choice (reference calls the float overloads).
//
//  Compile with -ffp-contract=off: FMA only where the reference calls std::fma.
// =====================================================================================================
#pragma once
#include <algorithm>
#include <array>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <limits>
#include <memory>
#include <queue>
#include <vector>

#include "../computational_ray_tracer_amd/data/spectra_data.h"

namespace rtcore {

// ---------------------------------------------------------------- constants (pch.h:39-46)
static const float OneMinusEpsilon = 1.0f - std::numeric_limits<float>::min();  // == 1.0f (quirk)
static const float Pi = 3.14159265358979323846f;
static const float InvPi = 0.31830988618379067154f;
static const float PiOver2 = 1.57079632679489661923f;
static const float PiOver4 = 0.78539816339744830961f;
static const float CIE_Y_integral = 106.856895f;  // spectrum.h:21
static const int NSpectrumSamples = 8;             // spectrum.h:19

// helpers.h:50-54 — MachineEpsilon is formed in double then stored as float; gamma(n) in float
static inline float MachineEpsilon() { return (float)((double)std::numeric_limits<float>::epsilon() * 0.5); }
static inline float gamma_(int n) {
    float me = MachineEpsilon();
    return ((float)n * me) / (1.0f - (float)n * me);
}

// ------------------------------------------------ transcendentals (documented build choice)
// sin/cos: a fixed float algorithm (Cody-Waite reduction by pi/2 + Cephes minimax polynomials, explicit
// fmaf) evaluated identically on host and device; accurate to ~1 ulp on the |x| <= 3pi/4 range the
// concentric-disk warp (Sampling.h:383-403) produces.  atanh/cosh: double evaluation rounded to float.
static inline void sincos_det(float x, float* s, float* c) {
    float k = std::rint(x * 0.636619772367581343f);
    float r = std::fmaf(-k, 1.57079637050628662109375f, x);
    r = std::fmaf(-k, -4.37113900018624283e-8f, r);
    float r2 = r * r;
    float sp = std::fmaf(std::fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2, -1.6666654611e-1f);
    float sr = std::fmaf(sp * r2, r, r);
    float cp = std::fmaf(std::fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2, 4.166664568298827e-2f);
    float cr = std::fmaf(cp * r2, r2, std::fmaf(-0.5f, r2, 1.0f));
    int q = (int)k & 3;
    *s = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
    *c = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
}
static inline float cos_f(float x) { float s, c; sincos_det(x, &s, &c); return c; }
static inline float sin_f(float x) { float s, c; sincos_det(x, &s, &c); return s; }
static inline float atanh_f(float x) { return (float)std::atanh((double)x); }
static inline float cosh_f(float x) { return (float)std::cosh((double)x); }

// ------------------------------------------------------------------------- glm restatement
struct vec2 { float x, y; };
struct vec3 {
    float x, y, z;
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
struct vec4 { float x, y, z, w; };
struct mat4 { float m[16]; };   // column-major: m[col*4+row] (glm layout)
struct mat3 { float m[9]; };    // column-major

static inline vec3 add(vec3 a, vec3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static inline vec3 sub(vec3 a, vec3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static inline vec3 mul(vec3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
// glm compute_dot<vec3>: tmp = a*b; (tmp.x + tmp.y) + tmp.z
static inline float dot(vec3 a, vec3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }
// glm compute_dot<vec4>: (tmp.x + tmp.y) + (tmp.z + tmp.w)
static inline float dot4(vec4 a, vec4 b) { return (a.x * b.x + a.y * b.y) + (a.z * b.z + a.w * b.w); }
// glm::cross
static inline vec3 cross(vec3 a, vec3 b) {
    return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y};
}
// glm::normalize = v * inversesqrt(dot(v,v)), inversesqrt(x) = 1/sqrt(x)
static inline vec3 normalize(vec3 v) { float s = 1.0f / std::sqrt(dot(v, v)); return mul(v, s); }
static inline vec4 normalize4(vec4 v) {
    float s = 1.0f / std::sqrt(dot4(v, v));
    return {v.x * s, v.y * s, v.z * s, v.w * s};
}
// glm mat4*vec4: Add2 = (m0*x + m1*y) + (m2*z + m3*w)
static inline vec4 mul(const mat4& M, vec4 v) {
    float o[4];
    for (int r = 0; r < 4; ++r) {
        float a0 = M.m[0 * 4 + r] * v.x, a1 = M.m[1 * 4 + r] * v.y;
        float a2 = M.m[2 * 4 + r] * v.z, a3 = M.m[3 * 4 + r] * v.w;
        o[r] = (a0 + a1) + (a2 + a3);
    }
    return {o[0], o[1], o[2], o[3]};
}
// glm mat3*vec3: (m0*x + m1*y) + m2*z
static inline vec3 mul(const mat3& M, vec3 v) {
    float o[3];
    for (int r = 0; r < 3; ++r) o[r] = (M.m[0 * 3 + r] * v.x + M.m[1 * 3 + r] * v.y) + M.m[2 * 3 + r] * v.z;
    return {o[0], o[1], o[2]};
}
// glm::max/min scalar: max(x,y) = (x < y) ? y : x ; min(x,y) = (y < x) ? y : x ; clamp = min(max(x,lo),hi)
static inline float gmax(float x, float y) { return (x < y) ? y : x; }
static inline float gmin(float x, float y) { return (y < x) ? y : x; }
static inline float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }

// helpers.h:56-62 DifferenceOfProducts (the one place the path uses FMA)
static inline float DifferenceOfProducts(float a, float b, float c, float d) {
    float cd = c * d;
    float dop = std::fmaf(a, b, -cd);
    float err = std::fmaf(-c, d, cd);
    return dop + err;
}
// helpers.h:64-71
static inline int MaxComponentIndex(vec3 t) { return (t.x > t.y) ? ((t.x > t.z) ? 0 : 2) : ((t.y > t.z) ? 1 : 2); }
static inline float MaxComponentValue(vec3 t) {  // std::max({x,y,z}) keeps the first largest
    float m = t.x;
    if (m < t.y) m = t.y;
    if (m < t.z) m = t.z;
    return m;
}
// helpers.h:154-157
static inline float Lerp(float x, float a, float b) { return (1 - x) * a + x * b; }
// helpers.h:159-172
template <typename P>
static inline size_t FindInterval(size_t sz, const P& pred) {
    long size = (long)sz - 2, first = 1;
    while (size > 0) {
        size_t half = (size_t)size >> 1, middle = first + half;
        bool r = pred((int)middle);
        first = r ? (long)middle + 1 : first;
        size = r ? size - (long)(half + 1) : (long)half;
    }
    long v = first - 1;
    long hi = (long)sz - 2;
    return (size_t)(v < 0 ? 0 : (v > hi ? hi : v));
}

// =============================================================== hashing / RNG (integer exact)
// hash.h:18-63
static inline uint64_t MurmurHash64A(const unsigned char* key, size_t len, uint64_t seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    const int r = 47;
    uint64_t h = seed ^ (len * m);
    const unsigned char* end = key + 8 * (len / 8);
    while (key != end) {
        uint64_t k;
        std::memcpy(&k, key, 8);
        key += 8;
        k *= m; k ^= k >> r; k *= m;
        h ^= k; h *= m;
    }
    switch (len & 7) {
        case 7: h ^= uint64_t(key[6]) << 48; [[fallthrough]];
        case 6: h ^= uint64_t(key[5]) << 40; [[fallthrough]];
        case 5: h ^= uint64_t(key[4]) << 32; [[fallthrough]];
        case 4: h ^= uint64_t(key[3]) << 24; [[fallthrough]];
        case 3: h ^= uint64_t(key[2]) << 16; [[fallthrough]];
        case 2: h ^= uint64_t(key[1]) << 8; [[fallthrough]];
        case 1: h ^= uint64_t(key[0]); h *= m;
    }
    h ^= h >> r; h *= m; h ^= h >> r;
    return h;
}
// hash.h:67-74 / HelperFunctions.h:137-144
static inline uint64_t MixBits(uint64_t v) {
    v ^= (v >> 31); v *= 0x7fb5d329728ea185ull;
    v ^= (v >> 27); v *= 0x81dadef4bc2dd44dull;
    v ^= (v >> 33);
    return v;
}
// hash.h:96-104 — Hash(ivec2 p, int seed): 12-byte packed key; Hash(ivec2 p, int dim, int seed): 16 bytes
static inline uint64_t Hash(int px, int py, int seed) {
    unsigned char buf[16];
    std::memcpy(buf + 0, &px, 4); std::memcpy(buf + 4, &py, 4); std::memcpy(buf + 8, &seed, 4);
    return MurmurHash64A(buf, 12, 0);
}
static inline uint64_t Hash(int px, int py, int dim, int seed) {
    unsigned char buf[16];
    std::memcpy(buf + 0, &px, 4); std::memcpy(buf + 4, &py, 4);
    std::memcpy(buf + 8, &dim, 4); std::memcpy(buf + 12, &seed, 4);
    return MurmurHash64A(buf, 16, 0);
}
// HelperFunctions.h:175-203
static inline int PermutationElement(uint32_t i, uint32_t l, uint32_t p) {
    uint32_t w = l - 1;
    w |= w >> 1; w |= w >> 2; w |= w >> 4; w |= w >> 8; w |= w >> 16;
    do {
        i ^= p; i *= 0xe170893du; i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8; i *= 0x0929eb3fu;
        i ^= p >> 23; i ^= (i & w) >> 1; i *= 1u | p >> 27; i *= 0x6935fa69u; i ^= (i & w) >> 11;
        i *= 0x74dcb303u; i ^= (i & w) >> 2; i *= 0x9e501cc3u; i ^= (i & w) >> 2; i *= 0xc860a3dfu;
        i &= w; i ^= i >> 5;
    } while (i >= l);
    return (int)((i + p) % l);
}

// rng.h:19-144 — PCG32
struct RNG {
    static constexpr uint64_t DefaultState = 0x853c49e6748fea9bull;
    static constexpr uint64_t DefaultStream = 0xda3e39cb94b95bdbull;
    static constexpr uint64_t Mult = 0x5851f42d4c957f2dull;
    uint64_t state = DefaultState, inc = DefaultStream;

    uint32_t UniformU32() {  // rng.h:76-82
        uint64_t old = state;
        state = old * Mult + inc;
        uint32_t xorshifted = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xorshifted >> rot) | (xorshifted << ((~rot + 1u) & 31));
    }
    void SetSequence(uint64_t seqIndex, uint64_t seed) {  // rng.h:113-119
        state = 0u;
        inc = (seqIndex << 1u) | 1u;
        UniformU32();
        state += seed;
        UniformU32();
    }
    void SetSequence(uint64_t seqIndex) { SetSequence(seqIndex, MixBits(seqIndex)); }  // rng.h:36-39
    float UniformF() {  // rng.h:122-124 (OneMinusEpsilon == 1.0f, so the min is a no-op)
        float v = (float)UniformU32() * 0x1p-32f;
        return std::min<float>(OneMinusEpsilon, v);
    }
    void Advance(int64_t idelta) {  // rng.h:131-144
        uint64_t curMult = Mult, curPlus = inc, accMult = 1u, accPlus = 0u, delta = (uint64_t)idelta;
        while (delta > 0) {
            if (delta & 1) { accMult *= curMult; accPlus = accPlus * curMult + curPlus; }
            curPlus = (curMult + 1) * curPlus;
            curMult *= curMult;
            delta /= 2;
        }
        state = accMult * state + accPlus;
    }
};

// ============================================================================== Sobol (samplers.h:139-327)
// SobolMatrices32 is declared but never defined in the reference (HelperFunctions.h:208-210): this build generates
// 32 dimensions from the Joe-Kuo (new-joe-kuo-6.21201) direction numbers, dimension 0 = van der Corput.  The
// SobolIntervalToIndex tables are derived by GF(2) inversion; they equal the reference's VdCSobolMatrices(Inv)
// (HelperFunctions.h:212-470) for every m.
static const int NSobolDims = 32, SobolMatrixSize = 52;
struct SobolData {
    uint32_t mats[NSobolDims * SobolMatrixSize];
    uint64_t fwd[SobolMatrixSize], inv[SobolMatrixSize];
    int m = 0;
    void Build(int m_) {
        static const int JK[31][9] = {  // s, a, m_1..m_s
            {1, 0, 1}, {2, 1, 1, 3}, {3, 1, 1, 3, 1}, {3, 2, 1, 1, 1}, {4, 1, 1, 1, 3, 3}, {4, 4, 1, 3, 5, 13},
            {5, 2, 1, 1, 5, 5, 17}, {5, 4, 1, 1, 5, 5, 5}, {5, 7, 1, 1, 7, 11, 19}, {5, 11, 1, 1, 5, 1, 1},
            {5, 13, 1, 1, 1, 3, 11}, {5, 14, 1, 3, 5, 5, 31}, {6, 1, 1, 3, 3, 9, 7, 49}, {6, 13, 1, 1, 1, 15, 21, 21},
            {6, 16, 1, 3, 1, 13, 27, 49}, {6, 19, 1, 1, 1, 15, 7, 5}, {6, 22, 1, 3, 1, 15, 13, 25},
            {6, 25, 1, 1, 5, 5, 19, 61}, {7, 1, 1, 3, 7, 11, 23, 15, 103}, {7, 4, 1, 3, 7, 13, 13, 15, 69},
            {7, 7, 1, 1, 3, 13, 7, 35, 63}, {7, 8, 1, 3, 5, 9, 1, 25, 53}, {7, 14, 1, 3, 1, 13, 9, 35, 107},
            {7, 19, 1, 3, 1, 5, 27, 61, 31}, {7, 21, 1, 1, 5, 11, 19, 41, 61}, {7, 28, 1, 3, 5, 3, 3, 13, 69},
            {7, 31, 1, 1, 7, 13, 1, 19, 1}, {7, 32, 1, 3, 7, 5, 13, 19, 59}, {7, 37, 1, 1, 3, 9, 25, 29, 41},
            {7, 41, 1, 3, 5, 13, 23, 1, 55}, {7, 42, 1, 3, 7, 3, 13, 59, 17}};
        for (int j = 0; j < SobolMatrixSize; ++j) mats[j] = j < 32 ? 1u << (31 - j) : 0u;
        for (int d = 1; d < NSobolDims; ++d) {
            int s = JK[d - 1][0], a = JK[d - 1][1];
            uint64_t mm[SobolMatrixSize];
            for (int i = 0; i < s; ++i) mm[i] = (uint64_t)JK[d - 1][2 + i];
            for (int i = s; i < SobolMatrixSize; ++i) {
                uint64_t v = mm[i - s] ^ (mm[i - s] << s);
                for (int k = 1; k < s; ++k)
                    if ((a >> (s - 1 - k)) & 1) v ^= mm[i - k] << k;
                mm[i] = v;
            }
            for (int j = 0; j < SobolMatrixSize; ++j) mats[d * SobolMatrixSize + j] = (uint32_t)((mm[j] << (63 - j)) >> 32);
        }
        m = m_;
        for (int c = 0; c < SobolMatrixSize; ++c) fwd[c] = inv[c] = 0;
        if (m == 0) return;
        auto top = [&](uint32_t v) { return (uint64_t)(v >> (32 - m)); };
        int n = 2 * m;
        for (int c = 0; c + n < SobolMatrixSize; ++c) fwd[c] = (top(mats[n + c]) << m) | top(mats[SobolMatrixSize + n + c]);
        // columns j of the 2m x 2m map (index bit j -> pixel bits), inverted by Gauss-Jordan over GF(2)
        uint64_t rows[64];
        for (int r = 0; r < n; ++r) {
            uint64_t row = 0;
            for (int j = 0; j < n; ++j) {
                uint64_t colj = (top(mats[j]) << m) | top(mats[SobolMatrixSize + j]);
                row |= ((colj >> r) & 1ull) << j;
            }
            rows[r] = row | (1ull << (n + r));  // [M | I] needs 4m <= 64 bits: m <= 16
        }
        for (int col = 0; col < n; ++col) {
            int piv = col;
            while (!((rows[piv] >> col) & 1)) ++piv;
            std::swap(rows[piv], rows[col]);
            for (int r = 0; r < n; ++r)
                if (r != col && ((rows[r] >> col) & 1)) rows[r] ^= rows[col];
        }
        for (int c = 0; c < n; ++c) {
            uint64_t v = 0;
            for (int r = 0; r < n; ++r) v |= ((rows[r] >> (n + c)) & 1ull) << r;
            inv[c] = v;
        }
    }
};
// hash.h:96-104 Hash(int dimension, int seed): an 8-byte key
static inline uint64_t Hash2(int a, int b) {
    unsigned char buf[8];
    std::memcpy(buf, &a, 4); std::memcpy(buf + 4, &b, 4);
    return MurmurHash64A(buf, 8, 0);
}
static inline uint32_t ReverseBits32(uint32_t n) {  // HelperFunctions.h:154-162
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ff) << 8) | ((n & 0xff00ff00) >> 8);
    n = ((n & 0x0f0f0f0f) << 4) | ((n & 0xf0f0f0f0) >> 4);
    n = ((n & 0x33333333) << 2) | ((n & 0xcccccccc) >> 2);
    n = ((n & 0x55555555) << 1) | ((n & 0xaaaaaaaa) >> 1);
    return n;
}
// samplers.h:198-209 SobolSample with the scramblers of 147-190
static inline float SobolSampleF(const SobolData& D, int64_t a, int dimension, int randomize, uint32_t seed) {
    uint32_t v = 0;
    for (int i = dimension * SobolMatrixSize; a != 0; a >>= 1, i++)
        if (a & 1) v ^= D.mats[i];
    if (randomize == 1) {
        v ^= seed;
    } else if (randomize == 2) {
        v = ReverseBits32(v);
        v ^= v * 0x3d20adea;
        v += seed;
        v *= (seed >> 16) | 1;
        v ^= v * 0x05526c56;
        v ^= v * 0x53a22864;
        v = ReverseBits32(v);
    } else if (randomize == 3) {
        if (seed & 1) v ^= 1u << 31;
        for (int b = 1; b < 32; ++b) {
            uint32_t mask = (~0u) << (32 - b);
            if ((uint32_t)MixBits((v & mask) ^ seed) & (1u << b)) v ^= 1u << (31 - b);
        }
    }
    const float FloatOneMinusEpsilon = 0x1.fffffep-1;
    return std::min(v * 0x1p-32f, FloatOneMinusEpsilon);
}
// samplers.h:211-227 SobolIntervalToIndex
static inline uint64_t SobolIntervalToIndex(const SobolData& D, uint32_t m, uint64_t frame, int px, int py) {
    if (m == 0) return frame;
    uint64_t index = frame << (2 * m);
    uint64_t delta = 0;
    for (int c = 0; frame; frame >>= 1, ++c)
        if (frame & 1) delta ^= D.fwd[c];
    uint64_t b = (((uint64_t)((uint32_t)px) << m) | ((uint32_t)py)) ^ delta;
    for (int c = 0; b; b >>= 1, ++c)
        if (b & 1) index ^= D.inv[c];
    return index;
}

// ============================================================================== samplers
// samplers.h:38-62 IndependentSampler ; samplers.h:66-136 StratifiedSampler ; samplers.h:229-327 SobolSampler
struct Sampler {
    int kind = 1;  // 0 = Independent, 1 = Stratified, 2 = Sobol
    int xPixelSamples = 1, yPixelSamples = 1, seed = 0;
    bool jitter = false;
    RNG rng;
    int px = 0, py = 0, sampleIndex = 0, dimension = 0;
    int randomize = 0, scale = 1;                // Sobol
    int64_t sobolIndex = 0;
    std::shared_ptr<const SobolData> sobol;
    void InitSobol(int resX, int resY) {         // samplers.h:236-245: scale = RoundUpPow2(max(res))
        int v = std::max(resX, resY) - 1;
        v |= v >> 1; v |= v >> 2; v |= v >> 4; v |= v >> 8; v |= v >> 16;
        scale = v + 1;
        auto d = std::make_shared<SobolData>();
        d->Build((int)std::log2((float)scale));
        sobol = d;
    }
    float SobolDim(int dim) const {               // samplers.h:305-318 SampleDimension
        uint32_t hash = randomize == 0 ? 0u : (uint32_t)Hash2(dim, seed);
        return SobolSampleF(*sobol, sobolIndex, dim, randomize, hash);
    }

    int SamplesPerPixel() const { return kind == 0 ? xPixelSamples : xPixelSamples * yPixelSamples; }
    // returns false where the reference prints "more sampels than pixels for strat" and keeps stale state
    bool StartPixelSample(int x, int y, int index, int dim) {
        if (kind == 2) {  // samplers.h:258-263
            px = x; py = y; sampleIndex = index;
            dimension = std::max(2, dim);
            sobolIndex = (int64_t)SobolIntervalToIndex(*sobol, (uint32_t)sobol->m, (uint64_t)index, x, y);
            return true;
        }
        if (kind == 1 && jitter == false && index >= SamplesPerPixel()) return false;  // samplers.h:83-87
        px = x; py = y; sampleIndex = index; dimension = dim;
        rng.SetSequence(Hash(x, y, seed));
        rng.Advance((int64_t)((uint64_t)index * 65536ull + (uint64_t)dim));
        return true;
    }
    float Get1D() {
        if (kind == 0) return rng.UniformF();
        if (kind == 2) {  // samplers.h:266-271
            if (dimension >= NSobolDims) dimension = 2;
            return SobolDim(dimension++);
        }
        uint64_t hash = Hash(px, py, dimension, seed);                                     // samplers.h:98
        int stratum = PermutationElement((uint32_t)sampleIndex, (uint32_t)SamplesPerPixel(), (uint32_t)hash);
        ++dimension;
        float delta = jitter ? rng.UniformF() : 0.5f;
        return ((float)stratum + delta) / (float)SamplesPerPixel();
    }
    vec2 Get2D() {
        if (kind == 0) { float a = rng.UniformF(); float b = rng.UniformF(); return {a, b}; }
        if (kind == 2) {  // samplers.h:274-281
            if (dimension + 1 >= NSobolDims) dimension = 2;
            vec2 u = {SobolDim(dimension), SobolDim(dimension + 1)};
            dimension += 2;
            return u;
        }
        if (sampleIndex >= SamplesPerPixel()) return {0, 0};                                // samplers.h:109-112
        uint64_t hash = Hash(px, py, dimension, seed);
        int stratum = PermutationElement((uint32_t)sampleIndex, (uint32_t)SamplesPerPixel(), (uint32_t)hash);
        dimension += 2;
        int x = stratum % xPixelSamples, y = stratum / xPixelSamples;
        float dx = jitter ? rng.UniformF() : 0.5f;
        float dy = jitter ? rng.UniformF() : 0.5f;
        return {((float)x + dx) / (float)xPixelSamples, ((float)y + dy) / (float)yPixelSamples};
    }
    vec2 GetPixel2D() {
        if (kind != 2) return Get2D();
        // samplers.h:283-297: un-randomised dimensions 0 and 1, remapped into the pixel (clamped to [0, 1])
        float u[2] = {SobolSampleF(*sobol, sobolIndex, 0, 0, 0), SobolSampleF(*sobol, sobolIndex, 1, 0, 0)};
        float p[2] = {(float)px, (float)py};
        for (int d = 0; d < 2; ++d) u[d] = gclamp(u[d] * (float)scale - p[d], 0.0f, OneMinusEpsilon);
        return {u[0], u[1]};
    }
};

// ============================================================================ sampling
// Sampling.h:63-67
static inline float VisibleWavelengthsPDF(float lambda) {
    if (lambda < 360 || lambda > 830) return 0;
    float c = cosh_f(0.0072f * (lambda - 538));
    return (float)((double)0.0039398042f / ((double)c * (double)c));
}
// Sampling.h:69-71
static inline float SampleVisibleWavelengths(float u) {
    return 538 - 138.888889f * atanh_f(0.85691062f - 1.82750197f * u);
}
// Sampling.h:205-211
static inline float SampleLinear(float u, float a, float b) {
    if (u == 0 && a == 0) return 0;
    float x = (u * (a + b)) / (a + std::sqrt(Lerp(u, a * a, b * b)));
    return std::min(x, OneMinusEpsilon);
}
// Sampling.h:228-235 with the coin taken deterministically from u (pbrt-v4 SampleDiscrete remap) instead
// of the global mt19937 (non-deterministic in the reference) — build-defined, documented.
static inline float SampleTentDet(float u, float r) {
    if (u < 0.5f) {
        float up = std::min(u * 2.0f, OneMinusEpsilon);
        return -r + r * SampleLinear(up, 0, 1);
    }
    float up = std::min((u - 0.5f) * 2.0f, OneMinusEpsilon);
    return r * SampleLinear(up, 1, 0);
}
// Sampling.h:383-403
static inline vec2 SampleUniformDiskConcentric(vec2 u) {
    vec2 o = {2.0f * u.x - 1.0f, 2.0f * u.y - 1.0f};
    if (o.x == 0 && o.y == 0) return {0, 0};
    float theta, r;
    if (std::fabs(o.x) > std::fabs(o.y)) { r = o.x; theta = PiOver4 * (o.y / o.x); }
    else { r = o.y; theta = PiOver2 - PiOver4 * (o.x / o.y); }
    return {r * cos_f(theta), r * sin_f(theta)};
}
// Sampling.h:449-454 (+ HelperFunctions SafeSqrt)
static inline vec3 SampleCosineHemisphere(vec2 u) {
    vec2 d = SampleUniformDiskConcentric(u);
    float z = std::sqrt(std::max(0.f, 1 - d.x * d.x - d.y * d.y));
    return {d.x, d.y, z};
}

// ============================================================================ spectra
// spectrum.h:458-496 / spectrum.cpp:60-71 PiecewiseLinearSpectrum
struct Piecewise {
    std::vector<float> lambdas, values;
    float Query(float lambda) const {
        if (lambdas.empty() || lambda < lambdas.front() || lambda > lambdas.back()) return 0;
        int o = (int)FindInterval(lambdas.size(), [&](int i) { return lambdas[i] <= lambda; });
        float t = (lambda - lambdas[o]) / (lambdas[o + 1] - lambdas[o]);
        return Lerp(t, values[o], values[o + 1]);
    }
};
// spectrum.h:376-456 DenselySampledSpectrum (lambda_min 360, lambda_max 830)
struct Dense {
    int lambda_min = 360, lambda_max = 830;
    std::vector<float> values;
    float Query(float lambda) const {  // spectrum.h:430-437 / Sample 386-398
        long offset = std::lround(lambda) - lambda_min;
        if (offset < 0 || offset >= (long)values.size()) return 0;
        return values[(size_t)offset];
    }
};
template <typename S>
static inline Dense MakeDense(const S& s) {  // spectrum.h:412-419
    Dense d;
    d.values.resize(471);
    for (int lambda = 360; lambda <= 830; ++lambda) d.values[lambda - 360] = s.Query((float)lambda);
    return d;
}
// spectrum.h:762-768 InnerProduct (float loop variable, sequential float sum)
template <typename F, typename G>
static inline float InnerProduct(const F& f, const G& g) {
    float integral = 0;
    for (float lambda = 360; lambda <= 830; ++lambda) integral += f.Query(lambda) * g.Query(lambda);
    return integral;
}
struct Spectra {
    Dense X, Y, Z;
    Piecewise D65, F1;   // normalized (FromInterleaved(..., true))
    Dense D65dense;      // RGBColorSpace::illuminant (colorspace.cpp:13-14 → spectrum.h:412-419)
    Piecewise FromInterleaved(const float* s, int n, bool normalize) const {  // spectrum.cpp:134-165
        Piecewise p;
        int half = n / 2;
        if (s[0] > 360) { p.lambdas.push_back(360 - 1); p.values.push_back(s[1]); }
        for (int i = 0; i < half; ++i) { p.lambdas.push_back(s[2 * i]); p.values.push_back(s[2 * i + 1]); }
        if (p.lambdas.back() < 830) { p.lambdas.push_back(830 + 1); p.values.push_back(p.values.back()); }
        if (normalize) {
            float scale = CIE_Y_integral / InnerProduct(p, Y);
            for (float& v : p.values) v *= scale;   // spectrum.h:464-468 Scale
        }
        return p;
    }
    void Init() {  // spectrum.cpp:2612-2622 (X/Y/Z dense from piecewise over CIE_lambda), 2624-2634
        auto dense_from_table = [](const float* vals) {
            Piecewise p;
            for (int i = 0; i < 471; ++i) { p.lambdas.push_back(rtdata::cie_lambda[i]); p.values.push_back(vals[i]); }
            return MakeDense(p);
        };
        X = dense_from_table(rtdata::cie_x);
        Y = dense_from_table(rtdata::cie_y);
        Z = dense_from_table(rtdata::cie_z);
        D65 = FromInterleaved(rtdata::illum_d65, rtdata::illum_d65_n, true);
        F1 = FromInterleaved(rtdata::illum_f1, rtdata::illum_f1_n, true);
        D65dense = MakeDense(D65);
        SR = X; SG = Y; SB = Z;
    }
    Dense SR, SG, SB;    // the film's PixelSensor r_bar, g_bar, b_bar (XYZ sensor: X, Y, Z)
};

// Spectra::Init named illuminants (spectrum.cpp:2620-2637, normalized): RT_ILLUM_* order
static inline Piecewise NamedIlluminant(const Spectra& sp, int which) {
    switch (which) {
        case 1: return sp.FromInterleaved(rtdata::illum_a, rtdata::illum_a_n, true);
        case 2: return sp.FromInterleaved(rtdata::illum_d50, rtdata::illum_d50_n, true);
        case 3: return sp.FromInterleaved(rtdata::illum_f1, rtdata::illum_f1_n, true);
        case 4: return sp.FromInterleaved(rtdata::illum_f2, rtdata::illum_f2_n, true);
        case 5: return sp.FromInterleaved(rtdata::illum_f3, rtdata::illum_f3_n, true);
        case 6: return sp.FromInterleaved(rtdata::illum_f4, rtdata::illum_f4_n, true);
        case 7: return sp.FromInterleaved(rtdata::illum_f5, rtdata::illum_f5_n, true);
        case 8: return sp.FromInterleaved(rtdata::illum_f6, rtdata::illum_f6_n, true);
        case 9: return sp.FromInterleaved(rtdata::illum_f7, rtdata::illum_f7_n, true);
        case 10: return sp.FromInterleaved(rtdata::illum_f8, rtdata::illum_f8_n, true);
        case 11: return sp.FromInterleaved(rtdata::illum_f9, rtdata::illum_f9_n, true);
        case 12: return sp.FromInterleaved(rtdata::illum_f10, rtdata::illum_f10_n, true);
        case 13: return sp.FromInterleaved(rtdata::illum_f11, rtdata::illum_f11_n, true);
        case 14: return sp.FromInterleaved(rtdata::illum_f12, rtdata::illum_f12_n, true);
        case 15: return sp.FromInterleaved(rtdata::illum_aces_d60, rtdata::illum_aces_d60_n, true);
        default: return sp.D65;
    }
}

// pixelsensor.h:104-117 PixelSensor::ProjectReflectance
template <class R, class I, class B1, class B2, class B3>
static inline vec3 ProjectReflectance(const R& refl, const I& illum, const B1& b1, const B2& b2, const B3& b3) {
    vec3 result{0, 0, 0};
    float g_integral = 0;
    for (float lambda = 360; lambda <= 830; ++lambda) {
        g_integral += b2.Query(lambda) * illum.Query(lambda);
        result.x += b1.Query(lambda) * refl.Query(lambda) * illum.Query(lambda);
        result.y += b2.Query(lambda) * refl.Query(lambda) * illum.Query(lambda);
        result.z += b3.Query(lambda) * refl.Query(lambda) * illum.Query(lambda);
    }
    return vec3{result.x / g_integral, result.y / g_integral, result.z / g_integral};
}

// 8-wavelength sampled values (spectrum.h:52-343)
struct SW { float lambda[8], pdf[8]; };
struct SS { float v[8]; };
// spectrum.h:322-336 SampledWavelengths::SampleVisible
static inline SW SampleVisible(float u) {
    SW s;
    for (int i = 0; i < NSpectrumSamples; ++i) {
        float up = u + float(i) / NSpectrumSamples;
        if (up > 1) up -= 1;
        s.lambda[i] = SampleVisibleWavelengths(up);
        s.pdf[i] = VisibleWavelengthsPDF(s.lambda[i]);
    }
    return s;
}
// color.h:373-399 RGBSigmoidPolynomial (EvaluatePolynomial via FMA, helpers.h:117-126)
struct Sigmoid {
    float c0 = 0, c1 = 0, c2 = 0;
    static float s(float x) {
        if (std::isinf(x)) return x > 0 ? 1 : 0;
        return .5f + x / (2 * std::sqrt(1 + (x * x)));
    }
    float operator()(float lambda) const { return s(std::fmaf(lambda, std::fmaf(lambda, c0, c1), c2)); }
};
// color.cpp:35-37 uniform-RGB branch of RGBToSpectrumTable (the only branch usable without the missing table)
static inline Sigmoid SigmoidFromGrey(float g) { return {0, 0, (g - .5f) / std::sqrt(g * (1 - g))}; }
// color.cpp:26-72 RGBToSpectrumTable::operator() over a table in the layout Init reads (color.cpp:107-171):
// zNodes[res], coeffs[3][res][res][res][3] (the build regenerates the missing file, tools/rgb2spec_gen.cpp)
static inline Sigmoid RGBToSpectrumTableLookup(const float* zNodes, const float* coeffs, int res, const float rgb[3]) {
    if (rgb[0] == rgb[1] && rgb[1] == rgb[2]) return SigmoidFromGrey(rgb[0]);
    int maxc = (rgb[0] > rgb[1]) ? ((rgb[0] > rgb[2]) ? 0 : 2) : ((rgb[1] > rgb[2]) ? 1 : 2);
    float z = rgb[maxc];
    float x = rgb[(maxc + 1) % 3] * (res - 1) / z;
    float y = rgb[(maxc + 2) % 3] * (res - 1) / z;
    int xi = std::min((int)x, res - 2), yi = std::min((int)y, res - 2);
    int zi = (int)FindInterval(res, [&](int i) { return zNodes[i] < z; });
    float dx = x - xi, dy = y - yi, dz = (z - zNodes[zi]) / (zNodes[zi + 1] - zNodes[zi]);
    float c[3];
    for (int i = 0; i < 3; ++i) {
        auto co = [&](int ox, int oy, int oz) {
            return coeffs[(size_t)maxc * 64 * 64 * 64 * 3 + (size_t)(zi + oz) * 64 * 64 * 3 + (size_t)(yi + oy) * 64 * 3 +
                          (size_t)(xi + ox) * 3 + i];
        };
        c[i] = Lerp(dz, Lerp(dy, Lerp(dx, co(0, 0, 0), co(1, 0, 0)), Lerp(dx, co(0, 1, 0), co(1, 1, 0))),
                    Lerp(dy, Lerp(dx, co(0, 0, 1), co(1, 0, 1)), Lerp(dx, co(0, 1, 1), co(1, 1, 1))));
    }
    return {c[0], c[1], c[2]};
}

// pixelsensor.h:81-87 ToSensorRGB (XYZ sensor: r_bar=X, g_bar=Y, b_bar=Z), imagingRatio = 1/CIE_Y_integral
static inline void ToSensorRGB(const Spectra& sp, SS L, const SW& w, float imagingRatio, float rgb[3]) {
    for (int i = 0; i < 8; ++i) L.v[i] = (w.pdf[i] != 0) ? L.v[i] / w.pdf[i] : 0.f;  // spectrum.h:643-649
    const Dense* bars[3] = {&sp.SR, &sp.SG, &sp.SB};
    for (int c = 0; c < 3; ++c) {
        float prod[8];
        for (int i = 0; i < 8; ++i) prod[i] = bars[c]->Query(w.lambda[i]) * L.v[i];
        float sum = prod[0];                                   // spectrum.h:238-244 Average
        for (int i = 1; i < 8; ++i) sum += prod[i];
        rgb[c] = imagingRatio * (sum / 8);
    }
}

// ============================================================================== geometry
struct Ray { vec3 o, d; };
// Shapes.h:37-41 Ray::Transform
static inline Ray TransformRay(Ray r, const mat4& M) {
    vec4 o4 = mul(M, vec4{r.o.x, r.o.y, r.o.z, 1});
    vec4 d4 = normalize4(mul(M, vec4{r.d.x, r.d.y, r.d.z, 0}));
    return {{o4.x, o4.y, o4.z}, {d4.x, d4.y, d4.z}};
}
struct Bounds3 { vec3 pmin, pmax; };
// Shapes.h:100-124 Bounds3::IntersectP
static inline bool IntersectP(const Bounds3& b, const Ray& ray, float tMax) {
    float min_t = 0, max_t = tMax;
    const float g3 = 1 + 2 * gamma_(3);
    for (int i = 0; i < 3; ++i) {
        float invRayDir = 1 / ray.d[i];
        float tNear = ((i == 0 ? b.pmin.x : i == 1 ? b.pmin.y : b.pmin.z) - ray.o[i]) * invRayDir;
        float tFar = ((i == 0 ? b.pmax.x : i == 1 ? b.pmax.y : b.pmax.z) - ray.o[i]) * invRayDir;
        if (tNear > tFar) std::swap(tNear, tFar);
        tFar *= g3;
        min_t = tNear > min_t ? tNear : min_t;
        max_t = tFar < max_t ? tFar : max_t;
        if (min_t > max_t) return false;
    }
    return true;
}

struct TriIsect { float b0, b1, b2, t; };
// Shapes.h:1101-1260 Triangle::BasicIntersect — pbrt-v4 watertight test on world-space vertices
static inline bool BasicIntersect(vec3 p0w, vec3 p1w, vec3 p2w, const Ray& ray, float tMax, TriIsect* out) {
    // Shapes.h:1131 degenerate: pow(length(cross),2) == 0  <=>  dot(c,c) == 0
    vec3 c = cross(sub(p2w, p0w), sub(p1w, p0w));
    if (dot(c, c) == 0) return false;
    vec3 p0t = sub(p0w, ray.o), p1t = sub(p1w, ray.o), p2t = sub(p2w, ray.o);
    vec3 ad = {std::fabs(ray.d.x), std::fabs(ray.d.y), std::fabs(ray.d.z)};
    int kz = MaxComponentIndex(ad);
    int kx = kz + 1; if (kx == 3) kx = 0;
    int ky = kx + 1; if (ky == 3) ky = 0;
    vec3 d = {ray.d[kx], ray.d[ky], ray.d[kz]};
    p0t = {p0t[kx], p0t[ky], p0t[kz]};
    p1t = {p1t[kx], p1t[ky], p1t[kz]};
    p2t = {p2t[kx], p2t[ky], p2t[kz]};
    float Sx = -d.x / d.z, Sy = -d.y / d.z, Sz = 1 / d.z;
    p0t.x += Sx * p0t.z; p0t.y += Sy * p0t.z;
    p1t.x += Sx * p1t.z; p1t.y += Sy * p1t.z;
    p2t.x += Sx * p2t.z; p2t.y += Sy * p2t.z;
    float e0 = DifferenceOfProducts(p1t.x, p2t.y, p1t.y, p2t.x);
    float e1 = DifferenceOfProducts(p2t.x, p0t.y, p2t.y, p0t.x);
    float e2 = DifferenceOfProducts(p0t.x, p1t.y, p0t.y, p1t.x);
    if (e0 == 0.0f || e1 == 0.0f || e2 == 0.0f) {  // Shapes.h:1174-1184 double fallback
        double p2txp1ty = (double)p2t.x * (double)p1t.y, p2typ1tx = (double)p2t.y * (double)p1t.x;
        e0 = (float)(p2typ1tx - p2txp1ty);
        double p0txp2ty = (double)p0t.x * (double)p2t.y, p0typ2tx = (double)p0t.y * (double)p2t.x;
        e1 = (float)(p0typ2tx - p0txp2ty);
        double p1txp0ty = (double)p1t.x * (double)p0t.y, p1typ0tx = (double)p1t.y * (double)p0t.x;
        e2 = (float)(p1typ0tx - p1txp0ty);
    }
    if ((e0 < 0 || e1 < 0 || e2 < 0) && (e0 > 0 || e1 > 0 || e2 > 0)) return false;
    float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0t.z *= Sz; p1t.z *= Sz; p2t.z *= Sz;
    float tScaled = e0 * p0t.z + e1 * p1t.z + e2 * p2t.z;
    if (det < 0 && (tScaled >= 0 || tScaled < tMax * det)) return false;
    else if (det > 0 && (tScaled <= 0 || tScaled > tMax * det)) return false;
    float invDet = 1 / det;
    float b0 = e0 * invDet, b1 = e1 * invDet, b2 = e2 * invDet;
    float t = tScaled * invDet;
    if (std::isnan(t)) return false;
    float maxZt = MaxComponentValue({std::fabs(p0t.z), std::fabs(p1t.z), std::fabs(p2t.z)});
    float deltaZ = gamma_(3) * maxZt;
    float maxXt = MaxComponentValue({std::fabs(p0t.x), std::fabs(p1t.x), std::fabs(p2t.x)});
    float maxYt = MaxComponentValue({std::fabs(p0t.y), std::fabs(p1t.y), std::fabs(p2t.y)});
    float deltaX = gamma_(5) * (maxXt + maxZt);
    float deltaY = gamma_(5) * (maxYt + maxZt);
    float deltaE = 2 * (gamma_(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    float maxE = MaxComponentValue({std::fabs(e0), std::fabs(e1), std::fabs(e2)});
    float deltaT = 3 * (gamma_(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * std::fabs(invDet);
    if (t <= deltaT) return false;
    *out = {b0, b1, b2, t};
    return true;
}

// ------------------------------------------------------------------ Möller triangle/box overlap
// AABB_triangle_Moller.h:187-474 (incl. the AxisTest_Z0 quirk at :342 that never rejects)
static inline void FindMinMax(float x0, float x1, float x2, float& mn, float& mx) {
    mn = mx = x0;
    if (x1 < mn) mn = x1;
    if (x1 > mx) mx = x1;
    if (x2 < mn) mn = x2;
    if (x2 > mx) mx = x2;
}
static inline int planeBoxOverlap(vec3 normal, vec3 vert, vec3 maxbox) {
    float vmin[3], vmax[3];
    for (int q = 0; q <= 2; ++q) {
        float v = vert[q], n = normal[q], mb = maxbox[q];
        if (n > 0.0f) { vmin[q] = -mb - v; vmax[q] = mb - v; }
        else { vmin[q] = mb - v; vmax[q] = -mb - v; }
    }
    if (dot(normal, {vmin[0], vmin[1], vmin[2]}) > 0.0f) return 0;
    if (dot(normal, {vmax[0], vmax[1], vmax[2]}) >= 0.0f) return 1;
    return 0;
}
static inline bool triBoxOverlap(vec3 boxcenter, vec3 bh, vec3 t0, vec3 t1, vec3 t2) {
    vec3 v0 = sub(t0, boxcenter), v1 = sub(t1, boxcenter), v2 = sub(t2, boxcenter);
    vec3 e0 = sub(v1, v0), e1 = sub(v2, v1), e2 = sub(v0, v2);
    float mn, mx, p0, p1, p2, rad;
    auto X01 = [&](float a, float b, float fa, float fb) {
        p0 = a * v0.y - b * v0.z; p2 = a * v2.y - b * v2.z;
        if (p0 < p2) { mn = p0; mx = p2; } else { mn = p2; mx = p0; }
        rad = fa * bh.y + fb * bh.z;
        return !(mn > rad || mx < -rad);
    };
    auto X2 = [&](float a, float b, float fa, float fb) {
        p0 = a * v0.y - b * v0.z; p1 = a * v1.y - b * v1.z;
        if (p0 < p1) { mn = p0; mx = p1; } else { mn = p1; mx = p0; }
        rad = fa * bh.y + fb * bh.z;
        return !(mn > rad || mx < -rad);
    };
    auto Y02 = [&](float a, float b, float fa, float fb) {
        p0 = -a * v0.x + b * v0.z; p2 = -a * v2.x + b * v2.z;
        if (p0 < p2) { mn = p0; mx = p2; } else { mn = p2; mx = p0; }
        rad = fa * bh.x + fb * bh.z;
        return !(mn > rad || mx < -rad);
    };
    auto Y1 = [&](float a, float b, float fa, float fb) {
        p0 = -a * v0.x + b * v0.z; p1 = -a * v1.x + b * v1.z;
        if (p0 < p1) { mn = p0; mx = p1; } else { mn = p1; mx = p0; }
        rad = fa * bh.x + fb * bh.z;
        return !(mn > rad || mx < -rad);
    };
    auto Z0 = [&](float a, float b, float fa, float fb) {  // :334-345 — returns true on both paths
        p0 = a * v0.x - b * v0.y; p1 = a * v1.x - b * v1.y;
        if (p0 < p1) { mn = p0; mx = p1; } else { mn = p1; mx = p0; }
        rad = fa * bh.x + fb * bh.y;
        return true;
    };
    auto Z12 = [&](float a, float b, float fa, float fb) {
        p1 = a * v1.x - b * v1.y; p2 = a * v2.x - b * v2.y;
        if (p2 < p1) { mn = p2; mx = p1; } else { mn = p1; mx = p2; }
        rad = fa * bh.x + fb * bh.y;
        return !(mn > rad || mx < -rad);
    };
    float fex = std::fabs(e0.x), fey = std::fabs(e0.y), fez = std::fabs(e0.z);
    if (!X01(e0.z, e0.y, fez, fey)) return false;
    if (!Y02(e0.z, e0.x, fez, fex)) return false;
    if (!Z12(e0.y, e0.x, fey, fex)) return false;
    fex = std::fabs(e1.x); fey = std::fabs(e1.y); fez = std::fabs(e1.z);
    if (!X01(e1.z, e1.y, fez, fey)) return false;
    if (!Y02(e1.z, e1.x, fez, fex)) return false;
    if (!Z0(e1.y, e1.x, fey, fex)) return false;
    fex = std::fabs(e2.x); fey = std::fabs(e2.y); fez = std::fabs(e2.z);
    if (!X2(e2.z, e2.y, fez, fey)) return false;
    if (!Y1(e2.z, e2.x, fez, fex)) return false;
    if (!Z12(e2.y, e2.x, fey, fex)) return false;
    FindMinMax(v0.x, v1.x, v2.x, mn, mx);
    if (mn > bh.x || mx < -bh.x) return false;
    FindMinMax(v0.y, v1.y, v2.y, mn, mx);
    if (mn > bh.y || mx < -bh.y) return false;
    FindMinMax(v0.z, v1.z, v2.z, mn, mx);
    if (mn > bh.z || mx < -bh.z) return false;
    vec3 normal = cross(e0, e1);
    if (!planeBoxOverlap(normal, v0, bh)) return false;
    return true;
}

// ------------------------------------------------------------------------------ TriModel
// Shapes.h:1272-1491 + 913-1083 (one mesh).  Positions/normals are object space; ObjectToRender is
// rigidtransform * permutation_y_z (Shapes.h:175-181), provided by the caller.
struct TriModel {
    std::vector<vec3> pos, nrm;         // object space
    std::vector<uint32_t> idx;          // 3 per triangle
    mat4 objectToRender;
    mat3 normalToRender;                // mat3(transpose(inverse(ObjectToRender))), caller-provided
    std::vector<vec3> wpos;             // ObjectToRender * p (per vertex; = per-test transform Shapes.h:1119)
    std::vector<uint8_t> back_facing;   // ComputeBackFace flags (empty when culling disabled)
    bool cull = false;
    size_t ntri() const { return idx.size() / 3; }
    void Prepare() {
        wpos.resize(pos.size());
        for (size_t i = 0; i < pos.size(); ++i) {
            vec4 w = mul(objectToRender, vec4{pos[i].x, pos[i].y, pos[i].z, 1});
            wpos[i] = {w.x, w.y, w.z};
        }
    }
    vec3 P(size_t t, int k) const { return wpos[idx[3 * t + k]]; }
    // Shapes.h:1339-1380 ComputeBackFace
    void ComputeBackFace(vec3 look, bool enable) {
        cull = enable;
        back_facing.clear();
        if (!enable) return;
        vec3 look_dir = normalize(look);
        back_facing.resize(ntri());
        for (size_t t = 0; t < ntri(); ++t) {
            vec3 n1 = nrm[idx[3 * t]], n2 = nrm[idx[3 * t + 1]], n3 = nrm[idx[3 * t + 2]];
            vec3 s = add(add(n1, n2), n3);
            vec3 N = normalize({s.x / 3.0f, s.y / 3.0f, s.z / 3.0f});
            N = normalize(mul(normalToRender, N));
            back_facing[t] = dot(look_dir, N) > 0 ? 1 : 0;
        }
    }
    // Shapes.h:1390-1397 Bounds(): object-space min/max (max initialised with FLT_MIN — quirk, :1292)
    // transformed by Bounds3::Transform (Shapes.h:60-98, same FLT_MIN quirk at :80-82)
    Bounds3 Bounds() const {
        vec3 mn = {std::numeric_limits<float>::max(), std::numeric_limits<float>::max(), std::numeric_limits<float>::max()};
        vec3 mx = {std::numeric_limits<float>::min(), std::numeric_limits<float>::min(), std::numeric_limits<float>::min()};
        for (const vec3& p : pos) {
            mn.x = std::min(mn.x, p.x); mn.y = std::min(mn.y, p.y); mn.z = std::min(mn.z, p.z);
            mx.x = std::max(mx.x, p.x); mx.y = std::max(mx.y, p.y); mx.z = std::max(mx.z, p.z);
        }
        vec3 corners[8] = {{mn.x, mn.y, mn.z}, {mn.x, mx.y, mn.z}, {mn.x, mx.y, mx.z}, {mn.x, mn.y, mx.z},
                           {mx.x, mx.y, mx.z}, {mx.x, mn.y, mx.z}, {mx.x, mn.y, mn.z}, {mx.x, mx.y, mn.z}};
        float xm = std::numeric_limits<float>::max(), xM = std::numeric_limits<float>::min();
        float ym = xm, yM = xM, zm = xm, zM = xM;
        for (auto& c : corners) {
            vec4 w = mul(objectToRender, vec4{c.x, c.y, c.z, 1});
            xm = std::min(xm, w.x); xM = std::max(xM, w.x);
            ym = std::min(ym, w.y); yM = std::max(yM, w.y);
            zm = std::min(zm, w.z); zM = std::max(zM, w.z);
        }
        return {{xm, ym, zm}, {xM, yM, zM}};
    }
};

// --------------------------------------------------------------------------- Octtree_Model
// Octtree_Model.h:9-388
struct Octree {
    struct Node {
        Bounds3 bounds;
        std::vector<int> tris;
        bool leaf = true;
        int parent = -1;
        std::vector<int> child;
    };
    static const int TRIANGLE_CAPACITY_DEFAULT = 40;  // Octtree_Model.h:388
    int capacity = TRIANGLE_CAPACITY_DEFAULT;
    std::vector<Node> nodes;
    const TriModel* model = nullptr;

    // Octtree_Model.h:361-367
    bool triBounds(vec3 p0, vec3 p1, vec3 p2, const Bounds3& b) const {
        vec3 half = {(b.pmax.x - b.pmin.x) / 2.0f, (b.pmax.y - b.pmin.y) / 2.0f, (b.pmax.z - b.pmin.z) / 2.0f};
        vec3 C = add(b.pmin, half);
        return triBoxOverlap(C, half, p0, p1, p2);
    }
    // Octtree_Model.h:279-358
    void Split(int id) {
        Bounds3 B = nodes[id].bounds;
        float padding = 0.01f;
        vec3 half = {(B.pmax.x - B.pmin.x) / 2.0f, (B.pmax.y - B.pmin.y) / 2.0f, (B.pmax.z - B.pmin.z) / 2.0f};
        vec3 C = add(B.pmin, half);
        half = add(half, {padding, padding, padding});
        auto box = [&](vec3 a, vec3 b) { return Bounds3{add(C, a), add(C, b)}; };
        Bounds3 bb[8] = {
            box({-half.x, 0, -half.z}, {0, half.y, 0}),      box({0, 0, -half.z}, {half.x, half.y, 0}),
            box({-half.x, 0, 0}, {0, half.y, half.z}),       box({0, 0, 0}, {half.x, half.y, half.z}),
            box({-half.x, -half.y, -half.z}, {0, 0, 0}),     box({0, -half.y, -half.z}, {half.x, 0, 0}),
            box({-half.x, -half.y, 0}, {0, 0, half.z}),      box({0, -half.y, 0}, {half.x, 0, half.z})};
        Node nn[8];
        for (int n = 0; n < 8; ++n) nn[n].bounds = bb[n];
        for (int t : nodes[id].tris)
            for (int n = 0; n < 8; ++n)
                if (triBounds(model->P(t, 0), model->P(t, 1), model->P(t, 2), nn[n].bounds)) nn[n].tris.push_back(t);
        int cnt = (int)nodes[id].tris.size();
        for (int n = 0; n < 8; ++n)
            if ((int)nn[n].tris.size() == cnt) return;  // abort rule :331-340
        nodes[id].child.clear();
        for (int n = 0; n < 8; ++n) {
            nn[n].parent = id;
            nodes.push_back(nn[n]);
            nodes[id].child.push_back((int)nodes.size() - 1);
        }
        nodes[id].tris.clear();
        nodes[id].leaf = false;
    }
    // Octtree_Model.h:180-277
    void AddTriangle(int t) {
        vec3 p0 = model->P(t, 0), p1 = model->P(t, 1), p2 = model->P(t, 2);
        std::queue<int> q;
        q.push(0);
        while (!q.empty()) {
            int cur = q.front(); q.pop();
            if (triBounds(p0, p1, p2, nodes[cur].bounds)) {
                if (nodes[cur].leaf) {
                    nodes[cur].tris.push_back(t);
                    if ((int)nodes[cur].tris.size() >= capacity) Split(cur);
                } else {
                    for (int i = 0; i < 8; ++i) q.push(nodes[cur].child[i]);
                }
            }
        }
    }
    // Octtree_Model.h:33-63
    void Create(const TriModel& m, int cap = TRIANGLE_CAPACITY_DEFAULT) {
        model = &m;
        capacity = cap;
        nodes.clear();
        Node root;
        root.bounds = m.Bounds();
        root.parent = 0;
        nodes.push_back(root);
        for (size_t t = 0; t < m.ntri(); ++t) AddTriangle((int)t);
    }

    struct Hit { int tri = -1; TriIsect isect{}; long nodes_tested = 0, tris_tested = 0; };
    // The BFS queue of Traverse / Occluded: std::queue's FIFO order (Octtree_Model.h:70-75) over one buffer per host
    // thread, reused from ray to ray.  A std::queue per ray allocates a deque block on every call, and the CPU
    // baseline's threads then contend in malloc (bench.py cpu_baseline); the visiting order is unchanged.
    struct Fifo {
        std::vector<int> v;
        size_t h = 0;
        void push(int x) { v.push_back(x); }
        bool empty() const { return h == v.size(); }
        int pop() { return v[h++]; }
    };
    static Fifo& fifo(int which) {
        thread_local Fifo f[2];
        f[which].v.clear();
        f[which].h = 0;
        return f[which];
    }
    // Octtree_Model.h:66-127 Traverse — BFS with a shrinking tMax, first hit in BFS order wins ties
    Hit Traverse(const Ray& ray, bool use_cull) const {
        Hit h;
        float tMax = std::numeric_limits<float>::max();
        Fifo& q = fifo(0);
        q.push(0);
        while (!q.empty()) {
            int cur = q.pop();
            ++h.nodes_tested;
            if (IntersectP(nodes[cur].bounds, ray, tMax)) {
                if (nodes[cur].leaf) {
                    for (int t : nodes[cur].tris) {
                        if (use_cull && model->cull && !model->back_facing.empty() && model->back_facing[t]) continue;
                        ++h.tris_tested;
                        TriIsect is;
                        if (BasicIntersect(model->P(t, 0), model->P(t, 1), model->P(t, 2), ray, tMax, &is)) {
                            if (is.t < tMax) { tMax = is.t; h.tri = t; h.isect = is; }
                        }
                    }
                } else {
                    for (int i = 0; i < 8; ++i) q.push(nodes[cur].child[i]);
                }
            }
        }
        return h;
    }
    // any-hit with a fixed tMax (path mode shadow rays, build-defined): order-independent answer
    bool Occluded(const Ray& ray, float tMax) const {
        Fifo& q = fifo(1);
        q.push(0);
        while (!q.empty()) {
            int cur = q.pop();
            if (!IntersectP(nodes[cur].bounds, ray, tMax)) continue;
            if (nodes[cur].leaf) {
                for (int t : nodes[cur].tris) {
                    TriIsect is;
                    if (BasicIntersect(model->P(t, 0), model->P(t, 1), model->P(t, 2), ray, tMax, &is) && is.t < tMax)
                        return true;
                }
            } else {
                for (int i = 0; i < 8; ++i) q.push(nodes[cur].child[i]);
            }
        }
        return false;
    }

    // ---- Canonical (order-independent) rule of the GPU's fast traversal.
    // NOT the reference's algorithm: this restates the rule the GPU applies while walking its own BVH, so a CPU test
    // can check, over millions of rays, that it always returns what Traverse / Occluded return.
    //  * closest hit: t1 = the smallest t of any triangle passing the watertight test (any tMax above it), t2 the
    //    next distinct triangle's; pruning with cut = t1 + 2 W(t1) is conservative (a triangle's hit point lies in
    //    a leaf whose box the ray enters before that t).  If t2 > t1 + W(t1) the BFS must accept t1's triangle, with
    //    the same (b, t), and nothing after it (every other hit is > W farther: the scaled tMax test and t < tMax
    //    decide robustly); otherwise the ray is *ambiguous* and the caller runs the reference BFS.
    //  * any hit (fixed tMax): a passing triangle with t < tMax - W(tMax) proves the BFS finds an occluder (its hit
    //    leaf is entered before tMax); passing triangles only inside [tMax - W, tMax) are ambiguous -> BFS.
    // W(t) = t 2^-16 + wabs, wabs = max |world coordinate| 2^-20: far above the few-ulp rounding of t and of the
    // box entry distances, far below any real gap between distinct surfaces (Cornell light to ceiling: 0.1).
    float wabs = 0;
    static float Window(float t, float wabs) { return t * 0x1p-16f + wabs; }
    void SetWindow() {
        float m = 0;
        for (const vec3& p : model->wpos) m = std::max(m, std::max(std::fabs(p.x), std::max(std::fabs(p.y), std::fabs(p.z))));
        wabs = m * 0x1p-20f;
    }
    struct Canon { int tri = -1; TriIsect isect{}; int tri2 = -1; float t2 = std::numeric_limits<float>::infinity(); bool amb = false; };
    Canon ClosestCanonical(const Ray& ray, bool use_cull) const {
        Canon c;
        float cut = std::numeric_limits<float>::max();
        std::vector<int> stack{0};
        while (!stack.empty()) {
            int cur = stack.back();
            stack.pop_back();
            if (!IntersectP(nodes[cur].bounds, ray, cut)) continue;
            if (!nodes[cur].leaf) {
                for (int i = 7; i >= 0; --i) stack.push_back(nodes[cur].child[i]);
                continue;
            }
            for (int t : nodes[cur].tris) {
                if (t == c.tri || t == c.tri2) continue;  // the octree stores a triangle in every leaf it overlaps
                if (use_cull && model->cull && !model->back_facing.empty() && model->back_facing[t]) continue;
                TriIsect is;
                if (!BasicIntersect(model->P(t, 0), model->P(t, 1), model->P(t, 2), ray, cut, &is) || !(is.t < cut)) continue;
                if (c.tri < 0 || is.t < c.isect.t) {
                    c.tri2 = c.tri; c.t2 = c.tri < 0 ? c.t2 : c.isect.t;
                    c.tri = t; c.isect = is;
                    cut = std::min(cut, is.t + 2 * Window(is.t, wabs));
                } else if (is.t < c.t2) {
                    c.tri2 = t; c.t2 = is.t;
                }
            }
        }
        c.amb = c.tri >= 0 && c.tri2 >= 0 && c.t2 <= c.isect.t + Window(c.isect.t, wabs);
        return c;
    }
    // 1 occluded, 0 not, -1 ambiguous
    int OccludedCanonical(const Ray& ray, float tMax) const {
        const float sure = tMax - Window(tMax, wabs);
        bool amb = false;
        std::vector<int> stack{0};
        while (!stack.empty()) {
            int cur = stack.back();
            stack.pop_back();
            if (!IntersectP(nodes[cur].bounds, ray, tMax)) continue;
            if (!nodes[cur].leaf) {
                for (int i = 7; i >= 0; --i) stack.push_back(nodes[cur].child[i]);
                continue;
            }
            for (int t : nodes[cur].tris) {
                TriIsect is;
                if (BasicIntersect(model->P(t, 0), model->P(t, 1), model->P(t, 2), ray, tMax, &is) && is.t < tMax) {
                    if (is.t < sure) return 1;
                    amb = true;
                }
            }
        }
        return amb ? -1 : 0;
    }
};

// ---- The GPU's fast multi-level walk restated (rt_kernels.hip bvh8_walk / bvh_closest / bvh_anyhit, DESIGN.md
// §6b).  NOT the reference's algorithm and not the product's code: a CPU restatement, operation for operation
// (std::fma where the kernel calls fma, the same IEEE min / max order, the same 19-comparator sorting network and
// push order), over the BVH the product builds (exported through rt_bvh_export / rt_debug_bvh_build: 32 floats per
// node, 12 per tile).  With it a CPU test checks, on millions of rays, that the canonical rule over THIS BVH returns
// what Octree::Traverse / Occluded return, and a GPU test checks the device walk against it ray by ray.
// The device's speculative walk (RT_SPEC, the default) tests a lane's held leaf after the nodes its wave opens
// meanwhile, i.e. in an order that depends on the other lanes; this restates one ray's walk alone (the RT_SPEC=0
// order).  Answers agree either way: the canonical rule's result and its ambiguity do not depend on the order in
// which triangles are tested; only stack overflows (ambiguous, BFS-decided) may fall elsewhere.
struct Bvh8 {
    const float* nodes = nullptr;   // 32 floats per node (rt_bvh.cpp layout)
    const float* tiles = nullptr;   // 12 floats per tile: (p0.xyz, p1.x) (p1.yz, p2.xy) (p2.z, bits(id), 0, 0)
    int n_nodes = 0, n_tiles = 0;
    float wabs = 0, oguard = 0;
    int stack_cap = 16;             // kBvhStack (closest hit)
    int any_cap = 24;               // kAnyStack (any hit)
    static constexpr unsigned kNo = 0xffffffffu;
    struct Stats { int64_t nodes = 0, boxes = 0, tris = 0; int max_sp = 0; };
    struct Result { int tri = -1; TriIsect isect{}; bool amb = false; int occluded = 0; };

    static uint32_t U(float f) { uint32_t u; std::memcpy(&u, &f, 4); return u; }
    static float F(uint32_t u) { float f; std::memcpy(&f, &u, 4); return f; }
    const float* N(int i) const { return nodes + 32 * (size_t)i; }
    static float ClampInv(float d) { return 1 / std::copysign(std::max(std::fabs(d), 0x1p-80f), d); }

    void Keys(int node, const vec3& inv, const vec3& oi, float tcut, unsigned k[8]) const {
        const float* n = N(node);
        const uint32_t w0 = U(n[3]);
        const float s[3] = {std::ldexp(inv.x, (int)(w0 & 255u) - 127), std::ldexp(inv.y, (int)((w0 >> 8) & 255u) - 127),
                            std::ldexp(inv.z, (int)((w0 >> 16) & 255u) - 127)};
        const float b[3] = {std::fma(n[0], inv.x, -oi.x), std::fma(n[1], inv.y, -oi.y), std::fma(n[2], inv.z, -oi.z)};
        const float iv[3] = {inv.x, inv.y, inv.z};
        const uint32_t valid = U(n[7]);
        for (int sl = 0; sl < 8; ++sl) {
            float tnear[3], tfar[3];
            for (int a = 0; a < 3; ++a) {
                const float* q = n + 8 + 4 * a;  // lo bytes (words 0, 1), hi bytes (words 2, 3)
                const uint32_t lo = (U(q[sl >> 2]) >> (8 * (sl & 3))) & 255u, hi = (U(q[2 + (sl >> 2)]) >> (8 * (sl & 3))) & 255u;
                const bool pos = iv[a] >= 0.f;
                tnear[a] = std::fma((float)(pos ? lo : hi), s[a], b[a]);
                tfar[a] = std::fma((float)(pos ? hi : lo), s[a], b[a]);
            }
            const float tn = std::fmax(std::fmax(tnear[0], tnear[1]), std::fmax(tnear[2], 0.f));
            const float tf = std::fmin(std::fmin(tfar[0], tfar[1]), std::fmin(tfar[2], tcut)) * 1.00000048f;
            k[sl] = (((valid >> sl) & 1u) && tn <= tf) ? ((U(tn) & 0x7ffffff8u) | (unsigned)sl) : kNo;
        }
        auto sw = [&](int i, int j) { if (k[j] < k[i]) std::swap(k[i], k[j]); };
        sw(0, 1); sw(2, 3); sw(4, 5); sw(6, 7);
        sw(0, 2); sw(1, 3); sw(4, 6); sw(5, 7);
        sw(1, 2); sw(5, 6);
        sw(0, 4); sw(1, 5); sw(2, 6); sw(3, 7);
        sw(2, 4); sw(3, 5);
        sw(1, 2); sw(3, 4); sw(5, 6);
    }
    int Word(int node, unsigned key) const {
        const float* n = N(node);
        const unsigned s = key & 7u, imask = U(n[3]) >> 24;
        if ((imask >> s) & 1u) return (int)(U(n[4]) + (unsigned)__builtin_popcount(imask & ((1u << s) - 1u)));
        const unsigned counts = U(n[6]), cnt = (counts >> (4 * s)) & 15u;
        unsigned first = U(n[5]);
        for (unsigned j = 0; j < s; ++j) first += (counts >> (4 * j)) & 15u;
        return (int)(0x80000000u | first << 4 | (cnt - 1u));
    }
    // the walk; leaf(first, count) returns true to stop; false on a stack overflow
    // any: the any-hit walk (no cull on pop, twice the stack entries: 4-byte words in the same LDS)
    template <class Leaf>
    bool Walk(const Ray& ray, float& cut, Stats& st, bool any, Leaf&& leaf) const {
        const int cap = any ? any_cap : stack_cap;
        const vec3 inv = {ClampInv(ray.d.x), ClampInv(ray.d.y), ClampInv(ray.d.z)};
        const vec3 oi = {ray.o.x * inv.x, ray.o.y * inv.y, ray.o.z * inv.z};
        std::vector<std::pair<int, unsigned>> stk;
        bool overflow = false;
        int node = 0;
        while (true) {
            int lf = 0, lc = 0;
            while (lc == 0) {
                if (node < 0) {
                    if (stk.empty()) break;
                    auto e = stk.back();
                    stk.pop_back();
                    if (!any && F(e.second & 0x7ffffff8u) > cut) continue;
                    if (e.first >= 0) node = e.first;
                    else { lf = (e.first >> 4) & 0x7ffffff; lc = (e.first & 15) + 1; }
                    continue;
                }
                ++st.nodes;
                st.boxes += __builtin_popcount(U(N(node)[7]));
                unsigned k[8];
                Keys(node, inv, oi, cut, k);
                const int cur = node;
                node = -1;
                for (int i = 7; i >= 1; --i)
                    if (k[i] != kNo) {
                        if ((int)stk.size() < cap) stk.emplace_back(Word(cur, k[i]), k[i]);
                        else overflow = true;
                    }
                st.max_sp = std::max(st.max_sp, (int)stk.size());
                if (k[0] != kNo) {
                    const int w = Word(cur, k[0]);
                    if (w >= 0) node = w;
                    else { lf = (w >> 4) & 0x7ffffff; lc = (w & 15) + 1; }
                }
            }
            if (lc == 0) break;
            if (leaf(lf, lc)) break;
        }
        return !overflow;
    }
    void Tri(int i, vec3& p0, vec3& p1, vec3& p2, int& id) const {
        const float* q = tiles + 12 * (size_t)i;
        p0 = {q[0], q[1], q[2]}; p1 = {q[3], q[4], q[5]}; p2 = {q[6], q[7], q[8]};
        id = (int)U(q[9]);
    }
    bool Guarded(const Ray& r) const {
        return std::fmax(std::fmax(std::fabs(r.o.x), std::fabs(r.o.y)), std::fabs(r.o.z)) <= oguard;
    }
    // bvh_closest: the canonical closest hit (amb: the BFS decides)
    Result Closest(const Ray& ray, Stats& st) const {
        Result res;
        if (!Guarded(ray)) { res.amb = true; return res; }
        float cut = std::numeric_limits<float>::max(), t2 = std::numeric_limits<float>::infinity();
        int best = -1, second = -1;
        const bool ok = Walk(ray, cut, st, false, [&](int lf, int lc) {
            for (int k = 0; k < lc; ++k) {
                vec3 p0, p1, p2;
                int id;
                Tri(lf + k, p0, p1, p2, id);
                ++st.tris;
                TriIsect is;
                if (BasicIntersect(p0, p1, p2, ray, cut, &is) && is.t < cut) {
                    if (best < 0 || is.t < res.isect.t) {
                        t2 = best < 0 ? t2 : res.isect.t;
                        second = best;
                        best = id;
                        res.isect = is;
                        const float c2 = is.t + 2.f * Octree::Window(is.t, wabs);
                        cut = c2 < cut ? c2 : cut;
                    } else if (is.t < t2) {
                        second = id;
                        t2 = is.t;
                    }
                }
            }
            return false;
        });
        res.tri = best;
        res.amb = !ok || (second >= 0 && t2 <= res.isect.t + Octree::Window(res.isect.t, wabs));
        return res;
    }
    // bvh_anyhit: occluded = 1 / 0 (amb: the BFS decides)
    Result AnyHit(const Ray& ray, float tMax, Stats& st) const {
        Result res;
        if (!Guarded(ray)) { res.amb = true; return res; }
        const float sure = tMax - Octree::Window(tMax, wabs);
        bool window = false, occ = false;
        float cut = tMax;
        const bool ok = Walk(ray, cut, st, true, [&](int lf, int lc) {
            for (int k = 0; k < lc; ++k) {
                vec3 p0, p1, p2;
                int id;
                Tri(lf + k, p0, p1, p2, id);
                ++st.tris;
                TriIsect is;
                if (BasicIntersect(p0, p1, p2, ray, tMax, &is) && is.t < tMax) {
                    if (is.t < sure) { occ = true; return true; }
                    window = true;
                }
            }
            return false;
        });
        res.occluded = occ ? 1 : 0;
        res.amb = !occ && (window || !ok);
        return res;
    }
};

// ------------------------------------------------------------------------------- camera
// Cameras.h:273-297 PerspectiveCamera::generateRay; matrices are the values CameraBase holds
struct Camera {
    mat4 rasterToCamera, cameraToWorld;
    float lensRadius = 0, focalDistance = 0;
    int type = 0;                       // 0 perspective, 1 orthographic, 2 pinhole, 3 thin lens
    mat4 rasterToScreen{};
    float pinholeDepth = 0, thinF = 0, thinAperture = 0, sensorDepth = 0;
    Ray generateRay(vec2 pixel, Sampler* sampler) const {
        if (type == 1) {  // Cameras.h:230-243 OrthographicCamera::generateRay
            vec4 cp = mul(rasterToCamera, vec4{pixel.x, pixel.y, 0, 1});
            return TransformRay(Ray{{cp.x, cp.y, cp.z}, {0, 0, 1}}, cameraToWorld);
        }
        if (type == 2) {  // Cameras.h:328-339 PinholeCamera::generateRay(pixel, sampler): the hole's centre
            vec4 s4 = mul(rasterToScreen, vec4{pixel.x, pixel.y, 0, 1});
            vec3 sp = {s4.x, s4.y, s4.z};
            vec3 pin = {0.0f, 0.0f, pinholeDepth};
            return TransformRay(Ray{sp, normalize(sub(pin, sp))}, cameraToWorld);
        }
        if (type == 3) {  // Cameras.h:378-400 ThinlensCamera, (lens_angle, len_percent_r) = (360 u0, u1)
            vec2 u = sampler ? sampler->Get2D() : vec2{0, 0};
            float lens_angle = u.x * 360.0f;
            float len_percent_r = u.y;
            vec4 s4 = mul(rasterToScreen, vec4{pixel.x, pixel.y, 0, 1});
            vec3 sp = {s4.x, s4.y, s4.z};
            float ang = lens_angle * 0.01745329251994329576923690768489f;  // glm::radians
            float half = thinAperture / 2.0f;
            vec3 lens_pos = {len_percent_r * half * cos_f(ang), len_percent_r * half * sin_f(ang), sensorDepth};
            vec3 lens_center = {0, 0, sensorDepth};
            vec3 tmp = normalize(sub(lens_center, sp));
            float t = thinF / tmp.z;
            vec3 fpos = add(lens_center, mul(tmp, t));
            return TransformRay(Ray{lens_pos, normalize(sub(fpos, lens_pos))}, cameraToWorld);
        }
        vec4 np = mul(rasterToCamera, vec4{pixel.x, pixel.y, 0, 1});
        vec3 near_pos = {np.x / np.w, np.y / np.w, np.z / np.w};
        Ray ray{{0, 0, 0}, normalize(near_pos)};
        if (lensRadius > 0 && sampler) {
            vec2 dsk = SampleUniformDiskConcentric(sampler->Get2D());
            vec2 lens = {lensRadius * dsk.x, lensRadius * dsk.y};
            float ft = focalDistance / ray.d.z;
            vec3 pfocus = add(ray.o, mul(ray.d, ft));
            ray.o = {lens.x, lens.y, 0};
            ray.d = normalize(sub(pfocus, ray.o));
        }
        return TransformRay(ray, cameraToWorld);
    }
};

// ----------------------------------------------------------------------------- filters
// filters.h:66-93 BoxFilter::Sample ; filters.h:285-290 TriangleFilter::Sample (deterministic coin)
// Sampling.h:781-877 Continuous_Inversion_Sampler: Riemann-sum CDF over N bins of [a, b], renormalised, then a
// binary search + linear interpolation (the reference draws U itself; here U is the sample's GetPixel2D value).
struct InversionTable {
    int N = 0;
    float a = 0, b = 0;
    std::vector<float> cdf;
    template <class F>
    void Build(F pdf, float a_, float b_, int N_) {
        a = a_; b = b_; N = N_;
        cdf.assign(N + 1, 0.0f);
        float delta_x = (b - a) / (float)N;
        float sum = 0;
        for (int n = 1; n < N + 1; n++) {
            float x = a + delta_x * n;
            float current_x = x < a ? a : (b < x ? b : x);  // std::clamp
            sum += delta_x * pdf(current_x);
            cdf[n] = sum;
        }
        float scaling_term = 1.0f / cdf[N];
        for (int n = 1; n < N; n++) cdf[n] *= scaling_term;
        cdf[N] = 1.0f;
    }
    float Sample(float U) const {
        int index = -1, low = 0, high = N;
        while (low <= high) {
            int mid = (int)((float)low + (float)(high - low) / 2.0f);
            if (cdf[mid] < U && U <= cdf[mid + 1]) { index = mid; break; }
            if (cdf[mid] < U) low = mid + 1;
            else high = mid - 1;
        }
        if (index == -1) return 0;
        float q = (U - cdf[index]) / (cdf[index + 1] - cdf[index]);
        float t = q < 0.0f ? 0.0f : (1.f < q ? 1.f : q);
        float delta_x = (b - a) / (float)N;
        return (a + delta_x * index) + t * (delta_x * (index + 1) - delta_x * index);
    }
};
// helpers.h:221-251 Gaussian / SinXOverX / Sinc / WindowedSinc (powf(v, 2) written v * v)
static inline float GaussianF(float x, float mu, float sigma) {
    float v = x - mu;
    return 1.0f / std::sqrt(2 * Pi * sigma * sigma) * std::exp(-(v * v) / (2 * sigma * sigma));
}
static inline float SinXOverX(float x) {
    if (1 - x * x == 1) return 1;
    return std::sin(x) / x;
}
static inline float WindowedSinc(float x, float radius, float tau) {
    if (std::fabs(x) > radius) return 0;
    return SinXOverX(Pi * x) * SinXOverX(Pi * (x / tau));
}
struct Filter {
    int kind = 0;  // 0 box, 1 triangle, 2 gaussian, 3 lanczos sinc
    float rx = 0.5f, ry = 0.5f;
    InversionTable tx, ty;
    void Init(float param) {  // filters.h:101-107 (Gaussian, N 10000) / 228-231 (Lanczos, N 2000)
        if (kind == 2) {
            float sigma = param > 0 ? param : 0.5f;
            float expX = GaussianF(rx, 0, sigma), expY = GaussianF(ry, 0, sigma);
            tx.Build([&](float x) { return std::max<float>(0, GaussianF(x, 0, sigma) - expX); }, -rx, rx, 10000);
            ty.Build([&](float y) { return std::max<float>(0, GaussianF(y, 0, sigma) - expY); }, -ry, ry, 10000);
        } else if (kind == 3) {
            float tau = param > 0 ? param : 3.f;
            tx.Build([&](float x) { return WindowedSinc(x, rx, tau); }, -rx, rx, 2000);
            ty.Build([&](float y) { return WindowedSinc(y, ry, tau); }, -ry, ry, 2000);
        }
    }
    // FilterSample weight f(p)/(pdf_x pdf_y) with pdf = the filter's own 1-D factors: 1
    vec2 Sample(vec2 u, float* weight) const {
        *weight = 1.0f;
        if (kind == 0) return {Lerp(u.x, -rx, rx), Lerp(u.y, -ry, ry)};
        if (kind == 1) return {SampleTentDet(u.x, rx), SampleTentDet(u.y, ry)};
        return {tx.Sample(u.x), ty.Sample(u.y)};
    }
};

// ======================================================================= analytic shapes (a21)
// Shape (Shapes.h:172-207): rays go to object space through RenderToObject; hits come back through
// LocalSurfaceInfo::Transform(ObjectToRender) (Shapes.h:147-160).  Full spheres / disks only (φmax = 360°),
// so the atan2 φ clips (Shapes.h:343-349, 710-713) can never reject and are not evaluated.
struct AShape {
    int type = 0;          // 0 sphere, 1 disk, 2 TriangleSimple
    mat4 o2r, r2o;
    mat3 n2r;
    float r = 1, zmin = -1, zmax = 1;
    float h = 0, ri = 0, ro = 1;
    vec3 p1{}, p2{}, p3{};
    int material = 0;
};
struct ShapeHit { vec3 phit; float t; };   // object-space hit point

static inline void ObjRay(const AShape& s, const Ray& ray, vec3* o, vec3* d) {
    vec4 o4 = mul(s.r2o, vec4{ray.o.x, ray.o.y, ray.o.z, 1});
    vec4 d4 = mul(s.r2o, vec4{ray.d.x, ray.d.y, ray.d.z, 0});
    *o = {o4.x, o4.y, o4.z};
    *d = {d4.x, d4.y, d4.z};
}
// Shapes.h:294-376 Sphere::BasicIntersect
static inline bool SphereIntersect(const AShape& s, vec3 o, vec3 d, float tMax, ShapeHit* out) {
    const float r = s.r;
    float a = d.x * d.x + d.y * d.y + d.z * d.z;
    float b = 2 * (d.x * o.x + d.y * o.y + d.z * o.z);
    float c = o.x * o.x + o.y * o.y + o.z * o.z - r * r;
    vec3 v = sub(o, mul(d, b / (2 * a)));
    float length = std::sqrt(dot(v, v));
    float discrim = 4 * a * (r + length) * (r - length);
    if (discrim < 0) return false;
    float rootDiscrim = std::sqrt(discrim);
    float q = (b < 0) ? -.5f * (b - rootDiscrim) : -.5f * (b + rootDiscrim);
    float t0 = q / a, t1 = c / q;
    if (t0 > t1) std::swap(t0, t1);
    if (t0 > tMax || t1 <= 0) return false;
    float tShapeHit = t0;
    if (tShapeHit <= 0) {
        tShapeHit = t1;
        if (tShapeHit > tMax) return false;
    }
    auto refine = [&](float th) {
        vec3 hp = add(o, mul(d, th));
        hp = mul(hp, r / std::sqrt(dot(hp, hp)));  // hitp *= r / distance(hitp, 0)
        if (hp.x == 0 && hp.y == 0) hp.x = (float)(1e-5 * (double)r);
        return hp;
    };
    vec3 hitp = refine(tShapeHit);
    if (hitp.z < s.zmin || hitp.z > s.zmax) {
        if (tShapeHit == t1) return false;
        if (t1 > tMax) return false;
        tShapeHit = t1;
        hitp = refine(tShapeHit);
        if (hitp.z < s.zmin || hitp.z > s.zmax) return false;
    }
    *out = {hitp, tShapeHit};
    return true;
}
// Shapes.h:684-716 Disk::BasicIntersect
static inline bool DiskIntersect(const AShape& s, vec3 o, vec3 d, float tMax, ShapeHit* out) {
    float t0 = (s.h - o.z) / d.z;
    if (t0 <= 0 || t0 >= tMax) return false;
    if (d.z == 0) return false;
    vec3 phit = add(o, mul(d, t0));
    float dist2 = phit.x * phit.x + phit.y * phit.y;
    if (dist2 > s.ro * s.ro || dist2 < s.ri * s.ri) return false;
    *out = {phit, t0};
    return true;
}
// Shapes.h:842-880 TriangleSimple::BasicIntersect (Cramer's rule in object space)
static inline bool TriSimpleIntersect(const AShape& s, vec3 orig, vec3 dir, float tMax, ShapeHit* out) {
    float a = s.p1.x - s.p2.x, b = s.p1.y - s.p2.y, c = s.p1.z - s.p2.z;
    float d = s.p1.x - s.p3.x, e = s.p1.y - s.p3.y, f = s.p1.z - s.p3.z;
    float g = dir.x, h = dir.y, i = dir.z;
    float j = s.p1.x - orig.x, k = s.p1.y - orig.y, l = s.p1.z - orig.z;
    float M = a * (e * i - h * f) + b * (g * f - d * i) + c * (d * h - e * g);
    float t = -(f * (a * k - j * b) + e * (j * c - a * l) + d * (b * l - k * c)) / M;
    if (t < 0 || t >= tMax) return false;
    float Y = (i * (a * k - j * b) + h * (j * c - a * l) + g * (b * l - k * c)) / M;
    if (Y < 0 || Y > 1) return false;
    float B = (j * (e * i - h * f) + k * (g * f - d * i) + l * (d * h - e * g)) / M;
    if (B < 0 || B > 1 - Y) return false;
    *out = {add(orig, mul(dir, t)), t};
    return true;
}
static inline bool ShapeIntersect(const AShape& s, const Ray& ray, float tMax, ShapeHit* out) {
    vec3 o, d;
    ObjRay(s, ray, &o, &d);
    if (s.type == 0) return SphereIntersect(s, o, d, tMax, out);
    if (s.type == 1) return DiskIntersect(s, o, d, tMax, out);
    return TriSimpleIntersect(s, o, d, tMax, out);
}
// object-space normal (Shapes.h:417-422 sphere gradient, 744-752 disk +z, 897-901 TriangleSimple)
static inline vec3 ShapeNormalObj(const AShape& s, vec3 p) {
    if (s.type == 0) return normalize({2 * p.x, 2 * p.y, 2 * p.z});
    if (s.type == 1) return {0, 0, 1};
    return normalize(cross(sub(s.p3, s.p1), sub(s.p2, s.p1)));
}

// ========================================================================= the integrators
// Build-defined materials and lights (Shading.h:1-21, Lights.h:1-10 are stubs) — DESIGN.md §5.
struct Material { int type = 0; float c[3] = {0, 0, 0}; float emit = 0; float eta = 0; };  // Le = emit * D65
struct Light {
    int type = 0;          // 0 quad, 1 disk, 2 point, 3 distant
    vec3 p{}, e1{}, e2{}, n{}, dir{};
    float scale = 0, area = 0;
    int material = -1, shape = -1;
};

struct Scene {
    Spectra spectra;
    Piecewise bk7;       // FromInterleaved(GlassBK7_eta, false) (spectrum.cpp:2674-2675)
    TriModel model;
    Octree octree;
    Camera camera;
    Sampler sampler;
    Filter filter;
    int resX = 500, resY = 500;
    float imagingRatio = 1.0f / CIE_Y_integral;
    // reference mode (RayTracerTestApp.h:218-284)
    float albedo_rgb[3] = {0.5f, 0.5f, 0.5f};
    // path mode (build-defined)
    std::vector<int> tri_material;
    std::vector<Material> materials;
    std::vector<Light> lights;
    std::vector<AShape> shapes;
    std::vector<int> light_of_material, light_of_shape;   // area light index of an emitter, or -1
    bool mis = false;
    int max_depth = 5;
};

// color.h:537-557 LinearToSRGB / LinearToSRGB8 (pbrt ColorEncoding::sRGB; EvaluatePolynomial = FMA Horner chain)
static inline float EvalPoly6(float t, float c0, float c1, float c2, float c3, float c4, float c5) {
    return std::fmaf(t, std::fmaf(t, std::fmaf(t, std::fmaf(t, std::fmaf(t, c5, c4), c3), c2), c1), c0);
}
static inline float LinearToSRGB(float value) {
    if (value <= 0.0031308f) return 12.92f * value;
    float sqrtValue = std::sqrt(std::max(0.f, value));
    float p = EvalPoly6(sqrtValue, -0.0016829072605308378f, 0.03453868659826638f, 0.7642611304733891f,
                        2.0041169284241644f, 0.7551545191665577f, -0.016202083165206348f);
    float q = EvalPoly6(sqrtValue, 4.178892964897981e-7f, -0.00004375359692957097f, 0.03467195408529984f,
                        0.6085338522168684f, 1.8970238036421054f, 1.f);
    return p / q * value;
}
static inline uint8_t LinearToSRGB8(float value) {
    if (value <= 0) return 0;
    if (value >= 1) return 255;
    float r = std::round(255.f * LinearToSRGB(value));
    return (uint8_t)(r < 0 ? 0 : (r > 255 ? 255 : r));
}

// Per-sample debug record (for golden fixtures / kernel-level parity)
struct SampleRecord {
    float lambda[8], pdf[8];
    float ro[3], rd[3];
    int prim;
    float b[3], t;
    float L[8];
    float rgb[3];
    float weight;
};

// RayTracerTestApp.h:289-291 — raster coordinate of a pixel id (y in [1, resY], a kept quirk)
static inline void PixelCoord(int pixel_id, int resX, int resY, int* x, int* y) {
    *x = pixel_id % resX;
    *y = (int)((float)resY - std::floor((float)pixel_id / (float)resX));
}

// RayTracerTestApp.h:218-284 Li (active branch): ambient 0.3*F1 + clamp(n.(0,0,-1))*(light*albedo)
static inline SS LiReference(const Scene& S, const Ray& ray, const SW& w, SampleRecord* rec, long* counters) {
    Octree::Hit h = S.octree.Traverse(ray, true);
    if (counters) { counters[0] += h.nodes_tested; counters[1] += h.tris_tested; counters[2] += (h.tri >= 0); }
    if (rec) { rec->prim = h.tri; rec->b[0] = h.isect.b0; rec->b[1] = h.isect.b1; rec->b[2] = h.isect.b2; rec->t = h.isect.t; }
    SS r{};
    if (h.tri < 0) return r;  // SampledSpectrum(0)
    const TriModel& m = S.model;
    // Shapes.h:1066-1075 — object-space interpolated normal, flipped against normalize(ray.d)
    vec3 n1 = m.nrm[m.idx[3 * h.tri]], n2 = m.nrm[m.idx[3 * h.tri + 1]], n3 = m.nrm[m.idx[3 * h.tri + 2]];
    vec3 n = normalize(add(add(mul(n1, h.isect.b0), mul(n2, h.isect.b1)), mul(n3, h.isect.b2)));
    vec3 rayd = normalize(ray.d);  // Shapes.h:1259
    if (dot(n, rayd) > 0) n = {-n.x, -n.y, -n.z};
    // color.cpp:35-37 uniform branch; RGBAlbedo(rgb) -> constant s(c2)
    Sigmoid alb = SigmoidFromGrey(S.albedo_rgb[0]);
    float cosv = gclamp(dot(n, {0, 0, -1}), 0.0f, 1.0f);
    for (int i = 0; i < 8; ++i) {
        float light = (2.0f * 0.5f) * S.spectra.D65dense.Query(w.lambda[i]);  // spectrum.h:621-629 (scale*rsp)*illum
        float amb = S.spectra.F1.Query(w.lambda[i]) * 0.3f;                    // 0.3f * illumF->Sample
        float mat = alb(w.lambda[i]);
        float radiance = 0.0f + amb;                                          // radiance += ambient
        radiance += (light * mat) * cosv;                                     // radiance += cos*(light*mat)
        r.v[i] = radiance;
    }
    return r;
}

// ---- scene queries (build-defined combination): the octree's closest hit first, then every
// analytic shape in list order with the running tMax and that shape's own acceptance rule.
struct SceneHit { int kind = 0; int id = -1; TriIsect tri{}; ShapeHit sh{}; };  // kind 0 miss, 1 triangle, 2 shape
static inline SceneHit Closest(const Scene& S, const Ray& ray, bool use_cull, long* counters) {
    SceneHit h;
    Octree::Hit oh = S.octree.Traverse(ray, use_cull);
    if (counters) { counters[0] += oh.nodes_tested; counters[1] += oh.tris_tested; }
    float tMax = std::numeric_limits<float>::max();
    if (oh.tri >= 0) { h.kind = 1; h.id = oh.tri; h.tri = oh.isect; tMax = oh.isect.t; }
    for (size_t i = 0; i < S.shapes.size(); ++i) {
        ShapeHit sh;
        if (ShapeIntersect(S.shapes[i], ray, tMax, &sh)) { h.kind = 2; h.id = (int)i; h.sh = sh; tMax = sh.t; }
    }
    if (counters) { counters[2] += (h.kind != 0); counters[3] += 1; }
    return h;
}
static inline bool SceneOccluded(const Scene& S, const Ray& ray, float tMax) {
    if (S.octree.Occluded(ray, tMax)) return true;
    for (const AShape& sh : S.shapes) {
        ShapeHit x;
        if (ShapeIntersect(sh, ray, tMax, &x)) return true;
    }
    return false;
}
// Surface at a hit: world point p, world normal n turned against the ray (Shapes.h:1074, 262-263), the
// front-side normal nout (triangle winding Shapes.h:1073 / shape outward normal) and whether the ray arrives
// on the front side.
struct Surf { vec3 p, n, nout; bool front; int material; };
static inline Surf SurfaceAt(const Scene& S, const SceneHit& h, const Ray& ray) {
    Surf sf;
    vec3 rayd = normalize(ray.d);
    if (h.kind == 1) {
        const TriModel& m = S.model;
        vec3 p0 = m.P(h.id, 0), p1 = m.P(h.id, 1), p2 = m.P(h.id, 2);
        vec3 ng = normalize(cross(sub(p0, p2), sub(p1, p2)));
        sf.p = add(add(mul(p0, h.tri.b0), mul(p1, h.tri.b1)), mul(p2, h.tri.b2));
        sf.nout = ng;
        sf.front = dot(ng, rayd) < 0;
        sf.n = ng;
        if (dot(sf.n, rayd) > 0) sf.n = {-ng.x, -ng.y, -ng.z};
        sf.material = S.tri_material[h.id];
    } else {
        const AShape& s = S.shapes[h.id];
        vec3 o, d;
        ObjRay(s, ray, &o, &d);
        vec3 rd = normalize(d);                               // ray_d = glm::normalize(d) (Shapes.h:375)
        vec3 n = ShapeNormalObj(s, h.sh.phit);
        bool flip = dot(n, rd) > 0;
        if (flip) n = {-n.x, -n.y, -n.z};
        vec3 nw = normalize(mul(s.n2r, n));                   // LocalSurfaceInfo::Transform (Shapes.h:150-151)
        vec4 pw = mul(s.o2r, vec4{h.sh.phit.x, h.sh.phit.y, h.sh.phit.z, 1});
        sf.p = {pw.x, pw.y, pw.z};
        sf.n = nw;
        sf.front = !flip;
        sf.nout = flip ? vec3{-nw.x, -nw.y, -nw.z} : nw;
        sf.material = s.material;
    }
    return sf;
}
// pbrt-v4 PowerHeuristic(1, f, 1, g)
static inline float PowerHeuristic(float f, float g) {
    float f2 = f * f, g2 = g * g;
    if (std::isinf(f2)) return 1;
    return f2 / (f2 + g2);
}
// pbrt-v4 FrDielectric (smooth dielectric Fresnel reflectance)
static inline float FrDielectric(float cosTheta_i, float eta) {
    cosTheta_i = gclamp(cosTheta_i, -1.0f, 1.0f);
    if (cosTheta_i < 0) { eta = 1 / eta; cosTheta_i = -cosTheta_i; }
    float sin2Theta_i = 1 - cosTheta_i * cosTheta_i;
    float sin2Theta_t = sin2Theta_i / (eta * eta);
    if (sin2Theta_t >= 1) return 1.f;
    float cosTheta_t = std::sqrt(std::max(0.f, 1 - sin2Theta_t));
    float r_parl = (eta * cosTheta_i - cosTheta_t) / (eta * cosTheta_i + cosTheta_t);
    float r_perp = (cosTheta_i - eta * cosTheta_t) / (cosTheta_i + eta * cosTheta_t);
    return (r_parl * r_parl + r_perp * r_perp) / 2;
}
// pbrt-v4 Refract(wi, n, eta, &etap, &wt)
static inline bool Refract(vec3 wi, vec3 n, float eta, float* etap, vec3* wt) {
    float cosTheta_i = dot(n, wi);
    if (cosTheta_i < 0) { eta = 1 / eta; cosTheta_i = -cosTheta_i; n = {-n.x, -n.y, -n.z}; }
    float sin2Theta_i = std::max(0.f, 1 - cosTheta_i * cosTheta_i);
    float sin2Theta_t = sin2Theta_i / (eta * eta);
    if (sin2Theta_t >= 1) return false;
    float cosTheta_t = std::sqrt(std::max(0.f, 1 - sin2Theta_t));
    vec3 a = {-wi.x / eta, -wi.y / eta, -wi.z / eta};
    *wt = add(a, mul(n, cosTheta_i / eta - cosTheta_t));
    *etap = eta;
    return true;
}
// glm::reflect(I, N) = I - N * dot(N, I) * 2
static inline vec3 Reflect(vec3 I, vec3 N) { return sub(I, mul(mul(N, dot(N, I)), 2.0f)); }
// spectrum.h:302-310 SampledWavelengths::TerminateSecondary
static inline void TerminateSecondary(SW& w) {
    bool terminated = true;
    for (int i = 1; i < NSpectrumSamples; ++i) if (w.pdf[i] != 0) terminated = false;
    if (terminated) return;
    for (int i = 1; i < NSpectrumSamples; ++i) w.pdf[i] = 0;
    w.pdf[0] /= NSpectrumSamples;
}

// Build-defined path integrator (pbrt-v4 PathIntegrator semantics): Lambert R/π, perfect mirror,
// smooth dielectric (BK7 dispersion → TerminateSecondary); one light sample per light at every diffuse vertex;
// emitters are one-sided and end the path.  Sample dimensions per vertex: diffuse = one Get2D per light, then
// Get2D for the cosine direction; mirror = none; dielectric = Get1D.  With `mis` (RT_INTEGRATOR_PATH_MIS) light
// samples of area lights and BSDF-sampled emitter hits are weighted by the power heuristic; without it emitters
// count only on camera rays and after specular bounces.
static inline SS LiPath(const Scene& S, Ray ray, SW& w, Sampler& smp, long* counters) {
    SS L{}, beta;
    for (int i = 0; i < 8; ++i) beta.v[i] = 1.0f;
    float prevPdf = 0;  // solid-angle pdf of the last diffuse bounce; 0 = camera ray or specular bounce
    for (int depth = 0;; ++depth) {
        SceneHit h = Closest(S, ray, false, counters);
        if (h.kind == 0) break;
        Surf sf = SurfaceAt(S, h, ray);
        const Material& mat = S.materials[sf.material];
        if (mat.emit > 0) {  // pure emitter: one-sided, terminates the path
            if (sf.front) {
                if (prevPdf == 0) {
                    for (int i = 0; i < 8; ++i) L.v[i] += beta.v[i] * (mat.emit * S.spectra.D65dense.Query(w.lambda[i]));
                } else if (S.mis) {
                    int li = h.kind == 1 ? S.light_of_material[sf.material] : S.light_of_shape[h.id];
                    if (li >= 0) {
                        const Light& Lt = S.lights[li];
                        vec3 dv = sub(sf.p, ray.o);
                        float dist2 = dot(dv, dv);
                        float cl = -dot(Lt.n, normalize(ray.d));
                        if (cl > 0) {
                            float wb = PowerHeuristic(prevPdf, dist2 / (cl * Lt.area));
                            for (int i = 0; i < 8; ++i)
                                L.v[i] += (beta.v[i] * (mat.emit * S.spectra.D65dense.Query(w.lambda[i]))) * wb;
                        }
                    }
                }
            }
            break;
        }
        if (depth == S.max_depth) break;
        vec3 n = sf.n, p = sf.p;
        vec3 rayd = normalize(ray.d);
        float ap = MaxComponentValue({std::fabs(p.x), std::fabs(p.y), std::fabs(p.z)});
        float off = 1e-4f * (1.0f + ap);
        float R[8];
        Sigmoid sg{mat.c[0], mat.c[1], mat.c[2]};
        for (int i = 0; i < 8; ++i) R[i] = sg(w.lambda[i]);
        if (mat.type == 1) {  // perfect mirror
            for (int i = 0; i < 8; ++i) beta.v[i] *= R[i];
            ray = Ray{add(p, mul(n, off)), Reflect(rayd, n)};
            prevPdf = 0;
            continue;
        }
        if (mat.type == 2) {  // smooth dielectric
            if (mat.eta == 0) TerminateSecondary(w);
            float eta = mat.eta != 0 ? mat.eta : S.bk7.Query(w.lambda[0]);
            float u = smp.Get1D();
            vec3 wo = {-rayd.x, -rayd.y, -rayd.z};
            float Fr = FrDielectric(dot(sf.nout, wo), eta);
            vec3 wt;
            float etap;
            if (u < Fr || !Refract(wo, sf.nout, eta, &etap, &wt)) {
                ray = Ray{add(p, mul(n, off)), Reflect(rayd, n)};
            } else {
                for (int i = 0; i < 8; ++i) beta.v[i] /= (etap * etap);
                ray = Ray{sub(p, mul(n, off)), wt};
            }
            prevPdf = 0;
            continue;
        }
        vec3 po = add(p, mul(n, off));
        // --- NEE: one sample per light, in list order
        for (size_t li = 0; li < S.lights.size(); ++li) {
            const Light& Lt = S.lights[li];
            vec2 ul = smp.Get2D();
            if (Lt.type <= 1) {  // quad / disk area light, uniform area sampling
                vec3 pl;
                if (Lt.type == 0) {
                    pl = add(add(Lt.p, mul(Lt.e1, ul.x)), mul(Lt.e2, ul.y));
                } else {  // Sampling.h:383-403 on the object-space disk z = h, then ObjectToRender
                    const AShape& ds = S.shapes[Lt.shape];
                    vec2 dk = SampleUniformDiskConcentric(ul);
                    vec4 pw = mul(ds.o2r, vec4{ds.ro * dk.x, ds.ro * dk.y, ds.h, 1});
                    pl = {pw.x, pw.y, pw.z};
                }
                vec3 wv = sub(pl, po);
                float dist2 = dot(wv, wv);
                float dist = std::sqrt(dist2);
                vec3 wi = mul(wv, 1.0f / dist);
                float cs = dot(n, wi);
                float cl = -dot(Lt.n, wi);
                if (cs > 0 && cl > 0) {
                    if (counters) counters[4] += 1;
                    if (!SceneOccluded(S, Ray{po, wi}, dist * 0.999f)) {
                        const Material& lm = S.materials[Lt.material];
                        float G = (cs * cl) / dist2;
                        float wgt = G * Lt.area;
                        if (S.mis) wgt = wgt * PowerHeuristic(dist2 / (cl * Lt.area), cs * InvPi);
                        for (int i = 0; i < 8; ++i) {
                            float Le = lm.emit * S.spectra.D65dense.Query(w.lambda[i]);
                            L.v[i] += ((beta.v[i] * (R[i] * InvPi)) * Le) * wgt;
                        }
                    }
                }
            } else {  // point (intensity) / distant (irradiance) light
                vec3 wi;
                float tmax, fall;
                if (Lt.type == 2) {
                    vec3 wv = sub(Lt.p, po);
                    float dist2 = dot(wv, wv);
                    float dist = std::sqrt(dist2);
                    wi = mul(wv, 1.0f / dist);
                    tmax = dist * 0.999f;
                    fall = 1.0f / dist2;
                } else {
                    wi = Lt.dir;
                    tmax = std::numeric_limits<float>::max();
                    fall = 1.0f;
                }
                float cs = dot(n, wi);
                if (cs > 0) {
                    if (counters) counters[4] += 1;
                    if (!SceneOccluded(S, Ray{po, wi}, tmax)) {
                        float wgt = cs * fall;
                        for (int i = 0; i < 8; ++i) {
                            float I = Lt.scale * S.spectra.D65dense.Query(w.lambda[i]);
                            L.v[i] += ((beta.v[i] * (R[i] * InvPi)) * I) * wgt;
                        }
                    }
                }
            }
        }
        // --- BSDF sampling: cosine hemisphere around n (frame: Shapes.h:1025-1029 CoordinateSystem)
        vec2 ub = smp.Get2D();
        vec3 wl = SampleCosineHemisphere(ub);
        if (wl.z == 0) break;
        float sign = std::copysign(1.0f, n.z);
        float a = -1 / (sign + n.z);
        float b = n.x * n.y * a;
        vec3 s = {1 + sign * (n.x * n.x) * a, sign * b, -sign * n.x};
        vec3 t = {b, sign + (n.y * n.y) * a, -n.y};
        vec3 wi = add(add(mul(s, wl.x), mul(t, wl.y)), mul(n, wl.z));
        for (int i = 0; i < 8; ++i) beta.v[i] *= R[i];
        prevPdf = wl.z * InvPi;  // CosineHemispherePDF
        ray = Ray{po, wi};
    }
    return L;
}

// RayTracerTestApp.h:287-345 evaluate_pixel (film accumulation in place)
static inline void EvaluatePixel(const Scene& S, Sampler& smp, int pixel_id, int index, bool path_mode, float* px,
                                 SampleRecord* rec, long* counters) {
    int x, y;
    PixelCoord(pixel_id, S.resX, S.resY, &x, &y);
    if (!smp.StartPixelSample(x, y, index, 0)) return;
    SW w = SampleVisible(smp.Get1D());
    vec2 up = smp.GetPixel2D();
    float fw;
    vec2 fp = S.filter.Sample(up, &fw);
    vec2 pos = {((float)x + .5f) + fp.x, ((float)y + .5f) + fp.y};
    Ray ray = S.camera.generateRay(pos, &smp);
    SS L = path_mode ? LiPath(S, ray, w, smp, counters) : LiReference(S, ray, w, rec, counters);
    float rgb[3];
    ToSensorRGB(S.spectra, L, w, S.imagingRatio, rgb);
    for (int c = 0; c < 3; ++c) rgb[c] = gclamp(rgb[c], 0.0f, 1.0f);
    px[0] += fw * rgb[0];
    px[1] += fw * rgb[1];
    px[2] += fw * rgb[2];
    px[3] += fw;
    if (rec) {
        std::memcpy(rec->lambda, w.lambda, 32); std::memcpy(rec->pdf, w.pdf, 32);
        rec->ro[0] = ray.o.x; rec->ro[1] = ray.o.y; rec->ro[2] = ray.o.z;
        rec->rd[0] = ray.d.x; rec->rd[1] = ray.d.y; rec->rd[2] = ray.d.z;
        std::memcpy(rec->L, L.v, 32); std::memcpy(rec->rgb, rgb, 12);
        rec->weight = fw;
    }
}

}  // namespace rtcore
