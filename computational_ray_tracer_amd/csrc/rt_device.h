// Device-side building blocks of the MI355X ray-tracing inner loop (gfx950, wave64).
//
// Every function restates one reference function (file:line cited) with the SAME float operation order
// as the CPU oracle, compiled with -ffp-contract=off: FMA appears only where the reference calls std::fma
// (DifferenceOfProducts helpers.h:56-62, EvaluatePolynomial helpers.h:117-126).  Transcendentals are
// evaluated in double and rounded to float (documented build choice).
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "rt_internal.h"
#include "rt_mathf.h"

namespace rtmi {

#define RT_DEV __device__ __forceinline__

// sin/cos: fixed float algorithm shared (as a definition, not as code) with the oracle — Cody-Waite reduction
// by pi/2 + Cephes minimax polynomials with explicit fma; ~1 ulp on |x| <= 3pi/4 (concentric disk range).
RT_DEV void sincos_det(float x, float& s, float& c) {
    float k = __builtin_rintf(x * 0.636619772367581343f);
    float r = __builtin_fmaf(-k, 1.57079637050628662109375f, x);
    r = __builtin_fmaf(-k, -4.37113900018624283e-8f, r);
    float r2 = r * r;
    float sp = __builtin_fmaf(__builtin_fmaf(-1.9515295891e-4f, r2, 8.3321608736e-3f), r2, -1.6666654611e-1f);
    float sr = __builtin_fmaf(sp * r2, r, r);
    float cp = __builtin_fmaf(__builtin_fmaf(2.443315711809948e-5f, r2, -1.388731625493765e-3f), r2, 4.166664568298827e-2f);
    float cr = __builtin_fmaf(cp * r2, r2, __builtin_fmaf(-0.5f, r2, 1.0f));
    int q = (int)k & 3;
    s = q == 0 ? sr : (q == 1 ? cr : (q == 2 ? -sr : -cr));
    c = q == 0 ? cr : (q == 1 ? -sr : (q == 2 ? -cr : sr));
}
// (float)atanh((double)x) / (float)cosh((double)x) as the oracle computes them: the fast double evaluation of
// rt_mathf.h, and the full-precision library call only when that result is within 2^-46 of a float rounding midpoint
// (about 1 input in 3.4e7; tools/verify_warps.cpp checks every input float of the warps against glibc)
template <class T = rtm::TabConst>
RT_DEV float f_atanh(float x) {
    double r = rtm::atanh_fast<T>(x);
    float f = (float)r;
    if (rtm::near_midpoint(r, f)) f = (float)atanh((double)x);
    return f;
}
template <class T = rtm::TabConst>
RT_DEV float f_cosh(float x) {
    double r = rtm::cosh_fast<T>(x);
    float f = (float)r;
    if (rtm::near_midpoint(r, f)) f = (float)cosh((double)x);
    return f;
}

// helpers.h:50-54
RT_DEV float gamma_n(int n) {
    const float me = 0x1p-24f;  // numeric_limits<float>::epsilon() * 0.5
    return ((float)n * me) / (1.0f - (float)n * me);
}
// glm scalar min/max/clamp
RT_DEV float gmax(float x, float y) { return (x < y) ? y : x; }
RT_DEV float gmin(float x, float y) { return (y < x) ? y : x; }
RT_DEV float gclamp(float x, float lo, float hi) { return gmin(gmax(x, lo), hi); }
// helpers.h:56-62
RT_DEV float dop(float a, float b, float c, float d) {
    float cd = c * d;
    float x = __builtin_fmaf(a, b, -cd);
    float e = __builtin_fmaf(-c, d, cd);
    return x + e;
}
// std::max({a,b,c}) — first largest
RT_DEV float max3f(float a, float b, float c) {
    float m = a;
    if (m < b) m = b;
    if (m < c) m = c;
    return m;
}
RT_DEV float lerpf_(float x, float a, float b) { return (1 - x) * a + x * b; }  // helpers.h:154-157

struct V3 { float x, y, z; };
RT_DEV V3 v3(float x, float y, float z) { return {x, y, z}; }
RT_DEV V3 vadd(V3 a, V3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
RT_DEV V3 vsub(V3 a, V3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
RT_DEV V3 vmul(V3 a, float s) { return {a.x * s, a.y * s, a.z * s}; }
RT_DEV float vdot(V3 a, V3 b) { return (a.x * b.x + a.y * b.y) + a.z * b.z; }           // glm dot vec3
RT_DEV V3 vcross(V3 a, V3 b) { return {a.y * b.z - b.y * a.z, a.z * b.x - b.z * a.x, a.x * b.y - b.x * a.y}; }
RT_DEV V3 vnorm(V3 v) { float s = 1.0f / sqrtf(vdot(v, v)); return vmul(v, s); }      // glm normalize

// glm mat4*vec4 = (m0*x + m1*y) + (m2*z + m3*w), column-major m[c*4+r]
RT_DEV void mat4_mul(const float* M, float x, float y, float z, float w, float o[4]) {
#pragma unroll
    for (int r = 0; r < 4; ++r) {
        float a0 = M[0 * 4 + r] * x, a1 = M[1 * 4 + r] * y, a2 = M[2 * 4 + r] * z, a3 = M[3 * 4 + r] * w;
        o[r] = (a0 + a1) + (a2 + a3);
    }
}

// ------------------------------------------------------------------ hashing + PCG32 (integer exact)
RT_DEV uint64_t murmur_mix_block(uint64_t h, uint64_t k) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    k *= m; k ^= k >> 47; k *= m;
    h ^= k; h *= m;
    return h;
}
RT_DEV uint64_t murmur_final(uint64_t h) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    h ^= h >> 47; h *= m; h ^= h >> 47;
    return h;
}
// hash.h:96-104 Hash(ivec2 p, int seed) — 12-byte key: one 8-byte block (x | y<<32) + 4-byte tail (seed)
RT_DEV uint64_t hash_pixel(int x, int y, int seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 0ull ^ (12ull * m);
    h = murmur_mix_block(h, (uint64_t)(uint32_t)x | ((uint64_t)(uint32_t)y << 32));
    h ^= (uint64_t)(uint32_t)seed;  // tail bytes key[8..11], hash.h:47-55
    h *= m;
    return murmur_final(h);
}
// Hash(ivec2 p, int dim, int seed) — 16-byte key: two blocks
RT_DEV uint64_t hash_pixel_dim(int x, int y, int dim, int seed) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 0ull ^ (16ull * m);
    h = murmur_mix_block(h, (uint64_t)(uint32_t)x | ((uint64_t)(uint32_t)y << 32));
    h = murmur_mix_block(h, (uint64_t)(uint32_t)dim | ((uint64_t)(uint32_t)seed << 32));
    return murmur_final(h);
}
RT_DEV uint64_t mix_bits(uint64_t v) {  // hash.h:67-74
    v ^= (v >> 31); v *= 0x7fb5d329728ea185ull;
    v ^= (v >> 27); v *= 0x81dadef4bc2dd44dull;
    v ^= (v >> 33);
    return v;
}
// HelperFunctions.h:175-203
RT_DEV int permutation_element(uint32_t i, uint32_t l, uint32_t p) {
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

// PermutationElement for a power-of-two l: the cycle-walking loop runs once (w = l - 1 masks every value below l,
// and i ^ (i >> 5) stays below it) and (i + p) % l is (i + p) & (l - 1) on the wrapped 32-bit sum
RT_DEV int permutation_element_p2(uint32_t i, uint32_t l, uint32_t p) {
    const uint32_t w = l - 1;
    i ^= p; i *= 0xe170893du; i ^= p >> 16; i ^= (i & w) >> 4; i ^= p >> 8; i *= 0x0929eb3fu;
    i ^= p >> 23; i ^= (i & w) >> 1; i *= 1u | p >> 27; i *= 0x6935fa69u; i ^= (i & w) >> 11;
    i *= 0x74dcb303u; i ^= (i & w) >> 2; i *= 0x9e501cc3u; i ^= (i & w) >> 2; i *= 0xc860a3dfu;
    i &= w; i ^= i >> 5;
    return (int)((i + p) & w);
}

struct Pcg {  // rng.h:24-144
    uint64_t state, inc;
    RT_DEV uint32_t next() {
        uint64_t old = state;
        state = old * 0x5851f42d4c957f2dull + inc;
        uint32_t xs = (uint32_t)(((old >> 18u) ^ old) >> 27u);
        uint32_t rot = (uint32_t)(old >> 59u);
        return (xs >> rot) | (xs << ((~rot + 1u) & 31));
    }
    RT_DEV float uniform() {  // rng.h:122-124, OneMinusEpsilon == 1.0f
        float v = (float)next() * 0x1p-32f;
        return (1.0f < v) ? 1.0f : v;  // std::min<float>(1, v)
    }
    RT_DEV void set_sequence(uint64_t seq) {  // rng.h:36-39, 113-119
        uint64_t seed = mix_bits(seq);
        state = 0u;
        inc = (seq << 1u) | 1u;
        next();
        state += seed;
        next();
    }
    // rng.h:131-144.  The square-and-multiply's curMult after i halvings is M^(2^i) and its curPlus is inc times
    // prod_{k<i} (M^(2^k) + 1), both mod 2^64: they come from a constant table (kPcgJump), so only the set bits of
    // delta cost multiplications — the same ring values, hence the same state.
    RT_DEV void advance(uint64_t delta);
};

struct PcgJumpTable {
    uint64_t mult[64], plus[64];
};
constexpr PcgJumpTable make_pcg_jump() {
    PcgJumpTable t{};
    uint64_t m = 0x5851f42d4c957f2dull, p = 1;
    for (int i = 0; i < 64; ++i) {
        t.mult[i] = m;
        t.plus[i] = p;
        p = (m + 1) * p;
        m *= m;
    }
    return t;
}
__constant__ constexpr PcgJumpTable kPcgJump = make_pcg_jump();

RT_DEV void Pcg::advance(uint64_t delta) {
    // (r03 A/B: Cornell +0.5 %, k_generate -6 %)
    // accPlus is inc times a value P(delta) of the jump table alone (the recurrence is linear in inc, mod 2^64), so
    // the loop does not depend on the lane; when the wave shares delta (k_generate: one sample index per wave) it runs
    // once per wave on the scalar unit, and each lane makes two 64-bit multiply-adds
    const uint32_t lo = (uint32_t)delta, hi = (uint32_t)(delta >> 32);
    const uint32_t lo0 = __builtin_amdgcn_readfirstlane(lo), hi0 = __builtin_amdgcn_readfirstlane(hi);
    if (__ballot(lo != lo0 || hi != hi0) == 0) {
        uint64_t d = (uint64_t)lo0 | ((uint64_t)hi0 << 32), M = 1u, P = 0u;
        for (int i = 0; d > 0; ++i, d >>= 1) {
            if (d & 1) {
                const uint64_t cm = kPcgJump.mult[i];
                M *= cm;
                P = P * cm + kPcgJump.plus[i];
            }
        }
        state = M * state + inc * P;
        return;
    }
    uint64_t accMult = 1u, accPlus = 0u;
    for (int i = 0; delta > 0; ++i, delta >>= 1) {
        if (delta & 1) {
            const uint64_t cm = kPcgJump.mult[i];
            accMult *= cm;
            accPlus = accPlus * cm + inc * kPcgJump.plus[i];
        }
    }
    state = accMult * state + accPlus;
}

// ------------------------------------------------------------------------------------- Sobol
// hash.h:96-104 Hash(int, int): an 8-byte key, one block, no tail
RT_DEV uint64_t hash_int2(int a, int b) {
    const uint64_t m = 0xc6a4a7935bd1e995ull;
    uint64_t h = 0ull ^ (8ull * m);
    h = murmur_mix_block(h, (uint64_t)(uint32_t)a | ((uint64_t)(uint32_t)b << 32));
    return murmur_final(h);
}
// samplers.h:198-209 SobolSample + the scramblers of samplers.h:147-190 (ReverseBits32 = bit reversal)
RT_DEV float sobol_sample(const DevSampler& S, uint64_t a, int dimension, int randomize, uint32_t seed) {
    uint32_t v = 0;
    const uint32_t* C = S.sobol_mats + dimension * kSobolMatrixSize;
    for (int i = 0; a != 0; a >>= 1, i++)
        if (a & 1) v ^= C[i];
    if (randomize == 1) {
        v ^= seed;
    } else if (randomize == 2) {
        v = __builtin_bitreverse32(v);
        v ^= v * 0x3d20adeau;
        v += seed;
        v *= (seed >> 16) | 1u;
        v ^= v * 0x05526c56u;
        v ^= v * 0x53a22864u;
        v = __builtin_bitreverse32(v);
    } else if (randomize == 3) {
        if (seed & 1) v ^= 1u << 31;
        for (int b = 1; b < 32; ++b) {
            uint32_t mask = (~0u) << (32 - b);
            if ((uint32_t)mix_bits((uint64_t)((v & mask) ^ seed)) & (1u << b)) v ^= 1u << (31 - b);
        }
    }
    float f = (float)v * 0x1p-32f;
    const float ome = 0x1.fffffep-1f;  // FloatOneMinusEpsilon (samplers.h:141)
    return ome < f ? ome : f;          // std::min(f, ome)
}
// samplers.h:211-227 SobolIntervalToIndex
RT_DEV uint64_t sobol_interval_to_index(const DevSampler& S, uint64_t frame, int px, int py) {
    const uint32_t m = (uint32_t)S.sobol_m;
    if (m == 0) return frame;
    uint64_t index = frame << (2 * m);
    uint64_t delta = 0;
    for (int c = 0; frame; frame >>= 1, ++c)
        if (frame & 1) delta ^= S.sobol_fwd[c];
    uint64_t b = (((uint64_t)(uint32_t)px << m) | (uint32_t)py) ^ delta;
    for (int c = 0; b; b >>= 1, ++c)
        if (b & 1) index ^= S.sobol_inv[c];
    return index;
}

// samplers.h:38-136, 229-327 — Independent / Stratified / Sobol sampler state of one camera sample (Sobol keeps its
// sobolIndex in rng.state)
struct Smp {
    Pcg rng;
    int px, py, index, dim;
    // samplers.h:80-93 / 47-51 (caller guarantees the stratified jitter==false index < spp precondition)
    RT_DEV void start(const DevSampler& S, int x, int y, int idx, int d) {
        px = x; py = y; index = idx; dim = d;
        if (S.kind == 2) {  // samplers.h:258-263
            dim = d > 2 ? d : 2;
            rng.state = sobol_interval_to_index(S, (uint64_t)idx, x, y);
            rng.inc = 0;
            return;
        }
        rng.set_sequence(hash_pixel(x, y, S.seed));
        rng.advance((uint64_t)idx * 65536ull + (uint64_t)d);
    }
    RT_DEV float sobol_dim(const DevSampler& S, int d) const {  // samplers.h:305-318
        uint32_t h = S.randomize ? (uint32_t)hash_int2(d, S.seed) : 0u;
        return sobol_sample(S, rng.state, d, S.randomize, h);
    }
    RT_DEV void get_pixel2d(const DevSampler& S, float& u0, float& u1) {  // samplers.h:283-297
        if (S.kind != 2) { get2d(S, u0, u1); return; }
        float a = sobol_sample(S, rng.state, 0, 0, 0u), b = sobol_sample(S, rng.state, 1, 0, 0u);
        u0 = gclamp(a * (float)S.scale - (float)px, 0.0f, 1.0f);  // OneMinusEpsilon == 1.0f (pch.h:39)
        u1 = gclamp(b * (float)S.scale - (float)py, 0.0f, 1.0f);
    }
    RT_DEV float get1d(const DevSampler& S) {  // samplers.h:95-104
        if (S.kind == 0) return rng.uniform();
        if (S.kind == 2) {
            if (dim >= kSobolDims) dim = 2;
            return sobol_dim(S, dim++);
        }
        uint64_t h = hash_pixel_dim(px, py, dim, S.seed);
        int stratum = S.p2 ? permutation_element_p2((uint32_t)index, (uint32_t)S.spp, (uint32_t)h)
                           : permutation_element((uint32_t)index, (uint32_t)S.spp, (uint32_t)h);
        ++dim;
        float delta = S.jitter ? rng.uniform() : 0.5f;
        return S.p2 ? ((float)stratum + delta) * S.inv_spp : ((float)stratum + delta) / (float)S.spp;
    }
    RT_DEV void get2d(const DevSampler& S, float& u0, float& u1) {  // samplers.h:107-123
        if (S.kind == 0) { u0 = rng.uniform(); u1 = rng.uniform(); return; }
        if (S.kind == 2) {
            if (dim + 1 >= kSobolDims) dim = 2;
            u0 = sobol_dim(S, dim);
            u1 = sobol_dim(S, dim + 1);
            dim += 2;
            return;
        }
        if (index >= S.spp) { u0 = 0; u1 = 0; return; }
        uint64_t h = hash_pixel_dim(px, py, dim, S.seed);
        dim += 2;
        if (S.p2) {  // power-of-two strata: the same values without integer or float divisions
            int stratum = permutation_element_p2((uint32_t)index, (uint32_t)S.spp, (uint32_t)h);
            int x = stratum & (S.xs - 1), y = stratum >> S.lg_xs;
            float dx = S.jitter ? rng.uniform() : 0.5f;
            float dy = S.jitter ? rng.uniform() : 0.5f;
            u0 = ((float)x + dx) * S.inv_xs;
            u1 = ((float)y + dy) * S.inv_ys;
            return;
        }
        int stratum = permutation_element((uint32_t)index, (uint32_t)S.spp, (uint32_t)h);
        int x = stratum % S.xs, y = stratum / S.xs;
        float dx = S.jitter ? rng.uniform() : 0.5f;
        float dy = S.jitter ? rng.uniform() : 0.5f;
        u0 = ((float)x + dx) / (float)S.xs;
        u1 = ((float)y + dy) / (float)S.ys;
    }
};

// ------------------------------------------------------------------------------ sampling warps
template <class T = rtm::TabConst>
RT_DEV float visible_pdf(float lambda) {  // Sampling.h:63-67
    if (lambda < 360 || lambda > 830) return 0;
    float c = f_cosh<T>(0.0072f * (lambda - 538));
    return (float)((double)0.0039398042f / ((double)c * (double)c));
}
template <class T = rtm::TabConst>
RT_DEV float sample_visible_wavelength(float u) {  // Sampling.h:69-71
    return 538 - 138.888889f * f_atanh<T>(0.85691062f - 1.82750197f * u);
}
RT_DEV float sample_linear(float u, float a, float b) {  // Sampling.h:205-211
    if (u == 0 && a == 0) return 0;
    float x = (u * (a + b)) / (a + sqrtf(lerpf_(u, a * a, b * b)));
    return (1.0f < x) ? 1.0f : x;
}
RT_DEV float sample_tent(float u, float r) {  // Sampling.h:228-235 with the coin taken from u (build-defined)
    if (u < 0.5f) {
        float up = u * 2.0f; up = (1.0f < up) ? 1.0f : up;
        return -r + r * sample_linear(up, 0, 1);
    }
    float up = (u - 0.5f) * 2.0f; up = (1.0f < up) ? 1.0f : up;
    return r * sample_linear(up, 1, 0);
}
RT_DEV void disk_concentric(float u0, float u1, float& ox, float& oy) {  // Sampling.h:383-403
    float x = 2.0f * u0 - 1.0f, y = 2.0f * u1 - 1.0f;
    if (x == 0 && y == 0) { ox = 0; oy = 0; return; }
    float theta, r;
    if (fabsf(x) > fabsf(y)) { r = x; theta = 0.78539816339744830961f * (y / x); }
    else { r = y; theta = 1.57079632679489661923f - 0.78539816339744830961f * (x / y); }
    float sn, cs;
    sincos_det(theta, sn, cs);
    ox = r * cs;
    oy = r * sn;
}

// ------------------------------------------------------------------------------------ spectra
RT_DEV float dense_query(const float* tab, float lambda) {  // spectrum.h:386-398 / 430-437
    long off = (long)roundf(lambda) - 360;  // std::lround: half away from zero
    if (off < 0 || off >= kSpecN) return 0;
    return tab[off];
}
RT_DEV float piecewise_query(const float* lam, const float* val, int n, float lambda) {  // spectrum.cpp:60-71
    if (n == 0 || lambda < lam[0] || lambda > lam[n - 1]) return 0;
    long size = (long)n - 2, first = 1;  // helpers.h:159-172 FindInterval
    while (size > 0) {
        long half = size >> 1, middle = first + half;
        bool r = lam[middle] <= lambda;
        first = r ? middle + 1 : first;
        size = r ? size - (half + 1) : half;
    }
    long o = first - 1;
    o = o < 0 ? 0 : (o > n - 2 ? n - 2 : o);
    float t = (lambda - lam[o]) / (lam[o + 1] - lam[o]);
    return lerpf_(t, val[o], val[o + 1]);
}
RT_DEV float sigmoid_eval(float c0, float c1, float c2, float lambda) {  // color.h:373-399
    float x = __builtin_fmaf(lambda, __builtin_fmaf(lambda, c0, c1), c2);
    if (__builtin_isinf(x)) return x > 0 ? 1 : 0;
    return .5f + x / (2 * sqrtf(1 + (x * x)));
}
// pixelsensor.h:81-87 XYZ sensor ToSensorRGB (SafeDiv by pdf, Average, * imagingRatio)
RT_DEV void to_sensor_rgb(const DevSpectra* sp, const float L_[8], const float lam[8], const float pdf[8], float ir,
                          float rgb[3]) {
    float L[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) L[i] = (pdf[i] != 0) ? L_[i] / pdf[i] : 0.f;
    const float* bars[3] = {sp->SR, sp->SG, sp->SB};  // X/Y/Z for the XYZ sensor, camera curves otherwise
#pragma unroll
    for (int c = 0; c < 3; ++c) {
        float sum = dense_query(bars[c], lam[0]) * L[0];
#pragma unroll
        for (int i = 1; i < 8; ++i) sum += dense_query(bars[c], lam[i]) * L[i];
        rgb[c] = ir * (sum / 8);
    }
}

// ------------------------------------------------------------------------------ geometry tests
// Per-ray precomputation for the watertight test (Shapes.h:1138-1160): the permutation and shear depend
// only on the ray, so they are hoisted (bit-identical to recomputing them per triangle).
struct TriRay {
    int kx, ky, kz;
    float Sx, Sy, Sz;
    float ox, oy, oz;     // ray origin, permuted
};
RT_DEV float sel3(int k, float x, float y, float z) { return k == 0 ? x : (k == 1 ? y : z); }
RT_DEV int dominant_axis(V3 d) {  // helpers.h:64-66 MaxComponentIndex(Abs(d))
    float ax = fabsf(d.x), ay = fabsf(d.y), az = fabsf(d.z);
    return (ax > ay) ? ((ax > az) ? 0 : 2) : ((ay > az) ? 1 : 2);
}
// KZ >= 0: the caller guarantees dominant_axis(d) == KZ, so the permutation is resolved at compile time
// (no per-triangle selects); KZ < 0: per-lane permutation.
template <int KZ>
RT_DEV TriRay make_triray(V3 o, V3 d) {
    TriRay t;
    t.kz = KZ >= 0 ? KZ : dominant_axis(d);
    t.kx = t.kz + 1; if (t.kx == 3) t.kx = 0;
    t.ky = t.kx + 1; if (t.ky == 3) t.ky = 0;
    float dx = sel3(t.kx, d.x, d.y, d.z), dy = sel3(t.ky, d.x, d.y, d.z), dz = sel3(t.kz, d.x, d.y, d.z);
    t.Sx = -dx / dz; t.Sy = -dy / dz; t.Sz = 1 / dz;
    t.ox = sel3(t.kx, o.x, o.y, o.z); t.oy = sel3(t.ky, o.x, o.y, o.z); t.oz = sel3(t.kz, o.x, o.y, o.z);
    return t;
}
// Shapes.h:1101-1260 Triangle::BasicIntersect on pre-transformed world vertices (degenerate triangles were
// removed from the tiles at upload, Shapes.h:1131).  Returns true and (b0,b1,b2,t) on a hit.
template <int KZ>
RT_DEV bool tri_intersect(const TriRay& R, float tMax, float4 A, float4 B, float4 Cc, float& b0, float& b1, float& b2,
                          float& tt) {
    constexpr int KX = KZ == 0 ? 1 : (KZ == 1 ? 2 : 0), KY = KZ == 0 ? 2 : (KZ == 1 ? 0 : 1);
    const int kx = KZ >= 0 ? KX : R.kx, ky = KZ >= 0 ? KY : R.ky, kz = KZ >= 0 ? KZ : R.kz;
    // vertices p0=(A.x,A.y,A.z) p1=(A.w,B.x,B.y) p2=(B.z,B.w,C.x); translate after permuting (same ops)
    float p0x = sel3(kx, A.x, A.y, A.z) - R.ox, p0y = sel3(ky, A.x, A.y, A.z) - R.oy, p0z = sel3(kz, A.x, A.y, A.z) - R.oz;
    float p1x = sel3(kx, A.w, B.x, B.y) - R.ox, p1y = sel3(ky, A.w, B.x, B.y) - R.oy, p1z = sel3(kz, A.w, B.x, B.y) - R.oz;
    float p2x = sel3(kx, B.z, B.w, Cc.x) - R.ox, p2y = sel3(ky, B.z, B.w, Cc.x) - R.oy, p2z = sel3(kz, B.z, B.w, Cc.x) - R.oz;
    p0x += R.Sx * p0z; p0y += R.Sy * p0z;
    p1x += R.Sx * p1z; p1y += R.Sy * p1z;
    p2x += R.Sx * p2z; p2y += R.Sy * p2z;
    float e0 = dop(p1x, p2y, p1y, p2x);
    float e1 = dop(p2x, p0y, p2y, p0x);
    float e2 = dop(p0x, p1y, p0y, p1x);
    // Same decisions as Shapes.h:1174-1190, ordered so the common miss (no zero edge, mixed signs) leaves
    // through a single branch: the double-precision fallback only ever runs when some edge is exactly 0.
    bool zero = (e0 == 0.0f) | (e1 == 0.0f) | (e2 == 0.0f);
    bool mixed = ((e0 < 0) | (e1 < 0) | (e2 < 0)) & ((e0 > 0) | (e1 > 0) | (e2 > 0));
    if (!zero & mixed) return false;
    if (zero) {  // Shapes.h:1174-1184
        e0 = (float)((double)p2y * (double)p1x - (double)p2x * (double)p1y);
        e1 = (float)((double)p0y * (double)p2x - (double)p0x * (double)p2y);
        e2 = (float)((double)p1y * (double)p0x - (double)p1x * (double)p0y);
        if (((e0 < 0) | (e1 < 0) | (e2 < 0)) & ((e0 > 0) | (e1 > 0) | (e2 > 0))) return false;
    }
    float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0z *= R.Sz; p1z *= R.Sz; p2z *= R.Sz;
    float tScaled = e0 * p0z + e1 * p1z + e2 * p2z;
    if (det < 0 && (tScaled >= 0 || tScaled < tMax * det)) return false;
    else if (det > 0 && (tScaled <= 0 || tScaled > tMax * det)) return false;
    float invDet = 1 / det;
    float t = tScaled * invDet;
    if (__builtin_isnan(t)) return false;
    float maxZt = max3f(fabsf(p0z), fabsf(p1z), fabsf(p2z));
    float deltaZ = gamma_n(3) * maxZt;
    float maxXt = max3f(fabsf(p0x), fabsf(p1x), fabsf(p2x));
    float maxYt = max3f(fabsf(p0y), fabsf(p1y), fabsf(p2y));
    float deltaX = gamma_n(5) * (maxXt + maxZt);
    float deltaY = gamma_n(5) * (maxYt + maxZt);
    float deltaE = 2 * (gamma_n(2) * maxXt * maxYt + deltaY * maxXt + deltaX * maxYt);
    float maxE = max3f(fabsf(e0), fabsf(e1), fabsf(e2));
    float deltaT = 3 * (gamma_n(3) * maxE * maxZt + deltaE * maxZt + deltaZ * maxE) * fabsf(invDet);
    if (t <= deltaT) return false;
    b0 = e0 * invDet; b1 = e1 * invDet; b2 = e2 * invDet;
    tt = t;
    return true;
}

// One vertex translated, permuted and sheared exactly as tri_intersect does it: a pure function of the vertex and
// the ray, so a vertex shared by two triangles is transformed once.
struct XV {
    float x, y, z;
};
template <int KZ>
RT_DEV XV tri_xform(const TriRay& R, float a, float b, float c) {
    constexpr int KX = KZ == 0 ? 1 : (KZ == 1 ? 2 : 0), KY = KZ == 0 ? 2 : (KZ == 1 ? 0 : 1);
    const int kx = KZ >= 0 ? KX : R.kx, ky = KZ >= 0 ? KY : R.ky, kz = KZ >= 0 ? KZ : R.kz;
    XV v;
    v.x = sel3(kx, a, b, c) - R.ox; v.y = sel3(ky, a, b, c) - R.oy; v.z = sel3(kz, a, b, c) - R.oz;
    v.x += R.Sx * v.z; v.y += R.Sy * v.z;
    return v;
}
RT_DEV bool tri_candidate_x(const TriRay& R, XV q0, XV q1, XV q2);
// The tMax-independent rejections of tri_intersect (same operations, same order): false means the reference
// test rejects this triangle for every tMax, so a caller may skip it without changing any result.
template <int KZ>
RT_DEV bool tri_candidate(const TriRay& R, float4 A, float4 B, float4 Cc) {
    return tri_candidate_x(R, tri_xform<KZ>(R, A.x, A.y, A.z), tri_xform<KZ>(R, A.w, B.x, B.y),
                           tri_xform<KZ>(R, B.z, B.w, Cc.x));
}
// A fan pair (a,b,c),(a,c,d) — the host flags tile pairs whose second triangle starts with the first one's
// vertices 0 and 2 bit for bit — transforms 4 vertices instead of 6.  Bit i of the result = triangle i passes.
template <int KZ>
RT_DEV unsigned tri_candidate_pair(const TriRay& R, float4 A, float4 B, float4 Cc, float4 B2, float4 C2) {
    XV v0 = tri_xform<KZ>(R, A.x, A.y, A.z), v1 = tri_xform<KZ>(R, A.w, B.x, B.y);
    XV v2 = tri_xform<KZ>(R, B.z, B.w, Cc.x), v3 = tri_xform<KZ>(R, B2.z, B2.w, C2.x);
    return (tri_candidate_x(R, v0, v1, v2) ? 1u : 0u) | (tri_candidate_x(R, v0, v2, v3) ? 2u : 0u);
}
RT_DEV bool tri_candidate_x(const TriRay& R, XV q0, XV q1, XV q2) {
    float p0x = q0.x, p0y = q0.y, p0z = q0.z, p1x = q1.x, p1y = q1.y, p1z = q1.z, p2x = q2.x, p2y = q2.y, p2z = q2.z;
    float e0 = dop(p1x, p2y, p1y, p2x);
    float e1 = dop(p2x, p0y, p2y, p0x);
    float e2 = dop(p0x, p1y, p0y, p1x);
    bool zero = (e0 == 0.0f) | (e1 == 0.0f) | (e2 == 0.0f);
    bool mixed = ((e0 < 0) | (e1 < 0) | (e2 < 0)) & ((e0 > 0) | (e1 > 0) | (e2 > 0));
    if (!zero & mixed) return false;
    // An edge exactly 0: the reference recomputes the edges in double (tri_intersect does), which this filter
    // skips — it keeps the triangle as a candidate, and the full test of pass 2 decides it exactly.  (Rare; the
    // double block's registers set the single-leaf kernels' allocation.)
    if (zero) return true;
    float det = e0 + e1 + e2;
    if (det == 0) return false;
    p0z *= R.Sz; p1z *= R.Sz; p2z *= R.Sz;
    float tScaled = e0 * p0z + e1 * p1z + e2 * p2z;
    if (det < 0 && tScaled >= 0) return false;
    if (det > 0 && tScaled <= 0) return false;
    return true;
}

// Shapes.h:100-124 Bounds3::IntersectP.  1/d is hoisted (same value as computed per node); the per-axis
// early return is folded into one final compare (min_t only grows, max_t only shrinks, NaN axes are no-ops).
RT_DEV bool box_hit(float4 a, float4 b, V3 o, V3 inv, float tMax) {
    const float g = 1 + 2 * gamma_n(3);
    float mn = 0, mx = tMax;
    float tn, tf, s;
    tn = (a.x - o.x) * inv.x; tf = (b.x - o.x) * inv.x;
    if (tn > tf) { s = tn; tn = tf; tf = s; }
    tf *= g; mn = tn > mn ? tn : mn; mx = tf < mx ? tf : mx;
    tn = (a.y - o.y) * inv.y; tf = (b.y - o.y) * inv.y;
    if (tn > tf) { s = tn; tn = tf; tf = s; }
    tf *= g; mn = tn > mn ? tn : mn; mx = tf < mx ? tf : mx;
    tn = (a.z - o.z) * inv.z; tf = (b.z - o.z) * inv.z;
    if (tn > tf) { s = tn; tn = tf; tf = s; }
    tf *= g; mn = tn > mn ? tn : mn; mx = tf < mx ? tf : mx;
    return !(mn > mx);
}

// Conservative box test for the single-leaf culling clusters only — never an octree node, whose test keeps
// Bounds3::IntersectP's exact operations above.  Same slab distances and tFar factor as box_hit, reduced with
// v_min/v_max (IEEE minNum/maxNum) instead of compare-and-select chains.  The one behavioural difference: a plane
// distance that is NaN (d_axis == 0 with the origin exactly on that plane) makes the other plane of the axis decide
// the slab; such a ray lies in the box's face plane, at least the cluster pad away from every triangle of the
// cluster (rt_host.cpp upload), so no candidate test of the cluster can pass and skipping it is exact.
RT_DEV bool cluster_hit(float4 a, float4 b, V3 o, V3 inv, float tMax) {
    const float g = 1 + 2 * gamma_n(3);
    const float x0 = (a.x - o.x) * inv.x, x1 = (b.x - o.x) * inv.x;
    const float y0 = (a.y - o.y) * inv.y, y1 = (b.y - o.y) * inv.y;
    const float z0 = (a.z - o.z) * inv.z, z1 = (b.z - o.z) * inv.z;
    const float mn = fmaxf(fmaxf(fminf(x0, x1), fminf(y0, y1)), fmaxf(fminf(z0, z1), 0.f));
    const float mx = fminf(fminf(fmaxf(x0, x1), fmaxf(y0, y1)), fmaxf(z0, z1)) * g;
    return mn <= fminf(mx, tMax);
}

// Sampling.h:809-840 Continuous_Inversion_Sampler::Sample: binary search of U in the CDF table, then linear
// interpolation inside the bin (table built on the host, rt_host.cpp inversion_table).
RT_DEV float inversion_sample(const float* cdf, int N, float a, float b, float U) {
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

// ---------------------------------------------------------------------- analytic shapes (a21)
// Restated from Shapes.h like oracle/rtcore.hpp (same op order): the ray goes to object space through
// RenderToObject, hits come back through LocalSurfaceInfo::Transform (Shapes.h:147-160).  Full spheres and
// disks only (φmax = 360°, checked at upload), so the atan2 φ clips are never evaluated.
RT_DEV V3 m4_point(const float* M, V3 p) { float o[4]; mat4_mul(M, p.x, p.y, p.z, 1.f, o); return v3(o[0], o[1], o[2]); }
RT_DEV V3 m4_dir(const float* M, V3 d) { float o[4]; mat4_mul(M, d.x, d.y, d.z, 0.f, o); return v3(o[0], o[1], o[2]); }
RT_DEV V3 m3_mul(const float* M, V3 v) {  // glm mat3*vec3: (m0 x + m1 y) + m2 z
    return v3((M[0] * v.x + M[3] * v.y) + M[6] * v.z, (M[1] * v.x + M[4] * v.y) + M[7] * v.z,
              (M[2] * v.x + M[5] * v.y) + M[8] * v.z);
}
// Shapes.h:294-376 Sphere::BasicIntersect
RT_DEV bool sphere_isect(const DevShape& s, V3 o, V3 d, float tMax, V3& ph, float& th) {
    const float r = s.r;
    float a = d.x * d.x + d.y * d.y + d.z * d.z;
    float b = 2 * (d.x * o.x + d.y * o.y + d.z * o.z);
    float c = o.x * o.x + o.y * o.y + o.z * o.z - r * r;
    V3 v = vsub(o, vmul(d, b / (2 * a)));
    float length = sqrtf(vdot(v, v));
    float discrim = 4 * a * (r + length) * (r - length);
    if (discrim < 0) return false;
    float rootDiscrim = sqrtf(discrim);
    float q = (b < 0) ? -.5f * (b - rootDiscrim) : -.5f * (b + rootDiscrim);
    float t0 = q / a, t1 = c / q;
    if (t0 > t1) { float x = t0; t0 = t1; t1 = x; }
    if (t0 > tMax || t1 <= 0) return false;
    float tsh = t0;
    if (tsh <= 0) {
        tsh = t1;
        if (tsh > tMax) return false;
    }
    const float fixx = (float)(1e-5 * (double)r);
    V3 hp = vadd(o, vmul(d, tsh));
    hp = vmul(hp, r / sqrtf(vdot(hp, hp)));
    if (hp.x == 0 && hp.y == 0) hp.x = fixx;
    if (hp.z < s.zmin || hp.z > s.zmax) {
        if (tsh == t1) return false;
        if (t1 > tMax) return false;
        tsh = t1;
        hp = vadd(o, vmul(d, tsh));
        hp = vmul(hp, r / sqrtf(vdot(hp, hp)));
        if (hp.x == 0 && hp.y == 0) hp.x = fixx;
        if (hp.z < s.zmin || hp.z > s.zmax) return false;
    }
    ph = hp; th = tsh;
    return true;
}
// Shapes.h:684-716 Disk::BasicIntersect
RT_DEV bool disk_isect(const DevShape& s, V3 o, V3 d, float tMax, V3& ph, float& th) {
    float t0 = (s.h - o.z) / d.z;
    if (t0 <= 0 || t0 >= tMax) return false;
    if (d.z == 0) return false;
    V3 p = vadd(o, vmul(d, t0));
    float dist2 = p.x * p.x + p.y * p.y;
    if (dist2 > s.ro * s.ro || dist2 < s.ri * s.ri) return false;
    ph = p; th = t0;
    return true;
}
// Shapes.h:842-880 TriangleSimple::BasicIntersect
RT_DEV bool trisimple_isect(const DevShape& s, V3 orig, V3 dir, float tMax, V3& ph, float& th) {
    float a = s.p1[0] - s.p2[0], b = s.p1[1] - s.p2[1], c = s.p1[2] - s.p2[2];
    float d = s.p1[0] - s.p3[0], e = s.p1[1] - s.p3[1], f = s.p1[2] - s.p3[2];
    float g = dir.x, h = dir.y, i = dir.z;
    float j = s.p1[0] - orig.x, k = s.p1[1] - orig.y, l = s.p1[2] - orig.z;
    float M = a * (e * i - h * f) + b * (g * f - d * i) + c * (d * h - e * g);
    float t = -(f * (a * k - j * b) + e * (j * c - a * l) + d * (b * l - k * c)) / M;
    if (t < 0 || t >= tMax) return false;
    float Y = (i * (a * k - j * b) + h * (j * c - a * l) + g * (b * l - k * c)) / M;
    if (Y < 0 || Y > 1) return false;
    float B = (j * (e * i - h * f) + k * (g * f - d * i) + l * (d * h - e * g)) / M;
    if (B < 0 || B > 1 - Y) return false;
    ph = vadd(orig, vmul(dir, t)); th = t;
    return true;
}
// A conservative cull ahead of the exact tests: a ray segment [0, tMax] whose closest approach to the shape's padded
// render-space bounding sphere lies outside it cannot hit the shape, so the exact test (two 4x4 transforms, square
// roots, divisions) would return false — skipping it changes no result.  The slack 1e-4 |c - o|^2 covers the rounding
// of this test and of the exact one far from the origin; a degenerate direction (d.d not > 0, NaN) is never culled.
RT_DEV bool shape_culled(const DevShape& s, V3 o, V3 d, float tMax) {
    const V3 oc = v3(s.bs[0] - o.x, s.bs[1] - o.y, s.bs[2] - o.z);
    const float dd = vdot(d, d);
    if (!(dd > 0.f)) return false;
    float t = vdot(oc, d) * __builtin_amdgcn_rcpf(dd);
    t = t < 0.f ? 0.f : t;
    t = t > tMax ? tMax : t;
    const V3 q = v3(oc.x - d.x * t, oc.y - d.y * t, oc.z - d.z * t);
    return vdot(q, q) > s.bs[3] + 1e-4f * vdot(oc, oc);
}
// CULL = false: the exact test alone (kernels of single-leaf scenes, where the cull's registers would raise the
// allocation of a kernel that never meets a shape in the bench scenes)
template <bool CULL = true>
RT_DEV bool shape_isect(const DevShape& s, V3 o, V3 d, float tMax, V3& ph, float& th) {
    if (CULL && shape_culled(s, o, d, tMax)) return false;
    V3 oo = m4_point(s.r2o, o), dd = m4_dir(s.r2o, d);
    if (s.type == 0) return sphere_isect(s, oo, dd, tMax, ph, th);
    if (s.type == 1) return disk_isect(s, oo, dd, tMax, ph, th);
    return trisimple_isect(s, oo, dd, tMax, ph, th);
}
// object-space normal: sphere gradient (Shapes.h:417-422), disk +z (744-752), TriangleSimple (897-901)
RT_DEV V3 shape_normal_obj(const DevShape& s, V3 p) {
    if (s.type == 0) return vnorm(v3(2 * p.x, 2 * p.y, 2 * p.z));
    if (s.type == 1) return v3(0, 0, 1);
    return vnorm(vcross(vsub(v3(s.p3[0], s.p3[1], s.p3[2]), v3(s.p1[0], s.p1[1], s.p1[2])),
                        vsub(v3(s.p2[0], s.p2[1], s.p2[2]), v3(s.p1[0], s.p1[1], s.p1[2]))));
}

// ------------------------------------------------------------------ scattering (pbrt-v4)
RT_DEV float power_heuristic(float f, float g) {
    float f2 = f * f, g2 = g * g;
    if (__builtin_isinf(f2)) return 1;
    return f2 / (f2 + g2);
}
RT_DEV float fr_dielectric(float cosi, float eta) {
    cosi = gclamp(cosi, -1.0f, 1.0f);
    if (cosi < 0) { eta = 1 / eta; cosi = -cosi; }
    float sin2i = 1 - cosi * cosi;
    float sin2t = sin2i / (eta * eta);
    if (sin2t >= 1) return 1.f;
    float x = 1 - sin2t;
    float cost = sqrtf(x > 0.f ? x : 0.f);
    float r_parl = (eta * cosi - cost) / (eta * cosi + cost);
    float r_perp = (cosi - eta * cost) / (cosi + eta * cost);
    return (r_parl * r_parl + r_perp * r_perp) / 2;
}
RT_DEV bool refract_dir(V3 wi, V3 n, float eta, float& etap, V3& wt) {
    float cosi = vdot(n, wi);
    if (cosi < 0) { eta = 1 / eta; cosi = -cosi; n = v3(-n.x, -n.y, -n.z); }
    float x = 1 - cosi * cosi;
    float sin2i = x > 0.f ? x : 0.f;   // std::max(0, .)
    float sin2t = sin2i / (eta * eta);
    if (sin2t >= 1) return false;
    float y = 1 - sin2t;
    float cost = sqrtf(y > 0.f ? y : 0.f);
    wt = vadd(v3(-wi.x / eta, -wi.y / eta, -wi.z / eta), vmul(n, cosi / eta - cost));
    etap = eta;
    return true;
}
RT_DEV V3 reflect_dir(V3 I, V3 N) { return vsub(I, vmul(vmul(N, vdot(N, I)), 2.0f)); }  // glm::reflect

// Bounds3::IntersectP (Shapes.h:100-124) split at tMax: with F the ternary chain-min of the inflated far planes
// (NaN axes skipped, as in box_hit) and mn the chain-max of the near planes, the test passes for a given tMax iff
// mn <= min(tMax, F), i.e. iff box_entry(..) <= tMax (+inf when mn > F: never passes).
RT_DEV float box_entry(float4 a, float4 b, V3 o, V3 inv) {
    const float g = 1 + 2 * gamma_n(3);
    float mn = 0, F = __builtin_inff();
    float tn, tf, s;
    tn = (a.x - o.x) * inv.x; tf = (b.x - o.x) * inv.x;
    if (tn > tf) { s = tn; tn = tf; tf = s; }
    tf *= g; mn = tn > mn ? tn : mn; F = tf < F ? tf : F;
    tn = (a.y - o.y) * inv.y; tf = (b.y - o.y) * inv.y;
    if (tn > tf) { s = tn; tn = tf; tf = s; }
    tf *= g; mn = tn > mn ? tn : mn; F = tf < F ? tf : F;
    tn = (a.z - o.z) * inv.z; tf = (b.z - o.z) * inv.z;
    if (tn > tf) { s = tn; tn = tf; tf = s; }
    tf *= g; mn = tn > mn ? tn : mn; F = tf < F ? tf : F;
    return mn > F ? __builtin_inff() : mn;
}

}  // namespace rtmi
