// Sanitizer driver for the oracle ("TSan/ASan build of the CPU restatement"): one translation unit with
// oracle/rtcore_capi.cpp, built twice by tests/sanitize/Makefile — ASan + UBSan and TSan — and run by
// tests/test_sanitizers.py.  It exercises the threaded paths the Python suite drives through ctypes: the octree build
// (a tessellated sphere forces a multi-level tree), the reference-order BFS and the canonical-rule check on several
// threads, and the reference / path / MIS integrators rendering on several threads with contiguous pixel ranges
// (RayTracerTestApp.h:372-397).  Exit status 0 = no sanitizer report (they abort on the first error).
#include "../../oracle/rtcore_capi.cpp"

#include <cstdio>
#include <random>

namespace {

void quad(std::vector<float>& P, std::vector<float>& N, std::vector<uint32_t>& I, std::vector<int>& M, const float* a,
          const float* b, const float* c, const float* d, const float* n, int mat) {
    const uint32_t base = (uint32_t)(P.size() / 3);
    for (const float* v : {a, b, c, d}) {
        P.insert(P.end(), v, v + 3);
        N.insert(N.end(), n, n + 3);
    }
    for (uint32_t k : {0u, 1u, 2u, 0u, 2u, 3u}) I.push_back(base + k);
    M.push_back(mat);
    M.push_back(mat);
}

void ident(float* m) {
    for (int i = 0; i < 16; ++i) m[i] = (i % 5 == 0) ? 1.f : 0.f;
}

}  // namespace

int main() {
    // a unit-ish box (walls facing inwards), a ceiling light quad and a tessellated sphere inside
    std::vector<float> P, N;
    std::vector<uint32_t> I;
    std::vector<int> M;
    const float a[3] = {0, 0, 0}, b[3] = {10, 0, 0}, c[3] = {10, 0, 10}, d[3] = {0, 0, 10};
    const float e[3] = {0, 10, 0}, f[3] = {10, 10, 0}, g[3] = {10, 10, 10}, h[3] = {0, 10, 10};
    const float up[3] = {0, 1, 0}, dn[3] = {0, -1, 0}, px[3] = {1, 0, 0}, nx[3] = {-1, 0, 0}, nz[3] = {0, 0, -1};
    quad(P, N, I, M, a, b, c, d, up, 0);   // floor
    quad(P, N, I, M, e, h, g, f, dn, 0);   // ceiling
    quad(P, N, I, M, a, d, h, e, px, 1);   // left
    quad(P, N, I, M, b, f, g, c, nx, 0);   // right
    quad(P, N, I, M, d, c, g, h, nz, 0);   // back
    const float l0[3] = {4, 9.99f, 4}, l1[3] = {6, 9.99f, 4}, l2[3] = {6, 9.99f, 6}, l3[3] = {4, 9.99f, 6};
    quad(P, N, I, M, l0, l3, l2, l1, dn, 2);  // light
    const int slices = 24, stacks = 16;    // sphere: 2 x 24 x 16 = 768 triangles
    for (int s = 0; s < stacks; ++s)
        for (int t = 0; t < slices; ++t) {
            auto pt = [&](int ss, int tt, float* o, float* n) {
                float th = 3.14159265f * ss / stacks, ph = 6.2831853f * tt / slices;
                n[0] = std::sin(th) * std::cos(ph); n[1] = std::cos(th); n[2] = std::sin(th) * std::sin(ph);
                o[0] = 5 + 2.5f * n[0]; o[1] = 3 + 2.5f * n[1]; o[2] = 5 + 2.5f * n[2];
            };
            float q[4][3], qn[4][3];
            pt(s, t, q[0], qn[0]); pt(s + 1, t, q[1], qn[1]); pt(s + 1, t + 1, q[2], qn[2]); pt(s, t + 1, q[3], qn[3]);
            const uint32_t base = (uint32_t)(P.size() / 3);
            for (int k = 0; k < 4; ++k) { P.insert(P.end(), q[k], q[k] + 3); N.insert(N.end(), qn[k], qn[k] + 3); }
            for (uint32_t k : {0u, 1u, 2u, 0u, 2u, 3u}) I.push_back(base + k);
            M.push_back(0);
            M.push_back(0);
        }
    rt_material mats[3] = {{RT_MAT_DIFFUSE, {0, 0, 0}, 0, 0}, {RT_MAT_DIFFUSE, {0.0001f, -0.1f, 25.f}, 0, 0},
                           {RT_MAT_DIFFUSE, {0, 0, 0}, 10.f, 0}};
    rt_light light{};
    light.type = RT_LIGHT_QUAD;
    const float lp[3] = {4, 9.99f, 4}, le1[3] = {0, 0, 2}, le2[3] = {2, 0, 0};
    for (int k = 0; k < 3; ++k) { light.p[k] = lp[k]; light.e1[k] = le1[k]; light.e2[k] = le2[k]; light.n[k] = dn[k]; }
    light.material = 2;
    rt_scene_desc sd{};
    sd.n_vertices = (int)(P.size() / 3);
    sd.positions = P.data();
    sd.normals = N.data();
    sd.n_triangles = (int)(I.size() / 3);
    sd.indices = I.data();
    ident(sd.object_to_render);
    for (int i = 0; i < 9; ++i) sd.normal_to_render[i] = (i % 4 == 0) ? 1.f : 0.f;
    sd.cull_backfaces = 1;
    sd.cull_look[2] = 1;
    sd.octree_capacity = 8;
    sd.tri_material = M.data();
    sd.n_materials = 3;
    sd.materials = mats;
    sd.n_lights = 1;
    sd.lights = &light;
    const int W = 32, H = 24;
    rt_camera_desc cam{};
    cam.type = RT_CAMERA_PERSPECTIVE;
    // raster (x, y) -> camera (x / W - .5, y / H - .5, 1): the camera looks down +z from (5, 5, -8)
    for (int i = 0; i < 16; ++i) cam.raster_to_camera[i] = 0.f;
    cam.raster_to_camera[0] = 1.f / W; cam.raster_to_camera[5] = 1.f / H;
    cam.raster_to_camera[12] = -.5f; cam.raster_to_camera[13] = -.5f; cam.raster_to_camera[14] = 1.f;
    cam.raster_to_camera[15] = 1.f;
    ident(cam.camera_to_world);
    cam.camera_to_world[12] = 5; cam.camera_to_world[13] = 5; cam.camera_to_world[14] = -8;
    rt_sampler_desc smp{RT_SAMPLER_STRATIFIED, 2, 2, 1, 0, 0};
    rt_film_desc film{W, H, RT_FILTER_BOX, {0.5f, 0.5f}, 1.f / 106.856895f, 0.f, RT_SENSOR_XYZ, RT_ILLUM_D65};
    int bad = 0;
    for (int kind : {RT_INTEGRATOR_REFERENCE, RT_INTEGRATOR_PATH, RT_INTEGRATOR_PATH_MIS}) {
        rt_integrator_desc integ{kind, 4, {0.5f, 0.5f, 0.5f}};
        void* h = orc_scene_create(&sd, &cam, &smp, &film, &integ);
        int nn = 0, nr = 0, depth = 0;
        orc_octree_info(h, &nn, &nr, &depth);
        if (depth < 1) { std::printf("expected a multi-level octree\n"); bad = 1; }
        std::vector<float> px4((size_t)W * H * 4, 0.f);
        std::vector<int64_t> ctr(5, 0);
        orc_render(h, 0, 4, px4.data(), 4, ctr.data(), nullptr, 0);
        std::vector<uint8_t> out((size_t)W * H * 3);
        orc_resolve(h, px4.data(), out.data());
        // random rays through the box: canonical rule vs the BFS on 4 threads
        std::mt19937 rng(7);
        std::uniform_real_distribution<float> U(0.5f, 9.5f), D(-1.f, 1.f);
        const int n = 4000;
        std::vector<float> ro(3 * n), rd(3 * n), tmax(n);
        for (int i = 0; i < n; ++i) {
            float v[3] = {D(rng), D(rng), D(rng)};
            float l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]) + 1e-6f;
            for (int k = 0; k < 3; ++k) { ro[3 * i + k] = U(rng); rd[3 * i + k] = v[k] / l; }
            tmax[i] = U(rng);
        }
        int64_t st[8];
        orc_canonical_check(h, n, ro.data(), rd.data(), tmax.data(), kind == RT_INTEGRATOR_REFERENCE, 4, st);
        if (st[0] || st[2]) { std::printf("canonical mismatch %lld %lld\n", (long long)st[0], (long long)st[2]); bad = 1; }
        std::printf("integrator %d: nodes %d depth %d samples %lld rays %lld hits %lld\n", kind, nn, depth,
                    (long long)ctr[3], (long long)st[6], (long long)st[4]);
        orc_scene_destroy(h);
    }
    return bad;
}
