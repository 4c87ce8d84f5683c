// Sanitizer driver for the host-only C-ABI entry points (rt_load_obj, rt_mesh_free, rt_image_write,
// rt_rgb_to_sigmoid, rt_rgb_fit_sigmoid: csrc/rt_io.cpp and csrc/rt_color.cpp, no GPU), built with ASan + UBSan by
// tests/sanitize/Makefile and run by tests/test_sanitizers.py, including malformed inputs and the exception firewall.
#include <cstdio>
#include <cstdlib>
#include <string>

#include "../../include/rtmi355x.h"

int main(int argc, char** argv) {
    const std::string dir = argc > 1 ? argv[1] : "/tmp";
    int bad = 0;
    auto expect = [&](bool ok, const char* what) {
        if (!ok) { std::printf("FAIL %s\n", what); bad = 1; }
    };
    const std::string obj = dir + "/s.obj", obj2 = dir + "/bad.obj";
    FILE* f = std::fopen(obj.c_str(), "w");
    std::fputs("v 0 0 0\nv 1 0 0\nv 1 1 0\nv 0 1 0\nvt 0 0\nvt 1 1\nvn 0 0 1\nf 1/1/1 2/2/1 3/1/1 4/2/1\nf -4 -3 -2\n", f);
    std::fclose(f);
    f = std::fopen(obj2.c_str(), "w");
    std::fputs("v 0 0 0\nf 1 2 99\n", f);
    std::fclose(f);
    rt_mesh* m = nullptr;
    expect(rt_load_obj(obj.c_str(), &m) == RT_OK && m && m->n_triangles == 3, "load obj");
    rt_mesh_free(m);
    m = nullptr;
    expect(rt_load_obj(obj2.c_str(), &m) == RT_E_ARG && !m, "reject bad obj");
    expect(rt_load_obj((dir + "/missing.obj").c_str(), &m) == RT_E_ARG, "missing obj");
    unsigned char img[5 * 3 * 3];
    for (int i = 0; i < (int)sizeof(img); ++i) img[i] = (unsigned char)(i * 17);
    expect(rt_image_write((dir + "/a.png").c_str(), 5, 3, img, 1) == RT_OK, "png");
    expect(rt_image_write((dir + "/a.ppm").c_str(), 5, 3, img, 0) == RT_OK, "ppm");
    expect(rt_image_write((dir + "/a.png").c_str(), 0, 3, img, 0) == RT_E_ARG, "bad size");
    for (int i = 0; i < 64; ++i) {
        float rgb[3] = {(float)((i * 37) % 101) / 100.f, (float)((i * 53) % 101) / 100.f, (float)((i * 71) % 101) / 100.f};
        float c[3];
        expect(rt_rgb_to_sigmoid(rgb, c) == RT_OK, "table lookup");
        if (i % 16 == 0) expect(rt_rgb_fit_sigmoid(rgb, c) == RT_OK, "fit");
    }
    float out_of_range[3] = {1.5f, 0.f, 0.f}, c[3];
    expect(rt_rgb_to_sigmoid(out_of_range, c) == RT_E_ARG, "range");
    // the release entry points are exempt from fault injection: a mesh loaded before the fault is still freed
    // (LeakSanitizer fails the run otherwise)
    expect(rt_load_obj(obj.c_str(), &m) == RT_OK && m, "load before fault");
    setenv("RTMI_FAULT_INJECT", "bad_alloc", 1);
    rt_mesh* m2 = nullptr;
    expect(rt_load_obj(obj.c_str(), &m2) == RT_E_OOM && !m2, "firewall");
    rt_mesh_free(m);
    unsetenv("RTMI_FAULT_INJECT");
    return bad;
}
