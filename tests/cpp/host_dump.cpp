// Dumps the C++ host mirror's scene and camera records (no GPU work):
//   for each scene (config1, reference, rtiow, ten_thousand):
//     u32 n, n x rt_sphere, u32 m, m x rt_material
//   then the default RayTraceCamera's rt_camera.
// tests/test_host_cpp.py compares the bytes with the Python mirror's.
#include <cstdio>
#include <vector>

#include "rt_host.hpp"

template <typename T>
static void put(FILE* f, const std::vector<T>& v) {
    const uint32_t n = (uint32_t)v.size();
    fwrite(&n, 4, 1, f);
    if (n) fwrite(v.data(), sizeof(T), n, f);
}

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    FILE* f = fopen(argv[1], "wb");
    if (!f) return 3;
    const rt::Scene scenes[] = {rt::config1_scene(), rt::reference_scene(),
                                rt::rtiow_final_scene(), rt::ten_thousand_scene()};
    for (const rt::Scene& s : scenes) {
        put(f, s.objects_gpu());
        put(f, s.materials_gpu());
    }
    const rt_camera cam = rt::RayTraceCamera{}.to_gpu();
    fwrite(&cam, sizeof(cam), 1, f);
    fclose(f);
    return 0;
}
