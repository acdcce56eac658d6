// Drives the C++ plugin surface on the GPU (rt_host.hpp): RayTracePlugin::build
// with the config-1 scene at 64x36, 2 spp per frame, depth 8, then three
// frames through RayTracePlugin::frame, editing one sphere and one material
// between frames 1 and 2 (the node's dirty tracking uploads only those).
// Writes: u32 frames, then per frame u32 frame0, u32 segments (low 32 bits),
// W*H*4 floats; then u32 uploads.full, spheres, materials.
// tests/test_host_cpp.py renders the same frames with the oracle.
#include <cstdio>

#include "rt_host.hpp"

int main(int argc, char** argv) {
    if (argc < 2) return 2;
    try {
        rt::World world;
        world.camera = rt::RayTraceCamera{64, 36};
        rt::RayTraceSettings s;
        s.samples_per_ray = 2;
        s.max_depth = 8;
        s.flags = argc > 2 ? (uint32_t)atoi(argv[2]) : 0u;
        rt::RayTracePlugin plugin(s, rt::config1_scene());
        rt::RayTraceNode node = plugin.build(world);
        FILE* f = fopen(argv[1], "wb");
        if (!f) return 3;
        const uint32_t frames = 3;
        fwrite(&frames, 4, 1, f);
        for (uint32_t i = 0; i < frames; ++i) {
            if (i == 1) {  // scene edit between frames
                world.scene->spheres[1].radius = 0.75f;
                world.scene->materials.at(2).color = {0.9f, 0.2f, 0.1f, 1.0f};
                world.scene->materials.at(2).reflectance = rt::Reflectance::Metallic;
                world.scene->materials.at(2).fuzziness = 0.3f;
            }
            const uint32_t f0 = world.frame_counter.frame;
            const rt_stats st = rt::RayTracePlugin::frame(world, node);
            const uint32_t segs = (uint32_t)st.segments;
            fwrite(&f0, 4, 1, f);
            fwrite(&segs, 4, 1, f);
            fwrite(world.output.data.data(), 4, world.output.data.size(), f);
        }
        const uint32_t up[3] = {node.uploads().full, node.uploads().spheres,
                                node.uploads().materials};
        fwrite(up, 4, 3, f);
        fclose(f);
    } catch (const rt::Error& e) {
        fprintf(stderr, "rt error %d: %s\n", e.status, e.what());
        return 4;
    }
    return 0;
}
