// rt_host.hpp -- C++ host side above the C-ABI (include/rt_hip.h): the
// reference's main-world / render-world interface for the path tracer,
// restated in C++ because the reference is compiled Rust and rustc is not in
// this image (the Rust drop-in files themselves are in bevy_shim/).
//
// Mirrors (all paths under the reference's src/):
//   Reflectance            ray_trace_materials.rs:12-17
//   RayTraceMaterial       ray_trace_materials.rs:25-31
//   MaterialCache          ray_trace_materials.rs:50-67 (IndexMap: insertion order = GPU index)
//   init_materials_cache   ray_trace_materials.rs:83-127
//   Sphere                 sphere.rs:31-35 (+ its Transform translation, 171-176)
//   init_spheres           sphere.rs:37-148 (seeded PCG32 instead of thread_rng: SURVEY D4)
//   extract / prepare      sphere.rs:166-197, ray_trace_materials.rs:129-164
//   RayTraceCamera         camera.rs:13-37; CameraGPU packing ray_trace_camera.rs:43-68
//   GlobalsGPU.frame       ray_trace_globals.rs:56-68 (+1 per frame per sample)
//   RayTraceOutputImage    ray_trace_output.rs:19-61 (Rgba32Float W x H)
//   RayTraceNode           ray_trace_node.rs:173-224 (update: upload what changed; run: one frame)
//   RayTracePlugin         plugin.rs:19-47 + SphereRenderPlugin sphere.rs:150-164
// The same API exists in Python (bevy_raytrace_amd/scene.py, camera.py,
// plugin.py); both produce byte-identical scene and camera records
// (tests/test_host_cpp.py). Errors from the library throw rt::Error with the
// library's message (rt_last_error); nothing here renders on the CPU.
#pragma once

#include <array>
#include <cstdint>
#include <optional>
#include <stdexcept>
#include <string>
#include <unordered_map>
#include <utility>
#include <vector>

#include "rt_hip.h"

namespace rt {

struct Error : std::runtime_error {
    int status;
    Error(int s, const std::string& msg) : std::runtime_error(msg), status(s) {}
};

enum class Reflectance : int32_t { Lambertian = 0, Metallic = 1, Dielectric = 2 };

struct RayTraceMaterial {
    std::array<float, 4> color{0.0f, 0.0f, 0.0f, 1.0f};
    Reflectance reflectance = Reflectance::Lambertian;
    float fuzziness = 0.0f;
    float index_of_refraction = 0.0f;
};

// Ordered name -> material map (IndexMap semantics: re-inserting a name keeps
// its position and replaces the value).
class MaterialCache {
public:
    void insert(const std::string& name, const RayTraceMaterial& m);
    const RayTraceMaterial& get(const std::string& name) const;
    uint32_t get_index_of(const std::string& name) const;
    size_t size() const { return items_.size(); }
    RayTraceMaterial& at(size_t i) { return items_[i].second; }
    // MaterialGPU records (ray_trace_materials.rs:144-153: colour passed raw)
    std::vector<rt_material> to_gpu() const;

private:
    std::vector<std::pair<std::string, RayTraceMaterial>> items_;
    std::unordered_map<std::string, size_t> index_;
};

struct Sphere {
    std::array<float, 3> center{0.0f, 0.0f, 0.0f};
    float radius = 1.0f;
    uint32_t material = 0;
};

struct Scene {
    std::vector<Sphere> spheres;
    MaterialCache materials;
    std::string name = "scene";
    // ObjectListGPU.spheres (sphere.rs:166-197), query order = spawn order
    std::vector<rt_sphere> objects_gpu() const;
    std::vector<rt_material> materials_gpu() const { return materials.to_gpu(); }
};

// PCG-XSH-RR 32; f32() in [0, 1) with 24 bits (same stream as scene.py Pcg32).
class Pcg32 {
public:
    explicit Pcg32(uint64_t seed, uint64_t stream = 54);
    uint32_t next_u32();
    float f32();

private:
    uint64_t state_ = 0, inc_ = 0;
};

// split: "reference" (sphere.rs:61-91), "rtiow" (the commented RTIOW block,
// sphere.rs:101-120) or "config1".
MaterialCache init_materials_cache(const std::string& split = "reference");
Scene init_spheres(int sphere_dim = 7, const std::string& split = "reference",
                   uint64_t seed = 20221015, std::optional<uint32_t> max_grid = std::nullopt);
Scene config1_scene();
Scene rtiow_final_scene(uint64_t seed = 20221015);
Scene ten_thousand_scene(uint64_t seed = 20221015);
Scene reference_scene(uint64_t seed = 20221015);

// Translation + rotation basis (columns right, up, back), Bevy-style.
struct Transform {
    std::array<float, 3> translation{0.0f, 0.0f, 0.0f};
    std::array<std::array<float, 3>, 3> basis{{{1, 0, 0}, {0, 1, 0}, {0, 0, 1}}};  // [col][row]
    static Transform from_xyz(float x, float y, float z);
    // Transform::looking_at: back = normalize(eye - target),
    // right = normalize(up x back), up' = back x right (f32 throughout)
    Transform looking_at(std::array<float, 3> target,
                         std::array<float, 3> up = {0.0f, 1.0f, 0.0f}) const;
    std::array<float, 16> compute_matrix() const;  // column-major, m[col*4 + row]
};

// src/ray_trace_camera.rs:12, 59-61
constexpr float CAMERA_FOV = 1.5708f;
constexpr float IMAGE_PLANE_DISTANCE = 10.0f;
constexpr float LENS_FOCAL_LENGTH = 0.1f;
inline float fstop_default() { return 1.0f / 32.0f; }

struct RayTraceCamera {
    uint32_t render_width = 1920;
    uint32_t render_height = 1080;
    Transform transform = Transform::from_xyz(13.0f, 2.0f, 3.0f).looking_at({0.0f, 0.0f, 0.0f});
    rt_camera to_gpu() const;  // CameraGPU exactly as ray_trace_camera.rs:43-68 packs it
};

// RAII owner of an rt_ctx (one per device).
class Renderer {
public:
    explicit Renderer(int device = 0);
    ~Renderer();
    Renderer(const Renderer&) = delete;
    Renderer& operator=(const Renderer&) = delete;
    void set_scene(const std::vector<rt_sphere>& sp, const std::vector<rt_material>& mt);
    void update_spheres(uint32_t first, const rt_sphere* sp, uint32_t count);
    void update_materials(uint32_t first, const rt_material* mt, uint32_t count);
    // allocate the work buffers of nframes-frame renders of p up front (rt_reserve)
    void reserve(const rt_params& p, uint32_t nframes);
    // synchronous frame into host RGBA32F (rows x width x 4 floats)
    rt_stats render(const rt_camera& cam, const rt_params& p, float* out);
    rt_ctx* ctx() const { return ctx_; }

private:
    void check(int rc) const;
    rt_ctx* ctx_ = nullptr;
};

rt_params make_params(uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth,
                      uint32_t frame0 = 0, uint32_t flags = 0);

// ---- plugin surface -------------------------------------------------------
constexpr uint32_t RENDER_TARGET_W = 1920, RENDER_TARGET_H = 1080;  // src/lib.rs:25
constexpr uint32_t SAMPLES_PER_RAY = 1;                             // src/lib.rs:26
constexpr uint32_t MAX_DEPTH = 3;                                   // ray_trace_node.rs:213

struct RayTraceOutputImage {
    uint32_t width = 0, height = 0;
    std::vector<float> data;  // height x width x 4, Rgba32Float
};

struct RayTraceSettings {
    uint32_t samples_per_ray = SAMPLES_PER_RAY;
    uint32_t max_depth = MAX_DEPTH;
    int device = 0;
    uint32_t flags = 0;
};

struct FrameCounter {
    uint32_t frame = 0;
};

// The render world's resources the node reads (a plain struct: the resource
// map of the reference's World for exactly these types).
struct World {
    std::optional<Scene> scene;
    std::optional<RayTraceCamera> camera;
    RayTraceSettings settings;
    FrameCounter frame_counter;
    RayTraceOutputImage output;
};

struct UploadCounts {
    uint32_t full = 0, spheres = 0, materials = 0;
};

class RayTraceNode {
public:
    // extract + prepare (sphere.rs:166-197): upload only what changed (one
    // contiguous dirty range of records per list; a count change re-uploads all)
    void update(World& world);
    // one frame into world.output; advances the frame counter by spp
    rt_stats run(World& world);
    const UploadCounts& uploads() const { return uploads_; }
    const rt_stats& last_stats() const { return last_; }

private:
    std::optional<Renderer> renderer_;
    std::vector<rt_sphere> sp_;
    std::vector<rt_material> mt_;
    UploadCounts uploads_;
    rt_stats last_{};
    // (width, height, spp, max_depth) the work buffers were last sized for
    std::array<uint32_t, 4> reserved_{};
};

class RayTracePlugin {
public:
    explicit RayTracePlugin(RayTraceSettings s = {}, std::optional<Scene> scene = std::nullopt)
        : settings_(s), scene_(std::move(scene)) {}
    // installs the camera (camera.rs:31-37), settings, frame counter, output
    // image and the scene (sphere.rs:37-148) unless present; returns the node
    RayTraceNode build(World& world) const;
    // one Render-stage pass: update then run (Bevy's graph runner order)
    static rt_stats frame(World& world, RayTraceNode& node);

private:
    RayTraceSettings settings_;
    std::optional<Scene> scene_;
};

}  // namespace rt
