// rt_host.cpp -- see rt_host.hpp. Every f32 expression is written in the
// order of the reference's Rust / the Python mirror and compiled with
// -ffp-contract=off, so scene and camera records match byte for byte.
#include "rt_host.hpp"

#include <cmath>
#include <cstring>

namespace rt {

// ---- materials --------------------------------------------------------------
void MaterialCache::insert(const std::string& name, const RayTraceMaterial& m) {
    auto it = index_.find(name);
    if (it != index_.end()) {
        items_[it->second].second = m;
        return;
    }
    index_.emplace(name, items_.size());
    items_.emplace_back(name, m);
}

const RayTraceMaterial& MaterialCache::get(const std::string& name) const {
    return items_.at(index_.at(name)).second;
}

uint32_t MaterialCache::get_index_of(const std::string& name) const {
    return (uint32_t)index_.at(name);
}

std::vector<rt_material> MaterialCache::to_gpu() const {
    std::vector<rt_material> out(items_.size());
    for (size_t i = 0; i < items_.size(); ++i) {
        const RayTraceMaterial& m = items_[i].second;
        rt_material g{};
        for (int c = 0; c < 4; ++c) g.color[c] = m.color[c];
        g.reflectance = (int32_t)m.reflectance;
        g.fuzziness = m.fuzziness;
        g.index_of_refraction = m.index_of_refraction;
        out[i] = g;
    }
    return out;
}

std::vector<rt_sphere> Scene::objects_gpu() const {
    std::vector<rt_sphere> out(spheres.size());
    for (size_t i = 0; i < spheres.size(); ++i) {
        rt_sphere g{};
        for (int c = 0; c < 3; ++c) g.center[c] = spheres[i].center[c];
        g.radius = spheres[i].radius;
        g.material = spheres[i].material;
        out[i] = g;
    }
    return out;
}

// ---- seeded generator ----------------------------------------------
Pcg32::Pcg32(uint64_t seed, uint64_t stream) {
    inc_ = (stream << 1) | 1u;
    state_ = 0;
    next_u32();
    state_ += seed;
    next_u32();
}

uint32_t Pcg32::next_u32() {
    const uint64_t old = state_;
    state_ = old * 6364136223846793005ull + inc_;
    const uint32_t xorshifted = (uint32_t)(((old >> 18) ^ old) >> 27);
    const uint32_t rot = (uint32_t)(old >> 59);
    return (xorshifted >> rot) | (xorshifted << ((0u - rot) & 31u));
}

float Pcg32::f32() { return (float)((double)(next_u32() >> 8) * (1.0 / 16777216.0)); }

MaterialCache init_materials_cache(const std::string& split) {
    using R = Reflectance;
    MaterialCache c;
    c.insert("ground", {{0.5f, 0.5f, 0.5f, 1.0f}, R::Lambertian, 1.0f, 0.0f});
    if (split == "reference") {
        c.insert("center", {{0.7f, 0.3f, 0.3f, 1.0f}, R::Lambertian, 1.0f, 0.0f});
        c.insert("left", {{0.8f, 0.8f, 0.8f, 1.0f}, R::Metallic, 0.1f, 1.5f});
        c.insert("right", {{0.7f, 0.6f, 0.5f, 1.0f}, R::Metallic, 0.0f, 1.5f});
    } else if (split == "rtiow") {
        c.insert("center", {{1.0f, 1.0f, 1.0f, 1.0f}, R::Dielectric, 0.0f, 1.5f});
        c.insert("left", {{0.4f, 0.2f, 0.1f, 1.0f}, R::Lambertian, 1.0f, 0.0f});
        c.insert("right", {{0.7f, 0.6f, 0.5f, 1.0f}, R::Metallic, 0.0f, 1.5f});
    } else if (split == "config1") {
        c.insert("center", {{0.7f, 0.3f, 0.3f, 1.0f}, R::Lambertian, 1.0f, 0.0f});
        c.insert("left", {{1.0f, 1.0f, 1.0f, 1.0f}, R::Dielectric, 0.0f, 1.5f});
        c.insert("right", {{0.7f, 0.6f, 0.5f, 1.0f}, R::Metallic, 0.0f, 1.5f});
    } else {
        throw std::invalid_argument("unknown split " + split);
    }
    return c;
}

// sphere.rs:37-148. Per candidate the draws are centre.x, centre.z, then (if
// accepted) the material; C++ argument order is unspecified, so every draw is
// its own statement.
Scene init_spheres(int dim, const std::string& split, uint64_t seed,
                   std::optional<uint32_t> max_grid) {
    using R = Reflectance;
    Pcg32 rng(seed);
    Scene sc;
    sc.materials = init_materials_cache(split);
    sc.spheres.push_back({{0.0f, -1000.0f, -1.0f}, 1000.0f, sc.materials.get_index_of("ground")});
    const float refp[3] = {4.0f, 0.2f, 0.0f};
    uint32_t accepted = 0;
    for (int a = -dim; a < dim; ++a) {
        for (int b = -dim; b < dim; ++b) {
            const float ux = rng.f32();
            const float cx = (float)a + 0.9f * ux;
            const float uz = rng.f32();
            const float cz = (float)b + 0.9f * uz;
            const float d0 = cx - refp[0], d1 = 0.2f - refp[1], d2 = cz - refp[2];
            const float len = std::sqrt((d0 * d0 + d1 * d1) + d2 * d2);
            if (!(len > 0.9f)) continue;
            if (max_grid && accepted >= *max_grid) continue;
            const std::string name = "material_" + std::to_string(a) + "_" + std::to_string(b);
            const float choose = rng.f32();
            RayTraceMaterial m;
            if (split == "reference" || split == "config1") {
                if (choose < 0.8f) {
                    const float r = rng.f32(), g = rng.f32(), bl = rng.f32();
                    m = {{r, g, bl, 1.0f}, R::Lambertian, 1.0f, 0.0f};
                } else {
                    const float r = rng.f32(), g = rng.f32(), bl = rng.f32();
                    const float fz = rng.f32() * 0.5f;
                    m = {{r, g, bl, 1.0f}, R::Metallic, fz, 0.0f};
                }
            } else {
                if (choose < 0.8f) {
                    float c1[3], c2[3];
                    for (float& v : c1) v = rng.f32();
                    for (float& v : c2) v = rng.f32();
                    m = {{c1[0] * c2[0], c1[1] * c2[1], c1[2] * c2[2], 1.0f}, R::Lambertian, 1.0f,
                         0.0f};
                } else if (choose < 0.95f) {
                    float col[3];
                    for (float& v : col) v = 0.5f + 0.5f * rng.f32();
                    const float fz = 0.5f * rng.f32();
                    m = {{col[0], col[1], col[2], 1.0f}, R::Metallic, fz, 0.0f};
                } else {
                    m = {{1.0f, 1.0f, 1.0f, 1.0f}, R::Dielectric, 0.0f, 1.5f};
                }
            }
            sc.materials.insert(name, m);
            sc.spheres.push_back({{cx, 0.2f, cz}, 0.2f, sc.materials.get_index_of(name)});
            ++accepted;
        }
    }
    sc.spheres.push_back({{0.0f, 1.0f, 0.0f}, 1.0f, sc.materials.get_index_of("center")});
    sc.spheres.push_back({{-4.0f, 1.0f, 0.0f}, 1.0f, sc.materials.get_index_of("left")});
    sc.spheres.push_back({{4.0f, 1.0f, 0.0f}, 1.0f, sc.materials.get_index_of("right")});
    sc.name = "grid" + std::to_string(dim) + "_" + split + "_" + std::to_string(seed);
    return sc;
}

Scene config1_scene() {
    Scene sc;
    sc.materials = init_materials_cache("config1");
    sc.spheres = {{{0.0f, -1000.0f, -1.0f}, 1000.0f, 0},
                  {{0.0f, 1.0f, 0.0f}, 1.0f, 1},
                  {{-4.0f, 1.0f, 0.0f}, 1.0f, 2},
                  {{4.0f, 1.0f, 0.0f}, 1.0f, 3}};
    sc.name = "config1";
    return sc;
}

Scene rtiow_final_scene(uint64_t seed) { return init_spheres(11, "rtiow", seed); }
Scene ten_thousand_scene(uint64_t seed) { return init_spheres(50, "rtiow", seed, 9996u); }
Scene reference_scene(uint64_t seed) { return init_spheres(7, "reference", seed); }

// ---- camera -----------------------------------------------------------------------
namespace {
using V3 = std::array<float, 3>;
V3 cross(const V3& a, const V3& b) {
    return {a[1] * b[2] - a[2] * b[1], a[2] * b[0] - a[0] * b[2], a[0] * b[1] - a[1] * b[0]};
}
V3 normalize(const V3& v) {
    const float l = std::sqrt((v[0] * v[0] + v[1] * v[1]) + v[2] * v[2]);
    return {v[0] / l, v[1] / l, v[2] / l};
}
}  // namespace

Transform Transform::from_xyz(float x, float y, float z) {
    Transform t;
    t.translation = {x, y, z};
    return t;
}

Transform Transform::looking_at(std::array<float, 3> target, std::array<float, 3> up) const {
    const V3 back = normalize({translation[0] - target[0], translation[1] - target[1],
                               translation[2] - target[2]});
    const V3 right = normalize(cross(up, back));
    const V3 upv = cross(back, right);
    Transform t;
    t.translation = translation;
    t.basis = {right, upv, back};
    return t;
}

std::array<float, 16> Transform::compute_matrix() const {
    std::array<float, 16> m{};
    for (int c = 0; c < 3; ++c)
        for (int r = 0; r < 3; ++r) m[c * 4 + r] = basis[c][r];
    m[12] = translation[0];
    m[13] = translation[1];
    m[14] = translation[2];
    m[15] = 1.0f;
    return m;
}

rt_camera RayTraceCamera::to_gpu() const {
    rt_camera c;
    std::memset(&c, 0, sizeof(c));
    const std::array<float, 16> m = transform.compute_matrix();
    std::memcpy(c.transform, m.data(), sizeof(c.transform));
    for (int i = 0; i < 3; ++i) {
        c.forward[i] = -transform.basis[2][i];
        c.up[i] = transform.basis[1][i];
        c.right[i] = transform.basis[0][i];
        c.position[i] = transform.translation[i];
    }
    c.fov = CAMERA_FOV;
    c.image_plane_distance = IMAGE_PLANE_DISTANCE;
    c.lens_focal_length = LENS_FOCAL_LENGTH;
    c.fstop = fstop_default();
    return c;
}

// ---- renderer -------------------------------------------------------------------
Renderer::Renderer(int device) {
    const int rc = rt_create(device, &ctx_);
    if (rc) throw Error(rc, rt_last_error(nullptr) ? rt_last_error(nullptr) : "rt_create failed");
}

Renderer::~Renderer() {
    if (ctx_) rt_destroy(ctx_);
}

void Renderer::check(int rc) const {
    if (rc) {
        const char* m = rt_last_error(ctx_);
        throw Error(rc, m ? m : "rt error");
    }
}

void Renderer::set_scene(const std::vector<rt_sphere>& sp, const std::vector<rt_material>& mt) {
    check(rt_set_scene(ctx_, sp.data(), (uint32_t)sp.size(), mt.data(), (uint32_t)mt.size()));
}

void Renderer::update_spheres(uint32_t first, const rt_sphere* sp, uint32_t count) {
    check(rt_update_spheres(ctx_, first, sp, count));
}

void Renderer::update_materials(uint32_t first, const rt_material* mt, uint32_t count) {
    check(rt_update_materials(ctx_, first, mt, count));
}

void Renderer::reserve(const rt_params& p, uint32_t nframes) { check(rt_reserve(ctx_, &p, nframes)); }

rt_stats Renderer::render(const rt_camera& cam, const rt_params& p, float* out) {
    rt_stats st{};
    check(rt_render(ctx_, &cam, &p, out, &st));
    return st;
}

rt_params make_params(uint32_t width, uint32_t height, uint32_t spp, uint32_t max_depth,
                      uint32_t frame0, uint32_t flags) {
    rt_params p;
    std::memset(&p, 0, sizeof(p));
    p.width = width;
    p.height = height;
    p.spp = spp;
    p.max_depth = max_depth;
    p.frame0 = frame0;
    p.row_block = 8;
    p.shard_count = 1;
    p.shard_index = 0;
    p.flags = flags;
    return p;
}

// ---- plugin surface -------------------------------------------------------------
namespace {
// [first, last) of the records whose bytes differ, or first == last
template <typename T>
std::pair<size_t, size_t> dirty_range(const std::vector<T>& a, const std::vector<T>& b) {
    size_t lo = a.size(), hi = 0;
    for (size_t i = 0; i < a.size(); ++i)
        if (std::memcmp(&a[i], &b[i], sizeof(T)) != 0) {
            if (i < lo) lo = i;
            hi = i + 1;
        }
    return lo < hi ? std::make_pair(lo, hi) : std::make_pair(size_t(0), size_t(0));
}
}  // namespace

void RayTraceNode::update(World& world) {
    if (!renderer_) renderer_.emplace(world.settings.device);
    const Scene& sc = world.scene.value();
    std::vector<rt_sphere> sp = sc.objects_gpu();
    std::vector<rt_material> mt = sc.materials_gpu();
    if (uploads_.full == 0 || sp.size() != sp_.size() || mt.size() != mt_.size()) {
        renderer_->set_scene(sp, mt);
        ++uploads_.full;
    } else {
        const auto dm = dirty_range(mt, mt_);
        if (dm.second > dm.first) {
            renderer_->update_materials((uint32_t)dm.first, mt.data() + dm.first,
                                        (uint32_t)(dm.second - dm.first));
            ++uploads_.materials;
        }
        const auto ds = dirty_range(sp, sp_);
        if (ds.second > ds.first) {
            renderer_->update_spheres((uint32_t)ds.first, sp.data() + ds.first,
                                      (uint32_t)(ds.second - ds.first));
            ++uploads_.spheres;
        }
    }
    sp_ = std::move(sp);
    mt_ = std::move(mt);
    // size the frame's work buffers here, as the reference re-sizes its ray
    // and intersection buffers in prepare when the ray count changes
    // (ray_trace_rays.rs:50-66), not inside run
    if (world.camera) {
        const std::array<uint32_t, 4> key{world.camera->render_width, world.camera->render_height,
                                          world.settings.samples_per_ray, world.settings.max_depth};
        if (key != reserved_) {
            renderer_->reserve(make_params(key[0], key[1], key[2], key[3], 0,
                                           world.settings.flags), 1);
            reserved_ = key;
        }
    }
}

rt_stats RayTraceNode::run(World& world) {
    const RayTraceCamera& cam = world.camera.value();
    RayTraceOutputImage& out = world.output;
    out.width = cam.render_width;
    out.height = cam.render_height;
    out.data.resize((size_t)out.width * out.height * 4);
    const rt_params p = make_params(cam.render_width, cam.render_height,
                                    world.settings.samples_per_ray, world.settings.max_depth,
                                    world.frame_counter.frame, world.settings.flags);
    last_ = renderer_.value().render(cam.to_gpu(), p, out.data.data());
    world.frame_counter.frame += world.settings.samples_per_ray;  // ray_trace_globals.rs:67
    return last_;
}

RayTraceNode RayTracePlugin::build(World& world) const {
    if (!world.camera) world.camera = RayTraceCamera{RENDER_TARGET_W, RENDER_TARGET_H};
    world.settings = settings_;
    world.frame_counter = FrameCounter{};
    world.output.width = world.camera->render_width;
    world.output.height = world.camera->render_height;
    world.output.data.assign((size_t)world.output.width * world.output.height * 4, 1.0f);
    if (!world.scene) world.scene = scene_ ? *scene_ : init_spheres();
    return RayTraceNode{};
}

rt_stats RayTracePlugin::frame(World& world, RayTraceNode& node) {
    node.update(world);
    return node.run(world);
}

}  // namespace rt
