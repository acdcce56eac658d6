/*
 * rt_oracle.c — CPU oracle (TEST INFRASTRUCTURE ONLY; see rt_oracle.h).
 *
 * Scalar restatement of brandon-reinhart/bevy_raytrace's WGSL path:
 *   clear.wgsl:71-87 -> generate.wgsl:66-129 -> D x (intersect.wgsl:94-163,
 *   shade.wgsl:105-258) -> collect.wgsl:99-125, scheduled as in
 *   src/ray_trace_node.rs:195-224 with the loop count generalised to D.
 *
 * Build: gcc -O2 -ffp-contract=off -fno-fast-math (oracle/Makefile). Every f32
 * operation below is one IEEE-754 round-to-nearest op; no FMA contraction, no
 * reassociation. Op forms fixed by this restatement (the WGSL leaves them to
 * the driver -- the one part the WGSL-interpreter fixtures cannot pin):
 *   dot(a,b)     = (a.x*b.x + a.y*b.y) + a.z*b.z
 *   length(v)    = sqrt(dot(v,v))                (correctly rounded sqrt)
 *   normalize(v) = v / length(v)                 (3 correctly rounded divides)
 *   sqr(x)       = x*x
 *   pow(x, 5.0)  = ((x*x)*(x*x))*x
 *   tan(fov/2)   = (float)tan((double)(fov/2))   (host, once per frame)
 *   M*v          = ((M[0]*v.x + M[1]*v.y) + M[2]*v.z) + M[3]*v.w (columns)
 * Documented divergences: exact integer pixel
 * addressing, every pixel processed, sample s == frame frame0+s, samples summed
 * in blocks of RT_SAMPLE_BLOCK (rt_hip.h).
 */
#include "rt_oracle.h"

#include <math.h>
#include <pthread.h>
#include <stdlib.h>
#include <string.h>

#define VERY_FAR 1e20f          /* every shader, line 1 */
#define EPSILON  0.001f         /* every shader, line 2 */
#define PI_F     3.14159265358979f

typedef struct { float x, y, z; } v3;

static inline v3 mk(float x, float y, float z) { v3 r = {x, y, z}; return r; }
static inline v3 add(v3 a, v3 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z); }
static inline v3 sub(v3 a, v3 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z); }
static inline v3 mul(v3 a, v3 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z); }
static inline v3 scale(v3 a, float s) { return mk(a.x * s, a.y * s, a.z * s); }
static inline v3 neg(v3 a) { return mk(-a.x, -a.y, -a.z); }
static inline float dot(v3 a, v3 b) {
    float r = a.x * b.x;
    r = r + a.y * b.y;
    r = r + a.z * b.z;
    return r;
}
static inline float length(v3 a) { return sqrtf(dot(a, a)); }
static inline v3 normalize(v3 a) {
    float l = length(a);
    return mk(a.x / l, a.y / l, a.z / l);
}
static inline float sqr(float x) { return x * x; }

/* shade.wgsl:105-116 (Hugo Elias integer hash, u32 wraparound). */
void rto_hash3(uint32_t n, float out[3]) {
    n = (n << 13) ^ n;
    n = n * (n * n * 15731u + 789221u) + 1376312589u;
    uint32_t kx = n * n;
    uint32_t ky = n * (n * 16807u);
    uint32_t kz = n * (n * 48271u);
    const float den = 2147483648.0f; /* f32(0x7fffffff) rounds to 2^31 */
    out[0] = (float)(kx & 0x7fffffffu) / den;
    out[1] = (float)(ky & 0x7fffffffu) / den;
    out[2] = (float)(kz & 0x7fffffffu) / den;
}

float rto_tan_half(float fov) { return (float)tan((double)(fov / 2.0f)); }

/* rt_sincos (rt_hip.h "Opt-in camera sampling"): q = rint(theta * 2/pi),
 * r = theta - q*(pi/2) by a 3-constant Cody-Waite split, Taylor polynomials
 * on |r| <= pi/4, quadrant swap. Plain f32 ops (no FMA), as the kernel. */
void rto_sincos(float theta, float* s_out, float* c_out) {
    const float q = rintf(theta * 0x1.45f306p-1f);
    float r = theta - q * 0x1.92p+0f;
    r = r - q * 0x1.fb5444p-12f;
    r = r - q * 0x1.68cp-39f;
    const float r2 = r * r;
    const float sr = r + r * (r2 * (-0x1.555556p-3f +
                                    r2 * (0x1.111112p-7f +
                                          r2 * (-0x1.a01a02p-13f + r2 * 0x1.71de3ap-19f))));
    const float cr = 1.0f + r2 * (-0x1p-1f +
                                  r2 * (0x1.555556p-5f +
                                        r2 * (-0x1.6c16c2p-10f +
                                              r2 * (0x1.a01a02p-16f + r2 * -0x1.27e4fcp-22f))));
    switch ((int)q & 3) {
        case 0: *s_out = sr; *c_out = cr; break;
        case 1: *s_out = cr; *c_out = -sr; break;
        case 2: *s_out = -sr; *c_out = -cr; break;
        default: *s_out = -cr; *c_out = sr; break;
    }
}

typedef struct {
    float T[16];
    float tan_half;
    float focus_plane;
    float aspect, half_w, half_h;
    float coc;           /* lens_focal_length / (2 * fstop), generate.wgsl:97 */
    uint32_t flags;      /* RT_FLAG_JITTER / RT_FLAG_THIN_LENS */
    uint32_t width, height;
} cam_t;

static void cam_prepare(const rt_camera* c, uint32_t width, uint32_t height, cam_t* out) {
    memcpy(out->T, c->transform, sizeof(out->T));
    out->tan_half = rto_tan_half(c->fov);
    /* generate.wgsl:94-95 */
    out->focus_plane = (c->image_plane_distance * c->lens_focal_length) /
                       (c->image_plane_distance - c->lens_focal_length);
    out->aspect = (float)width;                 /* generate.wgsl:70 */
    out->half_w = (float)width / 2.0f;          /* generate.wgsl:75 */
    out->half_h = (float)height / 2.0f;         /* generate.wgsl:76 */
    out->coc = c->lens_focal_length / (2.0f * c->fstop);
    out->flags = 0;
    out->width = width;
    out->height = height;
}

/* generate.wgsl:66-129 for pixel (x, y) and seed frame `frame` (the frame
 * only matters with the opt-in jitter / thin-lens flags). */
static void primary(const cam_t* c, uint32_t x, uint32_t y, uint32_t frame, v3* o, v3* d) {
    float px = (float)x, py = (float)y;
    const uint32_t idx = x + c->width * y + (c->width * c->height) * frame;
    if (c->flags & RT_FLAG_JITTER) {            /* opt-in sub-pixel jitter */
        float j[3];
        rto_hash3(idx * RT_JITTER_HASH_MUL, j);
        px = px + (j[0] - 0.5f);
        py = py + (j[1] - 0.5f);
    }
    /* pinhole_ray, generate.wgsl:78-79 */
    v3 dir = mk(((px - c->half_w) * c->tan_half) / c->aspect,
                ((-py + c->half_h) * c->tan_half) / c->aspect, -1.0f);
    dir = normalize(dir);
    /* thin_lens_ray, generate.wgsl:85-107. lens_offset = (0,0) (the
     * reference): radius 0 => u = v = 0 exactly whatever cos/sin(2*PI) round
     * to, so origin = 0. */
    float denom = dot(dir, mk(0.0f, 0.0f, -1.0f));
    v3 focus_point = scale(dir, c->focus_plane / denom);
    v3 origin = mk(0.0f, 0.0f, 0.0f);
    if (c->flags & RT_FLAG_THIN_LENS) {         /* opt-in lens sample */
        float l[3], sn, cs;
        rto_hash3(idx * RT_LENS_HASH_MUL, l);
        const float theta = (2.0f * PI_F) * l[0] + 2.0f * PI_F;   /* :89 */
        const float sr = sqrtf(l[1]);                                /* :90-93 */
        rto_sincos(theta, &sn, &cs);
        const float u = cs * sr, v = sn * sr;
        const float a = u * c->coc, b = v * c->coc;                  /* :99-100 */
        origin = add(mk(1.0f * a, 0.0f * a, 0.0f * a), mk(0.0f * b, 1.0f * b, 0.0f * b));
    }
    dir = normalize(sub(focus_point, origin));
    /* generate.wgsl:125-126 */
    const float* T = c->T;
    origin = add(origin, mk(T[12], T[13], T[14]));
    v3 td;
    td.x = ((T[0] * dir.x + T[4] * dir.y) + T[8] * dir.z) + T[12] * 0.0f;
    td.y = ((T[1] * dir.x + T[5] * dir.y) + T[9] * dir.z) + T[13] * 0.0f;
    td.z = ((T[2] * dir.x + T[6] * dir.y) + T[10] * dir.z) + T[14] * 0.0f;
    *o = origin;
    *d = td;
}

void rto_primary_ray(const rt_camera* cam, uint32_t width, uint32_t height, uint32_t x,
                     uint32_t y, float origin[3], float dir[3]) {
    cam_t c;
    cam_prepare(cam, width, height, &c);
    v3 o, d;
    primary(&c, x, y, 0, &o, &d);
    origin[0] = o.x; origin[1] = o.y; origin[2] = o.z;
    dir[0] = d.x; dir[1] = d.y; dir[2] = d.z;
}

/* shade.wgsl:189-197 */
static v3 sky(v3 d) {
    v3 unit = normalize(d);
    float t = 0.5f * unit.y + 1.0f;
    float omt = (1.0f - t) * 1.0f;
    return mk(omt + t * 0.5f, omt + t * 0.7f, omt + t * 1.0f);
}

void rto_sky(const float dir[3], float out[3]) {
    v3 s = sky(mk(dir[0], dir[1], dir[2]));
    out[0] = s.x; out[1] = s.y; out[2] = s.z;
}

typedef struct {
    float t;
    v3 pos, normal;
    uint32_t material, front_face;
} hit_t;

/* intersect.wgsl:94-143. Returns winning sphere index or -1. */
static int intersect_world(const rt_sphere* s, uint32_t n, v3 o, v3 d, hit_t* h) {
    const float a = sqr(length(d));          /* intersect.wgsl:98 */
    float best_t = VERY_FAR;                 /* default_intersection, :86-88 */
    int best = -1;
    for (uint32_t i = 0; i < n; ++i) {
        v3 c = mk(s[i].center[0], s[i].center[1], s[i].center[2]);
        v3 oc = sub(o, c);                                     /* :97 */
        float half_b = dot(oc, d);                             /* :99 */
        float cc = sqr(length(oc)) - sqr(s[i].radius);         /* :100 */
        float dis = sqr(half_b) - a * cc;                      /* :102 */
        if (dis < 0.0f) continue;                              /* :103 */
        float sqrtd = sqrtf(dis);                              /* :107 */
        float root = (-half_b - sqrtd) / a;                    /* :109 */
        if (root < EPSILON || VERY_FAR < root) {               /* :110 */
            root = (-half_b + sqrtd) / a;                      /* :111 */
            if (root < EPSILON || VERY_FAR < root) continue;   /* :112-113 */
        }
        if (root < best_t) { best_t = root; best = (int)i; }   /* :137 strict < */
    }
    if (best >= 0) {
        /* record of the winner, intersect.wgsl:117-127 */
        const rt_sphere* w = &s[best];
        v3 c = mk(w->center[0], w->center[1], w->center[2]);
        h->t = best_t;
        h->pos = add(o, scale(d, best_t));                    /* point_at, :82-84 */
        v3 q = sub(h->pos, c);
        h->normal = normalize(mk(q.x / w->radius, q.y / w->radius, q.z / w->radius));
        h->front_face = 1u;
        if (dot(d, h->normal) > 0.0f) {
            h->normal = neg(h->normal);
            h->front_face = 0u;
        }
        h->material = w->material;
    }
    return best;
}

int rto_intersect(const rt_sphere* spheres, uint32_t n, const float origin[3],
                  const float dir[3], float* t, float pos[3], float normal[3],
                  uint32_t* front_face) {
    hit_t h;
    int i = intersect_world(spheres, n, mk(origin[0], origin[1], origin[2]),
                            mk(dir[0], dir[1], dir[2]), &h);
    if (i >= 0) {
        *t = h.t;
        pos[0] = h.pos.x; pos[1] = h.pos.y; pos[2] = h.pos.z;
        normal[0] = h.normal.x; normal[1] = h.normal.y; normal[2] = h.normal.z;
        *front_face = h.front_face;
    } else {
        *t = VERY_FAR;
    }
    return i;
}

typedef struct {
    const rt_sphere* s;
    uint32_t n;
    const float* rays;
    uint32_t nrays;
    int32_t* idx;
    float* t;
    int tid, nt;
} ijob_t;

static void* iworker(void* arg) {
    ijob_t* j = (ijob_t*)arg;
    for (uint32_t r = (uint32_t)j->tid; r < j->nrays; r += (uint32_t)j->nt) {
        const float* q = j->rays + (size_t)r * 6;
        hit_t h;
        int i = intersect_world(j->s, j->n, mk(q[0], q[1], q[2]), mk(q[3], q[4], q[5]), &h);
        j->idx[r] = i;
        j->t[r] = i >= 0 ? h.t : VERY_FAR;
    }
    return NULL;
}

void rto_intersect_batch(const rt_sphere* spheres, uint32_t n, const float* rays,
                         uint32_t nrays, int32_t* idx, float* t, int nthreads) {
    if (nthreads <= 0) nthreads = 1;
    ijob_t* jobs = (ijob_t*)calloc((size_t)nthreads, sizeof(ijob_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int k = 0; k < nthreads; ++k) {
        jobs[k] = (ijob_t){spheres, n, rays, nrays, idx, t, k, nthreads};
        pthread_create(&th[k], NULL, iworker, &jobs[k]);
    }
    for (int k = 0; k < nthreads; ++k) pthread_join(th[k], NULL);
    free(jobs);
    free(th);
}

static inline v3 reflect(v3 v, v3 n) {                   /* shade.wgsl:132-134 */
    float k = 2.0f * dot(v, n);
    return sub(v, scale(n, k));
}

static inline float reflectance(float cosine, float ref_idx) {   /* shade.wgsl:156-161 */
    float r0 = (1.0f - ref_idx) / (1.0f + ref_idx);
    r0 = r0 * r0;
    float x = 1.0f - cosine;
    float x2 = x * x;
    float p5 = (x2 * x2) * x;
    return r0 + (1.0f - r0) * p5;
}

static inline v3 refract(v3 uv, v3 n, float etai_over_etat) {    /* shade.wgsl:148-154 */
    float cos_theta = fminf(dot(neg(uv), n), 1.0f);
    v3 r_out_perp = scale(add(uv, scale(n, cos_theta)), etai_over_etat);
    float l = length(r_out_perp);
    float par = -sqrtf(fabsf(1.0f - (l * l)));
    v3 r_out_parallel = scale(n, par);
    return normalize(add(r_out_perp, r_out_parallel));
}

/* One path; returns the sample colour (xyz of the throughput, shade.wgsl:227-257). */
static v3 trace_path(const cam_t* cam, const rt_sphere* sph, uint32_t n,
                     const rt_material* mats, uint32_t width, uint32_t height, uint32_t x,
                     uint32_t y, uint32_t frame, uint32_t D, uint32_t* segs) {
    v3 o, d;
    primary(cam, x, y, frame, &o, &d);
    v3 color = mk(1.0f, 1.0f, 1.0f);                            /* clear.wgsl:82-86 */
    /* seed, shade.wgsl:216-218: identical for every bounce of (pixel, frame) */
    float sd[3];
    rto_hash3(x + width * y + (width * height) * frame, sd);
    v3 seed = mk(sd[0], sd[1], sd[2]);
    for (uint32_t b = 0; b < D; ++b) {
        hit_t h;
        ++*segs;
        int hi = intersect_world(sph, n, o, d, &h);
        if (hi < 0) {                                            /* shade.wgsl:229-233 */
            color = mul(color, sky(d));
            break;
        }
        if (b == D - 1) {                                        /* shade.wgsl:236-238 */
            color = mk(0.0f, 0.0f, 0.0f);
            break;
        }
        const rt_material* m = &mats[h.material];
        v3 mc = mk(m->color[0], m->color[1], m->color[2]);
        if (m->reflectance == RT_LAMBERTIAN) {                   /* shade.wgsl:118-130 */
            v3 dest = add(add(h.pos, h.normal), normalize(seed));
            v3 e_origin = h.pos;
            d = normalize(sub(dest, e_origin));
            o = e_origin;
            color = mul(color, mc);
        } else if (m->reflectance == RT_METALLIC) {              /* shade.wgsl:136-146 */
            v3 e_origin = add(h.pos, scale(h.normal, EPSILON));
            v3 reflected = normalize(reflect(d, h.normal));
            v3 noise = scale(normalize(seed), m->fuzziness);
            d = normalize(add(reflected, noise));
            o = e_origin;
            color = mul(color, mc);
        } else {                                                 /* shade.wgsl:163-187 */
            float ratio = m->index_of_refraction;
            if (h.front_face == 1u) ratio = 1.0f / m->index_of_refraction;
            v3 unit_dir = normalize(d);
            float cos_theta = fminf(dot(neg(unit_dir), h.normal), 1.0f);
            float sin_theta = sqrtf(1.0f - cos_theta * cos_theta);
            int cannot_refract = ratio * sin_theta > 1.0f;
            v3 e_dir;
            if (cannot_refract || reflectance(cos_theta, ratio) > seed.x)
                e_dir = reflect(d, h.normal);
            else
                e_dir = refract(unit_dir, h.normal, ratio);
            o = add(h.pos, scale(h.normal, EPSILON));
            d = e_dir;
            /* attenuation 1: colour unchanged */
        }
    }
    return color;
}

void rto_trace_path(const rt_camera* cam, const rt_sphere* spheres, uint32_t n,
                    const rt_material* materials, uint32_t m, uint32_t width,
                    uint32_t height, uint32_t x, uint32_t y, uint32_t frame,
                    uint32_t max_depth, float color[3], uint32_t* segments) {
    (void)m;
    cam_t c;
    cam_prepare(cam, width, height, &c);
    uint32_t s = 0;
    v3 col = trace_path(&c, spheres, n, materials, width, height, x, y, frame,
                        max_depth, &s);
    color[0] = col.x; color[1] = col.y; color[2] = col.z;
    *segments = s;
}

/* ------------------------------------------------------------------ render */

typedef struct {
    const cam_t* cam;
    const rt_sphere* sph;
    uint32_t n;
    const rt_material* mats;
    const rt_params* p;
    const uint32_t* rows;
    uint32_t nrows;
    float* out;
    int tid, nthreads;
    uint64_t segs;
} job_t;

static void render_pixel(const job_t* j, uint32_t x, uint32_t y, float* px, uint64_t* segs) {
    const rt_params* p = j->p;
    float acc[3] = {0.0f, 0.0f, 0.0f};
    for (uint32_t s0 = 0; s0 < p->spp; s0 += RT_SAMPLE_BLOCK) {
        uint32_t s1 = s0 + RT_SAMPLE_BLOCK < p->spp ? s0 + RT_SAMPLE_BLOCK : p->spp;
        float bs[3] = {0.0f, 0.0f, 0.0f};
        for (uint32_t s = s0; s < s1; ++s) {
            uint32_t sg = 0;
            v3 c = trace_path(j->cam, j->sph, j->n, j->mats, p->width, p->height, x, y,
                              p->frame0 + s, p->max_depth, &sg);
            *segs += sg;
            bs[0] = bs[0] + c.x; bs[1] = bs[1] + c.y; bs[2] = bs[2] + c.z;
        }
        acc[0] = acc[0] + bs[0]; acc[1] = acc[1] + bs[1]; acc[2] = acc[2] + bs[2];
    }
    if (p->flags & RTO_FLAG_RAW_SUMS) {
        px[0] = acc[0]; px[1] = acc[1]; px[2] = acc[2]; px[3] = 0.0f;
        return;
    }
    const float fs = (float)p->spp;                     /* collect.wgsl:122 */
    px[0] = acc[0] / fs;
    px[1] = acc[1] / fs;
    px[2] = acc[2] / fs;
    px[3] = 1.0f;
}

static void* worker(void* arg) {
    job_t* j = (job_t*)arg;
    uint64_t segs = 0;
    const uint32_t W = j->p->width;
    /* interleave 32-pixel row pieces over threads for load balance (a few
     * rows of an 8K frame still keep every thread busy); pixels are
     * independent, so the split does not change any result */
    const uint32_t pieces = (W + 31u) / 32u;
    const uint64_t units = (uint64_t)j->nrows * pieces;
    for (uint64_t u = (uint64_t)j->tid; u < units; u += (uint64_t)j->nthreads) {
        const uint32_t r = (uint32_t)(u / pieces);
        const uint32_t x0 = (uint32_t)(u % pieces) * 32u;
        const uint32_t x1 = x0 + 32u < W ? x0 + 32u : W;
        const uint32_t y = j->rows[r];
        for (uint32_t x = x0; x < x1; ++x)
            render_pixel(j, x, y, j->out + ((size_t)r * W + x) * 4, &segs);
    }
    j->segs = segs;
    return NULL;
}

static int check(const rt_camera* cam, const rt_sphere* spheres, uint32_t n,
                 const rt_material* materials, uint32_t m, const rt_params* p) {
    if (!cam || !p || (n && !spheres) || (m && !materials)) return -1;
    if (p->width == 0 || p->height == 0 || p->spp == 0 || p->max_depth == 0) return -1;
    for (uint32_t i = 0; i < n; ++i) {
        if (spheres[i].material >= m) return -1;
        int r = materials[spheres[i].material].reflectance;
        if (r < 0 || r > 2) return -1;
    }
    return 0;
}

int rto_render_rows(const rt_camera* cam, const rt_sphere* spheres, uint32_t n,
                    const rt_material* materials, uint32_t m, const rt_params* params,
                    const uint32_t* rows, uint32_t nrows, float* out_rgba,
                    uint64_t* segments, int nthreads) {
    if (check(cam, spheres, n, materials, m, params)) return -1;
    for (uint32_t r = 0; r < nrows; ++r)
        if (rows[r] >= params->height) return -1;
    if (nthreads <= 0) nthreads = 1;
    cam_t c;
    cam_prepare(cam, params->width, params->height, &c);
    c.flags = params->flags & (RT_FLAG_JITTER | RT_FLAG_THIN_LENS);
    job_t* jobs = (job_t*)calloc((size_t)nthreads, sizeof(job_t));
    pthread_t* th = (pthread_t*)calloc((size_t)nthreads, sizeof(pthread_t));
    for (int t = 0; t < nthreads; ++t) {
        jobs[t] = (job_t){&c, spheres, n, materials, params, rows, nrows, out_rgba, t,
                          nthreads, 0};
        if (nthreads > 1)
            pthread_create(&th[t], NULL, worker, &jobs[t]);
        else
            worker(&jobs[t]);
    }
    uint64_t segs = 0;
    for (int t = 0; t < nthreads; ++t) {
        if (nthreads > 1) pthread_join(th[t], NULL);
        segs += jobs[t].segs;
    }
    free(jobs);
    free(th);
    if (segments) *segments = segs;
    return 0;
}

/* Row block b -> owning shard (rt_hip.h rt_params: groups of K blocks dealt
 * serpentine). The row tiling is this build's own multi-GPU design (the
 * reference renders on one adapter), so there is no reference line to cite. */
static uint32_t rto_block_owner(uint32_t b, uint32_t K) {
    uint32_t g = b / K, i = b % K;
    return (g & 1u) ? K - 1u - i : i;
}

int rto_render(const rt_camera* cam, const rt_sphere* spheres, uint32_t n,
               const rt_material* materials, uint32_t m, const rt_params* params,
               float* out_rgba, uint64_t* segments, int nthreads) {
    if (!params) return -1;
    uint32_t B = params->row_block ? params->row_block : 1;
    uint32_t K = params->shard_count ? params->shard_count : 1;
    uint32_t k = params->shard_index;
    if (k >= K) return -1;
    uint32_t* rows = (uint32_t*)malloc(sizeof(uint32_t) * (params->height + 1));
    uint32_t nr = 0;
    for (uint32_t y = 0; y < params->height; ++y)
        if (rto_block_owner(y / B, K) == k) rows[nr++] = y;
    int rc = rto_render_rows(cam, spheres, n, materials, m, params, rows, nr, out_rgba,
                             segments, nthreads);
    free(rows);
    return rc;
}
