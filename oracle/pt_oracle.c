/*
 * pt_oracle.c -- CPU restatement of the reference path-tracing kernel
 * (/root/reference/internal/ocl/tracer.cl, `trace`, lines 831-1188).
 *
 * TEST INFRASTRUCTURE ONLY.  Used by tests/, __graft_entry__.smoke() and
 * bench.py's cpu_baseline leg as the checker / CPU baseline.  The product
 * (pathtracer-ocl_amd/csrc, libptmi.so) never links or calls it.
 *
 * Parity contract: this file restates the reference AS THE AMD
 * OPENCL TOOLCHAIN BUILDS IT (oracle/Makefile, -ffp-contract=off): user code
 * is separately rounded; OpenCL builtins follow ROCm device-libs --
 *   dot(a,b)   = fma(a.w,b.w, fma(a.z,b.z, fma(a.y,b.y, a.x*b.x)))  (opencl.bc)
 *   cross(a,b) = fma(a.y,b.z, b.y*-a.z), ... , w = 0                 (opencl.bc)
 *   normalize  = v * rsqrt(dot(v,v)) with range scaling              (opencl.bc)
 *   max/min    = IEEE maxNum/minNum (NaN-ignoring)                   (ocml)
 *   sin(float) = __ocml_sin_f32, fract = __ocml_fract_f32            (ocml_sinf.h)
 * Double transcendental builtins (sin/cos/pow/sqrt on double) come from glibc
 * here and ocml on the GPU: they may differ in the last ulp, which moves the
 * image by ~1e-16 (parity tolerance 1e-4, north_star).
 *
 * Deliberate, output-preserving differences from the literal reference:
 *   - a missed ray ends the bounce loop (the reference re-traces the identical
 *     ray until b == MAX_BOUNCES; every such iteration is a no-op, tracer.cl:884);
 *   - intersections are reduced on the fly (first t > EPSILON strictly below
 *     the running best, in the reference's recording order, tracer.cl:728-739)
 *     instead of being stored in the 64-entry ctx, whose overflow is UB there.
 *   - textures (read_imagef, tracer.cl:907-914/1077-1092): the kernel's sampler
 *     (tracer.cl:829: normalized coords, REPEAT, LINEAR, RGBA UNORM8) is restated
 *     with the OpenCL 1.2 s8.2 formulas in FP32, separately rounded in the same
 *     order as the HIP kernel.  PARITY UNPINNED for the sampler: gfx950 has no
 *     image instructions, so the reference kernel cannot sample a texture on this
 *     hardware (DESIGN.md "Textures"); sphericalMap's atan2/acos are glibc here and
 *     ocml on the GPU (last-ulp differences, invisible after the float cast).
 */
#include <math.h>
#include <stdint.h>
#include <stdlib.h>
#include <string.h>

#ifdef _OPENMP
#include <omp.h>
#endif

#include "ocml_sinf.h"

/* Event counters for the algorithmic-flop model (bench.py roofline; built only
 * into oracle/build/libptoracle_count.so with -DPTO_COUNT).  Event names and
 * their FP64 flop costs live in pathtracer-ocl_amd/ptmi/flops.py. */
enum {
    EV_SAMPLE, EV_CAMERA, EV_CAMERA_DOF, EV_OBJ_TEST, EV_PLANE, EV_SPHERE, EV_SPHERE_DISC, EV_CYL, EV_CYL_DISC,
    EV_CUBE, EV_GROUP_BOX, EV_NODE_BOX, EV_TRI_DET, EV_TRI_U, EV_TRI_V, EV_TRI_FULL, EV_HIT, EV_NRM_SPHERE,
    EV_NRM_CYL, EV_NRM_CUBE, EV_NRM_TRI, EV_REFLECT, EV_SCHLICK, EV_SCHLICK_TIR_BRANCH, EV_REFRACT, EV_UNDER,
    EV_DIFFUSE, EV_REDUCE, EV_NOISE, EV_COUNT
};
#ifdef PTO_COUNT
static __thread uint64_t g_ev[EV_COUNT];
static uint64_t g_ev_total[EV_COUNT];
#define CNT(e) (g_ev[(e)]++)
/* The reference's ctx entries of one findClosestIntersection call (every candidate it
 * records, t != 0, negative t included; tracer.cl:553-672) and their maximum over a trace:
 * its ctx arrays hold 64 (tracer.cl:97-99), so a scene whose maximum exceeds 64 overflows
 * them in the reference (undefined behaviour) and cannot be a live-reference
 * parity case. */
static __thread int g_xs, g_xs_max;
static int g_xs_max_total;
#define XS_RECORD() (g_xs++)
#else
#define CNT(e) ((void)0)
#define XS_RECORD() ((void)0)
#endif

#define MAX_EFFECTIVE_BOUNCES 4u /* tracer.cl:2 */
#define MAX_BOUNCES 10u          /* tracer.cl:3 */
static const double EPSILON = 0.0001;          /* tracer.cl:4 */
static const double PI = (double)3.14159265359f; /* tracer.cl:1: a FLOAT literal */

typedef struct { double x, y, z, w; } d4;

static inline d4 mk(double x, double y, double z, double w) { d4 r = {x, y, z, w}; return r; }
static inline d4 add4(d4 a, d4 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
static inline d4 sub4(d4 a, d4 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
static inline d4 mul4(d4 a, d4 b) { return mk(a.x * b.x, a.y * b.y, a.z * b.z, a.w * b.w); }
static inline d4 scl4(d4 a, double s) { return mk(a.x * s, a.y * s, a.z * s, a.w * s); }
static inline d4 neg4(d4 a) { return mk(-a.x, -a.y, -a.z, -a.w); }

/* OpenCL dot(double4) as built by device-libs (fmuladd -> fma). */
static inline double dot4(d4 a, d4 b) {
    double d = a.x * b.x;
    d = fma(a.y, b.y, d);
    d = fma(a.z, b.z, d);
    return fma(a.w, b.w, d);
}
/* OpenCL cross(double4) (opencl.bc _Z5crossDv4_dS_). */
static inline d4 cross4(d4 a, d4 b) {
    return mk(fma(a.y, b.z, b.y * -a.z), fma(a.z, b.x, b.z * -a.x), fma(a.x, b.y, b.x * -a.y), 0.0);
}
/* __ocml_rsqrt_f64: hardware seed refined by one 2nd-order Newton step; the seed
 * is taken as the correctly rounded 1/sqrt here. */
static inline double rsqrt_ocml(double x) {
    double r0 = 1.0 / sqrt(x);
    if (!(isfinite(r0) && r0 > 0.0)) return r0;
    double e = fma(r0 * -x, r0, 1.0);
    return fma(r0 * e, fma(e, 0.375, 0.5), r0);
}
/* OpenCL normalize(double4) (opencl.bc _Z9normalizeDv4_d). */
static d4 normalize4(d4 v) {
    if (v.x == 0.0 && v.y == 0.0 && v.z == 0.0 && v.w == 0.0) return v;
    double d = dot4(v, v);
    d4 p = v;
    if (d < 0x1p-1022) {
        p = scl4(v, 0x1p563);
        d = dot4(p, p);
    } else if (d == INFINITY) {
        p = scl4(v, 0x1p-514);
        d = dot4(p, p);
        if (d == INFINITY) {
            p = mk(copysign(isinf(p.x) ? 1.0 : 0.0, p.x), copysign(isinf(p.y) ? 1.0 : 0.0, p.y),
                   copysign(isinf(p.z) ? 1.0 : 0.0, p.z), copysign(isinf(p.w) ? 1.0 : 0.0, p.w));
            d = dot4(p, p);
        }
    }
    return scl4(p, rsqrt_ocml(d));
}
/* maxX/minX (tracer.cl:110-111) over OpenCL max/min == maxNum/minNum. */
static inline double maxX(double a, double b, double c) { return fmax(fmax(a, b), c); }
static inline double minX(double a, double b, double c) { return fmin(fmin(a, b), c); }

/* mul (tracer.cl:369-376): row-major mat4 x vec4, each row summed x+y+z+w. */
static inline d4 mat_mul(const double* m, d4 v) {
    return mk(((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3] * v.w,
              ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7] * v.w,
              ((m[8] * v.x + m[9] * v.y) + m[10] * v.z) + m[11] * v.w,
              ((m[12] * v.x + m[13] * v.y) + m[14] * v.z) + m[15] * v.w);
}

/* noise3D (tracer.cl:314-317), float math throughout. */
static inline float noise3d(float x, float y, float z) {
    CNT(EV_NOISE);
    float a = x * 112.9898f;
    float b = y * 179.233f;
    float c = z * 237.212f;
    float s = (a + b) + c;
    return pto_fractf(pto_sinf(s) * 43758.5453f);
}

/* ---------------- input records (packed byte layouts, layout.py) ---------- */
typedef struct {
    double transform[16], inverse[16], inverse_transpose[16];
    d4 color, emission;
    double refractive_index;
    int64_t type;
    double min_y, max_y, reflectivity;
    d4 bb_min, bb_max;
    int32_t child_count;
    int32_t children[64];
    uint8_t is_textured, is_textured_nm, texture_index, texture_index_nm;
    double texture_scale[4]; /* X, Y, XNM, YNM (ocltracer.go:36-39) */
} object_t;

/* One image2d_array_t of the kernel (tracer.cl:833): n layers of w x h NRGBA8
 * texels (prepareTextures, ocltracer.go:228-254); n == 0: the all-zero fake image. */
typedef struct {
    const uint8_t* pix;
    uint32_t w, h, n;
} tex_t;

typedef struct {
    d4 bb_min, bb_max;
    int32_t tri_offset, tri_count;
    int32_t children[2];
} group_t;

typedef struct { d4 p1, e1, e2, n1, n2, n3, color; } tri_t;

typedef struct {
    int32_t width, height;
    double pixel_size, half_width, half_height, aperture, focal_length;
    double inverse[16];
} camera_t;

static d4 ld4(const uint8_t* p) { d4 r; memcpy(&r, p, 32); return r; }

static void unpack_object(const uint8_t* b, object_t* o) {
    memcpy(o->transform, b + 0, 128);
    memcpy(o->inverse, b + 128, 128);
    memcpy(o->inverse_transpose, b + 256, 128);
    o->color = ld4(b + 384);
    o->emission = ld4(b + 416);
    memcpy(&o->refractive_index, b + 448, 8);
    memcpy(&o->type, b + 456, 8);
    memcpy(&o->min_y, b + 464, 8);
    memcpy(&o->max_y, b + 472, 8);
    memcpy(&o->reflectivity, b + 480, 8);
    o->bb_min = ld4(b + 520);
    o->bb_max = ld4(b + 552);
    memcpy(&o->child_count, b + 584, 4);
    memcpy(o->children, b + 588, 256);
    o->is_textured = b[844];
    o->texture_index = b[845];
    o->is_textured_nm = b[846];
    o->texture_index_nm = b[847];
    memcpy(o->texture_scale, b + 488, 32);
}

static void unpack_group(const uint8_t* b, group_t* g) {
    g->bb_min = ld4(b + 0);
    g->bb_max = ld4(b + 32);
    memcpy(&g->tri_offset, b + 128, 4);
    memcpy(&g->tri_count, b + 132, 4);
    memcpy(g->children, b + 140, 8);
}

static void unpack_tri(const uint8_t* b, tri_t* t) {
    t->p1 = ld4(b + 0);
    t->e1 = ld4(b + 96);
    t->e2 = ld4(b + 128);
    t->n1 = ld4(b + 160);
    t->n2 = ld4(b + 192);
    t->n3 = ld4(b + 224);
    t->color = ld4(b + 256);
}

static void unpack_camera(const uint8_t* b, camera_t* c) {
    memcpy(&c->width, b + 0, 4);
    memcpy(&c->height, b + 4, 4);
    memcpy(&c->pixel_size, b + 16, 8);
    memcpy(&c->half_width, b + 24, 8);
    memcpy(&c->half_height, b + 32, 8);
    memcpy(&c->aperture, b + 40, 8);
    memcpy(&c->focal_length, b + 48, 8);
    memcpy(c->inverse, b + 56, 128);
}

typedef struct {
    const object_t* objects;
    uint32_t n_obj;
    const group_t* groups;
    uint32_t n_grp;
    const tri_t* tris;
    uint32_t n_tri;
    camera_t cam;
    tex_t tex[3]; /* textures, sphereTextures, cubeMapTextures */
} scene_t;

/* ---------------- textures (tracer.cl:113-213, 829) -------------------------- */
typedef struct { float r, g, b; } rgb_t;

/* CLK_ADDRESS_REPEAT + CLK_FILTER_LINEAR along one axis (OpenCL 1.2 s8.2). */
static void tex_axis(float s, int n, int* i0, int* i1, float* a) {
    if (!isfinite(s)) s = 0.0f; /* undefined in OpenCL; pinned to 0 (same as the HIP kernel) */
    float u = (s - floorf(s)) * (float)n;
    float um = u - 0.5f;
    float fl = floorf(um);
    *i0 = (int)fl;
    *i1 = *i0 + 1;
    if (*i0 < 0) *i0 = n + *i0;
    if (*i1 > n - 1) *i1 = *i1 - n;
    *a = um - fl;
}

static rgb_t texel(const tex_t* T, int l, int i, int j) {
    const uint8_t* p = T->pix + 4 * (((size_t)l * T->h + (size_t)j) * T->w + (size_t)i);
    rgb_t c = {(float)p[0] / 255.0f, (float)p[1] / 255.0f, (float)p[2] / 255.0f};
    return c;
}

/* read_imagef(array, sampler, (float4)(s, t, layer, 0)).xyz */
static rgb_t tex_sample(const tex_t* T, float s, float t, float layer) {
    rgb_t z = {0.0f, 0.0f, 0.0f};
    if (T->n == 0) return z;
    int l = (int)fminf(fmaxf(rintf(layer), 0.0f), (float)(T->n - 1));
    int i0, i1, j0, j1;
    float a, b;
    tex_axis(s, (int)T->w, &i0, &i1, &a);
    tex_axis(t, (int)T->h, &j0, &j1, &b);
    rgb_t t00 = texel(T, l, i0, j0), t10 = texel(T, l, i1, j0), t01 = texel(T, l, i0, j1), t11 = texel(T, l, i1, j1);
    float w00 = (1.0f - a) * (1.0f - b), w10 = a * (1.0f - b), w01 = (1.0f - a) * b, w11 = a * b;
    rgb_t c = {((w00 * t00.r + w10 * t10.r) + w01 * t01.r) + w11 * t11.r,
               ((w00 * t00.g + w10 * t10.g) + w01 * t01.g) + w11 * t11.g,
               ((w00 * t00.b + w10 * t10.b) + w01 * t01.b) + w11 * t11.b};
    return c;
}

/* OpenCL length(double4) (opencl.bc _Z6lengthDv4_d): sqrt(dot) with range scaling. */
static double length4(d4 v) {
    double d = dot4(v, v);
    if (d < 0x1p-1022) {
        d4 p = scl4(v, 0x1p563);
        return sqrt(dot4(p, p)) * 0x1p-563;
    }
    if (d == INFINITY) {
        d4 p = scl4(v, 0x1p-514);
        return sqrt(dot4(p, p)) * 0x1p514;
    }
    return sqrt(d);
}

/* sphericalMap (tracer.cl:178-213). */
static void spherical_map(d4 p, double* u, double* v) {
    double theta = atan2(p.x, p.z);
    double radius = length4(mk(p.x, p.y, p.z, 0.0));
    double phi = acos(p.y / radius);
    double raw_u = theta / (2.0 * PI);
    *u = 1 - (raw_u + 0.5);
    *v = 1 - phi / PI;
}

/* cubeUV and the six cubeUV*Cross faces (tracer.cl:113-175). */
static void cube_uv(d4 p, double* u, double* v) {
    double coord = maxX(fabs(p.x), fabs(p.y), fabs(p.z));
    if (coord == p.x) { /* right */
        *u = 0.5 + fmod(1.0 - p.z, 2) / 2.0 * 0.25;
        *v = 0.6666666 - fmod(p.y + 1.0, 2) / 2.0 * 0.333333;
    } else if (coord == -p.x) { /* left */
        *u = fmod(p.z + 1.0, 2) / 2.0 * 0.25;
        *v = 0.6666666 - fmod(p.y + 1.0, 2) / 2.0 * 0.333333;
    } else if (coord == p.y) { /* up */
        *u = 0.25 + fmod(p.x + 1.0, 2) / 2.0 * 0.25;
        *v = 1.0 - fmod(1.0 - p.z, 2) / 2.0 * 0.333333;
    } else if (coord == -p.y) { /* down */
        *u = 0.25 + fmod(p.x + 1.0, 2) / 2.0 * 0.25;
        *v = fmod(p.z + 1.0, 2) / 2.0 * 0.333333;
    } else if (coord == p.z) { /* front */
        *u = 0.25 + fmod(p.x + 1.0, 2) / 2.0 * 0.25;
        *v = 0.6666666 - fmod(p.y + 1.0, 2) / 2.0 * 0.333333;
    } else { /* back */
        *u = 0.75 + fmod(1.0 - p.x, 2) / 2.0 * 0.25;
        *v = 0.6666666 - fmod(p.y + 1.0, 2) / 2.0 * 0.333333;
    }
}

/* ---------------- intersectors --------------------------------------------- */

/* checkAxis (tracer.cl:250-268) */
static inline void check_axis(double origin, double direction, double min_bb, double max_bb,
                              double* tmin, double* tmax) {
    double tminn = min_bb - origin, tmaxn = max_bb - origin;
    double a, b;
    if (fabs(direction) >= EPSILON) {
        a = tminn / direction;
        b = tmaxn / direction;
    } else {
        a = tminn * HUGE_VAL;
        b = tmaxn * HUGE_VAL;
    }
    if (a > b) { double t = a; a = b; b = t; }
    *tmin = a;
    *tmax = b;
}

/* intersectRayWithBox (tracer.cl:270-280): a LINE test, no t range. */
static inline int ray_box(d4 o, d4 d, d4 mn, d4 mx) {
    double x0, x1, y0, y1, z0, z1;
    check_axis(o.x, d.x, mn.x, mx.x, &x0, &x1);
    check_axis(o.y, d.y, mn.y, mx.y, &y0, &y1);
    check_axis(o.z, d.z, mn.z, mx.z, &z0, &z1);
    return maxX(x0, y0, z0) < minX(x1, y1, z1);
}

/* Running closest-hit state: equals the reference's scan over ctx (728-739). */
typedef struct {
    double t;
    int obj;
    int tri;          /* triangle index of the winning group hit, else -1 */
    double u, v;
} hit_t;

static inline void consider(hit_t* h, double t, int obj, int tri, double u, double v) {
    XS_RECORD();
    if (t > EPSILON && t < h->t) {
        h->t = t;
        h->obj = obj;
        h->tri = tri;
        h->u = u;
        h->v = v;
    }
}

/* findClosestIntersection (tracer.cl:537-742). */
static hit_t find_closest_(const scene_t* S, d4 ro, d4 rd);
static hit_t find_closest(const scene_t* S, d4 ro, d4 rd) {
#ifdef PTO_COUNT
    g_xs = 0;
    const hit_t h = find_closest_(S, ro, rd);
    if (g_xs > g_xs_max) g_xs_max = g_xs;
    return h;
#else
    return find_closest_(S, ro, rd);
#endif
}
static hit_t find_closest_(const scene_t* S, d4 ro, d4 rd) {
    hit_t h = {1024.0, -1, -1, 0.0, 0.0};
    for (uint32_t j = 0; j < S->n_obj; j++) {
        const object_t* ob = &S->objects[j];
        CNT(EV_OBJ_TEST);
        d4 o = mat_mul(ob->inverse, ro);
        d4 d = mat_mul(ob->inverse, rd);
        if (ob->type == 0) { /* intersectPlane 478-483 */
            CNT(EV_PLANE);
            double t = fabs(d.y) > EPSILON ? -o.y / d.y : 0.0;
            if (t != 0.0) consider(&h, t, (int)j, -1, 0, 0);
        } else if (ob->type == 1) { /* intersectSphere 448-476 */
            CNT(EV_SPHERE);
            d4 vtc = sub4(o, mk(0.0, 0.0, 0.0, 1.0));
            double a = dot4(d, d);
            double b = 2.0 * dot4(d, vtc);
            double c = dot4(vtc, vtc) - 1.0;
            double disc = (b * b) - 4 * a * c;
            if (disc > 0.0) {
                CNT(EV_SPHERE_DISC);
                double t1 = (-b - sqrt(disc)) / (2 * a);
                double t2 = (-b + sqrt(disc)) / (2 * a);
                if (t1 != 0.0) consider(&h, t1, (int)j, -1, 0, 0);
                if (t2 != 0.0) consider(&h, t2, (int)j, -1, 0, 0);
            }
        } else if (ob->type == 2) { /* intersectCylinder 396-446 (caps disabled) */
            CNT(EV_CYL);
            double rdx2 = d.x * d.x, rdz2 = d.z * d.z;
            double a = rdx2 + rdz2;
            if (!(fabs(a) < EPSILON)) {
                double b = 2 * o.x * d.x + 2 * o.z * d.z;
                double rox2 = o.x * o.x, roz2 = o.z * o.z;
                double c1 = rox2 + roz2 - 1;
                double disc = b * b - 4 * a * c1;
                if (!(disc < 0.0)) {
                    CNT(EV_CYL_DISC);
                    double t0 = (-b - sqrt(disc)) / (2 * a);
                    double t1 = (-b + sqrt(disc)) / (2 * a);
                    double o0 = 0.0, o1 = 0.0;
                    double y0 = o.y + t0 * d.y;
                    if (y0 > ob->min_y && y0 < ob->max_y) o0 = t0;
                    double y1 = o.y + t1 * d.y;
                    if (y1 > ob->min_y && y1 < ob->max_y) o1 = t1;
                    if (o0 != 0) consider(&h, o0, (int)j, -1, 0, 0);
                    if (o1 != 0) consider(&h, o1, (int)j, -1, 0, 0);
                }
            }
        } else if (ob->type == 3) { /* intersectCube 378-394 */
            CNT(EV_CUBE);
            double x0, x1, y0, y1, z0, z1;
            check_axis(o.x, d.x, -1.0, 1.0, &x0, &x1);
            check_axis(o.y, d.y, -1.0, 1.0, &y0, &y1);
            check_axis(o.z, d.z, -1.0, 1.0, &z0, &z1);
            double tmin = maxX(x0, y0, z0), tmax = minX(x1, y1, z1);
            if (!(tmin > tmax)) {
                if (tmin != 0.0) consider(&h, tmin, (int)j, -1, 0, 0);
                if (tmax != 0.0) consider(&h, tmax, (int)j, -1, 0, 0);
            }
        } else if (ob->type == 4) { /* groups 598-720 */
            CNT(EV_GROUP_BOX);
            if (!ray_box(o, d, ob->bb_min, ob->bb_max)) continue;
            for (int ci = 0; ci < ob->child_count; ci++) {
                /* Iterative preorder walk exactly as 621-719 (stack of node ids). */
                int stack[64];
                int sidx = 0;
                int cur_idx = ob->children[ci];
                const group_t* cur = &S->groups[cur_idx];
                for (;;) {
                    while (cur && (CNT(EV_NODE_BOX), ray_box(o, d, cur->bb_min, cur->bb_max))) {
                        for (int n = cur->tri_offset; n < cur->tri_offset + cur->tri_count; n++) {
                            const tri_t* T = &S->tris[n];
                            CNT(EV_TRI_DET);
                            d4 dce2 = cross4(d, T->e2);
                            double det = dot4(T->e1, dce2);
                            if (fabs(det) < EPSILON) continue;
                            double f = 1.0 / det;
                            d4 p1o = sub4(o, T->p1);
                            double u = f * dot4(p1o, dce2);
                            CNT(EV_TRI_U);
                            if (u < 0 || u > 1) continue;
                            CNT(EV_TRI_V);
                            d4 oce1 = cross4(p1o, T->e1);
                            double v = f * dot4(d, oce1);
                            if (v < 0 || (u + v) > 1) continue;
                            CNT(EV_TRI_FULL);
                            double t = f * dot4(T->e2, oce1);
                            consider(&h, t, (int)j, n, u, v);
                        }
                        stack[sidx++] = cur_idx;
                        if (cur->children[0] > 0) {
                            cur_idx = cur->children[0];
                            cur = &S->groups[cur_idx];
                        } else {
                            cur = NULL;
                        }
                    }
                    sidx--;
                    if (sidx == -1) break;
                    cur = &S->groups[stack[sidx]];
                    if (cur->children[1] > 0) {
                        cur_idx = cur->children[1];
                        cur = &S->groups[cur_idx];
                    } else {
                        cur = NULL;
                    }
                }
            }
        }
    }
    return h;
}

/* ---------------- shading helpers ------------------------------------------ */

/* schlick (tracer.cl:485-505) */
static double schlick(d4 eye, d4 nrm, double n1, double n2) {
    CNT(EV_SCHLICK);
    double c = dot4(eye, nrm);
    if (n1 > n2) {
        CNT(EV_SCHLICK_TIR_BRANCH);
        double n = n1 / n2;
        double sin2t = (n * n) * (1.0 - (c * c));
        if (sin2t > 1.0) return 1.0;
        c = sqrt(1.0 - sin2t);
    }
    double tmp = (n1 - n2) / (n1 + n2);
    double r0 = tmp * tmp;
    return r0 + (1 - r0) * pow(1 - c, 5);
}

/* computeRefractedRay (tracer.cl:507-533) */
static d4 refracted(d4 eye, d4 nrm, double n1, double n2) {
    CNT(EV_REFRACT);
    double nr = n1 / n2;
    double cosi = dot4(eye, nrm);
    double sin2t = (nr * nr) * (1.0 - (cosi * cosi));
    if (sin2t > 1.0) return mk(0, 0, 0, 0);
    double cost = sqrt(1.0 - sin2t);
    return sub4(scl4(nrm, (nr * cosi) - cost), scl4(eye, nr));
}

/* randomVectorInHemisphere (tracer.cl:348-366); x,y,z are doubles holding floats. */
static d4 random_hemisphere(d4 nv, double x, double y, double z) {
    CNT(EV_DIFFUSE);
    double rand1 = 2.0 * PI * (double)noise3d((float)x, (float)y, (float)z);
    double rand2 = (double)noise3d((float)y, (float)z, (float)x);
    double rand2s = sqrt(rand2);
    d4 axis = fabs(nv.x) > 0.1 ? mk(0.0, 1.0, 0.0, 0.0) : mk(1.0, 0.0, 0.0, 0.0);
    d4 u = normalize4(cross4(axis, nv));
    d4 v = cross4(nv, u);
    return add4(add4(scl4(scl4(u, cos(rand1)), rand2s), scl4(scl4(v, sin(rand1)), rand2s)),
                scl4(nv, sqrt(1.0 - rand2)));
}

/* sunflowerRadius / sunflower (tracer.cl:221-248), randomize == false */
static void sunflower(int amount, double alpha, int point, double* ox, double* oy) {
    double idx = (double)point;
    double sqp = sqrt((double)amount);
    double b = round(alpha * sqp);
    double phi = (sqrt(5.0) + 1.0) / 2.0;
    double n = (double)amount;
    double r = 1.0;
    if (idx <= (n - b)) r = sqrt(idx - 0.5) / sqrt(n - (b + 1.0) / 2.0);
    double theta = 2.0 * PI * idx / (phi * phi);
    *ox = r * cos(theta);
    *oy = r * sin(theta);
}

/* rayForPixel (tracer.cl:745-779) */
static void ray_for_pixel(const camera_t* cam, unsigned x, unsigned y, float rx, float ry, int sample,
                          int total, d4* ro, d4* rd) {
    double xo = cam->pixel_size * ((double)x + rx);
    double yo = cam->pixel_size * ((double)y + ry);
    d4 piv = mk(cam->half_width - xo, cam->half_height - yo, -1.0, 1.0);
    d4 pixel = mat_mul(cam->inverse, piv);
    d4 origin = mat_mul(cam->inverse, mk(0.0, 0.0, 0.0, 1.0));
    d4 dir = normalize4(sub4(pixel, origin));
    CNT(EV_CAMERA);
    if (cam->aperture != 0) {
        CNT(EV_CAMERA_DOF);
        d4 pos = add4(origin, scl4(dir, cam->focal_length));
        double sx, sy;
        sunflower(total, 2, sample, &sx, &sy);
        d4 no = mk(origin.x + (sy * cam->aperture), origin.y + (sx * cam->aperture), origin.z, 1.0);
        dir = sub4(pos, no);
        origin = no;
    }
    *ro = origin;
    *rd = dir;
}

typedef struct {
    d4 color, emission;
    double cosine;
    int is_refraction;
} bounce_t;

/* One pixel: the body of `trace` (tracer.cl:837-1187) for samples [s0, s1). */
static d4 trace_pixel(const scene_t* S, const double* seeds, uint32_t i, uint32_t samples, uint32_t s0,
                      uint32_t s1) {
    const camera_t* cam = &S->cam;
    float fgi = (float)(seeds[i] / (double)S->n_obj);
    float fgi2 = (float)(seeds[i] / (double)samples);
    unsigned x = i % (unsigned)cam->width;
    unsigned y = i / (unsigned)cam->width;
    d4 colors = mk(0, 0, 0, 0);
    const d4 origin_point = mk(0.0, 0.0, 0.0, 1.0);
    for (uint32_t n = s0; n < s1; n++) {
        CNT(EV_SAMPLE);
        d4 ro, rd;
        ray_for_pixel(cam, x, y, noise3d(fgi, (float)n, fgi2), noise3d(fgi, fgi2, (float)n), (int)n,
                      (int)samples, &ro, &rd);
        unsigned actual = 0, effective = 0;
        bounce_t bounces[16];
        int inside = 0;
        for (uint32_t b = 0; b < MAX_BOUNCES && effective < MAX_EFFECTIVE_BOUNCES; b++) {
            hit_t h = find_closest(S, ro, rd);
            if (h.obj < 0) break; /* miss: the reference repeats the same miss to b == 10 */
            const object_t* ob = &S->objects[h.obj];
            CNT(EV_HIT);
            d4 pos = add4(ro, scl4(rd, h.t));
            d4 eye = neg4(rd);
            d4 on;
            if (ob->type == 0 && ob->is_textured_nm) { /* normal map (tracer.cl:907-911) */
                d4 lp = mat_mul(ob->inverse, pos);
                rgb_t c = tex_sample(&S->tex[0], (float)(fabs(lp.x) * ob->texture_scale[2]),
                                     (float)(fabs(lp.z) * ob->texture_scale[3]), (float)ob->texture_index_nm);
                on = normalize4(mk((double)c.r, (double)c.g, (double)c.b, 0.0));
            } else if (ob->type == 0) {
                on = mk(0.0, 1.0, 0.0, 0.0);
            } else if (ob->type == 1) {
                CNT(EV_NRM_SPHERE);
                on = sub4(mat_mul(ob->inverse, pos), origin_point);
            } else if (ob->type == 2) {
                CNT(EV_NRM_CYL);
                d4 lp = mat_mul(ob->inverse, pos);
                double dist = pow(lp.x, 2) + pow(lp.z, 2);
                if (dist < 1 && lp.y >= ob->max_y - EPSILON) on = mk(0.0, 1.0, 0.0, 0.0);
                else if (dist < 1 && lp.y <= ob->min_y + EPSILON) on = mk(0.0, -1.0, 0.0, 0.0);
                else on = mk(lp.x, 0.0, lp.z, 0.0);
            } else if (ob->type == 3) {
                CNT(EV_NRM_CUBE);
                d4 lp = mat_mul(ob->inverse, pos);
                double mc = maxX(fabs(lp.x), fabs(lp.y), fabs(lp.z));
                if (mc == fabs(lp.x)) on = mk(lp.x, 0.0, 0.0, 0.0);
                else if (mc == fabs(lp.y)) on = mk(0.0, lp.y, 0.0, 0.0);
                else on = mk(0.0, 0.0, lp.z, 0.0);
            } else { /* type 4: interpolated vertex normal of the winning triangle (669) */
                CNT(EV_NRM_TRI);
                const tri_t* T = &S->tris[h.tri];
                on = add4(add4(scl4(T->n2, h.u), scl4(T->n3, h.v)), scl4(T->n1, 1.0 - h.u - h.v));
            }
            d4 nv = mat_mul(ob->inverse_transpose, on);
            nv.w = 0.0;
            nv = normalize4(nv);
            if (dot4(eye, nv) < 0.0) nv = scl4(nv, -1.0);
            d4 over = add4(pos, scl4(nv, EPSILON));
            double cosine = 1.0;
            int entering = 0, exiting = 0, reflecting = 0;
            if (ob->reflectivity != 0.0 && noise3d(fgi, (float)n, (float)b) < ob->reflectivity) {
                CNT(EV_REFLECT);
                rd = sub4(rd, scl4(scl4(nv, 2.0), dot4(rd, nv)));
                reflecting = 1;
            } else if (ob->refractive_index == -1.0) {
                if (schlick(eye, nv, 1.0, 1.5) < noise3d(fgi, (float)(n * n), (float)b)) {
                    CNT(EV_UNDER);
                    over = sub4(pos, scl4(nv, EPSILON));
                } else {
                    CNT(EV_REFLECT);
                rd = sub4(rd, scl4(scl4(nv, 2.0), dot4(rd, nv)));
                    reflecting = 1;
                }
            } else if (ob->refractive_index != 1.0) {
                if (!inside) {
                    double sch = schlick(eye, nv, 1.0, ob->refractive_index);
                    double rnd = noise3d(fgi, (float)(n * n), (float)b);
                    if (sch < rnd) {
                        rd = refracted(eye, nv, 1.0, ob->refractive_index);
                        CNT(EV_UNDER);
                    over = sub4(pos, scl4(nv, EPSILON));
                        inside = 1;
                        entering = 1;
                        exiting = 0;
                    } else {
                        CNT(EV_REFLECT);
                rd = sub4(rd, scl4(scl4(nv, 2.0), dot4(rd, nv)));
                        reflecting = 1;
                    }
                } else {
                    double sch = schlick(eye, nv, ob->refractive_index, 1.0);
                    if (sch < noise3d(fgi, (float)(n * n), (float)b)) {
                        rd = refracted(eye, nv, ob->refractive_index, 1.0);
                        CNT(EV_UNDER);
                    over = sub4(pos, scl4(nv, EPSILON));
                        inside = 0;
                        entering = 0;
                        exiting = 1;
                    } else {
                        CNT(EV_REFLECT);
                rd = sub4(rd, scl4(scl4(nv, 2.0), dot4(rd, nv)));
                        entering = 0;
                        exiting = 0;
                        reflecting = 1;
                    }
                }
            } else {
                rd = random_hemisphere(nv, (double)fgi, (double)b, (double)n);
                cosine = dot4(rd, nv);
            }
            ro = over;
            bounce_t* bn = &bounces[b];
            bn->cosine = cosine;
            bn->is_refraction = entering || exiting;
            if (ob->type == 4) {
                bn->color = S->tris[h.tri].color;
                bn->emission = mk(0, 0, 0, 0);
            } else {
                bn->color = ob->color;
                bn->emission = ob->emission;
                if (ob->is_textured && (ob->type == 0 || ob->type == 1 || ob->type == 3)) { /* tracer.cl:1077-1092 */
                    d4 lp = mat_mul(ob->inverse, pos);
                    rgb_t c;
                    if (ob->type == 0) {
                        c = tex_sample(&S->tex[0], (float)(lp.x * ob->texture_scale[0]),
                                       (float)(lp.z * ob->texture_scale[1]), (float)ob->texture_index);
                    } else if (ob->type == 1) {
                        double u, v;
                        spherical_map(lp, &u, &v);
                        c = tex_sample(&S->tex[1], (float)u, (float)(1.0 - v), (float)ob->texture_index);
                    } else {
                        double u, v;
                        cube_uv(lp, &u, &v);
                        c = tex_sample(&S->tex[2], (float)u, (float)v, (float)ob->texture_index);
                    }
                    bn->color = mk((double)c.r, (double)c.g, (double)c.b, 1.0);
                }
            }
            if (!entering && !exiting && !reflecting) effective++;
            actual++;
            if (ob->emission.x > 0.0) break;
        }
        /* Shading reduction (tracer.cl:1116-1176). */
        d4 accum = mk(0, 0, 0, 0);
        d4 mask = mk(1, 1, 1, 1);
        for (unsigned k = 0; k < actual; k++) {
            const bounce_t* bn = &bounces[k];
            if (bn->is_refraction) continue;
            CNT(EV_REDUCE);
            accum = add4(accum, mul4(mask, bn->emission));
            if (bn->emission.x > 0.0) {
                if (k == 0) accum = bn->color;
                break;
            }
            mask = mul4(mask, bn->color);
            mask = scl4(mask, bn->cosine);
        }
        colors = add4(colors, accum);
    }
    return colors;
}

/* ---------------- C API ------------------------------------------------------ */

/* Renders rows [row0, row0+rows) of the frame.  With the full sample range the
 * output is the reference's RGBA (colors * 1/samples, alpha 1, tracer.cl:1184-1187);
 * with a partial range it is the un-normalised RGB sum and alpha = #samples.
 * `tex_pix/w/h/n` (may be NULL): the three texture arrays (ptmi_textures layout).
 * Returns 0, or <0 for bad input. */
int pto_trace_tex(const void* objects, uint32_t n_obj, const void* tris, uint32_t n_tri, const void* groups,
                  uint32_t n_grp, const void* camera, uint32_t samples, const double* seeds, uint32_t row0,
                  uint32_t rows, uint32_t s0, uint32_t s1, int threads, const uint8_t* const* tex_pix,
                  const uint32_t* tex_w, const uint32_t* tex_h, const uint32_t* tex_n, double* out) {
    if (n_obj == 0 || n_obj > 16 || samples == 0 || s1 > samples || s0 > s1) return -1;
    object_t* ob = (object_t*)calloc(n_obj, sizeof(object_t));
    group_t* gr = (group_t*)calloc(n_grp ? n_grp : 1, sizeof(group_t));
    tri_t* tr = (tri_t*)calloc(n_tri ? n_tri : 1, sizeof(tri_t));
    scene_t S;
    int rc = 0;
    for (uint32_t i = 0; i < n_obj; i++) {
        unpack_object((const uint8_t*)objects + 1024u * i, &ob[i]);
    }
    for (int k = 0; k < 3; k++) {
        S.tex[k].pix = NULL;
        S.tex[k].w = S.tex[k].h = S.tex[k].n = 0;
        if (tex_pix && tex_n[k] && tex_pix[k] && tex_w[k] && tex_h[k]) {
            S.tex[k].pix = tex_pix[k];
            S.tex[k].w = tex_w[k];
            S.tex[k].h = tex_h[k];
            S.tex[k].n = tex_n[k];
        }
    }
    for (uint32_t i = 0; i < n_grp; i++) unpack_group((const uint8_t*)groups + 256u * i, &gr[i]);
    for (uint32_t i = 0; i < n_tri; i++) unpack_tri((const uint8_t*)tris + 512u * i, &tr[i]);
    unpack_camera((const uint8_t*)camera, &S.cam);
    S.objects = ob;
    S.n_obj = n_obj;
    S.groups = gr;
    S.n_grp = n_grp;
    S.tris = tr;
    S.n_tri = n_tri;
    if (rc == 0) {
        const uint32_t W = (uint32_t)S.cam.width;
        const int full = (s0 == 0 && s1 == samples);
        const double cw = 1.0 / samples;
        const long npx = (long)W * rows;
#ifdef _OPENMP
        if (threads > 0) omp_set_num_threads(threads);
#endif
#ifdef PTO_COUNT
        memset(g_ev_total, 0, sizeof g_ev_total);
        g_xs_max_total = 0;
#pragma omp parallel
        {
            memset(g_ev, 0, sizeof g_ev);
            g_xs_max = 0;
#pragma omp for schedule(dynamic, 16)
            for (long p = 0; p < npx; p++) {
                uint32_t i = row0 * W + (uint32_t)p;
                d4 c = trace_pixel(&S, seeds, i, samples, s0, s1);
                double* o = out + 4 * p;
                o[0] = full ? c.x * cw : c.x;
                o[1] = full ? c.y * cw : c.y;
                o[2] = full ? c.z * cw : c.z;
                o[3] = full ? 1.0 : (double)(s1 - s0);
            }
#pragma omp critical
            {
                for (int e = 0; e < EV_COUNT; e++) g_ev_total[e] += g_ev[e];
                if (g_xs_max > g_xs_max_total) g_xs_max_total = g_xs_max;
            }
        }
#else
#pragma omp parallel for schedule(dynamic, 16)
        for (long p = 0; p < npx; p++) {
            uint32_t i = row0 * W + (uint32_t)p;
            d4 c = trace_pixel(&S, seeds, i, samples, s0, s1);
            double* o = out + 4 * p;
            if (full) {
                o[0] = c.x * cw;
                o[1] = c.y * cw;
                o[2] = c.z * cw;
                o[3] = 1.0;
            } else {
                o[0] = c.x;
                o[1] = c.y;
                o[2] = c.z;
                o[3] = (double)(s1 - s0);
            }
        }
#endif
    }
    free(ob);
    free(gr);
    free(tr);
    return rc;
}

int pto_trace(const void* objects, uint32_t n_obj, const void* tris, uint32_t n_tri, const void* groups,
              uint32_t n_grp, const void* camera, uint32_t samples, const double* seeds, uint32_t row0,
              uint32_t rows, uint32_t s0, uint32_t s1, int threads, double* out) {
    return pto_trace_tex(objects, n_obj, tris, n_tri, groups, n_grp, camera, samples, seeds, row0, rows, s0, s1,
                         threads, NULL, NULL, NULL, NULL, out);
}

/* Texture helpers exported for the unit tests (sampler and UV maps alone). */
void pto_tex_sample(const uint8_t* pix, uint32_t w, uint32_t h, uint32_t n, float s, float t, float layer,
                    float* rgb) {
    tex_t T = {pix, w, h, n};
    rgb_t c = tex_sample(&T, s, t, layer);
    rgb[0] = c.r, rgb[1] = c.g, rgb[2] = c.b;
}
void pto_spherical_map(double x, double y, double z, double* uv) { spherical_map(mk(x, y, z, 1.0), &uv[0], &uv[1]); }
void pto_cube_uv(double x, double y, double z, double* uv) { cube_uv(mk(x, y, z, 1.0), &uv[0], &uv[1]); }

float pto_noise3d(float x, float y, float z) { return noise3d(x, y, z); }
/* intersectRayWithBox (tracer.cl:270-280) on a ray given as o[4], d[4] and a box mn[3], mx[3]. */
int pto_ray_box(const double* o, const double* d, const double* mn, const double* mx) {
    return ray_box(mk(o[0], o[1], o[2], o[3]), mk(d[0], d[1], d[2], d[3]), mk(mn[0], mn[1], mn[2], 1.0),
                   mk(mx[0], mx[1], mx[2], 1.0));
}

/* Event totals of the last pto_trace call (PTO_COUNT build; else returns 0). */
int pto_event_counts(uint64_t* out, int n) {
#ifdef PTO_COUNT
    for (int e = 0; e < n && e < EV_COUNT; e++) out[e] = g_ev_total[e];
    return EV_COUNT;
#else
    (void)out;
    (void)n;
    return 0;
#endif
}
/* The most ctx entries one findClosestIntersection call of the last pto_trace recorded
 * (PTO_COUNT build; else -1). */
int pto_max_candidates(void) {
#ifdef PTO_COUNT
    return g_xs_max_total;
#else
    return -1;
#endif
}
float pto_sinf32(float x) { return pto_sinf(x); }
void pto_sinf_many(const float* in, float* out, size_t n) {
    for (size_t i = 0; i < n; i++) out[i] = pto_sinf(in[i]);
}
