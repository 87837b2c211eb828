// ptmi_kernels.hip -- gfx950 (MI355X / CDNA4) path-tracing kernels.
//
// One lane = one pixel of an 8x8 tile (one wave64 per tile), looping over a
// chunk of that pixel's samples; FP64 throughout, float RNG exactly as the
// reference (tracer.cl:314-317).  The integrator restates `trace`
// (tracer.cl:831-1188); every helper cites the reference lines it follows.
//
// Compiled with -ffp-contract=off (separately rounded user arithmetic, as the
// pinned reference build) and calls the same ROCm device-library functions the
// reference's OpenCL builtins resolve to (ocml sin_f32 / sin/cos/pow/sqrt/rsqrt
// f64, maxnum/minnum), so on the same inputs the image matches the reference
// kernel bit-for-bit in practice (tests/test_gpu_parity.py).
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "ptmi_device.h"

namespace ptmi {

static constexpr unsigned kMaxEffectiveBounces = 4;  // tracer.cl:2
static constexpr unsigned kMaxBounces = 10;          // tracer.cl:3
static constexpr double kEps = 0.0001;               // tracer.cl:4
static constexpr double kPi = (double)3.14159265359f;  // tracer.cl:1 (a float literal)

struct d4 {
    double x, y, z, w;
};
__device__ __forceinline__ d4 mk(double x, double y, double z, double w) { return d4{x, y, z, w}; }
__device__ __forceinline__ d4 add4(d4 a, d4 b) { return mk(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w); }
__device__ __forceinline__ d4 sub4(d4 a, d4 b) { return mk(a.x - b.x, a.y - b.y, a.z - b.z, a.w - b.w); }
__device__ __forceinline__ d4 scl4(d4 a, double s) { return mk(a.x * s, a.y * s, a.z * s, a.w * s); }
__device__ __forceinline__ d4 ld4(const double* p) { return mk(p[0], p[1], p[2], p[3]); }

// OpenCL dot/cross(double4) as ROCm device-libs implement them (fmuladd == fma).
__device__ __forceinline__ double dot4(d4 a, d4 b) {
    double d = a.x * b.x;
    d = fma(a.y, b.y, d);
    d = fma(a.z, b.z, d);
    return fma(a.w, b.w, d);
}
__device__ __forceinline__ d4 cross4(d4 a, d4 b) {
    return mk(fma(a.y, b.z, b.y * -a.z), fma(a.z, b.x, b.z * -a.x), fma(a.x, b.y, b.x * -a.y), 0.0);
}
// OpenCL normalize(double4) (opencl.bc): zero passthrough, range scaling, rsqrt.
__device__ __noinline__ d4 normalize4(d4 v) {
    if (v.x == 0.0 && v.y == 0.0 && v.z == 0.0 && v.w == 0.0) return v;
    double d = dot4(v, v);
    d4 p = v;
    if (d < 0x1p-1022) {
        p = scl4(v, 0x1p563);
        d = dot4(p, p);
    } else if (d == __builtin_inf()) {
        p = scl4(v, 0x1p-514);
        d = dot4(p, p);
        if (d == __builtin_inf()) {
            p = mk(copysign(isinf(p.x) ? 1.0 : 0.0, p.x), copysign(isinf(p.y) ? 1.0 : 0.0, p.y),
                   copysign(isinf(p.z) ? 1.0 : 0.0, p.z), copysign(isinf(p.w) ? 1.0 : 0.0, p.w));
            d = dot4(p, p);
        }
    }
    return scl4(p, rsqrt(d));
}
// maxX / minX (tracer.cl:110-111): OpenCL max/min -> maxnum/minnum.
__device__ __forceinline__ double max3(double a, double b, double c) { return fmax(fmax(a, b), c); }
__device__ __forceinline__ double min3(double a, double b, double c) { return fmin(fmin(a, b), c); }

// mul (tracer.cl:369-376): row-major mat4 x vec4, rows summed x+y+z+w.
__device__ __forceinline__ d4 mat_mul(const double* __restrict__ m, d4 v) {
    return mk(((m[0] * v.x + m[1] * v.y) + m[2] * v.z) + m[3] * v.w,
              ((m[4] * v.x + m[5] * v.y) + m[6] * v.z) + m[7] * v.w,
              ((m[8] * v.x + m[9] * v.y) + m[10] * v.z) + m[11] * v.w,
              ((m[12] * v.x + m[13] * v.y) + m[14] * v.z) + m[15] * v.w);
}

// noise3D (tracer.cl:314-317): float math, ocml sin_f32, ocml fract_f32.
__device__ __forceinline__ float noise3d(float x, float y, float z) {
    float a = x * 112.9898f;
    float b = y * 179.233f;
    float c = z * 237.212f;
    float s = (a + b) + c;
    float v = sinf(s) * 43758.5453f;
    float r = fminf(v - floorf(v), 0x1.fffffep-1f);
    return isnan(v) ? v : (isinf(v) ? 0.0f : r);
}

// checkAxis (tracer.cl:250-268)
__device__ __forceinline__ void check_axis(double o, double d, double mn, double mx, double& t0, double& t1) {
    double a0 = mn - o, a1 = mx - o;
    double a, b;
    if (fabs(d) >= kEps) {
        a = a0 / d;
        b = a1 / d;
    } else {
        a = a0 * __builtin_huge_val();
        b = a1 * __builtin_huge_val();
    }
    t0 = a > b ? b : a;
    t1 = a > b ? a : b;
}

// intersectRayWithBox (tracer.cl:270-280): a line test (no t range).
__device__ __forceinline__ bool ray_box(d4 o, d4 d, const double* mn, const double* mx) {
    double x0, x1, y0, y1, z0, z1;
    check_axis(o.x, d.x, mn[0], mx[0], x0, x1);
    check_axis(o.y, d.y, mn[1], mx[1], y0, y1);
    check_axis(o.z, d.z, mn[2], mx[2], z0, z1);
    return max3(x0, y0, z0) < min3(x1, y1, z1);
}

struct Hit {
    double t;
    int obj;
    int tri;
    double u, v;
};

// The reference records every candidate then picks the first t > EPSILON that
// is strictly below the running best (start 1024) in recording order
// (tracer.cl:728-739); reducing on the fly in the same order is identical.
__device__ __forceinline__ void consider(Hit& h, double t, int obj) {
    if (t > kEps && t < h.t) {
        h.t = t;
        h.obj = obj;
        h.tri = -1;
    }
}

// Stack-based BVH walk of one group root, in the reference's preorder
// (tracer.cl:621-719), Moller-Trumbore per triangle (640-675).
__device__ __noinline__ void walk_group(const DevScene& S, int root, int obj, d4 o, d4 d, Hit& h) {
    int stack[64];
    int sidx = 0;
    int cur_idx = root;
    const DevNode* cur = &S.nodes[cur_idx];
    for (;;) {
        while (cur && ray_box(o, d, cur->bb_min, cur->bb_max)) {
            const int end = cur->tri_offset + cur->tri_count;
            for (int n = cur->tri_offset; n < end; n++) {
                const DevTri& T = S.tris[n];
                const d4 e1 = ld4(T.e1), e2 = ld4(T.e2);
                d4 dce2 = cross4(d, e2);
                double det = dot4(e1, dce2);
                if (fabs(det) < kEps) continue;
                double f = 1.0 / det;
                d4 p1o = sub4(o, ld4(T.p1));
                double u = f * dot4(p1o, dce2);
                if (u < 0 || u > 1) continue;
                d4 oce1 = cross4(p1o, e1);
                double v = f * dot4(d, oce1);
                if (v < 0 || (u + v) > 1) continue;
                double t = f * dot4(e2, oce1);
                if (t > kEps && t < h.t) {
                    h.t = t;
                    h.obj = obj;
                    h.tri = n;
                    h.u = u;
                    h.v = v;
                }
            }
            stack[sidx++] = cur_idx;
            if (cur->child0 > 0) {
                cur_idx = cur->child0;
                cur = &S.nodes[cur_idx];
            } else {
                cur = nullptr;
            }
        }
        sidx--;
        if (sidx == -1) break;
        cur = &S.nodes[stack[sidx]];
        if (cur->child1 > 0) {
            cur_idx = cur->child1;
            cur = &S.nodes[cur_idx];
        } else {
            cur = nullptr;
        }
    }
}

// findClosestIntersection (tracer.cl:537-742).  The object loop index is
// wave-uniform, so the per-object matrices come in through scalar loads.
__device__ __forceinline__ Hit find_closest(const DevScene& S, d4 ro, d4 rd) {
    Hit h{1024.0, -1, -1, 0.0, 0.0};
    for (uint32_t j = 0; j < S.n_obj; j++) {
        const DevObject& ob = S.objs[j];
        const int type = ob.type;
        d4 o = mat_mul(ob.inv, ro);
        d4 d = mat_mul(ob.inv, rd);
        if (type == 0) {  // intersectPlane (478-483)
            double t = fabs(d.y) > kEps ? -o.y / d.y : 0.0;
            if (t != 0.0) consider(h, t, (int)j);
        } else if (type == 1) {  // intersectSphere (448-476)
            d4 vtc = mk(o.x - 0.0, o.y - 0.0, o.z - 0.0, o.w - 1.0);
            double a = dot4(d, d);
            double b = 2.0 * dot4(d, vtc);
            double c = dot4(vtc, vtc) - 1.0;
            double disc = (b * b) - 4 * a * c;
            if (disc > 0.0) {
                double sq = sqrt(disc);
                double t1 = (-b - sq) / (2 * a);
                double t2 = (-b + sq) / (2 * a);
                if (t1 != 0.0) consider(h, t1, (int)j);
                if (t2 != 0.0) consider(h, t2, (int)j);
            }
        } else if (type == 2) {  // intersectCylinder (396-446), caps disabled
            double a = d.x * d.x + d.z * d.z;
            if (!(fabs(a) < kEps)) {
                double b = 2 * o.x * d.x + 2 * o.z * d.z;
                double c1 = o.x * o.x + o.z * o.z - 1;
                double disc = b * b - 4 * a * c1;
                if (!(disc < 0.0)) {
                    double sq = sqrt(disc);
                    double t0 = (-b - sq) / (2 * a);
                    double t1 = (-b + sq) / (2 * a);
                    double y0 = o.y + t0 * d.y;
                    double y1 = o.y + t1 * d.y;
                    double r0 = (y0 > ob.min_y && y0 < ob.max_y) ? t0 : 0.0;
                    double r1 = (y1 > ob.min_y && y1 < ob.max_y) ? t1 : 0.0;
                    if (r0 != 0) consider(h, r0, (int)j);
                    if (r1 != 0) consider(h, r1, (int)j);
                }
            }
        } else if (type == 3) {  // intersectCube (378-394)
            double x0, x1, y0, y1, z0, z1;
            check_axis(o.x, d.x, -1.0, 1.0, x0, x1);
            check_axis(o.y, d.y, -1.0, 1.0, y0, y1);
            check_axis(o.z, d.z, -1.0, 1.0, z0, z1);
            double tmin = max3(x0, y0, z0), tmax = min3(x1, y1, z1);
            if (!(tmin > tmax)) {
                if (tmin != 0.0) consider(h, tmin, (int)j);
                if (tmax != 0.0) consider(h, tmax, (int)j);
            }
        } else if (type == 4) {  // groups (598-720)
            if (!ray_box(o, d, ob.bb_min, ob.bb_max)) continue;
            for (int ci = 0; ci < ob.child_count; ci++) walk_group(S, S.roots[ob.child_base + ci], (int)j, o, d, h);
        }
    }
    return h;
}

// schlick (tracer.cl:485-505)
__device__ __noinline__ double schlick(d4 eye, d4 nrm, double n1, double n2) {
    double c = dot4(eye, nrm);
    if (n1 > n2) {
        double n = n1 / n2;
        double s2 = (n * n) * (1.0 - (c * c));
        if (s2 > 1.0) return 1.0;
        c = sqrt(1.0 - s2);
    }
    double tmp = (n1 - n2) / (n1 + n2);
    double r0 = tmp * tmp;
    return r0 + (1 - r0) * pow(1 - c, 5.0);
}

// computeRefractedRay (tracer.cl:507-533)
__device__ __noinline__ d4 refracted(d4 eye, d4 nrm, double n1, double n2) {
    double nr = n1 / n2;
    double ci = dot4(eye, nrm);
    double s2 = (nr * nr) * (1.0 - (ci * ci));
    if (s2 > 1.0) return mk(0, 0, 0, 0);
    double ct = sqrt(1.0 - s2);
    return sub4(scl4(nrm, (nr * ci) - ct), scl4(eye, nr));
}

__device__ __forceinline__ d4 reflect(d4 rd, d4 nv) { return sub4(rd, scl4(scl4(nv, 2.0), dot4(rd, nv))); }

// randomVectorInHemisphere (tracer.cl:348-366); x, y, z hold float-valued doubles.
__device__ __forceinline__ d4 random_hemisphere(d4 nv, float fx, float fy, float fz) {
    double rand1 = 2.0 * kPi * (double)noise3d(fx, fy, fz);
    double rand2 = (double)noise3d(fy, fz, fx);
    double rand2s = sqrt(rand2);
    d4 axis = fabs(nv.x) > 0.1 ? mk(0.0, 1.0, 0.0, 0.0) : mk(1.0, 0.0, 0.0, 0.0);
    d4 u = normalize4(cross4(axis, nv));
    d4 v = cross4(nv, u);
    double cr = cos(rand1), sr = sin(rand1);
    return add4(add4(scl4(scl4(u, cr), rand2s), scl4(scl4(v, sr), rand2s)), scl4(nv, sqrt(1.0 - rand2)));
}

// sunflower (tracer.cl:221-248), randomize == false.
__device__ __noinline__ void sunflower(int amount, int point, double& ox, double& oy) {
    double idx = (double)point;
    double sqp = sqrt((double)amount);
    double b = round(2.0 * sqp);
    const double phi = (sqrt(5.0) + 1.0) / 2.0;
    double n = (double)amount;
    double r = 1.0;
    if (idx <= (n - b)) r = sqrt(idx - 0.5) / sqrt(n - (b + 1.0) / 2.0);
    double theta = 2.0 * kPi * idx / (phi * phi);
    ox = r * cos(theta);
    oy = r * sin(theta);
}

// rayForPixel (tracer.cl:745-779)
__device__ __forceinline__ void ray_for_pixel(const DevCamera& cam, unsigned x, unsigned y, float rx, float ry,
                                              int sample, int total, d4& ro, d4& rd) {
    double xo = cam.pixel_size * ((double)x + (double)rx);
    double yo = cam.pixel_size * ((double)y + (double)ry);
    d4 piv = mk(cam.half_width - xo, cam.half_height - yo, -1.0, 1.0);
    d4 pixel = mat_mul(cam.inv, piv);
    d4 origin = mat_mul(cam.inv, mk(0.0, 0.0, 0.0, 1.0));
    d4 dir = normalize4(sub4(pixel, origin));
    if (cam.aperture != 0) {
        d4 pos = add4(origin, scl4(dir, cam.focal_length));
        double sx, sy;
        sunflower(total, sample, sx, sy);
        d4 no = mk(origin.x + (sy * cam.aperture), origin.y + (sx * cam.aperture), origin.z, 1.0);
        dir = sub4(pos, no);
        origin = no;
    }
    ro = origin;
    rd = dir;
}

// One path (the body of the sample loop, tracer.cl:867-1179) with the shading
// reduction (1116-1176) applied as bounces are produced: identical arithmetic,
// no bounce array.  Returns the path's accumColor.xyz.
__device__ __forceinline__ void trace_path(const DevScene& S, float fgi, float fgi2, unsigned x, unsigned y,
                                           uint32_t n, uint32_t samples, double& ar, double& ag, double& ab) {
    d4 ro, rd;
    ray_for_pixel(S.cam, x, y, noise3d(fgi, (float)n, fgi2), noise3d(fgi, fgi2, (float)n), (int)n, (int)samples, ro,
                  rd);
    double mr = 1.0, mg = 1.0, mb = 1.0;  // mask
    ar = ag = ab = 0.0;                    // accumColor
    bool done = false;                     // the reduction has hit its `break`
    bool inside = false;
    unsigned effective = 0, k = 0;
    for (uint32_t b = 0; b < kMaxBounces && effective < kMaxEffectiveBounces; b++) {
        Hit h = find_closest(S, ro, rd);
        if (h.obj < 0) break;  // a miss repeats identically until b == 10 in the reference
        const DevObject& ob = S.objs[h.obj];
        const int type = ob.type;
        d4 pos = add4(ro, scl4(rd, h.t));
        d4 eye = mk(-rd.x, -rd.y, -rd.z, -rd.w);
        d4 on;
        if (type == 0) {
            on = mk(0.0, 1.0, 0.0, 0.0);
        } else if (type == 1) {
            d4 lp = mat_mul(ob.inv, pos);
            on = mk(lp.x - 0.0, lp.y - 0.0, lp.z - 0.0, lp.w - 1.0);
        } else if (type == 2) {
            d4 lp = mat_mul(ob.inv, pos);
            double dist = lp.x * lp.x + lp.z * lp.z;  // pow(v, 2) folds to v*v
            if (dist < 1 && lp.y >= ob.max_y - kEps) on = mk(0.0, 1.0, 0.0, 0.0);
            else if (dist < 1 && lp.y <= ob.min_y + kEps) on = mk(0.0, -1.0, 0.0, 0.0);
            else on = mk(lp.x, 0.0, lp.z, 0.0);
        } else if (type == 3) {
            d4 lp = mat_mul(ob.inv, pos);
            double mc = max3(fabs(lp.x), fabs(lp.y), fabs(lp.z));
            if (mc == fabs(lp.x)) on = mk(lp.x, 0.0, 0.0, 0.0);
            else if (mc == fabs(lp.y)) on = mk(0.0, lp.y, 0.0, 0.0);
            else on = mk(0.0, 0.0, lp.z, 0.0);
        } else {  // group: interpolated vertex normal of the winning triangle (tracer.cl:669, 949)
            const DevTriShade& T = S.tri_shade[h.tri];
            on = add4(add4(scl4(ld4(T.n2), h.u), scl4(ld4(T.n3), h.v)), scl4(ld4(T.n1), 1.0 - h.u - h.v));
        }
        d4 nv = mat_mul(ob.inv_t, on);
        nv.w = 0.0;
        nv = normalize4(nv);
        if (dot4(eye, nv) < 0.0) nv = scl4(nv, -1.0);
        d4 over = add4(pos, scl4(nv, kEps));
        double cosine = 1.0;
        bool entering = false, exiting = false, reflecting = false;
        // Material decision (tracer.cl:973-1061)
        if (ob.reflectivity != 0.0 && noise3d(fgi, (float)n, (float)b) < ob.reflectivity) {
            rd = reflect(rd, nv);
            reflecting = true;
        } else if (ob.refractive_index == -1.0) {
            if (schlick(eye, nv, 1.0, 1.5) < noise3d(fgi, (float)(n * n), (float)b)) {
                over = sub4(pos, scl4(nv, kEps));
            } else {
                rd = reflect(rd, nv);
                reflecting = true;
            }
        } else if (ob.refractive_index != 1.0) {
            const double ri = ob.refractive_index;
            const double sch = inside ? schlick(eye, nv, ri, 1.0) : schlick(eye, nv, 1.0, ri);
            if (sch < noise3d(fgi, (float)(n * n), (float)b)) {
                rd = inside ? refracted(eye, nv, ri, 1.0) : refracted(eye, nv, 1.0, ri);
                over = sub4(pos, scl4(nv, kEps));
                entering = !inside;
                exiting = inside;
                inside = !inside;
            } else {
                rd = reflect(rd, nv);
                reflecting = true;
            }
        } else {
            rd = random_hemisphere(nv, fgi, (float)b, (float)n);
            cosine = dot4(rd, nv);
        }
        ro = over;
        // Bounce record + reduction step (tracer.cl:1071-1096, 1148-1175).
        if (!done && !(entering || exiting)) {
            double er, eg, eb, cr, cg, cb;
            if (type == 4) {
                const DevTriShade& T = S.tri_shade[h.tri];
                er = eg = eb = 0.0;
                cr = T.color[0];
                cg = T.color[1];
                cb = T.color[2];
            } else {
                er = ob.emission[0];
                eg = ob.emission[1];
                eb = ob.emission[2];
                cr = ob.color[0];
                cg = ob.color[1];
                cb = ob.color[2];
            }
            ar = ar + mr * er;
            ag = ag + mg * eg;
            ab = ab + mb * eb;
            if (er > 0.0) {
                if (k == 0) {
                    ar = cr;
                    ag = cg;
                    ab = cb;
                }
                done = true;
            } else {
                mr = mr * cr;
                mg = mg * cg;
                mb = mb * cb;
                mr = mr * cosine;
                mg = mg * cosine;
                mb = mb * cosine;
            }
        }
        if (!entering && !exiting && !reflecting) effective++;
        k++;
        if (ob.emission[0] > 0.0) break;
    }
}

// grid: x = 4 tiles per block (one 8x8 tile per wave), y = sample chunk.
// Writes the chunk's RGB sums (A = #samples) to out[(chunk*npix + pixel)*4].
__global__ __launch_bounds__(256) void trace_kernel(DevScene S, uint32_t samples, uint32_t s_begin, uint32_t s_end,
                                                    uint32_t chunk_len, uint32_t tile_stride, uint32_t tile_offset,
                                                    const double* __restrict__ seeds, double* __restrict__ out) {
    const int W = S.cam.width, H = S.cam.height;
    const int tiles_x = (W + kTile - 1) / kTile;
    const int tiles_y = (H + kTile - 1) / kTile;
    const int wave = threadIdx.x >> 6, lane = threadIdx.x & 63;
    const int tile = blockIdx.x * kWavesPerBlock + wave;
    if (tile >= tiles_x * tiles_y) return;
    if ((uint32_t)tile % tile_stride != tile_offset) return;
    const int px = (tile % tiles_x) * kTile + (lane & 7);
    const int py = (tile / tiles_x) * kTile + (lane >> 3);
    if (px >= W || py >= H) return;
    const uint32_t i = (uint32_t)py * (uint32_t)W + (uint32_t)px;
    const uint32_t c0 = s_begin + blockIdx.y * chunk_len;
    const uint32_t c1 = min(s_end, c0 + chunk_len);
    // fgi / fgi2 (tracer.cl:839-841): double division rounded to float.
    const double seed = seeds[i];
    const float fgi = (float)(seed / (double)S.n_obj);
    const float fgi2 = (float)(seed / (double)samples);
    double cr = 0.0, cg = 0.0, cb = 0.0;
    for (uint32_t n = c0; n < c1; n++) {
        double ar, ag, ab;
        trace_path(S, fgi, fgi2, (unsigned)px, (unsigned)py, n, samples, ar, ag, ab);
        cr = cr + ar;
        cg = cg + ag;
        cb = cb + ab;
    }
    double* o = out + ((size_t)blockIdx.y * ((size_t)W * H) + i) * 4;
    o[0] = cr;
    o[1] = cg;
    o[2] = cb;
    o[3] = (double)(c1 > c0 ? c1 - c0 : 0);
}

// Sum chunk partials in chunk order (deterministic); zero un-owned pixels.
__global__ __launch_bounds__(256) void reduce_chunks_kernel(const double* __restrict__ part, double* __restrict__ sums,
                                                            uint32_t npix, uint32_t nchunks, int W, int H,
                                                            uint32_t tile_stride, uint32_t tile_offset) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const int px = (int)(i % (uint32_t)W), py = (int)(i / (uint32_t)W);
    const int tiles_x = (W + kTile - 1) / kTile;
    const uint32_t tile = (uint32_t)((py / kTile) * tiles_x + px / kTile);
    double r = 0.0, g = 0.0, b = 0.0, a = 0.0;
    if (tile % tile_stride == tile_offset) {
        for (uint32_t c = 0; c < nchunks; c++) {
            const double* p = part + ((size_t)c * npix + i) * 4;
            r = r + p[0];
            g = g + p[1];
            b = b + p[2];
            a = a + p[3];
        }
    }
    double* o = sums + (size_t)i * 4;
    o[0] = r;
    o[1] = g;
    o[2] = b;
    o[3] = a;
}

// colors * (1.0 / samples), alpha 1 (tracer.cl:837, 1184-1187).
__global__ __launch_bounds__(256) void finalize_kernel(const double* __restrict__ sums, double* __restrict__ out,
                                                       uint32_t npix, uint32_t samples) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= npix) return;
    const double w = 1.0 / samples;
    out[4 * (size_t)i + 0] = sums[4 * (size_t)i + 0] * w;
    out[4 * (size_t)i + 1] = sums[4 * (size_t)i + 1] * w;
    out[4 * (size_t)i + 2] = sums[4 * (size_t)i + 2] * w;
    out[4 * (size_t)i + 3] = 1.0;
}

// Seeds with Go rand.Float64 granularity (k / 2^53) from a SplitMix64 stream.
__global__ __launch_bounds__(256) void seeds_kernel(double* __restrict__ seeds, uint32_t n, uint64_t stream) {
    const uint32_t i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t z = stream + 0x9E3779B97F4A7C15ull * (uint64_t)(i + 1);
    z = (z ^ (z >> 30)) * 0xBF58476D1CE4E5B9ull;
    z = (z ^ (z >> 27)) * 0x94D049BB133111EBull;
    z = z ^ (z >> 31);
    seeds[i] = (double)(z >> 11) * 0x1p-53;
}

// ---- host-side launch wrappers (called from ptmi_api.cpp) ----------------------
const void* trace_kernel_symbol() { return reinterpret_cast<const void*>(&trace_kernel); }

hipError_t launch_trace(const DevScene& S, uint32_t samples, uint32_t s_begin, uint32_t s_end, uint32_t chunk_len,
                        uint32_t nchunks, uint32_t tile_stride, uint32_t tile_offset, const double* seeds,
                        double* out, hipStream_t st) {
    const int tiles = ((S.cam.width + kTile - 1) / kTile) * ((S.cam.height + kTile - 1) / kTile);
    dim3 grid((tiles + kWavesPerBlock - 1) / kWavesPerBlock, nchunks);
    hipLaunchKernelGGL(trace_kernel, grid, dim3(256), 0, st, S, samples, s_begin, s_end, chunk_len, tile_stride,
                       tile_offset, seeds, out);
    return hipGetLastError();
}

hipError_t launch_reduce(const double* part, double* sums, uint32_t npix, uint32_t nchunks, int W, int H,
                         uint32_t tile_stride, uint32_t tile_offset, hipStream_t st) {
    hipLaunchKernelGGL(reduce_chunks_kernel, dim3((npix + 255) / 256), dim3(256), 0, st, part, sums, npix, nchunks, W,
                       H, tile_stride, tile_offset);
    return hipGetLastError();
}

hipError_t launch_finalize(const double* sums, double* out, uint32_t npix, uint32_t samples, hipStream_t st) {
    hipLaunchKernelGGL(finalize_kernel, dim3((npix + 255) / 256), dim3(256), 0, st, sums, out, npix, samples);
    return hipGetLastError();
}

hipError_t launch_seeds(double* seeds, uint32_t n, uint64_t stream, hipStream_t st) {
    hipLaunchKernelGGL(seeds_kernel, dim3((n + 255) / 256), dim3(256), 0, st, seeds, n, stream);
    return hipGetLastError();
}

}  // namespace ptmi
