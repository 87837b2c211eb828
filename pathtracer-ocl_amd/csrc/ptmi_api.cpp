// ptmi_api.cpp -- C ABI of libptmi.so (include/ptmi.h): record validation and
// conversion to the HBM layout (ptmi_device.h), device residency, launch
// orchestration.  Replaces the reference host driver internal/ocl/ocltracer.go
// (Trace / computeBatch, ocltracer.go:98-376).
#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdlib>
#include <cstdarg>
#include <cstdio>
#include <cstddef>
#include <cstring>
#include <mutex>
#include <string>
#include <thread>
#include <vector>

#include "../../include/ptmi.h"
#include "../../include/ptmi_diag.h"
#include "ptmi_bvh.h"
#include "ptmi_device.h"
#include "ptmi_f16.h"

// DIAGNOSTIC study build (make study): the split execution form, the standalone walk
// kernels and the measured tile order (ptmi_kernels.hip PTMI_STUDY).  The product has 0.
#ifndef PTMI_STUDY
#define PTMI_STUDY 0
#endif

namespace ptmi {
hipError_t launch_trace(const DevScene& S, int flags, uint32_t samples, const WorkPlan& WP, const double* seeds,
                        const double* sunf, double* sums, double* part, uint32_t* item_ctr,
                        hipStream_t st);
hipError_t launch_sunflower(double* out, uint32_t samples, hipStream_t st);
hipError_t launch_reduce(const double* part, double* sums, const WorkPlan& WP, int W, int H, bool planes,
                         hipStream_t st);
hipError_t launch_finalize(const double* sums, double* out, uint32_t npix, uint32_t samples, hipStream_t st);
hipError_t launch_seeds(double* seeds, uint32_t n, uint64_t stream, hipStream_t st);
hipError_t launch_plane_normals(DevObject* objs, int n, hipStream_t st);
hipError_t launch_hemi_table(double* out, int* mismatch, hipStream_t st);
hipError_t launch_combine(const double* parts, uint32_t nparts, size_t npix, double* out, uint32_t samples,
                          hipStream_t st);
const void* trace_kernel_symbol(int flags);
bool tile_list_supported(int flags);
int trace_kernel_flags(int flags);
#if PTMI_STUDY
hipError_t launch_tile_order(unsigned long long* cost, uint32_t n_whole, uint32_t n_tail, uint32_t stride,
                             uint32_t offset, uint32_t* order, hipStream_t st);
bool split_supported(int flags);
const void* trace_split_symbol(int flags);
const void* walk_split_symbol();
hipError_t launch_split_pass(const DevScene& S, int flags, uint32_t samples, const WorkPlan& WP, const SplitBufs& B,
                             const double* seeds, const double* sunf, double* part, uint32_t walk_grid,
                             hipStream_t st);
#endif
int trace_block_threads(int flags);
int trace_tiles_per_block(int flags);
}  // namespace ptmi

using namespace ptmi;

// What mesh_tile_cost needs of a scene, kept with it so the tile classes are computed on
// the first render that orders tiles, and only for the tiles that render owns: the camera
// and, per group object, rows 0-2 of its inverse and its roots' hulls.
struct TileCostInput {
    DevCamera cam{};
    struct Obj {
        double inv[12];
        std::vector<std::array<double, 6>> hulls;  // (mn xyz, mx xyz) per root
    };
    std::vector<Obj> objs;
};

struct ptmi_scene {
    int device = 0;
    DevScene dev{};
    void* buffers[15] = {};  // [10..12]: texture arrays, [13]: hemisphere table, [14]: camera record
    double* partial = nullptr;  // chunk partial sums, grown on demand
    double* sunf = nullptr;     // DoF aperture table for sunf_samples (sunflower_kernel)
    uint32_t sunf_samples = 0;
    size_t partial_bytes = 0;
    int resident_waves = 0;  // device-wide resident waves of trace_kernel
    uint32_t tail_tiles = 0;  // chunked tiles at the end of an automatic launch; 0: default (see render)
    uint32_t tail_items = 6;  // chunk items per resident wave slot in the tail (scenes without meshes; see render)
    uint32_t mesh_items = 32;  // chunk items per resident wave slot, mesh scenes (every tile chunked)
    uint32_t mesh_items_share = 48;  // ... in a sample-split rank's share (a sub-range of the samples)
    uint32_t min_chunk = 32;   // fewest samples per chunk item (see render)
    uint32_t tail_split = 4;   // mesh scenes: the last chunk round cut into this many (see render)
    uint32_t tail_min = 0;     // ... while those keep at least this many samples; 0: automatic (see render)
    // Mesh scenes: per-tile cost class (mesh_tile_cost) and the dispatch order built from it
    // for the last (tile_stride, tile_offset) rendered (see render).
    // 0: raster order, 1: static (hull-hit classes), 2: measured by the last launch (needs a
    // build with PTMI_TILE_COST=1 -- see ptmi_kernels.hip item_cost_add; else the order is
    // arbitrary within the static plan, which never changes a result)
    int tile_order = 1;
    TileCostInput tc_in;              // mesh scenes: the inputs of the tile classes
    std::vector<uint8_t> tile_cost;   // per tile: its class, or kCostUnset until a render needs it
    std::vector<uint32_t> order_host;
    uint32_t* order_dev = nullptr;
    unsigned long long* cost_dev = nullptr;  // study build: per-tile durations of the launches since the last order
    uint32_t order_stride = 0, order_offset = 0, order_n = 0, order_whole = 0, order_cap = 0;
    // Tile-split launches of the affine mesh kernels: the owned-tile list (WorkPlan::tiles)
    // of the last (tile_stride, tile_offset) rendered with one (see owned_tile).
    std::vector<uint32_t> tlist_host;
    uint32_t* tlist_dev = nullptr;
    uint32_t* item_ctr = nullptr;  // the mesh kernels' work-item counter (ptmi_kernels.hip take_item), zeroed per launch
    uint32_t tlist_stride = 0, tlist_offset = 0, tlist_cap = 0;
    bool order_tlist = false;  // the dispatch order was built for a list launch
    uint32_t width = 0, height = 0;
    int flags = 0;  // scene features -> kernel instantiation (ptmi_kernels.hip F_*)
    int hemi_mismatch = 0;  // hemisphere-table records where affine and generic sequences differ (upload_scene)
    int rng = PTMI_RNG_NOISE3D;  // ptmi_scene_set_rng: PTMI_RNG_XOSHIRO launches the F_XRNG instantiations
    bool timing = false;
    std::vector<std::pair<hipEvent_t, hipEvent_t>> events;  // pending (start, stop) pairs
    std::vector<hipEvent_t> spare;
#if PTMI_STUDY
    // Split execution of affine mesh scenes (ptmi_kernels.hip trace_split_kernel): a measured
    // alternative (3.3x slower than the one-kernel form on C4), study build only;
    // ptmi_diag_set_split(s, 1) selects it, ptmi_diag_set_knob tunes it.
    int split = 0;
    uint32_t split_chunk = 64;       // samples per pixel-chunk (PTMI_KNOB_SPLIT_CHUNK)
    uint32_t split_per_lane = 4;     // slots per tracer lane slot (PTMI_KNOB_SPLIT_SLOTS)
    uint32_t split_sync = 8;         // passes between completion checks (PTMI_KNOB_SPLIT_SYNC)
    uint32_t split_budget = 4;       // samples a slot starts per pass (PTMI_KNOB_SPLIT_BUDGET)
    SplitBufs sb{};
    void* split_mem = nullptr;
    size_t split_bytes = 0;
    uint32_t* split_host = nullptr;  // pinned: the request count read back at a check
    uint32_t split_passes = 0;       // passes of the last split render (diagnostics)
#endif
};

// ptmi_diag_force_flags: kernel flags forced onto every scene created after the call
// (-1: none).  Test hook for the generic instantiations.
static std::atomic<int> g_force_flags{-1};

namespace {

void set_err(char* err, size_t n, const char* fmt, ...) {
    if (!err || n == 0) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err, n, fmt, ap);
    va_end(ap);
}

#define HIP_TRY(call)                                                                             \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            set_err(err, err_len, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                                    \
            return PTMI_ERR_HIP;                                                                  \
        }                                                                                         \
    } while (0)

template <typename T>
T rd(const uint8_t* p) {
    T v;
    std::memcpy(&v, p, sizeof(T));
    return v;
}

int check_device(int idx, char* err, size_t err_len) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) {
        set_err(err, err_len, "no HIP device available (ptmi requires an MI355X / gfx950)");
        return PTMI_ERR_DEVICE;
    }
    if (idx < 0 || idx >= n) {
        set_err(err, err_len, "device index %d out of bounds: highest device index: %d", idx, n - 1);
        return PTMI_ERR_DEVICE;
    }
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, idx) != hipSuccess) {
        set_err(err, err_len, "hipGetDeviceProperties(%d) failed", idx);
        return PTMI_ERR_DEVICE;
    }
    if (std::strncmp(p.gcnArchName, "gfx950", 6) != 0) {
        set_err(err, err_len, "device %d is %s; libptmi is built for gfx950 only", idx, p.gcnArchName);
        return PTMI_ERR_DEVICE;
    }
    return PTMI_OK;
}

// Convert + validate the packed reference records (layout.py / tracer.cl:24-93).
// Zero-pattern predicates (exact zeros, +-0 included).
bool is_st_pattern(const double* m) {  // [a 0 0 d; 0 b 0 e; 0 0 c f; 0 0 0 g]
    static const int z[] = {1, 2, 4, 6, 8, 9, 12, 13, 14};
    for (int i : z)
        if (m[i] != 0.0) return false;
    return true;
}
bool is_diag3(const double* m) {  // rows 0-2 diagonal (row 3 unused)
    static const int z[] = {1, 2, 3, 4, 6, 7, 8, 9, 11};
    for (int i : z)
        if (m[i] != 0.0) return false;
    return true;
}

int convert_scene(const uint8_t* objects, uint32_t n_obj, const uint8_t* tris, uint32_t n_tri, const uint8_t* groups,
                  uint32_t n_grp, const uint8_t* camera, std::vector<DevObject>& objs, std::vector<int32_t>& roots,
                  std::vector<DevNode>& nodes, RootIndex& index, std::vector<RootRec>& root_rec,
                  std::vector<DevTriShade>& st, DevCamera& cam, int32_t run_end[5], char* err, size_t err_len) {
    if (!objects || n_obj == 0 || n_obj > PTMI_MAX_OBJECTS) {
        set_err(err, err_len, "need 1..%d objects (tracer.cl:846 __local object objects[16]), got %u",
                PTMI_MAX_OBJECTS, n_obj);
        return PTMI_ERR_ARG;
    }
    if (!camera || (n_tri && !tris) || (n_grp && !groups)) {
        set_err(err, err_len, "NULL record pointer");
        return PTMI_ERR_ARG;
    }
    cam.width = rd<int32_t>(camera + 0);
    cam.height = rd<int32_t>(camera + 4);
    cam.pixel_size = rd<double>(camera + 16);
    cam.half_width = rd<double>(camera + 24);
    cam.half_height = rd<double>(camera + 32);
    cam.aperture = rd<double>(camera + 40);
    cam.focal_length = rd<double>(camera + 48);
    std::memcpy(cam.inv, camera + 56, 128);
    for (int r = 0; r < 4; r++)  // mul (tracer.cl:369-376) of the point (0,0,0,1); no contraction (Makefile)
        cam.origin[r] = ((cam.inv[4 * r] * 0.0 + cam.inv[4 * r + 1] * 0.0) + cam.inv[4 * r + 2] * 0.0) +
                        cam.inv[4 * r + 3] * 1.0;
    if (cam.width <= 0 || cam.height <= 0 || (int64_t)cam.width * cam.height > (int64_t)1 << 30) {
        set_err(err, err_len, "bad camera size %dx%d", cam.width, cam.height);
        return PTMI_ERR_ARG;
    }
    std::vector<DevObject> all(n_obj);
    for (uint32_t i = 0; i < n_obj; i++) {
        const uint8_t* b = objects + (size_t)PTMI_OBJECT_BYTES * i;
        DevObject& o = all[i];
        std::memset(&o, 0, sizeof o);
        o.key = (int32_t)i;
        std::memcpy(o.inv, b + 128, 128);
        std::memcpy(o.inv_t, b + 256, 128);
        std::memcpy(o.color, b + 384, 32);
        std::memcpy(o.emission, b + 416, 32);
        o.refractive_index = rd<double>(b + 448);
        const int64_t type = rd<int64_t>(b + 456);
        o.type = (type >= 0 && type <= 4) ? (int32_t)type : 999;
        o.min_y = rd<double>(b + 464);
        o.max_y = rd<double>(b + 472);
        o.reflectivity = rd<double>(b + 480);
        std::memcpy(o.bb_min, b + 520, 32);
        o.st = is_st_pattern(o.inv) ? 1 : 0;
        o.invt_diag = is_diag3(o.inv_t) ? 1 : 0;
        std::memcpy(o.bb_max, b + 552, 32);
        o.tex = b[844] ? 1 : 0;  // isTextured, textureIndex, isTexturedNM, textureIndexNM (ocltracer.go:44-47)
        o.tex_index = b[845];
        o.tex_nm = b[846] ? 1 : 0;
        o.tex_index_nm = b[847];
        std::memcpy(o.tex_scale, b + 488, 32);  // textureScaleX, Y, XNM, YNM (ocltracer.go:36-39)
        o.child_count = 0;
        o.child_base = (int32_t)roots.size();
        if (o.type == 4) {
            const int32_t cc = rd<int32_t>(b + 584);
            if (cc < 0 || cc > 64) {
                set_err(err, err_len, "object %u: childCount %d out of range", i, cc);
                return PTMI_ERR_ARG;
            }
            for (int32_t c = 0; c < cc; c++) {
                const int32_t r = rd<int32_t>(b + 588 + 4 * c);
                if (r < 0 || (uint32_t)r >= n_grp) {
                    set_err(err, err_len, "object %u: child root %d outside %u groups", i, r, n_grp);
                    return PTMI_ERR_ARG;
                }
                roots.push_back(r);
            }
            o.child_count = cc;
        }
    }
    // Intersectable objects in type runs [planes | spheres | cylinders | cubes |
    // groups], list order inside a run.  Types > 4 and groups without BVH roots
    // can never record an intersection (tracer.cl:551-720) and are left out.
    objs.clear();
    for (int t = 0; t < 5; t++) {
        for (const DevObject& o : all)
            if (o.type == t && (t != 4 || o.child_count > 0)) objs.push_back(o);
        run_end[t] = (int32_t)objs.size();
    }
    nodes.resize(n_grp);
    std::vector<int32_t> tri_off(n_grp), tri_cnt(n_grp);
    for (uint32_t g = 0; g < n_grp; g++) {
        const uint8_t* b = groups + (size_t)PTMI_GROUP_BYTES * g;
        DevNode& n = nodes[g];
        std::memcpy(n.bb_min, b + 0, 24);
        std::memcpy(n.bb_max, b + 32, 24);
        tri_off[g] = rd<int32_t>(b + 128);
        tri_cnt[g] = rd<int32_t>(b + 132);
        n.child0 = rd<int32_t>(b + 140);
        n.child1 = rd<int32_t>(b + 144);
        if (tri_cnt[g] < 0 || tri_off[g] < 0 || (int64_t)tri_off[g] + tri_cnt[g] > (int64_t)n_tri ||
            n.child0 >= (int32_t)n_grp || n.child1 >= (int32_t)n_grp) {
            set_err(err, err_len, "group %u: triangle range [%d,+%d) / children (%d,%d) out of range", g,
                    tri_off[g], tri_cnt[g], n.child0, n.child1);
            return PTMI_ERR_ARG;
        }
    }
    // Children must follow their parent (BuildCLGroup preorder numbering): the
    // trees are then acyclic and every walk terminates.
    for (int32_t g = 0; g < (int32_t)n_grp; g++)
        if ((nodes[g].child0 > 0 && nodes[g].child0 <= g) || (nodes[g].child1 > 0 && nodes[g].child1 <= g)) {
            set_err(err, err_len, "group %d: child index not in preorder (BuildCLGroup numbering)", g);
            return PTMI_ERR_ARG;
        }
    st.resize(n_tri);
    for (uint32_t t = 0; t < n_tri; t++) {
        const uint8_t* b = tris + (size_t)PTMI_TRIANGLE_BYTES * t;
        std::memcpy(st[t].n1, b + 160, 32);
        std::memcpy(st[t].n2, b + 192, 32);
        std::memcpy(st[t].n3, b + 224, 32);
        std::memcpy(st[t].color, b + 256, 32);
    }
    // Per group object: one traversal index over all its roots' triangles
    // (ptmi_bvh.cpp); the object then refers to its RootRec (child_count 1).
    index = RootIndex{};
    root_rec.clear();
    for (DevObject& o : objs) {
        if (o.type != 4) continue;
        RootRec rec;
        const int rc = build_object_index(tris, nodes, tri_off, tri_cnt, roots.data() + o.child_base, o.child_count,
                                          o.bb_min, o.bb_max, index, &rec, err, err_len);
        if (rc) return rc;
        o.child_base = (int32_t)root_rec.size();
        o.child_count = 1;
        root_rec.push_back(rec);
    }
    return PTMI_OK;
}

template <typename T>
int upload(const std::vector<T>& v, void** dst, char* err, size_t err_len) {
    const size_t bytes = std::max<size_t>(v.size() * sizeof(T), 256);
    HIP_TRY(hipMalloc(dst, bytes));
    if (!v.empty()) HIP_TRY(hipMemcpy(*dst, v.data(), v.size() * sizeof(T), hipMemcpyHostToDevice));
    return PTMI_OK;
}


// A scene converted on the host once (records validated and split into the device
// layouts, traversal indices built, kernel flags chosen), uploadable to any device.
struct HostScene {
    std::vector<DevObject> objs;
    std::vector<int32_t> roots;
    std::vector<DevNode> nodes;
    RootIndex index;
    std::vector<RootRec> root_rec;
    std::vector<DevTriShade> st;
    std::vector<PlaneRec> planes;
    std::vector<SphereRec> spheres;
    DevCamera cam{};
    int32_t run_end[5] = {};
    int flags = 0;
    int32_t leaf_bit = kLeafNarrow;  // Node4 child code format (finalize_index_codes)
    uint32_t n_list = 0, n_grp = 0, n_tri = 0;
    int32_t n_planes_y = 0;
};

int prepare_scene(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri, const void* groups,
                  uint32_t n_grp, const void* camera, const ptmi_textures* textures, HostScene& hs, char* err,
                  size_t err_len) {
    int rc = convert_scene((const uint8_t*)objects, n_obj, (const uint8_t*)triangles, n_tri, (const uint8_t*)groups,
                           n_grp, (const uint8_t*)camera, hs.objs, hs.roots, hs.nodes, hs.index, hs.root_rec, hs.st,
                           hs.cam, hs.run_end, err, err_len);
    if (rc) return rc;
    hs.leaf_bit = finalize_index_codes(hs.index, hs.root_rec);
    const DevCamera& cam = hs.cam;
    int flags = 0;
    for (const DevObject& o : hs.objs) {
        if (o.type == 4) flags |= 1;                                    // F_GROUPS
        if (o.type == 2 || o.type == 3) flags |= 2;                     // F_CYLCUBE
        if (o.reflectivity != 0.0 || o.refractive_index != 1.0) flags |= 4;  // F_MATERIALS
    }
    if (cam.aperture != 0) flags |= 8;                                  // F_DOF
    // Affine scene (ptmi_kernels.hip dotv): every inverse ends in (+-0, +-0, +-0, 1),
    // inverse transposes have +-0 in column 3 of rows 0-2, triangle normals have a
    // finite w.  Otherwise F_PROJ: the generic instantiation with the w lanes.
    bool affine = cam.inv[12] == 0.0 && cam.inv[13] == 0.0 && cam.inv[14] == 0.0 && cam.inv[15] == 1.0;
    for (const DevObject& o : hs.objs)
        affine = affine && o.inv[12] == 0.0 && o.inv[13] == 0.0 && o.inv[14] == 0.0 && o.inv[15] == 1.0 &&
                 o.inv_t[3] == 0.0 && o.inv_t[7] == 0.0 && o.inv_t[11] == 0.0;
    for (const DevTriShade& t : hs.st)
        affine = affine && std::isfinite(t.n1[3]) && std::isfinite(t.n2[3]) && std::isfinite(t.n3[3]);
    // The affine instantiations also use the compiler's divide / sqrt cores for sphere
    // roots (ptmi_kernels.hip div_core), which needs 2a = 2|M d|^2
    // far above the denormal range for every unit-scale ray direction d: each sphere's
    // inverse has linear-part entries <= 2^64 and |det| >= 2^-64, so its smallest singular
    // value is >= 2^-196.  Scenes outside that take the generic instantiation.
    // The same bound on the camera inverse keeps |pixel - origin| >= 2^-196 for its
    // normalize's core, and on sphere inverses (through their transposes) keeps sphere
    // normals >= 2^-196 long.
    auto tame = [](const double* m) {
        double mx = 0.0;
        for (int r = 0; r < 3; r++)
            for (int c = 0; c < 3; c++) mx = std::max(mx, std::fabs(m[4 * r + c]));
        const double det = m[0] * (m[5] * m[10] - m[6] * m[9]) - m[1] * (m[4] * m[10] - m[6] * m[8]) +
                           m[2] * (m[4] * m[9] - m[5] * m[8]);
        return mx <= 0x1p64 && std::fabs(det) >= 0x1p-64;
    };
    affine = affine && tame(cam.inv);
    for (const DevObject& o : hs.objs)
        if (o.type == 1) affine = affine && tame(o.inv);
    if (!affine) flags |= 16;                                           // F_PROJ
    // Child codes past 16 bits (>= 2^15 Node4s or triangles): a traversal stack of 32-bit
    // entries -- the affine F_WIDE instantiation (ptmi_kernels.hip trace_groups), or the
    // generic one for non-affine scenes (round 5 sent every such scene to the generic one).
    const int wide = hs.leaf_bit != kLeafNarrow ? 256 : 0;              // F_WIDE
    // Textured plane/sphere/cube colours or plane normal maps: the one textured
    // instantiation (generic arithmetic + software sampler, tracer.cl:907-914, 1077-1092).
    for (const DevObject& o : hs.objs)
        if ((o.tex && (o.type == 0 || o.type == 1 || o.type == 3)) || (o.tex_nm && o.type == 0)) flags = 63;
    const int forced = g_force_flags.load();  // ptmi_diag_force_flags (tests): one load
    if (forced >= 0) flags = forced & 63;
    flags |= wide;  // (never a 16-bit stack for 31-bit codes: F_PROJ and F_TEX kernels have 32-bit ones)
    if (textures) {
        for (int k = 0; k < 3; k++) {
            const uint64_t texels = (uint64_t)textures->width[k] * textures->height[k] * textures->count[k];
            if (textures->count[k] &&
                (!textures->pixels[k] || textures->width[k] == 0 || textures->height[k] == 0 ||
                 textures->width[k] > (1u << 16) || textures->height[k] > (1u << 16) || textures->count[k] > 256 ||
                 texels > ((uint64_t)1 << 32))) {
                set_err(err, err_len, "texture array %d: bad size %ux%u x %u layers (or NULL pixels)", k,
                        textures->width[k], textures->height[k], textures->count[k]);
                return PTMI_ERR_ARG;
            }
        }
    }
    hs.flags = flags;
    // compact plane / scale+translate sphere records (ptmi_device.h)
    for (size_t k = 0; k < hs.objs.size(); k++) {
        const DevObject& o = hs.objs[k];
        if (o.type == 0) {
            PlaneRec r{};
            std::memcpy(r.row1, o.inv + 4, 32);
            r.slot = (int32_t)k;
            r.key = o.key;
            r.nz = (r.row1[0] != 0.0 ? 1 : 0) | (r.row1[1] != 0.0 ? 2 : 0) | (r.row1[2] != 0.0 ? 4 : 0);
            hs.planes.push_back(r);
        } else if (o.type == 1 && o.st) {
            SphereRec r{};
            r.m0 = o.inv[0];
            r.m3 = o.inv[3];
            r.m5 = o.inv[5];
            r.m7 = o.inv[7];
            r.m10 = o.inv[10];
            r.m11 = o.inv[11];
            r.m15 = o.inv[15];
            r.slot = (int32_t)k;
            r.key = o.key;
            hs.spheres.push_back(r);
        }
    }
    // The leading planes (list order kept) whose row 1 has +-0 x and z entries, and the
    // parallel pairs (identical row1[0..2]) as the affine plane loops pair the planes:
    // (0,1), (2,3), ... below n_planes_y, then on from there (find_closest_prims).
    {
        const int np = (int)hs.planes.size();
        int npy = 0;
        while (npy < np && hs.planes[npy].row1[0] == 0.0 && hs.planes[npy].row1[2] == 0.0) npy++;
        hs.n_planes_y = npy;
        auto same = [&](int a, int b) { return std::memcmp(hs.planes[a].row1, hs.planes[b].row1, 24) == 0; };
        int p = 0;
        for (; p + 1 < npy; p += 2) hs.planes[p].par = same(p, p + 1);
        for (; p + 1 < np; p += 2) hs.planes[p].par = same(p, p + 1);
    }
    hs.n_list = n_obj;
    hs.n_grp = n_grp;
    hs.n_tri = n_tri;
    return PTMI_OK;
}

// Device-wide resident tile waves of the scene's trace_kernel instantiation (its work
// plan is sized by them, ptmi_scene_render).
hipError_t resident_waves(ptmi_scene* s) {
    hipDeviceProp_t p;
    hipError_t e = hipGetDeviceProperties(&p, s->device);
    if (e != hipSuccess) return e;
    const int flags = s->flags | (s->rng == PTMI_RNG_XOSHIRO ? 64 : 0);  // F_XRNG
    s->resident_waves = p.multiProcessorCount * 16;
    int blocks_per_cu = 0;
    if (hipOccupancyMaxActiveBlocksPerMultiprocessor(&blocks_per_cu, trace_kernel_symbol(flags),
                                                     trace_block_threads(flags), 0) == hipSuccess &&
        blocks_per_cu > 0)
        s->resident_waves = p.multiProcessorCount * blocks_per_cu * trace_tiles_per_block(flags);
    return hipSuccess;
}

// Mesh scenes: a cost class per 8x8 tile for the dispatch order of the chunked tiles --
// how many of 9 primary rays (a 3x3 grid of pixel centres) pass the conservative hull
// cull of some group object (group_needs_walk without the primitives' best).  Tiles whose
// camera rays reach a mesh walk on every bounce; their chunks are the long items of a
// launch (C4 at 2048 spp: 20 ms on average, up to 82 ms), and in raster order the last
// round of chunks ends on them (a 43 ms drain, 6 % of the slot-time; tools/timeline.py).
// Dispatching them first within each chunk round leaves short items for the end.  Only the
// order of work items changes, never a pixel's sums or their order.  Plain host doubles: a
// heuristic, not an exactness argument.
constexpr uint8_t kCostUnset = 0xFF;

// The mesh kernels' walk batch for a scene (DevScene::walk_batch): larger meshes have longer walks
// (gopher: 9.8 Node4 visits and 5.3 triangle tests per walk against the teapot's 6.7 and 2.3), so
// a walk phase is worth more parked lanes.  Scenes without meshes never walk.
static int32_t walk_batch_for(const HostScene& hs) {
    if (!(hs.flags & 1)) return 64;
    return hs.n_tri >= 12000 ? 32 : 28;
}

TileCostInput tile_cost_input(const HostScene& hs) {
    TileCostInput in;
    in.cam = hs.cam;
    for (int j = hs.run_end[3]; j < hs.run_end[4]; j++) {
        const DevObject& ob = hs.objs[j];
        TileCostInput::Obj o;
        std::memcpy(o.inv, ob.inv, sizeof(o.inv));
        for (int ci = 0; ci < ob.child_count; ci++) {
            const RootRec& R = hs.root_rec[ob.child_base + ci];
            o.hulls.push_back({R.hull_mn[0], R.hull_mn[1], R.hull_mn[2], R.hull_mx[0], R.hull_mx[1], R.hull_mx[2]});
        }
        in.objs.push_back(std::move(o));
    }
    return in;
}

// The class of tile t (raster index).
uint8_t mesh_tile_class(const TileCostInput& in, const std::vector<std::array<double, 3>>& org, int t) {
    const DevCamera& c = in.cam;
    const int tx = (c.width + 7) / 8;
    const double* m = c.inv;
    int hits = 0;
    for (int q = 0; q < 9; q++) {
        const double x = (t % tx) * 8 + 1 + 3 * (q % 3) + 0.5, y = (t / tx) * 8 + 1 + 3 * (q / 3) + 0.5;
        const double a = c.half_width - c.pixel_size * x, b = c.half_height - c.pixel_size * y;
        double d[3];
        for (int r = 0; r < 3; r++) d[r] = m[4 * r] * a + m[4 * r + 1] * b - m[4 * r + 2] + m[4 * r + 3] - c.origin[r];
        bool hit = false;
        for (size_t j = 0; j < in.objs.size() && !hit; j++) {
            const TileCostInput::Obj& ob = in.objs[j];
            double inv_d[3];
            for (int r = 0; r < 3; r++) {
                const double* mi = ob.inv + 4 * r;
                inv_d[r] = 1.0 / (mi[0] * d[0] + mi[1] * d[1] + mi[2] * d[2]);
            }
            for (const auto& H : ob.hulls) {
                double tn = 0.0, tf = INFINITY;
                for (int r = 0; r < 3; r++) {
                    const double t0 = (H[r] - org[j][r]) * inv_d[r], t1 = (H[3 + r] - org[j][r]) * inv_d[r];
                    tn = std::max(tn, std::min(t0, t1));
                    tf = std::min(tf, std::max(t0, t1));
                }
                if (tn <= tf) {  // NaN slabs (ray in a hull face plane) count as misses: a heuristic
                    hit = true;
                    break;
                }
            }
        }
        hits += hit ? 1 : 0;
    }
    return (uint8_t)hits;
}

// Classes of the tiles owned(0), owned(1), ... owned(n - 1) not computed yet, into cost
// (sized to the frame's tiles, kCostUnset where unknown).  The camera origin in each group
// object's space is computed once per call, not per ray.
template <typename Owned>
void mesh_tile_cost(const TileCostInput& in, std::vector<uint8_t>& cost, uint32_t n, Owned owned) {
    const DevCamera& c = in.cam;
    const size_t tiles = (size_t)((c.width + 7) / 8) * ((c.height + 7) / 8);
    if (cost.size() != tiles) cost.assign(tiles, kCostUnset);
    std::vector<std::array<double, 3>> org(in.objs.size());
    for (size_t j = 0; j < in.objs.size(); j++)
        for (int r = 0; r < 3; r++) {
            const double* mi = in.objs[j].inv + 4 * r;
            org[j][r] = mi[0] * c.origin[0] + mi[1] * c.origin[1] + mi[2] * c.origin[2] + mi[3];
        }
    for (uint32_t k = 0; k < n; k++) {
        const uint32_t t = owned(k);
        if (cost[t] == kCostUnset) cost[t] = mesh_tile_class(in, org, (int)t);
    }
}

int upload_scene(const HostScene& hs, int device_index, const ptmi_textures* textures, ptmi_scene** out, char* err,
                 size_t err_len) {
    HIP_TRY(hipSetDevice(device_index));
    ptmi_scene* s = new ptmi_scene();
    s->flags = hs.flags;
    s->device = device_index;
    s->width = (uint32_t)hs.cam.width;
    s->height = (uint32_t)hs.cam.height;
    int rc;
    if ((rc = upload(hs.objs, &s->buffers[0], err, err_len)) || (rc = upload(hs.roots, &s->buffers[1], err, err_len)) ||
        (rc = upload(hs.nodes, &s->buffers[2], err, err_len)) ||
        (rc = upload(hs.index.tris, &s->buffers[3], err, err_len)) || (rc = upload(hs.st, &s->buffers[4], err, err_len)) ||
        (rc = upload(hs.planes, &s->buffers[5], err, err_len)) ||
        (rc = upload(hs.spheres, &s->buffers[6], err, err_len)) ||
        (rc = upload(hs.index.nodes, &s->buffers[7], err, err_len)) ||
        (rc = upload(hs.index.chain_boxes, &s->buffers[8], err, err_len)) ||
        (rc = upload(hs.root_rec, &s->buffers[9], err, err_len))) {
        ptmi_scene_destroy(s);
        return rc;
    }
    for (int k = 0; k < 3; k++) {  // texture arrays (prepareTextures, ocltracer.go:228-254)
        DevTexArray& T = s->dev.tex[k];
        T = DevTexArray{};
        if (!textures || textures->count[k] == 0) continue;  // the all-zero fake image
        const size_t bytes = (size_t)textures->width[k] * textures->height[k] * textures->count[k] * 4;
        hipError_t e = hipMalloc(&s->buffers[10 + k], bytes);
        if (e == hipSuccess) e = hipMemcpy(s->buffers[10 + k], textures->pixels[k], bytes, hipMemcpyHostToDevice);
        if (e != hipSuccess) {
            set_err(err, err_len, "texture array %d upload (%zu B): %s", k, bytes, hipGetErrorString(e));
            ptmi_scene_destroy(s);
            return PTMI_ERR_HIP;
        }
        T.texels = (const uint32_t*)s->buffers[10 + k];
        T.w = (int32_t)textures->width[k];
        T.h = (int32_t)textures->height[k];
        T.layers = (int32_t)textures->count[k];
    }
    s->dev.objs = (const DevObject*)s->buffers[0];
    for (int t = 0; t < 5; t++) s->dev.run_end[t] = hs.run_end[t];
    s->dev.planes = (const PlaneRec*)s->buffers[5];
    s->dev.n_planes = (int32_t)hs.planes.size();
    s->dev.n_planes_y = hs.n_planes_y;
    s->dev.spheres = (const SphereRec*)s->buffers[6];
    s->dev.n_spheres_st = (int32_t)hs.spheres.size();
    // HIP failures from here on release the half-built scene.
#define SCENE_TRY(call)                                                                            \
    do {                                                                                           \
        hipError_t e_ = (call);                                                                    \
        if (e_ != hipSuccess) {                                                                    \
            set_err(err, err_len, "%s failed: %s (%s:%d)", #call, hipGetErrorString(e_), __FILE__, \
                    __LINE__);                                                                     \
            ptmi_scene_destroy(s);                                                                 \
            return PTMI_ERR_HIP;                                                                   \
        }                                                                                          \
    } while (0)
    if (!hs.objs.empty()) {
        SCENE_TRY(launch_plane_normals((DevObject*)s->buffers[0], (int)hs.objs.size(), nullptr));
        SCENE_TRY(hipDeviceSynchronize());
    }
    {  // randomVectorInHemisphere table (ptmi_kernels.hip hemi_table_kernel) + its check counter
        const size_t tab = (size_t)65536 * 4 * sizeof(double);
        SCENE_TRY(hipMalloc(&s->buffers[13], tab + 256));
        int* mismatch = (int*)((char*)s->buffers[13] + tab);
        SCENE_TRY(hipMemset(mismatch, 0, sizeof(int)));
        SCENE_TRY(launch_hemi_table((double*)s->buffers[13], mismatch, nullptr));
        // Only the affine instantiations read the table (ptmi_kernels.hip bounce_shade), and
        // its records are the affine sequences' own results, so a record where the generic
        // (full-operator) sequences give other bits -- a toolchain or ocml change -- affects
        // no image: it is counted and reported, not a scene failure.
        SCENE_TRY(hipMemcpy(&s->hemi_mismatch, mismatch, sizeof(int), hipMemcpyDeviceToHost));
        // (ptmi_diag_hemi_mismatch returns the count; tests/test_gpu_rng.py expects 0.)
        if (s->hemi_mismatch && getenv("PTMI_VERBOSE"))
            fprintf(stderr, "ptmi: hemisphere table: %d records where the affine and generic sequences differ "
                            "(generic instantiations compute, they never read the table)\n", s->hemi_mismatch);
        s->dev.hemi = (const double*)s->buffers[13];
    }
    s->dev.roots = (const int32_t*)s->buffers[1];
    s->dev.nodes = (const DevNode*)s->buffers[2];
    s->dev.tris = (const DevTri*)s->buffers[3];
    s->dev.tri_shade = (const DevTriShade*)s->buffers[4];
    s->dev.nodes4 = (const Node4*)s->buffers[7];
    s->dev.chains = (const ChainBox*)s->buffers[8];
    s->dev.root_rec = (const RootRec*)s->buffers[9];
    s->dev.n_obj = (uint32_t)hs.objs.size();
    s->dev.n_list = hs.n_list;
    s->dev.n_nodes = hs.n_grp;
    s->dev.n_nodes4 = (int32_t)hs.index.nodes.size();
    s->dev.leaf_bit = hs.leaf_bit;
    // Walk batch of the mesh kernels (parked lanes that start a wave's walk phase; ptmi_kernels.hip
    // trace_groups / trace_groups_pool): a walk phase lasts as long as its longest walk, so the
    // batch trades the parked lanes' waiting against the phases' idle lanes.  Round 6, with the
    // path pool (2048 spp, one MI355X, profiles/r6/tune): teapot (C4) 24 / 28 / 32 -> 490.5 / 489.4 /
    // 493.6 ms, gopher (C5) 784.2 / 768.2 / 759.6 ms.
    s->dev.walk_batch = walk_batch_for(hs);
    // The hemisphere table in the mesh kernels: the 1-MB (sin, cos) plane shares each XCD's 4-MB L2
    // with the traversal index.  Round 6, with the path pool, on the gopher (C5, index ~3.7 MB) the
    // table costs HBM traffic -- 2.1-2.25 GB per launch with it, 0.76 GB without (profiles/r6/hbm1):
    // its lines are evicted and refetched -- but it still saves time: 753.3 / 754.2 / 755.2 ms with,
    // 766.7 / 767.7 / 768.3 ms without, alternated on one box (profiles/r6/hm2); the teapot (C4)
    // 488.5-490.0 with, 503.1 ms without.  At ~3 GB/s the traffic binds nothing, so every mesh scene
    // reads the table; PTMI_KNOB_HEMI_MESH 0 trades the 1.7 % for the traffic.
    s->dev.hemi_mesh = 1;
    // (Tests and tuning studies change the plan through ptmi_diag_set_knob; the library reads
    // no tuning variable from the environment.)
    // Mesh scenes: >= 64 samples per chunk.  It binds only on short sample ranges (a rank's
    // share): the C4 8-rank shares (256 samples) take 81.3 ms on average with 4 chunks of 64
    // against 85.4 ms with 7 of 37 (the items' start-up and end-of-item idle lanes), 93.5 ms
    // with 2 of 128 (a coarser drain); the C5 tile-split shares are flat (profiles/r4/shards).
    if (hs.flags & 1) s->min_chunk = 64;
    if (hs.flags & 1) s->tc_in = tile_cost_input(hs);  // tile classes: on the first ordered render
    s->dev.n_tri = hs.n_tri;
    s->dev.cam = hs.cam;
    {  // the camera record in device memory (ptmi_kernels.hip camera_ptr)
        SCENE_TRY(hipMalloc(&s->buffers[14], sizeof(DevCamera)));
        SCENE_TRY(hipMemcpy(s->buffers[14], &hs.cam, sizeof(DevCamera), hipMemcpyHostToDevice));
        s->dev.camg = (const DevCamera*)s->buffers[14];
    }
    SCENE_TRY(resident_waves(s));
#undef SCENE_TRY
    *out = s;
    return PTMI_OK;
}


#if PTMI_STUDY
// Split execution of an affine mesh scene (ptmi_kernels.hip trace_split_kernel): pixel-chunks
// of chunk_len samples over every owned tile, traced pass by pass by a pool of L path slots
// (L = the tracer's resident lanes x split_per_lane), each pass followed by the walks it
// asked for, until a pass asks for none.  Chunk records go to `part` in the WorkPlan's
// chunk-major layout (store_sums' records), summed by reduce_chunks_kernel as for the
// one-kernel form's chunk items.
int render_split(ptmi_scene* s, uint32_t samples, const WorkPlan& wp, const double* seeds, double* sums,
                 hipStream_t st, char* err, size_t err_len) {
    const int flags = s->flags;
    hipDeviceProp_t p;
    HIP_TRY(hipGetDeviceProperties(&p, s->device));
    int per_cu = 0, walk_cu = 0;
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, trace_split_symbol(flags), 64, 0));
    HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&walk_cu, walk_split_symbol(), 64, 0));
    const uint32_t waves = (uint32_t)std::max(1, per_cu) * (uint32_t)p.multiProcessorCount;
    const uint32_t walk_grid = (uint32_t)std::max(1, walk_cu) * (uint32_t)p.multiProcessorCount;
    const uint32_t per_wave = 64u * s->split_per_lane;
    const uint64_t n_items64 = (uint64_t)wp.n_tail * 64u * wp.nchunks;
    if (n_items64 >= 0xFFFFFFF0ull) {
        set_err(err, err_len, "split render: %llu pixel-chunks exceed 32-bit ids", (unsigned long long)n_items64);
        return PTMI_ERR_UNSUPPORTED;
    }
    const uint32_t n_items = (uint32_t)n_items64;
    // Slots: the tracer's resident waves x per_wave, but no more than there are pixel-chunks.
    uint32_t L = waves * per_wave;
    L = std::max<uint32_t>(64, std::min<uint32_t>(L, (n_items + 63) / 64 * 64));
    const uint32_t n_waves = (L + per_wave - 1) / per_wave;
    const size_t need = (size_t)L * (kSlotBytes + 4) + (size_t)n_waves * 12 + 512;
    if (need > s->split_bytes) {
        if (s->split_mem) {
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipFree(s->split_mem));
            s->split_mem = nullptr;
            s->split_bytes = 0;
        }
        HIP_TRY(hipMalloc(&s->split_mem, need));
        s->split_bytes = need;
    }
    if (!s->split_host) HIP_TRY(hipHostMalloc((void**)&s->split_host, 64, hipHostMallocDefault));
    char* m = (char*)s->split_mem;
    SplitBufs& B = s->sb;
    B.rec = m;
    m += (size_t)L * kSlotBytes;
    B.req = (uint32_t*)m;
    m += (size_t)L * 4;
    B.seg = (uint32_t*)m;
    m += (size_t)n_waves * 4;
    B.wcl = (uint32_t*)m;
    m += (size_t)n_waves * 8;
    B.cnt = (uint32_t*)m;
    B.L = L;
    B.per_wave = per_wave;
    B.n_items = n_items;
    B.budget = s->split_budget;
    HIP_TRY(hipMemset2DAsync(B.rec + offsetof(SplitRec, u), kSlotBytes, 0xFF, 4, L, st));  // every slot kSlotFree
    HIP_TRY(hipMemsetAsync(B.cnt, 0, 16, st));
    HIP_TRY(hipMemsetAsync(B.wcl, 0, (size_t)n_waves * 8, st));  // no block claimed yet
    // A bound no render reaches: every pass finishes or advances at least one pixel-chunk
    // by a bounce, so a runaway loop means a bug; fail instead of spinning.
    const uint64_t max_passes = ((uint64_t)n_items / L + 1) * 11ull * wp.chunk_len + 1024;
    uint32_t pass = 0;
    for (;;) {
        HIP_TRY(hipMemsetAsync(B.cnt, 0, 4, st));  // this pass's request count
        HIP_TRY(hipMemsetAsync(B.cnt + 2, 0, 4, st));  // and yield count
        HIP_TRY(launch_split_pass(s->dev, flags, samples, wp, B, seeds, s->sunf, s->partial, walk_grid, st));
        pass++;
        if (pass % s->split_sync == 0) {
            HIP_TRY(hipMemcpyAsync(s->split_host, B.cnt, 12, hipMemcpyDeviceToHost, st));
            HIP_TRY(hipStreamSynchronize(st));
            if (s->split_host[0] == 0 && s->split_host[2] == 0 && s->split_host[1] >= n_items) break;
        }
        if (pass > max_passes) {
            set_err(err, err_len, "split render did not finish in %u passes", pass);
            return PTMI_ERR_HIP;
        }
    }
    s->split_passes = pass;
    if (getenv("PTMI_SPLIT_DEBUG")) {  // (study build) slot states after the last pass
        std::vector<uint32_t> it(L);
        HIP_TRY(hipMemcpy2D(it.data(), 4, B.rec + offsetof(SplitRec, u), kSlotBytes, 4, L, hipMemcpyDeviceToHost));
        uint32_t cnt[4];
        HIP_TRY(hipMemcpy(cnt, B.cnt, 16, hipMemcpyDeviceToHost));
        size_t fr = 0, dead = 0, busy = 0;
        for (uint32_t v : it) (v == kSlotFree ? fr : v == kSlotDead ? dead : busy)++;
        fprintf(stderr, "split: L %u items %u passes %u walk_grid %u per_cu %d: free %zu dead %zu busy %zu req %u claims %u walks %u\n",
                L, n_items, pass, walk_grid, per_cu, fr, dead, busy, cnt[0], cnt[1], cnt[3]);
    }
    (void)sums;
    return PTMI_OK;
}
#endif  // PTMI_STUDY

}  // namespace

extern "C" {

int ptmi_device_count(void) {
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess) return 0;
    return n;
}

int ptmi_device_name(int device_index, char* buf, size_t len) {
    hipDeviceProp_t p;
    if (hipGetDeviceProperties(&p, device_index) != hipSuccess) return PTMI_ERR_DEVICE;
    if (buf && len) snprintf(buf, len, "%s (%s, %d CUs)", p.name, p.gcnArchName, p.multiProcessorCount);
    return PTMI_OK;
}

const char* ptmi_build_info(void) {
    return "ptmi abi=1 arch=gfx950 fp=fp64 contract=off kernels=trace_kernel<F>,reduce_chunks_kernel,finalize_kernel";
}

int ptmi_index_stats(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri, const void* groups,
                     uint32_t n_grp, const void* camera, double* out, int n_out, char* err, size_t err_len) {
    if (!out || n_out <= 0) {
        set_err(err, err_len, "out == NULL");
        return PTMI_ERR_ARG;
    }
    HostScene hs;
    int rc = prepare_scene(objects, n_obj, triangles, n_tri, groups, n_grp, camera, nullptr, hs, err, err_len);
    if (rc) return rc;
    double st[8] = {(double)hs.index.nodes.size(), 0.0, 0.0, 0.0, 0.0, (double)hs.root_rec.size(), 0.0,
                    (double)hs.leaf_bit};
    for (const RootRec& R : hs.root_rec) {
        st[4] = std::max(st[4], std::log2((double)R.sc));
        std::vector<std::pair<int32_t, int>> todo;  // (Node4, its level)
        const int32_t lb = hs.leaf_bit, empty = lb | ((int32_t)hs.index.tris.size() - 1);  // the sentinel leaf
        if (R.entry < lb) todo.push_back({R.entry, 1});
        while (!todo.empty()) {  // the root's Node4s (children >= 0 are Node4 indices)
            const auto [ni, lv] = todo.back();
            const Node4& nd = hs.index.nodes[ni];
            todo.pop_back();
            st[6] = std::max(st[6], (double)lv);
            for (int i = 0; i < 4; i++) {
                if (nd.child[i] == empty) continue;
                if (nd.child[i] < lb) todo.push_back({nd.child[i], lv + 1});
                double e[3];
                for (int k = 0; k < 3; k++) {
                    const double lo = f16_value(nd.bnd[k][0][i]), hi = f16_value(nd.bnd[k][1][i]);
                    st[3] += (std::isinf(lo) ? 1 : 0) + (std::isinf(hi) ? 1 : 0);
                    e[k] = (hi - lo) * R.sc;
                }
                st[1] += 1.0;
                st[2] += 2.0 * (e[0] * e[1] + e[1] * e[2] + e[2] * e[0]);
            }
        }
    }
    for (int i = 0; i < n_out && i < 8; i++) out[i] = st[i];
    return PTMI_OK;
}

int ptmi_scene_create(int device_index, const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                      const void* groups, uint32_t n_grp, const void* camera, ptmi_scene** out, char* err,
                      size_t err_len) {
    return ptmi_scene_create_textured(device_index, objects, n_obj, triangles, n_tri, groups, n_grp, camera, nullptr,
                                      out, err, err_len);
}

int ptmi_scene_create_textured(int device_index, const void* objects, uint32_t n_obj, const void* triangles,
                               uint32_t n_tri, const void* groups, uint32_t n_grp, const void* camera,
                               const ptmi_textures* textures, ptmi_scene** out, char* err, size_t err_len) {
    if (!out) {
        set_err(err, err_len, "out == NULL");
        return PTMI_ERR_ARG;
    }
    *out = nullptr;
    if (device_index < 0) device_index = 0;  // ocltracer.go:138-140
    int rc = check_device(device_index, err, err_len);
    if (rc) return rc;
    HostScene hs;
    if ((rc = prepare_scene(objects, n_obj, triangles, n_tri, groups, n_grp, camera, textures, hs, err, err_len)))
        return rc;
    return upload_scene(hs, device_index, textures, out, err, err_len);
}

void ptmi_scene_destroy(ptmi_scene* s) {
    if (!s) return;
    (void)hipSetDevice(s->device);
    for (void* b : s->buffers)
        if (b) (void)hipFree(b);
    if (s->partial) (void)hipFree(s->partial);
    if (s->sunf) (void)hipFree(s->sunf);
#if PTMI_STUDY
    if (s->split_mem) (void)hipFree(s->split_mem);
    if (s->split_host) (void)hipHostFree(s->split_host);
#endif
    if (s->order_dev) (void)hipFree(s->order_dev);
    if (s->tlist_dev) (void)hipFree(s->tlist_dev);
    if (s->item_ctr) (void)hipFree(s->item_ctr);
    if (s->cost_dev) (void)hipFree(s->cost_dev);
    for (auto& e : s->events) {
        (void)hipEventDestroy(e.first);
        (void)hipEventDestroy(e.second);
    }
    for (auto e : s->spare) (void)hipEventDestroy(e);
    delete s;
}

int ptmi_scene_size(const ptmi_scene* s, uint32_t* w, uint32_t* h) {
    if (!s) return PTMI_ERR_ARG;
    if (w) *w = s->width;
    if (h) *h = s->height;
    return PTMI_OK;
}

// Tile ownership of a tile-split render (ptmi_scene_render): diagonal for affine narrow-code
// mesh scenes in parity mode whose tile rows divide by the stride (the F_TLIST instantiations),
// raster striding otherwise.  Exported as ptmi_diag_tile_ownership, so callers that mask shards
// use the library's own decision (ptmi/dist.py had restated it).
static bool diagonal_tiles(const ptmi_scene* s, uint32_t tile_stride) {
    const int kflags0 = s->flags | (s->rng == PTMI_RNG_XOSHIRO ? 64 : 0);
    const uint32_t tiles_x = (s->width + kTile - 1) / kTile;
#if PTMI_STUDY
    if (s->split) return false;
#endif
    return tile_stride > 1 && tile_list_supported(kflags0) && tiles_x % tile_stride == 0;
}

int ptmi_scene_render(ptmi_scene* s, uint32_t samples, uint32_t sample_begin, uint32_t sample_end,
                      uint32_t tile_stride, uint32_t tile_offset, const double* seeds_dev, double* sums_dev,
                      uint32_t chunks, void* hip_stream, char* err, size_t err_len) {
    if (!s || !seeds_dev || !sums_dev || samples == 0 || sample_begin > sample_end || sample_end > samples ||
        tile_stride == 0 || tile_offset >= tile_stride) {
        set_err(err, err_len, "bad render arguments (samples %u range [%u,%u) tiles %u/%u)", samples, sample_begin,
                sample_end, tile_offset, tile_stride);
        return PTMI_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)hip_stream;
    const uint32_t W = s->width, H = s->height, npix = W * H;
    const uint32_t range = sample_end - sample_begin;
    const uint32_t tiles_x = (W + kTile - 1) / kTile, tiles = tiles_x * ((H + kTile - 1) / kTile);
    const int kflags0 = s->flags | (s->rng == PTMI_RNG_XOSHIRO ? 64 : 0);
    // Tile ownership of a tile-split launch.  Raster: tiles offset, offset + stride, ...; with
    // 160 tiles per row (1280 px) and stride 8 that gives every rank the same tile columns in
    // every row -- vertical stripes, which split a mesh unevenly (C5 8 ranks: max/mean 1.05).
    // Affine mesh scenes whose tile rows divide by the stride take the diagonal instead --
    // tile (x, y) belongs to rank (x + y) mod stride, each row holding tiles_x / stride of a
    // rank's tiles -- through the F_TLIST instantiations (WorkPlan::tiles), so the one-GPU
    // kernels are untouched (profiles/r5/tile_skew).  Every pixel's sums are the same either way.
    const bool tlist = diagonal_tiles(s, tile_stride);
    const uint32_t per_row = tiles_x / tile_stride;
    auto owned_tile = [&](uint32_t k) -> uint32_t {
        if (!tlist) return tile_offset + k * tile_stride;
        const uint32_t ty = k / per_row, j = k - ty * per_row;
        return ty * tiles_x + (tile_offset + tile_stride - ty % tile_stride) % tile_stride + j * tile_stride;
    };
    const uint32_t owned_tiles = tlist ? tiles / tile_stride : (tiles + tile_stride - 1 - tile_offset) / tile_stride;
    // Work items (WorkPlan, ptmi_device.h).  Automatic (chunks == 0), scenes without
    // meshes: whole tiles first, then the last ~0.5 resident waves' worth of tiles
    // split into sample chunks, so that short items fill the end of the launch (~6 per
    // resident wave slot, >= 32 samples each).  A whole-tile item pays its start-up
    // and the spread of its lanes' path lengths once for the whole range, and sums in
    // sample order without a partial buffer.  C2 (2048 spp, 4096 resident waves): 185.3 ms
    // with every tile chunked; 181.6 / 178.2 / 177.5 / 176.8 / 182.5 ms with 9000 / 4096 /
    // 3072 / 2048 / 1024 chunked tail tiles.
    // Round 3: ~6 items per slot, with the partials as r, g, b planes (24 B per lane and
    // item): C2 2048 spp 154.0 / 154.5 / 154.9 / 155.3 ms and 0.164 / 0.143 / 0.131 / 0.12 GB
    // of HBM traffic per launch at 8 / 6 / 5 / 4 items (profiles/r3/tail_items).
    // Mesh scenes chunk every tile (~32 items per slot): a tile's cost there depends on
    // how much mesh it sees, so whole tiles leave a long tail (C4 801 -> 1008 ms).
    // An explicit chunk count splits every tile.
    WorkPlan wp{};
    wp.s_begin = sample_begin;
    wp.s_end = sample_end;
    wp.tile_stride = tile_stride;
    wp.tile_offset = tile_offset;
    // Affine mesh scenes in parity mode, when the split form is selected (render_split): pixel-chunks of
    // split_chunk samples (an explicit `chunks` sets the chunk count as for the one-kernel
    // form, so both forms then sum the same chunks in the same order).
    const int kflags = kflags0 | (tlist ? 128 : 0);  // F_TLIST
#if PTMI_STUDY
    const bool split = s->split && split_supported(kflags) && range > 0;
#else
    constexpr bool split = false;
#endif
#if PTMI_STUDY
    if (split) {
        uint32_t nch = chunks ? chunks : (range + s->split_chunk - 1) / s->split_chunk;
        nch = std::max<uint32_t>(1, std::min<uint32_t>(nch, range));
        wp.chunk_len = (range + nch - 1) / nch;
        wp.nchunks = (range + wp.chunk_len - 1) / wp.chunk_len;
        wp.n_long = wp.nchunks;
        wp.tail_len = wp.chunk_len;
        wp.n_whole = 0;
        wp.n_tail = owned_tiles;
    }
#endif
    uint32_t n_tail = owned_tiles;
    const bool auto_chunks = chunks == 0;
    if (split) {
        chunks = wp.nchunks;
    } else if (chunks == 0) {
        const bool mesh = (s->flags & 1) != 0;  // F_GROUPS
        if (!mesh || s->tail_tiles)
            n_tail = std::min<uint32_t>(owned_tiles, s->tail_tiles ? s->tail_tiles : (uint32_t)(s->resident_waves / 2));
        // A sample-split rank of a mesh scene holding at most a quarter of the samples (every tile):
        // 48 items per slot instead of 32 (round 6, C4 8 ranks: projected efficiency 0.896 -> 0.904;
        // at 2 ranks 48 cost 0.962 -> 0.940, and the one-GPU frame 1.7 %, so those keep 32).
        // Tile-split ranks keep 32 (C5: 0.857 / 0.854).
        const bool sample_share = mesh && tile_stride == 1 && (uint64_t)range * 4 <= samples;
        const uint64_t want =
            (uint64_t)s->resident_waves * (mesh ? (sample_share ? s->mesh_items_share : s->mesh_items) : s->tail_items);
        // A mesh scene's tile-split rank owns 1/N of the tiles, so a chunk round is a fraction
        // of the machine (2,400 items at N = 8 against 4,096 wave slots) and the 64-sample floor
        // held it at ~19 items per slot; half the floor lets the items-per-slot target bind
        // (C5 8 ranks: 55 chunks of 38 samples, projected efficiency 0.81 -> 0.84; C4 tile split
        // 0.80 -> 0.81).  Sample-split ranks keep every tile and the floor (C4 0.90 -> 0.86 at
        // the half floor; profiles/r5/shards/chunks).
        const uint32_t floor = (mesh && tile_stride > 1) ? std::max<uint32_t>(1, s->min_chunk / 2) : s->min_chunk;
        chunks = (uint32_t)std::min<uint64_t>((want + n_tail - 1) / std::max<uint32_t>(n_tail, 1),
                                              std::max<uint32_t>(range / floor, 1));
    }
    // The path pool of the tile-list kernels numbers an item's paths 64 x its samples in 32 bits.
    if (tlist) chunks = std::max<uint32_t>(chunks, (range + (1u << 25) - 1) >> 25);
    chunks = std::max<uint32_t>(1, std::min<uint32_t>(chunks, std::max<uint32_t>(range, 1)));
    const uint32_t chunk_len = range == 0 ? 1 : (range + chunks - 1) / chunks;
    chunks = range == 0 ? 1 : (range + chunk_len - 1) / chunk_len;
    if (chunks == 1 && !split) n_tail = 0;  // one chunk: every tile is whole
    wp.n_whole = owned_tiles - n_tail;
    wp.n_tail = n_tail;
    wp.nchunks = chunks;
    wp.chunk_len = chunk_len;
    wp.n_long = chunks;
    wp.tail_len = chunk_len;
    // Mesh scenes, automatic plans: the last chunk round is cut into tail_split shorter rounds,
    // numbered last (and so dispatched last), so the launch drains on short items -- the
    // end-of-launch ramp was 3.1 % of the one-GPU C5 frame's slot-time (profiles/r4/timeline).
    // 2048 spp, one MI355X (profiles/r5/tail_split): C5 876 -> 865 ms, C4 unchanged.  Only
    // while the short chunks keep >= min_chunk / 2 samples: on 8-rank shares (64-sample chunks)
    // 16-sample ones cost C4's sample split more at each item's end than they saved at the
    // launch's (projected efficiency 0.893 -> 0.878) and left C5's tile split as it was.
    // Round 6: the path-pool kernels (affine mesh scenes in parity mode) have no per-item lane
    // drain, so their short chunks may go down to 8 samples (tail_min): an 8-rank C5 tile share
    // (38-sample chunks) drained 9.8 ms of its 108.9 ms on its last round's costliest tiles
    // (profiles/r6/timeline).  Chunks are summed in chunk order either way.
    const bool pooled = (kflags0 & 1) && !(kflags0 & (16 | 32 | 64));  // F_GROUPS, not F_PROJ / F_TEX / F_XRNG
    const uint32_t tail_min = s->tail_min ? s->tail_min : pooled ? 8u : s->min_chunk / 2;
    const uint32_t tl = (chunk_len + std::max<uint32_t>(s->tail_split, 1) - 1) / std::max<uint32_t>(s->tail_split, 1);
    if (!split && auto_chunks && (s->flags & 1) && chunks > 1 && s->tail_split > 1 && tl >= tail_min) {
        const uint32_t rest = range - (chunks - 1) * chunk_len;
        wp.n_long = chunks - 1;
        wp.tail_len = tl;
        wp.nchunks = wp.n_long + (rest + tl - 1) / tl;
        chunks = wp.nchunks;
    }
    wp.order = nullptr;
    wp.cost = nullptr;
    wp.tiles = nullptr;
    if (tlist) {
        if (s->tlist_stride != tile_stride || s->tlist_offset != tile_offset || s->tlist_host.size() != owned_tiles) {
            HIP_TRY(hipStreamSynchronize(st));  // tlist_host may still feed an earlier copy
            s->tlist_host.resize(owned_tiles);
            for (uint32_t k = 0; k < owned_tiles; k++) s->tlist_host[k] = owned_tile(k);
            if (s->tlist_dev && s->tlist_cap < owned_tiles) {
                HIP_TRY(hipFree(s->tlist_dev));
                s->tlist_dev = nullptr;
            }
            if (!s->tlist_dev) {
                HIP_TRY(hipMalloc((void**)&s->tlist_dev, (size_t)owned_tiles * sizeof(uint32_t)));
                s->tlist_cap = owned_tiles;
            }
            HIP_TRY(hipMemcpyAsync(s->tlist_dev, s->tlist_host.data(), (size_t)owned_tiles * sizeof(uint32_t),
                                   hipMemcpyHostToDevice, st));
            s->tlist_stride = tile_stride;
            s->tlist_offset = tile_offset;
            s->order_n = 0;  // the dispatch order indexes owned tiles: rebuild it
        }
        wp.tiles = s->tlist_dev;
    }
    const bool mesh_plan = (s->flags & 1) != 0;  // F_GROUPS
    if (!split && s->tile_order && owned_tiles > 0 && mesh_plan) {
        // Mesh scenes: the dispatch order of the work items -- whole tiles among themselves,
        // then each chunk round's tiles among themselves (which tiles are whole and which
        // chunked stays the raster-defined plan above, so no pixel's sums change).  A rank's
        // first launch (or one after its tile ownership or plan changed) takes the static
        // order (mesh_tile_cost's hull-hit classes, costliest first, raster order within a
        // class); with tile_order 2 every launch also measures its items and
        // tile_order_kernel writes the next launch's order from those durations.  (The
        // kernels without meshes do not measure: see item_cost_add.)
#if PTMI_STUDY
        if (s->tile_order == 2 && !s->cost_dev) {
            HIP_TRY(hipMalloc((void**)&s->cost_dev, (size_t)tiles * sizeof(unsigned long long)));
            HIP_TRY(hipMemsetAsync(s->cost_dev, 0, (size_t)tiles * sizeof(unsigned long long), st));
        }
#endif
        if (s->order_stride != tile_stride || s->order_offset != tile_offset || s->order_n != owned_tiles ||
            s->order_tlist != tlist ||
            s->order_whole != wp.n_whole) {
            HIP_TRY(hipStreamSynchronize(st));  // order_host may still feed an earlier copy
            mesh_tile_cost(s->tc_in, s->tile_cost, owned_tiles, owned_tile);  // this render's tiles, once
            s->order_host.resize(owned_tiles);
            for (uint32_t k = 0; k < wp.n_whole; k++) s->order_host[k] = k;
            for (uint32_t k = 0; k < n_tail; k++) s->order_host[wp.n_whole + k] = k;
            std::stable_sort(s->order_host.begin() + wp.n_whole, s->order_host.end(), [&](uint32_t a, uint32_t b) {
                    return s->tile_cost[owned_tile(wp.n_whole + a)] > s->tile_cost[owned_tile(wp.n_whole + b)];
                });
            if (s->order_dev && s->order_cap < owned_tiles) {
                HIP_TRY(hipFree(s->order_dev));
                s->order_dev = nullptr;
            }
            if (!s->order_dev) {
                HIP_TRY(hipMalloc((void**)&s->order_dev, (size_t)owned_tiles * sizeof(uint32_t)));
                s->order_cap = owned_tiles;
            }
            HIP_TRY(hipMemcpyAsync(s->order_dev, s->order_host.data(), (size_t)owned_tiles * sizeof(uint32_t),
                                   hipMemcpyHostToDevice, st));
            s->order_stride = tile_stride;
            s->order_offset = tile_offset;
            s->order_n = owned_tiles;
            s->order_tlist = tlist;
            s->order_whole = wp.n_whole;
        }
        wp.order = s->order_dev;
#if PTMI_STUDY
        wp.cost = s->tile_order == 2 ? s->cost_dev : nullptr;
#endif
    }
    if ((s->flags & 8) && s->dev.cam.aperture != 0 && s->sunf_samples != samples) {  // DoF table for this S
        if (s->sunf) {
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipFree(s->sunf));
            s->sunf = nullptr;
        }
        HIP_TRY(hipMalloc((void**)&s->sunf, (size_t)samples * 2 * sizeof(double)));
        HIP_TRY(launch_sunflower(s->sunf, samples, st));
        s->sunf_samples = samples;
    }
    hipEvent_t ev0 = nullptr, ev1 = nullptr;
    if (s->timing) {
        for (hipEvent_t* e : {&ev0, &ev1}) {
            if (!s->spare.empty()) {
                *e = s->spare.back();
                s->spare.pop_back();
            } else {
                HIP_TRY(hipEventCreate(e));
            }
        }
    }
    if (tile_stride > 1) HIP_TRY(hipMemsetAsync(sums_dev, 0, (size_t)npix * 4 * sizeof(double), st));  // un-owned tiles
    const bool planes = (s->flags & 1) == 0 || (PTMI_MESH_PLANES && !split);  // partial layout (ptmi_kernels.hip store_sums)
    const size_t need = (size_t)wp.n_tail * 64 * chunks * (planes ? 3 : 4) * sizeof(double);
    if (need > s->partial_bytes) {
        if (s->partial) {
            HIP_TRY(hipStreamSynchronize(st));
            HIP_TRY(hipFree(s->partial));
            s->partial = nullptr;
            s->partial_bytes = 0;
        }
        HIP_TRY(hipMalloc((void**)&s->partial, need));
        s->partial_bytes = need;
    }
    if (!split) {  // the launch's work-item counter, zeroed outside the timed span
        if (!s->item_ctr) HIP_TRY(hipMalloc((void**)&s->item_ctr, 256));
        HIP_TRY(hipMemsetAsync(s->item_ctr, 0, sizeof(uint32_t), st));
    }
    if (ev0) HIP_TRY(hipEventRecord(ev0, st));
#if PTMI_STUDY
    if (split) {
        const int rc = render_split(s, samples, wp, seeds_dev, sums_dev, st, err, err_len);
        if (rc) return rc;
    } else
#endif
    {
        HIP_TRY(launch_trace(s->dev, kflags, samples, wp, seeds_dev, s->sunf, sums_dev, s->partial, s->item_ctr, st));
    }
    if (ev1) {
        HIP_TRY(hipEventRecord(ev1, st));
        s->events.emplace_back(ev0, ev1);
    }
#if PTMI_STUDY
    // after the timed launch: the next launch's order from this one's item durations
    if (wp.cost) HIP_TRY(launch_tile_order(wp.cost, wp.n_whole, wp.n_tail, tile_stride, tile_offset, s->order_dev, st));
#endif
    HIP_TRY(launch_reduce(s->partial, sums_dev, wp, (int)W, (int)H, planes, st));
    return PTMI_OK;
}

int ptmi_scene_set_rng(ptmi_scene* s, int mode, char* err, size_t err_len) {
    if (!s || (mode != PTMI_RNG_NOISE3D && mode != PTMI_RNG_XOSHIRO)) {
        set_err(err, err_len, "ptmi_scene_set_rng: bad scene or mode %d", mode);
        return PTMI_ERR_ARG;
    }
    if (mode == PTMI_RNG_XOSHIRO && (s->flags & (16 | 32))) {  // F_PROJ | F_TEX
        set_err(err, err_len, "the statistical RNG mode exists for affine, untextured scenes only (this scene is %s)",
                (s->flags & 32) ? "textured" : "not affine");
        return PTMI_ERR_UNSUPPORTED;
    }
    s->rng = mode;
    HIP_TRY(hipSetDevice(s->device));
    HIP_TRY(resident_waves(s));
    return PTMI_OK;
}

int ptmi_scene_set_timing(ptmi_scene* s, int enable) {
    if (!s) return PTMI_ERR_ARG;
    s->timing = enable != 0;
    return PTMI_OK;
}

int ptmi_scene_kernel_time(ptmi_scene* s, double* total_ms, uint32_t* launches, char* err, size_t err_len) {
    if (!s) {
        set_err(err, err_len, "scene == NULL");
        return PTMI_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    double tot = 0.0;
    for (auto& e : s->events) {
        HIP_TRY(hipEventSynchronize(e.second));
        float ms = 0.f;
        HIP_TRY(hipEventElapsedTime(&ms, e.first, e.second));
        tot += ms;
        s->spare.push_back(e.first);
        s->spare.push_back(e.second);
    }
    if (total_ms) *total_ms = tot;
    if (launches) *launches = (uint32_t)s->events.size();
    s->events.clear();
    return PTMI_OK;
}

int ptmi_finalize(const double* sums_dev, double* out_dev, uint32_t n_pixels, uint32_t samples, void* hip_stream,
                  char* err, size_t err_len) {
    if (!sums_dev || !out_dev || samples == 0) {
        set_err(err, err_len, "bad finalize arguments");
        return PTMI_ERR_ARG;
    }
    HIP_TRY(launch_finalize(sums_dev, out_dev, n_pixels, samples, (hipStream_t)hip_stream));
    return PTMI_OK;
}

int ptmi_fill_seeds(double* seeds_dev, uint32_t n, uint64_t seed_stream, void* hip_stream, char* err,
                    size_t err_len) {
    if (!seeds_dev) {
        set_err(err, err_len, "seeds_dev == NULL");
        return PTMI_ERR_ARG;
    }
    HIP_TRY(launch_seeds(seeds_dev, n, seed_stream, (hipStream_t)hip_stream));
    return PTMI_OK;
}

int ptmi_trace(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri, const void* groups,
               uint32_t n_grp, int device_index, uint32_t samples, const void* camera, const double* seeds,
               uint64_t seed_stream, const ptmi_textures* textures, double* out_rgba, char* err, size_t err_len) {
    if (!out_rgba || samples == 0) {
        set_err(err, err_len, "out_rgba == NULL or samples == 0");
        return PTMI_ERR_ARG;
    }
    ptmi_scene* s = nullptr;
    int rc = ptmi_scene_create_textured(device_index, objects, n_obj, triangles, n_tri, groups, n_grp, camera,
                                        textures, &s, err, err_len);
    if (rc) return rc;
    const uint32_t npix = s->width * s->height;
    double *d_seeds = nullptr, *d_sums = nullptr;
    hipStream_t st = nullptr;
    auto fail = [&](int code) {
        if (st) (void)hipStreamDestroy(st);
        if (d_seeds) (void)hipFree(d_seeds);
        if (d_sums) (void)hipFree(d_sums);
        ptmi_scene_destroy(s);
        return code;
    };
#define TRY_OR_FAIL(call)                                                                         \
    do {                                                                                          \
        hipError_t e_ = (call);                                                                   \
        if (e_ != hipSuccess) {                                                                   \
            set_err(err, err_len, "%s failed: %s", #call, hipGetErrorString(e_));                 \
            return fail(PTMI_ERR_HIP);                                                            \
        }                                                                                         \
    } while (0)
    TRY_OR_FAIL(hipStreamCreateWithFlags(&st, hipStreamNonBlocking));
    TRY_OR_FAIL(hipMalloc((void**)&d_seeds, (size_t)npix * sizeof(double)));
    TRY_OR_FAIL(hipMalloc((void**)&d_sums, (size_t)npix * 4 * sizeof(double)));
    if (seeds) {
        TRY_OR_FAIL(hipMemcpyAsync(d_seeds, seeds, (size_t)npix * sizeof(double), hipMemcpyHostToDevice, st));
    } else if ((rc = ptmi_fill_seeds(d_seeds, npix, seed_stream, st, err, err_len))) {
        return fail(rc);
    }
    if ((rc = ptmi_scene_render(s, samples, 0, samples, 1, 0, d_seeds, d_sums, 0, st, err, err_len))) return fail(rc);
    if ((rc = ptmi_finalize(d_sums, d_sums, npix, samples, st, err, err_len))) return fail(rc);
    TRY_OR_FAIL(hipMemcpyAsync(out_rgba, d_sums, (size_t)npix * 4 * sizeof(double), hipMemcpyDeviceToHost, st));
    TRY_OR_FAIL(hipStreamSynchronize(st));
#undef TRY_OR_FAIL
    fail(PTMI_OK);
    return PTMI_OK;
}

}  // extern "C"


// Sample split by cost, not count: the first sample index of device g of n (g = n ->
// samples).  Samples past n ~ 553 / ~731 put the hemisphere / anti-aliasing noise on
// the large-argument sin reduction and cost ~1 / ~2 % more (x100 weights 100, 101, 102; round 6,
// re-measured on the round-6 kernel's 8-rank shares -- round 5's 50 / 51 / 52 left rank 0 2.5 %
// over the mean).  Same table as ptmi/dist.py's sample_split_point.
static uint32_t split_point(int g, int n, uint32_t samples) {
    static const uint64_t knot[2] = {553, 731}, w[3] = {100, 101, 102};
    auto cost = [&](uint64_t m) {
        return w[0] * std::min<uint64_t>(m, knot[0]) + w[1] * (std::min<uint64_t>(std::max<uint64_t>(m, knot[0]), knot[1]) - knot[0]) +
               w[2] * (std::max<uint64_t>(m, knot[1]) - knot[1]);
    };
    const uint64_t target = ((uint64_t)g * cost(samples) + (uint64_t)n - 1) / (uint64_t)n;
    uint64_t m;
    if (target <= w[0] * knot[0])
        m = (target + w[0] - 1) / w[0];
    else if (target <= cost(knot[1]))
        m = knot[0] + (target - cost(knot[0]) + w[1] - 1) / w[1];
    else
        m = knot[1] + (target - cost(knot[1]) + w[2] - 1) / w[2];
    return (uint32_t)std::min<uint64_t>(m, samples);
}

extern "C" uint32_t ptmi_sample_split_point(int g, int n, uint32_t samples) {
    if (n <= 0 || g < 0) return 0;
    if (g >= n) return samples;
    return split_point(g, n, samples);
}

extern "C" int ptmi_trace_multi_timed(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                                      const void* groups, uint32_t n_grp, const int* devices, uint32_t n_devices,
                                      int split, uint32_t samples, const void* camera, const double* seeds,
                                      uint64_t seed_stream, const ptmi_textures* textures, double* out_rgba,
                                      ptmi_multi_timing* timing, char* err, size_t err_len) {
    using clk = std::chrono::steady_clock;
    auto ms_since = [](clk::time_point a, clk::time_point b) {
        return std::chrono::duration<double, std::milli>(b - a).count();
    };
    const clk::time_point t_start = clk::now();
    if (!out_rgba || samples == 0 || !devices || n_devices == 0 || (split != 0 && split != 1) || !camera) {
        set_err(err, err_len, "ptmi_trace_multi: bad arguments");
        return PTMI_ERR_ARG;
    }
    for (uint32_t d = 0; d < n_devices; d++) {
        const int rc = check_device(devices[d], err, err_len);
        if (rc) return rc;
    }
    // The scene is converted and its traversal index built once, on the host.
    HostScene hs;
    int rc = prepare_scene(objects, n_obj, triangles, n_tri, groups, n_grp, camera, textures, hs, err, err_len);
    if (rc) return rc;
    const clk::time_point t_prep = clk::now();
    const size_t npix = (size_t)hs.cam.width * hs.cam.height;
    const size_t frame_bytes = npix * 4 * sizeof(double);
    const int root = devices[0];
    // Device-side combine: every device's partial frame is copied (xGMI peer copy) into
    // its slot of a gather buffer on the first device, which sums the slots in device
    // order (deterministic) and normalises (tracer.cl:1184-1187).
    double* gather = nullptr;
    HIP_TRY(hipSetDevice(root));
    HIP_TRY(hipMalloc((void**)&gather, frame_bytes * n_devices));
    std::vector<int> rcs(n_devices, PTMI_OK);
    std::vector<int> peer(n_devices, -1);  // per shard: 1 direct peer access, 0 staged copy, -1 root itself
    std::vector<std::string> msgs(n_devices);
    std::vector<clk::time_point> t_rendered(n_devices, t_prep);
    // Per-device resources, released after the combine and read-back (hipFree
    // synchronises; freeing inside the device threads delayed the combine).
    std::vector<ptmi_scene*> scenes(n_devices, nullptr);
    std::vector<double*> seeds_d(n_devices, nullptr), sums_d(n_devices, nullptr);
    std::vector<hipStream_t> streams(n_devices, nullptr);
    auto shard = [&](uint32_t d) {
        char e[512] = {0};
        int& drc = rcs[d];
        const int dev = devices[d];
        ptmi_scene*& s = scenes[d];
        double*& d_seeds = seeds_d[d];
        double*& d_sums = sums_d[d];
        hipStream_t& st = streams[d];
        drc = upload_scene(hs, dev, textures, &s, e, sizeof(e));
        if (!drc && dev != root) {  // direct xGMI access to the gather buffer where the link allows it
            // hipMemcpyPeerAsync works without peer access (the runtime stages the copy), so a
            // refusal is not an error: it is reported (timing->peer_direct) and its sticky error
            // state is cleared, so it cannot surface later through launch_trace's hipGetLastError.
            int can = 0;
            peer[d] = 0;
            if (hipDeviceCanAccessPeer(&can, dev, root) == hipSuccess && can) {
                const hipError_t pe = hipDeviceEnablePeerAccess(root, 0);
                if (pe == hipSuccess || pe == hipErrorPeerAccessAlreadyEnabled) peer[d] = 1;
            }
            (void)hipGetLastError();
        }
        if (!drc && (hipStreamCreateWithFlags(&st, hipStreamNonBlocking) != hipSuccess ||
                     hipMalloc((void**)&d_seeds, npix * sizeof(double)) != hipSuccess ||
                     hipMalloc((void**)&d_sums, frame_bytes) != hipSuccess)) {
            drc = PTMI_ERR_HIP;
            std::snprintf(e, sizeof(e), "device %d: allocation failed", dev);
        }
        if (!drc) {
            if (seeds) {
                if (hipMemcpyAsync(d_seeds, seeds, npix * sizeof(double), hipMemcpyHostToDevice, st) != hipSuccess)
                    drc = PTMI_ERR_HIP;
            } else {
                drc = ptmi_fill_seeds(d_seeds, (uint32_t)npix, seed_stream, st, e, sizeof(e));
            }
        }
        if (!drc) {
            const uint32_t s0 = split == 0 ? split_point(d, n_devices, samples) : 0;
            const uint32_t s1 = split == 0 ? split_point(d + 1, n_devices, samples) : samples;
            // an empty range writes zeros (A = 0), so every slot of the gather buffer is defined
            drc = ptmi_scene_render(s, samples, s0, s1, split == 1 ? n_devices : 1, split == 1 ? d : 0, d_seeds, d_sums,
                                    0, st, e, sizeof(e));
        }
        if (!drc && hipStreamSynchronize(st) != hipSuccess) drc = PTMI_ERR_HIP;
        t_rendered[d] = clk::now();
        if (!drc && (hipMemcpyPeerAsync(gather + (size_t)d * npix * 4, root, d_sums, dev, frame_bytes, st) !=
                         hipSuccess ||
                     hipStreamSynchronize(st) != hipSuccess)) {
            drc = PTMI_ERR_HIP;
            std::snprintf(e, sizeof(e), "device %d: peer copy to device %d failed", dev, root);
        }
        msgs[d] = e;
    };
    auto release = [&]() {
        for (uint32_t d = 0; d < n_devices; d++) {
            (void)hipSetDevice(devices[d]);
            if (streams[d]) (void)hipStreamDestroy(streams[d]);
            if (seeds_d[d]) (void)hipFree(seeds_d[d]);
            if (sums_d[d]) (void)hipFree(sums_d[d]);
            if (scenes[d]) ptmi_scene_destroy(scenes[d]);
        }
        (void)hipSetDevice(root);
        (void)hipFree(gather);
    };
    std::vector<std::thread> threads;
    for (uint32_t d = 0; d < n_devices; d++) threads.emplace_back(shard, d);
    for (auto& t : threads) t.join();
    for (uint32_t d = 0; d < n_devices; d++)
        if (rcs[d]) {
            release();
            set_err(err, err_len, "device %d: %s", devices[d], msgs[d].empty() ? "render failed" : msgs[d].c_str());
            return rcs[d];
        }
    const clk::time_point t_all_rendered = *std::max_element(t_rendered.begin(), t_rendered.end());
    hipError_t he = hipSetDevice(root);
    if (he != hipSuccess) {
        release();
        set_err(err, err_len, "hipSetDevice(%d) before the combine: %s", root, hipGetErrorString(he));
        return PTMI_ERR_HIP;
    }
    double* frame = gather;  // slot 0 is overwritten in place by the ordered sum
    he = launch_combine(gather, n_devices, npix, frame, samples, nullptr);
    if (he == hipSuccess) he = hipDeviceSynchronize();
    const clk::time_point t_combined = clk::now();
    if (he == hipSuccess) he = hipMemcpy(out_rgba, frame, frame_bytes, hipMemcpyDeviceToHost);
    const clk::time_point t_end = clk::now();
    release();
    const clk::time_point t_done = clk::now();
    if (he != hipSuccess) {
        set_err(err, err_len, "combine / read-back on device %d: %s", root, hipGetErrorString(he));
        return PTMI_ERR_HIP;
    }
    if (timing) {
        timing->prepare_ms = ms_since(t_start, t_prep);
        timing->render_ms = ms_since(t_prep, t_all_rendered);
        timing->combine_ms = ms_since(t_all_rendered, t_combined);
        timing->readback_ms = ms_since(t_combined, t_end);
        timing->total_ms = ms_since(t_start, t_done);
        timing->peer_direct = (int32_t)std::count(peer.begin(), peer.end(), 1);
        timing->peer_staged = (int32_t)std::count(peer.begin(), peer.end(), 0);
    }
    return PTMI_OK;
}

// The device-side combine of ptmi_trace_multi, for callers that gather their own partial
// frames (one per GPU) into one device buffer: slots summed in slot order, x 1/S, alpha 1.
extern "C" int ptmi_combine_frames(const double* parts_dev, uint32_t n_parts, uint32_t n_pixels, double* out_dev,
                                   uint32_t samples, void* hip_stream, char* err, size_t err_len) {
    if (!parts_dev || !out_dev || n_parts == 0 || samples == 0) {
        set_err(err, err_len, "bad combine arguments");
        return PTMI_ERR_ARG;
    }
    HIP_TRY(launch_combine(parts_dev, n_parts, n_pixels, out_dev, samples, (hipStream_t)hip_stream));
    return PTMI_OK;
}

extern "C" int ptmi_trace_multi(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                                const void* groups, uint32_t n_grp, const int* devices, uint32_t n_devices, int split,
                                uint32_t samples, const void* camera, const double* seeds, uint64_t seed_stream,
                                const ptmi_textures* textures, double* out_rgba, char* err, size_t err_len) {
    return ptmi_trace_multi_timed(objects, n_obj, triangles, n_tri, groups, n_grp, devices, n_devices, split, samples,
                                  camera, seeds, seed_stream, textures, out_rgba, nullptr, err, err_len);
}

#if PTMI_STATS
namespace ptmi {
int stats_read(unsigned long long* out, int reset);
}
// DIAGNOSTIC build only: traversal counters (see PTMI_STATS in ptmi_kernels.hip).
extern "C" int ptmi_stats_read(unsigned long long* out, int reset) { return ptmi::stats_read(out, reset); }
#endif

// ---- Diagnostics (include/ptmi_diag.h) -------------------------------------------------
namespace ptmi {
#if PTMI_STUDY
hipError_t launch_walk(const DevScene& S, int flags, int mode, const WalkReq* req, uint32_t n, WalkRes* res,
                       uint32_t* next, uint32_t grid, hipStream_t st);
const void* walk_kernel_symbol(int mode);
#endif
hipError_t capture_setup(WalkReq* req, WalkRes* res, uint32_t cap);
hipError_t capture_count(uint32_t* n);
hipError_t timeline_setup(unsigned long long* buf, uint32_t cap);
}  // namespace ptmi

extern "C" int ptmi_diag_timeline_setup(void* buf_dev, uint32_t cap, char* err, size_t err_len) {
    const hipError_t e = timeline_setup((unsigned long long*)buf_dev, cap);
    if (e == hipErrorNotSupported) {
        set_err(err, err_len, "not a timeline build (make -C pathtracer-ocl_amd timeline)");
        return PTMI_ERR_UNSUPPORTED;
    }
    HIP_TRY(e);
    return PTMI_OK;
}

extern "C" int ptmi_diag_capture_setup(void* req_dev, void* res_dev, uint32_t cap, char* err, size_t err_len) {
    const hipError_t e = capture_setup((WalkReq*)req_dev, (WalkRes*)res_dev, cap);
    if (e == hipErrorNotSupported) {
        set_err(err, err_len, "not a capture build (make -C pathtracer-ocl_amd capture)");
        return PTMI_ERR_UNSUPPORTED;
    }
    HIP_TRY(e);
    return PTMI_OK;
}

extern "C" int ptmi_diag_capture_count(uint32_t* n, char* err, size_t err_len) {
    const hipError_t e = capture_count(n);
    if (e == hipErrorNotSupported) {
        set_err(err, err_len, "not a capture build");
        return PTMI_ERR_UNSUPPORTED;
    }
    HIP_TRY(e);
    return PTMI_OK;
}

extern "C" int ptmi_diag_walk(ptmi_scene* s, int mode, const void* req_dev, uint32_t n, void* res_dev,
                              uint32_t* counter_dev, void* hip_stream, float* ms, char* err, size_t err_len) {
#if !PTMI_STUDY
    (void)s, (void)mode, (void)req_dev, (void)n, (void)res_dev, (void)counter_dev, (void)hip_stream, (void)ms;
    set_err(err, err_len, "the standalone walk kernels are in the study build (make -C pathtracer-ocl_amd study)");
    return PTMI_ERR_UNSUPPORTED;
#else
    if (!s || !req_dev || !res_dev || (mode != 0 && mode != 1) || (mode == 1 && !counter_dev)) {
        set_err(err, err_len, "ptmi_diag_walk: bad arguments");
        return PTMI_ERR_ARG;
    }
    HIP_TRY(hipSetDevice(s->device));
    hipStream_t st = (hipStream_t)hip_stream;
    uint32_t grid = 0;
    if (mode == 1) {  // persistent: the resident waves of the pool kernel
        hipDeviceProp_t p;
        HIP_TRY(hipGetDeviceProperties(&p, s->device));
        int per_cu = 0;
        HIP_TRY(hipOccupancyMaxActiveBlocksPerMultiprocessor(&per_cu, walk_kernel_symbol(1), 64, 0));
        grid = (uint32_t)std::max(1, per_cu) * (uint32_t)p.multiProcessorCount;
        HIP_TRY(hipMemsetAsync(counter_dev, 0, sizeof(uint32_t), st));
    }
    hipEvent_t e0, e1;
    HIP_TRY(hipEventCreate(&e0));
    HIP_TRY(hipEventCreate(&e1));
    HIP_TRY(hipEventRecord(e0, st));
    const hipError_t le = launch_walk(s->dev, s->flags, mode, (const WalkReq*)req_dev, n, (WalkRes*)res_dev,
                                      counter_dev, grid, st);
    HIP_TRY(hipEventRecord(e1, st));
    HIP_TRY(hipEventSynchronize(e1));
    float t = 0.f;
    HIP_TRY(hipEventElapsedTime(&t, e0, e1));
    (void)hipEventDestroy(e0);
    (void)hipEventDestroy(e1);
    if (le == hipErrorInvalidValue) {
        set_err(err, err_len, "standalone walks need an affine, untextured mesh scene");
        return PTMI_ERR_UNSUPPORTED;
    }
    HIP_TRY(le);
    if (ms) *ms = t;
    return PTMI_OK;
#endif
}

extern "C" int ptmi_diag_tile_cost(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                                   const void* groups, uint32_t n_grp, const void* camera, uint8_t* out, uint32_t n_out,
                                   char* err, size_t err_len) {
    if (!out) {
        set_err(err, err_len, "out == NULL");
        return PTMI_ERR_ARG;
    }
    HostScene hs;
    const int rc = prepare_scene(objects, n_obj, triangles, n_tri, groups, n_grp, camera, nullptr, hs, err, err_len);
    if (rc) return rc;
    const uint32_t tiles = (uint32_t)(((hs.cam.width + 7) / 8) * ((hs.cam.height + 7) / 8));
    if (n_out < tiles) {
        set_err(err, err_len, "out holds %u tiles, the frame has %u", n_out, tiles);
        return PTMI_ERR_ARG;
    }
    if (hs.flags & 1) {
        std::vector<uint8_t> c;
        mesh_tile_cost(tile_cost_input(hs), c, tiles, [](uint32_t k) { return k; });
        std::memcpy(out, c.data(), tiles);
    } else {
        std::memset(out, 0, tiles);
    }
    return PTMI_OK;
}

extern "C" int ptmi_diag_set_split(ptmi_scene* s, int enable) {
    if (!s) return PTMI_ERR_ARG;
#if PTMI_STUDY
    s->split = enable != 0;
    return PTMI_OK;
#else
    return enable ? PTMI_ERR_UNSUPPORTED : PTMI_OK;  // the one-kernel form is the only one here
#endif
}

extern "C" int ptmi_diag_split_passes(const ptmi_scene* s) {
#if PTMI_STUDY
    return s ? (int)s->split_passes : -1;
#else
    return s ? 0 : -1;
#endif
}

extern "C" int ptmi_diag_set_knob(ptmi_scene* s, int knob, int value) {
    if (!s) return PTMI_ERR_ARG;
    const uint32_t pos = (uint32_t)std::max(1, value);
    switch (knob) {
    case PTMI_KNOB_TAIL_TILES: s->tail_tiles = (uint32_t)std::max(0, value); return PTMI_OK;
    case PTMI_KNOB_TAIL_ITEMS: s->tail_items = pos; return PTMI_OK;
    case PTMI_KNOB_MESH_ITEMS: s->mesh_items = pos; return PTMI_OK;
    case PTMI_KNOB_MESH_ITEMS_SHARE: s->mesh_items_share = pos; return PTMI_OK;
    case PTMI_KNOB_MIN_CHUNK: s->min_chunk = pos; return PTMI_OK;
    case PTMI_KNOB_TAIL_SPLIT: s->tail_split = pos; return PTMI_OK;
    case PTMI_KNOB_TAIL_MIN: s->tail_min = (uint32_t)std::max(0, value); return PTMI_OK;
    case PTMI_KNOB_WALK_BATCH: s->dev.walk_batch = (int32_t)std::min<uint32_t>(pos, 64); return PTMI_OK;
    case PTMI_KNOB_HEMI_MESH: s->dev.hemi_mesh = value != 0; return PTMI_OK;
    case PTMI_KNOB_TILE_ORDER:
        // 2 (the order measured by the last launch) needs the item timing that only the study
        // build compiles in (ptmi_kernels.hip PTMI_TILE_COST).
        if (value < 0 || value > (PTMI_STUDY ? 2 : 1)) return PTMI_ERR_UNSUPPORTED;
        s->tile_order = value;
        s->order_n = 0;  // rebuild the order at the next render
        return PTMI_OK;
#if PTMI_STUDY
    case PTMI_KNOB_SPLIT_CHUNK: s->split_chunk = pos; return PTMI_OK;
    case PTMI_KNOB_SPLIT_SLOTS: s->split_per_lane = pos; return PTMI_OK;
    case PTMI_KNOB_SPLIT_SYNC: s->split_sync = pos; return PTMI_OK;
    case PTMI_KNOB_SPLIT_BUDGET: s->split_budget = pos; return PTMI_OK;
#endif
    default: return PTMI_ERR_UNSUPPORTED;
    }
}

extern "C" int ptmi_diag_force_flags(int flags) {
    if (flags > 63) return PTMI_ERR_ARG;
    g_force_flags.store(flags < 0 ? -1 : flags);
    return PTMI_OK;
}

extern "C" int ptmi_diag_hemi_mismatch(const ptmi_scene* s) { return s ? s->hemi_mismatch : -1; }

extern "C" int ptmi_diag_scene_flags(const ptmi_scene* s) {
    return s ? trace_kernel_flags(s->flags | (s->rng == PTMI_RNG_XOSHIRO ? 64 : 0)) : -1;
}

extern "C" int ptmi_diag_tile_ownership(const ptmi_scene* s, uint32_t tile_stride) {
    if (!s || tile_stride == 0) return -1;
    return diagonal_tiles(s, tile_stride) ? 1 : 0;
}
