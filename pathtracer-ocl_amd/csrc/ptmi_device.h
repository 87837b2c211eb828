// ptmi_device.h -- HBM layout of a resident scene (host converter + gfx950 kernels).
//
// The reference's 1024/512/256-B packed records (tracer.cl:24-93) carry ~60 %
// padding and force every work-item to copy whole objects around
// (tracer.cl:846-849, 890).  Here they are split by access pattern:
//   * DevObject  -- per-object data, read with wave-UNIFORM indices inside the
//                   object loop (scalar s_load path, SGPR matrix operands);
//   * DevNode    -- 64-B BVH node (box + triangle range + 2 children), preorder
//                   numbering kept so traversal order == reference order;
//   * DevTri     -- 96-B hot triangle data (p1, e1, e2) streamed by the
//                   Moller-Trumbore loop; DevTriShade (n1..n3, color) is read
//                   only for the winning triangle of a ray.
// All doubles keep their 4th (w) component where the reference's double4 math
// reads it, so results are bit-faithful (see DESIGN.md "Parity contract").
#pragma once
#include <stdint.h>
#include <limits.h>

namespace ptmi {

struct alignas(16) DevObject {
    double inv[16];    // object inverse (tracer.cl:547-548)
    double inv_t[16];  // inverse transpose (tracer.cl:953)
    double color[4];
    double emission[4];
    double refractive_index;
    double min_y, max_y;  // cylinder clip (tracer.cl:426-434)
    double reflectivity;
    double bb_min[4], bb_max[4];  // group bounds in group space (tracer.cl:609)
    double plane_n[4];            // planes: normalize(mul(invT, (0,1,0,0))) with w = 0 (tracer.cl:913, 953-955),
                                  // computed on the device at upload with the kernel's own arithmetic
    int32_t type;                 // 0 plane 1 sphere 2 cylinder 3 cube 4 group
    int32_t child_count;          // group roots (tracer.cl:617-621)
    int32_t child_base;           // index of the first root in DevScene::roots
    int32_t key;                  // index in the reference's object list (tie-break order)
    int32_t st;                   // inv has the scale+translate zero pattern (see xform_st)
    int32_t invt_diag;            // rows 0-2 of inv_t are diagonal
    uint8_t tex, tex_index;       // isTextured, textureIndex (ocltracer.go:44-45)
    uint8_t tex_nm, tex_index_nm; // isTexturedNM, textureIndexNM (planes only, tracer.cl:907-914)
    int32_t pad;
    double tex_scale[4];          // textureScaleX, Y, XNM, YNM (ocltracer.go:36-39)
};
static_assert(sizeof(DevObject) == 512, "DevObject must stay 512 B");

// One texture array (image2d_array_t of tracer.cl:833): `layers` NRGBA8 images
// of w x h texels, row-major, layers concatenated.  layers == 0: the reference's
// all-zero fake image (ocltracer.go:249-251).
struct DevTexArray {
    const uint32_t* texels;
    int32_t w, h, layers, pad;
};

// Reference BVH node (CLGroup, tracer.cl:24-35): its box gates the triangles
// below it (the kernel tests it with the reference's exact line-box decision).
struct alignas(16) DevNode {
    double bb_min[3];
    double bb_max[3];
    int32_t child0, child1;  // > 0 means present (tracer.cl:683, 704)
    int32_t pad[2];
};
static_assert(sizeof(DevNode) == 64, "DevNode must stay 64 B");

// Triangle in traversal-index leaf order; `n` is its index in the reference's
// triangle list (tie-break order and DevTriShade slot), `chain` (bit 31 masked off:
// kLastTri marks a leaf's last triangle) locates its gate chain: ChainBox[chain >> 5 ..
// + (chain & 31)), followed by the chain's core box (the intersection of its boxes) at
// ChainBox[(chain >> 5) + (chain & 31)] (see ptmi_bvh.cpp and chain_certified).
struct alignas(16) DevTri {
    double p1[3];
    double e1[3];
    double e2[3];
    int32_t n, chain;
};
static_assert(sizeof(DevTri) == 80, "DevTri must stay 80 B");

// Box of a reference node on a triangle's gate chain.
struct alignas(16) ChainBox {
    double mn[3], mx[3];
};

// 4-wide traversal node over one reference root's triangles (ptmi_bvh.cpp): one
// 64-B line.  Box bounds are IEEE binary16 bit patterns rounded outward from the
// (slightly widened) double bounds in the root's frame (RootRec), +-infinity past
// binary16's range; binary16 -> float is exact, so the kernel's FP32 slab test is the
// one it ran on float boxes, with the same error bound.  Per axis the four children's
// minima and maxima share one 16-B row, bnd[axis][0 = min, 1 = max][child], so a lane
// picks its entry and exit planes by the sign of its ray direction with two selects per
// 8-B half (node_children).  child[i] is a child code: a Node4 index (< leaf bit) or
// leaf bit | first, the leaf's triangles being DevScene::tris[first ..] up to and including
// the first one whose chain has bit 31 set (kLastTri).  The leaf bit is kLeafNarrow when
// every code of the scene fits 16 bits (the affine kernels' traversal stack holds 16-bit
// entries in LDS), else kLeafWide (the generic instantiations, 32-bit entries);
// DevScene::leaf_bit says which.  An empty slot's code is a leaf of one degenerate
// triangle (DevScene::tris' last record, kLastTri set): never a candidate, so entering it
// -- only a NaN ray can -- is harmless, and the walk needs no third case.
struct alignas(64) Node4 {
    uint16_t bnd[3][2][4];  // [axis][min (rounded toward -inf), max (toward +inf)][child]
    int32_t child[4];
};
static_assert(sizeof(Node4) == 64, "Node4 must stay 64 B");
constexpr int32_t kLeafNarrow = 0x8000;      // 16-bit codes: nodes < 2^15, leaves 2^15 | first
constexpr int32_t kLeafWide = 0x40000000;    // 31-bit codes (and the builder's own format)
constexpr int32_t kEmptyChild = INT32_MIN;   // the builder's empty slot (ptmi_bvh.cpp), re-coded at upload
constexpr int32_t kLastTri = INT32_MIN;      // DevTri::chain bit 31: the last triangle of its leaf
constexpr int32_t kChainMask = 0x7FFFFFFF;

// One BVH root of a group object: the widened hull of all its triangles (the
// cull test before its walk) and the entry code of its Node4 index.  The Node4
// bounds of the root are stored relative to its frame: value = (bound - ctr) / sc,
// ctr the hull centre rounded to float (an exact double), sc = 2^s (s >= 0) the
// smallest power of two that brings the root's extent under binary16's range.
// A mesh far from the origin (an OBJ in millimetres at |x| ~ 1e4) or larger than
// 65504 units then keeps binary16's 11 significant bits on its own extent.
struct alignas(16) RootRec {
    double hull_mn[3], hull_mx[3];
    double ctr[3];
    int32_t entry;
    float bmax;  // max finite |bound - ctr| over the root's decoded Node4 boxes (FP32 slab error bound)
    float sc;    // 2^s: the kernel multiplies the ray's FP32 reciprocal by it (walk_setup)
    int32_t pad;
};
static_assert(sizeof(RootRec) == 96, "RootRec must stay 96 B");

struct alignas(16) DevTriShade {
    double n1[4], n2[4], n3[4];
    double color[4];
};

struct DevCamera {
    int32_t width, height;
    double pixel_size, half_width, half_height, aperture, focal_length;
    double inv[16];
    double origin[4];  // mul(inv, (0,0,0,1)) (tracer.cl:760), computed once on the host with the
                       // same separately rounded IEEE arithmetic: a frame constant in kernel args
};

// Compact records for the two hottest intersection loops (read with scalar
// loads; one object = one or two s_load_dwordx8/x16):
struct alignas(16) PlaneRec {  // intersectPlane needs row 1 of the inverse only
    double row1[4];
    int32_t slot, key;  // DevScene::objs slot, reference list index
    int32_t par;        // affine pairing (find_closest_prims): the next plane has the same row1[0..2]
    int32_t nz;         // bit i set: row1[i] (i < 3) is not +-0 (the affine kernels skip +-0 terms)
};
struct alignas(16) SphereRec {  // sphere with the scale+translate inverse pattern
    double m0, m3, m5, m7, m10, m11, m15, pad;
    int32_t slot, key;
    int32_t pad2[2];
};

// Passed BY VALUE as a kernel argument: everything here is wave-uniform.
// objs[] holds the intersectable objects sorted into type runs
// [planes | spheres | cylinders | cubes | groups]; run_end[t] is the end of run t.
struct DevScene {
    const DevObject* objs;
    int32_t run_end[5];  // slots [run_end[t-1], run_end[t]) hold type t
    int32_t n_planes;
    int32_t n_planes_y;  // leading planes whose row 1 is (+-0, m1, +-0, m3) (find_closest_prims)
    const PlaneRec* planes;      // all planes
    const SphereRec* spheres;    // scale+translate spheres (the rest: DevObject path)
    int32_t n_spheres_st;
    int32_t n_nodes4;  // Node4 count
    const int32_t* roots;  // concatenated group roots of all type-4 objects
    const RootRec* root_rec;  // per roots[] slot
    const DevNode* nodes;
    const Node4* nodes4;
    const ChainBox* chains;
    const DevTri* tris;
    const DevTriShade* tri_shade;
    int32_t leaf_bit;  // kLeafNarrow or kLeafWide (Node4 child codes)
    int32_t walk_batch;  // parked lanes that start a wave's BVH walk phase (mesh kernels; ptmi_api.cpp)
    int32_t hemi_mesh;   // mesh kernels read the hemisphere table's (sin, cos) plane (1) or compute (0)
    uint32_t n_obj;   // intersectable objects in objs[]
    uint32_t n_nodes, n_tri;
    uint32_t n_list;  // numObjects of the reference's list (fgi = seed / numObjects, tracer.cl:840)
    DevCamera cam;
    const DevCamera* camg;  // the same record in device memory (camera_ptr: reloaded where used)
    DevTexArray tex[3];  // textures, sphereTextures, cubeMapTextures (tracer.cl:833)
    const double* hemi;  // randomVectorInHemisphere table, 2^16 x 4 doubles (hemi_table_kernel)
};

// One BVH walk of a ray (walk_kernel / walk_pool_kernel): the world-space ray and the
// best primitive hit so far (t, pk as Hit::pk), one 64-B line; and its result, the
// closest hit over the primitives and every group object (tri / ti -1 when no triangle
// wins; u, v the winner's barycentrics).
struct alignas(16) WalkReq {
    double o[3], d[3];
    double t;
    int32_t pk, pad;
};
static_assert(sizeof(WalkReq) == 64, "WalkReq must stay 64 B");
struct alignas(16) WalkRes {
    double t;
    int32_t pk, tri, ti, pad;
    double u, v;
};
static_assert(sizeof(WalkRes) == 40 || sizeof(WalkRes) == 48, "WalkRes size");

// Split execution of mesh scenes (trace_split_kernel + walk_split_kernel, round 4): a
// pool of L path slots in HBM, structure of arrays.  A slot works on one pixel-chunk
// (pixel x sample range) at a time, its samples in order; when its ray needs a BVH walk
// the tracer saves the path here and appends the slot to the request list, the walker
// walks the list, and the next tracer pass resumes the path with the result.
struct SplitBufs {
    char* rec;     // [L] slot records of kSlotBytes (SplitRec), one slot's state on 4 cache lines
    uint32_t* req; // [L]: this pass's walk requests (slot ids); tracer wave w appends to its own
                   // segment [w * per_wave, + seg[w]) -- no atomics on a shared counter
    uint32_t* seg; // [L / per_wave]: requests in each wave's segment
    uint32_t* wcl; // [2 L / per_wave]: each wave's claimed block of pixel-chunks [next, end), kept
                   // from pass to pass (a block left half used at a pass's end is not lost)
    uint32_t* cnt; // [0] requests of the pass, [1] next pixel-chunk block to claim, [2] yields of the pass
    uint32_t L, per_wave, n_items, budget;  // budget: samples a slot starts per pass before it yields
};
// One slot (SplitBufs::rec): d = ro xyz, rd xyz, mask rgb, accumColor rgb, pixel-chunk sums rgb,
// best t; u = pixel-chunk id (or kSlotFree / kSlotDead), sample index, path flags, best pk;
// f = fgi, fgi2; res = the walk result.  Records rather than arrays per field: a resume or a
// save touches one slot's lines, not 20 arrays (TLB, load instructions).
struct alignas(256) SplitRec {
    double d[16];
    uint32_t u[4];
    float f[2];
    uint32_t pad[2];
    WalkRes res;
};
constexpr size_t kSlotBytes = sizeof(SplitRec);
static_assert(kSlotBytes == 256, "SplitRec must stay 256 B");
constexpr int kSplitD = 16;
constexpr int kSplitU = 4;
constexpr uint32_t kSlotFree = 0xFFFFFFFFu, kSlotDead = 0xFFFFFFFEu;

constexpr int kTile = 8;          // a wave64 covers an 8x8 pixel tile

// Chunk partials of the mesh kernels as r, g, b planes, as the kernels without meshes store
// them, instead of (r, g, b, samples) records (ptmi_kernels.hip store_sums; round 6).
#ifndef PTMI_MESH_PLANES
#define PTMI_MESH_PLANES 1
#endif

// One launch's work items (trace_kernel, by value).  The owned tiles are
// tile_offset + k * tile_stride, k = 0, 1, ... (or tiles[k], see below)  The first n_whole of them are one
// item each over the whole sample range [s_begin, s_end), summed straight into the
// frame; the last n_tail are split into nchunks sample chunks of chunk_len, one
// item each, whose sums go to a partial buffer (chunk-major: chunk c of tail tile tt,
// lane l at slot (c * n_tail + tt) * 64 + l of three planes r, g, b, or, in the mesh
// kernels, as one (r, g, b, samples) record per slot) that reduce_chunks_kernel adds
// up in chunk order.  Items are numbered whole tiles first, so the short chunk items
// fill the end of the launch.
struct WorkPlan {
    uint32_t s_begin, s_end;
    uint32_t tile_stride, tile_offset;
    uint32_t n_whole, n_tail;
    uint32_t nchunks, chunk_len;
    // Chunks [0, n_long) hold chunk_len samples each; the rest (the last rounds of a mesh
    // scene's automatic plan) hold tail_len each, so the launch ends on short items.
    // Uniform plans: n_long = nchunks, tail_len = chunk_len.
    uint32_t n_long, tail_len;
    // Optional dispatch order of the chunked tiles within each chunk round: item tq of a
    // round runs chunked tile order[n_whole + tq] (a permutation of [0, n_tail)); nullptr =
    // identity.  The tile keeps its own partial slot, so the sums and their order do not
    // change.  (Entries [0, n_whole) are the identity: whole tiles run in raster order.)
    const uint32_t* order;
    // Optional per-tile cost accumulator (mesh kernels): each work item adds its duration
    // (wall-clock ticks) at cost[tile]; tile_order_kernel turns it into the next order.
    unsigned long long* cost;
    // Optional owned-tile list (tile-split launches of the affine mesh kernels, the F_TLIST
    // instantiations): owned tile k is tiles[k] (raster index) instead of tile_offset +
    // k * tile_stride.  nullptr in every other launch.
    const uint32_t* tiles;
};

}  // namespace ptmi
