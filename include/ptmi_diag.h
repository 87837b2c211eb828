/* ptmi_diag.h -- DIAGNOSTIC entry points of libptmi.so (not part of the drop-in
 * boundary, include/ptmi.h): test hooks, tuning knobs, and the study build's standalone
 * BVH walk kernels and split execution form (DESIGN.md sections 4-5).  The product
 * library reads no tuning variable from the environment (PTMI_VERBOSE only); tests and
 * tuning scripts set the knobs below. */
#ifndef PTMI_DIAG_H
#define PTMI_DIAG_H
#include <stddef.h>
#include <stdint.h>

#include "ptmi.h"

#ifdef __cplusplus
extern "C" {
#endif

/* Capture builds only (make -C pathtracer-ocl_amd capture -> build/libptmi_capture.so):
 * the mesh kernels append each walk of their walk phases, up to cap of them, as a
 * 64-B request (world ray, primitive best t / key) to req_dev and its result (40 B + pad,
 * ptmi_device.h WalkRes) to res_dev.  Other builds return PTMI_ERR_UNSUPPORTED. */
int ptmi_diag_capture_setup(void* req_dev, void* res_dev, uint32_t cap, char* err, size_t err_len);
int ptmi_diag_capture_count(uint32_t* n, char* err, size_t err_len);

/* Timeline builds only (make -C pathtracer-ocl_amd timeline -> build/libptmi_timeline.so):
 * trace_kernel writes work item b's start and end wall-clock ticks (wall_clock64, 100 MHz)
 * to buf_dev[2b], buf_dev[2b + 1] for b < cap.  Other builds return PTMI_ERR_UNSUPPORTED. */
int ptmi_diag_timeline_setup(void* buf_dev, uint32_t cap, char* err, size_t err_len);

/* Study build only (make -C pathtracer-ocl_amd study -> build/libptmi_study.so; the product
 * returns PTMI_ERR_UNSUPPORTED): walk n requests of scene s with a standalone kernel,
 * results to res_dev; *ms = its time (HIP events on hip_stream).  mode 0: one request per
 * lane (walk_kernel); mode 1: persistent waves with per-lane refill from *counter_dev
 * (walk_pool_kernel). */
int ptmi_diag_walk(ptmi_scene* s, int mode, const void* req_dev, uint32_t n, void* res_dev,
                   uint32_t* counter_dev, void* hip_stream, float* ms, char* err, size_t err_len);

/* Host only (no device call): the static dispatch class of every 8x8 tile of a mesh
 * scene (ptmi_api.cpp mesh_tile_cost: how many of 9 camera rays through the tile pass a
 * group object's hull cull, 0..9), raster order, into out[0 .. tiles); all 0 without
 * meshes.  A rank's first launch dispatches each chunk round's tiles in this order. */
int ptmi_diag_tile_cost(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                        const void* groups, uint32_t n_grp, const void* camera, uint8_t* out, uint32_t n_out,
                        char* err, size_t err_len);

/* Mesh-scene execution form (study build; the product has only the one-kernel form and
 * returns PTMI_ERR_UNSUPPORTED for enable != 0): enable != 0 renders affine mesh scenes in
 * the split form (trace_split_kernel + walk_split_kernel, pass by pass), 0 (the default)
 * in the one-kernel form (trace_kernel with in-loop walk phases).  Both give the same
 * image for the same chunking.  ptmi_diag_split_passes: passes of the last split render. */
int ptmi_diag_set_split(ptmi_scene* s, int enable);
int ptmi_diag_split_passes(const ptmi_scene* s);

/* Work-plan knobs of a resident scene (ptmi_api.cpp ptmi_scene_render); the defaults are
 * the product's.  TAIL_TILES: chunked tail tiles of an automatic plan in scenes without
 * meshes (0 = automatic); TAIL_ITEMS / MESH_ITEMS: chunk items per resident wave slot;
 * MIN_CHUNK: fewest samples per chunk item; TILE_ORDER: dispatch order of a mesh scene's
 * chunked tiles, 0 raster, 1 costliest static class first (default), 2 from the last
 * launch's measured item durations (study build only); SPLIT_*: the split form's pool
 * (study build only); TAIL_SPLIT: a mesh scene's automatic plan cuts its last chunk round into
 * this many shorter rounds (1 = off); TAIL_MIN: the fewest samples of such a short chunk (0 =
 * automatic: 8 for the path-pool kernels, MIN_CHUNK / 2 otherwise); WALK_BATCH: parked lanes that
 * start a mesh kernel's walk phase (1-64; default by scene, ptmi_api.cpp); HEMI_MESH: 1 = the mesh
 * kernels read the hemisphere table (default), 0 = they compute it.  PTMI_ERR_UNSUPPORTED for a knob or value this build
 * lacks. */
enum {
    PTMI_KNOB_TAIL_TILES = 1,
    PTMI_KNOB_TAIL_ITEMS = 2,
    PTMI_KNOB_MESH_ITEMS = 3,
    PTMI_KNOB_MIN_CHUNK = 4,
    PTMI_KNOB_TILE_ORDER = 5,
    PTMI_KNOB_SPLIT_CHUNK = 6,
    PTMI_KNOB_SPLIT_SLOTS = 7,
    PTMI_KNOB_SPLIT_SYNC = 8,
    PTMI_KNOB_SPLIT_BUDGET = 9,
    PTMI_KNOB_TAIL_SPLIT = 10,
    PTMI_KNOB_MESH_ITEMS_SHARE = 11,
    PTMI_KNOB_TAIL_MIN = 12,
    PTMI_KNOB_WALK_BATCH = 13,
    PTMI_KNOB_HEMI_MESH = 14
};
int ptmi_diag_set_knob(ptmi_scene* s, int knob, int value);

/* Kernel feature flags (ptmi_kernels.hip F_*) forced onto every scene created after the
 * call, process-wide; -1 (the default) lets each scene choose.  Test hook: the generic
 * instantiations must give the specialised ones' images (tests/test_gpu_parity.py). */
int ptmi_diag_force_flags(int flags);

/* Records of the scene's hemisphere table where the generic (full-operator) sequences
 * give other bits than the affine ones the table holds (ptmi_kernels.hip
 * hemi_table_kernel): 0 on a sound toolchain; -1 for a NULL scene. */
int ptmi_diag_hemi_mismatch(const ptmi_scene* s);

/* The trace_kernel instantiation the scene's renders launch (its F_* kernel flags, e.g. 0 for
 * the reference scene, 5 for teapot / gopher, 271 for an affine mesh scene with wide child
 * codes, 31 for a non-affine scene); -1 for a NULL scene. */
int ptmi_diag_scene_flags(const ptmi_scene* s);

/* Tile ownership a tile-split ptmi_scene_render with this stride uses: 1 diagonal (tile (x, y)
 * to rank (x + y) mod stride), 0 raster (tile t to rank t mod stride); -1 for bad arguments. */
int ptmi_diag_tile_ownership(const ptmi_scene* s, uint32_t tile_stride);

#ifdef __cplusplus
}
#endif
#endif /* PTMI_DIAG_H */
