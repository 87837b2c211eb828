/*
 * ptmi.h -- C ABI of libptmi.so, the MI355X (gfx950) path-tracing backend that
 * replaces the reference's OpenCL host driver + kernel
 * (eriklupander/pathtracer-ocl  internal/ocl/ocltracer.go + internal/ocl/tracer.cl).
 *
 * The input records are consumed BYTE-FOR-BYTE in the reference's packed layouts:
 *   objects   : n_obj * 1024 B  CLObject   (ocltracer.go:25-51  == tracer.cl:37-63)
 *   triangles : n_tri *  512 B  CLTriangle (ocltracer.go:66-78  == tracer.cl:82-93)
 *   groups    : n_grp *  256 B  CLGroup    (ocltracer.go:53-64  == tracer.cl:24-35)
 *   camera    :          256 B  CLCamera   (ocltracer.go:85-96  == tracer.cl:6-17)
 * so a cgo caller passes &slice[0] of the slices BuildSceneBufferCL returns
 * (see INTEGRATION.md).  No pointer is retained after a call returns.
 *
 * Output: float64 RGBA, row-major, W*H*4 values, RGB = sum of samples / samples,
 * A = 1.0 (tracer.cl:1184-1187).
 *
 * Every entry point returns PTMI_OK (0) or a negative PTMI_ERR_* code and, when
 * `err` is non-NULL, a NUL-terminated message.  There is no silent fallback:
 * without a usable gfx950 device the calls fail.
 */
#ifndef PTMI_H
#define PTMI_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define PTMI_ABI_VERSION 1
#define PTMI_OBJECT_BYTES 1024
#define PTMI_TRIANGLE_BYTES 512
#define PTMI_GROUP_BYTES 256
#define PTMI_CAMERA_BYTES 256
#define PTMI_MAX_OBJECTS 16 /* tracer.cl:846 `__local object objects[16]` */

enum {
    PTMI_OK = 0,
    PTMI_ERR_ARG = -1,         /* bad sizes / NULL pointers / out-of-range indices   */
    PTMI_ERR_DEVICE = -2,      /* no such device, or not a gfx950 device            */
    PTMI_ERR_HIP = -3,         /* a HIP runtime call failed                          */
    PTMI_ERR_UNSUPPORTED = -4, /* input outside what this build implements (e.g. BVH too deep) */
    PTMI_ERR_NOMEM = -5
};

/* Texture arrays of ocl.Trace (textures / sphereTextures / cubeTextures,
 * ocltracer.go:178-183, 228-254): array k holds count[k] layers of
 * width[k] x height[k] NRGBA8 pixels (image.NRGBA.Pix, rows top to bottom), the
 * layers concatenated in slice order -- exactly the bytes prepareTextures hands
 * to clCreateImage.  [0] backs plane colours and plane normal maps, [1] sphere
 * colours (sphericalMap), [2] cube colours (cubeUV cross), tracer.cl:907-914,
 * 1077-1092.  A NULL struct or count 0 is the reference's all-zero fake image.
 * Sampling follows the kernel's sampler (tracer.cl:829): normalized
 * coordinates, CLK_ADDRESS_REPEAT, CLK_FILTER_LINEAR, UNORM8 -> c/255, layer =
 * clamp(rint(index), 0, count-1) -- in software (OpenCL 1.2 s8.2 formulas, FP32):
 * gfx950 has no image instructions (DESIGN.md "Textures").  Pixels are copied to the
 * device during the call; the pointers are not retained. */
typedef struct ptmi_textures {
    const uint8_t* pixels[3];
    uint32_t width[3], height[3], count[3];
} ptmi_textures;

/*
 * ptmi_trace -- drop-in for `func Trace(objects []CLObject, triangles []CLTriangle,
 *   groups []CLGroup, deviceIndex, samples int, camera CLCamera, textures,
 *   sphereTextures, cubeTextures []image.Image) []float64`   (ocltracer.go:100-226).
 *
 *  - empty triangle / group slices are allowed (n = 0): the reference pads them
 *    with one zero record (ocltracer.go:106-120), which is equivalent;
 *  - device_index < 0 selects device 0 (ocltracer.go:138-140), an index past the
 *    last device is an error (ocltracer.go:135-137: logrus.Fatalf);
 *  - seeds: W*H per-pixel seeds in [0,1), row-major (the reference draws one
 *    rand.Float64() per pixel, ocltracer.go:260-263).  NULL -> generated from
 *    `seed_stream` (Go-Float64 granularity k/2^53, SplitMix64-derived);
 *  - the frame is rendered in one resident launch sequence (the reference's 4-row
 *    batches exist only to dodge a display watchdog, ocltracer.go:212-213).
 */
int ptmi_trace(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
               const void* groups, uint32_t n_grp, int device_index, uint32_t samples,
               const void* camera, const double* seeds, uint64_t seed_stream,
               const ptmi_textures* textures, double* out_rgba, char* err, size_t err_len);

/*
 * ptmi_trace_multi -- ptmi_trace over several GPUs of this process:
 * one host thread per entry of devices[0..n_devices) (an index may repeat), each
 * rendering its shard of the frame into its own partial sums:
 *   split 0 (sample): device d renders a contiguous range of sample indices of
 *                     every pixel (global indices, as ptmi_scene_render), balanced
 *                     by cost: late indices weigh ~4 % more (ptmi/dist.py);
 *   split 1 (tile)  : device d renders every sample of the 8x8 tiles t with
 *                     t % n == d.
 * The host converts the scene and builds its traversal index once; each device
 * uploads it.  The partial frames are combined on the device side: peer copies
 * over xGMI into a gather buffer on devices[0], summed there in device order
 * (deterministic) and normalised as ptmi_finalize, then read back once.  The
 * result equals ptmi_trace's up to FP64 summation order: each device plans its own
 * work items (ptmi_scene_render, chunks = 0), and where that plan splits a tile's
 * samples into chunks differently from the one-device plan, the tile's per-pixel
 * sums are added in a different grouping (bit-identical when every tile is one
 * whole item on both sides, e.g. short sample ranges).  Same record / seed / error contract as ptmi_trace.  (The
 * torch.distributed driver, bench.py, does the same with one process per GPU and
 * an RCCL reduce.)
 */
int ptmi_trace_multi(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                     const void* groups, uint32_t n_grp, const int* devices, uint32_t n_devices, int split,
                     uint32_t samples, const void* camera, const double* seeds, uint64_t seed_stream,
                     const ptmi_textures* textures, double* out_rgba, char* err, size_t err_len);

/* Wall-clock phases of one ptmi_trace_multi call (milliseconds). */
typedef struct ptmi_multi_timing {
    double prepare_ms;  /* host: record conversion + traversal-index build, once for all devices */
    double render_ms;   /* until the slowest device has its partial frame: upload, seeds, kernels */
    double combine_ms;  /* from then: xGMI peer copies into the first device + the ordered sum */
    double readback_ms; /* the RGBA frame to host memory */
    double total_ms;    /* the whole call, releasing the device buffers included */
    int32_t peer_direct; /* shards on other devices with direct peer (xGMI) access to devices[0] */
    int32_t peer_staged; /* shards on other devices whose copy the runtime stages (peer access refused) */
} ptmi_multi_timing;

/* ptmi_trace_multi, also reporting its phases in *timing (may be NULL). */
int ptmi_trace_multi_timed(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                           const void* groups, uint32_t n_grp, const int* devices, uint32_t n_devices, int split,
                           uint32_t samples, const void* camera, const double* seeds, uint64_t seed_stream,
                           const ptmi_textures* textures, double* out_rgba, ptmi_multi_timing* timing, char* err,
                           size_t err_len);

/* The combine step of ptmi_trace_multi, for callers that gather their own partial
 * frames: parts_dev holds n_parts frames of n_pixels * 4 doubles (RGB sums, A = the
 * sample count) back to back on one device; out_dev[4i + c] = (sum over parts, in part
 * order, of part[4i + c]) * (1.0 / samples) for RGB and 1.0 for A (tracer.cl:1184-1187).
 * out_dev may alias parts_dev (slot 0).  Asynchronous on hip_stream. */
int ptmi_combine_frames(const double* parts_dev, uint32_t n_parts, uint32_t n_pixels, double* out_dev,
                        uint32_t samples, void* hip_stream, char* err, size_t err_len);

/* First sample index of device g of n in ptmi_trace_multi's cost-balanced sample
 * split (g = n -> samples); the same table as bench.py's ranks (ptmi/dist.py). */
uint32_t ptmi_sample_split_point(int g, int n, uint32_t samples);

/* --list-devices (cmd/pt/main.go:98-112). */
int ptmi_device_count(void);
int ptmi_device_name(int device_index, char* buf, size_t len);

/* ------------------------------------------------------------------------
 * Resident-scene API: the scene is converted and uploaded to HBM once, frames
 * are rendered from device-resident seeds into device-resident sums on a
 * caller-supplied HIP stream (hipStream_t passed as void*).  Used by bench.py,
 * the multi-GPU driver and any caller that renders several frames / sample
 * ranges per scene.  All device pointers are allocations on the scene's device.
 * ------------------------------------------------------------------------ */
typedef struct ptmi_scene ptmi_scene;

int ptmi_scene_create(int device_index, const void* objects, uint32_t n_obj, const void* triangles,
                      uint32_t n_tri, const void* groups, uint32_t n_grp, const void* camera,
                      ptmi_scene** out, char* err, size_t err_len);
/* ptmi_scene_create with the scene's texture arrays (see ptmi_textures; NULL =
 * no textures).  ptmi_scene_create(...) == ptmi_scene_create_textured(..., NULL, ...). */
int ptmi_scene_create_textured(int device_index, const void* objects, uint32_t n_obj, const void* triangles,
                               uint32_t n_tri, const void* groups, uint32_t n_grp, const void* camera,
                               const ptmi_textures* textures, ptmi_scene** out, char* err, size_t err_len);
void ptmi_scene_destroy(ptmi_scene* s);
int ptmi_scene_size(const ptmi_scene* s, uint32_t* width, uint32_t* height);

/*
 * Render samples [sample_begin, sample_end) of a `samples`-spp frame.
 *   seeds_dev  : W*H doubles
 *   sums_dev   : W*H*4 doubles, OVERWRITTEN with RGB sums over the sample range
 *                (A = number of samples) for owned pixels, 0 for the others.
 *   tile_stride/tile_offset: pixel ownership for a tile split -- 8x8 tile t is
 *                owned when t % tile_stride == tile_offset (1/0 = all pixels).
 *   chunks     : sample chunks per pixel for every owned tile (load balance), or
 *                0 = auto: most tiles are one work item over the whole range
 *                (summed in sample order), the tiles at the end of the launch are
 *                split into chunks; mesh scenes chunk every tile.  Chunk sums are
 *                combined in a fixed order, so results are deterministic.  The
 *                affine mesh kernels hand a work item's (pixel, sample) paths to
 *                whichever lanes are free (the path pool) and add a pixel's paths
 *                in completion order: every path is the reference's, the sums
 *                differ from sample order only by FP64 rounding, and a render
 *                is reproducible bit for bit.
 * Sample indices are GLOBAL (fgi2 = seed/samples and the DoF aperture pattern
 * depend on n and on the total, tracer.cl:841, 766), so any split of
 * [0, samples) sums to the same frame.
 */
int ptmi_scene_render(ptmi_scene* s, uint32_t samples, uint32_t sample_begin, uint32_t sample_end,
                      uint32_t tile_stride, uint32_t tile_offset, const double* seeds_dev,
                      double* sums_dev, uint32_t chunks, void* hip_stream, char* err, size_t err_len);

/* out_dev[i] = sums_dev[i] * (1.0 / samples) for RGB, 1.0 for A (tracer.cl:837,1184-1187). */
int ptmi_finalize(const double* sums_dev, double* out_dev, uint32_t n_pixels, uint32_t samples,
                  void* hip_stream, char* err, size_t err_len);

/* Fill seeds_dev[0..n) with the generator ptmi_trace uses for seeds == NULL. */
int ptmi_fill_seeds(double* seeds_dev, uint32_t n, uint64_t seed_stream, void* hip_stream, char* err,
                    size_t err_len);

/* Random numbers of the scene's renders.  PTMI_RNG_NOISE3D (the default) is the
 * reference's noise3D hash (tracer.cl:314-317, called at :869, 982, 993, 1014, 1038,
 * 1057), bit for bit: images equal the reference kernel's.  PTMI_RNG_XOSHIRO is an
 * opt-in STATISTICAL mode: the same uniforms drawn from xoshiro128**, one stream per
 * (pixel, sample) path seeded from the pixel's seed and the sample index (32-bit hash),
 * so images are deterministic and independent of the work split, and converge to the
 * same expectation as the parity mode, but do not equal the reference's.  Affine,
 * untextured scenes only (else PTMI_ERR_UNSUPPORTED). */
enum { PTMI_RNG_NOISE3D = 0, PTMI_RNG_XOSHIRO = 1 };
int ptmi_scene_set_rng(ptmi_scene* s, int mode, char* err, size_t err_len);

/* Kernel timing: with timing enabled, every trace_kernel launch of the scene is
 * bracketed by HIP events recorded on the launch stream; ptmi_scene_kernel_time
 * waits for them, returns the summed kernel milliseconds and launch count since
 * the last call, and resets the tally. */
int ptmi_scene_set_timing(ptmi_scene* s, int enable);
int ptmi_scene_kernel_time(ptmi_scene* s, double* total_ms, uint32_t* launches, char* err, size_t err_len);

/* Build / ABI identification (kernel name, offload arch, flags). */
const char* ptmi_build_info(void);

/* Diagnostics, host only (no device call): the traversal index ptmi_scene_create would
 * build for these records (ptmi_bvh.cpp), summarised into out[0..n_out):
 *   [0] Node4 count  [1] occupied child slots  [2] sum over occupied slots of the
 *   decoded child box's surface area, in object-space units  [3] infinite bounds among
 *   them  [4] largest root scale exponent s (bounds stored as (b - ctr) / 2^s)
 *   [5] roots  [6] longest chain of Node4s (the walk's stack holds <= 3 entries per
 *   level; ptmi_bvh.cpp keeps it <= 7)  [7] the child codes' leaf bit: 2^15 when every
 *   code fits the affine kernels' 16-bit traversal stack, else 2^30 (an affine scene then
 *   runs the wide-code instantiation, 32-bit stack).  Index quality (box inflation from the
 *   binary16 bounds) can be compared across translated or scaled copies of one mesh. */
int ptmi_index_stats(const void* objects, uint32_t n_obj, const void* triangles, uint32_t n_tri,
                     const void* groups, uint32_t n_grp, const void* camera, double* out, int n_out,
                     char* err, size_t err_len);

#ifdef __cplusplus
}
#endif
#endif /* PTMI_H */
