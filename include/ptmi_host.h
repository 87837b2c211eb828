/*
 * ptmi_host.h -- C ABI of libptmi_host.so: the Go-free host side around the
 * path-tracing backend.
 *
 * It restates, in C++, what the reference's Go program does on either side of
 * ocl.Trace, producing byte-identical kernel input records:
 *   - the scene factories of cmd/pt (internal/app/scenes/<name>.go) with the camera
 *     (camera/camera.go), transforms (geom/matrix.go, Go math.Sin/Cos/Tan),
 *     shapes and bounding boxes (internal/app/shapes), the OBJ/MTL reader
 *     (obj/objparser.go), ComputeVertexNormals and the BVH Divide (shapes/bvh.go),
 *     and BuildSceneBufferCL / BuildCLGroup (internal/ocl/scene.go:14-155);
 *   - the output writers: the PNG clamp (tracer/pathtracer.go:50-59) and the
 *     .raw float32 image (raw/writer.go:11-35).
 * Records are the packed layouts of include/ptmi.h (1024/512/256/256 B).
 *
 * Every entry point returns 0 or a negative PTMI_ERR_* code (include/ptmi.h) and,
 * when `err` is non-NULL, a NUL-terminated message.
 */
#ifndef PTMI_HOST_H
#define PTMI_HOST_H

#include <stddef.h>
#include <stdint.h>

#include "ptmi.h" /* ptmi_textures, PTMI_ERR_* */

#ifdef __cplusplus
extern "C" {
#endif

typedef struct ptmi_records {
    uint8_t* objects;   /* n_obj * 1024 B (CLObject)   */
    uint32_t n_obj;
    uint8_t* triangles; /* n_tri * 512 B  (CLTriangle) -- may be NULL with n_tri == 0 */
    uint32_t n_tri;
    uint8_t* groups;    /* n_grp * 256 B  (CLGroup)    -- may be NULL with n_grp == 0 */
    uint32_t n_grp;
    uint8_t camera[256]; /* CLCamera as renderPixelPathTracer fills it (renderer.go:44-56) */
} ptmi_records;

/* Build the records of a named cmd/pt scene (cmd/pt/main.go:26-42 names) for a
 * width x height image.  `assets_dir` holds teapot.obj / gopher.obj (+ .mtl) for
 * the mesh scenes (NULL: "assets", as the reference reads them relative to its
 * CWD).  Free with ptmi_host_free_records. */
int ptmi_host_build_scene(const char* name, int width, int height, double aperture, double focal_length,
                          const char* assets_dir, ptmi_records* out, char* err, size_t err_len);
void ptmi_host_free_records(ptmi_records* r);

/* Newline-separated scene names this build restates (--list-scenes). */
const char* ptmi_host_scene_names(void);

/* PNG of a W*H*4 float64 RGBA frame: clamp(round(v * 255)) per channel, alpha 255
 * (pathtracer.go:40-59), 8-bit RGBA. */
int ptmi_host_write_png(const char* path, const double* rgba, int width, int height, char* err, size_t err_len);

/* .raw image (raw/writer.go:11-35): big-endian int32 1, 0, width, height, then
 * width*height big-endian float32 (R, G, B) triples; alpha is dropped. */
int ptmi_host_write_raw(const char* path, const double* rgba, int width, int height, char* err, size_t err_len);

/* LoadImage (internal/app/scenes/scene.go:30-56): a PNG file decoded as Go's
 * image/png does, converted to NRGBA8 as draw.Draw(NRGBA, Src) does; *nrgba gets
 * width*height*4 bytes (free with ptmi_host_free_image).  .jpg/.jpeg: image/jpeg is
 * not restated -- a PNG with the same stem is read instead when present, else error. */
int ptmi_host_load_image(const char* path, uint8_t** nrgba, uint32_t* width, uint32_t* height, char* err,
                         size_t err_len);
void ptmi_host_free_image(uint8_t* nrgba);

/* The texture arrays a named scene passes to ocl.Trace (Scene.Textures /
 * SphereTextures / CubeTextures) loaded from `assets_dir` and packed as
 * prepareTextures does (ocltracer.go:228-254): per list, width/height of its first
 * image and the NRGBA bytes of all its images concatenated.  Scenes without
 * textures get all counts 0.  Free with ptmi_host_free_textures. */
int ptmi_host_load_scene_textures(const char* name, const char* assets_dir, ptmi_textures* out, char* err,
                                  size_t err_len);
void ptmi_host_free_textures(ptmi_textures* t);

#ifdef __cplusplus
}
#endif
#endif /* PTMI_HOST_H */
