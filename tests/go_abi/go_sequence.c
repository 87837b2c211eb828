/* go_sequence.c -- the C calls go/ocltracer_hip.go makes, with the arguments it passes,
 * in the order it passes them, so the cgo binding's argument sequence runs on the GPU
 * although this image has no Go toolchain (tests/test_gpu_go_abi.py runs it).
 *
 *   go_sequence <scene> <width> <height> <samples> <out_dir>
 *
 * Records come from libptmi_host.so's restatement of BuildSceneBufferCL (byte-identical
 * to the Go slices, tests/test_host.py): `&slice[0]` of each slice, or NULL for an empty
 * one (records()); W*H seeds in [0,1) at Go rand.Float64 granularity (frameSeeds());
 * texture lists empty -> a zeroed ptmi_textures (textureArrays()); a caller-owned
 * W*H*4 output (make([]float64, n*4)); a 512-byte error buffer.  Then TraceMulti's call
 * with a C-allocated device list.  Writes seeds.f64, trace.f64, multi_tile.f64 and
 * multi_sample.f64 (raw little-endian doubles) to out_dir and exits 0, or prints the
 * error and exits 1.  Also checks the deviceIndex contract (ocltracer.go:135-140). */
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "ptmi.h"
#include "ptmi_host.h"

static int save(const char* dir, const char* name, const double* v, size_t n) {
    char path[1024];
    snprintf(path, sizeof path, "%s/%s", dir, name);
    FILE* f = fopen(path, "wb");
    if (!f || fwrite(v, sizeof(double), n, f) != n) {
        fprintf(stderr, "cannot write %s\n", path);
        return 1;
    }
    fclose(f);
    return 0;
}

int main(int argc, char** argv) {
    if (argc != 6) {
        fprintf(stderr, "usage: %s scene width height samples out_dir\n", argv[0]);
        return 2;
    }
    const int W = atoi(argv[2]), H = atoi(argv[3]), S = atoi(argv[4]);
    const char* dir = argv[5];
    char err[512];
    ptmi_records r;
    if (ptmi_host_build_scene(argv[1], W, H, 0.0, 0.0, NULL, &r, err, sizeof err)) {
        fprintf(stderr, "scene: %s\n", err);
        return 1;
    }
    /* frameSeeds(): one rand.Float64() per pixel -- here a fixed 64-bit LCG's top 53 bits */
    const size_t n = (size_t)W * H;
    double* seeds = malloc(n * sizeof(double));
    uint64_t x = 0x9E3779B97F4A7C15ull;
    for (size_t i = 0; i < n; i++) {
        x = x * 6364136223846793005ull + 1442695040888963407ull;
        seeds[i] = (double)(x >> 11) * 0x1p-53;
    }
    /* records(): &slice[0], nil for an empty slice */
    const void* obj = r.n_obj ? (const void*)r.objects : NULL;
    const void* tris = r.n_tri ? (const void*)r.triangles : NULL;
    const void* grps = r.n_grp ? (const void*)r.groups : NULL;
    ptmi_textures tex;
    memset(&tex, 0, sizeof tex); /* textureArrays(nil, nil, nil) */
    double* out = calloc(n * 4, sizeof(double));
    int rc = ptmi_trace(obj, r.n_obj, tris, r.n_tri, grps, r.n_grp, 0, (uint32_t)S, r.camera, seeds, 0, &tex, out,
                        err, sizeof err);
    if (rc != PTMI_OK) {
        fprintf(stderr, "ptmi_trace failed (%d): %s\n", rc, err);
        return 1;
    }
    /* deviceIndex < 0 selects device 0; past the last device is an error (logrus.Fatalf in Go) */
    double* out2 = calloc(n * 4, sizeof(double));
    rc = ptmi_trace(obj, r.n_obj, tris, r.n_tri, grps, r.n_grp, -1, (uint32_t)S, r.camera, seeds, 0, &tex, out2,
                    err, sizeof err);
    if (rc != PTMI_OK || memcmp(out, out2, n * 4 * sizeof(double)) != 0) {
        fprintf(stderr, "deviceIndex -1: rc %d (%s) or a different image\n", rc, err);
        return 1;
    }
    rc = ptmi_trace(obj, r.n_obj, tris, r.n_tri, grps, r.n_grp, ptmi_device_count(), (uint32_t)S, r.camera, seeds,
                    0, &tex, out2, err, sizeof err);
    if (rc != PTMI_ERR_DEVICE || strstr(err, "out of bounds") == NULL) {
        fprintf(stderr, "deviceIndex past the last device: rc %d (%s), want PTMI_ERR_DEVICE\n", rc, err);
        return 1;
    }
    /* TraceMulti: devices {0, 0} (this box has one GPU) in C memory, mode 1 (tile), then 0 (sample) */
    int* devs = malloc(2 * sizeof(int));
    devs[0] = devs[1] = 0;
    double* tile = calloc(n * 4, sizeof(double));
    double* smp = calloc(n * 4, sizeof(double));
    rc = ptmi_trace_multi(obj, r.n_obj, tris, r.n_tri, grps, r.n_grp, devs, 2, 1, (uint32_t)S, r.camera, seeds, 0,
                          &tex, tile, err, sizeof err);
    if (rc == PTMI_OK)
        rc = ptmi_trace_multi(obj, r.n_obj, tris, r.n_tri, grps, r.n_grp, devs, 2, 0, (uint32_t)S, r.camera, seeds,
                              0, &tex, smp, err, sizeof err);
    if (rc != PTMI_OK) {
        fprintf(stderr, "ptmi_trace_multi failed (%d): %s\n", rc, err);
        return 1;
    }
    if (save(dir, "seeds.f64", seeds, n) || save(dir, "trace.f64", out, n * 4) ||
        save(dir, "multi_tile.f64", tile, n * 4) || save(dir, "multi_sample.f64", smp, n * 4))
        return 1;
    ptmi_host_free_records(&r);
    free(devs), free(seeds), free(out), free(out2), free(tile), free(smp);
    printf("go_sequence: %s %dx%d %d spp ok\n", argv[1], W, H, S);
    return 0;
}
