/*
 * ref_launch.c -- TEST INFRASTRUCTURE ONLY (oracle).  Never linked into the product.
 *
 * Runs the *reference* kernel itself: /root/reference/internal/ocl/tracer.cl,
 * compiled by oracle/Makefile with ROCm's own OpenCL C toolchain and device
 * libraries into oracle/_ref/tracer_ref.hsaco, dispatched through the HSA runtime
 * exactly as an OpenCL runtime would (one NDRange over W*H work-items, yOffset 0,
 * the full-frame seed array -- ocltracer.go:346-353 with one batch).
 *
 * Why HSA and not HIP: the reference is an OpenCL kernel with image2d_array_t
 * arguments and OpenCL hidden arguments (global offsets, printf buffer); HIP's
 * module launcher interprets image arguments as runtime objects.  Here the
 * kernarg segment is laid out by hand from the code object's metadata
 * (oracle/_ref/tracer_ref.args, emitted by the Makefile from the ELF notes).
 * The three image arguments point at zeroed descriptors: the benchmark scenes
 * are untextured so read_imagef is never executed (tracer.cl:907, 1077).
 *
 * Exported C API (ctypes, see tests/oracle_ref.py):
 *   int ptref_trace(const char* hsaco, int device_index,
 *                   const void* objects, uint32_t n_obj, const void* tris, uint32_t n_tri,
 *                   const void* groups, uint32_t n_grp, const void* camera256,
 *                   uint32_t samples, const double* seeds, uint32_t n_pixels,
 *                   uint32_t wg_size, double* out_rgba, double timeout_s,
 *                   char* err, size_t err_len);
 */
#define _GNU_SOURCE
#include <hsa/hsa.h>
#include <hsa/hsa_ext_amd.h>
#include <stdarg.h>
#include <stdint.h>
#include <stdio.h>
#include <stdlib.h>
#include <string.h>
#include <time.h>

static void seterr(char* err, size_t n, const char* fmt, ...) {
    if (!err || !n) return;
    va_list ap;
    va_start(ap, fmt);
    vsnprintf(err, n, fmt, ap);
    va_end(ap);
}

#define CHK(x, what)                                                             \
    do {                                                                         \
        hsa_status_t s_ = (x);                                                   \
        if (s_ != HSA_STATUS_SUCCESS && s_ != HSA_STATUS_INFO_BREAK) {           \
            const char* m_ = 0;                                                  \
            hsa_status_string(s_, &m_);                                          \
            seterr(err, err_len, "%s failed: 0x%x %s", what, (unsigned)s_, m_ ? m_ : ""); \
            rc = -1;                                                             \
            goto out;                                                            \
        }                                                                        \
    } while (0)

typedef struct {
    int want;
    int seen;
    hsa_agent_t gpu;
    hsa_agent_t cpu;
    int have_gpu, have_cpu;
} agent_find_t;

static hsa_status_t agent_cb(hsa_agent_t a, void* data) {
    agent_find_t* f = (agent_find_t*)data;
    hsa_device_type_t t;
    hsa_agent_get_info(a, HSA_AGENT_INFO_DEVICE, &t);
    if (t == HSA_DEVICE_TYPE_GPU) {
        if (f->seen == f->want && !f->have_gpu) {
            f->gpu = a;
            f->have_gpu = 1;
        }
        f->seen++;
    } else if (t == HSA_DEVICE_TYPE_CPU && !f->have_cpu) {
        f->cpu = a;
        f->have_cpu = 1;
    }
    return HSA_STATUS_SUCCESS;
}

typedef struct {
    hsa_amd_memory_pool_t pool;
    int found;
    int want_kernarg; /* 1: kernarg-capable fine grained (CPU); 0: coarse grained (GPU) */
} pool_find_t;

static hsa_status_t pool_cb(hsa_amd_memory_pool_t p, void* data) {
    pool_find_t* f = (pool_find_t*)data;
    hsa_amd_segment_t seg;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_SEGMENT, &seg);
    if (seg != HSA_AMD_SEGMENT_GLOBAL) return HSA_STATUS_SUCCESS;
    uint32_t flags = 0;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_GLOBAL_FLAGS, &flags);
    bool alloc = false;
    hsa_amd_memory_pool_get_info(p, HSA_AMD_MEMORY_POOL_INFO_RUNTIME_ALLOC_ALLOWED, &alloc);
    if (!alloc || f->found) return HSA_STATUS_SUCCESS;
    if (f->want_kernarg && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_KERNARG_INIT)) {
        f->pool = p;
        f->found = 1;
    } else if (!f->want_kernarg && (flags & HSA_AMD_MEMORY_POOL_GLOBAL_FLAG_COARSE_GRAINED)) {
        f->pool = p;
        f->found = 1;
    }
    return HSA_STATUS_SUCCESS;
}

/* Kernarg offsets from the code object metadata (tracer.cl:831-833 + hidden args). */
typedef struct {
    int objects, num_objects, triangles, groups, output, seeds, samples, camera, y_offset;
    int img0, img1, img2;
    int block_count_x, block_count_y, block_count_z;
    int group_size_x, group_size_y, group_size_z;
    int remainder_x, remainder_y, remainder_z;
    int global_offset_x, global_offset_y, global_offset_z;
    int grid_dims, printf_buffer;
} karg_layout_t;

static int load_layout(const char* hsaco, karg_layout_t* L, char* err, size_t err_len) {
    char path[4096];
    snprintf(path, sizeof path, "%s.args", hsaco);
    FILE* f = fopen(path, "r");
    if (!f) {
        seterr(err, err_len, "cannot open %s", path);
        return -1;
    }
    memset(L, 0xff, sizeof *L); /* -1 == absent */
    char kind[128];
    int off;
    int idx = 0;
    while (fscanf(f, "%127s %d", kind, &off) == 2) {
        if (!strcmp(kind, "arg")) {
            int* explicit_[] = {&L->objects, &L->num_objects, &L->triangles, &L->groups, &L->output,
                                &L->seeds, &L->samples, &L->camera, &L->y_offset,
                                &L->img0, &L->img1, &L->img2};
            if (idx < 12) *explicit_[idx] = off;
            idx++;
        }
#define H(name) else if (!strcmp(kind, "hidden_" #name)) L->name = off;
        H(block_count_x) H(block_count_y) H(block_count_z)
        H(group_size_x) H(group_size_y) H(group_size_z)
        H(remainder_x) H(remainder_y) H(remainder_z)
        H(global_offset_x) H(global_offset_y) H(global_offset_z)
        H(grid_dims) H(printf_buffer)
#undef H
    }
    fclose(f);
    if (idx != 12) {
        seterr(err, err_len, "%s: expected 12 explicit args, got %d", path, idx);
        return -1;
    }
    return 0;
}

static void* read_file(const char* p, size_t* n) {
    FILE* f = fopen(p, "rb");
    if (!f) return NULL;
    fseek(f, 0, SEEK_END);
    long sz = ftell(f);
    fseek(f, 0, SEEK_SET);
    void* b = malloc((size_t)sz);
    if (b && fread(b, 1, (size_t)sz, f) != (size_t)sz) {
        free(b);
        b = NULL;
    }
    fclose(f);
    *n = (size_t)sz;
    return b;
}

int ptref_trace(const char* hsaco, int device_index, const void* objects, uint32_t n_obj,
                const void* tris, uint32_t n_tri, const void* groups, uint32_t n_grp,
                const void* camera256, uint32_t samples, const double* seeds, uint32_t n_pixels,
                uint32_t wg_size, double* out_rgba, double timeout_s, char* err, size_t err_len) {
    int rc = 0;
    int inited = 0;
    hsa_queue_t* q = NULL;
    hsa_signal_t sig = {0};
    hsa_executable_t exe = {0};
    hsa_code_object_reader_t rdr = {0};
    void* code = NULL;
    void* dev[8] = {0};
    void* host = NULL;
    void* karg = NULL;
    void* printf_buf = NULL;
    karg_layout_t L;

    if (n_pixels == 0 || wg_size == 0 || n_pixels % wg_size) {
        seterr(err, err_len, "n_pixels (%u) must be a positive multiple of wg_size (%u): the reference "
               "kernel is built with uniform work-groups", n_pixels, wg_size);
        return -2;
    }
    if (load_layout(hsaco, &L, err, err_len)) return -2;

    CHK(hsa_init(), "hsa_init");
    inited = 1;
    agent_find_t af = {device_index < 0 ? 0 : device_index, 0};
    CHK(hsa_iterate_agents(agent_cb, &af), "hsa_iterate_agents");
    if (!af.have_gpu || !af.have_cpu) {
        seterr(err, err_len, "GPU agent %d not found (%d GPUs)", device_index, af.seen);
        rc = -3;
        goto out;
    }
    pool_find_t gp = {.want_kernarg = 0}, kp = {.want_kernarg = 1};
    CHK(hsa_amd_agent_iterate_memory_pools(af.gpu, pool_cb, &gp), "iterate gpu pools");
    CHK(hsa_amd_agent_iterate_memory_pools(af.cpu, pool_cb, &kp), "iterate cpu pools");
    if (!gp.found || !kp.found) {
        seterr(err, err_len, "memory pools not found (gpu %d kernarg %d)", gp.found, kp.found);
        rc = -3;
        goto out;
    }

    size_t code_len = 0;
    code = read_file(hsaco, &code_len);
    if (!code) {
        seterr(err, err_len, "cannot read %s", hsaco);
        rc = -2;
        goto out;
    }
    CHK(hsa_code_object_reader_create_from_memory(code, code_len, &rdr), "code object reader");
    CHK(hsa_executable_create_alt(HSA_PROFILE_FULL, HSA_DEFAULT_FLOAT_ROUNDING_MODE_DEFAULT, NULL, &exe),
        "executable create");
    CHK(hsa_executable_load_agent_code_object(exe, af.gpu, rdr, NULL, NULL), "load code object");
    CHK(hsa_executable_freeze(exe, NULL), "freeze");
    hsa_executable_symbol_t sym;
    CHK(hsa_executable_get_symbol_by_name(exe, "trace.kd", &af.gpu, &sym), "symbol trace.kd");
    uint64_t kobj;
    uint32_t kseg, gseg, pseg;
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_OBJECT, &kobj), "kobj");
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_KERNARG_SEGMENT_SIZE, &kseg), "kseg");
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_GROUP_SEGMENT_SIZE, &gseg), "gseg");
    CHK(hsa_executable_symbol_get_info(sym, HSA_EXECUTABLE_SYMBOL_INFO_KERNEL_PRIVATE_SEGMENT_SIZE, &pseg), "pseg");

    /* Device buffers: objects, triangles, groups, output, seeds, camera, images. */
    size_t sz[7] = {(size_t)n_obj * 1024, (size_t)n_tri * 512, (size_t)n_grp * 256,
                    (size_t)n_pixels * 32, (size_t)n_pixels * 8, 256, 3 * 64};
    size_t total_host = 0;
    for (int i = 0; i < 7; i++) {
        CHK(hsa_amd_memory_pool_allocate(gp.pool, sz[i], 0, &dev[i]), "device alloc");
        total_host += sz[i];
    }
    CHK(hsa_amd_memory_pool_allocate(kp.pool, total_host, 0, &host), "host staging alloc");
    CHK(hsa_amd_agents_allow_access(1, &af.gpu, NULL, host), "allow host");
    {
        char* h = (char*)host;
        const void* src[7] = {objects, tris, groups, NULL, seeds, camera256, NULL};
        size_t o = 0;
        for (int i = 0; i < 7; i++) {
            if (src[i]) memcpy(h + o, src[i], sz[i]);
            else memset(h + o, 0, sz[i]);
            o += sz[i];
        }
    }
    CHK(hsa_signal_create(1, 0, NULL, &sig), "signal");
    {
        size_t o = 0;
        for (int i = 0; i < 7; i++) {
            hsa_signal_store_relaxed(sig, 1);
            CHK(hsa_amd_memory_async_copy(dev[i], af.gpu, (char*)host + o, af.cpu, sz[i], 0, NULL, sig),
                "h2d copy");
            hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
            o += sz[i];
        }
    }
    /* printf buffer (tracer.cl printf at fixed pixels): {u32 offset, u32 size, data} (ockl __printf_alloc). */
    const uint32_t pf_size = 1u << 20;
    CHK(hsa_amd_memory_pool_allocate(kp.pool, pf_size, 0, &printf_buf), "printf alloc");
    CHK(hsa_amd_agents_allow_access(1, &af.gpu, NULL, printf_buf), "allow printf");
    memset(printf_buf, 0, pf_size);
    ((uint32_t*)printf_buf)[1] = pf_size - 8;

    CHK(hsa_amd_memory_pool_allocate(kp.pool, kseg < 512 ? 512 : kseg, 0, &karg), "kernarg alloc");
    CHK(hsa_amd_agents_allow_access(1, &af.gpu, NULL, karg), "allow kernarg");
    memset(karg, 0, kseg);
    {
        char* k = (char*)karg;
#define PUT(off, T, v) do { if ((off) >= 0) { T v_ = (T)(v); memcpy(k + (off), &v_, sizeof v_); } } while (0)
        PUT(L.objects, uint64_t, (uintptr_t)dev[0]);
        PUT(L.num_objects, uint32_t, n_obj);
        PUT(L.triangles, uint64_t, (uintptr_t)dev[1]);
        PUT(L.groups, uint64_t, (uintptr_t)dev[2]);
        PUT(L.output, uint64_t, (uintptr_t)dev[3]);
        PUT(L.seeds, uint64_t, (uintptr_t)dev[4]);
        PUT(L.samples, uint32_t, samples);
        PUT(L.camera, uint64_t, (uintptr_t)dev[5]);
        PUT(L.y_offset, uint32_t, 0);
        PUT(L.img0, uint64_t, (uintptr_t)dev[6]);
        PUT(L.img1, uint64_t, (uintptr_t)dev[6] + 64);
        PUT(L.img2, uint64_t, (uintptr_t)dev[6] + 128);
        PUT(L.block_count_x, uint32_t, n_pixels / wg_size);
        PUT(L.block_count_y, uint32_t, 1);
        PUT(L.block_count_z, uint32_t, 1);
        PUT(L.group_size_x, uint16_t, wg_size);
        PUT(L.group_size_y, uint16_t, 1);
        PUT(L.group_size_z, uint16_t, 1);
        PUT(L.grid_dims, uint16_t, 1);
        PUT(L.printf_buffer, uint64_t, (uintptr_t)printf_buf);
#undef PUT
    }

    CHK(hsa_queue_create(af.gpu, 1024, HSA_QUEUE_TYPE_SINGLE, NULL, NULL, UINT32_MAX, UINT32_MAX, &q),
        "queue create");
    {
        hsa_signal_store_relaxed(sig, 1);
        uint64_t idx = hsa_queue_add_write_index_relaxed(q, 1);
        hsa_kernel_dispatch_packet_t* pkt =
            (hsa_kernel_dispatch_packet_t*)q->base_address + (idx & (q->size - 1));
        memset((char*)pkt + 4, 0, sizeof(*pkt) - 4);
        pkt->workgroup_size_x = (uint16_t)wg_size;
        pkt->workgroup_size_y = 1;
        pkt->workgroup_size_z = 1;
        pkt->grid_size_x = n_pixels;
        pkt->grid_size_y = 1;
        pkt->grid_size_z = 1;
        pkt->private_segment_size = pseg;
        pkt->group_segment_size = gseg;
        pkt->kernel_object = kobj;
        pkt->kernarg_address = karg;
        pkt->completion_signal = sig;
        uint16_t setup = 1 << HSA_KERNEL_DISPATCH_PACKET_SETUP_DIMENSIONS;
        uint16_t header = (HSA_PACKET_TYPE_KERNEL_DISPATCH << HSA_PACKET_HEADER_TYPE) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCACQUIRE_FENCE_SCOPE) |
                          (HSA_FENCE_SCOPE_SYSTEM << HSA_PACKET_HEADER_SCRELEASE_FENCE_SCOPE);
        __atomic_store_n((uint32_t*)pkt, (uint32_t)header | ((uint32_t)setup << 16), __ATOMIC_RELEASE);
        hsa_signal_store_screlease(q->doorbell_signal, (hsa_signal_value_t)idx);
        struct timespec t0, t1;
        clock_gettime(CLOCK_MONOTONIC, &t0);
        for (;;) {
            hsa_signal_value_t v = hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1,
                                                             100000000ull, HSA_WAIT_STATE_BLOCKED);
            if (v < 1) break;
            clock_gettime(CLOCK_MONOTONIC, &t1);
            double el = (t1.tv_sec - t0.tv_sec) + 1e-9 * (t1.tv_nsec - t0.tv_nsec);
            if (timeout_s > 0 && el > timeout_s) {
                seterr(err, err_len, "reference kernel did not finish within %.1f s", timeout_s);
                fflush(stderr);
                /* The dispatch cannot be cancelled; the caller must end the process. */
                return -4;
            }
        }
    }
    {
        size_t out_off = sz[0] + sz[1] + sz[2];
        hsa_signal_store_relaxed(sig, 1);
        CHK(hsa_amd_memory_async_copy((char*)host + out_off, af.cpu, dev[3], af.gpu, sz[3], 0, NULL, sig),
            "d2h copy");
        hsa_signal_wait_scacquire(sig, HSA_SIGNAL_CONDITION_LT, 1, UINT64_MAX, HSA_WAIT_STATE_BLOCKED);
        memcpy(out_rgba, (char*)host + out_off, sz[3]);
    }
out:
    if (q) hsa_queue_destroy(q);
    if (sig.handle) hsa_signal_destroy(sig);
    if (exe.handle) hsa_executable_destroy(exe);
    if (rdr.handle) hsa_code_object_reader_destroy(rdr);
    for (int i = 0; i < 8; i++)
        if (dev[i]) hsa_amd_memory_pool_free(dev[i]);
    if (host) hsa_amd_memory_pool_free(host);
    if (karg) hsa_amd_memory_pool_free(karg);
    if (printf_buf) hsa_amd_memory_pool_free(printf_buf);
    free(code);
    /* hsa_init() is reference counted; the runtime is left up (a HIP runtime in the
     * same process shares it). */
    (void)inited;
    return rc;
}
