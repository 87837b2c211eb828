// pt.cpp -- Go-free counterpart of the reference CLI (cmd/pt/main.go): builds a
// named scene natively (libptmi_host.so), renders it through the drop-in
// boundary ptmi_trace (libptmi.so, MI355X) and writes the PNG the reference
// writes (tracer/pathtracer.go:17-38, "out-<samples>-<W>x<H>.png").
//
// Flags as cmd/pt/main.go:47-56 (same names and defaults):
//   --width 640 --height 480 --samples 1 --aperture 0 --focal-length 0
//   --scene gopher --device-index 0 --list-devices --list-scenes
// plus: --assets DIR (OBJ/MTL directory, default ./assets as the reference reads
// them), --out FILE.png, --raw FILE.raw (raw/writer.go format), --gpus N and
// --split sample|tile (ptmi_trace_multi over devices 0..N-1), --seed N
// (per-pixel seeds from a fixed stream; default: time-seeded like Go's
// rand.Float64 per pixel, ocltracer.go:260-263).
// An unknown --scene renders the OCL scene, as main.go:86-88 does.
#include <chrono>
#include <cstdint>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ptmi.h"
#include "../../include/ptmi_host.h"

namespace {

struct Cfg {
    int width = 640, height = 480, samples = 1, device_index = 0;
    double aperture = 0.0, focal_length = 0.0;
    std::string scene = "gopher", assets = "assets", out, raw, split = "sample";
    int gpus = 1;
    bool list_devices = false, list_scenes = false, have_seed = false;
    uint64_t seed = 0;
};

[[noreturn]] void usage(const char* msg) {
    std::fprintf(stderr,
                 "%s\nusage: pt [--width N] [--height N] [--samples N] [--aperture F] [--focal-length F]\n"
                 "          [--scene NAME] [--device-index N] [--list-devices] [--list-scenes]\n"
                 "          [--assets DIR] [--out FILE.png] [--raw FILE.raw] [--gpus N] [--split sample|tile]\n"
                 "          [--seed N]\n",
                 msg);
    std::exit(2);
}

Cfg parse(int argc, char** argv) {
    Cfg c;
    for (int i = 1; i < argc; i++) {
        std::string a = argv[i], v;
        const size_t eq = a.find('=');
        bool inl = false;
        if (a.rfind("--", 0) == 0 && eq != std::string::npos) {
            v = a.substr(eq + 1);
            a = a.substr(0, eq);
            inl = true;
        }
        auto val = [&]() -> std::string {
            if (inl) return v;
            if (i + 1 >= argc) usage(("missing value for " + a).c_str());
            return argv[++i];
        };
        if (a == "--width") c.width = std::atoi(val().c_str());
        else if (a == "--height") c.height = std::atoi(val().c_str());
        else if (a == "--samples") c.samples = std::atoi(val().c_str());
        else if (a == "--aperture") c.aperture = std::atof(val().c_str());
        else if (a == "--focal-length") c.focal_length = std::atof(val().c_str());
        else if (a == "--scene") c.scene = val();
        else if (a == "--device-index") c.device_index = std::atoi(val().c_str());
        else if (a == "--list-devices") c.list_devices = true;
        else if (a == "--list-scenes") c.list_scenes = true;
        else if (a == "--assets") c.assets = val();
        else if (a == "--out") c.out = val();
        else if (a == "--raw") c.raw = val();
        else if (a == "--gpus") c.gpus = std::atoi(val().c_str());
        else if (a == "--split") c.split = val();
        else if (a == "--seed") c.seed = std::strtoull(val().c_str(), nullptr, 10), c.have_seed = true;
        else usage(("unknown flag " + a).c_str());
    }
    if (c.width <= 0 || c.height <= 0 || c.samples <= 0) usage("width, height and samples must be positive");
    if (c.gpus <= 0 || (c.split != "sample" && c.split != "tile")) usage("--gpus must be >= 1, --split sample|tile");
    return c;
}

bool known_scene(const std::string& s) {
    const std::string names = ptmi_host_scene_names();
    size_t a = 0;
    while (a < names.size()) {
        const size_t b = names.find('\n', a);
        if (names.compare(a, b - a, s) == 0 && b - a == s.size()) return true;
        a = b + 1;
    }
    return false;
}

}  // namespace

int main(int argc, char** argv) {
    const Cfg c = parse(argc, argv);
    char err[512] = {0};
    if (c.list_devices) {  // main.go:98-112
        const int n = ptmi_device_count();
        for (int i = 0; i < n; i++) {
            char name[256];
            if (ptmi_device_name(i, name, sizeof(name)) == PTMI_OK)
                std::printf("Index: %d Type: GPU Name: %s\n", i, name);
        }
        return 0;
    }
    if (c.list_scenes) {
        std::fputs(ptmi_host_scene_names(), stdout);
        return 0;
    }
    const std::string scene = known_scene(c.scene) ? c.scene : "default";
    const auto t0 = std::chrono::steady_clock::now();
    ptmi_records r;
    int rc = ptmi_host_build_scene(scene.c_str(), c.width, c.height, c.aperture, c.focal_length, c.assets.c_str(),
                                   &r, err, sizeof(err));
    if (rc) {
        std::fprintf(stderr, "scene build failed (%d): %s\n", rc, err);
        return 1;
    }
    ptmi_textures tex;  // the scene's texture arrays (texturedplanets / envmap / cubemap)
    if ((rc = ptmi_host_load_scene_textures(scene.c_str(), c.assets.c_str(), &tex, err, sizeof(err)))) {
        ptmi_host_free_records(&r);
        std::fprintf(stderr, "%s\n", err);  // the reference: LoadImage panics
        return 1;
    }
    const bool textured = tex.count[0] || tex.count[1] || tex.count[2];
    const auto t1 = std::chrono::steady_clock::now();
    const size_t n = (size_t)c.width * c.height;
    std::vector<double> out(n * 4);
    const uint64_t stream =
        c.have_seed ? c.seed : (uint64_t)std::chrono::system_clock::now().time_since_epoch().count();
    ptmi_multi_timing mt{};
    if (c.gpus == 1) {
        rc = ptmi_trace(r.objects, r.n_obj, r.triangles, r.n_tri, r.groups, r.n_grp, c.device_index,
                        (uint32_t)c.samples, r.camera, nullptr, stream, textured ? &tex : nullptr, out.data(), err,
                        sizeof(err));
    } else {
        std::vector<int> devs(c.gpus);
        for (int d = 0; d < c.gpus; d++) devs[d] = d;
        rc = ptmi_trace_multi_timed(r.objects, r.n_obj, r.triangles, r.n_tri, r.groups, r.n_grp, devs.data(),
                                    (uint32_t)c.gpus, c.split == "tile" ? 1 : 0, (uint32_t)c.samples, r.camera,
                                    nullptr, stream, textured ? &tex : nullptr, out.data(), &mt, err, sizeof(err));
    }
    ptmi_host_free_records(&r);
    ptmi_host_free_textures(&tex);
    if (rc) {
        std::fprintf(stderr, "ptmi_trace failed (%d): %s\n", rc, err);  // the reference: logrus.Fatalf
        return 1;
    }
    const auto t2 = std::chrono::steady_clock::now();
    const std::string png = c.out.empty() ? "out-" + std::to_string(c.samples) + "-" + std::to_string(c.width) + "x" +
                                                std::to_string(c.height) + ".png"
                                          : c.out;
    if ((rc = ptmi_host_write_png(png.c_str(), out.data(), c.width, c.height, err, sizeof(err)))) {
        std::fprintf(stderr, "%s\n", err);
        return 1;
    }
    if (!c.raw.empty() && (rc = ptmi_host_write_raw(c.raw.c_str(), out.data(), c.width, c.height, err, sizeof(err)))) {
        std::fprintf(stderr, "%s\n", err);
        return 1;
    }
    const double build_s = std::chrono::duration<double>(t1 - t0).count();
    const double trace_s = std::chrono::duration<double>(t2 - t1).count();
    std::fprintf(stderr, "scene %s built in %.3f s; %dx%d x %d spp traced in %.3f s (%.1f Msamples/s); wrote %s\n",
                 scene.c_str(), build_s, c.width, c.height, c.samples, trace_s,
                 (double)n * c.samples / trace_s / 1e6, png.c_str());
    if (c.gpus > 1)
        std::fprintf(stderr,
                     "%d GPUs (%s split): prepare %.3f ms, render %.3f ms, combine %.3f ms, read-back %.3f ms\n",
                     c.gpus, c.split.c_str(), mt.prepare_ms, mt.render_ms, mt.combine_ms, mt.readback_ms);
    return 0;
}
