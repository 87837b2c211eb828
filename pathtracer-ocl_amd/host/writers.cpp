// writers.cpp -- the reference's output writers:
//   PNG: writeDataToPNG + clamp (internal/app/tracer/pathtracer.go:40-59): each
//        channel -> uint8(clamp(math.Round(v * 255), 0, 255)), alpha 255, 8-bit RGBA;
//   raw: WriteRawImage (internal/app/raw/writer.go:11-35): big-endian int32
//        1, 0, width, height, then big-endian float32 R, G, B per pixel.
// The PNG pixel data equals Go's image.RGBA; the container bytes (zlib level,
// filters) are this encoder's own, as any PNG decoder sees the same pixels.
#include <zlib.h>

#include <cmath>
#include <cstdio>
#include <cstring>
#include <string>
#include <vector>

#include "../../include/ptmi.h"
#include "../../include/ptmi_host.h"

namespace {

void set_err(char* err, size_t len, const std::string& msg) {
    if (err && len) std::snprintf(err, len, "%s", msg.c_str());
}

// clamp (pathtracer.go:50-59); math.Round rounds half away from zero == std::round.
uint8_t clamp8(double v) {
    double r = std::round(v * 255.0);
    if (r > 255.0)
        r = 255.0;
    else if (r < 0.0)
        r = 0.0;
    return (uint8_t)r;  // NaN: Go's uint8(NaN) is implementation-defined; 0 here
}

void be32(std::vector<uint8_t>& b, uint32_t v) {
    b.push_back((uint8_t)(v >> 24));
    b.push_back((uint8_t)(v >> 16));
    b.push_back((uint8_t)(v >> 8));
    b.push_back((uint8_t)v);
}

void chunk(std::vector<uint8_t>& out, const char* type, const std::vector<uint8_t>& data) {
    be32(out, (uint32_t)data.size());
    const size_t start = out.size();
    out.insert(out.end(), type, type + 4);
    out.insert(out.end(), data.begin(), data.end());
    const uint32_t crc = (uint32_t)crc32(0L, out.data() + start, (uInt)(out.size() - start));
    be32(out, crc);
}

int write_file(const char* path, const std::vector<uint8_t>& bytes, char* err, size_t err_len) {
    FILE* f = std::fopen(path, "wb");
    if (!f) {
        set_err(err, err_len, std::string("cannot open ") + path);
        return PTMI_ERR_ARG;
    }
    const size_t n = std::fwrite(bytes.data(), 1, bytes.size(), f);
    const int rc = std::fclose(f);
    if (n != bytes.size() || rc != 0) {
        set_err(err, err_len, std::string("write failed: ") + path);
        return PTMI_ERR_ARG;
    }
    return PTMI_OK;
}

}  // namespace

extern "C" int ptmi_host_write_png(const char* path, const double* rgba, int width, int height, char* err,
                                   size_t err_len) {
    if (!path || !rgba || width <= 0 || height <= 0) {
        set_err(err, err_len, "ptmi_host_write_png: bad arguments");
        return PTMI_ERR_ARG;
    }
    // Scanlines with filter byte 0 (None).
    std::vector<uint8_t> raw;
    raw.reserve((size_t)height * ((size_t)width * 4 + 1));
    for (int y = 0; y < height; y++) {
        raw.push_back(0);
        for (int x = 0; x < width; x++) {
            const double* p = rgba + ((size_t)y * width + x) * 4;
            raw.push_back(clamp8(p[0]));
            raw.push_back(clamp8(p[1]));
            raw.push_back(clamp8(p[2]));
            raw.push_back(255);
        }
    }
    uLongf zlen = compressBound((uLong)raw.size());
    std::vector<uint8_t> z(zlen);
    if (compress2(z.data(), &zlen, raw.data(), (uLong)raw.size(), Z_DEFAULT_COMPRESSION) != Z_OK) {
        set_err(err, err_len, "zlib compression failed");
        return PTMI_ERR_NOMEM;
    }
    z.resize(zlen);
    std::vector<uint8_t> out = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    std::vector<uint8_t> ihdr;
    be32(ihdr, (uint32_t)width);
    be32(ihdr, (uint32_t)height);
    ihdr.insert(ihdr.end(), {8, 6, 0, 0, 0});  // 8-bit, RGBA, deflate, adaptive filtering, no interlace
    chunk(out, "IHDR", ihdr);
    chunk(out, "IDAT", z);
    chunk(out, "IEND", {});
    return write_file(path, out, err, err_len);
}

extern "C" int ptmi_host_write_raw(const char* path, const double* rgba, int width, int height, char* err,
                                   size_t err_len) {
    if (!path || !rgba || width <= 0 || height <= 0) {
        set_err(err, err_len, "ptmi_host_write_raw: bad arguments");
        return PTMI_ERR_ARG;
    }
    std::vector<uint8_t> out;
    out.reserve(16 + (size_t)width * height * 12);
    be32(out, 1);  // fileFormatVersionMajor
    be32(out, 0);  // fileFormatVersionMinor
    be32(out, (uint32_t)width);
    be32(out, (uint32_t)height);
    const size_t n = (size_t)width * height;
    for (size_t i = 0; i < n; i++)
        for (int c = 0; c < 3; c++) {
            const float f = (float)rgba[i * 4 + c];  // float32(indata[i]) (raw/writer.go:15-17)
            uint32_t u;
            std::memcpy(&u, &f, 4);
            be32(out, u);
        }
    return write_file(path, out, err, err_len);
}
