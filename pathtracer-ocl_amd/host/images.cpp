// images.cpp -- texture images for the textured scenes, as the reference loads them:
//   LoadImage (internal/app/scenes/scene.go:30-56): png.Decode, then -- unless the
//   result already is an *image.NRGBA -- draw.Draw(NRGBA, Src), i.e. every pixel
//   through color.NRGBAModel (Go 1.19 image/color, image/draw generic path);
//   prepareTextures (internal/ocl/ocltracer.go:228-254): one RGBA UNORM8 array per
//   list, width/height of the first image, the Pix bytes of all images concatenated.
//
// PNG decoding follows Go's image/png reader: colour types 0/2/3/4/6, bit depths
// 1-16, tRNS (palette alpha, gray/RGB colour keys), Adam7 interlacing, the five
// scanline filters.  JPEG decoding (image/jpeg) is NOT restated: a .jpg/.jpeg
// asset is read from a PNG of the same stem when one exists, else the call fails.
#include <zlib.h>

#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/ptmi.h"
#include "../../include/ptmi_host.h"

namespace {

void set_err(char* err, size_t len, const std::string& msg) {
    if (err && len) std::snprintf(err, len, "%s", msg.c_str());
}

uint32_t rd_be32(const uint8_t* p) { return (uint32_t)p[0] << 24 | (uint32_t)p[1] << 16 | (uint32_t)p[2] << 8 | p[3]; }

// color.NRGBAModel applied to a premultiplied 16-bit colour (image/color/color.go).
void nrgba_from_premul(uint32_t r, uint32_t g, uint32_t b, uint32_t a, uint8_t* o) {
    if (a == 0xffff) {
        o[0] = (uint8_t)(r >> 8), o[1] = (uint8_t)(g >> 8), o[2] = (uint8_t)(b >> 8), o[3] = 0xff;
    } else if (a == 0) {
        o[0] = o[1] = o[2] = o[3] = 0;
    } else {
        o[0] = (uint8_t)(((r * 0xffff) / a) >> 8);
        o[1] = (uint8_t)(((g * 0xffff) / a) >> 8);
        o[2] = (uint8_t)(((b * 0xffff) / a) >> 8);
        o[3] = (uint8_t)(a >> 8);
    }
}
// color.NRGBA.RGBA() then the model (the draw.Draw round trip of an 8-bit NRGBA pixel).
void nrgba8_roundtrip(uint8_t R, uint8_t G, uint8_t B, uint8_t A, uint8_t* o) {
    auto ch = [&](uint32_t c) {
        c |= c << 8;
        c *= A;
        return c / 0xff;
    };
    nrgba_from_premul(ch(R), ch(G), ch(B), (uint32_t)A | (uint32_t)A << 8, o);
}
// color.NRGBA64.RGBA() then the model.
void nrgba16_roundtrip(uint32_t R, uint32_t G, uint32_t B, uint32_t A, uint8_t* o) {
    nrgba_from_premul(R * A / 0xffff, G * A / 0xffff, B * A / 0xffff, A, o);
}

struct Png {
    uint32_t w = 0, h = 0;
    int depth = 0, ctype = 0, interlace = 0;
    std::vector<uint8_t> palette;  // RGBA per entry (tRNS applied)
    bool has_trns = false;
    uint16_t trns[3] = {0, 0, 0};  // gray or RGB colour key (at the image's bit depth)
    std::vector<uint8_t> idat;
};

int channels(int ctype) { return ctype == 0 ? 1 : ctype == 2 ? 3 : ctype == 3 ? 1 : ctype == 4 ? 2 : 4; }

uint8_t paeth(uint8_t a, uint8_t b, uint8_t c) {
    const int p = (int)a + b - c, pa = std::abs(p - a), pb = std::abs(p - b), pc = std::abs(p - c);
    return (pa <= pb && pa <= pc) ? a : (pb <= pc ? b : c);
}

// Unfilter one pass of `pw x ph` pixels starting at raw[pos]; returns the rows.
std::vector<uint8_t> unfilter(const std::vector<uint8_t>& raw, size_t& pos, uint32_t pw, uint32_t ph, int bpp_bits) {
    const size_t row = ((size_t)pw * bpp_bits + 7) / 8;
    const size_t bpp = (size_t)((bpp_bits + 7) / 8);
    std::vector<uint8_t> out(row * ph);
    std::vector<uint8_t> prev(row, 0);
    for (uint32_t y = 0; y < ph; y++) {
        if (pos + 1 + row > raw.size()) throw std::runtime_error("png: truncated image data");
        const uint8_t f = raw[pos++];
        uint8_t* cur = out.data() + (size_t)y * row;
        std::memcpy(cur, raw.data() + pos, row);
        pos += row;
        for (size_t i = 0; i < row; i++) {
            const uint8_t a = i >= bpp ? cur[i - bpp] : 0, b = prev[i], c = i >= bpp ? prev[i - bpp] : 0;
            switch (f) {
                case 0: break;
                case 1: cur[i] = (uint8_t)(cur[i] + a); break;
                case 2: cur[i] = (uint8_t)(cur[i] + b); break;
                case 3: cur[i] = (uint8_t)(cur[i] + (uint8_t)(((int)a + b) / 2)); break;
                case 4: cur[i] = (uint8_t)(cur[i] + paeth(a, b, c)); break;
                default: throw std::runtime_error("png: bad filter type");
            }
        }
        std::memcpy(prev.data(), cur, row);
    }
    return out;
}

// Pixel (x) of an unfiltered row -> NRGBA8 as LoadImage ends up with it.
void convert_pixel(const Png& P, const uint8_t* row, uint32_t x, uint8_t* o) {
    const int d = P.depth;
    auto sample16 = [&](int ch) -> uint32_t {  // 16-bit sample ch of pixel x
        const uint8_t* p = row + ((size_t)x * channels(P.ctype) + ch) * 2;
        return (uint32_t)p[0] << 8 | p[1];
    };
    if (P.ctype == 0) {
        uint32_t y;
        if (d == 16) {
            y = sample16(0);
            if (P.has_trns && y == P.trns[0]) return nrgba16_roundtrip(y, y, y, 0, o);
            return nrgba_from_premul(y, y, y, 0xffff, o);
        }
        const uint32_t raw = (row[(size_t)x * d / 8] >> (8 - d - (int)((size_t)x * d % 8))) & ((1u << d) - 1);
        y = d == 8 ? raw : d == 4 ? raw * 0x11 : d == 2 ? raw * 0x55 : raw * 0xff;
        if (P.has_trns && raw == P.trns[0]) {  // Go: NRGBA with alpha 0 (the colour kept)
            o[0] = o[1] = o[2] = (uint8_t)y, o[3] = 0;
            return;
        }
        o[0] = o[1] = o[2] = (uint8_t)y, o[3] = 0xff;
    } else if (P.ctype == 2) {
        if (d == 16) {
            const uint32_t r = sample16(0), g = sample16(1), b = sample16(2);
            if (P.has_trns && r == P.trns[0] && g == P.trns[1] && b == P.trns[2])
                return nrgba16_roundtrip(r, g, b, 0, o);
            return nrgba_from_premul(r, g, b, 0xffff, o);
        }
        const uint8_t* p = row + (size_t)x * 3;
        o[0] = p[0], o[1] = p[1], o[2] = p[2];
        o[3] = (P.has_trns && p[0] == P.trns[0] && p[1] == P.trns[1] && p[2] == P.trns[2]) ? 0 : 0xff;
    } else if (P.ctype == 3) {
        const uint32_t idx = (row[(size_t)x * d / 8] >> (8 - d - (int)((size_t)x * d % 8))) & ((1u << d) - 1);
        uint8_t c[4] = {0, 0, 0, 0xff};  // beyond the palette: opaque black (png/reader.go)
        if ((size_t)idx * 4 < P.palette.size()) std::memcpy(c, P.palette.data() + (size_t)idx * 4, 4);
        nrgba8_roundtrip(c[0], c[1], c[2], c[3], o);
    } else if (P.ctype == 4) {
        if (d == 16) return nrgba16_roundtrip(sample16(0), sample16(0), sample16(0), sample16(1), o);
        const uint8_t* p = row + (size_t)x * 2;  // decoded as *image.NRGBA: returned as is
        o[0] = o[1] = o[2] = p[0], o[3] = p[1];
    } else {
        if (d == 16) return nrgba16_roundtrip(sample16(0), sample16(1), sample16(2), sample16(3), o);
        std::memcpy(o, row + (size_t)x * 4, 4);  // already *image.NRGBA: returned as decoded
    }
}

std::vector<uint8_t> decode_png(const std::vector<uint8_t>& f, uint32_t& W, uint32_t& H) {
    static const uint8_t sig[8] = {0x89, 'P', 'N', 'G', '\r', '\n', 0x1a, '\n'};
    if (f.size() < 8 || std::memcmp(f.data(), sig, 8) != 0) throw std::runtime_error("png: not a PNG file");
    Png P;
    size_t pos = 8;
    bool seen_end = false;
    while (pos + 12 <= f.size() && !seen_end) {
        const uint32_t n = rd_be32(f.data() + pos);
        if (pos + 12 + (size_t)n > f.size()) throw std::runtime_error("png: truncated chunk");
        const std::string type((const char*)f.data() + pos + 4, 4);
        const uint8_t* b = f.data() + pos + 8;
        if ((uint32_t)crc32(crc32(0L, nullptr, 0), f.data() + pos + 4, n + 4) != rd_be32(b + n))
            throw std::runtime_error("png: bad CRC in " + type);
        if (type == "IHDR") {
            if (n != 13) throw std::runtime_error("png: bad IHDR");
            P.w = rd_be32(b), P.h = rd_be32(b + 4), P.depth = b[8], P.ctype = b[9], P.interlace = b[12];
            if (b[10] != 0 || b[11] != 0 || P.interlace > 1) throw std::runtime_error("png: unsupported method");
        } else if (type == "PLTE") {
            P.palette.assign((size_t)(n / 3) * 4, 0xff);
            for (uint32_t i = 0; i < n / 3; i++) std::memcpy(&P.palette[(size_t)i * 4], b + 3 * i, 3);
        } else if (type == "tRNS") {
            if (P.ctype == 3) {
                for (uint32_t i = 0; i < n && (size_t)i * 4 + 3 < P.palette.size(); i++) P.palette[(size_t)i * 4 + 3] = b[i];
            } else if (P.ctype == 0 && n >= 2) {
                P.has_trns = true, P.trns[0] = (uint16_t)(b[0] << 8 | b[1]);
            } else if (P.ctype == 2 && n >= 6) {
                P.has_trns = true;
                for (int k = 0; k < 3; k++) P.trns[k] = (uint16_t)(b[2 * k] << 8 | b[2 * k + 1]);
            }
        } else if (type == "IDAT") {
            P.idat.insert(P.idat.end(), b, b + n);
        } else if (type == "IEND") {
            seen_end = true;
        }
        pos += 12 + (size_t)n;
    }
    const int d = P.depth, ct = P.ctype;
    const bool ok = (ct == 0 && (d == 1 || d == 2 || d == 4 || d == 8 || d == 16)) ||
                    (ct == 3 && (d == 1 || d == 2 || d == 4 || d == 8)) ||
                    ((ct == 2 || ct == 4 || ct == 6) && (d == 8 || d == 16));
    if (!ok || P.w == 0 || P.h == 0 || P.w > (1u << 16) || P.h > (1u << 16))
        throw std::runtime_error("png: unsupported colour type / bit depth / size");
    if (ct == 3 && P.palette.empty()) throw std::runtime_error("png: paletted image without PLTE");
    // inflate the zlib stream
    std::vector<uint8_t> raw;
    z_stream zs{};
    if (inflateInit(&zs) != Z_OK) throw std::runtime_error("png: inflateInit failed");
    zs.next_in = P.idat.data();
    zs.avail_in = (uInt)P.idat.size();
    std::vector<uint8_t> buf(1 << 16);
    int zr;
    do {
        zs.next_out = buf.data();
        zs.avail_out = (uInt)buf.size();
        zr = inflate(&zs, Z_NO_FLUSH);
        if (zr != Z_OK && zr != Z_STREAM_END) {
            inflateEnd(&zs);
            throw std::runtime_error("png: corrupt image data");
        }
        raw.insert(raw.end(), buf.data(), buf.data() + (buf.size() - zs.avail_out));
    } while (zr != Z_STREAM_END && (zs.avail_in > 0 || zs.avail_out == 0));
    inflateEnd(&zs);
    const int bpp_bits = channels(ct) * d;
    W = P.w, H = P.h;
    std::vector<uint8_t> out((size_t)W * H * 4);
    size_t rpos = 0;
    if (!P.interlace) {
        const std::vector<uint8_t> rows = unfilter(raw, rpos, W, H, bpp_bits);
        const size_t stride = ((size_t)W * bpp_bits + 7) / 8;
        for (uint32_t y = 0; y < H; y++)
            for (uint32_t x = 0; x < W; x++) convert_pixel(P, rows.data() + y * stride, x, &out[((size_t)y * W + x) * 4]);
    } else {  // Adam7 (png/reader.go interlacing)
        static const int xo[7] = {0, 4, 0, 2, 0, 1, 0}, yo[7] = {0, 0, 4, 0, 2, 0, 1};
        static const int xf[7] = {8, 8, 4, 4, 2, 2, 1}, yf[7] = {8, 8, 8, 4, 4, 2, 2};
        for (int p = 0; p < 7; p++) {
            const uint32_t pw = (W - xo[p] + xf[p] - 1) / xf[p], ph = (H - yo[p] + yf[p] - 1) / yf[p];
            if (W <= (uint32_t)xo[p] || H <= (uint32_t)yo[p] || pw == 0 || ph == 0) continue;
            const std::vector<uint8_t> rows = unfilter(raw, rpos, pw, ph, bpp_bits);
            const size_t stride = ((size_t)pw * bpp_bits + 7) / 8;
            for (uint32_t y = 0; y < ph; y++)
                for (uint32_t x = 0; x < pw; x++) {
                    const size_t X = (size_t)xo[p] + (size_t)x * xf[p], Y = (size_t)yo[p] + (size_t)y * yf[p];
                    convert_pixel(P, rows.data() + y * stride, x, &out[(Y * W + X) * 4]);
                }
        }
    }
    return out;
}

std::vector<uint8_t> read_file(const std::string& path) {
    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot read " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    const std::string s = ss.str();
    return std::vector<uint8_t>(s.begin(), s.end());
}

bool ends_with(const std::string& s, const char* suf) {
    const size_t n = std::strlen(suf);
    return s.size() >= n && s.compare(s.size() - n, n, suf) == 0;
}

// LoadImage(path) -> NRGBA pixels (scene.go:30-56).
std::vector<uint8_t> load_image(const std::string& path, uint32_t& w, uint32_t& h) {
    if (ends_with(path, ".jpg") || ends_with(path, ".jpeg")) {
        const std::string png = path.substr(0, path.rfind('.')) + ".png";
        std::ifstream probe(png, std::ios::binary);
        if (!probe)
            throw std::runtime_error("JPEG decoding (image/jpeg) is not restated: " + path +
                                     " -- provide the same image as " + png);
        return decode_png(read_file(png), w, h);
    }
    if (!ends_with(path, ".png")) throw std::runtime_error("unsupported texture image format: " + path);
    return decode_png(read_file(path), w, h);
}

// The texture lists of the textured cmd/pt scenes (scene.go:19-27 fields).
struct SceneTex {
    const char* scene;
    std::vector<const char*> lists[3];
};
const std::vector<SceneTex>& scene_textures() {
    static const std::vector<SceneTex> t = {
        {"textures",  // texturedplanets.go:123-133
         {{"concrete_squares.png", "seamless-cobblestone-texture.jpg", "floor_boards.png", "concrete_squares_nm2.png"},
          {"planet.png", "jupiter2_6k_contrast.png"},
          {}}},
        {"envmap", {{}, {"alps_field_8k.png"}, {}}},        // envmap.go:54
        {"cubemap", {{}, {}, {"shrine_cubemap.jpeg"}}},    // cubemap.go:55
    };
    return t;
}

}  // namespace

extern "C" int ptmi_host_load_image(const char* path, uint8_t** nrgba, uint32_t* width, uint32_t* height, char* err,
                                    size_t err_len) {
    if (!path || !nrgba || !width || !height) {
        set_err(err, err_len, "ptmi_host_load_image: bad arguments");
        return PTMI_ERR_ARG;
    }
    *nrgba = nullptr;
    try {
        uint32_t w = 0, h = 0;
        const std::vector<uint8_t> px = load_image(path, w, h);
        uint8_t* p = (uint8_t*)std::malloc(px.size());
        if (!p) {
            set_err(err, err_len, "out of host memory");
            return PTMI_ERR_NOMEM;
        }
        std::memcpy(p, px.data(), px.size());
        *nrgba = p, *width = w, *height = h;
    } catch (const std::exception& e) {
        set_err(err, err_len, e.what());
        return PTMI_ERR_ARG;
    }
    return PTMI_OK;
}

extern "C" void ptmi_host_free_image(uint8_t* nrgba) { std::free(nrgba); }

extern "C" int ptmi_host_load_scene_textures(const char* name, const char* assets_dir, ptmi_textures* out,
                                             char* err, size_t err_len) {
    if (!name || !out) {
        set_err(err, err_len, "ptmi_host_load_scene_textures: bad arguments");
        return PTMI_ERR_ARG;
    }
    std::memset(out, 0, sizeof(*out));
    const std::string dir = assets_dir ? assets_dir : "assets";
    for (const SceneTex& st : scene_textures()) {
        if (std::strcmp(st.scene, name) != 0) continue;
        try {
            for (int k = 0; k < 3; k++) {
                const auto& files = st.lists[k];
                if (files.empty()) continue;
                // prepareTextures: size of the first image, Pix of all images concatenated;
                // a layer past the concatenated bytes is zero here (the reference would
                // read past its buffer).
                std::vector<uint8_t> all;
                uint32_t w0 = 0, h0 = 0;
                for (size_t i = 0; i < files.size(); i++) {
                    uint32_t w = 0, h = 0;
                    const std::vector<uint8_t> px = load_image(dir + "/" + files[i], w, h);
                    if (i == 0) w0 = w, h0 = h;
                    all.insert(all.end(), px.begin(), px.end());
                }
                const size_t bytes = (size_t)w0 * h0 * 4 * files.size();
                all.resize(bytes, 0);
                uint8_t* p = (uint8_t*)std::malloc(bytes);
                if (!p) throw std::runtime_error("out of host memory");
                std::memcpy(p, all.data(), bytes);
                out->pixels[k] = p;
                out->width[k] = w0, out->height[k] = h0, out->count[k] = (uint32_t)files.size();
            }
        } catch (const std::exception& e) {
            ptmi_host_free_textures(out);
            set_err(err, err_len, std::string("scene '") + name + "' textures: " + e.what());
            return PTMI_ERR_ARG;
        }
    }
    return PTMI_OK;
}

extern "C" void ptmi_host_free_textures(ptmi_textures* t) {
    if (!t) return;
    for (int k = 0; k < 3; k++) {
        std::free((void*)t->pixels[k]);
        t->pixels[k] = nullptr;
        t->width[k] = t->height[k] = t->count[k] = 0;
    }
}
