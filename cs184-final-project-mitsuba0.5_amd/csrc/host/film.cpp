/*
 * film.cpp -- develop the accumulated ImageBlock (R, G, B, W per pixel) into
 * the output image the way the reference's films do, and write it.
 *
 *   ldrfilm (src/films/ldrfilm.cpp:132-190, 300-351): optional Reinhard
 *     tonemapping (bitmap.cpp:1711-1852), exposure multiplier 2^exposure,
 *     gamma / sRGB curve, 8-bit rounding (fmtconv.cpp:1093-1160), banner,
 *     PNG.  JPEG output is refused (no encoder on the path).
 *   hdrfilm (src/films/hdrfilm.cpp:205-340, 480-537): float16 / float32 /
 *     uint32 components, banner at 1024, OpenEXR (uncompressed scanlines),
 *     RGBE (run-length encoded like bitmap.cpp:3504-3570, 3691-3750) or PFM
 *     (bitmap.cpp:3816-3850).
 *
 * The ImageBlock keeps no alpha channel on this path (every shipped scene
 * asks for rgb), so alpha pixel formats are rejected when the film is parsed.
 * Metadata / log attachments of the reference writers are not reproduced.
 */
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>

#include "host_scene.h"

namespace hpt {

namespace {

std::string lower(std::string s) {
    for (auto &ch : s) ch = (char) std::tolower((unsigned char) ch);
    return s;
}

/* fmtconv.cpp:1104-1111 */
float applyGamma(float value, float invGamma) {
    if (invGamma == -1)
        return (value <= 0.0031308f) ? 12.92f * value : 1.055f * std::pow(value, (float) (1.0 / 2.4)) - 0.055f;
    return std::pow(value, invGamma);
}

/* fmtconv.cpp:1135-1160 convertScalar<uint8_t>(float) */
uint8_t toU8(float value, float multiplier, float invGamma) {
    value *= multiplier;
    if (invGamma != 1) value = applyGamma(value, invGamma);
    return (uint8_t) std::min(255.0f, std::max(0.0f, value * 255.0f + 0.5f));
}

/* fmtconv.cpp:1158 clamps to (float) UINT32_MAX == 2^32 and casts (undefined
   for 2^32); saturate at UINT32_MAX instead */
uint32_t toU32(float value) {
    double v = std::min((float) 4294967295.0, std::max(0.0f, value * (float) 4294967295.0 + 0.5f));
    return v >= 4294967295.0 ? 4294967295u : (uint32_t) v;
}

/* bitmap.cpp:1711-1852, monochrome and RGB versions */
void tonemapReinhard(float *data, size_t pixels, int channels, float key, float burn) {
    float maxLuminance = 0, logAvgLuminance = 0;
    float *ptr = data;
    for (size_t i = 0; i < pixels; ++i) {
        float luminance = channels == 3 ? (float) (ptr[0] * 0.212671f + ptr[1] * 0.715160f + ptr[2] * 0.072169f)
                                        : ptr[0];
        if (luminance == 1024) maxLuminance = 0.0f;
        maxLuminance = std::max(maxLuminance, luminance);
        logAvgLuminance += (float) std::log((double) (1e-3f + luminance));
        ptr += channels;
    }
    logAvgLuminance = (float) std::exp((double) (logAvgLuminance / pixels));
    if (maxLuminance == 0) return;
    burn = std::min(1.0f, std::max(1e-8f, 1 - burn));
    float scale = key / logAvgLuminance, Lwhite = maxLuminance * scale;
    float invWp2 = 1 / (Lwhite * Lwhite * std::pow(burn, 4.0f));
    for (size_t i = 0; i < pixels; ++i, data += channels) {
        if (channels == 1) {
            float Lp = data[0] * scale;
            data[0] = Lp * (1.0f + Lp * invWp2) / (1.0f + Lp);
            continue;
        }
        float X = data[0] * 0.412453f + data[1] * 0.357580f + data[2] * 0.180423f;
        float Y = data[0] * 0.212671f + data[1] * 0.715160f + data[2] * 0.072169f;
        float Z = data[0] * 0.019334f + data[1] * 0.119193f + data[2] * 0.950227f;
        float normalization = 1 / (X + Y + Z), x = X * normalization, y = Y * normalization, Lp = Y * scale;
        Y = Lp * (1.0f + Lp * invWp2) / (1.0f + Lp);
        float ratio = Y / y;
        X = ratio * x;
        Z = ratio * (1.0f - x - y);
        data[0] = 3.240479f * X + -1.537150f * Y + -0.498535f * Z;
        data[1] = -0.969256f * X + 1.875991f * Y + 0.041556f * Z;
        data[2] = 0.055648f * X + -0.204043f * Y + 1.057311f * Z;
    }
}

bool loadBanner(const std::string &dataDir, std::vector<uint8_t> &mask, int &bw, int &bh) {
    bw = 108;
    bh = 5; /* data/film/banner.json (tools/extract_banner.py) */
    std::ifstream f(dataDir + "/film/banner.u8", std::ios::binary);
    if (!f) return false;
    mask.assign((size_t) bw * bh, 0);
    f.read((char *) mask.data(), (std::streamsize) mask.size());
    return (bool) f;
}

/* ---- PNG (stored deflate) ---- */
uint32_t crc32(const unsigned char *p, size_t n, uint32_t c = 0xffffffffu) {
    static uint32_t table[256];
    static bool init = false;
    if (!init) {
        for (uint32_t i = 0; i < 256; ++i) {
            uint32_t v = i;
            for (int k = 0; k < 8; ++k) v = (v & 1) ? 0xedb88320u ^ (v >> 1) : v >> 1;
            table[i] = v;
        }
        init = true;
    }
    for (size_t i = 0; i < n; ++i) c = table[(c ^ p[i]) & 0xff] ^ (c >> 8);
    return c;
}
void be32(std::vector<unsigned char> &v, uint32_t x) {
    v.push_back((unsigned char) (x >> 24));
    v.push_back((unsigned char) (x >> 16));
    v.push_back((unsigned char) (x >> 8));
    v.push_back((unsigned char) x);
}
void pngChunk(std::ofstream &f, const char *type, const std::vector<unsigned char> &data) {
    std::vector<unsigned char> buf;
    be32(buf, (uint32_t) data.size());
    std::vector<unsigned char> td(type, type + 4);
    td.insert(td.end(), data.begin(), data.end());
    buf.insert(buf.end(), td.begin(), td.end());
    be32(buf, crc32(td.data(), td.size()) ^ 0xffffffffu);
    f.write((const char *) buf.data(), (std::streamsize) buf.size());
}
bool writePNG(const std::string &path, const FilmImage &img) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    const unsigned char sig[8] = {137, 80, 78, 71, 13, 10, 26, 10};
    f.write((const char *) sig, 8);
    std::vector<unsigned char> ihdr;
    be32(ihdr, (uint32_t) img.width);
    be32(ihdr, (uint32_t) img.height);
    const unsigned char colorType = img.channels == 1 ? 0 : img.channels == 2 ? 4 : img.channels == 3 ? 2 : 6;
    ihdr.insert(ihdr.end(), {8, colorType, 0, 0, 0});
    pngChunk(f, "IHDR", ihdr);
    /* sRGB chunk like png_set_sRGB_gAMA_and_cHRM for gamma -1 is omitted: plain 8-bit data */
    const size_t row = (size_t) img.width * img.channels;
    std::vector<unsigned char> raw;
    raw.reserve((size_t) img.height * (row + 1));
    for (int y = 0; y < img.height; ++y) {
        raw.push_back(0);
        raw.insert(raw.end(), img.bytes.begin() + (size_t) y * row, img.bytes.begin() + (size_t) (y + 1) * row);
    }
    std::vector<unsigned char> z = {0x78, 0x01};
    uint32_t a = 1, b = 0;
    for (unsigned char c : raw) {
        a = (a + c) % 65521;
        b = (b + a) % 65521;
    }
    size_t pos = 0;
    do {
        size_t n = std::min((size_t) 65535, raw.size() - pos);
        bool last = pos + n >= raw.size();
        z.push_back(last ? 1 : 0);
        z.push_back((unsigned char) (n & 0xff));
        z.push_back((unsigned char) (n >> 8));
        z.push_back((unsigned char) (~n & 0xff));
        z.push_back((unsigned char) ((~n >> 8) & 0xff));
        z.insert(z.end(), raw.begin() + pos, raw.begin() + pos + n);
        pos += n;
    } while (pos < raw.size());
    be32(z, (b << 16) | a);
    pngChunk(f, "IDAT", z);
    pngChunk(f, "IEND", {});
    return (bool) f;
}

/* ---- PFM (bitmap.cpp:3816-3850): bottom row first, little endian ---- */
bool writePFMImage(const std::string &path, const FilmImage &img) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    f << 'P' << (img.channels == 3 ? 'F' : 'f') << '\n' << img.width << ' ' << img.height << '\n' << "-1" << '\n';
    const size_t row = (size_t) img.width * img.channels * 4;
    for (int y = img.height - 1; y >= 0; --y) f.write((const char *) img.bytes.data() + (size_t) y * row, (std::streamsize) row);
    return (bool) f;
}

/* ---- RGBE (bitmap.cpp:3504-3570, 3691-3750; Ward's run-length scheme) ---- */
void rgbeFromFloat(const float *d, uint8_t rgbe[4]) {
    float mx = std::max(std::max(d[0], d[1]), d[2]);
    if (mx < 1e-32) {
        rgbe[0] = rgbe[1] = rgbe[2] = rgbe[3] = 0;
    } else {
        int e;
        mx = std::frexp(mx, &e) * 256.0f / mx;
        rgbe[0] = (uint8_t) (d[0] * mx);
        rgbe[1] = (uint8_t) (d[1] * mx);
        rgbe[2] = (uint8_t) (d[2] * mx);
        rgbe[3] = (uint8_t) (e + 128);
    }
}
void rgbeRLE(std::ofstream &f, const uint8_t *data, int numbytes) {
    int cur = 0;
    uint8_t buf[2];
    while (cur < numbytes) {
        int begRun = cur, runCount = 0, oldRunCount = 0;
        while (runCount < 4 && begRun < numbytes) { /* next run of >= 4 equal bytes */
            begRun += runCount;
            oldRunCount = runCount;
            runCount = 1;
            while (begRun + runCount < numbytes && runCount < 127 && data[begRun] == data[begRun + runCount])
                runCount++;
        }
        if (oldRunCount > 1 && oldRunCount == begRun - cur) { /* short run before it */
            buf[0] = (uint8_t) (128 + oldRunCount);
            buf[1] = data[cur];
            f.write((const char *) buf, 2);
            cur = begRun;
        }
        while (cur < begRun) { /* literal bytes up to the run */
            int nonrun = std::min(128, begRun - cur);
            buf[0] = (uint8_t) nonrun;
            f.write((const char *) buf, 1);
            f.write((const char *) &data[cur], nonrun);
            cur += nonrun;
        }
        if (runCount >= 4) {
            buf[0] = (uint8_t) (128 + runCount);
            buf[1] = data[begRun];
            f.write((const char *) buf, 2);
            cur += runCount;
        }
    }
}
bool writeRGBEImage(const std::string &path, const FilmImage &img) {
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    f << "#?RGBE\n" << "FORMAT=32-bit_rle_rgbe\n\n" << "-Y " << img.height << " +X " << img.width << "\n";
    const float *data = (const float *) img.bytes.data();
    const int W = img.width;
    if (W < 8 || W > 0x7fff) {
        for (size_t i = 0; i < (size_t) W * img.height; ++i, data += 3) {
            uint8_t e[4];
            rgbeFromFloat(data, e);
            f.write((const char *) e, 4);
        }
        return (bool) f;
    }
    std::vector<uint8_t> buffer(4 * (size_t) W);
    for (int y = 0; y < img.height; ++y) {
        uint8_t hdr[4] = {2, 2, (uint8_t) (W >> 8), (uint8_t) (W & 0xff)};
        f.write((const char *) hdr, 4);
        for (int x = 0; x < W; ++x, data += 3) {
            uint8_t e[4];
            rgbeFromFloat(data, e);
            for (int c = 0; c < 4; ++c) buffer[(size_t) c * W + x] = e[c];
        }
        for (int c = 0; c < 4; ++c) rgbeRLE(f, &buffer[(size_t) c * W], W);
    }
    return (bool) f;
}

/* ---- OpenEXR, single part, scanline, NO_COMPRESSION ---- */
void le32(std::vector<unsigned char> &v, uint32_t x) {
    for (int i = 0; i < 4; ++i) v.push_back((unsigned char) (x >> (8 * i)));
}
void le64(std::vector<unsigned char> &v, uint64_t x) {
    for (int i = 0; i < 8; ++i) v.push_back((unsigned char) (x >> (8 * i)));
}
void attr(std::vector<unsigned char> &h, const char *name, const char *type, const std::vector<unsigned char> &val) {
    h.insert(h.end(), name, name + std::strlen(name) + 1);
    h.insert(h.end(), type, type + std::strlen(type) + 1);
    le32(h, (uint32_t) val.size());
    h.insert(h.end(), val.begin(), val.end());
}
bool writeEXRImage(const std::string &path, const FilmImage &img) {
    const int W = img.width, H = img.height, C = img.channels;
    const uint32_t pixType = img.component == 1 ? 1 : img.component == 2 ? 2 : 0; /* HALF 1, FLOAT 2, UINT 0 */
    const int compBytes = img.component == 1 ? 2 : 4;
    /* channels in alphabetical order (B, G, R / Y); data is stored per channel per scanline */
    std::vector<std::pair<char, int>> ch; /* name, index in the pixel */
    if (C == 1) ch = {{'Y', 0}};
    else ch = {{'B', 2}, {'G', 1}, {'R', 0}};
    std::vector<unsigned char> h = {0x76, 0x2f, 0x31, 0x01, 2, 0, 0, 0};
    std::vector<unsigned char> v;
    for (auto &c : ch) {
        v.push_back((unsigned char) c.first);
        v.push_back(0);
        le32(v, pixType);
        v.insert(v.end(), {0, 0, 0, 0}); /* pLinear, reserved */
        le32(v, 1);
        le32(v, 1);
    }
    v.push_back(0);
    attr(h, "channels", "chlist", v);
    attr(h, "compression", "compression", {0});
    v.clear();
    for (uint32_t x : {0u, 0u, (uint32_t) (W - 1), (uint32_t) (H - 1)}) le32(v, x);
    attr(h, "dataWindow", "box2i", v);
    attr(h, "displayWindow", "box2i", v);
    attr(h, "lineOrder", "lineOrder", {0});
    v.clear();
    float one = 1.0f;
    uint32_t bits;
    std::memcpy(&bits, &one, 4);
    le32(v, bits);
    attr(h, "pixelAspectRatio", "float", v);
    v.clear();
    le32(v, 0);
    le32(v, 0);
    attr(h, "screenWindowCenter", "v2f", v);
    v.clear();
    le32(v, bits);
    attr(h, "screenWindowWidth", "float", v);
    h.push_back(0); /* end of header */
    const size_t lineBytes = (size_t) W * C * compBytes;
    const uint64_t tableEnd = h.size() + 8ull * H;
    for (int y = 0; y < H; ++y) le64(h, tableEnd + (uint64_t) y * (8 + lineBytes));
    std::ofstream f(path, std::ios::binary);
    if (!f) return false;
    f.write((const char *) h.data(), (std::streamsize) h.size());
    std::vector<unsigned char> line(8 + lineBytes);
    for (int y = 0; y < H; ++y) {
        line.clear();
        le32(line, (uint32_t) y);
        le32(line, (uint32_t) lineBytes);
        for (auto &c : ch)
            for (int x = 0; x < W; ++x) {
                const unsigned char *px = img.bytes.data() + (((size_t) y * W + x) * C + c.second) * compBytes;
                line.insert(line.end(), px, px + compBytes);
            }
        f.write((const char *) line.data(), (std::streamsize) line.size());
    }
    return (bool) f;
}

} // namespace

bool checkFilm(FilmDesc &f, std::string &err) {
    f.type = lower(f.type);
    f.pixelFormat = lower(f.pixelFormat);
    f.componentFormat = lower(f.componentFormat);
    f.tonemapMethod = lower(f.tonemapMethod);
    if (f.fileFormat.empty()) f.fileFormat = f.type == "ldrfilm" ? "png" : "openexr";
    f.fileFormat = lower(f.fileFormat);
    if (f.pixelFormat == "rgba" || f.pixelFormat == "luminancealpha") {
        err = "pixelFormat \"" + f.pixelFormat + "\": the hair path records no alpha channel (use rgb or luminance)";
        return false;
    }
    if (f.pixelFormat != "rgb" && f.pixelFormat != "luminance") {
        err = "The \"pixelFormat\" parameter \"" + f.pixelFormat + "\" is not supported (rgb, luminance)";
        return false;
    }
    if (f.type == "ldrfilm") {
        if (f.fileFormat == "jpg" || f.fileFormat == "jpeg") {
            err = "ldrfilm: JPEG output is not supported here (use png)";
            return false;
        }
        if (f.fileFormat != "png") {
            err = "The \"fileFormat\" parameter must either be equal to \"png\" or \"jpeg\"!";
            return false;
        }
        if (f.tonemapMethod != "gamma" && f.tonemapMethod != "reinhard") {
            err = "The \"method\" parameter must either be equal to \"gamma\" or \"reinhard\"!";
            return false;
        }
        return true;
    }
    if (f.fileFormat != "openexr" && f.fileFormat != "rgbe" && f.fileFormat != "pfm") {
        err = "The \"fileFormat\" parameter must either be equal to \"openexr\", \"rgbe\", or \"pfm\"!";
        return false;
    }
    if (f.componentFormat != "float16" && f.componentFormat != "float32" && f.componentFormat != "uint32") {
        err = "The \"componentFormat\" parameter must either be equal to \"float16\", \"float32\", or \"uint32\"!";
        return false;
    }
    /* hdrfilm.cpp:314-339: RGBE and PFM override the formats they cannot store */
    if (f.fileFormat == "rgbe") {
        f.pixelFormat = "rgb";
        f.componentFormat = "float32";
    } else if (f.fileFormat == "pfm") {
        f.componentFormat = "float32";
    }
    return true;
}

bool developFilm(const float *rgbw, int w, int h, const FilmDesc &f, const std::string &dataDir, FilmImage &out,
                 std::string &err) {
    const bool ldr = f.type == "ldrfilm";
    const int C = f.pixelFormat == "luminance" ? 1 : 3;
    const size_t N = (size_t) w * h;
    /* ImageBlock -> RGB / luminance: spec * (1 / weight) (fmtconv.cpp:956-990) */
    std::vector<float> px(N * C);
    for (size_t i = 0; i < N; ++i) {
        const float *s = rgbw + 4 * i;
        float weight = s[3], invWeight = weight != 0 ? 1 / weight : weight;
        if (C == 1) {
            px[i] = (s[0] * 0.212671f + s[1] * 0.715160f + s[2] * 0.072169f) * invWeight;
        } else {
            for (int c = 0; c < 3; ++c) px[3 * i + c] = s[c] * invWeight;
        }
    }
    out.width = w;
    out.height = h;
    out.channels = C;
    std::vector<uint8_t> mask;
    int bw = 0, bh = 0;
    const bool banner = f.banner && w > 108 + 5 && h > 5 + 5;
    if (banner && !loadBanner(dataDir, mask, bw, bh)) {
        err = "cannot read the banner mask from " + dataDir + "/film/banner.u8";
        return false;
    }
    auto bannerAt = [&](int x, int y) {
        if (!banner) return false;
        int bx = x - (w - bw - 5), by = y - (h - bh - 5);
        return bx >= 0 && bx < bw && by >= 0 && by < bh && !mask[(size_t) bx + (size_t) by * bw];
    };
    if (ldr) {
        float multiplier = 1.0f;
        if (f.tonemapMethod == "reinhard") tonemapReinhard(px.data(), N, C, f.key, f.burn);
        else multiplier = std::pow(2.0f, f.exposure);
        const float invGamma = f.gamma == -1 ? -1.0f : 1.0f / f.gamma;
        out.component = 0;
        out.bytes.resize(N * C);
        for (size_t i = 0; i < N * C; ++i) out.bytes[i] = toU8(px[i], multiplier, invGamma);
        for (int y = 0; y < h; ++y)
            for (int x = 0; x < w; ++x)
                if (bannerAt(x, y))
                    for (int c = 0; c < C; ++c) out.bytes[((size_t) y * w + x) * C + c] = 255;
        return true;
    }
    for (int y = 0; y < h; ++y) /* hdrfilm.cpp:492-502: Spectrum(1024) */
        for (int x = 0; x < w; ++x)
            if (bannerAt(x, y))
                for (int c = 0; c < C; ++c) px[((size_t) y * w + x) * C + c] = 1024.0f;
    if (f.componentFormat == "float16") {
        out.component = 1;
        out.bytes.resize(N * C * 2);
        for (size_t i = 0; i < N * C; ++i) {
            uint16_t v = floatToHalf(px[i]);
            std::memcpy(&out.bytes[2 * i], &v, 2);
        }
    } else if (f.componentFormat == "float32") {
        out.component = 2;
        out.bytes.resize(N * C * 4);
        std::memcpy(out.bytes.data(), px.data(), N * C * 4);
    } else {
        out.component = 3;
        out.bytes.resize(N * C * 4);
        for (size_t i = 0; i < N * C; ++i) {
            uint32_t v = toU32(px[i]);
            std::memcpy(&out.bytes[4 * i], &v, 4);
        }
    }
    return true;
}

bool writeFilm(const std::string &path, const FilmImage &img, const FilmDesc &f, std::string &written,
               std::string &err) {
    std::string ext = f.type == "ldrfilm" ? ".png" : f.fileFormat == "openexr" ? ".exr"
                                                   : f.fileFormat == "rgbe"    ? ".rgbe"
                                                                               : ".pfm";
    /* ldrfilm.cpp:335-345 / hdrfilm.cpp:508-519: replace a wrong extension */
    written = path;
    size_t slash = path.find_last_of('/'), dot = path.find_last_of('.');
    std::string cur = (dot != std::string::npos && (slash == std::string::npos || dot > slash)) ? lower(path.substr(dot)) : "";
    if (cur != ext) written = (cur.empty() ? path : path.substr(0, dot)) + ext;
    bool ok;
    if (f.type == "ldrfilm") ok = writePNG(written, img);
    else if (f.fileFormat == "openexr") ok = writeEXRImage(written, img);
    else if (f.fileFormat == "rgbe") ok = writeRGBEImage(written, img);
    else ok = writePFMImage(written, img);
    if (!ok) err = "cannot write " + written;
    return ok;
}

} // namespace hpt
