/*
 * sunsky_ref.cpp -- oracle restatement of the `sunsky` emitter's rasterisation
 * into the lat-long bitmap it hands to a nested `envmap`.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Written from the reference
 * source, not from the product's csrc/host/sunsky.cpp, so that the parity
 * tests light the oracle's scene with a bitmap the product did not make:
 *
 *   SunSkyEmitter ctor        src/emitters/sunsky.cpp:100-240
 *   SkyEmitter                src/emitters/sky.cpp:222-252 (state), :405-433 (radiance)
 *   Hosek-Wilkie RGB model    src/emitters/sunsky/skymodel.cpp:80-239, 346-397
 *   sun position / spectrum   src/emitters/sunsky/sunmodel.h:90-105, 206-244, 316-371
 *   spectrum -> RGB           src/libcore/spectrum.cpp:172-191, 222-227, 546-568, 650-714
 *   Gauss-Lobatto quadrature  src/libcore/quad.cpp:287-415
 *   (0,2)-sequence, cone warp include/mitsuba/core/qmc.h:43-126, src/libcore/warp.cpp:54-63
 *
 * Types follow the reference's SINGLE_PRECISION build: Float = float, and
 * M_PI is the float M_PI_FLT (include/mitsuba/core/constants.h:79-80), so an
 * expression promotes to double only through a double literal or variable.
 * math::fastexp(float) is the double exp (math.h:185-187, Linux x86_64) and
 * math::sincos(float) is sincosf (math.h:219-221).
 *
 * Scope: sunDirection given (every shipped scene), emitter toWorld identity,
 * extend = false, sunRadiusScale > 0; anything else is refused.
 * Data: the reference's tables as extracted into the package's data/sunsky
 * (sha256-pinned to the extraction by tests/test_host.py).
 */
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <cstring>
#include <fstream>
#include <functional>
#include <limits>
#include <sstream>
#include <string>
#include <vector>

#include "lobatto.h"

namespace {

const float kPiF = 3.14159265358979323846f; /* M_PI under SINGLE_PRECISION */
const float kEps = 1e-4f;                   /* Epsilon (constants.h:28) */

struct V {
    float x, y, z;
};
V operator*(V a, float f) { return {a.x * f, a.y * f, a.z * f}; }
V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }

/* sunmodel.h:64-105 */
struct Spherical {
    float elevation, azimuth;
};
V toSphere(Spherical c) {
    float sinTheta, cosTheta, sinPhi, cosPhi;
    sincosf(c.elevation, &sinTheta, &cosTheta);
    sincosf(c.azimuth, &sinPhi, &cosPhi);
    return {sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta};
}
Spherical fromSphere(V d) {
    float azimuth = std::atan2(d.x, -d.z);
    float elevation = std::acos(std::min(1.0f, std::max(-1.0f, d.y))); /* math::safe_acos */
    if (azimuth < 0) azimuth += 2 * kPiF;
    return {elevation, azimuth};
}

/* ---------------- Hosek-Wilkie (skymodel.cpp) ---------------- */
double quinticBlend(const double *m, int stride, double s) {
    return std::pow(1.0 - s, 5.0) * m[0] + 5.0 * std::pow(1.0 - s, 4.0) * s * m[stride] +
           10.0 * std::pow(1.0 - s, 3.0) * std::pow(s, 2.0) * m[2 * stride] +
           10.0 * std::pow(1.0 - s, 2.0) * std::pow(s, 3.0) * m[3 * stride] +
           5.0 * (1.0 - s) * std::pow(s, 4.0) * m[4 * stride] + std::pow(s, 5.0) * m[5 * stride];
}

/* ArHosekSkyModel_CookConfiguration (:80-161): 9 coefficients.  The four
   (albedo, turbidity) corners are added in the reference's order. */
void cookConfig(const double *ds, double cfg[9], double turbidity, double albedo, double elevation) {
    const int it = (int) turbidity;
    const double rem = turbidity - (double) it;
    const double s = std::pow(elevation / ((double) kPiF / 2.0), (1.0 / 3.0));
    const double *corner[4] = {ds + 9 * 6 * (it - 1), ds + (9 * 6 * 10 + 9 * 6 * (it - 1)), ds + 9 * 6 * it,
                               ds + (9 * 6 * 10 + 9 * 6 * it)};
    const double wt[4] = {(1.0 - albedo) * (1.0 - rem), albedo * (1.0 - rem), (1.0 - albedo) * rem, albedo * rem};
    for (int k = 0; k < 4; ++k) {
        if (k == 2 && it == 10) break;
        for (int i = 0; i < 9; ++i) {
            const double v = wt[k] * quinticBlend(corner[k] + i, 9, s);
            cfg[i] = k == 0 ? v : cfg[i] + v;
        }
    }
}
/* ArHosekSkyModel_CookRadianceConfiguration (:163-224) */
double cookRad(const double *ds, double turbidity, double albedo, double elevation) {
    const int it = (int) turbidity;
    const double rem = turbidity - (double) it;
    const double s = std::pow(elevation / ((double) kPiF / 2.0), (1.0 / 3.0));
    double res = (1.0 - albedo) * (1.0 - rem) * quinticBlend(ds + 6 * (it - 1), 1, s);
    res += albedo * (1.0 - rem) * quinticBlend(ds + (6 * 10 + 6 * (it - 1)), 1, s);
    if (it == 10) return res;
    res += (1.0 - albedo) * rem * quinticBlend(ds + 6 * it, 1, s);
    res += albedo * rem * quinticBlend(ds + (6 * 10 + 6 * it), 1, s);
    return res;
}
/* ArHosekSkyModel_GetRadianceInternal (:226-239) */
double hosekInternal(const double c[9], double theta, double gamma) {
    const double expM = std::exp(c[4] * gamma);
    const double rayM = std::cos(gamma) * std::cos(gamma);
    const double mieM =
        (1.0 + std::cos(gamma) * std::cos(gamma)) / std::pow((1.0 + c[8] * c[8] - 2.0 * c[8] * std::cos(gamma)), 1.5);
    const double zenith = std::sqrt(std::cos(theta));
    return (1.0 + c[0] * std::exp(c[1] / (std::cos(theta) + 0.01))) *
           (c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith);
}

/* ---------------- spectra (spectrum.cpp) ---------------- */
struct Tabulated { /* InterpolatedSpectrum */
    std::vector<float> x, y;
    float eval(float lambda) const { /* :688-714 */
        if (x.size() < 2 || lambda < x.front() || lambda > x.back()) return 0.0f;
        const auto lo = std::lower_bound(x.begin(), x.end(), lambda);
        const auto hi = std::upper_bound(x.begin(), x.end(), lambda);
        const size_t i1 = (size_t) (lo - x.begin()), i2 = (size_t) (hi - x.begin());
        if (i1 == i2) {
            const float a = x[i1 - 1], b = x[i1], t = (lambda - a) / (b - a);
            return (1.0f - t) * y[i1 - 1] + t * y[i1]; /* math::lerp */
        }
        return y[i1];
    }
    float average(float lo, float hi) const { /* :650-686: exact trapezoids */
        if (x.size() < 2) return 0.0f;
        const float rs = std::max(lo, x.front()), re = std::min(hi, x.back());
        if (re <= rs) return 0.0f;
        size_t e = std::max((size_t) (std::lower_bound(x.begin(), x.end(), rs) - x.begin()), (size_t) 1) - 1;
        float sum = 0.0f;
        for (; e + 1 < x.size() && re >= x[e]; ++e) {
            const float a = x[e], b = x[e + 1], ca = std::max(a, rs), cb = std::min(b, re);
            const float fa = y[e], fb = y[e + 1], invAB = 1.0f / (b - a);
            if (cb <= ca) continue;
            const float ta = (ca - a) * invAB, tb = (cb - a) * invAB;
            const float ia = (1.0f - ta) * fa + ta * fb, ib = (1.0f - tb) * fa + tb * fb;
            sum += 0.5f * (ia + ib) * (cb - ca);
        }
        return sum / (hi - lo);
    }
};

/* GaussLobattoIntegrator: oracle/lobatto.h (useConvergenceEstimate = false here) */
using orc_quad::Lobatto;

/* ContinuousSpectrum::average (:546-568) of f over [lo, hi] in 50 nm pieces */
float averageOf(const std::function<float(float)> &f, float lo, float hi) {
    const Lobatto q(10000, kEps, kEps, false);
    if (hi <= lo) return 0.0f;
    const size_t n = std::max((size_t) 1, (size_t) std::ceil((hi - lo) / 50));
    const float stepSize = (hi - lo) / n;
    float pos = lo, acc = 0;
    for (size_t i = 0; i < n; ++i) {
        acc += q.integrate(f, pos, pos + stepSize);
        pos += stepSize;
    }
    return acc / (hi - lo);
}

struct Tables {
    std::vector<double> hosek; /* datasetsRGB[3] (1080 each), then datasetsRGBRad[3] (120 each) */
    Tabulated cie[3];          /* CIE 1931 x, y, z over 360..830 nm */
    Tabulated kO, kG, kWa, sol;
};

bool loadTables(const std::string &dir, Tables &t, std::string &err) {
    std::ifstream h(dir + "/hosek_rgb.f64", std::ios::binary), c(dir + "/cie1931.f32", std::ios::binary);
    std::ifstream js(dir + "/sun_tables.json");
    if (!h || !c || !js) {
        err = "sunsky tables not found under " + dir;
        return false;
    }
    t.hosek.resize(3 * 1080 + 3 * 120);
    h.read((char *) t.hosek.data(), (std::streamsize) (t.hosek.size() * 8));
    std::vector<float> cie(4 * 471);
    c.read((char *) cie.data(), (std::streamsize) (cie.size() * 4));
    if (!h || !c) {
        err = "short sunsky table";
        return false;
    }
    for (int k = 0; k < 3; ++k) {
        t.cie[k].x.assign(cie.begin(), cie.begin() + 471);
        t.cie[k].y.assign(cie.begin() + 471 * (k + 1), cie.begin() + 471 * (k + 2));
    }
    std::stringstream ss;
    ss << js.rdbuf();
    const std::string s = ss.str();
    auto list = [&](const std::string &key, std::vector<float> &out) {
        const size_t k = s.find("\"" + key + "\"");
        if (k == std::string::npos) return false;
        const size_t a = s.find('[', k), b = s.find(']', a);
        out.clear();
        std::stringstream in(s.substr(a + 1, b - a - 1));
        std::string tok;
        while (std::getline(in, tok, ',')) out.push_back((float) std::strtod(tok.c_str(), nullptr));
        return !out.empty();
    };
    bool ok = list("k_oWavelengths", t.kO.x) && list("k_oAmplitudes", t.kO.y) && list("k_gWavelengths", t.kG.x) &&
              list("k_gAmplitudes", t.kG.y) && list("k_waWavelengths", t.kWa.x) &&
              list("k_waAmplitudes", t.kWa.y) && list("solWavelengths", t.sol.x) && list("solAmplitudes", t.sol.y);
    if (!ok) {
        err = "malformed sun_tables.json";
        return false;
    }
    t.kO.y.resize(t.kO.x.size()); /* InterpolatedSpectrum(k_oWavelengths, k_oAmplitudes, 64): 65 amplitudes declared */
    return true;
}

/* Spectrum::fromContinuousSpectrum (RGB mode) + fromXYZ */
void toRGB(const Tables &t, const Tabulated &smooth, float rgb[3]) {
    const float lo = t.cie[0].x.front(), hi = t.cie[0].x.back();
    float xyz[3];
    for (int k = 0; k < 3; ++k)
        xyz[k] = averageOf([&](float l) { return smooth.eval(l) * t.cie[k].eval(l); }, lo, hi);
    const float norm = 1.0f / t.cie[1].average(lo, hi);
    for (float &v : xyz) v *= norm;
    rgb[0] = 3.240479f * xyz[0] + -1.537150f * xyz[1] + -0.498535f * xyz[2];
    rgb[1] = -0.969256f * xyz[0] + 1.875991f * xyz[1] + 0.041556f * xyz[2];
    rgb[2] = 0.055648f * xyz[0] + -0.204043f * xyz[1] + 1.057311f * xyz[2];
}

float fexp(float v) { return (float) std::exp((double) v); } /* math::fastexp (Linux x86_64) */

/* computeSunRadiance (sunmodel.h:316-371) */
void sunRadiance(const Tables &t, float theta, float turbidity, float rgb[3]) {
    Tabulated spec;
    const float beta = 0.04608365822050f * turbidity - 0.04586025928522f;
    const float m = 1.0f / (std::cos(theta) + 0.15f * std::pow(93.885f - theta / kPiF * 180.0f, (float) -1.253f));
    float lambda = 350;
    for (int i = 0; i < 91; ++i, lambda += 5) {
        const float tauR = fexp(-m * 0.008735f * std::pow(lambda / 1000.0f, (float) -4.08));
        const float alpha = 1.3f;
        const float tauA = fexp(-m * beta * std::pow(lambda / 1000.0f, -alpha));
        const float lOzone = .35f;
        const float tauO = fexp(-m * t.kO.eval(lambda) * lOzone);
        const float tauG =
            fexp(-1.41f * t.kG.eval(lambda) * m / std::pow(1 + 118.93f * t.kG.eval(lambda) * m, (float) 0.45f));
        const float w = 2.0;
        const float tauWA = fexp(-0.2385f * t.kWa.eval(lambda) * w * m /
                                 std::pow(1 + 20.07f * t.kWa.eval(lambda) * w * m, (float) 0.45f));
        spec.y.push_back(t.sol.eval(lambda) * tauR * tauA * tauO * tauG * tauWA);
        spec.x.push_back(lambda);
    }
    toRGB(t, spec, rgb);
    for (int k = 0; k < 3; ++k) rgb[k] = std::max(rgb[k], 0.0f); /* clampNegative */
}

/* sample02 (qmc.h:115-126, SINGLE_PRECISION): van der Corput (24 bits) and Sobol' */
float vdc24(uint32_t n) {
    n = (n << 16) | (n >> 16);
    n = ((n & 0x00ff00ffu) << 8) | ((n & 0xff00ff00u) >> 8);
    n = ((n & 0x0f0f0f0fu) << 4) | ((n & 0xf0f0f0f0u) >> 4);
    n = ((n & 0x33333333u) << 2) | ((n & 0xccccccccu) >> 2);
    n = ((n & 0x55555555u) << 1) | ((n & 0xaaaaaaaau) >> 1);
    return (float) (n >> 8) / (float) (1U << 24);
}
float sobolDim2(uint32_t n) {
    uint32_t r = 0;
    for (uint32_t v = 1U << 31; n != 0; n >>= 1, v ^= v >> 1)
        if (n & 1) r ^= v;
    return (float) r / (float) (1ULL << 32);
}

} // namespace

extern "C" {

/* The sunsky emitter's bitmap (resolution x resolution/2 RGB floats, row-major,
   rgb must hold resolution*resolution/2*3 floats).  Returns 0 on success. */
int orc_rasterize_sunsky(const char *data_dir, const float sun_dir[3], float turbidity, float albedo,
                         float stretch, float sky_scale, float sun_scale, float sun_radius_scale, int resolution,
                         float *rgb) {
    Tables t;
    std::string err;
    if (!loadTables(data_dir, t, err)) return -1;
    if (!(sun_radius_scale > 0) || turbidity < 1 || turbidity > 10 || stretch < 1 || stretch > 2) return -2;
    const int W = resolution, H = resolution / 2;
    /* computeSunCoordinates(sunDirection, identity) = fromSphere(normalize(v)) (sunmodel.h:206-208) */
    const float len = std::sqrt(sun_dir[0] * sun_dir[0] + sun_dir[1] * sun_dir[1] + sun_dir[2] * sun_dir[2]);
    const float inv = 1.0f / len;
    Spherical sun = fromSphere({sun_dir[0] * inv, sun_dir[1] * inv, sun_dir[2] * inv});

    /* SkyEmitter (sky.cpp:222-252): one RGB state per channel, with that channel's albedo */
    const float sunElevation = 0.5f * kPiF - sun.elevation;
    if (sunElevation < 0) return -3;
    double cfg[3][9], rad[3];
    for (int ch = 0; ch < 3; ++ch) {
        cookConfig(t.hosek.data() + 1080 * ch, cfg[ch], turbidity, albedo, sunElevation);
        rad[ch] = cookRad(t.hosek.data() + 3 * 1080 + 120 * ch, turbidity, albedo, sunElevation);
    }
    /* sky rasterisation (sunsky.cpp:126-150 -> sky.cpp:405-433) */
    const float fx = (2 * kPiF) / W, fy = kPiF / H;
    for (int y = 0; y < H; ++y) {
        const float thetaPix = (y + .5f) * fy;
        for (int x = 0; x < W; ++x) {
            const float phiPix = (x + .5f) * fx;
            const Spherical c = fromSphere(toSphere({thetaPix, phiPix}));
            float *o = rgb + 3 * ((size_t) y * W + x);
            const float theta = c.elevation / stretch;
            if (std::cos(theta) <= 0) {
                o[0] = o[1] = o[2] = 0.0f;
                continue;
            }
            const float cosGamma = std::cos(theta) * std::cos(sun.elevation) +
                                   std::sin(theta) * std::sin(sun.elevation) * std::cos(c.azimuth - sun.azimuth);
            const float gamma = std::acos(std::min(1.0f, std::max(-1.0f, cosGamma)));
            for (int ch = 0; ch < 3; ++ch) {
                float v = (float) (hosekInternal(cfg[ch], theta, gamma) * rad[ch] / 106.856980);
                o[ch] = std::max(v, 0.0f) * sky_scale;
            }
        }
    }

    /* the sun as (0,2)-sequence cone samples (sunsky.cpp:163-218) */
    float sr[3];
    sunRadiance(t, sun.elevation, turbidity, sr);
    for (float &v : sr) v *= sun_scale;
    sun.elevation *= stretch;
    const V n = toSphere(sun);
    V s, tt; /* Frame(n): coordinateSystem (util.cpp:592-601) */
    if (std::abs(n.x) > std::abs(n.y)) {
        const float il = 1.0f / std::sqrt(n.x * n.x + n.z * n.z);
        tt = {n.z * il, 0.0f, -n.x * il};
    } else {
        const float il = 1.0f / std::sqrt(n.y * n.y + n.z * n.z);
        tt = {0.0f, n.z * il, -n.y * il};
    }
    s = {tt.y * n.z - tt.z * n.y, tt.z * n.x - tt.x * n.z, tt.x * n.y - tt.y * n.x}; /* cross(c, a) */
    const float kSunAppRadius = (float) (0.5358 * 0.5f);                              /* SUN_APP_RADIUS * 0.5f */
    const float theta = kSunAppRadius * (kPiF / 180.0f);                               /* degToRad */
    const size_t pixelCount = (size_t) resolution * resolution / 2;
    const float cosTheta = std::cos(theta * sun_radius_scale);
    const float covered = 0.5f * (1 - cosTheta);
    const size_t nSamples = (size_t) std::max((float) 100, (pixelCount * covered * 1000));
    const float gx = W / (2 * kPiF), gy = H / kPiF;
    float value[3];
    const float k1 = 2 * kPiF * (1 - std::cos(theta)), k2 = (float) (W * H);
    const float rk3 = 1.0f / (2 * kPiF * kPiF * (float) nSamples);
    for (int ch = 0; ch < 3; ++ch) value[ch] = sr[ch] * k1 * k2 * rk3;
    for (size_t i = 0; i < nSamples; ++i) {
        const float u = vdc24((uint32_t) i), v = sobolDim2((uint32_t) i);
        const float ct = (1 - u) + u * cosTheta; /* warp::squareToUniformCone */
        const float st = std::sqrt(std::max(0.0f, 1.0f - ct * ct));
        float sinPhi, cosPhi;
        sincosf(2.0f * kPiF * v, &sinPhi, &cosPhi);
        const V d = s * (cosPhi * st) + tt * (sinPhi * st) + n * ct; /* Frame::toWorld */
        const float sinT = std::sqrt(std::max(0.0f, 1 - d.y * d.y));
        const Spherical c = fromSphere(d);
        const int px = std::min(std::max(0, (int) (c.azimuth * gx)), W - 1);
        const int py = std::min(std::max(0, (int) (c.elevation * gy)), H - 1);
        const float r = 1.0f / std::max((float) 1e-3f, sinT);
        float *o = rgb + 3 * ((size_t) py * W + px);
        for (int ch = 0; ch < 3; ++ch) o[ch] += value[ch] * r;
    }
    return 0;
}

} /* extern "C" */
