/*
 * oracle.cpp -- CPU restatement of the reference's hair path-tracing hot
 * path (ja5087/cs184-final-project-mitsuba0.5).
 *
 * TEST INFRASTRUCTURE ONLY: loaded by tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py, never by the product.  Pinned by independent restatements (see
 * oracle.h); where it is not pinned it follows the cited reference lines
 * statement by statement, in single precision, without fused multiply-adds.
 *
 * Deliberate, documented deviations from the reference binary:
 *   - Primary-ray environment lookups use the level-0 bilinear filter; the
 *     reference's EWA path (mipmap.h:631-715) reduces to exactly that when the
 *     ellipse's major radius is < 1 texel, which the oracle checks and counts
 *     (stats[5]); parity tests assert that count is 0 for every config.
 *   - kajiyakay.cpp:162-170 builds and discards an ostringstream per specular
 *     evaluation; it has no numeric effect and is omitted.
 *   - Splat order: each 32x32 block is splatted row-major, blocks are merged
 *     in block order (the reference uses Hilbert order and completion order);
 *     this only changes float summation order.
 */
#include "oracle.h"
#include "ref_core.h"
#include "lobatto.h"

#include <algorithm>
#include <atomic>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <functional>
#include <map>
#include <memory>
#include <sstream>
#include <stdexcept>
#include <string>
#include <thread>
#include <vector>

using namespace orc;

namespace {

/* ------------------------------------------------------------------ */
/* IEEE half conversion (round to nearest even), as OpenEXR's half(float) */
/* used for the envmap MIP level 0 (envmap.cpp:102-103, mipmap.h:228-234) */
/* ------------------------------------------------------------------ */
uint16_t floatToHalf(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u;
    uint32_t absx = x & 0x7fffffffu;
    if (absx >= 0x7f800000u) { /* inf / nan */
        return (uint16_t) (sign | 0x7c00u | (absx > 0x7f800000u ? 0x200u : 0u));
    }
    if (absx >= 0x477ff000u) /* rounds to >= 65520 -> inf */
        return (uint16_t) (sign | 0x7c00u);
    if (absx < 0x38800000u) { /* half subnormal or zero */
        if (absx < 0x33000000u) /* < 2^-25 : rounds to zero */
            return (uint16_t) sign;
        uint32_t m = (absx & 0x007fffffu) | 0x00800000u;
        int e = (int) (absx >> 23); /* biased float exponent, 102..112 */
        int shift = 126 - e;        /* 14..24 */
        uint32_t half_m = m >> shift;
        uint32_t rem = m & ((1u << shift) - 1u);
        uint32_t halfway = 1u << (shift - 1);
        if (rem > halfway || (rem == halfway && (half_m & 1u)))
            half_m++;
        return (uint16_t) (sign | half_m);
    }
    uint32_t e = ((absx >> 23) - 112u) << 10;
    uint32_t m = (absx >> 13) & 0x3ffu;
    uint32_t rem = absx & 0x1fffu;
    uint32_t h = e | m;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u)))
        h++;
    return (uint16_t) (sign | h);
}

float halfToFloat(uint16_t h) {
    uint32_t sign = (uint32_t) (h & 0x8000u) << 16;
    uint32_t e = (h >> 10) & 0x1fu;
    uint32_t m = h & 0x3ffu;
    uint32_t x;
    if (e == 0) {
        if (m == 0) {
            x = sign;
        } else {
            int ee = -1;
            do { ee++; m <<= 1; } while (!(m & 0x400u));
            x = sign | ((uint32_t) (112 - ee) << 23) | ((m & 0x3ffu) << 13);
        }
    } else if (e == 31) {
        x = sign | 0x7f800000u | (m << 13);
    } else {
        x = sign | ((e + 112u) << 23) | (m << 13);
    }
    float f;
    std::memcpy(&f, &x, 4);
    return f;
}

/* ------------------------------------------------------------------ */
/* libcore/spline.cpp:23-61, 236-304, 379-451 (extrapolate = false)     */
/* ------------------------------------------------------------------ */
float evalCubicInterp1D(float x, const float *values, size_t size, float min, float max) {
    if (!(x >= min && x <= max))
        return 0.0f;
    float t = ((x - min) * (size - 1)) / (max - min);
    size_t k = std::max((size_t) 0, std::min((size_t) t, size - 2));
    float f0 = values[k], f1 = values[k + 1], d0, d1;
    if (k > 0)
        d0 = 0.5f * (values[k + 1] - values[k - 1]);
    else
        d0 = values[k + 1] - values[k];
    if (k + 2 < size)
        d1 = 0.5f * (values[k + 2] - values[k]);
    else
        d1 = values[k + 1] - values[k];
    t = t - (float) k;
    float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 +
           (t3 - t2) * d1;
}

bool knotWeights(float p, size_t size, float *weights, size_t &knot) {
    if (!(p >= 0.0f && p <= 1.0f))
        return false;
    float t = ((p - 0.0f) * (size - 1)) / (1.0f - 0.0f);
    knot = std::min((size_t) t, size - 2);
    t = t - (float) knot;
    float t2 = t * t, t3 = t2 * t;
    weights[0] = 0.0f;
    weights[1] = 2 * t3 - 3 * t2 + 1;
    weights[2] = -2 * t3 + 3 * t2;
    weights[3] = 0.0f;
    float d0 = t3 - 2 * t2 + t, d1 = t3 - t2;
    if (knot > 0) {
        weights[2] += 0.5f * d0;
        weights[0] -= 0.5f * d0;
    } else {
        weights[2] += d0;
        weights[1] -= d0;
    }
    if (knot + 2 < size) {
        weights[3] += 0.5f * d1;
        weights[1] -= 0.5f * d1;
    } else {
        weights[2] += d1;
        weights[1] -= d1;
    }
    return true;
}

float evalCubicInterp2D(float px, float py, const float *values, size_t sx, size_t sy) {
    float kw[2][4];
    size_t knot[2];
    if (!knotWeights(px, sx, kw[0], knot[0])) return 0.0f;
    if (!knotWeights(py, sy, kw[1], knot[1])) return 0.0f;
    float result = 0.0f;
    for (int y = -1; y <= 2; ++y) {
        float wy = kw[1][y + 1];
        for (int x = -1; x <= 2; ++x) {
            float wxy = kw[0][x + 1] * wy;
            if (wxy == 0)
                continue;
            size_t pos = (knot[1] + y) * sx + knot[0] + x;
            result += values[pos] * wxy;
        }
    }
    return result;
}

float evalCubicInterp3D(float px, float py, float pz, const float *values, size_t sx, size_t sy,
                        size_t sz) {
    float kw[3][4];
    size_t knot[3];
    if (!knotWeights(px, sx, kw[0], knot[0])) return 0.0f;
    if (!knotWeights(py, sy, kw[1], knot[1])) return 0.0f;
    if (!knotWeights(pz, sz, kw[2], knot[2])) return 0.0f;
    float result = 0.0f;
    for (int z = -1; z <= 2; ++z) {
        float wz = kw[2][z + 1];
        for (int y = -1; y <= 2; ++y) {
            float wyz = kw[1][y + 1] * wz;
            for (int x = -1; x <= 2; ++x) {
                float wxyz = kw[0][x + 1] * wyz;
                if (wxyz == 0)
                    continue;
                size_t pos = ((knot[2] + z) * sy + (knot[1] + y)) * sx + knot[0] + x;
                result += values[pos] * wxyz;
            }
        }
    }
    return result;
}

/* ------------------------------------------------------------------ */
/* bsdfs/rtrans.h:81-377 -- RoughTransmittance                          */
/* ------------------------------------------------------------------ */
struct RoughTransmittance {
    size_t etaSamples = 0, alphaSamples = 0, thetaSamples = 0;
    float etaMin = 0, etaMax = 0, alphaMin = 0, alphaMax = 0;
    std::vector<float> trans, diffTrans;
    bool etaFixed = false, alphaFixed = false;

    bool load(const std::string &path) {
        std::ifstream f(path, std::ios::binary);
        if (!f) return false;
        char hdr[17];
        f.read(hdr, 17);
        if (std::memcmp(hdr, "MTS_TRANSMITTANCE", 17) != 0) return false;
        uint64_t sz[3];
        f.read((char *) sz, 24);
        etaSamples = sz[0]; alphaSamples = sz[1]; thetaSamples = sz[2];
        float mm[4];
        f.read((char *) mm, 16);
        etaMin = mm[0]; etaMax = mm[1]; alphaMin = mm[2]; alphaMax = mm[3];
        size_t transSize = 2 * etaSamples * alphaSamples * thetaSamples;
        size_t diffSize = 2 * etaSamples * alphaSamples;
        std::vector<float> temp(transSize + diffSize);
        f.read((char *) temp.data(), (std::streamsize) (temp.size() * 4));
        if (!f) return false;
        trans.resize(transSize);
        diffTrans.resize(diffSize);
        const float *ptr = temp.data();
        size_t fdrEntry = 0, dataEntry = 0;
        for (size_t i = 0; i < 2 * etaSamples; ++i)
            for (size_t j = 0; j < alphaSamples; ++j) {
                for (size_t k = 0; k < thetaSamples; ++k)
                    trans[dataEntry++] = *ptr++;
                diffTrans[fdrEntry++] = *ptr++;
            }
        return true;
    }

    float eval(float cosTheta) const { /* both fixed (rtrans.h:183-199) */
        float warpedCosTheta = std::pow(std::abs(cosTheta), (float) 0.25f), result;
        if (!(cosTheta >= 0))
            return 0.f;
        result = evalCubicInterp1D(warpedCosTheta, trans.data(), thetaSamples, 0.0f, 1.0f);
        return std::min((float) 1.0f, std::max((float) 0.0f, result));
    }

    float evalDiffuse(float alpha) const { /* eta fixed, alpha free (rtrans.h:249-263) */
        float result;
        if (alphaFixed && etaFixed) {
            result = diffTrans[0];
        } else {
            float warpedAlpha = std::pow((alpha - alphaMin) / (alphaMax - alphaMin), (float) 0.25f);
            result = evalCubicInterp1D(warpedAlpha, diffTrans.data(), alphaSamples, 0.0f, 1.0f);
        }
        return std::min((float) 1.0f, std::max((float) 0.0f, result));
    }

    void setEta(float eta) { /* rtrans.h:292-345 */
        if (etaFixed) return;
        const float *tr = trans.data(), *dtr = diffTrans.data();
        if (eta < 1) {
            tr += etaSamples * alphaSamples * thetaSamples;
            dtr += etaSamples * alphaSamples;
            eta = 1.0f / eta;
        }
        if (eta < etaMin)
            eta = etaMin;
        float warpedEta = std::pow((eta - etaMin) / (etaMax - etaMin), (float) 0.25f);
        std::vector<float> newTrans(alphaSamples * thetaSamples), newDiff(alphaSamples);
        float dAlpha = 1.0f / (alphaSamples - 1), dTheta = 1.0f / (thetaSamples - 1);
        for (size_t i = 0; i < alphaSamples; ++i) {
            for (size_t j = 0; j < thetaSamples; ++j)
                newTrans[i * thetaSamples + j] = evalCubicInterp3D(
                    j * dTheta, i * dAlpha, warpedEta, tr, thetaSamples, alphaSamples, etaSamples);
            newDiff[i] = evalCubicInterp2D(i * dAlpha, warpedEta, dtr, alphaSamples, etaSamples);
        }
        trans.swap(newTrans);
        diffTrans.swap(newDiff);
        etaFixed = true;
    }

    void setAlpha(float alpha) { /* rtrans.h:353-377 */
        if (alphaFixed) return;
        float warpedAlpha = std::pow((alpha - alphaMin) / (alphaMax - alphaMin), (float) 0.25f);
        std::vector<float> newTrans(thetaSamples), newDiff(1);
        float dTheta = 1.0f / (thetaSamples - 1);
        for (size_t i = 0; i < thetaSamples; ++i)
            newTrans[i] = evalCubicInterp2D(i * dTheta, warpedAlpha, trans.data(), thetaSamples,
                                            alphaSamples);
        newDiff[0] = evalCubicInterp1D(warpedAlpha, diffTrans.data(), alphaSamples, 0.0f, 1.0f);
        trans.swap(newTrans);
        diffTrans.swap(newDiff);
        alphaFixed = true;
    }
};

/* ------------------------------------------------------------------ */
/* bsdfs/gausssexylingerie.hpp:11-93 -- GaussLegendre<N>               */
/* ------------------------------------------------------------------ */
template <int N> struct GaussLegendre {
    float points[N], weights[N];
    static double legendre(double x, int n) {
        if (n == 0) return 1.0;
        if (n == 1) return x;
        double P0 = 1.0, P1 = x;
        for (int i = 2; i <= n; ++i) {
            double Pi = ((2.0 * i - 1.0) * x * P1 - (i - 1.0) * P0) / i;
            P0 = P1;
            P1 = Pi;
        }
        return P1;
    }
    static double legendreDeriv(double x, int n) {
        return n / (x * x - 1.0) * (x * legendre(x, n) - legendre(x, n - 1));
    }
    static double kthRoot(int k) {
        double x = std::cos(kPi * (4.0 * k - 1.0) / (4.0 * N + 2.0)) *
                   (1.0 - 1.0 / (8.0 * N * N) + 1.0 / (8.0 * N * N * N));
        for (int i = 0; i < 100; ++i) {
            double f = legendre(x, N);
            x -= f / legendreDeriv(x, N);
            if (std::abs(f) < 1e-6)
                break;
        }
        return x;
    }
    GaussLegendre() {
        for (int i = 0; i < N; ++i) {
            points[i] = float(kthRoot(i + 1));
            weights[i] = float(2.0 / ((1.0 - points[i] * points[i]) * legendreDeriv(points[i], N) *
                                      legendreDeriv(points[i], N)));
        }
    }
};

/* ------------------------------------------------------------------ */
/* bsdfs/InterpolatedDistribution1D.hpp:7-111                           */
/* ------------------------------------------------------------------ */
struct InterpolatedDistribution1D {
    int size, numDist;
    std::vector<float> pdfs, cdfs, sums;
    InterpolatedDistribution1D(std::vector<float> weights, int size_, int numDist_)
        : size(size_), numDist(numDist_), pdfs(std::move(weights)), cdfs((size_ + 1) * numDist_),
          sums(numDist_) {
        for (int dist = 0; dist < numDist; ++dist) {
            cdf(0, dist) = 0.0f;
            for (int x = 0; x < size; ++x)
                cdf(x + 1, dist) = pdf_(x, dist) + cdf(x, dist);
            sums[dist] = cdf(size, dist);
            if (sums[dist] < 1e-4f) {
                float ratio = 1.0f / size;
                for (int x = 0; x < size; ++x) {
                    pdf_(x, dist) = ratio;
                    cdf(x, dist) = x * ratio;
                }
            } else {
                float scale = 1.0f / sums[dist];
                for (int x = 0; x < size; ++x) {
                    pdf_(x, dist) *= scale;
                    cdf(x, dist) *= scale;
                }
            }
            cdf(size, dist) = 1.0f;
        }
    }
    float &cdf(int x, int d) { return cdfs[x + d * (size + 1)]; }
    float &pdf_(int x, int d) { return pdfs[x + d * size]; }
    float cdfc(int x, int d) const { return cdfs[x + d * (size + 1)]; }
    float pdfc(int x, int d) const { return pdfs[x + d * size]; }
    void warp(float distribution, float &u, int &x) const {
        int d0 = clampv(int(distribution), 0, numDist - 1);
        int d1 = std::min(d0 + 1, numDist - 1);
        float v = clampv(distribution - d0, 0.0f, 1.0f);
        int lower = 0, upper = size;
        float lowerU = 0.0f, upperU = 1.0f;
        while (upper - lower != 1) {
            int midpoint = (upper + lower) / 2;
            float midpointU = cdfc(midpoint, d0) * (1.0f - v) + cdfc(midpoint, d1) * v;
            if (midpointU < u) {
                lower = midpoint;
                lowerU = midpointU;
            } else {
                upper = midpoint;
                upperU = midpointU;
            }
        }
        x = lower;
        u = clampv((u - lowerU) / (upperU - lowerU), 0.0f, 1.0f);
    }
    float pdf(float distribution, int x) const {
        int d0 = clampv(int(distribution), 0, numDist - 1);
        int d1 = std::min(d0 + 1, numDist - 1);
        float v = clampv(distribution - d0, 0.0f, 1.0f);
        return pdfc(x, d0) * (1.0f - v) + pdfc(x, d1) * v;
    }
    float sum(float distribution) const {
        int d0 = clampv(int(distribution), 0, numDist - 1);
        int d1 = std::min(d0 + 1, numDist - 1);
        float v = clampv(distribution - d0, 0.0f, 1.0f);
        return sums[d0] * (1.0f - v) + sums[d1] * v;
    }
};

/* ------------------------------------------------------------------ */
/* marschner_diffuse.cpp:39-109 -- Azimuthal                            */
/* ------------------------------------------------------------------ */
static const int kAzRes = 64;

struct Azimuthal {
    std::vector<V3> table; /* Vector3f RGB, index x + y*64 */
    std::unique_ptr<InterpolatedDistribution1D> sampler;
    explicit Azimuthal(std::vector<V3> t) : table(std::move(t)) {
        const int Size = kAzRes;
        std::vector<float> weights(Size * Size);
        for (int i = 0; i < Size * Size; ++i)
            weights[i] = std::max(std::max(table[i].x, table[i].y), table[i].z);
        for (int y = 0; y < Size; ++y) {
            for (int x = 0; x < Size - 1; ++x)
                weights[x + y * Size] = std::max(weights[x + y * Size], weights[x + 1 + y * Size]);
            for (int x = Size - 1; x > 0; --x)
                weights[x + y * Size] = std::max(weights[x + y * Size], weights[x - 1 + y * Size]);
        }
        for (int x = 0; x < Size; ++x) {
            for (int y = 0; y < Size - 1; ++y)
                weights[x + y * Size] = std::max(weights[x + y * Size], weights[x + (y + 1) * Size]);
            for (int y = Size - 1; y > 0; --y)
                weights[x + y * Size] = std::max(weights[x + y * Size], weights[x + (y - 1) * Size]);
        }
        sampler.reset(new InterpolatedDistribution1D(std::move(weights), Size, Size));
    }
    void sample(float cosThetaD, float xi, float &phi) const {
        float v = (kAzRes - 1) * cosThetaD;
        int x;
        sampler->warp(v, xi, x);
        phi = 2.0f * kPi * (x + xi) * (1.0f / kAzRes);
    }
    V3 eval(float phi, float cosThetaD) const {
        float u = (kAzRes - 1) * phi * (1.0f / (2.0f * kPi));
        float v = (kAzRes - 1) * cosThetaD;
        int x0 = clampv(int(u), 0, kAzRes - 2);
        int y0 = clampv(int(v), 0, kAzRes - 2);
        int x1 = x0 + 1, y1 = y0 + 1;
        u = clampv(u - x0, 0.0f, 1.0f);
        v = clampv(v - y0, 0.0f, 1.0f);
        return (table[x0 + y0 * kAzRes] * (1.0f - u) + table[x1 + y0 * kAzRes] * u) * (1.0f - v) +
               (table[x0 + y1 * kAzRes] * (1.0f - u) + table[x1 + y1 * kAzRes] * u) * v;
    }
    float weight(float cosThetaD) const {
        float v = (kAzRes - 1) * cosThetaD;
        return sampler->sum(v) * (2.0f * kPi / kAzRes);
    }
};

inline V3 mulv(const V3 &a, const V3 &b) { return V3(a.x * b.x, a.y * b.y, a.z * b.z); }
inline V3 expv(const V3 &v) { return V3(std::exp(v.x), std::exp(v.y), std::exp(v.z)); }

/* BSDF type flags (include/mitsuba/render/bsdf.h:224-285) */
enum : uint32_t {
    ENull = 0x00001, EDiffuseReflection = 0x00002, EDiffuseTransmission = 0x00004,
    EGlossyReflection = 0x00008, EGlossyTransmission = 0x00010, EDeltaReflection = 0x00020,
    EDeltaTransmission = 0x00040, EDelta1D = 0x00080,
};
static const uint32_t EDelta = ENull | EDeltaReflection | EDeltaTransmission;

/* ------------------------------------------------------------------ */
/* marschner_diffuse.cpp:111-847 -- plugin "marschner"                  */
/* ------------------------------------------------------------------ */
struct Marschner {
    float eta = 1.55f, invEta2 = 0, alpha = 0.1f;
    Spec diffuse{0.5f}, specular{0.5f};
    float specularSamplingWeight = 0;
    float betaR = 0.1f, betaTT = 0.05f, betaTRT = 0.2f, scaleAngleRad = -0.1f;
    float vR = 0, vTT = 0, vTRT = 0;
    V3 sigmaA{0.5f};
    std::unique_ptr<Azimuthal> nR, nTT, nTRT;
    RoughTransmittance ext, internal;
    float Fdr = 0;

    static float I0(float x) { /* :279-290 */
        float result = 1.0f, xSq = x * x, xi = xSq, denom = 4.0f;
        for (int i = 1; i <= 10; ++i) {
            result += xi / denom;
            xi *= xSq;
            denom *= 4.0f * float((i + 1) * (i + 1));
        }
        return result;
    }
    static float logI0(float x) { /* :292-299 */
        if (x > 12.0f)
            return x + 0.5f * (std::log(1.0f / (kPi * 2.0f * x)) + 1.0f / (8.0f * x));
        else
            return std::log(I0(x));
    }
    static float g(float beta, float theta) { /* :301-303 */
        return std::exp(-theta * theta / (2.0f * beta * beta)) / (std::sqrt(2.0f * kPi) * beta);
    }
    static float D(float beta, float phi) { /* :305-315 */
        float result = 0.0f, delta, shift = 0.0f;
        do {
            delta = g(beta, phi + shift) + g(beta, phi - shift - 2 * kPi);
            result += delta;
            shift += 2 * kPi;
        } while (delta > 1e-4f);
        return result;
    }
    static float Phi(float gammaI, float gammaT, int p) { /* :317-319 */
        return 2.0f * p * gammaT - 2.0f * gammaI + p * kPi;
    }
    static float M(float v, float sinThetaI, float sinThetaO, float cosThetaI, float cosThetaO) {
        /* :364-374 */
        float a = cosThetaI * cosThetaO / v;
        float b = sinThetaI * sinThetaO / v;
        if (v < 0.1f)
            return std::exp(-b + logI0(a) - 1.0f / v + 0.6931f + std::log(1.0f / (2.0f * v)));
        else
            return std::exp(-b) * I0(a) / (2.0f * v * std::sinh(1.0f / v));
    }
    static float trigInverse(float x) { /* :484-486 */
        return std::min(std::sqrt(std::max(1.0f - x * x, 0.0f)), 1.0f);
    }

    void precompute() { /* :751-834 */
        const int Resolution = kAzRes;
        std::vector<V3> valuesR(Resolution * Resolution), valuesTT(Resolution * Resolution),
            valuesTRT(Resolution * Resolution);
        const int NumPoints = 140;
        static const GaussLegendre<140> integrator;
        const float *points = integrator.points, *weights = integrator.weights;
        float gammaIs[NumPoints];
        for (int i = 0; i < NumPoints; ++i)
            gammaIs[i] = std::asin(points[i]);
        const int NumGaussianSamples = 2048;
        std::vector<float> Ds[3];
        for (int p = 0; p < 3; ++p) {
            Ds[p].resize(NumGaussianSamples);
            for (int i = 0; i < NumGaussianSamples; ++i)
                Ds[p][i] = D(betaR, i / (NumGaussianSamples - 1.0f) * 2 * kPi);
        }
        auto approxD = [&](int p, float phi) {
            float u = std::abs(phi * (1.0 / (2 * kPi) * (NumGaussianSamples - 1)));
            int x0 = int(u);
            int x1 = x0 + 1;
            u -= x0;
            return Ds[p][x0 % NumGaussianSamples] * (1.0f - u) + Ds[p][x1 % NumGaussianSamples] * u;
        };
        for (int y = 0; y < Resolution; ++y) {
            float cosHalfAngle = y / (Resolution - 1.0f);
            float iorPrime = std::sqrt(eta * eta - (1.0f - cosHalfAngle * cosHalfAngle)) / cosHalfAngle;
            float cosThetaT = std::sqrt(1.0f - (1.0f - cosHalfAngle * cosHalfAngle) * (1.0f / eta) *
                                                   (1.0f / eta));
            V3 sigmaAPrime = sigmaA / cosThetaT;
            float fresnelTerms[NumPoints], gammaTs[NumPoints];
            V3 absorptions[NumPoints];
            for (int i = 0; i < NumPoints; ++i) {
                gammaTs[i] = std::asin(clampv(points[i] / iorPrime, -1.0f, 1.0f));
                fresnelTerms[i] = fresnelDielectricExt(1.0f / eta, cosHalfAngle * std::cos(gammaIs[i]));
                absorptions[i] = expv(-sigmaAPrime * 2.0f * std::cos(gammaTs[i]));
            }
            for (int phiI = 0; phiI < Resolution; ++phiI) {
                float phi = kPi * 2 * phiI / (Resolution - 1.0f);
                float integralR = 0.0f;
                V3 integralTT(0.0f), integralTRT(0.0f);
                for (int i = 0; i < NumPoints; ++i) {
                    float fR = fresnelTerms[i];
                    V3 T = absorptions[i];
                    float AR = fR;
                    V3 ATT = (1.0f - fR) * (1.0f - fR) * T;
                    V3 ATRT = mulv(ATT * fR, T);
                    integralR += weights[i] * approxD(0, phi - Phi(gammaIs[i], gammaTs[i], 0)) * AR;
                    integralTT += weights[i] * approxD(1, phi - Phi(gammaIs[i], gammaTs[i], 1)) * ATT;
                    integralTRT += weights[i] * approxD(2, phi - Phi(gammaIs[i], gammaTs[i], 2)) * ATRT;
                }
                valuesR[phiI + y * Resolution] = V3(0.5f * integralR);
                valuesTT[phiI + y * Resolution] = 0.5f * integralTT;
                valuesTRT[phiI + y * Resolution] = 0.5f * integralTRT;
            }
        }
        nR.reset(new Azimuthal(std::move(valuesR)));
        nTT.reset(new Azimuthal(std::move(valuesTT)));
        nTRT.reset(new Azimuthal(std::move(valuesTRT)));
    }

    bool configure(int distribution, const std::string &datDir, std::string &err) {
        /* constructor :113-160 (betas, scale tilt, precompute) + configure :193-247 */
        betaR = 0.1f;
        betaTT = betaR * 0.5f;
        betaTRT = betaR * 2.0f;
        scaleAngleRad = -0.1f;
        precompute();
        vR = betaR * betaR;
        vTT = betaTT * betaTT;
        vTRT = betaTRT * betaTRT;
        /* ensureEnergyConservation(specularReflectance, max 1) -- bsdf.cpp:88-113 */
        float smax = specular.max();
        if (smax > 1.0f)
            specular *= 0.99f * (1.0f / smax);
        float dAvg = diffuse.getLuminance(), sAvg = specular.getLuminance();
        specularSamplingWeight = sAvg / (dAvg + sAvg);
        invEta2 = 1.0f / (eta * eta);
        const char *names[3] = {"beckmann", "ggx", "phong"};
        if (distribution < 0 || distribution > 2) { err = "bad distribution"; return false; }
        std::string path = datDir + "/" + names[distribution] + ".dat";
        if (!ext.load(path)) { err = "cannot load " + path; return false; }
        internal = ext;
        ext.setEta(eta);
        internal.setEta(1 / eta);
        ext.setAlpha(alpha);
        Fdr = 1 - internal.evalDiffuse(alpha);
        return true;
    }

    Spec eval(const V3 &wi, const V3 &wo) const { /* :377-482 (hasDiffuse = true) */
        float sinThetaI = wi.y, sinThetaO = wo.y;
        float cosThetaO = trigInverse(sinThetaO);
        float thetaI = std::asin(clampv(sinThetaI, -1.0f, 1.0f));
        float thetaO = std::asin(clampv(sinThetaO, -1.0f, 1.0f));
        float thetaD = (thetaO - thetaI) * 0.5f;
        float cosThetaD = std::cos(thetaD);
        float phi = std::atan2(wo.x, wo.z);
        if (phi < 0.0f)
            phi += kPi * 2.0f;
        float thetaIR = thetaI - 2.0f * scaleAngleRad;
        float thetaITT = thetaI + scaleAngleRad;
        float thetaITRT = thetaI + 4.0f * scaleAngleRad;
        float MR = M(vR, std::sin(thetaIR), sinThetaO, std::cos(thetaIR), cosThetaO);
        float MTT = M(vTT, std::sin(thetaITT), sinThetaO, std::cos(thetaITT), cosThetaO);
        float MTRT = M(vTRT, std::sin(thetaITRT), sinThetaO, std::cos(thetaITRT), cosThetaO);
        V3 temp = 0.15f * MR * nR->eval(phi, cosThetaD) + MTT * nTT->eval(phi, cosThetaD) +
                  MTRT * nTRT->eval(phi, cosThetaD);
        Spec result(temp.x, temp.y, temp.z);
        Spec diff = diffuse;
        float T12 = ext.eval(wi.z);
        float T21 = ext.eval(wo.z);
        diff /= 1 - Fdr;
        result += diff * (kInvPi * wo.z * T12 * T21 * invEta2);
        return result;
    }

    float pdf() const { return 1.0f; } /* :517-520 -- hasDiffuse => 1 */

    Spec sample(const V3 &wi, float sx, float sy, V3 &wo, float &pdfOut, uint32_t &type) const {
        /* :594-744 */
        float xiNx = sx, xiNy = sy, xiMx = sx, xiMy = sy;
        float sinThetaI = wi.y;
        float cosThetaI = trigInverse(sinThetaI);
        float thetaI = std::asin(clampv(sinThetaI, -1.0f, 1.0f));
        float thetaIR = thetaI - 2.0f * scaleAngleRad;
        float thetaITT = thetaI + scaleAngleRad;
        float thetaITRT = thetaI + 4.0f * scaleAngleRad;
        float weightR = nR->weight(cosThetaI);
        float weightTT = nTT->weight(cosThetaI);
        float weightTRT = nTRT->weight(cosThetaI);
        const Azimuthal *lobe;
        float v, theta;
        float target = xiNx * (weightR + weightTT + weightTRT);
        if (target < weightR) {
            v = vR; theta = thetaIR; lobe = nR.get();
        } else if (target < weightR + weightTT) {
            v = vTT; theta = thetaITT; lobe = nTT.get();
        } else {
            v = vTRT; theta = thetaITRT; lobe = nTRT.get();
        }
        float sinThetaO = sampleM(v, std::sin(theta), std::cos(theta), xiMx, xiMy);
        float cosThetaO = trigInverse(sinThetaO);
        float thetaO = std::asin(clampv(sinThetaO, -1.0f, 1.0f));
        float thetaD = (thetaO - thetaI) * 0.5f;
        float cosThetaD = std::cos(thetaD);
        float phi;
        lobe->sample(cosThetaD, xiNy, phi);
        float sinPhi = std::sin(phi);
        float cosPhi = std::cos(phi);
        bool choseSpecular = true;
        float probSpecular = 1 - ext.eval(wi.z);
        probSpecular = (probSpecular * specularSamplingWeight) /
                       (probSpecular * specularSamplingWeight +
                        (1 - probSpecular) * (1 - specularSamplingWeight));
        if (sy < probSpecular) {
        } else {
            choseSpecular = false;
        }
        if (choseSpecular) {
            wo = V3(sinPhi * cosThetaO, sinThetaO, cosPhi * cosThetaO);
            type = EDeltaReflection;
        } else {
            type = EDiffuseReflection;
            wo = squareToCosineHemisphere(sx, sy);
        }
        pdfOut = pdf();
        if (pdfOut <= 0)
            return Spec(0.0f);
        return eval(wi, wo) / pdfOut;
    }

    static float sampleM(float v, float sinThetaI, float cosThetaI, float xi1, float xi2) {
        /* :582-592 */
        float cosTheta = 1.0f + v * std::log(xi1 + (1.0f - xi1) * std::exp(-2.0f / v));
        float sinTheta = trigInverse(cosTheta);
        float cosPhi = std::cos(2 * kPi * xi2);
        return -cosTheta * sinThetaI + sinTheta * cosPhi * cosThetaI;
    }
};

/* ------------------------------------------------------------------ */
/* kajiyakay.cpp:60-273                                                 */
/* ------------------------------------------------------------------ */
struct KajiyaKay {
    Spec kd{0.5f}, ks{0.2f};
    float exponent = 30.0f, specularSamplingWeight = 0;
    void configure() { /* :80-107 */
        Spec sum = ks + kd;
        float actualMax = sum.max();
        if (actualMax > 1.0f) {
            float scale = 0.99f * (1.0f / actualMax);
            ks *= scale;
            kd *= scale;
        }
        float dAvg = kd.getLuminance(), sAvg = ks.getLuminance();
        specularSamplingWeight = sAvg / (dAvg + sAvg);
    }
    Spec eval(const V3 &wi, const V3 &wo) const { /* :122-180 */
        if (wi.z <= 0 || wo.z <= 0)
            return Spec(0.0f);
        Spec result(0.0f);
        float tl = std::abs(wi.x), te = std::abs(wo.x);
        float sin_tl = std::sqrt(1 - tl * tl), sin_te = std::sqrt(1 - te * te);
        float a = tl * te + sin_tl * sin_te;
        if (a > 0.0f && wi.x * wo.x < 0) {
            Spec res = 0.15f * ks * ((exponent + 2) * kInvFourPi * std::pow(a, exponent));
            result += res;
        }
        result += kd * kInvPi;
        return result * wo.z;
    }
    float pdf(const V3 &wi, const V3 &wo) const { /* :182-214 */
        if (wi.z <= 0 || wo.z <= 0)
            return 0.0f;
        float diffuseProb = kInvPi * wo.z, specProb = 0.0f;
        float a = dot(wo, V3(-wi.x, -wi.y, wi.z));
        if (a > 0)
            specProb = std::pow(a, exponent) * (exponent + 1.0f) / (2.0f * kPi);
        return specularSamplingWeight * specProb + (1 - specularSamplingWeight) * diffuseProb;
    }
    Spec sample(const V3 &wi, float sx, float sy, V3 &wo, float &pdfOut, uint32_t &type) const {
        /* :216-265 */
        bool choseSpecular = true;
        if (sx <= specularSamplingWeight) {
            sx /= specularSamplingWeight;
        } else {
            sx = (sx - specularSamplingWeight) / (1 - specularSamplingWeight);
            choseSpecular = false;
        }
        if (choseSpecular) {
            V3 R(-wi.x, -wi.y, wi.z);
            float sinAlpha = std::sqrt(1 - std::pow(sy, 2 / (exponent + 1)));
            float cosAlpha = std::pow(sy, 1 / (exponent + 1));
            float phi = (2.0f * kPi) * sx;
            V3 localDir(sinAlpha * std::cos(phi), sinAlpha * std::sin(phi), cosAlpha);
            wo = frameFromNormal(R).toWorld(localDir);
            type = EGlossyReflection;
            if (wo.z <= 0) {
                pdfOut = 0.0f;
                return Spec(0.0f);
            }
        } else {
            wo = squareToCosineHemisphere(sx, sy);
            type = EDiffuseReflection;
        }
        pdfOut = pdf(wi, wo);
        if (pdfOut == 0)
            return Spec(0.0f);
        return eval(wi, wo) / pdfOut;
    }
};

/* ------------------------------------------------------------------ */
/* microfacet.h:36-720 -- MicrofacetDistribution (isotropic instances)  */
/* ------------------------------------------------------------------ */
namespace mathx {
inline float fastexp(float v) { return (float) ::exp((double) v); } /* math.h:185-199 (Linux) */
inline float fastlog(float v) { return (float) ::log((double) v); }
inline float signum(float v) { return std::copysign(1.0f, v); }     /* math.h:270-276 */
float erfinv(float x) { /* math.cpp:25-53 */
    float w = -fastlog((1.0f - x) * (1.0f + x)), p;
    if (w < 5.0f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = 3.43273939e-07f + p * w;
        p = -3.5233877e-06f + p * w;
        p = -4.39150654e-06f + p * w;
        p = 0.00021858087f + p * w;
        p = -0.00125372503f + p * w;
        p = -0.00417768164f + p * w;
        p = 0.246640727f + p * w;
        p = 1.50140941f + p * w;
    } else {
        w = std::sqrt(w) - 3.0f;
        p = -0.000200214257f;
        p = 0.000100950558f + p * w;
        p = 0.00134934322f + p * w;
        p = -0.00367342844f + p * w;
        p = 0.00573950773f + p * w;
        p = -0.0076224613f + p * w;
        p = 0.00943887047f + p * w;
        p = 1.00167406f + p * w;
        p = 2.83297682f + p * w;
    }
    return p * x;
}
float erf(float x) { /* math.cpp:55-72 (A&S 7.1.26) */
    const float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f;
    const float a4 = -1.453152027f, a5 = 1.061405429f, p = 0.3275911f;
    float sign = signum(x);
    x = std::abs(x);
    float t = 1.0f / (1.0f + p * x);
    float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * fastexp(-x * x);
    return sign * y;
}
float hypot2(float a, float b) { /* math.cpp:74-86 */
    float r;
    if (std::abs(a) > std::abs(b)) {
        r = b / a;
        r = std::abs(a) * std::sqrt(1.0f + r * r);
    } else if (b != 0.0f) {
        r = a / b;
        r = std::abs(b) * std::sqrt(1.0f + r * r);
    } else {
        r = 0.0f;
    }
    return r;
}
} // namespace mathx

struct Microfacet {
    enum EType { EBeckmann = 0, EGGX = 1, EPhong = 2 };
    int type = EBeckmann;
    float alpha = 0.1f, exponent = 0.0f;
    bool sampleVisible = true;

    Microfacet() {}
    Microfacet(int t, float a, bool sv) : type(t), alpha(std::max(a, 1e-4f)), sampleVisible(sv) { /* :67-75 */
        if (type == EPhong) exponent = std::max(2.0f / (alpha * alpha) - 2.0f, 0.0f); /* :701-704 */
    }
    float eval(const V3 &m) const { /* :190-237 */
        if (m.z <= 0) return 0.0f;
        float cosTheta2 = m.z * m.z;
        float beckmannExponent = ((m.x * m.x) / (alpha * alpha) + (m.y * m.y) / (alpha * alpha)) / cosTheta2;
        float result;
        if (type == EBeckmann) {
            result = mathx::fastexp(-beckmannExponent) / (kPi * alpha * alpha * cosTheta2 * cosTheta2);
        } else if (type == EGGX) {
            float root = (1.0f + beckmannExponent) * cosTheta2;
            result = 1.0f / (kPi * alpha * alpha * root * root);
        } else {
            result = std::sqrt((exponent + 2) * (exponent + 2)) * kInvTwoPi * std::pow(m.z, exponent);
        }
        if (result * m.z < 1e-20f) result = 0;
        return result;
    }
    float smithG1(const V3 &v, const V3 &m) const { /* :451-484 */
        if (dot(v, m) * v.z <= 0) return 0.0f;
        float temp = 1 - v.z * v.z;
        float tanTheta = std::abs(temp <= 0.0f ? 0.0f : std::sqrt(temp) / v.z);
        if (tanTheta == 0.0f) return 1.0f;
        if (type == EGGX) {
            float root = alpha * tanTheta;
            return 2.0f / (1.0f + mathx::hypot2(1.0f, root));
        }
        float a = 1.0f / (alpha * tanTheta);
        if (a >= 1.6f) return 1.0f;
        float aSqr = a * a;
        return (3.535f * a + 2.181f * aSqr) / (1.0f + 2.276f * a + 2.577f * aSqr);
    }
    float pdf(const V3 &wi, const V3 &m) const { /* :275-280, :436-441, :396-400 */
        if (sampleVisible) {
            if (wi.z == 0) return 0.0f;
            return smithG1(wi, m) * absDot(wi, m) * eval(m) / std::abs(wi.z);
        }
        return eval(m) * m.z;
    }
    void sampleVisible11(float thetaI, float sx, float sy, float &slx, float &sly) const { /* :567-686 */
        const float SQRT_PI_INV = 1 / std::sqrt(kPi);
        if (type == EBeckmann) {
            if (thetaI < 1e-4f) {
                float r = std::sqrt(-mathx::fastlog(1.0f - sx));
                float ang = 2 * kPi * sy;
                slx = r * std::cos(ang);
                sly = r * std::sin(ang);
                return;
            }
            float tanThetaI = std::tan(thetaI), cotThetaI = 1 / tanThetaI;
            float a = -1, c = mathx::erf(cotThetaI);
            float sample_x = std::max(sx, 1e-6f);
            float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
            float b = c - (1 + c) * std::pow(1 - sample_x, fit);
            float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * std::exp(-cotThetaI * cotThetaI));
            for (int it = 1; it < 10; ++it) {
                if (!(b >= a && b <= c)) b = 0.5f * (a + c);
                float invErf = mathx::erfinv(b);
                float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * std::exp(-invErf * invErf)) - sample_x;
                float derivative = normalization * (1 - invErf * tanThetaI);
                if (std::abs(value) < 1e-5f) break;
                if (value > 0) c = b;
                else a = b;
                b -= value / derivative;
            }
            slx = mathx::erfinv(b);
            sly = mathx::erfinv(2.0f * std::max(sy, 1e-6f) - 1.0f);
            return;
        }
        if (thetaI < 1e-4f) {
            float r = safe_sqrt(sx / (1 - sx));
            float ang = 2 * kPi * sy;
            slx = r * std::cos(ang);
            sly = r * std::sin(ang);
            return;
        }
        float tanThetaI = std::tan(thetaI), a = 1 / tanThetaI;
        float G1 = 2.0f / (1.0f + safe_sqrt(1.0f + 1.0f / (a * a)));
        float A = 2.0f * sx / G1 - 1.0f;
        if (std::abs(A) == 1) A -= mathx::signum(A) * kEpsilon;
        float tmp = 1.0f / (A * A - 1.0f), B = tanThetaI;
        float D = safe_sqrt(B * B * tmp * tmp - (A * A - B * B) * tmp);
        float x1 = B * tmp - D, x2 = B * tmp + D;
        slx = (A < 0.0f || x2 > 1.0f / tanThetaI) ? x1 : x2;
        float S;
        if (sy > 0.5f) {
            S = 1.0f;
            sy = 2.0f * (sy - 0.5f);
        } else {
            S = -1.0f;
            sy = 2.0f * (0.5f - sy);
        }
        float z = (sy * (sy * (sy * -0.365728915865723f + 0.790235037209296f) - 0.424965825137544f) +
                   0.000152998850436920f) /
                  (sy * (sy * (sy * (sy * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) + 1.0f) -
                   0.539825872510702f);
        sly = S * z * std::sqrt(1.0f + slx * slx);
    }
    V3 sample(const V3 &wi_, float sx, float sy) const { /* :258-269 */
        if (sampleVisible) { /* sampleVisible :355-393 */
            V3 wi = normalize(V3(alpha * wi_.x, alpha * wi_.y, wi_.z));
            float theta = 0, phi = 0;
            if (wi.z < 0.99999f) {
                theta = std::acos(wi.z);
                phi = std::atan2(wi.y, wi.x);
            }
            float sinPhi = std::sin(phi), cosPhi = std::cos(phi);
            float slx, sly;
            sampleVisible11(theta, sx, sy, slx, sly);
            float rx = cosPhi * slx - sinPhi * sly, ry = sinPhi * slx + cosPhi * sly;
            rx *= alpha;
            ry *= alpha;
            float normalization = 1.0f / std::sqrt(rx * rx + ry * ry + 1.0f);
            return V3(-rx * normalization, -ry * normalization, normalization);
        }
        /* sampleAll (:291-385), isotropic */
        float cosThetaM, sinPhiM, cosPhiM;
        if (type == EPhong) {
            float phiM = (2.0f * kPi) * sy;
            sinPhiM = std::sin(phiM);
            cosPhiM = std::cos(phiM);
            cosThetaM = std::pow(sx, 1.0f / (exponent + 2.0f));
        } else {
            float ang = (2.0f * kPi) * sy;
            sinPhiM = std::sin(ang);
            cosPhiM = std::cos(ang);
            float alphaSqr = alpha * alpha;
            float tanThetaMSqr = type == EBeckmann ? alphaSqr * -mathx::fastlog(1.0f - sx)
                                                   : alphaSqr * sx / (1.0f - sx);
            cosThetaM = 1.0f / std::sqrt(1.0f + tanThetaMSqr);
        }
        float sinThetaM = std::sqrt(std::max(0.0f, 1 - cosThetaM * cosThetaM));
        return V3(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
    }
};

/* ------------------------------------------------------------------ */
/* roughplastic.cpp:197-506 (constant textures, both components)       */
/* ------------------------------------------------------------------ */
struct RoughPlastic {
    int type = 0;
    bool sampleVisible = true, nonlinear = false;
    float alphaTex = 0.1f; /* ConstantFloatTexture(distr.getAlpha()) */
    float eta = 1.49f, invEta2 = 0, specularSamplingWeight = 0;
    Spec diffuse{0.5f}, specular{1.0f};
    RoughTransmittance ext, internal;

    float alphaEval() const { return Spec(alphaTex).average(); } /* m_alpha->eval(its).average() */

    bool configure(const std::string &datDir, std::string &err) { /* :268-299 */
        float mx = specular.max();
        if (mx > 1.0f) specular *= 0.99f * (1.0f / mx);
        mx = diffuse.max();
        if (mx > 1.0f) diffuse *= 0.99f * (1.0f / mx);
        float dAvg = diffuse.getLuminance(), sAvg = specular.getLuminance();
        specularSamplingWeight = sAvg / (dAvg + sAvg);
        invEta2 = 1.0f / (eta * eta);
        const char *names[3] = {"beckmann", "ggx", "phong"};
        std::string path = datDir + "/" + names[type] + ".dat";
        if (!ext.load(path)) { err = "cannot load " + path; return false; }
        float etaC = eta < 1 ? 1 / eta : eta;
        if (etaC < ext.etaMin || etaC > ext.etaMax) { err = "eta outside the supported range"; return false; }
        if (alphaEval() < ext.alphaMin || alphaEval() > ext.alphaMax) {
            err = "alpha outside the supported range";
            return false;
        }
        internal = ext;
        ext.setEta(eta);
        internal.setEta(1 / eta);
        ext.setAlpha(alphaEval());
        return true;
    }
    Microfacet distr() const { return Microfacet(type, alphaEval(), sampleVisible); }

    Spec eval(const V3 &wi, const V3 &wo) const { /* :305-360 */
        if (wi.z <= 0 || wo.z <= 0) return Spec(0.0f);
        Microfacet d = distr();
        Spec result(0.0f);
        {
            V3 H = normalize(wo + wi);
            float D = d.eval(H);
            float F = fresnelDielectricExt(dot(wi, H), eta);
            float G = d.smithG1(wi, H) * d.smithG1(wo, H);
            float value = F * D * G / (4.0f * wi.z);
            result += specular * value;
        }
        {
            Spec diff = diffuse;
            float T12 = ext.eval(wi.z), T21 = ext.eval(wo.z);
            float Fdr = 1 - internal.evalDiffuse(d.alpha);
            if (nonlinear) {
                for (int i = 0; i < 3; ++i) diff.s[i] /= 1.0f - diff.s[i] * Fdr;
            } else {
                diff /= 1 - Fdr;
            }
            result += diff * (kInvPi * wo.z * T12 * T21 * invEta2);
        }
        return result;
    }
    float pdf(const V3 &wi, const V3 &wo) const { /* :362-436 */
        if (wi.z <= 0 || wo.z <= 0) return 0.0f;
        Microfacet d = distr();
        V3 H = normalize(wo + wi);
        float probSpecular = 1 - ext.eval(wi.z);
        probSpecular = (probSpecular * specularSamplingWeight) /
                       (probSpecular * specularSamplingWeight + (1 - probSpecular) * (1 - specularSamplingWeight));
        float probDiffuse = 1 - probSpecular;
        float dwh_dwo = 1.0f / (4.0f * dot(wo, H));
        float prob = d.pdf(wi, H);
        float result = prob * dwh_dwo * probSpecular;
        result += probDiffuse * (kInvPi * wo.z);
        return result;
    }
    Spec sample(const V3 &wi, float sx, float sy, V3 &wo, float &pdfOut, uint32_t &type_) const { /* :438-499 */
        pdfOut = 0;
        type_ = 0;
        if (wi.z <= 0) return Spec(0.0f);
        bool choseSpecular = true;
        Microfacet d = distr();
        float probSpecular = 1 - ext.eval(wi.z);
        probSpecular = (probSpecular * specularSamplingWeight) /
                       (probSpecular * specularSamplingWeight + (1 - probSpecular) * (1 - specularSamplingWeight));
        if (sy < probSpecular) {
            sy /= probSpecular;
        } else {
            sy = (sy - probSpecular) / (1 - probSpecular);
            choseSpecular = false;
        }
        if (choseSpecular) {
            V3 m = d.sample(wi, sx, sy);
            wo = 2 * dot(wi, m) * m - wi;
            type_ = EGlossyReflection;
            if (wo.z <= 0) return Spec(0.0f);
        } else {
            type_ = EDiffuseReflection;
            wo = squareToCosineHemisphere(sx, sy);
        }
        pdfOut = pdf(wi, wo);
        if (pdfOut == 0) return Spec(0.0f);
        return eval(wi, wo) / pdfOut;
    }
};

/* ------------------------------------------------------------------ */
/* marschnerdielectric.cpp:145-529 -- thin-sheet "MarschnerDielectric"  */
/* Restated with its measure / component gates; the integrator calls     */
/* eval/pdf with ESolidAngle, typeMask EAll, component -1.               */
/* ------------------------------------------------------------------ */
struct MarschnerDielectric {
    enum EMeasure { ESolidAngle = 1, EDiscrete = 3 };
    float eta = 1.501f, specularSamplingWeight = 0;
    Spec diffuse{0.5f}, specR{0.1f}, specT{0.1f};
    float exponent = 30.0f;
    static constexpr float DeltaEpsilon = 1e-3f;                /* constants.h:31 */

    void configure() { /* :189-211 */
        float mx = specR.max();
        if (mx > 1.0f) specR *= 0.99f * (1.0f / mx);
        mx = specT.max();
        if (mx > 1.0f) specT *= 0.99f * (1.0f / mx);
        float dAvg = diffuse.getLuminance(), sAvg = specR.getLuminance(), tAvg = specT.getLuminance();
        specularSamplingWeight = (sAvg + tAvg) / (dAvg + sAvg + tAvg);
    }
    static V3 reflect(const V3 &wi) { return V3(-wi.x, -wi.y, wi.z); }
    static V3 transmit(const V3 &wi) { return V3(-wi.x, -wi.y, -wi.z); }
    float fresnelR(const V3 &wi) const {
        float R = fresnelDielectricExt(std::abs(wi.z), eta), T = 1 - R;
        if (R < 1) R += T * T * R / (1 - R * R);
        return R;
    }
    Spec eval(const V3 &wi, const V3 &wo, EMeasure measure = ESolidAngle) const { /* :232-283 */
        const bool sampleReflection = measure == EDiscrete, sampleTransmission = measure == EDiscrete;
        const bool hasDiffuse = true;
        if (wi.z <= 0 || wo.z <= 0 || measure != ESolidAngle) return Spec(0.0f);
        Spec result(0.0f);
        float R = fresnelR(wi);
        if (wi.z * wo.z >= 0) {
            if (!sampleReflection || std::abs(dot(reflect(wi), wo) - 1) > DeltaEpsilon) return Spec(0.0f);
            float tl = std::abs(wi.x), te = std::abs(wo.x);
            float alpha = tl * te + std::sqrt(1 - tl * tl) * std::sqrt(1 - te * te);
            if (alpha > 0.0f && wi.x * wo.x < 0)
                result += 0.15f * specR * ((exponent + 2) * kInvFourPi * std::pow(alpha, exponent));
        } else {
            if (!sampleTransmission || std::abs(dot(transmit(wi), wo) - 1) > DeltaEpsilon) return Spec(0.0f);
            result += specT * (1 - R);
        }
        if (hasDiffuse) result += diffuse * kInvPi;
        return result * wo.z;
    }
    float pdf(const V3 &wi, const V3 &wo, EMeasure measure = ESolidAngle) const { /* :285-358 */
        const bool sampleReflection = measure == EDiscrete, sampleTransmission = measure == EDiscrete;
        const bool hasDiffuse = true;
        if (measure != ESolidAngle || wi.z <= 0 || wo.z <= 0 ||
            (!sampleReflection && !sampleTransmission && !hasDiffuse))
            return 0.0f;
        float diffuseProb = kInvPi * wo.z, specProb = 0.0f;
        if (sampleReflection) {
            float alpha = dot(wo, reflect(wi));
            if (alpha > 0) specProb = std::pow(alpha, exponent) * (exponent + 1.0f) / (2.0f * kPi);
        }
        float R = fresnelR(wi), tProb = 0.0f, rProb = 0.0f;
        if (wi.z * wo.z >= 0) {
            if (!sampleReflection || std::abs(dot(reflect(wi), wo) - 1) > DeltaEpsilon) return diffuseProb;
            tProb = sampleTransmission ? R : 1.0f;
        } else {
            if (!sampleTransmission || std::abs(dot(transmit(wi), wo) - 1) > DeltaEpsilon) return diffuseProb;
            rProb = sampleReflection ? 1 - R : 1.0f;
        }
        if (sampleReflection) return specularSamplingWeight * specProb * rProb + (1 - specularSamplingWeight) * diffuseProb;
        if (sampleTransmission) return specularSamplingWeight * specProb * tProb + (1 - specularSamplingWeight) * diffuseProb;
        return diffuseProb;
    }
    Spec sample(const V3 &wi, float sx, float sy, V3 &wo, float &pdfOut, uint32_t &type) const { /* :424-500 */
        bool choseSpecular = true;
        if (sx <= specularSamplingWeight) {
            sx /= specularSamplingWeight;
        } else {
            sx = (sx - specularSamplingWeight) / (1 - specularSamplingWeight);
            choseSpecular = false;
        }
        if (choseSpecular) {
            float R = fresnelR(wi);
            if (sx <= R) {
                type = EDeltaReflection;
                wo = reflect(wi);
                pdfOut = R;
                return specR;
            }
            type = ENull;
            wo = transmit(wi);
            pdfOut = 1 - R;
            return specT;
        }
        wo = squareToCosineHemisphere(sx, sy);
        type = EDiffuseReflection;
        pdfOut = pdf(wi, wo);
        if (pdfOut == 0) return Spec(0.0f);
        return eval(wi, wo) / pdfOut;
    }
};

/* ------------------------------------------------------------------ */
/* thindielectric.cpp:70-252 (constant textures)                       */
/* ------------------------------------------------------------------ */
struct ThinDielectric {
    float eta = 1.5046f;
    Spec specR{1.0f}, specT{1.0f};
    void configure() { /* :110-125 */
        float mx = specR.max();
        if (mx > 1.0f) specR *= 0.99f * (1.0f / mx);
        mx = specT.max();
        if (mx > 1.0f) specT *= 0.99f * (1.0f / mx);
    }
    float fresnelR(const V3 &wi) const {
        float R = fresnelDielectricExt(std::abs(wi.z), eta), T = 1 - R;
        if (R < 1) R += T * T * R / (1 - R * R);
        return R;
    }
    /* eval / pdf need EDiscrete for both components (:151-201): zero for the
       integrator's solid-angle queries, which it never makes (no ESmooth) */
    Spec eval(const V3 &, const V3 &) const { return Spec(0.0f); }
    float pdf(const V3 &, const V3 &) const { return 0.0f; }
    Spec sample(const V3 &wi, float sx, float, V3 &wo, float &pdfOut, uint32_t &type) const { /* :203-232 */
        float R = fresnelR(wi);
        if (sx <= R) {
            type = EDeltaReflection;
            wo = V3(-wi.x, -wi.y, wi.z);
            pdfOut = R;
            return specR;
        }
        type = ENull;
        wo = V3(-wi.x, -wi.y, -wi.z);
        pdfOut = 1 - R;
        return specT;
    }
};

#include "mesh_bsdf.h"

/* ------------------------------------------------------------------ */
/* diffuse.cpp:60-140 (SmoothDiffuse: a constant or checkerboard reflectance) */
/* ------------------------------------------------------------------ */
struct SmoothDiffuse {
    Spec reflectance{0.5f};
    bool textured = false;
    Checkerboard tex;
    void configure() { /* ensureEnergyConservation (bsdf.cpp:88-112): a ScalingTexture */
        float mx = maxReflectance();
        if (mx > 1.0f) {
            const float scale = 0.99f * (1.0f / mx);
            reflectance *= scale;
            tex.color0 *= scale;
            tex.color1 *= scale;
        }
    }
    float maxReflectance() const { return textured ? tex.maximum().max() : reflectance.max(); }
    Spec refl(const float *uv) const { return textured ? tex.eval(uv ? uv[0] : 0.0f, uv ? uv[1] : 0.0f) : reflectance; }
    Spec eval(const V3 &wi, const V3 &wo, const float *uv = nullptr) const {
        if (wi.z <= 0 || wo.z <= 0) return Spec(0.0f);
        return refl(uv) * (kInvPi * wo.z);
    }
    float pdf(const V3 &wi, const V3 &wo) const {
        if (wi.z <= 0 || wo.z <= 0) return 0.0f;
        return kInvPi * wo.z;
    }
    Spec sample(const V3 &wi, float sx, float sy, V3 &wo, float &pdfOut, uint32_t &type,
                const float *uv = nullptr) const {
        pdfOut = 0;
        type = 0;
        if (wi.z <= 0) return Spec(0.0f);
        wo = squareToCosineHemisphere(sx, sy);
        type = EDiffuseReflection;
        pdfOut = kInvPi * wo.z;
        return refl(uv);
    }
};

/* One BSDF instance: of a hair shape (the default is Shape::configure's 0.5
   Lambertian, shape.cpp:57-64) or of a mesh shape.  uv = the intersection's
   texture coordinates (only the checkerboard diffuse reads them; NULL = (0, 0)). */
struct BsdfInst {
    int kind = 5; /* 0 marschner, 1 kajiyakay, 2 roughplastic, 3 marschnerdielectric, 4 thindielectric, 5 diffuse,
                     6 plastic, 7 twosided */
    Marschner marschner;
    KajiyaKay kk;
    RoughPlastic rp;
    MarschnerDielectric md;
    ThinDielectric td;
    SmoothDiffuse df;
    SmoothPlastic pl;
    std::shared_ptr<BsdfInst> nested[2]; /* twosided.cpp:84-89: nested[1] = nested[0] when absent */
    /* the combined type has an ESmooth component (path.cpp:175 gate) */
    bool smooth() const {
        if (kind == 7) return nested[0]->smooth() || nested[1]->smooth();
        return kind != 4 && !(kind == 5 && df.maxReflectance() <= 0);
    }
    Spec eval(const V3 &wi, const V3 &wo, const float *uv = nullptr) const {
        switch (kind) {
        case 0: return marschner.eval(wi, wo);
        case 1: return kk.eval(wi, wo);
        case 2: return rp.eval(wi, wo);
        case 3: return md.eval(wi, wo);
        case 4: return td.eval(wi, wo);
        case 6: return pl.eval(wi, wo);
        case 7: /* twosided.cpp:108-120 */
            if (wi.z > 0) return nested[0]->eval(wi, wo, uv);
            return nested[1]->eval(V3(wi.x, wi.y, -wi.z), V3(wo.x, wo.y, -wo.z), uv);
        default: return df.eval(wi, wo, uv);
        }
    }
    float pdf(const V3 &wi, const V3 &wo, const float *uv = nullptr) const {
        switch (kind) {
        case 0: return marschner.pdf();
        case 1: return kk.pdf(wi, wo);
        case 2: return rp.pdf(wi, wo);
        case 3: return md.pdf(wi, wo);
        case 4: return td.pdf(wi, wo);
        case 6: return pl.pdf(wi, wo);
        case 7: /* :122-134 */
            if (wi.z > 0) return nested[0]->pdf(wi, wo, uv);
            return nested[1]->pdf(V3(wi.x, wi.y, -wi.z), V3(wo.x, wo.y, -wo.z), uv);
        default: return df.pdf(wi, wo);
        }
    }
    Spec sample(const V3 &wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type,
                const float *uv = nullptr) const {
        switch (kind) {
        case 0: return marschner.sample(wi, sx, sy, wo, pdf, type);
        case 1: return kk.sample(wi, sx, sy, wo, pdf, type);
        case 2: return rp.sample(wi, sx, sy, wo, pdf, type);
        case 3: return md.sample(wi, sx, sy, wo, pdf, type);
        case 4: return td.sample(wi, sx, sy, wo, pdf, type);
        case 6: return pl.sample(wi, sx, sy, wo, pdf, type);
        case 7: { /* :161-183 */
            const bool flipped = wi.z < 0;
            const V3 w = flipped ? V3(wi.x, wi.y, -wi.z) : wi;
            Spec result = nested[flipped ? 1 : 0]->sample(w, sx, sy, wo, pdf, type, uv);
            if (flipped && !result.isZero() && pdf != 0) wo.z *= -1;
            return result;
        }
        default: return df.sample(wi, sx, sy, wo, pdf, type, uv);
        }
    }
};

/* ------------------------------------------------------------------ */
/* Hair shape: hair.cpp                                                 */
/* ------------------------------------------------------------------ */
struct HairGeom {
    std::vector<V3> v;
    std::vector<uint8_t> start; /* size n+1, last = 1 */
    /* several HairShapes, concatenated: shape k owns vertices [shapeFirst[k], shapeFirst[k+1]) */
    std::vector<uint32_t> shapeFirst;
    std::vector<float> shapeRadius;
    std::vector<int> shapeBsdf;
    uint32_t shapeOf(uint32_t iv) const {
        return (uint32_t) (std::upper_bound(shapeFirst.begin(), shapeFirst.end(), iv) - shapeFirst.begin() - 1);
    }
    float radius(uint32_t iv) const { return shapeRadius[shapeOf(iv)]; }

    V3 firstVertex(uint32_t iv) const { return v[iv]; }
    V3 secondVertex(uint32_t iv) const { return v[iv + 1]; }
    V3d firstVertexD(uint32_t iv) const { return V3d(v[iv]); }
    V3d secondVertexD(uint32_t iv) const { return V3d(v[iv + 1]); }
    V3d prevVertexD(uint32_t iv) const { return V3d(v[iv - 1]); }
    V3d nextVertexD(uint32_t iv) const { return V3d(v[iv + 2]); }
    bool prevSegmentExists(uint32_t iv) const { return !start[iv]; }
    bool nextSegmentExists(uint32_t iv) const { return !start[iv + 2]; }
    V3 tangent(uint32_t iv) const { return normalize(secondVertex(iv) - firstVertex(iv)); }
    V3 prevTangent(uint32_t iv) const { return normalize(firstVertex(iv) - v[iv - 1]); }
    V3 nextTangent(uint32_t iv) const { return normalize(v[iv + 2] - secondVertex(iv)); }
    V3d tangentD(uint32_t iv) const { return normalize(V3d(secondVertex(iv)) - V3d(firstVertex(iv))); }
    V3d prevTangentD(uint32_t iv) const { return normalize(firstVertexD(iv) - prevVertexD(iv)); }
    V3d nextTangentD(uint32_t iv) const { return normalize(nextVertexD(iv) - secondVertexD(iv)); }
    V3 firstMiterNormal(uint32_t iv) const {
        return prevSegmentExists(iv) ? normalize(prevTangent(iv) + tangent(iv)) : tangent(iv);
    }
    V3 secondMiterNormal(uint32_t iv) const {
        return nextSegmentExists(iv) ? normalize(tangent(iv) + nextTangent(iv)) : tangent(iv);
    }
    V3d firstMiterNormalD(uint32_t iv) const {
        return prevSegmentExists(iv) ? normalize(prevTangentD(iv) + tangentD(iv)) : tangentD(iv);
    }
    V3d secondMiterNormalD(uint32_t iv) const {
        return nextSegmentExists(iv) ? normalize(tangentD(iv) + nextTangentD(iv)) : tangentD(iv);
    }

    /* hair.cpp:246-286 */
    static bool intersectCylPlane(V3 planePt, V3 planeNrml, V3 cylPt, V3 cylD, float radius,
                                  V3 &center, V3 *axes, float *lengths) {
        if (absDot(planeNrml, cylD) < kEpsilon)
            return false;
        V3 B, A = cylD - dot(cylD, planeNrml) * planeNrml;
        float length = A.length();
        if (length > kEpsilon && planeNrml != cylD) {
            A /= length;
            B = cross(planeNrml, A);
        } else {
            coordinateSystem(planeNrml, A, B);
        }
        V3 delta = planePt - cylPt, deltaProj = delta - cylD * dot(delta, cylD);
        float aDotD = dot(A, cylD);
        float bDotD = dot(B, cylD);
        float c0 = 1 - aDotD * aDotD;
        float c1 = 1 - bDotD * bDotD;
        float c2 = 2 * dot(A, deltaProj);
        float c3 = 2 * dot(B, deltaProj);
        float c4 = dot(delta, deltaProj) - radius * radius;
        float lambda = (c2 * c2 / (4 * c0) + c3 * c3 / (4 * c1) - c4) / (c0 * c1);
        float alpha0 = -c2 / (2 * c0), beta0 = -c3 / (2 * c1);
        lengths[0] = std::sqrt(c1 * lambda);
        lengths[1] = std::sqrt(c0 * lambda);
        center = planePt + alpha0 * A + beta0 * B;
        axes[0] = A;
        axes[1] = B;
        return true;
    }

    /* hair.cpp:349-378 getAABB(index) with radius*(1-Epsilon) */
    void segmentAABB(uint32_t iv, V3 &mn, V3 &mx) const {
        mn = V3(kInf);
        mx = V3(-kInf);
        V3 center, axes[2];
        float lengths[2] = {0.0f, 0.0f};
        for (int end = 0; end < 2; ++end) {
            bool ok = end == 0
                          ? intersectCylPlane(firstVertex(iv), firstMiterNormal(iv), firstVertex(iv),
                                              tangent(iv), radius(iv) * (1 - kEpsilon), center, axes, lengths)
                          : intersectCylPlane(secondVertex(iv), secondMiterNormal(iv), secondVertex(iv),
                                              tangent(iv), radius(iv) * (1 - kEpsilon), center, axes, lengths);
            (void) ok;
            axes[0] *= lengths[0];
            axes[1] *= lengths[1];
            for (int i = 0; i < 3; ++i) {
                float range = std::sqrt(axes[0][i] * axes[0][i] + axes[1][i] * axes[1][i]);
                mn[i] = std::min(mn[i], center[i] - range);
                mx[i] = std::max(mx[i], center[i] + range);
            }
        }
    }

    /* hair.cpp:485-548 HairKDTree::intersect */
    bool intersect(const V3 &o, const V3 &d, uint32_t iv, float mint, float maxt, float &t,
                   V3 *pOut) const {
        V3d axis = tangentD(iv);
        V3d rayO(o), rayD(d);
        V3d v1 = firstVertexD(iv);
        V3d relOrigin = rayO - v1;
        V3d projOrigin = relOrigin - dot(axis, relOrigin) * axis;
        V3d projDirection = rayD - dot(axis, rayD) * axis;
        const double A = projDirection.lengthSquared();
        const double B = 2 * dot(projOrigin, projDirection);
        const float r = radius(iv);
        const double C = projOrigin.lengthSquared() - r * r;
        double nearT, farT;
        if (!solveQuadraticDouble(A, B, C, nearT, farT))
            return false;
        if (!(nearT <= maxt && farT >= mint))
            return false;
        V3d pointNear = rayO + rayD * nearT;
        V3d pointFar = rayO + rayD * farT;
        V3d n1 = firstMiterNormalD(iv);
        V3d n2 = secondMiterNormalD(iv);
        V3d v2 = secondVertexD(iv);
        V3d p;
        if (dot(pointNear - v1, n1) >= 0 && dot(pointNear - v2, n2) <= 0 && nearT >= mint) {
            p = rayO + rayD * nearT;
            t = (float) nearT;
        } else if (dot(pointFar - v1, n1) >= 0 && dot(pointFar - v2, n2) <= 0) {
            if (farT > maxt)
                return false;
            p = rayO + rayD * farT;
            t = (float) farT;
        } else {
            return false;
        }
        if (pOut)
            *pOut = V3((float) p.x, (float) p.y, (float) p.z);
        return true;
    }
};

/* ------------------------------------------------------------------ */
/* Ray + AABB (core/ray.h, core/aabb.h:308-338)                         */
/* ------------------------------------------------------------------ */
struct Ray {
    V3 o, d, dRcp;
    float mint, maxt;
    Ray() : mint(kEpsilon), maxt(kInf) {}
    Ray(const V3 &o_, const V3 &d_, float mint_, float maxt_) : o(o_), d(d_), mint(mint_), maxt(maxt_) {
        for (int i = 0; i < 3; ++i) dRcp[i] = (float) 1 / d[i];
    }
    V3 at(float t) const { return o + t * d; }
};

struct AABB {
    V3 min{kInf}, max{-kInf};
    bool rayIntersect(const Ray &ray, float &nearT, float &farT) const {
        nearT = -kInf;
        farT = kInf;
        for (int i = 0; i < 3; i++) {
            const float origin = ray.o[i];
            const float minVal = min[i], maxVal = max[i];
            if (ray.d[i] == 0) {
                if (origin < minVal || origin > maxVal)
                    return false;
            } else {
                float t1 = (minVal - origin) * ray.dRcp[i];
                float t2 = (maxVal - origin) * ray.dRcp[i];
                if (t1 > t2)
                    std::swap(t1, t2);
                nearT = std::max(t1, nearT);
                farT = std::min(t2, farT);
                if (!(nearT <= farT))
                    return false;
            }
        }
        return true;
    }
    void expandBy(const V3 &p) {
        for (int i = 0; i < 3; ++i) {
            min[i] = std::min(min[i], p[i]);
            max[i] = std::max(max[i], p[i]);
        }
    }
};

struct Hit {
    float t = kInf;
    uint32_t iv = 0;
    V3 p;
    /* mesh hits (mesh_geom.h): kind 1 = triangle (shape = mesh, prim = triangle, u/v = barycentrics),
       kind 2 = rectangle (shape = rectangle, u/v = local x/y) */
    int kind = 0;
    uint32_t shape = 0, prim = 0;
    float u = 0, v = 0;
    bool valid() const { return t < kInf; }
};

struct Stats {
    uint64_t rays = 0, shadowRays = 0, nodes = 0, prims = 0, paths = 0, ewaViolations = 0,
             bounces = 0, badSamples = 0;
};

/* kd-tree node (product format; DESIGN.md "Hair kd-tree"):
 *   inner: w0 = (leftChild << 2) | axis, w1 = split (float bits); right = left + 1
 *   leaf : w0 = 0x80000000 | primStart,   w1 = primEnd                              */
struct KDTree {
    std::vector<uint32_t> nodes; /* 2 words per node */
    std::vector<uint32_t> indices;
    bool empty() const { return nodes.empty(); }
};

/* ------------------------------------------------------------------ */
/* Environment map (emitters/envmap.cpp + mipmap.h)                    */
/* ------------------------------------------------------------------ */
struct EnvMap {
    int w = 0, h = 0;
    std::vector<float> texel; /* half-rounded RGB as float, w*h*3 */
    std::vector<float> cdfRows, cdfCols, rowWeights;
    float normalization = 0, scale = 1.0f;
    float pixelSizeX = 0, pixelSizeY = 0;
    bool identity = true;
    float m[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1}, minv[9] = {1, 0, 0, 0, 1, 0, 0, 0, 1};
    V3 bsCenter;
    float bsRadius = 0;
    /* MIP pyramid (mipmap.h:155-302): half-rounded RGB per level, m_sizeRatio, EWA LUT */
    std::vector<std::vector<float>> lev;
    std::vector<int> lw, lh;
    std::vector<float> ratioX, ratioY;
    float lut[64];
    float maxAnisotropy = 10.0f; /* envmap.cpp:142 */

    /* LanczosSincFilter::eval, lobes = 2 (lanczos.cpp:43-55; envmap.cpp:167-172) */
    static float lanczos(float x) {
        x = std::abs(x);
        if (x < kEpsilon) return 1.0f;
        else if (x > 2.0f) return 0.0f;
        float x1 = kPi * x;
        float x2 = x1 / 2.0f;
        return (std::sin(x1) * std::sin(x2)) / (x1 * x2);
    }
    /* Resampler<float> + resampleAndClamp(min 0, max inf) along one axis (rfilter.h:123-280, 437-458) */
    static void resampleAxis(const float *src, size_t sStride, float *dst, size_t dStride, int sourceRes,
                             int targetRes, bool repeat) {
        float filterRadius = 2.0f, scale = 1.0f, invScale = 1.0f;
        if (targetRes < sourceRes) {
            scale = (float) sourceRes / (float) targetRes;
            invScale = 1 / scale;
            filterRadius *= scale;
        }
        const int taps = (int) std::ceil(filterRadius * 2);
        std::vector<float> wts(taps);
        for (int i = 0; i < targetRes; i++) {
            float center = (i + 0.5f) / targetRes * sourceRes;
            int start = (int) std::floor(center - filterRadius + 0.5f);
            float sum = 0;
            for (int j = 0; j < taps; j++) {
                float w = lanczos((start + j + 0.5f - center) * invScale);
                wts[j] = w;
                sum += w;
            }
            float normalization = 1.0f / sum;
            for (int j = 0; j < taps; j++) wts[j] = wts[j] * normalization;
            for (int ch = 0; ch < 3; ++ch) {
                float result = 0;
                for (int j = 0; j < taps; ++j) {
                    int pos = start + j;
                    if (pos < 0 || pos >= sourceRes) pos = repeat ? modulo(pos, sourceRes) : clampv(pos, 0, sourceRes - 1);
                    result += src[sStride * 3 * (size_t) pos + ch] * wts[j];
                }
                result = std::max(0.0f, result);
                dst[dStride * 3 * (size_t) i + ch] = std::min(std::numeric_limits<float>::infinity(), result);
            }
        }
    }
    void buildPyramid(const float *rgb) {
        std::vector<float> bmp((size_t) w * h * 3);
        for (size_t i = 0; i < bmp.size(); ++i) bmp[i] = std::max(rgb[i], 0.0f);
        auto keep = [&](const std::vector<float> &b, int W, int H) {
            std::vector<float> q(b.size());
            for (size_t i = 0; i < b.size(); ++i) q[i] = halfToFloat(floatToHalf(b[i]));
            lev.push_back(q);
            lw.push_back(W);
            lh.push_back(H);
            ratioX.push_back((float) W / (float) w);
            ratioY.push_back((float) H / (float) h);
        };
        lev.clear(), lw.clear(), lh.clear(), ratioX.clear(), ratioY.clear();
        keep(bmp, w, h);
        int W = w, H = h;
        while (W > 1 || H > 1) { /* Bitmap::resample (bitmap.cpp:2230-2329): x (repeat), then y (clamp) */
            int nW = std::max(1, (W + 1) / 2), nH = std::max(1, (H + 1) / 2);
            if (nW != W) {
                std::vector<float> t((size_t) nW * H * 3);
                for (int y = 0; y < H; ++y) resampleAxis(&bmp[(size_t) y * W * 3], 1, &t[(size_t) y * nW * 3], 1, W, nW, true);
                bmp.swap(t);
            }
            if (nH != H) {
                std::vector<float> t((size_t) nW * nH * 3);
                for (int x = 0; x < nW; ++x) resampleAxis(&bmp[(size_t) x * 3], nW, &t[(size_t) x * 3], nW, H, nH, false);
                bmp.swap(t);
            }
            W = nW, H = nH;
            keep(bmp, W, H);
        }
        for (int i = 0; i < 64; ++i) {
            float r2 = (float) i / (float) 63;
            lut[i] = (float) ::exp((double) (-2.0f * r2)) - (float) ::exp((double) -2.0f); /* math::fastexp */
        }
    }
    /* mipmap.h:503-563 at level l */
    Spec texL(int l, int x, int y) const {
        if (x < 0 || x >= lw[l]) x = modulo(x, lw[l]);
        if (y < 0 || y >= lh[l]) y = clampv(y, 0, lh[l] - 1);
        const float *p = &lev[l][3 * ((size_t) y * lw[l] + x)];
        return Spec(p[0], p[1], p[2]);
    }
    Spec evalBox(int l, float ux, float uy) const { /* :566-569 */
        return texL(l, floorToInt(ux * lw[l]), floorToInt(uy * lh[l]));
    }
    Spec evalBilinear(int l, float ux, float uy) const { /* :575-596 */
        if (!std::isfinite(ux) || !std::isfinite(uy)) return Spec(0.0f);
        if (l >= (int) lev.size()) return evalBox((int) lev.size() - 1, ux, uy);
        float u = ux * lw[l] - 0.5f, v = uy * lh[l] - 0.5f;
        int xPos = floorToInt(u), yPos = floorToInt(v);
        float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
        return texL(l, xPos, yPos) * dx2 * dy2 + texL(l, xPos, yPos + 1) * dx2 * dy1 +
               texL(l, xPos + 1, yPos) * dx1 * dy2 + texL(l, xPos + 1, yPos + 1) * dx1 * dy1;
    }
    Spec evalEWA(int l, float ux, float uy, float A, float B, float C) const { /* :764-834 */
        if (!std::isfinite(A + B + C + ux + uy)) return Spec(0.0f);
        if (l >= (int) lev.size()) return evalBox((int) lev.size() - 1, ux, uy);
        float u = ux * lw[l] - 0.5f, v = uy * lh[l] - 0.5f;
        A /= ratioX[l] * ratioX[l];
        B /= ratioX[l] * ratioY[l];
        C /= ratioY[l] * ratioY[l];
        float invDet = 1.0f / (-B * B + 4.0f * A * C), deltaU = 2.0f * std::sqrt(C * invDet),
              deltaV = 2.0f * std::sqrt(A * invDet);
        int u0 = (int) std::ceil(u - deltaU), u1 = floorToInt(u + deltaU);
        int v0 = (int) std::ceil(v - deltaV), v1 = floorToInt(v + deltaV);
        float As = A * 64, Bs = B * 64, Cs = C * 64;
        Spec result(0.0f);
        float denominator = 0.0f;
        float ddq = 2 * As, uu0 = (float) u0 - u;
        for (int vt = v0; vt <= v1; ++vt) {
            const float vv = (float) vt - v;
            float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
            float dq = As * (2 * uu0 + 1) + Bs * vv;
            for (int ut = u0; ut <= u1; ++ut) {
                if (q < (float) 64) {
                    uint32_t qi = (uint32_t) q;
                    if (qi < 64) {
                        const float weight = lut[(int) q];
                        result += texL(l, ut, vt) * weight;
                        denominator += weight;
                    }
                }
                q += dq;
                dq += ddq;
            }
        }
        if (denominator == 0) return evalBilinear(l, ux, uy);
        return result / denominator;
    }
    static float log2f_(float x) { return (float) ::log((double) x) * (1.0f / std::log(2.0f)); } /* math.cpp:103 */
    static float hypot2f_(float a, float b) {                                                       /* math.cpp:74 */
        float r;
        if (std::abs(a) > std::abs(b)) {
            r = b / a;
            r = std::abs(a) * std::sqrt(1.0f + r * r);
        } else if (b != 0.0f) {
            r = a / b;
            r = std::abs(b) * std::sqrt(1.0f + r * r);
        } else {
            r = 0.0f;
        }
        return r;
    }
    /* MIPMap::eval, EEWA (mipmap.h:629-720) */
    Spec mipEval(float ux, float uy, float d0x, float d0y, float d1x, float d1y) const {
        float du0 = d0x * lw[0], dv0 = d0y * lh[0], du1 = d1x * lw[0], dv1 = d1y * lh[0];
        float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1,
              F = A * C - B * B * 0.25f;
        float root = hypot2f_(A - C, B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root),
              majorRadius = Aprime != 0 ? std::sqrt(F / Aprime) : 0,
              minorRadius = Cprime != 0 ? std::sqrt(F / Cprime) : 0;
        if (!(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
            float level = log2f_(std::max(majorRadius, kEpsilon));
            int ilevel = floorToInt(level);
            if (ilevel < 0) return evalBilinear(0, ux, uy);
            float a = level - ilevel;
            return evalBilinear(ilevel, ux, uy) * (1.0f - a) + evalBilinear(ilevel + 1, ux, uy) * a;
        }
        if (minorRadius * maxAnisotropy < majorRadius) {
            minorRadius = majorRadius / maxAnisotropy;
            float theta = 0.5f * std::atan(B / (A - C)), sinTheta = std::sin(theta), cosTheta = std::cos(theta);
            float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
                  cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
            A = a2 * cosTheta2 + b2 * sinTheta2;
            B = (a2 - b2) * sin2Theta;
            C = a2 * sinTheta2 + b2 * cosTheta2;
            F = a2 * b2;
        }
        float scl = 1.0f / F;
        A *= scl;
        B *= scl;
        C *= scl;
        float level = std::max((float) 0.0f, log2f_(minorRadius));
        int ilevel = (int) level;
        float a = level - ilevel;
        if (majorRadius < 1 || !(A > 0 && C > 0)) return evalBilinear(ilevel, ux, uy);
        return evalEWA(ilevel, ux, uy, A, B, C) * (1.0f - a) + evalEWA(ilevel + 1, ux, uy, A, B, C) * a;
    }
    /* evalEnvironment of a RayDifferential with differentials (envmap.cpp:380-410) */
    Spec evalEnvironmentFiltered(const V3 &dir, const V3 &rxDir, const V3 &ryDir) const {
        V3 v = toLocal(dir);
        float ux = std::atan2(v.x, -v.z) * kInvTwoPi, uy = safe_acos(v.y) * kInvPi;
        V3 dvdx = toLocal(rxDir) - v, dvdy = toLocal(ryDir) - v;
        float t1 = kInvTwoPi / (v.x * v.x + v.z * v.z), t2 = -kInvPi / std::max(safe_sqrt(1.0f - v.y * v.y), kEpsilon);
        return mipEval(ux, uy, t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y, t1 * (dvdy.z * v.x - dvdy.x * v.z),
                       t2 * dvdy.y) *
               scale;
    }

    Spec tex(int x, int y) const { /* mipmap.h:503-563, bcu=repeat, bcv=clamp */
        if (x < 0 || x >= w) x = modulo(x, w);
        if (y < 0 || y >= h) y = clampv(y, 0, h - 1);
        const float *p = &texel[3 * ((size_t) y * w + x)];
        return Spec(p[0], p[1], p[2]);
    }
    void build(const float *rgb) { /* envmap.cpp:244-314 */
        buildPyramid(rgb);
        texel.resize((size_t) w * h * 3);
        for (size_t i = 0; i < (size_t) w * h * 3; ++i)
            texel[i] = halfToFloat(floatToHalf(std::max(rgb[i], 0.0f)));
        size_t nEntries = (size_t) (w + 1) * (size_t) h;
        cdfCols.assign(nEntries, 0.0f);
        cdfRows.assign(h + 1, 0.0f);
        rowWeights.assign(h, 0.0f);
        size_t colPos = 0, rowPos = 0;
        float rowSum = 0.0f;
        cdfRows[rowPos++] = 0;
        for (int y = 0; y < h; ++y) {
            float colSum = 0;
            cdfCols[colPos++] = 0;
            for (int x = 0; x < w; ++x) {
                Spec value = tex(x, y);
                colSum += value.getLuminance();
                cdfCols[colPos++] = (float) colSum;
            }
            float norm = 1.0f / (float) colSum;
            for (int x = 1; x < w; ++x)
                cdfCols[colPos - x - 1] *= norm;
            cdfCols[colPos - 1] = 1.0f;
            float weight = std::sin((y + 0.5f) * kPi / h);
            rowWeights[y] = weight;
            rowSum += colSum * weight;
            cdfRows[rowPos++] = (float) rowSum;
        }
        float norm = 1.0f / (float) rowSum;
        for (int y = 1; y < h; ++y)
            cdfRows[rowPos - y - 1] *= norm;
        cdfRows[rowPos - 1] = 1.0f;
        normalization = 1.0f / (rowSum * (2 * kPi / w) * (kPi / h));
        pixelSizeX = 2 * kPi / w;
        pixelSizeY = kPi / h;
    }
    V3 toWorld(const V3 &v) const {
        if (identity) return v;
        return V3(m[0] * v.x + m[1] * v.y + m[2] * v.z, m[3] * v.x + m[4] * v.y + m[5] * v.z,
                  m[6] * v.x + m[7] * v.y + m[8] * v.z);
    }
    V3 toLocal(const V3 &v) const {
        if (identity) return v;
        return V3(minv[0] * v.x + minv[1] * v.y + minv[2] * v.z,
                  minv[3] * v.x + minv[4] * v.y + minv[5] * v.z,
                  minv[6] * v.x + minv[7] * v.y + minv[8] * v.z);
    }
    static uint32_t sampleReuse(const float *cdf, uint32_t size, float &sample) { /* :657-662 */
        const float *entry = std::lower_bound(cdf, cdf + size + 1, (float) sample);
        uint32_t index = std::min((uint32_t) std::max((ptrdiff_t) 0, entry - cdf - 1), size - 1);
        sample = (sample - (float) cdf[index]) / (float) (cdf[index + 1] - cdf[index]);
        return index;
    }
    /* :567-600 */
    void internalSampleDirection(float sx, float sy, V3 &d, Spec &value, float &pdf) const {
        uint32_t row = sampleReuse(cdfRows.data(), h, sy),
                 col = sampleReuse(cdfCols.data() + row * (w + 1), w, sx);
        float posx = (float) col + intervalToTent(sx), posy = (float) row + intervalToTent(sy);
        int xPos = floorToInt(posx), yPos = floorToInt(posy);
        float dx1 = posx - xPos, dx2 = 1.0f - dx1, dy1 = posy - yPos, dy2 = 1.0f - dy1;
        Spec value1 = tex(xPos, yPos) * dx2 * dy2 + tex(xPos + 1, yPos) * dx1 * dy2;
        Spec value2 = tex(xPos, yPos + 1) * dx2 * dy1 + tex(xPos + 1, yPos + 1) * dx1 * dy1;
        value = (value1 + value2) * scale;
        pdf = (value1.getLuminance() * rowWeights[clampv(yPos, 0, h - 1)] +
               value2.getLuminance() * rowWeights[clampv(yPos + 1, 0, h - 1)]) *
              normalization;
        float sinPhi = std::sin(pixelSizeX * (posx + 0.5f)), cosPhi = std::cos(pixelSizeX * (posx + 0.5f));
        float sinTheta = std::sin(pixelSizeY * (posy + 0.5f)), cosTheta = std::cos(pixelSizeY * (posy + 0.5f));
        d = V3(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
        pdf /= std::max(std::abs(sinTheta), kEpsilon);
    }
    /* :603-633 */
    float internalPdfDirection(const V3 &d) const {
        float uvx = std::atan2(d.x, -d.z) * kInvTwoPi, uvy = safe_acos(d.y) * kInvPi;
        if (!std::isfinite(uvx) || !std::isfinite(uvy))
            return 0.0f;
        float u = uvx * w - 0.5f, v = uvy * h - 0.5f;
        int xPos = floorToInt(u), yPos = floorToInt(v);
        float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
        Spec value1 = tex(xPos, yPos) * dx2 * dy2 + tex(xPos + 1, yPos) * dx1 * dy2;
        Spec value2 = tex(xPos, yPos + 1) * dx2 * dy1 + tex(xPos + 1, yPos + 1) * dx1 * dy1;
        float sinTheta = safe_sqrt(1 - d.y * d.y);
        return (value1.getLuminance() * rowWeights[clampv(yPos, 0, h - 1)] +
                value2.getLuminance() * rowWeights[clampv(yPos + 1, 0, h - 1)]) *
               normalization / std::max(std::abs(sinTheta), kEpsilon);
    }
    /* :380-410 + mipmap.h:575-596 (bilinear at level 0) */
    Spec evalEnvironment(const V3 &dir) const {
        V3 v = toLocal(dir);
        float uvx = std::atan2(v.x, -v.z) * kInvTwoPi, uvy = safe_acos(v.y) * kInvPi;
        Spec value;
        if (!std::isfinite(uvx) || !std::isfinite(uvy)) {
            value = Spec(0.0f);
        } else {
            float u = uvx * w - 0.5f, vv = uvy * h - 0.5f;
            int xPos = floorToInt(u), yPos = floorToInt(vv);
            float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = vv - yPos, dy2 = 1.0f - dy1;
            value = tex(xPos, yPos) * dx2 * dy2 + tex(xPos, yPos + 1) * dx2 * dy1 +
                    tex(xPos + 1, yPos) * dx1 * dy2 + tex(xPos + 1, yPos + 1) * dx1 * dy1;
        }
        return value * scale;
    }
    /* EWA ellipse major radius for a primary ray (envmap.cpp:391-405, mipmap.h:631-660) */
    float ewaMajorRadius(const V3 &dir, const V3 &rxDir, const V3 &ryDir) const {
        V3 v = toLocal(dir);
        V3 dvdx = toLocal(rxDir) - v, dvdy = toLocal(ryDir) - v;
        float t1 = kInvTwoPi / (v.x * v.x + v.z * v.z),
              t2 = -kInvPi / std::max(safe_sqrt(1.0f - v.y * v.y), kEpsilon);
        float dudx0 = t1 * (dvdx.z * v.x - dvdx.x * v.z), dudx1 = t2 * dvdx.y;
        float dudy0 = t1 * (dvdy.z * v.x - dvdy.x * v.z), dudy1 = t2 * dvdy.y;
        float du0 = dudx0 * w, dv0 = dudx1 * h, du1 = dudy0 * w, dv1 = dudy1 * h;
        float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1),
              C = du0 * du0 + du1 * du1, F = A * C - B * B * 0.25f;
        float root = std::hypot(A - C, B), Aprime = 0.5f * (A + C - root);
        float majorRadius = Aprime != 0 ? std::sqrt(F / Aprime) : 0;
        return majorRadius;
    }
    bool bsphereIntersect(const Ray &ray, float &nearT, float &farT) const { /* bsphere.h:88-95 */
        V3 o = ray.o - bsCenter;
        float A = ray.d.lengthSquared();
        float B = 2 * dot(o, ray.d);
        float C = o.lengthSquared() - bsRadius * bsRadius;
        return solveQuadratic(A, B, C, nearT, farT);
    }
};

/* ---------------- transforms (transform.h, matrix.h/.inl) ---------------- */
inline V3 xformPoint(const float *M, const V3 &p) { /* transform.h:108-125 */
    float x = M[0] * p.x + M[1] * p.y + M[2] * p.z + M[3];
    float y = M[4] * p.x + M[5] * p.y + M[6] * p.z + M[7];
    float z = M[8] * p.x + M[9] * p.y + M[10] * p.z + M[11];
    float w = M[12] * p.x + M[13] * p.y + M[14] * p.z + M[15];
    if (w == 1.0f)
        return V3(x, y, z);
    return V3(x, y, z) / w;
}
inline V3 xformVector(const float *M, const V3 &v) { /* transform.h:175-183 */
    float x = M[0] * v.x + M[1] * v.y + M[2] * v.z;
    float y = M[4] * v.x + M[5] * v.y + M[6] * v.z;
    float z = M[8] * v.x + M[9] * v.y + M[10] * v.z;
    return V3(x, y, z);
}

/* Matrix4x4 (matrix.h) in float: product (matrix.h:743-756) and the
   Gauss-Jordan inverse with full pivoting (matrix.inl:138-190) */
struct Mat4 {
    float m[4][4];
};
static Mat4 matMul(const Mat4 &a, const Mat4 &b) {
    Mat4 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float sum = 0;
            for (int k = 0; k < 4; ++k) sum += a.m[i][k] * b.m[k][j];
            r.m[i][j] = sum;
        }
    return r;
}
static bool matInvert(const Mat4 &src, Mat4 &target) {
    const int N = 4;
    int indxc[N], indxr[N], ipiv[N];
    std::memset(ipiv, 0, sizeof(ipiv));
    target = src;
    for (int i = 0; i < N; i++) {
        int irow = -1, icol = -1;
        float big = 0;
        for (int j = 0; j < N; j++) {
            if (ipiv[j] != 1) {
                for (int k = 0; k < N; k++) {
                    if (ipiv[k] == 0) {
                        if (std::abs(target.m[j][k]) >= big) {
                            big = std::abs(target.m[j][k]);
                            irow = j;
                            icol = k;
                        }
                    } else if (ipiv[k] > 1) {
                        return false;
                    }
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < N; ++k) std::swap(target.m[irow][k], target.m[icol][k]);
        indxr[i] = irow;
        indxc[i] = icol;
        if (target.m[icol][icol] == 0) return false;
        float pivinv = 1.f / target.m[icol][icol];
        target.m[icol][icol] = 1.f;
        for (int j = 0; j < N; j++) target.m[icol][j] *= pivinv;
        for (int j = 0; j < N; j++) {
            if (j != icol) {
                float save = target.m[j][icol];
                target.m[j][icol] = 0;
                for (int k = 0; k < N; k++) target.m[j][k] -= target.m[icol][k] * save;
            }
        }
    }
    for (int j = N - 1; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < N; k++) std::swap(target.m[k][indxr[j]], target.m[k][indxc[j]]);
    return true;
}
/* Transform = (matrix, inverse); operator* (transform.cpp:28-31) */
struct Xform {
    Mat4 t, inv;
    Xform operator*(const Xform &o) const { return Xform{matMul(t, o.t), matMul(o.inv, inv)}; }
};
static Xform xformScale(float x, float y, float z) { /* transform.cpp:49-62 */
    return Xform{{{{x, 0, 0, 0}, {0, y, 0, 0}, {0, 0, z, 0}, {0, 0, 0, 1}}},
                 {{{1.0f / x, 0, 0, 0}, {0, 1.0f / y, 0, 0}, {0, 0, 1.0f / z, 0}, {0, 0, 0, 1}}}};
}
static Xform xformTranslate(float x, float y, float z) { /* transform.cpp:33-47 */
    return Xform{{{{1, 0, 0, x}, {0, 1, 0, y}, {0, 0, 1, z}, {0, 0, 0, 1}}},
                 {{{1, 0, 0, -x}, {0, 1, 0, -y}, {0, 0, 1, -z}, {0, 0, 0, 1}}}};
}

#include "mesh_geom.h"

} // namespace

/* ------------------------------------------------------------------ */
/* The scene                                                            */
/* ------------------------------------------------------------------ */
struct orc_scene {
    std::string err;
    /* sobol */
    std::vector<uint32_t> m32;
    uint64_t scramble = 0; /* after sampleTEA */
    std::vector<uint64_t> vdc, vdcInv;
    int vdcRows = 0, invRows = 0;
    /* camera */
    float toWorld[16];
    float fov = 35, nearClip = 1e-2f, farClip = 1e4f;
    int width = 0, height = 0;
    float s2c[16]; /* sampleToCamera, row-major */
    float dx[3], dy[3];
    float invResX = 0, invResY = 0;
    uint32_t logRes = 0;
    float resolution = 1;
    /* scene */
    HairGeom hair;
    KDTree tree;
    AABB aabb;                   /* hair AABB */
    /* C1 mesh shapes (mesh_geom.h): CPU path only */
    std::vector<TriMesh> meshes;
    std::vector<RectShape> rects;
    MeshBVH bvh;
    AABB sceneAabb;              /* == aabb for hair-only scenes */
    bool hasMeshes() const { return !meshes.empty() || !rects.empty(); }
    bool hasHair() const { return !hair.shapeFirst.empty(); }
    std::vector<BsdfInst> bsdfs; /* hair shapes: one each (orc_set_* sets the last one's); meshes index it */
    EnvMap env;
    bool hasEnv = false;
    int maxDepth = -1, rrDepth = 5;
    int sampleCount = 1; /* sampler->getSampleCount() for the ray-differential scale */
    bool strictNormals = false, hideEmitters = false;
    bool prepared = false;
};

namespace {

/* ---------------- Sobol: sobolseq.h:43-58, 99-131; sobol.cpp:204-250 ---------------- */
inline float sobolSample(const orc_scene *s, uint64_t index, uint32_t dim) {
    uint32_t result = (uint32_t) s->scramble; /* sobolseq.h:43-58 with (uint32_t) scramble */
    for (uint32_t i = dim * 52; index; index >>= 1, ++i)
        if (index & 1)
            result ^= s->m32[i];
    return std::min(result * (1.0f / (1ULL << 32)), kOneMinusEps);
}

inline uint64_t sobolLookUp(const orc_scene *s, uint32_t m, uint32_t frame, uint32_t px, uint32_t py) {
    const uint32_t m2 = m << 1;
    uint64_t index = uint64_t(frame) << m2;
    uint64_t delta = 0;
    for (uint32_t c = 0; frame; frame >>= 1, ++c)
        if (frame & 1)
            delta ^= s->vdc[(m - 1) * 52 + c];
    uint64_t scramble = (s->scramble & 0xFFFFFFFF) >> (32 - m); /* sobolseq.h:119-123 */
    uint64_t b = (((uint64_t) (px ^ scramble) << m) | (py ^ scramble)) ^ delta;
    for (uint32_t c = 0; b; b >>= 1, ++c)
        if (b & 1)
            index ^= s->vdcInv[(m - 1) * 52 + c];
    return index;
}

struct Sampler {
    const orc_scene *s;
    uint64_t sobolIndex = 0, sampleIndex = 0;
    uint32_t dimension = 0;
    int px = 0, py = 0;
    void setSampleIndex(uint64_t j) {
        dimension = 0;
        sampleIndex = j;
        if (s->logRes > 1 && px >= 0)
            sobolIndex = sobolLookUp(s, s->logRes, (uint32_t) j, px, py);
        else
            sobolIndex = j;
    }
    float next1D() { return sobolSample(s, sobolIndex, dimension++); }
    void next2D(float &a, float &b) {
        if (dimension == 0 && sobolIndex != sampleIndex) {
            a = sobolSample(s, sobolIndex, dimension++) * s->resolution - px;
            b = sobolSample(s, sobolIndex, dimension++) * s->resolution - py;
        } else {
            a = sobolSample(s, sobolIndex, dimension++);
            b = sobolSample(s, sobolIndex, dimension++);
        }
    }
};

/* ---------------- camera: perspective.cpp:125-165, 271-298 ---------------- */
/* PerspectiveCameraImpl::configure (perspective.cpp:125-165): m_cameraToSample =
   S(1/relSize) T(-relOffset) S(-0.5, -0.5 aspect, 1) T(-1, -1/aspect, 0) perspective(...),
   m_sampleToCamera = its inverse (the Transform's stored inverse matrix) */
void setupCamera(orc_scene *s) {
    float aspect = s->width / (float) s->height; /* sensor.cpp:101-102 */
    Xform persp; /* Transform::perspective (transform.cpp:99-119) -> Transform(Matrix4x4) inverts */
    {
        float recip = 1.0f / (s->farClip - s->nearClip);
        float cot = 1.0f / std::tan(degToRad(s->fov / 2.0f));
        persp.t = Mat4{{{cot, 0, 0, 0}, {0, cot, 0, 0}, {0, 0, s->farClip * recip, -s->nearClip * s->farClip * recip},
                        {0, 0, 1, 0}}};
        if (!matInvert(persp.t, persp.inv)) throw std::runtime_error("Unable to invert singular matrix");
    }
    float relSizeX = (float) s->width / (float) s->width, relSizeY = (float) s->height / (float) s->height;
    float relOffsetX = (float) 0 / (float) s->width, relOffsetY = (float) 0 / (float) s->height;
    Xform cameraToSample = xformScale(1.0f / relSizeX, 1.0f / relSizeY, 1.0f) *
                           xformTranslate(-relOffsetX, -relOffsetY, 0.0f) *
                           xformScale(-0.5f, -0.5f * aspect, 1.0f) *
                           xformTranslate(-1.0f, -1.0f / aspect, 0.0f) * persp;
    for (int r = 0; r < 4; ++r)
        for (int c = 0; c < 4; ++c) s->s2c[r * 4 + c] = cameraToSample.inv.m[r][c];
    s->invResX = 1.0f / (float) s->width;
    s->invResY = 1.0f / (float) s->height;
    V3 p0 = xformPoint(s->s2c, V3(0.0f, 0.0f, 0.0f));
    V3 pdx = xformPoint(s->s2c, V3(s->invResX, 0.0f, 0.0f)) - p0;
    V3 pdy = xformPoint(s->s2c, V3(0.0f, s->invResY, 0.0f)) - p0;
    s->dx[0] = pdx.x; s->dx[1] = pdx.y; s->dx[2] = pdx.z;
    s->dy[0] = pdy.x; s->dy[1] = pdy.y; s->dy[2] = pdy.z;
    /* sobol.cpp:147-158 (bucketed: path is a SamplingIntegrator, integrator.cpp:37-41) */
    uint32_t r = (uint32_t) std::max(s->width, s->height);
    r--; r |= r >> 1; r |= r >> 2; r |= r >> 4; r |= r >> 8; r |= r >> 16; r++;
    s->resolution = (float) r;
    uint32_t lg = 0;
    while ((r >> lg) != 0) lg++;
    s->logRes = lg - 1;
}

struct CamRay {
    Ray ray;
    V3 rxDir, ryDir;
};

CamRay cameraRay(const orc_scene *s, float sx, float sy) {
    V3 nearP = xformPoint(s->s2c, V3(sx * s->invResX, sy * s->invResY, 0.0f));
    V3 d = normalize(nearP);
    float invZ = 1.0f / d.z;
    float mint = s->nearClip * invZ, maxt = s->farClip * invZ;
    const float *T = s->toWorld;
    V3 o(T[0] * 0.0f + T[1] * 0.0f + T[2] * 0.0f + T[3], T[4] * 0.0f + T[5] * 0.0f + T[6] * 0.0f + T[7],
         T[8] * 0.0f + T[9] * 0.0f + T[10] * 0.0f + T[11]);
    CamRay cr;
    cr.ray = Ray(o, xformVector(T, d), mint, maxt);
    cr.rxDir = xformVector(T, normalize(nearP + V3(s->dx[0], s->dx[1], s->dx[2])));
    cr.ryDir = xformVector(T, normalize(nearP + V3(s->dy[0], s->dy[1], s->dy[2])));
    /* integrator.cpp:143-144,178: sensorRay.scaleDifferential(1/sqrt(sampleCount)) (ray.h:163-168) */
    const float amount = 1.0f / std::sqrt((float) s->sampleCount);
    cr.rxDir = cr.ray.d + (cr.rxDir - cr.ray.d) * amount;
    cr.ryDir = cr.ray.d + (cr.ryDir - cr.ray.d) * amount;
    return cr;
}

/* ---------------- traversal: sahkdtree3.h:178-308 (Havran) ---------------- */
struct HavranEntry {
    uint32_t node;
    float t;
    uint32_t prev;
    V3 p;
};

template <bool shadowRay>
bool rayIntersectHavran(const orc_scene *s, const Ray &ray, float mint, float maxt, float &t,
                        Hit *hit, Stats *st) {
    HavranEntry stack[64];
    const uint32_t *N = s->tree.nodes.data();
    const uint32_t kNull = 0xffffffffu;
    uint32_t enPt = 0;
    stack[enPt].t = mint;
    stack[enPt].p = ray.at(mint);
    uint32_t exPt = 1;
    stack[exPt].t = maxt;
    stack[exPt].p = ray.at(maxt);
    stack[exPt].node = kNull;
    bool found = false;
    uint32_t curr = 0;
    while (curr != kNull) {
        while (!(N[2 * curr] & 0x80000000u)) {
            if (st) st->nodes++;
            float splitVal;
            std::memcpy(&splitVal, &N[2 * curr + 1], 4);
            const int axis = (int) (N[2 * curr] & 3u);
            const uint32_t left = N[2 * curr] >> 2;
            uint32_t farChild;
            if (stack[enPt].p[axis] <= splitVal) {
                if (stack[exPt].p[axis] <= splitVal) {
                    curr = left;
                    continue;
                }
                if (stack[enPt].p[axis] == splitVal) {
                    curr = left + 1;
                    continue;
                }
                curr = left;
                farChild = left + 1;
            } else {
                if (splitVal < stack[exPt].p[axis]) {
                    curr = left + 1;
                    continue;
                }
                farChild = left;
                curr = left + 1;
            }
            float distToSplit = (splitVal - ray.o[axis]) * ray.dRcp[axis];
            const uint32_t tmp = exPt++;
            if (exPt == enPt)
                ++exPt;
            stack[exPt].prev = tmp;
            stack[exPt].t = distToSplit;
            stack[exPt].node = farChild;
            stack[exPt].p = ray.at(distToSplit);
            stack[exPt].p[axis] = splitVal;
        }
        if (st) st->nodes++;
        uint32_t start = N[2 * curr] & 0x7fffffffu, end = N[2 * curr + 1];
        for (uint32_t entry = start; entry != end; entry++) {
            const uint32_t primIdx = s->tree.indices[entry];
            if (st) st->prims++;
            bool result;
            float tt;
            V3 pp;
            if (!shadowRay)
                result = s->hair.intersect(ray.o, ray.d, primIdx, mint, maxt, tt, &pp);
            else
                result = s->hair.intersect(ray.o, ray.d, primIdx, mint, maxt, tt, nullptr);
            if (result) {
                if (shadowRay)
                    return true;
                t = tt;
                maxt = tt;
                hit->iv = primIdx;
                hit->p = pp;
                found = true;
            }
        }
        if (stack[exPt].t > maxt)
            break;
        enPt = exPt;
        curr = stack[exPt].node;
        exPt = stack[enPt].prev;
    }
    return found;
}

/* brute force over all segments (test aid: same per-primitive semantics) */
template <bool shadowRay>
bool rayIntersectBrute(const orc_scene *s, const Ray &ray, float mint, float maxt, float &t, Hit *hit) {
    bool found = false;
    const size_t n = s->hair.v.size();
    for (size_t i = 0; i + 1 < n; ++i) {
        if (s->hair.start[i + 1]) continue;
        float tt;
        V3 pp;
        if (s->hair.intersect(ray.o, ray.d, (uint32_t) i, mint, maxt, tt, shadowRay ? nullptr : &pp)) {
            if (shadowRay) return true;
            t = tt;
            maxt = tt;
            hit->iv = (uint32_t) i;
            hit->p = pp;
            found = true;
        }
    }
    return found;
}

/* the hair shape inside the scene-level kd-tree (hair.cpp:200-217): clip to the hair AABB,
   then HairKDTree::rayIntersect */
bool hairIntersect(const orc_scene *s, const Ray &ray, float mint, float maxt, Hit &hit, Stats *st, bool brute) {
    float m2, M2;
    if (!s->aabb.rayIntersect(ray, m2, M2)) return false;
    if (mint > m2) m2 = mint;
    if (maxt < M2) M2 = maxt;
    if (!(M2 > m2)) return false;
    float t = kInf;
    bool ok = brute ? rayIntersectBrute<false>(s, ray, m2, M2, t, &hit) : rayIntersectHavran<false>(s, ray, m2, M2, t, &hit, st);
    if (ok) {
        hit.t = t;
        hit.kind = 0;
    }
    return ok;
}

/* skdtree.cpp:112-141 */
bool sceneIntersect(const orc_scene *s, const Ray &ray, Hit &hit, Stats *st, bool brute = false) {
    hit.t = kInf;
    float mint, maxt;
    if (st) st->rays++;
    if (s->sceneAabb.rayIntersect(ray, mint, maxt)) {
        float rayMinT = ray.mint;
        if (rayMinT == kEpsilon)
            rayMinT *= std::max(std::max(std::max(std::abs(ray.o.x), std::abs(ray.o.y)), std::abs(ray.o.z)),
                                kEpsilon);
        if (rayMinT > mint) mint = rayMinT;
        if (ray.maxt < maxt) maxt = ray.maxt;
        if (maxt > mint) {
            /* meshes first (any order gives the closest hit: maxt shrinks), then the hair shape */
            bool found = s->hasMeshes() && meshIntersect<false>(s->meshes, s->rects, s->bvh, ray, mint, maxt, &hit, st);
            if (s->hasHair() && hairIntersect(s, ray, mint, maxt, hit, st, brute)) found = true;
            if (found) return true;
        }
    }
    hit.t = kInf;
    return false;
}

/* skdtree.cpp:207-226 */
bool sceneOccluded(const orc_scene *s, const Ray &ray, Stats *st, bool brute = false) {
    float mint, maxt, t = kInf;
    if (st) st->shadowRays++;
    if (s->sceneAabb.rayIntersect(ray, mint, maxt)) {
        float rayMinT = ray.mint;
        if (rayMinT == kEpsilon)
            rayMinT *= std::max(std::max(std::abs(ray.o.x), std::abs(ray.o.y)), std::abs(ray.o.z));
        if (rayMinT > mint) mint = rayMinT;
        if (ray.maxt < maxt) maxt = ray.maxt;
        if (maxt > mint) {
            if (s->hasMeshes() && meshIntersect<true>(s->meshes, s->rects, s->bvh, ray, mint, maxt, nullptr, st))
                return true;
            if (!s->hasHair()) return false;
            float m2, M2;
            if (s->aabb.rayIntersect(ray, m2, M2)) {
                if (mint > m2) m2 = mint;
                if (maxt < M2) M2 = maxt;
                if (M2 > m2) {
                    Hit dummy;
                    return brute ? rayIntersectBrute<true>(s, ray, m2, M2, t, &dummy)
                                 : rayIntersectHavran<true>(s, ray, m2, M2, t, &dummy, st);
                }
            }
        }
    }
    return false;
}

struct Intersection {
    float t;
    uint32_t iv; /* segment (its first vertex) -> shape -> BSDF */
    V3 p;
    Frame geoFrame, shFrame;
    V3 wi;
    float uv[2] = {0, 0};
    int bsdf = 0; /* index into orc_scene::bsdfs */
    V3 toWorld(const V3 &v) const { return shFrame.toWorld(v); }
    V3 toLocal(const V3 &v) const { return shFrame.toLocal(v); }
};

/* skdtree.h:343-428 (fillIntersectionRecord<true>) for a triangle, rectangle.cpp:155-168 for a rectangle */
void fillMeshIntersection(const orc_scene *s, const Ray &ray, const Hit &hit, Intersection &its) {
    its.t = hit.t;
    its.iv = 0;
    V3 dpdu;
    if (hit.kind == 1) {
        const TriMesh &m = s->meshes[hit.shape];
        const uint32_t i0 = m.idx[3 * hit.prim], i1 = m.idx[3 * hit.prim + 1], i2 = m.idx[3 * hit.prim + 2];
        const V3 b(1 - hit.u - hit.v, hit.u, hit.v);
        const V3 &p0 = m.p[i0], &p1 = m.p[i1], &p2 = m.p[i2];
        its.p = p0 * b.x + p1 * b.y + p2 * b.z;
        const V3 side1 = p1 - p0, side2 = p2 - p0;
        V3 faceNormal = cross(side1, side2);
        const float length = faceNormal.length();
        if (!faceNormal.isZero()) faceNormal /= length;
        dpdu = m.dpdu.empty() ? side1 : m.dpdu[hit.prim];
        V3 shN;
        if (!m.n.empty()) {
            shN = normalize(m.n[i0] * b.x + m.n[i1] * b.y + m.n[i2] * b.z);
            if (dot(faceNormal, shN) < 0) faceNormal = -faceNormal;
        } else {
            shN = faceNormal;
        }
        its.geoFrame = frameFromNormal(faceNormal);
        if (!m.uv.empty()) {
            its.uv[0] = m.uv[2 * i0] * b.x + m.uv[2 * i1] * b.y + m.uv[2 * i2] * b.z;
            its.uv[1] = m.uv[2 * i0 + 1] * b.x + m.uv[2 * i1 + 1] * b.y + m.uv[2 * i2 + 1] * b.z;
        } else {
            its.uv[0] = b.y;
            its.uv[1] = b.z;
        }
        its.shFrame.n = shN;
        its.bsdf = m.bsdf;
    } else {
        const RectShape &r = s->rects[hit.shape];
        its.geoFrame = r.frame;
        its.shFrame = frameFromNormal(its.geoFrame.n);
        dpdu = r.dpdu;
        its.uv[0] = 0.5f * (hit.u + 1);
        its.uv[1] = 0.5f * (hit.v + 1);
        its.p = ray.at(its.t);
        its.bsdf = r.bsdf;
    }
    computeShadingFrame(its.shFrame.n, dpdu, its.shFrame);
    its.wi = its.toLocal(-ray.d);
}

/* hair.cpp:825-862 + skdtree.h:422-427 */
void fillIntersection(const orc_scene *s, const Ray &ray, const Hit &hit, Intersection &its) {
    if (hit.kind != 0) {
        fillMeshIntersection(s, ray, hit, its);
        return;
    }
    its.bsdf = s->hair.shapeBsdf[s->hair.shapeOf(hit.iv)];
    its.uv[0] = its.uv[1] = 0;
    its.t = hit.t;
    its.iv = hit.iv;
    its.p = hit.p;
    const V3 axis = s->hair.tangent(hit.iv);
    its.geoFrame.s = axis;
    const V3 relHitPoint = its.p - s->hair.firstVertex(hit.iv);
    its.geoFrame.n = normalize(relHitPoint - dot(axis, relHitPoint) * axis);
    its.geoFrame.t = cross(its.geoFrame.n, its.geoFrame.s);
    const V3 local = its.geoFrame.toLocal(relHitPoint);
    its.p += its.geoFrame.n * (s->hair.radius(hit.iv) - std::sqrt(local.y * local.y + local.z * local.z));
    its.shFrame = its.geoFrame;
    V3 dpdu = its.geoFrame.s;
    computeShadingFrame(its.shFrame.n, dpdu, its.shFrame);
    its.wi = its.toLocal(-ray.d);
}

inline float miWeight(float pdfA, float pdfB) { /* path.cpp:296-300 */
    pdfA *= pdfA;
    pdfB *= pdfB;
    return pdfA / (pdfA + pdfB);
}

/* the BSDF of the shape a hit belongs to; the batch entry points use the last loaded shape's */
const BsdfInst &bsdfOf(const orc_scene *s, uint32_t iv) { return s->bsdfs[s->hair.shapeBsdf[s->hair.shapeOf(iv)]]; }
BsdfInst &lastBsdf(orc_scene *s) {
    if (s->bsdfs.empty()) s->bsdfs.emplace_back();
    return s->bsdfs.back();
}
Spec bsdfEval(const orc_scene *s, const V3 &wi, const V3 &wo) { return s->bsdfs.back().eval(wi, wo); }
float bsdfPdf(const orc_scene *s, const V3 &wi, const V3 &wo) { return s->bsdfs.back().pdf(wi, wo); }
Spec bsdfSample(const orc_scene *s, const V3 &wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type) {
    return s->bsdfs.back().sample(wi, sx, sy, wo, pdf, type);
}

/* envmap.cpp:516-543 + scene.cpp:828-852; returns value (0 if occluded/failed) */
Spec sampleEmitterDirect(const orc_scene *s, const V3 &ref, float sx, float sy, V3 &dOut, float &pdfOut,
                         Stats *st) {
    const EnvMap &E = s->env;
    Spec value;
    V3 d;
    float pdf;
    E.internalSampleDirection(sx, sy, d, value, pdf);
    Ray ray(ref, E.toWorld(d), 0.0f, kInf);
    float nearT, farT;
    if (value.isZero() || pdf == 0 || !E.bsphereIntersect(ray, nearT, farT) || nearT >= 0 || farT <= 0) {
        pdfOut = 0;
        return Spec(0.0f);
    }
    pdfOut = pdf;
    float dist = farT;
    dOut = ray.d;
    Spec v = value / pdf;
    Ray shadow(ref, ray.d, kEpsilon, dist * (1 - kShadowEpsilon));
    if (sceneOccluded(s, shadow, st))
        return Spec(0.0f);
    /* dRec.pdf *= emPdf (1); value /= emPdf (1) */
    v /= 1.0f;
    return v;
}

/* path.cpp:119-294 -- MIPathTracer::Li for one camera sample */
Spec Li(const orc_scene *s, const CamRay &cr, Sampler &sampler, Stats *st, int *depthOut) {
    Ray ray = cr.ray;
    Spec Li(0.0f);
    bool scattered = false;
    bool emitted = true; /* rRec.type & EEmittedRadiance */
    int depth = 1;
    Hit hit;
    sceneIntersect(s, ray, hit, st);
    Intersection its;
    bool valid = hit.valid();
    if (valid) fillIntersection(s, ray, hit, its);
    ray.mint = kEpsilon;
    Spec throughput(1.0f);
    float eta = 1.0f;
    bool primary = true;
    while (depth <= s->maxDepth || s->maxDepth < 0) {
        if (!valid) {
            if (emitted && (!s->hideEmitters || scattered)) {
                if (s->hasEnv) {
                    /* a camera ray keeps its differentials (EWA lookup); after a bounce
                       ray = Ray(...) drops them (ray.h:196-208): bilinear at level 0 */
                    if (primary) {
                        if (st && s->env.ewaMajorRadius(cr.ray.d, cr.rxDir, cr.ryDir) >= 1.0f) st->ewaViolations++;
                        Li += throughput * s->env.evalEnvironmentFiltered(cr.ray.d, cr.rxDir, cr.ryDir);
                    } else {
                        Li += throughput * s->env.evalEnvironment(ray.d);
                    }
                }
            }
            break;
        }
        if ((depth >= s->maxDepth && s->maxDepth > 0) ||
            (s->strictNormals && dot(ray.d, its.geoFrame.n) * its.wi.z >= 0))
            break;
        if (st) st->bounces++;
        const BsdfInst &bsdf = s->bsdfs[its.bsdf];
        /* direct illumination, only for BSDFs with an ESmooth component (path.cpp:175) */
        float nx, ny;
        if (bsdf.smooth()) sampler.next2D(nx, ny);
        if (bsdf.smooth() && s->hasEnv) {
            V3 dRecD;
            float dRecPdf;
            Spec value = sampleEmitterDirect(s, its.p, nx, ny, dRecD, dRecPdf, st);
            if (!value.isZero()) {
                V3 wo = its.toLocal(dRecD);
                const Spec bsdfVal = bsdf.eval(its.wi, wo, its.uv);
                if (!bsdfVal.isZero() && (!s->strictNormals || dot(its.geoFrame.n, dRecD) * wo.z > 0)) {
                    float bp = bsdf.pdf(its.wi, wo, its.uv);
                    float weight = miWeight(dRecPdf, bp);
                    Li += throughput * value * bsdfVal * weight;
                }
            }
        }
        /* BSDF sampling */
        float bx, by;
        sampler.next2D(bx, by);
        float bsdfPdfV = 0;
        uint32_t sampledType = 0;
        V3 woLocal;
        Spec bsdfWeight = bsdf.sample(its.wi, bx, by, woLocal, bsdfPdfV, sampledType, its.uv);
        if (bsdfWeight.isZero())
            break;
        scattered |= sampledType != ENull;
        const V3 wo = its.toWorld(woLocal);
        float woDotGeoN = dot(its.geoFrame.n, wo);
        if (s->strictNormals && woDotGeoN * woLocal.z <= 0)
            break;
        bool hitEmitter = false;
        Spec value;
        V3 dRecD;
        ray = Ray(its.p, wo, kEpsilon, kInf);
        primary = false;
        Hit nh;
        if (sceneIntersect(s, ray, nh, st)) {
            fillIntersection(s, ray, nh, its);
            valid = true;
        } else {
            valid = false;
            if (s->hasEnv) {
                if (s->hideEmitters && !scattered)
                    break;
                value = s->env.evalEnvironment(ray.d);
                float nearT, farT;
                if (!s->env.bsphereIntersect(ray, nearT, farT) || nearT > 0 || farT < 0)
                    break;
                dRecD = ray.d;
                hitEmitter = true;
            } else {
                break;
            }
        }
        throughput *= bsdfWeight;
        eta *= 1.0f;
        if (hitEmitter) {
            const float lumPdf = (!(sampledType & EDelta)) ? s->env.internalPdfDirection(s->env.toLocal(dRecD)) : 0;
            Li += throughput * value * miWeight(bsdfPdfV, lumPdf);
        }
        if (!valid)
            break;
        emitted = false;
        if (depth++ >= s->rrDepth) {
            float q = std::min(throughput.max() * eta * eta, (float) 0.95f);
            if (sampler.next1D() >= q)
                break;
            throughput /= q;
        }
    }
    if (depthOut) *depthOut = depth;
    if (st) st->paths++;
    return Li;
}

/* rfilter.cpp:38-56 + tent.cpp:30-46 */
struct TentLUT {
    float values[32];
    float scaleFactor;
    TentLUT() {
        const int R = 31;
        float radius = 1.0f, sum = 0.0f;
        for (int i = 0; i < R; ++i) {
            float x = (radius * i) / R;
            float value = std::max((float) 0.0f, 1.0f - std::abs(x / radius));
            values[i] = value;
            sum += value;
        }
        values[R] = 0.0f;
        scaleFactor = R / radius;
        sum *= 2 * radius / R;
        float normalization = 1.0f / sum;
        for (int i = 0; i < R; ++i)
            values[i] *= normalization;
    }
    float eval(float x) const { return values[std::min((int) std::abs(x * scaleFactor), 31)]; }
};
static const TentLUT gTent;

/* imageblock.h:124-204 splat into a full-frame RGBW film (A == W since alpha == 1) */
bool splat(float *film, int W, int H, float posx, float posy, const Spec &spec) {
    float value[5] = {spec.s[0], spec.s[1], spec.s[2], 1.0f, 1.0f};
    for (int i = 0; i < 5; ++i)
        if (!std::isfinite(value[i]) || value[i] < 0)
            return false;
    const float filterRadius = 1.0f;
    const float px = posx - 0.5f, py = posy - 0.5f;
    int minx = std::max((int) std::ceil(px - filterRadius), 0),
        miny = std::max((int) std::ceil(py - filterRadius), 0),
        maxx = std::min((int) std::floor(px + filterRadius), W - 1),
        maxy = std::min((int) std::floor(py + filterRadius), H - 1);
    float wx[4], wy[4];
    for (int x = minx, idx = 0; x <= maxx; ++x) wx[idx++] = gTent.eval(x - px);
    for (int y = miny, idx = 0; y <= maxy; ++y) wy[idx++] = gTent.eval(y - py);
    for (int y = miny, yr = 0; y <= maxy; ++y, ++yr) {
        const float weightY = wy[yr];
        for (int x = minx, xr = 0; x <= maxx; ++x, ++xr) {
            const float weight = wx[xr] * weightY;
            float *dst = film + 4 * ((size_t) y * W + x);
            dst[0] += weight * value[0];
            dst[1] += weight * value[1];
            dst[2] += weight * value[2];
            dst[3] += weight * value[4];
        }
    }
    return true;
}

void prepareScene(orc_scene *s) {
    /* hair AABB = union of segment AABBs (gkdtree.h:990-994) */
    s->aabb = AABB();
    const size_t n = s->hair.v.size();
    for (size_t i = 0; i + 1 < n; ++i) {
        if (s->hair.start[i + 1]) continue;
        V3 mn, mx;
        s->hair.segmentAABB((uint32_t) i, mn, mx);
        s->aabb.expandBy(mn);
        s->aabb.expandBy(mx);
    }
    s->sceneAabb = s->aabb;
    if (s->hasMeshes()) {
        buildMeshBVH(s->meshes, s->rects, s->bvh);
        AABB a;
        if (s->hasHair()) {
            a.expandBy(s->aabb.min);
            a.expandBy(s->aabb.max);
        }
        for (const TriMesh &m : s->meshes) {
            a.expandBy(m.aabb.min);
            a.expandBy(m.aabb.max);
        }
        for (const RectShape &r : s->rects) {
            a.expandBy(r.aabb.min);
            a.expandBy(r.aabb.max);
        }
        /* the scene kd-tree's bounds, slightly enlarged (gkdtree.h:1213-1220; max uses the new min) */
        const float eps = 1e-3f;
        a.min -= (a.max - a.min) * eps + V3(eps);
        a.max += (a.max - a.min) * eps + V3(eps);
        s->sceneAabb = a;
    }
    /* scene.cpp:386-412 + envmap.cpp:336-347: bsphere of (scene AABB U camera position) * 1.5 */
    AABB sc = s->sceneAabb;
    sc.expandBy(V3(s->toWorld[3], s->toWorld[7], s->toWorld[11]));
    V3 center = (sc.max + sc.min) * 0.5f;
    float radius = (center - sc.max).length();
    s->env.bsCenter = center;
    s->env.bsRadius = std::max(kEpsilon, radius * 1.5f);
    s->prepared = true;
}

} // namespace

/* ================================================================== */
/* C API                                                               */
/* ================================================================== */
extern "C" {

orc_scene *orc_scene_create(void) {
    orc_scene *s = new orc_scene();
    for (int i = 0; i < 16; ++i) s->toWorld[i] = (i % 5 == 0) ? 1.0f : 0.0f;
    return s;
}
void orc_scene_destroy(orc_scene *s) { delete s; }
const char *orc_last_error(orc_scene *s) { return s->err.c_str(); }

int orc_set_sobol(orc_scene *s, const uint32_t *m32, const uint64_t *vdc, int vdc_rows,
                  const uint64_t *vdc_inv, int inv_rows) {
    s->m32.assign(m32, m32 + 1024 * 52);
    s->vdc.assign(vdc, vdc + (size_t) vdc_rows * 52);
    s->vdcInv.assign(vdc_inv, vdc_inv + (size_t) inv_rows * 52);
    s->vdcRows = vdc_rows;
    s->invRows = inv_rows;
    return 0;
}

int orc_set_sobol_scramble(orc_scene *s, uint64_t scramble) { /* sobol.cpp:92-102 */
    s->scramble = 0;
    if (scramble) {
        union {
            uint64_t ui64;
            uint32_t v[2];
        } u = {scramble};
        /* qmc.h:146-156 sampleTEA(v0, v1, 4) */
        uint32_t v0 = u.v[0], v1 = u.v[1], sum = 0;
        for (int i = 0; i < 4; ++i) {
            sum += 0x9e3779b9;
            v0 += ((v1 << 4) + 0xA341316C) ^ (v1 + sum) ^ ((v1 >> 5) + 0xC8013EA4);
            v1 += ((v0 << 4) + 0xAD90777D) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7E95761E);
        }
        s->scramble = ((uint64_t) v1 << 32) + v0;
    }
    return 0;
}

int orc_set_camera(orc_scene *s, const float to_world[16], float fov_x_deg, int width, int height,
                   float near_clip, float far_clip) {
    std::memcpy(s->toWorld, to_world, sizeof(float) * 16);
    s->fov = fov_x_deg;
    s->width = width;
    s->height = height;
    s->nearClip = near_clip;
    s->farClip = far_clip;
    setupCamera(s);
    return 0;
}

/* SFMT19937 (src/libcore/random.cpp) as the hair loader's `new Random()` uses it:
   Random() -> seed() -> init_gen_rand(5489) (:473-489, random.h:113), the state
   viewed as 64-bit words (psfmt64), gen_rand_all with the portable do_recursion
   (:170-186, :330-360), gen_rand64 (:296-304), single-precision nextFloat (:630-640). */
struct OracleSfmt {
    enum { N = 19937 / 128 + 1, N32 = N * 4, N64 = N * 2, POS1 = 122, SL1 = 18, SL2 = 1, SR1 = 11, SR2 = 1 };
    union {
        uint64_t u64[N][2];
        uint32_t u32[N][4];
        uint64_t psfmt64[N64];
        uint32_t psfmt32[N32];
    };
    int idx;
    static void rshift128(uint64_t out[2], const uint64_t in[2], int shift) {
        out[0] = (in[0] >> (shift * 8)) | (in[1] << (64 - shift * 8));
        out[1] = in[1] >> (shift * 8);
    }
    static void lshift128(uint64_t out[2], const uint64_t in[2], int shift) {
        out[1] = (in[1] << (shift * 8)) | (in[0] >> (64 - shift * 8));
        out[0] = in[0] << (shift * 8);
    }
    void doRecursion(int r, int a, int b, int c, int d) {
        static const uint32_t MSK[4] = {0xdfffffefU, 0xddfecb7fU, 0xbffaffffU, 0xbffffff6U};
        uint64_t x[2], y[2];
        lshift128(x, u64[a], SL2);
        rshift128(y, u64[c], SR2);
        uint32_t xs[4] = {(uint32_t) x[0], (uint32_t) (x[0] >> 32), (uint32_t) x[1], (uint32_t) (x[1] >> 32)};
        uint32_t ys[4] = {(uint32_t) y[0], (uint32_t) (y[0] >> 32), (uint32_t) y[1], (uint32_t) (y[1] >> 32)};
        uint32_t out[4];
        for (int k = 0; k < 4; ++k)
            out[k] = u32[a][k] ^ xs[k] ^ ((u32[b][k] >> SR1) & MSK[k]) ^ ys[k] ^ (u32[d][k] << SL1);
        for (int k = 0; k < 4; ++k) u32[r][k] = out[k];
    }
    explicit OracleSfmt(uint64_t seed) {
        psfmt64[0] = seed;
        for (int i = 1; i < N64; ++i)
            psfmt64[i] = 6364136223846793005ULL * (psfmt64[i - 1] ^ (psfmt64[i - 1] >> 62)) + (uint64_t) i;
        idx = N32;
        const uint32_t parity[4] = {0x00000001U, 0x00000000U, 0x00000000U, 0x13c9e684U};
        int inner = 0;
        for (int i = 0; i < 4; ++i) inner ^= psfmt32[i] & parity[i];
        for (int i = 16; i > 0; i >>= 1) inner ^= inner >> i;
        if ((inner & 1) == 1) return;
        for (int i = 0; i < 4; ++i) {
            uint32_t work = 1;
            for (int j = 0; j < 32; ++j) {
                if ((work & parity[i]) != 0) {
                    psfmt32[i] ^= work;
                    return;
                }
                work = work << 1;
            }
        }
    }
    uint64_t nextULong() {
        if (idx >= N32) {
            int i, r1 = N - 2, r2 = N - 1;
            for (i = 0; i < N - POS1; ++i) {
                doRecursion(i, i, i + POS1, r1, r2);
                r1 = r2;
                r2 = i;
            }
            for (; i < N; ++i) {
                doRecursion(i, i, i + POS1 - N, r1, r2);
                r1 = r2;
                r2 = i;
            }
            idx = 0;
        }
        uint64_t r = psfmt64[idx / 2];
        idx += 2;
        return r;
    }
    float nextFloat() {
        union {
            uint32_t u;
            float f;
        } x;
        x.u = ((nextULong() & 0xFFFFFFFF) >> 9) | 0x3f800000UL;
        return x.f - 1.0f;
    }
};

/* hair.cpp:609-785 */
int orc_load_hair(orc_scene *s, const char *path, float radius, float angle_threshold_deg,
                  const float *to_world) {
    return orc_load_hair_reduced(s, path, radius, angle_threshold_deg, 0.0f, to_world);
}

int orc_load_hair_reduced(orc_scene *s, const char *path, float radius, float angle_threshold_deg,
                          float reduction, const float *to_world) {
    float angleThreshold = degToRad(angle_threshold_deg);
    float dpThresh = std::cos(angleThreshold);
    float M[16];
    bool ident = true;
    if (to_world) {
        std::memcpy(M, to_world, sizeof(M));
        for (int i = 0; i < 16; ++i) ident &= M[i] == ((i % 5 == 0) ? 1.0f : 0.0f);
    }
    if (reduction < 0 || reduction >= 1) {
        s->err = "The 'reduction' parameter must have a value in [0, 1)!";
        return -1;
    } else if (reduction > 0) {
        float correction = 1.0f / (1 - reduction); /* hair.cpp:622-626 */
        radius *= correction;
    }
    OracleSfmt random(5489ULL);
    bool ignore = false;
    if (!ident) radius *= xformVector(M, V3(0, 0, 1)).length();
    std::ifstream f(path, std::ios::binary);
    if (!f) { s->err = std::string("cannot open ") + path; return -1; }
    std::vector<char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());
    std::vector<V3> vertices;
    std::vector<uint8_t> starts;
    V3 tangent(0.0f), p, lastP(0.0f);
    size_t nDegenerate = 0;
    auto addPoint = [&](V3 pt, bool &newFiber) {
        if (!ident) pt = xformPoint(M, pt);
        if (newFiber) {
            vertices.push_back(pt);
            starts.push_back(1);
            lastP = pt;
            tangent = V3(0.0f);
        } else if (pt != lastP) {
            if (tangent.isZero()) {
                vertices.push_back(pt);
                starts.push_back(0);
                tangent = normalize(pt - lastP);
                lastP = pt;
            } else {
                V3 nextTangent = normalize(pt - lastP);
                if (dot(nextTangent, tangent) > dpThresh) {
                    tangent = normalize(pt - vertices[vertices.size() - 2]);
                    vertices[vertices.size() - 1] = pt;
                } else {
                    vertices.push_back(pt);
                    starts.push_back(0);
                    tangent = nextTangent;
                }
                lastP = pt;
            }
        } else {
            nDegenerate++;
        }
        newFiber = false;
    };
    /* hair.cpp:641-646 reads 11 header bytes first; FileStream::read throws on EOF (fstream.cpp:317) */
    if (buf.size() < 11) { s->err = "truncated hair file (shorter than the 11-byte header)"; return -1; }
    if (std::memcmp(buf.data(), "BINARY_HAIR", 11) == 0) {
        if (buf.size() < 15) { s->err = "truncated hair file"; return -1; }
        uint32_t vertexCount;
        std::memcpy(&vertexCount, buf.data() + 11, 4);
        size_t off = 15;
        auto rd = [&](float &v) -> bool {
            if (off + 4 > buf.size()) return false;
            std::memcpy(&v, buf.data() + off, 4);
            off += 4;
            return true;
        };
        bool newFiber = true;
        for (size_t verticesRead = 0; verticesRead != vertexCount; ++verticesRead) {
            float value;
            if (!rd(value)) { s->err = "truncated hair file"; return -1; }
            if (std::isinf(value)) {
                if (!rd(p.x) || !rd(p.y) || !rd(p.z)) { s->err = "truncated hair file"; return -1; }
                newFiber = true;
                if (reduction > 0) ignore = random.nextFloat() < reduction;
            } else {
                p.x = value;
                if (!rd(p.y) || !rd(p.z)) { s->err = "truncated hair file"; return -1; }
            }
            if (ignore)
                newFiber = false; /* ++nSkipped */
            else
                addPoint(p, newFiber);
        }
    } else {
        std::string text(buf.begin(), buf.end());
        std::istringstream is(text);
        std::string line;
        bool newFiber = true;
        while (is.good()) {
            std::getline(is, line);
            if (line.length() > 0 && line[0] == '#') {
                newFiber = true;
                continue;
            }
            std::istringstream iss(line);
            iss >> p.x >> p.y >> p.z;
            if (!iss.fail()) {
                if (ignore)
                    newFiber = false; /* ++nSkipped */
                else
                    addPoint(p, newFiber);
            } else {
                newFiber = true;
                if (reduction > 0) ignore = random.nextFloat() < reduction;
            }
        }
    }
    starts.push_back(1);
    /* another HairShape of the scene: appended; its first vertex starts a fiber */
    HairGeom &H = s->hair;
    if (!H.start.empty()) H.start.pop_back();
    const uint32_t base = (uint32_t) H.v.size();
    H.v.insert(H.v.end(), vertices.begin(), vertices.end());
    H.start.insert(H.start.end(), starts.begin(), starts.end());
    H.shapeFirst.push_back(base);
    H.shapeRadius.push_back(radius);
    s->bsdfs.emplace_back(); /* Shape::configure default until orc_set_* */
    H.shapeBsdf.push_back((int) s->bsdfs.size() - 1);
    return 0;
}

int64_t orc_hair_vertex_count(orc_scene *s) { return (int64_t) s->hair.v.size(); }

int orc_hair_get(orc_scene *s, float *xyz, uint8_t *starts_fiber) {
    for (size_t i = 0; i < s->hair.v.size(); ++i) {
        xyz[3 * i] = s->hair.v[i].x;
        xyz[3 * i + 1] = s->hair.v[i].y;
        xyz[3 * i + 2] = s->hair.v[i].z;
    }
    std::memcpy(starts_fiber, s->hair.start.data(), s->hair.start.size());
    return 0;
}

int orc_set_kdtree(orc_scene *s, const uint32_t *nodes, int64_t n_nodes, const uint32_t *indices,
                   int64_t n_indices) {
    s->tree.nodes.assign(nodes, nodes + 2 * n_nodes);
    s->tree.indices.assign(indices, indices + n_indices);
    return 0;
}

int orc_hair_aabb(orc_scene *s, float out_min[3], float out_max[3]) {
    if (!s->prepared) prepareScene(s);
    for (int i = 0; i < 3; ++i) {
        out_min[i] = s->aabb.min[i];
        out_max[i] = s->aabb.max[i];
    }
    return 0;
}

int orc_set_marschner(orc_scene *s, float eta, int distribution, float alpha, const float diffuse[3],
                      const float specular[3], const char *dat_dir) {
    BsdfInst &b = lastBsdf(s);
    b.kind = 0;
    b.marschner = Marschner();
    b.marschner.eta = eta;
    b.marschner.alpha = std::max(alpha, (float) 1e-4f); /* microfacet.h:131-132 */
    b.marschner.diffuse = Spec(diffuse[0], diffuse[1], diffuse[2]);
    b.marschner.specular = Spec(specular[0], specular[1], specular[2]);
    if (!b.marschner.configure(distribution, dat_dir, s->err))
        return -1;
    return 0;
}

int orc_set_kajiyakay(orc_scene *s, const float kd[3], const float ks[3], float exponent) {
    BsdfInst &b = lastBsdf(s);
    b.kind = 1;
    b.kk = KajiyaKay();
    b.kk.kd = Spec(kd[0], kd[1], kd[2]);
    b.kk.ks = Spec(ks[0], ks[1], ks[2]);
    b.kk.exponent = exponent;
    b.kk.configure();
    return 0;
}

int orc_set_roughplastic(orc_scene *s, float eta, int distribution, float alpha, int sample_visible,
                         int nonlinear, const float diffuse[3], const float specular[3], const char *dat_dir) {
    if (distribution < 0 || distribution > 2) { s->err = "bad distribution"; return -1; }
    BsdfInst &b = lastBsdf(s);
    b.kind = 2;
    RoughPlastic &r = b.rp;
    r = RoughPlastic();
    r.type = distribution;
    r.eta = eta;
    r.alphaTex = std::max(alpha, 1e-4f);                             /* microfacet.h:135 */
    r.sampleVisible = distribution == 2 ? false : sample_visible != 0; /* microfacet.h:139-143 */
    r.nonlinear = nonlinear != 0;
    r.diffuse = Spec(diffuse[0], diffuse[1], diffuse[2]);
    r.specular = Spec(specular[0], specular[1], specular[2]);
    return r.configure(dat_dir, s->err) ? 0 : -1;
}

int orc_set_marschnerdielectric(orc_scene *s, float eta, const float diffuse[3], const float spec_r[3],
                                const float spec_t[3]) {
    BsdfInst &b = lastBsdf(s);
    b.kind = 3;
    MarschnerDielectric &m = b.md;
    m = MarschnerDielectric();
    m.eta = eta;
    m.diffuse = Spec(diffuse[0], diffuse[1], diffuse[2]);
    m.specR = Spec(spec_r[0], spec_r[1], spec_r[2]);
    m.specT = Spec(spec_t[0], spec_t[1], spec_t[2]);
    m.configure();
    return 0;
}

int orc_set_thindielectric(orc_scene *s, float eta, const float spec_r[3], const float spec_t[3]) {
    BsdfInst &b = lastBsdf(s);
    b.kind = 4;
    b.td = ThinDielectric();
    b.td.eta = eta;
    b.td.specR = Spec(spec_r[0], spec_r[1], spec_r[2]);
    b.td.specT = Spec(spec_t[0], spec_t[1], spec_t[2]);
    b.td.configure();
    return 0;
}

int orc_set_diffuse(orc_scene *s, const float reflectance[3]) {
    BsdfInst &b = lastBsdf(s);
    b.kind = 5;
    b.df = SmoothDiffuse();
    b.df.reflectance = Spec(reflectance[0], reflectance[1], reflectance[2]);
    b.df.configure();
    return 0;
}

/* ---- C1 mesh scene (mesh_bsdf.h, mesh_geom.h) ---- */
int orc_new_bsdf(orc_scene *s) {
    s->bsdfs.emplace_back();
    s->prepared = false;
    return (int) s->bsdfs.size() - 1;
}

int orc_set_diffuse_checkerboard(orc_scene *s, const float color0[3], const float color1[3], float uoffset,
                                 float voffset, float uscale, float vscale) {
    BsdfInst &b = lastBsdf(s);
    b.kind = 5;
    b.df = SmoothDiffuse();
    b.df.textured = true;
    b.df.tex.color0 = Spec(color0[0], color0[1], color0[2]);
    b.df.tex.color1 = Spec(color1[0], color1[1], color1[2]);
    b.df.tex.uoffset = uoffset;
    b.df.tex.voffset = voffset;
    b.df.tex.uscale = uscale;
    b.df.tex.vscale = vscale;
    b.df.configure();
    return 0;
}

int orc_set_plastic(orc_scene *s, float eta, int nonlinear, const float diffuse[3], const float specular[3],
                    int ensure_energy_conservation) {
    BsdfInst &b = lastBsdf(s);
    b.kind = 6;
    b.pl = SmoothPlastic();
    b.pl.eta = eta;
    b.pl.nonlinear = nonlinear != 0;
    b.pl.ensureEnergyConservation = ensure_energy_conservation != 0;
    b.pl.diffuse = Spec(diffuse[0], diffuse[1], diffuse[2]);
    b.pl.specular = Spec(specular[0], specular[1], specular[2]);
    b.pl.configure();
    return 0;
}

int orc_set_twosided(orc_scene *s, int nested0, int nested1) {
    const int n = (int) s->bsdfs.size();
    if (nested0 < 0 || nested0 >= n - 1 || nested1 >= n - 1) { s->err = "twosided: bad nested bsdf index"; return -1; }
    if (nested1 < 0) nested1 = nested0;
    for (int k : {nested0, nested1}) {
        const int kind = s->bsdfs[k].kind;
        if (kind == 0 || kind == 1 || kind == 3 || kind == 4) {
            s->err = "Only materials without a transmission component can be nested!";
            return -1;
        }
    }
    /* the nestable kinds (roughplastic, diffuse, plastic, twosided) are plain values */
    auto copyOf = [&](int k) {
        const BsdfInst &src = s->bsdfs[k];
        auto p = std::make_shared<BsdfInst>();
        p->kind = src.kind;
        p->rp = src.rp;
        p->df = src.df;
        p->pl = src.pl;
        p->nested[0] = src.nested[0];
        p->nested[1] = src.nested[1];
        return p;
    };
    BsdfInst &b = s->bsdfs.back();
    b.nested[0] = copyOf(nested0);
    b.nested[1] = copyOf(nested1);
    b.kind = 7;
    return 0;
}

int orc_add_obj(orc_scene *s, const char *path, const float *to_world, int face_normals, int flip_normals,
                int flip_tex_coords, int bsdf) {
    if (bsdf < 0 || bsdf >= (int) s->bsdfs.size()) { s->err = "obj: bad bsdf index"; return -1; }
    try {
        loadOBJ(path, to_world, face_normals != 0, flip_normals != 0, flip_tex_coords != 0, bsdf, s->meshes);
    } catch (const std::exception &e) {
        s->err = e.what();
        return -1;
    }
    s->prepared = false;
    return 0;
}

int orc_add_rectangle(orc_scene *s, const float *to_world, int flip_normals, int bsdf) {
    if (bsdf < 0 || bsdf >= (int) s->bsdfs.size()) { s->err = "rectangle: bad bsdf index"; return -1; }
    try {
        s->rects.push_back(makeRectangle(to_world, flip_normals != 0, bsdf));
    } catch (const std::exception &e) {
        s->err = e.what();
        return -1;
    }
    s->prepared = false;
    return 0;
}

int orc_mesh_info(orc_scene *s, int64_t *out /* [4]: meshes, triangles, vertices, rectangles */) {
    int64_t tris = 0, verts = 0;
    for (const TriMesh &m : s->meshes) {
        tris += (int64_t) m.triangles();
        verts += (int64_t) m.p.size();
    }
    out[0] = (int64_t) s->meshes.size();
    out[1] = tris;
    out[2] = verts;
    out[3] = (int64_t) s->rects.size();
    return 0;
}

/* BSDF batch with texture coordinates (the last BSDF) */
void orc_bsdf_eval_uv(orc_scene *s, int n, const float *wi, const float *wo, const float *uv, float *out_rgb,
                      float *out_pdf) {
    const BsdfInst &b = s->bsdfs.back();
    for (int i = 0; i < n; ++i) {
        const V3 a(wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]), c(wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]);
        const Spec v = b.eval(a, c, uv + 2 * i);
        for (int k = 0; k < 3; ++k) out_rgb[3 * i + k] = v.s[k];
        out_pdf[i] = b.pdf(a, c, uv + 2 * i);
    }
}

float orc_fresnel_diffuse_reflectance(float eta) { return fresnelDiffuseReflectance(eta); }

/* trace a batch of rays through the whole scene (meshes and hair): t (inf on miss), the
   hit record's shading normal, uv and bsdf index */
void orc_trace_scene(orc_scene *s, int n, const float *o, const float *d, float *out_t, float *out_n,
                     float *out_uv, int32_t *out_bsdf) {
    if (!s->prepared) prepareScene(s);
    for (int i = 0; i < n; ++i) {
        Ray ray(V3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), V3(d[3 * i], d[3 * i + 1], d[3 * i + 2]), kEpsilon, kInf);
        Hit hit;
        out_t[i] = kInf;
        out_bsdf[i] = -1;
        if (!sceneIntersect(s, ray, hit, nullptr)) continue;
        Intersection its;
        fillIntersection(s, ray, hit, its);
        out_t[i] = its.t;
        for (int k = 0; k < 3; ++k) out_n[3 * i + k] = its.shFrame.n[k];
        out_uv[2 * i] = its.uv[0];
        out_uv[2 * i + 1] = its.uv[1];
        out_bsdf[i] = its.bsdf;
    }
}

int orc_set_envmap(orc_scene *s, const float *rgb, int w, int h, float scale, const float *to_world) {
    s->env.w = w;
    s->env.h = h;
    s->env.scale = scale;
    s->env.identity = true;
    if (to_world) {
        for (int i = 0; i < 16; ++i) s->env.identity &= to_world[i] == ((i % 5 == 0) ? 1.0f : 0.0f);
        if (!s->env.identity) {
            double m[9], inv[9];
            for (int r = 0; r < 3; ++r)
                for (int c = 0; c < 3; ++c) {
                    s->env.m[r * 3 + c] = to_world[r * 4 + c];
                    m[r * 3 + c] = to_world[r * 4 + c];
                }
            /* rotation-only: inverse = transpose computed in double (documented) */
            double det = m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
                         m[2] * (m[3] * m[7] - m[4] * m[6]);
            inv[0] = (m[4] * m[8] - m[5] * m[7]) / det;
            inv[1] = (m[2] * m[7] - m[1] * m[8]) / det;
            inv[2] = (m[1] * m[5] - m[2] * m[4]) / det;
            inv[3] = (m[5] * m[6] - m[3] * m[8]) / det;
            inv[4] = (m[0] * m[8] - m[2] * m[6]) / det;
            inv[5] = (m[2] * m[3] - m[0] * m[5]) / det;
            inv[6] = (m[3] * m[7] - m[4] * m[6]) / det;
            inv[7] = (m[1] * m[6] - m[0] * m[7]) / det;
            inv[8] = (m[0] * m[4] - m[1] * m[3]) / det;
            for (int i = 0; i < 9; ++i) s->env.minv[i] = (float) inv[i];
        }
    }
    s->env.build(rgb);
    s->hasEnv = true;
    return 0;
}

int orc_set_sample_count(orc_scene *s, int spp) {
    s->sampleCount = spp > 0 ? spp : 1;
    return 0;
}

int orc_set_integrator(orc_scene *s, int max_depth, int rr_depth, int strict_normals, int hide_emitters) {
    s->maxDepth = max_depth;
    s->rrDepth = rr_depth;
    s->strictNormals = strict_normals != 0;
    s->hideEmitters = hide_emitters != 0;
    return 0;
}

int orc_prepare(orc_scene *s) {
    if (s->m32.empty()) { s->err = "sobol tables not set"; return -1; }
    if (s->width <= 0) { s->err = "camera not set"; return -1; }
    if (!s->hasHair() && !s->hasMeshes()) { s->err = "no shape"; return -1; }
    try {
        prepareScene(s);
    } catch (const std::exception &e) {
        s->err = e.what();
        return -1;
    }
    return 0;
}

int orc_get_camera(orc_scene *s, float sample_to_camera[16], float dx[3], float dy[3]) {
    if (s->width <= 0) { s->err = "camera not set"; return -1; }
    try {
        setupCamera(s);
    } catch (const std::exception &e) {
        s->err = e.what();
        return -1;
    }
    std::memcpy(sample_to_camera, s->s2c, sizeof(s->s2c));
    std::memcpy(dx, s->dx, sizeof(s->dx));
    std::memcpy(dy, s->dy, sizeof(s->dy));
    return 0;
}

static int renderImpl(orc_scene *s, int spp_begin, int spp_end, int n_threads, int shard, int n_shards,
                      float *film, uint64_t *stats) {
    if (!s->prepared && orc_prepare(s) != 0) return -1;
    if (s->hasHair() && s->tree.empty()) { s->err = "kd-tree not set"; return -1; }
    const int W = s->width, H = s->height, BS = 32;
    const int nbx = (W + BS - 1) / BS, nby = (H + BS - 1) / BS, nblocks = nbx * nby;
    /* shard ownership as the GPU renderer deals it (hpt_capi.cpp blockOrder): every
       n_shards-th block along a Hilbert curve over the block grid */
    std::vector<int> myBlocks;
    {
        int n = 1;
        while (n < std::max(nbx, nby)) n <<= 1;
        int k = 0;
        for (long d = 0; d < (long) n * n; ++d) {
            int x = 0, y = 0;
            long t = d;
            for (int sq = 1; sq < n; sq <<= 1) {
                const int rx = 1 & (int) (t / 2), ry = 1 & (int) (t ^ rx);
                if (ry == 0) {
                    if (rx == 1) x = sq - 1 - x, y = sq - 1 - y;
                    std::swap(x, y);
                }
                x += sq * rx;
                y += sq * ry;
                t /= 4;
            }
            if (x < nbx && y < nby) {
                if (k % n_shards == shard) myBlocks.push_back(y * nbx + x);
                ++k;
            }
        }
    }
    (void) nblocks;
    /* each block renders into a (BS+2)^2 RGBW tile with a 1-pixel border, merged in block order */
    const int TS = BS + 2;
    std::vector<float> tiles(myBlocks.size() * (size_t) TS * TS * 4, 0.0f);
    std::atomic<size_t> next(0);
    std::vector<Stats> tstats(std::max(1, n_threads));
    auto worker = [&](int tid) {
        Stats *st = &tstats[tid];
        while (true) {
            size_t bi = next.fetch_add(1);
            if (bi >= myBlocks.size()) break;
            int b = myBlocks[bi];
            int bx0 = (b % nbx) * BS, by0 = (b / nbx) * BS;
            int bw = std::min(BS, W - bx0), bh = std::min(BS, H - by0);
            float *tile = &tiles[bi * (size_t) TS * TS * 4];
            for (int yy = 0; yy < bh; ++yy)
                for (int xx = 0; xx < bw; ++xx) {
                    int px = bx0 + xx, py = by0 + yy;
                    Sampler smp{s};
                    smp.px = px;
                    smp.py = py;
                    for (int j = spp_begin; j < spp_end; ++j) {
                        smp.setSampleIndex((uint64_t) j);
                        float ox, oy;
                        smp.next2D(ox, oy);
                        float posx = px + ox, posy = py + oy;
                        CamRay cr = cameraRay(s, posx, posy);
                        Spec L = Li(s, cr, smp, st, nullptr);
                        /* imageblock.h:124-204 in block-relative coordinates: the block bitmap
                           covers [bx0-1, bx0+bw+1) x [by0-1, by0+bh+1) (border = 1) */
                        float value[5] = {L.s[0], L.s[1], L.s[2], 1.0f, 1.0f};
                        bool ok = true;
                        for (int i = 0; i < 5; ++i)
                            if (!std::isfinite(value[i]) || value[i] < 0) ok = false;
                        if (!ok) { st->badSamples++; continue; }
                        const int sizeX = bw + 2, sizeY = bh + 2;
                        const float rx = posx - 0.5f - (float) (bx0 - 1), ry = posy - 0.5f - (float) (by0 - 1);
                        int minx = std::max((int) std::ceil(rx - 1.0f), 0),
                            miny = std::max((int) std::ceil(ry - 1.0f), 0),
                            maxx = std::min((int) std::floor(rx + 1.0f), sizeX - 1),
                            maxy = std::min((int) std::floor(ry + 1.0f), sizeY - 1);
                        float wx[4], wy[4];
                        for (int x = minx, idx = 0; x <= maxx; ++x) wx[idx++] = gTent.eval(x - rx);
                        for (int y = miny, idx = 0; y <= maxy; ++y) wy[idx++] = gTent.eval(y - ry);
                        for (int y = miny, yr = 0; y <= maxy; ++y, ++yr)
                            for (int x = minx, xr = 0; x <= maxx; ++x, ++xr) {
                                const float weight = wx[xr] * wy[yr];
                                float *dst = tile + 4 * ((size_t) y * TS + x);
                                dst[0] += weight * value[0];
                                dst[1] += weight * value[1];
                                dst[2] += weight * value[2];
                                dst[3] += weight * value[4];
                            }
                    }
                }
        }
    };
    int nt = std::max(1, n_threads);
    std::vector<std::thread> th;
    for (int t = 0; t < nt; ++t) th.emplace_back(worker, t);
    for (auto &t : th) t.join();
    for (size_t bi = 0; bi < myBlocks.size(); ++bi) {
        int b = myBlocks[bi];
        int bx0 = (b % nbx) * BS, by0 = (b / nbx) * BS;
        const float *tile = &tiles[bi * (size_t) TS * TS * 4];
        for (int ty = 0; ty < TS; ++ty)
            for (int tx = 0; tx < TS; ++tx) {
                int x = bx0 - 1 + tx, y = by0 - 1 + ty;
                if (x < 0 || y < 0 || x >= W || y >= H) continue;
                const float *src = tile + 4 * ((size_t) ty * TS + tx);
                float *dst = film + 4 * ((size_t) y * W + x);
                for (int k = 0; k < 4; ++k) dst[k] += src[k];
            }
    }
    if (stats) {
        Stats tot;
        for (auto &t : tstats) {
            tot.rays += t.rays; tot.shadowRays += t.shadowRays; tot.nodes += t.nodes; tot.prims += t.prims;
            tot.paths += t.paths; tot.ewaViolations += t.ewaViolations; tot.bounces += t.bounces;
            tot.badSamples += t.badSamples;
        }
        stats[0] = tot.rays; stats[1] = tot.shadowRays; stats[2] = tot.nodes; stats[3] = tot.prims;
        stats[4] = tot.paths; stats[5] = tot.ewaViolations; stats[6] = tot.bounces; stats[7] = tot.badSamples;
    }
    return 0;
}

int orc_render(orc_scene *s, int spp_begin, int spp_end, int n_threads, float *film_rgbw, uint64_t *stats) {
    return renderImpl(s, spp_begin, spp_end, n_threads, 0, 1, film_rgbw, stats);
}

int orc_render_shard(orc_scene *s, int spp_begin, int spp_end, int n_threads, int shard, int n_shards,
                     float *film_rgbw, uint64_t *stats) {
    return renderImpl(s, spp_begin, spp_end, n_threads, shard, n_shards, film_rgbw, stats);
}

void orc_sobol_lookup(orc_scene *s, int m, int n, const uint32_t *frame, const uint32_t *px,
                      const uint32_t *py, uint64_t *out_index) {
    for (int i = 0; i < n; ++i) out_index[i] = sobolLookUp(s, (uint32_t) m, frame[i], px[i], py[i]);
}

void orc_sobol_sample(orc_scene *s, int n, const uint64_t *index, const uint32_t *dim, float *out) {
    for (int i = 0; i < n; ++i) out[i] = sobolSample(s, index[i], dim[i]);
}

void orc_camera_rays(orc_scene *s, int n, const float *sample_pos, float *o, float *d, float *mint,
                     float *maxt) {
    for (int i = 0; i < n; ++i) {
        CamRay cr = cameraRay(s, sample_pos[2 * i], sample_pos[2 * i + 1]);
        for (int k = 0; k < 3; ++k) {
            o[3 * i + k] = cr.ray.o[k];
            d[3 * i + k] = cr.ray.d[k];
        }
        mint[i] = cr.ray.mint;
        maxt[i] = cr.ray.maxt;
    }
}

void orc_trace_closest(orc_scene *s, int n, const float *o, const float *d, const float *mint,
                       const float *maxt, float *out_t, int32_t *out_iv, float *out_p, int brute_force) {
    if (!s->prepared) prepareScene(s);
    for (int i = 0; i < n; ++i) {
        Ray r(V3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), V3(d[3 * i], d[3 * i + 1], d[3 * i + 2]), mint[i], maxt[i]);
        Hit h;
        bool ok = sceneIntersect(s, r, h, nullptr, brute_force != 0);
        out_t[i] = ok ? h.t : kInf;
        out_iv[i] = ok ? (int32_t) h.iv : -1;
        for (int k = 0; k < 3; ++k) out_p[3 * i + k] = ok ? h.p[k] : 0.0f;
    }
}

void orc_trace_shadow(orc_scene *s, int n, const float *o, const float *d, const float *mint,
                      const float *maxt, uint8_t *out_hit, int brute_force) {
    if (!s->prepared) prepareScene(s);
    for (int i = 0; i < n; ++i) {
        Ray r(V3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), V3(d[3 * i], d[3 * i + 1], d[3 * i + 2]), mint[i], maxt[i]);
        out_hit[i] = sceneOccluded(s, r, nullptr, brute_force != 0) ? 1 : 0;
    }
}

void orc_bsdf_eval(orc_scene *s, int n, const float *wi, const float *wo, float *out_rgb, float *out_pdf) {
    for (int i = 0; i < n; ++i) {
        V3 a(wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]), b(wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]);
        Spec v = bsdfEval(s, a, b);
        for (int k = 0; k < 3; ++k) out_rgb[3 * i + k] = v.s[k];
        out_pdf[i] = bsdfPdf(s, a, b);
    }
}

void orc_bsdf_sample(orc_scene *s, int n, const float *wi, const float *u, float *out_wo, float *out_weight,
                     float *out_pdf, uint32_t *out_type) {
    for (int i = 0; i < n; ++i) {
        V3 a(wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]), wo;
        float pdf = 0;
        uint32_t type = 0;
        Spec v = bsdfSample(s, a, u[2 * i], u[2 * i + 1], wo, pdf, type);
        for (int k = 0; k < 3; ++k) {
            out_wo[3 * i + k] = wo[k];
            out_weight[3 * i + k] = v.s[k];
        }
        out_pdf[i] = pdf;
        out_type[i] = type;
    }
}

int orc_marschner_tables(orc_scene *s, float *nR, float *nTT, float *nTRT, float *out_fdr,
                         float *out_trans100, float *out_spec_weight) {
    if (s->bsdfs.empty() || s->bsdfs.back().kind != 0) return -1;
    const Marschner &mar = s->bsdfs.back().marschner;
    const Azimuthal *lobes[3] = {mar.nR.get(), mar.nTT.get(), mar.nTRT.get()};
    float *outs[3] = {nR, nTT, nTRT};
    for (int l = 0; l < 3; ++l)
        for (int i = 0; i < kAzRes * kAzRes; ++i) {
            outs[l][3 * i] = lobes[l]->table[i].x;
            outs[l][3 * i + 1] = lobes[l]->table[i].y;
            outs[l][3 * i + 2] = lobes[l]->table[i].z;
        }
    *out_fdr = mar.Fdr;
    for (size_t i = 0; i < mar.ext.trans.size() && i < 100; ++i) out_trans100[i] = mar.ext.trans[i];
    *out_spec_weight = mar.specularSamplingWeight;
    return 0;
}

void orc_sfmt(uint64_t seed, int n, uint64_t *out) {
    OracleSfmt r(seed);
    for (int i = 0; i < n; ++i) out[i] = r.nextULong();
}

void orc_gauss_legendre140(float *points, float *weights) {
    GaussLegendre<140> g;
    std::memcpy(points, g.points, sizeof(g.points));
    std::memcpy(weights, g.weights, sizeof(g.weights));
}

void orc_idist_warp(const float *weights, int size, int ndist, int n, const float *dist, const float *u,
                    int *out_x, float *out_u, float *out_pdf, float *out_sum) {
    InterpolatedDistribution1D d(std::vector<float>(weights, weights + (size_t) size * ndist), size, ndist);
    for (int i = 0; i < n; ++i) {
        float uu = u[i];
        int x;
        d.warp(dist[i], uu, x);
        out_x[i] = x;
        out_u[i] = uu;
        out_pdf[i] = d.pdf(dist[i], x);
        out_sum[i] = d.sum(dist[i]);
    }
}

void orc_env_sample(orc_scene *s, int n, const float *ref_p, const float *u, float *out_d, float *out_value,
                    float *out_pdf, float *out_dist) {
    if (!s->prepared) prepareScene(s);
    const EnvMap &E = s->env;
    for (int i = 0; i < n; ++i) {
        Spec value;
        V3 d;
        float pdf;
        E.internalSampleDirection(u[2 * i], u[2 * i + 1], d, value, pdf);
        V3 ref(ref_p[3 * i], ref_p[3 * i + 1], ref_p[3 * i + 2]);
        Ray ray(ref, E.toWorld(d), 0.0f, kInf);
        float nearT, farT;
        bool ok = !(value.isZero() || pdf == 0 || !E.bsphereIntersect(ray, nearT, farT) || nearT >= 0 || farT <= 0);
        Spec v = ok ? value / pdf : Spec(0.0f);
        for (int k = 0; k < 3; ++k) {
            out_d[3 * i + k] = ray.d[k];
            out_value[3 * i + k] = v.s[k];
        }
        out_pdf[i] = ok ? pdf : 0.0f;
        out_dist[i] = ok ? farT : 0.0f;
    }
}

void orc_env_eval(orc_scene *s, int n, const float *d, float *out_rgb, float *out_pdf) {
    for (int i = 0; i < n; ++i) {
        V3 dd(d[3 * i], d[3 * i + 1], d[3 * i + 2]);
        Spec v = s->env.evalEnvironment(dd);
        for (int k = 0; k < 3; ++k) out_rgb[3 * i + k] = v.s[k];
        out_pdf[i] = s->env.internalPdfDirection(s->env.toLocal(dd));
    }
}

void orc_env_eval_filtered(orc_scene *s, int n, const float *d, const float *rx, const float *ry, float *out_rgb) {
    for (int i = 0; i < n; ++i) {
        Spec v = s->env.evalEnvironmentFiltered(V3(d[3 * i], d[3 * i + 1], d[3 * i + 2]),
                                                V3(rx[3 * i], rx[3 * i + 1], rx[3 * i + 2]),
                                                V3(ry[3 * i], ry[3 * i + 1], ry[3 * i + 2]));
        for (int k = 0; k < 3; ++k) out_rgb[3 * i + k] = v.s[k];
    }
}

int orc_env_level(orc_scene *s, int level, float *rgb, int *w, int *h) {
    const int n = (int) s->env.lev.size();
    if (level < 0 || level >= n) return n;
    if (w) *w = s->env.lw[level];
    if (h) *h = s->env.lh[level];
    if (rgb) std::memcpy(rgb, s->env.lev[level].data(), s->env.lev[level].size() * sizeof(float));
    return n;
}

void orc_trace_paths(orc_scene *s, int n, const uint32_t *px, const uint32_t *py, const uint32_t *frame,
                     float *out_rgb, float *out_pos, int32_t *out_depth) {
    if (!s->prepared) orc_prepare(s);
    for (int i = 0; i < n; ++i) {
        Sampler smp{s};
        smp.px = (int) px[i];
        smp.py = (int) py[i];
        smp.setSampleIndex(frame[i]);
        float ox, oy;
        smp.next2D(ox, oy);
        float posx = px[i] + ox, posy = py[i] + oy;
        CamRay cr = cameraRay(s, posx, posy);
        int depth = 0;
        Spec L = Li(s, cr, smp, nullptr, &depth);
        for (int k = 0; k < 3; ++k) out_rgb[3 * i + k] = L.s[k];
        out_pos[2 * i] = posx;
        out_pos[2 * i + 1] = posy;
        out_depth[i] = depth;
    }
}

} /* extern "C" */
