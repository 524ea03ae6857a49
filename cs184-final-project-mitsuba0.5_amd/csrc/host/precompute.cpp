/*
 * precompute.cpp -- per-scene host precomputation for the hair path tracer.
 *
 *   Marschner ("marschner" plugin = src/bsdfs/marschner_diffuse.cpp):
 *     azimuthal scattering tables N_R, N_TT, N_TRT (64x64, :751-847) by a
 *     140-point Gauss-Legendre quadrature (gausssexylingerie.hpp) over a
 *     wrapped-Gaussian detector table; per-lobe sampling CDFs
 *     (Azimuthal ctor :41-62 -> InterpolatedDistribution1D ctor); the rough
 *     dielectric transmittance reduced to a 1-D slice (rtrans.h:292-377) and
 *     the diffuse Fresnel term Fdr (configure :222-238).
 *   Kajiya-Kay (kajiyakay.cpp:80-107): energy conservation + sampling weight.
 *   Environment map (envmap.cpp:244-314): fp16 texels, luminance*sin(theta)
 *     marginal/conditional CDFs, normalisation.
 *   Camera (perspective.cpp:125-165, sobol.cpp:147-158), tent filter LUT
 *     (rfilter.cpp:38-56).
 *
 * All arithmetic is single precision in the reference's operation order,
 * compiled without FMA contraction, so the device consumes the same table
 * bits the reference's constructor would produce.
 */
#include <algorithm>
#include <limits>
#include <array>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"

namespace hpt {
namespace {

const float kPi = 3.14159265358979323846f;
const float kEps = 1e-4f;

inline float clampf(float v, float lo, float hi) { return std::min(hi, std::max(lo, v)); }
inline int clampi(int v, int lo, int hi) { return std::min(hi, std::max(lo, v)); }

/* ---------------- cubic interpolation (libcore/spline.cpp) ---------------- */
float cubic1D(float x, const float *values, size_t size, float min, float max) {
    if (!(x >= min && x <= max)) return 0.0f;
    float t = ((x - min) * (size - 1)) / (max - min);
    size_t k = std::max((size_t) 0, std::min((size_t) t, size - 2));
    float f0 = values[k], f1 = values[k + 1], d0, d1;
    d0 = (k > 0) ? 0.5f * (values[k + 1] - values[k - 1]) : values[k + 1] - values[k];
    d1 = (k + 2 < size) ? 0.5f * (values[k + 2] - values[k]) : values[k + 1] - values[k];
    t = t - (float) k;
    float t2 = t * t, t3 = t2 * t;
    return (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
}

bool knotW(float p, size_t size, float *w, size_t &knot) {
    if (!(p >= 0.0f && p <= 1.0f)) return false;
    float t = ((p - 0.0f) * (size - 1)) / (1.0f - 0.0f);
    knot = std::min((size_t) t, size - 2);
    t = t - (float) knot;
    float t2 = t * t, t3 = t2 * t;
    w[0] = 0.0f;
    w[1] = 2 * t3 - 3 * t2 + 1;
    w[2] = -2 * t3 + 3 * t2;
    w[3] = 0.0f;
    float d0 = t3 - 2 * t2 + t, d1 = t3 - t2;
    if (knot > 0) { w[2] += 0.5f * d0; w[0] -= 0.5f * d0; }
    else { w[2] += d0; w[1] -= d0; }
    if (knot + 2 < size) { w[3] += 0.5f * d1; w[1] -= 0.5f * d1; }
    else { w[2] += d1; w[1] -= d1; }
    return true;
}

float cubic2D(float px, float py, const float *v, size_t sx, size_t sy) {
    float kw[2][4];
    size_t kn[2];
    if (!knotW(px, sx, kw[0], kn[0]) || !knotW(py, sy, kw[1], kn[1])) return 0.0f;
    float r = 0.0f;
    for (int y = -1; y <= 2; ++y) {
        float wy = kw[1][y + 1];
        for (int x = -1; x <= 2; ++x) {
            float w = kw[0][x + 1] * wy;
            if (w == 0) continue;
            r += v[(kn[1] + y) * sx + kn[0] + x] * w;
        }
    }
    return r;
}

float cubic3D(float px, float py, float pz, const float *v, size_t sx, size_t sy, size_t sz) {
    float kw[3][4];
    size_t kn[3];
    if (!knotW(px, sx, kw[0], kn[0]) || !knotW(py, sy, kw[1], kn[1]) || !knotW(pz, sz, kw[2], kn[2]))
        return 0.0f;
    float r = 0.0f;
    for (int z = -1; z <= 2; ++z) {
        float wz = kw[2][z + 1];
        for (int y = -1; y <= 2; ++y) {
            float wyz = kw[1][y + 1] * wz;
            for (int x = -1; x <= 2; ++x) {
                float w = kw[0][x + 1] * wyz;
                if (w == 0) continue;
                r += v[((kn[2] + z) * sy + (kn[1] + y)) * sx + kn[0] + x] * w;
            }
        }
    }
    return r;
}

/* ---------------- rough transmittance (rtrans.h) ---------------- */
struct RTrans {
    size_t nEta = 0, nAlpha = 0, nTheta = 0;
    float etaMin = 0, etaMax = 0, alphaMin = 0, alphaMax = 0;
    std::vector<float> trans, diff;
    bool load(const std::string &path) {
        std::ifstream f(path, std::ios::binary);
        if (!f) return false;
        char hdr[17];
        f.read(hdr, 17);
        if (!f || std::memcmp(hdr, "MTS_TRANSMITTANCE", 17) != 0) return false;
        uint64_t sz[3];
        f.read((char *) sz, 24);
        nEta = sz[0]; nAlpha = sz[1]; nTheta = sz[2];
        float mm[4];
        f.read((char *) mm, 16);
        etaMin = mm[0]; etaMax = mm[1]; alphaMin = mm[2]; alphaMax = mm[3];
        size_t ts = 2 * nEta * nAlpha * nTheta, ds = 2 * nEta * nAlpha;
        std::vector<float> raw(ts + ds);
        f.read((char *) raw.data(), (std::streamsize) (raw.size() * 4));
        if (!f) return false;
        trans.resize(ts);
        diff.resize(ds);
        size_t a = 0, b = 0, p = 0;
        for (size_t i = 0; i < 2 * nEta; ++i)
            for (size_t j = 0; j < nAlpha; ++j) {
                for (size_t k = 0; k < nTheta; ++k) trans[a++] = raw[p++];
                diff[b++] = raw[p++];
            }
        return true;
    }
    /* setEta (rtrans.h:292-345): returns the 2-D (alpha x theta) slice and the 1-D diffuse slice */
    void sliceEta(float eta, std::vector<float> &t2, std::vector<float> &d1) const {
        const float *tr = trans.data(), *dt = diff.data();
        if (eta < 1) {
            tr += nEta * nAlpha * nTheta;
            dt += nEta * nAlpha;
            eta = 1.0f / eta;
        }
        if (eta < etaMin) eta = etaMin;
        float we = std::pow((eta - etaMin) / (etaMax - etaMin), (float) 0.25f);
        t2.assign(nAlpha * nTheta, 0.0f);
        d1.assign(nAlpha, 0.0f);
        float dA = 1.0f / (nAlpha - 1), dT = 1.0f / (nTheta - 1);
        for (size_t i = 0; i < nAlpha; ++i) {
            for (size_t j = 0; j < nTheta; ++j)
                t2[i * nTheta + j] = cubic3D(j * dT, i * dA, we, tr, nTheta, nAlpha, nEta);
            d1[i] = cubic2D(i * dA, we, dt, nAlpha, nEta);
        }
    }
};

/* ---------------- Gauss-Legendre (gausssexylingerie.hpp) ---------------- */
double legendreP(double x, int n) {
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
double legendreD(double x, int n) { return n / (x * x - 1.0) * (x * legendreP(x, n) - legendreP(x, n - 1)); }

void gaussLegendre(int N, std::vector<float> &pts, std::vector<float> &wts) {
    pts.resize(N);
    wts.resize(N);
    for (int i = 0; i < N; ++i) {
        int k = i + 1;
        double x = std::cos(kPi * (4.0 * k - 1.0) / (4.0 * N + 2.0)) *
                   (1.0 - 1.0 / (8.0 * N * N) + 1.0 / (8.0 * N * N * N));
        for (int it = 0; it < 100; ++it) {
            double f = legendreP(x, N);
            x -= f / legendreD(x, N);
            if (std::abs(f) < 1e-6) break;
        }
        pts[i] = float(x);
        wts[i] = float(2.0 / ((1.0 - pts[i] * pts[i]) * legendreD(pts[i], N) * legendreD(pts[i], N)));
    }
}

/* util.cpp:651-681 via util.h:479 */
float fresnelExt(float cosThetaI_, float eta) {
    if (eta == 1) return 0.0f;
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta, cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) return 1.0f;
    float cI = std::abs(cosThetaI_), cT = std::sqrt(cosThetaTSqr);
    float Rs = (cI - eta * cT) / (cI + eta * cT), Rp = (eta * cI - cT) / (eta * cI + cT);
    return 0.5f * (Rs * Rs + Rp * Rp);
}

float gaussDetector(float beta, float theta) {
    return std::exp(-theta * theta / (2.0f * beta * beta)) / (std::sqrt(2.0f * kPi) * beta);
}
float wrappedGauss(float beta, float phi) {
    float result = 0.0f, delta, shift = 0.0f;
    do {
        delta = gaussDetector(beta, phi + shift) + gaussDetector(beta, phi - shift - 2 * kPi);
        result += delta;
        shift += 2 * kPi;
    } while (delta > 1e-4f);
    return result;
}
float lobePhi(float gammaI, float gammaT, int p) { return 2.0f * p * gammaT - 2.0f * gammaI + p * kPi; }

struct F3 {
    float x, y, z;
};

/* InterpolatedDistribution1D ctor (InterpolatedDistribution1D.hpp:36-66) -> cdfs + sums */
void buildIDist(std::vector<float> w, int size, int nd, std::vector<float> &cdf, std::vector<float> &sums) {
    cdf.assign((size_t) (size + 1) * nd, 0.0f);
    sums.assign(nd, 0.0f);
    for (int d = 0; d < nd; ++d) {
        float *c = &cdf[(size_t) d * (size + 1)];
        float *p = &w[(size_t) d * size];
        c[0] = 0.0f;
        for (int x = 0; x < size; ++x) c[x + 1] = p[x] + c[x];
        sums[d] = c[size];
        if (sums[d] < 1e-4f) {
            float ratio = 1.0f / size;
            for (int x = 0; x < size; ++x) {
                p[x] = ratio;
                c[x] = x * ratio;
            }
        } else {
            float scale = 1.0f / sums[d];
            for (int x = 0; x < size; ++x) {
                p[x] *= scale;
                c[x] *= scale;
            }
        }
        c[size] = 1.0f;
    }
}

} // namespace

bool precomputeMarschner(const BsdfDesc &d, const std::string &dataDir, MarschnerHost &out, std::string &err) {
    const float eta = d.intIOR / d.extIOR;
    const float betaR = 0.1f, betaTT = betaR * 0.5f, betaTRT = betaR * 2.0f;
    const F3 sigmaA{0.5f, 0.5f, 0.5f};
    const int R = HPT_AZ_RES, NP = 140, NG = 2048;
    std::vector<float> pts, wts;
    gaussLegendre(NP, pts, wts);
    std::vector<float> gammaI(NP);
    for (int i = 0; i < NP; ++i) gammaI[i] = std::asin(pts[i]);
    std::vector<float> Ds(NG);
    for (int i = 0; i < NG; ++i) Ds[i] = wrappedGauss(betaR, i / (NG - 1.0f) * 2 * kPi);
    auto approxD = [&](float phi) {
        float u = std::abs(phi * (1.0 / (2 * kPi) * (NG - 1)));
        int x0 = int(u), x1 = x0 + 1;
        u -= x0;
        return Ds[x0 % NG] * (1.0f - u) + Ds[x1 % NG] * u;
    };
    std::vector<F3> vals[3];
    for (auto &v : vals) v.resize(R * R);
    std::vector<float> fres(NP), gammaT(NP);
    std::vector<F3> absorb(NP);
    for (int y = 0; y < R; ++y) {
        float ch = y / (R - 1.0f);
        float iorPrime = std::sqrt(eta * eta - (1.0f - ch * ch)) / ch;
        float cosThetaT = std::sqrt(1.0f - (1.0f - ch * ch) * (1.0f / eta) * (1.0f / eta));
        float rc = 1.0f / cosThetaT;
        F3 sp{sigmaA.x * rc, sigmaA.y * rc, sigmaA.z * rc};
        for (int i = 0; i < NP; ++i) {
            gammaT[i] = std::asin(clampf(pts[i] / iorPrime, -1.0f, 1.0f));
            fres[i] = fresnelExt(1.0f / eta, ch * std::cos(gammaI[i])); /* swapped arguments, :809 */
            float c = std::cos(gammaT[i]);
            absorb[i] = {std::exp(-sp.x * 2.0f * c), std::exp(-sp.y * 2.0f * c), std::exp(-sp.z * 2.0f * c)};
        }
        for (int phiI = 0; phiI < R; ++phiI) {
            float phi = kPi * 2 * phiI / (R - 1.0f);
            float iR = 0.0f;
            F3 iTT{0, 0, 0}, iTRT{0, 0, 0};
            for (int i = 0; i < NP; ++i) {
                float fR = fres[i];
                F3 T = absorb[i];
                float k = (1.0f - fR) * (1.0f - fR);
                F3 ATT{k * T.x, k * T.y, k * T.z};
                F3 ATRT{ATT.x * fR * T.x, ATT.y * fR * T.y, ATT.z * fR * T.z};
                iR += wts[i] * approxD(phi - lobePhi(gammaI[i], gammaT[i], 0)) * fR;
                float wTT = wts[i] * approxD(phi - lobePhi(gammaI[i], gammaT[i], 1));
                iTT.x += wTT * ATT.x; iTT.y += wTT * ATT.y; iTT.z += wTT * ATT.z;
                float wTRT = wts[i] * approxD(phi - lobePhi(gammaI[i], gammaT[i], 2));
                iTRT.x += wTRT * ATRT.x; iTRT.y += wTRT * ATRT.y; iTRT.z += wTRT * ATRT.z;
            }
            float hR = 0.5f * iR;
            vals[0][phiI + y * R] = {hR, hR, hR};
            vals[1][phiI + y * R] = {0.5f * iTT.x, 0.5f * iTT.y, 0.5f * iTT.z};
            vals[2][phiI + y * R] = {0.5f * iTRT.x, 0.5f * iTRT.y, 0.5f * iTRT.z};
        }
    }
    for (int l = 0; l < 3; ++l) {
        out.table[l].resize(R * R);
        std::vector<float> w(R * R);
        for (int i = 0; i < R * R; ++i) {
            const F3 &v = vals[l][i];
            out.table[l][i] = {v.x, v.y, v.z, 0.0f};
            w[i] = std::max(std::max(v.x, v.y), v.z);
        }
        /* dilation (marschner_diffuse.cpp:47-59) */
        for (int y = 0; y < R; ++y) {
            for (int x = 0; x < R - 1; ++x) w[x + y * R] = std::max(w[x + y * R], w[x + 1 + y * R]);
            for (int x = R - 1; x > 0; --x) w[x + y * R] = std::max(w[x + y * R], w[x - 1 + y * R]);
        }
        for (int x = 0; x < R; ++x) {
            for (int y = 0; y < R - 1; ++y) w[x + y * R] = std::max(w[x + y * R], w[x + (y + 1) * R]);
            for (int y = R - 1; y > 0; --y) w[x + y * R] = std::max(w[x + y * R], w[x + (y - 1) * R]);
        }
        buildIDist(std::move(w), R, R, out.cdf[l], out.sums[l]);
    }
    out.vR = betaR * betaR;
    out.vTT = betaTT * betaTT;
    out.vTRT = betaTRT * betaTRT;
    out.scaleAngleRad = -0.1f;
    /* configure (:193-247) */
    float spec[3] = {d.specular[0], d.specular[1], d.specular[2]};
    float smax = std::max(std::max(spec[0], spec[1]), spec[2]);
    if (smax > 1.0f) {
        float s = 0.99f * (1.0f / smax);
        for (auto &v : spec) v *= s;
    }
    float dAvg = d.diffuse[0] * 0.212671f + d.diffuse[1] * 0.715160f + d.diffuse[2] * 0.072169f;
    float sAvg = spec[0] * 0.212671f + spec[1] * 0.715160f + spec[2] * 0.072169f;
    out.specularSamplingWeight = sAvg / (dAvg + sAvg);
    out.invEta2 = 1.0f / (eta * eta);
    for (int i = 0; i < 3; ++i) out.diffuse[i] = d.diffuse[i];
    /* rough transmittance slices (rtrans.h) */
    float alpha = std::max(d.alpha, 1e-4f);
    if (eta < 1) { err = "marschner: eta < 1 is not supported by the transmittance tables"; return false; }
    return roughTransmittance(dataDir, d.distribution, eta, alpha, alpha, out.trans, out.fdr, err);
}

bool roughTransmittance(const std::string &dataDir, const std::string &distribution, float eta, float alphaSlice,
                        float alphaDiffuse, std::vector<float> &trans, float &fdr, std::string &err) {
    RTrans rt;
    std::string path = dataDir + "/microfacet/" + distribution + ".dat";
    if (!rt.load(path)) {
        err = "cannot load rough transmittance data \"" + path + "\"";
        return false;
    }
    /* checkEta / checkAlpha (rtrans.h:390-407) */
    float etaC = eta < 1 ? 1 / eta : eta;
    if (etaC < rt.etaMin || etaC > rt.etaMax) {
        err = "the requested relative index of refraction eta=" + std::to_string(eta) +
              " is outside of the supported range";
        return false;
    }
    if (alphaSlice < rt.alphaMin || alphaSlice > rt.alphaMax) {
        err = "the requested roughness value alpha=" + std::to_string(alphaSlice) +
              " is outside of the supported range";
        return false;
    }
    std::vector<float> ext2, extD, int2, intD;
    rt.sliceEta(eta, ext2, extD);
    rt.sliceEta(1 / eta, int2, intD);
    /* setAlpha (rtrans.h:353-388) on the external copy */
    float wa = std::pow((alphaSlice - rt.alphaMin) / (rt.alphaMax - rt.alphaMin), (float) 0.25f);
    trans.resize(rt.nTheta);
    float dT = 1.0f / (rt.nTheta - 1);
    for (size_t i = 0; i < rt.nTheta; ++i) trans[i] = cubic2D(i * dT, wa, ext2.data(), rt.nTheta, rt.nAlpha);
    /* evalDiffuse(alpha) (rtrans.h:249-260) on the internal 2D copy */
    float wd = std::pow((alphaDiffuse - rt.alphaMin) / (rt.alphaMax - rt.alphaMin), (float) 0.25f);
    float internalDiffuse = cubic1D(wd, intD.data(), rt.nAlpha, 0.0f, 1.0f);
    internalDiffuse = std::min(1.0f, std::max(0.0f, internalDiffuse));
    fdr = 1 - internalDiffuse;
    return true;
}

bool configureRoughPlastic(const BsdfDesc &d, const std::string &dataDir, RoughPlasticHost &out, std::string &err) {
    /* RoughPlastic(props) + configure (roughplastic.cpp:197-299) */
    const float eta = d.intIOR / d.extIOR;
    if (d.intIOR < 0 || d.extIOR < 0 || d.intIOR == d.extIOR) {
        err = "roughplastic: the interior and exterior indices of refraction must be positive and differ";
        return false;
    }
    HptRoughPlastic &rp = out.p;
    rp.type = d.distribution == "beckmann" ? 0 : d.distribution == "ggx" ? 1 : 2;
    rp.sampleVisible = rp.type == 2 ? 0 : (d.sampleVisible ? 1 : 0);
    rp.nonlinear = d.nonlinear ? 1 : 0;
    /* m_alpha = ConstantFloatTexture(distr.getAlpha()); every use reads eval().average() (spectrum.h:481-486)
     * and a MicrofacetDistribution built from it clamps to 1e-4 again (microfacet.h:67-75) */
    const float a0 = std::max(d.alpha, 1e-4f);
    const float aAvg = (((0.0f + a0) + a0) + a0) * (1.0f / 3);
    rp.alpha = std::max(aAvg, 1e-4f);
    rp.exponent = std::max(2.0f / (rp.alpha * rp.alpha) - 2.0f, 0.0f); /* computePhongExponent (:701-704) */
    rp.eta = eta;
    rp.invEta2 = 1.0f / (eta * eta);
    float spec[3] = {d.specular[0], d.specular[1], d.specular[2]};
    float diff[3] = {d.diffuse[0], d.diffuse[1], d.diffuse[2]};
    if (d.ensureEnergyConservation) { /* bsdf.cpp:88-113, max = 1 */
        for (float *v : {spec, diff}) {
            float mx = std::max(std::max(v[0], v[1]), v[2]);
            if (mx > 1.0f) {
                float s = 0.99f * (1.0f / mx);
                for (int i = 0; i < 3; ++i) v[i] *= s;
            }
        }
    }
    float dAvg = diff[0] * 0.212671f + diff[1] * 0.715160f + diff[2] * 0.072169f;
    float sAvg = spec[0] * 0.212671f + spec[1] * 0.715160f + spec[2] * 0.072169f;
    rp.specularSamplingWeight = sAvg / (dAvg + sAvg);
    for (int i = 0; i < 3; ++i) {
        rp.diffuse[i] = diff[i];
        rp.specular[i] = spec[i];
    }
    if (!roughTransmittance(dataDir, d.distribution, eta, aAvg, rp.alpha, out.trans, rp.fdr, err)) {
        err = "roughplastic: " + err;
        return false;
    }
    rp.trans = nullptr;
    rp.transSize = (int) out.trans.size();
    return true;
}

void configureMarschnerDielectric(const BsdfDesc &d, HptMarschnerDielectric &out) {
    /* MarschnerDielectric(props) + configure (marschnerdielectric.cpp:147-211) */
    out.eta = d.intIOR / d.extIOR;
    float sr[3] = {d.specular[0], d.specular[1], d.specular[2]};
    float st[3] = {d.transmittance[0], d.transmittance[1], d.transmittance[2]};
    if (d.ensureEnergyConservation) { /* bsdf.cpp:88-113, each texture separately, max = 1 */
        for (float *v : {sr, st}) {
            float mx = std::max(std::max(v[0], v[1]), v[2]);
            if (mx > 1.0f) {
                float s = 0.99f * (1.0f / mx);
                for (int i = 0; i < 3; ++i) v[i] *= s;
            }
        }
    }
    float dAvg = d.diffuse[0] * 0.212671f + d.diffuse[1] * 0.715160f + d.diffuse[2] * 0.072169f;
    float sAvg = sr[0] * 0.212671f + sr[1] * 0.715160f + sr[2] * 0.072169f;
    float tAvg = st[0] * 0.212671f + st[1] * 0.715160f + st[2] * 0.072169f;
    out.specularSamplingWeight = (sAvg + tAvg) / (dAvg + sAvg + tAvg);
    for (int i = 0; i < 3; ++i) {
        out.specR[i] = sr[i];
        out.specT[i] = st[i];
    }
}

void configureThinDielectric(const BsdfDesc &d, HptMarschnerDielectric &out) {
    /* ThinDielectric(props) + configure (thindielectric.cpp:73-125) */
    out.eta = d.intIOR / d.extIOR;
    out.specularSamplingWeight = 1.0f; /* no diffuse component: the sample is never split */
    float sr[3] = {d.specular[0], d.specular[1], d.specular[2]};
    float st[3] = {d.transmittance[0], d.transmittance[1], d.transmittance[2]};
    if (d.ensureEnergyConservation) {
        for (float *v : {sr, st}) {
            float mx = std::max(std::max(v[0], v[1]), v[2]);
            if (mx > 1.0f) {
                float s = 0.99f * (1.0f / mx);
                for (int i = 0; i < 3; ++i) v[i] *= s;
            }
        }
    }
    for (int i = 0; i < 3; ++i) {
        out.specR[i] = sr[i];
        out.specT[i] = st[i];
    }
}

void configureDiffuse(const BsdfDesc &d, HptDiffuse &out) {
    /* SmoothDiffuse::configure (diffuse.cpp:77-88) */
    float v[3] = {d.diffuse[0], d.diffuse[1], d.diffuse[2]};
    float mx = std::max(std::max(v[0], v[1]), v[2]);
    if (d.ensureEnergyConservation && mx > 1.0f) {
        float s = 0.99f * (1.0f / mx);
        for (int i = 0; i < 3; ++i) v[i] *= s;
    }
    for (int i = 0; i < 3; ++i) out.refl[i] = v[i];
}

void configureKajiyaKay(const BsdfDesc &d, HptKajiyaKay &out) {
    float kd[3] = {d.diffuse[0], d.diffuse[1], d.diffuse[2]};
    float ks[3] = {d.specular[0], d.specular[1], d.specular[2]};
    float mx = std::max(std::max(ks[0] + kd[0], ks[1] + kd[1]), ks[2] + kd[2]);
    if (mx > 1.0f) {
        float s = 0.99f * (1.0f / mx);
        for (int i = 0; i < 3; ++i) { ks[i] *= s; kd[i] *= s; }
    }
    float dAvg = kd[0] * 0.212671f + kd[1] * 0.715160f + kd[2] * 0.072169f;
    float sAvg = ks[0] * 0.212671f + ks[1] * 0.715160f + ks[2] * 0.072169f;
    for (int i = 0; i < 3; ++i) { out.kd[i] = kd[i]; out.ks[i] = ks[i]; }
    out.exponent = d.exponent;
    out.specularSamplingWeight = sAvg / (dAvg + sAvg);
}

/* ---------------- IEEE half ---------------- */
uint16_t floatToHalf(float f) {
    uint32_t x;
    std::memcpy(&x, &f, 4);
    uint32_t sign = (x >> 16) & 0x8000u, ax = x & 0x7fffffffu;
    if (ax >= 0x7f800000u) return (uint16_t) (sign | 0x7c00u | (ax > 0x7f800000u ? 0x200u : 0u));
    if (ax >= 0x477ff000u) return (uint16_t) (sign | 0x7c00u);
    if (ax < 0x38800000u) {
        if (ax < 0x33000000u) return (uint16_t) sign;
        uint32_t m = (ax & 0x007fffffu) | 0x00800000u;
        int shift = 126 - (int) (ax >> 23);
        uint32_t hm = m >> shift, rem = m & ((1u << shift) - 1u), half = 1u << (shift - 1);
        if (rem > half || (rem == half && (hm & 1u))) hm++;
        return (uint16_t) (sign | hm);
    }
    uint32_t h = (((ax >> 23) - 112u) << 10) | ((ax >> 13) & 0x3ffu), rem = ax & 0x1fffu;
    if (rem > 0x1000u || (rem == 0x1000u && (h & 1u))) h++;
    return (uint16_t) (sign | h);
}

float halfToFloat(uint16_t h) {
    uint32_t sign = (uint32_t) (h & 0x8000u) << 16, e = (h >> 10) & 0x1fu, m = h & 0x3ffu, x;
    if (e == 0) {
        if (m == 0) x = sign;
        else {
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

/* ---------------- environment map (envmap.cpp:244-314) ---------------- */
void buildEnvMap(EnvHost &env) {
    const int w = env.w, h = env.h;
    env.texel.resize((size_t) w * h);
    for (size_t i = 0; i < (size_t) w * h; ++i) {
        float c[3];
        for (int k = 0; k < 3; ++k) c[k] = halfToFloat(floatToHalf(std::max(env.rgb[3 * i + k], 0.0f)));
        env.texel[i] = {c[0], c[1], c[2], 0.0f};
    }
    env.cdfCols.assign((size_t) (w + 1) * h, 0.0f);
    env.cdfRows.assign(h + 1, 0.0f);
    env.rowWeights.assign(h, 0.0f);
    size_t colPos = 0, rowPos = 0;
    float rowSum = 0.0f;
    env.cdfRows[rowPos++] = 0;
    for (int y = 0; y < h; ++y) {
        float colSum = 0;
        env.cdfCols[colPos++] = 0;
        for (int x = 0; x < w; ++x) {
            const HptF4 &t = env.texel[(size_t) y * w + x];
            colSum += t.x * 0.212671f + t.y * 0.715160f + t.z * 0.072169f;
            env.cdfCols[colPos++] = (float) colSum;
        }
        float norm = 1.0f / (float) colSum;
        for (int x = 1; x < w; ++x) env.cdfCols[colPos - x - 1] *= norm;
        env.cdfCols[colPos - 1] = 1.0f;
        float weight = std::sin((y + 0.5f) * kPi / h);
        env.rowWeights[y] = weight;
        rowSum += colSum * weight;
        env.cdfRows[rowPos++] = (float) rowSum;
    }
    float norm = 1.0f / (float) rowSum;
    for (int y = 1; y < h; ++y) env.cdfRows[rowPos - y - 1] *= norm;
    env.cdfRows[rowPos - 1] = 1.0f;
    if (rowSum == 0) throw std::runtime_error("The environment map is completely black -- this is not allowed.");
    if (!std::isfinite(rowSum))
        throw std::runtime_error("The environment map contains an invalid floating point value (nan/inf)");
    env.normalization = 1.0f / (rowSum * (2 * kPi / w) * (kPi / h));
    env.pixelSizeX = 2 * kPi / w;
    env.pixelSizeY = kPi / h;
    /* guide tables: the device's lower_bound starts between the entries bracketing
       sample's bucket [k/G, (k+1)/G) -- the same first entry >= sample */
    const int G = HPT_ENV_GUIDE;
    auto guide = [&](const float *cdf, uint32_t n, uint32_t *out) {
        for (int k = 0; k <= G; ++k)
            out[k] = (uint32_t) (std::lower_bound(cdf, cdf + n, (float) k / (float) G) - cdf);
    };
    env.guideRows.assign(G + 1, 0);
    guide(env.cdfRows.data(), (uint32_t) h + 1, env.guideRows.data());
    env.guideCols.assign((size_t) h * (G + 1), 0);
    for (int y = 0; y < h; ++y)
        guide(env.cdfCols.data() + (size_t) y * (w + 1), (uint32_t) w + 1, env.guideCols.data() + (size_t) y * (G + 1));
}

/* ---------------- MIP pyramid (envmap.cpp:165-182, mipmap.h:155-302) ---------------- */
namespace {
/* 2-lobed Lanczos sinc filter (lanczos.cpp:43-55) */
float lanczos2(float x) {
    const float radius = 2.0f;
    x = std::abs(x);
    if (x < 1e-4f) return 1.0f; /* Epsilon */
    if (x > radius) return 0.0f;
    const float x1 = kPi * x; /* M_PI is M_PI_FLT under SINGLE_PRECISION (constants.h:80) */
    const float x2 = x1 / radius;
    return (std::sin(x1) * std::sin(x2)) / (x1 * x2);
}

/* Resampler<float> (rfilter.h:107-198) resampling one axis from src to dst samples,
   then resampleAndClamp (:232-280) on `channels` interleaved channels */
struct AxisResampler {
    int src, dst, taps;
    bool repeat; /* ERepeat, else EClamp */
    std::vector<int> start;
    std::vector<float> weights;
    AxisResampler(int sourceRes, int targetRes, bool rep) : src(sourceRes), dst(targetRes), repeat(rep) {
        float filterRadius = 2.0f, scale = 1.0f, invScale = 1.0f;
        if (targetRes < sourceRes) {
            scale = (float) sourceRes / (float) targetRes;
            invScale = 1 / scale;
            filterRadius *= scale;
        }
        taps = (int) std::ceil(filterRadius * 2);
        start.resize(targetRes);
        weights.resize((size_t) taps * targetRes);
        for (int i = 0; i < targetRes; i++) {
            const float center = (i + 0.5f) / targetRes * sourceRes;
            start[i] = (int) std::floor(center - filterRadius + 0.5f);
            float sum = 0;
            for (int j = 0; j < taps; j++) {
                const float pos = start[i] + j + 0.5f - center;
                const float weight = lanczos2(pos * invScale);
                weights[(size_t) i * taps + j] = weight;
                sum += weight;
            }
            const float normalization = 1.0f / sum;
            for (int j = 0; j < taps; j++) weights[(size_t) i * taps + j] *= normalization;
        }
    }
    int at(int pos) const { /* lookup (rfilter.h:437-458) */
        if (pos < 0 || pos >= src) {
            if (repeat) {
                pos %= src;
                if (pos < 0) pos += src;
            } else {
                pos = std::min(std::max(pos, 0), src - 1);
            }
        }
        return pos;
    }
    /* clamp to [0, inf): min = 0, max = +infinity as MIPMap passes them (mipmap.h:261) */
    void run(const float *source, size_t sourceStride, float *target, size_t targetStride, int channels) const {
        const float mn = 0.0f, mx = std::numeric_limits<float>::infinity();
        for (int i = 0; i < dst; ++i)
            for (int ch = 0; ch < channels; ++ch) {
                float result = 0;
                for (int j = 0; j < taps; ++j)
                    result += source[sourceStride * channels * (size_t) at(start[i] + j) + ch] *
                              weights[(size_t) i * taps + j];
                const float lo = (mn < result) ? result : mn; /* std::max(min, result) */
                target[targetStride * channels * (size_t) i + ch] = (lo < mx) ? lo : mx; /* std::min(max, .) */
            }
    }
};

/* Bitmap::resample (bitmap.cpp:2230-2329): x pass (bcu = repeat) then y pass (bcv = clamp) */
std::vector<float> resampleRGB(const std::vector<float> &in, int w, int h, int nw, int nh) {
    std::vector<float> cur = in;
    int cw = w;
    if (nw != w) {
        AxisResampler r(w, nw, true);
        std::vector<float> tmp((size_t) nw * h * 3);
        for (int y = 0; y < h; ++y) r.run(&cur[(size_t) y * w * 3], 1, &tmp[(size_t) y * nw * 3], 1, 3);
        cur.swap(tmp);
        cw = nw;
    }
    if (nh != h) {
        AxisResampler r(h, nh, false);
        std::vector<float> tmp((size_t) cw * nh * 3);
        for (int x = 0; x < cw; ++x) r.run(&cur[(size_t) x * 3], cw, &tmp[(size_t) x * 3], cw, 3);
        cur.swap(tmp);
    }
    return cur;
}
} // namespace

void buildEnvMipmap(EnvHost &env) {
    const int w0 = env.w, h0 = env.h;
    /* level 0: the bitmap with negative values clamped (mipmap.h:226-240), stored as half */
    std::vector<float> bitmap(env.rgb.size());
    for (size_t i = 0; i < bitmap.size(); ++i) bitmap[i] = std::max(env.rgb[i], 0.0f);
    env.mip.clear();
    env.levelW.clear();
    env.levelH.clear();
    env.levelOff.clear();
    env.ratioX.clear();
    env.ratioY.clear();
    auto store = [&](const std::vector<float> &b, int w, int h) {
        env.levelW.push_back(w);
        env.levelH.push_back(h);
        env.levelOff.push_back((int) env.mip.size());
        env.ratioX.push_back((float) w / (float) w0);
        env.ratioY.push_back((float) h / (float) h0);
        for (size_t i = 0; i < (size_t) w * h; ++i)
            env.mip.push_back({halfToFloat(floatToHalf(b[3 * i])), halfToFloat(floatToHalf(b[3 * i + 1])),
                               halfToFloat(floatToHalf(b[3 * i + 2])), 0.0f});
    };
    store(bitmap, w0, h0);
    /* progressively downsample the float bitmap until 1x1 (mipmap.h:245-270) */
    int w = w0, h = h0;
    while (w > 1 || h > 1) {
        const int nw = std::max(1, (w + 1) / 2), nh = std::max(1, (h + 1) / 2);
        bitmap = resampleRGB(bitmap, w, h, nw, nh);
        w = nw;
        h = nh;
        store(bitmap, w, h);
    }
    /* Gaussian weight LUT (mipmap.h:296-301); fastexp(float) = (float) exp((double) x) on Linux/x86-64 */
    for (int i = 0; i < HPT_EWA_LUT; ++i) {
        const float r2 = (float) i / (float) (HPT_EWA_LUT - 1);
        env.ewaLut[i] = (float) std::exp((double) (-2.0f * r2)) - (float) std::exp((double) -2.0f);
    }
}

bool loadEnvFile(const std::string &path, EnvHost &env, std::string &err) {
    std::ifstream f(path, std::ios::binary);
    if (!f) { err = "cannot open environment map \"" + path + "\""; return false; }
    std::string line;
    std::getline(f, line);
    if (line == "PF") { /* portable float map */
        int w, h;
        float scale;
        f >> w >> h >> scale;
        f.get();
        std::vector<float> data((size_t) w * h * 3);
        f.read((char *) data.data(), (std::streamsize) (data.size() * 4));
        env.w = w;
        env.h = h;
        env.rgb.resize(data.size());
        for (int y = 0; y < h; ++y) /* PFM rows are bottom-to-top */
            std::memcpy(&env.rgb[(size_t) y * w * 3], &data[(size_t) (h - 1 - y) * w * 3], (size_t) w * 3 * 4);
        return true;
    }
    if (line.rfind("#?", 0) == 0) { /* Radiance RGBE */
        while (std::getline(f, line) && !line.empty()) {}
        std::getline(f, line);
        int w = 0, h = 0;
        char a[3], b[3];
        if (std::sscanf(line.c_str(), "%2s %d %2s %d", a, &h, b, &w) != 4) { err = "bad RGBE header"; return false; }
        std::vector<unsigned char> scan((size_t) w * 4);
        env.w = w;
        env.h = h;
        env.rgb.assign((size_t) w * h * 3, 0.0f);
        for (int y = 0; y < h; ++y) {
            int c0 = f.get(), c1 = f.get(), c2 = f.get(), c3 = f.get();
            if (c0 == 2 && c1 == 2 && ((c2 << 8) | c3) == w) { /* new RLE */
                for (int ch = 0; ch < 4; ++ch) {
                    int x = 0;
                    while (x < w) {
                        int cnt = f.get();
                        if (cnt > 128) {
                            cnt -= 128;
                            int v = f.get();
                            for (int k = 0; k < cnt && x < w; ++k) scan[(size_t) (x++) * 4 + ch] = (unsigned char) v;
                        } else {
                            for (int k = 0; k < cnt && x < w; ++k) scan[(size_t) (x++) * 4 + ch] = (unsigned char) f.get();
                        }
                    }
                }
            } else {
                scan[0] = (unsigned char) c0; scan[1] = (unsigned char) c1;
                scan[2] = (unsigned char) c2; scan[3] = (unsigned char) c3;
                f.read((char *) scan.data() + 4, (std::streamsize) ((size_t) w * 4 - 4));
            }
            for (int x = 0; x < w; ++x) {
                unsigned char *p = &scan[(size_t) x * 4];
                float s = p[3] ? std::ldexp(1.0f, p[3] - 136) : 0.0f;
                float *o = &env.rgb[3 * ((size_t) y * w + x)];
                o[0] = p[0] * s;
                o[1] = p[1] * s;
                o[2] = p[2] * s;
            }
        }
        return true;
    }
    err = "unsupported environment map format (need .pfm or Radiance .hdr): " + path;
    return false;
}

/* ---------------- camera (perspective.cpp:125-165) ---------------- */
/* The reference builds sampleToCamera from single-precision Transforms:
   m_cameraToSample = S(1/relSize) * T(-relOffset) * S(-0.5, -0.5 aspect, 1)
   * T(-1, -1/aspect, 0) * perspective(xfov, near, far) (perspective.cpp:
   150-155), each product of Transform (transform.cpp:28-31) multiplying the
   matrices left to right and the inverses right to left (matrix.h:743-756:
   sum = 0, sum += a_ik b_kj in k order), the inverse of perspective() coming
   from Matrix4x4::invert, a float Gauss-Jordan elimination with full
   pivoting (transform.h:50-55, matrix.inl:138-190); m_sampleToCamera is that
   composed inverse (perspective.cpp:157).  Everything below is float. */
namespace {
typedef std::array<float, 16> M44;
M44 mmul(const M44 &a, const M44 &b) {
    M44 r;
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float sum = 0;
            for (int k = 0; k < 4; ++k) sum += a[i * 4 + k] * b[k * 4 + j];
            r[i * 4 + j] = sum;
        }
    return r;
}
/* Matrix<4,4,float>::invert (matrix.inl:138-190) */
bool gaussJordanInvert(const M44 &src, M44 &t) {
    int indxc[4], indxr[4], ipiv[4] = {0, 0, 0, 0};
    t = src;
    auto m = [&](int r, int c) -> float & { return t[r * 4 + c]; };
    for (int i = 0; i < 4; i++) {
        int irow = -1, icol = -1;
        float big = 0;
        for (int j = 0; j < 4; j++) {
            if (ipiv[j] == 1) continue;
            for (int k = 0; k < 4; k++) {
                if (ipiv[k] == 0) {
                    if (std::abs(m(j, k)) >= big) {
                        big = std::abs(m(j, k));
                        irow = j;
                        icol = k;
                    }
                } else if (ipiv[k] > 1) {
                    return false;
                }
            }
        }
        ++ipiv[icol];
        if (irow != icol)
            for (int k = 0; k < 4; ++k) std::swap(m(irow, k), m(icol, k));
        indxr[i] = irow;
        indxc[i] = icol;
        if (m(icol, icol) == 0) return false;
        const float pivinv = 1.f / m(icol, icol);
        m(icol, icol) = 1.f;
        for (int j = 0; j < 4; j++) m(icol, j) *= pivinv;
        for (int j = 0; j < 4; j++) {
            if (j == icol) continue;
            const float save = m(j, icol);
            m(j, icol) = 0;
            for (int k = 0; k < 4; k++) m(j, k) -= m(icol, k) * save;
        }
    }
    for (int j = 3; j >= 0; j--)
        if (indxr[j] != indxc[j])
            for (int k = 0; k < 4; k++) std::swap(m(k, indxr[j]), m(k, indxc[j]));
    return true;
}
struct Xf {
    M44 m, inv;
};
Xf xfMul(const Xf &a, const Xf &b) { return Xf{mmul(a.m, b.m), mmul(b.inv, a.inv)}; }
Xf xfScale(float x, float y, float z) { /* transform.cpp:49-62 */
    return Xf{M44{x, 0, 0, 0, 0, y, 0, 0, 0, 0, z, 0, 0, 0, 0, 1},
              M44{1.0f / x, 0, 0, 0, 0, 1.0f / y, 0, 0, 0, 0, 1.0f / z, 0, 0, 0, 0, 1}};
}
Xf xfTranslate(float x, float y, float z) { /* transform.cpp:33-47 */
    return Xf{M44{1, 0, 0, x, 0, 1, 0, y, 0, 0, 1, z, 0, 0, 0, 1}, M44{1, 0, 0, -x, 0, 1, 0, -y, 0, 0, 1, -z, 0, 0, 0, 1}};
}
/* util.h:294-297 (M_PI is M_PI_FLT under SINGLE_PRECISION, constants.h:80) */
float degToRad(float v) { return v * (kPi / 180.0f); }
float radToDeg(float v) { return v * (180.0f / kPi); }
} // namespace

bool invertMatrix4(const float src[16], float out[16]) {
    M44 s, t;
    std::copy(src, src + 16, s.begin());
    if (!gaussJordanInvert(s, t)) return false;
    std::copy(t.begin(), t.end(), out);
    return true;
}

/* the horizontal field of view after PerspectiveCamera::configure (sensor.cpp:237-305) */
float cameraXFov(const SceneDesc &d) {
    const float aspect = (float) d.width / (float) d.height; /* sensor.cpp:101-102 */
    std::string axis = d.fovAxis;
    if (axis == "smaller") axis = aspect > 1 ? "y" : "x";
    else if (axis == "larger") axis = aspect > 1 ? "x" : "y";
    if (axis == "y") /* setYFov (:295-298) */
        return radToDeg(2 * std::atan(std::tan(0.5f * degToRad(d.fov)) * aspect));
    if (axis == "diagonal") { /* setDiagonalFov (:301-305) */
        const float diagonal = 2 * std::tan(0.5f * degToRad(d.fov));
        const float width = diagonal / std::sqrt(1.0f + 1.0f / (aspect * aspect));
        return radToDeg(2 * std::atan(width * 0.5f));
    }
    return d.fov;
}

bool cameraSampleToCamera(const SceneDesc &d, float s2c[16]) {
    const float aspect = (float) d.width / (float) d.height;
    const float xfov = cameraXFov(d);
    /* Transform::perspective (transform.cpp:99-119) and its Gauss-Jordan inverse */
    const float recip = 1.0f / (d.farClip - d.nearClip);
    const float cot = 1.0f / std::tan(degToRad(xfov / 2.0f));
    Xf P;
    P.m = M44{cot, 0, 0, 0, 0, cot, 0, 0, 0, 0, d.farClip * recip, -d.nearClip * d.farClip * recip, 0, 0, 1, 0};
    if (!gaussJordanInvert(P.m, P.inv)) return false;
    /* no crop window: relSize = 1, relOffset = 0 (perspective.cpp:133-138) */
    const float relSizeX = (float) d.width / (float) d.width, relSizeY = (float) d.height / (float) d.height;
    const float relOffX = 0.0f / (float) d.width, relOffY = 0.0f / (float) d.height;
    const Xf c2s = xfMul(xfMul(xfMul(xfMul(xfScale(1.0f / relSizeX, 1.0f / relSizeY, 1.0f),
                                           xfTranslate(-relOffX, -relOffY, 0.0f)),
                                     xfScale(-0.5f, -0.5f * aspect, 1.0f)),
                               xfTranslate(-1.0f, -1.0f / aspect, 0.0f)),
                         P);
    std::memcpy(s2c, c2s.inv.data(), 16 * sizeof(float));
    return true;
}

void setupCamera(const SceneDesc &d, HptCamera &cam) {
    /* PerspectiveCamera::setXFov (sensor.cpp:285-288) on the final horizontal field of view */
    const float xfov = cameraXFov(d);
    if (xfov <= 0 || xfov >= 180) throw std::runtime_error("The horizontal field of view must be in the interval (0, 180)!");
    if (!cameraSampleToCamera(d, cam.s2c))
        throw std::runtime_error("Unable to invert singular matrix (perspective camera)");
    std::memcpy(cam.toWorld, d.toWorld, sizeof(cam.toWorld));
    /* the origin of every camera ray: toWorld applied to (0, 0, 0) in the order the reference's
       Transform::operator()(Point) evaluates it (transform.h:108-121, fp32, no contraction) */
    for (int k = 0; k < 3; ++k) {
        const float *T = cam.toWorld + 4 * k;
        cam.origin[k] = T[0] * 0.0f + T[1] * 0.0f + T[2] * 0.0f + T[3];
    }
    cam.invResX = 1.0f / (float) d.width;
    cam.invResY = 1.0f / (float) d.height;
    /* position differentials on the near plane (perspective.cpp:160-163) */
    auto s2c = [&](float x, float y) {
        const float *M = cam.s2c;
        float px = M[0] * x + M[1] * y + M[2] * 0.0f + M[3], py = M[4] * x + M[5] * y + M[6] * 0.0f + M[7];
        float pz = M[8] * x + M[9] * y + M[10] * 0.0f + M[11], pw = M[12] * x + M[13] * y + M[14] * 0.0f + M[15];
        if (pw != 1.0f) {
            const float inv = 1.0f / pw;
            px *= inv, py *= inv, pz *= inv;
        }
        return std::array<float, 3>{px, py, pz};
    };
    const auto p0 = s2c(0.0f, 0.0f), px = s2c(cam.invResX, 0.0f), py = s2c(0.0f, cam.invResY);
    for (int k = 0; k < 3; ++k) {
        cam.dx[k] = px[k] - p0[k];
        cam.dy[k] = py[k] - p0[k];
    }
    /* sensorRay.scaleDifferential(1 / sqrt(sampleCount)) (integrator.cpp:143-144,178) */
    cam.diffScale = 1.0f / std::sqrt((float) std::max(1, d.spp));
    cam.nearClip = d.nearClip;
    cam.farClip = d.farClip;
    cam.width = d.width;
    cam.height = d.height;
    uint32_t r = (uint32_t) std::max(d.width, d.height);
    r--; r |= r >> 1; r |= r >> 2; r |= r >> 4; r |= r >> 8; r |= r >> 16; r++;
    cam.resolution = (float) r;
    uint32_t lg = 0;
    while ((r >> lg) != 0) lg++;
    cam.logRes = lg - 1;
}

void setupTent(float *lut, float &scale) {
    const int R = HPT_FILTER_RES;
    const float radius = 1.0f;
    float sum = 0.0f;
    for (int i = 0; i < R; ++i) {
        float x = (radius * i) / R;
        float v = std::max(0.0f, 1.0f - std::abs(x / radius));
        lut[i] = v;
        sum += v;
    }
    lut[R] = 0.0f;
    scale = R / radius;
    sum *= 2 * radius / R;
    float norm = 1.0f / sum;
    for (int i = 0; i < R; ++i) lut[i] *= norm;
}

} // namespace hpt
