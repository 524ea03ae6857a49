/*
 * hpt_math.h -- device-side scalar helpers for the gfx950 kernels.
 *
 * Single-precision semantics of the reference (SINGLE_PRECISION build):
 * division by a scalar multiplies by its reciprocal (core/vector.h:546-564,
 * spectrum.h:415-424), clamp = min(max(v, lo), hi) (core/math.h:50-52),
 * normalize(v) = v * (1/|v|).  Kernels are compiled with -ffp-contract=off
 * so that no multiply-add is fused and the host-precomputed tables, the
 * kd-tree decisions and the BSDF arithmetic round exactly like the reference.
 */
#ifndef HPT_MATH_H
#define HPT_MATH_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#define HD __device__ __forceinline__

namespace hk {

static constexpr float kEpsilon = 1e-4f;        /* constants.h:28 */
static constexpr float kShadowEpsilon = 1e-3f;  /* constants.h:29 */
static constexpr float kPi = 3.14159265358979323846f;
static constexpr float kInvPi = 0.31830988618379067154f;
static constexpr float kInvTwoPi = 0.15915494309189533577f;
static constexpr float kInvFourPi = 0.07957747154594766788f;
static constexpr float kOneMinusEps = 0x1.fffffep-1f;

HD float fminr(float a, float b) { return (b < a) ? b : a; } /* std::min semantics */
HD float fmaxr(float a, float b) { return (a < b) ? b : a; } /* std::max semantics */
HD int imin(int a, int b) { return (b < a) ? b : a; }
HD int imax(int a, int b) { return (a < b) ? b : a; }
HD float clampf(float v, float lo, float hi) { return fminr(hi, fmaxr(lo, v)); }
HD int clampi(int v, int lo, int hi) { return imin(hi, imax(lo, v)); }
HD float finf() { return __builtin_huge_valf(); }

struct V3 {
    float x, y, z;
    HD float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
};
HD V3 v3(float a, float b, float c) { V3 r; r.x = a; r.y = b; r.z = c; return r; }
HD V3 operator+(V3 a, V3 b) { return v3(a.x + b.x, a.y + b.y, a.z + b.z); }
HD V3 operator-(V3 a, V3 b) { return v3(a.x - b.x, a.y - b.y, a.z - b.z); }
HD V3 operator-(V3 a) { return v3(-a.x, -a.y, -a.z); }
HD V3 operator*(V3 a, float f) { return v3(a.x * f, a.y * f, a.z * f); }
HD V3 operator*(float f, V3 a) { return v3(a.x * f, a.y * f, a.z * f); }
HD V3 mul(V3 a, V3 b) { return v3(a.x * b.x, a.y * b.y, a.z * b.z); }
HD V3 divs(V3 a, float f) { float r = 1.0f / f; return v3(a.x * r, a.y * r, a.z * r); }
HD float dot(V3 a, V3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
HD float length(V3 a) { return sqrtf(a.x * a.x + a.y * a.y + a.z * a.z); }
HD V3 normalize(V3 a) { return divs(a, length(a)); }
HD V3 cross(V3 a, V3 b) {
    return v3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x);
}
HD bool isZero(V3 a) { return a.x == 0.0f && a.y == 0.0f && a.z == 0.0f; }
HD float maxc(V3 a) { return fmaxr(fmaxr(a.x, a.y), a.z); }
HD float lum(V3 a) { return a.x * 0.212671f + a.y * 0.715160f + a.z * 0.072169f; }

struct D3 {
    double x, y, z;
};
HD D3 d3(double a, double b, double c) { D3 r; r.x = a; r.y = b; r.z = c; return r; }
HD D3 operator+(D3 a, D3 b) { return d3(a.x + b.x, a.y + b.y, a.z + b.z); }
HD D3 operator-(D3 a, D3 b) { return d3(a.x - b.x, a.y - b.y, a.z - b.z); }
HD D3 operator*(D3 a, double f) { return d3(a.x * f, a.y * f, a.z * f); }
HD double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct Frame {
    V3 s, t, n;
    HD V3 toLocal(V3 v) const { return v3(dot(v, s), dot(v, t), dot(v, n)); }
    HD V3 toWorld(V3 v) const { return s * v.x + t * v.y + n * v.z; }
};

/* util.cpp:592-601 */
HD void coordinateSystem(V3 a, V3 &b, V3 &c) {
    if (fabsf(a.x) > fabsf(a.y)) {
        float invLen = 1.0f / sqrtf(a.x * a.x + a.z * a.z);
        c = v3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / sqrtf(a.y * a.y + a.z * a.z);
        c = v3(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}

/* util.cpp:487-525 */
HD bool solveQuadraticDouble(double a, double b, double c, double &x0, double &x1) {
    if (a == 0) {
        if (b != 0) {
            x0 = x1 = -c / b;
            return true;
        }
        return false;
    }
    double discrim = b * b - 4.0 * a * c;
    if (discrim < 0) return false;
    double temp, sq = sqrt(discrim);
    if (b < 0) temp = -0.5 * (b - sq);
    else temp = -0.5 * (b + sq);
    x0 = temp / a;
    x1 = c / temp;
    if (x0 > x1) {
        double t = x0;
        x0 = x1;
        x1 = t;
    }
    return true;
}

/* util.cpp solveQuadratic (single precision) */
HD bool solveQuadratic(float a, float b, float c, float &x0, float &x1) {
    if (a == 0) {
        if (b != 0) {
            x0 = x1 = -c / b;
            return true;
        }
        return false;
    }
    float discrim = b * b - 4.0f * a * c;
    if (discrim < 0) return false;
    float temp, sq = sqrtf(discrim);
    if (b < 0) temp = -0.5f * (b - sq);
    else temp = -0.5f * (b + sq);
    x0 = temp / a;
    x1 = c / temp;
    if (x0 > x1) {
        float t = x0;
        x0 = x1;
        x1 = t;
    }
    return true;
}

/* util.cpp:651-681 + util.h:479 */
HD float fresnelDielectricExt(float cosThetaI_, float eta) {
    if (eta == 1) return 0.0f;
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta;
    float cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) return 1.0f;
    float cI = fabsf(cosThetaI_), cT = sqrtf(cosThetaTSqr);
    float Rs = (cI - eta * cT) / (cI + eta * cT);
    float Rp = (eta * cI - cT) / (eta * cI + cT);
    return 0.5f * (Rs * Rs + Rp * Rp);
}

/* warp.cpp:81-105 concentric disk + warp.cpp:43-52 cosine hemisphere */
HD V3 squareToCosineHemisphere(float sx, float sy) {
    float r1 = 2.0f * sx - 1.0f, r2 = 2.0f * sy - 1.0f, phi, r;
    if (r1 == 0 && r2 == 0) {
        r = phi = 0;
    } else if (r1 * r1 > r2 * r2) {
        r = r1;
        phi = (kPi / 4.0f) * (r2 / r1);
    } else {
        r = r2;
        phi = (kPi / 2.0f) - (r1 / r2) * (kPi / 4.0f);
    }
    float px = r * cosf(phi), py = r * sinf(phi);
    float z = sqrtf(fmaxr(0.0f, 1.0f - px * px - py * py));
    if (z == 0) z = 1e-10f;
    return v3(px, py, z);
}

/* warp.cpp:143-156 */
HD float intervalToTent(float sample) {
    float sign;
    if (sample < 0.5f) {
        sign = 1;
        sample *= 2;
    } else {
        sign = -1;
        sample = 2 * (sample - 0.5f);
    }
    return sign * (1 - sqrtf(sample));
}

} // namespace hk
#endif
