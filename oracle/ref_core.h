/*
 * ref_core.h -- scalar math used by the oracle (CPU restatement of the
 * reference).  TEST INFRASTRUCTURE ONLY (see oracle.h).
 *
 * Every helper reproduces the single-precision semantics of the reference
 * (compiled with SINGLE_PRECISION, SPECTRUM_SAMPLES=3):
 *   - division by a scalar multiplies by the reciprocal
 *     (include/mitsuba/core/vector.h:546-564, point.h:515-522,
 *      spectrum.h:415-424)
 *   - math::clamp = std::min(max, std::max(min, v))   (core/math.h:50-52)
 *   - normalize(v) = v / v.length()                     (core/vector.h:191)
 *   - luminance = 0.212671 r + 0.715160 g + 0.072169 b  (core/spectrum.h:725)
 * Build with -ffp-contract=off so no multiply-add is fused.
 */
#ifndef HAIRPT_ORACLE_REF_CORE_H
#define HAIRPT_ORACLE_REF_CORE_H
#include <algorithm>
#include <cmath>
#include <cstdint>
#include <limits>

namespace orc {

/* include/mitsuba/core/constants.h:28-31,56-68 (SINGLE_PRECISION) */
static const float kEpsilon = 1e-4f;
static const float kShadowEpsilon = 1e-3f;
static const float kOneMinusEps = 0x1.fffffep-1f;
static const float kPi = 3.14159265358979323846f;
static const float kInvPi = 0.31830988618379067154f;
static const float kInvTwoPi = 0.15915494309189533577f;
static const float kInvFourPi = 0.07957747154594766788f;
static const float kInf = std::numeric_limits<float>::infinity();

template <typename T> inline T clampv(T v, T lo, T hi) { return std::min(hi, std::max(lo, v)); }
inline float degToRad(float v) { return v * (kPi / 180.0f); } /* util.h:297 */
inline float safe_sqrt(float v) { return std::sqrt(std::max(0.0f, v)); }
inline float safe_acos(float v) { return std::acos(std::min(1.0f, std::max(-1.0f, v))); }
inline int floorToInt(float v) { return (int) std::floor(v); }
inline int modulo(int a, int b) { int r = a % b; return (r < 0) ? r + b : r; }

struct V3 {
    float x, y, z;
    V3() : x(0), y(0), z(0) {}
    explicit V3(float v) : x(v), y(v), z(v) {}
    V3(float a, float b, float c) : x(a), y(b), z(c) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
    V3 operator+(const V3 &o) const { return V3(x + o.x, y + o.y, z + o.z); }
    V3 operator-(const V3 &o) const { return V3(x - o.x, y - o.y, z - o.z); }
    V3 operator-() const { return V3(-x, -y, -z); }
    V3 operator*(float f) const { return V3(x * f, y * f, z * f); }
    V3 operator/(float f) const { float r = 1.0f / f; return V3(x * r, y * r, z * r); }
    V3 &operator+=(const V3 &o) { x += o.x; y += o.y; z += o.z; return *this; }
    V3 &operator-=(const V3 &o) { x -= o.x; y -= o.y; z -= o.z; return *this; }
    V3 &operator*=(float f) { x *= f; y *= f; z *= f; return *this; }
    V3 &operator/=(float f) { float r = 1.0f / f; x *= r; y *= r; z *= r; return *this; }
    bool operator==(const V3 &o) const { return x == o.x && y == o.y && z == o.z; }
    bool operator!=(const V3 &o) const { return !(*this == o); }
    float lengthSquared() const { return x * x + y * y + z * z; }
    float length() const { return std::sqrt(lengthSquared()); }
    bool isZero() const { return x == 0 && y == 0 && z == 0; }
};
inline V3 operator*(float f, const V3 &v) { return v * f; }
inline float dot(const V3 &a, const V3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float absDot(const V3 &a, const V3 &b) { return std::abs(dot(a, b)); }
inline V3 cross(const V3 &v1, const V3 &v2) {
    /* core/vector.h cross(): (v1.y*v2.z - v1.z*v2.y, v1.z*v2.x - v1.x*v2.z, v1.x*v2.y - v1.y*v2.x) */
    return V3(v1.y * v2.z - v1.z * v2.y, v1.z * v2.x - v1.x * v2.z, v1.x * v2.y - v1.y * v2.x);
}
inline V3 normalize(const V3 &v) { return v / v.length(); }

struct V3d {
    double x, y, z;
    V3d() : x(0), y(0), z(0) {}
    V3d(double a, double b, double c) : x(a), y(b), z(c) {}
    explicit V3d(const V3 &v) : x(v.x), y(v.y), z(v.z) {}
    V3d operator+(const V3d &o) const { return V3d(x + o.x, y + o.y, z + o.z); }
    V3d operator-(const V3d &o) const { return V3d(x - o.x, y - o.y, z - o.z); }
    V3d operator*(double f) const { return V3d(x * f, y * f, z * f); }
    V3d operator/(double f) const { double r = 1.0 / f; return V3d(x * r, y * r, z * r); }
    double lengthSquared() const { return x * x + y * y + z * z; }
    double length() const { return std::sqrt(lengthSquared()); }
};
inline V3d operator*(double f, const V3d &v) { return v * f; }
inline double dot(const V3d &a, const V3d &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline V3d normalize(const V3d &v) { return v / v.length(); }

/* Spectrum (RGB, SPECTRUM_SAMPLES == 3) -- core/spectrum.h */
struct Spec {
    float s[3];
    Spec() { s[0] = s[1] = s[2] = 0.0f; }
    explicit Spec(float v) { s[0] = s[1] = s[2] = v; }
    Spec(float r, float g, float b) { s[0] = r; s[1] = g; s[2] = b; }
    Spec operator+(const Spec &o) const { return Spec(s[0] + o.s[0], s[1] + o.s[1], s[2] + o.s[2]); }
    Spec operator*(const Spec &o) const { return Spec(s[0] * o.s[0], s[1] * o.s[1], s[2] * o.s[2]); }
    Spec operator*(float f) const { return Spec(s[0] * f, s[1] * f, s[2] * f); }
    Spec operator/(float f) const { float r = 1.0f / f; return Spec(s[0] * r, s[1] * r, s[2] * r); }
    Spec operator-(const Spec &o) const { return Spec(s[0] - o.s[0], s[1] - o.s[1], s[2] - o.s[2]); }
    Spec &operator/=(const Spec &o) { for (int i = 0; i < 3; ++i) s[i] /= o.s[i]; return *this; } /* spectrum.h:170-175 */
    Spec &operator+=(const Spec &o) { for (int i = 0; i < 3; ++i) s[i] += o.s[i]; return *this; }
    Spec &operator*=(const Spec &o) { for (int i = 0; i < 3; ++i) s[i] *= o.s[i]; return *this; }
    Spec &operator*=(float f) { for (int i = 0; i < 3; ++i) s[i] *= f; return *this; }
    Spec &operator/=(float f) { float r = 1.0f / f; for (int i = 0; i < 3; ++i) s[i] *= r; return *this; }
    float max() const { return std::max(std::max(s[0], s[1]), s[2]); }
    bool isZero() const { return s[0] == 0.0f && s[1] == 0.0f && s[2] == 0.0f; }
    float getLuminance() const { return s[0] * 0.212671f + s[1] * 0.715160f + s[2] * 0.072169f; }
    float average() const { float r = 0.0f; for (int i = 0; i < 3; ++i) r += s[i]; return r * (1.0f / 3); } /* spectrum.h:481-486 */
};
inline Spec operator*(float f, const Spec &v) { return v * f; }

/* Frame -- core/frame.h:30-96 */
struct Frame {
    V3 s, t, n;
    Frame() {}
    V3 toLocal(const V3 &v) const { return V3(dot(v, s), dot(v, t), dot(v, n)); }
    V3 toWorld(const V3 &v) const { return s * v.x + t * v.y + n * v.z; }
};

/* util.cpp:592-601 */
inline void coordinateSystem(const V3 &a, V3 &b, V3 &c) {
    if (std::abs(a.x) > std::abs(a.y)) {
        float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = V3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = V3(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}
inline Frame frameFromNormal(const V3 &n) { Frame f; f.n = n; coordinateSystem(n, f.s, f.t); return f; }

/* util.cpp:603-608 */
inline void computeShadingFrame(const V3 &n, const V3 &dpdu, Frame &frame) {
    frame.n = n;
    frame.s = normalize(dpdu - frame.n * dot(frame.n, dpdu));
    frame.t = cross(frame.n, frame.s);
}

/* util.cpp:651-681 (+ util.h:479-480 two-argument wrapper) */
inline float fresnelDielectricExt(float cosThetaI_, float eta) {
    if (eta == 1)
        return 0.0f;
    float scale = (cosThetaI_ > 0) ? 1 / eta : eta,
          cosThetaTSqr = 1 - (1 - cosThetaI_ * cosThetaI_) * (scale * scale);
    if (cosThetaTSqr <= 0.0f)
        return 1.0f;
    float cosThetaI = std::abs(cosThetaI_);
    float cosThetaT = std::sqrt(cosThetaTSqr);
    float Rs = (cosThetaI - eta * cosThetaT) / (cosThetaI + eta * cosThetaT);
    float Rp = (eta * cosThetaI - cosThetaT) / (eta * cosThetaI + cosThetaT);
    return 0.5f * (Rs * Rs + Rp * Rp);
}

/* util.cpp:487-525 */
inline bool solveQuadraticDouble(double a, double b, double c, double &x0, double &x1) {
    if (a == 0) {
        if (b != 0) {
            x0 = x1 = -c / b;
            return true;
        }
        return false;
    }
    double discrim = b * b - 4.0f * a * c;
    if (discrim < 0)
        return false;
    double temp, sqrtDiscrim = std::sqrt(discrim);
    if (b < 0)
        temp = -0.5f * (b - sqrtDiscrim);
    else
        temp = -0.5f * (b + sqrtDiscrim);
    x0 = temp / a;
    x1 = c / temp;
    if (x0 > x1)
        std::swap(x0, x1);
    return true;
}

/* util.cpp solveQuadratic (float version, used by BSphere::rayIntersect) */
inline bool solveQuadratic(float a, float b, float c, float &x0, float &x1) {
    if (a == 0) {
        if (b != 0) {
            x0 = x1 = -c / b;
            return true;
        }
        return false;
    }
    float discrim = b * b - 4.0f * a * c;
    if (discrim < 0)
        return false;
    float temp, sqrtDiscrim = std::sqrt(discrim);
    if (b < 0)
        temp = -0.5f * (b - sqrtDiscrim);
    else
        temp = -0.5f * (b + sqrtDiscrim);
    x0 = temp / a;
    x1 = c / temp;
    if (x0 > x1)
        std::swap(x0, x1);
    return true;
}

/* warp.cpp:81-105 */
inline void squareToUniformDiskConcentric(float sx, float sy, float &ox, float &oy) {
    float r1 = 2.0f * sx - 1.0f;
    float r2 = 2.0f * sy - 1.0f;
    float phi, r;
    if (r1 == 0 && r2 == 0) {
        r = phi = 0;
    } else if (r1 * r1 > r2 * r2) {
        r = r1;
        phi = (kPi / 4.0f) * (r2 / r1);
    } else {
        r = r2;
        phi = (kPi / 2.0f) - (r1 / r2) * (kPi / 4.0f);
    }
    float sinPhi = std::sin(phi), cosPhi = std::cos(phi);
    ox = r * cosPhi;
    oy = r * sinPhi;
}

/* warp.cpp:43-52 */
inline V3 squareToCosineHemisphere(float sx, float sy) {
    float px, py;
    squareToUniformDiskConcentric(sx, sy, px, py);
    float z = safe_sqrt(1.0f - px * px - py * py);
    if (z == 0)
        z = 1e-10f;
    return V3(px, py, z);
}

/* warp.cpp:143-162 */
inline float intervalToTent(float sample) {
    float sign;
    if (sample < 0.5f) {
        sign = 1;
        sample *= 2;
    } else {
        sign = -1;
        sample = 2 * (sample - 0.5f);
    }
    return sign * (1 - std::sqrt(sample));
}

} // namespace orc
#endif
