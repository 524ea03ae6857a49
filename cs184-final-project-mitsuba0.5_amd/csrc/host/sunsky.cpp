/*
 * sunsky.cpp -- the `sunsky` emitter's rasterisation to a lat-long bitmap
 * (src/emitters/sunsky.cpp:100-240), which the reference then hands to a
 * nested `envmap` (envmap.cpp) -- exactly what buildEnvMap consumes here.
 *
 *   sky  : SkyEmitter::getSkyRadiance (src/emitters/sky.cpp:405-433) over the
 *          Hosek-Wilkie RGB model (src/emitters/sunsky/skymodel.cpp:80-397,
 *          coefficients extracted to data/sunsky/hosek_rgb.f64)
 *   sun  : computeSunRadiance (sunsky/sunmodel.h:316-371, Preetham's
 *          attenuation of the solar spectrum) converted to RGB like
 *          Spectrum::fromContinuousSpectrum (src/libcore/spectrum.cpp:172-191:
 *          CIE 1931 matching functions averaged with the adaptive
 *          Gauss-Lobatto rule of src/libcore/quad.cpp:287-415), splatted with
 *          (0,2)-sequence cone samples (sunsky.cpp:165-225)
 *   position: computeSunCoordinates (sunmodel.h:99-244) -- sunDirection or
 *          date/time/location.
 *
 * Arithmetic follows the reference's SINGLE_PRECISION types expression by
 * expression (float where the reference has Float, double where it promotes
 * through double literals or variables; M_PI itself is the float M_PI_FLT
 * under SINGLE_PRECISION, include/mitsuba/core/constants.h:79-80).
 */
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>
#include <limits>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"

namespace hpt {
namespace {

struct Vf {
    float x, y, z;
};
inline Vf operator+(Vf a, Vf b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline Vf operator*(Vf a, float f) { return {a.x * f, a.y * f, a.z * f}; }
inline Vf cross(Vf a, Vf b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }

inline float safeAcos(float v) { return std::acos(std::min(1.0f, std::max(-1.0f, v))); }
inline float safeSqrt(float v) { return std::sqrt(std::max(0.0f, v)); }
/* M_PI is M_PI_FLT under SINGLE_PRECISION (constants.h:80): every M_PI below is this float; an
   expression mixing it with a double literal or variable promotes only from there on */
const float kPiF = 3.14159265358979323846f;
inline float degToRad(float v) { return v * (kPiF / 180.0f); } /* util.h:297 */

struct Sph { /* SphericalCoordinates (sunmodel.h:64-88) */
    float elevation, azimuth;
};

Vf toSphere(Sph c) { /* sunmodel.h:90-97 */
    float sinTheta = std::sin(c.elevation), cosTheta = std::cos(c.elevation);
    float sinPhi = std::sin(c.azimuth), cosPhi = std::cos(c.azimuth);
    return {sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta};
}

Sph fromSphere(Vf d) { /* sunmodel.h:99-105 */
    float azimuth = std::atan2(d.x, -d.z);
    float elevation = safeAcos(d.y);
    if (azimuth < 0) azimuth += 2 * kPiF;
    return {elevation, azimuth};
}

void coordinateSystem(Vf a, Vf &b, Vf &c) { /* util.cpp:592-601 */
    if (std::abs(a.x) > std::abs(a.y)) {
        float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = {a.z * invLen, 0.0f, -a.x * invLen};
    } else {
        float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = {0.0f, a.z * invLen, -a.y * invLen};
    }
    b = cross(c, a);
}

/* computeSunCoordinates(dateTime, location) (sunmodel.h:115-204), in double */
Sph sunFromDateTime(int year, int month, int day, float hour, float minute, float second, float latitude,
                    float longitude, float timezone) {
    double decHours = hour - timezone + (minute + second / 60.0) / 60.0;
    int liAux1 = (month - 14) / 12;
    int liAux2 = (1461 * (year + 4800 + liAux1)) / 4 + (367 * (month - 2 - 12 * liAux1)) / 12 -
                 (3 * ((year + 4900 + liAux1) / 100)) / 4 + day - 32075;
    double dJulianDate = (double) liAux2 - 0.5 + decHours / 24.0;
    double elapsedJulianDays = dJulianDate - 2451545.0;

    double omega = 2.1429 - 0.0010394594 * elapsedJulianDays;
    double meanLongitude = 4.8950630 + 0.017202791698 * elapsedJulianDays;
    double anomaly = 6.2400600 + 0.0172019699 * elapsedJulianDays;
    double eclipticLongitude = meanLongitude + 0.03341607 * std::sin(anomaly) + 0.00034894 * std::sin(2 * anomaly) -
                               0.0001134 - 0.0000203 * std::sin(omega);
    double eclipticObliquity = 0.4090928 - 6.2140e-9 * elapsedJulianDays + 0.0000396 * std::cos(omega);

    double sinEclipticLongitude = std::sin(eclipticLongitude);
    double dY = std::cos(eclipticObliquity) * sinEclipticLongitude;
    double dX = std::cos(eclipticLongitude);
    double rightAscension = std::atan2(dY, dX);
    if (rightAscension < 0.0) rightAscension += (double) (2 * kPiF);
    double declination = std::asin(std::sin(eclipticObliquity) * sinEclipticLongitude);

    double greenwichMeanSiderealTime = 6.6974243242 + 0.0657098283 * elapsedJulianDays + decHours;
    double localMeanSiderealTime = degToRad((float) ((greenwichMeanSiderealTime * 15 + longitude)));
    double latitudeInRadians = degToRad(latitude);
    double cosLatitude = std::cos(latitudeInRadians);
    double sinLatitude = std::sin(latitudeInRadians);
    double hourAngle = localMeanSiderealTime - rightAscension;
    double cosHourAngle = std::cos(hourAngle);
    double elevation =
        std::acos(cosLatitude * cosHourAngle * std::cos(declination) + std::sin(declination) * sinLatitude);
    dY = -std::sin(hourAngle);
    dX = std::tan(declination) * cosLatitude - sinLatitude * cosHourAngle;
    double azimuth = std::atan2(dY, dX);
    if (azimuth < 0.0) azimuth += (double) (2 * kPiF);
    elevation += (6371.01 / 149597890) * std::sin(elevation); /* parallax */
    return {(float) elevation, (float) azimuth};
}

/* computeSunCoordinates(props) (sunmodel.h:206-244) */
Sph sunCoordinates(const SceneDesc &d, const float worldToLuminaire[9]) {
    if (d.sunDirectionGiven) {
        const float *m = worldToLuminaire;
        const float *v = d.sunDirection;
        Vf w = {m[0] * v[0] + m[1] * v[1] + m[2] * v[2], m[3] * v[0] + m[4] * v[1] + m[5] * v[2],
                m[6] * v[0] + m[7] * v[1] + m[8] * v[2]};
        float len = std::sqrt(w.x * w.x + w.y * w.y + w.z * w.z);
        float inv = 1.0f / len; /* TVector operator/(T): reciprocal multiply */
        return fromSphere(w * inv);
    }
    return sunFromDateTime(d.sunYear, d.sunMonth, d.sunDay, d.sunHour, d.sunMinute, d.sunSecond, d.sunLatitude,
                           d.sunLongitude, d.sunTimezone);
}

/* ---- Hosek-Wilkie RGB sky (skymodel.cpp:80-397) ---- */
typedef double HosekConfig[9];

void cookConfiguration(const double *dataset, HosekConfig config, double turbidity, double albedo,
                       double solarElevation) {
    int intTurbidity = (int) turbidity;
    double turbidityRem = turbidity - (double) intTurbidity;
    solarElevation = std::pow(solarElevation / ((double) kPiF / 2.0), (1.0 / 3.0));
    auto blend = [&](const double *em, int i) {
        return std::pow(1.0 - solarElevation, 5.0) * em[i] +
               5.0 * std::pow(1.0 - solarElevation, 4.0) * solarElevation * em[i + 9] +
               10.0 * std::pow(1.0 - solarElevation, 3.0) * std::pow(solarElevation, 2.0) * em[i + 18] +
               10.0 * std::pow(1.0 - solarElevation, 2.0) * std::pow(solarElevation, 3.0) * em[i + 27] +
               5.0 * (1.0 - solarElevation) * std::pow(solarElevation, 4.0) * em[i + 36] +
               std::pow(solarElevation, 5.0) * em[i + 45];
    };
    const double *em = dataset + (9 * 6 * (intTurbidity - 1));
    for (int i = 0; i < 9; ++i) config[i] = (1.0 - albedo) * (1.0 - turbidityRem) * blend(em, i);
    em = dataset + (9 * 6 * 10 + 9 * 6 * (intTurbidity - 1));
    for (int i = 0; i < 9; ++i) config[i] += (albedo) * (1.0 - turbidityRem) * blend(em, i);
    if (intTurbidity == 10) return;
    em = dataset + (9 * 6 * (intTurbidity));
    for (int i = 0; i < 9; ++i) config[i] += (1.0 - albedo) * (turbidityRem) * blend(em, i);
    em = dataset + (9 * 6 * 10 + 9 * 6 * (intTurbidity));
    for (int i = 0; i < 9; ++i) config[i] += (albedo) * (turbidityRem) * blend(em, i);
}

double cookRadiance(const double *dataset, double turbidity, double albedo, double solarElevation) {
    int intTurbidity = (int) turbidity;
    double turbidityRem = turbidity - (double) intTurbidity;
    solarElevation = std::pow(solarElevation / ((double) kPiF / 2.0), (1.0 / 3.0));
    auto blend = [&](const double *em) {
        return std::pow(1.0 - solarElevation, 5.0) * em[0] +
               5.0 * std::pow(1.0 - solarElevation, 4.0) * solarElevation * em[1] +
               10.0 * std::pow(1.0 - solarElevation, 3.0) * std::pow(solarElevation, 2.0) * em[2] +
               10.0 * std::pow(1.0 - solarElevation, 2.0) * std::pow(solarElevation, 3.0) * em[3] +
               5.0 * (1.0 - solarElevation) * std::pow(solarElevation, 4.0) * em[4] +
               std::pow(solarElevation, 5.0) * em[5];
    };
    double res = (1.0 - albedo) * (1.0 - turbidityRem) * blend(dataset + (6 * (intTurbidity - 1)));
    res += (albedo) * (1.0 - turbidityRem) * blend(dataset + (6 * 10 + 6 * (intTurbidity - 1)));
    if (intTurbidity == 10) return res;
    res += (1.0 - albedo) * (turbidityRem) * blend(dataset + (6 * (intTurbidity)));
    res += (albedo) * (turbidityRem) * blend(dataset + (6 * 10 + 6 * (intTurbidity)));
    return res;
}

double radianceInternal(const HosekConfig c, double theta, double gamma) {
    const double expM = std::exp(c[4] * gamma);
    const double rayM = std::cos(gamma) * std::cos(gamma);
    const double mieM = (1.0 + std::cos(gamma) * std::cos(gamma)) /
                        std::pow((1.0 + c[8] * c[8] - 2.0 * c[8] * std::cos(gamma)), 1.5);
    const double zenith = std::sqrt(std::cos(theta));
    return (1.0 + c[0] * std::exp(c[1] / (std::cos(theta) + 0.01))) *
           (c[2] + c[3] * expM + c[5] * rayM + c[6] * mieM + c[7] * zenith);
}

struct SkyModel {
    HosekConfig configs[3];
    double radiances[3];
    Sph sun;
    float scale, stretch;

    /* sky.cpp:222-252 + arhosek_rgb_skymodelstate_alloc_init (skymodel.cpp:346-373);
       Mitsuba allocates one RGB state per spectrum channel with that channel's
       albedo and reads channel i of state i */
    void init(const SunSkyTables &t, double turbidity, const float albedo[3], float sunElevation) {
        for (int ch = 0; ch < 3; ++ch) {
            cookConfiguration(t.hosek.data() + 1080 * ch, configs[ch], turbidity, albedo[ch], sunElevation);
            radiances[ch] = cookRadiance(t.hosek.data() + 3 * 1080 + 120 * ch, turbidity, albedo[ch], sunElevation);
        }
    }

    /* SkyEmitter::getSkyRadiance (sky.cpp:405-433), extend = false */
    void radiance(Sph coords, float out[3]) const {
        float theta = coords.elevation / stretch;
        if (std::cos(theta) <= 0) {
            out[0] = out[1] = out[2] = 0.0f;
            return;
        }
        float cosGamma = std::cos(theta) * std::cos(sun.elevation) +
                         std::sin(theta) * std::sin(sun.elevation) * std::cos(coords.azimuth - sun.azimuth);
        float gamma = safeAcos(cosGamma);
        for (int i = 0; i < 3; ++i) {
            float v = (float) (radianceInternal(configs[i], theta, gamma) * radiances[i] / 106.856980);
            out[i] = std::max(v, 0.0f) * scale; /* clampNegative, then * m_scale */
        }
    }
};

/* ---- spectra (spectrum.cpp) ---- */
struct InterpSpectrum { /* InterpolatedSpectrum (spectrum.cpp:604-720) */
    std::vector<float> wl, val;
    float eval(float lambda) const {
        if (wl.size() < 2 || lambda < wl[0] || lambda > wl.back()) return 0.0f;
        auto r = std::equal_range(wl.begin(), wl.end(), lambda);
        size_t i1 = (size_t) (r.first - wl.begin()), i2 = (size_t) (r.second - wl.begin());
        if (i1 == i2) {
            float a = wl[i1 - 1], b = wl[i1], fa = val[i1 - 1], fb = val[i1];
            float t = (lambda - a) / (b - a);
            return (1.0f - t) * fa + t * fb; /* math::lerp */
        }
        return val[i1];
    }
    float average(float lambdaMin, float lambdaMax) const { /* :650-686 */
        if (wl.size() < 2) return 0.0f;
        float rangeStart = std::max(lambdaMin, wl[0]), rangeEnd = std::min(lambdaMax, wl.back());
        if (rangeEnd <= rangeStart) return 0.0f;
        size_t entry = std::max((size_t) (std::lower_bound(wl.begin(), wl.end(), rangeStart) - wl.begin()),
                                (size_t) 1) - 1;
        float result = 0.0f;
        for (; entry + 1 < wl.size() && rangeEnd >= wl[entry]; ++entry) {
            float a = wl[entry], b = wl[entry + 1], ca = std::max(a, rangeStart), cb = std::min(b, rangeEnd),
                  fa = val[entry], fb = val[entry + 1], invAB = 1.0f / (b - a);
            if (cb <= ca) continue;
            float ta = (ca - a) * invAB, tb = (cb - a) * invAB;
            float interpA = (1.0f - ta) * fa + ta * fb, interpB = (1.0f - tb) * fa + tb * fb;
            result += 0.5f * (interpA + interpB) * (cb - ca);
        }
        return result / (lambdaMax - lambdaMin);
    }
};

/* GaussLobattoIntegrator (quad.cpp:287-415) with useConvergenceEstimate = false */
struct GaussLobatto {
    const float alpha = (float) std::sqrt(2.0 / 3.0), beta = (float) (1.0 / std::sqrt(5.0));
    const float x1 = (float) 0.94288241569547971906, x2 = (float) 0.64185334234578130578,
                x3 = (float) 0.23638319966214988028;
    float absError, relError;
    size_t maxEvals;
    /* an explicit constructor: brace-initialising this struct would assign the
       error bounds to alpha / beta (the first members) -- which round 1 did,
       and the sun came out 2-3 % off per channel */
    GaussLobatto(float absErr, float relErr, size_t evals) : absError(absErr), relError(relErr), maxEvals(evals) {}

    float integrate(const std::function<float(float)> &f, float a, float b) const {
        float factor = 1;
        size_t evals = 0;
        if (a == b) return 0;
        if (b < a) {
            std::swap(a, b);
            factor = -1;
        }
        const float absTol = absTolerance(f, a, b, evals);
        evals += 2;
        return factor * step(f, a, b, f(a), f(b), absTol, evals);
    }

    float absTolerance(const std::function<float(float)> &f, float a, float b, size_t &evals) const {
        const float m = (a + b) / 2, h = (b - a) / 2;
        const float y1 = f(a), y3 = f(m - alpha * h), y5 = f(m - beta * h), y7 = f(m), y9 = f(m + beta * h),
                    y11 = f(m + alpha * h), y13 = f(b);
        float acc = h * ((float) 0.0158271919734801831 * (y1 + y13) +
                         (float) 0.0942738402188500455 * (f(m - x1 * h) + f(m + x1 * h)) +
                         (float) 0.1550719873365853963 * (y3 + y11) +
                         (float) 0.1888215739601824544 * (f(m - x2 * h) + f(m + x2 * h)) +
                         (float) 0.1997734052268585268 * (y5 + y9) +
                         (float) 0.2249264653333395270 * (f(m - x3 * h) + f(m + x3 * h)) +
                         (float) 0.2426110719014077338 * y7);
        evals += 13;
        const float r = 1.0f, eps = std::numeric_limits<float>::epsilon();
        float result = std::numeric_limits<float>::infinity();
        if (relError != 0 && acc != 0) result = acc * std::max(relError, eps) / (r * eps);
        if (absError != 0) result = std::min(result, absError / (r * eps));
        return result;
    }

    float step(const std::function<float(float)> &f, float a, float b, float fa, float fb, float acc,
               size_t &evals) const {
        const float h = (b - a) / 2, m = (a + b) / 2;
        const float mll = m - alpha * h, ml = m - beta * h, mr = m + beta * h, mrr = m + alpha * h;
        const float fmll = f(mll), fml = f(ml), fm = f(m), fmr = f(mr), fmrr = f(mrr);
        const float integral2 = (h / 6) * (fa + fb + 5 * (fml + fmr));
        const float integral1 = (h / 1470) * (77 * (fa + fb) + 432 * (fmll + fmrr) + 625 * (fml + fmr) + 672 * fm);
        evals += 5;
        if (evals >= maxEvals) return integral1;
        volatile float dist = acc + (integral1 - integral2); /* the (dist == acc) test must round */
        if (dist == acc || mll <= a || b <= mrr) return integral1;
        return step(f, a, mll, fa, fmll, acc, evals) + step(f, mll, ml, fmll, fml, acc, evals) +
               step(f, ml, m, fml, fm, acc, evals) + step(f, m, mr, fm, fmr, acc, evals) +
               step(f, mr, mrr, fmr, fmrr, acc, evals) + step(f, mrr, b, fmrr, fb, acc, evals);
    }
};

/* ContinuousSpectrum::average (spectrum.cpp:546-568) */
float averageContinuous(const std::function<float(float)> &f, float lambdaMin, float lambdaMax) {
    const GaussLobatto gl(1e-4f, 1e-4f, 10000); /* Epsilon, SINGLE_PRECISION */
    if (lambdaMax <= lambdaMin) return 0.0f;
    float integral = 0;
    size_t nSteps = std::max((size_t) 1, (size_t) std::ceil((lambdaMax - lambdaMin) / 50));
    float stepSize = (lambdaMax - lambdaMin) / nSteps, pos = lambdaMin;
    for (size_t i = 0; i < nSteps; ++i) {
        integral += gl.integrate(f, pos, pos + stepSize);
        pos += stepSize;
    }
    return integral / (lambdaMax - lambdaMin);
}

/* Spectrum::fromContinuousSpectrum, RGB mode (spectrum.cpp:172-184) + fromXYZ (:222-227) */
void continuousToRGB(const SunSkyTables &t, const InterpSpectrum &smooth, float rgb[3]) {
    InterpSpectrum cx, cy, cz;
    const size_t n = 471;
    cx.wl.assign(t.cie.begin(), t.cie.begin() + n);
    cy.wl = cz.wl = cx.wl;
    cx.val.assign(t.cie.begin() + n, t.cie.begin() + 2 * n);
    cy.val.assign(t.cie.begin() + 2 * n, t.cie.begin() + 3 * n);
    cz.val.assign(t.cie.begin() + 3 * n, t.cie.begin() + 4 * n);
    const float start = cx.wl[0], end = cx.wl[n - 1];
    float X = averageContinuous([&](float l) { return smooth.eval(l) * cx.eval(l); }, start, end);
    float Y = averageContinuous([&](float l) { return smooth.eval(l) * cy.eval(l); }, start, end);
    float Z = averageContinuous([&](float l) { return smooth.eval(l) * cz.eval(l); }, start, end);
    float normalization = 1.0f / cy.average(start, end);
    X *= normalization;
    Y *= normalization;
    Z *= normalization;
    rgb[0] = 3.240479f * X + -1.537150f * Y + -0.498535f * Z;
    rgb[1] = -0.969256f * X + 1.875991f * Y + 0.041556f * Z;
    rgb[2] = 0.055648f * X + -0.204043f * Y + 1.057311f * Z;
}

inline float fastexp(float v) { return (float) std::exp((double) v); } /* math.h:185-187 (Linux x86_64) */

/* computeSunRadiance (sunmodel.h:316-371) */
void sunRadiance(const SunSkyTables &t, float theta, float turbidity, float rgb[3]) {
    InterpSpectrum kO{t.kOWl, t.kOAmp}, kG{t.kGWl, t.kGAmp}, kWa{t.kWaWl, t.kWaAmp}, sol{t.solWl, t.solAmp};
    InterpSpectrum spec;
    spec.wl.resize(91);
    spec.val.resize(91);
    float beta = 0.04608365822050f * turbidity - 0.04586025928522f;
    float m = (float) (1.0f / (std::cos(theta) + 0.15f * std::pow(93.885f - theta / kPiF * 180.0f, (float) -1.253f)));
    float lambda;
    int i;
    for (i = 0, lambda = 350; i < 91; i++, lambda += 5) {
        float tauR = fastexp(-m * 0.008735f * std::pow(lambda / 1000.0f, (float) -4.08));
        const float alpha = 1.3f;
        float tauA = fastexp(-m * beta * std::pow(lambda / 1000.0f, -alpha));
        const float lOzone = .35f;
        float tauO = fastexp(-m * kO.eval(lambda) * lOzone);
        float tauG = fastexp(-1.41f * kG.eval(lambda) * m / std::pow(1 + 118.93f * kG.eval(lambda) * m, (float) 0.45f));
        const float w = 2.0;
        float tauWA = fastexp(-0.2385f * kWa.eval(lambda) * w * m /
                              std::pow(1 + 20.07f * kWa.eval(lambda) * w * m, (float) 0.45f));
        spec.val[i] = sol.eval(lambda) * tauR * tauA * tauO * tauG * tauWA;
        spec.wl[i] = lambda;
    }
    continuousToRGB(t, spec, rgb);
    for (int c = 0; c < 3; ++c) rgb[c] = std::max(rgb[c], 0.0f); /* clampNegative */
}

/* sample02 (qmc.h:115-126, SINGLE_PRECISION) */
inline float radicalInverse2(uint32_t n) {
    n = __builtin_bswap32(n);
    n = ((n & 0x0f0f0f0f) << 4) | ((n & 0xf0f0f0f0) >> 4);
    n = ((n & 0x33333333) << 2) | ((n & 0xcccccccc) >> 2);
    n = ((n & 0x55555555) << 1) | ((n & 0xaaaaaaaa) >> 1);
    n = (n >> (32 - 24));
    return (float) n / (float) (1U << 24);
}
inline float sobol2(uint32_t n) {
    uint32_t scramble = 0;
    for (uint32_t v = 1U << 31; n != 0; n >>= 1, v ^= v >> 1)
        if (n & 1) scramble ^= v;
    return (float) scramble / (float) (1ULL << 32);
}

/* warp::squareToUniformCone (warp.cpp:54-63) */
Vf squareToUniformCone(float cosCutoff, float sx, float sy) {
    float cosTheta = (1 - sx) + sx * cosCutoff;
    float sinTheta = safeSqrt(1.0f - cosTheta * cosTheta);
    float phi = 2.0f * kPiF * sy;
    float sinPhi = std::sin(phi), cosPhi = std::cos(phi);
    return {cosPhi * sinTheta, sinPhi * sinTheta, cosTheta};
}

void invert3(const float m[16], float out[9]) { /* rotation / scale part of toWorld, inverted */
    double a[9] = {m[0], m[1], m[2], m[4], m[5], m[6], m[8], m[9], m[10]};
    double det = a[0] * (a[4] * a[8] - a[5] * a[7]) - a[1] * (a[3] * a[8] - a[5] * a[6]) +
                 a[2] * (a[3] * a[7] - a[4] * a[6]);
    double inv[9] = {(a[4] * a[8] - a[5] * a[7]) / det, (a[2] * a[7] - a[1] * a[8]) / det,
                     (a[1] * a[5] - a[2] * a[4]) / det, (a[5] * a[6] - a[3] * a[8]) / det,
                     (a[0] * a[8] - a[2] * a[6]) / det, (a[2] * a[3] - a[0] * a[5]) / det,
                     (a[3] * a[7] - a[4] * a[6]) / det, (a[1] * a[6] - a[0] * a[7]) / det,
                     (a[0] * a[4] - a[1] * a[3]) / det};
    for (int i = 0; i < 9; ++i) out[i] = (float) inv[i];
}

bool isIdentity(const float m[16]) {
    for (int i = 0; i < 16; ++i)
        if (m[i] != ((i % 5 == 0) ? 1.0f : 0.0f)) return false;
    return true;
}

} // namespace

bool loadSunSkyTables(const std::string &dataDir, SunSkyTables &t, std::string &err) {
    auto readBin = [&](const std::string &f, size_t bytes, void *dst) {
        std::ifstream in(dataDir + "/sunsky/" + f, std::ios::binary);
        if (!in) return false;
        in.read((char *) dst, (std::streamsize) bytes);
        return (bool) in && (size_t) in.gcount() == bytes;
    };
    t.hosek.resize(3 * 1080 + 3 * 120);
    t.cie.resize(4 * 471);
    if (!readBin("hosek_rgb.f64", t.hosek.size() * 8, t.hosek.data()) ||
        !readBin("cie1931.f32", t.cie.size() * 4, t.cie.data())) {
        err = "cannot read sunsky tables from " + dataDir + "/sunsky";
        return false;
    }
    std::ifstream js(dataDir + "/sunsky/sun_tables.json");
    if (!js) {
        err = "cannot read " + dataDir + "/sunsky/sun_tables.json";
        return false;
    }
    std::stringstream ss;
    ss << js.rdbuf();
    const std::string s = ss.str();
    auto arr = [&](const char *name, std::vector<float> &out) {
        size_t k = s.find(std::string("\"") + name + "\"");
        if (k == std::string::npos) return false;
        size_t a = s.find('[', k), b = s.find(']', a);
        std::stringstream vs(s.substr(a + 1, b - a - 1));
        std::string tok;
        out.clear();
        while (std::getline(vs, tok, ',')) out.push_back(std::stof(tok));
        return !out.empty();
    };
    if (!arr("k_oWavelengths", t.kOWl) || !arr("k_oAmplitudes", t.kOAmp) || !arr("k_gWavelengths", t.kGWl) ||
        !arr("k_gAmplitudes", t.kGAmp) || !arr("k_waWavelengths", t.kWaWl) || !arr("k_waAmplitudes", t.kWaAmp) ||
        !arr("solWavelengths", t.solWl) || !arr("solAmplitudes", t.solAmp)) {
        err = "malformed sun_tables.json";
        return false;
    }
    t.kOAmp.resize(t.kOWl.size()); /* InterpolatedSpectrum(k_o, 64) */
    return true;
}

void hosekSkyRGB(const SunSkyTables &t, double turbidity, double albedo, double solarElevation, double theta,
                 double gamma, double out[3]) {
    for (int ch = 0; ch < 3; ++ch) {
        HosekConfig c;
        cookConfiguration(t.hosek.data() + 1080 * ch, c, turbidity, albedo, solarElevation);
        out[ch] = radianceInternal(c, theta, gamma) *
                  cookRadiance(t.hosek.data() + 3 * 1080 + 120 * ch, turbidity, albedo, solarElevation);
    }
}

void sunRadianceRGB(const SunSkyTables &t, float theta, float turbidity, float rgb[3]) {
    sunRadiance(t, theta, turbidity, rgb);
}

void rasterizeSunSky(const SceneDesc &d, const SunSkyTables &t, EnvHost &env) {
    if (d.turbidity < 1 || d.turbidity > 10)
        throw std::runtime_error("The turbidity parameter must be in the range [1,10]!");
    if (d.skyStretch < 1 || d.skyStretch > 2) throw std::runtime_error("The stretch parameter must be in the range [1,2]!");
    for (int i = 0; i < 3; ++i)
        if (d.skyAlbedo[i] < 0 || d.skyAlbedo[i] > 1)
            throw std::runtime_error("The albedo parameter must be in the range [0,1]!");
    const int W = d.skyResolution, H = d.skyResolution / 2;
    env.w = W;
    env.h = H;
    env.rgb.assign((size_t) W * H * 3, 0.0f);

    float worldToLum[9];
    if (isIdentity(d.emitterToWorld)) {
        for (int i = 0; i < 9; ++i) worldToLum[i] = (i % 4 == 0) ? 1.0f : 0.0f;
    } else {
        invert3(d.emitterToWorld, worldToLum);
    }

    /* the nested sky (sunsky.cpp:110-118): sunDirection pre-transformed by
       toWorld^-1, toWorld removed -- i.e. the same sun coordinates */
    SkyModel sky;
    sky.sun = sunCoordinates(d, worldToLum);
    sky.scale = d.skyScale;
    sky.stretch = d.skyStretch;
    const float sunElevation = 0.5f * kPiF - sky.sun.elevation;
    if (sunElevation < 0)
        throw std::runtime_error("The sun is below the horizon -- this is not supported by the sky model.");
    sky.init(t, d.turbidity, d.skyAlbedo, sunElevation);

    /* rasterise the sky (sunsky.cpp:131-145) */
    const float fx = (2 * kPiF) / W, fy = kPiF / H;
    for (int y = 0; y < H; ++y) {
        const float theta = (y + .5f) * fy;
        for (int x = 0; x < W; ++x) {
            const float phi = (x + .5f) * fx;
            const Vf dir = toSphere({theta, phi});
            sky.radiance(fromSphere(dir), &env.rgb[3 * ((size_t) y * W + x)]);
        }
    }

    /* the sun (sunsky.cpp:154-225) */
    Sph sun = sunCoordinates(d, worldToLum);
    float sunRgb[3];
    sunRadiance(t, sun.elevation, d.turbidity, sunRgb);
    for (int c = 0; c < 3; ++c) sunRgb[c] *= d.sunScale;
    sun.elevation *= d.skyStretch;
    const Vf sn = toSphere(sun);
    Vf ss, st;
    coordinateSystem(sn, ss, st); /* Frame(n) */
    const float theta = degToRad((float) (0.5358 * 0.5f)); /* SUN_APP_RADIUS * 0.5f */
    if (d.sunRadiusScale == 0) {
        /* the reference adds a directional emitter instead (sunsky.cpp:172-183) */
        throw std::runtime_error("sunsky with sunRadiusScale = 0 (directional sun) is outside the hair hot path");
    }
    const size_t pixelCount = (size_t) d.skyResolution * d.skyResolution / 2;
    const float cosTheta = std::cos(theta * d.sunRadiusScale);
    const float coveredPortion = 0.5f * (1 - cosTheta);
    const size_t nSamples = (size_t) std::max((float) 100, (pixelCount * coveredPortion * 1000));
    const float gx = W / (2 * kPiF), gy = H / kPiF;
    float value[3];
    {
        const float k1 = 2 * kPiF * (1 - std::cos(theta));
        const float k2 = (float) (W * H);
        const float k3 = 2 * kPiF * kPiF * (float) nSamples;
        const float recip = 1.0f / k3;
        for (int c = 0; c < 3; ++c) value[c] = ((sunRgb[c] * k1) * k2) * recip;
    }
    for (size_t i = 0; i < nSamples; ++i) {
        const Vf l = squareToUniformCone(cosTheta, radicalInverse2((uint32_t) i), sobol2((uint32_t) i));
        const Vf dir = ss * l.x + st * l.y + sn * l.z; /* Frame::toWorld */
        const float sinTheta = safeSqrt(1 - dir.y * dir.y);
        const Sph sc = fromSphere(dir);
        const int px = std::min(std::max(0, (int) (sc.azimuth * gx)), W - 1);
        const int py = std::min(std::max(0, (int) (sc.elevation * gy)), H - 1);
        const float recip = 1.0f / std::max((float) 1e-3f, sinTheta);
        float *pix = &env.rgb[3 * ((size_t) py * W + px)];
        for (int c = 0; c < 3; ++c) pix[c] += value[c] * recip;
    }
    env.scale = 1.0f;
    std::memcpy(env.toWorld, d.emitterToWorld, sizeof(env.toWorld));
}

} // namespace hpt
