/*
 * lobatto.h -- oracle restatement of GaussLobattoIntegrator
 * (src/libcore/quad.cpp:287-409, include/mitsuba/core/quad.h:155-159).
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Float = float (SINGLE_PRECISION).
 * useConvergenceEstimate is the constructor's 4th argument, whose default in
 * the reference is true (quad.h:158); callers pass it explicitly:
 *   sunsky_ref.cpp  ContinuousSpectrum::average            false
 *   mesh_bsdf.h     fresnelDiffuseReflectance (util.cpp:856) true (default)
 */
#ifndef HAIRPT_ORACLE_LOBATTO_H
#define HAIRPT_ORACLE_LOBATTO_H
#include <algorithm>
#include <cmath>
#include <cstddef>
#include <functional>
#include <limits>
#include <utility>

namespace orc_quad {

class Lobatto {
public:
    Lobatto(size_t maxEvals, float absErr, float relErr, bool useConvergenceEstimate)
        : maxEvals_(maxEvals), abs_(absErr), rel_(relErr), conv_(useConvergenceEstimate) {}
    float integrate(const std::function<float(float)> &f, float a, float b) const { /* quad.cpp:305-323 */
        float sign = 1;
        size_t evals = 0;
        if (a == b) return 0;
        if (b < a) std::swap(a, b), sign = -1;
        const float tol = tolerance(f, a, b, evals);
        evals += 2;
        return sign * step(f, a, b, f(a), f(b), tol, evals);
    }

private:
    size_t maxEvals_;
    float abs_, rel_;
    bool conv_;
    static float A() { return (float) std::sqrt(2.0 / 3.0); }
    static float B() { return (float) (1.0 / std::sqrt(5.0)); }
    float tolerance(const std::function<float(float)> &f, float a, float b, size_t &evals) const { /* :325-369 */
        const float m = (a + b) / 2, h = (b - a) / 2;
        const float X1 = (float) 0.94288241569547971906, X2 = (float) 0.64185334234578130578,
                    X3 = (float) 0.23638319966214988028;
        const float y1 = f(a), y3 = f(m - A() * h), y5 = f(m - B() * h), y7 = f(m), y9 = f(m + B() * h),
                    y11 = f(m + A() * h), y13 = f(b);
        const float acc = h * ((float) 0.0158271919734801831 * (y1 + y13) +
                               (float) 0.0942738402188500455 * (f(m - X1 * h) + f(m + X1 * h)) +
                               (float) 0.1550719873365853963 * (y3 + y11) +
                               (float) 0.1888215739601824544 * (f(m - X2 * h) + f(m + X2 * h)) +
                               (float) 0.1997734052268585268 * (y5 + y9) +
                               (float) 0.2249264653333395270 * (f(m - X3 * h) + f(m + X3 * h)) +
                               (float) 0.2426110719014077338 * y7);
        evals += 13;
        float r = 1.0f;
        if (conv_) {
            const float integral2 = (h / 6) * (y1 + y13 + 5 * (y5 + y9));
            const float integral1 = (h / 1470) * (77 * (y1 + y13) + 432 * (y3 + y11) + 625 * (y5 + y9) + 672 * y7);
            if (std::abs(integral2 - acc) != 0.0) r = std::abs(integral1 - acc) / std::abs(integral2 - acc);
            if (r == 0.0 || r > 1.0) r = 1.0f;
        }
        const float eps = std::numeric_limits<float>::epsilon();
        float out = std::numeric_limits<float>::infinity();
        if (rel_ != 0 && acc != 0) out = acc * std::max(rel_, eps) / (r * eps);
        if (abs_ != 0) out = std::min(out, abs_ / (r * eps));
        return out;
    }
    float step(const std::function<float(float)> &f, float a, float b, float fa, float fb, float acc,
               size_t &evals) const { /* :371-409 */
        const float h = (b - a) / 2, m = (a + b) / 2;
        const float mll = m - A() * h, ml = m - B() * h, mr = m + B() * h, mrr = m + A() * h;
        const float fmll = f(mll), fml = f(ml), fm = f(m), fmr = f(mr), fmrr = f(mrr);
        const float i2 = (h / 6) * (fa + fb + 5 * (fml + fmr));
        const float i1 = (h / 1470) * (77 * (fa + fb) + 432 * (fmll + fmrr) + 625 * (fml + fmr) + 672 * fm);
        evals += 5;
        if (evals >= maxEvals_) return i1;
        const float dist = acc + (i1 - i2);
        if (dist == acc || mll <= a || b <= mrr) return i1;
        return step(f, a, mll, fa, fmll, acc, evals) + step(f, mll, ml, fmll, fml, acc, evals) +
               step(f, ml, m, fml, fm, acc, evals) + step(f, m, mr, fm, fmr, acc, evals) +
               step(f, mr, mrr, fmr, fmrr, acc, evals) + step(f, mrr, b, fmrr, fb, acc, evals);
    }
};

} // namespace orc_quad
#endif
