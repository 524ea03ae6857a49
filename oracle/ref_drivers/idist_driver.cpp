// Golden-vector driver for the REFERENCE's InterpolatedDistribution1D
// (src/bsdfs/InterpolatedDistribution1D.hpp:7-111).  Reads
//   size ndist n  / size*ndist weights / n pairs (dist u)
// from stdin and prints "x u' pdf sum" per query (hex floats).
#include <cmath>
#include <algorithm>
#include <cstdint>
#include <mitsuba/core/platform.h>
#include <mitsuba/core/constants.h>
#include <mitsuba/core/math.h>
#include <vector>
#include "InterpolatedDistribution1D.hpp"
#include <cstdio>
int main() {
    int size, ndist, n;
    if (std::scanf("%d %d %d", &size, &ndist, &n) != 3) return 1;
    std::vector<float> w((size_t) size * ndist);
    for (auto &v : w) { double d; if (std::scanf("%la", &d) != 1) return 1; v = (float) d; }
    mitsuba::InterpolatedDistribution1D dist(w, size, ndist);
    for (int i = 0; i < n; ++i) {
        double dd, uu;
        if (std::scanf("%la %la", &dd, &uu) != 2) return 1;
        float d = (float) dd, u = (float) uu;
        int x;
        dist.warp(d, u, x);
        std::printf("%d %a %a %a\n", x, (double) u, (double) dist.pdf(d, x), (double) dist.sum(d));
    }
    return 0;
}
