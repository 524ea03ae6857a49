// Golden-vector driver: instantiates the REFERENCE's GaussLegendre<140>
// (src/bsdfs/gausssexylingerie.hpp:11-93) exactly as marschner_diffuse.cpp:758
// does and prints nodes/weights as hex floats.  Built only from reference
// headers + system headers by oracle/ref.mk (no stand-in headers).
#include <mitsuba/core/constants.h>
#include "gausssexylingerie.hpp"
#include <cstdio>
int main() {
    mitsuba::GaussLegendre<140> g;
    for (int i = 0; i < 140; ++i)
        std::printf("%a %a\n", (double) g.points()[i], (double) g.weights()[i]);
    return 0;
}
