"""mitsuba_amd -- MI355X-native drop-in for the hair path-tracing hot path of
ja5087/cs184-final-project-mitsuba0.5 (path integrator x hair shape x
marschner / kajiyakay BSDFs x sunsky lighting).

The product is libhairpt.so (C ABI in include/hairpt.h, HIP kernels for
gfx950) plus the `mitsuba` CLI in bin/.  This package is the thin Python
mirror used by tests and bench.py.
"""
from . import scenes, synth_hair  # noqa: F401

__all__ = ["scenes", "synth_hair", "native"]
