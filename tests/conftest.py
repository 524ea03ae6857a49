import os
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
PKG = os.path.join(ROOT, "cs184-final-project-mitsuba0.5_amd")
for p in (HERE, PKG):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs an MI355X (gfx950) device; run with -m gpu")


def pytest_sessionstart(session):
    """Build the native library and the oracle if a fresh checkout lacks them
    (make is never run when the built files are present)."""
    import subprocess

    lib = os.path.join(PKG, "lib", "libhairpt.so")
    orc = os.path.join(ROOT, "oracle", "_build", "liboracle.so")
    jobs = str(min(16, os.cpu_count() or 4))
    if not os.path.exists(lib):
        subprocess.check_call(["make", "-j", jobs, "-C", PKG, "ARCH=gfx950"])
    if not os.path.exists(orc):
        subprocess.check_call(["make", "-j", jobs, "-C", os.path.join(ROOT, "oracle")])
