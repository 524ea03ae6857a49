"""The multi-device boundary under concurrency (include/hairpt.h, hpt_context_share_scene):
bin/mitsuba --gpus N shares one prepared source context from N - 1 threads at once.  Every
share here fails (an unprepared source, or a device index no machine has), and each failure
must reach its own thread through hpt_last_error(NULL) while the shared source stays
untouched.  The driver (tests/native/share_threads.cpp) runs against a ThreadSanitizer build
of the host code (`make tsan`): a write to the source from the workers is a reported race
and fails the run.  CPU only: no device is opened.
"""
import os
import subprocess

import pytest

import scene_util
from mitsuba_amd import native

PKG = os.path.join(os.path.dirname(native.__file__), "..")
BIN = os.path.join(PKG, "build", "tsan", "share_threads")


@pytest.fixture(scope="module")
def driver():
    if not os.path.exists(BIN):
        subprocess.check_call(["make", "-s", "-j8", "-C", PKG, "tsan"], stdout=subprocess.DEVNULL)
    return BIN


def test_share_failures_reach_their_threads_under_tsan(driver, tmp_path):
    xml = scene_util.scenes.make_scene("straight_kk", str(tmp_path), n_strands=100)
    env = dict(os.environ, TSAN_OPTIONS="halt_on_error=1 exitcode=66 report_signal_unsafe=0")
    res = subprocess.run([driver, xml, "16", os.path.join(PKG, "data")], capture_output=True, text=True, timeout=600, env=env)
    assert "ThreadSanitizer" not in res.stderr, res.stderr[-4000:]
    assert res.returncode == 0, res.stdout + res.stderr[-4000:]
    assert "16 threads, 16 failures reported per thread, 0 bad" in res.stdout
