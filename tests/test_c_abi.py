"""The boundary driven from C: bin/hpt_render_c (examples/hpt_render_c.c, C99, compiled
against include/hairpt.h alone with -Wall -Wextra -Werror -pedantic) loads a scene with
-D defines through hpt_load_scene_xml, prepares, renders and writes the film.

CPU: the defines reach the parsed scene (hpt_get_scene_info) and a host-only context
refuses to render.  GPU: the film the C program renders is bit-identical to the library
render of the same scene and defines through ctypes, and its PNG equals hpt_write_film's.
"""
import os
import subprocess
import sys

import numpy as np
import pytest

import scene_util
from mitsuba_amd import native

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import film as ref  # noqa: E402

BIN = os.path.join(os.path.dirname(native.__file__), "..", "bin", "hpt_render_c")
DEFINES = {"width": 40, "height": 24, "spp": 3, "maxDepth": 7}


def _cmd(xml, device, *extra):
    if not os.path.exists(BIN):
        raise RuntimeError("bin/hpt_render_c is missing: run __graft_entry__.build() (make -C the package)")
    cmd = [BIN, "-d", str(device)]
    for k, v in DEFINES.items():
        cmd += ["-D", "%s=%s" % (k, v)]
    return cmd + list(extra) + [xml]


def test_c_driver_forwards_defines_host_only(tmp_path):
    xml = scene_util.scenes.make_scene("straight_kk", str(tmp_path), n_strands=200)
    res = subprocess.run(_cmd(xml, native.HOST_ONLY), capture_output=True, text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    assert "scene 40x24 spp 3 maxDepth 7 rrDepth 5 shapes 1" in res.stdout
    assert "bsdf 1" in res.stdout  # Kajiya-Kay
    assert "host-only render refused: -3" in res.stdout
    # the same defines as the process-wide table (hpt_set_default_defines) reach the parse too
    res_p = subprocess.run(_cmd(xml, native.HOST_ONLY, "-P"), capture_output=True, text=True, timeout=120)
    assert res_p.returncode == 0 and res_p.stdout.splitlines()[0] == res.stdout.splitlines()[0]
    # without defines the scene's own <default> values apply
    res_d = subprocess.run([BIN, "-d", "-1", xml], capture_output=True, text=True, timeout=120)
    assert res_d.returncode == 0 and "scene 256x256 spp 64 maxDepth 65" in res_d.stdout
    # a malformed define is refused by the driver before the library sees it
    bad = subprocess.run([BIN, "-d", "-1", "-D", "width", xml], capture_output=True, text=True, timeout=60)
    assert bad.returncode == 2 and "bad define" in bad.stderr


@pytest.mark.gpu
def test_c_driver_renders_like_the_library(tmp_path):
    xml = scene_util.scenes.make_scene("straight_kk", str(tmp_path), n_strands=200)
    raw = tmp_path / "film.bin"
    res = subprocess.run(_cmd(xml, 0, "-c", str(raw), "-o", str(tmp_path / "c_out.jpg")), capture_output=True,
                         text=True, timeout=120)
    assert res.returncode == 0, res.stdout + res.stderr
    film_c = np.fromfile(str(raw), np.float32).reshape(24, 40, 4)
    r = native.Renderer(device=0)
    r.load_scene_xml(xml, DEFINES)
    r.prepare()
    film = r.render(0, 3)
    np.testing.assert_array_equal(film_c, film)
    out = r.write_film(tmp_path / "lib.png", film)
    np.testing.assert_array_equal(ref.read_png(str(tmp_path / "c_out.png")), ref.read_png(out))
