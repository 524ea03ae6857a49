"""One process, several devices (hpt_context_share_scene / hpt_render_multi; the reference loads
the scene once and hands it to every worker, src/mitsuba/mitsuba.cpp:281-329).

CPU: a host-only context shares a prepared scene without parsing, loading or building it again
(the kd-tree and every table are the source's: the build time is the source's own figure).
GPU: two contexts on device 0 (the box has one GPU; the shards time-share it) render the
Hilbert-cyclic halves of a frame and combine them on the device; the film equals the one-context
render up to the order of the per-pixel sums, and bit-for-bit the host sum of the two shard films.
The CLI's --devices 0,0 renders through the same path."""
import os
import subprocess

import numpy as np
import pytest

import scene_util
from mitsuba_amd import native


def _host_ctx(xml, defines):
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(xml, defines)
    r.prepare()
    return r


def test_share_scene_host_only(tmp_path):
    xml = scene_util.scenes.make_scene("furball_marschner", str(tmp_path), n_strands=600)
    src = _host_ctx(xml, {"spp": 4, "width": 40, "height": 24})
    dst = src.share_scene(native.HOST_ONLY)
    a, b = src.info(), dst.info()
    for f in ("width", "height", "spp", "max_depth", "segments", "kd_nodes", "kd_indices", "kd_depth", "bsdf"):
        assert getattr(a, f) == getattr(b, f), f
    # not rebuilt: the shared tree carries the source build's own timing
    assert a.kd_build_seconds == b.kd_build_seconds
    na, ia, _ = src.kdtree()
    nb, ib, _ = dst.kdtree()
    np.testing.assert_array_equal(na, nb)
    np.testing.assert_array_equal(ia, ib)
    assert src.scene_json() == dst.scene_json()
    dst.close()
    src.close()


def test_share_scene_needs_a_prepared_source(tmp_path):
    xml = scene_util.scenes.make_scene("furball_marschner", str(tmp_path), n_strands=100)
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(xml, {})
    with pytest.raises(native.HairPTError, match="not prepared"):
        r.share_scene(native.HOST_ONLY)
    # the message went to the calling thread (hpt_last_error(NULL)), not to the source context
    assert r.lib.hpt_last_error(r.h).decode() == ""
    assert "not prepared" in r.lib.hpt_last_error(None).decode()
    # a later create/share clears the thread's message first: after a success it no longer
    # describes the earlier failure
    r.prepare()
    dst = r.share_scene(native.HOST_ONLY)
    assert "not prepared" not in r.lib.hpt_last_error(None).decode()
    dst.close()
    r.close()


def test_block_weights_are_checked():
    # the deal's sort needs a strict weak order: NaN, negative or infinite weights are refused
    for bad in (np.nan, -1.0, np.inf):
        with pytest.raises(native.HairPTError):
            native.block_deal(64, 64, 2, [1.0, bad, 2.0, 3.0])
    assert list(native.block_deal(64, 64, 2, [4.0, 1.0, 2.0, 3.0])) == [0, 0, 1, 1]  # 4 | 3, 2 | 1


@pytest.mark.gpu
def test_render_multi_two_contexts_one_device(tmp_path):
    xml = scene_util.scenes.make_scene("furball_marschner", str(tmp_path), n_strands=1500)
    defs = {"spp": 8, "width": 96, "height": 64}
    r0 = native.Renderer(device=0)
    r0.load_scene_xml(xml, defs)
    r0.prepare()
    r1 = r0.share_scene(0)
    single = r0.render(0, 8)
    multi = native.Renderer.render_multi([r0, r1], 0, 8)
    # the same shards rendered separately and summed on the host, in shard order
    f0 = r0.render(0, 8, shard=0, n_shards=2)
    f1 = r1.render(0, 8, shard=1, n_shards=2)
    np.testing.assert_array_equal(multi, f0 + f1)
    np.testing.assert_allclose(multi, single, rtol=1e-5, atol=1e-5)
    # accumulating into a film (the CLI's -r chunks)
    acc = native.Renderer.render_multi([r0, r1], 0, 4)
    acc = native.Renderer.render_multi([r0, r1], 4, 8, film=acc)
    np.testing.assert_allclose(acc, single, rtol=1e-5, atol=1e-5)
    r1.close()
    r0.close()


@pytest.mark.gpu
def test_render_multi_weighted_deal_and_mismatches(tmp_path):
    """weights set before the share travel with it (every block rendered exactly once); contexts
    that would render different deals or scenes into one film are refused before rendering"""
    xml = scene_util.scenes.make_scene("furball_marschner", str(tmp_path), n_strands=1500)
    defs = {"spp": 4, "width": 96, "height": 64}
    r0 = native.Renderer(device=0)
    r0.load_scene_xml(xml, defs)
    r0.prepare()
    single = r0.render(0, 4)
    w = np.array([5.0, 1.0, 1.0, 1.0, 1.0, 9.0])
    r0.set_block_weights(w)
    r1 = r0.share_scene(0)
    multi = native.Renderer.render_multi([r0, r1], 0, 4)
    np.testing.assert_allclose(multi, single, rtol=1e-5, atol=1e-5)
    # every pixel's samples exactly once: a block rendered twice or never moves its filter weights
    # by whole samples (border pixels sum two shards, so the last bit may differ)
    np.testing.assert_allclose(multi[..., 3], single[..., 3], rtol=1e-6, atol=0)
    # a context whose weights differ from ctxs[0]'s
    r1.set_block_weights(w[::-1].copy())
    with pytest.raises(native.HairPTError, match="weights"):
        native.Renderer.render_multi([r0, r1], 0, 4)
    r1.set_block_weights(w)
    np.testing.assert_array_equal(native.Renderer.render_multi([r0, r1], 0, 4), multi)
    # a context prepared again renders a scene of its own
    r1.prepare()
    with pytest.raises(native.HairPTError, match="different prepared scene"):
        native.Renderer.render_multi([r0, r1], 0, 4)
    # weights for another frame size fail the render loudly
    r2 = native.Renderer(device=0)
    r2.load_scene_xml(xml, defs)
    r2.prepare()
    r2.set_block_weights(np.ones(4))
    with pytest.raises(native.HairPTError, match="block weights"):
        r2.render(0, 4)
    for r in (r2, r1, r0):
        r.close()


@pytest.mark.gpu
def test_cli_devices_share_one_scene(tmp_path):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
    import film as ref
    cli = os.path.join(os.path.dirname(native.__file__), "..", "bin", "mitsuba")
    xml = scene_util.scenes.make_scene("furball_marschner", str(tmp_path), n_strands=800)
    base = [cli, "-D", "spp=8", "-D", "width=64", "-D", "height=48"]
    one = subprocess.run(base + ["-o", str(tmp_path / "one.png"), xml], capture_output=True, text=True, timeout=300)
    assert one.returncode == 0, one.stderr
    two = subprocess.run(base + ["--devices", "0,0", "-o", str(tmp_path / "two.png"), xml], capture_output=True,
                         text=True, timeout=300)
    assert two.returncode == 0, two.stderr
    assert two.stdout.count("Scene \"") == 1 and "shared with 1 more device context" in two.stdout
    a = ref.read_png(str(tmp_path / "one.png")).astype(int)
    b = ref.read_png(str(tmp_path / "two.png")).astype(int)
    assert np.abs(a - b).max() <= 1
