"""Film development and output: hpt_write_film against
the numpy restatement in oracle/film.py, on a synthetic accumulated film
(no GPU needed: development is host code)."""
import os
import sys

import numpy as np
import pytest

import oracle_lib  # noqa: F401  (puts the package on sys.path)
from mitsuba_amd import native, scenes

sys.path.insert(0, os.path.join(os.path.dirname(__file__), "..", "oracle"))
import film as ref  # noqa: E402

DATA = os.path.join(os.path.dirname(native.__file__), "..", "data")
BANNER = open(os.path.join(DATA, "film", "banner.u8"), "rb").read()


def _film(w=131, h=23, seed=0):
    rng = np.random.default_rng(seed)
    f = np.empty((h, w, 4), np.float32)
    wgt = rng.uniform(0.5, 3.0, (h, w)).astype(np.float32)
    rgb = rng.lognormal(-1.0, 1.5, (h, w, 3)).astype(np.float32)
    rgb[0, 0] = 0
    rgb[1, 1] = [1e-5, 0.002, 0.0031]
    f[..., :3] = rgb * wgt[..., None]
    f[..., 3] = wgt
    f[2, 2] = 0  # a pixel no sample reached
    return f


def _params(**kw):
    p = native.FilmParams()
    p.ldr, p.file_format, p.luminance, p.component_format, p.reinhard = 1, native.FILE_PNG, 0, 0, 0
    p.gamma, p.exposure, p.key, p.burn, p.banner = -1.0, 0.0, 0.18, 0.0, 1
    for k, v in kw.items():
        setattr(p, k, v)
    return p


@pytest.fixture(scope="module")
def host():
    return native.Renderer(device=native.HOST_ONLY)


@pytest.mark.parametrize("gamma,exposure,lum,banner", [(-1.0, 0.0, 0, 1), (2.2, 0.0, 0, 0), (-1.0, 1.5, 0, 1),
                                                        (1.8, -0.5, 1, 1)])
def test_ldrfilm_gamma_exact(tmp_path, host, gamma, exposure, lum, banner):
    film = _film()
    out = host.write_film(tmp_path / "a.jpg", film, _params(gamma=gamma, exposure=exposure, luminance=lum,
                                                             banner=banner))
    assert out.endswith("a.png")  # ldrfilm.cpp:335-345 replaces the extension
    got = ref.read_png(out)
    h, w = film.shape[:2]
    mask = ref.banner_mask(BANNER, w, h) if banner else None
    exp = ref.develop_ldr(film, gamma=gamma, exposure=exposure, luminance=bool(lum), banner=mask)
    np.testing.assert_array_equal(got, exp)
    if banner:
        assert mask.sum() > 100 and np.all(got[mask] == 255)


def test_ldrfilm_reinhard(tmp_path, host):
    film = _film(seed=3)
    out = host.write_film(tmp_path / "r.png", film, _params(reinhard=1, key=0.3, burn=0.2, banner=0))
    got = ref.read_png(out).astype(int)
    exp = ref.develop_ldr(film, reinhard_tm=True, key=0.3, burn=0.2).astype(int)
    # the log-average is a float32 running sum over all pixels in both; rounding of
    # pow / exp may move a value across an 8-bit step
    assert np.abs(got - exp).max() <= 1
    assert np.mean(got == exp) > 0.995


@pytest.mark.parametrize("comp", [native.COMPONENT_FLOAT16, native.COMPONENT_FLOAT32, native.COMPONENT_UINT32])
@pytest.mark.parametrize("lum", [0, 1])
def test_hdrfilm_openexr(tmp_path, host, comp, lum):
    film = _film(seed=1)
    out = host.write_film(tmp_path / "x", film, _params(ldr=0, file_format=native.FILE_OPENEXR, component_format=comp,
                                                        luminance=lum, banner=1))
    assert out.endswith("x.exr")
    ch = ref.read_exr(out)
    px = ref.resolve(film, bool(lum))
    h, w = film.shape[:2]
    px[ref.banner_mask(BANNER, w, h)] = 1024.0  # hdrfilm.cpp:492-502
    names = ["Y"] if lum else ["R", "G", "B"]
    assert sorted(ch) == sorted(names)
    for i, n in enumerate(names):
        if comp == native.COMPONENT_FLOAT16:
            np.testing.assert_array_equal(ch[n], px[..., i].astype(np.float16).astype(np.float32))
        elif comp == native.COMPONENT_FLOAT32:
            np.testing.assert_array_equal(ch[n], px[..., i])
        else:
            # fmtconv.cpp:1158 clamps to (float) UINT32_MAX == 2^32, whose cast to uint32 is
            # undefined; saturating at UINT32_MAX is the defined choice made here
            v = np.minimum(np.float32(4294967295.0), np.maximum(0, px[..., i] * np.float32(4294967295.0)
                                                                + np.float32(0.5))).astype(np.float64)
            np.testing.assert_array_equal(ch[n], np.minimum(v, 4294967295.0).astype(np.uint32))


def test_hdrfilm_pfm_and_rgbe(tmp_path, host):
    film = _film(w=200, h=12, seed=2)
    px = ref.resolve(film)
    out = host.write_film(tmp_path / "p.exr", film, _params(ldr=0, file_format=native.FILE_PFM, banner=0))
    assert out.endswith("p.pfm")
    np.testing.assert_array_equal(ref.read_pfm(out), px)
    out = host.write_film(tmp_path / "e", film, _params(ldr=0, file_format=native.FILE_RGBE, banner=0,
                                                        component_format=native.COMPONENT_FLOAT16))
    assert out.endswith("e.rgbe")
    dec, raw = ref.read_rgbe(out)
    np.testing.assert_array_equal(raw, ref.rgbe_encode(px))  # RLE decodes to RGBE_FromFloat's bytes
    # one shared exponent per pixel: every channel is within 2^-7 of the pixel's largest
    assert np.all(np.abs(dec - px) <= px.max(axis=-1, keepdims=True) * 2.0 ** -7)


def test_film_properties_from_scene_xml(tmp_path):
    xml = scenes.make_scene("furball_marschner", str(tmp_path), n_strands=50)
    src = open(xml).read()
    r = native.Renderer(device=native.HOST_ONLY)
    r.load_scene_xml(xml)
    p = r.film_params()
    assert (p.ldr, p.file_format, p.luminance, p.banner) == (1, native.FILE_PNG, 0, 0) and p.gamma == np.float32(2.2)
    hdr = src.replace('<film type="ldrfilm">', '<film type="hdrfilm">').replace(
        '<string name="fileFormat" value="png"/>', '<string name="fileFormat" value="rgbe"/>').replace(
        '<float name="gamma" value="2.2"/>', '<string name="componentFormat" value="float16"/>')
    path = tmp_path / "hdr.xml"
    path.write_text(hdr)
    r.load_scene_xml(str(path))
    p = r.film_params()
    # hdrfilm.cpp:314-325: RGBE overrides the component format to float32
    assert (p.ldr, p.file_format, p.component_format, p.banner) == (0, native.FILE_RGBE, native.COMPONENT_FLOAT32, 0)
    for old, new, msg in [('<string name="pixelFormat" value="rgb"/>', '<string name="pixelFormat" value="rgba"/>',
                           "alpha"),
                          ('<string name="fileFormat" value="png"/>', '<string name="fileFormat" value="jpeg"/>',
                           "JPEG"),
                          ('<string name="fileFormat" value="png"/>', '<string name="fileFormat" value="tga"/>',
                           "fileFormat")]:
        path.write_text(src.replace(old, new))
        with pytest.raises(native.HairPTError, match=msg):
            r.load_scene_xml(str(path))
