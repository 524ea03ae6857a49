"""Independent float64 restatements of host precomputations (CPU tests).

The product's host code and the oracle are both C++ restatements of the
reference; a shared misreading would pass every product-vs-oracle test.  The
tables below are therefore also restated a third way, in float64 numpy
written from the reference source with different structure (vectorised, no
shared code), and the product's float32 tables must agree with them to
within float32 rounding:

  - the Marschner azimuthal tables N_R, N_TT, N_TRT
    (MarschnerDiffuse::precomputeAzimuthalDistributions,
    src/bsdfs/marschner_diffuse.cpp:751-847, with D / Phi / the swapped
    fresnelDielectricExt arguments of :302-318, :809 and util.cpp:651-681);
    Gauss-Legendre nodes come from numpy.polynomial.legendre.leggauss, not
    from the reference's GaussLegendre<140> (pinned separately by golden
    vectors in test_oracle_golden.py).
"""
import numpy as np
import pytest

import scene_util
from mitsuba_amd import native

RES = 64           # Azimuthal::AzimuthalResolution (marschner_diffuse.cpp:66)
NGAUSS = 2048      # NumGaussianSamples (:775)
PI_F = float(np.float32(np.pi))  # M_PI_FLT, the float constant the reference uses


def _fresnel_ext(cos_i, eta):
    """fresnelDielectricExt(cosThetaI_, eta) (util.cpp:651-681), float64, vectorised."""
    cos_i, eta = np.broadcast_arrays(np.asarray(cos_i, np.float64), np.asarray(eta, np.float64))
    with np.errstate(divide="ignore", invalid="ignore"):
        scale = np.where(cos_i > 0, 1.0 / eta, eta)
        ct2 = 1.0 - (1.0 - cos_i * cos_i) * scale * scale
        ci = np.abs(cos_i)
        ct = np.sqrt(np.maximum(ct2, 0.0))
        rs = (ci - eta * ct) / (ci + eta * ct)
        rp = (eta * ci - ct) / (eta * ci + ct)
        f = 0.5 * (rs * rs + rp * rp)
    f = np.where(ct2 <= 0.0, 1.0, f)
    return np.where(eta == 1.0, 0.0, f)


def _gauss(beta, theta):
    return np.exp(-theta * theta / (2 * beta * beta)) / (np.sqrt(2 * PI_F) * beta)


def _detector(beta, phi):
    """D(beta, phi) (:305-315): wrapped Gaussian, summed until a term pair <= 1e-4."""
    phi = np.asarray(phi, np.float64)
    result = np.zeros_like(phi)
    live = np.ones(phi.shape, bool)
    shift = 0.0
    while live.any():
        delta = _gauss(beta, phi + shift) + _gauss(beta, phi - shift - 2 * PI_F)
        result = np.where(live, result + delta, result)
        live &= delta > 1e-4
        shift += 2 * PI_F
    return result


def marschner_tables_f64(eta, sigma_a=0.5, beta_r=0.1):
    """(N_R, N_TT, N_TRT) as (64*64,) arrays (index phiI + y*64) in float64."""
    x, w = np.polynomial.legendre.leggauss(140)
    gamma_i = np.arcsin(x)
    # every lobe's detector uses _betaR (:778), tabulated at 2048 samples over [0, 2pi] (:776-779)
    dtab = _detector(beta_r, np.arange(NGAUSS) / (NGAUSS - 1.0) * 2 * PI_F)

    def approx_d(phi):  # :782-788: |phi| in table steps, wrapped linear interpolation
        u = np.abs(phi * (1.0 / (2 * PI_F) * (NGAUSS - 1)))
        x0 = np.floor(u).astype(np.int64)
        f = u - x0
        return dtab[x0 % NGAUSS] * (1 - f) + dtab[(x0 + 1) % NGAUSS] * f

    tables = [np.zeros(RES * RES), np.zeros(RES * RES), np.zeros(RES * RES)]
    phis = 2 * PI_F * np.arange(RES) / (RES - 1.0)
    for y in range(RES):
        c = y / (RES - 1.0)
        with np.errstate(divide="ignore"):
            ior_p = np.sqrt(eta * eta - (1 - c * c)) / c
        cos_t = np.sqrt(1 - (1 - c * c) / (eta * eta))
        sig = sigma_a / cos_t
        gamma_t = np.arcsin(np.clip(x / ior_p, -1, 1))
        fr = _fresnel_ext(1.0 / eta, c * np.cos(gamma_i))  # arguments swapped as at :809
        T = np.exp(-sig * 2 * np.cos(gamma_t))
        a_tt = (1 - fr) ** 2 * T
        a_trt = a_tt * fr * T
        for p, amp in enumerate((fr, a_tt, a_trt)):
            big_phi = 2 * p * gamma_t - 2 * gamma_i + p * PI_F  # Phi (:317-319)
            d = approx_d(phis[:, None] - big_phi[None, :])      # (phi, h)
            tables[p][y * RES:(y + 1) * RES] = 0.5 * (d * (w * amp)[None, :]).sum(1)
    return tables


@pytest.mark.parametrize("eta", [1.55, 1.3, 2.1])
def test_marschner_tables_match_float64_restatement(eta):
    cfg, cam, _ = scene_util.config_params("furball_marschner")
    r = native.Renderer(device=native.HOST_ONLY)
    xml = scene_util.scenes.make_scene("furball_marschner", scene_util.WORK, n_strands=200)
    src = open(xml).read().replace('<float name="intIOR" value="1.55"/>', '<float name="intIOR" value="%r"/>' % eta)
    path = xml[:-4] + "_eta%g.xml" % eta
    with open(path, "w") as f:
        f.write(src)
    r.load_scene_xml(path, {"width": 16, "height": 16, "spp": 1})
    r.prepare()
    prod, _, _, _ = r.marschner_tables()
    want = marschner_tables_f64(float(np.float32(eta) / np.float32(1.0)))
    for lobe, (p, q) in enumerate(zip(prod, want)):
        p = p.astype(np.float64)
        assert np.all(p[:, 0] == p[:, 1]) and np.all(p[:, 0] == p[:, 2])  # sigma_a is grey (:125)
        scale = max(q.max(), 1e-30)
        err = np.abs(p[:, 0] - q) / scale
        print("eta %.2f lobe %d: max |float32 - float64| / max = %.3g (max %.4g)" % (eta, lobe, err.max(), scale))
        # float32 accumulation of 140 Gauss-Legendre terms, float32 transcendental functions
        # and the float32 detector table: the tables agree to float32 rounding
        assert err.max() < 1e-5, (lobe, err.max())
        zero = q == 0
        np.testing.assert_array_equal(p[zero, 0], 0.0)
