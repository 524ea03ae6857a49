"""ctypes binding of libhairpt.so (include/hairpt.h).

This is the Python mirror of the reference's render entry points
(SamplingIntegrator::render -> MIPathTracer::Li, src/librender/integrator.cpp
:95-188, src/integrators/path/path.cpp:119-294).  There is no CPU fallback:
if the HIP library is missing or no gfx950 device is present, every call
raises.
"""
from __future__ import annotations

import ctypes as C
import os

import numpy as np

PKG = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.path.join(PKG, "lib", "libhairpt.so")
DATA_DIR = os.path.join(PKG, "data")
HOST_ONLY = -1  # include/hairpt.h HPT_HOST_ONLY: build/export the scene without a device

_f = C.POINTER(C.c_float)
_u8 = C.POINTER(C.c_uint8)
_u32 = C.POINTER(C.c_uint32)
_i32 = C.POINTER(C.c_int32)
_u64 = C.POINTER(C.c_uint64)
_i64 = C.POINTER(C.c_int64)


class SceneInfo(C.Structure):
    _fields_ = [("width", C.c_int), ("height", C.c_int), ("spp", C.c_int), ("max_depth", C.c_int),
                ("rr_depth", C.c_int), ("strict_normals", C.c_int), ("hide_emitters", C.c_int), ("bsdf", C.c_int),
                ("vertices", C.c_uint64), ("segments", C.c_uint64), ("kd_nodes", C.c_uint64),
                ("kd_indices", C.c_uint64), ("kd_depth", C.c_int), ("kd_build_seconds", C.c_double),
                ("aabb_min", C.c_float * 3), ("aabb_max", C.c_float * 3), ("bsphere_center", C.c_float * 3),
                ("bsphere_radius", C.c_float), ("n_shapes", C.c_int)]


class FilmParams(C.Structure):
    _fields_ = [("ldr", C.c_int), ("file_format", C.c_int), ("luminance", C.c_int), ("component_format", C.c_int),
                ("reinhard", C.c_int), ("gamma", C.c_float), ("exposure", C.c_float), ("key", C.c_float),
                ("burn", C.c_float), ("banner", C.c_int)]


FILE_PNG, FILE_OPENEXR, FILE_RGBE, FILE_PFM = 0, 1, 2, 3
COMPONENT_FLOAT16, COMPONENT_FLOAT32, COMPONENT_UINT32 = 0, 1, 2


class RenderParams(C.Structure):
    _fields_ = [("spp_begin", C.c_int), ("spp_end", C.c_int), ("shard", C.c_int), ("n_shards", C.c_int),
                ("max_wave_paths", C.c_uint64), ("collect_stats", C.c_int)]


class Stats(C.Structure):
    _fields_ = [("ms_total", C.c_double), ("ms_camera", C.c_double), ("ms_trace", C.c_double),
                ("ms_primary", C.c_double), ("ms_shade", C.c_double), ("ms_post", C.c_double),
                ("ms_gather", C.c_double), ("trace_launches", C.c_uint64), ("paths", C.c_uint64),
                ("closest_rays", C.c_uint64), ("shadow_rays", C.c_uint64), ("nodes", C.c_uint64),
                ("prims", C.c_uint64), ("bounces", C.c_uint64), ("shadow_unoccluded", C.c_uint64),
                ("waves", C.c_uint64), ("max_bounces", C.c_int), ("prim_exact", C.c_uint64),
                ("node_slots", C.c_uint64), ("prim_slots", C.c_uint64), ("ms_tail", C.c_double),
                ("tail_paths", C.c_uint64), ("ms_trace_packet", C.c_double), ("packet_launches", C.c_uint64),
                ("packet_rays", C.c_uint64), ("packet_nodes", C.c_uint64), ("packet_prims", C.c_uint64),
                ("packet_exact", C.c_uint64), ("packet_node_slots", C.c_uint64), ("packet_prim_slots", C.c_uint64),
                ("packet_fallbacks", C.c_uint64), ("max_leaf_rounds", C.c_uint64), ("max_restarts", C.c_uint64),
                ("restarted_rays", C.c_uint64), ("binary_nodes", C.c_uint64), ("waves_ahead", C.c_uint64),
                ("schedule_misses", C.c_uint64), ("schedule_extensions", C.c_uint64)]


# every symbol declared in include/hairpt.h: (restype, argtypes)
SIGNATURES = {
    "hpt_context_create": (C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    "hpt_context_destroy": (None, [C.c_void_p]),
    "hpt_last_error": (C.c_char_p, [C.c_void_p]),
    "hpt_set_data_dir": (C.c_int, [C.c_void_p, C.c_char_p]),
    "hpt_load_scene_xml": (C.c_int, [C.c_void_p, C.c_char_p, C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p)]),
    "hpt_set_default_defines": (C.c_int, [C.c_int, C.POINTER(C.c_char_p), C.POINTER(C.c_char_p)]),
    "hpt_export_scene_json": (C.c_int, [C.c_void_p, C.c_char_p, C.c_size_t, C.POINTER(C.c_size_t)]),
    "hpt_set_camera": (C.c_int, [C.c_void_p, _f, C.c_float, C.c_int, C.c_int, C.c_float, C.c_float]),
    "hpt_set_sampler": (C.c_int, [C.c_void_p, C.c_int]),
    "hpt_set_sampler_scramble": (C.c_int, [C.c_void_p, C.c_uint64]),
    "hpt_set_traversal_bounds": (C.c_int, [C.c_void_p, C.c_uint32, C.c_uint32]),
    "hpt_set_packet_stack": (C.c_int, [C.c_void_p, C.c_uint32]),
    "hpt_clear_schedules": (C.c_int, [C.c_void_p]),
    "hpt_get_block_costs": (C.c_int, [C.c_void_p, C.POINTER(C.c_uint64), C.c_int]),
    "hpt_set_block_weights": (C.c_int, [C.c_void_p, C.POINTER(C.c_double), C.c_int]),
    "hpt_block_deal": (C.c_int, [C.c_int, C.c_int, C.c_int, C.POINTER(C.c_double), C.POINTER(C.c_int32)]),
    "hpt_debug_sfmt": (C.c_int, [C.c_uint64, C.c_uint64, C.POINTER(C.c_uint64)]),
    "hpt_debug_fresnel_diffuse": (C.c_int, [C.c_int, C.POINTER(C.c_float), C.POINTER(C.c_float)]),
    "hpt_set_integrator": (C.c_int, [C.c_void_p, C.c_int, C.c_int, C.c_int, C.c_int]),
    "hpt_set_hair_file": (C.c_int, [C.c_void_p, C.c_char_p, C.c_float, C.c_float, _f]),
    "hpt_set_hair_reduction": (C.c_int, [C.c_void_p, C.c_float]),
    "hpt_set_hair_vertices": (C.c_int, [C.c_void_p, _f, _u8, C.c_uint64, C.c_float]),
    "hpt_set_bsdf_marschner": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_int, C.c_float, _f, _f]),
    "hpt_set_bsdf_kajiyakay": (C.c_int, [C.c_void_p, _f, _f, C.c_float]),
    "hpt_set_bsdf_roughplastic": (C.c_int, [C.c_void_p, C.c_float, C.c_float, C.c_int, C.c_float, C.c_int, C.c_int,
                                            _f, _f]),
    "hpt_set_bsdf_marschnerdielectric": (C.c_int, [C.c_void_p, C.c_float, C.c_float, _f, _f, _f]),
    "hpt_set_envmap_rgb": (C.c_int, [C.c_void_p, _f, C.c_int, C.c_int, C.c_float, _f]),
    "hpt_set_sunsky": (C.c_int, [C.c_void_p, _f, C.c_float, C.c_float, C.c_float, C.c_float, C.c_int]),
    "hpt_prepare": (C.c_int, [C.c_void_p]),
    "hpt_get_scene_info": (C.c_int, [C.c_void_p, C.POINTER(SceneInfo)]),
    "hpt_render": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), _f]),
    "hpt_render_device": (C.c_int, [C.c_void_p, C.POINTER(RenderParams), C.c_void_p]),
    "hpt_context_share_scene": (C.c_int, [C.c_void_p, C.c_int, C.POINTER(C.c_void_p)]),
    "hpt_render_multi": (C.c_int, [C.POINTER(C.c_void_p), C.c_int, C.POINTER(RenderParams), _f]),
    "hpt_get_stats": (C.c_int, [C.c_void_p, C.POINTER(Stats)]),
    "hpt_get_film_params": (C.c_int, [C.c_void_p, C.POINTER(FilmParams)]),
    "hpt_write_film": (C.c_int, [C.c_void_p, C.c_char_p, _f, C.c_int, C.c_int, C.POINTER(FilmParams), C.c_char_p,
                                 C.c_int]),
    "hpt_get_hair": (C.c_int64, [C.c_void_p, _f, _u8]),
    "hpt_get_kdtree": (C.c_int, [C.c_void_p, _u32, _i64, _u32, _i64, _f]),
    "hpt_get_pretest_records": (C.c_int, [C.c_void_p, _u32, _i64, _f, _u64]),
    "hpt_get_envmap": (C.c_int, [C.c_void_p, _f, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "hpt_get_marschner_tables": (C.c_int, [C.c_void_p, _f, _f, _f, _f, _f, _f]),
    "hpt_get_roughplastic_params": (C.c_int, [C.c_void_p, _f, _f, C.POINTER(C.c_int)]),
    "hpt_get_camera": (C.c_int, [C.c_void_p, _f, _f, _f]),
    "hpt_sobol_batch": (C.c_int, [C.c_void_p, C.c_int, C.c_int, _u32, _u32, _u32, _u32, _u64, _f]),
    "hpt_env_eval_filtered": (C.c_int, [C.c_void_p, C.c_int, _f, _f, _f, _f]),
    "hpt_get_env_level": (C.c_int, [C.c_void_p, C.c_int, _f, C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    "hpt_camera_batch": (C.c_int, [C.c_void_p, C.c_int, _f, _f, _f, _f, _f]),
    "hpt_trace_batch": (C.c_int, [C.c_void_p, C.c_int, _f, _f, _f, _f, C.c_int, _f, _i32, _f, _u8]),
    "hpt_bsdf_batch": (C.c_int, [C.c_void_p, C.c_int, _f, _f, _f, _f, _f, _f, _f, _f, _u32]),
    "hpt_env_batch": (C.c_int, [C.c_void_p, C.c_int, _f, _f, _f, _f, _f, _f, _f, _f, _f]),
}

_lib = None


def load_library(path: str = None):
    """Load libhairpt.so (raises OSError if it was not built -- no fallback).
    HAIRPT_LIB selects another build of the same library (kernel experiments)."""
    global _lib
    if path is None:
        path = os.environ.get("HAIRPT_LIB") or LIB_PATH
    if _lib is None:
        if not os.path.exists(path):
            raise OSError("libhairpt.so not built at %s (run __graft_entry__.build())" % path)
        lib = C.CDLL(path)
        experiment = path != LIB_PATH
        for name, (res, args) in SIGNATURES.items():
            if experiment and not hasattr(lib, name):
                continue  # an older experiment build: exports added since then stay unbound
            fn = getattr(lib, name)
            fn.restype = res
            fn.argtypes = args
        _lib = lib
    return _lib


def _p(a, t):
    return a.ctypes.data_as(t) if a is not None else None


def _f32(a, n=None):
    a = np.ascontiguousarray(a, dtype=np.float32)
    return a


class HairPTError(RuntimeError):
    """A hairpt call failed: code is the C ABI's negative status (HPT_E*)."""

    def __init__(self, msg, code=None):
        super().__init__(msg)
        self.code = code


def block_deal(width: int, height: int, n_shards: int, weights=None) -> np.ndarray:
    """shard of every 32x32 image block (hpt_block_deal): Hilbert-cyclic, or work-balanced"""
    lib = load_library()
    nb = ((width + 31) // 32) * ((height + 31) // 32)
    out = np.zeros(nb, dtype=np.int32)
    w = None if weights is None else np.ascontiguousarray(weights, dtype=np.float64)
    rc = lib.hpt_block_deal(width, height, n_shards, None if w is None else w.ctypes.data_as(C.POINTER(C.c_double)),
                            out.ctypes.data_as(C.POINTER(C.c_int32)))
    if rc != 0:
        raise HairPTError("hpt_block_deal failed (%d)" % rc, rc)
    return out


class Renderer:
    """One HIP context on one MI355X (the drop-in for a Mitsuba render job)."""

    def __init__(self, device: int = 0, data_dir: str = DATA_DIR, _handle=None):
        self.lib = load_library()
        if _handle is not None:  # share_scene
            self.h = _handle
            return
        h = C.c_void_p()
        rc = self.lib.hpt_context_create(device, C.byref(h))
        if rc != 0:
            raise HairPTError("hpt_context_create(%d) failed (%d): no gfx950 device?" % (device, rc))
        self.h = h
        self._check(self.lib.hpt_set_data_dir(self.h, data_dir.encode()))

    def share_scene(self, device: int) -> "Renderer":
        """a context on `device` rendering this prepared context's scene (parsed, loaded and built
        once, uploaded again: hpt_context_share_scene)"""
        h = C.c_void_p()
        rc = self.lib.hpt_context_share_scene(self.h, device, C.byref(h))
        if rc != 0:  # reported to this thread, not on the (shared, read-only) source context
            raise HairPTError("hairpt error %d: %s" % (rc, self.lib.hpt_last_error(None).decode()), rc)
        return Renderer(device, _handle=h)

    def close(self):
        if getattr(self, "h", None):
            self.lib.hpt_context_destroy(self.h)
            self.h = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def _check(self, rc):
        if rc != 0:
            raise HairPTError("hairpt error %d: %s" % (rc, self.lib.hpt_last_error(self.h).decode()), rc)
        return rc

    # ---- scene ----
    def load_scene_xml(self, path: str, defines: dict | None = None):
        defines = defines or {}
        keys = (C.c_char_p * max(1, len(defines)))(*[k.encode() for k in defines])
        vals = (C.c_char_p * max(1, len(defines)))(*[str(v).encode() for v in defines.values()])
        self._check(self.lib.hpt_load_scene_xml(self.h, path.encode(), len(defines), keys, vals))

    def scene_json(self) -> dict:
        """The parsed scene (hpt_export_scene_json), defaults resolved."""
        import json
        need = C.c_size_t(0)
        self._check(self.lib.hpt_export_scene_json(self.h, None, 0, C.byref(need)))
        buf = C.create_string_buffer(need.value)
        self._check(self.lib.hpt_export_scene_json(self.h, buf, need.value, C.byref(need)))
        return json.loads(buf.value.decode())

    def set_camera(self, to_world, fov_x, width, height, near=1e-2, far=1e4):
        m = _f32(to_world).reshape(16)
        self._check(self.lib.hpt_set_camera(self.h, _p(m, _f), fov_x, width, height, near, far))

    def set_sampler(self, spp):
        self._check(self.lib.hpt_set_sampler(self.h, spp))

    def set_scramble(self, scramble: int):
        self._check(self.lib.hpt_set_sampler_scramble(self.h, scramble))

    def set_traversal_bounds(self, max_leaf_rounds=1 << 18, max_restarts=1024):
        """test hook: lower the per-ray traversal bounds (a ray past them fails the call, code -5)"""
        self._check(self.lib.hpt_set_traversal_bounds(self.h, max_leaf_rounds, max_restarts))

    def set_packet_stack(self, entries=0):
        """test hook: limit the camera packets' stack (0 = the build's depth) to force the overflow path"""
        self._check(self.lib.hpt_set_packet_stack(self.h, entries))

    def block_costs(self, n_blocks: int) -> np.ndarray:
        """path-bounces shaded per image block since the last call (blocks this context owns)"""
        out = np.zeros(n_blocks, dtype=np.uint64)
        self._check(self.lib.hpt_get_block_costs(self.h, out.ctypes.data_as(C.POINTER(C.c_uint64)), n_blocks))
        return out

    def set_block_weights(self, weights=None):
        """work-balanced shard deal from per-block weights (None: the Hilbert-cyclic deal)"""
        if weights is None:
            self._check(self.lib.hpt_set_block_weights(self.h, None, 0))
            return
        w = np.ascontiguousarray(weights, dtype=np.float64)
        self._check(self.lib.hpt_set_block_weights(self.h, w.ctypes.data_as(C.POINTER(C.c_double)), len(w)))

    def clear_schedules(self):
        """forget the recorded bounce schedules: the next render of each wave reads every bounce back"""
        self._check(self.lib.hpt_clear_schedules(self.h))

    def set_integrator(self, max_depth, rr_depth=5, strict_normals=True, hide_emitters=False):
        self._check(self.lib.hpt_set_integrator(self.h, max_depth, rr_depth, int(strict_normals), int(hide_emitters)))

    def set_hair_file(self, path, radius, angle_threshold=1.0, reduction=0.0):
        self._check(self.lib.hpt_set_hair_file(self.h, path.encode(), radius, angle_threshold, None))
        if reduction:
            self._check(self.lib.hpt_set_hair_reduction(self.h, reduction))

    def set_hair_vertices(self, xyz, starts, radius):
        xyz = _f32(xyz).reshape(-1, 3)
        st = np.ascontiguousarray(starts, dtype=np.uint8)
        self._check(self.lib.hpt_set_hair_vertices(self.h, _p(xyz, _f), _p(st, _u8), xyz.shape[0], radius))

    def set_marschner(self, int_ior=1.55, ext_ior=1.0, distribution=1, alpha=0.2, diffuse=(0.5, 0.5, 0.5),
                      specular=(0.5, 0.5, 0.5)):
        d = _f32(diffuse)
        s = _f32(specular)
        self._check(self.lib.hpt_set_bsdf_marschner(self.h, int_ior, ext_ior, distribution, alpha, _p(d, _f), _p(s, _f)))

    def set_kajiyakay(self, kd, ks=(0.2, 0.2, 0.2), exponent=30.0):
        a = _f32(kd)
        b = _f32(ks)
        self._check(self.lib.hpt_set_bsdf_kajiyakay(self.h, _p(a, _f), _p(b, _f), exponent))

    def set_roughplastic(self, int_ior=1.49, ext_ior=1.000277, distribution=0, alpha=0.1, sample_visible=True,
                         nonlinear=False, diffuse=(0.5, 0.5, 0.5), specular=(1.0, 1.0, 1.0)):
        d = _f32(diffuse)
        s = _f32(specular)
        self._check(self.lib.hpt_set_bsdf_roughplastic(self.h, int_ior, ext_ior, distribution, alpha,
                                                       int(bool(sample_visible)), int(bool(nonlinear)),
                                                       _p(d, _f), _p(s, _f)))

    def set_marschnerdielectric(self, int_ior=1.501, ext_ior=1.000277, diffuse=(0.5, 0.5, 0.5),
                                specular_reflectance=(0.1, 0.1, 0.1), specular_transmittance=(0.1, 0.1, 0.1)):
        d, r, t = _f32(diffuse), _f32(specular_reflectance), _f32(specular_transmittance)
        self._check(self.lib.hpt_set_bsdf_marschnerdielectric(self.h, int_ior, ext_ior, _p(d, _f), _p(r, _f),
                                                              _p(t, _f)))

    def set_envmap(self, rgb, scale=1.0):
        rgb = _f32(rgb)
        h, w = rgb.shape[:2]
        self._check(self.lib.hpt_set_envmap_rgb(self.h, _p(rgb, _f), w, h, scale, None))

    def set_sunsky(self, sun_dir, turbidity=3.0, sky_scale=1.0, sun_scale=1.0, sun_radius_scale=1.0, resolution=512):
        d = _f32(sun_dir)
        self._check(self.lib.hpt_set_sunsky(self.h, _p(d, _f), turbidity, sky_scale, sun_scale, sun_radius_scale,
                                            resolution))

    def prepare(self):
        self._check(self.lib.hpt_prepare(self.h))

    def info(self) -> SceneInfo:
        si = SceneInfo()
        self._check(self.lib.hpt_get_scene_info(self.h, C.byref(si)))
        return si

    # ---- render ----
    def render(self, spp_begin=0, spp_end=None, shard=0, n_shards=1, max_wave_paths=0, collect_stats=False,
               film=None) -> np.ndarray:
        si = self.info()
        if spp_end is None:
            spp_end = si.spp
        if film is None:
            film = np.zeros((si.height, si.width, 4), dtype=np.float32)
        p = RenderParams(spp_begin, spp_end, shard, n_shards, max_wave_paths, int(collect_stats))
        self._check(self.lib.hpt_render(self.h, C.byref(p), _p(film, _f)))
        return film

    def render_device(self, device_ptr: int, spp_begin=0, spp_end=None, shard=0, n_shards=1, max_wave_paths=0,
                      collect_stats=False):
        si = self.info()
        if spp_end is None:
            spp_end = si.spp
        p = RenderParams(spp_begin, spp_end, shard, n_shards, max_wave_paths, int(collect_stats))
        self._check(self.lib.hpt_render_device(self.h, C.byref(p), C.c_void_p(device_ptr)))

    @staticmethod
    def render_multi(renderers, spp_begin=0, spp_end=None, max_wave_paths=0, collect_stats=False, film=None):
        """shard g of len(renderers) on renderers[g], films combined on renderers[0]'s device
        (hpt_render_multi); accumulates into film"""
        r0 = renderers[0]
        si = r0.info()
        if spp_end is None:
            spp_end = si.spp
        if film is None:
            film = np.zeros((si.height, si.width, 4), dtype=np.float32)
        hs = (C.c_void_p * len(renderers))(*[r.h for r in renderers])
        p = RenderParams(spp_begin, spp_end, 0, 1, max_wave_paths, int(collect_stats))
        r0._check(r0.lib.hpt_render_multi(hs, len(renderers), C.byref(p), _p(film, _f)))
        return film

    def stats(self) -> Stats:
        s = Stats()
        self._check(self.lib.hpt_get_stats(self.h, C.byref(s)))
        return s

    # ---- exports ----
    def hair(self):
        n = self.lib.hpt_get_hair(self.h, None, None)
        xyz = np.zeros((n, 3), np.float32)
        st = np.zeros(n + 1, np.uint8)
        self.lib.hpt_get_hair(self.h, _p(xyz, _f), _p(st, _u8))
        return xyz, st

    def film_params(self) -> FilmParams:
        p = FilmParams()
        self._check(self.lib.hpt_get_film_params(self.h, C.byref(p)))
        return p

    def write_film(self, path, film, params: FilmParams | None = None) -> str:
        """Develop an accumulated (H, W, 4) film like the scene's ldrfilm / hdrfilm
        and write it; returns the path written (extension fixed by the format)."""
        film = _f32(film)
        h, w = film.shape[:2]
        p = params or self.film_params()
        buf = C.create_string_buffer(4096)
        self._check(self.lib.hpt_write_film(self.h, str(path).encode(), _p(film, _f), w, h, C.byref(p), buf, 4096))
        return buf.value.decode()

    def kdtree(self):
        nn = C.c_int64()
        ni = C.c_int64()
        self._check(self.lib.hpt_get_kdtree(self.h, None, C.byref(nn), None, C.byref(ni), None))
        nodes = np.zeros((nn.value, 2), np.uint32)
        idx = np.zeros(ni.value, np.uint32)
        aabb = np.zeros(6, np.float32)
        self._check(self.lib.hpt_get_kdtree(self.h, _p(nodes, _u32), C.byref(nn), _p(idx, _u32), C.byref(ni),
                                            _p(aabb, _f)))
        return nodes, idx, aabb

    def pretest_records(self):
        """k_trace's 16-byte pre-test records in leaf order ((n, 4) u32: v1 bits, oct axis | pass << 31),
        the radius the unflagged records are tested at and the number of flagged records."""
        n = C.c_int64()
        self._check(self.lib.hpt_get_pretest_records(self.h, None, C.byref(n), None, None))
        rec = np.zeros((n.value, 4), np.uint32)
        radius = C.c_float()
        n_pass = C.c_uint64()
        self._check(self.lib.hpt_get_pretest_records(self.h, _p(rec, _u32), C.byref(n), C.byref(radius),
                                                     C.byref(n_pass)))
        return rec, radius.value, n_pass.value

    def envmap(self):
        w = C.c_int()
        h = C.c_int()
        self._check(self.lib.hpt_get_envmap(self.h, None, C.byref(w), C.byref(h)))
        rgb = np.zeros((h.value, w.value, 3), np.float32)
        self._check(self.lib.hpt_get_envmap(self.h, _p(rgb, _f), C.byref(w), C.byref(h)))
        return rgb

    def camera(self):
        """(sampleToCamera 4x4, dx, dy) as the host built them (perspective.cpp:150-163)."""
        m = np.zeros(16, np.float32)
        dx = np.zeros(3, np.float32)
        dy = np.zeros(3, np.float32)
        self._check(self.lib.hpt_get_camera(self.h, _p(m, _f), _p(dx, _f), _p(dy, _f)))
        return m.reshape(4, 4), dx, dy

    def marschner_tables(self):
        t = [np.zeros((64 * 64, 3), np.float32) for _ in range(3)]
        fdr = np.zeros(1, np.float32)
        tr = np.zeros(100, np.float32)
        sw = np.zeros(1, np.float32)
        self._check(self.lib.hpt_get_marschner_tables(self.h, _p(t[0], _f), _p(t[1], _f), _p(t[2], _f), _p(fdr, _f),
                                                      _p(tr, _f), _p(sw, _f)))
        return t, float(fdr[0]), tr, float(sw[0])

    def roughplastic_params(self):
        """(params dict, external rough-transmittance slice) of the prepared roughplastic BSDF"""
        v = np.zeros(16, np.float32)
        n = C.c_int()
        self._check(self.lib.hpt_get_roughplastic_params(self.h, _p(v, _f), None, C.byref(n)))
        tr = np.zeros(n.value, np.float32)
        self._check(self.lib.hpt_get_roughplastic_params(self.h, None, _p(tr, _f), C.byref(n)))
        keys = ("type", "sample_visible", "nonlinear", "alpha", "exponent", "eta", "inv_eta2", "spec_weight")
        d = {k: float(x) for k, x in zip(keys, v[:8])}
        d.update(diffuse=v[8:11].copy(), specular=v[11:14].copy(), fdr=float(v[14]))
        return d, tr

    # ---- batch kernels ----
    def sobol(self, m, frame, px, py, dim):
        frame, px, py, dim = [np.ascontiguousarray(a, np.uint32) for a in (frame, px, py, dim)]
        n = frame.size
        oi = np.zeros(n, np.uint64)
        ov = np.zeros(n, np.float32)
        self._check(self.lib.hpt_sobol_batch(self.h, m, n, _p(frame, _u32), _p(px, _u32), _p(py, _u32), _p(dim, _u32),
                                             _p(oi, _u64), _p(ov, _f)))
        return oi, ov

    def camera_rays(self, pos):
        """The device camera rays at film positions (n, 2) -> (o, d, mint, maxt)."""
        pos = _f32(pos).reshape(-1, 2)
        n = pos.shape[0]
        o = np.zeros((n, 3), np.float32)
        d = np.zeros((n, 3), np.float32)
        mint = np.zeros(n, np.float32)
        maxt = np.zeros(n, np.float32)
        self._check(self.lib.hpt_camera_batch(self.h, n, _p(pos, _f), _p(o, _f), _p(d, _f), _p(mint, _f),
                                              _p(maxt, _f)))
        return o, d, mint, maxt

    def trace(self, o, d, mint, maxt, shadow=False, tiny_stack=False, packet=False, split=True):
        o = _f32(o).reshape(-1, 3)
        d = _f32(d).reshape(-1, 3)
        n = o.shape[0]
        mint = _f32(np.broadcast_to(mint, (n,)))
        maxt = _f32(np.broadcast_to(maxt, (n,)))
        ot = np.zeros(n, np.float32)
        oiv = np.zeros(n, np.int32)
        op = np.zeros((n, 3), np.float32)
        oh = np.zeros(n, np.uint8)
        self._check(self.lib.hpt_trace_batch(self.h, n, _p(o, _f), _p(d, _f), _p(mint, _f), _p(maxt, _f),
                                             (1 if shadow else 0) | (2 if tiny_stack else 0) | (4 if packet else 0)
                                             | (0 if split else 8),
                                             _p(ot, _f), _p(oiv, _i32), _p(op, _f), _p(oh, _u8)))
        return oh.astype(bool) if shadow else (ot, oiv, op)

    def env_filtered(self, d, rx, ry):
        """evalEnvironment of rays with differentials (EWA over the MIP pyramid)"""
        d, rx, ry = (_f32(a).reshape(-1, 3) for a in (d, rx, ry))
        out = np.zeros_like(d)
        self._check(self.lib.hpt_env_eval_filtered(self.h, d.shape[0], _p(d, _f), _p(rx, _f), _p(ry, _f), _p(out, _f)))
        return out

    def env_levels(self):
        """The environment's MIP pyramid as a list of (h, w, 3) float32 arrays."""
        n = self.lib.hpt_get_env_level(self.h, -1, None, None, None)
        if n < 0:
            self._check(n)
        out = []
        for lv in range(n):
            w, h = C.c_int(), C.c_int()
            self.lib.hpt_get_env_level(self.h, lv, None, C.byref(w), C.byref(h))
            a = np.zeros((h.value, w.value, 3), np.float32)
            self.lib.hpt_get_env_level(self.h, lv, _p(a, _f), None, None)
            out.append(a)
        return out

    def bsdf(self, wi, wo, u):
        wi = _f32(wi).reshape(-1, 3)
        wo = _f32(wo).reshape(-1, 3)
        u = _f32(u).reshape(-1, 2)
        n = wi.shape[0]
        oe = np.zeros((n, 3), np.float32)
        opdf = np.zeros(n, np.float32)
        owo = np.zeros((n, 3), np.float32)
        ow = np.zeros((n, 3), np.float32)
        osp = np.zeros(n, np.float32)
        ot = np.zeros(n, np.uint32)
        self._check(self.lib.hpt_bsdf_batch(self.h, n, _p(wi, _f), _p(wo, _f), _p(u, _f), _p(oe, _f), _p(opdf, _f),
                                            _p(owo, _f), _p(ow, _f), _p(osp, _f), _p(ot, _u32)))
        return oe, opdf, owo, ow, osp, ot

    def env(self, ref_p, u, dq):
        ref_p = _f32(ref_p).reshape(-1, 3)
        u = _f32(u).reshape(-1, 2)
        dq = _f32(dq).reshape(-1, 3)
        n = ref_p.shape[0]
        od = np.zeros((n, 3), np.float32)
        ov = np.zeros((n, 3), np.float32)
        op = np.zeros(n, np.float32)
        odist = np.zeros(n, np.float32)
        oe = np.zeros((n, 3), np.float32)
        oep = np.zeros(n, np.float32)
        self._check(self.lib.hpt_env_batch(self.h, n, _p(ref_p, _f), _p(u, _f), _p(dq, _f), _p(od, _f), _p(ov, _f),
                                           _p(op, _f), _p(odist, _f), _p(oe, _f), _p(oep, _f)))
        return od, ov, op, odist, oe, oep


def develop(film: np.ndarray) -> np.ndarray:
    """RGBW film -> linear RGB (ΣwL / Σw), as the film's develop step (ldrfilm.cpp:300-330)."""
    w = film[..., 3:4]
    out = np.zeros(film.shape[:-1] + (3,), np.float32)
    np.divide(film[..., :3], w, out=out, where=w != 0)
    return out
