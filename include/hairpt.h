/*
 * hairpt.h -- C ABI of the MI355X hair path tracer (libhairpt.so).
 *
 * This is the drop-in boundary for the reference's hair hot path
 * (ja5087/cs184-final-project-mitsuba0.5).  The reference exposes the path
 * as C++ plugins loaded by dlopen (include/mitsuba/core/cobject.h:99-107,
 * src/libcore/plugin.cpp:71-121) and driven by the `mitsuba` CLI
 * (src/mitsuba/mitsuba.cpp:52-400).  Mitsuba's C++ plugin ABI (boost-typed
 * Properties, ref<> counting) cannot be linked here, so the boundary is
 * re-expressed as plain C entry points: each entry point names the reference
 * interface it replaces.  Conventions:
 *   - every function returns 0 on success and a negative HPT_E* code on
 *     failure; hpt_last_error() holds the message (the reference throws
 *     std::runtime_error through Log(EError, ...));
 *   - all buffers are caller-owned; host pointers unless the name says
 *     "device";
 *   - a context drives one HIP device; calls on one context are not
 *     thread-safe (one context per rank / GPU), except that several threads
 *     may call hpt_context_share_scene on one prepared source at once (it only
 *     reads the source);
 *   - calls that fail before they have a context of their own to report on
 *     (hpt_context_create, hpt_context_share_scene) leave the message for the
 *     calling thread: hpt_last_error(NULL); each such call clears it first, so
 *     after a success it is empty.
 */
#ifndef HAIRPT_H
#define HAIRPT_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define HPT_OK 0
#define HPT_EINVAL -1   /* bad argument / missing scene component          */
#define HPT_EIO -2      /* file could not be read or parsed                */
#define HPT_EDEVICE -3  /* HIP runtime error or no gfx950 device            */
#define HPT_ESTATE -4   /* call order violated (e.g. render before prepare) */
#define HPT_ETRAVERSAL -5 /* a ray hit the kd traversal's leaf-round or kd-restart bound: the
                             result would be unreliable, so the render / trace call fails */

typedef struct hpt_context hpt_context;

/* pass as 'device' to create a host-only context: it parses, loads, builds
   and exports the scene (kd-tree, tables) but cannot render */
#define HPT_HOST_ONLY -1

/* Context lifetime.  Replaces the Scheduler/LocalWorker setup of
   src/mitsuba/mitsuba.cpp:281-329 for one device. */
int hpt_context_create(int device, hpt_context **out);
void hpt_context_destroy(hpt_context *ctx);
const char *hpt_last_error(const hpt_context *ctx);
/* Directory holding sobol/ and microfacet/ data (default: <lib>/../data). */
int hpt_set_data_dir(hpt_context *ctx, const char *dir);

/* Parse a Mitsuba scene XML (src/librender/scenehandler.cpp) with -D style
   defines: integrator "path", sensor "perspective" + sampler "sobol" + film,
   shape "hair", bsdf "marschner"/"kajiyakay"/"roughplastic"/"marschnerdielectric"/"thindielectric"/"diffuse"
   (one per hair shape; several shapes per scene), emitter "sunsky"/"envmap"; or, for a
   triangle-mesh scene (C1, models/teapot), shape "obj"/"rectangle" with bsdf "diffuse" (constant
   or "checkerboard" texture) / "plastic" / "twosided" over those two. */
int hpt_load_scene_xml(hpt_context *ctx, const char *path, int n_defines, const char *const *keys,
                       const char *const *values);
/* Process-wide -D defines, merged under the explicit ones by every later
   hpt_load_scene_xml (replaces the previous table; n_defines = 0 clears it).
   The reference keeps its -D map local to main() (src/mitsuba/mitsuba.cpp:
   143-175) and hands it to SceneHandler (:354); a binding calls this right
   there, so a plugin shim that re-parses the scene file sees the job's defines
   (INTEGRATION.md section 1). */
int hpt_set_default_defines(int n_defines, const char *const *keys, const char *const *values);

/* The parsed scene as JSON: defaults resolved, paths absolute, every shape
   (hair and, for the C1 plumbing scene, obj / rectangle meshes) with its BSDF
   (plastic, twosided, diffuse with a checkerboard texture ...).  Replaces
   reading the SceneHandler's object graph (src/librender/scenehandler.cpp:
   endElement) from C.  With buf == NULL only *needed (bytes incl. the NUL) is
   set. */
int hpt_export_scene_json(hpt_context *ctx, char *buf, size_t capacity, size_t *needed);

/* ---- low-level scene setters (what a Mitsuba plugin shim would call) ---- */
/* PerspectiveCameraImpl (src/sensors/perspective.cpp:108-165); row-major 4x4 */
int hpt_set_camera(hpt_context *ctx, const float to_world[16], float fov_x_deg, int width, int height,
                   float near_clip, float far_clip);
/* SobolSampler sampleCount (src/samplers/sobol.cpp:80-106) */
int hpt_set_sampler(hpt_context *ctx, int sample_count);
/* SobolSampler "scramble" (sobol.cpp:92-102); 0 = unscrambled (the default) */
int hpt_set_sampler_scramble(hpt_context *ctx, uint64_t scramble);
/* Test hook: the hair loader's SFMT19937 (`reduction` culling, hair.cpp:628) seeded like
   Random(seed) (src/libcore/random.cpp:497-526), n outputs of Random::nextULong (:551-553);
   pinned by the reference's known answers for Random(4321) (src/tests/test_random.cpp:434-507) */
int hpt_debug_sfmt(uint64_t seed, uint64_t n, uint64_t *out);
/* Test hook: fresnelDiffuseReflectance(eta, fast = false) (src/libcore/util.cpp:808-859, the
   adaptive Gauss-Lobatto of quad.cpp:287-409) as the mesh path's plastic BSDF configures it
   (plastic.cpp:186-217), n values */
int hpt_debug_fresnel_diffuse(int n, const float *eta, float *out);
/* Test hook (no reference counterpart): lower the per-ray traversal bounds (leaf rounds, kd-restarts;
   defaults and maxima 2^18 and 1024) past which a render or trace call fails with HPT_ETRAVERSAL */
int hpt_set_traversal_bounds(hpt_context *ctx, uint32_t max_leaf_rounds, uint32_t max_restarts);
/* Test hook (no reference counterpart): limit the camera pass's packet stack to `entries` (0 = the
   build's 23; larger values are clamped) so that packets overflow and their rays take the
   per-lane fallback launch -- hits, and so the film, are unchanged */
int hpt_set_packet_stack(hpt_context *ctx, uint32_t entries);
/* Drop the bounce schedules recorded by earlier renders (no reference counterpart: the
   reference has no wavefront).  The next render of each wave of paths then reads every
   bounce's queue length back, as a first render does -- bench.py's first_render_ms */
int hpt_clear_schedules(hpt_context *ctx);
/* MonteCarloIntegrator params (src/librender/integrator.cpp:190-203) */
int hpt_set_integrator(hpt_context *ctx, int max_depth, int rr_depth, int strict_normals, int hide_emitters);
/* HairShape(Properties) (src/shapes/hair.cpp:609-785); to_world may be NULL */
int hpt_set_hair_file(hpt_context *ctx, const char *path, float radius, float angle_threshold_deg,
                      const float *to_world);
/* HairShape "reduction" property (hair.cpp:618-629, 671-673, 768-770) of the hair file set by
   hpt_set_hair_file: each strand is dropped with this probability, drawn from SFMT19937 seeded
   with 5489 like the reference's `new Random()` on Linux, and the radius grows by
   1 / (1 - reduction).  Must be in [0, 1). */
int hpt_set_hair_reduction(hpt_context *ctx, float reduction);
/* HairShape(Stream) equivalent (hair.cpp:787-801): vertices already merged;
   starts_fiber has n_vertices entries (a trailing terminator is implied). */
int hpt_set_hair_vertices(hpt_context *ctx, const float *xyz, const uint8_t *starts_fiber, uint64_t n_vertices,
                          float radius);
/* MarschnerDiffuse(Properties) (src/bsdfs/marschner_diffuse.cpp:113-160, plugin
   "marschner"); distribution 0 = beckmann, 1 = ggx, 2 = phong */
int hpt_set_bsdf_marschner(hpt_context *ctx, float int_ior, float ext_ior, int distribution, float alpha,
                           const float diffuse[3], const float specular[3]);
/* KajiyaKay(Properties) (src/bsdfs/kajiyakay.cpp:60-69) */
int hpt_set_bsdf_kajiyakay(hpt_context *ctx, const float kd[3], const float ks[3], float exponent);
/* RoughPlastic(Properties) (src/bsdfs/roughplastic.cpp:197-227) with constant
   textures; distribution 0 = beckmann, 1 = ggx, 2 = phong (sample_visible is
   forced off for phong, microfacet.h:139-143); diffuse/specular may be NULL
   (defaults 0.5 / 1.0).  The reference's anisotropic case is an error there
   and is not expressible here. */
int hpt_set_bsdf_roughplastic(hpt_context *ctx, float int_ior, float ext_ior, int distribution, float alpha,
                              int sample_visible, int nonlinear, const float diffuse[3], const float specular[3]);
/* MarschnerDielectric(Properties) (src/bsdfs/marschnerdielectric.cpp:147-169);
   NULL colours take the plugin defaults (0.5 / 0.1 / 0.1) */
int hpt_set_bsdf_marschnerdielectric(hpt_context *ctx, float int_ior, float ext_ior, const float diffuse[3],
                                     const float specular_reflectance[3], const float specular_transmittance[3]);
/* EnvironmentMap from a bitmap (src/emitters/envmap.cpp:105-189); rgb is w*h*3
   linear floats, to_world may be NULL */
int hpt_set_envmap_rgb(hpt_context *ctx, const float *rgb, int w, int h, float scale, const float *to_world);
/* SunSkyEmitter (src/emitters/sunsky.cpp:100-240): Hosek-Wilkie sky + Preetham
   sun rasterised into the envmap bitmap (sun_direction given explicitly) */
int hpt_set_sunsky(hpt_context *ctx, const float sun_direction[3], float turbidity, float sky_scale,
                   float sun_scale, float sun_radius_scale, int resolution);

/* Build the hair kd-tree (HairKDTree ctor, hair.cpp:108-159), precompute the
   BSDF / envmap tables and upload the scene to HBM (Scene::preprocess).  A scene whose
   shapes are obj / rectangle meshes (C1) is loaded instead (WavefrontOBJ, obj.cpp:199-349;
   TriMesh::configure, trimesh.cpp:362-386; Rectangle, rectangle.cpp:80-122) into a BVH, and
   hpt_render traces its paths with the mesh kernel (k_mesh_paths); hpt_get_scene_info then
   reports the BVH in its kd_* fields.  A scene mixing hair and meshes is refused (HPT_EINVAL). */
int hpt_prepare(hpt_context *ctx);

typedef struct hpt_scene_info {
    int width, height, spp, max_depth, rr_depth, strict_normals, hide_emitters;
    int bsdf;                      /* first shape's: 0 marschner, 1 kajiyakay, 2 roughplastic,
                                      3 marschnerdielectric, 4 thindielectric, 5 diffuse */
    uint64_t vertices, segments, kd_nodes, kd_indices;
    int kd_depth;
    double kd_build_seconds;
    float aabb_min[3], aabb_max[3];
    float bsphere_center[3], bsphere_radius;
    int n_shapes;                  /* hair shapes (merged into one kd-tree, each with its BSDF) */
} hpt_scene_info;
int hpt_get_scene_info(hpt_context *ctx, hpt_scene_info *out);

typedef struct hpt_render_params {
    int spp_begin, spp_end;        /* render samples [spp_begin, spp_end) of every pixel */
    int shard, n_shards;           /* the 32x32 blocks at positions shard, shard + n_shards, ... of a
                                      Hilbert curve over the block grid (multi-GPU; hpt_capi.cpp blockOrder) */
    uint64_t max_wave_paths;       /* 0 = automatic (HBM-sized waves) */
    int collect_stats;             /* 0 none, 1 per-kernel HIP event timing,
                                      2 timing + traversal counters (slower k_trace variant),
                                      3 HIP event timing of the traversal launches only
                                        (k_trace, k_trace_packet: the roofline's kernels) */
} hpt_render_params;

/* SamplingIntegrator::render/renderBlock + MIPathTracer::Li + ImageBlock::put
   (src/librender/integrator.cpp:95-188, src/integrators/path/path.cpp:119-294,
   include/mitsuba/render/imageblock.h:124-204).  film_rgbw is W*H*4 floats
   (sum of w*L per channel, sum of w) and is ACCUMULATED into. */
int hpt_render(hpt_context *ctx, const hpt_render_params *params, float *film_rgbw);
/* Same, accumulating into a device buffer of W*H float4 on this context's device. */
int hpt_render_device(hpt_context *ctx, const hpt_render_params *params, void *device_film_rgbw);

/* One process, several devices (src/mitsuba/mitsuba.cpp:281-329: the scene is loaded once and
   every worker renders from it).  hpt_context_share_scene makes a context on `device` from a
   prepared context's host-built scene -- the XML is not parsed, the hair not loaded and the
   kd-tree not built again, only uploaded -- and hpt_render_multi renders shard g of n on
   ctxs[g] (on their own threads), combines the films on ctxs[0]'s device (peer copies over
   xGMI, added in shard order: the same sum as adding the n host films) and ACCUMULATES the
   result into film_rgbw.  params->shard / n_shards are ignored.  The contexts must render one
   scene: shares of the same prepared context (a context prepared again renders a scene of its
   own), with equal camera / sampler / integrator settings and equal block weights (the shard
   deal; share_scene copies the source's) -- otherwise HPT_EINVAL before anything renders.  A
   share failure is reported to the calling thread (hpt_last_error(NULL)), never on src. */
int hpt_context_share_scene(hpt_context *src, int device, hpt_context **out);
int hpt_render_multi(hpt_context *const *ctxs, int n, const hpt_render_params *params, float *film_rgbw);

/* Work-balanced shard deal (no reference counterpart; the reference's scheduler hands out blocks
   on demand, src/librender/renderproc.cpp:68-85).  Every render counts, per 32x32 image block it
   owns, the path-bounces it shaded; hpt_get_block_costs copies those counts (by image block
   index by * ceil(W/32) + bx, zero for blocks other shards own) and resets them.  Ranks that add
   their counts up and pass the same totals to hpt_set_block_weights get the same deal: blocks by
   descending weight, each to the shard with the least weight so far (hpt_block_deal, which
   computes it without a context).  No weights (n_blocks 0): the Hilbert-cyclic deal.  Weights
   must be finite and >= 0 (HPT_EINVAL), and a render whose frame has a different number of
   blocks than the weights fails with HPT_EINVAL. */
int hpt_get_block_costs(hpt_context *ctx, uint64_t *costs, int n_blocks);
int hpt_set_block_weights(hpt_context *ctx, const double *weights, int n_blocks);
int hpt_block_deal(int width, int height, int n_shards, const double *weights, int32_t *shard_of_block);

typedef struct hpt_stats {
    double ms_total;               /* host wall time of the render call */
    double ms_camera, ms_trace, ms_primary, ms_shade, ms_post, ms_gather; /* HIP event sums */
    uint64_t trace_launches;
    uint64_t paths, closest_rays, shadow_rays, nodes, prims, bounces;
    uint64_t shadow_unoccluded;    /* shadow rays that reached the emitter */
    uint64_t waves;
    int max_bounces;
    uint64_t prim_exact;           /* segments that passed the fp32 pre-test (fp64 tests run) */
    uint64_t node_slots, prim_slots; /* SIMD lanes occupied by the node / primitive loops
                                        (64 per wave iteration): nodes / node_slots is the
                                        lane utilisation */
    double ms_tail;                /* HIP event sum of k_tail (the frame's last bounces, one launch) */
    uint64_t tail_paths;           /* live paths handed to k_tail */
    double ms_trace_packet;        /* HIP event sum of k_trace_packet (the camera rays, 64-ray packets) */
    uint64_t packet_launches;
    /* the packet pass's traversal counters (counted frames), like the ones above for k_trace */
    uint64_t packet_rays, packet_nodes /* binary-node visits per member lane */, packet_prims, packet_exact;
    uint64_t packet_node_slots, packet_prim_slots; /* 64 per packet step: visits / slots = lane use */
    uint64_t packet_fallbacks;     /* packets whose stack overflowed (their lanes traced alone) */
    /* counted frames: the longest ray of the per-lane traversal (k_trace) in leaf rounds, its most
       kd-restarts, and how many rays restarted at all (the bounds that fail a call with
       HPT_ETRAVERSAL are 2^18 rounds / 1024 restarts) */
    uint64_t max_leaf_rounds, max_restarts, restarted_rays;
    /* counted frames: binary kd-node visits of k_trace (inner nodes entered + leaves, the count of
       rayIntersectHavran, sahkdtree3.h:178-308; `nodes` counts the two-level HptNode4 fetches) */
    uint64_t binary_nodes;
    /* device-side bounce control: waves whose bounces were launched ahead on the schedule of an
       earlier render of the same spp range and shard (no queue length read back per bounce), and
       waves rendered again because a bounce outgrew its schedule (HPT_BOUNCE_AHEAD=0: neither) */
    uint64_t waves_ahead, schedule_misses;
    /* waves whose schedule was launched ahead but did not cover them (the tail declined, or
       bounces ran past it): finished bounce by bounce and their schedule re-recorded */
    uint64_t schedule_extensions;
} hpt_stats;
int hpt_get_stats(hpt_context *ctx, hpt_stats *out);

/* ---- film development (Film::develop) ----
   ldrfilm (src/films/ldrfilm.cpp:132-190, 300-351) / hdrfilm
   (src/films/hdrfilm.cpp:205-340, 480-537) applied to an accumulated
   film_rgbw (as filled by hpt_render). */
#define HPT_FILE_PNG 0
#define HPT_FILE_OPENEXR 1
#define HPT_FILE_RGBE 2
#define HPT_FILE_PFM 3
#define HPT_COMPONENT_FLOAT16 0
#define HPT_COMPONENT_FLOAT32 1
#define HPT_COMPONENT_UINT32 2
typedef struct hpt_film_params {
    int ldr;                       /* 1 ldrfilm, 0 hdrfilm */
    int file_format;               /* HPT_FILE_* (ldrfilm: PNG; JPEG is not supported) */
    int luminance;                 /* pixelFormat: 1 luminance, 0 rgb (no alpha channel on this path) */
    int component_format;          /* hdrfilm: HPT_COMPONENT_* (RGBE / PFM force float32) */
    int reinhard;                  /* ldrfilm tonemapMethod: 0 gamma, 1 reinhard */
    float gamma;                   /* ldrfilm: -1 = sRGB */
    float exposure, key, burn;     /* ldrfilm exposure (gamma method), Reinhard key / burn */
    int banner;                    /* the films' "banner" property (default 1) */
} hpt_film_params;
/* the scene's <film> after hpt_load_scene_xml */
int hpt_get_film_params(hpt_context *ctx, hpt_film_params *out);
/* develop + write; the file extension is replaced by the format's own (.png,
   .exr, .rgbe, .pfm) like the films do.  written (may be NULL) receives the
   path actually written.  ctx is used for the data directory and errors. */
int hpt_write_film(hpt_context *ctx, const char *path, const float *film_rgbw, int width, int height,
                   const hpt_film_params *params, char *written, int written_capacity);

/* ---- exports used by the parity tests ---- */
/* vertex count is returned; pass NULL buffers to query the size */
int64_t hpt_get_hair(hpt_context *ctx, float *xyz, uint8_t *starts_fiber /* n+1 */);
/* nodes: 2 u32 per node; indices: first-vertex index of each leaf entry */
int hpt_get_kdtree(hpt_context *ctx, uint32_t *nodes, int64_t *n_nodes, uint32_t *indices, int64_t *n_indices,
                   float aabb[6]);
/* k_trace's 16-byte pre-test records in leaf order (the order of hpt_get_kdtree's indices): 4 u32
   each -- the first vertex as 3 floats, then the axis oct-encoded (u bits 0-15, v bits 16-30) with
   bit 31 set on a record that passes every pre-test (a fold: its bound exceeds its shape's radius
   by more than 5 %) -- the radius the other records are tested at, and how many are flagged.
   NULL records / radius / n_pass are skipped (query n_records first). */
int hpt_get_pretest_records(hpt_context *ctx, uint32_t *records, int64_t *n_records, float *radius, uint64_t *n_pass);
int hpt_get_envmap(hpt_context *ctx, float *rgb, int *w, int *h);
/* the perspective camera's m_sampleToCamera (row-major 4x4) and near-plane position
   differentials m_dx / m_dy (src/sensors/perspective.cpp:150-163), built in float
   exactly as the reference (Transform products, Matrix4x4::invert Gauss-Jordan) */
int hpt_get_camera(hpt_context *ctx, float sample_to_camera[16], float dx[3], float dy[3]);
int hpt_get_marschner_tables(hpt_context *ctx, float *n_r, float *n_tt, float *n_trt, float *fdr, float *trans100,
                             float *spec_weight);
/* RoughPlastic's configured state (roughplastic.cpp:197-296, rtrans.h): params[16] =
   {type (0 beckmann, 1 ggx, 2 phong), sampleVisible, nonlinear, alpha, phong exponent, eta,
   1/eta^2, specularSamplingWeight, diffuse rgb, specular rgb, Fdr = 1 - internal diffuse
   transmittance, trans size}; trans = the external rough-transmittance slice at (eta, alpha) */
int hpt_get_roughplastic_params(hpt_context *ctx, float *params, float *trans, int *trans_size);

/* ---- per-function batch kernels (host arrays in/out, run on the device) ---- */
/* sobol::look_up + sobol::sampleSingle (src/samplers/sobolseq.h:43-131) */
int hpt_sobol_batch(hpt_context *ctx, int m, int n, const uint32_t *frame, const uint32_t *px, const uint32_t *py,
                    const uint32_t *dim, uint64_t *out_index, float *out_value);
/* PerspectiveCameraImpl::sampleRayDifferential (src/sensors/perspective.cpp:271-290): the
   device's camera ray at film positions pos (2n floats, pixels) -> origin, direction (3n), mint, maxt */
int hpt_camera_batch(hpt_context *ctx, int n, const float *pos, float *out_o, float *out_d, float *out_mint,
                     float *out_maxt);
/* ShapeKDTree::rayIntersect closest (skdtree.cpp:112-141) or shadow (:207-226);
   out_iv is the reference's primitive id (first vertex index of the segment) */
#define HPT_TRACE_SHADOW 1      /* any-hit query (out_hit) instead of closest hit */
#define HPT_TRACE_TINY_STACK 2  /* test hook: 2-entry traversal stack, forces kd-restarts */
#define HPT_TRACE_PACKET 4      /* closest hits through the 64-ray packet traversal (camera pass) */
#define HPT_TRACE_NO_SPLIT 8    /* test hook: no drain splitting (idle lanes wait for their wave's last ray) */
int hpt_trace_batch(hpt_context *ctx, int n, const float *o, const float *d, const float *mint, const float *maxt,
                    int flags, float *out_t, int32_t *out_iv, float *out_p, uint8_t *out_hit);
/* BSDF::eval / pdf / sample for the scene's hair BSDF (local frame) */
int hpt_bsdf_batch(hpt_context *ctx, int n, const float *wi, const float *wo, const float *u, float *out_eval,
                   float *out_pdf, float *out_wo, float *out_weight, float *out_sample_pdf, uint32_t *out_type);
/* EnvironmentMap::sampleDirect (envmap.cpp:516-543) for points ref_p and
   evalEnvironment / pdfDirect (:380-410, :545-556) for directions dq */
int hpt_env_batch(hpt_context *ctx, int n, const float *ref_p, const float *u, const float *dq, float *out_d,
                  float *out_value, float *out_pdf, float *out_dist, float *out_eval, float *out_eval_pdf);
/* evalEnvironment of rays WITH differentials -- camera rays: EWA-filtered MIP lookup
   (envmap.cpp:380-410, mipmap.h:629-834); d, rx, ry are world directions of the ray and
   of its x / y differential rays */
int hpt_env_eval_filtered(hpt_context *ctx, int n, const float *d, const float *rx, const float *ry,
                          float *out_rgb);
/* MIP level `level` of the environment (mipmap.h:155-302: Lanczos-2 downsampled, stored as
   half): width, height and w*h RGB texels (any pointer may be NULL).  Returns the number of
   levels (a level out of range only returns it). */
int hpt_get_env_level(hpt_context *ctx, int level, float *rgb, int *w, int *h);

#ifdef __cplusplus
}
#endif
#endif
