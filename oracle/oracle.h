/*
 * oracle.h -- C API of the CPU restatement ("oracle") of the reference hair
 * path-tracing hot path.
 *
 * TEST INFRASTRUCTURE ONLY.  Only tests/, __graft_entry__.smoke() and the
 * cpu_baseline leg of bench.py may load liboracle*.so.  The product
 * (cs184-final-project-mitsuba0.5_amd/) never links, loads or calls this code.
 *
 * Pinning status:
 *   - GaussLegendre<140> nodes/weights and InterpolatedDistribution1D warps are
 *     pinned against golden vectors produced by compiling the reference's own
 *     headers (src/bsdfs/gausssexylingerie.hpp, InterpolatedDistribution1D.hpp)
 *     with oracle/_ref/Makefile.
 *   - The Sobol sampler is pinned by known answers and (0,2)-stratification
 *     over the reference's own tables.
 *   - Everything else on the path (hair loader incl. SFMT reduction, hair
 *     intersection, Marschner eval / sample, Kajiya-Kay eval, envmap sampling /
 *     eval / pdf / EWA, sunsky, MIP pyramid, camera, MIPathTracer::Li and the
 *     tent splat) is pinned by independent numpy restatements written from the
 *     reference sources (tests/test_independent_pins.py, test_camera.py), not
 *     by the reference binary: it needs Boost/Xerces/... and cannot be built in
 *     this image.  roughplastic eval, thindielectric /
 *     marschnerdielectric sampling and the diffuse BSDF are pinned the same way;
 *     roughplastic sampling by a chi-square test (tests/test_oracle_bsdf.py).
 */
#ifndef HAIRPT_ORACLE_H
#define HAIRPT_ORACLE_H
#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

typedef struct orc_scene orc_scene;

orc_scene *orc_scene_create(void);
void orc_scene_destroy(orc_scene *s);
const char *orc_last_error(orc_scene *s);

/* Sobol tables (src/samplers/sobolseq.cpp data): 1024x52 u32, rows x 52 u64 */
int orc_set_sobol(orc_scene *s, const uint32_t *m32, const uint64_t *vdc, int vdc_rows,
                  const uint64_t *vdc_inv, int inv_rows);
/* perspective.cpp:125-165: toWorld row-major 4x4, x field of view in degrees */
/* sobol.cpp:92-102: the sampler's raw "scramble" property (TEA applied inside) */
int orc_set_sobol_scramble(orc_scene *s, uint64_t scramble);
int orc_set_camera(orc_scene *s, const float to_world[16], float fov_x_deg, int width,
                   int height, float near_clip, float far_clip);
/* m_sampleToCamera (row-major, perspective.cpp:150-157: float Transform products and the
   Gauss-Jordan inverse of matrix.inl:138-190) and the near-plane differentials m_dx / m_dy
   (:160-163) */
int orc_get_camera(orc_scene *s, float sample_to_camera[16], float dx[3], float dy[3]);
/* hair.cpp:609-785 loader restatement (BINARY_HAIR or ASCII); to_world may be NULL.
   Each call adds one HairShape (vertices appended after the previous shapes'),
   with the default 0.5 diffuse BSDF; the orc_set_<bsdf> calls below set the
   BSDF of the most recently added shape. */
int orc_load_hair(orc_scene *s, const char *path, float radius, float angle_threshold_deg,
                  const float *to_world);
/* same with HairShape's "reduction" (hair.cpp:618-629, 671-673, 768-770): strands dropped by
   SFMT19937 draws seeded with 5489 (Random() on Linux, random.cpp:473-489) */
int orc_load_hair_reduced(orc_scene *s, const char *path, float radius, float angle_threshold_deg,
                          float reduction, const float *to_world);
int64_t orc_hair_vertex_count(orc_scene *s);
int orc_hair_get(orc_scene *s, float *xyz, uint8_t *starts_fiber /* n+1 */);
/* kd-tree produced by the product's host builder (8-byte nodes: see DESIGN.md),
   indices = first-vertex index of each referenced segment */
int orc_set_kdtree(orc_scene *s, const uint32_t *nodes, int64_t n_nodes,
                   const uint32_t *indices, int64_t n_indices);
/* hair AABB as computed by the restated HairKDTree::getAABB union (hair.cpp:349-378) */
int orc_hair_aabb(orc_scene *s, float out_min[3], float out_max[3]);

/* marschner_diffuse.cpp: eta = intIOR/extIOR, distribution 0=beckmann 1=ggx 2=phong */
int orc_set_marschner(orc_scene *s, float eta, int distribution, float alpha,
                      const float diffuse[3], const float specular[3],
                      const char *microfacet_dat_dir);
/* kajiyakay.cpp */
int orc_set_kajiyakay(orc_scene *s, const float kd[3], const float ks[3], float exponent);
/* roughplastic.cpp (constant textures): eta = intIOR/extIOR, distribution 0=beckmann 1=ggx 2=phong */
int orc_set_roughplastic(orc_scene *s, float eta, int distribution, float alpha, int sample_visible,
                         int nonlinear, const float diffuse[3], const float specular[3],
                         const char *microfacet_dat_dir);
/* marschnerdielectric.cpp: eta = intIOR/extIOR */
int orc_set_marschnerdielectric(orc_scene *s, float eta, const float diffuse[3], const float spec_r[3],
                                const float spec_t[3]);
/* thindielectric.cpp / diffuse.cpp */
int orc_set_thindielectric(orc_scene *s, float eta, const float spec_r[3], const float spec_t[3]);
int orc_set_diffuse(orc_scene *s, const float reflectance[3]);
/* ---- C1 "teapot" plumbing scene (CPU path only; oracle/mesh_bsdf.h, mesh_geom.h) ----
   orc_new_bsdf appends a BSDF (default 0.5 diffuse) and returns its index; the orc_set_*
   calls configure the last one.  orc_set_twosided nests copies of two earlier BSDFs
   (nested1 < 0: nested0 on both sides).  Mesh shapes reference BSDFs by index. */
int orc_new_bsdf(orc_scene *s);
/* diffuse.cpp with a checkerboard reflectance (checkerboard.cpp, texture.cpp:81-121) */
int orc_set_diffuse_checkerboard(orc_scene *s, const float color0[3], const float color1[3], float uoffset,
                                 float voffset, float uscale, float vscale);
/* plastic.cpp (SmoothPlastic, constant reflectances): eta = intIOR/extIOR */
int orc_set_plastic(orc_scene *s, float eta, int nonlinear, const float diffuse[3], const float specular[3],
                    int ensure_energy_conservation);
int orc_set_twosided(orc_scene *s, int nested0, int nested1);
/* obj.cpp WavefrontOBJ (to_world row-major, may be NULL) / rectangle.cpp */
int orc_add_obj(orc_scene *s, const char *path, const float *to_world, int face_normals, int flip_normals,
                int flip_tex_coords, int bsdf);
int orc_add_rectangle(orc_scene *s, const float *to_world, int flip_normals, int bsdf);
int orc_mesh_info(orc_scene *s, int64_t *out /* meshes, triangles, vertices, rectangles */);
void orc_bsdf_eval_uv(orc_scene *s, int n, const float *wi, const float *wo, const float *uv, float *out_rgb,
                      float *out_pdf);
/* util.cpp:814-859 with fast = false */
float orc_fresnel_diffuse_reflectance(float eta);
/* closest hit over the whole scene: t (inf on miss), shading normal, uv, bsdf index (-1 on miss) */
void orc_trace_scene(orc_scene *s, int n, const float *o, const float *d, float *out_t, float *out_n,
                     float *out_uv, int32_t *out_bsdf);

/* envmap.cpp: linear RGB float bitmap (w x h x 3), to_world may be NULL */
int orc_set_envmap(orc_scene *s, const float *rgb, int w, int h, float scale,
                   const float *to_world);
int orc_set_integrator(orc_scene *s, int max_depth, int rr_depth, int strict_normals,
                       int hide_emitters);
/* SobolSampler sampleCount: scales the primary ray differentials (integrator.cpp:143) */
int orc_set_sample_count(orc_scene *s, int spp);
int orc_prepare(orc_scene *s);

/* The sunsky emitter's lat-long bitmap (sunsky.cpp:100-240, sky.cpp, skymodel.cpp,
   sunmodel.h), restated in oracle/sunsky_ref.cpp: resolution x resolution/2 RGB floats.
   sunDirection given, emitter toWorld identity.  data_dir = the package's data/sunsky. */
int orc_rasterize_sunsky(const char *data_dir, const float sun_dir[3], float turbidity, float albedo,
                         float stretch, float sky_scale, float sun_scale, float sun_radius_scale, int resolution,
                         float *rgb);

/* Render samples [spp_begin, spp_end) of every pixel; film_rgbw = W*H*4 floats
   (sum of w*L and sum of w, like the reference's RGBAW image block minus A). */
int orc_render(orc_scene *s, int spp_begin, int spp_end, int n_threads, float *film_rgbw,
               uint64_t *stats /* [8] or NULL */);
/* Same, restricted to pixels whose 32x32 block satisfies (block % n_shards)==shard. */
int orc_render_shard(orc_scene *s, int spp_begin, int spp_end, int n_threads, int shard,
                     int n_shards, float *film_rgbw, uint64_t *stats);

/* ---- fine-grained entry points for unit parity tests ---- */
/* sobolseq.h:43-58 + :99-131; index from look_up when m>1, value per dim */
void orc_sobol_lookup(orc_scene *s, int m, int n, const uint32_t *frame, const uint32_t *px,
                      const uint32_t *py, uint64_t *out_index);
void orc_sobol_sample(orc_scene *s, int n, const uint64_t *index, const uint32_t *dim,
                      float *out);
/* perspective.cpp:271-298 */
void orc_camera_rays(orc_scene *s, int n, const float *sample_pos /* 2n */, float *o /* 3n */,
                     float *d /* 3n */, float *mint, float *maxt);
/* ShapeKDTree::rayIntersect (closest) over the hair kd-tree; mint==1e-4 => adaptive eps.
   out_t = inf on miss; out_iv = first vertex of hit segment (or -1); out_p = hit point. */
void orc_trace_closest(orc_scene *s, int n, const float *o, const float *d, const float *mint,
                       const float *maxt, float *out_t, int32_t *out_iv, float *out_p,
                       int brute_force);
void orc_trace_shadow(orc_scene *s, int n, const float *o, const float *d, const float *mint,
                      const float *maxt, uint8_t *out_hit, int brute_force);
/* BSDF batch: wi, wo local (3n). eval -> rgb (3n), pdf (n) */
void orc_bsdf_eval(orc_scene *s, int n, const float *wi, const float *wo, float *out_rgb,
                   float *out_pdf);
/* sample: wi (3n), u (2n) -> wo (3n), weight rgb (3n), pdf (n), sampled type (n) */
void orc_bsdf_sample(orc_scene *s, int n, const float *wi, const float *u, float *out_wo,
                     float *out_weight, float *out_pdf, uint32_t *out_type);
/* Marschner precomputed tables: 3 lobes x 64 x 64 x RGB */
int orc_marschner_tables(orc_scene *s, float *nR, float *nTT, float *nTRT, float *out_fdr,
                         float *out_trans100, float *out_spec_weight);
/* Gauss-Legendre<140> restatement (gausssexylingerie.hpp) */
void orc_gauss_legendre140(float *points, float *weights);
/* OracleSfmt seeded like Random(seed): n outputs of nextULong */
void orc_sfmt(uint64_t seed, int n, uint64_t *out);
/* InterpolatedDistribution1D restatement over 'weights' (size x ndist) */
void orc_idist_warp(const float *weights, int size, int ndist, int n, const float *dist,
                    const float *u, int *out_x, float *out_u, float *out_pdf, float *out_sum);
/* envmap: direct sampling and pdf (world directions) */
void orc_env_sample(orc_scene *s, int n, const float *ref_p, const float *u, float *out_d,
                    float *out_value, float *out_pdf, float *out_dist);
void orc_env_eval(orc_scene *s, int n, const float *d, float *out_rgb, float *out_pdf);
/* evalEnvironment of rays with differentials: EWA over the MIP pyramid (envmap.cpp:380-410,
   mipmap.h:155-302, 629-834) */
void orc_env_eval_filtered(orc_scene *s, int n, const float *d, const float *rx, const float *ry, float *out_rgb);
/* MIP level of the environment (w*h RGB); returns the number of levels */
int orc_env_level(orc_scene *s, int level, float *rgb, int *w, int *h);
/* Full path radiance for one camera sample (debug / unit parity) */
void orc_trace_paths(orc_scene *s, int n, const uint32_t *px, const uint32_t *py,
                     const uint32_t *frame, float *out_rgb, float *out_pos, int32_t *out_depth);

#ifdef __cplusplus
}
#endif
#endif
