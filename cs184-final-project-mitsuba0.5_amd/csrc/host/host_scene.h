/*
 * host_scene.h -- host-side scene model of the MI355X hair path tracer.
 *
 * The host owns everything that is built once per scene: the parsed scene
 * description, the hair vertices (hair.cpp:609-785 loader semantics), the SAH
 * kd-tree over hair segments, the Marschner / Kajiya-Kay precomputations and
 * the environment-map sampling tables.  hpt_capi.cpp uploads the result to
 * HBM as an HptScene (hpt_device.h).
 */
#ifndef HPT_HOST_SCENE_H
#define HPT_HOST_SCENE_H
#include <algorithm>
#include <cstdint>
#include <map>
#include <memory>
#include <string>
#include <vector>

#include "../hpt_device.h"

namespace hpt {

struct Vec3f {
    float x = 0, y = 0, z = 0;
};

/* SAH kd-tree build parameters.  Defaults are HairKDTree's (hair.cpp:130-136,
 * gkdtree.h:731-746) except stopPrims: the reference splits down to single
 * segments; on gfx950 a leaf of up to 6 segments is cheaper to test (fp32
 * pre-test over contiguous records) than the extra dependent node fetches
 * (measured on the furball headline: stopPrims 1 -> 4 +19 % Mpaths/s in round 1;
 * with k_trace at 7 waves/SIMD, 2: 368, 3: 398, 4: 417, 5: 424, 6: 428-432,
 * 8: 426, 10: 414, 12: 400, 16: 369 Mpaths/s).  The scene-level names of scene.cpp:44-78 (kdIntersectionCost,
 * kdTraversalCost, kdEmptySpaceBonus, kdStopPrims, kdMaxDepth, kdClip,
 * kdMaxBadRefines) may be set on the hair shape.  The tree never changes a
 * result (traversal finds the exact closest hit), only the speed. */
struct KDBuildParams {
    float traversalCost = 10.0f;
    float queryCost = 15.0f;
    float emptySpaceBonus = 0.9f;
    int stopPrims = 6;             /* reference HairKDTree: 1 */
    int maxBadRefines = 3;
    int maxDepth = 0;              /* 0 = automatic: min(8 + 1.3 log2 N, 48) */
    int bins = 128;                /* min-max bins */
    bool clip = true;              /* perfect splits via getClippedAABB */
    int clipMinPrims = 0;          /* nodes with fewer primitives split boxes without clipping */
    int exactSweepMax = 256;       /* nodes up to this size sweep every bound event, larger ones bin */
    int threads = 0;               /* 0 = hardware concurrency */
};

/* ---- film development (ldrfilm.cpp:132-190, 300-351; hdrfilm.cpp:205-340, 480-537) ---- */
struct FilmDesc {
    std::string type = "hdrfilm";                  /* sensor.cpp: the default film */
    std::string fileFormat;                        /* "" = the film's default (png / openexr) */
    std::string pixelFormat = "rgb";               /* luminance | rgb (alpha is not recorded) */
    std::string componentFormat = "float16";       /* hdrfilm: float16 | float32 | uint32 */
    std::string tonemapMethod = "gamma";           /* ldrfilm: gamma | reinhard */
    float gamma = -1.0f, exposure = 0.0f, key = 0.18f, burn = 0.0f;
    bool banner = true;
};

/* ---- a procedural 2-D texture: only `checkerboard` (checkerboard.cpp:47-80 over the uv
   transform of Texture2D, texture.cpp:81-121) ---- */
struct TextureDesc {
    std::string type;                              /* "" = a constant colour (no texture) */
    float color0[3] = {0.4f, 0.4f, 0.4f}, color1[3] = {0.2f, 0.2f, 0.2f};
    float uoffset = 0.0f, voffset = 0.0f, uscale = 1.0f, vscale = 1.0f;
};

/* ---- one BSDF instance (constant colours, except a diffuse reflectance texture) ---- */
struct BsdfDesc {
    std::string type = "diffuse";                  /* Shape::configure default (shape.cpp:99-110) */
    float intIOR = 1.5046f, extIOR = 1.000277f;   /* ior.h: bk7 / air defaults */
    std::string distribution = "beckmann";
    float alpha = 0.1f;                            /* microfacet.h:99-140 defaults */
    float diffuse[3] = {0.5f, 0.5f, 0.5f};
    float specular[3] = {0.5f, 0.5f, 0.5f};        /* marschner default 0.5 */
    float transmittance[3] = {0.1f, 0.1f, 0.1f};   /* marschnerdielectric / thindielectric specularTransmittance */
    float exponent = 30.0f;
    bool nonlinear = false;
    bool sampleVisible = true, ensureEnergyConservation = true;
    TextureDesc reflectanceTexture;                /* diffuse: 'reflectance' given as a texture */
    std::vector<BsdfDesc> nested;                  /* twosided: the one or two nested BSDFs */
};

/* ---- a triangle-mesh shape (obj.cpp / rectangle.cpp): loaded by mesh.cpp, rendered by the mesh
   kernel (k_mesh_paths) -- a scene has hair shapes or mesh shapes, not both (hpt_prepare) ---- */
struct MeshShapeDesc {
    std::string type;                              /* obj | rectangle */
    std::string file;                              /* obj: resolved against the scene directory */
    float toWorld[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    bool faceNormals = false, flipNormals = false, flipTexCoords = true; /* obj.cpp:226-240 defaults */
    int bsdf = 0;                                  /* index into SceneDesc::bsdfs */
};

/* ---- one hair shape ---- */
struct HairShapeDesc {
    std::string file;
    float radius = 0.025f, angleThreshold = 1.0f, reduction = 0.0f;
    float toWorld[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    bool hasToWorld = false;
    int bsdf = 0;                                  /* index into SceneDesc::bsdfs */
};

/* ---- parsed scene description (subset of the Mitsuba 0.5 scene schema) ---- */
struct SceneDesc {
    /* integrator (integrator.cpp:190-203, path.cpp) */
    std::string integrator = "path";
    int maxDepth = -1, rrDepth = 5;
    bool strictNormals = false, hideEmitters = false;
    /* sensor (perspective.cpp) */
    float toWorld[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    float fov = 45.0f, nearClip = 1e-2f, farClip = 1e4f;
    std::string fovAxis = "x";
    /* sampler */
    std::string sampler = "sobol";
    int spp = 4;
    uint64_t scramble = 0;                         /* sobol "scramble" property */
    /* film */
    int width = 768, height = 576;
    FilmDesc film;
    std::string rfilter = "tent";
    /* hair shapes (hair.cpp:609-640), each referencing one of bsdfs */
    std::vector<HairShapeDesc> shapes;
    std::vector<MeshShapeDesc> meshes;
    std::vector<BsdfDesc> bsdfs;
    KDBuildParams kd;                              /* from the first hair shape */
    /* emitter */
    std::string emitter = "";
    std::string envFile;
    float envScale = 1.0f;
    float turbidity = 3.0f, skyScale = 1.0f, sunScale = 1.0f, sunRadiusScale = 1.0f;
    float sunDirection[3] = {0, 1, 0};
    bool sunDirectionGiven = false;
    int skyResolution = 512;
    float skyAlbedo[3] = {0.2f, 0.2f, 0.2f}, skyStretch = 1.0f;   /* sky.cpp:222-228 */
    /* date / time / location of the sun when no sunDirection is given (sunmodel.h:223-234) */
    float sunLatitude = 35.6894f, sunLongitude = 139.6917f, sunTimezone = 9.0f;
    int sunYear = 2010, sunMonth = 7, sunDay = 10;
    float sunHour = 15.0f, sunMinute = 0.0f, sunSecond = 0.0f;
    float emitterToWorld[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    std::string sceneDir;
};

/* Parse a Mitsuba scene XML (scenehandler.cpp semantics for the subset used by
 * models/ scenes: <default>, $-substitution, <ref>, nested objects, typed
 * properties, <transform> with matrix/lookat/translate/rotate/scale).
 * Throws std::runtime_error with a message on failure. */
SceneDesc parseSceneXML(const std::string &path, const std::map<std::string, std::string> &defines);
/* the parsed description as JSON (defaults resolved, paths absolute): what hpt_export_scene_json returns */
std::string sceneToJSON(const SceneDesc &d);

/* ---- hair geometry ---- */
struct HairData {
    std::vector<float> xyz;         /* 3 per vertex */
    std::vector<uint8_t> starts;    /* n + 1 entries, last = 1 */
    float radius = 0.025f;          /* radius of a single-shape set (== shapeRadius[0]) */
    /* merged hair shapes: shape k owns vertices [shapeFirst[k], shapeFirst[k+1]) */
    std::vector<uint32_t> shapeFirst{0};
    std::vector<float> shapeRadius;
    uint32_t shapeOf(uint32_t iv) const {
        return (uint32_t) (std::upper_bound(shapeFirst.begin(), shapeFirst.end(), iv) - shapeFirst.begin() - 1);
    }
    float radiusOf(uint32_t iv) const { return shapeRadius.empty() ? radius : shapeRadius[shapeOf(iv)]; }
    size_t nDegenerate = 0, nSkipped = 0;
    size_t vertexCount() const { return xyz.size() / 3; }
};

/* hair.cpp:609-785 (binary + ASCII).  to_world may be null. */
/* the loader's SFMT19937 seeded like Random(seed) (random.cpp:497-526): n outputs of nextULong */
void sfmtULongs(uint64_t seed, size_t n, uint64_t *out);
HairData loadHair(const std::string &path, float radius, float angleThresholdDeg, float reduction,
                  const float *toWorld);

/* ---- kd-tree ---- */
struct KDTreeHost {
    std::vector<HptNode> nodes;
    std::vector<uint32_t> prims;          /* segment index per leaf entry */
    std::vector<HptSegment> segs;         /* per segment (index = segment id) */
    std::vector<HptSegF> leafF;           /* fp32 pre-test records in leaf (prims) order */
    std::vector<HptSegQ> leafQ;           /* the same as 16-byte records (quantised axis) */
    float preRadius = 0.0f;               /* leafQ's pre-test radius (HptSegQ), flagged records aside */
    size_t prePassRecords = 0;            /* records flagged to pass every pre-test (HPT_PRE_PASS) */
    std::vector<HptNode4> nodes4;         /* two-level nodes for the device traversal */
    std::vector<uint32_t> leafTable;      /* (start, end) of leaves too large for an inline ref */
    std::vector<uint32_t> segFirstVertex; /* segment id -> first vertex index */
    float aabbMin[3], aabbMax[3];
    int maxDepthUsed = 0;
    size_t leaves = 0, emptyLeaves = 0;
    double buildSeconds = 0;
};

KDTreeHost buildHairKDTree(const HairData &hair, const KDBuildParams &params);
/* append shape b to a (a's first vertex of b starts a fiber) */
void appendHair(HairData &a, const HairData &b);

/* ---- precomputation ---- */
struct MarschnerHost {
    std::vector<HptF4> table[3];
    std::vector<float> cdf[3], sums[3];
    std::vector<float> trans;      /* 1D slice */
    float fdr = 0, invEta2 = 0, specularSamplingWeight = 0;
    float vR = 0, vTT = 0, vTRT = 0, scaleAngleRad = 0;
    float diffuse[3];
};

bool precomputeMarschner(const BsdfDesc &d, const std::string &dataDir, MarschnerHost &out,
                         std::string &err);
void configureKajiyaKay(const BsdfDesc &d, HptKajiyaKay &out);
void configureMarschnerDielectric(const BsdfDesc &d, HptMarschnerDielectric &out);
void configureThinDielectric(const BsdfDesc &d, HptMarschnerDielectric &out);
void configureDiffuse(const BsdfDesc &d, HptDiffuse &out);

/* roughplastic (roughplastic.cpp:197-299): device parameters + the 1-D external transmittance slice */
struct RoughPlasticHost {
    HptRoughPlastic p{};
    std::vector<float> trans;
};
bool configureRoughPlastic(const BsdfDesc &d, const std::string &dataDir, RoughPlasticHost &out, std::string &err);
/* RoughTransmittance (rtrans.h) for one distribution: the external 1-D slice at (eta, alphaSlice) and
 * Fdr = 1 - internal (1/eta) diffuse transmittance at alphaDiffuse */
bool roughTransmittance(const std::string &dataDir, const std::string &distribution, float eta, float alphaSlice,
                        float alphaDiffuse, std::vector<float> &trans, float &fdr, std::string &err);

struct EnvHost {
    int w = 0, h = 0;
    std::vector<float> rgb;        /* input bitmap (linear RGB) */
    std::vector<HptF4> texel;      /* half-rounded */
    /* MIP pyramid (mipmap.h:155-302): level l is levelW[l] x levelH[l] half-rounded texels at
       mip[levelOff[l] ...]; level 0 == texel.  sizeRatio (mipmap.h:264-266), EWA weight LUT (:296-301) */
    std::vector<HptF4> mip;
    std::vector<int> levelW, levelH, levelOff;
    std::vector<float> ratioX, ratioY;
    float ewaLut[HPT_EWA_LUT] = {};
    std::vector<float> cdfRows, cdfCols, rowWeights;
    std::vector<uint32_t> guideRows, guideCols; /* HptEnvMap::guideRows / guideCols */
    float normalization = 0, scale = 1, pixelSizeX = 0, pixelSizeY = 0;
    float toWorld[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
};

void buildEnvMap(EnvHost &env);                           /* envmap.cpp:244-314 */
void buildEnvMipmap(EnvHost &env);                        /* envmap.cpp:165-182, mipmap.h:155-302 */

/* sunsky (sunsky.cpp): tables extracted from the reference (tools/extract_sunsky_tables.py) */
struct SunSkyTables {
    std::vector<double> hosek;     /* datasetRGB1..3 (3 x 1080), datasetRGBRad1..3 (3 x 120) */
    std::vector<float> cie;        /* CIE 1931 wavelengths, x, y, z (4 x 471) */
    std::vector<float> kOWl, kOAmp, kGWl, kGAmp, kWaWl, kWaAmp, solWl, solAmp;
};
bool loadSunSkyTables(const std::string &dataDir, SunSkyTables &t, std::string &err);
void rasterizeSunSky(const SceneDesc &d, const SunSkyTables &t, EnvHost &env); /* sunsky.cpp:100-225 */
/* pieces exported for the golden-vector tests */
void hosekSkyRGB(const SunSkyTables &t, double turbidity, double albedo, double solarElevation, double theta,
                 double gamma, double out[3]);
void sunRadianceRGB(const SunSkyTables &t, float theta, float turbidity, float rgb[3]);
bool loadEnvFile(const std::string &path, EnvHost &env, std::string &err); /* .hdr / .pfm */

void setupCamera(const SceneDesc &d, HptCamera &cam);      /* perspective.cpp:125-165 */
/* m_sampleToCamera of PerspectiveCameraImpl::configure (perspective.cpp:150-157), row-major,
   built in float exactly as the reference (Transform products + Gauss-Jordan inverse) */
bool cameraSampleToCamera(const SceneDesc &d, float s2c[16]);
float cameraXFov(const SceneDesc &d);                       /* sensor.cpp:237-305 */
void setupTent(float *lut, float &scale);                 /* rfilter.cpp:38-56 */

/* Matrix4x4::invert (matrix.inl:138-190): float Gauss-Jordan with full pivoting, row-major */
bool invertMatrix4(const float src[16], float out[16]);

/* ---- triangle-mesh scenes (mesh.cpp): the C1 shapes and BSDFs, flattened for the device
   (HptMeshScene) ---- */
struct MeshSceneHost {
    std::vector<float> p, n, uv;         /* per vertex, world space */
    std::vector<float> dpdu;             /* per triangle */
    std::vector<HptTri> tris;
    std::vector<HptMeshInfo> meshes;
    std::vector<HptRect> rects;
    std::vector<HptBvhNode> nodes;
    std::vector<uint32_t> prims;
    std::vector<HptMeshBsdf> bsdfs;      /* desc.bsdfs first (same indices), nested records after */
    float aabbMin[3] = {0, 0, 0}, aabbMax[3] = {0, 0, 0};
    uint32_t depth = 0;                  /* BVH depth (levels) */
    size_t vertexCount() const { return p.size() / 3; }
};
/* obj.cpp / trimesh.cpp / rectangle.cpp loading of SceneDesc::meshes, the BSDF records of
   SceneDesc::bsdfs (diffuse, plastic, twosided), the BVH and the enlarged scene bounds.
   Throws std::runtime_error with the reference's message on failure. */
MeshSceneHost buildMeshScene(const SceneDesc &d);
/* fresnelDiffuseReflectance(eta, fast = false) (util.cpp:808-859): adaptive Gauss-Lobatto */
float fresnelDiffuseReflectance(float eta);

/* float <-> IEEE half (round to nearest even) */
uint16_t floatToHalf(float f);
float halfToFloat(uint16_t h);

/* image output (ldrfilm.cpp:300-330 / hdrfilm.cpp:214-227) */
/* film.cpp: ImageBlock (R, G, B, W per pixel) -> developed bitmap -> file */
struct FilmImage {
    int width = 0, height = 0, channels = 0;
    int component = 0;                             /* 0 uint8, 1 float16, 2 float32, 3 uint32 */
    std::vector<uint8_t> bytes;                    /* row-major, top row first */
};
bool checkFilm(FilmDesc &f, std::string &err);    /* validate + resolve defaults (constructors) */
bool developFilm(const float *rgbw, int w, int h, const FilmDesc &f, const std::string &dataDir, FilmImage &out,
                 std::string &err);
/* writes f's format; the extension is replaced by the proper one like the films do;
   returns the path written */
bool writeFilm(const std::string &path, const FilmImage &img, const FilmDesc &f, std::string &written,
               std::string &err);

} // namespace hpt
#endif
