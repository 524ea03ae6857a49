/*
 * hpt_capi.cpp -- the C ABI (include/hairpt.h) and the wavefront driver.
 *
 * The driver replaces SamplingIntegrator::render / BlockedRenderProcess
 * (src/librender/integrator.cpp:95-188, renderproc.cpp:26-145): instead of
 * one CPU worker per 32x32 block it runs every sample of every owned block
 * as one lane of a wave of paths resident in HBM, bouncing the whole wave
 * through k_shade -> k_trace -> k_post until its queue drains, then gathers
 * the wave into the film.  Waves are sized to HBM (hundreds of bytes per
 * path), so a 512x512x256 frame is a single wave on MI355X.
 */
#include <dlfcn.h>

#include <hip/hip_runtime.h>

#include <algorithm>
#include <array>
#include <atomic>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <map>
#include <mutex>
#include <thread>
#include <stdexcept>
#include <string>
#include <vector>

#include "../../include/hairpt.h"
#include "host/host_scene.h"
#include "hpt_device.h"
#include "kernels/hpt_kernels.h"

using namespace hpt;

struct DevBuf {
    void *p = nullptr;
    size_t bytes = 0;
};

/* live paths below which a frame's remaining bounces run as one k_tail
   launch (HPT_TAIL_PATHS overrides; 0 keeps the per-bounce launches) */
static uint32_t defaultTailPaths() {
    const char *v = std::getenv("HPT_TAIL_PATHS");
    return v ? (uint32_t) std::strtoul(v, nullptr, 10) : (1u << 17);
}

/* camera rays traced as 64-ray packets (k_trace_packet); HPT_PACKETS=0 traces them one per lane */
static bool defaultPackets() {
    const char *v = std::getenv("HPT_PACKETS");
    return v ? std::atoi(v) != 0 : true;
}

/* device-side bounce control (launch a wave's bounces ahead without reading queue lengths
   back); HPT_BOUNCE_AHEAD=0 reads every bounce's queue length on the host */
static bool defaultBounceAhead() {
    const char *v = std::getenv("HPT_BOUNCE_AHEAD");
    return v ? std::atoi(v) != 0 : true;
}

/* the bounce schedule of a wave of paths: the shade-queue length of each wavefront bounce,
   and whether a k_tail launch took the rest */
struct BounceSchedule {
    std::vector<uint32_t> shade;
    bool tail = false;
};

/* test hook: HPT_SCHEDULE_TEST=1 records schedules with half the queue lengths (the bounces
   launched ahead outgrow their grids: the wave is rendered again), =2 ends them one wavefront
   bounce early (the tail launched ahead finds too many live paths and leaves the bounce to
   k_shade: the host goes on bounce by bounce) */
static int scheduleTestHook() {
    const char *v = std::getenv("HPT_SCHEDULE_TEST");
    return v ? std::atoi(v) : 0;
}

struct hpt_context {
    int device = 0;
    uint32_t tailPaths = defaultTailPaths();
    bool bounceAhead = defaultBounceAhead();
    int scheduleTest = scheduleTestHook();
    /* schedules of the waves rendered since the last prepare, by (spp begin, spp count,
       shard, shards): a repeated wave launches its bounces ahead on that schedule */
    std::map<std::array<int64_t, 4>, BounceSchedule> schedules;
    uint32_t maxLeafRounds = HPT_MAX_LEAF_ROUNDS, maxRestarts = HPT_MAX_RESTARTS; /* traversal bounds */
    uint32_t packetStack = 0;      /* 0 = the kernel's packet stack depth */
    bool packets = defaultPackets();
    hipStream_t stream = nullptr;
    uint32_t *hostCnt = nullptr; /* pinned copy of the counter block */
    std::vector<uint8_t> scShadow; /* the HptScene last copied to scDev */
    std::string err;
    std::string dataDir;
    SceneDesc desc;
    bool haveCamera = false, haveHair = false, haveBSDF = false, haveEnv = false, prepared = false;
    bool hairFromFile = false;     /* desc.shapes are loaded from files at prepare */
    HairData hair;                 /* every hair shape, merged */
    KDTreeHost tree;
    /* a triangle-mesh scene (C1: obj / rectangle shapes, no hair): mesh.cpp's arrays and their
       device view; k_mesh_paths renders it */
    bool meshScene = false;
    MeshSceneHost mesh;
    HptMeshScene ms{};
    /* per BSDF of desc.bsdfs: host tables and the device record */
    std::vector<MarschnerHost> mar;
    std::vector<RoughPlasticHost> rp;
    std::vector<HptBsdf> bsdfRec;
    EnvHost env;
    bool envFromSunsky = false;
    SunSkyTables sunsky;
    std::vector<uint32_t> sobol32;
    std::vector<uint64_t> vdc, vdcInv;
    HptScene sc;
    HptScene *scDev = nullptr;     /* device copy of sc (kernels that read the scene through a pointer) */
    std::vector<DevBuf> sceneBufs;
    /* wave buffers */
    uint64_t capacity = 0;
    std::vector<DevBuf> waveBufs;
    HptPaths P;
    /* rays of the bounce; paths to shade by bounce parity (shadeQ[p] is post's output for p ^ 1) */
    uint32_t *qTrace = nullptr, *qShadow = nullptr, *qShade[2] = {nullptr, nullptr};
    uint32_t *counters = nullptr;
    uint64_t *dstats = nullptr;
    float4 *partial = nullptr;     /* film splat partials: slots x 9 (k_splat -> k_gather) */
    uint64_t partialSlots = 0;
    /* block ownership of the last render call's shard (blockOf / localOf of HptWave) */
    uint32_t *dBlockOf = nullptr;
    int32_t *dLocalOf = nullptr;
    int ownW = -1, ownH = -1, ownShard = -1, ownShards = -1, ownCap = 0, ownLocal = 0;
    uint64_t ownWeights = 0;            /* weightsVersion the ownership tables were dealt with */
    std::vector<uint32_t> ownBlocks;    /* the image blocks of dBlockOf, on the host */
    uint32_t *dBlockCost = nullptr;     /* path-bounces shaded per owned block (HptPaths::blockCost) */
    std::vector<double> blockWeights;   /* hpt_set_block_weights (empty: Hilbert-cyclic deal) */
    uint64_t weightsVersion = 0;
    /* the prepared scene this context renders: a process-unique number given by each successful
       hpt_prepare and copied by hpt_context_share_scene, so hpt_render_multi can refuse contexts
       that would render different scenes into one film (0: not prepared) */
    uint64_t sceneId = 0;
    hpt_stats stats;
    std::vector<hipEvent_t> evPool;
    /* hpt_render_multi: this context's shard film, and (on the receiving context) the staging
       buffer the other devices' films are copied into */
    float4 *mfilm = nullptr, *mstage = nullptr;
    size_t mfilmPixels = 0, mstagePixels = 0;
    std::vector<hipStream_t> peerStreams; /* one copy stream (and its done event) per peer film */
    std::vector<hipEvent_t> peerEvents;
};

namespace {
/* HptBsdf::kind / hpt_scene_info::bsdf numbering */
int bsdfKindOf(const std::string &b) {
    if (b == "marschner") return HPT_BSDF_MARSCHNER;
    if (b == "kajiyakay") return HPT_BSDF_KAJIYAKAY;
    if (b == "roughplastic") return HPT_BSDF_ROUGHPLASTIC;
    if (b == "marschnerdielectric") return HPT_BSDF_MARSCHNERDIELECTRIC;
    if (b == "thindielectric") return HPT_BSDF_THINDIELECTRIC;
    if (b == "diffuse") return HPT_BSDF_DIFFUSE;
    return -1;
}
/* the low-level setters describe a single BSDF used by every shape */
BsdfDesc &singleBsdf(SceneDesc &d, const char *type) {
    d.bsdfs.assign(1, BsdfDesc());
    for (auto &h : d.shapes) h.bsdf = 0;
    d.bsdfs[0].type = type;
    return d.bsdfs[0];
}

/* errors of calls that have no context of their own to report on (hpt_context_create,
   hpt_context_share_scene): per calling thread, read with hpt_last_error(NULL) */
thread_local std::string tlsErr;

int setErr(hpt_context *c, int code, const std::string &m) {
    if (c) c->err = m;
    else tlsErr = m;
    return code;
}

#define HIPCHK(ctx, expr)                                                                                   \
    do {                                                                                                    \
        hipError_t _e = (expr);                                                                             \
        if (_e != hipSuccess)                                                                               \
            return setErr(ctx, HPT_EDEVICE, std::string(#expr) + ": " + hipGetErrorString(_e));            \
    } while (0)

std::string defaultDataDir() {
    Dl_info info;
    if (dladdr((void *) &defaultDataDir, &info) && info.dli_fname) {
        std::string p = info.dli_fname;
        size_t s = p.find_last_of('/');
        std::string dir = s == std::string::npos ? "." : p.substr(0, s);
        return dir + "/../data";
    }
    return "data";
}

template <typename T> bool readFile(const std::string &path, std::vector<T> &out) {
    std::ifstream f(path, std::ios::binary | std::ios::ate);
    if (!f) return false;
    size_t n = (size_t) f.tellg();
    f.seekg(0);
    out.resize(n / sizeof(T));
    f.read((char *) out.data(), (std::streamsize) (out.size() * sizeof(T)));
    return (bool) f;
}

int upload(hpt_context *c, const void *src, size_t bytes, const void **dst) {
    if (c->device == HPT_HOST_ONLY) { /* keep host pointers: nothing leaves the host */
        *dst = src;
        return HPT_OK;
    }
    DevBuf b;
    b.bytes = std::max<size_t>(bytes, 16);
    HIPCHK(c, hipMalloc(&b.p, b.bytes));
    if (bytes) HIPCHK(c, hipMemcpy(b.p, src, bytes, hipMemcpyHostToDevice));
    c->sceneBufs.push_back(b);
    *dst = b.p;
    return HPT_OK;
}

void freeBufs(std::vector<DevBuf> &v) {
    for (auto &b : v)
        if (b.p) (void) hipFree(b.p);
    v.clear();
}

int ensureWave(hpt_context *c, uint64_t n) {
    if (n <= c->capacity) return HPT_OK;
    freeBufs(c->waveBufs);
    c->capacity = 0;
    auto alloc = [&](size_t bytes, void **p) -> int {
        DevBuf b;
        b.bytes = bytes;
        HIPCHK(c, hipMalloc(&b.p, bytes));
        c->waveBufs.push_back(b);
        *p = b.p;
        return HPT_OK;
    };
    int r = 0;
    r |= alloc(n * 16, (void **) &c->P.ro);
    r |= alloc(n * 16, (void **) &c->P.rd);
    r |= alloc(n * 8, (void **) &c->P.pos);
    r |= alloc(n * 8, (void **) &c->P.sobol);
    r |= alloc(n * 4, (void **) &c->P.state);
    r |= alloc(n * 16, (void **) &c->P.thr);
    r |= alloc(n * 16, (void **) &c->P.li);
    r |= alloc(n * 4, (void **) &c->P.hit);
    r |= alloc(n * 4, (void **) &c->P.hitQ);
    r |= alloc(n * 4, (void **) &c->P.hitS);
    r |= alloc(n * 64, (void **) &c->P.postRec);
    r |= alloc(n * 48, (void **) &c->P.shadowRec);
    r |= alloc(n * 48, (void **) &c->P.shadeRec);
    r |= alloc(n * 16, (void **) &c->P.bw);
    r |= alloc(n * 16, (void **) &c->P.sdir);
    r |= alloc(n * 16, (void **) &c->P.scontrib);
    r |= alloc(n * 4, (void **) &c->qTrace);
    r |= alloc(n * 4, (void **) &c->qShadow);
    r |= alloc(n * 4, (void **) &c->qShade[0]);
    r |= alloc(n * 4, (void **) &c->qShade[1]);
    r |= alloc(HPT_COUNTER_WORDS * 4, (void **) &c->counters);
    r |= alloc(2 * 24 * 8, (void **) &c->dstats); /* the counters, and a snapshot at the start of a wave */
    if (r) return HPT_EDEVICE;
    c->capacity = n;
    return HPT_OK;
}

/* the traversal-bound fault word (HptScene::fault): cleared before a call's
   launches, read after them; a set bit fails the call */
int clearFault(hpt_context *c) {
    HIPCHK(c, hipMemsetAsync(c->sc.fault, 0, 4, c->stream));
    return HPT_OK;
}
int checkFault(hpt_context *c) {
    uint32_t f = 0;
    HIPCHK(c, hipMemcpyAsync(&f, c->sc.fault, 4, hipMemcpyDeviceToHost, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    if (f & HPT_FAULT_LEAVES)
        return setErr(c, HPT_ETRAVERSAL, "kd-tree traversal exceeded 2^18 leaf rounds for a ray (malformed tree?)");
    if (f & HPT_FAULT_RESTARTS)
        return setErr(c, HPT_ETRAVERSAL, "kd-tree traversal exceeded its kd-restart bound for a ray");
    return HPT_OK;
}

hipEvent_t takeEvent(hpt_context *c, size_t &used) {
    if (used >= c->evPool.size()) {
        hipEvent_t e;
        (void) hipEventCreate(&e);
        c->evPool.push_back(e);
    }
    return c->evPool[used++];
}

} // namespace

extern "C" {

int hpt_context_create(int device, hpt_context **out) {
    tlsErr.clear(); /* hpt_last_error(NULL) describes this call only */
    if (!out) return HPT_EINVAL;
    *out = nullptr;
    if (device == HPT_HOST_ONLY) {
        /* host-only context: parses, loads, builds and exports the scene
           (kd-tree, tables) for inspection; every render / batch call fails */
        hpt_context *c = new hpt_context();
        c->device = HPT_HOST_ONLY;
        c->dataDir = defaultDataDir();
        std::memset(&c->sc, 0, sizeof(c->sc));
        std::memset(&c->stats, 0, sizeof(c->stats));
        *out = c;
        return HPT_OK;
    }
    int n = 0;
    if (hipGetDeviceCount(&n) != hipSuccess || n <= 0) return setErr(nullptr, HPT_EDEVICE, "no HIP device");
    if (device < 0 || device >= n)
        return setErr(nullptr, HPT_EINVAL, "device " + std::to_string(device) + " of " + std::to_string(n));
    if (hipSetDevice(device) != hipSuccess) return setErr(nullptr, HPT_EDEVICE, "hipSetDevice failed");
    hipDeviceProp_t prop;
    if (hipGetDeviceProperties(&prop, device) != hipSuccess)
        return setErr(nullptr, HPT_EDEVICE, "hipGetDeviceProperties failed");
    if (std::strncmp(prop.gcnArchName, "gfx950", 6) != 0)
        return setErr(nullptr, HPT_EDEVICE, std::string("not a gfx950 device: ") + prop.gcnArchName);
    hpt_context *c = new hpt_context();
    c->device = device;
    if (hipStreamCreateWithFlags(&c->stream, hipStreamNonBlocking) != hipSuccess ||
        hipHostMalloc((void **) &c->hostCnt, HPT_Q_COUNT * 4, hipHostMallocDefault) != hipSuccess) {
        delete c;
        return setErr(nullptr, HPT_EDEVICE, "stream / pinned counter allocation failed");
    }
    c->dataDir = defaultDataDir();
    std::memset(&c->sc, 0, sizeof(c->sc));
    std::memset(&c->stats, 0, sizeof(c->stats));
    *out = c;
    return HPT_OK;
}

void hpt_context_destroy(hpt_context *c) {
    if (!c) return;
    if (c->device == HPT_HOST_ONLY) {
        delete c;
        return;
    }
    (void) hipSetDevice(c->device);
    (void) hipStreamSynchronize(c->stream);
    freeBufs(c->sceneBufs);
    freeBufs(c->waveBufs);
    if (c->partial) (void) hipFree(c->partial);
    if (c->dBlockOf) (void) hipFree(c->dBlockOf);
    if (c->dLocalOf) (void) hipFree(c->dLocalOf);
    if (c->dBlockCost) (void) hipFree(c->dBlockCost);
    if (c->scDev) (void) hipFree(c->scDev);
    if (c->mfilm) (void) hipFree(c->mfilm);
    if (c->mstage) (void) hipFree(c->mstage);
    for (auto e : c->evPool) (void) hipEventDestroy(e);
    for (auto e : c->peerEvents) (void) hipEventDestroy(e);
    for (auto ps : c->peerStreams) (void) hipStreamDestroy(ps);
    (void) hipHostFree(c->hostCnt);
    (void) hipStreamDestroy(c->stream);
    delete c;
}

const char *hpt_last_error(const hpt_context *c) {
    if (c) return c->err.c_str();
    return tlsErr.empty() ? "null context" : tlsErr.c_str();
}

int hpt_set_data_dir(hpt_context *c, const char *dir) {
    if (!c || !dir) return HPT_EINVAL;
    c->dataDir = dir;
    return HPT_OK;
}

/* the process-wide -D table (hpt_set_default_defines) */
static std::mutex gDefinesMutex;
static std::map<std::string, std::string> gDefaultDefines;

int hpt_set_default_defines(int n_defines, const char *const *keys, const char *const *values) {
    if (n_defines < 0 || (n_defines > 0 && (!keys || !values))) return HPT_EINVAL;
    for (int i = 0; i < n_defines; ++i)
        if (!keys[i] || !values[i]) return HPT_EINVAL;
    std::lock_guard<std::mutex> lock(gDefinesMutex);
    gDefaultDefines.clear();
    for (int i = 0; i < n_defines; ++i) gDefaultDefines[keys[i]] = values[i];
    return HPT_OK;
}

int hpt_load_scene_xml(hpt_context *c, const char *path, int n_defines, const char *const *keys,
                       const char *const *values) {
    if (!c || !path) return HPT_EINVAL;
    /* the same argument checks as hpt_set_default_defines, before the context is touched */
    if (n_defines < 0 || (n_defines > 0 && (!keys || !values)))
        return setErr(c, HPT_EINVAL, "bad defines: n_defines < 0 or NULL key / value arrays");
    for (int i = 0; i < n_defines; ++i)
        if (!keys[i] || !values[i]) return setErr(c, HPT_EINVAL, "bad defines: NULL key or value");
    std::map<std::string, std::string> defs;
    {
        std::lock_guard<std::mutex> lock(gDefinesMutex);
        defs = gDefaultDefines;
    }
    for (int i = 0; i < n_defines; ++i) defs[keys[i]] = values[i]; /* explicit defines win */
    try {
        c->desc = parseSceneXML(path, defs);
    } catch (const std::exception &e) {
        return setErr(c, HPT_EIO, e.what());
    }
    const SceneDesc &d = c->desc;
    c->haveCamera = true;
    c->hairFromFile = true;
    c->haveHair = true;
    c->haveBSDF = true;
    c->haveEnv = true;
    c->envFromSunsky = d.emitter == "sunsky";
    if (d.emitter == "envmap") {
        std::string err;
        c->env = EnvHost();
        if (!loadEnvFile(d.envFile, c->env, err)) return setErr(c, HPT_EIO, err);
        c->env.scale = d.envScale;
        std::memcpy(c->env.toWorld, d.emitterToWorld, sizeof(c->env.toWorld));
    }
    c->prepared = false;
    return HPT_OK;
}

int hpt_export_scene_json(hpt_context *c, char *buf, size_t capacity, size_t *needed) {
    if (!c) return HPT_EINVAL;
    if (!c->hairFromFile) return setErr(c, HPT_ESTATE, "no scene loaded with hpt_load_scene_xml");
    const std::string js = sceneToJSON(c->desc);
    if (needed) *needed = js.size() + 1;
    if (!buf) return HPT_OK;
    if (capacity < js.size() + 1) return setErr(c, HPT_EINVAL, "buffer too small");
    std::memcpy(buf, js.c_str(), js.size() + 1);
    return HPT_OK;
}

int hpt_set_camera(hpt_context *c, const float to_world[16], float fov_x_deg, int width, int height,
                   float near_clip, float far_clip) {
    if (!c || !to_world || width <= 0 || height <= 0 || !(near_clip > 0) || !(near_clip < far_clip))
        return setErr(c, HPT_EINVAL, "invalid camera parameters");
    std::memcpy(c->desc.toWorld, to_world, sizeof(c->desc.toWorld));
    c->desc.fov = fov_x_deg;
    c->desc.fovAxis = "x";
    c->desc.width = width;
    c->desc.height = height;
    c->desc.nearClip = near_clip;
    c->desc.farClip = far_clip;
    c->haveCamera = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_sampler(hpt_context *c, int spp) {
    if (!c || spp <= 0) return setErr(c, HPT_EINVAL, "sampleCount must be positive");
    c->desc.spp = spp;
    return HPT_OK;
}

int hpt_set_sampler_scramble(hpt_context *c, uint64_t scramble) {
    if (!c) return HPT_EINVAL;
    c->desc.scramble = scramble;
    c->prepared = false;
    return HPT_OK;
}

int hpt_debug_sfmt(uint64_t seed, uint64_t n, uint64_t *out) {
    if (!out && n) return HPT_EINVAL;
    sfmtULongs(seed, (size_t) n, out);
    return HPT_OK;
}

int hpt_debug_fresnel_diffuse(int n, const float *eta, float *out) {
    if (n < 0 || (n > 0 && (!eta || !out))) return HPT_EINVAL;
    for (int i = 0; i < n; ++i) out[i] = fresnelDiffuseReflectance(eta[i]);
    return HPT_OK;
}

int hpt_set_traversal_bounds(hpt_context *c, uint32_t max_leaf_rounds, uint32_t max_restarts) {
    if (!c || max_leaf_rounds == 0) return HPT_EINVAL;
    c->maxLeafRounds = std::min<uint32_t>(max_leaf_rounds, HPT_MAX_LEAF_ROUNDS);
    c->maxRestarts = std::min<uint32_t>(max_restarts, HPT_MAX_RESTARTS);
    c->sc.maxLeafRounds = c->maxLeafRounds;
    c->sc.maxRestarts = c->maxRestarts;
    return HPT_OK;
}

int hpt_set_packet_stack(hpt_context *c, uint32_t entries) {
    if (!c) return HPT_EINVAL;
    c->packetStack = entries;
    c->sc.packetStack = entries;
    return HPT_OK;
}

int hpt_clear_schedules(hpt_context *c) {
    if (!c) return HPT_EINVAL;
    c->schedules.clear();
    return HPT_OK;
}

int hpt_set_integrator(hpt_context *c, int max_depth, int rr_depth, int strict_normals, int hide_emitters) {
    if (!c) return HPT_EINVAL;
    c->desc.maxDepth = max_depth;
    c->desc.rrDepth = rr_depth;
    c->desc.strictNormals = strict_normals != 0;
    c->desc.hideEmitters = hide_emitters != 0;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_hair_file(hpt_context *c, const char *path, float radius, float angle, const float *to_world) {
    if (!c || !path) return HPT_EINVAL;
    c->hairFromFile = true;
    HairShapeDesc h;
    h.file = path;
    h.radius = radius;
    h.angleThreshold = angle;
    h.hasToWorld = to_world != nullptr;
    if (to_world) std::memcpy(h.toWorld, to_world, sizeof(h.toWorld));
    c->desc.shapes.assign(1, h);
    c->haveHair = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_hair_reduction(hpt_context *c, float reduction) {
    if (!c) return HPT_EINVAL;
    if (!c->hairFromFile || c->desc.shapes.empty())
        return setErr(c, HPT_ESTATE, "hpt_set_hair_reduction: no hair file shape (hpt_set_hair_file first)");
    if (!(reduction >= 0 && reduction < 1))
        return setErr(c, HPT_EINVAL, "The 'reduction' parameter must have a value in [0, 1)!");
    c->desc.shapes.back().reduction = reduction;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_hair_vertices(hpt_context *c, const float *xyz, const uint8_t *starts, uint64_t n, float radius) {
    if (!c || (!xyz && n)) return HPT_EINVAL;
    c->hairFromFile = false;
    c->hair = HairData();
    c->hair.xyz.assign(xyz, xyz + 3 * n);
    c->hair.starts.assign(starts, starts + n);
    c->hair.starts.push_back(1);
    if (n) c->hair.starts[0] = 1;
    c->hair.radius = radius;
    c->hair.shapeRadius = {radius};
    c->hair.shapeFirst = {0};
    HairShapeDesc h;
    h.radius = radius;
    c->desc.shapes.assign(1, h);
    c->haveHair = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_bsdf_marschner(hpt_context *c, float int_ior, float ext_ior, int distribution, float alpha,
                           const float diffuse[3], const float specular[3]) {
    if (!c || distribution < 0 || distribution > 2 || !diffuse) return setErr(c, HPT_EINVAL, "bad marschner params");
    static const char *names[3] = {"beckmann", "ggx", "phong"};
    BsdfDesc &b = singleBsdf(c->desc, "marschner");
    b.intIOR = int_ior;
    b.extIOR = ext_ior;
    b.distribution = names[distribution];
    b.alpha = alpha;
    for (int i = 0; i < 3; ++i) {
        b.diffuse[i] = diffuse[i];
        b.specular[i] = specular ? specular[i] : 0.5f;
    }
    c->haveBSDF = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_bsdf_roughplastic(hpt_context *c, float int_ior, float ext_ior, int distribution, float alpha,
                              int sample_visible, int nonlinear, const float diffuse[3], const float specular[3]) {
    if (!c || distribution < 0 || distribution > 2) return setErr(c, HPT_EINVAL, "bad roughplastic params");
    if (int_ior < 0 || ext_ior < 0 || int_ior == ext_ior)
        return setErr(c, HPT_EINVAL, "The interior and exterior indices of refraction must be positive and differ!");
    static const char *names[3] = {"beckmann", "ggx", "phong"};
    BsdfDesc &b = singleBsdf(c->desc, "roughplastic");
    b.intIOR = int_ior;
    b.extIOR = ext_ior;
    b.distribution = names[distribution];
    b.alpha = alpha;
    b.sampleVisible = sample_visible != 0;
    b.nonlinear = nonlinear != 0;
    for (int i = 0; i < 3; ++i) {
        b.diffuse[i] = diffuse ? diffuse[i] : 0.5f;
        b.specular[i] = specular ? specular[i] : 1.0f;
    }
    c->haveBSDF = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_bsdf_marschnerdielectric(hpt_context *c, float int_ior, float ext_ior, const float diffuse[3],
                                     const float specular_reflectance[3], const float specular_transmittance[3]) {
    if (!c) return HPT_EINVAL;
    if (int_ior < 0 || ext_ior < 0)
        return setErr(c, HPT_EINVAL, "The interior and exterior indices of refraction must be positive!");
    BsdfDesc &b = singleBsdf(c->desc, "marschnerdielectric");
    b.intIOR = int_ior;
    b.extIOR = ext_ior;
    for (int i = 0; i < 3; ++i) {
        b.diffuse[i] = diffuse ? diffuse[i] : 0.5f;
        b.specular[i] = specular_reflectance ? specular_reflectance[i] : 0.1f;
        b.transmittance[i] = specular_transmittance ? specular_transmittance[i] : 0.1f;
    }
    c->haveBSDF = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_bsdf_kajiyakay(hpt_context *c, const float kd[3], const float ks[3], float exponent) {
    if (!c || !kd) return HPT_EINVAL;
    BsdfDesc &b = singleBsdf(c->desc, "kajiyakay");
    for (int i = 0; i < 3; ++i) {
        b.diffuse[i] = kd[i];
        b.specular[i] = ks ? ks[i] : 0.2f;
    }
    b.exponent = exponent;
    c->haveBSDF = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_envmap_rgb(hpt_context *c, const float *rgb, int w, int h, float scale, const float *to_world) {
    if (!c || !rgb || w <= 0 || h <= 0) return setErr(c, HPT_EINVAL, "bad envmap");
    c->env = EnvHost();
    c->env.w = w;
    c->env.h = h;
    c->env.rgb.assign(rgb, rgb + (size_t) w * h * 3);
    c->env.scale = scale;
    if (to_world) std::memcpy(c->env.toWorld, to_world, sizeof(c->env.toWorld));
    c->desc.emitter = "envmap";
    c->envFromSunsky = false;
    c->haveEnv = true;
    c->prepared = false;
    return HPT_OK;
}

int hpt_set_sunsky(hpt_context *c, const float sun_direction[3], float turbidity, float sky_scale, float sun_scale,
                   float sun_radius_scale, int resolution) {
    if (!c || !sun_direction || resolution < 4) return HPT_EINVAL;
    c->desc.emitter = "sunsky";
    for (int i = 0; i < 3; ++i) c->desc.sunDirection[i] = sun_direction[i];
    c->desc.turbidity = turbidity;
    c->desc.skyScale = sky_scale;
    c->desc.sunScale = sun_scale;
    c->desc.sunRadiusScale = sun_radius_scale;
    c->desc.skyResolution = resolution;
    c->desc.sunDirectionGiven = true;
    c->envFromSunsky = true;
    c->haveEnv = true;
    c->prepared = false;
    return HPT_OK;
}

static int uploadScene(hpt_context *c);

int hpt_prepare(hpt_context *c) {
    if (!c) return HPT_EINVAL;
    if (!c->haveCamera || !c->haveHair || !c->haveBSDF || !c->haveEnv)
        return setErr(c, HPT_ESTATE, "scene incomplete: need camera, hair, bsdf and emitter");
    if (!c->desc.meshes.empty() && !c->desc.shapes.empty())
        return setErr(c, HPT_EINVAL, "scene mixes hair with obj/rectangle shapes: the device path renders a hair "
                                     "scene or a triangle-mesh scene (C1), not both");
    c->prepared = false;
    c->meshScene = !c->desc.meshes.empty();
    const SceneDesc &d = c->desc;
    if (c->meshScene) {
        /* C1: the meshes, their BSDFs (diffuse / plastic / twosided) and the environment; the
           camera, sampler and film are the hair path's */
        try {
            if (c->sobol32.empty()) {
                std::string dir = c->dataDir + "/sobol/";
                if (!readFile(dir + "matrices32.u32", c->sobol32) || c->sobol32.size() != HPT_SOBOL_DIMS * HPT_SOBOL_BITS ||
                    !readFile(dir + "vdc.u64", c->vdc) || !readFile(dir + "vdc_inv.u64", c->vdcInv))
                    return setErr(c, HPT_EIO, "cannot read Sobol tables from " + dir);
            }
            if (d.emitter != "envmap" && d.emitter != "sunsky")
                return setErr(c, HPT_EINVAL, "mesh scene without an envmap / sunsky emitter");
            c->mesh = buildMeshScene(d);
            if (c->mesh.depth + 1 > HPT_MESH_STACK)
                return setErr(c, HPT_EINVAL, "mesh BVH deeper than the traversal stack");
            c->hair = HairData();
            c->tree = KDTreeHost();
            c->mar.clear();
            c->rp.clear();
            c->bsdfRec.clear();
            if (c->envFromSunsky) {
                if (c->sunsky.hosek.empty()) {
                    std::string err;
                    if (!loadSunSkyTables(c->dataDir, c->sunsky, err)) return setErr(c, HPT_EIO, err);
                }
                c->env = EnvHost();
                rasterizeSunSky(d, c->sunsky, c->env);
            }
            buildEnvMap(c->env);
            buildEnvMipmap(c->env);
        } catch (const std::exception &e) {
            return setErr(c, HPT_EINVAL, e.what());
        }
        c->sceneId = 0;
        const int rc = uploadScene(c);
        if (rc == HPT_OK) {
            static std::atomic<uint64_t> meshCounter{1ull << 62};
            c->sceneId = ++meshCounter;
        }
        return rc;
    }
    try {
        /* Sobol tables (data/sobol, extracted from src/samplers/sobolseq.cpp) */
        if (c->sobol32.empty()) {
            std::string dir = c->dataDir + "/sobol/";
            if (!readFile(dir + "matrices32.u32", c->sobol32) || c->sobol32.size() != HPT_SOBOL_DIMS * HPT_SOBOL_BITS ||
                !readFile(dir + "vdc.u64", c->vdc) || !readFile(dir + "vdc_inv.u64", c->vdcInv))
                return setErr(c, HPT_EIO, "cannot read Sobol tables from " + dir);
        }
        if (c->hairFromFile) {
            c->hair = HairData();
            c->hair.shapeRadius.clear();
            for (const HairShapeDesc &h : d.shapes)
                appendHair(c->hair, loadHair(h.file, h.radius, h.angleThreshold, h.reduction,
                                             h.hasToWorld ? h.toWorld : nullptr));
        }
        c->tree = buildHairKDTree(c->hair, d.kd);
        const size_t nb = d.bsdfs.size();
        c->mar.assign(nb, MarschnerHost());
        c->rp.assign(nb, RoughPlasticHost());
        c->bsdfRec.assign(nb, HptBsdf());
        for (size_t i = 0; i < nb; ++i) {
            const BsdfDesc &b = d.bsdfs[i];
            HptBsdf &rec = c->bsdfRec[i];
            std::memset(&rec, 0, sizeof(rec));
            rec.kind = bsdfKindOf(b.type);
            rec.smooth = 1;
            std::string err;
            switch (rec.kind) {
            case HPT_BSDF_MARSCHNER:
                if (!precomputeMarschner(b, c->dataDir, c->mar[i], err)) return setErr(c, HPT_EIO, err);
                break;
            case HPT_BSDF_KAJIYAKAY: configureKajiyaKay(b, rec.kk); break;
            case HPT_BSDF_ROUGHPLASTIC:
                if (!configureRoughPlastic(b, c->dataDir, c->rp[i], err)) return setErr(c, HPT_EINVAL, err);
                rec.rp = c->rp[i].p;
                break;
            case HPT_BSDF_MARSCHNERDIELECTRIC: configureMarschnerDielectric(b, rec.md); break;
            case HPT_BSDF_THINDIELECTRIC:
                configureThinDielectric(b, rec.md);
                rec.smooth = 0; /* EDeltaReflection | ENull only */
                break;
            case HPT_BSDF_DIFFUSE:
                configureDiffuse(b, rec.df);
                /* no component at all when the reflectance is 0 (diffuse.cpp:81-84) */
                rec.smooth = std::max(std::max(rec.df.refl[0], rec.df.refl[1]), rec.df.refl[2]) > 0 ? 1 : 0;
                break;
            default: return setErr(c, HPT_EINVAL, "unsupported bsdf " + b.type);
            }
        }
        if (d.shapes.empty() || nb == 0) return setErr(c, HPT_ESTATE, "no hair shape / bsdf");
        if (c->envFromSunsky) {
            if (c->sunsky.hosek.empty()) {
                std::string err;
                if (!loadSunSkyTables(c->dataDir, c->sunsky, err)) return setErr(c, HPT_EIO, err);
            }
            c->env = EnvHost();
            rasterizeSunSky(d, c->sunsky, c->env);
        }
        buildEnvMap(c->env);
        buildEnvMipmap(c->env);
    } catch (const std::exception &e) {
        return setErr(c, HPT_EIO, e.what());
    }
    c->sceneId = 0;
    const int rc = uploadScene(c);
    if (rc == HPT_OK) {
        static std::atomic<uint64_t> counter{0};
        c->sceneId = ++counter;
    }
    return rc;
}

/* the device half of hpt_prepare: the host-built scene (kd-tree, tables, envmap) to this
   context's device and the kernels' HptScene record.  hpt_context_share_scene runs it alone on a
   context that copied another's host scene */
static int uploadScene(hpt_context *c) {
    const SceneDesc &d = c->desc;
    if (c->device != HPT_HOST_ONLY) {
        HIPCHK(c, hipSetDevice(c->device));
        HIPCHK(c, hipStreamSynchronize(c->stream));
        freeBufs(c->sceneBufs);
    }
    HptScene &sc = c->sc;
    std::memset(&sc, 0, sizeof(sc));
    try {
        setupCamera(d, sc.cam);
    } catch (const std::exception &e) {
        return setErr(c, HPT_EINVAL, e.what());
    }
    int r = 0;
    r |= upload(c, c->tree.nodes.data(), c->tree.nodes.size() * sizeof(HptNode), (const void **) &sc.nodes);
    r |= upload(c, c->tree.nodes4.data(), c->tree.nodes4.size() * sizeof(HptNode4), (const void **) &sc.nodes4);
    r |= upload(c, c->tree.leafTable.data(), c->tree.leafTable.size() * 4, (const void **) &sc.leafTable);
    r |= upload(c, c->tree.leafF.data(), c->tree.leafF.size() * sizeof(HptSegF), (const void **) &sc.leafF);
    r |= upload(c, c->tree.leafQ.data(), c->tree.leafQ.size() * sizeof(HptSegQ), (const void **) &sc.leafQ);
    r |= upload(c, c->tree.prims.data(), c->tree.prims.size() * 4, (const void **) &sc.leafSeg);
    r |= upload(c, c->tree.segs.data(), c->tree.segs.size() * sizeof(HptSegment), (const void **) &sc.segs);
    for (int i = 0; i < 3; ++i) { /* the scene bounds: the hair kd-tree's, or the mesh scene's */
        sc.aabbMin[i] = c->meshScene ? c->mesh.aabbMin[i] : c->tree.aabbMin[i];
        sc.aabbMax[i] = c->meshScene ? c->mesh.aabbMax[i] : c->tree.aabbMax[i];
    }
    /* BSDF records: device tables first, then the records themselves */
    for (size_t i = 0; i < c->bsdfRec.size(); ++i) {
        HptBsdf &rec = c->bsdfRec[i];
        if (rec.kind == HPT_BSDF_MARSCHNER) {
            const MarschnerHost &m = c->mar[i];
            for (int l = 0; l < 3; ++l) {
                r |= upload(c, m.table[l].data(), m.table[l].size() * 16, (const void **) &rec.mar.table[l]);
                r |= upload(c, m.cdf[l].data(), m.cdf[l].size() * 4, (const void **) &rec.mar.cdf[l]);
                r |= upload(c, m.sums[l].data(), m.sums[l].size() * 4, (const void **) &rec.mar.sums[l]);
            }
            r |= upload(c, m.trans.data(), m.trans.size() * 4, (const void **) &rec.mar.trans);
            rec.mar.transSize = (int) m.trans.size();
            rec.mar.fdr = m.fdr;
            rec.mar.invEta2 = m.invEta2;
            rec.mar.specularSamplingWeight = m.specularSamplingWeight;
            rec.mar.vR = m.vR;
            rec.mar.vTT = m.vTT;
            rec.mar.vTRT = m.vTRT;
            rec.mar.scaleAngleRad = m.scaleAngleRad;
            const float lobeV[3] = {m.vR, m.vTT, m.vTRT};
            for (int l = 0; l < 3; ++l) {
                const float v = lobeV[l];
                rec.mar.lobeInvV[l] = 1.0f / v;
                rec.mar.lobeK[l] = v < 0.1f ? logf(1.0f / (2.0f * v)) : 2.0f * v * sinhf(1.0f / v);
            }
            for (int k = 0; k < 3; ++k) rec.mar.diffuse[k] = m.diffuse[k];
        } else if (rec.kind == HPT_BSDF_ROUGHPLASTIC) {
            r |= upload(c, c->rp[i].trans.data(), c->rp[i].trans.size() * 4, (const void **) &rec.rp.trans);
        }
    }
    const size_t nShapes = std::max<size_t>(1, c->hair.shapeRadius.size());
    if (nShapes > HPT_MAX_SHAPES) return setErr(c, HPT_EINVAL, "too many hair shapes");
    std::vector<HptShape> shapes(nShapes);
    for (size_t k = 0; k < nShapes; ++k) {
        shapes[k].radius = c->hair.shapeRadius.empty() ? c->hair.radius : c->hair.shapeRadius[k];
        shapes[k].bsdf = k < d.shapes.size() ? d.shapes[k].bsdf : 0;
    }
    sc.nShapes = (int) nShapes;
    sc.radius = shapes[0].radius;
    sc.maxRadius = 0.0f;
    for (const HptShape &h : shapes) sc.maxRadius = std::max(sc.maxRadius, h.radius);
    sc.preRadius = c->tree.preRadius;
    if (!c->bsdfRec.empty()) sc.bsdf = c->bsdfRec[shapes[0].bsdf];
    if (nShapes > 1) {
        r |= upload(c, shapes.data(), shapes.size() * sizeof(HptShape), (const void **) &sc.shapes);
        r |= upload(c, c->bsdfRec.data(), c->bsdfRec.size() * sizeof(HptBsdf), (const void **) &sc.bsdfs);
    }
    /* environment (envmap.cpp) + scene bounding sphere (scene.cpp:386-412, envmap.cpp:336-347) */
    HptEnvMap &E = sc.env;
    r |= upload(c, c->env.texel.data(), c->env.texel.size() * 16, (const void **) &E.texel);
    r |= upload(c, c->env.cdfRows.data(), c->env.cdfRows.size() * 4, (const void **) &E.cdfRows);
    r |= upload(c, c->env.cdfCols.data(), c->env.cdfCols.size() * 4, (const void **) &E.cdfCols);
    r |= upload(c, c->env.rowWeights.data(), c->env.rowWeights.size() * 4, (const void **) &E.rowWeights);
    r |= upload(c, c->env.guideRows.data(), c->env.guideRows.size() * 4, (const void **) &E.guideRows);
    r |= upload(c, c->env.guideCols.data(), c->env.guideCols.size() * 4, (const void **) &E.guideCols);
    {
        std::vector<HptMipLevel> lv(c->env.levelW.size());
        for (size_t l = 0; l < lv.size(); ++l)
            lv[l] = {c->env.levelW[l], c->env.levelH[l], c->env.levelOff[l], c->env.ratioX[l], c->env.ratioY[l]};
        r |= upload(c, c->env.mip.data(), c->env.mip.size() * 16, (const void **) &E.mip);
        r |= upload(c, lv.data(), lv.size() * sizeof(HptMipLevel), (const void **) &E.levels);
        r |= upload(c, c->env.ewaLut, sizeof(c->env.ewaLut), (const void **) &E.ewaLut);
        E.nLevels = (int) lv.size();
        E.maxAnisotropy = 10.0f; /* envmap.cpp:142 */
    }
    E.w = c->env.w;
    E.h = c->env.h;
    E.normalization = c->env.normalization;
    E.scale = c->env.scale;
    E.pixelSizeX = c->env.pixelSizeX;
    E.pixelSizeY = c->env.pixelSizeY;
    E.identity = 1;
    for (int i = 0; i < 16; ++i) E.identity &= c->env.toWorld[i] == ((i % 5 == 0) ? 1.0f : 0.0f);
    if (!E.identity) {
        double m[9], inv[9];
        for (int i = 0; i < 3; ++i)
            for (int j = 0; j < 3; ++j) {
                E.m[i * 3 + j] = c->env.toWorld[i * 4 + j];
                m[i * 3 + j] = c->env.toWorld[i * 4 + j];
            }
        double det = m[0] * (m[4] * m[8] - m[5] * m[7]) - m[1] * (m[3] * m[8] - m[5] * m[6]) +
                     m[2] * (m[3] * m[7] - m[4] * m[6]);
        inv[0] = (m[4] * m[8] - m[5] * m[7]) / det;
        inv[1] = (m[2] * m[7] - m[1] * m[8]) / det;
        inv[2] = (m[1] * m[5] - m[2] * m[4]) / det;
        inv[3] = (m[5] * m[6] - m[3] * m[8]) / det;
        inv[4] = (m[0] * m[8] - m[2] * m[6]) / det;
        inv[5] = (m[2] * m[3] - m[0] * m[5]) / det;
        inv[6] = (m[3] * m[7] - m[4] * m[6]) / det;
        inv[7] = (m[1] * m[6] - m[0] * m[7]) / det;
        inv[8] = (m[0] * m[4] - m[1] * m[3]) / det;
        for (int i = 0; i < 9; ++i) E.minv[i] = (float) inv[i];
    }
    {
        float mn[3], mx[3];
        for (int i = 0; i < 3; ++i) {
            mn[i] = sc.aabbMin[i];
            mx[i] = sc.aabbMax[i];
        }
        float cam[3] = {d.toWorld[3], d.toWorld[7], d.toWorld[11]};
        for (int i = 0; i < 3; ++i) {
            mn[i] = std::min(mn[i], cam[i]);
            mx[i] = std::max(mx[i], cam[i]);
        }
        float ctr[3], dd[3];
        for (int i = 0; i < 3; ++i) {
            ctr[i] = (mx[i] + mn[i]) * 0.5f;
            dd[i] = ctr[i] - mx[i];
        }
        float radius = std::sqrt(dd[0] * dd[0] + dd[1] * dd[1] + dd[2] * dd[2]);
        for (int i = 0; i < 3; ++i) E.bsCenter[i] = ctr[i];
        E.bsRadius = std::max(1e-4f, radius * 1.5f);
    }
    if (c->meshScene) { /* the mesh scene's arrays (HptMeshScene) */
        const MeshSceneHost &M = c->mesh;
        HptMeshScene &ms = c->ms;
        std::memset(&ms, 0, sizeof(ms));
        r |= upload(c, M.nodes.data(), M.nodes.size() * sizeof(HptBvhNode), (const void **) &ms.nodes);
        r |= upload(c, M.prims.data(), M.prims.size() * 4, (const void **) &ms.prims);
        r |= upload(c, M.tris.data(), M.tris.size() * sizeof(HptTri), (const void **) &ms.tris);
        r |= upload(c, M.rects.data(), M.rects.size() * sizeof(HptRect), (const void **) &ms.rects);
        r |= upload(c, M.meshes.data(), M.meshes.size() * sizeof(HptMeshInfo), (const void **) &ms.meshes);
        r |= upload(c, M.p.data(), M.p.size() * 4, (const void **) &ms.p);
        r |= upload(c, M.n.data(), M.n.size() * 4, (const void **) &ms.n);
        r |= upload(c, M.uv.data(), M.uv.size() * 4, (const void **) &ms.uv);
        r |= upload(c, M.dpdu.data(), M.dpdu.size() * 4, (const void **) &ms.dpdu);
        r |= upload(c, M.bsdfs.data(), M.bsdfs.size() * sizeof(HptMeshBsdf), (const void **) &ms.bsdfs);
        for (int i = 0; i < 3; ++i) ms.aabbMin[i] = M.aabbMin[i], ms.aabbMax[i] = M.aabbMax[i];
        ms.nNodes = (uint32_t) M.nodes.size();
        ms.stackDepth = M.depth + 1;
    }
    r |= upload(c, c->sobol32.data(), c->sobol32.size() * 4, (const void **) &sc.sobol);
    sc.scramble = 0;
    if (d.scramble) { /* sobol.cpp:96-102: sampleTEA of the two 32-bit halves (qmc.h:146-156) */
        uint32_t v0 = (uint32_t) d.scramble, v1 = (uint32_t) (d.scramble >> 32), sum = 0;
        for (int i = 0; i < 4; ++i) {
            sum += 0x9e3779b9u;
            v0 += ((v1 << 4) + 0xA341316Cu) ^ (v1 + sum) ^ ((v1 >> 5) + 0xC8013EA4u);
            v1 += ((v0 << 4) + 0xAD90777Du) ^ (v0 + sum) ^ ((v0 >> 5) + 0x7E95761Eu);
        }
        sc.scramble = v0; /* sampleSingle / look_up use the low 32 bits */
    }
    r |= upload(c, c->vdc.data(), c->vdc.size() * 8, (const void **) &sc.vdc);
    r |= upload(c, c->vdcInv.data(), c->vdcInv.size() * 8, (const void **) &sc.vdcInv);
    {
        static const uint32_t zero[4] = {0, 0, 0, 0};
        r |= upload(c, zero, sizeof(zero), (const void **) &sc.fault);
    }
    if (r) return HPT_EDEVICE;
    setupTent(sc.tent, sc.tentScale);
    sc.maxDepth = d.maxDepth;
    sc.rrDepth = d.rrDepth;
    sc.strictNormals = d.strictNormals ? 1 : 0;
    sc.hideEmitters = d.hideEmitters ? 1 : 0;
    if (sc.cam.logRes > (uint32_t) c->vdc.size() / HPT_SOBOL_BITS)
        return setErr(c, HPT_EINVAL, "image resolution exceeds the Sobol look-up tables");
    c->sc.maxLeafRounds = c->maxLeafRounds;
    c->sc.maxRestarts = c->maxRestarts;
    c->sc.packetStack = c->packetStack;
    c->schedules.clear();
    c->prepared = true;
    return HPT_OK;
}

int hpt_get_film_params(hpt_context *c, hpt_film_params *o) {
    if (!c || !o) return HPT_EINVAL;
    const FilmDesc &f = c->desc.film;
    std::memset(o, 0, sizeof(*o));
    o->ldr = f.type == "ldrfilm";
    o->file_format = o->ldr ? HPT_FILE_PNG
                     : f.fileFormat == "rgbe" ? HPT_FILE_RGBE
                     : f.fileFormat == "pfm"  ? HPT_FILE_PFM
                                              : HPT_FILE_OPENEXR;
    o->luminance = f.pixelFormat == "luminance";
    o->component_format = f.componentFormat == "float32" ? HPT_COMPONENT_FLOAT32
                          : f.componentFormat == "uint32" ? HPT_COMPONENT_UINT32
                                                          : HPT_COMPONENT_FLOAT16;
    o->reinhard = f.tonemapMethod == "reinhard";
    o->gamma = f.gamma;
    o->exposure = f.exposure;
    o->key = f.key;
    o->burn = f.burn;
    o->banner = f.banner;
    return HPT_OK;
}

int hpt_write_film(hpt_context *c, const char *path, const float *rgbw, int w, int h, const hpt_film_params *p,
                   char *written, int cap) {
    if (!c || !path || !rgbw || !p || w <= 0 || h <= 0) return setErr(c, HPT_EINVAL, "bad film arguments");
    FilmDesc f;
    f.type = p->ldr ? "ldrfilm" : "hdrfilm";
    static const char *files[4] = {"png", "openexr", "rgbe", "pfm"};
    static const char *comps[3] = {"float16", "float32", "uint32"};
    if (p->file_format < 0 || p->file_format > 3 || p->component_format < 0 || p->component_format > 2)
        return setErr(c, HPT_EINVAL, "bad film format");
    f.fileFormat = files[p->file_format];
    f.pixelFormat = p->luminance ? "luminance" : "rgb";
    f.componentFormat = comps[p->component_format];
    f.tonemapMethod = p->reinhard ? "reinhard" : "gamma";
    f.gamma = p->gamma;
    f.exposure = p->exposure;
    f.key = p->key;
    f.burn = p->burn;
    f.banner = p->banner != 0;
    std::string err, out;
    FilmImage img;
    if (!checkFilm(f, err) || !developFilm(rgbw, w, h, f, c->dataDir, img, err) || !writeFilm(path, img, f, out, err))
        return setErr(c, HPT_EIO, err);
    if (written && cap > 0) {
        std::strncpy(written, out.c_str(), (size_t) cap - 1);
        written[cap - 1] = 0;
    }
    return HPT_OK;
}

int hpt_get_scene_info(hpt_context *c, hpt_scene_info *o) {
    if (!c || !o) return HPT_EINVAL;
    std::memset(o, 0, sizeof(*o));
    const SceneDesc &d = c->desc;
    o->width = d.width;
    o->height = d.height;
    o->spp = d.spp;
    o->max_depth = d.maxDepth;
    o->rr_depth = d.rrDepth;
    o->strict_normals = d.strictNormals;
    o->hide_emitters = d.hideEmitters;
    o->bsdf = d.bsdfs.empty() ? -1 : bsdfKindOf(d.bsdfs[d.shapes.empty() ? 0 : d.shapes[0].bsdf].type);
    o->n_shapes = (int) std::max<size_t>(1, c->hair.shapeRadius.size());
    o->vertices = c->hair.vertexCount();
    o->segments = c->tree.segs.size();
    o->kd_nodes = c->tree.nodes.size();
    o->kd_indices = c->tree.prims.size();
    o->kd_depth = c->tree.maxDepthUsed;
    o->kd_build_seconds = c->tree.buildSeconds;
    for (int i = 0; i < 3; ++i) {
        o->aabb_min[i] = c->tree.aabbMin[i];
        o->aabb_max[i] = c->tree.aabbMax[i];
        o->bsphere_center[i] = c->sc.env.bsCenter[i];
    }
    o->bsphere_radius = c->sc.env.bsRadius;
    if (c->meshScene) { /* a mesh scene: its BVH in the kd fields, its bounds */
        o->kd_nodes = c->mesh.nodes.size();
        o->kd_indices = c->mesh.prims.size();
        o->kd_depth = (int) c->mesh.depth;
        o->vertices = c->mesh.vertexCount();
        for (int i = 0; i < 3; ++i) o->aabb_min[i] = c->mesh.aabbMin[i], o->aabb_max[i] = c->mesh.aabbMax[i];
    }
    return HPT_OK;
}

/* Image blocks in Hilbert-curve order over the nbx x nby grid of 32x32
   blocks.  Shard r of N owns every N-th block of this order (r, r+N, ...):
   N consecutive blocks of the curve are a compact patch of the image, so
   every shard gets one block of every patch and the hair's uneven screen
   coverage spreads evenly over the ranks (a plain b mod N deal gives
   whole block columns to a rank whenever N divides nbx). */
static std::vector<uint32_t> blockOrder(int nbx, int nby) {
    uint32_t n = 1;
    while (n < (uint32_t) std::max(nbx, nby)) n <<= 1;
    std::vector<uint32_t> order;
    order.reserve((size_t) nbx * nby);
    for (uint64_t d = 0; d < (uint64_t) n * n; ++d) {
        uint32_t x = 0, y = 0;
        uint64_t t = d;
        for (uint32_t sq = 1; sq < n; sq <<= 1) { /* Hilbert index -> (x, y) */
            const uint32_t rx = 1u & (uint32_t) (t / 2), ry = 1u & (uint32_t) (t ^ rx);
            if (ry == 0) {
                if (rx == 1) {
                    x = sq - 1 - x;
                    y = sq - 1 - y;
                }
                std::swap(x, y);
            }
            x += sq * rx;
            y += sq * ry;
            t /= 4;
        }
        if ((int) x < nbx && (int) y < nby) order.push_back(y * (uint32_t) nbx + x);
    }
    return order;
}

/* The shard of every image block.  Without weights: position i of the Hilbert order goes to
   shard i mod N (compact patches of N blocks, one block each).  With weights (the measured
   work of each block, hpt_set_block_weights): longest-processing-time first -- blocks in
   descending weight (ties in Hilbert order) each to the shard with the least weight so far
   (ties to the lowest shard) -- the same deal on every rank given the same weights. */
static std::vector<int> dealBlocks(int nbx, int nby, int nShards, const std::vector<double> &weights) {
    const std::vector<uint32_t> order = blockOrder(nbx, nby);
    std::vector<int> shardOf(order.size(), 0);
    if (weights.size() != order.size()) {
        for (size_t i = 0; i < order.size(); ++i) shardOf[order[i]] = (int) (i % (size_t) nShards);
        return shardOf;
    }
    std::vector<size_t> byWeight(order.size());
    for (size_t i = 0; i < order.size(); ++i) byWeight[i] = i; /* Hilbert positions */
    std::stable_sort(byWeight.begin(), byWeight.end(),
                     [&](size_t a, size_t b) { return weights[order[a]] > weights[order[b]]; });
    std::vector<double> load((size_t) nShards, 0.0);
    for (size_t k : byWeight) {
        const int r = (int) (std::min_element(load.begin(), load.end()) - load.begin());
        shardOf[order[k]] = r;
        load[(size_t) r] += weights[order[k]];
    }
    return shardOf;
}

/* upload this shard's block ownership tables (cached per frame shape, shard and deal) */
static int ensureOwnership(hpt_context *c, int W, int H, int nbx, int nby, int shard, int nShards) {
    if (c->ownW == W && c->ownH == H && c->ownShard == shard && c->ownShards == nShards &&
        c->ownWeights == c->weightsVersion)
        return HPT_OK;
    if (!c->blockWeights.empty() && c->blockWeights.size() != (size_t) nbx * nby)
        return setErr(c, HPT_EINVAL, "hpt_set_block_weights gave " + std::to_string(c->blockWeights.size()) +
                                         " block weights for a frame of " + std::to_string(nbx * nby) + " blocks");
    const std::vector<uint32_t> order = blockOrder(nbx, nby);
    const std::vector<int> shardOf = dealBlocks(nbx, nby, nShards, c->blockWeights);
    std::vector<uint32_t> blockOf;
    std::vector<int32_t> localOf(order.size(), -1);
    for (size_t i = 0; i < order.size(); ++i) /* a shard's blocks in Hilbert order (locality) */
        if (shardOf[order[i]] == shard) {
            localOf[order[i]] = (int32_t) blockOf.size();
            blockOf.push_back(order[i]);
        }
    const int n = (int) order.size();
    if (n > c->ownCap) {
        if (c->dBlockOf) (void) hipFree(c->dBlockOf);
        if (c->dLocalOf) (void) hipFree(c->dLocalOf);
        if (c->dBlockCost) (void) hipFree(c->dBlockCost);
        c->dBlockOf = nullptr;
        c->dLocalOf = nullptr;
        c->dBlockCost = nullptr;
        c->ownCap = 0;
        HIPCHK(c, hipMalloc((void **) &c->dBlockOf, n * sizeof(uint32_t)));
        HIPCHK(c, hipMalloc((void **) &c->dLocalOf, n * sizeof(int32_t)));
        /* HPT_COST_STRIPES stripes of n counters, + a snapshot of them per wave */
        HIPCHK(c, hipMalloc((void **) &c->dBlockCost, 2 * HPT_COST_STRIPES * n * sizeof(uint32_t)));
        c->ownCap = n;
    }
    if (!blockOf.empty())
        HIPCHK(c, hipMemcpy(c->dBlockOf, blockOf.data(), blockOf.size() * sizeof(uint32_t), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemcpy(c->dLocalOf, localOf.data(), localOf.size() * sizeof(int32_t), hipMemcpyHostToDevice));
    HIPCHK(c, hipMemset(c->dBlockCost, 0, HPT_COST_STRIPES * c->ownCap * sizeof(uint32_t))); /* costs are per ownership */
    c->ownW = W, c->ownH = H, c->ownShard = shard, c->ownShards = nShards, c->ownLocal = (int) blockOf.size();
    c->ownWeights = c->weightsVersion;
    c->ownBlocks.assign(blockOf.begin(), blockOf.end());
    return HPT_OK;
}

static int renderImpl(hpt_context *c, const hpt_render_params *prm, float4 *dFilm) {
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context cannot render");
    if (!c->prepared) return setErr(c, HPT_ESTATE, "hpt_prepare() must succeed before rendering");
    auto t0 = std::chrono::steady_clock::now();
    const HptScene &sc = c->sc;
    const int W = sc.cam.width, H = sc.cam.height;
    const int nbx = (W + HPT_BLOCK - 1) / HPT_BLOCK, nby = (H + HPT_BLOCK - 1) / HPT_BLOCK;
    const int nShards = std::max(1, prm->n_shards), shard = prm->shard;
    if (shard < 0 || shard >= nShards) return setErr(c, HPT_EINVAL, "bad shard");
    if (int r0 = ensureOwnership(c, W, H, nbx, nby, shard, nShards)) return r0;
    const int localBlocks = c->ownLocal;
    const uint64_t slots = (uint64_t) localBlocks * 1024u;
    const int sppBegin = prm->spp_begin, sppEnd = prm->spp_end;
    if (sppEnd < sppBegin || sppBegin < 0) return setErr(c, HPT_EINVAL, "bad spp range");
    std::memset(&c->stats, 0, sizeof(c->stats));
    if (slots == 0 || sppEnd == sppBegin) return HPT_OK;
    uint64_t maxWave = prm->max_wave_paths ? prm->max_wave_paths : (uint64_t) 1 << 26;
    uint32_t nSpp = (uint32_t) std::max<uint64_t>(1, std::min<uint64_t>(sppEnd - sppBegin, maxWave / slots));
    const uint64_t waveCap = slots * nSpp;
    if (waveCap > 0xffffffffull) return setErr(c, HPT_EINVAL, "wave too large");
    int r = ensureWave(c, waveCap);
    if (r) return r;
    const uint32_t tailPaths = c->tailPaths;
    if (slots > c->partialSlots) {
        if (c->partial) (void) hipFree(c->partial);
        c->partial = nullptr;
        c->partialSlots = 0;
        HIPCHK(c, hipMalloc((void **) &c->partial, slots * 9 * sizeof(float4)));
        c->partialSlots = slots;
    }
    hipStream_t s = c->stream;
    c->P.blockCost = c->dBlockCost;
    c->P.costStride = (uint32_t) c->ownCap;
    const size_t costWords = (size_t) HPT_COST_STRIPES * c->ownCap;
    if (!c->scDev) HIPCHK(c, hipMalloc((void **) &c->scDev, sizeof(HptScene)));
    if (c->scShadow.size() != sizeof(HptScene) || std::memcmp(c->scShadow.data(), &c->sc, sizeof(HptScene)) != 0) {
        HIPCHK(c, hipMemcpy(c->scDev, &c->sc, sizeof(HptScene), hipMemcpyHostToDevice));
        c->scShadow.assign((const uint8_t *) &c->sc, (const uint8_t *) &c->sc + sizeof(HptScene));
    }
    const bool st = prm->collect_stats != 0;      /* HIP event timing per kernel class */
    const bool counted = prm->collect_stats == 2; /* + traversal counters (k_trace_counted) */
    /* 3: events around the traversal launches only (k_trace, k_trace_packet): each event is a
       packet between two launches, and a frame of 22 launches pays ~4 us per event */
    const bool traceOnly = prm->collect_stats == 3;
    if (counted) HIPCHK(c, hipMemsetAsync(c->dstats, 0, 24 * 8, s));
    std::vector<std::pair<hipEvent_t, hipEvent_t>> evTrace, evOther[7];
    size_t evUsed = 0;
    auto timed = [&](int cls, auto fn) -> hipError_t {
        if (!st || (traceOnly && cls != -1 && cls != 6)) return fn();
        hipEvent_t a = takeEvent(c, evUsed), b = takeEvent(c, evUsed);
        (void) hipEventRecord(a, s);
        hipError_t e = fn();
        (void) hipEventRecord(b, s);
        if (cls < 0) evTrace.push_back({a, b});
        else evOther[cls].push_back({a, b});
        return e;
    };
    if (int rf = clearFault(c)) return rf;
    uint32_t *hostCnt = c->hostCnt;
    uint64_t bounces = 0;
    int maxB = 0;
    /* HPT_TRACE_REPORT=1 with counters on: per-launch traversal counters on stderr */
    const bool perLaunch = counted && std::getenv("HPT_TRACE_REPORT") != nullptr;
    /* HPT_BOUNCE_REPORT=1 with timing on: per-bounce queue sizes and trace time on stderr */
    const bool bounceReport = std::getenv("HPT_BOUNCE_REPORT") != nullptr;
    uint64_t prevSt[8] = {0, 0, 0, 0, 0, 0, 0, 0}, prevShadow[2] = {0, 0};
    auto reportLaunch = [&](const char *what) {
        if (!perLaunch) return;
        uint64_t hs[24];
        if (hipMemcpyAsync(hs, c->dstats, 24 * 8, hipMemcpyDeviceToHost, s) != hipSuccess ||
            hipStreamSynchronize(s) != hipSuccess || hipMemsetAsync(c->dstats + 8, 0, 32, s) != hipSuccess)
            return;
        if (c->packets && std::strcmp(what, "camera") == 0) {
            const double rays = (double) std::max<uint64_t>(1, hs[14]);
            std::fprintf(stderr, "[trace] packets  rays %10llu binary nodes/ray %6.2f prims/ray %6.2f exact/ray %5.2f "
                         "util nodes %.3f prims %.3f | fallbacks %llu\n", (unsigned long long) hs[14], hs[12] / rays,
                         hs[13] / rays, hs[15] / rays, hs[12] / std::max(1.0, (double) hs[16]),
                         hs[13] / std::max(1.0, (double) hs[17]), (unsigned long long) hs[18]);
            return;
        }
        uint64_t d[8];
        for (int i = 0; i < 8; ++i) d[i] = hs[i] - prevSt[i], prevSt[i] = hs[i];
        const uint64_t dsN = hs[19] - prevShadow[0], dsP = hs[20] - prevShadow[1];
        prevShadow[0] = hs[19], prevShadow[1] = hs[20];
        std::fprintf(stderr, "[trace] %-8s shadow rays: nodes/ray %6.2f prims/ray %6.2f | closest rays: nodes/ray %6.2f "
                     "prims/ray %6.2f\n", what, dsN / std::max(1.0, (double) d[3]), dsP / std::max(1.0, (double) d[3]),
                     (d[0] - dsN) / std::max(1.0, (double) d[2]), (d[1] - dsP) / std::max(1.0, (double) d[2]));
        const double rays = (double) (d[2] + d[3]);
        std::fprintf(stderr, "[trace] %-8s closest %10llu shadow %10llu nodes/ray %6.2f prims/ray %6.2f exact/ray %5.2f "
                     "util nodes %.3f prims %.3f | max rounds %llu max restarts %llu restarted rays %llu restarts %llu\n", what, (unsigned long long) d[2], (unsigned long long) d[3],
                     d[0] / std::max(1.0, rays), d[1] / std::max(1.0, rays), d[5] / std::max(1.0, rays),
                     d[0] / std::max(1.0, (double) d[6]), d[1] / std::max(1.0, (double) d[7]),
                     (unsigned long long) hs[8], (unsigned long long) hs[9], (unsigned long long) hs[10],
                     (unsigned long long) hs[11]);
    };
    hipError_t e = hipSuccess;
    for (int j0 = sppBegin; j0 < sppEnd && e == hipSuccess; j0 += (int) nSpp) {
        HptWave w;
        w.sppBegin = (uint32_t) j0;
        w.nSpp = (uint32_t) std::min<int>((int) nSpp, sppEnd - j0);
        w.nPaths = (uint32_t) (slots * w.nSpp);
        w.width = W;
        w.height = H;
        w.nbx = nbx;
        w.shard = shard;
        w.nShards = nShards;
        w.blockOf = c->dBlockOf;
        c->P.costSpp = w.nSpp;
        w.localOf = c->dLocalOf;
        w.doneIf = nullptr;
        w.doneParity = 0;
        c->stats.waves++;
        /* a wave rendered again after its schedule overflowed must not count twice: the timing
           events and traversal counters of the discarded attempt are rolled back to here */
        const size_t evMark = evTrace.size();
        size_t evMarkOther[7];
        for (int i = 0; i < 7; ++i) evMarkOther[i] = evOther[i].size();
        if (counted) HIPCHK(c, hipMemcpyAsync(c->dstats + 24, c->dstats, 24 * 8, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemcpyAsync(c->dBlockCost + costWords, c->dBlockCost, costWords * 4, hipMemcpyDeviceToDevice, s));
        HIPCHK(c, hipMemsetAsync(c->counters, 0, HPT_COUNTER_WORDS * 4, s));
        uint32_t *C = c->counters, *dst = counted ? (uint32_t *) c->dstats : nullptr;
        if (c->meshScene) {
            /* C1: every camera sample of the wave to termination in one launch (k_mesh_paths),
               then the film splat; its time is reported as ms_shade */
            e = timed(2, [&] { return hpt_launch_mesh_paths(sc, c->ms, w, c->P, C, s); });
            if (e) break;
            e = timed(4, [&] { return hpt_launch_gather(sc, w, c->P, c->partial, dFilm, s); });
            if (e) break;
            e = hipMemcpyAsync(hostCnt, C, HPT_Q_COUNT * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e) break;
            if (hostCnt[HPT_C_ERROR])
                return setErr(c, HPT_EINVAL, "Lookup dimension exceeds the direction number table size! You may have "
                                             "to reduce the 'maxDepth' parameter of your integrator.");
            uint64_t shaded = 0;
            std::memcpy(&shaded, hostCnt + HPT_C_BOUNCES, 8);
            bounces += shaded;
            c->stats.paths += w.nPaths;
            continue;
        }
        uint32_t *curPacket = C + HPT_CURSOR_SET(2), *curOverflow = C + HPT_CURSOR_SET(3);
        /* the camera pass is bounce 0 (parity 0) */
        e = timed(0, [&] { return hpt_launch_camera(sc, w, c->P, c->qTrace, C + HPT_C_TRACE(0), s); });
        if (e) break;
        /* the camera pass has no shadow rays: qShadow / C[SHADOW(0)] take the rays of overflowing packets */
        e = c->packets ? timed(6, [&] {
            return hpt_launch_trace_packet(sc, c->P, c->qTrace, C + HPT_C_TRACE(0), curPacket, dst, w.nPaths, c->qShadow,
                                           C + HPT_C_SHADOW(0), s);
        })
                       : timed(-1, [&] {
                             return hpt_launch_trace_camera(sc, c->P, c->qTrace, C + HPT_C_TRACE(0), curPacket, dst,
                                                            w.nPaths, s);
                         });
        if (e) break;
        reportLaunch("camera");
        if (c->packets) {
            /* overflowing packets' rays (none at the shipped configs), their own cursor set */
            e = hpt_launch_trace_overflow(sc, c->P, c->qTrace, c->qShadow, C + HPT_C_SHADOW(0), curOverflow,
                                          std::min<uint64_t>(w.nPaths, 1u << 16), s);
            if (e) break;
        }
        e = timed(1, [&] {
            return hpt_launch_primary(sc, c->P, c->qTrace, C + HPT_C_TRACE(0), c->qShade[1], C + HPT_C_SHADE(1), w.nPaths, s);
        });
        if (e) break;
        /* bounce b (parity p): shade -> trace -> clear -> post.  A wave whose schedule is known
           (the same spp range and shard rendered since the last prepare) launches its bounces
           ahead, each kernel reading its queue length on the device, and the k_tail launch
           that ended it; the device decides whether the tail takes its bounce (the queue is
           shorter than tailPaths) or leaves it to k_shade.  The host reads the counters back
           once, at the end of the schedule, and goes on bounce by bounce from there if paths
           are still live -- a schedule that does not fit costs launches, never paths.  A wave
           without a schedule reads each bounce's queue length back (grid sizes, the switch
           to k_tail) and records its schedule. */
        const std::array<int64_t, 4> key{(int64_t) w.sppBegin, (int64_t) w.nSpp, shard, nShards};
        auto known = c->schedules.find(key);
        const bool ahead = c->bounceAhead && !perLaunch && !bounceReport && known != c->schedules.end();
        bool fits = true; /* the schedule launched ahead was the whole wave */
        bool gatheredAhead = false, firstRead = true, doneAtFirstRead = false;
        bool learn = c->bounceAhead && !ahead, extended = false;
        BounceSchedule seen;
        int b = 1, bounce = 0;
        /* grid: the shade launch's (the trace launch's work is at most twice it, the post's at most it) */
        auto wavefrontBounce = [&](uint32_t p, uint64_t grid, uint32_t tailFrom) -> hipError_t {
            const uint32_t q = p ^ 1u;
            hipError_t e1 = timed(2, [&] {
                return hpt_launch_shade(sc, c->P, c->qShade[p], C + HPT_C_SHADE(p), c->qTrace, C + HPT_C_TRACE(p),
                                        c->qShadow, C + HPT_C_SHADOW(p), C, grid, tailFrom, s);
            });
            if (e1) return e1;
            e1 = timed(-1, [&] {
                return hpt_launch_trace(sc, c->P, c->qTrace, c->qShadow, C + HPT_C_TRACE(p), C + HPT_C_SHADOW(p),
                                        C + HPT_CURSOR_SET(p), dst, 2ull * grid, s, C, q);
            });
            if (e1) return e1;
            reportLaunch("bounce");
            if (bounceReport && st && !evTrace.empty()) {
                float ms = 0;
                (void) hipStreamSynchronize(s);
                (void) hipEventElapsedTime(&ms, evTrace.back().first, evTrace.back().second);
                std::fprintf(stderr, "[bounce %d] shade %llu -> trace %.3f ms\n", b, (unsigned long long) grid, ms);
            }
            return timed(3, [&] {
                return hpt_launch_post(sc, c->P, c->qTrace, C + HPT_C_TRACE(p), c->qShade[q], C + HPT_C_SHADE(q), C,
                                       grid, s);
            });
        };
        if (ahead) {
            const BounceSchedule &k = known->second;
            for (size_t i = 0; i < k.shade.size() && e == hipSuccess; ++i, ++b)
                e = wavefrontBounce((uint32_t) b & 1u, k.shade[i], 0u);
            if (e == hipSuccess && k.tail)
                e = timed(5, [&] {
                    const uint32_t p = (uint32_t) b & 1u;
                    return hpt_launch_tail(sc, c->P, c->qShade[p], C + HPT_C_SHADE(p), C, HPT_ITEMS_ON_DEVICE,
                                           tailPaths, s);
                });
            if (e) break;
            /* the gather right behind the schedule, guarded on the device (the wave is done: no
               live path in this bounce's shade queue, or the tail took it; no overflow), so the
               host's counter read-back no longer stands between the last bounce and it */
            if (!perLaunch) {
                HptWave wg = w;
                wg.doneIf = C;
                wg.doneParity = (uint32_t) b & 1u;
                e = timed(4, [&] { return hpt_launch_gather(sc, wg, c->P, c->partial, dFilm, s); });
                if (e) break;
                gatheredAhead = true;
            }
        }
        for (; e == hipSuccess; ++b) {
            const uint32_t p = (uint32_t) b & 1u;
            e = hipMemcpyAsync(hostCnt, C, HPT_Q_COUNT * 4, hipMemcpyDeviceToHost, s);
            if (e == hipSuccess) e = hipStreamSynchronize(s);
            if (e) break;
            const uint32_t n = hostCnt[HPT_C_SHADE(p)];
            if (firstRead) doneAtFirstRead = hptWaveDone(hostCnt, p); /* what the early gather's guard saw */
            firstRead = false;
            if (n == 0 || hostCnt[HPT_C_TAIL_PATHS] != 0) break; /* no live path, or k_tail took the rest */
            if (ahead && fits) {
                /* the schedule did not cover the wave (its tail declined, or bounces ran past it):
                   re-record it as the part launched ahead plus the bounces read back from here */
                seen.shade = known->second.shade;
                seen.tail = false;
                c->schedules.erase(key);
                fits = false;
                learn = extended = true;
                c->stats.schedule_extensions++;
            }
            if (n < tailPaths) {
                /* few live paths: finish them all in one launch (k_tail) */
                seen.tail = true;
                e = timed(5, [&] { return hpt_launch_tail(sc, c->P, c->qShade[p], C + HPT_C_SHADE(p), C, n, ~0u, s); });
                if (e) break;
                e = hipMemcpyAsync(hostCnt, C, HPT_Q_COUNT * 4, hipMemcpyDeviceToHost, s);
                if (e == hipSuccess) e = hipStreamSynchronize(s);
                break;
            }
            seen.shade.push_back(n);
            e = wavefrontBounce(p, n, 0u);
        }
        if (e) break;
        if (hostCnt[HPT_C_OVERFLOW] && !ahead) {
            (void) hipStreamSynchronize(s);
            return setErr(c, HPT_EDEVICE, "internal error: a shade grid sized from its read-back queue overflowed");
        }
        if (hostCnt[HPT_C_OVERFLOW]) {
            /* a bounce launched ahead had more live paths than its schedule's grid: drop the
               schedule and render the wave again, reading every queue length back (the
               film takes a wave's paths only at its gather) */
            c->schedules.erase(key);
            c->stats.waves--;
            c->stats.schedule_misses++;
            for (size_t i = evMark; i < evTrace.size(); ++i) evUsed -= 2; /* events back to the pool */
            evTrace.resize(evMark);
            for (int i = 0; i < 7; ++i) {
                for (size_t k = evMarkOther[i]; k < evOther[i].size(); ++k) evUsed -= 2;
                evOther[i].resize(evMarkOther[i]);
            }
            if (counted) HIPCHK(c, hipMemcpyAsync(c->dstats, c->dstats + 24, 24 * 8, hipMemcpyDeviceToDevice, s));
            HIPCHK(c, hipMemcpyAsync(c->dBlockCost, c->dBlockCost + costWords, costWords * 4, hipMemcpyDeviceToDevice, s));
            j0 -= (int) nSpp;
            continue;
        }
        if (learn) {
            /* (the test hooks shorten first recordings only, so an extended schedule is whole) */
            if (c->scheduleTest == 1 && !extended)
                for (auto &n : seen.shade) n = std::max<uint32_t>(1, n / 2);
            if (c->scheduleTest == 2 && !extended && seen.tail && !seen.shade.empty()) seen.shade.pop_back();
            if (c->schedules.size() >= 4096) c->schedules.clear(); /* e.g. a long run of -r passes */
            c->schedules[key] = seen;
        }
        if (ahead && fits) c->stats.waves_ahead++;
        /* the wave's bounce statistics, counted on the device */
        {
            uint64_t shaded = 0;
            std::memcpy(&shaded, hostCnt + HPT_C_BOUNCES, 8);
            bounces += shaded + hostCnt[HPT_C_TAIL_BOUNCES]; /* k_tail counts its first bounce too */
            c->stats.tail_paths += hostCnt[HPT_C_TAIL_PATHS];
            bounce = (int) hostCnt[HPT_C_LAUNCHES];
        }
        maxB = std::max(maxB, bounce);
        if (e) break;
        if (hostCnt[HPT_C_ERROR]) {
            (void) hipStreamSynchronize(s);
            return setErr(c, HPT_EINVAL, "Lookup dimension exceeds the direction number table size! You may have "
                                         "to reduce the 'maxDepth' parameter of your integrator.");
        }
        if (!(gatheredAhead && doneAtFirstRead)) /* (else the guarded gather launched ahead took the wave) */
            e = timed(4, [&] { return hpt_launch_gather(sc, w, c->P, c->partial, dFilm, s); });
        c->stats.paths += w.nPaths;
    }
    hipError_t e2 = hipStreamSynchronize(s);
    if (e != hipSuccess || e2 != hipSuccess)
        return setErr(c, HPT_EDEVICE, std::string("render failed: ") + hipGetErrorString(e ? e : e2));
    if (int rf = checkFault(c)) return rf;
    auto sumEv = [](std::vector<std::pair<hipEvent_t, hipEvent_t>> &v) {
        double tot = 0;
        for (auto &p : v) {
            float ms = 0;
            (void) hipEventElapsedTime(&ms, p.first, p.second);
            tot += ms;
        }
        return tot;
    };
    if (st) {
        c->stats.ms_trace = sumEv(evTrace);
        c->stats.trace_launches = evTrace.size();
        c->stats.ms_camera = sumEv(evOther[0]);
        c->stats.ms_primary = sumEv(evOther[1]);
        c->stats.ms_shade = sumEv(evOther[2]);
        c->stats.ms_post = sumEv(evOther[3]);
        c->stats.ms_gather = sumEv(evOther[4]);
        c->stats.ms_tail = sumEv(evOther[5]);
        c->stats.ms_trace_packet = sumEv(evOther[6]);
        c->stats.packet_launches = evOther[6].size();
    }
    if (counted) {
        uint64_t hs[24];
        HIPCHK(c, hipMemcpy(hs, c->dstats, 24 * 8, hipMemcpyDeviceToHost));
        c->stats.packet_nodes = hs[12];
        c->stats.packet_prims = hs[13];
        c->stats.packet_rays = hs[14];
        c->stats.packet_exact = hs[15];
        c->stats.packet_node_slots = hs[16];
        c->stats.packet_prim_slots = hs[17];
        c->stats.packet_fallbacks = hs[18];
        c->stats.max_leaf_rounds = hs[8];
        c->stats.max_restarts = hs[9];
        c->stats.restarted_rays = hs[10];
        c->stats.nodes = hs[0];
        c->stats.prims = hs[1];
        c->stats.closest_rays = hs[2];
        c->stats.shadow_rays = hs[3];
        c->stats.shadow_unoccluded = hs[4];
        c->stats.prim_exact = hs[5];
        c->stats.node_slots = hs[6];
        c->stats.prim_slots = hs[7];
        c->stats.binary_nodes = hs[21];
    }
    c->stats.bounces = bounces;
    c->stats.max_bounces = maxB;
    c->stats.ms_total = std::chrono::duration<double, std::milli>(std::chrono::steady_clock::now() - t0).count();
    return HPT_OK;
}

int hpt_render_device(hpt_context *c, const hpt_render_params *prm, void *dfilm) {
    if (!c || !prm || !dfilm) return HPT_EINVAL;
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context cannot render");
    HIPCHK(c, hipSetDevice(c->device));
    return renderImpl(c, prm, (float4 *) dfilm);
}

int hpt_render(hpt_context *c, const hpt_render_params *prm, float *film) {
    if (!c || !prm || !film) return HPT_EINVAL;
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context cannot render");
    HIPCHK(c, hipSetDevice(c->device));
    const size_t n = (size_t) c->desc.width * c->desc.height;
    float4 *d = nullptr;
    HIPCHK(c, hipMalloc(&d, n * 16));
    hipError_t e = hipMemcpy(d, film, n * 16, hipMemcpyHostToDevice);
    int r = e == hipSuccess ? renderImpl(c, prm, d) : HPT_EDEVICE;
    if (r == HPT_OK) e = hipMemcpy(film, d, n * 16, hipMemcpyDeviceToHost);
    (void) hipFree(d);
    if (r) return r;
    if (e != hipSuccess) return setErr(c, HPT_EDEVICE, hipGetErrorString(e));
    return HPT_OK;
}

int hpt_context_share_scene(hpt_context *src, int device, hpt_context **out) {
    tlsErr.clear(); /* hpt_last_error(NULL) describes this call only */
    if (!src || !out) return HPT_EINVAL;
    *out = nullptr;
    /* src is only read here (several threads may share one source at once): failures are
       reported to the calling thread, hpt_last_error(NULL), never written to src */
    if (!src->prepared) return setErr(nullptr, HPT_ESTATE, "hpt_context_share_scene: the source context is not prepared");
    hpt_context *c = nullptr;
    int rc = hpt_context_create(device, &c);
    if (rc)
        return setErr(nullptr, rc, "hpt_context_share_scene: no gfx950 context on device " + std::to_string(device));
    /* the host-built scene, as hpt_prepare left it on src */
    c->dataDir = src->dataDir;
    c->desc = src->desc;
    c->haveCamera = src->haveCamera, c->haveHair = src->haveHair, c->haveBSDF = src->haveBSDF;
    c->haveEnv = src->haveEnv, c->hairFromFile = src->hairFromFile, c->envFromSunsky = src->envFromSunsky;
    c->hair = src->hair;
    c->tree = src->tree;
    c->meshScene = src->meshScene;
    c->mesh = src->mesh;
    c->mar = src->mar;
    c->rp = src->rp;
    c->bsdfRec = src->bsdfRec;
    c->env = src->env;
    c->sobol32 = src->sobol32;
    c->vdc = src->vdc;
    c->vdcInv = src->vdcInv;
    c->maxLeafRounds = src->maxLeafRounds, c->maxRestarts = src->maxRestarts, c->packetStack = src->packetStack;
    c->tailPaths = src->tailPaths, c->bounceAhead = src->bounceAhead, c->packets = src->packets;
    /* the shard deal: hpt_render_multi gives shard g to context g, and every context must deal
       the blocks the same way or some blocks are rendered twice and others never */
    c->blockWeights = src->blockWeights;
    c->weightsVersion = src->weightsVersion + 1;
    rc = uploadScene(c);
    if (rc) {
        setErr(nullptr, rc, c->err);
        hpt_context_destroy(c);
        return rc;
    }
    c->sceneId = src->sceneId;
    *out = c;
    return HPT_OK;
}

int hpt_render_multi(hpt_context *const *ctxs, int n, const hpt_render_params *prm, float *film) {
    if (!ctxs || n <= 0 || !prm || !film) return HPT_EINVAL;
    hpt_context *c0 = ctxs[0];
    if (!c0) return HPT_EINVAL;
    for (int g = 0; g < n; ++g) {
        const hpt_context *c = ctxs[g];
        if (!c) return HPT_EINVAL;
        if (c->device == HPT_HOST_ONLY) return setErr(c0, HPT_EDEVICE, "host-only context cannot render");
        if (!c->prepared) return setErr(c0, HPT_ESTATE, "hpt_render_multi: a context is not prepared");
        /* one film from one scene: every context must be a share of the same prepared scene
           (re-preparing or re-configuring a context gives it a scene of its own), with the same
           camera and integrator settings and the same shard deal */
        if (c->sceneId != c0->sceneId)
            return setErr(c0, HPT_EINVAL, "hpt_render_multi: context " + std::to_string(g) +
                                              " renders a different prepared scene (share one with hpt_context_share_scene)");
        if (std::memcmp(&c->sc.cam, &c0->sc.cam, sizeof(HptCamera)) != 0 || c->sc.maxDepth != c0->sc.maxDepth ||
            c->sc.rrDepth != c0->sc.rrDepth || c->sc.strictNormals != c0->sc.strictNormals ||
            c->sc.hideEmitters != c0->sc.hideEmitters || c->sc.scramble != c0->sc.scramble || c->desc.spp != c0->desc.spp)
            return setErr(c0, HPT_EINVAL, "hpt_render_multi: context " + std::to_string(g) +
                                              " has a different camera, sampler or integrator setting");
        if (c->blockWeights != c0->blockWeights)
            return setErr(c0, HPT_EINVAL, "hpt_render_multi: context " + std::to_string(g) +
                                              " deals the blocks with different weights (hpt_set_block_weights on every context)");
    }
    const size_t pixels = (size_t) c0->sc.cam.width * c0->sc.cam.height;
    /* every context renders its shard into its own device film; the receiving context's film
       starts as the caller's (hpt_render accumulates), the others at zero */
    std::vector<int> rcs(n, HPT_OK);
    auto shard = [&](int g) {
        hpt_context *c = ctxs[g];
        auto fail = [&](hipError_t e) { rcs[g] = setErr(c, HPT_EDEVICE, hipGetErrorString(e)); };
        hipError_t e = hipSetDevice(c->device);
        if (e == hipSuccess && c->mfilmPixels < pixels) {
            if (c->mfilm) (void) hipFree(c->mfilm);
            c->mfilm = nullptr;
            c->mfilmPixels = 0;
            e = hipMalloc((void **) &c->mfilm, pixels * 16);
            if (e == hipSuccess) c->mfilmPixels = pixels;
        }
        if (e == hipSuccess)
            e = g == 0 ? hipMemcpyAsync(c->mfilm, film, pixels * 16, hipMemcpyHostToDevice, c->stream)
                       : hipMemsetAsync(c->mfilm, 0, pixels * 16, c->stream);
        if (e != hipSuccess) return fail(e);
        hpt_render_params p = *prm;
        p.shard = g;
        p.n_shards = n;
        rcs[g] = renderImpl(c, &p, c->mfilm);
        /* the film is complete on this context's stream before the receiving device reads it */
        if (rcs[g] == HPT_OK && g > 0 && (e = hipStreamSynchronize(c->stream)) != hipSuccess) fail(e);
    };
    {
        std::vector<std::thread> th;
        for (int g = 1; g < n; ++g) th.emplace_back(shard, g);
        shard(0);
        for (auto &t : th) t.join();
    }
    for (int g = 0; g < n; ++g)
        if (rcs[g]) {
            if (g) setErr(c0, rcs[g], "device " + std::to_string(ctxs[g]->device) + ": " + ctxs[g]->err);
            return rcs[g];
        }
    /* the film combine (renderproc.cpp:142-145) on the receiving device: every other film is
       pulled at once over xGMI (peer copies, one stream and staging buffer per peer), then
       added in shard order, so the sum is the host sum f0 + f1 + ... of the same films */
    HIPCHK(c0, hipSetDevice(c0->device));
    if (n > 1) {
        const size_t need = (size_t) (n - 1) * pixels;
        if (c0->mstagePixels < need) {
            if (c0->mstage) (void) hipFree(c0->mstage);
            c0->mstage = nullptr;
            c0->mstagePixels = 0;
            HIPCHK(c0, hipMalloc((void **) &c0->mstage, need * 16));
            c0->mstagePixels = need;
        }
        while ((int) c0->peerStreams.size() < n - 1) {
            hipStream_t ps;
            hipEvent_t pe;
            HIPCHK(c0, hipStreamCreateWithFlags(&ps, hipStreamNonBlocking));
            if (hipEventCreateWithFlags(&pe, hipEventDisableTiming) != hipSuccess) {
                (void) hipStreamDestroy(ps);
                return setErr(c0, HPT_EDEVICE, "hpt_render_multi: cannot create a copy event");
            }
            c0->peerStreams.push_back(ps);
            c0->peerEvents.push_back(pe);
        }
        for (int g = 1; g < n; ++g) {
            const int dg = ctxs[g]->device;
            if (dg != c0->device) {
                int can = 0;
                HIPCHK(c0, hipDeviceCanAccessPeer(&can, c0->device, dg));
                if (!can)
                    return setErr(c0, HPT_EDEVICE, "hpt_render_multi: device " + std::to_string(c0->device) +
                                                       " cannot access device " + std::to_string(dg) + " (no peer path)");
                const hipError_t pe = hipDeviceEnablePeerAccess(dg, 0);
                if (pe == hipErrorPeerAccessAlreadyEnabled) (void) hipGetLastError(); /* enabled by an earlier call */
                else if (pe != hipSuccess)
                    return setErr(c0, HPT_EDEVICE, "hipDeviceEnablePeerAccess(" + std::to_string(dg) +
                                                       "): " + hipGetErrorString(pe));
            }
            float4 *stage = c0->mstage + (size_t) (g - 1) * pixels;
            HIPCHK(c0, hipMemcpyPeerAsync(stage, c0->device, ctxs[g]->mfilm, dg, pixels * 16, c0->peerStreams[g - 1]));
            HIPCHK(c0, hipEventRecord(c0->peerEvents[g - 1], c0->peerStreams[g - 1]));
        }
        for (int g = 1; g < n; ++g) {
            HIPCHK(c0, hipStreamWaitEvent(c0->stream, c0->peerEvents[g - 1], 0));
            HIPCHK(c0, hpt_launch_film_add(c0->mfilm, c0->mstage + (size_t) (g - 1) * pixels, pixels, c0->stream));
        }
    }
    HIPCHK(c0, hipMemcpyAsync(film, c0->mfilm, pixels * 16, hipMemcpyDeviceToHost, c0->stream));
    HIPCHK(c0, hipStreamSynchronize(c0->stream));
    return HPT_OK;
}

int hpt_block_deal(int width, int height, int n_shards, const double *weights, int32_t *shard_of_block) {
    if (width <= 0 || height <= 0 || n_shards <= 0 || !shard_of_block) return HPT_EINVAL;
    const int nbx = (width + HPT_BLOCK - 1) / HPT_BLOCK, nby = (height + HPT_BLOCK - 1) / HPT_BLOCK;
    std::vector<double> w;
    if (weights) w.assign(weights, weights + (size_t) nbx * nby);
    /* the deal's sort needs a strict weak order: no NaN (and, as hpt_set_block_weights, no negative
       or infinite weight) */
    for (double x : w)
        if (!(x >= 0.0) || !std::isfinite(x)) return HPT_EINVAL;
    const std::vector<int> s = dealBlocks(nbx, nby, n_shards, w);
    for (size_t i = 0; i < s.size(); ++i) shard_of_block[i] = s[i];
    return HPT_OK;
}

int hpt_set_block_weights(hpt_context *c, const double *weights, int n_blocks) {
    if (!c || n_blocks < 0 || (n_blocks > 0 && !weights)) return HPT_EINVAL;
    for (int i = 0; i < n_blocks; ++i)
        if (!(weights[i] >= 0.0) || !std::isfinite(weights[i]))
            return setErr(c, HPT_EINVAL, "block weights must be finite and >= 0");
    c->blockWeights.assign(weights, weights + n_blocks);
    c->weightsVersion++;
    c->schedules.clear(); /* a shard's waves change with the deal: their bounce schedules do too */
    return HPT_OK;
}

int hpt_get_block_costs(hpt_context *c, uint64_t *costs, int n_blocks) {
    if (!c || !costs || n_blocks < 0) return HPT_EINVAL;
    std::memset(costs, 0, (size_t) n_blocks * sizeof(uint64_t));
    if (c->device == HPT_HOST_ONLY || !c->dBlockCost || c->ownBlocks.empty()) return HPT_OK;
    HIPCHK(c, hipSetDevice(c->device));
    const size_t words = (size_t) HPT_COST_STRIPES * c->ownCap;
    std::vector<uint32_t> local(words);
    HIPCHK(c, hipStreamSynchronize(c->stream));
    HIPCHK(c, hipMemcpy(local.data(), c->dBlockCost, words * 4, hipMemcpyDeviceToHost));
    HIPCHK(c, hipMemset(c->dBlockCost, 0, words * 4));
    for (size_t k = 0; k < c->ownBlocks.size(); ++k) {
        uint64_t sum = 0; /* the stripes of block k */
        for (int st = 0; st < HPT_COST_STRIPES; ++st) sum += local[(size_t) st * c->ownCap + k];
        if ((int) c->ownBlocks[k] < n_blocks) costs[c->ownBlocks[k]] = sum;
    }
    return HPT_OK;
}

int hpt_get_stats(hpt_context *c, hpt_stats *o) {
    if (!c || !o) return HPT_EINVAL;
    *o = c->stats;
    return HPT_OK;
}

int64_t hpt_get_hair(hpt_context *c, float *xyz, uint8_t *starts) {
    if (!c) return HPT_EINVAL;
    int64_t n = (int64_t) c->hair.vertexCount();
    if (xyz) std::memcpy(xyz, c->hair.xyz.data(), (size_t) n * 12);
    if (starts) std::memcpy(starts, c->hair.starts.data(), c->hair.starts.size());
    return n;
}

int hpt_get_kdtree(hpt_context *c, uint32_t *nodes, int64_t *n_nodes, uint32_t *indices, int64_t *n_indices,
                   float aabb[6]) {
    if (!c || !n_nodes || !n_indices) return HPT_EINVAL;
    *n_nodes = (int64_t) c->tree.nodes.size();
    *n_indices = (int64_t) c->tree.prims.size();
    if (nodes) std::memcpy(nodes, c->tree.nodes.data(), c->tree.nodes.size() * 8);
    if (indices)
        for (size_t i = 0; i < c->tree.prims.size(); ++i) indices[i] = c->tree.segFirstVertex[c->tree.prims[i]];
    if (aabb)
        for (int i = 0; i < 3; ++i) {
            aabb[i] = c->tree.aabbMin[i];
            aabb[3 + i] = c->tree.aabbMax[i];
        }
    return HPT_OK;
}

int hpt_get_pretest_records(hpt_context *c, uint32_t *records, int64_t *n_records, float *radius,
                            uint64_t *n_pass) {
    if (!c || !n_records) return HPT_EINVAL;
    static_assert(sizeof(HptSegQ) == 16, "hairpt.h documents 16-byte records");
    const size_t n = c->tree.leafQ.size();
    *n_records = (int64_t) n;
    if (records) std::memcpy(records, c->tree.leafQ.data(), n * sizeof(HptSegQ));
    if (radius) *radius = c->tree.preRadius;
    if (n_pass) *n_pass = c->tree.prePassRecords;
    return HPT_OK;
}

int hpt_get_envmap(hpt_context *c, float *rgb, int *w, int *h) {
    if (!c || !w || !h) return HPT_EINVAL;
    *w = c->env.w;
    *h = c->env.h;
    if (rgb) std::memcpy(rgb, c->env.rgb.data(), c->env.rgb.size() * 4);
    return HPT_OK;
}

int hpt_get_camera(hpt_context *c, float s2c[16], float dx[3], float dy[3]) {
    if (!c || !s2c || !dx || !dy) return HPT_EINVAL;
    if (!c->haveCamera) return setErr(c, HPT_ESTATE, "no camera");
    HptCamera cam;
    try {
        setupCamera(c->desc, cam);
    } catch (const std::exception &e) {
        return setErr(c, HPT_EINVAL, e.what());
    }
    std::memcpy(s2c, cam.s2c, sizeof(cam.s2c));
    std::memcpy(dx, cam.dx, sizeof(cam.dx));
    std::memcpy(dy, cam.dy, sizeof(cam.dy));
    return HPT_OK;
}

int hpt_get_marschner_tables(hpt_context *c, float *nR, float *nTT, float *nTRT, float *fdr, float *trans,
                             float *specw) {
    if (!c || !c->prepared || c->sc.bsdf.kind != HPT_BSDF_MARSCHNER)
        return setErr(c, HPT_ESTATE, "no marschner bsdf prepared");
    const MarschnerHost &m = c->mar[c->desc.shapes.empty() ? 0 : c->desc.shapes[0].bsdf];
    float *outs[3] = {nR, nTT, nTRT};
    for (int l = 0; l < 3; ++l)
        if (outs[l])
            for (size_t i = 0; i < m.table[l].size(); ++i) {
                outs[l][3 * i] = m.table[l][i].x;
                outs[l][3 * i + 1] = m.table[l][i].y;
                outs[l][3 * i + 2] = m.table[l][i].z;
            }
    if (fdr) *fdr = m.fdr;
    if (trans) std::memcpy(trans, m.trans.data(), std::min<size_t>(100, m.trans.size()) * 4);
    if (specw) *specw = m.specularSamplingWeight;
    return HPT_OK;
}

int hpt_get_roughplastic_params(hpt_context *c, float *params, float *trans, int *trans_size) {
    if (!c || !c->prepared || c->sc.bsdf.kind != HPT_BSDF_ROUGHPLASTIC || c->rp.empty())
        return setErr(c, HPT_ESTATE, "no roughplastic bsdf prepared");
    const RoughPlasticHost &h = c->rp[c->desc.shapes.empty() ? 0 : c->desc.shapes[0].bsdf];
    const HptRoughPlastic &p = h.p;
    if (params) {
        const float v[16] = {(float) p.type, (float) p.sampleVisible, (float) p.nonlinear, p.alpha, p.exponent, p.eta,
                             p.invEta2, p.specularSamplingWeight, p.diffuse[0], p.diffuse[1], p.diffuse[2],
                             p.specular[0], p.specular[1], p.specular[2], p.fdr, (float) h.trans.size()};
        std::memcpy(params, v, sizeof(v));
    }
    if (trans_size) *trans_size = (int) h.trans.size();
    if (trans) std::memcpy(trans, h.trans.data(), h.trans.size() * 4);
    return HPT_OK;
}

/* ---- batch helpers ---- */
} /* extern "C" */
namespace {
struct Scratch {
    std::vector<void *> ptrs;
    ~Scratch() {
        for (void *p : ptrs) (void) hipFree(p);
    }
    template <typename T> T *in(const T *src, size_t n) {
        void *p = nullptr;
        if (hipMalloc(&p, std::max<size_t>(n * sizeof(T), 16)) != hipSuccess) return nullptr;
        ptrs.push_back(p);
        if (src && n) (void) hipMemcpy(p, src, n * sizeof(T), hipMemcpyHostToDevice);
        return (T *) p;
    }
};
template <typename T> void fetch(T *dst, const T *src, size_t n) {
    if (dst) (void) hipMemcpy(dst, src, n * sizeof(T), hipMemcpyDeviceToHost);
}
} // namespace
extern "C" {

int hpt_sobol_batch(hpt_context *c, int m, int n, const uint32_t *frame, const uint32_t *px, const uint32_t *py,
                    const uint32_t *dim, uint64_t *oi, float *ov) {
    if (!c || !c->prepared) return setErr(c, HPT_ESTATE, "prepare first");
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context has no device");
    /* the kernel indexes the tables by m and dim: reject what they do not hold */
    const int rows = (int) std::min(c->vdc.size(), c->vdcInv.size()) / HPT_SOBOL_BITS;
    if (n < 0 || m < 0 || m > rows) return setErr(c, HPT_EINVAL, "Sobol look-up resolution out of range");
    for (int i = 0; i < n; ++i)
        if (dim[i] >= HPT_SOBOL_DIMS)
            return setErr(c, HPT_EINVAL, "Lookup dimension exceeds the direction number table size!");
    HIPCHK(c, hipSetDevice(c->device));
    Scratch S;
    const uint32_t *df = S.in(frame, n), *dx = S.in(px, n), *dy = S.in(py, n), *dd = S.in(dim, n);
    uint64_t *di = S.in<uint64_t>(nullptr, n);
    float *dv = S.in<float>(nullptr, n);
    HIPCHK(c, hpt_launch_sobol_batch(c->sc, m, n, df, dx, dy, dd, di, dv, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    fetch(oi, di, n);
    fetch(ov, dv, n);
    return HPT_OK;
}

int hpt_camera_batch(hpt_context *c, int n, const float *pos, float *oo, float *od, float *omint, float *omaxt) {
    if (!c || !c->prepared) return setErr(c, HPT_ESTATE, "prepare first");
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context has no device");
    HIPCHK(c, hipSetDevice(c->device));
    Scratch S;
    const float *dp = S.in(pos, 2 * (size_t) n);
    float *o = S.in<float>(nullptr, 3 * (size_t) n), *d = S.in<float>(nullptr, 3 * (size_t) n);
    float *a = S.in<float>(nullptr, n), *b = S.in<float>(nullptr, n);
    HIPCHK(c, hpt_launch_camera_batch(c->sc, n, dp, o, d, a, b, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    fetch(oo, o, 3 * (size_t) n);
    fetch(od, d, 3 * (size_t) n);
    fetch(omint, a, n);
    fetch(omaxt, b, n);
    return HPT_OK;
}

int hpt_trace_batch(hpt_context *c, int n, const float *o, const float *d, const float *mint, const float *maxt,
                    int flags, float *ot, int32_t *oiv, float *op, uint8_t *oh) {
    const int shadow = flags & HPT_TRACE_SHADOW;
    if (!c || !c->prepared) return setErr(c, HPT_ESTATE, "prepare first");
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context has no device");
    HIPCHK(c, hipSetDevice(c->device));
    Scratch S;
    const float *a = S.in(o, 3 * (size_t) n), *b = S.in(d, 3 * (size_t) n), *mi = S.in(mint, n), *ma = S.in(maxt, n);
    float *dt = S.in<float>(nullptr, n), *dp = S.in<float>(nullptr, 3 * (size_t) n);
    int32_t *ds = S.in<int32_t>(nullptr, n);
    uint8_t *dh = S.in<uint8_t>(nullptr, n);
    uint32_t *cur = S.in<uint32_t>(nullptr, HPT_CURSORS * HPT_CURSOR_STRIDE);
    if (int rf = clearFault(c)) return rf;
    HIPCHK(c, hpt_launch_trace_batch(c->sc, n, a, b, mi, ma, flags, dt, ds, dp, dh, cur, c->stream));
    if (int rf = checkFault(c)) return rf;
    if (shadow) {
        fetch(oh, dh, n);
    } else {
        fetch(ot, dt, n);
        fetch(op, dp, 3 * (size_t) n);
        std::vector<int32_t> seg(n);
        fetch(seg.data(), ds, n);
        if (oiv)
            for (int i = 0; i < n; ++i) oiv[i] = seg[i] < 0 ? -1 : (int32_t) c->tree.segFirstVertex[seg[i]];
    }
    return HPT_OK;
}

int hpt_bsdf_batch(hpt_context *c, int n, const float *wi, const float *wo, const float *u, float *oe, float *op,
                   float *owo, float *ow, float *osp, uint32_t *ot) {
    if (!c || !c->prepared) return setErr(c, HPT_ESTATE, "prepare first");
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context has no device");
    HIPCHK(c, hipSetDevice(c->device));
    Scratch S;
    const float *a = S.in(wi, 3 * (size_t) n), *b = S.in(wo, 3 * (size_t) n), *uu = S.in(u, 2 * (size_t) n);
    float *de = S.in<float>(nullptr, 3 * (size_t) n), *dp = S.in<float>(nullptr, n);
    float *dwo = S.in<float>(nullptr, 3 * (size_t) n), *dw = S.in<float>(nullptr, 3 * (size_t) n);
    float *dsp = S.in<float>(nullptr, n);
    uint32_t *dt = S.in<uint32_t>(nullptr, n);
    HIPCHK(c, hpt_launch_bsdf_batch(c->sc, n, a, b, uu, de, dp, dwo, dw, dsp, dt, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    fetch(oe, de, 3 * (size_t) n);
    fetch(op, dp, n);
    fetch(owo, dwo, 3 * (size_t) n);
    fetch(ow, dw, 3 * (size_t) n);
    fetch(osp, dsp, n);
    fetch(ot, dt, n);
    return HPT_OK;
}

int hpt_env_batch(hpt_context *c, int n, const float *refp, const float *u, const float *dq, float *od, float *ov,
                  float *op, float *odist, float *oe, float *oep) {
    if (!c || !c->prepared) return setErr(c, HPT_ESTATE, "prepare first");
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context has no device");
    HIPCHK(c, hipSetDevice(c->device));
    Scratch S;
    const float *a = S.in(refp, 3 * (size_t) n), *uu = S.in(u, 2 * (size_t) n), *q = S.in(dq, 3 * (size_t) n);
    float *dd = S.in<float>(nullptr, 3 * (size_t) n), *dv = S.in<float>(nullptr, 3 * (size_t) n);
    float *dp = S.in<float>(nullptr, n), *ddist = S.in<float>(nullptr, n), *de = S.in<float>(nullptr, 3 * (size_t) n);
    float *dep = S.in<float>(nullptr, n);
    HIPCHK(c, hpt_launch_env_batch(c->sc, n, a, uu, q, dd, dv, dp, ddist, de, dep, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    fetch(od, dd, 3 * (size_t) n);
    fetch(ov, dv, 3 * (size_t) n);
    fetch(op, dp, n);
    fetch(odist, ddist, n);
    fetch(oe, de, 3 * (size_t) n);
    fetch(oep, dep, n);
    return HPT_OK;
}

int hpt_env_eval_filtered(hpt_context *c, int n, const float *d, const float *rx, const float *ry, float *out_rgb) {
    if (!c || !c->prepared) return setErr(c, HPT_ESTATE, "prepare first");
    if (c->device == HPT_HOST_ONLY) return setErr(c, HPT_EDEVICE, "host-only context has no device");
    HIPCHK(c, hipSetDevice(c->device));
    Scratch S;
    const float *a = S.in(d, 3 * (size_t) n), *b = S.in(rx, 3 * (size_t) n), *q = S.in(ry, 3 * (size_t) n);
    float *dout = S.in<float>(nullptr, 3 * (size_t) n);
    HIPCHK(c, hpt_launch_env_filtered_batch(c->sc, n, a, b, q, dout, c->stream));
    HIPCHK(c, hipStreamSynchronize(c->stream));
    fetch(out_rgb, dout, 3 * (size_t) n);
    return HPT_OK;
}

int hpt_get_env_level(hpt_context *c, int level, float *rgb, int *w, int *h) {
    if (!c || !c->prepared) return setErr(c, HPT_ESTATE, "prepare first");
    const int n = (int) c->env.levelW.size();
    if (level < 0 || level >= n) return n;
    if (w) *w = c->env.levelW[level];
    if (h) *h = c->env.levelH[level];
    if (rgb) {
        const HptF4 *t = &c->env.mip[c->env.levelOff[level]];
        for (size_t i = 0; i < (size_t) c->env.levelW[level] * c->env.levelH[level]; ++i) {
            rgb[3 * i] = t[i].x;
            rgb[3 * i + 1] = t[i].y;
            rgb[3 * i + 2] = t[i].z;
        }
    }
    return n;
}

} /* extern "C" */
