/*
 * hpt_device.h -- data layout shared by the host builder and the gfx950
 * kernels of the wavefront hair path tracer.
 *
 * Everything here is POD.  The host fills these structures once per scene
 * (hpt_prepare) and uploads them to HBM; kernels receive the scene by value.
 */
#ifndef HPT_DEVICE_H
#define HPT_DEVICE_H
#include <stdint.h>

/* 16-byte vector used for coalesced dwordx4 traffic (host-compatible POD) */
struct __attribute__((aligned(16))) HptF4 {
    float x, y, z, w;
};

#define HPT_AZ_RES 64          /* marschner_diffuse.cpp:66 AzimuthalResolution */
#define HPT_SOBOL_DIMS 1024    /* sobolseq.h:33 */
#define HPT_SOBOL_BITS 52      /* sobolseq.h:34 */
#define HPT_BLOCK 32           /* mitsuba.cpp:144 block size */
#define HPT_FILTER_RES 31      /* rfilter.h:28 MTS_FILTER_RESOLUTION */

/* BSDF type flags (render/bsdf.h:224-285) */
#define HPT_ENULL 0x00001u
#define HPT_EDIFFUSE_REFLECTION 0x00002u
#define HPT_EGLOSSY_REFLECTION 0x00008u
#define HPT_EDELTA_REFLECTION 0x00020u
#define HPT_EDELTA (0x00001u | 0x00020u | 0x00040u)

/* One hair segment, everything the fp64 cylinder/miter test needs
 * (hair.cpp:485-548) precomputed on the host in double exactly as the
 * reference computes it per test: v1, axis = normalize(v2 - v1), miter
 * normals n1/n2 (hair.cpp:578-596), v2.  128 bytes = one cache line. */
struct HptSegment {
    double v1[3];
    double axis[3];
    double n1[3];
    double n2[3];
    double v2[3];
    uint32_t iv;   /* first vertex index (reference prim id, for parity) */
    uint32_t shape;/* hair shape the segment belongs to */
};

/* fp32 shadow of a segment for the conservative pre-test (32 bytes), stored
 * in leaf order (one record per leaf reference, so a leaf's candidates are
 * contiguous and need no index indirection).  The ray line must pass within
 * radius of the axis line for the fp64 quadratic to have real roots; the
 * pre-test rejects only when fp32 says the distance exceeds the radius by far
 * more than its rounding error, so the set of segments reaching the exact
 * fp64 test is a superset of those that can hit. */
struct HptSegF {
    float v1[3];
    float axis[3];
    uint32_t seg;  /* segment index (into HptScene::segs) */
    float radius;  /* its shape's radius */
};

/* 16-byte pre-test record of the per-lane traversal (k_trace), leaf order:
 * the segment's first vertex and its axis oct-encoded (u 16 bits, v 15 bits:
 * one dwordx4 per record instead of 24 of HptSegF's 32 bytes), bit 31 a pass
 * flag.  The quantised axis turns the pre-test line by an angle theta; a
 * record's bound is its shape's radius widened by its axial reach (up to the
 * miter planes) times sin(theta).  HptScene::preRadius covers every bound but
 * those of the flagged records, whose bound exceeds their shape's radius by
 * more than 5 % (a fold: a miter plane almost parallel to the axis) and which
 * pass every pre-test (kdtree_build.cpp), so a fold no longer widens the test
 * of every record.  Decoded by axisOctDecode (hpt_render.hip) and its host
 * twin in kdtree_build.cpp, with the same fp32 operations. */
#define HPT_PRE_PASS 0x80000000u
struct HptSegQ {
    float v1[3];
    uint32_t axisOct; /* bits 0-15 u, 16-30 v, 31 pass flag */
};

/* kd-tree node, 8 bytes (gkdtree.h:452-583 layout with absolute child index):
 *   inner: w0 = (left << 2) | axis, w1 = float bits of split; right = left + 1
 *   leaf : w0 = 0x80000000 | primStart, w1 = primEnd (indices into prim list) */
struct HptNode {
    uint32_t w0, w1;
};

/* Two-level kd node (32 bytes): a binary node fused with its two children,
 * so the device descent fetches once per two levels.
 *   w[0] split of the top node, w[1]/w[2] splits of its left/right child
 *   w[3] axis_top | axis_L << 2 | axis_R << 4 | L_inner << 6 | R_inner << 7
 *   w[4..7] grandchild refs LL, LR, RL, RR (a leaf child fills both of its
 *   slots with its own ref).  A ref is a node index (bit 31 clear) or a
 *   leaf: 0x80000000 | count << 24 | first primitive, with count ==
 *   HPT_LEAF_INLINE_MAX meaning "look up (first, end) in leafTable[index]". */
#define HPT_LEAF_INLINE_MAX 127u
struct HptNode4 {
    uint32_t w[8];
};

struct HptCamera {
    float s2c[16];      /* sampleToCamera, row-major (perspective.cpp:155) */
    float dx[3], dy[3]; /* near-plane position differentials (perspective.cpp:160-163) */
    float diffScale;    /* 1/sqrt(sampleCount): scaleDifferential (integrator.cpp:143-144) */
    float toWorld[16];  /* camera-to-world, row-major */
    float origin[3];    /* toWorld * (0, 0, 0): every camera ray's origin (setupCamera) */
    float invResX, invResY, nearClip, farClip;
    float resolution;   /* Sobol pixel resolution (sobol.cpp:147-158) */
    int width, height;
    uint32_t logRes;
};

struct HptMarschner {
    const HptF4 *table[3];     /* R, TT, TRT: 64x64 RGB(+pad), index x + y*64 */
    const float *cdf[3];        /* InterpolatedDistribution1D cdfs: 64 dists x 65 */
    const float *sums[3];       /* 64 */
    const float *trans;         /* external rough transmittance 1D slice */
    int transSize;
    float fdr, invEta2, specularSamplingWeight;
    float vR, vTT, vTRT, scaleAngleRad;
    float diffuse[3];
    /* longitudinalM's per-lobe constants (marschner_diffuse.cpp:364-374), R, TT, TRT: 1 / v, and
       log(1 / (2 v)) when v < 0.1, else 2 v sinh(1 / v) */
    float lobeInvV[3], lobeK[3];
};

struct HptKajiyaKay {
    float kd[3], ks[3];
    float exponent, specularSamplingWeight;
};

/* marschnerdielectric (marschnerdielectric.cpp:145-659): a thin dielectric
 * sheet -- delta reflection about the fiber, straight pass-through (ENull) and
 * a diffuse component whose solid-angle eval is identically zero there.
 * thindielectric (thindielectric.cpp:70-252) is the same sampler without the
 * diffuse choice (specularSamplingWeight = 1) and without NEE. */
struct HptMarschnerDielectric {
    float eta, specularSamplingWeight;
    float specR[3], specT[3];
};

/* diffuse (diffuse.cpp:60-140) */
struct HptDiffuse {
    float refl[3];
};

/* roughplastic (roughplastic.cpp:196-296): isotropic microfacet coating over
 * a diffuse base, constant textures */
struct HptRoughPlastic {
    int type;                   /* 0 beckmann, 1 ggx, 2 phong (microfacet.h:48-58) */
    int sampleVisible, nonlinear;
    float alpha, exponent;      /* exponent: Phong (computePhongExponent) */
    float eta, invEta2, specularSamplingWeight;
    float diffuse[3], specular[3];
    const float *trans;         /* external rough transmittance 1D slice (eta, alpha) */
    int transSize;
    float fdr;                  /* 1 - internal (1/eta) diffuse transmittance at alpha */
};

/* One BSDF instance.  kind: 0 marschner, 1 kajiyakay, 2 roughplastic,
 * 3 marschnerdielectric, 4 thindielectric, 5 diffuse.  smooth: the combined
 * type has an ESmooth component, so path.cpp:175 samples the emitter (and
 * consumes two sample dimensions) before the BSDF. */
#define HPT_BSDF_MARSCHNER 0
#define HPT_BSDF_KAJIYAKAY 1
#define HPT_BSDF_ROUGHPLASTIC 2
#define HPT_BSDF_MARSCHNERDIELECTRIC 3
#define HPT_BSDF_THINDIELECTRIC 4
#define HPT_BSDF_DIFFUSE 5
#define HPT_MAX_SHAPES 64
struct HptBsdf {
    int kind, smooth;
    HptMarschner mar;
    HptKajiyaKay kk;
    HptRoughPlastic rp;
    HptMarschnerDielectric md;
    HptDiffuse df;
};

struct HptShape {
    float radius;
    int bsdf;
};

/* EWA-filtered environment lookups for camera rays (envmap.cpp:391-406,
 * mipmap.h:629-834): the MIP pyramid's levels, and the 64-entry Gaussian LUT */
#define HPT_EWA_LUT 64
#define HPT_ENV_GUIDE 64
struct HptMipLevel {
    int w, h, off;
    float ratioX, ratioY; /* level size / level-0 size (m_sizeRatio) */
};

struct HptEnvMap {
    const HptF4 *texel;        /* w*h, half-rounded RGB stored as float (= level 0 of mip) */
    const HptF4 *mip;          /* every MIP level, level l at levels[l].off */
    const HptMipLevel *levels;
    const float *ewaLut;       /* HPT_EWA_LUT */
    int nLevels;
    float maxAnisotropy;       /* 10 (envmap.cpp:142) */
    const float *cdfRows;       /* h+1 */
    const float *cdfCols;       /* h*(w+1) */
    const float *rowWeights;    /* h */
    /* guide tables of the CDF searches: guideRows[k] = lower_bound(cdfRows, k / HPT_ENV_GUIDE)
       (k = 0..HPT_ENV_GUIDE), guideCols likewise per row (h x (HPT_ENV_GUIDE + 1)) */
    const uint32_t *guideRows, *guideCols;
    int w, h;
    float normalization, scale, pixelSizeX, pixelSizeY;
    float bsCenter[3], bsRadius;
    int identity;
    float m[9], minv[9];
};

struct HptScene {
    HptCamera cam;
    const HptNode *nodes;
    const HptNode4 *nodes4;
    const uint32_t *leafTable;
    const HptSegF *leafF;       /* leaf primitive list (fp32 pre-test records) */
    const HptSegQ *leafQ;       /* the same list as 16-byte records (k_trace's leaf pass) */
    const uint32_t *leafSeg;    /* segment id per leaf entry */
    const HptSegment *segs;
    float aabbMin[3], aabbMax[3];
    float radius;               /* shape 0's radius (every shape's when nShapes == 1) */
    float maxRadius;            /* largest shape radius: bound for the conservative fp32 pre-test */
    float preRadius;            /* the HptSegQ pre-test's radius (flagged records pass, see HptSegQ) */
    HptBsdf bsdf;               /* shape 0's BSDF */
    /* several hair shapes (hair-curl): HptSegment::shape indexes shapes[],
       which gives the radius and the entry of bsdfs[] (both in HBM: a kernel
       argument indexed per lane would be copied to scratch) */
    int nShapes;
    const HptShape *shapes;
    const HptBsdf *bsdfs;
    HptEnvMap env;
    const uint32_t *sobol;      /* 1024 x 52 */
    uint32_t scramble;          /* low 32 bits of sampleTEA(scramble) (sobol.cpp:92-102), 0 = off */
    const uint64_t *vdc;        /* rows x 52 */
    const uint64_t *vdcInv;     /* rows x 52 */
    float tent[HPT_FILTER_RES + 1];
    float tentScale;
    int maxDepth, rrDepth, strictNormals, hideEmitters;
    uint32_t *fault;            /* device word: HPT_FAULT_* bits set by the traversal bounds */
    uint32_t maxLeafRounds;     /* traversal bounds of one ray (HPT_MAX_LEAF_ROUNDS / HPT_MAX_RESTARTS unless */
    uint32_t maxRestarts;       /*  lowered through hpt_set_traversal_bounds, a test hook) */
    uint32_t packetStack;       /* camera packets' stack entries (0 = the build's; hpt_set_packet_stack, a test hook) */
};

/* ---- triangle-mesh scenes (C1, models/teapot: obj.cpp / rectangle.cpp shapes, diffuse /
 * plastic / twosided BSDFs, checkerboard texture), rendered by k_mesh_paths (hpt_mesh.h).
 * Geometry lives in world space; the camera, sampler, environment and film come from the
 * HptScene of the same context. */

/* one triangle: Wald's projection record (triaccel.h:37-158; k = 3 marks a degenerate
 * triangle, which never hits) and the vertex indices of the hit-record fill.  64 bytes. */
struct HptTri {
    uint32_t k;
    float n_u, n_v, n_d, a_u, a_v, b_nu, b_nv, c_nu, c_nv;
    uint32_t i0, i1, i2; /* into HptMeshScene::p / n / uv */
    uint32_t mesh;       /* into HptMeshScene::meshes */
    uint32_t pad[2];
};

/* per TriMesh (trimesh.cpp): its BSDF and which vertex attributes it has */
struct HptMeshInfo {
    int bsdf, hasNormals, hasUV, pad;
};

/* rectangle.cpp:80-168: the world-to-object affine rows, the geometric frame, dpdu */
struct HptRect {
    float w2o[12];
    float s[3], t[3], n[3];
    float dpdu[3];
    int bsdf;
    int pad[3];
};

/* BVH node (32 bytes) over triangles and rectangles: count == 0 is an inner node whose
 * left child is the next node and whose right child is node a; a leaf holds the
 * primitive references prims[a, a + count) */
struct HptBvhNode {
    float mn[3];
    uint32_t a;
    float mx[3];
    uint32_t count;
};
#define HPT_PRIM_RECT 0x80000000u /* a primitive reference to rectangle (ref & ~HPT_PRIM_RECT) */

/* mesh-scene BSDF instance (diffuse.cpp:60-140 with a constant or checkerboard reflectance,
 * plastic.cpp:143-440, twosided.cpp:84-183 over the records nested[0..1]) */
#define HPT_MBSDF_DIFFUSE 0
#define HPT_MBSDF_PLASTIC 1
#define HPT_MBSDF_TWOSIDED 2
struct HptMeshBsdf {
    int kind, smooth;
    /* diffuse */
    int textured;
    float refl[3], color0[3], color1[3];
    float uoffset, voffset, uscale, vscale;
    /* plastic */
    int nonlinear;
    float eta, invEta2, fdrInt, specularSamplingWeight;
    float diffuse[3], specular[3];
    /* twosided */
    int nested[2];
};

/* k_mesh_paths' per-lane BVH stack entries (LDS): hpt_prepare refuses a BVH deeper than this - 1
   levels -- the median-split build is ~log2(primitives / 4) + 1 deep, 14 for the teapot */
#define HPT_MESH_STACK 32
struct HptMeshScene {
    const HptBvhNode *nodes;
    const uint32_t *prims;     /* leaf primitive references */
    const HptTri *tris;
    const HptRect *rects;
    const HptMeshInfo *meshes;
    const float *p, *n, *uv;   /* per vertex: 3, 3 (meshes with normals), 2 (meshes with uv) floats */
    const float *dpdu;         /* per triangle, 3 floats: computeUVTangents, or p1 - p0 without uv */
    const HptMeshBsdf *bsdfs;
    float aabbMin[3], aabbMax[3]; /* the scene bounds, enlarged as gkdtree.h:1213-1220 does */
    uint32_t nNodes, stackDepth; /* the BVH's depth bounds the traversal stack (HPT_MESH_STACK) */
};

#endif
