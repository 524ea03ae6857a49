/*
 * hpt_render.hip -- gfx950 wavefront kernels for the reference's `path`
 * integrator over the `hair` shape with the `marschner` / `kajiyakay` BSDFs.
 *
 * MIPathTracer::Li (src/integrators/path/path.cpp:119-294) is split at its
 * two ray casts.  One path = one lane; paths live in SoA slots in HBM and
 * are driven by index queues:
 *
 *   k_camera      sampler->generate + camera ray (integrator.cpp:165-178)
 *   k_trace       closest-hit rays (continuation) and any-hit shadow rays in
 *                 one launch; kd-tree traversal with an LDS stack and the
 *                 fp64 cylinder/miter test (hair.cpp:485-548)
 *   k_primary     primary misses -> environment (path.cpp:136-143)
 *   k_shade       its -> strictNormals, NEE sample + BSDF eval (:170-199),
 *                 BSDF sample (:206-221); emits one shadow ray + one
 *                 continuation ray per path
 *   k_post        env hit + MIS (:236-264), throughput, Russian roulette
 *                 (:270-286); survivors re-enter the shade queue
 *   k_splat/k_gather  deterministic tent-filter accumulation of all samples
 *                 into an RGBW film (imageblock.h:124-204)
 *
 * Queues are compacted with a wave64 ballot + one atomic per wave.  A
 * path's arithmetic never depends on its queue position, so results are
 * independent of compaction order.
 */
#include <hip/hip_runtime.h>

#include <algorithm>
#include <cstdlib>
#include <map>
#include <mutex>
#include <utility>
#include <vector>

#include "../hpt_device.h"
#include "hpt_kernels.h"
#include "hpt_math.h"

using namespace hk;

/* block size of the queue-producing kernels (k_camera, k_primary, k_shade, k_post) */
#ifndef HPT_SHADE_BLOCK
#define HPT_SHADE_BLOCK 256 /* k_shade: 4 waves/SIMD of registers; 256-thread blocks overlap better than 1024 (shade 20.9 -> 18.1 ms) */
#endif
#ifndef HPT_POST_BLOCK
#define HPT_POST_BLOCK 1024
#endif
#ifndef HPT_QBLOCK
#define HPT_QBLOCK 1024
#endif

namespace {

/* ------------------------------------------------------------------ */
/* Sobol sampler: sobolseq.h:43-58 (sampleSingle), :99-131 (look_up),   */
/* sobol.cpp:204-250 (setSampleIndex / next1D / next2D)                 */
/* ------------------------------------------------------------------ */
HD float sobolSample(const HptScene &sc, uint64_t index, uint32_t dim) {
    uint32_t result = sc.scramble;
    const uint32_t *m = sc.sobol + dim * HPT_SOBOL_BITS;
    uint32_t lo = (uint32_t) index, hi = (uint32_t) (index >> 32);
    for (int i = 0; lo; lo >>= 1, ++i)
        if (lo & 1u) result ^= m[i];
    for (int i = 32; hi; hi >>= 1, ++i)
        if (hi & 1u) result ^= m[i];
    return fminr((float) result * (1.0f / 4294967296.0f), kOneMinusEps);
}

/* sobolSample for a dimension that is the same across the wave (k_shade /
   k_post: all paths of a bounce have consumed the same number of dimensions,
   path.cpp's sampler->next1D/next2D order).  The dimension's 52 direction
   numbers are then read once for the wave and every index bit is applied
   with a select, instead of a per-lane loop of dependent table loads.  Falls
   back to sobolSample when the wave disagrees.  Same XOR of the same
   matrix rows as sobolseq.h:43-58. */
/* sobolSample for a per-lane dimension in a latency-bound kernel (k_tail: the lanes of a wave are
   at different bounces, so their dimensions differ): the dimension's 52 direction numbers are read
   as 16-byte loads issued together, and every index bit is applied with a select -- one round trip
   where sobolSample's loop waits on one table load per set bit.  Same XOR of the same rows. */
HD float sobolSampleRow(const HptScene &sc, uint64_t index, uint32_t dim) {
    const uint4 *__restrict__ row = reinterpret_cast<const uint4 *>(sc.sobol + dim * HPT_SOBOL_BITS); /* 208-B rows */
    const uint32_t lo = (uint32_t) index, hi = (uint32_t) (index >> 32);
    uint32_t result = sc.scramble;
    uint4 q[8];
#pragma unroll
    for (int k = 0; k < 8; ++k) q[k] = row[k];
#pragma unroll
    for (int k = 0; k < 8; ++k) {
        result ^= ((lo >> (4 * k)) & 1u) ? q[k].x : 0u;
        result ^= ((lo >> (4 * k + 1)) & 1u) ? q[k].y : 0u;
        result ^= ((lo >> (4 * k + 2)) & 1u) ? q[k].z : 0u;
        result ^= ((lo >> (4 * k + 3)) & 1u) ? q[k].w : 0u;
    }
    if (hi) { /* index bits 32-51: words 32-51 of the row */
#pragma unroll
        for (int k = 0; k < 5; ++k) {
            const uint4 r = row[8 + k];
            result ^= ((hi >> (4 * k)) & 1u) ? r.x : 0u;
            result ^= ((hi >> (4 * k + 1)) & 1u) ? r.y : 0u;
            result ^= ((hi >> (4 * k + 2)) & 1u) ? r.z : 0u;
            result ^= ((hi >> (4 * k + 3)) & 1u) ? r.w : 0u;
        }
    }
    return fminr((float) result * (1.0f / 4294967296.0f), kOneMinusEps);
}

/* LAT: a wave that disagrees on the dimension takes sobolSampleRow (k_tail) instead of sobolSample */
template <bool LAT = false>
HD float sobolSampleUniform(const HptScene &sc, uint64_t index, uint32_t dim) {
    const uint32_t d0 = __builtin_amdgcn_readfirstlane(dim);
    if (__ballot(dim != d0) != 0) return LAT ? sobolSampleRow(sc, index, dim) : sobolSample(sc, index, dim);
    const uint32_t *__restrict__ m = sc.sobol + d0 * HPT_SOBOL_BITS;
    const uint32_t lo = (uint32_t) index, hi = (uint32_t) (index >> 32);
    uint32_t result = sc.scramble;
#pragma unroll
    for (int i = 0; i < 32; ++i) result ^= ((lo >> i) & 1u) ? m[i] : 0u;
    if (__ballot(hi != 0) != 0) {
#pragma unroll
        for (int i = 32; i < HPT_SOBOL_BITS; ++i) result ^= ((hi >> (i - 32)) & 1u) ? m[i] : 0u;
    }
    return fminr((float) result * (1.0f / 4294967296.0f), kOneMinusEps);
}

HD uint64_t sobolLookUp(const HptScene &sc, uint32_t m, uint32_t frame, uint32_t px, uint32_t py) {
    uint64_t index = (uint64_t) frame << (m << 1);
    uint64_t delta = 0;
    const uint64_t *vdc = sc.vdc + (m - 1) * HPT_SOBOL_BITS;
    const uint64_t *inv = sc.vdcInv + (m - 1) * HPT_SOBOL_BITS;
    for (uint32_t c = 0; frame; frame >>= 1, ++c)
        if (frame & 1u) delta ^= vdc[c];
    const uint32_t sm = sc.scramble >> (32 - m); /* (scramble & 0xFFFFFFFF) >> (32 - m), m >= 1 */
    uint64_t b = (((uint64_t) (px ^ sm) << m) | (py ^ sm)) ^ delta;
    for (uint32_t c = 0; b; b >>= 1, ++c)
        if (b & 1u) index ^= inv[c];
    return index;
}

/* sobolLookUp for a wave whose m (the resolution's log2) is uniform and whose frames are below
   2^frameBits (frameBits uniform, <= 32): the same XOR of the same table columns, as selects over a
   uniform run of columns read eight at a time by the scalar unit, instead of per-lane loops that
   wait on one table load per set bit.  vdc_sobol_matrices[m - 1][c] < 2^m, so delta < 2^m and
   b < 2^(2m): columns from 2m on are never read (sobolseq.h:98-131) */
HD uint64_t sobolLookUpWave(const HptScene &sc, uint32_t m, uint32_t frame, uint32_t px, uint32_t py,
                            uint32_t frameBits) {
    const uint64_t *vdc = sc.vdc + (m - 1) * HPT_SOBOL_BITS;
    const uint64_t *inv = sc.vdcInv + (m - 1) * HPT_SOBOL_BITS;
    uint32_t delta = 0;
    for (uint32_t c0 = 0; c0 < frameBits; c0 += 8) { /* uniform bound; c0 + 7 < 52 */
        uint64_t col[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) col[k] = vdc[c0 + k];
#pragma unroll
        for (int k = 0; k < 8; ++k) delta ^= ((frame >> (c0 + k)) & 1u) ? (uint32_t) col[k] : 0u;
    }
    const uint32_t sm = sc.scramble >> (32 - m);
    const uint64_t b = (((uint64_t) (px ^ sm) << m) | (py ^ sm)) ^ delta;
    uint64_t index = (uint64_t) frame << (m << 1);
    for (uint32_t c0 = 0; c0 < 2 * m; c0 += 8) { /* columns past the row's 52 read as 0 (b has no such bits) */
        uint64_t col[8];
#pragma unroll
        for (int k = 0; k < 8; ++k) col[k] = (c0 + k < HPT_SOBOL_BITS) ? inv[c0 + k] : 0ull;
#pragma unroll
        for (int k = 0; k < 8; ++k) index ^= ((b >> (c0 + k)) & 1ull) ? col[k] : 0ull;
    }
    return index;
}

/* ------------------------------------------------------------------ */
/* Camera (perspective.cpp:271-298)                                     */
/* ------------------------------------------------------------------ */
HD V3 xformPoint(const float *M, V3 p) {
    float x = M[0] * p.x + M[1] * p.y + M[2] * p.z + M[3];
    float y = M[4] * p.x + M[5] * p.y + M[6] * p.z + M[7];
    float z = M[8] * p.x + M[9] * p.y + M[10] * p.z + M[11];
    float w = M[12] * p.x + M[13] * p.y + M[14] * p.z + M[15];
    if (w == 1.0f) return v3(x, y, z);
    return divs(v3(x, y, z), w);
}
HD V3 xformVector(const float *M, V3 v) {
    return v3(M[0] * v.x + M[1] * v.y + M[2] * v.z, M[4] * v.x + M[5] * v.y + M[6] * v.z,
              M[8] * v.x + M[9] * v.y + M[10] * v.z);
}

/* ------------------------------------------------------------------ */
/* Ray / AABB (aabb.h:308-338)                                          */
/* ------------------------------------------------------------------ */
HD bool aabbIntersect(const HptScene &sc, V3 o, V3 d, V3 rcp, float &nearT, float &farT) {
    nearT = -finf();
    farT = finf();
    for (int i = 0; i < 3; ++i) {
        float origin = o[i], mn = sc.aabbMin[i], mx = sc.aabbMax[i];
        if (d[i] == 0) {
            if (origin < mn || origin > mx) return false;
        } else {
            float t1 = (mn - origin) * rcp[i], t2 = (mx - origin) * rcp[i];
            if (t1 > t2) {
                float t = t1;
                t1 = t2;
                t2 = t;
            }
            nearT = fmaxr(t1, nearT);
            farT = fminr(t2, farT);
            if (!(nearT <= farT)) return false;
        }
    }
    return true;
}

/* ------------------------------------------------------------------ */
/* Hair segment test: HairKDTree::intersect (hair.cpp:485-548) in fp64  */
/* ------------------------------------------------------------------ */
/* Register-lean staging: the quadratic needs only v1/axis, the miter tests
   load n1/v1 and n2/v2 when they are reached, and the memory clobbers keep
   the scheduler from hoisting those loads (which would keep ~30 extra VGPRs
   live across the traversal loop).  The arithmetic is operation for
   operation the reference's (dot = x*x' + y*y' + z*z', no contraction). */
template <class RecP>
HD bool insideMiters(RecP rec, D3 q) {
    asm volatile("" ::: "memory");
    const D3 v1 = d3(rec[0], rec[1], rec[2]), n1 = d3(rec[6], rec[7], rec[8]);
    if (!(dot(q - v1, n1) >= 0)) return false;
    asm volatile("" ::: "memory");
    const D3 v2 = d3(rec[12], rec[13], rec[14]), n2 = d3(rec[9], rec[10], rec[11]);
    return dot(q - v2, n2) <= 0;
}

/* The fp64 ray and the quadratic of hair.cpp:496-517 for the segment record
   rec (15 doubles: v1, axis, n1, n2, v2).  The fp32 ray is passed through
   opaque moves so the fp64 copies are not kept live across the traversal
   loop: they are re-derived per exact test (rare: the fp32 pre-test passes
   ~2 segments per ray). */
template <class RecP>
HD bool segQuadratic(RecP rec, V3 of, V3 df, double r2, D3 &rayO, D3 &rayD, double &nearT, double &farT) {
    float ox = of.x, oy = of.y, oz = of.z, dx = df.x, dy = df.y, dz = df.z;
    asm volatile("" : "+v"(ox), "+v"(oy), "+v"(oz), "+v"(dx), "+v"(dy), "+v"(dz));
    rayO = d3(ox, oy, oz);
    rayD = d3(dx, dy, dz);
    const D3 axis = d3(rec[3], rec[4], rec[5]);
    const D3 relOrigin = rayO - d3(rec[0], rec[1], rec[2]);
    const D3 projOrigin = relOrigin - axis * dot(axis, relOrigin);
    const D3 projDirection = rayD - axis * dot(axis, rayD);
    const double A = dot(projDirection, projDirection);
    const double B = 2 * dot(projOrigin, projDirection);
    const double C = dot(projOrigin, projOrigin) - r2;
    return solveQuadraticDouble(A, B, C, nearT, farT);
}

/* HairKDTree::intersect (hair.cpp:485-548): t of the accepted root and which
   root it was (farRoot: the near root was outside the miters or before mint).
   The hit point is not formed here: segHitPoint re-derives it from the same
   root with the same operations, in the kernel that shades the hit, so the
   traversal kernels carry no fp64 point (fewer registers, no point record). */
/* rayO + rayD * t with the fp64 ray re-derived from the fp32 one (opaque
   moves: the conversions are redone here instead of keeping 12 registers of
   fp64 ray live across the quadratic's solve) */
HD D3 rayPointD(V3 of, V3 df, double t) {
    float ox = of.x, oy = of.y, oz = of.z, dx = df.x, dy = df.y, dz = df.z;
    asm volatile("" : "+v"(ox), "+v"(oy), "+v"(oz), "+v"(dx), "+v"(dy), "+v"(dz));
    return d3(ox, oy, oz) + d3(dx, dy, dz) * t;
}

template <class RecP>
HD bool segIntersectRec(RecP rec, V3 of, V3 df, double r2, float mint, float maxt, float &t, uint32_t &farRoot) {
    double nearT, farT;
    {
        D3 rayO, rayD;
        if (!segQuadratic(rec, of, df, r2, rayO, rayD, nearT, farT)) return false;
    }
    if (!(nearT <= (double) maxt && farT >= (double) mint)) return false;
    if (nearT >= (double) mint && insideMiters(rec, rayPointD(of, df, nearT))) {
        t = (float) nearT;
        farRoot = 0;
        return true;
    }
    if (insideMiters(rec, rayPointD(of, df, farT))) {
        if (farT > (double) maxt) return false;
        t = (float) farT;
        farRoot = 1;
        return true;
    }
    return false;
}

HD bool segIntersect(const HptSegment *__restrict__ segs, uint32_t s, V3 of, V3 df, double r2, float mint,
                     float maxt, float &t, uint32_t &farRoot) {
    return segIntersectRec(reinterpret_cast<const double *>(segs + s), of, df, r2, mint, maxt, t, farRoot);
}

/* radius of segment s's hair shape (uniform branch: one shape in every shipped scene but hair-curl) */
HD float segRadius(const HptScene &sc, uint32_t s) {
    return sc.nShapes > 1 ? sc.shapes[sc.segs[s].shape].radius : sc.radius;
}

/* the hit point of an accepted root (hair.cpp:519-541: rayO + rayD * root, rounded to float) */
HD V3 segHitPoint(const HptScene &sc, uint32_t s, V3 of, V3 df, uint32_t farRoot) {
    const float rad = segRadius(sc, s);
    const double r2 = (double) (rad * rad); /* Float product (hair.cpp:500) */
    D3 rayO, rayD;
    double nearT = 0, farT = 0;
    segQuadratic(reinterpret_cast<const double *>(sc.segs + s), of, df, r2, rayO, rayD, nearT, farT);
    const D3 q = rayO + rayD * (farRoot ? farT : nearT);
    return v3((float) q.x, (float) q.y, (float) q.z);
}

/* Conservative fp32 pre-test (see HptSegF): false only when the ray line
   provably passes farther than radius from the segment's axis line, i.e.
   when the fp64 quadratic of segIntersect has no real root.  With
   n = d x axis, the exact condition is |w.n| <= r |n| (w = o - v1).  Error
   budget (u = 2^-24, |d| = |axis| = 1): rounding of w, of the cross product
   and of the fp32 axis against the fp64 one moves the computed |w.n| by at
   most 11u |w|_1 and r|n| by at most 12u r; the test keeps a 4x margin on
   both (3e-6 (r + |w|_1)) and never divides by |n|, so it holds for rays
   of any direction, near-parallel ones included. */

HD bool segMayHit(const float4 a, const float4 b, V3 o, V3 d, float r) {
    const float wx = o.x - a.x, wy = o.y - a.y, wz = o.z - a.z;
    const float ax = a.w, ay = b.x, az = b.y; /* axis */
    const float nx = d.y * az - d.z * ay, ny = d.z * ax - d.x * az, nz = d.x * ay - d.y * ax;
    const float nn = nx * nx + ny * ny + nz * nz;
    const float wn = fabsf(wx * nx + wy * ny + wz * nz);
    /* v_sqrt_f32 (<= 1 ulp) is covered by the 1e-6 relative margin */
    return wn <= r * __builtin_amdgcn_sqrtf(nn) * 1.000001f + 3e-6f * (r + fabsf(wx) + fabsf(wy) + fabsf(wz));
}

/* HptSegQ: the oct-decoded axis (kdtree_build.cpp's axisOctDecode does the same fp32 operations on
   the host to bound the quantisation angle) and the pre-test on it.  The axis is not unit length
   (|axis| in [1/sqrt(3), 1]): the test is scale-invariant in the axis except for the absolute rounding
   margin, which a shorter axis only makes looser.  preRadius covers the quantised axis's turn over
   the reach of every record but the flagged ones, which pass (HptSegQ). */
HD V3 axisOctDecode(uint32_t q) {
    const float u = (float) (q & 0xffffu) * (2.0f / 65535.0f) - 1.0f;
    const float v = (float) ((q >> 16) & 0x7fffu) * (2.0f / 32767.0f) - 1.0f;
    const float z = 1.0f - fabsf(u) - fabsf(v);
    const float fx = (1.0f - fabsf(v)) * (u >= 0.0f ? 1.0f : -1.0f);
    const float fy = (1.0f - fabsf(u)) * (v >= 0.0f ? 1.0f : -1.0f);
    return v3(z < 0.0f ? fx : u, z < 0.0f ? fy : v, z);
}
HD bool segMayHitQ(const uint4 q, V3 o, V3 d, float preRadius) {
    const V3 a = axisOctDecode(q.w);
    return segMayHit(make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), a.x),
                     make_float4(a.y, a.z, 0.0f, 0.0f), o, d, preRadius) |
           ((int) q.w < 0); /* HPT_PRE_PASS */
}
/* the same as a 0 / 1 word: the test's select falls back to the record's pass bit (one v_cndmask
   where a bool OR of the two costs a compare and a mask merge more) */
HD uint32_t segMayHitQBit(const uint4 q, V3 o, V3 d, float preRadius) {
    const V3 a = axisOctDecode(q.w);
    return segMayHit(make_float4(__uint_as_float(q.x), __uint_as_float(q.y), __uint_as_float(q.z), a.x),
                     make_float4(a.y, a.z, 0.0f, 0.0f), o, d, preRadius)
               ? 1u
               : q.w >> 31; /* HPT_PRE_PASS */
}

/* adaptive ray epsilon: skdtree.cpp:126-129 (closest) / :213-216 (shadow) */
HD float adaptiveMint(V3 o, float mint, bool shadow) {
    if (mint != kEpsilon) return mint;
    float m = fmaxr(fmaxr(fabsf(o.x), fabsf(o.y)), fabsf(o.z));
    if (!shadow) m = fmaxr(m, kEpsilon);
    return mint * m;
}

/* ------------------------------------------------------------------ */
/* kd-tree traversal (front-to-back, LDS ring stack with kd-restart),   */
/* as a resumable per-lane state machine so persistent waves can refill */
/* finished lanes with new rays.  Primitive tests use the ray's [mint,  */
/* best t] interval exactly like rayIntersectHavran (sahkdtree3.h:      */
/* 275-297), so the closest hit does not depend on the tree or on the   */
/* traversal order.                                                      */
/* ------------------------------------------------------------------ */
/* first item of cursor shard s when n items are split over HPT_CURSORS contiguous shards */
HD uint32_t shardLo(uint32_t n, uint32_t s) { return (uint32_t) ((uint64_t) n * s / HPT_CURSORS); }

struct TraceRay {
    V3 o, d, rcp;
    float mint, maxt;   /* ray interval after the scene-AABB clip and adaptive epsilon */
    float tmin, tmax;   /* interval of the current subtree */
    float tHit;
    uint32_t node, top, segHit;
    int sp;             /* mint, maxt, rcp are read from LDS by traceRound (stashRay) */
    uint32_t cnt;       /* leaves visited | kd-restarts << 20 (traceRound's bounds) */
    bool lost, found, shadow;
};

/* ShapeKDTree::rayIntersect / rayIntersect(shadow) prologue: scene AABB
   clip + adaptive ray epsilon (skdtree.cpp:112-141, :207-226).  False when
   there is nothing to traverse (the ray misses). */
HD bool beginRay(const HptScene &sc, TraceRay &r, V3 o, V3 d, float rmint, float rmaxt, bool shadow) {
    r.o = o;
    r.d = d;
    r.rcp = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    r.shadow = shadow;
    r.found = false;
    r.tHit = finf();
    r.segHit = 0;
    r.mint = r.maxt = 0.0f; /* defined for stashRay even when the ray misses */
    float mint, maxt;
    if (!aabbIntersect(sc, o, d, r.rcp, mint, maxt)) return false;
    const float rayMinT = adaptiveMint(o, rmint, shadow);
    if (rayMinT > mint) mint = rayMinT;
    if (rmaxt < maxt) maxt = rmaxt;
    if (!(maxt > mint)) return false;
    r.mint = r.tmin = mint;
    r.maxt = r.tmax = r.tHit = maxt;
    r.node = 0;
    r.top = 0;
    r.sp = 0;
    r.lost = false;
    return true;
}

struct TraceCounters {
    uint32_t nodes = 0, prims = 0, exact = 0, nodeSlots = 0, primSlots = 0;
    uint32_t shadowNodes = 0, shadowPrims = 0; /* the part of nodes / prims spent on shadow rays */
    uint32_t binNodes = 0; /* binary kd-node visits (Havran's count: inner nodes entered + leaves) */
};

HD bool waveLeader() { return __lane_id() == (uint32_t) (__ffsll((unsigned long long) __ballot(1)) - 1); }

/* One round: descend to the next leaf, test its segments, pop.  Returns
   true when the ray is finished (r.found / r.tHit / r.segHit hold
   the answer). */
/* Per-lane LDS area of the traversal: the STACK ring-stack entries, then
   HPT_RAY_ROWS rows holding the ray's cold values, so that none of them
   occupies a register while the fp64 exact test runs (that test is the
   register peak of the traversal kernels; registers decide how many waves a
   SIMD holds, and the latency-bound traversal runs faster with more):
     row STACK+0  rcp.x, rcp.y       read once per round
     row STACK+1  rcp.z, key         key: what the IO's finish() needs (path id / ray index)
     row STACK+2  mint, maxt         mint read by the exact tests, maxt at a kd-restart
   (recomputing rcp each round instead, 80 B of LDS per lane, measured
   slower: DESIGN.md 5).  Row k of lane i is stk[k * stride]. */
#define HPT_RAY_ROWS 3
#define HPT_ROW_KEY 1 /* .y */
#define HPT_ROW_MM 2
#define HPT_CNT_RESTART (1u << 20)
template <int STACK>
HD void stashRay(uint2 *stk, int stride, TraceRay &r, uint32_t key) {
    stk[STACK * stride] = make_uint2(__float_as_uint(r.rcp.x), __float_as_uint(r.rcp.y));
    stk[(STACK + 1) * stride] = make_uint2(__float_as_uint(r.rcp.z), key);
    stk[(STACK + HPT_ROW_MM) * stride] = make_uint2(__float_as_uint(r.mint), __float_as_uint(r.maxt));
    r.cnt = 0u;
    /* the rows must be re-read, not forwarded from these stores (forwarding keeps the values in registers) */
    asm volatile("" ::: "memory");
}
template <int STACK> HD uint32_t rayKey(const uint2 *stk, int stride) { return stk[(STACK + HPT_ROW_KEY) * stride].y; }
/* leaves visited / kd-restarts of the lane's current ray */
HD uint32_t rayLeaves(const TraceRay &r) { return r.cnt & (HPT_CNT_RESTART - 1u); }
HD uint32_t rayRestarts(const TraceRay &r) { return r.cnt / HPT_CNT_RESTART; }

template <int STACK, bool STATS, bool LAT = false>
HD bool traceRound(const HptScene &sc, TraceRay &r, uint2 *stk, int stride, TraceCounters &tc) {
    static_assert((STACK & (STACK - 1)) == 0, "the ring stack index is masked");
    static_assert(!(LAT && STATS), "the latency-mode leaf pass keeps no traversal counters");
    const float4 *__restrict__ leafF = reinterpret_cast<const float4 *>(sc.leafF);
    const uint4 *__restrict__ leafQ = reinterpret_cast<const uint4 *>(sc.leafQ);
    /* the ray as plain values: selecting among struct members by axis would be
       folded into a dynamically addressed load and push the state to scratch */
    const uint2 cr0 = stk[STACK * stride], cr1 = stk[(STACK + 1) * stride];
    const V3 o = r.o, d = r.d, rcp = v3(__uint_as_float(cr0.x), __uint_as_float(cr0.y), __uint_as_float(cr1.x));
    /* hard bound so every wave drains even on a malformed tree; the call fails loudly */
    {
        const uint32_t cnt = r.cnt + 1u;
        r.cnt = cnt;
        if ((cnt & (HPT_CNT_RESTART - 1u)) > sc.maxLeafRounds) {
            atomicOr(sc.fault, HPT_FAULT_LEAVES);
            return true;
        }
    }
    /* descent over two-level nodes (HptNode4): one 32-byte fetch decides the
       top split and the split of each child the ray interval reaches; the
       binary traversal's front-to-back order and intervals are kept exactly
       (the second side's children are pushed as the binary traversal would
       push that side and later split it) */
    const uint4 *__restrict__ nodes4 = reinterpret_cast<const uint4 *>(sc.nodes4);
    uint32_t ref = r.node;
    auto push = [&](uint32_t what, float tmaxOf) {
        stk[(r.top & (STACK - 1)) * stride] = make_uint2(what, __float_as_uint(tmaxOf));
        r.lost = r.lost | (r.sp == STACK);
        r.top += 1u;
        r.sp += (r.sp < STACK) ? 1 : 0;
    };
    while (!(ref & 0x80000000u)) {
        if (STATS) {
            ++tc.nodes;
            tc.shadowNodes += r.shadow ? 1u : 0u;
            if (waveLeader()) tc.nodeSlots += 64;
        }
        const uint4 na = nodes4[2 * ref], nb = nodes4[2 * ref + 1];
#if HPT_EXP_NODE_PAD
        /* experiment (make variant): 16 more bytes per node fetch, waited on with the node */
        {
            const uint4 nc = nodes4[2 * ref + 2];
            asm volatile("" ::"v"(nc.x), "v"(nc.y), "v"(nc.z), "v"(nc.w));
        }
#endif
        const uint32_t flags = na.w;
        /* top split */
        const uint32_t ax0 = flags & 3u;
        const float sp0 = __uint_as_float(na.x);
        const float oa0 = ax0 == 0 ? o.x : (ax0 == 1 ? o.y : o.z);
        const float da0 = ax0 == 0 ? d.x : (ax0 == 1 ? d.y : d.z);
        const float ra0 = ax0 == 0 ? rcp.x : (ax0 == 1 ? rcp.y : rcp.z);
        const float ts0 = (sp0 - oa0) * ra0;
        const bool below0 = (oa0 < sp0) | ((oa0 == sp0) & (da0 <= 0.0f));
        const bool near0 = !(ts0 <= r.tmax) | (ts0 <= 0.0f);
        const bool far0 = !near0 & (ts0 < r.tmin);
        const bool both0 = !(near0 | far0);
        const uint32_t firstSide = below0 ? 0u : 1u;
        const uint32_t sideA = far0 ? (firstSide ^ 1u) : firstSide, sideB = firstSide ^ 1u;
        const float tA = both0 ? ts0 : r.tmax;
        /* side B (visited after side A) is pushed first */
        if (both0) {
            const bool innerB = (flags >> (6 + sideB)) & 1u;
            const uint32_t rB0 = sideB ? nb.z : nb.x, rB1 = sideB ? nb.w : nb.y;
            if (innerB) {
                const uint32_t ax = (flags >> (2 + 2 * sideB)) & 3u;
                const float spl = __uint_as_float(sideB ? na.z : na.y);
                const float oa = ax == 0 ? o.x : (ax == 1 ? o.y : o.z);
                const float da = ax == 0 ? d.x : (ax == 1 ? d.y : d.z);
                const float ra = ax == 0 ? rcp.x : (ax == 1 ? rcp.y : rcp.z);
                const float ts = (spl - oa) * ra;
                const bool below = (oa < spl) | ((oa == spl) & (da <= 0.0f));
                const uint32_t f = below ? rB0 : rB1, sc2 = below ? rB1 : rB0;
                const bool nearB = !(ts <= r.tmax) | (ts <= 0.0f);
                const bool farB = !nearB & (ts < ts0);
                if (!(nearB | farB)) {
                    push(sc2, r.tmax);
                    push(f, ts);
                } else {
                    push(farB ? sc2 : f, r.tmax);
                }
            } else {
                push(rB0, r.tmax);
            }
        }
        /* side A, over [tmin, tA] */
        const bool innerA = (flags >> (6 + sideA)) & 1u;
        if (STATS) tc.binNodes += 1u + (innerA ? 1u : 0u) + ((both0 && ((flags >> (6 + sideB)) & 1u)) ? 1u : 0u);
        const uint32_t rA0 = sideA ? nb.z : nb.x, rA1 = sideA ? nb.w : nb.y;
        if (innerA) {
            const uint32_t ax = (flags >> (2 + 2 * sideA)) & 3u;
            const float spl = __uint_as_float(sideA ? na.z : na.y);
            const float oa = ax == 0 ? o.x : (ax == 1 ? o.y : o.z);
            const float da = ax == 0 ? d.x : (ax == 1 ? d.y : d.z);
            const float ra = ax == 0 ? rcp.x : (ax == 1 ? rcp.y : rcp.z);
            const float ts = (spl - oa) * ra;
            const bool below = (oa < spl) | ((oa == spl) & (da <= 0.0f));
            const uint32_t f = below ? rA0 : rA1, sc2 = below ? rA1 : rA0;
            const bool nearA = !(ts <= tA) | (ts <= 0.0f);
            const bool farA = !nearA & (ts < r.tmin);
            const bool bothA = !(nearA | farA);
            if (bothA) push(sc2, tA);
            ref = farA ? sc2 : f;
            r.tmax = bothA ? ts : tA;
        } else {
            ref = rA0;
            r.tmax = tA;
        }
    }
    if (STATS) {
        ++tc.nodes;
        ++tc.binNodes;
        tc.shadowNodes += r.shadow ? 1u : 0u;
        if (waveLeader()) tc.nodeSlots += 64;
    }
    uint32_t leafFirst = ref & 0x00ffffffu, leafLast = leafFirst + ((ref >> 24) & 0x7fu);
#if HPT_EXP_LEAF_RT
    /* experiment (make variant): one more dependent 4-byte fetch before a leaf's records */
    {
        uint32_t z;
        asm volatile("v_and_b32 %0, 0, %1" : "=v"(z) : "v"(sc.leafSeg[leafFirst]));
        leafFirst += z;
        leafLast += z;
    }
#endif
    if (((ref >> 24) & 0x7fu) == HPT_LEAF_INLINE_MAX) {
        leafLast = sc.leafTable[2 * leafFirst + 1];
        leafFirst = sc.leafTable[2 * leafFirst];
    }
    /* leaf, two passes: the fp32 pre-test marks candidates in a bit mask
       (32 records per chunk; the next record is fetched while the current one
       is tested), then the exact fp64 test runs on the marked ones -- the
       prefetched records are dead by then, so the fp64 test's registers do
       not stack on top of them.  Outside latency mode the pre-test reads the
       16-byte HptSegQ records (one dwordx4 per record: the kernel's vector
       memory path is busy ~3/4 of its cycles) */
    const uint32_t first = leafFirst, last = leafLast;
    if (LAT) {
        /* latency mode (k_tail: few waves, registers to spare): every record of a
           chunk of 8 is requested at once and each candidate's whole fp64 record in
           one go, so a leaf costs two memory round trips instead of one per record
           and three per exact test.  Same tests in the same order: identical hits. */
        for (uint32_t c0 = first; c0 < last; c0 += 8) {
            const uint32_t n = min(last - c0, 8u);
            float4 ra[8], rb[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k)
                if (k < n) {
                    ra[k] = leafF[2 * (c0 + k)];
                    rb[k] = leafF[2 * (c0 + k) + 1];
                }
            uint32_t mask = 0;
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k)
                if (k < n && segMayHit(ra[k], rb[k], o, d, rb[k].w)) mask |= 1u << k; /* its own radius */
            uint32_t segOf[8];
#pragma unroll
            for (uint32_t k = 0; k < 8; ++k) segOf[k] = __float_as_uint(rb[k].z);
            while (mask) {
                const uint32_t k = (uint32_t) (__ffs(mask) - 1);
                mask &= mask - 1;
                uint32_t s = segOf[0];
#pragma unroll
                for (uint32_t q = 1; q < 8; ++q) s = k == q ? segOf[q] : s;
                const float rad = segRadius(sc, s);
                const double r2 = (double) (rad * rad); /* Float product (hair.cpp:500) */
                const double *src = reinterpret_cast<const double *>(sc.segs + s);
                double rec[15];
#pragma unroll
                for (int q = 0; q < 15; ++q) rec[q] = src[q];
                float t;
                uint32_t far;
                const float mint = __uint_as_float(stk[(STACK + HPT_ROW_MM) * stride].x);
                if (segIntersectRec(rec, o, d, r2, mint, r.tHit, t, far)) {
                    r.found = true;
                    if (r.shadow) return true;
                    r.tHit = t;
                    r.segHit = s | (far << 31);
                }
            }
        }
    } else
    for (uint32_t c0 = first; c0 < last; c0 += 32) {
        const uint32_t c1 = min(last, c0 + 32);
        uint32_t mask = 0;
        uint4 nq = leafQ[c0];
        for (uint32_t e = c0; e < c1; ++e) {
            const uint4 fq = nq;
            if (e + 1 < c1) nq = leafQ[e + 1];
            if (STATS) {
                ++tc.prims;
                tc.shadowPrims += r.shadow ? 1u : 0u;
                if (waveLeader()) tc.primSlots += 64;
            }
            mask |= segMayHitQBit(fq, o, d, sc.preRadius) << (e - c0);
        }
        while (mask) {
            const uint32_t e = c0 + (uint32_t) (__ffs(mask) - 1);
            mask &= mask - 1;
            const uint32_t s = sc.leafSeg[e];
            const float rad = segRadius(sc, s);
            const double r2 = (double) (rad * rad); /* Float product (hair.cpp:500) */
            if (STATS) ++tc.exact;
            float t;
            uint32_t far;
            const float mint = __uint_as_float(stk[(STACK + HPT_ROW_MM) * stride].x);
            if (segIntersect(sc.segs, s, o, d, r2, mint, r.tHit, t, far)) {
                r.found = true;
                if (r.shadow) return true;
                r.tHit = t;
                r.segHit = s | (far << 31);
            }
        }
    }
    if (r.found && r.tHit <= r.tmax) return true;
    if (r.sp == 0) {
        const float maxt = __uint_as_float(stk[(STACK + HPT_ROW_MM) * stride].y);
        if (!r.lost || r.tmax >= maxt) return true;
        const uint32_t cnt = r.cnt + HPT_CNT_RESTART;
        r.cnt = cnt;
        if (cnt / HPT_CNT_RESTART > sc.maxRestarts) {
            atomicOr(sc.fault, HPT_FAULT_RESTARTS);
            return true;
        }
        /* kd-restart from the root for the remaining interval */
        r.lost = false;
        r.node = 0;
        r.tmin = r.tmax;
        r.tmax = maxt;
        return false;
    }
    r.top--;
    r.sp--;
    const uint2 e = stk[(r.top & (STACK - 1)) * stride];
    r.node = e.x;
    r.tmin = r.tmax;
    r.tmax = __uint_as_float(e.y);
    return r.tmin > r.tHit;
}

/* segment id / far-root flag of a finished closest-hit ray (TraceRay::segHit = id | far << 31) */
HD uint32_t hitSegment(const TraceRay &r) { return r.segHit & 0x7fffffffu; }
HD uint32_t hitFarRoot(const TraceRay &r) { return r.segHit >> 31; }

#ifndef HPT_REFILL
#define HPT_REFILL 16 /* idle lanes that trigger a refill of the wave */
#endif

/* Drain splitting.  Once a persistent wave's claims find the queue empty, its
   finished lanes would idle until the wave's slowest ray ends, and the launch
   ends with the slowest wave.  Instead an idle lane takes over the far part of
   a running ray's remaining interval: the ray (donor) keeps [its start, m] and
   the helper traces [m, end] from the root, the way a kd-restart resumes an
   interval.  The members of a split ray (same key, same kind) each know their
   interval's start (the LDS mint row, also the lower bound of their exact
   tests); the ray's answer is the hit of the member with the lowest start that
   found one, once every member below it has finished without one (shadow ray:
   any member's hit; no hit: every member finished).  Primitive tests accept
   t in [start, best] per member, so the union over members finds the same
   closest hit as one traversal over [mint, maxt] (hair.cpp:485-548: the root
   accepted for a segment depends only on which of its roots lie in the
   interval, and a root below a member's start is in a lower member's). */
#ifndef HPT_DRAIN_SPLIT
#define HPT_DRAIN_SPLIT 1
#endif
#ifndef HPT_SPLIT_MIN
#define HPT_SPLIT_MIN 8 /* idle lanes that trigger a split step (or as many idle as running) */
#endif
/* v of lane src (ds_bpermute; unlike __shfl no lane-id arithmetic, which would keep the
   lane id live through the traversal) */
HD int fromLane(int v, uint32_t src) { return __builtin_amdgcn_ds_bpermute((int) (src << 2), v); }
HD uint32_t fromLane(uint32_t v, uint32_t src) { return (uint32_t) fromLane((int) v, src); }
HD float fromLane(float v, uint32_t src) { return __int_as_float(fromLane(__float_as_int(v), src)); }
/* position of the k-th (0-based) set bit of m (k < popcount(m)) */
HD uint32_t selectBit(uint64_t m, uint32_t k) {
    uint32_t pos = 0, c = (uint32_t) __popc((uint32_t) m), x;
    if (k >= c) {
        k -= c;
        x = (uint32_t) (m >> 32);
        pos = 32;
    } else {
        x = (uint32_t) m;
    }
#pragma unroll
    for (int w = 16; w >= 1; w >>= 1) {
        c = (uint32_t) __popc(x & ((1u << w) - 1u));
        if (k >= c) {
            k -= c;
            x >>= w;
            pos += (uint32_t) w;
        }
    }
    return pos;
}

/* Persistent traversal: each wave keeps its 64 lanes busy by claiming new
   rays whenever HPT_REFILL lanes have finished.  The work range is split
   into HPT_CURSORS contiguous shards, each with its own cursor on its own
   128-byte line; a wave starts on shard (wave id mod HPT_CURSORS) and moves
   to the next one when its shard runs dry, so claims spread over 64
   addresses instead of serialising on one (device-scope atomics to a single
   word cost ~10 ns each) and neighbouring rays stay together.
   IO supplies count(), begin(k, r) (load ray k; false = nothing to trace),
   key() (after begin: what finish needs, kept in LDS while the ray is
   traced) and finish(key, r).  Every wave exits once all shards are exhausted and its
   lanes have drained, so the grid always completes. */
#include "hpt_probes.h"
/* Drain splitting (HPT_DRAIN_SPLIT).  Once a persistent wave's claims find the queue empty, an
   idle lane takes over part of a running ray of its wave (see above); the members of a split
   ray (same LDS key, same kind) each trace their interval and decide() gives the ray its
   answer once it is decided.  Wave-uniform state: the lanes of split rays, and those of them
   that have finished their interval while the ray's answer is still open.  Used by the drain of
   tracePersistent and by k_tail, whose few live rays leave most lanes of a wave idle. */
template <int STACK>
struct RaySplitter {
    uint2 *stk;
    int stride;
    uint64_t splitM = 0, waitM = 0;
    uint32_t rot = 0; /* rotates which running rays get helpers first */
    /* the j-th of n pieces of [a, b] starts here (the same expression on the donor and the helper) */
    static __device__ __forceinline__ float pieceStart(float a, float b, uint32_t j, uint32_t n) {
        return j >= n ? b : a + (b - a) * ((float) j / (float) n);
    }
    /* the lane index, recomputed where it is needed (kept live from the top it costs the
       traversal a register) */
    static __device__ __forceinline__ uint32_t laneNow() {
        uint32_t l;
        asm volatile("v_mbcnt_lo_u32_b32 %0, -1, 0\n\tv_mbcnt_hi_u32_b32 %0, -1, %0" : "=v"(l));
        return l;
    }
    /* whether this lane's ray is a member of a split ray (its answer is decide()'s) */
    __device__ __forceinline__ bool member() const { return ((splitM >> laneNow()) & 1u) != 0; }
    __device__ __forceinline__ void step(TraceRay &r, bool &active) {
        const uint32_t lane = laneNow();
        const uint64_t actM = __ballot(active), idleM = ~(actM | waitM);
        const float end = __uint_as_float(stk[(STACK + HPT_ROW_MM) * stride].y);
        const float b = fminr(r.tHit, end);
        /* what a helper takes: the bottom stack entry (the farthest pending subtree, entered at
           t0 = the end of the entry above it) and everything after it, or with an empty stack
           the far half of the remaining interval, from the root */
        const bool fromStack = r.sp > 0;
        uint32_t node = 0;
        float t0, t1 = end;
        if (fromStack) {
            const uint32_t bot = r.top - (uint32_t) r.sp;
            const uint2 e = stk[(bot & (STACK - 1)) * stride];
            node = e.x;
            t1 = __uint_as_float(e.y);
            t0 = r.sp > 1 ? __uint_as_float(stk[((bot + 1u) & (STACK - 1)) * stride].y) : r.tmax;
        } else {
            t0 = pieceStart(r.tmin, b, 1u, 2u);
        }
        const bool elig = active && t0 < b && t0 > r.tmin;
        const uint64_t eM = __ballot(elig);
        const uint32_t nE = (uint32_t) __popcll(eM), nI = (uint32_t) __popcll(idleM);
        if (nE == 0 || nI == 0 || (nI < HPT_SPLIT_MIN && nI < nE)) return;
        const uint32_t nS = min(nE, nI); /* helpers this step, one per donor */
        const uint32_t rE = __builtin_amdgcn_mbcnt_hi((uint32_t) (eM >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) eM, 0u));
        const uint32_t rI =
            __builtin_amdgcn_mbcnt_hi((uint32_t) (idleM >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) idleM, 0u));
        const uint32_t rr = rot % nE;
        const bool give = elig && (rE + nE - rr) % nE < nS;
        const bool take = ((idleM >> lane) & 1u) && rI < nS;
        const uint32_t donor = take ? selectBit(eM, (rI + rr) % nE) : lane;
        const uint2 cr0 = stk[STACK * stride], cr1 = stk[(STACK + 1) * stride];
        const uint32_t dnode = (uint32_t) fromLane((int) node, donor);
        const float dt0 = fromLane(t0, donor), dt1 = fromLane(t1, donor), de = fromLane(end, donor);
        const int dflags = fromLane((r.shadow ? 1 : 0) | (fromStack ? 2 : 0) | (r.lost ? 4 : 0), donor);
        const float ox = fromLane(r.o.x, donor), oy = fromLane(r.o.y, donor), oz = fromLane(r.o.z, donor);
        const float dx = fromLane(r.d.x, donor), dy = fromLane(r.d.y, donor), dz = fromLane(r.d.z, donor);
        const uint32_t c0 = (uint32_t) fromLane((int) cr0.x, donor), c1 = (uint32_t) fromLane((int) cr0.y, donor);
        const uint32_t c2 = (uint32_t) fromLane((int) cr1.x, donor), key = (uint32_t) fromLane((int) cr1.y, donor);
        if (give) {
            /* the donor keeps [its start, t0] */
            if (fromStack) {
                r.sp -= 1;
                r.lost = false; /* entries lost beyond the bottom one are now the helper's */
            }
            stk[(STACK + HPT_ROW_MM) * stride].y = __float_as_uint(t0);
            r.maxt = t0;
            if (!(r.found && r.tHit <= t0)) {
                r.found = false;
                r.tHit = t0;
            }
        }
        if (take) {
            /* the helper: [t0, the donor's end]; the last part ends at the ray's own end, not at
               a hit found beyond t0 (that t is the fp64 root rounded to float, maybe below it) */
            const bool stackPart = (dflags & 2) != 0;
            r.o = v3(ox, oy, oz);
            r.d = v3(dx, dy, dz);
            r.rcp = v3(__uint_as_float(c0), __uint_as_float(c1), __uint_as_float(c2));
            r.shadow = (dflags & 1) != 0;
            r.found = false;
            r.segHit = 0;
            r.node = stackPart ? dnode : 0u;
            r.mint = r.tmin = dt0;
            r.tmax = stackPart ? dt1 : de;
            r.maxt = r.tHit = de;
            /* a kd-restart covers what follows the stolen subtree */
            r.lost = stackPart && ((dflags & 4) != 0 || dt1 < de);
            r.top = 0;
            r.sp = 0;
            r.cnt = 0;
            stk[STACK * stride] = make_uint2(c0, c1);
            stk[(STACK + 1) * stride] = make_uint2(c2, key);
            stk[(STACK + HPT_ROW_MM) * stride] = make_uint2(__float_as_uint(dt0), __float_as_uint(de));
            active = true;
        }
        splitM |= __ballot(give) | __ballot(take);
        rot += nS;
        asm volatile("" ::: "memory"); /* traceRound re-reads the rows (see stashRay) */
    }
    /* newW: split lanes that finished their interval this round */
    template <class IO>
    __device__ __forceinline__ uint32_t decide(const HptScene &sc, IO &io, TraceRay &r, bool &active, uint64_t newW) {
        uint32_t nU = 0;
        const uint32_t lane = laneNow();
        waitM |= newW;
        const uint2 kr = stk[(STACK + 1) * stride], mm = stk[(STACK + HPT_ROW_MM) * stride];
        const uint32_t myKey = kr.y;
        const float lo = __uint_as_float(mm.x);
        const int myKind = r.shadow ? 1 : 0;
        while (newW) { /* wave-uniform: one split ray per pass */
            const int L = __ffsll((unsigned long long) newW) - 1;
            const uint32_t K = (uint32_t) __builtin_amdgcn_readlane((int) myKey, L);
            const int S = __builtin_amdgcn_readlane(myKind, L);
            const bool mem = ((splitM >> lane) & 1u) && myKey == K && myKind == S;
            const uint64_t memM = __ballot(mem);
            const bool w = (waitM >> lane) & 1u;
            const uint64_t fnd = __ballot(mem && w && r.found);
            int F = -1;
            float minLo = finf();
            for (uint64_t m = fnd; m; m &= m - 1) {
                const int l = __ffsll((unsigned long long) m) - 1;
                const float v = __int_as_float(__builtin_amdgcn_readlane(__float_as_int(lo), l));
                if (v < minLo) {
                    minLo = v;
                    F = l;
                }
            }
            /* shadow ray: any hit decides; closest: no running member below the lowest hit */
            const bool decided = S ? (fnd != 0 || (memM & ~waitM) == 0) : __ballot(mem && !w && lo < minLo) == 0;
            if (decided) {
                if ((int) lane == (F >= 0 ? F : L)) nU += io.finish(sc, K, r);
                if (mem) active = false;
                splitM &= ~memM;
                waitM &= ~memM;
            } else if (F >= 0) {
                /* members above the lowest hit cannot give the answer */
                const uint64_t dropM = __ballot(mem && lo > minLo);
                if ((dropM >> lane) & 1u) active = false;
                splitM &= ~dropM;
                waitM &= ~dropM;
            }
            newW &= ~memM;
        }
        return nU;
    }
    /* trace every active lane's ray to its answer, idle lanes helping (IO::finish writes it);
       returns the unoccluded shadow rays finished */
    template <bool LAT, class IO, class Probe>
    __device__ __forceinline__ uint32_t drain(const HptScene &sc, IO &io, TraceRay &r, bool &active, TraceCounters &tc,
                                              Probe &probe) {
        uint32_t nU = 0;
        while (true) {
            step(r, active);
            if (__ballot(active) == 0) break;
            probe.onDrainRound(__ballot(active));
            bool fin = false;
            if (active && traceRound<STACK, false, LAT>(sc, r, stk, stride, tc)) {
                fin = true;
                if (!member()) nU += io.finish(sc, rayKey<STACK>(stk, stride), r);
                active = false;
            }
            if (splitM) nU += decide(sc, io, r, active, __ballot(fin) & splitM);
        }
        return nU;
    }
};

template <int STACK, bool STATS, bool SPLIT = (!STATS && HPT_DRAIN_SPLIT), class IO>
__device__ __forceinline__ void tracePersistent(const HptScene &sc, IO &io, uint32_t *cursors, uint2 *stk,
                                                uint32_t *stats) {
    TraceProbe probe;
    const uint32_t lane = __lane_id();
    TraceRay r;
    TraceCounters tc;
    uint32_t nC = 0, nS = 0, nU = 0;
    uint32_t maxRounds = 0, maxRestarts = 0, restartRays = 0, restarts = 0; /* STATS: per-ray tails */
    auto rayDone = [&](uint32_t leaves, uint32_t rs) {
        if (STATS) {
            maxRounds = max(maxRounds, leaves);
            maxRestarts = max(maxRestarts, rs);
            restartRays += rs > 0 ? 1u : 0u;
            restarts += rs;
        }
    };
    bool active = false, exhausted = false;
    uint32_t shard = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % HPT_CURSORS;
    int tried = 0;
    static_assert(!(SPLIT && STATS), "the counted traversal is not split");
    while (true) {
        const uint64_t idle = __ballot(!active);
        if (!exhausted && __popcll(idle) >= HPT_REFILL) {
            const uint32_t n = (uint32_t) __popcll(idle);
            uint32_t start = 0, got = 0;
            while (true) { /* wave-uniform */
                const uint32_t size = io.shardSize(shard);
                uint32_t base = 0;
                if (lane == 0) base = atomicAdd(&cursors[shard * HPT_CURSOR_STRIDE], n);
                base = __shfl(base, 0);
                if (base < size) {
                    start = base; /* the first item claimed: its offset in the shard */
                    got = min(n, size - base);
                    break;
                }
                if (++tried >= HPT_CURSORS) {
                    exhausted = true;
                    probe.onExhausted(n);
                    break;
                }
                shard = (shard + 1) % HPT_CURSORS;
            }
            probe.onClaim(got);
            if (!active) {
                /* idle lanes below this one (v_mbcnt: no 64-bit lane mask kept live across the loop) */
                const uint32_t rank =
                    __builtin_amdgcn_mbcnt_hi((uint32_t) (idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) idle, 0u));
                if (rank < got) {
                    active = io.begin(sc, io.item(shard, start + rank), r);
                    if (STATS) {
                        nC += r.shadow ? 0u : 1u;
                        nS += r.shadow ? 1u : 0u;
                    }
                    /* the LDS rows are written unconditionally, right where they were
                       computed (under a branch, mint / maxt stayed live across the miss
                       path and were spilled); a miss never reads them */
                    stashRay<STACK>(stk, (int) blockDim.x, r, io.key());
                    if (!active) {
                        nU += io.finish(sc, io.key(), r);
                        rayDone(0u, 0u);
                    }
                }
            }
        }
        if (SPLIT && exhausted) break; /* the drain loop below */
        if (__ballot(active) == 0) {
            if (exhausted) break;
            continue;
        }
        if (exhausted) probe.onDrainStart();
        if (active && traceRound<STACK, STATS>(sc, r, stk, (int) blockDim.x, tc)) {
            nU += io.finish(sc, rayKey<STACK>(stk, (int) blockDim.x), r);
            if (STATS) rayDone(rayLeaves(r), rayRestarts(r));
            active = false;
        }
    }
    if (SPLIT && __ballot(active) != 0) {
        probe.onDrainStart();
        RaySplitter<STACK> split{stk, (int) blockDim.x};
        nU += split.template drain<false>(sc, io, r, active, tc, probe);
    }
    probe.finish();
    if (STATS) {
        /* traversal counters for the algorithmic byte model:
           [0] node visits [1] primitive tests [2] closest rays [3] shadow rays
           [4] unoccluded shadow rays [5] exact fp64 segment tests (pre-test
           survivors) [6]/[7] SIMD slots of the node / primitive loops (64
           per wave iteration: [0]/[6] is the lane utilisation); per-wave
           reduction, one atomic each */
        for (int off = 32; off > 0; off >>= 1) {
            tc.nodes += __shfl_down(tc.nodes, off);
            tc.prims += __shfl_down(tc.prims, off);
            tc.exact += __shfl_down(tc.exact, off);
            tc.nodeSlots += __shfl_down(tc.nodeSlots, off);
            tc.primSlots += __shfl_down(tc.primSlots, off);
            nC += __shfl_down(nC, off);
            nS += __shfl_down(nS, off);
            nU += __shfl_down(nU, off);
            tc.shadowNodes += __shfl_down(tc.shadowNodes, off);
            tc.shadowPrims += __shfl_down(tc.shadowPrims, off);
            tc.binNodes += __shfl_down(tc.binNodes, off);
            maxRounds = max(maxRounds, (uint32_t) __shfl_down(maxRounds, off));
            maxRestarts = max(maxRestarts, (uint32_t) __shfl_down(maxRestarts, off));
            restartRays += __shfl_down(restartRays, off);
            restarts += __shfl_down(restarts, off);
        }
        if (lane == 0) {
            unsigned long long *st = (unsigned long long *) stats;
            atomicAdd(&st[0], (unsigned long long) tc.nodes);
            atomicAdd(&st[1], (unsigned long long) tc.prims);
            atomicAdd(&st[2], (unsigned long long) nC);
            atomicAdd(&st[3], (unsigned long long) nS);
            atomicAdd(&st[4], (unsigned long long) nU);
            atomicAdd(&st[5], (unsigned long long) tc.exact);
            atomicAdd(&st[6], (unsigned long long) tc.nodeSlots);
            atomicAdd(&st[7], (unsigned long long) tc.primSlots);
            /* [8]/[9] max rounds (leaves visited) / kd-restarts of one ray, [10] rays that
               restarted, [11] restarts */
            atomicMax(&st[8], (unsigned long long) maxRounds);
            atomicMax(&st[9], (unsigned long long) maxRestarts);
            atomicAdd(&st[10], (unsigned long long) restartRays);
            atomicAdd(&st[11], (unsigned long long) restarts);
            /* [19]/[20] node visits / primitive tests of shadow rays */
            atomicAdd(&st[19], (unsigned long long) tc.shadowNodes);
            atomicAdd(&st[20], (unsigned long long) tc.shadowPrims);
            /* [21] binary kd-node visits (the byte model of SURVEY.md 8(d): 8 B per binary node) */
            atomicAdd(&st[21], (unsigned long long) tc.binNodes);
        }
    }
}

/* ------------------------------------------------------------------ */
/* Packet traversal for coherent rays (the camera pass)                 */
/* ------------------------------------------------------------------ */
/* The 64 rays of a wave (camera rays: 64 samples of one pixel, one
   origin) walk the binary kd-tree together: the node index, the stack and
   the leaf records are wave-uniform (scalar loads), each lane keeps its own
   ray interval and hit, and a lane takes part only in the subtrees its own
   Havran traversal (sahkdtree3.h:178-308) would enter.  At a split every
   member lane computes its own t and near/far/both decision exactly as
   traceRound does; the packet enters the first child if any lane needs it
   and stacks the second child for the lanes that need it ("both" lanes also
   stack their own tmax).  Lanes that disagree on the front-to-back order
   split the packet (the second group revisits the node later).  A lane
   therefore tests the same leaves in the same order with the same intervals
   as its own traversal, and its result is bit-identical.  A packet whose
   stack would overflow finishes lane by lane (traceRound). */
#ifndef HPT_PACKET_LEAF_BATCH
/* leaf records per round trip in the packet traversal.  Round 3 (mask kernel): 1 / 2 / 4 / 6 gave
   30.98 / 29.53 / 30.54 / 30.55 ms per headline frame; round 5 (lane words): 1 / 2 / 3 / 4 gave
   17.71 / 18.65 / 18.54 / 18.86 ms at 7 waves, and one record per trip needs 63 VGPRs, which lets
   the kernel run 8 waves/SIMD (17.08 ms) */
#define HPT_PACKET_LEAF_BATCH 1
#endif
#ifndef HPT_PACKET_STACK
#define HPT_PACKET_STACK 20 /* 5 KB of LDS per wave: 8 waves/SIMD fit the 160 KB (no packet overflowed at the headline) */
#endif
struct PacketLds {
    float saved[HPT_PACKET_STACK][64]; /* entry e: one word per lane (tracePacket) */
};
/* the batch entry point's per-lane fallback (tracePackets INLINE) puts an 8-entry ring stack and
   the ray rows in the packet's LDS: there it is declared with room for them */
union PacketLdsInline {
    PacketLds p;
    uint2 ring[(8 + HPT_RAY_ROWS) * 64];
};

/* The per-lane state lives in vector registers: a lane's "active", "done" and "found" are 0/1
   words, not lane masks, so their logic runs on the SIMDs' VALUs and not on the CU's one scalar
   unit (with wave masks the packet pass saturated it: SALU issue 0.85 at 24 waves per CU,
   profiles/r05_furball_marschner_kernels.md); a wave-uniform decision is one ballot of a word,
   compared with zero.  The stack keeps each entry's node in one lane of a vector register
   (lane e = entry e, bit 31 = revisit) and one LDS word per lane: the lane's saved tmax when it
   was "both" (any bit pattern below HPT_PK_FAR), HPT_PK_FAR when it skipped the first child,
   HPT_PK_OUT when it is not in the entry, and for a revisit entry HPT_PK_IN / HPT_PK_OUT. */
#define HPT_PK_FAR 0xFFFFFFFDu
#define HPT_PK_IN 0xFFFFFFFEu
#define HPT_PK_OUT 0xFFFFFFFFu
HD uint32_t pkWord(uint32_t x) { /* keep a 0/1 word a word (not folded back into a lane mask) */
#ifdef __HIP_DEVICE_COMPILE__
    asm("" : "+v"(x));
#endif
    return x;
}
HD uint32_t pkFlag(bool b) { return pkWord(b ? 1u : 0u); }
HD bool pkAny(uint32_t x) { return __builtin_amdgcn_ballot_w64(x != 0u) != 0; }

#define PK_OVERFLOW \
    status = 2;     \
    continue
#define PK_DONE \
    status = 1; \
    break
template <bool STATS>
HD bool tracePacket(const HptScene &sc, TraceRay &r, bool valid, PacketLds &L, TraceCounters &tc) {
    const uint32_t lane = __lane_id();
#ifdef __HIP_DEVICE_COMPILE__
    typedef const __attribute__((address_space(4))) char *CB;
    typedef const __attribute__((address_space(4))) uint2 *CU2;
    typedef const __attribute__((address_space(4))) float4 *CF4;
    const CB nodeB = (CB) sc.nodes, leafB = (CB) sc.leafF;
    auto nodes = [&](uint32_t i) {
        const uint2 v = *(CU2) (nodeB + (uint64_t) (i << 3));
        return HptNode{v.x, v.y};
    };
    auto leaf = [&](uint32_t i) { return *(CF4) (leafB + (uint64_t) (i << 4)); };
#else
    const HptNode *__restrict__ nodeP = sc.nodes;
    const float4 *__restrict__ leafP = reinterpret_cast<const float4 *>(sc.leafF);
    auto nodes = [&](uint32_t i) { return nodeP[i]; };
    auto leaf = [&](uint32_t i) { return leafP[i]; };
#endif
    uint32_t *const row = reinterpret_cast<uint32_t *>(&L.saved[0][0]) + lane; /* entry e at row[64 * e] */
    const V3 o = r.o, d = r.d, rcp = r.rcp;
    const int spMax = sc.packetStack ? min((int) sc.packetStack, HPT_PACKET_STACK) : HPT_PACKET_STACK;
    uint32_t act = pkFlag(valid), done = pkFlag(!valid);
    if (!pkAny(act)) return true;
    uint32_t found = pkFlag(r.found);
    uint32_t stackNode = 0; /* lane e: entry e's node | revisit << 31 */
    uint32_t node = 0;
    int sp = 0;
    uint32_t steps = 0;
    int status = 0; /* 0 running, 1 every lane done, 2 stack overflow / malformed tree */
    auto pushNode = [&](uint32_t v) { stackNode = (int) lane == sp ? v : stackNode; };
    while (status == 0) {
        const HptNode nd = nodes(node);
        if (!(nd.w0 & 0x80000000u)) {
            /* ---- an inner node ---- */
            if (STATS) {
                tc.nodes += act;
                if (lane == 0) tc.nodeSlots += 64;
            }
            const uint32_t axis = nd.w0 & 3u, left = nd.w0 >> 2;
            const float split = __uint_as_float(nd.w1);
            const float oa = axis == 0 ? o.x : (axis == 1 ? o.y : o.z);
            const float da = axis == 0 ? d.x : (axis == 1 ? d.y : d.z);
            const float ra = axis == 0 ? rcp.x : (axis == 1 ? rcp.y : rcp.z);
            const float ts = (split - oa) * ra;
            const uint32_t below = pkFlag(oa < split) | (pkFlag(oa == split) & pkFlag(da <= 0.0f));
            const uint32_t nearOnly = pkFlag(!(ts <= r.tmax)) | pkFlag(ts <= 0.0f);
            const uint32_t farOnly = (nearOnly ^ 1u) & pkFlag(ts < r.tmin);
            const uint32_t both = (nearOnly | farOnly) ^ 1u;
            const bool belowG = pkAny(act & below);
            if (belowG && pkAny(act & (below ^ 1u))) {
                /* the lanes disagree on the front-to-back order: the others revisit this node later */
                if (sp == spMax) {
                    PK_OVERFLOW;
                }
                row[64 * sp] = (act & (below ^ 1u)) ? HPT_PK_IN : HPT_PK_OUT;
                pushNode(node | 0x80000000u);
                ++sp;
                act &= below;
            }
            const uint32_t first = left + (belowG ? 0u : 1u), second = left + (belowG ? 1u : 0u);
            const uint32_t needFirst = act & (farOnly ^ 1u);
            if (!pkAny(needFirst)) { /* nobody needs the first child (so no lane is "both") */
                node = second;
                act &= farOnly;
                continue;
            }
            if (pkAny(act & (farOnly | both))) {
                if (sp == spMax) {
                    PK_OVERFLOW;
                }
                const uint32_t bMe = act & both;
                row[64 * sp] = bMe ? __float_as_uint(r.tmax) : ((act & farOnly) ? HPT_PK_FAR : HPT_PK_OUT);
                pushNode(second);
                ++sp;
                r.tmax = bMe ? ts : r.tmax;
            }
            node = first;
            act = needFirst;
            continue;
        }
        /* ---- leaf: the member lanes test its segments (pre-test, then exact) ---- */
        const bool me = act != 0u;
        if (STATS) {
            tc.nodes += act;
            if (lane == 0) tc.nodeSlots += 64;
        }
        const uint32_t lf = nd.w0 & 0x7fffffffu, ll = nd.w1;
        for (uint32_t c0 = lf; c0 < ll; c0 += HPT_PACKET_LEAF_BATCH) {
            const uint32_t n = min(ll - c0, (uint32_t) HPT_PACKET_LEAF_BATCH);
            float4 ra[HPT_PACKET_LEAF_BATCH], rb[HPT_PACKET_LEAF_BATCH];
#pragma unroll
            for (uint32_t k = 0; k < HPT_PACKET_LEAF_BATCH; ++k) {
                const uint32_t e = c0 + (k < n ? k : 0u);
                ra[k] = leaf(2 * e);
                rb[k] = leaf(2 * e + 1);
            }
            uint32_t mask = 0;
#pragma unroll
            for (uint32_t k = 0; k < HPT_PACKET_LEAF_BATCH; ++k) {
                if (k < n) {
                    if (STATS) {
                        tc.prims += act;
                        if (lane == 0) tc.primSlots += 64;
                    }
                    const bool may = segMayHit(ra[k], rb[k], o, d, rb[k].w); /* the record's own radius */
                    mask |= (me && may) ? 1u << k : 0u;
                }
            }
#ifdef HPT_PK_EXACT_STEPS /* probe variant: count the wave's exact-test steps (1) or the leaf batches
                             with any exact test (2) instead of its lanes' tests */
            if (STATS) {
                uint32_t steps = 0;
                for (uint32_t k = 0; k < HPT_PACKET_LEAF_BATCH; ++k) steps += __ballot((mask >> k) & 1u) != 0 ? 1u : 0u;
                if (lane == 0) tc.exact += HPT_PK_EXACT_STEPS == 2 ? (steps ? 1u : 0u) : steps;
            }
#endif
#pragma unroll
            for (uint32_t k = 0; k < HPT_PACKET_LEAF_BATCH; ++k) {
                if (mask & (1u << k)) {
                    const uint32_t sg = __float_as_uint(rb[k].z);
                    const float rad = segRadius(sc, sg);
                    const double r2 = (double) (rad * rad); /* Float product (hair.cpp:500) */
#ifndef HPT_PK_EXACT_STEPS
                    if (STATS) ++tc.exact;
#endif
                    float t;
                    uint32_t far;
                    if (segIntersect(sc.segs, sg, o, d, r2, r.mint, r.tHit, t, far)) {
                        found = 1u;
                        r.tHit = t;
                        r.segHit = sg | (far << 31);
                    }
                }
            }
        }
        done |= act & found & pkFlag(r.tHit <= r.tmax);
        if (++steps > (1u << 20)) { /* malformed tree: let the lanes finish alone */
            PK_OVERFLOW;
        }
        /* ---- pop the next subtree some unfinished lane needs ---- */
        while (true) {
            if (sp == 0) {
                PK_DONE;
            }
            --sp;
            const uint32_t en = (uint32_t) __builtin_amdgcn_readlane((int) stackNode, sp);
            const uint32_t w = row[64 * sp];
            const uint32_t live = done ^ 1u;
            if (en & 0x80000000u) {
                act = pkFlag(w == HPT_PK_IN) & live;
            } else {
                const uint32_t inB = pkFlag(w < HPT_PK_FAR) & live;
                r.tmin = inB ? r.tmax : r.tmin;
                r.tmax = inB ? __uint_as_float(w) : r.tmax;
                done |= inB & pkFlag(r.tmin > r.tHit);
                act = pkFlag(w <= HPT_PK_FAR) & (done ^ 1u);
            }
            if (pkAny(act)) {
                node = en & 0x7fffffffu;
                break;
            }
        }
    }
    r.found = found != 0u;
    return status == 1;
}
#undef PK_OVERFLOW
#undef PK_DONE

/* Persistent packet tracer: each wave claims 64 consecutive closest-hit rays
   (the camera queue keeps a pixel's samples together), traces them as one
   packet and writes the hits; the shard cursors are k_trace's.  A packet whose
   stack overflows is finished lane by lane: INLINE, right here (the batch entry
   point), or else its rays are appended to overflowQ for a k_trace_overflow launch
   (the camera pass), which keeps the per-lane traversal and its registers out of
   this kernel. */
template <bool STATS, bool INLINE, class IO>
__device__ __forceinline__ void tracePackets(const HptScene &sc, IO &io, uint32_t *cursors, PacketLds &L,
                                             uint32_t *stats, uint32_t *overflowQ = nullptr,
                                             uint32_t *nOverflow = nullptr) {
    const uint32_t total = io.count();
    const uint32_t lane = __lane_id();
    TraceCounters tc;
    uint32_t nC = 0, fallbacks = 0;
    uint32_t shard = (blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % HPT_CURSORS;
    int tried = 0;
    while (true) {
        uint32_t start = 0, got = 0;
        bool exhausted = false;
        while (true) { /* wave-uniform */
            /* shard bounds on multiples of 64, so a packet is 64 queue-consecutive rays
               (with nSpp a multiple of 64: the samples of one pixel) */
            auto bound = [&](uint32_t k) {
                return k >= HPT_CURSORS ? total : (uint32_t) ((uint64_t) total * k / HPT_CURSORS) & ~63u;
            };
            const uint32_t lo = bound(shard);
            const uint32_t size = bound(shard + 1) - lo;
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&cursors[shard * HPT_CURSOR_STRIDE], 64u);
            base = __shfl(base, 0);
            if (base < size) {
                start = lo + base;
                got = min(64u, size - base);
                break;
            }
            if (++tried >= HPT_CURSORS) {
                exhausted = true;
                break;
            }
            shard = (shard + 1) % HPT_CURSORS;
        }
        if (exhausted) break;
        const uint32_t k = start + lane;
        TraceRay r;
        bool valid = false;
        r.found = false;
        r.shadow = false;
        if (lane < got) valid = io.begin(sc, k, r);
        if (STATS) nC += lane < got ? 1u : 0u;
        const bool ok = tracePacket<STATS>(sc, r, valid, L, tc);
        if (!ok) {
            /* packet stack overflow: every lane re-traces its ray alone (same result) */
            if (STATS) fallbacks += lane == 0 ? 1u : 0u;
            if (INLINE) {
                uint2 *stk = reinterpret_cast<uint2 *>(&L) + lane;
                if (lane < got && io.begin(sc, k, r) && (stashRay<8>(stk, 64, r, io.key()), true))
                    while (!traceRound<8, STATS>(sc, r, stk, 64, tc)) {
                    }
            } else if (lane < got && valid) {
                overflowQ[atomicAdd(nOverflow, 1u)] = io.key();
            }
        }
        /* lanes handed to the overflow launch are finished there */
        if (lane < got && (ok || INLINE || !valid)) io.finish(sc, io.key(), r);
    }
    if (STATS) {
        for (int off = 32; off > 0; off >>= 1) {
            tc.nodes += __shfl_down(tc.nodes, off);
            tc.prims += __shfl_down(tc.prims, off);
            tc.exact += __shfl_down(tc.exact, off);
            tc.nodeSlots += __shfl_down(tc.nodeSlots, off);
            tc.primSlots += __shfl_down(tc.primSlots, off);
            nC += __shfl_down(nC, off);
            fallbacks += __shfl_down(fallbacks, off);
        }
        if (lane == 0) {
            unsigned long long *st = (unsigned long long *) stats;
            /* the packet pass's own counters: [12] binary node visits (8-byte HptNode)
               [13] primitive tests [14] rays [15] exact tests [16]/[17] node / primitive
               SIMD slots [18] packets that fell back to one ray per lane */
            atomicAdd(&st[12], (unsigned long long) tc.nodes);
            atomicAdd(&st[13], (unsigned long long) tc.prims);
            atomicAdd(&st[14], (unsigned long long) nC);
            atomicAdd(&st[15], (unsigned long long) tc.exact);
            atomicAdd(&st[16], (unsigned long long) tc.nodeSlots);
            atomicAdd(&st[17], (unsigned long long) tc.primSlots);
            atomicAdd(&st[18], (unsigned long long) fallbacks);
        }
    }
}

/* ------------------------------------------------------------------ */
/* Marschner (marschner_diffuse.cpp)                                    */
/* ------------------------------------------------------------------ */
HD float trigInverse(float x) { return fminr(sqrtf(fmaxr(1.0f - x * x, 0.0f)), 1.0f); }

HD float I0(float x) { /* :279-290 */
    float result = 1.0f, xSq = x * x, xi = xSq, denom = 4.0f;
#pragma unroll
    for (int i = 1; i <= 10; ++i) {
        result += xi / denom;
        xi *= xSq;
        denom *= 4.0f * float((i + 1) * (i + 1));
    }
    return result;
}
HD float logI0(float x) { /* :292-299 */
    if (x > 12.0f) return x + 0.5f * (logf(1.0f / (kPi * 2.0f * x)) + 1.0f / (8.0f * x));
    return logf(I0(x));
}
HD float longitudinalM(float v, float sinThetaI, float sinThetaO, float cosThetaI, float cosThetaO) { /* :364-374 */
    float a = cosThetaI * cosThetaO / v;
    float b = sinThetaI * sinThetaO / v;
    if (v < 0.1f) return expf(-b + logI0(a) - 1.0f / v + 0.6931f + logf(1.0f / (2.0f * v)));
    return expf(-b) * I0(a) / (2.0f * v * sinhf(1.0f / v));
}
/* the same with the lobe's constants 1 / v and log(1 / (2 v)) (v < 0.1) or 2 v sinh(1 / v), which
   depend on the BSDF only: the host computes them once at upload (HptMarschner::lobeInvV, lobeK) */
HD float longitudinalMc(float v, float invV, float k, float sinThetaI, float sinThetaO, float cosThetaI,
                        float cosThetaO) {
    float a = cosThetaI * cosThetaO / v;
    float b = sinThetaI * sinThetaO / v;
    if (v < 0.1f) return expf(-b + logI0(a) - invV + 0.6931f + k);
    return expf(-b) * I0(a) / k;
}

/* Azimuthal::eval (:80-94) */
HD V3 azEval(const HptF4 *__restrict__ tab, float phi, float cosThetaD) {
    float u = (HPT_AZ_RES - 1) * phi * (1.0f / (2.0f * kPi));
    float v = (HPT_AZ_RES - 1) * cosThetaD;
    int x0 = clampi(int(u), 0, HPT_AZ_RES - 2), y0 = clampi(int(v), 0, HPT_AZ_RES - 2);
    int x1 = x0 + 1, y1 = y0 + 1;
    u = clampf(u - x0, 0.0f, 1.0f);
    v = clampf(v - y0, 0.0f, 1.0f);
    HptF4 a = tab[x0 + y0 * HPT_AZ_RES], b = tab[x1 + y0 * HPT_AZ_RES];
    HptF4 c = tab[x0 + y1 * HPT_AZ_RES], e = tab[x1 + y1 * HPT_AZ_RES];
    V3 r0 = v3(a.x, a.y, a.z) * (1.0f - u) + v3(b.x, b.y, b.z) * u;
    V3 r1 = v3(c.x, c.y, c.z) * (1.0f - u) + v3(e.x, e.y, e.z) * u;
    return r0 * (1.0f - v) + r1 * v;
}
/* InterpolatedDistribution1D::sum via Azimuthal::weight (:102-106) */
HD float azWeight(const float *__restrict__ sums, float cosThetaD) {
    float dist = (HPT_AZ_RES - 1) * cosThetaD;
    int d0 = clampi(int(dist), 0, HPT_AZ_RES - 1), d1 = imin(d0 + 1, HPT_AZ_RES - 1);
    float v = clampf(dist - d0, 0.0f, 1.0f);
    return (sums[d0] * (1.0f - v) + sums[d1] * v) * (2.0f * kPi / HPT_AZ_RES);
}
/* Azimuthal::sample (:68-77) -> InterpolatedDistribution1D::warp (:69-92) */
HD float azSample(const float *__restrict__ cdfs, float cosThetaD, float xi) {
    float dist = (HPT_AZ_RES - 1) * cosThetaD;
    int d0 = clampi(int(dist), 0, HPT_AZ_RES - 1), d1 = imin(d0 + 1, HPT_AZ_RES - 1);
    float v = clampf(dist - d0, 0.0f, 1.0f);
    const float *c0 = cdfs + d0 * (HPT_AZ_RES + 1), *c1 = cdfs + d1 * (HPT_AZ_RES + 1);
    int lower = 0, upper = HPT_AZ_RES;
    float lowerU = 0.0f, upperU = 1.0f;
    while (upper - lower != 1) {
        int mid = (upper + lower) / 2;
        float mu = c0[mid] * (1.0f - v) + c1[mid] * v;
        if (mu < xi) {
            lower = mid;
            lowerU = mu;
        } else {
            upper = mid;
            upperU = mu;
        }
    }
    float u = clampf((xi - lowerU) / (upperU - lowerU), 0.0f, 1.0f);
    return 2.0f * kPi * (lower + u) * (1.0f / HPT_AZ_RES);
}

/* rtrans.h:183-199 (eta and alpha fixed) + spline.cpp:23-61 */
HD float roughTransSlice(const float *__restrict__ trans, int transSize, float cosTheta) {
    float w = powf(fabsf(cosTheta), 0.25f);
    if (!(cosTheta >= 0)) return 0.f;
    float result;
    if (!(w >= 0.0f && w <= 1.0f)) {
        result = 0.0f;
    } else {
        const size_t size = (size_t) transSize;
        float t = ((w - 0.0f) * (size - 1)) / (1.0f - 0.0f);
        size_t k = (size_t) t < size - 2 ? (size_t) t : size - 2;
        const float *val = trans;
        float f0 = val[k], f1 = val[k + 1], d0, d1;
        d0 = (k > 0) ? 0.5f * (val[k + 1] - val[k - 1]) : val[k + 1] - val[k];
        d1 = (k + 2 < size) ? 0.5f * (val[k + 2] - val[k]) : val[k + 1] - val[k];
        t = t - (float) k;
        float t2 = t * t, t3 = t2 * t;
        result = (2 * t3 - 3 * t2 + 1) * f0 + (-2 * t3 + 3 * t2) * f1 + (t3 - 2 * t2 + t) * d0 + (t3 - t2) * d1;
    }
    return fminr(1.0f, fmaxr(0.0f, result));
}
HD float roughTrans(const HptMarschner &m, float cosTheta) { return roughTransSlice(m.trans, m.transSize, cosTheta); }

/* The terms of MarschnerDiffuse::eval / ::sample that depend on wi only: a bounce evaluates
   the BSDF for its NEE direction, samples it and evaluates it again for the sampled direction,
   all with one wi, so k_shade computes them once (the same expressions: bit-identical) */
struct MarschnerWi {
    float thetaI;
    float sR, cR, sTT, cTT, sTRT, cTRT; /* sin / cos of thetaI shifted per lobe (:391-393) */
    float T12;                          /* roughTrans(wi.z) */
};
HD MarschnerWi marschnerWi(const HptMarschner &m, V3 wi) {
    MarschnerWi w;
    w.thetaI = asinf(clampf(wi.y, -1.0f, 1.0f));
    const float thetaIR = w.thetaI - 2.0f * m.scaleAngleRad;
    const float thetaITT = w.thetaI + m.scaleAngleRad;
    const float thetaITRT = w.thetaI + 4.0f * m.scaleAngleRad;
    w.sR = sinf(thetaIR), w.cR = cosf(thetaIR);
    w.sTT = sinf(thetaITT), w.cTT = cosf(thetaITT);
    w.sTRT = sinf(thetaITRT), w.cTRT = cosf(thetaITRT);
    w.T12 = roughTrans(m, wi.z);
    return w;
}
/* MarschnerDiffuse::eval (:377-482), hasDiffuse = true */
HD V3 marschnerEvalW(const HptMarschner &m, const MarschnerWi &w, V3 wo) {
    float T21 = roughTrans(m, wo.z); /* first: fewer values live across its powf */
    float sinThetaO = wo.y;
    float cosThetaO = trigInverse(sinThetaO);
    float thetaO = asinf(clampf(sinThetaO, -1.0f, 1.0f));
    float thetaD = (thetaO - w.thetaI) * 0.5f;
    float cosThetaD = cosf(thetaD);
    float phi = atan2f(wo.x, wo.z);
    if (phi < 0.0f) phi += kPi * 2.0f;
    float MR = longitudinalMc(m.vR, m.lobeInvV[0], m.lobeK[0], w.sR, sinThetaO, w.cR, cosThetaO);
    float MTT = longitudinalMc(m.vTT, m.lobeInvV[1], m.lobeK[1], w.sTT, sinThetaO, w.cTT, cosThetaO);
    float MTRT = longitudinalMc(m.vTRT, m.lobeInvV[2], m.lobeK[2], w.sTRT, sinThetaO, w.cTRT, cosThetaO);
    V3 result = (0.15f * MR) * azEval(m.table[0], phi, cosThetaD) + MTT * azEval(m.table[1], phi, cosThetaD) +
                MTRT * azEval(m.table[2], phi, cosThetaD);
    V3 diff = v3(m.diffuse[0], m.diffuse[1], m.diffuse[2]);
    diff = divs(diff, 1 - m.fdr);
    result = result + diff * (kInvPi * wo.z * w.T12 * T21 * m.invEta2);
    return result;
}
HD V3 marschnerEval(const HptMarschner &m, V3 wi, V3 wo) { return marschnerEvalW(m, marschnerWi(m, wi), wo); }
/* k_shade keeps a bounce's MarschnerWi in LDS between its NEE evaluation and its BSDF sample
   (nine more registers live across NEE would cost k_shade a wave per SIMD); row k of thread t at
   l[k * stride] */
#define HPT_WI_ROWS 8
HD void stashWi(float *l, int stride, const MarschnerWi &w) {
    l[0] = w.thetaI;
    l[stride] = w.sR;
    l[2 * stride] = w.cR;
    l[3 * stride] = w.sTT;
    l[4 * stride] = w.cTT;
    l[5 * stride] = w.sTRT;
    l[6 * stride] = w.cTRT;
    l[7 * stride] = w.T12;
    asm volatile("" ::: "memory"); /* re-read where used, not forwarded (forwarding keeps the registers) */
}
HD MarschnerWi loadWi(const float *l, int stride) {
    MarschnerWi w;
    w.thetaI = l[0];
    w.sR = l[stride];
    w.cR = l[2 * stride];
    w.sTT = l[3 * stride];
    w.cTT = l[4 * stride];
    w.sTRT = l[5 * stride];
    w.cTRT = l[6 * stride];
    w.T12 = l[7 * stride];
    return w;
}

/* k_shade also keeps the shading point's position, normal and shading tangent, wi and the shadow
   record in LDS, from the intersection record to the queue appends (stride HPT_SHADE_BLOCK): the
   registers they would hold across both BSDF evaluations keep k_shade at 6 waves per SIMD.
   Marschner reads only wi.y after marschnerWi (kRowWiY); the other BSDFs keep wi in rows 0-2. */
enum : int {
    kRowWiY = HPT_WI_ROWS,
    kRowP = kRowWiY + 1,
    kRowGeoN = kRowP + 3,
    kRowShS = kRowGeoN + 3,
    kRowSd = kRowShS + 3, /* shadow ray direction, max t */
    kRowSc = kRowSd + 4,  /* NEE contribution */
    kShadeRows = kRowSc + 3
};
HD void stashV3(float *l, int stride, int row, V3 v) {
    l[row * stride] = v.x;
    l[(row + 1) * stride] = v.y;
    l[(row + 2) * stride] = v.z;
}
HD V3 loadV3(const float *l, int stride, int row) {
    asm volatile("" ::: "memory"); /* read where used, not hoisted to the stash */
    return v3(l[row * stride], l[(row + 1) * stride], l[(row + 2) * stride]);
}

/* sampleM (:582-592) */
HD float sampleM(float v, float sinThetaI, float cosThetaI, float xi1, float xi2) {
    float cosTheta = 1.0f + v * logf(xi1 + (1.0f - xi1) * expf(-2.0f / v));
    float sinTheta = trigInverse(cosTheta);
    float cosPhi = cosf(2 * kPi * xi2);
    return -cosTheta * sinThetaI + sinTheta * cosPhi * cosThetaI;
}

/* Where MarschnerDiffuse::sample reads the per-lobe InterpolatedDistribution1D
   cdfs and sums: the scene's HBM arrays, through L2 (an LDS-staged copy was
   measured slower: DESIGN.md section 5, k_shade) */
struct GlobalTabs {
    const HptMarschner &m;
    HD const float *cdf(int l) const { return l == 0 ? m.cdf[0] : (l == 1 ? m.cdf[1] : m.cdf[2]); }
    HD const float *sums(int l) const { return l == 0 ? m.sums[0] : (l == 1 ? m.sums[1] : m.sums[2]); }
};

/* MarschnerDiffuse::sample (:594-744); pdf() == 1 (:517-520) */
template <class Tabs>
HD V3 marschnerSampleW(const HptMarschner &m, const MarschnerWi &w, const Tabs &tabs, V3 wi, float sx, float sy, V3 &wo,
                       uint32_t &type) {
    float sinThetaI = wi.y;
    float cosThetaI = trigInverse(sinThetaI);
    float weightR = azWeight(tabs.sums(0), cosThetaI);
    float weightTT = azWeight(tabs.sums(1), cosThetaI);
    float weightTRT = azWeight(tabs.sums(2), cosThetaI);
    int lobe;
    float v, sinTheta, cosTheta; /* of the chosen lobe's shifted thetaI (:624-641) */
    float target = sx * (weightR + weightTT + weightTRT);
    if (target < weightR) {
        lobe = 0; v = m.vR; sinTheta = w.sR; cosTheta = w.cR;
    } else if (target < weightR + weightTT) {
        lobe = 1; v = m.vTT; sinTheta = w.sTT; cosTheta = w.cTT;
    } else {
        lobe = 2; v = m.vTRT; sinTheta = w.sTRT; cosTheta = w.cTRT;
    }
    float sinThetaO = sampleM(v, sinTheta, cosTheta, sx, sy);
    float cosThetaO = trigInverse(sinThetaO);
    float thetaO = asinf(clampf(sinThetaO, -1.0f, 1.0f));
    float thetaD = (thetaO - w.thetaI) * 0.5f;
    float cosThetaD = cosf(thetaD);
    float phi = azSample(tabs.cdf(lobe), cosThetaD, sy);
    float sinPhi = sinf(phi), cosPhi = cosf(phi);
    float probSpecular = 1 - w.T12;
    const float sw = m.specularSamplingWeight;
    probSpecular = (probSpecular * sw) / (probSpecular * sw + (1 - probSpecular) * (1 - sw));
    if (sy < probSpecular) {
        wo = v3(sinPhi * cosThetaO, sinThetaO, cosPhi * cosThetaO);
        type = HPT_EDELTA_REFLECTION;
    } else {
        type = HPT_EDIFFUSE_REFLECTION;
        wo = squareToCosineHemisphere(sx, sy);
    }
    V3 e = marschnerEvalW(m, w, wo);
    return divs(e, 1.0f);
}
template <class Tabs>
HD V3 marschnerSample(const HptMarschner &m, const Tabs &tabs, V3 wi, float sx, float sy, V3 &wo, uint32_t &type) {
    return marschnerSampleW(m, marschnerWi(m, wi), tabs, wi, sx, sy, wo, type);
}

/* ------------------------------------------------------------------ */
/* Kajiya-Kay (kajiyakay.cpp:122-265)                                   */
/* ------------------------------------------------------------------ */
HD V3 kkEval(const HptKajiyaKay &k, V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return v3(0, 0, 0);
    V3 result = v3(0, 0, 0);
    float tl = fabsf(wi.x), te = fabsf(wo.x);
    float sin_tl = sqrtf(1 - tl * tl), sin_te = sqrtf(1 - te * te);
    float a = tl * te + sin_tl * sin_te;
    if (a > 0.0f && wi.x * wo.x < 0) {
        V3 ks = v3(k.ks[0], k.ks[1], k.ks[2]);
        V3 res = (ks * 0.15f) * ((k.exponent + 2) * kInvFourPi * powf(a, k.exponent));
        result = result + res;
    }
    result = result + v3(k.kd[0], k.kd[1], k.kd[2]) * kInvPi;
    return result * wo.z;
}
HD float kkPdf(const HptKajiyaKay &k, V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    float diffuseProb = kInvPi * wo.z, specProb = 0.0f;
    float a = dot(wo, v3(-wi.x, -wi.y, wi.z));
    if (a > 0) specProb = powf(a, k.exponent) * (k.exponent + 1.0f) / (2.0f * kPi);
    return k.specularSamplingWeight * specProb + (1 - k.specularSamplingWeight) * diffuseProb;
}
HD V3 kkSample(const HptKajiyaKay &k, V3 wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type) {
    bool choseSpecular = true;
    if (sx <= k.specularSamplingWeight) {
        sx /= k.specularSamplingWeight;
    } else {
        sx = (sx - k.specularSamplingWeight) / (1 - k.specularSamplingWeight);
        choseSpecular = false;
    }
    if (choseSpecular) {
        V3 R = v3(-wi.x, -wi.y, wi.z);
        float sinAlpha = sqrtf(1 - powf(sy, 2 / (k.exponent + 1)));
        float cosAlpha = powf(sy, 1 / (k.exponent + 1));
        float phi = (2.0f * kPi) * sx;
        V3 local = v3(sinAlpha * cosf(phi), sinAlpha * sinf(phi), cosAlpha);
        Frame f;
        f.n = R;
        coordinateSystem(R, f.s, f.t);
        wo = f.toWorld(local);
        type = HPT_EGLOSSY_REFLECTION;
        if (wo.z <= 0) {
            pdf = 0.0f;
            return v3(0, 0, 0);
        }
    } else {
        wo = squareToCosineHemisphere(sx, sy);
        type = HPT_EDIFFUSE_REFLECTION;
    }
    pdf = kkPdf(k, wi, wo);
    if (pdf == 0) return v3(0, 0, 0);
    return divs(kkEval(k, wi, wo), pdf);
}

/* ------------------------------------------------------------------ */
/* roughplastic (roughplastic.cpp:196-506) over the isotropic            */
/* MicrofacetDistribution (microfacet.h:67-720); constant textures.       */
/* math::fastexp/fastlog are double exp/log on Linux x86_64 (math.h:185). */
/* ------------------------------------------------------------------ */
HD float fastexpf(float v) { return (float) exp((double) v); }
HD float fastlogf(float v) { return (float) log((double) v); }

HD float mtsErf(float x) { /* math.cpp:55-72 */
    const float a1 = 0.254829592f, a2 = -0.284496736f, a3 = 1.421413741f, a4 = -1.453152027f,
                a5 = 1.061405429f, p = 0.3275911f;
    const float sign = copysignf(1.0f, x);
    x = fabsf(x);
    const float t = 1.0f / (1.0f + p * x);
    const float y = 1.0f - (((((a5 * t + a4) * t) + a3) * t + a2) * t + a1) * t * fastexpf(-x * x);
    return sign * y;
}
HD float mtsErfinv(float x) { /* math.cpp:25-53 (Giles) */
    float w = -fastlogf((1.0f - x) * (1.0f + x));
    float p;
    if (w < 5.0f) {
        w = w - 2.5f;
        p = 2.81022636e-08f;
        p = 3.43273939e-07f + p * w;
        p = -3.5233877e-06f + p * w;
        p = -4.39150654e-06f + p * w;
        p = 0.00021858087f + p * w;
        p = -0.00125372503f + p * w;
        p = -0.00417768164f + p * w;
        p = 0.246640727f + p * w;
        p = 1.50140941f + p * w;
    } else {
        w = sqrtf(w) - 3.0f;
        p = -0.000200214257f;
        p = 0.000100950558f + p * w;
        p = 0.00134934322f + p * w;
        p = -0.00367342844f + p * w;
        p = 0.00573950773f + p * w;
        p = -0.0076224613f + p * w;
        p = 0.00943887047f + p * w;
        p = 1.00167406f + p * w;
        p = 2.83297682f + p * w;
    }
    return p * x;
}
HD float hypot2f(float a, float b) { /* math.cpp:74-86 */
    float r;
    if (fabsf(a) > fabsf(b)) {
        r = b / a;
        r = fabsf(a) * sqrtf(1.0f + r * r);
    } else if (b != 0.0f) {
        r = a / b;
        r = fabsf(b) * sqrtf(1.0f + r * r);
    } else {
        r = 0.0f;
    }
    return r;
}

/* MicrofacetDistribution::eval (isotropic) */
HD float mfEval(const HptRoughPlastic &m, V3 h) {
    if (h.z <= 0) return 0.0f;
    const float cosTheta2 = h.z * h.z;
    const float a = m.alpha;
    const float beckmannExponent = ((h.x * h.x) / (a * a) + (h.y * h.y) / (a * a)) / cosTheta2;
    float result;
    /* M_PI is M_PI_FLT under SINGLE_PRECISION (constants.h:80): float throughout */
    if (m.type == 0) {
        result = fastexpf(-beckmannExponent) / (kPi * a * a * cosTheta2 * cosTheta2);
    } else if (m.type == 1) {
        const float root = (1.0f + beckmannExponent) * cosTheta2;
        result = 1.0f / (kPi * a * a * root * root);
    } else {
        result = sqrtf((m.exponent + 2) * (m.exponent + 2)) * kInvTwoPi * powf(h.z, m.exponent);
    }
    if (result * h.z < 1e-20f) result = 0;
    return result;
}
HD float mfSmithG1(const HptRoughPlastic &m, V3 v, V3 h) {
    if (dot(v, h) * v.z <= 0) return 0.0f;
    float temp = 1 - v.z * v.z;
    float tanTheta = fabsf(temp <= 0.0f ? 0.0f : sqrtf(temp) / v.z);
    if (tanTheta == 0.0f) return 1.0f;
    const float alpha = m.alpha; /* projectRoughness, isotropic */
    if (m.type == 1) {
        const float root = alpha * tanTheta;
        return 2.0f / (1.0f + hypot2f(1.0f, root));
    }
    const float a = 1.0f / (alpha * tanTheta);
    if (a >= 1.6f) return 1.0f;
    const float aSqr = a * a;
    return (3.535f * a + 2.181f * aSqr) / (1.0f + 2.276f * a + 2.577f * aSqr);
}
HD float mfPdf(const HptRoughPlastic &m, V3 wi, V3 h) {
    if (m.sampleVisible) {
        if (wi.z == 0) return 0.0f;
        return mfSmithG1(m, wi, h) * fabsf(dot(wi, h)) * mfEval(m, h) / fabsf(wi.z);
    }
    return mfEval(m, h) * h.z;
}
/* sampleVisible11 (microfacet.h:567-686), isotropic Beckmann / GGX */
HD void mfSampleVisible11(const HptRoughPlastic &m, float thetaI, float sx, float sy, float &slopeX, float &slopeY) {
    const float SQRT_PI_INV = 1 / sqrtf(kPi);
    if (m.type == 0) {
        if (thetaI < 1e-4f) {
            const float r = sqrtf(-fastlogf(1.0f - sx));
            const float ang = 2 * kPi * sy;
            slopeX = r * cosf(ang);
            slopeY = r * sinf(ang);
            return;
        }
        const float tanThetaI = tanf(thetaI), cotThetaI = 1 / tanThetaI;
        float a = -1, c = mtsErf(cotThetaI);
        const float sample_x = fmaxr(sx, 1e-6f);
        const float fit = 1 + thetaI * (-0.876f + thetaI * (0.4265f - 0.0594f * thetaI));
        float b = c - (1 + c) * powf(1 - sample_x, fit);
        const float normalization = 1 / (1 + c + SQRT_PI_INV * tanThetaI * expf(-cotThetaI * cotThetaI));
        int it = 0;
        while (++it < 10) {
            if (!(b >= a && b <= c)) b = 0.5f * (a + c);
            const float invErf = mtsErfinv(b);
            const float value = normalization * (1 + b + SQRT_PI_INV * tanThetaI * expf(-invErf * invErf)) - sample_x;
            const float derivative = normalization * (1 - invErf * tanThetaI);
            if (fabsf(value) < 1e-5f) break;
            if (value > 0) c = b;
            else a = b;
            b -= value / derivative;
        }
        slopeX = mtsErfinv(b);
        slopeY = mtsErfinv(2.0f * fmaxr(sy, 1e-6f) - 1.0f);
        return;
    }
    /* GGX */
    if (thetaI < 1e-4f) {
        const float r = sqrtf(fmaxr(0.0f, sx / (1 - sx)));
        const float ang = 2 * kPi * sy;
        slopeX = r * cosf(ang);
        slopeY = r * sinf(ang);
        return;
    }
    const float tanThetaI = tanf(thetaI);
    const float a = 1 / tanThetaI;
    const float G1 = 2.0f / (1.0f + sqrtf(fmaxr(0.0f, 1.0f + 1.0f / (a * a))));
    float A = 2.0f * sx / G1 - 1.0f;
    if (fabsf(A) == 1) A -= copysignf(1.0f, A) * kEpsilon;
    const float tmp = 1.0f / (A * A - 1.0f);
    const float B = tanThetaI;
    const float D = sqrtf(fmaxr(0.0f, B * B * tmp * tmp - (A * A - B * B) * tmp));
    const float slope_x_1 = B * tmp - D, slope_x_2 = B * tmp + D;
    slopeX = (A < 0.0f || slope_x_2 > 1.0f / tanThetaI) ? slope_x_1 : slope_x_2;
    float S;
    if (sy > 0.5f) {
        S = 1.0f;
        sy = 2.0f * (sy - 0.5f);
    } else {
        S = -1.0f;
        sy = 2.0f * (0.5f - sy);
    }
    const float z = (sy * (sy * (sy * (-0.365728915865723f) + 0.790235037209296f) - 0.424965825137544f) +
                     0.000152998850436920f) /
                    (sy * (sy * (sy * (sy * 0.169507819808272f - 0.397203533833404f) - 0.232500544458471f) + 1.0f) -
                     0.539825872510702f);
    slopeY = S * z * sqrtf(1.0f + slopeX * slopeX);
}
/* MicrofacetDistribution::sample(wi, sample) without pdf */
HD V3 mfSample(const HptRoughPlastic &m, V3 wiIn, float sx, float sy) {
    if (m.sampleVisible) {
        const V3 wi = normalize(v3(m.alpha * wiIn.x, m.alpha * wiIn.y, wiIn.z));
        float theta = 0, phi = 0;
        if (wi.z < 0.99999f) {
            theta = acosf(wi.z);
            phi = atan2f(wi.y, wi.x);
        }
        const float sinPhi = sinf(phi), cosPhi = cosf(phi);
        float slx, sly;
        mfSampleVisible11(m, theta, sx, sy, slx, sly);
        const float rx = cosPhi * slx - sinPhi * sly, ry = sinPhi * slx + cosPhi * sly;
        const float ux = rx * m.alpha, uy = ry * m.alpha;
        const float normalization = 1.0f / sqrtf(ux * ux + uy * uy + 1.0f);
        return v3(-ux * normalization, -uy * normalization, normalization);
    }
    /* sampleAll, isotropic */
    float cosThetaM, sinPhiM, cosPhiM;
    if (m.type == 2) {
        const float phiM = (2.0f * kPi) * sy;
        sinPhiM = sinf(phiM);
        cosPhiM = cosf(phiM);
        cosThetaM = powf(sx, 1.0f / (m.exponent + 2.0f));
    } else {
        const float ang = (2.0f * kPi) * sy;
        sinPhiM = sinf(ang);
        cosPhiM = cosf(ang);
        const float alphaSqr = m.alpha * m.alpha;
        const float tanThetaMSqr = (m.type == 0) ? alphaSqr * -fastlogf(1.0f - sx) : alphaSqr * sx / (1.0f - sx);
        cosThetaM = 1.0f / sqrtf(1.0f + tanThetaMSqr);
    }
    const float sinThetaM = sqrtf(fmaxr(0.0f, 1 - cosThetaM * cosThetaM));
    return v3(sinThetaM * cosPhiM, sinThetaM * sinPhiM, cosThetaM);
}

/* RoughPlastic::eval (:296-360) */
HD V3 rpEval(const HptRoughPlastic &m, V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return v3(0, 0, 0);
    V3 result = v3(0, 0, 0);
    {
        const V3 H = normalize(wo + wi);
        const float D = mfEval(m, H);
        const float F = fresnelDielectricExt(dot(wi, H), m.eta);
        const float G = mfSmithG1(m, wi, H) * mfSmithG1(m, wo, H);
        const float value = F * D * G / (4.0f * wi.z);
        result = result + v3(m.specular[0], m.specular[1], m.specular[2]) * value;
    }
    {
        V3 diff = v3(m.diffuse[0], m.diffuse[1], m.diffuse[2]);
        const float T12 = roughTransSlice(m.trans, m.transSize, wi.z);
        const float T21 = roughTransSlice(m.trans, m.transSize, wo.z);
        const float Fdr = m.fdr;
        if (m.nonlinear) diff = v3(diff.x / (1.0f - diff.x * Fdr), diff.y / (1.0f - diff.y * Fdr), diff.z / (1.0f - diff.z * Fdr));
        else diff = divs(diff, 1 - Fdr);
        result = result + diff * (kInvPi * wo.z * T12 * T21 * m.invEta2);
    }
    return result;
}
/* RoughPlastic::pdf (:362-436) */
HD float rpPdf(const HptRoughPlastic &m, V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    const V3 H = normalize(wo + wi);
    float probSpecular = 1 - roughTransSlice(m.trans, m.transSize, wi.z);
    probSpecular = (probSpecular * m.specularSamplingWeight) /
                   (probSpecular * m.specularSamplingWeight + (1 - probSpecular) * (1 - m.specularSamplingWeight));
    const float probDiffuse = 1 - probSpecular;
    const float dwh_dwo = 1.0f / (4.0f * dot(wo, H));
    const float prob = mfPdf(m, wi, H);
    float result = prob * dwh_dwo * probSpecular;
    result += probDiffuse * (kInvPi * wo.z);
    return result;
}
/* RoughPlastic::sample (:438-506) */
HD V3 rpSample(const HptRoughPlastic &m, V3 wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type) {
    pdf = 0.0f;
    type = 0;
    wo = v3(0, 0, 0);
    if (wi.z <= 0) return v3(0, 0, 0);
    bool choseSpecular = true;
    float probSpecular = 1 - roughTransSlice(m.trans, m.transSize, wi.z);
    probSpecular = (probSpecular * m.specularSamplingWeight) /
                   (probSpecular * m.specularSamplingWeight + (1 - probSpecular) * (1 - m.specularSamplingWeight));
    if (sy < probSpecular) {
        sy /= probSpecular;
    } else {
        sy = (sy - probSpecular) / (1 - probSpecular);
        choseSpecular = false;
    }
    if (choseSpecular) {
        const V3 mn = mfSample(m, wi, sx, sy);
        wo = mn * (2 * dot(wi, mn)) - wi; /* reflect (:281-283) */
        type = HPT_EGLOSSY_REFLECTION;
        if (wo.z <= 0) return v3(0, 0, 0);
    } else {
        type = HPT_EDIFFUSE_REFLECTION;
        wo = squareToCosineHemisphere(sx, sy);
    }
    pdf = rpPdf(m, wi, wo);
    if (pdf == 0) return v3(0, 0, 0);
    return divs(rpEval(m, wi, wo), pdf);
}

/* ------------------------------------------------------------------ */
/* marschnerdielectric (marschnerdielectric.cpp:226-529), typeMask EAll.  */
/* eval() and pdf() are called with ESolidAngle by the integrator, where  */
/* the specular branches require EDiscrete: eval is 0 for every pair and  */
/* pdf is the cosine-hemisphere density (:232-240, :285-335).             */
/* ------------------------------------------------------------------ */
HD V3 mdEval(const HptMarschnerDielectric &, V3, V3) { return v3(0, 0, 0); }
HD float mdPdf(const HptMarschnerDielectric &, V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    return kInvPi * wo.z;
}
HD V3 mdSample(const HptMarschnerDielectric &m, V3 wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type) {
    bool choseSpecular = true;
    if (sx <= m.specularSamplingWeight) {
        sx /= m.specularSamplingWeight;
    } else {
        sx = (sx - m.specularSamplingWeight) / (1 - m.specularSamplingWeight);
        choseSpecular = false;
    }
    if (choseSpecular) {
        float R = fresnelDielectricExt(fabsf(wi.z), m.eta), T = 1 - R;
        if (R < 1) R += T * T * R / (1 - R * R); /* R + TRT + TR^3T + .. */
        if (sx <= R) {
            type = HPT_EDELTA_REFLECTION;
            wo = v3(-wi.x, -wi.y, wi.z);
            pdf = R;
            return v3(m.specR[0], m.specR[1], m.specR[2]);
        }
        type = HPT_ENULL;
        wo = v3(-wi.x, -wi.y, -wi.z);
        pdf = 1 - R;
        return v3(m.specT[0], m.specT[1], m.specT[2]);
    }
    wo = squareToCosineHemisphere(sx, sy);
    type = HPT_EDIFFUSE_REFLECTION;
    pdf = mdPdf(m, wi, wo);
    return v3(0, 0, 0); /* eval / pdf with eval == 0 (or pdf == 0) */
}

/* thindielectric (thindielectric.cpp:138-252): no ESmooth component, so the
   integrator never evaluates it in solid angle (eval/pdf are 0 there) */
HD V3 tdSample(const HptMarschnerDielectric &m, V3 wi, float sx, V3 &wo, float &pdf, uint32_t &type) {
    float R = fresnelDielectricExt(fabsf(wi.z), m.eta), T = 1 - R;
    if (R < 1) R += T * T * R / (1 - R * R);
    if (sx <= R) {
        type = HPT_EDELTA_REFLECTION;
        wo = v3(-wi.x, -wi.y, wi.z);
        pdf = R;
        return v3(m.specR[0], m.specR[1], m.specR[2]);
    }
    type = HPT_ENULL;
    wo = v3(-wi.x, -wi.y, -wi.z);
    pdf = 1 - R;
    return v3(m.specT[0], m.specT[1], m.specT[2]);
}

/* diffuse (diffuse.cpp:111-140) */
HD V3 dfEval(const HptDiffuse &m, V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return v3(0, 0, 0);
    return v3(m.refl[0], m.refl[1], m.refl[2]) * (kInvPi * wo.z);
}
HD float dfPdf(V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    return kInvPi * wo.z;
}
HD V3 dfSample(const HptDiffuse &m, V3 wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type) {
    pdf = 0.0f;
    type = 0;
    wo = v3(0, 0, 0);
    if (wi.z <= 0) return v3(0, 0, 0);
    wo = squareToCosineHemisphere(sx, sy);
    type = HPT_EDIFFUSE_REFLECTION;
    pdf = kInvPi * wo.z;
    return v3(m.refl[0], m.refl[1], m.refl[2]);
}

HD V3 bsdfEval(const HptBsdf &b, V3 wi, V3 wo) {
    switch (b.kind) {
    case HPT_BSDF_MARSCHNER: return marschnerEval(b.mar, wi, wo);
    case HPT_BSDF_KAJIYAKAY: return kkEval(b.kk, wi, wo);
    case HPT_BSDF_ROUGHPLASTIC: return rpEval(b.rp, wi, wo);
    case HPT_BSDF_DIFFUSE: return dfEval(b.df, wi, wo);
    default: return v3(0, 0, 0); /* marschnerdielectric (:232-240), thindielectric */
    }
}
HD float bsdfPdf(const HptBsdf &b, V3 wi, V3 wo) {
    switch (b.kind) {
    case HPT_BSDF_MARSCHNER: return 1.0f;
    case HPT_BSDF_KAJIYAKAY: return kkPdf(b.kk, wi, wo);
    case HPT_BSDF_ROUGHPLASTIC: return rpPdf(b.rp, wi, wo);
    case HPT_BSDF_MARSCHNERDIELECTRIC: return mdPdf(b.md, wi, wo);
    case HPT_BSDF_DIFFUSE: return dfPdf(wi, wo);
    default: return 0.0f;
    }
}
template <class Tabs>
HD V3 bsdfSampleT(const HptBsdf &b, const Tabs &tabs, V3 wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type) {
    switch (b.kind) {
    case HPT_BSDF_MARSCHNER: pdf = 1.0f; return marschnerSample(b.mar, tabs, wi, sx, sy, wo, type);
    case HPT_BSDF_KAJIYAKAY: return kkSample(b.kk, wi, sx, sy, wo, pdf, type);
    case HPT_BSDF_ROUGHPLASTIC: return rpSample(b.rp, wi, sx, sy, wo, pdf, type);
    case HPT_BSDF_MARSCHNERDIELECTRIC: return mdSample(b.md, wi, sx, sy, wo, pdf, type);
    case HPT_BSDF_THINDIELECTRIC: return tdSample(b.md, wi, sx, wo, pdf, type);
    default: return dfSample(b.df, wi, sx, sy, wo, pdf, type);
    }
}
HD V3 bsdfSample(const HptBsdf &b, V3 wi, float sx, float sy, V3 &wo, float &pdf, uint32_t &type) {
    return bsdfSampleT(b, GlobalTabs{b.mar}, wi, sx, sy, wo, pdf, type);
}

/* ------------------------------------------------------------------ */
/* Environment map (envmap.cpp)                                         */
/* ------------------------------------------------------------------ */
HD V3 texel(const HptEnvMap &e, int x, int y) { /* mipmap.h:503-563: u repeat, v clamp */
    if (x < 0 || x >= e.w) {
        int r = x % e.w;
        x = (r < 0) ? r + e.w : r;
    }
    if (y < 0 || y >= e.h) y = clampi(y, 0, e.h - 1);
    HptF4 t = e.texel[y * e.w + x];
    return v3(t.x, t.y, t.z);
}
HD V3 envToLocal(const HptEnvMap &e, V3 v) {
    if (e.identity) return v;
    return v3(e.minv[0] * v.x + e.minv[1] * v.y + e.minv[2] * v.z, e.minv[3] * v.x + e.minv[4] * v.y + e.minv[5] * v.z,
              e.minv[6] * v.x + e.minv[7] * v.y + e.minv[8] * v.z);
}
HD V3 envToWorld(const HptEnvMap &e, V3 v) {
    if (e.identity) return v;
    return v3(e.m[0] * v.x + e.m[1] * v.y + e.m[2] * v.z, e.m[3] * v.x + e.m[4] * v.y + e.m[5] * v.z,
              e.m[6] * v.x + e.m[7] * v.y + e.m[8] * v.z);
}
/* evalEnvironment (:380-410) with the level-0 bilinear lookup (mipmap.h:575-596) */
HD V3 envEval(const HptEnvMap &e, V3 dir) {
    V3 v = envToLocal(e, dir);
    float uvx = atan2f(v.x, -v.z) * kInvTwoPi, uvy = acosf(fminr(1.0f, fmaxr(-1.0f, v.y))) * kInvPi;
    V3 value;
    if (!isfinite(uvx) || !isfinite(uvy)) {
        value = v3(0, 0, 0);
    } else {
        float u = uvx * e.w - 0.5f, vv = uvy * e.h - 0.5f;
        int xPos = (int) floorf(u), yPos = (int) floorf(vv);
        float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = vv - yPos, dy2 = 1.0f - dy1;
        value = texel(e, xPos, yPos) * dx2 * dy2 + texel(e, xPos, yPos + 1) * dx2 * dy1 +
                texel(e, xPos + 1, yPos) * dx1 * dy2 + texel(e, xPos + 1, yPos + 1) * dx1 * dy1;
    }
    return value * e.scale;
}
/* ---- filtered lookups of camera rays: MIPMap::eval with EWA (mipmap.h:503-834) ---- */
HD V3 mipTexel(const HptEnvMap &e, int level, int x, int y) { /* evalTexel (:503-563): u repeat, v clamp */
    const HptMipLevel L = e.levels[level];
    if (x < 0 || x >= L.w) {
        const int r = x % L.w;
        x = (r < 0) ? r + L.w : r;
    }
    if (y < 0 || y >= L.h) y = clampi(y, 0, L.h - 1);
    const HptF4 t = e.mip[L.off + y * L.w + x];
    return v3(t.x, t.y, t.z);
}
HD V3 mipBox(const HptEnvMap &e, int level, float ux, float uy) { /* evalBox (:566-569) */
    const HptMipLevel L = e.levels[level];
    return mipTexel(e, level, (int) floorf(ux * L.w), (int) floorf(uy * L.h));
}
HD V3 mipBilinear(const HptEnvMap &e, int level, float ux, float uy) { /* evalBilinear (:575-596) */
    if (!isfinite(ux) || !isfinite(uy)) return v3(0, 0, 0);
    if (level >= e.nLevels) return mipBox(e, e.nLevels - 1, ux, uy);
    const HptMipLevel L = e.levels[level];
    const float u = ux * L.w - 0.5f, v = uy * L.h - 0.5f;
    const int xPos = (int) floorf(u), yPos = (int) floorf(v);
    const float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    return mipTexel(e, level, xPos, yPos) * dx2 * dy2 + mipTexel(e, level, xPos, yPos + 1) * dx2 * dy1 +
           mipTexel(e, level, xPos + 1, yPos) * dx1 * dy2 + mipTexel(e, level, xPos + 1, yPos + 1) * dx1 * dy1;
}
/* evalEWA (:764-834) */
HD V3 mipEWA(const HptEnvMap &e, int level, float ux, float uy, float A, float B, float C) {
    if (!isfinite(A + B + C + ux + uy)) return v3(0, 0, 0);
    if (level >= e.nLevels) return mipBox(e, e.nLevels - 1, ux, uy);
    const HptMipLevel L = e.levels[level];
    const float u = ux * L.w - 0.5f, v = uy * L.h - 0.5f;
    A /= L.ratioX * L.ratioX;
    B /= L.ratioX * L.ratioY;
    C /= L.ratioY * L.ratioY;
    const float invDet = 1.0f / (-B * B + 4.0f * A * C), deltaU = 2.0f * sqrtf(C * invDet),
                deltaV = 2.0f * sqrtf(A * invDet);
    const int u0 = (int) ceilf(u - deltaU), u1 = (int) floorf(u + deltaU);
    const int v0 = (int) ceilf(v - deltaV), v1 = (int) floorf(v + deltaV);
    const float As = A * HPT_EWA_LUT, Bs = B * HPT_EWA_LUT, Cs = C * HPT_EWA_LUT;
    V3 result = v3(0, 0, 0);
    float denominator = 0.0f;
    const float ddq = 2 * As, uu0 = (float) u0 - u;
    for (int vt = v0; vt <= v1; ++vt) {
        const float vv = (float) vt - v;
        float q = As * uu0 * uu0 + (Bs * uu0 + Cs * vv) * vv;
        float dq = As * (2 * uu0 + 1) + Bs * vv;
        for (int ut = u0; ut <= u1; ++ut) {
            if (q < (float) HPT_EWA_LUT) {
                const uint32_t qi = (uint32_t) q;
                if (qi < HPT_EWA_LUT) {
                    const float weight = e.ewaLut[(int) q];
                    result = result + mipTexel(e, level, ut, vt) * weight;
                    denominator += weight;
                }
            }
            q += dq;
            dq += ddq;
        }
    }
    if (denominator == 0) return mipBilinear(e, level, ux, uy);
    return divs(result, denominator);
}
HD float log2Mts(float x) { return (float) log((double) x) * (1.0f / logf(2.0f)); } /* math.cpp:103-106 */
HD float hypot2Mts(float a, float b) {                                                  /* math.cpp:74-86 */
    if (fabsf(a) > fabsf(b)) {
        const float r = b / a;
        return fabsf(a) * sqrtf(1.0f + r * r);
    }
    if (b != 0.0f) {
        const float r = a / b;
        return fabsf(b) * sqrtf(1.0f + r * r);
    }
    return 0.0f;
}
/* MIPMap::eval(uv, d0, d1) with filterType EEWA (mipmap.h:629-720) */
HD V3 mipEval(const HptEnvMap &e, float ux, float uy, float d0x, float d0y, float d1x, float d1y) {
    const HptMipLevel L0 = e.levels[0];
    const float du0 = d0x * L0.w, dv0 = d0y * L0.h, du1 = d1x * L0.w, dv1 = d1y * L0.h;
    float A = dv0 * dv0 + dv1 * dv1, B = -2.0f * (du0 * dv0 + du1 * dv1), C = du0 * du0 + du1 * du1,
          F = A * C - B * B * 0.25f;
    const float root = hypot2Mts(A - C, B), Aprime = 0.5f * (A + C - root), Cprime = 0.5f * (A + C + root);
    float majorRadius = Aprime != 0 ? sqrtf(F / Aprime) : 0, minorRadius = Cprime != 0 ? sqrtf(F / Cprime) : 0;
    if (!(minorRadius > 0) || !(majorRadius > 0) || F < 0) {
        const float level = log2Mts(fmaxr(majorRadius, kEpsilon));
        const int ilevel = (int) floorf(level);
        if (ilevel < 0) return mipBilinear(e, 0, ux, uy);
        const float a = level - ilevel;
        return mipBilinear(e, ilevel, ux, uy) * (1.0f - a) + mipBilinear(e, ilevel + 1, ux, uy) * a;
    }
    if (minorRadius * e.maxAnisotropy < majorRadius) {
        /* artificially enlarge ellipses that are too skinny */
        minorRadius = majorRadius / e.maxAnisotropy;
        const float theta = 0.5f * atanf(B / (A - C));
        float sinTheta, cosTheta;
        sincosf(theta, &sinTheta, &cosTheta);
        const float a2 = majorRadius * majorRadius, b2 = minorRadius * minorRadius, sinTheta2 = sinTheta * sinTheta,
                    cosTheta2 = cosTheta * cosTheta, sin2Theta = 2 * sinTheta * cosTheta;
        A = a2 * cosTheta2 + b2 * sinTheta2;
        B = (a2 - b2) * sin2Theta;
        C = a2 * sinTheta2 + b2 * cosTheta2;
        F = a2 * b2;
    }
    const float scale = 1.0f / F;
    A *= scale;
    B *= scale;
    C *= scale;
    const float level = fmaxr(0.0f, log2Mts(minorRadius));
    const int ilevel = (int) level;
    const float a = level - ilevel;
    if (majorRadius < 1 || !(A > 0 && C > 0)) return mipBilinear(e, ilevel, ux, uy);
    return mipEWA(e, ilevel, ux, uy, A, B, C) * (1.0f - a) + mipEWA(e, ilevel + 1, ux, uy, A, B, C) * a;
}
/* evalEnvironment of a ray with differentials (envmap.cpp:380-410): camera rays */
HD V3 envEvalFiltered(const HptEnvMap &e, V3 dir, V3 rxDir, V3 ryDir) {
    const V3 v = envToLocal(e, dir);
    const float ux = atan2f(v.x, -v.z) * kInvTwoPi, uy = acosf(fminr(1.0f, fmaxr(-1.0f, v.y))) * kInvPi;
    const V3 dvdx = envToLocal(e, rxDir) - v, dvdy = envToLocal(e, ryDir) - v;
    const float t1 = kInvTwoPi / (v.x * v.x + v.z * v.z),
                t2 = -kInvPi / fmaxr(sqrtf(fmaxr(0.0f, 1.0f - v.y * v.y)), kEpsilon);
    const V3 value = mipEval(e, ux, uy, t1 * (dvdx.z * v.x - dvdx.x * v.z), t2 * dvdx.y,
                             t1 * (dvdy.z * v.x - dvdy.x * v.z), t2 * dvdy.y);
    return value * e.scale;
}

/* camera ray differential directions of a film sample (perspective.cpp:283-296, scaled by
   1/sqrt(sampleCount) like sensorRay.scaleDifferential, ray.h:163-168) */
HD void cameraDifferentials(const HptCamera &c, float posx, float posy, V3 dW, V3 &rx, V3 &ry) {
    const V3 nearP = xformPoint(c.s2c, v3(posx * c.invResX, posy * c.invResY, 0.0f));
    rx = xformVector(c.toWorld, normalize(nearP + v3(c.dx[0], c.dx[1], c.dx[2])));
    ry = xformVector(c.toWorld, normalize(nearP + v3(c.dy[0], c.dy[1], c.dy[2])));
    rx = dW + (rx - dW) * c.diffScale;
    ry = dW + (ry - dW) * c.diffScale;
}

/* internalPdfDirection (:603-633) */
HD float envPdf(const HptEnvMap &e, V3 d) {
    float uvx = atan2f(d.x, -d.z) * kInvTwoPi, uvy = acosf(fminr(1.0f, fmaxr(-1.0f, d.y))) * kInvPi;
    if (!isfinite(uvx) || !isfinite(uvy)) return 0.0f;
    float u = uvx * e.w - 0.5f, v = uvy * e.h - 0.5f;
    int xPos = (int) floorf(u), yPos = (int) floorf(v);
    float dx1 = u - xPos, dx2 = 1.0f - dx1, dy1 = v - yPos, dy2 = 1.0f - dy1;
    V3 value1 = texel(e, xPos, yPos) * dx2 * dy2 + texel(e, xPos + 1, yPos) * dx1 * dy2;
    V3 value2 = texel(e, xPos, yPos + 1) * dx2 * dy1 + texel(e, xPos + 1, yPos + 1) * dx1 * dy1;
    float sinTheta = sqrtf(fmaxr(0.0f, 1 - d.y * d.y));
    return (lum(value1) * e.rowWeights[clampi(yPos, 0, e.h - 1)] +
            lum(value2) * e.rowWeights[clampi(yPos + 1, 0, e.h - 1)]) *
           e.normalization / fmaxr(fabsf(sinTheta), kEpsilon);
}
/* sampleReuse (:657-662): std::lower_bound + rescale */
HD uint32_t sampleReuse(const float *cdf, uint32_t size, float &sample, const uint32_t *guide) {
    /* the first entry >= sample lies between the guide entries of sample's bucket
       (host-built from the same cdf, so the search returns std::lower_bound's entry) */
    const uint32_t k = min((uint32_t) (sample * (float) HPT_ENV_GUIDE), (uint32_t) HPT_ENV_GUIDE - 1u);
    uint32_t lo = guide[k], n = guide[k + 1] - guide[k] + 1;
    while (n > 0) { /* first entry >= sample */
        uint32_t half = n >> 1;
        if (cdf[lo + half] < sample) {
            lo += half + 1;
            n -= half + 1;
        } else {
            n = half;
        }
    }
    int idx = (int) lo - 1;
    uint32_t index = (uint32_t) imax(0, idx);
    if (index > size - 1) index = size - 1;
    sample = (sample - cdf[index]) / (cdf[index + 1] - cdf[index]);
    return index;
}
/* internalSampleDirection (:567-600) */
HD void envSampleDir(const HptEnvMap &e, float sx, float sy, V3 &d, V3 &value, float &pdf) {
    uint32_t row = sampleReuse(e.cdfRows, (uint32_t) e.h, sy, e.guideRows);
    uint32_t col = sampleReuse(e.cdfCols + row * (e.w + 1), (uint32_t) e.w, sx, e.guideCols + row * (HPT_ENV_GUIDE + 1));
    float posx = (float) col + intervalToTent(sx), posy = (float) row + intervalToTent(sy);
    int xPos = (int) floorf(posx), yPos = (int) floorf(posy);
    float dx1 = posx - xPos, dx2 = 1.0f - dx1, dy1 = posy - yPos, dy2 = 1.0f - dy1;
    V3 value1 = texel(e, xPos, yPos) * dx2 * dy2 + texel(e, xPos + 1, yPos) * dx1 * dy2;
    V3 value2 = texel(e, xPos, yPos + 1) * dx2 * dy1 + texel(e, xPos + 1, yPos + 1) * dx1 * dy1;
    value = (value1 + value2) * e.scale;
    pdf = (lum(value1) * e.rowWeights[clampi(yPos, 0, e.h - 1)] +
           lum(value2) * e.rowWeights[clampi(yPos + 1, 0, e.h - 1)]) *
          e.normalization;
    float sinPhi = sinf(e.pixelSizeX * (posx + 0.5f)), cosPhi = cosf(e.pixelSizeX * (posx + 0.5f));
    float sinTheta = sinf(e.pixelSizeY * (posy + 0.5f)), cosTheta = cosf(e.pixelSizeY * (posy + 0.5f));
    d = v3(sinPhi * sinTheta, cosTheta, -cosPhi * sinTheta);
    pdf /= fmaxr(fabsf(sinTheta), kEpsilon);
}
HD bool bsphereIntersect(const HptEnvMap &e, V3 o, V3 d, float &nearT, float &farT) { /* bsphere.h:88-95 */
    V3 oo = o - v3(e.bsCenter[0], e.bsCenter[1], e.bsCenter[2]);
    float A = dot(d, d);
    float B = 2 * dot(oo, d);
    float C = dot(oo, oo) - e.bsRadius * e.bsRadius;
    return solveQuadratic(A, B, C, nearT, farT);
}

HD float miWeight(float pdfA, float pdfB) { /* path.cpp:296-300 */
    pdfA *= pdfA;
    pdfB *= pdfB;
    return pdfA / (pdfA + pdfB);
}


/* Append to a queue with one atomic per BLOCK: wave ballots give per-wave
   counts, the block's waves are laid out in wave order after a single
   atomicAdd by thread 0.  A million same-address atomics per launch (one per
   wave) serialised in L2 and dominated k_camera / k_primary; per block they
   are 16x fewer.  Every thread of the block must call it (no early exits). */
template <int BLOCK>
__device__ __forceinline__ void qpushBlock(bool pred, uint32_t value, uint32_t *queue, uint32_t *counter) {
    constexpr int NW = BLOCK / 64;
    __shared__ uint32_t waveCount[NW];
    __shared__ uint32_t blockBase;
    const uint64_t mask = __ballot(pred);
    const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
    if (lane == 0) waveCount[wave] = (uint32_t) __popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < NW; ++w) {
            const uint32_t c = waveCount[w];
            waveCount[w] = tot;
            tot += c;
        }
        blockBase = tot ? atomicAdd(counter, tot) : 0u;
    }
    __syncthreads();
    if (pred) queue[blockBase + waveCount[wave] + (uint32_t) __popcll(mask & ((1ull << lane) - 1ull))] = value;
    __syncthreads(); /* waveCount / blockBase may be reused by a second push */
}

/* The camera queue's push: qpushBlock, but a pixel's samples are laid out by
   the quadrant of the pixel their film position falls in (then in sample
   order), so a 64-ray packet of k_trace_packet covers a quarter of the pixel
   instead of all of it when a wave holds 256 of its samples.  A segment is
   the wps consecutive waves holding one pixel's samples (wps = 1: no
   reordering); queue order is (segment, quadrant, wave, lane).  The per-(wave,
   quadrant) counts, 64 for a 1024-thread block, are scanned by wave 0 and the
   block takes one atomicAdd.  Only the queue order changes: every path's ray,
   hit and film contribution are its own. */
template <int BLOCK>
__device__ __forceinline__ void qpushCamera(bool pred, uint32_t quad, uint32_t wps, uint32_t value, uint32_t *queue,
                                            uint32_t *counter) {
    constexpr int NW = BLOCK / 64, NE = NW * 4;
    static_assert(NE <= 64, "one wave scans the (wave, quadrant) counts");
    __shared__ uint32_t cnt[NE];
    const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
    const uint32_t wIn = wave % wps;
    const uint32_t fBase = (wave - wIn) * 4 + wIn; /* + quadrant * wps */
    uint64_t mine = 0;
#pragma unroll
    for (uint32_t q = 0; q < 4; ++q) {
        const uint64_t m = __builtin_amdgcn_ballot_w64(pred && quad == q);
        if (lane == q) cnt[fBase + q * wps] = (uint32_t) __popcll(m);
        if (quad == q) mine = m;
    }
    __syncthreads();
    if (wave == 0) {
        const uint32_t c = lane < (uint32_t) NE ? cnt[lane] : 0u;
        uint32_t incl = c;
#pragma unroll
        for (int s = 1; s < 64; s <<= 1) {
            const uint32_t u = __shfl_up(incl, s);
            if (lane >= (uint32_t) s) incl += u;
        }
        uint32_t base = 0;
        if (lane == 63) base = incl ? atomicAdd(counter, incl) : 0u;
        base = __shfl(base, 63);
        if (lane < (uint32_t) NE) cnt[lane] = base + incl - c;
    }
    __syncthreads();
    if (pred) queue[cnt[fBase + quad * wps] + (uint32_t) __popcll(mine & ((1ull << lane) - 1ull))] = value;
}

/* qpushBlock that also stores value2 at the same position of a parallel array */
template <int BLOCK>
__device__ __forceinline__ void qpushBlock2(bool pred, uint32_t value, uint32_t *queue, uint32_t value2,
                                            uint32_t *array2, uint32_t *counter) {
    constexpr int NW = BLOCK / 64;
    __shared__ uint32_t waveCount[NW];
    __shared__ uint32_t blockBase;
    const uint64_t mask = __ballot(pred);
    const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
    if (lane == 0) waveCount[wave] = (uint32_t) __popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < NW; ++w) {
            const uint32_t c = waveCount[w];
            waveCount[w] = tot;
            tot += c;
        }
        blockBase = tot ? atomicAdd(counter, tot) : 0u;
    }
    __syncthreads();
    if (pred) {
        const uint32_t pos = blockBase + waveCount[wave] + (uint32_t) __popcll(mask & ((1ull << lane) - 1ull));
        queue[pos] = value;
        array2[pos] = value2;
    }
    __syncthreads();
}

/* qpushBlock that also stores an NR-float4 record at the same position of recs and, with
   array2, a word there */
template <int BLOCK, int NR>
__device__ __forceinline__ uint32_t qpushBlockRec(bool pred, uint32_t value, uint32_t *queue, uint32_t *counter,
                                                  float4 *recs, const float4 *rec, uint32_t *array2 = nullptr,
                                                  uint32_t value2 = 0u) {
    constexpr int NW = BLOCK / 64;
    __shared__ uint32_t waveCount[NW];
    __shared__ uint32_t blockBase;
    const uint64_t mask = __ballot(pred);
    const uint32_t lane = __lane_id(), wave = threadIdx.x >> 6;
    if (lane == 0) waveCount[wave] = (uint32_t) __popcll(mask);
    __syncthreads();
    if (threadIdx.x == 0) {
        uint32_t tot = 0;
        for (int w = 0; w < NW; ++w) {
            const uint32_t c = waveCount[w];
            waveCount[w] = tot;
            tot += c;
        }
        blockBase = tot ? atomicAdd(counter, tot) : 0u;
    }
    __syncthreads();
    const uint32_t pos = blockBase + waveCount[wave] + (uint32_t) __popcll(mask & ((1ull << lane) - 1ull));
    if (pred) {
        if (queue) queue[pos] = value;
#pragma unroll
        for (int i = 0; i < NR; ++i) recs[NR * pos + i] = rec[i];
        if (array2) array2[pos] = value2;
    }
    __syncthreads();
    return pos; /* the entry's queue position (meaningful where pred) */
}

/* one shaded path-bounce of path `id` per lane where pred, added to its block's cost: lanes
   of the same block share one atomic (a wave's paths are mostly of one or two blocks), into
   the wave's stripe of the counters (HptPaths::blockCost) */
__device__ __forceinline__ void countBlockCost(const HptPaths &P, bool pred, uint32_t id) {
    if (!P.blockCost) return;
    const uint32_t blk = pred ? (id / P.costSpp) >> 10 : 0xffffffffu;
    uint32_t *const stripe =
        P.blockCost + ((blockIdx.x * (blockDim.x >> 6) + (threadIdx.x >> 6)) % HPT_COST_STRIPES) * P.costStride;
    uint64_t todo = __ballot(pred);
    while (todo) { /* wave-uniform */
        const int L = __ffsll((unsigned long long) todo) - 1;
        const uint32_t b = (uint32_t) __builtin_amdgcn_readlane((int) blk, L);
        const uint64_t m = __ballot(pred && blk == b);
        if (__lane_id() == (uint32_t) L) atomicAdd(&stripe[b], (uint32_t) __popcll(m));
        todo &= ~m;
    }
}

/* append to a queue: one atomic per wave (wave64 ballot + mbcnt) */
HD void qpush(bool pred, uint32_t value, uint32_t *queue, uint32_t *counter) {
    uint64_t mask = __ballot(pred);
    if (mask == 0) return;
    uint32_t lane = __lane_id();
    uint32_t leader = __ffsll((unsigned long long) mask) - 1;
    uint32_t base = 0;
    if (lane == leader) base = atomicAdd(counter, (uint32_t) __popcll(mask));
    base = __shfl(base, leader);
    if (pred) {
        uint64_t below = mask & ((1ull << lane) - 1ull);
        queue[base + __popcll(below)] = value;
    }
}

} // namespace

/* ================================================================== */
/* Kernels                                                             */
/* ================================================================== */

/* PerspectiveCameraImpl::sampleRayDifferential, the ray itself (perspective.cpp:271-290).  The
   origin is the same for every ray (cameraOrigin), and mint / maxt are the clip distances times
   1 / d.z: k_camera stores the world direction and that factor, and the trace launch and
   k_primary rebuild the ray from them bit for bit (cameraRayFrom). */
HD V3 cameraOrigin(const HptCamera &c) { return v3(c.origin[0], c.origin[1], c.origin[2]); }
HD void cameraRay(const HptCamera &c, float posx, float posy, V3 &o, V3 &dw, float &mint, float &maxt,
                  float *invZOut = nullptr) {
    const V3 nearP = xformPoint(c.s2c, v3(posx * c.invResX, posy * c.invResY, 0.0f));
    const V3 d = normalize(nearP);
    const float invZ = 1.0f / d.z;
    o = cameraOrigin(c);
    dw = xformVector(c.toWorld, d);
    mint = c.nearClip * invZ;
    maxt = c.farClip * invZ;
    if (invZOut) *invZOut = invZ;
}
/* the camera ray from k_camera's record {world direction, 1 / d.z} */
HD void cameraRayFrom(const HptCamera &c, float4 rec, V3 &o, V3 &dw, float &mint, float &maxt) {
    o = cameraOrigin(c);
    dw = v3(rec.x, rec.y, rec.z);
    mint = c.nearClip * rec.w;
    maxt = c.farClip * rec.w;
}

/* Decode a path id of the current wave: id = slot * nSpp + (j - sppBegin),
   slot = (k-th block owned by this shard) << 10 | pixel within the block. */
HD bool decodePath(const HptWave &w, uint32_t id, int &px, int &py, uint32_t &j) {
    uint32_t slot = id / w.nSpp;
    j = w.sppBegin + (id - slot * w.nSpp);
    uint32_t lb = slot >> 10, inner = slot & 1023u;
    uint32_t b = w.blockOf[lb];
    px = (int) ((b % w.nbx) * HPT_BLOCK + (inner & 31u));
    py = (int) ((b / w.nbx) * HPT_BLOCK + (inner >> 5));
    return px < w.width && py < w.height;
}

extern "C" __global__ __launch_bounds__(HPT_QBLOCK) void k_camera(HptScene sc, HptWave w, HptPaths P,
                                                            uint32_t *__restrict__ traceQ,
                                                            uint32_t *__restrict__ nTrace) {
    uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    bool valid = id < w.nPaths;
    int px = 0, py = 0;
    uint32_t j = 0, quad = 0;
    if (valid) valid = decodePath(w, id, px, py, j);
    /* a pixel's samples as whole waves of the block: sort them by quadrant (qpushCamera) */
    const uint32_t wps = (w.nSpp % 64u == 0 && w.nSpp >= 128u && HPT_QBLOCK % w.nSpp == 0) ? w.nSpp / 64u : 1u;
    if (valid) {
        const HptCamera &c = sc.cam;
        /* the wave's frames are below sppBegin + nSpp: a uniform bound on their bits */
        const uint32_t lastFrame = w.sppBegin + w.nSpp - 1u;
        const uint32_t frameBits = lastFrame ? 32u - (uint32_t) __builtin_clz(lastFrame) : 0u;
        uint64_t sidx = (c.logRes > 1) ? sobolLookUpWave(sc, c.logRes, j, (uint32_t) px, (uint32_t) py, frameBits)
                                       : (uint64_t) j;
        float ox, oy;
        if (sidx != (uint64_t) j) {
            ox = sobolSample(sc, sidx, 0) * c.resolution - px;
            oy = sobolSample(sc, sidx, 1) * c.resolution - py;
        } else {
            ox = sobolSample(sc, sidx, 0);
            oy = sobolSample(sc, sidx, 1);
        }
        float posx = px + ox, posy = py + oy;
        if (wps > 1) quad = (posx - px >= 0.5f ? 1u : 0u) | (posy - py >= 0.5f ? 2u : 0u);
        /* the ray as its world direction and 1 / d.z (cameraRayFrom rebuilds the common origin
           and the clip distances): 16 bytes instead of 32.  A camera path's throughput (1), state
           (dim 2, depth 1) and radiance (0, or the environment on a miss) are k_primary's to
           write, so none of them goes through HBM here */
        V3 o, dw;
        float mint, maxt, invZ;
        cameraRay(c, posx, posy, o, dw, mint, maxt, &invZ);
        P.rd[id] = make_float4(dw.x, dw.y, dw.z, invZ);
        P.pos[id] = make_float2(posx, posy);
        P.sobol[id] = sidx;
    }
    qpushCamera<HPT_QBLOCK>(valid, quad, wps, id, traceQ, nTrace);
}

/* k_trace: the wave's closest-hit rays (traceQ[0, nTrace)) then its any-hit
   shadow rays (shadowQ) as one persistent grid; k_trace_counted adds the
   traversal counters of the byte model (one counted frame per bench run) */
/* Closest-hit records go to P.hitQ by trace-queue position (the wavefront
   kernels; k_primary / k_post read them in queue order), or to P.hit by path
   (byQueue false: k_tail).  A record is 4 bytes (segment | far root << 31, or
   HPT_MISS) and consecutive queue positions belong to the rays one wave
   claimed together, so a launch's record writes fill whole lines in L2
   instead of a 32-byte sector per lone path-indexed 16-byte store.
   posQ (k_trace_overflow): the queue positions of the rays to trace. */
struct PathIO {
    HptPaths P;
    const uint32_t *traceQ, *shadowQ;
    uint32_t nTrace, nShadow, id;
    bool byQueue;
    const uint32_t *posQ;
    bool recs; /* bounce launches: rays from the queue-ordered records, keys are queue positions */
    /* work indices: closest rays [0, nTrace), then shadow rays, in HPT_CURSORS contiguous shards */
    HD uint32_t count() const { return nTrace + nShadow; }
    HD uint32_t shardSize(uint32_t s) const { return shardLo(count(), s + 1) - shardLo(count(), s); }
    HD uint32_t item(uint32_t s, uint32_t j) const { return shardLo(count(), s) + j; }
    HD bool begin(const HptScene &sc, uint32_t k, TraceRay &r) {
        if (recs) { /* a bounce ray leaves the hit point at kEpsilon (path.cpp:213, scene.cpp:838) */
            if (k < nTrace) {
                id = k;
                const float4 o = P.postRec[4 * k], d = P.postRec[4 * k + 1];
                return beginRay(sc, r, v3(o.x, o.y, o.z), v3(d.x, d.y, d.z), kEpsilon, finf(), false);
            }
            id = k - nTrace;
            const float4 o = P.shadowRec[3 * id], d = P.shadowRec[3 * id + 1];
            return beginRay(sc, r, v3(o.x, o.y, o.z), v3(d.x, d.y, d.z), kEpsilon, d.w, true);
        }
        if (k < nTrace) {
            const uint32_t q = posQ ? posQ[k] : k;
            const uint32_t path = traceQ[q];
            id = byQueue ? q : path; /* the key: where finish() writes the record */
            if (byQueue) { /* the camera pass: k_camera's record {direction, 1 / d.z} */
                V3 o, dw;
                float mint, maxt;
                cameraRayFrom(sc.cam, P.rd[path], o, dw, mint, maxt);
                return beginRay(sc, r, o, dw, mint, maxt, false);
            }
            const float4 ro = P.ro[path], rd = P.rd[path];
            return beginRay(sc, r, v3(ro.x, ro.y, ro.z), v3(rd.x, rd.y, rd.z), ro.w, rd.w, false);
        }
        id = shadowQ[k - nTrace];
        const float4 ro = P.ro[id], sd = P.sdir[id];
        return beginRay(sc, r, v3(ro.x, ro.y, ro.z), v3(sd.x, sd.y, sd.z), kEpsilon, sd.w, true);
    }
    HD uint32_t key() const { return id; }
    /* id: the record's queue position / path (closest), the path (shadow ray);
       returns 1 for an unoccluded shadow ray */
    HD uint32_t finish(const HptScene &sc, uint32_t id, const TraceRay &r) {
        if (HPT_PROBE_WANTS_PATH) {
            const uint32_t path = r.shadow ? (recs ? shadowQ[id] : id) : (byQueue && traceQ && !posQ ? traceQ[id] : HPT_MISS);
            probeRayFinished(r, path, r.shadow ? nTrace + id : id, recs);
        }
        if (!r.shadow) {
            /* the shading kernel re-derives the point from the segment and the accepted root */
            (byQueue ? P.hitQ : P.hit)[id] = r.found ? r.segHit : HPT_MISS;
            return 0;
        }
        if (r.found) return 0;
        const uint32_t path = recs ? shadowQ[id] : id;
        const float4 c = recs ? P.shadowRec[3 * id + 2] : P.scontrib[id], l = P.li[path];
        P.li[path] = make_float4(l.x + c.x, l.y + c.y, l.z + c.z, l.w);
        return 1;
    }
};

/* The IO of a bounce's trace launch (k_trace): rays from the queue-ordered records.  Work
   indices: the closest rays [0, nTrace), then the shadow rays; the key of a ray is its work
   index (closest: its trace-queue position, where k_post reads the hit record; shadow: nTrace +
   its shadow-queue position). */
struct BounceIO {
    HptPaths P;
    const uint32_t *traceQ, *shadowQ;
    uint32_t nTrace, nShadow, id;
    HD uint32_t count() const { return nTrace + nShadow; }
    HD uint32_t shardSize(uint32_t s) const { return shardLo(count(), s + 1) - shardLo(count(), s); }
    HD uint32_t item(uint32_t s, uint32_t j) const { return shardLo(count(), s) + j; }
    HD uint32_t key() const { return id; }
    HD bool begin(const HptScene &sc, uint32_t k, TraceRay &r) {
        id = k;
        /* a bounce ray leaves the hit point at kEpsilon (path.cpp:213, scene.cpp:838) */
        if (k < nTrace) {
            const float4 o = P.postRec[4 * k], d = P.postRec[4 * k + 1];
            return beginRay(sc, r, v3(o.x, o.y, o.z), v3(d.x, d.y, d.z), kEpsilon, finf(), false);
        }
        const uint32_t j = k - nTrace;
        const float4 o = P.shadowRec[3 * j], d = P.shadowRec[3 * j + 1];
        return beginRay(sc, r, v3(o.x, o.y, o.z), v3(d.x, d.y, d.z), kEpsilon, d.w, true);
    }
    /* returns 1 for an unoccluded shadow ray */
    HD uint32_t finish(const HptScene &sc, uint32_t key, const TraceRay &r) {
        if (HPT_PROBE_WANTS_PATH) probeRayFinished(r, r.shadow ? shadowQ[key - nTrace] : traceQ[key], key, true);
        if (!r.shadow) {
            /* the shading kernel re-derives the point from the segment and the accepted root */
            P.hitQ[key] = r.found ? r.segHit : HPT_MISS;
            return 0;
        }
        if (r.found) return 0;
        const uint32_t j = key - nTrace;
        const float4 c = P.shadowRec[3 * j + 2];
        const uint32_t path = shadowQ[j];
        const float4 l = P.li[path];
        P.li[path] = make_float4(l.x + c.x, l.y + c.y, l.z + c.z, l.w);
        return 1;
    }
};


/* k_trace launch shape (measured on MI355X, furball 512^2 @ 256 spp):
   persistent 256-thread blocks (64 and 128 are within 1.5%); an 8-entry ring
   stack (64 B/lane, kd-restart on overflow) beats 16 (-5%) and 4 (-11%, +12%
   node visits) entries.  The traversal is latency-bound, so waves per SIMD
   decide its speed (k_trace per frame: 4 waves 141 ms, 5: 117, 6: 106, 7: 99):
   7 waves need <= 72 VGPRs and <= 91 B of LDS per lane (64 B stack + 24 B of
   ray rows), which the LDS ray rows, the fp64 ray re-derivation in the exact
   test and the hit point moved to k_shade make possible without spills.
   Overridable for experiments (make variant). */
#ifndef HPT_TRACE_BLOCK
#define HPT_TRACE_BLOCK 256
#endif
#ifndef HPT_STACK
#define HPT_STACK 8
#endif
#ifndef HPT_TRACE_WAVES
#define HPT_TRACE_WAVES 7
#endif
#if HPT_TRACE_WAVES > 0 /* occupancy target (waves per SIMD) for k_trace's register allocation */
#define HPT_TRACE_OCCUPANCY __attribute__((amdgpu_waves_per_eu(HPT_TRACE_WAVES)))
#else
#define HPT_TRACE_OCCUPANCY
#endif

/* the queue lengths come from device memory (the launch is enqueued before
   the host knows them) */
HD BounceIO bounceIO(const HptPaths &P, const uint32_t *traceQ, const uint32_t *shadowQ, const uint32_t *nTrace,
                     const uint32_t *nShadow) {
    return BounceIO{P, traceQ, shadowQ, *nTrace, *nShadow, 0};
}
/* the next bounce's counts and cursor set start at zero (what a separate clearing launch did):
   nothing of this launch reads them, and the next bounce's first kernel runs after it */
__device__ __forceinline__ void clearNextParity(uint32_t *counters, uint32_t q) {
    if (!counters || blockIdx.x != 0) return;
    uint32_t *cur = counters + HPT_CURSOR_SET(q);
    for (uint32_t i = threadIdx.x; i < HPT_CURSORS; i += blockDim.x) cur[i * HPT_CURSOR_STRIDE] = 0;
    if (threadIdx.x == 0) {
        counters[HPT_C_TRACE(q)] = 0;
        counters[HPT_C_SHADOW(q)] = 0;
        counters[HPT_C_SHADE(q)] = 0;
    }
}
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) HPT_TRACE_OCCUPANCY void k_trace(
    HptScene sc, HptPaths P, const uint32_t *__restrict__ traceQ, const uint32_t *__restrict__ shadowQ,
    const uint32_t *__restrict__ nTrace, const uint32_t *__restrict__ nShadow, uint32_t *__restrict__ cursors,
    uint32_t *counters, uint32_t nextParity) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    BounceIO io = bounceIO(P, traceQ, shadowQ, nTrace, nShadow);
    clearNextParity(counters, nextParity);
    tracePersistent<HPT_STACK, false>(sc, io, cursors, stk + threadIdx.x, nullptr);
}
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) void k_trace_counted(HptScene sc, HptPaths P,
                                                                              const uint32_t *__restrict__ traceQ,
                                                                              const uint32_t *__restrict__ shadowQ,
                                                                              const uint32_t *__restrict__ nTrace,
                                                                              const uint32_t *__restrict__ nShadow,
                                                                              uint32_t *__restrict__ cursors,
                                                                              uint32_t *counters, uint32_t nextParity,
                                                                              uint32_t *stats) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    BounceIO io = bounceIO(P, traceQ, shadowQ, nTrace, nShadow);
    clearNextParity(counters, nextParity);
    tracePersistent<HPT_STACK, true>(sc, io, cursors, stk + threadIdx.x, stats);
}

/* the camera pass's rays one per lane (HPT_PACKETS=0): camera-queue positions are the keys and
   the hits go to P.hitQ by position, as the packet kernel writes them */
template <bool STATS>
__device__ __forceinline__ void traceCamera(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ,
                                            const uint32_t *nTrace, uint32_t *cursors, uint32_t *stats, uint2 *stk) {
    PathIO io{P, traceQ, nullptr, *nTrace, 0, 0, true, nullptr, false};
    tracePersistent<HPT_STACK, STATS>(sc, io, cursors, stk, stats);
}
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) HPT_TRACE_OCCUPANCY void k_trace_camera(
    HptScene sc, HptPaths P, const uint32_t *__restrict__ traceQ, const uint32_t *__restrict__ nTrace,
    uint32_t *__restrict__ cursors) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    traceCamera<false>(sc, P, traceQ, nTrace, cursors, nullptr, stk + threadIdx.x);
}
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) void k_trace_camera_counted(
    HptScene sc, HptPaths P, const uint32_t *__restrict__ traceQ, const uint32_t *__restrict__ nTrace,
    uint32_t *__restrict__ cursors, uint32_t *stats) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    traceCamera<true>(sc, P, traceQ, nTrace, cursors, stats, stk + threadIdx.x);
}

/* k_trace_packet: the camera pass's closest-hit rays as 64-ray packets */
#ifndef HPT_PACKET_WAVES
#define HPT_PACKET_WAVES 8 /* 63 VGPRs, no spills (one leaf record per trip): 17.1 ms per frame (7 waves: 17.7) */
#endif
#ifndef HPT_PACKET_BLOCK
#define HPT_PACKET_BLOCK HPT_TRACE_BLOCK
#endif
extern "C" __global__ __launch_bounds__(HPT_PACKET_BLOCK) __attribute__((amdgpu_waves_per_eu(HPT_PACKET_WAVES))) void
k_trace_packet(HptScene sc, HptPaths P, const uint32_t *__restrict__ traceQ, const uint32_t *__restrict__ nTrace,
               uint32_t *__restrict__ cursors, uint32_t *__restrict__ overflowQ, uint32_t *__restrict__ nOverflow) {
    __shared__ PacketLds lds[HPT_PACKET_BLOCK / 64];
    PathIO io{P, traceQ, nullptr, *nTrace, 0, 0, true, nullptr, false};
    tracePackets<false, false>(sc, io, cursors, lds[threadIdx.x >> 6], nullptr, overflowQ, nOverflow);
}
extern "C" __global__ __launch_bounds__(HPT_PACKET_BLOCK) void k_trace_packet_counted(
    HptScene sc, HptPaths P, const uint32_t *__restrict__ traceQ, const uint32_t *__restrict__ nTrace,
    uint32_t *__restrict__ cursors, uint32_t *stats, uint32_t *__restrict__ overflowQ, uint32_t *__restrict__ nOverflow) {
    __shared__ PacketLds lds[HPT_PACKET_BLOCK / 64];
    PathIO io{P, traceQ, nullptr, *nTrace, 0, 0, true, nullptr, false};
    tracePackets<true, false>(sc, io, cursors, lds[threadIdx.x >> 6], stats, overflowQ, nOverflow);
}
/* the camera rays of packets whose stack overflowed, one lane per ray (k_trace's traversal;
   a separate symbol so the profiles keep k_trace's launches apart) */
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) HPT_TRACE_OCCUPANCY void k_trace_overflow(
    HptScene sc, HptPaths P, const uint32_t *__restrict__ traceQ, const uint32_t *__restrict__ overflowQ,
    const uint32_t *__restrict__ nOverflow, uint32_t *__restrict__ cursors) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    /* overflowQ holds camera-queue positions (the packet kernel's keys) */
    const uint32_t n = *nOverflow;
    /* none at the shipped configs: leave at once (the claim walk over every cursor shard took the
       empty launch 30 us per frame) */
    if (n == 0) return;
    PathIO io{P, traceQ, nullptr, n, 0, 0, true, overflowQ, false};
    tracePersistent<HPT_STACK, false>(sc, io, cursors, stk + threadIdx.x, nullptr);
}

/* fill the intersection record: hair.cpp:825-862 + skdtree.h:422-427 */
HD void fillIts(const HptScene &sc, uint32_t seg, V3 hp, V3 rayD, V3 &p, Frame &geo, Frame &sh, V3 &wi) {
    const double *rec = reinterpret_cast<const double *>(sc.segs + seg);
    V3 v1 = v3((float) rec[0], (float) rec[1], (float) rec[2]);
    V3 v2 = v3((float) rec[12], (float) rec[13], (float) rec[14]);
    V3 axis = normalize(v2 - v1);
    geo.s = axis;
    V3 rel = hp - v1;
    geo.n = normalize(rel - axis * dot(axis, rel));
    geo.t = cross(geo.n, geo.s);
    V3 local = geo.toLocal(rel);
    const float radius = segRadius(sc, seg);
    p = hp + geo.n * (radius - sqrtf(local.y * local.y + local.z * local.z));
    sh.n = geo.n;
    sh.s = normalize(geo.s - sh.n * dot(sh.n, geo.s));
    sh.t = cross(sh.n, sh.s);
    wi = sh.toLocal(-rayD);
}

/* primary hits / misses (path.cpp:128-143) */
extern "C" __global__ __launch_bounds__(HPT_QBLOCK) void k_primary(HptScene sc, HptPaths P,
                                                             const uint32_t *__restrict__ traceQ,
                                                             const uint32_t *__restrict__ nTrace,
                                                             uint32_t *__restrict__ shadeQ,
                                                             uint32_t *__restrict__ nShade) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = *nTrace;
    bool alive = false;
    uint32_t id = 0;
    uint32_t seg = HPT_MISS;
    float4 sOut[3];
    if (tid < n) {
        id = traceQ[tid];
        seg = P.hitQ[tid];
        V3 o, d;
        float mint, maxt;
        cameraRayFrom(sc.cam, P.rd[id], o, d, mint, maxt);
        float4 li = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
        if (seg != HPT_MISS) {
            alive = true;
            /* the shade record (hpt_kernels.h): the camera ray, its Sobol index, throughput 1 and
               the camera state (dim = 2, depth = 1) */
            const uint64_t sidx = P.sobol[id];
            sOut[0] = make_float4(o.x, o.y, o.z, __uint_as_float((uint32_t) sidx));
            sOut[1] = make_float4(d.x, d.y, d.z, __uint_as_float((uint32_t) (sidx >> 32)));
            sOut[2] = make_float4(1.0f, 1.0f, 1.0f, __uint_as_float(hptState(0u, 1u, 2u)));
        } else if (!sc.hideEmitters) {
            /* a camera ray keeps its differentials: EWA-filtered lookup (envmap.cpp:394-406) */
            const float2 pos = P.pos[id];
            V3 rx, ry;
            cameraDifferentials(sc.cam, pos.x, pos.y, d, rx, ry);
            V3 L = envEvalFiltered(sc.env, d, rx, ry); /* throughput == 1 */
            V3 T = v3(1.0f, 1.0f, 1.0f);
            V3 c = mul(T, L);
            li = make_float4(0.0f + c.x, 0.0f + c.y, 0.0f + c.z, 0.0f);
        }
        P.li[id] = li; /* every camera path's radiance starts here */
    }
    qpushBlockRec<HPT_QBLOCK, 3>(alive, id, shadeQ, nShade, P.shadeRec, sOut, P.hitS, seg);
}

/* one bounce of shading: path.cpp:145-232 up to the continuation ray cast.
   MULTI: several hair shapes, the hit shape's BSDF comes from sc.bsdfs (a
   separate kernel, so the single-shape one never mixes a kernel-argument
   pointer with a global one -- that would copy the scene to scratch) */
/* REC (the wavefront k_shade): the path comes from its shade record in[0..2] and the
   continuation / shadow ray go to the post record cOut[0..3] / shadow record sOut[0..2]
   (hpt_kernels.h), which the caller appends with the queues; k_tail (REC false) keeps
   everything by path */
template <bool MULTI, bool REC = false>
HD void shadePath(const HptScene &sc, HptPaths &P, uint32_t id, uint32_t hitRec, uint32_t *__restrict__ counters,
                  bool &cont, bool &shadow, const float4 *in, float4 *cOut, float4 *sOut, float *wiL) {
    {
        const int stride = REC ? HPT_SHADE_BLOCK : (int) blockDim.x; /* REC: k_shade's block, immediate LDS offsets */
        uint32_t st = REC ? __float_as_uint(in[2].w) : P.state[id];
        uint32_t dim = HPT_ST_DIM(st), depth = HPT_ST_DEPTH(st);
        const float4 ro = REC ? in[0] : P.ro[id], rd = REC ? in[1] : P.rd[id];
        V3 rayD = v3(rd.x, rd.y, rd.z);
        V3 p, wi;
        Frame geo, sh;
        const uint32_t seg = hitRec & 0x7fffffffu;
        /* the traced ray is still in ro / rd: the hit point from the accepted root (hair.cpp:519-541) */
        const V3 hp = segHitPoint(sc, seg, v3(ro.x, ro.y, ro.z), rayD, hitRec >> 31);
        fillIts(sc, seg, hp, rayD, p, geo, sh, wi);
        bool stop = ((int) depth >= sc.maxDepth && sc.maxDepth > 0) ||
                    (sc.strictNormals && dot(rayD, geo.n) * wi.z >= 0);
        if (!stop && dim + 3 >= HPT_SOBOL_DIMS) {
            /* sobol.cpp:236-238 raises "Lookup dimension exceeds the direction number table size" */
            atomicOr(&counters[HPT_C_ERROR], 1u);
            stop = true;
        }
        /* REC: p and the frame go to LDS rows and every later use reads them back (sh.n == geo.n,
           sh.t == cross(sh.n, sh.s) as fillIts computes it) */
        if (REC) {
            stashV3(wiL, stride, kRowP, p);
            stashV3(wiL, stride, kRowGeoN, geo.n);
            stashV3(wiL, stride, kRowShS, sh.s);
            asm volatile("" ::: "memory");
        }
        auto ldP = [&]() { return REC ? loadV3(wiL, stride, kRowP) : p; };
        auto ldGeoN = [&]() { return REC ? loadV3(wiL, stride, kRowGeoN) : geo.n; };
        auto ldSh = [&]() {
            if (!REC) return sh;
            Frame f;
            f.n = loadV3(wiL, stride, kRowGeoN);
            f.s = loadV3(wiL, stride, kRowShS);
            f.t = cross(f.n, f.s);
            return f;
        };
        /* one inlined copy per BSDF source: the scene's own (kernel
           argument, scalar loads) or, with several hair shapes, the hit
           shape's entry of sc.bsdfs */
        auto shadeWith = [&](const HptBsdf &B) {
            const uint64_t sidx = REC ? ((uint64_t) __float_as_uint(rd.w) << 32) | __float_as_uint(ro.w) : P.sobol[id];
            const float4 thr = REC ? in[2] : P.thr[id];
            V3 T = v3(thr.x, thr.y, thr.z);
            /* Marschner: the wi terms of the bounce's NEE evaluation and BSDF sample, once */
            const bool mar = B.kind == HPT_BSDF_MARSCHNER;
            if (REC) {
                if (mar) wiL[kRowWiY * stride] = wi.y;
                else stashV3(wiL, stride, 0, wi);
            }
            if (mar) stashWi(wiL, stride, marschnerWi(B.mar, wi));
            else if (REC) asm volatile("" ::: "memory");
            auto ldWi = [&]() {
                if (!REC) return wi;
                if (mar) {
                    asm volatile("" ::: "memory");
                    return v3(0.0f, wiL[kRowWiY * stride], 0.0f);
                }
                return loadV3(wiL, stride, 0);
            };
            /* ---- direct illumination (path.cpp:175, scene.cpp:828-852, envmap.cpp:516-543) ---- */
            if (B.smooth) {
                float nx = sobolSampleUniform<!REC>(sc, sidx, dim), ny = sobolSampleUniform<!REC>(sc, sidx, dim + 1);
                dim += 2;
                V3 dl, value;
                float pdf;
                envSampleDir(sc.env, nx, ny, dl, value, pdf);
                V3 dW = envToWorld(sc.env, dl);
                float nearT, farT;
                if (!(isZero(value) || pdf == 0 || !bsphereIntersect(sc.env, ldP(), dW, nearT, farT) || nearT >= 0 ||
                      farT <= 0)) {
                    V3 val = divs(value, pdf);
                    V3 wo = ldSh().toLocal(dW);
                    V3 bsdfVal = mar ? marschnerEvalW(B.mar, loadWi(wiL, stride), wo) : bsdfEval(B, ldWi(), wo);
                    if (!isZero(bsdfVal) && (!sc.strictNormals || dot(ldGeoN(), dW) * wo.z > 0)) {
                        float bp = bsdfPdf(B, ldWi(), wo);
                        float weight = miWeight(pdf, bp);
                        V3 c = mul(mul(T, val), bsdfVal) * weight;
                        const float4 sd = make_float4(dW.x, dW.y, dW.z, farT * (1 - kShadowEpsilon));
                        const float4 sc4 = make_float4(c.x, c.y, c.z, 0.0f);
                        if (REC) {
                            stashV3(wiL, stride, kRowSd, dW);
                            wiL[(kRowSd + 3) * stride] = sd.w;
                            stashV3(wiL, stride, kRowSc, c);
                            asm volatile("" ::: "memory");
                        } else {
                            P.sdir[id] = sd;
                            P.scontrib[id] = sc4;
                        }
                        shadow = true;
                    }
                }
            }
            /* ---- BSDF sampling ---- */
            float bx = sobolSampleUniform<!REC>(sc, sidx, dim), by = sobolSampleUniform<!REC>(sc, sidx, dim + 1);
            dim += 2;
            V3 woL;
            float bpdf = 0.0f;
            uint32_t type = 0;
            V3 w;
            if (mar) {
                bpdf = 1.0f;
                w = marschnerSampleW(B.mar, loadWi(wiL, stride), GlobalTabs{B.mar}, ldWi(), bx, by, woL, type);
            } else {
                w = bsdfSample(B, ldWi(), bx, by, woL, bpdf, type);
            }
            if (!isZero(w)) {
                V3 wo = ldSh().toWorld(woL);
                float woDotGeoN = dot(ldGeoN(), wo);
                if (!(sc.strictNormals && woDotGeoN * woL.z <= 0)) {
                    const float4 bw = make_float4(w.x, w.y, w.z, bpdf);
                    if (REC) {
                        const V3 p = ldP();
                        cOut[0] = make_float4(p.x, p.y, p.z, ro.w); /* the Sobol index travels in .w */
                        cOut[1] = make_float4(wo.x, wo.y, wo.z, rd.w);
                        cOut[2] = bw;
                        cOut[3] = thr;
                    } else {
                        P.ro[id] = make_float4(p.x, p.y, p.z, kEpsilon);
                        P.rd[id] = make_float4(wo.x, wo.y, wo.z, finf());
                        P.bw[id] = bw;
                    }
                    cont = true;
                    /* bits 24-30: sampled type; bit 31: 'scattered' (path.cpp:205) */
                    st = (st & 0x80ffffffu) | (type << 24) | (type != HPT_ENULL ? 0x80000000u : 0u);
                }
            }
            if (!REC && shadow && !cont) P.ro[id] = make_float4(p.x, p.y, p.z, kEpsilon);
        };
        if (!stop) {
            if (MULTI) shadeWith(sc.bsdfs[sc.shapes[sc.segs[seg].shape].bsdf]);
            else shadeWith(sc.bsdf);
        }
        st = (st & ~HPT_ST_DIM_MASK) | dim;
        if (REC) cOut[3].w = __uint_as_float(st);
        else P.state[id] = st;
    }
}
/* where a shading launch reads and appends: its shade queue's length, the
   next trace launch's queue lengths, and the counter block (error word) */
struct HptShadeIO {
    const uint32_t *nShade;
    uint32_t *nTrace, *nShadow, *counters;
    uint32_t tailFrom; /* a queue shorter than this is k_tail's (device-side bounce control); 0: always shade */
};
template <bool MULTI>
__device__ __forceinline__ void shadeBounce(const HptScene &sc, HptPaths &P, const uint32_t *__restrict__ shadeQ,
                                            uint32_t *__restrict__ traceQ, uint32_t *__restrict__ shadowQ,
                                            const HptShadeIO &q) {
    __shared__ float wiLds[kShadeRows * HPT_SHADE_BLOCK];
    float *const wiL = wiLds + threadIdx.x;
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n0 = *q.nShade;
    /* a short queue is the tail launch's bounce */
    const uint32_t n = n0 < q.tailFrom ? 0u : n0;
    if (blockIdx.x == 0 && threadIdx.x == 0 && n != 0) {
        atomicAdd((unsigned long long *) (q.counters + HPT_C_BOUNCES), (unsigned long long) n);
        atomicAdd(&q.counters[HPT_C_LAUNCHES], 1u);
        /* a grid sized from a schedule (bounces launched ahead) that is too small for the queue:
           the host renders the wave again, reading every queue length back */
        if ((uint64_t) n > (uint64_t) gridDim.x * blockDim.x) atomicOr(&q.counters[HPT_C_OVERFLOW], 1u);
    }
    bool cont = false, shadow = false;
    uint32_t id = 0;
    float4 in[3], cOut[4], sOut[3];
    countBlockCost(P, tid < n, tid < n ? shadeQ[tid] : 0u);
    if (tid < n) {
        id = shadeQ[tid];
#pragma unroll
        for (int i = 0; i < 3; ++i) in[i] = P.shadeRec[3 * tid + i];
        shadePath<MULTI, true>(sc, P, id, P.hitS[tid], q.counters, cont, shadow, in, cOut, sOut, wiL);
    }
    qpushBlockRec<HPT_SHADE_BLOCK, 4>(cont, id, traceQ, q.nTrace, P.postRec, cOut);
    if (shadow) { /* the shadow record from its LDS rows */
        const V3 p = loadV3(wiL, HPT_SHADE_BLOCK, kRowP), d = loadV3(wiL, HPT_SHADE_BLOCK, kRowSd);
        const V3 c = loadV3(wiL, HPT_SHADE_BLOCK, kRowSc);
        sOut[0] = make_float4(p.x, p.y, p.z, 0.0f);
        sOut[1] = make_float4(d.x, d.y, d.z, wiL[(kRowSd + 3) * HPT_SHADE_BLOCK]);
        sOut[2] = make_float4(c.x, c.y, c.z, 0.0f);
    }
    qpushBlockRec<HPT_SHADE_BLOCK, 3>(shadow, id, shadowQ, q.nShadow, P.shadowRec, sOut);
}
#ifndef HPT_SHADE_WAVES
/* 6: 72 VGPRs with the shading frame, wi and the shadow record in LDS (25 rows, 25.6 KB per block:
   six blocks fill the CU's LDS); 0: natural allocation (87 VGPRs = 5 waves/SIMD).
   Measured: k_shade 15.55 -> 15.14 ms per frame (C3) */
#define HPT_SHADE_WAVES 6
#endif
#if HPT_SHADE_WAVES > 0
#define HPT_SHADE_OCCUPANCY __attribute__((amdgpu_waves_per_eu(HPT_SHADE_WAVES)))
#else
#define HPT_SHADE_OCCUPANCY
#endif
extern "C" __global__ __launch_bounds__(HPT_SHADE_BLOCK) HPT_SHADE_OCCUPANCY void k_shade(HptScene sc, HptPaths P,
                                                           const uint32_t *__restrict__ shadeQ,
                                                           uint32_t *__restrict__ traceQ,
                                                           uint32_t *__restrict__ shadowQ, HptShadeIO q) {
    shadeBounce<false>(sc, P, shadeQ, traceQ, shadowQ, q);
}
extern "C" __global__ __launch_bounds__(HPT_SHADE_BLOCK) void k_shade_multi(HptScene sc, HptPaths P,
                                                                 const uint32_t *__restrict__ shadeQ,
                                                                 uint32_t *__restrict__ traceQ,
                                                                 uint32_t *__restrict__ shadowQ, HptShadeIO q) {
    shadeBounce<true>(sc, P, shadeQ, traceQ, shadowQ, q);
}

/* continuation result: path.cpp:225-286; true when the path goes on */
/* REC (k_post): the path from its post record rec[0..3], and a survivor's throughput and
   state go to sOut[2] of its next shade record (sOut[0..1] = the traced ray = rec[0..1]);
   k_tail (REC false) keeps everything by path */
template <bool REC = false>
HD bool postPath(const HptScene &sc, HptPaths &P, uint32_t id, bool hit, uint32_t *__restrict__ counters,
                 const float4 *rec = nullptr, float4 *sOut = nullptr) {
    bool alive = false;
    {
        uint32_t st = REC ? __float_as_uint(rec[3].w) : P.state[id];
        uint32_t dim = HPT_ST_DIM(st), depth = HPT_ST_DEPTH(st), type = (st >> 24) & 0x7fu;
        const bool scattered = (st >> 31) != 0;
        float4 bw = REC ? rec[2] : P.bw[id], thr = REC ? rec[3] : P.thr[id];
        V3 T = v3(thr.x, thr.y, thr.z);
        bool done = false, hitEmitter = false;
        V3 value = v3(0, 0, 0);
        V3 d = v3(0, 0, 0);
        if (!hit) {
            const float4 rd = REC ? rec[1] : P.rd[id]; /* the direction matters only for a miss */
            d = v3(rd.x, rd.y, rd.z);
            /* path.cpp:238-240: only a pass-through (ENull) chain from the camera is unscattered */
            value = envEval(sc.env, d);
            float4 ro = REC ? rec[0] : P.ro[id];
            float nearT, farT;
            if ((sc.hideEmitters && !scattered) ||
                !bsphereIntersect(sc.env, v3(ro.x, ro.y, ro.z), d, nearT, farT) || nearT > 0 || farT < 0) {
                done = true;
                hitEmitter = false;
            } else {
                hitEmitter = true;
            }
        }
        if (!(done && !hitEmitter)) {
            T = mul(T, v3(bw.x, bw.y, bw.z));
            if (hitEmitter) {
                float lumPdf = (!(type & HPT_EDELTA)) ? envPdf(sc.env, envToLocal(sc.env, d)) : 0.0f;
                V3 c = mul(T, value) * miWeight(bw.w, lumPdf);
                float4 l = P.li[id];
                P.li[id] = make_float4(l.x + c.x, l.y + c.y, l.z + c.z, l.w);
            }
            if (hit) {
                alive = true;
                if ((int) depth >= sc.rrDepth && dim >= HPT_SOBOL_DIMS) {
                    atomicOr(&counters[HPT_C_ERROR], 1u);
                    alive = false;
                } else if ((int) depth >= sc.rrDepth) {
                    float q = fminr(maxc(T) * 1.0f * 1.0f, 0.95f);
                    const uint64_t sidx =
                        REC ? ((uint64_t) __float_as_uint(rec[1].w) << 32) | __float_as_uint(rec[0].w) : P.sobol[id];
                    float u = sobolSampleUniform<!REC>(sc, sidx, dim);
                    dim += 1;
                    if (u >= q) alive = false;
                    else T = divs(T, q);
                }
                depth += 1;
                if (REC) {
                    sOut[0] = rec[0];
                    sOut[1] = rec[1];
                    sOut[2] = make_float4(T.x, T.y, T.z, __uint_as_float(hptState(st, depth, dim)));
                } else {
                    P.thr[id] = make_float4(T.x, T.y, T.z, 0.0f);
                    P.state[id] = hptState(st, depth, dim);
                }
            }
        }
    }
    return alive;
}
/* continuation results of a bounce (the paths of its trace queue) */
extern "C" __global__ __launch_bounds__(HPT_POST_BLOCK) void k_post(HptScene sc, HptPaths P,
                                                          const uint32_t *__restrict__ traceQ,
                                                          const uint32_t *__restrict__ nTrace,
                                                          uint32_t *__restrict__ shadeQ, uint32_t *__restrict__ nShade,
                                                          uint32_t *__restrict__ counters) {
    const uint32_t tid = blockIdx.x * blockDim.x + threadIdx.x;
    const uint32_t n = *nTrace; /* <= the bounce's shade queue, which k_shade checked against the grid */
    bool alive = false;
    uint32_t id = 0;
    uint32_t seg = HPT_MISS;
    float4 rec[4], sOut[3];
    if (tid < n) {
        id = traceQ[tid];
        seg = P.hitQ[tid];
#pragma unroll
        for (int i = 0; i < 4; ++i) rec[i] = P.postRec[4 * tid + i];
        alive = postPath<true>(sc, P, id, seg != HPT_MISS, counters, rec, sOut);
    }
    /* the survivors' shade records and hit records travel with the shade queue, in its order */
    qpushBlockRec<HPT_POST_BLOCK, 3>(alive, id, shadeQ, nShade, P.shadeRec, sOut, P.hitS, seg);
}

/* Tail of the frame (few live paths left, after Russian roulette has
   culled most of them): a lane pair carries its path through every
   remaining bounce -- shade, shadow ray, continuation ray, post -- inside
   one launch, so the tail costs the longest path's chain instead of one
   host-synchronised launch sequence per bounce, each waiting on its own
   slowest ray.  The even lane shades, traces the shadow ray and runs post;
   the odd lane traces the continuation ray at the same time.  Pairs take
   their paths from the shade queue, and a pair whose path ends claims the
   next one.  Every step is the
   wavefront kernels' own per-path function in the same order (the shadow
   contribution is added before post's emitter term, as k_trace finishes
   before k_post), so the film is bit-identical.  The traversal runs in
   latency mode (traceRound LAT): the tail is a chain of dependent memory
   round trips, not a bandwidth problem. */
struct HptTail {
    const uint32_t *shadeQ, *nShade;
    uint32_t pairs;    /* lane pairs per wave that take paths (1..32); 0: from the queue length, on the device */
    uint32_t tailFrom; /* the launch takes the queue only when it is shorter than this (device-side bounce control) */
};
#ifndef HPT_TAIL_SPLIT
#define HPT_TAIL_SPLIT 1 /* k_tail's idle lanes help trace its rays (RaySplitter); 0: one lane per ray, latency mode */
#endif
template <bool MULTI>
__device__ __forceinline__ void tailPaths(const HptScene &sc, HptPaths &P, const HptTail &T,
                                          uint32_t *__restrict__ counters, uint2 *stk) {
    __shared__ float wiLds[HPT_WI_ROWS * HPT_TRACE_BLOCK];
    float *const wiL = wiLds + threadIdx.x;
    const uint32_t lane = __lane_id(), partner = lane & ~1u;
    const bool odd = (lane & 1u) != 0;
    const uint32_t n0 = *T.nShade;
    const uint32_t total = n0 < T.tailFrom ? n0 : 0u;
    /* nothing to take (k_shade has the bounce, or no path is live): leave the claim cursor
       alone for a later tail launch of the same wave of paths */
    if (total == 0) return;
    if (blockIdx.x == 0 && threadIdx.x == 0) {
        atomicAdd(&counters[HPT_C_TAIL_PATHS], total);
        atomicAdd(&counters[HPT_C_LAUNCHES], 1u);
    }
    /* pairs per wave: the fewest that still cover the work in one residency of this grid */
    const uint32_t waves = gridDim.x * (blockDim.x >> 6);
    const uint32_t pairs = T.pairs ? T.pairs : min(32u, max(1u, (total + waves - 1) / waves));
    uint32_t id = 0, nb = 0, hitRec = 0;
    bool live = false, exhausted = false;
    TraceCounters tc;
    PathIO io{P, nullptr, nullptr, 0, 0, 0, false, nullptr, false};
    TailProbe probe;
    auto trace = [&](bool shadowRay) {
        TraceRay r;
        const float4 ro = P.ro[id], rd = shadowRay ? P.sdir[id] : P.rd[id];
        const bool act = beginRay(sc, r, v3(ro.x, ro.y, ro.z), v3(rd.x, rd.y, rd.z), shadowRay ? kEpsilon : ro.w, rd.w, shadowRay);
        stashRay<HPT_STACK>(stk, (int) blockDim.x, r, id);
        if (act)
            while (!traceRound<HPT_STACK, false, true>(sc, r, stk, (int) blockDim.x, tc)) probe.onRound();
        io.finish(sc, id, r);
    };
    while (true) {
        /* free pairs claim the next items (the even lane's rank, shared with the odd lane) */
        /* only the first `pairs` pairs of a wave take paths: a wave waits each bounce for
           its slowest ray, and the fewer paths share a wave, the shorter that wait is
           (the host spreads few paths thinly over the resident waves) */
        const uint64_t freeM = __ballot(!live && !odd && (lane >> 1) < pairs);
        if (!exhausted && freeM != 0) {
            uint32_t base = 0;
            if (lane == 0) base = atomicAdd(&counters[HPT_C_TAIL_CURSOR], (uint32_t) __popcll(freeM));
            base = __shfl(base, 0);
            if (base + (uint32_t) __popcll(freeM) >= total) exhausted = true;
            const uint32_t rk = __builtin_amdgcn_mbcnt_hi((uint32_t) (freeM >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) freeM, 0u));
            const uint32_t j = __shfl(base + rk, (int) partner);
            if (!live && (lane >> 1) < pairs && j < total) { /* exactly the pairs counted in freeM */
                id = T.shadeQ[j];
                hitRec = P.hitS[j];
                /* the shade record to the by-path arrays k_tail works on (both lanes of the
                   pair store the same values) */
                {
                    const float4 a = P.shadeRec[3 * j], b = P.shadeRec[3 * j + 1], c = P.shadeRec[3 * j + 2];
                    P.ro[id] = a;
                    P.rd[id] = b;
                    P.thr[id] = c;
                    P.state[id] = __float_as_uint(c.w);
                }
                live = true;
                probe.onItem(!odd);
            }
        }
        if (__ballot(live) == 0) {
            if (exhausted) break;
            continue;
        }
        probe.phase(0);
        bool cont = false, shadow = false;
        countBlockCost(P, live && !odd, id);
        if (live && !odd) {
            ++nb;
            shadePath<MULTI>(sc, P, id, hitRec, counters, cont, shadow, nullptr, nullptr, nullptr, wiL);
        }
        __threadfence_block(); /* the continuation ray is in HBM for the odd lane */
        const int f = __shfl((cont ? 1 : 0) | (shadow ? 2 : 0), (int) partner);
        cont = (f & 1) != 0;
        shadow = (f & 2) != 0;
        probe.phase(1);
        /* one call site: the shadow ray (even lane) and the continuation ray (odd
           lane) are traced at the same time, not one after the other */
        if (HPT_TAIL_SPLIT) {
            /* ... and the wave's idle lanes help: every pending subtree of a long ray can go to
               an idle lane (RaySplitter, the drain of k_trace), so a bounce waits for the
               wave's longest ray cut into pieces instead of whole */
            TraceRay r;
            bool act = false;
            if (live && (odd ? cont : shadow)) {
                const bool shadowRay = !odd;
                const float4 ro = P.ro[id], rd = shadowRay ? P.sdir[id] : P.rd[id];
                act = beginRay(sc, r, v3(ro.x, ro.y, ro.z), v3(rd.x, rd.y, rd.z), shadowRay ? kEpsilon : ro.w, rd.w,
                               shadowRay);
                stashRay<HPT_STACK>(stk, (int) blockDim.x, r, id);
                if (!act) io.finish(sc, id, r);
            }
            RaySplitter<HPT_STACK> split{stk, (int) blockDim.x};
            split.template drain<false>(sc, io, r, act, tc, probe);
        } else if (live && (odd ? cont : shadow)) {
            trace(!odd);
        }
        __threadfence_block(); /* the hit record is in HBM for the even lane */
        probe.phase(2);
        bool alive = false;
        if (live && !odd && cont) {
            hitRec = P.hit[id];
            alive = postPath(sc, P, id, hitRec != HPT_MISS, counters);
        }
        live = live && __shfl(alive ? 1 : 0, (int) partner) != 0;
        probe.phase(3);
    }
    for (int off = 32; off > 0; off >>= 1) nb += __shfl_down(nb, off);
    if (__lane_id() == 0 && nb) atomicAdd(&counters[HPT_C_TAIL_BOUNCES], nb);
    probe.finish();
}
/* persistent: pairs claim work, so any amount of it fits one launch.  No
   occupancy target: the tail is latency-bound and the traversal keeps its
   leaf records and exact-test records in registers (LAT) */
#ifndef HPT_TAIL_WAVES
#define HPT_TAIL_WAVES 2
#endif
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(HPT_TAIL_WAVES))) void
k_tail(HptScene sc, HptPaths P, HptTail T, uint32_t *__restrict__ counters) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    tailPaths<false>(sc, P, T, counters, stk + threadIdx.x);
}
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(HPT_TAIL_WAVES))) void
k_tail_multi(HptScene sc, HptPaths P, HptTail T, uint32_t *__restrict__ counters) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    tailPaths<true>(sc, P, T, counters, stk + threadIdx.x);
}

/* Deterministic film accumulation (imageblock.h:124-204 + renderproc.cpp:
   142-145) in two passes.  Weights use the sample's block-relative
   coordinates exactly like ImageBlock::put, and invalid samples (non-finite
   or negative, imageblock.h:147-151) are skipped.

   k_splat: one wave per owned pixel slot; its lanes read the slot's samples
   (consecutive path ids: coalesced) and accumulate the tent-weighted
   contribution to each of the 3x3 neighbour pixels, reduced across the wave
   with a fixed xor tree -> partial[slot][9] (RGB, weight). */
extern "C" __global__ __launch_bounds__(256) void k_splat(HptScene sc, HptWave w, HptPaths P,
                                                           float4 *__restrict__ partial) {
    if (w.doneIf && !hptWaveDone(w.doneIf, w.doneParity)) return; /* uniform: the host gathers later */
    const uint32_t slot = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
    const uint32_t lane = threadIdx.x & 63u;
    const uint32_t nSlots = w.nPaths / w.nSpp;
    if (slot >= nSlots) return; /* wave-uniform */
    const uint32_t lb = slot >> 10, inner = slot & 1023u;
    const uint32_t b = w.blockOf[lb];
    const int bx = (int) (b % w.nbx), by = (int) (b / w.nbx);
    const int px = bx * HPT_BLOCK + (int) (inner & 31u), py = by * HPT_BLOCK + (int) (inner >> 5);
    if (px >= w.width || py >= w.height) return; /* wave-uniform: never read back */
    const float ox = (float) (bx * HPT_BLOCK - 1), oy = (float) (by * HPT_BLOCK - 1);
    float acc[9][4];
#pragma unroll
    for (int k = 0; k < 9; ++k) acc[k][0] = acc[k][1] = acc[k][2] = acc[k][3] = 0.0f;
    /* the lane's samples lane, lane + 64, ... in that order (the film's summation order); their
       records are loaded four at a time ahead of the accumulation, so a wave waits on one round
       trip per four samples instead of one per sample */
    for (uint32_t j0 = lane; j0 < w.nSpp; j0 += 4 * 64) {
        float4 lk[4];
        float2 pk[4];
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const uint32_t jj = j0 + 64u * k;
            lk[k] = make_float4(-1.0f, 0.0f, 0.0f, 0.0f); /* past the wave's samples: rejected below */
            pk[k] = make_float2(0.0f, 0.0f);
            if (jj < w.nSpp) {
                lk[k] = P.li[slot * w.nSpp + jj];
                pk[k] = P.pos[slot * w.nSpp + jj];
            }
        }
#pragma unroll
        for (int k = 0; k < 4; ++k) {
            const float4 l = lk[k];
            if (!(isfinite(l.x) && isfinite(l.y) && isfinite(l.z)) || l.x < 0 || l.y < 0 || l.z < 0) continue;
            const float2 ps = pk[k];
            const float rx = ps.x - 0.5f - ox, ry = ps.y - 0.5f - oy;
            const float x0 = ceilf(rx - 1.0f), x1 = floorf(rx + 1.0f), y0 = ceilf(ry - 1.0f), y1 = floorf(ry + 1.0f);
#pragma unroll
            for (int dy = -1; dy <= 1; ++dy) {
                const float yr = (float) (py + dy) - oy;
                if (yr < y0 || yr > y1) continue;
                const float wy = sc.tent[imin((int) fabsf((yr - ry) * sc.tentScale), HPT_FILTER_RES)];
#pragma unroll
                for (int dx = -1; dx <= 1; ++dx) {
                    const float xr = (float) (px + dx) - ox;
                    if (xr < x0 || xr > x1) continue;
                    const float wx = sc.tent[imin((int) fabsf((xr - rx) * sc.tentScale), HPT_FILTER_RES)];
                    const float wgt = wx * wy;
                    float *a = acc[(dy + 1) * 3 + (dx + 1)];
                    a[0] += wgt * l.x;
                    a[1] += wgt * l.y;
                    a[2] += wgt * l.z;
                    a[3] += wgt * 1.0f;
                }
            }
        }
    }
#pragma unroll
    for (int k = 0; k < 9; ++k)
#pragma unroll
        for (int c = 0; c < 4; ++c)
#pragma unroll
            for (int off = 32; off > 0; off >>= 1) acc[k][c] += __shfl_xor(acc[k][c], off);
    if (lane == 0) {
#pragma unroll
        for (int k = 0; k < 9; ++k) partial[(size_t) slot * 9 + k] = make_float4(acc[k][0], acc[k][1], acc[k][2], acc[k][3]);
    }
}

/* k_gather: every pixel adds, in a fixed neighbour order, the partial sums
   its 3x3 neighbours (owned by this shard) addressed to it. */
extern "C" __global__ __launch_bounds__(256) void k_gather(HptScene sc, HptWave w, const float4 *__restrict__ partial,
                                                            float4 *film) {
    if (w.doneIf && !hptWaveDone(w.doneIf, w.doneParity)) return; /* uniform: the host gathers later */
    const uint32_t pix = blockIdx.x * blockDim.x + threadIdx.x;
    if (pix >= (uint32_t) (w.width * w.height)) return;
    const int x = (int) (pix % (uint32_t) w.width), y = (int) (pix / (uint32_t) w.width);
    float4 acc = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
    bool any = false;
    for (int qy = y - 1; qy <= y + 1; ++qy) {
        if (qy < 0 || qy >= w.height) continue;
        for (int qx = x - 1; qx <= x + 1; ++qx) {
            if (qx < 0 || qx >= w.width) continue;
            const int bx = qx / HPT_BLOCK, by = qy / HPT_BLOCK;
            const uint32_t b = (uint32_t) (by * w.nbx + bx);
            const int32_t lb = w.localOf[b];
            if (lb < 0) continue; /* another shard's block */
            const uint32_t slot = ((uint32_t) lb << 10) | ((uint32_t) (qy & 31) << 5) | (uint32_t) (qx & 31);
            const float4 p = partial[(size_t) slot * 9 + (y - qy + 1) * 3 + (x - qx + 1)];
            acc.x += p.x;
            acc.y += p.y;
            acc.z += p.z;
            acc.w += p.w;
            any = true;
        }
    }
    if (any) {
        float4 f = film[pix];
        film[pix] = make_float4(f.x + acc.x, f.y + acc.y, f.z + acc.z, f.w + acc.w);
    }
}

/* ------------------------------------------------------------------ */
/* Batch entry points for unit parity tests                             */
/* ------------------------------------------------------------------ */
extern "C" __global__ void k_sobol_batch(HptScene sc, int m, int n, const uint32_t *frame, const uint32_t *px,
                                         const uint32_t *py, const uint32_t *dim, uint64_t *outIdx, float *outVal) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    uint64_t idx = (m > 1) ? sobolLookUp(sc, (uint32_t) m, frame[i], px[i], py[i]) : (uint64_t) frame[i];
    outIdx[i] = idx;
    outVal[i] = sobolSample(sc, idx, dim[i]);
}

/* camera rays at film positions (pixels): k_camera's own ray construction */
extern "C" __global__ void k_camera_batch(HptScene sc, int n, const float *pos, float *o, float *d, float *mint,
                                          float *maxt) {
    const int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    V3 ro, rd;
    float a, b;
    cameraRay(sc.cam, pos[2 * i], pos[2 * i + 1], ro, rd, a, b);
    o[3 * i] = ro.x, o[3 * i + 1] = ro.y, o[3 * i + 2] = ro.z;
    d[3 * i] = rd.x, d[3 * i + 1] = rd.y, d[3 * i + 2] = rd.z;
    mint[i] = a;
    maxt[i] = b;
}

/* Batch trace through the production traversal (tracePersistent).  flags:
   bit 0 = any-hit shadow query, bit 1 = 2-entry stack (exercises the
   kd-restart path for the parity tests), bit 2 = closest hits through the
   packet traversal (tracePackets, 64 consecutive rays per packet), bit 3 = no
   drain splitting (the parity tests compare both) */
struct BatchIO {
    const float *o, *d, *mint, *maxt;
    float *outT, *outP;
    int32_t *outSeg;
    uint8_t *outHit;
    uint32_t n;
    bool shadow;
    uint32_t cur;
    HD uint32_t count() const { return n; }
    HD uint32_t shardSize(uint32_t s) const { return shardLo(n, s + 1) - shardLo(n, s); }
    HD uint32_t item(uint32_t s, uint32_t j) const { return shardLo(n, s) + j; }
    HD uint32_t key() const { return cur; }
    HD bool begin(const HptScene &sc, uint32_t i, TraceRay &r) {
        cur = i;
        return beginRay(sc, r, v3(o[3 * i], o[3 * i + 1], o[3 * i + 2]), v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]),
                        mint[i], maxt[i], shadow);
    }
    HD uint32_t finish(const HptScene &sc, uint32_t i, const TraceRay &r) {
        if (shadow) {
            outHit[i] = r.found ? 1 : 0;
            return 0;
        }
        outT[i] = r.found ? r.tHit : finf();
        outSeg[i] = r.found ? (int32_t) hitSegment(r) : -1;
        const V3 p = r.found ? segHitPoint(sc, hitSegment(r), r.o, r.d, hitFarRoot(r)) : v3(0.0f, 0.0f, 0.0f);
        outP[3 * i] = p.x;
        outP[3 * i + 1] = p.y;
        outP[3 * i + 2] = p.z;
        return 0;
    }
};

extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) void k_trace_batch(HptScene sc, int n, const float *o,
                                                                            const float *d, const float *mint,
                                                                            const float *maxt, int flags,
                                                                            float *outT, int32_t *outSeg,
                                                                            float *outP, uint8_t *outHit,
                                                                            uint32_t *cursor) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    __shared__ PacketLdsInline lds[HPT_TRACE_BLOCK / 64];
    BatchIO io{o, d, mint, maxt, outT, outP, outSeg, outHit, (uint32_t) n, (flags & 1) != 0, 0u};
    if ((flags & 4) && !(flags & 1))
        tracePackets<false, true>(sc, io, cursor, lds[threadIdx.x >> 6].p, nullptr);
    else if (flags & 2)
        tracePersistent<2, false>(sc, io, cursor, stk + threadIdx.x, nullptr);
    else if (flags & 8)
        tracePersistent<HPT_STACK, false, false>(sc, io, cursor, stk + threadIdx.x, nullptr);
    else
        tracePersistent<HPT_STACK, false>(sc, io, cursor, stk + threadIdx.x, nullptr);
}

extern "C" __global__ void k_bsdf_batch(HptScene sc, int n, const float *wi, const float *wo, const float *u,
                                        float *outEval, float *outPdf, float *outWo, float *outW, float *outSPdf,
                                        uint32_t *outType) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    V3 a = v3(wi[3 * i], wi[3 * i + 1], wi[3 * i + 2]), b = v3(wo[3 * i], wo[3 * i + 1], wo[3 * i + 2]);
    V3 e = bsdfEval(sc.bsdf, a, b);
    outEval[3 * i] = e.x;
    outEval[3 * i + 1] = e.y;
    outEval[3 * i + 2] = e.z;
    outPdf[i] = bsdfPdf(sc.bsdf, a, b);
    V3 so;
    float pdf = 0;
    uint32_t type = 0;
    V3 w = bsdfSample(sc.bsdf, a, u[2 * i], u[2 * i + 1], so, pdf, type);
    outWo[3 * i] = so.x;
    outWo[3 * i + 1] = so.y;
    outWo[3 * i + 2] = so.z;
    outW[3 * i] = w.x;
    outW[3 * i + 1] = w.y;
    outW[3 * i + 2] = w.z;
    outSPdf[i] = pdf;
    outType[i] = type;
}

extern "C" __global__ void k_env_batch(HptScene sc, int n, const float *refp, const float *u, const float *dq,
                                       float *outD, float *outV, float *outPdf, float *outDist, float *outEval,
                                       float *outEvalPdf) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    V3 dl, value;
    float pdf;
    envSampleDir(sc.env, u[2 * i], u[2 * i + 1], dl, value, pdf);
    V3 dW = envToWorld(sc.env, dl);
    V3 ref = v3(refp[3 * i], refp[3 * i + 1], refp[3 * i + 2]);
    float nearT, farT;
    bool ok = !(isZero(value) || pdf == 0 || !bsphereIntersect(sc.env, ref, dW, nearT, farT) || nearT >= 0 || farT <= 0);
    V3 v = ok ? divs(value, pdf) : v3(0, 0, 0);
    outD[3 * i] = dW.x;
    outD[3 * i + 1] = dW.y;
    outD[3 * i + 2] = dW.z;
    outV[3 * i] = v.x;
    outV[3 * i + 1] = v.y;
    outV[3 * i + 2] = v.z;
    outPdf[i] = ok ? pdf : 0.0f;
    outDist[i] = ok ? farT : 0.0f;
    V3 q = v3(dq[3 * i], dq[3 * i + 1], dq[3 * i + 2]);
    V3 e = envEval(sc.env, q);
    outEval[3 * i] = e.x;
    outEval[3 * i + 1] = e.y;
    outEval[3 * i + 2] = e.z;
    outEvalPdf[i] = envPdf(sc.env, envToLocal(sc.env, q));
}

extern "C" __global__ void k_env_filtered_batch(HptScene sc, int n, const float *d, const float *rx, const float *ry,
                                                 float *out) {
    int i = blockIdx.x * blockDim.x + threadIdx.x;
    if (i >= n) return;
    const V3 v = envEvalFiltered(sc.env, v3(d[3 * i], d[3 * i + 1], d[3 * i + 2]),
                                 v3(rx[3 * i], rx[3 * i + 1], rx[3 * i + 2]), v3(ry[3 * i], ry[3 * i + 1], ry[3 * i + 2]));
    out[3 * i] = v.x;
    out[3 * i + 1] = v.y;
    out[3 * i + 2] = v.z;
}


/* ------------------------------------------------------------------ */
/* host-side launch wrappers (declared in hpt_kernels.h)               */
/* ------------------------------------------------------------------ */
static inline unsigned blocksFor(uint64_t n, unsigned bs) { return (unsigned) ((n + bs - 1) / bs); }

hipError_t hpt_launch_camera(const HptScene &sc, const HptWave &w, const HptPaths &P, uint32_t *traceQ,
                             uint32_t *nTrace, hipStream_t s) {
    if (w.nPaths == 0) return hipSuccess;
    hipLaunchKernelGGL(k_camera, dim3(blocksFor(w.nPaths, HPT_QBLOCK)), dim3(HPT_QBLOCK), 0, s, sc, w, P, traceQ, nTrace);
    return hipGetLastError();
}
/* persistent grid: as many one-wave blocks as can be resident at once
   (occupancy API x CUs), capped by the work */
static unsigned persistentBlocks(const void *kernel, uint64_t items, int block = HPT_TRACE_BLOCK) {
    /* resident blocks per kernel, measured once (render calls of several contexts
       may run on several host threads: the cache is guarded) */
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, int> cached; /* (device, kernel): devices may differ */
    int resident = 0, dev = 0;
    (void) hipGetDevice(&dev);
    {
        std::lock_guard<std::mutex> lock(mu);
        auto it = cached.find({dev, kernel});
        if (it == cached.end()) {
            int perCU = 0;
            hipDeviceProp_t prop;
            if (hipGetDeviceProperties(&prop, dev) != hipSuccess ||
                hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kernel, block, 0) != hipSuccess ||
                perCU <= 0)
                perCU = 8, prop.multiProcessorCount = 256;
            it = cached.emplace(std::make_pair(dev, kernel), perCU * prop.multiProcessorCount).first;
        }
        resident = it->second;
    }
    /* HPT_PERSIST_FRAC=k: persistent grids take 1/k of the resident slots (experiments with
       several render calls sharing the device) */
    static const int frac = [] {
        const char *v = std::getenv("HPT_PERSIST_FRAC");
        return v ? std::max(1, std::atoi(v)) : 1;
    }();
    resident = std::max(1, resident / frac);
    const uint64_t need = (items + block - 1) / block;
    return (unsigned) std::max<uint64_t>(1, std::min<uint64_t>(need, (uint64_t) resident));
}

hipError_t hpt_launch_trace(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *shadowQ,
                            const uint32_t *nTrace, const uint32_t *nShadow, uint32_t *cursors, uint32_t *stats,
                            uint64_t maxItems, hipStream_t s, uint32_t *counters, uint32_t nextParity) {
    if (maxItems == 0) return hipSuccess;
    hptProbeBeforeTraceLaunch(s);
    if (stats)
        hipLaunchKernelGGL(k_trace_counted, dim3(persistentBlocks((const void *) k_trace_counted, maxItems)),
                           dim3(HPT_TRACE_BLOCK), 0, s, sc, P, traceQ, shadowQ, nTrace, nShadow, cursors,
                           counters, nextParity, stats);
    else
        hipLaunchKernelGGL(k_trace, dim3(persistentBlocks((const void *) k_trace, maxItems)), dim3(HPT_TRACE_BLOCK), 0, s,
                           sc, P, traceQ, shadowQ, nTrace, nShadow, cursors, counters, nextParity);
    return hipGetLastError();
}
hipError_t hpt_launch_trace_camera(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                                   uint32_t *cursors, uint32_t *stats, uint64_t maxItems, hipStream_t s) {
    if (maxItems == 0) return hipSuccess;
    if (stats)
        hipLaunchKernelGGL(k_trace_camera_counted, dim3(persistentBlocks((const void *) k_trace_camera_counted, maxItems)),
                           dim3(HPT_TRACE_BLOCK), 0, s, sc, P, traceQ, nTrace, cursors, stats);
    else
        hipLaunchKernelGGL(k_trace_camera, dim3(persistentBlocks((const void *) k_trace_camera, maxItems)),
                           dim3(HPT_TRACE_BLOCK), 0, s, sc, P, traceQ, nTrace, cursors);
    return hipGetLastError();
}
hipError_t hpt_launch_trace_packet(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                                   uint32_t *cursors, uint32_t *stats, uint64_t maxItems, uint32_t *overflowQ,
                                   uint32_t *nOverflow, hipStream_t s) {
    if (maxItems == 0) return hipSuccess;
    if (stats)
        hipLaunchKernelGGL(k_trace_packet_counted,
                           dim3(persistentBlocks((const void *) k_trace_packet_counted, maxItems, HPT_PACKET_BLOCK)),
                           dim3(HPT_PACKET_BLOCK), 0, s, sc, P, traceQ, nTrace, cursors, stats, overflowQ, nOverflow);
    else
        hipLaunchKernelGGL(k_trace_packet, dim3(persistentBlocks((const void *) k_trace_packet, maxItems, HPT_PACKET_BLOCK)),
                           dim3(HPT_PACKET_BLOCK), 0, s, sc, P, traceQ, nTrace, cursors, overflowQ, nOverflow);
    return hipGetLastError();
}
hipError_t hpt_launch_trace_overflow(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *overflowQ,
                                     const uint32_t *nOverflow, uint32_t *cursors, uint64_t maxItems, hipStream_t s) {
    if (maxItems == 0) return hipSuccess;
    /* overflowing packets are rare (none at the shipped configs): a small persistent grid that
       claims whatever the packet pass left, instead of a chip-filling launch that finds nothing */
    hipLaunchKernelGGL(k_trace_overflow, dim3(std::min(persistentBlocks((const void *) k_trace_overflow, maxItems), 32u)),
                       dim3(HPT_TRACE_BLOCK), 0, s, sc, P, traceQ, overflowQ, nOverflow, cursors);
    return hipGetLastError();
}
hipError_t hpt_launch_primary(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                              uint32_t *shadeQ, uint32_t *nShade, uint64_t maxItems, hipStream_t s) {
    if (maxItems == 0) return hipSuccess;
    hipLaunchKernelGGL(k_primary, dim3(blocksFor(maxItems, HPT_QBLOCK)), dim3(HPT_QBLOCK), 0, s, sc, P, traceQ, nTrace,
                       shadeQ, nShade);
    return hipGetLastError();
}
hipError_t hpt_launch_shade(const HptScene &sc, const HptPaths &P, const uint32_t *shadeQ, const uint32_t *nShade,
                            uint32_t *traceQ, uint32_t *nTrace, uint32_t *shadowQ, uint32_t *nShadow, uint32_t *counters,
                            uint64_t maxItems, uint32_t tailFrom, hipStream_t s) {
    if (maxItems == 0) return hipSuccess;
    const HptShadeIO q{nShade, nTrace, nShadow, counters, tailFrom};
    if (sc.nShapes > 1)
        hipLaunchKernelGGL(k_shade_multi, dim3(blocksFor(maxItems, HPT_SHADE_BLOCK)), dim3(HPT_SHADE_BLOCK), 0, s, sc, P, shadeQ,
                           traceQ, shadowQ, q);
    else
        hipLaunchKernelGGL(k_shade, dim3(blocksFor(maxItems, HPT_SHADE_BLOCK)), dim3(HPT_SHADE_BLOCK), 0, s, sc, P, shadeQ,
                           traceQ, shadowQ, q);
    return hipGetLastError();
}
hipError_t hpt_launch_post(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                           uint32_t *shadeQ, uint32_t *nShade, uint32_t *counters, uint64_t maxItems, hipStream_t s) {
    if (maxItems == 0) return hipSuccess;
    hipLaunchKernelGGL(k_post, dim3(blocksFor(maxItems, HPT_POST_BLOCK)), dim3(HPT_POST_BLOCK), 0, s, sc, P, traceQ, nTrace,
                       shadeQ, nShade, counters);
    return hipGetLastError();
}
hipError_t hpt_launch_tail(const HptScene &sc, const HptPaths &P, const uint32_t *shadeQ, const uint32_t *nShade,
                           uint32_t *counters, uint64_t items, uint32_t tailFrom, hipStream_t s) {
    if (items == 0) return hipSuccess;
    /* two lanes per path; persistent (pairs claim paths).  Paths are spread over all resident
       waves: K pairs per wave, the fewest that still cover the work in one residency.  With
       items = HPT_ITEMS_ON_DEVICE the host has not read the queue length: the whole resident
       grid is launched and K comes from the length on the device (the same K, the same
       number of waves with work) */
    const void *kern = sc.nShapes > 1 ? (const void *) k_tail_multi : (const void *) k_tail;
    const unsigned residentBlocks = persistentBlocks(kern, ~0ull >> 8);
    const uint64_t residentWaves = (uint64_t) residentBlocks * (HPT_TRACE_BLOCK / 64);
    const uint32_t K = items == HPT_ITEMS_ON_DEVICE
                           ? 0u
                           : (uint32_t) std::min<uint64_t>(32, std::max<uint64_t>(1, (items + residentWaves - 1) / residentWaves));
    const HptTail T{shadeQ, nShade, K, tailFrom};
    const unsigned blocks = K ? persistentBlocks(kern, (items + K - 1) / K * 64) : residentBlocks;
    if (sc.nShapes > 1)
        hipLaunchKernelGGL(k_tail_multi, dim3(blocks), dim3(HPT_TRACE_BLOCK), 0, s, sc, P, T, counters);
    else
        hipLaunchKernelGGL(k_tail, dim3(blocks), dim3(HPT_TRACE_BLOCK), 0, s, sc, P, T, counters);
    return hipGetLastError();
}
extern "C" __global__ __launch_bounds__(256) void k_film_add(float4 *__restrict__ dst, const float4 *__restrict__ src,
                                                             uint64_t n) {
    const uint64_t i = (uint64_t) blockIdx.x * blockDim.x + threadIdx.x;
    if (i < n) {
        const float4 a = dst[i], b = src[i];
        dst[i] = make_float4(a.x + b.x, a.y + b.y, a.z + b.z, a.w + b.w);
    }
}
hipError_t hpt_launch_film_add(float4 *dst, const float4 *src, size_t n, hipStream_t s) {
    if (n == 0) return hipSuccess;
    hipLaunchKernelGGL(k_film_add, dim3(blocksFor(n, 256)), dim3(256), 0, s, dst, src, (uint64_t) n);
    return hipGetLastError();
}
hipError_t hpt_launch_gather(const HptScene &sc, const HptWave &w, const HptPaths &P, float4 *partial, float4 *film,
                             hipStream_t s) {
    const uint64_t slots = w.nPaths / w.nSpp;
    hipLaunchKernelGGL(k_splat, dim3(blocksFor(slots * 64, 256)), dim3(256), 0, s, sc, w, P, partial);
    const uint64_t n = (uint64_t) w.width * (uint64_t) w.height;
    hipLaunchKernelGGL(k_gather, dim3(blocksFor(n, 256)), dim3(256), 0, s, sc, w, (const float4 *) partial, film);
    return hipGetLastError();
}
hipError_t hpt_launch_sobol_batch(const HptScene &sc, int m, int n, const uint32_t *frame, const uint32_t *px,
                                  const uint32_t *py, const uint32_t *dim, uint64_t *oi, float *ov, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_sobol_batch, dim3(blocksFor(n, 256)), dim3(256), 0, s, sc, m, n, frame, px, py, dim, oi, ov);
    return hipGetLastError();
}
hipError_t hpt_launch_camera_batch(const HptScene &sc, int n, const float *pos, float *o, float *d, float *mint,
                                   float *maxt, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_camera_batch, dim3(blocksFor(n, 256)), dim3(256), 0, s, sc, n, pos, o, d, mint, maxt);
    return hipGetLastError();
}
hipError_t hpt_launch_trace_batch(const HptScene &sc, int n, const float *o, const float *d, const float *mint,
                                  const float *maxt, int flags, float *ot, int32_t *os, float *op, uint8_t *oh,
                                  uint32_t *cursor, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipError_t e = hipMemsetAsync(cursor, 0, HPT_CURSORS * HPT_CURSOR_STRIDE * 4, s);
    if (e != hipSuccess) return e;
    hipLaunchKernelGGL(k_trace_batch, dim3(persistentBlocks((const void *) k_trace_batch, (uint64_t) n)),
                       dim3(HPT_TRACE_BLOCK), 0, s, sc, n, o, d, mint, maxt, flags, ot, os, op, oh, cursor);
    return hipGetLastError();
}
hipError_t hpt_launch_env_filtered_batch(const HptScene &sc, int n, const float *d, const float *rx, const float *ry,
                                        float *out, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_env_filtered_batch, dim3(blocksFor(n, 256)), dim3(256), 0, s, sc, n, d, rx, ry, out);
    return hipGetLastError();
}
hipError_t hpt_launch_bsdf_batch(const HptScene &sc, int n, const float *wi, const float *wo, const float *u,
                                 float *oe, float *op, float *owo, float *ow, float *osp, uint32_t *ot, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_bsdf_batch, dim3(blocksFor(n, 256)), dim3(256), 0, s, sc, n, wi, wo, u, oe, op, owo, ow, osp,
                       ot);
    return hipGetLastError();
}
hipError_t hpt_launch_env_batch(const HptScene &sc, int n, const float *refp, const float *u, const float *dq,
                                float *od, float *ov, float *op, float *odist, float *oe, float *oep, hipStream_t s) {
    if (n <= 0) return hipSuccess;
    hipLaunchKernelGGL(k_env_batch, dim3(blocksFor(n, 256)), dim3(256), 0, s, sc, n, refp, u, dq, od, ov, op, odist,
                       oe, oep);
    return hipGetLastError();
}

/* triangle-mesh scenes (C1): k_mesh_paths over this file's sampler, camera, environment and film */
#include "hpt_mesh.h"
