/*
 * hpt_kernels.h -- launch-side view of the wavefront kernels (hpt_render.hip).
 */
#ifndef HPT_KERNELS_H
#define HPT_KERNELS_H
#include <hip/hip_runtime.h>
#include <stdint.h>

#include "../hpt_device.h"

/* Counter block (uint32 words).  Bounce b uses the slots of parity
   p = b & 1 (the camera pass is bounce 0); bounce b's trace launch zeroes the other parity's
   slots (clearNextParity). */
#define HPT_C_TRACE(p) (0 + (p))  /* closest-hit rays of bounce b (traceQ[p]) */
#define HPT_C_SHADOW(p) (2 + (p)) /* shadow rays of bounce b (shadowQ[p]) */
#define HPT_C_SHADE(p) (4 + (p))  /* paths bounce b shades (shadeQ[p]: survivors of the previous post) */
#define HPT_C_BOUNCES 6      /* u64 (words 6-7): path-bounces shaded by k_shade */
#define HPT_C_LAUNCHES 8     /* bounces that shaded live paths (k_shade or k_tail launches with work) */
#define HPT_C_TAIL_PATHS 9   /* paths k_tail took over */
#define HPT_C_OVERFLOW 10    /* a k_shade grid (sized from a schedule) was shorter than its queue */
#define HPT_C_ERROR 12       /* set when a path runs out of Sobol dimensions */
#define HPT_C_TAIL_BOUNCES 13 /* path-bounces shaded inside k_tail */
#define HPT_C_TAIL_CURSOR 14  /* k_tail's work claims */
#define HPT_Q_COUNT 24
/* HptScene::fault bits: a traversal bound fired (the ray would otherwise end
   with whatever hit it had; the render / batch call fails instead) */
#define HPT_FAULT_LEAVES 1u   /* more than HptScene::maxLeafRounds (2^18) leaf rounds for one ray */
#define HPT_FAULT_RESTARTS 2u /* more than HptScene::maxRestarts (1024) kd-restarts for one ray */
#define HPT_MAX_LEAF_ROUNDS (1u << 18)
#define HPT_MAX_RESTARTS 1024u
/* k_trace work cursors (persistent waves claim rays from them), one per
   128-byte line, stored after the counters in the same buffer */
#define HPT_CURSORS 64
#define HPT_CURSOR_STRIDE 32
#define HPT_CURSOR_OFFSET 64
static_assert(HPT_Q_COUNT <= HPT_CURSOR_OFFSET, "the counters precede the cursor lines");
/* cursor sets: 0 / 1 the bounce trace launches of parity 0 / 1 (k_trace of parity p zeroes set
   p ^ 1 and the counts of parity p ^ 1 for the next bounce: no clearing launch), 2 the camera
   packets, 3 their overflow launch; all four start at zero with the wave's counter block */
#define HPT_CURSOR_SETS 4
#define HPT_CURSOR_SET(s) (HPT_CURSOR_OFFSET + (s) * HPT_CURSORS * HPT_CURSOR_STRIDE)
#define HPT_COUNTER_WORDS (HPT_CURSOR_OFFSET + HPT_CURSOR_SETS * HPT_CURSORS * HPT_CURSOR_STRIDE)

/* One wave of paths: every pixel of this shard's 32x32 blocks x samples
   [sppBegin, sppBegin + nSpp).  Path id = slot * nSpp + (j - sppBegin),
   slot = (localBlock << 10) | (y%32 << 5) | (x%32). */
struct HptWave {
    uint32_t nPaths;
    uint32_t sppBegin, nSpp;
    int width, height, nbx;
    int shard, nShards;
    const uint32_t *blockOf; /* this shard's k-th 32x32 block -> image block index (by * nbx + bx) */
    const int32_t *localOf;  /* image block index -> k, or -1 when another shard owns it */
    /* k_splat / k_gather launched before the host has read the wave's counters back (bounces
       launched ahead): they run only if the wave is done -- no live path left in shade queue
       doneParity, or k_tail took the rest; no overflow, no error.  nullptr: always */
    const uint32_t *doneIf;
    uint32_t doneParity;
};
__host__ __device__ inline bool hptWaveDone(const uint32_t *c, uint32_t p) {
    return (c[HPT_C_SHADE(p)] == 0u || c[HPT_C_TAIL_PATHS] != 0u) && c[HPT_C_OVERFLOW] == 0u &&
           c[HPT_C_ERROR] == 0u;
}

/* HptPaths::state packing.  dim < 2048 (the Sobol table has 1024 dimensions
   and a path stops before it runs out); depth < 8192, far beyond any path the
   1024 dimensions allow (>= 2 per bounce), so maxDepth = -1 (unlimited) cannot
   overflow it */
#define HPT_ST_DIM_MASK 0x7ffu
#define HPT_ST_DIM(st) ((st) & HPT_ST_DIM_MASK)
#define HPT_ST_DEPTH(st) (((st) >> 11) & 0x1fffu)
__host__ __device__ inline uint32_t hptState(uint32_t st, uint32_t depth, uint32_t dim) {
    return (st & 0xff000000u) | (depth << 11) | dim;
}

/* path state, structure of arrays in HBM (16-byte rows where possible) */
struct HptPaths {
    float4 *ro;        /* ray origin xyz, mint                       */
    float4 *rd;        /* ray direction xyz, maxt (k_camera: direction xyz, 1 / d.z in camera space) */
    float2 *pos;       /* film sample position (pixels)              */
    uint64_t *sobol;   /* Sobol index of the sample (look_up)        */
    uint32_t *state;   /* dim[0:11) | depth[11:24) | sampledType[24:31) | scattered[31] */
    float4 *thr;       /* throughput rgb                             */
    float4 *li;        /* accumulated radiance rgb                   */
    uint32_t *hit;     /* k_tail's hit records by path: segment id | far root << 31, HPT_MISS = miss */
    uint32_t *hitQ;    /* a trace launch's hit records by trace-queue position (k_primary / k_post read them in queue order) */
    uint32_t *hitS;    /* the next shade queue's hit records by shade-queue position (written with the queue) */
    /* Queue-ordered path records: a bounce's kernels read and write a path's state at its
       position in the queue they consume / fill (coalesced), not at its path id (a gather
       over scattered ids), so the state travels with the queues:
       postRec   by trace-queue position, written by k_shade with the queue, read by k_trace and
                 k_post: [4k] origin xyz | Sobol index bits 0-31, [4k+1] direction xyz | bits
                 32-63, [4k+2] bsdf weight rgb, pdf, [4k+3] throughput rgb, state bits
       shadowRec by shadow-queue position (k_shade -> k_trace): [3k] origin xyz, [3k+1]
                 direction xyz, maxt, [3k+2] NEE contribution rgb
       shadeRec  by shade-queue position (k_primary / k_post -> k_shade / k_tail): [3k] traced
                 origin xyz | Sobol bits 0-31, [3k+1] traced direction xyz | bits 32-63,
                 [3k+2] throughput rgb, state bits
       The by-path arrays above (ro, rd, thr, state, bw, sdir, scontrib) are k_camera's and
       k_tail's. */
    float4 *postRec, *shadowRec, *shadeRec;
    /* per owned 32x32 block: path-bounces shaded (k_shade, k_tail), the measured work the cost-
       balanced shard deal reads back (hpt_get_block_costs); nullptr: not counted.  costSpp is
       the wave's nSpp (path id -> block: id / nSpp >> 10).  The counts are striped: wave w adds
   to stripe w % HPT_COST_STRIPES at blockCost[stripe * costStride + block] (a bounce's queue
   is in block order, so every resident wave counts into the same block at once: one counter
   per block serialised ~70 k atomics per launch and cost k_shade 4 ms per frame) */
    uint32_t *blockCost;
    uint32_t costSpp, costStride;
    float4 *bw;        /* bsdf weight rgb, bsdf pdf                  */
    float4 *sdir;      /* shadow ray direction xyz, maxt             */
    float4 *scontrib;  /* NEE contribution rgb (added if unoccluded) */
};


#define HPT_COST_STRIPES 64
/* hit record of a miss (a segment id never has all 31 bits set) */
#define HPT_MISS 0xffffffffu

/* launch wrappers (hpt_render.hip).  Queue lengths are passed as device
   pointers (the kernels read them; the host only bounds the grids). */
hipError_t hpt_launch_camera(const HptScene &sc, const HptWave &w, const HptPaths &P, uint32_t *traceQ,
                             uint32_t *nTrace, hipStream_t s);
/* one persistent traversal launch: closest-hit rays traceQ[0, *nTrace), shadow rays shadowQ[0, *nShadow) */
/* counters (nullptr: none): a bounce launch of parity p = nextParity ^ 1 also zeroes the counts and
   cursor set of parity nextParity, which the next bounce appends to / claims from */
hipError_t hpt_launch_trace(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *shadowQ,
                            const uint32_t *nTrace, const uint32_t *nShadow, uint32_t *cursors, uint32_t *stats,
                            uint64_t maxItems, hipStream_t s, uint32_t *counters = nullptr, uint32_t nextParity = 0);
/* the camera pass's rays one per lane (HPT_PACKETS=0): traceQ[0, *nTrace), hits to P.hitQ by position */
hipError_t hpt_launch_trace_camera(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                                   uint32_t *cursors, uint32_t *stats, uint64_t maxItems, hipStream_t s);
hipError_t hpt_launch_env_filtered_batch(const HptScene &sc, int n, const float *d, const float *rx, const float *ry,
                                        float *out, hipStream_t s);
/* closest-hit rays as 64-ray packets (coherent rays: the camera pass); the rays of a packet whose
   stack overflows are appended to overflowQ / *nOverflow for hpt_launch_trace_overflow */
hipError_t hpt_launch_trace_packet(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                                   uint32_t *cursors, uint32_t *stats, uint64_t maxItems, uint32_t *overflowQ,
                                   uint32_t *nOverflow, hipStream_t s);
/* those rays, one lane each (persistent; maxItems only sizes the grid) */
hipError_t hpt_launch_trace_overflow(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *overflowQ,
                                     const uint32_t *nOverflow, uint32_t *cursors, uint64_t maxItems, hipStream_t s);
hipError_t hpt_launch_primary(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                              uint32_t *shadeQ, uint32_t *nShade, uint64_t maxItems, hipStream_t s);
/* tailFrom: the launch leaves a queue shorter than this to the tail launch of the same
   bounce (0: always shade); a queue longer than the grid (maxItems) sets HPT_C_OVERFLOW */
hipError_t hpt_launch_shade(const HptScene &sc, const HptPaths &P, const uint32_t *shadeQ, const uint32_t *nShade,
                            uint32_t *traceQ, uint32_t *nTrace, uint32_t *shadowQ, uint32_t *nShadow, uint32_t *counters,
                            uint64_t maxItems, uint32_t tailFrom, hipStream_t s);
hipError_t hpt_launch_post(const HptScene &sc, const HptPaths &P, const uint32_t *traceQ, const uint32_t *nTrace,
                           uint32_t *shadeQ, uint32_t *nShade, uint32_t *counters, uint64_t maxItems, hipStream_t s);
/* the rest of every live path (the shade queue) to termination in one launch, when the queue
   is shorter than tailFrom (~0u: always); items = HPT_ITEMS_ON_DEVICE when the host has not
   read the queue length (the launch then sizes its work from it on the device) */
#define HPT_ITEMS_ON_DEVICE (~0ull)
hipError_t hpt_launch_tail(const HptScene &sc, const HptPaths &P, const uint32_t *shadeQ, const uint32_t *nShade,
                           uint32_t *counters, uint64_t items, uint32_t tailFrom, hipStream_t s);
/* dst[i] += src[i] over n RGBW pixels (hpt_render_multi's film combine) */
hipError_t hpt_launch_film_add(float4 *dst, const float4 *src, size_t n, hipStream_t s);
/* k_splat + k_gather; partial = (nPaths / nSpp) * 9 float4 of scratch */
hipError_t hpt_launch_gather(const HptScene &sc, const HptWave &w, const HptPaths &P, float4 *partial, float4 *film,
                             hipStream_t s);
/* triangle-mesh scenes (C1, hpt_mesh.h): every camera sample of the wave to termination, one lane
   each; P.pos / P.li for hpt_launch_gather, path-bounces and the Sobol error to counters */
hipError_t hpt_launch_mesh_paths(const HptScene &sc, const HptMeshScene &ms, const HptWave &w, const HptPaths &P,
                                 uint32_t *counters, hipStream_t s);
hipError_t hpt_launch_sobol_batch(const HptScene &sc, int m, int n, const uint32_t *frame, const uint32_t *px,
                                  const uint32_t *py, const uint32_t *dim, uint64_t *oi, float *ov, hipStream_t s);
hipError_t hpt_launch_camera_batch(const HptScene &sc, int n, const float *pos, float *o, float *d, float *mint,
                                   float *maxt, hipStream_t s);
hipError_t hpt_launch_trace_batch(const HptScene &sc, int n, const float *o, const float *d, const float *mint,
                                  const float *maxt, int flags, float *ot, int32_t *os, float *op, uint8_t *oh,
                                  uint32_t *cursor, hipStream_t s);
hipError_t hpt_launch_bsdf_batch(const HptScene &sc, int n, const float *wi, const float *wo, const float *u,
                                 float *oe, float *op, float *owo, float *ow, float *osp, uint32_t *ot, hipStream_t s);
hipError_t hpt_launch_env_batch(const HptScene &sc, int n, const float *refp, const float *u, const float *dq,
                                float *od, float *ov, float *op, float *odist, float *oe, float *oep, hipStream_t s);
#endif
