/*
 * hpt_probes.h -- measurement probes of the traversal and tail kernels, for experiment builds only.
 *
 * The shipped library defines none of the switches below and every probe here compiles to
 * nothing; hpt_render.hip calls the probes unconditionally, so the product source carries no
 * instrumentation branches.  Build a probe with `make variant V=<name> KFLAGS=-D<switch>` and
 * select it with HAIRPT_LIB (the tools/ scripts read the records through the hpt_debug_* entry points):
 *
 *   HPT_TRACE_PROFILE  k_trace per-wave timeline: start, the moment its claims found every cursor
 *                      shard empty, end, rays claimed, rays in flight then, drain-loop rounds and
 *                      active lanes over them (tools/trace_profile.py)
 *   HPT_TAIL_PROFILE   k_tail per-wave split of shade / trace / post time (tools/tail_profile.py)
 *   HPT_COST_PROBE     leaf rounds of every path's closest / shadow ray per trace launch
 *                      (tools/cost_probe.py)
 *   HPT_RAY_LOG        every bounce ray of the first trace launches: origin, direction, clipped
 *                      interval, leaf rounds, path (tools/ray_order_probe.py; with -DHPT_DRAIN_SPLIT=0)
 *
 * Times are 100 MHz s_memrealtime ticks.  Included by hpt_render.hip after the traversal
 * (TraceRay, rayLeaves) and before tracePersistent.
 */
#ifndef HPT_PROBES_H
#define HPT_PROBES_H

/* ---------------- k_trace timeline ---------------- */
#ifdef HPT_TRACE_PROFILE
#define HPT_TRACE_PROFILE_LAUNCHES 16
#define HPT_TRACE_PROFILE_WAVES 16384
__device__ unsigned long long g_traceprof[HPT_TRACE_PROFILE_LAUNCHES][HPT_TRACE_PROFILE_WAVES][8];
__device__ uint32_t g_traceprof_slot;
#endif
struct TraceProbe {
#ifdef HPT_TRACE_PROFILE
    unsigned long long begin = __builtin_amdgcn_s_memrealtime(), exhausted = 0, claimed = 0, inFlight = 0;
    unsigned long long drainRounds = 0, drainLanes = 0;
    __device__ void onClaim(uint32_t got) { claimed += got; }
    /* the wave found every shard empty with `idle` of its lanes idle */
    __device__ void onExhausted(uint32_t idle) {
        exhausted = __builtin_amdgcn_s_memrealtime();
        inFlight = 64u - idle;
    }
    __device__ void onDrainStart() {
        if (exhausted == 0) exhausted = __builtin_amdgcn_s_memrealtime();
    }
    __device__ void onDrainRound(uint64_t activeMask) {
        ++drainRounds;
        drainLanes += (unsigned long long) __popcll(activeMask);
    }
    __device__ void finish() {
        const uint32_t wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        const uint32_t slot = g_traceprof_slot;
        if (__lane_id() == 0 && wv < HPT_TRACE_PROFILE_WAVES && slot < HPT_TRACE_PROFILE_LAUNCHES) {
            unsigned long long *rec = g_traceprof[slot][wv];
            rec[0] = begin;
            rec[1] = exhausted;
            rec[2] = __builtin_amdgcn_s_memrealtime();
            rec[3] = claimed;
            rec[4] = inFlight;
            rec[5] = drainRounds;
            rec[6] = drainLanes;
        }
    }
#else
    __device__ void onClaim(uint32_t) {}
    __device__ void onExhausted(uint32_t) {}
    __device__ void onDrainStart() {}
    __device__ void onDrainRound(uint64_t) {}
    __device__ void finish() {}
#endif
};

/* ---------------- k_tail timeline ---------------- */
#ifdef HPT_TAIL_PROFILE
#define HPT_TAIL_PROFILE_WAVES 65536
__device__ unsigned long long g_tailprof[HPT_TAIL_PROFILE_WAVES][8];
#endif
/* per wave [iterations, shade, trace, post ticks, begin, end, sum over iterations of the wave's
   longest ray in leaf rounds, items claimed] */
struct TailProbe {
#ifdef HPT_TAIL_PROFILE
    uint32_t rounds = 0;
    unsigned long long it = 0, tS = 0, tT = 0, tP = 0, sumRounds = 0, items = 0, mark[3] = {0, 0, 0};
    unsigned long long begin = __builtin_amdgcn_s_memrealtime();
    __device__ void onItem(bool counted) { items += counted ? 1u : 0u; }
    __device__ void onRound() { ++rounds; }
    __device__ void onDrainRound(uint64_t) { ++rounds; }
    /* phase 0: the iteration starts (shade), 1: trace starts, 2: post starts, 3: the iteration ends */
    __device__ void phase(int k) {
        const unsigned long long t = __builtin_amdgcn_s_memrealtime();
        if (k == 0) {
            rounds = 0;
            mark[0] = t;
            return;
        }
        if (k < 3) {
            mark[k] = t;
            return;
        }
        uint32_t rm = rounds;
        for (int off = 32; off > 0; off >>= 1) rm = max(rm, (uint32_t) __shfl_xor(rm, off));
        ++it;
        tS += mark[1] - mark[0];
        tT += mark[2] - mark[1];
        tP += t - mark[2];
        sumRounds += rm;
    }
    __device__ void finish() {
        for (int off = 32; off > 0; off >>= 1) items += __shfl_down(items, off);
        const uint32_t wv = (blockIdx.x * blockDim.x + threadIdx.x) >> 6;
        if (__lane_id() == 0 && wv < HPT_TAIL_PROFILE_WAVES) {
            unsigned long long *rec = g_tailprof[wv];
            rec[0] = it;
            rec[1] = tS;
            rec[2] = tT;
            rec[3] = tP;
            rec[4] = begin;
            rec[5] = __builtin_amdgcn_s_memrealtime();
            rec[6] = sumRounds;
            rec[7] = items;
        }
    }
#else
    __device__ void onItem(bool) {}
    __device__ void onRound() {}
    __device__ void onDrainRound(uint64_t) {}
    __device__ void phase(int) {}
    __device__ void finish() {}
#endif
};

/* ---------------- per-ray cost logs (PathIO::finish) ---------------- */
#ifdef HPT_COST_PROBE
#define HPT_COST_LAUNCHES 6
#define HPT_COST_PATHS (1 << 21)
__device__ uint16_t g_costprof[HPT_COST_LAUNCHES][2][HPT_COST_PATHS];
__device__ uint32_t g_cost_slot;
#endif
#ifdef HPT_RAY_LOG
#define HPT_RAYLOG_LAUNCHES 6
struct HptRayLogRec {
    float o[3], d[3], len;
    uint32_t cost, path, pad;
};
__device__ HptRayLogRec *g_raylog[HPT_RAYLOG_LAUNCHES];
__device__ uint32_t g_raylog_cap, g_raylog_slot;
#endif
/* a finished ray: `path` its path id (HPT_MISS when the launch does not know it), k its work index
   in a bounce launch (recs) */
__device__ __forceinline__ void probeRayFinished(const TraceRay &r, uint32_t path, uint32_t k, bool recs) {
#ifdef HPT_COST_PROBE
    {
        const uint32_t slot = g_cost_slot;
        if (path < HPT_COST_PATHS && slot < HPT_COST_LAUNCHES)
            g_costprof[slot][r.shadow ? 1 : 0][path] = (uint16_t) min(rayLeaves(r) + 1u, 65535u);
    }
#endif
#ifdef HPT_RAY_LOG
    {
        const uint32_t slot = g_raylog_slot;
        if (recs && slot < HPT_RAYLOG_LAUNCHES && g_raylog[slot] && k < g_raylog_cap) {
            HptRayLogRec q;
            q.o[0] = r.o.x, q.o[1] = r.o.y, q.o[2] = r.o.z;
            q.d[0] = r.d.x, q.d[1] = r.d.y, q.d[2] = r.d.z;
            q.len = r.maxt - r.mint;
            q.cost = min(rayLeaves(r), 65535u) | (r.found ? 1u << 16 : 0u) | (r.shadow ? 1u << 17 : 0u);
            q.path = path;
            q.pad = 0;
            g_raylog[slot][k] = q;
        }
    }
#endif
}
/* whether probeRayFinished needs the path id (a dependent load the product does not make) */
#if defined(HPT_COST_PROBE) || defined(HPT_RAY_LOG)
#define HPT_PROBE_WANTS_PATH 1
#else
#define HPT_PROBE_WANTS_PATH 0
#endif

/* ---------------- host side ---------------- */
/* before each trace launch: the launch's slot in the per-launch records */
static inline void hptProbeBeforeTraceLaunch(hipStream_t s) {
#ifdef HPT_COST_PROBE
    extern uint32_t g_costHostSlot;
    {
        const uint32_t slot = g_costHostSlot++;
        (void) hipMemcpyToSymbolAsync(HIP_SYMBOL(g_cost_slot), &slot, 4, 0, hipMemcpyHostToDevice, s);
        (void) hipStreamSynchronize(s); /* the slot word is read by the launch that follows */
    }
#endif
#ifdef HPT_RAY_LOG
    extern uint32_t g_raylogHostSlot;
    {
        const uint32_t slot = g_raylogHostSlot++;
        (void) hipMemcpyToSymbolAsync(HIP_SYMBOL(g_raylog_slot), &slot, 4, 0, hipMemcpyHostToDevice, s);
        (void) hipStreamSynchronize(s); /* the slot word is read by the launch that follows */
    }
#endif
#ifdef HPT_TRACE_PROFILE
    extern uint32_t g_traceprofHostSlot;
    {
        const uint32_t slot = g_traceprofHostSlot++;
        (void) hipMemcpyToSymbolAsync(HIP_SYMBOL(g_traceprof_slot), &slot, 4, 0, hipMemcpyHostToDevice, s);
        (void) hipStreamSynchronize(s); /* the slot word is read by the launch that follows */
    }
#endif
    (void) s;
}

#ifdef HPT_COST_PROBE
uint32_t g_costHostSlot = 0;
/* copy out (and clear) the cost records: HPT_COST_LAUNCHES x 2 x HPT_COST_PATHS u16 */
extern "C" int hpt_debug_costprof(uint16_t *out) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    const int n = (int) std::min<uint32_t>(g_costHostSlot, HPT_COST_LAUNCHES);
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_costprof), sizeof(uint16_t) * HPT_COST_LAUNCHES * 2 * HPT_COST_PATHS) != hipSuccess)
        return -1;
    std::vector<uint16_t> zeros((size_t) HPT_COST_LAUNCHES * 2 * HPT_COST_PATHS, 0);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_costprof), zeros.data(), zeros.size() * 2) != hipSuccess) return -1;
    g_costHostSlot = 0;
    return n;
}
#endif
#ifdef HPT_TRACE_PROFILE
uint32_t g_traceprofHostSlot = 0;
/* copy out (and clear) the k_trace timing records of the launches since the last call:
   launches x HPT_TRACE_PROFILE_WAVES x 8 u64; returns the number of launches recorded */
extern "C" int hpt_debug_traceprof(unsigned long long *out, int maxLaunches) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    const int n = (int) std::min<uint32_t>(g_traceprofHostSlot, (uint32_t) std::min(maxLaunches, HPT_TRACE_PROFILE_LAUNCHES));
    if (n > 0 && hipMemcpyFromSymbol(out, HIP_SYMBOL(g_traceprof), (size_t) n * HPT_TRACE_PROFILE_WAVES * 64) != hipSuccess)
        return -1;
    std::vector<unsigned long long> zeros((size_t) HPT_TRACE_PROFILE_LAUNCHES * HPT_TRACE_PROFILE_WAVES * 8, 0ull);
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_traceprof), zeros.data(), zeros.size() * 8) != hipSuccess) return -1;
    g_traceprofHostSlot = 0;
    return n;
}
#endif
#ifdef HPT_RAY_LOG
uint32_t g_raylogHostSlot = 0;
/* point the ray log at n device buffers of cap HptRayLogRec each (n = 0: off) and restart the
   launch count; returns the launches logged since the previous call */
extern "C" int hpt_debug_raylog(void *const *bufs, int n, uint32_t cap) {
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    const int got = (int) std::min<uint32_t>(g_raylogHostSlot, HPT_RAYLOG_LAUNCHES);
    HptRayLogRec *ptrs[HPT_RAYLOG_LAUNCHES] = {};
    for (int i = 0; i < n && i < HPT_RAYLOG_LAUNCHES; ++i) ptrs[i] = (HptRayLogRec *) bufs[i];
    if (hipMemcpyToSymbol(HIP_SYMBOL(g_raylog), ptrs, sizeof(ptrs)) != hipSuccess ||
        hipMemcpyToSymbol(HIP_SYMBOL(g_raylog_cap), &cap, 4) != hipSuccess)
        return -1;
    g_raylogHostSlot = 0;
    return got;
}
#endif
#ifdef HPT_TAIL_PROFILE
/* copy out (and clear) the k_tail timing records of the last frame: n waves x 8 u64 */
extern "C" int hpt_debug_tailprof(unsigned long long *out, int n) {
    if (n > HPT_TAIL_PROFILE_WAVES) n = HPT_TAIL_PROFILE_WAVES;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (hipMemcpyFromSymbol(out, HIP_SYMBOL(g_tailprof), (size_t) n * 64) != hipSuccess) return -1;
    static unsigned long long zeros[HPT_TAIL_PROFILE_WAVES][8];
    return hipMemcpyToSymbol(HIP_SYMBOL(g_tailprof), zeros, sizeof(zeros)) == hipSuccess ? n : -1;
}
#endif

#endif
