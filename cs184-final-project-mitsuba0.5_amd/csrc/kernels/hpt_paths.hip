/*
 * hpt_paths.hip -- k_paths, every bounce of a wave of paths in one persistent launch (gfx950).
 *
 * Its own translation unit: it reuses hpt_render.hip's device functions (the traversal, shadePath,
 * postPath) and is compiled with MachineLICM off (Makefile).  Inside k_paths' outer loop that pass
 * hoisted the shading code's constants (fp64 log / exp polynomial coefficients, scene scalars) out
 * of the loop into registers, and 72 VGPRs at 7 waves per SIMD then spilled ~50 of them to scratch;
 * without it the kernel keeps 72 VGPRs with a few spills.  The wavefront kernels keep the pass.
 */
#define HPT_DEVICE_LIB_ONLY 1
#include "hpt_render.hip"

#include <map>
#include <mutex>

namespace {
/* ------------------------------------------------------------------ */
/* k_paths: every bounce of a wave of paths in one persistent launch    */
/* ------------------------------------------------------------------ */
/* The wavefront bounce loop (k_shade -> k_trace -> k_post per bounce, then k_tail) ends each
   trace launch with a grid-wide drain: the launch waits for its slowest rays while most of the
   machine idles (~0.5 ms per launch), five times per frame.  The reference has no
   such barrier: each path runs to termination (path.cpp:135-287) under an on-demand block
   scheduler (renderproc.cpp:68-85).  k_paths restores that: its persistent waves take whatever
   work is ready -- rays to trace, or paths to post and shade -- so bounce b + 1 of one path runs
   while bounce b of another is still being traced, and the frame drains once.

   Work moves between waves through three queues (HptMega, hpt_kernels.h), all hand-offs between
   CUs in one launch (handoffStore / handoffLoad, published after handoffDrain):
     ray chunks  a shade step (one wave, 64 paths) writes 64 path-bounce slots -- the continuation
                 ray, the shadow ray, what post needs -- and publishes the chunk; tracing waves
                 claim chunks and refill idle lanes from them (HPT_REFILL, as k_trace does)
     slot state  the two rays of a slot finish on any lanes of any waves: each adds its result to
                 the slot's 64-bit state word (atomic); the one that finds itself last appends
                 the slot to its wave's post chunk (the hit word and the shadow result travel
                 in the item)
     post chunks a wave publishes its post chunk at 64 items, and a part-filled one when it runs
                 out of rays; a shade step posts those paths (NEE contribution first, then the
                 emitter term and roulette: path.cpp order, as k_trace -> k_post) and shades the
                 survivors into a new ray chunk
   Per path the arithmetic is the wavefront kernels' own functions (shadePath, postPath, the
   traversal) in the same order, and a path's radiance travels in its slot (field 4) instead of
   P.li, so the film is bit-identical to the wavefront loop's.

   Roles: a wave traces while rays are published; it leaves tracing (draining its lanes, idle
   lanes helping: RaySplitter) when none are left, or by choice when the ray backlog falls below
   HptMega::low and at most maxShaders waves have made that choice; it then shades post chunks
   (deepest paths first) or k_primary's queue until the backlog reaches high or no shading work
   is left.  Every wave leaves when every path of the wave has finished (HPT_MC_DONE), or on an
   abort (a capacity ran out: the host renders the wave again bounce by bounce), or when it has
   found no work for HPT_PATHS_IDLE_TICKS (HPT_FAULT_PATHS: the call fails, the grid drains). */
#ifndef HPT_PATHS_IDLE_TICKS
#define HPT_PATHS_IDLE_TICKS 2000000000ull /* 20 s of 100 MHz s_memrealtime ticks without work */
#endif
#define HPT_NO_TICKET 0xffffffffu

/* the wave's control-word atomics, issued by lane 0 and broadcast (called with the whole wave) */
HD uint32_t ctlLoad(const HptMega &M, int w) {
    return __hip_atomic_load(M.ctl + w * HPT_MC_STRIDE, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
}
HD uint32_t waveCtlAdd(const HptMega &M, int w, uint32_t v) {
    uint32_t r = 0;
    if (__lane_id() == 0) r = __hip_atomic_fetch_add(M.ctl + w * HPT_MC_STRIDE, v, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    return (uint32_t) __builtin_amdgcn_readfirstlane((int) r);
}
HD uint32_t waveCtlLoad(const HptMega &M, int w) {
    uint32_t r = 0;
    if (__lane_id() == 0) r = ctlLoad(M, w);
    return (uint32_t) __builtin_amdgcn_readfirstlane((int) r);
}
HD uint64_t waveHandoffLoad(const uint64_t *p) {
    uint64_t r = 0;
    if (__lane_id() == 0) r = handoffLoad(p);
    return ((uint64_t) (uint32_t) __builtin_amdgcn_readfirstlane((int) (r >> 32)) << 32) |
           (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) r);
}
HD float4 *slotFields(const HptMega &M, uint32_t slot) {
    return M.rec + (size_t) (slot >> 6) * (64 * HPT_MEGA_FIELDS) + (slot & 63u);
}
/* stop every wave: a capacity ran out (the host renders the wave again) */
HD void pathsAbort(const HptMega &M, uint32_t *counters) {
    if (__lane_id() == 0) {
        __hip_atomic_store(M.ctl + HPT_MC_ABORT * HPT_MC_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        atomicOr(&counters[HPT_C_OVERFLOW], 1u);
    }
}

/* A wave traces every ray of the ray chunks it claims, up to HPT_PATHS_ENTRIES chunks in flight (it
   refills lanes from the newest while the older ones' long rays finish), so a slot's two rays finish
   on lanes of one wave and its completion is known in LDS: no global atomic per ray (one with a
   return value, per ray, stalled every traversal round that finished a ray on a device round trip:
   3x the wave cycles).  The wave's state, in LDS (lane 0 writes, every lane reads the same word):
   kept out of SGPRs, which the traversal's loop needs */
#ifndef HPT_PATHS_ENTRIES
#define HPT_PATHS_ENTRIES 3
#endif
struct PathsWave {
    uint32_t rayTicket, postTicket;
    uint32_t cur, taken;          /* the entry the wave refills from (HPT_NO_TICKET: none), rays handed out */
    uint32_t postCur, postNext;   /* post chunks being filled */
    uint32_t fill;                /* items in them (postCur first, then postNext) */
    uint32_t shader;              /* counted in HPT_MC_SHADERS */
    uint32_t claims;              /* statistics: ray chunks claimed */
    uint32_t drains;              /* statistics: trace phases that ended in a drain */
    uint64_t rounds, lanes;       /* statistics: main-loop traversal rounds, active lanes over them */
    /* entries: a claimed chunk, its rays (closest-ray lanes, shadow-ray lanes), the slots one of
       whose two rays has finished, the unoccluded shadow rays, rays still running (0: free) */
    uint32_t chunk[HPT_PATHS_ENTRIES], total[HPT_PATHS_ENTRIES], left[HPT_PATHS_ENTRIES];
    uint64_t contM[HPT_PATHS_ENTRIES], shadowM[HPT_PATHS_ENTRIES], doneM[HPT_PATHS_ENTRIES],
        unoccM[HPT_PATHS_ENTRIES];
};
HD uint32_t uni(uint32_t v) { return (uint32_t) __builtin_amdgcn_readfirstlane((int) v); }
HD uint64_t uni64(uint64_t v) { return ((uint64_t) uni((uint32_t) (v >> 32)) << 32) | uni((uint32_t) v); }
/* lane 0 writes a field of the wave's state (the wave then reads it back) */
#define PW_SET(w, field, v)                  \
    do {                                     \
        const auto _v = (v);                 \
        if (__lane_id() == 0) (w)->field = _v; \
        __builtin_amdgcn_wave_barrier();     \
    } while (0)
#define PW_GET(w, field) uni((w)->field)

/* the trace side's IO (tracePersistent's interface, for traceRound / RaySplitter): a ray's key is
   entry << 7 | slot lane << 1 | shadow */
struct PathsIO {
    const HptMega *M;
    PathsWave *w;
    uint32_t id;
    HD uint32_t key() const { return id; }
    HD bool begin(const HptScene &sc, uint32_t key, TraceRay &r) {
        id = key;
        const uint32_t slot = w->chunk[key >> 7] * 64u + ((key >> 1) & 63u);
        const float4 *f = slotFields(*M, slot);
        const float4 o = handoffLoadF4(f);
        /* a bounce ray leaves the hit point at kEpsilon (path.cpp:213, scene.cpp:838) */
        if (!(key & 1u)) {
            const float4 d = handoffLoadF4(f + 64);
            return beginRay(sc, r, v3(o.x, o.y, o.z), v3(d.x, d.y, d.z), kEpsilon, finf(), false);
        }
        const float4 d = handoffLoadF4(f + 64 * 5);
        return beginRay(sc, r, v3(o.x, o.y, o.z), v3(d.x, d.y, d.z), kEpsilon, d.w, true);
    }
    /* a closest ray's hit word goes to its slot (the post step reads it there); a slot whose last
       ray this is joins the wave's post chunk.  Returns 1 for an unoccluded shadow ray */
    HD uint32_t finish(const HptScene &, uint32_t key, const TraceRay &r) {
        const uint32_t e = key >> 7, l = (key >> 1) & 63u;
        const uint64_t bit = 1ull << l;
        const uint32_t slot = w->chunk[e] * 64u + l;
        const bool shadowRay = (key & 1u) != 0;
        if (!shadowRay) handoffStore(M->slotSt + slot, (uint64_t) (r.found ? r.segHit : HPT_MISS));
        else if (!r.found) atomicOr((unsigned long long *) &w->unoccM[e], (unsigned long long) bit);
        const bool both = ((w->contM[e] & w->shadowM[e]) & bit) != 0;
        const uint64_t old = both ? atomicOr((unsigned long long *) &w->doneM[e], (unsigned long long) bit) : 0ull;
        if (!both || (old & bit)) { /* the slot's last ray */
            const uint32_t item = slot | ((w->unoccM[e] & bit) ? 0x80000000u : 0u);
            const uint32_t pos = atomicAdd(&w->fill, 1u); /* LDS; < 128: the wave publishes at 64 after every round */
            const uint32_t pc = pos < 64u ? w->postCur : w->postNext;
            if (pc < M->postCap) handoffStore(M->postItems + (size_t) pc * 64 + (pos & 63u), (uint64_t) item);
        }
        atomicSub(&w->left[e], 1u);
        return shadowRay && !r.found ? 1u : 0u;
    }
};

/* a new post chunk for the wave (lane 0 allocates); a full allocator aborts the wave render */
HD uint32_t reservePost(const HptMega &M, uint32_t *counters) {
    const uint32_t pc = waveCtlAdd(M, HPT_MC_POSTS, 1u);
    if (pc >= M.postCap) pathsAbort(M, counters);
    return pc;
}
/* publish the wave's post chunk when it holds 64 items (flush: whatever it holds); wave-uniform */
HD void postPublish(const HptMega &M, PathsWave *w, uint32_t *counters, bool flush) {
    uint32_t fill = PW_GET(w, fill);
    while (fill >= 64u || (flush && fill > 0u)) {
        const uint32_t n = min(fill, 64u), cur = PW_GET(w, postCur);
        handoffDrain(); /* every item (and hit word) this wave stored has been written through */
        if (cur < M.postCap) {
            const uint32_t pq = waveCtlAdd(M, HPT_MC_POST_TAIL, 1u);
            if (__lane_id() == 0) handoffStore(M.postQ + pq, (uint64_t) (cur + 1u) | ((uint64_t) n << 32));
        }
        PW_SET(w, postCur, PW_GET(w, postNext));
        PW_SET(w, postNext, reservePost(M, counters));
        fill -= n;
        PW_SET(w, fill, fill);
    }
}

HD uint32_t rayBacklog(const HptMega &M) {
    const uint32_t tail = waveCtlLoad(M, HPT_MC_RAY_TAIL), head = waveCtlLoad(M, HPT_MC_RAY_HEAD);
    return tail > head ? tail - head : 0u;
}
HD bool shadeWorkReady(const HptMega &M, uint32_t nInit) {
    return waveCtlLoad(M, HPT_MC_POST_TAIL) > waveCtlLoad(M, HPT_MC_POST_HEAD) || waveCtlLoad(M, HPT_MC_INIT) < nInit;
}
/* a free entry of the wave (HPT_NO_TICKET: none): no ray running and not the one being refilled from */
HD uint32_t freeEntry(PathsWave *w) {
    const uint32_t cur = PW_GET(w, cur);
#pragma unroll
    for (uint32_t e = 0; e < HPT_PATHS_ENTRIES; ++e)
        if (e != cur && PW_GET(w, left[e]) == 0u) return e;
    return HPT_NO_TICKET;
}
/* claim the next published ray chunk into entry e, once its ticket's chunk is published; false:
   none ready */
HD bool claimRayChunk(const HptMega &M, PathsWave *w, uint32_t e) {
    uint32_t t = PW_GET(w, rayTicket);
    if (t == HPT_NO_TICKET) {
        if (waveCtlLoad(M, HPT_MC_RAY_TAIL) <= waveCtlLoad(M, HPT_MC_RAY_HEAD)) return false;
        t = waveCtlAdd(M, HPT_MC_RAY_HEAD, 1u);
        PW_SET(w, rayTicket, t);
    }
    if (t >= M.chunkCap) return false; /* never published (the allocator would abort first) */
    const uint64_t g = waveHandoffLoad(M.rayQ + t);
    if (g == 0) return false;
    const uint32_t c = (uint32_t) g - 1u;
    if (c >= M.chunkCap) return false; /* (never: rayQ holds chunks this launch allocated) */
    const uint64_t cm = waveHandoffLoad(M.desc + 2 * (size_t) c), sm = waveHandoffLoad(M.desc + 2 * (size_t) c + 1);
    const uint32_t n = (uint32_t) (__popcll(cm) + __popcll(sm));
    PW_SET(w, rayTicket, HPT_NO_TICKET);
    PW_SET(w, chunk[e], c);
    PW_SET(w, contM[e], cm);
    PW_SET(w, shadowM[e], sm);
    PW_SET(w, doneM[e], 0ull);
    PW_SET(w, unoccM[e], 0ull);
    PW_SET(w, total[e], n);
    PW_SET(w, left[e], n);
    PW_SET(w, cur, e);
    PW_SET(w, taken, 0u);
    PW_SET(w, claims, PW_GET(w, claims) + 1u);
    return true;
}

/* Trace phase: refill idle lanes from the wave's ray chunks until none is ready (or the wave chooses
   to shade), then drain the lanes (idle lanes help: RaySplitter).  Returns once every lane is idle;
   every claimed chunk's rays have then finished. */
__device__ __forceinline__ void pathsTrace(const HptScene &sc, const HptMega &M, PathsWave *w, uint2 *stk,
                                           uint32_t *counters, uint32_t nInit) {
    const int stride = HPT_TRACE_BLOCK;
    PathsIO io{&M, w, 0};
    TraceRay r;
    TraceCounters tc;
    TraceProbe probe;
    bool active = false, stop = false;
    while (true) {
        const uint64_t idle = __ballot(!active);
        if (!stop && __popcll(idle) >= HPT_REFILL) {
            uint32_t cur = PW_GET(w, cur);
            const uint32_t e = (cur == HPT_NO_TICKET || PW_GET(w, taken) >= PW_GET(w, total[cur])) ? freeEntry(w)
                                                                                                   : HPT_NO_TICKET;
            if (e == HPT_NO_TICKET) {
                /* the chunk still has rays, or every entry has rays running: no global word is read */
                if (cur != HPT_NO_TICKET && PW_GET(w, taken) >= PW_GET(w, total[cur])) cur = HPT_NO_TICKET;
            } else {
                /* the current chunk is used up: the global words are read here only (once per chunk;
                   every wave reading them at every refill made them the launch's hottest lines) */
                if (waveCtlLoad(M, HPT_MC_ABORT) != 0u) stop = true;
                else if (PW_GET(w, shader) == 0u && rayBacklog(M) < M.low && shadeWorkReady(M, nInit)) {
                    /* the backlog runs low: leave tracing to shade, unless enough waves already do */
                    const uint32_t k = waveCtlAdd(M, HPT_MC_SHADERS, 1u);
                    if (k < M.maxShaders) {
                        PW_SET(w, shader, 1u);
                        stop = true;
                        waveCtlAdd(M, HPT_MC_SWITCHES, 1u);
                    } else {
                        waveCtlAdd(M, HPT_MC_SHADERS, ~0u);
                    }
                }
                if (!stop) {
                    if (claimRayChunk(M, w, e)) cur = e;
                    else stop = true; /* none ready: drain */
                }
            }
            if (!stop && cur != HPT_NO_TICKET) {
                const uint32_t taken = PW_GET(w, taken), total = PW_GET(w, total[cur]);
                const uint32_t got = min((uint32_t) __popcll(idle), total - taken);
                if (!active) {
                    const uint32_t rank =
                        __builtin_amdgcn_mbcnt_hi((uint32_t) (idle >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t) idle, 0u));
                    if (rank < got) {
                        const uint64_t cm = w->contM[cur], sm = w->shadowM[cur];
                        const uint32_t j = taken + rank, nC = (uint32_t) __popcll(cm);
                        const uint32_t sl = j < nC ? selectBit(cm, j) : selectBit(sm, j - nC);
                        const uint32_t key = (cur << 7) | (sl << 1) | (j < nC ? 0u : 1u);
                        active = io.begin(sc, key, r);
                        stashRay<HPT_STACK>(stk, stride, r, io.key());
                        if (!active) io.finish(sc, io.key(), r);
                    }
                }
                PW_SET(w, taken, taken + got);
                /* rays that missed the scene finished at once: their items count before the round's */
                postPublish(M, w, counters, false);
            }
        }
        if (__ballot(active) == 0) {
            if (stop) break;
            postPublish(M, w, counters, false);
            continue;
        }
        if (stop) {
            /* nothing more to claim (or the wave goes to shade): finish the running rays, idle lanes
               helping, publishing post items as they come */
            PW_SET(w, drains, PW_GET(w, drains) + 1u);
            RaySplitter<HPT_STACK> split{stk, stride};
            split.template drain<false>(sc, io, r, active, tc, probe, [&]() { postPublish(M, w, counters, false); });
            break;
        }
        {
            const uint64_t act = __ballot(active);
            if (__lane_id() == 0) {
                w->rounds += 1;
                w->lanes += (uint64_t) __popcll(act);
            }
        }
        if (active && traceRound<HPT_STACK, false>(sc, r, stk, stride, tc)) {
            io.finish(sc, rayKey<HPT_STACK>(stk, stride), r);
            active = false;
        }
        postPublish(M, w, counters, false);
    }
    /* every claimed chunk's rays have finished: no entry is being refilled from */
    PW_SET(w, cur, HPT_NO_TICKET);
}

/* k_shade keeps a path's radiance and id in the rows MODE 2 leaves free (the shadow record's) */
enum : int { kRowLi = kRowSd, kRowPath = kRowSd + 3 };

/* One shade step: up to 64 paths -- a post chunk's (posted first: NEE contribution, emitter term,
   roulette) or k_primary's -- shaded into a new ray chunk, which is published.  Returns false when
   no shading work was ready. */
template <bool MULTI>
__device__ __forceinline__ bool pathsShadeStep(const HptScene &sc, const HptPathsArgs &a, PathsWave *w, float *wiL,
                                               uint32_t nInit) {
    const HptMega &M = a.M;
    HptPaths P = a.P;
    const uint32_t *__restrict__ shadeQ0 = a.shadeQ0;
    uint32_t *const counters = a.counters;
    const uint32_t lane = __lane_id();
    /* the work: a published post chunk (its paths are the deeper ones), else k_primary's queue */
    uint32_t n = 0, pc = HPT_NO_TICKET, base = 0;
    uint32_t t = PW_GET(w, postTicket);
    if (t == HPT_NO_TICKET && waveCtlLoad(M, HPT_MC_POST_TAIL) > waveCtlLoad(M, HPT_MC_POST_HEAD)) {
        t = waveCtlAdd(M, HPT_MC_POST_HEAD, 1u);
        PW_SET(w, postTicket, t);
    }
    if (t != HPT_NO_TICKET && t < M.postCap) {
        /* published a moment ago, or about to be: its tail was counted before the entry was stored */
        for (int spin = 0; spin < 64; ++spin) {
            const uint64_t g = waveHandoffLoad(M.postQ + t);
            if (g != 0) {
                pc = (uint32_t) g - 1u;
                n = min((uint32_t) (g >> 32), 64u);
                if (pc >= M.postCap) n = 0, pc = 0; /* (never: postQ holds post chunks this launch allocated) */
                PW_SET(w, postTicket, HPT_NO_TICKET);
                break;
            }
            __builtin_amdgcn_s_sleep(2);
        }
    }
    if (pc == HPT_NO_TICKET) {
        if (waveCtlLoad(M, HPT_MC_INIT) >= nInit) return false;
        base = waveCtlAdd(M, HPT_MC_INIT, 64u);
        if (base >= nInit) return false;
        n = min(64u, nInit - base);
    }
    const uint32_t c = waveCtlAdd(M, HPT_MC_CHUNKS, 1u);
    if (c >= M.chunkCap) {
        pathsAbort(M, counters);
        return false;
    }
    const bool valid = lane < n;
    bool alive = false;
    uint32_t path = 0, hitRec = HPT_MISS;
    float4 in[3];
    {
        float4 li = make_float4(0.0f, 0.0f, 0.0f, 0.0f);
#ifndef XNO_POST
        if (valid && pc != HPT_NO_TICKET) {
#else
        if (false) {
#endif
            /* a posted slot: its rays have finished (the item carries the hit word and the shadow result) */
            const uint64_t item = handoffLoad(M.postItems + (size_t) pc * 64 + lane);
            uint32_t slot = (uint32_t) item & 0x7fffffffu;
            if (slot >= M.chunkCap * 64u) { /* a malformed item: fail the call loudly, never read past the chunks */
                atomicOr(sc.fault, HPT_FAULT_PATHS);
                slot = 0;
            }
            const float4 *f = slotFields(M, slot);
            const float4 f4 = handoffLoadF4(f + 64 * 4);
            li = make_float4(f4.x, f4.y, f4.z, 0.0f);
            const uint32_t pf = __float_as_uint(f4.w);
            path = pf & HPT_MEGA_PATH_MASK;
            if ((uint32_t) item & 0x80000000u) { /* the unoccluded shadow ray's NEE term first (k_trace's finish) */
                const float4 cn = handoffLoadF4(f + 64 * 6);
                li = make_float4(li.x + cn.x, li.y + cn.y, li.z + cn.z, li.w);
            }
            if (pf & 0x80000000u) {
                hitRec = (uint32_t) handoffLoad(M.slotSt + slot); /* the closest ray's hit word */
                float4 rec[4];
                rec[0] = handoffLoadF4(f);
                rec[1] = handoffLoadF4(f + 64);
                rec[2] = handoffLoadF4(f + 64 * 2);
                rec[3] = handoffLoadF4(f + 64 * 3);
                alive = postPath<true>(sc, P, path, hitRec != HPT_MISS, counters, rec, in, &li);
            }
        } else if (valid) {
            const uint32_t j = base + lane;
            path = shadeQ0[j];
#pragma unroll
            for (int i = 0; i < 3; ++i) in[i] = P.shadeRec[3 * j + i];
            hitRec = P.hitS[j];
            li = P.li[path];
            alive = true;
        }
        /* the radiance and the path id wait in LDS while the path is shaded */
        stashV3(wiL, HPT_SHADE_BLOCK, kRowLi, v3(li.x, li.y, li.z));
        wiL[kRowPath * HPT_SHADE_BLOCK] = __uint_as_float(path);
        asm volatile("" ::: "memory");
    }
    countBlockCost(P, alive, path);
    bool cont = false, shadow = false;
    float4 cOut[4];
    if (alive)
        shadePath<MULTI, 2>(sc, P, path, hitRec, counters, cont, shadow, in, cOut, nullptr, wiL,
                            M.rec + (size_t) c * (64 * HPT_MEGA_FIELDS));
    const bool finished = valid && !cont && !shadow;
    float4 *const out = M.rec + (size_t) c * (64 * HPT_MEGA_FIELDS) + lane;
    {
        const V3 li = loadV3(wiL, HPT_SHADE_BLOCK, kRowLi);
        path = __float_as_uint(wiL[kRowPath * HPT_SHADE_BLOCK]);
        if (finished) P.li[path] = make_float4(li.x, li.y, li.z, 0.0f); /* final (k_splat reads it after the launch) */
        if (cont || shadow) {
            if (cont) {
                handoffStore(out, cOut[0]);
                handoffStore(out + 64, cOut[1]);
                handoffStore(out + 64 * 2, cOut[2]);
                handoffStore(out + 64 * 3, cOut[3]);
            } else { /* the shadow ray's origin: the shading point */
                const V3 p = loadV3(wiL, HPT_SHADE_BLOCK, kRowP);
                handoffStore(out, make_float4(p.x, p.y, p.z, 0.0f));
            }
            handoffStore(out + 64 * 4, make_float4(li.x, li.y, li.z,
                                                   __uint_as_float(path | (shadow ? 0x40000000u : 0u) | (cont ? 0x80000000u : 0u))));
        }
    }
    const uint64_t contM = __ballot(cont), shadowM = __ballot(shadow);
    if (lane == 0) {
        handoffStore(M.desc + 2 * (size_t) c, contM);
        handoffStore(M.desc + 2 * (size_t) c + 1, shadowM);
    }
    handoffDrain(); /* the slots, states and lane masks are written through before the chunk is published */
    if ((contM | shadowM) != 0) {
        const uint32_t rq = waveCtlAdd(M, HPT_MC_RAY_TAIL, 1u);
        if (lane == 0) handoffStore(M.rayQ + rq, (uint64_t) c + 1u);
    }
    /* counts: atomics whose value nobody waits for (no return: the wave does not stall on them) */
    const uint32_t nFin = (uint32_t) __popcll(__ballot(finished)), nShaded = (uint32_t) __popcll(__ballot(alive));
    if (lane == 0) {
        if (nShaded) atomicAdd((unsigned long long *) (counters + HPT_C_BOUNCES), (unsigned long long) nShaded);
        if (nFin) (void) __hip_atomic_fetch_add(M.ctl + HPT_MC_DONE * HPT_MC_STRIDE, nFin, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        (void) __hip_atomic_fetch_add(M.ctl + HPT_MC_STEPS * HPT_MC_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
    }
    return true;
}

#ifndef HPT_PATHS_WAVES
#define HPT_PATHS_WAVES 7
#endif
/* The kernel's argument block, reached through the kernarg segment pointer with its value hidden
   from the optimiser: each phase of k_paths' loop loads the scalars it uses where it uses them
   (scalar loads, scalar cache) instead of every phase's scalars being hoisted out of the loop,
   where they overflowed the SGPRs and, spilled into VGPR lanes, pushed the VGPRs into scratch */
template <class T>
__device__ __forceinline__ const T &launder(const T *x) {
    typedef const __attribute__((address_space(4))) T *CP;
    const uint64_t v = (uint64_t) x;
    uint32_t lo = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) v);
    uint32_t hi = (uint32_t) __builtin_amdgcn_readfirstlane((int) (uint32_t) (v >> 32));
    asm volatile("" : "+s"(lo), "+s"(hi));
    return *(const T *) (CP) (((uint64_t) hi << 32) | lo);
}
template <bool MULTI>
__device__ __forceinline__ void pathsKernel(uint2 *stkBase, PathsWave *waves) {
    static_assert(HPT_TRACE_BLOCK == 256 && HPT_SHADE_BLOCK == 256, "the two LDS views below assume 256-thread blocks");
    static_assert((HPT_STACK + HPT_RAY_ROWS) * 2 >= kRowPath + 1, "the shade rows fit the traversal's LDS");
    const HptPathsArgs *const A = (const HptPathsArgs *) __builtin_amdgcn_kernarg_segment_ptr();
    /* One LDS arena, two views, and a wave's bytes are the same in both (a wave shades while the
       other waves of its block trace).  Shade rows are floats, row r of thread t at r * 256 + t:
       wave w owns bytes [1024 r + 256 w, + 256) of every row.  The traversal's uint2 rows (stride
       256) are laid out inside exactly those bytes: lanes 0-31 of wave w in float row 2k, lanes
       32-63 in row 2k + 1 (uint2 index 256 k + 128 (lane >> 5) + 32 w + (lane & 31)) */
    const uint32_t t = threadIdx.x;
    uint2 *const stk = stkBase + (128u * ((t & 63u) >> 5) + 32u * (t >> 6) + (t & 31u));
    float *const wiL = reinterpret_cast<float *>(stkBase) + t;
    PathsWave *const w = waves + (threadIdx.x >> 6);
    if (__lane_id() == 0) {
        w->rayTicket = w->postTicket = HPT_NO_TICKET;
        w->cur = HPT_NO_TICKET;
        w->taken = 0u;
        w->fill = 0u;
        w->shader = 0u;
        w->claims = 0u;
        w->drains = 0u;
        w->rounds = w->lanes = 0ull;
        for (int e = 0; e < HPT_PATHS_ENTRIES; ++e) w->left[e] = w->total[e] = 0u;
    }
    __builtin_amdgcn_wave_barrier();
    uint32_t nInit;
    {
        const HptPathsArgs &a = launder(A);
        PW_SET(w, postCur, reservePost(a.M, a.counters));
        PW_SET(w, postNext, reservePost(a.M, a.counters));
        nInit = a.counters[HPT_C_SHADE(1)];
        if (blockIdx.x == 0 && threadIdx.x == 0 && nInit) atomicAdd(&a.counters[HPT_C_LAUNCHES], 1u);
    }
    uint64_t idleSince = 0, tTrace = 0, tShade = 0, tIdle = 0, phases = 0;
    while (true) {
        {
            const HptPathsArgs &a = launder(A);
            if (waveCtlLoad(a.M, HPT_MC_DONE) >= nInit || waveCtlLoad(a.M, HPT_MC_ABORT) != 0u) break;
        }
        const uint64_t t0 = __builtin_amdgcn_s_memrealtime();
#ifndef XNO_TRACE
        {
            const HptPathsArgs &a = launder(A);
            pathsTrace(launder(a.sc), a.M, w, stk, a.counters, nInit);
        }
#endif
        {
            const HptPathsArgs &a = launder(A);
            postPublish(a.M, w, a.counters, true); /* out of rays: the part-filled post chunk goes out too */
        }
        const uint64_t t1 = __builtin_amdgcn_s_memrealtime();
        tTrace += t1 - t0;
        ++phases;
        /* shade while there is work and the backlog is short */
        bool worked = false;
        while (true) {
            const HptPathsArgs &a = launder(A);
#ifndef XNO_SHADE
            if (!pathsShadeStep<MULTI>(launder(a.sc), a, w, wiL, nInit)) break;
#else
            break;
#endif
            worked = true;
            if (rayBacklog(a.M) >= a.M.high) break;
        }
        tShade += __builtin_amdgcn_s_memrealtime() - t1;
        const HptPathsArgs &a = launder(A);
        if (PW_GET(w, shader)) {
            waveCtlAdd(a.M, HPT_MC_SHADERS, ~0u);
            PW_SET(w, shader, 0u);
        }
        if (worked) {
            idleSince = 0;
            continue;
        }
        /* nothing ready anywhere: wait a little (bounded: a grid that can make no progress fails
           the call instead of hanging) */
        const uint64_t now = __builtin_amdgcn_s_memrealtime();
        const uint64_t ti = __builtin_amdgcn_s_memrealtime();
        if (idleSince == 0) idleSince = now;
        else if (now - idleSince > HPT_PATHS_IDLE_TICKS) {
            if (__lane_id() == 0) {
                atomicOr(launder(a.sc).fault, HPT_FAULT_PATHS);
                __hip_atomic_store(a.M.ctl + HPT_MC_ABORT * HPT_MC_STRIDE, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            }
            break;
        }
        __builtin_amdgcn_s_sleep(8);
        tIdle += __builtin_amdgcn_s_memrealtime() - ti;
    }
    const HptPathsArgs &a = launder(A);
    if (__lane_id() == 0) {
        auto add64 = [&](int word, uint64_t v) {
            __hip_atomic_fetch_add(reinterpret_cast<uint64_t *>(a.M.ctl + word * HPT_MC_STRIDE), v, __ATOMIC_RELAXED,
                                   __HIP_MEMORY_SCOPE_AGENT);
        };
        add64(HPT_MC_T_TRACE, tTrace);
        add64(HPT_MC_T_SHADE, tShade);
        add64(HPT_MC_T_IDLE, tIdle);
        add64(HPT_MC_CLAIMS, w->claims);
        add64(HPT_MC_PHASES, phases);
        add64(HPT_MC_ROUNDS, w->rounds);
        add64(HPT_MC_LANES, w->lanes);
        add64(HPT_MC_DRAINS, w->drains);
    }
}
} // namespace

extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(HPT_PATHS_WAVES))) void
k_paths(HptPathsArgs) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    __shared__ PathsWave waves[HPT_TRACE_BLOCK / 64];
    pathsKernel<false>(stk, waves);
}
extern "C" __global__ __launch_bounds__(HPT_TRACE_BLOCK) __attribute__((amdgpu_waves_per_eu(HPT_PATHS_WAVES))) void
k_paths_multi(HptPathsArgs) {
    __shared__ uint2 stk[(HPT_STACK + HPT_RAY_ROWS) * HPT_TRACE_BLOCK];
    __shared__ PathsWave waves[HPT_TRACE_BLOCK / 64];
    pathsKernel<true>(stk, waves);
}


/* ------------------------------------------------------------------ */
/* host-side launch wrappers (declared in hpt_kernels.h)               */
/* ------------------------------------------------------------------ */
/* k_paths' resident blocks (occupancy API x CUs), measured once per (device, kernel) */
static unsigned pathsResidentBlocks(const void *kernel) {
    static std::mutex mu;
    static std::map<std::pair<int, const void *>, int> cached;
    int dev = 0;
    (void) hipGetDevice(&dev);
    std::lock_guard<std::mutex> lock(mu);
    auto it = cached.find({dev, kernel});
    if (it == cached.end()) {
        int perCU = 0;
        hipDeviceProp_t prop;
        if (hipGetDeviceProperties(&prop, dev) != hipSuccess ||
            hipOccupancyMaxActiveBlocksPerMultiprocessor(&perCU, kernel, HPT_TRACE_BLOCK, 0) != hipSuccess || perCU <= 0)
            perCU = 7, prop.multiProcessorCount = 256;
        it = cached.emplace(std::make_pair(dev, kernel), perCU * prop.multiProcessorCount).first;
    }
    return (unsigned) std::max(1, it->second);
}
uint32_t hpt_paths_resident_waves(bool multi) {
    return pathsResidentBlocks(multi ? (const void *) k_paths_multi : (const void *) k_paths) * (HPT_TRACE_BLOCK / 64);
}
hipError_t hpt_mega_reset(const HptMega &M, hipStream_t s) {
    hipError_t e = hipMemsetAsync(M.ctl, 0, HPT_MC_WORDS * HPT_MC_STRIDE * 4, s);
    if (e == hipSuccess) e = hipMemsetAsync(M.rayQ, 0, (size_t) M.chunkCap * 8, s);
    if (e == hipSuccess) e = hipMemsetAsync(M.postQ, 0, (size_t) M.postCap * 8, s);
    return e;
}
hipError_t hpt_launch_paths(const HptScene &sc, const HptScene *scDev, const HptPaths &P, const HptMega &M,
                            const uint32_t *shadeQ, uint32_t *counters, hipStream_t s) {
    const bool multi = sc.nShapes > 1;
    const void *kern = multi ? (const void *) k_paths_multi : (const void *) k_paths;
    const unsigned blocks = pathsResidentBlocks(kern);
    const HptPathsArgs args{scDev, P, M, shadeQ, counters};
    if (multi) hipLaunchKernelGGL(k_paths_multi, dim3(blocks), dim3(HPT_TRACE_BLOCK), 0, s, args);
    else hipLaunchKernelGGL(k_paths, dim3(blocks), dim3(HPT_TRACE_BLOCK), 0, s, args);
    return hipGetLastError();
}
