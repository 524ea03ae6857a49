/*
 * accel_experiment.cpp -- CPU count experiment (not product code): traversal
 * work per ray of the product's hair kd-tree versus a wide BVH with spatial
 * splits over the same segments, on camera rays of a scene and on secondary
 * rays (sun shadow rays + uniform continuation rays) from their hits.
 *
 * Build: g++ -O2 -std=c++17 -pthread -I cs184-final-project-mitsuba0.5_amd/csrc tools/accel_experiment.cpp \
 *          cs184-final-project-mitsuba0.5_amd/build/host/{scene_xml,hair_io,kdtree_build,precompute,sunsky,film}.o
 * Run:   ./accel_experiment scene.xml [nrays] [leafSize] [width]
 */
#include <algorithm>
#include <cmath>
#include <cstdio>
#include <cstring>
#include <functional>
#include <random>
#include <vector>

#include "host/host_scene.h"

using namespace hpt;

struct D3 {
    double x, y, z;
};
static D3 d3(double x, double y, double z) { return {x, y, z}; }
static D3 operator-(D3 a, D3 b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
static D3 operator+(D3 a, D3 b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
static D3 operator*(D3 a, double f) { return {a.x * f, a.y * f, a.z * f}; }
static double dot(D3 a, D3 b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

/* hair.cpp:485-548 (counting only: double, no bit-exactness needed) */
static bool segHit(const HptSegment &s, double r, D3 o, D3 d, double mint, double maxt, double &t) {
    D3 v1 = d3(s.v1[0], s.v1[1], s.v1[2]), ax = d3(s.axis[0], s.axis[1], s.axis[2]);
    D3 rel = o - v1, po = rel - ax * dot(ax, rel), pd = d - ax * dot(ax, d);
    double A = dot(pd, pd), B = 2 * dot(po, pd), C = dot(po, po) - r * r;
    double disc = B * B - 4 * A * C;
    if (A == 0 || disc < 0) return false;
    double sq = std::sqrt(disc), tmp = B < 0 ? -0.5 * (B - sq) : -0.5 * (B + sq);
    double t0 = tmp / A, t1 = C / tmp;
    if (t0 > t1) std::swap(t0, t1);
    if (!(t0 <= maxt && t1 >= mint)) return false;
    D3 n1 = d3(s.n1[0], s.n1[1], s.n1[2]), n2 = d3(s.n2[0], s.n2[1], s.n2[2]), v2 = d3(s.v2[0], s.v2[1], s.v2[2]);
    for (int k = 0; k < 2; ++k) {
        double tt = k ? t1 : t0;
        if (tt < mint || tt > maxt) continue;
        D3 p = o + d * tt;
        if (dot(p - v1, n1) >= 0 && dot(p - v2, n2) <= 0) {
            t = tt;
            return true;
        }
    }
    return false;
}

struct Ray {
    float o[3], d[3], mint, maxt;
    bool shadow;
};

struct Counts {
    double nodes = 0, prims = 0, boxes = 0, leaves = 0;
    /* node fetches if the binary tree were stored as G-level groups (group roots at depth % G == 0):
       eager[G] = the node4 scheme (a far side's splits evaluated at push time, so pops land on group
       roots), local3 = 3-level groups whose stack entries may point inside a group (a pop refetches) */
    double eager[5] = {0, 0, 0, 0, 0}, local3 = 0, maxStack = 0;
    uint64_t rays = 0;
};

/* ---------------- kd-tree (binary HptNode, front-to-back) ---------------- */
static std::vector<uint8_t> g_depth; /* binary depth of every kd node */
static bool traceKD(const KDTreeHost &kd, float radius, const Ray &r, double &tHit, uint32_t &seg, Counts &c) {
    float tmin = r.mint, tmax = r.maxt;
    /* scene AABB clip */
    for (int a = 0; a < 3; ++a) {
        float inv = 1.0f / r.d[a];
        float t0 = (kd.aabbMin[a] - r.o[a]) * inv, t1 = (kd.aabbMax[a] - r.o[a]) * inv;
        if (t0 > t1) std::swap(t0, t1);
        tmin = std::max(tmin, t0);
        tmax = std::min(tmax, t1);
    }
    c.rays++;
    if (!(tmax > tmin)) return false;
    struct E {
        uint32_t n;
        float tmin, tmax;
    } st[128];
    int sp = 0;
    uint32_t node = 0;
    double best = r.maxt;
    bool found = false;
    D3 o = d3(r.o[0], r.o[1], r.o[2]), d = d3(r.d[0], r.d[1], r.d[2]);
    bool popped = false;
    while (true) {
        const HptNode &n = kd.nodes[node];
        c.nodes++;
        if (!(n.w0 & 0x80000000u)) {
            const int dep = g_depth[node];
            for (int G = 1; G <= 4; ++G) c.eager[G] += (dep % G == 0) ? 1 : 0;
            c.local3 += (dep % 3 == 0 || popped) ? 1 : 0;
            popped = false;
            int ax = n.w0 & 3;
            uint32_t left = n.w0 >> 2;
            float split;
            std::memcpy(&split, &n.w1, 4);
            float ts = (split - r.o[ax]) / r.d[ax];
            bool below = r.o[ax] < split || (r.o[ax] == split && r.d[ax] <= 0);
            uint32_t first = below ? left : left + 1, second = below ? left + 1 : left;
            if (ts > tmax || ts <= 0) {
                node = first;
            } else if (ts < tmin) {
                node = second;
            } else {
                st[sp++] = {second, ts, tmax};
                node = first;
                tmax = ts;
            }
            continue;
        }
        c.leaves++;
        for (uint32_t e = n.w0 & 0x7fffffffu; e < n.w1; ++e) {
            c.prims++;
            double t;
            uint32_t s = kd.prims[e];
            if (segHit(kd.segs[s], radius, o, d, r.mint, best, t)) {
                found = true;
                if (r.shadow) {
                    tHit = t;
                    return true;
                }
                best = t;
                seg = s;
            }
        }
        if (found && best <= tmax) break;
        if (sp == 0) break;
        --sp;
        popped = true;
        node = st[sp].n;
        tmin = st[sp].tmin;
        tmax = st[sp].tmax;
        if (found && tmin > best) break;
    }
    tHit = best;
    return found;
}

/* The same traversal with G-level grouped nodes whose far sides are expanded at push time (the
   node4 scheme for G = 2): a pushed node inside a group is split on its interval right away and its
   children pushed instead (recursively, down to the next group root or a leaf).  Counts group
   fetches, the peak stack depth and how many rays would overflow an 8-entry ring stack. */
struct EagerCounts {
    double fetches = 0, peak = 0, over8 = 0, pushes = 0;
    uint64_t rays = 0, mism = 0;
};
static bool traceKDEager(const KDTreeHost &kd, int G, float radius, const Ray &r, double &tHit, uint32_t &seg,
                         EagerCounts &c) {
    float tmin = r.mint, tmax = r.maxt;
    for (int a = 0; a < 3; ++a) {
        float inv = 1.0f / r.d[a];
        float t0 = (kd.aabbMin[a] - r.o[a]) * inv, t1 = (kd.aabbMax[a] - r.o[a]) * inv;
        if (t0 > t1) std::swap(t0, t1);
        tmin = std::max(tmin, t0);
        tmax = std::min(tmax, t1);
    }
    c.rays++;
    if (!(tmax > tmin)) return false;
    struct E {
        uint32_t n;
        float tmin, tmax;
    } st[512];
    int sp = 0, peak = 0;
    auto split = [&](uint32_t node, float a, float b, uint32_t &first, uint32_t &second, float &ts, int &kind) {
        const HptNode &n = kd.nodes[node];
        int ax = n.w0 & 3;
        uint32_t left = n.w0 >> 2;
        float spl;
        std::memcpy(&spl, &n.w1, 4);
        ts = (spl - r.o[ax]) / r.d[ax];
        bool below = r.o[ax] < spl || (r.o[ax] == spl && r.d[ax] <= 0);
        first = below ? left : left + 1, second = below ? left + 1 : left;
        kind = (ts > b || ts <= 0) ? 0 : (ts < a ? 1 : 2); /* near only, far only, both */
    };
    /* push node X over [a, b], expanding it while it is an inner node inside a group */
    std::function<void(uint32_t, float, float)> push = [&](uint32_t x, float a, float b) {
        const HptNode &n = kd.nodes[x];
        if ((n.w0 & 0x80000000u) || g_depth[x] % G == 0) {
            st[sp++] = {x, a, b};
            c.pushes++;
            peak = std::max(peak, sp);
            return;
        }
        uint32_t f, s2;
        float ts;
        int kind;
        split(x, a, b, f, s2, ts, kind);
        if (kind == 0) push(f, a, b);
        else if (kind == 1) push(s2, a, b);
        else {
            push(s2, ts, b);
            push(f, a, ts);
        }
    };
    uint32_t node = 0;
    double best = r.maxt;
    bool found = false;
    D3 o = d3(r.o[0], r.o[1], r.o[2]), d = d3(r.d[0], r.d[1], r.d[2]);
    bool fetched = false; /* the current group is in registers */
    while (true) {
        const HptNode &n = kd.nodes[node];
        if (!(n.w0 & 0x80000000u)) {
            if (g_depth[node] % G == 0) c.fetches++;
            uint32_t f, s2;
            float ts;
            int kind;
            split(node, tmin, tmax, f, s2, ts, kind);
            if (kind == 0) node = f;
            else if (kind == 1) node = s2;
            else {
                push(s2, ts, tmax);
                node = f;
                tmax = ts;
            }
            continue;
        }
        for (uint32_t e = n.w0 & 0x7fffffffu; e < n.w1; ++e) {
            double t;
            uint32_t s = kd.prims[e];
            if (segHit(kd.segs[s], radius, o, d, r.mint, best, t)) {
                found = true;
                if (r.shadow) {
                    tHit = t;
                    goto done;
                }
                best = t;
                seg = s;
            }
        }
        if (found && best <= tmax) break;
        if (sp == 0) break;
        --sp;
        node = st[sp].n;
        tmin = st[sp].tmin;
        tmax = st[sp].tmax;
        if (found && tmin > best) break;
    }
    tHit = best;
done:
    c.peak += peak;
    c.over8 += peak > 8 ? 1 : 0;
    (void) fetched;
    return found;
}

/* ---------------- BVH with spatial splits (SBVH-style) ---------------- */
struct Box {
    float mn[3] = {1e30f, 1e30f, 1e30f}, mx[3] = {-1e30f, -1e30f, -1e30f};
    void grow(const Box &b) {
        for (int i = 0; i < 3; ++i) mn[i] = std::min(mn[i], b.mn[i]), mx[i] = std::max(mx[i], b.mx[i]);
    }
    void grow(const float p[3], float e) {
        for (int i = 0; i < 3; ++i) mn[i] = std::min(mn[i], p[i] - e), mx[i] = std::max(mx[i], p[i] + e);
    }
    float area() const {
        float dx = mx[0] - mn[0], dy = mx[1] - mn[1], dz = mx[2] - mn[2];
        if (dx < 0 || dy < 0 || dz < 0) return 0;
        return 2 * (dx * dy + dy * dz + dz * dx);
    }
    bool valid() const { return mx[0] >= mn[0] && mx[1] >= mn[1] && mx[2] >= mn[2]; }
    void clip(const Box &b) {
        for (int i = 0; i < 3; ++i) mn[i] = std::max(mn[i], b.mn[i]), mx[i] = std::min(mx[i], b.mx[i]);
    }
    float c(int a) const { return 0.5f * (mn[a] + mx[a]); }
};

struct SegInfo {
    float a[3], b[3]; /* axis segment extended by the miter overhang */
    float r;          /* radius (+ slack) */
    Box full;
};

struct PRef {
    uint32_t seg;
    Box b;
};

/* part of segment s's solid with coordinate on axis 'ax' within [lo, hi], bounded */
static Box clipSeg(const SegInfo &s, int ax, float lo, float hi, const Box &cur) {
    Box out;
    float pa = s.a[ax], pb = s.b[ax];
    float l = lo - s.r, h = hi + s.r;
    float t0 = 0, t1 = 1;
    float dd = pb - pa;
    if (dd == 0) {
        if (pa < l || pa > h) return out;
    } else {
        float u0 = (l - pa) / dd, u1 = (h - pa) / dd;
        if (u0 > u1) std::swap(u0, u1);
        t0 = std::max(t0, u0);
        t1 = std::min(t1, u1);
        if (t0 > t1) return out;
    }
    float p0[3], p1[3];
    for (int i = 0; i < 3; ++i) {
        p0[i] = s.a[i] + (s.b[i] - s.a[i]) * t0;
        p1[i] = s.a[i] + (s.b[i] - s.a[i]) * t1;
    }
    out.grow(p0, s.r);
    out.grow(p1, s.r);
    out.clip(cur);
    out.mn[ax] = std::max(out.mn[ax], lo);
    out.mx[ax] = std::min(out.mx[ax], hi);
    return out;
}

struct BNode {
    Box b;
    int kid[2] = {-1, -1};
    uint32_t first = 0, count = 0; /* leaf */
};

struct BVHBuilder {
    const std::vector<SegInfo> &S;
    int leafSize;
    bool spatial;
    float travCost = 1.0f, primCost = 1.0f;
    float rootArea = 0;
    std::vector<BNode> nodes;
    std::vector<uint32_t> prims;
    size_t refs = 0;

    int build(std::vector<PRef> &R, int depth) {
        Box bounds, cb;
        for (auto &r : R) {
            bounds.grow(r.b);
            float c[3] = {r.b.c(0), r.b.c(1), r.b.c(2)};
            cb.grow(c, 0);
        }
        if (depth == 0) rootArea = bounds.area();
        int id = (int) nodes.size();
        nodes.push_back(BNode());
        nodes[id].b = bounds;
        const size_t N = R.size();
        auto leaf = [&]() {
            nodes[id].first = (uint32_t) prims.size();
            nodes[id].count = (uint32_t) N;
            for (auto &r : R) prims.push_back(r.seg);
            return id;
        };
        if ((int) N <= leafSize || depth > 60) return leaf();
        const int B = 32;
        float bestCost = 1e30f;
        int bestAx = -1, bestBin = -1;
        bool bestSpatial = false;
        float invA = 1.0f / bounds.area();
        /* object splits over centroid bins */
        for (int ax = 0; ax < 3; ++ax) {
            float lo = cb.mn[ax], ext = cb.mx[ax] - lo;
            if (!(ext > 0)) continue;
            Box bb[B];
            size_t cnt[B] = {};
            for (auto &r : R) {
                int k = std::min(B - 1, (int) ((r.b.c(ax) - lo) / ext * B));
                bb[k].grow(r.b);
                cnt[k]++;
            }
            Box rb[B];
            size_t rc[B];
            Box acc;
            size_t ac = 0;
            for (int k = B - 1; k > 0; --k) {
                acc.grow(bb[k]);
                ac += cnt[k];
                rb[k] = acc;
                rc[k] = ac;
            }
            acc = Box();
            ac = 0;
            for (int k = 0; k < B - 1; ++k) {
                acc.grow(bb[k]);
                ac += cnt[k];
                if (ac == 0 || rc[k + 1] == 0) continue;
                float cost = travCost + primCost * (acc.area() * ac + rb[k + 1].area() * rc[k + 1]) * invA;
                if (cost < bestCost) bestCost = cost, bestAx = ax, bestBin = k, bestSpatial = false;
            }
        }
        /* spatial splits over bounds bins */
        float spLo[3], spExt[3];
        if (spatial) {
            for (int ax = 0; ax < 3; ++ax) {
                float lo = bounds.mn[ax], ext = bounds.mx[ax] - lo;
                spLo[ax] = lo;
                spExt[ax] = ext;
                if (!(ext > 0)) continue;
                Box bb[B];
                size_t enter[B] = {}, exitc[B] = {};
                for (auto &r : R) {
                    int k0 = std::min(B - 1, std::max(0, (int) ((r.b.mn[ax] - lo) / ext * B)));
                    int k1 = std::min(B - 1, std::max(0, (int) ((r.b.mx[ax] - lo) / ext * B)));
                    enter[k0]++;
                    exitc[k1]++;
                    for (int k = k0; k <= k1; ++k) {
                        float bl = lo + ext * k / B, bh = lo + ext * (k + 1) / B;
                        Box p = clipSeg(S[r.seg], ax, bl, bh, r.b);
                        if (p.valid()) bb[k].grow(p);
                    }
                }
                Box rb[B];
                size_t rc[B];
                Box acc;
                size_t ac = 0;
                for (int k = B - 1; k > 0; --k) {
                    acc.grow(bb[k]);
                    ac += exitc[k];
                    rb[k] = acc;
                    rc[k] = ac;
                }
                acc = Box();
                ac = 0;
                for (int k = 0; k < B - 1; ++k) {
                    acc.grow(bb[k]);
                    ac += enter[k];
                    if (ac == 0 || rc[k + 1] == 0) continue;
                    float cost = travCost + primCost * (acc.area() * ac + rb[k + 1].area() * rc[k + 1]) * invA;
                    if (cost < bestCost) bestCost = cost, bestAx = ax, bestBin = k, bestSpatial = true;
                }
            }
        }
        if (bestAx < 0 || (bestCost >= primCost * N && (int) N <= 4 * leafSize)) return leaf();
        std::vector<PRef> L, Rr;
        if (!bestSpatial) {
            float lo = cb.mn[bestAx], ext = cb.mx[bestAx] - lo;
            for (auto &r : R) {
                int k = std::min(B - 1, (int) ((r.b.c(bestAx) - lo) / ext * B));
                (k <= bestBin ? L : Rr).push_back(r);
            }
        } else {
            float pos = spLo[bestAx] + spExt[bestAx] * (bestBin + 1) / B;
            for (auto &r : R) {
                if (r.b.mx[bestAx] <= pos) L.push_back(r);
                else if (r.b.mn[bestAx] >= pos) Rr.push_back(r);
                else {
                    Box bl = clipSeg(S[r.seg], bestAx, r.b.mn[bestAx], pos, r.b);
                    Box br = clipSeg(S[r.seg], bestAx, pos, r.b.mx[bestAx], r.b);
                    if (bl.valid()) L.push_back({r.seg, bl});
                    if (br.valid()) Rr.push_back({r.seg, br});
                }
            }
            if (L.empty() || Rr.empty()) return leaf();
        }
        std::vector<PRef>().swap(R);
        int a = build(L, depth + 1);
        int b = build(Rr, depth + 1);
        nodes[id].kid[0] = a;
        nodes[id].kid[1] = b;
        return id;
    }
};

/* wide node: up to W children (node or leaf refs into the binary tree) */
struct WNode {
    int n = 0;
    int kid[8];
};

static void collapse(const std::vector<BNode> &bn, int W, std::vector<WNode> &out, std::vector<int> &map) {
    /* out[i] corresponds to binary inner node 'src'; children are binary nodes
       (inner -> wide node later, or leaves) */
    map.assign(bn.size(), -1);
    std::vector<int> todo = {0};
    while (!todo.empty()) {
        int src = todo.back();
        todo.pop_back();
        WNode w;
        std::vector<int> ch = {bn[src].kid[0], bn[src].kid[1]};
        while ((int) ch.size() < W) {
            /* open the child with the largest area that is an inner node */
            int best = -1;
            float ba = -1;
            for (int i = 0; i < (int) ch.size(); ++i) {
                const BNode &c = bn[ch[i]];
                if (c.kid[0] >= 0 && c.b.area() > ba) ba = c.b.area(), best = i;
            }
            if (best < 0) break;
            int c = ch[best];
            ch.erase(ch.begin() + best);
            ch.push_back(bn[c].kid[0]);
            ch.push_back(bn[c].kid[1]);
        }
        w.n = (int) ch.size();
        for (int i = 0; i < w.n; ++i) {
            w.kid[i] = ch[i];
            if (bn[ch[i]].kid[0] >= 0) todo.push_back(ch[i]);
        }
        map[src] = (int) out.size();
        out.push_back(w);
    }
}

static bool rayBox(const Box &b, const float o[3], const float inv[3], float tmin, float tmax, float &tn) {
    for (int a = 0; a < 3; ++a) {
        float t0 = (b.mn[a] - o[a]) * inv[a], t1 = (b.mx[a] - o[a]) * inv[a];
        if (t0 > t1) std::swap(t0, t1);
        tmin = std::max(tmin, t0);
        tmax = std::min(tmax, t1 * 1.0000004f);
    }
    tn = tmin;
    return tmin <= tmax;
}

static bool traceWide(const std::vector<BNode> &bn, const std::vector<WNode> &wn, const std::vector<int> &map,
                      const std::vector<uint32_t> &prims, const std::vector<HptSegment> &segs, float radius,
                      const Ray &r, double &tHit, uint32_t &seg, Counts &c) {
    float inv[3] = {1.0f / r.d[0], 1.0f / r.d[1], 1.0f / r.d[2]};
    c.rays++;
    D3 o = d3(r.o[0], r.o[1], r.o[2]), d = d3(r.d[0], r.d[1], r.d[2]);
    double best = r.maxt;
    bool found = false;
    struct E {
        int bnode;
        float t;
    } st[256];
    int sp = 0;
    float tn;
    if (!rayBox(bn[0].b, r.o, inv, r.mint, r.maxt, tn)) return false;
    st[sp++] = {0, tn};
    while (sp) {
        E e = st[--sp];
        if (e.t > best) continue;
        const BNode &b = bn[e.bnode];
        if (b.kid[0] < 0) {
            c.leaves++;
            for (uint32_t k = b.first; k < b.first + b.count; ++k) {
                c.prims++;
                double t;
                if (segHit(segs[prims[k]], radius, o, d, r.mint, best, t)) {
                    found = true;
                    if (r.shadow) {
                        tHit = t;
                        return true;
                    }
                    best = t;
                    seg = prims[k];
                }
            }
            continue;
        }
        c.nodes++;
        const WNode &w = wn[map[e.bnode]];
        E hit[8];
        int nh = 0;
        for (int i = 0; i < w.n; ++i) {
            c.boxes++;
            if (rayBox(bn[w.kid[i]].b, r.o, inv, r.mint, (float) best, tn)) hit[nh++] = {w.kid[i], tn};
        }
        std::sort(hit, hit + nh, [](const E &a, const E &b) { return a.t > b.t; });
        for (int i = 0; i < nh; ++i) st[sp++] = hit[i];
    }
    tHit = best;
    return found;
}

int main(int argc, char **argv) {
    if (argc < 2) {
        fprintf(stderr, "usage: %s scene.xml [nrays] [leafSize] [spatial]\n", argv[0]);
        return 1;
    }
    int nrays = argc > 2 ? atoi(argv[2]) : 20000;
    int leafSize = argc > 3 ? atoi(argv[3]) : 4;
    int spatial = argc > 4 ? atoi(argv[4]) : 1;
    SceneDesc d = parseSceneXML(argv[1], {});
    HairData hair;
    for (auto &h : d.shapes) {
        HairData one = loadHair(h.file, h.radius, h.angleThreshold, h.reduction, h.hasToWorld ? h.toWorld : nullptr);
        appendHair(hair, one);
    }
    KDTreeHost kd = buildHairKDTree(hair, d.kd);
    g_depth.assign(kd.nodes.size(), 0);
    for (size_t i = 0; i < kd.nodes.size(); ++i)
        if (!(kd.nodes[i].w0 & 0x80000000u)) {
            const uint32_t left = kd.nodes[i].w0 >> 2;
            g_depth[left] = g_depth[left + 1] = (uint8_t) (g_depth[i] + 1);
        }
    const size_t nseg = kd.segs.size();
    float radius = hair.radius;
    printf("segments %zu, kd nodes %zu, kd refs %zu (%.2f per segment), build %.2f s\n", nseg, kd.nodes.size(),
           kd.prims.size(), (double) kd.prims.size() / nseg, kd.buildSeconds);
    printf("radius %.6g, 16-byte pre-test radius %.6g (x%.5f), %zu records flagged to pass\n", hair.radius,
           kd.preRadius, kd.preRadius / hair.radius, kd.prePassRecords);
    if (argc > 5) return 0;

    /* segment solids: axis segment extended by the miter overhang, radius + slack */
    std::vector<SegInfo> S(nseg);
    for (size_t i = 0; i < nseg; ++i) {
        const HptSegment &s = kd.segs[i];
        double rr = hair.radiusOf(s.iv);
        double c1 = std::fabs(s.n1[0] * s.axis[0] + s.n1[1] * s.axis[1] + s.n1[2] * s.axis[2]);
        double c2 = std::fabs(s.n2[0] * s.axis[0] + s.n2[1] * s.axis[1] + s.n2[2] * s.axis[2]);
        double m1 = rr * std::sqrt(std::max(0.0, 1 - c1 * c1)) / std::max(c1, 1e-3);
        double m2 = rr * std::sqrt(std::max(0.0, 1 - c2 * c2)) / std::max(c2, 1e-3);
        for (int k = 0; k < 3; ++k) {
            S[i].a[k] = (float) (s.v1[k] - s.axis[k] * m1);
            S[i].b[k] = (float) (s.v2[k] + s.axis[k] * m2);
        }
        S[i].r = (float) (rr * 1.001 + 1e-6);
        S[i].full.grow(S[i].a, S[i].r);
        S[i].full.grow(S[i].b, S[i].r);
    }
    std::vector<PRef> R(nseg);
    for (size_t i = 0; i < nseg; ++i) R[i] = {(uint32_t) i, S[i].full};
    BVHBuilder bb{S, leafSize, spatial != 0};
    bb.build(R, 0);
    printf("bvh: %zu binary nodes, %zu refs (%.2f per segment)\n", bb.nodes.size(), bb.prims.size(),
           (double) bb.prims.size() / nseg);

    /* rays */
    HptCamera cam;
    setupCamera(d, cam);
    std::mt19937 rng(1);
    std::uniform_real_distribution<float> U(0, 1);
    std::vector<Ray> camRays, secRays, shRays;
    const float sun[3] = {-0.376047f, 0.758426f, 0.532333f};
    float sl = std::sqrt(sun[0] * sun[0] + sun[1] * sun[1] + sun[2] * sun[2]);
    for (int i = 0; i < nrays; ++i) {
        float px = U(rng) * cam.width, py = U(rng) * cam.height;
        float x = px * cam.invResX, y = py * cam.invResY;
        const float *M = cam.s2c;
        float nx = M[0] * x + M[1] * y + M[3], ny = M[4] * x + M[5] * y + M[7], nz = M[8] * x + M[9] * y + M[11],
              nw = M[12] * x + M[13] * y + M[15];
        nx /= nw, ny /= nw, nz /= nw;
        float l = std::sqrt(nx * nx + ny * ny + nz * nz);
        nx /= l, ny /= l, nz /= l;
        const float *T = cam.toWorld;
        Ray r;
        r.o[0] = T[3], r.o[1] = T[7], r.o[2] = T[11];
        r.d[0] = T[0] * nx + T[1] * ny + T[2] * nz;
        r.d[1] = T[4] * nx + T[5] * ny + T[6] * nz;
        r.d[2] = T[8] * nx + T[9] * ny + T[10] * nz;
        r.mint = cam.nearClip / nz;
        r.maxt = cam.farClip / nz;
        r.shadow = false;
        camRays.push_back(r);
    }
    printf("wide BVH: per ray  nodes(fetches) boxes  leaves prims | kd: binary nodes leaves prims\n");
    for (int W : {2, 4, 8}) {
        std::vector<WNode> wn;
        std::vector<int> map;
        collapse(bb.nodes, W, wn, map);
        Counts ck[3], cb[3];
        secRays.clear();
        shRays.clear();
        size_t mism = 0;
        for (auto &r : camRays) {
            double t1 = 0, t2 = 0;
            uint32_t s1 = 0, s2 = 0;
            bool h1 = traceKD(kd, radius, r, t1, s1, ck[0]);
            bool h2 = traceWide(bb.nodes, wn, map, bb.prims, kd.segs, radius, r, t2, s2, cb[0]);
            if (h1 != h2 || (h1 && s1 != s2)) mism++;
            if (h1 && W == 2) {
                Ray s;
                for (int k = 0; k < 3; ++k) s.o[k] = r.o[k] + r.d[k] * (float) t1;
                for (int k = 0; k < 3; ++k) s.d[k] = sun[k] / sl;
                s.mint = 1e-4f * std::max(std::fabs(s.o[0]), std::max(std::fabs(s.o[1]), std::fabs(s.o[2])));
                s.maxt = 1e30f;
                s.shadow = true;
                shRays.push_back(s);
                float z = 2 * U(rng) - 1, ph = 6.2831853f * U(rng), q = std::sqrt(1 - z * z);
                s.d[0] = q * std::cos(ph), s.d[1] = q * std::sin(ph), s.d[2] = z;
                s.shadow = false;
                secRays.push_back(s);
            }
        }
        static std::vector<Ray> sec0, sh0;
        if (W == 2) sec0 = secRays, sh0 = shRays;
        for (auto &r : sec0) {
            double t1 = 0, t2 = 0;
            uint32_t s1 = 0, s2 = 0;
            bool h1 = traceKD(kd, radius, r, t1, s1, ck[1]);
            bool h2 = traceWide(bb.nodes, wn, map, bb.prims, kd.segs, radius, r, t2, s2, cb[1]);
            if (h1 != h2 || (h1 && s1 != s2)) mism++;
        }
        for (auto &r : sh0) {
            double t1 = 0, t2 = 0;
            uint32_t s1 = 0, s2 = 0;
            bool h1 = traceKD(kd, radius, r, t1, s1, ck[2]);
            bool h2 = traceWide(bb.nodes, wn, map, bb.prims, kd.segs, radius, r, t2, s2, cb[2]);
            if (h1 != h2) mism++;
        }
        const char *nm[3] = {"camera", "continuation", "shadow"};
        for (int k = 0; k < 3; ++k) {
            double n = (double) std::max<uint64_t>(1, cb[k].rays);
            printf("W=%d %-12s  %6.2f %6.1f %6.2f %6.2f | %6.2f %6.2f %6.2f   (rays %llu)\n", W, nm[k],
                   cb[k].nodes / n, cb[k].boxes / n, cb[k].leaves / n, cb[k].prims / n, ck[k].nodes / n,
                   ck[k].leaves / n, ck[k].prims / n, (unsigned long long) cb[k].rays);
        }
        printf("W=%d wide nodes %zu, mismatches %zu\n", W, wn.size(), mism);
        if (W == 2)
            for (int G = 1; G <= 4; ++G) {
                const std::vector<Ray> *sets[3] = {&camRays, &sec0, &sh0};
                for (int k = 0; k < 3; ++k) {
                    EagerCounts ec;
                    for (auto &r : *sets[k]) {
                        double t1 = 0, t2 = 0;
                        uint32_t s1 = 0, s2 = 0;
                        Counts dummy;
                        bool h1 = traceKD(kd, radius, r, t1, s1, dummy);
                        bool h2 = traceKDEager(kd, G, radius, r, t2, s2, ec);
                        if (h1 != h2 || (h1 && !r.shadow && (s1 != s2 || t1 != t2))) ec.mism++;
                    }
                    double n = (double) std::max<uint64_t>(1, ec.rays);
                    printf("eager G=%d %-12s fetches %.2f  pushes %.2f  mean peak stack %.2f  rays over 8 entries "
                           "%.3f%%  mismatches %llu\n", G, nm[k], ec.fetches / n, ec.pushes / n, ec.peak / n,
                           100.0 * ec.over8 / n, (unsigned long long) ec.mism);
                }
            }
        if (W == 2)
            for (int k = 0; k < 3; ++k) {
                double n = (double) std::max<uint64_t>(1, ck[k].rays);
                printf("kd %-12s inner-node fetches: binary %.2f, eager 2-level %.2f, 3-level %.2f, 4-level %.2f; "
                       "3-level with in-group stack entries %.2f\n", nm[k], ck[k].eager[1] / n, ck[k].eager[2] / n,
                       ck[k].eager[3] / n, ck[k].eager[4] / n, ck[k].local3 / n);
            }
    }
    return 0;
}
