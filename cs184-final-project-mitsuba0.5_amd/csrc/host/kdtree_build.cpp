/*
 * kdtree_build.cpp -- SAH kd-tree over hair segments (host, multithreaded).
 *
 * Cost model and parameters follow HairKDTree (src/shapes/hair.cpp:108-159):
 * traversal cost 10, query cost 15, empty-space bonus 0.9, stop at 1
 * primitive, clipping ("perfect splits") on, retraction after 3 bad
 * refinements, depth cap 8 + 1.3 log2(N) limited to 48 (gkdtree.h:986-988).
 * Split search is min-max binning (128 bins) for large nodes and an exact
 * event sweep for small ones -- the same two-tier strategy as
 * GenericKDTree::buildTreeMinMax / buildTreeSAH, implemented independently.
 *
 * Primitive bounds use the reference's geometry:
 *   getAABB        -- ellipses cut by the two miter planes, radius*(1-1e-4)
 *                     (hair.cpp:349-378)
 *   getClippedAABB -- infinite cylinder (radius*(1+1e-4)) against the six
 *                     faces of the clipped box (hair.cpp:246-343)
 * in single precision like the reference.  The tree's AABB is the union of
 * getAABB over all segments, which the traversal uses for its entry clip
 * (hair.cpp:200-217, skdtree.cpp:124).
 *
 * Output layout (hpt_device.h HptNode): sibling pairs, so an inner node's
 * children are nodes[left] and nodes[left+1], packed breadth-first into
 * 128-byte treelet blocks (layoutTreelets).
 */
#include <algorithm>
#include <array>
#include <chrono>
#include <cmath>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <future>
#include <limits>
#include <stdexcept>
#include <thread>

#include "host_scene.h"

namespace hpt {
namespace {

const float kEps = 1e-4f;
const float kInf = std::numeric_limits<float>::infinity();

struct V {
    float x, y, z;
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    float &operator[](int i) { return i == 0 ? x : (i == 1 ? y : z); }
};
inline V operator+(V a, V b) { return {a.x + b.x, a.y + b.y, a.z + b.z}; }
inline V operator-(V a, V b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline V operator*(V a, float f) { return {a.x * f, a.y * f, a.z * f}; }
inline V operator*(float f, V a) { return a * f; }
inline float dot(V a, V b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
inline float len(V a) { return std::sqrt(dot(a, a)); }
inline V cross(V a, V b) { return {a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x}; }
inline V normalize(V a) { float r = 1.0f / len(a); return a * r; }
inline bool eq(V a, V b) { return a.x == b.x && a.y == b.y && a.z == b.z; }

struct Box {
    V mn{kInf, kInf, kInf}, mx{-kInf, -kInf, -kInf};
    bool valid() const { return mx.x >= mn.x && mx.y >= mn.y && mx.z >= mn.z; }
    void expand(V p) {
        for (int i = 0; i < 3; ++i) {
            mn[i] = std::min(mn[i], p[i]);
            mx[i] = std::max(mx[i], p[i]);
        }
    }
    void expand(const Box &b) {
        for (int i = 0; i < 3; ++i) {
            mn[i] = std::min(mn[i], b.mn[i]);
            mx[i] = std::max(mx[i], b.mx[i]);
        }
    }
    void clip(const Box &b) {
        for (int i = 0; i < 3; ++i) {
            mn[i] = std::max(mn[i], b.mn[i]);
            mx[i] = std::min(mx[i], b.mx[i]);
        }
    }
    bool contains(V p) const {
        for (int i = 0; i < 3; ++i)
            if (p[i] < mn[i] || p[i] > mx[i]) return false;
        return true;
    }
    float area() const {
        V d = mx - mn;
        return 2.0f * (d.x * d.y + d.y * d.z + d.z * d.x);
    }
};

void coordSystem(V a, V &b, V &c) { /* util.cpp:592-601 */
    if (std::abs(a.x) > std::abs(a.y)) {
        float inv = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = {a.z * inv, 0.0f, -a.x * inv};
    } else {
        float inv = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = {0.0f, a.z * inv, -a.y * inv};
    }
    b = cross(c, a);
}

bool solveQuadF(float a, float b, float c, float &x0, float &x1) {
    if (a == 0) {
        if (b != 0) { x0 = x1 = -c / b; return true; }
        return false;
    }
    float disc = b * b - 4.0f * a * c;
    if (disc < 0) return false;
    float sq = std::sqrt(disc), temp = (b < 0) ? -0.5f * (b - sq) : -0.5f * (b + sq);
    x0 = temp / a;
    x1 = c / temp;
    if (x0 > x1) std::swap(x0, x1);
    return true;
}

struct SegGeom {
    const HairData &h;
    explicit SegGeom(const HairData &hd) : h(hd) {}
    V vtx(uint32_t i) const { return {h.xyz[3 * i], h.xyz[3 * i + 1], h.xyz[3 * i + 2]}; }
    V tangent(uint32_t iv) const { return normalize(vtx(iv + 1) - vtx(iv)); }
    V firstMiter(uint32_t iv) const {
        return !h.starts[iv] ? normalize(normalize(vtx(iv) - vtx(iv - 1)) + tangent(iv)) : tangent(iv);
    }
    V secondMiter(uint32_t iv) const {
        return !h.starts[iv + 2] ? normalize(tangent(iv) + normalize(vtx(iv + 2) - vtx(iv + 1))) : tangent(iv);
    }

    /* ellipse from cutting an infinite cylinder with a plane (hair.cpp:246-286) */
    static bool cylPlane(V planePt, V planeN, V cylPt, V cylD, float radius, V &center, V *axes, float *lengths) {
        if (std::abs(dot(planeN, cylD)) < kEps) return false;
        V B, A = cylD - dot(cylD, planeN) * planeN;
        float l = len(A);
        if (l > kEps && !eq(planeN, cylD)) {
            A = A * (1.0f / l);
            B = cross(planeN, A);
        } else {
            coordSystem(planeN, A, B);
        }
        V delta = planePt - cylPt, deltaProj = delta - cylD * dot(delta, cylD);
        float aDotD = dot(A, cylD), bDotD = dot(B, cylD);
        float c0 = 1 - aDotD * aDotD, c1 = 1 - bDotD * bDotD;
        float c2 = 2 * dot(A, deltaProj), c3 = 2 * dot(B, deltaProj);
        float c4 = dot(delta, deltaProj) - radius * radius;
        float lambda = (c2 * c2 / (4 * c0) + c3 * c3 / (4 * c1) - c4) / (c0 * c1);
        float alpha0 = -c2 / (2 * c0), beta0 = -c3 / (2 * c1);
        lengths[0] = std::sqrt(c1 * lambda);
        lengths[1] = std::sqrt(c0 * lambda);
        center = planePt + alpha0 * A + beta0 * B;
        axes[0] = A;
        axes[1] = B;
        return true;
    }

    /* hair.cpp:349-378 */
    Box aabb(uint32_t iv) const {
        Box r;
        V c, ax[2];
        float l[2] = {0, 0};
        for (int end = 0; end < 2; ++end) {
            V p = end == 0 ? vtx(iv) : vtx(iv + 1);
            V n = end == 0 ? firstMiter(iv) : secondMiter(iv);
            if (!cylPlane(p, n, p, tangent(iv), h.radiusOf(iv) * (1 - kEps), c, ax, l)) {
                l[0] = l[1] = 0;
                c = p;
            }
            ax[0] = ax[0] * l[0];
            ax[1] = ax[1] * l[1];
            for (int i = 0; i < 3; ++i) {
                float range = std::sqrt(ax[0][i] * ax[0][i] + ax[1][i] * ax[1][i]);
                r.mn[i] = std::min(r.mn[i], c[i] - range);
                r.mx[i] = std::max(r.mx[i], c[i] + range);
            }
        }
        return r;
    }

    /* hair.cpp:289-343 */
    Box cylFace(int axis, V mn, V mx, V cylPt, V cylD, float radius) const {
        int a1 = (axis + 1) % 3, a2 = (axis + 2) % 3;
        V n{0, 0, 0};
        n[axis] = 1;
        V c, ax[2];
        float l[2];
        Box out;
        if (!cylPlane(mn, n, cylPt, cylD, radius * (1 + kEps), c, ax, l)) return out;
        for (int i = 0; i < 4; ++i) {
            V p1, p2;
            p1[axis] = p2[axis] = mn[axis];
            p1[a1] = ((i + 1) & 2) ? mn[a1] : mx[a1];
            p1[a2] = ((i + 0) & 2) ? mn[a2] : mx[a2];
            p2[a1] = ((i + 2) & 2) ? mn[a1] : mx[a1];
            p2[a2] = ((i + 1) & 2) ? mn[a2] : mx[a2];
            float p1x = dot(p1 - c, ax[0]) / l[0], p1y = dot(p1 - c, ax[1]) / l[1];
            float p2x = dot(p2 - c, ax[0]) / l[0], p2y = dot(p2 - c, ax[1]) / l[1];
            float rx = p2x - p1x, ry = p2y - p1y;
            float A = rx * rx + ry * ry, B = 2 * (p1x * rx + p1y * ry), C = p1x * p1x + p1y * p1y - 1;
            float x0, x1;
            if (solveQuadF(A, B, C, x0, x1)) {
                if (x0 >= 0 && x0 <= 1) out.expand(p1 + (p2 - p1) * x0);
                if (x1 >= 0 && x1 <= 1) out.expand(p1 + (p2 - p1) * x1);
            }
        }
        ax[0] = ax[0] * l[0];
        ax[1] = ax[1] * l[1];
        Box face;
        face.mn = mn;
        face.mx = mx;
        for (int i = 0; i < 2; ++i) {
            int j = (i == 0) ? a1 : a2;
            float alpha = ax[0][j], beta = ax[1][j];
            float tmp = 1 / std::sqrt(alpha * alpha + beta * beta);
            float cosT = alpha * tmp, sinT = beta * tmp;
            V q1 = c + cosT * ax[0] + sinT * ax[1];
            V q2 = c - cosT * ax[0] - sinT * ax[1];
            if (face.contains(q1)) out.expand(q1);
            if (face.contains(q2)) out.expand(q2);
        }
        return out;
    }

    /* getClippedAABB (hair.cpp:381-444) starting from the primitive's current
       bounds instead of its full AABB: those already contain the segment's
       part inside the parent cell, so the result stays conservative and
       each level avoids re-deriving the miter ellipses */
    Box clipped(uint32_t iv, const Box &cur, const Box &box) const {
        Box base = cur;
        base.clip(box);
        if (!base.valid()) return base;
        V cp = vtx(iv), cd = tangent(iv);
        const float rad = h.radiusOf(iv);
        Box r;
        const V &a = base.mn, &b = base.mx;
        r.expand(cylFace(0, {a.x, a.y, a.z}, {a.x, b.y, b.z}, cp, cd, rad));
        r.expand(cylFace(0, {b.x, a.y, a.z}, {b.x, b.y, b.z}, cp, cd, rad));
        r.expand(cylFace(1, {a.x, a.y, a.z}, {b.x, a.y, b.z}, cp, cd, rad));
        r.expand(cylFace(1, {a.x, b.y, a.z}, {b.x, b.y, b.z}, cp, cd, rad));
        r.expand(cylFace(2, {a.x, a.y, a.z}, {b.x, b.y, a.z}, cp, cd, rad));
        r.expand(cylFace(2, {a.x, a.y, b.z}, {b.x, b.y, b.z}, cp, cd, rad));
        r.clip(base);
        return r;
    }
};

struct Ref {
    uint32_t seg;
    Box b;
};

/* f(begin, end, chunk) over [0, n) in contiguous chunks, one thread each;
   chunk order is index order, so per-chunk outputs concatenated in chunk
   order equal the serial result */
template <class F> void parallelChunks(size_t n, int threads, size_t minPerThread, F f) {
    threads = (int) std::min<size_t>((size_t) std::max(1, threads), std::max<size_t>(1, n / minPerThread));
    if (threads <= 1) {
        f((size_t) 0, n, 0);
        return;
    }
    const size_t chunk = (n + threads - 1) / threads;
    std::vector<std::thread> th;
    for (int t = 1; t < threads; ++t) {
        size_t b = t * chunk, e = std::min(n, b + chunk);
        if (b < e) th.emplace_back(f, b, e, t);
    }
    f((size_t) 0, std::min(n, chunk), 0);
    for (auto &x : th) x.join();
}

struct BNode {
    int axis = -1;
    float split = 0;
    std::unique_ptr<BNode> kid[2];
    std::vector<uint32_t> prims;
    uint32_t pStart = 0, pEnd = 0; /* range in KDTreeHost::prims once laid out */
};

struct Builder {
    const SegGeom &g;
    const std::vector<uint32_t> &segIv;
    KDBuildParams P;
    int maxDepth;
    int hwThreads;

    struct Split {
        float cost = kInf;
        int axis = -1;
        float pos = 0;
        size_t nl = 0, nr = 0;
    };

    Split findSplit(const std::vector<Ref> &refs, const Box &bounds, int threads) const {
        Split best;
        const size_t N = refs.size();
        const float invSA = 1.0f / bounds.area();
        for (int axis = 0; axis < 3; ++axis) {
            float lo = bounds.mn[axis], hi = bounds.mx[axis], ext = hi - lo;
            if (!(ext > 0)) continue;
            auto evalCost = [&](float pos, size_t nl, size_t nr) {
                Box L = bounds, R = bounds;
                L.mx[axis] = pos;
                R.mn[axis] = pos;
                float c = P.traversalCost + P.queryCost * (L.area() * nl + R.area() * nr) * invSA;
                if (nl == 0 || nr == 0) c *= P.emptySpaceBonus;
                return c;
            };
            if ((int) N <= P.exactSweepMax) {
                /* exact sweep over primitive bound events */
                std::vector<std::pair<float, int>> ev;
                ev.reserve(2 * N);
                for (auto &r : refs) {
                    ev.push_back({r.b.mn[axis], 1}); /* start */
                    ev.push_back({r.b.mx[axis], 0}); /* end */
                }
                std::sort(ev.begin(), ev.end());
                size_t nl = 0, nr = N;
                for (size_t i = 0; i < ev.size();) {
                    float pos = ev[i].first;
                    size_t ends = 0, starts = 0;
                    while (i < ev.size() && ev[i].first == pos) {
                        if (ev[i].second == 0) ends++;
                        else starts++;
                        ++i;
                    }
                    nr -= ends;
                    if (pos > lo && pos < hi) {
                        float c = evalCost(pos, nl, nr);
                        if (c < best.cost) best = {c, axis, pos, nl, nr};
                    }
                    nl += starts;
                }
            } else {
                const int B = P.bins;
                std::vector<uint32_t> minB(B, 0), maxB(B, 0);
                float scale = B / ext;
                /* per-chunk histograms (integer counts: the sum is order independent) */
                const int T = std::max(1, threads);
                std::vector<std::vector<uint32_t>> hMin(T), hMax(T);
                parallelChunks(N, T, 1u << 16, [&](size_t b0, size_t e0, int t) {
                    std::vector<uint32_t> &mnB = hMin[t], &mxB = hMax[t];
                    mnB.assign(B, 0);
                    mxB.assign(B, 0);
                    for (size_t k = b0; k < e0; ++k) {
                        const Ref &r = refs[k];
                        int a = (int) ((r.b.mn[axis] - lo) * scale), b = (int) ((r.b.mx[axis] - lo) * scale);
                        a = std::min(std::max(a, 0), B - 1);
                        b = std::min(std::max(b, 0), B - 1);
                        mnB[a]++;
                        mxB[b]++;
                    }
                });
                for (int t = 0; t < T; ++t)
                    for (int i = 0; i < B && !hMin[t].empty(); ++i) {
                        minB[i] += hMin[t][i];
                        maxB[i] += hMax[t][i];
                    }
                size_t nl = 0, nEndedLeft = 0;
                for (int i = 0; i < B - 1; ++i) {
                    nl += minB[i];
                    nEndedLeft += maxB[i];
                    size_t nr = N - nEndedLeft;
                    float pos = lo + (float) (i + 1) * (ext / B);
                    if (!(pos > lo && pos < hi)) continue;
                    float c = evalCost(pos, nl, nr);
                    if (c < best.cost) best = {c, axis, pos, nl, nr};
                }
            }
        }
        return best;
    }

    std::unique_ptr<BNode> build(std::vector<Ref> refs, Box bounds, int depth, int badRefines) {
        std::unique_ptr<BNode> node(new BNode());
        const size_t N = refs.size();
        auto makeLeaf = [&]() {
            node->prims.reserve(N);
            for (auto &r : refs) node->prims.push_back(r.seg);
            return std::move(node);
        };
        if ((int) N <= P.stopPrims || depth >= maxDepth) return makeLeaf();
        float leafCost = P.queryCost * (float) N;
        /* threads for the data-parallel passes of this node: the top levels see
           most of the primitives while few subtrees run concurrently */
        const int threads = depth < 3 ? std::max(1, hwThreads >> depth) : 1;
        Split s = findSplit(refs, bounds, threads);
        if (s.axis < 0) return makeLeaf();
        if (s.cost >= leafCost) {
            if ((s.cost > 4 * leafCost && N < 16) || badRefines >= P.maxBadRefines) return makeLeaf();
            ++badRefines;
        }
        Box lb = bounds, rb = bounds;
        lb.mx[s.axis] = s.pos;
        rb.mn[s.axis] = s.pos;
        /* partition (straddling primitives are clipped to both halves); per-chunk
           outputs concatenated in chunk order == the serial order */
        std::vector<std::vector<Ref>> cL(std::max(1, threads)), cR(std::max(1, threads));
        parallelChunks(N, threads, 1u << 15, [&](size_t b0, size_t e0, int t) {
            std::vector<Ref> &LL = cL[t], &RR = cR[t];
            for (size_t k = b0; k < e0; ++k) {
                const Ref &r = refs[k];
                float a = r.b.mn[s.axis], b = r.b.mx[s.axis];
                if (b <= s.pos && !(a == b && b == s.pos)) {
                    LL.push_back(r);
                } else if (a >= s.pos) {
                    RR.push_back(r);
                } else {
                    Box cl = r.b, cr = r.b;
                    if (P.clip && (int) N >= P.clipMinPrims) {
                        cl = g.clipped(segIv[r.seg], r.b, lb);
                        cr = g.clipped(segIv[r.seg], r.b, rb);
                    } else {
                        cl.clip(lb);
                        cr.clip(rb);
                    }
                    if (cl.valid()) LL.push_back({r.seg, cl});
                    if (cr.valid()) RR.push_back({r.seg, cr});
                }
            }
        });
        std::vector<Ref> L, R;
        if (cL.size() == 1) {
            L.swap(cL[0]);
            R.swap(cR[0]);
        } else {
            size_t nl = 0, nr = 0;
            for (auto &v : cL) nl += v.size();
            for (auto &v : cR) nr += v.size();
            L.reserve(nl);
            R.reserve(nr);
            for (auto &v : cL) L.insert(L.end(), v.begin(), v.end());
            for (auto &v : cR) R.insert(R.end(), v.begin(), v.end());
        }
        std::vector<Ref>().swap(refs);
        node->axis = s.axis;
        node->split = s.pos;
        if (N > 20000 && depth < 6) {
            auto fut = std::async(std::launch::async, [&, lb, badRefines]() {
                return build(std::move(L), lb, depth + 1, badRefines);
            });
            node->kid[1] = build(std::move(R), rb, depth + 1, badRefines);
            node->kid[0] = fut.get();
        } else {
            node->kid[0] = build(std::move(L), lb, depth + 1, badRefines);
            node->kid[1] = build(std::move(R), rb, depth + 1, badRefines);
        }
        return node;
    }
};

/* Node layout: sibling pairs (16 B) packed into 128-byte blocks (one L2
 * line) treelet by treelet.  A block is filled breadth-first from a pair, so
 * a ray descending through the top three levels below it touches one line;
 * when a treelet ends before its block is full, the next pending treelet
 * continues in the same block (no padding).  Node 0 is the root, node 1 an
 * unused slot that keeps every pair 16-byte aligned. */
void layoutTreelets(const BNode *root, KDTreeHost &t) {
    const uint32_t kPairsPerBlock = 8;
    t.nodes.assign(2, HptNode{0x80000000u, 0u});
    struct Item {
        const BNode *n;
        uint32_t idx;
        int depth;
    };
    auto emit = [&](const Item &it) {
        t.maxDepthUsed = std::max(t.maxDepthUsed, it.depth);
        if (it.n->axis < 0) {
            uint32_t start = (uint32_t) t.prims.size();
            for (uint32_t p : it.n->prims) t.prims.push_back(p);
            BNode *ln = const_cast<BNode *>(it.n);
            ln->pStart = start;
            ln->pEnd = (uint32_t) t.prims.size();
            t.nodes[it.idx].w0 = 0x80000000u | start;
            t.nodes[it.idx].w1 = (uint32_t) t.prims.size();
            t.leaves++;
            if (it.n->prims.empty()) t.emptyLeaves++;
            return false;
        }
        return true;
    };
    std::vector<Item> pending; /* inner nodes whose child pair is not placed yet (FIFO) */
    size_t head = 0;
    if (emit({root, 0, 0})) pending.push_back({root, 0, 0});
    uint32_t used = 1; /* pairs used in the current block (slot 0 = root + pad) */
    while (head < pending.size()) {
        /* one treelet: breadth-first from pending[head] while the block has room */
        std::vector<Item> local{pending[head++]};
        size_t lh = 0;
        while (lh < local.size()) {
            if (used == kPairsPerBlock) {
                used = 0; /* block full: the rest of this treelet starts later blocks */
                for (size_t i = lh; i < local.size(); ++i) pending.push_back(local[i]);
                break;
            }
            const Item it = local[lh++];
            const uint32_t left = (uint32_t) t.nodes.size();
            if (left >= (1u << 29)) throw std::runtime_error("kd-tree too large");
            t.nodes.push_back({0, 0});
            t.nodes.push_back({0, 0});
            ++used;
            uint32_t sb;
            std::memcpy(&sb, &it.n->split, 4);
            t.nodes[it.idx].w0 = (left << 2) | (uint32_t) it.n->axis;
            t.nodes[it.idx].w1 = sb;
            for (int k = 0; k < 2; ++k) {
                Item c{it.n->kid[k].get(), left + (uint32_t) k, it.depth + 1};
                if (emit(c)) local.push_back(c);
            }
        }
        if (head > (1u << 20) && head * 2 > pending.size()) { /* compact the FIFO */
            pending.erase(pending.begin(), pending.begin() + (std::ptrdiff_t) head);
            head = 0;
        }
    }
}

/* Two-level node layout for the device traversal (HptNode4, hpt_device.h):
 * every node fuses a binary node with its two children, so one 32-byte fetch
 * advances the descent by two levels.  Built breadth-first from the binary
 * tree after layoutTreelets has assigned the leaves' primitive ranges. */
uint32_t leafRef(const BNode *n, KDTreeHost &t) {
    const uint32_t count = n->pEnd - n->pStart;
    if (count < HPT_LEAF_INLINE_MAX && n->pStart < (1u << 24)) return 0x80000000u | (count << 24) | n->pStart;
    const uint32_t idx = (uint32_t) t.leafTable.size() / 2;
    t.leafTable.push_back(n->pStart);
    t.leafTable.push_back(n->pEnd);
    return 0x80000000u | (HPT_LEAF_INLINE_MAX << 24) | idx;
}

void buildNode4(const BNode *root, KDTreeHost &t) {
    t.nodes4.clear();
    t.leafTable.clear();
    std::vector<const BNode *> queue;
    auto ref = [&](const BNode *n) -> uint32_t {
        if (n->axis < 0) return leafRef(n, t);
        queue.push_back(n);
        return (uint32_t) queue.size() - 1; /* node index = BFS position */
    };
    auto splitBits = [](float f) {
        uint32_t b;
        std::memcpy(&b, &f, 4);
        return b;
    };
    if (root->axis < 0) {
        /* single-leaf tree: a node whose top split sends every ray to one side */
        HptNode4 nd{};
        nd.w[0] = splitBits(std::numeric_limits<float>::infinity());
        nd.w[4] = nd.w[5] = nd.w[6] = nd.w[7] = leafRef(root, t);
        t.nodes4.push_back(nd);
        return;
    }
    queue.push_back(root);
    for (size_t qi = 0; qi < queue.size(); ++qi) {
        const BNode *n = queue[qi];
        HptNode4 nd{};
        nd.w[0] = splitBits(n->split);
        uint32_t flags = (uint32_t) n->axis;
        for (int k = 0; k < 2; ++k) {
            const BNode *c = n->kid[k].get();
            if (c->axis >= 0) {
                nd.w[1 + k] = splitBits(c->split);
                flags |= ((uint32_t) c->axis << (2 + 2 * k)) | (1u << (6 + k));
                nd.w[4 + 2 * k] = ref(c->kid[0].get());
                nd.w[5 + 2 * k] = ref(c->kid[1].get());
            } else {
                nd.w[4 + 2 * k] = nd.w[5 + 2 * k] = leafRef(c, t);
            }
        }
        nd.w[3] = flags;
        t.nodes4.push_back(nd);
    }
    if (t.leafTable.empty()) t.leafTable.push_back(0), t.leafTable.push_back(0);
}

/* HptSegQ's axis: oct encoding (u 16 bits, v 15 bits; bit 31 is the record's pass flag) of the
   fp64 axis, and its decode with the device's fp32 operations (axisOctDecode in hpt_render.hip) */
uint32_t axisOctEncode(const double a[3]) {
    const double l1 = std::fabs(a[0]) + std::fabs(a[1]) + std::fabs(a[2]);
    double u = a[0] / l1, v = a[1] / l1;
    if (a[2] < 0.0) {
        const double fu = (1.0 - std::fabs(v)) * (u >= 0.0 ? 1.0 : -1.0);
        const double fv = (1.0 - std::fabs(u)) * (v >= 0.0 ? 1.0 : -1.0);
        u = fu, v = fv;
    }
    auto q = [](double x, double m) { return (uint32_t) std::min(m, std::max(0.0, std::nearbyint((x * 0.5 + 0.5) * m))); };
    return q(u, 65535.0) | (q(v, 32767.0) << 16);
}
void axisOctDecode(uint32_t q, float &x, float &y, float &z) {
    const float u = (float) (q & 0xffffu) * (2.0f / 65535.0f) - 1.0f;
    const float v = (float) ((q >> 16) & 0x7fffu) * (2.0f / 32767.0f) - 1.0f;
    z = 1.0f - std::fabs(u) - std::fabs(v);
    x = u;
    y = v;
    if (z < 0.0f) {
        x = (1.0f - std::fabs(v)) * (u >= 0.0f ? 1.0f : -1.0f);
        y = (1.0f - std::fabs(u)) * (v >= 0.0f ? 1.0f : -1.0f);
    }
}

/* the radius bound that keeps the quantised-axis pre-test conservative: a point the exact test
   accepts lies within r of the axis line at an axial offset s from v1, s in [-r tan(phi1),
   len + r tan(phi2)] (phi = the angle between the axis and a miter plane's normal, hair.cpp:
   537-541), so it lies within r + |s| sin(theta) of the quantised line through v1 (theta = the
   angle between the two axes).  Returns r + max|s| sin(theta) for one segment. */
#define HPT_PASS_REACH 1.05
double quantisedReach(const HptSegment &g, double r, float ax, float ay, float az) {
    /* a NaN miter normal (a strand folding exactly back: the bisector of opposite tangents) fails
       both plane tests of hair.cpp:521-531, so the exact test never accepts the segment: NaN */
    for (int k = 0; k < 3; ++k)
        if (std::isnan(g.n1[k]) || std::isnan(g.n2[k])) return std::numeric_limits<double>::quiet_NaN();
    const double q[3] = {ax, ay, az};
    const double ql = std::sqrt(q[0] * q[0] + q[1] * q[1] + q[2] * q[2]);
    const double c[3] = {g.axis[1] * q[2] - g.axis[2] * q[1], g.axis[2] * q[0] - g.axis[0] * q[2],
                         g.axis[0] * q[1] - g.axis[1] * q[0]};
    const double sinTheta = std::sqrt(c[0] * c[0] + c[1] * c[1] + c[2] * c[2]) / ql;
    auto tanOf = [](const double n[3], const double a[3]) {
        const double cs = std::fabs(n[0] * a[0] + n[1] * a[1] + n[2] * a[2]);
        if (cs < 1e-9) return std::numeric_limits<double>::infinity();
        return std::sqrt(std::max(0.0, 1.0 - cs * cs)) / cs;
    };
    const double len = std::sqrt((g.v2[0] - g.v1[0]) * (g.v2[0] - g.v1[0]) + (g.v2[1] - g.v1[1]) * (g.v2[1] - g.v1[1]) +
                                 (g.v2[2] - g.v1[2]) * (g.v2[2] - g.v1[2]));
    const double reach = std::max(r * tanOf(g.n1, g.axis), len + r * tanOf(g.n2, g.axis));
    return sinTheta == 0.0 ? r : r + reach * sinTheta; /* an unturned axis: no widening, even for infinite reach */
}

} // namespace

KDTreeHost buildHairKDTree(const HairData &hair, const KDBuildParams &params) {
    auto t0 = std::chrono::steady_clock::now();
    KDTreeHost t;
    SegGeom g(hair);
    const size_t nv = hair.vertexCount();
    /* segment index list (hair.cpp:117-123) */
    std::vector<uint32_t> segIv;
    segIv.reserve(nv);
    for (size_t i = 0; i + 1 < nv; ++i)
        if (!hair.starts[i + 1]) segIv.push_back((uint32_t) i);
    const size_t S = segIv.size();
    t.segFirstVertex = segIv;

    /* double-precision per-segment records (hair.cpp:551-596) */
    t.segs.resize(S);
    for (size_t s = 0; s < S; ++s) {
        uint32_t iv = segIv[s];
        auto vd = [&](uint32_t i) {
            return std::array<double, 3>{(double) hair.xyz[3 * i], (double) hair.xyz[3 * i + 1],
                                         (double) hair.xyz[3 * i + 2]};
        };
        auto nrmd = [](std::array<double, 3> v) {
            double l = std::sqrt(v[0] * v[0] + v[1] * v[1] + v[2] * v[2]);
            double r = 1.0 / l;
            return std::array<double, 3>{v[0] * r, v[1] * r, v[2] * r};
        };
        auto subd = [](std::array<double, 3> a, std::array<double, 3> b) {
            return std::array<double, 3>{a[0] - b[0], a[1] - b[1], a[2] - b[2]};
        };
        auto addd = [](std::array<double, 3> a, std::array<double, 3> b) {
            return std::array<double, 3>{a[0] + b[0], a[1] + b[1], a[2] + b[2]};
        };
        auto v1 = vd(iv), v2 = vd(iv + 1);
        auto axis = nrmd(subd(v2, v1));
        std::array<double, 3> n1 = axis, n2 = axis;
        if (!hair.starts[iv]) n1 = nrmd(addd(nrmd(subd(v1, vd(iv - 1))), axis));
        if (!hair.starts[iv + 2]) n2 = nrmd(addd(axis, nrmd(subd(vd(iv + 2), v2))));
        HptSegment &r = t.segs[s];
        for (int k = 0; k < 3; ++k) {
            r.v1[k] = v1[k];
            r.axis[k] = axis[k];
            r.n1[k] = n1[k];
            r.n2[k] = n2[k];
            r.v2[k] = v2[k];
        }
        r.iv = iv;
        r.shape = hair.shapeOf(iv);
    }

    /* primitive bounds + tree AABB (gkdtree.h:990-994) */
    std::vector<Ref> refs(S);
    Box root;
    {
        const int hw0 = params.threads > 0 ? params.threads : (int) std::max(1u, std::thread::hardware_concurrency());
        parallelChunks(S, std::min(hw0, 64), 1u << 14, [&](size_t b0, size_t e0, int) {
            for (size_t s = b0; s < e0; ++s) {
                refs[s].seg = (uint32_t) s;
                refs[s].b = g.aabb(segIv[s]);
            }
        });
        for (size_t s = 0; s < S; ++s) root.expand(refs[s].b);
    }
    for (int i = 0; i < 3; ++i) {
        t.aabbMin[i] = root.mn[i];
        t.aabbMax[i] = root.mx[i];
    }
    if (S == 0) {
        t.nodes.push_back({0x80000000u, 0});
        t.leaves = 1;
        /* the two-level form too (every traversal kernel reads it): one empty leaf behind a
           split that sends every ray to it, like buildNode4's single-leaf tree; the empty
           box above does not stop rays (its slabs are [-inf, inf]) */
        HptNode4 nd{};
        const float inf = std::numeric_limits<float>::infinity();
        std::memcpy(&nd.w[0], &inf, 4);
        nd.w[4] = nd.w[5] = nd.w[6] = nd.w[7] = 0x80000000u;
        t.nodes4.push_back(nd);
        t.leafTable.push_back(0), t.leafTable.push_back(0);
        return t;
    }
    int lg = 0;
    while ((S >> (lg + 1)) != 0) lg++;
    const int autoDepth = std::min((int) (8 + 1.3f * lg), 48);
    const int hw = params.threads > 0 ? params.threads : (int) std::max(1u, std::thread::hardware_concurrency());
    Builder b{g, segIv, params, params.maxDepth > 0 ? std::min(params.maxDepth, 64) : autoDepth, std::min(hw, 64)};
    auto tb = std::chrono::steady_clock::now();
    std::unique_ptr<BNode> tree = b.build(std::move(refs), root, 0, 0);
    auto tl = std::chrono::steady_clock::now();
    t.nodes.reserve(2 * S);
    layoutTreelets(tree.get(), t);
    /* each segment's pre-test bound on its 16-byte record (quantisedReach) */
    std::vector<double> segBound(S);
    std::vector<float> segRad(S);
    for (size_t s = 0; s < S; ++s) {
        float x, y, z;
        axisOctDecode(axisOctEncode(t.segs[s].axis), x, y, z);
        segRad[s] = hair.radiusOf(segIv[s]);
        segBound[s] = quantisedReach(t.segs[s], (double) segRad[s], x, y, z);
    }
    buildNode4(tree.get(), t);
    if (std::getenv("HPT_KD_TIMING"))
        std::fprintf(stderr, "kd: bounds %.3f s, build %.3f s, layout %.3f s\n",
                     std::chrono::duration<double>(tb - t0).count(), std::chrono::duration<double>(tl - tb).count(),
                     std::chrono::duration<double>(std::chrono::steady_clock::now() - tl).count());
    /* leaf-ordered fp32 pre-test records */
    t.leafF.resize(t.prims.size());
    for (size_t e = 0; e < t.prims.size(); ++e) {
        const uint32_t s = t.prims[e];
        HptSegF &f = t.leafF[e];
        for (int k = 0; k < 3; ++k) {
            f.v1[k] = hair.xyz[3 * segIv[s] + k];
            f.axis[k] = (float) t.segs[s].axis[k];
        }
        f.seg = s;
        f.radius = hair.radiusOf(segIv[s]);
    }
    /* the 16-byte records.  A record whose bound exceeds its shape's radius by more than
       HPT_PASS_REACH -- a fold: a miter plane almost parallel to the axis, a bound of hundreds of
       radii or none at all -- is flagged to pass every pre-test (its exact test decides), and the
       scene's pre-test radius is the largest bound of the others: a fold no longer widens the
       test of every record.  (A NaN bound -- a NaN miter normal, which no exact test accepts,
       hair.cpp:521-531 -- needs neither.)  A 1e-5 relative slack covers the fp32 rounding of the
       radius itself and of the device's decode. */
    t.leafQ.resize(t.prims.size());
    double preBound = 0.0;
    t.prePassRecords = 0;
    for (size_t e = 0; e < t.prims.size(); ++e) {
        const uint32_t s = t.prims[e];
        HptSegQ &q = t.leafQ[e];
        for (int k = 0; k < 3; ++k) q.v1[k] = t.leafF[e].v1[k];
        q.axisOct = axisOctEncode(t.segs[s].axis);
        const double b = segBound[s];
        if (std::isnan(b)) continue;
        if (b > HPT_PASS_REACH * segRad[s]) {
            q.axisOct |= HPT_PRE_PASS;
            ++t.prePassRecords;
        } else {
            preBound = std::max(preBound, b);
        }
    }
    t.preRadius = (float) (preBound * (1.0 + 1e-5));
    t.buildSeconds = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
    return t;
}

} // namespace hpt
