/*
 * hair_io.cpp -- hair strand loader (binary BINARY_HAIR and ASCII formats).
 *
 * Semantics follow HairShape::HairShape (src/shapes/hair.cpp:609-785):
 *   - BINARY_HAIR: 11-byte magic, uint32 vertex count, float xyz triples; a
 *     single +inf value before a vertex starts a new strand (:656-716);
 *   - ASCII: one vertex per line, blank line or '#' line starts a strand (:717-772);
 *   - consecutive vertices whose tangent changes by less than angleThreshold
 *     degrees are merged into one segment (:615-616, :698-705);
 *   - coincident vertices are dropped as degenerate (:706-708);
 *   - 'reduction' drops each strand with probability `reduction` and scales the
 *     radius by 1 / (1 - reduction) (:618-629, :671-673, :768-770).  The draws
 *     come from `new Random()`, which on Linux seeds SFMT19937 with the default
 *     5489 (random.cpp:473-489, random.h:113) -- deterministic, so the same
 *     strands are dropped as in the reference: Sfmt19937 below restates it;
 *   - toWorld is applied to vertices and scales the radius (:632-633).
 */
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"

namespace hpt {
namespace {

struct P3 {
    float x, y, z;
    bool operator!=(const P3 &o) const { return x != o.x || y != o.y || z != o.z; }
};

inline P3 sub(const P3 &a, const P3 &b) { return {a.x - b.x, a.y - b.y, a.z - b.z}; }
inline P3 nrm(const P3 &v) {
    float len = std::sqrt(v.x * v.x + v.y * v.y + v.z * v.z);
    float r = 1.0f / len;
    return {v.x * r, v.y * r, v.z * r};
}
inline float dot3(const P3 &a, const P3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }

struct Builder {
    std::vector<float> &xyz;
    std::vector<uint8_t> &starts;
    float dpThresh;
    P3 tangent{0, 0, 0}, lastP{0, 0, 0};
    size_t nDegenerate = 0, nSkipped = 0;
    size_t count() const { return xyz.size() / 3; }
    P3 vtx(size_t i) const { return {xyz[3 * i], xyz[3 * i + 1], xyz[3 * i + 2]}; }
    void push(const P3 &p, bool start) {
        xyz.push_back(p.x);
        xyz.push_back(p.y);
        xyz.push_back(p.z);
        starts.push_back(start ? 1 : 0);
    }
    void add(const P3 &p, bool &newFiber) {
        if (newFiber) {
            push(p, true);
            lastP = p;
            tangent = {0, 0, 0};
        } else if (p != lastP) {
            if (tangent.x == 0 && tangent.y == 0 && tangent.z == 0) {
                push(p, false);
                tangent = nrm(sub(p, lastP));
                lastP = p;
            } else {
                P3 nextTangent = nrm(sub(p, lastP));
                if (dot3(nextTangent, tangent) > dpThresh) {
                    size_t n = count();
                    tangent = nrm(sub(p, vtx(n - 2)));
                    xyz[3 * (n - 1)] = p.x;
                    xyz[3 * (n - 1) + 1] = p.y;
                    xyz[3 * (n - 1) + 2] = p.z;
                    ++nSkipped;
                } else {
                    push(p, false);
                    tangent = nextTangent;
                }
                lastP = p;
            }
        } else {
            nDegenerate++;
        }
        newFiber = false;
    }
};

/* SFMT19937 as Random (src/libcore/random.cpp): init_gen_rand (:397-406, the
   64-bit LCG fill + period certification), gen_rand_all over 128-bit words
   (:330-360; the SSE recursion of :170-186 computes the same words as the
   portable one), gen_rand64 (:296-304) and the single-precision nextFloat
   (:630-640: the low 32 bits of a 64-bit output, >> 9 into [1, 2), minus 1). */
class Sfmt19937 {
    static const int kN = 19937 / 128 + 1, kN32 = kN * 4, kN64 = kN * 2, kPos1 = 122;
    static const int kSL1 = 18, kSL2 = 1, kSR1 = 11, kSR2 = 1;
    uint32_t st[kN32];
    int idx;

    /* 128-bit word k of the state (little-endian: st[4k] is the low 32 bits) */
    static void shl8(const uint32_t *in, uint32_t *out, int bytes) {
        uint64_t lo = (uint64_t) in[0] | ((uint64_t) in[1] << 32), hi = (uint64_t) in[2] | ((uint64_t) in[3] << 32);
        uint64_t oh = (hi << (bytes * 8)) | (lo >> (64 - bytes * 8)), ol = lo << (bytes * 8);
        out[0] = (uint32_t) ol, out[1] = (uint32_t) (ol >> 32), out[2] = (uint32_t) oh, out[3] = (uint32_t) (oh >> 32);
    }
    static void shr8(const uint32_t *in, uint32_t *out, int bytes) {
        uint64_t lo = (uint64_t) in[0] | ((uint64_t) in[1] << 32), hi = (uint64_t) in[2] | ((uint64_t) in[3] << 32);
        uint64_t ol = (lo >> (bytes * 8)) | (hi << (64 - bytes * 8)), oh = hi >> (bytes * 8);
        out[0] = (uint32_t) ol, out[1] = (uint32_t) (ol >> 32), out[2] = (uint32_t) oh, out[3] = (uint32_t) (oh >> 32);
    }
    void recursion(int r, int a, int b, int c, int d) {
        static const uint32_t msk[4] = {0xdfffffefu, 0xddfecb7fu, 0xbffaffffu, 0xbffffff6u};
        uint32_t x[4], y[4], out[4];
        shl8(&st[4 * a], x, kSL2);
        shr8(&st[4 * c], y, kSR2);
        for (int i = 0; i < 4; ++i)
            out[i] = st[4 * a + i] ^ x[i] ^ ((st[4 * b + i] >> kSR1) & msk[i]) ^ y[i] ^ (st[4 * d + i] << kSL1);
        std::memcpy(&st[4 * r], out, sizeof(out));
    }
    void genAll() {
        int r1 = kN - 2, r2 = kN - 1, i = 0;
        for (; i < kN - kPos1; ++i) {
            recursion(i, i, i + kPos1, r1, r2);
            r1 = r2;
            r2 = i;
        }
        for (; i < kN; ++i) {
            recursion(i, i, i + kPos1 - kN, r1, r2);
            r1 = r2;
            r2 = i;
        }
    }

public:
    explicit Sfmt19937(uint64_t seed = 5489ull) {
        uint64_t v = seed;
        for (int i = 0; i < kN64; ++i) {
            if (i) v = 6364136223846793005ull * (v ^ (v >> 62)) + (uint64_t) i;
            st[2 * i] = (uint32_t) v;
            st[2 * i + 1] = (uint32_t) (v >> 32);
        }
        idx = kN32;
        /* period certification (parity 0x1, 0, 0, 0x13c9e684) */
        static const uint32_t parity[4] = {0x00000001u, 0u, 0u, 0x13c9e684u};
        uint32_t inner = 0;
        for (int i = 0; i < 4; ++i) inner ^= st[i] & parity[i];
        for (int i = 16; i > 0; i >>= 1) inner ^= inner >> i;
        if (!(inner & 1u)) {
            for (int i = 0; i < 4; ++i)
                for (int j = 0; j < 32; ++j)
                    if (((1u << j) & parity[i]) != 0) {
                        st[i] ^= 1u << j;
                        return;
                    }
        }
    }
    uint64_t nextULong() {
        if (idx >= kN32) {
            genAll();
            idx = 0;
        }
        const uint64_t r = (uint64_t) st[idx] | ((uint64_t) st[idx + 1] << 32);
        idx += 2;
        return r;
    }
    float nextFloat() {
        uint32_t u = ((uint32_t) (nextULong() & 0xFFFFFFFFull) >> 9) | 0x3f800000u;
        float f;
        std::memcpy(&f, &u, 4);
        return f - 1.0f;
    }
};

inline P3 xform(const float *M, const P3 &p) {
    /* transform.h:108-125 (projective point transform) */
    float x = M[0] * p.x + M[1] * p.y + M[2] * p.z + M[3];
    float y = M[4] * p.x + M[5] * p.y + M[6] * p.z + M[7];
    float z = M[8] * p.x + M[9] * p.y + M[10] * p.z + M[11];
    float w = M[12] * p.x + M[13] * p.y + M[14] * p.z + M[15];
    if (w == 1.0f) return {x, y, z};
    float r = 1.0f / w;
    return {x * r, y * r, z * r};
}

} // namespace

void sfmtULongs(uint64_t seed, size_t n, uint64_t *out) {
    Sfmt19937 r(seed);
    for (size_t i = 0; i < n; ++i) out[i] = r.nextULong();
}

HairData loadHair(const std::string &path, float radius, float angleThresholdDeg, float reduction,
                  const float *toWorld) {
    if (reduction < 0 || reduction >= 1)
        throw std::runtime_error("The 'reduction' parameter must have a value in [0, 1)!");
    if (reduction > 0) radius *= 1.0f / (1 - reduction); /* hair.cpp:622-626 */
    Sfmt19937 random;                                     /* hair.cpp:628: new Random() */
    bool ignore = false;
    bool identity = true;
    if (toWorld)
        for (int i = 0; i < 16; ++i) identity &= toWorld[i] == ((i % 5 == 0) ? 1.0f : 0.0f);
    if (!identity) {
        float vx = toWorld[2], vy = toWorld[6], vz = toWorld[10];
        radius *= std::sqrt(vx * vx + vy * vy + vz * vz);
    }
    const float kPi = 3.14159265358979323846f;
    float angleThreshold = angleThresholdDeg * (kPi / 180.0f);
    float dpThresh = std::cos(angleThreshold);

    std::ifstream f(path, std::ios::binary);
    if (!f) throw std::runtime_error("cannot open hair file \"" + path + "\"");
    std::vector<char> buf((std::istreambuf_iterator<char>(f)), std::istreambuf_iterator<char>());

    /* the reference reads an 11-byte header before deciding the format (hair.cpp:641-646);
       FileStream::read throws on a shorter file (fstream.cpp:317-327), ASCII or not */
    if (buf.size() < 11) throw std::runtime_error("truncated hair file \"" + path + "\" (shorter than the 11-byte header)");
    HairData out;
    Builder b{out.xyz, out.starts, dpThresh};
    if (std::memcmp(buf.data(), "BINARY_HAIR", 11) == 0) {
        if (buf.size() < 15) throw std::runtime_error("truncated hair file \"" + path + "\"");
        uint32_t vertexCount;
        std::memcpy(&vertexCount, buf.data() + 11, 4);
        out.xyz.reserve((size_t) vertexCount * 3);
        out.starts.reserve(vertexCount + 1);
        const char *ptr = buf.data() + 15, *end = buf.data() + buf.size();
        auto rd = [&]() -> float {
            if (ptr + 4 > end) throw std::runtime_error("truncated hair file \"" + path + "\"");
            float v;
            std::memcpy(&v, ptr, 4);
            ptr += 4;
            return v;
        };
        bool newFiber = true;
        for (uint32_t read = 0; read != vertexCount; ++read) {
            float value = rd();
            P3 p;
            if (std::isinf(value)) {
                p.x = rd();
                p.y = rd();
                p.z = rd();
                newFiber = true;
                if (reduction > 0) ignore = random.nextFloat() < reduction; /* hair.cpp:671-673 */
            } else {
                p.x = value;
                p.y = rd();
                p.z = rd();
            }
            if (!identity) p = xform(toWorld, p);
            if (ignore) { /* hair.cpp:683-685 */
                ++b.nSkipped;
                newFiber = false;
            } else {
                b.add(p, newFiber);
            }
        }
    } else {
        std::string text(buf.begin(), buf.end());
        std::istringstream is(text);
        std::string line;
        bool newFiber = true;
        while (is.good()) {
            std::getline(is, line);
            if (line.length() > 0 && line[0] == '#') {
                newFiber = true;
                continue;
            }
            std::istringstream iss(line);
            P3 p;
            iss >> p.x >> p.y >> p.z;
            if (!iss.fail()) {
                if (!identity) p = xform(toWorld, p);
                if (ignore) { /* hair.cpp:734-736 */
                    ++b.nSkipped;
                    newFiber = false;
                } else {
                    b.add(p, newFiber);
                }
            } else {
                newFiber = true;
                if (reduction > 0) ignore = random.nextFloat() < reduction; /* hair.cpp:768-770 */
            }
        }
    }
    out.starts.push_back(1);
    out.radius = radius;
    out.shapeRadius = {radius};
    out.nDegenerate = b.nDegenerate;
    out.nSkipped = b.nSkipped;
    return out;
}

void appendHair(HairData &a, const HairData &b) {
    /* several HairShapes in one scene (ShapeKDTree over shapes, skdtree.cpp):
       concatenated vertex arrays; a shape's first vertex always starts a
       fiber, so no segment or miter spans two shapes */
    if (a.shapeRadius.empty()) {
        a = b;
        if (a.shapeRadius.empty()) a.shapeRadius = {a.radius};
        a.shapeFirst = {0};
        return;
    }
    const uint32_t base = (uint32_t) a.vertexCount();
    a.xyz.insert(a.xyz.end(), b.xyz.begin(), b.xyz.end());
    a.starts.pop_back(); /* a's terminator */
    a.starts.insert(a.starts.end(), b.starts.begin(), b.starts.end());
    if (b.vertexCount()) a.starts[base] = 1;
    a.shapeFirst.push_back(base);
    a.shapeRadius.push_back(b.radius);
    a.nDegenerate += b.nDegenerate;
    a.nSkipped += b.nSkipped;
}

} // namespace hpt
