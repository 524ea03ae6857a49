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
 *   - 'reduction' stochastically drops strands and enlarges the radius
 *     (:618-629) -- supported only for reduction == 0 here (the reference's
 *     culling draws from an unseeded Random, so it is not reproducible);
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

HairData loadHair(const std::string &path, float radius, float angleThresholdDeg, float reduction,
                  const float *toWorld) {
    if (reduction < 0 || reduction >= 1)
        throw std::runtime_error("The 'reduction' parameter must have a value in [0, 1)!");
    if (reduction > 0)
        throw std::runtime_error("hair 'reduction' > 0 is not supported (unseeded culling in the reference)");
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

    HairData out;
    Builder b{out.xyz, out.starts, dpThresh};
    if (buf.size() >= 11 && std::memcmp(buf.data(), "BINARY_HAIR", 11) == 0) {
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
            } else {
                p.x = value;
                p.y = rd();
                p.z = rd();
            }
            if (!identity) p = xform(toWorld, p);
            b.add(p, newFiber);
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
                b.add(p, newFiber);
            } else {
                newFiber = true;
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
