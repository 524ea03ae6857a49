/*
 * mesh.cpp -- host side of the triangle-mesh scenes (C1, models/teapot/scene.xml:31-84):
 * the shapes are loaded and flattened into world-space arrays for k_mesh_paths.
 *
 *   Wavefront OBJ          src/shapes/obj.cpp:165-186 (fetch_line), 199-349 (loader: one TriMesh
 *                          per g / usemtl group), 371-390 (face vertex), 577-715 (vertex merge)
 *   TriMesh::configure     src/librender/trimesh.cpp:362-386; computeNormals :608-681;
 *                          computeUVTangents :683-743; unitAngle core/util.h:309-314
 *   TriAccel::load         include/mitsuba/render/triaccel.h:37-70 (per triangle, skdtree.cpp:88-95)
 *   Rectangle              src/shapes/rectangle.cpp:80-122
 *   scene bounds           include/mitsuba/render/gkdtree.h:1213-1220 (MTS_KD_AABB_EPSILON)
 *   BSDFs                  diffuse.cpp:60-140 (+ checkerboard.cpp:47-100), plastic.cpp:143-217,
 *                          twosided.cpp:58-110; fresnelDiffuseReflectance util.cpp:808-859 over
 *                          GaussLobattoIntegrator quad.cpp:287-409
 *
 * The acceleration structure is our own (a BVH of 32-byte nodes, median splits on the
 * widest centroid axis); the closest hit does not depend on it up to exact ties in t, since
 * every primitive test runs against the running [mint, maxt] (sahkdtree3.h).
 */
#include <algorithm>
#include <cmath>
#include <cstring>
#include <fstream>
#include <functional>
#include <limits>
#include <map>
#include <sstream>
#include <stdexcept>
#include <string>
#include <vector>

#include "host_scene.h"

namespace hpt {
namespace {

const float kPiF = 3.14159265358979323846f;
const float kEps = 1e-4f; /* constants.h:28 */

struct F3 {
    float x = 0, y = 0, z = 0;
    F3() = default;
    F3(float a, float b, float c) : x(a), y(b), z(c) {}
    float operator[](int i) const { return i == 0 ? x : (i == 1 ? y : z); }
    F3 operator+(const F3 &o) const { return F3(x + o.x, y + o.y, z + o.z); }
    F3 operator-(const F3 &o) const { return F3(x - o.x, y - o.y, z - o.z); }
    F3 operator-() const { return F3(-x, -y, -z); }
    F3 operator*(float f) const { return F3(x * f, y * f, z * f); }
    F3 operator/(float f) const { const float r = 1.0f / f; return F3(x * r, y * r, z * r); } /* vector.h:546-564 */
    bool isZero() const { return x == 0 && y == 0 && z == 0; }
    float length() const { return std::sqrt(x * x + y * y + z * z); }
};
F3 operator*(float f, const F3 &v) { return v * f; }
float dot(const F3 &a, const F3 &b) { return a.x * b.x + a.y * b.y + a.z * b.z; }
F3 cross(const F3 &a, const F3 &b) { return F3(a.y * b.z - a.z * b.y, a.z * b.x - a.x * b.z, a.x * b.y - a.y * b.x); }
F3 normalize(const F3 &v) { return v / v.length(); }

/* Transform(Matrix4x4) application (transform.h:108-125 points, :175-183 vectors, :203-211
   normals through the inverse's transpose) */
F3 xfPoint(const float *M, const F3 &p) {
    const float x = M[0] * p.x + M[1] * p.y + M[2] * p.z + M[3];
    const float y = M[4] * p.x + M[5] * p.y + M[6] * p.z + M[7];
    const float z = M[8] * p.x + M[9] * p.y + M[10] * p.z + M[11];
    const float w = M[12] * p.x + M[13] * p.y + M[14] * p.z + M[15];
    if (w == 1.0f) return F3(x, y, z);
    return F3(x, y, z) / w;
}
F3 xfVector(const float *M, const F3 &v) {
    return F3(M[0] * v.x + M[1] * v.y + M[2] * v.z, M[4] * v.x + M[5] * v.y + M[6] * v.z,
              M[8] * v.x + M[9] * v.y + M[10] * v.z);
}
F3 xfNormal(const float *inv, const F3 &v) {
    return F3(inv[0] * v.x + inv[4] * v.y + inv[8] * v.z, inv[1] * v.x + inv[5] * v.y + inv[9] * v.z,
              inv[2] * v.x + inv[6] * v.y + inv[10] * v.z);
}
void matMul(const float *a, const float *b, float *r) { /* matrix.h:743-756: sum += a_ik b_kj */
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float s = 0;
            for (int k = 0; k < 4; ++k) s += a[i * 4 + k] * b[k * 4 + j];
            r[i * 4 + j] = s;
        }
}

/* util.cpp:592-601 */
void coordinateSystem(const F3 &a, F3 &b, F3 &c) {
    if (std::abs(a.x) > std::abs(a.y)) {
        const float invLen = 1.0f / std::sqrt(a.x * a.x + a.z * a.z);
        c = F3(a.z * invLen, 0.0f, -a.x * invLen);
    } else {
        const float invLen = 1.0f / std::sqrt(a.y * a.y + a.z * a.z);
        c = F3(0.0f, a.z * invLen, -a.y * invLen);
    }
    b = cross(c, a);
}

/* ---------------- GaussLobattoIntegrator (quad.cpp:287-409), Float = float ---------------- */
class Lobatto {
public:
    Lobatto(size_t maxEvals, float absErr, float relErr) : maxEvals_(maxEvals), abs_(absErr), rel_(relErr) {}
    float integrate(const std::function<float(float)> &f, float a, float b) const {
        if (a == b) return 0;
        float sign = 1;
        if (b < a) std::swap(a, b), sign = -1;
        size_t evals = 0;
        const float tol = tolerance(f, a, b, evals);
        evals += 2;
        return sign * step(f, a, b, f(a), f(b), tol, evals);
    }

private:
    size_t maxEvals_;
    float abs_, rel_;
    static float alpha() { return (float) std::sqrt(2.0 / 3.0); }
    static float beta() { return (float) (1.0 / std::sqrt(5.0)); }
    /* :325-369 with useConvergenceEstimate (the constructor default, quad.h:158) */
    float tolerance(const std::function<float(float)> &f, float a, float b, size_t &evals) const {
        const float m = (a + b) / 2, h = (b - a) / 2;
        const float x1 = (float) 0.94288241569547971906, x2 = (float) 0.64185334234578130578,
                    x3 = (float) 0.23638319966214988028;
        const float y1 = f(a), y3 = f(m - alpha() * h), y5 = f(m - beta() * h), y7 = f(m), y9 = f(m + beta() * h),
                    y11 = f(m + alpha() * h), y13 = f(b);
        const float acc = h * ((float) 0.0158271919734801831 * (y1 + y13) +
                               (float) 0.0942738402188500455 * (f(m - x1 * h) + f(m + x1 * h)) +
                               (float) 0.1550719873365853963 * (y3 + y11) +
                               (float) 0.1888215739601824544 * (f(m - x2 * h) + f(m + x2 * h)) +
                               (float) 0.1997734052268585268 * (y5 + y9) +
                               (float) 0.2249264653333395270 * (f(m - x3 * h) + f(m + x3 * h)) +
                               (float) 0.2426110719014077338 * y7);
        evals += 13;
        const float i2 = (h / 6) * (y1 + y13 + 5 * (y5 + y9));
        const float i1 = (h / 1470) * (77 * (y1 + y13) + 432 * (y3 + y11) + 625 * (y5 + y9) + 672 * y7);
        float r = 1.0f;
        if (std::abs(i2 - acc) != 0.0) r = std::abs(i1 - acc) / std::abs(i2 - acc);
        if (r == 0.0 || r > 1.0) r = 1.0f;
        const float eps = std::numeric_limits<float>::epsilon();
        float out = std::numeric_limits<float>::infinity();
        if (rel_ != 0 && acc != 0) out = acc * std::max(rel_, eps) / (r * eps);
        if (abs_ != 0) out = std::min(out, abs_ / (r * eps));
        return out;
    }
    /* :371-409 */
    float step(const std::function<float(float)> &f, float a, float b, float fa, float fb, float acc,
               size_t &evals) const {
        const float h = (b - a) / 2, m = (a + b) / 2;
        const float mll = m - alpha() * h, ml = m - beta() * h, mr = m + beta() * h, mrr = m + alpha() * h;
        const float fmll = f(mll), fml = f(ml), fm = f(m), fmr = f(mr), fmrr = f(mrr);
        const float i2 = (h / 6) * (fa + fb + 5 * (fml + fmr));
        const float i1 = (h / 1470) * (77 * (fa + fb) + 432 * (fmll + fmrr) + 625 * (fml + fmr) + 672 * fm);
        evals += 5;
        if (evals >= maxEvals_) return i1;
        const float dist = acc + (i1 - i2);
        if (dist == acc || mll <= a || b <= mrr) return i1;
        return step(f, a, mll, fa, fmll, acc, evals) + step(f, mll, ml, fmll, fml, acc, evals) +
               step(f, ml, m, fml, fm, acc, evals) + step(f, m, mr, fm, fmr, acc, evals) +
               step(f, mr, mrr, fmr, fmrr, acc, evals) + step(f, mrr, b, fmrr, fb, acc, evals);
    }
};

/* util.cpp:651-681 (fresnelDielectricExt with the two-argument wrapper, util.h:479-480) */
float fresnelDielectricExt(float cosThetaI, float eta) {
    if (eta == 1) return 0.0f;
    const float scale = (cosThetaI > 0) ? 1 / eta : eta, cosThetaTSqr = 1 - (1 - cosThetaI * cosThetaI) * (scale * scale);
    if (cosThetaTSqr <= 0.0f) return 1.0f;
    const float cI = std::abs(cosThetaI), cT = std::sqrt(cosThetaTSqr);
    const float Rs = (cI - eta * cT) / (cI + eta * cT), Rp = (eta * cI - cT) / (eta * cI + cT);
    return 0.5f * (Rs * Rs + Rp * Rp);
}

/* ---------------- TriMesh (trimesh.cpp) ---------------- */
struct Mesh {
    std::vector<F3> p, n;      /* n empty: face normals */
    std::vector<float> uv;     /* 2 per vertex, empty: none */
    std::vector<uint32_t> idx; /* 3 per triangle */
    int bsdf = 0;
    size_t triangles() const { return idx.size() / 3; }
};

float unitAngle(const F3 &u, const F3 &v) { /* util.h:309-314 */
    if (dot(u, v) < 0) return kPiF - 2 * std::asin(0.5f * (v + u).length());
    return 2 * std::asin(0.5f * (v - u).length());
}

/* trimesh.cpp:608-681: angle-weighted vertex normals unless the file gave them */
void computeNormals(Mesh &m, bool faceNormals, bool flipNormals, bool hasNormals) {
    if (faceNormals) {
        m.n.clear();
        if (flipNormals)
            for (size_t i = 0; i < m.triangles(); ++i) std::swap(m.idx[3 * i], m.idx[3 * i + 1]);
        return;
    }
    if (hasNormals) {
        if (flipNormals)
            for (F3 &n : m.n) n = n * -1.0f;
        return;
    }
    m.n.assign(m.p.size(), F3());
    for (size_t i = 0; i < m.triangles(); ++i) {
        F3 n;
        for (int j = 0; j < 3; ++j) {
            const F3 &v0 = m.p[m.idx[3 * i + j]], &v1 = m.p[m.idx[3 * i + (j + 1) % 3]],
                     &v2 = m.p[m.idx[3 * i + (j + 2) % 3]];
            const F3 sideA = v1 - v0, sideB = v2 - v0;
            if (j == 0) {
                n = cross(sideA, sideB);
                const float length = n.length();
                if (length == 0) break;
                n = n / length;
            }
            const float angle = unitAngle(normalize(sideA), normalize(sideB));
            m.n[m.idx[3 * i + j]] = m.n[m.idx[3 * i + j]] + n * angle;
        }
    }
    for (F3 &n : m.n) {
        float length = n.length();
        if (flipNormals) length *= -1;
        n = length != 0 ? n / length : F3(1, 0, 0);
    }
}

/* ---------------- Wavefront OBJ (obj.cpp) ---------------- */
struct Face {
    int p[3] = {0, 0, 0}, uv[3] = {0, 0, 0}, n[3] = {0, 0, 0};
};

bool fetchLine(std::istream &is, std::string &line) { /* obj.cpp:165-186: trailing '\' joins lines */
    if (!std::getline(is, line)) return false;
    if (line.empty()) return true;
    int last = (int) line.size() - 1;
    while (last >= 0 && (line[last] == '\r' || line[last] == '\n' || line[last] == '\t' || line[last] == ' ')) last--;
    if (last >= 0 && line[last] == '\\') {
        std::string next;
        fetchLine(is, next);
        line = line.substr(0, last) + next;
    } else {
        line.resize(last + 1);
    }
    return true;
}

void parseFaceVertex(Face &f, int i, const std::string &s) { /* obj.cpp:371-390 (tokenize drops empty tokens) */
    std::vector<std::string> tok;
    size_t a = s.find_first_not_of('/'), b = s.find_first_of('/', a);
    while (b != std::string::npos || a != std::string::npos) {
        tok.push_back(s.substr(a, b - a));
        a = s.find_first_not_of('/', b);
        b = s.find_first_of('/', a);
    }
    switch (tok.size()) {
    case 1: f.p[i] = std::atoi(tok[0].c_str()); break;
    case 2:
        f.p[i] = std::atoi(tok[0].c_str());
        if (s.find("//") == std::string::npos) f.uv[i] = std::atoi(tok[1].c_str());
        else f.n[i] = std::atoi(tok[1].c_str());
        break;
    case 3:
        f.p[i] = std::atoi(tok[0].c_str());
        f.uv[i] = std::atoi(tok[1].c_str());
        f.n[i] = std::atoi(tok[2].c_str());
        break;
    default: throw std::runtime_error("Invalid OBJ face format!");
    }
}

struct MergedVertex { /* obj.cpp:577-606: vertices merged on (p, n, uv) */
    F3 p, n;
    float u = 0, v = 0;
    bool operator<(const MergedVertex &o) const {
        const float a[8] = {p.x, p.y, p.z, n.x, n.y, n.z, u, v}, b[8] = {o.p.x, o.p.y, o.p.z, o.n.x, o.n.y, o.n.z, o.u, o.v};
        for (int i = 0; i < 8; ++i) {
            if (a[i] < b[i]) return true;
            if (a[i] > b[i]) return false;
        }
        return false;
    }
};

/* obj.cpp:608-715 createMesh, then TriMesh::configure's normals (computeUVTangents is the
   caller's, per triangle into the flat arrays) */
void createMesh(const std::vector<F3> &vertices, const std::vector<F3> &normals, const std::vector<float> &texcoords,
                const std::vector<Face> &faces, const float *toWorld, const float *toWorldInv,
                const MeshShapeDesc &sd, std::vector<Mesh> &out) {
    if (faces.empty()) return;
    std::map<MergedVertex, uint32_t> merged;
    std::vector<MergedVertex> buf;
    Mesh m;
    bool hasUV = false, hasNormals = false;
    const int nv = (int) vertices.size(), nn = (int) normals.size(), nt = (int) texcoords.size() / 2;
    for (const Face &f : faces)
        for (int j = 0; j < 3; ++j) {
            int vi = f.p[j], ni = f.n[j], ti = f.uv[j];
            if (vi < 0) vi += nv + 1;
            if (ni < 0) ni += nn + 1;
            if (ti < 0) ti += nt + 1;
            if (vi > nv || vi <= 0) throw std::runtime_error("Out of bounds: tried to access vertex " + std::to_string(vi));
            MergedVertex mv;
            mv.p = xfPoint(toWorld, vertices[vi - 1]);
            if (ni != 0) {
                if (ni > nn || ni < 0) throw std::runtime_error("Out of bounds: tried to access normal " + std::to_string(ni));
                mv.n = xfNormal(toWorldInv, normals[ni - 1]);
                if (!mv.n.isZero()) mv.n = normalize(mv.n);
                hasNormals = true;
            }
            if (ti != 0) {
                if (ti > nt || ti < 0)
                    throw std::runtime_error("Out of bounds: tried to access texture coordinate " + std::to_string(ti));
                mv.u = texcoords[2 * (ti - 1)];
                mv.v = texcoords[2 * (ti - 1) + 1];
                hasUV = true;
            }
            auto it = merged.find(mv);
            uint32_t key;
            if (it != merged.end()) {
                key = it->second;
            } else {
                key = (uint32_t) buf.size();
                merged[mv] = key;
                buf.push_back(mv);
            }
            m.idx.push_back(key);
        }
    for (const MergedVertex &v : buf) {
        m.p.push_back(v.p);
        if (hasNormals) m.n.push_back(v.n);
        if (hasUV) {
            m.uv.push_back(v.u);
            m.uv.push_back(v.v);
        }
    }
    m.bsdf = sd.bsdf;
    computeNormals(m, sd.faceNormals, sd.flipNormals, hasNormals);
    out.push_back(std::move(m));
}

void loadObj(const MeshShapeDesc &sd, std::vector<Mesh> &out) { /* obj.cpp:199-349 */
    std::ifstream is(sd.file);
    if (is.bad() || is.fail()) throw std::runtime_error("Wavefront OBJ file '" + sd.file + "' not found!");
    float inv[16];
    if (!invertMatrix4(sd.toWorld, inv)) throw std::runtime_error("obj: singular toWorld matrix");
    std::vector<F3> vertices, normals;
    std::vector<float> texcoords;
    std::vector<Face> faces;
    std::string line, tag;
    while (is.good() && !is.eof() && fetchLine(is, line)) {
        std::istringstream iss(line);
        if (!(iss >> tag)) continue;
        if (tag == "v") {
            F3 p;
            iss >> p.x >> p.y >> p.z;
            vertices.push_back(p);
        } else if (tag == "vn") {
            F3 n;
            iss >> n.x >> n.y >> n.z;
            normals.push_back(n);
        } else if (tag == "vt") {
            float u, v;
            iss >> u >> v;
            if (sd.flipTexCoords) v = 1 - v;
            texcoords.push_back(u);
            texcoords.push_back(v);
        } else if (tag == "g" || tag == "usemtl") { /* a new group ends the current TriMesh */
            createMesh(vertices, normals, texcoords, faces, sd.toWorld, inv, sd, out);
            faces.clear();
        } else if (tag == "mtllib") {
            throw std::runtime_error("obj: material libraries (mtllib) are outside this path");
        } else if (tag == "f") {
            std::string tok;
            Face f;
            for (int i = 0; i < 3; ++i) {
                iss >> tok;
                parseFaceVertex(f, i, tok);
            }
            faces.push_back(f);
            while (iss >> tok) { /* a convex polygon as a triangle fan */
                f.p[1] = f.p[2];
                f.uv[1] = f.uv[2];
                f.n[1] = f.n[2];
                parseFaceVertex(f, 2, tok);
                faces.push_back(f);
            }
        }
    }
    createMesh(vertices, normals, texcoords, faces, sd.toWorld, inv, sd, out);
}

/* triaccel.h:37-70 */
HptTri triAccel(const F3 &A, const F3 &B, const F3 &C) {
    static const int waldModulo[4] = {1, 2, 0, 1};
    HptTri t;
    std::memset(&t, 0, sizeof(t));
    const F3 b = C - A, c = B - A, N = cross(c, b);
    int k = 0;
    for (int j = 0; j < 3; j++)
        if (std::abs(N[j]) > std::abs(N[k])) k = j;
    const int u = waldModulo[k], v = waldModulo[k + 1];
    const float n_k = N[k], denom = b[u] * c[v] - b[v] * c[u];
    if (denom == 0) {
        t.k = 3;
        return t;
    }
    t.k = (uint32_t) k;
    t.n_u = N[u] / n_k;
    t.n_v = N[v] / n_k;
    t.n_d = dot(A, N) / n_k;
    t.b_nu = b[u] / denom;
    t.b_nv = -b[v] / denom;
    t.a_u = A[u];
    t.a_v = A[v];
    t.c_nu = c[v] / denom;
    t.c_nv = -c[u] / denom;
    return t;
}

/* ---------------- BSDF records ---------------- */
int addBsdf(const BsdfDesc &b, std::vector<HptMeshBsdf> &out, int slot) {
    HptMeshBsdf r;
    std::memset(&r, 0, sizeof(r));
    if (b.type == "diffuse") {
        r.kind = HPT_MBSDF_DIFFUSE;
        float c0[3], c1[3], rf[3];
        for (int i = 0; i < 3; ++i) {
            rf[i] = b.diffuse[i];
            c0[i] = b.reflectanceTexture.color0[i];
            c1[i] = b.reflectanceTexture.color1[i];
        }
        r.textured = b.reflectanceTexture.type == "checkerboard";
        if (!b.reflectanceTexture.type.empty() && !r.textured)
            throw std::runtime_error("diffuse: texture '" + b.reflectanceTexture.type + "' is outside this path");
        /* BSDF::ensureEnergyConservation (bsdf.cpp:88-112): the maximum of the constant or of
           the checkerboard (checkerboard.cpp:85-90) */
        float mx = r.textured ? std::max({std::max(c0[0], c1[0]), std::max(c0[1], c1[1]), std::max(c0[2], c1[2])})
                              : std::max({rf[0], rf[1], rf[2]});
        if (b.ensureEnergyConservation && mx > 1.0f) {
            const float s = 0.99f * (1.0f / mx);
            for (int i = 0; i < 3; ++i) rf[i] *= s, c0[i] *= s, c1[i] *= s;
            mx *= s;
        }
        for (int i = 0; i < 3; ++i) r.refl[i] = rf[i], r.color0[i] = c0[i], r.color1[i] = c1[i];
        r.uoffset = b.reflectanceTexture.uoffset;
        r.voffset = b.reflectanceTexture.voffset;
        r.uscale = b.reflectanceTexture.uscale;
        r.vscale = b.reflectanceTexture.vscale;
        r.smooth = mx > 0 ? 1 : 0; /* diffuse.cpp:81-84: no component at all for a zero reflectance */
    } else if (b.type == "plastic") {
        /* plastic.cpp:146-217 */
        r.kind = HPT_MBSDF_PLASTIC;
        r.smooth = 1;
        r.eta = b.intIOR / b.extIOR;
        r.nonlinear = b.nonlinear ? 1 : 0;
        float dif[3] = {b.diffuse[0], b.diffuse[1], b.diffuse[2]}, spe[3] = {b.specular[0], b.specular[1], b.specular[2]};
        float mx = std::max({spe[0], spe[1], spe[2]});
        if (b.ensureEnergyConservation && mx > 1.0f)
            for (float &v : spe) v *= 0.99f * (1.0f / mx);
        mx = std::max({dif[0], dif[1], dif[2]});
        if (b.ensureEnergyConservation && mx > 1.0f)
            for (float &v : dif) v *= 0.99f * (1.0f / mx);
        for (int i = 0; i < 3; ++i) r.diffuse[i] = dif[i], r.specular[i] = spe[i];
        r.fdrInt = fresnelDiffuseReflectance(1 / r.eta);
        const float dAvg = dif[0] * 0.212671f + dif[1] * 0.715160f + dif[2] * 0.072169f; /* getLuminance */
        const float sAvg = spe[0] * 0.212671f + spe[1] * 0.715160f + spe[2] * 0.072169f;
        r.specularSamplingWeight = sAvg / (dAvg + sAvg);
        r.invEta2 = 1 / (r.eta * r.eta);
    } else if (b.type == "twosided") {
        /* twosided.cpp:84-110: nested[1] = nested[0] when only one is given; records of the
           nested BSDFs go after the scene's own, so desc.bsdfs indices stay the same */
        if (b.nested.empty() || b.nested.size() > 2) throw std::runtime_error("twosided: needs one or two nested BSDFs");
        r.kind = HPT_MBSDF_TWOSIDED;
        if (slot < 0) {
            slot = (int) out.size();
            out.push_back(r);
        }
        int ids[2] = {0, 0};
        for (size_t k = 0; k < b.nested.size(); ++k) {
            if (b.nested[k].type != "diffuse" && b.nested[k].type != "plastic")
                throw std::runtime_error("twosided: nested '" + b.nested[k].type + "' is outside the mesh path");
            ids[k] = addBsdf(b.nested[k], out, -1);
        }
        if (b.nested.size() == 1) ids[1] = ids[0];
        r.nested[0] = ids[0];
        r.nested[1] = ids[1];
        r.smooth = out[ids[0]].smooth || out[ids[1]].smooth;
        out[slot] = r;
        return slot;
    } else {
        throw std::runtime_error("bsdf '" + b.type + "' on a mesh shape is outside this path "
                                 "(diffuse, plastic, twosided)");
    }
    if (slot < 0) {
        slot = (int) out.size();
        out.push_back(r);
    } else {
        out[slot] = r;
    }
    return slot;
}

/* ---------------- BVH ---------------- */
struct Box {
    F3 mn{std::numeric_limits<float>::infinity(), std::numeric_limits<float>::infinity(),
          std::numeric_limits<float>::infinity()};
    F3 mx{-std::numeric_limits<float>::infinity(), -std::numeric_limits<float>::infinity(),
          -std::numeric_limits<float>::infinity()};
    void expand(const F3 &p) {
        mn = F3(std::min(mn.x, p.x), std::min(mn.y, p.y), std::min(mn.z, p.z));
        mx = F3(std::max(mx.x, p.x), std::max(mx.y, p.y), std::max(mx.z, p.z));
    }
};

void buildBvh(MeshSceneHost &S, const std::vector<Box> &box) {
    const uint32_t n = (uint32_t) box.size();
    std::vector<uint32_t> order(n);
    std::vector<F3> centroid(n);
    for (uint32_t i = 0; i < n; ++i) {
        order[i] = i;
        centroid[i] = (box[i].mn + box[i].mx) * 0.5f;
    }
    S.nodes.clear();
    S.depth = 0;
    if (n == 0) return;
    S.nodes.emplace_back();
    std::function<void(uint32_t, uint32_t, uint32_t, uint32_t)> build = [&](uint32_t node, uint32_t lo, uint32_t hi,
                                                                           uint32_t level) {
        S.depth = std::max(S.depth, level + 1);
        Box b, cb;
        for (uint32_t i = lo; i < hi; ++i) {
            b.expand(box[order[i]].mn);
            b.expand(box[order[i]].mx);
            cb.expand(centroid[order[i]]);
        }
        HptBvhNode nd;
        std::memset(&nd, 0, sizeof(nd));
        for (int k = 0; k < 3; ++k) nd.mn[k] = b.mn[k], nd.mx[k] = b.mx[k];
        if (hi - lo <= 4) {
            nd.a = lo;
            nd.count = hi - lo;
            S.nodes[node] = nd;
            return;
        }
        const F3 ext = cb.mx - cb.mn;
        int axis = 0;
        if (ext.y > ext[axis]) axis = 1;
        if (ext.z > ext[axis]) axis = 2;
        const uint32_t mid = (lo + hi) / 2;
        std::nth_element(order.begin() + lo, order.begin() + mid, order.begin() + hi, [&](uint32_t a, uint32_t c) {
            if (centroid[a][axis] != centroid[c][axis]) return centroid[a][axis] < centroid[c][axis];
            return a < c;
        });
        const uint32_t left = (uint32_t) S.nodes.size();
        S.nodes.emplace_back();
        build(left, lo, mid, level + 1);
        const uint32_t right = (uint32_t) S.nodes.size();
        S.nodes.emplace_back();
        build(right, mid, hi, level + 1);
        nd.a = right;
        nd.count = 0;
        S.nodes[node] = nd;
    };
    build(0, 0, n, 0);
    std::vector<uint32_t> refs(n);
    const uint32_t nTris = (uint32_t) S.tris.size();
    for (uint32_t i = 0; i < n; ++i) refs[i] = order[i] < nTris ? order[i] : (HPT_PRIM_RECT | (order[i] - nTris));
    S.prims.swap(refs);
}

} // namespace

float fresnelDiffuseReflectance(float eta) { /* util.cpp:856-858 */
    const Lobatto quad(1024, 0, 1e-5f);
    return quad.integrate([eta](float xi) { return fresnelDielectricExt(std::sqrt(xi), eta); }, 0, 1);
}

MeshSceneHost buildMeshScene(const SceneDesc &d) {
    MeshSceneHost S;
    S.bsdfs.resize(d.bsdfs.size());
    for (size_t i = 0; i < d.bsdfs.size(); ++i) addBsdf(d.bsdfs[i], S.bsdfs, (int) i);
    std::vector<Mesh> meshes;
    std::vector<Box> box;
    Box scene;
    std::vector<HptRect> rects;
    std::vector<Box> rectBox;
    for (const MeshShapeDesc &sd : d.meshes) {
        if (sd.bsdf < 0 || sd.bsdf >= (int) d.bsdfs.size()) throw std::runtime_error("mesh shape: bad bsdf index");
        if (sd.type == "obj") {
            loadObj(sd, meshes);
        } else if (sd.type == "rectangle") {
            /* rectangle.cpp:80-122 */
            float o2w[16], w2o[16];
            std::memcpy(o2w, sd.toWorld, sizeof(o2w));
            if (!invertMatrix4(o2w, w2o)) throw std::runtime_error("rectangle: singular toWorld matrix");
            if (sd.flipNormals) { /* m_objectToWorld * Transform::scale(1, 1, -1) (transform.cpp:28-31, 49-62) */
                const float S1[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, -1, 0, 0, 0, 0, 1};
                const float S1i[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1.0f / -1.0f, 0, 0, 0, 0, 1};
                float a[16], b[16];
                matMul(o2w, S1, a);
                matMul(S1i, w2o, b);
                std::memcpy(o2w, a, sizeof(a));
                std::memcpy(w2o, b, sizeof(b));
            }
            HptRect r;
            std::memset(&r, 0, sizeof(r));
            std::memcpy(r.w2o, w2o, sizeof(r.w2o)); /* rows 0-2 */
            const F3 dpdu = xfVector(o2w, F3(2, 0, 0)), dpdv = xfVector(o2w, F3(0, 2, 0));
            const F3 normal = normalize(xfNormal(w2o, F3(0, 0, 1)));
            const F3 s = normalize(dpdu), t = normalize(dpdv);
            if (std::abs(dot(s, t)) > kEps) throw std::runtime_error("Error: 'toWorld' transformation contains shear!");
            for (int k = 0; k < 3; ++k) r.s[k] = s[k], r.t[k] = t[k], r.n[k] = normal[k], r.dpdu[k] = dpdu[k];
            r.bsdf = sd.bsdf;
            Box bb;
            for (float x : {-1.0f, 1.0f})
                for (float y : {-1.0f, 1.0f}) bb.expand(xfPoint(o2w, F3(x, y, 0)));
            rects.push_back(r);
            rectBox.push_back(bb);
        } else {
            throw std::runtime_error("shape '" + sd.type + "' is outside the mesh path");
        }
    }
    /* flatten: vertex arrays, triangle records (TriAccel + indices), per-triangle dpdu */
    for (uint32_t mi = 0; mi < meshes.size(); ++mi) {
        const Mesh &m = meshes[mi];
        const uint32_t base = (uint32_t) S.vertexCount();
        HptMeshInfo info;
        std::memset(&info, 0, sizeof(info));
        info.bsdf = m.bsdf;
        info.hasNormals = m.n.empty() ? 0 : 1;
        info.hasUV = m.uv.empty() ? 0 : 1;
        S.meshes.push_back(info);
        for (size_t v = 0; v < m.p.size(); ++v) {
            S.p.insert(S.p.end(), {m.p[v].x, m.p[v].y, m.p[v].z});
            const F3 nv = m.n.empty() ? F3() : m.n[v];
            S.n.insert(S.n.end(), {nv.x, nv.y, nv.z});
            S.uv.insert(S.uv.end(), {m.uv.empty() ? 0.0f : m.uv[2 * v], m.uv.empty() ? 0.0f : m.uv[2 * v + 1]});
        }
        for (size_t i = 0; i < m.triangles(); ++i) {
            const uint32_t i0 = m.idx[3 * i], i1 = m.idx[3 * i + 1], i2 = m.idx[3 * i + 2];
            HptTri t = triAccel(m.p[i0], m.p[i1], m.p[i2]);
            t.i0 = base + i0;
            t.i1 = base + i1;
            t.i2 = base + i2;
            t.mesh = mi;
            S.tris.push_back(t);
            /* trimesh.cpp:683-743 computeUVTangents (zero for a degenerate triangle), else the
               hit record's fallback dpdu = p1 - p0 (skdtree.h:390-396) */
            const F3 dP1 = m.p[i1] - m.p[i0], dP2 = m.p[i2] - m.p[i0];
            F3 dpdu = dP1;
            if (!m.uv.empty()) {
                dpdu = F3();
                const float du1 = m.uv[2 * i1] - m.uv[2 * i0], dv1 = m.uv[2 * i1 + 1] - m.uv[2 * i0 + 1];
                const float du2 = m.uv[2 * i2] - m.uv[2 * i0], dv2 = m.uv[2 * i2 + 1] - m.uv[2 * i0 + 1];
                const F3 nrm = cross(dP1, dP2);
                const float length = nrm.length();
                if (length != 0) {
                    const float det = du1 * dv2 - dv1 * du2;
                    if (det == 0) {
                        F3 dpdv;
                        coordinateSystem(nrm / length, dpdu, dpdv);
                    } else {
                        const float invDet = 1.0f / det;
                        dpdu = (dP1 * dv2 - dP2 * dv1) * invDet;
                    }
                }
            }
            S.dpdu.insert(S.dpdu.end(), {dpdu.x, dpdu.y, dpdu.z});
            Box b;
            b.expand(m.p[i0]);
            b.expand(m.p[i1]);
            b.expand(m.p[i2]);
            box.push_back(b);
            scene.expand(b.mn);
            scene.expand(b.mx);
        }
    }
    S.rects = rects;
    for (const Box &b : rectBox) {
        box.push_back(b);
        scene.expand(b.mn);
        scene.expand(b.mx);
    }
    if (box.empty()) throw std::runtime_error("mesh scene without primitives");
    buildBvh(S, box);
    /* the scene kd-tree's bounds, slightly enlarged (gkdtree.h:1213-1220: the max uses the new min) */
    const float eps = 1e-3f;
    for (int k = 0; k < 3; ++k) {
        const float mn = scene.mn[k], mx = scene.mx[k];
        S.aabbMin[k] = mn - ((mx - mn) * eps + eps);
        S.aabbMax[k] = mx + ((mx - S.aabbMin[k]) * eps + eps);
    }
    return S;
}

} // namespace hpt
