/*
 * mesh_geom.h -- oracle restatement of the triangle-mesh shapes of the C1
 * "teapot" plumbing scene (BASELINE.json configs[0]):
 *
 *   Wavefront OBJ loader      src/shapes/obj.cpp:165-186 (fetch_line), 199-349, 371-390, 577-715
 *   TriMesh::configure        src/librender/trimesh.cpp:362-386, computeNormals :608-681,
 *                             computeUVTangents :683-743, unitAngle (core/util.h:309-314)
 *   TriAccel                  include/mitsuba/render/triaccel.h:37-158 (Wald's projection test)
 *   triangle hit record       include/mitsuba/render/skdtree.h:343-428 (fillIntersectionRecord<true>)
 *   Rectangle                 src/shapes/rectangle.cpp:80-168
 *   scene AABB enlargement    include/mitsuba/render/gkdtree.h:1213-1220 (MTS_KD_AABB_EPSILON 1e-3)
 *
 * The acceleration structure is NOT the reference's: a plain median-split BVH
 * over triangles and rectangles.  The closest hit it returns is the one the
 * reference's kd-tree returns (every primitive test runs against the running
 * [mint, maxt] with maxt shrinking to the nearest hit, sahkdtree3.h), up to
 * exact ties in t.
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Included by oracle.cpp inside its
 * anonymous namespace after Ray / AABB / Hit / Stats / Mat4; no includes.
 */

/* ---------------- Transform = (matrix, Gauss-Jordan inverse) ---------------- */
struct MeshXform {
    Mat4 t, inv;
};
inline MeshXform meshXform(const float *rowMajor) { /* Transform(const Matrix4x4 &) -> invert */
    MeshXform x;
    std::memcpy(x.t.m, rowMajor, sizeof(x.t.m));
    if (!matInvert(x.t, x.inv)) throw std::runtime_error("singular toWorld matrix");
    return x;
}
inline V3 xfPoint(const Mat4 &M, const V3 &p) { return xformPoint(&M.m[0][0], p); }
inline V3 xfVector(const Mat4 &M, const V3 &v) { return xformVector(&M.m[0][0], v); }
inline V3 xfNormal(const MeshXform &X, const V3 &v) { /* transform.h:203-211: inverse transposed */
    const auto &m = X.inv.m;
    return V3(m[0][0] * v.x + m[1][0] * v.y + m[2][0] * v.z, m[0][1] * v.x + m[1][1] * v.y + m[2][1] * v.z,
              m[0][2] * v.x + m[1][2] * v.y + m[2][2] * v.z);
}
inline V3 xfPointAffine(const Mat4 &M, const V3 &p) { /* transform.h:139-146 */
    return V3(M.m[0][0] * p.x + M.m[0][1] * p.y + M.m[0][2] * p.z + M.m[0][3],
              M.m[1][0] * p.x + M.m[1][1] * p.y + M.m[1][2] * p.z + M.m[1][3],
              M.m[2][0] * p.x + M.m[2][1] * p.y + M.m[2][2] * p.z + M.m[2][3]);
}

/* ---------------- TriAccel (triaccel.h:37-158) ---------------- */
struct TriAccel {
    uint32_t k = 3;
    float n_u = 0, n_v = 0, n_d = 0, a_u = 0, a_v = 0, b_nu = 0, b_nv = 0, c_nu = 0, c_nv = 0;
    int load(const V3 &A, const V3 &B, const V3 &C) {
        static const int waldModulo[4] = {1, 2, 0, 1};
        const V3 b = C - A, c = B - A, N = cross(c, b);
        k = 0;
        for (int j = 0; j < 3; j++)
            if (std::abs(N[j]) > std::abs(N[k])) k = j;
        const uint32_t u = waldModulo[k], v = waldModulo[k + 1];
        const float n_k = N[k], denom = b[u] * c[v] - b[v] * c[u];
        if (denom == 0) {
            k = 3;
            return 1;
        }
        n_u = N[u] / n_k;
        n_v = N[v] / n_k;
        n_d = dot(A, N) / n_k;
        b_nu = b[u] / denom;
        b_nv = -b[v] / denom;
        a_u = A[u];
        a_v = A[v];
        c_nu = c[v] / denom;
        c_nv = -c[u] / denom;
        return 0;
    }
    bool rayIntersect(const Ray &ray, float mint, float maxt, float &u, float &v, float &t) const {
        float o_u, o_v, o_k, d_u, d_v, d_k;
        switch (k) {
        case 0: o_u = ray.o[1]; o_v = ray.o[2]; o_k = ray.o[0]; d_u = ray.d[1]; d_v = ray.d[2]; d_k = ray.d[0]; break;
        case 1: o_u = ray.o[2]; o_v = ray.o[0]; o_k = ray.o[1]; d_u = ray.d[2]; d_v = ray.d[0]; d_k = ray.d[1]; break;
        case 2: o_u = ray.o[0]; o_v = ray.o[1]; o_k = ray.o[2]; d_u = ray.d[0]; d_v = ray.d[1]; d_k = ray.d[2]; break;
        default: return false;
        }
        t = (n_d - o_u * n_u - o_v * n_v - o_k) / (d_u * n_u + d_v * n_v + d_k);
        if (t < mint || t > maxt) return false;
        const float hu = o_u + t * d_u - a_u, hv = o_v + t * d_v - a_v;
        u = hv * b_nu + hu * b_nv;
        v = hu * c_nu + hv * c_nv;
        return u >= 0 && v >= 0 && u + v <= 1.0f;
    }
};

/* ---------------- TriMesh (trimesh.cpp) ---------------- */
struct TriMesh {
    std::vector<V3> p, n;          /* n empty = no vertex normals (faceNormals) */
    std::vector<float> uv;         /* 2 per vertex, empty = no texcoords */
    std::vector<uint32_t> idx;     /* 3 per triangle */
    std::vector<V3> dpdu, dpdv;    /* per triangle, computeUVTangents (only with texcoords) */
    std::vector<TriAccel> acc;
    AABB aabb;
    int bsdf = 0;
    size_t triangles() const { return idx.size() / 3; }
};

/* core/util.h:309-314 (M_PI is the float M_PI_FLT in the single-precision build) */
inline float unitAngle(const V3 &u, const V3 &v) {
    if (dot(u, v) < 0) return kPi - 2 * std::asin(0.5f * (v + u).length());
    return 2 * std::asin(0.5f * (v - u).length());
}

/* trimesh.cpp:608-681 */
inline void computeNormals(TriMesh &m, bool faceNormals, bool flipNormals, bool hasNormals) {
    if (faceNormals) {
        m.n.clear();
        if (flipNormals)
            for (size_t i = 0; i < m.triangles(); ++i) std::swap(m.idx[3 * i], m.idx[3 * i + 1]);
        return;
    }
    if (hasNormals) {
        if (flipNormals)
            for (V3 &n : m.n) n *= -1;
        return;
    }
    m.n.assign(m.p.size(), V3(0.0f));
    for (size_t i = 0; i < m.triangles(); i++) {
        V3 n(0.0f);
        for (int j = 0; j < 3; ++j) {
            const V3 &v0 = m.p[m.idx[3 * i + j]], &v1 = m.p[m.idx[3 * i + (j + 1) % 3]],
                     &v2 = m.p[m.idx[3 * i + (j + 2) % 3]];
            const V3 sideA = v1 - v0, sideB = v2 - v0;
            if (j == 0) {
                n = cross(sideA, sideB);
                const float length = n.length();
                if (length == 0) break;
                n /= length;
            }
            const float angle = unitAngle(normalize(sideA), normalize(sideB));
            m.n[m.idx[3 * i + j]] += n * angle;
        }
    }
    for (V3 &n : m.n) {
        float length = n.length();
        if (flipNormals) length *= -1;
        if (length != 0)
            n /= length;
        else
            n = V3(1, 0, 0);
    }
}

/* trimesh.cpp:683-743 */
inline void computeUVTangents(TriMesh &m) {
    if (m.uv.empty()) return;
    m.dpdu.assign(m.triangles(), V3(0.0f));
    m.dpdv.assign(m.triangles(), V3(0.0f));
    for (size_t i = 0; i < m.triangles(); i++) {
        const uint32_t i0 = m.idx[3 * i], i1 = m.idx[3 * i + 1], i2 = m.idx[3 * i + 2];
        const V3 dP1 = m.p[i1] - m.p[i0], dP2 = m.p[i2] - m.p[i0];
        const float du1 = m.uv[2 * i1] - m.uv[2 * i0], dv1 = m.uv[2 * i1 + 1] - m.uv[2 * i0 + 1];
        const float du2 = m.uv[2 * i2] - m.uv[2 * i0], dv2 = m.uv[2 * i2 + 1] - m.uv[2 * i0 + 1];
        const V3 n = cross(dP1, dP2);
        const float length = n.length();
        if (length == 0) continue;
        const float determinant = du1 * dv2 - dv1 * du2;
        if (determinant == 0) {
            coordinateSystem(n / length, m.dpdu[i], m.dpdv[i]);
        } else {
            const float invDet = 1.0f / determinant;
            m.dpdu[i] = (dv2 * dP1 - dv1 * dP2) * invDet;
            m.dpdv[i] = ((-du2) * dP1 + du1 * dP2) * invDet;
        }
    }
}

/* ---------------- WavefrontOBJ (obj.cpp) ---------------- */
struct ObjTriangle {
    int p[3] = {0, 0, 0}, uv[3] = {0, 0, 0}, n[3] = {0, 0, 0};
};

/* obj.cpp:165-186 */
inline bool objFetchLine(std::istream &is, std::string &line) {
    if (!std::getline(is, line)) return false;
    if (line.empty()) return true;
    int last = (int) line.size() - 1;
    while (last >= 0 && (line[last] == '\r' || line[last] == '\n' || line[last] == '\t' || line[last] == ' ')) last--;
    if (last >= 0 && line[last] == '\\') {
        std::string next;
        objFetchLine(is, next);
        line = line.substr(0, last) + next;
    } else {
        line.resize(last + 1);
    }
    return true;
}

/* obj.cpp:371-390 over util.cpp:83-95 tokenize (empty tokens dropped) */
inline void objParseVertex(ObjTriangle &t, int i, const std::string &str) {
    std::vector<std::string> tok;
    std::string::size_type last = str.find_first_not_of('/', 0), pos = str.find_first_of('/', last);
    while (pos != std::string::npos || last != std::string::npos) {
        tok.push_back(str.substr(last, pos - last));
        last = str.find_first_not_of('/', pos);
        pos = str.find_first_of('/', last);
    }
    if (tok.size() == 1) {
        t.p[i] = std::atoi(tok[0].c_str());
    } else if (tok.size() == 2) {
        t.p[i] = std::atoi(tok[0].c_str());
        if (str.find("//") == std::string::npos)
            t.uv[i] = std::atoi(tok[1].c_str());
        else
            t.n[i] = std::atoi(tok[1].c_str());
    } else if (tok.size() == 3) {
        t.p[i] = std::atoi(tok[0].c_str());
        t.uv[i] = std::atoi(tok[1].c_str());
        t.n[i] = std::atoi(tok[2].c_str());
    } else {
        throw std::runtime_error("Invalid OBJ face format!");
    }
}

struct ObjVertex {
    V3 p, n;
    float u = 0, v = 0;
    bool operator<(const ObjVertex &o) const { /* obj.cpp:584-606 */
        const float a[8] = {p.x, p.y, p.z, n.x, n.y, n.z, u, v}, b[8] = {o.p.x, o.p.y, o.p.z, o.n.x, o.n.y, o.n.z, o.u, o.v};
        for (int i = 0; i < 8; ++i) {
            if (a[i] < b[i]) return true;
            if (a[i] > b[i]) return false;
        }
        return false;
    }
};

/* obj.cpp:608-715 createMesh + TriMesh::configure */
inline void objCreateMesh(const std::vector<V3> &vertices, const std::vector<V3> &normals,
                          const std::vector<float> &texcoords, const std::vector<ObjTriangle> &triangles,
                          const MeshXform &X, bool faceNormals, bool flipNormals, int bsdf,
                          std::vector<TriMesh> &out) {
    if (triangles.empty()) return;
    std::map<ObjVertex, uint32_t> vertexMap;
    std::vector<ObjVertex> buf;
    TriMesh m;
    bool hasTexcoords = false, hasNormals = false;
    const int nv = (int) vertices.size(), nn = (int) normals.size(), nt = (int) texcoords.size() / 2;
    for (const ObjTriangle &tri : triangles)
        for (int j = 0; j < 3; j++) {
            int vertexId = tri.p[j], normalId = tri.n[j], uvId = tri.uv[j];
            if (vertexId < 0) vertexId += nv + 1;
            if (normalId < 0) normalId += nn + 1;
            if (uvId < 0) uvId += nt + 1;
            if (vertexId > nv || vertexId <= 0) throw std::runtime_error("OBJ: vertex index out of bounds");
            ObjVertex vx;
            vx.p = xfPoint(X.t, vertices[vertexId - 1]);
            m.aabb.expandBy(vx.p);
            if (normalId != 0) {
                if (normalId > nn || normalId < 0) throw std::runtime_error("OBJ: normal index out of bounds");
                vx.n = xfNormal(X, normals[normalId - 1]);
                if (!vx.n.isZero()) vx.n = normalize(vx.n);
                hasNormals = true;
            }
            if (uvId != 0) {
                if (uvId > nt || uvId < 0) throw std::runtime_error("OBJ: uv index out of bounds");
                vx.u = texcoords[2 * (uvId - 1)];
                vx.v = texcoords[2 * (uvId - 1) + 1];
                hasTexcoords = true;
            }
            auto it = vertexMap.find(vx);
            uint32_t key;
            if (it != vertexMap.end()) {
                key = it->second;
            } else {
                key = (uint32_t) buf.size();
                vertexMap[vx] = key;
                buf.push_back(vx);
            }
            m.idx.push_back(key);
        }
    for (const ObjVertex &vx : buf) {
        m.p.push_back(vx.p);
        if (hasNormals) m.n.push_back(vx.n);
        if (hasTexcoords) {
            m.uv.push_back(vx.u);
            m.uv.push_back(vx.v);
        }
    }
    m.bsdf = bsdf;
    computeNormals(m, faceNormals, flipNormals, hasNormals);
    computeUVTangents(m);
    m.acc.resize(m.triangles());
    for (size_t i = 0; i < m.triangles(); ++i) /* skdtree.cpp:88-95 */
        m.acc[i].load(m.p[m.idx[3 * i]], m.p[m.idx[3 * i + 1]], m.p[m.idx[3 * i + 2]]);
    out.push_back(std::move(m));
}

/* obj.cpp:199-349: one TriMesh per group (g / usemtl split it); mtllib is refused */
inline void loadOBJ(const std::string &path, const float *toWorld, bool faceNormals, bool flipNormals,
                    bool flipTexCoords, int bsdf, std::vector<TriMesh> &out) {
    std::ifstream is(path);
    if (is.bad() || is.fail()) throw std::runtime_error("Wavefront OBJ file '" + path + "' not found!");
    static const float kIdentity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    const MeshXform X = meshXform(toWorld ? toWorld : kIdentity);
    std::vector<V3> vertices, normals;
    std::vector<float> texcoords;
    std::vector<ObjTriangle> triangles;
    std::string line, buf;
    while (is.good() && !is.eof() && objFetchLine(is, line)) {
        std::istringstream iss(line);
        if (!(iss >> buf)) continue;
        if (buf == "v") {
            V3 p;
            iss >> p.x >> p.y >> p.z;
            vertices.push_back(p);
        } else if (buf == "vn") {
            V3 n;
            iss >> n.x >> n.y >> n.z;
            normals.push_back(n);
        } else if (buf == "vt") {
            float u, v;
            iss >> u >> v;
            if (flipTexCoords) v = 1 - v;
            texcoords.push_back(u);
            texcoords.push_back(v);
        } else if (buf == "g" || buf == "usemtl") {
            objCreateMesh(vertices, normals, texcoords, triangles, X, faceNormals, flipNormals, bsdf, out);
            triangles.clear();
        } else if (buf == "mtllib") {
            throw std::runtime_error("OBJ material libraries are outside this path");
        } else if (buf == "f") {
            std::string tmp;
            ObjTriangle t;
            iss >> tmp; objParseVertex(t, 0, tmp);
            iss >> tmp; objParseVertex(t, 1, tmp);
            iss >> tmp; objParseVertex(t, 2, tmp);
            triangles.push_back(t);
            while (iss >> tmp) { /* convex n-gon: a fan */
                t.p[1] = t.p[2];
                t.uv[1] = t.uv[2];
                t.n[1] = t.n[2];
                objParseVertex(t, 2, tmp);
                triangles.push_back(t);
            }
        }
    }
    objCreateMesh(vertices, normals, texcoords, triangles, X, faceNormals, flipNormals, bsdf, out);
}

/* ---------------- Rectangle (rectangle.cpp:80-168) ---------------- */
struct RectShape {
    MeshXform o2w;
    Mat4 w2o;
    V3 dpdu, dpdv;
    Frame frame;
    AABB aabb;
    int bsdf = 0;
};

inline RectShape makeRectangle(const float *toWorld, bool flipNormals, int bsdf) {
    static const float kIdentity[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    RectShape r;
    r.o2w = meshXform(toWorld ? toWorld : kIdentity);
    if (flipNormals) { /* m_objectToWorld * Transform::scale(1, 1, -1) (transform.cpp:28-31, 49-62) */
        const Mat4 S = {{{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, -1, 0}, {0, 0, 0, 1}}};
        const Mat4 Si = {{{1, 0, 0, 0}, {0, 1, 0, 0}, {0, 0, 1.0f / -1.0f, 0}, {0, 0, 0, 1}}};
        r.o2w = MeshXform{matMul(r.o2w.t, S), matMul(Si, r.o2w.inv)};
    }
    r.w2o = r.o2w.inv; /* Transform::inverse(): the stored inverse matrix */
    r.dpdu = xfVector(r.o2w.t, V3(2, 0, 0));
    r.dpdv = xfVector(r.o2w.t, V3(0, 2, 0));
    const V3 normal = normalize(xfNormal(r.o2w, V3(0, 0, 1)));
    r.frame.s = normalize(r.dpdu);
    r.frame.t = normalize(r.dpdv);
    r.frame.n = normal;
    if (std::abs(dot(normalize(r.dpdu), normalize(r.dpdv))) > kEpsilon)
        throw std::runtime_error("Error: 'toWorld' transformation contains shear!");
    for (float x : {-1.0f, 1.0f})
        for (float y : {-1.0f, 1.0f}) r.aabb.expandBy(xfPoint(r.o2w.t, V3(x, y, 0)));
    r.bsdf = bsdf;
    return r;
}

/* :125-148; local = object-space (x, y) of the hit */
inline bool rectIntersect(const RectShape &r, const Ray &wr, float mint, float maxt, float &t, float &lx, float &ly) {
    const V3 o = xfPointAffine(r.w2o, wr.o), d = xfVector(r.w2o, wr.d);
    const float hit = -o.z / d.z;
    if (!(hit >= mint && hit <= maxt)) return false;
    const V3 local = o + d * hit;
    if (std::abs(local.x) <= 1 && std::abs(local.y) <= 1) {
        t = hit;
        lx = local.x;
        ly = local.y;
        return true;
    }
    return false;
}

/* ---------------- BVH over the mesh primitives (acceleration only) ---------------- */
struct MeshPrimRef {
    uint32_t shape, prim; /* shape < nTriMeshes: triangle prim of that mesh; else rectangle shape - nTriMeshes */
};
struct MeshBVHNode {
    AABB box;
    uint32_t first = 0, count = 0, right = 0; /* leaf: count > 0, prims [first, first+count); inner: left = this+1 */
};
struct MeshBVH {
    std::vector<MeshBVHNode> nodes;
    std::vector<MeshPrimRef> prims;
    bool empty() const { return prims.empty(); }
};

inline AABB meshPrimBox(const std::vector<TriMesh> &meshes, const std::vector<RectShape> &rects, const MeshPrimRef &r) {
    AABB b;
    if (r.shape < meshes.size()) {
        const TriMesh &m = meshes[r.shape];
        for (int j = 0; j < 3; ++j) b.expandBy(m.p[m.idx[3 * r.prim + j]]);
    } else {
        b = rects[r.shape - meshes.size()].aabb;
    }
    return b;
}

inline void buildMeshBVH(const std::vector<TriMesh> &meshes, const std::vector<RectShape> &rects, MeshBVH &bvh) {
    bvh.nodes.clear();
    bvh.prims.clear();
    for (uint32_t s = 0; s < meshes.size(); ++s)
        for (uint32_t i = 0; i < meshes[s].triangles(); ++i) bvh.prims.push_back({s, i});
    for (uint32_t r = 0; r < rects.size(); ++r) bvh.prims.push_back({(uint32_t) meshes.size() + r, 0});
    if (bvh.prims.empty()) return;
    std::vector<AABB> box(bvh.prims.size());
    std::vector<V3> centroid(bvh.prims.size());
    for (size_t i = 0; i < bvh.prims.size(); ++i) {
        box[i] = meshPrimBox(meshes, rects, bvh.prims[i]);
        centroid[i] = (box[i].min + box[i].max) * 0.5f;
    }
    std::vector<uint32_t> order(bvh.prims.size());
    for (size_t i = 0; i < order.size(); ++i) order[i] = (uint32_t) i;
    bvh.nodes.emplace_back();
    /* depth-first, the left child stored next to its parent */
    std::function<void(uint32_t, uint32_t, uint32_t)> build = [&](uint32_t node, uint32_t lo, uint32_t hi) {
        AABB b, cb;
        for (uint32_t i = lo; i < hi; ++i) {
            b.expandBy(box[order[i]].min);
            b.expandBy(box[order[i]].max);
            cb.expandBy(centroid[order[i]]);
        }
        bvh.nodes[node].box = b;
        if (hi - lo <= 4) {
            bvh.nodes[node].first = lo;
            bvh.nodes[node].count = hi - lo;
            return;
        }
        int axis = 0;
        const V3 ext = cb.max - cb.min;
        if (ext.y > ext[axis]) axis = 1;
        if (ext.z > ext[axis]) axis = 2;
        const uint32_t mid = (lo + hi) / 2;
        std::nth_element(order.begin() + lo, order.begin() + mid, order.begin() + hi, [&](uint32_t a, uint32_t c) {
            if (centroid[a][axis] != centroid[c][axis]) return centroid[a][axis] < centroid[c][axis];
            return a < c;
        });
        const uint32_t left = (uint32_t) bvh.nodes.size();
        bvh.nodes.emplace_back();
        build(left, lo, mid);
        const uint32_t right = (uint32_t) bvh.nodes.size();
        bvh.nodes.emplace_back();
        build(right, mid, hi);
        bvh.nodes[node].right = right;
    };
    build(0, 0, (uint32_t) order.size());
    std::vector<MeshPrimRef> sorted(order.size());
    for (size_t i = 0; i < order.size(); ++i) sorted[i] = bvh.prims[order[i]];
    bvh.prims.swap(sorted);
}

/* closest (or, for shadow rays, any) mesh hit with t in [mint, maxt]; maxt shrinks to the hit */
template <bool shadowRay>
bool meshIntersect(const std::vector<TriMesh> &meshes, const std::vector<RectShape> &rects, const MeshBVH &bvh,
                   const Ray &ray, float mint, float &maxt, Hit *hit, Stats *st) {
    if (bvh.empty()) return false;
    bool found = false;
    uint32_t stack[128];
    int sp = 0;
    stack[sp++] = 0;
    while (sp > 0) {
        const MeshBVHNode &nd = bvh.nodes[stack[--sp]];
        if (st) st->nodes++;
        float nearT, farT;
        if (!nd.box.rayIntersect(ray, nearT, farT) || farT < mint || nearT > maxt) continue;
        if (nd.count == 0) {
            stack[sp++] = nd.right;
            stack[sp++] = (uint32_t) (&nd - bvh.nodes.data()) + 1;
            continue;
        }
        for (uint32_t i = nd.first; i < nd.first + nd.count; ++i) {
            const MeshPrimRef &r = bvh.prims[i];
            if (st) st->prims++;
            float t, u, v;
            bool ok;
            if (r.shape < meshes.size())
                ok = meshes[r.shape].acc[r.prim].rayIntersect(ray, mint, maxt, u, v, t);
            else
                ok = rectIntersect(rects[r.shape - meshes.size()], ray, mint, maxt, t, u, v);
            if (!ok) continue;
            if (shadowRay) return true;
            maxt = t;
            found = true;
            hit->t = t;
            hit->kind = r.shape < meshes.size() ? 1 : 2;
            hit->shape = r.shape < meshes.size() ? r.shape : r.shape - (uint32_t) meshes.size();
            hit->prim = r.prim;
            hit->u = u;
            hit->v = v;
        }
    }
    return found;
}
