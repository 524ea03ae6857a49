/*
 * hpt_mesh.h -- k_mesh_paths: MIPathTracer::Li (src/integrators/path/path.cpp:119-294) over a
 * triangle-mesh scene (C1, models/teapot/scene.xml:31-84), one path per lane from the camera
 * sample to termination.  Included by hpt_render.hip after its helpers: the Sobol sampler,
 * the camera (cameraRay / cameraDifferentials), the environment (envSampleDir / envEval /
 * envEvalFiltered / envPdf / bsphereIntersect) and the film (k_splat / k_gather over
 * HptPaths::li and ::pos) are the hair kernels' own.
 *
 *   geometry   TriAccel::rayIntersect (triaccel.h:114-158), Rectangle::rayIntersect
 *              (rectangle.cpp:125-148) under a BVH of 32-byte nodes (HptBvhNode); the scene
 *              AABB clip and the adaptive ray epsilon of ShapeKDTree (skdtree.cpp:112-141,
 *              :207-226)
 *   hit record fillIntersectionRecord<true> for a triangle (skdtree.h:343-428), Rectangle::
 *              fillIntersectionRecord (rectangle.cpp:155-168), computeShadingFrame (util.cpp:603-608)
 *   BSDFs      SmoothDiffuse (diffuse.cpp:90-140) with a Checkerboard (checkerboard.cpp:47-80 over
 *              Texture2D's uv transform, texture.cpp:113), SmoothPlastic (plastic.cpp:219-417),
 *              TwoSidedBRDF (twosided.cpp:108-183)
 *
 * C1 is 64x64 @ 16 spp (65,536 paths): the configuration is plumbing, not throughput, so the
 * kernel is a plain per-lane megakernel (the BVH stack in LDS).  Every float operation
 * follows the oracle's restatement (oracle/mesh_geom.h, mesh_bsdf.h, oracle.cpp Li) in the
 * same order, built with -ffp-contract=off like the rest of the device code.
 */
namespace {

/* aabb.h:308-338 over a BVH node */
HD bool nodeHit(const HptBvhNode &nd, V3 o, V3 d, V3 rcp, float &nearT, float &farT) {
    nearT = -finf();
    farT = finf();
    const float mn[3] = {nd.mn[0], nd.mn[1], nd.mn[2]}, mx[3] = {nd.mx[0], nd.mx[1], nd.mx[2]};
    for (int i = 0; i < 3; ++i) {
        const float origin = o[i];
        if (d[i] == 0) {
            if (origin < mn[i] || origin > mx[i]) return false;
        } else {
            float t1 = (mn[i] - origin) * rcp[i], t2 = (mx[i] - origin) * rcp[i];
            if (t1 > t2) {
                const float t = t1;
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

/* the scene bounds (the scene kd-tree's AABB) */
HD bool sceneBoxHit(const HptMeshScene &ms, V3 o, V3 d, V3 rcp, float &nearT, float &farT) {
    HptBvhNode nd;
    for (int i = 0; i < 3; ++i) nd.mn[i] = ms.aabbMin[i], nd.mx[i] = ms.aabbMax[i];
    return nodeHit(nd, o, d, rcp, nearT, farT);
}

/* triaccel.h:114-158 */
HD bool triHit(const HptTri &tr, V3 o, V3 d, float mint, float maxt, float &u, float &v, float &t) {
    float o_u, o_v, o_k, d_u, d_v, d_k;
    switch (tr.k) {
    case 0: o_u = o.y; o_v = o.z; o_k = o.x; d_u = d.y; d_v = d.z; d_k = d.x; break;
    case 1: o_u = o.z; o_v = o.x; o_k = o.y; d_u = d.z; d_v = d.x; d_k = d.y; break;
    case 2: o_u = o.x; o_v = o.y; o_k = o.z; d_u = d.x; d_v = d.y; d_k = d.z; break;
    default: return false;
    }
    t = (tr.n_d - o_u * tr.n_u - o_v * tr.n_v - o_k) / (d_u * tr.n_u + d_v * tr.n_v + d_k);
    if (t < mint || t > maxt) return false;
    const float hu = o_u + t * d_u - tr.a_u, hv = o_v + t * d_v - tr.a_v;
    u = hv * tr.b_nu + hu * tr.b_nv;
    v = hu * tr.c_nu + hv * tr.c_nv;
    return u >= 0 && v >= 0 && u + v <= 1.0f;
}

/* rectangle.cpp:125-148; (lx, ly) = the hit in object space */
HD bool rectHit(const HptRect &r, V3 wo, V3 wd, float mint, float maxt, float &t, float &lx, float &ly) {
    const float *M = r.w2o;
    const V3 o = v3(M[0] * wo.x + M[1] * wo.y + M[2] * wo.z + M[3], M[4] * wo.x + M[5] * wo.y + M[6] * wo.z + M[7],
                    M[8] * wo.x + M[9] * wo.y + M[10] * wo.z + M[11]);
    const V3 d = v3(M[0] * wd.x + M[1] * wd.y + M[2] * wd.z, M[4] * wd.x + M[5] * wd.y + M[6] * wd.z,
                    M[8] * wd.x + M[9] * wd.y + M[10] * wd.z);
    const float hit = -o.z / d.z;
    if (!(hit >= mint && hit <= maxt)) return false;
    const V3 local = o + d * hit;
    if (fabsf(local.x) <= 1 && fabsf(local.y) <= 1) {
        t = hit;
        lx = local.x;
        ly = local.y;
        return true;
    }
    return false;
}

struct MeshHit {
    float t, u, v;
    uint32_t prim; /* triangle index, or HPT_PRIM_RECT | rectangle */
};

/* closest hit (or, SHADOW, any hit) in [mint, maxt], maxt shrinking to each hit in test order.
   stk: the lane's column of the block's LDS stack (entry e at stk[e * HPT_MESH_BLOCK]) */
#define HPT_MESH_BLOCK 256
template <bool SHADOW>
HD bool meshTraverse(const HptMeshScene &ms, V3 o, V3 d, float mint, float maxt, MeshHit &hit, uint32_t *stk) {
    const V3 rcp = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    auto stack = [&](int e) -> uint32_t & { return stk[e * HPT_MESH_BLOCK]; };
    int sp = 0;
    stack(sp++) = 0;
    bool found = false;
    while (sp > 0) {
        const uint32_t ni = stack(--sp);
        const HptBvhNode nd = ms.nodes[ni];
        float nearT, farT;
        if (!nodeHit(nd, o, d, rcp, nearT, farT) || farT < mint || nearT > maxt) continue;
        if (nd.count == 0) {
            stack(sp++) = nd.a;
            stack(sp++) = ni + 1;
            continue;
        }
        for (uint32_t k = nd.a; k < nd.a + nd.count; ++k) {
            const uint32_t ref = ms.prims[k];
            float t, u, v;
            const bool ok = (ref & HPT_PRIM_RECT) ? rectHit(ms.rects[ref & ~HPT_PRIM_RECT], o, d, mint, maxt, t, u, v)
                                                  : triHit(ms.tris[ref], o, d, mint, maxt, u, v, t);
            if (!ok) continue;
            if (SHADOW) return true;
            maxt = t;
            found = true;
            hit.t = t;
            hit.u = u;
            hit.v = v;
            hit.prim = ref;
        }
    }
    return found;
}

/* ShapeKDTree::rayIntersect (skdtree.cpp:112-141): scene-AABB clip + adaptive epsilon */
HD bool meshIntersect(const HptMeshScene &ms, V3 o, V3 d, float rmint, float rmaxt, MeshHit &hit, uint32_t *stk) {
    const V3 rcp = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float mint, maxt;
    if (!sceneBoxHit(ms, o, d, rcp, mint, maxt)) return false;
    const float rayMinT = adaptiveMint(o, rmint, false);
    if (rayMinT > mint) mint = rayMinT;
    if (rmaxt < maxt) maxt = rmaxt;
    if (!(maxt > mint)) return false;
    return meshTraverse<false>(ms, o, d, mint, maxt, hit, stk);
}
/* ShapeKDTree::rayIntersect(shadow) (skdtree.cpp:207-226) */
HD bool meshOccluded(const HptMeshScene &ms, V3 o, V3 d, float rmint, float rmaxt, uint32_t *stk) {
    const V3 rcp = v3(1.0f / d.x, 1.0f / d.y, 1.0f / d.z);
    float mint, maxt;
    if (!sceneBoxHit(ms, o, d, rcp, mint, maxt)) return false;
    const float rayMinT = adaptiveMint(o, rmint, true);
    if (rayMinT > mint) mint = rayMinT;
    if (rmaxt < maxt) maxt = rmaxt;
    if (!(maxt > mint)) return false;
    MeshHit unused;
    return meshTraverse<true>(ms, o, d, mint, maxt, unused, stk);
}

struct MeshIts {
    V3 p, wi;
    Frame geo, sh;
    float u, v; /* texture coordinates */
    int bsdf;
};

HD V3 vtx3(const float *a, uint32_t i) { return v3(a[3 * i], a[3 * i + 1], a[3 * i + 2]); }

/* fillIntersectionRecord<true> (skdtree.h:343-428) / Rectangle (rectangle.cpp:155-168) */
HD void meshFill(const HptMeshScene &ms, V3 o, V3 d, const MeshHit &h, MeshIts &its) {
    V3 dpdu, shN;
    if (h.prim & HPT_PRIM_RECT) {
        const HptRect &r = ms.rects[h.prim & ~HPT_PRIM_RECT];
        its.geo.s = v3(r.s[0], r.s[1], r.s[2]);
        its.geo.t = v3(r.t[0], r.t[1], r.t[2]);
        its.geo.n = v3(r.n[0], r.n[1], r.n[2]);
        shN = its.geo.n;
        dpdu = v3(r.dpdu[0], r.dpdu[1], r.dpdu[2]);
        its.u = 0.5f * (h.u + 1);
        its.v = 0.5f * (h.v + 1);
        its.p = o + d * h.t;
        its.bsdf = r.bsdf;
    } else {
        const HptTri &tr = ms.tris[h.prim];
        const HptMeshInfo mi = ms.meshes[tr.mesh];
        const float bx = 1 - h.u - h.v, by = h.u, bz = h.v;
        const V3 p0 = vtx3(ms.p, tr.i0), p1 = vtx3(ms.p, tr.i1), p2 = vtx3(ms.p, tr.i2);
        its.p = p0 * bx + p1 * by + p2 * bz;
        const V3 side1 = p1 - p0, side2 = p2 - p0;
        V3 fn = cross(side1, side2);
        const float len = length(fn);
        if (!isZero(fn)) fn = divs(fn, len);
        dpdu = vtx3(ms.dpdu, h.prim);
        if (mi.hasNormals) {
            shN = normalize(vtx3(ms.n, tr.i0) * bx + vtx3(ms.n, tr.i1) * by + vtx3(ms.n, tr.i2) * bz);
            if (dot(fn, shN) < 0) fn = -fn;
        } else {
            shN = fn;
        }
        its.geo.n = fn;
        coordinateSystem(fn, its.geo.s, its.geo.t);
        if (mi.hasUV) {
            its.u = ms.uv[2 * tr.i0] * bx + ms.uv[2 * tr.i1] * by + ms.uv[2 * tr.i2] * bz;
            its.v = ms.uv[2 * tr.i0 + 1] * bx + ms.uv[2 * tr.i1 + 1] * by + ms.uv[2 * tr.i2 + 1] * bz;
        } else {
            its.u = by;
            its.v = bz;
        }
        its.bsdf = mi.bsdf;
    }
    /* computeShadingFrame (util.cpp:603-608) */
    its.sh.n = shN;
    its.sh.s = normalize(dpdu - shN * dot(shN, dpdu));
    its.sh.t = cross(shN, its.sh.s);
    its.wi = its.sh.toLocal(-d);
}

/* ---------------- BSDFs ---------------- */
HD V3 f3v(const float *a) { return v3(a[0], a[1], a[2]); }

HD V3 diffuseRefl(const HptMeshBsdf &b, float u, float v) {
    if (!b.textured) return f3v(b.refl);
    /* texture.cpp:113 then checkerboard.cpp:65-73 */
    const float x0 = u * b.uscale + b.uoffset, y0 = v * b.vscale + b.voffset;
    auto modulo2 = [](int a) { const int r = a % 2; return r < 0 ? r + 2 : r; };
    const int x = 2 * modulo2((int) (x0 * 2)) - 1, y = 2 * modulo2((int) (y0 * 2)) - 1;
    return x * y == 1 ? f3v(b.color0) : f3v(b.color1);
}

HD V3 plasticDiffuseTerm(const HptMeshBsdf &b) { /* plastic.cpp:266-271 */
    V3 diff = f3v(b.diffuse);
    if (b.nonlinear) return v3(diff.x / (1.0f - diff.x * b.fdrInt), diff.y / (1.0f - diff.y * b.fdrInt),
                               diff.z / (1.0f - diff.z * b.fdrInt));
    return divs(diff, 1 - b.fdrInt);
}
HD float plasticProbSpecular(const HptMeshBsdf &b, float Fi) { /* :292-294 */
    const float w = b.specularSamplingWeight;
    return (Fi * w) / (Fi * w + (1 - Fi) * (1 - w));
}

/* a non-twosided record: diffuse or plastic (the solid-angle eval / pdf path.cpp asks for) */
HD V3 leafEval(const HptMeshBsdf &b, V3 wi, V3 wo, float u, float v) {
    if (wi.z <= 0 || wo.z <= 0) return v3(0, 0, 0);
    if (b.kind == HPT_MBSDF_DIFFUSE) return diffuseRefl(b, u, v) * (kInvPi * wo.z);
    const float Fi = fresnelDielectricExt(wi.z, b.eta), Fo = fresnelDielectricExt(wo.z, b.eta);
    return plasticDiffuseTerm(b) * (kInvPi * wo.z * b.invEta2 * (1 - Fi) * (1 - Fo));
}
HD float leafPdf(const HptMeshBsdf &b, V3 wi, V3 wo) {
    if (wi.z <= 0 || wo.z <= 0) return 0.0f;
    if (b.kind == HPT_MBSDF_DIFFUSE) return kInvPi * wo.z;
    const float pSpec = plasticProbSpecular(b, fresnelDielectricExt(wi.z, b.eta));
    return kInvPi * wo.z * (1 - pSpec);
}
HD V3 leafSample(const HptMeshBsdf &b, V3 wi, float sx, float sy, float u, float v, V3 &wo, float &pdf, uint32_t &type) {
    pdf = 0.0f;
    type = 0;
    if (wi.z <= 0) return v3(0, 0, 0);
    if (b.kind == HPT_MBSDF_DIFFUSE) {
        wo = squareToCosineHemisphere(sx, sy);
        type = HPT_EDIFFUSE_REFLECTION;
        pdf = kInvPi * wo.z;
        return diffuseRefl(b, u, v);
    }
    const float Fi = fresnelDielectricExt(wi.z, b.eta), pSpec = plasticProbSpecular(b, Fi);
    if (sx < pSpec) { /* plastic.cpp:383-392 */
        type = HPT_EDELTA_REFLECTION;
        wo = v3(-wi.x, -wi.y, wi.z);
        pdf = pSpec;
        return divs(f3v(b.specular) * Fi, pSpec);
    }
    type = HPT_EDIFFUSE_REFLECTION;
    wo = squareToCosineHemisphere((sx - pSpec) / (1 - pSpec), sy);
    const float Fo = fresnelDielectricExt(wo.z, b.eta);
    pdf = (1 - pSpec) * (kInvPi * wo.z);
    return plasticDiffuseTerm(b) * (b.invEta2 * (1 - Fi) * (1 - Fo) / (1 - pSpec));
}

/* TwoSidedBRDF (twosided.cpp:108-183) over its leaf records; other records as they are */
HD V3 meshBsdfEval(const HptMeshScene &ms, int bi, V3 wi, V3 wo, float u, float v) {
    const HptMeshBsdf &b = ms.bsdfs[bi];
    if (b.kind != HPT_MBSDF_TWOSIDED) return leafEval(b, wi, wo, u, v);
    if (wi.z > 0) return leafEval(ms.bsdfs[b.nested[0]], wi, wo, u, v);
    return leafEval(ms.bsdfs[b.nested[1]], v3(wi.x, wi.y, -wi.z), v3(wo.x, wo.y, -wo.z), u, v);
}
HD float meshBsdfPdf(const HptMeshScene &ms, int bi, V3 wi, V3 wo) {
    const HptMeshBsdf &b = ms.bsdfs[bi];
    if (b.kind != HPT_MBSDF_TWOSIDED) return leafPdf(b, wi, wo);
    if (wi.z > 0) return leafPdf(ms.bsdfs[b.nested[0]], wi, wo);
    return leafPdf(ms.bsdfs[b.nested[1]], v3(wi.x, wi.y, -wi.z), v3(wo.x, wo.y, -wo.z));
}
HD V3 meshBsdfSample(const HptMeshScene &ms, int bi, V3 wi, float sx, float sy, float u, float v, V3 &wo, float &pdf,
                     uint32_t &type) {
    const HptMeshBsdf &b = ms.bsdfs[bi];
    if (b.kind != HPT_MBSDF_TWOSIDED) return leafSample(b, wi, sx, sy, u, v, wo, pdf, type);
    const bool flipped = wi.z < 0;
    const V3 w = flipped ? v3(wi.x, wi.y, -wi.z) : wi;
    const V3 r = leafSample(ms.bsdfs[b.nested[flipped ? 1 : 0]], w, sx, sy, u, v, wo, pdf, type);
    if (flipped && !isZero(r) && pdf != 0) wo.z = -wo.z;
    return r;
}

} // namespace

/* one lane per camera sample of the wave (path id as k_camera decodes it): the camera ray,
   then path.cpp:119-294 to termination; the sample's film position and radiance go to
   P.pos / P.li for k_splat.  counters: HPT_C_BOUNCES (path-bounces), HPT_C_ERROR (Sobol
   dimensions exhausted) */
extern "C" __global__ __launch_bounds__(HPT_MESH_BLOCK) void k_mesh_paths(HptScene sc, HptMeshScene ms, HptWave w,
                                                                          HptPaths P, uint32_t *__restrict__ counters) {
    /* the BVH stacks in LDS (a lane's column, conflict-free), shared by the lane's closest and shadow
       queries: 32 entries x 256 lanes = 32 KB per block */
    __shared__ uint32_t stackLds[HPT_MESH_STACK * HPT_MESH_BLOCK];
    uint32_t *const stk = stackLds + threadIdx.x;
    const uint32_t id = blockIdx.x * blockDim.x + threadIdx.x;
    int px = 0, py = 0;
    uint32_t j = 0;
    const bool valid = id < w.nPaths && decodePath(w, id, px, py, j);
    uint64_t bounces = 0;
    bool error = false;
    if (valid) {
        const HptCamera &c = sc.cam;
        /* k_camera's sample (sampler->generate + next2D, integrator.cpp:165-178) */
        const uint32_t lastFrame = w.sppBegin + w.nSpp - 1u;
        const uint32_t frameBits = lastFrame ? 32u - (uint32_t) __builtin_clz(lastFrame) : 0u;
        const uint64_t sidx = (c.logRes > 1) ? sobolLookUpWave(sc, c.logRes, j, (uint32_t) px, (uint32_t) py, frameBits)
                                             : (uint64_t) j;
        float ox, oy;
        if (sidx != (uint64_t) j) {
            ox = sobolSample(sc, sidx, 0) * c.resolution - px;
            oy = sobolSample(sc, sidx, 1) * c.resolution - py;
        } else {
            ox = sobolSample(sc, sidx, 0);
            oy = sobolSample(sc, sidx, 1);
        }
        const float posx = px + ox, posy = py + oy;
        V3 ro, rd;
        float mint, maxt;
        cameraRay(c, posx, posy, ro, rd, mint, maxt);
        uint32_t dim = 2;
        V3 Li = v3(0, 0, 0), T = v3(1, 1, 1);
        bool scattered = false, emitted = true, primary = true;
        int depth = 1;
        MeshHit h;
        MeshIts its;
        bool hitValid = meshIntersect(ms, ro, rd, mint, maxt, h, stk);
        if (hitValid) meshFill(ms, ro, rd, h, its);
        while (depth <= sc.maxDepth || sc.maxDepth < 0) {
            if (!hitValid) {
                if (emitted && (!sc.hideEmitters || scattered)) {
                    if (primary) { /* a camera ray keeps its differentials: the EWA lookup (envmap.cpp:394-406) */
                        V3 rx, ry;
                        cameraDifferentials(c, posx, posy, rd, rx, ry);
                        Li = Li + mul(T, envEvalFiltered(sc.env, rd, rx, ry));
                    } else {
                        Li = Li + mul(T, envEval(sc.env, rd));
                    }
                }
                break;
            }
            if ((depth >= sc.maxDepth && sc.maxDepth > 0) || (sc.strictNormals && dot(rd, its.geo.n) * its.wi.z >= 0))
                break;
            if (dim + 3 >= HPT_SOBOL_DIMS) { /* sobol.cpp:236-238 */
                error = true;
                break;
            }
            ++bounces;
            const int bi = its.bsdf;
            const bool smooth = ms.bsdfs[bi].smooth != 0;
            /* direct illumination (path.cpp:170-199; scene.cpp:828-852; envmap.cpp:516-543) */
            if (smooth) {
                const float nx = sobolSample(sc, sidx, dim), ny = sobolSample(sc, sidx, dim + 1);
                dim += 2;
                V3 dl, value;
                float pdf;
                envSampleDir(sc.env, nx, ny, dl, value, pdf);
                const V3 dW = envToWorld(sc.env, dl);
                float nearT, farT;
                if (!(isZero(value) || pdf == 0 || !bsphereIntersect(sc.env, its.p, dW, nearT, farT) || nearT >= 0 ||
                      farT <= 0) &&
                    !meshOccluded(ms, its.p, dW, kEpsilon, farT * (1 - kShadowEpsilon), stk)) {
                    const V3 val = divs(value, pdf);
                    const V3 wo = its.sh.toLocal(dW);
                    const V3 bsdfVal = meshBsdfEval(ms, bi, its.wi, wo, its.u, its.v);
                    if (!isZero(bsdfVal) && (!sc.strictNormals || dot(its.geo.n, dW) * wo.z > 0)) {
                        const float bp = meshBsdfPdf(ms, bi, its.wi, wo);
                        Li = Li + mul(mul(T, val), bsdfVal) * miWeight(pdf, bp);
                    }
                }
            }
            /* BSDF sampling (path.cpp:206-221) */
            const float bx = sobolSample(sc, sidx, dim), by = sobolSample(sc, sidx, dim + 1);
            dim += 2;
            V3 woL;
            float bpdf = 0.0f;
            uint32_t type = 0;
            const V3 bw = meshBsdfSample(ms, bi, its.wi, bx, by, its.u, its.v, woL, bpdf, type);
            if (isZero(bw)) break;
            scattered |= type != HPT_ENULL;
            const V3 wo = its.sh.toWorld(woL);
            if (sc.strictNormals && dot(its.geo.n, wo) * woL.z <= 0) break;
            /* the continuation ray (path.cpp:225-264) */
            ro = its.p;
            rd = wo;
            primary = false;
            bool hitEmitter = false;
            V3 value = v3(0, 0, 0);
            hitValid = meshIntersect(ms, ro, rd, kEpsilon, finf(), h, stk);
            if (hitValid) {
                meshFill(ms, ro, rd, h, its);
            } else {
                if (sc.hideEmitters && !scattered) break;
                value = envEval(sc.env, rd);
                float nearT, farT;
                if (!bsphereIntersect(sc.env, ro, rd, nearT, farT) || nearT > 0 || farT < 0) break;
                hitEmitter = true;
            }
            T = mul(T, bw);
            if (hitEmitter) {
                const float lumPdf = !(type & HPT_EDELTA) ? envPdf(sc.env, envToLocal(sc.env, rd)) : 0.0f;
                Li = Li + mul(T, value) * miWeight(bpdf, lumPdf);
            }
            if (!hitValid) break;
            emitted = false;
            if (depth++ >= sc.rrDepth) { /* Russian roulette (path.cpp:270-286), eta = 1 */
                const float q = fminr(maxc(T) * 1.0f * 1.0f, 0.95f);
                if (sobolSample(sc, sidx, dim++) >= q) break;
                T = divs(T, q);
            }
        }
        P.pos[id] = make_float2(posx, posy);
        P.li[id] = make_float4(Li.x, Li.y, Li.z, 0.0f);
    }
    /* the wave's path-bounces, one atomic per wave */
    uint64_t sum = bounces;
#pragma unroll
    for (int off = 32; off > 0; off >>= 1) sum += __shfl_xor(sum, off);
    const uint64_t errs = __ballot(error);
    if (__lane_id() == 0) {
        if (sum) atomicAdd((unsigned long long *) (counters + HPT_C_BOUNCES), (unsigned long long) sum);
        if (errs) atomicOr(&counters[HPT_C_ERROR], 1u);
    }
}

hipError_t hpt_launch_mesh_paths(const HptScene &sc, const HptMeshScene &ms, const HptWave &w, const HptPaths &P,
                                 uint32_t *counters, hipStream_t s) {
    if (w.nPaths == 0) return hipSuccess;
    hipLaunchKernelGGL(k_mesh_paths, dim3((w.nPaths + HPT_MESH_BLOCK - 1) / HPT_MESH_BLOCK), dim3(HPT_MESH_BLOCK), 0, s,
                       sc, ms, w, P, counters);
    return hipGetLastError();
}
