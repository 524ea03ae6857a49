/*
 * mesh_bsdf.h -- oracle restatement of the BSDFs and the texture of the C1
 * "teapot" plumbing scene (BASELINE.json configs[0], models/teapot/scene.xml):
 *
 *   SmoothPlastic            src/bsdfs/plastic.cpp:143-440 (constant reflectances)
 *   fresnelDiffuseReflectance src/libcore/util.cpp:808-859 (fast = false)
 *   Checkerboard             src/textures/checkerboard.cpp:47-100 over the uv
 *                            transform of Texture2D::eval, src/librender/texture.cpp:81-121
 *   (TwoSidedBRDF, src/bsdfs/twosided.cpp:84-183, lives in BsdfInst: it nests BsdfInsts)
 *
 * TEST INFRASTRUCTURE ONLY (see oracle.h).  Included by oracle.cpp inside its
 * anonymous namespace, after ref_core.h; no includes of its own.
 */

/* util.cpp:856-858: GaussLobattoIntegrator(1024, 0, 1e-5f) of fresnelDielectricExt(sqrt(xi), eta) */
inline float fresnelDiffuseReflectance(float eta) {
    const orc_quad::Lobatto quad(1024, 0, 1e-5f, true);
    return quad.integrate([eta](float xi) { return fresnelDielectricExt(std::sqrt(xi), eta); }, 0, 1);
}

struct Checkerboard {
    Spec color0{0.4f}, color1{0.2f};
    float uoffset = 0, voffset = 0, uscale = 1, vscale = 1;
    Spec eval(float u, float v) const {
        /* texture.cpp:113: uv * scale + offset */
        const float x0 = u * uscale + uoffset, y0 = v * vscale + voffset;
        /* checkerboard.cpp:65-73 */
        const int x = 2 * modulo((int) (x0 * 2), 2) - 1, y = 2 * modulo((int) (y0 * 2), 2) - 1;
        return x * y == 1 ? color0 : color1;
    }
    Spec maximum() const { /* :85-90 */
        return Spec(std::max(color0.s[0], color1.s[0]), std::max(color0.s[1], color1.s[1]),
                    std::max(color0.s[2], color1.s[2]));
    }
};

struct SmoothPlastic {
    float eta = 1.49f; /* intIOR / extIOR (:147-156); polypropylene / air by default */
    bool nonlinear = false;
    Spec diffuse{0.5f}, specular{1.0f};
    float fdrInt = 0, fdrExt = 0, specularSamplingWeight = 0, invEta2 = 0;

    bool ensureEnergyConservation = true; /* BSDF::BSDF, bsdf.cpp:30-31 */
    void configure() { /* :186-217; BSDF::ensureEnergyConservation, bsdf.cpp:88-113 */
        float mx = specular.max();
        if (ensureEnergyConservation && mx > 1.0f) specular *= 0.99f * (1.0f / mx);
        mx = diffuse.max();
        if (ensureEnergyConservation && mx > 1.0f) diffuse *= 0.99f * (1.0f / mx);
        fdrInt = fresnelDiffuseReflectance(1 / eta);
        fdrExt = fresnelDiffuseReflectance(eta);
        const float dAvg = diffuse.getLuminance(), sAvg = specular.getLuminance();
        specularSamplingWeight = sAvg / (dAvg + sAvg);
        invEta2 = 1 / (eta * eta);
    }
    static V3 reflect(const V3 &wi) { return V3(-wi.x, -wi.y, wi.z); }
    Spec diffuseTerm() const { /* :266-271 */
        Spec diff = diffuse;
        if (nonlinear)
            diff /= Spec(1.0f) - diff * fdrInt;
        else
            diff /= 1 - fdrInt;
        return diff;
    }
    float probSpecular(float Fi) const { /* :292-294 */
        return (Fi * specularSamplingWeight) / (Fi * specularSamplingWeight + (1 - Fi) * (1 - specularSamplingWeight));
    }
    /* eval / pdf in ESolidAngle (what MIPathTracer asks for): the diffuse lobe only */
    Spec eval(const V3 &wi, const V3 &wo) const { /* :245-278 */
        if (wo.z <= 0 || wi.z <= 0) return Spec(0.0f);
        const float Fi = fresnelDielectricExt(wi.z, eta), Fo = fresnelDielectricExt(wo.z, eta);
        return diffuseTerm() * (kInvPi * wo.z * invEta2 * (1 - Fi) * (1 - Fo));
    }
    float pdf(const V3 &wi, const V3 &wo) const { /* :280-307 */
        if (wo.z <= 0 || wi.z <= 0) return 0.0f;
        const float pSpec = probSpecular(fresnelDielectricExt(wi.z, eta));
        return kInvPi * wo.z * (1 - pSpec);
    }
    Spec sample(const V3 &wi, float sx, float sy, V3 &wo, float &pdfOut, uint32_t &type) const { /* :372-417 */
        pdfOut = 0;
        type = 0;
        if (wi.z <= 0) return Spec(0.0f);
        const float Fi = fresnelDielectricExt(wi.z, eta);
        const float pSpec = probSpecular(Fi);
        if (sx < pSpec) {
            type = EDeltaReflection;
            wo = reflect(wi);
            pdfOut = pSpec;
            return specular * Fi / pSpec;
        }
        type = EDiffuseReflection;
        wo = squareToCosineHemisphere((sx - pSpec) / (1 - pSpec), sy);
        const float Fo = fresnelDielectricExt(wo.z, eta);
        pdfOut = (1 - pSpec) * (kInvPi * wo.z);
        return diffuseTerm() * (invEta2 * (1 - Fi) * (1 - Fo) / (1 - pSpec));
    }
};
