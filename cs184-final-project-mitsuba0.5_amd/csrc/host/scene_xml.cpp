/*
 * scene_xml.cpp -- Mitsuba 0.5 scene-XML front end for the hair path.
 *
 * Follows the reference's SceneHandler semantics (librender/scenehandler.cpp)
 * for the subset of the schema (data/schema/scene.xsd) that the bundled
 * models/ scenes use:
 *   - <default name value> supplies $name when no -D define overrides it
 *     (scenehandler.cpp:684-686), $name substitution in every attribute
 *     (scenehandler.cpp:210-219);
 *   - typed properties <integer|float|boolean|string|rgb|spectrum|vector|point>;
 *   - <transform> built from <matrix>, <lookat>, <translate>, <rotate>, <scale>
 *     (later elements pre-multiply, scenehandler.cpp transform handling);
 *   - objects: integrator, sensor(+sampler, film(+rfilter)), bsdf (top level
 *     with id or nested), shape type="hair", emitter (sunsky / envmap), <ref>.
 * Unsupported plugin types raise an error naming the plugin, as the reference
 * does for unknown plugins.
 */
#include <cctype>
#include <cmath>
#include <cstring>
#include <fstream>
#include <sstream>
#include <stdexcept>

#include "host_scene.h"

namespace hpt {
namespace {

struct XNode {
    std::string tag;
    std::vector<std::pair<std::string, std::string>> attrs;
    std::vector<std::unique_ptr<XNode>> kids;
    int line = 0;
    const std::string *attr(const std::string &k) const {
        for (auto &a : attrs)
            if (a.first == k) return &a.second;
        return nullptr;
    }
};

[[noreturn]] void fail(const std::string &file, int line, const std::string &msg) {
    std::ostringstream o;
    o << file << ":" << line << ": " << msg;
    throw std::runtime_error(o.str());
}

/* Minimal non-validating XML reader: elements, attributes, comments, PIs. */
std::unique_ptr<XNode> parseXML(const std::string &text, const std::string &file) {
    size_t i = 0, n = text.size();
    int line = 1;
    auto adv = [&](size_t k) {
        for (size_t j = 0; j < k && i < n; ++j, ++i)
            if (text[i] == '\n') ++line;
    };
    auto skipWs = [&]() {
        while (i < n && std::isspace((unsigned char) text[i])) adv(1);
    };
    std::vector<XNode *> stack;
    std::unique_ptr<XNode> root;
    while (i < n) {
        if (text[i] != '<') { adv(1); continue; }
        if (text.compare(i, 4, "<!--") == 0) {
            size_t e = text.find("-->", i + 4);
            if (e == std::string::npos) fail(file, line, "unterminated comment");
            adv(e + 3 - i);
            continue;
        }
        if (text.compare(i, 2, "<?") == 0 || text.compare(i, 2, "<!") == 0) {
            size_t e = text.find('>', i);
            if (e == std::string::npos) fail(file, line, "unterminated declaration");
            adv(e + 1 - i);
            continue;
        }
        if (text.compare(i, 2, "</") == 0) {
            size_t e = text.find('>', i);
            if (e == std::string::npos) fail(file, line, "unterminated end tag");
            std::string name = text.substr(i + 2, e - i - 2);
            while (!name.empty() && std::isspace((unsigned char) name.back())) name.pop_back();
            if (stack.empty() || stack.back()->tag != name)
                fail(file, line, "mismatched end tag </" + name + ">");
            stack.pop_back();
            adv(e + 1 - i);
            continue;
        }
        adv(1);
        size_t s = i;
        while (i < n && !std::isspace((unsigned char) text[i]) && text[i] != '>' && text[i] != '/') adv(1);
        std::unique_ptr<XNode> node(new XNode());
        node->tag = text.substr(s, i - s);
        node->line = line;
        bool selfClose = false;
        while (true) {
            skipWs();
            if (i >= n) fail(file, line, "unexpected end of file");
            if (text[i] == '/') {
                selfClose = true;
                adv(1);
                skipWs();
                if (i >= n || text[i] != '>') fail(file, line, "expected '>'");
                adv(1);
                break;
            }
            if (text[i] == '>') { adv(1); break; }
            size_t ks = i;
            while (i < n && text[i] != '=' && !std::isspace((unsigned char) text[i])) adv(1);
            std::string key = text.substr(ks, i - ks);
            skipWs();
            if (i >= n || text[i] != '=') fail(file, line, "expected '=' after attribute " + key);
            adv(1);
            skipWs();
            if (i >= n || (text[i] != '"' && text[i] != '\'')) fail(file, line, "expected quoted value");
            char q = text[i];
            adv(1);
            size_t vs = i;
            while (i < n && text[i] != q) adv(1);
            std::string val = text.substr(vs, i - vs);
            adv(1);
            node->attrs.push_back({key, val});
        }
        XNode *raw = node.get();
        if (stack.empty()) {
            if (root) fail(file, line, "multiple root elements");
            root = std::move(node);
        } else {
            stack.back()->kids.push_back(std::move(node));
        }
        if (!selfClose) stack.push_back(raw);
    }
    if (!stack.empty()) fail(file, line, "unterminated element <" + stack.back()->tag + ">");
    if (!root) fail(file, line, "empty document");
    return root;
}

struct Ctx {
    std::string file;
    std::map<std::string, std::string> defines;
    std::map<std::string, const XNode *> ids;
    std::map<const XNode *, int> bsdfIndex; /* one instance per <bsdf> element, shared by its refs */
};

std::string subst(const Ctx &c, const XNode &nd, const std::string &v) {
    /* scenehandler.cpp:210-219: replace $key by its value for every define */
    std::string out = v;
    for (auto &kv : c.defines) {
        std::string key = "$" + kv.first;
        size_t pos = 0;
        while ((pos = out.find(key, pos)) != std::string::npos) {
            out.replace(pos, key.size(), kv.second);
            pos += kv.second.size();
        }
    }
    if (out.find('$') != std::string::npos)
        fail(c.file, nd.line, "unresolved parameter in \"" + v + "\"");
    return out;
}

std::string attrS(const Ctx &c, const XNode &nd, const char *k, bool required = true) {
    const std::string *v = nd.attr(k);
    if (!v) {
        if (required) fail(c.file, nd.line, std::string("<") + nd.tag + "> lacks attribute '" + k + "'");
        return std::string();
    }
    return subst(c, nd, *v);
}

float toF(const Ctx &c, const XNode &nd, const std::string &s) {
    char *end = nullptr;
    float v = std::strtof(s.c_str(), &end);
    if (end == s.c_str()) fail(c.file, nd.line, "cannot parse float \"" + s + "\"");
    return v;
}

std::vector<float> toFloats(const Ctx &c, const XNode &nd, const std::string &s) {
    std::vector<float> out;
    std::string t = s;
    for (auto &ch : t)
        if (ch == ',') ch = ' ';
    std::istringstream is(t);
    std::string tok;
    while (is >> tok) out.push_back(toF(c, nd, tok));
    return out;
}

void matMul(const float *a, const float *b, float *out) {
    float r[16];
    for (int i = 0; i < 4; ++i)
        for (int j = 0; j < 4; ++j) {
            float acc = 0;
            for (int k = 0; k < 4; ++k) acc += a[i * 4 + k] * b[k * 4 + j];
            r[i * 4 + j] = acc;
        }
    std::memcpy(out, r, sizeof(r));
}

void parseTransform(const Ctx &c, const XNode &t, float *M) {
    float acc[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
    for (auto &kp : t.kids) {
        const XNode &k = *kp;
        float m[16] = {1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1, 0, 0, 0, 0, 1};
        if (k.tag == "matrix") {
            std::vector<float> v = toFloats(c, k, attrS(c, k, "value"));
            if (v.size() != 16) fail(c.file, k.line, "matrix needs 16 values");
            for (int i = 0; i < 16; ++i) m[i] = v[i];
        } else if (k.tag == "translate") {
            m[3] = k.attr("x") ? toF(c, k, attrS(c, k, "x")) : 0;
            m[7] = k.attr("y") ? toF(c, k, attrS(c, k, "y")) : 0;
            m[11] = k.attr("z") ? toF(c, k, attrS(c, k, "z")) : 0;
        } else if (k.tag == "scale") {
            if (k.attr("value")) {
                float s = toF(c, k, attrS(c, k, "value"));
                m[0] = m[5] = m[10] = s;
            } else {
                m[0] = k.attr("x") ? toF(c, k, attrS(c, k, "x")) : 1;
                m[5] = k.attr("y") ? toF(c, k, attrS(c, k, "y")) : 1;
                m[10] = k.attr("z") ? toF(c, k, attrS(c, k, "z")) : 1;
            }
        } else if (k.tag == "rotate") {
            /* transform.cpp Transform::rotate (Rodrigues, angle in degrees) */
            double x = k.attr("x") ? toF(c, k, attrS(c, k, "x")) : 0;
            double y = k.attr("y") ? toF(c, k, attrS(c, k, "y")) : 0;
            double z = k.attr("z") ? toF(c, k, attrS(c, k, "z")) : 0;
            double ang = toF(c, k, attrS(c, k, "angle")) * M_PI / 180.0;
            double len = std::sqrt(x * x + y * y + z * z);
            x /= len; y /= len; z /= len;
            double s = std::sin(ang), co = std::cos(ang), t1 = 1 - co;
            double r[9] = {x * x * t1 + co, x * y * t1 - z * s, x * z * t1 + y * s,
                           x * y * t1 + z * s, y * y * t1 + co, y * z * t1 - x * s,
                           x * z * t1 - y * s, y * z * t1 + x * s, z * z * t1 + co};
            for (int i = 0; i < 3; ++i)
                for (int j = 0; j < 3; ++j) m[i * 4 + j] = (float) r[i * 3 + j];
        } else if (k.tag == "lookat") {
            std::vector<float> o = toFloats(c, k, attrS(c, k, "origin"));
            std::vector<float> tg = toFloats(c, k, attrS(c, k, "target"));
            std::vector<float> up = k.attr("up") ? toFloats(c, k, attrS(c, k, "up")) : std::vector<float>{0, 1, 0};
            if (o.size() != 3 || tg.size() != 3 || up.size() != 3) fail(c.file, k.line, "bad lookat");
            double d[3] = {tg[0] - o[0], tg[1] - o[1], tg[2] - o[2]};
            double dl = std::sqrt(d[0] * d[0] + d[1] * d[1] + d[2] * d[2]);
            for (auto &v : d) v /= dl;
            double u[3] = {up[0], up[1], up[2]};
            double left[3] = {u[1] * d[2] - u[2] * d[1], u[2] * d[0] - u[0] * d[2], u[0] * d[1] - u[1] * d[0]};
            double ll = std::sqrt(left[0] * left[0] + left[1] * left[1] + left[2] * left[2]);
            for (auto &v : left) v /= ll;
            double nu[3] = {d[1] * left[2] - d[2] * left[1], d[2] * left[0] - d[0] * left[2],
                            d[0] * left[1] - d[1] * left[0]};
            for (int i = 0; i < 3; ++i) {
                m[i * 4 + 0] = (float) left[i];
                m[i * 4 + 1] = (float) nu[i];
                m[i * 4 + 2] = (float) d[i];
                m[i * 4 + 3] = o[i];
            }
        } else {
            fail(c.file, k.line, "unsupported transform element <" + k.tag + ">");
        }
        matMul(m, acc, acc);
    }
    std::memcpy(M, acc, sizeof(acc));
}

struct Props {
    std::map<std::string, std::string> str;
    std::map<std::string, std::vector<float>> num;
    std::map<std::string, const XNode *> xform;
};

void collectProps(const Ctx &c, const XNode &nd, Props &p) {
    for (auto &kp : nd.kids) {
        const XNode &k = *kp;
        if (k.tag == "integer" || k.tag == "float") {
            p.num[attrS(c, k, "name")] = {toF(c, k, attrS(c, k, "value"))};
        } else if (k.tag == "boolean") {
            std::string v = attrS(c, k, "value");
            for (auto &ch : v) ch = (char) std::tolower((unsigned char) ch);
            p.num[attrS(c, k, "name")] = {(v == "true" || v == "1") ? 1.0f : 0.0f};
        } else if (k.tag == "string") {
            p.str[attrS(c, k, "name")] = attrS(c, k, "value");
        } else if (k.tag == "rgb" || k.tag == "spectrum" || k.tag == "srgb") {
            std::vector<float> v = toFloats(c, k, attrS(c, k, "value"));
            if (v.size() == 1) v = {v[0], v[0], v[0]};
            if (v.size() != 3) fail(c.file, k.line, "<" + k.tag + "> needs 1 or 3 values");
            if (k.tag == "srgb") /* sRGB -> linear */
                for (auto &x : v)
                    x = x <= 0.04045f ? x / 12.92f : std::pow((x + 0.055f) / 1.055f, 2.4f);
            p.num[attrS(c, k, "name")] = v;
        } else if (k.tag == "vector" || k.tag == "point") {
            float x = k.attr("x") ? toF(c, k, attrS(c, k, "x")) : 0;
            float y = k.attr("y") ? toF(c, k, attrS(c, k, "y")) : 0;
            float z = k.attr("z") ? toF(c, k, attrS(c, k, "z")) : 0;
            p.num[attrS(c, k, "name")] = {x, y, z};
        } else if (k.tag == "transform") {
            p.xform[attrS(c, k, "name")] = &k;
        }
    }
}

float num1(const Props &p, const char *k, float def) {
    auto it = p.num.find(k);
    return it == p.num.end() ? def : it->second[0];
}
bool has(const Props &p, const char *k) { return p.num.count(k) || p.str.count(k); }

float lookupIOR(const Ctx &c, const XNode &nd, const Props &p, const char *key, const char *def) {
    /* ior.h:43-108 */
    static const std::pair<const char *, float> table[] = {
        {"vacuum", 1.0f}, {"helium", 1.000036f}, {"hydrogen", 1.000132f}, {"air", 1.000277f},
        {"carbon dioxide", 1.00045f}, {"water", 1.3330f}, {"acetone", 1.36f}, {"ethanol", 1.361f},
        {"carbon tetrachloride", 1.461f}, {"glycerol", 1.4729f}, {"benzene", 1.501f},
        {"silicone oil", 1.52045f}, {"bromine", 1.661f}, {"water ice", 1.31f}, {"fused quartz", 1.458f},
        {"pyrex", 1.470f}, {"acrylic glass", 1.49f}, {"polypropylene", 1.49f}, {"bk7", 1.5046f},
        {"sodium chloride", 1.544f}, {"amber", 1.55f}, {"pet", 1.5750f}, {"diamond", 2.419f}};
    auto it = p.num.find(key);
    if (it != p.num.end()) return it->second[0];
    std::string name = def;
    auto st = p.str.find(key);
    if (st != p.str.end()) name = st->second;
    for (auto &ch : name) ch = (char) std::tolower((unsigned char) ch);
    for (auto &e : table)
        if (name == e.first) return e.second;
    fail(c.file, nd.line, "Unable to find an IOR value for \"" + name + "\"");
}

/* <texture type="checkerboard"> (checkerboard.cpp:47-52, texture.cpp:81-95) */
void parseTexture(const Ctx &c, const XNode &t, TextureDesc &x) {
    x.type = attrS(c, t, "type");
    if (x.type != "checkerboard")
        fail(c.file, t.line, "texture \"" + x.type + "\" is outside this path (only \"checkerboard\")");
    Props p;
    collectProps(c, t, p);
    for (int i = 0; i < 3; ++i) {
        x.color0[i] = p.num.count("color0") ? p.num["color0"][i] : 0.4f;
        x.color1[i] = p.num.count("color1") ? p.num["color1"][i] : 0.2f;
    }
    if (p.str.count("coordinates") && p.str["coordinates"] != "uv")
        fail(c.file, t.line, "Only UV coordinates are supported at the moment!");
    x.uoffset = num1(p, "uoffset", 0.0f);
    x.voffset = num1(p, "voffset", 0.0f);
    const float uvscale = num1(p, "uvscale", 1.0f);
    x.uscale = num1(p, "uscale", uvscale);
    x.vscale = num1(p, "vscale", uvscale);
}

void parseBSDF(const Ctx &c, const XNode &b, BsdfDesc &d) {
    std::string type = attrS(c, b, "type");
    Props p;
    collectProps(c, b, p);
    d.type = type;
    if (type == "marschner") {
        /* marschner_diffuse.cpp:113-160 (plugin "marschner", SConscript:38) */
        d.intIOR = lookupIOR(c, b, p, "intIOR", "bk7");
        d.extIOR = lookupIOR(c, b, p, "extIOR", "air");
        if (p.str.count("distribution")) {
            std::string v = p.str["distribution"];
            for (auto &ch : v) ch = (char) std::tolower((unsigned char) ch);
            if (v == "as") v = "phong";
            if (v != "beckmann" && v != "ggx" && v != "phong")
                fail(c.file, b.line, "Specified an invalid distribution \"" + v + "\"");
            d.distribution = v;
        }
        d.alpha = num1(p, "alpha", 0.1f);
        if (p.num.count("alphaU") || p.num.count("alphaV"))
            d.alpha = num1(p, "alphaU", 0.1f);
        if (p.num.count("diffuseReflectance")) {
            auto &v = p.num["diffuseReflectance"];
            for (int i = 0; i < 3; ++i) d.diffuse[i] = v[i];
        } else {
            d.diffuse[0] = d.diffuse[1] = d.diffuse[2] = 0.5f;
        }
        if (p.num.count("specularReflectance")) {
            auto &v = p.num["specularReflectance"];
            for (int i = 0; i < 3; ++i) d.specular[i] = v[i];
        } else {
            d.specular[0] = d.specular[1] = d.specular[2] = 0.5f;
        }
        d.exponent = num1(p, "exponent", 30.0f);
        d.nonlinear = num1(p, "nonlinear", 0.0f) != 0.0f;
    } else if (type == "kajiyakay") {
        /* kajiyakay.cpp:60-69 */
        if (p.num.count("diffuseReflectance")) {
            auto &v = p.num["diffuseReflectance"];
            for (int i = 0; i < 3; ++i) d.diffuse[i] = v[i];
        } else {
            d.diffuse[0] = d.diffuse[1] = d.diffuse[2] = 0.5f;
        }
        if (p.num.count("specularReflectance")) {
            auto &v = p.num["specularReflectance"];
            for (int i = 0; i < 3; ++i) d.specular[i] = v[i];
        } else {
            d.specular[0] = d.specular[1] = d.specular[2] = 0.2f;
        }
        d.exponent = num1(p, "exponent", 30.0f);
    } else if (type == "roughplastic") {
        /* roughplastic.cpp:197-227 + MicrofacetDistribution(props) (microfacet.h:99-144) */
        d.intIOR = lookupIOR(c, b, p, "intIOR", "polypropylene");
        d.extIOR = lookupIOR(c, b, p, "extIOR", "air");
        if (d.intIOR < 0 || d.extIOR < 0 || d.intIOR == d.extIOR)
            fail(c.file, b.line, "The interior and exterior indices of refraction must be positive and differ!");
        d.distribution = "beckmann";
        if (p.str.count("distribution")) {
            std::string v = p.str["distribution"];
            for (auto &ch : v) ch = (char) std::tolower((unsigned char) ch);
            if (v == "as") v = "phong";
            if (v != "beckmann" && v != "ggx" && v != "phong")
                fail(c.file, b.line, "Specified an invalid distribution \"" + v +
                                         "\", must be \"beckmann\", \"ggx\", or \"phong\"/\"as\"!");
            d.distribution = v;
        }
        const bool hasA = p.num.count("alpha") != 0, hasU = p.num.count("alphaU") != 0,
                   hasV = p.num.count("alphaV") != 0;
        d.alpha = 0.1f;
        if (hasA) {
            if (hasU || hasV) fail(c.file, b.line, "Microfacet model: please specify either 'alpha' or 'alphaU'/'alphaV'.");
            d.alpha = num1(p, "alpha", 0.1f);
        } else if (hasU || hasV) {
            if (!(hasU && hasV)) fail(c.file, b.line, "Microfacet model: both 'alphaU' and 'alphaV' must be specified.");
            d.alpha = num1(p, "alphaU", 0.1f);
            if (std::max(num1(p, "alphaU", 0.1f), 1e-4f) != std::max(num1(p, "alphaV", 0.1f), 1e-4f))
                fail(c.file, b.line, "The 'roughplastic' plugin currently does not support anisotropic "
                                     "microfacet distributions!");
        }
        d.sampleVisible = num1(p, "sampleVisible", 1.0f) != 0.0f;
        d.nonlinear = num1(p, "nonlinear", 0.0f) != 0.0f;
        d.ensureEnergyConservation = num1(p, "ensureEnergyConservation", 1.0f) != 0.0f;
        for (int i = 0; i < 3; ++i) {
            d.diffuse[i] = p.num.count("diffuseReflectance") ? p.num["diffuseReflectance"][i] : 0.5f;
            d.specular[i] = p.num.count("specularReflectance") ? p.num["specularReflectance"][i] : 1.0f;
        }
    } else if (type == "marschnerdielectric") {
        /* marschnerdielectric.cpp:147-169 */
        d.intIOR = lookupIOR(c, b, p, "intIOR", "benzene");
        d.extIOR = lookupIOR(c, b, p, "extIOR", "air");
        if (d.intIOR < 0 || d.extIOR < 0)
            fail(c.file, b.line, "The interior and exterior indices of refraction must be positive!");
        for (int i = 0; i < 3; ++i) {
            d.diffuse[i] = p.num.count("diffuseReflectance") ? p.num["diffuseReflectance"][i] : 0.5f;
            d.specular[i] = p.num.count("specularReflectance") ? p.num["specularReflectance"][i] : 0.1f;
            d.transmittance[i] = p.num.count("specularTransmittance") ? p.num["specularTransmittance"][i] : 0.1f;
        }
        d.exponent = num1(p, "exponent", 30.0f); /* read by the plugin, unused on every evaluated branch */
        d.ensureEnergyConservation = num1(p, "ensureEnergyConservation", 1.0f) != 0.0f;
    } else if (type == "thindielectric") {
        /* thindielectric.cpp:73-89 */
        d.intIOR = lookupIOR(c, b, p, "intIOR", "bk7");
        d.extIOR = lookupIOR(c, b, p, "extIOR", "air");
        if (d.intIOR < 0 || d.extIOR < 0)
            fail(c.file, b.line, "The interior and exterior indices of refraction must be positive!");
        for (int i = 0; i < 3; ++i) {
            d.specular[i] = p.num.count("specularReflectance") ? p.num["specularReflectance"][i] : 1.0f;
            d.transmittance[i] = p.num.count("specularTransmittance") ? p.num["specularTransmittance"][i] : 1.0f;
        }
        d.ensureEnergyConservation = num1(p, "ensureEnergyConservation", 1.0f) != 0.0f;
    } else if (type == "diffuse") {
        /* diffuse.cpp:62-69: 'reflectance' or 'diffuseReflectance', a colour or a texture */
        const char *key = p.num.count("reflectance") ? "reflectance" : "diffuseReflectance";
        for (int i = 0; i < 3; ++i) d.diffuse[i] = p.num.count(key) ? p.num[key][i] : 0.5f;
        d.ensureEnergyConservation = num1(p, "ensureEnergyConservation", 1.0f) != 0.0f;
        for (auto &kp : b.kids)
            if (kp->tag == "texture") {
                const std::string name = attrS(c, *kp, "name", false);
                if (name != "reflectance" && name != "diffuseReflectance")
                    fail(c.file, kp->line, "diffuse: unexpected texture \"" + name + "\"");
                parseTexture(c, *kp, d.reflectanceTexture);
            }
    } else if (type == "plastic") {
        /* SmoothPlastic (plastic.cpp:146-165): constant colours */
        d.intIOR = lookupIOR(c, b, p, "intIOR", "polypropylene");
        d.extIOR = lookupIOR(c, b, p, "extIOR", "air");
        if (d.intIOR < 0 || d.extIOR < 0)
            fail(c.file, b.line, "The interior and exterior indices of refraction must be positive!");
        for (int i = 0; i < 3; ++i) {
            d.diffuse[i] = p.num.count("diffuseReflectance") ? p.num["diffuseReflectance"][i] : 0.5f;
            d.specular[i] = p.num.count("specularReflectance") ? p.num["specularReflectance"][i] : 1.0f;
        }
        d.nonlinear = num1(p, "nonlinear", 0.0f) != 0.0f;
        /* BSDF::BSDF (bsdf.cpp:30-31): reflectances above 1 are scaled unless disabled */
        d.ensureEnergyConservation = num1(p, "ensureEnergyConservation", 1.0f) != 0.0f;
        for (auto &kp : b.kids)
            if (kp->tag == "texture")
                fail(c.file, kp->line, "plastic: textured reflectances are outside this path (constant colours only)");
    } else if (type == "twosided") {
        /* TwoSidedBRDF (twosided.cpp:58-110): one or two nested BSDFs, no transmission */
        for (auto &kp : b.kids) {
            const XNode *nb = nullptr;
            if (kp->tag == "bsdf") {
                nb = kp.get();
            } else if (kp->tag == "ref") {
                auto it = c.ids.find(attrS(c, *kp, "id"));
                if (it == c.ids.end()) fail(c.file, kp->line, "unknown reference \"" + attrS(c, *kp, "id") + "\"");
                nb = it->second;
            }
            if (!nb) continue;
            if (d.nested.size() == 2) fail(c.file, kp->line, "No more than two nested BRDFs can be added!");
            BsdfDesc n;
            parseBSDF(c, *nb, n);
            if (n.type == "thindielectric" || n.type == "marschnerdielectric" || n.type == "marschner" ||
                n.type == "kajiyakay")
                fail(c.file, nb->line, "Only materials without a transmission component can be nested!");
            d.nested.push_back(n);
        }
        if (d.nested.empty()) fail(c.file, b.line, "A nested one-sided material is required!");
    } else {
        fail(c.file, b.line, "BSDF plugin \"" + type +
                                 "\" is outside this path (supported: marschner, kajiyakay, roughplastic, "
                                 "marschnerdielectric, thindielectric, diffuse, plastic, twosided)");
    }
}

/* the BSDF of a shape: a <ref>, a nested <bsdf>, or Shape::configure's 0.5 Lambertian
   (shape.cpp:48-64); one BsdfDesc per distinct XML node */
int shapeBSDF(Ctx &c, const XNode &nd, SceneDesc &d) {
    const XNode *bn = nullptr;
    for (auto &kp : nd.kids) {
        const XNode &k = *kp;
        if (k.tag == "ref") {
            std::string id = attrS(c, k, "id");
            auto it = c.ids.find(id);
            if (it == c.ids.end()) fail(c.file, k.line, "unknown reference \"" + id + "\"");
            bn = it->second;
        } else if (k.tag == "bsdf") {
            bn = &k;
        }
    }
    if (!bn) {
        d.bsdfs.push_back(BsdfDesc());
        return (int) d.bsdfs.size() - 1;
    }
    auto it = c.bsdfIndex.find(bn);
    if (it == c.bsdfIndex.end()) {
        BsdfDesc b;
        parseBSDF(c, *bn, b);
        d.bsdfs.push_back(b);
        it = c.bsdfIndex.emplace(bn, (int) d.bsdfs.size() - 1).first;
    }
    return it->second;
}

/* WavefrontOBJ (obj.cpp:199-240) / Rectangle (rectangle.cpp:81-87) */
void parseMeshShape(Ctx &c, const XNode &nd, const std::string &type, SceneDesc &d) {
    Props p;
    collectProps(c, nd, p);
    MeshShapeDesc m;
    m.type = type;
    if (type == "obj") {
        if (!p.str.count("filename")) fail(c.file, nd.line, "obj shape needs a filename");
        m.file = p.str["filename"];
        if (!m.file.empty() && m.file[0] != '/') m.file = d.sceneDir + "/" + m.file;
        m.faceNormals = num1(p, "faceNormals", 0.0f) != 0.0f;
        m.flipTexCoords = num1(p, "flipTexCoords", 1.0f) != 0.0f;
        if (p.num.count("maxSmoothAngle"))
            fail(c.file, nd.line, "obj: 'maxSmoothAngle' (mesh topology rebuild) is outside this path");
        if (p.num.count("shapeIndex") || num1(p, "collapse", 0.0f) != 0.0f)
            fail(c.file, nd.line, "obj: 'shapeIndex' / 'collapse' are outside this path");
    }
    m.flipNormals = num1(p, "flipNormals", 0.0f) != 0.0f;
    if (p.xform.count("toWorld")) parseTransform(c, *p.xform["toWorld"], m.toWorld);
    m.bsdf = shapeBSDF(c, nd, d);
    d.meshes.push_back(m);
}

void parseObject(Ctx &c, const XNode &nd, SceneDesc &d) {
    const std::string &tag = nd.tag;
    if (tag == "integrator") {
        d.integrator = attrS(c, nd, "type");
        if (d.integrator != "path")
            fail(c.file, nd.line, "integrator \"" + d.integrator + "\" is not supported (only \"path\")");
        Props p;
        collectProps(c, nd, p);
        d.maxDepth = (int) num1(p, "maxDepth", -1);
        d.rrDepth = (int) num1(p, "rrDepth", 5);
        d.strictNormals = num1(p, "strictNormals", 0) != 0;
        d.hideEmitters = num1(p, "hideEmitters", 0) != 0;
    } else if (tag == "sensor" || tag == "camera") {
        std::string type = attrS(c, nd, "type");
        if (type != "perspective")
            fail(c.file, nd.line, "sensor \"" + type + "\" is not supported (only \"perspective\")");
        Props p;
        collectProps(c, nd, p);
        if (p.xform.count("toWorld")) parseTransform(c, *p.xform["toWorld"], d.toWorld);
        if (p.num.count("fov")) {
            d.fov = num1(p, "fov", 45.0f);
            if (p.str.count("fovAxis")) { /* boost::to_lower_copy (sensor.cpp:247-248) */
                d.fovAxis = p.str["fovAxis"];
                for (char &ch : d.fovAxis) ch = (char) std::tolower((unsigned char) ch);
            }
        } else { /* no fov: a diagonal one from "focalLength" (sensor.cpp:264-276), 36x24 mm film */
            std::string f = p.str.count("focalLength") ? p.str["focalLength"] : std::string("50mm");
            if (f.size() >= 2 && f.compare(f.size() - 2, 2, "mm") == 0) f = f.substr(0, f.size() - 2);
            char *end = nullptr;
            const float value = (float) std::strtod(f.c_str(), &end);
            if (!end || *end != '\0')
                fail(c.file, nd.line, "Could not parse the focal length (must be of the form <x>mm, where <x> "
                                      "is a positive integer)!");
            const float kPiF = 3.14159265358979323846f; /* M_PI under SINGLE_PRECISION (constants.h:80) */
            d.fov = 2 * 180 / kPiF * std::atan(std::sqrt((float) (36 * 36 + 24 * 24)) / (2 * value));
            d.fovAxis = "diagonal";
        }
        if (d.fovAxis != "x" && d.fovAxis != "y" && d.fovAxis != "smaller" && d.fovAxis != "larger" &&
            d.fovAxis != "diagonal")
            fail(c.file, nd.line, "The 'fovAxis' parameter must be set to one of 'smaller', 'larger', 'diagonal', "
                                  "'x', or 'y'!");
        d.nearClip = num1(p, "nearClip", 1e-2f);
        d.farClip = num1(p, "farClip", 1e4f);
        for (auto &kp : nd.kids) {
            const XNode &k = *kp;
            if (k.tag == "sampler") {
                d.sampler = attrS(c, k, "type");
                if (d.sampler != "sobol")
                    fail(c.file, k.line, "sampler \"" + d.sampler + "\" is not supported (only \"sobol\")");
                Props sp;
                collectProps(c, k, sp);
                for (auto &sk : k.kids) /* an exact 64-bit integer (Properties::getSize) */
                    if (sk->tag == "integer" && attrS(c, *sk, "name") == "scramble")
                        d.scramble = std::stoull(attrS(c, *sk, "value"));
                d.spp = (int) num1(sp, "sampleCount", 4);
            } else if (k.tag == "film") {
                FilmDesc &fd = d.film;
                fd.type = attrS(c, k, "type");
                if (fd.type != "ldrfilm" && fd.type != "hdrfilm")
                    fail(c.file, k.line, "film \"" + fd.type + "\" is not supported (ldrfilm, hdrfilm)");
                Props fp;
                collectProps(c, k, fp);
                d.width = (int) num1(fp, "width", 768);
                d.height = (int) num1(fp, "height", 576);
                fd.gamma = num1(fp, "gamma", -1.0f);
                fd.exposure = num1(fp, "exposure", 0.0f);
                fd.key = num1(fp, "key", 0.18f);
                fd.burn = num1(fp, "burn", 0.0f);
                fd.banner = num1(fp, "banner", 1.0f) != 0.0f;
                if (fp.str.count("fileFormat")) fd.fileFormat = fp.str["fileFormat"];
                if (fp.str.count("pixelFormat")) fd.pixelFormat = fp.str["pixelFormat"];
                if (fp.str.count("componentFormat")) fd.componentFormat = fp.str["componentFormat"];
                if (fp.str.count("tonemapMethod")) fd.tonemapMethod = fp.str["tonemapMethod"];
                std::string err;
                if (!checkFilm(fd, err)) fail(c.file, k.line, err);
                for (auto &fk : k.kids)
                    if (fk->tag == "rfilter") {
                        d.rfilter = attrS(c, *fk, "type");
                        if (d.rfilter != "tent")
                            fail(c.file, fk->line, "rfilter \"" + d.rfilter + "\" is not supported (only \"tent\")");
                    }
            }
        }
    } else if (tag == "bsdf") {
        std::string id = attrS(c, nd, "id", false);
        if (!id.empty()) c.ids[id] = &nd;
        BsdfDesc unused; /* instantiated (and validated) even when no shape refers to it */
        parseBSDF(c, nd, unused);
    } else if (tag == "shape") {
        std::string type = attrS(c, nd, "type");
        if (type == "obj" || type == "rectangle") {
            parseMeshShape(c, nd, type, d);
            return;
        }
        if (type != "hair")
            fail(c.file, nd.line, "shape \"" + type + "\" is outside this path (hair; obj / rectangle on the CPU path)");
        Props p;
        collectProps(c, nd, p);
        if (!p.str.count("filename")) fail(c.file, nd.line, "hair shape needs a filename");
        HairShapeDesc h;
        h.file = p.str["filename"];
        if (!h.file.empty() && h.file[0] != '/') h.file = d.sceneDir + "/" + h.file;
        h.radius = num1(p, "radius", 0.025f);
        h.angleThreshold = num1(p, "angleThreshold", 1.0f);
        h.reduction = num1(p, "reduction", 0.0f);
        if (d.shapes.empty()) { /* one kd-tree over every hair shape: the first shape's build parameters */
            d.kd.queryCost = num1(p, "kdIntersectionCost", d.kd.queryCost);
            d.kd.traversalCost = num1(p, "kdTraversalCost", d.kd.traversalCost);
            d.kd.emptySpaceBonus = num1(p, "kdEmptySpaceBonus", d.kd.emptySpaceBonus);
            d.kd.stopPrims = (int) num1(p, "kdStopPrims", (float) d.kd.stopPrims);
            d.kd.maxDepth = (int) num1(p, "kdMaxDepth", (float) d.kd.maxDepth);
            d.kd.maxBadRefines = (int) num1(p, "kdMaxBadRefines", (float) d.kd.maxBadRefines);
            d.kd.clip = num1(p, "kdClip", d.kd.clip ? 1.0f : 0.0f) != 0.0f;
            /* build-speed knobs of this builder (no reference counterpart) */
            d.kd.clipMinPrims = (int) num1(p, "kdClipMinPrims", (float) d.kd.clipMinPrims);
            d.kd.exactSweepMax = (int) num1(p, "kdExactSweepMax", (float) d.kd.exactSweepMax);
        }
        if (p.xform.count("toWorld")) {
            parseTransform(c, *p.xform["toWorld"], h.toWorld);
            h.hasToWorld = true;
        }
        h.bsdf = shapeBSDF(c, nd, d);
        if (d.shapes.size() >= HPT_MAX_SHAPES) fail(c.file, nd.line, "too many hair shapes");
        d.shapes.push_back(h);
    } else if (tag == "emitter") {
        std::string type = attrS(c, nd, "type");
        Props p;
        collectProps(c, nd, p);
        d.emitter = type;
        if (p.xform.count("toWorld")) parseTransform(c, *p.xform["toWorld"], d.emitterToWorld);
        if (type == "sunsky") {
            float scale = num1(p, "scale", 1.0f);
            d.sunScale = num1(p, "sunScale", scale);
            d.skyScale = num1(p, "skyScale", scale);
            d.sunRadiusScale = num1(p, "sunRadiusScale", 1.0f);
            d.turbidity = num1(p, "turbidity", 3.0f);
            d.skyResolution = (int) num1(p, "resolution", 512);
            d.skyStretch = num1(p, "stretch", 1.0f);
            if (p.num.count("albedo")) {
                auto &v = p.num["albedo"];
                for (int i = 0; i < 3; ++i) d.skyAlbedo[i] = v[v.size() == 1 ? 0 : i];
            }
            if (p.num.count("sunDirection")) {
                auto &v = p.num["sunDirection"];
                for (int i = 0; i < 3; ++i) d.sunDirection[i] = v[i];
                d.sunDirectionGiven = true;
                for (const char *k : {"latitude", "longitude", "timezone", "day", "time"})
                    if (p.num.count(k))
                        fail(c.file, nd.line, "Both the 'sunDirection' parameter and time/location information "
                                              "were provided -- only one of them can be specified at a time!");
            }
            d.sunLatitude = num1(p, "latitude", d.sunLatitude);
            d.sunLongitude = num1(p, "longitude", d.sunLongitude);
            d.sunTimezone = num1(p, "timezone", d.sunTimezone);
            d.sunYear = (int) num1(p, "year", (float) d.sunYear);
            d.sunMonth = (int) num1(p, "month", (float) d.sunMonth);
            d.sunDay = (int) num1(p, "day", (float) d.sunDay);
            d.sunHour = num1(p, "hour", d.sunHour);
            d.sunMinute = num1(p, "minute", d.sunMinute);
            d.sunSecond = num1(p, "second", d.sunSecond);
        } else if (type == "envmap") {
            if (!p.str.count("filename")) fail(c.file, nd.line, "envmap needs a filename");
            d.envFile = p.str["filename"];
            d.envScale = num1(p, "scale", 1.0f);
        } else {
            fail(c.file, nd.line, "emitter \"" + type + "\" is not supported (sunsky, envmap)");
        }
    } else if (tag == "default" || tag == "include") {
        /* handled earlier / not used by the models */
    } else {
        fail(c.file, nd.line, "unsupported top-level element <" + tag + ">");
    }
}

} // namespace

SceneDesc parseSceneXML(const std::string &path, const std::map<std::string, std::string> &defines) {
    std::ifstream f(path);
    if (!f) throw std::runtime_error("cannot open scene file " + path);
    std::stringstream ss;
    ss << f.rdbuf();
    std::unique_ptr<XNode> root = parseXML(ss.str(), path);
    if (root->tag != "scene") fail(path, root->line, "root element must be <scene>");
    Ctx c;
    c.file = path;
    c.defines = defines;
    for (auto &kp : root->kids)
        if (kp->tag == "default") {
            const std::string *n = kp->attr("name"), *v = kp->attr("value");
            if (!n || !v) fail(path, kp->line, "<default> needs name and value");
            if (!c.defines.count(*n)) c.defines[*n] = *v;
        }
    SceneDesc d;
    size_t slash = path.find_last_of('/');
    d.sceneDir = slash == std::string::npos ? "." : path.substr(0, slash);
    for (auto &kp : root->kids) parseObject(c, *kp, d);
    if (d.shapes.empty() && d.meshes.empty()) fail(path, root->line, "scene has no shape");
    if (!d.envFile.empty() && d.envFile[0] != '/') d.envFile = d.sceneDir + "/" + d.envFile;
    if (d.emitter.empty()) {
        /* scene.cpp:358-372: no emitter -> default sun & sky */
        d.emitter = "sunsky";
        d.sunScale = d.skyScale = 2.0f;
        d.sunRadiusScale = 15.0f;
    }
    return d;
}

namespace {
struct Json {
    std::ostringstream o;
    bool first = true;
    void sep() {
        if (!first) o << ",";
        first = false;
    }
    void key(const char *k) {
        sep();
        o << "\"" << k << "\":";
    }
    static std::string esc(const std::string &s) {
        std::string r;
        for (char ch : s) {
            if (ch == '"' || ch == '\\') r += '\\';
            r += ch;
        }
        return r;
    }
    void str(const char *k, const std::string &v) {
        key(k);
        o << "\"" << esc(v) << "\"";
    }
    void num(const char *k, double v) {
        key(k);
        char b[40];
        std::snprintf(b, sizeof(b), "%.9g", v);
        o << b;
    }
    void boolean(const char *k, bool v) {
        key(k);
        o << (v ? "true" : "false");
    }
    void arr(const char *k, const float *v, int n) {
        key(k);
        o << "[";
        for (int i = 0; i < n; ++i) {
            char b[40];
            std::snprintf(b, sizeof(b), "%.9g", (double) v[i]);
            o << (i ? "," : "") << b;
        }
        o << "]";
    }
    void open(const char *k, char br) {
        if (k) key(k);
        else sep();
        o << br;
        first = true;
    }
    void close(char br) {
        o << br;
        first = false;
    }
};

void bsdfJSON(Json &j, const BsdfDesc &b) {
    j.open(nullptr, '{');
    j.str("type", b.type);
    j.num("intIOR", b.intIOR);
    j.num("extIOR", b.extIOR);
    j.str("distribution", b.distribution);
    j.num("alpha", b.alpha);
    j.arr("diffuse", b.diffuse, 3);
    j.arr("specular", b.specular, 3);
    j.arr("transmittance", b.transmittance, 3);
    j.num("exponent", b.exponent);
    j.boolean("nonlinear", b.nonlinear);
    j.boolean("sampleVisible", b.sampleVisible);
    j.boolean("ensureEnergyConservation", b.ensureEnergyConservation);
    if (!b.reflectanceTexture.type.empty()) {
        const TextureDesc &t = b.reflectanceTexture;
        j.open("reflectanceTexture", '{');
        j.str("type", t.type);
        j.arr("color0", t.color0, 3);
        j.arr("color1", t.color1, 3);
        j.num("uoffset", t.uoffset);
        j.num("voffset", t.voffset);
        j.num("uscale", t.uscale);
        j.num("vscale", t.vscale);
        j.close('}');
    }
    j.open("nested", '[');
    for (const BsdfDesc &n : b.nested) bsdfJSON(j, n);
    j.close(']');
    j.close('}');
}
} // namespace

std::string sceneToJSON(const SceneDesc &d) {
    Json j;
    j.open(nullptr, '{');
    j.open("integrator", '{');
    j.str("type", d.integrator);
    j.num("maxDepth", d.maxDepth);
    j.num("rrDepth", d.rrDepth);
    j.boolean("strictNormals", d.strictNormals);
    j.boolean("hideEmitters", d.hideEmitters);
    j.close('}');
    j.open("sensor", '{');
    j.arr("toWorld", d.toWorld, 16);
    j.num("fov", d.fov);
    j.str("fovAxis", d.fovAxis);
    j.num("xfov", cameraXFov(d));
    j.num("nearClip", d.nearClip);
    j.num("farClip", d.farClip);
    j.num("width", d.width);
    j.num("height", d.height);
    j.num("sampleCount", d.spp);
    j.str("film", d.film.type);
    j.str("rfilter", d.rfilter);
    j.close('}');
    j.open("bsdfs", '[');
    for (const BsdfDesc &b : d.bsdfs) bsdfJSON(j, b);
    j.close(']');
    j.open("hair", '[');
    for (const HairShapeDesc &h : d.shapes) {
        j.open(nullptr, '{');
        j.str("filename", h.file);
        j.num("radius", h.radius);
        j.num("angleThreshold", h.angleThreshold);
        j.num("reduction", h.reduction);
        j.arr("toWorld", h.toWorld, 16);
        j.num("bsdf", h.bsdf);
        j.close('}');
    }
    j.close(']');
    j.open("meshes", '[');
    for (const MeshShapeDesc &m : d.meshes) {
        j.open(nullptr, '{');
        j.str("type", m.type);
        j.str("filename", m.file);
        j.arr("toWorld", m.toWorld, 16);
        j.boolean("faceNormals", m.faceNormals);
        j.boolean("flipNormals", m.flipNormals);
        j.boolean("flipTexCoords", m.flipTexCoords);
        j.num("bsdf", m.bsdf);
        j.close('}');
    }
    j.close(']');
    j.open("emitter", '{');
    j.str("type", d.emitter);
    j.str("filename", d.envFile);
    j.num("scale", d.envScale);
    j.arr("toWorld", d.emitterToWorld, 16);
    j.close('}');
    j.close('}');
    return j.o.str();
}

} // namespace hpt
