/*
 * mitsuba_cli.cpp -- `mitsuba`-compatible command line front end.
 *
 * Mirrors src/mitsuba/mitsuba.cpp:52-400 for the hair path: parse options,
 * load each scene XML, render, develop the film and write it next to the
 * scene (or to -o).  Rendering runs on MI355X devices through libhairpt.so;
 * with --gpus N the scene is parsed, loaded and its kd-tree built ONCE and
 * shared with N device contexts (hpt_context_share_scene, uploaded in
 * parallel, like mitsuba.cpp:281-329 hands one scene to every worker); the
 * 32x32 blocks are dealt over the devices (Hilbert-cyclic) and the films are
 * combined on the first device over xGMI (hpt_render_multi) -- the
 * single-node analogue of the reference's -c remote workers.
 * -r sec writes the partial image every `sec` seconds like the reference's
 * flush timer (mitsuba.cpp:300-330): the samples are rendered in chunks and
 * the film accumulated so far is developed between chunks.
 *
 *   mitsuba [options] <scene.xml> [<scene2.xml> ...]
 *     -D key=val   define $key for the XML        -o fname   output file
 *     -p count     (accepted; GPU render)          -q         quiet
 *     -x           skip scenes whose output exists -r sec  write partial images
 *     -b/-z/-v (accepted)
 *     --spp N --width W --height H --max-depth D   overrides
 *     --device i   first device                    --gpus N   devices to use
 *     --devices a,b,...  explicit device of each shard (a device may repeat)
 *     --stats      print timing / traversal statistics
 */
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <fstream>
#include <string>
#include <thread>
#include <vector>

#include "hairpt.h"
#include "host/host_scene.h"

namespace {

void usage() {
    std::printf(
        "Mitsuba-compatible hair path tracer for AMD Instinct MI355X\n"
        "Usage: mitsuba [options] <scene.xml>...\n"
        "Options:\n"
        "   -h          Display this help text\n"
        "   -D key=val  Define a constant, which can referenced as \"$key\" in the scene\n"
        "   -o fname    Write the output image to the file denoted by \"fname\"\n"
        "   -p count    Override the detected number of processors (ignored: GPU render)\n"
        "   -q          Quiet mode - do not print any log messages to stdout\n"
        "   -x          Skip rendering of files where output already exists\n"
        "   -r sec      Write (partial) output images every 'sec' seconds\n"
        "   --spp N --width W --height H --max-depth D   override scene parameters\n"
        "   --device I --gpus N   render on N devices starting at I\n"
        "   --devices a,b,...     the device of each shard (a device may repeat)\n"
        "   --stats     print per-kernel timing and traversal counters\n");
}

struct Opts {
    std::vector<std::pair<std::string, std::string>> defines;
    std::string out;
    bool quiet = false, skipExisting = false, stats = false;
    int spp = 0, width = 0, height = 0, maxDepth = -2, device = 0, gpus = 1;
    double flushSec = 0; /* -r */
    std::vector<int> devices; /* --devices */
    std::vector<std::string> scenes;
};

bool exists(const std::string &p) {
    std::ifstream f(p);
    return (bool) f;
}

} // namespace

int main(int argc, char **argv) {
    Opts o;
    for (int i = 1; i < argc; ++i) {
        std::string a = argv[i];
        auto next = [&](const char *what) -> std::string {
            if (i + 1 >= argc) {
                std::fprintf(stderr, "missing argument for %s\n", what);
                std::exit(1);
            }
            return argv[++i];
        };
        if (a == "-h" || a == "--help") { usage(); return 0; }
        else if (a == "-D") {
            std::string kv = next("-D");
            size_t eq = kv.find('=');
            if (eq == std::string::npos) { std::fprintf(stderr, "-D expects key=value\n"); return 1; }
            o.defines.push_back({kv.substr(0, eq), kv.substr(eq + 1)});
        } else if (a == "-o") o.out = next("-o");
        else if (a == "-r") o.flushSec = std::atof(next("-r").c_str());
        else if (a == "-p" || a == "-b" || a == "-L" || a == "-a") (void) next(a.c_str());
        else if (a == "-q") o.quiet = true;
        else if (a == "-x") o.skipExisting = true;
        else if (a == "-v" || a == "-z" || a == "-t" || a == "-w") {}
        else if (a == "-c" || a == "-s") {
            std::fprintf(stderr, "network rendering (-c/-s) is replaced by --gpus on one MI355X node\n");
            return 1;
        } else if (a == "--spp") o.spp = std::atoi(next("--spp").c_str());
        else if (a == "--width") o.width = std::atoi(next("--width").c_str());
        else if (a == "--height") o.height = std::atoi(next("--height").c_str());
        else if (a == "--max-depth") o.maxDepth = std::atoi(next("--max-depth").c_str());
        else if (a == "--device") o.device = std::atoi(next("--device").c_str());
        else if (a == "--gpus") o.gpus = std::max(1, std::atoi(next("--gpus").c_str()));
        else if (a == "--devices") {
            const std::string list = next("--devices");
            o.devices.clear();
            for (size_t i = 0; i < list.size();) {
                size_t j = list.find(',', i);
                if (j == std::string::npos) j = list.size();
                o.devices.push_back(std::atoi(list.substr(i, j - i).c_str()));
                i = j + 1;
            }
            if (o.devices.empty()) { std::fprintf(stderr, "--devices needs a list\n"); return 1; }
        }
        else if (a == "--stats") o.stats = true;
        else if (!a.empty() && a[0] == '-') { std::fprintf(stderr, "unknown option %s\n", a.c_str()); usage(); return 1; }
        else o.scenes.push_back(a);
    }
    if (o.scenes.empty()) { usage(); return 1; }
    for (const std::string &scene : o.scenes) {
        std::vector<const char *> keys, vals;
        for (auto &kv : o.defines) { keys.push_back(kv.first.c_str()); vals.push_back(kv.second.c_str()); }
        hpt::SceneDesc desc;
        try {
            std::map<std::string, std::string> defs(o.defines.begin(), o.defines.end());
            desc = hpt::parseSceneXML(scene, defs);
        } catch (const std::exception &e) {
            std::fprintf(stderr, "Error while parsing \"%s\": %s\n", scene.c_str(), e.what());
            return 2;
        }
        /* output name: -o, else the scene file without its extension; the film
           appends its own extension (ldrfilm.cpp:335-345, hdrfilm.cpp:508-519) */
        const hpt::FilmDesc &fd = desc.film;
        const std::string ext = fd.type == "ldrfilm" ? ".png" : fd.fileFormat == "openexr" ? ".exr"
                                                           : fd.fileFormat == "rgbe"    ? ".rgbe"
                                                                                        : ".pfm";
        std::string out = o.out;
        if (out.empty()) {
            size_t dot = scene.find_last_of('.'), slash = scene.find_last_of('/');
            out = (dot == std::string::npos || (slash != std::string::npos && dot < slash)) ? scene : scene.substr(0, dot);
        }
        {
            size_t dot = out.find_last_of('.'), slash = out.find_last_of('/');
            std::string cur = (dot != std::string::npos && (slash == std::string::npos || dot > slash)) ? out.substr(dot) : "";
            for (auto &ch : cur) ch = (char) std::tolower((unsigned char) ch);
            if (cur != ext) out = (cur.empty() ? out : out.substr(0, dot)) + ext;
        }
        if (o.skipExisting && exists(out)) {
            if (!o.quiet) std::printf("Skipping \"%s\": output exists\n", scene.c_str());
            continue;
        }
        std::vector<int> devs = o.devices;
        if (devs.empty())
            for (int g = 0; g < o.gpus; ++g) devs.push_back(o.device + g);
        const int G = (int) devs.size();
        /* every context of this scene is destroyed on every way out of the iteration */
        struct Contexts {
            std::vector<hpt_context *> v;
            ~Contexts() {
                for (hpt_context *c : v) hpt_context_destroy(c);
            }
        } owned{std::vector<hpt_context *>(G, nullptr)};
        std::vector<hpt_context *> &ctx = owned.v;
        int W = 0, H = 0, spp = 0;
        /* the scene once: parse, hair, kd-tree, tables on the first device's context ... */
        const auto tLoad = std::chrono::steady_clock::now();
        {
            int rc = hpt_context_create(devs[0], &ctx[0]);
            if (rc) { std::fprintf(stderr, "cannot create a gfx950 context on device %d (%d)\n", devs[0], rc); return 3; }
            rc = hpt_load_scene_xml(ctx[0], scene.c_str(), (int) keys.size(), keys.data(), vals.data());
            if (rc) { std::fprintf(stderr, "%s\n", hpt_last_error(ctx[0])); return 2; }
            hpt_scene_info info;
            hpt_get_scene_info(ctx[0], &info);
            if (o.width || o.height || o.maxDepth != -2) {
                /* re-issue the camera / integrator with overrides */
                W = o.width ? o.width : info.width;
                H = o.height ? o.height : info.height;
                hpt_set_camera(ctx[0], desc.toWorld, desc.fov, W, H, desc.nearClip, desc.farClip);
                hpt_set_integrator(ctx[0], o.maxDepth != -2 ? o.maxDepth : info.max_depth, info.rr_depth,
                                   info.strict_normals, info.hide_emitters);
            }
            if (o.spp) hpt_set_sampler(ctx[0], o.spp);
            rc = hpt_prepare(ctx[0]);
            if (rc) { std::fprintf(stderr, "%s\n", hpt_last_error(ctx[0])); return 2; }
            hpt_get_scene_info(ctx[0], &info);
            W = info.width;
            H = info.height;
            spp = info.spp;
            if (!o.quiet)
                std::printf("Scene \"%s\": %dx%d @ %d spp, %llu hair segments, kd-tree %llu nodes (depth %d, %.2f s)\n",
                            scene.c_str(), W, H, spp, (unsigned long long) info.segments,
                            (unsigned long long) info.kd_nodes, info.kd_depth, info.kd_build_seconds);
        }
        const double loadSec = std::chrono::duration<double>(std::chrono::steady_clock::now() - tLoad).count();
        /* ... then uploaded to the other devices in parallel (no second parse or build) */
        if (G > 1) {
            const auto tShare = std::chrono::steady_clock::now();
            std::vector<int> rcs(G, 0);
            std::vector<std::thread> th;
            std::vector<std::string> shareErr(G);
            for (int g = 1; g < G; ++g)
                th.emplace_back([&, g] {
                    rcs[g] = hpt_context_share_scene(ctx[0], devs[g], &ctx[g]);
                    if (rcs[g]) shareErr[g] = hpt_last_error(nullptr); /* this thread's message */
                });
            for (auto &t : th) t.join();
            /* a failed share reports on the failing thread (hpt_last_error(NULL)), never on the shared
               source context, which every worker reads at once */
            for (int g = 1; g < G; ++g)
                if (rcs[g]) { std::fprintf(stderr, "device %d: %s\n", devs[g], shareErr[g].c_str()); return 3; }
            if (!o.quiet)
                std::printf("Scene loaded once (%.2f s) and shared with %d more device context%s (%.2f s)\n", loadSec,
                            G - 1, G > 2 ? "s" : "",
                            std::chrono::duration<double>(std::chrono::steady_clock::now() - tShare).count());
        }
        std::vector<float> film((size_t) W * H * 4, 0.0f);
        hpt_film_params fp;
        hpt_get_film_params(ctx[0], &fp);
        char written[4096];
        /* develop (Film::develop); the device films are combined by hpt_render_multi */
        auto develop = [&]() -> bool {
            if (hpt_write_film(ctx[0], out.c_str(), film.data(), W, H, &fp, written, sizeof(written))) {
                std::fprintf(stderr, "%s\n", hpt_last_error(ctx[0]));
                return false;
            }
            return true;
        };
        /* the samples in one call, or in chunks with a partial image every -r seconds */
        const int chunk = o.flushSec > 0 ? std::max(1, spp / 16) : spp;
        auto t0 = std::chrono::steady_clock::now(), lastFlush = t0;
        for (int j0 = 0; j0 < spp; j0 += chunk) {
            const int j1 = std::min(spp, j0 + chunk);
            hpt_render_params p;
            std::memset(&p, 0, sizeof(p));
            p.spp_begin = j0;
            p.spp_end = j1;
            p.collect_stats = o.stats ? 2 : 0;
            if (hpt_render_multi(ctx.data(), G, &p, film.data())) {
                std::fprintf(stderr, "render failed: %s\n", hpt_last_error(ctx[0]));
                return 4;
            }
            const auto now = std::chrono::steady_clock::now();
            if (j1 < spp && o.flushSec > 0 && std::chrono::duration<double>(now - lastFlush).count() >= o.flushSec) {
                if (!develop()) return 5;
                lastFlush = now;
                if (!o.quiet) std::printf("Wrote partial image (%d of %d spp) -> %s\n", j1, spp, written);
            }
        }
        double sec = std::chrono::duration<double>(std::chrono::steady_clock::now() - t0).count();
        if (!develop()) return 5;
        out = written;
        if (!o.quiet) {
            double paths = (double) W * H * spp;
            std::printf("Rendering finished (took %.3f s, %.2f Mpaths/s on %d GPU%s) -> %s\n", sec, paths / sec * 1e-6, G,
                        G > 1 ? "s" : "", out.c_str());
            if (o.stats) {
                hpt_stats s;
                hpt_get_stats(ctx[0], &s);
                std::printf("device 0 (last chunk): camera trace (packets) %.2f ms, trace %.2f ms (%llu launches), shade "
                            "%.2f post %.2f tail %.2f (%llu paths) camera %.2f gather %.2f; nodes %llu prims %llu "
                            "bounces %llu max bounce %d\n",
                            s.ms_trace_packet, s.ms_trace, (unsigned long long) s.trace_launches, s.ms_shade,
                            s.ms_post, s.ms_tail, (unsigned long long) s.tail_paths, s.ms_camera, s.ms_gather,
                            (unsigned long long) s.nodes, (unsigned long long) s.prims,
                            (unsigned long long) s.bounces, s.max_bounces);
            }
        }
    }
    return 0;
}
