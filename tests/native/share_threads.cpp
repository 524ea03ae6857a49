/*
 * share_threads.cpp -- several threads share one prepared source context at once
 * (hpt_context_share_scene, as bin/mitsuba --gpus N does) while every share fails: the
 * devices asked for do not exist here.  Each failure must reach its own thread through
 * hpt_last_error(NULL) and leave the shared source untouched (include/hairpt.h).  Built
 * against a ThreadSanitizer build of the host code (Makefile target `tsan`,
 * tests/test_share_threads.py), so a write to the source from the workers is a reported race.
 *
 *   share_threads scene.xml [threads] [data dir]
 */
#include <cstdio>
#include <cstdlib>
#include <cstring>
#include <string>
#include <thread>
#include <vector>

#include "hairpt.h"

int main(int argc, char **argv) {
    if (argc < 2) {
        std::fprintf(stderr, "usage: %s scene.xml [threads] [data dir]\n", argv[0]);
        return 2;
    }
    const int T = argc > 2 ? std::atoi(argv[2]) : 8;
    hpt_context *src = nullptr, *raw = nullptr;
    if (hpt_context_create(HPT_HOST_ONLY, &src) || hpt_context_create(HPT_HOST_ONLY, &raw)) return 3;
    if (argc > 3 && (hpt_set_data_dir(src, argv[3]) || hpt_set_data_dir(raw, argv[3]))) return 3;
    if (hpt_load_scene_xml(src, argv[1], 0, nullptr, nullptr) || hpt_prepare(src)) {
        std::fprintf(stderr, "source: %s\n", hpt_last_error(src));
        return 3;
    }
    if (hpt_load_scene_xml(raw, argv[1], 0, nullptr, nullptr)) return 3; /* loaded, never prepared */
    const std::string srcErr = hpt_last_error(src), rawErr = hpt_last_error(raw);
    std::vector<int> rcs(T, 0);
    std::vector<std::string> msgs(T);
    std::vector<hpt_context *> outs(T, nullptr);
    std::vector<std::thread> th;
    for (int t = 0; t < T; ++t)
        th.emplace_back([&, t] {
            /* odd threads: an unprepared source; even: a device index no machine has */
            hpt_context *from = (t & 1) ? raw : src;
            rcs[t] = hpt_context_share_scene(from, 4096 + t, &outs[t]);
            msgs[t] = hpt_last_error(nullptr);
        });
    for (auto &x : th) x.join();
    int bad = 0;
    for (int t = 0; t < T; ++t) {
        const bool ok = rcs[t] != HPT_OK && outs[t] == nullptr &&
                        msgs[t].find("hpt_context_share_scene") != std::string::npos &&
                        msgs[t].find((t & 1) ? "not prepared" : "device") != std::string::npos;
        if (!ok) {
            std::fprintf(stderr, "thread %d: rc %d out %p message '%s'\n", t, rcs[t], (void *) outs[t], msgs[t].c_str());
            ++bad;
        }
    }
    /* the sources kept their own (empty) messages: nothing was written to them */
    if (srcErr != hpt_last_error(src) || rawErr != hpt_last_error(raw)) {
        std::fprintf(stderr, "a shared source's error changed: '%s' / '%s'\n", hpt_last_error(src), hpt_last_error(raw));
        ++bad;
    }
    /* the main thread's own slot saw none of the workers' messages */
    if (std::strcmp(hpt_last_error(nullptr), "null context") != 0) {
        std::fprintf(stderr, "main thread's message: '%s'\n", hpt_last_error(nullptr));
        ++bad;
    }
    hpt_context_destroy(src);
    hpt_context_destroy(raw);
    std::printf("%d threads, %d failures reported per thread, %d bad\n", T, T - bad, bad);
    return bad ? 1 : 0;
}
