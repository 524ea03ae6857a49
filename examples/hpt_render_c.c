/*
 * hpt_render_c.c -- a plain C (C99) program that drives libhairpt.so through
 * include/hairpt.h alone: the boundary a reference-side binding (the plugin
 * shim of INTEGRATION.md section 1, a cgo / ctypes stub) compiles against.
 *
 *   hpt_render_c [-d device] [-D key=value ...] [-P] [-o out] [-c film.bin] scene.xml
 *
 * Loads the scene with the -D defines (hpt_load_scene_xml, like
 * `mitsuba -D key=value`, src/mitsuba/mitsuba.cpp:160-175), prepares it,
 * prints the scene info the defines produced, renders every sample
 * (hpt_render) and writes the film like the scene's <film> (hpt_write_film).
 * -P hands the defines over as the process-wide table instead
 * (hpt_set_default_defines, what a binding calls from mitsuba.cpp's main).
 * -d -1 makes a host-only context: it stops after printing the scene info
 * and checks that hpt_render refuses to run.  -c writes the raw RGBW film.
 *
 * Build (see tests/test_c_abi.py):
 *   gcc -std=c99 -Wall -Iinclude examples/hpt_render_c.c \
 *       -Lcs184-final-project-mitsuba0.5_amd/lib -lhairpt -Wl,-rpath,<lib dir> -o hpt_render_c
 */
#define _POSIX_C_SOURCE 200809L /* strdup */
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include "hairpt.h"

#define MAX_DEFINES 64

static int fail(hpt_context *ctx, const char *what, int rc) {
    fprintf(stderr, "%s failed (%d): %s\n", what, rc, ctx ? hpt_last_error(ctx) : "");
    if (ctx) hpt_context_destroy(ctx);
    return 1;
}

int main(int argc, char **argv) {
    int device = 0, n_defines = 0, process_defines = 0, i;
    const char *keys[MAX_DEFINES], *values[MAX_DEFINES];
    char *kv_store[MAX_DEFINES];
    const char *out = NULL, *raw = NULL, *scene = NULL;
    for (i = 1; i < argc; ++i) {
        if (!strcmp(argv[i], "-d") && i + 1 < argc) {
            device = atoi(argv[++i]);
        } else if (!strcmp(argv[i], "-o") && i + 1 < argc) {
            out = argv[++i];
        } else if (!strcmp(argv[i], "-P")) {
            process_defines = 1;
        } else if (!strcmp(argv[i], "-c") && i + 1 < argc) {
            raw = argv[++i];
        } else if (!strcmp(argv[i], "-D") && i + 1 < argc) {
            char *kv = strdup(argv[++i]), *eq = strchr(kv, '=');
            if (!eq || n_defines == MAX_DEFINES) {
                fprintf(stderr, "bad define '%s' (expected key=value)\n", argv[i]);
                return 2;
            }
            *eq = '\0';
            kv_store[n_defines] = kv;
            keys[n_defines] = kv;
            values[n_defines] = eq + 1;
            ++n_defines;
        } else {
            scene = argv[i];
        }
    }
    if (!scene) {
        fprintf(stderr, "usage: %s [-d device] [-D key=value ...] [-o out] [-c film.bin] scene.xml\n", argv[0]);
        return 2;
    }

    hpt_context *ctx = NULL;
    int rc;
    if (process_defines && (rc = hpt_set_default_defines(n_defines, keys, values)) != HPT_OK)
        return fail(NULL, "hpt_set_default_defines", rc);
    if ((rc = hpt_context_create(device, &ctx)) != HPT_OK) return fail(ctx, "hpt_context_create", rc);
    if (process_defines)
        rc = hpt_load_scene_xml(ctx, scene, 0, NULL, NULL);
    else
        rc = hpt_load_scene_xml(ctx, scene, n_defines, keys, values);
    if (rc != HPT_OK) return fail(ctx, "hpt_load_scene_xml", rc);
    if ((rc = hpt_prepare(ctx)) != HPT_OK) return fail(ctx, "hpt_prepare", rc);

    hpt_scene_info info;
    if ((rc = hpt_get_scene_info(ctx, &info)) != HPT_OK) return fail(ctx, "hpt_get_scene_info", rc);
    printf("scene %dx%d spp %d maxDepth %d rrDepth %d shapes %d segments %llu bsdf %d\n", info.width, info.height,
           info.spp, info.max_depth, info.rr_depth, info.n_shapes, (unsigned long long) info.segments, info.bsdf);

    size_t n = (size_t) info.width * (size_t) info.height * 4;
    float *film = (float *) calloc(n, sizeof(float));
    hpt_render_params p;
    memset(&p, 0, sizeof(p));
    p.spp_begin = 0;
    p.spp_end = info.spp;
    p.shard = 0;
    p.n_shards = 1;
    rc = hpt_render(ctx, &p, film);
    if (device == HPT_HOST_ONLY) {
        /* a host-only context parses and builds but never renders: the call must fail loudly */
        printf("host-only render refused: %d (%s)\n", rc, hpt_last_error(ctx));
        free(film);
        hpt_context_destroy(ctx);
        for (i = 0; i < n_defines; ++i) free(kv_store[i]);
        return rc == HPT_EDEVICE ? 0 : 1;
    }
    if (rc != HPT_OK) return fail(ctx, "hpt_render", rc);

    double sum = 0.0;
    for (i = 0; i < (int) n; ++i) sum += film[i];
    printf("film checksum %.9g\n", sum);
    if (raw) {
        FILE *f = fopen(raw, "wb");
        if (!f || fwrite(film, sizeof(float), n, f) != n) return fail(ctx, "writing the raw film", -2);
        fclose(f);
    }
    if (out) {
        hpt_film_params fp;
        char written[4096];
        if ((rc = hpt_get_film_params(ctx, &fp)) != HPT_OK) return fail(ctx, "hpt_get_film_params", rc);
        if ((rc = hpt_write_film(ctx, out, film, info.width, info.height, &fp, written, sizeof(written))) != HPT_OK)
            return fail(ctx, "hpt_write_film", rc);
        printf("wrote %s\n", written);
    }
    free(film);
    hpt_context_destroy(ctx);
    for (i = 0; i < n_defines; ++i) free(kv_store[i]);
    return 0;
}
