/*
 * fetch_calib.hip -- known-byte calibration of rocprofv3's FETCH_SIZE for the
 * access patterns of the traversal kernels (8-byte node words, 32-byte
 * records, 16-byte-per-lane streams), on MI355X.
 *
 * The guide (MI355X_MICROARCH.md, HBM) calibrates FETCH_SIZE x 2 only for wide
 * coalesced 16-B-per-lane streaming reads; k_trace gathers 8-B and 32-B
 * records.  Each kernel below reads a byte count known in advance:
 *   k_stream     every lane reads 16 B, consecutive (whole 128-B lines)
 *   k_gather<R>  every lane reads one R-byte record (R = 8, 32) from its own
 *                128-B line; lines are a bijective odd-multiplier map of the
 *                lane index over a power-of-two line count, so no line is
 *                read twice in a launch
 * over regions far from the last-written 256 MiB ("cold": every line comes
 * from HBM) and over a 64 MiB window read by a previous launch
 * ("resident": the lines sit in the Infinity Cache).  tools/fetch_calib.py
 * divides each launch's FETCH_SIZE (rocprofv3 --pmc FETCH_SIZE) by its lines
 * and by its record bytes.
 *
 * Build: hipcc --offload-arch=gfx950 -O3 tools/fetch_calib.hip -o tools/fetch_calib
 */
#include <hip/hip_runtime.h>

#include <cstdio>
#include <cstdlib>

#define CHECK(x)                                                                                    \
    do {                                                                                            \
        hipError_t e_ = (x);                                                                        \
        if (e_ != hipSuccess) {                                                                     \
            std::fprintf(stderr, "%s: %s\n", #x, hipGetErrorString(e_));                            \
            std::exit(1);                                                                           \
        }                                                                                           \
    } while (0)

/* the result of every read is folded into one word per wave, so nothing is dead code */
__global__ void k_stream(const float4 *__restrict__ src, uint64_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x) {
        const float4 v = src[i];
        acc ^= __float_as_uint(v.x) ^ __float_as_uint(v.y) ^ __float_as_uint(v.z) ^ __float_as_uint(v.w);
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

/* writes: 16 B per lane, consecutive (k_stream_w) or one 16-B store per 128-B line (k_scatter16,
   the hit-record pattern of k_trace: one path-indexed float4 per ray) */
__global__ void k_stream_w(float4 *__restrict__ dst, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x)
        dst[i] = make_float4((float) i, 1.0f, 2.0f, 3.0f);
}
__global__ void k_scatter16(uint8_t *__restrict__ base, uint64_t lineMask, uint64_t n) {
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x) {
        const uint64_t line = (i * 0x9E3779B97F4A7C15ull) & lineMask;
        *reinterpret_cast<float4 *>(base + line * 128) = make_float4((float) i, 1.0f, 2.0f, 3.0f);
    }
}

template <int R>
__global__ void k_gather(const uint8_t *__restrict__ base, uint64_t lineMask, uint64_t n, uint32_t *__restrict__ sink) {
    uint32_t acc = 0;
    for (uint64_t i = blockIdx.x * (uint64_t) blockDim.x + threadIdx.x; i < n; i += (uint64_t) gridDim.x * blockDim.x) {
        const uint64_t line = (i * 0x9E3779B97F4A7C15ull) & lineMask; /* odd multiplier: a bijection mod 2^k */
        const uint8_t *p = base + line * 128;
        if (R == 8) {
            const uint2 v = *reinterpret_cast<const uint2 *>(p);
            acc ^= v.x ^ v.y;
        } else {
            const uint4 a = reinterpret_cast<const uint4 *>(p)[0], b = reinterpret_cast<const uint4 *>(p)[1];
            acc ^= a.x ^ a.y ^ a.z ^ a.w ^ b.x ^ b.y ^ b.z ^ b.w;
        }
    }
    if (acc == 0x9e3779b9u) sink[0] = acc;
}

int main() {
    /* 6 GiB, filled once: the fill's last 256 MiB stay in the Infinity Cache, so the cold
       launches read regions far from it: gathers over [0, 2) and [2, 4) GiB, the stream
       over [4, 5) GiB */
    const uint64_t bufBytes = 6ull << 30, regionLines = (2ull << 30) / 128; /* 2^24 lines */
    const uint64_t winBytes = 64ull << 20, winLines = winBytes / 128;       /* 2^19 lines */
    uint8_t *buf = nullptr;
    uint32_t *sink = nullptr;
    CHECK(hipMalloc(&buf, bufBytes));
    CHECK(hipMalloc(&sink, 64));
    CHECK(hipMemset(buf, 1, bufBytes));
    CHECK(hipDeviceSynchronize());
    const dim3 grid(4096), block(256);
    const uint64_t gatherN = 1ull << 22; /* lines per cold gather launch */
    /* launch order = the order tools/fetch_calib.py expects */
    std::printf("launch 0 gather8_cold lines %llu record 8\n", (unsigned long long) gatherN);
    hipLaunchKernelGGL(k_gather<8>, grid, block, 0, 0, buf, regionLines - 1, gatherN, sink);
    std::printf("launch 1 gather32_cold lines %llu record 32\n", (unsigned long long) gatherN);
    hipLaunchKernelGGL(k_gather<32>, grid, block, 0, 0, buf + (2ull << 30), regionLines - 1, gatherN, sink);
    std::printf("launch 2 stream_cold lines %llu record 128\n", (unsigned long long) ((1ull << 30) / 128));
    hipLaunchKernelGGL(k_stream, grid, block, 0, 0, (const float4 *) (buf + (4ull << 30)), (1ull << 30) / 16, sink);
    /* resident: warm a 64 MiB window (launch 3), then gather from it (4, 5) */
    std::printf("launch 3 stream_warm lines %llu record 128\n", (unsigned long long) winLines);
    hipLaunchKernelGGL(k_stream, grid, block, 0, 0, (const float4 *) buf, winBytes / 16, sink);
    std::printf("launch 4 gather8_resident lines %llu record 8\n", (unsigned long long) winLines);
    hipLaunchKernelGGL(k_gather<8>, grid, block, 0, 0, buf, winLines - 1, winLines, sink);
    std::printf("launch 5 gather32_resident lines %llu record 32\n", (unsigned long long) winLines);
    hipLaunchKernelGGL(k_gather<32>, grid, block, 0, 0, buf, winLines - 1, winLines, sink);
    /* writes (WRITE_SIZE): 1 GiB streamed, then 2^22 lone 16-B stores into distinct lines */
    std::printf("launch 6 stream_write lines %llu record 128\n", (unsigned long long) ((1ull << 30) / 128));
    hipLaunchKernelGGL(k_stream_w, grid, block, 0, 0, (float4 *) (buf + (4ull << 30)), (1ull << 30) / 16);
    std::printf("launch 7 scatter16 lines %llu record 16\n", (unsigned long long) gatherN);
    hipLaunchKernelGGL(k_scatter16, grid, block, 0, 0, buf, regionLines - 1, gatherN);
    CHECK(hipDeviceSynchronize());
    CHECK(hipFree(buf));
    CHECK(hipFree(sink));
    return 0;
}
