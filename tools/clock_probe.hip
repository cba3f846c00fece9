// Clock under MFMA load (r06): the in-kernel clock method of MI355X_MICROARCH.md "DVFS give-back"
// item 6 — delta s_memtime / delta s_memrealtime x 100 MHz, stamped once around the loop of every workgroup, median over
// workgroups, after >= 2 s of back-to-back launches on random data — for MFMA-dense loops of the shapes the update and
// the C3 convolutions use, against a known cycle count (v_mfma_f32_32x32x16_bf16 issues back-to-back at 32 cycles per
// instruction on one SIMD, one wave per SIMD) and, in a separate rocprofv3 --pmc GRBM_GUI_ACTIVE pass of the same
// program, against GRBM_GUI_ACTIVE / 8 / duration on the same >= 10 ms dispatches.  Diagnostic only: nothing in the
// product library is built from this file.
//
//   hipcc --offload-arch=gfx950 -O3 -o tools/_probe/clock_probe tools/clock_probe.hip
//   tools/_probe/clock_probe            # JSON lines on stdout
#include <hip/hip_runtime.h>

#include <algorithm>
#include <chrono>
#include <cstdio>
#include <cstdlib>
#include <vector>

typedef __bf16 bf16x8 __attribute__((ext_vector_type(8)));
typedef float f32x16 __attribute__((ext_vector_type(16)));
typedef float f32x4 __attribute__((ext_vector_type(4)));

#define CHECK(x)                                                                        \
    do {                                                                                \
        hipError_t e_ = (x);                                                            \
        if (e_ != hipSuccess) {                                                         \
            std::fprintf(stderr, "%s:%d %s\n", __FILE__, __LINE__, hipGetErrorString(e_)); \
            std::exit(1);                                                               \
        }                                                                               \
    } while (0)

// MODE 0: v_mfma_f32_32x32x16_bf16 (the split GEMMs); 1: v_mfma_f32_32x32x2_f32; 2: v_mfma_f32_16x16x4f32 (K28 / K29).
// Four independent accumulators per wave; operands in registers, seeded from `seed` (random) or zero.
template <int MODE>
__global__ __launch_bounds__(256) void mfma_loop(int iters, int zero, const float *__restrict__ seed, float *out,
                                                 unsigned long long *stamps) {
    const int lane = threadIdx.x & 63;
    const float s0 = zero ? 0.f : seed[(blockIdx.x * 256 + threadIdx.x) & 4095];
    __syncthreads();
    unsigned long long t0 = 0, r0 = 0;
    if (threadIdx.x == 0) {
        t0 = __builtin_amdgcn_s_memtime();
        r0 = __builtin_amdgcn_s_memrealtime();
    }
    float res = 0.f;
    if constexpr (MODE == 0) {
        bf16x8 a, b;
        for (int k = 0; k < 8; ++k) {
            a[k] = (__bf16)(s0 * (float)(k + 1) + 0.001f * lane);
            b[k] = (__bf16)(s0 * (float)(8 - k) - 0.002f * lane);
        }
        f32x16 acc[4];
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x16_bf16(a, b, acc[j], 0, 0, 0);
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 16; ++r) res += acc[j][r];
    } else if constexpr (MODE == 1) {
        const float a = s0 + 0.001f * lane, b = s0 - 0.002f * lane;
        f32x16 acc[4];
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 16; ++r) acc[j][r] = 0.f;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_32x32x2f32(a, b, acc[j], 0, 0, 0);
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 16; ++r) res += acc[j][r];
    } else {
        const float a = s0 + 0.001f * lane, b = s0 - 0.002f * lane;
        f32x4 acc[4];
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 4; ++r) acc[j][r] = 0.f;
        for (int it = 0; it < iters; ++it)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[j] = __builtin_amdgcn_mfma_f32_16x16x4f32(a, b, acc[j], 0, 0, 0);
        for (int j = 0; j < 4; ++j)
            for (int r = 0; r < 4; ++r) res += acc[j][r];
    }
    __syncthreads();
    if (threadIdx.x == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;       // vector stores of the stamp pair (a buffer nothing else reads)
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    out[blockIdx.x * 256 + threadIdx.x] = res;
}

template <int MODE>
static void run(const char *name, int zero, int cycles_per_mfma, const float *seed, float *out,
                unsigned long long *stamps, int blocks) {
    // iterations so that one launch takes ~20 ms at ~2 GHz (4 MFMAs per iteration per wave, one wave per SIMD)
    const int cyc = cycles_per_mfma > 0 ? cycles_per_mfma : 32;
    const int iters = (int)(20e-3 * 2.0e9 / (4.0 * cyc));
    hipEvent_t e0, e1;
    CHECK(hipEventCreate(&e0));
    CHECK(hipEventCreate(&e1));
    const auto start = std::chrono::steady_clock::now();
    int warm = 0;
    while (std::chrono::duration<double>(std::chrono::steady_clock::now() - start).count() < 2.5) {
        hipLaunchKernelGGL(mfma_loop<MODE>, dim3(blocks), dim3(256), 0, 0, iters, zero, seed, out, stamps);
        if (++warm % 16 == 0) CHECK(hipDeviceSynchronize());
    }
    CHECK(hipDeviceSynchronize());
    CHECK(hipEventRecord(e0, 0));
    hipLaunchKernelGGL(mfma_loop<MODE>, dim3(blocks), dim3(256), 0, 0, iters, zero, seed, out, stamps);
    CHECK(hipEventRecord(e1, 0));
    CHECK(hipEventSynchronize(e1));
    float ms = 0.f;
    CHECK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> st(2 * blocks);
    CHECK(hipMemcpy(st.data(), stamps, st.size() * sizeof(unsigned long long), hipMemcpyDeviceToHost));
    std::vector<double> ghz(blocks);
    std::vector<double> wall_us(blocks);
    for (int b = 0; b < blocks; ++b) {
        ghz[b] = (double)st[2 * b] / (double)st[2 * b + 1] * 0.1;   // s_memrealtime ticks at 100 MHz
        wall_us[b] = (double)st[2 * b + 1] / 100.0;
    }
    std::sort(ghz.begin(), ghz.end());
    std::sort(wall_us.begin(), wall_us.end());
    const double med = ghz[blocks / 2];
    // the known-cycle clock: the loop's MFMA cycles over the workgroups' median stamped wall time
    const double known = cycles_per_mfma > 0 ? (double)iters * 4.0 * cycles_per_mfma / (wall_us[blocks / 2] * 1e3) : -1.0;
    std::printf("{\"mode\": \"%s\", \"data\": \"%s\", \"iters\": %d, \"blocks\": %d, \"warm_launches\": %d, "
                "\"launch_ms\": %.3f, \"inkernel_clock_ghz_median\": %.4f, \"inkernel_clock_ghz_p10\": %.4f, "
                "\"inkernel_clock_ghz_p90\": %.4f, \"known_cycle_clock_ghz\": %.4f}\n",
                name, zero ? "zero" : "random", iters, blocks, warm, ms, med, ghz[blocks / 10], ghz[blocks * 9 / 10],
                known);
    std::fflush(stdout);
    CHECK(hipEventDestroy(e0));
    CHECK(hipEventDestroy(e1));
}

int main() {
    hipDeviceProp_t p;
    CHECK(hipGetDeviceProperties(&p, 0));
    const int blocks = p.multiProcessorCount;   // one 4-wave block per CU = one wave per SIMD
    float *seed, *out;
    unsigned long long *stamps;
    CHECK(hipMalloc(&seed, 4096 * sizeof(float)));
    CHECK(hipMalloc(&out, (size_t)blocks * 256 * sizeof(float)));
    CHECK(hipMalloc(&stamps, (size_t)blocks * 2 * sizeof(unsigned long long)));
    std::vector<float> h(4096);
    unsigned s = 12345u;
    for (auto &v : h) {
        s = s * 1664525u + 1013904223u;
        v = ((s >> 8) & 0xFFFF) / 65536.0f - 0.5f;
    }
    CHECK(hipMemcpy(seed, h.data(), h.size() * sizeof(float), hipMemcpyHostToDevice));
    run<0>("mfma_f32_32x32x16_bf16", 0, 32, seed, out, stamps, blocks);
    run<0>("mfma_f32_32x32x16_bf16", 1, 32, seed, out, stamps, blocks);
    run<1>("mfma_f32_32x32x2_f32", 0, 0, seed, out, stamps, blocks);
    run<2>("mfma_f32_16x16x4_f32", 0, 0, seed, out, stamps, blocks);
    run<0>("mfma_f32_32x32x16_bf16", 0, 32, seed, out, stamps, blocks);   // again, after the f32 loops
    CHECK(hipFree(seed));
    CHECK(hipFree(out));
    CHECK(hipFree(stamps));
    return 0;
}
