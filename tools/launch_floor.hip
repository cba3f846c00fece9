// Launch-mode probe: how long does the same kernel take (as the rocprof kernel trace reports it) when it is
// dispatched (a) by hipLaunchKernelGGL, (b) by hipExtLaunchKernelGGL with dispatch-attached events, (c) from a
// replayed hipGraph — for an empty kernel, a copy of K1's bytes and K1 itself at 4096 x 128.
//
//   hipcc --offload-arch=gfx950 -O3 tools/launch_floor.hip -o gpurun_out/launch_floor
//   rocprofv3 --kernel-trace --stats -d gpurun_out/lf -o lf -- gpurun_out/launch_floor
//
// Run it with HIP_FORCE_DEV_KERNARG=0/1 to see whether kernel arguments in host memory set the floor.
#include <stdio.h>
#include <stdlib.h>

#include "../xuanpolicy_amd/csrc/gae.hip"

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ __launch_bounds__(256) void lf_empty_direct(float *p) {
    if (p && threadIdx.x == 255) p[0] = 0.f;
}
__global__ __launch_bounds__(256) void lf_empty_events(float *p) {
    if (p && threadIdx.x == 255) p[0] = 0.f;
}
__global__ __launch_bounds__(256) void lf_empty_graph(float *p) {
    if (p && threadIdx.x == 255) p[0] = 0.f;
}

template <int MODE>
__global__ __launch_bounds__(256) void lf_copy(const float *r, const float *v, const float *d, const float *q,
                                               float *a, float *o, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const f4 x = __builtin_nontemporal_load((const f4 *)r + i);
    const f4 y = __builtin_nontemporal_load((const f4 *)v + i);
    const f4 z = __builtin_nontemporal_load((const f4 *)d + i);
    const f4 w = __builtin_nontemporal_load((const f4 *)q + i);
    __builtin_nontemporal_store(x + y * z + w, (f4 *)a + i);
    __builtin_nontemporal_store(x * y + z, (f4 *)o + i);
}

__global__ __launch_bounds__(256) void lf_produce(float *r, float *v, float *d, uint8_t *c, int64_t n, int T,
                                                  uint32_t salt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = xpa_mix32((uint32_t)i ^ salt);
    r[i] = (float)(h & 0xffff) * 1e-4f;
    v[i] = (float)(h >> 16) * 1e-4f;
    const int t = (int)(i % T);
    d[i] = 0.f;
    c[i] = (t == T - 1) ? 1 : 0;
}

int main(int argc, char **argv) {
    const int64_t envs = argc > 1 ? atoll(argv[1]) : 4096;
    const int T = 128;
    const int64_t n = envs * T, n4 = n / 4;
    float *r, *v, *d, *q, *a, *o;
    uint8_t *c;
    CK(hipMalloc(&r, n * 4));
    CK(hipMalloc(&v, n * 4));
    CK(hipMalloc(&d, n * 4));
    CK(hipMalloc(&q, n * 4));
    CK(hipMalloc(&a, n * 4));
    CK(hipMalloc(&o, n * 4));
    CK(hipMalloc(&c, n));
    CK(hipMemset(q, 0, n * 4));
    hipStream_t s;
    CK(hipStreamCreateWithFlags(&s, hipStreamNonBlocking));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned pb = (unsigned)((n + 255) / 256), cb = (unsigned)((n4 + 255) / 256);
    const int reps = 40;
    // (a) plain launches, each after a produce (as in the training loop)
    for (int i = 0; i < reps; ++i) {
        hipLaunchKernelGGL(lf_produce, dim3(pb), dim3(256), 0, s, r, v, d, c, n, T, (uint32_t)i);
        hipLaunchKernelGGL(lf_empty_direct, dim3(1), dim3(256), 0, s, (float *)nullptr);
        hipLaunchKernelGGL(lf_copy<0>, dim3(cb), dim3(256), 0, s, r, v, d, q, a, o, n4);
        CK((hipError_t)xpa_gae_scan(r, v, d, c, q, envs, T, 0.99f, 0.95f, 1, a, o, s));
    }
    CK(hipStreamSynchronize(s));
    // (b) dispatch-attached events
    double ev_gae = 0, ev_empty = 0;
    for (int i = 0; i < reps; ++i) {
        hipLaunchKernelGGL(lf_produce, dim3(pb), dim3(256), 0, s, r, v, d, c, n, T, (uint32_t)i);
        hipExtLaunchKernelGGL(lf_empty_events, dim3(1), dim3(256), 0, s, e0, e1, 0, (float *)nullptr);
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        ev_empty += ms;
        hipExtLaunchKernelGGL(lf_copy<1>, dim3(cb), dim3(256), 0, s, e0, e1, 0, r, v, d, q, a, o, n4);
        CK((hipError_t)xpa_gae_scan_timed(r, v, d, c, q, envs, T, 0.99f, 0.95f, 1, a, o, e0, e1, s));
        CK(hipEventSynchronize(e1));
        CK(hipEventElapsedTime(&ms, e0, e1));
        ev_gae += ms;
    }
    // (c) graph replays of [produce, empty, copy, gae]
    hipGraph_t g;
    hipGraphExec_t ge;
    CK(hipStreamBeginCapture(s, hipStreamCaptureModeThreadLocal));
    hipLaunchKernelGGL(lf_produce, dim3(pb), dim3(256), 0, s, r, v, d, c, n, T, 7u);
    hipLaunchKernelGGL(lf_empty_graph, dim3(1), dim3(256), 0, s, (float *)nullptr);
    hipLaunchKernelGGL(lf_copy<2>, dim3(cb), dim3(256), 0, s, r, v, d, q, a, o, n4);
    CK((hipError_t)xpa_gae_scan(r, v, d, c, q, envs, T, 0.99f, 0.95f, 1, a, o, s));
    CK(hipStreamEndCapture(s, &g));
    CK(hipGraphInstantiate(&ge, g, nullptr, nullptr, 0));
    for (int i = 0; i < reps; ++i) CK(hipGraphLaunch(ge, s));
    CK(hipStreamSynchronize(s));
    const char *kv = getenv("HIP_FORCE_DEV_KERNARG");
    printf("{\"HIP_FORCE_DEV_KERNARG\": \"%s\", \"event_empty_us\": %.3f, \"event_gae_us\": %.3f}\n", kv ? kv : "unset",
           ev_empty / reps * 1e3, ev_gae / reps * 1e3);
    return 0;
}
