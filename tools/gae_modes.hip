// K1 launch-mode probe (4096 x 128): rocprof kernel-trace durations of the dense and compact GAE forms and
// of a 20-B/step copy, each dispatched (iso) to an idle queue after a host sync, (chain) right behind the
// kernel that produced its inputs on the same stream, (xs) on a second stream that waits on the producer's
// event.  Separate kernel names per mode so the trace tells them apart.
//
//   hipcc --offload-arch=gfx950 -O3 tools/gae_modes.hip -o tools/_probe/gae_modes
//   rocprofv3 --kernel-trace --stats -d gpurun_out/gm -o gm -- tools/_probe/gae_modes
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

template <int MODE>
__global__ __launch_bounds__(256) void gm_copy20(const float *r, const float *v, const float *d, float *a, float *o,
                                                 int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const f4 x = __builtin_nontemporal_load((const f4 *)r + i);
    const f4 y = __builtin_nontemporal_load((const f4 *)v + i);
    const f4 z = __builtin_nontemporal_load((const f4 *)d + i);
    __builtin_nontemporal_store(x + y * z, (f4 *)a + i);
    __builtin_nontemporal_store(x * y + z, (f4 *)o + i);
}

template <int MODE>
__global__ __launch_bounds__(256) void gm_empty(float *p) {
    if (p && threadIdx.x == 255) p[0] = 0.f;
}

__global__ __launch_bounds__(256) void gm_produce(float *r, float *v, float *d, uint8_t *c, float *q, int *slot,
                                                  int64_t n, int T, uint32_t salt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = xpa_mix32((uint32_t)i ^ salt);
    r[i] = (float)(h & 0xffff) * 1e-4f;
    v[i] = (float)(h >> 16) * 1e-4f;
    const int t = (int)(i % T);
    const bool term = (h % 101u) == 0;
    const bool trunc = !term && (h % 1009u) == 0;
    d[i] = term ? 1.f : 0.f;
    c[i] = (t == T - 1 || term || trunc) ? 1 : 0;
    q[i] = trunc ? 0.5f : 0.f;
    if (t == 0) slot[i / T] = ((h >> 7) % 8u == 0) ? (int)((h >> 11) % (unsigned)(T - 1)) : -1;
}

struct B {
    float *r, *v, *d, *q, *a, *o, *vb;
    uint8_t *c;
    int *slot;
    int64_t envs, n;
    int T;
};

template <int MODE>
static void launch(const B &b, int which, hipStream_t s) {
    const int64_t n4 = b.n / 4;
    switch (which) {
        case 0:
            hipLaunchKernelGGL(gm_empty<MODE>, dim3(1), dim3(256), 0, s, (float *)nullptr);
            break;
        case 1:
            hipLaunchKernelGGL(gm_copy20<MODE>, dim3((unsigned)((n4 + 255) / 256)), dim3(256), 0, s, b.r, b.v, b.d,
                               b.a, b.o, n4);
            break;
        case 2:
            CK((hipError_t)xpa_gae_scan(b.r, b.v, b.d, b.c, b.q, b.envs, b.T, 0.99f, 0.95f, 1, b.a, b.o, s));
            break;
        case 3:
            CK((hipError_t)xpa_gae_scan_compact(b.r, b.v, b.d, b.slot, b.vb, b.envs, b.T, 0.99f, 0.95f, 1, b.a, b.o,
                                                b.q, nullptr, nullptr, s));
            break;
    }
}

int main(int argc, char **argv) {
    B b;
    b.envs = argc > 1 ? atoll(argv[1]) : 4096;
    b.T = 128;
    b.n = b.envs * b.T;
    CK(hipMalloc(&b.r, b.n * 4));
    CK(hipMalloc(&b.v, b.n * 4));
    CK(hipMalloc(&b.d, b.n * 4));
    CK(hipMalloc(&b.q, b.n * 4));
    CK(hipMalloc(&b.a, b.n * 4));
    CK(hipMalloc(&b.o, b.n * 4));
    CK(hipMalloc(&b.vb, b.envs * 8));
    CK(hipMalloc(&b.c, b.n));
    CK(hipMalloc(&b.slot, b.envs * 4));
    CK(hipMemset(b.vb, 0, b.envs * 8));
    hipStream_t s1, s2;
    CK(hipStreamCreateWithFlags(&s1, hipStreamNonBlocking));
    CK(hipStreamCreateWithFlags(&s2, hipStreamNonBlocking));
    hipEvent_t ep, eg;
    CK(hipEventCreateWithFlags(&ep, hipEventDisableTiming));
    CK(hipEventCreateWithFlags(&eg, hipEventDisableTiming));
    const unsigned pb = (unsigned)((b.n + 255) / 256);
    const int reps = 30;
    for (int which = 0; which < 4; ++which) {
        for (int i = 0; i < reps; ++i) {  // iso: inputs produced, host sync, then the launch on an idle queue
            hipLaunchKernelGGL(gm_produce, dim3(pb), dim3(256), 0, s1, b.r, b.v, b.d, b.c, b.q, b.slot, b.n, b.T,
                               (uint32_t)i);
            CK(hipStreamSynchronize(s1));
            launch<0>(b, which, s1);
            CK(hipStreamSynchronize(s1));
        }
        for (int i = 0; i < reps; ++i) {  // chain: right behind the producer on the same stream
            hipLaunchKernelGGL(gm_produce, dim3(pb), dim3(256), 0, s1, b.r, b.v, b.d, b.c, b.q, b.slot, b.n, b.T,
                               (uint32_t)i);
            launch<1>(b, which, s1);
        }
        CK(hipStreamSynchronize(s1));
        for (int i = 0; i < reps; ++i) {  // xs: second stream waits on the producer's event
            hipLaunchKernelGGL(gm_produce, dim3(pb), dim3(256), 0, s1, b.r, b.v, b.d, b.c, b.q, b.slot, b.n, b.T,
                               (uint32_t)i);
            CK(hipEventRecord(ep, s1));
            CK(hipStreamWaitEvent(s2, ep, 0));
            launch<2>(b, which, s2);
            CK(hipEventRecord(eg, s2));
            CK(hipStreamWaitEvent(s1, eg, 0));
        }
        CK(hipStreamSynchronize(s1));
    }
    printf("done\n");
    return 0;
}
