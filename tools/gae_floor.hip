// Floor probe for the K1 GAE scan at the bench size (4096 x 128): how much of its launch time is the
// scan, how much the dependent bootstrap read, and how much any launch of this geometry costs.
//
//   hipcc --offload-arch=gfx950 -O3 -I xuanpolicy_amd/csrc tools/gae_floor.hip -o gpurun_out/gae_floor
//   gpurun_out/gae_floor [n_envs] [horizon]
//
// Every variant is timed by events the dispatch itself records (hipExtLaunchKernelGGL), like bench.py,
// in three cache states: "hot" (back-to-back relaunches), "produced" (a kernel rewrites the inputs just
// before, as the rollout does in the training loop), "flushed" (512 MiB written in between).
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

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

__global__ __launch_bounds__(1024) void empty_kernel(float *p) {
    if (p && threadIdx.x == 1023) p[0] = 0.f;
}

// dispatch-event duration of an empty kernel by grid / block size
static void empty_sweep() {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const unsigned grids[] = {1, 64, 256, 512, 1024, 2048, 8192};
    const unsigned blocks[] = {64, 256, 1024};
    for (unsigned bs : blocks)
        for (unsigned g : grids) {
            double tot = 0;
            for (int it = 0; it < 53; ++it) {
                hipExtLaunchKernelGGL(empty_kernel, dim3(g), dim3(bs), 0, 0, e0, e1, 0, (float *)nullptr);
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 3) tot += ms;
            }
            fprintf(stderr, "empty grid %5u x %4u: %.3f us\n", g, bs, tot / 50 * 1e3);
        }
}

// GAE's access pattern without the scan: 3 x 16-B nt loads + 1 dword per lane, 2 x 16-B nt stores.
__global__ __launch_bounds__(256) void copy_kernel(const float *r, const float *v, const float *d, const uint32_t *c,
                                                   float *a, float *o, int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const f4 x = __builtin_nontemporal_load((const f4 *)r + i);
    const f4 y = __builtin_nontemporal_load((const f4 *)v + i);
    const f4 z = __builtin_nontemporal_load((const f4 *)d + i);
    const uint32_t w = c[i];
    __builtin_nontemporal_store(x + y * z + (float)(w & 1), (f4 *)a + i);
    __builtin_nontemporal_store(x * y + z, (f4 *)o + i);
}

// what the rollout does before GAE: writes r, v, d, closed
__global__ __launch_bounds__(256) void produce_kernel(float *r, float *v, float *d, uint8_t *c, int64_t n, int T,
                                                      int with_mid, uint32_t salt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = xpa_mix32((uint32_t)i ^ salt);
    r[i] = (float)(h & 0xffff) * 1e-4f;
    v[i] = (float)(h >> 16) * 1e-4f;
    const int t = (int)(i % T);
    const bool mid = with_mid && (h % 997u == 0);
    d[i] = mid ? 1.f : 0.f;
    c[i] = (t == T - 1 || mid) ? 1 : 0;
}

__global__ __launch_bounds__(256) void flush_kernel(f4 *p, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
        p[i] = f4{1.f, 2.f, 3.f, 4.f};
}

struct Bufs {
    float *r, *v, *d, *boot, *adv, *ret;
    uint8_t *c;
    f4 *big;
    int64_t n, big4;
    int T;
};

enum Variant { EMPTY, COPY, GAE, GAE_NOCLOSE };
enum State { HOT, PRODUCED, FLUSHED };

static float run(const Bufs &b, Variant var, State st, int reps, int with_mid) {
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const int64_t n4 = b.n / 4;
    const unsigned gblocks = (unsigned)((n4 + 255) / 256);
    const int64_t envs = b.n / b.T;
    double tot = 0;
    int cnt = 0;
    for (int it = 0; it < reps + 3; ++it) {
        if (st == PRODUCED || it == 0)
            hipLaunchKernelGGL(produce_kernel, dim3((unsigned)((b.n + 255) / 256)), dim3(256), 0, 0, b.r, b.v, b.d,
                               b.c, b.n, b.T, var == GAE_NOCLOSE ? 0 : with_mid, (uint32_t)it);
        if (var == GAE_NOCLOSE && (st == PRODUCED || it == 0)) CK(hipMemset(b.c, 0, b.n));
        if (st == FLUSHED) hipLaunchKernelGGL(flush_kernel, dim3(4096), dim3(256), 0, 0, b.big, b.big4);
        switch (var) {
            case EMPTY:
                hipExtLaunchKernelGGL(empty_kernel, dim3(gblocks / 2), dim3(256), 0, 0, e0, e1, 0, (float *)nullptr);
                break;
            case COPY:
                hipExtLaunchKernelGGL(copy_kernel, dim3(gblocks), dim3(256), 0, 0, e0, e1, 0, b.r, b.v, b.d,
                                      (const uint32_t *)b.c, b.adv, b.ret, n4);
                break;
            default:
                CK((hipError_t)xpa_gae_scan_timed(b.r, b.v, b.d, b.c, b.boot, envs, b.T, 0.99f, 0.95f, 1, b.adv,
                                                  b.ret, e0, e1, 0));
        }
        CK(hipEventSynchronize(e1));
        float ms;
        CK(hipEventElapsedTime(&ms, e0, e1));
        if (it >= 3) {
            tot += ms;
            ++cnt;
        }
    }
    CK(hipEventDestroy(e0));
    CK(hipEventDestroy(e1));
    return (float)(tot / cnt * 1e3);
}

int main(int argc, char **argv) {
    const int64_t envs = argc > 1 ? atoll(argv[1]) : 4096;
    const int T = argc > 2 ? atoi(argv[2]) : 128;
    if (argc > 3 && !strcmp(argv[3], "empty")) {
        empty_sweep();
        return 0;
    }
    Bufs b;
    b.n = envs * T;
    b.T = T;
    CK(hipMalloc(&b.r, b.n * 4));
    CK(hipMalloc(&b.v, b.n * 4));
    CK(hipMalloc(&b.d, b.n * 4));
    CK(hipMalloc(&b.boot, b.n * 4));
    CK(hipMalloc(&b.adv, b.n * 4));
    CK(hipMalloc(&b.ret, b.n * 4));
    CK(hipMalloc(&b.c, b.n));
    CK(hipMemset(b.boot, 0, b.n * 4));
    b.big4 = (512ll << 20) / 16;
    CK(hipMalloc(&b.big, b.big4 * 16));
    const double alg = 20.0 * b.n;  // algorithmic bytes
    const char *vn[] = {"empty(same grid)", "copy(same bytes)", "gae", "gae(no closures)"};
    const char *sn[] = {"hot", "produced", "flushed"};
    printf("{\"n_envs\": %lld, \"horizon\": %d, \"algorithmic_bytes\": %.0f, \"us\": {", (long long)envs, T, alg);
    bool first = true;
    for (int v = 0; v < 4; ++v)
        for (int s = 0; s < 3; ++s) {
            const float us = run(b, (Variant)v, (State)s, 50, 1);
            printf("%s\"%s/%s\": %.3f", first ? "" : ", ", vn[v], sn[s], us);
            fprintf(stderr, "%-18s %-9s %8.3f us  %7.1f GB/s-alg\n", vn[v], sn[s], us, alg / us * 1e-3);
            first = false;
        }
    printf("}}\n");
    return 0;
}
