// K1 compact-form probe (the in-loop GAE launch of the C2 fast path, xpa_gae_scan_compact), built to be
// read by rocprofv3 --kernel-trace as well as by its own dispatch-attached events.
//
//   hipcc --offload-arch=gfx950 -O3 -I xuanpolicy_amd/csrc tools/gae_probe.hip -o tools/_probe/gae_probe
//   (A/B against another revision: -DGAE_SRC='"path/to/gae.hip"')
//   tools/_probe/gae_probe [n_envs] [horizon] [reps]
//   rocprofv3 --kernel-trace --output-format csv -d gpurun_out/gp -o gp -- tools/_probe/gae_probe
//   python tools/gae_probe_summary.py gpurun_out/gp/.../gp_kernel_trace.csv
//
// Each (variant, cache state) phase is opened by one `phase_marker` dispatch and the phase names are
// printed in order on stdout, so the trace can be cut into phases.  Cache states:
//   hot      back-to-back relaunches over the same inputs
//   produced a kernel rewrites r / v / d / slot_t just before (default-policy stores, as the rollout does)
//   dirty    produced, then a 16 MiB default-policy write to another buffer (the critic pass that precedes
//            the in-loop GAE leaves its activations dirty in L2)
//   flushed  produced, then 512 MiB written in between
#include <stdio.h>
#include <stdlib.h>
#include <string.h>

#include <algorithm>
#include <string>
#include <vector>

#ifndef GAE_SRC
#define GAE_SRC "../xuanpolicy_amd/csrc/gae.hip"
#endif
#include GAE_SRC

#define CK(x)                                                                                   \
    do {                                                                                        \
        hipError_t e_ = (x);                                                                    \
        if (e_ != hipSuccess) {                                                                 \
            fprintf(stderr, "%s:%d %s: %s\n", __FILE__, __LINE__, #x, hipGetErrorString(e_)); \
            exit(1);                                                                            \
        }                                                                                       \
    } while (0)

typedef float f4 __attribute__((ext_vector_type(4)));

__global__ void phase_marker(int *p) {
    if (p && threadIdx.x == 0) p[0] = 0;
}

__global__ __launch_bounds__(256) void empty_kernel(float *p) {
    if (p && threadIdx.x == 255) p[0] = 0.f;
}

// the compact form's bytes without the scan: 3 x 16-B nt loads, 2 x 16-B nt stores per lane
__global__ __launch_bounds__(256) void copy_kernel(const float *r, const float *v, const float *d, float *a, float *o,
                                                   int64_t n4) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n4) return;
    const f4 x = __builtin_nontemporal_load((const f4 *)r + i);
    const f4 y = __builtin_nontemporal_load((const f4 *)v + i);
    const f4 z = __builtin_nontemporal_load((const f4 *)d + i);
    __builtin_nontemporal_store(x + y * z, (f4 *)a + i);
    __builtin_nontemporal_store(x * y + z, (f4 *)o + i);
}

// as the rollout leaves the buffer: r, v, d columns, one truncation slot per ~1/8 of the envs
__global__ __launch_bounds__(256) void produce_kernel(float *r, float *v, float *d, int *slot, float *vboot,
                                                      int64_t n, int T, uint32_t salt) {
    const int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (i >= n) return;
    const uint32_t h = xpa_mix32((uint32_t)i ^ salt);
    r[i] = (float)(h & 0xffff) * 1e-4f;
    v[i] = (float)(h >> 16) * 1e-4f;
    d[i] = (h % 499u == 0) ? 1.f : 0.f;
    const int64_t envs = n / T;
    if (i < envs) {
        slot[i] = (h & 7u) == 0 ? (int)(h % (uint32_t)T) : -1;
        vboot[i] = 0.5f;
        vboot[envs + i] = 0.25f;
    }
}

__global__ __launch_bounds__(256) void fill_kernel(f4 *p, int64_t n4) {
    for (int64_t i = (int64_t)blockIdx.x * 256 + threadIdx.x; i < n4; i += (int64_t)gridDim.x * 256)
        p[i] = f4{1.f, 2.f, 3.f, 4.f};
}

enum Variant { EMPTY, COPY, GAE_COMPACT, NVAR };
enum State { HOT, PRODUCED, DIRTY, FLUSHED, NSTATE };
static const char *kVar[] = {"empty", "copy", "gae_compact"};
static const char *kState[] = {"hot", "produced", "dirty", "flushed"};

int main(int argc, char **argv) {
    const int64_t envs = argc > 1 ? atoll(argv[1]) : 4096;
    const int T = argc > 2 ? atoi(argv[2]) : 128;
    const int reps = argc > 3 ? atoi(argv[3]) : 40;
    const int64_t n = envs * T, n4 = n / 4;
    float *r, *v, *d, *adv, *ret, *boot, *vboot;
    int *slot, *mark;
    f4 *dirty, *big;
    CK(hipMalloc(&r, n * 4));
    CK(hipMalloc(&v, n * 4));
    CK(hipMalloc(&d, n * 4));
    CK(hipMalloc(&adv, n * 4));
    CK(hipMalloc(&ret, n * 4));
    CK(hipMalloc(&boot, n * 4));
    CK(hipMalloc(&vboot, 2 * envs * 4));
    CK(hipMalloc(&slot, envs * 4));
    CK(hipMalloc(&mark, 64));
    const int64_t dirty4 = (16ll << 20) / 16, big4 = (512ll << 20) / 16;
    CK(hipMalloc(&dirty, dirty4 * 16));
    CK(hipMalloc(&big, big4 * 16));
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    const double alg = 20.0 * n + 4.0 * envs;  // 20 B per (env, step) + 4 B per env
    const unsigned gblocks = (unsigned)((n4 + 255) / 256);
    // the compact launch's own geometry (xpa_gae_scan_compact: 64 / L rows per wave, 4 waves per block)
    int seg_log2 = 0;
    while ((1 << seg_log2) < (T + 3) / 4 && seg_log2 < 6) ++seg_log2;
    const unsigned gae_blocks = (unsigned)(((envs + (64 >> seg_log2) - 1) / (64 >> seg_log2) + 3) / 4);
    printf("{\"n_envs\": %lld, \"horizon\": %d, \"algorithmic_bytes\": %.0f, \"phases\": [", (long long)envs, T, alg);
    bool first = true;
    std::vector<std::string> lines;
    for (int var = 0; var < NVAR; ++var)
        for (int st = 0; st < NSTATE; ++st) {
            hipLaunchKernelGGL(phase_marker, dim3(1), dim3(64), 0, 0, mark);
            double tot = 0;
            std::vector<float> ts;
            for (int it = 0; it < reps + 3; ++it) {
                if (st != HOT || it == 0)
                    hipLaunchKernelGGL(produce_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, 0, r, v, d,
                                       slot, vboot, n, T, (uint32_t)it);
                if (st == DIRTY) hipLaunchKernelGGL(fill_kernel, dim3(1024), dim3(256), 0, 0, dirty, dirty4);
                if (st == FLUSHED) hipLaunchKernelGGL(fill_kernel, dim3(4096), dim3(256), 0, 0, big, big4);
                if (var == EMPTY)
                    hipExtLaunchKernelGGL(empty_kernel, dim3(gae_blocks), dim3(256), 0, 0, e0, e1, 0, (float *)nullptr);
                else if (var == COPY)
                    hipExtLaunchKernelGGL(copy_kernel, dim3(gblocks), dim3(256), 0, 0, e0, e1, 0, r, v, d, adv, ret, n4);
                else
                    CK((hipError_t)xpa_gae_scan_compact(r, v, d, slot, vboot, envs, T, 0.99f, 0.95f, 1, adv, ret, boot,
                                                        e0, e1, 0));
                CK(hipEventSynchronize(e1));
                float ms;
                CK(hipEventElapsedTime(&ms, e0, e1));
                if (it >= 3) {
                    tot += ms;
                    ts.push_back(ms * 1e3f);
                }
            }
            std::sort(ts.begin(), ts.end());
            const double mean = tot / reps * 1e3, med = ts[ts.size() / 2];
            printf("%s{\"phase\": \"%s/%s\", \"event_us_mean\": %.3f, \"event_us_median\": %.3f}", first ? "" : ", ",
                   kVar[var], kState[st], mean, med);
            fprintf(stderr, "%-12s %-9s event mean %7.3f us  median %7.3f us  %7.1f GB/s-alg\n", kVar[var], kState[st],
                    mean, med, alg / med * 1e-3);
            first = false;
        }
    printf("]}\n");
    CK(hipDeviceSynchronize());
    return 0;
}
