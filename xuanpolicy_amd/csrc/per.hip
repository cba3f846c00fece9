// K6 — prioritized replay on device: per-env sum / min segment trees, the store-time leaf write,
// the priority update and the proportional (stratified prefix-sum) sample (gfx950).
//
// Reference: SegmentTree / SumSegmentTree / MinSegmentTree (xuance/common/segtree_tool.py:4-86) and
// PerOffPolicyBuffer.store / sample / update_priorities (xuance/common/memory_tools.py:369-492),
// with the reference's pinned NumPy 1.21 arithmetic: every leaf and node is an f64
// (value-based casting makes np.float32 ** float a float64).
//
// Layout: one tree per env, [n_envs, 2 * cap] f64 (node 1 = root, leaf i at cap + i, element 0
// unused), neutral 0 (sum) / +inf (min) — the reference's list layout.  cap = next_pow2(n_size).
//
// Work is latency-bound (log2(cap) dependent levels), not bandwidth-bound: 2048 updates into
// 8 x 2^17-leaf trees touch ~35 k nodes (~0.6 MB).
#include "xpa_common.h"

#include <math.h>

namespace {

constexpr int kUpdThreads = 1024;

__device__ __forceinline__ double wave_max_d(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = fmax(v, __shfl_xor(v, o, 64));
    return v;
}

__global__ __launch_bounds__(64) void per_store_kernel(double *__restrict__ st, double *__restrict__ mt,
                                                       const double *__restrict__ max_p, int64_t n_envs,
                                                       int64_t cap, int64_t ptr, double alpha) {
    const int64_t e = (int64_t)blockIdx.x * 64 + threadIdx.x;
    if (e >= n_envs) return;
    double *s = st + e * 2 * cap, *m = mt + e * 2 * cap;
    const double v = pow(max_p[e], alpha);  // memory_tools.py:437-439
    int64_t node = cap + ptr;
    s[node] = v;
    m[node] = v;
    for (node >>= 1; node >= 1; node >>= 1) {
        s[node] = s[2 * node] + s[2 * node + 1];
        m[node] = fmin(m[2 * node], m[2 * node + 1]);
    }
}

// One block per env (memory_tools.py:482-492): a repeated index keeps the LAST entry's value
// (sequential semantics) — each leaf's winner is the largest batch position (atomicMax on a per-leaf
// scratch that is -1 between calls); max priority over every entry; ancestors rebuilt level by level.
__global__ __launch_bounds__(kUpdThreads) void per_update_kernel(double *__restrict__ st, double *__restrict__ mt,
                                                                 double *__restrict__ max_p, int *__restrict__ last,
                                                                 int64_t cap, int levels, int64_t size,
                                                                 const int64_t *__restrict__ idx,
                                                                 const float *__restrict__ prio, int64_t b,
                                                                 double alpha, int *__restrict__ err) {
    __shared__ double s_max[kUpdThreads / 64];
    const int64_t e = blockIdx.x;
    double *s = st + e * 2 * cap, *m = mt + e * 2 * cap;
    int *lst = last + e * cap;
    const int64_t *ix = idx + e * b;
    const float *pr = prio + e * b;
    for (int64_t k = threadIdx.x; k < b; k += kUpdThreads) {
        const int64_t i = ix[k];
        if (i < 0 || i >= size) {
            atomicAdd(err, 1);  // the reference asserts 0 <= idx < size
            continue;
        }
        atomicMax(lst + i, (int)k);
    }
    __syncthreads();
    double pmax = 0.0;
    for (int64_t k = threadIdx.x; k < b; k += kUpdThreads) {
        const int64_t i = ix[k];
        if (i < 0 || i >= size) continue;
        double p = (double)pr[k];
        if (p == 0.0) p += 1e-8;
        pmax = fmax(pmax, p);
        if (lst[i] == (int)k) {
            const double v = pow(p, alpha);
            s[cap + i] = v;
            m[cap + i] = v;
        }
    }
    pmax = wave_max_d(pmax);
    if ((threadIdx.x & 63) == 0) s_max[threadIdx.x >> 6] = pmax;
    __syncthreads();
    // ancestors, one level at a time (a node shared by several winners is written with one value)
    for (int lv = 1; lv <= levels; ++lv) {
        for (int64_t k = threadIdx.x; k < b; k += kUpdThreads) {
            const int64_t i = ix[k];
            if (i < 0 || i >= size || lst[i] != (int)k) continue;
            const int64_t node = (cap + i) >> lv;
            s[node] = s[2 * node] + s[2 * node + 1];
            m[node] = fmin(m[2 * node], m[2 * node + 1]);
        }
        __syncthreads();
    }
    for (int64_t k = threadIdx.x; k < b; k += kUpdThreads) {  // leave the scratch at -1
        const int64_t i = ix[k];
        if (i >= 0 && i < size && lst[i] == (int)k) lst[i] = -1;
    }
    if (threadIdx.x == 0) {
        double t = max_p[e];
        for (int w = 0; w < kUpdThreads / 64; ++w) t = fmax(t, s_max[w]);
        max_p[e] = t;
    }
}

__device__ __forceinline__ double u01_53(uint32_t seed, uint32_t ctr, uint32_t env, uint32_t k) {
    const uint32_t h1 = xpa_hash4(seed, ctr, env, 2u * k), h2 = xpa_hash4(seed, ctr, env, 2u * k + 1u);
    const uint64_t bits = ((uint64_t)(h1 >> 5) << 26) | (uint64_t)(h2 >> 6);
    return (double)bits * (1.0 / 9007199254740992.0);
}

// sum of leaves [0, last] in the reference's recursion order (segtree_tool.py:11-24 with
// start = 0): value[left child] + (rest of the prefix), nested to the right.
__device__ __forceinline__ double prefix_sum(const double *s, int64_t cap, int64_t last) {
    double terms[40];
    int n = 0;
    int64_t node = 1, lo = 0, hi = cap - 1;
    while (hi != last) {
        const int64_t mid = (lo + hi) >> 1;
        if (last <= mid) {
            node = 2 * node;
            hi = mid;
        } else {
            terms[n++] = s[2 * node];
            node = 2 * node + 1;
            lo = mid + 1;
        }
    }
    double acc = s[node];
    for (int j = n - 1; j >= 0; --j) acc = terms[j] + acc;
    return acc;
}

// Thread per sample (memory_tools.py:411-427 + 446-465).
__global__ __launch_bounds__(256) void per_sample_kernel(const double *__restrict__ st,
                                                         const double *__restrict__ mt, int64_t n_envs, int64_t cap,
                                                         int64_t size, int64_t b, int64_t n_size,
                                                         const double *__restrict__ uniforms, uint32_t seed,
                                                         uint32_t counter, double beta, int wrap_uint8,
                                                         int64_t *__restrict__ steps, int64_t *__restrict__ flat,
                                                         double *__restrict__ weights, int *__restrict__ err) {
    const int64_t g = (int64_t)blockIdx.x * 256 + threadIdx.x;
    if (g >= n_envs * b) return;
    const int64_t e = g / b, k = g - e * b;
    const double *s = st + e * 2 * cap, *m = mt + e * 2 * cap;
    const double p_total = prefix_sum(s, cap, size - 2);  // sum(0, size - 1): exclusive end
    const double every = p_total / (double)b;
    const double u = uniforms ? uniforms[g] : u01_53(seed, counter, (uint32_t)e, (uint32_t)k);
    double mass = u * every + (double)k * every;
    int64_t node = 1;
    while (node < cap) {  // find_prefixsum_idx (segtree_tool.py:62-71)
        const double l = s[2 * node];
        if (l > mass) {
            node = 2 * node;
        } else {
            mass -= l;
            node = 2 * node + 1;
        }
    }
    int64_t idx = node - cap;
    if (idx >= size) {  // mass at or past the stored total (rounding of u*len + k*len): a zero leaf — the reference
        if (err) atomicAdd(err, 1);  // would then assert in update_priorities; clamped to the last stored step
        idx = size - 1;
        node = cap + idx;
    }
    const double total = s[1];
    const double scale = pow((double)size, -beta);
    const double max_weight = (m[1] / total) * scale;
    const double weight = (s[node] / total) * scale;
    weights[g] = weight / max_weight;
    const int64_t step = wrap_uint8 ? (idx & 255) : idx;  // step_choices.astype(np.uint8)
    steps[g] = step;
    if (flat) flat[g] = e * n_size + step;
}

}  // namespace

XPA_API int xpa_per_store(double *sum_tree, double *min_tree, const double *max_priority, int64_t n_envs,
                          int64_t capacity, int64_t ptr, double alpha, xpa_stream_t stream) {
    if (n_envs <= 0 || capacity <= 0 || (capacity & (capacity - 1)) || ptr < 0 || ptr >= capacity || !sum_tree ||
        !min_tree || !max_priority)
        return (int)hipErrorInvalidValue;
    hipLaunchKernelGGL(per_store_kernel, dim3((unsigned)((n_envs + 63) / 64)), dim3(64), 0, (hipStream_t)stream,
                       sum_tree, min_tree, max_priority, n_envs, capacity, ptr, alpha);
    return xpa_launch_status();
}

XPA_API int xpa_per_update_priorities(double *sum_tree, double *min_tree, double *max_priority, int *scratch,
                                      int64_t n_envs, int64_t capacity, int64_t size, const int64_t *idx,
                                      const float *priorities, int64_t batch_per_env, double alpha, int *err,
                                      xpa_stream_t stream) {
    if (n_envs <= 0 || capacity <= 0 || (capacity & (capacity - 1)) || size <= 0 || size > capacity ||
        batch_per_env <= 0 || batch_per_env > (1 << 30) || !sum_tree || !min_tree || !max_priority || !scratch ||
        !idx || !priorities || !err)
        return (int)hipErrorInvalidValue;
    int levels = 0;
    while ((1LL << levels) < capacity) ++levels;
    hipLaunchKernelGGL(per_update_kernel, dim3((unsigned)n_envs), dim3(kUpdThreads), 0, (hipStream_t)stream, sum_tree,
                       min_tree, max_priority, scratch, capacity, levels, size, idx, priorities, batch_per_env, alpha,
                       err);
    return xpa_launch_status();
}

XPA_API int xpa_per_sample(const double *sum_tree, const double *min_tree, int64_t n_envs, int64_t capacity,
                           int64_t size, int64_t batch_per_env, int64_t n_size, const double *uniforms, uint32_t seed,
                           uint32_t counter, double beta, int wrap_uint8, int64_t *steps, int64_t *flat_index,
                           double *weights, int32_t *err, xpa_stream_t stream) {
    if (n_envs <= 0 || capacity <= 0 || (capacity & (capacity - 1)) || size < 2 || size > capacity ||
        n_size < size || batch_per_env <= 0 || !(beta > 0) || !sum_tree || !min_tree || !steps || !weights)
        return (int)hipErrorInvalidValue;
    const int64_t total = n_envs * batch_per_env;
    hipLaunchKernelGGL(per_sample_kernel, dim3((unsigned)((total + 255) / 256)), dim3(256), 0, (hipStream_t)stream,
                       sum_tree, min_tree, n_envs, capacity, size, batch_per_env, n_size, uniforms, seed, counter, beta,
                       wrap_uint8, steps, flat_index, weights, err);
    return xpa_launch_status();
}
